import ctypes as C, time
hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
hip.hipSetDevice(0)
p = C.c_void_p()
for sz in (1 << 20, 1 << 28, 1200 << 20, 1200 << 20, 100 << 20):
    t = time.perf_counter(); e = hip.hipMalloc(C.byref(p), C.c_size_t(sz)); t1 = time.perf_counter()
    e2 = hip.hipMemset(p, 0, C.c_size_t(64)); hip.hipDeviceSynchronize(); t2 = time.perf_counter()
    hip.hipFree(p); t3 = time.perf_counter()
    print("size %6d MB malloc %.2f ms first-touch %.2f ms free %.2f ms (err %d %d)" % (sz >> 20, 1e3*(t1-t), 1e3*(t2-t1), 1e3*(t3-t2), e, e2))
