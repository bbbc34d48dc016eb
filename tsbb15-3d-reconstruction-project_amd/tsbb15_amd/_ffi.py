"""ctypes binding of lib/librsamd.so (C ABI declared in include/rsamd.h).

The library is built in-tree (``make -C csrc``, or ``__graft_entry__.build()``).  There is no
fallback: if the shared object is missing or no GPU is visible, the compute entry points
raise.  Status codes map to the reference's exception types (ValueError for shape/argument
errors, as lab3.py:207-208 / lab3.py:283-284 / ransac.py:13-14 raise).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RSAMD_LIB", os.path.join(_PKG_ROOT, "lib", "librsamd.so"))
HEADER_PATH = os.path.join(os.path.dirname(_PKG_ROOT), "include", "rsamd.h")

RS_OK, RS_EINVAL, RS_EDEVICE, RS_ENODEV, RS_ECOMM, RS_ENOMEM = 0, -1, -2, -3, -4, -5
SAMPLER_PHILOX, SAMPLER_TUPLES = 0, 1
PNP_DLT6, PNP_EPNP5, PNP_P3P = 0, 1, 2
MT_N = 624
COMM_ID_BYTES = 128

_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)


class F8Result(C.Structure):
    _fields_ = [("F", C.c_double * 9), ("best_index", C.c_int64), ("best_count", C.c_int64),
                ("best_std", C.c_double), ("best_norm", C.c_double),
                ("max_count_fast", C.c_int64), ("n_candidates", C.c_int64),
                ("guard_mismatch", C.c_int64)]


class F8Candidate(C.Structure):
    _fields_ = [("index", C.c_int64), ("count", C.c_int64), ("std_d", C.c_double),
                ("norm_d", C.c_double), ("F", C.c_double * 9)]


class PnpResult(C.Structure):
    _fields_ = [("R", C.c_double * 9), ("t", C.c_double * 3), ("best_index", C.c_int64),
                ("best_count", C.c_int64)]


class PairResult(C.Structure):
    _fields_ = [("F", C.c_double * 9), ("best_index", C.c_int64), ("best_count", C.c_int64),
                ("best_std", C.c_double), ("best_norm", C.c_double),
                ("n_candidates", C.c_int64)]


class E5Result(C.Structure):
    _fields_ = [("E", C.c_double * 9), ("F", C.c_double * 9), ("best_sample", C.c_int64),
                ("best_solution", C.c_int64), ("best_count", C.c_int64)]


class GsInfo(C.Structure):
    _fields_ = [("cost_init", C.c_double), ("cost", C.c_double), ("iterations", C.c_int32),
                ("accepted", C.c_int32), ("status", C.c_int32), ("n", C.c_int32)]


_SIGS = {
    "rs_last_error": (C.c_char_p, []),
    "rs_version": (C.c_int, []),
    "rs_np_seed": (C.c_int, [C.c_uint32, _u32p, _i32p]),
    "rs_np_choice_tuples": (C.c_int, [_u32p, _i32p, C.c_int64, C.c_int32, C.c_int64, _i32p]),
    "rs_np_choice_tuples_gpu": (C.c_int, [C.c_void_p, _u32p, _i32p, C.c_int64, C.c_int32,
                                          C.c_int64, _i32p]),
    "rs_py_seed": (C.c_int, [_u32p, C.c_int32, _u32p, _i32p]),
    "rs_py_shuffle_tuples": (C.c_int, [_u32p, _i32p, C.c_int64, C.c_int32, C.c_int64, _i32p]),
    "rs_np_choice_tuples_multi": (C.c_int, [C.c_int64, _u32p, _u32p, _i32p, _i64p, C.c_int32,
                                            C.c_int64, _i32p, C.c_int32]),
    "rs_py_shuffle_tuples_gpu": (C.c_int, [C.c_void_p, _u32p, _i32p, C.c_int64, C.c_int32,
                                           C.c_int64, _i32p]),
    "rs_mt_jump": (C.c_int, [_u32p, C.c_int32, C.c_int64, _u32p, _i32p]),
    "rs_np_host_stats": (C.c_int, [C.POINTER(C.c_double), _i64p]),
    "rs_np_timing": (C.c_int, [C.c_void_p, C.c_int32, _dp, _dp, _i64p]),
    "rs_pnp_timing": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double),
                                C.POINTER(C.c_double)]),
    "rs_mt_poly_selftest": (C.c_int, [C.c_int64, C.c_int64]),
    "rs_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rs_ctx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "rs_ctx_destroy": (C.c_int, [C.c_void_p]),
    "rs_ctx_synchronize": (C.c_int, [C.c_void_p]),
    "rs_fmatrix_stls": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp]),
    "rs_fmatrix_stls_batch": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _i32p, C.c_int64, _dp]),
    "rs_fmatrix_residuals": (C.c_int, [C.c_void_p, _dp, _dp, _dp, C.c_int64, _dp]),
    "rs_f8_plan_create": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_void_p)]),
    "rs_f8_plan_destroy": (C.c_int, [C.c_void_p]),
    "rs_f8_plan_set_points": (C.c_int, [C.c_void_p, _dp, _dp]),
    "rs_f8_plan_run": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_uint64, C.c_uint64,
                                 _i32p, C.c_double]),
    "rs_f8_plan_run_np": (C.c_int, [C.c_void_p, C.c_int64, _u32p, _i32p, C.c_double]),
    "rs_f8_plan_run_np_slice": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, _u32p,
                                          _i32p, C.c_double]),
    "rs_f8_plan_result": (C.c_int, [C.c_void_p, C.POINTER(F8Result), _i64p, C.c_int64, _i64p]),
    "rs_f8_plan_candidates": (C.c_int, [C.c_void_p, C.POINTER(F8Candidate), C.c_int64, _i64p]),
    "rs_f8_plan_counts": (C.c_int, [C.c_void_p, _i32p, C.c_int64]),
    "rs_f8_plan_models": (C.c_int, [C.c_void_p, _dp, C.c_int64]),
    "rs_f8_plan_kernel_ms": (C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    "rs_f8_plan_kernel_avg": (C.c_int, [C.c_void_p, C.c_int64, _dp, _dp, _dp]),
    "rs_f8_plan_set_timing": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "rs_f8_plan_set_count_precision": (C.c_int, [C.c_void_p, C.c_int32]),
    "rs_f8_ransac_np": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, C.c_int64, _u32p, _i32p,
                                  C.c_double, C.POINTER(F8Result), _i64p, C.c_int64, _i64p]),
    "rs_pnp_dlt": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _dp]),
    "rs_pnp_ransac": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _dp, C.c_int64, C.c_int32,
                                C.c_int64, C.c_int32, C.c_uint64, _i32p, C.c_double,
                                C.POINTER(PnpResult), _i64p, _i64p, _i64p, _i64p]),
    "rs_pnp_count_poses": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, C.c_int64, C.c_double,
                                     _i32p]),
    "rs_pnp_ransac_cv": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, C.c_int64, C.c_uint64,
                                   C.c_double, C.c_double, C.c_int32, _dp, C.POINTER(PnpResult),
                                   _i64p, _i64p, _i64p]),
    "rs_pnp_minimal": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, C.c_int32, _dp, _dp, _dp]),
    "rs_pnp_refine_lm": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _dp, _dp, C.c_int32, _dp]),
    "rs_e5_solve": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _i32p]),
    "rs_e5_ransac": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _dp, C.c_int64, C.c_uint64,
                               C.c_double, C.POINTER(E5Result), _i64p, _i64p]),
    "rs_pairs_f8_ransac": (C.c_int, [C.c_void_p, _dp, _dp, _i64p, C.c_int64, C.c_int64,
                                     C.c_int32, C.c_uint64, _i64p, _i32p, C.c_double,
                                     C.POINTER(PairResult), _i32p]),
    "rs_pairs_two_view": (C.c_int, [C.c_void_p, _dp, _dp, _i64p, C.c_int64, C.c_int64,
                                    C.c_int32, C.c_uint64, _i64p, _i32p, C.c_double, C.c_int32,
                                    _dp, _dp, _dp, C.POINTER(PairResult), _i32p, _dp,
                                    C.POINTER(GsInfo), _dp, _dp, _i32p]),
    "rs_triangulate_optimal": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, _dp, _i32p,
                                         C.c_int64, _dp]),
    "rs_camera_resectioning": (C.c_int, [C.c_void_p, _dp, C.c_int64, _dp, _dp, _dp]),
    "rs_essential_from_f": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, C.c_int64, _dp]),
    "rs_relative_camera_pose": (C.c_int, [C.c_void_p, _dp, _dp, _dp, C.c_int64, _dp, _dp,
                                          _i32p]),
    "rs_fmatrix_cameras": (C.c_int, [C.c_void_p, _dp, C.c_int64, _dp]),
    "rs_fmatrix_from_cameras": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp]),
    "rs_gold_standard": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _i64p, C.c_int64, C.c_int32, _dp,
                                   _dp, _dp, C.POINTER(GsInfo)]),
    "rs_gs_residuals_fd": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp, C.c_int64, _dp, _dp]),
    "rs_match_observations": (C.c_int, [C.c_void_p, _dp, _i64p, C.c_int64, _dp, C.c_int64,
                                        C.c_double, _i64p]),
    "rs_e_from_cameras": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp]),
    "rs_add_new_points": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, C.c_int64, C.c_double, _i32p,
                                    _dp]),
    "rs_ba_residuals": (C.c_int, [C.c_void_p, _dp, C.c_int64, _dp, C.c_int64, _i32p, _i32p, _dp,
                                  C.c_int64, _dp]),
    "rs_ba_jacobian": (C.c_int, [C.c_void_p, _dp, C.c_int64, _dp, C.c_int64, _i32p, _i32p,
                                 C.c_int64, _dp, _dp]),
    "rs_np_shard_create": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_int32, C.POINTER(C.c_void_p)]),
    "rs_np_shard_destroy": (C.c_int, [C.c_void_p]),
    "rs_np_shard_parse": (C.c_int, [C.c_void_p, _u32p, C.c_int32, C.c_int64, _i64p]),
    "rs_np_shard_maps": (C.c_int, [C.c_void_p, _u8p, C.c_int64, _i64p]),
    "rs_np_shard_compose": (C.c_int, [C.c_void_p, _u8p, C.c_int64, _i64p, _i64p]),
    "rs_np_shard_tuples": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                     _i32p, _u32p, _i32p]),
    "rs_f8_plan_run_np_shard": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                          C.c_int64, C.c_int64, _u32p, _i32p, C.c_double]),
    "rs_comm_unique_id": (C.c_int, [_u8p]),
    "rs_comm_init": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, _u8p]),
    "rs_comm_destroy": (C.c_int, [C.c_void_p]),
    "rs_comm_allgather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    "rs_comm_allreduce_max_i64": (C.c_int, [C.c_void_p, _i64p]),
    "rs_comm_library": (C.c_int, [_i32p, C.c_char_p, C.c_int64]),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load librsamd.so once; raise loudly if it was not built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        f"{LIB_PATH} is missing: build the HIP extension first "
                        "(make -C tsbb15-3d-reconstruction-project_amd/csrc or "
                        "__graft_entry__.build()); there is no CPU fallback")
                L = C.CDLL(LIB_PATH)
                for name, (res, args) in _SIGS.items():
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = L
    return _lib


def check(status):
    if status == RS_OK:
        return
    msg = lib().rs_last_error().decode(errors="replace")
    if status == RS_EINVAL:
        raise ValueError(msg)
    if status == RS_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(f"rsamd error {status}: {msg}")


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def f64c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def rccl_library():
    """(version, path) of the RCCL shared object this process runs (rs_comm_library)."""
    v = C.c_int32(0)
    buf = C.create_string_buffer(4096)
    check(lib().rs_comm_library(C.byref(v), buf, 4096))
    return v.value, buf.value.decode(errors="replace")


def device_count():
    n = C.c_int(0)
    check(lib().rs_device_count(C.byref(n)))
    return n.value


class Context:
    """One HIP device + stream (rs_ctx)."""

    def __init__(self, device=0):
        h = C.c_void_p()
        check(lib().rs_ctx_create(int(device), C.byref(h)))
        self._h = h
        self.device = int(device)

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("context destroyed")
        return self._h

    def close(self):
        if self._h is not None:
            lib().rs_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        check(lib().rs_ctx_synchronize(self.handle))


_default = {}


def default_context():
    """Process-wide context on the device named by RSAMD_DEVICE / LOCAL_RANK (default 0)."""
    dev = int(os.environ.get("RSAMD_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    ctx = _default.get(dev)
    if ctx is None:
        ctx = Context(dev)
        _default[dev] = ctx
    return ctx


# ------------------------------------------------------------------------------------------
# host samplers
# ------------------------------------------------------------------------------------------
def np_choice_tuples(key, pos, n, k, count):
    """Replay ``count`` x np.random.choice(arange(n), k, replace=False); returns
    (tuples (count,k) int32, key', pos')."""
    key = np.array(key, dtype=np.uint32, copy=True)
    if key.shape != (MT_N,):
        raise ValueError("MT19937 key must have 624 words")
    p = C.c_int32(int(pos))
    out = np.empty((int(count), int(k)), dtype=np.int32)
    check(lib().rs_np_choice_tuples(ptr(key, C.c_uint32), C.byref(p), int(n), int(k),
                                    int(count), ptr(out, C.c_int32)))
    return out, key, p.value


def np_choice_tuples_gpu(key, pos, n, k, count, ctx=None):
    """np_choice_tuples computed on the GPU (rs_np_choice_tuples_gpu): the same tuples and
    (key', pos'), bit for bit."""
    ctx = ctx or default_context()
    key = np.array(key, dtype=np.uint32, copy=True)
    if key.shape != (MT_N,):
        raise ValueError("MT19937 key must have 624 words")
    p = C.c_int32(int(pos))
    out = np.empty((int(count), int(k)), dtype=np.int32)
    check(lib().rs_np_choice_tuples_gpu(ctx.handle, ptr(key, C.c_uint32), C.byref(p), int(n),
                                        int(k), int(count), ptr(out, C.c_int32)))
    return out, key, p.value


def np_choice_tuples_multi(keys, poss, ns, k, count, threads=0, seeds=None):
    """np_choice_tuples for B independent streams on host threads; returns
    (tuples (B, count, k), keys', poss').  With ``seeds`` the streams start from
    np.random.seed(seeds[b]) and keys / poss may be None.  Streams with n < k give zeros."""
    ns = np.ascontiguousarray(ns, dtype=np.int64).reshape(-1)
    B = ns.shape[0]
    sp = None
    if seeds is not None:
        seeds = np.asarray(seeds).reshape(-1)
        for sd in seeds:
            _check_np_seed(sd)
        seeds = np.ascontiguousarray(seeds.astype(np.int64), dtype=np.uint32).reshape(B)
        sp = ptr(seeds, C.c_uint32)
        keys = np.empty((B, MT_N), dtype=np.uint32)
        poss = np.empty(B, dtype=np.int32)
    else:
        keys = np.array(keys, dtype=np.uint32, copy=True).reshape(B, MT_N)
        poss = np.array(poss, dtype=np.int32, copy=True).reshape(B)
    out = np.empty((B, int(count), int(k)), dtype=np.int32)
    check(lib().rs_np_choice_tuples_multi(B, sp, ptr(keys, C.c_uint32), ptr(poss, C.c_int32),
                                          ptr(ns, C.c_int64), int(k), int(count),
                                          ptr(out, C.c_int32), int(threads)))
    return out, keys, poss


def py_shuffle_tuples(key, pos, n, k, count):
    """Replay ``count`` x ransac.gen_rnd_indices(n, k) on a CPython MT state."""
    key = np.array(key, dtype=np.uint32, copy=True)
    if key.shape != (MT_N,):
        raise ValueError("MT19937 key must have 624 words")
    p = C.c_int32(int(pos))
    out = np.empty((int(count), int(k)), dtype=np.int32)
    check(lib().rs_py_shuffle_tuples(ptr(key, C.c_uint32), C.byref(p), int(n), int(k),
                                     int(count), ptr(out, C.c_int32)))
    return out, key, p.value


def py_shuffle_tuples_gpu(key, pos, n, k, count, ctx=None):
    """py_shuffle_tuples computed on the GPU (rs_py_shuffle_tuples_gpu): the same tuples and
    (key', pos'), bit for bit."""
    ctx = ctx or default_context()
    key = np.array(key, dtype=np.uint32, copy=True)
    if key.shape != (MT_N,):
        raise ValueError("MT19937 key must have 624 words")
    p = C.c_int32(int(pos))
    out = np.empty((int(count), int(k)), dtype=np.int32)
    check(lib().rs_py_shuffle_tuples_gpu(ctx.handle, ptr(key, C.c_uint32), C.byref(p), int(n),
                                         int(k), int(count), ptr(out, C.c_int32)))
    return out, key, p.value


def pnp_timing(ctx, enable):
    """Enable / disable HIP events around rs_pnp_ransac's kernels; returns the last timed call's
    (solve_ms, count_ms), -1 when none."""
    a, b = C.c_double(0.0), C.c_double(0.0)
    check(lib().rs_pnp_timing(ctx.handle, int(enable), C.byref(a), C.byref(b)))
    return a.value, b.value


NP_STEPS = ("jump", "stream_pass1", "entry", "track", "compose", "starts", "tuples", "result",
            "stream_pass2", "parse_total")


def np_timing(ctx, enable):
    """Enable / disable the parse's step events (rs_np_timing); returns the last parse call's
    ({step: ms}, {stream_written, parse_read, tuples_read: bytes}, segments)."""
    ms, by, seg = np.zeros(len(NP_STEPS)), np.zeros(3), C.c_int64(0)
    check(lib().rs_np_timing(ctx.handle, int(enable), ptr(ms, C.c_double), ptr(by, C.c_double),
                             C.byref(seg)))
    return (dict(zip(NP_STEPS, ms.tolist())),
            dict(zip(("stream_written", "parse_read", "tuples_read"), by.tolist())), seg.value)


def np_host_stats():
    """(host ms spent building MT jump polynomials in this process, level sets built)."""
    ms, n = C.c_double(0.0), C.c_int64(0)
    check(lib().rs_np_host_stats(C.byref(ms), C.byref(n)))
    return ms.value, n.value


def mt_jump(key, pos, steps):
    """MT19937 (key, pos) after ``steps`` more 32-bit outputs (jump-ahead, no generation)."""
    key = np.ascontiguousarray(key, dtype=np.uint32)
    if key.shape != (MT_N,):
        raise ValueError("MT19937 key must have 624 words")
    out = np.empty(MT_N, dtype=np.uint32)
    p = C.c_int32(0)
    check(lib().rs_mt_jump(ptr(key, C.c_uint32), int(pos), int(steps), ptr(out, C.c_uint32),
                           C.byref(p)))
    return out, p.value


def _check_np_seed(seed):
    """np.random.seed's accepted range for an integer seed (it raises ValueError outside)."""
    s = int(seed)
    if s != seed or not 0 <= s < 2 ** 32:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    return s


def np_seed(seed):
    key = np.empty(MT_N, dtype=np.uint32)
    p = C.c_int32(0)
    check(lib().rs_np_seed(_check_np_seed(seed), ptr(key, C.c_uint32), C.byref(p)))
    return key, p.value


def py_seed(seed):
    n = abs(int(seed))
    words = []
    while n:
        words.append(n & 0xFFFFFFFF)
        n >>= 32
    w = np.array(words or [0], dtype=np.uint32)
    key = np.empty(MT_N, dtype=np.uint32)
    p = C.c_int32(0)
    check(lib().rs_py_seed(ptr(w, C.c_uint32), len(words), ptr(key, C.c_uint32), C.byref(p)))
    return key, p.value


class NpShard:
    """One rank's share of a parity-stream parse (rs_np_shard_*): the numpy (py=False) or
    CPython (py=True) stream cut into chunks, this rank parsing only its own.  The exchange
    between the steps is :func:`tsbb15_amd.parallel.np_sharded_segments`."""

    def __init__(self, ctx, n, k, world, rank, py=False):
        self.ctx, self.n, self.k = ctx, int(n), int(k)
        self.world, self.rank = int(world), int(rank)
        h = C.c_void_p()
        check(lib().rs_np_shard_create(ctx.handle, self.n, self.k, self.world, self.rank,
                                       1 if py else 0, C.byref(h)))
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("shard destroyed")
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().rs_np_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def parse(self, key, pos, count):
        """Step 1 (rank-local).  Returns the layout dict of this segment."""
        key = np.ascontiguousarray(key, dtype=np.uint32)
        if key.shape != (MT_N,):
            raise ValueError("MT19937 key must have 624 words")
        lay = np.zeros(6, np.int64)
        check(lib().rs_np_shard_parse(self.handle, ptr(key, C.c_uint32), int(pos), int(count),
                                      ptr(lay, C.c_int64)))
        return dict(zip(("count", "C", "Cr", "Wc", "D", "map_bytes"), lay.tolist()))

    def maps(self):
        """Step 2: this rank's chunk-map blob (bytes)."""
        nb = C.c_int64(0)
        check(lib().rs_np_shard_maps(self.handle, None, 0, C.byref(nb)))
        out = np.zeros(nb.value, np.uint8)
        check(lib().rs_np_shard_maps(self.handle, ptr(out, C.c_uint8), nb.value, C.byref(nb)))
        return out.tobytes()

    def compose(self, blobs):
        """Step 3: all ranks' blobs in rank order -> (own start count, first start)."""
        stride = max(len(b) for b in blobs)
        buf = np.zeros(stride * len(blobs), np.uint8)
        for r, b in enumerate(blobs):
            buf[r * stride:r * stride + len(b)] = np.frombuffer(b, np.uint8)
        ns, first = C.c_int64(0), C.c_int64(0)
        check(lib().rs_np_shard_compose(self.handle, ptr(buf, C.c_uint8), stride, C.byref(ns),
                                        C.byref(first)))
        return ns.value, first.value

    def tuples(self, base, hi, next_start, final_idx, key):
        """Step 4: own hypotheses [base, hi) as (hi - base, k) int32; with final_idx >= 0 also
        the (key, pos) after the segment (key: the segment's entry key, the default)."""
        cnt = int(hi) - int(base)
        out = np.empty((max(cnt, 0), self.k), np.int32)
        key2 = np.array(key, dtype=np.uint32, copy=True)
        p = C.c_int32(-1)
        check(lib().rs_np_shard_tuples(self.handle, int(base), int(hi), int(next_start),
                                       int(final_idx), ptr(out, C.c_int32),
                                       ptr(key2, C.c_uint32), C.byref(p)))
        return out, (key2, p.value) if final_idx >= 0 else None


# ------------------------------------------------------------------------------------------
# RANSAC-F plan
# ------------------------------------------------------------------------------------------
class F8Plan:
    """Correspondences resident in HBM + buffers for up to ``max_hyp`` hypotheses."""

    def __init__(self, ctx, n, max_hyp):
        self.ctx = ctx
        self.n = int(n)
        self.max_hyp = int(max_hyp)
        h = C.c_void_p()
        check(lib().rs_f8_plan_create(ctx.handle, self.n, self.max_hyp, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().rs_f8_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_points(self, p1, p2):
        p1, p2 = f64c(p1), f64c(p2)
        if p1.shape != (2, self.n) or p2.shape != (2, self.n):
            raise ValueError("points must be (2, n) matching the plan")
        check(lib().rs_f8_plan_set_points(self._h, ptr(p1, C.c_double), ptr(p2, C.c_double)))

    def run(self, H, mode=SAMPLER_PHILOX, seed=0, hyp_offset=0, tuples=None, thresh=1.5):
        tp = None
        if mode == SAMPLER_TUPLES:
            tuples = np.ascontiguousarray(tuples, dtype=np.int32)
            if tuples.shape != (int(H), 8):
                raise ValueError("tuples must be (H, 8)")
            tp = ptr(tuples, C.c_int32)
        check(lib().rs_f8_plan_run(self._h, int(H), int(mode), int(seed) & (2**64 - 1),
                                   int(hyp_offset), tp, float(thresh)))

    def run_np(self, H, key, pos, thresh=1.5):
        """Parity-mode run on the numpy legacy stream (key, pos), sampled on the GPU; returns
        the advanced (key, pos)."""
        key = np.array(key, dtype=np.uint32, copy=True)
        p = C.c_int32(int(pos))
        check(lib().rs_f8_plan_run_np(self._h, int(H), ptr(key, C.c_uint32), C.byref(p),
                                      float(thresh)))
        return key, p.value

    def run_np_slice(self, H, start, count, key, pos, thresh=1.5):
        """Hypotheses [start, start + count) of an H-hypothesis parity run (one rank's shard):
        the numpy stream of all H is parsed on the GPU, the slice is evaluated; returns the
        (key, pos) after all H.  Candidate indices of the run are slice-local."""
        key = np.array(key, dtype=np.uint32, copy=True)
        p = C.c_int32(int(pos))
        check(lib().rs_f8_plan_run_np_slice(self._h, int(H), int(start), int(count),
                                            ptr(key, C.c_uint32), C.byref(p), float(thresh)))
        return key, p.value

    def run_np_shard(self, shard, base, hi, next_start, final_idx, key, thresh=1.5):
        """Sharded parity mode: this rank's hypotheses [base, hi) of ``shard`` (after its
        compose step) evaluated as one run (candidate indices run-local: add base).  Returns
        the (key, pos) after the segment when final_idx >= 0, else None."""
        key2 = np.array(key, dtype=np.uint32, copy=True)
        p = C.c_int32(-1)
        check(lib().rs_f8_plan_run_np_shard(self._h, shard.handle, int(base), int(hi),
                                            int(next_start), int(final_idx),
                                            ptr(key2, C.c_uint32), C.byref(p), float(thresh)))
        return (key2, p.value) if final_idx >= 0 else None

    def result(self):
        r = F8Result()
        inl = np.empty(self.n, dtype=np.int64)
        k = C.c_int64(0)
        check(lib().rs_f8_plan_result(self._h, C.byref(r), ptr(inl, C.c_int64), self.n,
                                      C.byref(k)))
        return r, inl[:k.value].copy()

    def candidates(self):
        k = C.c_int64(0)
        check(lib().rs_f8_plan_candidates(self._h, None, 0, C.byref(k)))
        arr = (F8Candidate * max(1, k.value))()
        check(lib().rs_f8_plan_candidates(self._h, arr, k.value, C.byref(k)))
        return [arr[i] for i in range(k.value)]

    def counts(self, H):
        out = np.empty(int(H), dtype=np.int32)
        check(lib().rs_f8_plan_counts(self._h, ptr(out, C.c_int32), int(H)))
        return out

    def models(self, H):
        out = np.empty((int(H), 9), dtype=np.float64)
        check(lib().rs_f8_plan_models(self._h, ptr(out, C.c_double), int(H)))
        return out.reshape(-1, 3, 3)

    def set_count_precision(self, fp64):
        """fp64=True: the plain float64 counting kernel for later runs (same counts, slower)."""
        check(lib().rs_f8_plan_set_count_precision(self._h, 1 if fp64 else 0))

    def set_timing(self, level=1, every=1):
        """HIP timing events per run: level 0 none, 1 counting kernel, 2 also solve / run;
        recorded on every ``every``-th run (each event is a marker packet between kernels)."""
        check(lib().rs_f8_plan_set_timing(self._h, int(level), int(every)))

    def kernel_ms(self, last_n=1):
        """Device times of the last run, or averaged over the last ``last_n`` runs."""
        a, b, t = C.c_double(), C.c_double(), C.c_double()
        check(lib().rs_f8_plan_kernel_avg(self._h, int(last_n), C.byref(a), C.byref(b),
                                          C.byref(t)))
        return {"count_ms": a.value, "solve_ms": b.value, "total_ms": t.value}
