"""RANSAC hypotheses/s for the 8-point F hot path on MI355X (BASELINE.json metric).

One step = one full RANSAC run over one synthetic correspondence set already resident in
HBM (config C2: N = 2000 correspondences, 30 % outliers, 100 000 hypotheses): sample,
8-point solve, inlier count, select c*, reference-order re-score of the candidates, the
fun.py:320-328 replay, S_RANSAC extraction, and the result copied back to the host.

Multi-GPU (weak scaling): one process per GPU, each owning its own image pair (pairs shard
with no data-path collective); after the timed steps the per-pair best models are exchanged
with one RCCL all-gather over xGMI (inside the timed region).  Timing: barrier +
device sync on both sides, max over ranks.

Extra fields: roofline of the dominant kernel (k_f8_count) from HIP events on its stream,
the numpy-exact parity mode measured on the same workload, and the oracle CPU baseline.
"""
import os

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")  # CPU baseline is single-core numpy
os.environ.setdefault("OMP_NUM_THREADS", "1")

import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
sys.path.insert(0, REPO)

from tsbb15_amd import _ffi, synth  # noqa: E402


class _stdout_to_stderr:
    """RCCL prints a version banner on the process's stdout (C stdio) at communicator set-up;
    the bench's stdout carries exactly one JSON line, so file descriptor 1 points at stderr
    while the library runs (C stdio flushed before it is restored)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        ctypes.CDLL(None).fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False

METRIC = "RANSAC hypotheses/sec (8-pt F, 2k corr) at 1/2/4/8 GPUs; % HBM roofline"
N_CORR = 2000
OUTLIERS = 0.30
HYPS = 100_000
PEAK_FP64_VALU_TFLOPS = 78.6   # 256 CU x 4 SIMD x 16 fp64 FMA lanes x 2 x 2.4 GHz
PEAK_FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: 64 FLOP/clk/SIMD (v_pk_fma_f32)
TIMING_EVERY = 8               # HIP events around the counting kernel on every 8th timed run
PEAK_HBM_GBS = 8000.0
FLOP_PER_CORR = 42             # score work per (hypothesis, correspondence)
FLOP_SOLVE = 15000             # minimal solve per hypothesis


def dist_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


class Dist:
    """Barrier / max-reduce / broadcast for the harness, without torch.distributed: a TCP hub
    on MASTER_PORT + 1 (tsbb15_amd.parallel.TcpHub; torch.distributed.run's own store holds
    MASTER_PORT).  Nothing in this process imports torch, so librsamd's librccl.so resolves
    through its RUNPATH to /opt/rocm/lib (config.exchange_library records which one ran)."""

    def __init__(self, world):
        from tsbb15_amd import parallel
        self.world = world
        self.hub = parallel.TcpHub.from_env() if world > 1 else None

    def barrier(self):
        if self.hub:
            self.hub.barrier()

    def max(self, x):
        return float(x) if self.hub is None else self.hub.max_float(x)

    def bcast_bytes(self, b, src=0):
        return b if self.hub is None else self.hub.broadcast_bytes(b, src)

    def close(self):
        if self.hub:
            self.hub.close()


def _cpu_worker(args):
    """One host core: the oracle loop (numpy restatement of fun.py:303-328) for budget_s."""
    p1, p2, seed, budget_s = args
    from oracle import ransac_ref
    rs = np.random.RandomState(seed)
    done, t0 = 0, time.perf_counter()
    while True:
        ransac_ref.ransac_f(p1, p2, r=250, rng=rs)
        done += 250
        el = time.perf_counter() - t0
        if el >= budget_s:
            return done, el


def host_cores():
    """The host cores this process may use: the CPU affinity mask, bounded by the cgroup CPU
    quota and by OMP_NUM_THREADS (the box exports its CPU share there; nproc and
    os.cpu_count() show the whole machine).  Returns (cores, evidence)."""
    ev = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    n = ev["affinity"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            ev["cgroup_quota"] = float(q) / float(per)
            n = min(n, max(1, int(ev["cgroup_quota"])))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        ev["omp_num_threads"] = int(omp)
        n = min(n, int(omp))
    return n, ev


def cpu_baseline(p1, p2, budget_s, procs):
    """Oracle CPU baseline on the box's host cores, bounded sample: one process per core
    (independent seeds, BLAS threads = 1), forked BEFORE the GPU is initialised; plus the
    single-core figure."""
    import multiprocessing as mp
    one = _cpu_worker((p1, p2, 0, budget_s / 2))
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(p1, p2, 1 + k, budget_s) for k in range(procs)])
    agg = sum(d / e for d, e in res)
    cores, ev = host_cores()
    ref = None
    try:   # the reference loop itself, measured where it can run (tests/golden/make_ref_rate.py)
        with open(os.path.join(REPO, "tests", "golden", "ref_rate_c2.json")) as f:
            rr = json.load(f)
        ratio = rr["reference_over_port_single_core"]
        ref = {"measured_in": rr["where"], "what": rr["what"],
               "single_core_hyp_per_s": rr["single_core_hyp_per_s"],
               "all_cores_hyp_per_s": rr["all_cores_hyp_per_s"], "all_cores": rr["all_cores"],
               "port_single_core_hyp_per_s_same_host": rr["port_single_core_hyp_per_s"],
               "reference_over_port": ratio,
               "estimated_on_this_host": {"single_core": ratio * one[0] / one[1],
                                          "all_cores": ratio * agg, "cores": procs},
               "note": "the reference modules cannot run on the GPU box; their rate here is the "
                       "port's measured on-box rate times the reference/port ratio measured "
                       "side by side in the build container"}
    except (OSError, KeyError, ValueError):
        pass
    return {"value": agg, "unit": "hypotheses/s", "cores": procs, "kind": "port",
            "host_cores": ev, "reference_loop": ref,
            "single_core_value": one[0] / one[1],
            "sample": f"{sum(d for d, _ in res)} hypotheses of the same C2 pair "
                      f"(N={p1.shape[1]}) through oracle/ransac_ref.ransac_f (numpy, OpenBLAS "
                      f"1 thread) in {procs} processes x {budget_s:.0f} s; single core: "
                      f"{one[0]} hypotheses in {one[1]:.1f} s"}


class _CtxComm:
    """All-gather / max-all-reduce over the RCCL communicator already initialised on ``ctx``."""

    def __init__(self, ctx, rank, world):
        self.ctx, self.rank, self.world = ctx, rank, world

    def allreduce_max_int(self, v):
        x = ctypes.c_int64(int(v))
        _ffi.check(_ffi.lib().rs_comm_allreduce_max_i64(self.ctx.handle, ctypes.byref(x)))
        return int(x.value)

    def allgather_bytes(self, b):
        n = len(b)
        send = np.frombuffer(b, np.uint8).copy()
        recv = np.zeros(n * self.world, np.uint8)
        _ffi.check(_ffi.lib().rs_comm_allgather(self.ctx.handle,
                                                send.ctypes.data_as(ctypes.c_void_p),
                                                recv.ctypes.data_as(ctypes.c_void_p), n))
        return [recv[i * n:(i + 1) * n].tobytes() for i in range(self.world)]


class _HubComm:
    """Fallback record exchange over the harness's TCP hub, used only if the RCCL
    communicator cannot be created (reported as config.exchange)."""

    def __init__(self, dist, rank, world):
        self.hub, self.rank, self.world = dist.hub, rank, world

    def allgather_bytes(self, b):
        return self.hub.allgather_bytes(b)

    def allreduce_max_int(self, v):
        return self.hub.allreduce_max_int(v)


class _Solo:
    rank, world = 0, 1

    def allgather_bytes(self, b):
        return [b]

    def allreduce_max_int(self, v):
        return int(v)


def _blas_info():
    """numpy's BLAS build and the core type it dispatched for (the TRF path follows it)."""
    try:
        import threadpoolctl
        return [{k: d.get(k) for k in ("internal_api", "version", "architecture", "num_threads")}
                for d in threadpoolctl.threadpool_info() if d.get("user_api") == "blas"]
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)}


def _best_of(f, reps):
    best, out = float("inf"), None
    for _ in range(reps):
        t = time.perf_counter()
        out = f()
        best = min(best, time.perf_counter() - t)
    return best, out


def extras(ctx, rank, world, dist, comm):  # noqa: C901
    """The other BASELINE.json configs and the stages after the RANSAC loop, measured on the
    same box (not the headline): C3 PnP, C5 stress, C4 ring (sharded over all ranks, RCCL
    all-gather), the gold standard and the getFFromLabCode drop-in end to end."""
    import itertools
    from tsbb15_amd import fun, parallel, ransac, twoview
    out = {}
    # ---- C4: all C(36,2) pairs of the Dino ring, every rank, one all-gather -------------
    try:
        z = np.load(os.path.join(REPO, "tests", "golden", "dino_pnp_kat.npz"))
        Q = z["points2d"]
        pairs = []
        for i, j in itertools.combinations(range(36), 2):
            vis = np.flatnonzero(np.any(Q[i] != -1, axis=0) & np.any(Q[j] != -1, axis=0))
            pairs.append((np.ascontiguousarray(Q[i][:, vis]), np.ascontiguousarray(Q[j][:, vis])))
        c = comm if comm is not None else _Solo()
        solver = parallel.GpuPairBatchSolver(ctx, 1000)
        refiner = parallel.GpuPairRefiner(ctx, z["K_last"])
        parallel.run_pairs(c, pairs, 1000, solver, refine=refiner)   # warm-up
        ts = []
        for _ in range(5):
            dist.barrier()
            t0 = time.perf_counter()
            tab = parallel.run_pairs(c, pairs, 1000, solver, refine=refiner)
            ts.append(dist.max(time.perf_counter() - t0))
        el = min(ts)
        nv = int((tab["valid"] == 1).sum())
        out["c4_ring"] = {"pairs": len(pairs), "valid_pairs": nv, "n_gpus": world,
                          "hypotheses_per_pair": 1000, "ms": el * 1e3,
                          "pairs_per_s": nv / el, "hypotheses_per_s": nv * 1000 / el,
                          "posed_pairs": int((tab["pose"] > 0).sum()),
                          "stages": "batched RANSAC-F + gold standard + E/relative pose per "
                                    "rank (LPT over ranks), one RCCL all-gather of records"}
    except Exception as e:  # noqa: BLE001
        out["c4_ring"] = {"error": repr(e)}
    if rank != 0:
        return out
    # ---- C3: PnP DLT, M = 500, 30 % outliers, 50 000 hypotheses --------------------------
    try:
        X, _, y, _, _, _ = synth.pnp_scene(500, 0.30, seed=3)
        thr = (1.5 / 800.0) ** 2
        run = lambda: ransac.ransac_pnp(X, y, X, y, 50_000, thr, 6, sampler="philox", seed=11,
                                        ctx=ctx)
        run()
        el, r = _best_of(run, 5)
        # W_P(M) = 27 M + 37 000 flop per hypothesis (the 12 x 12 DLT null
        # space 37 000, scoring 27 per point, ransac.py:93-105); kernel times by HIP events on
        # the context stream around the solve and the count launches, best of 5 timed calls
        _ffi.pnp_timing(ctx, 1)
        ks, kc = [], []
        for _ in range(5):
            run()
            a, b = _ffi.pnp_timing(ctx, 1)
            ks.append(a)
            kc.append(b)
        _ffi.pnp_timing(ctx, 0)
        Hc, Mc = 50_000, 500
        fs, fc = 37_000.0 * Hc, 27.0 * Mc * Hc
        s_ms, c_ms3 = min(ks), min(kc)
        dom = ("k_pnp_solve", fs, s_ms) if s_ms >= c_ms3 else ("k_pnp_count", fc, c_ms3)
        ach = dom[1] / (dom[2] * 1e-3) / 1e12
        out["c3_pnp"] = {"metric": "PnP-DLT RANSAC hypotheses/s", "value": 50_000 / el,
                         "ms": el * 1e3, "points": 500, "hypotheses": 50_000,
                         "consensus": int(r[5]),
                         "roofline": {"bound": "valu (fp64)", "kernel": dom[0],
                                      "achieved": ach, "peak": PEAK_FP64_VALU_TFLOPS,
                                      "unit": "TFLOP/s", "frac": ach / PEAK_FP64_VALU_TFLOPS,
                                      "kernels_ms": {"k_pnp_solve": s_ms, "k_pnp_count": c_ms3},
                                      "flop_per_hypothesis": {"solve": 37_000, "count": 27 * Mc,
                                                              "total": 37_000 + 27 * Mc},
                                      "whole_call_tflops": (fs + fc) / el / 1e12,
                                      "note": "SURVEY.md 8(d) W_P(M) = 27 M + 37 000 flop per "
                                              "hypothesis; HIP events on the context stream, "
                                              "best of 5 calls"}}
        import random
        runp = lambda: ransac.ransac_pnp(X, y, X, y, 50_000, thr, 6, sampler="exact",
                                         rng=random.Random(0))
        runp()
        el, r = _best_of(runp, 5)
        out["c3_pnp_parity"] = {"metric": "PnP-DLT RANSAC hypotheses/s, parity mode "
                                          "(random.seed(0) stream of gen_rnd_indices, parsed "
                                          "on the GPU)",
                                "value": 50_000 / el, "ms": el * 1e3,
                                "best_index": int(r[4]), "consensus": int(r[5])}
    except Exception as e:  # noqa: BLE001
        out["c3_pnp"] = {"error": repr(e)}
    # ---- C5: N = 10 000, 60 % outliers, 1e6 hypotheses (throughput mode) ----------------
    try:
        p1, p2, _ = synth.two_view(10_000, 0.60, seed=5)
        H5 = 1_000_000
        plan = _ffi.F8Plan(ctx, 10_000, H5)
        plan.set_points(p1, p2)
        plan.run(H5, mode=_ffi.SAMPLER_PHILOX, seed=0xC5)
        plan.result()
        def one():
            plan.run(H5, mode=_ffi.SAMPLER_PHILOX, seed=0xC5)
            return plan.result()
        el, (r, inl) = _best_of(one, 3)
        out["c5_stress"] = {"metric": "RANSAC hypotheses/s (8-pt F, 10k corr, 60% outliers)",
                            "value": H5 / el, "ms": el * 1e3, "best_count": int(r.best_count),
                            "guard_mismatch": int(r.guard_mismatch)}
        if rank == 0:
            # the same pair in parity mode: np.random.seed(0), 1e6 numpy-exact choice tuples
            # sampled on the GPU, then the same pipeline.  The first full-size call (which
            # builds the 2^33-word segment jump polynomials and the segment buffers) is
            # reported on its own; then best of 3 warm calls.
            key0, pos0 = _ffi.np_seed(0)
            t = time.perf_counter()
            plan.run_np(H5, key0, pos0)
            plan.result()
            first = time.perf_counter() - t
            el, (rp, _) = _best_of(lambda: (plan.run_np(H5, key0, pos0), plan.result())[1], 3)
            out["c5_parity"] = {"metric": "RANSAC hypotheses/s, parity mode (numpy-exact stream)",
                                "value": H5 / el, "ms": el * 1e3, "first_call_ms": first * 1e3,
                                "timing": "best of 3 after one full-size (1e6) call",
                                "best_index": int(rp.best_index),
                                "best_count": int(rp.best_count)}
        plan.close()
    except Exception as e:  # noqa: BLE001
        out["c5_stress"] = {"error": repr(e)}
    # ---- gold standard on the C2 winner, and getFFromLabCode on the Dino pair ----------
    try:
        p1, p2, _ = synth.two_view(N_CORR, OUTLIERS, seed=1)
        res = fun.ransac_f(p1, p2, r=10_000, rng=np.random.RandomState(0))
        a, b = p1[:, res.inliers], p2[:, res.inliers]
        twoview.gold_standard_batch(res.F[None], [a], [b])
        el, g = _best_of(lambda: twoview.gold_standard_batch(res.F[None], [a], [b])[0], 5)
        out["gold_standard_c2"] = {"inliers": int(a.shape[1]), "ms": el * 1e3,
                                   "iterations": g.iterations, "cost_init": g.cost_init,
                                   "cost": g.cost}
        c1 = np.load(os.path.join(REPO, "tests", "golden", "dino_c1.npz"))
        def getf():
            np.random.seed(0)
            return fun.getFFromLabCode(c1["noisy_p1"], c1["noisy_p2"])
        getf()
        el, Fg = _best_of(getf, 3)
        # the same call's TRF path length: it depends on the host BLAS kernels
        np.random.seed(0)
        rr = fun.ransac_f(c1["noisy_p1"], c1["noisy_p2"])
        gt = twoview.gold_standard_trf_full(rr.F, c1["noisy_p1"][:, rr.inliers],
                                            c1["noisy_p2"][:, rr.inliers])
        gsi = {"nfev": int(gt.nfev), "status": int(gt.status)}
        # F_gold of the drop-in against the reference's own (dino_c1.npz, the unmodified
        # getFFromLabCode in the build container), both scaled to unit Frobenius norm with the
        # sign of the largest entry; the reference's TRF length / termination from its recorded
        # trace (tests/golden/gs_trace.npz, the build container's BLAS)
        def _nF(F):
            F = np.asarray(F, np.float64) / np.linalg.norm(F)
            return F * np.sign(F.flat[np.argmax(np.abs(F))])
        tr = np.load(os.path.join(REPO, "tests", "golden", "gs_trace.npz"))
        out["getFFromLabCode_dino_noisy"] = {
            "ms": el * 1e3, "n_corr": int(c1["noisy_p1"].shape[1]), "iterations": 10_000,
            "gold_standard": fun.GOLD_STANDARD, "trf_nfev": gsi.get("nfev"),
            "trf_status": gsi.get("status"),
            "dF_vs_reference": float(np.abs(_nF(Fg) - _nF(c1["noisy_full_F_gold"])).max()),
            "reference_trf_nfev": int(tr["noisy_nfev"]),
            "reference_trf_status": int(tr["noisy_status"]),
            "reference_trf_note": "the reference's own TRF from its own start in the build "
                                  "container (OpenBLAS SkylakeX, 1 thread); the path length "
                                  "follows the host BLAS; bar |dF| <= 1e-4 (DESIGN.md 2.2)",
            "blas": _blas_info(),
            "note": "drop-in end to end: numpy-exact sampling on the GPU, GPU RANSAC, the "
                    "reference's scipy TRF gold standard over GPU residuals / Jacobian; the "
                    "reference took {:.1f} s for the same call in the build container "
                    "(tests/golden/dino_c1.npz noisy_full_seconds)".format(
                        float(c1["noisy_full_seconds"]))}
        saved = fun.GOLD_STANDARD
        try:
            fun.GOLD_STANDARD = "lm"
            getf()
            el, _ = _best_of(getf, 3)
        finally:
            fun.GOLD_STANDARD = saved
        out["getFFromLabCode_dino_noisy_lm"] = {
            "ms": el * 1e3, "gold_standard": "lm",
            "note": "the same call with the converged GPU Levenberg-Marquardt gold standard"}
    except Exception as e:  # noqa: BLE001
        out["gold_standard_c2"] = {"error": repr(e)}
    # ---- five-point E-RANSAC on the C2 pair (a-15; no reference counterpart) ------------
    try:
        from tsbb15_amd import essential
        p1, p2, _ = synth.two_view(N_CORR, OUTLIERS, seed=1)
        S = 20_000
        essential.ransac_e(p1, p2, synth.K_SYNTH, samples=S, seed=1)
        # (best of 10: a 0.4 ms call whose spread box to box and call to call is ~5 %)
        el, r = _best_of(lambda: essential.ransac_e(p1, p2, synth.K_SYNTH, samples=S, seed=1), 10)
        out["e5_ransac_c2"] = {"metric": "five-point E-RANSAC minimal samples/s", "value": S / el,
                               "ms": el * 1e3, "samples": S, "hypotheses": 10 * S,
                               "consensus": r.count,
                               "round2_value": E5_ROUND2[0], "round2_source": E5_ROUND2[1],
                               "note": "k_e5_build (null basis, ten cubics) + k_e5_gj (Gauss-"
                                       "Jordan, 32 lanes per sample) + k_e5_roots (16 lanes per "
                                       "sample, a lane per root) + k_e5_pack (the real "
                                       "solutions' slots) + k_f8_count32q over those + selection, "
                                       "N = 2000"}
    except Exception as e:  # noqa: BLE001
        out["e5_ransac_c2"] = {"error": repr(e)}
    # ---- per-view table steps (tables.py:116-175, 260-380) at the reference's noisy sizes ----
    try:
        from tsbb15_amd import tables as gt
        z = np.load(os.path.join(REPO, "tests", "golden", "tables.npz"))
        g = lambda k: z["noisy_" + k]
        nC, nP = int(g("ba_n_views")), int(g("ba_n_points"))
        x = g("ba_x_final")
        cams, pts = x[:12 * nC].reshape(nC, 3, 4), x[12 * nC:].reshape(nP, 3)
        view, point, uv = g("ba_obs_view"), g("ba_obs_point"), g("ba_obs_coords")[:, :2]
        steps = {
            "match_observations": lambda: gt.match_observations(
                g("match_obs_coords"), g("match_obs_point"), g("match_queries")),
            "add_new_points": lambda: gt.add_new_points(g("new_y1_hom"), g("new_y2_hom"),
                                                         g("new_C1"), g("new_C2")),
            "ba_residuals": lambda: gt.ba_residuals(cams, pts, view, point, uv),
            "ba_jacobian": lambda: gt.ba_jacobian(cams, pts, view, point),
        }
        rec = {}
        for name, f in steps.items():
            f()
            rec[name + "_ms"] = _best_of(f, 10)[0] * 1e3
        rec.update({"observations": int(len(view)), "queries": int(len(g("match_queries"))),
                    "new_points": int(len(g("new_y1_hom"))),
                    "note": "one host call each (H2D + launch + D2H), latency-bound sizes"})
        out["tables_noisy"] = rec
    except Exception as e:  # noqa: BLE001
        out["tables_noisy"] = {"error": repr(e)}
    return out


# the counting kernel the plan runs: fp32 with the float64 guard re-test, or (RSAMD_COUNT=fp64,
# tools only) the plain float64 kernel
COUNT_KERNEL = {"fp32": "k_f8_count32q", "fp64": "k_f8_count"}


COUNT_BYTES_PER_HYP, COUNT_BYTES_PER_POINT = 9 * 4 + 16 + 4, 16

# e5_ransac_c2 before the scratch cut (k_e5_solve kept all ten solutions in a per-lane array:
# 1664 B of scratch per lane), as the round-2 driver bench measured it
E5_ROUND2 = (13389928.829414358, "BENCH_r02.json extras.e5_ransac_c2.value (1.494 ms / 20000)")


def load_pmc(n_corr, hyps):
    """The newest committed rocprofv3 summary of the counting kernel (profiles/r*_pmc_k_f8_count
    .json, tools/pmc_summary.py) for this workload: HBM bytes per launch from the PMC passes and
    the C2-only kernel-trace average.  Returns (hbm_bytes, record) or (None, None)."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_k_f8_count.json")))
    if not found:
        return None, None
    path = found[-1]
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("n_corr") == n_corr and d.get("hypotheses") == hyps:
            return d.get("hbm_bytes_per_launch"), dict(d, source=os.path.relpath(path, REPO))
    except Exception:
        return None, None
    return None, None


def _free_port_pair():
    """A port P with P and P + 1 both free on 127.0.0.1 (MASTER_PORT and the TcpHub's)."""
    import socket
    for _ in range(64):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
        if p >= 65535:
            continue
        try:
            with socket.socket() as a, socket.socket() as b:
                a.bind(("127.0.0.1", p))
                b.bind(("127.0.0.1", p + 1))
            return p
        except OSError:
            continue
    raise RuntimeError("no free port pair on 127.0.0.1")


def _die_with_parent():
    """preexec_fn of a rank process: SIGKILL it if the launcher dies (prctl PR_SET_PDEATHSIG),
    so a launcher killed by a time limit leaves no rank holding a GPU."""
    import signal
    ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGKILL), 0, 0, 0)


def launch_ranks(n, argv):
    """``bench.py --gpus N`` without a launcher: start N rank processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, the same as torch.distributed.run
    --nproc-per-node N would) BEFORE anything in this process touches a GPU (nothing here
    loads librsamd), wait for all of them, and re-print rank 0's single JSON line after
    checking it reports ``n_gpus == N``.  Any rank failing ends the others and the launcher
    exits non-zero with that rank's status; so does a line whose world differs.  Ranks other
    than 0 write their stdout to stderr."""
    import subprocess
    import threading
    port = _free_port_pair()
    procs, out0 = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), RSAMD_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      preexec_fn=_die_with_parent))
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = None
    while any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if p.poll() not in (None, 0) and failed is None:
                failed = (r, p.returncode)
        if failed:
            break
        time.sleep(0.1)
    if failed is None:
        failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode), None)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"error: bench rank {failed[0]} of {n} exited with status {failed[1]}",
              file=sys.stderr)
        return failed[1] if failed[1] > 0 else 1
    reader.join(timeout=30)
    text = (out0[0] if out0 else b"").decode(errors="replace")
    lines = [s for s in text.splitlines() if s.startswith("{")]
    if len(lines) != 1:
        print(f"error: rank 0 printed {len(lines)} JSON lines, expected 1", file=sys.stderr)
        return 1
    got = json.loads(lines[0]).get("n_gpus")
    if got != n:
        print(f"error: the ranks formed a world of {got}, --gpus asked for {n}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def exchange_policy(rccl_ok, pinned):
    """The per-pair record exchange of a multi-rank bench, decided on every rank alike.
    RCCL when its communicator came up on every rank.  Otherwise: a one-device rehearsal
    (RSAMD_BENCH_DEVICE pins every rank to one GPU, which RCCL refuses) exchanges over the TCP
    hub and says so; ranks on distinct GPUs raise instead -- a multi-GPU line must be an RCCL
    measurement or no line at all."""
    if rccl_ok:
        return "rccl all-gather"
    if pinned:
        return "tcp-hub all-gather (RCCL init failed; one-device rehearsal)"
    raise RuntimeError("RCCL communicator init failed on some rank while the ranks hold distinct "
                       "GPUs: refusing to report a multi-GPU line without RCCL")


def harness_only(rank, world, dist, args, cpu):
    """--harness-only: the launcher + TcpHub handshake, barrier, max-reduce and all-gather
    with no device opened (the CPU test of the multi-rank harness).  RSAMD_BENCH_FAKE_RCCL
    ("fail" / "ok") runs the transport decision of a real run on a simulated RCCL init."""
    import platform
    dist.barrier()
    t = dist.max(float(rank))
    info = {"rank": rank, "local_rank": dist_env()[1], "pid": os.getpid(),
            "host": platform.node(), "launched": os.environ.get("RSAMD_BENCH_LAUNCHED") == "1"}
    recs = [json.loads(b) for b in dist.hub.allgather_bytes(json.dumps(info).encode())] \
        if dist.hub else [info]
    line = {"harness_only": True, "n_gpus": world, "max_rank": t, "ranks": recs,
            "harness": "tcp hub (no torch.distributed)" if world > 1 else "one process"}
    fake = os.environ.get("RSAMD_BENCH_FAKE_RCCL")
    if fake and world > 1:
        ok = dist.max(0.0 if fake == "ok" else 1.0) == 0.0
        try:
            line["exchange"] = exchange_policy(ok, "RSAMD_BENCH_DEVICE" in os.environ)
        except RuntimeError as e:
            print(f"error: {e}", file=sys.stderr, flush=True)
            dist.close()
            sys.exit(4)
    if cpu is not None:
        line["cpu_baseline"] = cpu
    dist.barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)


def load_traffic():
    """The newest committed calibrated-traffic summary (profiles/r*_traffic.json,
    tools/traffic_summary.py): FETCH_SIZE / WRITE_SIZE factors measured per access shape on a
    known byte count, applied to the counting kernel's and the parse kernels' PMC passes."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_traffic.json")))
    if not found:
        return None
    try:
        with open(found[-1]) as f:
            d = json.load(f)
        d["source"] = os.path.relpath(found[-1], REPO)
        return d
    except (OSError, ValueError):
        return None


def load_parse_traffic():
    d = load_traffic()
    if not d or "parse" not in d:
        return None
    return dict(d["parse"], source=d["source"])


def load_clock():
    """The clock the counting kernel holds (newest committed profiles/r*_count_clock.json)."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_count_clock.json")))
    if not found:
        return None
    try:
        with open(found[-1]) as f:
            d = json.load(f)
        return {"held_clock_ghz": d["held_clock_ghz"], "source": os.path.relpath(found[-1], REPO),
                "valu_bound_us_at_held_clock": d.get("valu_bound_us_at_held_clock")}
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--hyps", type=int, default=HYPS)
    ap.add_argument("--n", type=int, default=N_CORR)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="oracle worker processes (default: host_cores())")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-mode", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-fp64-count", action="store_true")
    ap.add_argument("--fp64-steps", type=int, default=20)
    ap.add_argument("--no-split-projection", action="store_true")
    ap.add_argument("--harness-only", action="store_true",
                    help="launcher + TcpHub handshake only, no device (CPU test)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: this process becomes one, before any HIP call
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank, local_rank, world = dist_env()
    if world != args.gpus:
        sys.exit(f"error: WORLD_SIZE={world} but --gpus={args.gpus}; run "
                 f"'bench.py --gpus N' alone (it starts its N ranks) or under "
                 f"torch.distributed.run --nproc-per-node N")
    if args.harness_only:
        if os.environ.get("RSAMD_BENCH_FAIL_RANK") == str(rank):
            sys.exit(3)   # before the hub handshake: the other ranks would wait on it
        dist = Dist(world)
        cpu = None
        if rank == 0 and not args.no_cpu_baseline:
            cp1, cp2, _ = synth.two_view(args.n, OUTLIERS, seed=1)
            cpu = cpu_baseline(cp1, cp2, args.cpu_seconds, args.cpu_procs or host_cores()[0])
        harness_only(rank, world, dist, args, cpu)
        dist.close()
        return
    dist = Dist(world)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # before any HIP call of this process: the worker processes are forked from it.  At
        # world > 1 the other ranks wait for rank 0 at the first hub exchange meanwhile (their
        # GPUs idle: nothing of the timed region overlaps the CPU baseline)
        cp1, cp2, _ = synth.two_view(args.n, OUTLIERS, seed=1)
        cpu = cpu_baseline(cp1, cp2, args.cpu_seconds, args.cpu_procs or host_cores()[0])
    # RSAMD_BENCH_DEVICE pins every rank to one device: a multi-rank rehearsal on a one-GPU
    # box (RCCL refuses two ranks on one GPU, so that run exercises the TCP-hub exchange)
    ctx = _ffi.Context(int(os.environ.get("RSAMD_BENCH_DEVICE", local_rank)))

    # one synthetic pair per rank (weak scaling: per-GPU work fixed); p0_* is rank 0's pair
    p1, p2, _ = synth.two_view(args.n, OUTLIERS, seed=1 + rank)
    p0_1, p0_2, _ = synth.two_view(args.n, OUTLIERS, seed=1)
    H = args.hyps
    plan = _ffi.F8Plan(ctx, args.n, H)
    plan.set_points(p1, p2)
    # each HIP timing event is a marker packet between two kernels (~3.5 us): time the
    # counting kernel on every TIMING_EVERY-th run of the timed region, not on every run
    plan.set_timing(1, min(TIMING_EVERY, max(1, args.steps)))

    comm = world > 1
    exchange = "none (one GPU)"
    comm_ranks = [{"rank": 0, "device": ctx.device}]
    if comm:
        uid = np.zeros(_ffi.COMM_ID_BYTES, np.uint8)
        st = 0
        if rank == 0:
            with _stdout_to_stderr():
                st = _ffi.lib().rs_comm_unique_id(_ffi.ptr(uid, ctypes.c_uint8))
        uid = np.frombuffer(dist.bcast_bytes(uid.tobytes()), np.uint8).copy()
        if st == 0:
            with _stdout_to_stderr():
                st = _ffi.lib().rs_comm_init(ctx.handle, world, rank, _ffi.ptr(uid, ctypes.c_uint8))
        ok = dist.max(0.0 if st == 0 else 1.0) == 0.0   # every rank agrees on the transport
        try:
            exchange = exchange_policy(ok, "RSAMD_BENCH_DEVICE" in os.environ)
        except RuntimeError as e:
            print(f"error: {e} (this rank: status {st}: "
                  f"{_ffi.lib().rs_last_error().decode(errors='replace')})", file=sys.stderr,
                  flush=True)
            if st == 0:
                _ffi.lib().rs_comm_destroy(ctx.handle)
            dist.close()
            sys.exit(4)
        if ok:
            xcomm = _CtxComm(ctx, rank, world)
        else:
            if st == 0:
                _ffi.lib().rs_comm_destroy(ctx.handle)
            print(f"warning: RCCL communicator init failed on some rank (status {st}: {_ffi.lib().rs_last_error().decode(errors='replace')}); "
                  "exchanging the per-pair records over the TCP hub", file=sys.stderr)
            xcomm = _HubComm(dist, rank, world)
        # the first collective on a communicator sets up its channels (lazy, can take far
        # longer than the timed steps): do it before the timed region.  Its payload is every
        # rank's (rank, device): the communicator's own world and device map, in the line
        me = np.zeros(12, np.int64)
        me[0], me[1] = rank, ctx.device
        got = np.frombuffer(b"".join(xcomm.allgather_bytes(me.tobytes())), np.int64).reshape(-1, 12)
        comm_ranks = [{"rank": int(g[0]), "device": int(g[1])} for g in got]
        if [r["rank"] for r in comm_ranks] != list(range(world)):
            sys.exit(f"error: the communicator's all-gather returned ranks "
                     f"{[r['rank'] for r in comm_ranks]}, expected 0..{world - 1}")

    rccl_lib = None
    if comm:
        try:
            v, path = _ffi.rccl_library()
            rccl_lib = {"version": v, "path": path, "torch_imported": "torch" in sys.modules}
        except Exception as e:  # noqa: BLE001
            rccl_lib = {"error": repr(e)}
        rccl_lib["rank"], rccl_lib["device"] = rank, ctx.device
        # every rank's record: which library each process actually loaded
        rccl_lib = [json.loads(b) for b in
                    dist.hub.allgather_bytes(json.dumps(rccl_lib).encode())]

    def step(i):
        # one full RANSAC run; runs are stream-ordered and issued back to back (each run
        # copies its own result record + S_RANSAC into its own pinned slot)
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=0xC2, hyp_offset=i * H)

    for i in range(args.warmup):
        step(i)
    plan.result()
    ctx.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    r, inl = plan.result()          # waits for the last run
    assert r.best_count > 0 and len(inl) == r.best_count
    if comm:  # all-gather of the per-pair best models (F, count, index) over RCCL
        rec = np.zeros(12, np.float64)
        rec[:9] = r.F[:]
        rec[9], rec[10], rec[11] = r.best_count, r.best_index, rank
        out = np.frombuffer(b"".join(xcomm.allgather_bytes(rec.tobytes())), np.float64)
        assert int(out.reshape(world, 12)[rank, 11]) == rank
    ctx.synchronize()
    el = time.perf_counter() - t0
    dist.barrier()
    el = dist.max(el)
    total_hyps = H * args.steps * world
    value = total_hyps / el

    try:
        km = plan.kernel_ms(last_n=args.steps)   # HIP events of the timed runs (<= 64)
    except ValueError:  # RSAMD_TIMING=0: no per-run events (A/B of their marker cost)
        km = {"count_ms": float("nan"), "solve_ms": -1.0, "total_ms": -1.0}
    km = {k: (None if v is not None and v < 0 else v) for k, v in km.items()}
    c_ms = km["count_ms"]
    # 42 flop per (hypothesis, correspondence) of the reference's float64
    # score; the kernel computes it in fp32 with an exact fp64 guard band, so the bounding
    # peak is the FP32 vector rate (its FP64 fraction is reported beside it)
    achieved = H * FLOP_PER_CORR * args.n / (c_ms * 1e-3) / 1e12
    pmc, pmc_rec = load_pmc(args.n, H)
    pmc_raw, tcorr = pmc, None
    trd = load_traffic()
    if pmc and trd and "count" in trd and trd["count"].get("n_corr") == args.n and \
            trd["count"].get("hypotheses") == H:
        # FETCH_SIZE corrected per access shape (calibrated on known bytes, profiles/r*_traffic)
        pmc = trd["count"]["hbm_bytes_corrected"]
        tcorr = {k: trd["count"][k] for k in ("fetch_raw", "write_raw", "fetch_corrected",
                                               "factors", "method") if k in trd["count"]}
        tcorr["source"] = trd["source"]
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "hypotheses/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (exact f64 guard band; f64 solve / re-score)",
        "data": "synthetic (tsbb15_amd.synth.two_view, SURVEY.md 8(d) scene; one pair per GPU)",
        "config": {"workload": "C2: synthetic two-view pair, N=2000 correspondences, 30% "
                               "outliers, 100000 hypotheses per RANSAC run, 8-point F, "
                               "threshold 1.5 px",
                   "n_corr": args.n, "hypotheses_per_step": H, "sampler": "philox (throughput)",
                   "parallelism": f"pairs sharded, {world} pair(s) on {world} GPU(s)",
                   "exchange": exchange, "exchange_library": rccl_lib,
                   "comm_world": len(comm_ranks), "rank_devices": comm_ranks,
                   "harness": "tcp hub (no torch.distributed)" if world > 1 else "one process"},
        "roofline": {"bound": "valu", "kernel": COUNT_KERNEL["fp64" if os.environ.get("RSAMD_COUNT") == "fp64"
                                                         else "fp32"],
                     "achieved": achieved, "peak": PEAK_FP32_VALU_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP32_VALU_TFLOPS,
                     "traffic": pmc,
                     "traffic_raw_pmc": pmc_raw,
                     "traffic_correction": tcorr,
                     # algorithmic HBM bytes of one counting launch: per hypothesis the fp32
                     # model (36 B) + its guard-band float4 (16 B) + the count (4 B); the packed
                     # points once (16 B each); PMC traffic / this = re-read factor
                     "algorithmic_bytes": H * COUNT_BYTES_PER_HYP + args.n * COUNT_BYTES_PER_POINT,
                     "traffic_over_algorithmic": (pmc / (H * COUNT_BYTES_PER_HYP + args.n * COUNT_BYTES_PER_POINT)
                                                  if pmc else None),
                     "per_launch": {"hypotheses": H, "flop": H * FLOP_PER_CORR * args.n,
                                    "avg_ms": c_ms, "timed_launches_every": TIMING_EVERY},
                     # the same kernel in the committed C2-only rocprofv3 kernel trace (a
                     # profiled run on the profiling box: DVFS and the box set both figures)
                     "rocprof_c2_avg_us": (pmc_rec["rocprof_c2_avg_ns"] / 1e3
                                           if pmc_rec and pmc_rec.get("rocprof_c2_avg_ns") else None),
                     "rocprof_c2_frac": (H * FLOP_PER_CORR * args.n / (pmc_rec["rocprof_c2_avg_ns"] * 1e-9)
                                         / 1e12 / PEAK_FP32_VALU_TFLOPS
                                         if pmc_rec and pmc_rec.get("rocprof_c2_avg_ns") else None),
                     "rocprof_source": pmc_rec["source"] if pmc_rec else None,
                     "whole_run_nominal": {
                         "flop_per_hypothesis": FLOP_PER_CORR * args.n + FLOP_SOLVE,
                         "tflops": value * (FLOP_PER_CORR * args.n + FLOP_SOLVE) / 1e12,
                         "note": "SURVEY.md 8(d)'s nominal 15 000 flop per solve is an SVD "
                                 "estimate; the LQ solve does far less, so this is not a "
                                 "roofline figure"},
                     "note": "vector-ALU (issue) bound, SURVEY.md 8(d): 42 flop per "
                             "(hypothesis, correspondence) algorithmic; HBM traffic per launch "
                             "from rocprofv3 PMC in profiles/ (traffic, bytes)"},
        "kernels_ms": {"k_f8_count32q": c_ms, "k_f8_solve": km["solve_ms"],
                       "run_device_total": km["total_ms"]},
    }
    clk = load_clock()
    if clk:
        # DVFS: under this launch the chip holds ~1.95 GHz, not the 2.4 GHz of the nominal
        # peak; the fraction of the peak at the held clock (measured in-kernel, committed)
        peak_held = PEAK_FP32_VALU_TFLOPS * clk["held_clock_ghz"] / 2.4
        line["roofline"]["held_clock"] = dict(clk, peak_at_held_clock=peak_held,
                                              frac_at_held_clock=achieved / peak_held)
    if pmc:
        line["hbm_roofline"] = {"bound": "hbm", "achieved": pmc / (c_ms * 1e-3) / 1e9,
                                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": pmc / (c_ms * 1e-3) / 1e9 / PEAK_HBM_GBS}

    if not args.no_fp64_count:
        # the plain float64 counting kernel on the same runs: the precision question settled
        # by measurement (identical counts; bounded by the FP64 vector peak)
        plan.set_count_precision(True)
        for i in range(20):
            step(i)
        plan.result()
        dist.barrier()
        t = time.perf_counter()
        for i in range(args.fp64_steps):
            step(i)
        plan.result()
        el64 = dist.max(time.perf_counter() - t)
        k64 = plan.kernel_ms(last_n=args.fp64_steps)["count_ms"]
        plan.set_count_precision(False)
        a64 = H * FLOP_PER_CORR * args.n / (k64 * 1e-3) / 1e12
        line["fp64_count"] = {"value": H * args.fp64_steps * world / el64,
                              "unit": "hypotheses/s", "kernel": "k_f8_count",
                              "kernel_ms": k64, "achieved": a64, "peak": PEAK_FP64_VALU_TFLOPS,
                              "unit_roofline": "TFLOP/s", "frac": a64 / PEAK_FP64_VALU_TFLOPS,
                              "note": "RANSAC runs with the plain float64 counting kernel "
                                      "(reference-order residuals); counts are bit-identical "
                                      "to the fp32 + exact-guard-band default"}

    if not args.no_parity_mode:
        # numpy-exact sampling + the same GPU pipeline: the np.random stream parsed on the
        # GPU (rs_f8_plan_run_np).  Weak: every rank its own pair's run.  Sharded: ONE pair's
        # H hypotheses split over the ranks (rs_f8_plan_run_np_slice + c* all-reduce and
        # candidate all-gather), the fun.py:320-328 decision replayed on every rank.
        from tsbb15_amd import fun, parallel
        key0, pos0 = _ffi.np_seed(0)
        # the drop-in's first call (fun.ransac_f, the loop of getFFromLabCode) at this N in this
        # process: a fresh context -- new plan, new parse buffers -- and jump polynomials not
        # built yet; then the same call warm
        hs0 = _ffi.np_host_stats()
        cnew = _ffi.Context(ctx.device)
        t = time.perf_counter()
        fun.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0), ctx=cnew)
        first_call = time.perf_counter() - t
        hs1 = _ffi.np_host_stats()
        warm_call, _ = _best_of(lambda: fun.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0),
                                                     ctx=cnew), 3)
        cnew.close()
        tg = []
        for _ in range(6):
            dist.barrier()
            t = time.perf_counter()
            plan.run_np(H, key0, pos0)
            rser, _ = plan.result()
            tg.append(dist.max(time.perf_counter() - t))
        # the same run once more with HIP events between the parse's steps (rs_np_timing:
        # markers cost a few microseconds each, so the timed runs above carry none)
        _ffi.np_timing(ctx, 1)
        t = time.perf_counter()
        plan.run_np(H, key0, pos0)
        plan.result()
        wall_split = time.perf_counter() - t
        steps, nbytes, nseg = _ffi.np_timing(ctx, 0)
        kms = {k: v for k, v in steps.items()}
        kms["evaluate_and_host"] = wall_split * 1e3 - steps["parse_total"]
        kms["wall"] = wall_split * 1e3
        kms["segments"] = nseg
        kms["note"] = ("HIP events on the context stream between the parse's steps of one C2 "
                       "run (stream_pass2 on the second stream, beside entry; entry includes "
                       "its wait for pass 2); evaluate_and_host = wall - parse_total (solve, "
                       "count, selection, result copy and host calls)")
        alg = sum(nbytes.values())
        hbm = {"bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
               "algorithmic_bytes": dict(nbytes, total=alg),
               "achieved": alg / (steps["parse_total"] * 1e-3) / 1e9,
               "frac": alg / (steps["parse_total"] * 1e-3) / 1e9 / PEAK_HBM_GBS,
               "per_step_gbs": {
                   "stream (written, both passes)": nbytes["stream_written"] / max(
                       1e-9, (steps["stream_pass1"] + steps["stream_pass2"]) * 1e-3) / 1e9,
                   "entry + track (chunk draws read)": nbytes["parse_read"] / max(
                       1e-9, (steps["entry"] + steps["track"]) * 1e-3) / 1e9,
                   "tuples (hypothesis draws read)": nbytes["tuples_read"] / max(
                       1e-9, steps["tuples"] * 1e-3) / 1e9},
               "note": "algorithmic bytes of the parse of one C2 run (the MT words written once, "
                       "every chunk draw read once by entry + track, every hypothesis's draws "
                       "read once by the tuple kernel) / the parse's HIP-event time; measured "
                       "(calibrated PMC) bytes in `measured`"}
        tmeas = load_parse_traffic()
        if tmeas:
            hbm["measured"] = tmeas
        pm = {"value": world * H / min(tg[1:]), "unit": "hypotheses/s",
              "ms": 1e3 * min(tg[1:]), "scaling": "weak", "n_gpus": world,
              "kernels_ms": kms, "hbm": hbm,
              "first_call_ms": first_call * 1e3, "warm_call_ms": warm_call * 1e3,
              "first_call_host_jump_ms": hs1[0] - hs0[0],
              "first_call_note": "fun.ransac_f (getFFromLabCode's RANSAC, fun.py:298-328) on a "
                                 "fresh context at this N: plan and parse buffers allocated, MT "
                                 "jump polynomials built on the host (host_jump_ms); warm = best "
                                 "of 3 of the same call",
              "note": "np.random legacy stream (seed 0) reproduced bit-exactly on the GPU "
                      "(MT19937 jump-ahead windows, all-entry-state chunk parse + windowed "
                      "tracking, per-hypothesis swap trace), then the same GPU pipeline; one "
                      "pair per rank"}
        if world > 1:
            # ONE pair's H hypotheses over all ranks with the stream parse itself split: each
            # rank parses its share of the chunks, the chunk maps are all-gathered and composed
            # everywhere, each rank evaluates the hypotheses starting in its share
            c = xcomm
            sp = _ffi.F8Plan(ctx, args.n, H)
            sp.set_points(p0_1, p0_2)
            sh = _ffi.NpShard(ctx, args.n, 8, world, rank)
            ts = []
            for _ in range(4):
                dist.barrier()
                t = time.perf_counter()
                best, _, _ = parallel.ransac_f_split_np(c, ctx, p0_1, p0_2, H, key0, pos0,
                                                        plan=sp, shard=sh)
                ts.append(dist.max(time.perf_counter() - t))
            sh.close()
            sp.close()
            pm["sharded"] = {"value": H / min(ts[1:]), "unit": "hypotheses/s",
                             "ms": 1e3 * min(ts[1:]), "scaling": "strong", "n_gpus": world,
                             "best_index": int(best["index"]) if best is not None else -1,
                             "note": "one pair's H hypotheses over all ranks, the numpy stream "
                                     "parse split by chunk (rs_np_shard_*: per-rank parse, "
                                     "all-gather + compose of the chunk maps, start-count scan), "
                                     "then the c* all-reduce + candidate all-gather"}
        if rank == 0 and world == 1 and not args.no_split_projection:
            # the split parse's per-rank cost at W = 1/2/4/8, every rank's steps timed alone
            # on this GPU (a projection: the collectives between the steps are not timed)
            proj = {"label": "PROJECTION from one GPU (each emulated rank's steps run alone, "
                             "back to back; collectives not timed), not a multi-GPU measurement",
                    "serial_ms": pm["ms"], "worlds": {}}
            for W in (1, 2, 4, 8):
                pls = []
                for _ in range(W):
                    pl = _ffi.F8Plan(ctx, args.n, H)
                    pl.set_points(p1, p2)
                    pls.append(pl)
                shs = [_ffi.NpShard(ctx, args.n, 8, W, r) for r in range(W)]
                reps = []
                for _ in range(3):
                    rep, best, k2, ps2 = parallel.project_split_np(ctx, p1, p2, H, key0, pos0, W,
                                                                   plans=pls, shards=shs)
                    reps.append(rep)
                for o in pls + shs:
                    o.close()
                rep = min(reps[1:], key=lambda d: d["projected_ms"])
                rep["winner_equals_serial"] = bool(best is not None
                                                   and int(best["index"]) == int(rser.best_index))
                rep["strong_scaling_efficiency"] = pm["ms"] / (W * rep["projected_ms"])
                proj["worlds"][str(W)] = rep
            pm["split_projection"] = proj
        if rank == 0 and world == 1:
            th = []
            for _ in range(2):
                t = time.perf_counter()
                tup, _, _ = _ffi.np_choice_tuples(key0, pos0, args.n, 8, H)
                plan.run(H, mode=_ffi.SAMPLER_TUPLES, tuples=tup)
                plan.result()
                th.append(time.perf_counter() - t)
            pm["host_replay_value"] = H / min(th)
        line["parity_mode"] = pm
    if cpu is not None:
        line["cpu_baseline"] = cpu
    if not args.no_extras:
        ex = extras(ctx, rank, world, dist, xcomm if comm else None)
        if rank == 0:
            line["extras"] = ex
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm and isinstance(xcomm, _CtxComm):
        _ffi.lib().rs_comm_destroy(ctx.handle)
    plan.close()
    dist.close()


if __name__ == "__main__":
    main()
