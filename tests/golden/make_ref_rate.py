"""The reference loop's own rate at C2, measured in the build container (a labelled fixture
for bench.py's cpu_baseline; the reference never travels to the GPU box).

Imports the reference exactly as make_golden.py does (import-only cv2 stub) and times the
hypothesis loop of fun.py:303-328 on the C2 pair (synth.two_view(2000, 0.30, seed=1), the
bench's pair) with the reference's own lab3.fmatrix_stls / lab3.fmatrix_residuals
(make_golden._ref_loop, cross-checked there against the unmodified getFFromLabCode):

  * one core (OpenBLAS 1 thread), ~20 s;
  * every core of this container, one process per core (BLAS 1 thread each), ~20 s.

Writes tests/golden/ref_rate_c2.json.
Usage:  python tests/golden/make_ref_rate.py [--seconds 20]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = "1"
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))


def _timed(args):
    seconds, seed = args
    import make_golden as mg
    lab3, _, _, _ = mg.import_reference()
    from tsbb15_amd import synth
    p1, p2, _ = synth.two_view(2000, 0.30, seed=1)
    np.random.seed(seed)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        mg._ref_loop(lab3, p1, p2, 100)
        done += 100
    return done, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    a = ap.parse_args()
    import multiprocessing as mp
    one = _timed((a.seconds, 0))
    procs = len(os.sched_getaffinity(0))
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_timed, [(a.seconds, 1 + k) for k in range(procs)])
    # the oracle port (bench.py's cpu_baseline leg) on the same host, one core: the ratio
    # carries the reference's rate over to the GPU box's host, where only the port can run
    sys.path.insert(0, REPO)
    import bench
    from tsbb15_amd import synth
    p1, p2, _ = synth.two_view(2000, 0.30, seed=1)
    pd, pe = bench._cpu_worker((p1, p2, 0, a.seconds))
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    out = {
        "what": "fun.py:303-328 hypothesis loop with the reference's own lab3.fmatrix_stls / "
                "lab3.fmatrix_residuals (tests/golden/make_golden.py _ref_loop), C2 pair "
                "synth.two_view(2000, 0.30, seed=1)",
        "where": "build container (the reference is not on the GPU box)",
        "single_core_hyp_per_s": one[0] / one[1],
        "single_core_sample": f"{one[0]} hypotheses in {one[1]:.1f} s",
        "all_cores_hyp_per_s": sum(d / e for d, e in res),
        "all_cores": procs,
        "all_cores_sample": f"{sum(d for d, _ in res)} hypotheses, {procs} processes x "
                            f"{a.seconds:.0f} s",
        "port_single_core_hyp_per_s": pd / pe,
        "reference_over_port_single_core": (one[0] / one[1]) / (pd / pe),
        "cpu": cpu, "python": platform.python_version(), "numpy": np.__version__,
        "blas_threads": 1,
    }
    with open(os.path.join(HERE, "ref_rate_c2.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
