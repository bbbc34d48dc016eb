"""Summarise a gpu_round.sh output directory into profiles/: rocprofv3 --stats kernel table
and per-launch PMC counters of the dominant kernel.

  python tools/pmc_summary.py gpurun_out/<tag> <round-tag>

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE
reads half the bytes only for 16-B-per-lane streaming reads.  The count kernel's HBM-side
reads are 8-B-per-lane model loads (uncalibrated width), so both the raw sum and the
2x-corrected upper bound are recorded; `hbm_bytes_per_launch` is the raw (FETCH+WRITE)*1024.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

KERNEL = "k_f8_count32q"
# v_fma_f64 per executed float64 re-test (test64, one per ambiguous point of a pair; the
# kernel's only float64 FMAs, counted in its ISA)
FMA64_PER_RETEST = 10


def per_launch(path, kernel):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0].split("<")[0].endswith(kernel) or \
                r["Kernel_Name"].startswith(kernel + "<"):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "prof", "bench_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "prof_all", "bench_kernel_stats.csv")):
        shutil.copy(os.path.join(src, "prof_all", "bench_kernel_stats.csv"),
                    os.path.join(prof, f"{tag}_kernel_stats_all.csv"))
    bench = json.load(open(os.path.join(src, "bench.json")))
    counters, launches = {}, {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sqc"):
        p = os.path.join(src, sub, "pmc_counter_collection.csv")
        if os.path.exists(p):
            c, n = per_launch(p, KERNEL)
            counters.update(c)
            launches.update(n)
    stats = {r["Name"].split("(")[0]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                       "pct": float(r["Percentage"])}
             for r in csv.DictReader(open(os.path.join(src, "prof", "bench_kernel_stats.csv")))}
    # the C2-only kernel trace: every k_f8_count32q launch is C2-size; the timed steps are the
    # last `steps` launches of the trace
    c2 = [r for r in csv.DictReader(open(os.path.join(src, "prof", "bench_kernel_trace.csv")))
          if KERNEL in r["Kernel_Name"]]
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c2]
    steps = int(bench["steps"])
    c2_all_ns = sum(dur) / len(dur) if dur else None
    c2_timed_ns = sum(dur[-steps:]) / len(dur[-steps:]) if dur else None
    fetch = counters.get("FETCH_SIZE", 0.0) * 1024
    write = counters.get("WRITE_SIZE", 0.0) * 1024
    out = {
        "kernel": KERNEL,
        "n_corr": bench["config"]["n_corr"],
        "hypotheses": bench["config"]["hypotheses_per_step"],
        "counters_per_launch": counters,
        "launches_sampled": launches,
        "hbm_bytes_per_launch": fetch + write,
        "hbm_bytes_per_launch_fetch_x2_upper": 2 * fetch + write,
        "kernel_stats_avg_ns": next((v["avg_ns"] for k, v in stats.items() if KERNEL in k), None),
        "rocprof_c2_launches": len(dur),
        "rocprof_c2_avg_ns": c2_all_ns,
        "rocprof_c2_timed_avg_ns": c2_timed_ns,
        "rocprof_c2_note": "rocprofv3 --kernel-trace of bench.py with --no-parity-mode --no-fp64-count "
                           "--no-extras: every k_f8_count32q launch is a C2 launch (warm-up + steps); "
                           "timed = the last `steps` launches",
        "bench_hip_event_avg_ms": bench["kernels_ms"].get("k_f8_count32q",
                                                          bench["kernels_ms"].get("k_f8_count")),
        "valu_insts_per_wave_point": (counters.get("SQ_INSTS_VALU", 0.0) /
                                      (bench["config"]["hypotheses_per_step"] *
                                       bench["config"]["n_corr"] / 64.0)),
        "retests_per_launch_est": counters.get("SQ_INSTS_VALU_FMA_F64", 0.0) / FMA64_PER_RETEST,
        "ambiguous_pair_rate_est": (counters.get("SQ_INSTS_VALU_FMA_F64", 0.0) / FMA64_PER_RETEST /
                                    (bench["config"]["hypotheses_per_step"] / 64.0 *
                                     bench["config"]["n_corr"] / 2.0)),
        "sqc_dcache_hit_rate": (counters["SQC_DCACHE_HITS"] / counters["SQC_DCACHE_REQ"]
                                if counters.get("SQC_DCACHE_REQ") else None),
        "sqc_dcache_req_per_wave_point": (counters.get("SQC_DCACHE_REQ", 0.0) /
                                          (bench["config"]["hypotheses_per_step"] *
                                           bench["config"]["n_corr"] / 64.0)),
        "algorithmic_bytes_per_launch": bench["roofline"].get("algorithmic_bytes"),
        "pmc_run": "50 counted launches after 200 warm-up launches (clock ramped)",
        "source": f"rocprofv3 --pmc passes of bench.py (tools/gpu_round.sh), {src}",
    }
    with open(os.path.join(prof, f"{tag}_pmc_k_f8_count.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
