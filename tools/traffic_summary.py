"""Calibrated HBM traffic from a tools/r06_traffic.sh output directory (one JSON on stdout).

MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE (KiB) count the L2's fabric-side requests;
gfx950's FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and other widths
are uncalibrated.  So:

  1. calibration -- tools/ubench/fetch_calib streams a known 1 GiB once per access shape
     (4 / 8 / 16 B per lane loads, 64-B scalar loads, 4 / 16 B per lane stores); factor =
     true bytes / counter bytes per shape;
  2. counting kernel (k_f8_count32q, C2 launches of bench.py) -- its reads mix three shapes
     (fp32 model rows 4 B/lane, the guard float4 16 B/lane, the points by scalar loads):
     the FETCH factor is the algorithmic-byte-weighted mix, fetch_corrected = raw x mix (this
     assumes the excess over the algorithmic bytes comes in the same mix);
  3. parse kernels (tools/probe_np_c2.py, C2 parity runs) -- every stream access is a 4 B/lane
     coalesced load or store: the 4 B/lane factors; bytes per C2 run = sum over a run's launches,
     with the kernel durations of the kernel trace beside them.

Usage: python tools/traffic_summary.py gpurun_out/<tag>
"""
import csv
import json
import os
import sys
from collections import defaultdict


def base(name):
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    for ns in ("rsd::", "(anonymous namespace)::"):
        n = n.replace(ns, "")
    return n.split("(")[0].strip()


def dispatch_values(path, counter):
    """{kernel: [per-dispatch value]} for one counter (rows summed per dispatch)."""
    per = defaultdict(float)
    kn = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[d] += float(r["Counter_Value"])
        kn[d] = base(r["Kernel_Name"])
    out = defaultdict(list)
    for d in sorted(per, key=lambda x: int(x)):
        out[kn[d]].append(per[d] * 1024.0)   # KiB -> bytes
    return out


def find_csv(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    return None


def match(vals, key):
    return [v for k, vs in vals.items() if k == key or k.startswith(key + "<") for v in vs]


def main():
    src = sys.argv[1]
    cal = json.load(open(os.path.join(src, "cal.json")))
    nbytes = cal["bytes_per_launch"]
    fetch = dispatch_values(find_csv(os.path.join(src, "cal_FETCH_SIZE")), "FETCH_SIZE")
    write = dispatch_values(find_csv(os.path.join(src, "cal_WRITE_SIZE")), "WRITE_SIZE")
    shapes = {}
    keymap = {"load 4 B/lane": "ld32", "load 8 B/lane": "ld64", "load 16 B/lane": "ld128",
              "scalar load 64 B/wave (s_load_dwordx16)": "lds", "store 4 B/lane": "st32",
              "store 16 B/lane": "st128"}
    for k in cal["kernels"]:
        name = k["kernel"]
        vals = fetch.get(name) if "load" in k["shape"] else write.get(name)
        if not vals:
            continue
        meas = sum(vals[1:]) / len(vals[1:]) if len(vals) > 1 else vals[0]
        shapes[keymap[k["shape"]]] = {"shape": k["shape"], "kernel": name, "true_bytes": nbytes,
                                      "counter_bytes": meas, "factor": nbytes / meas,
                                      "launches": len(vals)}
    f = {k: v["factor"] for k, v in shapes.items()}
    out = {"calibration": shapes,
           "calibration_note": "factor = true bytes / counter bytes (FETCH_SIZE for loads, "
                               "WRITE_SIZE for stores), one 1 GiB stream per launch, launches "
                               "after the first averaged (tools/ubench/fetch_calib.hip)"}
    # ---- counting kernel (C2) --------------------------------------------------------------
    cf = find_csv(os.path.join(src, "count_FETCH_SIZE"))
    cw = find_csv(os.path.join(src, "count_WRITE_SIZE"))
    if cf and cw and {"ld32", "ld128", "lds", "st32"} <= set(f):
        H, N = 100_000, 2000
        vf = match(dispatch_values(cf, "FETCH_SIZE"), "k_f8_count32q")
        vw = match(dispatch_values(cw, "WRITE_SIZE"), "k_f8_count32q")
        vf, vw = vf[200:] or vf, vw[200:] or vw        # the 50 launches after 200 warm-up ones
        raw_f, raw_w = sum(vf) / len(vf), sum(vw) / len(vw)
        alg = {"ld32": 36.0 * H, "ld128": 16.0 * H, "lds": 16.0 * N}
        mix = sum(alg.values()) / sum(a / f[s] for s, a in alg.items())
        fc, wc = raw_f * mix, raw_w * f["st32"]
        algb = 56.0 * H + 16.0 * N
        out["count"] = {"kernel": "k_f8_count32q", "n_corr": N, "hypotheses": H,
                        "fetch_raw": raw_f, "write_raw": raw_w, "fetch_factor_mix": mix,
                        "fetch_corrected": fc, "write_corrected": wc,
                        "hbm_bytes_corrected": fc + wc, "algorithmic_bytes": algb,
                        "corrected_over_algorithmic": (fc + wc) / algb,
                        "factors": {"ld32": f["ld32"], "ld128": f["ld128"], "lds": f["lds"],
                                    "st32": f["st32"]},
                        "method": "FETCH x the algorithmic-byte-weighted mix of the calibrated "
                                  "factors (fp32 model rows 36 B/hyp at 4 B/lane, guard float4 "
                                  "16 B/hyp at 16 B/lane, points 16 B each by scalar loads); "
                                  "WRITE x the 4 B/lane store factor"}
    # ---- parse kernels (C2 parity runs) ------------------------------------------------------
    pf = find_csv(os.path.join(src, "parse_FETCH_SIZE"))
    pw = find_csv(os.path.join(src, "parse_WRITE_SIZE"))
    if pf and pw:
        runs = 4
        vf, vw = dispatch_values(pf, "FETCH_SIZE"), dispatch_values(pw, "WRITE_SIZE")
        dur = defaultdict(list)
        tr = None
        for root, _, files in os.walk(os.path.join(src, "parse_trace")):
            for fn in files:
                if fn.endswith("kernel_trace.csv"):
                    tr = os.path.join(root, fn)
        if tr:
            for r in csv.DictReader(open(tr)):
                dur[base(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        kern = {}
        for k in sorted(set(vf) | set(vw)):
            if not (k.startswith("k_np") or k.startswith("k_mt")):
                continue
            rf = sum(vf.get(k, [])) / runs
            rw = sum(vw.get(k, [])) / runs
            ms = sum(dur.get(k, [])) / (runs + 1) / 1e6 if dur.get(k) else None
            cb = rf * f["ld32"] + rw * f["st32"]
            kern[k] = {"launches_per_run": len(vf.get(k, [])) / runs, "fetch_raw": rf,
                       "write_raw": rw, "bytes_corrected": cb, "ms_per_run": ms,
                       "gbs": cb / (ms * 1e-3) / 1e9 if ms else None,
                       "frac_of_8tbs": cb / (ms * 1e-3) / 8e12 if ms else None}
        tot = sum(v["bytes_corrected"] for v in kern.values())
        tms = sum(v["ms_per_run"] or 0.0 for v in kern.values())
        out["parse"] = {"kernels": kern, "bytes_corrected_per_run": tot,
                        "kernel_ms_per_run": tms,
                        "gbs_over_kernel_time": tot / (tms * 1e-3) / 1e9 if tms else None,
                        "runs_counted": runs,
                        "method": "FETCH x the 4 B/lane load factor + WRITE x the 4 B/lane store "
                                  "factor per kernel, summed over one C2 run's launches "
                                  "(tools/probe_np_c2.py, 4 runs per pass); kernel times from "
                                  "the kernel trace of the same probe (5 runs, one with step "
                                  "events)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
