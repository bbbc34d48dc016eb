"""Chunk timeline of the numpy-exact parse (RSAMD_NP_TSTAMP, the product kernels' stamps):
where k_np_entry / k_np_track spend a C2 parse, chunk by chunk.

Per chunk the kernels stamp the 100 MHz real-time counter and shader-clock cycles at the
entry kernel's start / end, the tracking kernel's start / end and the checkpoint at which the
chunk's trajectories are down to one per wave, with the draw positions and hardware ids.

  python tools/np_timeline.py [n] [hyps] [runs] > summary.json
"""
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))

TS = 16
(E_R0, E_C0, E_R1, E_C1, E_T, E_M, E_HW, _7, T_R0, T_C0, S_R, S_T, T_R1, T_C1, T_HW, S_C) = range(16)


def records(path):
    raw = np.fromfile(path, dtype=np.uint64)
    out, o = [], 0
    while o + 8 <= len(raw):
        h = raw[o:o + 8].astype(np.int64)
        cr = int(h[1])
        out.append((h, raw[o + 8:o + 8 + cr * TS].reshape(cr, TS).astype(np.int64)))
        o += 8 + cr * TS
    return out


def pct(a, ps=(0, 10, 50, 90, 100)):
    a = np.asarray(a, dtype=np.float64)
    a = a[~np.isnan(a)]
    return [round(float(np.percentile(a, p)), 3) for p in ps] if a.size else None


def analyse(h, r):
    n1, C, W = int(h[0]), int(h[1]), int(h[2])
    us = lambda x: x * 0.01  # 100 MHz ticks -> us
    t0 = r[:, E_R0].min()
    e0, e1 = us(r[:, E_R0] - t0), us(r[:, E_R1] - t0)
    tracked = r[:, T_R0] > 0
    tr0, tr1 = us(r[:, T_R0] - t0), us(r[:, T_R1] - t0)
    sr = np.where(r[:, S_R] > 0, us(r[:, S_R] - t0), np.nan)
    clk_e = (r[:, E_C1] - r[:, E_C0]) / np.maximum(1, r[:, E_R1] - r[:, E_R0]) * 0.1  # GHz
    clk_t = (r[:, T_C1] - r[:, T_C0]) / np.maximum(1, r[:, T_R1] - r[:, T_R0]) * 0.1
    single_draws = W - r[:, S_T]
    single_cyc = r[:, T_C1] - r[:, S_C]
    cpd = np.where((r[:, S_R] > 0) & (single_draws > 0), single_cyc / np.maximum(1, single_draws), np.nan)
    multi_us = sr - tr0
    single_us = tr1 - sr
    last = int(np.argmax(np.where(tracked, tr1, e1)))
    hw = r[:, T_HW]
    hwid = hw >> 8   # HW_ID: cu [11:8], sh [12], se [15:13]; XCC_ID in the low byte of hw
    cu_key = (hw & 7) * 4096 + ((hwid >> 13) & 7) * 512 + ((hwid >> 12) & 1) * 256 + ((hwid >> 8) & 15)
    per_cu = {}
    for k, c in zip(cu_key, range(C)):
        per_cu.setdefault(int(k), []).append(c)
    sharing = [len(v) for v in per_cu.values()]
    out = {
        "n1": n1, "chunks": C, "chunk_draws": W,
        "entry_kernel_us": round(float(e1.max() - e0.min()), 1),
        "entry_start_skew_us": pct(e0),
        "entry_dur_us": pct(e1 - e0),
        "entry_hand_draws": pct(r[:, E_T]),
        "entry_hand_m": pct(r[:, E_M]),
        "entry_clock_ghz": pct(clk_e),
        "entry_cycles_per_draw": pct((r[:, E_C1] - r[:, E_C0]) / np.maximum(1, r[:, E_T])),
        "gap_entry_end_to_track_start_us": round(float(tr0[tracked].min() - e1.max()), 2) if tracked.any() else None,
        "track_start_skew_us": pct(tr0[tracked] - tr0[tracked].min()) if tracked.any() else None,
        "track_kernel_us": round(float(tr1[tracked].max() - tr0[tracked].min()), 1) if tracked.any() else 0.0,
        "chunks_tracked": int(tracked.sum()),
        "track_dur_us": pct((tr1 - tr0)[tracked]),
        "track_clock_ghz": pct(clk_t[tracked]),
        "multi_phase_us": pct(multi_us[tracked & ~np.isnan(sr)]),
        "multi_phase_draws": pct((r[:, S_T] - r[:, E_T])[tracked & (r[:, S_R] > 0)]),
        "single_phase_us": pct(single_us[tracked & ~np.isnan(sr)]),
        "single_phase_draws": pct(single_draws[tracked & (r[:, S_R] > 0)]),
        "single_cycles_per_draw": pct(cpd[~np.isnan(cpd)]),
        "chunks_per_cu": {str(k): sharing.count(k) for k in sorted(set(sharing))},
        "last_chunk": {"chunk": last, "entry_us": round(float(e1[last] - e0[last]), 1),
                       "hand_draws": int(r[last, E_T]), "hand_m": int(r[last, E_M]),
                       "track_start_us": round(float(tr0[last]), 1),
                       "multi_us": round(float(multi_us[last]), 1) if not np.isnan(multi_us[last]) else None,
                       "single_from_draw": int(r[last, S_T]),
                       "single_us": round(float(single_us[last]), 1) if not np.isnan(single_us[last]) else None,
                       "end_us": round(float(tr1[last]), 1),
                       "track_clock_ghz": round(float(clk_t[last]), 3),
                       "shares_cu_with": [c for c in per_cu[int(cu_key[last])] if c != last]},
    }
    # what the critical path would be at the measured per-phase rates with no skew:
    # entry max + track max, against the sum of per-chunk means
    out["sum_of_maxima_us"] = round(float((e1 - e0).max() + ((tr1 - tr0)[tracked].max() if tracked.any() else 0)), 1)
    out["max_of_sums_us"] = round(float(((e1 - e0) + np.where(tracked, tr1 - tr0, 0)).max()), 1)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    path = os.path.join(tempfile.mkdtemp(), "np_ts.bin")
    os.environ["RSAMD_NP_TSTAMP"] = path
    from tsbb15_amd import _ffi, synth
    p1, p2, _ = synth.two_view(n, 0.3, seed=1)
    ctx = _ffi.Context(0)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    key, pos = _ffi.np_seed(0)
    for _ in range(runs):
        plan.run_np(H, key, pos)
        plan.result()
    recs = records(path)
    res = {"n": n, "hypotheses": H, "runs": len(recs), "last_run": analyse(*recs[-1]),
           "first_run_track_kernel_us": analyse(*recs[0])["track_kernel_us"]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
