"""Sweep counts of k_e5_roots (diagnostic library, RSAMD_E5_STATS): per sample the sweeps its
row needed and the sweeps its wave ran; what grouping four samples of equal need would save."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
path = "/tmp/e5_stats.bin"
os.environ["RSAMD_E5_STATS"] = path
from tsbb15_amd import essential, synth  # noqa: E402

p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
essential.ransac_e(p1, p2, synth.K_SYNTH, samples=20000, seed=1)
raw = np.fromfile(path, dtype=np.int32).reshape(-1, 26)
np.save(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "e5_sweeps.npy"), raw)
s = raw[:, :4]
row, wave, deg, ok = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
print("samples", len(s), "ok", int(ok.sum()), "deg hist", np.bincount(deg, minlength=11).tolist())
print("row sweeps: mean %.2f p50 %d p90 %d p99 %d max %d" % (row.mean(), *np.percentile(row, [50, 90, 99]).astype(int), row.max()))
print("row hist", np.bincount(np.minimum(row, 40), minlength=41).tolist())
print("wave sweeps (per sample): mean %.2f" % wave.mean())
w4 = row[: len(row) // 4 * 4].reshape(-1, 4).max(axis=1)
print("sum of wave maxima (launch order) %d, sorted groups %d, sum of row sweeps / 4 %.0f" % (
    w4.sum(), np.sort(row)[: len(row) // 4 * 4].reshape(-1, 4).max(axis=1).sum(), row.sum() / 4))
