import numpy as np
raw = np.load("gpurun_out/e5_sweeps.npy")
sw = raw[:, 0].astype(float)
am = raw[:, 4:26].copy().view(np.float64)  # monic descending
N = len(sw)
def group_cost(order):
    x = sw[order][: N // 4 * 4].reshape(-1, 4).max(axis=1)
    return x.sum()
base = group_cost(np.arange(N)); best = group_cost(np.argsort(sw))
print("launch order", base, "perfect", best)
feats = {}
# numpy roots features
mind = np.zeros(N); nreal = np.zeros(N); spread = np.zeros(N); mrel = np.zeros(N)
for i in range(N):
    r = np.roots(am[i])
    nreal[i] = np.sum(np.abs(r.imag) <= 1e-6 * np.maximum(1, np.abs(r.real)))
    d = np.abs(r[:, None] - r[None, :]) + np.eye(len(r)) * 1e300
    sc = np.abs(r)[:, None] + np.abs(r)[None, :] + 1e-300
    mrel[i] = (d / sc).min()
    mind[i] = d.min()
    spread[i] = np.log(np.abs(r).max() / max(np.abs(r).min(), 1e-300))
feats["mrel"] = -mrel; feats["nreal"] = nreal; feats["spread"] = spread
# Newton polygon: number of edges, max edge multiplicity
lg = np.log(np.maximum(np.abs(am[:, ::-1]), 1e-300))  # ascending k? am descending: b_k = am[10-k]
ne = np.zeros(N); mm = np.zeros(N)
for i in range(N):
    l = np.log(np.maximum(np.abs(am[i][::-1]), 1e-300))  # l[k] = log|am[10-k]|
    hull = [0]
    for k in range(1, 11):
        while len(hull) >= 2:
            k1, k2 = hull[-2], hull[-1]
            if (l[k2] - l[k1]) * (k - k1) <= (l[k] - l[k1]) * (k2 - k1): hull.pop()
            else: break
        hull.append(k)
    ne[i] = len(hull) - 1; mm[i] = max(np.diff(hull))
feats["edges"] = -ne; feats["maxm"] = mm
from scipy.stats import spearmanr
for k, f in feats.items():
    print(k, "spearman %.3f" % spearmanr(f, sw).correlation, "sorted cost", group_cost(np.argsort(f, kind="stable")))
