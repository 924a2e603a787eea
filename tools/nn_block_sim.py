#!/usr/bin/env python3
"""CPU simulation behind DESIGN.md section 10 (candidate groups sharing one node stream): for a
uniform tree of T nodes in the joint box, the engine's Morton cells (<= 64 nodes, 36-bit keys)
and 262,144 Morton-sorted candidates, the nodes each candidate's exact nearest search must
evaluate, against the union over BLK consecutive candidates.

    python tools/nn_block_sim.py [T=690000] [BLK=64]
"""
import numpy as np, sys
from scipy.spatial import cKDTree
LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
rng = np.random.default_rng(0)
T = int(sys.argv[1]) if len(sys.argv) > 1 else 690000
B = 262144
BLK = int(sys.argv[2]) if len(sys.argv) > 2 else 64
def morton(q):
    g = np.clip(((q - LO) / (HI - LO) * 512).astype(np.int64), 0, 511)
    k = np.zeros(len(q), dtype=np.uint64)
    for b in range(8, -1, -1):
        for j in range(7):
            k = (k << np.uint64(1)) | ((g[:, j] >> b) & 1).astype(np.uint64)
    return k >> np.uint64(63 - 36)
nodes = LO + (HI - LO) * rng.random((T, 7))
nk = morton(nodes); o = np.argsort(nk, kind='stable'); nodes = nodes[o]; nk = nk[o]
# cells: maximal prefix subtrees with <= 64 nodes
cells = []
stack = [(0, T, 0)]
while stack:
    a, b, p = stack.pop()
    if b - a <= 64 or p >= 36:
        cells.append((a, b)); continue
    bit = np.uint64(1) << np.uint64(35 - p)
    m = a + np.searchsorted((nk[a:b] & bit) != 0, True)
    if m > a: stack.append((a, m, p + 1))
    if b > m: stack.append((m, b, p + 1))
cells.sort()
lo = np.array([nodes[a:b].min(0) for a, b in cells]); hi = np.array([nodes[a:b].max(0) for a, b in cells])
cnt = np.array([b - a for a, b in cells])
print("T", T, "cells", len(cells), "avg nodes/cell", cnt.mean())
cand = LO + (HI - LO) * rng.random((B, 7))
ck = morton(cand); cand = cand[np.argsort(ck, kind='stable')]
d, _ = cKDTree(nodes).query(cand)
d2 = d * d
nb = B // BLK
sel = rng.choice(nb, 40, replace=False)
per_cand, union = [], []
for s in sel:
    c = cand[s * BLK:(s + 1) * BLK]; r2 = d2[s * BLK:(s + 1) * BLK]
    gap = np.maximum(np.maximum(lo[None] - c[:, None], c[:, None] - hi[None]), 0)  # (64, C, 7)
    lb = (gap * gap).sum(-1)
    need = lb <= r2[:, None]
    per_cand.append(cnt[None].repeat(BLK, 0)[need].sum() / BLK)
    u = need.any(0)
    union.append((u.sum(), cnt[u].sum()))
union = np.array(union)
print("per-candidate needed nodes %.0f; block union: %.1f cells, %.0f nodes -> %.0f pair evals per candidate (x%.1f)"
      % (np.mean(per_cand), union[:, 0].mean(), union[:, 1].mean(), union[:, 1].mean(), union[:, 1].mean() / np.mean(per_cand)))
