"""Inscribed sphere sets of convex hulls: the "collision" certificate of the mesh exact tests.

A ball inside hull A and a ball inside hull B overlap by r_a + r_b - |c_a - c_b|; penetration
depth is monotone under inclusion, so depth(A, B) >= that overlap, and a sphere pair overlapping
by >= 0.04 (plus the kernels' fp32 guard) proves the pair collides at the reference's
-0.04 closest-points threshold (utils.py:2833) without running the hull-vs-hull test.

The set is chosen greedily for covered volume: interior grid points are the candidates, each
with the largest inscribed radius at it (min over the facet planes of d - n.x), and each pick is
the candidate whose ball covers the most still-uncovered interior grid points.
"""
import numpy as np

N_SPHERES = 16


def inscribed_spheres(verts, k=N_SPHERES, grid=24, n_cand=1200, seed=0):
    """-> [k, 4] float64 rows (cx, cy, cz, r): balls inside the convex hull of `verts`
    (same frame).  Fewer distinct balls than k are padded by repeating the first."""
    from .hull import hull_data
    v, pl, _ = hull_data(verts)
    n, d = pl[:, :3], pl[:, 3]
    lo, hi = v.min(0), v.max(0)
    ax = [np.linspace(lo[i], hi[i], grid + 2)[1:-1] for i in range(3)]
    X = np.stack(np.meshgrid(*ax, indexing="ij"), -1).reshape(-1, 3)
    r = (d[None, :] - X @ n.T).min(1)
    keep = r > 0
    X, r = X[keep], r[keep]
    if len(X) == 0:
        c = v.mean(0)
        return np.tile(np.concatenate([c, [0.0]]), (k, 1))
    rng = np.random.default_rng(seed)
    ci = np.arange(len(X)) if len(X) <= n_cand else rng.choice(len(X), n_cand, replace=False)
    C, rc = X[ci], r[ci]
    c32, x32 = C.astype(np.float32), X.astype(np.float32)
    d2 = (c32 * c32).sum(1)[:, None] + (x32 * x32).sum(1)[None, :] - 2.0 * (c32 @ x32.T)
    inside = d2 <= (rc * rc).astype(np.float32)[:, None]
    covered = np.zeros(len(X), bool)
    gain = inside.sum(1)
    out = []
    for _ in range(k):
        j = int(np.argmax(gain))
        if gain[j] == 0:
            break
        out.append(np.concatenate([C[j], [rc[j]]]))
        new = inside[j] & ~covered
        gain -= inside[:, new].sum(1)
        covered |= new
    while len(out) < k:
        out.append(out[0])
    s = np.array(out)
    # exact radius at the chosen centre (the grid value already is), shrunk by a relative 1e-9
    s[:, 3] = (d[None, :] - s[:, :3] @ n.T).min(1) * (1 - 1e-9)
    return s
