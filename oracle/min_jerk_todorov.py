"""Independent restatement of the Todorov & Jordan (1998) minimum-jerk solution that the
reference's src/min_jerk.py computes -- TEST INFRASTRUCTURE ONLY (imported
by tests/test_min_jerk_todorov.py, never by the product package).

The reference module cannot be imported (min_jerk.py:30-31: `.panda_utils` is missing from the
repository, `numexpr` is an undeclared third-party dependency; no pinned version exists), so no
golden vector of it can be made: parity UNPINNED.  Instead of restating its banded linear system
(min_jerk.py:150-215), this file derives the same optimum from first principles, so that the
package's restatement is checked against the mathematics rather than against itself:

  * a segment of duration T is the quintic with end positions, velocities and accelerations
    (x0, v0, a0) -> (x1, v1, a1); its jerk is 6 c3 + 24 c4 t + 60 c5 t^2 with (c3, c4, c5) linear
    in those six values (the coefficients min_jerk.py:135-139 evaluates);
  * its squared-jerk integral is then c^T Q(T) c with Q the exact integral of the monomials, and
    the path's cost a quadratic form in the interior (v_k, a_k), minimised by one linear solve
    of the assembled normal equations (numpy.linalg.solve, no explicit inverse);
  * samples are the segment polynomials in Horner form at the reference's sample times
    (uniform over [0, dur], the segment index advancing by at most one per sample,
    min_jerk.py:122-125).
"""
import numpy as np


def coeff_map(T):
    """3 x 6 matrix M with (c3, c4, c5) = M @ (x0, v0, a0, x1, v1, a1) for a segment of length T."""
    return np.array([
        [-10 / T ** 3, -6 / T ** 2, -1.5 / T, 10 / T ** 3, -4 / T ** 2, 0.5 / T],
        [15 / T ** 4, 8 / T ** 3, 1.5 / T ** 2, -15 / T ** 4, 7 / T ** 3, -1.0 / T ** 2],
        [-6 / T ** 5, -3 / T ** 4, -0.5 / T ** 3, 6 / T ** 5, -3 / T ** 4, 0.5 / T ** 3]])


def jerk_gram(T):
    """Q(T): integral over [0, T] of j(t) j(t)^T, j = (6, 24 t, 60 t^2)."""
    return np.array([[36 * T, 72 * T ** 2, 120 * T ** 3],
                     [72 * T ** 2, 192 * T ** 3, 360 * T ** 4],
                     [120 * T ** 3, 360 * T ** 4, 720 * T ** 5]])


def segment_hessian(T):
    """6 x 6 H with squared-jerk integral = z^T H z, z = (x0, v0, a0, x1, v1, a1)."""
    M = coeff_map(T)
    return M.T @ jerk_gram(T) @ M


def optimal_interior(x, times, v_end, a_end):
    """Interior velocities and accelerations minimising the total squared jerk of the path
    through the via points x (N x D) at knot times `times` (N), with the endpoint ones fixed.
    Returns (v, a), each (N-2) x D."""
    N, D = x.shape
    n = 2 * (N - 2)
    A = np.zeros((n, n))
    b = np.zeros((n, D))
    # unknown index of (velocity, acceleration) of point k (1..N-2): 2(k-1), 2(k-1)+1
    for s in range(N - 1):
        H = segment_hessian(times[s + 1] - times[s])
        # the six values of segment s: positions known; v / a unknown unless at the ends
        slots = []
        for k, base in ((s, 0), (s + 1, 3)):
            for j, kind in ((1, "v"), (2, "a")):
                if 1 <= k <= N - 2:
                    slots.append((base + j, 2 * (k - 1) + (0 if kind == "v" else 1), None))
                else:
                    e = 0 if k == 0 else 1
                    slots.append((base + j, None, (v_end if kind == "v" else a_end)[e]))
        known = np.zeros((6, D))
        known[0], known[3] = x[s], x[s + 1]
        for p, u, val in slots:
            if u is None:
                known[p] = val
        for p, u, _ in slots:
            if u is None:
                continue
            # d/dz_p of z^T H z = 2 (H z)_p: unknown-unknown terms into A, the rest into b
            for q, w, _ in slots:
                if w is not None:
                    A[u, w] += H[p, q]
            b[u] -= H[p] @ known
    sol = np.linalg.solve(A, b)
    return sol[0::2], sol[1::2]


def path_cost(x, times, v, a):
    """Total squared jerk of the piecewise quintic with all knot values given (N x D each)."""
    total = 0.0
    for s in range(len(x) - 1):
        H = segment_hessian(times[s + 1] - times[s])
        z = np.stack([x[s], v[s], a[s], x[s + 1], v[s + 1], a[s + 1]])
        total += float(np.einsum("pd,pq,qd->", z, H, z))
    return total


def sample(x, times, v, a, P):
    """P samples of the path at the reference's sample times (see the module docstring)."""
    N, D = x.shape
    out = np.zeros((int(P), D))
    k = 0
    for i in range(int(P)):
        t = i / (P - 1) * (times[-1] - times[0]) + times[0]
        if t > times[k + 1]:
            k += 1
        T = times[k + 1] - times[k]
        z = np.stack([x[k], v[k], a[k], x[k + 1], v[k + 1], a[k + 1]])
        c3, c4, c5 = coeff_map(T) @ z
        u = t - times[k]
        out[i] = x[k] + u * (v[k] + u * (0.5 * a[k] + u * (c3 + u * (c4 + u * c5))))
    return out
