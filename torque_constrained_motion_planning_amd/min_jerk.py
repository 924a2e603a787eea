"""Todorov & Jordan (1998) minimum-jerk trajectory through via points with optimised passage
times: the drop-in for the reference's src/min_jerk.py.

Upstream this module is dead code -- no caller imports it (panda_primitives.py:2 takes
min_jerk_v2) and it cannot be imported (min_jerk.py:30-31: `.panda_utils` is not in the
repository and `numexpr` is not a declared dependency) -- so parity against it is UNPINNED; the
restatement is checked against an independent derivation of the same optimum instead
(oracle/min_jerk_todorov.py: the segment quintics' jerk integrals as explicit quadratic forms,
minimised over the interior velocities and accelerations; tests/test_min_jerk_todorov.py).

Host-side numpy (the problems are a few dozen via points of 7 joints: one (2N-4)^2 solve per cost
evaluation, at most 750 evaluations in the passage-time search); the same names, argument
meaning, return shapes, printed output and failure modes as the reference:

  min_jerk(pos, dur, vel=None, acc=None, psg=None) -> (trj, psg, v, a)   (min_jerk.py:33-66)
  mjCOST(t, x, v0, a0, t0) -> summed squared-jerk integral                (min_jerk.py:72-98)
  mjTRJ(tx, x, v0, a0, t0, P) -> (X, v, a)                                (min_jerk.py:104-144)
  mjVelAcc(t, x, v0, a0, t0) -> (v, a) at the interior via points         (min_jerk.py:150-215)

Quirks kept: the initial passage times are the uniform ones halved (min_jerk.py:47-48);
mjCOST / mjVelAcc take N = max(x.shape) and D = min(x.shape) (fewer via points than joints
swaps them, as upstream); a two-point path has no passage times and fails in the final
np.append exactly as min_jerk.py:57 does; the segment index of mjTRJ advances by at most one per
sample (min_jerk.py:124-125).
"""
import numpy as np
import scipy.optimize


def min_jerk(pos=None, dur=None, vel=None, acc=None, psg=None):
    """Minimum-jerk trajectory of `dur` samples through the N x D via points `pos`
    (min_jerk.py:33-66).  vel / acc: 2 x D endpoint velocities / accelerations (zeros when None);
    psg: the N-2 passage times of the interior points, optimised by Nelder-Mead on mjCOST when
    None (scipy.optimize.fmin, maxfun=750, ftol=1e-2).  Returns (trj [dur x D], passage times as a
    list with 0 in front and the last repeated, velocities and accelerations at the via points as
    lists of rows with a zero row appended)."""
    print(pos)
    N, D = pos.shape[0], pos.shape[1]
    vel = np.zeros((2, D)) if vel is None else vel
    acc = np.zeros((2, D)) if acc is None else acc
    t0 = np.array([[0], [dur]])
    if psg is None:
        if N > 2:
            step = dur / (N - 1)
            x0 = 0.5 * np.arange(step, dur - step + 1, step).T
            psg = scipy.optimize.fmin(func=lambda p: mjCOST(p, pos, vel, acc, t0), x0=x0,
                                      maxfun=750, ftol=1e-2)
        else:
            psg = []
    print(psg)
    print(len(psg))
    trj, v, a = mjTRJ(psg, pos, vel, acc, t0, dur)
    zero = np.array([[0.0] * D])
    v = np.append(v, zero, axis=0)
    a = np.append(a, zero, axis=0)
    out = psg.tolist()
    out = [0.0] + out + [out[-1]]
    print("#" * 64)
    print(out)
    print("#" * 32)
    return trj, out, v.tolist(), a.tolist()


def _knots(t, t0):
    """[t0 start, passage times..., t0 end] (the reference's tt)."""
    return np.concatenate((t0[0], t, t0[1]), axis=0)


def _jerk_integrals(x0, x1, v0, v1, a0, a1, T):
    """Integral over [0, T] of the squared jerk of the quintic with these boundary values, for
    arrays of segments (the closed form min_jerk.py:89-94 evaluates with numexpr; here numpy,
    term for term)."""
    T2, T3, T4 = T ** 2, T ** 3, T ** 4
    s = (3 * a0 ** 2 * T4 - 2 * a0 * a1 * T4 + 3 * a1 ** 2 * T4 + 24 * a0 * T3 * v0
         - 16 * a1 * T3 * v0 + 64 * T2 * v0 ** 2 + 16 * a0 * T3 * v1
         - 24 * a1 * T3 * v1 + 112 * T2 * v0 * v1 + 64 * T2 * v1 ** 2
         + 40 * a0 * T2 * x0 - 40 * a1 * T2 * x0 + 240 * T * v0 * x0
         + 240 * T * v1 * x0 + 240 * x0 ** 2 - 40 * a0 * T2 * x1 + 40 * a1 * T2 * x1
         - 240 * T * v0 * x1 - 240 * T * v1 * x1 - 480 * x0 * x1 + 240 * x1 ** 2)
    return 3 * s / T ** 5


def mjCOST(t, x, v0, a0, t0):
    """Total squared jerk of the piecewise quintic through x with passage times t, the interior
    velocities / accelerations at their optimum (mjVelAcc) and the given endpoint ones
    (min_jerk.py:72-98)."""
    N, D = max(x.shape), min(x.shape)
    v, a = mjVelAcc(t, x, v0, a0, t0)
    aa = np.concatenate(([a0[0][:]], a, [a0[1][:]]), axis=0)
    vv = np.concatenate(([v0[0][:]], v, [v0[1][:]]), axis=0)
    T = np.diff(_knots(t, t0))[:, None] * np.ones((1, D))
    j = _jerk_integrals(x[:N - 1], x[1:N], vv[:N - 1], vv[1:N], aa[:N - 1], aa[1:N], T)
    return np.sum(np.abs(j))


def mjVelAcc(t, x, v0, a0, t0):
    """Velocities and accelerations at the N-2 interior via points that minimise the total
    squared jerk (min_jerk.py:150-215): the stationarity conditions form a banded (2N-4)^2 system
    over the unknowns (a_1, v_1, a_2, v_2, ...), solved as the reference does (explicit inverse,
    then a product).  Rows 2k / 2k+1 belong to interior point k+1 (durations T0 before, T1 after);
    their six band entries run from column 2k-2 / 2k-2, clipped at the matrix edges."""
    N, D = max(x.shape), min(x.shape)
    n = 2 * N - 4
    tt = _knots(t, t0)
    T0 = np.diff(tt)[:N - 2]          # segment before interior point k = 1..N-2
    T1 = np.diff(tt)[1:N - 1]         # segment after it
    band_a = np.stack([-6 / T0, -48 / T0 ** 2, 18 * (1 / T0 + 1 / T1),
                       72 * (1 / T1 ** 2 - 1 / T0 ** 2), -6 / T1, 48 / T1 ** 2], axis=1)
    band_v = np.stack([48 / T0 ** 2, 336 / T0 ** 3, 72 * (1 / T1 ** 2 - 1 / T0 ** 2),
                       384 * (1 / T1 ** 3 + 1 / T0 ** 3), -48 / T1 ** 2, 336 / T1 ** 3], axis=1)
    mat = np.zeros((n, n))
    for parity, band in ((0, band_a), (1, band_v)):
        rows = np.arange(parity, n, 2)              # row r = 2k + parity, interior point k + 1
        for m in range(6):
            cols = rows - 2 - parity + m
            ok = (cols >= 0) & (cols < n)
            mat[rows[ok], cols[ok]] = band[ok, m]
    xm, xk, xp = x[:N - 2], x[1:N - 1], x[2:N]
    vec = np.empty((n, D))
    vec[0::2] = 120 * (xm - xk) / T0[:, None] ** 3 + 120 * (xp - xk) / T1[:, None] ** 3
    vec[1::2] = 720 * (xk - xm) / T0[:, None] ** 4 + 720 * (xp - xk) / T1[:, None] ** 4
    # the endpoint velocities / accelerations move to the right-hand side
    Ts, Te = tt[1] - tt[0], tt[N - 1] - tt[N - 2]
    vec[0] = vec[0] + 6 / Ts * a0[0] + 48 / Ts ** 2 * v0[0]
    vec[1] = vec[1] - 48 / Ts ** 2 * a0[0] - 336 / Ts ** 3 * v0[0]
    vec[n - 2] = vec[n - 2] + 6 / Te * a0[1] - 48 / Te ** 2 * v0[1]
    vec[n - 1] = vec[n - 1] + 48 / Te ** 2 * a0[1] - 336 / Te ** 3 * v0[1]
    sol = np.linalg.inv(mat).dot(vec)
    return sol[1::2], sol[0::2]


def _segments(tt, P):
    """The segment each of the P samples falls in: the sample times span [tt[0], tt[-1]]
    uniformly, and the index advances by at most one per sample (min_jerk.py:122-125)."""
    span = tt[-1] - tt[0]
    ts = np.array([(i - 1) / (P - 1) for i in range(1, int(P) + 1)]) * span + tt[0]
    seg = np.empty(len(ts), dtype=np.int64)
    k = 0
    for i, ti in enumerate(ts.tolist()):
        if ti > tt[k + 1]:
            k += 1
        seg[i] = k
    return ts, seg


def mjTRJ(tx, x, v0, a0, t0, P):
    """P samples of the piecewise quintic through x (min_jerk.py:104-144): each segment's
    polynomial from its end positions, velocities and accelerations (the interior ones from
    mjVelAcc, or only the endpoint ones for a two-point path).  Returns (X [P x D], v, a)."""
    N, D = max(x.shape), min(x.shape)
    if len(tx) > 0:
        v, a = mjVelAcc(tx, x, v0, a0, t0)
        aa = np.concatenate(([a0[0][:]], a, [a0[1][:]]), axis=0)
        vv = np.concatenate(([v0[0][:]], v, [v0[1][:]]), axis=0)
        tt = _knots(tx, t0)
    else:
        v, a = np.array([]), np.array([])
        aa, vv, tt = a0, v0, t0
    tt = np.asarray(tt, dtype=np.float64).reshape(-1)
    ts, seg = _segments(tt, P)
    one = np.ones((1, D))
    T = (tt[seg + 1] - tt[seg])[:, None] * one
    t = (ts - tt[seg])[:, None] * one
    aa0, aa1, vv0, vv1 = aa[seg], aa[seg + 1], vv[seg], vv[seg + 1]
    xx0, xx1 = x[seg], x[seg + 1]
    c4 = (3 * aa0 * T ** 2 / 2 - aa1 * T ** 2 + 8 * T * vv0 + 7 * T * vv1 + 15 * xx0 - 15 * xx1)
    c5 = (-(aa0 * T ** 2) / 2 + aa1 * T ** 2 / 2 - 3 * T * vv0 - 3 * T * vv1 - 6 * xx0 + 6 * xx1)
    c3 = (-3 * aa0 * T ** 2 / 2 + aa1 * T ** 2 / 2 - 6 * T * vv0 - 4 * T * vv1 - 10 * xx0
          + 10 * xx1)
    X = (aa0 * t ** 2 / 2 + t * vv0 + xx0 + t ** 4 * c4 / T ** 4 + t ** 5 * c5 / T ** 5
         + t ** 3 * c3 / T ** 3)
    return X, v, a


def passage_search(pos, dur, vel=None, acc=None):
    """The passage-time search alone (min_jerk.py:45-53): the optimised interior passage times
    and the cost at the start and at the end of the search."""
    N, D = pos.shape
    vel = np.zeros((2, D)) if vel is None else vel
    acc = np.zeros((2, D)) if acc is None else acc
    t0 = np.array([[0], [dur]])
    step = dur / (N - 1)
    x0 = 0.5 * np.arange(step, dur - step + 1, step).T
    f = lambda p: mjCOST(p, pos, vel, acc, t0)  # noqa: E731
    best = scipy.optimize.fmin(func=f, x0=x0, maxfun=750, ftol=1e-2, disp=False)
    return best, f(x0), f(best)


__all__ = ["min_jerk", "mjCOST", "mjTRJ", "mjVelAcc", "passage_search"]
