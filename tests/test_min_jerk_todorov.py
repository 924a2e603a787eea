"""src/min_jerk.py (Todorov & Jordan 1998 minimum jerk with optimised passage times; SURVEY 8a
row a16) -- the package's restatement (torque_constrained_motion_planning_amd.min_jerk) against
an independent derivation of the same optimum (oracle/min_jerk_todorov.py).

Parity against the reference itself is UNPINNED: the upstream module cannot be imported
(min_jerk.py:30-31 -- `.panda_utils` is missing and `numexpr` undeclared) and no caller in the
reference uses it, so no golden vector exists.  What is pinned instead:
  * mjCOST's closed form (min_jerk.py:89-94) is the exact squared-jerk integral of each segment
    quintic (against the Gram-matrix form and against quadrature);
  * mjVelAcc's banded system (min_jerk.py:150-215) yields exactly the interior velocities and
    accelerations that minimise that cost (against the assembled normal equations);
  * mjTRJ's samples (min_jerk.py:104-144) are those quintics at the reference's sample times, with
    the reference's segment bookkeeping (the index advances at most one per sample);
  * min_jerk's passage-time search and outputs: shapes, the list conventions of its return
    values, the printed output, and the two-point failure (min_jerk.py:33-66).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import min_jerk_todorov as R  # noqa: E402  (test infrastructure)

from torque_constrained_motion_planning_amd import min_jerk as M  # noqa: E402


def _path(rng, N, D=7):
    x = np.cumsum(rng.normal(scale=0.4, size=(N, D)), axis=0)
    return x


def _knots(psg, dur):
    return np.concatenate(([0.0], np.asarray(psg, dtype=float), [float(dur)]))


# (the reference takes N = max(x.shape), D = min(x.shape): paths of fewer points than
# dimensions are not paths to it -- test_fewer_points_than_dimensions below)
@pytest.mark.parametrize("N,D", [(3, 2), (4, 3), (7, 7), (12, 7), (30, 7)])
def test_velacc_is_the_min_jerk_optimum(N, D):
    rng = np.random.default_rng(N)
    x = _path(rng, N, D)
    dur = 1000
    psg = np.sort(rng.uniform(50, 950, N - 2))
    v0 = rng.normal(size=(2, D)) * 0.1
    a0 = rng.normal(size=(2, D)) * 0.01
    t0 = np.array([[0], [dur]])
    v, a = M.mjVelAcc(psg, x, v0, a0, t0)
    rv, ra = R.optimal_interior(x, _knots(psg, dur), v0, a0)
    assert v.shape == (N - 2, D) and a.shape == (N - 2, D)
    scale_v, scale_a = np.abs(rv).max() + 1e-12, np.abs(ra).max() + 1e-12
    assert np.abs(v - rv).max() <= 1e-8 * scale_v
    assert np.abs(a - ra).max() <= 1e-8 * scale_a


@pytest.mark.parametrize("N", [7, 9, 16])
def test_cost_is_the_squared_jerk_integral(N):
    rng = np.random.default_rng(10 + N)
    x = _path(rng, N)
    dur = 500
    psg = np.sort(rng.uniform(40, 460, N - 2))
    v0, a0 = np.zeros((2, 7)), np.zeros((2, 7))
    t0 = np.array([[0], [dur]])
    J = M.mjCOST(psg, x, v0, a0, t0)
    tt = _knots(psg, dur)
    v, a = M.mjVelAcc(psg, x, v0, a0, t0)
    vv = np.concatenate([v0[:1], v, v0[1:]])
    aa = np.concatenate([a0[:1], a, a0[1:]])
    # (both forms cancel: the positions are ~1e4 times the jerk scale, so each is ~1e-8 from
    # the exact rational value of the same inputs -- checked once with fractions.Fraction)
    assert J == pytest.approx(R.path_cost(x, tt, vv, aa), rel=1e-7)
    # and against quadrature of the jerk of the sampled polynomials (Gauss-Legendre, exact for
    # the degree-4 integrand)
    g, w = np.polynomial.legendre.leggauss(5)
    q = 0.0
    for s in range(N - 1):
        T = tt[s + 1] - tt[s]
        z = np.stack([x[s], vv[s], aa[s], x[s + 1], vv[s + 1], aa[s + 1]])
        c3, c4, c5 = R.coeff_map(T) @ z
        u = 0.5 * T * (g + 1)
        jerk = 6 * c3[None] + 24 * c4[None] * u[:, None] + 60 * c5[None] * u[:, None] ** 2
        q += 0.5 * T * float((w[:, None] * jerk ** 2).sum())
    assert J == pytest.approx(q, rel=1e-7)
    # moving an interior velocity off the optimum can only raise the cost
    for k in range(N - 2):
        vb = vv.copy()
        vb[k + 1, 3] += 1e-3
        assert R.path_cost(x, tt, vb, aa) > R.path_cost(x, tt, vv, aa)


@pytest.mark.parametrize("N,dur", [(7, 200), (9, 999), (14, 2500)])
def test_trajectory_samples(N, dur):
    rng = np.random.default_rng(20 + N)
    x = _path(rng, N)
    psg = np.sort(rng.uniform(0.05 * dur, 0.95 * dur, N - 2))
    v0, a0 = np.zeros((2, 7)), np.zeros((2, 7))
    t0 = np.array([[0], [dur]])
    X, v, a = M.mjTRJ(psg, x, v0, a0, t0, dur)
    assert X.shape == (dur, 7)
    tt = _knots(psg, dur)
    vv = np.concatenate([v0[:1], v, v0[1:]])
    aa = np.concatenate([a0[:1], a, a0[1:]])
    ref = R.sample(x, tt, vv, aa, dur)
    assert np.abs(X - ref).max() <= 1e-9 * (1 + np.abs(x).max())
    assert np.allclose(X[0], x[0], atol=1e-12) and np.allclose(X[-1], x[-1], atol=1e-9)


def test_segment_index_lags_short_segments():
    """Two knots closer than one sample apart: the reference's index advances once per sample
    (min_jerk.py:124-125), so the sample after the short segment is still evaluated on it --
    reproduced, not 'fixed'."""
    x = _path(np.random.default_rng(3), 4, 3)
    dur = 11  # samples at 0, 1.1, 2.2, ... (times (i-1)/(P-1) * dur)
    psg = np.array([3.3, 3.5])
    t0 = np.array([[0], [dur]])
    z = np.zeros((2, 3))
    X, v, a = M.mjTRJ(psg, x, z, z, t0, dur)
    tt = _knots(psg, dur)
    vv = np.concatenate([z[:1], v, z[1:]])
    aa = np.concatenate([z[:1], a, z[1:]])
    assert np.abs(X - R.sample(x, tt, vv, aa, dur)).max() < 1e-9


def test_min_jerk_end_to_end(capsys):
    rng = np.random.default_rng(5)
    N, dur = 8, 400
    pos = _path(rng, N)
    trj, psg, v, a = M.min_jerk(pos, dur)
    out = capsys.readouterr().out
    assert "#" * 64 in out
    assert "Optimization terminated" in out or "Maximum number" in out  # scipy fmin's report
    assert trj.shape == (dur, 7)
    assert isinstance(psg, list) and len(psg) == N and psg[0] == 0.0 and psg[-1] == psg[-2]
    assert len(v) == N - 1 and len(a) == N - 1 and v[-1] == [0.0] * 7 and a[-1] == [0.0] * 7
    # the search lowered the cost from the reference's starting point (uniform times halved)
    best, c_start, c_end = M.passage_search(pos, dur)
    assert np.allclose(best, psg[1:-1])
    assert c_end <= c_start
    x0 = 0.5 * np.arange(dur / (N - 1), dur - dur / (N - 1) + 1, dur / (N - 1))
    assert c_start == M.mjCOST(x0, pos, np.zeros((2, 7)), np.zeros((2, 7)), np.array([[0], [dur]]))
    # given passage times: no search, the trajectory through them
    trj2, psg2, _, _ = M.min_jerk(pos, dur, psg=np.array(psg[1:-1]))
    assert np.array_equal(trj2, trj)


def test_min_jerk_two_points_fails_as_upstream():
    """N = 2: no passage times, and min_jerk.py:57 appends a 2-D row to the empty 1-D velocity
    array -- a ValueError upstream, and here."""
    pos = np.zeros((2, 7))
    pos[1] = 0.3
    with pytest.raises(ValueError):
        M.min_jerk(pos, 100)


def test_fewer_points_than_dimensions():
    """N = max(x.shape), D = min(x.shape) (min_jerk.py:74-75, 106-107, 152-153): three 7-D via
    points are read as seven 3-D ones and the right-hand side cannot be filled -- a ValueError
    upstream (min_jerk.py:178 broadcasting a 7-vector into a 3-row) and here."""
    x = _path(np.random.default_rng(1), 3)
    with pytest.raises(ValueError):
        M.mjVelAcc(np.array([500.0]), x, np.zeros((2, 7)), np.zeros((2, 7)),
                   np.array([[0], [1000]]))
