"""min_jerk_v2.py drop-in: minimum-jerk (quintic) segments through waypoints.

Reference: src/min_jerk_v2.py.  The planner's hot use -- sampling a whole RRT path
(dynam_fn, panda_primitives.py:299-316) -- is minjerk_waypoints(), which evaluates every
sample on the GPU (tcmp_minjerk).  The per-call utilities keep the reference's API and
output layout, vectorised over segments and samples:

Segment i runs from waypoint x_i to x_{i+1} over duration T_i with boundary velocity v_i at
both ends and zero boundary acceleration (the reference never updates its running
acceleration, min_jerk_v2.py:132-133).  The waypoint velocity is the mean of the adjacent
segment slopes when they agree in sign (product >= 1e-10), else 0, and 0 at both ends
(min_jerk_v2.py:109-118).  With A = (x_{i+1} - (x_i + v_i T)) / T^3 and
B = (v_{i+1} - v_i) / T^2 the quintic x(t) = x_i + v_i t + c3 t^3 + c4 t^4 + c5 t^5 has
c3 = 10A - 4B, c4 = (7B - 15A) / T, c5 = (6A - 3B) / T^2 (the boundary conditions
x(T) = x_{i+1}, x'(T) = v_{i+1}, x''(0) = x''(T) = 0 solved for c3..c5).
"""
import numpy as np

from . import _lib


def _durations(n_seg, duration_array):
    if duration_array is None:
        return np.ones(n_seg)
    T = np.asarray(duration_array, dtype=np.float64).reshape(-1)
    assert len(T) == n_seg, \
        "Invalid number of intervals chosen (must be equal to N+1={})".format(n_seg)
    return T


def minjerk_coefficients(points_array, duration_array=None):
    """min_jerk_v2.py:80-142 -> (k, N, 7) per joint and segment: a0..a5, duration."""
    P = np.asarray(points_array, dtype=np.float64)
    n_seg, k = P.shape[0] - 1, P.shape[1]
    T = _durations(n_seg, duration_array)
    slope = (P[1:] - P[:-1]) / T[:, None]                      # (N, k)
    vel = np.zeros_like(P)                                     # waypoint velocities
    agree = slope[:-1] * slope[1:] >= 1e-10
    vel[1:-1] = np.where(agree, 0.5 * (slope[:-1] + slope[1:]), 0.0)
    t = T[:, None]
    A = (P[1:] - (P[:-1] + vel[:-1] * t)) / (t * t * t)
    B = (vel[1:] - vel[:-1]) / (t * t)
    out = np.zeros((k, n_seg, 7))
    out[:, :, 0] = P[:-1].T
    out[:, :, 1] = vel[:-1].T
    out[:, :, 3] = (10 * A - 4 * B).T
    out[:, :, 4] = ((-15 * A + 7 * B) / t).T
    out[:, :, 5] = ((6 * A - 3 * B) / (t * t)).T
    out[:, :, 6] = T[None, :]
    return out


def _eval(c, t):
    """Position, velocity, acceleration of coefficient rows c (..., 7) at local time
    t * duration (Horner form)."""
    a0, a1, a2, a3, a4, a5, tm = np.moveaxis(c, -1, 0)
    t = t * tm
    x = a0 + t * (a1 + t * (a2 + t * (a3 + t * (a4 + t * a5))))
    v = a1 + t * (2 * a2 + t * (3 * a3 + t * (4 * a4 + t * 5 * a5)))
    a = 2 * a2 + t * (6 * a3 + t * (12 * a4 + t * 20 * a5))
    return x, v, a


def _minjerk_trajectory_point(m_coeff, t):
    """min_jerk_v2.py:184-222: one segment's coefficients (k, 7) at normalised time t."""
    return _eval(np.asarray(m_coeff), t)


def minjerk_trajectory(m_coeffs, num_intervals, duration_array=None):
    """min_jerk_v2.py:144-182: [x, v, a] per sample, num_intervals samples per segment at
    t = 1/n, ..., 1 (segment start excluded), segments in order."""
    assert num_intervals > 0, "Invalid number of intervals chosen (must be greater than 0)"
    C = np.asarray(m_coeffs)
    n_seg = C.shape[1]
    T = _durations(n_seg, duration_array)
    ts = np.linspace(1.0 / num_intervals, 1, num_intervals)
    # (segments, samples, joints): coefficient rows broadcast over the sample axis
    tt = (ts[None, :] * T[:, None])[:, :, None]
    x, v, a = _eval(np.transpose(C, (1, 0, 2))[:, None, :, :], tt)
    return [[x[i, j], v[i, j], a[i, j]] for i in range(n_seg) for j in range(num_intervals)]


def minjerk_point(m_coeffs, m_index, t):
    """min_jerk_v2.py:224-255: the start point for m_index <= 0, the end of the last segment
    past the end, else segment m_index - 1 at t clamped to [0, 1]."""
    C = np.asarray(m_coeffs)
    if m_index <= 0:
        return C[:, 0, 0]
    if m_index > C.shape[1]:
        return _eval(C[:, -1, :], 1)
    return _eval(C[:, m_index - 1, :], min(max(t, 0.0), 1.0))


def minjerk_waypoints(points, num_intervals):
    """GPU min-jerk sampling of a waypoint path: ((N-1)*ni x 7) q, qd, qdd -- the samples of
    minjerk_trajectory(minjerk_coefficients(points), ni)."""
    return _lib.engine().minjerk(np.asarray(points, dtype=np.float64), int(num_intervals))
