"""min_jerk_v2.py drop-in (Hoff-Arbib min-jerk through waypoints, unit segment durations).

Reference: src/min_jerk_v2.py.  minjerk_coefficients / _minjerk_trajectory_point /
minjerk_point keep the reference's numpy API (they are per-call utilities).  The planner's
hot use -- sampling a whole path (panda_primitives.py:299-316) -- goes through
minjerk_waypoints(), which evaluates every sample on the GPU (tcmp_minjerk).
"""
import numpy as np

from . import _lib


def minjerk_coefficients(points_array, duration_array=None):
    """min_jerk_v2.py:80-142.  Returns (k, N, 7): a0..a5, duration."""
    (rows, k) = np.shape(points_array)
    N = rows - 1
    m_coeffs = np.zeros(shape=(k, N, 7))
    x = points_array[0]
    v = np.zeros(k)
    a = np.zeros(k)
    if duration_array is None:
        duration_array = np.array([1.0] * N)
    assert len(duration_array) == N, \
        "Invalid number of intervals chosen (must be equal to N+1={})".format(N)
    for i in range(0, N):
        gx = points_array[i + 1]
        t = duration_array[i]
        if i == N - 1:
            gv = np.zeros(k)
        else:
            t0 = t
            t1 = duration_array[i + 1]
            d0 = points_array[i + 1] - points_array[i]
            d1 = points_array[i + 2] - points_array[i + 1]
            v0 = d0 / t0
            v1 = d1 / t1
            gv = np.where(np.multiply(v0, v1) >= 1e-10, 0.5 * (v0 + v1), np.zeros(k))
        ga = np.zeros(k)
        A = (gx - (x + v * t + (a / 2.0) * t * t)) / (t * t * t)
        B = (gv - (v + a * t)) / (t * t)
        C = (ga - a) / t
        m_coeffs[:, i, 0] = x
        m_coeffs[:, i, 1] = v
        m_coeffs[:, i, 2] = a / 2.0
        m_coeffs[:, i, 3] = 10 * A - 4 * B + 0.5 * C
        m_coeffs[:, i, 4] = (-15 * A + 7 * B - C) / t
        m_coeffs[:, i, 5] = (6 * A - 3 * B + 0.5 * C) / (t * t)
        m_coeffs[:, i, 6] = t
        x = gx
        v = gv
    return m_coeffs


def _minjerk_trajectory_point(m_coeff, t):
    """min_jerk_v2.py:184-222."""
    a0, a1, a2, a3, a4, a5, tm = (m_coeff[:, i] for i in range(7))
    t = t * tm
    x = a0 + a1 * t + a2 * np.power(t, 2) + a3 * np.power(t, 3) + a4 * np.power(t, 4) + a5 * np.power(t, 5)
    v = a1 + 2 * a2 * t + 3 * a3 * np.power(t, 2) + 4 * a4 * np.power(t, 3) + 5 * a5 * np.power(t, 4)
    a = 2 * a2 + 6 * a3 * t + 12 * a4 * np.power(t, 2) + 20 * a5 * np.power(t, 3)
    return x, v, a


def minjerk_trajectory(m_coeffs, num_intervals, duration_array=None):
    """min_jerk_v2.py:144-182: list of [x, v, a] per sample (segment start excluded)."""
    assert num_intervals > 0, "Invalid number of intervals chosen (must be greater than 0)"
    interval = 1.0 / num_intervals
    (_, num_mpts, _) = np.shape(m_coeffs)
    if duration_array is None:
        duration_array = np.array([1.0] * num_mpts)
    m_curve = []
    for current_mpt in range(num_mpts):
        m_coeff_set = m_coeffs[:, current_mpt, range(7)]
        for t in np.linspace(interval, 1, num_intervals):
            x, v, a = _minjerk_trajectory_point(m_coeff_set, t * duration_array[current_mpt])
            m_curve.append([x, v, a])
    return m_curve


def minjerk_point(m_coeffs, m_index, t):
    """min_jerk_v2.py:224-255."""
    if m_index <= 0:
        return m_coeffs[:, 0, 0]
    elif m_index > m_coeffs.shape[1]:
        return _minjerk_trajectory_point(m_coeffs[:, m_coeffs.shape[1] - 1, range(7)], 1)
    t = min(max(t, 0.0), 1.0)
    return _minjerk_trajectory_point(m_coeffs[:, m_index - 1, range(7)], t)


def minjerk_waypoints(points, num_intervals):
    """GPU min-jerk sampling of a waypoint path: ((N-1)*ni x 7) q, qd, qdd -- the same
    samples as minjerk_trajectory(minjerk_coefficients(points), ni)."""
    return _lib.engine().minjerk(np.asarray(points, dtype=np.float64), int(num_intervals))
