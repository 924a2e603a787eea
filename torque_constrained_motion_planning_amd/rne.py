"""rne.py drop-in: recursive Newton-Euler inverse dynamics of the Panda on the GPU.

Reference: src/rne.py.  The module keeps the reference's payload API (add_payload /
remove_payload / get_has_payload, rne.py:171-195) as module state, and rne(q, qd, qdd)
(rne.py:198) evaluates through libtcmp (tcmp_rne_batch).  rne_batch() evaluates many
samples in one launch.
"""
import numpy as np

from . import _lib

_payload_mass = 0.0
_has_payload = False


def get_has_payload():
    return _has_payload


def set_has_payload(val):
    global _has_payload
    _has_payload = bool(val)


def add_payload(r, m):
    """rne.py:181-188: `r` is ignored by the reference (COM fixed at the hand origin,
    inertia of a point mass 0.165 m along z)."""
    global _payload_mass
    remove_payload()
    if m > 0:
        set_has_payload(True)
        _payload_mass = float(m)


def remove_payload():
    global _payload_mass
    if get_has_payload():
        _payload_mass = 0.0
        set_has_payload(False)


def rne(q, qd, qdd):
    """tau = rne(q, qd, qdd) (rne.py:198-254): first len(q) joint torques, numpy array."""
    n = len(q)
    q7 = np.zeros(7); qd7 = np.zeros(7); qdd7 = np.zeros(7)
    q7[:n] = np.asarray(q, dtype=np.float64)[:7]
    qd7[:len(qd)] = np.asarray(qd, dtype=np.float64)[:7]
    qdd7[:len(qdd)] = np.asarray(qdd, dtype=np.float64)[:7]
    tau = _lib.engine().rne(q7, qd7, qdd7, _payload_mass if _has_payload else 0.0)[0]
    return tau[:n]


def rne_batch(q, qd, qdd, payload_mass=None):
    """Batched rne over rows of q/qd/qdd (n x 7).  payload_mass None = module state."""
    m = (_payload_mass if _has_payload else 0.0) if payload_mass is None else float(payload_mass)
    return _lib.engine().rne(q, qd, qdd, m)
