"""Trajectory output in the reference's data-collection format.

collect_data.py:108-131 (`save_traj_data`) writes one npz per planned trajectory with the
per-Conf arrays q, qd, qdd, torques, ts; collect_data.py:146-159 keeps a meta CSV with one row
per (method, set): planning_time, mass, distance, success, filename.  Same keys, same shapes,
same CSV header, so the reference's analysis scripts (data_analysis.py) read these files.
"""
import csv
import os

import numpy as np

META_HEADER = ["planning_time", "mass", "distance", "success", "filename"]


def save_traj_data(traj, data_path, filename):
    """collect_data.py:108-131.  `traj` is a Trajectory or a sequence of Conf (None: no-op)."""
    if traj is None:
        return None
    path = getattr(traj, "path", traj)
    confs = [c.values for c in path]
    velocities = [c.velocities for c in path]
    accelerations = [c.accelerations for c in path]
    torques = [c.torques for c in path]
    ts = [c.dt for c in path]
    os.makedirs(data_path, exist_ok=True)
    out = os.path.join(data_path, filename)
    np.savez(out, q=confs, qd=velocities, qdd=accelerations, torques=torques, ts=ts)
    return out if out.endswith(".npz") else out + ".npz"


def load_traj_data(path):
    """Inverse of save_traj_data: dict of the five arrays (allow_pickle stays off)."""
    z = np.load(path)
    return {k: z[k] for k in ("q", "qd", "qdd", "torques", "ts")}


class MetaWriter:
    """collect_data.py:146-159: the meta CSV (header once, then one row per trajectory)."""

    def __init__(self, path):
        self.path = path
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w", newline="") as f:
            csv.writer(f, delimiter=",").writerow(META_HEADER)

    def write(self, planning_time, mass, distance, success, filename):
        with open(self.path, "a", newline="") as f:
            csv.writer(f, delimiter=",").writerow(
                [planning_time, mass, distance, bool(success), filename])
