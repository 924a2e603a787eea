"""Multi-GPU query sharding: independent planning queries are dealt round-robin
to ranks (one process per GPU); each rank plans its queries with its own engines, and the
solved trajectories are gathered to rank 0 -- the only collective on the path, RCCL over
xGMI inside libtcmp.so (tcmp_gather_paths; no PyTorch).

Trajectory record per query: rows of [q(7), qd(7), qdd(7), dt(1)] (Conf values,
velocities, accelerations, dt of create_trajectory, utils.py:3340-3347), float64.
"""
import os

import numpy as np

from . import _lib

TRAJ_COLS = _lib.TRAJ_COLS


def queries_for_rank(n_queries, world, rank):
    """Round-robin deal of query ids (query q runs on rank q % world)."""
    return list(range(rank, n_queries, world))


def pack_trajectory(out):
    """{'q','qd','qdd','psg'} -> (K, 22) float64 (K = 0 when the query failed)."""
    if out is None or len(out["q"]) == 0:
        return np.zeros((0, TRAJ_COLS))
    return np.ascontiguousarray(np.concatenate(
        [out["q"], out["qd"], out["qdd"], np.asarray(out["psg"]).reshape(-1, 1)], axis=1))


def unpack_trajectory(a):
    a = np.asarray(a)
    return {"q": a[:, 0:7], "qd": a[:, 7:14], "qdd": a[:, 14:21], "psg": a[:, 21]}


def pack_paths(trajs, query_ids):
    """Local paths -> the wire form of tcmp_gather_paths: (ids, rows, data)."""
    ids = np.asarray(list(query_ids), dtype=np.int64)
    rows = np.asarray([len(t) for t in trajs], dtype=np.int64)
    data = (np.concatenate([np.asarray(t, dtype=np.float64).reshape(-1, TRAJ_COLS) for t in trajs])
            if len(trajs) else np.zeros((0, TRAJ_COLS)))
    return ids, rows, data


def unpack_paths(ids, rows, data):
    """(ids, rows, data) -> {query id: (K, 22) rows}."""
    out, r = {}, 0
    for q, k in zip(ids, rows):
        out[int(q)] = np.asarray(data[r:r + k]).copy()
        r += int(k)
    return out


def comm_from_env(device=None):
    """The job's communicator from the launcher's environment (torchrun / torch.distributed.run
    set RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).  The rendezvous of rank 0's
    RCCL id uses MASTER_PORT + 1 (the launcher's own store holds MASTER_PORT) unless
    TCMP_RDZV_PORT is set."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("TCMP_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
    return _lib.Comm(rank, world, local if device is None else device, addr, port)


def gather_trajectories(comm, trajs, query_ids):
    """Gather every rank's list of (K, 22) paths to rank 0 (tcmp_gather_paths over RCCL).
    Returns {query_id: (K, 22) array} on rank 0, None elsewhere."""
    ids, rows, data = pack_paths(trajs, query_ids)
    # one size exchange: rank 0 sizes its outputs from it and the gather reuses it
    sizes = comm.allgather_i64([len(ids), int(rows.sum())])
    got = comm.gather_paths(ids, rows, data, int(sizes[:, 0].sum()), int(sizes[:, 1].sum()),
                            sizes=sizes)
    if got is None:
        return None
    return unpack_paths(*got)


def gather_ok(got, expect_ids, sizes):
    """Rank 0's check of a gather: every expected query id arrived exactly once and the row
    counts add up to the all-gathered sizes."""
    sizes = np.asarray(sizes).reshape(-1, 2)
    if got is None or sorted(got) != sorted(int(i) for i in expect_ids):
        return False
    return sum(len(v) for v in got.values()) == int(sizes[:, 1].sum()) and \
        len(got) == int(sizes[:, 0].sum())


_M64 = (1 << 64) - 1


def _splitmix64(x):
    """splitmix64 on a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def tree_digest(cfg, cost, parent):
    """Host restatement of tcmp_plan_digest over a tree (cfg n x 7, cost n, parent n): the
    sum over nodes i of splitmix64 chained over (i, cfg[i] bits, cost[i] bits, parent[i]),
    mod 2^64.  Ranks of a shared-tree run compare it to prove they hold one tree."""
    cfg = np.ascontiguousarray(cfg, dtype=np.float64).reshape(-1, 7)
    n = len(cfg)
    words = np.concatenate([cfg, np.asarray(cost, dtype=np.float64).reshape(n, 1)], 1).view(np.uint64)
    x = _splitmix64(np.arange(n, dtype=np.uint64))
    for k in range(8):
        x = _splitmix64(x ^ words[:, k])
    x = _splitmix64(x ^ np.asarray(parent, dtype=np.int32).astype(np.uint32).astype(np.uint64))
    return int(x.astype(object).sum()) & _M64

