"""Multi-GPU query sharding: independent planning queries are dealt round-robin
to ranks (one process per GPU); each rank plans its queries with its own engine, and the
solved trajectories are gathered to rank 0 -- the only collective on the path (RCCL over
xGMI with the nccl backend, gloo in the CPU tests).

Trajectory record per query: rows of [q(7), qd(7), qdd(7), dt(1)] (Conf values,
velocities, accelerations, dt of create_trajectory, utils.py:3340-3347), float64.
"""
import numpy as np

TRAJ_COLS = 22


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


def gather_trajectories(dist, trajs, query_ids, world, rank, device="cpu"):
    """Gather every rank's list of (query_id, (K,22) array) to rank 0.

    One size exchange (all_gather of counts) and one padded gather of a single buffer per
    rank.  Returns {query_id: (K,22) array} on rank 0, None elsewhere."""
    import torch
    # header: per local query (id, rows)
    n_local = len(trajs)
    counts = torch.tensor([n_local, sum(len(t) for t in trajs)], dtype=torch.int64, device=device)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    max_q = max(int(c[0]) for c in all_counts)
    max_rows = max(int(c[1]) for c in all_counts)
    hdr = torch.full((max(max_q, 1), 2), -1, dtype=torch.int64, device=device)
    body = torch.zeros((max(max_rows, 1), TRAJ_COLS), dtype=torch.float64, device=device)
    r = 0
    for i, (qid, t) in enumerate(zip(query_ids, trajs)):
        hdr[i, 0] = int(qid)
        hdr[i, 1] = len(t)
        if len(t):
            body[r:r + len(t)] = torch.from_numpy(np.asarray(t, dtype=np.float64)).to(device)
        r += len(t)
    hdrs = [torch.zeros_like(hdr) for _ in range(world)] if rank == 0 else None
    bodies = [torch.zeros_like(body) for _ in range(world)] if rank == 0 else None
    dist.gather(hdr, hdrs, dst=0)
    dist.gather(body, bodies, dst=0)
    if rank != 0:
        return None
    result = {}
    for h, b in zip(hdrs, bodies):
        h = h.cpu().numpy()
        b = b.cpu().numpy()
        r = 0
        for qid, k in h:
            if qid < 0:
                continue
            result[int(qid)] = b[r:r + k].copy()
            r += k
    return result
