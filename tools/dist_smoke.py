#!/usr/bin/env python3
"""Multi-rank rehearsal of libtcmp.so's RCCL path on whatever GPUs are visible: `world`
processes (spawned, one communicator each; ranks share GPUs round-robin when there are fewer
GPUs than ranks -- RCCL may refuse that) run tcmp_dist_barrier, tcmp_dist_allreduce (sum and
max) and tcmp_gather_paths, and rank 0 checks the gathered paths.

usage: python tools/dist_smoke.py [world] [port]
"""
import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, world, port, ngpu, q):
    sys.path.insert(0, REPO)
    try:
        from torque_constrained_motion_planning_amd import _lib, shard
        comm = _lib.Comm(rank, world, rank % ngpu, "127.0.0.1", port)
        comm.barrier()
        s = comm.allreduce([rank + 1.0, -rank], _lib.REDUCE_SUM)
        m = comm.allreduce([float(rank)], _lib.REDUCE_MAX)
        rng = np.random.default_rng(rank)
        ids = list(range(rank, 3 * world, world))
        trajs = [rng.normal(size=(int(rng.integers(0, 40)), 22)) for _ in ids]
        got = shard.gather_trajectories(comm, trajs, ids)
        comm.barrier()
        comm.close()
        q.put((rank, "ok", s.tolist(), m.tolist(), None if got is None else
               {k: (v.shape[0], float(v.sum())) for k, v in got.items()}))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, "error: %s" % e, None, None, None))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    port = int(sys.argv[2]) if len(sys.argv) > 2 else 29611
    sys.path.insert(0, REPO)
    from torque_constrained_motion_planning_amd import _lib
    L = _lib.load_library()
    import ctypes
    n = ctypes.c_int(0)
    L.tcmp_device_count(ctypes.byref(n))
    ngpu = max(1, n.value)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, world, port, ngpu, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
    print("gpus", ngpu, "world", world)
    for r in sorted(res):
        print(res[r])
    ok = all(res[r][1] == "ok" for r in res)
    if ok:
        exp = [sum(range(1, world + 1)) * 1.0, -sum(range(world)) * 1.0]
        assert res[0][2] == exp, res[0][2]
        assert res[0][3] == [world - 1.0]
        g = res[0][4]
        assert sorted(g) == list(range(3 * world)), sorted(g)
        for r in range(world):
            rng = np.random.default_rng(r)
            for k in range(r, 3 * world, world):
                t = rng.normal(size=(int(rng.integers(0, 40)), 22))
                assert g[k][0] == t.shape[0] and abs(g[k][1] - float(t.sum())) < 1e-9
        print("dist smoke ok")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
