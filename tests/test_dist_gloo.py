"""CPU, world size 2 and 4: the multi-GPU sharding path without a GPU.

* tcmp_rendezvous (the TCP hand-off of rank 0's RCCL unique id, libtcmp.so) between real
  processes;
* tcmp_gather_paths' packing and unpacking through the C-ABI (a one-rank communicator needs
  no RCCL and touches no GPU);
* rank 0's receive layout of tcmp_gather_paths (tcmp_gather_layout) and the staging / unpacking
  around it at world sizes 2..8, ragged;
* the two-phase rendezvous failing on every rank together (a missing rank, another job);
* the 2-rank shard path: round-robin deal, per-rank planning (the CPU oracle stands in for the
  GPU engine), each rank's wire form from libtcmp.so's own tcmp_gather_pack, gloo moving the
  bytes to rank 0's offsets the way RCCL's send/recv does on the GPU, and rank 0's
  tcmp_gather_unpack -- only the byte transport is not libtcmp.so's; torch appears only in
  this test harness.
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rdzv_worker(rank, world, port, blob, q):
    sys.path.insert(0, REPO)
    from torque_constrained_motion_planning_amd import _lib
    got = _lib.rendezvous(rank, world, "127.0.0.1", port, blob if rank == 0 else bytes(len(blob)),
                          timeout_ms=60000)
    q.put((rank, got))


@pytest.mark.parametrize("world", [2, 4])
def test_rendezvous_processes(world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    blob = np.random.default_rng(world).bytes(128)  # the size of an ncclUniqueId
    procs = [ctx.Process(target=_rdzv_worker, args=(r, world, port, blob, q))
             for r in reversed(range(world))]  # non-root ranks first: they must retry
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(got) == list(range(world))
    assert all(v == blob for v in got.values())


def test_rendezvous_rejects_bad_arguments():
    sys.path.insert(0, REPO)
    from torque_constrained_motion_planning_amd import _lib
    with pytest.raises(_lib.TcmpError):
        _lib.rendezvous(2, 2, "127.0.0.1", 1234, b"x" * 8)
    assert _lib.rendezvous(0, 1, "127.0.0.1", 1234, b"abc") == b"abc"


def test_gather_paths_capi_one_rank():
    """tcmp_gather_paths packing/unpacking through the C-ABI (world 1: local copy)."""
    from torque_constrained_motion_planning_amd import _lib, shard
    comm = _lib.Comm(0, 1, 0)
    rng = np.random.default_rng(5)
    trajs = [rng.normal(size=(7, 22)), np.zeros((0, 22)), rng.normal(size=(3, 22))]
    got = shard.gather_trajectories(comm, trajs, [9, 4, 1])
    assert sorted(got) == [1, 4, 9]
    assert np.array_equal(got[9], trajs[0]) and np.array_equal(got[1], trajs[2])
    assert got[4].shape == (0, 22)
    # too small an output: status -4 after the collective, sizes reported
    ids, rows, data = shard.pack_paths(trajs, [9, 4, 1])
    with pytest.raises(_lib.TcmpError, match="capacity"):
        comm.gather_paths(ids, rows, data, 3, 5)
    assert (comm.allreduce([2.0, -1.0], _lib.REDUCE_MAX) == [2.0, -1.0]).all()
    assert (comm.allgather_i64([3, 4]) == [[3, 4]]).all()
    comm.barrier()
    comm.close()


def _plan(O, qid):
    start = np.array([0, -np.pi / 4, 0.0, -6 * np.pi / 8, 0, np.pi / 2, np.pi / 4])
    goal = np.array([0.5, 0.2, 0.1, -1.5, 0.3, 1.8, 0.2]) + 0.05 * (qid % 3)
    r = O.rrt_run(start, goal, 80, None, 2, 5.0, 0.3, batch=16, seed=qid)
    if r["status"] != 0:
        return None
    return r


def _shard_worker(rank, world, port, n_queries, q):
    """One rank of the shard path: round-robin deal, planning (the oracle stands in for the
    engine), the rank's wire form (tcmp_gather_pack), the size all-gather, gloo carrying the
    wire bytes to rank 0's offsets of tcmp_gather_layout (RCCL's ncclSend/ncclRecv on the
    GPU), and rank 0's tcmp_gather_unpack."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import dist_helpers
    import oracle as O
    from torque_constrained_motion_planning_amd import _lib, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids_local = shard.queries_for_rank(n_queries, world, rank)
    hdr, body = _lib.gather_pack(*shard.pack_paths(
        [shard.pack_trajectory(_plan(O, i)) for i in ids_local], ids_local))
    sizes = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([len(hdr), len(body)], dtype=torch.int64))
    sizes = torch.stack(sizes).numpy()
    if rank == 0:
        wires = [(hdr, body)]
        for r in range(1, world):
            nq, nr = (int(x) for x in sizes[r])
            h = torch.zeros(2 * nq, dtype=torch.int64)
            b = torch.zeros(22 * nr, dtype=torch.float64)
            dist.recv(h, src=r)
            dist.recv(b, src=r)
            wires.append((h.numpy().reshape(-1, 2), b.numpy().reshape(-1, 22)))
        got = shard.unpack_paths(*_lib.gather_unpack(sizes, *dist_helpers.stage_rank0(wires, sizes)))
        q.put((got, shard.gather_ok(got, range(n_queries), sizes)))
    else:
        dist.send(torch.from_numpy(hdr.reshape(-1).copy()), dst=0)
        dist.send(torch.from_numpy(body.reshape(-1).copy()), dst=0)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_gather_layout_and_staging(world):
    """tcmp_gather_layout (rank 0's receive offsets, libtcmp.so) + shard.pack_paths /
    stage_rank0 / unpack_paths at world sizes 2..8, ragged: ranks without queries, queries
    without rows (failed plans), 64 C4 queries dealt round-robin."""
    import dist_helpers
    from torque_constrained_motion_planning_amd import _lib, shard
    rng = np.random.default_rng(world)
    n_q = 64
    paths = {qid: rng.normal(size=(int(rng.integers(0, 40)) * (qid % 5 != 0), 22))
             for qid in range(n_q)}
    wires = []
    for r in range(world):
        mine = shard.queries_for_rank(n_q, world, r) if r != 1 else []  # rank 1 plans nothing
        wires.append(_lib.gather_pack(*shard.pack_paths([paths[i] for i in mine], mine)))
    sizes = np.array([[len(h), len(b)] for h, b in wires], dtype=np.int64)
    q_off, r_off, tq, tr = _lib.gather_layout(sizes)
    assert tq == sizes[:, 0].sum() and tr == sizes[:, 1].sum()
    assert q_off[0] == 0 and r_off[0] == 0
    assert np.array_equal(np.diff(q_off), sizes[:-1, 0]) and np.array_equal(np.diff(r_off), sizes[:-1, 1])
    hdr, staged = dist_helpers.stage_rank0(wires, sizes)
    assert (hdr >= 0).all() and not np.isnan(staged).any()  # every slot written exactly
    ids, rows, body = _lib.gather_unpack(sizes, hdr, staged)
    got = shard.unpack_paths(ids, rows, body)
    expect = [i for r in range(world) if r != 1 for i in shard.queries_for_rank(n_q, world, r)]
    assert shard.gather_ok(got, expect, sizes)
    assert list(ids) == expect  # rank order, then each rank's own order
    for qid in expect:
        assert np.array_equal(got[qid], paths[qid])
    # a lost or duplicated path fails the check
    assert not shard.gather_ok({k: v for k, v in got.items() if k != expect[-1]}, expect, sizes)
    assert not shard.gather_ok(got, expect + [999], sizes)
    with pytest.raises(_lib.TcmpError):
        _lib.gather_layout(-sizes - 1)
    # a header row lost or misplaced in transit: rank 0's unpacking refuses it (status -6)
    bad = hdr.copy()
    k = int(np.argmax(bad[:, 1]))
    bad[k, 1] += 1
    with pytest.raises(_lib.TcmpError, match="announced"):
        _lib.gather_unpack(sizes, bad, staged)
    # too small an output: the capacity error of tcmp_gather_paths
    with pytest.raises(_lib.TcmpError, match="capacity"):
        _lib.gather_unpack(sizes, hdr, staged, cap_rows=max(0, tr - 1))


def _rdzv_fail_worker(rank, world, port, job, q):
    sys.path.insert(0, REPO)
    os.environ["TCMP_JOB_ID"] = job
    from torque_constrained_motion_planning_amd import _lib
    try:
        _lib.rendezvous(rank, world, "127.0.0.1", port, b"\1" * 16 if rank == 0 else bytes(16),
                        timeout_ms=4000)
        q.put((rank, "ok"))
    except _lib.TcmpError as e:
        q.put((rank, str(e)))


@pytest.mark.parametrize("case", ["missing_rank", "other_job"])
def test_rendezvous_fails_together(case):
    """A rank that never arrives (world 3, two ranks started) or a rank of another job makes
    every started rank fail within the timeout -- nobody receives the id and goes on alone."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    if case == "missing_rank":
        specs = [(0, 3, "a"), (1, 3, "a")]
    else:
        specs = [(0, 2, "a"), (1, 2, "b")]
    procs = [ctx.Process(target=_rdzv_fail_worker, args=(r, w, port, j, q)) for r, w, j in specs]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v != "ok" for v in got.values()), got


def test_round_robin_deal():
    from torque_constrained_motion_planning_amd import shard
    world = 8
    seen = sorted(q for r in range(world) for q in shard.queries_for_rank(64, world, r))
    assert seen == list(range(64))
    assert shard.queries_for_rank(64, 8, 3)[:3] == [3, 11, 19]


def test_pack_roundtrip():
    from torque_constrained_motion_planning_amd import shard
    out = {"q": np.random.rand(5, 7), "qd": np.random.rand(5, 7), "qdd": np.random.rand(5, 7),
           "psg": np.arange(5.0)}
    a = shard.pack_trajectory(out)
    b = shard.unpack_trajectory(a)
    for k in out:
        assert np.array_equal(np.asarray(out[k]), b[k])
    assert shard.pack_trajectory(None).shape == (0, 22)


def test_gather_two_ranks_gloo():
    pytest.importorskip("torch")
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_queries = 5
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, n_queries, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from torque_constrained_motion_planning_amd import shard
    assert ok
    assert sorted(got) == list(range(n_queries))
    for qid in range(n_queries):
        ref = shard.pack_trajectory(_plan(O, qid))
        assert np.array_equal(got[qid], ref)
