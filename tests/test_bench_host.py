"""bench.py's host orchestration on the CPU: the step loop, --pipeline (steps in flight on
separate engines, kernel timings from a one-at-a-time pass), the multi-query deal and the JSON
line's fields, with the engine replaced by a stand-in (scene calls answered by the oracle, plan
calls returning synthetic results).  The GPU path itself is covered by the -m gpu tests."""
import json
import os
import sys
import threading
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


class _FakeEngine:
    """Scene calls from the oracle (gen_fullsize.OracleEngine); plan calls synthetic, with a
    short sleep so that concurrent steps really overlap in time."""
    live = 0
    peak = 0
    lock = threading.Lock()
    seeds = []

    def __init__(self, gpu=0):
        from gen_fullsize import OracleEngine
        self._o = OracleEngine()

    def __getattr__(self, name):  # set_scene / collides / torque_ok / check_edges
        return getattr(self._o, name)

    def microbench(self):
        return {"fp64_tflops": 1.0, "fp32_tflops": 2.0, "hbm_gbs": 3.0}

    def set_self_collision(self, enable):
        pass

    def set_timing(self, enable):
        self.timing = bool(enable)

    def plan_begin(self, start, goal, mode, mass, exec_time, max_nodes, max_batch, seed=0):
        from torque_constrained_motion_planning_amd import _lib
        self.n = max_nodes - 1
        with _FakeEngine.lock:
            _FakeEngine.seeds.append(seed)
        return _lib.PLAN_OK

    def plan_run(self, n_samples, batch):
        with _FakeEngine.lock:
            _FakeEngine.live += 1
            _FakeEngine.peak = max(_FakeEngine.peak, _FakeEngine.live)
        time.sleep(0.02)
        with _FakeEngine.lock:
            _FakeEngine.live -= 1

    def plan_finish(self):
        from torque_constrained_motion_planning_amd import _lib
        r = _lib.PlanResult()
        r.status, r.goal_found, r.n_samples, r.n_nodes = 0, 1, self.n, self.n // 2
        r.n_waypoints, r.n_traj, r.edge_steps, r.pairs_sat = 5, 40, 10 * self.n, self.n
        r.nn_pairs, r.nn_full_pairs, r.snap_sum = 800 * self.n, self.n * self.n, self.n
        r.ms_nearest, r.ms_nn_scan, r.ms_edges = 5.0, 4.0, 4.5
        r.launches_nearest, r.launches_nn_scan = 4, 3
        r.goal_node, r.goal_cost, r.goal_depth = self.n // 2 - 1, 3.5, 4
        return r

    def plan_fetch(self, r):
        K = r.n_traj
        return dict(waypoints=np.zeros((r.n_waypoints, 7)), q=np.zeros((K, 7)),
                    qd=np.zeros((K, 7)), qdd=np.zeros((K, 7)), psg=np.zeros(K),
                    tau=np.zeros((K, 7)))

    def synchronize(self):
        pass

    def close(self):
        pass


def _run_bench(monkeypatch, capsys, argv):
    import bench
    from torque_constrained_motion_planning_amd import _lib
    monkeypatch.setattr(_lib, "Engine", _FakeEngine)
    _FakeEngine.fused = []

    def fused(engines, n_samples, batch):  # tcmp_plan_run_fused: one call for the fleet
        _FakeEngine.fused.append(len(engines))
        engines[0].plan_run(n_samples, batch)

    monkeypatch.setattr(_lib, "plan_run_fused", fused)

    def begin_many(engines, cfgs):
        return [e.plan_begin(None, None, 0, 0.0, 0.0, c.max_nodes, c.max_batch, c.seed)
                for e, c in zip(engines, cfgs)]

    monkeypatch.setattr(_lib, "plan_begin_many", begin_many)
    monkeypatch.setattr(_lib, "plan_finish_many", lambda engines: [e.plan_finish() for e in engines])
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    _FakeEngine.live = _FakeEngine.peak = 0
    _FakeEngine.seeds = []
    bench.main()
    return json.loads(capsys.readouterr().out.strip().splitlines()[-1])


@pytest.mark.parametrize("pipe", [1, 2])
def test_bench_pipelined_single_query_steps(monkeypatch, capsys, pipe):
    line = _run_bench(monkeypatch, capsys, ["--workload", "c2", "--steps", "4", "--warmup", "1",
                                            "--pipeline", str(pipe), "--fleet", "0",
                                            "--no-cpu-baseline", "--no-alt"])
    assert line["steps"] == 4 and line["value"] > 0
    assert line["config"]["pipelined_steps"] == pipe
    assert line["config"]["streams_per_gpu"] == pipe
    assert _FakeEngine.peak == pipe  # the pipelined steps really ran concurrently
    # warmup (pipe queries) + 4 timed, + (1 warmup + 4) one-at-a-time queries when pipelined
    n = pipe + 4 + (5 if pipe > 1 else 0)
    assert len(_FakeEngine.seeds) == n and len(set(_FakeEngine.seeds)) == n
    assert ("one at a time" in line["kernel_timing"]) == (pipe > 1)
    assert line["config"]["queries_in_flight"] == pipe
    # the one-query-at-a-time figure rides beside the pipelined value
    assert ("config_single_query" in line) == (pipe > 1)
    if pipe > 1:
        sq = line["config_single_query"]
        assert sq["queries_in_flight"] == 1 and sq["steps"] == 4 and sq["value"] > 0
    # kernel figures per step from the synthetic results: 4.5 ms of edges in 4 launches
    assert line["kernel_ms_per_step"]["ms_edges"] == pytest.approx(4.5)
    assert line["roofline"]["avg_launch_ms"] == pytest.approx(
        4.0 / 3 if line["roofline"]["kernel"] == "k_nearest_wave32" else 4.5 / 4)
    assert line["stats_last_step"]["status"] == 0


def test_bench_fused_fleets(monkeypatch, capsys):
    """c4's default: a step's queries in fleets (fused rounds), `pipeline` fleets in flight,
    each on its own group of engines; every query still begins, finishes and is fetched on its
    own engine with its own seed."""
    line = _run_bench(monkeypatch, capsys, ["--workload", "c4", "--queries", "6", "--steps", "2",
                                            "--warmup", "1", "--pipeline", "2", "--fleet", "3",
                                            "--no-cpu-baseline"])
    c = line["config"]
    assert c["queries_per_step"] == 6 and c["fused_queries"] == 3
    assert c["streams_per_gpu"] == 6 and c["queries_in_flight"] == 6
    # two fleets per step: warmup 2 steps + 2 timed steps -> 8 fused calls of 3 plans, then
    # (1 warmup + 2) fleets one at a time for the kernel timings
    assert _FakeEngine.fused == [3] * 11
    assert _FakeEngine.peak == 2  # two fleets in flight
    # 4 steps x 6 queries + 3 one-at-a-time fleets x 3 queries, every seed distinct
    assert len(_FakeEngine.seeds) == 33 and len(set(_FakeEngine.seeds)) == 33
    assert "fleets of 3 queries" in line["kernel_timing"]
    assert line["value"] == pytest.approx(6 * 2 * 100_000 / (line["ms_per_step"] * 2e-3), rel=1e-6)


def test_bench_single_query_fleets(monkeypatch, capsys):
    """c3's default: consecutive steps' queries (one per step, each its own seed) in fleets of
    `fleet`, `pipeline` fleets in flight; the one-query-at-a-time line rides beside it."""
    line = _run_bench(monkeypatch, capsys, ["--workload", "c3", "--steps", "6", "--warmup", "1",
                                            "--fleet", "4", "--pipeline", "2",
                                            "--no-cpu-baseline", "--no-alt", "--no-sublines"])
    c = line["config"]
    assert c["fused_queries"] == 4 and c["queries_in_flight"] == 8 and c["streams_per_gpu"] == 8
    # warmup 1 x 2 x 4 = 8 steps (2 fleets of 4), timed 6 steps (two fleets of 3: one per
    # thread, rather than 4 + 2), 1 + 6 kernel-timing fleets of 4
    assert sorted(_FakeEngine.fused) == [3, 3] + [4] * 9  # (two threads: any order)
    assert line["steps"] == 6 and line["value"] > 0
    sq = line["config_single_query"]
    assert sq["queries_in_flight"] == 1 and sq["steps"] == 6
    # 8 + 6 + 7 x 4 fleet queries, + (1 + 6) one at a time: every seed distinct
    n = 8 + 6 + 28 + 7
    assert len(_FakeEngine.seeds) == n and len(set(_FakeEngine.seeds)) == n


def test_bench_multi_query_pipeline(monkeypatch, capsys):
    line = _run_bench(monkeypatch, capsys, ["--workload", "c4", "--queries", "3", "--steps", "2",
                                            "--warmup", "1", "--pipeline", "2", "--fleet", "0",
                                            "--no-cpu-baseline"])
    assert line["config"]["queries_per_step"] == 3 and line["config"]["fused_queries"] == 1
    assert _FakeEngine.fused == []
    assert line["config"]["streams_per_gpu"] == 6  # 3 queries x 2 steps in flight
    assert "one at a time" in line["kernel_timing"] and "config_single_query" not in line
    assert line["config"]["queries_in_flight"] == 6
    # warmup 2 steps x 3 queries + 2 timed steps x 3 queries, + (1 warmup + 2) one-at-a-time
    # kernel-timing queries; every seed distinct
    assert len(_FakeEngine.seeds) == 15 and len(set(_FakeEngine.seeds)) == 15
    assert line["value"] == pytest.approx(3 * 2 * 100_000 / (line["ms_per_step"] * 2e-3), rel=1e-6)


def test_bench_default_sublines(monkeypatch, capsys):
    """The default c3 command also measures BASELINE configs[3] (config_c4) and configs[4]
    (config_c5) after the headline, each a full line of its workload condensed into a sub-line
    (its own warmup, timed steps, rooflines and plan quality).  C5's one fleet in flight keeps
    event timing on its lead engine, so its kernel figures come from the timed steps (no second
    pass of 1e7-sample fleets)."""
    import bench
    small = dict(bench.WORKLOADS)
    small["c4"] = dict(small["c4"], queries=4, fleet=2, pipeline=2, samples=2000)
    small["c5"] = dict(small["c5"], meshes=2, samples=3000)
    monkeypatch.setattr(bench, "WORKLOADS", small)
    line = _run_bench(monkeypatch, capsys, ["--steps", "2", "--warmup", "1", "--samples", "5000",
                                            "--no-cpu-baseline", "--no-alt"])
    # --samples: not the default headline, so no sub-lines
    assert "config_c4" not in line and "config_c5" not in line
    small["c3"] = dict(small["c3"], samples=5000)
    line = _run_bench(monkeypatch, capsys, ["--steps", "2", "--warmup", "1", "--c5-steps", "3",
                                            "--no-cpu-baseline", "--no-alt"])
    q = line["quality"]
    assert q["queries"] == 2 and q["goal_rate"] == 1.0 and q["path_cost_mean"] == 3.5
    assert q["rounds_per_query"] == 4 and q["goal_depth_mean"] == 4
    c4, c5 = line["config_c4"], line["config_c5"]
    assert "error" not in c4 and "error" not in c5, (c4, c5)
    assert c4["steps"] == 2 and c4["config"]["queries_per_step"] == 4 and c4["value"] > 0
    assert c4["config"]["fused_queries"] == 2 and "roofline" in c4 and "quality" in c4
    assert c5["steps"] == 3 and c5["config"]["meshes"] == 2 and c5["config"]["fused_queries"] == 3
    assert c5["kernel_timing"].startswith("the timed steps")
    assert c5["roofline"]["avg_launch_ms"] > 0 and c5["quality"]["queries"] == 3
    assert "cpu_baseline" not in c4 and "config_alt" not in c5
