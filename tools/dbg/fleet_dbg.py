"""Fleet debug: one variant per process (tests/test_gpu_fleet.py case 5's shapes).
usage: python tools/dbg/fleet_dbg.py lone|fleet1|fleet2"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import test_gpu_fleet as T  # noqa: E402

mode = sys.argv[1]
plans = T._plans(5, [16, 12], [2], [5.0], base=405)
if mode == "lone":
    r = T._lone(plans, [10_000, 7_000], 4608)
elif mode == "fleet1":
    r = T._fleet(plans, [17_000], 4608)
elif mode == "fleet2a":
    r = T._fleet(plans, [10_000], 4608)
else:
    r = T._fleet(plans, [10_000, 7_000], 4608)
print(mode, "ok", [x[5] for x in r], flush=True)
