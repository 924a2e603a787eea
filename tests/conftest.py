import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (libtcmp.so compute calls)")


def engine_with_split(split):
    """A fresh engine whose k_edges lane groups are capped at `split` lanes per edge
    (TCMP_EDGE_SPLIT, read once at tcmp_create): 1 runs k_edges<., 1> -- the kernel of every
    full 262,144-lane bench round -- at any round size, 2 runs k_edges<., 2> wherever a round
    fits half the persistent grid.  None: the default engine choice (up to 4)."""
    from torque_constrained_motion_planning_amd import _lib
    old = os.environ.get("TCMP_EDGE_SPLIT")
    if split is not None:
        os.environ["TCMP_EDGE_SPLIT"] = str(split)
    try:
        return _lib.Engine(0)
    finally:
        if old is None:
            os.environ.pop("TCMP_EDGE_SPLIT", None)
        else:
            os.environ["TCMP_EDGE_SPLIT"] = old


@pytest.fixture(autouse=True)
def _oracle_state_reset():
    """The oracle library's scene state (installed convex meshes, self-collision switch) is
    module-level: a test that installs it (e.g. bench.py's C5 sub-line on the CPU fake engine)
    must not leak it into the next one."""
    yield
    if "oracle" in sys.modules:
        O = sys.modules["oracle"]
        try:
            O.set_meshes(None)
            O.set_self_collision(False)
        except OSError:  # the library never loaded
            pass
