"""MI355X-native torque-constrained RRT* engine (drop-in for the force-aware planning path of
HIRO-group/torque_constrained_motion_planning).

Python host API mirrors the reference modules (rrt_star, rne, min_jerk_v2, utils,
panda_primitives); compute runs in libtcmp.so (HIP, gfx950) through a ctypes C-ABI.
"""
from . import _lib  # noqa: F401
from ._lib import Engine, TcmpError, engine, load_library  # noqa: F401
from .scene import (Box, ConvexMesh, PandaRobot, Payload, get_mass, mesh_pack,  # noqa: F401
                    obstacle_array)

__version__ = "0.1.0"
