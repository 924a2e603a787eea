"""CPU: libtcmp.so builds for gfx950, loads without a GPU, and exports every entry point
include/tcmp.h declares.  No compute call is made here."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "tcmp.h")
LIB = os.path.join(REPO, "torque_constrained_motion_planning_amd", "libtcmp.so")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(?:int|const char\*)\s+(tcmp_\w+)\s*\(", txt)))


def test_header_declares_the_surface():
    names = declared()
    for must in ("tcmp_create", "tcmp_destroy", "tcmp_set_scene", "tcmp_check_edges",
                 "tcmp_nearest", "tcmp_rne_batch", "tcmp_minjerk", "tcmp_validate_traj",
                 "tcmp_plan_begin", "tcmp_plan_round", "tcmp_plan_run", "tcmp_plan_finish"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "torque_constrained_motion_planning_amd", "csrc")])
    L = ctypes.CDLL(LIB)
    for name in declared():
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (tcmp_\w+)", out))
    assert set(declared()) <= exported


def test_python_binding_matches_header():
    from torque_constrained_motion_planning_amd import _lib
    assert sorted(_lib.EXPORTS) == declared()


def test_struct_layouts():
    """ctypes mirrors of tcmp_plan_cfg / tcmp_plan_result have the C sizes."""
    from torque_constrained_motion_planning_amd import _lib
    src = r'''
#include <stdio.h>
#include "tcmp.h"
int main(void) { printf("%zu %zu\n", sizeof(tcmp_plan_cfg), sizeof(tcmp_plan_result)); return 0; }
'''
    tmp = os.path.join("/tmp", "tcmp_sizes_%d" % os.getpid())
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), tmp + ".c", "-o", tmp])
    a, b = map(int, subprocess.check_output([tmp]).split())
    os.remove(tmp)
    os.remove(tmp + ".c")
    assert a == ctypes.sizeof(_lib.PlanCfg)
    assert b == ctypes.sizeof(_lib.PlanResult)


def test_no_gpu_means_loud_failure():
    """Without a GPU the product path raises instead of falling back to the CPU."""
    from torque_constrained_motion_planning_amd import _lib
    n = ctypes.c_int(0)
    L = _lib.load_library()
    rc = L.tcmp_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.TcmpError):
        _lib.Engine(0)
