"""ctypes binding of libtcmp.so (include/tcmp.h).

The product path has no fallback: if the HIP library is missing or no GPU is visible, every
entry point raises.  Nothing here imports torch or the CPU oracle.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TCMP_LIB_PATH", os.path.join(HERE, "libtcmp.so"))

_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)

TORQUE_BASE, TORQUE_NOV, TORQUE_RNE, TORQUE_DYN = 0, 1, 2, 3
PLAN_OK, PLAN_START_GOAL_COLLISION, PLAN_NO_GOAL, PLAN_VALIDATION_FAILED, PLAN_MINJERK_ASSERT = range(5)

# C-ABI surface declared in include/tcmp.h (tests check the library exports all of them)
EXPORTS = [
    "tcmp_create", "tcmp_destroy", "tcmp_last_error", "tcmp_device_count", "tcmp_version",
    "tcmp_synchronize",
    "tcmp_set_scene", "tcmp_set_meshes", "tcmp_set_mesh_lods", "tcmp_set_mesh_spheres", "tcmp_set_self_collision", "tcmp_set_timing", "tcmp_rne_batch", "tcmp_torque_ok", "tcmp_check_configs",
    "tcmp_check_body", "tcmp_base_pd",
    "tcmp_check_edges", "tcmp_nearest", "tcmp_minjerk", "tcmp_validate_traj",
    "tcmp_plan_begin", "tcmp_plan_round", "tcmp_plan_goal", "tcmp_plan_run", "tcmp_plan_finish",
    "tcmp_plan_retrace",
    "tcmp_plan_run_shared", "tcmp_plan_run_group", "tcmp_plan_run_fused", "tcmp_plan_begin_many",
    "tcmp_plan_finish_many",
    "tcmp_plan_fetch", "tcmp_plan_tree", "tcmp_plan_digest", "tcmp_plan_debug_round", "tcmp_ik", "tcmp_fk",
    "tcmp_debug_counters", "tcmp_microbench",
    "tcmp_rendezvous", "tcmp_dist_init", "tcmp_dist_destroy", "tcmp_dist_rank",
    "tcmp_dist_barrier", "tcmp_dist_allreduce", "tcmp_dist_allgather_i64", "tcmp_gather_paths",
    "tcmp_gather_layout", "tcmp_gather_pack", "tcmp_gather_unpack", "tcmp_dist_rccl_ranks",
]
TRAJ_COLS = 22
REDUCE_SUM, REDUCE_MAX = 0, 1


class PlanCfg(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_double * 7), ("goal", ctypes.c_double * 7),
        ("weights", ctypes.c_double * 7), ("resolutions", ctypes.c_double * 7),
        ("radius", ctypes.c_double), ("goal_probability", ctypes.c_double),
        ("goal_tolerance", ctypes.c_double), ("payload_mass", ctypes.c_double),
        ("execution_time", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("max_nodes", ctypes.c_int64), ("max_batch", ctypes.c_int32),
        ("torque_mode", ctypes.c_int32),
    ]


class Hulls(ctypes.Structure):
    """struct tcmp_hulls"""
    _fields_ = [("verts", _dp), ("vert_off", _i32p), ("planes", _dp), ("plane_off", _i32p),
                ("edges", _i32p), ("edge_off", _i32p)]


class PlanResult(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32), ("goal_found", ctypes.c_int32),
        ("n_nodes", ctypes.c_int64), ("n_samples", ctypes.c_int64),
        ("goal_node", ctypes.c_int64), ("n_waypoints", ctypes.c_int64),
        ("n_traj", ctypes.c_int64), ("first_fail", ctypes.c_int64),
        ("edge_steps", ctypes.c_uint64), ("pairs_tested", ctypes.c_uint64),
        ("pairs_sat", ctypes.c_uint64), ("pairs_exact", ctypes.c_uint64),
        ("nn_pairs", ctypes.c_uint64),
        ("ms_nearest", ctypes.c_double), ("ms_edges", ctypes.c_double),
        ("ms_insert", ctypes.c_double), ("ms_rewire", ctypes.c_double),
        ("ms_finish", ctypes.c_double), ("launches_nearest", ctypes.c_int64),
        ("nn_box_tests", ctypes.c_uint64), ("ms_nn_scan", ctypes.c_double),
        ("snap_sum", ctypes.c_uint64), ("nn_full_pairs", ctypes.c_uint64),
        ("launches_nn_scan", ctypes.c_int64), ("n_rewires", ctypes.c_uint64),
        ("rewire_steps", ctypes.c_uint64), ("graph_launches", ctypes.c_int64),
        ("fused_plans", ctypes.c_int64), ("ms_edge_prep", ctypes.c_double),
        ("goal_cost", ctypes.c_double), ("goal_depth", ctypes.c_int64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class TcmpError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load_library(path=LIB_PATH):
    """Load libtcmp.so (no compute call: usable on a CPU-only host)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise TcmpError("libtcmp.so not built (%s): run __graft_entry__.build()" % path)
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        L.tcmp_last_error.restype = ctypes.c_char_p
        L.tcmp_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.tcmp_destroy.argtypes = [vp]
        L.tcmp_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.tcmp_synchronize.argtypes = [vp]
        L.tcmp_set_scene.argtypes = [vp, _dp, ctypes.c_int32]
        L.tcmp_set_meshes.argtypes = [vp, _dp, _i32p, _dp, _i32p, _i32p, _i32p, _dp, ctypes.c_int32]
        L.tcmp_set_mesh_lods.argtypes = [vp, ctypes.POINTER(Hulls), ctypes.POINTER(Hulls),
                                         ctypes.c_int32]
        if hasattr(L, "tcmp_set_mesh_spheres"):  # absent from A/B builds of older sources
            L.tcmp_set_mesh_spheres.argtypes = [vp, _dp, ctypes.c_int32, ctypes.c_int32]
        L.tcmp_set_self_collision.argtypes = [vp, ctypes.c_int32]
        if hasattr(L, "tcmp_set_timing"):  # absent from A/B builds of older sources
            L.tcmp_set_timing.argtypes = [vp, ctypes.c_int32]
        L.tcmp_rne_batch.argtypes = [vp, _dp, _dp, _dp, ctypes.c_int64, ctypes.c_double, _dp]
        L.tcmp_torque_ok.argtypes = [vp, _dp, _dp, _dp, ctypes.c_int64, ctypes.c_int32,
                                     ctypes.c_double, _i32p]
        L.tcmp_check_configs.argtypes = [vp, _dp, ctypes.c_int64, _i32p]
        L.tcmp_check_body.argtypes = [vp, _dp, ctypes.c_int64, _i32p]
        L.tcmp_base_pd.argtypes = [vp, _dp, ctypes.c_int32]
        L.tcmp_check_edges.argtypes = [vp, _dp, _dp, ctypes.c_int64, _dp, ctypes.c_int32,
                                       ctypes.c_double, _i32p, _i32p, _dp]
        L.tcmp_nearest.argtypes = [vp, _dp, ctypes.c_int64, _dp, ctypes.c_int64, _dp, _i32p]
        L.tcmp_minjerk.argtypes = [vp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp, _dp]
        L.tcmp_validate_traj.argtypes = [vp, _dp, _dp, _dp, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.c_double, _i64p, _dp]
        L.tcmp_plan_begin.argtypes = [vp, ctypes.POINTER(PlanCfg), ctypes.POINTER(PlanResult)]
        L.tcmp_plan_round.argtypes = [vp, _dp, _u8p, ctypes.c_int32, _i32p]
        L.tcmp_plan_goal.argtypes = [vp, _i64p, _dp]
        L.tcmp_plan_run_shared.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32]
        L.tcmp_plan_run_group.argtypes = [ctypes.POINTER(vp), ctypes.c_int32, ctypes.c_int64,
                                          ctypes.c_int32]
        L.tcmp_plan_run.argtypes = [vp, ctypes.c_int64, ctypes.c_int32]
        if hasattr(L, "tcmp_plan_run_fused"):  # absent from A/B builds of older sources
            L.tcmp_plan_run_fused.argtypes = [ctypes.POINTER(vp), ctypes.c_int32, ctypes.c_int64,
                                              ctypes.c_int32]
            L.tcmp_plan_begin_many.argtypes = [ctypes.POINTER(vp), ctypes.c_int32,
                                               ctypes.POINTER(PlanCfg), ctypes.POINTER(PlanResult)]
            L.tcmp_plan_finish_many.argtypes = [ctypes.POINTER(vp), ctypes.c_int32,
                                                ctypes.POINTER(PlanResult)]
        L.tcmp_plan_finish.argtypes = [vp, ctypes.POINTER(PlanResult)]
        L.tcmp_plan_retrace.argtypes = [vp, ctypes.POINTER(PlanResult)]
        L.tcmp_plan_fetch.argtypes = [vp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.tcmp_plan_tree.argtypes = [vp, ctypes.c_int64, _dp, _dp, _i32p, _i64p]
        if hasattr(L, "tcmp_plan_digest"):  # absent from A/B builds of older sources
            L.tcmp_plan_digest.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), _i64p]
        L.tcmp_plan_debug_round.argtypes = [vp, ctypes.c_int64, _dp, _i32p, _dp, _i64p, _i32p]
        L.tcmp_ik.argtypes = [vp, _dp, _dp, ctypes.c_int64, _dp, _i32p]
        L.tcmp_fk.argtypes = [vp, _dp, ctypes.c_int64, _dp]
        L.tcmp_debug_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
        if hasattr(L, "tcmp_microbench"):  # absent from A/B builds of older sources
            L.tcmp_microbench.argtypes = [vp, _dp]
        i32 = ctypes.c_int32
        L.tcmp_rendezvous.argtypes = [i32, i32, ctypes.c_char_p, i32, vp, i32, i32]
        L.tcmp_dist_init.argtypes = [i32, i32, i32, ctypes.c_char_p, i32, ctypes.POINTER(vp)]
        L.tcmp_dist_destroy.argtypes = [vp]
        L.tcmp_dist_rank.argtypes = [vp, _i32p, _i32p]
        L.tcmp_dist_barrier.argtypes = [vp]
        L.tcmp_dist_allreduce.argtypes = [vp, _dp, i32, i32]
        L.tcmp_dist_allgather_i64.argtypes = [vp, _i64p, i32, _i64p]
        L.tcmp_gather_paths.argtypes = [vp, i32, _i64p, _i64p, _dp, _i64p, ctypes.c_int64,
                                        ctypes.c_int64, _i64p, _i64p, _dp, _i64p, _i64p]
        L.tcmp_gather_layout.argtypes = [i32, _i64p, _i64p, _i64p, _i64p, _i64p]
        if hasattr(L, "tcmp_gather_pack"):  # absent from A/B builds of older sources
            L.tcmp_gather_pack.argtypes = [i32, _i64p, _i64p, _dp, _i64p, _dp]
            L.tcmp_gather_unpack.argtypes = [i32, _i64p, _i64p, _dp, ctypes.c_int64,
                                             ctypes.c_int64, _i64p, _i64p, _dp, _i64p, _i64p]
        L.tcmp_dist_rccl_ranks.argtypes = [vp, _i32p]
        _lib = L
        return L


def _d(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _rows(x, name="array"):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if a.ndim == 1:
        a = a.reshape(1, -1)
    if a.shape[-1] != 7:
        raise ValueError("%s must have 7 columns, got shape %s" % (name, a.shape))
    return a.reshape(-1, 7)


def pose_rows(poses):
    """(n, 4, 4) / (4, 4) homogeneous or (n, 12) rows -> contiguous (n, 12)."""
    a = np.asarray(poses, dtype=np.float64)
    if a.shape[-2:] == (4, 4):
        a = a.reshape(-1, 4, 4)
        a = np.concatenate([a[:, :3, :3].reshape(-1, 9), a[:, :3, 3]], axis=1)
    return np.ascontiguousarray(a.reshape(-1, 12))


class Engine:
    """One HIP device handle (tcmp_handle).  Not thread-safe; one per (thread, device)."""

    def __init__(self, device=0):
        self.L = load_library()
        h = ctypes.c_void_p()
        self._check(self.L.tcmp_create(int(device), ctypes.byref(h)))
        self.h = h
        self.device = device
        self._scene_key = None
        self._mesh_key = b""
        self._self_coll = False

    def _check(self, rc):
        if rc != 0:
            raise TcmpError("tcmp error %d: %s" % (rc, self.L.tcmp_last_error().decode()))

    def close(self):
        if getattr(self, "h", None):
            self.L.tcmp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        self._check(self.L.tcmp_synchronize(self.h))

    # ---- scene ------------------------------------------------------------------------
    def set_scene(self, obb, meshes=None):
        """Boxes (n, 15) and, optionally, convex meshes (a hull.MeshPack or ConvexMesh list)."""
        obb = np.ascontiguousarray(np.asarray(obb, dtype=np.float64).reshape(-1, 15))
        if meshes is not None and not hasattr(meshes, "key"):
            from .hull import pack_meshes
            meshes = pack_meshes(meshes)
        mkey = meshes.key() if meshes is not None and len(meshes) else b""
        key = (obb.tobytes(), mkey)
        if key == self._scene_key:
            return
        self._scene_key = None
        if self._mesh_key != mkey and not mkey:
            self._check(self.L.tcmp_set_meshes(self.h, None, None, None, None, None, None, None, 0))
        self._check(self.L.tcmp_set_scene(self.h, _d(obb) if len(obb) else None, len(obb)))
        if self._mesh_key != mkey and mkey:
            i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
            arrs = (np.ascontiguousarray(meshes.verts, dtype=np.float64), i32(meshes.vert_off),
                    np.ascontiguousarray(meshes.planes, dtype=np.float64), i32(meshes.plane_off),
                    i32(meshes.edges), i32(meshes.edge_off),
                    np.ascontiguousarray(meshes.boxes, dtype=np.float64))
            ip = lambda a: a.ctypes.data_as(_i32p)  # noqa: E731
            self._check(self.L.tcmp_set_meshes(self.h, _d(arrs[0]), ip(arrs[1]), _d(arrs[2]),
                                               ip(arrs[3]), ip(arrs[4]), ip(arrs[5]),
                                               _d(arrs[6]), int(len(meshes))))
            if getattr(meshes, "inner", None) is not None:
                keep = []

                def hulls(hs):
                    a = (np.ascontiguousarray(hs.verts, dtype=np.float64), i32(hs.vert_off),
                         np.ascontiguousarray(hs.planes, dtype=np.float64), i32(hs.plane_off),
                         i32(hs.edges), i32(hs.edge_off))
                    keep.append(a)
                    return Hulls(_d(a[0]), ip(a[1]), _d(a[2]), ip(a[3]), ip(a[4]), ip(a[5]))
                hi, ho = hulls(meshes.inner), hulls(meshes.outer)
                self._check(self.L.tcmp_set_mesh_lods(self.h, ctypes.byref(hi), ctypes.byref(ho),
                                                      int(len(meshes))))
            sph = getattr(meshes, "spheres", None)
            if sph is not None and hasattr(self.L, "tcmp_set_mesh_spheres"):
                sph = np.ascontiguousarray(sph, dtype=np.float64)
                self._check(self.L.tcmp_set_mesh_spheres(self.h, _d(sph), int(len(meshes)),
                                                         int(sph.shape[1])))
        self._mesh_key = mkey
        self._scene_key = key
        self._n_scene = len(obb) + (len(meshes) if meshes is not None else 0)

    # ---- batched physics --------------------------------------------------------------
    def rne(self, q, qd, qdd, payload_mass=0.0):
        q = _rows(q, "q"); qd = _rows(qd, "qd"); qdd = _rows(qdd, "qdd")
        tau = np.zeros_like(q)
        self._check(self.L.tcmp_rne_batch(self.h, _d(q), _d(qd), _d(qdd), len(q),
                                          float(payload_mass), _d(tau)))
        return tau

    def ik(self, poses, free_q7):
        """ikfast get_ik, batched: poses (n, 12) or (n, 4, 4) of panda_link8 in panda_link0,
        free_q7 (n,).  Returns (sols (n, 8, 7), count (n,)); row i has count[i] solutions."""
        poses = pose_rows(poses)
        free_q7 = np.ascontiguousarray(np.asarray(free_q7, dtype=np.float64).reshape(-1))
        if len(free_q7) != len(poses):
            raise ValueError("one free value per pose")
        sols = np.zeros((len(poses), 8, 7))
        cnt = np.zeros(len(poses), dtype=np.int32)
        self._check(self.L.tcmp_ik(self.h, _d(poses), _d(free_q7), len(poses), _d(sols),
                                   cnt.ctypes.data_as(_i32p)))
        return sols, cnt

    def debug_counters(self, n=8):
        out = (ctypes.c_uint64 * n)()
        self._check(self.L.tcmp_debug_counters(self.h, out, n))
        return list(out)

    def fk(self, q):
        """ikfast get_fk: q (n, 7) -> (n, 12) rows (rotation row-major, position)."""
        q = _rows(q, "q")
        out = np.zeros((len(q), 12))
        self._check(self.L.tcmp_fk(self.h, _d(q), len(q), _d(out)))
        return out

    def torque_ok(self, q, mode, mass, qd=None, qdd=None):
        q = _rows(q, "q")
        qd = None if qd is None else _rows(qd, "qd")
        qdd = None if qdd is None else _rows(qdd, "qdd")
        ok = np.zeros(len(q), dtype=np.int32)
        self._check(self.L.tcmp_torque_ok(self.h, _d(q), _d(qd), _d(qdd), len(q), int(mode),
                                          float(mass), ok.ctypes.data_as(_i32p)))
        return ok.astype(bool)

    def set_timing(self, enable):
        """Per-family device timing of plans on/off (tcmp_set_timing; on by default)."""
        self._check(self.L.tcmp_set_timing(self.h, int(bool(enable))))

    def set_self_collision(self, enable):
        """Self-collision pairs on/off for every later check (tcmp_set_self_collision)."""
        enable = bool(enable)
        if enable != self._self_coll:
            self._check(self.L.tcmp_set_self_collision(self.h, int(enable)))
            self._self_coll = enable

    def collides(self, q):
        q = _rows(q, "q")
        out = np.zeros(len(q), dtype=np.int32)
        self._check(self.L.tcmp_check_configs(self.h, _d(q), len(q), out.ctypes.data_as(_i32p)))
        return out.astype(bool)

    def collides_body(self, q):
        """any(pairwise_collision(robot, b) for b in obstacles) per configuration: every robot
        link, the static base panda_link0 included, no joint-limit test (tcmp_check_body)."""
        q = _rows(q, "q")
        out = np.zeros(len(q), dtype=np.int32)
        self._check(self.L.tcmp_check_body(self.h, _d(q), len(q), out.ctypes.data_as(_i32p)))
        return out.astype(bool)

    def base_pd(self):
        """panda_link0's penetration depth against each box, then each mesh (tcmp_base_pd)."""
        n = getattr(self, "_n_scene", 0)
        out = np.zeros(n)
        self._check(self.L.tcmp_base_pd(self.h, _d(out) if n else None, n))
        return out

    def check_edges(self, q_from, q_to, mode, mass, resolutions=None):
        a = _rows(q_from, "from"); b = _rows(q_to, "to")
        n = len(a)
        ns = np.zeros(n, dtype=np.int32); nt = np.zeros(n, dtype=np.int32)
        last = np.zeros((n, 7))
        res = None if resolutions is None else np.ascontiguousarray(resolutions, dtype=np.float64)
        self._check(self.L.tcmp_check_edges(self.h, _d(a), _d(b), n, _d(res), int(mode),
                                            float(mass), ns.ctypes.data_as(_i32p),
                                            nt.ctypes.data_as(_i32p), _d(last)))
        return ns, nt, last

    def nearest(self, tree, samples, weights=None):
        t = _rows(tree, "tree"); s = _rows(samples, "samples")
        idx = np.zeros(len(s), dtype=np.int32)
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        self._check(self.L.tcmp_nearest(self.h, _d(t), len(t), _d(s), len(s), _d(w),
                                        idx.ctypes.data_as(_i32p)))
        return idx

    def minjerk(self, waypoints, ni):
        P = _rows(waypoints, "waypoints")
        if int(ni) <= 0:
            raise AssertionError("Invalid number of intervals chosen (must be greater than 0)")
        K = (len(P) - 1) * int(ni)
        q = np.zeros((K, 7)); qd = np.zeros((K, 7)); qdd = np.zeros((K, 7))
        if K:
            self._check(self.L.tcmp_minjerk(self.h, _d(P), len(P), int(ni), _d(q), _d(qd), _d(qdd)))
        return q, qd, qdd

    def validate(self, q, qd, qdd, mode, mass, want_tau=True):
        q = _rows(q); qd = _rows(qd); qdd = _rows(qdd)
        ff = ctypes.c_int64(-1)
        tau = np.zeros_like(q) if want_tau else None
        self._check(self.L.tcmp_validate_traj(self.h, _d(q), _d(qd), _d(qdd), len(q), int(mode),
                                              float(mass), ctypes.byref(ff), _d(tau)))
        return ff.value, tau

    # ---- planner ----------------------------------------------------------------------
    def plan_begin(self, start, goal, mode, mass, exec_time, max_nodes, max_batch, seed=0,
                   weights=None, resolutions=None, radius=0.01, goal_probability=0.2,
                   goal_tolerance=1e-2):
        cfg = plan_cfg(start, goal, mode, mass, exec_time, max_nodes, max_batch, seed, weights,
                       resolutions, radius, goal_probability, goal_tolerance)
        res = PlanResult()
        self._check(self.L.tcmp_plan_begin(self.h, ctypes.byref(cfg), ctypes.byref(res)))
        return res.status

    def plan_round(self, samples=None, is_goal=None, nb=None, sync=True):
        gf = ctypes.c_int32(0)
        if samples is not None:
            s = _rows(samples)
            g = np.ascontiguousarray(np.asarray(is_goal, dtype=np.uint8).reshape(-1))
            self._check(self.L.tcmp_plan_round(self.h, _d(s), g.ctypes.data_as(_u8p), len(s),
                                               ctypes.byref(gf) if sync else None))
        else:
            self._check(self.L.tcmp_plan_round(self.h, None, None, int(nb),
                                               ctypes.byref(gf) if sync else None))
        return bool(gf.value)

    def plan_run_shared(self, comm, n_samples, batch):
        """Shared-tree rounds over the ranks of `comm` (tcmp_plan_run_shared): this rank takes
        its share of every round's `batch` lanes; afterwards every rank holds the whole tree."""
        self._check(self.L.tcmp_plan_run_shared(self.h, comm.h if comm is not None else None,
                                                int(n_samples), int(batch)))

    def plan_goal(self):
        """(goal node index or -1, its cost) of the open plan."""
        node = ctypes.c_int64(-1)
        cost = ctypes.c_double(0.0)
        self._check(self.L.tcmp_plan_goal(self.h, ctypes.byref(node), ctypes.byref(cost)))
        return node.value, cost.value

    def plan_run(self, n_samples, batch):
        self._check(self.L.tcmp_plan_run(self.h, int(n_samples), int(batch)))

    def plan_finish(self):
        r = PlanResult()
        self._check(self.L.tcmp_plan_finish(self.h, ctypes.byref(r)))
        return r

    def plan_retrace(self):
        """tcmp_plan_retrace: the waypoints only (a foreign dynam_fn follows)."""
        r = PlanResult()
        self._check(self.L.tcmp_plan_retrace(self.h, ctypes.byref(r)))
        return r

    def plan_fetch(self, r):
        W, K = r.n_waypoints, r.n_traj
        wp = np.zeros((W, 7)); q = np.zeros((K, 7)); qd = np.zeros((K, 7))
        qdd = np.zeros((K, 7)); psg = np.zeros(K); tau = np.zeros((K, 7))
        self._check(self.L.tcmp_plan_fetch(self.h, _d(wp), _d(q), _d(qd), _d(qdd), _d(psg), _d(tau)))
        return dict(waypoints=wp, q=q, qd=qd, qdd=qdd, psg=psg, tau=tau)

    def microbench(self):
        """Measured peaks of this device (tcmp_microbench): fp64 / packed-fp32 vector TFLOP/s
        and HBM GB/s of a 1 GiB device copy."""
        if not hasattr(self.L, "tcmp_microbench"):
            raise TcmpError("tcmp_microbench: not in this library build")
        out = np.zeros(4)
        self._check(self.L.tcmp_microbench(self.h, _d(out)))
        return {"fp64_tflops": float(out[0]), "fp32_tflops": float(out[1]),
                "hbm_gbs": float(out[2]), "hbm_copy_variant": int(out[3])}

    def plan_digest(self):
        """(digest, n_nodes) of the open plan's tree, computed on the device (tcmp_plan_digest;
        shard.tree_digest restates it on the host)."""
        d = ctypes.c_uint64(0)
        n = ctypes.c_int64(0)
        self._check(self.L.tcmp_plan_digest(self.h, ctypes.byref(d), ctypes.byref(n)))
        return int(d.value), int(n.value)

    def plan_tree(self, cap):
        cfg = np.zeros((cap, 7)); cost = np.zeros(cap); par = np.zeros(cap, dtype=np.int32)
        n = ctypes.c_int64(0)
        self._check(self.L.tcmp_plan_tree(self.h, int(cap), _d(cfg), _d(cost),
                                          par.ctypes.data_as(_i32p), ctypes.byref(n)))
        m = min(cap, n.value)
        return cfg[:m], cost[:m], par[:m], n.value

    def plan_debug_round(self, cap):
        """The last round's (candidates, nearest index, exact score, snapshot size)."""
        cand = np.zeros((cap, 7)); nn = np.zeros(cap, dtype=np.int32); score = np.zeros(cap)
        snap = ctypes.c_int64(0); nb = ctypes.c_int32(0)
        self._check(self.L.tcmp_plan_debug_round(self.h, int(cap), _d(cand),
                                                 nn.ctypes.data_as(_i32p), _d(score),
                                                 ctypes.byref(snap), ctypes.byref(nb)))
        m = min(cap, nb.value)
        return cand[:m], nn[:m], score[:m], snap.value


def check(rc):
    if rc != 0:
        raise TcmpError("tcmp error %d: %s" % (rc, load_library().tcmp_last_error().decode()))


class Comm:
    """tcmp_comm: the ranks of a multi-GPU job (one process per GPU) over RCCL; world == 1
    needs no communicator and touches no GPU."""

    def __init__(self, rank, world, device, addr="127.0.0.1", port=29500):
        self.L = load_library()
        self.rank, self.world = int(rank), int(world)
        h = ctypes.c_void_p()
        check(self.L.tcmp_dist_init(self.rank, self.world, int(device), addr.encode(), int(port),
                                    ctypes.byref(h)))
        self.h = h

    def barrier(self):
        check(self.L.tcmp_dist_barrier(self.h))

    def allreduce(self, values, op=REDUCE_SUM):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(-1)).copy()
        check(self.L.tcmp_dist_allreduce(self.h, _d(v), len(v), int(op)))
        return v

    def allgather_i64(self, values):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64).reshape(-1))
        out = np.zeros(self.world * len(v), dtype=np.int64)
        check(self.L.tcmp_dist_allgather_i64(self.h, v.ctypes.data_as(_i64p), len(v),
                                             out.ctypes.data_as(_i64p)))
        return out.reshape(self.world, len(v))

    def rccl_ranks(self):
        """ncclCommCount of the communicator (0: a one-rank job, no RCCL communicator)."""
        n = ctypes.c_int32(0)
        check(self.L.tcmp_dist_rccl_ranks(self.h, ctypes.byref(n)))
        return n.value

    def gather_paths(self, ids, rows, data, cap_queries, cap_rows, sizes=None):
        """tcmp_gather_paths: (ids, rows, data) on rank 0, None elsewhere.  sizes: the
        (world, 2) all-gathered (queries, rows) when the caller has them (no second
        size exchange)."""
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        data = np.ascontiguousarray(data, dtype=np.float64).reshape(-1, TRAJ_COLS)
        sz = None if sizes is None else np.ascontiguousarray(sizes, dtype=np.int64).reshape(-1)
        oi = np.zeros(max(cap_queries, 1), dtype=np.int64)
        orows = np.zeros(max(cap_queries, 1), dtype=np.int64)
        od = np.zeros((max(cap_rows, 1), TRAJ_COLS))
        nq, nr = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self.L.tcmp_gather_paths(self.h, len(ids), ids.ctypes.data_as(_i64p),
                                       rows.ctypes.data_as(_i64p), _d(data),
                                       None if sz is None else sz.ctypes.data_as(_i64p),
                                       int(cap_queries),
                                       int(cap_rows), oi.ctypes.data_as(_i64p),
                                       orows.ctypes.data_as(_i64p), _d(od), ctypes.byref(nq),
                                       ctypes.byref(nr)))
        if self.rank != 0:
            return None
        return oi[:nq.value], orows[:nq.value], od[:nr.value]

    def close(self):
        if getattr(self, "h", None):
            self.L.tcmp_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_layout(sizes):
    """tcmp_gather_layout: (q_off, r_off, total_q, total_r) of rank 0's receive buffer from
    the (world, 2) per-rank (queries, rows)."""
    sz = np.ascontiguousarray(np.asarray(sizes, dtype=np.int64).reshape(-1, 2))
    w = len(sz)
    qo = np.zeros(w, dtype=np.int64); ro = np.zeros(w, dtype=np.int64)
    tq, tr = ctypes.c_int64(0), ctypes.c_int64(0)
    check(load_library().tcmp_gather_layout(w, sz.ctypes.data_as(_i64p), qo.ctypes.data_as(_i64p),
                                            ro.ctypes.data_as(_i64p), ctypes.byref(tq),
                                            ctypes.byref(tr)))
    return qo, ro, tq.value, tr.value


def gather_pack(ids, rows, data):
    """tcmp_gather_pack: one rank's wire form of tcmp_gather_paths -- (hdr (n, 2) int64 of
    (id, rows), body (sum(rows), 22) float64), the bytes its transport sends to rank 0."""
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    data = np.ascontiguousarray(data, dtype=np.float64).reshape(-1, TRAJ_COLS)
    hdr = np.zeros((len(ids), 2), dtype=np.int64)
    body = np.zeros((max(int(rows.sum()) if len(rows) else 0, 0), TRAJ_COLS))
    check(load_library().tcmp_gather_pack(len(ids), ids.ctypes.data_as(_i64p),
                                          rows.ctypes.data_as(_i64p), _d(data),
                                          hdr.ctypes.data_as(_i64p), _d(body)))
    return hdr, body


def gather_unpack(sizes, hdr_all, body_all, cap_queries=None, cap_rows=None):
    """tcmp_gather_unpack (rank 0): every rank's wire form staged at tcmp_gather_layout's
    offsets -> (ids, rows, data) as tcmp_gather_paths returns them."""
    sz = np.ascontiguousarray(np.asarray(sizes, dtype=np.int64).reshape(-1, 2))
    hdr_all = np.ascontiguousarray(hdr_all, dtype=np.int64).reshape(-1, 2)
    body_all = np.ascontiguousarray(body_all, dtype=np.float64).reshape(-1, TRAJ_COLS)
    cq = len(hdr_all) if cap_queries is None else int(cap_queries)
    cr = len(body_all) if cap_rows is None else int(cap_rows)
    oi = np.zeros(max(cq, 1), dtype=np.int64)
    orows = np.zeros(max(cq, 1), dtype=np.int64)
    od = np.zeros((max(cr, 1), TRAJ_COLS))
    nq, nr = ctypes.c_int64(0), ctypes.c_int64(0)
    check(load_library().tcmp_gather_unpack(len(sz), sz.ctypes.data_as(_i64p),
                                            hdr_all.ctypes.data_as(_i64p), _d(body_all), cq, cr,
                                            oi.ctypes.data_as(_i64p), orows.ctypes.data_as(_i64p),
                                            _d(od), ctypes.byref(nq), ctypes.byref(nr)))
    return oi[:nq.value], orows[:nq.value], od[:nr.value]


def rendezvous(rank, world, addr, port, blob, timeout_ms=60000):
    """tcmp_rendezvous: rank 0's `blob` (bytes) to every rank; returns the received bytes."""
    buf = ctypes.create_string_buffer(bytes(blob) if rank == 0 else b"\0" * len(blob), len(blob))
    check(load_library().tcmp_rendezvous(int(rank), int(world), addr.encode(), int(port),
                                         ctypes.cast(buf, ctypes.c_void_p), len(blob),
                                         int(timeout_ms)))
    return buf.raw


_engines = {}


def plan_run_group(engines, n_samples, batch):
    """tcmp_plan_run_group: one process drives the shared-tree rounds of several engines (the
    same open plan on each); every engine ends with the tree one engine builds with
    plan_run(n_samples, batch)."""
    engines = list(engines)
    arr = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
    L = load_library()
    rc = L.tcmp_plan_run_group(arr, len(engines), int(n_samples), int(batch))
    if rc != 0:
        raise TcmpError("tcmp error %d: %s" % (rc, L.tcmp_last_error().decode()))


def plan_cfg(start, goal, mode, mass, exec_time, max_nodes, max_batch, seed=0, weights=None,
             resolutions=None, radius=0.01, goal_probability=0.2, goal_tolerance=1e-2):
    """tcmp_plan_cfg of one query (the reference's rrt_star arguments, rrt_star.py:151)."""
    cfg = PlanCfg()
    cfg.start[:] = [float(x) for x in start]
    cfg.goal[:] = [float(x) for x in goal]
    cfg.weights[:] = [float(x) for x in (weights if weights is not None else [10.0] * 7)]
    cfg.resolutions[:] = [float(x) for x in (resolutions if resolutions is not None else [0.1] * 7)]
    cfg.radius = float(radius)
    cfg.goal_probability = float(goal_probability)
    cfg.goal_tolerance = float(goal_tolerance)
    cfg.payload_mass = float(mass)
    cfg.execution_time = float(exec_time)
    cfg.seed = int(seed)
    cfg.max_nodes = int(max_nodes)
    cfg.max_batch = int(max_batch)
    cfg.torque_mode = int(mode)
    return cfg


def _many(engines):
    engines = list(engines)
    return engines, (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])


def plan_begin_many(engines, cfgs):
    """tcmp_plan_begin_many: plan_begin on every engine (cfgs: plan_cfg(...) each) with one
    host wait for all of them; returns the statuses."""
    engines, arr = _many(engines)
    c = (PlanCfg * len(engines))(*cfgs)
    res = (PlanResult * len(engines))()
    L = load_library()
    rc = L.tcmp_plan_begin_many(arr, len(engines), c, res)
    if rc != 0:
        raise TcmpError("tcmp error %d: %s" % (rc, L.tcmp_last_error().decode()))
    return [r.status for r in res]


def plan_finish_many(engines):
    """tcmp_plan_finish_many: plan_finish on every engine with one host wait for all."""
    engines, arr = _many(engines)
    res = (PlanResult * len(engines))()
    L = load_library()
    rc = L.tcmp_plan_finish_many(arr, len(engines), res)
    if rc != 0:
        raise TcmpError("tcmp error %d: %s" % (rc, L.tcmp_last_error().decode()))
    return list(res)


def plan_run_fused(engines, n_samples, batch):
    """tcmp_plan_run_fused: the open plans of several engines (one device, each its own scene,
    start, goal and seed, all at the same round) grow their trees in fused rounds -- one set of
    kernel launches per round for all of them.  Each engine ends with the tree its own
    plan_run(n_samples, batch) grows; finish and fetch each plan on its own engine."""
    engines = list(engines)
    arr = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
    L = load_library()
    rc = L.tcmp_plan_run_fused(arr, len(engines), int(n_samples), int(batch))
    if rc != 0:
        raise TcmpError("tcmp error %d: %s" % (rc, L.tcmp_last_error().decode()))


def engine(device=0):
    """Process-wide engine per device (the Python API's default handle)."""
    e = _engines.get(device)
    if e is None:
        e = Engine(device)
        _engines[device] = e
    return e
