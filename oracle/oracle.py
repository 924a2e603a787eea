"""ctypes wrapper of the CPU oracle (oracle/tcmp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, tests/golden/gen_golden.py,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIB_PATH: another build of the same sources (the sanitizer build, `make -C oracle asan`)
LIB_PATH = os.environ.get("ORC_LIB_PATH", os.path.join(HERE, "build", "liboracle.so"))

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


class RrtCfg(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_double * 7), ("goal", ctypes.c_double * 7),
        ("max_samples", ctypes.c_long), ("batch", ctypes.c_int), ("torque_mode", ctypes.c_int),
        ("mass", ctypes.c_double), ("exec_time", ctypes.c_double), ("radius", ctypes.c_double),
        ("goal_prob", ctypes.c_double), ("goal_tol", ctypes.c_double), ("seed", ctypes.c_uint64),
        ("replay_random", _dp), ("n_replay_random", ctypes.c_long),
        ("replay_uniform", _dp), ("n_replay_uniform", ctypes.c_long),
        ("obs", _dp), ("n_obs", ctypes.c_int), ("cull", ctypes.c_int), ("validate", ctypes.c_int),
        ("informed", ctypes.c_int),
    ]


class RrtResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int)] + [(n, ctypes.c_long) for n in (
        "n_nodes", "n_samples", "edge_steps", "goal_node", "n_waypoints", "n_traj", "first_fail",
        "n_rewires")]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_rne.argtypes = [_dp, _dp, _dp, ctypes.c_double, _dp]
        L.orc_rne_batch.argtypes = [_dp, _dp, _dp, ctypes.c_long, ctypes.c_double, _dp]
        L.orc_torque_ok.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_double]
        L.orc_dyn_tau.argtypes = [_dp, _dp, _dp, ctypes.c_double, _dp]
        L.orc_minjerk.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp]
        L.orc_fk_links.argtypes = [_dp, _dp]
        L.orc_collision.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int]
        L.orc_pair_pd.argtypes = [ctypes.c_int, _dp, _dp, ctypes.c_int]
        L.orc_pair_pd.restype = ctypes.c_double
        L.orc_check_edge.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                     ctypes.c_int, _ip, _dp]
        L.orc_fk8.argtypes = [_dp, _dp, _dp]
        L.orc_ik8.argtypes = [_dp, _dp, ctypes.c_double, _dp, ctypes.POINTER(ctypes.c_int)]
        L.orc_philox_uniforms.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _dp]
        L.orc_set_meshes.argtypes = [_dp, _ip, _dp, _ip, _ip, _ip, _dp, ctypes.c_int]
        L.orc_mesh_pair_pd.argtypes = [ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int]
        L.orc_mesh_pair_pd.restype = ctypes.c_double
        L.orc_set_self_collision.argtypes = [ctypes.c_int]
        L.orc_self_pairs.argtypes = [_ip]
        L.orc_self_pair_pd.argtypes = [ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int]
        L.orc_self_pair_pd.restype = ctypes.c_double
        L.orc_nearest.argtypes = [_dp, ctypes.c_long, _dp, ctypes.c_long, _dp, _ip, _dp]
        L.orc_set_threads.argtypes = [ctypes.c_int]
        L.orc_base_pd.argtypes = [_dp, ctypes.c_int, _dp]
        L.orc_body_collision.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int]
        L.orc_set_tree_out.argtypes = [_dp, _dp, _ip, ctypes.c_long]
        L.orc_rrt_run.argtypes = [ctypes.POINTER(RrtCfg), ctypes.POINTER(RrtResult), _dp,
                                  ctypes.c_long, _dp, _dp, _dp, _dp, ctypes.c_long]
        assert L.orc_sizeof_cfg() == ctypes.sizeof(RrtCfg), "oracle cfg layout mismatch"
        assert L.orc_sizeof_result() == ctypes.sizeof(RrtResult), "oracle result layout mismatch"
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(_dp)


def _arr(x, shape=None):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if shape is not None:
        a = a.reshape(shape)
    return a


def rne(q, qd, qdd, payload_mass=0.0):
    q = _arr(q, (-1, 7)); qd = _arr(qd, (-1, 7)); qdd = _arr(qdd, (-1, 7))
    tau = np.zeros_like(q)
    lib().orc_rne_batch(_d(q), _d(qd), _d(qdd), len(q), float(payload_mass), _d(tau))
    return tau


def dyn_tau(q, qd=None, qdd=None, mass=0.0):
    """dyn-mode joint torques (panda_primitives.py:60-116 restated, see tcmp_oracle.c)."""
    q = _arr(q, (7,))
    qd = np.zeros(7) if qd is None else _arr(qd, (7,))
    qdd = np.zeros(7) if qdd is None else _arr(qdd, (7,))
    tau = np.zeros(7)
    lib().orc_dyn_tau(_d(q), _d(qd), _d(qdd), float(mass), _d(tau))
    return tau


def torque_ok(q, mode, mass, qd=None, qdd=None):
    q = _arr(q, (7,))
    a = _arr(qd, (7,)) if qd is not None else None
    b = _arr(qdd, (7,)) if qdd is not None else None
    return bool(lib().orc_torque_ok(_d(q), _d(a) if a is not None else None,
                                    _d(b) if b is not None else None, int(mode), float(mass)))


def minjerk(waypoints, ni):
    P = _arr(waypoints, (-1, 7))
    K = (len(P) - 1) * ni
    q = np.zeros((max(K, 0), 7)); qd = np.zeros_like(q); qdd = np.zeros_like(q)
    rc = lib().orc_minjerk(_d(P), len(P), int(ni), _d(q), _d(qd), _d(qdd))
    if rc != 0:
        raise AssertionError("Invalid number of intervals chosen (must be greater than 0)")
    return q, qd, qdd


def fk_links(q):
    q = _arr(q, (7,))
    out = np.zeros((10, 12))
    lib().orc_fk_links(_d(q), _d(out))
    return out


def obstacles_array(obs):
    if obs is None or len(obs) == 0:
        return np.zeros((0, 15))
    return _arr(obs, (-1, 15))


def collision(q, obs, cull=1):
    q = _arr(q, (7,))
    o = obstacles_array(obs)
    return bool(lib().orc_collision(_d(q), _d(o) if len(o) else None, len(o), int(cull)))


def body_collision(q, obs, cull=1):
    """pairwise_collision(robot, b) over every obstacle b: all robot links, the static base
    panda_link0 included, at the -0.04 threshold, no joint-limit test."""
    o = obstacles_array(obs)
    return bool(lib().orc_body_collision(_d(_arr(q, (7,))), _d(o) if len(o) else None, len(o),
                                         int(cull)))


def base_pd(obs):
    """panda_link0's penetration depth against each box of `obs`, then each mesh set by
    set_meshes."""
    o = obstacles_array(obs)
    out = np.zeros(len(o) + lib().orc_mesh_count())
    if len(out):
        lib().orc_base_pd(_d(o) if len(o) else None, len(o), _d(out))
    return out


def pair_pd(link, q, box, method=0):
    """method 0: brute-force exact hull PD; 1: Gauss-map exact hull PD; 2: outer OBB PD;
    3: inner box PD."""
    q = _arr(q, (7,)); b = _arr(box, (15,))
    return lib().orc_pair_pd(int(link), _d(q), _d(b), int(method))


_mesh_keep = None


def set_meshes(pack):
    """Install convex-mesh obstacles (a hull.MeshPack, or None to clear) for every later
    collision / check_edge / rrt_run call (module-level state of the oracle library)."""
    global _mesh_keep
    L = lib()
    if pack is None or len(pack) == 0:
        L.orc_set_meshes(None, None, None, None, None, None, None, 0)
        _mesh_keep = None
        return
    arrs = (np.ascontiguousarray(pack.verts, dtype=np.float64),
            np.ascontiguousarray(pack.vert_off, dtype=np.intc),
            np.ascontiguousarray(pack.planes, dtype=np.float64),
            np.ascontiguousarray(pack.plane_off, dtype=np.intc),
            np.ascontiguousarray(pack.edges, dtype=np.intc),
            np.ascontiguousarray(pack.edge_off, dtype=np.intc),
            np.ascontiguousarray(pack.boxes, dtype=np.float64))
    _mesh_keep = arrs
    ip = lambda a: a.ctypes.data_as(_ip)  # noqa: E731
    L.orc_set_meshes(_d(arrs[0]), ip(arrs[1]), _d(arrs[2]), ip(arrs[3]), ip(arrs[4]),
                     ip(arrs[5]), _d(arrs[6]), int(pack.n))


def set_self_collision(on):
    """Self-collision pairs on/off for every later collision / check_edge / rrt_run call
    (module-level state of the oracle library)."""
    lib().orc_set_self_collision(int(bool(on)))


def self_pairs():
    """Collision-link index pairs of get_self_link_pairs (utils.py:3138-3149), restated."""
    out = np.zeros(2 * 66, dtype=np.intc)
    n = lib().orc_self_pairs(out.ctypes.data_as(_ip))
    return [tuple(int(x) for x in out[2 * i:2 * i + 2]) for i in range(n)]


def self_pair_pd(a, b, q, method=0):
    """Penetration depth of link hulls a, b at q; method 0 brute force, 1 Gauss-map."""
    q = _arr(q, (7,))
    return lib().orc_self_pair_pd(int(a), int(b), _d(q), int(method))


def mesh_pair_pd(link, q, m, method=0):
    """Penetration depth of link hull vs installed mesh m; method 0 brute force (every
    candidate axis), 1 Gauss-map pruned."""
    q = _arr(q, (7,))
    return lib().orc_mesh_pair_pd(int(link), _d(q), int(m), int(method))


def check_edge(q1, q2, obs, torque_mode, mass, cull=1):
    q1 = _arr(q1, (7,)); q2 = _arr(q2, (7,)); o = obstacles_array(obs)
    ns = ctypes.c_int(0)
    last = np.zeros(7)
    s = lib().orc_check_edge(_d(q1), _d(q2), _d(o) if len(o) else None, len(o),
                             int(torque_mode), float(mass), int(cull), ctypes.byref(ns), _d(last))
    return s, ns.value, last


def fk8(q):
    """T_0^8 (4x4) by the reference DH chain (rne.py:32-63)."""
    q = _arr(q, (7,))
    R = np.zeros(9)
    p = np.zeros(3)
    lib().orc_fk8(_d(q), _d(R), _d(p))
    T = np.eye(4)
    T[:3, :3] = R.reshape(3, 3)
    T[:3, 3] = p
    return T


def ik8(T, q7):
    """Closed-form IK of T_0^8 with joint 7 = q7: (solutions (k, 7), branch ids (k,))."""
    T = np.asarray(T, dtype=np.float64)
    R = np.ascontiguousarray(T[:3, :3]).reshape(9).copy()
    p = np.ascontiguousarray(T[:3, 3]).copy()
    sols = np.zeros(56)
    valid = np.zeros(8, dtype=np.intc)
    lib().orc_ik8(_d(R), _d(p), float(q7), _d(sols), valid.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    idx = np.nonzero(valid)[0]
    return sols.reshape(8, 7)[idx], idx


def nearest(tree, samples, weights=None):
    """argmin over tree rows of the weighted distance (rrt_star.py:9-14): (idx, dist)."""
    t = _arr(tree, (-1, 7)); s = _arr(samples, (-1, 7))
    w = _arr(np.full(7, 10.0) if weights is None else weights, (7,))
    idx = np.zeros(len(s), dtype=np.int32); dist = np.zeros(len(s))
    lib().orc_nearest(_d(t), len(t), _d(s), len(s), _d(w), idx.ctypes.data_as(_ip), _d(dist))
    return idx, dist


def philox_uniforms(seed, k):
    u = np.zeros(8)
    lib().orc_philox_uniforms(int(seed), int(k), _d(u))
    return u


def rrt_run(start, goal, max_samples, obs=None, torque_mode=0, mass=0.0, exec_time=5.0,
            batch=1, seed=0, replay_random=None, replay_uniform=None, radius=0.01,
            goal_prob=0.2, goal_tol=1e-2, cull=1, validate=True, cap_wp=1 << 16,
            cap_traj=1 << 20, informed=False, threads=1, tree=False):
    """Runs the restated RRT*; returns dict with status, counters, waypoints, traj.
    threads > 1 runs the per-lane loops of a round (nearest, edges, rewire scans) on that
    many OpenMP threads; results do not depend on it (used for bench-size fixtures).
    tree=True also returns the final tree ("tree_cfg", "tree_cost", "tree_parent")."""
    cfg = RrtCfg()
    cfg.start[:] = list(map(float, start)); cfg.goal[:] = list(map(float, goal))
    cfg.max_samples = int(max_samples); cfg.batch = int(batch); cfg.torque_mode = int(torque_mode)
    cfg.mass = float(mass); cfg.exec_time = float(exec_time); cfg.radius = float(radius)
    cfg.goal_prob = float(goal_prob); cfg.goal_tol = float(goal_tol); cfg.seed = int(seed)
    keep = []
    if replay_random is not None:
        rr = _arr(replay_random); keep.append(rr)
        cfg.replay_random = _d(rr); cfg.n_replay_random = len(rr)
    if replay_uniform is not None:
        ru = _arr(replay_uniform, (-1, 7)); keep.append(ru)
        cfg.replay_uniform = _d(ru); cfg.n_replay_uniform = len(ru)
    o = obstacles_array(obs); keep.append(o)
    cfg.obs = _d(o) if len(o) else None
    cfg.n_obs = len(o); cfg.cull = int(cull); cfg.validate = int(bool(validate))
    if informed and not (replay_uniform is not None and int(batch) == 1):
        raise ValueError("informed is restated for the replayed B = 1 loop only")
    cfg.informed = int(bool(informed))
    res = RrtResult()
    wp = np.zeros((cap_wp, 7))
    tq = np.zeros((cap_traj, 7)); tqd = np.zeros_like(tq); tqdd = np.zeros_like(tq)
    psg = np.zeros(cap_traj)
    lib().orc_set_threads(int(threads))
    if tree:
        cap_n = int(max_samples) + 1
        t_cfg = np.zeros((cap_n, 7)); t_cost = np.zeros(cap_n)
        t_par = np.zeros(cap_n, dtype=np.int32)
        lib().orc_set_tree_out(_d(t_cfg), _d(t_cost), t_par.ctypes.data_as(_ip), cap_n)
    try:
        lib().orc_rrt_run(ctypes.byref(cfg), ctypes.byref(res), _d(wp), cap_wp, _d(tq), _d(tqd),
                          _d(tqdd), _d(psg), cap_traj)
    finally:
        lib().orc_set_threads(1)
        if tree:
            lib().orc_set_tree_out(None, None, None, 0)
    out = {f: getattr(res, f) for f, _ in RrtResult._fields_}
    W = res.n_waypoints
    K = res.n_traj
    out["waypoints"] = wp[:W].copy()
    out["q"] = tq[:K].copy(); out["qd"] = tqd[:K].copy(); out["qdd"] = tqdd[:K].copy()
    out["psg"] = psg[:K].copy()
    if tree:
        n = res.n_nodes
        out["tree_cfg"] = t_cfg[:n]; out["tree_cost"] = t_cost[:n]; out["tree_parent"] = t_par[:n]
    return out
