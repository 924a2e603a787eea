#!/usr/bin/env python3
"""Generate the Panda collision/kinematics data baked into the engine.

Dev-time only: reads the reference robot model (URDF constants restated below with
file:line citations, collision meshes read from /root/reference) and writes

  torque_constrained_motion_planning_amd/csrc/panda_geometry.inc   (C data, shared by
      the HIP engine and the CPU oracle -- data only, no algorithm)
  torque_constrained_motion_planning_amd/data/panda_geometry.npz   (same data for Python)

Nothing here runs on the GPU box; the generated files are committed.

Collision links (utils.py:3117-3123 moving links of the 7 arm joints that have collision
geometry, utils.py:3169-3170):
  link1..link7 (panda_mod.urdf:95-285), panda_hand (:12-26), panda_leftfinger (:27-43),
  panda_rightfinger (:44-61, collision origin rpy 0 0 pi).
Meshes: src/models/meshes/panda/collision/*.stl (binary STL). Bullet wraps a mesh
collision shape in a convex hull of its vertices; the STL files are already convex hulls
(every vertex is a hull vertex, every triangle a hull facet), checked below.

Per link we store, in the link frame:
  * hull vertices            (exact hull-vs-box penetration test)
  * hull facet planes n, dmax=max n.v, wmin=min n.v
  * hull edge directions     (edge x box-axis SAT candidates)
  * outer OBB  (hull subset)  -> conservative "free" cull
  * inner box  (subset hull)  -> conservative "collision" accept

The static base panda_link0 (panda_mod.urdf:7-11, link0.stl, no collision origin) is not a
moving link, but the body-level check of a grasp configuration (pairwise_collision(robot, b),
franka_ik_fast.py:78, panda_primitives.py:260) covers every link of the robot body.  Its
hull goes to panda_base.inc (world frame = base frame) with the same vertex / facet / edge
layout.
"""
import os
import struct
import sys

import numpy as np
from scipy.spatial import ConvexHull
from scipy.spatial.transform import Rotation

REF = "/root/reference/src/models/meshes/panda/collision"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT_INC = os.path.join(REPO, "torque_constrained_motion_planning_amd", "csrc", "panda_geometry.inc")
OUT_NPZ = os.path.join(REPO, "torque_constrained_motion_planning_amd", "data", "panda_geometry.npz")
OUT_BASE = os.path.join(REPO, "torque_constrained_motion_planning_amd", "csrc", "panda_base.inc")

LINKS = ["link1", "link2", "link3", "link4", "link5", "link6", "link7", "hand",
         "finger", "finger"]
LINK_NAMES = ["panda_link1", "panda_link2", "panda_link3", "panda_link4", "panda_link5",
              "panda_link6", "panda_link7", "panda_hand", "panda_leftfinger",
              "panda_rightfinger"]


def read_stl(path):
    d = open(path, "rb").read()
    cnt = struct.unpack("<I", d[80:84])[0]
    tri = np.frombuffer(d[84:84 + cnt * 50], dtype=np.dtype(
        [("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    return np.unique(tri["v"].reshape(-1, 3).astype(np.float64), axis=0)


def obb_fit(v, n_random=4000, seed=0):
    """Minimum-volume-ish oriented box containing v: random rotations + local refinement."""
    rng = np.random.default_rng(seed)

    def vol(R):
        p = v @ R
        return np.prod(p.max(0) - p.min(0))

    best_R = np.eye(3)
    best = vol(best_R)
    for R in Rotation.random(n_random, random_state=seed).as_matrix():
        f = vol(R)
        if f < best:
            best, best_R = f, R
    step = 0.1
    while step > 1e-4:
        improved = False
        for _ in range(60):
            dR = Rotation.from_rotvec(rng.normal(size=3) * step).as_matrix()
            R = best_R @ dR
            f = vol(R)
            if f < best:
                best, best_R, improved = f, R, True
        if not improved:
            step *= 0.5
    # orthonormalise exactly enough
    u, _, wt = np.linalg.svd(best_R)
    R = u @ wt
    if np.linalg.det(R) < 0:
        R[:, 2] = -R[:, 2]
    p = v @ R
    lo, hi = p.min(0), p.max(0)
    half = (hi - lo) / 2 + 1e-9
    c = R @ ((hi + lo) / 2)
    return c, R, half


def inner_box(c, R, half, planes):
    """Largest scaled copy of the OBB (same centre/axes) inside the hull."""
    n, d = planes[:, :3], planes[:, 3]
    lo_s, hi_s = 0.0, 1.0
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    for _ in range(80):
        s = 0.5 * (lo_s + hi_s)
        pts = c + (corners * (half * s)) @ R.T
        if np.all(pts @ n.T <= d[None, :] - 1e-7):
            lo_s = s
        else:
            hi_s = s
    if not np.all(c @ n.T <= d - 1e-7):
        return np.zeros(3)
    return half * lo_s * (1 - 1e-6)


def link_data(stl, flip_z_pi):
    v = read_stl(os.path.join(REF, stl + ".stl"))
    if flip_z_pi:
        # panda_mod.urdf:54 collision origin rpy="0 0 3.14159265359"
        a = 3.14159265359
        Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
        v = v @ Rz.T
    h = ConvexHull(v)
    assert len(h.vertices) == len(v), "mesh is not its own convex hull"
    planes = []
    for eq in h.equations:
        nrm = eq[:3] / np.linalg.norm(eq[:3])
        proj = v @ nrm
        planes.append([nrm[0], nrm[1], nrm[2], proj.max(), proj.min()])
    planes = np.array(planes)
    # merge duplicate planes (coplanar triangles)
    _, idx = np.unique(np.round(planes[:, :4], 10), axis=0, return_index=True)
    planes = planes[np.sort(idx)]
    # hull edges with their two adjacent facets (Gauss-map arcs): edge record =
    # direction e (unit), endpoint va, adjacent facet normals n1, n2
    tri_plane = []
    for eq in h.equations:
        nrm = eq[:3] / np.linalg.norm(eq[:3])
        key = np.round(np.concatenate([nrm, [(v @ nrm).max()]]), 10)
        tri_plane.append(int(np.where(np.all(np.round(planes[:, :4], 10) == key, axis=1))[0][0]))
    adj = {}
    for ti, s in enumerate(h.simplices):
        for a, b in ((0, 1), (1, 2), (0, 2)):
            adj.setdefault(tuple(sorted((int(s[a]), int(s[b])))), []).append(tri_plane[ti])
    dirs = []
    eidx = []
    for (a, b), fs in sorted(adj.items()):
        assert len(fs) == 2, "non-manifold hull edge"
        if fs[0] == fs[1]:
            continue  # edge interior to a merged facet
        e = v[b] - v[a]
        e = e / np.linalg.norm(e)
        dirs.append(np.concatenate([e, v[a], planes[fs[0], :3], planes[fs[1], :3]]))
        eidx.append([a, b, fs[0], fs[1]])
    dirs = np.array(dirs)
    c, R, half = obb_fit(v)
    ih = inner_box(c, R, half, planes[:, [0, 1, 2, 3]])
    return dict(verts=v, planes=planes, edges=dirs, edge_idx=np.array(eidx), obb_c=c, obb_R=R, obb_half=half,
                in_half=ih, hull_volume=h.volume)


def fmt(x):
    return repr(float(x))


def main():
    links = []
    for i, stl in enumerate(LINKS):
        d = link_data(stl, flip_z_pi=(i == 9))
        links.append(d)
        print(LINK_NAMES[i], "verts", len(d["verts"]), "planes", len(d["planes"]), "edges",
              len(d["edges"]), "obb/hull vol %.3f" % (np.prod(2 * d["obb_half"]) / d["hull_volume"]),
              "inner/hull %.3f" % (np.prod(2 * d["in_half"]) / d["hull_volume"]), file=sys.stderr)

    nv = [len(d["verts"]) for d in links]
    nf = [len(d["planes"]) for d in links]
    ne = [len(d["edges"]) for d in links]
    ov = np.concatenate([[0], np.cumsum(nv)]).astype(int)
    of = np.concatenate([[0], np.cumsum(nf)]).astype(int)
    oe = np.concatenate([[0], np.cumsum(ne)]).astype(int)

    L = []
    L.append("/* GENERATED by tools/gen_panda_geometry.py -- do not edit.")
    L.append(" * Panda collision geometry (link frames), from reference")
    L.append(" * src/models/panda_mod.urdf + src/models/meshes/panda/collision/ (STL).")
    L.append(" * Data only: included by the HIP engine and by the CPU oracle. */")
    L.append("#ifndef TCMP_GEO_QUAL")
    L.append("#define TCMP_GEO_QUAL static const")
    L.append("#endif")
    L.append("#define TCMP_NLINKS 10")
    L.append("#define TCMP_TOTAL_VERTS %d" % ov[-1])
    L.append("#define TCMP_TOTAL_PLANES %d" % of[-1])
    L.append("#define TCMP_TOTAL_EDGES %d" % oe[-1])
    L.append("TCMP_GEO_QUAL int tcmp_geo_vert_off[TCMP_NLINKS + 1] = {%s};" % ", ".join(map(str, ov)))
    L.append("TCMP_GEO_QUAL int tcmp_geo_plane_off[TCMP_NLINKS + 1] = {%s};" % ", ".join(map(str, of)))
    L.append("TCMP_GEO_QUAL int tcmp_geo_edge_off[TCMP_NLINKS + 1] = {%s};" % ", ".join(map(str, oe)))
    L.append("/* verts: x y z 0 (padded to 4 doubles) */")
    L.append("TCMP_GEO_QUAL double tcmp_geo_verts[TCMP_TOTAL_VERTS * 4] = {")
    for d in links:
        for p in d["verts"]:
            L.append("  %s, %s, %s, 0.0," % tuple(fmt(x) for x in p))
    L.append("};")
    L.append("/* planes: nx ny nz dmax wmin 0 0 0 (padded to 8 doubles) */")
    L.append("TCMP_GEO_QUAL double tcmp_geo_planes[TCMP_TOTAL_PLANES * 8] = {")
    for d in links:
        for p in d["planes"]:
            L.append("  %s, %s, %s, %s, %s, 0.0, 0.0, 0.0," % tuple(fmt(x) for x in p))
    L.append("};")
    L.append("/* hull edges: e(3) 0 | endpoint va(3) 0 | facet normal n1(3) 0 | n2(3) 0 */")
    L.append("TCMP_GEO_QUAL double tcmp_geo_edges[TCMP_TOTAL_EDGES * 16] = {")
    for d in links:
        for p in d["edges"]:
            vals = list(p[0:3]) + [0.0] + list(p[3:6]) + [0.0] + list(p[6:9]) + [0.0] + list(p[9:12]) + [0.0]
            L.append("  " + ", ".join(fmt(x) for x in vals) + ",")
    L.append("};")
    L.append("/* hull edges as indices: va vb (global vertex rows) f1 f2 (global plane rows) */")
    L.append("TCMP_GEO_QUAL unsigned short tcmp_geo_edge_idx[TCMP_TOTAL_EDGES * 4] = {")
    for i, d in enumerate(links):
        for a, b, f1, f2 in d["edge_idx"]:
            L.append("  %d, %d, %d, %d," % (a + ov[i], b + ov[i], f1 + of[i], f2 + of[i]))
    L.append("};")
    L.append("/* per link box data: obb centre(3) axes R row-major (9, columns = box axes) "
             "outer half(3) inner half(3) -> 18 doubles */")
    L.append("TCMP_GEO_QUAL double tcmp_geo_boxes[TCMP_NLINKS * 18] = {")
    for d in links:
        vals = list(d["obb_c"]) + list(d["obb_R"].reshape(-1)) + list(d["obb_half"]) + list(d["in_half"])
        L.append("  " + ", ".join(fmt(x) for x in vals) + ",")
    L.append("};")
    os.makedirs(os.path.dirname(OUT_INC), exist_ok=True)
    with open(OUT_INC, "w") as f:
        f.write("\n".join(L) + "\n")
    base = link_data("link0", flip_z_pi=False)
    print("panda_link0 verts", len(base["verts"]), "planes", len(base["planes"]), "edges",
          len(base["edges"]), file=sys.stderr)
    B = []
    B.append("/* GENERATED by tools/gen_panda_geometry.py -- do not edit.")
    B.append(" * Static base panda_link0 (panda_mod.urdf:7-11, link0.stl): convex hull in the base")
    B.append(" * (= world) frame for the body-level grasp check.  Data only. */")
    B.append("#ifndef TCMP_GEO_QUAL")
    B.append("#define TCMP_GEO_QUAL static const")
    B.append("#endif")
    B.append("#define TCMP_BASE_NV %d" % len(base["verts"]))
    B.append("#define TCMP_BASE_NF %d" % len(base["planes"]))
    B.append("#define TCMP_BASE_NE %d" % len(base["edges"]))
    B.append("/* verts: x y z 0 */")
    B.append("TCMP_GEO_QUAL double tcmp_base_verts[TCMP_BASE_NV * 4] = {")
    for p in base["verts"]:
        B.append("  %s, %s, %s, 0.0," % tuple(fmt(x) for x in p))
    B.append("};")
    B.append("/* planes: nx ny nz dmax */")
    B.append("TCMP_GEO_QUAL double tcmp_base_planes[TCMP_BASE_NF * 4] = {")
    for p in base["planes"]:
        B.append("  %s, %s, %s, %s," % tuple(fmt(x) for x in p[:4]))
    B.append("};")
    B.append("/* edges: va vb f1 f2 (rows of the arrays above) */")
    B.append("TCMP_GEO_QUAL int tcmp_base_edges[TCMP_BASE_NE * 4] = {")
    for a, b, f1, f2 in base["edge_idx"]:
        B.append("  %d, %d, %d, %d," % (a, b, f1, f2))
    B.append("};")
    lo, hi = base["verts"].min(0), base["verts"].max(0)
    B.append("/* AABB lo(3) hi(3) */")
    B.append("TCMP_GEO_QUAL double tcmp_base_aabb[6] = {%s};" % ", ".join(fmt(x) for x in list(lo) + list(hi)))
    with open(OUT_BASE, "w") as f:
        f.write("\n".join(B) + "\n")
    os.makedirs(os.path.dirname(OUT_NPZ), exist_ok=True)
    np.savez(OUT_NPZ,
             verts=np.concatenate([d["verts"] for d in links]),
             planes=np.concatenate([d["planes"] for d in links]),
             edges=np.concatenate([d["edges"] for d in links]),
             edge_idx=np.concatenate([d["edge_idx"] + [ov[i], ov[i], of[i], of[i]]
                                      for i, d in enumerate(links)]),
             vert_off=ov, plane_off=of, edge_off=oe,
             boxes=np.array([np.concatenate([d["obb_c"], d["obb_R"].reshape(-1), d["obb_half"],
                                             d["in_half"]]) for d in links]),
             link_names=np.array(LINK_NAMES),
             base_verts=base["verts"], base_planes=base["planes"][:, :4],
             base_edge_idx=base["edge_idx"])
    print("wrote", OUT_INC, OUT_NPZ, file=sys.stderr)


if __name__ == "__main__":
    main()
