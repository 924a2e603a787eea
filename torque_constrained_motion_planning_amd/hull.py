"""Convex-mesh obstacle records (host side of tcmp_set_meshes).

The reference hands Bullet a mesh file and Bullet collides the convex hull of its vertices
(`createCollisionShape(GEOM_MESH)`, utils.py:2833-2880 closest points against it).  The
engine needs the hull itself, so each `ConvexMesh` is reduced here, once, to:

  * hull vertices (world frame)
  * hull facet planes n.x <= d (coplanar triangles merged, unit outward n)
  * hull edges as (va, vb, f1, f2): endpoints and the two adjacent facets (Gauss-map arcs)
  * an outer oriented box containing the hull and an inner box inside it (same centre and
    axes), the conservative "free" / "collision" bounds the kernels test before the exact
    hull-vs-hull penetration depth.

`pack_meshes()` concatenates the records into the flat arrays of include/tcmp.h
(`tcmp_set_meshes`).  Mesh-local indices; row offsets per mesh.
"""
import numpy as np


def hull_data(points):
    """Convex hull of `points` -> (verts, planes[F,4] (n, dmax), edges[E,4] (va, vb, f1, f2)).

    Coplanar triangles are merged into one facet (rounded to 1e-10), and edges interior to a
    merged facet are dropped, as tools/gen_panda_geometry.py does for the robot links."""
    from scipy.spatial import ConvexHull
    pts = np.unique(np.asarray(points, dtype=np.float64).reshape(-1, 3), axis=0)
    h = ConvexHull(pts)
    keep = np.sort(h.vertices)
    remap = -np.ones(len(pts), dtype=np.int64)
    remap[keep] = np.arange(len(keep))
    v = pts[keep]
    planes, tri_plane, index = [], [], {}
    for eq in h.equations:
        nrm = eq[:3] / np.linalg.norm(eq[:3])
        dmax = float((v @ nrm).max())
        key = tuple(np.round(np.concatenate([nrm, [dmax]]), 10))
        if key not in index:
            index[key] = len(planes)
            planes.append([nrm[0], nrm[1], nrm[2], dmax])
        tri_plane.append(index[key])
    adj = {}
    for ti, s in enumerate(h.simplices):
        s = remap[s]
        for a, b in ((0, 1), (1, 2), (0, 2)):
            adj.setdefault(tuple(sorted((int(s[a]), int(s[b])))), []).append(tri_plane[ti])
    edges = []
    for (a, b), fs in sorted(adj.items()):
        if len(fs) != 2:
            raise ValueError("non-manifold hull edge")
        if fs[0] != fs[1]:
            edges.append([a, b, fs[0], fs[1]])
    return v, np.array(planes, dtype=np.float64), np.array(edges, dtype=np.int32).reshape(-1, 4)


# Level-of-detail sizes (measured on C5, edges per 1e6 samples: outer 24 / 16 / 12 / 8 ->
# 421 / 405 / 375 / 453 ms): the outer LOD (the "free" certificate, tested on every undecided
# pair) takes the facet normals of a 12-vertex inner hull -- cheap, and it still certifies
# most free pairs; the inner LOD (the "collision" certificate, tested only when the outer
# one fails) keeps 48 vertices, so fewer colliding pairs fall through to the full
# hull-vs-hull pass (inner 32 / 48 / 64 -> 385 / 375 / 393 ms with the 12-vertex outer).
INNER_LOD_K = 48
OUTER_LOD_K = 12


def inner_lod(verts, k=24):
    """Inner level of detail: the hull of k of the hull's vertices (a subset of the hull),
    chosen greedily -- axis extremes first, then repeatedly the vertex farthest outside the
    current subset hull.  Any penetration depth computed with it is <= the full hull's."""
    from scipy.spatial import ConvexHull
    v = np.asarray(verts, dtype=np.float64)
    if len(v) <= k:
        return hull_data(v)
    idx = sorted({int(np.argmax(v @ d)) for d in np.vstack([np.eye(3), -np.eye(3)])})
    while len(idx) < 4:
        idx.append(next(i for i in range(len(v)) if i not in idx))
    while len(idx) < k:
        eq = ConvexHull(v[idx]).equations
        d = (v @ eq[:, :3].T + eq[:, 3]).max(1)
        j = int(np.argmax(d))
        if d[j] <= 1e-12:
            break
        idx.append(j)
    return hull_data(v[sorted(idx)])


def outer_lod(verts, inner_planes):
    """Outer level of detail: the H-polytope of the inner LOD's facet normals pushed out to
    the full hull's support (a superset of the hull -- exactly, the planes are supports --
    so depths computed with it are >= the full hull's), returned as the hull of its vertices
    (hull_data: facets re-derived from those vertices, so containment holds by construction)."""
    from scipy.spatial import HalfspaceIntersection
    v = np.asarray(verts, dtype=np.float64)
    n = inner_planes[:, :3] / np.linalg.norm(inner_planes[:, :3], axis=1)[:, None]
    d = (v @ n.T).max(0)
    hs = HalfspaceIntersection(np.hstack([n, -d[:, None]]), v.mean(0))
    return hull_data(hs.intersections)


def fit_boxes(verts, planes, n_random=300, seed=0):
    """Outer oriented box (contains the hull) and inner half extents (box of the same centre
    and axes inside the hull).  PCA axes refined over random rotations for a small volume;
    any containing box is correct, a tighter one only culls more."""
    from scipy.spatial.transform import Rotation
    v = np.asarray(verts, dtype=np.float64)
    mu = v.mean(0)
    _, _, wt = np.linalg.svd(v - mu, full_matrices=False)
    cands = [wt.T]
    cands += list(Rotation.random(n_random, random_state=seed).as_matrix())
    best, best_R = np.inf, None
    for R in cands:
        p = v @ R
        vol = np.prod(p.max(0) - p.min(0))
        if vol < best:
            best, best_R = vol, R
    R = best_R
    u, _, w2 = np.linalg.svd(R)
    R = u @ w2
    if np.linalg.det(R) < 0:
        R[:, 2] = -R[:, 2]
    p = v @ R
    lo, hi = p.min(0), p.max(0)
    half = (hi - lo) / 2 + 1e-9
    c = R @ ((hi + lo) / 2)
    # inner box: largest scaled copy of the outer box (same centre and axes) inside the hull
    n, d = planes[:, :3], planes[:, 3]
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    ih = np.zeros(3)
    if np.all(c @ n.T <= d - 1e-7):
        lo_s, hi_s = 0.0, 1.0
        for _ in range(60):
            s = 0.5 * (lo_s + hi_s)
            pts = c + (corners * (half * s)) @ R.T
            if np.all(pts @ n.T <= d[None, :] - 1e-7):
                lo_s = s
            else:
                hi_s = s
        ih = half * lo_s * (1 - 1e-6)
    return c, R, half, ih


class ConvexMesh:
    """A fixed convex-mesh obstacle: vertices in the mesh frame, a scale, and a world pose
    (rotation R, translation p).  Bullet collides the hull of the vertices; so does the
    engine."""

    def __init__(self, vertices, rotation=None, position=(0.0, 0.0, 0.0), scale=1.0,
                 name="mesh"):
        self.vertices = np.asarray(vertices, dtype=np.float64).reshape(-1, 3)
        self.rotation = np.eye(3) if rotation is None else np.asarray(rotation, dtype=np.float64).reshape(3, 3)
        self.position = np.asarray(position, dtype=np.float64).reshape(3)
        self.scale = float(scale)
        self.name = name
        self._rec = None
        self._sph = None

    def world_vertices(self):
        return (self.vertices * self.scale) @ self.rotation.T + self.position

    def record(self):
        """(verts, planes, edges, box18, inner LOD, outer LOD) in the world frame; cached.
        The LODs are (verts, planes, edges) hulls inside / around the hull."""
        if self._rec is None:
            v, pl, e = hull_data(self.world_vertices())
            c, R, half, ih = fit_boxes(v, pl)
            box = np.concatenate([c, R.reshape(-1), half, ih])
            inner = inner_lod(v, INNER_LOD_K)
            outer = outer_lod(v, inner_lod(v, OUTER_LOD_K)[1])
            self._rec = (v, pl, e, box, inner, outer)
        return self._rec

    def spheres(self):
        """[spheres.N_SPHERES, 4] balls inside the hull (world frame); cached.  The kernels'
        lane-parallel certificate ahead of the exact test (tcmp_set_mesh_spheres)."""
        if self._sph is None:
            from .spheres import inscribed_spheres
            self._sph = inscribed_spheres(self.record()[0])
        return self._sph

    def __repr__(self):
        return "ConvexMesh(%s, %d verts, scale %.3g)" % (self.name, len(self.vertices), self.scale)


class HullSet:
    """Concatenated (verts, planes, edges) hulls with row offsets (struct tcmp_hulls)."""

    def __init__(self, hulls):
        self.verts = np.ascontiguousarray(np.concatenate([h[0] for h in hulls]) if hulls else np.zeros((0, 3)))
        self.planes = np.ascontiguousarray(np.concatenate([h[1] for h in hulls]) if hulls else np.zeros((0, 4)))
        self.edges = np.ascontiguousarray((np.concatenate([h[2] for h in hulls]) if hulls
                                           else np.zeros((0, 4))).astype(np.int32))
        self.vert_off = np.concatenate([[0], np.cumsum([len(h[0]) for h in hulls])]).astype(np.int32)
        self.plane_off = np.concatenate([[0], np.cumsum([len(h[1]) for h in hulls])]).astype(np.int32)
        self.edge_off = np.concatenate([[0], np.cumsum([len(h[2]) for h in hulls])]).astype(np.int32)

    def arrays(self):
        return (self.verts, self.vert_off, self.planes, self.plane_off, self.edges, self.edge_off)


class MeshPack(HullSet):
    """Flat arrays of tcmp_set_meshes (include/tcmp.h): the exact hulls, their boxes and the
    inner / outer level-of-detail hulls (tcmp_set_mesh_lods)."""

    def __init__(self, meshes):
        recs = [m.record() for m in meshes]
        HullSet.__init__(self, [r[:3] for r in recs])
        self.n = len(recs)
        self.boxes = np.ascontiguousarray(np.array([r[3] for r in recs]).reshape(-1, 18))
        self.inner = HullSet([r[4] for r in recs])
        self.outer = HullSet([r[5] for r in recs])
        from .spheres import N_SPHERES
        self.spheres = np.ascontiguousarray(
            np.array([m.spheres() for m in meshes]).reshape(-1, N_SPHERES, 4))

    def key(self):
        return b"".join(a.tobytes() for a in self.arrays() + (self.boxes,) + self.inner.arrays()
                        + self.outer.arrays())

    def __len__(self):
        return self.n


def pack_meshes(meshes):
    if isinstance(meshes, MeshPack):
        return meshes
    return MeshPack(list(meshes or []))


def library_shapes():
    """The Panda's collision hulls (panda_mod.urdf STL meshes, link frames), the shape
    library SURVEY 8d names for the dense-clutter config (C5): name -> vertices."""
    import os
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "panda_geometry.npz"))
    off, names = d["vert_off"], [str(s) for s in d["link_names"]]
    shapes = {}
    for i, nm in enumerate(names):
        if nm == "panda_rightfinger":
            continue  # the left finger's mesh, turned about z
        shapes[nm.replace("panda_", "")] = d["verts"][off[i]:off[i + 1]].copy()
    return shapes
