"""Scene records that replace the reference's pybullet body handles.

The reference passes pybullet body ids around (`Problem.robot`, `Problem.fixed`,
`Problem.payload`, utils.py:86-93) and asks Bullet for link poses and closest points.  The
engine needs only geometry, so bodies become plain records:

  PandaRobot  -- the Panda of src/models/panda_mod.urdf (joint limits, efforts, fingers open)
  Box         -- a fixed oriented box obstacle (URDF <box> collision, e.g. table_wooden.urdf)
  Payload     -- the grasped object (mass for the torque tests, cylinder/box for grasps)
  ConvexMesh  -- a fixed convex-mesh obstacle (URDF <mesh>; Bullet collides its hull), hull.py

`obstacle_array()` packs boxes into the C-ABI layout (15 doubles per box); `mesh_pack()`
packs the convex meshes (tcmp_set_meshes).
"""
import numpy as np

from .hull import ConvexMesh, MeshPack, library_shapes, pack_meshes

# panda_mod.urdf:121-285
JOINT_LOWER = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
JOINT_UPPER = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
JOINT_EFFORT = np.array([87.0, 87.0, 87.0, 87.0, 12.0, 12.0, 12.0])
JOINT_VELOCITY = np.array([2.175, 2.175, 2.175, 2.175, 2.61, 2.61, 2.61])
ARM_JOINT_NAMES = ['panda_joint1', 'panda_joint2', 'panda_joint3', 'panda_joint4',
                   'panda_joint5', 'panda_joint6', 'panda_joint7']  # utils.py:29-30
COLLISION_LINK_NAMES = ['panda_link1', 'panda_link2', 'panda_link3', 'panda_link4',
                        'panda_link5', 'panda_link6', 'panda_link7', 'panda_hand',
                        'panda_leftfinger', 'panda_rightfinger']


class PandaRobot:
    """The planning robot (replaces the pybullet body id of panda_mod.urdf).

    Base frame = world frame; fingers held open at 0.04 (open_arm, panda_primitives.py:320).
    """
    name = "panda"

    def __init__(self):
        self.joints = list(range(7))
        self.lower = JOINT_LOWER.copy()
        self.upper = JOINT_UPPER.copy()
        self.effort = JOINT_EFFORT.copy()
        self.velocity = JOINT_VELOCITY.copy()
        self.conf = None

    def __repr__(self):
        return "PandaRobot()"


def rotation_rpy(roll=0.0, pitch=0.0, yaw=0.0):
    cr, sr = np.cos(roll), np.sin(roll)
    cp, sp = np.cos(pitch), np.sin(pitch)
    cy, sy = np.cos(yaw), np.sin(yaw)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


class Box:
    """Fixed oriented box obstacle: centre, full size (URDF <box size>), rotation."""

    def __init__(self, center, size=None, half_extents=None, rotation=None, name="box"):
        self.center = np.asarray(center, dtype=np.float64).reshape(3)
        if half_extents is None:
            half_extents = np.asarray(size, dtype=np.float64).reshape(3) / 2.0
        self.half_extents = np.asarray(half_extents, dtype=np.float64).reshape(3)
        self.rotation = np.eye(3) if rotation is None else np.asarray(rotation, dtype=np.float64).reshape(3, 3)
        self.name = name

    def obb15(self):
        return np.concatenate([self.center, self.rotation.reshape(-1), self.half_extents])

    def __repr__(self):
        return "Box(%s, half=%s)" % (np.round(self.center, 4).tolist(), np.round(self.half_extents, 4).tolist())


class Payload:
    """Grasped object: mass (get_mass) and a cylinder/box shape for top grasps."""

    def __init__(self, mass, radius=0.015, height=0.05, pose=None, name="payload",
                 center=(0.0, 0.0, 0.0), size=None):
        self.mass = float(mass)
        self.radius = float(radius)
        self.height = float(height)
        self.pose = pose
        self.name = name
        # AABB of the collision shape in the body frame (approximate_as_prism, utils.py:2762):
        # centre and full extents (w, l, h).  A cylinder's extents are (2r, 2r, h)
        # (vertices_from_data, utils.py:2690-2695); a box passes size=(w, l, h).
        self.center = np.asarray(center, dtype=np.float64).reshape(3)
        if size is None:
            size = (2 * self.radius, 2 * self.radius, self.height)
        self.size = np.asarray(size, dtype=np.float64).reshape(3)

    @classmethod
    def coke(cls, mass):
        """src/models/coke.urdf: cylinder r=0.015, length 0.05 at the link origin, inertial
        origin z=-0.023.  pybullet reports base poses and collision frames relative to the
        inertial frame, so the shape centre sits at +0.023 in the pose frame."""
        return cls(mass, radius=0.015, height=0.05, name="coke", center=(0.0, 0.0, 0.023))


def get_mass(body):
    """utils.get_mass replacement (pybullet getDynamicsInfo mass)."""
    return float(getattr(body, "mass", 0.0))


def obstacle_array(fixed):
    """Pack the boxes of Problem.fixed into the (n, 15) C-ABI layout (convex meshes are
    packed separately by mesh_pack)."""
    if fixed is None or isinstance(fixed, MeshPack):
        fixed = []
    if isinstance(fixed, np.ndarray):
        if fixed.size == 0:
            return np.zeros((0, 15))
        return np.ascontiguousarray(fixed.astype(np.float64).reshape(-1, 15))
    rows = []
    for b in fixed:
        if isinstance(b, ConvexMesh):
            continue
        if isinstance(b, Box):
            rows.append(b.obb15())
        else:
            a = np.asarray(b, dtype=np.float64).reshape(-1)
            if a.size != 15:
                raise TypeError("obstacles must be Box records or 15-vectors (centre, R, half)")
            rows.append(a)
    if not rows:
        return np.zeros((0, 15))
    return np.ascontiguousarray(np.array(rows, dtype=np.float64))


def random_box_scene(rng, n, avoid=(), collides=None, aligned=True, max_tries=100000):
    """SURVEY 8d synthetic scene: centres U([0.2,0.8]x[-0.6,0.6]x[0,0.8]) m, half extents
    U[0.03,0.12] m, rejected while any configuration in `avoid` collides (collides(q, obs))."""
    boxes = []
    tries = 0
    while len(boxes) < n:
        tries += 1
        if tries > max_tries:
            raise RuntimeError("could not place %d boxes" % n)
        c = rng.uniform([0.2, -0.6, 0.0], [0.8, 0.6, 0.8])
        h = rng.uniform(0.03, 0.12, 3)
        R = np.eye(3)
        if not aligned:
            R = rotation_rpy(*rng.uniform(-np.pi, np.pi, 3))
        b = Box(c, half_extents=h, rotation=R)
        if collides is not None and avoid:
            arr = obstacle_array([b])
            if any(collides(q, arr) for q in avoid):
                continue
        boxes.append(b)
    return boxes


def mesh_pack(fixed):
    """The ConvexMesh records of Problem.fixed as a hull.MeshPack (None when there are none)."""
    if fixed is None or isinstance(fixed, np.ndarray):
        return None
    if isinstance(fixed, MeshPack):
        return fixed
    meshes = [b for b in fixed if isinstance(b, ConvexMesh)]
    return pack_meshes(meshes) if meshes else None


def random_rotation(rng):
    """Uniform random rotation (Shoemake quaternion)."""
    u1, u2, u3 = rng.uniform(0.0, 1.0, 3)
    a, b = np.sqrt(1 - u1), np.sqrt(u1)
    x, y, z, w = a * np.sin(2 * np.pi * u2), a * np.cos(2 * np.pi * u2), b * np.sin(2 * np.pi * u3), b * np.cos(2 * np.pi * u3)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


# C5 clutter region: around the arm's reach (the SURVEY 8d box region, widened to both sides)
MESH_REGION_LO = (-0.8, -0.8, 0.0)
MESH_REGION_HI = (0.8, 0.8, 1.0)


def random_mesh_scene(rng, n, avoid=(), collides=None, scale=(0.5, 1.5), lo=MESH_REGION_LO,
                      hi=MESH_REGION_HI, keep_out=0.12, max_tries=200000):
    """n convex meshes = the Panda's collision hulls (panda_mod.urdf STL
    meshes) scaled U[0.5, 1.5] with uniform random orientations, centres uniform in the
    region [lo, hi] outside a cylinder of radius keep_out around the base, rejected while any
    configuration in `avoid` collides (collides(q, [mesh]) -> bool)."""
    shapes = list(library_shapes().items())
    out = []
    tries = 0
    while len(out) < n:
        tries += 1
        if tries > max_tries:
            raise RuntimeError("could not place %d meshes" % n)
        name, verts = shapes[int(rng.integers(len(shapes)))]
        s = float(rng.uniform(*scale))
        c = rng.uniform(lo, hi)
        if np.hypot(c[0], c[1]) < keep_out:
            continue
        m = ConvexMesh(verts - verts.mean(0), rotation=random_rotation(rng), position=c, scale=s,
                       name=name)
        if collides is not None and avoid:
            if any(collides(q, [m]) for q in avoid):
                continue
        out.append(m)
    return out
