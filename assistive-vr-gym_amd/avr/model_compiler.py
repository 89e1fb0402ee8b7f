"""Offline model compiler: reference assets (URDF / DAE / VHACD-OBJ) + the human link tables
-> one flat, self-contained scene description (`avr/data/<task>.npz`).

It runs only in the build container (it reads `/root/reference`); the compiled `.npz` is what
ships.  Nothing here is on the step path.  What it restates, with reference citations:

* Link numbering is the multibody DFS pre-order of the URDF tree, children in declaration
  order (checked against the hard-coded indices `world_creation.py:283`
  arm [1..7], `world_creation.py:320` fingers [9,11,13], tool link 8 `world_creation.py:334`).
* Inertia is recomputed from the collision compound's AABB because Jaco/spoon/bowl are loaded
  without URDF_USE_INERTIA_FROM_FILE (`world_creation.py:282`, `feeding.py:185`,
  `world_creation.py:343`); the URDF inertial origin is kept.  (Bullet behaviour)
* DAE collision meshes become one convex hull of all vertices; OBJ files with several `o`
  objects become a compound of one hull per object.  URDF shapes get margin 0.001.
* The human is `HumanCreation.create_human` (`human_creation.py:57-301`) with its creation
  order remapped to DFS order (legend `human_creation.py:5-45`).
* Collision filters: Jaco self-collision except parent/child (`world_creation.py:282`),
  spoon vs gripper links 7..14 off (`world_creation.py:359-361`), static-vs-static never.
"""
import copy
import functools
import json
import os
import re
import struct
import xml.etree.ElementTree as ET

import numpy as np

from . import geom as G

REF_ASSETS = '/root/reference/assistive_gym/envs/assets'
DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data')

# Every builder that reads the reference's assets goes through asset_cached: its result is kept
# in data/asset_cache.npz (written by compile_all in the build container), so that scene_arrays
# can rebuild a scene at another human height where the reference's assets are absent (the GPU
# box).  The cache holds the builders' parsed and hulled geometry -- the same numbers the
# committed scene npz files hold, not the asset files -- as JSON (structure) plus arrays, read
# with np.load(allow_pickle=False): nothing in it executes.
ASSET_CACHE = os.path.join(DATA_DIR, 'asset_cache.npz')
_asset_memo = None


def _enc(x, arrs):
    if isinstance(x, np.ndarray):
        arrs.append(x)
        return {'__nd__': len(arrs) - 1}
    if isinstance(x, (Shape, Hull)):
        return {'__%s__' % type(x).__name__: {k: _enc(v, arrs) for k, v in vars(x).items()}}
    if isinstance(x, dict):
        assert all(isinstance(k, str) for k in x)
        return {'__dict__': {k: _enc(v, arrs) for k, v in x.items()}}
    if isinstance(x, tuple):
        return {'__tuple__': [_enc(v, arrs) for v in x]}
    if isinstance(x, list):
        return [_enc(v, arrs) for v in x]
    assert x is None or isinstance(x, (str, bool, int, float)), type(x)
    return x


def _dec(x, arrs):
    if isinstance(x, list):
        return [_dec(v, arrs) for v in x]
    if not isinstance(x, dict):
        return x
    (tag, v), = x.items()
    if tag == '__nd__':
        return arrs['a%d' % v]
    if tag in ('__Shape__', '__Hull__'):
        o = object.__new__(Shape if tag == '__Shape__' else Hull)
        o.__dict__.update({k: _dec(w, arrs) for k, w in v.items()})
        return o
    if tag == '__dict__':
        return {k: _dec(w, arrs) for k, w in v.items()}
    if tag == '__tuple__':
        return tuple(_dec(w, arrs) for w in v)
    raise ValueError('asset cache: unknown tag %r' % tag)


def _memo():
    global _asset_memo
    if _asset_memo is None:
        _asset_memo = {}
        if os.path.exists(ASSET_CACHE):
            with np.load(ASSET_CACHE, allow_pickle=False) as z:
                arrs = {k: z[k] for k in z.files}
            meta = json.loads(bytes(arrs.pop('meta')).decode())
            _asset_memo = {tuple(k): _dec(v, arrs) for k, v in meta}
    return _asset_memo


def asset_cached(fn):
    @functools.wraps(fn)
    def wrapper(*args):
        M = _memo()
        key = (fn.__name__,) + tuple(args)
        if key not in M:
            if not os.path.isdir(REF_ASSETS):
                raise RuntimeError('%s%r: not in %s and the reference assets (%s) are absent; run '
                                   'model_compiler.compile_all in the build container' % (fn.__name__, args, ASSET_CACHE, REF_ASSETS))
            M[key] = fn(*args)
        return copy.deepcopy(M[key])
    return wrapper


def save_asset_cache(path=ASSET_CACHE):
    arrs = []
    meta = [[list(k), _enc(v, arrs)] for k, v in _memo().items()]
    out = {'a%d' % i: a for i, a in enumerate(arrs)}
    out['meta'] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(path, **out)


URDF_MARGIN = 0.001          # gUrdfDefaultCollisionMargin (assumed Bullet default)
CONTACT_BREAKING = 0.02      # gContactBreakingThreshold (assumed Bullet default)

SPHERE, CAPSULE, BOX, HULL = 0, 1, 2, 3
KIND_ROBOT, KIND_FREE, KIND_STATIC, KIND_HUMAN, KIND_RSTATIC = 0, 1, 2, 3, 4
J_FIXED, J_REVOLUTE, J_PRISMATIC = 0, 1, 2


# ----------------------------------------------------------------------------- meshes
def dae_vertices(path):
    s = open(path).read()
    out = []
    for m in re.finditer(r'<float_array id="[^"]*positions-array" count="(\d+)">([^<]*)<', s):
        out.append(np.array(m.group(2).split(), float).reshape(-1, 3))
    return np.concatenate(out, 0)


def stl_vertices(path):
    """Vertices of an STL mesh (binary or ASCII), duplicates removed."""
    data = open(path, 'rb').read()
    n = struct.unpack('<I', data[80:84])[0] if len(data) >= 84 else 0
    if len(data) == 84 + 50 * n:
        rec = np.frombuffer(data, dtype=np.dtype([('n', '<f4', 3), ('v', '<f4', (3, 3)), ('a', '<u2')]), count=n, offset=84)
        v = rec['v'].reshape(-1, 3).astype(float)
    else:
        v = np.array([[float(x) for x in m.groups()] for m in
                      re.finditer(rb'vertex\s+(\S+)\s+(\S+)\s+(\S+)', data)], float)
    return np.unique(v, axis=0)


def cylinder_vertices(radius, length):
    """URDF cylinder as Bullet's URDF importer builds it without URDF_USE_IMPLICIT_CYLINDER: a
    convex hull of two 32-gons at z = +-length/2 (BulletUrdfImporter, [ext] SURVEY A.7)."""
    out = []
    for i in range(32):
        a = 2.0 * np.pi * i / 32.0
        for z in (0.5 * length, -0.5 * length):
            out.append([radius * np.sin(a), radius * np.cos(a), z])
    return np.array(out)


def obj_groups(path):
    groups, cur = [], None
    for line in open(path):
        if line.startswith('o ') or line.startswith('g '):
            cur = []
            groups.append(cur)
        elif line.startswith('v '):
            if cur is None:
                cur = []
                groups.append(cur)
            cur.append([float(x) for x in line.split()[1:4]])
    return [np.array(g, float) for g in groups if len(g) >= 4]


class Hull:
    """Convex hull of a point set: hull vertices + merged face planes n.x <= d (core, no margin)."""

    def __init__(self, pts):
        from scipy.spatial import ConvexHull     # (build container only: cached hulls need no scipy)
        pts = np.asarray(pts, float)
        h = ConvexHull(pts)
        self.verts = pts[h.vertices]
        planes = []
        for eq in h.equations:
            n, d = eq[:3], -eq[3]
            dup = False
            for p in planes:
                if np.dot(p[:3], n) > 1.0 - 1e-9 and abs(p[3] - d) < 1e-9:
                    dup = True
                    break
            if not dup:
                planes.append(np.array([n[0], n[1], n[2], d]))
        self.planes = np.array(planes)


# ----------------------------------------------------------------------------- shapes
class Shape:
    def __init__(self, kind, pos=(0, 0, 0), quat=(0, 0, 0, 1), radius=0.0, half_height=0.0,
                 half_extents=(0, 0, 0), hull=None, margin=URDF_MARGIN, gender=-1):
        self.kind = kind
        self.pos = np.asarray(pos, float)
        self.quat = np.asarray(quat, float)
        self.radius = float(radius)
        self.half_height = float(half_height)
        self.half_extents = np.asarray(half_extents, float)
        self.hull = hull
        self.margin = float(margin) if kind in (BOX, HULL) else float(radius)
        self.gender = gender

    def local_aabb(self):
        """(center, half) of the shape's AABB in its OWN frame, Bullet getAabb semantics."""
        if self.kind == SPHERE:
            return np.zeros(3), np.full(3, self.radius)
        if self.kind == CAPSULE:
            return np.zeros(3), np.array([self.radius, self.radius, self.radius + self.half_height])
        if self.kind == BOX:
            return np.zeros(3), self.half_extents.copy()
        v = self.hull.verts
        lo, hi = v.min(0) - self.margin, v.max(0) + self.margin
        # btTransformAabb adds the margin again on top of the cached local AABB (Bullet quirk)
        return 0.5 * (lo + hi), 0.5 * (hi - lo) + self.margin

    def aabb_in(self, pos, quat):
        """AABB of this shape (placed at self.pos/self.quat in a parent frame) expressed in
        the frame (pos, quat) * parent."""
        c, h = self.local_aabb()
        p, q = G.tf_mul(pos, quat, self.pos, self.quat)
        R = G.quat_to_mat(q)
        cw = p + R @ c
        hw = np.abs(R) @ h
        return cw - hw, cw + hw


def compound_aabb(shapes):
    lo = np.full(3, np.inf)
    hi = np.full(3, -np.inf)
    for s in shapes:
        a, b = s.aabb_in(np.zeros(3), np.array([0, 0, 0, 1.0]))
        lo, hi = np.minimum(lo, a), np.maximum(hi, b)
    return lo, hi


def box_inertia(mass, lo, hi):
    lx, ly, lz = hi - lo
    return mass / 12.0 * np.array([ly * ly + lz * lz, lx * lx + lz * lz, lx * lx + ly * ly])


def breaking_threshold(shapes):
    """btCollisionShape::getContactBreakingThreshold = angular-motion disc * 0.02, disc from the
    root shape's bounding sphere (CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD)."""
    lo, hi = compound_aabb(shapes)
    c = 0.5 * (lo + hi)
    r = 0.5 * np.linalg.norm(hi - lo)
    return CONTACT_BREAKING * (r + np.linalg.norm(c))


# ----------------------------------------------------------------------------- URDF
def _origin(el):
    if el is None:
        return np.zeros(3), np.array([0, 0, 0, 1.0])
    xyz = np.array([float(x) for x in el.get('xyz', '0 0 0').split()])
    rpy = [float(x) for x in el.get('rpy', '0 0 0').split()]
    return xyz, G.quat_from_euler(rpy)


class Link:
    pass


def parse_urdf(path):
    root = ET.parse(path).getroot()
    base_dir = os.path.dirname(path)
    links = {}
    order = []
    for le in root.findall('link'):
        L = Link()
        L.name = le.get('name')
        ine = le.find('inertial')
        L.tensor = np.zeros((3, 3))
        if ine is not None:
            L.mass = float(ine.find('mass').get('value'))
            L.com_pos, L.com_quat = _origin(ine.find('origin'))
            it = ine.find('inertia')
            if it is not None:
                g = lambda k: float(it.get(k, 0.0))
                L.tensor = np.array([[g('ixx'), g('ixy'), g('ixz')], [g('ixy'), g('iyy'), g('iyz')], [g('ixz'), g('iyz'), g('izz')]])
        else:
            L.mass = 0.0
            L.com_pos, L.com_quat = np.zeros(3), np.array([0, 0, 0, 1.0])
        L.collisions = []
        for ce in le.findall('collision'):
            pos, quat = _origin(ce.find('origin'))
            ge = ce.find('geometry')
            me, be, se, ce = ge.find('mesh'), ge.find('box'), ge.find('sphere'), ge.find('cylinder')
            if ce is not None:
                L.collisions.append(('cylinder', float(ce.get('radius')), float(ce.get('length')), pos, quat))
            elif me is not None:
                scale = np.array([float(x) for x in me.get('scale', '1 1 1').split()])
                L.collisions.append(('mesh', os.path.join(base_dir, me.get('filename')), scale, pos, quat))
            elif be is not None:
                size = np.array([float(x) for x in be.get('size').split()])
                L.collisions.append(('box', size, None, pos, quat))
            elif se is not None:
                L.collisions.append(('sphere', float(se.get('radius')), None, pos, quat))
        friction = 0.5
        ct = le.find('contact')
        if ct is not None and ct.find('lateral_friction') is not None:
            friction = float(ct.find('lateral_friction').get('value'))
        L.friction = friction
        # <contact> rolling / spinning friction (PyBullet's URDF importer; default 0)
        L.rolling = float(ct.find('rolling_friction').get('value')) if ct is not None and ct.find('rolling_friction') is not None else 0.0
        L.spinning = float(ct.find('spinning_friction').get('value')) if ct is not None and ct.find('spinning_friction') is not None else 0.0
        links[L.name] = L
        order.append(L.name)
    joints = []
    for je in root.findall('joint'):
        J = dict(name=je.get('name'), type=je.get('type'), parent=je.find('parent').get('link'),
                 child=je.find('child').get('link'))
        J['pos'], J['quat'] = _origin(je.find('origin'))
        ax = je.find('axis')
        J['axis'] = np.array([float(x) for x in ax.get('xyz').split()]) if ax is not None else np.zeros(3)
        lim = je.find('limit')
        J['lower'] = float(lim.get('lower', 0)) if lim is not None else 0.0
        J['upper'] = float(lim.get('upper', -1)) if lim is not None else -1.0
        joints.append(J)
    children = {}
    child_set = set()
    for J in joints:
        children.setdefault(J['parent'], []).append(J)
        child_set.add(J['child'])
    root_name = [n for n in order if n not in child_set][0]
    # DFS pre-order over joints, children in declaration order
    dfs = []

    def visit(name, parent_idx):
        for J in children.get(name, []):
            idx = len(dfs)
            dfs.append((J, parent_idx))
            visit(J['child'], idx)
    visit(root_name, -1)
    return links, root_name, dfs


def urdf_shapes(L, scale_override=None):
    """Collision shapes of a URDF link, placed relative to the link's INERTIAL frame."""
    inv_p, inv_q = G.tf_inv(L.com_pos, L.com_quat)
    shapes = []
    for kind, a, b, pos, quat in L.collisions:
        p, q = G.tf_mul(inv_p, inv_q, pos, quat)
        if kind == 'mesh':
            path, scale = a, b
            if path.endswith('.dae'):
                shapes.append(Shape(HULL, p, q, hull=Hull(dae_vertices(path) * scale)))
            elif path.lower().endswith('.stl'):
                shapes.append(Shape(HULL, p, q, hull=Hull(stl_vertices(path) * scale)))
            else:
                for g in obj_groups(path):
                    shapes.append(Shape(HULL, p, q, hull=Hull(g * scale)))
        elif kind == 'box':
            shapes.append(Shape(BOX, p, q, half_extents=0.5 * a))
        elif kind == 'sphere':
            shapes.append(Shape(SPHERE, p, q, radius=a))
        elif kind == 'cylinder':
            shapes.append(Shape(HULL, p, q, hull=Hull(cylinder_vertices(a, b))))
    return shapes


# ----------------------------------------------------------------------------- human
def _capsule(radius, length, pos=(0, 0, 0), orient=(0, 0, 0, 1)):
    return Shape(CAPSULE, pos, orient, radius=radius, half_height=0.5 * length)


def _sphere(radius, pos=(0, 0, 0)):
    return Shape(SPHERE, pos, (0, 0, 0, 1), radius=radius)


DEFAULT_HEIGHT = {'male': 0.6, 'female': 0.54}          # feeding.py:174, scratch_itch.py:161, bed_bathing.py:187


def human_heights(heights=None):
    """Per-gender hipbone_to_mouth_height of a compiled scene: None (both defaults) or a dict
    {gender: height}; a missing gender keeps its default."""
    h = dict(DEFAULT_HEIGHT)
    for g, v in (heights or {}).items():
        if g not in h:
            raise ValueError('heights: gender must be male or female, got %r' % (g,))
        if v is not None:
            v = float(v)
            if not 0.3 <= v <= 1.0:
                raise ValueError('hipbone_to_mouth_height %.4f outside [0.3, 1.0] m' % v)
            h[g] = v
    return h


def default_heights(heights):
    return human_heights(heights) == DEFAULT_HEIGHT


@asset_cached
def head_hulls(head_file):
    """The head's VHACD parts at meshScale 0.89 (human_creation.py:98-99,141-142)."""
    return [Hull(g * 0.89) for g in obj_groups(os.path.join(REF_ASSETS, 'head_female_male', head_file))]


@asset_cached
def bed_frame_hulls():
    """The hospital bed frame's VHACD parts at meshScale [1, 1.2, 1] (bed_bathing.py:214-216)."""
    return [Hull(g * np.array([1, 1.2, 1])) for g in obj_groups(os.path.join(REF_ASSETS, 'bed', 'hospital_bed_frame_vhacd.obj'))]


def build_human(gender, hipbone_to_mouth_height=None, limit_scale=1.0):
    """Restatement of HumanCreation.create_human (human_creation.py:57-301), non-`new`,
    non-cloth.  Returns (base_shapes, links[DFS]); each link dict carries parent (DFS index or
    -1 for base), joint type, axis, origin (relative to parent COM frame), limits, mass,
    shapes (relative to the link frame == its COM frame, inertial offsets are zero)."""
    mass = {'male': 78.4, 'female': 62.5}[gender]               # config.ini:46-53
    rs, hs = 1.0, 1.0
    if hipbone_to_mouth_height is None:
        hipbone_to_mouth_height = 0.6 if gender == 'male' else 0.54  # feeding.py:174
    hs *= hipbone_to_mouth_height / (0.6 if gender == 'male' else 0.54)   # :60-63,75
    q_y90 = G.quat_from_euler([0, np.pi / 2, 0])
    q_x90 = G.quat_from_euler([np.pi / 2, 0, 0])
    head_orient = G.quat_from_euler([np.pi / 2.0, 0, 0])
    if gender == 'male':                                          # human_creation.py:76-115
        chest = _capsule(0.127 * rs, 0.056, orient=q_y90)
        r_sh = _capsule(0.106 * rs, 0.253 / 8, pos=[-0.253 / 2.5 + 0.253 / 16, 0, 0], orient=q_y90)
        l_sh = _capsule(0.106 * rs, 0.253 / 8, pos=[0.253 / 2.5 - 0.253 / 16, 0, 0], orient=q_y90)
        neck = _capsule(0.06 * rs, 0.124 * hs, pos=[0, 0, (0.2565 - 0.1415 - 0.025) * hs])
        upperarm = lambda: _capsule(0.043 * rs, 0.279 * hs, pos=[0, 0, -0.279 / 2.0 * hs])
        forearm = lambda: _capsule(0.033 * rs, 0.257 * hs, pos=[0, 0, -0.257 / 2.0 * hs])
        hand = lambda: _sphere(0.043 * rs, pos=[0, 0, -0.043 * rs])
        waist = _capsule(0.1205 * rs, 0.049, orient=q_y90)
        hips = _capsule(0.1335 * rs, 0.094, pos=[0, 0, -0.08125 * hs], orient=q_y90)
        thigh = lambda: _capsule(0.08 * rs, 0.424 * hs, pos=[0, 0, -0.424 / 2.0 * hs])
        shin = lambda: _capsule(0.05 * rs, 0.403 * hs, pos=[0, 0, -0.403 / 2.0 * hs])
        foot = lambda: _capsule(0.05 * rs, 0.215 * hs, pos=[0, -0.1, -0.025 * rs], orient=q_x90)
        head_file = 'BaseHeadMeshes_v5_male_cropped_reduced_compressed_vhacd.obj'
        head_pos = [0.09, 0.08, -0.07 + 0.01]
        chest_p = [0, 0, 0.156 * hs]
        shoulders_p = [0, 0, 0.1415 / 2 * hs]
        neck_p = [0, 0, 0.1515 * hs]
        head_p = [0, 0, (0.399 - 0.1415 - 0.1205) * hs]
        right_upperarm_p = [-0.106 * rs - 0.073, 0, 0]
        left_upperarm_p = [0.106 * rs + 0.073, 0, 0]
        forearm_p = [0, 0, -0.279 * hs]
        hand_p = [0, 0, -(0.033 * rs + 0.257 * hs)]
        waist_p = [0, 0, 0.08125 * hs]
        right_thigh_p = [-0.08 * rs - 0.009, 0, -0.08125 * hs]
        left_thigh_p = [0.08 * rs + 0.009, 0, -0.08125 * hs]
        shin_p = [0, 0, -0.424 * hs]
        foot_p = [0, 0, -0.403 * hs - 0.025]
    else:                                                         # human_creation.py:117-161
        chest = _capsule(0.127 * rs, 0.01, orient=q_y90)
        r_sh = _capsule(0.092 * rs, 0.225 / 8, pos=[-0.225 / 2.5 + 0.225 / 16, 0, 0], orient=q_y90)
        l_sh = _capsule(0.092 * rs, 0.225 / 8, pos=[0.225 / 2.5 - 0.225 / 16, 0, 0], orient=q_y90)
        neck = _capsule(0.05 * rs, 0.121 * hs, pos=[0, 0, (0.2565 - 0.1415 - 0.025) * hs])
        upperarm = lambda: _capsule(0.0355 * rs, 0.264 * hs, pos=[0, 0, -0.264 / 2.0 * hs])
        forearm = lambda: _capsule(0.027 * rs, 0.234 * hs, pos=[0, 0, -0.234 / 2.0 * hs])
        hand = lambda: _sphere(0.0355 * rs, pos=[0, 0, -0.0355 * rs])
        waist = _capsule(0.11 * rs, 0.009, orient=q_y90)
        hips = _capsule(0.127 * rs, 0.117, pos=[0, 0, -0.15 / 2 * hs], orient=q_y90)
        thigh = lambda: _capsule(0.0775 * rs, 0.391 * hs, pos=[0, 0, -0.391 / 2.0 * hs])
        shin = lambda: _capsule(0.045 * rs, 0.367 * hs, pos=[0, 0, -0.367 / 2.0 * hs])
        foot = lambda: _capsule(0.045 * rs, 0.195 * hs, pos=[0, -0.09, -0.0225 * rs], orient=q_x90)
        head_file = 'BaseHeadMeshes_v5_female_cropped_reduced_compressed_vhacd.obj'
        head_pos = [-0.089, -0.09, -0.07]
        chest_p = [0, 0, 0.15 * hs]
        shoulders_p = [0, 0, 0.132 / 2 * hs]
        neck_p = [0, 0, 0.132 * hs]
        head_p = [0, 0, 0.12 * hs]
        right_upperarm_p = [-0.092 * rs - 0.067, 0, 0]
        left_upperarm_p = [0.092 * rs + 0.067, 0, 0]
        forearm_p = [0, 0, -0.264 * hs]
        hand_p = [0, 0, -(0.027 * rs + 0.234 * hs)]
        waist_p = [0, 0, 0.15 / 2 * hs]
        right_thigh_p = [-0.0775 * rs - 0.0145, 0, -0.15 / 2 * hs]
        left_thigh_p = [0.0775 * rs + 0.0145, 0, -0.15 / 2 * hs]
        shin_p = [0, 0, -0.391 * hs]
        foot_p = [0, 0, -0.367 * hs - 0.045 / 2]
    gidx = 0 if gender == 'male' else 1
    head_shapes = [Shape(HULL, head_pos, head_orient, hull=h, gender=gidx) for h in head_hulls(head_file)]
    jp = [0, 0, 0]
    d = np.deg2rad
    R, F = J_REVOLUTE, J_FIXED
    # creation-order tables (human_creation.py:177-274); parent indices are 1-based (0 = base)
    C = []   # (mass_frac, shapes, pos, parent1, jtype, axis, lo, hi)
    C += [(0, [], waist_p, 0, F, [0, 0, 0], 0, 0), (0, [], jp, 1, F, [0, 0, 0], 0, 0),
          (0.13, [waist], jp, 2, F, [0, 0, 0], 0, 0), (0.1, [chest], chest_p, 3, F, [0, 0, 0], 0, 0)]
    ls = limit_scale
    C += [(0, [], shoulders_p, 4, F, [0, 0, 0], 0, 0), (0, [], shoulders_p, 5, F, [0, 0, 0], 0, 0),
          (0.05, [r_sh], jp, 6, F, [0, 0, 0], 0, 0), (0, [], shoulders_p, 4, F, [0, 0, 0], 0, 0),
          (0, [], shoulders_p, 8, F, [0, 0, 0], 0, 0), (0.05, [l_sh], jp, 9, F, [0, 0, 0], 0, 0),
          (0.01, [neck], neck_p, 4, R, [1, 0, 0], d(-10) * ls, d(20) * ls),
          (0, [], head_p, 11, R, [1, 0, 0], d(-50) * ls, d(50) * ls),
          (0, [], jp, 12, R, [0, 1, 0], d(-34) * ls, d(34) * ls),
          (0.07, head_shapes, jp, 13, R, [0, 0, 1], d(-70) * ls, d(70) * ls)]
    arm_axes = [[0, 1, 0], [1, 0, 0], [0, 0, 1], [1, 0, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0]]
    ra_lo = [5, -188, -90, -128, -90, -81, -27]
    ra_hi = [198, 61, 90, 0, 90, 90, 47]
    la_lo = [-198, -188, -90, -128, -90, -81, -47]
    la_hi = [-5, 61, 90, 0, 90, 90, 27]
    arm_mass = [0, 0, 0.033, 0, 0.019, 0, 0.0065]
    for side, up_p, par0, lo, hi in (('r', right_upperarm_p, 7, ra_lo, ra_hi), ('l', left_upperarm_p, 10, la_lo, la_hi)):
        shp = [[], [], [upperarm()], [], [forearm()], [], [hand()]]
        pos = [up_p, jp, jp, forearm_p, jp, hand_p, jp]
        base = len(C)
        for k in range(7):
            C.append((arm_mass[k], shp[k], pos[k], par0 if k == 0 else base + k, R, arm_axes[k],
                      d(lo[k]) * ls, d(hi[k]) * ls))
    leg_axes = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]]
    rl_lo, rl_hi = [-127, -40, -45, 0, -35, -23, -43], [30, 45, 40, 130, 38, 24, 35]
    ll_lo, ll_hi = [-127, -45, -40, 0, -35, -24, -35], [30, 40, 45, 130, 38, 23, 43]
    leg_mass = [0, 0, 0.105, 0.0475, 0, 0, 0.014]
    for th_p, lo, hi in ((right_thigh_p, rl_lo, rl_hi), (left_thigh_p, ll_lo, ll_hi)):
        shp = [[], [], [thigh()], [shin()], [], [], [foot()]]
        pos = [th_p, jp, jp, shin_p, foot_p, jp, jp]
        base = len(C)
        for k in range(7):
            C.append((leg_mass[k], shp[k], pos[k], 0 if k == 0 else base + k, R, leg_axes[k],
                      d(lo[k]), d(hi[k])))
    assert len(C) == 42
    # DFS remap: children (in creation order) of each creation node; base = -1
    kids = {}
    for i, c in enumerate(C):
        kids.setdefault(c[3] - 1, []).append(i)
    dfs_of = {}
    order = []

    def visit(node):
        for ch in kids.get(node, []):
            dfs_of[ch] = len(order)
            order.append(ch)
            visit(ch)
    visit(-1)
    links = []
    for ci in order:
        mf, shp, pos, par1, jt, ax, lo, hi = C[ci]
        links.append(dict(parent=-1 if par1 == 0 else dfs_of[par1 - 1], jtype=jt, axis=np.array(ax, float),
                          pos=np.array(pos, float), lower=lo, upper=hi, mass=mass * mf, shapes=shp))
    return [hips], links


HEAD_CHAIN = (24, 25, 26, 27)    # human joints driven under 'tremor' (feeding.py:219, env.py:307-337)
ARM_CHAIN = (7, 8, 9, 10, 11, 12, 13)   # ScratchItch: the right arm's revolute joints (controllable 4..13, scratch_itch.py:191; 4..6 are fixed)
HC_CAP = 8                        # avr_model_desc hc_* capacity (AVR_DESC_HC)


def head_chain(S, joints=HEAD_CHAIN, cap=HC_CAP):
    """Arrays of an articulated human chain (include/avr_model.h hc_*): joint origins, axes,
    masses and inertias per gender (human_creation.py:163-274; inertia from the collision
    shapes' compound AABB as for every other link), limits at limit_scale 1, and the human slot /
    collision body of each link.  Feeding's tremor head/neck chain is joints 24..27
    (human_creation.py:195-207); ScratchItch's is the right arm, joints 7..13
    (human_creation.py:214-226).  The arrays are padded to `cap` links."""
    n = len(joints)
    out = dict(hc_jpos=np.zeros((2, cap, 3)), hc_axis=np.zeros((cap, 3)), hc_mass=np.zeros((2, cap)),
               hc_inertia=np.zeros((2, cap, 3)), hc_lower=np.zeros(cap), hc_upper=np.zeros(cap),
               hc_slot=np.full(cap, -1, np.int32), hc_body=np.full(cap, -1, np.int32), hc_n=np.int32(n),
               hc_joint=np.full(cap, -1, np.int32))
    for g, gender in enumerate(('male', 'female')):
        hl = S.human[gender][1]
        for k, li in enumerate(joints):
            L = hl[li]
            assert L['jtype'] == J_REVOLUTE and L['parent'] == (hl[joints[0]]['parent'] if k == 0 else li - 1)
            out['hc_jpos'][g, k] = L['pos']
            out['hc_mass'][g, k] = L['mass']
            if L['shapes'] and L['mass'] > 0:
                lo, hi = compound_aabb(L['shapes'])
                out['hc_inertia'][g, k] = box_inertia(L['mass'], lo, hi)
            out['hc_axis'][k] = L['axis']
            out['hc_lower'][k], out['hc_upper'][k] = L['lower'], L['upper']
            out['hc_joint'][k] = li
    out['hc_parent_slot'] = np.int32(S.human_slots.index(S.human['male'][1][joints[0]]['parent']))
    for k, li in enumerate(joints):
        if li in S.human_slots:
            out['hc_slot'][k] = S.human_slots.index(li)
            out['hc_body'][k] = S.human_body[li]
    return out


def human_fk(links, base_pos, base_quat, q):
    """World poses of the human link frames (== COM frames) for joint angles q[42]."""
    n = len(links)
    P = np.zeros((n, 3))
    Q = np.zeros((n, 4))
    for i, L in enumerate(links):
        if L['parent'] < 0:
            pp, pq = np.asarray(base_pos, float), np.asarray(base_quat, float)
        else:
            pp, pq = P[L['parent']], Q[L['parent']]
        p, qq = G.tf_mul(pp, pq, L['pos'], [0, 0, 0, 1])
        if L['jtype'] == J_REVOLUTE:
            qq = G.quat_mul(qq, G.quat_axis_angle(L['axis'], q[i]))
        P[i], Q[i] = p, qq
    return P, Q


# ----------------------------------------------------------------------------- scene
class Scene:
    """Flat scene description consumed by the C-ABI (see include/avr_model.h)."""

    def __init__(self):
        self.bodies = []     # dicts: kind, index, shapes(list[Shape]), friction, name
        self.robot = None
        self.free = []
        self.static = []
        self.pairs = []
        self.task = {}

    def add_body(self, kind, index, shapes, friction, name, single=False, rolling=0.0, spinning=0.0):
        # single=True: a bare (non-compound) collision shape (createMultiBody without a frame
        # offset) -- Bullet runs convex-convex on it directly, no child AABB culling.
        # rolling / spinning: the body's rolling and spinning friction (URDF <contact>,
        # p.changeDynamics); a contact's torsional rows use the combined coefficients
        self.bodies.append(dict(kind=kind, index=index, shapes=shapes, friction=friction, name=name, single=single,
                                rolling=rolling, spinning=spinning))
        return len(self.bodies) - 1


@asset_cached
def build_jaco():
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, 'jaco', 'j2s7s300_gym.urdf'))
    rob = dict(name=[], parent=[], jtype=[], dof=[], jpos=[], jquat=[], axis=[], com_pos=[], com_quat=[],
               mass=[], inertia=[], lower=[], upper=[], has_limit=[], shapes=[], friction=[])
    ndof = 0
    for J, parent in dfs:
        L = links[J['child']]
        t = {'fixed': J_FIXED, 'revolute': J_REVOLUTE, 'continuous': J_REVOLUTE, 'prismatic': J_PRISMATIC}[J['type']]
        rob['name'].append(L.name)
        rob['parent'].append(parent)
        rob['jtype'].append(t)
        rob['dof'].append(ndof if t != J_FIXED else -1)
        if t != J_FIXED:
            ndof += 1
        rob['jpos'].append(J['pos'])
        rob['jquat'].append(J['quat'])
        rob['axis'].append(J['axis'] / max(np.linalg.norm(J['axis']), 1e-12) if t != J_FIXED else np.zeros(3))
        rob['com_pos'].append(L.com_pos)
        rob['com_quat'].append(L.com_quat)
        rob['mass'].append(L.mass)
        shapes = urdf_shapes(L)
        rob['shapes'].append(shapes)
        if shapes and L.mass > 0:
            lo, hi = compound_aabb(shapes)
            rob['inertia'].append(box_inertia(L.mass, lo, hi))
        else:
            rob['inertia'].append(np.zeros(3))
        # continuous joints are reported as (0,-1) = no limit (world_creation.py:122-124)
        lim = t == J_REVOLUTE and J['type'] == 'revolute' and J['lower'] <= J['upper']
        rob['lower'].append(J['lower'] if lim else 0.0)
        rob['upper'].append(J['upper'] if lim else -1.0)
        rob['has_limit'].append(1 if lim else 0)
        rob['friction'].append(L.friction)
    rob['ndof'] = ndof
    return rob


@asset_cached
def build_free_urdf(rel):
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, rel))
    assert not dfs
    L = links[root]
    shapes = urdf_shapes(L)
    lo, hi = compound_aabb(shapes)
    return dict(mass=L.mass, inertia=box_inertia(L.mass, lo, hi), shapes=shapes, friction=L.friction)


@asset_cached
def build_static_urdf(rel):
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, rel))
    L = links[root]
    return dict(shapes=urdf_shapes(L), friction=L.friction)


def compile_feeding_jaco(heights=None):
    """FeedingJaco-v0 scene (feeding.py:144-331 + world_creation.py:27-93,274-293,330-365).
    heights: per-gender hipbone_to_mouth_height (human_heights); the human is built at it
    (human_creation.py:60-63,75)."""
    H = human_heights(heights)
    S = Scene()
    rob = build_jaco()
    S.robot = rob
    S.robot_base_pos = np.array([-0.35, -0.3, 0.36])                      # feeding.py:188
    S.robot_base_quat = np.array([0.0, 0.0, -0.7071067811865475, 0.7071067811865476])
    robot_body = {}
    for i in range(len(rob['name'])):
        if rob['shapes'][i]:
            robot_body[i] = S.add_body(KIND_ROBOT, i, rob['shapes'][i], rob['friction'][i], rob['name'][i])
    # free bodies: spoon, bowl, 8 food spheres (feeding.py:280,185,291-308)
    spoon = build_free_urdf('dinnerware/spoon.urdf')
    bowl = build_free_urdf('dinnerware/bowl.urdf')
    food_r, food_m = 0.005, 0.001
    food_shape = [Shape(SPHERE, radius=food_r)]
    S.free = [dict(name='spoon', mass=spoon['mass'], inertia=spoon['inertia'], gravity=np.zeros(3)),
              dict(name='bowl', mass=bowl['mass'], inertia=bowl['inertia'], gravity=np.array([0, 0, -9.81]))]
    for k in range(8):
        S.free.append(dict(name='food%d' % k, mass=food_m, inertia=np.full(3, 0.4 * food_m * food_r * food_r),
                           gravity=np.array([0, 0, -9.81])))
    free_body = [S.add_body(KIND_FREE, 0, spoon['shapes'], spoon['friction'], 'spoon'),
                 S.add_body(KIND_FREE, 1, bowl['shapes'], bowl['friction'], 'bowl')]
    for k in range(8):
        free_body.append(S.add_body(KIND_FREE, 2 + k, food_shape, 0.5, 'food%d' % k, single=True))
    # statics: plane, wheelchair, table (world_creation.py:37,45-49; feeding.py:182)
    plane = build_static_urdf('plane/plane.urdf')
    chair = build_static_urdf('wheelchair/wheelchair.urdf')
    table = build_static_urdf('table/table_tall.urdf')
    S.static = [dict(name='plane', pos=np.zeros(3), quat=np.array([0, 0, 0, 1.0])),
                dict(name='wheelchair', pos=np.array([0.0, 0.09, -0.01]),
                     quat=G.quat_from_euler([np.pi / 2.0, 0, -np.pi / 2.0 - 0.05])),
                dict(name='table', pos=np.array([0.35, -0.9, 0]), quat=np.array([0, 0, 0, 1.0]))]
    static_body = [S.add_body(KIND_STATIC, 0, plane['shapes'], plane['friction'], 'plane'),
                   S.add_body(KIND_STATIC, 1, chair['shapes'], chair['friction'], 'wheelchair'),
                   S.add_body(KIND_STATIC, 2, table['shapes'], table['friction'], 'table')]
    # human: per-env static bodies; shapes of both genders are compiled, a per-env gender
    # selects which (head VHACD differs; capsule dims differ -> one slot set per gender).
    S.human = {}
    human_body = {}
    for gender in ('male', 'female'):
        base_shapes, hl = build_human(gender, H[gender])
        S.human[gender] = (base_shapes, hl)
    # human slot list: base + DFS links that carry shapes; the slot set is identical for both
    # genders, shapes differ -> store per-gender shapes on the same slot (gender-tagged).
    slot_links = [-1] + [i for i, L in enumerate(S.human['male'][1]) if L['shapes']]
    S.human_slots = slot_links
    for si, li in enumerate(slot_links):
        shapes = []
        for gi, gender in enumerate(('male', 'female')):
            base_shapes, hl = S.human[gender]
            for s in (base_shapes if li < 0 else hl[li]['shapes']):
                s.gender = gi
                shapes.append(s)
        human_body[li] = S.add_body(KIND_HUMAN, si, shapes, 0.5, 'human%d' % li)
    # candidate body pairs (broadphase filter)
    rb = sorted(robot_body.items())
    dyn = [b for _, b in rb] + free_body
    stat = static_body + [human_body[k] for k in slot_links]
    parent = rob['parent']
    pairs = []
    for ia in range(len(rb)):
        for ib in range(ia + 1, len(rb)):
            la, lb = rb[ia][0], rb[ib][0]
            if parent[lb] == la or parent[la] == lb:
                continue                      # self-collision excludes parent/child
            pairs.append((rb[ia][1], rb[ib][1]))
    for li, b in rb:
        for fb in free_body:
            if fb == free_body[0] and 7 <= li <= 14:
                continue                      # spoon vs gripper links (world_creation.py:359-361)
            pairs.append((b, fb))
        for sb in stat:
            pairs.append((b, sb))
    for i in range(len(free_body)):
        for j in range(i + 1, len(free_body)):
            pairs.append((free_body[i], free_body[j]))
        for sb in stat:
            pairs.append((free_body[i], sb))
    # impairment 'tremor' makes the head/neck links dynamic (world_creation.py:157-159 keeps the
    # masses of controllable joints): they then also collide with the static bodies.  These
    # pairs come last and are skipped in the other envs (n_pairs_base).
    S.n_pairs_base = len(pairs)
    for li in HEAD_CHAIN:
        if li in human_body:
            for sb in static_body:
                pairs.append((human_body[li], sb))
    S.pairs = pairs
    S.robot_body = robot_body
    S.table_body = static_body[2]
    S.free_body = free_body
    S.static_body = static_body
    S.human_body = human_body
    S.task = dict(
        arm_dofs=[rob['dof'][j] for j in range(1, 8)],        # joints 1..7 (world_creation.py:283)
        finger_dofs=[rob['dof'][j] for j in (9, 11, 13)],      # world_creation.py:320
        tool_link=8, torso_link=0,                             # world_creation.py:363, feeding.py:124
        tool_pos_offset=np.array([0.1, -0.0225, 0.03]),        # feeding.py:280
        tool_orient_offset=G.quat_from_euler([-0.1, -np.pi / 2.0, 0]),
        head_link=27, mouth_pos={'male': [0, -0.11, 0.03], 'female': [0, -0.1, 0.03]},  # feeding.py:253
    )
    return S


# ----------------------------------------------------------------------------- ScratchItchPR2
PR2_URDF = 'PR2/pr2_no_torso_lift_tall.urdf'
PR2_LEFT_ROOT = 64                                       # l_shoulder_pan_joint (DFS index)
PR2_LEFT_ARM = (64, 65, 66, 68, 69, 71, 72)             # world_creation.py:189
PR2_RIGHT_ARM = (42, 43, 44, 46, 47, 49, 50)            # world_creation.py:188
PR2_RIGHT_ARM_RESET = (-1.75, 1.25, -1.5, -0.5, -1, 0, -1)   # env.py:459-460 (reset_robot_joints)
PR2_LEFT_FINGERS = (79, 80, 81, 82)                     # world_creation.py:311
PR2_TOOL_LINK = 76                                       # l_gripper_tool_frame (world_creation.py:332,363)
PR2_TORSO_LINK = 15                                      # scratch_itch.py:105 (obs origin)
PR2_TOOL_FILTER = range(71, 86)                          # world_creation.py:357-360: tool vs these links off
# static PR2 links (not in the left arm's subtree), grouped into robot-fixed bodies: base +
# casters, torso + head + laser, right arm
PR2_STATIC_GROUPS = (('pr2_base', range(0, 15)), ('pr2_torso', list(range(15, 42)) + [86]), ('pr2_right_arm', range(42, 64)))


def principal_frame(L):
    """URDF_USE_INERTIA_FROM_FILE (world_creation.py:187): Bullet diagonalises the file inertia
    tensor and turns the link's inertial frame onto its principal axes [ext, SURVEY A.2].
    Returns (principal moments, inertial-frame quaternion)."""
    T = L.tensor
    if not np.any(T):
        return np.zeros(3), L.com_quat
    w, V = np.linalg.eigh(T)
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    # rotation matrix -> quaternion (x, y, z, w)
    R = V
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        S4 = np.sqrt(tr + 1.0) * 2
        q = np.array([(R[2, 1] - R[1, 2]) / S4, (R[0, 2] - R[2, 0]) / S4, (R[1, 0] - R[0, 1]) / S4, 0.25 * S4])
    else:
        i = int(np.argmax([R[0, 0], R[1, 1], R[2, 2]]))
        j, k = (i + 1) % 3, (i + 2) % 3
        S4 = np.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = np.zeros(4)
        q[i] = 0.25 * S4
        q[j] = (R[j, i] + R[i, j]) / S4
        q[k] = (R[k, i] + R[i, k]) / S4
        q[3] = (R[k, j] - R[j, k]) / S4
    q = q / np.linalg.norm(q)
    return w, G.quat_mul(L.com_quat, q)


def pr2_fk(dfs, q_of):
    """URDF link frames of every PR2 link in the base_footprint frame for joint values q_of[i]."""
    n = len(dfs)
    P = np.zeros((n, 3)); Q = np.zeros((n, 4))
    for i, (J, parent) in enumerate(dfs):
        pp, pq = (np.zeros(3), np.array([0, 0, 0, 1.0])) if parent < 0 else (P[parent], Q[parent])
        p, qq = G.tf_mul(pp, pq, J['pos'], J['quat'])
        ax = J['axis'] / max(np.linalg.norm(J['axis']), 1e-12)
        v = q_of.get(i, 0.0)
        if J['type'] in ('revolute', 'continuous'):
            qq = G.quat_mul(qq, G.quat_axis_angle(ax, v))
        elif J['type'] == 'prismatic':
            p = p + G.quat_rotate(qq, ax) * v
        P[i], Q[i] = p, qq
    return P, Q


@asset_cached
def build_pr2():
    """The PR2 as ScratchItchPR2-v0 simulates it (world_creation.py:181-217, env.py:450-464):
    fixed base, inertia from file, no self-collision.  Its articulated part is the left arm's
    subtree (links 64..85, 14 DoF); every other link keeps the pose of reset_robot_joints
    (zeros, right arm tucked) for the whole episode -- zero gravity (scratch_itch.py:259), no
    motor target change and no contact pushes them -- and collides as robot-fixed geometry."""
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, PR2_URDF))
    for J, _ in dfs:
        L = links[J['child']]
        L.inertia, L.com_quat = principal_frame(L)
    rootL = links[root]
    rootL.inertia, rootL.com_quat = principal_frame(rootL)
    q_of = {j: v for j, v in zip(PR2_RIGHT_ARM, PR2_RIGHT_ARM_RESET)}
    P, Q = pr2_fk(dfs, q_of)
    # subtree of the left arm root, in DFS order
    sub = [PR2_LEFT_ROOT]
    for i in range(PR2_LEFT_ROOT + 1, len(dfs)):
        if dfs[i][1] in sub:
            sub.append(i)
    rob = dict(name=[], parent=[], jtype=[], dof=[], jpos=[], jquat=[], axis=[], com_pos=[], com_quat=[],
               mass=[], inertia=[], lower=[], upper=[], has_limit=[], shapes=[], friction=[], urdf=[])
    ndof = 0
    for i in sub:
        J, parent = dfs[i]
        L = links[J['child']]
        t = {'fixed': J_FIXED, 'revolute': J_REVOLUTE, 'continuous': J_REVOLUTE, 'prismatic': J_PRISMATIC}[J['type']]
        rob['urdf'].append(i)
        rob['name'].append(L.name)
        if i == PR2_LEFT_ROOT:
            rob['parent'].append(-1)
            jp, jq = G.tf_mul(P[parent], Q[parent], J['pos'], J['quat'])   # torso_lift_link (static) x joint origin
        else:
            rob['parent'].append(sub.index(parent))
            jp, jq = J['pos'], J['quat']
        rob['jtype'].append(t)
        rob['dof'].append(ndof if t != J_FIXED else -1)
        if t != J_FIXED:
            ndof += 1
        rob['jpos'].append(np.asarray(jp))
        rob['jquat'].append(np.asarray(jq))
        rob['axis'].append(J['axis'] / max(np.linalg.norm(J['axis']), 1e-12) if t != J_FIXED else np.zeros(3))
        rob['com_pos'].append(L.com_pos)
        rob['com_quat'].append(L.com_quat)
        rob['mass'].append(L.mass)
        rob['inertia'].append(L.inertia)
        rob['shapes'].append(urdf_shapes(L))
        lim = J['type'] in ('revolute', 'prismatic') and J['lower'] <= J['upper']
        rob['lower'].append(J['lower'] if lim else 0.0)
        rob['upper'].append(J['upper'] if lim else -1.0)
        rob['has_limit'].append(1 if lim else 0)
        rob['friction'].append(L.friction)
    rob['ndof'] = ndof
    # robot-fixed geometry: shapes of the static links placed in the base_footprint frame
    groups = []
    for name, members in PR2_STATIC_GROUPS:
        shapes = []
        for i in members:
            if i in sub:
                continue
            L = links[dfs[i][0]['child']]
            cp, cq = G.tf_mul(P[i], Q[i], L.com_pos, L.com_quat)
            for s in urdf_shapes(L):
                s.pos, s.quat = G.tf_mul(cp, cq, s.pos, s.quat)
                s.urdf_link = i
                shapes.append(s)
        groups.append((name, shapes))
    L15 = links[dfs[PR2_TORSO_LINK][0]['child']]
    torso_com = G.tf_mul(P[PR2_TORSO_LINK], Q[PR2_TORSO_LINK], L15.com_pos, L15.com_quat)[0]
    # base_footprint: inertial origin 0, so PyBullet's base (COM) pose is the URDF root frame
    assert np.allclose(rootL.com_pos, 0)
    return rob, groups, torso_com, sub


@asset_cached
def pr2_frozen_joints():
    """The PR2 joints the build holds at the reset pose (every joint outside the left arm's
    subtree), in the base_footprint frame: per DFS index the parent, the joint type (J_*), the
    joint origin and the world axis at the reset pose.  The reference drives them with PyBullet's
    default velocity motors (world_creation.py:187); tests/test_pr2_frozen_branches.py sets the
    contact impulses the build's rollouts put on these joints against those motors' limit."""
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, PR2_URDF))
    P, Q = pr2_fk(dfs, {j: v for j, v in zip(PR2_RIGHT_ARM, PR2_RIGHT_ARM_RESET)})
    sub = {PR2_LEFT_ROOT}
    for i in range(PR2_LEFT_ROOT + 1, len(dfs)):
        if dfs[i][1] in sub:
            sub.add(i)
    n = len(dfs)
    parent, jtype = np.full(n, -1, np.int32), np.zeros(n, np.int32)
    axis = np.zeros((n, 3))
    for i, (J, par) in enumerate(dfs):
        parent[i] = par
        if i in sub:
            continue
        jtype[i] = {'fixed': J_FIXED, 'revolute': J_REVOLUTE, 'continuous': J_REVOLUTE, 'prismatic': J_PRISMATIC}[J['type']]
        if jtype[i] != J_FIXED:
            axis[i] = G.quat_rotate(Q[i], J['axis'] / max(np.linalg.norm(J['axis']), 1e-12))
    return dict(pr2_parent=parent, pr2_jtype=jtype, pr2_jorigin=P.copy(), pr2_jaxis=axis)


def build_composite_tool(rel, tip_link):
    """A tool URDF loaded by init_tool (world_creation.py:330-365): a base link plus links welded
    by fixed joints, loaded without URDF_USE_INERTIA_FROM_FILE (inertia per link from its
    collision AABB).  A floating base with only fixed links moves as one rigid body: the links
    are composed into one free body at the composite COM, axes those of the base (every link's
    principal axes are the base's).  Returns the body plus the offsets, in that body frame, of
    the base origin (the fixed constraint's child pivot, world_creation.py:363) and of `tip_link`'s
    COM (the tool link getLinkState(tool, 1) reads), and the number of leading shapes that do not
    belong to tip_link (handle_shapes: the shapes the tool-force-at-target rule skips)."""
    links, root, dfs = parse_urdf(os.path.join(REF_ASSETS, rel))
    parts = [(links[root], np.zeros(3), np.array([0, 0, 0, 1.0]))]
    frames = {root: (np.zeros(3), np.array([0, 0, 0, 1.0]))}
    for J, parent in dfs:
        pp, pq = frames[J['parent']]
        frames[J['child']] = G.tf_mul(pp, pq, J['pos'], J['quat'])
        parts.append((links[J['child']],) + frames[J['child']])
    mass = sum(L.mass for L, _, _ in parts)
    coms = [G.tf_mul(p, q, L.com_pos, L.com_quat)[0] for L, p, q in parts]
    c = sum(L.mass * cm for (L, _, _), cm in zip(parts, coms)) / mass
    I = np.zeros(3)
    shapes = []
    lead = None
    for (L, p, q), cm in zip(parts, coms):
        sh = urdf_shapes(L)
        if L.name == tip_link:
            lead = len(shapes)
        lo, hi = compound_aabb(sh)
        Ii = box_inertia(L.mass, lo, hi)
        assert np.allclose(q, [0, 0, 0, 1]) and np.allclose(L.com_quat, [0, 0, 0, 1])
        d = cm - c
        I += Ii + L.mass * (np.dot(d, d) - d * d)        # parallel axes (offsets along the base axes)
        lp, lq = G.tf_mul(p, q, L.com_pos, L.com_quat)
        for s in sh:
            s.pos, s.quat = G.tf_mul(lp - c, lq, s.pos, s.quat)
            shapes.append(s)
    tip = frames[tip_link][0] + links[tip_link].com_pos
    # every link of both composite tools carries the same <contact> block (tool_scratch.urdf:22-25,
    # wiper.urdf:21-24): the composite body takes it
    assert all(links[L.name].rolling == links[root].rolling and links[L.name].spinning == links[root].spinning for L, _, _ in parts)
    return dict(mass=mass, inertia=I, shapes=shapes, friction=links[root].friction, rolling=links[root].rolling, spinning=links[root].spinning,
                pivot=-c, tip=tip - c, handle_shapes=lead)


@asset_cached
def build_scratcher():
    """tool_scratch.urdf (world_creation.py:344): handle (base) + tool cylinder + tip sphere; the
    tool-force-at-target rule counts tool links 0 and 1 (scratch_itch.py:95), i.e. every shape
    after the handle's."""
    t = build_composite_tool('scratcher/tool_scratch.urdf', 'tool_tip')
    links, root, _ = parse_urdf(os.path.join(REF_ASSETS, 'scratcher', 'tool_scratch.urdf'))
    t['handle_shapes'] = len(urdf_shapes(links[root]))
    return t


@asset_cached
def build_wiper():
    """bed_bathing/wiper.urdf (world_creation.py:346): handle (base) + 'tool' box + 'cloth' box;
    bed_bathing.py counts and wipes with tool link 1 only (the cloth, :97)."""
    return build_composite_tool('bed_bathing/wiper.urdf', 'cloth')


def compile_scratch_pr2(heights=None):
    """ScratchItchPR2-v0 scene (scratch_itch.py:130-273 + world_creation.py:27-93,181-217,
    330-365): plane, wheelchair, the human (right arm 7..13 articulated: controllable joints
    4..13 keep their masses, world_creation.py:157-161), the PR2 and the scratcher.  heights:
    per-gender hipbone_to_mouth_height (human_heights).  The scratch target stays on the
    unscaled capsule (generate_target uses the default lengths, scratch_itch.py:277-280)."""
    H = human_heights(heights)
    S = Scene()
    rob, groups, torso_com, sub = build_pr2()
    S.robot = rob
    S.robot_base_pos = np.zeros(3)                 # per env (position_robot_toc): lives in the state
    S.robot_base_quat = np.array([0, 0, 0, 1.0])
    robot_body = {}
    for i in range(len(rob['name'])):
        if rob['shapes'][i]:
            robot_body[i] = S.add_body(KIND_ROBOT, i, rob['shapes'][i], rob['friction'][i], rob['name'][i])
    rstatic_body = [S.add_body(KIND_RSTATIC, k, shapes, 0.5, name) for k, (name, shapes) in enumerate(groups)]
    tool = build_scratcher()
    S.free = [dict(name='scratcher', mass=tool['mass'], inertia=tool['inertia'], gravity=np.zeros(3))]
    tool_body = S.add_body(KIND_FREE, 0, tool['shapes'], tool['friction'], 'scratcher', rolling=tool['rolling'], spinning=tool['spinning'])
    plane = build_static_urdf('plane/plane.urdf')
    chair = build_static_urdf('wheelchair/wheelchair.urdf')
    S.static = [dict(name='plane', pos=np.zeros(3), quat=np.array([0, 0, 0, 1.0])),
                dict(name='wheelchair', pos=np.array([0.0, 0.09, -0.01]),
                     quat=G.quat_from_euler([np.pi / 2.0, 0, -np.pi / 2.0 - 0.05]))]
    static_body = [S.add_body(KIND_STATIC, 0, plane['shapes'], plane['friction'], 'plane'),
                   S.add_body(KIND_STATIC, 1, chair['shapes'], chair['friction'], 'wheelchair')]
    S.human = {}
    human_body = {}
    for gender in ('male', 'female'):
        S.human[gender] = build_human(gender, H[gender])
    slot_links = [-1] + [i for i, L in enumerate(S.human['male'][1]) if L['shapes']]
    S.human_slots = slot_links
    for si, li in enumerate(slot_links):
        shapes = []
        for gi, gender in enumerate(('male', 'female')):
            base_shapes, hl = S.human[gender]
            for s in (base_shapes if li < 0 else hl[li]['shapes']):
                s.gender = gi
                shapes.append(s)
        human_body[li] = S.add_body(KIND_HUMAN, si, shapes, 0.5, 'human%d' % li)
    chain = [human_body[li] for li in ARM_CHAIN if li in human_body]
    # right arm self-collision partners (human_creation.py:283-285: links 7..13 vs -1..3, 14..41)
    arm_partners = [human_body[li] for li in slot_links if li < 4 or li >= 14]
    pairs = []
    for li, b in sorted(robot_body.items()):
        if not (PR2_LEFT_ROOT + li in PR2_TOOL_FILTER):
            pairs.append((b, tool_body))
        for sb in static_body:
            pairs.append((b, sb))
        for h in slot_links:
            pairs.append((b, human_body[h]))
    for rb in rstatic_body:                        # robot-fixed geometry vs the moving bodies
        pairs.append((rb, tool_body))
        for hb in chain:
            pairs.append((rb, hb))
    for sb in static_body:
        pairs.append((tool_body, sb))
    for h in slot_links:
        pairs.append((tool_body, human_body[h]))
    for hb in chain:
        for sb in static_body:
            pairs.append((hb, sb))
        for pb in arm_partners:
            pairs.append((hb, pb))
    S.n_pairs_base = len(pairs)
    S.pairs = pairs
    S.robot_body = robot_body
    S.free_body = [tool_body]
    S.static_body = static_body
    S.human_body = human_body
    S.rstatic = groups
    S.task = dict(
        arm_dofs=[rob['dof'][sub.index(j)] for j in PR2_LEFT_ARM],
        finger_dofs=[rob['dof'][sub.index(j)] for j in PR2_LEFT_FINGERS],
        tool_link=sub.index(PR2_TOOL_LINK), torso_com=torso_com,
        tool_pos_offset=np.zeros(3), tool_orient_offset=np.array([0, 0, 0, 1.0]),   # scratch_itch.py:193
        tool_pivot=tool['pivot'], tool_tip=tool['tip'], tool_handle_shapes=tool['handle_shapes'],
        # generate_target (scratch_itch.py:275-287): limb link, capsule length and radius per gender
        limbs={'male': [(9, 0.279, 0.043), (11, 0.257, 0.033)], 'female': [(9, 0.264, 0.0355), (11, 0.234, 0.027)]},
    )
    return S


BED_Y_OFFSET = -0.53                                     # bed_bathing.py:203
BED_FRICTION = 5.0                                       # bed_bathing.py:281-282 (lateralFriction)
BED_ROLLING = BED_SPINNING = 5.0                         # bed_bathing.py:282 (rollingFriction, spinningFriction)
BED_JOINT_TARGETS = ((7, 50), (8, -50), (17, -30), (28, -60), (35, -60))   # bed_bathing.py:283 (degrees)
BED_HUMAN_BASE = (np.array([0, 0, 0.7]), G.quat_from_euler([np.deg2rad(-30), 0, 0]))   # bed_bathing.py:194


def capsule_points(p1, p2, radius, distance_between_points=0.05, position_scale=1.0):
    """util.capsule_points (util.py:134-167): rings of points around a capsule's axis."""
    p1, p2 = np.asarray(p1, float), np.asarray(p2, float)
    axis = (p2 - p1) / np.linalg.norm(p2 - p1)
    m = int(np.argmax(np.abs(axis)))                     # util.orthogonal_vector (util.py:168-176)
    y = np.zeros(3)
    y[(m + 1) % 3] = 1
    ortho = np.cross(axis, y)
    ortho = ortho / np.linalg.norm(ortho)
    normal = np.cross(axis, ortho)
    sections = int(np.linalg.norm(p2 - p1) / distance_between_points)
    out = []
    for i in range(sections):
        sec = (p2 - p1) / (sections + 1) * (i + 1)
        theta_dist = distance_between_points / radius
        for j in range(int(2 * np.pi * radius / distance_between_points)):
            th = theta_dist * j
            out.append(p1 + sec * position_scale + radius * np.cos(th) * ortho + radius * np.sin(th) * normal)
    return np.array(out)


def bed_targets(heights=None):
    """generate_targets (bed_bathing.py:359-380): wipe targets on the upper arm (link 9) and
    forearm (link 11) capsules, 3 cm apart, in the link frame, per gender.  The ring count
    follows the unscaled capsule length and the axial positions scale by hmhs
    (position_scale, :369-370); hmhs 1 at the default heights."""
    H = human_heights(heights)
    limbs = {'male': ((9, 0.279, 0.043), (11, 0.257, 0.033)), 'female': ((9, 0.264, 0.0355), (11, 0.234, 0.027))}
    out = {}
    for g, ((lu, Lu, ru), (lf, Lf, rf)) in limbs.items():
        hmhs = H[g] / DEFAULT_HEIGHT[g]
        kw = {} if hmhs == 1.0 else dict(position_scale=hmhs)
        out[g] = (capsule_points([0, 0, 0], [0, 0, -Lu], ru, 0.03, **kw), capsule_points([0, 0, 0], [0, 0, -Lf], rf, 0.03, **kw))
    return out


def compile_bedbath_pr2(heights=None):
    """BedBathingPR2-v0 scene (bed_bathing.py:155-357 + world_creation.py:27-93,181-217,330-365):
    plane, the two mattress boxes and the VHACD bed frame (bed_bathing.py:201-218; the bed loaded
    by create_new_world is removed at :202), the human lying on the bed (base at [0, 0, 0.7]
    pitched -30 deg, :194; right arm 7..13 articulated for the reset's 100-frame settle onto the
    mattress under gravity -1, :283-289, static during the episode, :292-300), the PR2 and the
    wiper.  heights: per-gender hipbone_to_mouth_height (human_heights)."""
    H = human_heights(heights)
    S = Scene()
    rob, groups, torso_com, sub = build_pr2()
    S.robot = rob
    S.robot_base_pos = np.zeros(3)                 # per env (position_robot_toc): lives in the state
    S.robot_base_quat = np.array([0, 0, 0, 1.0])
    robot_body = {}
    for i in range(len(rob['name'])):
        if rob['shapes'][i]:
            robot_body[i] = S.add_body(KIND_ROBOT, i, rob['shapes'][i], rob['friction'][i], rob['name'][i])
    rstatic_body = [S.add_body(KIND_RSTATIC, k, shapes, 0.5, name) for k, (name, shapes) in enumerate(groups)]
    tool = build_wiper()
    S.free = [dict(name='wiper', mass=tool['mass'], inertia=tool['inertia'], gravity=np.zeros(3))]
    tool_body = S.add_body(KIND_FREE, 0, tool['shapes'], tool['friction'], 'wiper', rolling=tool['rolling'], spinning=tool['spinning'])
    plane = build_static_urdf('plane/plane.urdf')
    m1 = [Shape(BOX, (0, 0, 0.15 / 2.0), half_extents=(0.88 / 2.0, 1.25 / 2.0, 0.15 / 2.0))]
    m2 = [Shape(BOX, (0, 0.7 / 2.0, 0), half_extents=(0.88 / 2.0, 0.7 / 2.0, 0.15 / 2.0))]
    frame = [Shape(HULL, hull=h) for h in bed_frame_hulls()]
    S.static = [dict(name='plane', pos=np.zeros(3), quat=np.array([0, 0, 0, 1.0])),
                dict(name='mattress', pos=np.array([0, BED_Y_OFFSET, 0.4]), quat=np.array([0, 0, 0, 1.0])),
                dict(name='mattress_head', pos=np.array([0, 1.25 / 2.0 + BED_Y_OFFSET, 0.4 + 0.15 / 2.0]), quat=G.quat_from_euler([np.deg2rad(60), 0, 0])),
                dict(name='bed_frame', pos=np.array([0, BED_Y_OFFSET + 0.45, 0.42]), quat=G.quat_from_euler([np.pi / 2.0, 0, -np.pi / 2.0]))]
    static_body = [S.add_body(KIND_STATIC, 0, plane['shapes'], plane['friction'], 'plane'),
                   S.add_body(KIND_STATIC, 1, m1, BED_FRICTION, 'mattress', single=False, rolling=BED_ROLLING, spinning=BED_SPINNING),
                   S.add_body(KIND_STATIC, 2, m2, BED_FRICTION, 'mattress_head', single=False, rolling=BED_ROLLING, spinning=BED_SPINNING),
                   S.add_body(KIND_STATIC, 3, frame, BED_FRICTION, 'bed_frame', rolling=BED_ROLLING, spinning=BED_SPINNING)]
    S.human = {}
    human_body = {}
    for gender in ('male', 'female'):
        S.human[gender] = build_human(gender, H[gender])
    slot_links = [-1] + [i for i, L in enumerate(S.human['male'][1]) if L['shapes']]
    S.human_slots = slot_links
    for si, li in enumerate(slot_links):
        shapes = []
        for gi, gender in enumerate(('male', 'female')):
            base_shapes, hl = S.human[gender]
            for s in (base_shapes if li < 0 else hl[li]['shapes']):
                s.gender = gi
                shapes.append(s)
        human_body[li] = S.add_body(KIND_HUMAN, si, shapes, 0.5, 'human%d' % li)
    chain = [human_body[li] for li in ARM_CHAIN if li in human_body]
    arm_partners = [human_body[li] for li in slot_links if li < 4 or li >= 14]
    pairs = []
    for li, b in sorted(robot_body.items()):
        if not (PR2_LEFT_ROOT + li in PR2_TOOL_FILTER):
            pairs.append((b, tool_body))
        for sb in static_body:
            pairs.append((b, sb))
        for h in slot_links:
            pairs.append((b, human_body[h]))
    for rb in rstatic_body:
        pairs.append((rb, tool_body))
        for hb in chain:
            pairs.append((rb, hb))
    for sb in static_body:
        pairs.append((tool_body, sb))
    for h in slot_links:
        pairs.append((tool_body, human_body[h]))
    for hb in chain:                               # the reset's settle: the arm onto the mattress / itself
        for sb in static_body:
            pairs.append((hb, sb))
        for pb in arm_partners:
            pairs.append((hb, pb))
    S.n_pairs_base = len(pairs)
    S.pairs = pairs
    S.robot_body = robot_body
    S.free_body = [tool_body]
    S.static_body = static_body
    S.human_body = human_body
    S.rstatic = groups
    S.task = dict(
        arm_dofs=[rob['dof'][sub.index(j)] for j in PR2_LEFT_ARM],
        finger_dofs=[rob['dof'][sub.index(j)] for j in PR2_LEFT_FINGERS],
        tool_link=sub.index(PR2_TOOL_LINK), torso_com=torso_com,
        tool_pos_offset=np.zeros(3), tool_orient_offset=np.array([0, 0, 0, 1.0]),   # bed_bathing.py:320
        tool_pivot=tool['pivot'], tool_tip=tool['tip'], tool_handle_shapes=tool['handle_shapes'],
        targets=bed_targets(H),
    )
    return S


def to_arrays(S):
    """Flatten a Scene into the arrays of include/avr_model.h (float64 / int32)."""
    rob = S.robot
    A = {}
    nl = len(rob['name'])
    A['rl_parent'] = np.array(rob['parent'], np.int32)
    A['rl_jtype'] = np.array(rob['jtype'], np.int32)
    A['rl_dof'] = np.array(rob['dof'], np.int32)
    A['rl_jpos'] = np.array(rob['jpos'])
    A['rl_jquat'] = np.array(rob['jquat'])
    A['rl_axis'] = np.array(rob['axis'])
    A['rl_com_pos'] = np.array(rob['com_pos'])
    A['rl_com_quat'] = np.array(rob['com_quat'])
    A['rl_mass'] = np.array(rob['mass'])
    A['rl_inertia'] = np.array(rob['inertia'])
    A['rl_lower'] = np.array(rob['lower'])
    A['rl_upper'] = np.array(rob['upper'])
    A['rl_has_limit'] = np.array(rob['has_limit'], np.int32)
    A['robot_base'] = np.concatenate([S.robot_base_pos, S.robot_base_quat])
    A['fb_mass'] = np.array([f['mass'] for f in S.free])
    A['fb_inertia'] = np.array([f['inertia'] for f in S.free])
    A['fb_gravity'] = np.array([f['gravity'] for f in S.free])
    A['st_pose'] = np.array([np.concatenate([s['pos'], s['quat']]) for s in S.static])
    # shapes, sorted by body
    shape_rows, hv = [], []
    b_start, b_count, b_kind, b_index, b_fric, b_thr, b_aabb, b_flags = [], [], [], [], [], [], [], []
    for b in S.bodies:
        b_start.append(len(shape_rows))
        b_count.append(len(b['shapes']))
        b_kind.append(b['kind'])
        b_index.append(b['index'])
        b_fric.append(b['friction'])
        if b['kind'] == KIND_HUMAN:
            # per-gender AABBs; threshold: min over genders (they differ by <10%)
            per = [[s for s in b['shapes'] if s.gender == g] for g in (0, 1)]
            thr = min(breaking_threshold(p) for p in per)
            boxes = [compound_aabb(p) for p in per]
        else:
            thr = breaking_threshold(b['shapes'])
            boxes = [compound_aabb(b['shapes'])] * 2
        b_thr.append(thr)
        b_aabb.append(np.concatenate([np.concatenate([0.5 * (lo + hi), 0.5 * (hi - lo)]) for lo, hi in boxes]))
        b_flags.append(1 if b.get('single', False) else 0)
        for s in b['shapes']:
            c, h = s.local_aabb()
            row = dict(kind=s.kind, body=len(b_start) - 1, pos=s.pos, quat=s.quat, margin=s.margin,
                       gender=s.gender, aabb=np.concatenate([c, h]), link=getattr(s, 'urdf_link', -1))
            if s.kind == SPHERE:
                row['param'] = [s.radius, 0, 0, 0]
            elif s.kind == CAPSULE:
                row['param'] = [s.radius, s.half_height, 0, 0]
            elif s.kind == BOX:
                row['param'] = [s.half_extents[0], s.half_extents[1], s.half_extents[2], 0]
            else:
                row['param'] = [0, 0, 0, 0]
            if s.kind == HULL:
                row['hull'] = [len(hv), len(s.hull.verts), 0, 0]
                hv.extend(s.hull.verts)
            else:
                row['hull'] = [0, 0, 0, 0]
            shape_rows.append(row)
    A['body_kind'] = np.array(b_kind, np.int32)
    A['body_index'] = np.array(b_index, np.int32)
    A['body_shape_start'] = np.array(b_start, np.int32)
    A['body_shape_count'] = np.array(b_count, np.int32)
    A['body_friction'] = np.array(b_fric)
    A['body_rolling'] = np.array([b['rolling'] for b in S.bodies], np.float64)
    A['body_spinning'] = np.array([b['spinning'] for b in S.bodies], np.float64)
    A['body_threshold'] = np.array(b_thr)
    A['body_aabb'] = np.array(b_aabb)
    A['body_flags'] = np.array(b_flags, np.int32)
    A['shape_kind'] = np.array([r['kind'] for r in shape_rows], np.int32)
    A['shape_body'] = np.array([r['body'] for r in shape_rows], np.int32)
    A['shape_gender'] = np.array([r['gender'] for r in shape_rows], np.int32)
    A['shape_hull'] = np.array([r['hull'] for r in shape_rows], np.int32)
    A['shape_pose'] = np.array([np.concatenate([r['pos'], r['quat']]) for r in shape_rows])
    A['shape_param'] = np.array([r['param'] for r in shape_rows], float)
    A['shape_margin'] = np.array([r['margin'] for r in shape_rows])
    A['shape_aabb'] = np.array([r['aabb'] for r in shape_rows])
    if any(r['link'] >= 0 for r in shape_rows):       # (robot-fixed PR2 geometry: the URDF link of each shape)
        A['shape_urdf_link'] = np.array([r['link'] for r in shape_rows], np.int32)
    A['hull_verts'] = np.array(hv).reshape(-1, 3)
    A['pair_a'] = np.array([p[0] for p in S.pairs], np.int32)
    A['pair_b'] = np.array([p[1] for p in S.pairs], np.int32)
    A['n_links'] = np.int32(nl)
    A['n_dof'] = np.int32(rob['ndof'])
    return A


def _human_tables(S, A):
    """Human kinematic tables for the host reset path, both genders."""
    for gender in ('male', 'female'):
        base_shapes, hl = S.human[gender]
        A['human_%s_parent' % gender] = np.array([L['parent'] for L in hl], np.int32)
        A['human_%s_jtype' % gender] = np.array([L['jtype'] for L in hl], np.int32)
        A['human_%s_axis' % gender] = np.array([L['axis'] for L in hl])
        A['human_%s_pos' % gender] = np.array([L['pos'] for L in hl])
        A['human_%s_lower' % gender] = np.array([L['lower'] for L in hl])
        A['human_%s_upper' % gender] = np.array([L['upper'] for L in hl])
    A['human_slot_link'] = np.array(S.human_slots, np.int32)
    A['n_pairs_base'] = np.int32(S.n_pairs_base)


def feeding_arrays(heights=None):
    S = compile_feeding_jaco(heights)
    A = to_arrays(S)
    _human_tables(S, A)
    A.update(head_chain(S, HEAD_CHAIN, cap=4))
    t = S.task
    A['task_arm_dofs'] = np.array(t['arm_dofs'], np.int32)
    A['task_finger_dofs'] = np.array(t['finger_dofs'], np.int32)
    A['task_tool_link'] = np.int32(t['tool_link'])
    A['task_torso_link'] = np.int32(t['torso_link'])
    A['task_tool_offset'] = np.concatenate([t['tool_pos_offset'], t['tool_orient_offset']])
    A['task_head_link'] = np.int32(t['head_link'])
    A['task_mouth_male'] = np.array(t['mouth_pos']['male'], float)
    A['task_mouth_female'] = np.array(t['mouth_pos']['female'], float)
    A['task_spoon_body'] = np.int32(S.free_body[0])
    A['task_bowl_body'] = np.int32(S.free_body[1])
    A['task_food_body0'] = np.int32(S.free_body[2])
    A['task_table_body'] = np.int32(S.table_body)
    A['task_human_body0'] = np.int32(S.human_body[S.human_slots[0]])
    A['task_head_slot'] = np.int32(S.human_slots.index(t['head_link']))
    return A


def compile_feeding(out_dir=DATA_DIR):
    os.makedirs(out_dir, exist_ok=True)
    A = feeding_arrays()
    path = os.path.join(out_dir, 'feeding_jaco.npz')
    np.savez_compressed(path, **A)
    return path, A


def scratch_arrays(heights=None):
    S = compile_scratch_pr2(heights)
    A = to_arrays(S)
    _human_tables(S, A)
    A.update(head_chain(S, ARM_CHAIN, cap=HC_CAP))
    t = S.task
    A['task_arm_dofs'] = np.array(t['arm_dofs'], np.int32)
    A['task_finger_dofs'] = np.array(t['finger_dofs'], np.int32)
    A['task_tool_link'] = np.int32(t['tool_link'])
    A['task_tool_offset'] = np.concatenate([t['tool_pos_offset'], t['tool_orient_offset']])
    A['task_torso_com'] = np.asarray(t['torso_com'], float)
    A['task_tool_pivot'] = np.asarray(t['tool_pivot'], float)
    A['task_tool_tip'] = np.asarray(t['tool_tip'], float)
    A['task_tool_handle_shapes'] = np.int32(t['tool_handle_shapes'])
    A['task_tool_body'] = np.int32(S.free_body[0])
    A['task_human_body0'] = np.int32(S.human_body[S.human_slots[0]])
    A['task_limbs'] = np.array([[[li, ln, r] for li, ln, r in t['limbs'][g]] for g in ('male', 'female')], float)
    A['n_rstatic'] = np.int32(len(S.rstatic))
    A['rl_urdf'] = np.array(S.robot['urdf'], np.int32)
    A.update(pr2_frozen_joints())
    return A


def compile_scratch(out_dir=DATA_DIR):
    os.makedirs(out_dir, exist_ok=True)
    A = scratch_arrays()
    path = os.path.join(out_dir, 'scratch_itch_pr2.npz')
    np.savez_compressed(path, **A)
    return path, A


def bedbath_arrays(heights=None):
    S = compile_bedbath_pr2(heights)
    A = to_arrays(S)
    _human_tables(S, A)
    A.update(head_chain(S, ARM_CHAIN, cap=HC_CAP))
    t = S.task
    A['task_arm_dofs'] = np.array(t['arm_dofs'], np.int32)
    A['task_finger_dofs'] = np.array(t['finger_dofs'], np.int32)
    A['task_tool_link'] = np.int32(t['tool_link'])
    A['task_tool_offset'] = np.concatenate([t['tool_pos_offset'], t['tool_orient_offset']])
    A['task_torso_com'] = np.asarray(t['torso_com'], float)
    A['task_tool_pivot'] = np.asarray(t['tool_pivot'], float)
    A['task_tool_tip'] = np.asarray(t['tool_tip'], float)
    A['task_tool_handle_shapes'] = np.int32(t['tool_handle_shapes'])
    A['task_tool_body'] = np.int32(S.free_body[0])
    A['task_human_body0'] = np.int32(S.human_body[S.human_slots[0]])
    A['n_rstatic'] = np.int32(len(S.rstatic))
    A['rl_urdf'] = np.array(S.robot['urdf'], np.int32)
    A.update(pr2_frozen_joints())
    # wipe targets [gender][k] = (x, y, z in the limb frame, limb 0 upper arm / 1 forearm)
    T = np.zeros((2, 160, 4))
    NT = np.zeros((2, 2), np.int32)
    for g, gender in enumerate(('male', 'female')):
        up, fo = t['targets'][gender]
        NT[g] = len(up), len(fo)
        T[g, :len(up), :3] = up
        T[g, len(up):len(up) + len(fo), :3] = fo
        T[g, len(up):len(up) + len(fo), 3] = 1.0
    A['bb_targets'] = T
    A['bb_ntgt'] = NT
    A['bb_limb_slots'] = np.array([S.human_slots.index(9), S.human_slots.index(11)], np.int32)
    A['bb_joint_slots'] = np.array([S.human_slots.index(9), S.human_slots.index(11), S.human_slots.index(13)], np.int32)
    A['bb_human_base'] = np.concatenate(BED_HUMAN_BASE)
    A['bb_bed_bodies'] = np.array(S.static_body[1:], np.int32)
    return A


def compile_bedbath(out_dir=DATA_DIR):
    os.makedirs(out_dir, exist_ok=True)
    A = bedbath_arrays()
    path = os.path.join(out_dir, 'bed_bathing_pr2.npz')
    np.savez_compressed(path, **A)
    return path, A


SCENE_ARRAYS = {'feeding_jaco': feeding_arrays, 'scratch_itch_pr2': scratch_arrays, 'bed_bathing_pr2': bedbath_arrays}


def scene_arrays(name, heights=None):
    """A compiled scene's arrays (what the committed npz holds at the default heights) with the
    human built at per-gender hipbone_to_mouth_height `heights` (human_heights)."""
    A = SCENE_ARRAYS[name](heights)
    A['human_heights'] = np.array([human_heights(heights)[g] for g in ('male', 'female')])
    return A


def compile_all(out_dir=DATA_DIR):
    """All compiled scenes, and the asset cache scene_arrays rebuilds them from; returns the
    FeedingJaco one (path, arrays) first."""
    global _asset_memo
    _asset_memo = {}                     # rebuilt from the reference's assets
    out = compile_feeding(out_dir)
    compile_scratch(out_dir)
    compile_bedbath(out_dir)
    save_asset_cache(os.path.join(out_dir, 'asset_cache.npz'))
    return out


if __name__ == '__main__':
    for path, A in (compile_feeding(), compile_scratch(), compile_bedbath()):
        print(path)
        for k, v in A.items():
            print('%-24s %s %s' % (k, getattr(v, 'shape', ()), getattr(v, 'dtype', type(v))))
