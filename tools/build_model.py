#!/usr/bin/env python3
"""Offline asset pipeline: reference URDF + meshes -> committed scene model (JSON).

Runs ONLY in the build container (it reads /root/reference/assets, which does not exist on the GPU
box). Its output, ``isaacgym-hand-arm_amd/handarm_hip/assets/ur5sih_scene.json``, is committed and is
the only thing the runtime reads.

What it restates (and why), with reference citations:

* Robot asset: ``assets/hand_arm/robot/hand_arm_collision_is_visual.urdf`` loaded with
  ``fix_base_link``, ``override_com``, ``override_inertia``, ``disable_gravity``
  (``tasks/hand_arm/base/ur5sih.py:169-180``) and actor pose ``(0, 0, table_height)``
  (``ur5sih.py:125``).
* Body / DOF order: Isaac Gym orders bodies depth-first; siblings are visited in link-name order
  (inferred, SURVEY.md §8 a2: it puts ``thumb_opposition`` at DOF 14 exactly as
  ``Ur5SihBase.yaml:8`` and the gain table ``Ur5SihBase.yaml:3-4`` require).
* Collision geometry: PhysX cooks a convex hull (<= 64 vertices on the GPU pipeline) for every
  dynamic mesh shape; we do the same offline (scipy Qhull) and reduce to <= ``MAX_LINK_VERTS`` /
  ``MAX_OBJ_VERTS`` vertices by farthest-point sampling. YCB objects are V-HACD decomposed in the
  reference (``multi_object.py:37-43``); the three default objects are close to convex, so one hull
  each is used (documented deviation, parity vs PhysX unpinned).
* The SIH palm visual mesh is missing from the reference checkout (``.MISSING_LARGE_BLOBS:58``); the
  palm uses the five convex collision pieces that ``hand_arm.urdf:360-385`` assigns to it.
* Mass properties: links/objects with an URDF ``<inertial>`` keep its mass; COM and inertia come from
  the collision hulls (override_com / override_inertia). Links without ``<inertial>`` get
  density 1000 kg/m^3 x hull volume (Isaac Gym's default asset density).
* Object bounding boxes (``multi_object.py:84-88,743-768``): trimesh ``oriented_bounds`` is absent
  here; we compute a minimum-volume box over hull-facet-normal candidate frames (2-D rotating
  calipers in the orthogonal plane), which is the same search trimesh performs. Parity unpinned.
"""
import json
import math
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

REF = "/root/reference"
ASSETS = os.path.join(REF, "assets", "hand_arm")
ROBOT_URDF = os.path.join(ASSETS, "robot", "hand_arm_collision_is_visual.urdf")
PALM_URDF = os.path.join(ASSETS, "robot", "hand_arm.urdf")
OUT = os.path.join(os.path.dirname(__file__), "..", "isaacgym-hand-arm_amd", "handarm_hip",
                   "assets", "ur5sih_scene.json")

MAX_LINK_VERTS = 32
MAX_OBJ_VERTS = 64
DENSITY = 1000.0
TABLE_HEIGHT = 0.5  # Ur5SihMultiObject.yaml:48
YCB_POOL = ["015_peach", "005_tomato_soup_can", "006_mustard_bottle",   # default set (yaml:11)
            "004_sugar_box", "007_tuna_fish_can", "008_pudding_box", "009_gelatin_box",
            "010_potted_meat_can", "013_apple", "014_lemon", "016_pear", "017_orange",
            "018_plum", "025_mug", "061_foam_brick", "077_rubiks_cube"]


# ----------------------------------------------------------------------------- math helpers
def rpy_to_matrix(r, p, y):
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def scipy_quat(R):
    """Rotation matrix -> quaternion exactly as the reference converts the bounding-box frame
    (scipy Rotation.from_matrix(...).as_quat(), multi_object.py:751-753): same rotation as matrix_to_quat but
    scipy's sign choice, which the observed bounding-box quaternion (quat_mul with it) inherits."""
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(np.asarray(R, float)).as_quat()


def matrix_to_quat(R):
    """Rotation matrix -> quaternion (x, y, z, w), w >= 0."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        w, x, y, z = (R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        w, x, y, z = (R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        w, x, y, z = (R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s
    q = np.array([x, y, z, w])
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


# ----------------------------------------------------------------------------- mesh IO
def load_obj(path):
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(t) for t in line.split()[1:4]])
            elif line.startswith("f "):
                idx = [int(t.split("/")[0]) - 1 for t in line.split()[1:]]
                for k in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[k], idx[k + 1]])
    return np.array(verts, dtype=np.float64), np.array(faces, dtype=np.int64)


def load_stl(path):
    with open(path, "rb") as f:
        data = f.read()
    n = struct.unpack("<I", data[80:84])[0]
    if 84 + 50 * n == len(data):
        rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)),
                                                        ("a", "<u2")]), count=n)
        tri = rec["v"].astype(np.float64).reshape(-1, 3)
    else:  # ascii
        tri = np.array([[float(t) for t in ln.split()[1:4]] for ln in data.decode().splitlines()
                        if ln.strip().startswith("vertex")])
    faces = np.arange(len(tri)).reshape(-1, 3)
    return tri, faces


def load_mesh(path, scale):
    v, f = load_obj(path) if path.lower().endswith(".obj") else load_stl(path)
    return v * np.asarray(scale, dtype=np.float64), f


# ----------------------------------------------------------------------------- hulls
def reduce_points(points, max_verts):
    hull = ConvexHull(points)
    pts = points[hull.vertices]
    if len(pts) <= max_verts:
        return pts
    c = pts.mean(0)
    chosen = [int(np.argmax(np.linalg.norm(pts - c, axis=1)))]
    d = np.linalg.norm(pts - pts[chosen[0]], axis=1)
    while len(chosen) < max_verts:
        i = int(np.argmax(d))
        chosen.append(i)
        d = np.minimum(d, np.linalg.norm(pts - pts[i], axis=1))
    return pts[chosen]


def hull_planes(points):
    hull = ConvexHull(points)
    planes = []
    for eq in hull.equations:  # n.x + d <= 0 inside
        n, d = eq[:3], eq[3]
        dup = False
        for p in planes:
            if np.dot(p[:3], n) > 1 - 1e-6 and abs(p[3] - d) < 1e-7:
                dup = True
                break
        if not dup:
            planes.append(np.concatenate([n, [d]]))
    verts = points[hull.vertices]
    return verts, np.array(planes), hull


def polyhedron_mass_props(points):
    """Volume, centroid and inertia (about centroid, unit density) of the convex hull of points."""
    hull = ConvexHull(points)
    P = hull.points
    c0 = P[hull.vertices].mean(0)
    tri = P[hull.simplices]                                   # (F, 3, 3)
    flip = np.einsum("fi,fi->f", np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]),
                     hull.equations[:, :3]) < 0
    tri[flip] = tri[flip][:, [0, 2, 1]]
    A = np.transpose(tri - c0, (0, 2, 1))                     # columns = a-c0, b-c0, c-c0
    det = np.linalg.det(A)
    vol = det.sum() / 6.0
    com = (det[:, None] / 6.0 * (tri.sum(1) + c0) / 4.0).sum(0) / vol
    canon = np.array([[2, 1, 1], [1, 2, 1], [1, 1, 2]]) / 120.0
    cov = np.einsum("f,fij,jk,flk->il", det, A, canon, A)
    d = com - c0
    cov_com = cov - vol * np.outer(d, d)
    inertia = np.trace(cov_com) * np.eye(3) - cov_com
    return vol, com, inertia


def min_volume_obb(points):
    """Minimum-volume oriented box over facet-normal candidate frames (trimesh-style search)."""
    verts, _, hull = hull_planes(points)
    best = None
    for eq in hull.equations:
        n = eq[:3] / np.linalg.norm(eq[:3])
        a = np.array([1.0, 0, 0]) if abs(n[0]) < 0.9 else np.array([0, 1.0, 0])
        u = np.cross(n, a)
        u /= np.linalg.norm(u)
        w = np.cross(n, u)
        p2 = np.stack([verts @ u, verts @ w], 1)
        h2 = ConvexHull(p2)
        hp = p2[h2.vertices]
        hn = verts @ n
        for k in range(len(hp)):
            e = hp[(k + 1) % len(hp)] - hp[k]
            e /= np.linalg.norm(e)
            ep = np.array([-e[1], e[0]])
            s1, s2 = p2 @ e, p2 @ ep
            ext = np.array([s1.max() - s1.min(), s2.max() - s2.min(), hn.max() - hn.min()])
            vol = ext.prod()
            if best is None or vol < best[0]:
                ax = e[0] * u + e[1] * w
                ay = ep[0] * u + ep[1] * w
                az = np.cross(ax, ay)
                R = np.stack([ax, ay, az], 1)
                cz = verts @ az
                ext[2] = cz.max() - cz.min()
                ctr = ax * (s1.max() + s1.min()) / 2 + ay * (s2.max() + s2.min()) / 2 + az * (cz.max() + cz.min()) / 2
                best = (ext.prod(), R, ctr, ext)
    _, R, ctr, ext = best
    # trimesh convention: extents sorted is not guaranteed; keep frame as found.
    return R, ctr, ext


def hull_record(points, max_verts):
    pts = reduce_points(points, max_verts)
    verts, planes, _ = hull_planes(pts)
    center = 0.5 * (verts.min(0) + verts.max(0))
    radius = float(np.linalg.norm(verts - center, axis=1).max())
    return {"verts": verts.tolist(), "planes": planes.tolist(), "center": center.tolist(),
            "radius": radius}


# ----------------------------------------------------------------------------- URDF
def parse_origin(el):
    if el is None:
        return np.zeros(3), np.eye(3)
    xyz = [float(t) for t in el.get("xyz", "0 0 0").split()]
    rpy = [float(t) for t in el.get("rpy", "0 0 0").split()]
    return np.array(xyz), rpy_to_matrix(*rpy)


def link_collision_points(link_el, base_dir, palm_override=None):
    pts = []
    pieces = []
    colls = link_el.findall("collision")
    if palm_override is not None:
        colls = palm_override
    for c in colls:
        g = c.find("geometry/mesh")
        if g is None:
            continue
        path = os.path.join(base_dir, g.get("filename"))
        if not os.path.exists(path):
            return None
        scale = [float(t) for t in g.get("scale", "1 1 1").split()]
        v, _ = load_mesh(path, scale)
        o, R = parse_origin(c.find("origin"))
        v = v @ R.T + o
        pieces.append(v)
        pts.append(v)
    if not pts:
        return []
    return pieces


def build_robot():
    base_dir = os.path.dirname(ROBOT_URDF)
    root = ET.parse(ROBOT_URDF).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    children = {}
    parent_joint = {}
    for j in joints:
        p, c = j.find("parent").get("link"), j.find("child").get("link")
        children.setdefault(p, []).append(c)
        parent_joint[c] = j
    roots = [n for n in links if n not in parent_joint]
    assert roots == ["base_link"], roots
    order = []

    def dfs(n):
        order.append(n)
        for c in sorted(children.get(n, [])):
            dfs(c)
    dfs("base_link")
    idx = {n: i for i, n in enumerate(order)}

    palm_colls = [l for l in ET.parse(PALM_URDF).getroot().findall("link") if l.get("name") == "palm"][0]
    palm_colls = palm_colls.findall("collision")

    prop_gain = [120., 120., 120., 120., 120., 120., 20., 10., 20., 10., 20., 10., 20., 10., 20., 20., 10.]
    deriv_gain = [20., 20., 20., 20., 20., 20., 6., 2., 6., 2., 6., 2., 6., 2., 6., 6., 2.]

    out_links, dofs, hulls = [], [], []
    for n in order:
        el = links[n]
        j = parent_joint.get(n)
        rec = {"name": n, "parent": -1, "joint": None, "type": "fixed", "origin_pos": [0, 0, 0],
               "origin_quat": [0, 0, 0, 1], "axis": [0, 0, 1], "dof": -1}
        if j is not None:
            o, R = parse_origin(j.find("origin"))
            rec.update(parent=idx[j.find("parent").get("link")], joint=j.get("name"),
                       type=j.get("type"), origin_pos=o.tolist(), origin_quat=matrix_to_quat(R).tolist())
            ax = j.find("axis")
            if ax is not None:
                a = np.array([float(t) for t in ax.get("xyz").split()])
                rec["axis"] = (a / np.linalg.norm(a)).tolist()
            if j.get("type") == "revolute":
                lim = j.find("limit")
                rec["dof"] = len(dofs)
                dofs.append({"name": j.get("name"), "link": idx[n], "lower": float(lim.get("lower")),
                             "upper": float(lim.get("upper")), "effort": float(lim.get("effort")),
                             "velocity": float(lim.get("velocity")),
                             "kp": prop_gain[len(dofs)], "kd": deriv_gain[len(dofs)]})
        pieces = link_collision_points(el, base_dir, palm_colls if n == "palm" else None)
        inertial = el.find("inertial")
        mass = float(inertial.find("mass").get("value")) if inertial is not None else None
        if pieces:
            allp = np.concatenate(pieces, 0)
            vol, com, I_unit = polyhedron_mass_props(allp)
            if mass is None:
                mass = DENSITY * vol
            inertia = I_unit * (mass / vol)
            for pc in pieces:
                h = hull_record(pc, MAX_LINK_VERTS)
                h.update(owner="link", index=idx[n])
                hulls.append(h)
        elif inertial is not None:
            o, R = parse_origin(inertial.find("origin"))
            ie = inertial.find("inertia")
            I = np.array([[float(ie.get("ixx")), float(ie.get("ixy")), float(ie.get("ixz"))],
                          [float(ie.get("ixy")), float(ie.get("iyy")), float(ie.get("iyz"))],
                          [float(ie.get("ixz")), float(ie.get("iyz")), float(ie.get("izz"))]])
            com, inertia = o, R @ I @ R.T
        else:
            mass, com, inertia = 0.0, np.zeros(3), np.zeros((3, 3))
        rec.update(mass=float(mass), com=np.asarray(com).tolist(), inertia=np.asarray(inertia).reshape(-1).tolist())
        out_links.append(rec)
    return {"links": out_links, "dofs": dofs, "base_pos": [0.0, 0.0, TABLE_HEIGHT],
            "base_quat": [0.0, 0.0, 0.0, 1.0]}, hulls


# Pool objects whose collision shape is a set of convex pieces, like the reference's V-HACD
# (multi_object.py:37-43): the mug is the one clearly non-convex pool object (mesh volume 138 cm3 against 525 cm3
# for its convex hull; every other pool object is within 20 %), so it alone is decomposed (tools/convex_decomp.py
# decompose_vessel: base slab, 6 wall sectors, 2 handle pieces; the cavity and the handle gap stay open).
DECOMPOSE = {"025_mug": "vessel"}
# The wide pool (round 5, verdict f1): the clearly concave objects of the reference's commented dataset list
# (Ur5SihMultiObject.yaml:8; mesh volume under half of the convex hull's), each decomposed like the mug -
# (kind, voxel pitch): "acd" the general voxel ACD (tools/convex_decomp.py decompose, <= 8 pieces), "vessel" the
# handle-less cups as a base slab and six wall sectors. Pieces are cooked to <= MAX_PIECE_VERTS vertices.
CONCAVE_POOL = {"031_spoon": ("acd", 0.002), "033_spatula": ("acd", 0.0025), "037_scissors": ("acd", 0.002),
                "042_adjustable_wrench": ("acd", 0.002), "050_medium_clamp": ("acd", 0.0015),
                "065-a_cups": ("vessel", 0.001), "065-d_cups": ("vessel", 0.001), "073-a_lego_duplo": ("acd", 0.0015)}
MAX_PIECE_VERTS = 32


def build_object(name):
    urdf = os.path.join(ASSETS, "object_sets", "urdf", "ycb", name + ".urdf")
    root = ET.parse(urdf).getroot()
    link = root.find("link")
    mass = float(link.find("inertial/mass").get("value"))
    mesh = link.find("collision/geometry/mesh").get("filename")
    v, f = load_mesh(os.path.normpath(os.path.join(os.path.dirname(urdf), mesh)), [1, 1, 1])
    hull = hull_record(v, MAX_OBJ_VERTS)
    vol, com, I_unit = polyhedron_mass_props(v)
    R, ctr, ext = min_volume_obb(reduce_points(v, 256))
    rec = {"name": name, "mass": mass, "com": com.tolist(),
           "inertia": (I_unit * mass / vol).reshape(-1).tolist(), "hull": hull,
           "bbox_from_origin_pos": ctr.tolist(), "bbox_from_origin_quat": scipy_quat(R).tolist(),
           "bbox_extents": ext.tolist()}
    if name in DECOMPOSE or name in CONCAVE_POOL:
        import convex_decomp as CD
        if name in DECOMPOSE:
            pieces, _ = CD.decompose_vessel(v, f)
            rec["hulls"] = [hull_record(p, MAX_OBJ_VERTS) for p in pieces]
        else:
            kind, h = CONCAVE_POOL[name]
            pieces, _ = (CD.decompose_vessel(v, f, h=h, sectors=6, handle_pieces=0) if kind == "vessel"
                         else CD.decompose(v, f, h=h, max_pieces=8, tol=0.1))
            rec["hulls"] = [hull_record(p, MAX_PIECE_VERTS) for p in pieces]
        # mass properties of the actual (non-convex) shape: the closed mesh itself
        vol, com, I_unit = CD.mesh_volume_props(v, f)
        rec["com"] = com.tolist()
        rec["inertia"] = (I_unit * mass / vol).reshape(-1).tolist()
    return rec


def box_hull(half):
    hx, hy, hz = half
    verts = [[sx * hx, sy * hy, sz * hz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    planes = [[1, 0, 0, -hx], [-1, 0, 0, -hx], [0, 1, 0, -hy], [0, -1, 0, -hy], [0, 0, 1, -hz], [0, 0, -1, -hz]]
    return {"verts": verts, "planes": planes, "center": [0, 0, 0], "radius": float(np.linalg.norm(half))}


# ----------------------------------------------------------------------------- AllegroHand (config C3)
ALLEGRO_URDF = os.path.join(REF, "assets", "urdf", "kuka_allegro_description", "allegro_touch_sensor.urdf")
ALLEGRO_OUT = os.path.join(os.path.dirname(__file__), "..", "isaacgym-hand-arm_amd", "handarm_hip",
                           "assets", "allegro_hand_scene.json")


def quat_mul_np(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def quat_axis_angle(axis, angle):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    return np.concatenate([a * math.sin(angle / 2), [math.cos(angle / 2)]])


def urdf_joint_friction(j):
    """<dynamics friction> of a URDF joint (0 without one): the DOF friction Isaac Gym loads from the URDF."""
    dyn = j.find("dynamics")
    return float(dyn.get("friction", 0.0)) if dyn is not None else 0.0


def build_collapsed(urdf, dof_props, base_pos, base_quat):
    """A URDF loaded with fix_base_link + collapse_fixed_joints (fixed children merged into their parent
    body, which keeps the parent's frame). Mass properties come from the URDF inertials (no
    override_com/inertia), combined with the parallel-axis rule when bodies merge. dof_props(name) gives
    the drive settings of a joint. Mesh paths resolve against the URDF's directory, its parent, then the
    asset root (the order Isaac Gym's URDF importer tries)."""
    asset_root = os.path.join(REF, "assets")
    root = ET.parse(urdf).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    parent_joint = {j.find("child").get("link"): j for j in root.findall("joint")}
    children = {}
    for j in root.findall("joint"):
        children.setdefault(j.find("parent").get("link"), []).append(j.find("child").get("link"))

    def T_of(j):
        o, R = parse_origin(j.find("origin"))
        T = np.eye(4)
        T[:3, :3], T[:3, 3] = R, o
        return T
    # body of each link (collapse fixed joints) and the link frame in its body frame
    body_of, T_in_body = {}, {}
    rootname = [n for n in links if n not in parent_joint][0]

    def visit(n, body, T):
        body_of[n], T_in_body[n] = body, T
        for c in children.get(n, []):
            j = parent_joint[c]
            if j.get("type") == "fixed":
                visit(c, body, T @ T_of(j))
            else:
                visit(c, c, np.eye(4))
    visit(rootname, rootname, np.eye(4))
    bodies = []

    def dfs(b):
        bodies.append(b)
        kids = sorted({c for n in links if body_of[n] == b for c in children.get(n, [])
                       if parent_joint[c].get("type") != "fixed"})
        for c in kids:
            dfs(c)
    dfs(rootname)
    bidx = {b: i for i, b in enumerate(bodies)}
    out_links, dofs, hulls = [], [], []
    for b in bodies:
        rec = {"name": b, "parent": -1, "joint": None, "type": "fixed", "origin_pos": [0, 0, 0],
               "origin_quat": [0, 0, 0, 1], "axis": [0, 0, 1], "dof": -1}
        j = parent_joint.get(b)
        if j is not None:
            plink = j.find("parent").get("link")
            T = T_in_body[plink] @ T_of(j)
            rec.update(parent=bidx[body_of[plink]], joint=j.get("name"), type=j.get("type"),
                       origin_pos=T[:3, 3].tolist(), origin_quat=matrix_to_quat(T[:3, :3]).tolist())
            a = np.array([float(t) for t in j.find("axis").get("xyz").split()])
            rec["axis"] = (a / np.linalg.norm(a)).tolist()
            lim = j.find("limit")
            rec["dof"] = len(dofs)
            d = {"name": j.get("name"), "link": bidx[b], "lower": float(lim.get("lower")),
                 "upper": float(lim.get("upper")), "velocity": float(lim.get("velocity"))}
            d["friction"] = urdf_joint_friction(j)
            d.update(dof_props(j.get("name")))
            dofs.append(d)
        mass, mc, Isum = 0.0, np.zeros(3), np.zeros((3, 3))
        parts = []
        for n in links:
            if body_of[n] != b:
                continue
            T = T_in_body[n]
            el = links[n]
            inn = el.find("inertial")
            if inn is not None:
                o, R = parse_origin(inn.find("origin"))
                m_ = float(inn.find("mass").get("value"))
                ie = inn.find("inertia")
                I = np.array([[float(ie.get("ixx")), float(ie.get("ixy")), float(ie.get("ixz"))],
                              [float(ie.get("ixy")), float(ie.get("iyy")), float(ie.get("iyz"))],
                              [float(ie.get("ixz")), float(ie.get("iyz")), float(ie.get("izz"))]])
                Rb = T[:3, :3] @ R
                parts.append((m_, T[:3, :3] @ o + T[:3, 3], Rb @ I @ Rb.T))
            for c in el.findall("collision"):
                g = c.find("geometry/mesh")
                if g is None:
                    continue
                fn = g.get("filename")
                for base in (os.path.dirname(urdf), os.path.dirname(os.path.dirname(urdf)), asset_root):
                    path = os.path.join(base, fn)
                    if os.path.exists(path):
                        break
                v, _ = load_mesh(path, [float(t) for t in g.get("scale", "1 1 1").split()])
                o, R = parse_origin(c.find("origin"))
                v = (v @ R.T + o) @ T[:3, :3].T + T[:3, 3]
                h = hull_record(v, MAX_LINK_VERTS)
                h.update(owner="link", index=bidx[b])
                hulls.append(h)
        for m_, c_, _ in parts:
            mass += m_
            mc += m_ * c_
        com = mc / mass if mass > 0 else np.zeros(3)
        for m_, c_, I_ in parts:
            d = c_ - com
            Isum += I_ + m_ * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        rec.update(mass=float(mass), com=com.tolist(), inertia=Isum.reshape(-1).tolist())
        out_links.append(rec)
    robot = {"links": out_links, "dofs": dofs, "base_pos": list(base_pos), "base_quat": list(base_quat)}
    return robot, hulls


def build_allegro():
    """allegro_touch_sensor.urdf loaded like tasks/allegro_hand.py:232-268: fix_base_link,
    collapse_fixed_joints, disable_gravity, DOF_MODE_POS with stiffness 3, damping 0.1, effort 0.5,
    armature 0.001 (:264-268)."""
    # hand_start_pose (allegro_hand.py:284-286): p = (0, 0, 0.5), r = Qy(pi) * Qx(0.47 pi) * Qz(0.25 pi)
    q = quat_mul_np(quat_mul_np(quat_axis_angle([0, 1, 0], math.pi), quat_axis_angle([1, 0, 0], 0.47 * math.pi)),
                    quat_axis_angle([0, 0, 1], 0.25 * math.pi))
    return build_collapsed(ALLEGRO_URDF, lambda name: {"effort": 0.5, "kp": 3.0, "kd": 0.1, "armature": 0.001,
                                                       "friction": 0.01},     # allegro_hand.py:264-268
                           [0.0, 0.0, 0.5], q.tolist())


def build_cube(size=0.065, density=400.0):
    """cube_multicolor_allegro.urdf: box 0.065, density 400 (the URDF gives no mass)."""
    half = [size / 2] * 3
    mass = density * size ** 3
    I = mass / 6.0 * size ** 2
    return {"name": "cube_multicolor_allegro", "mass": mass, "com": [0, 0, 0],
            "inertia": [I, 0, 0, 0, I, 0, 0, 0, I], "hull": box_hull(half)}


def build_egg(density=1000.0):
    """mjcf/open_ai_assets/hand/egg.xml: ellipsoid, semi-axes 0.03 x 0.03 x 0.04 (the object geom; MJCF default density
    1000) as a 32-vertex hull: the two tips and five rings (5, 6, 8, 6, 5 points, one on the equator), scaled about
    the centre so that the hull's volume is the ellipsoid's (the mass and inertia are the ellipsoid's; round 6: the
    inscribed hull without an equator ring was about 10% narrower than the ellipsoid at the equator)."""
    from scipy.spatial import ConvexHull
    a, b, c = 0.03, 0.03, 0.04
    pts = [[0.0, 0.0, c], [0.0, 0.0, -c]]
    for k, (zf, n) in enumerate(((-0.8, 5), (-0.45, 6), (0.0, 8), (0.45, 6), (0.8, 5))):
        for j in range(n):
            t = 2 * math.pi * (j + 0.5 * k) / n
            r = math.sqrt(1 - zf * zf)
            pts.append([a * r * math.cos(t), b * r * math.sin(t), c * zf])
    mass = density * 4.0 / 3.0 * math.pi * a * b * c
    pts = np.array(pts) * (4.0 / 3.0 * math.pi * a * b * c / ConvexHull(np.array(pts)).volume) ** (1.0 / 3.0)
    I = [mass / 5 * (b * b + c * c), mass / 5 * (a * a + c * c), mass / 5 * (a * a + b * b)]
    return {"name": "egg", "mass": mass, "com": [0, 0, 0], "inertia": [I[0], 0, 0, 0, I[1], 0, 0, 0, I[2]],
            "hull": hull_record(np.array(pts), 32)}


def build_pen(density=1000.0):
    """mjcf/open_ai_assets/hand/pen.xml: capsule, radius 0.008, half-length 0.1 along z (MJCF default density 1000) as
    a 32-vertex hull (two 8-point rings at the ends of the cylinder, two 7-point rings on the caps, the tips); mass and
    inertia of the capsule."""
    r, hl = 0.008, 0.1
    pts = [[0.0, 0.0, hl + r], [0.0, 0.0, -hl - r]]
    for z, rr, n, off in ((hl, r, 8, 0.0), (-hl, r, 8, 0.0), (hl + 0.7 * r, r * math.sqrt(1 - 0.49), 7, 0.5),
                          (-hl - 0.7 * r, r * math.sqrt(1 - 0.49), 7, 0.5)):
        for j in range(n):
            t = 2 * math.pi * (j + off) / n
            pts.append([rr * math.cos(t), rr * math.sin(t), z])
    h = 2 * hl
    m_cyl = density * math.pi * r * r * h
    m_sph = density * 4.0 / 3.0 * math.pi * r ** 3
    Ixx = m_cyl * (h * h / 12 + r * r / 4) + m_sph * (2 * r * r / 5 + h * h / 4 + 3 * h * r / 8)
    Izz = m_cyl * r * r / 2 + m_sph * 2 * r * r / 5
    return {"name": "pen", "mass": m_cyl + m_sph, "com": [0, 0, 0], "inertia": [Ixx, 0, 0, 0, Ixx, 0, 0, 0, Izz],
            "hull": hull_record(np.array(pts), 32)}


# self-collision of the Allegro actors (ha_model_t v12): every non-adjacent link pair ("exclude" can drop pairs). The
# lists are empty: at each task's reset pose (AllegroHand: zero DOF positions clamped to the limits; AllegroKuka: the
# arm's desired pose, fingers 0) no pair of cooked hulls is within the contact offset, so the hand starts without
# standing self contacts (tests/test_self_collision.py::test_no_self_contacts_at_the_reset_poses)
ALLEGRO_SELF_COLLISION = {"exclude": []}
KUKA_SELF_COLLISION = {"exclude": []}


def main_allegro():
    robot, link_hulls = build_allegro()
    L = len(robot["links"])
    # objectType block / egg / pen (allegro_hand.py:82-97): pool entries 0 / 1 / 2
    scene = {"robot": robot, "link_hulls": link_hulls, "objects": [build_cube(), build_egg(), build_pen()], "table": None,
             "objects_per_env": 1,
             # actors hand 0, object 1, goal 2; bodies hand links, object, goal (allegro_hand.py:330-357)
             "layout": {"n_actors": 3, "actor_robot": 0, "actor_object0": 1, "actor_goal": 2, "actor_table": -1,
                        "n_bodies": L + 2, "body_robot0": 0, "body_object0": L, "body_goal": L + 1,
                        "body_table": -1},
             # hand actor with collision filter -1 (allegro_hand.py:334-335): its links collide with each other
             "self_collision": ALLEGRO_SELF_COLLISION,
             "generator": "tools/build_model.py --allegro (reference assets @ /root/reference/assets/urdf)"}
    with open(ALLEGRO_OUT, "w") as f:
        json.dump(scene, f, indent=None, separators=(",", ":"))
    print(f"allegro: links={L} dofs={len(robot['dofs'])} hulls={len(link_hulls)} "
          f"dof order={[d['name'] for d in robot['dofs']]} -> {ALLEGRO_OUT}")


# ----------------------------------------------------------------------------- AllegroKuka (config C2)
KUKA_URDF = os.path.join(REF, "assets", "urdf", "kuka_allegro_description", "kuka_allegro_touch_sensor.urdf")
KUKA_OUT = os.path.join(os.path.dirname(__file__), "..", "isaacgym-hand-arm_amd", "handarm_hip",
                        "assets", "kuka_allegro_scene.json")


def kuka_object_dims(small=True, big=True, sticks=True):
    """The procedurally generated cuboid family (allegro_kuka/generate_cuboids.py:37-137) as per-axis
    scales of the 0.05 m base cube, in the order envs receive them: file names sorted, then shuffled
    with numpy default_rng(42) (allegro_kuka_base.py:411-428, 485-512). Files of the four generators
    share one directory, so equal names overwrite each other exactly as on disk. The flags are the config's
    withSmallCuboids / withBigCuboids / withSticks (AllegroKuka.yaml:77-79; throw: small only, env/throw.yaml)."""
    files = set()

    def gen(scales, min_volume, max_volume, filters):
        idx = 0
        for x in scales:
            for y in scales:
                for z in scales:
                    volume = x * y * z / (100 * 100 * 100)
                    if volume > max_volume or volume < min_volume:
                        continue
                    cs = sorted([x, y, z])
                    if any(f(cs) for f in filters):
                        continue
                    files.add(f"{idx:03d}_cube_{x}_{y}_{z}.urdf")
                    idx += 1

    def thin(s):
        s = sorted(s)
        return s[0] * 3 <= s[1]

    def non_elongated(s):
        s = sorted(s)
        return s[2] <= s[0] * 3 or s[2] <= s[1] * 3
    gen([100], 1.0, 1.0, [])                                                          # default cube
    if small:
        gen([100, 50, 66, 75, 90, 110, 125, 150, 175, 200, 250, 300], 1.0, 2.5, [])   # withSmallCuboids
    if big:
        gen([100, 125, 150, 200, 250, 300, 350], 2.5, 15.0, [thin])                   # withBigCuboids
    if sticks:
        gen([100, 50, 75, 200, 300, 400, 500, 600], 2.5, 6.0, [thin, non_elongated])  # withSticks
    names = sorted(files)
    scales = [[float(t) / 100 for t in os.path.splitext(f)[0].split("_")[2:]] for f in names]
    pairs = list(zip(names, scales))
    np.random.default_rng(42).shuffle(pairs)
    return [p[1] for p in pairs]


def build_kuka_allegro():
    """kuka_allegro_touch_sensor.urdf loaded like allegro_kuka_base.py:559-575 (fix_base_link,
    collapse_fixed_joints, disable_gravity, DOF_MODE_POS), DOF props from populate_dof_properties
    (allegro_kuka_utils.py:66-83) with AllegroKuka.yaml:56-71: stiffness 40 / damping 5 for all DOFs,
    effort 300 (arm) / 0.35 (hand), armature 0. Arm pose (0, 0.8, 0), identity (:608-610)."""
    def props(name):
        arm = name.startswith("iiwa7_joint")
        return {"effort": 300.0 if arm else 0.35, "kp": 40.0, "kd": 5.0, "armature": 0.0}
    return build_collapsed(KUKA_URDF, props, [0.0, 0.8, 0.0], [0.0, 0.0, 0.0, 1.0])


def build_box_object(size=0.05, density=400.0):
    """cube_multicolor_allegro.urdf.template at scale 1: box of objectBaseSize 0.05 m, density 400
    (the template gives no mass). Per-env dimensions scale this hull and its mass properties."""
    half = [size / 2] * 3
    mass = density * size ** 3
    I = mass / 6.0 * size ** 2
    return {"name": "cuboid_base", "mass": mass, "com": [0, 0, 0],
            "inertia": [I, 0, 0, 0, I, 0, 0, 0, I], "hull": box_hull(half)}


def main_kuka():
    robot, link_hulls = build_kuka_allegro()
    L = len(robot["links"])
    # table_narrow.urdf: box 0.475 x 0.4 x 0.3 at allegro_pose + (0, -0.8, 0.38) (allegro_kuka_base.py:622-628)
    table = {"pos": [0.0, 0.0, 0.38], "quat": [0, 0, 0, 1], "half_extents": [0.2375, 0.2, 0.15]}
    table["hull"] = box_hull(table["half_extents"])
    scene = {"robot": robot, "link_hulls": link_hulls, "objects": [build_box_object()], "table": table,
             "objects_per_env": 1, "object_dims": kuka_object_dims(),
             # actors allegro 0, object 1, table 2, goal 3 (allegro_kuka_base.py:660-730); bodies likewise
             "layout": {"n_actors": 4, "actor_robot": 0, "actor_object0": 1, "actor_goal": 3, "actor_table": 2,
                        "n_bodies": L + 3, "body_robot0": 0, "body_object0": L, "body_goal": L + 2,
                        "body_table": L + 1},
             # arm + hand actor with collision filter -1 (allegro_kuka_base.py:664): its links collide with each other
             "self_collision": KUKA_SELF_COLLISION,
             "generator": "tools/build_model.py --kuka (reference assets @ /root/reference/assets/urdf)"}
    with open(KUKA_OUT, "w") as f:
        json.dump(scene, f, indent=None, separators=(",", ":"))
    print(f"kuka_allegro: links={L} dofs={len(robot['dofs'])} hulls={len(link_hulls)} "
          f"objects dims={len(scene['object_dims'])} bodies={[l['name'] for l in robot['links']]} "
          f"dof order={[d['name'] for d in robot['dofs']]} -> {KUKA_OUT} ({os.path.getsize(KUKA_OUT)} B)")


BUCKET_OBJ = os.path.join(REF, "assets", "urdf", "objects", "meshes", "bucket.obj")


def bucket_pieces():
    """bucket.urdf (allegro_kuka_throw.py:51-66; the reference V-HACDs its mesh) as convex pieces in the bucket's
    frame: meshes/bucket.obj is a 12-sided vessel (outer wall from the bottom ring r 0.082 at z 0 to the rim r 0.12
    at z 0.198, inner wall from the floor ring r 0.0705 at z 0.0099 to r 0.1035 at the rim). Pieces: the 12 wall
    sectors (the outer bottom, rim and inner rim vertices at two neighbouring angles, with the floor ring's vertices
    brought down to the bottom plane z 0, so a sector's underside is the flat bottom and no sector face points down
    into the bucket's inside: an object on the floor next to the wall is pushed up and inward, never down) and the
    floor: the floor ring's 12-gon prism from the floor top (z 0.0099) down to 3 cm under the bottom, so that a
    cuboid falling in at up to ~5 m/s cannot cross the slab's mid-plane within one substep (a 1 cm slab let the
    fastest drops tunnel). Each piece's hull is stored about its box centre, with the box as the static's half
    extents (the broad phase's sphere-near-box test needs the box to contain the hull)."""
    v, _ = load_obj(BUCKET_OBJ)
    ctr = np.array([0.0, v[:, 1].min() + 0.5 * (v[:, 1].max() - v[:, 1].min()), 0.0])
    ctr[0] = 0.5 * (v[:, 0].min() + v[:, 0].max())
    rel = v - ctr
    r = np.hypot(rel[:, 0], rel[:, 1])
    ang = np.round(np.degrees(np.arctan2(rel[:, 1], rel[:, 0])) / 30.0).astype(int) % 12
    zlo, zhi = v[:, 2].min(), v[:, 2].max()
    rings = {}
    for name, sel in (("outer_bottom", np.isclose(v[:, 2], zlo, atol=1e-4)),
                      ("floor", (v[:, 2] > zlo + 1e-3) & (v[:, 2] < zhi - 1e-3)),
                      ("rim_outer", np.isclose(v[:, 2], zhi, atol=1e-4) & (r > 0.11)),
                      ("rim_inner", np.isclose(v[:, 2], zhi, atol=1e-4) & (r < 0.11))):
        idx = np.nonzero(sel)[0]
        assert len(idx) == 12, (name, len(idx))
        ring = np.zeros((12, 3))
        ring[ang[idx]] = v[idx]
        assert len(set(ang[idx])) == 12, name
        rings[name] = ring
    under = rings["floor"].copy()
    under[:, 2] = zlo - 0.03
    clouds = [np.concatenate([rings["floor"], under])]
    base = rings["floor"].copy()
    base[:, 2] = rings["outer_bottom"][:, 2]
    wall = dict(rings, floor=base)
    for i in range(12):
        j = (i + 1) % 12
        clouds.append(np.stack([wall[n][k] for n in wall for k in (i, j)]))
    pieces = []
    for pts in clouds:
        lo, hi = pts.min(0), pts.max(0)
        c = 0.5 * (lo + hi)
        rec = hull_record(pts - c, MAX_PIECE_VERTS)
        assert len(rec["verts"]) == len(pts), "every ring vertex is a hull vertex"
        half = (0.5 * (hi - lo) * (1 + 1e-5) + 1e-6).tolist()
        pieces.append({"pos": c.tolist(), "quat": [0.0, 0.0, 0.0, 1.0], "half_extents": half, "hull": rec})
    return pieces


def main_throw():
    """Adds the AllegroKuka throw subtask's data to the committed Kuka scene without rebuilding it: the bucket's
    convex pieces as statics carried by the actor in the goal slot (allegro_kuka_throw.py:68-82: the bucket is the
    actor created after the table, actor 3 / body 26 like reorientation's goal), and the throw object family
    (env/throw.yaml: withSmallCuboids only)."""
    with open(KUKA_OUT) as f:
        scene = json.load(f)
    pieces = bucket_pieces()
    scene["posed_statics"] = {"bucket": {"actor": "actor_goal", "pieces": pieces,
                                         "source": "urdf/objects/bucket.urdf (meshes/bucket.obj), floor + 12 sectors"}}
    scene["object_dims_throw"] = kuka_object_dims(small=True, big=False, sticks=False)
    with open(KUKA_OUT, "w") as f:
        json.dump(scene, f, indent=None, separators=(",", ":"))
    print(f"throw: bucket {len(pieces)} pieces, verts {[len(p['hull']['verts']) for p in pieces]}, "
          f"object dims {len(scene['object_dims_throw'])} -> {KUKA_OUT}")


def main():
    robot, link_hulls = build_robot()
    objects = [build_object(n) for n in YCB_POOL
               if os.path.exists(os.path.join(ASSETS, "object_sets", "urdf", "ycb", n + ".urdf"))]
    table = {"pos": [0.2925, 0.38, TABLE_HEIGHT / 2], "quat": [0, 0, 0, 1],    # multi_object.py:536,628
             "half_extents": [0.375, 0.55, TABLE_HEIGHT / 2]}
    table["hull"] = box_hull(table["half_extents"])
    scene = {"robot": robot, "link_hulls": link_hulls, "objects": objects, "table": table,
             "goal_radius": 0.02,
             "generator": "tools/build_model.py (reference assets @ /root/reference/assets/hand_arm)"}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(scene, f, indent=None, separators=(",", ":"))
    nm = sum(1 for l in robot["links"] if l["mass"] > 0)
    print(f"links={len(robot['links'])} dofs={len(robot['dofs'])} massive={nm} link_hulls={len(link_hulls)} "
          f"objects={[o['name'] for o in objects]} -> {OUT} ({os.path.getsize(OUT)} B)")


# ----------------------------------------------------------------------------- bin-picking (config C5)
BIN_OUT = os.path.join(os.path.dirname(__file__), "..", "isaacgym-hand-arm_amd", "handarm_hip", "assets",
                       "ur5sih_bin_scene.json")
BIN_POS = (0.28, 0.53, 0.0)                    # Ur5SihMultiObject.yaml bin.pos (z += table_height, multi_object.py:506)
BIN_QUAT = (0.0, 0.0, -0.707, 0.707)           # bin.quat (gymapi.Quat, normalised by PhysX)
HARD_BIN_EXTENT = [[-0.18, -0.2975, -0.19], [0.18, 0.2975, 0.065]]   # assets/hand_arm/hard_bin/bin_info.yaml


def qrot_np(q, v):
    x, y, z, w = q
    u = np.array([x, y, z])
    v = np.asarray(v, float)
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def tote_boxes():
    """Box decomposition of hard_bin/assets/tote.obj (the reference V-HACDs it, multi_object.py:497-504; no
    V-HACD here, so the tote becomes five boxes): a 1 cm floor under the inner floor (mesh z 0.005) and four
    1 cm walls whose inner faces run from the inner bottom corner (outer bottom |x| 0.286, |y| 0.163, minus the
    wall) to the inner top edge of bin_info.yaml (|x| 0.2975, |y| 0.18 in the mesh frame) at the rim (z 0.1955),
    i.e. tilted outward like the tote. Poses in the bin link frame (collision origin z -0.19, bin.urdf)."""
    t, zb, zt, zo = 0.01, 0.005, 0.1955, -0.19
    boxes = [([0.0, 0.0, zb - t / 2 + zo], [0, 0, 0, 1], [0.286, 0.163, t / 2])]
    for axis, bot, top, length in ((0, 0.286 - t, 0.2975, 0.187), (1, 0.163 - t, 0.18, 0.308)):
        dz = zt - zb
        ang = math.atan2(top - bot, dz)
        half_h = 0.5 * math.hypot(top - bot, dz)
        for sgn in (1.0, -1.0):
            up = np.zeros(3)
            up[axis] = sgn * math.sin(ang)
            up[2] = math.cos(ang)
            out = np.zeros(3)                          # outward wall normal (perpendicular to up, in the plane)
            out[axis] = sgn * math.cos(ang)
            out[2] = -math.sin(ang)
            inner_mid = np.zeros(3)
            inner_mid[axis] = sgn * 0.5 * (bot + top)
            inner_mid[2] = 0.5 * (zb + zt)
            c = inner_mid + out * (t / 2)
            c[2] += zo
            # local z -> up: rotation about the other horizontal axis
            rot_axis = [0.0, 1.0, 0.0] if axis == 0 else [1.0, 0.0, 0.0]
            a = sgn * ang if axis == 0 else -sgn * ang
            q = quat_axis_angle(rot_axis, a)
            assert np.allclose(qrot_np(q, [0, 0, 1]), up, atol=1e-9)
            half = [t / 2, length, half_h] if axis == 0 else [length, t / 2, half_h]
            boxes.append((c.tolist(), q.tolist(), half))
    return boxes


def table_with_hole_boxes(height, hole_x, hole_y, x_range=(-0.095, 0.655), y_range=(-0.17, 0.93)):
    """generate_table_with_hole (utils/urdf.py:125-210) as four boxes in the table frame (link origins of its
    fixed joints); siblings in link-name order like the robot (back, front, left, right wall)."""
    x0, x1 = x_range
    y0, y1 = y_range
    walls = {
        "front_wall": ([x0 + 0.5 * (hole_x[0] - x0), y0 + 0.5 * (y1 - y0), 0.0], [hole_x[0] - x0, y1 - y0, height]),
        "back_wall": ([(hole_x[1] + x1) / 2, y0 + 0.5 * (y1 - y0), 0.0], [x1 - hole_x[1], y1 - y0, height]),
        "right_wall": ([x0 + 0.5 * (x1 - x0), y0 + 0.5 * (hole_y[0] - y0), 0.0], [x1 - x0, hole_y[0] - y0, height]),
        "left_wall": ([x0 + 0.5 * (x1 - x0), (hole_y[1] + y1) / 2, 0.0], [x1 - x0, y1 - hole_y[1], height]),
    }
    return [(n, walls[n][0], [0.5 * v for v in walls[n][1]]) for n in sorted(walls)]


def main_bin(n_objects=8):
    """Ur5SihMultiObject with bin.asset hard_bin (BASELINE config 5): table with a hole
    under the bin (multi_object.py:535-540), the bin actor (:497-507, 635-637) and n_objects YCB objects per
    env. Actors: goal 0, robot 1, table 2, bin 3, objects 4.. (creation order, multi_object.py:579-644).
    Bodies: goal, 29 robot links, table base_link + 4 walls, bin, objects."""
    base = json.load(open(OUT))
    L = len(base["robot"]["links"])
    ext = HARD_BIN_EXTENT
    hole_x = (ext[0][0] + BIN_POS[0], ext[1][0] + BIN_POS[0])
    hole_y = (ext[0][1] + BIN_POS[1], ext[1][1] + BIN_POS[1])
    table_pose = [0.0, 0.0, TABLE_HEIGHT / 2, 0, 0, 0, 1]              # multi_object.py:630
    qn = np.asarray(BIN_QUAT, float)
    qn = qn / np.linalg.norm(qn)
    bin_pos = np.array([BIN_POS[0], BIN_POS[1], BIN_POS[2] + TABLE_HEIGHT])
    statics, fixed = [], [table_pose]
    for name, c, half in table_with_hole_boxes(TABLE_HEIGHT, hole_x, hole_y):
        pos = [c[0], c[1], c[2] + TABLE_HEIGHT / 2]
        statics.append({"name": "table_" + name, "pos": pos, "quat": [0, 0, 0, 1], "half_extents": half,
                        "hull": box_hull(half)})
        fixed.append(pos + [0, 0, 0, 1])
    for k, (c, q, half) in enumerate(tote_boxes()):
        pos = (bin_pos + qrot_np(qn, c)).tolist()
        quat = quat_mul_np(qn, q)
        statics.append({"name": f"bin_{k}", "pos": pos, "quat": (quat / np.linalg.norm(quat)).tolist(),
                        "half_extents": half, "hull": box_hull(half)})
    fixed.append(bin_pos.tolist() + qn.tolist())
    n_obj = n_objects
    body_table = 1 + L
    scene = {
        "extends": os.path.basename(OUT), "table": None, "statics": statics, "objects_per_env": n_obj,
        "layout": {"n_actors": 4 + n_obj, "actor_robot": 1, "actor_object0": 4, "actor_goal": 0, "actor_table": 2,
                   "n_bodies": 1 + L + 5 + 1 + n_obj, "body_robot0": 1, "body_object0": body_table + 6, "body_goal": 0,
                   "body_table": body_table},
        "fixed_bodies": fixed, "body_fixed0": body_table,
        "static_actors": [{"actor": 2, "pose": table_pose}, {"actor": 3, "pose": bin_pos.tolist() + qn.tolist()}],
        "bin_extent": [[hole_x[0], hole_y[0], ext[0][2] + TABLE_HEIGHT + BIN_POS[2]],    # objects_in_bin
                       [hole_x[1], hole_y[1], ext[1][2] + TABLE_HEIGHT + BIN_POS[2]]],    # (multi_object.py:705-718)
        "generator": "tools/build_model.py --bin (reference assets @ /root/reference/assets/hand_arm)",
    }
    with open(BIN_OUT, "w") as f:
        json.dump(scene, f, indent=1)
    print(f"bin scene: {len(statics)} static boxes, {len(fixed)} fixed bodies, {n_obj} objects/env, "
          f"bin extent {scene['bin_extent']} -> {BIN_OUT}")


# ----------------------------------------------------------------------------- synthetic point clouds (§8f #2)
PC_OUT = os.path.join(os.path.dirname(__file__), "..", "isaacgym-hand-arm_amd", "handarm_hip", "assets",
                      "ur5sih_pointclouds.npz")
PC_MAX_POINTS = 128                  # Ur5SihMultiObject.yaml pointclouds.max_num_points
ROBOT_PC_DENSITY = 1500.0            # samples per m^2 (ur5sih.py:90-91)
# links whose collision meshes the reference samples: every link with a collision mesh in URDF order minus the
# six UR5 arm links (ur5sih.py:70-88, use_reduced_robot)
ROBOT_PC_SKIP = {"shoulder_link", "upper_arm_link", "forearm_link", "wrist_1_link", "wrist_2_link", "wrist_3_link"}


def sample_surface(v, f, count, rng):
    """trimesh.sample.sample_surface (trimesh==3.23.5, setup.py:28; absent here) restated: faces drawn with
    probability proportional to area (searchsorted on the cumulative area), then a uniform point in the
    triangle from two uniforms folded back into the triangle when their sum exceeds 1."""
    tri = v[f]
    area = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1)
    cum = np.cumsum(area)
    face = np.searchsorted(cum, rng.random(count) * cum[-1])
    origins = tri[face, 0]
    vecs = tri[face, 1:] - origins[:, None]
    lengths = rng.random((count, 2, 1))
    fold = lengths.sum(axis=1).reshape(-1) > 1.0
    lengths[fold] -= 1.0
    lengths = np.abs(lengths)
    return (vecs * lengths).sum(axis=1) + origins, float(area.sum())


def link_collision_mesh(link_el, base_dir, colls=None):
    """urdfpy Link.collision_mesh: the link's collision meshes in the link frame, concatenated."""
    vs, fs, n = [], [], 0
    for c in (colls if colls is not None else link_el.findall("collision")):
        g = c.find("geometry/mesh")
        if g is None:
            continue
        path = os.path.join(base_dir, g.get("filename"))
        if not os.path.exists(path):
            return None
        v, fa = load_mesh(path, [float(t) for t in g.get("scale", "1 1 1").split()])
        o, R = parse_origin(c.find("origin"))
        vs.append(v @ R.T + o)
        fs.append(fa + n)
        n += len(v)
    if not vs:
        return None
    return np.concatenate(vs), np.concatenate(fs)


def main_pointclouds(seed=0):
    """Surface samples of the object pool and the reduced robot (multi_object.py:774-790, ur5sih.py:347-359).
    Objects: PC_MAX_POINTS samples and the mesh area per pool object; the runtime takes the first
    int(average_num_points * area / mean_area) of them for the configured pool ('area' sample mode) and pads
    to max_num_points. Robot: int(1500 * area) samples per link in the link frame, with the link's index."""
    rng = np.random.default_rng(seed)
    scene = json.load(open(OUT))
    names, samples, areas = [], [], []
    for rec in scene["objects"]:
        urdf = os.path.join(ASSETS, "object_sets", "urdf", "ycb", rec["name"] + ".urdf")
        link = ET.parse(urdf).getroot().find("link")
        v, f = link_collision_mesh(link, os.path.dirname(urdf))
        pts, area = sample_surface(v, f, PC_MAX_POINTS, rng)
        names.append(rec["name"])
        samples.append(pts)
        areas.append(area)
    base_dir = os.path.dirname(ROBOT_URDF)
    root = ET.parse(ROBOT_URDF).getroot()
    link_index = {l["name"]: i for i, l in enumerate(scene["robot"]["links"])}
    palm_colls = [l for l in ET.parse(PALM_URDF).getroot().findall("link") if l.get("name") == "palm"][0]
    r_pts, r_link, r_names, r_counts = [], [], [], []
    for el in root.findall("link"):                    # URDF document order (urdfpy URDF.links)
        n = el.get("name")
        if n in ROBOT_PC_SKIP or not el.findall("collision"):
            continue
        mesh = link_collision_mesh(el, base_dir, palm_colls.findall("collision") if n == "palm" else None)
        if mesh is None:
            continue
        tri = mesh[0][mesh[1]]
        area = float(0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1).sum())
        count = int(ROBOT_PC_DENSITY * area)
        pts, _ = sample_surface(mesh[0], mesh[1], count, rng)
        r_pts.append(pts)
        r_link += [link_index[n]] * count
        r_names.append(n)
        r_counts.append(count)
    np.savez_compressed(PC_OUT, object_names=np.array(names), object_samples=np.array(samples, np.float32),
                        object_areas=np.array(areas, np.float64), robot_samples=np.concatenate(r_pts).astype(np.float32),
                        robot_link=np.array(r_link, np.int32), robot_link_names=np.array(r_names),
                        robot_link_counts=np.array(r_counts, np.int32))
    print(f"point clouds: {len(names)} objects x {PC_MAX_POINTS} samples, robot {sum(r_counts)} samples over "
          f"{list(zip(r_names, r_counts))} -> {PC_OUT}")


def main_concave():
    """Adds the CONCAVE_POOL objects to the committed Ur5Sih scene (after the 16-object pool, whose entries stay
    untouched; the bin scene extends it) and their point-cloud samples to the committed npz (a generator seeded per
    object name, so the existing samples - which the point-cloud goldens were made with - do not change)."""
    import zlib
    scene = json.load(open(OUT))
    have = {o["name"] for o in scene["objects"]}
    added = []
    for name in CONCAVE_POOL:
        if name in have:
            continue
        rec = build_object(name)
        scene["objects"].append(rec)
        added.append((name, len(rec["hulls"]), [len(h["verts"]) for h in rec["hulls"]]))
    with open(OUT, "w") as f:
        json.dump(scene, f, indent=None, separators=(",", ":"))
    d = dict(np.load(PC_OUT))
    names = [str(n) for n in d["object_names"]]
    samples, areas = list(d["object_samples"]), list(d["object_areas"])
    for rec in scene["objects"]:
        if rec["name"] in names:
            continue
        urdf = os.path.join(ASSETS, "object_sets", "urdf", "ycb", rec["name"] + ".urdf")
        link = ET.parse(urdf).getroot().find("link")
        v, f = link_collision_mesh(link, os.path.dirname(urdf))
        pts, area = sample_surface(v, f, PC_MAX_POINTS, np.random.default_rng(zlib.crc32(rec["name"].encode())))
        names.append(rec["name"])
        samples.append(pts.astype(np.float32))
        areas.append(area)
    d["object_names"], d["object_samples"], d["object_areas"] = np.array(names), np.array(samples, np.float32), \
        np.array(areas, np.float64)
    np.savez_compressed(PC_OUT, **d)
    print(f"concave pool: added {added} -> {OUT}; point clouds for {len(names)} objects -> {PC_OUT}")


def main_dof_friction():
    """Adds the DOF friction to the committed Allegro scenes without rebuilding their hulls: AllegroHand 0.01
    (allegro_hand.py:267), AllegroKuka the URDF's <dynamics friction> (AllegroKuka.yaml:58 dofFriction -1 keeps
    the URDF values, allegro_kuka_utils.py:79-80)."""
    root = ET.parse(KUKA_URDF).getroot()
    fr = {j.get("name"): urdf_joint_friction(j) for j in root.findall("joint")}
    for path, get in ((ALLEGRO_OUT, lambda n: 0.01), (KUKA_OUT, lambda n: fr[n])):
        with open(path) as f:
            scene = json.load(f)
        for d in scene["robot"]["dofs"]:
            d["friction"] = get(d["name"])
        with open(path, "w") as f:
            json.dump(scene, f, indent=None, separators=(",", ":"))
        print(path, [d["friction"] for d in scene["robot"]["dofs"]])


if __name__ == "__main__":
    if "--throw" in sys.argv:
        sys.exit(main_throw())
    if "--dof-friction" in sys.argv:
        sys.exit(main_dof_friction())
    if "--pointclouds" in sys.argv:
        sys.exit(main_pointclouds())
    if "--concave" in sys.argv:
        sys.exit(main_concave())
    if "--bin" in sys.argv:
        sys.exit(main_bin())
    if "--allegro" in sys.argv:
        sys.exit(main_allegro())
    sys.exit(main_kuka() if "--kuka" in sys.argv else main())
