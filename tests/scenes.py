"""Seeded synthetic scene states shared by the parity tests and bench.py's CPU-baseline leg.

Layouts are the Isaac Gym tensor layouts of handarm_hip.model.state_spec (host numpy)."""
import numpy as np

RESET_POSE = np.array([0.6985, -1.4106, 1.2932, 0.1174, 0.6983, 1.5708, 0., 0., 0., 0., 0., 0., 0., 0., -1.571,
                       0., 0.], np.float32)


def rand_quat(rng, shape):
    q = rng.standard_normal(shape + (4,)).astype(np.float32)
    return (q / np.linalg.norm(q, axis=-1, keepdims=True)).astype(np.float32)


def fill_scene(st, num_envs, seed=0, near_hand=0.3, n_obj=3, fingertip_pos=None):
    """Robot near its reset pose, objects resting-ish on the table, some dropped into the hand."""
    rng = np.random.default_rng(seed)
    N, A = num_envs, 3 + n_obj
    rs = st["root_state"].reshape(N, A, 13)
    rs[:] = 0
    rs[..., 6] = 1.0
    rs[:, 0, 0:3] = [0.28, 0.58, 0.8]
    rs[:, 1, 0:3] = [0.0, 0.0, 0.5]
    rs[:, 2, 0:3] = [0.2925, 0.38, 0.25]
    for o in range(n_obj):
        rs[:, 3 + o, 0] = 0.08 + 0.17 * o + rng.uniform(-0.03, 0.03, N)
        rs[:, 3 + o, 1] = rng.uniform(0.45, 0.75, N)
        rs[:, 3 + o, 2] = rng.uniform(0.56, 0.62, N)
        rs[:, 3 + o, 3:7] = rand_quat(rng, (N,))
        rs[:, 3 + o, 7:10] = rng.uniform(-0.2, 0.2, (N, 3))
        rs[:, 3 + o, 10:13] = rng.uniform(-1.0, 1.0, (N, 3))
    if fingertip_pos is not None:
        sel = rng.random(N) < near_hand
        rs[sel, 3, 0:3] = fingertip_pos[sel] + rng.uniform(-0.02, 0.02, (int(sel.sum()), 3))
    ds = st["dof_state"].reshape(N, 17, 2)
    ds[..., 0] = RESET_POSE + rng.uniform(-0.05, 0.05, (N, 17)).astype(np.float32)
    ds[..., 0, ] = np.clip(ds[..., 0], -6, 6)
    ds[:, 6:14, 0] = np.clip(ds[:, 6:14, 0], -1.571, 0.0)
    ds[:, 14, 0] = np.clip(ds[:, 14, 0], -1.571, 0.0)
    ds[:, 15:17, 0] = np.clip(ds[:, 15:17, 0], 0.0, 1.571)
    ds[..., 1] = rng.uniform(-0.3, 0.3, (N, 17))
    st["sim_targets"][:] = RESET_POSE + rng.uniform(-0.3, 0.3, (N, 17)).astype(np.float32)
    st["object_indices"][:] = np.stack([rng.permutation(3) for _ in range(N)])
    st["collision_enabled"][:] = 1
    return st


def fill_allegro_scene(st, num_envs, lower, upper, seed=0, in_hand=1.0):
    """AllegroHand: hand joints inside their limits, the cube resting on / just above the palm
    (object start pose (0, -0.2, 0.56) +- noise, random orientation), random goal orientation."""
    rng = np.random.default_rng(seed)
    N = num_envs
    rs = st["root_state"].reshape(N, 3, 13)
    rs[:] = 0
    rs[..., 6] = 1.0
    rs[:, 1, 0:3] = np.array([0.0, -0.2, 0.56], np.float32) + rng.uniform(-0.01, 0.01, (N, 3))
    lift = rng.random(N) >= in_hand
    rs[lift, 1, 2] += 0.1
    rs[:, 1, 3:7] = rand_quat(rng, (N,))
    rs[:, 1, 7:10] = rng.uniform(-0.1, 0.1, (N, 3))
    rs[:, 1, 10:13] = rng.uniform(-0.5, 0.5, (N, 3))
    rs[:, 2, 0:3] = [-0.2, -0.26, 0.64]
    rs[:, 2, 3:7] = rand_quat(rng, (N,))
    st["goal_state"][:, 0:3] = [0.0, -0.2, 0.52]
    st["goal_state"][:, 3:7] = rs[:, 2, 3:7]
    ds = st["dof_state"].reshape(N, 16, 2)
    ds[..., 0] = lower + (upper - lower) * rng.uniform(0.1, 0.9, (N, 16)).astype(np.float32)
    ds[..., 1] = rng.uniform(-0.5, 0.5, (N, 16))
    st["sim_targets"][:] = lower + (upper - lower) * rng.uniform(0.0, 1.0, (N, 16)).astype(np.float32)
    st["object_indices"][:] = 0
    st["collision_enabled"][:] = 1
    return st


def fill_kuka_scene(st, num_envs, lower, upper, reset_pose, scales, table_pos, seed=0, object_force=0.0):
    """AllegroKuka: arm near its default pose (reset_pose +- 0.1), fingers inside their limits, the cuboid
    (per-env dimensions `scales`) resting on / dropping onto the table top with a random orientation, goal
    somewhere in the target volume, optional random object forces."""
    rng = np.random.default_rng(seed)
    N = num_envs
    rs = st["root_state"].reshape(N, 4, 13)
    rs[:] = 0
    rs[..., 6] = 1.0
    half_z = 0.025 * scales[:, 0, :].max(-1)
    rs[:, 1, 0:2] = rng.uniform(-0.08, 0.08, (N, 2))
    rs[:, 1, 2] = 0.53 + half_z + rng.uniform(0.0, 0.05, N)
    rs[:, 1, 3:7] = rand_quat(rng, (N,))
    rs[:, 1, 7:10] = rng.uniform(-0.1, 0.1, (N, 3))
    rs[:, 1, 10:13] = rng.uniform(-0.5, 0.5, (N, 3))
    rs[:, 2, 0:3] = table_pos
    rs[:, 3, 0:3] = rng.uniform([-0.4, 0.0, 0.68], [0.4, 0.35, 1.05], (N, 3))
    st["goal_state"][:, 0:3] = rs[:, 3, 0:3]
    st["goal_state"][:, 6] = 1.0
    D = len(lower)
    ds = st["dof_state"].reshape(N, D, 2)
    base = np.array(reset_pose[:D], np.float32)
    ds[..., 0] = np.clip(base + rng.uniform(-0.1, 0.1, (N, D)), lower, upper)
    ds[:, 7:, 0] = lower[7:] + (upper[7:] - lower[7:]) * rng.uniform(0.1, 0.9, (N, D - 7)).astype(np.float32)
    ds[..., 1] = rng.uniform(-0.3, 0.3, (N, D))
    st["sim_targets"][:] = np.clip(ds[..., 0] + rng.uniform(-0.2, 0.2, (N, D)), lower, upper)
    st["object_indices"][:] = 0
    st["object_scale"][:] = scales
    st["collision_enabled"][:] = 1
    st["object_force"][:] = object_force * rng.standard_normal((N, 1, 3))
    return st


def bin_pool_ids(rng, n_envs, n_obj=8, pool=16):
    """Per-env object subsets: random.sample of the pool (multi_object.py:569)."""
    return np.stack([rng.permutation(pool)[:n_obj] for _ in range(n_envs)])


def fill_bin_scene(st, num_envs, scene, seed=0, n_obj=8, spread=1.0, pool=16):
    """Bin-picking (BASELINE config 5): the robot near its reset pose and n_obj objects on a 2 x 4 grid inside
    the tote (bin extent of the scene), lower layer touching the floor, upper layer falling onto it, random
    orientations and small velocities. Actor layout of the bin scene: goal 0, robot 1, table 2, bin 3,
    objects 4.."""
    rng = np.random.default_rng(seed)
    N = num_envs
    A = 4 + n_obj
    lo, hi = np.array(scene["bin_extent"][0]), np.array(scene["bin_extent"][1])
    rs = st["root_state"].reshape(N, A, 13)
    rs[:] = 0
    rs[..., 6] = 1.0
    rs[:, 0, 0:3] = [0.28, 0.58, 0.8]
    rs[:, 1, 0:3] = [0.0, 0.0, 0.5]
    for sa in scene["static_actors"]:
        rs[:, sa["actor"], 0:7] = sa["pose"]
    cols = np.linspace(lo[0] + 0.09, hi[0] - 0.09, 2)
    rows = np.linspace(lo[1] + 0.08, hi[1] - 0.08, 4)
    for o in range(n_obj):
        a = 4 + o
        rs[:, a, 0] = cols[o % 2] + spread * rng.uniform(-0.02, 0.02, N)
        rs[:, a, 1] = rows[(o // 2) % 4] + spread * rng.uniform(-0.02, 0.02, N)
        rs[:, a, 2] = lo[2] + 0.06 + 0.1 * (o // 8) + rng.uniform(0.0, 0.03, N)
        rs[:, a, 3:7] = rand_quat(rng, (N,))
        rs[:, a, 7:10] = rng.uniform(-0.1, 0.1, (N, 3))
        rs[:, a, 10:13] = rng.uniform(-0.5, 0.5, (N, 3))
    ds = st["dof_state"].reshape(N, 17, 2)
    ds[..., 0] = RESET_POSE + rng.uniform(-0.05, 0.05, (N, 17)).astype(np.float32)
    ds[:, 6:14, 0] = np.clip(ds[:, 6:14, 0], -1.571, 0.0)
    ds[:, 14, 0] = np.clip(ds[:, 14, 0], -1.571, 0.0)
    ds[:, 15:17, 0] = np.clip(ds[:, 15:17, 0], 0.0, 1.571)
    ds[..., 1] = rng.uniform(-0.3, 0.3, (N, 17))
    st["sim_targets"][:] = RESET_POSE + rng.uniform(-0.3, 0.3, (N, 17)).astype(np.float32)
    st["object_indices"][:] = bin_pool_ids(rng, N, n_obj, pool)
    st["collision_enabled"][:] = 1
    return st


# the persistent contact manifolds (v13) are physics state too: the next call's contacts depend on them
PHYSICS_OUTPUTS = ("dof_state", "root_state", "rigid_body_state", "net_contact_force", "dof_force", "contact_cache")


def assert_physics_bit_identical(sim, st, n, fields=PHYSICS_OUTPUTS, tag=""):
    """Every physics output of every env is bit-identical between the HIP path (sim, through the C ABI) and
    the C oracle (st): the kernels and oracle/physics_oracle.c evaluate the same float32 operations in the same
    order (shared sin/cos in include/ha_fmath.h, the emulated DPP reduction tree, deterministic child sums,
    correctly rounded division and square root on both sides, no contraction)."""
    import torch
    torch.cuda.synchronize()
    for k in fields:
        g = sim.t[k].cpu().numpy().reshape(n, -1)
        o = np.asarray(st[k]).reshape(n, -1)
        assert np.isfinite(g).all(), f"{tag} {k}: non-finite GPU output"
        same = (g.view(np.uint32) == o.view(np.uint32)).all(1)
        assert same.all(), (f"{tag} {k}: {int((~same).sum())}/{n} envs differ from the oracle, "
                            f"max |d| {np.abs(g - o).max():.3e}")


# ----------------------------------------------------------------------------- box scenes (narrow-phase tests)
def box_hull_record(half):
    """A box hull record (tools/build_model.py box_hull): 8 vertices, 6 face planes n.x + d <= 0 inside."""
    hx, hy, hz = (float(h) for h in half)
    verts = [[sx * hx, sy * hy, sz * hz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    planes = [[1, 0, 0, -hx], [-1, 0, 0, -hx], [0, 1, 0, -hy], [0, -1, 0, -hy], [0, 0, 1, -hz], [0, 0, -1, -hz]]
    return {"verts": verts, "planes": planes, "center": [0.0, 0.0, 0.0], "radius": float(np.linalg.norm([hx, hy, hz]))}


def box_pool_scene(halves, density=400.0):
    """The Ur5Sih scene (robot, table) with a pool of boxes (half extents `halves`) instead of the YCB objects."""
    from handarm_hip import model as HM
    scene = dict(HM.load_scene(HM.ASSET))
    objs = []
    for i, h in enumerate(halves):
        hx, hy, hz = h
        m = density * 8 * hx * hy * hz
        I = [m / 3 * (hy * hy + hz * hz), 0, 0, 0, m / 3 * (hx * hx + hz * hz), 0, 0, 0, m / 3 * (hx * hx + hy * hy)]
        objs.append({"name": f"box{i}", "mass": m, "com": [0.0, 0.0, 0.0], "inertia": I, "hull": box_hull_record(h),
                     "bbox_extents": [2 * hx, 2 * hy, 2 * hz]})
    scene["objects"] = objs
    return scene


def axis_quat(axis, ang):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    return np.concatenate([a * np.sin(ang / 2), [np.cos(ang / 2)]]).astype(np.float32)


TABLE_TOP, TABLE_X1 = 0.5, 0.2925 + 0.375       # Ur5SihMultiObject table: top z, far edge x (multi_object.py:536)
EDGE_BOXES = [(0.03, 0.05, 0.03), (0.05, 0.03, 0.03), (0.04, 0.04, 0.02)]


def fill_box_scene(st, num_envs, kind, seed=0, pen=0.0005):
    """Robot at its reset pose (clear of the objects) and the three boxes of box_pool_scene(EDGE_BOXES) in an
    edge-contact configuration, poses jittered per env (seeded):
      "crossed":    box 1 rotated 45 deg about x (a ridge along x on top) stands on its bottom edge on the table; box 0
                    rotated 45 deg about y (a ridge along y at its bottom) lies across it, ridges crossing at 90 deg,
                    ~pen deep: an edge-edge contact no face axis finds;
      "table_edge": box 0 rotated 45 deg about x, its bottom ridge (along x) across the table's far edge (along y);
      "overhang":   box 2 flat on the table, its centre 1 cm inside the far edge (37.5% over it): the support
                    polygon reaches the table edge only through clipped edge points."""
    rng = np.random.default_rng(seed)
    N = num_envs
    rs = st["root_state"].reshape(N, 6, 13)
    rs[:] = 0
    rs[..., 6] = 1.0
    rs[:, 0, 0:3] = [0.28, 0.58, 0.8]
    rs[:, 1, 0:3] = [0.0, 0.0, 0.5]
    rs[:, 2, 0:3] = [0.2925, 0.38, 0.25]
    r2 = np.sqrt(2.0)
    jit = rng.uniform(-1.0, 1.0, (N, 3)).astype(np.float32)
    if kind == "crossed":
        h1, h0 = EDGE_BOXES[1], EDGE_BOXES[0]
        z1 = TABLE_TOP + (h1[1] + h1[2]) / r2
        rs[:, 4, 0:3] = np.stack([0.45 + 0.002 * jit[:, 0], 0.80 + 0.002 * jit[:, 1], np.full(N, z1)], 1)
        rs[:, 4, 3:7] = axis_quat([1, 0, 0], np.pi / 4)
        top1 = z1 + (h1[1] + h1[2]) / r2
        z0 = top1 + (h0[0] + h0[2]) / r2 - pen * (1.0 + 0.5 * jit[:, 2])
        rs[:, 3, 0:3] = np.stack([rs[:, 4, 0], rs[:, 4, 1], z0], 1)
        rs[:, 3, 3:7] = axis_quat([0, 1, 0], np.pi / 4)
    elif kind == "table_edge":
        h0 = EDGE_BOXES[0]
        rs[:, 3, 0:3] = np.stack([TABLE_X1 + 0.003 * jit[:, 0], 0.80 + 0.01 * jit[:, 1],
                                  TABLE_TOP + (h0[1] + h0[2]) / r2 - pen * (1.0 + 0.5 * jit[:, 2])], 1)
        rs[:, 3, 3:7] = axis_quat([1, 0, 0], np.pi / 4)
        rs[:, 4, 0:3] = [0.10, 0.85, TABLE_TOP + EDGE_BOXES[1][2]]
    elif kind == "overhang":
        h2 = EDGE_BOXES[2]
        rs[:, 5, 0:3] = np.stack([TABLE_X1 - 0.01 + 0.002 * jit[:, 0], 0.80 + 0.01 * jit[:, 1],
                                  np.full(N, TABLE_TOP + h2[2] - 0.0002)], 1)
        rs[:, 5, 3:7] = axis_quat([0, 0, 1], 0.05 * jit[:, 2].mean())
        rs[:, 3, 0:3] = [0.10, 0.85, TABLE_TOP + EDGE_BOXES[0][2]]
        rs[:, 4, 0:3] = [0.20, 0.85, TABLE_TOP + EDGE_BOXES[1][2]]
    else:
        raise ValueError(kind)
    if kind != "overhang":
        rs[:, 5, 0:3] = [0.20, 0.88, TABLE_TOP + EDGE_BOXES[2][2]]
    ds = st["dof_state"].reshape(N, 17, 2)
    ds[..., 0] = RESET_POSE
    ds[..., 1] = 0.0
    st["sim_targets"][:] = RESET_POSE
    st["object_indices"][:] = [0, 1, 2]
    st["collision_enabled"][:] = 1
    return st


def link_hull_world_verts(model, body_state_env, link):
    """World vertices of every hull of robot link `link` (model hull_link), posed by its rigid_body_state row."""
    from handarm_hip import model as HM   # noqa: F401
    row = body_state_env[model.body_robot0 + link]
    p, q = row[0:3].astype(np.float64), row[3:7].astype(np.float64)
    x, y, z, w = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    out = []
    for k in range(model.n_link_hulls):
        if model.hull_link[k] != link:
            continue
        s, nv = model.hull_vert_start[k], model.hull_nverts[k]
        v = np.array([list(model.verts[s + i])[:3] for i in range(nv)], np.float64)
        out.append(v @ R.T + p)
    return np.concatenate(out)


def place_cuboid_edge_on_link(st, model, body_state, link, pen=0.0003):
    """AllegroKuka: each env's cuboid (its object_scale dims of the 0.05 m base cube) rotated 45 deg about x, its
    bottom ridge (along x) `pen` below the highest vertex of link `link`'s hulls and over it, at rest."""
    N, A = st.num_envs, model.n_actors
    rs = st["root_state"].reshape(N, A, 13)
    sc = st["object_scale"].reshape(N, 3)
    body = body_state.reshape(N, model.n_bodies, 13)
    q = axis_quat([1, 0, 0], np.pi / 4)
    for e in range(N):
        v = link_hull_world_verts(model, body[e], link)
        top = v[np.argmax(v[:, 2])]
        hy, hz = 0.025 * sc[e, 1], 0.025 * sc[e, 2]
        # the lowest ridge is the (-y, -z) edge, offset (hz - hy)/sqrt(2) in y from the centre
        rs[e, model.actor_object0, 0:3] = [top[0], top[1] - (hz - hy) / np.sqrt(2.0),
                                           top[2] + (hy + hz) / np.sqrt(2.0) - pen]
        rs[e, model.actor_object0, 3:7] = q
        rs[e, model.actor_object0, 7:13] = 0.0
    st["object_force"][:] = 0.0
    return st
