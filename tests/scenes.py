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


PHYSICS_OUTPUTS = ("dof_state", "root_state", "rigid_body_state", "net_contact_force", "dof_force")


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
