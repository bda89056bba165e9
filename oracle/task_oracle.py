"""ORACLE (test infrastructure only) - numpy restatement of the reference hand-arm task math.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / CPU baseline. The product path (``handarm_hip``) never calls it.

Pinned by golden vectors produced by running the reference code itself (``tests/golden/*.npz``,
generator ``tests/golden/make_goldens.py``). One third-party piece is *unpinned*: the SIH
servo->joint map evaluates ``torchcubicspline`` natural cubic splines (package absent from the
reference checkout and from ``setup.py``; no version pinned). ``NaturalCubicSpline`` below restates
that package's published algorithm (knot-derivative tridiagonal solve, Thomas algorithm, piecewise
cubic evaluated with ``bucketize(t) - 1`` clamped to the end pieces, i.e. cubic extrapolation).

All arithmetic is float32 in the reference's operation order so results match torch's CPU float32
kernels to the last ulp in almost every element.
"""
import numpy as np

F = np.float32

# ----------------------------------------------------------------------------- quaternions (xyzw)
# reference: isaacgymenvs/utils/torch_jit_utils.py:41-123, 233-240


def quat_mul(a, b):
    """torch_jit_utils.py:41-62 (8-multiplication form)."""
    a = np.asarray(a, F)
    b = np.asarray(b, F)
    x1, y1, z1, w1 = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    x2, y2, z2, w2 = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = F(0.5) * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return np.stack([x, y, z, w], -1)


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1)


def quat_apply(a, b):
    """torch_jit_utils.py:70-77: b + w*t + xyz x t, t = 2 (xyz x b)."""
    a = np.asarray(a, F)
    b = np.asarray(b, F)
    xyz = a[..., :3]
    t = cross(xyz, b) * F(2)
    return b + a[..., 3:] * t + cross(xyz, t)


def quat_conjugate(a):
    a = np.asarray(a, F)
    return np.concatenate([-a[..., :3], a[..., 3:]], -1)


def normalize(x, eps=1e-9):
    n = np.sqrt(np.sum(x * x, -1, keepdims=True, dtype=F)).astype(F)
    return x / np.maximum(n, F(eps))


def quat_from_angle_axis(angle, axis):
    """torch_jit_utils.py:118-123."""
    theta = (np.asarray(angle, F) / F(2))[..., None]
    xyz = normalize(np.asarray(axis, F)) * np.sin(theta)
    w = np.cos(theta)
    return normalize(np.concatenate([xyz, w], -1))


def randomize_rotation(rand0, rand1):
    """multi_object_manipulation.py:12-15 with x/y unit axes."""
    n = np.shape(rand0)
    xu = np.broadcast_to(np.array([1, 0, 0], F), n + (3,))
    yu = np.broadcast_to(np.array([0, 1, 0], F), n + (3,))
    return quat_mul(quat_from_angle_axis(np.asarray(rand0, F) * F(np.pi), xu),
                    quat_from_angle_axis(np.asarray(rand1, F) * F(np.pi), yu))


def scale(x, lower, upper):
    return F(0.5) * (np.asarray(x, F) + F(1.0)) * (upper - lower) + lower


def unscale(x, lower, upper):
    return (F(2.0) * np.asarray(x, F) - upper - lower) / (upper - lower)


# ----------------------------------------------------------------------------- splines
class NaturalCubicSpline:
    """Restatement of torchcubicspline (natural_cubic_spline_coeffs + NaturalCubicSpline.evaluate).

    PARITY UNPINNED (third-party, absent, unversioned). Call sites: ur5sih.py:442-455, 508-522.
    """

    def __init__(self, knots, values):
        t = np.asarray(knots, F)
        x = np.asarray(values, F)
        n = len(t)
        if n == 2:
            a = x[:1]
            b = (x[1:] - x[:1]) / (t[1:] - t[:1])
            two_c = np.zeros_like(b)
            three_d = np.zeros_like(b)
        else:
            dt = t[1:] - t[:-1]
            r = (F(1) / dt).astype(F)
            r2 = (r ** 2).astype(F)
            three = F(3) * (x[1:] - x[:-1])
            six = F(2) * three
            scaled = three * r2
            diag = np.empty(n, F)
            diag[:-1] = r
            diag[-1] = 0
            diag[1:] += r
            diag *= F(2)
            rhs = np.empty(n, F)
            rhs[:-1] = scaled
            rhs[-1] = 0
            rhs[1:] += scaled
            # Thomas algorithm (torchcubicspline.misc.tridiagonal_solve)
            nb = np.empty(n, F)
            nd = np.empty(n, F)
            out = np.empty(n, F)
            nb[0], nd[0] = rhs[0], diag[0]
            for i in range(1, n):
                w = r[i - 1] / nd[i - 1]
                nd[i] = diag[i] - w * r[i - 1]
                nb[i] = rhs[i] - w * nb[i - 1]
            out[n - 1] = nb[n - 1] / nd[n - 1]
            for i in range(n - 2, -1, -1):
                out[i] = (nb[i] - r[i] * out[i + 1]) / nd[i]
            a = x[:-1]
            b = out[:-1]
            two_c = (six * r - F(4) * out[:-1] - F(2) * out[1:]) * r
            three_d = (-six * r + F(3) * (out[:-1] + out[1:])) * r2
        self.t, self.a, self.b, self.two_c, self.three_d = t, a.astype(F), b.astype(F), two_c.astype(F), three_d.astype(F)

    def table(self):
        """(5, n_pieces): knot start, a, b, two_c, three_d - the layout the HIP kernel consumes."""
        return np.stack([self.t[:-1], self.a, self.b, self.two_c, self.three_d]).astype(F)

    def evaluate(self, q):
        q = np.asarray(q, F)
        idx = np.searchsorted(self.t, q, side="left") - 1     # torch.bucketize(right=False) - 1
        idx = np.clip(idx, 0, len(self.b) - 1)
        f = q - self.t[idx]
        inner = F(0.5) * self.two_c[idx] + self.three_d[idx] * f / F(3)
        inner = self.b[idx] + inner * f
        return self.a[idx] + inner * f


# ur5sih.py:437-456
SERVO_LOWER = np.array([0, -2000, -1250, -400, -1350], F)
SERVO_UPPER = np.array([2650, 250, 1450, 2300, 1000], F)
SPLINES = {
    "thumb_proximal": ([-1850, -1175, -975, -600, -225], [-1.51, -1.31, -1.175, -0.6, 0.]),
    "thumb_distal": ([-1318.125, -906.25, -200], [-1.235, -0.855, 0.]),
    "index_proximal": ([-1250, -250, 150, 350, 540, 730, 1085, 1400], [-1.53, -1.4425, -1.315, -1.25, -1.18, -1.15, -0.6, 0.]),
    "index_distal": ([-408.606, 793.515, 1400], [-1.665, -0.735, 0]),
    "middle_proximal": ([-500, 500, 1350, 1625, 1700, 1980, 2240], [-1.571, -1.445, -1.055, -0.91, -0.9, -0.48, 0.]),
    "middle_distal": ([442.6, 1147, 1750.6, 2240], [-1.65, -1.125, -0.62, 0.]),
    "ring_proximal": ([-1050, -500, -250, 0, 370, 500, 700, 940], [-1.571, -1.45, -1.35, -1.225, -0.95, -0.9, -0.533, 0.]),
    "ring_distal": ([-719, 408.8, 686.8, 939.2], [-1.64, -0.69, -0.425, 0.]),
}
PROXIMAL_COEF = {"thumb": F(-625.0), "index": F(-582.61), "middle": F(-600.0), "ring": F(-488.0)}
SPLINE_OBJS = {k: NaturalCubicSpline(*v) for k, v in SPLINES.items()}

# DOF order (depth-first, siblings by link name; see tools/build_model.py)
DOF_NAMES = ["shoulder_pan_joint", "shoulder_lift_joint", "elbow_joint", "wrist_1_joint", "wrist_2_joint",
             "wrist_3_joint", "index_finger", "if_proximal_to_if_distal", "palm_to_lf_proximal",
             "lf_proximal_to_lf_distal", "middle_finger", "mf_proximal_to_mf_distal", "ring_finger",
             "rf_proximal_to_rf_distal", "thumb_opposition", "thumb_flexion", "th_inter_to_th_distal"]
D = {n: i for i, n in enumerate(DOF_NAMES)}
DT = F(0.016666667)          # Ur5SihBase.yaml:28 (VecTask.dt = sim_params.dt, vec_task.py:267)
RESET_POSE = np.array([0.6985, -1.4106, 1.2932, 0.1174, 0.6983, 1.5708, 0., 0., 0., 0., 0., 0., 0., 0., -1.571,
                       0., 0.], F)  # Ur5SihBase.yaml:9


def controller_step(actions, dof_pos, ur5_target, servo, smoothed, alpha=0.8):
    """One pre_physics_step of the two actionables (ur5sih.py:397-405 relative, 485-527 smoothed_relative).

    Returns (dof_position_targets[N,17], ur5_target, servo, smoothed) - new arrays.
    """
    actions = np.asarray(actions, F)
    ur5_target = ur5_target + DT * F(1.0) * actions[:, 0:6]
    smoothed = F(alpha) * actions[:, 6:11] + F(1 - alpha) * smoothed   # python-double (1-alpha), cast once
    servo = servo + F(100) * smoothed
    servo = np.minimum(np.maximum(servo, SERVO_LOWER), SERVO_UPPER)
    n = actions.shape[0]
    tgt = np.zeros((n, 17), F)
    tgt[:, 0:6] = ur5_target
    s = SPLINE_OBJS
    tgt[:, D["thumb_opposition"]] = F(-1.571 / 2675) * servo[:, 0]
    tgt[:, D["thumb_flexion"]] = -s["thumb_proximal"].evaluate(servo[:, 1])
    tgt[:, D["th_inter_to_th_distal"]] = -s["thumb_distal"].evaluate(
        servo[:, 1] + PROXIMAL_COEF["thumb"] * dof_pos[:, D["thumb_flexion"]])
    tgt[:, D["index_finger"]] = s["index_proximal"].evaluate(servo[:, 2])
    tgt[:, D["if_proximal_to_if_distal"]] = s["index_distal"].evaluate(
        servo[:, 2] + PROXIMAL_COEF["index"] * dof_pos[:, D["index_finger"]])
    tgt[:, D["middle_finger"]] = s["middle_proximal"].evaluate(servo[:, 3])
    tgt[:, D["mf_proximal_to_mf_distal"]] = s["middle_distal"].evaluate(
        servo[:, 3] + PROXIMAL_COEF["middle"] * dof_pos[:, D["middle_finger"]])
    tgt[:, D["ring_finger"]] = s["ring_proximal"].evaluate(servo[:, 4])
    tgt[:, D["rf_proximal_to_rf_distal"]] = s["ring_distal"].evaluate(
        servo[:, 4] + PROXIMAL_COEF["ring"] * dof_pos[:, D["ring_finger"]])
    tgt[:, D["palm_to_lf_proximal"]] = tgt[:, D["ring_finger"]]
    tgt[:, D["lf_proximal_to_lf_distal"]] = tgt[:, D["rf_proximal_to_rf_distal"]]
    return tgt, ur5_target, servo, smoothed


# ----------------------------------------------------------------------------- observations
# env body indices: goal 0, robot 1..29 (robot body order), table 30, objects 31..33
FLANGE_BODY = 1 + 9
FINGERTIP_BODIES = [1 + 28, 1 + 15, 1 + 21, 1 + 24, 1 + 18]   # thumb, index, middle, ring, little (ur5sih.py:613)
OBJECT_ACTORS = [3, 4, 5]
GOAL_ACTOR = 0
OBS_LAYOUT = [("ur5_joint_pos", 6), ("ur5_flange_pose", 7), ("sih_fingertip_pos", 15), ("sih_fingertip_quat", 20),
              ("sih_fingertip_linvel", 15), ("dof_position_targets", 17), ("object_pos", 9),
              ("object_bounding_box", 30), ("target_object_bounding_box", 10),
              ("sih_fingertip_to_target_object_pos", 15), ("target_object_to_goal_pos", 3)]


def observations(root, body, dof, targets, goal_pos, target_idx, bbox_pos, bbox_quat, bbox_ext,
                 prev_object_pose, object_actors=None):
    """post_step callbacks + compute_observations (Ur5SihMultiObjectManipulation.yaml:24-26,43-44).

    root (N,6,13) body (N,34,13) dof (N,17,2) targets (N,17) goal_pos (N,3) target_idx (N,) int
    bbox_pos (N,3,3) bbox_quat (N,3,4) bbox_ext (N,3,3); prev_object_pose (N,3,7) = the object
    pos/quat cached by the PREVIOUS post_step refresh. Returns obs (N,147), object_bbox (N,3,10).
    With n objects (object_actors = their actor rows, e.g. 4..11 in the bin scene) the object blocks grow
    to 3n and 10n: obs (N, 108 + 13 n).

    Reference quirk reproduced: the observable refresh order is the reversed networkx topological
    sort (observables.py:231-243) and ``object_bounding_box`` declares no ``requires``, so its
    post_step runs BEFORE ``object_pos``/``object_quat`` are refreshed (order: target_object_pos,
    sih_fingertip_pos, ur5_joint_state, object_bounding_box, dof_position_targets, object_pos, ...).
    The bounding boxes therefore use the object pose of the previous refresh (one-step lag).
    """
    n = root.shape[0]
    ar = np.arange(n)
    actors = np.asarray(OBJECT_ACTORS if object_actors is None else object_actors)
    no = len(actors)
    object_pos = root[:, actors, 0:3]
    bbox = np.zeros((n, no, 10), F)
    bbox[..., 0:3] = prev_object_pose[..., 0:3] + quat_apply(prev_object_pose[..., 3:7], bbox_pos)  # :771
    bbox[..., 3:7] = quat_mul(prev_object_pose[..., 3:7], bbox_quat)                              # :772
    bbox[..., 7:10] = bbox_ext
    target_pos = root[ar, actors[target_idx], 0:3]        # multi_object.py:214
    tips = body[:, FINGERTIP_BODIES]
    parts = [dof[:, 0:6, 0],
             body[:, FLANGE_BODY, 0:7],
             tips[..., 0:3].reshape(n, 15),
             tips[..., 3:7].reshape(n, 20),
             tips[..., 7:10].reshape(n, 15),
             targets,
             object_pos.reshape(n, 3 * no),
             bbox.reshape(n, 10 * no),
             bbox[ar, target_idx],
             (target_pos[:, None, :] - tips[..., 0:3]).reshape(n, 15),
             goal_pos - target_pos]
    return np.concatenate(parts, -1).astype(F), bbox


REWARD_SCALES = {"reaching": F(1.0), "lifting": F(5.0), "goal": F(50.0), "success": F(50.0)}
LIFT_THRESHOLD = F(0.05)
GOAL_THRESHOLD = F(0.05)
MAX_EPISODE_LENGTH = 200


def norm3(x):
    return np.sqrt(np.sum(x * x, -1, dtype=F)).astype(F)


def reward(root, body, goal_pos, target_idx, cfg_idx, object_pos_initial, object_actors=None):
    """_update_rew_buf (multi_object_manipulation.py:237-313) with its helpers :353-387.

    Returns rew (N,), goal_reached (N,) bool, per-term rewards dict.
    """
    n = root.shape[0]
    ar = np.arange(n)
    actors = np.asarray(OBJECT_ACTORS if object_actors is None else object_actors)
    target_pos = root[ar, actors[target_idx], 0:3]
    dist = norm3(target_pos - goal_pos)
    reached = dist < GOAL_THRESHOLD
    init = object_pos_initial[ar, cfg_idx][ar, target_idx]
    delta = target_pos - init
    lifted = delta[:, 2] > LIFT_THRESHOLD
    tips = body[:, FINGERTIP_BODIES, 0:3]
    terms = {}
    rew = np.zeros(n, F)
    for name, sc in REWARD_SCALES.items():
        if name == "lifting":
            dh = np.clip(LIFT_THRESHOLD - delta[:, 2], F(0), LIFT_THRESHOLD) / LIFT_THRESHOLD
            r = sc * (np.exp(F(-3.0) * dh) - np.exp(F(-3.0) * np.ones_like(dh)))
        elif name == "reaching":
            fd = norm3(tips - target_pos[:, None, :])
            fd[:, 0] *= F(4.0)
            r = sc * np.exp(F(-3.0) * np.sum(fd, 1, dtype=F))
        elif name == "goal":
            r = sc * lifted.astype(F) * np.exp(F(-5.0) * dist)
        else:
            r = sc * reached.astype(F)
        terms[name] = r.astype(F)
        rew = (rew + r).astype(F)
    return rew, reached, terms


def done(progress, reset_buf):
    """_update_reset_buf (:232-235) and VecTask timeout rule (vec_task.py:424). Integers, exact."""
    reset = np.where(progress >= MAX_EPISODE_LENGTH, 1, reset_buf).astype(np.int64)
    timeout = (progress >= MAX_EPISODE_LENGTH - 1) & (reset != 0)
    return reset, timeout


class SuccessTracker:
    """_update_success_rate (multi_object_manipulation.py:316-351) from per-step counts.

    The device accumulates (num_resets, num_successes) overall and per object; the EWMA is a host
    scalar update, exactly as the reference does after its .item() syncs.
    """

    def __init__(self, n_objects, num_envs):
        self.ewma = 0.0
        self.obj = [0.0] * n_objects
        self.num_envs = num_envs
        self.total_resets = 0
        self.total_successes = 0

    def update(self, num_resets, num_successes, obj_resets, obj_successes):
        log = {}
        if num_resets > 0:
            rate = np.float32(num_successes) / np.float32(num_resets)
            alpha = np.float32(0.2) * (np.float32(num_resets) / np.float32(self.num_envs))
            self.ewma = float(alpha * rate + (np.float32(1) - alpha) * np.float32(self.ewma))
            log["overall"] = self.ewma
            self.total_resets += num_resets
            self.total_successes += num_successes
        for i in range(len(self.obj)):
            if obj_resets[i] > 0:
                rate = np.float32(obj_successes[i]) / np.float32(obj_resets[i])
                alpha = np.float32(0.2) * (np.float32(obj_resets[i]) / np.float32(self.num_envs)) * np.float32(len(self.obj))
                self.obj[i] = float(alpha * rate + (np.float32(1) - alpha) * np.float32(self.obj[i]))
                log[i] = self.obj[i]
        return log


def success_counts(reset, reached, object_indices, target_idx, n_objects):
    ar = np.arange(len(reset))
    tgt_global = object_indices[ar, target_idx]
    num_resets = int(reset.sum())
    num_succ = int(reached.sum())
    obj_resets = [int(reset[tgt_global == i].sum()) for i in range(n_objects)]
    obj_succ = [int(reached[tgt_global == i].sum()) for i in range(n_objects)]
    return num_resets, num_succ, obj_resets, obj_succ


# ----------------------------------------------------------------------------- reset (steady state)
GOAL_POS = np.array([0.28, 0.58, 0.8], F)      # Ur5SihMultiObject.yaml:16-19
GOAL_NOISE = np.array([0.15, 0.15, 0.1], F)


def goal_from_draw(draw):
    """_get_random_object_pos(key='goal') (:175-184): pos + (2(u-0.5)) @ diag(noise)."""
    noise = F(2) * (np.asarray(draw, F) - F(0.5))
    noise = noise * GOAL_NOISE          # @ diag(noise) == column scaling (single product per element)
    return GOAL_POS[None, :] + noise


def reset_state(root, dof, draw_cfg, draw_target, draw_goal, object_pos_initial, object_quat_initial):
    """reset_idx steady state for ALL envs (multi_object_manipulation.py:33-71).

    root (N,6,13) dof (N,17,2) are modified copies; returns dict of the task-side buffers.
    """
    root = root.copy()
    dof = dof.copy()
    n = root.shape[0]
    ar = np.arange(n)
    pos0 = object_pos_initial[ar, draw_cfg]
    quat0 = object_quat_initial[ar, draw_cfg]
    for i, a in enumerate(OBJECT_ACTORS):
        root[:, a, 0:3] = pos0[:, i]
        root[:, a, 3:7] = quat0[:, i]
        root[:, a, 7:13] = 0
    goal = goal_from_draw(draw_goal)
    root[:, GOAL_ACTOR, 0:3] = goal
    dof[:, :, 0] = RESET_POSE
    dof[:, :, 1] = 0
    targets = np.tile(RESET_POSE, (n, 1))       # as pushed to the sim (ur5sih.py:622-628)
    task_targets = targets.copy()
    task_targets[:, 6:] = 0                     # _reset_sih_servo_pos_controller (ur5sih.py:477)
    return dict(root=root, dof=dof, sim_targets=targets, targets=task_targets, goal_pos=goal,
                target_idx=np.asarray(draw_target), cfg_idx=np.asarray(draw_cfg),
                servo=np.tile(SERVO_UPPER, (n, 1)), smoothed=np.zeros((n, 5), F),
                ur5_target=dof[:, 0:6, 0].copy())


# ----------------------------------------------------------------------------- synthetic point clouds (§8f #2)
def object_pointcloud(pose, samples, perm):
    """object_synthetic_pointcloud (multi_object.py:792-800): pose (N, n_obj, 7) object pos+quat,
    samples (N, n_obj, P, 4) per-env pool-frame samples (w 1 / 0 padding), perm (P,).
    ordered = pos + quat_apply(quat, samples); xyz *= w; then the point axis permuted. -> (N, n_obj*P, 4)"""
    pose = np.asarray(pose, F)
    samples = np.asarray(samples, F)
    n, no, p = samples.shape[:3]
    pos = np.broadcast_to(pose[:, :, None, 0:3], (n, no, p, 3))
    quat = np.broadcast_to(pose[:, :, None, 3:7], (n, no, p, 4))
    ordered = samples.copy()
    ordered[..., 0:3] = pos + quat_apply(quat, samples[..., 0:3])
    ordered[..., 0:3] *= ordered[..., 3:4]
    return ordered[:, :, np.asarray(perm)].reshape(n, no * p, 4)


def target_pointcloud(object_pc, target_idx, n_obj):
    """target_object_synthetic_pointcloud (multi_object.py:802-804): gather the target row, w *= TARGET (2)."""
    n = object_pc.shape[0]
    pc = object_pc.reshape(n, n_obj, -1, 4)[np.arange(n), np.asarray(target_idx)].copy()
    pc[..., 3] *= F(2)
    return pc


def robot_pointcloud(body, link_bodies, samples):
    """ur5sih_synthetic_pointcloud (ur5sih.py:361-374, relative=False): body (N, B, 13) rigid-body states,
    link_bodies (R,) env body index per sample, samples (R, 3) link-frame points. w = 1."""
    body = np.asarray(body, F)
    b = body[:, np.asarray(link_bodies)]
    out = np.ones((body.shape[0], len(link_bodies), 4), F)
    out[..., 0:3] = b[..., 0:3] + quat_apply(b[..., 3:7], np.broadcast_to(np.asarray(samples, F), b[..., 0:3].shape))
    return out


def fingertip_pointcloud(body, tip_bodies):
    """sih_fingertip_pointcloud (ur5sih.py:337-345): fingertip positions with id 3."""
    b = np.asarray(body, F)[:, np.asarray(tip_bodies), 0:3]
    return np.concatenate([b, np.full(b.shape[:-1] + (1,), 3, F)], -1)


def goal_pointcloud(goal_pos):
    """goal_synthetic_pointcloud (multi_object.py:383-389)."""
    g = np.asarray(goal_pos, F)
    return np.concatenate([g, np.full((len(g), 1), 3, F)], -1)[:, None]


def relative_goal_pointcloud(goal_pos, flange_pose):
    """relative_goal_synthetic_pointcloud (multi_object.py:391-401, 806-809)."""
    fl = np.asarray(flange_pose, F)
    rel = quat_apply(quat_conjugate(fl[:, 3:7]), np.asarray(goal_pos, F) - fl[:, 0:3])
    return np.concatenate([rel, np.full((len(rel), 1), 3, F)], -1)[:, None]
