"""ORACLE (test infrastructure only) - numpy restatement of the reference AllegroKuka task math
(tasks/allegro_kuka/allegro_kuka_base.py + allegro_kuka_regrasping.py / allegro_kuka_reorientation.py,
cfg/task/AllegroKuka.yaml; config C2 of BASELINE.json).

Only ``tests/`` may import this module. Pinned by ``tests/golden/kuka_*.npz``, which the reference itself
produced (``tests/golden/make_goldens_kuka.py``). float32 in the reference's operation order. The per-env
task tensors travel in the device's ``task_state`` row layout (handarm_hip.model AK_*).
"""
import numpy as np

from handarm_hip import model as HM
from oracle import f32

F = np.float32
D, NARM = 23, 7
DRAW_GOAL = 0


def goal_draws(p):
    """Draws of one reset_target_pose (ak_task.h ak_goal_draws): 9, throw 10 (bucket side, offset, y, z + the
    object's 6)."""
    return 10 if p.ak_subtask == 2 else 9


def draw_slots(p):
    """ak_task.h AK_DRAW_*: reset goal, object, force prob, dof, vel, force u, force n."""
    G = goal_draws(p)
    return dict(RESET_GOAL=G, OBJ=2 * G, FORCE_PROB=2 * G + 6, DOF=2 * G + 7, VEL=2 * G + 30, FORCE_U=2 * G + 53,
                FORCE_N=2 * G + 54)


def quat_rotate(q, v):
    """torch_jit_utils.py:81-90 (xyzw), batched over the leading axis."""
    q, v = q.astype(F), v.astype(F)
    qw = q[:, 3:4]
    a = v * (F(2.0) * (qw * qw) - F(1.0))
    qv = q[:, :3]
    cr = np.stack([qv[:, 1] * v[:, 2] - qv[:, 2] * v[:, 1], qv[:, 2] * v[:, 0] - qv[:, 0] * v[:, 2],
                   qv[:, 0] * v[:, 1] - qv[:, 1] * v[:, 0]], 1)
    b = cr * qw * F(2.0)
    dt = ((qv[:, 0] * v[:, 0] + qv[:, 1] * v[:, 1]) + qv[:, 2] * v[:, 2])[:, None]
    c = qv * dt * F(2.0)
    return (a + b + c).astype(F)


def norm3(v):
    return np.sqrt((v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1]) + v[..., 2] * v[..., 2]).astype(F)


def random_quat(u):
    """get_random_quat (allegro_kuka_base.py:1178-1189) from uvw draws (n, 3)."""
    two_pi = F(2 * np.pi)
    a, b = np.sqrt(F(1.0) - u[:, 0]), np.sqrt(u[:, 0])
    s1, c1 = f32.sincos(two_pi * u[:, 1])       # the kernels' shared sine / cosine (include/ha_fmath.h)
    s2, c2 = f32.sincos(two_pi * u[:, 2])
    return np.stack([a * c1, b * s2, b * c2, a * s1], 1).astype(F)


def post(p, ts, dof_pos, dof_vel, rb, obj, goal, progress, successes, reset_buf, scale, scalars, lo, up, obs_only=False):
    """compute_observations + compute_full_state + compute_kuka_reward + reward slot + clamp
    (allegro_kuka_base.py:991-1176,1426-1447). ts is updated in place. Returns obs, rew, reset, reset_goal,
    progress, successes."""
    N = dof_pos.shape[0]
    nkp = p.ak_num_keypoints
    ts = ts
    palm = rb[:, p.ak_palm_link]
    palm_c = palm[:, 0:3] + quat_rotate(palm[:, 3:7], np.tile(np.array(p.ak_palm_offset, F), (N, 1)))
    ft = np.zeros((N, 4, 3), F)
    for i in range(4):
        tip = rb[:, p.ak_fingertip_links[i]]
        ft[:, i] = tip[:, 0:3] + quat_rotate(tip[:, 3:7], np.tile(np.array(p.ak_fingertip_offsets[i], F), (N, 1)))
    curr = norm3(ft - obj[:, None, 0:3])
    cft = ts[:, HM.AK_CLOSEST_FT:HM.AK_CLOSEST_FT + 4]
    cft[:] = np.where(cft < 0, curr, cft)
    ts[:, HM.AK_FURTHEST] = np.where(ts[:, HM.AK_FURTHEST] < 0, curr[:, 0], ts[:, HM.AK_FURTHEST])
    ft_rel_palm = ft - palm_c[:, None]
    kpo = ts[:, HM.AK_KP:HM.AK_KP + 3 * nkp].reshape(N, nkp, 3)
    okp = np.stack([obj[:, 0:3] + quat_rotate(obj[:, 3:7], kpo[:, j]) for j in range(nkp)], 1)
    gkp = np.stack([goal[:, 0:3] + quat_rotate(goal[:, 3:7], kpo[:, j]) for j in range(nkp)], 1)
    rel_goal = okp - gkp
    rel_palm = okp - palm_c[:, None]
    kmax = norm3(rel_goal).max(-1)
    ts[:, HM.AK_CLOSEST_KP] = np.where(ts[:, HM.AK_CLOSEST_KP] < 0, kmax, ts[:, HM.AK_CLOSEST_KP])
    obs = np.concatenate([
        (F(2.0) * dof_pos - up - lo) / (up - lo), dof_vel, palm_c, palm[:, 3:13], obj[:, 3:13],
        ft_rel_palm.reshape(N, 12), rel_palm.reshape(N, 3 * nkp), rel_goal.reshape(N, 3 * nkp), scale,
        ts[:, HM.AK_CLOSEST_KP:HM.AK_CLOSEST_KP + 1], cft.copy(), ts[:, HM.AK_LIFTED:HM.AK_LIFTED + 1],
        np.log(progress.astype(F) / F(10) + F(1))[:, None], np.log(successes + F(1))[:, None],
        np.zeros((N, 1), F)], 1).astype(F)
    rew = np.zeros(N, F)
    reset = reset_buf.copy()
    reset_goal = np.zeros(N, np.int64)
    progress = progress.copy()
    successes = successes.copy()
    if not obs_only:
        z_lift = (F(0.05) + obj[:, 2]) - F(p.ak_object_init[2])
        lifting_rew = np.clip(z_lift, F(0), F(0.5))
        was = ts[:, HM.AK_LIFTED] != 0
        lifted = (z_lift > F(p.ak_lifting_bonus_threshold)) | was
        lift_bonus = F(p.ak_lifting_bonus) * (lifted & ~was).astype(F)
        lifting_rew = lifting_rew * (~lifted).astype(F)
        ts[:, HM.AK_LIFTED] = lifted.astype(F)
        fdc = cft - curr
        cft[:] = np.minimum(cft, curr)
        hdf = ts[:, HM.AK_FURTHEST] - curr[:, 0]
        ts[:, HM.AK_FURTHEST] = np.maximum(ts[:, HM.AK_FURTHEST], curr[:, 0])
        fdr = np.clip(fdc, F(0), F(10)) * F(1)
        fdr = (((fdr[:, 0] + fdr[:, 1]) + fdr[:, 2]) + fdr[:, 3]) * (~lifted).astype(F)
        hdp = np.clip(hdf, F(-10), F(0)) * (~lifted).astype(F) * F(4)
        mkd = ts[:, HM.AK_CLOSEST_KP] - kmax
        ts[:, HM.AK_CLOSEST_KP] = np.minimum(ts[:, HM.AK_CLOSEST_KP], kmax)
        kr = np.clip(mkd, F(0), F(100)) * lifted.astype(F)
        near = kmax <= scalars[3]
        ts[:, HM.AK_NEAR_GOAL] += near.astype(F)
        is_success = ts[:, HM.AK_NEAR_GOAL] >= p.ak_success_steps
        successes = (successes + is_success.astype(F)).astype(F)
        ep = ts[:, HM.AK_REW_EP:HM.AK_REW_EP + 12]
        ep[:, 0] += fdr
        ep[:, 1] += hdp
        ep[:, 2] += lifting_rew
        ep[:, 3] += kr
        fdr = fdr * F(p.ak_distance_delta_rew_scale)
        hdp = hdp * F(0.0)
        lifting_rew = lifting_rew * F(p.ak_lifting_rew_scale)
        kr = kr * F(p.ak_keypoint_rew_scale)
        sa = np.abs(dof_vel[:, :NARM]).sum(-1, dtype=F)
        sh = np.abs(dof_vel[:, NARM:]).sum(-1, dtype=F)
        kap = F(-1) * (sa * F(p.ak_kuka_actions_penalty_scale))
        aap = F(-1) * (sh * F(p.ak_allegro_actions_penalty_scale))
        bonus = near.astype(F) * F(p.ak_bonus_rew)
        rew = ((((((fdr + hdp) + lifting_rew) + lift_bonus) + kr) + kap) + aap) + bonus
        reset = np.where(obj[:, 2] < F(0.1), 1, reset).astype(np.int64)
        if p.ak_max_consecutive_successes > 0:
            progress = np.where(is_success, 0, progress)
            reset = np.where(successes >= p.ak_max_consecutive_successes, 1, reset)
        reset = np.where(progress >= p.max_episode_length - 1, 1, reset)
        if p.ak_subtask == 1:
            reset = np.where(curr.max(-1) > F(1.5), 1, reset)
        tol_obj = scalars[1]
        ts[:, HM.AK_TRUE_OBJ] = np.where(scalars[2] != 0, successes * F(0.01) + tol_obj, successes + tol_obj)
        ep[:, 4] += fdr
        ep[:, 5] += hdp
        ep[:, 6] += lifting_rew
        ep[:, 7] += lift_bonus
        ep[:, 8] += kr
        ep[:, 9] += bonus
        ep[:, 10] += kap
        ep[:, 11] += aap
        reset_goal = is_success.astype(np.int64)
    obs[:, -1] = rew * F(0.01)
    obs = np.clip(obs, -F(p.ak_clamp_abs_obs), F(p.ak_clamp_abs_obs))
    return obs, rew.astype(F), reset, reset_goal, progress, successes


def _reset_object_pose(p, st, ids, dr, k0):
    ini = np.array(p.ak_object_init, F)
    noise = np.array(p.ak_reset_noise, F)
    obj = st["root"][ids, 1]
    obj[:] = 0
    obj[:, 0:3] = ini + noise * dr[ids, k0:k0 + 3]
    obj[:, 3:7] = random_quat(dr[ids, k0 + 3:k0 + 6])
    st["root"][ids, 1] = obj
    st["ts"][ids, HM.AK_CLOSEST_FT:HM.AK_CLOSEST_FT + 4] = -1
    st["ts"][ids, HM.AK_FURTHEST] = -1


def _reset_target_pose(p, st, ids, dr, k0):
    if p.ak_subtask == 2:
        # throw (allegro_kuka_throw.py:85-103): the bucket (actor 3) left / right of the table, goal 5 cm above it
        lr = dr[ids, k0]
        x = np.where(lr > 0, F(0.5), F(-0.5)).astype(F) + (np.sign(lr) * dr[ids, k0 + 1]).astype(F)
        y, z = dr[ids, k0 + 2], dr[ids, k0 + 3]
        st["root"][ids, 3, 0] = x
        st["root"][ids, 3, 1] = y
        st["root"][ids, 3, 2] = z
        st["goal"][ids, 0] = x
        st["goal"][ids, 1] = y
        st["goal"][ids, 2] = z + F(0.05)
        _reset_object_pose(p, st, ids, dr, k0 + 4)
        st["ts"][ids, HM.AK_LIFTED] = 0
        st["reset_goal"][ids] = 0
        st["ts"][ids, HM.AK_NEAR_GOAL] = 0
        st["ts"][ids, HM.AK_CLOSEST_KP] = -1
        return
    lo, size = np.array(p.ak_target_lo, F), np.array(p.ak_target_size, F)
    tgt = lo + dr[ids, k0:k0 + 3] * size
    st["goal"][ids, 0:3] = tgt
    st["root"][ids, 3, 0:3] = tgt
    if p.ak_subtask == 0:
        _reset_object_pose(p, st, ids, dr, k0 + 3)
        st["ts"][ids, HM.AK_LIFTED] = 0
    else:
        q = random_quat(dr[ids, k0 + 3:k0 + 6])
        st["goal"][ids, 3:7] = q
        st["root"][ids, 3, 3:7] = q
        st["root"][ids, 3, 7:13] = 0
    st["reset_goal"][ids] = 0
    st["ts"][ids, HM.AK_NEAR_GOAL] = 0
    st["ts"][ids, HM.AK_CLOSEST_KP] = -1


def pre(p, st, actions, dr, lo, up):
    """pre_physics_step (allegro_kuka_base.py:1355-1414) on st (dict of numpy arrays, updated in place)."""
    goal_ids = np.nonzero(st["reset_goal"])[0]
    reset_ids = np.nonzero(st["reset"])[0]
    ds = draw_slots(p)
    if len(goal_ids):
        _reset_target_pose(p, st, goal_ids, dr, DRAW_GOAL)
    if len(reset_ids):
        ids = reset_ids
        _reset_target_pose(p, st, ids, dr, ds["RESET_GOAL"])
        st["ts"][ids, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3] = 0
        _reset_object_pose(p, st, ids, dr, ds["OBJ"])
        llo, lhi = np.log(F(p.ak_force_prob_lo)), np.log(F(p.ak_force_prob_hi))
        st["ts"][ids, HM.AK_FORCE_PROB] = np.exp((llo - lhi) * dr[ids, ds["FORCE_PROB"]] + lhi)
        default = np.array(list(p.reset_pose)[:D], F)
        dmax, dmin = up - default, lo - default
        rd = dmin + (dmax - dmin) * dr[ids, ds["DOF"]:ds["DOF"] + D]
        coeff = np.array([p.ak_dof_noise_arm] * NARM + [p.ak_dof_noise_fingers] * (D - NARM), F)
        pos = default + coeff * rd
        st["dof"][ids, :, 0] = pos
        st["dof"][ids, :, 1] = F(p.ak_dof_vel_noise) * dr[ids, ds["VEL"]:ds["VEL"] + D]
        st["targets"][ids] = pos
        st["progress"][ids] = 0
        st["reset"][ids] = 0
        ts = st["ts"]
        ts[ids, HM.AK_PREV_SUCC] = st["successes"][ids]
        st["successes"][ids] = 0
        ts[ids, HM.AK_PREV_TRUE_OBJ] = ts[ids, HM.AK_TRUE_OBJ]
        ts[ids, HM.AK_TRUE_OBJ] = 0
        ts[ids, HM.AK_LIFTED] = 0
        ts[ids, HM.AK_CLOSEST_KP] = -1
        ts[ids, HM.AK_CLOSEST_FT:HM.AK_CLOSEST_FT + 4] = -1
        ts[ids, HM.AK_FURTHEST] = -1
        ts[ids, HM.AK_NEAR_GOAL] = 0
        ts[ids, HM.AK_REW_EP:HM.AK_REW_EP + 12] = 0
    # targets (:1373-1397)
    prev = st["targets"]
    cur = np.empty_like(prev)
    h = slice(NARM, D)
    cur[:, h] = F(0.5) * (actions[:, h] + F(1.0)) * (up[h] - lo[h]) + lo[h]
    cur[:, h] = F(p.ak_act_moving_average) * cur[:, h] + F(p.ak_one_minus_ama) * prev[:, h]
    cur[:, h] = np.maximum(np.minimum(cur[:, h], up[h]), lo[h])
    t = prev[:, :NARM] + F(p.ak_dof_speed_scale) * actions[:, :NARM]
    cur[:, :NARM] = np.maximum(np.minimum(t, up[:NARM]), lo[:NARM])
    st["targets"][:] = cur
    # random forces (:1399-1414)
    if p.ak_force_scale <= 0:                 # forceScale 0 (throw): no decay, no draws (:1399)
        return
    rf = st["ts"][:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3]
    rf *= F(p.ak_force_decay_step)
    sel = dr[:, ds["FORCE_U"]] < st["ts"][:, HM.AK_FORCE_PROB]
    rf[sel] = (dr[sel, ds["FORCE_N"]:ds["FORCE_N"] + 3] * F(p.ak_object_rb_mass)) * F(p.ak_force_scale)


def timeout(p, progress, reset):
    return (progress >= p.max_episode_length - 1) & (reset != 0)         # vec_task.py:424
