"""ORACLE (test infrastructure only) - numpy restatement of the reference AllegroHand task math
(tasks/allegro_hand.py, cfg/task/AllegroHand.yaml; config C3 of BASELINE.json).

Only ``tests/`` may import this module. Pinned by ``tests/golden/allegro_*.npz``, which the
reference itself produced (``tests/golden/make_goldens_allegro.py``). float32 in the reference's
operation order.
"""
import numpy as np

from oracle import f32
from oracle.task_oracle import F, quat_conjugate, quat_mul, scale, unscale

NUM_OBS, NUM_ACT, D = 88, 16, 16
DRAW_GOAL, DRAW_RESET, DRAW_RESET_GOAL = 0, 4, 41       # ah_task.h AH_DRAW_*

CFG = dict(dist_reward_scale=-10.0, rot_reward_scale=1.0, rot_eps=0.1, action_penalty_scale=-0.0002,
           success_tolerance=0.1, reach_goal_bonus=250.0, fall_dist=0.24, fall_penalty=0.0,
           max_consecutive_successes=0, av_factor=0.1, max_episode_length=600, vel_obs_scale=0.2,
           force_torque_obs_scale=10.0, reset_position_noise=0.01, reset_dof_pos_noise=0.2,
           reset_dof_vel_noise=0.0, act_moving_average=1.0,
           object_init=(0.0, -0.2, 0.56, 0.0, 0.0, 0.0, 1.0), goal_init=(0.0, -0.2, 0.52),
           goal_displacement=(-0.2, -0.06, 0.12), obs_type="full_state", asymmetric=False, relative_control=False,
           dof_speed_scale=20.0, dt=0.01667, force_scale=0.0, force_prob_range=(0.001, 0.1), force_decay=0.99,
           force_decay_interval=0.08, object_rb_mass=0.10985)
DRAW_FORCE_PROB, DRAW_FORCE_U, DRAW_FORCE_N, DRAW_FORCE_SEL = 45, 46, 47, 50   # ah_task.h AH_DRAW_FORCE_*


def force_prob(u, c=CFG):
    """random_force_prob (allegro_hand.py:557-560): exp((log lo - log hi) u + log hi) in float32."""
    lo, hi = np.log(np.asarray(c["force_prob_range"], F)).astype(F)
    return np.exp((lo - hi) * np.asarray(u, F) + hi).astype(F)


def forces_step(force, draws, c=CFG):
    """pre_physics_step's random forces (:617-623) on force (N, 3), object frame: decay by
    torch.pow(forceDecay, dt / forceDecayInterval) (fp32), then N(0, 1)^3 * mass * forceScale for the envs the
    draws select (slot 50: the reference's torch.rand(N) < random_force_prob)."""
    import torch
    decay = F(torch.pow(torch.tensor(c["force_decay"], dtype=torch.float32), c["dt"] / c["force_decay_interval"]))
    force = (force * decay).astype(F)
    sel = draws[:, DRAW_FORCE_SEL] != 0
    force[sel] = (draws[sel, DRAW_FORCE_N:DRAW_FORCE_N + 3] * F(c["object_rb_mass"])) * F(c["force_scale"])
    return force


def _quat_from_angle_axis(angle, axis):
    """torch_jit_utils.py:118-123 for a unit axis (0: x, 1: y), as ah_task.h ah_quat_from_angle_axis evaluates it:
    the shared float32 sine / cosine (oracle/f32.py, include/ha_fmath.h), then quat_unit."""
    th = np.asarray(angle, F) / F(2.0)
    sn, cs = f32.sincos(th)
    z = F(0.0) * sn
    q = [sn if axis == 0 else z, sn if axis == 1 else z, sn if axis == 2 else z, cs]
    n = np.sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]).astype(F)
    n = np.maximum(n, F(1e-9))
    return np.stack([c / n for c in q], -1).astype(F)


def randomize_rotation(rand0, rand1):
    """allegro_hand.py:722-725 (x, then y unit axis; quat_mul of torch_jit_utils.py:41-62)."""
    pi = F(np.pi)
    return quat_mul(_quat_from_angle_axis(np.asarray(rand0, F) * pi, 0),
                    _quat_from_angle_axis(np.asarray(rand1, F) * pi, 1))


def observations(dof_pos, dof_vel, dof_force, obj, goal_state, actions, lo, up, c=CFG):
    """compute_full_state (allegro_hand.py:486-504): 88 floats."""
    N = dof_pos.shape[0]
    o = np.zeros((N, NUM_OBS), F)
    o[:, 0:16] = unscale(dof_pos, lo, up)
    o[:, 16:32] = F(c["vel_obs_scale"]) * dof_vel
    o[:, 32:48] = F(c["force_torque_obs_scale"]) * dof_force
    o[:, 48:55] = obj[:, 0:7]
    o[:, 55:58] = obj[:, 7:10]
    o[:, 58:61] = F(c["vel_obs_scale"]) * obj[:, 10:13]
    o[:, 61:68] = goal_state[:, 0:7]
    o[:, 68:72] = quat_mul(obj[:, 3:7], quat_conjugate(goal_state[:, 3:7]))
    o[:, 72:88] = actions
    return o


def observations_typed(obs_type, dof_pos, dof_vel, dof_force, obj, goal_state, actions, lo, up, c=CFG):
    """compute_observations (allegro_hand.py:425-432): compute_full_observations(no_vel) (:437-460) for "full_no_vel"
    (50 floats) and "full" (72), compute_full_state (:484-504) for "full_state" (88)."""
    if obs_type == "full_state":
        return observations(dof_pos, dof_vel, dof_force, obj, goal_state, actions, lo, up, c)
    N = dof_pos.shape[0]
    qd = quat_mul(obj[:, 3:7], quat_conjugate(goal_state[:, 3:7]))
    if obs_type == "full_no_vel":
        o = np.zeros((N, 50), F)
        o[:, 0:16] = unscale(dof_pos, lo, up)
        o[:, 16:23] = obj[:, 0:7]
        o[:, 23:30] = goal_state[:, 0:7]
        o[:, 30:34] = qd
        o[:, 34:50] = actions
        return o
    o = np.zeros((N, 72), F)
    o[:, 0:16] = unscale(dof_pos, lo, up)
    o[:, 16:32] = F(c["vel_obs_scale"]) * dof_vel
    o[:, 32:39] = obj[:, 0:7]
    o[:, 39:42] = obj[:, 7:10]
    o[:, 42:45] = F(c["vel_obs_scale"]) * obj[:, 10:13]
    o[:, 45:52] = goal_state[:, 0:7]
    o[:, 52:56] = qd
    o[:, 56:72] = actions
    return o


def reward(obj, goal_state, actions, reset_buf, reset_goal_buf, progress, successes, cons, c=CFG):
    """compute_hand_reward (allegro_hand.py:663-719). Returns reward, resets, goal_resets, progress,
    successes, consecutive_successes."""
    diff = obj[:, 0:3] - goal_state[:, 0:3]
    goal_dist = np.sqrt((diff[:, 0] * diff[:, 0] + diff[:, 1] * diff[:, 1]) + diff[:, 2] * diff[:, 2]).astype(F)
    qd = quat_mul(obj[:, 3:7], quat_conjugate(goal_state[:, 3:7]))
    rn = np.sqrt((qd[:, 0] * qd[:, 0] + qd[:, 1] * qd[:, 1]) + qd[:, 2] * qd[:, 2]).astype(F)
    rot_dist = F(2.0) * np.arcsin(np.minimum(rn, F(1.0))).astype(F)
    dist_rew = goal_dist * F(c["dist_reward_scale"])
    rot_rew = F(1.0) / (np.abs(rot_dist) + F(c["rot_eps"])) * F(c["rot_reward_scale"])
    ap = np.sum(actions * actions, -1, dtype=F)
    rew = dist_rew + rot_rew + ap * F(c["action_penalty_scale"])
    goal_resets = np.where(np.abs(rot_dist) <= F(c["success_tolerance"]), 1, reset_goal_buf).astype(np.int64)
    successes = (successes + goal_resets).astype(F)
    rew = np.where(goal_resets == 1, rew + F(c["reach_goal_bonus"]), rew)
    rew = np.where(goal_dist >= F(c["fall_dist"]), rew + F(c["fall_penalty"]), rew)
    resets = np.where(goal_dist >= F(c["fall_dist"]), 1, reset_buf).astype(np.int64)
    progress = np.asarray(progress, np.int64).copy()
    if c["max_consecutive_successes"] > 0:
        progress = np.where(np.abs(rot_dist) <= F(c["success_tolerance"]), 0, progress)
        resets = np.where(successes >= c["max_consecutive_successes"], 1, resets)
    timed_out = progress >= c["max_episode_length"] - 1
    resets = np.where(timed_out, 1, resets)
    if c["max_consecutive_successes"] > 0:
        rew = np.where(timed_out, rew + F(0.5) * F(c["fall_penalty"]), rew)
    n = resets.sum()
    fin = np.sum(successes * resets.astype(F), dtype=F)
    av = F(c["av_factor"])
    cons = F(av * fin / F(n) + (F(1.0) - av) * F(cons)) if n > 0 else F(cons)
    return rew.astype(F), resets, goal_resets, progress, successes, cons


def goal_reset(goal_state, root, env, g0, g1, c=CFG):
    """reset_target_pose for one env (allegro_hand.py:506-522); root is (N, 3, 13)."""
    rot = randomize_rotation(np.array([g0], F), np.array([g1], F))[0]
    goal_state[env, 0:3] = c["goal_init"]
    goal_state[env, 3:7] = rot
    root[env, 2, 0:3] = np.asarray(c["goal_init"], F) + np.asarray(c["goal_displacement"], F)
    root[env, 2, 3:7] = rot
    root[env, 2, 7:13] = 0


def randomize_rotation_pen(rand0):
    """allegro_hand.py:729-732 with max_angle torch.tensor(0.3): x by 0.5 pi + rand0 0.3, then z by rand0 pi."""
    r0 = np.asarray(rand0, F)
    return quat_mul(_quat_from_angle_axis(F(0.5 * np.pi) + r0 * F(0.3), 0), _quat_from_angle_axis(r0 * F(np.pi), 2))


def env_reset(root, dof_pos, dof_vel, targets, env, r, lo, up, c=CFG):
    """reset_idx body for one env (allegro_hand.py:533-579) from its 37 draws r."""
    init = np.asarray(c["object_init"], F)
    noise = F(c["reset_position_noise"])
    root[env, 1, 0:3] = init[0:3] + noise * r[0:3]
    if c.get("object_type") == "pen":
        root[env, 1, 3:7] = randomize_rotation_pen(np.array([r[3]], F))[0]
    else:
        root[env, 1, 3:7] = randomize_rotation(np.array([r[3]], F), np.array([r[4]], F))[0]
    root[env, 1, 7:13] = 0
    dmax, dmin = up - F(0), lo - F(0)
    rd = dmin + ((dmax - dmin) * F(0.5)) * (r[5:5 + D] + F(1))
    pos = F(0) + F(c["reset_dof_pos_noise"]) * rd
    dof_pos[env] = pos
    dof_vel[env] = F(0) + F(c["reset_dof_vel_noise"]) * r[5 + D:5 + 2 * D]
    targets[env] = pos


def targets_from_actions(actions, prev, lo, up, c=CFG):
    """allegro_hand.py:611-618 (absolute control, moving average, clamp)."""
    cur = scale(actions, lo, up)
    ama = F(c["act_moving_average"])
    beta = F(1.0 - c["act_moving_average"])
    cur = ama * cur + beta * prev
    return np.maximum(np.minimum(cur, up), lo).astype(F)


def targets_relative(actions, prev, lo, up, c=CFG):
    """allegro_hand.py:602-605 (useRelativeControl): prev_targets + dofSpeedScale * dt * actions, clamped; the scalar
    product is a python double, rounded once where it meets the float32 tensor."""
    cur = prev + F(c["dof_speed_scale"] * c["dt"]) * actions
    return np.maximum(np.minimum(cur, up), lo).astype(F)


def step_no_physics(st, actions, draws, lo, up, c=CFG):
    """pre_physics_step -> (no simulate) -> post_physics_step on dict st (mutated):
    dof (N,16,2), root (N,3,13), goal_state (N,7), targets (N,16), reset, reset_goal, progress, successes, cons."""
    N = actions.shape[0]
    for e in range(N):
        goal, full = st["reset_goal"][e] != 0, st["reset"][e] != 0
        if goal or full:
            base = DRAW_RESET_GOAL if full else DRAW_GOAL
            goal_reset(st["goal_state"], st["root"], e, draws[e, base], draws[e, base + 1], c)
            st["reset_goal"][e] = 0
        if full:
            env_reset(st["root"], st["dof"][..., 0], st["dof"][..., 1], st["targets"], e,
                      draws[e, DRAW_RESET:DRAW_RESET + 37], lo, up, c)
            st["progress"][e], st["reset"][e], st["successes"][e] = 0, 0, 0
            if "force" in st:                                    # rb_forces = 0, random_force_prob (:532,557-560)
                st["force"][e] = 0
                st["prob"][e] = force_prob(draws[e, DRAW_FORCE_PROB], c)
    if c.get("relative_control", False):
        st["targets"] = targets_relative(actions, st["targets"], lo, up, c)
    else:
        st["targets"] = targets_from_actions(actions, st["targets"], lo, up, c)
    if c.get("force_scale", 0.0) > 0.0:
        st["force"] = forces_step(st["force"], draws, c)
    st["progress"] = st["progress"] + 1
    args = (st["dof"][..., 0], st["dof"][..., 1], np.zeros((N, D), F), st["root"][:, 1], st["goal_state"], actions,
            lo, up, c)
    obs = observations_typed(c.get("obs_type", "full_state"), *args)
    if c.get("asymmetric", False):
        st["states"] = observations(*args)
    rew, st["reset"], st["reset_goal"], st["progress"], st["successes"], st["cons"] = reward(
        st["root"][:, 1], st["goal_state"], actions, st["reset"], st["reset_goal"], st["progress"], st["successes"],
        st["cons"], c)
    timeout = (st["progress"] >= c["max_episode_length"] - 1) & (st["reset"] != 0)
    return obs, rew, timeout
