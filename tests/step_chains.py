"""Oracle chains of the fused step kernels (test infrastructure).

One ``VecTask.step()`` of each task family, restated on the host from the oracles, in the order the fused step
kernel runs it (``csrc/handarm_hip.hip`` env_body, MODE_STEP):

* AllegroKuka (``ak_step_kernel``, allegro_kuka_base.py:1355-1447): numpy ``pre_physics_step``
  (oracle/kuka_oracle.pre: goal / env resets from replayed draws, targets, random forces), the local-space
  force rotated to world by the object's pose, ``control_freq_inv`` gym.simulate calls of the C oracle,
  progress + 1, numpy ``compute_observations`` + ``compute_kuka_reward`` (kuka_oracle.post).
* AllegroHand (``ah_step_kernel``, allegro_hand.py:586-629,663-719): goal / env resets, absolute targets,
  C-oracle physics, progress + 1, ``compute_full_state`` (with the physics' joint forces) and the reward.
* Ur5Sih, 3 objects with DR rows (``ha_step_kernel``, configurable_vec_task.py:347-414) and the 8-object clutter
  family (``hb_step_kernel``): the C oracle's controller, reset_idx for reset envs (replayed draws, DR rows from
  the device-mode hash), reset_idx's extra gym.simulate, the ``control_freq_inv`` calls, the observables, the
  DR observation noise, reward and done.

Each chain mutates an ``oracle.oracle_lib.HostState`` in place. Only tests import this module.
"""
import numpy as np

from handarm_hip import model as HM
from oracle import f32
from oracle import allegro_oracle as AO
from oracle import dr_oracle as DO
from oracle import kuka_oracle as KO
from oracle import task_oracle as TO

F = np.float32


# ----------------------------------------------------------------------------- AllegroKuka
def kuka_step(orc, hs, p, lo, up, scalars, draws):
    """ak_step_kernel on hs (HostState of the Kuka layout). Returns (obs, rew, timeout)."""
    N, D = hs.num_envs, 23
    A = orc.model.n_actors
    st = dict(dof=hs["dof_state"].reshape(N, D, 2), root=hs["root_state"].reshape(N, A, 13), goal=hs["goal_state"],
              targets=hs["dof_position_targets"], reset=hs["reset_buf"], reset_goal=hs["reset_goal_buf"],
              progress=hs["progress_buf"], successes=hs["successes"], ts=hs["task_state"])
    dr_pre(p, orc.model, hs)
    act = noisy_actions(p, hs, hs["actions"])
    # privilegedActions: torque actions 0..2; the hand reads actions[:, 3:][:, 7:23], the arm self.actions[:, :7]
    pv = 3 if p.ak_privileged_actions else 0
    eff = np.concatenate([act[:, :7], act[:, 7 + pv:23 + pv]], 1) if pv else act
    KO.pre(p, st, eff, draws, lo, up)
    hs["sim_targets"][:] = hs["dof_position_targets"]
    if pv:
        hs["object_torque"].reshape(N, 3)[:] = act[:, 0:3] * F(p.ak_privileged_torque)
    # apply_rigid_body_force_tensors(LOCAL_SPACE) at the object COM: world force = R(q_object) F_local (ak_forces)
    a0 = orc.model.actor_object0
    fl = hs["task_state"][:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3]
    fw = f32.qrot(st["root"][:, a0, 3:7], fl) if p.ak_force_scale > 0 else np.zeros((N, 3), F)
    hs["object_force"].reshape(N, 3)[:] = fw
    orc.simulate(hs, p.control_freq_inv)
    hs["progress_buf"][:] = hs["progress_buf"] + 1
    rb = hs["rigid_body_state"].reshape(N, orc.model.n_bodies, 13)[:, orc.model.body_robot0:]
    obs, rew, rs, rg, pr, sc = KO.post(p, hs["task_state"], st["dof"][..., 0], st["dof"][..., 1], rb, st["root"][:, a0],
                                       hs["goal_state"], hs["progress_buf"], hs["successes"], hs["reset_buf"],
                                       hs["object_scale"].reshape(N, 3), scalars, lo, up)
    hs["reset_buf"][:], hs["reset_goal_buf"][:], hs["progress_buf"][:], hs["successes"][:] = rs, rg, pr, sc
    if p.dr_enable:
        obs = DO.obs_noise(p, hs["dr_global"], obs)
    hs["rew"][:] = rew
    hs["obs"][:] = obs
    return obs, rew, KO.timeout(p, pr, rs)


# ----------------------------------------------------------------------------- AllegroHand
def allegro_step(orc, hs, p, lo, up, draws):
    """ah_step_kernel on hs (HostState of the AllegroHand layout). Returns (obs, rew, timeout, cons)."""
    N, D = hs.num_envs, 16
    c = dict(AO.CFG)
    c["act_moving_average"] = float(p.ah_act_moving_average)
    root = hs["root_state"].reshape(N, 3, 13)
    dof = hs["dof_state"].reshape(N, D, 2)
    dr_pre(p, orc.model, hs)
    act = noisy_actions(p, hs, hs["actions"])               # self.actions: targets, obs and the action penalty
    for e in range(N):
        goal, full = hs["reset_goal_buf"][e] != 0, hs["reset_buf"][e] != 0
        if goal or full:
            base = AO.DRAW_RESET_GOAL if full else AO.DRAW_GOAL
            AO.goal_reset(hs["goal_state"], root, e, draws[e, base], draws[e, base + 1], c)
            hs["reset_goal_buf"][e] = 0
        if full:
            AO.env_reset(root, dof[..., 0], dof[..., 1], hs["dof_position_targets"], e,
                         draws[e, AO.DRAW_RESET:AO.DRAW_RESET + 37], lo, up, c)
            hs["progress_buf"][e], hs["reset_buf"][e], hs["successes"][e] = 0, 0, 0
            hs["task_state"][e, 0:3] = 0                              # rb_forces[env_ids] = 0 (ah_task.h AH_TS_*)
    hs["dof_position_targets"][:] = AO.targets_from_actions(act, hs["dof_position_targets"], lo, up, c)
    hs["sim_targets"][:] = hs["dof_position_targets"]
    if p.ah_force_scale > 0:
        # random forces (ah_forces, replayed selection): decay, new N(0,1)^3 * mass * scale, LOCAL_SPACE -> world force
        # of the step's first physics call (the oracle's simulate applies object_force to its first call only)
        f = hs["task_state"][:, 0:3] * F(p.ah_force_decay_step)
        sel = draws[:, AO.DRAW_FORCE_SEL] != 0
        f[sel] = (draws[sel, AO.DRAW_FORCE_N:AO.DRAW_FORCE_N + 3] * F(p.ah_object_rb_mass)) * F(p.ah_force_scale)
        hs["task_state"][:, 0:3] = f
        hs["object_force"].reshape(N, 3)[:] = f32.qrot(root[:, 1, 3:7], f)
    orc.simulate(hs, p.control_freq_inv)
    hs["progress_buf"][:] = hs["progress_buf"] + 1
    obs = AO.observations(dof[..., 0], dof[..., 1], hs["dof_force"], root[:, 1], hs["goal_state"], act, lo, up, c)
    rew, rs, rg, pr, sc, cons = AO.reward(root[:, 1], hs["goal_state"], act, hs["reset_buf"],
                                          hs["reset_goal_buf"], hs["progress_buf"], hs["successes"],
                                          hs["consecutive_successes"][0], c)
    hs["reset_buf"][:], hs["reset_goal_buf"][:], hs["progress_buf"][:], hs["successes"][:] = rs, rg, pr, sc
    hs["consecutive_successes"][0] = cons
    if p.dr_enable:
        obs = DO.obs_noise(p, hs["dr_global"], obs)
    hs["rew"][:] = rew
    hs["obs"][:] = obs
    timeout = (pr >= c["max_episode_length"] - 1) & (rs != 0)
    return obs, rew, timeout, cons


# ----------------------------------------------------------------------------- Ur5Sih (3 objects / clutter)
def dr_pre(p, model, hs, mode=0, full=None):
    """The DR launch that precedes a step / reset launch (ha_dr_global_kernel) and each env's dr_env_pre, on hs
    (oracle/dr_oracle.py). full: the envs being reset (default: reset_buf). Returns the envs that sampled."""
    if not p.dr_enable:
        return None
    N = hs.num_envs
    full = (hs["reset_buf"] != 0) if full is None else np.asarray(full, bool)
    DO.global_update(p, hs["dr_global"], bool(full.any()), mode)
    pools = hs["object_indices"].reshape(N, -1)
    all_ = hs["dr_global"].view(np.int32)[HM.DRG_ALL] != 0
    smp = DO.env_pre(p, model, hs["dr_scale"], hs["randomize_buf"], hs["episode"], pools, full, hs["dr_global"],
                     mode == 0)
    if DO.active(p, HM.DRA_OBJ_SCALE, all_) and hs["contact_cache"] is not None and hs["contact_cache"].size:
        hs["contact_cache"][smp, :, 3] = 0            # a rescaled object's persistent manifolds are void
    return smp


def noisy_actions(p, hs, raw):
    """act_at's action noise (oracle/dr_oracle.py act_noise) on the raw actions of this step."""
    return DO.act_noise(p, hs["dr_global"], raw) if p.dr_enable else np.asarray(raw, F)


def ur5sih_step(orc, hs, p, model, draws):
    """ha_step_kernel / hb_step_kernel on hs (replayed reset draws: [0] configuration, [1] target object,
    [2:5] goal noise). Returns (teacher_obs, obs, rew, timeout)."""
    N, D, NO = hs.num_envs, 17, int(p.n_objects)
    A, B = model.n_actors, model.n_bodies
    a0 = model.actor_object0
    actors = np.arange(a0, a0 + NO)
    dr_pre(p, model, hs)
    raw = hs["actions"].copy()
    hs["actions"][:] = noisy_actions(p, hs, raw)          # the controller reads them through act_at
    orc.controller(hs)
    hs["actions"][:] = raw
    root = hs["root_state"].reshape(N, A, 13)
    dof = hs["dof_state"].reshape(N, D, 2)
    resets = np.nonzero(hs["reset_buf"])[0]
    if len(resets):
        cfgs = np.clip(draws[resets, 0].astype(np.int64), 0, int(p.num_initial_poses) - 1)
        tgts = np.clip(draws[resets, 1].astype(np.int64), 0, NO - 1)
        for i, e in enumerate(resets):
            cfg = cfgs[i]
            pos0 = hs["object_pos_initial"][e, cfg]
            quat0 = hs["object_quat_initial"][e, cfg]
            root[e, actors, 0:3] = pos0
            root[e, actors, 3:7] = quat0
            root[e, actors, 7:13] = 0
            g = np.array(p.goal_pos, F) + (F(2.0) * (draws[e, 2:5].astype(F) - F(0.5))) * np.array(p.goal_noise, F)
            hs["goal_pos"][e] = g
            root[e, model.actor_goal, 0:3] = g
            hs["target_object_index"][e] = tgts[i]
            hs["object_configuration_indices"][e] = cfg
            hs["servo"][e] = np.array(p.servo_upper, F)
            hs["smoothed"][e] = 0
            rp = np.array(list(p.reset_pose)[:D], F)
            dof[e, :, 0] = rp
            dof[e, :, 1] = 0
            hs["sim_targets"][e] = rp
            tt = rp.copy()
            tt[6:] = 0
            hs["dof_position_targets"][e] = tt
            # reset_idx's gym.simulate, then the step's control_freq_inv calls: the kernel keeps the env's state in
            # LDS across them (no round trip through the root-state tensor, as PhysX keeps its bodies between
            # calls), so the oracle runs them as one 1 + control_freq_inv call sequence; the joint positions after
            # the first call set ur5_target (ur5sih.py:388-389)
            probe = hs.copy()
            orc.simulate(probe, 1, begin=int(e), end=int(e) + 1)
            hs["ur5_target"][e] = probe["dof_state"].reshape(N, D, 2)[e, 0:6, 0]
            orc.simulate(hs, 1 + p.control_freq_inv, begin=int(e), end=int(e) + 1)
            hs["reset_buf"][e] = 0
            hs["progress_buf"][e] = 0
            hs["goal_reached_before"][e] = 0
            hs["episode"][e] = hs["episode"][e] + 1
    for e in np.nonzero(~np.isin(np.arange(N), resets))[0]:
        orc.simulate(hs, p.control_freq_inv, begin=int(e), end=int(e) + 1)
    body = hs["rigid_body_state"].reshape(N, B, 13)
    pid = hs["object_indices"]
    bb = lambda arr: np.array([[list(arr[i]) for i in row] for row in pid], F)       # noqa: E731
    teacher, _ = TO.observations(root, body, dof, hs["dof_position_targets"], hs["goal_pos"], hs["target_object_index"],
                                 bb(model.pool_bbox_pos), bb(model.pool_bbox_quat), bb(model.pool_bbox_ext),
                                 hs["obs_cache"], object_actors=actors)
    obs = DO.obs_noise(p, hs["dr_global"], teacher) if p.dr_enable else teacher.copy()
    hs["obs_cache"][:] = root[:, actors, 0:7]
    prog = hs["progress_buf"] + 1
    hs["progress_buf"][:] = prog
    rs = np.where(prog >= p.max_episode_length, 1, hs["reset_buf"]).astype(np.int64)
    timeout = (prog >= p.max_episode_length - 1) & (rs != 0)
    hs["reset_buf"][:] = rs
    rew, reached, _ = TO.reward(root, body, hs["goal_pos"], hs["target_object_index"],
                                hs["object_configuration_indices"], hs["object_pos_initial"], object_actors=actors)
    hs["goal_reached_before"][:] = (hs["goal_reached_before"] != 0) | reached
    hs["rew"][:] = rew
    return teacher, obs, rew, timeout

