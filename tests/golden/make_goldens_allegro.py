#!/usr/bin/env python3
"""Golden vectors for the AllegroHand task (config C3) by RUNNING THE REFERENCE (tasks/allegro_hand.py).

Run in the build container only (needs /root/reference):  python tests/golden/make_goldens_allegro.py
Writes ``allegro_*.npz`` (data only) next to this file.

Reference code exercised, unmodified, through a fake ``self`` carrying what ``_create_envs`` /
``VecTask.__init__`` would have allocated:
  * ``compute_observations`` -> ``compute_full_state`` (allegro_hand.py:406-504), ``compute_reward`` ->
    the jit ``compute_hand_reward`` (:384-404, 663-719): ``allegro_obs_reward.npz``;
  * ``pre_physics_step`` (:586-625) with ``reset_target_pose`` (:506-522) and ``reset_idx`` (:524-584),
    then ``post_physics_step`` (:627-633) and VecTask.step's timeout rule (vec_task.py:424), over several
    steps with goal and env resets: ``allegro_steps.npz``. ``torch_rand_float`` is wrapped to record its
    draws per env in the order the device replays them (ah_task.h AH_DRAW_*).
  * the same steps run with observationType "full" + useRelativeControl, "full_no_vel" + asymmetric_observations,
    objectType egg and pen (:82-97, 295-296, 542-546, 675-676) and forceScale 1 (:99-124, 425-504, 557-560, 602-605, 617-623; torch.rand / torch.randn recorded too):
    ``allegro_variants.npz`` (``--variants`` writes only it).
``gym.simulate`` is a no-op in the fake gym: these goldens pin the task math only.
"""
import json
import os
import sys
from unittest import mock

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402

SCENE = os.path.join(HERE, "..", "..", "isaacgym-hand-arm_amd", "handarm_hip", "assets", "allegro_hand_scene.json")
DRAW_STRIDE = 48


def make_task(N, seed=0):
    mod = refload.load("isaacgymenvs.tasks.allegro_hand")
    scene = json.load(open(SCENE))
    dofs = scene["robot"]["dofs"]
    D = len(dofs)
    t = object.__new__(mod.AllegroHand)
    # cfg/task/AllegroHand.yaml values (allegro_hand.py:44-80)
    t.cfg = {"env": {"numEnvs": N}}
    t.dist_reward_scale, t.rot_reward_scale, t.rot_eps = -10.0, 1.0, 0.1
    t.action_penalty_scale, t.success_tolerance, t.reach_goal_bonus = -0.0002, 0.1, 250.0
    t.fall_dist, t.fall_penalty = 0.24, 0.0
    t.vel_obs_scale, t.force_torque_obs_scale = 0.2, 10.0
    t.reset_position_noise, t.reset_rotation_noise = 0.01, 0.0
    t.reset_dof_pos_noise, t.reset_dof_vel_noise = 0.2, 0.0
    t.force_scale, t.force_prob_range, t.force_decay, t.force_decay_interval = 0.0, torch.tensor([0.001, 0.1]), \
        torch.tensor(0.99), 0.08
    t.shadow_hand_dof_speed_scale, t.use_relative_control, t.act_moving_average = 20.0, False, 1.0
    t.max_episode_length, t.max_consecutive_successes = 600, 0
    t.av_factor = torch.tensor(0.1)
    t.object_type, t.obs_type, t.asymmetric_obs = "block", "full_state", False
    t.print_success_stat, t.debug_viz, t.viewer = False, False, None
    t.num_environments, t.device, t.up_axis_idx, t.dt = N, "cpu", 2, 0.01667
    t.num_shadow_hand_dofs, t.num_actions = D, 16
    t.num_observations = 88
    t.actuated_dof_indices = torch.arange(D)
    t.shadow_hand_dof_lower_limits = torch.tensor([d["lower"] for d in dofs], dtype=torch.float32)
    t.shadow_hand_dof_upper_limits = torch.tensor([d["upper"] for d in dofs], dtype=torch.float32)
    t.shadow_hand_dof_default_pos = torch.zeros(D)
    t.shadow_hand_default_dof_pos = torch.zeros(D)
    t.shadow_hand_dof_default_vel = torch.zeros(D)
    t.gym, t.sim = mock.MagicMock(), None
    # _create_envs (allegro_hand.py:282-375): actor order hand 0, object 1, goal 2
    t.hand_indices = torch.arange(N) * 3
    t.object_indices = torch.arange(N) * 3 + 1
    t.goal_object_indices = torch.arange(N) * 3 + 2
    init = torch.tensor([0.0, -0.2, 0.56, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0])
    t.object_init_state = init.repeat(N, 1)
    t.goal_states = t.object_init_state.clone()
    t.goal_states[:, 2] -= 0.04
    t.goal_init_state = t.goal_states.clone()
    t.goal_displacement_tensor = torch.tensor([-0.2, -0.06, 0.12])
    t.root_state_tensor = torch.zeros(N * 3, 13)
    t.root_state_tensor[:, 6] = 1.0
    t.dof_state = torch.zeros(N * D, 2)
    t.shadow_hand_dof_state = t.dof_state.view(N, -1, 2)[:, :D]
    t.shadow_hand_dof_pos = t.shadow_hand_dof_state[..., 0]
    t.shadow_hand_dof_vel = t.shadow_hand_dof_state[..., 1]
    t.dof_force_tensor = torch.zeros(N, D)
    t.prev_targets = torch.zeros(N, D)
    t.cur_targets = torch.zeros(N, D)
    t.x_unit_tensor = torch.tensor([1.0, 0, 0]).repeat(N, 1)
    t.y_unit_tensor = torch.tensor([0, 1.0, 0]).repeat(N, 1)
    t.z_unit_tensor = torch.tensor([0, 0, 1.0]).repeat(N, 1)
    # VecTask.allocate_buffers
    t.obs_buf = torch.zeros(N, 88)
    t.rew_buf = torch.zeros(N)
    t.reset_buf = torch.ones(N, dtype=torch.long)
    t.timeout_buf = torch.zeros(N, dtype=torch.long)
    t.progress_buf = torch.zeros(N, dtype=torch.long)
    t.randomize_buf = torch.zeros(N, dtype=torch.long)
    t.reset_goal_buf = t.reset_buf.clone()
    t.successes = torch.zeros(N)
    t.consecutive_successes = torch.zeros(1)
    t.extras = {}
    # allegro_hand.py:191-194: the __init__ draw from the global generator (the first draw of a seeded run)
    t.force_prob_range = torch.tensor([0.001, 0.1])
    t.random_force_prob = torch.exp((torch.log(t.force_prob_range[0]) - torch.log(t.force_prob_range[1]))
                                    * torch.rand(N) + torch.log(t.force_prob_range[1]))
    t.rb_forces = torch.zeros(N, 19, 3)
    t.object_rb_handles = torch.tensor([17])
    t.object_rb_masses = torch.tensor([0.10985])
    return mod, t


def obs_reward(N=32, steps=5, seed=1):
    torch.manual_seed(seed)
    mod, t = make_task(N)
    g = torch.Generator().manual_seed(seed)
    lo, up = t.shadow_hand_dof_lower_limits, t.shadow_hand_dof_upper_limits
    out = {k: [] for k in ["dof_state", "dof_force", "root_state", "goal_state", "actions", "reset_in",
                           "reset_goal_in", "progress_in", "successes_in", "cons_in", "obs", "rew", "reset",
                           "reset_goal", "progress", "successes", "cons"]}
    for s in range(steps):
        q = lo + (up - lo) * torch.rand(N, 16, generator=g)
        t.shadow_hand_dof_pos[:] = q
        t.shadow_hand_dof_vel[:] = torch.randn(N, 16, generator=g)
        t.dof_force_tensor[:] = 0.3 * torch.randn(N, 16, generator=g)
        r = t.root_state_tensor.view(N, 3, 13)
        r[:, 1, 0:3] = torch.tensor([0.0, -0.2, 0.56]) + 0.15 * torch.randn(N, 3, generator=g)
        qo = torch.randn(N, 4, generator=g)
        r[:, 1, 3:7] = qo / qo.norm(dim=-1, keepdim=True)
        r[:, 1, 7:13] = torch.randn(N, 6, generator=g)
        gq = torch.randn(N, 4, generator=g)
        gq = gq / gq.norm(dim=-1, keepdim=True)
        # a few envs right at the goal orientation (successes) and some far away (falls)
        near = torch.rand(N, generator=g) < 0.2
        gq[near] = r[near, 1, 3:7]
        t.goal_states[:, 3:7] = gq
        t.actions = 2 * torch.rand(N, 16, generator=g) - 1
        t.reset_buf[:] = (torch.rand(N, generator=g) < 0.1).long()
        t.reset_goal_buf[:] = (torch.rand(N, generator=g) < 0.1).long()
        t.progress_buf[:] = torch.randint(0, 600, (N,), generator=g)
        t.progress_buf[:3] = 599
        t.successes[:] = torch.randint(0, 5, (N,), generator=g).float()
        for k, v in [("dof_state", t.dof_state), ("dof_force", t.dof_force_tensor), ("root_state", t.root_state_tensor),
                     ("goal_state", t.goal_states[:, 0:7]), ("actions", t.actions), ("reset_in", t.reset_buf),
                     ("reset_goal_in", t.reset_goal_buf), ("progress_in", t.progress_buf),
                     ("successes_in", t.successes), ("cons_in", t.consecutive_successes)]:
            out[k].append(v.clone().numpy())
        t.compute_observations()
        t.compute_reward(t.actions)
        for k, v in [("obs", t.obs_buf), ("rew", t.rew_buf), ("reset", t.reset_buf), ("reset_goal", t.reset_goal_buf),
                     ("progress", t.progress_buf), ("successes", t.successes), ("cons", t.consecutive_successes)]:
            out[k].append(v.clone().numpy())
    np.savez_compressed(os.path.join(HERE, "allegro_obs_reward.npz"), **{k: np.stack(v) for k, v in out.items()})


VARIANTS = {  # the allegro_variants.npz runs: (observationType, asymmetric_observations, useRelativeControl, forceScale,
    #            objectType)
    "full_rel": ("full", False, True, 0.0, "block"),
    "novel_asym": ("full_no_vel", True, False, 0.0, "block"),
    "force": ("full_state", False, False, 1.0, "block"),
    "egg": ("full_state", False, False, 0.0, "egg"),
    "pen": ("full_state", False, False, 0.0, "pen"),
}
FORCE_STRIDE = 51            # draw slots with the random-force draws (ah_task.h AH_DRAW_FORCE_*)


def steps(N=24, T=8, seed=2, variant=None):
    """pre_physics_step -> (no physics) -> post_physics_step, with replayable draws. variant: a VARIANTS key (the
    task's obs_type / asymmetric_obs / use_relative_control set as allegro_hand.py:99-124 would; returns the arrays)."""
    torch.manual_seed(seed)          # seeded before the task is built: __init__'s draw is part of the stream
    mod, t = make_task(N)
    if variant is not None:
        t.obs_type, t.asymmetric_obs, t.use_relative_control, t.force_scale, t.object_type = VARIANTS[variant]
        if t.object_type == "pen":
            # object_start_pose.p.z = hand z + 0.02 (:295-296), goal_states = object - 0.04 z (:363-365)
            t.object_init_state[:, 2] = float(np.float32(0.5 + 0.02))
            t.goal_states = t.object_init_state.clone()
            t.goal_states[:, 2] -= 0.04
            t.goal_init_state = t.goal_states.clone()
        t.num_observations = {"full_no_vel": 50, "full": 72, "full_state": 88}[t.obs_type]
        t.obs_buf = torch.zeros(N, t.num_observations)
        t.num_states = 88 if t.asymmetric_obs else 0
        t.states_buf = torch.zeros(N, 88)
    g = torch.Generator().manual_seed(seed)
    draws = np.zeros((T, N, DRAW_STRIDE if variant is None else FORCE_STRIDE), np.float32)
    cur = {"step": 0, "phase": None, "ids": None}
    real = getattr(mod, "_real_torch_rand_float", mod.torch_rand_float)     # (a previous run left its wrapper)
    mod._real_torch_rand_float = real

    def rec(lower, upper, shape, device):
        v = real(lower, upper, shape, device)
        ids = cur["ids"]
        base = {"goal": 0, "reset": 4, "reset_goal": 41}[cur["phase"]]
        draws[cur["step"], ids.numpy(), base:base + shape[1]] = v.numpy()
        if cur["phase"] == "reset":
            cur["phase"] = "reset_goal"      # the next draw in reset_idx is reset_target_pose(env_ids)
        return v
    mod.torch_rand_float = rec
    orig_rtp, orig_ri = t.reset_target_pose, t.reset_idx

    def rtp(env_ids, apply_reset=False):
        if cur["phase"] is None:
            cur["phase"], cur["ids"] = "goal", env_ids
        else:
            cur["ids"] = env_ids
        return orig_rtp(env_ids, apply_reset)

    def ri(env_ids, goal_env_ids):
        cur["phase"], cur["ids"] = "reset", env_ids
        r = orig_ri(env_ids, goal_env_ids)
        cur["phase"] = "after_reset"             # (the force block's torch.rand follows)
        return r
    t.reset_target_pose, t.reset_idx = rtp, ri
    keys = ["dof_state", "root_state", "goal_state", "targets", "actions", "reset_in", "reset_goal_in",
            "progress_in", "successes_in", "obs", "rew", "reset", "reset_goal", "progress", "successes", "timeout",
            "cons"]
    out = {k: [] for k in keys + ["targets_after", "dof_after", "root_after"]}
    for s in range(T):
        cur["step"], cur["phase"] = s, None
        if s > 0:   # perturb the object so goal successes / falls / timeouts happen
            r = t.root_state_tensor.view(N, 3, 13)
            r[:, 1, 0:3] += 0.06 * torch.randn(N, 3, generator=g)
            sel = torch.rand(N, generator=g) < 0.3
            r[sel, 1, 3:7] = t.goal_states[sel, 3:7]
            t.progress_buf[torch.rand(N, generator=g) < 0.1] = 598
        actions = 2 * torch.rand(N, 16, generator=g) - 1
        for k, v in [("dof_state", t.dof_state), ("root_state", t.root_state_tensor), ("goal_state", t.goal_states[:, 0:7]),
                     ("targets", t.prev_targets), ("reset_in", t.reset_buf), ("reset_goal_in", t.reset_goal_buf),
                     ("progress_in", t.progress_buf), ("successes_in", t.successes)]:
            out[k].append(v.clone().numpy())
        out["actions"].append(actions.clone().numpy())
        if variant is None:
            t.pre_physics_step(actions)
        else:
            # torch.rand / torch.randn of pre_physics_step: random_force_prob inside reset_idx (:559-560, after its
            # reset_target_pose), the force selection torch.rand(num_envs) and the selected envs' torch.randn (:621-623)
            real_rand, real_randn = torch.rand, torch.randn
            sel = {}

            def rand_rec(*a, **kw):
                v = real_rand(*a, **kw)
                if cur["phase"] == "reset_goal":
                    draws[cur["step"], cur["ids"].numpy(), 45] = v.numpy()
                else:
                    draws[cur["step"], :, 46] = v.numpy()
                    sel["ids"] = (v < t.random_force_prob).nonzero(as_tuple=False)[:, 0].numpy()
                return v

            def randn_rec(*a, **kw):
                v = real_randn(*a, **kw)
                ids = sel["ids"]
                draws[cur["step"], ids, 47:50] = v.reshape(len(ids), 3).numpy()
                draws[cur["step"], ids, 50] = 1.0
                return v
            with mock.patch.object(torch, "rand", rand_rec), mock.patch.object(torch, "randn", randn_rec):
                t.pre_physics_step(actions)
            out.setdefault("force_after", []).append(t.rb_forces[:, 17, :].clone().numpy())
            out.setdefault("prob_after", []).append(t.random_force_prob.clone().numpy())
        cur["phase"] = None
        t.post_physics_step()
        t.timeout_buf = (t.progress_buf >= t.max_episode_length - 1) & (t.reset_buf != 0)   # vec_task.py:424
        for k, v in [("obs", t.obs_buf), ("rew", t.rew_buf), ("reset", t.reset_buf), ("reset_goal", t.reset_goal_buf),
                     ("progress", t.progress_buf), ("successes", t.successes), ("timeout", t.timeout_buf),
                     ("cons", t.consecutive_successes), ("targets_after", t.prev_targets), ("dof_after", t.dof_state),
                     ("root_after", t.root_state_tensor)]:
            out[k].append(v.clone().numpy())
        if variant is not None:
            out.setdefault("states", []).append(t.states_buf.clone().numpy())
    res = {k: np.stack(v) for k, v in out.items()}
    res["draws"] = draws
    res["seed"] = np.array(seed)
    if variant is not None:
        return res
    np.savez_compressed(os.path.join(HERE, "allegro_steps.npz"), **res)


def variants():
    """allegro_variants.npz: the steps run per VARIANTS entry, keys '<variant>/<array>'."""
    out = {}
    for v in VARIANTS:
        for k, a in steps(variant=v, seed=5).items():
            out[v + "/" + k] = a
    np.savez_compressed(os.path.join(HERE, "allegro_variants.npz"), **out)


if __name__ == "__main__":
    refload.install()
    if "--variants" not in sys.argv:
        obs_reward()
        steps()
        print("wrote allegro_obs_reward.npz, allegro_steps.npz")
    variants()
    print("wrote allegro_variants.npz")
