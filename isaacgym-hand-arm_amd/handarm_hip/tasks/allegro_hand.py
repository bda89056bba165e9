"""AllegroHand (in-hand cube reorientation) with the IsaacGymEnvs VecTask surface, backed by libhandarm_hip.

Drop-in for tasks/allegro_hand.py:40 (registered as "AllegroHand" in tasks/__init__.py). Config
cfg/task/AllegroHand.yaml: 16 DOF Allegro hand (allegro_touch_sensor.urdf, fixed base, gravity off),
one 0.065 m cube (objectType block; egg and pen too), a goal object that only carries a pose, observationType "full_state" (88 floats; "full" 72 and
"full_no_vel" 50 too, and asymmetric_observations' 88-float states buffer), absolute or relative control
(useRelativeControl, dofSpeedScale), random object forces (forceScale), controlFrequencyInv 2, episodeLength 600.

One fused kernel per step (ha_task_step -> ah_step_kernel): goal resets, reset_idx, targets (absolute with moving
average, or relative), 2 x 2 physics substeps, refresh, observations, compute_hand_reward; then a
one-thread kernel updates the global consecutive_successes average (allegro_hand.py:714-717). No host
syncs on the step path.
"""
import numpy as np
import torch

from .. import model as HM
from .. import ref_rng as RR
from ..sim import HandArmSim
from .ur5sih_multi_object_manipulation import Box


class AllegroHand:
    def __init__(self, cfg, rl_device="cuda:0", sim_device="cuda:0", graphics_device_id=-1, headless=True,
                 virtual_screen_capture=False, force_render=False):
        self.cfg = cfg
        self.rl_device = rl_device
        self.device = sim_device
        env = cfg.get("env", {})
        c = HM.ALLEGRO_TASK
        self.num_environments = int(env.get("numEnvs", 16384))
        self.num_agents = 1
        self.obs_type = env.get("observationType", "full_state")
        if self.obs_type not in HM.AH_OBS_TYPES:                      # allegro_hand.py:102-104
            raise Exception("Unknown type of observations!\nobservationType should be one of: [openai, full_no_vel, "
                            "full, full_state]")
        self.object_type = env.get("objectType", "block")
        assert self.object_type in HM.AH_OBJECT_TYPES                  # allegro_hand.py:82-83
        self.ignore_z = self.object_type == "pen"
        self.asymmetric_obs = bool(env.get("asymmetric_observations", False))
        self.use_relative_control = bool(env.get("useRelativeControl", False))
        self.control_freq_inv = int(env.get("controlFrequencyInv", c["control_freq_inv"]))
        self.clip_obs = float(env.get("clipObservations", c["clip_observations"]))
        self.clip_actions = float(env.get("clipActions", c["clip_actions"]))
        self.max_episode_length = int(env.get("episodeLength", c["max_episode_length"]))
        task_cfg = dict(task=HM.TASK_ALLEGRO_HAND, control_freq_inv=self.control_freq_inv,
                        max_episode_length=self.max_episode_length, seed=int(cfg.get("seed", 42)),
                        obs_type=self.obs_type, asymmetric=self.asymmetric_obs,
                        relative_control=self.use_relative_control, object_type=self.object_type)
        for key, name in [("distRewardScale", "dist_reward_scale"), ("rotRewardScale", "rot_reward_scale"),
                          ("rotEps", "rot_eps"), ("actionPenaltyScale", "action_penalty_scale"),
                          ("successTolerance", "success_tolerance"), ("reachGoalBonus", "reach_goal_bonus"),
                          ("fallDistance", "fall_dist"), ("fallPenalty", "fall_penalty"),
                          ("maxConsecutiveSuccesses", "max_consecutive_successes"), ("averFactor", "av_factor"),
                          ("resetPositionNoise", "reset_position_noise"),
                          ("resetDofPosRandomInterval", "reset_dof_pos_noise"),
                          ("resetDofVelRandomInterval", "reset_dof_vel_noise"),
                          ("actionsMovingAverage", "act_moving_average"), ("dofSpeedScale", "dof_speed_scale"),
                          ("forceScale", "force_scale"), ("forceDecay", "force_decay"),
                          ("forceDecayInterval", "force_decay_interval")]:
            if key in env:
                task_cfg[name] = type(c[name])(env[key])
        if "forceProbRange" in env:
            task_cfg["force_prob_range"] = tuple(float(x) for x in env["forceProbRange"])
        # task.randomize (AllegroHand.yaml:67-150): the reference's AllegroHand counts randomize_buf but never calls
        # apply_randomizations; here the same device engine as AllegroKuka's runs the schema (handarm_hip/dr.py)
        task = cfg.get("task", {}) or {}
        self.randomize = bool(task.get("randomize", False))
        if self.randomize:
            task_cfg["dr_enable"] = 1
            task_cfg["randomization_params"] = task.get("randomization_params")
        self.sim = HandArmSim(self.num_environments, sim_device, task_cfg=task_cfg, task=HM.TASK_ALLEGRO_HAND)
        self.sim_flags = 0
        N, t = self.num_environments, self.sim.t
        # numObservations by observationType, numStates 88 with asymmetric observations (allegro_hand.py:106-124)
        self.num_observations, self.num_actions = HM.AH_NUM_OBS[self.obs_type], 16
        self.num_states = HM.AH_NUM_STATES if self.asymmetric_obs else 0
        self.obs_buf = t["obs"]
        self.states_buf = t["teacher_obs"] if self.asymmetric_obs else None
        self.rew_buf = t["rew"]
        self.reset_buf = t["reset_buf"]
        self.reset_goal_buf = t["reset_goal_buf"]
        self.randomize_buf = t["randomize_buf"]           # vec_task.py:352 (counted on the device)
        self.progress_buf = t["progress_buf"]
        self.timeout_buf = t["timeout_buf"]
        self.successes = t["successes"]
        self.consecutive_successes = t["consecutive_successes"]
        self.actions_buf = t["actions"]
        self.goal_states = t["goal_state"]
        self.dof_state = t["dof_state"]
        self.dof_force_tensor = t["dof_force"].view(N, 16)
        self.root_state_tensor = t["root_state"]
        self.rigid_body_states = t["rigid_body_state"].view(N, -1, 13)
        self.prev_targets = t["dof_position_targets"]
        self.shadow_hand_dof_lower_limits = torch.tensor(list(self.sim.model.dof_lower)[:16], device=sim_device)
        self.shadow_hand_dof_upper_limits = torch.tensor(list(self.sim.model.dof_upper)[:16], device=sim_device)
        # initial state (allegro_hand.py:282-375, vec_task.py:346-347): everything resets on the first step
        r = self.root_state_tensor.view(N, 3, 13)
        r[:, 0, 0:3] = torch.tensor(list(self.sim.model.base_pos), device=sim_device)
        r[:, 0, 3:7] = torch.tensor(list(self.sim.model.base_quat), device=sim_device)
        r[:, 1, 0:7] = torch.tensor(list(self.sim.params.ah_object_init), device=sim_device)
        self.goal_states[:, 0:3] = torch.tensor(list(self.sim.params.ah_goal_init), device=sim_device)
        self.goal_states[:, 3:7] = torch.tensor([0.0, 0.0, 0.0, 1.0], device=sim_device)
        r[:, 2, 0:3] = self.goal_states[:, 0:3] + torch.tensor(c["goal_displacement"], device=sim_device)
        r[:, 2, 6] = 1.0
        self.reset_buf.fill_(1)
        self.reset_goal_buf.fill_(1)
        # seed-faithful draws (handarm_hip/ref_rng.py): every reset value from torch's global CPU generator in
        # the reference's order (the __init__ random_force_prob draw happens here, as at allegro_hand.py:193)
        self.reference_rng = bool(cfg.get("sim", {}).get("reference_rng", False))
        self._rr = RR.AllegroDraws(N, force_scale=self.sim.cfg["force_scale"],
                                   force_prob_range=self.sim.cfg["force_prob_range"]) if self.reference_rng else None
        self.extras = {}
        self.obs_dict = {}
        # obs_dict["obs"] = clamp(obs_buf) by the step launch (ha_task_step_io) into one of two alternating buffers: step t's obs
        # (and extras["consecutive_successes"], a view of the task's counter) stay valid through step t+1 and are
        # overwritten by step t+2. env.freshOutputs=True returns new tensors every step, as the reference's
        # torch.clamp / .mean() do (allegro_hand.py:393,707)
        self.fresh_outputs = bool(env.get("freshOutputs", False))
        self._obs_out = torch.zeros((2, N, self.num_observations), device=sim_device)
        self.control_steps = 0
        self.total_successes = 0
        self.total_resets = 0

    def contact_stats(self, reset=False):
        """Contact-list diagnostics of the physics since the last reset (HandArmSim.contact_stats)."""
        return self.sim.contact_stats(reset)

    # ---------------------------------------------------------------- VecTask surface
    @property
    def num_envs(self):
        return self.num_environments

    @property
    def num_obs(self):
        return self.num_observations

    @property
    def num_acts(self):
        return self.num_actions

    @property
    def observation_space(self):
        return Box(np.ones(self.num_obs) * -np.inf, np.ones(self.num_obs) * np.inf)

    @property
    def action_space(self):
        return Box(np.ones(self.num_acts) * -1.0, np.ones(self.num_acts) * 1.0)

    @property
    def state_space(self):
        return Box(np.ones(self.num_states) * -np.inf, np.ones(self.num_states) * np.inf)

    def get_number_of_agents(self):
        return self.num_agents

    def set_train_info(self, env_frames, *args, **kwargs):
        self.env_frames = env_frames

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass

    def zero_actions(self):
        return torch.zeros((self.num_envs, self.num_actions), dtype=torch.float32, device=self.rl_device)

    def step(self, actions):
        """VecTask.step (vec_task.py:390-441) -> pre_physics_step / simulate x2 / post_physics_step, fused.
        obs_dict["obs"] is valid until the step after next unless env.freshOutputs is set (see __init__)."""
        out = torch.empty_like(self._obs_out[0]) if self.fresh_outputs else self._obs_out[(self.control_steps + 1) & 1]
        # one launch: the action clamp into actions_buf (vec_task.py:400-404), the fused step and obs_dict["obs"] =
        # clamp(obs_buf) into `out` (ha_task_step_io)
        self.sim.task_step_io(self.sim_flags | self._reference_draws(), actions, self.clip_actions, out, self.clip_obs)
        self.control_steps += 1
        self.extras["time_outs"] = self.timeout_buf.view(torch.bool).to(self.rl_device)
        cs = self.consecutive_successes.view(())                                     # allegro_hand.py:393 (1 value)
        self.extras["consecutive_successes"] = cs.clone() if self.fresh_outputs else cs
        self.obs_dict["obs"] = out.to(self.rl_device)
        self._put_states()
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    def get_state(self):
        """VecTask.get_state (vec_task.py:375-376): the clamped states buffer."""
        return torch.clamp(self.states_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)

    def _put_states(self):
        if self.num_states > 0:                                        # vec_task.py:438-439,471-472,488-489
            self.obs_dict["states"] = self.get_state()

    def reset(self):
        """VecTask.reset (vec_task.py:459-474): compute_observations only."""
        self.sim.task_observe(HM.FLAG_OBS_ONLY)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        self._put_states()
        return self.obs_dict

    def reset_idx(self, env_ids, goal_env_ids=None):
        """reset_idx (allegro_hand.py:524-584) for the listed envs (and goal resets for goal_env_ids)."""
        self.reset_buf[env_ids] = 1
        if goal_env_ids is not None:
            self.reset_goal_buf[goal_env_ids] = 1
        self.sim.task_reset(self.sim_flags | self._reference_draws())

    def _reference_draws(self):
        """reference_rng: this step's reset draws on the host (one read of the reset flags), uploaded for
        HA_FLAG_REPLAY_DRAWS. Returns the extra launch flags."""
        if self._rr is None:
            return 0
        d = self._rr.step(self.reset_buf.cpu(), self.reset_goal_buf.cpu())
        self.sim.t["reset_draws"].copy_(d)
        return HM.FLAG_REPLAY_DRAWS

    def reset_done(self):
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        self._put_states()
        return self.obs_dict, done_env_ids

