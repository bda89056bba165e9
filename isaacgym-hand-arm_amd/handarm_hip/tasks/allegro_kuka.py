"""AllegroKuka (KUKA iiwa7 + Allegro hand, 23 DOF) with the IsaacGymEnvs VecTask surface, backed by
libhandarm_hip.

Drop-in for tasks/allegro_kuka/allegro_kuka_regrasping.py:38, allegro_kuka_reorientation.py:41 and
allegro_kuka_throw.py:39 (registered as "AllegroKukaRegrasping" / "AllegroKukaReorientation" /
"AllegroKukaThrow" in tasks/__init__.py, and as "AllegroKuka" with the subtask picked by cfg env.subtask like
tasks/__init__.py's resolver). Config cfg/task/AllegroKuka.yaml +
env/<subtask>.yaml: observationType "full_state" (93 + 6 x keypoints floats, clamped to +-10), procedurally
generated cuboids (947 sizes, env i gets size i % 947; throw: 654 small ones), random object forces, tolerance
curriculum. Throw adds the bucket (a per-env fixed-base actor whose convex pieces the physics collides with).

One fused kernel per step (ha_task_step -> ak_step_kernel): goal resets, reset_idx, hand/arm targets, random
forces, 1 x 2 physics substeps, refresh, full_state observations, compute_kuka_reward and resets. The host only
runs the tolerance curriculum (allegro_kuka_utils.py:86-119), which reads prev_episode_successes once per
curriculum interval (3000 steps); no other host sync on the step path.
"""
import numpy as np
import torch

from .. import model as HM
from .. import ref_rng as RR
from .. import state_files as SF
from ..sim import HandArmSim
from .ur5sih_multi_object_manipulation import Box


def tolerance_curriculum(last_curriculum_update, frames_since_restart, curriculum_interval, mean_prev_successes,
                         success_tolerance, initial_tolerance, target_tolerance, increment):
    """allegro_kuka_utils.py:86-119: returns (new tolerance, new last_curriculum_update)."""
    if frames_since_restart - last_curriculum_update < curriculum_interval:
        return success_tolerance, last_curriculum_update
    if mean_prev_successes < 3.0:
        return success_tolerance, last_curriculum_update
    success_tolerance *= increment
    success_tolerance = min(success_tolerance, initial_tolerance)
    success_tolerance = max(success_tolerance, target_tolerance)
    return success_tolerance, frames_since_restart


class AllegroKuka:
    # cfg key (AllegroKuka.yaml) -> model.ALLEGRO_KUKA_TASK key
    CFG_KEYS = [("liftingRewScale", "lifting_rew_scale"), ("liftingBonus", "lifting_bonus"),
                ("liftingBonusThreshold", "lifting_bonus_threshold"), ("keypointRewScale", "keypoint_rew_scale"),
                ("distanceDeltaRewScale", "distance_delta_rew_scale"), ("reachGoalBonus", "reach_goal_bonus"),
                ("kukaActionsPenaltyScale", "kuka_actions_penalty_scale"),
                ("allegroActionsPenaltyScale", "allegro_actions_penalty_scale"), ("dofSpeedScale", "dof_speed_scale"),
                ("actionsMovingAverage", "act_moving_average"), ("keypointScale", "keypoint_scale"),
                ("objectBaseSize", "object_base_size"), ("successTolerance", "success_tolerance"),
                ("targetSuccessTolerance", "target_success_tolerance"),
                ("toleranceCurriculumIncrement", "tolerance_curriculum_increment"),
                ("toleranceCurriculumInterval", "tolerance_curriculum_interval"),
                ("maxConsecutiveSuccesses", "max_consecutive_successes"),
                ("clampAbsObservations", "clamp_abs_observations"), ("forceScale", "force_scale"),
                ("forceDecay", "force_decay"), ("forceDecayInterval", "force_decay_interval"),
                ("resetDofPosRandomIntervalFingers", "reset_dof_pos_noise_fingers"),
                ("resetDofPosRandomIntervalArm", "reset_dof_pos_noise_arm"),
                ("resetDofVelRandomInterval", "reset_dof_vel_noise")]

    def __init__(self, cfg, rl_device="cuda:0", sim_device="cuda:0", graphics_device_id=-1, headless=True,
                 virtual_screen_capture=False, force_render=False, subtask=None):
        self.cfg = cfg
        self.rl_device = rl_device
        self.device = sim_device
        env = cfg.get("env", {})
        c = HM.ALLEGRO_KUKA_TASK
        sub = subtask or env.get("subtask") or c["subtask"]
        if env.get("observationType", "full_state") != "full_state" or env.get("objectType", "block") != "block":
            raise NotImplementedError("observationType 'full_state' and objectType 'block' (the AllegroKuka.yaml "
                                      "values) are implemented")
        if env.get("useRelativeControl", False):       # the reference's own answer (allegro_kuka_base.py:1373-1374)
            raise NotImplementedError("Use relative control False for now")
        if env.get("randomizeObjectDimensions", True) is False:
            raise NotImplementedError("only the AllegroKuka.yaml default for object dimensions is implemented")
        family = (True, False, False) if sub == "throw" else (True, True, True)      # env/throw.yaml:15-18
        if tuple(bool(env.get(k, d)) for k, d in zip(("withSmallCuboids", "withBigCuboids", "withSticks"), family)) \
                != family:
            raise NotImplementedError(f"the {sub} subtask's cuboid family (withSmallCuboids / withBigCuboids / "
                                      f"withSticks = {family}) is the one implemented")
        self.num_environments = int(env.get("numEnvs", 8192))
        self.num_agents = 1
        task_cfg = dict(task=HM.TASK_ALLEGRO_KUKA, subtask=sub, seed=int(cfg.get("seed", 42)))
        for key, name in self.CFG_KEYS:
            if key in env:
                task_cfg[name] = type(c[name])(env[key])
        if "episodeLength" in env:
            task_cfg["max_episode_length_override"] = int(env["episodeLength"])
        if "successSteps" in env:
            task_cfg["success_steps"] = int(env["successSteps"])
        if "resetPositionNoiseX" in env:
            task_cfg["reset_position_noise"] = (float(env["resetPositionNoiseX"]), float(env["resetPositionNoiseY"]),
                                                float(env["resetPositionNoiseZ"]))
        if "forceProbRange" in env:
            task_cfg["force_prob_range"] = tuple(float(x) for x in env["forceProbRange"])
        # privilegedActions / privilegedActionsTorque (AllegroKuka.yaml:54-55, allegro_kuka_base.py:62-74): 3 object
        # torque actions ahead of the 23
        self.privileged_actions = bool(env.get("privilegedActions", False))
        task_cfg["privileged_actions"] = self.privileged_actions
        task_cfg["privileged_actions_torque"] = float(env.get("privilegedActionsTorque", 0.02))
        # task.randomize / task.randomization_params (AllegroKuka.yaml:115-207): apply_randomizations from reset_idx
        # (allegro_kuka_base.py:1248-1249), on the device (handarm_hip/dr.py, csrc/ha_dr.h)
        task = cfg.get("task", {}) or {}
        self.randomize = bool(task.get("randomize", False))
        if self.randomize:
            task_cfg["dr_enable"] = 1
            task_cfg["randomization_params"] = task.get("randomization_params")
        self.sim = HandArmSim(self.num_environments, sim_device, task_cfg=task_cfg, task=HM.TASK_ALLEGRO_KUKA)
        self.tcfg = self.sim.cfg
        p = self.sim.params
        self.subtask = sub
        if sub == "throw":
            # the bucket actors (allegro_kuka_throw.py:77-82): root_state rows n_actors e + actor 3, rigid body 26
            self.bucket_object_indices = torch.arange(self.num_environments, device=sim_device) * \
                self.sim.model.n_actors + self.sim.model.actor_goal
        self.clip_obs = float(env.get("clipObservations", np.inf))
        self.clip_actions = float(env.get("clipActions", np.inf))
        self.max_episode_length = p.max_episode_length
        self.sim_flags = 0
        N, t = self.num_environments, self.sim.t
        self.num_observations = self.num_states = p.num_obs
        self.num_actions = p.num_actions                # 23, or 26 with privilegedActions
        self.obs_buf = t["obs"]
        self.states_buf = torch.zeros((N, self.num_states), device=sim_device)    # allocated, never written
        self.rew_buf = t["rew"]
        self.reset_buf = t["reset_buf"]
        self.reset_goal_buf = t["reset_goal_buf"]
        self.randomize_buf = t["randomize_buf"]           # vec_task.py:352 (counted on the device)
        self.progress_buf = t["progress_buf"]
        self.timeout_buf = t["timeout_buf"]
        self.successes = t["successes"]
        self.actions_buf = t["actions"]
        self.goal_states = t["goal_state"]
        self.dof_state = t["dof_state"]
        self.root_state_tensor = t["root_state"]
        self.rigid_body_states = t["rigid_body_state"].view(N, -1, 13)
        self.prev_targets = t["dof_position_targets"]
        self.object_scales = t["object_scale"].view(N, 3)
        ts = t["task_state"]
        self.task_state = ts
        self.prev_episode_successes = ts[:, HM.AK_PREV_SUCC]
        self.true_objective = ts[:, HM.AK_TRUE_OBJ]
        self.prev_episode_true_objective = ts[:, HM.AK_PREV_TRUE_OBJ]
        self.lifted_object = ts[:, HM.AK_LIFTED]
        self.random_force_prob = ts[:, HM.AK_FORCE_PROB]
        self.rewards_episode = {k: ts[:, HM.AK_REW_EP + i] for i, k in enumerate(HM.AK_REWARD_KEYS)}
        self.arm_hand_dof_lower_limits = torch.tensor(list(self.sim.model.dof_lower)[:23], device=sim_device)
        self.arm_hand_dof_upper_limits = torch.tensor(list(self.sim.model.dof_upper)[:23], device=sim_device)
        self.initial_tolerance = self.success_tolerance = float(self.tcfg["success_tolerance"])
        self.target_tolerance = float(self.tcfg["target_success_tolerance"])
        self.last_curriculum_update = 0
        self.frame_since_restart = 0
        self.extras = {}
        self.obs_dict = {}
        # step tail (in the step launch, ha_task_step_io): obs_dict["obs"] = clamp(obs_buf) and the extras means
        # (successes, true_objective mean/min/max). Lifetime: by default they land in one of two alternating
        # buffers, so the tensors step t returns stay valid through step t+1 and are overwritten by step t+2 (no
        # allocation per step). env.freshOutputs=True gives every step new tensors, as the reference's
        # torch.clamp / .mean() do (allegro_kuka_base.py:908-917,1445), for a consumer that keeps them longer
        self.fresh_outputs = bool(env.get("freshOutputs", False))
        self._obs_out = torch.zeros((2, N, self.num_observations), device=sim_device)
        self._scalars = torch.zeros((2, 4), device=sim_device)
        # seed-faithful draws (handarm_hip/ref_rng.py): every reset / force value from torch's global CPU
        # generator in the reference's order; random_force_prob is drawn here, as at allegro_kuka_base.py:323-327
        self.reference_rng = bool(cfg.get("sim", {}).get("reference_rng", False))
        self._rr = None
        if self.reference_rng:
            self._rr = RR.KukaDraws(N, sub, tuple(self.tcfg["force_prob_range"]), float(self.tcfg["force_scale"]))
            self.random_force_prob.copy_(self._rr.prob.to(sim_device))
        # state dump / replay (allegro_kuka_base.py:95-101,545-546): off in AllegroKuka.yaml. Either one moves the
        # resets of a step into their own launch (ha_task_reset, then ha_task_step finds no reset flags), so the
        # loaded states can be written in between, as reset_idx does before its set_*_tensor_indexed calls
        self.save_states = bool(env.get("saveStates", False))
        self.save_states_filename = env.get("saveStatesFile", "rootTensorsDofStates.bin")
        self.should_load_initial_states = bool(env.get("loadInitialStates", False))
        self.load_states_filename = env.get("loadStatesFile", "rootTensorsDofStates.bin")
        self.initial_root_state_tensors = self.initial_dof_state_tensors = None
        self.initial_state_idx = self.num_initial_states = 0
        self._recorder = SF.EpisodeStateRecorder(N) if self.save_states else None
        if self.should_load_initial_states:
            self.initial_root_state_tensors, self.initial_dof_state_tensors = SF.read_state_file(
                self.load_states_filename, device=sim_device)
            self.num_initial_states = len(self.initial_root_state_tensors)

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
        """allegro_kuka_base.py:472-479: the curriculum state travels with checkpoints."""
        return dict(success_tolerance=self.success_tolerance)

    def set_env_state(self, env_state):
        if env_state and env_state.get("success_tolerance") is not None:
            self._set_tolerance(float(env_state["success_tolerance"]))

    def _set_tolerance(self, tol):
        self.success_tolerance = tol
        self.sim.t["task_scalars"].copy_(torch.from_numpy(HM.kuka_tolerance_scalars(tol, self.tcfg)))

    def zero_actions(self):
        return torch.zeros((self.num_envs, self.num_actions), dtype=torch.float32, device=self.rl_device)

    def _curriculum(self):
        """_extra_curriculum -> tolerance_curriculum, before the observations of this step (:1432)."""
        interval = int(self.tcfg["tolerance_curriculum_interval"])
        if self.frame_since_restart - self.last_curriculum_update < interval:
            return
        mean = float(self.prev_episode_successes.mean())           # the only host read, once per interval
        tol, self.last_curriculum_update = tolerance_curriculum(
            self.last_curriculum_update, self.frame_since_restart, interval, mean, self.success_tolerance,
            self.initial_tolerance, self.target_tolerance, float(self.tcfg["tolerance_curriculum_increment"]))
        if tol != self.success_tolerance:
            self._set_tolerance(tol)

    def step(self, actions):
        """VecTask.step (vec_task.py:390-441) -> pre_physics_step / simulate / post_physics_step, fused.
        obs_dict["obs"] and the extras means are valid until the step after next unless env.freshOutputs is set
        (see __init__); rew / reset / time_outs are the task's buffers, as in the reference."""
        self.frame_since_restart += 1
        self._curriculum()
        flags = self.sim_flags | self._reference_draws()
        if self.save_states or self.should_load_initial_states:
            env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()     # host read, only with state files on
            if len(env_ids) > 0:
                self.sim.task_reset(flags)
                self._after_reset(env_ids)
        if self.fresh_outputs:
            out = torch.empty_like(self._obs_out[0])
            sc = torch.empty_like(self._scalars[0])
        else:
            k = self.frame_since_restart & 1
            out, sc = self._obs_out[k], self._scalars[k]
        # one launch: the action clamp into actions_buf (vec_task.py:400-404), the fused step, obs_dict["obs"] =
        # clamp(obs_buf) into `out` and the extras means into `sc` (ha_task_step_io)
        self.sim.task_step_io(flags, actions, self.clip_actions, out, self.clip_obs, sc)
        if self._recorder is not None:                                      # post_physics_step, :1445-1446
            N = self.num_environments
            self._recorder.accumulate(self.root_state_tensor.view(N, -1, 13), self.dof_state.view(N, -1, 2))
        ex = self.extras
        ex["time_outs"] = self.timeout_buf.view(torch.bool).to(self.rl_device)
        ex["successes"] = sc[0]                                                # :908-917
        ex["true_objective"] = self.true_objective
        ex["true_objective_mean"] = sc[1]
        ex["true_objective_min"] = sc[2]
        ex["true_objective_max"] = sc[3]
        ex["rewards_episode"] = self.rewards_episode
        ex["scalars"] = {"success_tolerance": self.success_tolerance}
        self.obs_dict["obs"] = out.to(self.rl_device)
        self.obs_dict["states"] = self.states_buf
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    def reset(self):
        """VecTask.reset (vec_task.py:459-474): compute_observations only."""
        self.sim.task_observe(HM.FLAG_OBS_ONLY)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        self.obs_dict["states"] = self.states_buf
        return self.obs_dict

    def reset_idx(self, env_ids):
        """reset_idx (allegro_kuka_base.py:1246-1353) for the listed envs."""
        self.reset_buf[env_ids] = 1
        if self.save_states or self.should_load_initial_states:
            env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        self.sim.task_reset(self.sim_flags | self._reference_draws(forces=False))
        if self.save_states or self.should_load_initial_states:
            self._after_reset(env_ids)

    def _after_reset(self, env_ids):
        """The end of reset_idx (allegro_kuka_base.py:1292-1312,1349-1350) for envs the reset launch just reset:
        DOF states and the cube's root state from the loaded file, cycling through it (the targets keep the
        randomised reset pose, as in the reference), then the dump of the envs' recorded episodes."""
        N = self.num_environments
        if self.should_load_initial_states:
            n = len(env_ids)
            if n > self.num_initial_states:
                print(f"Not enough initial states to load {n}/{self.num_initial_states}...")
            else:
                if self.initial_state_idx + n > self.num_initial_states:
                    self.initial_state_idx = 0
                sl = slice(self.initial_state_idx, self.initial_state_idx + n)
                a0 = self.sim.model.actor_object0
                self.dof_state.view(N, -1, 2)[env_ids] = self.initial_dof_state_tensors[sl].clone()
                self.root_state_tensor.view(N, -1, 13)[env_ids, a0] = self.initial_root_state_tensors[sl, a0].clone()
                self.initial_state_idx += n
        if self._recorder is not None:
            SF.append_chunks(self.save_states_filename, self._recorder.dump(env_ids.tolist()))

    def _reference_draws(self, forces=True):
        """reference_rng: this step's draws on the host (one read of the reset flags), uploaded for
        HA_FLAG_REPLAY_DRAWS. Returns the extra launch flags."""
        if self._rr is None:
            return 0
        goal = self.reset_goal_buf.cpu() if forces else torch.zeros(self.num_envs, dtype=torch.int64)
        d, _ = self._rr.step(self.reset_buf.cpu(), goal, forces=forces)
        self.sim.t["reset_draws"].copy_(d)
        return HM.FLAG_REPLAY_DRAWS

    def reset_done(self):
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        return self.obs_dict, done_env_ids


class AllegroKukaRegrasping(AllegroKuka):
    def __init__(self, cfg, *args, **kwargs):
        super().__init__(cfg, *args, subtask="regrasping", **kwargs)


class AllegroKukaReorientation(AllegroKuka):
    def __init__(self, cfg, *args, **kwargs):
        super().__init__(cfg, *args, subtask="reorientation", **kwargs)


class AllegroKukaThrow(AllegroKuka):
    """allegro_kuka_throw.py:39-124: throw the cuboid into a bucket placed left or right of the table each goal.
    The bucket is actor 3 (root_state rows 4 e + 3, rigid body 26) and its convex pieces collide as statics carried
    by that actor (ha_model_t v14); bucket_object_indices names its actors like the reference's."""
    def __init__(self, cfg, *args, **kwargs):
        super().__init__(cfg, *args, subtask="throw", **kwargs)
