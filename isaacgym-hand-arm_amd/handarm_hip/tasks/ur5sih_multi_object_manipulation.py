"""Ur5SihMultiObjectManipulation with the IsaacGymEnvs VecTask surface, backed by libhandarm_hip.

Drop-in for tasks/hand_arm/task/multi_object_manipulation.py:19 (registered as
"Ur5SihMultiObjectManipulation" in tasks/__init__.py:122). The upper surface is the one
rl_games' RLGPUEnv reads (utils/rlgames_utils.py:252-310): step / reset / reset_done / reset_idx,
observation/action spaces, observation_keys, teacher observation space, log_data, extras.

Everything per step runs in ONE fused kernel (ha_task_step): controllers -> [reset + its extra
simulate] -> control_freq_inv x substeps physics -> refresh -> observables -> reward -> done.
There are no host syncs on the step path; reward-term means and success EWMAs (the reference's
.item() logging, multi_object_manipulation.py:311-351) are accumulated on the device and folded into
``log_data`` lazily.
"""
import math
import random
import sys

import numpy as np
import torch

import ctypes as C

from .. import _lib
from .. import model as HM
from .. import observables as OB
from .. import parallel
from .. import ref_rng as RR
from ..cameras import IMAGE_TYPES, CameraSensor
from ..pointclouds import SyntheticPointclouds
from ..sim import HandArmSim
from ..torch_utils import randomize_rotation, torch_rand_float

OBSERVATIONS = ["ur5_joint_pos", "ur5_flange_pose", "sih_fingertip_pos", "sih_fingertip_quat", "sih_fingertip_linvel",
                "dof_position_targets", "object_pos", "object_bounding_box", "target_object_bounding_box",
                "sih_fingertip_to_target_object_pos", "target_object_to_goal_pos"]
OBS_SIZES = [6, 7, 15, 20, 15, 17, 9, 30, 10, 15, 3]     # at the default 3 objects (see obs_sizes)
ACTIONS = ["ur5_relative_joint_pos", "sih_smoothed_relative_servo_pos"]
REWARD_TERMS = ["reaching", "lifting", "goal", "success"]
DEFAULT_OBJECTS = ["015_peach", "005_tomato_soup_can", "006_mustard_bottle"]   # Ur5SihMultiObject.yaml:11


def obs_sizes(n_objects):
    """Observation block sizes for n objects (object_pos 3 and object_bounding_box 10 per object,
    multi_object.py:128,245)."""
    return [6, 7, 15, 20, 15, 17, 3 * n_objects, 10 * n_objects, 10, 15, 3]


# no_bin extent (multi_object.py:421-423) + bin.pos: the drop-init in-bin test without a bin
NO_BIN_EXTENT = [[0.03, 0.28, 0.5], [0.53, 0.78, 0.7]]


# drop rounds after which the initialisation gives up with an error (objects.drop.max_rounds unset); the
# reference has no limit (multi_object_manipulation.py:97), a full 8192-env shard needs a handful of rounds
DROP_ROUNDS_LIMIT = 1000

class Box:
    """Minimal gym.spaces.Box (openai-gym is not a dependency here)."""

    def __init__(self, low, high):
        self.low = np.asarray(low, dtype=np.float32)
        self.high = np.asarray(high, dtype=np.float32)
        self.shape = self.low.shape
        self.dtype = np.float32

    def __repr__(self):
        return f"Box({self.shape})"


def _get(cfg, path, default):
    cur = cfg
    for k in path.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return default
        cur = cur[k]
    return cur


class Ur5SihMultiObjectManipulation:
    def __init__(self, cfg, rl_device="cuda:0", sim_device="cuda:0", graphics_device_id=-1, headless=True,
                 virtual_screen_capture=False, force_render=False):
        self.cfg = cfg
        self.rl_device = rl_device
        self.device = sim_device
        self.headless = headless
        env = cfg.get("env", {})
        self.num_environments = int(env.get("numEnvs", 16384))
        self.num_agents = 1
        self.control_freq_inv = int(env.get("controlFrequencyInv", 3))
        self.clip_obs = float(env.get("clipObservations", math.inf))
        self.clip_actions = float(env.get("clipActions", math.inf))
        self.max_episode_length = int(_get(cfg, "rl.reset.max_episode_length", 200))
        objects = _get(cfg, "objects.dataset.ycb", DEFAULT_OBJECTS)
        self.num_objects = int(_get(cfg, "objects.num_objects", 3))
        self.num_initial_poses = int(_get(cfg, "objects.drop.num_initial_poses", 1))
        task_cfg = dict(control_freq_inv=self.control_freq_inv, max_episode_length=self.max_episode_length,
                        n_objects=self.num_objects, num_initial_poses=self.num_initial_poses,
                        seed=int(cfg.get("seed", 42)))
        # BASELINE config 4 "DR on": device-side domain randomization (handarm_hip/dr.py, csrc/ha_dr.h: actor
        # properties resampled at reset, action and observation noise in the step kernel). The reference's Ur5Sih
        # `randomize` flag has no consumer, so this is the build's own switch: cfg["task"]["randomize"],
        # with cfg["task"]["randomization_params"] in the reference's schema, or the build's config-4 schema
        # (dr.UR5SIH_SCHEMA) when it has none
        self.randomize = bool(_get(cfg, "task.randomize", False))
        # seed-faithful draws (handarm_hip/ref_rng.py): resets, drops and cloud permutations from torch's global
        # CPU generator in the reference's order, instead of the device counter hash
        self.reference_rng = bool(_get(cfg, "sim.reference_rng", False))
        task_cfg["dr_enable"] = int(self.randomize)
        if self.randomize:
            task_cfg["randomization_params"] = _get(cfg, "task.randomization_params", None)
        rew = _get(cfg, "rl.reward", None)
        if rew:
            for k in REWARD_TERMS:
                task_cfg["reward_" + k] = float(rew.get(k, 0.0))
        # bin.asset (Ur5SihMultiObject.yaml:21-24): 'no_bin' (default) or 'hard_bin', the bin-picking scene of
        # BASELINE config 5 (table with a hole, the tote as static boxes; tools/build_model.py --bin)
        self.bin_asset = str(_get(cfg, "bin.asset", "no_bin"))
        if self.bin_asset not in ("no_bin", "hard_bin"):
            raise ValueError(f"bin.asset {self.bin_asset!r}: this build ships 'no_bin' and 'hard_bin'")
        scene = HM.load_scene(HM.BIN_ASSET if self.bin_asset == "hard_bin" else HM.ASSET)
        if len(objects) < self.num_objects:      # multi_object.py:567-568
            raise ValueError("Number of objects per environment cannot be larger that the total number of objects used.")
        self.scene = scene
        self.sim = HandArmSim(self.num_environments, sim_device, task_cfg=task_cfg, scene=scene, pool_names=objects)
        self.task_cfg = self.sim.cfg
        self.objects = objects
        t = self.sim.t
        N, A, B, D = self.num_envs, self.sim.num_actors, self.sim.num_bodies, self.sim.num_dofs
        self.num_actors, self.num_bodies, self.num_dofs = A, B, D
        # gym tensors and the reference's views (observable_vec_task.py:123-155)
        self.root_state = t["root_state"]
        self.body_state = t["rigid_body_state"]
        self.dof_state = t["dof_state"]
        self.contact_force = t["net_contact_force"].view(N, B, 3)
        self.root_pos = self.root_state.view(N, A, 13)[..., 0:3]
        self.root_quat = self.root_state.view(N, A, 13)[..., 3:7]
        self.root_linvel = self.root_state.view(N, A, 13)[..., 7:10]
        self.root_angvel = self.root_state.view(N, A, 13)[..., 10:13]
        self.body_pos = self.body_state.view(N, B, 13)[..., 0:3]
        self.body_quat = self.body_state.view(N, B, 13)[..., 3:7]
        self.body_linvel = self.body_state.view(N, B, 13)[..., 7:10]
        self.body_angvel = self.body_state.view(N, B, 13)[..., 10:13]
        self.dof_pos = self.dof_state.view(N, D, 2)[..., 0]
        self.dof_vel = self.dof_state.view(N, D, 2)[..., 1]
        # VecTask buffers (vec_task.py:329-354)
        self.obs_buf = t["obs"]
        self.teacher_obs_buf = t["teacher_obs"]
        self.rew_buf = t["rew"]
        self.reset_buf = t["reset_buf"]
        self.randomize_buf = t["randomize_buf"]           # vec_task.py:352 (counted on the device)
        self.progress_buf = t["progress_buf"]
        self.timeout_buf = t["timeout_buf"]
        self.goal_pos = t["goal_pos"]
        self.goal_reached_before = t["goal_reached_before"]
        self.target_object_index = t["target_object_index"]
        self.object_configuration_indices = t["object_configuration_indices"]
        self.dof_position_targets = t["dof_position_targets"]
        self.actions_buf = t["actions"]
        self.reset_buf.fill_(1)
        self.states_buf = torch.zeros((N, 0), device=self.device)
        sizes = obs_sizes(self.num_objects)
        self.num_observations = sum(sizes)
        self.num_teacher_observations = self.num_observations
        self.num_states = 0
        self.num_actions = 11
        self.obs_space = Box(np.full(self.num_observations, -np.inf), np.full(self.num_observations, np.inf))
        self.teacher_obs_space = self.obs_space
        self.state_space = Box(np.zeros(0), np.zeros(0))
        self.act_space = Box(-np.ones(self.num_actions), np.ones(self.num_actions))
        start = np.cumsum([0] + sizes)
        self.observations_start_end = {n: (int(start[i]), int(start[i + 1])) for i, n in enumerate(OBSERVATIONS)}
        self.teacher_observations_start_end = dict(self.observations_start_end)
        self._init_observation_lists(cfg, env, objects, N)
        self.extras = {}
        self.obs_dict = {}
        self._log_data = {}
        self.control_steps = 0
        self.total_train_env_frames = 0
        self.dt = self.sim.params.dt
        # actor layout: goal 0, robot 1, table 2, [bin 3,] objects (multi_object.py:562-663)
        m = self.sim.model
        self.actor_object0 = a0 = m.actor_object0
        ar = torch.arange(N, dtype=torch.int32, device=self.device)
        self.goal_actor_indices = ar * A + m.actor_goal
        self.ur5sih_actor_indices = ar * A + m.actor_robot
        self.object_actor_indices = ar[:, None] * A + a0 + torch.arange(self.num_objects, dtype=torch.int32,
                                                                           device=self.device)[None]
        self.object_actor_env_indices = [a0 + i for i in range(self.num_objects)]
        self.bin_extent = scene.get("bin_extent", NO_BIN_EXTENT)
        # per-env object subset: random.sample of the pool (multi_object.py:569)
        pool = list(range(len(objects)))
        idx = [random.sample(pool, self.num_objects) for _ in range(N)]
        t["object_indices"].copy_(torch.tensor(idx, dtype=torch.int64))
        self.object_indices = t["object_indices"]
        self._bind_gather_sources()
        # initial actor poses (create_actor start poses)
        rs = self.root_state.view(N, A, 13)
        rs[:, m.actor_robot, 0:3] = torch.tensor(m.base_pos[:], device=self.device)
        statics = scene.get("static_actors") or [{"actor": m.actor_table, "pose": list(m.table_pos) + [0, 0, 0, 1]}]
        for sa in statics:                                                    # table (and bin) start poses
            rs[:, sa["actor"], 0:7] = torch.tensor(sa["pose"], dtype=torch.float32, device=self.device)
        rs[:, a0:a0 + self.num_objects, 0:3] = torch.tensor([0.0, 0.0, 0.5], device=self.device)   # ObjectAsset.start_pose
        self.dof_pos[:] = torch.tensor(self.sim.params.reset_pose[:D], device=self.device)
        t["sim_targets"].copy_(self.dof_pos)
        self._sync_obs_cache()      # observables' post_step in ConfigurableVecTask.__init__
        if self.pointclouds is not None:
            # the clouds' post_step there too (configurable_vec_task.py:43-44): with sim.reference_rng its
            # torch.randperm is a draw from the global CPU generator before the first reset's (multi_object.py:806)
            self.pointclouds.refresh()
        self.objects_dropped = False
        # the reference drops until every object lands in the extent (multi_object_manipulation.py:97-136); a
        # round cap is a diagnostic option only (objects.drop.max_rounds: stop there, or with
        # objects.drop.place_remaining place the rest upright above the extent centre)
        mr = _get(cfg, "objects.drop.max_rounds", None)
        self.max_drop_rounds = None if mr is None else int(mr)
        self.max_drop_rounds_place = bool(_get(cfg, "objects.drop.place_remaining", False))
        self._stat_pending = 0
        self._stat_folded = 0
        self._success_rate_ewma = 0.0
        self._object_ewma = [0.0] * len(objects)
        self.total_num_resets = 0
        self.total_num_successes = 0
        self.sim_flags = 0

    def _init_observation_lists(self, cfg, env, objects, N):
        """cfg["env"]["observations"] / ["teacher_observations"] (observable_vec_task.py:15-29). The default
        lists are what the fused step kernel writes; a custom observation list (e.g. the point-cloud student
        list, Ur5SihMultiObjectManipulation.yaml:45) is assembled on the device from the kernel's obs row and
        goal_pos (ha_gather_obs), and its synthetic point clouds come from ONE ha_pointclouds launch per step
        into obs_dict[name] (observables.py:199-210). The post-step order decides which object pose a cloud
        sees (handarm_hip/observables.py)."""
        self.obs_names = list(env.get("observations") or OB.DEFAULT_OBSERVATIONS)
        teacher = list(env.get("teacher_observations") or OB.DEFAULT_OBSERVATIONS)
        # a custom teacher list (cfg teacher_observations, observable_vec_task.py:17-18,194-203) is gathered like a
        # custom student list: its "obs"-key observables concatenated into obs_dict["teacher"]["obs"], its clouds
        # in obs_dict["teacher"][name]
        self.teacher_names = teacher
        self.custom_teacher = teacher != OB.DEFAULT_OBSERVATIONS
        # camera observables `{camera}_{depth,segmentation,pointcloud}` (observable_vec_task.py:36-82): one sensor
        # per camera of cfg["cameras"] that the list names; refreshed after every other observable
        # (configurable_vec_task.py:91-114), so they do not enter the post-step order
        self.cameras, self.camera_obs = {}, {}
        for cam_name, cam_cfg in (_get(cfg, "cameras", {}) or {}).items():
            kinds = [n[len(cam_name) + 1:] for n in self.obs_names if n.startswith(cam_name + "_")]
            if not kinds:
                continue
            for k in kinds:
                if k not in IMAGE_TYPES:
                    raise NotImplementedError(f"camera observable {cam_name}_{k}: this build renders {IMAGE_TYPES}")
            if "pos" not in cam_cfg:
                raise NotImplementedError(f"camera {cam_name}: ROS cameras are out of scope")
            self.cameras[cam_name] = CameraSensor(self.sim, cam_cfg["pos"], cam_cfg["quat"], cam_cfg.get("fovx", 87),
                                                  cam_cfg.get("resolution", (160, 90)), kinds, self.scene,
                                                  max_num_points=int(_get(cfg, "pointclouds.max_num_points", 128)))
            for k in kinds:
                self.camera_obs[f"{cam_name}_{k}"] = (cam_name, k)
        for n in self.obs_names:
            if n.endswith(("_pointcloud", "_depth", "_segmentation", "_color")) and n not in OB.POINTCLOUDS \
                    and n not in self.camera_obs:
                raise NotImplementedError(f"observable {n!r}: this build produces the synthetic clouds "
                                          f"{OB.POINTCLOUDS} and camera images {IMAGE_TYPES} of cfg['cameras']")
        for n in teacher:
            if n.endswith(("_pointcloud", "_depth", "_segmentation", "_color")) and n not in OB.POINTCLOUDS:
                raise NotImplementedError(f"teacher observable {n!r}: a teacher list takes the low-dimensional "
                                          f"observables and the synthetic clouds {OB.POINTCLOUDS}")
        order = OB.post_step_order([n for n in self.obs_names if n not in self.camera_obs], teacher)
        if not OB.sees_previous_object_pose(order, "object_bounding_box"):
            raise NotImplementedError("observation list refreshes object_bounding_box after object_pos; the step "
                                      "kernel implements the default order (bbox sees the previous pose)")
        self.custom_obs = self.obs_names != OB.DEFAULT_OBSERVATIONS
        self.pointclouds = None
        pc_names = [n for n in dict.fromkeys(self.obs_names + teacher) if n in OB.POINTCLOUDS]
        if pc_names:
            g = torch.Generator(device=self.device).manual_seed(int(cfg.get("seed", 42)))
            self.pointclouds = SyntheticPointclouds(self.sim, pc_names, objects, _get(cfg, "pointclouds", {}), g)
            self.pointclouds.reference_rng = bool(_get(cfg, "sim.reference_rng", False))
            if any(OB.sees_previous_object_pose(order, n) for n in
                   ("object_synthetic_pointcloud", "target_object_synthetic_pointcloud") if n in order):
                self.pointclouds.use_previous_object_pose()
        if not (self.custom_obs or self.custom_teacher):
            return
        m = self.sim.model
        layout = dict(a0=m.actor_object0, body_robot0=m.body_robot0, n_dofs=m.n_dofs)
        self._obs_layout = layout
        if self.custom_teacher:
            tcols = OB.obs_columns(teacher, self.num_objects, layout)
            self._teacher_cols = torch.tensor(tcols, dtype=torch.int32, device=self.device)
            self.teacher_custom_buf = torch.zeros((N, len(tcols)), dtype=torch.float32, device=self.device)
            self.num_teacher_observations = len(tcols)
            self.teacher_obs_space = Box(np.full(len(tcols), -np.inf), np.full(len(tcols), np.inf))
            start, self.teacher_observations_start_end = 0, {}
            for n in teacher:
                k = len(OB.obs_columns([n], self.num_objects, layout))
                if k:
                    self.teacher_observations_start_end[n] = (start, start + k)
                    start += k
        if not self.custom_obs:
            return
        cols = OB.obs_columns(self.obs_names, self.num_objects, layout)
        self._obs_cols = torch.tensor(cols, dtype=torch.int32, device=self.device)
        self.student_obs_buf = torch.zeros((N, len(cols)), dtype=torch.float32, device=self.device)
        self.num_observations = len(cols)
        self.obs_space = Box(np.full(self.num_observations, -np.inf), np.full(self.num_observations, np.inf))
        start, self.observations_start_end = 0, {}
        for n in self.obs_names:                  # _compute_num_observations: only key-"obs" observables
            k = len(OB.obs_columns([n], self.num_objects, layout))
            if k:
                self.observations_start_end[n] = (start, start + k)
                start += k

    def _bind_gather_sources(self):
        """ha_gather_obs sources of a custom observation list (observables.SRC_*), once the objects are chosen.
        object_mass / object_com / object_inertia (multi_object.py:907-925) are the pool properties of each env's
        objects, fixed at creation (the reference reads them once, at post_init)."""
        if not (self.custom_obs or self.custom_teacher):
            return
        m, N = self.sim.model, self.num_envs
        pm = torch.tensor(np.ctypeslib.as_array(m.pool_mass)[:m.n_pool], dtype=torch.float32)
        pc = torch.tensor(np.ctypeslib.as_array(m.pool_com)[:m.n_pool], dtype=torch.float32)
        pi = torch.tensor(np.ctypeslib.as_array(m.pool_inertia)[:m.n_pool], dtype=torch.float32)
        props = torch.cat([pm[:, None], pc, pi], 1)                      # (pool, 13)
        self.object_props = props.to(self.device)[self.sim.t["object_indices"]].reshape(N, -1).contiguous()
        t = self.sim.t
        srcs = [self.obs_buf, self.goal_pos, t["root_state"], t["rigid_body_state"], t["dof_state"], self.object_props]
        self._gather_src = (C.c_void_p * len(srcs))(*[x.data_ptr() for x in srcs])
        self._gather_stride = (C.c_int32 * len(srcs))(self.obs_buf.shape[1], 3, self.num_actors * 13,
                                                       self.num_bodies * 13, self.num_dofs * 2, self.num_objects * 13)

    def _observations(self):
        """compute_observations (observable_vec_task.py:183-203) from the device buffers."""
        obs = self.obs_buf
        if self.custom_obs:
            _lib.check(self.sim.lib.ha_gather_obs(self.sim.h, self._gather_src, self._gather_stride, 6,
                                                  self._obs_cols.data_ptr(), len(self._obs_cols),
                                                  self.student_obs_buf.data_ptr(), self.sim._stream()),
                       "ha_gather_obs")
            obs = self.student_obs_buf
        self.obs_dict["obs"] = torch.clamp(obs, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.pointclouds is not None:
            for n, t in self.pointclouds.outputs.items():
                if n in self.obs_names:
                    self.obs_dict[n] = t.to(self.rl_device)
        for n, (cam, kind) in self.camera_obs.items():
            img = self.cameras[cam].images[kind]
            # PointcloudObservable's FlattenPointcloud transform (transforms.py:17-20): (N, H * W, 4)
            self.obs_dict[n] = (img.flatten(1, 2) if kind == "pointcloud" else img).to(self.rl_device)
        teacher = self.teacher_obs_buf
        if self.custom_teacher:
            _lib.check(self.sim.lib.ha_gather_obs(self.sim.h, self._gather_src, self._gather_stride, 6,
                                                  self._teacher_cols.data_ptr(), len(self._teacher_cols),
                                                  self.teacher_custom_buf.data_ptr(), self.sim._stream()),
                       "ha_gather_obs")
            teacher = self.teacher_custom_buf
        self.obs_dict["teacher"] = {"obs": torch.clamp(teacher, -self.clip_obs, self.clip_obs).to(self.rl_device)}
        if self.pointclouds is not None:
            for n in self.teacher_names:
                if n in self.pointclouds.outputs:
                    self.obs_dict["teacher"][n] = self.pointclouds.outputs[n].to(self.rl_device)
        return self.obs_dict

    # ------------------------------------------------------------------ VecTask properties
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
    def num_teacher_obs(self):
        return self.num_teacher_observations

    @property
    def observation_space(self):
        return self.obs_space

    def teacher_observation_space(self):
        return self.teacher_obs_space

    @property
    def action_space(self):
        return self.act_space

    @property
    def observation_start_end(self):
        # reference quirk (vec_task.py:176 vs observable_vec_task.py:24): always None
        return getattr(self, "_observation_start_end", None)

    @property
    def teacher_observation_start_end(self):
        return getattr(self, "_teacher_observation_start_end", None)

    @property
    def observation_keys(self):
        # observable_vec_task.py:205-211: "obs" for low-dimensional observables, the name for point clouds
        keys = []
        for n in self.obs_names:
            k = n if (n in OB.POINTCLOUDS or n in self.camera_obs) else "obs"
            if k not in keys:
                keys.append(k)
        return keys

    def get_number_of_agents(self):
        return self.num_agents

    def set_train_info(self, env_frames, *args, **kwargs):
        self.total_train_env_frames = env_frames

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass

    def zero_actions(self):
        return torch.zeros((self.num_envs, self.num_actions), dtype=torch.float32, device=self.rl_device)

    # ------------------------------------------------------------------ internals
    def _sync_obs_cache(self):
        n, a, a0 = self.num_envs, self.num_actors, self.actor_object0
        self.sim.t["obs_cache"].copy_(self.root_state.view(n, a, 13)[:, a0:a0 + self.num_objects, 0:7])

    def _random_object_pos(self, n, key):
        c = self.task_cfg
        pos = torch.tensor(c[key + "_pos"], device=self.device).unsqueeze(0).repeat(n, 1)
        noise = 2 * (torch.rand((n, 3), dtype=torch.float32, device=self.device) - 0.5)
        return pos + noise * torch.tensor(c[key + "_noise"], device=self.device)

    def _reset_ur5sih(self, pose):
        self.dof_pos[:] = torch.tensor(pose, device=self.device)
        self.dof_vel[:] = 0.0
        self.sim.t["sim_targets"].copy_(self.dof_pos)
        self.dof_position_targets.copy_(self.dof_pos)

    def _drop_initialisation(self):
        """First reset: find initial object poses by dropping (multi_object_manipulation.py:36-61, 93-173)."""
        N, A, n_obj = self.num_envs, self.num_actors, self.num_objects
        P = self.num_initial_poses
        rs = self.root_state.view(N, A, 13)[:, self.actor_object0:self.actor_object0 + n_obj]   # the object rows
        self._reset_ur5sih(self.task_cfg["bringup_pose"])
        # objects_in_bin extent (multi_object.py:705-718): no_bin default or the bin's bin_info.yaml + bin.pos
        bin_lo = torch.tensor(self.bin_extent[0], device=self.device)
        bin_hi = torch.tensor(self.bin_extent[1], device=self.device)
        bin_mid = 0.5 * (bin_lo + bin_hi)
        pos_init = self.sim.t["object_pos_initial"]
        quat_init = self.sim.t["object_quat_initial"]
        for p in range(P):
            enabled = torch.zeros((N, n_obj), dtype=torch.uint8, device=self.device)
            self.sim.set_object_collisions(enabled)
            rs[:, :, 0:3] = torch.tensor([1.1, 0.0, 0.5], device=self.device)        # _init_object_poses
            rs[:, :, 7:13] = 0.0
            self.sim.simulate(1)
            in_bin = torch.zeros((N, n_obj), dtype=torch.bool, device=self.device)
            rounds = 0
            while not bool(in_bin.all()):
                if rounds == self.max_drop_rounds and self.max_drop_rounds_place:
                    # diagnostic option (not the reference's behaviour): place the remaining objects
                    print(f"[handarm_hip] drop init: {int((~in_bin).sum())} objects outside the bin extent after "
                          f"{rounds} rounds; placing them upright above the bin centre", file=sys.stderr, flush=True)
                    bad = (~in_bin).nonzero(as_tuple=False)
                    xy = bin_mid[0:2] + 0.1 * (torch.rand((len(bad), 2), device=self.device) - 0.5)
                    rs[bad[:, 0], bad[:, 1], 0:2] = xy
                    rs[bad[:, 0], bad[:, 1], 2] = 0.65        # above the table top and the bin rim
                    rs[bad[:, 0], bad[:, 1], 3:7] = torch.tensor([0.0, 0.0, 0.0, 1.0], device=self.device)
                    rs[bad[:, 0], bad[:, 1], 7:13] = 0.0
                    self.sim.simulate(self.task_cfg["drop_num_steps"])
                    break
                if rounds == self.max_drop_rounds:          # diagnostic: stop, leaving the objects where they are
                    break
                if self.max_drop_rounds is None and rounds >= DROP_ROUNDS_LIMIT:
                    # the reference loops forever on an object that never lands in the extent; fail loudly instead
                    bad = (~in_bin).nonzero(as_tuple=False)[:10].tolist()
                    raise RuntimeError(f"drop initialisation: {int((~in_bin).sum())} objects still outside the bin "
                                       f"extent after {rounds} rounds (env, object): {bad}")
                rounds += 1
                print(f"[handarm_hip] drop init pose {p}: round {rounds}, {int((~in_bin).sum())} objects to drop",
                      file=sys.stderr, flush=True)
                # envs stepped while object i drops: the reference steps every env (multi_object_manipulation.py:
                # 123-125); with sim.reference_rng so does this loop. Otherwise the envs that dropped any object in
                # this round so far (an env that re-dropped object j < i keeps stepping while object i drops, as in
                # the reference); envs with nothing in flight this round wait (they settle with all envs below)
                dropping = torch.zeros(N, dtype=torch.bool, device=self.device)
                for i in range(n_obj):
                    enabled[:, i] = 1
                    self.sim.set_object_collisions(enabled)
                    env_ids = (~in_bin[:, i]).nonzero(as_tuple=False).squeeze(-1)
                    if len(env_ids) > 0:
                        if self.reference_rng:
                            pos, quat = RR.ur5sih_drop_pose(len(env_ids), self.task_cfg["drop_pos"],
                                                            self.task_cfg["drop_noise"])
                            rs[env_ids, i, 0:3] = pos.to(self.device)
                            rs[env_ids, i, 3:7] = quat.to(self.device)
                        else:
                            rs[env_ids, i, 0:3] = self._random_object_pos(len(env_ids), "drop")
                            rf = torch_rand_float(-1.0, 1.0, (len(env_ids), 2), device=self.device)
                            rs[env_ids, i, 3:7] = randomize_rotation(rf[:, 0], rf[:, 1])
                        rs[env_ids, i, 7:13] = 0.0
                        dropping |= ~in_bin[:, i]
                        step_ids = None if self.reference_rng else dropping.nonzero(as_tuple=False).squeeze(-1)
                        self.sim.simulate(self.task_cfg["drop_num_steps"],
                                          env_ids=step_ids if step_ids is not None and len(step_ids) < N else None)
                obj_pos = rs[:, :, 0:3]
                in_bin = ((obj_pos >= bin_lo) & (obj_pos <= bin_hi)).all(-1)
            for _ in range(600):                                                    # settle
                self.sim.simulate(1)
                if bool((rs[:, :, 7:10].norm(dim=2).max(dim=1).values < 0.01).all()):
                    break
            pos_init[:, p] = rs[:, :, 0:3]
            quat_init[:, p] = rs[:, :, 3:7]
            self._sync_obs_cache()
            if self.pointclouds is not None:
                # every observable's post_step after the settle (multi_object_manipulation.py:149-150): the object
                # cloud's randperm draw, in the reference's order with sim.reference_rng
                self.pointclouds.refresh()
        self.objects_dropped = True

    def contact_stats(self, reset=False):
        """Contact-list diagnostics of the physics since the last reset (HandArmSim.contact_stats)."""
        return self.sim.contact_stats(reset)

    def _reference_draws(self, all_envs=False):
        """reference_rng: if this step resets, draw its values on the host in the reference's order and hand them
        to the kernel (HA_FLAG_REPLAY_DRAWS). One device->host read of reset_buf per step (the reference's
        reset_buf.nonzero() in post_physics_step). Returns the extra launch flags."""
        if not self.reference_rng:
            return 0
        if not all_envs:
            reset = self.reset_buf.cpu()
            if not bool(reset.any()):
                return 0
            assert bool(reset.all()), "All environments should be reset simultaneously."      # ur5sih.py:617
        d = RR.ur5sih_reset_draws(self.num_envs, self.num_initial_poses, self.num_objects)
        self.sim.t["reset_draws"][:, 0:5].copy_(d)
        return HM.FLAG_REPLAY_DRAWS

    def _fold_stats(self):
        """Fold the device-side per-step counters into log_data (reference :311-351 semantics). With several
        ranks only reduced slots are folded (parallel.reduce_episode_stats, a collective every rank runs at the
        same step); rl_games reads log_data on rank 0 alone, so the fold here must not start a collective."""
        if parallel.world() == 1:
            parallel.fold_pending(self, self.num_envs)

    @property
    def log_data(self):
        """Read (and cleared) by RLGPUAlgoObserver (rlgames_utils.py:212-219); device counters folded in."""
        self._fold_stats()
        return self._log_data

    @log_data.setter
    def log_data(self, value):
        self._log_data = value

    def log(self, data):
        self._log_data.update(data)

    # ------------------------------------------------------------------ VecTask API
    def step(self, actions):
        if not self.objects_dropped and bool(self.reset_buf.any()):
            self._drop_initialisation()
        # (DR action noise: added by the step kernel where it reads the actions, ha_dr.h act_at; with the HandArm
        # configs' clipActions unset the clamp below is the identity, so noise-then-clamp (vec_task.py:400-404) is kept)
        torch.clamp(actions, -self.clip_actions, self.clip_actions, out=self.actions_buf)
        if self._stat_pending >= self.sim.stats_ring - 1:
            # ring full (this step's launch clears the slot after its own, the oldest pending one): reduce
            # across ranks (if any), then fold
            parallel.reduce_episode_stats(self)
        if self.pointclouds is not None:           # object_pos as of the previous refresh (see observables.py)
            self.pointclouds.snapshot_object_pose(self.sim.t["obs_cache"])
        self.sim.task_step(self.sim_flags | self._reference_draws())
        if self.pointclouds is not None:           # the clouds' post_step refresh, one launch
            self.pointclouds.refresh()
        for cam in self.cameras.values():          # render_all_camera_sensors + image refresh, one launch each
            cam.render()
        self._stat_pending += 1
        self.control_steps += 1
        self.extras["time_outs"] = self.timeout_buf.view(torch.bool).to(self.rl_device)
        self._observations()
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    def reset(self):
        """VecTask.reset (vec_task.py:459-474): compute_observations only."""
        self.sim.task_observe(HM.FLAG_OBS_ONLY)
        return self._observations()

    def reset_idx(self, env_ids):
        """Immediate reset of ALL envs (the reference asserts it, ur5sih.py:617)."""
        assert len(env_ids) == self.num_envs, "All environments should be reset simultaneously."
        if not self.objects_dropped:
            self._drop_initialisation()
        self.sim.task_reset(self.sim_flags | self._reference_draws(all_envs=True))

    def reset_done(self):
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self._observations()
        return self.obs_dict, done_env_ids

