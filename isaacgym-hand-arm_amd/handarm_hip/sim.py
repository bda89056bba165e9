"""Gym-style simulation object over the HIP library: the lower surface the reference task code uses.

``HandArmSim`` owns one ``ha_handle`` and every device tensor (torch, on ``device``). Method names and
semantics follow the Isaac Gym tensor API the hand_arm task calls:

  acquire_actor_root_state_tensor / acquire_rigid_body_state_tensor / acquire_dof_state_tensor /
  acquire_net_contact_force_tensor   -> the live state tensors (zero-copy: they ARE the sim state)
  refresh_*                          -> no-ops (the kernels write the tensors in place)
  simulate(n)                        -> n gym.simulate() calls in ONE kernel launch
  set_actor_root_state_tensor_indexed / set_dof_state_tensor_indexed /
  set_dof_position_target_tensor(_indexed)  -> copy-in for the listed global actor indices (int32)

Difference to Isaac Gym worth knowing: because the acquired tensors are the simulation state,
writes into them take effect even without a set_*_indexed call (the reference always calls it).
"""
import ctypes as C
import os

import torch

from . import _lib
from . import model as HM

TORCH_DTYPE = {"float32": torch.float32, "int64": torch.int64, "uint8": torch.uint8, "int32": torch.int32,
               "uint32": torch.int32}


class HandArmSim:
    def __init__(self, num_envs, device="cuda:0", task_cfg=None, scene=None, pool_names=None, stats_ring=64,
                 task=None, rebalance_every=None):
        if not str(device).startswith("cuda"):
            raise _lib.HandArmError("libhandarm_hip runs on a HIP device only (device must be 'cuda:N')")
        self.lib = _lib.load()
        self.device = torch.device(device)
        if task is None:
            task = (task_cfg or {}).get("task", HM.TASK_UR5SIH)
        self.task = task
        default_scene = {HM.TASK_ALLEGRO_HAND: HM.ALLEGRO_ASSET, HM.TASK_ALLEGRO_KUKA: HM.KUKA_ASSET}.get(task, HM.ASSET)
        self.scene = scene if scene is not None else HM.load_scene(default_scene)
        self.model = HM.build_model(self.scene, pool_names, posed=HM.posed_group(task, task_cfg))
        self.params, self.cfg = HM.build_params(task_cfg, task=task)
        self.num_envs = num_envs
        self.n_obj = self.params.n_objects
        self.num_dofs = self.model.n_dofs
        self.num_links = self.model.n_links
        self.num_actors = self.model.n_actors
        self.num_bodies = self.model.n_bodies
        self.stats_ring = stats_ring
        spec = HM.state_spec(num_envs, n_links=self.num_links, n_dofs=self.num_dofs, n_obj=self.n_obj,
                             num_initial_poses=self.params.num_initial_poses, num_actions=self.params.num_actions,
                             num_obs=self.params.num_obs, n_actors=self.num_actors, n_bodies=self.num_bodies,
                             n_pcm_slots=HM.pcm_slots(self.model, self.n_obj, self.params),
                             num_states=HM.num_states(self.params))
        spec["stats"] = ((stats_ring, HM.STAT_SIZE), spec["stats"][1])
        spec["term_sums"] = ((stats_ring, 4), spec["term_sums"][1])
        with torch.cuda.device(self.device):
            self.t = {k: torch.zeros(shape, dtype=TORCH_DTYPE[dt.__name__], device=self.device)
                      for k, (shape, dt) in spec.items()}
        self.t["root_state"].view(num_envs, self.num_actors, 13)[..., 6] = 1.0
        self.t["goal_state"][:, 6] = 1.0
        self.t["collision_enabled"].fill_(1)
        if task == HM.TASK_ALLEGRO_HAND:          # objectType: the scene's pool entry in every env
            self.t["object_indices"].fill_(int(self.params.ah_object_type))
        # domain-randomization rows start at the nominal values (mass ratio 1, friction, the model's DOF gains and
        # limits, scale 1) until an env's first sample, and the shard-wide state at frame 0 (handarm_hip/dr.py)
        from . import dr as DR
        self.t["dr_scale"].copy_(torch.from_numpy(DR.default_rows(self.model, self.params, num_envs)))
        self.t["dr_global"].copy_(torch.from_numpy(DR.init_global(self.params)))
        if task == HM.TASK_ALLEGRO_KUKA:
            self._init_kuka()
        h = C.c_void_p()
        if task == HM.TASK_ALLEGRO_HAND:            # object_rb_masses (allegro_hand.py:355-357): the object's mass
            self.params.ah_object_rb_mass = self.model.pool_mass[self.params.ah_object_type]
        _lib.check(self.lib.ha_create(C.byref(self.model), C.byref(self.params), num_envs, C.byref(h)), "ha_create")
        self.h = h
        # contacts per substep the kernel family holds (clutter 84, Ur5Sih 21, AllegroKuka 21, AllegroHand 12)
        self.contact_capacity = int(self.lib.ha_contact_capacity(self.h))
        # persistent-manifold records per env (the contact_cache rows; zero = empty)
        assert int(self.lib.ha_contact_cache_slots(self.h)) == self.t["contact_cache"].shape[1]
        self.state = HM.HaState()
        null = HM.null_fields(task)
        for k in HM.STATE_FIELDS:
            setattr(self.state, k, None if k in null else self.t[k].data_ptr())
        _lib.check(self.lib.ha_bind_state(self.h, C.byref(self.state)), "ha_bind_state")
        _lib.check(self.lib.ha_set_stats_ring(self.h, stats_ring), "ha_set_stats_ring")
        # longest-first dispatch order of the fused step (ha_set_env_order), refreshed every `rebalance_every` steps
        # (0: identity order; one ha_update_env_order launch per refresh). An explicit argument wins; HA_REBALANCE (A/B
        # scripts) only replaces the default 1
        if rebalance_every is None:
            rebalance_every = int(os.environ.get("HA_REBALANCE", 1))
        self.rebalance_every = int(rebalance_every)
        self._snake = int(os.environ.get("HA_ORDER_SNAKE", 0))     # A/B: alternate-block reversal of the order
        # the refresh sorts by each env's workgroup span in the last step launch (round 4: C4 +13% against the
        # contacts offered). AllegroHand sorts by the contacts offered instead: its spans repeat poorly from step to
        # step (correlation 0.38 against C5's 0.60, profiles/r06_order_quality.txt) and the contact count, which
        # tracks an env's span at 0.8, measured its kernel 0.5-0.7% faster. HA_ORDER_COST overrides (A/B runs)
        order_cost = os.environ.get("HA_ORDER_COST", "contacts" if task == HM.TASK_ALLEGRO_HAND else "time")
        if order_cost not in ("time", "contacts"):
            raise ValueError(f"HA_ORDER_COST must be 'time' or 'contacts', not {order_cost!r}")
        self.order_cost = order_cost
        self._rb_count = 0
        if self.rebalance_every > 0:
            self._env_order = torch.arange(num_envs, dtype=torch.int32, device=self.device)
            self._cost_prev = torch.zeros(num_envs, dtype=torch.int32, device=self.device)
            if order_cost == "time":
                _lib.check(self.lib.ha_set_order_cost(self.h, 1), "ha_set_order_cost")
                self._cost_prev.zero_()             # the estimates restart with the cost they measure
            _lib.check(self.lib.ha_set_env_order(self.h, C.c_void_p(self._env_order.data_ptr()), num_envs),
                       "ha_set_env_order")

    def snapshot(self):
        """Device copy of the env-state SoA (every tensor the kernels read or write: gym state tensors, targets,
        controller and task state, counters, DR rows, draws). restore() puts the shard back exactly, so the next
        steps reproduce bit for bit (SURVEY.md §5 checkpoint row; the task classes' get_env_state / set_env_state
        keep the host-side curriculum values, as in the reference). One device-to-device copy per tensor."""
        return {k: v.clone() for k, v in self.t.items()}

    def restore(self, snap):
        """Copy a snapshot() back into the bound tensors (same shapes; the kernels keep their pointers)."""
        for k, v in snap.items():
            self.t[k].copy_(v)

    def rebalance(self):
        """Dispatch the envs that offered the most contacts since the last call first (device argsort, stable, no
        host sync). In a launch with more envs than resident workgroup slots, the slots that free up take the
        cheaper envs last, so the launch's tail shrinks (longest-processing-time order); a one-round launch spreads
        its heavy envs over the CUs. Results do not depend on the order (one workgroup per env)."""
        _lib.check(self.lib.ha_update_env_order(self.h, C.c_void_p(self._env_order.data_ptr()),
                                                C.c_void_p(self._cost_prev.data_ptr()), self._snake, self._stream()),
                   "ha_update_env_order")

    def _init_kuka(self):
        """AllegroKuka buffers at env creation: per-env object dims and keypoint offsets, goal_states
        (object start - 0.04 z, allegro_kuka_base.py:738-740), object/goal root states, the tolerance
        scalars, random_force_prob drawn at __init__ (:339-343) and the -1 'unset' markers (:356-360).
        reset_buf / reset_goal_buf start at 1 (vec_task.py allocate_buffers), so the first step resets all."""
        N, c, p = self.num_envs, self.cfg, self.params
        scales, offs = HM.kuka_env_tables(N, self.scene, c)
        self.t["object_scale"].copy_(torch.from_numpy(scales))
        ts = self.t["task_state"]
        ts[:, HM.AK_KP:HM.AK_KP + 12] = torch.from_numpy(offs.reshape(N, 12)).to(self.device)
        ts[:, HM.AK_CLOSEST_KP] = -1.0
        ts[:, HM.AK_CLOSEST_FT:HM.AK_CLOSEST_FT + 4] = -1.0
        ts[:, HM.AK_FURTHEST] = -1.0
        g = torch.Generator(device=self.device).manual_seed(int(p.seed))
        lo, hi = torch.log(torch.tensor(c["force_prob_range"], device=self.device))
        ts[:, HM.AK_FORCE_PROB] = torch.exp((lo - hi) * torch.rand(N, device=self.device, generator=g) + hi)
        init = torch.tensor(list(p.ak_object_init), device=self.device)
        self.t["goal_state"][:, 0:3] = init
        self.t["goal_state"][:, 2] -= 0.04
        root = self.t["root_state"].view(N, self.num_actors, 13)
        root[:, self.model.actor_object0, 0:3] = init
        root[:, self.model.actor_goal, 0:3] = self.t["goal_state"][:, 0:3]
        if p.ak_subtask == 2:
            # throw: the bucket actor at bucket_pose = allegro_pose + (-0.6, -1, 0.45) in gymapi.Vec3 (float32) until
            # the first reset places it (allegro_kuka_throw.py:68-72)
            root[:, self.model.actor_goal, 0:3] = torch.tensor(HM.AK_BUCKET_POSE, device=self.device)
        root[:, self.model.actor_table, 0:3] = torch.tensor(list(self.model.table_pos), device=self.device)
        self.t["task_scalars"].copy_(torch.from_numpy(HM.kuka_tolerance_scalars(c["success_tolerance"], c)))
        self.t["reset_buf"].fill_(1)
        self.t["reset_goal_buf"].fill_(1)
        self.t["dof_state"].view(N, self.num_dofs, 2)[..., 0] = torch.tensor(list(p.reset_pose)[:self.num_dofs],
                                                                              device=self.device)
        self.t["dof_position_targets"].copy_(self.t["dof_state"].view(N, self.num_dofs, 2)[..., 0])
        self.t["sim_targets"].copy_(self.t["dof_position_targets"])

    # -------------------------------------------------------------- helpers
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.ha_destroy(self.h)
        except Exception:
            pass

    # -------------------------------------------------------------- Isaac Gym tensor API
    def acquire_actor_root_state_tensor(self):
        return self.t["root_state"]

    def acquire_rigid_body_state_tensor(self):
        return self.t["rigid_body_state"]

    def acquire_dof_state_tensor(self):
        return self.t["dof_state"]

    def acquire_net_contact_force_tensor(self):
        return self.t["net_contact_force"]

    def refresh_actor_root_state_tensor(self):
        _lib.check(self.lib.ha_refresh(self.h, self._stream()), "ha_refresh")

    refresh_rigid_body_state_tensor = refresh_actor_root_state_tensor
    refresh_dof_state_tensor = refresh_actor_root_state_tensor
    refresh_net_contact_force_tensor = refresh_actor_root_state_tensor

    def simulate(self, n_calls=1, flags=0, env_ids=None):
        """gym.simulate n_calls times; env_ids (device tensor of distinct env indices): those envs only."""
        if env_ids is None:
            _lib.check(self.lib.ha_simulate(self.h, n_calls, flags, self._stream()), "ha_simulate")
            return
        ids = env_ids.to(device=self.device, dtype=torch.int32).contiguous()
        _lib.check(self.lib.ha_simulate_envs(self.h, n_calls, flags, C.c_void_p(ids.data_ptr()), ids.numel(),
                                             self._stream()), "ha_simulate_envs")

    def fetch_results(self, wait=True):
        if wait:
            torch.cuda.current_stream(self.device).synchronize()

    def _indexed(self, fn, data, idx, name):
        idx = idx.to(device=self.device, dtype=torch.int32).contiguous()
        data = data.contiguous()
        _lib.check(fn(self.h, C.c_void_p(data.data_ptr()), C.c_void_p(idx.data_ptr()), idx.numel(), self._stream()),
                   name)

    def set_actor_root_state_tensor_indexed(self, root_state, actor_indices):
        self._indexed(self.lib.ha_set_actor_root_state_indexed, root_state, actor_indices, "set_actor_root_state")

    def set_dof_state_tensor_indexed(self, dof_state, actor_indices):
        self._indexed(self.lib.ha_set_dof_state_indexed, dof_state, actor_indices, "set_dof_state")

    def set_dof_position_target_tensor_indexed(self, targets, actor_indices):
        self._indexed(self.lib.ha_set_dof_position_target_indexed, targets, actor_indices, "set_dof_target")

    def set_dof_position_target_tensor(self, targets):
        targets = targets.contiguous()
        _lib.check(self.lib.ha_set_dof_position_target(self.h, C.c_void_p(targets.data_ptr()), self._stream()),
                   "set_dof_position_target")

    def set_object_collisions(self, enabled):
        """enabled: (N, n_obj) bool/uint8 - replaces the per-env shape-filter loop (multi_object.py:693-703)."""
        self.t["collision_enabled"].copy_(enabled.to(torch.uint8))

    # -------------------------------------------------------------- fused task entry points
    def task_step(self, flags=0):
        if self.rebalance_every > 0:
            self._rb_count += 1
            if self._rb_count >= self.rebalance_every:
                self._rb_count = 0
                self.rebalance()
        _lib.check(self.lib.ha_task_step(self.h, flags, self._stream()), "ha_task_step")

    def task_step_io(self, flags, actions, clip_actions, obs_out, clip_obs, scalars=None):
        """task_step with VecTask.step's action clamp and the epilogue's outputs in the same launch (Allegro tasks):
        actions (raw, N x num_actions float32 on the device) clamped into the actions tensor, obs_out = clamp(obs),
        scalars (AllegroKuka, 4 floats) = the extras means."""
        if self.rebalance_every > 0:
            self._rb_count += 1
            if self._rb_count >= self.rebalance_every:
                self._rb_count = 0
                self.rebalance()
        a = actions
        if a.dtype != torch.float32 or a.device != self.device or not a.is_contiguous():
            a = a.to(self.device, torch.float32).contiguous()
        _lib.check(self.lib.ha_task_step_io(self.h, flags, C.c_void_p(a.data_ptr()), float(clip_actions),
                                            C.c_void_p(obs_out.data_ptr()), float(clip_obs),
                                            C.c_void_p(scalars.data_ptr()) if scalars is not None else None,
                                            self._stream()), "ha_task_step_io")
        # the launch reads the converted copy asynchronously: hold it until the next step replaces it (a caller on
        # another stream than the launch's would otherwise let the caching allocator reuse it too early)
        self._act_hold = a
        return a

    def task_observe(self, flags=0):
        _lib.check(self.lib.ha_task_observe(self.h, flags, self._stream()), "ha_task_observe")

    def task_reset(self, flags=0):
        _lib.check(self.lib.ha_task_reset(self.h, flags, self._stream()), "ha_task_reset")

    def contact_stats(self, reset=False):
        """Contact-list diagnostics since the last reset (ha_state_t.contact_stats, added up by every launch):
        substeps, fraction of substeps whose narrow phases offered more contacts than the list holds (the
        shallowest are then dropped), mean and max contacts offered per substep, and percentiles of the per-env
        maximum. One device read."""
        cs = self.t["contact_stats"].cpu().numpy().astype("int64")
        if reset:
            self.t["contact_stats"].zero_()
        sub = int(cs[:, 0].sum())
        import numpy as np
        ref, nar = int(cs[:, 5].sum()), int(cs[:, 6].sum())
        return {"capacity": self.contact_capacity, "substeps": sub,
                "at_capacity_frac": float(cs[:, 1].sum() / max(sub, 1)),
                "offered_mean": float(cs[:, 3].sum() / max(sub, 1)), "offered_max": int(cs[:, 2].max()),
                "env_max_p50": float(np.percentile(cs[:, 2], 50)), "env_max_p99": float(np.percentile(cs[:, 2], 99)),
                "self_offered_mean": float(cs[:, 4].sum() / max(sub, 1)),
                "pcm_refreshed_per_substep": ref / max(sub, 1), "narrow_phases_per_substep": nar / max(sub, 1),
                "pcm_refreshed_frac": ref / max(ref + nar, 1)}

    def last_kernel_ms(self):
        return float(self.lib.ha_last_kernel_ms(self.h))

    def enable_kernel_timing(self, max_launches):
        _lib.check(self.lib.ha_enable_kernel_timing(self.h, max_launches), "ha_enable_kernel_timing")

    def kernel_times_ms(self, max_n=1 << 16):
        buf = (C.c_float * max_n)()
        n = C.c_int32()
        _lib.check(self.lib.ha_kernel_times(self.h, buf, max_n, C.byref(n)), "ha_kernel_times")
        return list(buf[:n.value])
