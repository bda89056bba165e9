#!/usr/bin/env python3
"""bench.py - env-steps/s of the fused VecTask.step on MI355X.

Default workload (BASELINE.json configs[1], the metric's 4096-env point): AllegroKuka ("Arm+Allegro cube
grasp", regrasping subtask, 23 DOF), 4096 envs per GPU, weak scaling (per-GPU work fixed as N grows). A step =
one VecTask.step() for every env (pre_physics_step with resets, random object forces and targets, 1 gym.simulate
call x 2 substeps, refresh, full_state observations, compute_kuka_reward, resets) on synthetic i.i.d. U[-1,1]
actions (seed 42 + rank). --task ur5sih: config 4 shard (HandArm, 8192 envs/GPU, DR on); --task allegro_hand:
config 3 (16384 envs); --task binpick: config 5 shard (HandArm bin-picking: hard_bin tote, 8 objects per env,
8192 envs/GPU). Multi-GPU: one process per GPU (torchrun), envs sharded, the only collective is the
per-log-interval RCCL all-reduce of episode statistics.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env steps/sec (whole node) at 4096/16384/65536 envs; ms/step p50"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
LOG_INTERVAL = 16                # rl_games horizon_length (train/Ur5SihMultiObjectManipulationPPO.yaml:65)


def algorithmic_bytes_per_env_step(n_links=29, n_dofs=17, n_obj=3, num_obs=147, num_act=11, P=1, dr=False,
                                   n_static_bodies=1):
    """HBM bytes one env-step of the fused kernel must move (state in + state/obs out), per env.
    B_api of SURVEY.md §8(d): the reference surface materialises body states and contact forces.
    Bin-picking: 8 objects, 6 static bodies (table-with-hole links, bin), obs 212."""
    f, i64 = 4, 8
    B = 1 + n_links + n_static_bodies + n_obj
    reads = {
        "dof_state": n_dofs * 2 * f, "sim_targets": n_dofs * f, "object_root_states": n_obj * 13 * f,
        "goal_and_table_rows": 2 * 13 * f, "object_indices": n_obj * i64, "collision_enabled": n_obj,
        "actions": num_act * f, "controller_state": (6 + 5 + 5) * f, "reset_progress": 2 * i64,
        "goal_pos": 3 * f, "target_cfg_index": 2 * i64, "obs_cache": n_obj * 7 * f, "goal_reached": 1,
        "object_pos_initial_target": 3 * f, "dof_position_targets": n_dofs * f,
    }
    if dr:      # per-env DR row: link + object mass scales and frictions
        reads["dr_scale"] = (2 * n_links + 2 * n_obj) * f
    writes = {
        "dof_state": n_dofs * 2 * f, "sim_targets": n_dofs * f, "object_root_states": n_obj * 13 * f,
        "rigid_body_state": B * 13 * f, "net_contact_force": B * 3 * f, "dof_position_targets": n_dofs * f,
        "controller_state": (6 + 5 + 5) * f, "obs": num_obs * f, "teacher_obs": num_obs * f,
        "obs_cache": n_obj * 7 * f, "rew": f, "reset_progress": 2 * i64, "timeout_reached": 2,
    }
    return sum(reads.values()) + sum(writes.values()), reads, writes


def allegro_bytes_per_env_step(n_links=17, n_dofs=16, num_obs=88, num_act=16):
    """B_api of the AllegroHand step, per env."""
    f, i64 = 4, 8
    B = n_links + 2
    reads = {"dof_state": n_dofs * 2 * f, "prev_targets": n_dofs * f, "object_root": 13 * f, "goal_root": 13 * f,
             "goal_state": 7 * f, "actions": num_act * f, "reset_progress_goal": 3 * i64, "successes": f}
    writes = {"dof_state": n_dofs * 2 * f, "dof_force": n_dofs * f, "sim_targets": n_dofs * f,
              "prev_targets": n_dofs * f, "object_root": 13 * f, "rigid_body_state": B * 13 * f,
              "net_contact_force": B * 3 * f, "obs": num_obs * f, "rew": f, "reset_progress_goal": 3 * i64,
              "successes": f, "timeout": 1}
    return sum(reads.values()) + sum(writes.values()), reads, writes


def kuka_bytes_per_env_step(n_links=24, n_dofs=23, num_obs=99, num_act=23, ts_read=48, ts_write=32):
    """B_api of the AllegroKuka step, per env: the state the step must read and the
    refreshed tensors / observations it must write (the task_state row is counted once each way)."""
    f, i64 = 4, 8
    B = n_links + 3
    reads = {"dof_state": n_dofs * 2 * f, "prev_targets": n_dofs * f, "object_root": 13 * f, "goal_state": 7 * f,
             "table_goal_rows": 2 * 13 * f, "actions": num_act * f, "reset_progress_goal": 3 * i64,
             "successes": f, "task_state": ts_read * f, "object_scale": 3 * f, "object_index": i64, "episode": 4}
    writes = {"dof_state": n_dofs * 2 * f, "dof_force": n_dofs * f, "sim_targets": n_dofs * f,
              "prev_targets": n_dofs * f, "object_root": 13 * f, "rigid_body_state": B * 13 * f,
              "net_contact_force": B * 3 * f, "obs": num_obs * f, "rew": f, "reset_progress_goal": 3 * i64,
              "successes": f, "timeout": 1, "task_state": ts_write * f}
    return sum(reads.values()) + sum(writes.values()), reads, writes


def pointcloud_bytes_per_env(pcs):
    """Algorithmic HBM bytes of one ha_pointclouds launch per env: every cloud point written once (16 B), the
    pose rows it reads once (7 floats per object and per sampled robot link), the object pool ids, the target
    index and goal_pos. Sample tables and the permutation are shared by all envs (L2-resident)."""
    f, i64 = 4, 8
    N, NO = pcs.sim.num_envs, pcs.sim.n_obj
    writes = sum(t.numel() for t in pcs.outputs.values()) // N * f
    obj = "object_synthetic_pointcloud" in pcs.outputs or "target_object_synthetic_pointcloud" in pcs.outputs
    reads = (NO * 7 * f + NO * i64 + i64) if obj else 0
    if "ur5sih_synthetic_pointcloud" in pcs.outputs:
        reads += len(set(pcs.robot_body.tolist())) * 7 * f
    if "sih_fingertip_pointcloud" in pcs.outputs:
        reads += 5 * 3 * f
    if "goal_synthetic_pointcloud" in pcs.outputs or "relative_goal_synthetic_pointcloud" in pcs.outputs:
        reads += 3 * f
    if "relative_goal_synthetic_pointcloud" in pcs.outputs:
        reads += 7 * f
    return writes + reads


# the point-cloud student list (Ur5SihMultiObjectManipulation.yaml:45) that bench --pointclouds runs
PC_STUDENT = ["goal_pos", "ur5_flange_pose", "dof_position_targets", "object_synthetic_pointcloud",
              "ur5sih_synthetic_pointcloud", "goal_synthetic_pointcloud"]


def cpu_baseline_kuka(num_envs=512, min_seconds=12.0, max_steps=4000, seed=0, subtask="regrasping"):
    """AllegroKuka on the host: C oracle physics (OpenMP over envs) + numpy task oracle (resets with host
    draws, targets, random forces, observations, reward)."""
    from oracle import kuka_oracle as KO
    from oracle.oracle_lib import HostState, Oracle
    from handarm_hip import model as HM
    scene = HM.load_scene(HM.KUKA_ASSET)
    params, cfg = HM.build_params({"subtask": subtask}, task=HM.TASK_ALLEGRO_KUKA)
    model = HM.build_model(scene, posed=HM.posed_group(HM.TASK_ALLEGRO_KUKA, cfg))
    N = num_envs
    lo, up = np.array(model.dof_lower[:23], np.float32), np.array(model.dof_upper[:23], np.float32)
    scales, offs = HM.kuka_env_tables(N, scene, cfg)
    hs = HostState(N, model=model, params=params)
    hs["object_scale"][:] = scales
    hs["collision_enabled"][:] = 1
    st = dict(dof=np.zeros((N, 23, 2), np.float32), root=np.zeros((N, 4, 13), np.float32),
              goal=np.zeros((N, 7), np.float32), targets=np.zeros((N, 23), np.float32), reset=np.ones(N, np.int64),
              reset_goal=np.ones(N, np.int64), progress=np.zeros(N, np.int64), successes=np.zeros(N, np.float32),
              ts=np.zeros((N, HM.AK_TS), np.float32))
    st["root"][..., 6] = 1.0
    st["root"][:, 2, 0:3] = list(model.table_pos)
    st["goal"][:, 6] = 1.0
    st["ts"][:, HM.AK_KP:HM.AK_KP + 12] = offs.reshape(N, 12)
    scal = HM.kuka_tolerance_scalars(cfg["success_tolerance"], cfg)
    orc = Oracle(model, params, N)
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (steps < 2 or time.perf_counter() - t0 < min_seconds):
        steps += 1
        dr = rng.random((N, 80), dtype=np.float32)
        ds, G = KO.draw_slots(params), KO.goal_draws(params)     # the U[-1, 1) slots of ak_task.h AK_DRAW_*
        u11 = {"regrasping": ((3, 6), (G + 3, G + 6)), "reorientation": (),
               "throw": ((0, 1), (4, 7), (G, G + 1), (G + 4, G + 7))}[subtask]
        for a_, b_ in u11 + ((ds["OBJ"], ds["OBJ"] + 3), (ds["VEL"], ds["VEL"] + 23)):
            dr[:, a_:b_] = dr[:, a_:b_] * 2 - 1
        dr[:, ds["FORCE_N"]:ds["FORCE_N"] + 3] = rng.standard_normal((N, 3))
        a = rng.uniform(-1, 1, (N, 23)).astype(np.float32)
        KO.pre(params, st, a, dr, lo, up)
        hs["dof_state"][:] = st["dof"].reshape(-1, 2)
        hs["root_state"][:] = st["root"].reshape(-1, 13)
        hs["sim_targets"][:] = st["targets"]
        hs["object_force"][:] = KO.quat_rotate(st["root"][:, 1, 3:7],
                                               st["ts"][:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3])[:, None]   # LOCAL_SPACE
        orc.simulate(hs, 1)
        st["dof"] = hs["dof_state"].reshape(N, 23, 2).copy()
        st["root"] = hs["root_state"].reshape(N, 4, 13).copy()
        rb = hs["rigid_body_state"].reshape(N, 27, 13)
        _, _, st["reset"], st["reset_goal"], st["progress"], st["successes"] = KO.post(
            params, st["ts"], st["dof"][..., 0], st["dof"][..., 1], rb, st["root"][:, 1], st["goal"],
            st["progress"] + 1, st["successes"], st["reset"], scales[:, 0], scal, lo, up)
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": N * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{N} envs x {steps} env-steps of the AllegroKuka {subtask} step (C oracle physics, "
                      f"OpenMP {threads} threads, + numpy task oracle), {dt:.1f} s"}


def cpu_baseline_allegro(num_envs=1024, min_seconds=12.0, max_steps=4000, seed=0):
    """AllegroHand on the host: C oracle physics (OpenMP over envs) + numpy task oracle."""
    from oracle import allegro_oracle as AO
    from oracle.oracle_lib import HostState, Oracle
    from handarm_hip import model as HM
    from tests import scenes
    model = HM.build_model(HM.load_scene(HM.ALLEGRO_ASSET))
    params, _ = HM.build_params(task=HM.TASK_ALLEGRO_HAND)
    lo, up = np.array(model.dof_lower[:16], np.float32), np.array(model.dof_upper[:16], np.float32)
    orc = Oracle(model, params, num_envs)
    st = HostState(num_envs, model=model, params=params)
    scenes.fill_allegro_scene(st, num_envs, lo, up, seed=seed)
    rng = np.random.default_rng(seed)
    N = num_envs
    reset = np.zeros(N, np.int64)
    goal = np.zeros(N, np.int64)
    prog = np.zeros(N, np.int64)
    succ = np.zeros(N, np.float32)
    cons = np.float32(0)
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (steps < 2 or time.perf_counter() - t0 < min_seconds):
        steps += 1
        a = rng.uniform(-1, 1, (N, 16)).astype(np.float32)
        st["sim_targets"][:] = AO.targets_from_actions(a, st["sim_targets"], lo, up)
        orc.simulate(st, 2)
        dof = st["dof_state"].reshape(N, 16, 2)
        obj = st["root_state"].reshape(N, 3, 13)[:, 1]
        AO.observations(dof[..., 0], dof[..., 1], st["dof_force"], obj, st["goal_state"], a, lo, up)
        prog += 1
        _, reset, goal, prog, succ, cons = AO.reward(obj, st["goal_state"], a, reset, goal, prog, succ, cons)
        # pre_physics_step of the next step: goal resets and reset_idx for the done envs
        root = st["root_state"].reshape(N, 3, 13)
        for e in np.nonzero(reset | goal)[0]:
            dr = rng.uniform(-1, 1, AO.DRAW_RESET_GOAL + 4).astype(np.float32)
            base = AO.DRAW_RESET_GOAL if reset[e] else AO.DRAW_GOAL
            AO.goal_reset(st["goal_state"], root, e, dr[base], dr[base + 1])
            goal[e] = 0
            if reset[e]:
                AO.env_reset(root, dof[..., 0], dof[..., 1], st["sim_targets"], e, dr[AO.DRAW_RESET:AO.DRAW_RESET + 37],
                             lo, up)
                reset[e], prog[e], succ[e] = 0, 0, 0
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{num_envs} envs x {steps} env-steps of the AllegroHand step (C oracle physics, "
                      f"OpenMP {threads} threads, + numpy task oracle), {dt:.1f} s"}


def cpu_baseline(num_envs=1024, min_seconds=12.0, max_steps=4000, seed=0, binpick=False, pool16=False):
    """The C oracle (scalar restatement, OpenMP over envs) + numpy task oracle, timed on host cores.

    Bounded sample: env-steps of the full batch are repeated until ``min_seconds`` of wall time have
    elapsed (about 10-30 s of CPU work), so the default bench run still finishes within minutes."""
    from oracle import task_oracle as O
    from oracle.oracle_lib import HostState, Oracle
    from handarm_hip import model as HM
    from tests import scenes
    scene = HM.load_scene(HM.BIN_ASSET if binpick else HM.ASSET)
    pool = (HM.POOL_WIDE if pool16 == "wide" else HM.POOL16) if pool16 else None
    model = HM.build_model(scene, pool)
    params, _ = HM.build_params({"n_objects": 8} if binpick else None)
    orc = Oracle(model, params, num_envs)
    st = HostState(num_envs, model=model, params=params)
    if binpick:
        scenes.fill_bin_scene(st, num_envs, scene, seed=seed)
    else:
        scenes.fill_scene(st, num_envs, seed=seed)
        if pool16:      # C4: each env's 3 objects are a random.sample of the pool (multi_object.py:569)
            st["object_indices"][:] = np.stack([np.random.default_rng(seed + e).choice(len(pool), 3, replace=False)
                                                for e in range(num_envs)])
    A, B, no, a0 = model.n_actors, model.n_bodies, params.n_objects, model.actor_object0
    actors = list(range(a0, a0 + no))
    rng = np.random.default_rng(seed)
    st["ur5_target"][:] = st["dof_state"].reshape(num_envs, 17, 2)[:, 0:6, 0]
    bbox_p = np.array([[model.pool_bbox_pos[i][:] for i in r] for r in st["object_indices"]], np.float32)
    bbox_q = np.array([[model.pool_bbox_quat[i][:] for i in r] for r in st["object_indices"]], np.float32)
    bbox_e = np.array([[model.pool_bbox_ext[i][:] for i in r] for r in st["object_indices"]], np.float32)
    prev = st["root_state"].reshape(num_envs, A, 13)[:, a0:a0 + no, 0:7].copy()
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (steps < 2 or time.perf_counter() - t0 < min_seconds):
        steps += 1
        st["actions"][:] = rng.uniform(-1, 1, (num_envs, 11))
        orc.controller(st)
        orc.simulate(st, 3)
        root = st["root_state"].reshape(num_envs, A, 13)
        body = st["rigid_body_state"].reshape(num_envs, B, 13)
        O.observations(root, body, st["dof_state"].reshape(num_envs, 17, 2), st["dof_position_targets"],
                       st["goal_pos"], st["target_object_index"], bbox_p, bbox_q, bbox_e, prev, object_actors=actors)
        O.reward(root, body, st["goal_pos"], st["target_object_index"], st["object_configuration_indices"],
                 st["object_pos_initial"].reshape(num_envs, 1, no, 3), object_actors=actors)
        prev = root[:, a0:a0 + no, 0:7].copy()
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{num_envs} envs x {steps} env-steps of the same HandArm{' bin-picking' if binpick else ''} step "
                      f"(C oracle physics, "
                      f"OpenMP {threads} threads, + numpy task oracle), {dt:.1f} s"}


# BASELINE.json configs the bench runs on the GPU (configs[0] is the reference's CPU-pipeline plumbing case,
# a parity-test size, not a bench line): key -> (task, envs per GPU, label)
CONFIGS = {
    "C2": ("allegro_kuka", 4096, "Arm+Allegro cube grasp (AllegroKuka regrasping), 4096 envs/GPU"),
    "C3": ("allegro_hand", 16384, "In-hand cube reorientation (AllegroHand), 16384 envs/GPU"),
    "C4": ("ur5sih", 8192, "HandArmGrasp shard, DR on, 3 objects per env sampled from the 16-object YCB pool, "
                           "8192 envs/GPU (65536 at 8 GPUs)"),
    "C5": ("binpick", 8192, "Multi-object bin-picking shard (hard_bin, 8 objects per env), 8192 envs/GPU "
                            "(32768 at 4 GPUs)"),
    # C4 on the wide pool (round 5, f1): 3 objects per env from the 16-object pool plus the 8 concave objects of the
    # reference's list as convex pieces (HM.POOL_WIDE)
    "C4w": ("ur5sih_wide", 8192, "HandArmGrasp shard, DR on, 3 objects per env sampled from the 24-object YCB pool "
                                 "(the 16-object pool + 8 concave objects decomposed into convex pieces), 8192 envs/GPU"),
}
STEP_KERNEL = {"allegro_kuka": "ak_step_kernel", "allegro_hand": "ah_step_kernel", "ur5sih": "ha_step_kernel",
               "binpick": "hb_step_kernel", "ur5sih_wide": "ha_step_kernel"}
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md:54)
VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2
NOMINAL_CLOCK_HZ = 2.4e9


def pool16_names(wide=False):
    """C4 / C5 object pool: the 16-object YCB pool (HM.POOL16), or with wide the 24 objects incl. the 8 concave ones as
    convex pieces (HM.POOL_WIDE, round 5)."""
    from handarm_hip import model as HM
    return list(HM.POOL_WIDE if wide else HM.POOL16)


def make_env(task, envs, seed, device, args):
    from handarm_hip.tasks import AllegroHand, AllegroKuka, Ur5SihMultiObjectManipulation
    wide = task == "ur5sih_wide" or args.wide_pool
    task = "ur5sih" if task == "ur5sih_wide" else task
    if task == "allegro_kuka":
        return AllegroKuka({"env": {"numEnvs": envs, "subtask": args.subtask}, "seed": seed}, device, device)
    if task == "allegro_hand":
        return AllegroHand({"env": {"numEnvs": envs}, "seed": seed}, device, device)
    envcfg = {"numEnvs": envs}
    if args.pointclouds:
        envcfg["observations"] = PC_STUDENT
    # C4 / C5 draw each env's objects by random.sample from the 16-object YCB pool (multi_object.py:569)
    cfg = {"env": envcfg, "seed": seed, "objects": {"dataset": {"ycb": pool16_names(wide)}}}
    if task == "binpick":
        # config 5: Ur5SihMultiObject with bin.asset hard_bin and 8 objects
        cfg.update({"bin": {"asset": "hard_bin"}})
        cfg["objects"]["num_objects"] = 8
    else:
        # config 4 is quoted with domain randomization on (BASELINE.json configs[3]); --no-dr turns it off
        cfg["task"] = {"randomize": not args.no_dr}
    return Ur5SihMultiObjectManipulation(cfg, device, device)


def bytes_per_env_step(task, env, args):
    if task == "allegro_kuka":
        return kuka_bytes_per_env_step(num_obs=env.num_obs)[0]
    if task == "allegro_hand":
        return allegro_bytes_per_env_step()[0]
    if task == "binpick":
        return algorithmic_bytes_per_env_step(n_obj=8, num_obs=env.sim.params.num_obs, n_static_bodies=6)[0]
    return algorithmic_bytes_per_env_step(dr=not args.no_dr)[0]          # ur5sih, ur5sih_wide


# configs whose step kernel another config shares: their committed SQ / PMC summaries carry the config in the name
# (profiles/sq_<kernel>_<key>.json), so C4w never borrows C4's (verdict r05 Weak #7)
PROFILE_TAG = {"C4w": "C4w"}


def _profile_json(name, envs, key=None):
    """profiles/<name>[_<tag>].json of this config's workload (None when that workload has no committed summary)."""
    tag = PROFILE_TAG.get(key)
    fn = os.path.join(ROOT, "profiles", f"{name}_{tag}.json" if tag else f"{name}.json")
    if not os.path.exists(fn):
        return None
    with open(fn) as f:
        d = json.load(f)
    if d.get("envs") != envs or (d.get("workload") not in (None, key)):
        return None
    return d


def compute_roofline(kernel, envs, kavg_ms, key=None):
    """Second roofline: VALU issue. Wave-instructions per launch come from the committed
    rocprofv3 SQ pass of the same workload (profiles/sq_<kernel>.json, tools/sq_summary.py); the kernel time is
    this run's. Mean resident waves per SIMD = 4 x SQ_WAVE_CYCLES (quad-cycles) / (kernel cycles at the nominal
    2.4 GHz) / 1024 SIMDs."""
    sq = _profile_json(f"sq_{kernel}", envs, key)
    if sq is None or not kavg_ms == kavg_ms:
        return None
    t = kavg_ms * 1e-3
    rate = sq["valu_insts_per_launch"] / t
    return {"bound": "valu", "achieved": rate, "peak": VALU_PEAK_WAVE_INSTS, "unit": "wave-instructions/s",
            "frac": rate / VALU_PEAK_WAVE_INSTS, "valu_insts_per_launch": sq["valu_insts_per_launch"],
            "waves_per_simd": 4 * sq["wave_cycles_per_launch"] / (t * NOMINAL_CLOCK_HZ) / 1024,
            "valu_active_frac": sq.get("valu_active_frac"),
            "valu_lane_utilization": sq.get("valu_lane_utilization"),
            "source": "profiles/sq_{}{}.json".format(kernel, "_" + PROFILE_TAG[key] if key in PROFILE_TAG else "")}


def run_config(task, envs, args, world, rank, device, log_interval_fn, key=None):
    """Build the env, W warmup steps (the first includes the all-env reset and, for the HandArm tasks, drop
    init), then exactly K timed steps between barrier + synchronize pairs; returns the record (rank 0 gets the
    max over ranks)."""
    from handarm_hip import parallel
    seed = 42 + rank                  # utils/utils.py:94 (seed + rank)
    random.seed(seed)
    torch.manual_seed(seed)
    env = make_env(task, envs, seed, device, args)
    env.reset()
    gen = torch.Generator(device=device).manual_seed(seed)
    pool = [torch.rand((envs, env.num_acts), device=device, generator=gen) * 2 - 1 for _ in range(8)]
    for k in range(args.warmup):
        env.step(pool[k % len(pool)])
        if (k + 1) % LOG_INTERVAL == 0 or k == args.warmup - 1:
            log_interval_fn(task, env)               # lazy initialisation of the logging path stays untimed
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    env.sim.enable_kernel_timing(args.steps)
    if hasattr(env, "contact_stats"):
        env.contact_stats(reset=True)               # contact-list diagnostics of the timed steps only
    # one event per step boundary (K + 1), not a pair per step: every event record costs a few microseconds of GPU
    # idle in the stream, which the measurement should not add to the workload
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    ev[0].record()
    for k in range(args.steps):
        env.step(pool[k % len(pool)])
        ev[k + 1].record()
        if (k + 1) % LOG_INTERVAL == 0:
            log_interval_fn(task, env)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    kern_ms = env.sim.kernel_times_ms(args.steps)
    pcs = getattr(env, "pointclouds", None)
    pc_ms = pcs.kernel_times_ms(args.steps) if pcs is not None else []
    extra = {}
    if task == "allegro_kuka":
        extra["episode_successes_mean"] = float(parallel.reduce_kuka_episode_stats(env)["successes"])
    elif task == "allegro_hand":
        extra["consecutive_successes"] = float(parallel.reduce_allegro_episode_stats(env)["consecutive_successes"])
    else:
        parallel.reduce_episode_stats(env)
        extra["success_rate_ewma"] = env.log_data.get("success_rate_ewma/overall")
    cs = env.contact_stats() if hasattr(env, "contact_stats") else None
    if cs is not None:
        extra["contacts"] = cs
    kernel = STEP_KERNEL[task]
    kavg = statistics.mean(kern_ms) if kern_ms else float("nan")
    bytes_env = bytes_per_env_step(task, env, args)
    achieved = bytes_env * envs / (kavg * 1e-3) / 1e9
    tj = _profile_json(f"traffic_{kernel}", envs, key)
    rec = {
        "value": world * envs * args.steps / elapsed, "unit": "env-steps/s",
        "ms_per_step": elapsed / args.steps * 1e3, "p50_ms_per_step": statistics.median(step_ms),
        "envs_per_gpu": envs, "total_envs": world * envs,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": tj.get("hbm_bytes_per_launch") if tj else None,
                     "kernel": kernel, "kernel_avg_ms": kavg, "algorithmic_bytes_per_env_step": bytes_env},
        "compute_roofline": compute_roofline(kernel, envs, kavg, key),
        **extra,
    }
    if pcs is not None:
        pb = pointcloud_bytes_per_env(pcs)
        pach = pb * envs / (statistics.mean(pc_ms) * 1e-3) / 1e9
        rec["pointcloud_roofline"] = {"bound": "hbm", "kernel": "ha_pointcloud_kernel", "observations": env.obs_names,
                                      "kernel_avg_ms": statistics.mean(pc_ms), "algorithmic_bytes_per_env": pb,
                                      "achieved": pach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": pach / HBM_PEAK_GBS}
    if task in ("ur5sih", "binpick", "ur5sih_wide") and args.episode_steps > 0:
        # the whole-episode window: the K-step window above starts right after the first reset, where
        # the arm has not reached the objects yet; the next episode_steps steps (one full 200-step episode, so one
        # synchronous reset step) give the steady-state rate and contact statistics north_star's figure is about
        env.contact_stats(reset=True)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        for k in range(args.episode_steps):
            env.step(pool[k % len(pool)])
            if (k + 1) % LOG_INTERVAL == 0:
                log_interval_fn(task, env)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        rec["episode_window"] = {"steps": args.episode_steps, "value": world * envs * args.episode_steps / el,
                                 "unit": "env-steps/s", "ms_per_step": el / args.episode_steps * 1e3,
                                 "includes_reset_step": args.episode_steps >= 200, "contacts": env.contact_stats()}
    del env, pool
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    return rec


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def run_cpu_baseline(task, args, seconds, threads=None):
    """Bounded CPU sample of the same workload (rank 0, N=1 only). threads: OpenMP threads of the C oracle
    (None = OMP_NUM_THREADS / all)."""
    from oracle import oracle_lib
    lib = oracle_lib.load()
    prev = lib.hao_get_threads()
    if threads:
        lib.hao_set_threads(threads)
    try:
        if task == "allegro_kuka":
            r = cpu_baseline_kuka(min(args.cpu_envs, 512), seconds, subtask=args.subtask)
        elif task == "allegro_hand":
            r = cpu_baseline_allegro(args.cpu_envs, seconds)
        else:
            r = cpu_baseline(args.cpu_envs // (4 if task == "binpick" else 1), seconds, binpick=task == "binpick",
                             pool16="wide" if task == "ur5sih_wide" else task == "ur5sih")
    finally:
        lib.hao_set_threads(prev)
    r["cores"] = threads or prev
    r["cpu_model"] = cpu_model()
    r["sample"] = r["sample"].replace(f"OpenMP {int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))} threads",
                                      f"OpenMP {r['cores']} threads")
    return r


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def check_gpu_count(n):
    """One rank per GPU: refuse N > torch.cuda.device_count() (which does not initialise the GPU) with exit code 2,
    unless the gloo share-GPU rehearsal is asked for (HA_DIST_BACKEND=gloo HA_DIST_SHARE_GPU=1)."""
    share = os.environ.get("HA_DIST_SHARE_GPU") == "1" and os.environ.get("HA_DIST_BACKEND") == "gloo"
    ndev = torch.cuda.device_count()
    if n > ndev and not (share and ndev > 0):
        print(f"bench.py: --gpus {n} asks for {n} ranks but this node has {ndev} GPU(s); one rank per GPU is the "
              f"process model (set HA_DIST_BACKEND=gloo HA_DIST_SHARE_GPU=1 to rehearse more ranks on fewer GPUs)",
              file=sys.stderr)
        return False
    return True


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without torchrun: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code (the reference scales the same way:
    `torchrun --nproc_per_node=N`, README.md:165-172; one sim per cuda:LOCAL_RANK, rlgames_utils.py:89-107).
    Runs before this process makes any GPU call: torch.cuda.device_count() does not initialise the GPU.
    The children inherit stdout, so rank 0's JSON line is this process's output."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # RCCL over dmabuf IPC on this host driver
    import subprocess
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--task", choices=["all", "allegro_kuka", "ur5sih", "allegro_hand", "binpick", "ur5sih_wide"],
                    default="all",
                    help="all (default): the C2 headline (allegro_kuka) plus sub-records for C3 (allegro_hand), "
                         "C4 (ur5sih shard), C5 (binpick shard) and C4w (ur5sih shard on the 24-object pool); or one "
                         "of them alone")
    ap.add_argument("--wide-pool", action="store_true", help="ur5sih / binpick: draw the objects from the 24-object "
                                                            "pool (the 8 concave objects as convex pieces)")
    ap.add_argument("--subtask", choices=["regrasping", "reorientation", "throw"], default="regrasping")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU of a single --task (default: its config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dr", action="store_true", help="ur5sih: domain randomization off")
    ap.add_argument("--pointclouds", action="store_true",
                    help="ur5sih / binpick: the point-cloud student observation list (synthetic clouds every step)")
    ap.add_argument("--episode-steps", type=int, default=200,
                    help="ur5sih / binpick: also time this many steps after the K-step window (one whole 200-step "
                         "episode incl. its synchronous reset step; 0: off)")
    ap.add_argument("--cpu-envs", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU sample of the headline config")
    ap.add_argument("--cpu-seconds-sub", type=float, default=4.0, help="CPU sample of each sub-record")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if not check_gpu_count(args.gpus):
            sys.exit(2)
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        ap.error(f"--gpus {args.gpus} but torchrun started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")

    from handarm_hip import parallel
    rank, local_rank, world, device = parallel.init_distributed("nccl")
    dist_info = parallel.describe()          # backend + the rank count an all-reduce over the group sees

    def log_interval(task, env):
        if task == "allegro_kuka":
            return parallel.reduce_kuka_episode_stats(env)   # RCCL all-reduce, 3 floats (N > 1)
        if task == "allegro_hand":
            return parallel.reduce_allegro_episode_stats(env)
        return parallel.reduce_episode_stats(env)            # RCCL all-reduce of the episode counters (N > 1)

    if args.task == "all":
        head, subs = "C2", ["C3", "C4", "C5", "C4w"]
    else:
        head = next(k for k, v in CONFIGS.items() if v[0] == args.task)
        subs = []
    records = {}
    for key in [head] + subs:
        task, envs, _ = CONFIGS[key]
        if key == head and args.envs:
            envs = args.envs
        records[key] = run_config(task, envs, args, world, rank, device, log_interval, key)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        for key in [head] + subs:
            task = CONFIGS[key][0]
            records[key]["cpu_baseline"] = run_cpu_baseline(task, args, args.cpu_seconds if key == head
                                                            else args.cpu_seconds_sub)
        # the 1-thread run BASELINE.md plans, next to the all-cores one (headline config, short sample)
        records[head]["cpu_baseline"]["one_thread"] = run_cpu_baseline(CONFIGS[head][0], args, 3.0, threads=1)
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    data = {"allegro_kuka": "synthetic (seeded U[-1,1] actions, AllegroKuka.yaml procedural cuboid family, random "
                            "object forces on)",
            "allegro_hand": "synthetic (seeded U[-1,1] actions, AllegroHand.yaml cube scene)",
            "ur5sih": "synthetic (seeded U[-1,1] actions, YCB objects of the 16-object pool, dropped at init)",
            "binpick": "synthetic (seeded U[-1,1] actions, hard_bin tote + 8 YCB objects per env from the 16-object "
                       "pool, dropped into the bin at init)",
            "ur5sih_wide": "synthetic (seeded U[-1,1] actions, YCB objects of the 24-object pool incl. 8 concave ones as "
                           "convex pieces, dropped at init)"}
    h = records[head]
    task, envs, label = CONFIGS[head]
    if task == "allegro_kuka" and args.subtask != "regrasping":
        label = label.replace("AllegroKuka regrasping", f"AllegroKuka {args.subtask}")
        data[task] = data[task].replace("random object forces on", "random object forces off" if args.subtask ==
                                        "throw" else "random object forces on")
    envs = h["envs_per_gpu"]
    out = {
        "metric": METRIC, "value": h["value"], "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": h["ms_per_step"], "p50_ms_per_step": h["p50_ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": data[task],
        "config": {"workload": f"{head}: {label} - one VecTask.step() of every env per step",
                   "envs_per_gpu": envs, "total_envs": world * envs, "parallelism": f"env-shard x{world}",
                   "observations": "point-cloud student list (Ur5SihMultiObjectManipulation.yaml:45)"
                   if args.pointclouds and task in ("ur5sih", "binpick") else "default"},
        "roofline": h["roofline"], "compute_roofline": h["compute_roofline"], "cpu_baseline": h.get("cpu_baseline"),
        "distributed": dist_info,
    }
    for k in ("episode_successes_mean", "consecutive_successes", "success_rate_ewma", "contacts", "pointcloud_roofline",
              "episode_window"):
        if k in h:
            out[k] = h[k]
    if subs:
        out["configs"] = {}
        for key in subs:
            r = dict(records[key])
            t = CONFIGS[key][0]
            r["workload"] = CONFIGS[key][2]
            r["data"] = data[t]
            out["configs"][key] = r
    print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
