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
    model = HM.build_model(scene)
    params, cfg = HM.build_params({"subtask": subtask}, task=HM.TASK_ALLEGRO_KUKA)
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
        for a_, b_ in ((3, 6), (12, 15), (18, 21), (48, 71)):
            dr[:, a_:b_] = dr[:, a_:b_] * 2 - 1
        dr[:, 72:75] = rng.standard_normal((N, 3))
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


def cpu_baseline(num_envs=1024, min_seconds=12.0, max_steps=4000, seed=0, binpick=False):
    """The C oracle (scalar restatement, OpenMP over envs) + numpy task oracle, timed on host cores.

    Bounded sample: env-steps of the full batch are repeated until ``min_seconds`` of wall time have
    elapsed (about 10-30 s of CPU work), so the default bench run still finishes within minutes."""
    from oracle import task_oracle as O
    from oracle.oracle_lib import HostState, Oracle
    from handarm_hip import model as HM
    from tests import scenes
    scene = HM.load_scene(HM.BIN_ASSET if binpick else HM.ASSET)
    model = HM.build_model(scene)
    params, _ = HM.build_params({"n_objects": 8} if binpick else None)
    orc = Oracle(model, params, num_envs)
    st = HostState(num_envs, model=model, params=params)
    if binpick:
        scenes.fill_bin_scene(st, num_envs, scene, seed=seed)
    else:
        scenes.fill_scene(st, num_envs, seed=seed)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--task", choices=["allegro_kuka", "ur5sih", "allegro_hand", "binpick"], default="allegro_kuka",
                    help="allegro_kuka: BASELINE config 2 (default); ur5sih: config 4 shard; allegro_hand: config 3; "
                         "binpick: config 5 shard")
    ap.add_argument("--subtask", choices=["regrasping", "reorientation"], default="regrasping")
    ap.add_argument("--envs", type=int, default=None,
                    help="envs per GPU (4096 allegro_kuka, 8192 ur5sih, 16384 allegro_hand, 8192 binpick)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dr", action="store_true", help="ur5sih: domain randomization off")
    ap.add_argument("--pointclouds", action="store_true",
                    help="ur5sih / binpick: the point-cloud student observation list (synthetic clouds every step)")
    ap.add_argument("--cpu-envs", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()
    allegro = args.task == "allegro_hand"
    kuka = args.task == "allegro_kuka"
    binpick = args.task == "binpick"
    if args.envs is None:
        args.envs = {"allegro_kuka": 4096, "ur5sih": 8192, "allegro_hand": 16384, "binpick": 8192}[args.task]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    device = f"cuda:{local_rank}"
    torch.cuda.set_device(device)
    seed = 42 + rank                  # utils/utils.py:94 (seed + rank)
    random.seed(seed)
    torch.manual_seed(seed)

    from handarm_hip.tasks import AllegroHand, AllegroKuka, Ur5SihMultiObjectManipulation
    from handarm_hip import parallel
    if kuka:
        env = AllegroKuka({"env": {"numEnvs": args.envs, "subtask": args.subtask}, "seed": seed}, device, device)
    elif binpick:
        # config 5: Ur5SihMultiObject with bin.asset hard_bin and 8 objects from the YCB pool
        from handarm_hip import model as HM
        pool = [o["name"] for o in HM.load_scene()["objects"]]
        envcfg = {"numEnvs": args.envs}
        if args.pointclouds:
            envcfg["observations"] = PC_STUDENT
        env = Ur5SihMultiObjectManipulation({"env": envcfg, "seed": seed, "bin": {"asset": "hard_bin"},
                                             "objects": {"num_objects": 8, "dataset": {"ycb": pool}}}, device, device)
    else:
        cls = AllegroHand if allegro else Ur5SihMultiObjectManipulation
        envcfg = {"numEnvs": args.envs}
        if args.pointclouds and not allegro:
            envcfg["observations"] = PC_STUDENT
        # config 4 is quoted with domain randomization on (BASELINE.json configs[3]); --no-dr turns it off
        env = cls({"env": envcfg, "seed": seed, "task": {"randomize": not (allegro or args.no_dr)}},
                  device, device)
    env.reset()
    gen = torch.Generator(device=device).manual_seed(seed)
    pool = [torch.rand((args.envs, env.num_acts), device=device, generator=gen) * 2 - 1 for _ in range(8)]
    def log_interval():
        if kuka:
            return parallel.reduce_kuka_episode_stats(env)   # RCCL all-reduce, 3 floats (N > 1)
        if not allegro:
            parallel.reduce_episode_stats(env)       # RCCL all-reduce of the episode counters (N > 1)
        return {}
    for k in range(args.warmup):
        env.step(pool[k % len(pool)])
        if (k + 1) % LOG_INTERVAL == 0 or k == args.warmup - 1:
            log_interval()                          # lazy initialisation of the logging path stays untimed
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    env.sim.enable_kernel_timing(args.steps)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    host_t = []
    for k in range(args.steps):
        ev[k][0].record()
        env.step(pool[k % len(pool)])
        ev[k][1].record()
        host_t.append(time.perf_counter())
        if (k + 1) % LOG_INTERVAL == 0:
            log_interval()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = [a.elapsed_time(b) for a, b in ev]
    if os.environ.get("BENCH_DEBUG"):
        gaps = [(b - a) * 1e3 for a, b in zip([t0] + host_t[:-1], host_t)]
        print("host ms/step issue:", [round(x, 3) for x in gaps], "\ngpu ms/step:", [round(x, 3) for x in step_ms],
              file=sys.stderr)
    kern_ms = env.sim.kernel_times_ms(args.steps)
    pcs = getattr(env, "pointclouds", None)
    pc_ms = pcs.kernel_times_ms(args.steps) if pcs is not None else []
    log = {} if (allegro or kuka) else env.log_data
    kstats = parallel.reduce_kuka_episode_stats(env) if kuka else {}
    if rank == 0:
        total_env_steps = world * args.envs * args.steps
        value = total_env_steps / elapsed
        if kuka:
            bytes_env, _, _ = kuka_bytes_per_env_step(num_obs=env.num_obs)
        elif allegro:
            bytes_env, _, _ = allegro_bytes_per_env_step()
        elif binpick:
            bytes_env, _, _ = algorithmic_bytes_per_env_step(n_obj=8, num_obs=env.num_obs, n_static_bodies=6)
        else:
            bytes_env, _, _ = algorithmic_bytes_per_env_step(dr=not args.no_dr)
        kernel = {"allegro_kuka": "ak_step_kernel", "allegro_hand": "ah_step_kernel", "ur5sih": "ha_step_kernel",
                  "binpick": "hb_step_kernel"}[args.task]
        kavg = statistics.mean(kern_ms) if kern_ms else float("nan")
        achieved = bytes_env * args.envs / (kavg * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", {"allegro_kuka": "traffic_ak_step_kernel.json",
                                             "allegro_hand": "traffic_ah_step_kernel.json",
                                             "ur5sih": "traffic_ha_step_kernel.json",
                                             "binpick": "traffic_hb_step_kernel.json"}[args.task])
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("envs") == args.envs:
                traffic = tj.get("hbm_bytes_per_launch")
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            if kuka:
                cpu = cpu_baseline_kuka(min(args.cpu_envs, 512), args.cpu_seconds, subtask=args.subtask)
            elif allegro:
                cpu = cpu_baseline_allegro(args.cpu_envs, args.cpu_seconds)
            else:
                cpu = cpu_baseline(args.cpu_envs, args.cpu_seconds, binpick=binpick)
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "p50_ms_per_step": statistics.median(step_ms), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": {"allegro_kuka": "synthetic (seeded U[-1,1] actions, AllegroKuka.yaml procedural cuboid family, "
                                     "random object forces on)",
                     "allegro_hand": "synthetic (seeded U[-1,1] actions, AllegroHand.yaml cube scene)",
                     "ur5sih": "synthetic (seeded U[-1,1] actions, YCB scene of Ur5SihMultiObject.yaml, objects "
                               "dropped at init)",
                     "binpick": "synthetic (seeded U[-1,1] actions, hard_bin tote + 8 YCB objects per env from the "
                                "16-object pool, dropped into the bin at init)"}[args.task],
            "config": {"workload": {
                "allegro_kuka": f"AllegroKuka{args.subtask.capitalize()} VecTask.step, 1x2 substeps, {args.envs} envs/GPU "
                                "(BASELINE config 2, Arm+Allegro cube grasp)",
                "allegro_hand": f"AllegroHand VecTask.step, 2x2 substeps, {args.envs} envs/GPU (BASELINE config 3)",
                "ur5sih": "HandArm Ur5SihMultiObjectManipulation VecTask.step, 3x2 substeps, "
                          f"{args.envs} envs/GPU (BASELINE config 4 shard, DR {'off' if args.no_dr else 'on'})",
                "binpick": "HandArm bin-picking Ur5SihMultiObjectManipulation VecTask.step, 3x2 substeps, 8 objects, "
                           f"{args.envs} envs/GPU (BASELINE config 5 shard)"}[args.task],
                       "envs_per_gpu": args.envs, "total_envs": world * args.envs, "parallelism": f"env-shard x{world}",
                       "observations": "point-cloud student list (Ur5SihMultiObjectManipulation.yaml:45)" if pcs is not None
                       else "default"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel, "kernel_avg_ms": kavg,
                         "algorithmic_bytes_per_env_step": bytes_env},
            "cpu_baseline": cpu,
            "pointcloud_roofline": None if pcs is None else {
                "bound": "hbm", "kernel": "ha_pointcloud_kernel", "observations": env.obs_names,
                "kernel_avg_ms": statistics.mean(pc_ms), "algorithmic_bytes_per_env": pointcloud_bytes_per_env(pcs),
                "achieved": pointcloud_bytes_per_env(pcs) * args.envs / (statistics.mean(pc_ms) * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": pointcloud_bytes_per_env(pcs) * args.envs / (statistics.mean(pc_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "success_rate_ewma": log.get("success_rate_ewma/overall"),
            "consecutive_successes": float(env.consecutive_successes.item()) if allegro else None,
            "episode_successes_mean": float(kstats["successes"]) if kuka else None,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
