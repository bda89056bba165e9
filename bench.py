#!/usr/bin/env python3
"""bench.py - env-steps/s of the fused HandArm (Ur5SihMultiObjectManipulation) VecTask.step on MI355X.

Workload (BASELINE.json config 4 per GPU): 8192 envs per GPU = one shard of the 65 536-env HandArmGrasp
node config, weak scaling (per-GPU work fixed as N grows). A step = one VecTask.step() for every env
(3 gym.simulate calls x 2 substeps + controllers + observables + reward + done + resets) on synthetic
i.i.d. U[-1,1] actions (seed 42 + rank). Multi-GPU: one process per GPU (torchrun), envs sharded, the
only collective is the per-log-interval RCCL all-reduce of episode counters.

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


def algorithmic_bytes_per_env_step(n_links=29, n_dofs=17, n_obj=3, num_obs=147, num_act=11, P=1, dr=False):
    """HBM bytes one env-step of the fused kernel must move (state in + state/obs out), per env.
    B_api of SURVEY.md §8(d): the reference surface materialises body states and contact forces."""
    f, i64 = 4, 8
    B = 1 + n_links + 1 + n_obj
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


def cpu_baseline(num_envs=1024, min_seconds=12.0, max_steps=4000, seed=0):
    """The C oracle (scalar restatement, OpenMP over envs) + numpy task oracle, timed on host cores.

    Bounded sample: env-steps of the full batch are repeated until ``min_seconds`` of wall time have
    elapsed (about 10-30 s of CPU work), so the default bench run still finishes within minutes."""
    from oracle import task_oracle as O
    from oracle.oracle_lib import HostState, Oracle
    from handarm_hip import model as HM
    from tests import scenes
    model = HM.build_model(HM.load_scene())
    params, _ = HM.build_params()
    orc = Oracle(model, params, num_envs)
    st = HostState(num_envs)
    scenes.fill_scene(st, num_envs, seed=seed)
    rng = np.random.default_rng(seed)
    st["ur5_target"][:] = st["dof_state"].reshape(num_envs, 17, 2)[:, 0:6, 0]
    bbox_p = np.array([[model.pool_bbox_pos[i][:] for i in r] for r in st["object_indices"]], np.float32)
    bbox_q = np.array([[model.pool_bbox_quat[i][:] for i in r] for r in st["object_indices"]], np.float32)
    bbox_e = np.array([[model.pool_bbox_ext[i][:] for i in r] for r in st["object_indices"]], np.float32)
    prev = st["root_state"].reshape(num_envs, 6, 13)[:, 3:, 0:7].copy()
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (steps < 2 or time.perf_counter() - t0 < min_seconds):
        steps += 1
        st["actions"][:] = rng.uniform(-1, 1, (num_envs, 11))
        orc.controller(st)
        orc.simulate(st, 3)
        root = st["root_state"].reshape(num_envs, 6, 13)
        body = st["rigid_body_state"].reshape(num_envs, 34, 13)
        O.observations(root, body, st["dof_state"].reshape(num_envs, 17, 2), st["dof_position_targets"],
                       st["goal_pos"], st["target_object_index"], bbox_p, bbox_q, bbox_e, prev)
        O.reward(root, body, st["goal_pos"], st["target_object_index"], st["object_configuration_indices"],
                 st["object_pos_initial"].reshape(num_envs, 1, 3, 3))
        prev = root[:, 3:, 0:7].copy()
    dt = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{num_envs} envs x {steps} env-steps of the same HandArm step (C oracle physics, "
                      f"OpenMP {threads} threads, + numpy task oracle), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--task", choices=["ur5sih", "allegro_hand"], default="ur5sih",
                    help="ur5sih: BASELINE config 4 shard (default); allegro_hand: config 3")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (8192 ur5sih, 16384 allegro_hand)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dr", action="store_true", help="ur5sih: domain randomization off")
    ap.add_argument("--cpu-envs", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()
    allegro = args.task == "allegro_hand"
    if args.envs is None:
        args.envs = 16384 if allegro else 8192

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

    from handarm_hip.tasks import AllegroHand, Ur5SihMultiObjectManipulation
    from handarm_hip import parallel
    cls = AllegroHand if allegro else Ur5SihMultiObjectManipulation
    # config 4 is quoted with domain randomization on (BASELINE.json configs[3]); --no-dr turns it off
    env = cls({"env": {"numEnvs": args.envs}, "seed": seed, "task": {"randomize": not (allegro or args.no_dr)}},
              device, device)
    env.reset()
    gen = torch.Generator(device=device).manual_seed(seed)
    pool = [torch.rand((args.envs, env.num_acts), device=device, generator=gen) * 2 - 1 for _ in range(8)]
    for k in range(args.warmup):
        env.step(pool[k % len(pool)])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    env.sim.enable_kernel_timing(args.steps)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        env.step(pool[k % len(pool)])
        ev[k][1].record()
        if (k + 1) % LOG_INTERVAL == 0 and not allegro:
            parallel.reduce_episode_stats(env)       # RCCL all-reduce of the episode counters (N > 1)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = [a.elapsed_time(b) for a, b in ev]
    kern_ms = env.sim.kernel_times_ms(args.steps)
    log = {} if allegro else env.log_data
    if rank == 0:
        total_env_steps = world * args.envs * args.steps
        value = total_env_steps / elapsed
        bytes_env, _, _ = allegro_bytes_per_env_step() if allegro else algorithmic_bytes_per_env_step(dr=not args.no_dr)
        kernel = "ah_step_kernel" if allegro else "ha_step_kernel"
        kavg = statistics.mean(kern_ms) if kern_ms else float("nan")
        achieved = bytes_env * args.envs / (kavg * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic_ah_step_kernel.json" if allegro else "traffic_step_kernel.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("envs") == args.envs:
                traffic = tj.get("hbm_bytes_per_launch")
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = (cpu_baseline_allegro if allegro else cpu_baseline)(args.cpu_envs, args.cpu_seconds)
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "p50_ms_per_step": statistics.median(step_ms), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic (seeded U[-1,1] actions, AllegroHand.yaml cube scene)" if allegro else
                     "synthetic (seeded U[-1,1] actions, YCB scene of Ur5SihMultiObject.yaml, objects dropped at init)"),
            "config": {"workload": (f"AllegroHand VecTask.step, 2x2 substeps, {args.envs} envs/GPU (BASELINE config 3)"
                                    if allegro else "HandArm Ur5SihMultiObjectManipulation VecTask.step, 3x2 substeps, "
                                   f"{args.envs} envs/GPU (BASELINE config 4 shard, DR "
                                   f"{'off' if args.no_dr else 'on'})"),
                       "envs_per_gpu": args.envs, "total_envs": world * args.envs, "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel, "kernel_avg_ms": kavg,
                         "algorithmic_bytes_per_env_step": bytes_env},
            "cpu_baseline": cpu,
            "success_rate_ewma": log.get("success_rate_ewma/overall"),
            "consecutive_successes": float(env.consecutive_successes.item()) if allegro else None,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
