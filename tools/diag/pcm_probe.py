"""Diagnostic (CPU, C oracle): how often the persistent contact manifolds (ha_params_t v13) replace a pair's narrow
phase in the bench workloads, and what the oracle's step costs with them, for a few tolerances.

    python tools/diag/pcm_probe.py [--task kuka|allegro|ur5sih|bin] [--envs 64] [--steps 120] [--tol off 5e-4,0.99999 ...]

Runs the same host loops as bench.py's cpu_baseline legs (random U[-1,1] actions, resets, random forces) and reports
the per-substep pair counts from contact_stats: manifolds refreshed from their record, narrow phases run, contacts
offered, and the oracle's wall time per step.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
import bench  # noqa: E402
from handarm_hip import model as HM  # noqa: E402
from oracle.oracle_lib import HostState, Oracle  # noqa: E402


def run_kuka(n, steps, seed=0):
    from oracle import kuka_oracle as KO
    scene = HM.load_scene(HM.KUKA_ASSET)
    model = HM.build_model(scene)
    params, cfg = HM.build_params({"subtask": "regrasping"}, task=HM.TASK_ALLEGRO_KUKA)
    lo, up = np.array(model.dof_lower[:23], np.float32), np.array(model.dof_upper[:23], np.float32)
    scales, offs = HM.kuka_env_tables(n, scene, cfg)
    hs = HostState(n, model=model, params=params)
    hs["object_scale"][:] = scales
    hs["collision_enabled"][:] = 1
    st = dict(dof=np.zeros((n, 23, 2), np.float32), root=np.zeros((n, 4, 13), np.float32),
              goal=np.zeros((n, 7), np.float32), targets=np.zeros((n, 23), np.float32), reset=np.ones(n, np.int64),
              reset_goal=np.ones(n, np.int64), progress=np.zeros(n, np.int64), successes=np.zeros(n, np.float32),
              ts=np.zeros((n, HM.AK_TS), np.float32))
    st["root"][..., 6] = 1.0
    st["root"][:, 2, 0:3] = list(model.table_pos)
    st["goal"][:, 6] = 1.0
    st["ts"][:, HM.AK_KP:HM.AK_KP + 12] = offs.reshape(n, 12)
    scal = HM.kuka_tolerance_scalars(cfg["success_tolerance"], cfg)
    orc = Oracle(model, params, n)
    rng = np.random.default_rng(seed)
    t_phys = 0.0
    for _ in range(steps):
        dr = rng.random((n, 80), dtype=np.float32)
        for a_, b_ in ((3, 6), (12, 15), (18, 21), (48, 71)):
            dr[:, a_:b_] = dr[:, a_:b_] * 2 - 1
        dr[:, 72:75] = rng.standard_normal((n, 3))
        a = rng.uniform(-1, 1, (n, 23)).astype(np.float32)
        KO.pre(params, st, a, dr, lo, up)
        hs["dof_state"][:] = st["dof"].reshape(-1, 2)
        hs["root_state"][:] = st["root"].reshape(-1, 13)
        hs["sim_targets"][:] = st["targets"]
        hs["object_force"][:] = KO.quat_rotate(st["root"][:, 1, 3:7], st["ts"][:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3])[:, None]
        t0 = time.perf_counter()
        orc.simulate(hs, 1)
        t_phys += time.perf_counter() - t0
        st["dof"] = hs["dof_state"].reshape(n, 23, 2).copy()
        st["root"] = hs["root_state"].reshape(n, 4, 13).copy()
        rb = hs["rigid_body_state"].reshape(n, 27, 13)
        _, _, st["reset"], st["reset_goal"], st["progress"], st["successes"] = KO.post(
            params, st["ts"], st["dof"][..., 0], st["dof"][..., 1], rb, st["root"][:, 1], st["goal"],
            st["progress"] + 1, st["successes"], st["reset"], scales[:, 0], scal, lo, up)
    return hs, t_phys


def run_ur5sih(n, steps, binpick=False, seed=0):
    from tests import scenes
    scene = HM.load_scene(HM.BIN_ASSET if binpick else HM.ASSET)
    pool = HM.POOL_WIDE if os.environ.get("HA_WIDE_POOL") else HM.POOL16
    model = HM.build_model(scene, None if binpick else pool)
    params, _ = HM.build_params({"n_objects": 8} if binpick else None)
    orc = Oracle(model, params, n)
    hs = HostState(n, model=model, params=params)
    if binpick:
        scenes.fill_bin_scene(hs, n, scene, seed=seed)
    else:
        scenes.fill_scene(hs, n, seed=seed)
        hs["object_indices"][:] = np.stack([np.random.default_rng(seed + e).choice(len(pool), 3, replace=False)
                                            for e in range(n)])
    rng = np.random.default_rng(seed)
    hs["ur5_target"][:] = hs["dof_state"].reshape(n, 17, 2)[:, 0:6, 0]
    t_phys = 0.0
    for _ in range(steps):
        hs["actions"][:] = rng.uniform(-1, 1, (n, 11))
        orc.controller(hs)
        t0 = time.perf_counter()
        orc.simulate(hs, 3)
        t_phys += time.perf_counter() - t0
    return hs, t_phys


def run_allegro(n, steps, seed=0):
    from oracle import allegro_oracle as AO
    from tests import scenes
    model = HM.build_model(HM.load_scene(HM.ALLEGRO_ASSET))
    params, _ = HM.build_params(task=HM.TASK_ALLEGRO_HAND)
    lo, up = np.array(model.dof_lower[:16], np.float32), np.array(model.dof_upper[:16], np.float32)
    orc = Oracle(model, params, n)
    hs = HostState(n, model=model, params=params)
    scenes.fill_allegro_scene(hs, n, lo, up, seed=seed)
    rng = np.random.default_rng(seed)
    t_phys = 0.0
    for _ in range(steps):
        a = rng.uniform(-1, 1, (n, 16)).astype(np.float32)
        hs["sim_targets"][:] = AO.targets_from_actions(a, hs["sim_targets"], lo, up)
        t0 = time.perf_counter()
        orc.simulate(hs, 2)
        t_phys += time.perf_counter() - t0
    return hs, t_phys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="kuka", choices=["kuka", "allegro", "ur5sih", "bin"])
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--tol", nargs="*", default=["off", "5e-4,0.99999"])
    a = ap.parse_args()
    for tol in a.tol:
        os.environ["HA_PCM"] = tol
        if a.task == "kuka":
            hs, t = run_kuka(a.envs, a.steps)
        elif a.task == "allegro":
            hs, t = run_allegro(a.envs, a.steps)
        else:
            hs, t = run_ur5sih(a.envs, a.steps, binpick=a.task == "bin")
        cs = hs["contact_stats"].astype(np.int64)
        sub = cs[:, 0].sum()
        print(f"{a.task} tol={tol:>16}: oracle {1e3 * t / a.steps:7.2f} ms/step  offered {cs[:, 3].sum() / sub:6.2f}/substep "
              f"(self {cs[:, 4].sum() / sub:5.2f})  refreshed {cs[:, 5].sum() / sub:5.2f}  narrow {cs[:, 6].sum() / sub:5.2f}"
              f"  over cap {cs[:, 1].sum() / sub:.4f}", flush=True)


if __name__ == "__main__":
    bench.__name__  # noqa: B018 (bench on sys.path for its helpers)
    main()
