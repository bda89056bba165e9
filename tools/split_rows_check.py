"""Bit-identity check of the split constraint rows (clutter and Ur5Sih families) (PhysCfg::split in csrc/ha_physics.h)
against a build that keeps every family on dense rows (-DHA_DENSE_ROWS).

    python tools/split_rows_check.py --build                  # here: libhandarm_hip_dense.so next to the product lib
    python tools/split_rows_check.py --run dense gpurun_out/rows_dense.npz     # GPU box, one process per build
    python tools/split_rows_check.py --run split gpurun_out/rows_split.npz
    python tools/split_rows_check.py --compare gpurun_out/rows_dense.npz gpurun_out/rows_split.npz

Scenes (bin-picking, 8 objects, 256 envs, 3 gym.simulate calls each): the settled-clutter test scene; three
objects on hand link hulls (more link contacts than the family's LDS link slots (HA_LINK_SLOTS 4 for Ur5Sih, HB_LINK_SLOTS 2 for the clutter family, HA_AK_LINK_SLOTS 4 for AllegroKuka) -> global spill rows); eight objects
on link hulls (contact list at capacity). Ur5Sih (3 objects, 256 envs, 3 calls): the test scene, and
the three objects placed on hand link hulls (link contacts into the LDS link slots and beyond)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import _lib, build  # noqa: E402

DENSE_LIB = os.path.join(build.PKG, "libhandarm_hip_dense.so")
OUT_FIELDS = ("dof_state", "root_state", "rigid_body_state", "net_contact_force")


def run(kind, out):
    if kind == "dense":
        _lib.LIB_PATH = DENSE_LIB
    import torch
    from handarm_hip import model as HM
    from handarm_hip.sim import HandArmSim
    from tests import scenes
    n, NO, A, B = 256, 8, 12, 44
    res = {}
    for name, on_links in [("clutter", 0), ("links3", 3), ("links8", 8)]:
        sim = HandArmSim(n, "cuda:0", task_cfg={"n_objects": NO}, scene=HM.load_scene(HM.BIN_ASSET))
        st = {k: sim.t[k].cpu().numpy().copy() for k in HM.STATE_FIELDS
              if k not in ("stats", "term_sums") and k not in HM.null_fields(sim.task)}
        scenes.fill_bin_scene(st, n, sim.scene, seed=7)
        for k, v in st.items():
            sim.t[k].copy_(torch.as_tensor(v).reshape(sim.t[k].shape))
        if on_links:
            sim.simulate(1)
            torch.cuda.synchronize()
            body = sim.t["rigid_body_state"].cpu().numpy().reshape(n, B, 13)
            hl = sorted({int(sim.model.hull_link[k]) for k in range(sim.model.n_link_hulls)})
            links = [hl[-1 - 3 * i] for i in range(3)] if on_links == 3 else hl[-8:]
            rs = st["root_state"].reshape(n, A, 13)
            rs[:, 4:4 + on_links, 0:3] = body[:, sim.model.body_robot0 + np.array(links), 0:3]
            rs[:, 4:4 + on_links, 7:13] = 0.0
            for k, v in st.items():
                sim.t[k].copy_(torch.as_tensor(v).reshape(sim.t[k].shape))
        sim.simulate(3)
        torch.cuda.synchronize()
        for k in OUT_FIELDS:
            res[f"{name}/{k}"] = sim.t[k].cpu().numpy().copy()
        print(f"{kind} {name}: done", flush=True)
    for name, on_links in [("ur5sih", 0), ("ur5sih_links", 3)]:
        sim = HandArmSim(n, "cuda:0")
        st = {k: sim.t[k].cpu().numpy().copy() for k in HM.STATE_FIELDS
              if k not in ("stats", "term_sums") and k not in HM.null_fields(sim.task)}
        scenes.fill_scene(st, n, seed=11, n_obj=sim.n_obj)
        for k, v in st.items():
            sim.t[k].copy_(torch.as_tensor(v).reshape(sim.t[k].shape))
        if on_links:
            sim.simulate(1)
            torch.cuda.synchronize()
            body = sim.t["rigid_body_state"].cpu().numpy().reshape(n, sim.num_bodies, 13)
            hl = sorted({int(sim.model.hull_link[k]) for k in range(sim.model.n_link_hulls)})
            links = [hl[-1 - 2 * i] for i in range(on_links)]
            rs = st["root_state"].reshape(n, sim.num_actors, 13)
            rs[:, 3:3 + on_links, 0:3] = body[:, sim.model.body_robot0 + np.array(links), 0:3]
            rs[:, 3:3 + on_links, 7:13] = 0.0
            for k, v in st.items():
                sim.t[k].copy_(torch.as_tensor(v).reshape(sim.t[k].shape))
        sim.simulate(3)
        torch.cuda.synchronize()
        for k in OUT_FIELDS:
            res[f"{name}/{k}"] = sim.t[k].cpu().numpy().copy()
        print(f"{kind} {name}: done", flush=True)
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        print(f"{k:40s} {'bit-identical' if same else 'DIFFERENT (max |d| %.3e)' % np.abs(A[k] - B[k]).max()}")
        bad += not same
    print("split rows vs dense rows:", "bit-identical" if not bad else f"{bad} arrays differ")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--build":
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *build.FLAGS, "-DHA_DENSE_ROWS", "-I", build.INCLUDE,
               "-o", DENSE_LIB, os.path.join(build.CSRC, "handarm_hip.hip")]
        subprocess.check_call(cmd)
    elif sys.argv[1] == "--run":
        run(sys.argv[2], sys.argv[3])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
