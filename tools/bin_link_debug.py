"""GPU diagnostic: the bin link-contact parity scene (tests/test_gpu_bin.py) per narrow-phase switch: envs whose
physics differs from the oracle, and for those the oracle's contacts vs the GPU's offered count.
Usage (GPU box): python tools/bin_link_debug.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import model as HM  # noqa: E402
from handarm_hip import _lib  # noqa: E402
if os.environ.get("HA_LIB"):                 # a variant build instead of the product
    _lib.LIB_PATH = os.environ["HA_LIB"]
from oracle.oracle_lib import HostState, Oracle  # noqa: E402
from tests import scenes  # noqa: E402
from tests import test_gpu_bin as T  # noqa: E402

n = 64
for flags in (0, 1, 2, 3):
    sim = T.make_bin_sim(n, narrow_phase_flags=flags)
    orc = Oracle(sim.model, sim.params, n)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_bin_scene(st, n, sim.scene, seed=3)
    for k in HM.STATE_FIELDS:
        if k in ("stats", "term_sums") or k in HM.null_fields(sim.task):
            continue
        T.put(sim, k, st[k])
    sim.simulate(1)
    body = T.get(sim, "rigid_body_state").reshape(n, T.B, 13)
    hull_links = sorted({int(sim.model.hull_link[k]) for k in range(sim.model.n_link_hulls)})
    links = [hull_links[-1], hull_links[-4], hull_links[-7]]
    rs = st["root_state"].reshape(n, T.A, 13)
    rs[:, 4:7, 0:3] = body[:, sim.model.body_robot0 + np.array(links), 0:3]
    rs[:, 4:7, 7:13] = 0.0
    T.put(sim, "root_state", st["root_state"])
    for k in ("dof_state", "sim_targets"):
        T.put(sim, k, st[k])
    sim.t["contact_stats"].zero_()
    c0 = {}
    st0 = st.copy()
    sim.simulate(1)
    orc.simulate(st, 1)
    torch.cuda.synchronize()
    g = sim.t["dof_state"].cpu().numpy().reshape(n, -1)
    o = np.asarray(st["dof_state"]).reshape(n, -1)
    bad = np.where(~(g.view(np.uint32) == o.view(np.uint32)).all(1))[0]
    cs = sim.t["contact_stats"].cpu().numpy().reshape(n, 4)
    print(f"flags {flags}: differing envs {bad.tolist()}", flush=True)
    for e in bad[:3]:
        c = Oracle(sim.model, sim.params, n).contacts(st0, int(e))
        print(f"  env {e}: oracle contacts substep0 {len(c)}, GPU offered (2 substeps) {cs[e, 3]}, stats {cs[e].tolist()}")
        for r in c:
            print("    ", np.array2string(np.asarray(r), precision=5, max_line_width=200))
