"""Bin-picking (BASELINE config 5) on the GPU: Ur5Sih with the hard_bin tote, a table with
a hole and 8 objects per env. These run the clutter kernel family (hb_*_kernel: 8 object slots, two contact
chunks of 21, a 65-coordinate generalized velocity) through the C ABI.

* task math: reference-generated goldens at 8 objects with the bin actor layout (tests/golden/
  make_goldens.py --bin), bit-exact for ints / done masks, <= 2e-7 for observation copies;
* physics: the scalar C oracle (same algorithm, same contact capacity and velocity-word layout), bit-identical
  on every env after 1 and 5 gym.simulate calls; over many calls, physical properties
  (objects settle inside the bin extent, the net contact force carries each object's weight);
* the VecTask surface at a shard size: drop initialisation into the bin, exact done / timeout masks.
"""
import os

import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
NO, A, B = 8, 12, 44


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make_bin_sim(n, **cfg):
    need_gpu()
    from handarm_hip.sim import HandArmSim
    c = {"n_objects": NO}
    c.update(cfg)
    return HandArmSim(n, "cuda:0", task_cfg=c, scene=HM.load_scene(HM.BIN_ASSET))


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


def test_bin_observe_reward_done_against_reference_goldens():
    d = np.load(os.path.join(G, "ur5sih_obs_reward_bin8.npz"))
    steps, n = d["rew"].shape
    sim = make_bin_sim(n, num_initial_poses=2)
    assert sim.num_actors == A and sim.num_bodies == B and sim.params.num_obs == 212
    # the golden's pool is the first 8 scene objects; their bbox constants are the model's
    put(sim, "object_indices", d["object_indices"])
    put(sim, "object_pos_initial", d["object_pos_initial"])
    put(sim, "object_quat_initial", d["object_quat_initial"])
    prev = np.zeros((n, NO, 7), np.float32)
    for s in range(steps):
        for name, key in [("root_state", "root"), ("rigid_body_state", "body"), ("dof_state", "dof"),
                          ("dof_position_targets", "targets"), ("goal_pos", "goal_pos"),
                          ("target_object_index", "target_idx"), ("object_configuration_indices", "cfg_idx"),
                          ("progress_buf", "progress_in"), ("reset_buf", "reset_in"),
                          ("goal_reached_before", "reached_in")]:
            put(sim, name, d[key][s])
        put(sim, "obs_cache", prev)
        sim.task_observe()
        obs = get(sim, "obs")
        np.testing.assert_allclose(obs, d["obs"][s], rtol=0, atol=2e-7)
        np.testing.assert_array_equal(get(sim, "teacher_obs"), obs)
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][s])
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][s])
        np.testing.assert_array_equal(get(sim, "timeout_buf").astype(bool), d["timeout"][s])
        np.testing.assert_array_equal(get(sim, "goal_reached_before").astype(bool), d["reached"][s])
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][s], rtol=1e-5, atol=1e-5)
        stats = get(sim, "stats")[0]
        assert stats[0] == d["reset"][s].sum() and stats[1] == d["reached"][s].sum()
        terms = get(sim, "term_sums")[0] / n
        np.testing.assert_allclose(terms, d["log_terms"][s], rtol=1e-4, atol=1e-6)
        cur = d["root"][s].reshape(n, A, 13)[:, 4:, 0:7]
        np.testing.assert_array_equal(get(sim, "obs_cache"), cur)
        prev = cur.copy()


def _bin_oracle_and_sim(n, seed):
    from oracle.oracle_lib import HostState, Oracle
    sim = make_bin_sim(n)
    orc = Oracle(sim.model, sim.params, n)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_bin_scene(st, n, sim.scene, seed=seed)
    for k in HM.STATE_FIELDS:
        if k in ("stats", "term_sums") or k in HM.null_fields(sim.task):
            continue
        put(sim, k, st[k])
    return sim, orc, st


@pytest.mark.parametrize("seed,calls", [(0, 1), (1, 1), (1, 5)])
def test_bin_simulate_matches_oracle_bit_for_bit(seed, calls):
    """Clutter family (8 objects, 42-contact list, 65-coordinate velocity, split rows) vs the C oracle: every
    physics output bit-identical on every env, including the deepest-kept contact replacement at capacity."""
    n = 128
    sim, orc, st = _bin_oracle_and_sim(n, seed)
    sim.simulate(calls)
    orc.simulate(st, calls)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"bin seed {seed} calls {calls}")
    gpu = {"rigid_body_state": get(sim, "rigid_body_state")}
    # fixed bodies (table-with-hole links, bin) come from the model, bit-exact
    body = gpu["rigid_body_state"].reshape(n, B, 13)
    fixed = np.array([list(sim.model.body_fixed_pose[k]) for k in range(sim.model.n_fixed_bodies)], np.float32)
    f0 = sim.model.body_fixed0
    np.testing.assert_array_equal(body[:, f0:f0 + len(fixed), 0:7], np.broadcast_to(fixed, (n,) + fixed.shape))
    np.testing.assert_array_equal(body[:, f0:f0 + len(fixed), 7:13], 0.0)


def test_bin_link_contacts_spill_rows_match_oracle():
    """Three objects placed on hand link hulls: more robot-link contacts per env than the clutter kernel's 2 LDS
    link slots (HB_LINK_SLOTS), so the split rows' global spill area (PhysCfg::split) carries part of the robot
    blocks, while the contact list stays below capacity. Bit-identical to the C oracle on every env, like the
    single-call test. (tools/split_rows_check.py checks this scene bit for bit against a dense-row build.)"""
    n = 64
    sim, orc, st = _bin_oracle_and_sim(n, 3)
    sim.simulate(1)                  # link poses of this scene (rigid_body_state rows of the robot)
    body = get(sim, "rigid_body_state").reshape(n, B, 13)
    hull_links = sorted({int(sim.model.hull_link[k]) for k in range(sim.model.n_link_hulls)})
    links = [hull_links[-1], hull_links[-4], hull_links[-7]]
    rs = st["root_state"].reshape(n, A, 13)
    rs[:, 4:7, 0:3] = body[:, sim.model.body_robot0 + np.array(links), 0:3]
    rs[:, 4:7, 7:13] = 0.0
    put(sim, "root_state", st["root_state"])
    for k in ("dof_state", "sim_targets", "contact_cache"):     # (the probe call above wrote manifold records)
        put(sim, k, st[k])
    sim.simulate(1)
    orc.simulate(st, 1)
    gpu = {k: get(sim, k) for k in ("dof_state", "root_state", "rigid_body_state", "net_contact_force")}
    assert np.isfinite(gpu["dof_state"]).all() and np.isfinite(gpu["root_state"]).all()
    f = gpu["net_contact_force"].reshape(n, B, 3)[:, sim.model.body_robot0:sim.model.body_robot0 + sim.model.n_links]
    touched = (np.abs(f).sum(-1) > 0).sum(1)
    print("link-contact scene: robot links in contact per env: median %d, max %d" % (np.median(touched), touched.max()))
    assert np.median(touched) >= 3
    scenes.assert_physics_bit_identical(sim, st, n, tag="bin link contacts")


def test_bin_simulate_many_calls_settles_in_bin():
    n = 512
    sim, orc, st = _bin_oracle_and_sim(n, 5)
    sim.simulate(90)                 # 1.5 s of simulated time
    root = get(sim, "root_state").reshape(n, A, 13)
    assert np.isfinite(root).all()
    lo, hi = np.array(sim.scene["bin_extent"][0]), np.array(sim.scene["bin_extent"][1])
    pos = root[:, 4:, 0:3]
    inside = ((pos >= lo - 0.01) & (pos <= hi + 0.01)).all(-1)
    print("bin settle: inside %.4f, z range %.3f..%.3f, median speed %.4f"
          % (inside.mean(), pos[..., 2].min(), pos[..., 2].max(), np.median(np.abs(root[:, 4:, 7:10]))))
    assert inside.mean() > 0.995, "objects must stay inside the tote"
    assert pos[..., 2].min() > 0.30, "nothing falls through the bin floor (top at z = 0.315)"
    assert np.median(np.abs(root[:, 4:, 7:10])) < 0.02
    f = get(sim, "net_contact_force").reshape(n, B, 3)[:, 36:44]
    mass = np.array([sim.model.pool_mass[i] for i in range(16)])[get(sim, "object_indices")]
    np.testing.assert_allclose(np.median(f[..., 2] / (9.81 * mass)), 1.0, rtol=0.15)


def test_bin_gpu_runs_are_bitwise_deterministic():
    outs = []
    for _ in range(2):
        sim, _, _ = _bin_oracle_and_sim(64, 11)
        sim.simulate(5)
        outs.append(get(sim, "root_state").copy())
    np.testing.assert_array_equal(outs[0], outs[1])


def test_bin_vectask_episode():
    """Ur5SihMultiObjectManipulation with bin.asset hard_bin and 8 objects: drop initialisation into the tote
    (objects_in_bin, multi_object.py:705-718), obs 212 wide, exact done / timeout masks at 200 steps."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    n = 2048
    cfg = {"env": {"numEnvs": n}, "bin": {"asset": "hard_bin"},
           "objects": {"num_objects": NO, "dataset": {"ycb": HM.POOL16}}}
    env = Ur5SihMultiObjectManipulation(cfg, "cuda:0", "cuda:0")
    obs = env.reset()["obs"]
    assert obs.shape == (n, 212) and env.num_actors == A and env.num_bodies == B
    g = torch.Generator(device="cuda:0").manual_seed(42)
    lo = torch.tensor(env.bin_extent[0], device="cuda:0")
    hi = torch.tensor(env.bin_extent[1], device="cuda:0")
    for step in range(1, 202):
        a = torch.rand((n, 11), device="cuda:0", generator=g) * 2 - 1
        obs_dict, rew, reset, extras = env.step(a)
        if step % 50 == 1:
            print(f"bin episode: step {step}", flush=True)
        if step == 1:
            torch.cuda.synchronize()
            init = env.sim.t["object_pos_initial"][:, 0]
            inb = ((init >= lo - 1e-3) & (init <= hi + 1e-3)).all(-1)
            print("bin episode: initial poses inside the tote %.4f" % inb.float().mean().item())
            assert inb.float().mean() > 0.99
            assert (env.progress_buf == 1).all()
        if step in (1, 100, 200, 201):
            torch.cuda.synchronize()
            assert torch.isfinite(obs_dict["obs"]).all() and torch.isfinite(rew).all()
        if step == 199:
            assert (reset == 0).all()
        if step == 200:
            assert (reset == 1).all() and extras["time_outs"].all()
        if step == 201:
            assert (env.progress_buf == 1).all() and (reset == 0).all()
    o = env.obs_buf
    a0 = env.actor_object0
    torch.testing.assert_close(o[:, 80:80 + 3 * NO], env.root_pos[:, a0:a0 + NO].reshape(n, 3 * NO), rtol=0, atol=0)
    log = env.log_data
    assert "success_rate_ewma/overall" in log
