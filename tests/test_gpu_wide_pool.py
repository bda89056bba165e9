"""The wide object pool (round 5, f1: the 8 concave objects of the reference's list as convex pieces) on the HIP path:
ha_simulate_kernel and the fused ha_step_kernel bit-identical to the C oracle with concave objects in every env, and a
VecTask episode on the 24-object pool."""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def _wide_scene(n, seed):
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState
    sim = HandArmSim(n, "cuda:0", pool_names=HM.POOL_WIDE)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_scene(st, n, seed=seed)
    rng = np.random.default_rng(seed)
    first = len(HM.POOL16)
    # object 0 concave in every env (all 8 in turn), objects 1, 2 from the whole pool (more concave ones among them)
    ids = np.stack([np.concatenate([[first + e % 8], rng.choice([k for k in range(24) if k != first + e % 8], 2,
                                                                replace=False)]) for e in range(n)])
    st["object_indices"][:] = ids
    # the objects dropped low over the table, slow: resting and colliding contacts within the window
    rs = st["root_state"].reshape(n, 6, 13)
    rs[:, 3:6, 2] = rng.uniform(0.54, 0.6, (n, 3))
    rs[:, 3:6, 7:13] *= 0.2
    return sim, st


@pytest.mark.parametrize("calls", [1, 10])
def test_wide_pool_simulate_matches_oracle_bit_for_bit(calls):
    need_gpu()
    from oracle.oracle_lib import Oracle
    n = 64
    sim, st = _wide_scene(n, 5)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums") and k not in HM.null_fields(sim.task):
            put(sim, k, st[k])
    sim.simulate(calls)
    Oracle(sim.model, sim.params, n).simulate(st, calls)
    cs = sim.t["contact_stats"].cpu().numpy()
    print(f"wide pool calls {calls}: contacts offered/substep {cs[:, 3].sum() / cs[:, 0].sum():.2f}, "
          f"narrow phases {cs[:, 6].sum() / cs[:, 0].sum():.2f}, refreshed {cs[:, 5].sum() / cs[:, 0].sum():.2f}")
    assert (cs[:, :6] == st["contact_stats"][:, :6]).all()
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"wide pool calls {calls}")


def test_wide_pool_vectask_episode():
    """Ur5SihMultiObjectManipulation on the 24-object pool (3 per env by random.sample, multi_object.py:569), DR on: drop
    initialisation, then 60 steps; everything finite and the objects on the table or in the hand."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    n = 512
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 3, "task": {"randomize": True},
                                         "objects": {"dataset": {"ycb": HM.POOL_WIDE}}}, "cuda:0", "cuda:0")
    env.reset()
    ids = env.sim.t["object_indices"].cpu().numpy()
    assert (ids >= len(HM.POOL16)).any(axis=1).mean() > 0.5        # most envs hold a concave object
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(60):
        obs, rew, done, extras = env.step(torch.rand((n, env.num_acts), device="cuda:0", generator=g) * 2 - 1)
    root = env.sim.t["root_state"].view(n, env.sim.num_actors, 13).cpu().numpy()
    a0 = env.sim.model.actor_object0
    assert np.isfinite(root).all() and torch.isfinite(obs["obs"]).all()
    z = root[:, a0:a0 + 3, 2]
    assert (z > 0.45).mean() > 0.99, "objects stay on (or above) the table"
