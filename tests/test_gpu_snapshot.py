"""Snapshot / restore of the device env-state SoA (HandArmSim.snapshot / restore; SURVEY.md §5 checkpoint row):
steps after a restore reproduce the steps after the snapshot bit for bit, for the three task classes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(env, n, na, seed):
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    out = []
    for _ in range(n):
        od, rew, reset, _ = env.step(torch.rand((env.num_envs, na), device="cuda:0", generator=g) * 2 - 1)
        out.append((od["obs"].clone(), rew.clone(), reset.clone(), env.sim.t["dof_state"].clone(),
                    env.sim.t["root_state"].clone()))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("task", ["allegro_kuka", "allegro_hand", "ur5sih"])
def test_restore_reproduces_the_steps_after_the_snapshot(task):
    from handarm_hip.tasks import AllegroHand, AllegroKuka, Ur5SihMultiObjectManipulation
    n = 256
    cls = {"allegro_kuka": AllegroKuka, "allegro_hand": AllegroHand, "ur5sih": Ur5SihMultiObjectManipulation}[task]
    env = cls({"env": {"numEnvs": n}, "seed": 3}, "cuda:0", "cuda:0")
    env.reset()
    na = env.num_acts
    _run(env, 6, na, seed=1)                      # past the first all-env reset
    snap = env.sim.snapshot()
    a = _run(env, 12, na, seed=2)
    env.sim.restore(snap)
    b = _run(env, 12, na, seed=2)
    for s, (x, y) in enumerate(zip(a, b)):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(u.cpu().numpy(), v.cpu().numpy(), err_msg=f"{task} step {s}")
