"""AllegroHand random object forces in DEVICE mode (the counter-hash draws training runs with; the other force tests
replay the reference's draws): allegro_hand.py:557-560 (random_force_prob = exp((log lo - log hi) U + log hi) at
reset) and :617-625 (each step: rb_forces *= forceDecay ** (dt / forceDecayInterval); with probability
random_force_prob a new force N(0, 1)^3 * mass * forceScale).

Over 4096 envs x 60 NO_PHYSICS steps: every env's probability lies in [0.001, 0.1] and is log-uniform; a step either
decays the force by exactly ah_force_decay_step or draws a new one; the selection rate tracks the envs'
probabilities (overall and per probability tercile); the new forces' components are N(0, 1) x mass x forceScale;
the env's RNG counter advances once per step."""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM

pytestmark = pytest.mark.gpu

AH_TS_FORCE, AH_TS_PROB, AH_TS_RNG = 0, 3, 4          # ah_task.h AH_TS_*


def test_allegro_device_mode_random_forces():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from handarm_hip.sim import HandArmSim
    n, T, scale = 4096, 60, 2.0
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_HAND, "force_scale": scale},
                     task=HM.TASK_ALLEGRO_HAND)
    p = sim.params
    sim.t["reset_buf"].fill_(1)
    sim.task_step(HM.FLAG_NO_PHYSICS)                         # reset_idx draws the probabilities, then one step
    ts = sim.t["task_state"].cpu().numpy()
    prob = ts[:, AH_TS_PROB].copy()
    assert prob.min() >= 0.001 * (1 - 1e-5) and prob.max() <= 0.1 * (1 + 1e-5)
    lp = np.log(prob)
    assert abs(lp.mean() - 0.5 * (np.log(0.001) + np.log(0.1))) < 0.05      # log-uniform
    sim.t["reset_buf"].zero_()
    sel = np.zeros((T, n), bool)
    fresh = []
    f_prev, c_prev = ts[:, 0:3].copy(), ts[:, AH_TS_RNG].view(np.uint32).copy()
    decay = np.float32(p.ah_force_decay_step)
    for t in range(T):
        sim.t["reset_buf"].zero_()
        sim.t["reset_goal_buf"].zero_()
        sim.task_step(HM.FLAG_NO_PHYSICS)
        ts = sim.t["task_state"].cpu().numpy()
        f = ts[:, 0:3]
        c = ts[:, AH_TS_RNG].view(np.uint32)
        assert (c == c_prev + 1).all(), f"step {t}: the force RNG counter must advance once per step"
        np.testing.assert_array_equal(ts[:, AH_TS_PROB], prob)                  # no reset: the probability stays
        dec = (f_prev * decay).astype(np.float32)
        new = (f != dec).any(1)
        assert (f[~new] == dec[~new]).all()
        sel[t] = new
        fresh.append(f[new] / np.float32(p.ah_object_rb_mass * scale))
        f_prev, c_prev = f.copy(), c.copy()
    rate = sel.mean()
    np.testing.assert_allclose(rate, prob.mean(), rtol=0.06)
    order = np.argsort(prob)
    for part in np.array_split(order, 3):                                      # low / mid / high probability envs
        np.testing.assert_allclose(sel[:, part].mean(), prob[part].mean(), rtol=0.15)
    z = np.concatenate(fresh)
    assert len(z) > 3000
    assert abs(z.mean()) < 0.05 and abs(z.std() - 1.0) < 0.05
