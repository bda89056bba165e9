"""Dispatch-order refresh on the device (ha_update_env_order, HandArmSim.rebalance): one launch turns the contacts each
env offered since the last refresh into a longest-first permutation of the envs. The order is a scheduling hint
(results never depend on it: every parity test runs with it refreshed each step); here it must be a permutation,
non-increasing in the clamped cost, and leave cost_prev at the current counters."""
import numpy as np
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("n", [300, 4096])
def test_env_order_is_a_longest_first_permutation(n):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from handarm_hip.tasks import isaacgym_task_map
    env = isaacgym_task_map["AllegroKuka"]({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
    env.reset()
    sim = env.sim
    assert sim.rebalance_every > 0
    assert sim.lib.ha_set_order_cost(sim.h, 0) == 0      # the contacts-offered cost (the default sorts by spans)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(3):
        env.step(torch.rand((n, env.num_acts), device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    prev = sim._cost_prev.cpu().numpy().astype(np.int64)
    cs = sim.t["contact_stats"][:, 3].cpu().numpy().astype(np.int64)
    sim.rebalance()
    torch.cuda.synchronize()
    order = sim._env_order.cpu().numpy()
    assert np.array_equal(np.sort(order), np.arange(n))
    cost = np.clip(cs - prev, 0, 1023)[order]
    assert (np.diff(cost) <= 0).all()
    assert np.array_equal(sim._cost_prev.cpu().numpy(), cs.astype(np.int32))
    assert cost[0] > cost[-1]           # the envs did differ in contacts


@pytest.mark.gpu
def test_env_order_by_workgroup_spans_is_a_permutation():
    """The default cost (AllegroKuka, Ur5Sih): each env's workgroup span in the last step launch (stamped by the step
    kernel per launch slot, mapped to envs through the order that launch used). AllegroHand sorts by the contacts
    offered by default (round 6)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from handarm_hip.tasks import isaacgym_task_map
    n = 1000
    ah = isaacgym_task_map["AllegroHand"]({"env": {"numEnvs": 64}}, "cuda:0", "cuda:0")
    assert ah.sim.order_cost == "contacts"
    del ah
    env = isaacgym_task_map["AllegroKuka"]({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
    assert env.sim.order_cost == "time"
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    orders = []
    for _ in range(4):
        env.step(torch.rand((n, env.num_acts), device="cuda:0", generator=g) * 2 - 1)
        torch.cuda.synchronize()
        orders.append(env.sim._env_order.cpu().numpy().copy())
    for o in orders:
        assert np.array_equal(np.sort(o), np.arange(n))
    assert not all(np.array_equal(orders[0], o) for o in orders[1:])   # the spans differ, so does the order
