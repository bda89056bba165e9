"""Lifetime of the tensors VecTask.step returns: by default obs_dict["obs"] (and the Kuka extras
means) live in two alternating device buffers, valid through the next step and overwritten by the step after;
env.freshOutputs=True returns new tensors every step, as the reference's torch.clamp / .mean() do."""
import pytest
import torch

from handarm_hip.tasks import AllegroHand, AllegroKuka

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(cls, fresh):
    n = 64
    env = cls({"env": {"numEnvs": n, "freshOutputs": fresh}, "seed": 3}, "cuda:0", "cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(3)
    act = lambda: torch.rand((n, env.num_acts), device="cuda:0", generator=g) * 2 - 1   # noqa: E731
    obs_t, _, _, ex_t = env.step(act())
    held, snap = obs_t["obs"], obs_t["obs"].clone()
    key = "successes" if cls is AllegroKuka else "consecutive_successes"
    held_s, snap_s = ex_t[key], ex_t[key].clone()
    o1, _, _, _ = env.step(act())
    assert torch.equal(held, snap), "step t's obs changed by step t+1"
    assert torch.equal(held_s, snap_s)
    p1 = o1["obs"].data_ptr()
    o2, _, _, ex2 = env.step(act())
    torch.cuda.synchronize()
    return env, held, snap, p1, o2["obs"], held_s, ex2[key]


@pytest.mark.parametrize("cls", [AllegroHand, AllegroKuka])
def test_default_outputs_alternate_two_buffers(cls):
    need_gpu()
    env, held, snap, p1, o2, _, _ = _run(cls, False)
    assert held.data_ptr() == o2.data_ptr() != p1                  # step t+2 reuses step t's buffer
    assert torch.equal(held, o2)


@pytest.mark.parametrize("cls", [AllegroHand, AllegroKuka])
def test_fresh_outputs_survive_later_steps(cls):
    need_gpu()
    env, held, snap, p1, o2, held_s, s2 = _run(cls, True)
    assert held.data_ptr() != o2.data_ptr()
    assert torch.equal(held, snap), "a fresh obs tensor was overwritten"
    assert not torch.equal(o2, snap)
    assert held_s.data_ptr() != s2.data_ptr()
