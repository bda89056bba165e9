"""VecTask.step's head and tail folded into the step launch (ha_task_step_io, the Allegro tasks).

The reference's VecTask.step clamps the policy's actions (vec_task.py:400-404), the task stores them, and the step
returns obs_dict["obs"] = clamp(obs_buf) (vec_task.py:437) plus, for AllegroKuka, the extras means of
allegro_kuka_base.py:908-917. The build does all of it inside the one step launch; these tests check it against the
separate torch ops on the same step: actions outside +-1 land clamped in actions_buf, the returned obs equal
torch.clamp(obs_buf), and the extras equal torch's mean / min / max of the task-state columns, over several steps
(the group counters must be back at zero for the next launch) and at a shard size that is not a multiple of 64."""
import pytest
import torch

from handarm_hip import model as HM


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _actions(n, na, g):
    return (torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1) * 1.7        # partly outside +-1


@pytest.mark.gpu
@pytest.mark.parametrize("n", [100, 4096])
def test_kuka_step_io_matches_torch_ops(n):
    need_gpu()
    from handarm_hip.tasks import isaacgym_task_map
    env = isaacgym_task_map["AllegroKuka"]({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(11)
    for step in range(6):
        a = _actions(n, env.num_acts, g)
        obs_dict, rew, reset, ex = env.step(a)
        torch.cuda.synchronize()
        assert torch.equal(env.actions_buf, torch.clamp(a, -env.clip_actions, env.clip_actions)), step
        assert torch.equal(obs_dict["obs"], torch.clamp(env.obs_buf, -env.clip_obs, env.clip_obs)), step
        ts = env.sim.t["task_state"].view(n, -1)
        ps, to = ts[:, HM.AK_PREV_SUCC], ts[:, HM.AK_TRUE_OBJ]
        torch.testing.assert_close(ex["successes"], ps.mean(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(ex["true_objective_mean"], to.mean(), rtol=1e-5, atol=1e-6)
        assert float(ex["true_objective_min"]) == float(to.min()) and float(ex["true_objective_max"]) == float(to.max())
    # the same scalars again from a fresh launch of the separate epilogue kernel (its own reduction order)
    sc = torch.zeros(4, device="cuda:0")
    out = torch.empty_like(env.obs_buf)
    assert env.sim.lib.ha_task_epilogue(env.sim.h, out.data_ptr(), env.clip_obs, sc.data_ptr(), env.sim._stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, obs_dict["obs"])
    torch.testing.assert_close(sc[0], ex["successes"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sc[1], ex["true_objective_mean"], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_allegro_hand_step_io_matches_torch_ops():
    need_gpu()
    from handarm_hip.tasks import isaacgym_task_map
    n = 130
    env = isaacgym_task_map["AllegroHand"]({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(12)
    for step in range(4):
        a = _actions(n, env.num_acts, g)
        obs_dict, rew, reset, ex = env.step(a)
        torch.cuda.synchronize()
        ca = torch.clamp(a, -env.clip_actions, env.clip_actions)
        assert torch.equal(env.actions_buf, ca), step
        assert torch.equal(obs_dict["obs"], torch.clamp(env.obs_buf, -env.clip_obs, env.clip_obs)), step
        assert torch.equal(env.obs_buf[:, 72:88], ca), step          # the obs' action block is the clamped action


@pytest.mark.gpu
def test_step_io_rejects_ur5sih_handles():
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": 8}, "seed": 1}, "cuda:0", "cuda:0")
    out = torch.empty_like(env.obs_buf)
    assert env.sim.lib.ha_task_step_io(env.sim.h, 0, None, 1.0, out.data_ptr(), 5.0, None, env.sim._stream()) != 0
