"""AllegroKuka state dump / replay (cfg env.saveStates / env.loadInitialStates, allegro_kuka_base.py:1292-1312,
1349-1350,1445-1446,1493-1592) through the VecTask class on the GPU:
* saveStates: every dumped state is one the env actually passed through, with its own root and DOF rows;
* loadInitialStates: reset_idx writes the file's DOF states and cube root states into the reset envs, cycling
  through the file, while the position targets keep the randomised reset pose;
* the split reset (ha_task_reset, then ha_task_step) that state files switch on leaves trajectories unchanged.
"""
import pytest
import torch

from handarm_hip import model as HM
from handarm_hip import state_files as SF

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env(n, **env):
    from handarm_hip.tasks import isaacgym_task_map
    cfg = {"env": dict({"numEnvs": n, "subtask": "regrasping", "episodeLength": 30}, **env)}
    return isaacgym_task_map["AllegroKuka"](cfg, "cuda:0", "cuda:0")


def _run(env, steps, seed=5, record=None):
    n = env.num_envs
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    for _ in range(steps):
        env.step(torch.rand((n, 23), device="cuda:0", generator=g) * 2 - 1)
        if record is not None:
            record.append((env.root_state_tensor.view(n, -1, 13).cpu().clone(), env.dof_state.view(n, -1, 2).cpu().clone()))
    torch.cuda.synchronize()


def test_save_then_load_initial_states(tmp_path):
    need_gpu()
    n, path = 64, str(tmp_path / "states.bin")
    env = _env(n, saveStates=True, saveStatesFile=path)
    hist = []
    _run(env, 75, record=hist)
    seen = {}
    for root, dof in hist:
        for e in range(n):
            seen[dof[e].numpy().tobytes()] = root[e]
    root, dof = SF.read_state_file(path)
    assert root.shape[1:] == (4, 13) and dof.shape[1:] == (23, 2) and len(root) >= n
    for i in range(len(root)):
        key = dof[i].cpu().numpy().tobytes()
        assert key in seen, f"state {i} was never an env state"
        assert torch.equal(seen[key], root[i].cpu())

    env2 = _env(n, loadInitialStates=True, loadStatesFile=path)
    assert env2.num_initial_states == len(root)
    ids = torch.arange(n, device="cuda:0")
    env2.reset_idx(ids)
    torch.cuda.synchronize()
    a0 = env2.sim.model.actor_object0
    assert torch.equal(env2.dof_state.view(n, -1, 2).cpu(), dof[:n].cpu())
    assert torch.equal(env2.root_state_tensor.view(n, -1, 13)[:, a0].cpu(), root[:n, a0].cpu())
    assert not torch.equal(env2.prev_targets.view(n, -1).cpu(), dof[:n, :, 0].cpu())   # targets: reset pose
    assert env2.initial_state_idx == n

    # through step(): every env flagged, physics off, so the step's state is the loaded one (next slice of the
    # file, or its start when the slice would run past the end)
    start = n if 2 * n <= len(root) else 0
    env2.sim_flags = HM.FLAG_NO_PHYSICS
    env2.reset_buf[:] = 1
    env2.step(torch.zeros((n, 23), device="cuda:0"))
    torch.cuda.synchronize()
    torch.testing.assert_close(env2.dof_state.view(n, -1, 2).cpu(), dof[start:start + n].cpu(), rtol=0, atol=1e-6)
    torch.testing.assert_close(env2.root_state_tensor.view(n, -1, 13)[:, a0, :7].cpu(),
                               root[start:start + n, a0, :7].cpu(), rtol=0, atol=1e-5)


def test_split_reset_keeps_trajectories(tmp_path):
    """saveStates moves each step's resets into their own launch; the states it produces are the fused step's."""
    need_gpu()
    n = 64
    a, b = [], []
    _run(_env(n), 40, record=a)
    _run(_env(n, saveStates=True, saveStatesFile=str(tmp_path / "s.bin")), 40, record=b)
    worst = 0.0
    for (ra, da), (rb, db) in zip(a, b):
        worst = max(worst, float((ra - rb).abs().max()), float((da - db).abs().max()))
    print(f"split reset vs fused: max abs difference over 40 steps {worst:.3g}")
    assert worst == 0.0
