"""GPU parity of the camera sensors (ha_render_camera), called through the C ABI: the depth ->
point-cloud arithmetic against the reference's own _compute_pointcloud (tests/golden/camera_pointcloud.npz), the
ray-cast depth / segmentation against the numpy oracle on simulated states, and the camera observables through
the VecTask.

Tolerances: points within 2e-6 of the reference golden (it adds and removes a global env offset in float32) and
validity equal on >= 99.5% of pixels; ray-cast segmentation equal to the oracle on >= 99% of pixels (a ray that
grazes a silhouette edge may flip with the last-ulp differences of tanf / division), depth within 1e-5 relative
where both hit the same body."""
import os

import numpy as np
import pytest
import torch

from handarm_hip import cameras as CAM
from handarm_hip import model as HM
from oracle import camera_oracle as CO

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
TOPVIEW = dict(pos=[0.28, 1.05, 0.9], quat=[0.213, 0.213, -0.674, 0.674], fovx=87)


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def cpu(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def test_pointcloud_from_depth_against_reference_golden():
    need_gpu()
    from handarm_hip.sim import HandArmSim
    d = np.load(os.path.join(G, "camera_pointcloud.npz"))
    N, H, W = d["depth"].shape
    sim = HandArmSim(N, "cuda:0")
    cam = CAM.CameraSensor(sim, d["pos"].tolist(), d["quat"].tolist(), float(d["fovx"]), (W, H), ["pointcloud"])
    cam.images["depth"].copy_(torch.from_numpy(d["depth"]))
    cam.render(from_depth=True)
    got = cpu(cam.images["pointcloud"])
    np.testing.assert_allclose(got[..., 0:3], d["pointcloud"][..., 0:3], rtol=0, atol=2e-6)
    assert np.mean(got[..., 3] == d["pointcloud"][..., 3]) >= 0.995


@pytest.mark.parametrize("bin_scene", [False, True])
def test_raycast_against_oracle(bin_scene):
    """Simulated states (reset pose, objects dropped from above the table / bin for 0.5 s), 64x36 images."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from tests import scenes
    N, W, H = 6, 64, 36
    scene = HM.load_scene(HM.BIN_ASSET if bin_scene else HM.ASSET)
    n_obj = 8 if bin_scene else 3
    sim = HandArmSim(N, "cuda:0", task_cfg={"n_objects": n_obj}, scene=scene)
    from oracle.oracle_lib import HostState
    st = HostState(N, model=sim.model, params=sim.params)
    if bin_scene:
        scenes.fill_bin_scene(st, N, scene, seed=3)
    else:
        scenes.fill_scene(st, N, seed=3)
    for k in ("root_state", "dof_state", "sim_targets", "object_indices", "goal_pos"):
        sim.t[k].copy_(torch.from_numpy(np.ascontiguousarray(st[k])).reshape(sim.t[k].shape).to(sim.t[k].dtype))
    sim.simulate(30)
    cam = CAM.CameraSensor(sim, TOPVIEW["pos"], TOPVIEW["quat"], TOPVIEW["fovx"], (W, H), scene=scene)
    cam.render()
    depth, seg, pc = cpu(cam.images["depth"]), cpu(cam.images["segmentation"]), cpu(cam.images["pointcloud"])
    root = cpu(sim.t["root_state"]).reshape(N, sim.num_actors, 13)
    body = cpu(sim.t["rigid_body_state"]).reshape(N, sim.num_bodies, 13)
    oi = cpu(sim.t["object_indices"])
    goal = cpu(sim.t["goal_pos"])
    c = dict(TOPVIEW, width=W, height=H, goal_radius=scene.get("goal_radius", 0.02),
             static_seg=CAM.static_segmentation_ids(scene))
    m = sim.model
    for e in range(N):
        dref, sref = CO.render_depth_segmentation(m, c, root[e], body[e], oi[e], goal[e], m.actor_object0,
                                                  m.body_robot0, n_obj)
        agree = seg[e] == sref
        assert agree.mean() >= 0.99, (e, agree.mean())
        both = agree & np.isfinite(dref)
        np.testing.assert_allclose(depth[e][both], dref[both], rtol=1e-5, atol=1e-6)
        assert (sref >= 3).any()                                          # objects are in view
    vinv = cam.view_inv
    want = CO.pointcloud_from_depth(depth, 2 * np.tan(np.radians(TOPVIEW["fovx"] / 2)),
                                    2 * np.tan(np.radians(TOPVIEW["fovx"] / 2)) * H / W, vinv)
    np.testing.assert_allclose(pc[..., 0:3], want[..., 0:3], rtol=0, atol=2e-6)


def test_camera_observables_through_vectask():
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    N = 32
    obs = ["ur5_flange_pose", "topview_depth", "topview_segmentation", "topview_pointcloud"]
    cfg = {"env": {"numEnvs": N, "observations": obs}, "seed": 1,
           "cameras": {"topview": dict(TOPVIEW, resolution=[160, 90])}}
    env = Ur5SihMultiObjectManipulation(cfg, "cuda:0", "cuda:0")
    assert env.observation_keys == ["obs", "topview_depth", "topview_segmentation", "topview_pointcloud"]
    out, _, _, _ = env.step(torch.zeros((N, 11), device="cuda:0"))
    assert out["obs"].shape == (N, 7)
    assert out["topview_depth"].shape == (N, 90, 160) and out["topview_segmentation"].dtype == torch.int32
    assert out["topview_pointcloud"].shape == (N, 90 * 160, 4)
    seg = cpu(out["topview_segmentation"])
    assert (seg >= 3).any()
    with pytest.raises(NotImplementedError):
        Ur5SihMultiObjectManipulation({"env": {"numEnvs": 4, "observations": ["topview_color"]},
                                       "cameras": {"topview": dict(TOPVIEW)}}, "cuda:0", "cuda:0")


def test_target_object_pointcloud():
    """<= P target points: exactly the oracle (pixel order, zero padding, w x 2); > P: P distinct target points
    (a random subset: every selected point is a target pixel's point, no repeats), a different subset per refresh."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from tests import scenes
    from oracle.oracle_lib import HostState
    N, W, H = 8, 160, 90
    sim = HandArmSim(N, "cuda:0")
    st = HostState(N, model=sim.model, params=sim.params)
    scenes.fill_scene(st, N, seed=4)
    for k in ("root_state", "dof_state", "sim_targets", "object_indices", "goal_pos"):
        sim.t[k].copy_(torch.from_numpy(np.ascontiguousarray(st[k])).reshape(sim.t[k].shape).to(sim.t[k].dtype))
    sim.simulate(10)
    for P in (4096, 64):
        cam = CAM.CameraSensor(sim, TOPVIEW["pos"], TOPVIEW["quat"], TOPVIEW["fovx"], (W, H),
                               ["target_object_pointcloud"], max_num_points=P)
        for tgt in range(3):
            sim.t["target_object_index"].fill_(tgt)
            cam.render()
            pc = cpu(cam.images["pointcloud"]).reshape(N, -1, 4)
            seg = cpu(cam.images["segmentation"]).reshape(N, -1)
            got = cpu(cam.images["target_object_pointcloud"])
            counts = (seg == 3 + tgt).sum(1)
            if P == 4096:
                assert counts.max() <= P
                np.testing.assert_array_equal(got, CO.target_pointcloud(pc, seg, np.full(N, tgt), P))
                continue
            first = got.copy()
            cam.render()
            again = cpu(cam.images["target_object_pointcloud"])
            for e in range(N):
                pts = pc[e][seg[e] == 3 + tgt].copy()
                pts[:, 3] *= 2
                k = min(counts[e], P)
                rows = {tuple(r) for r in pts.tolist()}
                assert all(tuple(r) in rows for r in first[e, :k].tolist())
                assert len({tuple(r) for r in first[e, :k].tolist()}) == len({tuple(r) for r in pts.tolist()} & {tuple(r) for r in first[e, :k].tolist()})
                assert np.all(first[e, k:] == 0)
                if counts[e] > P + 16:
                    assert not np.array_equal(first[e], again[e])
