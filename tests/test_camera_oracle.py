"""Camera sensors on the CPU: the oracle's depth -> point-cloud arithmetic against the reference's
own _compute_pointcloud (tests/golden/camera_pointcloud.npz), and the camera model's self-consistency (a ray cast
hit, converted back through the view / projection matrices, lands where the ray hit)."""
import os

import numpy as np
import pytest
import torch

from handarm_hip import cameras as CAM
from handarm_hip import model as HM
from oracle import camera_oracle as CO

G = os.path.join(os.path.dirname(__file__), "golden")


def test_pointcloud_from_depth_matches_reference():
    """Points within 2e-6 (the reference adds and removes a global env offset of up to 2 m in float32),
    validity bit-exact except on that rounding."""
    d = np.load(os.path.join(G, "camera_pointcloud.npz"))
    P = d["proj"]
    fu, fv = np.float32(2) / P[0, 0], np.float32(2) / P[1, 1]
    vinv = torch.linalg.inv(torch.from_numpy(d["view_local"])).numpy()
    got = CO.pointcloud_from_depth(d["depth"], fu, fv, vinv)
    want = d["pointcloud"]
    np.testing.assert_allclose(got[..., 0:3], want[..., 0:3], rtol=0, atol=2e-6)
    assert np.mean(got[..., 3] == want[..., 3]) > 0.995
    assert 0.2 < want[..., 3].mean() < 0.9                  # the golden exercises both validity branches


def test_view_and_projection_conventions():
    """Camera looks along its local +X (Isaac Gym); the topview camera of Ur5SihMultiObject.yaml looks toward
    the table (-y) and down; the view matrix maps the camera position to the origin."""
    pos, quat = [0.28, 1.05, 0.5], [0.213, 0.213, -0.674, 0.674]
    V = CAM.view_matrix(pos, quat).astype(np.float64)
    np.testing.assert_allclose(np.r_[pos, 1.0] @ V, [0, 0, 0, 1], atol=1e-6)
    fwd = -V[0:3, 2]                                          # view z axis points backwards
    assert fwd[1] < -0.5 and fwd[2] < -0.3
    R = CO.camera_axes(quat)
    np.testing.assert_allclose(R, V[0:3, 0:3], atol=1e-6)


def test_raycast_points_round_trip():
    """Oracle ray cast of a small image of the default scene, then depth -> points: every hit pixel's point is
    where its ray hit (pos + t d), so the camera model and the reference's inverse mapping agree."""
    scene = HM.load_scene()
    m = HM.build_model(scene)
    W, H = 32, 18
    cam = dict(pos=[0.28, 1.05, 0.9], quat=[0.213, 0.213, -0.674, 0.674], fovx=87.0, width=W, height=H,
               goal_radius=0.02, static_seg=[0])
    B, A = m.n_bodies, m.n_actors
    body = np.zeros((B, 13), np.float32)
    body[:, 6] = 1
    body[1:1 + m.n_links, 0:3] = [0.0, 0.0, 0.5]
    root = np.zeros((A, 13), np.float32)
    root[:, 6] = 1
    root[3:6, 0:3] = [[0.2, 0.55, 0.55], [0.3, 0.6, 0.56], [0.4, 0.5, 0.58]]
    depth, seg = CO.render_depth_segmentation(m, cam, root, body, [0, 1, 2], [0.28, 0.58, 0.8], m.actor_object0,
                                              m.body_robot0, 3)
    assert np.isfinite(depth).mean() > 0.9 and (seg >= 3).sum() > 0 and (seg == 0).sum() > 0
    V = CAM.view_matrix(cam["pos"], cam["quat"])
    vinv = np.linalg.inv(V.astype(np.float64)).astype(np.float32)
    tanx = np.tan(np.radians(43.5))
    pc = CO.pointcloud_from_depth(depth[None], 2 * tanx, 2 * tanx * H / W, vinv, max_depth=10.0)[0]
    d = CO.rays(W, H, 87.0, cam["quat"]).reshape(H, W, 3)
    hit = np.isfinite(depth)
    expect = np.asarray(cam["pos"], np.float32) + d * (-depth)[..., None]
    np.testing.assert_allclose(pc[hit][:, 0:3], expect[hit], rtol=0, atol=2e-5)


def test_static_segmentation_ids():
    assert CAM.static_segmentation_ids(HM.load_scene()) == [0]
    ids = CAM.static_segmentation_ids(HM.load_scene(HM.BIN_ASSET))
    assert ids.count(2) == 5 and ids.count(0) == 4
