"""Camera sensors of Ur5SihMultiObject on the device.

Host side of ``ha_render_camera`` (include/handarm_abi.h). A camera is configured like the reference's
``CameraSensorProperties`` (hand_arm/utils/camera.py:84-208, cameras of Ur5SihMultiObject.yaml:35-53: pos, quat,
fovx, resolution) and produces the images of ``IsaacGymCameraSensor`` (:250-333): depth and segmentation
(here ray cast against the collision geometry, see csrc/ha_camera.h) and the point cloud of
``_compute_pointcloud`` (:302-311). One kernel launch renders every env.

Conventions (Isaac Gym's, restated): the camera looks along its local +X with +Z up; the view matrix is the
OpenGL one in row-vector form (points as rows, ``[p, 1] @ V``), so depth is the negative view-space z; the
projection matrix's [0][0] / [1][1] are 1 / tan(fov / 2) with square pixels. Envs are rendered in their own
frame, so the reference's ``global_to_environment_points`` (:72-81) offset is zero here.
"""
import ctypes as C
import math

import numpy as np
import torch

from . import _lib
from . import model as HM

IMAGE_TYPES = ("depth", "segmentation", "pointcloud", "target_object_pointcloud")
WORKSPACE = (-0.07, 0.63, 0.33, 0.83)     # camera.py:303-304 x_range, y_range
MAX_DEPTH = 10.0                          # camera.py:302


def quat_to_matrix(q):
    x, y, z, w = np.asarray(q, np.float64) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def view_matrix(pos, quat):
    """(4, 4) float32 OpenGL view matrix, row-vector convention: view axes x right = -Y_cam, y up = Z_cam,
    z back = -X_cam (camera frame: +X forward, +Z up)."""
    Rc = quat_to_matrix(quat)
    Rgl = np.stack([-Rc[:, 1], Rc[:, 2], -Rc[:, 0]], axis=1)     # columns: view axes in the env frame
    V = np.eye(4)
    V[0:3, 0:3] = Rgl
    V[3, 0:3] = -np.asarray(pos, np.float64) @ Rgl
    return V.astype(np.float32)


def projection_matrix(fovx_deg, width, height):
    """(4, 4) float32 perspective matrix whose [0][0], [1][1] are what camera.py:316-319 reads."""
    tx = math.tan(0.5 * math.radians(fovx_deg))
    ty = tx * height / width
    P = np.zeros((4, 4), np.float32)
    P[0, 0], P[1, 1] = 1.0 / tx, 1.0 / ty
    P[2, 2], P[2, 3], P[3, 2] = -1.0, -1.0, -0.02          # near 0.01 (only [0][0], [1][1] are used)
    return P


def static_segmentation_ids(scene):
    """Segmentation id per static box: the table (and the table-with-hole links) 0, bin pieces 2
    (multi_object.py:631,636)."""
    statics = scene.get("statics")
    if not statics:
        return [0]
    return [2 if s["name"].startswith("bin") else 0 for s in statics]


class CameraSensor:
    """One camera over every env of ``sim``. ``images[kind]`` for kind in ``outputs``: depth (N, H, W) f32,
    segmentation (N, H, W) int32, pointcloud (N, H, W, 4) f32 - the reference's current_sensor_observation."""

    def __init__(self, sim, pos, quat, fovx=87, resolution=(160, 90), outputs=IMAGE_TYPES, scene=None,
                 max_depth=MAX_DEPTH, workspace=WORKSPACE, max_num_points=128):
        if sim.task != HM.TASK_UR5SIH:
            raise NotImplementedError("camera sensors are built for the Ur5Sih scenes")
        for k in outputs:
            if k not in IMAGE_TYPES:
                raise NotImplementedError(f"camera image type {k!r}: this build renders {IMAGE_TYPES} "
                                          "(no colour: the collision geometry has no materials)")
        if not 0 < fovx < 180:
            raise ValueError(f"Horizontal field-of-view (fovx) should be in [0, 180], but found '{fovx}'.")
        self.sim = sim
        self.width, self.height = int(resolution[0]), int(resolution[1])
        self.fovx = float(fovx)
        self.pos, self.quat = list(pos), list(quat)
        N, H, W = sim.num_envs, self.height, self.width
        dev = sim.device
        scene = scene if scene is not None else sim.scene
        self.view = view_matrix(pos, quat)
        self.proj = projection_matrix(fovx, W, H)
        # camera.py:68 multiplies by view_mat.inverse(): the same fp32 inverse, computed once on the host
        self.view_inv = torch.linalg.inv(torch.from_numpy(self.view)).numpy().astype(np.float32)
        self.images = {}
        if "depth" in outputs or "pointcloud" in outputs:
            self.images["depth"] = torch.zeros((N, H, W), dtype=torch.float32, device=dev)
        target = "target_object_pointcloud" in outputs      # needs the segmentation and the point cloud
        if "segmentation" in outputs or target:
            self.images["segmentation"] = torch.zeros((N, H, W), dtype=torch.int32, device=dev)
        if "pointcloud" in outputs or target:
            self.images["pointcloud"] = torch.zeros((N, H, W, 4), dtype=torch.float32, device=dev)
        if target:
            self.images["target_object_pointcloud"] = torch.zeros((N, int(max_num_points), 4), dtype=torch.float32,
                                                                  device=dev)
        c = HM.HaCamera()
        c.pos[:] = [float(v) for v in pos]
        c.quat[:] = [float(v) for v in quat]
        c.fovx_deg = self.fovx
        c.width, c.height = W, H
        c.max_depth = float(max_depth)
        c.workspace[:] = [float(v) for v in workspace]
        c.goal_radius = float(scene.get("goal_radius", 0.02))
        seg = static_segmentation_ids(scene)
        for k, v in enumerate(seg):
            c.static_seg[k] = v
        c.depth = self.images["depth"].data_ptr() if "depth" in self.images else None
        c.segmentation = self.images["segmentation"].data_ptr() if "segmentation" in self.images else None
        c.pointcloud = self.images["pointcloud"].data_ptr() if "pointcloud" in self.images else None
        c.target_pc = self.images["target_object_pointcloud"].data_ptr() if target else None
        c.target_points = int(max_num_points)
        c.rng_counter = 0
        self.args = c
        self._vinv = (C.c_float * 16)(*self.view_inv.reshape(-1).tolist())

    @property
    def projection_matrix(self):
        """camera.py:313-320: diag(2 / P[0][0], 2 / P[1][1], 1)."""
        return torch.tensor([[2 / self.proj[0, 0], 0.0, 0.0], [0.0, 2 / self.proj[1, 1], 0.0], [0.0, 0.0, 1.0]])

    def render(self, from_depth=False):
        """render_all_camera_sensors + refresh of every image (one launch). from_depth: only recompute the point
        cloud from images["depth"] (HA_CAM_FROM_DEPTH)."""
        flags = HM.CAM_FROM_DEPTH if from_depth else 0
        self.args.rng_counter = (self.args.rng_counter + 1) & 0xFFFFFFFF     # a fresh random subset per refresh
        _lib.check(self.sim.lib.ha_render_camera(self.sim.h, C.byref(self.args), self._vinv, flags,
                                                 self.sim._stream()), "ha_render_camera")
