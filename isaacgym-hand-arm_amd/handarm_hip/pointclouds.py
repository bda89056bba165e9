"""Synthetic point-cloud observables of Ur5SihMultiObject on the device.

Host side of ``ha_pointclouds`` (include/handarm_abi.h): the surface samples the reference draws at post_init
(``_acquire_object_synthetic_pointcloud`` multi_object.py:774-790, ``_acquire_ur5sih_synthetic_pointcloud``
ur5sih.py:347-359) come from the committed asset ``assets/ur5sih_pointclouds.npz`` (tools/build_model.py
--pointclouds: trimesh's area-weighted surface sampling restated, since trimesh is absent; the samples are
random draws, so their values are "parity unpinned" while the pose/permute/pad arithmetic on them is pinned by
tests/golden/ur5sih_pointclouds_*.npz). Every refresh is ONE kernel launch for all clouds and envs; the
per-step ``torch.randperm(max_num_points)`` (multi_object.py:800) is drawn on the device from the task's
generator.
"""
import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from . import model as HM
from .observables import POINTCLOUDS

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "ur5sih_pointclouds.npz")
TIP_LINKS = [28, 15, 21, 24, 18]     # thumb, index, middle, ring, little fingertip links (ur5sih.py:609-614)
FLANGE_LINK = 9


def object_sample_table(pool_names, average_num_points=100, max_num_points=128, sample_mode="area", asset=None):
    """(n_pool, max_num_points, 4) pool-frame samples with w = 1 for the first num_i points, 0 padding
    (multi_object.py:774-786): 'uniform' -> average_num_points each; 'area' -> int(average * area / mean_area),
    the mean over the configured pool."""
    d = np.load(asset or ASSET)
    names = [str(n) for n in d["object_names"]]
    idx = [names.index(n) for n in pool_names]
    areas = d["object_areas"][idx]
    if sample_mode == "uniform":
        num = [average_num_points] * len(idx)
    elif sample_mode == "area":
        mean_area = sum(float(a) for a in areas) / len(areas)
        num = [int(average_num_points * float(a) / mean_area) for a in areas]
    else:
        raise ValueError(f"pointclouds.sample_mode {sample_mode!r}")
    if d["object_samples"].shape[1] < max_num_points:
        raise ValueError(f"the asset holds {d['object_samples'].shape[1]} samples per object < {max_num_points}")
    out = np.zeros((len(idx), max_num_points, 4), np.float32)
    for i, k in enumerate(idx):
        n = min(num[i], max_num_points)
        out[i, :n, 0:3] = d["object_samples"][k, :n]
        out[i, :n, 3] = 1.0
    return out


class SyntheticPointclouds:
    """Device buffers and one-launch refresh of the requested clouds. ``outputs[name]`` is the (N, points, 4)
    tensor that goes into ``obs_dict[name]`` (observable_vec_task.py:188-191)."""

    def __init__(self, sim, names, pool_names, cfg_pc=None, generator=None, asset=None):
        cfg_pc = cfg_pc or {}
        for n in names:
            if n not in POINTCLOUDS:
                raise NotImplementedError(f"point cloud {n!r}: this build produces {POINTCLOUDS}")
        self.sim = sim
        self.names = list(names)
        dev = sim.device
        N, NO = sim.num_envs, sim.n_obj
        m = sim.model
        self.P = int(cfg_pc.get("max_num_points", 128))
        table = object_sample_table(pool_names, int(cfg_pc.get("average_num_points", 100)), self.P,
                                    cfg_pc.get("sample_mode", "area"), asset)
        d = np.load(asset or ASSET)
        rs = np.zeros((len(d["robot_samples"]), 4), np.float32)
        rs[:, 0:3] = d["robot_samples"]
        rs[:, 3] = 1.0                                           # ur5sih.py:359
        body = d["robot_link"].astype(np.int32) + m.body_robot0
        # the rigid bodies a launch reads (robot sample links, fingertips, flange): staged per env in LDS
        tips = [m.body_robot0 + link for link in TIP_LINKS]
        links = sorted(set(body.tolist()) | set(tips) | {m.body_robot0 + FLANGE_LINK})
        assert len(links) <= HM.PC_MAX_LINKS and max(links) < m.n_bodies and min(links) >= 0
        slot = np.array([links.index(b) for b in body], np.int32)
        self.R = len(rs)
        self.robot_body = body
        self.object_samples = torch.from_numpy(table).to(dev)
        self.robot_samples = torch.from_numpy(rs).to(dev)
        self.robot_slot = torch.from_numpy(slot).to(dev)
        self.gen = generator
        self.reference_rng = False      # True: torch.randperm on the CPU global generator (ref_rng.py)
        self.perm = torch.arange(self.P, dtype=torch.int64, device=dev)
        self.prev_pose = None                      # snapshot buffer when the object clouds see the previous pose
        shapes = {"object_synthetic_pointcloud": (N, NO * self.P, 4), "target_object_synthetic_pointcloud": (N, self.P, 4),
                  "ur5sih_synthetic_pointcloud": (N, self.R, 4), "sih_fingertip_pointcloud": (N, 5, 4),
                  "goal_synthetic_pointcloud": (N, 1, 4), "relative_goal_synthetic_pointcloud": (N, 1, 4)}
        self.outputs = {n: torch.zeros(shapes[n], dtype=torch.float32, device=dev) for n in self.names}
        if "ur5sih_synthetic_pointcloud" in self.outputs:
            self.outputs["ur5sih_synthetic_pointcloud"][..., 3] = 1.0           # post_init (ur5sih.py:358-359)
        # the reference keeps object_synthetic_pointcloud when only the target cloud is listed (it requires it)
        self._object_buf = self.outputs.get("object_synthetic_pointcloud")
        if "target_object_synthetic_pointcloud" in self.outputs and self._object_buf is None:
            self._object_buf = torch.zeros(shapes["object_synthetic_pointcloud"], dtype=torch.float32, device=dev)
        s = HM.HaPointcloud()
        s.object_samples = self.object_samples.data_ptr()
        s.robot_samples = self.robot_samples.data_ptr()
        s.robot_slot = self.robot_slot.data_ptr()
        s.perm = self.perm.data_ptr()
        s.object_pose = None
        s.object_pc = self._object_buf.data_ptr() if self._object_buf is not None else None
        s.target_pc = self._ptr("target_object_synthetic_pointcloud")
        s.robot_pc = self._ptr("ur5sih_synthetic_pointcloud")
        s.fingertip_pc = self._ptr("sih_fingertip_pointcloud")
        s.goal_pc = self._ptr("goal_synthetic_pointcloud")
        s.relative_goal_pc = self._ptr("relative_goal_synthetic_pointcloud")
        s.n_pool, s.P, s.R = len(table), self.P, self.R
        s.n_links = len(links)
        for k, b in enumerate(links):
            s.links[k] = b
        for f, b in enumerate(tips):
            s.fingertip_slot[f] = links.index(b)
        s.flange_slot = links.index(m.body_robot0 + FLANGE_LINK)
        self.args = s

    def _ptr(self, name):
        return self.outputs[name].data_ptr() if name in self.outputs else None

    def use_previous_object_pose(self):
        """Object clouds pose their samples with the previous refresh's object pose (post-step order puts them
        before object_pos): the caller snapshots it with ``snapshot_object_pose`` before the step."""
        self.prev_pose = torch.zeros((self.sim.num_envs, self.sim.n_obj, 7), dtype=torch.float32,
                                     device=self.sim.device)
        self.args.object_pose = self.prev_pose.data_ptr()

    def snapshot_object_pose(self, pose):
        if self.prev_pose is not None:
            self.prev_pose.copy_(pose)

    def refresh(self, perm=None):
        """One launch: every requested cloud of every env. perm: explicit (P,) permutation (tests); default a
        fresh torch.randperm on the device."""
        if perm is not None:
            p = torch.as_tensor(np.asarray(perm), dtype=torch.int64).to(self.sim.device)
            if p.shape != (self.P,) or not torch.equal(torch.sort(p).values, self.perm.new_tensor(range(self.P))):
                raise ValueError("perm must be a permutation of range(max_num_points)")
            self.perm.copy_(p)
        elif self._object_buf is not None:
            if self.reference_rng:      # multi_object.py:806: torch.randperm without a device is a CPU draw
                self.perm.copy_(torch.randperm(self.P))
            else:
                self.perm.copy_(torch.randperm(self.P, generator=self.gen, device=self.sim.device))
        _lib.check(self.sim.lib.ha_pointclouds(self.sim.h, C.byref(self.args), self.sim._stream()), "ha_pointclouds")

    def kernel_times_ms(self, max_n=1 << 16):
        buf = (C.c_float * max_n)()
        n = C.c_int32()
        _lib.check(self.sim.lib.ha_pointcloud_times(self.sim.h, buf, max_n, C.byref(n)), "ha_pointcloud_times")
        return list(buf[:n.value])
