"""ORACLE (test infrastructure only) - numpy restatement of the camera sensor path (csrc/ha_camera.h).

Only ``tests/`` may import this module, as the checker. It restates, in float32 and in the kernel's operation
order:
  * the ray cast of depth / segmentation against the collision geometry (the build's stand-in for Isaac Gym's
    closed renderer: parity against that renderer is unpinned);
  * ``depth_image_to_global_points`` + ``_compute_pointcloud`` (hand_arm/utils/camera.py:50-69, 302-311), whose
    reference arithmetic is pinned by tests/golden/camera_pointcloud.npz (made by running the reference code).
"""
import math

import numpy as np

F = np.float32


def qrot(q, v):
    """Rotate v (..., 3) by unit quaternion q (4,) xyzw: v + w t + u x t, t = 2 u x v (ha_device.h qrot)."""
    u = np.asarray(q[:3], F)
    w = F(q[3])
    t = np.cross(np.broadcast_to(u, v.shape), v).astype(F) * F(2)
    return (v + t * w) + np.cross(np.broadcast_to(u, t.shape), t).astype(F)


def camera_axes(quat):
    """View axes in the env frame as the C launch computes them (columns x right, y up, z back)."""
    q = np.asarray(quat, F)
    n = F(math.sqrt(float(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])))
    x, y, z, w = q / n
    Rc = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], F)
    return np.stack([-Rc[:, 1], Rc[:, 2], -Rc[:, 0]], 1).astype(F)


def rays(width, height, fovx_deg, quat):
    """(H*W, 3) world ray directions through the integer pixel positions (x, y, -1 in view space)."""
    tanx = F(math.tan(0.5 * fovx_deg * math.pi / 180.0))
    tany = F(tanx * F(height) / F(width))
    row, col = np.divmod(np.arange(width * height), width)
    xv = ((col.astype(F) - F(0.5) * F(width)) / F(width)) * (F(2) * tanx)
    yv = -(((row.astype(F) - F(0.5) * F(height)) / F(height))) * (F(2) * tany)
    R = camera_axes(quat)
    return np.stack([R[r, 0] * xv + R[r, 1] * yv - R[r, 2] for r in range(3)], -1).astype(F)


def hulls_of_env(m, root, body, object_indices, a0, body_robot0, static_seg):
    """[(origin, quat, hull, seg)] in the kernel's order: link hulls (robot, seg 1), objects (3 + i), statics."""
    out = []
    for k in range(m.n_link_hulls):
        r = body[body_robot0 + m.hull_link[k]]
        out.append((r[0:3], r[3:7], k, 1))
    for o, pid in enumerate(object_indices):
        r = root[a0 + o]
        for j in range(m.pool_nhull[int(pid)]):            # every convex piece of the object (ha_model_t v8)
            out.append((r[0:3], r[3:7], m.pool_hull[int(pid)] + j, 3 + o))
    for s in range(m.n_static):
        out.append((np.array(m.static_pos[s][:], F), np.array(m.static_quat[s][:], F), m.static_hull[s],
                    static_seg[s]))
    return out


def render_depth_segmentation(m, cam, root, body, object_indices, goal_pos, a0, body_robot0, n_obj):
    """Depth (H, W) and segmentation (H, W) of one env (see csrc/ha_camera.h)."""
    W, H = cam["width"], cam["height"]
    d = rays(W, H, cam["fovx"], cam["quat"])
    o = np.asarray(cam["pos"], F)
    dd = (d * d).sum(-1, dtype=F)
    inv_len = F(1) / np.sqrt(dd)
    best = np.full(W * H, F(3.0e38), F)
    seg = np.zeros(W * H, np.int32)
    ground = d[:, 2] < 0
    tg = np.where(ground, -o[2] / np.where(ground, d[:, 2], F(-1)), F(-1)).astype(F)
    hitg = ground & (tg > 0)
    best = np.where(hitg, tg, best)
    oc = o - np.asarray(goal_pos, F)
    b = (oc * d).sum(-1, dtype=F)
    c = F((oc * oc).sum(dtype=F) - F(cam["goal_radius"]) * F(cam["goal_radius"]))
    disc = b * b - dd * c
    tgoal = ((-b - np.sqrt(np.maximum(disc, 0))) / dd).astype(F)
    hit = (disc >= 0) & (tgoal > 0) & (tgoal < best)
    best = np.where(hit, tgoal, best)
    seg = np.where(hit, 3 + n_obj, seg)
    planes = np.array(m.planes, F)
    for p, q, hull, sg in hulls_of_env(m, root, body, object_indices, a0, body_robot0, cam["static_seg"]):
        p = np.asarray(p, F)
        q = np.asarray(q, F)
        cw = p + qrot(q, np.array(m.hull_center[hull][:], F))
        r = F(m.hull_radius[hull])
        occ = cw - o
        tc = ((occ * d).sum(-1, dtype=F) / dd).astype(F)
        off = occ - d * tc[:, None]
        cand = ((off * off).sum(-1, dtype=F) <= r * r) & ~(tc - F(1.001) * r * inv_len > best)
        idx = np.nonzero(cand)[0]
        if len(idx) == 0:
            continue
        qi = np.array([-q[0], -q[1], -q[2], q[3]], F)
        ol = qrot(qi, np.broadcast_to(o - p, (len(idx), 3)).astype(F))
        dl = qrot(qi, d[idx])
        t0 = np.zeros(len(idx), F)
        t1 = best[idx].copy()
        ok = np.ones(len(idx), bool)
        ps, npl = m.hull_plane_start[hull], m.hull_nplanes[hull]
        for i in range(npl):
            n = planes[ps + i, 0:3]
            num = -((ol * n).sum(-1, dtype=F) + planes[ps + i, 3])
            den = (dl * n).sum(-1, dtype=F)
            with np.errstate(divide="ignore", invalid="ignore"):
                t = (num / den).astype(F)
            t0 = np.where(den < 0, np.maximum(t0, t), t0)
            t1 = np.where(den > 0, np.minimum(t1, t), t1)
            ok &= ~((den == 0) & (num < 0))
            ok &= ~(t0 > t1)
        take = ok & (t0 > 0) & (t0 < best[idx])
        best[idx] = np.where(take, t0, best[idx])
        seg[idx] = np.where(take, sg, seg[idx])
    anyhit = best < F(3.0e38)
    depth = np.where(anyhit, -best, F(-np.inf)).astype(F)
    seg = np.where(anyhit, seg, 0)
    return depth.reshape(H, W), seg.reshape(H, W).astype(np.int32)


def pointcloud_from_depth(depth, fu, fv, view_inv, max_depth=10.0, workspace=(-0.07, 0.63, 0.33, 0.83)):
    """_compute_pointcloud (camera.py:302-311) over depth_image_to_global_points (:50-69), kernel op order.
    depth (N, H, W) -> (N, H, W, 4) xyz + validity."""
    depth = np.asarray(depth, F)
    N, H, W = depth.shape
    dep = np.maximum(depth, F(-max_depth))
    row, col = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    x0 = -((col.astype(F) - F(0.5) * F(W)) / F(W))
    y0 = (row.astype(F) - F(0.5) * F(H)) / F(H)
    x0 = x0 * dep
    y0 = y0 * dep
    h0, h1, h2 = x0 * F(fu), y0 * F(fv), dep
    Vi = np.asarray(view_inv, F).reshape(4, 4)
    xyz = np.stack([((h0 * Vi[0, j] + h1 * Vi[1, j]) + h2 * Vi[2, j]) + Vi[3, j] for j in range(3)], -1)
    valid = ((depth > F(-max_depth)) & (xyz[..., 0] > F(workspace[0])) & (xyz[..., 0] < F(workspace[1]))
             & (xyz[..., 1] > F(workspace[2])) & (xyz[..., 1] < F(workspace[3])))
    return np.concatenate([xyz, valid[..., None].astype(F)], -1)


def target_pointcloud(pointcloud, segmentation, target_index, P):
    """{camera}_target_object_pointcloud (multi_object.py:837-855) where the target has <= P points: the target's
    points in pixel order, zero padding, w *= 2. pointcloud (N, H*W, 4), segmentation (N, H*W)."""
    N = pointcloud.shape[0]
    out = np.zeros((N, P, 4), F)
    for e in range(N):
        pts = pointcloud[e][segmentation[e] == 3 + int(target_index[e])]
        assert len(pts) <= P
        out[e, :len(pts)] = pts
    out[..., 3] *= F(2)
    return out
