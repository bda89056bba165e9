"""Independent articulated-body dynamics in float64 numpy, straight from a scene JSON (test infrastructure).

Written from the textbook formulas, not from csrc/ha_physics.h or oracle/physics_oracle.c, so a defect the kernel and
the C oracle share (they share include/ha_fmath.h and one restatement of CRBA / RNEA / the drive rows) fails a test
that compares either of them with this module (verdict r05 Weak #2 / Next #7):

* forward kinematics with rotation matrices: each link's frame = parent frame x joint origin (xyzw quaternion) x
  rotation about the joint axis by q (URDF revolute semantics);
* joint-space inertia M(q) = sum_i m_i Jv_i^T Jv_i + Jw_i^T (R_i I_i R_i^T) Jw_i + diag(armature), with the COM
  Jacobians Jv_i (columns a_d x (c_i - o_d)) and Jw_i (columns a_d) over link i's ancestor DOFs;
* link damping (PhysX linear / angular damping as a wrench on the COM twist): D(q) = sum_i cl m_i Jv_i^T Jv_i +
  ca Jw_i^T I_i,w Jw_i;
* Coriolis / centrifugal forces from M by central differences: C qd = Mdot qd - 1/2 d/dq (qd^T M qd);
* the implicit PD step the drive rows solve (PhysX articulation drive): with every joint's
  soft row gamma = 1 / (h (kd + h kp)) converged, (M + h (kd + h kp)) qd' = M qd_free - h kp (q - q*), with
  qd_free = qd - h M^-1 (C qd + D qd), then q' = q + h qd'.
"""
import json

import numpy as np


def quat_matrix(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def quat_mul(a, b):
    """Hamilton product of xyzw quaternions."""
    x1, y1, z1, w1 = a
    x2, y2, z2, w2 = b
    return np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])


def axis_angle(a, t):
    a = np.asarray(a, np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * (K @ K)


class Chain:
    def __init__(self, scene):
        if isinstance(scene, str):
            with open(scene) as f:
                scene = json.load(f)
        rob = scene["robot"]
        self.links, self.dofs = rob["links"], rob["dofs"]
        self.L, self.D = len(self.links), len(self.dofs)
        self.base_p = np.asarray(rob["base_pos"], np.float64)
        self.base_quat = np.asarray(rob["base_quat"], np.float64)
        self.base_R = quat_matrix(self.base_quat)
        for i, l in enumerate(self.links):
            assert l["type"] in ("revolute", "fixed", "continuous"), l["type"]
            assert l["parent"] < i, "links must come after their parent"
        self.armature = np.array([d.get("armature", 0.0) for d in self.dofs])
        self.kp = np.array([d["kp"] for d in self.dofs])
        self.kd = np.array([d["kd"] for d in self.dofs])

    def fk(self, q):
        """World (R, p) of every link frame, and each DOF's world axis and anchor."""
        R, p = [None] * self.L, [None] * self.L
        ax, an = np.zeros((self.D, 3)), np.zeros((self.D, 3))
        for i, l in enumerate(self.links):
            if l["parent"] < 0:
                Rp, pp = self.base_R, self.base_p
            else:
                Rp, pp = R[l["parent"]], p[l["parent"]]
            p[i] = pp + Rp @ np.asarray(l["origin_pos"], np.float64)
            Ri = Rp @ quat_matrix(np.asarray(l["origin_quat"], np.float64))
            d = l["dof"]
            if d >= 0:
                Ri = Ri @ axis_angle(l["axis"], q[d])
                ax[d] = Ri @ (np.asarray(l["axis"], np.float64) / np.linalg.norm(l["axis"]))
                an[d] = p[i]
            R[i] = Ri
        return R, p, ax, an

    def ancestors(self, i):
        out = []
        while i >= 0:
            if self.links[i]["dof"] >= 0:
                out.append(self.links[i]["dof"])
            i = self.links[i]["parent"]
        return out

    def jacobians(self, q):
        """Per link: (mass, world inertia about the COM, Jv (3 x D) of the COM, Jw (3 x D)), and the frames."""
        R, p, ax, an = self.fk(q)
        out = []
        for i, l in enumerate(self.links):
            c = p[i] + R[i] @ np.asarray(l["com"], np.float64)
            Jv, Jw = np.zeros((3, self.D)), np.zeros((3, self.D))
            for d in self.ancestors(i):
                Jw[:, d] = ax[d]
                Jv[:, d] = np.cross(ax[d], c - an[d])
            I = np.asarray(l["inertia"], np.float64).reshape(3, 3)
            out.append((float(l["mass"]), R[i] @ I @ R[i].T, Jv, Jw))
        return out, (R, p)

    def mass_matrix(self, q):
        M = np.diag(self.armature.copy())
        for m, Iw, Jv, Jw in self.jacobians(q)[0]:
            M += m * Jv.T @ Jv + Jw.T @ Iw @ Jw
        return M

    def damping_matrix(self, q, cl, ca):
        Dm = np.zeros((self.D, self.D))
        for m, Iw, Jv, Jw in self.jacobians(q)[0]:
            Dm += cl * m * Jv.T @ Jv + ca * Jw.T @ Iw @ Jw
        return Dm

    def coriolis(self, q, qd, eps=1e-6):
        q, qd = np.asarray(q, np.float64), np.asarray(qd, np.float64)
        Mdot = (self.mass_matrix(q + eps * qd) - self.mass_matrix(q - eps * qd)) / (2 * eps)
        grad = np.zeros(self.D)
        for k in range(self.D):
            e = np.zeros(self.D)
            e[k] = eps
            grad[k] = qd @ ((self.mass_matrix(q + e) - self.mass_matrix(q - e)) / (2 * eps)) @ qd
        return Mdot @ qd - 0.5 * grad

    def body_states(self, q, qd):
        """(L, 13) rigid-body rows of the links: origin position, orientation (xyzw, composed as parent x joint origin
        x axis rotation, the quaternion product order Isaac Gym's rows carry), COM linear velocity Jv qd, angular
        velocity Jw qd."""
        q, qd = np.asarray(q, np.float64), np.asarray(qd, np.float64)
        (bodies, (R, p)) = self.jacobians(q)
        quats = [None] * self.L
        for i, l in enumerate(self.links):
            base = np.asarray(self.base_quat, np.float64) if l["parent"] < 0 else quats[l["parent"]]
            qi = quat_mul(base, np.asarray(l["origin_quat"], np.float64))
            if l["dof"] >= 0:
                a = np.asarray(l["axis"], np.float64)
                a = a / np.linalg.norm(a)
                t = q[l["dof"]] / 2
                qi = quat_mul(qi, np.array([a[0] * np.sin(t), a[1] * np.sin(t), a[2] * np.sin(t), np.cos(t)]))
            quats[i] = qi
            assert np.allclose(quat_matrix(qi / np.linalg.norm(qi)), R[i], atol=1e-9)
        out = np.zeros((self.L, 13))
        for i, (m, Iw, Jv, Jw) in enumerate(bodies):
            out[i, 0:3] = p[i]
            out[i, 3:7] = quats[i]
            out[i, 7:10] = Jv @ qd
            out[i, 10:13] = Jw @ qd
        return out

    def implicit_pd_step(self, q, qd, target, h, cl=0.0, ca=0.0, kp=None, kd=None):
        """One substep of the converged drive rows (no contacts, no active limits, efforts not saturated).
        Returns (q', qd')."""
        q, qd, target = (np.asarray(x, np.float64) for x in (q, qd, target))
        kp = self.kp if kp is None else np.asarray(kp, np.float64)
        kd = self.kd if kd is None else np.asarray(kd, np.float64)
        M = self.mass_matrix(q)
        cb = self.coriolis(q, qd) + self.damping_matrix(q, cl, ca) @ qd
        v_free = qd - h * np.linalg.solve(M, cb)
        A = M + h * np.diag(kd + h * kp)
        v = np.linalg.solve(A, M @ v_free - h * kp * (q - target))
        return q + h * v, v
