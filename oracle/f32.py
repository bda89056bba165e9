"""ORACLE (test infrastructure only) - float32 helpers that restate, operation for operation, device expressions
the task oracles need bit for bit: the shared sine / cosine of include/ha_fmath.h, the kernels' quaternion
rotation (csrc/ha_device.h qrot) and the device-mode counter hash (csrc/ha_task.h mix32 / uniform01).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.
Every operation is a numpy float32 (or uint32) array operation, so each one is rounded exactly like the
corresponding IEEE single-precision instruction without contraction (the kernels build with -ffp-contract=off).
"""
import numpy as np

F = np.float32
U = np.uint32


def sincos(x):
    """include/ha_fmath.h ha_sincosf: Cody-Waite reduction by pi/2 (three-part constant), Cephes minimax
    polynomials on [-pi/4, pi/4], quadrant select. Returns (sin x, cos x) as float32 arrays."""
    x = np.asarray(x, F)
    k = np.floor(x * F(0.636619772367581343) + F(0.5)).astype(F)
    r = ((x - k * F(1.5703125)) - k * F(4.83751296997070312e-4)) - k * F(7.54978995489188216e-8)
    z = r * r
    sp = ((F(-1.9515295891e-4) * z + F(8.3321608736e-3)) * z - F(1.6666654611e-1)) * z * r + r
    cp = ((F(2.443315711809948e-5) * z - F(1.388731625493765e-3)) * z + F(4.166664568298827e-2)) * z * z \
        - F(0.5) * z + F(1.0)
    kq = k - F(4.0) * np.floor(k * F(0.25)).astype(F)
    q = kq.astype(np.int32)
    odd = (q & 1) != 0
    s = np.where(odd, cp, sp).astype(F)
    c = np.where(odd, sp, cp).astype(F)
    c = np.where((q == 1) | (q == 2), -c, c).astype(F)
    s = np.where(q >= 2, -s, s).astype(F)
    return s, c


def cross(a, b):
    """ha_device.h cross3 (per component a.y b.z - a.z b.y ...)."""
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1).astype(F)


def qrot(q, v):
    """ha_device.h qrot: t = 2 (u x v), (v + t w) + u x t, with u = q.xyz (xyzw quaternions)."""
    q = np.asarray(q, F)
    v = np.asarray(v, F)
    u = q[..., 0:3]
    t = cross(u, v) * F(2.0)
    return ((v + t * q[..., 3:4]) + cross(u, t)).astype(F)


def mix32(x):
    """ha_task.h mix32 (uint32 arithmetic, wrapping)."""
    x = np.asarray(x, U)
    with np.errstate(over="ignore"):
        x = x ^ (x >> U(16))
        x = (x * U(0x7FEB352D)).astype(U)
        x = x ^ (x >> U(15))
        x = (x * U(0x846CA68B)).astype(U)
        x = x ^ (x >> U(16))
    return x.astype(U)


def uniform01(seed, env, episode, k):
    """ha_task.h uniform01: the device-mode counter hash -> [0, 1) on the 2^-24 grid (exact in float32)."""
    seed = int(seed)
    lo, hi = U(seed & 0xFFFFFFFF), U((seed >> 32) & 0xFFFFFFFF)
    env = np.asarray(env, U)
    episode = np.asarray(episode, U)
    with np.errstate(over="ignore"):
        inner = mix32((episode * U(0x85EBCA6B)).astype(U) + U(k) + hi)
        h = mix32(lo ^ mix32((env * U(0x9E3779B9)).astype(U) ^ inner))
    return ((h >> U(8)).astype(F) * F(1.0 / 16777216.0)).astype(F)


def gauss01(seed, env, ctr, k):
    """ha_task.h gauss01 (Box-Muller from two hashed uniforms). The kernel's logf / cosf / sqrtf are the device
    library's, so this agrees to about one ulp, not bit for bit: tests compare its products within a tolerance."""
    s2 = (int(seed) ^ 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    u1 = uniform01(s2, env, ctr, 2 * k)
    u2 = uniform01(s2, env, ctr, 2 * k + 1)
    u1 = np.maximum(u1, F(1.0 / 16777216.0))
    return (np.sqrt(F(-2.0) * np.log(u1)) * np.cos(F(6.28318530717958647692) * u2)).astype(F)
