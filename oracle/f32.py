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


def logf(x):
    """include/ha_fmath.h ha_logf (Cephes logf, exponent split by bits) for positive normal float32 arrays."""
    x = np.asarray(x, F)
    ix = x.view(np.int32)
    e = ((ix >> 23) & 0xFF) - 126
    m = ((ix & 0x007FFFFF) | 0x3F000000).astype(np.int32).view(F)
    low = m < F(0.707106781186547524)
    e = np.where(low, e - 1, e)
    m = np.where(low, (m + m) - F(1.0), m - F(1.0)).astype(F)
    z = m * m
    y = F(7.0376836292e-2) * m - F(1.1514610310e-1)
    for c in (1.1676998740e-1, -1.2420140846e-1, 1.4249322787e-1, -1.6668057665e-1, 2.0000714765e-1,
              -2.4999993993e-1, 3.3333331174e-1):
        y = y * m + F(c)
    y = (y * m) * z
    fe = e.astype(F)
    y = y + F(-2.12194440e-4) * fe
    y = y + F(-0.5) * z
    r = m + y
    return (r + F(0.693359375) * fe).astype(F)


def expf(x):
    """include/ha_fmath.h ha_expf (Cephes expf, two-part ln 2, result exponent by bits)."""
    x = np.clip(np.asarray(x, F), F(-87.0), F(88.0)).astype(F)
    z = np.floor(F(1.44269504088896341) * x + F(0.5)).astype(F)
    x = x - z * F(0.693359375)
    x = x - z * F(-2.12194440e-4)
    n = z.astype(np.int32)
    xx = x * x
    y = F(1.9875691500e-4) * x + F(1.3981999507e-3)
    for c in (8.3334519073e-3, 4.1665795894e-2, 1.6666665459e-1, 5.0000001201e-1):
        y = y * x + F(c)
    y = (y * xx + x) + F(1.0)
    return (y * ((n + 127) << 23).astype(np.int32).view(F)).astype(F)


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
