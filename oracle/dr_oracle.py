"""ORACLE (test infrastructure only) - the schema-driven domain randomization of csrc/ha_dr.h restated in numpy /
Python, operation for operation, so tests compare the device's dr_scale rows, dr_global state, noisy actions and
noisy observations with it bit for bit.

It follows the reference's engine: tasks/base/vec_task.py:646-876 (apply_randomizations: frequency gate,
first_randomization, last_rand_step, the observation / action noise lambdas with their correlated term, sim_params
gravity, actor properties) and utils/dr_utils.py:71-208 (generate_random_samples' schedules and distributions,
get_bucketed_val, apply_random_samples). The draws are the device counter hash (f32.uniform01, dr_gauss), not numpy's
global generator.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module.
"""
import numpy as np

from handarm_hip import model as HM
from oracle import f32

F = np.float32
M64 = (1 << 64) - 1
SALT_ENV = 0x5D0E6A3C11B2C4E7
SALT_GRAV = 0x3C6EF372FE94F82B
SALT_OBS_W = 0xA54FF53A5F1D36F1
SALT_OBS_C = 0x510E527FADE682D1
SALT_ACT_W = 0x9B05688C2B3E6C1F
SALT_ACT_C = 0x1F83D9ABFB41BD6B
DIST_OFF, DIST_UNIFORM, DIST_LOGUNIFORM, DIST_GAUSSIAN = 0, 1, 2, 3
OP_ADDITIVE, OP_SCALING = 0, 1
SCHED_NONE, SCHED_LINEAR, SCHED_CONSTANT = 0, 1, 2


def salted(seed, salt):
    return (int(seed) ^ salt) & M64


def gauss(seed, env, ctr, k):
    """ha_dr.h dr_gauss: Box-Muller with the shared ha_logf / ha_sincosf (f32.logf / f32.sincos)."""
    k = np.asarray(k, np.uint32)
    u1 = np.maximum(f32.uniform01(seed, env, ctr, np.uint32(2) * k), F(1.0 / 16777216.0))
    u2 = f32.uniform01(seed, env, ctr, np.uint32(2) * k + np.uint32(1))
    _, c = f32.sincos(F(6.28318530717958647692) * u2)
    return (np.sqrt(F(-2.0) * f32.logf(u1)) * c).astype(F)


def sched(a, frame):
    """dr_sched (dr_utils.py:82-87): python double."""
    if a.sched == SCHED_LINEAR:
        return 1.0 / a.sched_steps * min(frame, a.sched_steps)
    if a.sched == SCHED_CONSTANT:
        return 0.0 if frame < a.sched_steps else 1.0
    return 1.0


def scheduled_range(a, frame):
    """dr_range (dr_utils.py:98-130): (mu, var) for gaussian, else (lo, hi), in python double."""
    s = sched(a, frame)
    lo, hi = float(a.range[0]), float(a.range[1])
    if a.dist == DIST_GAUSSIAN:
        if a.op == OP_ADDITIVE:
            lo *= s
            hi *= s
        else:
            hi = hi * s
            lo = lo * s + 1.0 * (1.0 - s)
    else:
        if a.op == OP_ADDITIVE:
            lo *= s
            hi *= s
        else:
            lo = lo * s + 1.0 * (1.0 - s)
            hi = hi * s + 1.0 * (1.0 - s)
    return lo, hi


def bucket(v, a):
    """dr_bucket (get_bucketed_val, dr_utils.py:135-145), in double: below the grid takes the last bucket
    (bisect - 1 = -1)."""
    v = np.asarray(v, np.float64)
    if a.dist == DIST_UNIFORM:
        lo, hi = float(a.range[0]), float(a.range[1])
    else:
        sd = np.sqrt(float(a.range[1]))
        lo, hi = float(a.range[0]) - 2.0 * sd, float(a.range[0]) + 2.0 * sd
    nb = int(a.num_buckets)
    w = hi - lo
    with np.errstate(invalid="ignore"):
        t = np.floor((v - lo) / w * float(nb))
    i = np.where(~(t >= 0), nb - 1, np.where(t > nb - 1, nb - 1, np.nan_to_num(t, nan=0).astype(np.int64)))
    return w * i.astype(np.float64) / float(nb) + lo


def value(a, r0, r1, og, u, g):
    """dr_value: one sample applied to the nominal value og, in double (the draw u / g float32), rounded to float32;
    loguniform through the shared float32 log / exp."""
    og = np.asarray(og, F).astype(np.float64)
    if a.dist == DIST_GAUSSIAN:
        smp = r0 + r1 * np.asarray(g, F).astype(np.float64)
    elif a.dist == DIST_LOGUNIFORM:
        l0, l1 = f32.logf(np.array([r0], F))[0], f32.logf(np.array([r1], F))[0]
        smp = f32.expf(l0 + (l1 - l0) * np.asarray(u, F)).astype(np.float64)
    else:
        smp = r0 + (r1 - r0) * np.asarray(u, F).astype(np.float64)
    v = og * smp if a.op == OP_SCALING else og + smp
    if a.num_buckets > 0:
        v = bucket(v, a)
    return np.asarray(v).astype(F)


def attr_sample(p, attr, env, ep, k, frame, og):
    """dr_attr_sample for arrays of (env, episode, element k)."""
    a = p.dr_attr[attr]
    r0, r1 = scheduled_range(a, frame)
    key = np.uint32(64 * attr) + np.asarray(k, np.uint32)
    seed = salted(p.seed, SALT_ENV)
    if a.dist == DIST_GAUSSIAN:
        return value(a, r0, r1, og, 0, gauss(seed, env, ep, key))
    return value(a, r0, r1, og, f32.uniform01(seed, env, ep, key), 0)


def mass_ratio(p, attr, env, ep, k, frame, og, own=None):
    """dr_mass_ratio: og the value the sample multiplies, own the body's nominal mass (default og)."""
    a = p.dr_attr[attr]
    og = np.asarray(og, F)
    own = og if own is None else np.asarray(own, F)
    with np.errstate(invalid="ignore", divide="ignore"):     # massless bodies (own 0): og == own, `simple` is taken
        general = (attr_sample(p, attr, env, ep, k, frame, og) / own).astype(F)
    if not (a.op == OP_SCALING and a.num_buckets == 0):
        return general
    simple = attr_sample(p, attr, env, ep, k, frame, F(1.0))        # elementwise where og == own (the device's test)
    same = np.broadcast_to(og == own, general.shape)
    return np.where(same, np.broadcast_to(simple, general.shape), general).astype(F)


def active(p, attr, all_):
    a = p.dr_attr[attr]
    return a.dist != DIST_OFF and (all_ or not a.setup_only)


def elems(p, attr, all_, n):
    """dr_elem: the elements of a robot list property re-sampled in this randomization."""
    a = p.dr_attr[attr]
    if not active(p, attr, all_):
        return 0
    return n if (all_ or a.later_elems < 0) else min(n, a.later_elems)


def env_pre(p, model, rows, rb, episode, pools, reset, g, step):
    """dr_env_pre over every env (numpy, in place): the gate, the samples into `rows` (N, DR_SIZE), randomize_buf `rb`.
    pools: (N, n_obj) pool ids; reset: (N,) bool of the envs being reset; g: dr_global (as the step launch reads it).
    Returns the bool mask of the envs that sampled (their persistent-manifold records are cleared on a rescale)."""
    gi = g.view(np.int32)
    all_ = gi[HM.DRG_ALL] != 0
    frame = int(gi[HM.DRG_FRAME])
    N = rows.shape[0]
    smp = np.ones(N, bool) if all_ else (np.asarray(reset, bool) & (rb >= p.dr_frequency))
    if not all_:
        rb[smp] = 0
    if step:
        rb += 1
    envs = np.nonzero(smp)[0].astype(np.uint32)
    if len(envs) == 0:
        return smp
    ep = np.asarray(episode, np.uint32)[envs]
    E, EP = envs[:, None], ep[:, None]
    L, D, NO = model.n_links, model.n_dofs, pools.shape[1]
    li, di, oi = np.arange(L, dtype=np.uint32)[None], np.arange(D, dtype=np.uint32)[None], np.arange(NO, dtype=np.uint32)[None]
    n = elems(p, HM.DRA_LINK_MASS, all_, L)
    if n:
        own = np.array(list(model.link_mass)[:n], F)[None]
        og = own
        if not all_ and p.dr_attr[HM.DRA_LINK_MASS].later_og_object:
            og = np.array(list(model.pool_mass), F)[pools[envs, 0]][:, None]
        rows[envs, HM.DR_LINK_MASS:HM.DR_LINK_MASS + n] = mass_ratio(p, HM.DRA_LINK_MASS, E, EP, li[:, :n], frame, og, own)
    n = elems(p, HM.DRA_LINK_FRIC, all_, L)
    if n:
        rows[envs, HM.DR_LINK_FRIC:HM.DR_LINK_FRIC + n] = attr_sample(p, HM.DRA_LINK_FRIC, E, EP, li[:, :n], frame,
                                                                       F(p.friction))
    for attr, slot, name in ((HM.DRA_DOF_KD, HM.DR_DOF_KD, "dof_kd"), (HM.DRA_DOF_KP, HM.DR_DOF_KP, "dof_kp"),
                             (HM.DRA_DOF_LOWER, HM.DR_DOF_LOWER, "dof_lower"),
                             (HM.DRA_DOF_UPPER, HM.DR_DOF_UPPER, "dof_upper")):
        if active(p, attr, all_):
            og = np.array(list(getattr(model, name))[:D], F)[None]
            rows[envs, slot:slot + D] = attr_sample(p, attr, E, EP, di, frame, og)
    if active(p, HM.DRA_OBJ_MASS, all_):
        og = np.array(list(model.pool_mass), F)[pools[envs]]
        rows[envs, HM.DR_OBJ_MASS:HM.DR_OBJ_MASS + NO] = mass_ratio(p, HM.DRA_OBJ_MASS, E, EP, oi, frame, og)
    if active(p, HM.DRA_OBJ_FRIC, all_):
        rows[envs, HM.DR_OBJ_FRIC:HM.DR_OBJ_FRIC + NO] = attr_sample(p, HM.DRA_OBJ_FRIC, E, EP, oi, frame, F(p.friction))
    if active(p, HM.DRA_OBJ_SCALE, all_):
        rows[envs, HM.DR_OBJ_SCALE:HM.DR_OBJ_SCALE + NO] = attr_sample(p, HM.DRA_OBJ_SCALE, E, EP, oi, frame, F(1.0))
    return smp


def noise_params(a, frame):
    """dr_noise_params (vec_task.py:684-754): (corr scale, corr offset, white scale, white offset), double -> float."""
    s = sched(a, frame)
    r0, r1, c0, c1 = float(a.range[0]), float(a.range[1]), float(a.range_corr[0]), float(a.range_corr[1])
    if a.dist == DIST_GAUSSIAN:
        if a.op == OP_ADDITIVE:
            r0, r1, c0, c1 = r0 * s, r1 * s, c0 * s, c1 * s
        else:
            r1, r0 = r1 * s, r0 * s + 1.0 * (1.0 - s)
            c1, c0 = c1 * s, c0 * s + 1.0 * (1.0 - s)
        return np.array([c1, c0, r1, r0], F)
    if a.op == OP_ADDITIVE:
        r0, r1, c0, c1 = r0 * s, r1 * s, c0 * s, c1 * s
    else:
        r0, r1 = r0 * s + 1.0 * (1.0 - s), r1 * s + 1.0 * (1.0 - s)
        c0, c1 = c0 * s + 1.0 * (1.0 - s), c1 * s + 1.0 * (1.0 - s)
    return np.array([c1 - c0, c0, r1 - r0, r0], F)


def global_update(p, g, any_reset, mode):
    """dr_global_update on the float32 array g (HA_DRG_SIZE, int fields as int32 bits), in place."""
    gi = g.view(np.int32)
    if mode == 0:
        g[HM.DRG_ACT_USE:HM.DRG_ACT_USE + 4] = g[HM.DRG_ACT:HM.DRG_ACT + 4]
        gi[HM.DRG_ACT_EPOCH] = gi[HM.DRG_EPOCH]
        gi[HM.DRG_ACT_ON] = 1 if (gi[HM.DRG_VALID] and p.dr_attr[HM.DRA_ACT].dist != DIST_OFF) else 0
        gi[HM.DRG_STEP] += 1
    frame = int(gi[HM.DRG_FRAME_NEXT])
    gi[HM.DRG_FRAME] = frame
    nonenv = all_ = 0
    if any_reset:
        if gi[HM.DRG_FIRST]:
            nonenv = all_ = 1
        else:
            nonenv = 1 if frame - int(gi[HM.DRG_LAST_RAND]) >= p.dr_frequency else 0
        gi[HM.DRG_FIRST] = 0
    gi[HM.DRG_ALL] = all_
    if nonenv:
        gi[HM.DRG_LAST_RAND] = frame
        gi[HM.DRG_EPOCH] += 1
        epoch = int(gi[HM.DRG_EPOCH])
        gi[HM.DRG_VALID] = 1
        g[HM.DRG_OBS:HM.DRG_OBS + 4] = noise_params(p.dr_attr[HM.DRA_OBS], frame)
        g[HM.DRG_ACT:HM.DRG_ACT + 4] = noise_params(p.dr_attr[HM.DRA_ACT], frame)
        a = p.dr_attr[HM.DRA_GRAVITY]
        if a.dist != DIST_OFF:
            r0, r1 = scheduled_range(a, frame)
            seed = salted(p.seed, SALT_GRAV)
            k = np.arange(3, dtype=np.uint32)
            gg = gauss(seed, np.uint32(0), np.uint32(epoch), k) if a.dist == DIST_GAUSSIAN else np.zeros(3, F)
            u = f32.uniform01(seed, np.uint32(0), np.uint32(epoch), k) if a.dist != DIST_GAUSSIAN else np.zeros(3, F)
            og = np.array(list(p.gravity), F) if all_ else g[HM.DRG_GRAVITY_OG:HM.DRG_GRAVITY_OG + 3].copy()
            g[HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3] = value(a, r0, r1, og, u, gg)
            if all_:
                g[HM.DRG_GRAVITY_OG:HM.DRG_GRAVITY_OG + 3] = g[HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3]
    frames = p.control_freq_inv if mode == 0 else 0
    if p.task == HM.TASK_UR5SIH and any_reset:
        frames += 1
    gi[HM.DRG_FRAME_NEXT] = frame + frames
    return g


def _noise(a, P, sw, sc, env, step, epoch, k, x):
    corr = gauss(sc, env, np.uint32(epoch), k)
    white = gauss(sw, env, np.uint32(step), k) if a.dist == DIST_GAUSSIAN else f32.uniform01(sw, env, np.uint32(step), k)
    n = ((corr * P[0] + P[1]) + white * P[2]) + P[3]
    x = np.asarray(x, F)
    return (x * n if a.op == OP_SCALING else x + n).astype(F)


def obs_noise(p, g, x):
    """dr_obs on a (N, O) float32 observation block (obs_buf after post_physics_step)."""
    gi = g.view(np.int32)
    a = p.dr_attr[HM.DRA_OBS]
    if not gi[HM.DRG_VALID] or a.dist == DIST_OFF:
        return np.asarray(x, F)
    N, O = x.shape
    env = np.arange(N, dtype=np.uint32)[:, None]
    k = np.arange(O, dtype=np.uint32)[None, :]
    return _noise(a, g[HM.DRG_OBS:HM.DRG_OBS + 4], salted(p.seed, SALT_OBS_W), salted(p.seed, SALT_OBS_C), env,
                  int(gi[HM.DRG_STEP]), int(gi[HM.DRG_EPOCH]), k, x)


def act_noise(p, g, a_raw):
    """act_at's noise on a (N, A) float32 raw-action block (before the clamp)."""
    gi = g.view(np.int32)
    if not gi[HM.DRG_ACT_ON]:
        return np.asarray(a_raw, F)
    N, A = a_raw.shape
    env = np.arange(N, dtype=np.uint32)[:, None]
    k = np.arange(A, dtype=np.uint32)[None, :]
    return _noise(p.dr_attr[HM.DRA_ACT], g[HM.DRG_ACT_USE:HM.DRG_ACT_USE + 4], salted(p.seed, SALT_ACT_W),
                  salted(p.seed, SALT_ACT_C), env, int(gi[HM.DRG_STEP]), int(gi[HM.DRG_ACT_EPOCH]), k, a_raw)
