// ha_dr.h - device RNG and schema-driven domain randomization (task.randomization_params) on the device.
//
// The reference's DR engine (tasks/base/vec_task.py:646-876 apply_randomizations, utils/dr_utils.py:71-238) runs on
// the host inside reset_idx (allegro_kuka_base.py:1248-1249): a Python loop over the reset envs calls the gym property
// getters / setters per actor, and two lambdas add noise to the actions and observations of every step. Here:
//   * the shard-wide part (frame count, first_randomization, last_rand_step, the non-env randomizations: noise
//     parameters under their schedules, gravity) is one 256-thread launch before each step / reset launch
//     (ha_dr_global_kernel): it ORs the reset flags (reset_idx runs apply_randomizations only when an env resets,
//     allegro_kuka_base.py:1367-1368) and updates ha_state_t.dr_global;
//   * the per-env part (vec_task.py:788-864: mass, friction, DOF stiffness / damping / limits, actor scale) is
//     sampled by the env's own wavefront inside the step launch, lane-parallel over links / DOFs / objects, into the
//     env's dr_scale row, which the physics reads in place of the nominal model values;
//   * the action / observation noise (vec_task.py:400-402,426-428) is applied where the step launch reads an action
//     and writes an observation, white and correlated terms from the counter hash (no noise tensors in HBM).
// Every sample is a function of (seed, env, counter, index) through uniform01 / dr_gauss, whose log / sine come from
// include/ha_fmath.h, so oracle/dr_oracle.py restates the rows, the global state and the noise bit for bit.
#pragma once
#include "ha_physics.h"

// ----------------------------------------------------------------------------- RNG (device mode)
HD uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
HD float uniform01(uint64_t seed, uint32_t env, uint32_t episode, uint32_t k) {
    uint32_t h = mix32((uint32_t)seed ^ mix32(env * 0x9E3779B9U ^ mix32(episode * 0x85EBCA6BU + k + (uint32_t)(seed >> 32))));
    return (h >> 8) * (1.0f / 16777216.0f);
}

// standard normal by Box-Muller from two counter-based uniforms
HD float gauss01(uint64_t seed, uint32_t env, uint32_t ctr, uint32_t k) {
    float u1 = uniform01(seed ^ 0x9E3779B97F4A7C15ULL, env, ctr, 2 * k);
    float u2 = uniform01(seed ^ 0x9E3779B97F4A7C15ULL, env, ctr, 2 * k + 1);
    u1 = fmaxf(u1, 1.0f / 16777216.0f);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
}

// Box-Muller with the shared log / cosine (include/ha_fmath.h): the DR samples are restated bit for bit by the oracle
HD float dr_gauss(uint64_t seed, uint32_t env, uint32_t ctr, uint32_t k) {
    float u1 = fmaxf(uniform01(seed, env, ctr, 2 * k), 1.0f / 16777216.0f);
    float u2 = uniform01(seed, env, ctr, 2 * k + 1);
    float s, c;
    ha_sincosf(6.28318530717958647692f * u2, &s, &c);
    return sqrtf(-2.0f * ha_logf(u1)) * c;
}

// counter-hash streams of the DR samples (xor-ed into ha_params_t.seed)
#define DR_SALT_ENV 0x5D0E6A3C11B2C4E7ULL     // per-env actor properties: (env, episode, 64 attr + index)
#define DR_SALT_GRAV 0x3C6EF372FE94F82BULL    // gravity: (0, epoch, k)
#define DR_SALT_OBS_W 0xA54FF53A5F1D36F1ULL   // observation noise, white: (env, step, k)
#define DR_SALT_OBS_C 0x510E527FADE682D1ULL   // observation noise, correlated: (env, epoch, k)
#define DR_SALT_ACT_W 0x9B05688C2B3E6C1FULL   // action noise, white
#define DR_SALT_ACT_C 0x1F83D9ABFB41BD6BULL   // action noise, correlated

HD int drg_i(const float* g, int k) { return __float_as_int(g[k]); }

// schedule factor (dr_utils.py:82-87, vec_task.py:692-698) at gym frame `frame`, in python double
HD double dr_sched(const ha_dr_attr_t& a, int frame) {
    if (a.sched == HA_DR_SCHED_LINEAR) return 1.0 / (double)a.sched_steps * (double)(frame < a.sched_steps ? frame : a.sched_steps);
    if (a.sched == HA_DR_SCHED_CONSTANT) return frame < a.sched_steps ? 0.0 : 1.0;
    return 1.0;
}

// the scheduled range (dr_utils.py:98-130): gaussian (mu, var), else (lo, hi), in python double
HD void dr_range(const ha_dr_attr_t& a, int frame, double& r0, double& r1) {
    double s = dr_sched(a, frame), lo = a.range[0], hi = a.range[1];
    if (a.dist == HA_DR_DIST_GAUSSIAN) {
        if (a.op == HA_DR_OP_ADDITIVE) { lo *= s; hi *= s; }
        else { hi = hi * s; lo = lo * s + 1.0 * (1.0 - s); }
    } else {
        if (a.op == HA_DR_OP_ADDITIVE) { lo *= s; hi *= s; }
        else { lo = lo * s + 1.0 * (1.0 - s); hi = hi * s + 1.0 * (1.0 - s); }
    }
    r0 = lo;
    r1 = hi;
}

// get_bucketed_val (dr_utils.py:135-145): the bucket grid over the unscheduled range (2 sqrt(var) around mu for a
// non-uniform distribution), in python double; bisect(buckets, v) - 1, so a value below the grid takes the LAST
// bucket (index -1)
HD double dr_bucket(double v, const ha_dr_attr_t& a) {
    double lo, hi;
    if (a.dist == HA_DR_DIST_UNIFORM) {
        lo = a.range[0];
        hi = a.range[1];
    } else {
        double sd = sqrt(a.range[1]);
        lo = a.range[0] - 2.0 * sd;
        hi = a.range[0] + 2.0 * sd;
    }
    int nb = a.num_buckets;
    double w = hi - lo;
    double t = floor((v - lo) / w * (double)nb);
    int i = !(t >= 0.0) ? nb - 1 : (t > (double)(nb - 1) ? nb - 1 : (int)t);
    return w * (double)i / (double)nb + lo;
}

// one sample (generate_random_samples) applied to the nominal value og (apply_random_samples, dr_utils.py:186-208),
// in python double like the reference (the draw u / g is a float32 value), rounded once to the float32 property
HD float dr_value(const ha_dr_attr_t& a, double r0, double r1, float og, float u, float g) {
    double smp;
    if (a.dist == HA_DR_DIST_GAUSSIAN) {
        smp = r0 + r1 * (double)g;                              // np.random.normal(mu, var): var is the std
    } else if (a.dist == HA_DR_DIST_LOGUNIFORM) {
        float l0 = ha_logf((float)r0), l1 = ha_logf((float)r1);     // the shared float32 log / exp (oracle: f32.py)
        smp = (double)ha_expf(l0 + (l1 - l0) * u);
    } else {
        smp = r0 + (r1 - r0) * (double)u;
    }
    double v = a.op == HA_DR_OP_SCALING ? (double)og * smp : (double)og + smp;
    if (a.num_buckets > 0) v = dr_bucket(v, a);
    return (float)v;
}

// one randomized quantity of this env, element k (lane-parallel callers): the dr_scale entry it leaves
HD float dr_attr_sample(const ha_params_t& p, int attr, int env, uint32_t ep, int k, int frame, float og) {
    const ha_dr_attr_t& a = p.dr_attr[attr];
    double r0, r1;
    dr_range(a, frame, r0, r1);
    uint32_t key = 64u * (uint32_t)attr + (uint32_t)k;
    float u = 0.0f, g = 0.0f;
    if (a.dist == HA_DR_DIST_GAUSSIAN) g = dr_gauss(p.seed ^ DR_SALT_ENV, env, ep, key);
    else u = uniform01(p.seed ^ DR_SALT_ENV, env, ep, key);
    return dr_value(a, r0, r1, og, u, g);
}
// mass attributes keep the ratio new / nominal mass (inertia scales with it: recomputeInertia, dr_utils.py:63-64);
// og: the value the reference's sample multiplies (its original_props entry), own: the body's nominal mass
HD float dr_mass_ratio(const ha_params_t& p, int attr, int env, uint32_t ep, int k, int frame, float og, float own) {
    const ha_dr_attr_t& a = p.dr_attr[attr];
    if (a.op == HA_DR_OP_SCALING && a.num_buckets == 0 && og == own)
        return dr_attr_sample(p, attr, env, ep, k, frame, 1.0f);
    return dr_attr_sample(p, attr, env, ep, k, frame, og) / own;
}
HD bool dr_active(const ha_params_t& p, int attr, bool all) {
    const ha_dr_attr_t& a = p.dr_attr[attr];
    return a.dist != HA_DR_DIST_OFF && (all || !a.setup_only);
}
// element k of a robot list property is re-sampled in this randomization (ha_dr_attr_t.later_elems)
HD bool dr_elem(const ha_params_t& p, int attr, bool all, int k) {
    const ha_dr_attr_t& a = p.dr_attr[attr];
    return dr_active(p, attr, all) && (all || a.later_elems < 0 || k < a.later_elems);
}

// object o's dimension scale in LDS: the env's object_scale row (AllegroKuka's cuboid dims) times the DR actor scale;
// unscaled (osc[3] = 0, the bit-identical plain path) when neither applies
HD void dr_object_scale(SimCtx& c, const ha_state_t& st, int env, int o) {
    float s = c.dr ? c.dr[HA_DR_OBJ_SCALE + o] : 1.0f;
    if (st.object_scale) {
        const float* sc = st.object_scale + ((size_t)env * c.NO + o) * 3;
        c.o[o].osc[0] = sc[0] * s; c.o[o].osc[1] = sc[1] * s; c.o[o].osc[2] = sc[2] * s; c.o[o].osc[3] = 1.0f;
    } else if (s != 1.0f) {
        c.o[o].osc[0] = c.o[o].osc[1] = c.o[o].osc[2] = s;
        c.o[o].osc[3] = 1.0f;
    } else {
        c.o[o].osc[0] = c.o[o].osc[1] = c.o[o].osc[2] = 1.0f;
        c.o[o].osc[3] = 0.0f;
    }
}

// apply_randomizations' actor part for this env (vec_task.py:662-671,788-864), before the task's reset of the env:
// the first randomization samples every env; later ones the envs being reset (`full`) whose randomize_buf reached
// `frequency`, which restart their count (the first one leaves the counts as they are, as the reference does). Then
// randomize_buf += 1 for a step launch (post_physics_step, allegro_kuka_base.py:1430).
HD void dr_env_pre(SimCtx& c, const ha_state_t& st, int env, bool full, bool step) {
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    const float* G = c.drg;
    int lane = c.lane;
    bool all = drg_i(G, HA_DRG_ALL) != 0;
    int frame = drg_i(G, HA_DRG_FRAME);
    int rb = st.randomize_buf ? st.randomize_buf[env] : 0;
    bool smp = all || (full && rb >= p.dr_frequency);
    if (smp && !all) rb = 0;
    if (st.randomize_buf && lane == 0) st.randomize_buf[env] = rb + (step ? 1 : 0);
    if (!smp) return;
    float* row = st.dr_scale + (size_t)env * HA_DR_SIZE;
    uint32_t ep = st.episode[env];
    if (lane < c.L) {
        // after the first randomization the robot's list properties may take the object's original value (later_og)
        if (dr_elem(p, HA_DRA_LINK_MASS, all, lane)) {
            float own = m.link_mass[lane];
            float og = (!all && p.dr_attr[HA_DRA_LINK_MASS].later_og_object) ? m.pool_mass[c.o[0].pool] : own;
            row[HA_DR_LINK_MASS + lane] = dr_mass_ratio(p, HA_DRA_LINK_MASS, env, ep, lane, frame, og, own);
        }
        if (dr_elem(p, HA_DRA_LINK_FRIC, all, lane))
            row[HA_DR_LINK_FRIC + lane] = dr_attr_sample(p, HA_DRA_LINK_FRIC, env, ep, lane, frame, p.friction);
    }
    if (lane < c.D) {
        if (dr_active(p, HA_DRA_DOF_KD, all))
            row[HA_DR_DOF_KD + lane] = dr_attr_sample(p, HA_DRA_DOF_KD, env, ep, lane, frame, m.dof_kd[lane]);
        if (dr_active(p, HA_DRA_DOF_KP, all))
            row[HA_DR_DOF_KP + lane] = dr_attr_sample(p, HA_DRA_DOF_KP, env, ep, lane, frame, m.dof_kp[lane]);
        if (dr_active(p, HA_DRA_DOF_LOWER, all))
            row[HA_DR_DOF_LOWER + lane] = dr_attr_sample(p, HA_DRA_DOF_LOWER, env, ep, lane, frame, m.dof_lower[lane]);
        if (dr_active(p, HA_DRA_DOF_UPPER, all))
            row[HA_DR_DOF_UPPER + lane] = dr_attr_sample(p, HA_DRA_DOF_UPPER, env, ep, lane, frame, m.dof_upper[lane]);
    }
    bool rescale = dr_active(p, HA_DRA_OBJ_SCALE, all);
    if (lane < c.NO) {
        int o = lane;
        if (dr_active(p, HA_DRA_OBJ_MASS, all))
            row[HA_DR_OBJ_MASS + o] = dr_mass_ratio(p, HA_DRA_OBJ_MASS, env, ep, o, frame, m.pool_mass[c.o[o].pool],
                                                    m.pool_mass[c.o[o].pool]);
        if (dr_active(p, HA_DRA_OBJ_FRIC, all))
            row[HA_DR_OBJ_FRIC + o] = dr_attr_sample(p, HA_DRA_OBJ_FRIC, env, ep, o, frame, p.friction);
        if (rescale) {
            row[HA_DR_OBJ_SCALE + o] = dr_attr_sample(p, HA_DRA_OBJ_SCALE, env, ep, o, frame, 1.0f);
            dr_object_scale(c, st, env, o);
            // the COM offset moves with the scale: the object's pose (origin) stays where the root state put it
            const float* r = st.root_state + ((size_t)env * m.n_actors + m.actor_object0 + o) * 13;
            st3(c.o[o].oc, ld3(r) + qrot(ldq(c.o[o].oq), scale3(c, o, ld3(m.pool_com[c.o[o].pool]))));
        }
    }
    // a new geometry invalidates the env's persistent contact manifolds (ha_state_t.contact_cache contract)
    if (rescale && c.pcm) {
        int NO = c.NO, NS = m.n_static, NLH = m.n_link_hulls;
        int slots = NO * (1 + NS + NLH) + NO * (NO - 1) / 2 + NLH * NS + m.n_self_pairs;
        for (int k = lane; k < slots; k += 64) c.pcm[(size_t)k * HA_PCM_REC + 3] = 0.0f;
    }
    wsync();
}

// noise of one element (vec_task.py:718-726 gaussian, 745-752 uniform): op(x, (corr * P0 + P1) + white * P2 + P3) with
// corr ~ N(0, 1) per (env, element) redrawn at each non-env randomization (the reference's randn_like even for the
// uniform distribution) and white ~ N(0, 1) (gaussian) or U[0, 1) (uniform) per step
HD float dr_noise(const ha_dr_attr_t& a, const float* P, uint64_t sw, uint64_t sc, int env, uint32_t step,
                  uint32_t epoch, int k, float x) {
    float corr = dr_gauss(sc, env, epoch, k);
    float white = a.dist == HA_DR_DIST_GAUSSIAN ? dr_gauss(sw, env, step, k) : uniform01(sw, env, step, k);
    float n = ((corr * P[0] + P[1]) + white * P[2]) + P[3];
    return a.op == HA_DR_OP_SCALING ? x * n : x + n;
}
// obs_buf element k of this env after post_physics_step (vec_task.py:426-428)
HD float dr_obs(const SimCtx& c, int env, int k, float x) {
    const float* G = c.drg;
    if (!G || !drg_i(G, HA_DRG_VALID) || c.p->dr_attr[HA_DRA_OBS].dist == HA_DR_DIST_OFF) return x;
    return dr_noise(c.p->dr_attr[HA_DRA_OBS], G + HA_DRG_OBS, c.p->seed ^ DR_SALT_OBS_W, c.p->seed ^ DR_SALT_OBS_C, env,
                    (uint32_t)drg_i(G, HA_DRG_STEP), (uint32_t)drg_i(G, HA_DRG_EPOCH), k, x);
}

// action k of this env as the task reads it: the caller's raw action (ha_task_step_io) or the bound actions tensor,
// with the action noise of this step (vec_task.py:400-402), clamped to +-clip_actions when the launch got raw
// actions (vec_task.py:404, torch.clamp)
HD float act_at(const SimCtx& c, const ha_state_t& st, int env, int k, int na) {
    size_t i = (size_t)env * na + k;
    float a = c.act_in ? c.act_in[i] : st.actions[i];
    const float* G = c.drg;
    if (G && drg_i(G, HA_DRG_ACT_ON))
        a = dr_noise(c.p->dr_attr[HA_DRA_ACT], G + HA_DRG_ACT_USE, c.p->seed ^ DR_SALT_ACT_W, c.p->seed ^ DR_SALT_ACT_C,
                     env, (uint32_t)drg_i(G, HA_DRG_STEP), (uint32_t)drg_i(G, HA_DRG_ACT_EPOCH), k, a);
    if (c.act_in) a = fminf(fmaxf(a, -c.clip_act), c.clip_act);
    return a;
}

// the noise parameters of observations / actions at frame `frame` (vec_task.py:684-754), python double, rounded once:
// P = (corr scale, corr offset, white scale, white offset)
HD void dr_noise_params(const ha_dr_attr_t& a, int frame, float* P) {
    double s = dr_sched(a, frame);
    double r0 = a.range[0], r1 = a.range[1], c0 = a.range_corr[0], c1 = a.range_corr[1];
    if (a.dist == HA_DR_DIST_GAUSSIAN) {
        if (a.op == HA_DR_OP_ADDITIVE) { r0 *= s; r1 *= s; c0 *= s; c1 *= s; }
        else { r1 = r1 * s; r0 = r0 * s + 1.0 * (1.0 - s); c1 = c1 * s; c0 = c0 * s + 1.0 * (1.0 - s); }
        P[0] = (float)c1; P[1] = (float)c0; P[2] = (float)r1; P[3] = (float)r0;
    } else {
        if (a.op == HA_DR_OP_ADDITIVE) { r0 *= s; r1 *= s; c0 *= s; c1 *= s; }
        else {
            r0 = r0 * s + 1.0 * (1.0 - s); r1 = r1 * s + 1.0 * (1.0 - s);
            c0 = c0 * s + 1.0 * (1.0 - s); c1 = c1 * s + 1.0 * (1.0 - s);
        }
        P[0] = (float)(c1 - c0); P[1] = (float)c0; P[2] = (float)(r1 - r0); P[3] = (float)r0;
    }
}

// The shard-wide part of apply_randomizations before a step (mode 0) or reset (mode 1) launch; `any`: some env's
// reset_buf is set (reset_idx, and with it apply_randomizations, runs). Frames: the gym.simulate calls of the launch
// (control_freq_inv, plus the Ur5Sih reset_idx's extra call when an env resets).
HD void dr_global_update(const ha_params_t& p, float* g, int any, int mode) {
    auto gi = [&](int k) -> int { return __float_as_int(g[k]); };
    auto si = [&](int k, int v) { g[k] = __int_as_float(v); };
    if (mode == 0) {
        // this step's action noise is the one set by the last apply_randomizations BEFORE its pre_physics_step
        for (int k = 0; k < 4; k++) g[HA_DRG_ACT_USE + k] = g[HA_DRG_ACT + k];
        si(HA_DRG_ACT_EPOCH, gi(HA_DRG_EPOCH));
        si(HA_DRG_ACT_ON, gi(HA_DRG_VALID) && p.dr_attr[HA_DRA_ACT].dist != HA_DR_DIST_OFF ? 1 : 0);
        si(HA_DRG_STEP, gi(HA_DRG_STEP) + 1);
    }
    int frame = gi(HA_DRG_FRAME_NEXT);
    si(HA_DRG_FRAME, frame);
    int first = gi(HA_DRG_FIRST);
    int nonenv = 0, all = 0;
    if (any) {
        if (first) {
            nonenv = 1;
            all = 1;
        } else {
            nonenv = frame - gi(HA_DRG_LAST_RAND) >= p.dr_frequency ? 1 : 0;
        }
        si(HA_DRG_FIRST, 0);
    }
    si(HA_DRG_ALL, all);
    if (nonenv) {
        si(HA_DRG_LAST_RAND, frame);
        int epoch = gi(HA_DRG_EPOCH) + 1;
        si(HA_DRG_EPOCH, epoch);
        si(HA_DRG_VALID, 1);
        dr_noise_params(p.dr_attr[HA_DRA_OBS], frame, g + HA_DRG_OBS);
        dr_noise_params(p.dr_attr[HA_DRA_ACT], frame, g + HA_DRG_ACT);
        const ha_dr_attr_t& a = p.dr_attr[HA_DRA_GRAVITY];
        if (a.dist != HA_DR_DIST_OFF) {
            // gravity = original op sample per axis (dr_utils.py:163-173). The reference's original gravity is the
            // first randomization's prop, rewritten in place by that call: later samples apply to its result
            double r0, r1;
            dr_range(a, frame, r0, r1);
            for (int k = 0; k < 3; k++) {
                float u = 0.0f, gg = 0.0f;
                if (a.dist == HA_DR_DIST_GAUSSIAN) gg = dr_gauss(p.seed ^ DR_SALT_GRAV, 0, (uint32_t)epoch, k);
                else u = uniform01(p.seed ^ DR_SALT_GRAV, 0, (uint32_t)epoch, k);
                float og = all ? p.gravity[k] : g[HA_DRG_GRAVITY_OG + k];
                float v = dr_value(a, r0, r1, og, u, gg);
                g[HA_DRG_GRAVITY + k] = v;
                if (all) g[HA_DRG_GRAVITY_OG + k] = v;
            }
        }
    }
    int frames = mode == 0 ? p.control_freq_inv : 0;
    if (p.task == HA_TASK_UR5SIH && any) frames += 1;
    si(HA_DRG_FRAME_NEXT, frame + frames);
}
