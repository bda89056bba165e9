// ah_task.h - AllegroHand in-hand cube reorientation (tasks/allegro_hand.py, cfg/task/AllegroHand.yaml)
// on the device: one wavefront per env, fused with the physics of VecTask.step in ah_step_kernel.
//   pre_physics_step  allegro_hand.py:586-625  (goal resets, reset_idx, absolute targets + moving average)
//   reset_target_pose allegro_hand.py:506-522
//   reset_idx         allegro_hand.py:524-584
//   compute_observations allegro_hand.py:406-504 (observationType "full_state" 88 floats, "full" 72, "full_no_vel" 50;
//                        asymmetric_observations: the full_state vector to the states buffer too)
//   compute_hand_reward allegro_hand.py:663-719
#pragma once
#include "ha_task.h"

#define AH_ND 16
#define AH_NUM_OBS 88           /* full_state; ha_params_t.num_obs is the observation type's size */
#define AH_NUM_STATES 88
#define AH_NUM_ACT 16

// replayed draws (HA_FLAG_REPLAY_DRAWS) in reset_draws[env][...], in the reference's draw order:
//   [0, 4)   reset_target_pose(goal_env_ids): torch_rand_float(-1, 1, (n, 4))
//   [4, 41)  reset_idx rand_floats: torch_rand_float(-1, 1, (n, 2 * 16 + 5))
//   [41, 45) reset_idx -> reset_target_pose(env_ids): torch_rand_float(-1, 1, (n, 4))
//   [45]     reset_idx: random_force_prob's torch.rand (:559-560)
//   [46]     pre_physics_step: torch.rand(num_envs) against random_force_prob (:621)
//   [47, 50) torch.randn(3) of a selected env (:622-623); [50] 1 when the reference selected the env (the host's
//            comparison, so a replayed run cannot differ from it by a last-bit difference of exp / log)
#define AH_DRAW_GOAL 0
#define AH_DRAW_RESET 4
#define AH_DRAW_RESET_GOAL 41
#define AH_DRAW_FORCE_PROB 45
#define AH_DRAW_FORCE_U 46
#define AH_DRAW_FORCE_N 47
#define AH_DRAW_FORCE_SEL 50
// an AllegroHand env's task_state row (random object forces, forceScale > 0): the force in the object frame, its
// random_force_prob and the counter of its device-mode force draws
#define AH_TS_FORCE 0
#define AH_TS_PROB 3
#define AH_TS_RNG 4
#define AH_TS_N 8

// What the observation reads after the refresh: dof pos / vel / force, object root state.
struct AhIn {
    float q[AH_ND], qd[AH_ND], f[AH_ND];
    float obj[13];
};

HD float ah_draw(const SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k) {
    if (flags & HA_FLAG_REPLAY_DRAWS) return st.reset_draws[(size_t)env * HA_DRAW_STRIDE + k];
    return 2.0f * uniform01(c.p->seed, env, st.episode[env], 64 + k) - 1.0f;      // torch_rand_float(-1, 1)
}

// torch_jit_utils.py:118-123 quat_from_angle_axis with a unit axis, then quat_unit
HD void ah_quat_from_angle_axis(float angle, int axis, float* q) {
    float th = angle / 2.0f;
    float sn, cs;
    ha_sincosf(th, &sn, &cs);           // the shared sine / cosine (include/ha_fmath.h, oracle/f32.py sincos)
    q[0] = axis == 0 ? sn : 0.0f * sn;
    q[1] = axis == 1 ? sn : 0.0f * sn;
    q[2] = axis == 2 ? sn : 0.0f * sn;
    q[3] = cs;
    float n = sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
    n = fmaxf(n, 1e-9f);
#pragma unroll
    for (int k = 0; k < 4; k++) q[k] = q[k] / n;
}
// allegro_hand.py:722-725 randomize_rotation(rand0, rand1, x_unit, y_unit)
HD void ah_randomize_rotation(float r0, float r1, float* q) {
    const float PI_F = 3.14159265358979323846f;
    float qa[4], qb[4];
    ah_quat_from_angle_axis(r0 * PI_F, 0, qa);
    ah_quat_from_angle_axis(r1 * PI_F, 1, qb);
    ref_quat_mul(qa, qb, q);
}

// Goal and env resets of pre_physics_step for this env (allegro_hand.py:586-599). A goal-only reset
// uses draw [0, 4); a full reset re-draws the goal at [41, 45) after the object/hand draw [4, 41), so
// the later draw wins exactly as in the reference. The hand/object state is reset in LDS (load_env ran
// first) and in the root/dof tensors.
HD void ah_reset(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, bool goal, bool full, float& tsv) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, A = m.n_actors;
    if (goal || full) {
        int base = full ? AH_DRAW_RESET_GOAL : AH_DRAW_GOAL;
        float g0 = ah_draw(c, st, env, flags, base), g1 = ah_draw(c, st, env, flags, base + 1);
        float rot[4];
        ah_randomize_rotation(g0, g1, rot);
        float* gs = st.goal_state + (size_t)env * 7;
        float* gr = st.root_state + ((size_t)env * A + m.actor_goal) * 13;
        if (lane < 3) {
            gs[lane] = p.ah_goal_init[lane];
            gr[lane] = p.ah_goal_init[lane] + p.ah_goal_displacement[lane];
        } else if (lane < 7) {
            gs[lane] = rot[lane - 3];
            gr[lane] = rot[lane - 3];
        } else if (lane < 13) {
            gr[lane] = 0.0f;
        } else if (lane == 13) {
            st.reset_goal_buf[env] = 0;
        }
    }
    if (full) {
        const float* ini = p.ah_object_init;
        float noise = p.ah_reset_position_noise;
        float pos[3];
#pragma unroll
        for (int k = 0; k < 3; k++) pos[k] = ini[k] + noise * ah_draw(c, st, env, flags, AH_DRAW_RESET + k);
        float rot[4];
        if (p.ah_object_type == 2) {
            // randomize_rotation_pen(rand0, rand1, 0.3) (:542-546, 729-732): about x by 0.5 pi + rand0 max_angle, then
            // about z by rand0 pi (rand1 unused)
            const float PI_F = 3.14159265358979323846f;
            float r0 = ah_draw(c, st, env, flags, AH_DRAW_RESET + 3);
            float qa[4], qb[4];
            ah_quat_from_angle_axis(1.57079632679489661923f + r0 * 0.3f, 0, qa);
            ah_quat_from_angle_axis(r0 * PI_F, 2, qb);
            ref_quat_mul(qa, qb, rot);
        } else {
            ah_randomize_rotation(ah_draw(c, st, env, flags, AH_DRAW_RESET + 3),
                                  ah_draw(c, st, env, flags, AH_DRAW_RESET + 4), rot);
        }
        float* r = st.root_state + ((size_t)env * A + m.actor_object0) * 13;
        if (lane < 13) r[lane] = lane < 3 ? pos[lane] : (lane < 7 ? rot[lane - 3] : 0.0f);
        if (lane == 0) {
            qf q = qf{rot[0], rot[1], rot[2], rot[3]};
            stq(c.o[0].oq, q);
            st3(c.o[0].oc, mk3(pos[0], pos[1], pos[2]) + qrot(q, ld3(m.pool_com[c.o[0].pool])));
            st3(c.o[0].ov, mk3(0, 0, 0));
            st3(c.o[0].ow, mk3(0, 0, 0));
        }
        if (lane < D) {
            float lo = m.dof_lower[lane], up = m.dof_upper[lane];
            float dmax = up - 0.0f, dmin = lo - 0.0f;
            float rd = dmin + ((dmax - dmin) * 0.5f) * (ah_draw(c, st, env, flags, AH_DRAW_RESET + 5 + lane) + 1.0f);
            float pos_d = 0.0f + p.ah_reset_dof_pos_noise * rd;
            float vel_d = 0.0f + p.ah_reset_dof_vel_noise * ah_draw(c, st, env, flags, AH_DRAW_RESET + 5 + D + lane);
            s.q[lane] = pos_d;
            s.qd[lane] = vel_d;
            s.tgt[lane] = pos_d;
            st.dof_position_targets[(size_t)env * D + lane] = pos_d;      // prev_targets
        }
        if (lane == 0) {
            st.progress_buf[env] = 0;
            st.reset_buf[env] = 0;
            st.successes[env] = 0.0f;
        }
        // rb_forces[env_ids] = 0; random_force_prob = exp((log lo - log hi) * U[0, 1) + log hi) (:532,557-560)
        if (lane >= AH_TS_FORCE && lane < AH_TS_FORCE + 3) tsv = 0.0f;
        if (lane == AH_TS_PROB) {
            float u = (flags & HA_FLAG_REPLAY_DRAWS) ? st.reset_draws[(size_t)env * HA_DRAW_STRIDE + AH_DRAW_FORCE_PROB]
                                                     : uniform01(p.seed, env, st.episode[env], 64 + AH_DRAW_FORCE_PROB);
            float llo = logf(p.ah_force_prob_lo), lhi = logf(p.ah_force_prob_hi);
            tsv = expf((llo - lhi) * u + lhi);
        }
    }
    if (lane == 0 && (goal || full)) st.episode[env] = st.episode[env] + 1;
    wsync();
}

// targets (allegro_hand.py:602-616): useRelativeControl prev + dofSpeedScale * dt * action, else absolute targets with
// the moving average; clamped either way
HD void ah_controller(SimCtx& c, const ha_state_t& st, int env) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    if (lane < D) {
        float lo = m.dof_lower[lane], up = m.dof_upper[lane];
        float a = act_at(c, st, env, lane, AH_NUM_ACT);
        if (c.act_in) const_cast<float*>(st.actions)[(size_t)env * AH_NUM_ACT + lane] = a;          // the task's stored actions
        float* prev = st.dof_position_targets + (size_t)env * D;
        float cur;
        if (p.ah_relative_control) {
            cur = prev[lane] + p.ah_speed_dt * a;
        } else {
            cur = 0.5f * (a + 1.0f) * (up - lo) + lo;                            // scale()
            cur = p.ah_act_moving_average * cur + p.sih_beta * prev[lane];       // sih_beta := 1 - ama (python double)
        }
        cur = fmaxf(fminf(cur, up), lo);                                         // tensor_clamp
        prev[lane] = cur;
        s.tgt[lane] = cur;
    }
    wsync();
}

// random object forces (allegro_hand.py:617-625): decay, a new N(0, 1)^3 * mass * forceScale force with probability
// random_force_prob, applied in LOCAL_SPACE at the object COM -> the world force of the step's first physics call
HD void ah_forces(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, float& tsv) {
    const ha_params_t& p = *c.p;
    int lane = c.lane;
    if (p.ah_force_scale <= 0.0f) return;
    bool replay = (flags & HA_FLAG_REPLAY_DRAWS) != 0;
    const float* dr = st.reset_draws + (size_t)env * HA_DRAW_STRIDE;
    uint32_t ctr = __float_as_uint(bcast(tsv, AH_TS_RNG));
    float prob = bcast(tsv, AH_TS_PROB);
    float u = replay ? dr[AH_DRAW_FORCE_U] : uniform01(p.seed ^ 0x5EED5EEDULL, env, ctr, 0);
    bool sel = replay ? dr[AH_DRAW_FORCE_SEL] != 0.0f : u < prob;
    if (lane >= AH_TS_FORCE && lane < AH_TS_FORCE + 3) {
        int k = lane - AH_TS_FORCE;
        tsv = tsv * p.ah_force_decay_step;
        if (sel) {
            float g = replay ? dr[AH_DRAW_FORCE_N + k] : gauss01(p.seed ^ 0x5EED5EEDULL, env, ctr, 1 + k);
            tsv = (g * p.ah_object_rb_mass) * p.ah_force_scale;
        }
    }
    if (lane == AH_TS_RNG) tsv = __uint_as_float(ctr + 1u);
    f3 fl = mk3(bcast(tsv, AH_TS_FORCE), bcast(tsv, AH_TS_FORCE + 1), bcast(tsv, AH_TS_FORCE + 2));
    if (lane == 0) st3(c.o[0].ofx, qrot(ldq(c.o[0].oq), fl));
    wsync();
}

// observations (compute_full_state) + compute_hand_reward for one env
HD void ah_post(SimCtx& c, const ha_state_t& st, int env, const AhIn& in, bool obs_only) {
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    const float* gs = st.goal_state + (size_t)env * 7;
    float qdiff[4];
    {
        float gc[4] = {-gs[3], -gs[4], -gs[5], gs[6]};
        ref_quat_mul(&in.obj[3], gc, qdiff);
    }
    // compute_full_state (:484-504): 88 floats; element k of it
    auto full_state = [&](int k) -> float {
        if (k < 16) {
            float lo = m.dof_lower[k], up = m.dof_upper[k];
            return (2.0f * in.q[k] - up - lo) / (up - lo);                       // unscale()
        }
        if (k < 32) return p.ah_vel_obs_scale * in.qd[k - 16];
        if (k < 48) return p.ah_force_torque_obs_scale * in.f[k - 32];
        if (k < 58) return in.obj[k - 48];                                       // pose + linvel
        if (k < 61) return p.ah_vel_obs_scale * in.obj[k - 48];                  // angvel
        if (k < 68) return gs[k - 61];
        if (k < 72) return qdiff[k - 68];
        return act_at(c, st, env, k - 72, AH_NUM_ACT);
    };
    const int nobs = p.num_obs;
    float* ob = st.obs + (size_t)env * nobs;
    for (int k = lane; k < nobs; k += 64) {
        float v;
        if (p.ah_obs_type == 0) {
            v = full_state(k);
        } else if (p.ah_obs_type == 1) {
            // compute_full_observations (:448-460): dof pos, vel, object pose / linvel / angvel, goal, qdiff, actions
            v = full_state(k < 32 ? k : k + 16);
        } else {
            // compute_full_observations(no_vel=True) (:439-446): dof pos, object pose, goal pose, qdiff, actions
            v = full_state(k < 16 ? k : (k < 23 ? k + 32 : k + 38));
        }
        if (!obs_only) v = dr_obs(c, env, k, v);        // DR observation noise on obs_buf (vec_task.py:426-428)
        ob[k] = v;
        obs_out_put(c, (size_t)env * nobs + k, v);
    }
    if (p.ah_asymmetric && st.teacher_obs) {
        float* sb = st.teacher_obs + (size_t)env * AH_NUM_STATES;
        for (int k = lane; k < AH_NUM_STATES; k += 64) sb[k] = full_state(k);
    }
    if (obs_only) return;
    if (lane == 0) {
        float dx = in.obj[0] - gs[0], dy = in.obj[1] - gs[1], dz = in.obj[2] - gs[2];
        float goal_dist = sqrtf((dx * dx + dy * dy) + dz * dz);
        float rn = sqrtf((qdiff[0] * qdiff[0] + qdiff[1] * qdiff[1]) + qdiff[2] * qdiff[2]);
        float rot_dist = 2.0f * asinf(fminf(rn, 1.0f));
        float dist_rew = goal_dist * p.ah_dist_reward_scale;
        float rot_rew = 1.0f / (fabsf(rot_dist) + p.ah_rot_eps) * p.ah_rot_reward_scale;
        float ap = 0.0f;
        for (int k = 0; k < AH_NUM_ACT; k++) {
            float ak = act_at(c, st, env, k, AH_NUM_ACT);
            ap += ak * ak;
        }
        float reward = dist_rew + rot_rew + ap * p.ah_action_penalty_scale;
        int64_t goal_resets = fabsf(rot_dist) <= p.ah_success_tolerance ? 1 : st.reset_goal_buf[env];
        float succ = st.successes[env] + (float)goal_resets;
        if (goal_resets == 1) reward = reward + p.ah_reach_goal_bonus;
        if (goal_dist >= p.ah_fall_dist) reward = reward + p.ah_fall_penalty;
        int64_t resets = goal_dist >= p.ah_fall_dist ? 1 : st.reset_buf[env];
        int64_t prog = st.progress_buf[env];
        if (p.ah_max_consecutive_successes > 0) {
            if (fabsf(rot_dist) <= p.ah_success_tolerance) prog = 0;
            if (succ >= (float)p.ah_max_consecutive_successes) resets = 1;
        }
        bool timed_out = (float)prog >= (float)p.max_episode_length - 1.0f;
        if (timed_out) resets = 1;
        if (p.ah_max_consecutive_successes > 0 && timed_out) reward = reward + 0.5f * p.ah_fall_penalty;
        st.rew[env] = reward;
        st.reset_buf[env] = resets;
        st.reset_goal_buf[env] = goal_resets;
        st.progress_buf[env] = prog;
        st.successes[env] = succ;
        st.timeout_buf[env] = (prog >= (int64_t)p.max_episode_length - 1) && resets != 0;   // vec_task.py:424
        if (resets) {
            atomicAdd(&st.stats[0], 1);                                   // num_resets
            atomicAdd(&st.term_sums[0], succ);                            // sum(successes * resets)
        }
        (void)D;
    }
}

// consecutive_successes EWMA over the whole shard (allegro_hand.py:714-717), after all envs of the step
extern "C" __global__ void ah_consecutive_successes_kernel(const int32_t* stats, const float* term_sums,
                                                           float* cons, float av_factor) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        int n = stats[0];
        if (n > 0) cons[0] = av_factor * term_sums[0] / (float)n + (1.0f - av_factor) * cons[0];
    }
}
