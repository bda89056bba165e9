// ha_task.h - Ur5SihMultiObjectManipulation task math on the device (one wavefront per env).
// Reference: tasks/hand_arm/base/ur5sih.py (controllers), env/multi_object.py (observables),
// task/multi_object_manipulation.py (reset, reward, done). Compiled with -ffp-contract=off and the
// reference's own quaternion formulas so observations are bit-exact against the oracle.
#pragma once
#include "ha_dr.h"

#define NUM_ACT 11
// observation size for n objects: 80 + 3 n (object_pos) + 10 n (object_bounding_box) + 10 + 15 + 3
// (Ur5SihMultiObjectManipulation.yaml:24-26 with num_objects = n; 147 at the default 3)
HD constexpr int ur5sih_num_obs(int n_objects) { return 108 + 13 * n_objects; }
// robot link indices (body index in env = 1 + link)
#define LINK_FLANGE 9
__constant__ int c_tip_links[5] = {28, 15, 21, 24, 18};   // thumb, index, middle, ring, little (ur5sih.py:613)

// DOF indices (depth-first order, tools/build_model.py)
#define DI_INDEX 6
#define DI_IF_DISTAL 7
#define DI_LF 8
#define DI_LF_DISTAL 9
#define DI_MIDDLE 10
#define DI_MF_DISTAL 11
#define DI_RING 12
#define DI_RF_DISTAL 13
#define DI_TH_OPP 14
#define DI_TH_FLEX 15
#define DI_TH_DISTAL 16

// ----------------------------------------------------------------------------- reference quaternion forms
// torch_jit_utils.py:41-62 (8-multiplication form)
HD void ref_quat_mul(const float* a, const float* b, float* out) {
    float x1 = a[0], y1 = a[1], z1 = a[2], w1 = a[3];
    float x2 = b[0], y2 = b[1], z2 = b[2], w2 = b[3];
    float ww = (z1 + x1) * (x2 + y2);
    float yy = (w1 - y1) * (w2 + z2);
    float zz = (w1 + y1) * (w2 - z2);
    float xx = ww + yy + zz;
    float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
    out[3] = qq - ww + (z1 - y1) * (y2 - z2);
    out[0] = qq - xx + (x1 + w1) * (x2 + w2);
    out[1] = qq - yy + (w1 - x1) * (y2 + z2);
    out[2] = qq - zz + (z1 + y1) * (w2 - x2);
}
// torch_jit_utils.py:70-77
HD void ref_quat_apply(const float* a, const float* b, float* out) {
    float tx = (a[1] * b[2] - a[2] * b[1]) * 2.0f;
    float ty = (a[2] * b[0] - a[0] * b[2]) * 2.0f;
    float tz = (a[0] * b[1] - a[1] * b[0]) * 2.0f;
    out[0] = b[0] + a[3] * tx + (a[1] * tz - a[2] * ty);
    out[1] = b[1] + a[3] * ty + (a[2] * tx - a[0] * tz);
    out[2] = b[2] + a[3] * tz + (a[0] * ty - a[1] * tx);
}

// natural cubic spline piece evaluation (torchcubicspline semantics, see oracle/task_oracle.py)
HD float spline_eval(const ha_params_t& p, int sidx, float t) {
    int n = p.spline_pieces[sidx];
    int idx = 0;
    for (int k = 1; k < n; k++)
        if (t > p.spline[sidx][0][k]) idx = k;
    float f = t - p.spline[sidx][0][idx];
    float inner = 0.5f * p.spline[sidx][3][idx] + p.spline[sidx][4][idx] * f / 3.0f;
    inner = p.spline[sidx][2][idx] + inner * f;
    return p.spline[sidx][1][idx] + inner * f;
}

// ----------------------------------------------------------------------------- controllers
// ur5sih.py:397-405 (relative joint targets) and 485-527 (smoothed relative servo -> joint map).
HD void controller_step(SimCtx& c, const ha_state_t& st, int env) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    float* tgt = st.dof_position_targets + (size_t)env * D;
    float* servo_sh = s.u.xfer + 8;
    if (lane < 6) {
        float u = st.ur5_target[env * 6 + lane] + p.action_dt * act_at(c, st, env, lane, NUM_ACT);
        st.ur5_target[env * 6 + lane] = u;
        s.u.xfer[lane] = u;
    } else if (lane < 11) {
        int i = lane - 6;
        float beta = p.sih_beta;
        float sm = p.sih_alpha * act_at(c, st, env, lane, NUM_ACT) + beta * st.smoothed[env * 5 + i];
        st.smoothed[env * 5 + i] = sm;
        float sv = st.servo[env * 5 + i] + 100.0f * sm;
        sv = sv < p.servo_lower[i] ? p.servo_lower[i] : sv;
        sv = sv > p.servo_upper[i] ? p.servo_upper[i] : sv;
        st.servo[env * 5 + i] = sv;
        servo_sh[i] = sv;
    }
    wsync();
    if (lane < D) {
        int d = lane;
        float v = 0.0f;
        if (d < 6) v = s.u.xfer[d];
        else if (d == DI_TH_OPP) v = p.thumb_opposition_gain * servo_sh[0];
        else if (d == DI_TH_FLEX) v = -spline_eval(p, 0, servo_sh[1]);
        else if (d == DI_TH_DISTAL) v = -spline_eval(p, 1, servo_sh[1] + p.proximal_coef[0] * s.q[DI_TH_FLEX]);
        else if (d == DI_INDEX) v = spline_eval(p, 2, servo_sh[2]);
        else if (d == DI_IF_DISTAL) v = spline_eval(p, 3, servo_sh[2] + p.proximal_coef[1] * s.q[DI_INDEX]);
        else if (d == DI_MIDDLE) v = spline_eval(p, 4, servo_sh[3]);
        else if (d == DI_MF_DISTAL) v = spline_eval(p, 5, servo_sh[3] + p.proximal_coef[2] * s.q[DI_MIDDLE]);
        else if (d == DI_RING || d == DI_LF) v = spline_eval(p, 6, servo_sh[4]);
        else if (d == DI_RF_DISTAL || d == DI_LF_DISTAL) v = spline_eval(p, 7, servo_sh[4] + p.proximal_coef[3] * s.q[DI_RING]);
        tgt[d] = v;
        s.tgt[d] = v;        // set_dof_position_target_tensor (actionable_vec_task.py:39-40)
    }
    wsync();
}

// (the device RNG, mix32 / uniform01 / gauss01, lives in ha_dr.h)

// ----------------------------------------------------------------------------- reset_idx (steady state)
// multi_object_manipulation.py:62-71 + _reset_objects :73-91, _reset_target_object :193-209,
// _reset_goal :211-230 + _get_random_object_pos :175-184, Ur5Sih._reset_ur5sih (ur5sih.py:616-632),
// controller resets (ur5sih.py:466-478). Draw order = reference order: cfg, target, goal[3].
HD void task_reset(SimCtx& c, const ha_state_t& st, int env, uint32_t flags) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, NO = c.NO, A = m.n_actors, P = p.num_initial_poses;
    float dr[5];
    if (flags & HA_FLAG_REPLAY_DRAWS) {
#pragma unroll
        for (int k = 0; k < 5; k++) dr[k] = st.reset_draws[env * HA_DRAW_STRIDE + k];
    } else {
        uint32_t ep = st.episode[env];
        float u0 = uniform01(p.seed, env, ep, 0), u1 = uniform01(p.seed, env, ep, 1);
        dr[0] = floorf(u0 * (float)P);
        dr[1] = floorf(u1 * (float)NO);
#pragma unroll
        for (int k = 0; k < 3; k++) dr[2 + k] = uniform01(p.seed, env, ep, 2 + k);
    }
    int cfg = (int)dr[0], tgt_obj = (int)dr[1];
    cfg = cfg < 0 ? 0 : (cfg >= P ? P - 1 : cfg);
    tgt_obj = tgt_obj < 0 ? 0 : (tgt_obj >= NO ? NO - 1 : tgt_obj);
    if (lane < NO) {
        int o = lane;
        const float* pos0 = st.object_pos_initial + (((size_t)env * P + cfg) * NO + o) * 3;
        const float* quat0 = st.object_quat_initial + (((size_t)env * P + cfg) * NO + o) * 4;
        float* r = st.root_state + ((size_t)env * A + m.actor_object0 + o) * 13;
        r[0] = pos0[0]; r[1] = pos0[1]; r[2] = pos0[2];
        r[3] = quat0[0]; r[4] = quat0[1]; r[5] = quat0[2]; r[6] = quat0[3];
        for (int k = 7; k < 13; k++) r[k] = 0.0f;
        qf q = ldq(quat0);
        stq(c.o[o].oq, q);
        st3(c.o[o].oc, ld3(pos0) + qrot(q, scale3(c, o, ld3(c.m->pool_com[c.o[o].pool]))));
        st3(c.o[o].ov, mk3(0, 0, 0));
        st3(c.o[o].ow, mk3(0, 0, 0));
    } else if (lane >= 8 && lane < 11) {
        int k = lane - 8;
        float noise = 2.0f * (dr[2 + k] - 0.5f);
        noise = noise * p.goal_noise[k];
        float g = p.goal_pos[k] + noise;
        st.goal_pos[env * 3 + k] = g;
        st.root_state[((size_t)env * A + m.actor_goal) * 13 + k] = g;
    } else if (lane == 12) {
        st.target_object_index[env] = tgt_obj;
        st.object_configuration_indices[env] = cfg;
        st.reset_draws[env * HA_DRAW_STRIDE + 0] = dr[0];
        st.reset_draws[env * HA_DRAW_STRIDE + 1] = dr[1];
    } else if (lane >= 16 && lane < 21) {
        int i = lane - 16;
        st.servo[env * 5 + i] = p.servo_upper[i];
        st.smoothed[env * 5 + i] = 0.0f;
    }
    if (lane < D) {
        float rp = p.reset_pose[lane];
        s.q[lane] = rp;
        s.qd[lane] = 0.0f;
        s.tgt[lane] = rp;                                   // set_dof_position_target_tensor_indexed
        st.dof_position_targets[(size_t)env * D + lane] = lane < 6 ? rp : 0.0f;   // ur5sih.py:477
    }
    wsync();
}

// reset bookkeeping after the post-reset simulate (ur5sih.py:388-389; configurable_vec_task.py:426-428;
// multi_object_manipulation.py:389-398)
HD void task_reset_finish(SimCtx& c, const ha_state_t& st, int env) {
    EnvLDS& s = *c.s;
    int lane = c.lane;
    if (lane < 6) st.ur5_target[env * 6 + lane] = s.q[lane];
    if (lane == 0) {
        st.reset_buf[env] = 0;
        st.progress_buf[env] = 0;
        st.goal_reached_before[env] = 0;
        st.episode[env] = st.episode[env] + 1;
    }
}

// ----------------------------------------------------------------------------- observation snapshot
// What the observables read after refresh_simulation_tensors(): flange pose, fingertip states,
// dof positions, object root states.  Filled from FK (fused step) or from the state tensors (observe).

HD void post_step(SimCtx& c, const ha_state_t& st, int env, const ObsIn& in, bool obs_only) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D, NO = c.NO;
    float* ob = s.u.pd.obs;
    int tgt = (int)st.target_object_index[env];
    int cfg = (int)st.object_configuration_indices[env];
    const float* goal = st.goal_pos + env * 3;
    const float* cache = st.obs_cache + (size_t)env * NO * 7;
    // observation vector (Ur5SihMultiObjectManipulation.yaml:24-26), computed lane-parallel; object blocks
    // sized by the object count (multi_object.py:128,245)
    const int NOBS = ur5sih_num_obs(NO);
    const int e_bb = 80 + 3 * NO, e_tb = e_bb + 10 * NO, e_ft = e_tb + 10, e_tg = e_ft + 15;
    for (int e = lane; e < NOBS; e += 64) {
        float v;
        if (e < 6) v = in.dofpos[e];
        else if (e < 13) v = in.flange[e - 6];
        else if (e < 28) { int t = (e - 13) / 3, k = (e - 13) % 3; v = in.tip[t][k]; }
        else if (e < 48) { int t = (e - 28) / 4, k = (e - 28) % 4; v = in.tip[t][3 + k]; }
        else if (e < 63) { int t = (e - 48) / 3, k = (e - 48) % 3; v = in.tip[t][7 + k]; }
        else if (e < 80) v = st.dof_position_targets[(size_t)env * D + (e - 63)];
        else if (e < e_bb) { int o = (e - 80) / 3, k = (e - 80) % 3; v = in.obj[o][k]; }
        else if (e < e_ft) {
            // object bounding boxes from the PREVIOUS refresh's object pose (reference refresh order,
            // see oracle/task_oracle.py observations())
            int o = e < e_tb ? (e - e_bb) / 10 : tgt;
            int k = e < e_tb ? (e - e_bb) % 10 : e - e_tb;
            int pid = c.o[o].pool;
            const float* cq = cache + o * 7;
            if (k < 3) {
                float r3[3];
                ref_quat_apply(cq + 3, m.pool_bbox_pos[pid], r3);
                v = cq[k] + r3[k];
            } else if (k < 7) {
                float r4[4];
                ref_quat_mul(cq + 3, m.pool_bbox_quat[pid], r4);
                v = r4[k - 3];
            } else {
                v = m.pool_bbox_ext[pid][k - 7];
            }
        } else if (e < e_tg) { int t = (e - e_ft) / 3, k = (e - e_ft) % 3; v = in.obj[tgt][k] - in.tip[t][k]; }
        else { int k = e - e_tg; v = goal[k] - in.obj[tgt][k]; }
        ob[e] = v;
    }
    wsync();
    // DR observation noise (vec_task.py:427-428: applied to obs_buf after post_physics_step, not to the
    // teacher observations and not in VecTask.reset)
    for (int e = lane; e < NOBS; e += 64) {
        float v = ob[e];
        st.teacher_obs[(size_t)env * NOBS + e] = v;
        if (!obs_only) v = dr_obs(c, env, e, v);
        st.obs[(size_t)env * NOBS + e] = v;
    }
    if (obs_only) return;     // VecTask.reset(): compute_observations without a refresh
    // refresh the observable cache with the current object pose
    for (int e = lane; e < NO * 7; e += 64) {
        int o = e / 7, k = e % 7;
        st.obs_cache[(size_t)env * NO * 7 + e] = in.obj[o][k];
    }
    // reward (multi_object_manipulation.py:237-313), done mask (:232-235), timeout (vec_task.py:424)
    if (lane == 0) {
        int64_t prog = st.progress_buf[env] + 1;     // configurable_vec_task.py:360
        st.progress_buf[env] = prog;
        int64_t rb = st.reset_buf[env];
        rb = prog >= p.max_episode_length ? 1 : rb;
        st.reset_buf[env] = rb;
        st.timeout_buf[env] = (prog >= p.max_episode_length - 1) && (rb != 0);
        const float* tp = in.obj[tgt];
        float dx = tp[0] - goal[0], dy = tp[1] - goal[1], dz = tp[2] - goal[2];
        float dist = sqrtf(dx * dx + dy * dy + dz * dz);
        bool reached = dist < p.goal_threshold;
        const float* init = st.object_pos_initial + (((size_t)env * p.num_initial_poses + cfg) * NO + tgt) * 3;
        float dh_z = tp[2] - init[2];
        bool lifted = dh_z > p.lifting_threshold;
        float r_reach, r_lift, r_goal, r_succ;
        {
            float dsum = 0.0f;
            for (int t = 0; t < 5; t++) {
                float ax_ = in.tip[t][0] - tp[0], ay_ = in.tip[t][1] - tp[1], az_ = in.tip[t][2] - tp[2];
                float fd = sqrtf(ax_ * ax_ + ay_ * ay_ + az_ * az_);
                if (t == 0) fd *= 4.0f;
                dsum += fd;
            }
            r_reach = p.reward_reaching * expf(-3.0f * dsum);
        }
        {
            float lt = p.lifting_threshold;
            float dh = fminf(fmaxf(lt - dh_z, 0.0f), lt) / lt;
            r_lift = p.reward_lifting * (expf(-3.0f * dh) - expf(-3.0f));
        }
        r_goal = p.reward_goal * (lifted ? 1.0f : 0.0f) * expf(-5.0f * dist);
        r_succ = p.reward_success * (reached ? 1.0f : 0.0f);
        float rew = 0.0f;
        rew = rew + r_reach;       // yaml order: reaching, lifting, goal, success
        rew = rew + r_lift;
        rew = rew + r_goal;
        rew = rew + r_succ;
        st.rew[env] = rew;
        bool before = st.goal_reached_before[env] != 0 || reached;
        st.goal_reached_before[env] = before;
        // device-side log accumulators (the reference does these with .item() host syncs)
        int pid = c.o[tgt].pool;
        if (rb != 0) {
            atomicAdd(&st.stats[0], 1);
            atomicAdd(&st.stats[2 + 2 * pid], 1);
        }
        if (before) {
            atomicAdd(&st.stats[1], 1);
            atomicAdd(&st.stats[3 + 2 * pid], 1);
        }
        atomicAdd(&st.term_sums[0], r_reach);
        atomicAdd(&st.term_sums[1], r_lift);
        atomicAdd(&st.term_sums[2], r_goal);
        atomicAdd(&st.term_sums[3], r_succ);
    }
}
