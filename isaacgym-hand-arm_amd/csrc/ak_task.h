// ak_task.h - AllegroKuka (KUKA iiwa7 + Allegro, 23 DOF) regrasping / reorientation on the device:
// one wavefront per env, fused with the physics of VecTask.step in ak_step_kernel.
//   pre_physics_step     allegro_kuka_base.py:1355-1424 (goal resets, reset_idx, hand absolute targets with
//                        moving average, arm relative targets, random object forces)
//   reset_target_pose    :1191-1196 -> _reset_target (allegro_kuka_regrasping.py:76-98 /
//                        allegro_kuka_reorientation.py:106-131)
//   reset_object_pose    :1198-1224, get_random_quat :1178-1189
//   reset_idx            :1246-1353
//   compute_observations :991-1089, compute_full_state :1091-1172 (observationType "full_state")
//   compute_kuka_reward  :854-930 with _lifting_reward / _distance_delta_rewards / _keypoint_reward /
//                        _action_penalties / _compute_resets (:759-849)
// The tolerance curriculum (allegro_kuka_utils.py:86-119) is host logic; its scalars reach the kernel in
// ha_state_t.task_scalars.
#pragma once
#include "ah_task.h"

#define AK_ND 23
#define AK_NUM_ACT 23
#define AK_MAX_OBS 120

// replayed draws (HA_FLAG_REPLAY_DRAWS) in reset_draws[env][...], in the reference's draw order. G = the draws of one
// reset_target_pose: 9 (regrasping: target (3, U[0,1)) + reset_object_pose's position noise (3, U[-1,1)) and
// get_random_quat uvw (3, U[0,1)); reorientation: target (3) + goal quat uvw (3)), 10 for throw (bucket side
// U[-1,1), side offset U[0,0.4), y U[-1,0.7), z U[0,1) + reset_object_pose (6); allegro_kuka_throw.py:85-101)
//   [0, G)        reset_target_pose(goal_env_ids)
//   [G, 2G)       reset_idx -> reset_target_pose(env_ids), same layout
//   [2G, 2G+6)    reset_idx -> reset_object_pose: position noise (3) + quat uvw (3)
//   [2G+6]        random_force_prob draw, [2G+7, 2G+30) dof draws U[0,1), [2G+30, 2G+53) dof velocity draws U[-1,1)
//   [2G+53]       per-step force selection torch.rand(N), [2G+54, 2G+57) torch.randn(3) of a selected env
// (G = 9: 0, 9, 18, 24, 25, 48, 71, 72 as before v14; G = 10 ends at 77 < HA_DRAW_STRIDE)
HD int ak_goal_draws(const ha_params_t& p) { return p.ak_subtask == 2 ? 10 : 9; }
#define AK_DRAW_GOAL 0
#define AK_DRAW_RESET_GOAL(p) (ak_goal_draws(p))
#define AK_DRAW_OBJ(p) (2 * ak_goal_draws(p))
#define AK_DRAW_FORCE_PROB(p) (2 * ak_goal_draws(p) + 6)
#define AK_DRAW_DOF(p) (2 * ak_goal_draws(p) + 7)
#define AK_DRAW_VEL(p) (2 * ak_goal_draws(p) + 30)
#define AK_DRAW_FORCE_U(p) (2 * ak_goal_draws(p) + 53)
#define AK_DRAW_FORCE_N(p) (2 * ak_goal_draws(p) + 54)
// per-env keypoint offsets (host-computed in python double, allegro_kuka_base.py:705-715) in task_state
#define AK_TS_KP HA_AK_KP

// What the observation reads after the refresh: dof state, palm / fingertip rigid-body states, object root.
struct AkIn {
    float q[AK_ND], qd[AK_ND];
    float palm[13];
    float tip[4][7];
    float obj[13];
};
// post-physics staging; lives at s.u.pd.in (free after store_env: in, obs, cforce, dforce)
struct AkPost {
    AkIn in;
    float ts[HA_AK_TS];
    float obs[AK_MAX_OBS];
};

HD float ak_draw01(const SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k) {
    if (flags & HA_FLAG_REPLAY_DRAWS) return st.reset_draws[(size_t)env * HA_DRAW_STRIDE + k];
    return uniform01(c.p->seed, env, st.episode[env], 128 + k);                  // torch_rand_float(0, 1)
}
HD float ak_draw11(const SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k) {
    if (flags & HA_FLAG_REPLAY_DRAWS) return st.reset_draws[(size_t)env * HA_DRAW_STRIDE + k];
    return 2.0f * uniform01(c.p->seed, env, st.episode[env], 128 + k) - 1.0f;    // torch_rand_float(-1, 1)
}

HD float ak_draw_range(const SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k, float lo, float span) {
    if (flags & HA_FLAG_REPLAY_DRAWS) return st.reset_draws[(size_t)env * HA_DRAW_STRIDE + k];
    return span * uniform01(c.p->seed, env, st.episode[env], 128 + k) + lo;      // torch_rand_float(lo, lo + span)
}

// torch_jit_utils.py:81-90 quat_rotate (xyzw)
HD void ak_quat_rotate(const float* q, const float* v, float* out) {
    float qw = q[3];
    float aw = 2.0f * (qw * qw) - 1.0f;
    float cx = q[1] * v[2] - q[2] * v[1], cy = q[2] * v[0] - q[0] * v[2], cz = q[0] * v[1] - q[1] * v[0];
    float dt = (q[0] * v[0] + q[1] * v[1]) + q[2] * v[2];
    out[0] = (v[0] * aw + (cx * qw) * 2.0f) + (q[0] * dt) * 2.0f;
    out[1] = (v[1] * aw + (cy * qw) * 2.0f) + (q[1] * dt) * 2.0f;
    out[2] = (v[2] * aw + (cz * qw) * 2.0f) + (q[2] * dt) * 2.0f;
}
HD float ak_norm3(const float* v) { return sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]); }

// get_random_quat (allegro_kuka_base.py:1178-1189) from uvw draws
HD void ak_random_quat(float u0, float u1, float u2, float* q) {
    const float TWO_PI = 6.283185307179586f;      // 2 * np.pi, rounded by the tensor multiply
    float a = sqrtf(1.0f - u0), b = sqrtf(u0);
    // the shared sine / cosine (include/ha_fmath.h), so the oracle chain of the fused step reproduces the reset
    // pose bit for bit (oracle/f32.py sincos)
    float s1, c1, s2, c2;
    ha_sincosf(TWO_PI * u1, &s1, &c1);
    ha_sincosf(TWO_PI * u2, &s2, &c2);
    q[3] = a * s1;
    q[0] = a * c1;
    q[1] = b * s2;
    q[2] = b * c2;
}

// reset_object_pose for this env (draw base k0: position noise [k0, k0+3), quat uvw [k0+3, k0+6)).
// tsv is this lane's task_state element (lane = field index).
HD void ak_reset_object_pose(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k0, float& tsv) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    int lane = c.lane;
    float pos[3], q[4];
#pragma unroll
    for (int k = 0; k < 3; k++) pos[k] = p.ak_object_init[k] + p.ak_reset_noise[k] * ak_draw11(c, st, env, flags, k0 + k);
    ak_random_quat(ak_draw01(c, st, env, flags, k0 + 3), ak_draw01(c, st, env, flags, k0 + 4),
                   ak_draw01(c, st, env, flags, k0 + 5), q);
    float* r = st.root_state + ((size_t)env * m.n_actors + m.actor_object0) * 13;
    if (lane < 13) r[lane] = lane < 3 ? pos[lane] : (lane < 7 ? q[lane - 3] : 0.0f);
    if (lane == 0) {
        qf qq = qf{q[0], q[1], q[2], q[3]};
        stq(c.o[0].oq, qq);
        st3(c.o[0].oc, mk3(pos[0], pos[1], pos[2]) + qrot(qq, scale3(c, 0, ld3(m.pool_com[c.o[0].pool]))));
        st3(c.o[0].ov, mk3(0, 0, 0));
        st3(c.o[0].ow, mk3(0, 0, 0));
    }
    if (lane >= HA_AK_CLOSEST_FT && lane < HA_AK_CLOSEST_FT + 4) tsv = -1.0f;
    if (lane == HA_AK_FURTHEST) tsv = -1.0f;
}

// reset_target_pose (draw base k0)
HD void ak_reset_target_pose(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, int k0, float& tsv) {
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    int lane = c.lane;
    float tgt[3];
    float* gs = st.goal_state + (size_t)env * 7;
    float* gr = st.root_state + ((size_t)env * m.n_actors + m.actor_goal) * 13;
    if (p.ak_subtask == 2) {
        // throw (allegro_kuka_throw.py:85-103): the bucket (the actor in the goal slot, carrying the posed statics)
        // left or right of the table, the goal 5 cm above its origin, the object back on the table
        float lr = ak_draw11(c, st, env, flags, k0);
        float off = ak_draw_range(c, st, env, flags, k0 + 1, 0.0f, 0.4f);
        float sg = lr > 0.0f ? 1.0f : (lr < 0.0f ? -1.0f : 0.0f);                // torch.sign
        tgt[0] = (lr > 0.0f ? 0.5f : -0.5f) + sg * off;
        tgt[1] = ak_draw_range(c, st, env, flags, k0 + 2, -1.0f, 1.7f);
        tgt[2] = ak_draw01(c, st, env, flags, k0 + 3);
        if (lane < 3) {
            gr[lane] = tgt[lane];
            gs[lane] = lane == 2 ? tgt[2] + 0.05f : tgt[lane];
            c.s->sb[lane] = tgt[lane];                        // the posed statics follow the bucket this launch
        }
        ak_reset_object_pose(c, st, env, flags, k0 + 4, tsv);
        if (lane == HA_AK_LIFTED) tsv = 0.0f;
        if (lane == 0) st.reset_goal_buf[env] = 0;
        if (lane == HA_AK_NEAR_GOAL) tsv = 0.0f;
        if (lane == HA_AK_CLOSEST_KP) tsv = -1.0f;
        return;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) tgt[k] = p.ak_target_lo[k] + ak_draw01(c, st, env, flags, k0 + k) * p.ak_target_size[k];
    if (lane < 3) {
        gs[lane] = tgt[lane];
        gr[lane] = tgt[lane];
    }
    if (p.ak_subtask == 0) {
        ak_reset_object_pose(c, st, env, flags, k0 + 3, tsv);           // regrasping: object back on the table
        if (lane == HA_AK_LIFTED) tsv = 0.0f;
    } else {
        float q[4];
        ak_random_quat(ak_draw01(c, st, env, flags, k0 + 3), ak_draw01(c, st, env, flags, k0 + 4),
                       ak_draw01(c, st, env, flags, k0 + 5), q);
        if (lane >= 3 && lane < 7) {
            gs[lane] = q[lane - 3];
            gr[lane] = q[lane - 3];
        } else if (lane >= 7 && lane < 13) {
            gr[lane] = 0.0f;
        }
    }
    if (lane == 0) st.reset_goal_buf[env] = 0;
    if (lane == HA_AK_NEAR_GOAL) tsv = 0.0f;
    if (lane == HA_AK_CLOSEST_KP) tsv = -1.0f;
}

// goal resets then reset_idx of pre_physics_step (allegro_kuka_base.py:1362-1368)
HD void ak_reset(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, bool goal, bool full, float& tsv) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D;
    if (goal) ak_reset_target_pose(c, st, env, flags, AK_DRAW_GOAL, tsv);
    if (full) {
        ak_reset_target_pose(c, st, env, flags, AK_DRAW_RESET_GOAL(p), tsv);
        if (lane >= HA_AK_RB_FORCE && lane < HA_AK_RB_FORCE + 3) tsv = 0.0f;
        ak_reset_object_pose(c, st, env, flags, AK_DRAW_OBJ(p), tsv);
        if (lane == HA_AK_FORCE_PROB) {
            float llo = logf(p.ak_force_prob_lo), lhi = logf(p.ak_force_prob_hi);
            tsv = expf((llo - lhi) * ak_draw01(c, st, env, flags, AK_DRAW_FORCE_PROB(p)) + lhi);
        }
        if (lane < D) {
            float lo = m.dof_lower[lane], up = m.dof_upper[lane], def = p.reset_pose[lane];
            float dmax = up - def, dmin = lo - def;
            float rd = dmin + (dmax - dmin) * ak_draw01(c, st, env, flags, AK_DRAW_DOF(p) + lane);
            float coeff = lane < p.ak_num_arm_dofs ? p.ak_dof_noise_arm : p.ak_dof_noise_fingers;
            float pos = def + coeff * rd;
            float vel = p.ak_dof_vel_noise * ak_draw11(c, st, env, flags, AK_DRAW_VEL(p) + lane);
            s.q[lane] = pos;
            s.qd[lane] = vel;
            s.tgt[lane] = pos;
            st.dof_position_targets[(size_t)env * D + lane] = pos;      // prev_targets
        }
        float succ = st.successes[env];
        float tobj = bcast(tsv, HA_AK_TRUE_OBJ);
        if (lane == HA_AK_PREV_SUCC) tsv = succ;
        if (lane == HA_AK_PREV_TRUE_OBJ) tsv = tobj;
        if (lane == HA_AK_TRUE_OBJ || lane == HA_AK_LIFTED || lane == HA_AK_NEAR_GOAL) tsv = 0.0f;
        if (lane == HA_AK_CLOSEST_KP || lane == HA_AK_FURTHEST) tsv = -1.0f;
        if (lane >= HA_AK_CLOSEST_FT && lane < HA_AK_CLOSEST_FT + 4) tsv = -1.0f;
        if (lane >= HA_AK_REW_EP && lane < HA_AK_REW_EP + 12) tsv = 0.0f;
        wsync();
        if (lane == 0) {
            st.progress_buf[env] = 0;
            st.reset_buf[env] = 0;
            st.successes[env] = 0.0f;
        }
    }
    if (lane == 0 && (goal || full)) st.episode[env] = st.episode[env] + 1;
    wsync();
}

// hand: absolute targets with moving average and clamp; arm: relative targets (allegro_kuka_base.py:1373-1397)
HD void ak_controller(SimCtx& c, const ha_state_t& st, int env) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D, na = p.num_actions;
    // privilegedActions (v16): actions[:, :3] are the object torque and the hand reads actions[:, 3:][:, 7:23], while
    // the arm reads self.actions[:, :7] - the unstripped actions, torque columns included (allegro_kuka_base.py:1357-
    // 1397, as written)
    int pv = p.ak_privileged_actions ? 3 : 0;
    if (c.act_in && lane < na)
        const_cast<float*>(st.actions)[(size_t)env * na + lane] = act_at(c, st, env, lane, na);    // self.actions
    if (lane < D) {
        float lo = m.dof_lower[lane], up = m.dof_upper[lane];
        float a = act_at(c, st, env, lane >= p.ak_num_arm_dofs ? lane + pv : lane, na);
        float* prev = st.dof_position_targets + (size_t)env * D;
        float cur;
        if (lane >= p.ak_num_arm_dofs) {
            cur = 0.5f * (a + 1.0f) * (up - lo) + lo;                              // scale()
            cur = p.ak_act_moving_average * cur + p.ak_one_minus_ama * prev[lane];
        } else {
            cur = prev[lane] + p.ak_dof_speed_scale * a;                           // dofSpeedScale * dt, rounded
        }
        cur = fmaxf(fminf(cur, up), lo);                                           // tensor_clamp
        prev[lane] = cur;
        s.tgt[lane] = cur;
    }
    wsync();
}

// random object forces (allegro_kuka_base.py:1399-1414): decay, re-draw with probability random_force_prob,
// applied in LOCAL_SPACE at the object COM -> world force for this physics call; then the privileged actions' object
// torque (:1417-1424): actions[:, :3] x privilegedActionsTorque in ENV_SPACE
HD void ak_forces(SimCtx& c, const ha_state_t& st, int env, uint32_t flags, float& tsv) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    int lane = c.lane;
    if (p.ak_privileged_actions && lane < 3) c.o[0].otq[lane] = act_at(c, st, env, lane, p.num_actions) * p.ak_privileged_torque;
    if (p.ak_force_scale <= 0.0f) {
        wsync();
        return;
    }
    uint32_t ctr = __float_as_uint(bcast(tsv, HA_AK_RNG));
    float prob = bcast(tsv, HA_AK_FORCE_PROB);
    float u = (flags & HA_FLAG_REPLAY_DRAWS) ? st.reset_draws[(size_t)env * HA_DRAW_STRIDE + AK_DRAW_FORCE_U(p)]
                                             : uniform01(p.seed ^ 0xA5A5A5A5ULL, env, ctr, 0);
    if (lane >= HA_AK_RB_FORCE && lane < HA_AK_RB_FORCE + 3) {
        int k = lane - HA_AK_RB_FORCE;
        tsv = tsv * p.ak_force_decay_step;
        if (u < prob) {
            float g = (flags & HA_FLAG_REPLAY_DRAWS) ? st.reset_draws[(size_t)env * HA_DRAW_STRIDE + AK_DRAW_FORCE_N(p) + k]
                                                     : gauss01(p.seed, env, ctr, 1 + k);
            tsv = (g * p.ak_object_rb_mass) * p.ak_force_scale;
        }
    }
    if (lane == HA_AK_RNG) tsv = __uint_as_float(ctr + 1u);
    f3 fl = mk3(bcast(tsv, HA_AK_RB_FORCE), bcast(tsv, HA_AK_RB_FORCE + 1), bcast(tsv, HA_AK_RB_FORCE + 2));
    if (lane == 0) st3(c.o[0].ofx, qrot(ldq(c.o[0].oq), fl));
    wsync();
}

// compute_observations + compute_full_state (+ compute_kuka_reward, resets, obs reward slot, clamp)
HD void ak_post(SimCtx& c, const ha_state_t& st, int env, AkPost& ak, bool obs_only) {
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    float* tsg = st.task_state + (size_t)env * HA_AK_TS;
    if (lane < HA_AK_TS) ak.ts[lane] = tsg[lane];
    wsync();
    int nobs = p.num_obs;
    if (lane == 0) {
        const AkIn& in = ak.in;
        float* T = ak.ts;
        float* ob = ak.obs;
        const float* gs = st.goal_state + (size_t)env * 7;
        const float* obj = in.obj;
        float palm_c[3], ft[4][3], curr[4];
        ak_quat_rotate(&in.palm[3], p.ak_palm_offset, palm_c);
        for (int k = 0; k < 3; k++) palm_c[k] = in.palm[k] + palm_c[k];
        for (int i = 0; i < 4; i++) {
            float off[3];
            ak_quat_rotate(&in.tip[i][3], p.ak_fingertip_offsets[i], off);
            float rel[3];
            for (int k = 0; k < 3; k++) {
                ft[i][k] = in.tip[i][k] + off[k];
                rel[k] = ft[i][k] - obj[k];
            }
            curr[i] = ak_norm3(rel);
            if (T[HA_AK_CLOSEST_FT + i] < 0.0f) T[HA_AK_CLOSEST_FT + i] = curr[i];
        }
        if (T[HA_AK_FURTHEST] < 0.0f) T[HA_AK_FURTHEST] = curr[0];
        int o = 0;
        for (int d = 0; d < AK_ND; d++) {
            float lo = m.dof_lower[d], up = m.dof_upper[d];
            ob[o++] = (2.0f * in.q[d] - up - lo) / (up - lo);                  // unscale()
        }
        for (int d = 0; d < AK_ND; d++) ob[o++] = in.qd[d];
        for (int k = 0; k < 3; k++) ob[o++] = palm_c[k];
        for (int k = 3; k < 13; k++) ob[o++] = in.palm[k];
        for (int k = 3; k < 13; k++) ob[o++] = obj[k];
        for (int i = 0; i < 4; i++)
            for (int k = 0; k < 3; k++) ob[o++] = ft[i][k] - palm_c[k];
        int nkp = p.ak_num_keypoints;
        float kmax = 0.0f;
        int o_rel_goal = o + 3 * nkp;
        for (int j = 0; j < nkp; j++) {
            float okp[3], gkp[3], rg[3];
            ak_quat_rotate(&obj[3], &T[AK_TS_KP + 3 * j], okp);
            ak_quat_rotate(&gs[3], &T[AK_TS_KP + 3 * j], gkp);
            for (int k = 0; k < 3; k++) {
                okp[k] = obj[k] + okp[k];
                gkp[k] = gs[k] + gkp[k];
                rg[k] = okp[k] - gkp[k];
                ob[o + 3 * j + k] = okp[k] - palm_c[k];                          // keypoints_rel_palm
                ob[o_rel_goal + 3 * j + k] = rg[k];                              // keypoints_rel_goal
            }
            float dj = ak_norm3(rg);
            kmax = j == 0 ? dj : fmaxf(kmax, dj);
        }
        o += 6 * nkp;
        if (T[HA_AK_CLOSEST_KP] < 0.0f) T[HA_AK_CLOSEST_KP] = kmax;
        const float* osc = st.object_scale + (size_t)env * 3;
        for (int k = 0; k < 3; k++) ob[o++] = osc[k];
        ob[o++] = T[HA_AK_CLOSEST_KP];
        for (int i = 0; i < 4; i++) ob[o++] = T[HA_AK_CLOSEST_FT + i];
        ob[o++] = T[HA_AK_LIFTED];
        int64_t prog = st.progress_buf[env];
        ob[o++] = logf((float)prog / 10.0f + 1.0f);
        float succ = st.successes[env];
        ob[o++] = logf(succ + 1.0f);
        int o_rew = o;
        float reward = st.rew[env];
        if (!obs_only) {
            // _lifting_reward
            float z_lift = (0.05f + obj[2]) - p.ak_object_init[2];
            float lifting_rew = fminf(fmaxf(z_lift, 0.0f), 0.5f);
            bool was_lifted = T[HA_AK_LIFTED] != 0.0f;
            bool lifted = (z_lift > p.ak_lifting_bonus_threshold) || was_lifted;
            float lift_bonus_rew = (lifted && !was_lifted) ? p.ak_lifting_bonus : 0.0f;
            float not_lifted = lifted ? 0.0f : 1.0f, is_lifted = lifted ? 1.0f : 0.0f;
            lifting_rew = lifting_rew * not_lifted;
            T[HA_AK_LIFTED] = is_lifted;
            // _distance_delta_rewards
            float fdr = 0.0f;
            for (int i = 0; i < 4; i++) {
                float dlt = T[HA_AK_CLOSEST_FT + i] - curr[i];
                T[HA_AK_CLOSEST_FT + i] = fminf(T[HA_AK_CLOSEST_FT + i], curr[i]);
                fdr += fminf(fmaxf(dlt, 0.0f), 10.0f) * 1.0f;                     // finger_rew_coeffs
            }
            fdr = fdr * not_lifted;
            float hdf = T[HA_AK_FURTHEST] - curr[0];
            T[HA_AK_FURTHEST] = fmaxf(T[HA_AK_FURTHEST], curr[0]);
            float hdp = (fminf(fmaxf(hdf, -10.0f), 0.0f) * not_lifted) * 4.0f;
            // _keypoint_reward
            float mkd = T[HA_AK_CLOSEST_KP] - kmax;
            T[HA_AK_CLOSEST_KP] = fminf(T[HA_AK_CLOSEST_KP], kmax);
            float kr = fminf(fmaxf(mkd, 0.0f), 100.0f) * is_lifted;
            // successes
            bool near = kmax <= st.task_scalars[3];
            T[HA_AK_NEAR_GOAL] = T[HA_AK_NEAR_GOAL] + (near ? 1.0f : 0.0f);
            bool is_success = T[HA_AK_NEAR_GOAL] >= (float)p.ak_success_steps;
            succ = succ + (is_success ? 1.0f : 0.0f);
            float* ep = &T[HA_AK_REW_EP];
            ep[0] += fdr;
            ep[1] += hdp;
            ep[2] += lifting_rew;
            ep[3] += kr;
            fdr = fdr * p.ak_distance_delta_rew_scale;
            hdp = hdp * 0.0f;                                                     // currently disabled
            lifting_rew = lifting_rew * p.ak_lifting_rew_scale;
            kr = kr * p.ak_keypoint_rew_scale;
            float sa = 0.0f, sh = 0.0f;
            for (int d = 0; d < p.ak_num_arm_dofs; d++) sa += fabsf(in.qd[d]);
            for (int d = p.ak_num_arm_dofs; d < AK_ND; d++) sh += fabsf(in.qd[d]);
            float kap = -1.0f * (sa * p.ak_kuka_actions_penalty_scale);
            float aap = -1.0f * (sh * p.ak_allegro_actions_penalty_scale);
            float bonus = near ? p.ak_bonus_rew : 0.0f;
            reward = ((((((fdr + hdp) + lifting_rew) + lift_bonus_rew) + kr) + kap) + aap) + bonus;
            // _compute_resets (+ reorientation's _extra_reset_rules)
            int64_t resets = obj[2] < 0.1f ? 1 : st.reset_buf[env];
            if (p.ak_max_consecutive_successes > 0) {
                if (is_success) prog = 0;
                if (succ >= (float)p.ak_max_consecutive_successes) resets = 1;
            }
            if (prog >= (int64_t)p.max_episode_length - 1) resets = 1;
            if (p.ak_subtask == 1 && fmaxf(fmaxf(curr[0], curr[1]), fmaxf(curr[2], curr[3])) > 1.5f) resets = 1;
            // true objective (tolerance_successes_objective, allegro_kuka_utils.py:135-163)
            float tol_obj = st.task_scalars[1];
            T[HA_AK_TRUE_OBJ] = st.task_scalars[2] != 0.0f ? succ * 0.01f + tol_obj : succ + tol_obj;
            ep[4] += fdr;
            ep[5] += hdp;
            ep[6] += lifting_rew;
            ep[7] += lift_bonus_rew;
            ep[8] += kr;
            ep[9] += bonus;
            ep[10] += kap;
            ep[11] += aap;
            st.rew[env] = reward;
            st.reset_buf[env] = resets;
            st.reset_goal_buf[env] = is_success ? 1 : 0;
            st.progress_buf[env] = prog;
            st.successes[env] = succ;
            st.timeout_buf[env] = (prog >= (int64_t)p.max_episode_length - 1) && resets != 0;   // vec_task.py:424
            if (resets) {
                atomicAdd(&st.stats[0], 1);
                atomicAdd(&st.term_sums[0], succ);
            }
            if (is_success) atomicAdd(&st.stats[1], 1);
        }
        ob[o_rew] = reward * 0.01f;
        (void)D;
    }
    wsync();
    float clampv = p.ak_clamp_abs_obs;
    float* og = st.obs + (size_t)env * nobs;
    for (int k = lane; k < nobs; k += 64) {
        float v = ak.obs[k];
        if (clampv > 0.0f && !obs_only) v = fminf(fmaxf(v, -clampv), clampv);   // clamp_obs (post_physics_step)
        if (!obs_only) v = dr_obs(c, env, k, v);        // DR observation noise on obs_buf (vec_task.py:426-428)
        og[k] = v;
        obs_out_put(c, (size_t)env * nobs + k, v);
    }
    if (lane < AK_TS_KP) tsg[lane] = ak.ts[lane];
}
