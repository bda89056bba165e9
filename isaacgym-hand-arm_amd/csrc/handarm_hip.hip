// handarm_hip.hip - kernels and C ABI of libhandarm_hip.so (MI355X / gfx950).
//
// One 64-lane wavefront simulates one environment; a launch has one 64-thread workgroup per env,
// so a 8192-env shard is 8192 workgroups (32 per CU). Per-env state is staged in LDS (EnvLDS) for
// the whole env-step (all substeps) and written back once; the gym tensors keep the Isaac Gym
// env-major layouts so one env's slice is contiguous and its loads/stores are coalesced.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ak_task.h"
#include "ha_pointcloud.h"
#include "ha_camera.h"

#define HA_ND 17         /* Ur5Sih DOF count (UR5 + SIH); AH_ND = 16 (Allegro) */

enum { MODE_SIMULATE = 0, MODE_STEP = 1, MODE_OBSERVE = 2, MODE_RESET = 3 };

// Kernel families: one per task, plus the Ur5Sih clutter family (bin-picking, BASELINE config 5: up to 8
// objects, two contact chunks, a 65-coordinate velocity) that runs the same Ur5Sih task math. ha_create
// picks the family from the task and the object count.
#define FAM_UR5SIH_CLUTTER 3
template <int FAM>
__host__ __device__ constexpr int fam_task() { return FAM == FAM_UR5SIH_CLUTTER ? HA_TASK_UR5SIH : FAM; }
template <int FAM>
__host__ __device__ constexpr int task_nd() {
    return FAM == HA_TASK_ALLEGRO_HAND ? AH_ND : (FAM == HA_TASK_ALLEGRO_KUKA ? AK_ND : HA_ND);
}
// object slots in LDS per env (objects per env the family's kernels support)
template <int FAM>
__host__ __device__ constexpr int task_obj_capacity() {
    return FAM == FAM_UR5SIH_CLUTTER ? HA_MAX_OBJ : (FAM == HA_TASK_UR5SIH ? 3 : 1);
}
// contact chunks (MAXC contacts each). The clutter family holds 84 contacts per substep: a settled 8-object bin
// offers 59 on average and at most ~90 (bench contact_stats), 42 were at capacity in 99% of substeps.
#ifndef HB_CHUNKS
#define HB_CHUNKS 4
#endif
// clutter chunks whose object-block rows stay in LDS (0..4); the rest go to the env's global row area, which the
// PGS reads one contact ahead. 0: env block 16.8 KB, 9 workgroups per CU (1: 22.0 KB, 7 per CU): C5 shard
// 23.0 -> 19.5 ms (tools/ab_variants.sh binpick)
#ifndef HB_LDS_CHUNKS
#define HB_LDS_CHUNKS 0
#endif
// Ur5Sih (3 objects) and AllegroHand: overflow chunks (PhysCfg OVF). Chunk 0 keeps the one-chunk LDS layout (21 /
// 12 contacts); the further chunks' contact entries, rows and row constants live in the env's global area, touched
// only by substeps with more contacts than chunk 0 holds. Round 3 measured C4 over 21 contacts in 5.4% of the
// substeps of a whole episode (per-env maximum 57 at p99) and C3 over 12 in 3.2% (maximum 41)
#ifndef HA_CHUNKS
#define HA_CHUNKS 4
#endif
#ifndef HA_AH_CHUNKS
#define HA_AH_CHUNKS 4
#endif
// AllegroKuka: with the hand's self-collision (v12) a substep offers 12 contacts on average and up to ~50 under random
// actions; chunk 0 holds 21 in LDS, a second chunk in the env's global area takes the rest
#ifndef HA_AK_CHUNKS
#define HA_AK_CHUNKS 2
#endif
template <int FAM>
__host__ __device__ constexpr int task_contact_chunks() {
    return FAM == FAM_UR5SIH_CLUTTER ? HB_CHUNKS
           : (FAM == HA_TASK_UR5SIH ? HA_CHUNKS : (FAM == HA_TASK_ALLEGRO_HAND ? HA_AH_CHUNKS : HA_AK_CHUNKS));
}
template <int FAM>
__host__ __device__ constexpr bool task_overflow() { return FAM != FAM_UR5SIH_CLUTTER; }
// persistent contact manifolds (v13) are compiled into every family but AllegroHand: with them its kernel needs 76 B/lane
// of register spills (44 without) and measured 4.8 -> 5.0 ms per C3 step with twice the HBM traffic; its hand closes on
// the cube and on itself every step, so few of its pairs keep a record long enough to pay back
template <int FAM>
__host__ __device__ constexpr bool task_pcm() { return FAM != HA_TASK_ALLEGRO_HAND; }
static inline bool family_pcm(int fam) { return fam != HA_TASK_ALLEGRO_HAND; }
// clutter family: 1 recomputes the object blocks of the contact rows in registers from the contact entries in the
// rows phase and at every PGS fetch (PhysCfg RC) instead of storing them in the env's global row area. Measured on
// C5 (round 3): 22.1 -> 30.8 ms per step, the ~140 VALU per fetch cost more than the stored rows' traffic, which the
// one-contact-ahead prefetch hides; the product keeps the stored rows
#ifndef HB_RECOMPUTE
#define HB_RECOMPUTE 0
#endif
// clutter family: the contacts that touch no robot link are solved in packed passes (four contacts on disjoint objects
// per pass, one per 16-lane row) instead of one whole-wave contact block after another (PhysCfg PACK);
// the oracle follows the same order for the configurations this family runs (physics_oracle.c packed_pgs)
#ifndef HB_PACKED_PGS
#define HB_PACKED_PGS 1
#endif
// the Ur5Sih 3-object family can pack the substeps whose contacts fit chunk 0 (<= 21: rows in LDS, the constants per
// contact in PK, the rest serial over the overflow chunks): measured off. Three objects give passes of at most three
// contacts, a bench env offers ~12 of which ~4 objects' worth share an object, so a sweep still runs ~4-5 passes of
// ~2-3 contacts, each slower than the serial block it replaces: C4 shard 3.14 -> 3.60 ms per step (r5j-r5p,
// bit-identical; with lane-permuted constants 3.69 ms). A -DHA_PACKED_PGS=1 build needs the oracle's h->packed = 1
#ifndef HA_PACKED_PGS
#define HA_PACKED_PGS 0
#endif
// clutter family: link contacts whose robot blocks stay in LDS (the rest use the global spill rows). 2 slots
// keep the env block at <= 20 KB, i.e. 8 workgroups per CU (8 slots: 22.8 KB, 7 per CU)
#ifndef HB_LINK_SLOTS
#define HB_LINK_SLOTS 2
#endif
// the Ur5Sih 3-object family's LDS link slots (split rows, HA_SPLIT_ABOVE_OCAP): 4 put the env block at 13.5 KB,
// 12 workgroups per CU (8 slots: 15.1 KB, 10 per CU): C4 shard 5.24 -> 5.01 ms; more link contacts use the
// global spill rows (tests/test_gpu_parity.py::test_link_contacts_spill_rows_match_oracle)
#ifndef HA_LINK_SLOTS
#define HA_LINK_SLOTS 4
#endif
// minimum waves per SIMD asked of the Ur5Sih (3-object) kernels' register allocation: 3 (<= 168 VGPRs; 149
// without spills now) so the VGPRs allow the 12 workgroups per CU the LDS does
#ifndef HA_WAVES_PER_EU
#define HA_WAVES_PER_EU 3
#endif
// AllegroKuka / AllegroHand (one dense chunk): contacts per substep, and waves per SIMD asked of their
// register allocation. 12 contacts put the env block at 13.6 KB of LDS and 3 waves per SIMD cap the kernels at
// 168 VGPRs (84 / 72 B/lane scratch), so 12 workgroups run per CU instead of 8 (LDS 20.1 / 16.6 KB, 193
// VGPRs): C2 0.705 -> 0.652 ms, C3 3.23 -> 2.70 ms (tools/ab_variants.sh). The list is then over capacity in
// 1.3% (C2) / 2.0% (C3) of substeps, where the shallowest contacts give way (bench contact_stats).
// AllegroKuka holds a full chunk (21) since round 3: with 2 LDS link slots its rows still fit in front of S in the
// phase union (9.3 KB env block, 16 workgroups per CU); C2 over capacity 1.3% -> 0.09% of substeps for +2.7%
// step time. AllegroHand stays at 12: 21 in the compact layout cost +9% (0.12%), the dense rows do not fit.
// Waves per SIMD: AllegroKuka asks for 3 since round 5 (168 VGPRs, 8 B/lane scratch): with the self pass and the
// persistent manifolds it needed 120 B/lane of spills at 4, whose scratch write-backs were 43% of its HBM traffic
// (48.8 -> 27.8 KB per env) and cost more than the fourth wave won (C2 kernel 1.064 -> 1.043 ms,
// tools/diag/ab_traffic.sh); AllegroHand stays at 4 (16384 envs: the fourth wave per SIMD is worth 10% there).
#ifndef HA_AK_CONTACTS
#define HA_AK_CONTACTS 21
#endif
#ifndef HA_AH_CONTACTS
#define HA_AH_CONTACTS 12
#endif
#ifndef HA_AK_WAVES_PER_EU
#define HA_AK_WAVES_PER_EU 3
#endif
#ifndef HA_AH_WAVES_PER_EU
#define HA_AH_WAVES_PER_EU 4
#endif
template <int FAM>
__host__ __device__ constexpr int task_chunk_capacity() {
    return FAM == HA_TASK_ALLEGRO_KUKA ? HA_AK_CONTACTS : (FAM == HA_TASK_ALLEGRO_HAND ? HA_AH_CONTACTS : MAXC);
}
#ifndef HB_WAVES_PER_EU
#define HB_WAVES_PER_EU 3
#endif
template <int FAM>
__host__ __device__ constexpr int task_waves_per_eu() {
    return FAM == HA_TASK_UR5SIH ? HA_WAVES_PER_EU
           : (FAM == HA_TASK_ALLEGRO_KUKA ? HA_AK_WAVES_PER_EU
                                          : (FAM == HA_TASK_ALLEGRO_HAND ? HA_AH_WAVES_PER_EU : HB_WAVES_PER_EU));
}
// largest hull a family's narrow-phase scratch holds: the YCB pool hulls have up to 64 vertices and 124 face
// planes; the Allegro scenes' hulls (cooked to <= 32 vertices, <= 60 planes) take half, which puts the
// AllegroHand env block at 10.2 KB: 16 workgroups per CU with 4 waves per SIMD
template <int FAM>
__host__ __device__ constexpr int task_col_verts() { return (FAM == HA_TASK_ALLEGRO_KUKA || FAM == HA_TASK_ALLEGRO_HAND) ? 32 : 64; }
template <int FAM>
__host__ __device__ constexpr int task_col_planes() { return (FAM == HA_TASK_ALLEGRO_KUKA || FAM == HA_TASK_ALLEGRO_HAND) ? 64 : 124; }
// AllegroKuka env block (PhysCfg SPLIT / NG / MU): split rows with HA_AK_LINK_SLOTS link contacts in LDS, no
// compound-object gather buffer (its one object is a cuboid; ha_create enforces one hull per pool object) and
// S ~ M^-1 inside the phase union: 13.3 -> 9.1 KB, so 16 workgroups per CU hold the 4096 envs of config C2 in
// one round (12 per CU ran them in 1.33 rounds). HA_AK_COMPACT=0 restores the round-2 layout (A/B timing).
#ifndef HA_AK_COMPACT
#define HA_AK_COMPACT 1
#endif
// (3 in round 4: with the hand's self contacts most contacts touch links. 9 since round 5: at 3 waves per SIMD the
// CU holds 12 workgroups, so the LDS may grow to 13.3 KB per env (552 B per slot; 9 is the most that keeps 12 per CU).
// A/B on C2 (profiles/README.md): 3 slots 1.037 ms / 27.8 KB HBM per env, 6 slots 1.018 ms / 20.5 KB, 9 slots
// 1.015 ms / 14.5 KB)
#ifndef HA_AK_LINK_SLOTS
#define HA_AK_LINK_SLOTS 9
#endif
// AllegroHand in the same compact layout (split rows, no gather buffer, S in the union): every AllegroHand contact
// touches a finger link, so its rows are robot blocks in HA_AH_LINK_SLOTS LDS slots and the global spill rows
#ifndef HA_AH_COMPACT
#define HA_AH_COMPACT 0
#endif
#ifndef HA_AH_LINK_SLOTS
#define HA_AH_LINK_SLOTS 5
#endif
template <int FAM>
__host__ __device__ constexpr bool task_compact() {
    return (FAM == HA_TASK_ALLEGRO_KUKA && HA_AK_COMPACT) || (FAM == HA_TASK_ALLEGRO_HAND && HA_AH_COMPACT);
}
template <int FAM>
__host__ __device__ constexpr int task_link_slots() {
    return FAM == FAM_UR5SIH_CLUTTER ? HB_LINK_SLOTS
                                     : (!task_compact<FAM>() ? HA_LINK_SLOTS
                                                              : (FAM == HA_TASK_ALLEGRO_KUKA ? HA_AK_LINK_SLOTS : HA_AH_LINK_SLOTS));
}
template <int FAM>
using FamPhys = PhysCfg<task_nd<FAM>(), task_obj_capacity<FAM>(), task_contact_chunks<FAM>(), task_link_slots<FAM>(),
                        FAM == FAM_UR5SIH_CLUTTER ? HB_LDS_CHUNKS : task_contact_chunks<FAM>(),
                        task_chunk_capacity<FAM>(), task_col_verts<FAM>(), task_col_planes<FAM>(),
                        task_compact<FAM>() ? 1 : -1, task_compact<FAM>() ? 0 : HA_MAX_GATHER, task_compact<FAM>(),
                        FAM == FAM_UR5SIH_CLUTTER && HB_RECOMPUTE, task_overflow<FAM>(),
#ifdef HA_X_NO_SELF     /* A/B timing builds only: the Allegro families without their self-collision pass */
                        false,
#else
                        FAM == HA_TASK_ALLEGRO_HAND || FAM == HA_TASK_ALLEGRO_KUKA,
#endif
                        (FAM == FAM_UR5SIH_CLUTTER && HB_PACKED_PGS) || (FAM == HA_TASK_UR5SIH && HA_PACKED_PGS)>;


// ----------------------------------------------------------------------------- state load/store
// Generic over the env layout in ha_model_t (actor / rigid-body creation order of the task).
// take_force: consume st.object_force (ha_simulate = gym.simulate after apply_rigid_body_force_tensors)
__device__ __forceinline__ void load_env(SimCtx& c, const ha_state_t& st, int env, bool take_force = false) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, NO = c.NO, A = m.n_actors;
    if (lane < D) {
        s.q[lane] = st.dof_state[((size_t)env * D + lane) * 2];
        s.qd[lane] = st.dof_state[((size_t)env * D + lane) * 2 + 1];
        s.tgt[lane] = st.sim_targets[(size_t)env * D + lane];
        s.u.pd.dforce[lane] = 0.0f;
    }
    if (lane < NO) {
        int o = lane;
        const float* r = st.root_state + ((size_t)env * A + m.actor_object0 + o) * 13;
        int pid = (int)st.object_indices[(size_t)env * NO + o];
        c.o[o].pool = pid;
        dr_object_scale(c, st, env, o);         // object_scale row x the DR actor scale (ha_dr.h)
        c.o[o].ofx[0] = c.o[o].ofx[1] = c.o[o].ofx[2] = c.o[o].ofx[3] = 0.0f;
        c.o[o].otq[0] = c.o[o].otq[1] = c.o[o].otq[2] = 0.0f;
        if (take_force && st.object_force) {
            float* fo = st.object_force + ((size_t)env * NO + o) * 3;
            c.o[o].ofx[0] = fo[0]; c.o[o].ofx[1] = fo[1]; c.o[o].ofx[2] = fo[2];
            fo[0] = fo[1] = fo[2] = 0.0f;
        }
        if (take_force && st.object_torque) {
            float* tq = st.object_torque + ((size_t)env * NO + o) * 3;
            c.o[o].otq[0] = tq[0]; c.o[o].otq[1] = tq[1]; c.o[o].otq[2] = tq[2];
            tq[0] = tq[1] = tq[2] = 0.0f;
        }
        qf q = ldq(r + 3);
        stq(c.o[o].oq, q);
        st3(c.o[o].oc, ld3(r) + qrot(q, scale3(c, o, ld3(m.pool_com[pid]))));
        st3(c.o[o].ov, ld3(r + 7));
        st3(c.o[o].ow, ld3(r + 10));
        c.o[o].coll = st.collision_enabled ? st.collision_enabled[(size_t)env * NO + o] : 1;
    }
    for (int b = lane; b < MAXB; b += 64) s.u.pd.cforce[b][0] = s.u.pd.cforce[b][1] = s.u.pd.cforce[b][2] = 0.0f;
    if (lane < HA_CSTAT) s.cst[lane] = 0;
    if (m.posed_actor >= 0 && lane < 8)          // the actor carrying posed statics (v14): p[3], pad, q[4]
        s.sb[lane] = lane == 3 ? 0.0f : st.root_state[((size_t)env * A + m.posed_actor) * 13 + (lane < 3 ? lane : lane - 1)];
    wsync();
}

// link twists into s.u.pd.Vl (level-synchronous); needs fk()
__device__ __forceinline__ void link_twists(SimCtx& c) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, L = c.L;
    if (lane == 0) for (int k = 0; k < 6; k++) s.u.pd.Vl[0][k] = 0.f;
    wsync();
    for (int lev = 1; lev <= m.max_level; lev++) {
        if (lane < L && m.link_level[lane] == lev) {
            int i = lane, par = m.link_parent[i], d = m.link_dof[i];
            f3 vw = ld3(&s.u.pd.Vl[par][0]), vv = ld3(&s.u.pd.Vl[par][3]);
            if (d >= 0) {
                f3 axd = ld3(s.ax[d]);
                vw = vw + axd * s.qd[d];
                vv = vv + cross3(ld3(s.an[d]), axd) * s.qd[d];
            }
            st3(&s.u.pd.Vl[i][0], vw);
            st3(&s.u.pd.Vl[i][3], vv);
        }
        wsync();
    }
}

// rigid-body row k (13 floats: pos, quat, COM linvel, angvel) of robot link i from LDS
__device__ float link_state(const SimCtx& c, int i, int k) {
    const EnvLDS& s = *c.s;
    if (k < 3) return s.lp[i][k];
    if (k < 7) return s.lq[i][k - 3];
    if (k < 10) {
        f3 cc = ld3(s.lp[i]) + qrot(ldq(s.lq[i]), ld3(c.m->link_com[i]));
        f3 lin = ld3(&s.u.pd.Vl[i][3]) + cross3(ld3(&s.u.pd.Vl[i][0]), cc);
        return k == 7 ? lin.x : (k == 8 ? lin.y : lin.z);
    }
    return s.u.pd.Vl[i][k - 10];        // angular velocity: Vl = (w, v at the world origin)
}
// root-state row k of object o (origin pose, not COM) from LDS
__device__ float object_state(const SimCtx& c, int o, int k) {
    const EnvLDS& s = *c.s;
    if (k < 3) {
        f3 pos = ld3(c.o[o].oc) - qrot(ldq(c.o[o].oq), scale3(c, o, ld3(c.m->pool_com[c.o[o].pool])));
        return k == 0 ? pos.x : (k == 1 ? pos.y : pos.z);
    }
    if (k < 7) return c.o[o].oq[k - 3];
    if (k < 10) return c.o[o].ov[k - 7];
    return c.o[o].ow[k - 10];
}

// writes dof_state, dof_force, sim targets, object root states, rigid_body_state and net_contact_force
// (the refresh_* tensors). Leaves the link twists in s.u.pd.Vl for the task's observation snapshot.
__device__ __forceinline__ void store_env(SimCtx& c, const ha_state_t& st, int env) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, NO = c.NO, A = m.n_actors, L = c.L, B = m.n_bodies;
    fk(c);
    link_twists(c);
    if (lane < D) {
        st.dof_state[((size_t)env * D + lane) * 2] = s.q[lane];
        st.dof_state[((size_t)env * D + lane) * 2 + 1] = s.qd[lane];
        st.sim_targets[(size_t)env * D + lane] = s.tgt[lane];
        if (st.dof_force) st.dof_force[(size_t)env * D + lane] = s.u.pd.dforce[lane];
    }
    for (int e = lane; e < NO * 13; e += 64)
        st.root_state[((size_t)env * A + m.actor_object0 + e / 13) * 13 + e % 13] = object_state(c, e / 13, e % 13);
    wsync();
    float* bs = st.rigid_body_state + (size_t)env * B * 13;
    const float* rs = st.root_state + (size_t)env * A * 13;
    for (int e = lane; e < B * 13; e += 64) {
        int b = e / 13, k = e % 13;
        float v;
        if (b >= m.body_robot0 && b < m.body_robot0 + L) v = link_state(c, b - m.body_robot0, k);
        else if (b >= m.body_object0 && b < m.body_object0 + NO) v = object_state(c, b - m.body_object0, k);
        else if (b == m.body_goal) v = rs[m.actor_goal * 13 + k];
        else if (b >= m.body_fixed0 && b < m.body_fixed0 + m.n_fixed_bodies) v = k < 7 ? m.body_fixed_pose[b - m.body_fixed0][k] : 0.0f;
        else v = rs[m.actor_table * 13 + k];
        bs[e] = v;
    }
    for (int e = lane; e < B * 3; e += 64) st.net_contact_force[(size_t)env * B * 3 + e] = s.u.pd.cforce[e / 3][e % 3];
    if (st.contact_stats && lane < HA_CSTAT) {
        int32_t* cs = st.contact_stats + (size_t)env * HA_CSTAT + lane;
        *cs = lane == 2 ? (s.cst[2] > *cs ? s.cst[2] : *cs) : *cs + s.cst[lane];
    }
    wsync();
}

// Ur5Sih observation snapshot (what the observables read after refresh_*): from the LDS state after
// store_env (same final kinematics)
__device__ __forceinline__ void ur5sih_obs_in(SimCtx& c, ObsIn* in) {
    EnvLDS& s = *c.s;
    int lane = c.lane, D = c.D, NO = c.NO;
    if (lane < 7) in->flange[lane] = lane < 3 ? s.lp[LINK_FLANGE][lane] : s.lq[LINK_FLANGE][lane - 3];
    if (lane < 50) {
        int t = lane / 10, k = lane % 10;
        in->tip[t][k] = link_state(c, c_tip_links[t], k);
    }
    if (lane < D) in->dofpos[lane] = s.q[lane];
    for (int e = lane; e < NO * 13; e += 64) in->obj[e / 13][e % 13] = object_state(c, e / 13, e % 13);
    wsync();
}

// observation snapshot straight from the (refreshed) state tensors
__device__ void snapshot_from_tensors(SimCtx& c, const ha_state_t& st, int env, ObsIn* in) {
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, NO = c.NO, A = m.n_actors, B = m.n_bodies, R0 = m.body_robot0;
    const float* bs = st.rigid_body_state + (size_t)env * B * 13;
    if (lane < 7) in->flange[lane] = bs[(R0 + LINK_FLANGE) * 13 + lane];
    if (lane < 50) {
        int t = lane / 10, k = lane % 10;
        in->tip[t][k] = bs[(R0 + c_tip_links[t]) * 13 + k];
    }
    if (lane < D) in->dofpos[lane] = st.dof_state[((size_t)env * D + lane) * 2];
    for (int e = lane; e < NO * 13; e += 64)
        in->obj[e / 13][e % 13] = st.root_state[((size_t)env * A + m.actor_object0) * 13 + e];
    if (lane < NO) c.o[lane].pool = (int)st.object_indices[(size_t)env * NO + lane];
    wsync();
}

// always inlined: as an outlined call (the inliner's choice once it grows past its threshold) the step runs
// ~40% slower (call ABI: stack spills, no cross-phase register allocation)
template <class PC>
// n_calls gym.simulate calls. An applied object force (ha_state_t.object_force for ha_simulate, the tasks' random
// forces) lasts one call: apply_rigid_body_force_tensors acts on the next simulate (the oracle's simulate_env alike)
__device__ __forceinline__ void run_physics(SimCtx& c, int n_calls) {
    float hdt = c.p->dt / (float)c.p->substeps;
    for (int k = 0; k < n_calls; k++) {
        for (int sub = 0; sub < c.p->substeps; sub++) substep<PC>(c, hdt);
        if (c.lane < c.NO) {
            c.o[c.lane].ofx[0] = c.o[c.lane].ofx[1] = c.o[c.lane].ofx[2] = 0.0f;
            c.o[c.lane].otq[0] = c.o[c.lane].otq[1] = c.o[c.lane].otq[2] = 0.0f;
        }
        wsync();
    }
}

// AllegroHand observation staging
__device__ __forceinline__ void ah_in_from_lds(SimCtx& c, AhIn* in) {
    EnvLDS& s = *c.s;
    int lane = c.lane, D = c.D;
    if (lane < D) {
        in->q[lane] = s.q[lane];
        in->qd[lane] = s.qd[lane];
        in->f[lane] = s.u.pd.dforce[lane];
    }
    if (lane < 13) in->obj[lane] = object_state(c, 0, lane);
    wsync();
}
__device__ void ah_in_from_tensors(SimCtx& c, const ha_state_t& st, int env, AhIn* in) {
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D;
    if (lane < D) {
        in->q[lane] = st.dof_state[((size_t)env * D + lane) * 2];
        in->qd[lane] = st.dof_state[((size_t)env * D + lane) * 2 + 1];
        in->f[lane] = st.dof_force[(size_t)env * D + lane];
    }
    if (lane < 13) in->obj[lane] = st.root_state[((size_t)env * m.n_actors + m.actor_object0) * 13 + lane];
    wsync();
}

// AllegroKuka observation staging (palm = iiwa7_link_7, fingertips = *_link_3)
__device__ __forceinline__ void ak_in_from_lds(SimCtx& c, AkIn* in) {
    EnvLDS& s = *c.s;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    if (lane < D) {
        in->q[lane] = s.q[lane];
        in->qd[lane] = s.qd[lane];
    }
    if (lane < 13) {
        in->palm[lane] = link_state(c, p.ak_palm_link, lane);
        in->obj[lane] = object_state(c, 0, lane);
    }
    if (lane < 28) in->tip[lane / 7][lane % 7] = link_state(c, p.ak_fingertip_links[lane / 7], lane % 7);
    wsync();
}
__device__ void ak_in_from_tensors(SimCtx& c, const ha_state_t& st, int env, AkIn* in) {
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D;
    const float* bs = st.rigid_body_state + (size_t)env * m.n_bodies * 13;
    if (lane < D) {
        in->q[lane] = st.dof_state[((size_t)env * D + lane) * 2];
        in->qd[lane] = st.dof_state[((size_t)env * D + lane) * 2 + 1];
    }
    if (lane < 13) {
        in->palm[lane] = bs[(m.body_robot0 + p.ak_palm_link) * 13 + lane];
        in->obj[lane] = st.root_state[((size_t)env * m.n_actors + m.actor_object0) * 13 + lane];
    }
    if (lane < 28) in->tip[lane / 7][lane % 7] = bs[(m.body_robot0 + p.ak_fingertip_links[lane / 7]) * 13 + lane % 7];
    wsync();
}
static_assert(sizeof(AkPost) <= sizeof(PostScratch) - offsetof(PostScratch, in), "AkPost must fit after pd.dyn");
static_assert(HA_ND + 6 * HA_MAX_OBJ <= MAXV, "bin-picking (8 objects) must fit the generalized velocity (MAXV)");

// ----------------------------------------------------------------------------- the kernels
// One kernel per (task, mode) (one workgroup = one wavefront = one env): each is compiled with only its
// own path, which keeps every kernel's code small, gives the DOF count to the compiler as a constant, and
// gives the profiler a distinct name per kernel.
// After the physics the env index and lane id are re-derived through an opaque move, so the per-lane 64-bit
// tensor addresses load_env computed are recomputed by store_env / the task epilogue instead of being kept
// live (spilled to scratch: 8 B per lane each) across the whole physics
__device__ __forceinline__ void after_physics(SimCtx& c, int& env) {
    asm volatile("" : "+s"(env));
    asm volatile("" : "+v"(c.lane));
}

// VecTask.step's head and tail inside the step launch (ha_task_step_io, the Allegro families); all null: the plain step.
// act_in: the caller's raw actions, clamped to +-clip_act where the task reads them and stored clamped into the
// actions tensor (vec_task.py:400-404); obs_out: clamp(obs, +-clip_obs), the fresh obs_dict["obs"] (vec_task.py:437);
// scalars: AllegroKuka's extras means (allegro_kuka_base.py:908-917) by the last workgroups (ak_extras)
struct StepIO {
    const float* act_in;
    float* obs_out;
    float* scalars;
    float* partials;        // 4 floats per group of 64 envs
    int32_t* counters;      // per group, then one for the groups; zero between launches
    float clip_act, clip_obs;
    // ha_set_order_cost(h, 1): each env's workgroup start and end in this launch (100 MHz clock) for the
    // dispatch-order refresh (null: off)
    unsigned long long* tstart;
    unsigned long long* tend;
};

// AllegroKuka extras: mean prev_episode_successes, mean / min / max true_objective over the shard, in the step launch.
// Each env's workgroup publishes its task_state (ak_post) and counts itself into its group of 64 envs; the group's
// last workgroup reduces the group (lane = env, fixed DPP tree) into a partial and counts the group in; the last group
// reduces the partials (lane l: groups l, l + 64, ... in order, then the same tree). Fixed order: deterministic.
__device__ __forceinline__ void ak_extras(const SimCtx& c, const ha_state_t& S, int env, const StepIO& io, int N) {
    int lane = c.lane;
    int g = env >> 6, G = (N + 63) >> 6;
    int gsize = N - 64 * g < 64 ? N - 64 * g : 64;
    __threadfence();
    int last = 0;
    if (lane == 0) last = atomicAdd(&io.counters[g], 1) == gsize - 1 ? 1 : 0;
    if (!__builtin_amdgcn_readfirstlane(last)) return;
    __threadfence();
    float ps = 0.0f, to = 0.0f, mn = 3.0e38f, mx = -3.0e38f;
    if (lane < gsize) {
        const float* t = S.task_state + (size_t)(64 * g + lane) * HA_AK_TS;
        ps = t[HA_AK_PREV_SUCC];
        to = t[HA_AK_TRUE_OBJ];
        mn = to;
        mx = to;
    }
    ps = wave_sum_rows(ps); to = wave_sum_rows(to); mn = wave_min(mn); mx = wave_max(mx);
    if (lane == 0) {
        float* q = io.partials + 4 * g;
        q[0] = ps; q[1] = to; q[2] = mn; q[3] = mx;
        io.counters[g] = 0;
    }
    __threadfence();
    last = 0;
    if (lane == 0) last = atomicAdd(&io.counters[G], 1) == G - 1 ? 1 : 0;
    if (!__builtin_amdgcn_readfirstlane(last)) return;
    __threadfence();
    float a0 = 0.0f, a1 = 0.0f, a2 = 3.0e38f, a3 = -3.0e38f;
    for (int q = lane; q < G; q += 64) {
        const float* r = io.partials + 4 * q;
        a0 += r[0]; a1 += r[1]; a2 = fminf(a2, r[2]); a3 = fmaxf(a3, r[3]);
    }
    a0 = wave_sum_rows(a0); a1 = wave_sum_rows(a1); a2 = wave_min(a2); a3 = wave_max(a3);
    if (lane == 0) {
        io.scalars[0] = a0 / (float)N;
        io.scalars[1] = a1 / (float)N;
        io.scalars[2] = a2;
        io.scalars[3] = a3;
        io.counters[G] = 0;
    }
}

template <int FAM, int MODE>
__device__ __forceinline__ void env_body(const ha_model_t* __restrict__ model, const ha_params_t* __restrict__ params,
                                         const ha_state_t& st, int num_envs, int n_calls, uint32_t flags,
                                         int stat_slot, float* __restrict__ spill,
                                         const int32_t* __restrict__ env_ids, const StepIO& io) {
    constexpr int TASK = fam_task<FAM>();
    constexpr int ND = task_nd<FAM>();
    constexpr int NCH = task_contact_chunks<FAM>();
    using PC = FamPhys<FAM>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // one workgroup per env; ha_simulate_envs launches one per listed env
    int env = env_ids ? env_ids[blockIdx.x] : (int)blockIdx.x;
    if (env < 0 || env >= num_envs) return;
    SimCtx c;
    c.gather = false;
#ifdef HA_AB_TIMING
    c.dry = false;
#endif
    c.m = model;
    c.p = params;
    c.s = reinterpret_cast<EnvLDS*>(smem);
    c.Minv = reinterpret_cast<float*>(smem + minv_lds_offset<PC>());
    c.col = col_view<PC>(&c.s->u);
    c.o = reinterpret_cast<ObjLDS*>(smem + obj_lds_offset<PC>());
    c.k = reinterpret_cast<ContactLDS*>(smem + contact_lds_offset<PC>());
    c.spill = (PC::split || PC::ovf || PC::selfc) ? spill + (size_t)env * PC::spill_floats : nullptr;
    c.selfc = PC::selfc ? reinterpret_cast<uint8_t*>(c.spill + PC::off_selfc) : nullptr;
    // separating-face records of the broad phase's pairs: the clutter family only. There most candidate object pairs in
    // the bin are apart (5.8 narrow phases a substep, 0.2 with contacts) and each needs a fresh hull setup; with the
    // records 4.8 of them are skipped (narrow phases 13.8% -> 2.2% of the substep, checks 5.9%). In the Allegro
    // families the separated pairs are link hulls against the cube, whose side is cached across consecutive pairs so
    // the narrow phase's sphere cull is cheaper than a record check (C3: checks 6.8% for 3.5% saved), and the record
    // register cost spills (tools/phase_profile.py, r5l)
    c.pairf = (c.spill && FAM == FAM_UR5SIH_CLUTTER) ? reinterpret_cast<uint8_t*>(c.spill + PC::off_pairf) : nullptr;
#ifdef HA_X_NO_PAIRF    /* A/B builds only: no separating-face records for the broad phase's pairs */
    c.pairf = nullptr;
#endif
    c.selfm = PC::selfc ? reinterpret_cast<uint32_t*>(smem + selfm_lds_offset<PC>()) : nullptr;
    c.sepf = 0xFF;
    // persistent contact manifolds (ha_params_t v13): the env's records, when the caller bound the buffer and the
    // tolerance is on; slots = detect's pairs (per object: ground, statics, later objects, link hulls; link hulls x
    // statics) + the self pairs (ha_contact_cache_slots)
    {
        int NO = params->n_objects, NS = model->n_static, NLH = model->n_link_hulls;
        size_t slots = (size_t)NO * (1 + NS + NLH) + (size_t)(NO * (NO - 1) / 2) + (size_t)NLH * NS + model->n_self_pairs;
        c.pcm = (st.contact_cache && params->pcm_lin_tol > 0.0f) ? st.contact_cache + (size_t)env * slots * HA_PCM_REC
                                                                   : nullptr;
    }
    if constexpr (!task_pcm<FAM>()) c.pcm = nullptr;
#ifdef HA_X_NO_PCM     /* A/B builds only: the persistent-manifold code compiled out */
    c.pcm = nullptr;
#endif
    c.pslot = -1;
    c.pkind = c.pA = c.pB = 0;
    c.pemit = 0;
#ifdef HA_PROFILE
    c.pcls = 0;
#endif
    c.act_in = MODE == MODE_STEP ? io.act_in : nullptr;
    c.obs_out = MODE == MODE_STEP ? io.obs_out : nullptr;
    c.clip_act = io.clip_act;
    c.clip_obs = io.clip_obs;
    c.maxc = PC::cap * NCH;
    // overflow chunks: contact entries past chunk 0 in the env's global area (null otherwise: ct_global folds away)
    c.kg = PC::ovf ? reinterpret_cast<ContactLDS*>(c.spill + PC::off_ct) : nullptr;
    c.kc0 = PC::ovf ? PC::cap : PC::cap * NCH;
    c.lane = threadIdx.x;
    c.D = ND;                     // == model->n_dofs (ha_create); a constant, so loops over D unroll
    c.NO = params->n_objects;
    c.L = model->n_links;
    c.dr = (params->dr_enable && st.dr_scale) ? st.dr_scale + (size_t)env * HA_DR_SIZE : nullptr;
    // v16: the shard-wide DR state (ha_dr_global_kernel ran before this launch); with it the per-env sampling, the
    // noise and the randomized gravity are on
    c.drg = (c.dr && st.dr_global) ? st.dr_global : nullptr;
    ObsIn& in = c.s->u.pd.in;
    AhIn& ain = *reinterpret_cast<AhIn*>(&c.s->u.pd.in);
    AkPost& akp = *reinterpret_cast<AkPost*>(&c.s->u.pd.in);
    ha_state_t S = st;
    if (MODE == MODE_STEP || MODE == MODE_OBSERVE) {
        S.stats = st.stats + stat_slot * HA_STAT_SIZE;
        S.term_sums = st.term_sums + stat_slot * 4;
    }
    if (MODE == MODE_STEP && env == 0) {
        // MODE_STEP: n_calls = the stats-ring slot of the NEXT step, cleared here (this launch only adds into
        // stat_slot; the next step's launch runs after this one on the stream), so no memset per step
        if (c.lane < HA_STAT_SIZE) st.stats[n_calls * HA_STAT_SIZE + c.lane] = 0;
        if (c.lane < 4) st.term_sums[n_calls * 4 + c.lane] = 0.0f;
    }
    if (MODE == MODE_OBSERVE) {
        if (TASK == HA_TASK_ALLEGRO_KUKA) {
            ak_in_from_tensors(c, S, env, &akp.in);
            ak_post(c, S, env, akp, (flags & HA_FLAG_OBS_ONLY) != 0);
        } else if (TASK == HA_TASK_ALLEGRO_HAND) {
            ah_in_from_tensors(c, S, env, &ain);
            ah_post(c, S, env, ain, (flags & HA_FLAG_OBS_ONLY) != 0);
        } else {
            snapshot_from_tensors(c, S, env, &in);
            post_step(c, S, env, in, (flags & HA_FLAG_OBS_ONLY) != 0);
        }
        return;
    }
    load_env(c, S, env, MODE == MODE_SIMULATE);
    if (MODE == MODE_SIMULATE) {
        run_physics<PC>(c, n_calls);
        after_physics(c, env);
        store_env(c, S, env);
        return;
    }
    // apply_randomizations' per-env part (ha_dr.h) before the task's resets; the Ur5Sih reset launch resets every env
    if (c.drg) dr_env_pre(c, S, env, (MODE == MODE_RESET && TASK == HA_TASK_UR5SIH) || S.reset_buf[env] != 0,
                          MODE == MODE_STEP);
    if (TASK == HA_TASK_ALLEGRO_KUKA) {
        // pre_physics_step (allegro_kuka_base.py:1355-1424). Lane k holds task_state field k in tsv; it goes
        // back to HBM before the physics (whose LDS union overwrites everything) and ak_post reloads it.
        float* tsg = S.task_state + (size_t)env * HA_AK_TS;
        float tsv = c.lane < HA_AK_TS ? tsg[c.lane] : 0.0f;
        bool goal = S.reset_goal_buf[env] != 0, full = S.reset_buf[env] != 0;
        if (goal || full) ak_reset(c, S, env, flags, goal, full, tsv);
        if (MODE == MODE_RESET) {
            if (c.lane < AK_TS_KP) tsg[c.lane] = tsv;
            store_env(c, S, env);
            return;
        }
        ak_controller(c, S, env);
        ak_forces(c, S, env, flags, tsv);
        if (c.lane < AK_TS_KP) tsg[c.lane] = tsv;
        if (!(flags & HA_FLAG_NO_PHYSICS)) run_physics<PC>(c, c.p->control_freq_inv);   // vec_task.py:409-412
        after_physics(c, env);
        store_env(c, S, env);
        if (c.lane == 0) S.progress_buf[env] = S.progress_buf[env] + 1;                // allegro_kuka_base.py:1429
        ak_in_from_lds(c, &akp.in);
        ak_post(c, S, env, akp, false);
        if (MODE == MODE_STEP && io.scalars) ak_extras(c, S, env, io, num_envs);
        return;
    }
    if (TASK == HA_TASK_ALLEGRO_HAND) {
        // pre_physics_step (allegro_hand.py:586-625): goal / env resets, targets from the actions, random forces.
        // Lane k holds task_state field k (AH_TS_*) in tsv
        float* tsg = S.task_state ? S.task_state + (size_t)env * HA_AK_TS : nullptr;
        float tsv = (tsg && c.lane < AH_TS_N) ? tsg[c.lane] : 0.0f;
        bool goal = S.reset_goal_buf[env] != 0, full = S.reset_buf[env] != 0;
        if (goal || full) ah_reset(c, S, env, flags, goal, full, tsv);
        if (MODE == MODE_RESET) {
            if (tsg && c.lane < AH_TS_N) tsg[c.lane] = tsv;
            store_env(c, S, env);
            return;
        }
        ah_controller(c, S, env);
        ah_forces(c, S, env, flags, tsv);
        if (tsg && c.lane < AH_TS_N) tsg[c.lane] = tsv;
        if (!(flags & HA_FLAG_NO_PHYSICS)) run_physics<PC>(c, c.p->control_freq_inv);   // vec_task.py:409-412
        after_physics(c, env);
        store_env(c, S, env);
        if (c.lane == 0) S.progress_buf[env] = S.progress_buf[env] + 1;                // allegro_hand.py:629
        ah_in_from_lds(c, &ain);
        ah_post(c, S, env, ain, false);
        return;
    }
    if (MODE == MODE_RESET) {
        task_reset(c, S, env, flags);
        if (!(flags & HA_FLAG_NO_PHYSICS)) run_physics<PC>(c, 1);
        after_physics(c, env);
        task_reset_finish(c, S, env);
        store_env(c, S, env);
        return;
    }
    // MODE_STEP: VecTask.step (vec_task.py:390-441) for Ur5SihMultiObjectManipulation
    bool do_reset = S.reset_buf[env] != 0;                   // configurable_vec_task.py:348
    controller_step(c, S, env);                               // :350-354
    if (do_reset) task_reset(c, S, env, flags);               // :356-357 -> reset_idx
    // phase 0 (reset envs only): reset_idx's extra gym.simulate (multi_object_manipulation.py:67). The
    // reference resets every env on the same step (ur5sih.py:617 asserts it), so a per-env extra call is
    // equivalent. Phase 1: the control_freq_inv physics calls (vec_task.py:409-412). One call site keeps
    // a single copy of the physics code.
    for (int ph = do_reset ? 0 : 1; ph < 2; ph++) {
        if (!(flags & HA_FLAG_NO_PHYSICS)) run_physics<PC>(c, ph == 0 ? 1 : c.p->control_freq_inv);
        after_physics(c, env);
        if (ph == 0) task_reset_finish(c, S, env);
    }
    store_env(c, S, env);
    ur5sih_obs_in(c, &in);
    post_step(c, S, env, in, false);                           // configurable_vec_task.py:359-390
}

#if defined(HA_PROFILE) || defined(HA_ENVT)
// diagnostic builds: each workgroup's start / end on the constant 100 MHz clock (s_memrealtime), by launch slot
__device__ unsigned long long g_envt[2 * 65536];
// and where it ran: HW_ID (wave, SIMD, CU, SH, SE bits) and XCC_ID of its wave
__device__ unsigned int g_envhw[2 * 65536];
// (the start stamp is stored right away: an s_memrealtime value kept live across the whole kernel made the backend
// stop with "illegal VGPR to SGPR copy" in the overflow-chunk families)
#define HA_ENV_T0()                                                                               \
    do {                                                                                          \
        unsigned long long _e0 = __builtin_amdgcn_s_memrealtime();                                \
        if (threadIdx.x == 0 && blockIdx.x < 65536) g_envt[2 * blockIdx.x] = _e0;                 \
    } while (0)
#define HA_ENV_T1()                                                                               \
    do {                                                                                          \
        __syncthreads();                                                                          \
        if (threadIdx.x == 0 && blockIdx.x < 65536) {                                            \
            g_envt[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();                          \
            g_envhw[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                    \
            g_envhw[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);               \
        }                                                                                           \
    } while (0)
#else
#define HA_ENV_T0()
#define HA_ENV_T1()
#endif
#define HA_KERNEL(name, FAM, MODE)                                                                              \
    extern "C" __global__ void __launch_bounds__(64)                                                          \
        __attribute__((amdgpu_waves_per_eu(task_waves_per_eu<FAM>())))                                        \
        name(const ha_model_t* __restrict__ model, const ha_params_t* __restrict__ params, ha_state_t st,       \
             int num_envs, int n_calls, uint32_t flags, int stat_slot, float* spill, const int32_t* env_ids,     \
             StepIO io) {                                                                                       \
        HA_ENV_T0();                                                                                            \
        if (MODE == MODE_STEP && io.tend) {  /* by launch slot, like HA_ENV_T0 / T1 */                        \
            unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                           \
            if (threadIdx.x == 0) io.tstart[blockIdx.x] = t_;                                                   \
        }                                                                                                       \
        env_body<FAM, MODE>(model, params, st, num_envs, n_calls, flags, stat_slot, spill, env_ids, io);       \
        if (MODE == MODE_STEP && io.tend) {                                                                     \
            __syncthreads();                                                                                    \
            if (threadIdx.x == 0) io.tend[blockIdx.x] = __builtin_amdgcn_s_memrealtime();                      \
        }                                                                                                       \
        HA_ENV_T1();                                                                                            \
    }
HA_KERNEL(ha_step_kernel, HA_TASK_UR5SIH, MODE_STEP)
HA_KERNEL(ha_simulate_kernel, HA_TASK_UR5SIH, MODE_SIMULATE)
HA_KERNEL(ha_observe_kernel, HA_TASK_UR5SIH, MODE_OBSERVE)
HA_KERNEL(ha_reset_kernel, HA_TASK_UR5SIH, MODE_RESET)
HA_KERNEL(hb_step_kernel, FAM_UR5SIH_CLUTTER, MODE_STEP)
HA_KERNEL(hb_simulate_kernel, FAM_UR5SIH_CLUTTER, MODE_SIMULATE)
HA_KERNEL(hb_observe_kernel, FAM_UR5SIH_CLUTTER, MODE_OBSERVE)
HA_KERNEL(hb_reset_kernel, FAM_UR5SIH_CLUTTER, MODE_RESET)
HA_KERNEL(ah_step_kernel, HA_TASK_ALLEGRO_HAND, MODE_STEP)
HA_KERNEL(ah_simulate_kernel, HA_TASK_ALLEGRO_HAND, MODE_SIMULATE)
HA_KERNEL(ah_observe_kernel, HA_TASK_ALLEGRO_HAND, MODE_OBSERVE)
HA_KERNEL(ah_reset_kernel, HA_TASK_ALLEGRO_HAND, MODE_RESET)
HA_KERNEL(ak_step_kernel, HA_TASK_ALLEGRO_KUKA, MODE_STEP)
HA_KERNEL(ak_simulate_kernel, HA_TASK_ALLEGRO_KUKA, MODE_SIMULATE)
HA_KERNEL(ak_observe_kernel, HA_TASK_ALLEGRO_KUKA, MODE_OBSERVE)
HA_KERNEL(ak_reset_kernel, HA_TASK_ALLEGRO_KUKA, MODE_RESET)

typedef void (*env_kernel_t)(const ha_model_t*, const ha_params_t*, ha_state_t, int, int, uint32_t, int, float*,
                             const int32_t*, StepIO);
static env_kernel_t kernel_for(int fam, int mode) {
    if (fam == FAM_UR5SIH_CLUTTER) {
        switch (mode) {
            case MODE_STEP: return hb_step_kernel;
            case MODE_SIMULATE: return hb_simulate_kernel;
            case MODE_OBSERVE: return hb_observe_kernel;
            default: return hb_reset_kernel;
        }
    }
    if (fam == HA_TASK_ALLEGRO_KUKA) {
        switch (mode) {
            case MODE_STEP: return ak_step_kernel;
            case MODE_SIMULATE: return ak_simulate_kernel;
            case MODE_OBSERVE: return ak_observe_kernel;
            default: return ak_reset_kernel;
        }
    }
    if (fam == HA_TASK_ALLEGRO_HAND) {
        switch (mode) {
            case MODE_STEP: return ah_step_kernel;
            case MODE_SIMULATE: return ah_simulate_kernel;
            case MODE_OBSERVE: return ah_observe_kernel;
            default: return ah_reset_kernel;
        }
    }
    switch (mode) {
        case MODE_STEP: return ha_step_kernel;
        case MODE_SIMULATE: return ha_simulate_kernel;
        case MODE_OBSERVE: return ha_observe_kernel;
        default: return ha_reset_kernel;
    }
}

// ----------------------------------------------------------------------------- indexed setters
extern "C" __global__ void ha_copy_indexed_kernel(float* dst, const float* src, const int32_t* idx, int n, int row,
                                                  int rows_per_index) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int per = row * rows_per_index;
    if (t >= n * per) return;
    int i = t / per, k = t % per;
    size_t base = (size_t)idx[i] * per;
    dst[base + k] = src[base + k];
}

// ----------------------------------------------------------------------------- domain randomization, shard-wide
// apply_randomizations' non-env part before a step (mode 0) or reset (mode 1) launch (ha_dr.h dr_global_update): one
// workgroup ORs the reset flags (reset_idx runs, and with it apply_randomizations, when any env resets), then one
// lane updates dr_global. force_any: the launch resets every env regardless of the flags (the Ur5Sih reset launch).
extern "C" __global__ void __launch_bounds__(256) ha_dr_global_kernel(const ha_params_t* __restrict__ params,
                                                                       const int64_t* __restrict__ reset_buf, int n,
                                                                       float* __restrict__ g, int mode, int force_any) {
    __shared__ int any;
    if (threadIdx.x == 0) any = force_any;
    __syncthreads();
    int a = 0;
    for (int i = threadIdx.x; i < n; i += 256) a |= reset_buf[i] != 0 ? 1 : 0;
    if (a) any = 1;                     // every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) dr_global_update(*params, g, any, mode);
}

// ----------------------------------------------------------------------------- step epilogue
// VecTask.step's tail as ONE launch (instead of a clamp kernel plus one reduction kernel per logged scalar):
// obs_out = clamp(obs, -clip, clip) (vec_task.py:437, a fresh buffer for obs_dict["obs"]), and for AllegroKuka the
// extras scalars of allegro_kuka_base.py:908-917: mean prev_episode_successes, mean / min / max true_objective.
// Block 0 reduces (fixed-order strided partial sums, then an LDS tree: deterministic); every block copies.
extern "C" __global__ void __launch_bounds__(256) ha_epilogue_kernel(const float* __restrict__ obs,
                                                                      float* __restrict__ obs_out, long long n_obs,
                                                                      float clip, const float* __restrict__ ts,
                                                                      int ts_stride, int n_env, float* __restrict__ out) {
    // block 0 reduces the task scalars (when asked); the obs clamp runs on the other blocks
    bool red_block = ts && out && blockIdx.x == 0;
    if (obs_out && !(red_block && gridDim.x > 1)) {
        long long b = red_block ? 0 : (ts && out ? blockIdx.x - 1 : blockIdx.x);
        long long nb = ts && out && gridDim.x > 1 ? gridDim.x - 1 : gridDim.x;
        for (long long k = b * 256 + threadIdx.x; k < n_obs; k += nb * 256) obs_out[k] = fminf(fmaxf(obs[k], -clip), clip);
    }
    if (!red_block) return;
    __shared__ float red[4][256];
    float s0 = 0.0f, s1 = 0.0f, mn = 3.0e38f, mx = -3.0e38f;
    // the thread's envs e = tid, tid + 256, ... in order; eight rows' loads are issued before they are added, so the
    // strided reads overlap instead of costing one round trip each (same sums in the same order)
    for (int e0 = threadIdx.x; e0 < n_env; e0 += 256 * 8) {
        float ps[8], to[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            int e = e0 + 256 * u;
            ps[u] = e < n_env ? ts[(size_t)e * ts_stride + HA_AK_PREV_SUCC] : 0.0f;
            to[u] = e < n_env ? ts[(size_t)e * ts_stride + HA_AK_TRUE_OBJ] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (e0 + 256 * u < n_env) {
                s0 += ps[u];
                s1 += to[u];
                mn = fminf(mn, to[u]);
                mx = fmaxf(mx, to[u]);
            }
        }
    }
    red[0][threadIdx.x] = s0; red[1][threadIdx.x] = s1; red[2][threadIdx.x] = mn; red[3][threadIdx.x] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            red[0][threadIdx.x] += red[0][threadIdx.x + w];
            red[1][threadIdx.x] += red[1][threadIdx.x + w];
            red[2][threadIdx.x] = fminf(red[2][threadIdx.x], red[2][threadIdx.x + w]);
            red[3][threadIdx.x] = fmaxf(red[3][threadIdx.x], red[3][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = red[0][0] / (float)n_env;
        out[1] = red[1][0] / (float)n_env;
        out[2] = red[2][0];
        out[3] = red[3][0];
    }
}

// ----------------------------------------------------------------------------- C ABI
struct ha_handle_s {
    ha_model_t* d_model;
    ha_params_t* d_params;
    ha_params_t h_params;
    int N, NO, D, L, A, B, task, fam;
    int a0;               // actor_object0 (host copy)
    int pcm_slots;        // persistent-manifold record slots per env (ha_contact_cache_slots)
    ha_state_t st;
    int bound;
    int stat_slots;
    long long step_counter;
    hipEvent_t ev0, ev1;
    int timed;
    int t_max, t_count;
    hipEvent_t* t_ev;     // 2 * t_max events
    int pc_count;
    hipEvent_t* pc_ev;    // 2 * t_max events (ha_pointclouds launches)
    float* d_spill;       // split-row families: robot-block rows beyond the LDS slots, N x spill_floats
    const int32_t* order; // ha_set_env_order: env of workgroup i in full-shard launches (null: identity)
    StepIO io;            // ha_task_step_io: the step launch's folded head / tail (zero otherwise)
    unsigned long long* d_tstart;   // ha_set_order_cost(1): workgroup start / end stamps per env
    unsigned long long* d_tend;
    float* d_io_partials; // AllegroKuka extras: 4 floats per group of 64 envs
    int32_t* d_io_counters;   // and ceil(N / 64) + 1 counters, zero between launches
};

#define HIPCHK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "handarm_hip: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return HA_E_HIP;                                                          \
        }                                                                             \
    } while (0)

// per-family shape (object capacity, LDS bytes, row stride), from the same templates the kernels use
template <int FAM>
static size_t fam_lds_bytes() { return task_lds_bytes<FamPhys<FAM>>(); }
static size_t spill_floats(int fam) {
    switch (fam) {
        case FAM_UR5SIH_CLUTTER: return FamPhys<FAM_UR5SIH_CLUTTER>::spill_floats;
        case HA_TASK_ALLEGRO_HAND: return FamPhys<HA_TASK_ALLEGRO_HAND>::spill_floats;
        case HA_TASK_ALLEGRO_KUKA: return FamPhys<HA_TASK_ALLEGRO_KUKA>::spill_floats;
        default: return FamPhys<HA_TASK_UR5SIH>::spill_floats;
    }
}
static int pairf_bytes(int fam) {
    switch (fam) {
        case FAM_UR5SIH_CLUTTER: return FamPhys<FAM_UR5SIH_CLUTTER>::pairf_bytes;
        case HA_TASK_ALLEGRO_HAND: return FamPhys<HA_TASK_ALLEGRO_HAND>::pairf_bytes;
        case HA_TASK_ALLEGRO_KUKA: return FamPhys<HA_TASK_ALLEGRO_KUKA>::pairf_bytes;
        default: return FamPhys<HA_TASK_UR5SIH>::pairf_bytes;
    }
}
static int obj_capacity(int fam) {
    switch (fam) {
        case FAM_UR5SIH_CLUTTER: return task_obj_capacity<FAM_UR5SIH_CLUTTER>();
        case HA_TASK_ALLEGRO_HAND: return task_obj_capacity<HA_TASK_ALLEGRO_HAND>();
        case HA_TASK_ALLEGRO_KUKA: return task_obj_capacity<HA_TASK_ALLEGRO_KUKA>();
        default: return task_obj_capacity<HA_TASK_UR5SIH>();
    }
}
static size_t lds_bytes(int fam) {
    switch (fam) {
        case FAM_UR5SIH_CLUTTER: return fam_lds_bytes<FAM_UR5SIH_CLUTTER>();
        case HA_TASK_ALLEGRO_HAND: return fam_lds_bytes<HA_TASK_ALLEGRO_HAND>();
        case HA_TASK_ALLEGRO_KUKA: return fam_lds_bytes<HA_TASK_ALLEGRO_KUKA>();
        default: return fam_lds_bytes<HA_TASK_UR5SIH>();
    }
}
template <int FAM>
static int fam_contacts() { return FamPhys<FAM>::cap * FamPhys<FAM>::nch; }
static int contact_capacity(int fam) {
    switch (fam) {
        case FAM_UR5SIH_CLUTTER: return fam_contacts<FAM_UR5SIH_CLUTTER>();
        case HA_TASK_ALLEGRO_HAND: return fam_contacts<HA_TASK_ALLEGRO_HAND>();
        case HA_TASK_ALLEGRO_KUKA: return fam_contacts<HA_TASK_ALLEGRO_KUKA>();
        default: return fam_contacts<HA_TASK_UR5SIH>();
    }
}
static int task_row_stride(int task) {
    return task == HA_TASK_ALLEGRO_KUKA ? row_stride<AK_ND>()
                                        : (task == HA_TASK_ALLEGRO_HAND ? row_stride<AH_ND>() : row_stride<HA_ND>());
}
// kernel family of a task configuration: Ur5Sih with more objects than the dense family's 3 slots runs the
// clutter family (bin-picking)
static int family_of(const ha_params_t* p) {
    if (p->task == HA_TASK_UR5SIH && p->n_objects > task_obj_capacity<HA_TASK_UR5SIH>()) return FAM_UR5SIH_CLUTTER;
    return p->task;
}

extern "C" {

int ha_abi_version(void) { return HA_ABI_VERSION; }

int ha_struct_sizes(int32_t* model_size, int32_t* params_size, int32_t* state_size) {
    if (!model_size || !params_size || !state_size) return HA_E_ARG;
    *model_size = (int32_t)sizeof(ha_model_t);
    *params_size = (int32_t)sizeof(ha_params_t);
    *state_size = (int32_t)sizeof(ha_state_t);
    return HA_OK;
}

// hull k's vertices inside its hull_obb box (centre, half extents, orientation in the body frame), within 1e-5 m
static bool hull_in_box(const ha_model_t* m, int k) {
    const float* ob = m->hull_obb[k];
    if (!(ob[3] >= 0.0f && ob[4] >= 0.0f && ob[5] >= 0.0f)) return false;
    const float zero[3] = {0.0f, 0.0f, 0.0f}, id[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    float c[3], R[9];
    ha_obb_world(zero, id, ob, c, R);
    for (int v = 0; v < m->hull_nverts[k]; v++) {
        const float* x = m->verts[m->hull_vert_start[k] + v];
        float d[3] = {x[0] - c[0], x[1] - c[1], x[2] - c[2]};
        for (int i = 0; i < 3; i++) {
            float l = R[i] * d[0] + R[3 + i] * d[1] + R[6 + i] * d[2];
            if (fabsf(l) > ob[3 + i] + 1e-5f) return false;
        }
    }
    return true;
}

int ha_create(const ha_model_t* model, const ha_params_t* params, int32_t num_envs, ha_handle* out) {
    if (!model || !params || !out || num_envs <= 0) return HA_E_ARG;
    if (params->task != HA_TASK_UR5SIH && params->task != HA_TASK_ALLEGRO_HAND && params->task != HA_TASK_ALLEGRO_KUKA)
        return HA_E_ARG;
    // the kernels are compiled for the task's DOF count (register-resident factorization)
    int nd = params->task == HA_TASK_ALLEGRO_HAND ? AH_ND : (params->task == HA_TASK_ALLEGRO_KUKA ? AK_ND : HA_ND);
    if (model->n_dofs != nd) return HA_E_MODEL;
    if (params->task == HA_TASK_ALLEGRO_KUKA) {
        if (params->n_objects != 1 || params->ak_num_keypoints < 1 || params->ak_num_keypoints > 4 ||
            params->num_obs > AK_MAX_OBS || params->num_obs != 93 + 6 * params->ak_num_keypoints)
            return HA_E_ARG;
        if (params->ak_palm_link < 0 || params->ak_palm_link >= model->n_links) return HA_E_MODEL;
        for (int i = 0; i < 4; i++)
            if (params->ak_fingertip_links[i] < 0 || params->ak_fingertip_links[i] >= model->n_links) return HA_E_MODEL;
        // privilegedActions (v16): 3 torque actions ahead of the 23
        if (params->num_actions != AK_NUM_ACT + (params->ak_privileged_actions ? 3 : 0)) return HA_E_ARG;
    }
    // the DR schema (v16): known distributions / operations / schedules, positive loguniform ranges, a frequency
    if (params->dr_enable) {
        if (params->dr_frequency < 1) return HA_E_ARG;
        for (int k = 0; k < HA_DRA_N; k++) {
            const ha_dr_attr_t& a = params->dr_attr[k];
            if (a.dist < HA_DR_DIST_OFF || a.dist > HA_DR_DIST_GAUSSIAN || a.op < HA_DR_OP_ADDITIVE ||
                a.op > HA_DR_OP_SCALING || a.sched < HA_DR_SCHED_NONE || a.sched > HA_DR_SCHED_CONSTANT ||
                (a.sched == HA_DR_SCHED_LINEAR && a.sched_steps < 1) || a.num_buckets < 0)
                return HA_E_ARG;
            if (a.dist == HA_DR_DIST_LOGUNIFORM && !(a.range[0] > 0.0f && a.range[1] > 0.0f)) return HA_E_ARG;
            if ((k == HA_DRA_OBS || k == HA_DRA_ACT) && a.dist == HA_DR_DIST_LOGUNIFORM) return HA_E_ARG;
        }
    }
    if (model->n_actors < 1 || model->n_bodies < model->n_links + params->n_objects) return HA_E_MODEL;
    int fam = family_of(params);
    if (params->task == HA_TASK_UR5SIH && params->num_obs != 108 + 13 * params->n_objects) return HA_E_ARG;
    // AllegroHand observation types (v15): num_obs is the type's size (allegro_hand.py:106-112)
    if (params->task == HA_TASK_ALLEGRO_HAND &&
        (params->ah_obs_type < 0 || params->ah_obs_type > 2 ||
         params->num_obs != (params->ah_obs_type == 0 ? 88 : (params->ah_obs_type == 1 ? 72 : 50))))
        return HA_E_ARG;
    if (model->actor_object0 < 0 || model->actor_object0 + params->n_objects > model->n_actors ||
        model->body_object0 < 0 || model->body_object0 + params->n_objects > model->n_bodies)
        return HA_E_MODEL;
    if (model->n_fixed_bodies < 0 || model->n_fixed_bodies > HA_MAX_FIXED_BODIES ||
        (model->n_fixed_bodies > 0 && (model->body_fixed0 < 0 || model->body_fixed0 + model->n_fixed_bodies > model->n_bodies)))
        return HA_E_MODEL;
    if (model->n_links > HA_MAX_LINKS || params->n_objects < 1 || params->n_objects > obj_capacity(fam) ||
        model->n_dofs + 6 * (params->n_objects < 2 ? params->n_objects : 2) > task_row_stride(params->task) ||
        model->n_dofs + 6 * params->n_objects > MAXV || model->n_bodies > MAXB ||
        model->n_static < 0 || model->n_static > HA_MAX_STATIC || model->n_pool < 1 || model->n_pool > HA_MAX_POOL ||
        model->n_hulls > HA_MAX_HULLS)
        return HA_E_MODEL;
    // posed statics (v14): one carrying actor per env; the throw bucket is the actor in the goal slot
    if (model->posed_actor < -1 || model->posed_actor >= model->n_actors) return HA_E_MODEL;
    for (int k = 0; k < model->n_static; k++)
        if (model->static_posed[k] && model->posed_actor < 0) return HA_E_MODEL;
    if (params->task == HA_TASK_ALLEGRO_KUKA && params->ak_subtask == 2 && model->posed_actor != model->actor_goal)
        return HA_E_MODEL;
    // every hull must fit the family's narrow-phase scratch (ColLayout)
    int col_v = (fam == HA_TASK_ALLEGRO_KUKA || fam == HA_TASK_ALLEGRO_HAND) ? FamPhys<HA_TASK_ALLEGRO_HAND>::colv
                                                                           : FamPhys<HA_TASK_UR5SIH>::colv;
    int col_p = (fam == HA_TASK_ALLEGRO_KUKA || fam == HA_TASK_ALLEGRO_HAND) ? FamPhys<HA_TASK_ALLEGRO_HAND>::colp
                                                                           : FamPhys<HA_TASK_UR5SIH>::colp;
    static_assert(FamPhys<HA_TASK_ALLEGRO_HAND>::colv == FamPhys<HA_TASK_ALLEGRO_KUKA>::colv &&
                      FamPhys<HA_TASK_ALLEGRO_HAND>::colp == FamPhys<HA_TASK_ALLEGRO_KUKA>::colp &&
                      FamPhys<HA_TASK_UR5SIH>::colv == FamPhys<FAM_UR5SIH_CLUTTER>::colv &&
                      FamPhys<HA_TASK_UR5SIH>::colp == FamPhys<FAM_UR5SIH_CLUTTER>::colp,
                  "narrow-phase scratch limits per family pair");
    for (int k = 0; k < model->n_hulls; k++) {
        if (model->hull_nverts[k] > col_v || model->hull_nplanes[k] > col_p) return HA_E_MODEL;
        // v10 topology: the edge-edge SAT keeps a hull's culled edge list as bytes in the scratch's candidate arrays
        // (4 x col_v bytes each); a clipped manifold's candidates take 2 lanes per incident loop edge and one per
        // reference loop vertex (FaceCands), so loops hold <= HA_MAX_FACE_LOOP vertices
        if (model->hull_nedges[k] < 0 || model->hull_nedges[k] > 4 * col_v || model->hull_nplanes[k] > 256 ||
            model->hull_edge_start[k] < 0 || model->hull_edge_start[k] + model->hull_nedges[k] > HA_MAX_EDGES)
            return HA_E_MODEL;
        // the topology records index the hull's LDS vertex / plane scratch directly: every index must be in range
        int nv = model->hull_nverts[k], np_ = model->hull_nplanes[k];
        if (model->hull_vert_start[k] < 0 || model->hull_vert_start[k] + nv > HA_MAX_VERTS ||
            model->hull_plane_start[k] < 0 || model->hull_plane_start[k] + np_ > HA_MAX_PLANES)
            return HA_E_MODEL;
        for (int j = 0; j < np_; j++) {
            int pl = model->plane_loop[model->hull_plane_start[k] + j];
            if ((pl >> 16) < 3 || (pl >> 16) > HA_MAX_FACE_LOOP || (pl & 0xFFFF) + (pl >> 16) > HA_MAX_LOOP)
                return HA_E_MODEL;
            for (int t = 0; t < (pl >> 16); t++)
                if (model->loop_v[(pl & 0xFFFF) + t] >= nv) return HA_E_MODEL;
        }
        for (int j = 0; j < model->hull_nedges[k]; j++) {
            uint32_t e = model->edges[model->hull_edge_start[k] + j];
            if ((int)(e & 255u) >= nv || (int)((e >> 8) & 255u) >= nv || (int)((e >> 16) & 255u) >= np_ ||
                (int)(e >> 24) >= np_)
                return HA_E_MODEL;
        }
    }
    // the broad phase's box cull (ha_physics.h pair_boxes_near): every link hull and every one-piece pool object's hull
    // inside its hull_obb box
    if (model->n_link_hulls < 0 || model->n_link_hulls > model->n_hulls) return HA_E_MODEL;
    for (int k = 0; k < model->n_hulls; k++) {
        bool boxed = k < model->n_link_hulls, obj = false;
        for (int p = 0; p < model->n_pool; p++) {
            obj = obj || (model->pool_nhull[p] == 1 && model->pool_hull[p] == k);
            // a compound object's pieces: the piece-pair box cull (ha_physics.h piece_boxes_near, round 6)
            boxed = boxed || (model->pool_nhull[p] > 1 && k >= model->pool_hull[p] &&
                              k < model->pool_hull[p] + model->pool_nhull[p]);
        }
        if ((boxed || obj) && !hull_in_box(model, k)) return HA_E_MODEL;
        // a one-piece object's box is read with the identity orientation (ha_physics.h object_box): refuse any other
        const float* oq = model->hull_obb[k] + 6;
        if (obj && !(oq[0] == 0.0f && oq[1] == 0.0f && oq[2] == 0.0f && oq[3] == 1.0f)) return HA_E_MODEL;
    }
    // self-collision pairs (v12): two link hulls of the model each; only the Allegro families' kernels run them
    if (model->n_self_pairs < 0 || model->n_self_pairs > HA_MAX_SELF_PAIRS) return HA_E_MODEL;
    if (model->n_self_pairs > 0 && params->task == HA_TASK_UR5SIH) return HA_E_MODEL;
    // the self-pair pass keeps a 64-byte world box per link hull, a 2-byte entry per pair and 64 candidate entries in
    // the narrow-phase scratch (detect_self)
    if (model->n_self_pairs > 0 &&
        (size_t)model->n_link_hulls * 64 + 2 * (size_t)model->n_self_pairs + 128 > (fam == HA_TASK_ALLEGRO_HAND ? FamPhys<HA_TASK_ALLEGRO_HAND>::col_bytes
                                                                        : FamPhys<HA_TASK_ALLEGRO_KUKA>::col_bytes))
        return HA_E_MODEL;
    for (int k = 0; k < model->n_self_pairs; k++) {
        int a = model->self_pair[k] & 255, b = model->self_pair[k] >> 8;
        if (a >= model->n_link_hulls || b >= model->n_link_hulls || a == b) return HA_E_MODEL;
    }
    // a family without a gather buffer (ColLayout NG = 0) takes single-hull pool objects only
    bool one_hull = (fam == HA_TASK_ALLEGRO_KUKA && FamPhys<HA_TASK_ALLEGRO_KUKA>::colg == 0) ||
                    (fam == HA_TASK_ALLEGRO_HAND && FamPhys<HA_TASK_ALLEGRO_HAND>::colg == 0);
    for (int i = 0; i < model->n_pool; i++)
        if (model->pool_nhull[i] < 1 || model->pool_hull[i] < 0 ||
            model->pool_hull[i] + model->pool_nhull[i] > model->n_hulls || (one_hull && model->pool_nhull[i] != 1))
            return HA_E_MODEL;
    if (params->num_initial_poses < 1 || params->num_initial_poses > HA_MAX_INIT_POSES) return HA_E_ARG;
    ha_handle h = (ha_handle)calloc(1, sizeof(ha_handle_s));
    h->N = num_envs;
    h->NO = params->n_objects;
    h->D = model->n_dofs;
    h->L = model->n_links;
    h->A = model->n_actors;
    h->B = model->n_bodies;
    h->a0 = model->actor_object0;
    h->task = params->task;
    h->fam = fam;
    h->h_params = *params;
    h->stat_slots = 1;
    // the broad phase's pairs must fit the family's separating-face records (one byte each in the env's global area)
    {
        int NO = params->n_objects, NS = model->n_static, NLH = model->n_link_hulls;
        if (NO * (1 + NS + NLH) + NO * (NO - 1) / 2 + NLH * NS > pairf_bytes(fam)) return HA_E_MODEL;
    }
    // persistent-manifold records (v13): none when the tolerance is off, and none in a family built without them
    if (params->pcm_lin_tol > 0.0f && !family_pcm(fam)) return HA_E_ARG;
    h->pcm_slots = params->pcm_lin_tol <= 0.0f ? 0 :
                   params->n_objects * (1 + model->n_static + model->n_link_hulls) +
                   params->n_objects * (params->n_objects - 1) / 2 + model->n_link_hulls * model->n_static +
                   model->n_self_pairs;
    HIPCHK(hipMalloc(&h->d_model, sizeof(ha_model_t)));
    HIPCHK(hipMalloc(&h->d_params, sizeof(ha_params_t)));
    HIPCHK(hipMemcpy(h->d_model, model, sizeof(ha_model_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_params, params, sizeof(ha_params_t), hipMemcpyHostToDevice));
    if (spill_floats(fam)) {
        HIPCHK(hipMalloc(&h->d_spill, sizeof(float) * spill_floats(fam) * (size_t)num_envs));
        // every byte 0xFF: the self-collision records start as "no separating face" (the other areas are written
        // before they are read)
        HIPCHK(hipMemset(h->d_spill, 0xFF, sizeof(float) * spill_floats(fam) * (size_t)num_envs));
    }
    if (fam == HA_TASK_ALLEGRO_KUKA) {
        size_t G = ((size_t)num_envs + 63) / 64;
        HIPCHK(hipMalloc(&h->d_io_partials, sizeof(float) * 4 * G));
        HIPCHK(hipMalloc(&h->d_io_counters, sizeof(int32_t) * (G + 1)));
        HIPCHK(hipMemset(h->d_io_counters, 0, sizeof(int32_t) * (G + 1)));
    }
    for (int mode : {MODE_STEP, MODE_SIMULATE, MODE_OBSERVE, MODE_RESET})
        HIPCHK(hipFuncSetAttribute((const void*)kernel_for(h->fam, mode), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_bytes(h->fam)));
    HIPCHK(hipEventCreate(&h->ev0));
    HIPCHK(hipEventCreate(&h->ev1));
    *out = h;
    return HA_OK;
}

int ha_destroy(ha_handle h) {
    if (!h) return HA_E_ARG;
    (void)hipFree(h->d_model);
    (void)hipFree(h->d_params);
    if (h->d_spill) (void)hipFree(h->d_spill);
    if (h->d_io_partials) (void)hipFree(h->d_io_partials);
    if (h->d_io_counters) (void)hipFree(h->d_io_counters);
    if (h->d_tstart) (void)hipFree(h->d_tstart);
    if (h->d_tend) (void)hipFree(h->d_tend);
    (void)hipEventDestroy(h->ev0);
    (void)hipEventDestroy(h->ev1);
    free(h);
    return HA_OK;
}

int ha_bind_state(ha_handle h, const ha_state_t* state) {
    if (!h || !state) return HA_E_ARG;
    const void* req[] = {state->root_state, state->rigid_body_state, state->dof_state, state->net_contact_force,
                         state->sim_targets};
    for (auto p : req)
        if (!p) return HA_E_ARG;
    h->st = *state;
    h->bound = 1;
    return HA_OK;
}

static int launch(ha_handle h, int mode, int n_calls, uint32_t flags, int slot, void* stream,
                  const int32_t* env_ids = nullptr, int n_ids = 0) {
    if (!h || !h->bound) return HA_E_STATE;
    hipStream_t s = (hipStream_t)stream;
    // HIP events only while timing is enabled (ha_enable_kernel_timing): an event record in the stream costs a few
    // microseconds of GPU idle between the kernels, which a training loop should not pay
    bool rec = h->t_ev && h->t_count < h->t_max;
    if (rec) (void)hipEventRecord(h->t_ev[2 * h->t_count], s);
    if (!env_ids && h->order) {            // full shard in the caller's dispatch order (ha_set_env_order)
        env_ids = h->order;
        n_ids = h->N;
    }
    hipLaunchKernelGGL(kernel_for(h->fam, mode), dim3(env_ids ? n_ids : h->N), dim3(64), lds_bytes(h->fam), s, h->d_model,
                       h->d_params, h->st, h->N, n_calls, flags, slot, h->d_spill, env_ids,
                       mode == MODE_STEP ? h->io : StepIO{});
    HIPCHK(hipGetLastError());
    if (rec) {
        (void)hipEventRecord(h->t_ev[2 * h->t_count + 1], s);
        h->t_count++;
    }
    h->timed = rec ? 1 : 0;         // ha_last_kernel_ms: -1 for an untimed launch instead of an older launch's time
    return HA_OK;
}

int ha_simulate(ha_handle h, int32_t n_calls, uint32_t flags, void* stream) {
    if (n_calls < 0) return HA_E_ARG;
    if (n_calls == 0 || (flags & HA_FLAG_NO_PHYSICS)) return HA_OK;
    return launch(h, MODE_SIMULATE, n_calls, flags, 0, stream);
}

// Longest-first dispatch order from the contacts each env offered since the last call (contact_stats column 3 minus
// cost_prev, which is then updated): one workgroup, a counting sort on the cost clamped to 1023 (descending; envs of
// equal cost in arbitrary order: the order is a scheduling hint, results do not depend on it). One launch instead of
// the ~10 small torch kernels of a device argsort
extern "C" __global__ void __launch_bounds__(1024) ha_env_order_kernel(const int32_t* __restrict__ stats,
                                                                        int32_t* __restrict__ cost_prev,
                                                                        int32_t* __restrict__ order, int n,
                                                                        int snake,
                                                                        const unsigned long long* __restrict__ t0,
                                                                        const unsigned long long* __restrict__ t1) {
    __shared__ int cnt[1024], pos[1024];
    __shared__ int span_max;
    int t = threadIdx.x;
    if (t == 0) span_max = 1;
    __syncthreads();
    if (t1) {
        // the spans are per launch slot: slot s ran env order[s] (the order being replaced); cost_prev holds them per
        // env for the passes below (100 MHz clock ticks)
        int m = 1;
        for (int q = t; q < n; q += 1024) {
            unsigned long long d = t1[q] >= t0[q] ? t1[q] - t0[q] : 0ull;
            int v = d > 0x7FFFFFFFull ? 0x7FFFFFFF : (int)d;
#ifndef HA_X_ORDER_LAST_SPAN    /* A/B: the last span alone */
            // half the last span plus half the previous estimate (C5 +1%, C4 +0.7% against the last span alone)
            v = (int)(((long long)v + cost_prev[order[q]]) >> 1);
#endif
            cost_prev[order[q]] = v;
            m = v > m ? v : m;
        }
        atomicMax(&span_max, m);
        __syncthreads();
    }
    const long long smax = span_max;
    auto bucket = [&](int e) {
        // the span scaled so that the longest lands in bucket 0 (the spans of a long launch, C5's ~7 ms per env,
        // would saturate a fixed unit), or the contacts offered since the last refresh
        int cost = t1 ? (int)((long long)cost_prev[e] * 1023 / smax) : stats[HA_CSTAT * (size_t)e + 3] - cost_prev[e];
#ifdef HA_X_ORDER_FIXED_UNIT    /* A/B: the fixed 5.12 us bucket of the first span-based order */
        if (t1) cost = cost_prev[e] >> 9;
#endif
        return 1023 - (cost < 0 ? 0 : (cost > 1023 ? 1023 : cost));      // bucket 0: the most expensive envs
    };
    cnt[t] = 0;
    __syncthreads();
    for (int e = t; e < n; e += 1024) atomicAdd(&cnt[bucket(e)], 1);
    __syncthreads();
    pos[t] = cnt[t];
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {           // inclusive scan of the bucket counts (Hillis-Steele)
        int v = t >= off ? pos[t - off] : 0;
        __syncthreads();
        pos[t] += v;
        __syncthreads();
    }
    pos[t] -= cnt[t];                                    // exclusive: each bucket's first slot
    __syncthreads();
    for (int e = t; e < n; e += 1024) {
        int q = atomicAdd(&pos[bucket(e)], 1);
        if (snake > 0) {
            // rank q -> position: every other block of `snake` positions reversed, so that the workgroups dispatched
            // to the same CU in successive blocks alternate heavy and light (block = the CU count: one wave per CU
            // per block)
            int blk = q / snake, j = q - blk * snake;
            int last = blk * snake + snake <= n ? snake : n - blk * snake;
            if (blk & 1) q = blk * snake + (last - 1 - j);
        }
        order[q] = e;
        if (!t1) cost_prev[e] = stats[HA_CSTAT * (size_t)e + 3];
    }
}

int ha_update_env_order(ha_handle h, int32_t* order, int32_t* cost_prev, int32_t snake, void* stream) {
    if (!h || !h->bound || !order || !cost_prev || !h->st.contact_stats || snake < 0) return HA_E_ARG;
    // span mode maps launch slot q to env order[q]: only right for the order the step launches used
    if (h->d_tend && order != h->order) return HA_E_ARG;
    hipLaunchKernelGGL(ha_env_order_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, h->st.contact_stats,
                       cost_prev, order, h->N, snake, (const unsigned long long*)h->d_tstart,
                       (const unsigned long long*)h->d_tend);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

// the dispatch-order refresh's cost: 0 the contacts each env offered (default), 1 each env's workgroup span in the
// last step launch (measured by the step kernels: two clock reads and two stores per env)
int ha_set_order_cost(ha_handle h, int32_t mode) {
    if (!h || mode < 0 || mode > 1) return HA_E_ARG;
    if (mode == 1 && !h->d_tend) {
        HIPCHK(hipMalloc(&h->d_tstart, sizeof(unsigned long long) * (size_t)h->N));
        HIPCHK(hipMalloc(&h->d_tend, sizeof(unsigned long long) * (size_t)h->N));
        HIPCHK(hipMemset(h->d_tstart, 0, sizeof(unsigned long long) * (size_t)h->N));
        HIPCHK(hipMemset(h->d_tend, 0, sizeof(unsigned long long) * (size_t)h->N));
    } else if (mode == 0 && h->d_tend) {
        (void)hipFree(h->d_tstart);
        (void)hipFree(h->d_tend);
        h->d_tstart = nullptr;
        h->d_tend = nullptr;
    }
    h->io.tstart = h->d_tstart;
    h->io.tend = h->d_tend;
    return HA_OK;
}

int ha_contact_cache_slots(ha_handle h) {
    if (!h) return HA_E_ARG;
    return h->pcm_slots;
}

int ha_set_env_order(ha_handle h, const int32_t* order, int32_t n) {
    if (!h || (order && n != h->N)) return HA_E_ARG;
    h->order = order;
    return HA_OK;
}

int ha_simulate_envs(ha_handle h, int32_t n_calls, uint32_t flags, const int32_t* env_ids, int32_t n_envs, void* stream) {
    if (!h || n_calls < 0 || n_envs < 0 || (n_envs > 0 && !env_ids) || n_envs > h->N) return HA_E_ARG;
    if (n_calls == 0 || n_envs == 0 || (flags & HA_FLAG_NO_PHYSICS)) return HA_OK;
    return launch(h, MODE_SIMULATE, n_calls, flags, 0, stream, env_ids, n_envs);
}

// The bound tensors ARE the simulation state (zero-copy), so refresh has nothing to copy.
int ha_refresh(ha_handle h, void* stream) {
    (void)stream;
    return (h && h->bound) ? HA_OK : HA_E_STATE;
}

int ha_set_dof_position_target(ha_handle h, const float* targets, void* stream) {
    if (!h || !h->bound || !targets) return HA_E_ARG;
    if (targets != h->st.sim_targets)
        HIPCHK(hipMemcpyAsync(h->st.sim_targets, targets, sizeof(float) * h->N * h->D, hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
    return HA_OK;
}

static int copy_indexed(ha_handle h, float* dst, const float* src, const int32_t* idx, int n, int row, int rpi,
                        void* stream) {
    if (!h || !h->bound || !src || !idx || n < 0) return HA_E_ARG;
    if (n == 0 || src == dst) return HA_OK;
    int total = n * row * rpi;
    hipLaunchKernelGGL(ha_copy_indexed_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, dst, src,
                       idx, n, row, rpi);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

// actor indices are global (env * A + actor); the root-state tensor row of actor a is a
int ha_set_actor_root_state_indexed(ha_handle h, const float* root_state, const int32_t* actor_indices, int32_t n,
                                    void* stream) {
    return copy_indexed(h, h ? h->st.root_state : nullptr, root_state, actor_indices, n, 13, 1, stream);
}

// only the robot actor owns DOFs; its DOF rows of env e are e*D .. e*D+D-1 (actor index -> env = a / A)
__global__ void ha_copy_dof_kernel(float* dst, const float* src, const int32_t* idx, int n, int A, int D, int w) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * D * w) return;
    int i = t / (D * w), k = t % (D * w);
    size_t env = (size_t)(idx[i] / A);
    dst[env * D * w + k] = src[env * D * w + k];
}

static int copy_dof_indexed(ha_handle h, float* dst, const float* src, const int32_t* idx, int n, int w,
                            void* stream) {
    if (!h || !h->bound || !src || !idx || n < 0) return HA_E_ARG;
    if (n == 0 || src == dst) return HA_OK;
    int total = n * h->D * w;
    hipLaunchKernelGGL(ha_copy_dof_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, dst, src,
                       idx, n, h->A, h->D, w);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

int ha_set_dof_state_indexed(ha_handle h, const float* dof_state, const int32_t* actor_indices, int32_t n,
                             void* stream) {
    return copy_dof_indexed(h, h ? h->st.dof_state : nullptr, dof_state, actor_indices, n, 2, stream);
}

int ha_set_dof_position_target_indexed(ha_handle h, const float* targets, const int32_t* actor_indices, int32_t n,
                                       void* stream) {
    return copy_dof_indexed(h, h ? h->st.sim_targets : nullptr, targets, actor_indices, n, 1, stream);
}

int ha_set_object_collision_filter(ha_handle h, const uint8_t* enabled, void* stream) {
    if (!h || !h->bound || !enabled || !h->st.collision_enabled) return HA_E_ARG;
    if (enabled != h->st.collision_enabled)
        HIPCHK(hipMemcpyAsync(h->st.collision_enabled, enabled, (size_t)h->N * h->NO, hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
    return HA_OK;
}

// n_slots >= 2: a step clears the next step's slot (so a slot folds no later than n_slots - 1 steps after it
// was written). Clears the whole ring.
int ha_set_stats_ring(ha_handle h, int32_t n_slots) {
    if (!h || n_slots < 2) return HA_E_ARG;
    h->stat_slots = n_slots;
    h->step_counter = 0;
    if (h->bound && h->st.stats) HIPCHK(hipMemset(h->st.stats, 0, sizeof(int32_t) * HA_STAT_SIZE * (size_t)n_slots));
    if (h->bound && h->st.term_sums) HIPCHK(hipMemset(h->st.term_sums, 0, sizeof(float) * 4 * (size_t)n_slots));
    return HA_OK;
}

// the task buffers a fused entry point needs besides the physics tensors
static bool task_bound(ha_handle h) {
    const ha_state_t& s = h->st;
    // DR on (v16): the rows, the shard-wide state and the per-env counters the sampling keys on
    if (h->h_params.dr_enable && !(s.dr_scale && s.dr_global && s.randomize_buf && s.episode && s.reset_buf))
        return false;
    if (h->task == HA_TASK_ALLEGRO_KUKA)
        return s.task_state && s.task_scalars && s.object_scale && s.goal_state && s.successes && s.reset_goal_buf &&
               s.dof_position_targets && s.reset_buf && s.progress_buf && s.rew && s.timeout_buf && s.episode;
    // AllegroHand random forces keep their decayed force, probability and RNG counter in task_state (AH_TS_*)
    if (h->task == HA_TASK_ALLEGRO_HAND && h->h_params.ah_force_scale > 0.0f && !s.task_state) return false;
    return true;
}

// the shard-wide DR update before a step / reset launch (dr_enable only)
static int dr_global(ha_handle h, int mode, void* stream) {
    if (!h->h_params.dr_enable) return HA_OK;
    hipLaunchKernelGGL(ha_dr_global_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, h->d_params, h->st.reset_buf,
                       h->N, h->st.dr_global, mode, mode == 1 && h->task == HA_TASK_UR5SIH ? 1 : 0);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

int ha_task_step(ha_handle h, uint32_t flags, void* stream) {
    if (!h || !h->bound || !h->st.actions || !h->st.obs || !h->st.stats || !h->st.term_sums || !task_bound(h))
        return HA_E_STATE;
    if (h->stat_slots < 2) return HA_E_STATE;
    int slot = (int)(h->step_counter % h->stat_slots);
    int next = (int)((h->step_counter + 1) % h->stat_slots);
    h->step_counter++;
    int rc = dr_global(h, 0, stream);
    if (rc != HA_OK) return rc;
    rc = launch(h, MODE_STEP, next, flags, slot, stream);         // clears `next` for the following step
    if (rc == HA_OK && h->task == HA_TASK_ALLEGRO_HAND && h->st.consecutive_successes) {
        // consecutive_successes EWMA over the shard's resets of this step (allegro_hand.py:714-717)
        hipLaunchKernelGGL(ah_consecutive_successes_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                           h->st.stats + slot * HA_STAT_SIZE, h->st.term_sums + slot * 4, h->st.consecutive_successes,
                           h->h_params.ah_av_factor);
        HIPCHK(hipGetLastError());
    }
    return rc;
}

int ha_task_step_io(ha_handle h, uint32_t flags, const float* actions, float clip_actions, float* obs_out,
                    float clip_obs, float* scalars, void* stream) {
    if (!h) return HA_E_ARG;
    if (h->fam != HA_TASK_ALLEGRO_KUKA && h->fam != HA_TASK_ALLEGRO_HAND) return HA_E_ARG;
    if (scalars && (h->fam != HA_TASK_ALLEGRO_KUKA || !h->d_io_counters)) return HA_E_ARG;
    if ((actions && !(clip_actions >= 0.0f)) || (obs_out && !(clip_obs >= 0.0f))) return HA_E_ARG;
    h->io = StepIO{actions, obs_out, scalars, h->d_io_partials, h->d_io_counters, clip_actions, clip_obs,
                   h->d_tstart, h->d_tend};
    int rc = ha_task_step(h, flags, stream);
    h->io = StepIO{};
    h->io.tstart = h->d_tstart;
    h->io.tend = h->d_tend;
    return rc;
}

int ha_task_epilogue(ha_handle h, float* obs_out, float clip_obs, float* scalars, void* stream) {
    if (!h || !h->bound || !h->st.obs) return HA_E_STATE;
    if (scalars && (h->task != HA_TASK_ALLEGRO_KUKA || !h->st.task_state)) return HA_E_ARG;
    long long n = (long long)h->N * h->h_params.num_obs;
    int blocks = (int)((n + 255) / 256);
    blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
    hipLaunchKernelGGL(ha_epilogue_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, h->st.obs, obs_out, n,
                       clip_obs, scalars ? h->st.task_state : nullptr, HA_AK_TS, h->N, scalars);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

int ha_task_observe(ha_handle h, uint32_t flags, void* stream) {
    if (!h || !h->bound || !h->st.obs || !task_bound(h)) return HA_E_STATE;
    HIPCHK(hipMemsetAsync(h->st.stats, 0, sizeof(int32_t) * HA_STAT_SIZE, (hipStream_t)stream));
    HIPCHK(hipMemsetAsync(h->st.term_sums, 0, sizeof(float) * 4, (hipStream_t)stream));
    return launch(h, MODE_OBSERVE, 0, flags, 0, stream);
}

int ha_task_reset(ha_handle h, uint32_t flags, void* stream) {
    if (!h || !h->bound || !task_bound(h)) return HA_E_STATE;
    int rc = dr_global(h, 1, stream);
    if (rc != HA_OK) return rc;
    return launch(h, MODE_RESET, 0, flags, 0, stream);
}

int ha_enable_kernel_timing(ha_handle h, int32_t max_launches) {
    if (!h || max_launches < 0) return HA_E_ARG;
    if (h->t_ev) {
        for (int i = 0; i < 2 * h->t_max; i++) {
            (void)hipEventDestroy(h->t_ev[i]);
            (void)hipEventDestroy(h->pc_ev[i]);
        }
        free(h->t_ev);
        free(h->pc_ev);
        h->t_ev = h->pc_ev = nullptr;
    }
    h->t_max = max_launches;
    h->t_count = h->pc_count = 0;
    if (max_launches == 0) return HA_OK;
    h->t_ev = (hipEvent_t*)calloc(2 * max_launches, sizeof(hipEvent_t));
    h->pc_ev = (hipEvent_t*)calloc(2 * max_launches, sizeof(hipEvent_t));
    for (int i = 0; i < 2 * max_launches; i++) {
        HIPCHK(hipEventCreate(&h->t_ev[i]));
        HIPCHK(hipEventCreate(&h->pc_ev[i]));
    }
    return HA_OK;
}

int ha_kernel_times(ha_handle h, float* out_ms, int32_t max, int32_t* n_out) {
    if (!h || !out_ms || !n_out) return HA_E_ARG;
    int n = h->t_count < max ? h->t_count : max;
    for (int i = 0; i < n; i++) {
        HIPCHK(hipEventSynchronize(h->t_ev[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&out_ms[i], h->t_ev[2 * i], h->t_ev[2 * i + 1]));
    }
    *n_out = n;
    return HA_OK;
}

int ha_pointcloud_times(ha_handle h, float* out_ms, int32_t max, int32_t* n_out) {
    if (!h || !out_ms || !n_out) return HA_E_ARG;
    int n = h->pc_count < max ? h->pc_count : max;
    for (int i = 0; i < n; i++) {
        HIPCHK(hipEventSynchronize(h->pc_ev[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&out_ms[i], h->pc_ev[2 * i], h->pc_ev[2 * i + 1]));
    }
    *n_out = n;
    return HA_OK;
}

int ha_pointclouds(ha_handle h, const ha_pointcloud_t* pc, void* stream) {
    if (!h || !h->bound || !pc) return HA_E_ARG;
    if (h->task != HA_TASK_UR5SIH || !h->st.object_indices || !h->st.target_object_index || !h->st.goal_pos)
        return HA_E_STATE;
    PcLaunch L;
    L.pc = *pc;
    L.root = h->st.root_state;
    L.body = h->st.rigid_body_state;
    L.object_indices = h->st.object_indices;
    L.target_index = h->st.target_object_index;
    L.goal_pos = h->st.goal_pos;
    L.N = h->N;
    L.A = h->A;
    L.B = h->B;
    L.a0 = h->a0;
    L.NO = h->NO;
    // segment table; every index the kernel will form is checked here, on the host
    bool obj = pc->object_pc || pc->target_pc;
    if (obj && (!pc->object_samples || !pc->perm || pc->P < 1 || pc->P > HA_PC_MAX_P || pc->n_pool < 1))
        return HA_E_ARG;
    if (pc->robot_pc && pc->R > HA_PC_MAX_R) return HA_E_ARG;
    if (pc->robot_pc && (!pc->robot_samples || !pc->robot_slot || pc->R < 1)) return HA_E_ARG;
    if (pc->n_links < 0 || pc->n_links > HA_PC_MAX_LINKS || h->NO > HA_MAX_OBJ) return HA_E_ARG;
    for (int l = 0; l < pc->n_links; l++)
        if (pc->links[l] < 0 || pc->links[l] >= h->B) return HA_E_ARG;
    for (int f = 0; f < 5 && pc->fingertip_pc; f++)
        if (pc->fingertip_slot[f] < 0 || pc->fingertip_slot[f] >= pc->n_links) return HA_E_ARG;
    if (pc->relative_goal_pc && (pc->flange_slot < 0 || pc->flange_slot >= pc->n_links)) return HA_E_ARG;
    if (pc->robot_pc && pc->n_links < 1) return HA_E_ARG;   // robot_slot entries are validated by the caller
    int len[6] = {pc->object_pc ? h->NO * pc->P : 0, pc->target_pc ? pc->P : 0, pc->robot_pc ? pc->R : 0,
                  pc->fingertip_pc ? 5 : 0, pc->goal_pc ? 1 : 0, pc->relative_goal_pc ? 1 : 0};
    L.seg[0] = 0;
    for (int k = 0; k < 6; k++) L.seg[k + 1] = L.seg[k] + len[k];
    int W = L.seg[PC_END];
    if (W == 0) return HA_OK;
    if ((long long)W * h->N >= (1ll << 31)) return HA_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    bool rec = h->pc_ev && h->pc_count < h->t_max;
    if (rec) (void)hipEventRecord(h->pc_ev[2 * h->pc_count], s);
    hipLaunchKernelGGL(ha_pointcloud_kernel, dim3(h->N), dim3(256), 0, s, L);
    HIPCHK(hipGetLastError());
    if (rec) (void)hipEventRecord(h->pc_ev[2 * h->pc_count++ + 1], s);
    return HA_OK;
}

int ha_gather_obs(ha_handle h, const float* const* sources, const int32_t* strides, int32_t n_sources,
                  const int32_t* cols, int32_t n_cols, float* out, void* stream) {
    if (!h || !sources || !strides || !cols || !out || n_sources < 1 || n_sources > HA_MAX_OBS_SOURCES ||
        n_cols < 0)
        return HA_E_ARG;
    if (n_cols == 0) return HA_OK;
    if ((long long)n_cols * h->N >= (1ll << 31)) return HA_E_ARG;
    ObsGather g;
    for (int q = 0; q < HA_MAX_OBS_SOURCES; q++) {
        g.src[q] = sources[q < n_sources ? q : 0];
        g.stride[q] = strides[q < n_sources ? q : 0];
        if (!g.src[q]) return HA_E_ARG;
    }
    g.cols = cols;
    g.target = h->st.target_object_index;
    g.out = out;
    g.N = h->N;
    g.n_cols = n_cols;
    unsigned total = (unsigned)n_cols * (unsigned)h->N;
    hipLaunchKernelGGL(ha_obs_gather_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, g);
    HIPCHK(hipGetLastError());
    return HA_OK;
}

int ha_render_camera(ha_handle h, const ha_camera_t* cam, const float* view_inv, uint32_t flags, void* stream) {
    if (!h || !h->bound || !cam || !view_inv) return HA_E_ARG;
    if (h->task != HA_TASK_UR5SIH || !h->st.object_indices || !h->st.goal_pos) return HA_E_STATE;
    if (cam->width < 1 || cam->height < 1 || (long long)cam->width * cam->height > (1 << 24) ||
        !(cam->fovx_deg > 0.0f && cam->fovx_deg < 180.0f) || !(cam->max_depth > 0.0f))
        return HA_E_ARG;
    if ((flags & HA_CAM_FROM_DEPTH) && (!cam->depth || !cam->pointcloud)) return HA_E_ARG;
    if (h->NO > HA_MAX_OBJ) return HA_E_ARG;
    ha_model_t hm;      // the host copy of the few model fields the launch needs
    HIPCHK(hipMemcpy(&hm.n_link_hulls, &h->d_model->n_link_hulls, sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&hm.n_static, &h->d_model->n_static, sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&hm.body_robot0, &h->d_model->body_robot0, sizeof(int32_t), hipMemcpyDeviceToHost));
    // the most pieces any env's objects can have: the NO largest pool_nhull
    int nh[HA_MAX_POOL], pieces = 0;
    for (int i = 0; i < hm.n_pool && i < HA_MAX_POOL; i++) nh[i] = hm.pool_nhull[i];
    for (int o = 0; o < h->NO; o++) {
        int bi = -1;
        for (int i = 0; i < hm.n_pool && i < HA_MAX_POOL; i++)
            if (nh[i] > 0 && (bi < 0 || nh[i] > nh[bi])) bi = i;
        if (bi >= 0) { pieces += nh[bi]; nh[bi] = 0; }
    }
    if (hm.n_link_hulls + pieces + hm.n_static > HA_CAM_MAX_HULLS || hm.n_link_hulls > 256) return HA_E_MODEL;
    CamLaunch L;
    L.cam = *cam;
    L.m = h->d_model;
    L.root = h->st.root_state;
    L.body = h->st.rigid_body_state;
    L.object_indices = h->st.object_indices;
    L.goal_pos = h->st.goal_pos;
    L.N = h->N;
    L.A = h->A;
    L.B = h->B;
    L.a0 = h->a0;
    L.NO = h->NO;
    L.body_robot0 = hm.body_robot0;
    L.n_link_hulls = hm.n_link_hulls;
    L.n_static = hm.n_static;
    // camera frame (Isaac Gym: +X forward, +Y left, +Z up) -> view axes (x right = -Y, y up = Z, z back = -X)
    const float* q = cam->quat;
    float qn = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    float x = q[0] / qn, y = q[1] / qn, z = q[2] / qn, w = q[3] / qn;
    float Rc[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                   2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                   2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
    for (int r = 0; r < 3; r++) {
        L.R[3 * r + 0] = -Rc[3 * r + 1];
        L.R[3 * r + 1] = Rc[3 * r + 2];
        L.R[3 * r + 2] = -Rc[3 * r + 0];
    }
    const float pi = 3.14159265358979f;
    L.tanx = tanf(0.5f * cam->fovx_deg * pi / 180.0f);
    L.tany = L.tanx * (float)cam->height / (float)cam->width;
    L.fu = 2.0f * L.tanx;               // 2 / proj[0][0] (camera.py:317)
    L.fv = 2.0f * L.tany;               // 2 / proj[1][1] (camera.py:318)
    for (int k = 0; k < 16; k++) L.vinv[k] = view_inv[k];
    L.flags = flags;
    int pixels = cam->width * cam->height;
    if (cam->target_pc && (!cam->segmentation || !cam->pointcloud || cam->target_points < 1 || !h->st.target_object_index))
        return HA_E_ARG;
    hipLaunchKernelGGL(ha_camera_kernel, dim3((pixels + 255) / 256, h->N), dim3(256), 0, (hipStream_t)stream, L);
    HIPCHK(hipGetLastError());
    if (cam->target_pc) {
        CamTargetLaunch T;
        T.pointcloud = cam->pointcloud;
        T.segmentation = cam->segmentation;
        T.target_index = h->st.target_object_index;
        T.out = cam->target_pc;
        T.N = h->N;
        T.HW = pixels;
        T.P = cam->target_points;
        T.seed = h->h_params.seed;
        T.counter = cam->rng_counter;
        hipLaunchKernelGGL(ha_camera_target_kernel, dim3(h->N), dim3(256), 0, (hipStream_t)stream, T);
        HIPCHK(hipGetLastError());
    }
    return HA_OK;
}

int ha_contact_capacity(ha_handle h) { return h ? contact_capacity(h->fam) : HA_E_ARG; }

float ha_last_kernel_ms(ha_handle h) {
    if (!h || !h->timed || !h->t_ev || h->t_count < 1) return -1.0f;
    float ms = -1.0f;
    int k = h->t_count - 1;
    if (hipEventSynchronize(h->t_ev[2 * k + 1]) != hipSuccess) return -1.0f;
    if (hipEventElapsedTime(&ms, h->t_ev[2 * k], h->t_ev[2 * k + 1]) != hipSuccess) return -1.0f;
    return ms;
}

}  // extern "C"

#ifdef HA_PROFILE
// diagnostic build only: per-phase s_memtime totals summed over waves (see PROF in ha_physics.h), 96 counters
extern "C" int ha_profile_read(unsigned long long* out32, int reset) {
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 192) != hipSuccess) return HA_E_HIP;
    if (reset) {
        unsigned long long z[192] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return HA_E_HIP;
    }
    return HA_OK;
}
#endif
#if defined(HA_PROFILE) || defined(HA_ENVT)
// per-workgroup (start, end) stamps of the last launch of a kernel family (n workgroups)
extern "C" int ha_profile_env_times(unsigned long long* out, int n) {
    if (n < 0 || n > 65536) return HA_E_ARG;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_envt), sizeof(unsigned long long) * 2 * n) != hipSuccess) return HA_E_HIP;
    return HA_OK;
}
// (HW_ID, XCC_ID) of each workgroup of that launch
extern "C" int ha_profile_env_hw(unsigned int* out, int n) {
    if (n < 0 || n > 65536) return HA_E_ARG;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_envhw), sizeof(unsigned int) * 2 * n) != hipSuccess) return HA_E_HIP;
    return HA_OK;
}
#endif
