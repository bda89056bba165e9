// ha_pointcloud.h - synthetic point-cloud observables and observation-vector assembly.
//
// References (tasks/hand_arm/...): object_synthetic_pointcloud env/multi_object.py:774-800,
// target_object_synthetic_pointcloud :802-804, goal / relative-goal clouds :383-401,806-809,
// ur5sih_synthetic_pointcloud base/ur5sih.py:347-374, sih_fingertip_pointcloud :337-345, point types
// utils/camera.py:43-47 (PADDING 0, REGULAR 1, TARGET 2, GOAL 3).
//
// HBM-bound streaming: one thread per output point (16 B, one global_store_dwordx4), so a wave writes 1 KB of
// contiguous cloud per store. The pose of each point's body (7 floats of a root/body row, shared by P points)
// and the surface samples (pool table, a few tens of KB) are L2-resident reads; the algorithmic traffic is the
// clouds written plus the pose rows read once per env.
#pragma once
#include "ha_task.h"

// per-launch segment table (host-computed): points per env = sum of the active segment lengths
struct PcLaunch {
    ha_pointcloud_t pc;
    const float* root;            // root_state [N][A][13]
    const float* body;            // rigid_body_state [N][B][13]
    const int64_t* object_indices;
    const int64_t* target_index;
    const float* goal_pos;        // [N][3]
    int N, A, B, a0, NO;
    int seg[7];                   // segment starts: object, target, robot, fingertip, goal, relative goal, end
};

enum { PC_OBJECT = 0, PC_TARGET, PC_ROBOT, PC_FINGERTIP, PC_GOAL, PC_REL_GOAL, PC_END };

__device__ __forceinline__ void pc_pose_point(const float* pose, const float* s, float* v) {
    float r[3];
    ref_quat_apply(pose + 3, s, r);                   // quat_apply(q, sample) (torch_jit_utils.py:70-77)
    v[0] = pose[0] + r[0];
    v[1] = pose[1] + r[1];
    v[2] = pose[2] + r[2];
}

typedef float pc_f4 __attribute__((ext_vector_type(4)));

// per-env inputs of a launch, staged once per workgroup: object poses and pool ids, the poses of the robot
// bodies the clouds read, goal_pos and the target index (a few hundred bytes of scattered row reads done
// once, instead of once per point)
struct PcEnvLDS {
    float obj[HA_MAX_OBJ][8];         // pos xyz, quat xyzw
    float link[HA_PC_MAX_LINKS][8];
    float goal[4];
    int pool[HA_MAX_OBJ];
    int tgt;
    // launch-wide tables, copied per workgroup so every point does one dependent global load (its sample)
    int perm[HA_PC_MAX_P];
    unsigned char slot[HA_PC_MAX_R];
};

// store flavour and table staging are compile-time choices measured by tools/pc_probe.py --variants
#ifndef HA_PC_NT_STORE
#define HA_PC_NT_STORE 1
#endif
#ifndef HA_PC_STAGE_TABLES
#define HA_PC_STAGE_TABLES 0
#endif

__device__ __forceinline__ void pc_store(float* out, const float* v) {
    pc_f4 w = {v[0], v[1], v[2], v[3]};
    if (HA_PC_NT_STORE) __builtin_nontemporal_store(w, reinterpret_cast<pc_f4*>(out));
    else *reinterpret_cast<pc_f4*>(out) = w;
}

// One workgroup per env: the env's inputs go to LDS, then its W points are spread over the 256 threads (no
// per-thread division by W), and the env's output rows are contiguous, so each wave store covers 1 KB of cloud.
extern "C" __global__ void __launch_bounds__(256) ha_pointcloud_kernel(PcLaunch L) {
    __shared__ PcEnvLDS e;
    const int env = blockIdx.x;
    if (env >= L.N) return;
    const ha_pointcloud_t& pc = L.pc;
    const int tid = threadIdx.x, P = pc.P, NO = L.NO;
    if (tid < NO * 7) {
        const int o = tid / 7, k = tid - o * 7;
        e.obj[o][k] = pc.object_pose ? pc.object_pose[((size_t)env * NO + o) * 7 + k]
                                     : L.root[((size_t)env * L.A + L.a0 + o) * 13 + k];
    }
    if (tid < pc.n_links * 7) {
        const int l = tid / 7, k = tid - l * 7;
        e.link[l][k] = L.body[((size_t)env * L.B + pc.links[l]) * 13 + k];
    }
    // device-resident indices are range-checked (an invalid target / pool id / permutation entry reads entry 0
    // instead of faulting); the host wrapper validates them
    if (tid < NO) {
        const int pool = (int)L.object_indices[(size_t)env * NO + tid];
        e.pool[tid] = (unsigned)pool < (unsigned)pc.n_pool ? pool : 0;
    }
    if (tid < 3) e.goal[tid] = L.goal_pos[(size_t)env * 3 + tid];
    if (tid == 0) {
        const int t = (int)L.target_index[env];
        e.tgt = (unsigned)t < (unsigned)NO ? t : 0;
    }
    if (HA_PC_STAGE_TABLES && L.seg[PC_ROBOT] > L.seg[PC_OBJECT])
        for (int j = tid; j < P; j += 256) {
            const int pj = (int)pc.perm[j];
            e.perm[j] = (unsigned)pj < (unsigned)P ? pj : 0;
        }
    if (HA_PC_STAGE_TABLES && L.seg[PC_FINGERTIP] > L.seg[PC_ROBOT])
        for (int r = tid; r < pc.R; r += 256) e.slot[r] = (unsigned char)(pc.robot_slot[r] & (HA_PC_MAX_LINKS - 1));
    __syncthreads();
    const int W = L.seg[PC_END];
    for (int i = tid; i < W; i += 256) {
        float v[4];
        float* out;
        if (i < L.seg[PC_ROBOT]) {
            // object / target clouds: ordered = pos + quat_apply(quat, samples); xyz *= w; then the point axis
            // permuted (multi_object.py:799-800). Target: the target object's row with w *= TARGET (:803-804).
            const bool tgt = i >= L.seg[PC_TARGET];
            int o, j;
            if (tgt) {
                o = e.tgt;
                j = i - L.seg[PC_TARGET];
                out = pc.target_pc + ((size_t)env * P + j) * 4;
            } else {
                o = i / P;
                j = i - o * P;
                out = pc.object_pc + (((size_t)env * NO + o) * P + j) * 4;
            }
            int pj;
            if (HA_PC_STAGE_TABLES) {
                pj = e.perm[j];
            } else {
                pj = (int)pc.perm[j];
                pj = (unsigned)pj < (unsigned)P ? pj : 0;
            }
            const float4 s = reinterpret_cast<const float4*>(pc.object_samples)[(size_t)e.pool[o] * P + pj];
            const float sv[3] = {s.x, s.y, s.z};
            pc_pose_point(e.obj[o], sv, v);
            v[0] *= s.w;
            v[1] *= s.w;
            v[2] *= s.w;
            v[3] = tgt ? s.w * 2.0f : s.w;
        } else if (i < L.seg[PC_FINGERTIP]) {
            // robot cloud: body_pos + quat_apply(body_quat, link-frame samples) (ur5sih.py:366-368); w from the
            // sample
            const int r = i - L.seg[PC_ROBOT];
            const float4 s = reinterpret_cast<const float4*>(pc.robot_samples)[r];
            const float sv[3] = {s.x, s.y, s.z};
            const int sl = HA_PC_STAGE_TABLES ? e.slot[r] : (pc.robot_slot[r] & (HA_PC_MAX_LINKS - 1));
            pc_pose_point(e.link[sl], sv, v);
            v[3] = s.w;
            out = pc.robot_pc + ((size_t)env * pc.R + r) * 4;
        } else if (i < L.seg[PC_GOAL]) {
            // fingertip positions with the fingertip semantic id 3 (ur5sih.py:337-342)
            const int f = i - L.seg[PC_FINGERTIP];
            const float* lp = e.link[pc.fingertip_slot[f]];
            v[0] = lp[0];
            v[1] = lp[1];
            v[2] = lp[2];
            v[3] = 3.0f;
            out = pc.fingertip_pc + ((size_t)env * 5 + f) * 4;
        } else if (i < L.seg[PC_REL_GOAL]) {
            v[0] = e.goal[0];
            v[1] = e.goal[1];
            v[2] = e.goal[2];
            v[3] = 3.0f;                               // PointType.GOAL (multi_object.py:387)
            out = pc.goal_pc + (size_t)env * 4;
        } else {
            // relative goal: quat_apply(quat_conjugate(flange_quat), goal_pos - flange_pos) (multi_object.py:806-809)
            const float* fl = e.link[pc.flange_slot];
            const float d[3] = {e.goal[0] - fl[0], e.goal[1] - fl[1], e.goal[2] - fl[2]};
            const float qc[4] = {-fl[3], -fl[4], -fl[5], fl[6]};
            ref_quat_apply(qc, d, v);
            v[3] = 3.0f;
            out = pc.relative_goal_pc + (size_t)env * 4;
        }
        pc_store(out, v);
    }
}

// observation-vector assembly for a custom observation list (observable_vec_task.py:183-192): column k of
// out[N][n_cols] = sources[src[k]][env * stride[src[k]] + col[k]]. One thread per output float.
struct ObsGather {
    const float* src[HA_MAX_OBS_SOURCES];
    int stride[HA_MAX_OBS_SOURCES];
    const int32_t* cols;          // [n_cols][2] (source | HA_OBS_SRC_TARGET, column)
    const int64_t* target;        // target_object_index (for HA_OBS_SRC_TARGET columns)
    float* out;
    int N, n_cols;
};

extern "C" __global__ void __launch_bounds__(256) ha_obs_gather_kernel(ObsGather g) {
    unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= (unsigned)g.N * (unsigned)g.n_cols) return;
    const int env = (int)(t / (unsigned)g.n_cols), k = (int)(t % (unsigned)g.n_cols);
    const int sc = g.cols[2 * k], s = sc & (HA_OBS_SRC_TARGET - 1);
    long long c = g.cols[2 * k + 1];
    if ((sc & HA_OBS_SRC_TARGET) && g.target) c += g.target[env] * 13;
    const float* src = g.src[0];
    int stride = g.stride[0];
#pragma unroll
    for (int q = 1; q < HA_MAX_OBS_SOURCES; q++)
        if (s == q) {
            src = g.src[q];
            stride = g.stride[q];
        }
    g.out[t] = src[(size_t)env * stride + c];
}
