// ha_camera.h - camera sensors of Ur5SihMultiObject: depth and segmentation images ray-cast
// against the collision geometry, and the camera point cloud computed from the depth image.
//
// References (tasks/hand_arm/...): CameraSensorProperties / IsaacGymCameraSensor utils/camera.py:84-333
// (pose, fovx, resolution; depth, segmentation and point-cloud images), depth_image_to_global_points :50-69,
// _compute_pointcloud :302-311, segmentation ids env/multi_object.py:581-642 + base/ur5sih.py:123-125
// (table 0, robot 1, bin 2, object i 3 + i, goal 3 + num_objects).
//
// Isaac Gym rasterises the visual meshes with its closed renderer; here every pixel's ray is intersected with the
// convex collision hulls the physics uses (robot links, objects, static boxes), the goal sphere and the ground
// plane, so images match the simulated geometry, not the visual meshes ("parity unpinned" against the renderer).
// The depth-to-points arithmetic follows camera.py:50-69 step by step and is pinned by reference goldens.
//
// Launch: grid (pixel tiles of 256, envs). The env's hull poses and world bounding spheres are staged in LDS once
// per workgroup; each thread casts one ray: a sphere test per hull (front-to-back pruned), then the plane slab of
// the hull in its own frame (local planes read from the model, L1/L2-resident).
#pragma once
#include "ha_task.h"

#define HA_CAM_MAX_HULLS (HA_MAX_HULLS + 1)

struct CamLaunch {
    ha_camera_t cam;
    const ha_model_t* m;
    const float* root;          // root_state [N][A][13]
    const float* body;          // rigid_body_state [N][B][13]
    const int64_t* object_indices;
    const float* goal_pos;      // [N][3]
    int N, A, B, a0, NO, body_robot0, n_link_hulls, n_static;
    float R[9];                 // view axes in the env frame, row-major columns: x right, y up, z back
    float vinv[16];             // inverse view matrix (row-vector convention), host-computed
    float tanx, tany, fu, fv;
    uint32_t flags;
};

struct CamHullLDS {
    float p[4], qi[4];          // hull body pose: origin, inverse rotation
    float c[4];                 // world bounding sphere: centre, radius in c[3]
    int hull, seg, pad0, pad1;
};

__device__ __forceinline__ f3 cam_qrot(const float* q, f3 v) { return qrot(qf{q[0], q[1], q[2], q[3]}, v); }

extern "C" __global__ void __launch_bounds__(256) ha_camera_kernel(CamLaunch L) {
    __shared__ CamHullLDS hl[HA_CAM_MAX_HULLS];
    const int env = blockIdx.y;
    const ha_camera_t& cam = L.cam;
    const ha_model_t& m = *L.m;
    const int tid = threadIdx.x;
    const int W = cam.width, H = cam.height;
    // this env's hull list: link hulls, then every convex piece of each object (ha_model_t v8), then static boxes
    int n_pieces = 0;
    for (int o = 0; o < L.NO; o++) {
        int pool = (int)L.object_indices[(size_t)env * L.NO + o];
        pool = (unsigned)pool < (unsigned)m.n_pool ? pool : 0;
        n_pieces += m.pool_nhull[pool];
    }
    const int NH = L.n_link_hulls + n_pieces + L.n_static;
    const bool cast = !(L.flags & HA_CAM_FROM_DEPTH);
    if (cast && tid < NH) {
        const int k = tid;
        int hull, seg;
        float p[3], q[4];
        if (k < L.n_link_hulls) {
            hull = k;
            seg = 1;                                                   // robot (ur5sih.py:123)
            const float* r = L.body + ((size_t)env * L.B + L.body_robot0 + m.hull_link[k]) * 13;
            p[0] = r[0]; p[1] = r[1]; p[2] = r[2];
            q[0] = r[3]; q[1] = r[4]; q[2] = r[5]; q[3] = r[6];
        } else if (k < L.n_link_hulls + n_pieces) {
            int o = 0, j = k - L.n_link_hulls, pool = 0;
            for (; o < L.NO; o++) {
                pool = (int)L.object_indices[(size_t)env * L.NO + o];
                pool = (unsigned)pool < (unsigned)m.n_pool ? pool : 0;
                if (j < m.pool_nhull[pool]) break;
                j -= m.pool_nhull[pool];
            }
            hull = m.pool_hull[pool] + j;
            seg = 3 + o;                                               // multi_object.py:642
            const float* r = L.root + ((size_t)env * L.A + L.a0 + o) * 13;
            p[0] = r[0]; p[1] = r[1]; p[2] = r[2];
            q[0] = r[3]; q[1] = r[4]; q[2] = r[5]; q[3] = r[6];
        } else {
            const int s = k - L.n_link_hulls - n_pieces;
            hull = m.static_hull[s];
            seg = cam.static_seg[s];
            p[0] = m.static_pos[s][0]; p[1] = m.static_pos[s][1]; p[2] = m.static_pos[s][2];
            q[0] = m.static_quat[s][0]; q[1] = m.static_quat[s][1]; q[2] = m.static_quat[s][2];
            q[3] = m.static_quat[s][3];
        }
        CamHullLDS& e = hl[k];
        e.p[0] = p[0]; e.p[1] = p[1]; e.p[2] = p[2];
        e.qi[0] = -q[0]; e.qi[1] = -q[1]; e.qi[2] = -q[2]; e.qi[3] = q[3];
        const f3 cw = mk3(p[0], p[1], p[2]) + cam_qrot(q, ld3(m.hull_center[hull]));
        e.c[0] = cw.x; e.c[1] = cw.y; e.c[2] = cw.z; e.c[3] = m.hull_radius[hull];
        e.hull = hull;
        e.seg = seg;
    }
    __syncthreads();
    const int pix = blockIdx.x * 256 + tid;
    if (pix >= W * H) return;
    const int row = pix / W, col = pix - row * W;
    const size_t out = (size_t)env * W * H + pix;
    float depth;
    if (cast) {
        // ray through pixel (col, row): view direction (x, y, -1) with x = (col - W/2)/W * 2 tan(fovx/2),
        // y = -(row - H/2)/H * 2 tan(fovy/2) -- the inverse of camera.py:57-63, so a hit maps back onto its pixel
        const float xv = ((float)col - 0.5f * (float)W) / (float)W * (2.0f * L.tanx);
        const float yv = -(((float)row - 0.5f * (float)H) / (float)H) * (2.0f * L.tany);
        const f3 o = mk3(cam.pos[0], cam.pos[1], cam.pos[2]);
        const f3 d = mk3(L.R[0] * xv + L.R[1] * yv - L.R[2], L.R[3] * xv + L.R[4] * yv - L.R[5],
                         L.R[6] * xv + L.R[7] * yv - L.R[8]);
        const float dd = dot3(d, d);
        const float inv_len = 1.0f / sqrtf(dd);
        float best = 3.0e38f;
        int bseg = 0;
        if (d.z < 0.0f) {                                              // ground plane z = 0 (ur5sih.py:159-167)
            const float t = -o.z / d.z;
            if (t > 0.0f) { best = t; bseg = 0; }
        }
        {                                                              // goal sphere (visual only, multi_object.py:581)
            const float* g = L.goal_pos + (size_t)env * 3;
            const f3 oc = o - mk3(g[0], g[1], g[2]);
            const float b = dot3(oc, d), c = dot3(oc, oc) - cam.goal_radius * cam.goal_radius;
            const float disc = b * b - dd * c;
            if (disc >= 0.0f) {
                const float t = (-b - sqrtf(disc)) / dd;
                if (t > 0.0f && t < best) { best = t; bseg = 3 + L.NO; }
            }
        }
        for (int k = 0; k < NH; k++) {
            const CamHullLDS& e = hl[k];
            const f3 oc = mk3(e.c[0], e.c[1], e.c[2]) - o;
            const float tc = dot3(oc, d) / dd;                         // closest approach to the sphere centre
            const f3 off = oc - d * tc;
            const float r = e.c[3];
            if (dot3(off, off) > r * r) continue;
            if (tc - 1.001f * r * inv_len > best) continue;              // entirely behind the best hit
            // slab over the hull's planes (n . x + d <= 0 inside), ray in the hull frame
            const f3 ol = cam_qrot(e.qi, o - mk3(e.p[0], e.p[1], e.p[2]));
            const f3 dl = cam_qrot(e.qi, d);
            float t0 = 0.0f, t1 = best;
            const int ps = m.hull_plane_start[e.hull], np = m.hull_nplanes[e.hull];
            bool hit = true;
            for (int i = 0; i < np; i++) {
                const float4 pl = reinterpret_cast<const float4*>(m.planes)[ps + i];
                const f3 n = mk3(pl.x, pl.y, pl.z);
                const float num = -(dot3(n, ol) + pl.w), den = dot3(n, dl);
                if (den < 0.0f) {
                    const float t = num / den;
                    t0 = t > t0 ? t : t0;
                } else if (den > 0.0f) {
                    const float t = num / den;
                    t1 = t < t1 ? t : t1;
                } else if (num < 0.0f) {
                    hit = false;
                }
                if (t0 > t1) { hit = false; break; }
            }
            if (hit && t0 > 0.0f && t0 < best) { best = t0; bseg = e.seg; }
        }
        const bool any = best < 3.0e38f;
        depth = any ? -best : -INFINITY;                               // OpenGL view z of the hit (negative)
        if (cam.depth) cam.depth[out] = depth;
        if (cam.segmentation) cam.segmentation[out] = any ? bseg : 0;
    } else {
        depth = cam.depth[out];
    }
    if (cam.pointcloud) {
        // _compute_pointcloud (camera.py:302-311) with depth_image_to_global_points (:50-69): clamp, pixel ->
        // view coordinates scaled by depth, x proj (fu, fv, 1), homogeneous x inverse view matrix, workspace test
        const float dep = fmaxf(depth, -cam.max_depth);
        float x0 = -((float)col - 0.5f * (float)W) / (float)W;
        float y0 = ((float)row - 0.5f * (float)H) / (float)H;
        x0 = x0 * dep;
        y0 = y0 * dep;
        const float h0 = x0 * L.fu, h1 = y0 * L.fv, h2 = dep;
        float xyz[3];
#pragma unroll
        for (int j = 0; j < 3; j++)
            xyz[j] = ((h0 * L.vinv[0 * 4 + j] + h1 * L.vinv[1 * 4 + j]) + h2 * L.vinv[2 * 4 + j]) + L.vinv[3 * 4 + j];
        const bool valid = depth > -cam.max_depth && xyz[0] > cam.workspace[0] && xyz[0] < cam.workspace[1] &&
                           xyz[1] > cam.workspace[2] && xyz[1] < cam.workspace[3];
        float4 v4 = make_float4(xyz[0], xyz[1], xyz[2], valid ? 1.0f : 0.0f);
        reinterpret_cast<float4*>(cam.pointcloud)[out] = v4;
    }
}

// {camera}_target_object_pointcloud (_refresh_segmented_pointcloud, multi_object.py:837-855): the camera points
// whose segmentation is the target object's (3 + target index), in pixel order; more than P of them -> a uniformly
// random subset of P (the reference: torch.randperm(len)[:P]; here the P smallest per-pixel hash keys, exact
// radix select, written in pixel order), fewer -> zero padding; then w *= TARGET (2).
// One workgroup per env; thread t owns the contiguous pixel strip [t C, (t + 1) C), so block prefix sums keep
// pixel order.
struct CamTargetLaunch {
    const float* pointcloud;      // [N][H*W][4]
    const int32_t* segmentation;  // [N][H*W]
    const int64_t* target_index;  // [N]
    float* out;                   // [N][P][4]
    int N, HW, P;
    uint64_t seed;
    uint32_t counter;
};

__device__ __forceinline__ uint32_t cam_key(uint64_t seed, uint32_t counter, uint32_t env, uint32_t pix) {
    return mix32(mix32(mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + counter)) + env) + pix * 0x9E3779B9u);
}

// exclusive block prefix sum of one int per thread (256 threads); returns the total
__device__ __forceinline__ int cam_block_scan(int v, int* sh, int& total) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        int x = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += x;
        __syncthreads();
    }
    total = sh[255];
    int excl = sh[tid] - v;
    __syncthreads();
    return excl;
}

extern "C" __global__ void __launch_bounds__(256) ha_camera_target_kernel(CamTargetLaunch L) {
    __shared__ int sh[256];
    __shared__ int hist[256];
    __shared__ uint32_t s_prefix;
    __shared__ int s_need;
    const int env = blockIdx.x, tid = threadIdx.x;
    const int C = (L.HW + 255) / 256;
    const int p0 = tid * C, p1 = min(p0 + C, L.HW);
    const int tgt = 3 + (int)L.target_index[env];
    const int32_t* seg = L.segmentation + (size_t)env * L.HW;
    const float4* pc = reinterpret_cast<const float4*>(L.pointcloud) + (size_t)env * L.HW;
    float4* out = reinterpret_cast<float4*>(L.out) + (size_t)env * L.P;
    int mine = 0;
    for (int p = p0; p < p1; p++) mine += seg[p] == tgt;
    int K;
    int off = cam_block_scan(mine, sh, K);
    if (K <= L.P) {
        // all target points in pixel order, then zero padding (multi_object.py:848-850)
        int j = off;
        for (int p = p0; p < p1; p++)
            if (seg[p] == tgt) {
                float4 v = pc[p];
                v.w *= 2.0f;
                out[j++] = v;
            }
        for (int j2 = K + tid; j2 < L.P; j2 += 256) out[j2] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    // K > P: the P smallest keys among the target pixels (radix select over 4 bytes, most significant first)
    uint32_t prefix = 0;
    int need = L.P;                 // how many of the remaining candidates (keys with this prefix) to take
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[tid] = 0;
        __syncthreads();
        const uint32_t hi_mask = shift == 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
        for (int p = p0; p < p1; p++) {
            if (seg[p] != tgt) continue;
            const uint32_t k = cam_key(L.seed, L.counter, env, p);
            if ((k & hi_mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0, b = 0;
            for (; b < 256; b++) {
                if (acc + hist[b] >= need) break;
                acc += hist[b];
            }
            s_prefix = prefix | ((uint32_t)b << shift);
            s_need = need - acc;
        }
        __syncthreads();
        prefix = s_prefix;
        need = s_need;
    }
    // selected: key < T, plus the first `need` pixels (pixel order) whose key == T
    const uint32_t T = prefix;
    int lt = 0, eq = 0;
    for (int p = p0; p < p1; p++) {
        if (seg[p] != tgt) continue;
        const uint32_t k = cam_key(L.seed, L.counter, env, p);
        lt += k < T;
        eq += k == T;
    }
    int nlt, neq;
    const int off_lt = cam_block_scan(lt, sh, nlt);
    const int off_eq = cam_block_scan(eq, sh, neq);
    // output slots in pixel order: a selected pixel's slot = (selected pixels before it)
    int sel_here = lt + max(0, min(eq, need - off_eq));
    int tot;
    int j = cam_block_scan(sel_here, sh, tot);
    (void)off_lt;
    int eq_seen = off_eq;
    for (int p = p0; p < p1; p++) {
        if (seg[p] != tgt) continue;
        const uint32_t k = cam_key(L.seed, L.counter, env, p);
        bool take = k < T;
        if (k == T) {
            take = eq_seen < need;
            eq_seen++;
        }
        if (take) {
            float4 v = pc[p];
            v.w *= 2.0f;
            out[j++] = v;
        }
    }
}
