// ha_device.h - gfx950 device helpers: small vector/quaternion math and wavefront (64-lane) primitives.
// One environment is simulated by one 64-lane wavefront; `lane` = threadIdx.x.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ha_fmath.h"

#define HD __device__ __forceinline__

struct f3 { float x, y, z; };
struct qf { float x, y, z, w; };

HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
HD float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
HD f3 cross3(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
HD f3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }
HD void st3(float* p, f3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
HD qf ldq(const float* p) { return qf{p[0], p[1], p[2], p[3]}; }
HD void stq(float* p, qf q) { p[0] = q.x; p[1] = q.y; p[2] = q.z; p[3] = q.w; }

// Hamilton product (same expression as the C oracle)
HD qf qmul(qf a, qf b) {
    return qf{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
              a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
HD f3 qrot(qf q, f3 v) {
    f3 u = mk3(q.x, q.y, q.z);
    f3 t = cross3(u, v) * 2.0f;
    return (v + t * q.w) + cross3(u, t);
}
HD qf qnormalize(qf q) {
    float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return qf{q.x / n, q.y / n, q.z / n, q.w / n};
}
// sin / cos from the shared ha_sincosf (include/ha_fmath.h): the same float32 operations as the C oracle
HD qf qaxis(f3 a, float ang) {
    float s, c;
    ha_sincosf(0.5f * ang, &s, &c);
    return qf{a.x * s, a.y * s, a.z * s, c};
}
HD void qmat(qf q, float R[9]) {
    float x = q.x, y = q.y, z = q.z, w = q.w;
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
HD f3 mv3(const float M[9], f3 v) {
    return mk3(M[0] * v.x + M[1] * v.y + M[2] * v.z, M[3] * v.x + M[4] * v.y + M[5] * v.z,
               M[6] * v.x + M[7] * v.y + M[8] * v.z);
}
HD void rart3(const float R[9], const float* A, float out[9]) {
    float T[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) T[i * 3 + j] = R[i * 3] * A[j] + R[i * 3 + 1] * A[3 + j] + R[i * 3 + 2] * A[6 + j];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            out[i * 3 + j] = T[i * 3] * R[j * 3] + T[i * 3 + 1] * R[j * 3 + 1] + T[i * 3 + 2] * R[j * 3 + 2];
}
HD void inv3(const float A[9], float out[9]) {
    float c0 = A[4] * A[8] - A[5] * A[7], c1 = A[5] * A[6] - A[3] * A[8], c2 = A[3] * A[7] - A[4] * A[6];
    float det = A[0] * c0 + A[1] * c1 + A[2] * c2;
    float id = 1.0f / det;
    out[0] = c0 * id; out[1] = (A[2] * A[7] - A[1] * A[8]) * id; out[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    out[3] = c1 * id; out[4] = (A[0] * A[8] - A[2] * A[6]) * id; out[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    out[6] = c2 * id; out[7] = (A[1] * A[6] - A[0] * A[7]) * id; out[8] = (A[0] * A[4] - A[1] * A[3]) * id;
}

// ---------------------------------------------------------------- wavefront primitives (wave64)
HD int lane_id() { return threadIdx.x & 63; }
// Block == one wavefront (every env kernel is __launch_bounds__(64)): lanes exchange data through LDS (and the
// env's global rows) inside one wave, whose memory operations the hardware performs in program order. A
// wavefront-scope release / acquire pair is then all the ordering needed: it stops the compiler from moving
// memory operations across the point, and unlike __syncthreads() (workgroup scope: s_waitcnt lgkmcnt(0) at every
// call even with the s_barrier elided for one wave) it does not stall on in-flight LDS and scalar loads.
#ifdef HA_X_WSYNC_BLOCK     /* A/B: the workgroup-scope barrier */
HD void wsync() { __syncthreads(); }
#else
HD void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif

// value of lane `src` in every lane; src must be wave-uniform (v_readlane_b32 -> SGPR)
HD float bcast(float x, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src));
}
HD int bcast_i(int x, int src) { return __builtin_amdgcn_readlane(x, src); }

// Reductions: DPP inside each 16-lane row (quad_perm xor1, xor2, row_half_mirror, row_mirror leave the
// row's result in all 16 lanes), then across rows with row_bcast:15 (row 3 += row 2, row 1 += row 0) and
// row_bcast:31 (rows 2, 3 += lane 31), and the result read from lane 63 (one v_readlane). Lane 63 holds
// (r3 op r2) op (r1 op r0) of the four row results r0..r3, which for + is bitwise the (r0 + r1) + (r2 + r3)
// the oracle's wave_dot emulates (IEEE addition is commutative). No LDS round trips (a __shfl_xor is a
// ds_bpermute). Results are wave-uniform.
#define HA_DPP(x, ctrl) __builtin_amdgcn_mov_dpp((x), (ctrl), 0xF, 0xF, true)
template <int CTRL>
HD float dpp_f(float x) { return __int_as_float(HA_DPP(__float_as_int(x), CTRL)); }
template <int CTRL>
HD int dpp_i(int x) { return HA_DPP(x, CTRL); }
// cross-row steps: lanes outside the row mask get `old` (only lane 63's result is read)
template <int CTRL, int RM>
HD float dpp_row_f(float old, float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), CTRL, RM, 0xF, false));
}
template <int CTRL, int RM>
HD int dpp_row_i(int old, int x) { return __builtin_amdgcn_update_dpp(old, x, CTRL, RM, 0xF, false); }
HD float lane63(float x) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63)); }

// sum of the four row results: (r3 + r2) + (r1 + r0) in lane 63
HD float rows_sum(float x) {
    x = x + dpp_row_f<0x142, 0xA>(0.0f, x);
    x = x + dpp_row_f<0x143, 0xC>(0.0f, x);
    return lane63(x);
}
HD float wave_max(float x) {
    x = fmaxf(x, dpp_f<0xB1>(x));
    x = fmaxf(x, dpp_f<0x4E>(x));
    x = fmaxf(x, dpp_f<0x141>(x));
    x = fmaxf(x, dpp_f<0x140>(x));
    x = fmaxf(x, dpp_row_f<0x142, 0xA>(x, x));
    x = fmaxf(x, dpp_row_f<0x143, 0xC>(x, x));
    return lane63(x);
}
HD float wave_min(float x) {
    x = fminf(x, dpp_f<0xB1>(x));
    x = fminf(x, dpp_f<0x4E>(x));
    x = fminf(x, dpp_f<0x141>(x));
    x = fminf(x, dpp_f<0x140>(x));
    x = fminf(x, dpp_row_f<0x142, 0xA>(x, x));
    x = fminf(x, dpp_row_f<0x143, 0xC>(x, x));
    return lane63(x);
}
HD int wave_min_i(int x) {
    x = min(x, dpp_i<0xB1>(x));
    x = min(x, dpp_i<0x4E>(x));
    x = min(x, dpp_i<0x141>(x));
    x = min(x, dpp_i<0x140>(x));
    x = min(x, dpp_row_i<0x142, 0xA>(x, x));
    x = min(x, dpp_row_i<0x143, 0xC>(x, x));
    return __builtin_amdgcn_readlane(x, 63);
}
// arg-min / arg-max with ties broken toward the smaller index (matches a sequential strict-compare
// scan): the extreme value first, then the smallest index among the lanes that hold it.
HD void wave_argmin(float& v, int& i) {
    float m = wave_min(v);
    i = wave_min_i(v == m ? i : 0x7fffffff);
    v = m;
}
HD void wave_argmax(float& v, int& i) {
    float m = wave_max(v);
    i = wave_min_i(v == m ? i : 0x7fffffff);
    v = m;
}

