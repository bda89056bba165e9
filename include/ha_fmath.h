/* ha_fmath.h - float32 sine / cosine shared by the HIP kernels (csrc/ha_physics.h) and the C oracle
 * (oracle/physics_oracle.c).
 *
 * Device sinf/cosf (ROCm ocml) and glibc sinf/cosf are different implementations; each is accurate to about
 * 1 ulp, but they round differently on a small fraction of arguments. Inside the physics step one ulp of a
 * joint rotation is amplified by the stiff finger chains, so a libm mismatch alone makes the GPU and the
 * oracle disagree. Both sides therefore evaluate this one explicit sequence of IEEE float32 operations
 * (multiply, add, floor, compare; built with -ffp-contract=off on both sides, so no fused multiply-add),
 * which gives bit-identical results on the two compilers.
 *
 * Algorithm: Cody-Waite reduction by pi/2 with a three-part constant (the first two parts have short
 * mantissas, so k * part is exact for |k| < 2^12), then minimax polynomials on [-pi/4, pi/4] (Cephes sinf /
 * cosf coefficients). Max error about 1 ulp for |x| < 4096 (the physics only passes half joint angles,
 * |x| < 4).
 */
#ifndef HA_FMATH_H
#define HA_FMATH_H

#ifdef __HIPCC__
#define HA_FM_FN __host__ __device__ static inline
#else
#define HA_FM_FN static inline
#endif

HA_FM_FN float ha_floorf_(float x) {
#ifdef __HIPCC__
    return __builtin_floorf(x);
#else
    return __builtin_floorf(x);
#endif
}

/* sin and cos of x in one reduction */
HA_FM_FN void ha_sincosf(float x, float* s_out, float* c_out) {
    const float two_over_pi = 0.636619772367581343f;
    const float p1 = 1.5703125f;                 /* pi/2 split: 8 + 12 + 24 significant bits */
    const float p2 = 4.83751296997070312e-4f;
    const float p3 = 7.54978995489188216e-8f;
    float k = ha_floorf_(x * two_over_pi + 0.5f);
    float r = ((x - k * p1) - k * p2) - k * p3;
    float z = r * r;
    float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
    float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
               - 0.5f * z + 1.0f;
    /* quadrant q = k mod 4: (sin, cos) = (sp, cp), (cp, -sp), (-sp, -cp), (-cp, sp) */
    float kq = k - 4.0f * ha_floorf_(k * 0.25f);
    int q = (int)kq;
    float s = (q & 1) ? cp : sp;
    float c = (q & 1) ? sp : cp;
    if (q == 1 || q == 2) c = -c;
    if (q >= 2) s = -s;
    *s_out = s;
    *c_out = c;
}

#undef HA_FM_FN
#endif
