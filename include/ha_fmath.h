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

/* Natural logarithm and exponential for the domain-randomization samplers (loguniform, Box-Muller gaussian), shared
 * for the same reason: the C oracle and numpy (oracle/f32.py) restate the samples bit for bit. Cephes logf / expf:
 * the argument split by its exponent bits (log) or by round(x / ln 2) with a two-part ln 2 (exp), then a minimax
 * polynomial; about 1 ulp. ha_logf takes positive normal arguments (the samplers' u >= 2^-24 and positive ranges);
 * ha_expf clamps its result exponent to the normal range. */
HA_FM_FN float ha_bits_float_(int i) {
    union { int i; float f; } u;
    u.i = i;
    return u.f;
}
HA_FM_FN int ha_float_bits_(float f) {
    union { int i; float f; } u;
    u.f = f;
    return u.i;
}
HA_FM_FN float ha_logf(float x) {
    int ix = ha_float_bits_(x);
    int e = ((ix >> 23) & 0xff) - 126;                        /* x = m 2^e, m in [0.5, 1) */
    float m = ha_bits_float_((ix & 0x007fffff) | 0x3f000000);
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = (m + m) - 1.0f;
    } else {
        m = m - 1.0f;
    }
    float z = m * m;
    float y = ((((((((7.0376836292e-2f * m - 1.1514610310e-1f) * m + 1.1676998740e-1f) * m - 1.2420140846e-1f) * m
                   + 1.4249322787e-1f) * m - 1.6668057665e-1f) * m + 2.0000714765e-1f) * m - 2.4999993993e-1f) * m
               + 3.3333331174e-1f) * m * z;
    float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    return r + 0.693359375f * fe;
}
HA_FM_FN float ha_expf(float x) {
    x = x > 88.0f ? 88.0f : (x < -87.0f ? -87.0f : x);
    float z = ha_floorf_(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    float xx = x * x;
    float y = (((((1.9875691500e-4f * x + 1.3981999507e-3f) * x + 8.3334519073e-3f) * x + 4.1665795894e-2f) * x
                + 1.6666665459e-1f) * x + 5.0000001201e-1f) * xx + x + 1.0f;
    return y * ha_bits_float_((n + 127) << 23);
}

#undef HA_FM_FN
#endif
