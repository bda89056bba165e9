/* ha_obb.h - the oriented-box mid-phase of the robot's link-link (self-collision) pairs, shared by the HIP kernels
 * (csrc/ha_physics.h detect) and the C oracle (oracle/physics_oracle.c detect).
 *
 * One text for both sides, so both evaluate the same float32 operations in the same order (each is built with
 * -ffp-contract=off) and cull exactly the same pairs.
 *
 * A link hull's box (ha_model_t.hull_obb: centre, half extents and orientation in the link frame; tools/build_model.py
 * fits it to the hull's vertices) is posed by its link and tested against the other's on the 15 axes of the
 * separating-axis theorem for boxes (Gottschalk, Lin and Manocha 1996), each grown by the contact margin. A pair
 * separated on any axis cannot touch within the margin, so its narrow phase is skipped. The test is conservative:
 * the nine edge-edge axes keep their unnormalised length (|A_i x B_j| <= 1), which only shrinks the projected
 * extents against the margin, and every |R_ij| carries 1e-6 for nearly parallel axes.
 */
#ifndef HA_OBB_H
#define HA_OBB_H

#ifdef __HIPCC__
#define HA_OB_FN __host__ __device__ static inline
#else
#define HA_OB_FN static inline
#endif

/* world box of a link hull: link pose lp[3], lq[4] (xyzw) and the hull_obb record ob (centre[3], half[3], quat[4] in
 * the link frame) -> centre c[3] and the box axes as the columns of R (row-major 3 x 3) */
HA_OB_FN void ha_obb_world(const float* lp, const float* lq, const float* ob, float* c, float* R) {
    float x = lq[0], y = lq[1], z = lq[2], w = lq[3];
    float bx = ob[6], by = ob[7], bz = ob[8], bw = ob[9];
    /* q = lq * q_box (Hamilton product) */
    float qx = w * bx + x * bw + y * bz - z * by;
    float qy = w * by - x * bz + y * bw + z * bx;
    float qz = w * bz + x * by - y * bx + z * bw;
    float qw = w * bw - x * bx - y * by - z * bz;
    R[0] = 1.0f - 2.0f * (qy * qy + qz * qz); R[1] = 2.0f * (qx * qy - qz * qw); R[2] = 2.0f * (qx * qz + qy * qw);
    R[3] = 2.0f * (qx * qy + qz * qw); R[4] = 1.0f - 2.0f * (qx * qx + qz * qz); R[5] = 2.0f * (qy * qz - qx * qw);
    R[6] = 2.0f * (qx * qz - qy * qw); R[7] = 2.0f * (qy * qz + qx * qw); R[8] = 1.0f - 2.0f * (qx * qx + qy * qy);
    /* c = lp + rot(lq) centre: t = 2 (u x v), v + w t + u x t */
    float vx = ob[0], vy = ob[1], vz = ob[2];
    float tx = 2.0f * (y * vz - z * vy), ty = 2.0f * (z * vx - x * vz), tz = 2.0f * (x * vy - y * vx);
    c[0] = lp[0] + ((vx + w * tx) + (y * tz - z * ty));
    c[1] = lp[1] + ((vy + w * ty) + (z * tx - x * tz));
    c[2] = lp[2] + ((vz + w * tz) + (x * ty - y * tx));
}

/* radius of a box's circumscribed sphere (half extents h) */
HA_OB_FN float ha_obb_radius(const float* h) { return sqrtf((h[0] * h[0] + h[1] * h[1]) + h[2] * h[2]); }

/* the circumscribed spheres (centres ca, cb, radii ra, rb from ha_obb_radius) within the margin mg */
HA_OB_FN int ha_obb_spheres_near(const float* ca, float ra, const float* cb, float rb, float mg) {
    float T0 = cb[0] - ca[0], T1 = cb[1] - ca[1], T2 = cb[2] - ca[2];
    float rs = (ra + rb) + mg;
    return !((T0 * T0 + T1 * T1) + T2 * T2 > rs * rs);
}

/* boxes (ca, Ra, half extents ha) and (cb, Rb, hb) not separated by more than mg on any of the 15 SAT axes */
HA_OB_FN int ha_obb_sat(const float* ca, const float* Ra, const float* ha, const float* cb, const float* Rb,
                        const float* hb, float mg) {
    float T0 = cb[0] - ca[0], T1 = cb[1] - ca[1], T2 = cb[2] - ca[2];
    float R[3][3], AR[3][3], t[3];
    for (int i = 0; i < 3; i++) {
        t[i] = (Ra[i] * T0 + Ra[3 + i] * T1) + Ra[6 + i] * T2;
        for (int j = 0; j < 3; j++) {
            R[i][j] = (Ra[i] * Rb[j] + Ra[3 + i] * Rb[3 + j]) + Ra[6 + i] * Rb[6 + j];
            AR[i][j] = (R[i][j] < 0.0f ? -R[i][j] : R[i][j]) + 1e-6f;
        }
    }
    for (int i = 0; i < 3; i++) {           /* A's axes */
        float rb = (hb[0] * AR[i][0] + hb[1] * AR[i][1]) + hb[2] * AR[i][2];
        float d = t[i] < 0.0f ? -t[i] : t[i];
        if (d > (ha[i] + rb) + mg) return 0;
    }
    for (int j = 0; j < 3; j++) {           /* B's axes */
        float ra = (ha[0] * AR[0][j] + ha[1] * AR[1][j]) + ha[2] * AR[2][j];
        float tb = (t[0] * R[0][j] + t[1] * R[1][j]) + t[2] * R[2][j];
        float d = tb < 0.0f ? -tb : tb;
        if (d > (ra + hb[j]) + mg) return 0;
    }
    for (int i = 0; i < 3; i++) {           /* A_i x B_j */
        int i1 = i == 2 ? 0 : i + 1, i2 = i == 0 ? 2 : i - 1;
        for (int j = 0; j < 3; j++) {
            int j1 = j == 2 ? 0 : j + 1, j2 = j == 0 ? 2 : j - 1;
            float tl = t[i2] * R[i1][j] - t[i1] * R[i2][j];
            float ra = ha[i1] * AR[i2][j] + ha[i2] * AR[i1][j];
            float rb = hb[j1] * AR[i][j2] + hb[j2] * AR[i][j1];
            float d = tl < 0.0f ? -tl : tl;
            if (d > (ra + rb) + mg) return 0;
        }
    }
    return 1;
}

/* boxes (ca, Ra, half extents ha) and (cb, Rb, hb) within the margin mg of each other: their circumscribed spheres
 * first (one distance), then all 15 SAT axes */
HA_OB_FN int ha_obb_near(const float* ca, const float* Ra, const float* ha, const float* cb, const float* Rb,
                         const float* hb, float mg) {
    if (!ha_obb_spheres_near(ca, ha_obb_radius(ha), cb, ha_obb_radius(hb), mg)) return 0;
    return ha_obb_sat(ca, Ra, ha, cb, Rb, hb, mg);
}

/* Two posed boxes within the margin on all 15 axes, from the bodies' poses (p, q xyzw) and the boxes' records ob
 * (centre, half extents, quat in the body frame): ha_obb_world of each, then ha_obb_sat - the compound piece-pair cull
 * of the step kernels and the oracle (round 6). (A form in box A's frame from the relative quaternion held half the
 * live values and removed the kernels' spills, but measured 2% slower on C4 / C4w / C5: profiles/r06_ab_*) */
HA_OB_FN int ha_obb_pair_near(const float* p1, const float* q1, const float* ob1, const float* p2, const float* q2,
                              const float* ob2, float mg) {
    float c1[3], R1[9], c2[3], R2[9];
    ha_obb_world(p1, q1, ob1, c1, R1);
    ha_obb_world(p2, q2, ob2, c2, R2);
    return ha_obb_sat(c1, R1, ob1 + 3, c2, R2, ob2 + 3, mg);
}

#undef HA_OB_FN
#endif
