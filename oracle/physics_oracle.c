/*
 * ORACLE (test infrastructure only) - scalar C restatement of the hand-arm simulator + task step.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library
 * (oracle/_build/libhandarm_oracle.so), and only as the checker / CPU baseline; the product path
 * (libhandarm_hip.so) never links or calls it.
 *
 * Physics: Isaac Gym / PhysX is a closed binary that is absent here, so PHYSICS
 * PARITY VS PHYSX IS UNPINNED.  This file restates, one env at a time and in plain loops, the
 * algorithm the HIP kernels implement (see DESIGN.md "Physics"):
 *   - fixed-base articulation in reduced coordinates; world-frame spatial algebra; forward
 *     kinematics; CRBA joint-space inertia; RNEA velocity-product (Coriolis) forces
 *     (PhysX articulation semantics: gravity disabled on the robot, ur5sih.py:176);
 *   - implicit PD position drives  (DOF_MODE_POS, kp/kd of Ur5SihBase.yaml:3-4, effort limit
 *     from the URDF <limit effort>) folded into the joint-space inertia, saturating at the effort;
 *   - free rigid objects (gravity, Isaac Gym default angular damping 0.5);
 *   - convex-hull contact generation (SAT over face normals, reference-face / incident-vertex
 *     manifold reduced to <= 4 points per pair), ground plane and table box;
 *   - projected Gauss-Seidel on the Delassus system J M^-1 J^T (normal + 2 friction rows per
 *     contact, joint-limit rows), Baumgarte + speculative contacts, `solver_iters` sweeps;
 *   - symplectic Euler integration, `substeps` substeps per gym.simulate() call.
 * Task math (controllers, reset, observations, reward, done) restates the reference exactly as
 * oracle/task_oracle.py does; that file is the one pinned against reference-generated goldens.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/handarm_abi.h"
#include "../include/ha_fmath.h"
#include "../include/ha_obb.h"

#define MAXC HA_MAX_CONTACTS   /* contact list capacity; a handle uses 21 (<= 3 objects) or 84 (clutter) */
#define MAXR (3 * MAXC)
#define NOBJ HA_MAX_OBJ
#define MAXB 48                  /* rigid bodies per env (ha_physics.h MAXB) */
#define MAXV (HA_MAX_DOFS + 6 * NOBJ)

typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 mul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 crs(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static v3 ld3(const float* p) { return V(p[0], p[1], p[2]); }
static void st3(float* p, v3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

typedef struct { float x, y, z, w; } qt;
static qt Q(float x, float y, float z, float w) { qt r = {x, y, z, w}; return r; }
static qt ldq(const float* p) { return Q(p[0], p[1], p[2], p[3]); }
static void stq(float* p, qt q) { p[0] = q.x; p[1] = q.y; p[2] = q.z; p[3] = q.w; }
static qt qmul(qt a, qt b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
             a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
static v3 qrot(qt q, v3 v) {
    v3 u = V(q.x, q.y, q.z);
    v3 t = mul(crs(u, v), 2.0f);
    return add(add(v, mul(t, q.w)), crs(u, t));
}
static qt qnorm(qt q) {
    float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Q(q.x / n, q.y / n, q.z / n, q.w / n);
}
static qt qaxis(v3 a, float ang) {
    float s, c;
    ha_sincosf(0.5f * ang, &s, &c);     /* the kernels' sin / cos (include/ha_fmath.h), not libm */
    return Q(a.x * s, a.y * s, a.z * s, c);
}
/* 3x3 rotation from quat */
static void qmat(qt q, float R[9]) {
    float x = q.x, y = q.y, z = q.z, w = q.w;
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
static v3 mv(const float M[9], v3 v) {
    return V(M[0] * v.x + M[1] * v.y + M[2] * v.z, M[3] * v.x + M[4] * v.y + M[5] * v.z,
             M[6] * v.x + M[7] * v.y + M[8] * v.z);
}
/* out = R A R^T */
static void rart(const float R[9], const float A[9], float out[9]) {
    float T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[i * 3 + j] = R[i * 3] * A[j] + R[i * 3 + 1] * A[3 + j] + R[i * 3 + 2] * A[6 + j];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            out[i * 3 + j] = T[i * 3] * R[j * 3] + T[i * 3 + 1] * R[j * 3 + 1] + T[i * 3 + 2] * R[j * 3 + 2];
}
static int inv3(const float A[9], float out[9]) {
    float c0 = A[4] * A[8] - A[5] * A[7], c1 = A[5] * A[6] - A[3] * A[8], c2 = A[3] * A[7] - A[4] * A[6];
    float det = A[0] * c0 + A[1] * c1 + A[2] * c2;
    if (fabsf(det) < 1e-30f) return -1;
    float id = 1.0f / det;
    out[0] = c0 * id; out[1] = (A[2] * A[7] - A[1] * A[8]) * id; out[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    out[3] = c1 * id; out[4] = (A[0] * A[8] - A[2] * A[6]) * id; out[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    out[6] = c2 * id; out[7] = (A[1] * A[6] - A[0] * A[7]) * id; out[8] = (A[0] * A[4] - A[1] * A[3]) * id;
    return 0;
}

/* spatial inertia at the world origin: (m, h = m c, J = I_c + m(|c|^2 1 - c c^T)) */
typedef struct { float m; v3 h; float J[9]; } sinert;
typedef struct { v3 w, v; } twist;   /* (omega, velocity of the point at the world origin) */

static void inert_apply(const sinert* I, twist t, v3* n, v3* f) {
    *n = add(mv(I->J, t.w), crs(I->h, t.v));
    *f = sub(mul(t.v, I->m), crs(I->h, t.w));
}

typedef struct {
    int nr;                 /* rows */
    float J[MAXR][MAXV];
    float Y[MAXR][MAXV];
    float vt[MAXR];         /* target velocity */
    float lo[MAXR], hi[MAXR];
    int fric_of[MAXR];      /* normal row index for friction rows, -1 otherwise */
    int contact[MAXR];      /* contact index or -1 */
} rows_t;

typedef struct {
    v3 x, n;      /* point, normal from B to A */
    float sep;
    int a, b;     /* body codes: -1 static, 0..NOBJ-1 object, 100+link robot */
} contact_t;

struct hao_s {
    ha_model_t m;
    ha_params_t p;
    int N, A, B, D, NO;
    int maxc;     /* contact capacity of the device kernel family (handarm_hip.hip family_of) */
    int pcm_slots;/* persistent-manifold record slots per env (hao_pcm_slots) */
    int packed;   /* packed PGS passes: 2 the clutter family (Ur5Sih, > 3 objects), 1 Ur5Sih <= 3 objects (nc <= 21) */
};
typedef struct hao_s* hao_handle;

/* ------------------------------------------------------------------ env scratch (one env) */
typedef struct {
    float q[HA_MAX_DOFS], qd[HA_MAX_DOFS], tgt[HA_MAX_DOFS];
    v3 lp[HA_MAX_LINKS];      /* link origin world */
    qt lq[HA_MAX_LINKS];      /* link rotation */
    v3 ax[HA_MAX_DOFS], an[HA_MAX_DOFS];
    /* objects */
    v3 oc[NOBJ], ov[NOBJ], ow[NOBJ];
    qt oq[NOBJ];
    float om[NOBJ], oIinv[NOBJ][9];
    int pool[NOBJ];
    int coll[NOBJ];
    float osc[NOBJ][3];             /* per-env object dimension scale (ha_state_t.object_scale) */
    int oscaled[NOBJ];
    v3 ofx[NOBJ];                   /* world force on the object COM for this call (object_force) */
    v3 otq[NOBJ];                   /* world torque on the object for this call (object_torque, v16) */
    float cforce[MAXB][3];
    float dforce[HA_MAX_DOFS];      /* joint force of the last substep: (drive + lower - upper impulse) / h */
    const float* dr;                /* this env's DR row (HA_DR_*) or NULL (ha_physics.h SimCtx::dr) */
    const float* drg;               /* the shard-wide DR state (HA_DRG_*) or NULL (ha_physics.h SimCtx::drg, v16) */
    float* pcm;                     /* this env's persistent-manifold records (ha_state_t.contact_cache) or NULL */
    int cst[HA_CSTAT];              /* contact_stats of this call sequence (ha_physics.h EnvLDS::cst) */
    float sb[8];                    /* the posed-static actor's pose (v14, ha_physics.h EnvLDS::sb): p, pad, q */
} env_t;

static float body_friction(const hao_handle h, const env_t* e, int b);

static int dofn(const hao_handle h) { return h->D; }

static void fk(const hao_handle h, env_t* e) {
    const ha_model_t* m = &h->m;
    for (int i = 0; i < m->n_links; i++) {
        int par = m->link_parent[i];
        if (par < 0) {
            e->lp[i] = ld3(m->base_pos);
            e->lq[i] = ldq(m->base_quat);
            continue;
        }
        e->lp[i] = add(e->lp[par], qrot(e->lq[par], ld3(m->link_origin_pos[i])));
        qt r = qmul(e->lq[par], ldq(m->link_origin_quat[i]));
        int d = m->link_dof[i];
        if (d >= 0) {
            r = qmul(r, qaxis(ld3(m->link_axis[i]), e->q[d]));
            e->ax[d] = qrot(r, ld3(m->link_axis[i]));
            e->an[d] = e->lp[i];
        }
        e->lq[i] = r;
    }
}

static void link_inertia(const hao_handle h, const env_t* e, int i, sinert* I) {
    const ha_model_t* m = &h->m;
    float R[9], Iw[9];
    qmat(e->lq[i], R);
    v3 c = add(e->lp[i], qrot(e->lq[i], ld3(m->link_com[i])));
    rart(R, m->link_inertia[i], Iw);
    float sc = e->dr ? e->dr[HA_DR_LINK_MASS + i] : 1.0f;
    for (int k = 0; k < 9; k++) Iw[k] = Iw[k] * sc;
    float mm = m->link_mass[i] * sc;
    I->m = mm;
    I->h = mul(c, mm);
    float cc = dot(c, c);
    float cv[3] = {c.x, c.y, c.z};
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) I->J[a * 3 + b] = Iw[a * 3 + b] + mm * ((a == b ? cc : 0.0f) - cv[a] * cv[b]);
}

/* joint-space inertia M (D x D) and velocity-product forces C (D) */
static void dynamics(const hao_handle h, env_t* e, float* M, float* C) {
    const ha_model_t* m = &h->m;
    int D = dofn(h), L = m->n_links;
    sinert I[HA_MAX_LINKS], Ic[HA_MAX_LINKS];
    twist Vl[HA_MAX_LINKS], Al[HA_MAX_LINKS];
    v3 Fn[HA_MAX_LINKS], Ff[HA_MAX_LINKS];
    for (int i = 0; i < L; i++) {
        link_inertia(h, e, i, &I[i]);
        Ic[i] = I[i];
        int par = m->link_parent[i], d = m->link_dof[i];
        twist vp = {V(0, 0, 0), V(0, 0, 0)}, ap = {V(0, 0, 0), V(0, 0, 0)};
        if (par >= 0) { vp = Vl[par]; ap = Al[par]; }
        Vl[i] = vp;
        Al[i] = ap;
        if (d >= 0) {
            twist s = {mul(e->ax[d], e->qd[d]), mul(crs(e->an[d], e->ax[d]), e->qd[d])};
            Vl[i].w = add(vp.w, s.w);
            Vl[i].v = add(vp.v, s.v);
            /* A += crm(V) s */
            Al[i].w = add(ap.w, crs(Vl[i].w, s.w));
            Al[i].v = add(ap.v, add(crs(Vl[i].w, s.v), crs(Vl[i].v, s.w)));
        }
        v3 n1, f1, n2, f2;
        inert_apply(&I[i], Al[i], &n1, &f1);
        inert_apply(&I[i], Vl[i], &n2, &f2);
        /* crf(V) (n2,f2) = (w x n2 + v x f2, w x f2) */
        Fn[i] = add(n1, add(crs(Vl[i].w, n2), crs(Vl[i].v, f2)));
        Ff[i] = add(f1, crs(Vl[i].w, f2));
        /* link damping (ha_params_t v10, ha_physics.h dynamics): the wrench cl m v_com, ca I_com w about the origin,
         * from the momentum (n2, f2) = (I_com w + c x m v_com, m v_com); g = c x m v_com = h x f2 / m */
        float cl = h->p.link_lin_damping, ca = h->p.link_ang_damping;
        if (cl != 0.0f || ca != 0.0f) {
            v3 g = I[i].m > 0.0f ? mul(crs(I[i].h, f2), 1.0f / I[i].m) : V(0, 0, 0);
            Fn[i] = add(Fn[i], add(mul(sub(n2, g), ca), mul(g, cl)));
            Ff[i] = add(Ff[i], mul(f2, cl));
        }
    }
    for (int i = 0; i < D; i++) C[i] = 0;
    for (int i = L - 1; i >= 0; i--) {
        int par = m->link_parent[i], d = m->link_dof[i];
        if (d >= 0) C[d] = dot(e->ax[d], Fn[i]) + dot(crs(e->an[d], e->ax[d]), Ff[i]);
        if (par >= 0) {
            Fn[par] = add(Fn[par], Fn[i]);
            Ff[par] = add(Ff[par], Ff[i]);
            Ic[par].m += Ic[i].m;
            Ic[par].h = add(Ic[par].h, Ic[i].h);
            for (int k = 0; k < 9; k++) Ic[par].J[k] += Ic[i].J[k];
        }
    }
    for (int i = 0; i < D * D; i++) M[i] = 0;
    for (int i = 0; i < L; i++) {
        int d = m->link_dof[i];
        if (d < 0) continue;
        twist s = {e->ax[d], crs(e->an[d], e->ax[d])};
        v3 n, f;
        inert_apply(&Ic[i], s, &n, &f);
        for (int j = i; j >= 0; j = m->link_parent[j]) {
            int dd = m->link_dof[j];
            if (dd < 0) continue;
            float v = dot(e->ax[dd], n) + dot(crs(e->an[dd], e->ax[dd]), f);
            if (dd == d) v += m->dof_armature[d];
            M[d * D + dd] = v;
            M[dd * D + d] = v;
        }
    }
}

/* in-place Cholesky (lower triangle, stride n), left-looking; the pivot is floored at 1e-30 exactly like
 * the GPU (isaacgym-hand-arm_amd/csrc/ha_physics.h cholesky) */
static void cholesky(float* A, int n) {
    for (int j = 0; j < n; j++) {
        float s = A[j * n + j];
        for (int k = 0; k < j; k++) s = fmaf(-A[j * n + k], A[j * n + k], s);
        A[j * n + j] = sqrtf(fmaxf(s, 1e-30f));
        for (int i = j + 1; i < n; i++) {
            float t = A[i * n + j];
            for (int k = 0; k < j; k++) t = fmaf(-A[i * n + k], A[j * n + k], t);
            A[i * n + j] = t / A[j * n + j];
        }
    }
}
/* M^-1 from the Cholesky factor (ha_physics.h factor_inverse): rl[i] = 1 / L[i][i]; column j of L^-1 by
 * forward substitution (Li[j][j] = rl[j], Li[i][j] = -(sum_{k=j}^{i-1} L[i][k] Li[k][j]) rl[i]); then
 * x = L^-T (L^-1 e_j) by back substitution. Stored as S[j][i] = x_j[i] (row j = column j of M^-1). */
static void inverse_from_cholesky(const float* Lm, int n, float* Li, float* S) {
    float rl[HA_MAX_DOFS];
    for (int i = 0; i < n; i++) rl[i] = 1.0f / Lm[i * n + i];
    for (int j = 0; j < n; j++) {
        for (int i = 0; i < j; i++) Li[i * n + j] = 0.0f;
        Li[j * n + j] = rl[j];
        for (int i = j + 1; i < n; i++) {
            float t = 0.0f;
            for (int k = j; k < i; k++) t = fmaf(Lm[i * n + k], Li[k * n + j], t);
            Li[i * n + j] = -t * rl[i];
        }
    }
    for (int j = 0; j < n; j++) {
        float x[HA_MAX_DOFS];
        for (int i = n - 1; i >= 0; i--) {
            float t = Li[i * n + j];
            for (int k = i + 1; k < n; k++) t = fmaf(-Lm[k * n + i], x[k], t);
            x[i] = t * rl[i];
        }
        for (int i = 0; i < n; i++) S[j * n + i] = x[i];
    }
}
/* The GPU's 64-lane dot product (ha_physics.h wave_sum_rows): a DPP butterfly inside each 16-lane row
 * gives ((x0+x1)+(x2+x3)) + ((x4+x5)+(x6+x7)) + ... as ((Q0+Q1)+(Q2+Q3)), then (R0+R1)+(R2+R3). Lanes
 * beyond n contribute exact zeros. With more than 64 coordinates (bin-picking: 65), lane i also holds
 * coordinate 64 + i and adds its product to its own first (ha_physics.h vregh). */
static float wave_dot(const float* a, const float* b, int n) {
    float x[64];
    for (int i = 0; i < 64; i++) x[i] = i < n ? a[i] * b[i] : 0.0f;
    if (n > 64)
        for (int i = 0; i < 64; i++) x[i] = x[i] + (64 + i < n ? a[64 + i] * b[64 + i] : 0.0f * 0.0f);
    float R[4];
    for (int r = 0; r < 4; r++) {
        float Q[4];
        for (int q = 0; q < 4; q++) {
            const float* y = x + 16 * r + 4 * q;
            Q[q] = (y[0] + y[1]) + (y[2] + y[3]);
        }
        R[r] = (Q[0] + Q[1]) + (Q[2] + Q[3]);
    }
    return (R[0] + R[1]) + (R[2] + R[3]);
}

/* ------------------------------------------------------------------ collision */
typedef struct { v3 p; qt q; } pose_t;

/* Per-env object dimensions: sc = diag scale of the hull in its body frame, or NULL (unscaled). Mirrors
 * scale3 / scale_radius / world_plane in ha_physics.h. */
static v3 scl(const float* sc, v3 v) { return sc ? V(v.x * sc[0], v.y * sc[1], v.z * sc[2]) : v; }
static float scl_r(const float* sc, float r) { return sc ? r * fmaxf(fmaxf(sc[0], sc[1]), sc[2]) : r; }
static const float* env_scale(const env_t* e, int b) { return (b >= 0 && b < NOBJ && e->oscaled[b]) ? e->osc[b] : NULL; }

static v3 hull_vert(const ha_model_t* m, int hull, int i, pose_t P, const float* sc) {
    const float* v = m->verts[m->hull_vert_start[hull] + i];
    return add(P.p, qrot(P.q, scl(sc, V(v[0], v[1], v[2]))));
}
static void hull_plane(const ha_model_t* m, int hull, int k, pose_t P, const float* sc, v3* n, float* d) {
    const float* pl = m->planes[m->hull_plane_start[hull] + k];
    v3 nl = V(pl[0], pl[1], pl[2]);
    float dl = pl[3];
    if (sc) {
        nl = V(pl[0] * (1.0f / sc[0]), pl[1] * (1.0f / sc[1]), pl[2] * (1.0f / sc[2]));
        float inv = 1.0f / sqrtf(dot(nl, nl));
        nl = mul(nl, inv);
        dl = dl * inv;
    }
    *n = qrot(P.q, nl);
    *d = dl - dot(*n, P.p);
}

/* reduce candidate list (points, sep) to <= 4 contacts; returns count appended. The area criterion measures
   about normal n, or (per-candidate normals nrm, compound objects) about the deepest candidate's normal. */
static int reduce_manifold(const v3* pts, const float* seps, int nc, v3 n, const v3* nrm, float window, int* out_idx) {
    if (nc <= 0) return 0;
    int i0 = 0;
    for (int i = 1; i < nc; i++)
        if (seps[i] < seps[i0]) i0 = i;
    out_idx[0] = i0;
    if (nrm) n = nrm[i0];
    if (nc == 1) return 1;
    float lim = seps[i0] + window;      /* points 2-4: within the window of the deepest point */
    int i1 = -1;
    float best = 1e-12f;
    for (int i = 0; i < nc; i++) {
        if (seps[i] > lim) continue;
        v3 d = sub(pts[i], pts[i0]);
        float dd = dot(d, d);
        if (dd > best) { best = dd; i1 = i; }
    }
    if (i1 < 0) return 1;
    out_idx[1] = i1;
    v3 e = sub(pts[i1], pts[i0]);
    int i2 = -1, i3 = -1;
    float bmax = 1e-12f, bmin = -1e-12f;
    for (int i = 0; i < nc; i++) {
        if (seps[i] > lim) continue;
        float s = dot(crs(e, sub(pts[i], pts[i0])), n);
        if (s > bmax) { bmax = s; i2 = i; }
        if (s < bmin) { bmin = s; i3 = i; }
    }
    int k = 2;
    if (i2 >= 0) out_idx[k++] = i2;
    if (i3 >= 0) out_idx[k++] = i3;
    return k;
}

#define MAXCAND 256      /* (1) <= 64 incident vertices, (2) <= 128 clip points, (3) <= 64 reference vertices */
#define MAXGATHER 32     /* ha_physics.h HA_MAX_GATHER */
/* Compound objects (several convex pieces, ha_model_t v8): between gather_begin and gather_end every piece
   pair's reduced points collect in a per-thread buffer (at most MAXGATHER, later ones dropped) and the object
   pair then emits ONE manifold of <= 4 points chosen from them, each keeping its piece pair's normal. */
static __thread int g_on, g_n;
static __thread float g_window;     /* ha_params_t.manifold_window of the running detect() */
static __thread float g_edge_rel, g_edge_abs;   /* ha_params_t.edge_rel_tol / edge_abs_tol of the running detect() */
static __thread int g_np_flags;                 /* ha_params_t.narrow_phase_flags */
static __thread v3 g_pt[MAXGATHER], g_nrm[MAXGATHER];
static __thread float g_sep[MAXGATHER];
static __thread int g_code[MAXGATHER];
/* contact_stats of the running detect(): contacts offered, self-collision contacts offered (both bodies links) */
static __thread int g_noff, g_nself;
/* A manifold point's anchor (ha_physics.h PCM_*): the feature the point came from - a vertex (or clipped edge point)
 * of side A, of side B, or neither (the midpoint of two closest edge points) - and the body whose face carries the
 * normal (the reference face; B for the ground and edge-edge contacts) */
#define PCM_FEAT_A 0
#define PCM_FEAT_B 1
#define PCM_FEAT_MID 2
#define PCM_NORMAL_A 4
/* persistent manifold (ha_params_t v13) of the running pair: its record (NULL: none) and the two body poses */
static __thread float* g_rec;
static __thread pose_t g_PA, g_PB;

static qt qconj(qt q) { return Q(-q.x, -q.y, -q.z, q.w); }
/* the record of a pair's chosen points (ha_physics.h pcm_store): relative pose, then per point its point on A in A's
 * frame, its point on B in B's frame and its normal in B's frame. x is midway between the two surface points, which
 * sit half the separation along the normal on either side */
static void pcm_store(float* rec, const v3* pts, const float* seps, const v3* nrm, v3 n, const int* codes,
                      const int* idx, int k) {
    qt qac = qconj(g_PA.q), qbc = qconj(g_PB.q);
    for (int i = 0; i < k; i++) {
        v3 x = pts[idx[i]], ni = nrm ? nrm[idx[i]] : n;
        int code = codes[idx[i]];
        float hs = 0.5f * seps[idx[i]];
        v3 la = qrot(qac, sub(add(x, mul(ni, hs)), g_PA.p));
        v3 lb = qrot(qbc, sub(sub(x, mul(ni, hs)), g_PB.p));
        v3 ln = qrot((code & PCM_NORMAL_A) ? qac : qbc, ni);
        float* r = rec + 8 + 9 * i;
        st3(r, la); st3(r + 3, lb); st3(r + 6, ln);
        rec[44 + i] = (float)code;
    }
    st3(rec, qrot(qbc, sub(g_PA.p, g_PB.p)));
    rec[3] = (float)k;
    stq(rec + 4, qmul(qbc, g_PA.q));
}

static void store_points(contact_t* out, int* nout, int maxout, const v3* pts, const float* seps, const v3* nrm,
                         v3 n, const int* idx, int k, int a, int b) {
    g_noff += k;
    if (a >= 100 && b >= 100) g_nself += k;
    for (int i = 0; i < k; i++) {
        v3 ni = nrm ? nrm[idx[i]] : n;
        if (*nout >= maxout) {
            /* replace the shallowest stored contact if this one is deeper */
            int w = 0;
            for (int j = 1; j < maxout; j++)
                if (out[j].sep > out[w].sep) w = j;
            if (out[w].sep <= seps[idx[i]]) continue;
            out[w].x = pts[idx[i]]; out[w].n = ni; out[w].sep = seps[idx[i]]; out[w].a = a; out[w].b = b;
            continue;
        }
        contact_t* c = &out[(*nout)++];
        c->x = pts[idx[i]]; c->n = ni; c->sep = seps[idx[i]]; c->a = a; c->b = b;
    }
}
static int emit(contact_t* out, int* nout, int maxout, v3* pts, float* seps, const int* codes, int nc, v3 n, int a,
                int b) {
    int idx[4];
    int k = reduce_manifold(pts, seps, nc, n, NULL, g_window, idx);
    if (g_on) {
        for (int i = 0; i < k && g_n < MAXGATHER; i++, g_n++) {
            g_pt[g_n] = pts[idx[i]]; g_sep[g_n] = seps[idx[i]]; g_nrm[g_n] = n; g_code[g_n] = codes[idx[i]];
        }
        return k;
    }
    if (g_rec && k > 0) pcm_store(g_rec, pts, seps, NULL, n, codes, idx, k);
    store_points(out, nout, maxout, pts, seps, NULL, n, idx, k, a, b);
    return k;
}
static void gather_begin(void) { g_on = 1; g_n = 0; }
static void gather_end(contact_t* out, int* nout, int maxout, int a, int b) {
    int idx[4];
    g_on = 0;
    int k = reduce_manifold(g_pt, g_sep, g_n, V(0, 0, 0), g_nrm, g_window, idx);
    if (g_rec && k > 0) pcm_store(g_rec, g_pt, g_sep, g_nrm, V(0, 0, 0), g_code, idx, k);
    store_points(out, nout, maxout, g_pt, g_sep, g_nrm, V(0, 0, 0), idx, k, a, b);
}
/* A pair's persistent manifold (ha_physics.h pcm_refresh): when its record holds points and the pair's relative pose
 * (side A's body in side B's frame) is within pcm_lin_tol / pcm_cos_tol of the pose the record was built at, each
 * point is re-evaluated from the current poses (the two surface points and the normal carried by their bodies; the
 * separation along the normal; the point midway), those within the contact margin are emitted in record order, and
 * the pair's narrow phase is skipped (returns 1). Otherwise returns 0 and leaves the record to the narrow phase. */
static int pcm_refresh(const ha_params_t* p, float* rec, pose_t PA, pose_t PB, int a, int b, contact_t* out, int* nout,
                       int maxout) {
    int k = (int)rec[3];
    if (k <= 0) return 0;
    qt qbc = qconj(PB.q);
    v3 d = sub(qrot(qbc, sub(PA.p, PB.p)), ld3(rec));
    float lt = p->pcm_lin_tol;
    if (dot(d, d) > lt * lt) return 0;
    qt qr = qmul(qbc, PA.q);
    float cq = ((qr.x * rec[4] + qr.y * rec[5]) + qr.z * rec[6]) + qr.w * rec[7];
    if (fabsf(cq) < p->pcm_cos_tol) return 0;
    v3 pts[4], nrm[4];
    float seps[4];
    int idx[4], kv = 0;
    for (int t = 0; t < k && t < 4; t++) {
        const float* r = rec + 8 + 9 * t;
        int code = (int)rec[44 + t];
        v3 wa = add(PA.p, qrot(PA.q, ld3(r)));
        v3 wb = add(PB.p, qrot(PB.q, ld3(r + 3)));
        v3 n = qrot((code & PCM_NORMAL_A) ? PA.q : PB.q, ld3(r + 6));
        float sp = dot(n, sub(wa, wb));
        if (sp > p->contact_margin) continue;
        int f = code & 3;
        /* the point where the narrow phase puts it: half the separation off its feature along the normal */
        pts[kv] = f == PCM_FEAT_A ? sub(wa, mul(n, 0.5f * sp)) : (f == PCM_FEAT_B ? add(wb, mul(n, 0.5f * sp))
                                                                                   : mul(add(wa, wb), 0.5f));
        nrm[kv] = n;
        seps[kv] = sp;
        idx[kv] = kv;
        kv++;
    }
    store_points(out, nout, maxout, pts, seps, nrm, V(0, 0, 0), idx, kv, a, b);
    return 1;
}

/* squared distance from point q to the segment p0 + t (p1 - p0), t in [0, 1] (ha_physics.h seg_point_d2) */
static float seg_point_d2(v3 p0, v3 p1, v3 q) {
    v3 d = sub(p1, p0);
    float dd = dot(d, d);
    float t = dd > 0.0f ? dot(sub(q, p0), d) / dd : 0.0f;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
    v3 r = sub(q, add(p0, mul(d, t)));
    return dot(r, r);
}
/* side plane of edge j of a face loop (world vertices wv, loop indices lv[0..n), face normal nf): through the edge,
 * perpendicular to the face, unit outward normal cross(e, nf) (ha_physics.h side_plane) */
static v3 side_plane(const v3* wv, const uint8_t* lv, int j, int n, v3 nf, float* d) {
    v3 v0 = wv[lv[j]];
    v3 sn = crs(sub(wv[lv[j + 1 == n ? 0 : j + 1]], v0), nf);
    sn = mul(sn, 1.0f / sqrtf(dot(sn, sn)));
    *d = -dot(sn, v0);
    return sn;
}
/* world face planes of a hull (hull_plane of every k) */
typedef struct { v3 n; float d; } wplane_t;

/* edge pair of the edge-edge SAT (ha_physics.h edge_axis, Gregorius GDC 2013): the Gauss-map arcs of edge ea of A
 * (between its faces' normals) and of edge eb of B (negated normals) cross -> a face of the Minkowski difference,
 * axis N = e1 x e2 oriented away from B's centre cb, separation N . (pA - pB); -3e38 otherwise */
static float edge_axis(uint32_t ea, uint32_t eb, const wplane_t* wpa, const wplane_t* wpb, const v3* va, const v3* vb,
                       v3 cb, v3* n, v3* pa, v3* e1, v3* pb, v3* e2) {
    v3 a = wpa[(ea >> 16) & 255u].n, b = wpa[ea >> 24].n;
    v3 cc = mul(wpb[(eb >> 16) & 255u].n, -1.0f), dd = mul(wpb[eb >> 24].n, -1.0f);
    v3 bxa = crs(b, a), dxc = crs(dd, cc);
    float cba = dot(cc, bxa), dba = dot(dd, bxa), adc = dot(a, dxc), bdc = dot(b, dxc);
    if (!(cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f)) return -3.0e38f;
    *pa = va[ea & 255u];
    *e1 = sub(va[(ea >> 8) & 255u], *pa);
    *pb = vb[eb & 255u];
    *e2 = sub(vb[(eb >> 8) & 255u], *pb);
    v3 nn = crs(*e1, *e2);
    float l2 = dot(nn, nn);
    if (l2 < 2.5e-5f * (dot(*e1, *e1) * dot(*e2, *e2))) return -3.0e38f;
    nn = mul(nn, 1.0f / sqrtf(l2));
    if (dot(nn, sub(*pb, cb)) < 0.0f) nn = mul(nn, -1.0f);
    *n = nn;
    return dot(nn, sub(*pa, *pb));
}
/* midpoint of the closest points of the segments pa + s e1, pb + t e2 (ha_physics.h edge_closest_mid) */
static v3 edge_closest_mid(v3 pa, v3 e1, v3 pb, v3 e2) {
    v3 r = sub(pa, pb);
    float aa = dot(e1, e1), ee = dot(e2, e2), bb = dot(e1, e2), cc = dot(e1, r), ff = dot(e2, r);
    float den = aa * ee - bb * bb;
    float sa = den > 0.0f ? (bb * ff - cc * ee) / den : 0.0f;
    sa = sa < 0.0f ? 0.0f : (sa > 1.0f ? 1.0f : sa);
    float tb = (bb * sa + ff) / ee;
    if (tb < 0.0f) {
        tb = 0.0f;
        sa = -cc / aa;
        sa = sa < 0.0f ? 0.0f : (sa > 1.0f ? 1.0f : sa);
    } else if (tb > 1.0f) {
        tb = 1.0f;
        sa = (bb - cc) / aa;
        sa = sa < 0.0f ? 0.0f : (sa > 1.0f ? 1.0f : sa);
    }
    return mul(add(add(pa, mul(e1, sa)), add(pb, mul(e2, tb))), 0.5f);
}

/* hull A (body a) vs hull B (body b); contact normal from B to A. Face axes of both hulls, then the edge-edge axes
 * (v10), then the contact: one edge-edge point, or the clipped face manifold (ha_physics.h collide_hulls) */
static void collide_hulls(const ha_model_t* m, int ha, pose_t PA, int hb, pose_t PB, float margin, int a, int b,
                          const float* sca, const float* scb, contact_t* out, int* nout, int maxout) {
    int nva = m->hull_nverts[ha], nvb = m->hull_nverts[hb];
    int npa = m->hull_nplanes[ha], npb = m->hull_nplanes[hb];
    /* bounding spheres */
    v3 ca = add(PA.p, qrot(PA.q, scl(sca, ld3(m->hull_center[ha]))));
    v3 cb = add(PB.p, qrot(PB.q, scl(scb, ld3(m->hull_center[hb]))));
    v3 dc = sub(ca, cb);
    float rr = scl_r(sca, m->hull_radius[ha]) + scl_r(scb, m->hull_radius[hb]) + margin;
    if (dot(dc, dc) > rr * rr) return;
    v3 va[64], vb[64];
    for (int i = 0; i < nva; i++) va[i] = hull_vert(m, ha, i, PA, sca);
    for (int i = 0; i < nvb; i++) vb[i] = hull_vert(m, hb, i, PB, scb);
    wplane_t wpa[128], wpb[128];
    for (int k = 0; k < npa; k++) hull_plane(m, ha, k, PA, sca, &wpa[k].n, &wpa[k].d);
    for (int k = 0; k < npb; k++) hull_plane(m, hb, k, PB, scb, &wpb[k].n, &wpb[k].d);
    /* SAT over face normals */
    float sepA = -1e30f, sepB = -1e30f;
    int kA = -1, kB = -1;
    for (int k = 0; k < npa; k++) {
        float mn = 1e30f;
        for (int i = 0; i < nvb; i++) { float s = dot(wpa[k].n, vb[i]) + wpa[k].d; if (s < mn) mn = s; }
        if (mn > sepA) { sepA = mn; kA = k; }
    }
    if (sepA > margin) return;
    for (int k = 0; k < npb; k++) {
        float mn = 1e30f;
        for (int i = 0; i < nva; i++) { float s = dot(wpb[k].n, va[i]) + wpb[k].d; if (s < mn) mn = s; }
        if (mn > sepB) { sepB = mn; kB = k; }
    }
    if (sepB > margin) return;
    /* edge-edge axes: the edges of each hull within R of the other's centre, every (A, B) pair in list order */
    int nea = m->hull_nedges[ha], neb = m->hull_nedges[hb];
    if (g_np_flags & HA_NP_NO_EDGE_AXES) nea = 0;
    if (nea > 0 && neb > 0) {
        float smax = fmaxf(sepA, sepB);
        float pen = smax < 0.0f ? -smax : 0.0f;
        float RA = (scl_r(sca, m->hull_radius[ha]) + margin) + pen;
        float RB = (scl_r(scb, m->hull_radius[hb]) + margin) + pen;
        const uint32_t* EA = m->edges + m->hull_edge_start[ha];
        const uint32_t* EB = m->edges + m->hull_edge_start[hb];
        int la[256], lb[256], nA = 0, nB = 0;
        for (int i = 0; i < nea; i++)
            if (seg_point_d2(va[EA[i] & 255u], va[(EA[i] >> 8) & 255u], cb) <= RB * RB) la[nA++] = i;
        for (int i = 0; i < neb; i++)
            if (seg_point_d2(vb[EB[i] & 255u], vb[(EB[i] >> 8) & 255u], ca) <= RA * RA) lb[nB++] = i;
        float best = -3.0e38f;
        int bw = -1;
        for (int i = 0; i < nA; i++)
            for (int j = 0; j < nB; j++) {
                v3 n, pa, pb, e1, e2;
                float sv = edge_axis(EA[la[i]], EB[lb[j]], wpa, wpb, va, vb, cb, &n, &pa, &e1, &pb, &e2);
                if (sv > best) { best = sv; bw = i * nB + j; }
            }
        if (best > margin) return;              /* separated along an edge-edge axis */
        if (best > g_edge_rel * smax + g_edge_abs) {
            v3 n, pa, pb, e1, e2;
            edge_axis(EA[la[bw / nB]], EB[lb[bw % nB]], wpa, wpb, va, vb, cb, &n, &pa, &e1, &pb, &e2);
            v3 x = edge_closest_mid(pa, e1, pb, e2);
            int code = PCM_FEAT_MID;
            emit(out, nout, maxout, &x, &best, &code, 1, n, a, b);
            return;
        }
    }
    /* face contact, candidates in the kernel's id order: (1) incident vertices near the reference face and inside its
     * hull's other planes, (2) per incident-face loop edge its entry / exit point clipped to the reference face's side
     * planes, (3) the reference face's loop vertices projected onto the incident face */
    v3 pts[MAXCAND];
    float seps[MAXCAND];
    int codes[MAXCAND];
    for (int pass = 0; pass < 2; pass++) {
        int refB = (sepB >= sepA) ? (pass == 0) : (pass == 1);
        /* anchors: candidates (1), (2) on the incident hull, (3) on the reference hull; the normal on the reference */
        int nA = refB ? 0 : PCM_NORMAL_A;
        int c_inc = (refB ? PCM_FEAT_A : PCM_FEAT_B) | nA, c_ref = (refB ? PCM_FEAT_B : PCM_FEAT_A) | nA;
        int hr = refB ? hb : ha, hi = refB ? ha : hb, kr = refB ? kB : kA;
        const wplane_t* wpr = refB ? wpb : wpa;
        const wplane_t* wpi = refB ? wpa : wpb;
        v3* vi = refB ? va : vb;
        v3* vr = refB ? vb : va;
        int nvi = refB ? nva : nvb, npr = refB ? npb : npa, npi = refB ? npa : npb;
        v3 nref = wpr[kr].n;
        float dref = wpr[kr].d;
        int nc = 0;
        for (int i = 0; i < nvi; i++) {
            float dist = dot(nref, vi[i]) + dref;
            if (dist > margin) continue;
            float mx = -1e30f;
            for (int k = 0; k < npr; k++) {
                if (k == kr) continue;
                float s = dot(wpr[k].n, vi[i]) + wpr[k].d;
                if (s > mx) mx = s;
            }
            if (mx > margin) continue;
            pts[nc] = sub(vi[i], mul(nref, 0.5f * dist));
            seps[nc] = dist;
            codes[nc] = c_inc;
            nc++;
        }
        int ki = -1;
        float vmin = 3.0e38f;
        for (int k = 0; k < npi; k++) {
            float dv = dot(wpi[k].n, nref);
            if (dv < vmin) { vmin = dv; ki = k; }
        }
        int lpi = m->plane_loop[m->hull_plane_start[hi] + ki], lpr = m->plane_loop[m->hull_plane_start[hr] + kr];
        int li0 = lpi & 0xFFFF, lni = lpi >> 16, lr0 = lpr & 0xFFFF, lnr = lpr >> 16;
        if (g_np_flags & HA_NP_NO_CLIP) lni = lnr = 0;
        /* the kernel holds the candidates one per lane: the valid vertices at lanes [0, nv1), edge j's entry / exit
         * point at lane nv1 + 2 j (+ 1), reference vertex r at lane nv1 + 2 lni + r; lanes past 63 are dropped */
        int nv1 = nc;
        for (int j = 0; j < lni; j++) {
            v3 p0 = vi[m->loop_v[li0 + j]], p1 = vi[m->loop_v[li0 + (j + 1 == lni ? 0 : j + 1)]];
            float tin = 0.0f, tout = 1.0f;
            int outside = 0;
            for (int jj = 0; jj < lnr; jj++) {
                float sd;
                v3 sn = side_plane(vr, m->loop_v + lr0, jj, lnr, nref, &sd);
                float f0 = dot(sn, p0) + sd, f1 = dot(sn, p1) + sd;
                if (f0 > 0.0f && f1 > 0.0f) outside = 1;
                else if (f0 > 0.0f) tin = fmaxf(tin, f0 / (f0 - f1));
                else if (f1 > 0.0f) tout = fminf(tout, f0 / (f0 - f1));
            }
            v3 e = sub(p1, p0);
            v3 xe = add(p0, mul(e, tin)), xx = add(p0, mul(e, tout));
            float de = dot(nref, xe) + dref, dx = dot(nref, xx) + dref;
            if (!outside && tin > 0.0f && tin <= tout && de <= margin && nv1 + 2 * j < 64) {
                pts[nc] = sub(xe, mul(nref, 0.5f * de));
                codes[nc] = c_inc;
                seps[nc++] = de;
            }
            if (!outside && tout < 1.0f && tin < tout && dx <= margin && nv1 + 2 * j + 1 < 64) {
                pts[nc] = sub(xx, mul(nref, 0.5f * dx));
                codes[nc] = c_inc;
                seps[nc++] = dx;
            }
        }
        v3 ni = wpi[ki].n;
        float di = wpi[ki].d;
        float den = dot(ni, nref);
        if (den < -1e-6f) {
            for (int r = 0; r < lnr; r++) {
                v3 q = vr[m->loop_v[lr0 + r]];
                float sr = -(dot(ni, q) + di) / den;
                v3 x = add(q, mul(nref, sr));
                float mx = -3.0e38f;
                for (int jj = 0; jj < lni; jj++) {
                    float sd;
                    v3 sn = side_plane(vi, m->loop_v + li0, jj, lni, ni, &sd);
                    mx = fmaxf(mx, dot(sn, x) + sd);
                }
                if (sr <= margin && mx <= 0.0f && nv1 + 2 * lni + r < 64) {
                    pts[nc] = add(q, mul(nref, 0.5f * sr));
                    codes[nc] = c_ref;
                    seps[nc++] = sr;
                }
            }
        }
        if (nc > 0) {
            v3 n = refB ? nref : mul(nref, -1.0f);
            emit(out, nout, maxout, pts, seps, codes, nc, n, a, b);
            return;
        }
    }
}

static void collide_ground(const ha_model_t* m, int ha, pose_t PA, float margin, int a, const float* sca,
                           contact_t* out, int* nout, int maxout) {
    v3 c = add(PA.p, qrot(PA.q, scl(sca, ld3(m->hull_center[ha]))));
    if (c.z - scl_r(sca, m->hull_radius[ha]) > margin) return;
    v3 pts[64];
    float seps[64];
    int codes[64];
    int nc = 0;
    for (int i = 0; i < m->hull_nverts[ha]; i++) {
        v3 v = hull_vert(m, ha, i, PA, sca);
        if (v.z <= margin) { pts[nc] = sub(v, V(0, 0, 0.5f * v.z)); seps[nc] = v.z; codes[nc] = PCM_FEAT_A; nc++; }
    }
    emit(out, nout, maxout, pts, seps, codes, nc, V(0, 0, 1), a, -1);
}

/* sphere (center c, radius r) vs the table box: exact sphere-box overlap test (broad phase) */
/* sphere (center c, radius r) vs static box k: exact sphere-box overlap test (broad phase) */
static int near_box(const float* half, pose_t Pb, v3 c, float r) {
    qt qi = Q(-Pb.q.x, -Pb.q.y, -Pb.q.z, Pb.q.w);
    v3 pl = qrot(qi, sub(c, Pb.p));
    float dx = fmaxf(fabsf(pl.x) - half[0], 0.0f);
    float dy = fmaxf(fabsf(pl.y) - half[1], 0.0f);
    float dz = fmaxf(fabsf(pl.z) - half[2], 0.0f);
    return dx * dx + dy * dy + dz * dz <= r * r;
}
/* two unscaled hulls' oriented boxes posed by their bodies within the margin on all 15 axes (include/ha_obb.h;
 * ha_physics.h piece_boxes_near): a compound pair's piece pair that fails it is skipped (round 6) */
static int piece_boxes_near(const ha_model_t* m, int h1, pose_t P1, int h2, pose_t P2, float mg) {
    float p1[3] = {P1.p.x, P1.p.y, P1.p.z}, q1[4] = {P1.q.x, P1.q.y, P1.q.z, P1.q.w};
    float p2[3] = {P2.p.x, P2.p.y, P2.p.z}, q2[4] = {P2.q.x, P2.q.y, P2.q.z, P2.q.w};
    return ha_obb_pair_near(p1, q1, m->hull_obb[h1], p2, q2, m->hull_obb[h2], mg);
}
/* static k's world pose; a static carried by the env's posed actor composes that actor's pose with its own (v14,
 * ha_physics.h static_pose) */
static pose_t static_pose(const ha_model_t* m, const env_t* e, int k) {
    pose_t P = {ld3(m->static_pos[k]), ldq(m->static_quat[k])};
    if (m->static_posed[k]) {
        v3 bp = ld3(e->sb);
        qt bq = ldq(e->sb + 4);
        pose_t R = {add(bp, qrot(bq, P.p)), qmul(bq, P.q)};
        P = R;
    }
    return P;
}

/* The pairs in the kernel's order (ha_physics.h pair_desc: per object its ground, statics, later objects and link hulls,
 * then link hulls x statics, then the self pairs), each first through the kernel's broad phase (ha_physics.h detect:
 * bounding spheres, the exact box for statics) - the persistent manifold (v13) is consulted for exactly the pairs that
 * pass it - then its record or its narrow phase. pidx is the pair's record slot. */
static const pose_t g_identity = {{0, 0, 0}, {0, 0, 0, 1}};
static void pcm_begin(float* rec, pose_t PA, pose_t PB) { g_rec = rec; g_PA = PA; g_PB = PB; }

static int detect(const hao_handle h, env_t* e, contact_t* out) {
    const ha_model_t* m = &h->m;
    const ha_params_t* p = &h->p;
    int nout = 0;
    float mg = p->contact_margin;
    g_window = p->manifold_window;
    g_edge_rel = p->edge_rel_tol;
    g_edge_abs = p->edge_abs_tol;
    g_np_flags = p->narrow_phase_flags;
    g_noff = g_nself = 0;
    g_rec = NULL;
    int NO = h->NO, NS = m->n_static, NLH = m->n_link_hulls;
    float* pcm = (e->pcm && p->pcm_lin_tol > 0.0f) ? e->pcm : NULL;
    int pidx = 0, nref = 0, nnar = 0;
#define PCM_REC(k) (pcm ? pcm + (size_t)(k) * HA_PCM_REC : NULL)
#define PCM_TRY(k, PA, PB, a, b) (pcm && pcm_refresh(p, PCM_REC(k), PA, PB, a, b, out, &nout, h->maxc) ? (nref++, 1) : 0)
    for (int o = 0; o < NO; o++) {
        int pa = e->pool[o];
        int ho = m->pool_hull[pa], no = m->pool_nhull[pa];     /* the object's convex pieces (ABI v8) */
        const float* so = env_scale(e, o);
        pose_t Po = {sub(e->oc[o], qrot(e->oq[o], scl(so, ld3(m->pool_com[pa])))), e->oq[o]};
        /* the object's bounding sphere over all its pieces (the kernel's broad phase) */
        v3 co = add(Po.p, qrot(Po.q, scl(so, ld3(m->pool_center[pa]))));
        float ro = scl_r(so, m->pool_radius[pa]);
        /* a compound object (no > 1 pieces) emits one manifold per object pair (gather_begin / gather_end) */
        if (e->coll[o] && co.z - ro <= mg && !PCM_TRY(pidx, Po, g_identity, o, -1)) {
            pcm_begin(PCM_REC(pidx), Po, g_identity);
            nnar += no;
            if (no > 1) gather_begin();
            for (int j = 0; j < no; j++) collide_ground(m, ho + j, Po, mg, o, so, out, &nout, h->maxc);
            if (no > 1) gather_end(out, &nout, h->maxc, o, -1);
            g_rec = NULL;
        }
        pidx++;
        for (int st = 0; st < NS; st++, pidx++) {
            pose_t Pst = static_pose(m, e, st);
            int hs = m->static_hull[st];
            v3 dc = sub(co, add(Pst.p, qrot(Pst.q, ld3(m->hull_center[hs]))));
            float rr = ro + m->hull_radius[hs] + mg;
            if (!e->coll[o] || !(dot(dc, dc) <= rr * rr) || !near_box(m->static_half[st], Pst, co, ro + mg)) continue;
            if (PCM_TRY(pidx, Po, Pst, o, -1)) continue;
            pcm_begin(PCM_REC(pidx), Po, Pst);
            if (no > 1) gather_begin();
            for (int j = 0; j < no; j++)     /* each piece's own sphere against the exact box too */
                if (near_box(m->static_half[st], Pst, add(Po.p, qrot(Po.q, scl(so, ld3(m->hull_center[ho + j])))),
                             scl_r(so, m->hull_radius[ho + j]) + mg)) {
                    nnar++;
                    collide_hulls(m, ho + j, Po, hs, Pst, mg, o, -1, so, NULL, out, &nout, h->maxc);
                }
            if (no > 1) gather_end(out, &nout, h->maxc, o, -1);
            g_rec = NULL;
        }
        for (int o2 = o + 1; o2 < NO; o2++, pidx++) {
            int pb = e->pool[o2];
            int h2 = m->pool_hull[pb], n2 = m->pool_nhull[pb];
            const float* s2 = env_scale(e, o2);
            pose_t P2 = {sub(e->oc[o2], qrot(e->oq[o2], scl(s2, ld3(m->pool_com[pb])))), e->oq[o2]};
            v3 dc = sub(co, add(P2.p, qrot(P2.q, scl(s2, ld3(m->pool_center[pb])))));
            float rr = ro + scl_r(s2, m->pool_radius[pb]) + mg;
            if (!e->coll[o] || !e->coll[o2] || !(dot(dc, dc) <= rr * rr)) continue;
            if (PCM_TRY(pidx, Po, P2, o, o2)) continue;
            pcm_begin(PCM_REC(pidx), Po, P2);
            if (no * n2 > 1) gather_begin();
            for (int j = 0; j < no; j++)
                for (int j2 = 0; j2 < n2; j2++) {
                    /* a compound pair's piece pair: the pieces' own spheres first (ha_physics.h narrow_phase, round 6) */
                    if (no * n2 > 1) {
                        v3 c1 = add(Po.p, qrot(Po.q, scl(so, ld3(m->hull_center[ho + j]))));
                        v3 c2 = add(P2.p, qrot(P2.q, scl(s2, ld3(m->hull_center[h2 + j2]))));
                        float rp = scl_r(so, m->hull_radius[ho + j]) + scl_r(s2, m->hull_radius[h2 + j2]) + mg;
                        v3 dp = sub(c1, c2);
                        if (!(dot(dp, dp) <= rp * rp)) continue;
                        if (!so && !s2 && !piece_boxes_near(m, ho + j, Po, h2 + j2, P2, mg)) continue;
                    }
                    nnar++;
                    collide_hulls(m, ho + j, Po, h2 + j2, P2, mg, o, o2, so, s2, out, &nout, h->maxc);
                }
            if (no * n2 > 1) gather_end(out, &nout, h->maxc, o, o2);
            g_rec = NULL;
        }
        for (int k = 0; k < NLH; k++, pidx++) {
            int L = m->hull_link[k];
            pose_t PL = {e->lp[L], e->lq[L]};
            v3 dc = sub(co, add(PL.p, qrot(PL.q, ld3(m->hull_center[k]))));
            float rr = ro + m->hull_radius[k] + mg;
            if (!e->coll[o] || !(dot(dc, dc) <= rr * rr)) continue;
            if (PCM_TRY(pidx, PL, Po, 100 + L, o)) continue;
            pcm_begin(PCM_REC(pidx), PL, Po);
            if (no > 1) gather_begin();
            for (int j = 0; j < no; j++) {
                if (no > 1) {       /* the link hull's sphere against the piece's */
                    v3 c1 = add(PL.p, qrot(PL.q, ld3(m->hull_center[k])));
                    v3 c2 = add(Po.p, qrot(Po.q, scl(so, ld3(m->hull_center[ho + j]))));
                    float rp = m->hull_radius[k] + scl_r(so, m->hull_radius[ho + j]) + mg;
                    v3 dp = sub(c1, c2);
                    if (!(dot(dp, dp) <= rp * rp)) continue;
                    if (!so && !piece_boxes_near(m, k, PL, ho + j, Po, mg)) continue;
                }
                nnar++;
                collide_hulls(m, k, PL, ho + j, Po, mg, 100 + L, o, NULL, so, out, &nout, h->maxc);
            }
            if (no > 1) gather_end(out, &nout, h->maxc, 100 + L, o);
            g_rec = NULL;
        }
    }
    for (int k = 0; k < NLH; k++) {
        int L = m->hull_link[k];
        pose_t PL = {e->lp[L], e->lq[L]};
        v3 ch = add(PL.p, qrot(PL.q, ld3(m->hull_center[k])));
        for (int st = 0; st < NS; st++, pidx++) {
            if (!m->link_table_collide[L]) continue;
            pose_t Pst = static_pose(m, e, st);
            int hs = m->static_hull[st];
            v3 dc = sub(ch, add(Pst.p, qrot(Pst.q, ld3(m->hull_center[hs]))));
            float rr = m->hull_radius[k] + m->hull_radius[hs] + mg;
            if (!(dot(dc, dc) <= rr * rr) || !near_box(m->static_half[st], Pst, ch, m->hull_radius[k] + mg)) continue;
            if (PCM_TRY(pidx, PL, Pst, 100 + L, -1)) continue;
            pcm_begin(PCM_REC(pidx), PL, Pst);
            nnar++;
            collide_hulls(m, k, PL, hs, Pst, mg, 100 + L, -1, NULL, NULL, out, &nout, h->maxc);
            g_rec = NULL;
        }
    }
    /* self-collision (v12): link hull pairs of non-adjacent links whose oriented boxes come within the margin
       (include/ha_obb.h, the kernel's mid-phase) */
    for (int k = 0; k < m->n_self_pairs; k++, pidx++) {
        int ha = m->self_pair[k] & 255, hb = m->self_pair[k] >> 8;
        int la = m->hull_link[ha], lb = m->hull_link[hb];
        float pa[3] = {e->lp[la].x, e->lp[la].y, e->lp[la].z}, qa[4] = {e->lq[la].x, e->lq[la].y, e->lq[la].z, e->lq[la].w};
        float pb[3] = {e->lp[lb].x, e->lp[lb].y, e->lp[lb].z}, qb[4] = {e->lq[lb].x, e->lq[lb].y, e->lq[lb].z, e->lq[lb].w};
        float ca[3], Ra[9], cb[3], Rb[9];
        ha_obb_world(pa, qa, m->hull_obb[ha], ca, Ra);
        ha_obb_world(pb, qb, m->hull_obb[hb], cb, Rb);
        if (!ha_obb_near(ca, Ra, m->hull_obb[ha] + 3, cb, Rb, m->hull_obb[hb] + 3, mg)) continue;
        /* hull b on side A, hull a on side B (ha_physics.h narrow_phase kind 5): normal from a to b */
        pose_t PA = {e->lp[lb], e->lq[lb]}, PB = {e->lp[la], e->lq[la]};
        if (PCM_TRY(pidx, PA, PB, 100 + lb, 100 + la)) continue;
        pcm_begin(PCM_REC(pidx), PA, PB);
        nnar++;
        collide_hulls(m, hb, PA, ha, PB, mg, 100 + lb, 100 + la, NULL, NULL, out, &nout, h->maxc);
        g_rec = NULL;
    }
#undef PCM_TRY
#undef PCM_REC
    /* contact_stats (ha_physics.h substep, EnvLDS::cst) */
    e->cst[0] += 1;
    e->cst[1] += g_noff > h->maxc ? 1 : 0;
    e->cst[2] = g_noff > e->cst[2] ? g_noff : e->cst[2];
    e->cst[3] += g_noff;
    e->cst[4] += g_nself;
    e->cst[5] += nref;
    e->cst[6] += nnar;
    return nout;
}

/* record slots of an env (ha_contact_cache_slots): the kernel's pair enumeration, then the self pairs */
int hao_pcm_slots(const ha_model_t* m, int n_objects) {
    int NO = n_objects, NS = m->n_static, NLH = m->n_link_hulls, n = 0;
    for (int o = 0; o < NO; o++) n += 1 + NS + (NO - 1 - o) + NLH;
    return n + NLH * NS + m->n_self_pairs;
}

/* Jacobian row: relative velocity of body a minus body b at point x along dir, into J (len D+6*NO) */
static void jac_body(const hao_handle h, const env_t* e, int body, v3 x, v3 dir, float sgn, float* J) {
    int D = dofn(h);
    if (body < 0) return;
    if (body < 100) {
        int o = body;
        v3 r = sub(x, e->oc[o]);
        v3 ang = crs(r, dir);
        float* Jo = J + D + 6 * o;
        Jo[0] += sgn * dir.x; Jo[1] += sgn * dir.y; Jo[2] += sgn * dir.z;
        Jo[3] += sgn * ang.x; Jo[4] += sgn * ang.y; Jo[5] += sgn * ang.z;
        return;
    }
    int L = body - 100;
    for (int j = L; j >= 0; j = h->m.link_parent[j]) {
        int d = h->m.link_dof[j];
        if (d < 0) continue;
        J[d] += sgn * dot(e->ax[d], crs(sub(x, e->an[d]), dir));
    }
}

/* Y = M^-1 J^T for one row: robot block through the explicit inverse, object blocks 1/m and I_w^-1 */
static void apply_minv(const hao_handle h, const env_t* e, const float* Minv, const float* J, float* Y) {
    int D = dofn(h);
    for (int i = 0; i < D; i++) {
        float acc = 0.0f;
        for (int j = 0; j < D; j++) acc = fmaf(Minv[i * D + j], J[j], acc);
        Y[i] = acc;
    }
    for (int o = 0; o < h->NO; o++) {
        const float* Jo = J + D + 6 * o;
        float* Yo = Y + D + 6 * o;
        float im = 1.0f / e->om[o];
        Yo[0] = Jo[0] * im; Yo[1] = Jo[1] * im; Yo[2] = Jo[2] * im;
        v3 a = mv(e->oIinv[o], V(Jo[3], Jo[4], Jo[5]));
        Yo[3] = a.x; Yo[4] = a.y; Yo[5] = a.z;
    }
}

static void tangents(v3 n, v3* t1, v3* t2) {
    v3 a = fabsf(n.x) < 0.9f ? V(1, 0, 0) : V(0, 1, 0);
    v3 t = crs(n, a);
    float l = sqrtf(dot(t, t));
    *t1 = mul(t, 1.0f / l);
    *t2 = crs(n, *t1);
}

/* One substep; the same operation order as ha_physics.h substep (the GPU lane-parallel version). */
/* friction of a contact body: link 100+L, object o, static -1 (PhysX average combine per contact) */
static float body_friction(const hao_handle h, const env_t* e, int b) {
    if (!e->dr || b < 0) return h->p.friction;
    return b >= 100 ? e->dr[HA_DR_LINK_FRIC + (b - 100)] : e->dr[HA_DR_OBJ_FRIC + b];
}

/* ---- packed PGS passes (ha_physics.h PhysCfg PACK: the clutter family) */
static int is_link_contact(const contact_t* c) { return c->a >= 100 || c->b >= 100; }
/* object slots of a contact's compact row (ha_physics.h contact_slots): so0 the lower object index */
static void contact_slots(int a, int b, int* so0, int* so1) {
    int oa = (a >= 0 && a < 100) ? a : -1, ob = (b >= 0 && b < 100) ? b : -1;
    *so0 = oa < 0 ? ob : (ob < 0 ? oa : (oa < ob ? oa : ob));
    *so1 = (oa >= 0 && ob >= 0) ? (oa < ob ? ob : oa) : -1;
}
/* The contacts that touch no link, four per pass on pairwise disjoint objects: each pass takes, in contact order, the
 * remaining contacts whose objects it does not hold yet (static bodies never conflict). Returns the pass count. */
static int packed_passes(const contact_t* cs, int nc, int passes[][4]) {
    int done[MAXC] = {0}, np = 0, left = 0;
    for (int c = 0; c < nc; c++) {
        done[c] = is_link_contact(&cs[c]);
        left += !done[c];
    }
    while (left > 0) {
        unsigned objm = 0u;
        int k = 0;
        for (int q = 0; q < 4; q++) passes[np][q] = -1;
        for (int c = 0; c < nc && k < 4; c++) {
            if (done[c]) continue;
            int so0, so1;
            contact_slots(cs[c].a, cs[c].b, &so0, &so1);
            if ((so0 >= 0 && ((objm >> so0) & 1u)) || (so1 >= 0 && ((objm >> so1) & 1u))) continue;
            objm |= (so0 >= 0 ? 1u << so0 : 0u) | (so1 >= 0 ? 1u << so1 : 0u);
            passes[np][k++] = c;
            done[c] = 1;
            left--;
        }
        np++;
    }
    return np;
}
/* One free contact of a pass (ha_physics.h free passes): the J.v sums over the 16-lane row that holds the contact's
 * compact row (lanes 0-5 object slot 0, 6-11 slot 1, 12-15 empty; a missing slot adds zeros) by the row butterfly
 * (Q0+Q1)+(Q2+Q3), the block arithmetic of the serial contact, and the updates of its objects' coordinates. */
static float row_dot16(const float* x) {
    float Q[4];
    for (int q = 0; q < 4; q++) Q[q] = (x[4 * q] + x[4 * q + 1]) + (x[4 * q + 2] + x[4 * q + 3]);
    return (Q[0] + Q[1]) + (Q[2] + Q[3]);
}
static void contact_block_packed(const contact_t* ct, int D, const float* J0, const float* J1, const float* J2,
                                 const float* Y0, const float* Y1, const float* Y2, const float* vt, const float* winv,
                                 float* lam, float mu, float a10, float a20, float a21, float* v) {
    int so0, so1, idx[12];
    contact_slots(ct->a, ct->b, &so0, &so1);
    float x0[16] = {0}, x1[16] = {0}, x2[16] = {0};
    for (int t = 0; t < 12; t++) {
        int o = t < 6 ? so0 : so1;
        idx[t] = o >= 0 ? D + 6 * o + (t < 6 ? t : t - 6) : -1;
        if (idx[t] < 0) continue;
        x0[t] = J0[idx[t]] * v[idx[t]];
        x1[t] = J1[idx[t]] * v[idx[t]];
        x2[t] = J2[idx[t]] * v[idx[t]];
    }
    float jv0 = row_dot16(x0), jv1 = row_dot16(x1), jv2 = row_dot16(x2);
    float l0 = lam[0], l1 = lam[1], l2 = lam[2];
    float n0 = l0 - (jv0 - vt[0]) * winv[0];
    n0 = n0 < 0.0f ? 0.0f : (n0 > 3.0e38f ? 3.0e38f : n0);
    float d0 = n0 - l0;
    float hi = mu * n0;
    float n1 = l1 - (fmaf(a10, d0, jv1) - vt[1]) * winv[1];
    n1 = n1 < -hi ? -hi : (n1 > hi ? hi : n1);
    float d1 = n1 - l1;
    float n2 = l2 - (fmaf(a21, d1, fmaf(a20, d0, jv2)) - vt[2]) * winv[2];
    n2 = n2 < -hi ? -hi : (n2 > hi ? hi : n2);
    float d2 = n2 - l2;
    lam[0] = n0; lam[1] = n1; lam[2] = n2;
    for (int t = 0; t < 12; t++) {
        int i = idx[t];
        if (i < 0) continue;
        float vv = v[i];
        if (d0 != 0.0f) vv = fmaf(Y0[i], d0, vv);
        if (d1 != 0.0f) vv = fmaf(Y1[i], d1, vv);
        if (d2 != 0.0f) vv = fmaf(Y2[i], d2, vv);
        v[i] = vv;
    }
}

static void substep(const hao_handle h, env_t* e, float hdt) {
    const ha_model_t* m = &h->m;
    const ha_params_t* p = &h->p;
    int D = dofn(h), NO = h->NO, NV = D + 6 * NO;
    static __thread float M[HA_MAX_DOFS * HA_MAX_DOFS], Li[HA_MAX_DOFS * HA_MAX_DOFS],
        Minv[HA_MAX_DOFS * HA_MAX_DOFS];
    float C[HA_MAX_DOFS];
    fk(h, e);
    dynamics(h, e, M, C);
    cholesky(M, D);
    inverse_from_cholesky(M, D, Li, Minv);
    /* free motion: velocity-product forces only (drives are constraint rows of the PGS below) */
    float v[MAXV];
    for (int i = 0; i < D; i++) {
        float acc = 0.0f;
        for (int j = 0; j < D; j++) acc = fmaf(Minv[i * D + j], -hdt * C[j], acc);
        v[i] = e->qd[i] + acc;
    }
    for (int o = 0; o < NO; o++) {
        float damp = 1.0f / (1.0f + hdt * p->object_ang_damping);
        float R[9], Iw[9], Il[9];
        const float* I0 = m->pool_inertia[e->pool[o]];
        float sc = e->dr ? e->dr[HA_DR_OBJ_MASS + o] : 1.0f;
        float mass = m->pool_mass[e->pool[o]];
        for (int k = 0; k < 9; k++) Il[k] = I0[k];
        if (e->oscaled[o]) {
            /* uniform density scaled by S: C = tr(I)/2 Id - I, C' = det(S) S C S, I' = tr(C') Id - C' */
            const float* sv = e->osc[o];
            float det = (sv[0] * sv[1]) * sv[2];
            float hh = 0.5f * ((I0[0] + I0[4]) + I0[8]);
            float Cs[9];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) Cs[3 * i + j] = det * (sv[i] * (((i == j ? hh : 0.0f) - I0[3 * i + j]) * sv[j]));
            float tr = (Cs[0] + Cs[4]) + Cs[8];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) Il[3 * i + j] = (i == j ? tr : 0.0f) - Cs[3 * i + j];
            mass = mass * det;
        }
        qmat(e->oq[o], R);
        rart(R, Il, Iw);
        for (int k = 0; k < 9; k++) Iw[k] = Iw[k] * sc;
        inv3(Iw, e->oIinv[o]);
        mass = mass * sc;
        e->om[o] = mass;
        const float* grav = e->drg ? e->drg + HA_DRG_GRAVITY : p->gravity;
        v3 lv = add(add(e->ov[o], mul(ld3(grav), hdt)), mul(e->ofx[o], hdt / mass));
        v3 av = add(mul(e->ow[o], damp), mul(mv(e->oIinv[o], e->otq[o]), hdt));
        float* vo = v + D + 6 * o;
        vo[0] = lv.x; vo[1] = lv.y; vo[2] = lv.z; vo[3] = av.x; vo[4] = av.y; vo[5] = av.z;
    }
    /* contacts -> rows (normal, friction 1, friction 2 per contact) */
    contact_t cs[MAXC];
    int nc = detect(h, e, cs);
    static __thread rows_t R;
    int nr = 3 * nc;
    float winv[MAXR], lam[MAXR];
    for (int r = 0; r < nr; r++) {
        int c = r / 3, k = r % 3;
        v3 t1, t2;
        tangents(cs[c].n, &t1, &t2);
        v3 dir = k == 0 ? cs[c].n : (k == 1 ? t1 : t2);
        memset(R.J[r], 0, sizeof(R.J[r]));
        memset(R.Y[r], 0, sizeof(R.Y[r]));
        jac_body(h, e, cs[c].a, cs[c].x, dir, 1.0f, R.J[r]);
        jac_body(h, e, cs[c].b, cs[c].x, dir, -1.0f, R.J[r]);
        R.contact[r] = c;
        if (k == 0) {
            float s = cs[c].sep;
            float sb = s + p->contact_slop < 0.0f ? s + p->contact_slop : 0.0f;   /* penetration beyond the slop */
            float vt = s > 0 ? -s / hdt : -p->baumgarte * sb / hdt;
            if (vt > p->max_depen_vel) vt = p->max_depen_vel;
            R.vt[r] = vt; R.lo[r] = 0; R.hi[r] = 3.0e38f; R.fric_of[r] = -1;
        } else {
            R.vt[r] = 0; R.lo[r] = 0; R.hi[r] = 0; R.fric_of[r] = r - k;
        }
        apply_minv(h, e, Minv, R.J[r], R.Y[r]);
        float a = 0.0f;
        for (int t = 0; t < NV; t++) a = fmaf(R.J[r][t], R.Y[r][t], a);
        winv[r] = 1.0f / (a + 1e-9f);
        lam[r] = 0.0f;
    }
    /* coupling inside each contact's 3-row block: a10 = J_1 . Y_0, a20 = J_2 . Y_0, a21 = J_2 . Y_1 */
    float a10[MAXC], a20[MAXC], a21[MAXC];
    for (int c = 0; c < nc; c++) {
        const float *J1 = R.J[3 * c + 1], *J2 = R.J[3 * c + 2], *Y0 = R.Y[3 * c], *Y1 = R.Y[3 * c + 1];
        float x = 0.0f, y = 0.0f, z = 0.0f;
        for (int t = 0; t < NV; t++) x = fmaf(J1[t], Y0[t], x);
        for (int t = 0; t < NV; t++) y = fmaf(J2[t], Y0[t], y);
        for (int t = 0; t < NV; t++) z = fmaf(J2[t], Y1[t], z);
        a10[c] = x; a20[c] = y; a21[c] = z;
    }
    /* joint rows of dof d: PD drive as a soft, impulse-bounded constraint (PhysX articulation drive
     * semantics: implicit spring-damper gamma = 1/(h(kd + h kp)), bias = kp/(kd + h kp)(q - q*),
     * |lambda| <= effort h) and the hard lower/upper limits (active within joint_limit_margin) */
    float dgam[HA_MAX_DOFS], dbias[HA_MAX_DOFS], dwinv[HA_MAX_DOFS], dlim[HA_MAX_DOFS], dlam[HA_MAX_DOFS];
    float lwinv[HA_MAX_DOFS], vt_lo[HA_MAX_DOFS], vt_up[HA_MAX_DOFS], lam_lo[HA_MAX_DOFS], lam_up[HA_MAX_DOFS];
    /* joint friction row: |impulse| <= dof_friction |drive + lower - upper impulse| (a coefficient, Isaac Gym's DOF
     * "friction", docs/domain_randomization.md:197), re-bounded each sweep (ha_physics.h) */
    float fcoef[HA_MAX_DOFS], lam_fr[HA_MAX_DOFS];
    int act_lo[HA_MAX_DOFS], act_up[HA_MAX_DOFS];
    for (int d = 0; d < D; d++) {
        /* DR (v16): the env's dof_properties stiffness / damping / lower / upper (ha_physics.h joint rows) */
        float kp = e->dr ? e->dr[HA_DR_DOF_KP + d] : m->dof_kp[d];
        float kd = e->dr ? e->dr[HA_DR_DOF_KD + d] : m->dof_kd[d];
        float jlo = e->dr ? e->dr[HA_DR_DOF_LOWER + d] : m->dof_lower[d];
        float jup = e->dr ? e->dr[HA_DR_DOF_UPPER + d] : m->dof_upper[d];
        float den = kd + hdt * kp;
        float mii = Minv[d * D + d];
        dgam[d] = 1.0f / (hdt * den);
        dbias[d] = kp / den * (e->q[d] - e->tgt[d]);
        dwinv[d] = 1.0f / (mii + dgam[d]);
        dlim[d] = m->dof_effort[d] * hdt;
        dlam[d] = 0.0f;
        lwinv[d] = 1.0f / (mii + 1e-9f);
        float s_lo = e->q[d] - jlo, s_up = jup - e->q[d];
        act_lo[d] = s_lo <= p->joint_limit_margin;
        act_up[d] = s_up <= p->joint_limit_margin;
        vt_lo[d] = s_lo > 0 ? -s_lo / hdt : -p->baumgarte * s_lo / hdt;
        vt_up[d] = s_up > 0 ? -s_up / hdt : -p->baumgarte * s_up / hdt;
        lam_lo[d] = lam_up[d] = 0.0f;
        fcoef[d] = m->dof_friction[d];
        lam_fr[d] = 0.0f;
    }
    int packed = h->packed == 2 || (h->packed == 1 && nc <= 21);
    int passes[MAXC][4], npass = packed ? packed_passes(cs, nc, passes) : 0;
    /* projected Gauss-Seidel, velocity form: joint rows d = 0..D-1 (drive, lower, upper), then the
     * contact rows; v is updated after every row */
    for (int it = 0; it < p->solver_iters; it++) {
        for (int d = 0; d < D; d++) {
            const float* mrow = Minv + d * D;
            float nl = dlam[d] - (v[d] + dbias[d] + dgam[d] * dlam[d]) * dwinv[d];
            nl = nl < -dlim[d] ? -dlim[d] : (nl > dlim[d] ? dlim[d] : nl);
            float dl = nl - dlam[d];
            if (dl != 0.0f) {
                dlam[d] = nl;
                for (int k = 0; k < D; k++) v[k] = fmaf(mrow[k], dl, v[k]);
            }
            if (act_lo[d]) {
                float n0 = lam_lo[d] - (v[d] - vt_lo[d]) * lwinv[d];
                n0 = n0 < 0.0f ? 0.0f : n0;
                float d0 = n0 - lam_lo[d];
                if (d0 != 0.0f) {
                    lam_lo[d] = n0;
                    for (int k = 0; k < D; k++) v[k] = fmaf(mrow[k], d0, v[k]);
                }
            }
            if (act_up[d]) {
                float n1 = lam_up[d] - (-v[d] - vt_up[d]) * lwinv[d];
                n1 = n1 < 0.0f ? 0.0f : n1;
                float d1 = n1 - lam_up[d];
                if (d1 != 0.0f) {
                    lam_up[d] = n1;
                    for (int k = 0; k < D; k++) v[k] = fmaf(-mrow[k], d1, v[k]);
                }
            }
            if (fcoef[d] > 0.0f) {
                float flim = fcoef[d] * fabsf((dlam[d] + lam_lo[d]) - lam_up[d]);
                float nf = lam_fr[d] - v[d] * lwinv[d];
                nf = nf < -flim ? -flim : (nf > flim ? flim : nf);
                float df = nf - lam_fr[d];
                if (df != 0.0f) {
                    lam_fr[d] = nf;
                    for (int k = 0; k < D; k++) v[k] = fmaf(mrow[k], df, v[k]);
                }
            }
        }
        /* contact blocks (ha_physics.h): the three J.v reductions of a contact from the same v; the
         * friction rows see the normal / first-friction update through the block's Delassus entries. The packed
         * configuration (the clutter family) solves the link contacts this way in contact order and then the free
         * passes (contact_block_packed) */
        for (int c = 0; c < nc; c++) {
            if (packed && !is_link_contact(&cs[c])) continue;
            int r0 = 3 * c;
            float jv0 = wave_dot(R.J[r0], v, NV), jv1 = wave_dot(R.J[r0 + 1], v, NV), jv2 = wave_dot(R.J[r0 + 2], v, NV);
            float l0 = lam[r0], l1 = lam[r0 + 1], l2 = lam[r0 + 2];
            float n0 = l0 - (jv0 - R.vt[r0]) * winv[r0];
            n0 = n0 < 0.0f ? 0.0f : (n0 > 3.0e38f ? 3.0e38f : n0);
            float d0 = n0 - l0;
            float hi = (0.5f * (body_friction(h, e, cs[c].a) + body_friction(h, e, cs[c].b))) * n0;
            jv1 = fmaf(a10[c], d0, jv1);
            float n1 = l1 - (jv1 - R.vt[r0 + 1]) * winv[r0 + 1];
            n1 = n1 < -hi ? -hi : (n1 > hi ? hi : n1);
            float d1 = n1 - l1;
            jv2 = fmaf(a21[c], d1, fmaf(a20[c], d0, jv2));
            float n2 = l2 - (jv2 - R.vt[r0 + 2]) * winv[r0 + 2];
            n2 = n2 < -hi ? -hi : (n2 > hi ? hi : n2);
            float d2 = n2 - l2;
            lam[r0] = n0; lam[r0 + 1] = n1; lam[r0 + 2] = n2;
            if (d0 != 0.0f) for (int k = 0; k < NV; k++) v[k] = fmaf(R.Y[r0][k], d0, v[k]);
            if (d1 != 0.0f) for (int k = 0; k < NV; k++) v[k] = fmaf(R.Y[r0 + 1][k], d1, v[k]);
            if (d2 != 0.0f) for (int k = 0; k < NV; k++) v[k] = fmaf(R.Y[r0 + 2][k], d2, v[k]);
        }
        if (packed)
            for (int q = 0; q < npass; q++)
                for (int k = 0; k < 4; k++)
                    if (passes[q][k] >= 0) {
                        int c = passes[q][k], r0 = 3 * c;
                        float mu = 0.5f * (body_friction(h, e, cs[c].a) + body_friction(h, e, cs[c].b));
                        contact_block_packed(&cs[c], D, R.J[r0], R.J[r0 + 1], R.J[r0 + 2], R.Y[r0], R.Y[r0 + 1],
                                             R.Y[r0 + 2], R.vt + r0, winv + r0, lam + r0, mu, a10[c], a20[c], a21[c], v);
                    }
    }
    for (int d = 0; d < D; d++) e->dforce[d] = (((dlam[d] + lam_lo[d]) - lam_up[d]) + lam_fr[d]) / hdt;
    /* contact forces per body (net_contact_force): the last substep's forces */
    memset(e->cforce, 0, sizeof(e->cforce));
    for (int c = 0; c < nc; c++) {
        int r0 = 3 * c;
        v3 t1, t2;
        tangents(cs[c].n, &t1, &t2);
        v3 f = add(add(mul(cs[c].n, lam[r0]), mul(t1, lam[r0 + 1])), mul(t2, lam[r0 + 2]));
        f = mul(f, 1.0f / hdt);
        int bodies[2] = {cs[c].a, cs[c].b};
        for (int s = 0; s < 2; s++) {
            int bd = bodies[s];
            float sg = s == 0 ? 1.0f : -1.0f;
            int idx = -1;
            if (bd >= 100) idx = m->body_robot0 + (bd - 100);
            else if (bd >= 0) idx = m->body_object0 + bd;
            if (idx < 0) continue;
            e->cforce[idx][0] += sg * f.x; e->cforce[idx][1] += sg * f.y; e->cforce[idx][2] += sg * f.z;
        }
    }
    /* integrate (symplectic Euler) */
    for (int d = 0; d < D; d++) {
        e->qd[d] = v[d];
        e->q[d] += hdt * v[d];
    }
    for (int o = 0; o < NO; o++) {
        float* vo = v + D + 6 * o;
        e->ov[o] = V(vo[0], vo[1], vo[2]);
        e->ow[o] = V(vo[3], vo[4], vo[5]);
        e->oc[o] = add(e->oc[o], mul(e->ov[o], hdt));
        qt dq = qmul(Q(e->ow[o].x, e->ow[o].y, e->ow[o].z, 0.0f), e->oq[o]);
        qt q = e->oq[o];
        e->oq[o] = qnorm(Q(q.x + 0.5f * hdt * dq.x, q.y + 0.5f * hdt * dq.y, q.z + 0.5f * hdt * dq.z,
                           q.w + 0.5f * hdt * dq.w));
    }
}

/* ------------------------------------------------------------------ state load/store */
static void load_env(const hao_handle h, const ha_state_t* S, int env, env_t* e, int take_force) {
    const ha_model_t* m = &h->m;
    int D = h->D, A = h->A;
    e->dr = (h->p.dr_enable && S->dr_scale) ? S->dr_scale + (size_t)env * HA_DR_SIZE : NULL;
    e->drg = (e->dr && S->dr_global) ? S->dr_global : NULL;
    for (int d = 0; d < D; d++) {
        e->q[d] = S->dof_state[(env * D + d) * 2];
        e->qd[d] = S->dof_state[(env * D + d) * 2 + 1];
        e->tgt[d] = S->sim_targets[env * D + d];
    }
    for (int o = 0; o < h->NO; o++) {
        const float* r = S->root_state + (env * A + m->actor_object0 + o) * 13;
        int pid = (int)S->object_indices[env * h->NO + o];
        e->pool[o] = pid;
        /* object_scale row x the DR actor scale (ha_dr.h dr_object_scale); unscaled when neither applies */
        float ds = e->dr ? e->dr[HA_DR_OBJ_SCALE + o] : 1.0f;
        e->oscaled[o] = S->object_scale != NULL || ds != 1.0f;
        for (int k = 0; k < 3; k++) e->osc[o][k] = (S->object_scale ? S->object_scale[(env * h->NO + o) * 3 + k] : 1.0f) * ds;
        if (!e->oscaled[o]) e->osc[o][0] = e->osc[o][1] = e->osc[o][2] = 1.0f;
        e->ofx[o] = V(0, 0, 0);
        e->otq[o] = V(0, 0, 0);
        if (take_force && S->object_force) {
            float* fo = S->object_force + (env * h->NO + o) * 3;
            e->ofx[o] = ld3(fo);
            fo[0] = fo[1] = fo[2] = 0.0f;
        }
        if (take_force && S->object_torque) {
            float* tq = S->object_torque + (env * h->NO + o) * 3;
            e->otq[o] = ld3(tq);
            tq[0] = tq[1] = tq[2] = 0.0f;
        }
        e->oq[o] = ldq(r + 3);
        e->oc[o] = add(ld3(r), qrot(e->oq[o], scl(env_scale(e, o), ld3(m->pool_com[pid]))));
        e->ov[o] = ld3(r + 7);
        e->ow[o] = ld3(r + 10);
        e->coll[o] = S->collision_enabled ? S->collision_enabled[env * h->NO + o] : 1;
    }
    memset(e->cforce, 0, sizeof(e->cforce));
    memset(e->dforce, 0, sizeof(e->dforce));
    memset(e->cst, 0, sizeof(e->cst));
    e->pcm = S->contact_cache ? S->contact_cache + (size_t)env * h->pcm_slots * HA_PCM_REC : NULL;
    memset(e->sb, 0, sizeof(e->sb));
    if (m->posed_actor >= 0) {
        const float* r = S->root_state + (env * A + m->posed_actor) * 13;
        e->sb[0] = r[0]; e->sb[1] = r[1]; e->sb[2] = r[2];
        e->sb[4] = r[3]; e->sb[5] = r[4]; e->sb[6] = r[5]; e->sb[7] = r[6];
    }
}

static void store_env(const hao_handle h, ha_state_t* S, int env, env_t* e) {
    const ha_model_t* m = &h->m;
    int D = h->D, A = h->A, B = h->B;
    for (int d = 0; d < D; d++) {
        S->dof_state[(env * D + d) * 2] = e->q[d];
        S->dof_state[(env * D + d) * 2 + 1] = e->qd[d];
        if (S->dof_force) S->dof_force[env * D + d] = e->dforce[d];
    }
    for (int o = 0; o < h->NO; o++) {
        float* r = S->root_state + (env * A + m->actor_object0 + o) * 13;
        v3 pos = sub(e->oc[o], qrot(e->oq[o], scl(env_scale(e, o), ld3(m->pool_com[e->pool[o]]))));
        st3(r, pos); stq(r + 3, e->oq[o]); st3(r + 7, e->ov[o]); st3(r + 10, e->ow[o]);
    }
    /* rigid body states in the env's layout: robot links, objects, goal and table copied from the roots */
    fk(h, e);
    float* bs = S->rigid_body_state + (size_t)env * B * 13;
    const float* rs = S->root_state + (size_t)env * A * 13;
    if (m->body_goal >= 0) memcpy(bs + m->body_goal * 13, rs + m->actor_goal * 13, 13 * sizeof(float));
    twist Vl[HA_MAX_LINKS];
    for (int i = 0; i < m->n_links; i++) {
        int par = m->link_parent[i], d = m->link_dof[i];
        twist vp = {V(0, 0, 0), V(0, 0, 0)};
        if (par >= 0) vp = Vl[par];
        Vl[i] = vp;
        if (d >= 0) {
            Vl[i].w = add(vp.w, mul(e->ax[d], e->qd[d]));
            Vl[i].v = add(vp.v, mul(crs(e->an[d], e->ax[d]), e->qd[d]));
        }
        float* b = bs + (m->body_robot0 + i) * 13;
        v3 c = add(e->lp[i], qrot(e->lq[i], ld3(m->link_com[i])));
        v3 lin = add(Vl[i].v, crs(Vl[i].w, c));
        st3(b, e->lp[i]); stq(b + 3, e->lq[i]); st3(b + 7, lin); st3(b + 10, Vl[i].w);
    }
    if (m->body_table >= 0) memcpy(bs + m->body_table * 13, rs + m->actor_table * 13, 13 * sizeof(float));
    for (int k = 0; k < m->n_fixed_bodies; k++) {      /* fixed bodies: model pose, zero velocity */
        float* b = bs + (m->body_fixed0 + k) * 13;
        for (int t = 0; t < 13; t++) b[t] = t < 7 ? m->body_fixed_pose[k][t] : 0.0f;
    }
    for (int o = 0; o < h->NO; o++)
        memcpy(bs + (m->body_object0 + o) * 13, rs + (m->actor_object0 + o) * 13, 13 * sizeof(float));
    for (int b = 0; b < B; b++)
        for (int k = 0; k < 3; k++) S->net_contact_force[((size_t)env * B + b) * 3 + k] = e->cforce[b][k];
    if (S->contact_stats) {     /* added up over launches like the kernel's (column 2: the maximum) */
        int32_t* cs = S->contact_stats + (size_t)env * HA_CSTAT;
        for (int k = 0; k < HA_CSTAT; k++) cs[k] = k == 2 ? (e->cst[2] > cs[2] ? e->cst[2] : cs[2]) : cs[k] + e->cst[k];
    }
}

/* ------------------------------------------------------------------ public oracle API */
int hao_pcm_slots(const ha_model_t* m, int n_objects);
hao_handle hao_create(const ha_model_t* model, const ha_params_t* params, int num_envs) {
    hao_handle h = (hao_handle)calloc(1, sizeof(struct hao_s));
    h->m = *model;
    h->p = *params;
    h->N = num_envs;
    h->NO = params->n_objects;
    h->A = model->n_actors;
    h->D = model->n_dofs;
    h->B = model->n_bodies;
    /* the device family's capacity (ha_contact_capacity): clutter 4 chunks of 21 (handarm_hip.hip HB_CHUNKS),
       Ur5Sih 4 chunks of 21 (HA_CHUNKS), AllegroKuka 2 chunks of 21 (HA_AK_CONTACTS x HA_AK_CHUNKS), AllegroHand
       4 chunks of 12 (HA_AH_CONTACTS x HA_AH_CHUNKS); hao_set_capacity overrides it for A/B builds */
    h->maxc = params->task == HA_TASK_UR5SIH ? 4 * 21 : (params->task == HA_TASK_ALLEGRO_KUKA ? 2 * 21 : 4 * 12);
    h->pcm_slots = params->pcm_lin_tol > 0.0f ? hao_pcm_slots(model, params->n_objects) : 0;
    /* packed PGS passes (handarm_hip.hip HB_PACKED_PGS): 2 every substep of the clutter family; 1 would pack the 3-object
     * family's substeps whose contacts fit its chunk 0 (21), as a -DHA_PACKED_PGS=1 kernel build does (off: slower) */
    h->packed = params->task == HA_TASK_UR5SIH && params->n_objects > 3 ? 2 : 0;
    return h;
}
void hao_destroy(hao_handle h) { free(h); }
/* contact capacity of the device build under test (ha_contact_capacity): a build with other chunk macros */
void hao_set_capacity(hao_handle h, int maxc) { if (maxc > 0 && maxc <= MAXC) h->maxc = maxc; }
/* OpenMP threads of hao_simulate (bench.py's cpu_baseline reports an all-cores and a 1-thread sample) */
void hao_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
int hao_get_threads(void) { return omp_get_max_threads(); }
/* test hook: the compound piece-pair box test (include/ha_obb.h ha_obb_pair_near), for tests/test_box_cull.py */
int hao_obb_pair_near(const float* p1, const float* q1, const float* ob1, const float* p2, const float* q2,
                      const float* ob2, float mg) {
    return ha_obb_pair_near(p1, q1, ob1, p2, q2, ob2, mg);
}
int hao_struct_sizes(int32_t* model_size, int32_t* params_size, int32_t* state_size) {
    *model_size = (int32_t)sizeof(ha_model_t);
    *params_size = (int32_t)sizeof(ha_params_t);
    *state_size = (int32_t)sizeof(ha_state_t);
    return 0;
}

static void simulate_env(const hao_handle h, ha_state_t* S, int env, int n_calls) {
    env_t e;
    load_env(h, S, env, &e, 1);
    float hdt = h->p.dt / (float)h->p.substeps;
    for (int c = 0; c < n_calls; c++) {
        for (int s = 0; s < h->p.substeps; s++) substep(h, &e, hdt);
        /* an applied force lasts one gym.simulate (apply_rigid_body_force_tensors, then the next simulate call):
         * the later calls of a multi-call launch run without it (handarm_hip.hip run_physics force_once) */
        for (int o = 0; o < NOBJ; o++) e.ofx[o] = e.otq[o] = (v3){0.0f, 0.0f, 0.0f};
    }
    /* net contact force of the last substep (PhysX reports the last substep's forces) */
    store_env(h, S, env, &e);
}

/* the contacts detect() produces for env's current state (test helper): rows of 9 floats x[3], n[3], sep, a, b */
int hao_contacts(hao_handle h, ha_state_t* S, int env, float* out, int max_rows) {
    env_t e;
    load_env(h, S, env, &e, 0);
    e.pcm = NULL;                       /* the narrow phase's contacts, no persistent manifold */
    fk(h, &e);
    contact_t cs[MAXC];
    int nc = detect(h, &e, cs);
    for (int i = 0; i < nc && i < max_rows; i++) {
        float* r = out + 9 * i;
        r[0] = cs[i].x.x; r[1] = cs[i].x.y; r[2] = cs[i].x.z;
        r[3] = cs[i].n.x; r[4] = cs[i].n.y; r[5] = cs[i].n.z;
        r[6] = cs[i].sep; r[7] = (float)cs[i].a; r[8] = (float)cs[i].b;
    }
    return nc;
}

void hao_simulate(hao_handle h, ha_state_t* S, int n_calls, int env_begin, int env_end) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int env = env_begin; env < env_end; env++) simulate_env(h, S, env, n_calls);
}

/* --------------------------------------------------------------- task math (see task_oracle.py) */
static float spline_eval(const ha_params_t* p, int s, float t) {
    int n = p->spline_pieces[s];
    /* bucketize(t, knots) - 1 clamped to [0, n-1]; knots[k] = t0[k], knots[n] not needed */
    int idx = 0;
    for (int k = 1; k < n; k++)
        if (t > p->spline[s][0][k]) idx = k;
    float f = t - p->spline[s][0][idx];
    float inner = 0.5f * p->spline[s][3][idx] + p->spline[s][4][idx] * f / 3.0f;
    inner = p->spline[s][2][idx] + inner * f;
    return p->spline[s][1][idx] + inner * f;
}

enum { D_INDEX = 6, D_IF_DISTAL, D_LF, D_LF_DISTAL, D_MIDDLE, D_MF_DISTAL, D_RING, D_RF_DISTAL, D_TH_OPP, D_TH_FLEX,
       D_TH_DISTAL };

void hao_controller(hao_handle h, ha_state_t* S, int env) {
    const ha_params_t* p = &h->p;
    const float* a = S->actions + env * 11;
    float* ur5 = S->ur5_target + env * 6;
    float* servo = S->servo + env * 5;
    float* sm = S->smoothed + env * 5;
    float* tgt = S->dof_position_targets + env * h->D;
    const float* dof = S->dof_state + (size_t)env * h->D * 2;
    for (int i = 0; i < 6; i++) ur5[i] = ur5[i] + p->action_dt * a[i];
    float alpha = p->sih_alpha, beta = p->sih_beta;
    for (int i = 0; i < 5; i++) {
        sm[i] = alpha * a[6 + i] + beta * sm[i];
        float s = servo[i] + 100.0f * sm[i];
        s = s < p->servo_lower[i] ? p->servo_lower[i] : s;
        s = s > p->servo_upper[i] ? p->servo_upper[i] : s;
        servo[i] = s;
    }
    for (int i = 0; i < 6; i++) tgt[i] = ur5[i];
    tgt[D_TH_OPP] = p->thumb_opposition_gain * servo[0];
    tgt[D_TH_FLEX] = -spline_eval(p, 0, servo[1]);
    tgt[D_TH_DISTAL] = -spline_eval(p, 1, servo[1] + p->proximal_coef[0] * dof[2 * D_TH_FLEX]);
    tgt[D_INDEX] = spline_eval(p, 2, servo[2]);
    tgt[D_IF_DISTAL] = spline_eval(p, 3, servo[2] + p->proximal_coef[1] * dof[2 * D_INDEX]);
    tgt[D_MIDDLE] = spline_eval(p, 4, servo[3]);
    tgt[D_MF_DISTAL] = spline_eval(p, 5, servo[3] + p->proximal_coef[2] * dof[2 * D_MIDDLE]);
    tgt[D_RING] = spline_eval(p, 6, servo[4]);
    tgt[D_RF_DISTAL] = spline_eval(p, 7, servo[4] + p->proximal_coef[3] * dof[2 * D_RING]);
    tgt[D_LF] = tgt[D_RING];
    tgt[D_LF_DISTAL] = tgt[D_RF_DISTAL];
    for (int d = 0; d < h->D; d++) S->sim_targets[env * h->D + d] = tgt[d];
}

/* test helper: the shared float32 sine / cosine (include/ha_fmath.h) over an array, for the numpy port in
   oracle/f32.py */
void hao_sincos(const float* x, int n, float* s, float* c) {
    for (int i = 0; i < n; i++) ha_sincosf(x[i], &s[i], &c[i]);
}
/* test helper: ha_logf(x) and ha_expf(1e-3 x - 3) (the DR samplers' shared log / exp, include/ha_fmath.h) */
void hao_logexp(const float* x, int n, float* lo, float* ex) {
    for (int i = 0; i < n; i++) {
        lo[i] = ha_logf(x[i]);
        ex[i] = ha_expf(x[i] * 1e-3f - 3.0f);
    }
}
