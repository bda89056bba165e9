// ha_physics.h - one-wavefront-per-environment articulated + rigid-body physics for gfx950.
//
// Algorithm (identical to oracle/physics_oracle.c, which is its scalar restatement):
//   FK (level-synchronous over the link tree) -> CRBA joint-space inertia + RNEA velocity-product
//   forces in world-frame spatial algebra -> Cholesky (lane i owns row i) -> triangular inverse
//   (lane j owns column j) -> explicit M^-1 = L^-T L^-1 -> convex-hull contacts (SAT + incident vertices,
//   <= 4 per pair) -> projected Gauss-Seidel in velocity form:
//     * joint rows (PD drives as impulse-bounded soft constraints, joint limits) live in lane d and need
//       no reduction (J = +-e_d, J v = v[d]);
//     * contact rows (normal + 2 friction) keep J_r and Y_r = M^-1 J_r^T in LDS; J_r . v is one DPP
//       row reduction + 4 v_readlane; the velocity update is one LDS read + FMA per lane.
//   Generalised velocity v lives one coordinate per lane for the whole solve -> symplectic Euler.
// Everything loops at run time (small code: the kernel must stay resident in the instruction cache),
// and the phase-local scratch (dynamics, collision, rows) shares one LDS union.
#pragma once
#include <type_traits>

#include "ha_device.h"
#include "../../include/handarm_abi.h"
#include "../../include/ha_obb.h"

#define MAXC 21          /* contacts per chunk: 3 rows each -> 63 rows, one per lane (lane 63 idle) */
#define MAXR (3 * MAXC)
#define RS 35            /* max row stride: D + 6 * n_obj <= 35 (Ur5Sih); see row_stride<ND>() */
#define NOBJ HA_MAX_OBJ
#define MAXD 24
#define HA_ND 17         /* DOF count the kernels are compiled for (UR5 + SIH); checked by ha_create */
// compound object pair: reduced points gathered over its piece pairs (later ones dropped; the oracle's MAXGATHER)
#define HA_MAX_GATHER 32
#define MAXB 44          /* rigid bodies per env (contact-force rows): robot links + objects + statics (bin scene: 44) */
#define MAXV 72          /* generalized velocity coordinates D + 6 x objects (17 + 6 x 8 = 65 for bin-picking) */

// What the task observables read after refresh_simulation_tensors(): flange pose, fingertip states,
// dof positions, object root states (filled from FK in the fused step, or from the state tensors).
struct ObsIn {
    float flange[8];
    float tip[5][10];      // pos, quat, linvel
    float dofpos[MAXD];
    float obj[NOBJ][13];
    float pad[2];
};

struct DynScratch {
    float Ic[HA_MAX_LINKS][13];                 // composite spatial inertia (m, h, J) at world origin
    float Al[HA_MAX_LINKS][6], Fl[HA_MAX_LINKS][6];
};
// Narrow-phase scratch in the phase union, laid out per kernel family for its largest hull (NV vertices, NP face
// planes; ha_create checks the model against it): world vertices and planes of both hull sides, the clipping
// candidates and their max side-plane distances, and a compound pair's gathered points and normals
// (NG gathered points: HA_MAX_GATHER, or 0 for a family without compound objects, which ha_create enforces)
template <int NV, int NP, int NG = HA_MAX_GATHER>
struct ColLayout {
    static constexpr size_t wvA = 0, wvB = wvA + 16 * NV, wpA = wvB + 16 * NV, wpB = wpA + 16 * NP;
    static constexpr size_t cand = wpB + 16 * NP, cmax = cand + 4 * NV, gp = cmax + 4 * NV;
    static constexpr size_t gn = gp + 16 * NG, bytes = gn + 16 * NG;
};
struct ColView {
    float (*wvA)[4], (*wvB)[4];         // world vertices of both hulls
    float (*wpA)[4], (*wpB)[4];         // world face planes (n, d) of both hulls
    int* cand;                          // clipping: candidate incident vertices
    int* cmax;                          // clipping: per-candidate max plane distance (order-preserving int)
    float (*gp)[4], (*gn)[4];           // compound object pair: gathered points (x, sep) and normals
};
struct RowScratch {
    float J[MAXR * RS];
    float Y[MAXR * RS];
};
// Dynamics (M + spatial scratch) and, after the physics, the refresh / observation staging, which overlap:
// the staging and the last substep's joint / contact forces (written after each substep's PGS) are only read
// after the last substep, and the next substep's dynamics may overwrite them. The link twists Vl are written
// by the dynamics and again by the refresh (link_twists), and read by the observation staging, so they stay
// outside the overlap.
struct PostScratch {
    float Vl[HA_MAX_LINKS][6];                  // link twists (w, v at the world origin)
    union {
        struct {
            float M[MAXD * MAXD];               // M, then its Cholesky factor L (stride D)
            DynScratch dyn;
        };
        struct {
            ObsIn in;
            float obs[216];                     // Ur5Sih: 108 + 13 x objects (212 at 8 objects)
            float cforce[MAXB][3];
            float dforce[MAXD];                 // joint force of the last substep (drive + limits) / h
        };
    };
};

// One free object's state (LDS). These live after the EnvLDS block, one per object slot of the task
// (Ur5Sih 3, bin-picking 7, AllegroHand / AllegroKuka 1), so the object capacity costs only the tasks
// that use it.
struct ObjLDS {
    float oc[4], oq[4], ov[4], ow[4];   // COM position, orientation, linear / angular velocity
    float oIinv[9];                     // world inverse inertia (3x3)
    float otq[3];                       // v16: world torque for this physics call (apply_rigid_body_force_tensors)
    float osc[4];                       // per-env dimension scale of the pool hull; [3] = 1 when scaled
    float ofx[4];                       // world force on the COM for this physics call (apply_rigid_body_force)
    float om;                           // mass
    int pool, coll;                     // pool id, collision enabled
};

// One contact point (LDS, after the object slots): up to MAXC x chunks per env (task_lds_bytes).
// 32 bytes: the combined friction is not stored (contact_friction(a, b) again in the rows phase, the same
// value), and the body codes fit 16 bits
struct ContactLDS {
    float x[3], n[3];                   // world point, normal from body b to body a
    float sep;                          // separation (< 0: penetration)
    short a, b;                         // body codes: -1 static, 0..NOBJ-1 object, 100 + link
};
static_assert(sizeof(ContactLDS) == 32, "ContactLDS layout");

struct EnvLDS {
    float q[MAXD], qd[MAXD], tgt[MAXD];
    float lp[HA_MAX_LINKS][3], lq[HA_MAX_LINKS][4];
    float ax[MAXD][3], an[MAXD][3];
    float Cb[MAXD];
    float v[MAXV];
    int nc, nr, noff, ng;                       // contacts kept / rows / contacts offered this substep /
                                                // points gathered for a compound object pair
    int cst[HA_CSTAT];                          // contact_stats of this launch (see ha_state_t)
    float sb[8];                                // pose of the actor carrying posed statics (v14): p[3], pad, q[4]
    union {
        PostScratch pd;                         // (the narrow-phase scratch, ColLayout, is sized per family)
        RowScratch rows;
        float xfer[MAXR * HA_MAX_CONTACTS / MAXC];  // lane exchange outside the physics phases (controller;
                                                    // PGS impulses of every row -> contact forces). Must stay
                                                    // below the rows' RK area (static_assert in PhysCfg users)
    } u;
};

// Compact constraint rows: a contact touches at most two free objects, so a row stores the robot block (D)
// plus one 6-wide block per object slot (slot 0 = the lower object index, slot 1 = the other), instead of
// all D + 6 x n_obj coordinates. Ur5Sih (3 objects): stride 17 + 12; one-object tasks (AllegroHand 16,
// AllegroKuka 23 DOF): D + 6. Dot products over a compact row visit the nonzero terms in the same order as
// the dense row, so results are unchanged; the LDS saving is what lets these kernels run 8 workgroups per CU.
template <int ND>
__host__ __device__ constexpr int row_slots() { return ND == HA_ND ? 2 : 1; }
template <int ND>
__host__ __device__ constexpr int row_stride() { return ND + 6 * row_slots<ND>(); }
// object slots of a contact between bodies a and b (codes: -1 static, 0..NOBJ-1 object, 100+ link)
HD void contact_slots(int a, int b, int& so0, int& so1) {
    int oa = (a >= 0 && a < 100) ? a : -1, ob = (b >= 0 && b < 100) ? b : -1;
    so0 = oa < 0 ? ob : (ob < 0 ? oa : (oa < ob ? oa : ob));
    so1 = (oa >= 0 && ob >= 0) ? (oa < ob ? ob : oa) : -1;
}
// index of generalized coordinate `lane` in a compact row (-1: not touched by the contact)
HD int compact_index(int lane, int D, int so0, int so1) {
    if (lane < D) return lane;
    int t = lane - D;
    if (so0 >= 0 && t >= 6 * so0 && t < 6 * so0 + 6) return D + t - 6 * so0;
    if (so1 >= 0 && t >= 6 * so1 && t < 6 * so1 + 6) return D + 6 + t - 6 * so1;
    return -1;
}
// LDS block of one env: EnvLDS up to the phase union, the union at the task's row stride and contact
// chunks (J and Y of MAXR x chunks rows), then the object slots (ObjLDS x capacity), then the contact list
// (ContactLDS x MAXC x chunks), 16-byte aligned
__host__ __device__ inline size_t obj_lds_offset_rows(size_t rows) {
    size_t u = sizeof(PostScratch);
    if (rows > u) u = rows;
    return (offsetof(EnvLDS, u) + u + 15) & ~(size_t)15;
}

// Compile-time shape of a kernel family's physics: DOF count, object slots, contact chunks (MAXC contacts
// each) and velocity words per lane (coordinates lane and lane + 64 when D + 6 x objects > 64).
//
// Split rows (split = true): most clutter contacts touch no robot link (object-bin, object-object), and such a
// row's robot block is zero in J and in Y = M^-1 J^T. The rows then keep only their object blocks in LDS (OW =
// 6 x object slots floats each of J and Y), and the robot blocks of the contacts that do touch a link get a slot
// of their own: the first KL link contacts in LDS, the rest in a per-env global spill area (ha_create allocates
// it; L2-resident, rare). Every dot product visits the nonzero terms in the dense order and a skipped zero block
// adds exact zeros, so results are bit-identical to the dense rows. The Ur5Sih families (3 and 8 object slots)
// split by default (HA_SPLIT_ABOVE_OCAP); AllegroKuka (one object slot, SPLIT = 1) splits too: its cube-table
// contacts, most of the list, touch no link.
//
// Minv in the union (MU = true, AllegroKuka): S ~ M^-1 sits at the END of the phase union, over the dynamics
// scratch (dead once dynamics() has produced M and Cb) and clear of M (which factor_inverse reads while writing
// S), of the narrow-phase scratch (detect runs while S is live) and of the constraint rows (the rows phase and
// the PGS read S): the static_asserts below check the three. Otherwise S follows the union.
#ifndef HA_SPLIT_ABOVE_OCAP
#define HA_SPLIT_ABOVE_OCAP 2   /* families with more object slots use split rows (Ur5Sih 3 objects, clutter) */
#endif
//
// Overflow chunks (OVF = true, the Ur5Sih and AllegroHand families): chunk 0 keeps the family's LDS layout (contact
// entries, rows, the PGS row constants in registers), and chunks 1..NCH-1 keep their contact entries, constraint rows
// and row constants in the env's global area (L2-resident), so the contact capacity grows without LDS. A substep
// with <= CAP contacts never touches that area; a substep over CAP swaps every chunk's row constants through it.
#define HA_PAIRF_LINK_HULLS 64     /* link hulls the pair face records are sized for */
template <int ND, int OCAP, int NCH, int KL = 8, int LCH = NCH, int CAP = MAXC, int CV = 64, int CP = 128,
          int SPLIT = -1, int NG = HA_MAX_GATHER, bool MU = false, bool RC = false, bool OVF = false, bool SELF = false,
          bool PACK = false>
struct PhysCfg {
    static constexpr int nd = ND, ocap = OCAP, nch = NCH;
    // packed PGS passes (the clutter family): the contacts that touch no robot link are solved four at a time, one
    // per 16-lane row, in passes of contacts on disjoint objects (ha_physics.h substep, "free passes"); their
    // object-block rows must all be in the env's global row area
    static constexpr bool pack = PACK;
    // overflow families pack only the substeps whose contacts fit chunk 0 (their rows in LDS); max_passes also counts
    // the contacts whose constants PK holds
    static constexpr int max_passes = OVF ? CAP : CAP * NCH;
    // the family's robot collides with itself (ha_model_t v12 self pairs; the Allegro families). Without it the
    // self-pair pass is not compiled (its registers would count against every family)
    static constexpr bool selfc = SELF;
    static constexpr int colv = CV, colp = CP, colg = NG;   // largest hull: vertices, face planes; gather points
    static constexpr size_t col_bytes = ColLayout<CV, CP, NG>::bytes;
    // contacts per chunk (MAXC, or fewer: the rows and the LDS list shrink with it)
    static constexpr int cap = CAP;
    static constexpr bool ovf = OVF && NCH > 1;
    static constexpr int rpc = 3 * CAP;             // constraint rows per chunk
    static constexpr int vw = ND + 6 * OCAP > 64 ? 2 : 1;
#ifdef HA_DENSE_ROWS    /* diagnostic build (tools/split_rows_check.py): every family on dense rows */
    static constexpr bool split = false;
#else
    static constexpr bool split = SPLIT >= 0 ? SPLIT != 0 : OCAP > HA_SPLIT_ABOVE_OCAP;
#endif
    static constexpr int ow = 6 * row_slots<ND>();  // split rows: object-block width
    static constexpr int kl = KL;
    static constexpr bool minv_in_union = MU;
    // split rows with recomputed object blocks (RC, the clutter family): no object-block rows are stored at all; the
    // rows phase and the PGS evaluate a contact row's object blocks in registers from the contact entry (obj_blocks)
    static constexpr bool rc = RC && split;
    // split rows: the object blocks of chunks [0, lch) live in LDS, those of chunks [lch, nch) in the env's global
    // row area after the robot-block spill rows (written by the rows phase, read back by the PGS one contact ahead)
    // (OVF: chunk 0's rows in LDS, split or dense, the others in the global area)
    static constexpr int lch = ovf ? 1 : (split ? LCH : NCH);
    static constexpr int spill_robot = split ? 2 * 3 * (CAP * NCH - KL) * ND : 0;   // per env: J then Y
    static constexpr int spill_obj = split && !rc ? 2 * rpc * (NCH - lch) * ow : 0;  // per env: J then Y
    // OVF global area after those: dense rows of chunks 1.. (J then Y), the row constants of every chunk (6 x rpc x
    // NCH, the LDS RK layout), the contact entries of chunks 1.. (8 floats each)
    static constexpr int spill_dense = ovf && !split ? 2 * rpc * (NCH - 1) * row_stride<ND>() : 0;
    // PGS row constants (RK): 6 arrays of rk_stride floats (impulse, target velocity, 1/diagonal, friction, two Delassus
    // entries), each indexed by the row over all chunks. The kernel's rk() indexes with rk_stride and both RK areas (LDS
    // for the non-overflow multi-chunk family, the global area for OVF) are sized from it: one constant, so the index
    // range and the allocation cannot disagree (the first overflow build indexed with the LDS layout's 63-row MAXR
    // stride while AllegroHand's 12-contact chunks have 36 rows: DESIGN.md §3.12)
    static constexpr int rk_stride = rpc * NCH;
    static constexpr int spill_rk = ovf ? 6 * rk_stride : 0;
    static constexpr int spill_ct = ovf ? 8 * CAP * (NCH - 1) : 0;
    static constexpr int off_dense = spill_robot + spill_obj, off_rk = off_dense + spill_dense,
                         off_ct = off_rk + spill_rk;
    // self-collision families: one byte per self pair, the separating face of the pair's last narrow phase
    static constexpr int spill_selfc = SELF ? HA_MAX_SELF_PAIRS / 4 : 0;
    static constexpr int off_selfc = off_ct + spill_ct;
    // every family: one byte per candidate pair of detect's enumeration, the separating face of the pair's last narrow
    // phase (the self pairs' record, for the other pairs); bounded for up to HA_PAIRF_LINK_HULLS link hulls and
    // HA_MAX_STATIC statics (ha_create checks the model against it)
    static constexpr int pairf_bytes = OCAP * (1 + HA_MAX_STATIC + OCAP + HA_PAIRF_LINK_HULLS) + HA_PAIRF_LINK_HULLS * HA_MAX_STATIC;
    static constexpr int spill_pairf = (pairf_bytes + 3) / 4;
    static constexpr int off_pairf = off_selfc + spill_selfc;
    static constexpr int spill_floats = off_pairf + spill_pairf;
    static_assert(ND + 6 * OCAP <= MAXV, "generalized velocity exceeds MAXV");
    static_assert(!split || (KL >= 0 && KL <= CAP * NCH), "LDS link slots must not exceed the contact capacity");
    static_assert(!split || CAP * NCH <= 128, "split rows: <= 128 contacts");
    static_assert(split || CAP * NCH <= 64, "dense rows: <= 64 contacts (one ballot)");
    static_assert(lch >= 0 && lch <= NCH, "LDS row chunks");
    static_assert(CAP * NCH <= HA_MAX_CONTACTS, "contact capacity exceeds HA_MAX_CONTACTS");
    static_assert(CAP >= 1 && CAP <= MAXC, "contacts per chunk");
    static_assert(!ovf || !rc, "overflow chunks with recomputed object blocks");
    static_assert(NG == 0 || NG == HA_MAX_GATHER, "gather buffer: HA_MAX_GATHER points or none");
    static_assert(CP >= 8, "sat_planes reads plane slots 0..7 of the narrow-phase scratch");
    static_assert(!PACK || (SPLIT != 0 && OCAP > HA_SPLIT_ABOVE_OCAP && !RC && NCH > 1 && (OVF ? CAP <= 21 : LCH == 0)),
                  "packed passes: split rows; either every object-block row in the global area with RK in LDS, or "
                  "(overflow chunks) chunk 0's rows in LDS with their constants in registers");
};
// bytes of the constraint rows proper, then (several contact chunks only) the per-row PGS constants of every
// chunk (impulse, target velocity, 1/diag, friction, two Delassus entries: 6 floats x MAXR x chunks), which the
// PGS swaps into registers one chunk at a time
template <class PC>
__host__ __device__ constexpr size_t pc_rowdata_bytes() {
    return PC::split ? 2 * sizeof(float) * ((size_t)PC::rpc * PC::lch * PC::ow + 3 * (size_t)PC::kl * PC::nd)
                     : 2 * sizeof(float) * (size_t)PC::rpc * PC::lch * row_stride<PC::nd>();
}
// packed families (PhysCfg PACK) keep a packed substep's PGS constants per contact instead (PK, 12 floats: impulses
// l0 l1 l2, the normal row's target velocity, the three 1/diagonals, the friction coefficient, the Delassus entries
// a10 a20 a21, 0; the friction rows' target velocities are 0)
#define HA_PK 12
template <class PC>
__host__ __device__ constexpr size_t pc_rows_bytes() {
    return PC::pack ? pc_rowdata_bytes<PC>() + sizeof(float) * HA_PK * (size_t)PC::max_passes
                    : pc_rowdata_bytes<PC>() + (PC::nch > 1 && !PC::ovf ? 6 * sizeof(float) * (size_t)PC::rk_stride : 0);
}
template <class PC>
__host__ __device__ constexpr size_t pc_pk_offset() { return pc_rowdata_bytes<PC>(); }

// S ~ M^-1 (factor_inverse), D x D at stride D, sized for the family's DOF count: at the end of the union
// (minv_in_union) or after it
// (after the constraint rows when those reach past it: the union then grows by the difference, which the
// AllegroKuka layout spends on a third LDS link slot)
template <class PC>
__host__ __device__ constexpr size_t minv_union_offset() {
    size_t a = (sizeof(PostScratch) - (size_t)PC::nd * PC::nd * sizeof(float)) & ~(size_t)15;
    size_t r = (pc_rows_bytes<PC>() + 15) & ~(size_t)15;
    return a > r ? a : r;
}
template <class PC>
__host__ __device__ inline size_t minv_lds_offset() {
    if constexpr (PC::minv_in_union) {
        static_assert(offsetof(PostScratch, M) + (size_t)PC::nd * PC::nd * sizeof(float) <= minv_union_offset<PC>(),
                      "S must not overlap M (factor_inverse reads M while writing S)");
        static_assert(offsetof(PostScratch, dyn) <= minv_union_offset<PC>(), "S may overlap only the dynamics scratch");
        static_assert(PC::col_bytes <= minv_union_offset<PC>(), "S must not overlap the narrow-phase scratch");
        static_assert(pc_rows_bytes<PC>() <= minv_union_offset<PC>(), "S must not overlap the constraint rows");
        return offsetof(EnvLDS, u) + minv_union_offset<PC>();
    } else {
        return obj_lds_offset_rows(pc_rows_bytes<PC>() > PC::col_bytes ? pc_rows_bytes<PC>() : PC::col_bytes);
    }
}
// the family's narrow-phase scratch view into the phase union
template <class PC>
__device__ inline ColView col_view(void* u) {
    using L = ColLayout<PC::colv, PC::colp, PC::colg>;
    char* b = reinterpret_cast<char*>(u);
    ColView v;
    v.wvA = reinterpret_cast<float(*)[4]>(b + L::wvA); v.wvB = reinterpret_cast<float(*)[4]>(b + L::wvB);
    v.wpA = reinterpret_cast<float(*)[4]>(b + L::wpA); v.wpB = reinterpret_cast<float(*)[4]>(b + L::wpB);
    v.cand = reinterpret_cast<int*>(b + L::cand); v.cmax = reinterpret_cast<int*>(b + L::cmax);
    v.gp = reinterpret_cast<float(*)[4]>(b + L::gp); v.gn = reinterpret_cast<float(*)[4]>(b + L::gn);
    return v;
}
template <class PC>
__host__ __device__ inline size_t obj_lds_offset() {
    if constexpr (PC::minv_in_union) {
        size_t u = pc_rows_bytes<PC>() > PC::col_bytes ? pc_rows_bytes<PC>() : PC::col_bytes;
        size_t se = minv_union_offset<PC>() + (size_t)PC::nd * PC::nd * sizeof(float);
        return obj_lds_offset_rows(u > se ? u : se);
    }
    else
        return (minv_lds_offset<PC>() + (size_t)PC::nd * PC::nd * sizeof(float) + 15) & ~(size_t)15;
}
template <class PC>
__host__ __device__ inline size_t contact_lds_offset() {
    return obj_lds_offset<PC>() + (size_t)PC::ocap * sizeof(ObjLDS);
}
template <class PC>
__host__ __device__ inline size_t selfm_lds_offset() {
    return contact_lds_offset<PC>() + (size_t)PC::cap * (PC::ovf ? 1 : PC::nch) * sizeof(ContactLDS);
}
// the self-collision candidate bits (detect_self), a bit a pair, after the contact list: only in the families that
// collide the robot with itself, so the others' env blocks do not grow
template <typename PC>
__host__ __device__ inline size_t task_lds_bytes() {
    return selfm_lds_offset<PC>() + (PC::selfc ? HA_MAX_SELF_PAIRS / 8 : 0);
}

struct SimCtx {
    const ha_model_t* __restrict__ m;
    const ha_params_t* __restrict__ p;
    EnvLDS* s;
    ObjLDS* o;              // the env's object slots (after the EnvLDS block, see task_lds_bytes)
    ContactLDS* k;          // the env's contact list (after the object slots): entries [0, kc0)
    ContactLDS* kg;         // overflow chunks (PhysCfg OVF): entries [kc0, maxc) in the env's global area; null
                            // otherwise (a constant the compiler folds: ct_global is then false)
    int kc0;                // entries in LDS
    float* Minv;            // S ~ M^-1, D x D (after the phase union, see obj_lds_offset)
    ColView col;            // narrow-phase scratch of the family (col_view)
    int lane, D, NO, L;
    int maxc;               // contact capacity (MAXC x chunks of the kernel family)
    const float* dr;        // this env's domain-randomization row (HA_DR_*), or null when DR is off
    const float* drg;       // v16: the shard-wide randomization state (ha_state_t.dr_global, HA_DRG_*), null: DR off
    float* spill;           // split rows: this env's global robot-block rows beyond the LDS slots (J, then Y)
    // narrow-phase cache: (hull, body) whose world vertices / planes are in ColScratch side A / side B. Within one
    // detect() the poses do not change, so consecutive pairs that share a side skip its setup (same values).
    int colA_h, colA_b, colB_h, colB_b;
    bool colA_p;            // side A's world planes are in ColScratch too (SAT B runs first and may exit before them)
    bool gather;            // a compound object pair's piece pairs: reduced points go to ColScratch gp / gn
    // self-collision pairs (PhysCfg SELF): the separating face the last narrow phase found (0x80 | k: face k of side B,
    // k: face k of side A, 0xFF: none), and the env's per-pair record of it in its global area (null otherwise)
    int sepf;
    uint8_t* selfc;
    uint8_t* pairf;         // the candidate pairs' separating-face records (PhysCfg off_pairf; null: off)
    uint32_t* selfm;        // LDS: this substep's self-pair candidates, a bit a pair (selfm_lds_offset; null otherwise)
    // VecTask.step's head and tail folded into the step launch (ha_task_step_io; null / unused otherwise): the caller's
    // raw actions, clamped to +-clip_act where the task reads them (act_at), and a second, clamped copy of obs
    const float* act_in;
    float* obs_out;
    float clip_act, clip_obs;
    // persistent contact manifolds (ha_params_t v13): this env's records (ha_state_t.contact_cache; null: off), and
    // the running pair's slot (-1: none) and description, whose narrow phase writes the record it emits
    float* pcm;
    int pslot, pkind, pA, pB;
    int pemit;              // points of the running pair's manifold staged for its record (pcm_commit), 0: none
#ifdef HA_PROFILE
    int pk;                 // profiled build: kind of the running pair
    int pcls;               // profiled build: this substep is heavy (g_prof's second set)
#endif
#ifdef HA_AB_TIMING
    bool dry;               // A/B timing builds only: a repeated phase that must not emit contacts
#endif
};

// obs_dict["obs"] = clamp(obs_buf, -clip, clip) (vec_task.py:437) next to obs_buf, when the launch asks for it
HD void obs_out_put(const SimCtx& c, size_t i, float v) {
    if (c.obs_out) c.obs_out[i] = fminf(fmaxf(v, -c.clip_obs), c.clip_obs);
}

// Contact entry ci of the list: LDS for [0, kc0), the env's global overflow entries after that (PhysCfg OVF). Read and
// written by value: a pointer that may address either LDS or global memory would be a flat pointer, so each access
// keeps its two address spaces on separate paths.
HD bool ct_global(const SimCtx& c, int ci) { return c.kg != nullptr && ci >= c.kc0; }
// The two branches address different memories on purpose; the address-space casts keep the compiler from merging
// them into one generic (flat) access through a selected pointer: a flat load waits on the vector-memory counter
// too, so one in the PGS loop (ct_ab) would also wait for the global rows prefetched for the next contact
#define HA_AS_LDS __attribute__((address_space(3)))
#define HA_AS_GLB __attribute__((address_space(1)))
HD const HA_AS_LDS ContactLDS* ct_lds(const SimCtx& c, int ci) { return (const HA_AS_LDS ContactLDS*)(c.k + ci); }
HD const HA_AS_GLB ContactLDS* ct_glb(const SimCtx& c, int ci) {
    return (const HA_AS_GLB ContactLDS*)(c.kg + (ci - c.kc0));
}
HD ContactLDS ct_get(const SimCtx& c, int ci) {
    ContactLDS r;
    if (ct_global(c, ci)) {
        const HA_AS_GLB ContactLDS* g = ct_glb(c, ci);
        r.x[0] = g->x[0]; r.x[1] = g->x[1]; r.x[2] = g->x[2];
        r.n[0] = g->n[0]; r.n[1] = g->n[1]; r.n[2] = g->n[2];
        r.sep = g->sep; r.a = g->a; r.b = g->b;
    } else {
        const HA_AS_LDS ContactLDS* l = ct_lds(c, ci);
        r.x[0] = l->x[0]; r.x[1] = l->x[1]; r.x[2] = l->x[2];
        r.n[0] = l->n[0]; r.n[1] = l->n[1]; r.n[2] = l->n[2];
        r.sep = l->sep; r.a = l->a; r.b = l->b;
    }
    return r;
}
HD float ct_sep(const SimCtx& c, int ci) {
    if (ct_global(c, ci)) return ct_glb(c, ci)->sep;
    return ct_lds(c, ci)->sep;
}
HD void ct_ab(const SimCtx& c, int ci, int& a, int& b) {
    if (ct_global(c, ci)) {
        a = ct_glb(c, ci)->a;
        b = ct_glb(c, ci)->b;
    } else {
        a = ct_lds(c, ci)->a;
        b = ct_lds(c, ci)->b;
    }
}
// typed views of a row pointer the caller knows to be LDS / global (the PGS fetch's two load paths stay apart). T =
// false keeps the generic pointer: the compact AllegroKuka layout at 128 VGPRs measured +1.6% with typed paths (more
// live registers, 72 -> 84 B/lane of spills), the other families -1 to -2%
template <bool T = true>
HD auto lds_f(const float* p) {
    if constexpr (T) return (const HA_AS_LDS float*)p;
    else return p;
}
template <bool T = true>
HD auto glb_f(const float* p) {
    if constexpr (T) return (const HA_AS_GLB float*)p;
    else return p;
}
template <typename Q>
HD void ct_fill(Q* q, f3 x, f3 n, float sep, int a, int b) {
    // eight dword stores: the two 16-bit body codes go as one packed word
    q[0] = x.x; q[1] = x.y; q[2] = x.z; q[3] = n.x; q[4] = n.y; q[5] = n.z; q[6] = sep;
    q[7] = __int_as_float((a & 0xFFFF) | (b << 16));
}
HD void ct_put(const SimCtx& c, int ci, f3 x, f3 n, float sep, int a, int b) {
    if (ct_global(c, ci)) ct_fill((HA_AS_GLB float*)(c.kg + (ci - c.kc0)), x, n, sep, a, b);
    else ct_fill((HA_AS_LDS float*)(c.k + ci), x, n, sep, a, b);
}

// friction of a contact body (link 100+L, object o, static -1) and of a contact (PhysX average combine)
HD float body_friction(const SimCtx& c, int b) {
    if (!c.dr || b < 0) return c.p->friction;
    return b >= 100 ? c.dr[HA_DR_LINK_FRIC + (b - 100)] : c.dr[HA_DR_OBJ_FRIC + b];
}
HD float contact_friction(const SimCtx& c, int a, int b) { return 0.5f * (body_friction(c, a) + body_friction(c, b)); }

// 64-lane sum: DPP butterfly inside each 16-lane row (xor1, xor2, half-mirror, mirror), then the four
// row sums via v_readlane. Every lane gets the same bits; the oracle emulates this exact tree.
HD float wave_sum_rows(float x) {
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true));  // row_half_mirror
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, true));  // row_mirror
    return rows_sum(x);     // (r3 + r2) + (r1 + r0) == (r0 + r1) + (r2 + r3) bitwise
}

// Diagnostic phase timers (built only into libhandarm_hip_prof.so, -DHA_PROFILE): lane 0 of every
// wave adds the s_memtime delta of each phase; read back with ha_profile_read().
#ifdef HA_PROFILE
// [32 + 8 kind + phase]: the hull-hull split per pair kind; a second set of 96 for the substeps whose narrow phases
// offered more than HA_PROFILE_HEAVY contacts (the previous substep's class for the phases before detect)
__device__ unsigned long long g_prof[2 * 96];
#ifndef HA_PROFILE_HEAVY
#define HA_PROFILE_HEAVY 24
#endif
#define PROF_BEGIN() unsigned long long _pt = __builtin_amdgcn_s_memtime();
#define PROF_COUNT(i, v)                                               \
    do {                                                               \
        if (c.lane == 0) atomicAdd(&g_prof[(i) + 96 * c.pcls], (unsigned long long)(v)); \
    } while (0)
#define PROF(i)                                                        \
    do {                                                               \
        wsync();                                                       \
        unsigned long long _n = __builtin_amdgcn_s_memtime();          \
        if (c.lane == 0) atomicAdd(&g_prof[(i) + 96 * c.pcls], _n - _pt); \
        _pt = _n;                                                      \
    } while (0)
#else
#define PROF_BEGIN()
#define PROF(i)
#define PROF_COUNT(i, v)
#endif

// three independent wave_sum_rows, interleaved step by step so the DPP read-after-write wait states of
// one chain are filled by the others (same reduction tree per value)
HD void wave_sum_rows3(float& a, float& b, float& c) {
    a += dpp_f<0xB1>(a); b += dpp_f<0xB1>(b); c += dpp_f<0xB1>(c);
    a += dpp_f<0x4E>(a); b += dpp_f<0x4E>(b); c += dpp_f<0x4E>(c);
    a += dpp_f<0x141>(a); b += dpp_f<0x141>(b); c += dpp_f<0x141>(c);
    a += dpp_f<0x140>(a); b += dpp_f<0x140>(b); c += dpp_f<0x140>(c);
    a = a + dpp_row_f<0x142, 0xA>(0.0f, a); b = b + dpp_row_f<0x142, 0xA>(0.0f, b); c = c + dpp_row_f<0x142, 0xA>(0.0f, c);
    a = a + dpp_row_f<0x143, 0xC>(0.0f, a); b = b + dpp_row_f<0x143, 0xC>(0.0f, b); c = c + dpp_row_f<0x143, 0xC>(0.0f, c);
    a = lane63(a); b = lane63(b); c = lane63(c);
}
// three 16-lane row sums (the first four steps of wave_sum_rows3): every lane of a row gets its row's
// ((x0+x1)+(x2+x3)) + ((x4+x5)+(x6+x7)) ... = (Q0+Q1)+(Q2+Q3), the oracle's row_dot16
HD void row_sum3(float& a, float& b, float& c) {
    a += dpp_f<0xB1>(a); b += dpp_f<0xB1>(b); c += dpp_f<0xB1>(c);
    a += dpp_f<0x4E>(a); b += dpp_f<0x4E>(b); c += dpp_f<0x4E>(c);
    a += dpp_f<0x141>(a); b += dpp_f<0x141>(b); c += dpp_f<0x141>(c);
    a += dpp_f<0x140>(a); b += dpp_f<0x140>(b); c += dpp_f<0x140>(c);
}

// ----------------------------------------------------------------------------- kinematics
HD void fk(SimCtx& c) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane;
    // lane i owns link i: its model constants and its joint rotation (one sincos per lane) are loaded and
    // computed before the level chain, so each level only waits on its parent's LDS pose
    bool own = lane < c.L;
    int lev = -1, par = 0, d = -1;
    f3 op = mk3(0, 0, 0), ax = mk3(0, 0, 0);
    qf oq = qf{0, 0, 0, 1}, qa = qf{0, 0, 0, 1};
    if (own) {
        lev = m.link_level[lane];
        par = m.link_parent[lane];
        d = m.link_dof[lane];
        op = ld3(m.link_origin_pos[lane]);
        oq = ldq(m.link_origin_quat[lane]);
        if (d >= 0) {
            ax = ld3(m.link_axis[lane]);
            qa = qaxis(ax, s.q[d]);
        }
    }
    if (lane == 0) {
        st3(s.lp[0], ld3(m.base_pos));
        stq(s.lq[0], ldq(m.base_quat));
    }
    wsync();
    for (int l = 1; l <= m.max_level; l++) {
        if (lev == l) {
            qf pq = ldq(s.lq[par]);
            f3 p = ld3(s.lp[par]) + qrot(pq, op);
            qf r = qmul(pq, oq);
            if (d >= 0) {
                r = qmul(r, qa);
                st3(s.ax[d], qrot(r, ax));
                st3(s.an[d], p);
            }
            st3(s.lp[lane], p);
            stq(s.lq[lane], r);
        }
        wsync();
    }
}

struct SInert { float m; f3 h; float J[9]; };

HD void inert_apply(const SInert& I, f3 w, f3 v, f3& n, f3& f) {
    n = mv3(I.J, w) + cross3(I.h, v);
    f = v * I.m - cross3(I.h, w);
}
HD void inert_apply_lds(const float* Ic, f3 w, f3 v, f3& n, f3& f) {
    f3 h = mk3(Ic[1], Ic[2], Ic[3]);
    n = mv3(Ic + 4, w) + cross3(h, v);
    f = v * Ic[0] - cross3(h, w);
}

// joint-space inertia s.M (D x D) and velocity-product forces s.Cb
HD void dynamics(SimCtx& c) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, D = c.D, L = c.L;
    SInert I;
    bool own = lane < L;
    if (own) {
        int i = lane;
        float R[9], Iw[9];
        qf lq = ldq(s.lq[i]);
        qmat(lq, R);
        f3 cc = ld3(s.lp[i]) + qrot(lq, ld3(m.link_com[i]));
        rart3(R, m.link_inertia[i], Iw);
        float sc = c.dr ? c.dr[HA_DR_LINK_MASS + i] : 1.0f;     // DR: mass and inertia scale together
#pragma unroll
        for (int k = 0; k < 9; k++) Iw[k] = Iw[k] * sc;
        float mm = m.link_mass[i] * sc;
        I.m = mm;
        I.h = cc * mm;
        float ccd = dot3(cc, cc);
        float cv[3] = {cc.x, cc.y, cc.z};
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) I.J[a * 3 + b] = Iw[a * 3 + b] + mm * ((a == b ? ccd : 0.0f) - cv[a] * cv[b]);
        float* ic = s.u.pd.dyn.Ic[i];
        ic[0] = I.m; ic[1] = I.h.x; ic[2] = I.h.y; ic[3] = I.h.z;
#pragma unroll
        for (int k = 0; k < 9; k++) ic[4 + k] = I.J[k];
        if (i == 0) {
#pragma unroll
            for (int k = 0; k < 6; k++) { s.u.pd.Vl[0][k] = 0.f; s.u.pd.dyn.Al[0][k] = 0.f; }
        }
    }
    // zero M
    for (int k = lane; k < D * D; k += 64) s.u.pd.M[k] = 0.0f;
    wsync();
    // twists / bias accelerations, level by level (per-lane link constants and joint axis read once)
    int my_lev = own ? m.link_level[lane] : -1;
    int my_par = own ? m.link_parent[lane] : 0;
    int my_d = own ? m.link_dof[lane] : -1;
    f3 my_sw = mk3(0, 0, 0), my_sv = mk3(0, 0, 0);
    if (my_d >= 0) {
        f3 axd = ld3(s.ax[my_d]), and_ = ld3(s.an[my_d]);
        float qd = s.qd[my_d];
        my_sw = axd * qd;
        my_sv = cross3(and_, axd) * qd;
    }
    for (int lev = 1; lev <= m.max_level; lev++) {
        if (my_lev == lev) {
            int i = lane, par = my_par, d = my_d;
            f3 vw = ld3(&s.u.pd.Vl[par][0]), vv = ld3(&s.u.pd.Vl[par][3]);
            f3 aw = ld3(&s.u.pd.dyn.Al[par][0]), av = ld3(&s.u.pd.dyn.Al[par][3]);
            if (d >= 0) {
                f3 sw = my_sw, sv = my_sv;
                vw = vw + sw;
                vv = vv + sv;
                aw = aw + cross3(vw, sw);
                av = av + (cross3(vw, sv) + cross3(vv, sw));
            }
            st3(&s.u.pd.Vl[i][0], vw); st3(&s.u.pd.Vl[i][3], vv);
            st3(&s.u.pd.dyn.Al[i][0], aw); st3(&s.u.pd.dyn.Al[i][3], av);
        }
        wsync();
    }
    if (own) {
        int i = lane;
        f3 vw = ld3(&s.u.pd.Vl[i][0]), vv = ld3(&s.u.pd.Vl[i][3]);
        f3 aw = ld3(&s.u.pd.dyn.Al[i][0]), av = ld3(&s.u.pd.dyn.Al[i][3]);
        f3 n1, f1, n2, f2;
        inert_apply(I, aw, av, n1, f1);
        inert_apply(I, vw, vv, n2, f2);
        f3 fn = n1 + (cross3(vw, n2) + cross3(vv, f2));
        f3 ff = f1 + cross3(vw, f2);
        // link damping (ha_params_t v10): the wrench cl m v_com, ca I_com w (moment about the world origin) with the
        // momentum (n2, f2) = (I_com w + c x m v_com, m v_com): g = c x m v_com = h x f2 / m
        float cl = c.p->link_lin_damping, ca = c.p->link_ang_damping;
        if (cl != 0.0f || ca != 0.0f) {
            f3 g = I.m > 0.0f ? cross3(I.h, f2) * (1.0f / I.m) : mk3(0, 0, 0);
            fn = fn + ((n2 - g) * ca + g * cl);
            ff = ff + f2 * cl;
        }
        st3(&s.u.pd.dyn.Fl[i][0], fn); st3(&s.u.pd.dyn.Fl[i][3], ff);
    }
    wsync();
    // backward accumulation of forces and composite inertia, deepest level first. Each parent lane gathers
    // its children itself, highest link index first: the oracle's order (it visits links L-1 .. 0 and adds
    // each into its parent), so the float sums round identically. (LDS float atomics from the children
    // would add in whatever order the hardware serialises them.)
    uint32_t chm = 0;                           // this lane's child links (HA_MAX_LINKS = 32)
    for (int j = 1; j < L; j++) chm |= (m.link_parent[j] == lane) ? (1u << j) : 0u;
    for (int lev = m.max_level - 1; lev >= 0; lev--) {
        if (my_lev == lev && chm) {
            float* F = s.u.pd.dyn.Fl[lane];
            float* C = s.u.pd.dyn.Ic[lane];
            float f[6], ic[13];
#pragma unroll
            for (int k = 0; k < 6; k++) f[k] = F[k];
#pragma unroll
            for (int k = 0; k < 13; k++) ic[k] = C[k];
            for (uint32_t mm = chm; mm;) {
                int j = 31 - __clz(mm);
                mm &= ~(1u << j);
#pragma unroll
                for (int k = 0; k < 6; k++) f[k] = f[k] + s.u.pd.dyn.Fl[j][k];
#pragma unroll
                for (int k = 0; k < 13; k++) ic[k] = ic[k] + s.u.pd.dyn.Ic[j][k];
            }
#pragma unroll
            for (int k = 0; k < 6; k++) F[k] = f[k];
#pragma unroll
            for (int k = 0; k < 13; k++) C[k] = ic[k];
        }
        wsync();
    }
    if (lane < D) {
        int i = m.dof_link[lane];
        f3 axd = ld3(s.ax[lane]), and_ = ld3(s.an[lane]);
        s.Cb[lane] = dot3(axd, ld3(&s.u.pd.dyn.Fl[i][0])) + dot3(cross3(and_, axd), ld3(&s.u.pd.dyn.Fl[i][3]));
    }
    for (int k = lane; k < m.n_mpairs; k += 64) {
        int d = m.mpair[k][0], e = m.mpair[k][1];
        int i = m.dof_link[d];
        f3 axd = ld3(s.ax[d]), and_ = ld3(s.an[d]);
        f3 n, f;
        inert_apply_lds(s.u.pd.dyn.Ic[i], axd, cross3(and_, axd), n, f);
        f3 axe = ld3(s.ax[e]), ane = ld3(s.an[e]);
        float val = dot3(axe, n) + dot3(cross3(ane, axe), f);
        if (d == e) val += m.dof_armature[d];
        s.u.pd.M[d * D + e] = val;
        s.u.pd.M[e * D + d] = val;
    }
    wsync();
}


// M^-1 from M in registers, no LDS round trips or barriers (ND = compile-time DOF count):
//   1. Cholesky M = L L^T, left-looking, lane i holds row i of L (row j of L via v_readlane);
//   2. lane j builds column j of L^-1 by forward substitution;
//   3. lane j back-substitutes L^T x = (L^-1 e_j) -> x = column j of M^-1.
// Stored as S[j][i] = x_j[i] (row j of S = column j of M^-1; S is M^-1 up to rounding, not forced
// symmetric). Every use below reads S the same way the oracle does.
template <int ND>
HD void factor_inverse(SimCtx& c) {
    EnvLDS& s = *c.s;
    const int lane = c.lane;
    const float* Mm = s.u.pd.M;
    float a[ND];
#pragma unroll
    for (int k = 0; k < ND; k++) a[k] = (lane < ND && k <= lane) ? Mm[lane * ND + k] : 0.0f;
#pragma unroll
    for (int j = 0; j < ND; j++) {
        float t = a[j];
#pragma unroll
        for (int k = 0; k < j; k++) t = fmaf(-a[k], bcast(a[k], j), t);
        float ljj = sqrtf(fmaxf(bcast(t, j), 1e-30f));
        a[j] = lane == j ? ljj : (lane > j ? t / ljj : a[j]);
    }
    float rl[ND];
#pragma unroll
    for (int i = 0; i < ND; i++) rl[i] = 1.0f / bcast(a[i], i);
    float y[ND];
#pragma unroll
    for (int i = 0; i < ND; i++) {
        float t = 0.0f;
#pragma unroll
        for (int k = 0; k < i; k++) {
            float lik = bcast(a[k], i);
            t = k >= lane ? fmaf(lik, y[k], t) : t;
        }
        y[i] = i == lane ? rl[i] : (i > lane ? -t * rl[i] : 0.0f);
    }
    float x[ND];
#pragma unroll
    for (int i = ND - 1; i >= 0; i--) {
        float t = y[i];
#pragma unroll
        for (int k = i + 1; k < ND; k++) t = fmaf(-bcast(a[i], k), x[k], t);
        x[i] = t * rl[i];
    }
    if (lane < ND) {
#pragma unroll
        for (int i = 0; i < ND; i++) c.Minv[lane * ND + i] = x[i];
    }
    wsync();
}

struct PoseF { f3 p; qf q; };

// Per-env object dimensions (AllegroKuka's cuboid family): the pool hull of object o is scaled by
// diag(osc[o]) in its body frame. Unscaled bodies (links, static geometry, objects without a scale) take
// the unscaled expressions, bit for bit.
HD bool body_scaled(const SimCtx& c, int b) { return b >= 0 && b < c.NO && c.o[b].osc[3] != 0.0f; }
HD f3 scale3(const SimCtx& c, int b, f3 v) {
    if (!body_scaled(c, b)) return v;
    const float* sc = c.o[b].osc;
    return mk3(v.x * sc[0], v.y * sc[1], v.z * sc[2]);
}
HD float scale_radius(const SimCtx& c, int b, float r) {
    if (!body_scaled(c, b)) return r;
    const float* sc = c.o[b].osc;
    return r * fmaxf(fmaxf(sc[0], sc[1]), sc[2]);
}

HD PoseF object_pose(const SimCtx& c, int o) {
    const EnvLDS& s = *c.s;
    qf q = ldq(c.o[o].oq);
    return PoseF{ld3(c.o[o].oc) - qrot(q, scale3(c, o, ld3(c.m->pool_com[c.o[o].pool]))), q};
}
// object o's pool id when o is wave-uniform (narrow phase): in an SGPR, so the model reads it indexes are scalar
HD int upool(const SimCtx& c, int o) { return __builtin_amdgcn_readfirstlane(c.o[o].pool); }
HD PoseF object_pose_u(const SimCtx& c, int o) {
    qf q = ldq(c.o[o].oq);
    return PoseF{ld3(c.o[o].oc) - qrot(q, scale3(c, o, ld3(c.m->pool_com[upool(c, o)]))), q};
}

// face plane k of a hull in world space; for a scaled body (inv_sc = 1 / scale, read once per hull pair by
// the caller) n' = S^-1 n / |S^-1 n|, d' = d / |S^-1 n|
HD void world_plane(const ha_model_t& m, int hull, int k, PoseF P, bool scaled, f3 inv_sc, f3& n, float& d) {
    const float* pl = m.planes[m.hull_plane_start[hull] + k];
    f3 nl = mk3(pl[0], pl[1], pl[2]);
    float dl = pl[3];
    if (scaled) {
        nl = mk3(pl[0] * inv_sc.x, pl[1] * inv_sc.y, pl[2] * inv_sc.z);
        float inv = 1.0f / sqrtf(dot3(nl, nl));
        nl = nl * inv;
        dl = dl * inv;
    }
    n = qrot(P.q, nl);
    d = dl - dot3(n, P.p);
}
HD f3 inv_scale(const SimCtx& c, int b) {
    if (!body_scaled(c, b)) return mk3(1, 1, 1);
    const float* sc = c.o[b].osc;
    return mk3(1.0f / sc[0], 1.0f / sc[1], 1.0f / sc[2]);
}

HD void store_chosen(SimCtx& c, int k, const f3* P, const f3* N, const float* S, const int* CD, int a, int b);
// A manifold point's anchor for its persistent record (v13; the oracle's PCM_*): the feature it came from - a vertex or
// clipped edge point of side A, of side B, or neither (the midpoint of two edges' closest points) - plus PCM_NORMAL_A
// when the normal is carried by side A (the reference face is A's; B for the ground and edge-edge contacts)
#define PCM_FEAT_A 0
#define PCM_FEAT_B 1
#define PCM_FEAT_MID 2
#define PCM_NORMAL_A 4
// the contacts a pair offers to the list (lane 0; contact_stats columns 3 and 4 via EnvLDS noff / cst)
HD void count_offered(SimCtx& c, int k, int a, int b) {
    EnvLDS& s = *c.s;
    if (c.lane == 0) {
        s.noff += k;
        if (a >= 100 && b >= 100) s.cst[4] += k;
    }
}

// append up to 4 reduced contacts (lane 0 does the list bookkeeping, same policy as the oracle). n is the
// lane's normal: one value over the wave for a convex pair; a compound object pair's gathered points keep
// their piece pair's normal, and the area criterion then measures about the deepest point's normal. While
// c.gather is set (a compound pair's piece pairs) the reduced points go to the gather buffer instead.
HD void emit_contacts(SimCtx& c, bool valid, f3 pt, float sep, f3 n, int a, int b, int code) {
    EnvLDS& s = *c.s;
    int lane = c.lane;
#ifdef HA_AB_TIMING
    if (c.dry) return;
#endif
    // the chosen lanes live in scalars, never in an indexed private array (which would go to scratch)
    float v0 = valid ? sep : 3.0e38f;
    int i0 = valid ? lane : 1 << 20;
    wave_argmin(v0, i0);
    if (i0 >= (1 << 20)) return;
    int k = 1, j1 = 0, j2 = 0, j3 = 0;        // chosen lanes of points 1..3 (valid below k)
    f3 p0 = mk3(bcast(pt.x, i0), bcast(pt.y, i0), bcast(pt.z, i0));
    // points 2-4 only among the candidates within manifold_window of the deepest one (ha_params_t v9)
    bool near = valid && sep <= v0 + c.p->manifold_window;
    f3 dd = pt - p0;
    float v1 = near ? dot3(dd, dd) : -1.0f;
    int i1 = lane;
    wave_argmax(v1, i1);
    if (v1 > 1e-12f) {
        j1 = i1;
        k = 2;
        f3 p1 = mk3(bcast(pt.x, i1), bcast(pt.y, i1), bcast(pt.z, i1));
        f3 e = p1 - p0;
        f3 n0 = mk3(bcast(n.x, i0), bcast(n.y, i0), bcast(n.z, i0));
        float sv = dot3(cross3(e, pt - p0), n0);
        float v2 = near ? sv : -3.0e38f;
        int i2 = lane;
        wave_argmax(v2, i2);
        float v3 = near ? sv : 3.0e38f;
        int i3 = lane;
        wave_argmin(v3, i3);
        bool h2 = v2 > 1e-12f, h3 = v3 < -1e-12f;
        j2 = h2 ? i2 : i3;
        j3 = i3;
        k = 2 + (h2 ? 1 : 0) + (h3 ? 1 : 0);
    }
#ifndef HA_EMIT_PARALLEL
#define HA_EMIT_PARALLEL 1
#endif
    // the chosen lanes' ranks: point t of the manifold (the oracle's idx order)
    int t = lane == i0 ? 0 : (k > 1 && lane == j1 ? 1 : (k > 2 && lane == j2 ? 2 : (k > 3 && lane == j3 ? 3 : -1)));
    if (c.pslot >= 0 && !c.gather) {
        // the pair's manifold for its persistent record (ha_params_t v13), staged in the clipping candidates' scratch
        // (free once the narrow phase has emitted; not part of the hull-side cache): point t = x, n, sep, anchor.
        // pcm_commit writes the record after the pair, at one call site instead of one per emit site
        float* q = reinterpret_cast<float*>(c.col.cand) + 8 * (t < 0 ? 0 : t);
        if (t >= 0) {
            q[0] = pt.x; q[1] = pt.y; q[2] = pt.z; q[3] = n.x; q[4] = n.y; q[5] = n.z; q[6] = sep;
            q[7] = __int_as_float(code);
        }
        c.pemit = k;
    }
    if (HA_EMIT_PARALLEL && !c.gather) {
        int nc0 = s.nc;
        if (nc0 + k <= c.maxc) {
            // room for all k points (the common case): each chosen lane writes its own point into slot nc + t,
            // the values lane 0 would write after broadcasting them (the chosen lanes are distinct)
            count_offered(c, k, a, b);
            if (lane == 0) s.nc = nc0 + k;
            if (t >= 0) ct_put(c, nc0 + t, pt, n, sep, a, b);
            wsync();
            return;
        }
    }
    // the chosen points to every lane
    f3 P[4], N[4];
    float S[4];
    int CD[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        int src = t == 0 ? i0 : (t < k ? (t == 1 ? j1 : (t == 2 ? j2 : j3)) : 0);
        P[t] = mk3(bcast(pt.x, src), bcast(pt.y, src), bcast(pt.z, src));
        N[t] = mk3(bcast(n.x, src), bcast(n.y, src), bcast(n.z, src));
        S[t] = bcast(sep, src);
        CD[t] = bcast_i(code, src);
    }
    store_chosen(c, k, P, N, S, CD, a, b);
}

// the k <= 4 chosen points of a manifold (wave-uniform P, N, S) into the gather buffer (a compound pair's piece
// pairs) or the contact list: lane 0 appends, or (list full) replaces the shallowest contact if the new one is deeper
HD void store_chosen(SimCtx& c, int k, const f3* P, const f3* N, const float* S, const int* CD, int a, int b) {
    EnvLDS& s = *c.s;
    int lane = c.lane;
    if (c.gather) {
        // compound pair: the chosen points (in the oracle's index order) join the gather buffer
        if (lane == 0) {
            const ColView& cs = c.col;
            int ng = s.ng;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if (t < k && ng < HA_MAX_GATHER) {
                    st3(cs.gp[ng], P[t]);
                    cs.gp[ng][3] = S[t];
                    st3(cs.gn[ng], N[t]);
                    cs.gn[ng][3] = __int_as_float(CD[t]);       // the point's persistent-record anchor
                    ng++;
                }
            }
            s.ng = ng;
        }
        wsync();
        return;
    }
    count_offered(c, k, a, b);
    // lane 0 appends, or (list full) replaces the shallowest contact if this one is deeper: the shallowest is the first
    // maximum of sep over the list (the oracle's sequential strict-compare scan), found by a wave arg-max over
    // lanes = contacts instead of a scan on lane 0 (clutter scenes run with the list full)
#pragma unroll
    for (int t = 0; t < 4; t++) {
        if (t >= k) break;
        int nc = s.nc, slot;
        if (nc >= c.maxc) {
            float sv = lane < c.maxc ? ct_sep(c, lane) : -3.0e38f;
            int w = lane;
            if (c.maxc > 64) {          // contacts 64.. in the same lanes; a tie keeps the lower index
                float s2 = lane + 64 < c.maxc ? ct_sep(c, lane + 64) : -3.0e38f;
                if (s2 > sv) { sv = s2; w = lane + 64; }
            }
            wave_argmax(sv, w);
            if (sv <= S[t]) continue;
            slot = w;
        } else {
            slot = nc;
        }
        if (lane == 0) {
            if (slot == nc) s.nc = nc + 1;
            ct_put(c, slot, P[t], N[t], S[t], a, b);
        }
        wsync();
    }
    wsync();
}

HD void collide_ground(SimCtx& c, int hull, PoseF P, int a) {
    const ha_model_t& m = *c.m;
    float mg = c.p->contact_margin;
    f3 ctr = P.p + qrot(P.q, scale3(c, a, ld3(m.hull_center[hull])));
    if (ctr.z - scale_radius(c, a, m.hull_radius[hull]) > mg) return;
    int lane = c.lane;
    bool valid = false;
    f3 pt = mk3(0, 0, 0);
    float sep = 0;
    if (lane < m.hull_nverts[hull]) {
        f3 v = P.p + qrot(P.q, scale3(c, a, ld3(m.verts[m.hull_vert_start[hull] + lane])));
        if (v.z <= mg) {
            valid = true;
            pt = v - mk3(0, 0, 0.5f * v.z);
            sep = v.z;
        }
    }
    emit_contacts(c, valid, pt, sep, mk3(0, 0, 1), a, -1, PCM_FEAT_A);
}

// float <-> int mapping that preserves order (for LDS atomicMax over floats)
HD int f2ord(float f) {
    int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
HD float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// SAT over the face planes wp[0..np) of one hull against the world vertices wv[0..nv) of the other:
// sep = max_k min_i (n_k . v_i + d_k), k = its argmax (ties -> smaller k). Every (k, i) value is the
// same expression as in the oracle; only the parallel order of the (exact) min/max differs.
HD void sat_planes(const SimCtx& c, const float (*wp)[4], int np, const float (*wv)[4], int nv, float& sep, int& kbest) {
    int lane = c.lane;
#ifdef HA_X_SAT_LANE_VERTEX   /* A/B: lane = vertex, one wave min per plane */
    if (np <= 8) {
        // few planes (boxes): lane = vertex, one wave min per plane. The eight plane slots are unrolled so their
        // independent DPP reduction chains interleave (slots k >= np read in-bounds scratch and are masked), then
        // the strict-compare scan over k keeps the oracle's first maximum
        f3 v = mk3(0, 0, 0);
        if (lane < nv) v = ld3(wv[lane]);
        float mn[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            f3 n = ld3(wp[k]);
            float d = wp[k][3];
            mn[k] = wave_min(lane < nv && k < np ? dot3(n, v) + d : 3.0e38f);
        }
        float best = -3.0e38f;
        int bk = 1 << 20;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k < np && mn[k] > best) { best = mn[k]; bk = k; }
        sep = best;
        kbest = bk;
        return;
    }
#else
    if (np <= 8) {
        // few planes (boxes): lane = (plane k = lane / 8, vertex group g = lane % 8). A lane takes the min over its
        // group's vertices g, g + 8, ..., then the plane's eight lanes combine (quad_perm xor1, xor2,
        // row_half_mirror: a min inside each 8-lane group), then one wave max over the planes; its first k is the
        // lowest lane holding it (the oracle's strict-compare scan keeps the first maximum). Every (k, i) value is
        // the oracle's expression and min / max are exact, so the order does not matter
        int k = lane >> 3, g = lane & 7;
        float m = 3.0e38f;
        if (k < np) {
            f3 n = ld3(wp[k]);
            float d = wp[k][3];
#pragma unroll 1
            for (int i = g; i < nv; i += 8) m = fminf(m, dot3(n, ld3(wv[i])) + d);
        }
        m = fminf(m, dpp_f<0xB1>(m));
        m = fminf(m, dpp_f<0x4E>(m));
        m = fminf(m, dpp_f<0x141>(m));
        float v = k < np ? m : -3.0e38f;
        float best = wave_max(v);
        uint64_t hit = __ballot(k < np && v == best);
        sep = best;
        kbest = (int)((__ffsll((unsigned long long)hit) - 1) >> 3);
        return;
    }
#endif
    // lane = plane (k = lane, lane + 64), loop over the vertices with batched LDS loads
    float best = -3.0e38f;
    int bk = 1 << 20;
    for (int k = lane; k < np; k += 64) {
        f3 n = ld3(wp[k]);
        float d = wp[k][3];
        float m0 = 3.0e38f, m1 = 3.0e38f;
        int i = 0;
        for (; i + 4 <= nv; i += 4) {
            float4 a = *reinterpret_cast<const float4*>(wv[i]);
            float4 b = *reinterpret_cast<const float4*>(wv[i + 1]);
            float4 e = *reinterpret_cast<const float4*>(wv[i + 2]);
            float4 f = *reinterpret_cast<const float4*>(wv[i + 3]);
            m0 = fminf(m0, dot3(n, mk3(a.x, a.y, a.z)) + d);
            m1 = fminf(m1, dot3(n, mk3(b.x, b.y, b.z)) + d);
            m0 = fminf(m0, dot3(n, mk3(e.x, e.y, e.z)) + d);
            m1 = fminf(m1, dot3(n, mk3(f.x, f.y, f.z)) + d);
        }
        for (; i < nv; i++) m0 = fminf(m0, dot3(n, ld3(wv[i])) + d);
        float mn = fminf(m0, m1);
        if (mn > best) { best = mn; bk = k; }
    }
    wave_argmax(best, bk);
    sep = best;
    kbest = bk;
}

// squared distance from point q to the segment p0 + t (p1 - p0), t in [0, 1] (the oracle's seg_point_d2)
HD float seg_point_d2(f3 p0, f3 p1, f3 q) {
    f3 d = p1 - p0;
    float dd = dot3(d, d);
    float t = dd > 0.0f ? dot3(q - p0, d) / dd : 0.0f;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
    f3 r = q - (p0 + d * t);
    return dot3(r, r);
}
// the edges of one hull (records E[0..ne), world vertices wv) within sqrt(r2) of the other hull's centre ctr, as a
// byte list of edge indices in edge order (an edge farther away cannot touch the other hull); returns the count
HD int edge_cull(const SimCtx& c, const uint32_t* E, int ne, const float (*wv)[4], f3 ctr, float r2, uint8_t* out) {
    int n = 0;
#pragma unroll 1
    for (int base = 0; base < ne; base += 64) {
        int i = base + c.lane;
        bool keep = false;
        if (i < ne) {
            uint32_t e = E[i];
            keep = seg_point_d2(ld3(wv[e & 255u]), ld3(wv[(e >> 8) & 255u]), ctr) <= r2;
        }
        uint64_t mk = __ballot(keep);
        if (keep) out[n + __popcll(mk & ((1ull << c.lane) - 1ull))] = (uint8_t)i;
        n += __popcll(mk);
    }
    return n;
}
// Edge pair (ea of hull A, eb of hull B; edge records v0 | v1 << 8 | f0 << 16 | f1 << 24) of the edge-edge SAT
// (Gregorius, GDC 2013): when the Gauss-map arcs of the two edges (between their faces' normals; B's negated)
// cross, the pair is a face of the Minkowski difference and N = e1 x e2, oriented away from B's centre cb, is a
// separating-axis candidate with separation N . (pA - pB). Returns -3e38 for any other pair (arcs apart, or edges
// within 0.3 degrees of parallel). n, pa / e1, pb / e2: the axis and the edges (start, direction).
HD float edge_axis(const ColView& cs, uint32_t ea, uint32_t eb, f3 cb, f3& n, f3& pa, f3& e1, f3& pb, f3& e2) {
    // the outputs are set on every path (the caller reads them after the winning pair's call)
    pa = ld3(cs.wvA[ea & 255u]);
    e1 = ld3(cs.wvA[(ea >> 8) & 255u]) - pa;
    pb = ld3(cs.wvB[eb & 255u]);
    e2 = ld3(cs.wvB[(eb >> 8) & 255u]) - pb;
    n = cross3(e1, e2);
    f3 a = ld3(cs.wpA[(ea >> 16) & 255u]), b = ld3(cs.wpA[ea >> 24]);
    f3 cc = ld3(cs.wpB[(eb >> 16) & 255u]) * -1.0f, dd = ld3(cs.wpB[eb >> 24]) * -1.0f;
    f3 bxa = cross3(b, a), dxc = cross3(dd, cc);
    float cba = dot3(cc, bxa), dba = dot3(dd, bxa), adc = dot3(a, dxc), bdc = dot3(b, dxc);
    if (!(cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f)) return -3.0e38f;
    float l2 = dot3(n, n);
    if (l2 < 2.5e-5f * (dot3(e1, e1) * dot3(e2, e2))) return -3.0e38f;
    n = n * (1.0f / sqrtf(l2));
    if (dot3(n, pb - cb) < 0.0f) n = n * -1.0f;
    return dot3(n, pa - pb);
}
// midpoint of the closest points of the segments pa + s e1 and pb + t e2 (s, t in [0, 1]; not parallel)
HD f3 edge_closest_mid(f3 pa, f3 e1, f3 pb, f3 e2) {
    f3 r = pa - pb;
    float aa = dot3(e1, e1), ee = dot3(e2, e2), bb = dot3(e1, e2), cc = dot3(e1, r), ff = dot3(e2, r);
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
    return ((pa + e1 * sa) + (pb + e2 * tb)) * 0.5f;
}

// hull A (body a) vs hull B (body b); normal from B to A. keyA / keyB identify the posed hull of each side for
// the ColScratch cache (the body code, or -100 - k for static body k: statics may share a hull)
HD void collide_hulls(SimCtx& c, int ha, PoseF PA, int hb, PoseF PB, int a, int b, int keyA, int keyB) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    float mg = c.p->contact_margin;
    int lane = c.lane;
    f3 ca = PA.p + qrot(PA.q, scale3(c, a, ld3(m.hull_center[ha])));
    f3 cb = PB.p + qrot(PB.q, scale3(c, b, ld3(m.hull_center[hb])));
    f3 dc = ca - cb;
    float rr = scale_radius(c, a, m.hull_radius[ha]) + scale_radius(c, b, m.hull_radius[hb]) + mg;
    c.sepf = 0xFF;
    if (dot3(dc, dc) > rr * rr) return;
    int nva = m.hull_nverts[ha], nvb = m.hull_nverts[hb];
    int npa = m.hull_nplanes[ha], npb = m.hull_nplanes[hb];
    const ColView& cs = c.col;
#ifdef HA_PROFILE
    unsigned long long _h0 = __builtin_amdgcn_s_memtime();
#define HPROF(i) do { wsync(); unsigned long long _h1 = __builtin_amdgcn_s_memtime(); PROF_COUNT(i, _h1 - _h0); \
                          PROF_COUNT(32 + 8 * c.pk + (i) - 25, _h1 - _h0); _h0 = _h1; } while (0)
#else
#define HPROF(i)
#endif
    // world vertices and planes of both hulls, unless this side's (hull, body) is already in ColScratch
    bool needA = ha != c.colA_h || keyA != c.colA_b, needB = hb != c.colB_h || keyB != c.colB_b;
    if (needB) {
        if (lane < nvb) st3(cs.wvB[lane], PB.p + qrot(PB.q, scale3(c, b, ld3(m.verts[m.hull_vert_start[hb] + lane]))));
        bool scB = body_scaled(c, b);
        f3 isB = inv_scale(c, b);
        for (int k = lane; k < npb; k += 64) {
            f3 n; float d;
#ifdef HA_X_PLANE_INLOOP    /* diagnostic: the inverse scale read inside the plane loop */
            isB = inv_scale(c, b);
#endif
            world_plane(m, hb, k, PB, scB, isB, n, d);
            st3(cs.wpB[k], n);
            cs.wpB[k][3] = d;
        }
        c.colB_h = hb; c.colB_b = keyB;
        wsync();
    }
    // side A's bounding sphere against B's face planes before A's setup: a plane the sphere clears by more than
    // the margin (with a 1 mm allowance for rounding) clears every vertex of A too, so SAT over B's planes would
    // separate the pair; such a pair (most link hulls near an object) skips A's setup and the SAT. No result
    // changes: the oracle runs the full test and finds the same separation
    if (c.p->narrow_phase_flags & HA_NP_NO_SPHERE_CULL) {
    } else {
        float sc = -3.0e38f;
        int kc = 1 << 20;
        for (int k = lane; k < npb; k += 64) {
            float v = dot3(ld3(cs.wpB[k]), ca) + cs.wpB[k][3];
            if (v > sc) { sc = v; kc = k; }
        }
        float scm = wave_max(sc);
        if (scm - scale_radius(c, a, m.hull_radius[ha]) > mg + 1e-3f) {
            if (c.selfc || c.pairf) {       // B's face k separates A: the hint the pair's next detection checks first
                wave_argmax(sc, kc);
                c.sepf = 0x80 | kc;
            }
            return;
        }
    }
    if (needA) {
        if (lane < nva) st3(cs.wvA[lane], PA.p + qrot(PA.q, scale3(c, a, ld3(m.verts[m.hull_vert_start[ha] + lane]))));
        c.colA_h = ha; c.colA_b = keyA; c.colA_p = false;
        wsync();
    }
    HPROF(25);
    // B's face planes against A's vertices first: side A's planes (a link hull's up to 60) are only built when
    // that test does not separate the pair. Either test alone separating means no contact, so the order changes
    // no result
    float sepA, sepB;
    int kA, kB;
    sat_planes(c, cs.wpB, npb, cs.wvA, nva, sepB, kB);
    HPROF(27);
    if (sepB > mg) {
        c.sepf = 0x80 | kB;
        return;
    }
    if (!c.colA_p) {
        bool scA = body_scaled(c, a);
        f3 isA = inv_scale(c, a);
        for (int k = lane; k < npa; k += 64) {
            f3 n; float d;
#ifdef HA_X_PLANE_INLOOP
            isA = inv_scale(c, a);
#endif
            world_plane(m, ha, k, PA, scA, isA, n, d);
            st3(cs.wpA[k], n);
            cs.wpA[k][3] = d;
        }
        c.colA_p = true;
        wsync();
    }
    HPROF(25);
    sat_planes(c, cs.wpA, npa, cs.wvB, nvb, sepA, kA);
    HPROF(26);
    if (sepA > mg) {
        c.sepf = kA;
        return;
    }
    // ---- edge-edge axes (v10): a hull pair whose face axes leave it within the margin may still be separated along,
    //      or touch through, a pair of edges
    int nea = m.hull_nedges[ha], neb = m.hull_nedges[hb];
    if (c.p->narrow_phase_flags & HA_NP_NO_EDGE_AXES) nea = 0;
    if (nea > 0 && neb > 0) {
        float smax = fmaxf(sepA, sepB);
        float pen = smax < 0.0f ? -smax : 0.0f;
        float RA = (scale_radius(c, a, m.hull_radius[ha]) + mg) + pen;
        float RB = (scale_radius(c, b, m.hull_radius[hb]) + mg) + pen;
        uint8_t* la = reinterpret_cast<uint8_t*>(cs.cand);
        uint8_t* lb = reinterpret_cast<uint8_t*>(cs.cmax);
        const uint32_t* EA = m.edges + m.hull_edge_start[ha];
        const uint32_t* EB = m.edges + m.hull_edge_start[hb];
        // side B first (the static box, or the object of a link pair): its list is empty for most pairs (a table's
        // edges are far from an object resting on its face), and then no pair exists and side A's cull is skipped
        int nB = edge_cull(c, EB, neb, cs.wvB, ca, RA * RA, lb);
        int nA = nB > 0 ? edge_cull(c, EA, nea, cs.wvA, cb, RB * RB, la) : 0;
        wsync();
        float best = -3.0e38f;
        int bw = 1 << 30;
        // pairs (i, j) of the two lists, w = i nB + j: the lanes take the elements of the longer list (64 at a time)
        // and loop over the shorter one, whose element is wave-uniform per iteration. Per-edge terms (start,
        // direction, face normals, the Gauss-arc normal, the B edge's offset from cb) are formed once per element,
        // by the same expressions edge_axis evaluates per pair; the winner (max, then lowest w) is the oracle's
        // i-major scan
        if (nA > 0 && nB > 0) {
            bool aLong = nA >= nB;
            int nL = aLong ? nA : nB, nS = aLong ? nB : nA;
            const uint8_t* lL = aLong ? la : lb;
            const uint8_t* lS = aLong ? lb : la;
            const uint32_t* EL = aLong ? EA : EB;
            const uint32_t* ES = aLong ? EB : EA;
            const float (*wvL)[4] = aLong ? cs.wvA : cs.wvB;
            const float (*wvS)[4] = aLong ? cs.wvB : cs.wvA;
            const float (*wpL)[4] = aLong ? cs.wpA : cs.wpB;
            const float (*wpS)[4] = aLong ? cs.wpB : cs.wpA;
            // the short list's records, element t in lane t (t < 64)
            uint32_t recS = lane < nS ? ES[lS[lane]] : 0u;
#pragma unroll 1
            for (int base = 0; base < nL; base += 64) {
                int li = base + lane;
                bool act = li < nL;
                uint32_t rl = act ? EL[lL[li]] : EL[lL[0]];
                // this lane's edge: A side (pa, e1, a, b, bxa) or B side (pb, e2, -f0, -f1, dxc, pb - cb)
                f3 lp = ld3(wvL[rl & 255u]);
                f3 le = ld3(wvL[(rl >> 8) & 255u]) - lp;
                f3 lf0 = ld3(wpL[(rl >> 16) & 255u]), lf1 = ld3(wpL[rl >> 24]);
                if (!aLong) { lf0 = lf0 * -1.0f; lf1 = lf1 * -1.0f; }
                f3 lx = cross3(lf1, lf0);
                f3 lo = lp - cb;
                // two passes per 64 short-list edges: (1) the Gauss-map test of this lane's edge against each of them
                // (wave-uniform short edge, its face normals broadcast from LDS) into a bit mask; (2) each lane walks
                // its own passing pairs in increasing order and evaluates their axes. The same pairs, values and
                // first-max-wins order as one loop evaluating every pair, but the axis arithmetic runs only on the
                // lanes whose pair passed instead of on the whole wave whenever any lane's did
#pragma unroll 1
                for (int sb = 0; sb < nS; sb += 64) {
                    int ns = nS - sb < 64 ? nS - sb : 64;
                    uint64_t pm = 0;
#pragma unroll 1
                    for (int t = 0; t < ns; t++) {
                        int si = sb + t;
                        uint32_t rs = si < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)recS, si)
                                              : ES[__builtin_amdgcn_readfirstlane(lS[si])];
                        f3 sf0 = ld3(wpS[(rs >> 16) & 255u]), sf1 = ld3(wpS[rs >> 24]);
                        if (aLong) { sf0 = sf0 * -1.0f; sf1 = sf1 * -1.0f; }
                        f3 sx = cross3(sf1, sf0);
                        // A: (a, b, bxa) = (f0, f1, f1 x f0); B: (c, d, dxc) = (-f0, -f1, (-f1) x (-f0))
                        f3 a = aLong ? lf0 : sf0, b = aLong ? lf1 : sf1, bxa = aLong ? lx : sx;
                        f3 cc = aLong ? sf0 : lf0, dd = aLong ? sf1 : lf1, dxc = aLong ? sx : lx;
                        float cba = dot3(cc, bxa), dba = dot3(dd, bxa), adc = dot3(a, dxc), bdc = dot3(b, dxc);
                        bool pass = cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f;
                        pm |= (uint64_t)(pass ? 1u : 0u) << t;
                    }
                    if (!act) pm = 0;
#pragma unroll 1
                    while (__ballot(pm != 0) != 0ull) {
                        // (the short edge's record comes from its lane with every lane active: a lane permute whose
                        // source lane is inactive would not read its value)
                        int t = pm != 0 ? __ffsll((unsigned long long)pm) - 1 : 0;
                        int si = sb + t;
                        uint32_t rs = (uint32_t)__shfl((int)recS, t);
                        if (pm == 0) continue;
                        pm &= pm - 1;
                        if (sb > 0) rs = ES[lS[si]];
                        f3 sp = ld3(wvS[rs & 255u]);
                        f3 se = ld3(wvS[(rs >> 8) & 255u]) - sp;
                        f3 pa = aLong ? lp : sp, e1 = aLong ? le : se, pb = aLong ? sp : lp, e2 = aLong ? se : le;
                        f3 n = cross3(e1, e2);
                        float l2 = dot3(n, n);
                        if (l2 < 2.5e-5f * (dot3(e1, e1) * dot3(e2, e2))) continue;
                        n = n * (1.0f / sqrtf(l2));
                        f3 pbo = aLong ? sp - cb : lo;
                        if (dot3(n, pbo) < 0.0f) n = n * -1.0f;
                        float sv = dot3(n, pa - pb);
                        int w = aLong ? li * nB + si : si * nB + li;
                        if (sv > best) { best = sv; bw = w; }
                    }
                }
            }
        }
        if (nA > 0 && nB > 0) wave_argmax(best, bw);      // (no pair: best stays -3e38, no reduction needed)
        HPROF(30);
        if (best > mg) return;                              // separated along an edge-edge axis
        if (best > c.p->edge_rel_tol * smax + c.p->edge_abs_tol) {
            // edge contact: one point midway between the edges' closest points, normal the axis
            int bi = bw / nB;
            f3 n, pa, pb, e1, e2;
            edge_axis(cs, EA[la[bi]], EB[lb[bw - bi * nB]], cb, n, pa, e1, pb, e2);
            f3 x = edge_closest_mid(pa, e1, pb, e2);
            emit_contacts(c, lane == 0, x, best, n, a, b, PCM_FEAT_MID);
            return;
        }
        wsync();                                            // the edge lists (cand / cmax) are reused below
    }
    // ---- face contact: the reference face (the face axis of larger separation; the other if it yields nothing) and
    //      the incident hull, candidates (1) incident vertices near the reference face and inside its hull's other
    //      planes, (2) the incident face's edges clipped to the reference face's side planes, (3) the reference face's
    //      vertices over the incident face
    for (int pass = 0; pass < 2; pass++) {
        bool refB = (sepB >= sepA) ? (pass == 0) : (pass == 1);
        int kr = refB ? kB : kA;
        int hr = refB ? hb : ha, hi = refB ? ha : hb;
        int nvi = refB ? nva : nvb, npr = refB ? npb : npa, npi = refB ? npa : npb;
        const float (*wpr)[4] = refB ? cs.wpB : cs.wpA;
        const float (*wpi)[4] = refB ? cs.wpA : cs.wpB;
        const float (*wvi)[4] = refB ? cs.wvA : cs.wvB;
        const float (*wvr)[4] = refB ? cs.wvB : cs.wvA;
        f3 nref = ld3(wpr[kr]);
        float dref = wpr[kr][3];
        // (1) incident vertices within the margin of the reference face
        f3 vi = mk3(0, 0, 0);
        float dist = 0;
        bool cand = false;
        if (lane < nvi) {
            vi = ld3(wvi[lane]);
            dist = dot3(nref, vi) + dref;
            cand = dist <= mg;
        }
        uint64_t cm = __ballot(cand);
        int ncand = __popcll(cm);
        int slot = __popcll(cm & ((1ull << lane) - 1ull));
        if (cand) {
            cs.cand[slot] = lane;
            cs.cmax[slot] = f2ord(-3.0e38f);
        }
        wsync();
        // side planes of the reference face: max distance per candidate over (candidate, plane) pairs
        // spread across the lanes (exact max -> order-independent)
        int total = ncand * npr;
        int j = lane / npr, k = lane - j * npr;
        int step_j = 64 / npr, step_k = 64 - step_j * npr;
        for (int w = lane; w < total; w += 64) {
            if (k != kr) {
                f3 v = ld3(wvi[cs.cand[j]]);
                float val = dot3(ld3(wpr[k]), v) + wpr[k][3];
                atomicMax(&cs.cmax[j], f2ord(val));
            }
            j += step_j;
            k += step_k;
            if (k >= npr) { k -= npr; j++; }
        }
        wsync();
        HPROF(28);
        bool valid = cand && ord2f(cs.cmax[slot]) <= mg;
        // the candidate set, one per lane in the oracle's list order: lanes [0, nv1) the valid incident vertices
        // in vertex order (moved there by a forward permute), then, from lane nv1 on, the incident-face edges'
        // entry / exit points and the reference-face vertices (lanes past 63 dropped, as by the oracle)
        uint64_t vm = __ballot(valid);
        int nv1 = __popcll(vm);
        int rk = __popcll(vm & ((1ull << lane) - 1ull));
        int to = valid ? rk : nv1 + (lane - rk);        // a permutation of the lanes
        f3 pt = vi - nref * (0.5f * dist);
        f3 x = mk3(__int_as_float(__builtin_amdgcn_ds_permute(to << 2, __float_as_int(pt.x))),
                   __int_as_float(__builtin_amdgcn_ds_permute(to << 2, __float_as_int(pt.y))),
                   __int_as_float(__builtin_amdgcn_ds_permute(to << 2, __float_as_int(pt.z))));
        float sv = __int_as_float(__builtin_amdgcn_ds_permute(to << 2, __float_as_int(dist)));
        bool ok = lane < nv1;
        // the incident face: the incident hull's face most anti-parallel to the reference normal (first minimum)
        float vmin = 3.0e38f;
        int ki = 1 << 20;
        for (int kk = lane; kk < npi; kk += 64) {
            float dv = dot3(ld3(wpi[kk]), nref);
            if (dv < vmin) { vmin = dv; ki = kk; }
        }
        wave_argmin(vmin, ki);
        int lpi = m.plane_loop[m.hull_plane_start[hi] + ki], lpr = m.plane_loop[m.hull_plane_start[hr] + kr];
        int li0 = lpi & 0xFFFF, lni = lpi >> 16, lr0 = lpr & 0xFFFF, lnr = lpr >> 16;
        if (c.p->narrow_phase_flags & HA_NP_NO_CLIP) lni = lnr = 0;
        f3 ni = ld3(wpi[ki]);
        float di = wpi[ki][3];
        float den = dot3(ni, nref);
        // the two face loops staged in lanes: lane j holds loop vertex j of each face and the side plane through
        // loop edge j (side_plane, the same expression for every (candidate, plane) pair), so the clipping loops
        // below read them with v_readlane instead of re-deriving them per candidate from the model's loop lists
        int rv = lane < lnr ? m.loop_v[lr0 + lane] : 0, iv = lane < lni ? m.loop_v[li0 + lane] : 0;
        f3 rsn = mk3(0, 0, 0), isn = mk3(0, 0, 0);
        float rsd = 0.0f, isd = 0.0f;
        if (lane < lnr) {
            int rv1 = m.loop_v[lr0 + (lane + 1 == lnr ? 0 : lane + 1)];
            f3 v0 = ld3(wvr[rv]);
            rsn = cross3(ld3(wvr[rv1]) - v0, nref);
            rsn = rsn * (1.0f / sqrtf(dot3(rsn, rsn)));
            rsd = -dot3(rsn, v0);
        }
        if (lane < lni) {
            int iv1 = m.loop_v[li0 + (lane + 1 == lni ? 0 : lane + 1)];
            f3 v0 = ld3(wvi[iv]);
            isn = cross3(ld3(wvi[iv1]) - v0, ni);
            isn = isn * (1.0f / sqrtf(dot3(isn, isn)));
            isd = -dot3(isn, v0);
        }
        int q = lane - nv1;
        int qe = q >> 1, qr = q - 2 * lni;
        int ivq0 = __shfl(iv, qe < 0 ? 0 : qe), ivq1 = __shfl(iv, qe + 1 >= lni ? 0 : qe + 1);
        int rvq = __shfl(rv, qr < 0 ? 0 : qr);
        // (2) lanes q < 2 lni: incident-face loop edge q / 2 clipped (Cyrus-Beck) to the reference face's side planes
        //     (through its loop edges, perpendicular to it): the entry (even q) or exit (odd q) point, when inside the
        //     segment and within the margin of the reference face
        // (3) lanes 2 lni <= q < 2 lni + lnr: reference-face loop vertex q - 2 lni projected along the reference normal
        //     onto the incident face's plane: a candidate when inside the incident face's side planes and within the
        //     margin
        // The plane loops run in wave-uniform control flow: a v_readlane of a lane's side plane inside a divergent
        // branch would read a register the allocator may reuse in that lane on the other branch
        bool isclip = q >= 0 && q < 2 * lni;
        bool isref = q >= 2 * lni && q < 2 * lni + lnr;
        f3 p0 = ld3(wvi[ivq0]), p1 = ld3(wvi[ivq1]);
        f3 r = ld3(wvr[rvq]);
        float sr = den < -1e-6f ? -(dot3(ni, r) + di) / den : 0.0f;
        f3 xr = r + nref * sr;
        float tin = 0.0f, tout = 1.0f, mx = -3.0e38f;
        bool out = false;
#pragma unroll 1
        for (int jj = 0; jj < lnr; jj++) {
            f3 sn = mk3(bcast(rsn.x, jj), bcast(rsn.y, jj), bcast(rsn.z, jj));
            float sd = bcast(rsd, jj);
            float f0 = dot3(sn, p0) + sd, f1 = dot3(sn, p1) + sd;
            if (f0 > 0.0f && f1 > 0.0f) out = true;
            else if (f0 > 0.0f) tin = fmaxf(tin, f0 / (f0 - f1));
            else if (f1 > 0.0f) tout = fminf(tout, f0 / (f0 - f1));
        }
#pragma unroll 1
        for (int jj = 0; jj < lni; jj++) {
            f3 sn = mk3(bcast(isn.x, jj), bcast(isn.y, jj), bcast(isn.z, jj));
            mx = fmaxf(mx, dot3(sn, xr) + bcast(isd, jj));
        }
        if (isclip) {
            bool ex = (q & 1) != 0;
            f3 xc = p0 + (p1 - p0) * (ex ? tout : tin);
            float dx = dot3(nref, xc) + dref;
            ok = !out && (ex ? (tout < 1.0f && tin < tout) : (tin > 0.0f && tin <= tout)) && dx <= mg;
            x = xc - nref * (0.5f * dx);
            sv = dx;
        } else if (isref) {
            ok = den < -1e-6f && sr <= mg && mx <= 0.0f;
            x = r + nref * (0.5f * sr);
            sv = sr;
        }
        HPROF(31);
        if (__ballot(ok)) {
            f3 n = refB ? nref : nref * -1.0f;
            // anchors: candidates (1) and (2) on the incident hull, (3) on the reference hull; the normal on the reference
            int nA = refB ? 0 : PCM_NORMAL_A;
            int code = (isref ? (refB ? PCM_FEAT_B : PCM_FEAT_A) : (refB ? PCM_FEAT_A : PCM_FEAT_B)) | nA;
            emit_contacts(c, ok, x, sv, n, a, b, code);
            HPROF(29);
            return;
        }
        wsync();
    }
}
#undef HPROF

// does a sphere (center c, radius r) reach the table box? Conservative for the hull inside the sphere,
// so culling with it never removes a contact the narrow phase would produce.
HD bool sphere_near_box(const float* half, PoseF Pb, f3 c, float r) {
    qf qi = qf{-Pb.q.x, -Pb.q.y, -Pb.q.z, Pb.q.w};
    f3 pl = qrot(qi, c - Pb.p);
    float dx = fmaxf(fabsf(pl.x) - half[0], 0.0f);
    float dy = fmaxf(fabsf(pl.y) - half[1], 0.0f);
    float dz = fmaxf(fabsf(pl.z) - half[2], 0.0f);
    return dx * dx + dy * dy + dz * dz <= r * r;
}
// Two unscaled hulls' oriented boxes (hull_obb: link hulls and, since round 6, every piece of a compound object),
// posed by their bodies, within the margin on all 15 axes (include/ha_obb.h, the oracle's text too): a compound pair's
// piece pair that fails it cannot touch, so its narrow phase is skipped in both. Elongated pieces (spoon, wrench,
// scissors) have loose spheres: in the C4w tail envs the boxes reject two thirds of the piece pairs the spheres keep
#ifdef HA_PIECE_BOX_CALL      /* A/B: the box test as a real call (C4w 6.27 vs 6.17 ms inline, profiles/r06_ab_*) */
__device__ __attribute__((noinline))
#else
HD
#endif
bool piece_boxes_near(const ha_model_t& m, int h1, PoseF P1, int h2, PoseF P2, float mg) {
    float p1[3] = {P1.p.x, P1.p.y, P1.p.z}, q1[4] = {P1.q.x, P1.q.y, P1.q.z, P1.q.w};
    float p2[3] = {P2.p.x, P2.p.y, P2.p.z}, q2[4] = {P2.q.x, P2.q.y, P2.q.z, P2.q.w};
    return ha_obb_pair_near(p1, q1, m.hull_obb[h1], p2, q2, m.hull_obb[h2], mg) != 0;
}
// static k's world pose: its model pose, composed with the env's posed actor (s.sb) when the actor carries it (v14)
HD PoseF static_pose(const SimCtx& c, int k) {
    const ha_model_t& m = *c.m;
    PoseF P{ld3(m.static_pos[k]), ldq(m.static_quat[k])};
    if (m.static_posed[k]) {
        f3 bp = ld3(c.s->sb);
        qf bq = ldq(c.s->sb + 4);
        P = PoseF{bp + qrot(bq, P.p), qmul(bq, P.q)};
    }
    return P;
}
// Oriented boxes of the broad phase's box cull (pair_boxes_near): centre, orientation, half extents. A link hull's fitted
// box (hull_obb) posed by its link; a one-piece object's box (its hull's bounding box in the body frame, identity
// orientation, model.py object_box) scaled by the env's object scale and posed by the object; a static's box
// (static_half) at its pose. ha_create checks that every such hull lies inside its box.
HD void link_box(const SimCtx& c, int h, f3& bc, qf& bq, f3& hh) {
    int L = c.m->hull_link[h];
    const float* ob = c.m->hull_obb[h];
    qf lq = ldq(c.s->lq[L]);
    bc = ld3(c.s->lp[L]) + qrot(lq, ld3(ob));
    bq = qmul(lq, ldq(ob + 6));
    hh = ld3(ob + 3);
}
HD void object_box(const SimCtx& c, int o, f3& bc, qf& bq, f3& hh) {
    const float* ob = c.m->hull_obb[c.m->pool_hull[c.o[o].pool]];
    PoseF P = object_pose(c, o);
    bc = P.p + qrot(P.q, scale3(c, o, ld3(ob)));
    bq = P.q;
    hh = scale3(c, o, ld3(ob + 3));
}
HD void static_box(const SimCtx& c, int k, f3& bc, qf& bq, f3& hh) {
    PoseF P = static_pose(c, k);
    bc = P.p;
    bq = P.q;
    hh = ld3(c.m->static_half[k]);
}
// Box cull of a broad-phase candidate (kinds 1-4; lane-parallel in detect): false when the two sides' boxes are
// separated by more than the contact margin + 1 mm on one of the 15 box SAT axes (ha_obb.h ha_obb_sat, conservative;
// the 1 mm covers the rounding of the posed boxes). Their hulls are then apart too and the narrow phase would emit nothing (nor write a
// persistent-manifold record: pcm_commit writes none for an empty manifold); the oracle has no such cull and runs the
// narrow phase, which finds the same empty result. Compound objects (several pieces) are not culled here
HD bool pair_boxes_near(const SimCtx& c, int kind, int A, int B, float mg) {
    const ha_model_t& m = *c.m;
    if (kind <= 3 && m.pool_nhull[c.o[A].pool] != 1) return true;
    if (kind == 2 && m.pool_nhull[c.o[B].pool] != 1) return true;
    f3 ca, cb, ha, hb;
    qf qa, qb;
    if (kind == 4) link_box(c, A, ca, qa, ha);
    else object_box(c, A, ca, qa, ha);
    if (kind == 1 || kind == 4) static_box(c, B, cb, qb, hb);
    else if (kind == 2) object_box(c, B, cb, qb, hb);
    else link_box(c, B, cb, qb, hb);
    // the posed boxes as ha_obb.h records (centre, half, quat) at the origin, then its 15-axis test
    float ra[12] = {0.0f, 0.0f, 0.0f, ha.x, ha.y, ha.z, qa.x, qa.y, qa.z, qa.w, 0.0f, 0.0f};
    float rb[12] = {0.0f, 0.0f, 0.0f, hb.x, hb.y, hb.z, qb.x, qb.y, qb.z, qb.w, 0.0f, 0.0f};
    const float id[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    float pa[3] = {ca.x, ca.y, ca.z}, pb[3] = {cb.x, cb.y, cb.z};
    float xa[3], Ra[9], xb[3], Rb[9];
    ha_obb_world(pa, id, ra, xa, Ra);
    ha_obb_world(pb, id, rb, xb, Rb);
    return ha_obb_sat(xa, Ra, ra + 3, xb, Rb, rb + 3, mg + 1e-3f) != 0;
}

// pair enumeration in the oracle's order (see detect() in physics_oracle.c)
// pair p -> (kind, A, B): kinds 0 object-ground, 1 object-static B, 2 object-object, 3 link hull B - object,
// 4 link hull A - static B; then (detect's self-pair pass) 5: self-collision pair A of the model (v12 self_pair)
HD bool pair_desc(const SimCtx& c, int p, int& kind, int& A, int& B) {
    int NO = c.NO, NLH = c.m->n_link_hulls, NS = c.m->n_static;
    for (int o = 0; o < NO; o++) {
        int n = 1 + NS + (NO - 1 - o) + NLH;
        if (p < n) {
            A = o;
            if (p == 0) { kind = 0; B = -1; }
            else if (p < 1 + NS) { kind = 1; B = p - 1; }
            else if (p < 1 + NS + (NO - 1 - o)) { kind = 2; B = o + 1 + (p - 1 - NS); }
            else { kind = 3; B = p - 1 - NS - (NO - 1 - o); }
            return true;
        }
        p -= n;
    }
    if (p < NLH * NS) { kind = 4; A = p / NS; B = p - A * NS; return true; }
    return false;
}

// ----------------------------------------------------------------------------- hierarchical broad phase (round 6)
// Most of the enumeration above is link-hull pairs (C5: 176 object-link and 132 link-static of 392), and in a bin
// scene nearly all of them fail the sphere / box tests. Before the 64-pair batches, detect() bounds the link hulls
// in quads (hulls 4g .. 4g+3, one DPP quad of lanes): centre C_g = the mean of the quad's hull centres, radius R_g =
// max_k (|c_k - C_g| + r_k). A pair (object o, hull k) passes the sphere test only if |c_o - c_k| <= r_o + r_k + mg,
// and then |c_o - C_g| <= r_o + R_g + mg (triangle inequality); a link-static pair passes the box test only if the
// box distance of c_k is <= r_k + mg, and the box distance is 1-Lipschitz, so that of C_g is <= R_g + mg. The quad
// tests (with 0.1% + 1 mm of slack over float rounding) therefore reject only pairs the per-pair tests reject, and
// the batches run over the pairs of the quads that pass, in the enumeration's order with their enumeration index
// (record slots, face records): the contacts, their order and every record are those of the flat enumeration,
// which the oracle keeps. om: bit o*G + g = object o near quad g; sm: bit g*NS + b = static b near quad g.
HD int quad_hulls(uint32_t g, int G, int NLH) {
    return 4 * __builtin_popcount(g) - (int)((g >> (G - 1)) & 1u) * (4 * G - NLH);
}
// the t-th hull of the quads set in g
HD int quad_hull(uint32_t g, int t, int NLH) {
    for (int q = 0; g; q++, g >>= 1) {
        if (!(g & 1u)) continue;
        int nh = min(4, NLH - 4 * q);
        if (t < nh) return 4 * q + t;
        t -= nh;
    }
    return -1;
}
// pair r of the culled enumeration: its kind / sides, and p = its index in the flat one (pair_desc)
HD bool pair_compact(const SimCtx& c, int G, uint64_t om, uint64_t sm, int& p, int& kind, int& A, int& B) {
    int NO = c.NO, NLH = c.m->n_link_hulls, NS = c.m->n_static;
    int r = p, orig = 0;
    uint32_t gm = (1u << G) - 1u;
    for (int o = 0; o < NO; o++) {
        int head = 1 + NS + (NO - 1 - o);
        uint32_t g = (uint32_t)(om >> (o * G)) & gm;
        int nl = quad_hulls(g, G, NLH);
        if (r < head + nl) {
            A = o;
            if (r == 0) { kind = 0; B = -1; }
            else if (r < 1 + NS) { kind = 1; B = r - 1; }
            else if (r < head) { kind = 2; B = o + 1 + (r - 1 - NS); }
            else { kind = 3; B = quad_hull(g, r - head, NLH); }
            p = orig + (kind == 3 ? head + B : r);
            return true;
        }
        r -= head + nl;
        orig += head + NLH;
    }
    uint32_t bm = (1u << NS) - 1u;
    for (int q = 0; q < G; q++) {
        uint32_t s = (uint32_t)(sm >> (q * NS)) & bm;
        int pc = __builtin_popcount(s), cnt = min(4, NLH - 4 * q) * pc;
        if (r < cnt) {
            int h = r / pc, k = r - h * pc;
            for (; k > 0; k--) s &= s - 1u;
            kind = 4; A = 4 * q + h; B = __builtin_ctz(s);
            p = orig + A * NS + B;
            return true;
        }
        r -= cnt;
    }
    return false;
}
// the quads' object / static masks and the culled pair count (G quads; G * NO <= 64, G * NS <= 64)
HD void broad_quads(const SimCtx& c, int G, uint64_t& om, uint64_t& sm, int& neff) {
    const EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, NO = c.NO, NLH = m.n_link_hulls, NS = m.n_static;
    float mg = c.p->contact_margin;
    bool hv = lane < NLH;
    f3 ch = mk3(0.0f, 0.0f, 0.0f);
    float rk = 0.0f;
    if (hv) {
        int Lk = m.hull_link[lane];
        ch = ld3(s.lp[Lk]) + qrot(ldq(s.lq[Lk]), ld3(m.hull_center[lane]));
        rk = m.hull_radius[lane];
    }
    f3 C = ch;
    C.x += dpp_f<0xB1>(C.x); C.y += dpp_f<0xB1>(C.y); C.z += dpp_f<0xB1>(C.z);
    C.x += dpp_f<0x4E>(C.x); C.y += dpp_f<0x4E>(C.y); C.z += dpp_f<0x4E>(C.z);
    C = C * (1.0f / (float)max(1, min(4, NLH - (lane & ~3))));
    f3 dc = ch - C;
    float d = hv ? sqrtf(dot3(dc, dc)) + rk : 0.0f;
    d = fmaxf(d, dpp_f<0xB1>(d));
    d = fmaxf(d, dpp_f<0x4E>(d));
    float R = d * 1.001f + mg + 1.0e-3f;
    // statics near each quad (every lane of a quad holds its sphere; lane 4g's bits are read)
    uint32_t sb = 0;
    for (int b = 0; b < NS; b++)
        if (sphere_near_box(m.static_half[b], static_pose(c, b), C, R)) sb |= 1u << b;
    // quads near each object (lane o; an object with collisions off has no candidate pairs)
    f3 co = mk3(0.0f, 0.0f, 0.0f);
    float ro = -1.0e30f;
    if (lane < NO && c.o[lane].coll != 0) {
        int pa = c.o[lane].pool;
        PoseF Po = object_pose(c, lane);
        co = Po.p + qrot(Po.q, scale3(c, lane, ld3(m.pool_center[pa])));
        ro = scale_radius(c, lane, m.pool_radius[pa]);
    }
    uint32_t ob = 0;
    sm = 0;
    neff = 0;
    for (int q = 0; q < G; q++) {
        f3 Cq = mk3(bcast(C.x, 4 * q), bcast(C.y, 4 * q), bcast(C.z, 4 * q));
        float rr = (ro + bcast(R, 4 * q)) * 1.0001f;
        f3 dq = co - Cq;
        if (ro > -1.0e29f && dot3(dq, dq) <= rr * rr) ob |= 1u << q;
        uint32_t sq = (uint32_t)bcast_i((int)sb, 4 * q);
        sm |= (uint64_t)sq << (q * NS);
        neff += min(4, NLH - 4 * q) * __builtin_popcount(sq);
    }
    om = 0;
    for (int o = 0; o < NO; o++) {
        uint32_t g = (uint32_t)bcast_i((int)ob, o);
        om |= (uint64_t)g << (o * G);
        neff += 1 + NS + (NO - 1 - o) + quad_hulls(g, G, NLH);
    }
}
// the two link hulls of self-collision pair k
HD void self_pair_hulls(const ha_model_t& m, int k, int& ha, int& hb) {
    uint32_t sp = m.self_pair[k];
    ha = (int)(sp & 255u);
    hb = (int)(sp >> 8);
}

// ----------------------------------------------------------------------------- persistent contact manifolds (v13)
// PhysX keeps a pair's contact manifold across substeps (persistent contact manifolds, PCM; inferred, its source is
// closed) and refreshes its points from the bodies' current poses while their relative motion stays small. Here a
// record per candidate pair (ha_state_t.contact_cache, slot = the pair's index in detect's enumeration, then the self
// pairs) holds the manifold a narrow phase emitted: the relative pose it was built at, and per point the point on each
// body in that body's frame and the normal in side B's frame. The oracle restates every expression (pcm_store,
// pcm_refresh in physics_oracle.c), so results stay bit-identical.
//
// Side A / side B body poses and body codes of candidate pair (kind, A, B): the sides narrow_phase gives collide_hulls
// (UNIFORM: the pair is wave-uniform and its object poses read the pool id through an SGPR; false: a per-lane pair)
template <bool UNIFORM = true>
HD void pair_bodies(const SimCtx& c, int kind, int A, int B, PoseF& PA, PoseF& PB, int& a, int& b) {
    const EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    auto opose = [&](int o) { return UNIFORM ? object_pose_u(c, o) : object_pose(c, o); };
    if (kind <= 2) {
        PA = opose(A);
        a = A;
        if (kind == 0) { PB = PoseF{mk3(0, 0, 0), qf{0, 0, 0, 1}}; b = -1; }    // the ground plane z = 0
        else if (kind == 1) { PB = static_pose(c, B); b = -1; }
        else { PB = opose(B); b = B; }
    } else if (kind == 3) {
        int Lk = m.hull_link[B];
        PA = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])};
        a = 100 + Lk;
        PB = opose(A);
        b = A;
    } else if (kind == 4) {
        int Lk = m.hull_link[A];
        PA = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])};
        a = 100 + Lk;
        PB = static_pose(c, B);
        b = -1;
    } else {                                    // self pair A: hull b on side A, hull a on side B
        int ha_, hb_;
        self_pair_hulls(m, A, ha_, hb_);
        int La = m.hull_link[ha_], Lb = m.hull_link[hb_];
        PA = PoseF{ld3(s.lp[Lb]), ldq(s.lq[Lb])};
        a = 100 + Lb;
        PB = PoseF{ld3(s.lp[La]), ldq(s.lq[La])};
        b = 100 + La;
    }
}
HD qf qconj(qf q) { return qf{-q.x, -q.y, -q.z, q.w}; }

// The record of the running pair's manifold (c.pslot), from the points emit_contacts staged: lane t < k its point on
// A (x + n sep / 2) in A's frame, its point on B (x - n sep / 2) in B's frame, its normal in the frame of the body that
// carries it and its anchor; lane 0 the relative pose and k. Vector stores: every record access of the kernel is a
// per-lane vector access
HD void pcm_commit(SimCtx& c) {
    int k = c.pemit;
    c.pemit = 0;
    if (c.pslot < 0 || k <= 0) return;
    wsync();
    PoseF PA, PB;
    int a_, b_;
    pair_bodies(c, c.pkind, c.pA, c.pB, PA, PB, a_, b_);
    float* rec = c.pcm + (size_t)c.pslot * HA_PCM_REC;
    qf qbc = qconj(PB.q);
    int t = c.lane < k ? c.lane : -1;
    if (t >= 0) {
        const float* q = reinterpret_cast<const float*>(c.col.cand) + 8 * t;
        f3 x = mk3(q[0], q[1], q[2]), n = mk3(q[3], q[4], q[5]);
        float sep = q[6];
        int code = __float_as_int(q[7]);
        float hs = 0.5f * sep;
        qf qac = qconj(PA.q);
        f3 la = qrot(qac, (x + n * hs) - PA.p);
        f3 lb = qrot(qbc, (x - n * hs) - PB.p);
        f3 ln = qrot((code & PCM_NORMAL_A) ? qac : qbc, n);
        float* r = rec + 8 + 9 * t;
        st3(r, la);
        st3(r + 3, lb);
        st3(r + 6, ln);
        rec[44 + t] = (float)code;
    }
    if (c.lane == 0) {
        st3(rec, qrot(qbc, PA.p - PB.p));
        rec[3] = (float)k;
        stq(rec + 4, qmul(qbc, PA.q));
    }
}

// already-reduced points (lanes in order, valid ones only) into the contact list: the refreshed manifold of a record
HD void emit_points(SimCtx& c, bool valid, f3 pt, float sep, f3 n, int a, int b) {
    EnvLDS& s = *c.s;
    int lane = c.lane;
    uint64_t vm = __ballot(valid);
    int k = __popcll(vm);
    if (k == 0) return;
    int nc0 = s.nc;
    if (nc0 + k <= c.maxc) {
        count_offered(c, k, a, b);
        if (lane == 0) s.nc = nc0 + k;
        if (valid) ct_put(c, nc0 + __popcll(vm & ((1ull << lane) - 1ull)), pt, n, sep, a, b);
        wsync();
        return;
    }
    f3 P[4], N[4];
    float S[4];
    int CD[4] = {0, 0, 0, 0};           // (the list path does not read the anchors)
    uint64_t mk = vm;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        int src = mk ? __ffsll((unsigned long long)mk) - 1 : 0;
        mk &= mk - 1;
        P[t] = mk3(bcast(pt.x, src), bcast(pt.y, src), bcast(pt.z, src));
        N[t] = mk3(bcast(n.x, src), bcast(n.y, src), bcast(n.z, src));
        S[t] = bcast(sep, src);
    }
    store_chosen(c, k, P, N, S, CD, a, b);
}

// Pair slot `slot`'s record test (the oracle's pcm_refresh): it applies when it holds points and the pair's relative
// pose (A's body in B's frame) is within pcm_lin_tol / pcm_cos_tol of the pose it was built at. Evaluated per lane for a
// whole batch of candidate pairs at once (the broad phase's batch, or the first 64 self-pair candidates), so a pair whose
// record does not apply costs no load latency of its own. The header comes in two 16-byte loads per lane
HD bool pcm_valid_lane(const SimCtx& c, int slot, int kind, int A, int B) {
    const ha_params_t& p = *c.p;
    const float4* h = reinterpret_cast<const float4*>(c.pcm + (size_t)slot * HA_PCM_REC);
    float4 h0 = h[0], h1 = h[1];
    if ((int)h0.w <= 0) return false;
    PoseF PA, PB;
    int a_, b_;
    pair_bodies<false>(c, kind, A, B, PA, PB, a_, b_);
    qf qbc = qconj(PB.q);
    f3 d = qrot(qbc, PA.p - PB.p) - mk3(h0.x, h0.y, h0.z);
    float lt = p.pcm_lin_tol;
    if (dot3(d, d) > lt * lt) return false;
    qf qr = qmul(qbc, PA.q);
    float cq = ((qr.x * h1.x + qr.y * h1.y) + qr.z * h1.z) + qr.w * h1.w;
    return !(fabsf(cq) < p.pcm_cos_tol);
}
// one record in one register: lane i < HA_PCM_REC holds word i (a 192-byte coalesced load, issued a pair ahead)
HD float pcm_load(const SimCtx& c, int slot) {
    return c.lane < HA_PCM_REC ? c.pcm[(size_t)slot * HA_PCM_REC + c.lane] : 0.0f;
}
// A pair whose record applies (pcm_valid_lane): every point is re-evaluated from the current poses - the surface points
// carried by their bodies, the normal by the body that owns it, the separation along the normal, the point half the
// separation off its feature - those within the contact margin go to the list in record order, and the pair needs no
// narrow phase. rv = the record (pcm_load); lane t < k gathers its point's words by lane permutes
HD void pcm_emit_record(SimCtx& c, float rv, int kind, int A, int B) {
    const ha_params_t& p = *c.p;
    int lane = c.lane;
    int k = (int)bcast(rv, 3);
    PoseF PA, PB;
    int a, b;
    pair_bodies(c, kind, A, B, PA, PB, a, b);
    int t = lane < 4 ? lane : 0;
    float r[9];
#pragma unroll
    for (int f = 0; f < 9; f++) r[f] = __shfl(rv, 8 + 9 * t + f);
    int code = (int)__shfl(rv, 44 + t);
    bool valid = false;
    f3 x = mk3(0, 0, 0), n = mk3(0, 0, 0);
    float sp = 0.0f;
    if (lane < k && lane < 4) {
        f3 wa = PA.p + qrot(PA.q, mk3(r[0], r[1], r[2]));
        f3 wb = PB.p + qrot(PB.q, mk3(r[3], r[4], r[5]));
        n = qrot((code & PCM_NORMAL_A) ? PA.q : PB.q, mk3(r[6], r[7], r[8]));
        sp = dot3(n, wa - wb);
        valid = sp <= p.contact_margin;
        int f = code & 3;
        x = f == PCM_FEAT_A ? wa - n * (0.5f * sp) : (f == PCM_FEAT_B ? wb + n * (0.5f * sp) : (wa + wb) * 0.5f);
    }
    emit_points(c, valid, x, sp, n, a, b);
    if (lane == 0) c.s->cst[5] += 1;
}

// piece pairs of a candidate pair (1 unless an object is a compound of several convex pieces)
HD int pair_pieces(const SimCtx& c, int kind, int A, int B) {
    const ha_model_t& m = *c.m;
    if (kind >= 4) return 1;
    int n = m.pool_nhull[upool(c, A)];
    if (kind == 2) n *= m.pool_nhull[upool(c, B)];
    return n;
}

// Compound pairs (kinds 2, 3; round 6): which of piece pairs j0 .. j0 + 63 can touch. Lane t tests piece pair j0 + t:
// the two pieces' own spheres, then (unscaled bodies) their oriented boxes (piece_boxes_near); PhysX's broad phase
// sees each convex shape of an actor on its own. The oracle tests each piece pair the same way before its narrow phase
// (physics_oracle.c detect). A block of its own that derives everything from the pair's indices again, so that none of
// its values stay live into the narrow phases (VGPRs); the result is one 64-bit mask (SGPRs)
HD uint64_t piece_mask(const SimCtx& c, int kind, int A, int B, int j0, int np) {
    const EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int jj = j0 + c.lane;
    bool near = false;
    if (jj < np) {
        int ho = m.pool_hull[upool(c, A)];
        float mg = c.p->contact_margin;
        int h1, h2, b1, b2;
        PoseF P1, P2;
        f3 c1;
        float r1;
        if (kind == 2) {
            int pb = upool(c, B), n2 = m.pool_nhull[pb];
            int j1 = jj / n2;
            h1 = ho + j1; h2 = m.pool_hull[pb] + (jj - j1 * n2);
            P1 = object_pose_u(c, A); P2 = object_pose_u(c, B); b1 = A; b2 = B;
            c1 = P1.p + qrot(P1.q, scale3(c, A, ld3(m.hull_center[h1])));
            r1 = scale_radius(c, A, m.hull_radius[h1]);
        } else {
            int Lk = m.hull_link[B];
            h1 = B; P1 = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; b1 = -1;
            h2 = ho + jj; P2 = object_pose_u(c, A); b2 = A;
            c1 = P1.p + qrot(P1.q, ld3(m.hull_center[B]));
            r1 = m.hull_radius[B];
        }
        f3 c2 = P2.p + qrot(P2.q, scale3(c, b2, ld3(m.hull_center[h2])));
        float rr = r1 + scale_radius(c, b2, m.hull_radius[h2]) + mg;
        f3 dc = c1 - c2;
        near = dot3(dc, dc) <= rr * rr;
#ifndef HA_X_NO_PIECE_BOX      /* A/B timing builds only (the oracle keeps the box test): the piece spheres alone */
        if (near && !body_scaled(c, b1) && !body_scaled(c, b2)) near = piece_boxes_near(m, h1, P1, h2, P2, mg);
#endif
    }
    return __ballot(near);
}

// narrow phase of piece pair j of candidate pair (kind, A, B): the two sides' hulls, poses and body codes
HD void narrow_phase(SimCtx& c, int kind, int A, int B, int j) {
    const EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    if (kind == 0) {
        if (c.lane == 0) c.s->cst[6] += 1;
        collide_ground(c, m.pool_hull[upool(c, A)] + j, object_pose_u(c, A), A);
        return;
    }
    int h1, h2, b1, b2, k2;
    PoseF P1, P2;
    if (kind <= 3) {
        // the objects of the pair: A on side A (kinds 1, 2), and the object on side B (kind 2: B, kind 3: A), posed by
        // one call each, so that the branches below only pick values (the branches share no look-alike calls)
        int pa = upool(c, A), ho = m.pool_hull[pa];
        int ob = kind == 2 ? B : A;
        int pb = upool(c, ob), n2 = m.pool_nhull[pb];
        PoseF Po = object_pose_u(c, A);
        PoseF Pb = object_pose_u(c, ob);
        if (kind == 1) {
            h1 = ho + j; P1 = Po; b1 = A; h2 = m.static_hull[B]; P2 = static_pose(c, B); b2 = -1; k2 = -100 - B;
            // the piece's own sphere against the exact box (the oracle's per-piece near_box; for a one-hull object
            // the broad phase's test again)
            f3 cp = Po.p + qrot(Po.q, scale3(c, A, ld3(m.hull_center[h1])));
            if (!sphere_near_box(m.static_half[B], P2, cp, scale_radius(c, A, m.hull_radius[h1]) + c.p->contact_margin))
                return;
        } else if (kind == 2) {
            int j1 = j / n2;
            h1 = ho + j1; P1 = Po; b1 = A; h2 = m.pool_hull[pb] + (j - j1 * n2); P2 = Pb; b2 = B; k2 = B;
        } else {
            int Lk = m.hull_link[B];
            h1 = B; P1 = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; b1 = 100 + Lk; h2 = ho + j; P2 = Pb; b2 = A; k2 = A;
        }
    } else if (kind == 4) {
        int Lk = m.hull_link[A];
        h1 = A; P1 = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; b1 = 100 + Lk; h2 = m.static_hull[B];
        P2 = static_pose(c, B); b2 = -1; k2 = -100 - B;
    } else {
        // self-collision pair (a, b), a < b: hull b on side A, hull a on side B (normal from a to b). Consecutive pairs
        // share hull a, so side B's world vertices / planes stay in the scratch and a pair whose side-A sphere clears one
        // of a's planes never sets up side A
        int ha_, hb_;
        self_pair_hulls(m, A, ha_, hb_);
        int La = m.hull_link[ha_], Lb = m.hull_link[hb_];
        h1 = hb_; P1 = PoseF{ld3(s.lp[Lb]), ldq(s.lq[Lb])}; b1 = 100 + Lb;
        h2 = ha_; P2 = PoseF{ld3(s.lp[La]), ldq(s.lq[La])}; b2 = 100 + La; k2 = b2;
    }
    if (c.lane == 0) c.s->cst[6] += 1;         // contact_stats: hull-pair narrow phases run (diagnostics)
    collide_hulls(c, h1, P1, h2, P2, b1, b2, b1, k2);
}

// a compound pair's gathered points (lane = point, in gather order) -> one manifold of <= 4 contacts
HD void gather_emit(SimCtx& c, int kind, int A, int B) {
    EnvLDS& s = *c.s;
    const ColView& cs = c.col;
    wsync();
    int lane = c.lane;
    bool valid = lane < s.ng;
    f3 pt = mk3(0, 0, 0), n = mk3(0, 0, 0);
    float sep = 0;
    int code = 0;
    if (valid) {
        pt = ld3(cs.gp[lane]);
        sep = cs.gp[lane][3];
        n = ld3(cs.gn[lane]);
        code = __float_as_int(cs.gn[lane][3]);
    }
    int a = kind == 3 ? 100 + c.m->hull_link[B] : A;
    int b = kind == 2 ? B : (kind == 3 ? A : -1);
    emit_contacts(c, valid, pt, sep, n, a, b, code);
}

// self-collision pass (ha_model_t v12; after every other pair, the oracle's order):
//  1. the link hulls' world boxes (lane = hull, include/ha_obb.h ha_obb_world) and their circumscribed radii into the
//     narrow-phase scratch, component-major (lanes reading different hulls read consecutive words);
//  2. one lane per pair tests the two spheres (ha_obb_spheres_near); the pairs that pass are compacted, in pair order,
//     and one lane per such pair runs the 15 SAT axes (ha_obb_sat) - the oracle's ha_obb_near, split so that the
//     axis tests run on full waves. The candidate bits go to the env's LDS bit set (the narrow phases below overwrite the
//     scratch), and the first 64 candidates' records are loaded into a register at once;
//  3. per candidate, in pair order: if the pair's last narrow phase ended on a separating face (the env's per-pair
//     byte in its global area), that one face is tested first, with the narrow phase's own expressions (world plane,
//     the other hull's world vertices, min): still separating by more than the margin means the full narrow phase
//     would stop on a face too (its SAT maximises over every face), so the pair is skipped with the same result.
//     The record is a hint only: results never depend on it (the oracle has none);
//  4. otherwise the hull narrow phase, which records the separating face for the next substep.
HD void detect_self(SimCtx& c, int npairs) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane, NLH = m.n_link_hulls, nsp = m.n_self_pairs;
    float mg = c.p->contact_margin;
    float* tab = reinterpret_cast<float*>(c.col.wvA);        // tab[comp NLH + hull]: centre 3, R 9, half 3, radius
    uint16_t* spl = reinterpret_cast<uint16_t*>(tab + 16 * NLH);     // pairs whose spheres are near
    uint16_t* cdl = spl + nsp;                                       // the first 64 candidates
#ifdef HA_PROFILE
    unsigned long long _s0 = __builtin_amdgcn_s_memtime();
#endif
    if (lane < NLH) {
        int L = m.hull_link[lane];
        float w[15];
        ha_obb_world(s.lp[L], s.lq[L], m.hull_obb[lane], w, w + 3);
        w[12] = m.hull_obb[lane][3]; w[13] = m.hull_obb[lane][4]; w[14] = m.hull_obb[lane][5];
        for (int i = 0; i < 15; i++) tab[i * NLH + lane] = w[i];
        tab[15 * NLH + lane] = ha_obb_radius(w + 12);
    }
    if (lane < HA_MAX_SELF_PAIRS / 32) c.selfm[lane] = 0u;
    c.colA_h = c.colB_h = -1;           // the box table overwrote the cached hull sides
    c.colA_p = false;
    wsync();
    const uint64_t below = (1ull << lane) - 1ull;
    int nsl = 0;
#pragma unroll 1
    for (int base = 0; base < nsp; base += 64) {
        int p = base + lane;
        bool near = false;
        if (p < nsp) {
            int h1, h2;
            self_pair_hulls(m, p, h1, h2);
            float ca[3] = {tab[h1], tab[NLH + h1], tab[2 * NLH + h1]};
            float cb[3] = {tab[h2], tab[NLH + h2], tab[2 * NLH + h2]};
            near = ha_obb_spheres_near(ca, tab[15 * NLH + h1], cb, tab[15 * NLH + h2], mg) != 0;
        }
        uint64_t mk = __ballot(near);
        if (near) spl[nsl + __popcll(mk & below)] = (uint16_t)p;
        nsl += __popcll(mk);
    }
    wsync();
    int ncd = 0;
#pragma unroll 1
    for (int base = 0; base < nsl; base += 64) {
        int i = base + lane, p = 0;
        bool cand = false;
        if (i < nsl) {
            p = spl[i];
            int h1, h2;
            self_pair_hulls(m, p, h1, h2);
            float A[15], B[15];
            for (int q = 0; q < 15; q++) { A[q] = tab[q * NLH + h1]; B[q] = tab[q * NLH + h2]; }
            cand = ha_obb_sat(A, A + 3, A + 12, B, B + 3, B + 12, mg) != 0;
        }
        uint64_t mk = __ballot(cand);
        if (cand) {
            atomicOr(&c.selfm[p >> 5], 1u << (p & 31));
            int r = ncd + __popcll(mk & below);
            if (r < 64) cdl[r] = (uint16_t)p;
        }
        ncd += __popcll(mk);
    }
    wsync();
    // the records of the first 64 candidates (in pair order, the order of the loop below), one load for all; and the
    // point counts of their persistent manifolds (slot npairs + pair)
    int crec = 0xFF;
    if (c.selfc && lane < ncd) crec = c.selfc[cdl[lane]];
    // the first 64 candidates whose persistent-manifold record applies (lane = candidate rank), tested at once; their
    // records are loaded a candidate ahead
    // (in a block of its own before the candidate loop, so that none of its values stay live into the narrow phases)
    bool pv = false;
    if (c.pcm && lane < ncd) pv = pcm_valid_lane(c, npairs + cdl[lane], 5, cdl[lane], -1);
    uint64_t vmask = __ballot(pv);
    asm volatile("" : "+s"(vmask));
#ifdef HA_PROFILE
    PROF_COUNT(83, __builtin_amdgcn_s_memtime() - _s0);              // box table + box tests
#endif
    int rank = 0;
#pragma unroll 1
    for (int w32 = 0; w32 < (nsp + 31) >> 5; w32++) {
        uint32_t mask = c.selfm[w32];
#pragma unroll 1
        while (mask) {
            int bit = __ffs(mask) - 1;
            mask &= mask - 1;
            int k = __builtin_amdgcn_readfirstlane(32 * w32 + bit);
            int h1, h2;
            self_pair_hulls(m, k, h1, h2);
            int La = m.hull_link[h1], Lb = m.hull_link[h2];
#ifdef HA_PROFILE
            unsigned long long _r0 = __builtin_amdgcn_s_memtime();
            PROF_COUNT(85, 1);                                              // candidates
#endif
            int rec;
            bool refresh = false;
            if (rank < 64) {
                rec = __builtin_amdgcn_readlane(crec, rank);
                refresh = (vmask >> rank) & 1ull;
            } else {
                rec = __builtin_amdgcn_readfirstlane(c.selfc ? (int)c.selfc[k] : 0xFF);
            }
            c.pslot = -1;
            if (c.pcm) {
                // the pair's persistent manifold first (it decides the pair's contacts); then the separating-face record
#ifdef HA_PROFILE
                unsigned long long _q0 = __builtin_amdgcn_s_memtime();
#endif
                // (past the first 64 candidates: the same test in turn, on every lane)
                if (rank >= 64) refresh = __ballot(pcm_valid_lane(c, npairs + k, 5, k, -1)) != 0ull;
                if (refresh) pcm_emit_record(c, pcm_load(c, npairs + k), 5, k, -1);
#ifdef HA_PROFILE
                wsync();
                PROF_COUNT(88, __builtin_amdgcn_s_memtime() - _q0);
                PROF_COUNT(89, refresh);
#endif
                rank++;
                if (refresh) continue;
                c.pslot = npairs + k; c.pkind = 5; c.pA = k; c.pB = -1;
            } else {
                rank++;
            }
#ifdef HA_PROFILE
            PROF_COUNT(86, rec != 0xFF);                                    // candidates with a record
#endif
            if (rec != 0xFF) {
                // the recorded face (side B: hull a = h1, side A: hull b = h2) against the other hull's vertices
                bool fb = (rec & 0x80) != 0;
                int hf = fb ? h1 : h2, hv = fb ? h2 : h1, kf = rec & 0x7F;
                int Lf = fb ? La : Lb, Lv = fb ? Lb : La;
                if (kf < m.hull_nplanes[hf]) {
                    PoseF PF = PoseF{ld3(s.lp[Lf]), ldq(s.lq[Lf])}, PV = PoseF{ld3(s.lp[Lv]), ldq(s.lq[Lv])};
                    f3 n;
                    float d;
                    world_plane(m, hf, kf, PF, false, mk3(1, 1, 1), n, d);
                    float v = 3.0e38f;
                    if (lane < m.hull_nverts[hv]) v = dot3(n, PV.p + qrot(PV.q, ld3(m.verts[m.hull_vert_start[hv] + lane]))) + d;
                    bool skip = wave_min(v) > mg;
#ifdef HA_PROFILE
                    wsync();
                    PROF_COUNT(84, __builtin_amdgcn_s_memtime() - _r0);    // record checks
                    PROF_COUNT(87, skip);                                   // skipped by their record
#endif
                    if (skip) continue;                     // separated on that face, as the narrow phase would find
                }
            }
#ifdef HA_X_SELF_NO_NARROW    /* A/B timing builds only: the self pass without its narrow phases */
            continue;
#endif
#ifdef HA_PROFILE
            c.pk = 5;
            unsigned long long _k0 = __builtin_amdgcn_s_memtime();
            int _nc0 = s.nc;
#endif
#ifdef HA_X_SELF_DRY      /* A/B timing builds only: self narrow phases that emit no contacts */
            c.dry = true;
#endif
            narrow_phase(c, 5, k, -1, 0);
#ifdef HA_X_SELF_DRY
            c.dry = false;
#endif
            pcm_commit(c);
            c.pslot = -1;
            if (c.selfc && lane == 0 && c.sepf != rec) c.selfc[k] = (uint8_t)c.sepf;
#ifdef HA_PROFILE
            wsync();
            PROF_COUNT(80, __builtin_amdgcn_s_memtime() - _k0);          // self pairs: time / pairs / with contacts
            PROF_COUNT(81, 1);
            PROF_COUNT(82, s.nc != _nc0);
#endif
        }
    }
    wsync();
}

// The separating-face record of a one-piece candidate pair (PhysCfg off_pairf): the face its last narrow phase ended on
// (bit 7 set: a face of side B's hull, else of side A's; the low 7 bits its plane) against the other side's world
// vertices at the current poses, with the narrow phase's own expressions (world_plane, the posed vertices, dot + d).
// Separated by more than the margin, the hull SAT would end on a face as well and the pair has no contacts: skipping it
// changes no result (the oracle has no record and runs the narrow phase). Sides as narrow_phase gives them
HD bool sep_face_skip(const SimCtx& c, int kind, int A, int B, int rec) {
    const EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int h1, h2, b1, b2;
    PoseF P1, P2;
    if (kind == 1) {
        h1 = m.pool_hull[upool(c, A)]; P1 = object_pose_u(c, A); b1 = A;
        h2 = m.static_hull[B]; P2 = static_pose(c, B); b2 = -1;
    } else if (kind == 2) {
        h1 = m.pool_hull[upool(c, A)]; P1 = object_pose_u(c, A); b1 = A;
        h2 = m.pool_hull[upool(c, B)]; P2 = object_pose_u(c, B); b2 = B;
    } else if (kind == 3) {
        int Lk = m.hull_link[B];
        h1 = B; P1 = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; b1 = 100 + Lk;
        h2 = m.pool_hull[upool(c, A)]; P2 = object_pose_u(c, A); b2 = A;
    } else {
        int Lk = m.hull_link[A];
        h1 = A; P1 = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; b1 = 100 + Lk;
        h2 = m.static_hull[B]; P2 = static_pose(c, B); b2 = -1;
    }
    bool fb = (rec & 0x80) != 0;
    int kf = rec & 0x7F;
    int hf = fb ? h2 : h1, hv = fb ? h1 : h2, bf = fb ? b2 : b1, bv = fb ? b1 : b2;
    PoseF PF = fb ? P2 : P1, PV = fb ? P1 : P2;
    if (kf >= m.hull_nplanes[hf]) return false;
    f3 n;
    float d;
    world_plane(m, hf, kf, PF, body_scaled(c, bf), inv_scale(c, bf), n, d);
    float v = 3.0e38f;
    if (c.lane < m.hull_nverts[hv])
        v = dot3(n, PV.p + qrot(PV.q, scale3(c, bv, ld3(m.verts[m.hull_vert_start[hv] + c.lane])))) + d;
    return wave_min(v) > c.p->contact_margin;
}

template <bool SELF>
HD void detect(SimCtx& c) {
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    int lane = c.lane;
    if (lane == 0) { s.nc = 0; s.noff = 0; }
    c.colA_h = c.colB_h = -1;       // poses changed since the last detect(): no cached hull sides
    c.colA_p = false;
    c.colA_b = c.colB_b = -1000;
    int NO = c.NO, NLH = m.n_link_hulls, NS = m.n_static;
    int npairs = 0;
    for (int o = 0; o < NO; o++) npairs += 1 + NS + (NO - 1 - o) + NLH;
    npairs += NLH * NS;
    wsync();
    // the quad cull (above pair_compact) where the flat enumeration takes more than one batch
    int G = (NLH + 3) >> 2, neff = npairs;
    uint64_t om = 0, sm = 0;
#ifdef HA_X_FLAT_BROAD      /* A/B timing builds only: the flat enumeration */
    bool hier = false;
#else
    // (the Allegro scenes' enumerations fit one batch: compiled out of their kernels)
    bool hier = !SELF && npairs > 64 && G >= 1 && G * NO <= 64 && G * NS <= 64;
#endif
    if (hier) broad_quads(c, G, om, sm, neff);
    for (int base = 0; base < neff; base += 64) {
#ifdef HA_PROFILE
        unsigned long long _b0 = __builtin_amdgcn_s_memtime();
#endif
        // parallel broad phase: one pair per lane (p: its index in the flat enumeration)
        bool cand = false;
        int p = base + lane;
        int kind = -1, A = -1, B = -1;
        if (p < neff && (hier ? pair_compact(c, G, om, sm, p, kind, A, B) : pair_desc(c, p, kind, A, B))) {
            float mg = c.p->contact_margin;
            if (kind <= 3) {
                cand = c.o[A].coll != 0;
                if (kind == 2) cand = cand && c.o[B].coll != 0;
                if (cand) {
                    // an object's bounding sphere covers all its convex pieces (ha_model_t v8)
                    int pa = c.o[A].pool;
                    PoseF Po = object_pose(c, A);
                    f3 co = Po.p + qrot(Po.q, scale3(c, A, ld3(m.pool_center[pa])));
                    float ro = scale_radius(c, A, m.pool_radius[pa]);
                    if (kind == 0) {
                        cand = co.z - ro <= mg;
                    } else {
                        PoseF Pb;
                        f3 cl;
                        float rb;
                        if (kind == 1) {
                            int hb = m.static_hull[B];
                            Pb = static_pose(c, B); cl = ld3(m.hull_center[hb]); rb = m.hull_radius[hb];
                        } else if (kind == 2) {
                            int pb = c.o[B].pool;
                            Pb = object_pose(c, B); cl = ld3(m.pool_center[pb]); rb = m.pool_radius[pb];
                        } else {
                            int Lk = m.hull_link[B];
                            Pb = PoseF{ld3(s.lp[Lk]), ldq(s.lq[Lk])}; cl = ld3(m.hull_center[B]); rb = m.hull_radius[B];
                        }
                        int bb = kind == 2 ? B : -1;
                        f3 cbb = Pb.p + qrot(Pb.q, scale3(c, bb, cl));
                        f3 dc = co - cbb;
                        float rr = ro + scale_radius(c, bb, rb) + mg;
                        cand = dot3(dc, dc) <= rr * rr;
                        if (kind == 1) cand = cand && sphere_near_box(m.static_half[B], Pb, co, ro + mg);
                    }
                }
            } else {
                int Lk = m.hull_link[A];
                cand = m.link_table_collide[Lk] != 0;
                if (cand) {
                    PoseF Pst = static_pose(c, B);
                    int hs = m.static_hull[B];
                    f3 ch = ld3(s.lp[Lk]) + qrot(ldq(s.lq[Lk]), ld3(m.hull_center[A]));
                    f3 ct = Pst.p + qrot(Pst.q, ld3(m.hull_center[hs]));
                    f3 dc = ch - ct;
                    float rr = m.hull_radius[A] + m.hull_radius[hs] + mg;
                    cand = dot3(dc, dc) <= rr * rr;
                    // a table's bounding sphere (0.71 m) contains the whole hand: cull on the exact box
                    cand = cand && sphere_near_box(m.static_half[B], Pst, ch, m.hull_radius[A] + mg);
                }
            }
        }
        uint64_t mask = __ballot(cand);
#ifndef HA_X_NO_BOX_CULL     /* A/B timing builds only: the broad phase without its box cull */
        // the box cull of the candidates (pair_boxes_near), in a block of its own that derives everything from the pair
        // index again, so that none of its values stay live into the narrow phases (VGPRs). The Allegro families only
        // (SELF): A/B on one box, C3 4.94 -> 4.71 ms, C2 1.010 -> 0.975 ms; C4 +1%, C5 +0.5% (their link hulls seldom
        // come near an object, and the cull's registers cost the Ur5Sih kernels spills)
        if (SELF && mask) {
            bool keep = false;
            if ((mask >> lane) & 1ull) {
                int kd, a_, b_;
                pair_desc(c, p, kd, a_, b_);
                keep = kd == 0 || pair_boxes_near(c, kd, a_, b_, c.p->contact_margin);
            }
            mask = __ballot(keep);
            asm volatile("" : "+s"(mask));
            cand = (mask >> lane) & 1ull;
        }
#endif
        // the candidates whose persistent-manifold record applies (ha_params_t v13), tested for the whole batch at once;
        // each record is loaded at its turn (loading it one refresh ahead measured C4 +1.5%, C5 -0.7%, C2 / C4w +-0:
        // profiles/r06_ab_record_prefetch.txt)
        uint64_t vmask = __ballot(c.pcm && cand && pcm_valid_lane(c, p, kind, A, B));
        // and the candidates' separating-face records, one byte load each
        int frec = (cand && c.pairf) ? (int)c.pairf[p] : 0xFF;
#ifdef HA_PROFILE
        {   // the batch's broad phase: sphere / box tests, record validity, face-record loads (waited for here)
            int fw = wave_min_i(frec);
            wsync();
            PROF_COUNT(93, __builtin_amdgcn_s_memtime() - _b0 + (fw < -1 ? 1 : 0));
            PROF_COUNT(94, 1);
        }
#endif
        // one iteration per piece pair: a compound object (several convex pieces, ha_model_t v8) runs piece
        // pairs j = 0 .. np-1 of a candidate pair and then emits a single <= 4-point manifold for the object pair
        // (the oracle's gather_begin / gather_end). One loop and one call site per narrow phase (a single inlined
        // copy; a nested piece loop would keep its hoisted invariants live over the narrow phase: VGPRs)
        int j = 0;
        uint64_t pmask = 0;
        while (mask) {
            int bit = __ffsll((unsigned long long)mask) - 1;
            int q = base + bit;
            if (hier) pair_compact(c, G, om, sm, q, kind, A, B);
            else pair_desc(c, q, kind, A, B);
            // the pair is wave-uniform: say so, so that the narrow phase branches on scalars (no exec-masked regions)
#ifndef HA_X_DIVERGENT_PAIR   /* diagnostic: the pair indices left as the compiler sees them */
            kind = __builtin_amdgcn_readfirstlane(kind);
            A = __builtin_amdgcn_readfirstlane(A);
            B = __builtin_amdgcn_readfirstlane(B);
#endif
#ifdef HA_PROFILE
            c.pk = kind;
#endif
            if (j == 0 && c.pcm) {
                // the pair's persistent manifold: refreshed from its record, or the narrow phase writes the record
                c.pslot = -1;
                if ((vmask >> bit) & 1ull) {
#ifdef HA_PROFILE
                    unsigned long long _r0 = __builtin_amdgcn_s_memtime();
#endif
                    pcm_emit_record(c, pcm_load(c, q), kind, A, B);
#ifdef HA_PROFILE
                    wsync();
                    PROF_COUNT(88, __builtin_amdgcn_s_memtime() - _r0);     // refreshes
                    PROF_COUNT(89, 1);
#endif
                    mask &= mask - 1;
                    continue;
                }
                c.pslot = q; c.pkind = kind; c.pA = A; c.pB = B;
            }
            int np = pair_pieces(c, kind, A, B);
            int rec = 0xFF;
            if (c.pairf && kind != 0 && np == 1) {
                rec = __builtin_amdgcn_readlane(frec, bit);
#ifdef HA_PROFILE
                unsigned long long _f0 = __builtin_amdgcn_s_memtime();
#endif
                bool fskip = rec != 0xFF && sep_face_skip(c, kind, A, B, rec);
#ifdef HA_PROFILE
                if (rec != 0xFF) {
                    wsync();
                    PROF_COUNT(90, __builtin_amdgcn_s_memtime() - _f0);     // face-record checks: time / checks / skips
                    PROF_COUNT(91, 1);
                    PROF_COUNT(92, fskip);
                }
#endif
                if (fskip) {
                    c.pslot = -1;
                    mask &= mask - 1;
                    continue;                    // separated on that face, as the narrow phase would find
                }
            }
#ifdef HA_PROFILE
            unsigned long long _k0 = __builtin_amdgcn_s_memtime();
            int _nc0 = s.nc;
#endif
            if (np > 1 && j == 0) {
                if (lane == 0) s.ng = 0;
                c.gather = true;
                wsync();
            }
            // a compound pair's piece pairs that can touch (piece_mask, 64 at a time); the others run no narrow phase
            bool run = true;
            if constexpr (!SELF) {
                if (np > 1 && (kind == 2 || kind == 3)) {
                    if ((j & 63) == 0) pmask = piece_mask(c, kind, A, B, j, np);
                    uint64_t rest = pmask >> (j & 63);
                    run = (rest & 1ull) != 0;
                    if (!run) {
                        // straight to the next piece pair that can touch (or the chunk's end): the loop's ++j lands there
                        rest >>= 1;
                        int nxt = rest ? j + __ffsll((unsigned long long)rest) : (j | 63) + 1;
                        j = (nxt < np ? nxt : np) - 1;
                    }
                }
            }
#ifdef HA_AB_NARROW_TWICE
            for (int rep = 0; rep < 2 && run; rep++) {     // one call site: the same code size as the product
                if (rep == 1) { c.dry = true; c.colA_h = c.colB_h = -1; }
                narrow_phase(c, kind, A, B, j);
            }
            c.dry = false;
#else
            if (run) narrow_phase(c, kind, A, B, j);
#endif
            if (++j < np) continue;
            j = 0;
            mask &= mask - 1;
            if (np > 1) {
                c.gather = false;
                gather_emit(c, kind, A, B);
            }
            pcm_commit(c);
            c.pslot = -1;
            if (c.pairf && kind != 0 && np == 1 && lane == 0 && c.sepf != rec) c.pairf[q] = (uint8_t)c.sepf;
#ifdef HA_PROFILE
            wsync();
            PROF_COUNT(10 + kind, __builtin_amdgcn_s_memtime() - _k0);     // time / pairs / pairs with contacts
            PROF_COUNT(15 + kind, 1);
            PROF_COUNT(20 + kind, s.nc != _nc0);
#endif
        }
    }
    wsync();
    if constexpr (SELF) detect_self(c, npairs);
}

// ----------------------------------------------------------------------------- constraint rows
// Jacobian of body `body` into a compact row: robot block J (D wide; only touched for a link) and object
// blocks Job (slot so0 -> 0, else 1; Job = J + D for a dense row)
HD void jac_body(const SimCtx& c, int body, f3 x, f3 dir, float sgn, float* J, float* Job, int so0) {
    const EnvLDS& s = *c.s;
    if (body < 0) return;
    if (body < 100) {
        f3 r = x - ld3(c.o[body].oc);
        f3 ang = cross3(r, dir);
        float* Jo = Job + (body == so0 ? 0 : 6);
        Jo[0] += sgn * dir.x; Jo[1] += sgn * dir.y; Jo[2] += sgn * dir.z;
        Jo[3] += sgn * ang.x; Jo[4] += sgn * ang.y; Jo[5] += sgn * ang.z;
        return;
    }
    for (int j = body - 100; j >= 0; j = c.m->link_parent[j]) {
        int d = c.m->link_dof[j];
        if (d < 0) continue;
        J[d] += sgn * dot3(ld3(s.ax[d]), cross3(x - ld3(s.an[d]), dir));
    }
}

HD void tangents(f3 n, f3& t1, f3& t2) {
    f3 a = fabsf(n.x) < 0.9f ? mk3(1, 0, 0) : mk3(0, 1, 0);
    f3 t = cross3(n, a);
    float l = sqrtf(dot3(t, t));
    t1 = t * (1.0f / l);
    t2 = cross3(n, t1);
}

// Object blocks of one contact row (slot 0: object so0, slot 1: so1; row direction dir), in registers, by the
// expressions of jac_body and the stored rows: J = (0 + sgn dir, 0 + sgn (x - c_o) x dir) with sgn +1 for body a
// and -1 for body b, Y = (J_lin (1 / m), I_w^-1 J_ang); an absent slot is zero. Used by the families that recompute
// instead of storing them (PhysCfg RC), so every value equals the stored-row value bit for bit.
HD void obj_block(const SimCtx& c, int o, int a, f3 x, f3 dir, float* j6, float* y6) {
    if (o < 0) {
#pragma unroll
        for (int t = 0; t < 6; t++) { j6[t] = 0.0f; y6[t] = 0.0f; }
        return;
    }
    float sgn = o == a ? 1.0f : -1.0f;
    f3 ang = cross3(x - ld3(c.o[o].oc), dir);
    j6[0] = 0.0f + sgn * dir.x; j6[1] = 0.0f + sgn * dir.y; j6[2] = 0.0f + sgn * dir.z;
    j6[3] = 0.0f + sgn * ang.x; j6[4] = 0.0f + sgn * ang.y; j6[5] = 0.0f + sgn * ang.z;
    float im = c.o[o].oc[3];
    y6[0] = j6[0] * im; y6[1] = j6[1] * im; y6[2] = j6[2] * im;
    f3 ya = mv3(c.o[o].oIinv, mk3(j6[3], j6[4], j6[5]));
    y6[3] = ya.x; y6[4] = ya.y; y6[5] = ya.z;
}
// entry t (0..5) of slot object o's block of row direction dir: (J, Y), the values obj_block gives
HD void obj_entry(const SimCtx& c, int o, int a, f3 x, f3 dir, int t, float& j, float& y) {
    float sgn = o == a ? 1.0f : -1.0f;
    f3 ang = cross3(x - ld3(c.o[o].oc), dir);
    f3 jl = mk3(0.0f + sgn * dir.x, 0.0f + sgn * dir.y, 0.0f + sgn * dir.z);
    f3 ja = mk3(0.0f + sgn * ang.x, 0.0f + sgn * ang.y, 0.0f + sgn * ang.z);
    f3 ya = mv3(c.o[o].oIinv, ja);
    float im = c.o[o].oc[3];
    float jv = t == 0 ? jl.x : (t == 1 ? jl.y : (t == 2 ? jl.z : (t == 3 ? ja.x : (t == 4 ? ja.y : ja.z))));
    j = jv;
    y = t < 3 ? jv * im : (t == 3 ? ya.x : (t == 4 ? ya.y : ya.z));
}


template <class PC>
HD void substep(SimCtx& c, float hdt) {
    constexpr int ND = PC::nd, NCH = PC::nch, VW = PC::vw;
    constexpr int RSN = row_stride<ND>();
    // the lane id goes through an opaque move each substep: the per-lane 64-bit model addresses are then
    // recomputed here (one or two VALU ops) instead of being hoisted out of the substep loop and spilled
    asm volatile("" : "+v"(c.lane));
    PROF_BEGIN();
    EnvLDS& s = *c.s;
    const ha_model_t& m = *c.m;
    const ha_params_t& p = *c.p;
    int lane = c.lane, D = c.D, NO = c.NO;
    int NV = D + 6 * NO;
#ifdef HA_AB_DYN_TWICE
    for (int rep = 0; rep < 2; rep++) {
        fk(c);
        dynamics(c);
    }
#else
    fk(c);
    PROF(0);
    dynamics(c);
#endif
    PROF(1);
#ifdef HA_AB_FACTOR_TWICE
    for (int rep = 0; rep < 2; rep++)
#endif
    factor_inverse<ND>(c);
    // free motion: velocity-product forces only (drives are constraint rows of the PGS below)
    if (lane < D) {
        float acc = 0.0f;
        for (int j = 0; j < D; j++) acc = fmaf(c.Minv[lane * D + j], -hdt * s.Cb[j], acc);
        s.v[lane] = s.qd[lane] + acc;
    }
    if (lane < NO) {
        int o = lane;
        float damp = 1.0f / (1.0f + hdt * p.object_ang_damping);
        float R[9], Iw[9], Ii[9], Il[9];
        const float* I0 = m.pool_inertia[c.o[o].pool];
        float sc = c.dr ? c.dr[HA_DR_OBJ_MASS + o] : 1.0f;
        float mass = m.pool_mass[c.o[o].pool];
#pragma unroll
        for (int k = 0; k < 9; k++) Il[k] = I0[k];
        if (body_scaled(c, o)) {
            // uniform density scaled by S: C = tr(I)/2 Id - I (second moments), C' = det(S) S C S,
            // I' = tr(C') Id - C', m' = det(S) m
            const float* sv = c.o[o].osc;
            float det = (sv[0] * sv[1]) * sv[2];
            float h = 0.5f * ((I0[0] + I0[4]) + I0[8]);
            float Cs[9];
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) Cs[3 * i + j] = det * (sv[i] * (((i == j ? h : 0.0f) - I0[3 * i + j]) * sv[j]));
            float tr = (Cs[0] + Cs[4]) + Cs[8];
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) Il[3 * i + j] = (i == j ? tr : 0.0f) - Cs[3 * i + j];
            mass = mass * det;
        }
        qmat(ldq(c.o[o].oq), R);
        rart3(R, Il, Iw);
#pragma unroll
        for (int k = 0; k < 9; k++) Iw[k] = Iw[k] * sc;
        inv3(Iw, Ii);
#pragma unroll
        for (int k = 0; k < 9; k++) c.o[o].oIinv[k] = Ii[k];
        mass = mass * sc;
        c.o[o].om = mass;
        c.o[o].oc[3] = 1.0f / mass;     // the rows' 1 / m (obj_blocks reads it instead of dividing per PGS fetch)
        // external force and torque (zero unless a task applied them): constant over the call's substeps. Gravity: the
        // shard's randomized sim_params gravity when DR is on (v16)
        const float* grav = c.drg ? c.drg + HA_DRG_GRAVITY : p.gravity;
        f3 lv = (ld3(c.o[o].ov) + ld3(grav) * hdt) + ld3(c.o[o].ofx) * (hdt / mass);
        f3 av = ld3(c.o[o].ow) * damp + mv3(Ii, ld3(c.o[o].otq)) * hdt;
        float* vo = s.v + D + 6 * o;
        vo[0] = lv.x; vo[1] = lv.y; vo[2] = lv.z; vo[3] = av.x; vo[4] = av.y; vo[5] = av.z;
    }
    wsync();
    PROF(2);
#ifdef HA_AB_DETECT_TWICE
    for (int rep = 0; rep < 2; rep++) {
        int nc0 = s.nc;
        wsync();
        c.dry = rep == 1;
        detect<PC::selfc>(c);
        c.dry = false;
        if (rep == 1 && lane == 0) s.nc = nc0;
        wsync();
    }
#else
    detect<PC::selfc>(c);
#endif
    PROF(3);
#ifdef HA_PROFILE
    c.pcls = s.noff > HA_PROFILE_HEAVY ? 1 : 0;
#endif
    if (lane == 0) {        // contact-list diagnostics (ha_state_t.contact_stats)
        int off = s.noff;
        s.cst[0] += 1;
        s.cst[1] += off > c.maxc ? 1 : 0;
        s.cst[2] = off > s.cst[2] ? off : s.cst[2];
        s.cst[3] += off;
    }
    PROF_COUNT(8, s.nc);
    PROF_COUNT(9, 1);
    // ---- contact rows: in chunk ch, lane r < RPC owns global row RPC ch + r (normal, friction 1, friction 2 of
    //      contact CAP ch + r / 3). Rows are packed with the task's stride (J then Y), so a one-object task needs less
    //      LDS (row_stride, task_lds_bytes)
    constexpr int CAP = PC::cap, RPC = PC::rpc;
    float* Jb = s.u.rows.J;
    float* Yb = Jb + RPC * PC::lch * RSN;
    int nc = __builtin_amdgcn_readfirstlane(s.nc);      // wave-uniform (an SGPR: the chunk loops branch on it)
    int nr = 3 * nc;    // nc <= CAP x NCH -> <= RPC x NCH rows
    // split rows (PhysCfg): object blocks of every row (OW wide, J then Y), then the robot blocks of the
    // first KL link contacts (J then Y), then the env's global spill area for the link contacts after those
    constexpr int OW = PC::ow, KL = PC::kl, LCH = PC::lch, SPJ = 3 * (CAP * NCH - KL) * ND;
    float* Ob = Jb;
    float* ObY = Ob + RPC * LCH * OW;
    float* Rb = ObY + RPC * LCH * OW;
    float* RbY = Rb + 3 * KL * ND;
    // overflow chunks (PhysCfg OVF): dense rows of chunks 1.. in the env's global area (J, then Y)
    float* gJ = PC::ovf ? c.spill + PC::off_dense : nullptr;
    float* gY = PC::ovf ? gJ + RPC * (NCH - 1) * RSN : nullptr;
    // contacts that touch a robot link (split rows only): contacts 0..63 in lmask0, 64.. in lmask1
    uint64_t lmask0 = 0, lmask1 = 0;
    if constexpr (PC::split) {
        int a0 = 0, b0 = 0, a1 = 0, b1 = 0;
        if (lane < nc) ct_ab(c, lane, a0, b0);
        lmask0 = __ballot(lane < nc && (a0 >= 100 || b0 >= 100));
        if constexpr (CAP * NCH > 64) {
            if (lane + 64 < nc) ct_ab(c, lane + 64, a1, b1);
            lmask1 = __ballot(lane + 64 < nc && (a1 >= 100 || b1 >= 100));
        }
    }
    // robot-block slot of contact ci (-1: no link), and row k of its J or Y robot block
    auto lslot = [&](int ci) -> int {
        if (CAP * NCH <= 64 || ci < 64)
            return ((lmask0 >> ci) & 1ull) ? (int)__popcll(lmask0 & ((1ull << ci) - 1ull)) : -1;
        int cj = ci - 64;
        return ((lmask1 >> cj) & 1ull) ? (int)(__popcll(lmask0) + __popcll(lmask1 & ((1ull << cj) - 1ull))) : -1;
    };
    auto rrow = [&](int ls, int k, bool y) -> float* {
        if (ls < KL) return (y ? RbY : Rb) + (3 * ls + k) * ND;
        return c.spill + (y ? SPJ : 0) + (3 * (ls - KL) + k) * ND;
    };
    // object blocks (J or Y) of row r in the env's global row area (chunks LCH..)
    auto orow_g = [&](int r, bool y) -> float* {
        return c.spill + PC::spill_robot + (y ? RPC * (NCH - LCH) * OW : 0) + (r - RPC * LCH) * OW;
    };
    // PGS row constants of the lane's row in the current chunk: impulse, target velocity, 1/diagonal, friction and
    // the block's Delassus entries. One chunk: kept in registers. Several: stored per row in RK (after the rows, or
    // for overflow chunks in the env's global area) and swapped into registers chunk by chunk, so registers do not
    // grow with the contact capacity. Overflow chunks: while a substep has <= CAP contacts (chunk 0 only) the
    // constants stay in registers and RK is not touched
    float klam = 0.f, kvt = 0.f, kwinv = 0.f, kcmu = 0.f, kca0 = 0.f, kca1 = 0.f;
    float* RK;
    if constexpr (PC::ovf) RK = c.spill + PC::off_rk;
    else RK = reinterpret_cast<float*>(reinterpret_cast<char*>(s.u.rows.J) + pc_rowdata_bytes<PC>());
    static_assert(PC::rk_stride == RPC * NCH, "RK: one row-constant array per field, every chunk's rows");
    auto rk = [&](int q, int row) -> float& { return RK[q * PC::rk_stride + row]; };   // q < 6, row < rk_stride
    const bool multi = NCH > 1 && (!PC::ovf || nc > CAP);       // wave-uniform
    // packed sweeps (PhysCfg PACK): every substep of the clutter family, the overflow families' substeps whose contacts
    // fit chunk 0. Their row constants go to PK (per contact) instead of registers / RK
    const bool packed = PC::pack && (!PC::ovf || nc <= CAP);           // wave-uniform
    float* PK = PC::pack ? reinterpret_cast<float*>(reinterpret_cast<char*>(s.u.rows.J) + pc_pk_offset<PC>()) : nullptr;
    // chunk ch's rows. LDS (true) / global (false) dense rows are separate instantiations, so that no pointer may
    // address both (a flat pointer would make chunk 0's LDS rows flat accesses too)
    auto rows_chunk = [&](int ch, auto lds_tag) {
        constexpr bool LDSROWS = decltype(lds_tag)::value;
        float vt_ = 0.f, winv_ = 0.f, cmu_ = 0.f;
        int r = RPC * ch + lane;
        if (lane < RPC && r < nr) {
            const ContactLDS ct = ct_get(c, r / 3);
            cmu_ = contact_friction(c, ct.a, ct.b);
            int k = r % 3;
            // robot block Jr / Yr (null: the contact touches no link, the block is zero) and object blocks Jo / Yo
            float *Jr, *Yr, *Jo, *Yo;
            float jo_rc[PC::rc ? OW : 1], yo_rc[PC::rc ? OW : 1];     // RC: this row's object blocks, in registers
            if constexpr (PC::split) {
                int ls = lslot(r / 3);
                Jr = ls >= 0 ? rrow(ls, k, false) : nullptr;
                Yr = ls >= 0 ? rrow(ls, k, true) : nullptr;
                if constexpr (PC::rc) {
                    Jo = jo_rc;
                    Yo = yo_rc;
                } else {
                    if constexpr (LDSROWS) {
                        Jo = Ob + r * OW;
                        Yo = ObY + r * OW;
                    } else {
                        Jo = orow_g(r, false);
                        Yo = orow_g(r, true);
                    }
                    for (int t = 0; t < OW; t++) Jo[t] = 0.0f;
                }
                if (Jr)
                    for (int t = 0; t < ND; t++) Jr[t] = 0.0f;
            } else {
                if constexpr (LDSROWS) {
                    Jr = Jb + r * RSN;
                    Yr = Yb + r * RSN;
                } else {
                    Jr = gJ + (r - RPC) * RSN;
                    Yr = gY + (r - RPC) * RSN;
                }
                Jo = Jr + D;
                Yo = Yr + D;
                for (int t = 0; t < RSN; t++) Jr[t] = 0.0f;
            }
            f3 n = ld3(ct.n), t1, t2;
            tangents(n, t1, t2);
            f3 dir = k == 0 ? n : (k == 1 ? t1 : t2);
            f3 x = ld3(ct.x);
            int so0, so1;
            contact_slots(ct.a, ct.b, so0, so1);
            if constexpr (PC::rc) {
                // robot block from the link bodies; both object blocks (and their Y) straight into registers
                if (ct.a >= 100) jac_body(c, ct.a, x, dir, 1.0f, Jr, nullptr, so0);
                if (ct.b >= 100) jac_body(c, ct.b, x, dir, -1.0f, Jr, nullptr, so0);
                obj_block(c, so0, ct.a, x, dir, jo_rc, yo_rc);
                obj_block(c, so1, ct.a, x, dir, jo_rc + 6, yo_rc + 6);
            } else {
                jac_body(c, ct.a, x, dir, 1.0f, Jr, Jo, so0);
                jac_body(c, ct.b, x, dir, -1.0f, Jr, Jo, so0);
            }
            if (k == 0) {
                float sp = ct.sep;
                float sb = sp + p.contact_slop < 0.0f ? sp + p.contact_slop : 0.0f;   // penetration beyond the slop
                float v0 = sp > 0 ? -sp / hdt : -p.baumgarte * sb / hdt;
                if (v0 > p.max_depen_vel) v0 = p.max_depen_vel;
                vt_ = v0;
            }
            // Y_r = M^-1 J_r^T (robot block through the explicit inverse, object blocks 1/m, I_w^-1). The robot terms of
            // J_r . Y_r (the dense row's first terms, in its order) accumulate here from registers, so the block is
            // not read back: Jr / Yr may be a global spill row (a generic pointer, flat accesses)
            float a = 0.0f;
            if (Jr) {
                // J_r to registers first: read once here instead of D times in the product loop (same sums, same order)
                float jr[ND];
#pragma unroll
                for (int j = 0; j < ND; j++) jr[j] = Jr[j];
                for (int i = 0; i < D; i++) {
                    float acc = 0.0f;
#pragma unroll
                    for (int j = 0; j < ND; j++) acc = fmaf(c.Minv[i * D + j], jr[j], acc);
                    Yr[i] = acc;
                    a = fmaf(jr[i], acc, a);
                }
            }
            for (int sl = 0; sl < (PC::rc ? 0 : row_slots<ND>()); sl++) {    // RC: Y already from obj_block
                int o = sl == 0 ? so0 : so1;
                const float* Jos = Jo + 6 * sl;
                float* Yos = Yo + 6 * sl;
                if (o < 0) {
                    for (int t = 0; t < 6; t++) Yos[t] = 0.0f;
                    continue;
                }
                float im = 1.0f / c.o[o].om;
                Yos[0] = Jos[0] * im; Yos[1] = Jos[1] * im; Yos[2] = Jos[2] * im;
                f3 a = mv3(c.o[o].oIinv, mk3(Jos[3], Jos[4], Jos[5]));
                Yos[3] = a.x; Yos[4] = a.y; Yos[5] = a.z;
            }
            // same term order as the dense row: robot block (above), then the object blocks
            for (int t = 0; t < RSN - D; t++) a = fmaf(Jo[t], Yo[t], a);
            winv_ = 1.0f / (a + 1e-9f);
        }
        if (NCH == 1 || (PC::ovf && ch == 0)) {
            kvt = vt_; kwinv = winv_; kcmu = cmu_;
        }
        if (packed) {
            if (lane < RPC && r < nr) {
                int ck = r / 3, k = r - 3 * ck;
                HA_AS_LDS float* q = (HA_AS_LDS float*)(PK + HA_PK * ck);
                q[k] = 0.0f;                                // the impulse
                q[4 + k] = winv_;
                if (k == 0) q[3] = vt_;
                if (k == 1) q[7] = cmu_;
                if (k == 2) q[11] = 0.0f;
            }
        } else if (multi && lane < RPC) {
            rk(0, r) = 0.0f; rk(1, r) = vt_; rk(2, r) = winv_; rk(3, r) = cmu_;
        }
    };
#pragma unroll 1
    for (int ch = 0; ch < NCH; ch++) {
        if (NCH > 1 && RPC * ch >= nr && (PC::ovf || ch > 0)) break;      // wave-uniform: no rows left
        if (ch < LCH) rows_chunk(ch, std::true_type{});       // LDS rows (every chunk of a dense one-layout family)
        else rows_chunk(ch, std::false_type{});
    }
    wsync();
    // coupling inside each contact's 3-row block (Delassus entries J_ri . M^-1 J_rj^T, i > j): lane of
    // friction row 1 holds a10, lane of friction row 2 holds a20 and a21
    auto delassus_chunk = [&](int ch, auto lds_tag) {
        constexpr bool LDSROWS = decltype(lds_tag)::value;
        float ca0_ = 0.f, ca1_ = 0.f;
        int r = RPC * ch + lane;
        if (lane < RPC && r < nr && r % 3 != 0) {
            int k = r % 3, r0 = r - k;
            const float *Jo, *Y0o;
            float a = 0.0f, b = 0.0f;           // robot-block partial sums (J_rk . Y_r0, J_rk . Y_r1), t = 0 .. D-1
            auto rdot = [&](const float* Jr, const float* Y0r, const float* Y1r) {
                for (int t = 0; t < D; t++) a = fmaf(Jr[t], Y0r[t], a);
                if (k == 2)
                    for (int t = 0; t < D; t++) b = fmaf(Jr[t], Y1r[t], b);
            };
            float jo_rc[PC::rc ? OW : 1], y0_rc[PC::rc ? 2 * OW : 1];     // RC: J of this row, Y of rows r0, r0 + 1
            if constexpr (PC::split) {
                // LDS slot or global spill row on separate paths, so each keeps its own address space
                int ls = lslot(r / 3);
                if (ls >= 0 && ls < KL) rdot(Rb + (3 * ls + k) * ND, RbY + 3 * ls * ND, RbY + (3 * ls + 1) * ND);
                else if (ls >= KL) {
                    const float* sr = c.spill + 3 * (ls - KL) * ND;
                    rdot(sr + k * ND, sr + SPJ, sr + SPJ + ND);
                }
                if constexpr (PC::rc) {
                    const ContactLDS ct = ct_get(c, r / 3);
                    f3 n = ld3(ct.n), t1, t2;
                    tangents(n, t1, t2);
                    f3 x = ld3(ct.x);
                    int so0, so1;
                    contact_slots(ct.a, ct.b, so0, so1);
                    float scratch[OW];
                    f3 dk = k == 1 ? t1 : t2;
                    obj_block(c, so0, ct.a, x, dk, jo_rc, scratch);
                    obj_block(c, so1, ct.a, x, dk, jo_rc + 6, scratch + 6);
                    obj_block(c, so0, ct.a, x, n, scratch, y0_rc);
                    obj_block(c, so1, ct.a, x, n, scratch + 6, y0_rc + 6);
                    obj_block(c, so0, ct.a, x, t1, scratch, y0_rc + OW);
                    obj_block(c, so1, ct.a, x, t1, scratch + 6, y0_rc + OW + 6);
                    Jo = jo_rc;
                    Y0o = y0_rc;
                } else if constexpr (LDSROWS) {
                    Jo = Ob + r * OW;
                    Y0o = ObY + r0 * OW;
                } else {
                    Jo = orow_g(r, false);
                    Y0o = orow_g(r0, true);
                }
            } else if constexpr (LDSROWS) {
                rdot(Jb + r * RSN, Yb + r0 * RSN, Yb + (r0 + 1) * RSN);
                Jo = Jb + r * RSN + D;
                Y0o = Yb + r0 * RSN + D;
            } else {
                rdot(gJ + (r - RPC) * RSN, gY + (r0 - RPC) * RSN, gY + (r0 + 1 - RPC) * RSN);
                Jo = gJ + (r - RPC) * RSN + D;
                Y0o = gY + (r0 - RPC) * RSN + D;
            }
            const float* Y1o = Y0o + (PC::split ? OW : RSN);
            for (int t = 0; t < RSN - D; t++) a = fmaf(Jo[t], Y0o[t], a);
            ca0_ = a;
            if (k == 2) {
                for (int t = 0; t < RSN - D; t++) b = fmaf(Jo[t], Y1o[t], b);
                ca1_ = b;
            }
        }
        if (NCH == 1 || (PC::ovf && ch == 0)) {
            kca0 = ca0_; kca1 = ca1_;
        }
        if (packed) {
            if (lane < RPC && r < nr && r % 3 != 0) {
                int ck = r / 3, k = r - 3 * ck;
                HA_AS_LDS float* q = (HA_AS_LDS float*)(PK + HA_PK * ck);
                if (k == 1) q[8] = ca0_;
                else { q[9] = ca0_; q[10] = ca1_; }
            }
        } else if (multi && lane < RPC) {
            rk(4, r) = ca0_; rk(5, r) = ca1_;
        }
    };
#pragma unroll 1
    for (int ch = 0; ch < NCH; ch++) {
        if (NCH > 1 && RPC * ch >= nr && (PC::ovf || ch > 0)) break;
        if (ch < LCH) delassus_chunk(ch, std::true_type{});
        else delassus_chunk(ch, std::false_type{});
    }
    // ---- free passes (PhysCfg PACK): the contacts that touch no robot link, packed four per pass on pairwise disjoint
    //      objects by a greedy scan in contact order (each pass takes the lowest-index remaining contacts whose objects
    //      the pass does not hold yet: physics_oracle.c packed_passes). A pass is four contact bytes (0xFF: none), in
    //      the union after RK. Lane i holds contacts i and 64 + i; one ballot per pick
    int npass = 0;
    // the pass list stays in registers: pass p is lane p's pair (plo, phi) (p >= 64: plo2, phi2), four 16-bit fields,
    // one per contact: its index (0xFF: none), object slot 0 + 1 and object slot 1 + 1 (contact_slots), so that a
    // sweep decodes a pass from two scalars without an LDS round trip
    uint32_t plo = 0xFFFFFFFFu, phi = 0xFFFFFFFFu, plo2 = 0xFFFFFFFFu, phi2 = 0xFFFFFFFFu;
    if (packed) {
        int o00 = -1, o01 = -1, o10 = -1, o11 = -1;
        if (lane < nc) {
            int a_, b_;
            ct_ab(c, lane, a_, b_);
            o00 = (a_ >= 0 && a_ < 100) ? a_ : -1;
            o01 = (b_ >= 0 && b_ < 100) ? b_ : -1;
        }
        if (CAP * NCH > 64 && lane + 64 < nc) {
            int a_, b_;
            ct_ab(c, lane + 64, a_, b_);
            o10 = (a_ >= 0 && a_ < 100) ? a_ : -1;
            o11 = (b_ >= 0 && b_ < 100) ? b_ : -1;
        }
        uint64_t rem0 = __ballot(lane < nc) & ~lmask0;
        uint64_t rem1 = CAP * NCH > 64 ? __ballot(lane + 64 < nc) & ~lmask1 : 0ull;
        while (rem0 | rem1) {
            uint32_t objm = 0u;
            uint64_t pk = ~0ull;
            uint64_t cand0 = rem0, cand1 = rem1;
            for (int k = 0; k < 4 && (cand0 | cand1); k++) {
                int ci = cand0 ? __ffsll((unsigned long long)cand0) - 1 : 64 + __ffsll((unsigned long long)cand1) - 1;
                int oa = ci < 64 ? __builtin_amdgcn_readlane(o00, ci) : __builtin_amdgcn_readlane(o10, ci - 64);
                int ob = ci < 64 ? __builtin_amdgcn_readlane(o01, ci) : __builtin_amdgcn_readlane(o11, ci - 64);
                objm |= (oa >= 0 ? 1u << oa : 0u) | (ob >= 0 ? 1u << ob : 0u);
                int so0 = oa < 0 ? ob : (ob < 0 ? oa : (oa < ob ? oa : ob));
                int so1 = (oa >= 0 && ob >= 0) ? (oa < ob ? ob : oa) : -1;
                uint64_t fld = (uint64_t)ci | ((uint64_t)(so0 + 1) << 8) | ((uint64_t)(so1 + 1) << 12);
                pk = (pk & ~(0xFFFFull << (16 * k))) | (fld << (16 * k));
                if (ci < 64) rem0 &= ~(1ull << ci);
                else rem1 &= ~(1ull << (ci - 64));
                bool t0 = (o00 >= 0 && ((objm >> o00) & 1u)) || (o01 >= 0 && ((objm >> o01) & 1u));
                bool t1 = (o10 >= 0 && ((objm >> o10) & 1u)) || (o11 >= 0 && ((objm >> o11) & 1u));
                cand0 = rem0 & ~__ballot(t0);
                cand1 = rem1 & ~__ballot(t1);
            }
            if (npass < 64) {
                if (lane == npass) { plo = (uint32_t)pk; phi = (uint32_t)(pk >> 32); }
            } else if (lane == npass - 64) {
                plo2 = (uint32_t)pk; phi2 = (uint32_t)(pk >> 32);
            }
            npass++;
        }
    }
    PROF(4);
    // ---- joint rows, lane d: PD drive (soft implicit spring-damper, |impulse| <= effort h) and the
    //      lower/upper joint limits (hard, unilateral)
    float dgam = 0.f, dbias = 0.f, dwinv = 0.f, dlim = 0.f, dlam = 0.f;
    float lwinv = 0.f, vt_lo = 0.f, vt_up = 0.f, lam_lo = 0.f, lam_up = 0.f;
    // joint friction row (Isaac Gym DOF property "friction", a coefficient: "a generalized friction force is calculated
    // as DOF force multiplied by friction", docs/domain_randomization.md:197): target velocity 0 and
    // |impulse| <= dof_friction |drive + lower - upper impulse| of the DOF, re-bounded each sweep like a contact's
    // friction rows by its normal impulse
    float fcoef = 0.f, lam_fr = 0.f;
    int act_lo = 0, act_up = 0;
    if (lane < D) {
        fcoef = m.dof_friction[lane];
        // DR (v16): the env's dof_properties stiffness / damping / lower / upper (dr_scale row: nominal until sampled)
        float kp = c.dr ? c.dr[HA_DR_DOF_KP + lane] : m.dof_kp[lane];
        float kd = c.dr ? c.dr[HA_DR_DOF_KD + lane] : m.dof_kd[lane];
        float jlo = c.dr ? c.dr[HA_DR_DOF_LOWER + lane] : m.dof_lower[lane];
        float jup = c.dr ? c.dr[HA_DR_DOF_UPPER + lane] : m.dof_upper[lane];
        float den = kd + hdt * kp;
        float mii = c.Minv[lane * D + lane];
        dgam = 1.0f / (hdt * den);
        dbias = kp / den * (s.q[lane] - s.tgt[lane]);
        dwinv = 1.0f / (mii + dgam);
        dlim = m.dof_effort[lane] * hdt;
        lwinv = 1.0f / (mii + 1e-9f);
        float s_lo = s.q[lane] - jlo, s_up = jup - s.q[lane];
        act_lo = s_lo <= p.joint_limit_margin;
        act_up = s_up <= p.joint_limit_margin;
        vt_lo = s_lo > 0 ? -s_lo / hdt : -p.baumgarte * s_lo / hdt;
        vt_up = s_up > 0 ? -s_up / hdt : -p.baumgarte * s_up / hdt;
    }
    const uint64_t lo_mask = __ballot(act_lo != 0), up_mask = __ballot(act_up != 0), fr_mask = __ballot(fcoef > 0.0f);
    // generalized velocity: coordinate `lane` in vreg, coordinate 64 + lane in vregh (VW == 2 only)
    float vreg = lane < NV ? s.v[lane] : 0.0f;
    float vregh = (VW == 2 && lane + 64 < NV) ? s.v[lane + 64] : 0.0f;
    wsync();
    PROF(5);
    // ---- projected Gauss-Seidel (velocity form): joint rows d = 0..D-1 (drive, lower, upper), then
    //      contact rows r = 0..nr-1.  Same row order and arithmetic as the oracle.
    const float* J = Jb;
    const float* Y = Yb;
    // several chunks: the row constants of the chunk after the current one, loaded while the current one is solved
    float sl = 0.f, svt = 0.f, swinv = 0.f, scmu = 0.f, sca0 = 0.f, sca1 = 0.f;
    auto stage = [&](int ch) {
        int row = RPC * ch + lane;
        sl = rk(0, row); svt = rk(1, row); swinv = rk(2, row);
        scmu = rk(3, row); sca0 = rk(4, row); sca1 = rk(5, row);
    };
    if (!packed && multi && lane < RPC) stage(0);
    const int nca = (nc + CAP - 1) / CAP;                   // chunks in use (wave-uniform)
#ifdef HA_AB_PGS_TWICE
    for (int it = 0; it < 2 * p.solver_iters; it++) {
#else
    for (int it = 0; it < p.solver_iters; it++) {
#endif
        // Each joint row's update is computed by the lane that owns the joint (its own v[d], lambda and row
        // constants: the same operands the oracle uses), and only the impulse change crosses lanes (one
        // v_readlane); the joint-limit rows run only for the joints whose limit is active (ballot masks).
        for (int d = 0; d < D; d++) {
            float mrow = lane < D ? c.Minv[d * D + lane] : 0.0f;
            float nl = dlam - (vreg + dbias + dgam * dlam) * dwinv;
            nl = nl < -dlim ? -dlim : (nl > dlim ? dlim : nl);
            float dl = bcast(nl - dlam, d);
            if (dl != 0.0f) {
                if (lane == d) dlam = nl;
                vreg = fmaf(mrow, dl, vreg);
            }
            if ((lo_mask >> d) & 1ull) {
                float n0 = lam_lo - (vreg - vt_lo) * lwinv;
                n0 = n0 < 0.0f ? 0.0f : n0;
                float d0 = bcast(n0 - lam_lo, d);
                if (d0 != 0.0f) {
                    if (lane == d) lam_lo = n0;
                    vreg = fmaf(mrow, d0, vreg);
                }
            }
            if ((up_mask >> d) & 1ull) {
                float n1 = lam_up - (-vreg - vt_up) * lwinv;
                n1 = n1 < 0.0f ? 0.0f : n1;
                float d1 = bcast(n1 - lam_up, d);
                if (d1 != 0.0f) {
                    if (lane == d) lam_up = n1;
                    vreg = fmaf(-mrow, d1, vreg);
                }
            }
            if ((fr_mask >> d) & 1ull) {
                float flim = fcoef * fabsf((dlam + lam_lo) - lam_up);
                float nf = lam_fr - vreg * lwinv;
                nf = nf < -flim ? -flim : (nf > flim ? flim : nf);
                float df = bcast(nf - lam_fr, d);
                if (df != 0.0f) {
                    if (lane == d) lam_fr = nf;
                    vreg = fmaf(mrow, df, vreg);
                }
            }
        }
        // contact blocks: the three J.v reductions of a contact run together; the friction rows see the
        // normal (and first friction) update through the block's Delassus entries, which equals
        // re-reducing J.v after each row (row-by-row Gauss-Seidel) up to rounding
        // lane = generalized coordinate; its entry of a compact row is at compact_index (or absent -> 0).
        // The next contact's row entries are prefetched while the current one reduces.
        // (two contacts ahead: the m set is filled by fetch, the n set is the next contact's; an overflow chunk's rows
        // and most link contacts' robot blocks come from the env's global area, whose latency one contact of
        // reductions does not cover)
        float j0n = 0.f, j1n = 0.f, j2n = 0.f, y0n = 0.f, y1n = 0.f, y2n = 0.f;
        float h0n = 0.f, h1n = 0.f, h2n = 0.f, g0n = 0.f, g1n = 0.f, g2n = 0.f;   // coordinate 64 + lane
        float j0m = 0.f, j1m = 0.f, j2m = 0.f, y0m = 0.f, y1m = 0.f, y2m = 0.f;
        float h0m = 0.f, h1m = 0.f, h2m = 0.f, g0m = 0.f, g1m = 0.f, g2m = 0.f;
        constexpr bool TF = !PC::minv_in_union;        // typed fetch paths (lds_f), except the compact AllegroKuka layout
        auto fetch = [&](int ci) {
            float &j0n = j0m, &j1n = j1m, &j2n = j2m, &y0n = y0m, &y1n = y1m, &y2n = y2m;
            float &h0n = h0m, &h1n = h1m, &h2n = h2m, &g0n = g0m, &g1n = g1m, &g2n = g2m;
            int ix = lane < RSN ? lane : -1;       // one slot: the compact row is the dense row
            int ixh = -1;
            if constexpr (row_slots<ND>() == 2) {
                int ca, cb, so0, so1;
                ct_ab(c, ci, ca, cb);
                contact_slots(ca, cb, so0, so1);
                ix = compact_index(lane, D, so0, so1);
                if (VW == 2) ixh = compact_index(lane + 64, D, so0, so1);
            }
            j0n = 0.f; j1n = 0.f; j2n = 0.f; y0n = 0.f; y1n = 0.f; y2n = 0.f;
            h0n = 0.f; h1n = 0.f; h2n = 0.f; g0n = 0.f; g1n = 0.f; g2n = 0.f;
            if constexpr (PC::rc) {
                // object coordinates recomputed from the contact entry (obj_entry: the rows phase's values);
                // robot coordinates from the contact's link slot (LDS for the first KL, else the spill rows)
                const ContactLDS ct = ct_get(c, ci);
                int so0, so1;
                contact_slots(ct.a, ct.b, so0, so1);
                bool o1 = ix >= D, o2 = VW == 2 && ixh >= D;
                if (o1 || o2) {
                    f3 n = ld3(ct.n), t1, t2;
                    tangents(n, t1, t2);
                    f3 x = ld3(ct.x);
                    if (o1) {
                        int t = ix - D, o = t < 6 ? so0 : so1, e = t < 6 ? t : t - 6;
                        obj_entry(c, o, ct.a, x, n, e, j0n, y0n);
                        obj_entry(c, o, ct.a, x, t1, e, j1n, y1n);
                        obj_entry(c, o, ct.a, x, t2, e, j2n, y2n);
                    }
                    if (o2) {
                        int t = ixh - D, o = t < 6 ? so0 : so1, e = t < 6 ? t : t - 6;
                        obj_entry(c, o, ct.a, x, n, e, h0n, g0n);
                        obj_entry(c, o, ct.a, x, t1, e, h1n, g1n);
                        obj_entry(c, o, ct.a, x, t2, e, h2n, g2n);
                    }
                }
                if (ix >= 0 && ix < D) {
                    int ls = lslot(ci);         // wave-uniform: one path per contact, LDS or global
                    if (ls >= 0 && ls < KL) {
                        const float* Rn = Rb + 3 * ls * ND;
                        const float* RYn = RbY + 3 * ls * ND;
                        j0n = Rn[ix]; j1n = Rn[ND + ix]; j2n = Rn[2 * ND + ix];
                        y0n = RYn[ix]; y1n = RYn[ND + ix]; y2n = RYn[2 * ND + ix];
                    } else if (ls >= KL) {
                        const float* Rn = c.spill + 3 * (ls - KL) * ND;
                        const float* RYn = c.spill + SPJ + 3 * (ls - KL) * ND;
                        j0n = Rn[ix]; j1n = Rn[ND + ix]; j2n = Rn[2 * ND + ix];
                        y0n = RYn[ix]; y1n = RYn[ND + ix]; y2n = RYn[2 * ND + ix];
                    }
                }
                return;
            }
            if constexpr (PC::split) {
                // object coordinates from the object blocks (LDS for chunks < LCH, else the env's global row area);
                // robot coordinates from the contact's link slot (LDS for the first KL, else the global spill rows),
                // absent -> 0. LDS and global sources stay on separate paths (both conditions are wave-uniform)
                int lsc = lslot(ci);
                bool lds_obj = LCH == NCH || ci < CAP * LCH;
                if (lds_obj && lsc < KL) {
                    // every entry of this contact is in LDS: one set of loads, each lane's block (object block at
                    // stride OW, or the link slot's robot block at stride ND) chosen per lane
                    const float* On = Ob + 3 * ci * OW;
                    const float* OYn = ObY + 3 * ci * OW;
                    bool ob = ix >= D, rb = ix >= 0 && ix < D && lsc >= 0;
                    const float* P = ob ? On + (ix - D) : Rb + 3 * lsc * ND + ix;
                    const float* PY = ob ? OYn + (ix - D) : RbY + 3 * lsc * ND + ix;
                    int st = ob ? OW : ND;
                    if (ob || rb) {
                        j0n = P[0]; j1n = P[st]; j2n = P[2 * st];
                        y0n = PY[0]; y1n = PY[st]; y2n = PY[2 * st];
                    }
                } else if (ix >= D) {
                    int t = ix - D;
                    auto ldo = [&](auto On, auto OYn) {
                        j0n = On[t]; j1n = On[OW + t]; j2n = On[2 * OW + t];
                        y0n = OYn[t]; y1n = OYn[OW + t]; y2n = OYn[2 * OW + t];
                    };
                    if (lds_obj) ldo(lds_f<TF>(Ob + 3 * ci * OW), lds_f<TF>(ObY + 3 * ci * OW));
                    else ldo(glb_f<TF>(orow_g(3 * ci, false)), glb_f<TF>(orow_g(3 * ci, true)));
                } else if (ix >= 0) {
                    int ls = lsc;
                    auto ld6 = [&](auto Rn, auto RYn) {
                        j0n = Rn[ix]; j1n = Rn[ND + ix]; j2n = Rn[2 * ND + ix];
                        y0n = RYn[ix]; y1n = RYn[ND + ix]; y2n = RYn[2 * ND + ix];
                    };
                    if (ls >= 0 && ls < KL) ld6(lds_f<TF>(Rb + 3 * ls * ND), lds_f<TF>(RbY + 3 * ls * ND));
                    else if (ls >= KL) ld6(glb_f<TF>(c.spill + 3 * (ls - KL) * ND), glb_f<TF>(c.spill + SPJ + 3 * (ls - KL) * ND));
                }
                if (VW == 2 && ixh >= D) {
                    int t = ixh - D;
                    auto ldh = [&](auto On, auto OYn) {
                        h0n = On[t]; h1n = On[OW + t]; h2n = On[2 * OW + t];
                        g0n = OYn[t]; g1n = OYn[OW + t]; g2n = OYn[2 * OW + t];
                    };
                    if (lds_obj) ldh(lds_f<TF>(Ob + 3 * ci * OW), lds_f<TF>(ObY + 3 * ci * OW));
                    else ldh(glb_f<TF>(orow_g(3 * ci, false)), glb_f<TF>(orow_g(3 * ci, true)));
                }
                return;
            }
            auto ldd = [&](auto Jn, auto Yn) {
                if (ix >= 0) {
                    j0n = Jn[ix]; j1n = Jn[RSN + ix]; j2n = Jn[2 * RSN + ix];
                    y0n = Yn[ix]; y1n = Yn[RSN + ix]; y2n = Yn[2 * RSN + ix];
                }
                if (VW == 2) {
                    if (ixh >= 0) {
                        h0n = Jn[ixh]; h1n = Jn[RSN + ixh]; h2n = Jn[2 * RSN + ixh];
                        g0n = Yn[ixh]; g1n = Yn[RSN + ixh]; g2n = Yn[2 * RSN + ixh];
                    }
                }
            };
            if (PC::ovf && ci >= CAP) ldd(glb_f<TF>(gJ + 3 * (ci - CAP) * RSN), glb_f<TF>(gY + 3 * (ci - CAP) * RSN));   // wave-uniform
            else ldd(lds_f<TF>(J + 3 * ci * RSN), lds_f<TF>(Y + 3 * ci * RSN));
        };
        auto advance = [&]() {
            j0n = j0m; j1n = j1m; j2n = j2m; y0n = y0m; y1n = y1m; y2n = y2m;
            h0n = h0m; h1n = h1m; h2n = h2m; g0n = g0m; g1n = g1m; g2n = g2m;
        };
        // packed families: a contact block's constants (impulses, target velocities, 1/diagonals of its three rows, the
        // friction coefficient, the Delassus entries a10 a20 a21) - from RK (LDS), or with overflow chunks from the
        // registers of the lanes that own its rows in chunk 0 - and the serial block's arithmetic on them (n0, d0,
        // hi, n1 through the Delassus entries, n2), evaluated alike by every lane that calls it
        auto consts = [&](int ci, float* K) {                // three 16-byte LDS loads (a broadcast per row)
            typedef float f4v __attribute__((ext_vector_type(4)));
            const HA_AS_LDS f4v* q = (const HA_AS_LDS f4v*)(PK + HA_PK * ci);
            f4v a = q[0], b = q[1], e = q[2];
            K[0] = a.x; K[1] = a.y; K[2] = a.z; K[3] = a.w;
            K[4] = b.x; K[5] = b.y; K[6] = b.z; K[7] = b.w;
            K[8] = e.x; K[9] = e.y; K[10] = e.z;
        };
        // the friction rows' target velocity is 0: x - 0 is x, so the oracle's (jv1 - vt1) is jv1 here
        auto block = [&](const float* K, float jv0, float jv1, float jv2, float& n0, float& n1, float& n2, float& d0,
                         float& d1, float& d2) {
            n0 = K[0] - (jv0 - K[3]) * K[4];
            n0 = n0 < 0.0f ? 0.0f : (n0 > 3.0e38f ? 3.0e38f : n0);
            d0 = n0 - K[0];
            float hi = K[7] * n0;
            n1 = K[1] - fmaf(K[8], d0, jv1) * K[5];
            n1 = n1 < -hi ? -hi : (n1 > hi ? hi : n1);
            d1 = n1 - K[1];
            n2 = K[2] - fmaf(K[10], d1, fmaf(K[9], d0, jv2)) * K[6];
            n2 = n2 < -hi ? -hi : (n2 > hi ? hi : n2);
            d2 = n2 - K[2];
        };
        auto put_lams = [&](int ci, float n0, float n1, float n2) {
            HA_AS_LDS float* q = (HA_AS_LDS float*)(PK + HA_PK * ci);
            q[0] = n0; q[1] = n1; q[2] = n2;
        };
        HA_AS_LDS float* sv = (HA_AS_LDS float*)s.v;      // the generalized velocity of the passes (LDS accesses)
        if (packed) {
            // link contacts: whole-wave blocks in contact order, as the other families solve every contact
            uint64_t lk0 = lmask0, lk1 = lmask1;
            while (lk0 | lk1) {
                int ci = lk0 ? __ffsll((unsigned long long)lk0) - 1 : 64 + __ffsll((unsigned long long)lk1) - 1;
                if (ci < 64) lk0 &= lk0 - 1ull;
                else lk1 &= lk1 - 1ull;
                fetch(ci);
                advance();
                float jv0 = j0n * vreg, jv1 = j1n * vreg, jv2 = j2n * vreg;
                if (VW == 2) {
                    jv0 = jv0 + h0n * vregh;
                    jv1 = jv1 + h1n * vregh;
                    jv2 = jv2 + h2n * vregh;
                }
                wave_sum_rows3(jv0, jv1, jv2);
                float K[11], n0, n1, n2, d0, d1, d2;
                consts(ci, K);
                block(K, jv0, jv1, jv2, n0, n1, n2, d0, d1, d2);
                if (lane == 0) put_lams(ci, n0, n1, n2);
                if (d0 != 0.0f) { vreg = fmaf(y0n, d0, vreg); if (VW == 2) vregh = fmaf(g0n, d0, vregh); }
                if (d1 != 0.0f) { vreg = fmaf(y1n, d1, vreg); if (VW == 2) vregh = fmaf(g1n, d1, vregh); }
                if (d2 != 0.0f) { vreg = fmaf(y2n, d2, vreg); if (VW == 2) vregh = fmaf(g2n, d2, vregh); }
            }
            // free passes: row rr = lane / 16 takes the pass's contact rr, its lane t < 12 the coordinate t of the
            // contact's compact row (object slot t / 6, entry t % 6). The generalized velocity goes through LDS for the
            // passes (contacts of one pass share no object, so their lanes read and write disjoint coordinates)
            if (npass > 0) {
                if (lane < NV) sv[lane] = vreg;
                if (VW == 2 && lane + 64 < NV) sv[lane + 64] = vregh;
                wsync();
                const int rr = lane >> 4, t = lane & 15;
#pragma unroll 1
                for (int pp = 0; pp < npass; pp++) {
                    uint32_t lo, hi;
                    if (CAP * NCH <= 64 || pp < 64) {
                        lo = __builtin_amdgcn_readlane(plo, pp);
                        hi = __builtin_amdgcn_readlane(phi, pp);
                    } else {
                        lo = __builtin_amdgcn_readlane(plo2, pp - 64);
                        hi = __builtin_amdgcn_readlane(phi2, pp - 64);
                    }
                    uint32_t fld = ((rr < 2 ? lo : hi) >> (16 * (rr & 1))) & 0xFFFFu;
                    int ci = (int)(fld & 0xFFu);
                    bool act = ci != 0xFF;
                    int idx = -1;
                    float x0 = 0.0f, x1 = 0.0f, x2 = 0.0f, y0 = 0.0f, y1 = 0.0f, y2 = 0.0f, vv = 0.0f;
                    if (act && t < 12) {
                        int o = (int)(t < 6 ? (fld >> 8) & 0xFu : fld >> 12) - 1;
                        if (o >= 0) {
                            idx = D + 6 * o + (t < 6 ? t : t - 6);
                            float j0, j1, j2;
                            if constexpr (PC::ovf) {            // chunk 0's object rows, in LDS
                                auto Jl = lds_f<true>(Ob + 3 * ci * OW);
                                auto Yl = lds_f<true>(ObY + 3 * ci * OW);
                                j0 = Jl[t]; j1 = Jl[OW + t]; j2 = Jl[2 * OW + t];
                                y0 = Yl[t]; y1 = Yl[OW + t]; y2 = Yl[2 * OW + t];
                            } else {                            // the env's global row area
                                auto Jg = glb_f<true>(orow_g(3 * ci, false));
                                auto Yg = glb_f<true>(orow_g(3 * ci, true));
                                j0 = Jg[t]; j1 = Jg[OW + t]; j2 = Jg[2 * OW + t];
                                y0 = Yg[t]; y1 = Yg[OW + t]; y2 = Yg[2 * OW + t];
                            }
                            vv = sv[idx];
                            x0 = j0 * vv; x1 = j1 * vv; x2 = j2 * vv;
                        }
                    }
                    row_sum3(x0, x1, x2);
                    if (act) {
                        float K[11], n0, n1, n2, d0, d1, d2;
                        consts(ci, K);
                        block(K, x0, x1, x2, n0, n1, n2, d0, d1, d2);
                        if (idx >= 0) {
                            if (d0 != 0.0f) vv = fmaf(y0, d0, vv);
                            if (d1 != 0.0f) vv = fmaf(y1, d1, vv);
                            if (d2 != 0.0f) vv = fmaf(y2, d2, vv);
                            sv[idx] = vv;
                        }
                        if (t == 0) put_lams(ci, n0, n1, n2);
                    }
                    wsync();
                }
                vreg = lane < NV ? sv[lane] : 0.0f;
                vregh = (VW == 2 && lane + 64 < NV) ? sv[lane + 64] : 0.0f;
                wsync();
            }
        } else {
        if (nc > 0) { fetch(0); advance(); }
        if (nc > 1) fetch(1);
#pragma unroll 1
        for (int ch = 0; ch < NCH; ch++) {
            int cend = nc < CAP * (ch + 1) ? nc : CAP * (ch + 1);
            if (NCH > 1) {
                if (CAP * ch >= nc) break;
                if (multi && (nca > 1 || it == 0)) {
                    // this chunk's row constants from the staging registers; the next chunk's (or the next
                    // iteration's chunk 0, whose impulses were stored at its end) are loaded now, under this chunk.
                    // One chunk in use (nca == 1): its constants stay in registers after the first iteration
                    klam = sl; kvt = svt; kwinv = swinv; kcmu = scmu; kca0 = sca0; kca1 = sca1;
                    int nx = (ch + 1 < NCH && CAP * (ch + 1) < nc) ? ch + 1 : 0;
                    if (nca > 1 && lane < RPC) stage(nx);
                }
            }
            for (int ci = CAP * ch; ci < cend; ci++) {
                int r0 = 3 * (ci - CAP * ch);       // row of this contact within the chunk (= its lane)
                float j0 = j0n, j1 = j1n, j2 = j2n, y0 = y0n, y1 = y1n, y2 = y2n;
                float h0 = h0n, h1 = h1n, h2 = h2n, g0 = g0n, g1 = g1n, g2 = g2n;
                advance();
                if (ci + 2 < nc) fetch(ci + 2);
                float jv0 = j0 * vreg, jv1 = j1 * vreg, jv2 = j2 * vreg;
                if (VW == 2) {
                    jv0 = jv0 + h0 * vregh;
                    jv1 = jv1 + h1 * vregh;
                    jv2 = jv2 + h2 * vregh;
                }
                wave_sum_rows3(jv0, jv1, jv2);
                // the block's three rows live in lanes r0, r0 + 1, r0 + 2: each lane evaluates its own row with
                // its own lambda and constants (the oracle's operands) and only n0, d0, d1, d2 cross lanes
                float lm = klam;
                float n0 = lm - (jv0 - kvt) * kwinv;
                n0 = n0 < 0.0f ? 0.0f : (n0 > 3.0e38f ? 3.0e38f : n0);
                float d0 = bcast(n0 - lm, r0);
                n0 = bcast(n0, r0);
                float hi = kcmu * n0;
                float n1 = lm - (fmaf(kca0, d0, jv1) - kvt) * kwinv;
                n1 = n1 < -hi ? -hi : (n1 > hi ? hi : n1);
                float d1 = bcast(n1 - lm, r0 + 1);
                float n2 = lm - (fmaf(kca1, d1, fmaf(kca0, d0, jv2)) - kvt) * kwinv;
                n2 = n2 < -hi ? -hi : (n2 > hi ? hi : n2);
                float d2 = bcast(n2 - lm, r0 + 2);
                if (lane == r0) klam = n0;
                if (lane == r0 + 1) klam = n1;
                if (lane == r0 + 2) klam = n2;
                if (d0 != 0.0f) { vreg = fmaf(y0, d0, vreg); if (VW == 2) vregh = fmaf(g0, d0, vregh); }
                if (d1 != 0.0f) { vreg = fmaf(y1, d1, vreg); if (VW == 2) vregh = fmaf(g1, d1, vregh); }
                if (d2 != 0.0f) { vreg = fmaf(y2, d2, vreg); if (VW == 2) vregh = fmaf(g2, d2, vregh); }
            }
            if (multi && lane < RPC) rk(0, RPC * ch + lane) = klam;     // swap the impulses out
        }
        }
    }
    // impulse of global row RPC ch + lane (xfer sits before RK / PK in the union: no overlap)
    if (packed) {
        for (int r = lane; r < nr; r += 64) s.u.xfer[r] = ((HA_AS_LDS float*)PK)[HA_PK * (r / 3) + r % 3];
    } else if (!multi) {
        if (lane < RPC) s.u.xfer[lane] = klam;
    } else {
#pragma unroll 1
        for (int ch = 0; ch < NCH; ch++)
            if (lane < RPC && CAP * ch < nc) s.u.xfer[RPC * ch + lane] = rk(0, RPC * ch + lane);
    }
    if (lane < D) s.u.pd.dforce[lane] = (((dlam + lam_lo) - lam_up) + lam_fr) / hdt;
    wsync();
    if (lane < NV) s.v[lane] = vreg;
    if (VW == 2 && lane + 64 < NV) s.v[lane + 64] = vregh;
    PROF(6);
    // contact forces (last substep wins, like the oracle)
    if (lane == 0) {
        for (int b = 0; b < MAXB; b++) s.u.pd.cforce[b][0] = s.u.pd.cforce[b][1] = s.u.pd.cforce[b][2] = 0.f;
        for (int ci = 0; ci < nc; ci++) {
            int r0 = 3 * ci;
            const ContactLDS ct = ct_get(c, ci);
            f3 n = ld3(ct.n), t1, t2;
            tangents(n, t1, t2);
            f3 f = (n * s.u.xfer[r0] + t1 * s.u.xfer[r0 + 1]) + t2 * s.u.xfer[r0 + 2];
            f = f * (1.0f / hdt);
            int bodies[2] = {ct.a, ct.b};
            for (int sd = 0; sd < 2; sd++) {
                int bd = bodies[sd];
                float sg = sd == 0 ? 1.0f : -1.0f;
                int idx = -1;
                if (bd >= 100) idx = m.body_robot0 + (bd - 100);
                else if (bd >= 0) idx = m.body_object0 + bd;
                if (idx < 0) continue;
                s.u.pd.cforce[idx][0] += sg * f.x; s.u.pd.cforce[idx][1] += sg * f.y; s.u.pd.cforce[idx][2] += sg * f.z;
            }
        }
    }
    wsync();
    // ---- integrate
    if (lane < D) {
        float vv = s.v[lane];
        s.qd[lane] = vv;
        s.q[lane] += hdt * vv;
    }
    if (lane < NO) {
        int o = lane;
        const float* vo = s.v + D + 6 * o;
        f3 lv = mk3(vo[0], vo[1], vo[2]), av = mk3(vo[3], vo[4], vo[5]);
        st3(c.o[o].ov, lv);
        st3(c.o[o].ow, av);
        st3(c.o[o].oc, ld3(c.o[o].oc) + lv * hdt);
        qf q = ldq(c.o[o].oq);
        qf dq = qmul(qf{av.x, av.y, av.z, 0.0f}, q);
        stq(c.o[o].oq, qnormalize(qf{q.x + 0.5f * hdt * dq.x, q.y + 0.5f * hdt * dq.y, q.z + 0.5f * hdt * dq.z,
                                   q.w + 0.5f * hdt * dq.w}));
    }
    wsync();
    PROF(7);
}
