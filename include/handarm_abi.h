/*
 * handarm_abi.h - C ABI of the MI355X hand-arm simulator (libhandarm_hip.so).
 *
 * This is the drop-in boundary for the reference's LOWER surface, the Isaac Gym tensor API that
 * the hand_arm task code calls, plus one fused entry point that runs the task's
 * whole VecTask.step() on the device.  Plain pointers and sizes only; all device pointers are HIP
 * device memory (allocated by the caller, e.g. torch); every call is asynchronous on `stream`
 * (a hipStream_t passed as void*; NULL = default stream) and single-threaded per handle.
 * Every function returns 0 on success or a negative HA_E_* code.
 *
 * Reference call each entry point replaces (file:line under /root/reference/isaacgymenvs):
 *   ha_create / ha_bind_state      gym.create_sim + prepare_sim + acquire_*_tensor + wrap_tensor
 *                                  (tasks/base/vec_task.py:58-64,288; hand_arm/base/observable_vec_task.py:123-155)
 *   ha_simulate                    gym.simulate (vec_task.py:412; multi_object_manipulation.py:67,124,139,172)
 *   ha_simulate_envs               gym.simulate of _drop_objects (multi_object_manipulation.py:124), stepping only
 *                                  the envs that still have an object to drop
 *   ha_refresh                     gym.refresh_{dof_state,actor_root_state,rigid_body_state,net_contact_force}_tensor
 *                                  (observable_vec_task.py:173-177)
 *   ha_set_dof_position_target     gym.set_dof_position_target_tensor (hand_arm/base/actionable_vec_task.py:39-40)
 *   ha_set_actor_root_state_indexed   gym.set_actor_root_state_tensor_indexed (multi_object_manipulation.py:89,118,167,228)
 *   ha_set_dof_state_indexed          gym.set_dof_state_tensor_indexed (hand_arm/base/ur5sih.py:630)
 *   ha_set_dof_position_target_indexed gym.set_dof_position_target_tensor_indexed (ur5sih.py:626)
 *   ha_set_object_collision_filter gym.set_actor_rigid_shape_properties(filter) loop (multi_object.py:693-703)
 *   ha_task_step                   VecTask.step for Ur5SihMultiObjectManipulation, fused
 *                                  (vec_task.py:390-441 -> configurable_vec_task.py:347-414)
 *   ha_task_observe                post_step callbacks + compute_reward + compute_observations alone
 *   ha_task_reset                  reset_idx steady state (multi_object_manipulation.py:33-71)
 *   ha_task_epilogue               VecTask.step's torch.clamp(obs_buf) and the AllegroKuka extras means
 *                                  (vec_task.py:437, allegro_kuka_base.py:908-917)
 *   ha_task_step_io                VecTask.step whole for the Allegro tasks: the action clamp (vec_task.py:400-404),
 *                                  the fused step and the epilogue's outputs, in ONE launch
 *   ha_pointclouds                 synthetic point-cloud observables' post_step refresh
 *                                  (multi_object.py:792-809, ur5sih.py:361-374)
 *   ha_gather_obs                  compute_observations' torch.cat for a custom observation list
 *                                  (observable_vec_task.py:183-203)
 *   ha_render_camera               render_all_camera_sensors + camera image refresh (utils/camera.py:278-311)
 * The fused entry points serve three tasks (ha_params_t.task): Ur5Sih (above), AllegroHand
 * (allegro_hand.py:586-633) and AllegroKuka (allegro_kuka_base.py:1355-1447).
 */
#ifndef HANDARM_ABI_H
#define HANDARM_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HA_ABI_VERSION 16

/* capacities of the static model */
#define HA_MAX_LINKS 32
#define HA_MAX_DOFS 24
#define HA_MAX_HULLS 128    /* v13: 128 (the concave YCB objects' convex pieces) */
#define HA_MAX_VERTS 8192
#define HA_MAX_PLANES 16384
#define HA_MAX_EDGES 16384     /* hull edges, all hulls (v10) */
#define HA_MAX_LOOP 32768      /* face-loop entries, all hulls (v10): 2 per edge (16-bit loop starts) */
#define HA_MAX_FACE_LOOP 21    /* vertices of one face loop (v10): a clipped manifold's 2 x 21 + 21 candidates fit a wave */
#define HA_MAX_POOL 32
#define HA_MAX_OBJ 8           /* objects per env: 3 in Ur5SihMultiObject.yaml:2, 8 for bin-picking (config 5) */
#define HA_MAX_STATIC 16       /* static hulls per env (table, table-with-hole walls + bin pieces, v14: the throw bucket) */
#define HA_MAX_FIXED_BODIES 8  /* fixed rigid bodies with a model pose (table-with-hole links, bin) */
#define HA_MAX_CONTACTS 84     /* contacts per env and substep: 21 (<= 3 objects), 84 (clutter, > 3 objects) */
#define HA_MAX_INIT_POSES 4    /* objects.drop.num_initial_poses */
#define HA_MAX_SPLINE_PIECES 8
#define HA_N_SPLINES 8
#define HA_MAX_MPAIRS 192
#define HA_MAX_SELF_PAIRS 512  /* robot link-hull pairs tested for self-collision (v12) */
#define HA_DRAW_STRIDE 80     /* floats of reset_draws per env (replayed host RNG draws) */
/* v13: persistent contact manifolds (ha_state_t.contact_cache): one record of HA_PCM_REC floats per candidate pair
 * slot of an env. Record: [0..2] the pair's relative position (side A's body origin in side B's body frame) when the
 * manifold was built, [3] its point count k (0 = empty), [4..7] the relative rotation conj(q_B) q_A (xyzw), then per
 * point t < k at 8 + 9 t: the point on A in A's frame (3), the point on B in B's frame (3), the normal in B's frame (3) */
#define HA_PCM_REC 48
#define HA_CSTAT 8             /* ha_state_t.contact_stats columns (v13: 8, was 4) */
/* per-env domain-randomization samples (ha_state_t.dr_scale rows): the actor properties of the env as
 * apply_randomizations last set them (tasks/base/vec_task.py:788-864). Rows hold the nominal values until an env's
 * first sample (handarm_hip/dr.py default_rows). */
#define HA_DR_LINK_MASS 0      /* [HA_MAX_LINKS] robot link mass (and inertia) scale: new mass / nominal mass */
#define HA_DR_OBJ_MASS 32      /* [HA_MAX_OBJ] object mass (and inertia) scale */
#define HA_DR_LINK_FRIC 40     /* [HA_MAX_LINKS] robot link friction */
#define HA_DR_OBJ_FRIC 72      /* [HA_MAX_OBJ] object friction */
#define HA_DR_DOF_KP 80        /* [HA_MAX_DOFS] v16: drive stiffness (dof_properties stiffness) */
#define HA_DR_DOF_KD 104       /* [HA_MAX_DOFS] v16: drive damping (dof_properties damping) */
#define HA_DR_DOF_LOWER 128    /* [HA_MAX_DOFS] v16: joint lower limit the physics enforces (dof_properties lower) */
#define HA_DR_DOF_UPPER 152    /* [HA_MAX_DOFS] v16: joint upper limit (dof_properties upper) */
#define HA_DR_OBJ_SCALE 176    /* [HA_MAX_OBJ] v16: object actor scale (set_actor_scale; geometry x s, mass x s^3) */
#define HA_DR_SIZE 184

/* v16: schema-driven domain randomization (task.randomization_params, vec_task.py:646-876, dr_utils.py:71-238).
 * One ha_dr_attr_t per randomized quantity, ha_params_t.dr_attr[HA_DRA_*]; dist 0 = not randomized. */
#define HA_DRA_OBS 0           /* observations: noise on obs_buf after post_physics_step (vec_task.py:426-428) */
#define HA_DRA_ACT 1           /* actions: noise before the action clamp (vec_task.py:400-402) */
#define HA_DRA_GRAVITY 2       /* sim_params gravity (dr_utils.py:163-173), one value for the shard */
#define HA_DRA_LINK_MASS 3     /* robot actor rigid_body_properties mass (per link) */
#define HA_DRA_LINK_FRIC 4     /* robot actor rigid_shape_properties friction (per link: its shapes share one draw) */
#define HA_DRA_DOF_KD 5        /* robot actor dof_properties damping (per DOF) */
#define HA_DRA_DOF_KP 6        /* robot actor dof_properties stiffness (per DOF) */
#define HA_DRA_DOF_LOWER 7     /* robot actor dof_properties lower (per DOF) */
#define HA_DRA_DOF_UPPER 8     /* robot actor dof_properties upper (per DOF) */
#define HA_DRA_OBJ_MASS 9      /* object actor rigid_body_properties mass */
#define HA_DRA_OBJ_FRIC 10     /* object actor rigid_shape_properties friction */
#define HA_DRA_OBJ_SCALE 11    /* object actor scale */
#define HA_DRA_N 12
#define HA_DR_DIST_OFF 0
#define HA_DR_DIST_UNIFORM 1
#define HA_DR_DIST_LOGUNIFORM 2
#define HA_DR_DIST_GAUSSIAN 3
#define HA_DR_OP_ADDITIVE 0
#define HA_DR_OP_SCALING 1
#define HA_DR_SCHED_NONE 0
#define HA_DR_SCHED_LINEAR 1   /* min(frame, schedule_steps) / schedule_steps */
#define HA_DR_SCHED_CONSTANT 2 /* 0 before schedule_steps frames, 1 after */
typedef struct ha_dr_attr_t {
    int32_t dist, op, sched, sched_steps;
    double range[2];           /* uniform / loguniform: lo, hi; gaussian: mu, sigma (np.random.normal(mu, var));
                                * python doubles, as the reference computes the schedules and samples in double */
    double range_corr[2];      /* observations / actions: range_correlated (default 0, 0) */
    int32_t num_buckets;       /* > 0: the value snaps to the bucket grid over `range` (get_bucketed_val) */
    int32_t setup_only;        /* sampled at the first randomization only */
    /* robot list properties (link mass / friction) when the object actor randomizes the same property after the robot:
     * apply_randomizations keeps ONE original_props entry per property name, written by every actor at the first
     * randomization (the object, processed last, wins; vec_task.py:828-832), so later randomizations zip the robot's
     * bodies with the object's one: only the first later_elems elements are re-sampled, from the object's nominal
     * value (later_og_object). later_elems -1: every element, from its own nominal value */
    int32_t later_elems;
    int32_t later_og_object;
} ha_dr_attr_t;

/* v16: the shard-wide randomization state (ha_state_t.dr_global, HA_DRG_SIZE floats; int fields as int32 bits), kept
 * by the launch that precedes every step (and reset) launch while dr_enable is on: gym.get_frame_count, last_rand_step,
 * first_randomization, and the non-env randomizations (noise parameters, gravity) of apply_randomizations. The host
 * writes it once (handarm_hip/dr.py init_global). */
#define HA_DRG_FRAME 0         /* int: gym frame count when this step's pre_physics_step runs (the schedules' clock) */
#define HA_DRG_FRAME_NEXT 1    /* int: frame count after this step's gym.simulate calls */
#define HA_DRG_LAST_RAND 2     /* int: last_rand_step (frame of the last non-env randomization; -1 none) */
#define HA_DRG_FIRST 3         /* int: 1 until the first apply_randomizations ran */
#define HA_DRG_ALL 4           /* int: this step's randomization is the first one: every env samples */
#define HA_DRG_STEP 5          /* int: step counter of the white noise */
#define HA_DRG_EPOCH 6         /* int: non-env randomizations so far (the correlated noise is redrawn at each) */
#define HA_DRG_VALID 7         /* int: dr_randomizations holds observations / actions (after the first one) */
#define HA_DRG_OBS 8           /* [4] observation noise: corr scale, corr offset, white scale, white offset */
#define HA_DRG_ACT 12          /* [4] action noise (current) */
#define HA_DRG_ACT_USE 16      /* [4] action noise this step's VecTask.step applies (before its apply_randomizations) */
#define HA_DRG_ACT_EPOCH 20    /* int: epoch of that action noise's correlated term */
#define HA_DRG_ACT_ON 21       /* int: this step's actions get noise */
#define HA_DRG_GRAVITY 24      /* [3] sim_params gravity (current) */
#define HA_DRG_GRAVITY_OG 27   /* [3] the gravity the samples apply to: the first randomization's result after it (the
                                * reference's original_props["sim_params"] holds the prop whose gravity that call
                                * rewrote in place, vec_task.py:760-766, dr_utils.py:163-173) */
#define HA_DRG_SIZE 32

/* tasks (ha_params_t.task) */
#define HA_TASK_UR5SIH 0        /* Ur5SihMultiObjectManipulation (tasks/hand_arm/task/multi_object_manipulation.py) */
#define HA_TASK_ALLEGRO_HAND 1  /* AllegroHand in-hand reorientation (tasks/allegro_hand.py) */
#define HA_TASK_ALLEGRO_KUKA 2  /* AllegroKuka regrasping / reorientation / throw (tasks/allegro_kuka/) */

/* AllegroKuka per-env task state (ha_state_t.task_state rows, floats; allegro_kuka_base.py:330-389) */
#define HA_AK_LIFTED 0          /* lifted_object (0/1) */
#define HA_AK_CLOSEST_KP 1      /* closest_keypoint_max_dist (-1 = unset) */
#define HA_AK_CLOSEST_FT 2      /* [4] closest_fingertip_dist */
#define HA_AK_FURTHEST 6        /* furthest_hand_dist */
#define HA_AK_NEAR_GOAL 7       /* near_goal_steps */
#define HA_AK_PREV_SUCC 8       /* prev_episode_successes */
#define HA_AK_TRUE_OBJ 9        /* true_objective */
#define HA_AK_PREV_TRUE_OBJ 10  /* prev_episode_true_objective */
#define HA_AK_FORCE_PROB 11     /* random_force_prob */
#define HA_AK_RB_FORCE 12       /* [3] rb_forces of the object (LOCAL_SPACE) */
#define HA_AK_RNG 15            /* per-env step counter of the device RNG (uint32 bits) */
#define HA_AK_REW_EP 16         /* [12] rewards_episode, in the reference's reward_keys order */
#define HA_AK_KP 32             /* [4][3] object_keypoint_offsets (static per env, host-computed) */
#define HA_AK_TS 48

/* error codes */
#define HA_OK 0
#define HA_E_ARG -1
#define HA_E_HIP -2
#define HA_E_STATE -3
#define HA_E_MODEL -4

/* ha_params_t.narrow_phase_flags */
#define HA_NP_NO_EDGE_AXES 1
#define HA_NP_NO_CLIP 2
#define HA_NP_NO_SPHERE_CULL 4

/* flags for ha_task_step / ha_simulate */
#define HA_FLAG_NO_PHYSICS 1u      /* skip physics substeps (task-math parity tests) */
#define HA_FLAG_REPLAY_DRAWS 2u    /* reset draws come from ha_state_t.reset_draws (host RNG replay) */
#define HA_FLAG_OBS_ONLY 4u        /* ha_task_observe: compute_observations only (VecTask.reset) */

/* Static scene model (built offline by tools/build_model.py, packed by handarm_hip/model.py). */
typedef struct ha_model_t {
    int32_t n_links, n_dofs, n_link_hulls, n_pool, n_hulls;
    int32_t link_parent[HA_MAX_LINKS];
    int32_t link_dof[HA_MAX_LINKS];             /* -1 = fixed joint */
    int32_t link_table_collide[HA_MAX_LINKS];   /* 1 = link hulls collide with table/ground */
    float link_origin_pos[HA_MAX_LINKS][3];     /* joint origin in parent frame */
    float link_origin_quat[HA_MAX_LINKS][4];    /* xyzw */
    float link_axis[HA_MAX_LINKS][3];           /* joint axis in joint frame */
    float link_mass[HA_MAX_LINKS];
    float link_com[HA_MAX_LINKS][3];            /* link frame */
    float link_inertia[HA_MAX_LINKS][9];        /* about COM, link frame, row-major */
    float dof_lower[HA_MAX_DOFS], dof_upper[HA_MAX_DOFS], dof_effort[HA_MAX_DOFS];
    float dof_kp[HA_MAX_DOFS], dof_kd[HA_MAX_DOFS];
    float base_pos[3], base_quat[4];
    /* convex hulls: [0, n_link_hulls) robot, then object pool hulls, then the table */
    int32_t hull_link[HA_MAX_HULLS];            /* owning robot link, or -1 */
    int32_t hull_vert_start[HA_MAX_HULLS], hull_nverts[HA_MAX_HULLS];
    int32_t hull_plane_start[HA_MAX_HULLS], hull_nplanes[HA_MAX_HULLS];
    float hull_center[HA_MAX_HULLS][3], hull_radius[HA_MAX_HULLS];
    float verts[HA_MAX_VERTS][4];               /* xyz, pad */
    float planes[HA_MAX_PLANES][4];             /* n.x + d <= 0 inside */
    /* object pool */
    int32_t pool_hull[HA_MAX_POOL];
    float pool_mass[HA_MAX_POOL], pool_com[HA_MAX_POOL][3], pool_inertia[HA_MAX_POOL][9];
    float pool_bbox_pos[HA_MAX_POOL][3], pool_bbox_quat[HA_MAX_POOL][4], pool_bbox_ext[HA_MAX_POOL][3];
    /* static geometry */
    int32_t table_hull;
    float table_pos[3], table_quat[4];
    /* derived topology (filled by the host packer) */
    int32_t link_level[HA_MAX_LINKS];           /* depth in the tree, root = 0 */
    int32_t max_level;
    int32_t dof_link[HA_MAX_DOFS];
    int32_t n_mpairs;                           /* (d, e) with e an ancestor-or-self DOF of d */
    int32_t mpair[HA_MAX_MPAIRS][2];
    float table_half[3];                        /* table box half extents (broad phase) */
    /* v2: joint armature (added to the joint-space inertia diagonal; PhysX use_physx_armature) */
    float dof_armature[HA_MAX_DOFS];
    /* v2: env layout of the gym tensors (actor / rigid-body creation order); -1 = absent */
    int32_t n_actors, actor_robot, actor_object0, actor_goal, actor_table;
    int32_t n_bodies, body_robot0, body_object0, body_goal, body_table;
    /* v4: static boxes, collided with the objects and (link_table_collide) the robot links; static 0 is the
     * table of table_* when there is one. Pairs are enumerated object by object (ground, statics, objects,
     * link hulls), then link hull by link hull over the statics. */
    int32_t n_static;
    int32_t static_hull[HA_MAX_STATIC];
    float static_pos[HA_MAX_STATIC][3], static_quat[HA_MAX_STATIC][4], static_half[HA_MAX_STATIC][3];
    /* v5: fixed rigid bodies whose rigid_body_state rows come from the model (world pose, zero velocity):
     * bodies [body_fixed0, body_fixed0 + n_fixed_bodies), e.g. the table-with-hole links and the bin
     * (multi_object.py:626-637). 0 = the table row copies the table actor's root state (earlier scenes). */
    int32_t n_fixed_bodies, body_fixed0;
    float body_fixed_pose[HA_MAX_FIXED_BODIES][7];
    /* v8: compound pool objects (convex pieces, like the reference's V-HACD, multi_object.py:37-43): pool
     * object i collides with hulls pool_hull[i] .. pool_hull[i] + pool_nhull[i] - 1; pool_center / pool_radius
     * (object frame) bound all of them (= the hull's own sphere for a one-hull object). Pairs with a compound
     * object run the narrow phase piece by piece (A's pieces outer, B's inner). */
    int32_t pool_nhull[HA_MAX_POOL];
    float pool_center[HA_MAX_POOL][3], pool_radius[HA_MAX_POOL];
    /* v10: hull topology (handarm_hip/model.py hull_topology, from each hull's convex-hull triangulation), for the
     * edge-edge SAT axes and the clipped face manifolds of the narrow phase.
     *   edges[hull_edge_start[h] + i] = v0 | v1 << 8 | f0 << 16 | f1 << 24: edge i of hull h, its hull-local
     *     vertices and the two faces (hull-local plane indices) it separates; v0 -> v1 runs counter-clockwise about
     *     f0's outward normal.
     *   plane_loop[p] = start | count << 16: the face of (global) plane p as a counter-clockwise loop (about its
     *     outward normal) of hull-local vertices loop_v[start .. start + count), count <= HA_MAX_FACE_LOOP. */
    int32_t hull_edge_start[HA_MAX_HULLS], hull_nedges[HA_MAX_HULLS];
    uint32_t edges[HA_MAX_EDGES];
    int32_t plane_loop[HA_MAX_PLANES];
    uint8_t loop_v[HA_MAX_LOOP];
    /* v10: joint friction coefficient per DOF (Isaac Gym DOF property "friction", a coefficient: the friction force is
     * the DOF force times it, docs/domain_randomization.md:197): a PGS row with target velocity 0 and
     * |impulse| <= dof_friction |drive + limit impulse of the DOF| (AllegroHand 0.01, allegro_hand.py:267; AllegroKuka
     * the URDF's <dynamics friction>, AllegroKuka.yaml:58 dofFriction -1; Ur5Sih 0 from its URDF) */
    float dof_friction[HA_MAX_DOFS];
    /* v12: self-collision of the robot's links. The Allegro families create the hand actor with collision filter -1
     * (allegro_hand.py:334-335, allegro_kuka_base.py:664: the asset's filters, which a URDF does not set), so PhysX
     * collides every link pair of the articulation except parent and child. self_pair[k] = hull a | hull b << 8
     * (link hulls of two such links, a < b), tested after the link-static pairs; hull_obb[h] = the link hull's
     * oriented box in the link frame (centre[3], half extents[3], quat[4] xyzw, pad[2]) for the mid-phase cull
     * (include/ha_obb.h). n_self_pairs = 0: no self-collision (Ur5Sih: filter 0b1, ur5sih.py:123-125).
     * A one-piece pool object's hull carries a box too: its bounding box in the body frame with the identity
     * orientation (scaled with the env's object_scale), for the broad phase's box cull of the Allegro families.
     * Each piece of a compound pool object (pool_nhull > 1) carries its fitted box (any orientation), for the
     * piece-pair cull of compound pairs (round 6, include/ha_obb.h ha_obb_pair_near; unscaled bodies only).
     * ha_create refuses a model whose link hulls, one-piece object hulls or compound pieces do not lie inside their
     * boxes. */
    int32_t n_self_pairs;
    uint16_t self_pair[HA_MAX_SELF_PAIRS];
    float hull_obb[HA_MAX_HULLS][12];
    /* v14: statics carried by a per-env fixed-base actor (the AllegroKuka throw bucket, allegro_kuka_throw.py:51-82,
     * moved by _reset_target :88-103). posed_actor = that actor's index in the env's root_state rows (-1: none); a
     * static with static_posed[k] != 0 sits at static_pos / static_quat in that actor's frame, so its world pose is
     * root_state[posed_actor] composed with it (p_actor + q_actor static_pos, q_actor static_quat), read at the
     * start of each launch and after a reset moves the actor. Its rigid-body row is the actor's root state
     * (body_goal / actor_goal name the actor's slot). */
    int32_t posed_actor;
    int32_t static_posed[HA_MAX_STATIC];
} ha_model_t;

/* Simulation + task parameters (Ur5SihBase.yaml, Ur5SihMultiObject*.yaml). */
typedef struct ha_params_t {
    float dt;                  /* sim dt, 1/60 */
    int32_t substeps;          /* 2 */
    int32_t control_freq_inv;  /* 3 */
    int32_t solver_iters;      /* position iterations, 8 */
    float gravity[3];
    float friction;            /* 1.0 */
    float contact_margin;      /* speculative contact distance */
    float baumgarte;           /* penetration correction per substep */
    float max_depen_vel;
    float object_ang_damping;  /* Isaac Gym asset default 0.5 */
    float joint_limit_margin;
    /* task */
    int32_t n_objects;         /* 3 */
    int32_t num_initial_poses; /* P */
    int32_t max_episode_length;/* 200 */
    float action_dt;           /* dt used by the UR5 relative controller (VecTask.dt = sim dt) */
    float sih_alpha;           /* 0.8 */
    float sih_beta;            /* 1 - alpha evaluated in double then rounded (python-float semantics) */
    float reward_reaching, reward_lifting, reward_goal, reward_success;
    float lifting_threshold, goal_threshold;
    float goal_pos[3], goal_noise[3];
    float reset_pose[HA_MAX_DOFS];
    float servo_lower[5], servo_upper[5];
    float proximal_coef[4];    /* thumb, index, middle, ring */
    int32_t spline_pieces[HA_N_SPLINES];
    /* [spline][field t0,a,b,two_c,three_d][piece] */
    float spline[HA_N_SPLINES][5][HA_MAX_SPLINE_PIECES];
    float thumb_opposition_gain;  /* -1.571 / 2675 */
    uint64_t seed;
    /* v2 */
    int32_t task;              /* HA_TASK_* */
    int32_t num_actions, num_obs;
    /* AllegroHand (cfg/task/AllegroHand.yaml:7-52, tasks/allegro_hand.py:44-80) */
    float ah_dist_reward_scale, ah_rot_reward_scale, ah_rot_eps, ah_action_penalty_scale;
    float ah_success_tolerance, ah_reach_goal_bonus, ah_fall_dist, ah_fall_penalty;
    int32_t ah_max_consecutive_successes;
    float ah_av_factor;
    float ah_reset_position_noise, ah_reset_dof_pos_noise, ah_reset_dof_vel_noise;
    float ah_act_moving_average;
    float ah_vel_obs_scale, ah_force_torque_obs_scale;
    float ah_object_init[7];   /* object start pose (pos, quat xyzw) */
    float ah_goal_init[3];     /* goal_init_state position (object start - 0.04 z) */
    float ah_goal_displacement[3];
    /* v2: domain randomization on (v16: schema-driven, dr_attr below). Contact friction = mean of the two bodies'
     * frictions (PhysX average combine); static geometry keeps `friction`. */
    int32_t dr_enable;                 /* v16: the schema of dr_attr / dr_frequency below */
    /* v3: AllegroKuka (cfg/task/AllegroKuka.yaml:9-94, env/regrasping.yaml, allegro_kuka_base.py:53-400) */
    int32_t ak_subtask;                /* 0 regrasping, 1 reorientation, 2 throw (v14) */
    int32_t ak_num_keypoints;          /* 1 (regrasping) or 4 */
    float ak_keypoints[4][3];          /* unit keypoint offsets (_object_keypoint_offsets) */
    float ak_object_base_size, ak_keypoint_scale;
    float ak_initial_tolerance, ak_target_tolerance;
    float ak_lifting_rew_scale, ak_lifting_bonus, ak_lifting_bonus_threshold;
    float ak_keypoint_rew_scale, ak_distance_delta_rew_scale, ak_reach_goal_bonus;
    float ak_kuka_actions_penalty_scale, ak_allegro_actions_penalty_scale;
    int32_t ak_success_steps, ak_max_consecutive_successes;
    float ak_bonus_rew;                /* reach_goal_bonus / success_steps (python float, rounded) */
    float ak_reset_noise[3];           /* resetPositionNoiseX/Y/Z */
    float ak_dof_noise_arm, ak_dof_noise_fingers, ak_dof_vel_noise;
    float ak_force_scale, ak_force_prob_lo, ak_force_prob_hi;
    float ak_force_decay_step;         /* force_decay ** (dt / force_decay_interval) in fp32 (torch.pow) */
    float ak_object_rb_mass;           /* object_rb_masses: env 0's object mass (allegro_kuka_base.py:734-735) */
    float ak_dof_speed_scale;          /* arm relative-target speed (dofSpeedScale) */
    float ak_act_moving_average, ak_one_minus_ama;
    float ak_clamp_abs_obs;
    float ak_object_init[3];           /* object_start_pose position (identity rotation) */
    float ak_goal_init[3];             /* reorientation goal start position */
    float ak_target_origin[3], ak_target_lo[3], ak_target_size[3];   /* target volume (min corner, size) */
    float ak_palm_offset[3];
    float ak_fingertip_offsets[4][3];
    int32_t ak_palm_link, ak_fingertip_links[4];
    int32_t ak_num_arm_dofs;           /* 7 */
    /* v9: resting-contact stability. Penetration up to contact_slop gets no Baumgarte push-out (the push-out
     * velocity is kept by the body, and re-adding it every substep rocks resting objects); a manifold's points
     * 2-4 are chosen only among candidates within manifold_window of its deepest point (speculative points
     * higher up a rounded side would otherwise displace the true support corners). */
    float contact_slop;                /* 0.001 m */
    float manifold_window;             /* 0.002 m */
    /* v10: robot link velocity damping (asset_options linear_damping / angular_damping: Ur5Sih 0.01 / 0.01,
     * ur5sih.py:178-179; AllegroKuka 0.01 / 0.01, allegro_kuka_base.py:565-566; AllegroHand 0 / 0.01,
     * allegro_hand.py:231), a damping wrench on every link's COM twist in the velocity-product forces */
    float link_lin_damping, link_ang_damping;
    /* v10: a hull pair's contact comes from its deepest edge-edge axis (one point at the edges' closest points)
     * when that axis separates by more than edge_rel_tol x the best face axis + edge_abs_tol, else from the
     * clipped face manifold (Gregorius, "The Separating Axis Test between Convex Polyhedra", GDC 2013) */
    float edge_rel_tol, edge_abs_tol;
    /* v10: narrow-phase switches (A/B timing, diagnostics; 0 = the full narrow phase): HA_NP_NO_EDGE_AXES skips
     * the edge-edge axes, HA_NP_NO_CLIP keeps a face manifold to its incident vertices (the v9 narrow phase) */
    int32_t narrow_phase_flags;
    /* v13: persistent contact manifolds (PhysX's persistent contact manifold, PCM; inferred: its source is closed). A
     * candidate pair whose relative pose moved less than pcm_lin_tol (m) and whose relative rotation stayed within
     * pcm_cos_tol (|dot| of the relative quaternions, cos of half the angle) of the pose its record was built at
     * reuses the record's points: each point's separation, position and normal are re-evaluated from the current
     * body poses (points separated by more than contact_margin are dropped), and the narrow phase does not run.
     * Otherwise the narrow phase runs and a pair that yields contacts rewrites its record. pcm_lin_tol <= 0 or a
     * null contact_cache: every candidate pair runs the narrow phase (the round-4 behaviour). */
    float pcm_lin_tol, pcm_cos_tol;
    /* v15: AllegroHand options (allegro_hand.py:66-121,406-504,602-616; cfg/task/AllegroHand.yaml observationType,
     * asymmetric_observations, useRelativeControl, dofSpeedScale) */
    int32_t ah_obs_type;               /* 0 "full_state" (88 floats), 1 "full" (72), 2 "full_no_vel" (50); = num_obs */
    int32_t ah_asymmetric;             /* compute_full_state(True): the 88-float state vector (dof forces included) goes
                                        * to teacher_obs ([N][88], VecTask's states_buf) as well */
    int32_t ah_relative_control;       /* targets = prev_targets + dofSpeedScale * dt * actions, clamped (no average) */
    float ah_speed_dt;                 /* shadow_hand_dof_speed_scale * dt: python double, rounded once */
    /* random object forces (forceScale > 0; allegro_hand.py:66-70,557-560,617-625): decay by ah_force_decay_step
     * (torch.pow(forceDecay, dt / forceDecayInterval) in fp32) each step, then with probability random_force_prob
     * (drawn log-uniformly in [lo, hi] at reset) a new force N(0, 1)^3 * mass * forceScale in the object frame, applied
     * to the first physics call of the step (an applied force lasts one gym.simulate). Per-env state in task_state
     * (AH_TS_* of ah_task.h) */
    float ah_force_scale, ah_force_prob_lo, ah_force_prob_hi, ah_force_decay_step;
    float ah_object_rb_mass;           /* object_rb_masses: the object's mass */
    int32_t ah_object_type;            /* objectType 0 block, 1 egg, 2 pen (allegro_hand.py:82-97; the pool entry of
                                        * the scene; pen: randomize_rotation_pen at reset, :542-546) */
    /* v16: task.randomization_params (vec_task.py:646-876): `frequency` (env steps between re-randomizations of an
     * env, and frames between non-env randomizations) and one spec per randomized quantity (HA_DRA_*) */
    int32_t dr_frequency;
    ha_dr_attr_t dr_attr[HA_DRA_N];
    /* v16: AllegroKuka privilegedActions (allegro_kuka_base.py:62-74,1359-1361,1417-1424): 3 leading actions are an
     * object torque x privilegedActionsTorque (ENV_SPACE, the step's physics call); num_actions = 26 */
    int32_t ak_privileged_actions;
    float ak_privileged_torque;
} ha_params_t;

/* Device buffers (caller-allocated). Layouts match the Isaac Gym tensors exactly. */
typedef struct ha_state_t {
    float* root_state;          /* [N][A=3+n_obj][13] pos, quat xyzw, linvel(COM), angvel */
    float* rigid_body_state;    /* [N][B=1+n_links+1+n_obj][13] */
    float* dof_state;           /* [N][D][2] pos, vel */
    float* net_contact_force;   /* [N][B][3] */
    float* sim_targets;         /* [N][D] position targets the physics sees */
    float* dof_position_targets;/* [N][D] task-side tensor (observed) */
    /* task */
    const float* actions;       /* [N][11] (ha_task_step_io stores the clamped caller actions here) */
    float* obs;                 /* [N][147] */
    float* teacher_obs;         /* [N][147] (AllegroHand with ah_asymmetric: [N][88], the states buffer) */
    float* rew;                 /* [N] */
    int64_t* reset_buf;         /* [N] */
    int64_t* progress_buf;      /* [N] */
    uint8_t* timeout_buf;       /* [N] bool */
    uint8_t* goal_reached_before; /* [N] bool */
    float* goal_pos;            /* [N][3] */
    int64_t* target_object_index;      /* [N] */
    int64_t* object_configuration_indices; /* [N] */
    int64_t* object_indices;    /* [N][n_obj] pool ids */
    float* object_pos_initial;  /* [N][P][n_obj][3] */
    float* object_quat_initial; /* [N][P][n_obj][4] */
    float* ur5_target;          /* [N][6] */
    float* servo;               /* [N][5] */
    float* smoothed;            /* [N][5] */
    float* obs_cache;           /* [N][n_obj][7] object pose seen by the previous observable refresh */
    float* reset_draws;         /* [N][HA_DRAW_STRIDE] replayed reset draws; Ur5Sih: cfg-draw, target-draw
                                 * (as float ints), goal u[3]; AllegroHand: see ah_task.h */
    uint32_t* episode;          /* [N] episode counter (device RNG stream) */
    int32_t* stats;             /* [S] per-step counters, see HA_STAT_* */
    float* term_sums;           /* [4] reward term sums for the step */
    int32_t* flags;             /* [4] device flags: [0] any env needs reset (written by the step kernel) */
    uint8_t* collision_enabled; /* [N][n_obj] object collision filter (drop init) */
    /* v2 */
    float* dof_force;           /* [N][D] joint force of the last substep (drive + limit impulses / h) */
    int64_t* reset_goal_buf;    /* [N] AllegroHand goal resets */
    float* successes;           /* [N] AllegroHand consecutive successes in the episode */
    float* goal_state;          /* [N][7] AllegroHand goal_states[:, 0:7] */
    float* consecutive_successes; /* [1] AllegroHand global average (device EWMA) */
    float* dr_scale;            /* [N][HA_DR_SIZE] per-env DR samples (read when dr_enable) */
    /* v3 */
    float* object_scale;        /* [N][n_obj][3] per-env object dimension scale of the pool hull (null = 1);
                                 * mass scales with the volume, inertia with the scaled second moments */
    float* object_force;        /* [N][n_obj][3] world force at the object COM for the next ha_simulate
                                 * (gym.apply_rigid_body_force_tensors; consumed, i.e. zeroed, by it). Since v15 it
                                 * acts on the FIRST of the n_calls gym.simulate calls of that ha_simulate only (an
                                 * applied force lasts one simulate; before v15 it acted on all n) */
    float* task_state;          /* [N][HA_AK_TS] AllegroKuka per-env task state */
    float* task_scalars;        /* [4] AllegroKuka host-curriculum scalars: success_tolerance,
                                 * tolerance objective, 1 if tolerance > target, keypoint success tolerance */
    /* v7 */
    int32_t* contact_stats;     /* [N][HA_CSTAT] contact-list diagnostics added up by every launch (null = off):
                                 * [0] substeps, [1] substeps whose pairs offered more contacts than the list holds
                                 * (the shallowest are dropped), [2] max contacts offered in one substep, [3] sum of
                                 * contacts offered, [4] sum of self-collision contacts offered (both bodies robot
                                 * links), [5] pair manifolds refreshed from their persistent record (v13),
                                 * [6] hull-pair narrow phases run (kernel diagnostics: exact culls such as the
                                 * separating-face record are not counted), [7] 0 */
    /* v13 */
    float* contact_cache;       /* [N][ha_contact_cache_slots][HA_PCM_REC] persistent contact manifolds (null = off);
                                 * zero-initialised by the caller; slot = the pair's index in the broad phase's
                                 * enumeration (objects: ground, statics, later objects, link hulls; then link hulls x
                                 * statics), then n_self_pairs self pairs. Keyed by relative pose: a caller that
                                 * changes an env's object geometry (object_indices, object_scale) zeroes its rows */
    /* v16 */
    float* dr_global;           /* [HA_DRG_SIZE] shard-wide randomization state (dr_enable; see HA_DRG_*) */
    int32_t* randomize_buf;     /* [N] steps since the env's actor properties were last randomized (vec_task.py:352) */
    float* object_torque;       /* [N][n_obj][3] world torque on the object for the next ha_simulate
                                 * (apply_rigid_body_force_tensors' torque tensor; consumed like object_force, on
                                 * the first of its n_calls calls; null = none) */
} ha_state_t;

/* stats layout (int32): [0] num_resets, [1] num_successes, then per pool object
 * [2 + 2*i] resets with pool object i as target, [3 + 2*i] successes */
#define HA_STAT_SIZE (2 + 2 * HA_MAX_POOL)

/* Synthetic point-cloud observables (SyntheticPointcloudObservable, hand_arm/utils/observables.py:199-216),
 * computed from the refreshed state tensors bound with ha_bind_state. Each output is optional (NULL = skip)
 * and is a dense float4 array (x, y, z, point type; utils/camera.py:43-47):
 *   object_pc      [N][n_obj][P][4]  object_synthetic_pointcloud (multi_object.py:792-800): pool-frame
 *                  samples posed by the object pose, padding points (w 0) zeroed, then the point axis
 *                  permuted by perm (torch.randperm(P), one permutation for every env and object)
 *   target_pc      [N][P][4]         target_object_synthetic_pointcloud (:802-804): the target object's
 *                  row of object_pc with w *= 2 (PointType.TARGET)
 *   robot_pc       [N][R][4]         ur5sih_synthetic_pointcloud (ur5sih.py:361-374): link-frame samples
 *                  posed by rigid_body_state rows robot_body[r], w from the sample (1)
 *   fingertip_pc   [N][5][4]         sih_fingertip_pointcloud (ur5sih.py:338-345): fingertip positions, w 3
 *   goal_pc        [N][1][4]         goal_synthetic_pointcloud (multi_object.py:383-389): goal_pos, w 3
 *   relative_goal_pc [N][1][4]       relative_goal_synthetic_pointcloud (:391-401, 806-809): goal_pos in
 *                  the flange frame, w 3
 * The object clouds pose their samples with object_pose rows when given ([N][n_obj][7]: the caller's snapshot
 * of the previous observable refresh, for observation lists whose post-step order puts the cloud before
 * object_pos, see handarm_hip/observables.py), else with this refresh's root_state rows. */
#define HA_PC_MAX_LINKS 32      /* robot bodies a point-cloud launch reads (staged per env in LDS) */
#define HA_PC_MAX_P 256         /* max_num_points per object cloud */
#define HA_PC_MAX_R 2048        /* robot cloud points */
typedef struct ha_pointcloud_t {
    const float* object_samples;   /* [n_pool][P][4] pool-frame surface samples, w 1 (valid) / 0 (padding) */
    const float* robot_samples;    /* [R][4] link-frame surface samples, w = point type */
    const int32_t* robot_slot;     /* [R] index into links[] of each robot sample's body */
    const int64_t* perm;           /* [P] object point permutation (torch.randperm output) */
    const float* object_pose;      /* [N][n_obj][7] object poses (pos, quat) to use, or NULL = root_state */
    float* object_pc;
    float* target_pc;
    float* robot_pc;
    float* fingertip_pc;
    float* goal_pc;
    float* relative_goal_pc;
    int32_t n_pool, P, R;
    int32_t n_links;               /* <= HA_PC_MAX_LINKS */
    int32_t links[HA_PC_MAX_LINKS];/* env-local rigid-body indices whose poses the clouds read */
    int32_t fingertip_slot[5];     /* links[] slots of the five fingertips (thumb, index, middle, ring, little) */
    int32_t flange_slot;           /* links[] slot of the UR5 flange */
} ha_pointcloud_t;

#define HA_MAX_OBS_SOURCES 8
/* ha_gather_obs: a column whose source index has this bit reads its source row at an extra offset of
 * target_object_index[env] * 13 floats (the target object's root-state row: target_object_* observables) */
#define HA_OBS_SRC_TARGET 16

/* Camera sensors (hand_arm/utils/camera.py:84-333; cameras of Ur5SihMultiObject.yaml:35-53). The camera looks along
 * its local +X axis with +Z up (Isaac Gym camera frame); images are [N][height][width] like the reference's
 * current_sensor_observation. Each output is optional (NULL = skip). */
#define HA_CAM_FROM_DEPTH 1u    /* ha_render_camera flag: skip ray casting, compute the point cloud from `depth` */
typedef struct ha_camera_t {
    float pos[3], quat[4];      /* camera pose in the env frame (xyzw) */
    float fovx_deg;             /* horizontal field of view (camera.py:144-153) */
    int32_t width, height;      /* resolution [width, height] (camera.py:179-185) */
    float max_depth;            /* 10: depth clamp and validity of the point cloud (camera.py:302-306) */
    float workspace[4];         /* x0, x1, y0, y1 of the point cloud's in-workspace test (camera.py:303-309) */
    float goal_radius;          /* goal sphere radius (rendered, collides with nothing) */
    int32_t static_seg[HA_MAX_STATIC]; /* segmentation id of each static box (table links 0, bin pieces 2) */
    float* depth;               /* [N][H][W] view-space z of the hit (negative), -inf where the ray hits nothing */
    int32_t* segmentation;      /* [N][H][W] segmentation id of the hit actor (table 0, robot 1, bin 2, object i
                                 * 3 + i, goal 3 + n_obj; 0 on a miss) */
    float* pointcloud;          /* [N][H][W][4] xyz in the env frame + validity (depth_image_to_global_points) */
    float* target_pc;           /* [N][P][4] {camera}_target_object_pointcloud (multi_object.py:837-855): the target
                                 * object's points (segmentation 3 + target index); needs segmentation and pointcloud */
    int32_t target_points;      /* P = pointclouds.max_num_points */
    uint32_t rng_counter;       /* per-call counter of the random subset when more than P points are on the target */
} ha_camera_t;

typedef struct ha_handle_s* ha_handle;

int ha_abi_version(void);
/* sizeof the three structs as compiled into the library (host-side mirror check) */
int ha_struct_sizes(int32_t* model_size, int32_t* params_size, int32_t* state_size);
/* HA_E_MODEL when the model exceeds what the task's kernel family is compiled for: DOF count, links, bodies, hulls
 * larger than the family's narrow-phase scratch, pool size, and (AllegroKuka) pool objects of more than one hull */
int ha_create(const ha_model_t* model, const ha_params_t* params, int32_t num_envs, ha_handle* out);
int ha_destroy(ha_handle h);
int ha_bind_state(ha_handle h, const ha_state_t* state);
/* gym-style tensor API */
int ha_simulate(ha_handle h, int32_t n_calls, uint32_t flags, void* stream);
/* v9: ha_simulate for a subset of envs (device array of n_envs distinct env indices; the other envs do not move).
 * The drop initialisation's later rounds step only the envs that still have an object to drop. */
int ha_simulate_envs(ha_handle h, int32_t n_calls, uint32_t flags, const int32_t* env_ids, int32_t n_envs,
                     void* stream);
int ha_refresh(ha_handle h, void* stream);
int ha_set_dof_position_target(ha_handle h, const float* targets, void* stream);
int ha_set_actor_root_state_indexed(ha_handle h, const float* root_state, const int32_t* actor_indices,
                                    int32_t n, void* stream);
int ha_set_dof_state_indexed(ha_handle h, const float* dof_state, const int32_t* actor_indices, int32_t n,
                             void* stream);
int ha_set_dof_position_target_indexed(ha_handle h, const float* targets, const int32_t* actor_indices,
                                       int32_t n, void* stream);
int ha_set_object_collision_filter(ha_handle h, const uint8_t* enabled, void* stream);
/* fused task entry points */
/* per-step log counters go to slot (step_counter % n_slots) of stats[n_slots][HA_STAT_SIZE] and
 * term_sums[n_slots][4]. Each step launch clears the NEXT step's slot, so a written slot must be read within
 * n_slots - 1 steps. n_slots >= 2; setting the ring clears it. */
int ha_set_stats_ring(ha_handle h, int32_t n_slots);
int ha_task_step(ha_handle h, uint32_t flags, void* stream);
int ha_task_observe(ha_handle h, uint32_t flags, void* stream);
int ha_task_reset(ha_handle h, uint32_t flags, void* stream);
/* VecTask.step's tail in one launch (vec_task.py:437, allegro_kuka_base.py:908-917): obs_out (if non-null,
 * N x num_obs floats) = clamp(obs, -clip_obs, clip_obs); AllegroKuka only: scalars (if non-null, 4 floats) =
 * mean prev_episode_successes, mean / min / max true_objective over the shard. */
int ha_task_epilogue(ha_handle h, float* obs_out, float clip_obs, float* scalars, void* stream);
/* ha_task_step with VecTask.step's head and tail inside the same launch (AllegroHand / AllegroKuka handles; HA_E_ARG
 * otherwise): actions (if non-null, N x num_actions floats, the caller's raw actions) are clamped to
 * +-clip_actions where the task reads them and stored clamped into the bound actions tensor (vec_task.py:400-404);
 * obs_out and scalars as ha_task_epilogue (scalars: AllegroKuka only; reduced in a fixed order by the launch's last
 * workgroups, so the values are deterministic but may differ from ha_task_epilogue's in the last bits). */
int ha_task_step_io(ha_handle h, uint32_t flags, const float* actions, float clip_actions, float* obs_out,
                    float clip_obs, float* scalars, void* stream);
/* v9: contacts per substep the handle's kernel family holds (over it, the shallowest give way) */
int ha_contact_capacity(ha_handle h);
/* v13: persistent-manifold record slots per env (ha_state_t.contact_cache rows of HA_PCM_REC floats) */
int ha_contact_cache_slots(ha_handle h);
/* v11: dispatch order of the full-shard launches (no gym counterpart: a scheduling hint; results do not depend on
 * it). order: device array of the N env indices, a permutation, that workgroup i of every later full-shard launch
 * simulates (kept by pointer: the caller keeps it alive), or NULL for the identity. Envs expected to take longest
 * first shortens a multi-round launch's tail (longest-processing-time order; handarm_hip/sim.py rebalance). */
int ha_set_env_order(ha_handle h, const int32_t* order, int32_t n);
/* v12: refresh a dispatch order in place on the device (one launch, no host sync): the envs that offered the most
 * contacts since the last refresh (contact_stats column 3 minus cost_prev[N], which is then updated) first; order[N]
 * is typically the array handed to ha_set_env_order. snake > 0 reverses every other block of `snake` positions */
int ha_update_env_order(ha_handle h, int32_t* order, int32_t* cost_prev, int32_t snake, void* stream);
/* v12: the cost that refresh sorts by: 0 the contacts each env offered since the last refresh (the handle's
 * default), 1 a running estimate of each env's workgroup span in the step launches (half the last span plus half the
 * previous estimate; the step kernels then stamp their start and end per launch slot). HandArmSim selects 1 */
int ha_set_order_cost(ha_handle h, int32_t mode);
/* time in ms of the most recent physics/step launch, from its HIP events; -1 when that launch was not timed (timing
 * off, or the ha_enable_kernel_timing record buffer full) or none ran */
float ha_last_kernel_ms(ha_handle h);
/* per-launch HIP-event timing of the env kernel (bench roofline): record up to max_launches launches
 * (0 disables); ha_kernel_times synchronises and returns the recorded durations in ms */
int ha_enable_kernel_timing(ha_handle h, int32_t max_launches);
int ha_kernel_times(ha_handle h, float* out_ms, int32_t max, int32_t* n_out);
/* Synthetic point clouds (see ha_pointcloud_t) for all envs in one launch: replaces the post_step callbacks
 * _refresh_object_synthetic_pointcloud / _refresh_target_object_synthetic_pointcloud (multi_object.py:792-804),
 * _refresh_ur5sih_synthetic_pointcloud (ur5sih.py:361-374) and the goal / fingertip cloud get_state lambdas.
 * Ur5Sih task only. If timing is enabled (ha_enable_kernel_timing) its launches are recorded separately
 * (ha_pointcloud_times). */
int ha_pointclouds(ha_handle h, const ha_pointcloud_t* pc, void* stream);
int ha_pointcloud_times(ha_handle h, float* out_ms, int32_t max, int32_t* n_out);
/* Observation vector of a custom observation list (observable_vec_task.py:183-192): out[N][n_cols], column k
 * = sources[cols[2k]][env * strides[cols[2k]] + cols[2k+1]]. sources / strides are host arrays of n_sources
 * (<= HA_MAX_OBS_SOURCES) device pointers / row strides in floats; cols is a device int32 array. */
int ha_gather_obs(ha_handle h, const float* const* sources, const int32_t* strides, int32_t n_sources,
                  const int32_t* cols, int32_t n_cols, float* out, void* stream);
/* One camera for all envs (render_all_camera_sensors + refresh_{depth,segmentation,pointcloud}, camera.py:278-311):
 * depth and segmentation by ray casting the collision geometry of the bound state, then the point cloud.
 * view_inv: the inverse view matrix (row-vector convention, 16 floats, host memory) the point cloud uses, as
 * camera.py:68 multiplies by view_mat.inverse(). Ur5Sih task only. */
int ha_render_camera(ha_handle h, const ha_camera_t* cam, const float* view_inv, uint32_t flags, void* stream);

#ifdef __cplusplus
}
#endif
#endif
