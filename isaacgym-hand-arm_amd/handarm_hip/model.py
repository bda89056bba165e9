"""Host-side model packing: scene JSON + task config -> the C-ABI structs of include/handarm_abi.h.

The ctypes classes below mirror ``ha_model_t`` / ``ha_params_t`` / ``ha_state_t`` field for field;
``tests/test_abi.py`` checks their sizes against the compiled libraries (``ha_struct_sizes``).
Config values and their reference sources:
  sim:    dt 1/60, substeps 2, position iterations 8      (cfg/task/Ur5SihBase.yaml:27-31)
  task:   controlFrequencyInv 3, episode length 200, reward scales, thresholds
          (cfg/task/Ur5SihMultiObjectManipulation.yaml:21,55-74)
  env:    3 objects, drop/goal regions, table height 0.5   (cfg/task/Ur5SihMultiObject.yaml)
  robot:  reset pose, kp/kd                                 (cfg/task/Ur5SihBase.yaml:3-9)
  servo:  limits, spline knots, proximal coefficients       (tasks/hand_arm/base/ur5sih.py:437-456)
"""
import ctypes as C
import json
import os

import numpy as np

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "ur5sih_scene.json")
ALLEGRO_ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "allegro_hand_scene.json")
KUKA_ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "kuka_allegro_scene.json")
BIN_ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "ur5sih_bin_scene.json")

MAX_LINKS, MAX_DOFS, MAX_HULLS, MAX_VERTS, MAX_PLANES = 32, 24, 128, 8192, 16384
MAX_EDGES, MAX_LOOP, MAX_FACE_LOOP = 16384, 32768, 21
MAX_POOL, MAX_OBJ, MAX_INIT_POSES, MAX_SPLINE_PIECES, N_SPLINES = 32, 8, 4, 8, 8
MAX_STATIC = 16
MAX_FIXED_BODIES = 8
MAX_MPAIRS = 192
MAX_SELF_PAIRS = 512
STAT_SIZE = 2 + 2 * MAX_POOL
DRAW_STRIDE = 80
DR_SIZE = 184
DR_LINK_MASS, DR_OBJ_MASS, DR_LINK_FRIC, DR_OBJ_FRIC = 0, 32, 40, 72
DR_DOF_KP, DR_DOF_KD, DR_DOF_LOWER, DR_DOF_UPPER, DR_OBJ_SCALE = 80, 104, 128, 152, 176      # v16
# v16: randomized quantities (ha_params_t.dr_attr[HA_DRA_*]) and the shard-wide DR state (ha_state_t.dr_global)
DRA_OBS, DRA_ACT, DRA_GRAVITY, DRA_LINK_MASS, DRA_LINK_FRIC, DRA_DOF_KD, DRA_DOF_KP, DRA_DOF_LOWER, DRA_DOF_UPPER, \
    DRA_OBJ_MASS, DRA_OBJ_FRIC, DRA_OBJ_SCALE = range(12)
DRA_N = 12
DR_DIST = {"off": 0, "uniform": 1, "loguniform": 2, "gaussian": 3}
DR_OP = {"additive": 0, "scaling": 1}
DR_SCHED = {None: 0, "linear": 1, "constant": 2}
DRG_FRAME, DRG_FRAME_NEXT, DRG_LAST_RAND, DRG_FIRST, DRG_ALL, DRG_STEP, DRG_EPOCH, DRG_VALID = range(8)
DRG_OBS, DRG_ACT, DRG_ACT_USE, DRG_ACT_EPOCH, DRG_ACT_ON, DRG_GRAVITY, DRG_GRAVITY_OG = 8, 12, 16, 20, 21, 24, 27
DRG_SIZE = 32
TASK_UR5SIH, TASK_ALLEGRO_HAND, TASK_ALLEGRO_KUKA = 0, 1, 2
# AllegroKuka task_state row (HA_AK_* in handarm_abi.h)
AK_TS = 48
AK_LIFTED, AK_CLOSEST_KP, AK_CLOSEST_FT, AK_FURTHEST, AK_NEAR_GOAL = 0, 1, 2, 6, 7
AK_PREV_SUCC, AK_TRUE_OBJ, AK_PREV_TRUE_OBJ, AK_FORCE_PROB, AK_RB_FORCE, AK_RNG, AK_REW_EP, AK_KP = \
    8, 9, 10, 11, 12, 15, 16, 32
AK_REWARD_KEYS = ["raw_fingertip_delta_rew", "raw_hand_delta_penalty", "raw_lifting_rew", "raw_keypoint_rew",
                  "fingertip_delta_rew", "hand_delta_penalty", "lifting_rew", "lift_bonus_rew", "keypoint_rew",
                  "bonus_rew", "kuka_actions_penalty", "allegro_actions_penalty"]   # allegro_kuka_base.py:361-374

FLAG_NO_PHYSICS = 1
FLAG_REPLAY_DRAWS = 2
FLAG_OBS_ONLY = 4
NP_NO_EDGE_AXES, NP_NO_CLIP = 1, 2      # ha_params_t.narrow_phase_flags

f32, i32 = C.c_float, C.c_int32


class HaDrAttr(C.Structure):
    """ha_dr_attr_t (include/handarm_abi.h v16): one randomized quantity of task.randomization_params."""
    _fields_ = [("dist", i32), ("op", i32), ("sched", i32), ("sched_steps", i32), ("range", C.c_double * 2),
                ("range_corr", C.c_double * 2), ("num_buckets", i32), ("setup_only", i32), ("later_elems", i32),
                ("later_og_object", i32)]


def arr(t, *dims):
    for d in reversed(dims):
        t = t * d
    return t


class HaModel(C.Structure):
    _fields_ = [
        ("n_links", i32), ("n_dofs", i32), ("n_link_hulls", i32), ("n_pool", i32), ("n_hulls", i32),
        ("link_parent", arr(i32, MAX_LINKS)), ("link_dof", arr(i32, MAX_LINKS)),
        ("link_table_collide", arr(i32, MAX_LINKS)),
        ("link_origin_pos", arr(f32, MAX_LINKS, 3)), ("link_origin_quat", arr(f32, MAX_LINKS, 4)),
        ("link_axis", arr(f32, MAX_LINKS, 3)), ("link_mass", arr(f32, MAX_LINKS)),
        ("link_com", arr(f32, MAX_LINKS, 3)), ("link_inertia", arr(f32, MAX_LINKS, 9)),
        ("dof_lower", arr(f32, MAX_DOFS)), ("dof_upper", arr(f32, MAX_DOFS)), ("dof_effort", arr(f32, MAX_DOFS)),
        ("dof_kp", arr(f32, MAX_DOFS)), ("dof_kd", arr(f32, MAX_DOFS)),
        ("base_pos", arr(f32, 3)), ("base_quat", arr(f32, 4)),
        ("hull_link", arr(i32, MAX_HULLS)), ("hull_vert_start", arr(i32, MAX_HULLS)),
        ("hull_nverts", arr(i32, MAX_HULLS)), ("hull_plane_start", arr(i32, MAX_HULLS)),
        ("hull_nplanes", arr(i32, MAX_HULLS)), ("hull_center", arr(f32, MAX_HULLS, 3)),
        ("hull_radius", arr(f32, MAX_HULLS)),
        ("verts", arr(f32, MAX_VERTS, 4)), ("planes", arr(f32, MAX_PLANES, 4)),
        ("pool_hull", arr(i32, MAX_POOL)), ("pool_mass", arr(f32, MAX_POOL)), ("pool_com", arr(f32, MAX_POOL, 3)),
        ("pool_inertia", arr(f32, MAX_POOL, 9)), ("pool_bbox_pos", arr(f32, MAX_POOL, 3)),
        ("pool_bbox_quat", arr(f32, MAX_POOL, 4)), ("pool_bbox_ext", arr(f32, MAX_POOL, 3)),
        ("table_hull", i32), ("table_pos", arr(f32, 3)), ("table_quat", arr(f32, 4)),
        ("link_level", arr(i32, MAX_LINKS)), ("max_level", i32), ("dof_link", arr(i32, MAX_DOFS)),
        ("n_mpairs", i32), ("mpair", arr(i32, MAX_MPAIRS, 2)), ("table_half", arr(f32, 3)),
        ("dof_armature", arr(f32, MAX_DOFS)),
        ("n_actors", i32), ("actor_robot", i32), ("actor_object0", i32), ("actor_goal", i32), ("actor_table", i32),
        ("n_bodies", i32), ("body_robot0", i32), ("body_object0", i32), ("body_goal", i32), ("body_table", i32),
        ("n_static", i32), ("static_hull", arr(i32, MAX_STATIC)), ("static_pos", arr(f32, MAX_STATIC, 3)),
        ("static_quat", arr(f32, MAX_STATIC, 4)), ("static_half", arr(f32, MAX_STATIC, 3)),
        ("n_fixed_bodies", i32), ("body_fixed0", i32), ("body_fixed_pose", arr(f32, MAX_FIXED_BODIES, 7)),
        ("pool_nhull", arr(i32, MAX_POOL)), ("pool_center", arr(f32, MAX_POOL, 3)), ("pool_radius", arr(f32, MAX_POOL)),
        ("hull_edge_start", arr(i32, MAX_HULLS)), ("hull_nedges", arr(i32, MAX_HULLS)),          # v10
        ("edges", arr(C.c_uint32, MAX_EDGES)), ("plane_loop", arr(i32, MAX_PLANES)),
        ("loop_v", arr(C.c_uint8, MAX_LOOP)),
        ("dof_friction", arr(f32, MAX_DOFS)),
        ("n_self_pairs", i32), ("self_pair", arr(C.c_uint16, MAX_SELF_PAIRS)), ("hull_obb", arr(f32, MAX_HULLS, 12)),  # v12
        ("posed_actor", i32), ("static_posed", arr(i32, MAX_STATIC)),                                                 # v14
    ]


class HaParams(C.Structure):
    _fields_ = [
        ("dt", f32), ("substeps", i32), ("control_freq_inv", i32), ("solver_iters", i32),
        ("gravity", arr(f32, 3)), ("friction", f32), ("contact_margin", f32), ("baumgarte", f32),
        ("max_depen_vel", f32), ("object_ang_damping", f32), ("joint_limit_margin", f32),
        ("n_objects", i32), ("num_initial_poses", i32), ("max_episode_length", i32),
        ("action_dt", f32), ("sih_alpha", f32), ("sih_beta", f32),
        ("reward_reaching", f32), ("reward_lifting", f32), ("reward_goal", f32), ("reward_success", f32),
        ("lifting_threshold", f32), ("goal_threshold", f32),
        ("goal_pos", arr(f32, 3)), ("goal_noise", arr(f32, 3)), ("reset_pose", arr(f32, MAX_DOFS)),
        ("servo_lower", arr(f32, 5)), ("servo_upper", arr(f32, 5)), ("proximal_coef", arr(f32, 4)),
        ("spline_pieces", arr(i32, N_SPLINES)), ("spline", arr(f32, N_SPLINES, 5, MAX_SPLINE_PIECES)),
        ("thumb_opposition_gain", f32), ("seed", C.c_uint64),
        ("task", i32), ("num_actions", i32), ("num_obs", i32),
        ("ah_dist_reward_scale", f32), ("ah_rot_reward_scale", f32), ("ah_rot_eps", f32),
        ("ah_action_penalty_scale", f32), ("ah_success_tolerance", f32), ("ah_reach_goal_bonus", f32),
        ("ah_fall_dist", f32), ("ah_fall_penalty", f32), ("ah_max_consecutive_successes", i32), ("ah_av_factor", f32),
        ("ah_reset_position_noise", f32), ("ah_reset_dof_pos_noise", f32), ("ah_reset_dof_vel_noise", f32),
        ("ah_act_moving_average", f32), ("ah_vel_obs_scale", f32), ("ah_force_torque_obs_scale", f32),
        ("ah_object_init", arr(f32, 7)), ("ah_goal_init", arr(f32, 3)), ("ah_goal_displacement", arr(f32, 3)),
        ("dr_enable", i32),
        ("ak_subtask", i32), ("ak_num_keypoints", i32), ("ak_keypoints", arr(f32, 4, 3)),
        ("ak_object_base_size", f32), ("ak_keypoint_scale", f32), ("ak_initial_tolerance", f32),
        ("ak_target_tolerance", f32), ("ak_lifting_rew_scale", f32), ("ak_lifting_bonus", f32),
        ("ak_lifting_bonus_threshold", f32), ("ak_keypoint_rew_scale", f32), ("ak_distance_delta_rew_scale", f32),
        ("ak_reach_goal_bonus", f32), ("ak_kuka_actions_penalty_scale", f32), ("ak_allegro_actions_penalty_scale", f32),
        ("ak_success_steps", i32), ("ak_max_consecutive_successes", i32), ("ak_bonus_rew", f32),
        ("ak_reset_noise", arr(f32, 3)), ("ak_dof_noise_arm", f32), ("ak_dof_noise_fingers", f32),
        ("ak_dof_vel_noise", f32), ("ak_force_scale", f32), ("ak_force_prob_lo", f32), ("ak_force_prob_hi", f32),
        ("ak_force_decay_step", f32), ("ak_object_rb_mass", f32), ("ak_dof_speed_scale", f32),
        ("ak_act_moving_average", f32), ("ak_one_minus_ama", f32), ("ak_clamp_abs_obs", f32),
        ("ak_object_init", arr(f32, 3)), ("ak_goal_init", arr(f32, 3)), ("ak_target_origin", arr(f32, 3)),
        ("ak_target_lo", arr(f32, 3)), ("ak_target_size", arr(f32, 3)), ("ak_palm_offset", arr(f32, 3)),
        ("ak_fingertip_offsets", arr(f32, 4, 3)), ("ak_palm_link", i32), ("ak_fingertip_links", arr(i32, 4)),
        ("ak_num_arm_dofs", i32),
        ("contact_slop", f32), ("manifold_window", f32),                       # v9
        ("link_lin_damping", f32), ("link_ang_damping", f32), ("edge_rel_tol", f32), ("edge_abs_tol", f32),  # v10
        ("narrow_phase_flags", i32),
        ("pcm_lin_tol", f32), ("pcm_cos_tol", f32),                           # v13
        ("ah_obs_type", i32), ("ah_asymmetric", i32), ("ah_relative_control", i32), ("ah_speed_dt", f32),   # v15
        ("ah_force_scale", f32), ("ah_force_prob_lo", f32), ("ah_force_prob_hi", f32), ("ah_force_decay_step", f32),
        ("ah_object_rb_mass", f32), ("ah_object_type", i32),
        ("dr_frequency", i32), ("dr_attr", HaDrAttr * 12),                   # v16
        ("ak_privileged_actions", i32), ("ak_privileged_torque", f32),
    ]


P = C.c_void_p


STATE_FIELDS = ["root_state", "rigid_body_state", "dof_state", "net_contact_force", "sim_targets",
                "dof_position_targets", "actions", "obs", "teacher_obs", "rew", "reset_buf", "progress_buf",
                "timeout_buf", "goal_reached_before", "goal_pos", "target_object_index",
                "object_configuration_indices", "object_indices", "object_pos_initial", "object_quat_initial",
                "ur5_target", "servo", "smoothed", "obs_cache", "reset_draws", "episode", "stats", "term_sums",
                "flags", "collision_enabled", "dof_force", "reset_goal_buf", "successes", "goal_state",
                "consecutive_successes", "dr_scale", "object_scale", "object_force", "task_state", "task_scalars",
                "contact_stats", "contact_cache", "dr_global", "randomize_buf", "object_torque"]
PCM_REC = 48        # HA_PCM_REC: floats per persistent-manifold record (include/handarm_abi.h v13)
CSTAT = 8           # HA_CSTAT: contact_stats columns


# The committed Ur5Sih scene's object pools (tools/build_model.py): the 16 objects of rounds 1-4 (the reference's default
# set, Ur5SihMultiObject.yaml:11, plus 13 of its commented list, the mug decomposed), then the 8 clearly concave objects of
# that list as convex pieces (round 5, f1). POOL16 is the bench's C4 / C5 pool; POOL_WIDE = all 24
POOL16 = ["015_peach", "005_tomato_soup_can", "006_mustard_bottle", "004_sugar_box", "007_tuna_fish_can",
          "008_pudding_box", "009_gelatin_box", "010_potted_meat_can", "013_apple", "014_lemon", "016_pear", "017_orange",
          "018_plum", "025_mug", "061_foam_brick", "077_rubiks_cube"]
CONCAVE_POOL = ["031_spoon", "033_spatula", "037_scissors", "042_adjustable_wrench", "050_medium_clamp", "065-a_cups",
                "065-d_cups", "073-a_lego_duplo"]
POOL_WIDE = POOL16 + CONCAVE_POOL


def pcm_slots(model, n_obj, params=None):
    """Persistent-manifold record slots per env (ha_contact_cache_slots): the broad phase's pair enumeration (per object
    its ground, statics, later objects and link hulls; then link hulls x statics), then the self pairs; none when the
    params turn the records off (pcm_lin_tol 0: AllegroHand's default)."""
    if params is not None and params.pcm_lin_tol <= 0:
        return 0
    NS, NLH = model.n_static, model.n_link_hulls
    return sum(1 + NS + (n_obj - 1 - o) + NLH for o in range(n_obj)) + NLH * NS + model.n_self_pairs


_DEFAULT_SLOTS = {}


def default_pcm_slots(n_obj=3):
    """pcm_slots of the default Ur5Sih scene (state buffers sized without a model in hand)."""
    if n_obj not in _DEFAULT_SLOTS:
        _DEFAULT_SLOTS[n_obj] = pcm_slots(build_model(load_scene()), n_obj)
    return _DEFAULT_SLOTS[n_obj]


def state_spec(num_envs, n_links=29, n_dofs=17, n_obj=3, num_initial_poses=1, num_actions=11, num_obs=147,
               n_actors=None, n_bodies=None, n_pcm_slots=None, num_states=None):
    """name -> (shape, numpy dtype) of every ha_state_t buffer (Isaac Gym tensor layouts). n_pcm_slots: persistent-
    manifold slots per env (pcm_slots of the model; None: the default Ur5Sih scene's)."""
    if n_pcm_slots is None:
        n_pcm_slots = default_pcm_slots(n_obj)
    N, D, P = num_envs, n_dofs, num_initial_poses
    A = n_actors if n_actors is not None else 3 + n_obj
    B = n_bodies if n_bodies is not None else 1 + n_links + 1 + n_obj
    f, i64, u8, i32, u32 = np.float32, np.int64, np.uint8, np.int32, np.uint32
    return {
        "root_state": ((N * A, 13), f), "rigid_body_state": ((N * B, 13), f), "dof_state": ((N * D, 2), f),
        "net_contact_force": ((N * B, 3), f), "sim_targets": ((N, D), f), "dof_position_targets": ((N, D), f),
        "actions": ((N, num_actions), f), "obs": ((N, num_obs), f),
        "teacher_obs": ((N, num_states if num_states is not None else num_obs), f),
        "rew": ((N,), f), "reset_buf": ((N,), i64), "progress_buf": ((N,), i64), "timeout_buf": ((N,), u8),
        "goal_reached_before": ((N,), u8), "goal_pos": ((N, 3), f), "target_object_index": ((N,), i64),
        "object_configuration_indices": ((N,), i64), "object_indices": ((N, n_obj), i64),
        "object_pos_initial": ((N, P, n_obj, 3), f), "object_quat_initial": ((N, P, n_obj, 4), f),
        "ur5_target": ((N, 6), f), "servo": ((N, 5), f), "smoothed": ((N, 5), f), "obs_cache": ((N, n_obj, 7), f),
        "reset_draws": ((N, DRAW_STRIDE), f), "episode": ((N,), u32), "stats": ((STAT_SIZE,), i32),
        "term_sums": ((4,), f), "flags": ((4,), i32), "collision_enabled": ((N, n_obj), u8),
        "dof_force": ((N, D), f), "reset_goal_buf": ((N,), i64), "successes": ((N,), f), "goal_state": ((N, 7), f),
        "consecutive_successes": ((1,), f), "dr_scale": ((N, DR_SIZE), f),
        "object_scale": ((N, n_obj, 3), f), "object_force": ((N, n_obj, 3), f), "task_state": ((N, AK_TS), f),
        "task_scalars": ((4,), f), "contact_stats": ((N, CSTAT), i32),
        "contact_cache": ((N, n_pcm_slots, PCM_REC), f),
        "dr_global": ((DRG_SIZE,), f), "randomize_buf": ((N,), i32), "object_torque": ((N, n_obj, 3), f),
    }


class HaState(C.Structure):
    _fields_ = [(n, P) for n in STATE_FIELDS]


PC_MAX_LINKS = 32


class HaPointcloud(C.Structure):
    """ha_pointcloud_t (include/handarm_abi.h): synthetic point-cloud inputs / outputs (device pointers)."""
    _fields_ = [("object_samples", P), ("robot_samples", P), ("robot_slot", P), ("perm", P),
                ("object_pose", P), ("object_pc", P), ("target_pc", P), ("robot_pc", P), ("fingertip_pc", P),
                ("goal_pc", P), ("relative_goal_pc", P), ("n_pool", C.c_int32), ("P", C.c_int32), ("R", C.c_int32),
                ("n_links", C.c_int32), ("links", C.c_int32 * PC_MAX_LINKS), ("fingertip_slot", C.c_int32 * 5),
                ("flange_slot", C.c_int32)]


CAM_FROM_DEPTH = 1


class HaCamera(C.Structure):
    """ha_camera_t (include/handarm_abi.h)."""
    _fields_ = [("pos", C.c_float * 3), ("quat", C.c_float * 4), ("fovx_deg", C.c_float), ("width", C.c_int32),
                ("height", C.c_int32), ("max_depth", C.c_float), ("workspace", C.c_float * 4), ("goal_radius", C.c_float),
                ("static_seg", C.c_int32 * MAX_STATIC), ("depth", P), ("segmentation", P), ("pointcloud", P),
                ("target_pc", P), ("target_points", C.c_int32), ("rng_counter", C.c_uint32)]


def null_fields(task):
    """State buffers left NULL for a task: object_scale switches the physics to per-env scaled object
    geometry, which only AllegroKuka's cuboid family uses (bit-identical unscaled path otherwise)."""
    return set() if task == TASK_ALLEGRO_KUKA else {"object_scale"}


def load_scene(path=ASSET):
    """Scene JSON; an overlay scene names its base with "extends" (same directory) and replaces its keys."""
    with open(path) as f:
        scene = json.load(f)
    base = scene.pop("extends", None)
    if base:
        merged = load_scene(os.path.join(os.path.dirname(path), base))
        merged.update(scene)
        return merged
    return scene


def _ccw_polygon(pts2):
    """Indices of the 2D convex hull of pts2 in counter-clockwise order (Andrew's monotone chain; collinear
    boundary points dropped), starting at the lexicographically smallest point."""
    order = sorted(range(len(pts2)), key=lambda i: (pts2[i][0], pts2[i][1]))

    def cross(o, a, b):
        return (pts2[a][0] - pts2[o][0]) * (pts2[b][1] - pts2[o][1]) - (pts2[a][1] - pts2[o][1]) * (pts2[b][0] - pts2[o][0])
    lower, upper = [], []
    for i in order:
        while len(lower) >= 2 and cross(lower[-2], lower[-1], i) <= 0:
            lower.pop()
        lower.append(i)
    for i in reversed(order):
        while len(upper) >= 2 and cross(upper[-2], upper[-1], i) <= 0:
            upper.pop()
        upper.append(i)
    return lower[:-1] + upper[:-1]


def hull_topology(verts, planes, tol=2e-7):
    """Edges and face loops of a convex hull given its vertices and face planes (tools/build_model.py hull_planes).

    The face of plane k is the convex polygon of the hull vertices within tol of the plane (hull_planes merged
    coplanar facets whose offsets agree to 1e-7), counter-clockwise about the outward normal. The plane across a
    loop edge is, of the other planes through both its vertices, the one whose normal differs most from plane k's
    (a hull can keep near-duplicate planes of one face apart, and those are not neighbours). A hull edge is a loop
    edge between two planes that are not near-duplicates (normals within 1e-6).

    Returns (edges, loops): edges = [(v0, v1, f0, f1)], each hull edge once, with v0 -> v1 counter-clockwise about
    f0's outward normal and f1 the plane across; loops[k] = [(v, adj)], the face of plane k as a counter-clockwise
    vertex loop, adj = the plane across the loop edge v -> next v. Indices are hull-local."""
    v = np.asarray(verts, np.float64)
    P = np.asarray(planes, np.float64)
    dist = v @ P[:, :3].T + P[:, 3]                         # (V, K): signed distance of vertex to plane
    on = np.abs(dist) <= tol
    loops = []
    for k in range(len(P)):
        idx = np.nonzero(on[:, k])[0]
        assert len(idx) >= 3, f"plane {k} holds {len(idx)} hull vertices"
        n = P[k, :3] / np.linalg.norm(P[k, :3])
        a = np.array([1.0, 0, 0]) if abs(n[0]) < 0.9 else np.array([0, 1.0, 0])
        u = np.cross(n, a)
        u /= np.linalg.norm(u)
        w = np.cross(n, u)                                  # (u, w, n) right-handed: CCW about n in (u, w)
        pts2 = [(float(v[i] @ u), float(v[i] @ w)) for i in idx]
        poly = [int(idx[i]) for i in _ccw_polygon(pts2)]
        loop = []
        for j, a_ in enumerate(poly):
            b_ = poly[(j + 1) % len(poly)]
            cand = [l for l in range(len(P)) if l != k and on[a_, l] and on[b_, l]]
            if cand:
                adj = min(cand, key=lambda l: (float(P[l, :3] @ P[k, :3]), l))
            else:       # an edge bridging near-duplicate faces: the plane both ends lie closest to
                far = [l for l in range(len(P)) if P[l, :3] @ P[k, :3] <= 1 - 1e-6]
                adj = min(far, key=lambda l: (max(abs(dist[a_, l]), abs(dist[b_, l])), l))
            loop.append((a_, adj))
        loops.append(loop)
    edges, seen = [], set()
    for k, loop in enumerate(loops):                        # each edge once, where its first face lists it
        for j, (a_, adj) in enumerate(loop):
            b_ = loop[(j + 1) % len(loop)][0]
            key = (min(a_, b_), max(a_, b_))
            if key in seen or P[adj, :3] @ P[k, :3] > 1 - 1e-6:
                continue
            seen.add(key)
            edges.append((a_, b_, k, adj))
    return edges, loops


_TOPO_CACHE = {}


def _topology(h):
    """hull_topology of a scene hull record, cached by its vertex / plane data."""
    key = (np.asarray(h["verts"], np.float64).tobytes(), np.asarray(h["planes"], np.float64).tobytes())
    if key not in _TOPO_CACHE:
        _TOPO_CACHE[key] = hull_topology(h["verts"], h["planes"])
    return _TOPO_CACHE[key]


# links whose hulls may touch the table (the base-mounted shoulder/upper arm sit on it and would
# only produce contacts against a fixed joint; SURVEY.md §8 a16 robot filter 0b1 vs table 0)
NO_TABLE_CONTACT = {"shoulder_link", "upper_arm_link"}


def build_model(scene, pool_names=None, posed=None):
    """posed: name of a group in scene["posed_statics"] (the AllegroKuka throw "bucket") whose convex pieces become
    statics carried by a per-env actor (ha_model_t v14 posed_actor / static_posed)."""
    m = HaModel()
    rob = scene["robot"]
    links, dofs = rob["links"], rob["dofs"]
    assert len(links) <= MAX_LINKS and len(dofs) <= MAX_DOFS
    m.n_links, m.n_dofs = len(links), len(dofs)
    for i, l in enumerate(links):
        m.link_parent[i] = l["parent"]
        m.link_dof[i] = l["dof"]
        m.link_table_collide[i] = 0 if l["name"] in NO_TABLE_CONTACT else 1
        m.link_origin_pos[i][:] = l["origin_pos"]
        m.link_origin_quat[i][:] = l["origin_quat"]
        m.link_axis[i][:] = l["axis"]
        m.link_mass[i] = l["mass"]
        m.link_com[i][:] = l["com"]
        m.link_inertia[i][:] = l["inertia"]
    for d, rec in enumerate(dofs):
        m.dof_lower[d], m.dof_upper[d], m.dof_effort[d] = rec["lower"], rec["upper"], rec["effort"]
        m.dof_kp[d], m.dof_kd[d] = rec["kp"], rec["kd"]
        m.dof_armature[d] = rec.get("armature", 0.0)
        m.dof_friction[d] = rec.get("friction", 0.0)
    m.base_pos[:] = rob["base_pos"]
    m.base_quat[:] = rob["base_quat"]
    objects = scene["objects"]
    if pool_names is not None:
        byname = {o["name"]: o for o in objects}
        objects = [byname[n] for n in pool_names]
    table = scene.get("table")
    # static boxes: the table (static 0) and any extra pieces (table-with-hole walls, bin parts)
    statics = ([table] if table else []) + list(scene.get("statics", []))
    n_world = len(statics)
    group = scene["posed_statics"][posed] if posed else None
    if group:
        statics += group["pieces"]
    assert len(statics) <= MAX_STATIC
    # object pieces: the convex decomposition when the scene has one ("hulls", tools/convex_decomp.py), else the hull
    obj_hulls = [o.get("hulls") or [o["hull"]] for o in objects]
    hulls = [(h, h["index"]) for h in scene["link_hulls"]] + [(h, -1) for oh in obj_hulls for h in oh] + \
            [(st["hull"], -1) for st in statics]
    assert len(hulls) <= MAX_HULLS
    vs, ps, es, ls = 0, 0, 0, 0
    verts = np.ctypeslib.as_array(m.verts)
    planes = np.ctypeslib.as_array(m.planes)
    edges = np.ctypeslib.as_array(m.edges)
    loop_v = np.ctypeslib.as_array(m.loop_v)
    for k, (h, link) in enumerate(hulls):
        v = np.asarray(h["verts"], np.float32)
        p = np.asarray(h["planes"], np.float32)
        assert len(v) <= 64, "hull vertex count must fit one wavefront"
        m.hull_link[k] = link
        m.hull_vert_start[k], m.hull_nverts[k] = vs, len(v)
        m.hull_plane_start[k], m.hull_nplanes[k] = ps, len(p)
        m.hull_center[k][:] = h["center"]
        m.hull_radius[k] = h["radius"]
        verts[vs:vs + len(v), :3] = v
        planes[ps:ps + len(p)] = p
        # v10 topology: edges (v0, v1, f0, f1) and per-plane face loops
        he, hl = _topology(h)
        assert es + len(he) <= MAX_EDGES and ls + sum(len(l) for l in hl) <= MAX_LOOP
        assert max(len(l) for l in hl) <= MAX_FACE_LOOP, "face loop longer than HA_MAX_FACE_LOOP"
        m.hull_edge_start[k], m.hull_nedges[k] = es, len(he)
        for i, (a, b, f0, f1) in enumerate(he):
            edges[es + i] = a | (b << 8) | (f0 << 16) | (f1 << 24)
        es += len(he)
        for j, loop in enumerate(hl):
            m.plane_loop[ps + j] = ls | (len(loop) << 16)
            for t, (a, adj) in enumerate(loop):
                loop_v[ls + t] = a
            ls += len(loop)
        vs += len(v)
        ps += len(p)
    assert vs <= MAX_VERTS and ps <= MAX_PLANES
    m.n_link_hulls = len(scene["link_hulls"])
    m.n_pool = len(objects)
    m.n_hulls = len(hulls)
    first = m.n_link_hulls
    for i, o in enumerate(objects):
        m.pool_hull[i] = first
        m.pool_nhull[i] = len(obj_hulls[i])
        first += len(obj_hulls[i])
        if len(obj_hulls[i]) == 1:          # the hull's own sphere (bit-identical broad phase for one-hull objects)
            m.pool_center[i][:] = obj_hulls[i][0]["center"]
            m.pool_radius[i] = obj_hulls[i][0]["radius"]
            m.hull_obb[m.pool_hull[i]][:] = object_box(obj_hulls[i][0]["verts"])
        else:
            pts = np.concatenate([np.asarray(h["verts"], np.float64) for h in obj_hulls[i]])
            ctr = 0.5 * (pts.min(0) + pts.max(0))
            m.pool_center[i][:] = ctr
            m.pool_radius[i] = float(np.linalg.norm(pts - ctr, axis=1).max()) * (1 + 1e-6)
            for j, h in enumerate(obj_hulls[i]):      # each piece's oriented box (the piece-pair box cull, round 6)
                m.hull_obb[m.pool_hull[i] + j][:] = hull_obb(h["verts"])
        m.pool_mass[i] = o["mass"]
        m.pool_com[i][:] = o["com"]
        m.pool_inertia[i][:] = o["inertia"]
        m.pool_bbox_pos[i][:] = o.get("bbox_from_origin_pos", (0, 0, 0))
        m.pool_bbox_quat[i][:] = o.get("bbox_from_origin_quat", (0, 0, 0, 1))
        m.pool_bbox_ext[i][:] = o.get("bbox_extents", (0, 0, 0))
    first_static = len(hulls) - len(statics)
    m.n_static = len(statics)
    for k, st in enumerate(statics):
        m.static_hull[k] = first_static + k
        m.static_pos[k][:] = st["pos"]
        m.static_quat[k][:] = st["quat"]
        m.static_half[k][:] = st["half_extents"]
        m.static_posed[k] = int(k >= n_world)
    m.posed_actor = scene["layout"][group["actor"]] if group else -1
    if table:
        m.table_hull = first_static
        m.table_pos[:] = table["pos"]
        m.table_quat[:] = table["quat"]
        m.table_half[:] = table["half_extents"]
    else:
        m.table_hull = -1
        m.table_quat[:] = (0, 0, 0, 1)
    # gym tensor layout (actor and rigid-body creation order). Default: Ur5SihMultiObject (multi_object.py:
    # 562-663): goal 0, robot 1, table 2, objects 3..; bodies goal, robot links, table, objects.
    L = len(links)
    n_obj = scene.get("objects_per_env", 3)
    lay = scene.get("layout") or dict(n_actors=3 + n_obj, actor_robot=1, actor_object0=3, actor_goal=0, actor_table=2,
                                      n_bodies=1 + L + 1 + n_obj, body_robot0=1, body_object0=L + 2, body_goal=0,
                                      body_table=L + 1)
    for k, v in lay.items():
        setattr(m, k, v)
    # fixed bodies with a model pose (table-with-hole links, bin: multi_object.py:626-637)
    fixed = scene.get("fixed_bodies", [])
    assert len(fixed) <= MAX_FIXED_BODIES
    m.n_fixed_bodies = len(fixed)
    m.body_fixed0 = scene.get("body_fixed0", -1) if fixed else -1
    for k, pose in enumerate(fixed):
        m.body_fixed_pose[k][:] = pose
    # derived topology for the level-synchronous wave kernels
    level = []
    for i, l in enumerate(links):
        assert l["parent"] < i, "links must be in depth-first (parent-first) order"
        level.append(0 if l["parent"] < 0 else level[l["parent"]] + 1)
        m.link_level[i] = level[-1]
        if l["dof"] >= 0:
            m.dof_link[l["dof"]] = i
    m.max_level = max(level)
    pairs = []
    for d in range(len(dofs)):
        j = m.dof_link[d]
        while j >= 0:
            if links[j]["dof"] >= 0:
                pairs.append((d, links[j]["dof"]))
            j = links[j]["parent"]
    assert len(pairs) <= MAX_MPAIRS
    m.n_mpairs = len(pairs)
    for k, (d, e) in enumerate(pairs):
        m.mpair[k][0], m.mpair[k][1] = d, e
    _self_collision(m, scene, links)
    return m


def hull_obb(verts):
    """Oriented box of a hull's vertices (principal axes of the vertex cloud, extents from the projections, a
    right-handed frame): centre[3], half extents[3], quat[4] (xyzw), pad[2] -- the ha_model_t.hull_obb record."""
    v = np.asarray(verts, np.float64)
    c0 = v.mean(0)
    _, _, vt = np.linalg.svd(v - c0)
    R = vt.T.copy()
    if np.linalg.det(R) < 0:
        R[:, 2] = -R[:, 2]
    loc = (v - c0) @ R
    lo, hi = loc.min(0), loc.max(0)
    c = c0 + R @ ((lo + hi) / 2)
    half = (hi - lo) / 2 * (1 + 1e-5) + 1e-6          # float32 rounding of the pose must not cut a vertex off
    # rotation matrix -> quaternion (xyzw), largest-component branch
    tr = np.trace(R)
    if tr > 0:
        S = np.sqrt(tr + 1.0) * 2
        q = [(R[2, 1] - R[1, 2]) / S, (R[0, 2] - R[2, 0]) / S, (R[1, 0] - R[0, 1]) / S, 0.25 * S]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        S = np.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = [0.0] * 4
        q[i] = 0.25 * S
        q[j] = (R[j, i] + R[i, j]) / S
        q[k] = (R[k, i] + R[i, k]) / S
        q[3] = (R[k, j] - R[j, k]) / S
    q = np.asarray(q) / np.linalg.norm(q)
    return list(c) + list(half) + list(q) + [0.0, 0.0]


def object_box(verts):
    """A one-piece pool object's box for the broad phase's box cull (ha_physics.h pair_boxes_near): the hull's bounding
    box in the body frame (identity orientation, so a per-env object scale scales its centre and half extents), padded
    like hull_obb; the same 12-float record."""
    v = np.asarray(verts, np.float64)
    lo, hi = v.min(0), v.max(0)
    half = (hi - lo) / 2 * (1 + 1e-5) + 1e-6
    return list((lo + hi) / 2) + list(half) + [0.0, 0.0, 0.0, 1.0, 0.0, 0.0]


def _self_collision(m, scene, links):
    """ha_model_t v12 self-collision pairs: with scene["self_collision"] (the Allegro scenes: their hand actors use
    collision filter -1, allegro_hand.py:334-335, allegro_kuka_base.py:664), every pair of link hulls on two links
    that are not parent and child (PhysX's articulation filter), minus scene["self_collision"]["exclude"] link pairs.
    Every link hull gets its oriented box (hull_obb) either way."""
    for k, h in enumerate(scene["link_hulls"]):
        m.hull_obb[k][:] = hull_obb(h["verts"])
    sc = scene.get("self_collision")
    m.n_self_pairs = 0
    if not sc:
        return
    excl = {tuple(sorted(p)) for p in sc.get("exclude", [])}
    hl = [h["index"] for h in scene["link_hulls"]]
    pairs = []
    for a in range(len(hl)):
        for b in range(a + 1, len(hl)):
            la, lb = hl[a], hl[b]
            if la == lb or links[la]["parent"] == lb or links[lb]["parent"] == la or tuple(sorted((la, lb))) in excl:
                continue
            pairs.append(a | (b << 8))
    assert len(pairs) <= MAX_SELF_PAIRS
    m.n_self_pairs = len(pairs)
    for k, v in enumerate(pairs):
        m.self_pair[k] = v


# ----------------------------------------------------------------------------- splines (host)
SPLINE_ORDER = ["thumb_proximal", "thumb_distal", "index_proximal", "index_distal", "middle_proximal",
                "middle_distal", "ring_proximal", "ring_distal"]
SPLINE_KNOTS = {   # ur5sih.py:442-455
    "thumb_proximal": ([-1850, -1175, -975, -600, -225], [-1.51, -1.31, -1.175, -0.6, 0.]),
    "thumb_distal": ([-1318.125, -906.25, -200], [-1.235, -0.855, 0.]),
    "index_proximal": ([-1250, -250, 150, 350, 540, 730, 1085, 1400], [-1.53, -1.4425, -1.315, -1.25, -1.18, -1.15, -0.6, 0.]),
    "index_distal": ([-408.606, 793.515, 1400], [-1.665, -0.735, 0]),
    "middle_proximal": ([-500, 500, 1350, 1625, 1700, 1980, 2240], [-1.571, -1.445, -1.055, -0.91, -0.9, -0.48, 0.]),
    "middle_distal": ([442.6, 1147, 1750.6, 2240], [-1.65, -1.125, -0.62, 0.]),
    "ring_proximal": ([-1050, -500, -250, 0, 370, 500, 700, 940], [-1.571, -1.45, -1.35, -1.225, -0.95, -0.9, -0.533, 0.]),
    "ring_distal": ([-719, 408.8, 686.8, 939.2], [-1.64, -0.69, -0.425, 0.]),
}


def natural_cubic_spline_table(knots, values):
    """Coefficients of the natural cubic spline through (knots, values), in float32 and in the
    operation order of torchcubicspline.natural_cubic_spline_coeffs (tridiagonal knot-derivative
    system, Thomas algorithm).  Returns (5, pieces): piece start, a, b, two_c, three_d."""
    F = np.float32
    t = np.asarray(knots, F)
    x = np.asarray(values, F)
    n = len(t)
    dt = t[1:] - t[:-1]
    r = (F(1) / dt).astype(F)
    r2 = (r ** 2).astype(F)
    three = F(3) * (x[1:] - x[:-1])
    six = F(2) * three
    scaled = three * r2
    diag = np.empty(n, F)
    diag[:-1] = r
    diag[-1] = 0
    diag[1:] += r
    diag *= F(2)
    rhs = np.empty(n, F)
    rhs[:-1] = scaled
    rhs[-1] = 0
    rhs[1:] += scaled
    nb, nd, out = np.empty(n, F), np.empty(n, F), np.empty(n, F)
    nb[0], nd[0] = rhs[0], diag[0]
    for i in range(1, n):
        w = r[i - 1] / nd[i - 1]
        nd[i] = diag[i] - w * r[i - 1]
        nb[i] = rhs[i] - w * nb[i - 1]
    out[n - 1] = nb[n - 1] / nd[n - 1]
    for i in range(n - 2, -1, -1):
        out[i] = (nb[i] - r[i] * out[i + 1]) / nd[i]
    two_c = (six * r - F(4) * out[:-1] - F(2) * out[1:]) * r
    three_d = (-six * r + F(3) * (out[:-1] + out[1:])) * r2
    return np.stack([t[:-1], x[:-1], out[:-1], two_c, three_d]).astype(F)


DEFAULT_TASK = dict(
    dt=0.016666667, substeps=2, control_freq_inv=3, solver_iters=8, gravity=(0.0, 0.0, -9.81),
    friction=1.0, contact_margin=0.01, baumgarte=0.2, max_depen_vel=1.0, object_ang_damping=0.5,
    contact_slop=0.001, manifold_window=0.002,
    link_lin_damping=0.01, link_ang_damping=0.01,       # ur5sih.py:178-179
    edge_rel_tol=0.9, edge_abs_tol=0.0005,              # edge-edge vs face axis (handarm_abi.h v10)
    narrow_phase_flags=0,                               # HA_NP_* (A/B and diagnostics only)
    # persistent contact manifolds (handarm_abi.h v13): a pair's record is reused while its relative pose stays within
    # pcm_lin_tol (m) and pcm_cos_tol (cos of half the relative rotation angle: 0.9998 = 2.3 degrees, PhysX's PCM
    # rotation threshold) of the pose it was built at
    pcm_lin_tol=0.001, pcm_cos_tol=0.9998,
    joint_limit_margin=0.02, n_objects=3, num_initial_poses=1, max_episode_length=200,
    sih_alpha=0.8, reward_reaching=1.0, reward_lifting=5.0, reward_goal=50.0, reward_success=50.0,
    lifting_threshold=0.05, goal_threshold=0.05, goal_pos=(0.28, 0.58, 0.8), goal_noise=(0.15, 0.15, 0.1),
    dr_enable=0,           # task.randomize; the schema: handarm_hip/dr.py (apply_schema)
    drop_pos=(0.28, 0.58, 1.5), drop_noise=(0.1, 0.1, 0.0), drop_num_steps=100,
    reset_pose=(0.6985, -1.4106, 1.2932, 0.1174, 0.6983, 1.5708, 0., 0., 0., 0., 0., 0., 0., 0., -1.571, 0., 0.),
    bringup_pose=(0., -1.571, 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., -1.571, 0., 0.),
    servo_lower=(0, -2000, -1250, -400, -1350), servo_upper=(2650, 250, 1450, 2300, 1000),
    proximal_coef=(-625.0, -582.61, -600.0, -488.0), seed=42,
)


# AllegroHand (config C3): cfg/task/AllegroHand.yaml + tasks/allegro_hand.py
ALLEGRO_TASK = dict(
    DEFAULT_TASK, task=TASK_ALLEGRO_HAND, num_actions=16, num_obs=88, n_objects=1,
    dt=0.01667, substeps=2, control_freq_inv=2, solver_iters=8,          # AllegroHand.yaml:23,160-173
    pcm_lin_tol=0.0, pcm_cos_tol=1.0,        # no persistent manifolds in the AllegroHand family
    link_lin_damping=0.0, link_ang_damping=0.01,                         # allegro_hand.py:231 (linear: default 0)
    contact_margin=0.002, max_depen_vel=1000.0,                          # contact_offset, max_depenetration_velocity
    max_episode_length=600,                                              # episodeLength
    dist_reward_scale=-10.0, rot_reward_scale=1.0, rot_eps=0.1, action_penalty_scale=-0.0002,
    success_tolerance=0.1, reach_goal_bonus=250.0, fall_dist=0.24, fall_penalty=0.0,
    max_consecutive_successes=0, av_factor=0.1,                          # allegro_hand.py:79 averFactor default
    reset_position_noise=0.01, reset_dof_pos_noise=0.2, reset_dof_vel_noise=0.0, act_moving_average=1.0,
    vel_obs_scale=0.2, force_torque_obs_scale=10.0,                      # allegro_hand.py:57-58
    clip_observations=5.0, clip_actions=1.0,
    # observationType, asymmetric_observations, useRelativeControl, dofSpeedScale (AllegroHand.yaml:14-19,42-43)
    obs_type="full_state", asymmetric=False, relative_control=False, dof_speed_scale=20.0,
    # forceScale, forceProbRange, forceDecay, forceDecayInterval (AllegroHand.yaml:26-29; allegro_hand.py:66-70)
    force_scale=0.0, force_prob_range=(0.001, 0.1), force_decay=0.99, force_decay_interval=0.08,
    # hand at (0, 0, 0.5); object at hand + (0, -0.2, 0.06); goal_states = object - 0.04 z; goal actor at
    # goal_states + displacement (allegro_hand.py:284-300,363-365)
    object_init=(0.0, -0.2, 0.56, 0.0, 0.0, 0.0, 1.0), goal_init=(0.0, -0.2, 0.52),
    goal_displacement=(-0.2, -0.06, 0.12),
)


# AllegroHand observation types (allegro_hand.py:99-112): ha_params_t.ah_obs_type and num_obs; the states buffer of
# asymmetric observations is the 88-float full_state vector (num_states, allegro_hand.py:121-124)
AH_OBS_TYPES = {"full_state": 0, "full": 1, "full_no_vel": 2}
AH_NUM_OBS = {"full_state": 88, "full": 72, "full_no_vel": 50}
AH_NUM_STATES = 88
# objectType (allegro_hand.py:82-97): the AllegroHand scene's pool entries (tools/build_model.py main_allegro)
AH_OBJECT_TYPES = {"block": 0, "egg": 1, "pen": 2}


def num_states(params):
    """teacher_obs width: AllegroHand's states buffer (asymmetric observations) or the task's observation size."""
    return AH_NUM_STATES if params.task == TASK_ALLEGRO_HAND and params.ah_asymmetric else params.num_obs


# AllegroKuka (config C2): cfg/task/AllegroKuka.yaml:9-94,210-231 + env/regrasping.yaml (default subtask here:
# BASELINE.json config 2 "Arm+Allegro cube grasp") or env/reorientation.yaml; allegro_kuka_base.py:53-400
def _f32(x):
    return float(np.float32(x))


ALLEGRO_KUKA_TASK = dict(
    DEFAULT_TASK, task=TASK_ALLEGRO_KUKA, num_actions=23, n_objects=1, subtask="regrasping",
    dt=0.01667, substeps=2, control_freq_inv=1, solver_iters=8,          # AllegroKuka.yaml:27,210-223
    contact_margin=0.002, max_depen_vel=1000.0,                          # :226-229
    episode_length={"regrasping": 300, "reorientation": 600, "throw": 300},
    success_steps={"regrasping": 30, "reorientation": 1, "throw": 5},
    reset_position_noise=(0.1, 0.1, 0.02), reset_dof_pos_noise_fingers=0.1, reset_dof_pos_noise_arm=0.1,
    reset_dof_vel_noise=0.5, force_scale=2.0, force_prob_range=(0.001, 0.1), force_decay=0.99,
    force_decay_interval=0.08, lifting_rew_scale=20.0, lifting_bonus=300.0, lifting_bonus_threshold=0.15,
    keypoint_rew_scale=200.0, distance_delta_rew_scale=50.0, reach_goal_bonus=1000.0,
    kuka_actions_penalty_scale=0.003, allegro_actions_penalty_scale=0.0003, dof_speed_scale=10.0,
    act_moving_average=1.0, keypoint_scale=1.5, object_base_size=0.05, success_tolerance=0.075,
    target_success_tolerance=0.01, tolerance_curriculum_increment=0.9, tolerance_curriculum_interval=3000,
    max_consecutive_successes=50, clamp_abs_observations=10.0,
    # desired_kuka_pos pose v1 (allegro_kuka_base.py:316-319), fingers 0
    reset_pose=(-1.571, 1.571, -0.000, 1.376, -0.000, 1.485, 2.358) + (0.0,) * 16,
    # allegro_pose (0, 0.8, 0) in gymapi.Vec3 (float32); object_start_pose = allegro_pose + (0, -0.8, 0.38 + 0.25)
    # computed by Vec3 arithmetic (allegro_kuka_base.py:401-413,608-628)
    object_init=(0.0, _f32(_f32(0.8) + -0.8), _f32(0.0 + (0.38 + 0.25))),
    target_volume_origin=(0.0, 0.05, 0.8), target_volume_extent=((-0.4, 0.4), (-0.05, 0.3), (-0.12, 0.25)),
    palm_offset=(-0.00, -0.02, 0.16), fingertip_offsets=((0.05, 0.005, 0), (0.05, 0.005, 0), (0.05, 0.005, 0),
                                                        (0.06, 0.005, 0)),
    palm_link="iiwa7_link_7", fingertip_links=("index_link_3", "middle_link_3", "ring_link_3", "thumb_link_3"),
    num_arm_dofs=7,
)
AK_KEYPOINTS = {"regrasping": [[0, 0, 0]],                                          # allegro_kuka_regrasping.py:46-48
                "reorientation": [[1, 1, 1], [1, 1, -1], [-1, -1, 1], [-1, -1, -1]],   # reorientation.py:48-54
                "throw": [[0, 0, 0]]}                                               # allegro_kuka_throw.py:47-49
AK_SUBTASKS = {"regrasping": 0, "reorientation": 1, "throw": 2}                     # ha_params_t.ak_subtask
# the throw bucket's creation pose: allegro_pose (0, 0.8, 0) + (-0.6, -1, 0.45) in gymapi.Vec3 float32 arithmetic
# (allegro_kuka_base.py:606-607,632, allegro_kuka_throw.py:68-72)
AK_BUCKET_POSE = (_f32(0.0 - 0.6), _f32(_f32(0.8) - 1.0), _f32(0.0 + 0.45))
# env/<subtask>.yaml values beyond episodeLength / successSteps: throw has no random forces, a fixed 7.5 cm tolerance
# and small cuboids only (env/throw.yaml:5-18; the object family is the scene's "object_dims_throw")
AK_SUBTASK_CFG = {"throw": dict(force_scale=0.0, success_tolerance=0.075, target_success_tolerance=0.075)}


def posed_group(task, cfg):
    """The group of posed statics (ha_model_t v14) a task's model carries: the AllegroKuka throw bucket."""
    if task == TASK_ALLEGRO_KUKA and (cfg or {}).get("subtask", ALLEGRO_KUKA_TASK["subtask"]) == "throw":
        return "bucket"
    return None


def kuka_object_dims(scene, c):
    """The subtask's cuboid family (allegro_kuka_base.py:485-512 with its with* flags)."""
    return scene.get("object_dims_" + c["subtask"], scene["object_dims"])


def kuka_tolerance_scalars(success_tolerance, c):
    """task_scalars for the device: success_tolerance, tolerance_successes_objective's tolerance term and
    branch, keypoint success tolerance (python double arithmetic, allegro_kuka_utils.py:122-163,
    allegro_kuka_base.py:862), each rounded once to float32 like a python scalar in a tensor op."""
    ini, tgt = c["success_tolerance"], c["target_success_tolerance"]
    tol_obj = (ini - success_tolerance) / (ini - tgt) if ini > tgt else 1.0
    return np.array([success_tolerance, tol_obj, 1.0 if success_tolerance > tgt else 0.0,
                     success_tolerance * c["keypoint_scale"]], np.float32)


def kuka_env_tables(num_envs, scene, c):
    """Per-env object scales (env i gets object_dims[i % len], allegro_kuka_base.py:687-707) and keypoint
    offsets (:708-715, python double, rounded once by to_torch)."""
    dims = kuka_object_dims(scene, c)
    kps = AK_KEYPOINTS[c["subtask"]]
    scales = np.zeros((num_envs, 1, 3), np.float32)
    offs = np.zeros((num_envs, 4, 3), np.float32)
    for i in range(num_envs):
        sc = dims[i % len(dims)]
        scales[i, 0] = sc
        for j, kp in enumerate(kps):
            offs[i, j] = [kp[k] * (sc[k] * c["object_base_size"] * c["keypoint_scale"] / 2) for k in range(3)]
    return scales, offs


def ur5sih_num_obs(n_objects):
    """Ur5Sih observation size: 80 + 13 per object + 28 (object_pos 3 and object_bounding_box 10 per object,
    multi_object.py:128,245; 147 at the default 3 objects)."""
    return 108 + 13 * n_objects


def build_params(cfg=None, task=None):
    want = task if task is not None else (cfg or {}).get("task")
    c = dict(ALLEGRO_TASK if want == TASK_ALLEGRO_HAND else (ALLEGRO_KUKA_TASK if want == TASK_ALLEGRO_KUKA
                                                             else DEFAULT_TASK))
    if want == TASK_ALLEGRO_KUKA:
        c.update(AK_SUBTASK_CFG.get((cfg or {}).get("subtask", c["subtask"]), {}))
    if cfg:
        c.update(cfg)
    p = HaParams()
    for k in ["dt", "substeps", "control_freq_inv", "solver_iters", "friction", "contact_margin", "baumgarte",
              "contact_slop", "manifold_window", "link_lin_damping", "link_ang_damping", "edge_rel_tol",
              "edge_abs_tol", "narrow_phase_flags", "pcm_lin_tol", "pcm_cos_tol",
              "max_depen_vel", "object_ang_damping", "joint_limit_margin", "n_objects", "num_initial_poses",
              "max_episode_length", "sih_alpha", "reward_reaching", "reward_lifting", "reward_goal",
              "reward_success", "lifting_threshold", "goal_threshold", "seed"]:
        setattr(p, k, c[k])
    if os.environ.get("HA_NP_FLAGS"):          # A/B timing of the narrow-phase stages (HA_NP_*), diagnostics only
        p.narrow_phase_flags = int(os.environ["HA_NP_FLAGS"])
    if os.environ.get("HA_PCM"):               # A/B of the persistent manifolds: "off" or "lin,cos" (diagnostics only)
        v = os.environ["HA_PCM"]
        p.pcm_lin_tol, p.pcm_cos_tol = (0.0, 1.0) if v == "off" else tuple(float(x) for x in v.split(","))
    p.gravity[:] = c["gravity"]
    p.action_dt = c["dt"]                      # VecTask.dt = sim_params.dt (vec_task.py:267)
    p.sih_beta = 1.0 - c["sih_alpha"]          # (1 - alpha) * s: python double, cast once (ur5sih.py:496)
    p.goal_pos[:] = c["goal_pos"]
    p.goal_noise[:] = c["goal_noise"]
    p.reset_pose[:len(c["reset_pose"])] = c["reset_pose"]
    p.servo_lower[:] = c["servo_lower"]
    p.servo_upper[:] = c["servo_upper"]
    p.proximal_coef[:] = c["proximal_coef"]
    sp = np.ctypeslib.as_array(p.spline)
    for i, name in enumerate(SPLINE_ORDER):
        tab = natural_cubic_spline_table(*SPLINE_KNOTS[name])
        p.spline_pieces[i] = tab.shape[1]
        sp[i, :, :tab.shape[1]] = tab
    p.thumb_opposition_gain = np.float32(-1.571 / 2675)
    p.task = c.get("task", TASK_UR5SIH)
    # domain randomization (v16): task.randomize + task.randomization_params (handarm_hip/dr.py); dr_enable without a
    # schema takes the task family's default (Ur5Sih: the build's config-4 definition)
    p.dr_enable = int(c.get("dr_enable", 0))
    if p.dr_enable:
        from . import dr as DR
        DR.apply_schema(p, c.get("randomization_params"), p.task)
    p.num_actions = c.get("num_actions", 11)
    p.num_obs = c.get("num_obs", ur5sih_num_obs(int(c["n_objects"])))
    if p.task == TASK_ALLEGRO_HAND:
        for k in ["dist_reward_scale", "rot_reward_scale", "rot_eps", "action_penalty_scale", "success_tolerance",
                  "reach_goal_bonus", "fall_dist", "fall_penalty", "max_consecutive_successes", "av_factor",
                  "reset_position_noise", "reset_dof_pos_noise", "reset_dof_vel_noise", "act_moving_average",
                  "vel_obs_scale", "force_torque_obs_scale"]:
            setattr(p, "ah_" + k, c[k])
        p.ah_obs_type = AH_OBS_TYPES[c["obs_type"]]
        p.num_obs = AH_NUM_OBS[c["obs_type"]]                 # allegro_hand.py:106-112
        p.ah_asymmetric = int(bool(c["asymmetric"]))
        p.ah_relative_control = int(bool(c["relative_control"]))
        p.ah_speed_dt = c["dof_speed_scale"] * c["dt"]       # shadow_hand_dof_speed_scale * self.dt (python double)
        import torch
        p.ah_force_scale = c["force_scale"]
        p.ah_force_prob_lo, p.ah_force_prob_hi = c["force_prob_range"]
        # torch.pow(to_torch(forceDecay), dt / forceDecayInterval): a float32 tensor to a python-double power
        p.ah_force_decay_step = float(torch.pow(torch.tensor(c["force_decay"], dtype=torch.float32),
                                                c["dt"] / c["force_decay_interval"]))
        p.ah_object_type = AH_OBJECT_TYPES[c.get("object_type", "block")]
        obj_init, goal_init = list(c["object_init"]), list(c["goal_init"])
        if c.get("object_type") == "pen":
            # object_start_pose.p.z = hand z + 0.02 (a gymapi.Vec3 float), goal_states z - 0.04 in fp32 (:295-296,
            # 363-365); compute_hand_reward doubles the success tolerance (ignore_z_rot, :675-676)
            obj_init[2] = float(np.float32(0.5 + 0.02))
            goal_init[2] = float(np.float32(np.float32(obj_init[2]) - np.float32(0.04)))
            p.ah_success_tolerance = 2.0 * c["success_tolerance"]
        p.ah_object_init[:] = obj_init
        p.ah_goal_init[:] = goal_init
        p.ah_goal_displacement[:] = c["goal_displacement"]
        # (1.0 - act_moving_average) * prev_targets: python double, cast once (allegro_hand.py:612-613)
        p.sih_beta = 1.0 - c["act_moving_average"]
        p.action_dt = c["dt"]
    if p.task == TASK_ALLEGRO_KUKA:
        _kuka_params(p, c)
    return p, c


def _kuka_params(p, c):
    import torch
    sub = c["subtask"]
    assert sub in AK_KEYPOINTS, sub
    kps = AK_KEYPOINTS[sub]
    p.ak_subtask = AK_SUBTASKS[sub]
    p.ak_num_keypoints = len(kps)
    for j, kp in enumerate(kps):
        p.ak_keypoints[j][:] = kp
    p.num_obs = 93 + 6 * len(kps)                      # full_state_size (allegro_kuka_base.py:185-220)
    # privilegedActions: 3 object-torque actions ahead of the 23 (allegro_kuka_base.py:62-74), privilegedActionsTorque
    p.ak_privileged_actions = int(bool(c.get("privileged_actions", False)))
    p.ak_privileged_torque = c.get("privileged_actions_torque", 0.02)
    p.num_actions = 23 + 3 * p.ak_privileged_actions
    p.max_episode_length = c.get("max_episode_length_override") or c["episode_length"][sub]
    p.ak_success_steps = c["success_steps"][sub] if isinstance(c["success_steps"], dict) else c["success_steps"]
    for k in ["object_base_size", "keypoint_scale", "lifting_rew_scale", "lifting_bonus", "lifting_bonus_threshold",
              "keypoint_rew_scale", "distance_delta_rew_scale", "reach_goal_bonus", "kuka_actions_penalty_scale",
              "allegro_actions_penalty_scale", "max_consecutive_successes", "force_scale", "act_moving_average"]:
        setattr(p, "ak_" + k, c[k])
    p.ak_initial_tolerance = c["success_tolerance"]
    p.ak_target_tolerance = c["target_success_tolerance"]
    p.ak_bonus_rew = c["reach_goal_bonus"] / p.ak_success_steps
    p.ak_reset_noise[:] = c["reset_position_noise"]
    p.ak_dof_noise_arm = c["reset_dof_pos_noise_arm"]
    p.ak_dof_noise_fingers = c["reset_dof_pos_noise_fingers"]
    p.ak_dof_vel_noise = c["reset_dof_vel_noise"]
    p.ak_force_prob_lo, p.ak_force_prob_hi = c["force_prob_range"]
    # torch.pow(force_decay (fp32 tensor), dt / force_decay_interval) (allegro_kuka_base.py:1402)
    p.ak_force_decay_step = float(torch.pow(torch.tensor(c["force_decay"], dtype=torch.float32),
                                            c["dt"] / c["force_decay_interval"]))
    p.ak_dof_speed_scale = c["dof_speed_scale"] * c["dt"]          # python double, rounded by the tensor op
    p.ak_one_minus_ama = 1.0 - c["act_moving_average"]
    p.ak_clamp_abs_obs = c["clamp_abs_observations"]
    p.ak_object_init[:] = c["object_init"]
    p.ak_goal_init[:] = (c["object_init"][0], c["object_init"][1], np.float32(c["object_init"][2]) - np.float32(0.04))
    o = np.asarray(c["target_volume_origin"], np.float32)
    ext = np.asarray(c["target_volume_extent"], np.float32)
    lo, hi = o + ext[:, 0], o + ext[:, 1]
    p.ak_target_origin[:] = o
    p.ak_target_lo[:] = lo
    p.ak_target_size[:] = hi - lo
    p.ak_palm_offset[:] = c["palm_offset"]
    for i in range(4):
        p.ak_fingertip_offsets[i][:] = c["fingertip_offsets"][i]
    p.ak_num_arm_dofs = c["num_arm_dofs"]
    scene = load_scene(c.get("scene_path", KUKA_ASSET))
    names = [l["name"] for l in scene["robot"]["links"]]
    p.ak_palm_link = names.index(c["palm_link"])                    # find_asset_rigid_body_index (:642-644)
    p.ak_fingertip_links[:] = [names.index(n) for n in c["fingertip_links"]]
    # object_rb_masses: the object of env 0 (allegro_kuka_base.py:734-735), box of density 400
    d0 = kuka_object_dims(scene, c)[0]
    p.ak_object_rb_mass = 400.0 * (c["object_base_size"] * d0[0]) * (c["object_base_size"] * d0[1]) * \
        (c["object_base_size"] * d0[2])
