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

MAX_LINKS, MAX_DOFS, MAX_HULLS, MAX_VERTS, MAX_PLANES = 32, 24, 64, 4096, 8192
MAX_POOL, MAX_OBJ, MAX_INIT_POSES, MAX_SPLINE_PIECES, N_SPLINES = 32, 3, 4, 8, 8
MAX_MPAIRS = 192
STAT_SIZE = 2 + 2 * MAX_POOL
DRAW_STRIDE = 48
DR_SIZE = 72
DR_LINK_MASS, DR_OBJ_MASS, DR_LINK_FRIC, DR_OBJ_FRIC = 0, 32, 36, 68
TASK_UR5SIH, TASK_ALLEGRO_HAND = 0, 1

FLAG_NO_PHYSICS = 1
FLAG_REPLAY_DRAWS = 2
FLAG_OBS_ONLY = 4

f32, i32 = C.c_float, C.c_int32


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
        ("dr_enable", i32), ("dr_mass_lo", f32), ("dr_mass_hi", f32), ("dr_fric_lo", f32), ("dr_fric_hi", f32),
        ("dr_fric_buckets", i32), ("dr_obs_noise", f32), ("dr_act_noise", f32),
    ]


P = C.c_void_p


STATE_FIELDS = ["root_state", "rigid_body_state", "dof_state", "net_contact_force", "sim_targets",
                "dof_position_targets", "actions", "obs", "teacher_obs", "rew", "reset_buf", "progress_buf",
                "timeout_buf", "goal_reached_before", "goal_pos", "target_object_index",
                "object_configuration_indices", "object_indices", "object_pos_initial", "object_quat_initial",
                "ur5_target", "servo", "smoothed", "obs_cache", "reset_draws", "episode", "stats", "term_sums",
                "flags", "collision_enabled", "dof_force", "reset_goal_buf", "successes", "goal_state",
                "consecutive_successes", "dr_scale"]


def state_spec(num_envs, n_links=29, n_dofs=17, n_obj=3, num_initial_poses=1, num_actions=11, num_obs=147,
               n_actors=None, n_bodies=None):
    """name -> (shape, numpy dtype) of every ha_state_t buffer (Isaac Gym tensor layouts)."""
    N, D, P = num_envs, n_dofs, num_initial_poses
    A = n_actors if n_actors is not None else 3 + n_obj
    B = n_bodies if n_bodies is not None else 1 + n_links + 1 + n_obj
    f, i64, u8, i32, u32 = np.float32, np.int64, np.uint8, np.int32, np.uint32
    return {
        "root_state": ((N * A, 13), f), "rigid_body_state": ((N * B, 13), f), "dof_state": ((N * D, 2), f),
        "net_contact_force": ((N * B, 3), f), "sim_targets": ((N, D), f), "dof_position_targets": ((N, D), f),
        "actions": ((N, num_actions), f), "obs": ((N, num_obs), f), "teacher_obs": ((N, num_obs), f),
        "rew": ((N,), f), "reset_buf": ((N,), i64), "progress_buf": ((N,), i64), "timeout_buf": ((N,), u8),
        "goal_reached_before": ((N,), u8), "goal_pos": ((N, 3), f), "target_object_index": ((N,), i64),
        "object_configuration_indices": ((N,), i64), "object_indices": ((N, n_obj), i64),
        "object_pos_initial": ((N, P, n_obj, 3), f), "object_quat_initial": ((N, P, n_obj, 4), f),
        "ur5_target": ((N, 6), f), "servo": ((N, 5), f), "smoothed": ((N, 5), f), "obs_cache": ((N, n_obj, 7), f),
        "reset_draws": ((N, DRAW_STRIDE), f), "episode": ((N,), u32), "stats": ((STAT_SIZE,), i32),
        "term_sums": ((4,), f), "flags": ((4,), i32), "collision_enabled": ((N, n_obj), u8),
        "dof_force": ((N, D), f), "reset_goal_buf": ((N,), i64), "successes": ((N,), f), "goal_state": ((N, 7), f),
        "consecutive_successes": ((1,), f), "dr_scale": ((N, DR_SIZE), f),
    }


class HaState(C.Structure):
    _fields_ = [(n, P) for n in STATE_FIELDS]


def load_scene(path=ASSET):
    with open(path) as f:
        return json.load(f)


# links whose hulls may touch the table (the base-mounted shoulder/upper arm sit on it and would
# only produce contacts against a fixed joint; SURVEY.md §8 a16 robot filter 0b1 vs table 0)
NO_TABLE_CONTACT = {"shoulder_link", "upper_arm_link"}


def build_model(scene, pool_names=None):
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
    m.base_pos[:] = rob["base_pos"]
    m.base_quat[:] = rob["base_quat"]
    objects = scene["objects"]
    if pool_names is not None:
        byname = {o["name"]: o for o in objects}
        objects = [byname[n] for n in pool_names]
    table = scene.get("table")
    hulls = [(h, h["index"]) for h in scene["link_hulls"]] + [(o["hull"], -1) for o in objects] + \
            ([(table["hull"], -1)] if table else [])
    assert len(hulls) <= MAX_HULLS
    vs, ps = 0, 0
    verts = np.ctypeslib.as_array(m.verts)
    planes = np.ctypeslib.as_array(m.planes)
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
        vs += len(v)
        ps += len(p)
    assert vs <= MAX_VERTS and ps <= MAX_PLANES
    m.n_link_hulls = len(scene["link_hulls"])
    m.n_pool = len(objects)
    m.n_hulls = len(hulls)
    for i, o in enumerate(objects):
        m.pool_hull[i] = m.n_link_hulls + i
        m.pool_mass[i] = o["mass"]
        m.pool_com[i][:] = o["com"]
        m.pool_inertia[i][:] = o["inertia"]
        m.pool_bbox_pos[i][:] = o.get("bbox_from_origin_pos", (0, 0, 0))
        m.pool_bbox_quat[i][:] = o.get("bbox_from_origin_quat", (0, 0, 0, 1))
        m.pool_bbox_ext[i][:] = o.get("bbox_extents", (0, 0, 0))
    if table:
        m.table_hull = len(hulls) - 1
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
    return m


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
    joint_limit_margin=0.02, n_objects=3, num_initial_poses=1, max_episode_length=200,
    sih_alpha=0.8, reward_reaching=1.0, reward_lifting=5.0, reward_goal=50.0, reward_success=50.0,
    lifting_threshold=0.05, goal_threshold=0.05, goal_pos=(0.28, 0.58, 0.8), goal_noise=(0.15, 0.15, 0.1),
    dr_enable=0, dr_mass=(0.5, 1.5), dr_friction=(0.7, 1.3), dr_friction_buckets=250, dr_obs_noise=0.002,
    dr_act_noise=0.05,     # BASELINE config 4 "DR on" (ranges of AllegroKuka.yaml:121-207)
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
    contact_margin=0.002, max_depen_vel=1000.0,                          # contact_offset, max_depenetration_velocity
    max_episode_length=600,                                              # episodeLength
    dist_reward_scale=-10.0, rot_reward_scale=1.0, rot_eps=0.1, action_penalty_scale=-0.0002,
    success_tolerance=0.1, reach_goal_bonus=250.0, fall_dist=0.24, fall_penalty=0.0,
    max_consecutive_successes=0, av_factor=0.1,                          # allegro_hand.py:79 averFactor default
    reset_position_noise=0.01, reset_dof_pos_noise=0.2, reset_dof_vel_noise=0.0, act_moving_average=1.0,
    vel_obs_scale=0.2, force_torque_obs_scale=10.0,                      # allegro_hand.py:57-58
    clip_observations=5.0, clip_actions=1.0,
    # hand at (0, 0, 0.5); object at hand + (0, -0.2, 0.06); goal_states = object - 0.04 z; goal actor at
    # goal_states + displacement (allegro_hand.py:284-300,363-365)
    object_init=(0.0, -0.2, 0.56, 0.0, 0.0, 0.0, 1.0), goal_init=(0.0, -0.2, 0.52),
    goal_displacement=(-0.2, -0.06, 0.12),
)


def build_params(cfg=None, task=None):
    c = dict(ALLEGRO_TASK if (task == TASK_ALLEGRO_HAND or (cfg or {}).get("task") == TASK_ALLEGRO_HAND)
             else DEFAULT_TASK)
    if cfg:
        c.update(cfg)
    p = HaParams()
    for k in ["dt", "substeps", "control_freq_inv", "solver_iters", "friction", "contact_margin", "baumgarte",
              "max_depen_vel", "object_ang_damping", "joint_limit_margin", "n_objects", "num_initial_poses",
              "max_episode_length", "sih_alpha", "reward_reaching", "reward_lifting", "reward_goal",
              "reward_success", "lifting_threshold", "goal_threshold", "seed"]:
        setattr(p, k, c[k])
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
    p.dr_enable = int(c.get("dr_enable", 0))
    p.dr_mass_lo, p.dr_mass_hi = c.get("dr_mass", (0.5, 1.5))
    p.dr_fric_lo, p.dr_fric_hi = c.get("dr_friction", (0.7, 1.3))
    p.dr_fric_buckets = int(c.get("dr_friction_buckets", 250))
    p.dr_obs_noise = c.get("dr_obs_noise", 0.002)
    p.dr_act_noise = c.get("dr_act_noise", 0.05)
    p.task = c.get("task", TASK_UR5SIH)
    p.num_actions = c.get("num_actions", 11)
    p.num_obs = c.get("num_obs", 147)
    if p.task == TASK_ALLEGRO_HAND:
        for k in ["dist_reward_scale", "rot_reward_scale", "rot_eps", "action_penalty_scale", "success_tolerance",
                  "reach_goal_bonus", "fall_dist", "fall_penalty", "max_consecutive_successes", "av_factor",
                  "reset_position_noise", "reset_dof_pos_noise", "reset_dof_vel_noise", "act_moving_average",
                  "vel_obs_scale", "force_torque_obs_scale"]:
            setattr(p, "ah_" + k, c[k])
        p.ah_object_init[:] = c["object_init"]
        p.ah_goal_init[:] = c["goal_init"]
        p.ah_goal_displacement[:] = c["goal_displacement"]
        # (1.0 - act_moving_average) * prev_targets: python double, cast once (allegro_hand.py:612-613)
        p.sih_beta = 1.0 - c["act_moving_average"]
        p.action_dt = c["dt"]
    return p, c
