"""Domain randomization schema: ``task.randomization_params`` -> ``ha_params_t.dr_attr`` (include/handarm_abi.h v16).

The reference's engine (tasks/base/vec_task.py:646-876 ``apply_randomizations``, utils/dr_utils.py:71-238) reads the
schema of cfg/task/AllegroKuka.yaml:115-207 / AllegroHand.yaml:68-150 on every call and loops over the reset envs on
the host. Here the schema is parsed once into one ``ha_dr_attr_t`` per randomized quantity; the device does the rest
(csrc/ha_dr.h): the frequency gate, the linear / constant schedules on the gym frame count, the per-env samples of
the actor properties at reset, gravity, and the white + correlated observation / action noise.

What is built, per key of the schema (anything else raises NotImplementedError):

* ``frequency`` (default 1).
* ``observations``, ``actions``: gaussian or uniform, additive or scaling, ``range``, ``range_correlated``,
  ``schedule`` / ``schedule_steps``.
* ``sim_params``: ``gravity`` (per-axis sample on the original gravity). ``sim_params: None`` is taken as empty: in
  AllegroKuka.yaml:136-142 ``gravity`` sits one level too high, so the reference's loop over ``sim_params.items()``
  would fail on None (vec_task.py:764); the stray top-level ``gravity`` key is not read by the reference, nor here.
* ``actor_params``: the task's robot actor (AllegroKuka ``allegro``, AllegroHand ``hand``, Ur5Sih ``robot``) with
  ``dof_properties`` damping / stiffness / lower / upper (per DOF), ``rigid_body_properties`` mass (per link; inertia
  scales with it) and ``rigid_shape_properties`` friction (per link: a link's shapes share one draw, PhysX's average
  combine with the other body); the ``object`` actor with ``scale``, mass and friction; ``color`` is accepted and
  ignored (no renderer). ``num_buckets`` snaps a value to get_bucketed_val's grid. One original value per property
  name (vec_task.py:828-832): with the object after the robot, later randomizations re-sample only the robot's first
  link, from the object's value (ha_dr_attr_t.later_elems / later_og_object). ``setup_only``: sampled at the
  first randomization only; a property group with one setup_only attribute is not re-applied after it
  (``set_random_properties = False``, vec_task.py:843-864). AllegroKuka runs its first apply_randomizations from
  reset_idx after the sim is initialised (vec_task.py:286-289, allegro_kuka_base.py:1248), so its setup_only
  attributes are never applied, as there.

The samples come from the device counter hash, not numpy's global generator: the distributions and schedules are the
reference's, the draws are not seed-faithful (parity: tests/test_dr_schema.py, tests/test_gpu_dr_schema.py).
"""
import copy

import numpy as np

from . import model as HM

# the actor names of each task's DR schema -> the build's two actor kinds
ACTORS = {HM.TASK_ALLEGRO_KUKA: {"allegro": "robot", "object": "object"},
          HM.TASK_ALLEGRO_HAND: {"hand": "robot", "object": "object"},
          HM.TASK_UR5SIH: {"robot": "robot", "object": "object"}}
# (actor kind, property, attribute) -> HA_DRA_*
PROPS = {("robot", "rigid_body_properties", "mass"): HM.DRA_LINK_MASS,
         ("robot", "rigid_shape_properties", "friction"): HM.DRA_LINK_FRIC,
         ("robot", "dof_properties", "damping"): HM.DRA_DOF_KD,
         ("robot", "dof_properties", "stiffness"): HM.DRA_DOF_KP,
         ("robot", "dof_properties", "lower"): HM.DRA_DOF_LOWER,
         ("robot", "dof_properties", "upper"): HM.DRA_DOF_UPPER,
         ("object", "rigid_body_properties", "mass"): HM.DRA_OBJ_MASS,
         ("object", "rigid_shape_properties", "friction"): HM.DRA_OBJ_FRIC}
ATTR_KEYS = {"range", "operation", "distribution", "schedule", "schedule_steps", "num_buckets", "setup_only"}

# cfg/task/AllegroKuka.yaml:115-207 (task.randomization_params), used when task.randomize is on and the cfg carries
# no schema of its own
ALLEGRO_KUKA_SCHEMA = {
    "frequency": 480,
    "observations": {"range": [0, .002], "range_correlated": [0, .001], "operation": "additive",
                     "distribution": "gaussian", "schedule": "linear", "schedule_steps": 40000},
    "actions": {"range": [0., .05], "range_correlated": [0, .015], "operation": "additive", "distribution": "gaussian",
                "schedule": "linear", "schedule_steps": 40000},
    "sim_params": None,
    "gravity": {"range": [0, 0.4], "operation": "additive", "distribution": "gaussian", "schedule": "linear",
                "schedule_steps": 40000},
    "actor_params": {
        "allegro": {
            "color": True,
            "dof_properties": {
                "damping": {"range": [0.3, 3.0], "operation": "scaling", "distribution": "loguniform",
                            "schedule": "linear", "schedule_steps": 30000},
                "stiffness": {"range": [0.75, 1.5], "operation": "scaling", "distribution": "loguniform",
                              "schedule": "linear", "schedule_steps": 30000},
                "lower": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian",
                          "schedule": "linear", "schedule_steps": 30000},
                "upper": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian",
                          "schedule": "linear", "schedule_steps": 30000}},
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                               "schedule": "linear", "schedule_steps": 30000}},
            "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3], "operation": "scaling",
                                                    "distribution": "uniform", "schedule": "linear",
                                                    "schedule_steps": 30000}}},
        "object": {
            "scale": {"range": [0.5, 2.0], "operation": "scaling", "distribution": "uniform", "schedule": "linear",
                      "schedule_steps": 1},
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                               "schedule": "linear", "schedule_steps": 30000}},
            "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3], "operation": "scaling",
                                                    "distribution": "uniform", "schedule": "linear",
                                                    "schedule_steps": 30000}}}},
}

# cfg/task/AllegroHand.yaml:68-150 (the reference's AllegroHand never calls apply_randomizations: allegro_hand.py only
# counts randomize_buf; the build runs the engine when task.randomize is on)
ALLEGRO_HAND_SCHEMA = {
    "frequency": 720,
    "observations": {"range": [0, .002], "range_correlated": [0, .001], "operation": "additive",
                     "distribution": "gaussian"},
    "actions": {"range": [0., .05], "range_correlated": [0, .015], "operation": "additive", "distribution": "gaussian"},
    "sim_params": {"gravity": {"range": [0, 0.4], "operation": "additive", "distribution": "gaussian"}},
    "actor_params": {
        "hand": {
            "color": True,
            "dof_properties": {
                "damping": {"range": [0.3, 3.0], "operation": "scaling", "distribution": "loguniform"},
                "stiffness": {"range": [0.75, 1.5], "operation": "scaling", "distribution": "loguniform"},
                "lower": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"},
                "upper": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"}},
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                               "setup_only": True}},
            "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3], "operation": "scaling",
                                                    "distribution": "uniform"}}},
        "object": {
            "scale": {"range": [0.95, 1.05], "operation": "scaling", "distribution": "uniform", "setup_only": True},
            "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                               "setup_only": True}},
            "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3], "operation": "scaling",
                                                    "distribution": "uniform"}}}},
}

# BASELINE config 4 "DR on": the reference's Ur5Sih DR flag has no consumer, so this is the build's own
# schema, with AllegroKuka.yaml's ranges: link / object mass x U[0.5, 1.5], friction x U[0.7, 1.3] in
# 250 buckets, obs noise N(0, 0.002), action noise N(0, 0.05); every reset re-randomizes the env (frequency 1)
UR5SIH_SCHEMA = {
    "frequency": 1,
    "observations": {"range": [0, .002], "operation": "additive", "distribution": "gaussian"},
    "actions": {"range": [0., .05], "operation": "additive", "distribution": "gaussian"},
    "actor_params": {
        "robot": {"rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling",
                                                     "distribution": "uniform"}},
                  "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3],
                                                          "operation": "scaling", "distribution": "uniform"}}},
        "object": {"rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling",
                                                      "distribution": "uniform"}},
                   "rigid_shape_properties": {"friction": {"num_buckets": 250, "range": [0.7, 1.3],
                                                           "operation": "scaling", "distribution": "uniform"}}}},
}
DEFAULT_SCHEMA = {HM.TASK_ALLEGRO_KUKA: ALLEGRO_KUKA_SCHEMA, HM.TASK_ALLEGRO_HAND: ALLEGRO_HAND_SCHEMA,
                  HM.TASK_UR5SIH: UR5SIH_SCHEMA}


def _attr(spec, where, noise=False, setup_only=False):
    """One schema entry -> HaDrAttr."""
    if not isinstance(spec, dict):
        raise NotImplementedError(f"randomization_params {where}: expected a mapping, got {spec!r}")
    extra = set(spec) - ATTR_KEYS - ({"range_correlated"} if noise else set())
    if extra:
        raise NotImplementedError(f"randomization_params {where}: keys {sorted(extra)} are not implemented")
    a = HM.HaDrAttr()
    dist = spec["distribution"]
    if dist not in ("uniform", "loguniform", "gaussian") or (noise and dist == "loguniform"):
        # vec_task.py:700-754 knows gaussian / uniform noise; dr_utils.py:98-130 the three property distributions
        raise NotImplementedError(f"randomization_params {where}: distribution {dist!r} is not implemented")
    if spec["operation"] not in HM.DR_OP:
        raise NotImplementedError(f"randomization_params {where}: operation {spec['operation']!r} is not implemented")
    sched = spec.get("schedule")
    if sched not in HM.DR_SCHED:
        raise NotImplementedError(f"randomization_params {where}: schedule {sched!r} is not implemented")
    a.dist, a.op, a.sched = HM.DR_DIST[dist], HM.DR_OP[spec["operation"]], HM.DR_SCHED[sched]
    a.sched_steps = int(spec.get("schedule_steps", 0)) if sched else 0
    if sched == "linear" and a.sched_steps < 1:
        raise ValueError(f"randomization_params {where}: a linear schedule needs schedule_steps >= 1")
    lo, hi = spec["range"]
    a.range[0], a.range[1] = float(lo), float(hi)
    if dist == "loguniform" and not (lo > 0 and hi > 0):
        raise ValueError(f"randomization_params {where}: a loguniform range must be positive")
    if noise:
        c0, c1 = spec.get("range_correlated", [0.0, 0.0])
        a.range_corr[0], a.range_corr[1] = float(c0), float(c1)
    a.num_buckets = int(spec.get("num_buckets", 0) or 0)
    a.setup_only = int(bool(spec.get("setup_only", False)) or setup_only)
    a.later_elems = -1
    return a


def parse(rp, task):
    """randomization_params -> (frequency, {HA_DRA_*: HaDrAttr}). NotImplementedError for any key not built."""
    if rp is None:
        rp = DEFAULT_SCHEMA[task]
    rp = copy.deepcopy(dict(rp))
    attrs = {}
    frequency = int(rp.pop("frequency", 1))
    if frequency < 1:
        raise ValueError("randomization_params frequency must be >= 1")
    for key, idx in (("observations", HM.DRA_OBS), ("actions", HM.DRA_ACT)):
        if key in rp:
            attrs[idx] = _attr(rp.pop(key), key, noise=True)
    sim = rp.pop("sim_params", None)
    if "gravity" in rp and sim is None:
        rp.pop("gravity")          # AllegroKuka.yaml's stray key: not read by the reference (module docstring)
    for attr, spec in (sim or {}).items():
        if attr != "gravity":
            raise NotImplementedError(f"randomization_params sim_params.{attr} is not implemented (gravity is)")
        attrs[HM.DRA_GRAVITY] = _attr(spec, "sim_params.gravity")
    actors = ACTORS[task]
    order = []                                   # (actor kind, property) in the schema's order
    for actor, props in (rp.pop("actor_params", None) or {}).items():
        if actor not in actors:
            raise NotImplementedError(f"randomization_params actor_params.{actor}: the {sorted(actors)} actors are "
                                      f"the ones implemented for this task")
        kind = actors[actor]
        for prop, pattrs in props.items():
            where = f"actor_params.{actor}.{prop}"
            if prop == "color":
                continue                                  # visual only (vec_task.py:803-809)
            if prop == "scale":
                if kind != "object":
                    raise NotImplementedError(f"randomization_params {where}: only the object actor's scale is "
                                              f"implemented")
                attrs[HM.DRA_OBJ_SCALE] = _attr(pattrs, where)
                continue
            if not isinstance(pattrs, dict) or not any(k[:2] == (kind, prop) for k in PROPS):
                raise NotImplementedError(f"randomization_params {where} is not implemented")
            order.append((kind, prop))
            # one setup_only attribute keeps the whole property from being set again (vec_task.py:843-864)
            group_setup = any(isinstance(v, dict) and v.get("setup_only", False) for v in pattrs.values())
            for attr, spec in pattrs.items():
                idx = PROPS.get((kind, prop, attr))
                if idx is None:
                    raise NotImplementedError(f"randomization_params {where}.{attr} is not implemented")
                attrs[idx] = _attr(spec, f"{where}.{attr}", setup_only=group_setup)
    if rp:
        raise NotImplementedError(f"randomization_params keys {sorted(rp)} are not implemented")
    # apply_randomizations keeps one original_props entry per property NAME, written by every actor at the first
    # randomization (vec_task.py:828-832): the actor processed last wins, and later randomizations zip the other
    # actor's bodies / shapes with that one entry. With the robot first and the object (one body, one shape in the
    # Allegro scenes) last, later randomizations re-sample only the robot's first link, from the object's nominal value
    for prop, idx in (("rigid_body_properties", HM.DRA_LINK_MASS), ("rigid_shape_properties", HM.DRA_LINK_FRIC)):
        kinds = [k for k, pr in order if pr == prop]
        if idx in attrs:
            attrs[idx].later_elems = -1
        if "robot" in kinds and "object" in kinds:
            if kinds.index("object") < kinds.index("robot"):
                raise NotImplementedError(f"randomization_params: the object's {prop} before the robot's (its shared "
                                          f"original_props entry would be the robot's) is not implemented")
            if idx in attrs:
                attrs[idx].later_elems = 1
                attrs[idx].later_og_object = 1
    if task == HM.TASK_ALLEGRO_KUKA:
        # the first apply_randomizations runs from reset_idx, after sim_initialized: setup_only never applies
        attrs = {k: a for k, a in attrs.items() if not a.setup_only}
    return frequency, attrs


def apply_schema(p, rp, task):
    """Write the parsed schema into HaParams p (dr_frequency, dr_attr)."""
    frequency, attrs = parse(rp, task)
    p.dr_frequency = frequency
    for k in range(HM.DRA_N):
        off = HM.HaDrAttr()
        off.later_elems = -1
        p.dr_attr[k] = attrs.get(k, off)


def default_rows(model, params, num_envs, object_mass=None):
    """dr_scale rows at the nominal values (mass ratio 1, friction, the model's DOF gains and limits, scale 1): what an
    env's physics reads until its first sample."""
    r = np.zeros((num_envs, HM.DR_SIZE), np.float32)
    r[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + HM.MAX_LINKS] = 1.0
    r[:, HM.DR_OBJ_MASS:HM.DR_OBJ_MASS + HM.MAX_OBJ] = 1.0
    r[:, HM.DR_LINK_FRIC:HM.DR_LINK_FRIC + HM.MAX_LINKS] = params.friction
    r[:, HM.DR_OBJ_FRIC:HM.DR_OBJ_FRIC + HM.MAX_OBJ] = params.friction
    for slot, name in ((HM.DR_DOF_KP, "dof_kp"), (HM.DR_DOF_KD, "dof_kd"), (HM.DR_DOF_LOWER, "dof_lower"),
                       (HM.DR_DOF_UPPER, "dof_upper")):
        r[:, slot:slot + HM.MAX_DOFS] = np.array(list(getattr(model, name)), np.float32)
    r[:, HM.DR_OBJ_SCALE:HM.DR_OBJ_SCALE + HM.MAX_OBJ] = 1.0
    return r


def init_global(params):
    """dr_global before the first step: frame 0, last_rand_step -1 (vec_task.py:281), first_randomization on,
    gravity = the sim params' (the randomized value replaces it at the first non-env randomization)."""
    g = np.zeros(HM.DRG_SIZE, np.float32)
    gi = g.view(np.int32)
    gi[HM.DRG_LAST_RAND] = -1
    gi[HM.DRG_FIRST] = 1
    g[HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3] = list(params.gravity)
    g[HM.DRG_GRAVITY_OG:HM.DRG_GRAVITY_OG + 3] = list(params.gravity)
    return g


def describe(params):
    """The active schema as a plain dict (for logs / the bench record)."""
    names = ["observations", "actions", "gravity", "link_mass", "link_friction", "dof_damping", "dof_stiffness",
             "dof_lower", "dof_upper", "object_mass", "object_friction", "object_scale"]
    dist = {v: k for k, v in HM.DR_DIST.items()}
    out = {"frequency": int(params.dr_frequency)}
    for k, n in enumerate(names):
        a = params.dr_attr[k]
        if a.dist:
            out[n] = {"distribution": dist[a.dist], "range": [float(a.range[0]), float(a.range[1])],
                      "operation": "scaling" if a.op else "additive", "schedule_steps": int(a.sched_steps)}
    return out
