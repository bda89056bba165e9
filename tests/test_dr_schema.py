"""The DR engine's restatement (oracle/dr_oracle.py, which csrc/ha_dr.h matches bit for bit on the GPU:
tests/test_gpu_dr_schema.py) against the REFERENCE's apply_randomizations run with recorded draws
(tests/golden/make_goldens_dr.py -> dr_reference.npz, dr_schemas.json), and the schema parser (handarm_hip/dr.py).

Pinned against the reference, per call of a 10-call sequence for AllegroKuka.yaml's and AllegroHand.yaml's schemas
(frequency 3, frames crossing the 30000-frame schedules):
* the frequency gate: which envs are re-randomized, the non-env randomization frames (last_rand_step), the
  randomize_buf counts after the call (the first call leaves them);
* the observation / action noise parameters each non-env randomization stores, under the schedules;
* every property value set (DOF damping / stiffness / lower / upper, link and object mass, friction with its
  250-bucket grid, object scale, gravity), fed the same draws: scheduled ranges, distributions, operations, buckets,
  setup_only;
* the noise lambdas on a fixed tensor with the same correlated / white draws.
"""
import copy
import json
import os

import numpy as np
import pytest

from handarm_hip import dr as DR
from handarm_hip import model as HM
from oracle import dr_oracle as DO

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
F = np.float32
# (property kind, attribute) codes of make_goldens_dr.py -> HA_DRA_*
PK_SIM, PK_DOF, PK_BODY, PK_SHAPE, PK_SCALE = range(5)
ATTRS = ["gravity", "damping", "stiffness", "lower", "upper", "mass", "friction", "scale"]


@pytest.fixture(scope="module")
def ref():
    return np.load(os.path.join(G, "dr_reference.npz"))


def _params(task, schema, frequency=3):
    sc = copy.deepcopy(schema)
    sc["frequency"] = frequency
    p, _ = HM.build_params({"dr_enable": 1, "randomization_params": sc}, task=task)
    return p


def _setup(name):
    if name == "kuka":
        task, asset, schema = HM.TASK_ALLEGRO_KUKA, HM.KUKA_ASSET, DR.ALLEGRO_KUKA_SCHEMA
    else:
        task, asset, schema = HM.TASK_ALLEGRO_HAND, HM.ALLEGRO_ASSET, DR.ALLEGRO_HAND_SCHEMA
    return _params(task, schema), HM.build_model(HM.load_scene(asset))


def test_schemas_are_the_reference_yaml():
    """dr.ALLEGRO_KUKA_SCHEMA / ALLEGRO_HAND_SCHEMA are cfg/task/AllegroKuka.yaml:115-207 / AllegroHand.yaml:68-150
    as yaml.safe_load reads them (AllegroKuka's `sim_params: None` and its stray top-level `gravity` included)."""
    with open(os.path.join(G, "dr_schemas.json")) as f:
        ref = json.load(f)
    assert ref["AllegroKuka"] == json.loads(json.dumps(DR.ALLEGRO_KUKA_SCHEMA))
    assert ref["AllegroHand"] == json.loads(json.dumps(DR.ALLEGRO_HAND_SCHEMA))


@pytest.mark.parametrize("name", ["kuka", "hand"])
def test_frequency_gate_and_first_randomization(ref, name):
    p, m = _setup(name)
    N = ref[f"{name}_reset"].shape[1]
    g = DR.init_global(p)
    gi = g.view(np.int32)
    for c in range(len(ref[f"{name}_frame"])):
        gi[HM.DRG_FRAME_NEXT] = int(ref[f"{name}_frame"][c])
        DO.global_update(p, g, True, 1)
        assert gi[HM.DRG_LAST_RAND] == ref[f"{name}_last_rand"][c], f"call {c}"
        assert gi[HM.DRG_ALL] == (1 if c == 0 else 0)
        rb = ref[f"{name}_rb_before"][c].astype(np.int32).copy()
        reset = ref[f"{name}_reset"][c] != 0
        rows = DR.default_rows(m, p, N)
        smp = DO.env_pre(p, m, rows, rb, np.zeros(N, np.uint32), np.zeros((N, 1), np.int64), reset, g, False)
        np.testing.assert_array_equal(smp, ref[f"{name}_randomized"][c], err_msg=f"call {c}")
        np.testing.assert_array_equal(rb, ref[f"{name}_rb_after"][c], err_msg=f"call {c}")


@pytest.mark.parametrize("name", ["kuka", "hand"])
def test_noise_parameters_under_schedules(ref, name):
    """mu / var / mu_corr / var_corr of the observations and actions at each non-env randomization."""
    p, _ = _setup(name)
    for c in np.nonzero(ref[f"{name}_nonenv"])[0]:
        frame = int(ref[f"{name}_frame"][c])
        for key, attr in (("obs_params", HM.DRA_OBS), ("act_params", HM.DRA_ACT)):
            mu, var, mu_c, var_c = ref[f"{name}_{key}"][c]
            P = DO.noise_params(p.dr_attr[attr], frame)
            np.testing.assert_array_equal(P, np.array([var_c, mu_c, var, mu], F), err_msg=f"{key} call {c}")


def _attr_of(pk, actor, attr):
    a = ATTRS[int(attr)]
    if pk == PK_SIM:
        return HM.DRA_GRAVITY
    if pk == PK_SCALE:
        return HM.DRA_OBJ_SCALE
    if pk == PK_DOF:
        return {"damping": HM.DRA_DOF_KD, "stiffness": HM.DRA_DOF_KP, "lower": HM.DRA_DOF_LOWER,
                "upper": HM.DRA_DOF_UPPER}[a]
    robot = actor == 0
    if a == "mass":
        return HM.DRA_LINK_MASS if robot else HM.DRA_OBJ_MASS
    return HM.DRA_LINK_FRIC if robot else HM.DRA_OBJ_FRIC


@pytest.mark.parametrize("name", ["kuka", "hand"])
def test_property_values_from_the_same_draws(ref, name):
    """Each property value the reference set, recomputed by the restatement from the same draw: the scheduled range,
    the distribution, the operation on the nominal value and the bucket grid."""
    p, m = _setup(name)
    vals = ref[f"{name}_values"]
    frames = ref[f"{name}_frame"]
    assert len(vals) > 500
    nominal = {HM.DRA_DOF_KD: list(m.dof_kd), HM.DRA_DOF_KP: list(m.dof_kp), HM.DRA_DOF_LOWER: list(m.dof_lower),
               HM.DRA_DOF_UPPER: list(m.dof_upper), HM.DRA_LINK_MASS: list(m.link_mass)}
    seen, edge = set(), 0
    for call, env, pk, actor, elem, attr, kind, draw, value in vals:
        k = _attr_of(int(pk), int(actor), attr)
        a = p.dr_attr[k]
        assert a.dist != 0, f"{ATTRS[int(attr)]}: randomized by the reference, off in the parsed schema"
        seen.add(k)
        if k == HM.DRA_LINK_MASS and call > 0:
            # after the first randomization the robot's bodies zip with the object's original_props entry
            assert a.later_elems == 1 and a.later_og_object and int(elem) == 0
            og = F(m.pool_mass[0])
        elif k in nominal:
            og = F(nominal[k][int(elem)])
        elif k == HM.DRA_GRAVITY:
            # the original gravity is the first call's prop, rewritten in place by that call (aliasing in
            # original_props): later samples apply to the first call's result
            og = F([0.0, 0.0, -9.81][int(elem)]) if call == 0 else F(ref[f"{name}_gravity"][0][int(elem)])
        elif k == HM.DRA_OBJ_MASS:
            og = F(m.pool_mass[0])
        else:
            og = F(1.0)
        r0, r1 = DO.scheduled_range(a, int(frames[int(call)]))
        u, g = (F(draw), 0) if kind == 0 else (0, F(draw))
        mine = float(DO.value(a, r0, r1, og, u, g))
        if a.num_buckets > 0 and abs(mine - value) > 1e-6:
            # a draw within rounding of a bucket edge may land in the neighbouring bucket (float32 vs double)
            w = (a.range[1] - a.range[0]) / a.num_buckets
            assert abs(abs(mine - value) - w) < 1e-5, (ATTRS[int(attr)], call, env, mine, value)
            edge += 1
            continue
        np.testing.assert_allclose(mine, value, rtol=2e-6, atol=2e-7, err_msg=f"{ATTRS[int(attr)]} call {call}")
    assert edge <= 2
    want = {HM.DRA_DOF_KD, HM.DRA_DOF_KP, HM.DRA_DOF_LOWER, HM.DRA_DOF_UPPER, HM.DRA_LINK_MASS, HM.DRA_LINK_FRIC,
            HM.DRA_OBJ_MASS, HM.DRA_OBJ_FRIC, HM.DRA_OBJ_SCALE} | ({HM.DRA_GRAVITY} if name == "hand" else set())
    assert seen == want


def test_setup_only_is_sampled_at_the_first_randomization_only(ref):
    """AllegroHand.yaml's setup_only mass / scale: set by the setup call, never again (vec_task.py:834-864); the
    parser marks them, and the restatement gates them the same way."""
    vals = ref["hand_values"]
    later = vals[vals[:, 0] > 0]
    assert not np.isin(later[:, 5], [ATTRS.index("mass"), ATTRS.index("scale")]).any()
    p, _ = _setup("hand")
    for k in (HM.DRA_LINK_MASS, HM.DRA_OBJ_MASS, HM.DRA_OBJ_SCALE):
        assert p.dr_attr[k].setup_only == 1 and DO.active(p, k, True) and not DO.active(p, k, False)
    assert not p.dr_attr[HM.DRA_DOF_KD].setup_only and not p.dr_attr[HM.DRA_LINK_FRIC].setup_only


@pytest.mark.parametrize("name", ["kuka", "hand"])
def test_noise_lambdas(ref, name):
    """noise_lambda (vec_task.py:718-726) on a fixed tensor with the same correlated / white draws."""
    p, _ = _setup(name)
    c = int(np.nonzero(ref[f"{name}_nonenv"])[0][-1])
    frame = int(ref[f"{name}_frame"][c])
    for key, attr in (("observations", HM.DRA_OBS), ("actions", HM.DRA_ACT)):
        x, corr, white, y = (ref[f"{name}_noise_{key}_{k}"] for k in ("x", "corr", "white", "y"))
        P = DO.noise_params(p.dr_attr[attr], frame)
        n = ((corr * P[0] + P[1]) + white * P[2]) + P[3]
        np.testing.assert_array_equal((x + n).astype(F), y)


def test_parser_refuses_what_is_not_built():
    base = copy.deepcopy(DR.ALLEGRO_KUKA_SCHEMA)
    for bad in ({"actor_params": {"table": {"rigid_body_properties": {"mass": {"range": [0.5, 1.5],
                                                                              "operation": "scaling",
                                                                              "distribution": "uniform"}}}}},
                {"actor_params": {"allegro": {"tendon_properties": {}}}},
                {"actor_params": {"allegro": {"dof_properties": {"friction": {"range": [0, 1], "operation": "scaling",
                                                                               "distribution": "uniform"}}}}},
                {"sim_params": {"rest_offset": {"range": [0, 0.01], "operation": "additive",
                                                "distribution": "uniform"}}},
                {"observations": {"range": [0.5, 1], "operation": "scaling", "distribution": "loguniform"}},
                {"something": 1}):
        sc = copy.deepcopy(base)
        sc.update(bad)
        with pytest.raises(NotImplementedError):
            DR.parse(sc, HM.TASK_ALLEGRO_KUKA)


def test_parser_setup_only_rules():
    """A property group with one setup_only attribute is setup-only as a whole (set_random_properties = False,
    vec_task.py:843-864); AllegroKuka drops setup_only attributes (its first randomization is after sim_initialized)."""
    sc = copy.deepcopy(DR.ALLEGRO_HAND_SCHEMA)
    sc["actor_params"]["hand"]["dof_properties"]["damping"]["setup_only"] = True
    _, attrs = DR.parse(sc, HM.TASK_ALLEGRO_HAND)
    for k in (HM.DRA_DOF_KD, HM.DRA_DOF_KP, HM.DRA_DOF_LOWER, HM.DRA_DOF_UPPER):
        assert attrs[k].setup_only
    sck = copy.deepcopy(DR.ALLEGRO_KUKA_SCHEMA)
    sck["actor_params"]["object"]["scale"]["setup_only"] = True
    _, attrs = DR.parse(sck, HM.TASK_ALLEGRO_KUKA)
    assert HM.DRA_OBJ_SCALE not in attrs and HM.DRA_OBJ_MASS in attrs
    # AllegroKuka.yaml's sim_params: None + stray gravity: no gravity randomization, no error
    _, attrs = DR.parse(DR.ALLEGRO_KUKA_SCHEMA, HM.TASK_ALLEGRO_KUKA)
    assert HM.DRA_GRAVITY not in attrs


def test_allegro_tasks_refuse_unbuilt_config_and_accept_randomize():
    """AllegroKuka / AllegroHand raise on config they do not build instead of ignoring it (verdict r05 Weak #9); the
    DR flag builds its params (the GPU runs it: tests/test_gpu_dr_schema.py)."""
    p, _ = HM.build_params({"dr_enable": 1, "randomization_params": None}, task=HM.TASK_ALLEGRO_KUKA)
    assert p.dr_enable == 1 and p.dr_frequency == 480
    assert p.dr_attr[HM.DRA_DOF_KD].dist == HM.DR_DIST["loguniform"]
    p, _ = HM.build_params({"dr_enable": 1}, task=HM.TASK_ALLEGRO_HAND)
    assert p.dr_frequency == 720 and p.dr_attr[HM.DRA_GRAVITY].dist == HM.DR_DIST["gaussian"]
    p, _ = HM.build_params({"privileged_actions": True}, task=HM.TASK_ALLEGRO_KUKA)
    assert p.num_actions == 26 and abs(p.ak_privileged_torque - 0.02) < 1e-9


def test_log_exp_restatement_matches_the_c_oracle():
    """f32.logf / expf (numpy) == include/ha_fmath.h ha_logf / ha_expf as compiled into the C oracle, bit for bit."""
    import ctypes as C
    from oracle import f32, oracle_lib
    lib = oracle_lib.load()
    lib.hao_logexp.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(2 ** -24, 1, 20000), np.exp(rng.uniform(-20, 20, 20000))]).astype(F)
    lo, ex = np.empty_like(x), np.empty_like(x)
    lib.hao_logexp(x.ctypes.data, x.size, lo.ctypes.data, ex.ctypes.data)
    np.testing.assert_array_equal(f32.logf(x).view(np.int32), lo.view(np.int32))
    xe = (x * F(1e-3) - F(3.0)).astype(F)
    np.testing.assert_array_equal(f32.expf(xe).view(np.int32), ex.view(np.int32))
    assert np.abs(f32.logf(x) - np.log(x.astype(np.float64))).max() < 2e-6
