"""Physics checks independent of the shared restatement (verdict r05 Weak #2 / Next #7).

ha_physics.h (kernel) and physics_oracle.c (oracle) are one restatement compiled twice, bit-identical to each other;
a defect they share cannot fail a kernel-vs-oracle test. tests/kinematics.py derives the same quantities in float64
from the scene JSON with textbook formulas (rotation-matrix FK, M = sum J^T M_i J, Coriolis from dM/dq by finite
differences, link damping from the COM Jacobians, the converged implicit PD drive step), so here:
* the oracle's rigid-body rows (FK: positions, quaternions with their sign, COM and angular velocities) equal the
  independent FK within float32 rounding, for the three robots (Ur5Sih, AllegroHand, AllegroKuka);
* one substep of the oracle's physics with the drive rows converged (solver_iters 4000, no contacts, no active
  limits, joint friction 0) equals the closed-form implicit PD step, with random joint velocities (Coriolis and link
  damping in play): this pins CRBA / the mass matrix with armature, RNEA's velocity-product forces, the drive rows'
  gamma / bias and the symplectic integration;
* the GPU kernel does the same on the device (``-m gpu``);
* the shared float32 math (include/ha_fmath.h: sincos, log, exp) is held against float64 numpy.
The AllegroKuka golden vectors' fingertip / palm rows come from this FK too (tests/golden/make_goldens_kuka.py)."""
import copy

import numpy as np
import pytest

from handarm_hip import model as HM
from tests.kinematics import Chain

ROBOTS = [(HM.TASK_UR5SIH, HM.ASSET), (HM.TASK_ALLEGRO_HAND, HM.ALLEGRO_ASSET), (HM.TASK_ALLEGRO_KUKA, HM.KUKA_ASSET)]
H = 1.0 / 120.0


def _scene_no_friction(asset):
    """The scene with the DOF friction rows off (their |impulse| <= mu |drive impulse| coupling has no closed form)."""
    s = copy.deepcopy(HM.load_scene(asset))
    for d in s["robot"]["dofs"]:
        d["friction"] = 0.0
    return s


def _case(model, params, n, seed):
    """Joint positions 0.1 rad around the reset pose, kept 0.08 rad inside the limits (no limit row active), random
    velocities, targets within 0.01 rad; objects parked far away with collisions off."""
    D = model.n_dofs
    rng = np.random.default_rng(seed)
    lo, up = np.array(list(model.dof_lower)[:D]), np.array(list(model.dof_upper)[:D])
    rp = np.array(list(params.reset_pose)[:D])
    q = np.clip(rp + rng.uniform(-0.1, 0.1, (n, D)), lo + 0.08, up - 0.08).astype(np.float32)
    qd = rng.uniform(-0.3, 0.3, (n, D)).astype(np.float32)
    tgt = (q + rng.uniform(-0.01, 0.01, (n, D))).astype(np.float32)
    return q, qd, tgt


def _fill(st, model, params, q, qd, tgt):
    n, D, A = q.shape[0], model.n_dofs, model.n_actors
    root = st["root_state"].reshape(n, A, 13)
    root[..., 6] = 1.0
    root[:, model.actor_object0:model.actor_object0 + params.n_objects, 0:3] = [5.0, 5.0, 5.0]
    if model.actor_table >= 0:
        root[:, model.actor_table, 0:3] = list(model.table_pos)
    st["collision_enabled"][:] = 0
    dof = st["dof_state"].reshape(n, D, 2)
    dof[..., 0], dof[..., 1] = q, qd
    st["sim_targets"][:] = tgt
    if params.task == HM.TASK_ALLEGRO_KUKA:
        st["object_scale"][:] = 1.0


def _check_step(chain, params, q, qd, tgt, out, tag):
    n = q.shape[0]
    for e in range(n):
        q1, v1 = chain.implicit_pd_step(q[e], qd[e], tgt[e], H, cl=params.link_lin_damping, ca=params.link_ang_damping)
        ev = np.abs(out[e, :, 1] - v1).max() / np.abs(v1).max()
        eq = np.abs(out[e, :, 0] - q1).max()
        assert ev < 3e-5 and eq < 1e-6, f"{tag} env {e}: joint velocity rel err {ev:.2e}, position err {eq:.2e}"


@pytest.mark.parametrize("task,asset", ROBOTS)
def test_oracle_fk_matches_independent_fk(task, asset):
    from oracle.oracle_lib import HostState, Oracle
    scene = HM.load_scene(asset)
    m = HM.build_model(scene)
    p, _ = HM.build_params(task=task)
    n, D = 6, m.n_dofs
    st = HostState(n, model=m, params=p)
    rng = np.random.default_rng(3)
    q = (rng.uniform(-0.6, 0.6, (n, D))).astype(np.float32)
    qd = rng.uniform(-1, 1, (n, D)).astype(np.float32)
    _fill(st, m, p, q, qd, q)
    Oracle(m, p, n).simulate(st, 0)                       # zero calls: the refresh (FK + link twists) only
    rb = st["rigid_body_state"].reshape(n, m.n_bodies, 13)[:, m.body_robot0:m.body_robot0 + m.n_links]
    ch = Chain(scene)
    for e in range(n):
        ref = ch.body_states(q[e], qd[e])
        np.testing.assert_allclose(rb[e], ref, rtol=0, atol=3e-6, err_msg=f"task {task} env {e}")


@pytest.mark.parametrize("task,asset", ROBOTS)
def test_oracle_drive_step_matches_closed_form(task, asset):
    from oracle.oracle_lib import HostState, Oracle
    scene = _scene_no_friction(asset)
    m = HM.build_model(scene)
    p, _ = HM.build_params({"solver_iters": 4000, "substeps": 1, "dt": H}, task=task)
    n = 8
    st = HostState(n, model=m, params=p)
    q, qd, tgt = _case(m, p, n, seed=task)
    _fill(st, m, p, q, qd, tgt)
    Oracle(m, p, n).simulate(st, 1)
    _check_step(Chain(scene), p, q, qd, tgt, st["dof_state"].reshape(n, m.n_dofs, 2), f"oracle task {task}")


@pytest.mark.gpu
@pytest.mark.parametrize("task,asset", ROBOTS)
def test_kernel_drive_step_matches_closed_form(task, asset):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState
    scene = _scene_no_friction(asset)
    sim = HandArmSim(64, "cuda:0", task_cfg={"task": task, "solver_iters": 4000, "substeps": 1, "dt": H}, task=task,
                     scene=scene)
    m, p = sim.model, sim.params
    n = 64
    st = HostState(n, model=m, params=p)
    for k in HM.STATE_FIELDS:
        if k not in HM.null_fields(task) and k not in ("stats", "term_sums"):
            st[k][...] = sim.t[k].cpu().numpy().reshape(st[k].shape)
    q, qd, tgt = _case(m, p, n, seed=10 + task)
    _fill(st, m, p, q, qd, tgt)
    for k in ("root_state", "dof_state", "sim_targets", "collision_enabled", "object_scale"):
        if k not in HM.null_fields(task):
            sim.t[k].copy_(torch.as_tensor(st[k]).reshape(sim.t[k].shape).to(sim.t[k].dtype))
    sim.simulate(1)
    torch.cuda.synchronize()
    out = sim.t["dof_state"].cpu().numpy().reshape(n, m.n_dofs, 2)
    _check_step(Chain(scene), p, q, qd, tgt, out, f"kernel task {task}")


def _ulp_err(got, ref):
    return np.abs(got.astype(np.float64) - ref) / np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)


def test_shared_float32_math_against_float64():
    """include/ha_fmath.h is one text compiled into the kernels and the C oracle, so a bit-identity test cannot see a
    defect in it. Here its sine / cosine, log and exp (as compiled into the oracle; the kernels are bit-identical to
    the oracle in every fused-step test) are held against float64 numpy: within 1.5 ulp of the float32-rounded exact
    value (sincos where |f| > 1e-3, absolute 8e-8 below that), log and exp within 1 ulp."""
    import ctypes as C
    from oracle import oracle_lib
    lib = oracle_lib.load()
    lib.hao_sincos.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.hao_logexp.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    F = np.float32
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-3.2, 3.2, 100000), rng.uniform(-2000, 2000, 100000)]).astype(F)
    s, c = np.empty_like(x), np.empty_like(x)
    lib.hao_sincos(x.ctypes.data, x.size, s.ctypes.data, c.ctypes.data)
    for got, ref in ((s, np.sin(x.astype(np.float64))), (c, np.cos(x.astype(np.float64)))):
        big = np.abs(ref) > 1e-3
        assert _ulp_err(got[big], ref[big]).max() < 1.5
        assert np.abs(got[~big] - ref[~big]).max() < 8e-8
    xl = np.concatenate([rng.uniform(2 ** -24, 1, 100000), np.exp(rng.uniform(-80, 80, 100000))]).astype(F)
    y = rng.uniform(-80, 80, xl.size)
    xe = ((y + 3.0) / 1e-3).astype(F)                 # hao_logexp's exp argument is 1e-3 x - 3 (float32)
    lo, _ = np.empty_like(xl), np.empty_like(xl)
    lib.hao_logexp(xl.ctypes.data, xl.size, lo.ctypes.data, _.ctypes.data)
    ref = np.log(xl.astype(np.float64))
    big = np.abs(ref) > 1e-3
    assert _ulp_err(lo[big], ref[big]).max() < 1.0
    _, ex = np.empty_like(xe), np.empty_like(xe)
    lib.hao_logexp(xe.ctypes.data, xe.size, _.ctypes.data, ex.ctypes.data)
    arg = (xe * F(1e-3)).astype(F) - F(3.0)
    assert _ulp_err(ex, np.exp(arg.astype(np.float64))).max() < 1.0
