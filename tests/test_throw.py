"""AllegroKuka throw (tasks/allegro_kuka/allegro_kuka_throw.py, cfg/task/env/throw.yaml) on the CPU: the bucket as
convex pieces carried by the actor in the goal slot (ha_model_t v14 posed statics) on the C physics oracle, the
subtask's config, and its host surface. The task math is pinned by the reference-run goldens
(tests/test_kuka_golden.py, kuka_*_throw.npz); the kernel is compared with these oracles in test_gpu_kuka.py
(goldens, bucket drop) and test_gpu_fused_steps.py (the fused step with the bucket at the hand)."""
import numpy as np

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes

BUCKET_FLOOR = 0.009911          # meshes/bucket.obj inner floor height (bucket frame)


def setup(n, bucket, seed=0):
    scene = HM.load_scene(HM.KUKA_ASSET)
    params, cfg = HM.build_params({"subtask": "throw"}, task=HM.TASK_ALLEGRO_KUKA)
    model = HM.build_model(scene, posed=HM.posed_group(HM.TASK_ALLEGRO_KUKA, cfg))
    lo, up = np.array(model.dof_lower[:23], np.float32), np.array(model.dof_upper[:23], np.float32)
    scales, _ = HM.kuka_env_tables(n, scene, cfg)
    st = HostState(n, model=model, params=params)
    scenes.fill_kuka_scene(st, n, lo, up, list(params.reset_pose), scales, list(model.table_pos), seed=seed)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 3] = 0
    root[:, 3, 0:3] = bucket
    root[:, 3, 6] = 1
    return scene, model, params, st, scales


def test_throw_config_and_model():
    """env/throw.yaml over AllegroKuka.yaml: 300-step episodes, no random forces, a fixed 7.5 cm tolerance (so the
    curriculum never moves it and true_objective = successes + 1), 5 success steps, one keypoint (99 observations),
    small cuboids; the bucket's 13 pieces follow the table as statics carried by actor 3."""
    scene = HM.load_scene(HM.KUKA_ASSET)
    p, cfg = HM.build_params({"subtask": "throw"}, task=HM.TASK_ALLEGRO_KUKA)
    assert (p.ak_subtask, p.max_episode_length, p.ak_success_steps, p.ak_force_scale) == (2, 300, 5, 0.0)
    assert p.num_obs == 99 and p.ak_num_keypoints == 1
    np.testing.assert_array_equal(HM.kuka_tolerance_scalars(cfg["success_tolerance"], cfg),
                                  np.array([0.075, 1.0, 0.0, 0.075 * 1.5], np.float32))
    assert abs(p.ak_bonus_rew - 1000.0 / 5) < 1e-4
    m = HM.build_model(scene, posed="bucket")
    assert m.n_static == 14 and m.posed_actor == 3 and list(m.static_posed)[:14] == [0] + [1] * 13
    assert HM.build_model(scene).posed_actor == -1 and HM.build_model(scene).n_static == 1
    dims = np.array(scene["object_dims_throw"])
    assert dims.max() <= 3.0 and (dims.prod(1) <= 2.5 + 1e-9).all()          # small cuboids: volume <= 2.5 x cube


def test_bucket_pieces_follow_the_mesh():
    """The pieces span the mesh's rim height and outer radius, the floor slab's top is the mesh's inner floor and it
    reaches 3 cm under the bottom (tools/build_model.py bucket_pieces), every piece's hull lies inside its static box
    (the broad phase's cull) and holds its vertices within its planes."""
    scene = HM.load_scene(HM.KUKA_ASSET)
    pieces = scene["posed_statics"]["bucket"]["pieces"]
    assert len(pieces) == 13
    verts = []
    for pc in pieces:
        v = np.array(pc["hull"]["verts"])
        assert (np.abs(v) <= np.array(pc["half_extents"])).all()
        verts.append(v + np.array(pc["pos"]))
    allv = np.concatenate(verts)
    # the rim is 0.198 high, the outer radius 0.12 (bucket.obj); the floor slab's top is the inner floor
    assert abs(allv[:, 2].max() - 0.197743) < 1e-6 and abs(allv[:, 2].min() - (0.000047 - 0.03)) < 1e-6
    assert abs(verts[0][:, 2].max() - BUCKET_FLOOR) < 1e-6
    r = np.hypot(allv[:, 0], allv[:, 1] + 0.002016)
    assert abs(r.max() - 0.12) < 1e-5
    for pc in pieces:
        pl = np.array(pc["hull"]["planes"])
        ctr = np.array(pc["pos"])
        # each piece contains its own vertices within 1e-9 of its planes
        v = np.array(pc["hull"]["verts"])
        assert (v @ pl[:, :3].T + pl[:, 3] <= 1e-9).all()
        assert np.isfinite(ctr).all()


def test_cuboid_dropped_into_the_bucket_rests_on_its_floor():
    """A 5 cm cube dropped into buckets hanging at different places of the arena (fixed base, like the reference's
    fix_base_link) comes to rest on the bucket's floor inside its wall, in every env."""
    n = 4
    buckets = np.array([[0.7, -0.3, 0.2], [-0.7, -0.5, 0.05], [0.6, 0.4, 0.6], [-0.85, -0.9, 0.9]], np.float32)
    scene, model, params, st, scales = setup(n, buckets)
    root = st["root_state"].reshape(n, 4, 13)
    st["object_scale"][:] = 1.0
    root[:, 1] = 0
    root[:, 1, 0:3] = buckets + [0.01, -0.02, 0.12]
    q = np.array([0.1, 0.05, 0.0, 1.0])
    root[:, 1, 3:7] = q / np.linalg.norm(q)
    orc = Oracle(model, params, n)
    for _ in range(90):
        st["dof_state"].reshape(n, 23, 2)[..., 1] = 0
        orc.simulate(st, 1)
    obj = root[:, 1]
    assert np.isfinite(obj).all()
    np.testing.assert_allclose(obj[:, 2], buckets[:, 2] + BUCKET_FLOOR + 0.025, atol=2.5e-3)
    d = np.hypot(obj[:, 0] - buckets[:, 0], obj[:, 1] - buckets[:, 1] + 0.002016)
    assert (d < 0.07).all(), d
    assert np.abs(obj[:, 7:13]).max() < 0.05
    assert (st["contact_stats"][:, 3] > 0).all()


def test_the_pieces_follow_the_bucket_actor():
    """The posed statics read the actor's root state at each call: moving the bucket out from under a resting cube
    (as _reset_target does) lets it fall, and the bucket pose of one env does not affect another."""
    n = 2
    buckets = np.array([[0.7, -0.3, 0.3], [0.7, -0.3, 0.3]], np.float32)
    scene, model, params, st, scales = setup(n, buckets)
    root = st["root_state"].reshape(n, 4, 13)
    st["object_scale"][:] = 1.0
    root[:, 1] = 0
    root[:, 1, 0:3] = buckets + [0.0, -0.002016, BUCKET_FLOOR + 0.025 + 0.001]
    root[:, 1, 6] = 1
    orc = Oracle(model, params, n)
    for _ in range(20):
        orc.simulate(st, 1)
    z_rest = root[:, 1, 2].copy()
    root[1, 3, 0] += 0.5                                  # env 1's bucket moves away, env 0's stays
    for _ in range(20):
        orc.simulate(st, 1)
    assert abs(root[0, 1, 2] - z_rest[0]) < 1e-3
    assert root[1, 1, 2] < z_rest[1] - 0.2                # ~20 calls of free fall
