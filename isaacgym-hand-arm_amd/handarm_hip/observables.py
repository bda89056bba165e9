"""Observation lists of Ur5SihMultiObjectManipulation: post-step order and the obs-vector layout.

The reference computes observables in the order ``ActiveObservables.sort`` gives
(tasks/hand_arm/utils/observables.py:219-257): the active set is every ``required`` observable in
registration order (observable_vec_task.py:105-108) followed by the observation and teacher lists (:19-21);
the dependency graph is built by popping from the end of that list and the post-step order is the reversed
``networkx.topological_sort``. The order matters because observables read each other's buffers: an
observable refreshed before ``object_pos`` / ``object_quat`` sees the object pose of the previous refresh
(object_bounding_box in the default lists; object_synthetic_pointcloud in some point-cloud lists). This module
restates that sort over the registration table extracted from the reference
(assets/ur5sih_observables.json, tests/golden/make_observables_table.py); networkx is the image's 3.4.2 (the
reference pins no version, so the tie order between independent observables is "parity unpinned" beyond it,
and pinned for the two point-cloud lists by tests/golden/ur5sih_pointclouds_*.npz).
"""
import json
import os

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "ur5sih_observables.json")

# default teacher / observation list (Ur5SihMultiObjectManipulation.yaml:24-26,43-44) and its block sizes
DEFAULT_OBSERVATIONS = ["ur5_joint_pos", "ur5_flange_pose", "sih_fingertip_pos", "sih_fingertip_quat",
                        "sih_fingertip_linvel", "dof_position_targets", "object_pos", "object_bounding_box",
                        "target_object_bounding_box", "sih_fingertip_to_target_object_pos",
                        "target_object_to_goal_pos"]

# synthetic point-cloud observables this build produces (ha_pointclouds) -> number of points (None = per model)
POINTCLOUDS = ["object_synthetic_pointcloud", "target_object_synthetic_pointcloud", "ur5sih_synthetic_pointcloud",
               "sih_fingertip_pointcloud", "goal_synthetic_pointcloud", "relative_goal_synthetic_pointcloud"]


def default_sizes(n_objects):
    """Block sizes of DEFAULT_OBSERVATIONS for n objects (object_pos 3 and object_bounding_box 10 per object,
    multi_object.py:128,245)."""
    return [6, 7, 15, 20, 15, 17, 3 * n_objects, 10 * n_objects, 10, 15, 3]


def registry():
    with open(ASSET) as f:
        return json.load(f)["observables"]


def post_step_order(observations, teacher_observations):
    """ActiveObservables.sort restated (observables.py:231-257)."""
    import networkx as nx
    reg = {}
    active = []
    for o in registry():
        reg[o["name"]] = o["requires"]
        if o["required"] and o["name"] not in active:
            active.append(o["name"])
    for name in list(observations) + list(teacher_observations):
        if name not in reg:
            raise KeyError(f"observable {name!r} is not registered by Ur5SihMultiObject")
        if name not in active:
            active.append(name)
    graph = {}
    explore = list(active)
    while explore:
        cur = explore.pop()
        graph[cur] = []
        for r in reg[cur]:
            if r not in graph:
                explore.append(r)
            graph[cur].append(r)
    return list(reversed(list(nx.topological_sort(nx.DiGraph(graph)))))


def sees_previous_object_pose(order, name):
    """True when observable `name` is refreshed before object_pos / object_quat, i.e. reads the object pose
    of the previous refresh."""
    i = order.index(name)
    return i < order.index("object_pos") or i < order.index("object_quat")


# ha_gather_obs sources of a custom observation list (include/handarm_abi.h): the step kernel's obs row, goal_pos,
# the refreshed gym tensors and the per-env object properties
SRC_OBS, SRC_GOAL, SRC_ROOT, SRC_BODY, SRC_DOF, SRC_PROPS = range(6)
SRC_TARGET = 16                 # HA_OBS_SRC_TARGET: + target_object_index * 13 (the target object's root row)
TIP_LINKS = [28, 15, 21, 24, 18]  # thumb, index, middle, ring, little fingertip links (ur5sih.py:609-614)
PROPS = 13                      # object_props row per object: mass, com (3), inertia (9)


def default_layout(n_objects):
    """Env layout of the Ur5SihMultiObject gym tensors without a bin (multi_object.py:562-663)."""
    return dict(a0=3, body_robot0=1, n_dofs=17)


def obs_columns(observations, n_objects, layout=None):
    """(source, column) per obs-vector column for a custom observation list (sources above). Point clouds are
    not in the vector (their observation key is their name, observables.py:199-210; observable_vec_task.py:
    188-191). Low-dimensional observables registered by the reference (multi_object.py:121-417, ur5sih.py:233-345)
    are copies of the refreshed state, so each is a set of fixed columns of a source:
      ur5_joint_state: dof positions 0..5 then velocities (ur5sih.py:606-607);
      sih_fingertip_angvel: rigid_body_state angvel of the 5 fingertips (ur5sih.py:309);
      object_quat / object_linvel / object_angvel: the objects' root-state rows (multi_object.py:137-172);
      object_mass / object_com / object_inertia: the pool properties of each env's objects (:907-925);
      target_object_pos / target_object_quat / target_object_pos_initial: the target object's root row (the
      last one re-gathers the current position every post_step, :229-240)."""
    lay = layout or default_layout(n_objects)
    a0, r0 = lay["a0"], lay["body_robot0"]
    sizes = default_sizes(n_objects)
    start = {n: sum(sizes[:i]) for i, n in enumerate(DEFAULT_OBSERVATIONS)}
    size = dict(zip(DEFAULT_OBSERVATIONS, sizes))
    root = lambda o, k: (SRC_ROOT, (a0 + o) * 13 + k)                      # noqa: E731
    extra = {
        "goal_pos": [(SRC_GOAL, k) for k in range(3)],
        "ur5_joint_state": [(SRC_DOF, 2 * d) for d in range(6)] + [(SRC_DOF, 2 * d + 1) for d in range(6)],
        "sih_fingertip_angvel": [(SRC_BODY, (r0 + t) * 13 + 10 + k) for t in TIP_LINKS for k in range(3)],
        "object_quat": [root(o, 3 + k) for o in range(n_objects) for k in range(4)],
        "object_linvel": [root(o, 7 + k) for o in range(n_objects) for k in range(3)],
        "object_angvel": [root(o, 10 + k) for o in range(n_objects) for k in range(3)],
        "object_mass": [(SRC_PROPS, o * PROPS) for o in range(n_objects)],
        "object_com": [(SRC_PROPS, o * PROPS + 1 + k) for o in range(n_objects) for k in range(3)],
        "object_inertia": [(SRC_PROPS, o * PROPS + 4 + k) for o in range(n_objects) for k in range(9)],
        "target_object_pos": [(SRC_ROOT | SRC_TARGET, a0 * 13 + k) for k in range(3)],
        "target_object_quat": [(SRC_ROOT | SRC_TARGET, a0 * 13 + 3 + k) for k in range(4)],
        "target_object_pos_initial": [(SRC_ROOT | SRC_TARGET, a0 * 13 + k) for k in range(3)],
    }
    cols = []
    for n in observations:
        if n in POINTCLOUDS or n.endswith(("_depth", "_segmentation", "_pointcloud", "_color")):
            continue
        if n in start:
            cols += [(SRC_OBS, start[n] + k) for k in range(size[n])]
        elif n in extra:
            cols += extra[n]
        else:
            raise NotImplementedError(f"observable {n!r}: this build produces {DEFAULT_OBSERVATIONS}, "
                                      f"{sorted(extra)} and the synthetic point clouds {POINTCLOUDS}")
    return cols
