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


def obs_columns(observations, n_objects):
    """(source, column) per obs-vector column for a custom observation list: source 0 = the step kernel's obs
    row (DEFAULT_OBSERVATIONS layout), 1 = goal_pos. Point clouds are not in the vector (their observation
    key is their name, observables.py:199-210; observable_vec_task.py:188-191). Raises for a low-dimensional
    observable this build does not produce."""
    sizes = default_sizes(n_objects)
    start = {n: sum(sizes[:i]) for i, n in enumerate(DEFAULT_OBSERVATIONS)}
    size = dict(zip(DEFAULT_OBSERVATIONS, sizes))
    cols = []
    for n in observations:
        if n in POINTCLOUDS or n.endswith(("_depth", "_segmentation", "_pointcloud", "_color")):
            continue
        if n in start:
            cols += [(0, start[n] + k) for k in range(size[n])]
        elif n == "goal_pos":
            cols += [(1, k) for k in range(3)]
        else:
            raise NotImplementedError(f"observable {n!r}: this build produces {DEFAULT_OBSERVATIONS}, goal_pos and "
                                      f"the synthetic point clouds {POINTCLOUDS}")
    return cols
