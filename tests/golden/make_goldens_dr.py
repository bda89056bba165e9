#!/usr/bin/env python3
"""Golden vectors for the domain-randomization engine by RUNNING THE REFERENCE's apply_randomizations
(tasks/base/vec_task.py:646-876) and utils/dr_utils.py (generate_random_samples, get_bucketed_val,
apply_random_samples) against a fake gym that stores actor properties, with numpy's and torch's random draws
intercepted: every draw is taken from a recorded stream (uniform quantiles q, standard normals z, correlated /
white noise tensors), so the build's restatement (oracle/dr_oracle.py, bit-identical to csrc/ha_dr.h on the GPU) can
be fed the same draws and compared value for value.

Run in the build container only (needs /root/reference):  python tests/golden/make_goldens_dr.py
Writes ``dr_reference.npz`` + ``dr_schemas.json`` (data only) next to this file.

Recorded per scenario (AllegroKuka.yaml's and AllegroHand.yaml's randomization_params, read with yaml.safe_load):
  * a sequence of apply_randomizations calls (gym frame count, reset_buf, randomize_buf before the call): which envs
    were randomized, whether the non-env part ran, last_rand_step, the noise parameters it stored
    (dr_randomizations), the sim params' gravity;
  * every actor property value it set, with the draws that produced it (per env, property, element);
  * the noise lambdas applied to a fixed tensor with recorded correlated / white draws.
The AllegroKuka scenario runs with sim_params taken as empty (the yaml's `sim_params:` is None and the reference's
loop would fail on None.items(), vec_task.py:764; handarm_hip/dr.py documents the same reading).
"""
import json
import os
import sys
from unittest import mock

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "isaacgym-hand-arm_amd"))
import refload  # noqa: E402
from handarm_hip import model as HM  # noqa: E402

CFG = "/root/reference/isaacgymenvs/cfg/task"


class Vec3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = x, y, z


class SimParams:
    def __init__(self):
        self.gravity = Vec3(0.0, 0.0, -9.81)

        class P:
            rest_offset = 0.0
        self.physx = P()


class Body:
    def __init__(self, mass):
        self.mass = mass


class Shape:
    def __init__(self, friction):
        self.friction = friction


DOF_DT = np.dtype([("damping", "f4"), ("stiffness", "f4"), ("lower", "f4"), ("upper", "f4")])


class FakeGym:
    """Actor properties of N envs with actors [robot, object]: the robot's links (one shape each) and DOFs, the object."""

    def __init__(self, n, robot, model, pool_mass):
        self.n, self.robot, self.frame = n, robot, 0
        L, D = model.n_links, model.n_dofs
        dof = np.zeros(D, DOF_DT)
        dof["damping"] = list(model.dof_kd)[:D]
        dof["stiffness"] = list(model.dof_kp)[:D]
        dof["lower"] = list(model.dof_lower)[:D]
        dof["upper"] = list(model.dof_upper)[:D]
        self.dof = [dof.copy() for _ in range(n)]
        self.bodies = [[[Body(float(np.float32(model.link_mass[i]))) for i in range(L)], [Body(pool_mass)]]
                       for _ in range(n)]
        self.shapes = [[[Shape(1.0) for _ in range(L)], [Shape(1.0)]] for _ in range(n)]
        self.scale = [[1.0, 1.0] for _ in range(n)]
        self.sim_params = SimParams()
        self.names = [robot, "object"]

    # lookup
    def get_frame_count(self, sim):
        return self.frame

    def find_actor_handle(self, env, name):
        return self.names.index(name)

    def get_actor_count(self, env):
        return 2

    def get_actor_handle(self, env, i):
        return i

    def get_actor_name(self, env, h):
        return self.names[h]

    def get_actor_rigid_shape_count(self, env, h):
        return len(self.shapes[env][h])

    def get_actor_rigid_body_count(self, env, h):
        return len(self.bodies[env][h])

    def set_rigid_body_color(self, *a):
        pass

    # properties (getters return copies, as Isaac Gym does; the reference writes them back with the setters)
    def get_actor_dof_properties(self, env, h):
        return self.dof[env].copy() if h == 0 else np.zeros(0, DOF_DT)

    def set_actor_dof_properties(self, env, h, props):
        if h == 0:
            self.dof[env] = props.copy()

    def get_actor_rigid_body_properties(self, env, h):
        return [Body(b.mass) for b in self.bodies[env][h]]

    def set_actor_rigid_body_properties(self, env, h, props, recompute=True):
        self.bodies[env][h] = [Body(float(np.float32(np.asarray(b.mass).reshape(-1)[0]))) for b in props]

    def get_actor_rigid_shape_properties(self, env, h):
        return [Shape(s.friction) for s in self.shapes[env][h]]

    def set_actor_rigid_shape_properties(self, env, h, props):
        self.shapes[env][h] = [Shape(float(np.float32(np.asarray(s.friction).reshape(-1)[0]))) for s in props]

    def set_actor_scale(self, env, h, s):
        self.scale[env][h] = float(np.float32(np.asarray(s).reshape(-1)[0]))
        # the scale's draw went through generate_random_samples directly (vec_task.py:811-823): tag it
        ctx, kind, v = self.draws.log[-1]
        self.draws.log[-1] = (("scale", env), kind, v)

    def get_actor_tendon_properties(self, env, h):
        return []

    def set_actor_tendon_properties(self, env, h, p):
        pass

    def get_sim_params(self, sim):
        p = SimParams()
        p.gravity = Vec3(self.sim_params.gravity.x, self.sim_params.gravity.y, self.sim_params.gravity.z)
        return p

    def set_sim_params(self, sim, p):
        self.sim_params = p


class Draws:
    """np.random.uniform / normal replacements: the value is computed from a recorded quantile q / normal z, tagged
    with the (env, property, attribute) that apply_random_samples is working on."""

    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.ctx = None
        self.log = []

    def uniform(self, lo, hi, shape):
        q = self.rng.random(np.atleast_1d(np.empty(shape)).shape if not isinstance(shape, int) else shape)
        self.log.append((self.ctx, "u", np.atleast_1d(q).astype(np.float64)))
        return lo + (hi - lo) * q

    def normal(self, mu, var, shape):
        z = self.rng.standard_normal(np.atleast_1d(np.empty(shape)).shape if not isinstance(shape, int) else shape)
        self.log.append((self.ctx, "g", np.atleast_1d(z).astype(np.float64)))
        return mu + var * z


def run(schema, robot, model, pool_mass, calls, sim_initialized, seed):
    vt = refload.load("isaacgymenvs.tasks.base.vec_task")
    du = refload.load("isaacgymenvs.utils.dr_utils")
    du.gymapi.SimParams = SimParams
    vt.gymapi.Vec3 = Vec3
    N = len(calls[0][1])
    gym = FakeGym(N, robot, model, pool_mass)
    # a concrete subclass of the reference's VecTask (its step hooks are abstract); only apply_randomizations runs
    Task = type("DRTask", (vt.VecTask,), {"pre_physics_step": lambda self, a: None,
                                           "post_physics_step": lambda self: None})
    t = object.__new__(Task)
    t.gym, t.sim, t.num_environments, t.envs = gym, None, N, list(range(N))
    t.first_randomization, t.original_props, t.dr_randomizations = True, {}, {}
    t.actor_params_generator, t.extern_actor_params = None, {i: None for i in range(N)}
    t.last_step, t.last_rand_step, t.sim_initialized = -1, -1, sim_initialized
    t.randomize_buf = torch.zeros(N, dtype=torch.long)
    draws = Draws(seed)
    gym.draws = draws
    orig = du.apply_random_samples

    def tagged(prop, og_prop, attr, params, step, extern_sample=None, bucketing_randomization_params=None):
        draws.ctx = (id(prop), attr)
        return orig(prop, og_prop, attr, params, step, extern_sample, bucketing_randomization_params)

    out = {"frame": [], "reset": [], "rb_before": [], "randomized": [], "nonenv": [], "last_rand": [],
           "obs_params": [], "act_params": [], "gravity": [], "values": []}
    with mock.patch.object(du.np.random, "uniform", draws.uniform), mock.patch.object(du.np.random, "normal",
                                                                                        draws.normal), \
            mock.patch.object(vt, "apply_random_samples", tagged):
        for frame, reset, rb in calls:
            gym.frame = frame
            t.reset_buf = torch.tensor(reset, dtype=torch.long)
            t.randomize_buf = torch.tensor(rb, dtype=torch.long)
            before_rand = t.last_rand_step
            draws.log.clear()
            ids = {}
            # tag every property object the getters hand out: wrap the getters once per call
            g0 = (gym.get_actor_dof_properties, gym.get_actor_rigid_body_properties,
                  gym.get_actor_rigid_shape_properties)

            keep = []                         # hold every handed-out object: ids must not be recycled in the call

            def wrap(fn, kind):
                def w(env, h):
                    r = fn(env, h)
                    keep.append(r)
                    if isinstance(r, list):
                        for i, x in enumerate(r):
                            ids[id(x)] = (env, gym.names[h], kind, i)
                    else:
                        ids[id(r)] = (env, gym.names[h], kind, -1)
                    return r
                return w
            gym.get_actor_dof_properties = wrap(g0[0], "dof")
            gym.get_actor_rigid_body_properties = wrap(g0[1], "body")
            gym.get_actor_rigid_shape_properties = wrap(g0[2], "shape")
            t.apply_randomizations(schema)
            t.sim_initialized = True          # create_sim -> prepare_sim done after the setup call (vec_task.py:286-289)
            gym.get_actor_dof_properties, gym.get_actor_rigid_body_properties, gym.get_actor_rigid_shape_properties = g0
            randomized = np.zeros(N, bool)
            for ctx, kind, v in draws.log:
                if ctx is not None and ctx[0] in ids:
                    randomized[ids[ctx[0]][0]] = True
                elif ctx is not None and ctx[0] == "scale":
                    randomized[ctx[1]] = True
            out["frame"].append(frame)
            out["reset"].append(np.asarray(reset))
            out["rb_before"].append(np.asarray(rb))
            out["randomized"].append(randomized)
            out["nonenv"].append(t.last_rand_step != before_rand or (before_rand == -1 and len(out["frame"]) == 1))
            out["last_rand"].append(t.last_rand_step)
            out["rb_after"] = out.get("rb_after", []) + [t.randomize_buf.numpy().copy()]
            for key in ("observations", "actions"):
                d = t.dr_randomizations.get(key)
                vals = [d[k] for k in ("mu", "var", "mu_corr", "var_corr")] if d and "mu" in d else \
                    ([d[k] for k in ("lo", "hi", "lo_corr", "hi_corr")] if d else [np.nan] * 4)
                out["obs_params" if key == "observations" else "act_params"].append(np.array(vals, np.float64))
            g = gym.sim_params.gravity
            out["gravity"].append(np.array([g.x, g.y, g.z], np.float64))
            # every draw with the value it produced: (call, env, actor, kind, element index, attr, dist, draw, value)
            for ctx, kind, v in draws.log:
                if ctx is None:
                    continue
                if ctx[0] == "scale":
                    out["values"].append((len(out["frame"]) - 1, ctx[1], "object", "scale", 0, "scale", kind, v,
                                          np.array([gym.scale[ctx[1]][1]])))
                    continue
                if ctx[0] not in ids:          # sim params (gravity): one 3-vector draw
                    out["values"].append((len(out["frame"]) - 1, -1, "sim", "sim", -1, ctx[1], kind, v,
                                          out["gravity"][-1].copy()))
                    continue
                env, actor, pk, i = ids[ctx[0]]
                attr = ctx[1]
                if pk == "dof":
                    val = gym.dof[env][attr].astype(np.float64)
                elif pk == "body":
                    val = np.array([gym.bodies[env][0 if actor == robot else 1][i].mass])
                else:
                    val = np.array([gym.shapes[env][0 if actor == robot else 1][i].friction])
                out["values"].append((len(out["frame"]) - 1, env, actor, pk, i, attr, kind, v, val))
            # actor scale (drawn through generate_random_samples with shape 1 outside apply_random_samples)
            draws.ctx = None
    return out, gym, t


def noise_case(t, seed):
    """The stored noise lambdas on a fixed tensor, with recorded correlated and white draws."""
    rng = np.random.default_rng(seed)
    x = torch.tensor(rng.uniform(-1, 1, (4, 6)), dtype=torch.float32)
    res = {}
    for key in ("observations", "actions"):
        d = t.dr_randomizations.get(key)
        if not d:
            continue
        d.pop("corr", None)
        c = torch.tensor(rng.standard_normal((4, 6)), dtype=torch.float32)
        w = torch.tensor(rng.standard_normal((4, 6)) if "mu" in d else rng.random((4, 6)), dtype=torch.float32)
        seq = iter([c, w])
        with mock.patch.object(torch, "randn_like", lambda t_: next(seq)), \
                mock.patch.object(torch, "rand_like", lambda t_: next(seq)):
            y = d["noise_lambda"](x.clone())
        res[key] = (x.numpy(), c.numpy(), w.numpy(), y.numpy())
    return res


def main():
    schemas = {}
    for name in ("AllegroKuka", "AllegroHand"):
        with open(os.path.join(CFG, name + ".yaml")) as f:
            schemas[name] = yaml.safe_load(f)["task"]["randomization_params"]
    with open(os.path.join(HERE, "dr_schemas.json"), "w") as f:
        json.dump(schemas, f, indent=1, sort_keys=True)
    arrays = {}
    N = 6
    # AllegroKuka: the first apply_randomizations from reset_idx, after sim_initialized (setup_only never applies);
    # AllegroHand's schema as a task would run it from create_sim (the setup call before sim_initialized)
    for name, robot, task, asset, sim_init in (("kuka", "allegro", HM.TASK_ALLEGRO_KUKA, HM.KUKA_ASSET, True),
                                               ("hand", "hand", HM.TASK_ALLEGRO_HAND, HM.ALLEGRO_ASSET, False)):
        sc = dict(schemas["AllegroKuka" if name == "kuka" else "AllegroHand"])
        if sc.get("sim_params", 1) is None:
            sc.pop("sim_params")                 # see the module docstring
        sc["frequency"] = 3
        model = HM.build_model(HM.load_scene(asset), posed=None)
        pool_mass = float(np.float32(model.pool_mass[0]))
        f0 = 29994 if name == "kuka" else 0
        calls = [(f0, [1] * N, [0] * N)]
        rb = np.zeros(N, int)
        for s in range(1, 10):
            rb += 1
            reset = [1 if (e + s) % 3 == 0 else 0 for e in range(N)]
            calls.append((f0 + s, reset, rb.tolist()))
            rb = np.where((np.array(reset) == 1) & (rb >= 3), 0, rb)
        out, gym, t = run(sc, robot, model, pool_mass, calls, sim_init, seed=7 if name == "kuka" else 8)
        for k in ("frame", "last_rand"):
            arrays[f"{name}_{k}"] = np.array(out[k])
        for k in ("reset", "rb_before", "randomized", "rb_after", "obs_params", "act_params", "gravity"):
            arrays[f"{name}_{k}"] = np.stack(out[k])
        arrays[f"{name}_nonenv"] = np.array(out["nonenv"], bool)
        rows = []
        for call, env, actor, pk, i, attr, kind, v, val in out["values"]:
            for j in range(len(v)):
                elem = j if pk in ("dof", "sim") else i
                value = val[j] if len(val) > 1 else val[0]
                rows.append((call, env, {"sim": 0, "dof": 1, "body": 2, "shape": 3, "scale": 4}[pk],
                             0 if actor in ("allegro", "hand", "sim") else 1, elem,
                             ["gravity", "damping", "stiffness", "lower", "upper", "mass", "friction",
                              "scale"].index(attr),
                             0 if kind == "u" else 1, v[j], value))
        arrays[f"{name}_values"] = np.array(rows, np.float64)
        arrays[f"{name}_scale"] = np.array([[s[1] for s in gym.scale]], np.float64)
        nz = noise_case(t, 11 if name == "kuka" else 12)
        for key, (x, c, w, y) in nz.items():
            for k, a in (("x", x), ("corr", c), ("white", w), ("y", y)):
                arrays[f"{name}_noise_{key}_{k}"] = a
    np.savez_compressed(os.path.join(HERE, "dr_reference.npz"), **arrays)
    print("wrote", sorted(arrays))


if __name__ == "__main__":
    main()
