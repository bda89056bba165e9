"""ORACLE (test infrastructure only): ctypes front-end of oracle/_build/libhandarm_oracle.so.

Operates on host numpy buffers laid out exactly like the device tensors (handarm_hip.model.state_spec).
"""
import ctypes as C
import os
import subprocess

import numpy as np

from handarm_hip import model as HM

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libhandarm_oracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    build()   # make is a no-op when the library is up to date
    lib = C.CDLL(LIB)
    lib.hao_create.restype = C.c_void_p
    lib.hao_create.argtypes = [C.POINTER(HM.HaModel), C.POINTER(HM.HaParams), C.c_int]
    lib.hao_destroy.argtypes = [C.c_void_p]
    lib.hao_simulate.argtypes = [C.c_void_p, C.POINTER(HM.HaState), C.c_int, C.c_int, C.c_int]
    lib.hao_controller.argtypes = [C.c_void_p, C.POINTER(HM.HaState), C.c_int]
    lib.hao_struct_sizes.argtypes = [C.POINTER(C.c_int32)] * 3
    lib.hao_contacts.restype = C.c_int
    lib.hao_contacts.argtypes = [C.c_void_p, C.POINTER(HM.HaState), C.c_int, C.c_void_p, C.c_int]
    lib.hao_sincos.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.hao_pcm_slots.restype = C.c_int
    lib.hao_pcm_slots.argtypes = [C.POINTER(HM.HaModel), C.c_int]
    return lib


def sincos(x):
    """include/ha_fmath.h ha_sincosf over a float32 array, as compiled into the C oracle."""
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    load().hao_sincos(x.ctypes.data, x.size, s.ctypes.data, c.ctypes.data)
    return s, c


class HostState:
    """numpy buffers for every ha_state_t field."""

    def __init__(self, num_envs, n_obj=3, num_initial_poses=1, model=None, params=None):
        kw = {}
        if params is not None:
            kw.update(num_actions=params.num_actions, num_obs=params.num_obs, num_states=HM.num_states(params))
            n_obj = params.n_objects
        if model is not None:       # sizes/layout of the model's task (default: Ur5Sih)
            kw.update(n_links=model.n_links, n_dofs=model.n_dofs, n_actors=model.n_actors, n_bodies=model.n_bodies,
                      n_pcm_slots=HM.pcm_slots(model, n_obj, params))
        self.spec = HM.state_spec(num_envs, n_obj=n_obj, num_initial_poses=num_initial_poses, **kw)
        self.null = HM.null_fields(params.task if params is not None else HM.TASK_UR5SIH)
        self.arrays = {k: np.zeros(shape, dtype) for k, (shape, dtype) in self.spec.items()}
        self.num_envs = num_envs
        if params is not None and params.dr_enable:
            # DR on: nominal rows and the frame-0 shard state, as HandArmSim starts them (handarm_hip/dr.py)
            from handarm_hip import dr as DR
            m = model if model is not None else HM.build_model(HM.load_scene())
            self.arrays["dr_scale"][:] = DR.default_rows(m, params, num_envs)
            self.arrays["dr_global"][:] = DR.init_global(params)

    def __getitem__(self, k):
        return self.arrays[k]

    def ctypes(self):
        s = HM.HaState()
        for k in HM.STATE_FIELDS:
            setattr(s, k, None if k in self.null else self.arrays[k].ctypes.data)
        return s

    def copy(self):
        o = HostState.__new__(HostState)
        o.spec, o.num_envs, o.null = self.spec, self.num_envs, self.null
        o.arrays = {k: v.copy() for k, v in self.arrays.items()}
        return o


class Oracle:
    def __init__(self, model, params, num_envs):
        self.lib = load()
        self.model, self.params = model, params
        self.h = self.lib.hao_create(C.byref(model), C.byref(params), num_envs)
        self.num_envs = num_envs

    def simulate(self, st, n_calls=1, begin=0, end=None):
        # the records this oracle's params use (0 when they turn the persistent manifolds off) must fit the state's
        # contact_cache rows: a HostState sized for params with the records off has none
        need = HM.pcm_slots(self.model, self.params.n_objects, self.params)
        have = st["contact_cache"].shape[1] if st["contact_cache"] is not None else 0
        if need and have != need:
            raise ValueError(f"contact_cache has {have} record slots per env, these params use {need}")
        s = st.ctypes()
        self.lib.hao_simulate(self.h, C.byref(s), n_calls, begin, self.num_envs if end is None else end)

    def contacts(self, st, env):
        """(x[3], n[3], sep, a, b) rows of the contacts detect() produces for env (normal from body b to a)."""
        out = np.zeros((256, 9), np.float32)
        s = st.ctypes()
        n = self.lib.hao_contacts(self.h, C.byref(s), env, out.ctypes.data, 256)
        return out[:min(n, 256)]

    def controller(self, st):
        s = st.ctypes()
        for e in range(self.num_envs):
            self.lib.hao_controller(self.h, C.byref(s), e)

    def __del__(self):
        try:
            self.lib.hao_destroy(self.h)
        except Exception:
            pass
