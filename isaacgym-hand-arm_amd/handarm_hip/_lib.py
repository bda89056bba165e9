"""ctypes binding of libhandarm_hip.so (the C ABI in include/handarm_abi.h).

The product path has no fallback: if the HIP library is missing or fails to load, this raises.
"""
import ctypes as C
import os
import re

from . import model as HM

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libhandarm_hip.so")
HEADER = os.path.join(os.path.dirname(os.path.dirname(PKG)), "include", "handarm_abi.h")

_lib = None

H = C.c_void_p
S = C.c_void_p   # hipStream_t
fp = C.c_void_p  # device pointers

SIGNATURES = {
    "ha_abi_version": ([], C.c_int),
    "ha_struct_sizes": ([C.POINTER(C.c_int32)] * 3, C.c_int),
    "ha_create": ([C.POINTER(HM.HaModel), C.POINTER(HM.HaParams), C.c_int32, C.POINTER(H)], C.c_int),
    "ha_destroy": ([H], C.c_int),
    "ha_bind_state": ([H, C.POINTER(HM.HaState)], C.c_int),
    "ha_simulate": ([H, C.c_int32, C.c_uint32, S], C.c_int),
    "ha_simulate_envs": ([H, C.c_int32, C.c_uint32, C.c_void_p, C.c_int32, S], C.c_int),
    "ha_refresh": ([H, S], C.c_int),
    "ha_set_dof_position_target": ([H, fp, S], C.c_int),
    "ha_set_actor_root_state_indexed": ([H, fp, fp, C.c_int32, S], C.c_int),
    "ha_set_dof_state_indexed": ([H, fp, fp, C.c_int32, S], C.c_int),
    "ha_set_dof_position_target_indexed": ([H, fp, fp, C.c_int32, S], C.c_int),
    "ha_set_object_collision_filter": ([H, fp, S], C.c_int),
    "ha_set_stats_ring": ([H, C.c_int32], C.c_int),
    "ha_task_step": ([H, C.c_uint32, S], C.c_int),
    "ha_task_observe": ([H, C.c_uint32, S], C.c_int),
    "ha_task_epilogue": ([H, C.c_void_p, C.c_float, C.c_void_p, S], C.c_int),
    "ha_task_step_io": ([H, C.c_uint32, C.c_void_p, C.c_float, C.c_void_p, C.c_float, C.c_void_p, S], C.c_int),
    "ha_task_reset": ([H, C.c_uint32, S], C.c_int),
    "ha_last_kernel_ms": ([H], C.c_float),
    "ha_contact_capacity": ([H], C.c_int),
    "ha_contact_cache_slots": ([H], C.c_int),
    "ha_set_env_order": ([H, C.c_void_p, C.c_int32], C.c_int),
    "ha_update_env_order": ([H, C.c_void_p, C.c_void_p, C.c_int32, S], C.c_int),
    "ha_set_order_cost": ([H, C.c_int32], C.c_int),
    "ha_enable_kernel_timing": ([H, C.c_int32], C.c_int),
    "ha_kernel_times": ([H, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32)], C.c_int),
    "ha_pointclouds": ([H, C.POINTER(HM.HaPointcloud), S], C.c_int),
    "ha_pointcloud_times": ([H, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32)], C.c_int),
    "ha_render_camera": ([H, C.POINTER(HM.HaCamera), C.POINTER(C.c_float), C.c_uint32, S], C.c_int),
    "ha_gather_obs": ([H, C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.c_int32, fp, C.c_int32, fp, S], C.c_int),
}


class HandArmError(RuntimeError):
    pass


def header_symbols(path=HEADER):
    """Function names declared in include/handarm_abi.h."""
    with open(path) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|float)\s+(ha_\w+)\s*\(", txt, re.M)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HandArmError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                           "g.build()'` (hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    for name, (args, res) in SIGNATURES.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        raise HandArmError(f"{what} failed with code {rc}")
    return rc
