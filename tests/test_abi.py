"""C-ABI boundary checks that need no GPU: the library loads, exports every declared symbol, and
the ctypes mirrors of the structs match the compiled layouts (HIP library and C oracle)."""
import ctypes as C

import pytest

from handarm_hip import _lib
from handarm_hip import model as HM


@pytest.fixture(scope="module")
def lib():
    from handarm_hip import build
    build.build()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _lib.header_symbols()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with include/handarm_abi.h"


def test_struct_layouts_match(lib):
    a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.ha_struct_sizes(C.byref(a), C.byref(b), C.byref(c)) == 0
    assert (a.value, b.value, c.value) == (C.sizeof(HM.HaModel), C.sizeof(HM.HaParams), C.sizeof(HM.HaState))
    assert lib.ha_abi_version() == 16


def test_oracle_struct_layouts_match():
    from oracle import oracle_lib
    ol = oracle_lib.load()
    a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
    ol.hao_struct_sizes(C.byref(a), C.byref(b), C.byref(c))
    assert (a.value, b.value, c.value) == (C.sizeof(HM.HaModel), C.sizeof(HM.HaParams), C.sizeof(HM.HaState))


def test_create_rejects_bad_arguments(lib):
    m = HM.build_model(HM.load_scene())
    p, _ = HM.build_params()
    h = C.c_void_p()
    assert lib.ha_create(C.byref(m), C.byref(p), 0, C.byref(h)) == -1        # HA_E_ARG, no GPU touched
    p.num_initial_poses = 0
    assert lib.ha_create(C.byref(m), C.byref(p), 4, C.byref(h)) == -1
    assert lib.ha_simulate(None, 1, 0, None) != 0
    assert lib.ha_task_step(None, 0, None) != 0


def test_no_cpu_fallback_on_cpu_device():
    from handarm_hip.sim import HandArmSim
    with pytest.raises(_lib.HandArmError):
        HandArmSim(4, device="cpu")
