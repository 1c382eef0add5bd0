"""Device RNG code (csrc/sfl_rng.h, host-compiled) against numpy's own PCG64 / SeedSequence."""
import ctypes as C

import numpy as np
import pytest

from tests import hostsim
from oracle import flatland_lite as fl


def _self_test(value, n, bound):
    d = hostsim.lib().dll
    f = d.sflh_rng_selftest
    f.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_double),
                  C.c_uint32, C.POINTER(C.c_uint32)]
    o64 = np.zeros(n, np.uint64)
    o32 = np.zeros(n, np.uint32)
    od = np.zeros(n)
    ob = np.zeros(n, np.uint32)
    f(value, n, o64.ctypes.data_as(C.POINTER(C.c_uint64)), o32.ctypes.data_as(C.POINTER(C.c_uint32)),
      od.ctypes.data_as(C.POINTER(C.c_double)), bound, ob.ctypes.data_as(C.POINTER(C.c_uint32)))
    return o64, o32, od, ob


def _gen(v):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(v))))


@pytest.mark.parametrize("value", [0, 1, 2, 7, 450565, 2 ** 31 - 2, 123456789, 2 ** 32 - 1])
@pytest.mark.parametrize("bound", [0, 1, 2, 4, 8, 2147483646])
def test_streams_match_numpy(value, bound):
    n = 64
    o64, o32, od, ob = _self_test(value, n, bound)
    assert o64.tolist() == _gen(value).bit_generator.random_raw(n).tolist()
    g = _gen(value)
    assert o32.tolist() == [int(g.integers(0, 2 ** 32)) for _ in range(n)]
    assert od.tolist() == _gen(value).random(n).tolist()
    g = _gen(value)
    assert ob.tolist() == [int(g.integers(0, bound + 1)) for _ in range(n)]


def test_discrete_sample_equivalence():
    """gymnasium Discrete(n).seed(s); sample(mask) == valid[bounded(len(valid)-1)] of a fresh stream."""
    for s in range(300):
        valid = np.array([0, 2, 3, 6, 8])[: 1 + s % 5]
        ref = _gen(s).choice(valid)
        _, _, _, ob = _self_test(s, 1, len(valid) - 1)
        assert valid[ob[0]] == ref


def test_malfunction_draw_matches_spec():
    d = hostsim.lib().dll
    f = d.sflh_mf_draw
    f.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
    z = C.c_uint64()
    for seed, tick, h in [(0, 0, 0), (450565, 17, 3), (2 ** 40 + 5, 1234, 127), (12345, 1, 31)]:
        f(seed, tick, h, C.byref(z))
        assert z.value == fl.mf_draw(seed, tick, h)
