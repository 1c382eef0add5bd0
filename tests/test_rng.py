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


def test_malfunction_proposal_integer_forms_match_the_spec():
    """mf_propose decides u < rate as (z >> 11) < ceil(rate * 2^53) and takes the duration's 64-bit remainder with
    a multiply-high (round 5: the f64 conversion and the ~200-instruction 64-bit `%` left the GPU tick).  Same
    proposals as the spec's float compare and remainder (oracle/flatland_lite.py mf_uniform / mf_duration) for
    rates around and beyond the edges and duration ranges from one step to 2^31."""
    d = hostsim.lib().dll
    f = d.sflh_mf_propose
    f.argtypes = [C.c_double, C.c_int32, C.c_int32, C.c_uint64, C.c_uint32, C.POINTER(C.c_int32),
                  C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]
    rng = np.random.default_rng(5)
    n = 4000
    ticks = rng.integers(0, 2 ** 31 - 1, n).astype(np.int32)
    hs = rng.integers(0, 128, n).astype(np.int32)
    out = np.zeros(n, np.uint32)
    P = C.POINTER
    for rate in (0.0, 1e-9, 0.01, 0.3, 0.5, 1.0 - 2 ** -53, 1.0, 7.5, float("nan")):
        for lo, hi in ((5, 15), (0, 0), (3, 3), (1, 255), (0, 2 ** 31 - 2)):
            seed = int(rng.integers(0, 2 ** 63))
            f(rate, lo, hi, seed, n, ticks.ctypes.data_as(P(C.c_int32)), hs.ctypes.data_as(P(C.c_int32)),
              out.ctypes.data_as(P(C.c_uint32)))
            for i in range(0, n, 7):
                z = fl.mf_draw(seed, int(ticks[i]), int(hs[i]))
                want = (fl.mf_duration(z, lo, hi) + 1) if (rate > 0.0 and fl.mf_uniform(z) < rate) else 0
                assert int(out[i]) == want, (rate, lo, hi, i)
