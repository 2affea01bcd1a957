"""The oracle's numpy Generator(PCG64) restatement equals numpy itself
(the reference's only RNG: masurvival_env.py:50; shuffle semantics.py:74,
normal :111-118, random :745-746, :391)."""
import ctypes

import numpy as np
import pytest

import oracle
from masurvival.config import pcg64_state


class Pcg(ctypes.Structure):
    _fields_ = [('st_hi', ctypes.c_uint64), ('st_lo', ctypes.c_uint64), ('inc_hi', ctypes.c_uint64),
                ('inc_lo', ctypes.c_uint64), ('has_uint32', ctypes.c_int32), ('uinteger', ctypes.c_uint32)]


def _gen(seed):
    st = pcg64_state(seed)
    return Pcg(int(st[0]), int(st[1]), int(st[2]), int(st[3]), int(st[4]), int(st[5]))


@pytest.fixture(scope='module')
def L():
    lib = oracle.lib()
    lib.ora_pcg64_random.restype = ctypes.c_double
    lib.ora_pcg64_random.argtypes = [ctypes.POINTER(Pcg)]
    lib.ora_random_interval.restype = ctypes.c_uint64
    lib.ora_random_interval.argtypes = [ctypes.POINTER(Pcg), ctypes.c_uint64]
    lib.ora_standard_normal.restype = ctypes.c_double
    lib.ora_standard_normal.argtypes = [ctypes.POINTER(Pcg)]
    lib.ora_pcg64_next64.restype = ctypes.c_uint64
    lib.ora_pcg64_next64.argtypes = [ctypes.POINTER(Pcg)]
    return lib


@pytest.mark.parametrize('seed', [0, 1, 42, 2**40 + 7])
def test_random_matches_numpy(L, seed):
    g = np.random.default_rng(seed)
    r = _gen(seed)
    ref = g.random(2000)
    mine = np.array([L.ora_pcg64_random(ctypes.byref(r)) for _ in range(2000)])
    assert np.array_equal(ref, mine)


@pytest.mark.parametrize('seed', [0, 5, 123])
@pytest.mark.parametrize('n', [16, 36, 64])
def test_shuffle_matches_numpy(L, seed, n):
    g = np.random.default_rng(seed)
    x = list(range(n))
    g.shuffle(x)
    r = _gen(seed)
    y = list(range(n))
    for i in reversed(range(1, n)):
        j = L.ora_random_interval(ctypes.byref(r), i)
        y[i], y[j] = y[j], y[i]
    assert x == y
    # the stream continues identically afterwards (buffered uint32 included)
    assert g.random() == L.ora_pcg64_random(ctypes.byref(r))


@pytest.mark.parametrize('seed', [0, 9])
def test_normal_matches_numpy(L, seed):
    g = np.random.default_rng(seed)
    r = _gen(seed)
    ref = np.array([g.normal(loc=1.0, scale=0.5) for _ in range(5000)])
    mine = np.array([1.0 + 0.5 * L.ora_standard_normal(ctypes.byref(r)) for _ in range(5000)])
    assert np.array_equal(ref, mine)
