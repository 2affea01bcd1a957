"""The HIP library loads here (no GPU needed to dlopen) and exports every
symbol include/masurvival.h declares, with the ABI version the header states."""
import ctypes
import os
import re

import pytest

from masurvival import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, 'include', 'masurvival.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int|int64_t|int32_t|const char\*)\s+(mas_\w+)\s*\(', txt, re.M)))


def test_header_symbols_known():
    syms = header_symbols()
    assert len(syms) >= 12
    assert set(syms) == set(abi.SIGNATURES), set(syms) ^ set(abi.SIGNATURES)


def test_library_exports_all_symbols():
    if not os.path.exists(abi.LIB_PATH):
        import __graft_entry__  # noqa
        __graft_entry__.build()
    lib = ctypes.CDLL(abi.LIB_PATH)
    for s in header_symbols():
        assert hasattr(lib, s), s
    lib.mas_abi_version.restype = ctypes.c_int32
    assert lib.mas_abi_version() == 3


def test_create_rejects_bad_config_without_gpu():
    lib = abi.load_library()
    from masurvival.config import ResolvedConfig
    cfg = ResolvedConfig(None).to_struct()
    cfg.n_agents = 1
    h = ctypes.c_void_p()
    rc = lib.mas_create(ctypes.byref(cfg), 4, 0, ctypes.byref(h))
    assert rc == -1
    assert b'n_agents' in lib.mas_last_error()


@pytest.mark.parametrize('val', ['1', '3', 'x'])
def test_create_rejects_unknown_split_mode_without_gpu(val, monkeypatch):
    """MAS_SPLIT takes 0 (one stream) or 2 (the slow split); the removed
    modes and anything else are refused before any device allocation (ADVICE
    r04)."""
    monkeypatch.setenv('MAS_SPLIT', val)
    lib = abi.load_library()
    from masurvival.config import ResolvedConfig
    cfg = ResolvedConfig(None).to_struct()
    h = ctypes.c_void_p()
    rc = lib.mas_create(ctypes.byref(cfg), 4, 0, ctypes.byref(h))
    assert rc == -1
    assert b'MAS_SPLIT' in lib.mas_last_error()


def test_policy_counted_waits_cover_their_copies():
    """k_policy_train_db's land_db<NST> waits: in the built ISA at
    least min(NST, 63) vector memory instructions follow the copies each one
    waits for (scripts/check_policy_waits.py, also run by build())."""
    import subprocess
    import sys
    if not os.path.exists(abi.LIB_PATH) or not os.path.exists('/opt/rocm/lib/llvm/bin/llvm-objdump'):
        pytest.skip('library or llvm-objdump absent')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'check_policy_waits.py')],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'counted waits OK' in r.stdout
