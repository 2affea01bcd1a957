"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host
code only; `make -C oracle asan`): random-action episodes with auto-reset on
four threads plus one env's reset/step/flush/debug pass, for the 1v1, 2v2
and FFA4 configs.  Any out-of-bounds access, use-after-free, leak or UB
aborts the run."""
import ctypes
import os
import subprocess

import pytest

from masurvival.config import C1_CONFIG, C3_CONFIG, C5_CONFIG, ResolvedConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORA = os.path.join(ROOT, 'oracle')
BIN = os.path.join(ORA, 'build_asan', 'ora_asan_check')


@pytest.fixture(scope='module')
def asan_bin():
    subprocess.check_call(['make', '-s', '-C', ORA, 'asan'])
    return BIN


@pytest.mark.parametrize('cfg,name', [(C1_CONFIG, '1v1'), (C3_CONFIG, '2v2'), (C5_CONFIG, 'ffa4')])
def test_oracle_clean_under_asan_ubsan(asan_bin, tmp_path, cfg, name):
    st = ResolvedConfig(cfg).to_struct()
    blob = tmp_path / f'{name}.bin'
    blob.write_bytes(ctypes.string_at(ctypes.addressof(st), ctypes.sizeof(st)))
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1', UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([asan_bin, str(blob), '8', '300', '4'], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith('ok'), r.stdout + r.stderr
