"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the C oracle (oracle/mas_oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline.  The product (gym-ma-survival-2d_amd/) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char_p, c_float, c_int8, c_int32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'build', 'libmas_oracle.so')
_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.ora_env_create.restype = c_void_p
        L.ora_env_create.argtypes = [c_void_p, c_char_p, c_int32]
        L.ora_env_destroy.argtypes = [c_void_p]
        L.ora_env_obs_dim.restype = c_int32
        L.ora_env_obs_dim.argtypes = [c_void_p]
        L.ora_env_set_rng.argtypes = [c_void_p, POINTER(c_uint64)]
        L.ora_env_get_rng.argtypes = [c_void_p, POINTER(c_uint64)]
        L.ora_env_reset.argtypes = [c_void_p, POINTER(c_float)]
        L.ora_env_step.restype = c_int32
        L.ora_env_step.argtypes = [c_void_p, POINTER(c_int8), POINTER(c_float), POINTER(c_float)]
        L.ora_env_flush_stats.argtypes = [c_void_p, POINTER(c_float)]
        L.ora_env_debug.restype = c_int32
        L.ora_env_debug.argtypes = [c_void_p, POINTER(c_float), c_int32]
        L.ora_counters.argtypes = [POINTER(ctypes.c_int64), c_int32]
        L.ora_bench_run.restype = c_int32
        L.ora_bench_run.argtypes = [c_void_p, POINTER(c_uint64), ctypes.c_int64, c_int32, ctypes.c_double,
                                    POINTER(ctypes.c_double)]
        _lib = L
    return _lib


COUNTER_NAMES = ['toi_event', 'toi_restore', 'sleep', 'box_broken', 'box_placed', 'item_picked', 'give_ok',
                 'give_lost', 'drop_items', 'heal_used', 'double_pick', 'aa_contact', 'island_contacts', 'islands',
                 'islands_k_gt2', 'islands_k_gt4', 'islands_k_gt8', 'toi_cap']


def counters(reset=True):
    out = np.zeros(len(COUNTER_NAMES), dtype=np.int64)
    lib().ora_counters(out.ctypes.data_as(POINTER(ctypes.c_int64)), int(reset))
    return dict(zip(COUNTER_NAMES, out.tolist()))


def _f32p(a):
    return a.ctypes.data_as(POINTER(c_float))


class OracleEnv:
    """One env of the CPU restatement; same config struct as the C-ABI."""

    def __init__(self, cfg_struct, seed_state=None):
        L = lib()
        err = ctypes.create_string_buffer(256)
        self._h = L.ora_env_create(ctypes.byref(cfg_struct), err, 256)
        if not self._h:
            raise ValueError(err.value.decode())
        self.A = cfg_struct.n_agents
        self.D = L.ora_env_obs_dim(self._h)
        if seed_state is not None:
            self.set_rng(seed_state)

    def __del__(self):
        if getattr(self, '_h', None) and _lib is not None:
            _lib.ora_env_destroy(self._h)
            self._h = None

    def set_rng(self, st6):
        st = np.ascontiguousarray(st6, dtype=np.uint64)
        lib().ora_env_set_rng(self._h, st.ctypes.data_as(POINTER(c_uint64)))

    def get_rng(self):
        st = np.zeros(6, dtype=np.uint64)
        lib().ora_env_get_rng(self._h, st.ctypes.data_as(POINTER(c_uint64)))
        return st

    def reset(self):
        obs = np.zeros((self.A, self.D), dtype=np.float32)
        lib().ora_env_reset(self._h, _f32p(obs))
        return obs

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int8).reshape(self.A, 6)
        obs = np.zeros((self.A, self.D), dtype=np.float32)
        rew = np.zeros(self.A, dtype=np.float32)
        done = lib().ora_env_step(self._h, a.ctypes.data_as(POINTER(c_int8)), _f32p(obs), _f32p(rew))
        return obs, rew, bool(done)

    def flush_stats(self):
        s = np.zeros(19, dtype=np.float32)
        lib().ora_env_flush_stats(self._h, _f32p(s))
        return s

    def debug(self):
        out = np.zeros(512, dtype=np.float32)
        n = lib().ora_env_debug(self._h, _f32p(out), 512)
        return out[:n]


def bench_run(cfg_struct, seed_states, threads=1, budget_s=5.0):
    """CPU baseline loop (ora_bench.c): the envs with PCG64 states
    seed_states [n, 6] stepped round-robin with uniform-random actions and
    auto-reset on `threads` threads for about budget_s seconds, all in C.
    Returns (env_steps, seconds)."""
    st = np.ascontiguousarray(seed_states, dtype=np.uint64)
    out = (ctypes.c_double * 2)()
    rc = lib().ora_bench_run(ctypes.byref(cfg_struct), st.ctypes.data_as(POINTER(c_uint64)), st.shape[0],
                             int(threads), float(budget_s), out)
    if rc != 0:
        raise RuntimeError('ora_bench_run failed')
    return int(out[0]), float(out[1])
