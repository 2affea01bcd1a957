"""VecMaSurvival: N MaSurvival envs stepped by the HIP kernels (libmas.so).

The batched surface of the build: ``reset() -> obs[N,A,D]``,
``step(actions int[N,A,6]) -> (obs[N,A,D], rewards[N,A], done[N], info)``,
all torch tensors resident on the GPU.  Each env is one reference
``MaSurvival`` (masurvival_env.py:241-389) with its own numpy PCG64 stream;
``step`` auto-resets finished envs (the returned obs rows are then the first
observation of the new episode, rewards/done describe the finished step).
There is no CPU fallback: construction fails loudly without the HIP library
or a GPU.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Any, Dict, Optional, Sequence

import numpy as np

from . import spaces
from .abi import MAS_STATS_WIDTH, MasObsLayout, check, load_library
from .config import ResolvedConfig, pcg64_state


def _torch():
    import torch
    return torch


MAS_RENDER_VIEW_FLOATS = 320  # include/masurvival.h


def parse_render_view(v: np.ndarray) -> Dict[str, Any]:
    """The float layout of mas_render_view (include/masurvival.h) as arrays."""
    A, nb, ni, nh = (int(v[k]) for k in range(4))
    AM, BM, HM = (int(v[k]) for k in range(7, 10))
    o = 32
    agents = v[o:o + 5 * AM].reshape(AM, 5)[:A]
    o += 5 * AM
    boxes = v[o:o + 5 * BM].reshape(BM, 5)[:nb]
    o += 5 * BM
    items = v[o:o + 4 * BM].reshape(BM, 4)[:ni]
    o += 4 * BM
    heals = v[o:o + 2 * HM].reshape(HM, 2)[:nh]
    return {'agents': agents, 'boxes': boxes, 'items': items, 'heals': heals,
            'zone': v[4:7].copy(), 'floor_size': float(v[10]), 'walls': v[12:32].reshape(4, 5).copy()}


class VecMaSurvival:
    def __init__(self, config: Optional[Dict[str, Dict[str, Any]]] = None, n_envs: int = 1, device=None,
                 seeds: Optional[Sequence[int]] = None, auto_reset: bool = True):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError('VecMaSurvival needs a ROCm GPU (the env step runs only as HIP kernels)')
        self.rc = ResolvedConfig(config)
        self.n_envs = int(n_envs)
        self.device = torch.device('cuda', torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.auto_reset = bool(auto_reset)
        self._lib = load_library()
        self._cfg = self.rc.to_struct()
        h = ctypes.c_void_p()
        check(self._lib.mas_create(ctypes.byref(self._cfg), self.n_envs, self.device.index, ctypes.byref(h)))
        self._h = h
        lay = MasObsLayout()
        check(self._lib.mas_get_obs_layout(self._h, ctypes.byref(lay)))
        self.n_agents = lay.n_agents
        self.obs_dim = lay.obs_dim
        self.layout = OrderedDict()
        for k in range(lay.n_keys):
            name = lay.key_name[k].value.decode()
            nd = lay.key_ndim[k]
            shape = (lay.key_shape[k][0],) if nd == 1 else (lay.key_shape[k][0], lay.key_shape[k][1])
            self.layout[name] = (lay.key_offset[k], shape)
        N, A, D = self.n_envs, self.n_agents, self.obs_dim
        dev = self.device
        self.obs = torch.zeros((N, A, D), dtype=torch.float32, device=dev)
        self.rewards = torch.zeros((N, A), dtype=torch.float32, device=dev)
        self.dones = torch.zeros((N,), dtype=torch.uint8, device=dev)
        self._act = torch.zeros((N, A, 6), dtype=torch.int8, device=dev)
        self.observation_space = self._single_obs_space()
        self.action_space = spaces.Tuple((spaces.MultiDiscrete([3, 3, 3, 2, 2, 2]),) * A)
        self.seed(seeds)

    # ------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def _single_obs_space(self):
        R = dict(low=float('-inf'), high=float('inf'))
        d = {k: spaces.Box(**R, shape=(self.n_agents,) + shp) for k, (_, shp) in self.layout.items()}
        return spaces.Dict(d)

    def seed(self, seeds: Optional[Sequence[int]] = None):
        """One numpy ``default_rng(seed)`` stream per env (env e: seeds[e], default e)."""
        if seeds is None:
            seeds = range(self.n_envs)
        seeds = list(seeds)
        if len(seeds) != self.n_envs:
            raise ValueError('need one seed per env')
        st = np.stack([pcg64_state(int(s)) for s in seeds]).astype(np.uint64)
        self.set_rng_states(st)

    def set_rng_states(self, states: np.ndarray):
        """Inject raw numpy PCG64 states, uint64 [N, 6] (see config.pcg64_state)."""
        st = np.ascontiguousarray(states, dtype=np.uint64)
        assert st.shape == (self.n_envs, 6)
        _torch().cuda.synchronize(self.device)
        check(self._lib.mas_seed(self._h, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), self._stream()))

    def reset(self, mask=None):
        """BaseEnv.reset for every env (or those with mask != 0); returns obs [N,A,D]."""
        mptr = None
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch_uint8()).contiguous()
            mptr = ctypes.c_void_p(mask.data_ptr())
        check(self._lib.mas_reset(self._h, mptr, ctypes.c_void_p(self.obs.data_ptr()), self._stream()))
        return self.obs

    def step(self, actions, out=None, validate=False):
        """actions: int tensor [N,A,6] (MultiDiscrete [3,3,3,2,2,2]).
        out: optional (obs, rewards, done) tensors to write into (e.g. a
        rollout-buffer slice); defaults to the env's own buffers.
        validate: check every action against the action space first (the
        reference's assert, masurvival_env.py:80; synchronises).  Without it
        out-of-range entries are clamped on device and counted
        (:meth:`invalid_actions`)."""
        torch = _torch()
        a = actions
        N, A = self.n_envs, self.n_agents
        if tuple(a.shape) != (N, A, 6):
            raise ValueError(f'actions must have shape {(N, A, 6)}, got {tuple(a.shape)}')
        if validate:
            hi = torch.tensor([3, 3, 3, 2, 2, 2], device=a.device)
            if bool(((a < 0) | (a >= hi)).any()):
                raise AssertionError('Invalid action: outside MultiDiscrete([3, 3, 3, 2, 2, 2])')
        if a.dtype != torch.int8 or a.device != self.device or not a.is_contiguous():
            self._act.copy_(a)
            a = self._act
        obs, rew, done = (self.obs, self.rewards, self.dones) if out is None else out
        if out is not None:
            for t, shp, dt in ((obs, (N, A, self.obs_dim), torch.float32), (rew, (N, A), torch.float32),
                               (done, (N,), torch.uint8)):
                if tuple(t.shape) != shp or t.dtype != dt or not t.is_contiguous() or t.device != self.device:
                    raise ValueError(f'out tensor must be contiguous {dt} {shp} on {self.device}')
        check(self._lib.mas_step(self._h, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
                                 ctypes.c_void_p(rew.data_ptr()), ctypes.c_void_p(done.data_ptr()),
                                 int(self.auto_reset), self._stream()))
        return obs, rew, done, {}

    def supports_step_x(self) -> bool:
        """mas_step_x can run this env (no lidars; an auto-reset in place)."""
        return bool(self._lib.mas_step_x_supported(self._h, int(self.auto_reset)))

    def step_x(self, actions, x, rewards, dones):
        """mas_step writing the observation rows as bf16 policy-input rows:
        x bf16 [N * A, Dx] (or [N, A, Dx]), Dx a multiple of 4 >= obs_dim;
        columns [0, obs_dim) are written (the fp32 rows of `step` rounded to
        bf16), the rest untouched.  rewards [N, A] fp32, dones [N] uint8.
        actions as for `step` (int8, contiguous, on this device)."""
        torch = _torch()
        N, A = self.n_envs, self.n_agents
        if tuple(actions.shape) != (N, A, 6) or actions.dtype != torch.int8 or not actions.is_contiguous():
            raise ValueError('actions must be contiguous int8 [N, A, 6]')
        if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.numel() % (N * A) != 0:
            raise ValueError('x must be contiguous bf16 [N * A, Dx]')
        Dx = x.numel() // (N * A)
        check(self._lib.mas_step_x(self._h, ctypes.c_void_p(actions.data_ptr()), ctypes.c_void_p(x.data_ptr()), Dx,
                                   ctypes.c_void_p(rewards.data_ptr()), ctypes.c_void_p(dones.data_ptr()),
                                   int(self.auto_reset), self._stream()))

    def flush_stats(self):
        """Per-env stats accumulated since the last flush, float [N, 19]
        (reward0..7, kills0..7, steps, heals_used, boxes_placed)."""
        torch = _torch()
        s = torch.zeros((self.n_envs, MAS_STATS_WIDTH), dtype=torch.float32, device=self.device)
        check(self._lib.mas_flush_stats(self._h, ctypes.c_void_p(s.data_ptr()), self._stream()))
        return s

    def split(self, flat):
        """View a [..., A, D] obs tensor as the reference's obs dict."""
        out = OrderedDict()
        for k, (off, shp) in self.layout.items():
            size = int(np.prod(shp))
            out[k] = flat[..., off:off + size].reshape(*flat.shape[:-1], *shp)
        return out

    def debug_counters(self):
        """{'phys_general_envs': envs of the last step that ran the general
        physics kernel (left the contact-free fast path)}; synchronises."""
        out = (ctypes.c_int64 * 1)()
        check(self._lib.mas_debug_counters(self._h, out))
        return {'phys_general_envs': int(out[0])}

    def debug_guards(self):
        """{'list_overflow': appends to the general-path / SolveTOI lists that
        their bounds refused (0 unless a kernel breaks the list invariant)};
        synchronises."""
        out = (ctypes.c_int64 * 1)()
        check(self._lib.mas_debug_guards(self._h, out))
        return {'list_overflow': int(out[0])}

    def force_general(self, on: bool = True, one_lane_solve: bool = False):
        """Test diagnostics: every env takes the general physics path (on);
        one_lane_solve (test library libmas_ab.so only): the general path runs
        the one-lane k_gen_solve + k_gen_toi instead of k_gen_solve_g."""
        bits = getattr(self, '_dbg_bits', 0) & 12
        self._dbg_bits = bits | int(bool(on)) | (2 if one_lane_solve else 0)
        check(self._lib.mas_debug_force_general(self._h, self._dbg_bits))

    def split_step(self, mode=None):
        """Test diagnostics: how mas_step uses the side stream (same results):
        0 the caller's stream alone, None the handle's default (the slow
        split, MAS_SPLIT)."""
        bits = {0: 8, None: 0}[mode]
        self._dbg_bits = (getattr(self, '_dbg_bits', 0) & 3) | bits
        check(self._lib.mas_debug_force_general(self._h, self._dbg_bits))

    def invalid_actions(self, reset: bool = True) -> int:
        """Env-steps whose actions were out of range (clamped on device) since
        the last reset of the count (mas_invalid_actions; synchronises)."""
        out = ctypes.c_int64()
        check(self._lib.mas_invalid_actions(self._h, ctypes.byref(out), int(reset)))
        return int(out.value)

    def gen_flags(self, out=None):
        """uint8 [N] device tensor: 1 where the env left the contact-free
        physics fast path in the last step (test diagnostics)."""
        torch = _torch()
        if out is None:
            out = torch.empty((self.n_envs,), dtype=torch.uint8, device=self.device)
        check(self._lib.mas_debug_gen_flags(self._h, ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def set_toi_counter(self, counts=None):
        """Test diagnostics: accumulate per-env SolveTOI events (+65536 per
        agent that hit the sub-step cap) into the int32 [N] device tensor
        `counts` on every step; None stops."""
        if counts is not None:
            torch = _torch()
            assert counts.dtype == torch.int32 and counts.shape == (self.n_envs,) and counts.is_contiguous()
        self._toi_counts = counts  # keep alive while the kernels write it
        check(self._lib.mas_debug_set_toi_counter(self._h, None if counts is None else
                                                   ctypes.c_void_p(counts.data_ptr())))

    def render_view(self, env: int = 0) -> Dict[str, Any]:
        """Bodies of env `env` for rendering (mas_render_view; synchronises)."""
        buf = (ctypes.c_float * MAS_RENDER_VIEW_FLOATS)()
        check(self._lib.mas_render_view(self._h, int(env), buf))
        return parse_render_view(np.frombuffer(buf, dtype=np.float32).copy())

    def state_bytes(self) -> int:
        return int(self._lib.mas_state_bytes(self._h))

    def get_state(self):
        torch = _torch()
        buf = torch.empty((self.state_bytes(),), dtype=torch.uint8, device=self.device)
        check(self._lib.mas_get_state(self._h, ctypes.c_void_p(buf.data_ptr()), self._stream()))
        return buf

    def set_state(self, buf):
        if buf.numel() != self.state_bytes() or buf.device != self.device:
            raise ValueError(f'env state image of {buf.numel()} bytes, expected {self.state_bytes()} on {self.device}')
        buf = buf.contiguous()
        check(self._lib.mas_set_state(self._h, ctypes.c_void_p(buf.data_ptr()), self._stream()))

    def state_meta(self):
        """What a mas_get_state image depends on: the resolved config struct
        (its bytes, hashed), the number of envs and the image size (which
        encodes the capacity class and the state stride).  Plain Python values,
        stored in PPOTrainer checkpoints and compared on load."""
        import hashlib
        cfg = bytes(memoryview(self._cfg))
        return {'config_sha256': hashlib.sha256(cfg).hexdigest(), 'n_envs': self.n_envs, 'shards': [self.n_envs],
                'state_bytes': self.state_bytes(), 'n_agents': self.n_agents, 'obs_dim': self.obs_dim}

    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            self._lib.mas_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def torch_uint8():
    return _torch().uint8


class ShardedVecMaSurvival:
    """N envs as `shards` independent VecMaSurvival handles over consecutive
    env ranges, each stepped on its own HIP stream.

    The env step is latency-bound (one lane per env: at N = 65536 one wave per
    SIMD, each kernel as long as its slowest wave), so independent shards on
    separate streams overlap: one shard's kernels fill the SIMDs another
    shard's tail leaves idle, and in the PPO rollout each shard's policy
    forward overlaps the other shards' env kernels (`PPOTrainer` launches
    act + step per shard through `shard_slices`).  Results are identical to
    one handle over all N envs: env e keeps seed seeds[e], and the policy's
    sampling RNG is keyed by the global row (`mas_policy_act_rows`).

    `step` / `reset` order the shards after the caller's current stream and
    the caller's stream after all shards, so callers see one env."""

    def __init__(self, config: Optional[Dict[str, Dict[str, Any]]] = None, n_envs: int = 1, shards: int = 2,
                 device=None, seeds: Optional[Sequence[int]] = None, auto_reset: bool = True):
        torch = _torch()
        n_envs, shards = int(n_envs), int(shards)
        if shards < 1 or n_envs < shards:
            raise ValueError('need 1 <= shards <= n_envs')
        seeds = list(range(n_envs)) if seeds is None else list(seeds)
        if len(seeds) != n_envs:
            raise ValueError('need one seed per env')
        bounds = [n_envs * k // shards for k in range(shards + 1)]
        self.envs = [VecMaSurvival(config, n_envs=bounds[k + 1] - bounds[k], device=device,
                                   seeds=seeds[bounds[k]:bounds[k + 1]], auto_reset=auto_reset)
                     for k in range(shards)]
        self.bounds = bounds
        e0 = self.envs[0]
        self.rc, self.device, self.auto_reset = e0.rc, e0.device, e0.auto_reset
        self.n_envs, self.n_agents, self.obs_dim, self.layout = n_envs, e0.n_agents, e0.obs_dim, e0.layout
        self.observation_space, self.action_space = e0.observation_space, e0.action_space
        self.streams = [torch.cuda.Stream(device=self.device) for _ in range(shards)]
        N, A, D = n_envs, self.n_agents, self.obs_dim
        self.obs = torch.zeros((N, A, D), dtype=torch.float32, device=self.device)
        self.rewards = torch.zeros((N, A), dtype=torch.float32, device=self.device)
        self.dones = torch.zeros((N,), dtype=torch.uint8, device=self.device)

    def shard_slices(self):
        """[(env, stream, first env, end env)] per shard."""
        return [(e, s, self.bounds[k], self.bounds[k + 1]) for k, (e, s) in enumerate(zip(self.envs, self.streams))]

    def fork(self):
        """Shard streams wait for the caller's current stream."""
        cur = _torch().cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)

    def join(self):
        """The caller's current stream waits for every shard."""
        cur = _torch().cuda.current_stream(self.device)
        for s in self.streams:
            cur.wait_stream(s)

    def reset(self, mask=None):
        torch = _torch()
        self.fork()
        for e, s, lo, hi in self.shard_slices():
            with torch.cuda.stream(s):
                o = e.reset(None if mask is None else mask[lo:hi])
                self.obs[lo:hi].copy_(o)
        self.join()
        return self.obs

    def step(self, actions, out=None, validate=False):
        """As VecMaSurvival.step over the shards; validate checks every
        action against the action space first (the reference's assert,
        masurvival_env.py:80), otherwise out-of-range entries are clamped on
        device and counted (:meth:`invalid_actions`)."""
        torch = _torch()
        N, A = self.n_envs, self.n_agents
        if tuple(actions.shape) != (N, A, 6):
            raise ValueError(f'actions must have shape {(N, A, 6)}, got {tuple(actions.shape)}')
        if validate:
            hi = torch.tensor([3, 3, 3, 2, 2, 2], device=actions.device)
            if bool(((actions < 0) | (actions >= hi)).any()):
                raise AssertionError('Invalid action: outside MultiDiscrete([3, 3, 3, 2, 2, 2])')
        obs, rew, done = (self.obs, self.rewards, self.dones) if out is None else out
        self.fork()
        for e, s, lo, hi in self.shard_slices():
            with torch.cuda.stream(s):
                e.step(actions[lo:hi], out=(obs[lo:hi], rew[lo:hi], done[lo:hi]))
        self.join()
        return obs, rew, done, {}

    def invalid_actions(self, reset: bool = True) -> int:
        """Sum over the shards of VecMaSurvival.invalid_actions (synchronises)."""
        self.join()
        return sum(e.invalid_actions(reset) for e in self.envs)

    def supports_step_x(self) -> bool:
        return all(e.supports_step_x() for e in self.envs)

    def flush_stats(self):
        self.join()
        return _torch().cat([e.flush_stats() for e in self.envs])

    def debug_counters(self):
        _torch().cuda.synchronize(self.device)
        d = [e.debug_counters() for e in self.envs]
        return {k: sum(x[k] for x in d) for k in d[0]}

    def split(self, flat):
        return self.envs[0].split(flat)

    def state_bytes(self) -> int:
        return sum(e.state_bytes() for e in self.envs)

    def get_state(self):
        """The shards' mas_get_state images, concatenated in shard order."""
        self.join()
        return _torch().cat([e.get_state() for e in self.envs])

    def set_state(self, buf):
        """Split a get_state() image at the shards' byte counts and restore
        each shard from its part."""
        sizes = [e.state_bytes() for e in self.envs]
        if buf.numel() != sum(sizes) or buf.device != self.device:
            raise ValueError(f'env state image of {buf.numel()} bytes, expected {sum(sizes)} on {self.device}')
        self.join()
        off = 0
        for e, n in zip(self.envs, sizes):
            e.set_state(buf[off:off + n])
            off += n
        _torch().cuda.synchronize(self.device)

    def state_meta(self):
        """What a checkpoint's env state depends on (see VecMaSurvival.state_meta)."""
        m = self.envs[0].state_meta()
        m['n_envs'] = self.n_envs
        m['shards'] = [e.n_envs for e in self.envs]
        m['state_bytes'] = self.state_bytes()
        return m

    def close(self):
        for e in self.envs:
            e.close()
