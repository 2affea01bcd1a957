"""On-device PPO rollout for VecMaSurvival.

The reference ships no trainer; this is the consumer the batched env step is
built for.  Everything stays in HBM:

* ``RolloutBuffer`` -- obs [T+1, N, A, D] (the env kernel writes each step's
  observation straight into row t+1), actions int8 [T, N, A, 6], log-probs,
  values [T+1, N, A], rewards [T, N, A], dones uint8 [T, N]; advantages and
  returns [T, N, A].
* GAE(gamma, lambda) is the HIP ``mas_gae`` kernel (one lane per agent
  column, backward over T), which also returns the fp64 advantage sums.
* The policy is a shared-parameter MLP (obs D -> 256 -> 256, tanh) with six
  categorical heads (MultiDiscrete [3,3,3,2,2,2]) and a value head; forward
  passes run under bf16 autocast (hipBLASLt GEMMs), losses in fp32.

Multi-GPU (one process per GPU, envs sharded): the only collectives are one
fp64 all-reduce of (sum adv, sum adv^2, count) per rollout and one flat
gradient all-reduce (average) per minibatch -- RCCL over xGMI when the process
group is 'nccl', gloo in the CPU tests.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .abi import check, load_library

HEADS = (3, 3, 3, 2, 2, 2)
N_LOGITS = sum(HEADS)

# MAS_ROCTX=1 brackets the trainer's phases (rollout, gae, update) with roctx
# ranges (torch.cuda.nvtx is roctx on ROCm) for rocprofv3 --marker-trace.
_ROCTX = os.environ.get('MAS_ROCTX', '0') == '1'


class _phase:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if _ROCTX:
            torch.cuda.nvtx.range_push(self.name)

    def __exit__(self, *exc):
        if _ROCTX:
            torch.cuda.nvtx.range_pop()


@dataclass
class PPOConfig:
    horizon: int = 64          # T
    gamma: float = 0.99
    lam: float = 0.95
    hidden: int = 256
    lr: float = 3e-4
    epochs: int = 1
    minibatches: int = 4
    clip: float = 0.2
    vf_coef: float = 0.5
    ent_coef: float = 0.01
    max_grad_norm: float = 0.5
    autocast_bf16: bool = True
    # fused HIP policy kernels (mas_policy_act / mas_policy_train): default on
    # a GPU when hidden == 256; the torch path stays as the CPU / reference path
    fused: Optional[bool] = None
    # the advantage-statistics and gradient all-reduces: None = when the
    # process group has more than one rank; True forces them at world size 1
    # too (the one-GPU RCCL test runs the exact calls of the 8-GPU bench)
    allreduce: Optional[bool] = None
    # fused path: the env writes the policy's bf16 input rows itself
    # (mas_step_x) instead of fp32 obs rows the act kernel re-reads and
    # converts; None = whenever the env supports it (same bits either way)
    x_obs: Optional[bool] = None


def _split_k(m: int, cap: int = int(os.environ.get('MAS_SPLITK_CAP', '128'))) -> int:
    c = 1
    while c < cap and m % (2 * c) == 0 and m // (2 * c) >= 4096:
        c *= 2
    return c


class _LinearSplitKFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is computed split-K: for a PPO
    minibatch of millions of rows, dW = dY^T X has a tiny M x N and a huge K,
    and a single GEMM there launches a handful of tiles; a batched GEMM over
    row chunks followed by a sum fills the GPU."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        x2 = x.reshape(-1, x.shape[-1])
        g2 = gy.reshape(-1, gy.shape[-1])
        gx = (g2 @ w).reshape(x.shape) if ctx.needs_input_grad[0] else None
        m = x2.shape[0]
        c = _split_k(m)
        gw = torch.bmm(g2.reshape(c, m // c, -1).transpose(1, 2), x2.reshape(c, m // c, -1)).sum(0)
        gb = g2.reshape(c, m // c, -1).sum(1).sum(0)
        return gx, gw.to(w.dtype), gb


class LinearSplitK(nn.Linear):
    def forward(self, x):
        if torch.is_autocast_enabled(x.device.type):
            dt = torch.get_autocast_dtype(x.device.type)
            with torch.autocast(x.device.type, enabled=False):
                return _LinearSplitKFn.apply(x.to(dt), self.weight.to(dt), self.bias.to(dt))
        return _LinearSplitKFn.apply(x, self.weight, self.bias)


class PolicyMLP(nn.Module):
    """Shared across agents: obs [.., D] -> (logits [.., 15], value [..])."""

    def __init__(self, obs_dim: int, hidden: int = 256):
        super().__init__()
        self.body = nn.Sequential(LinearSplitK(obs_dim, hidden), nn.Tanh(), LinearSplitK(hidden, hidden), nn.Tanh())
        self.head = LinearSplitK(hidden, N_LOGITS + 1)

    def forward(self, x):
        h = self.head(self.body(x))
        return h[..., :N_LOGITS].float(), h[..., N_LOGITS].float()

    def forward_raw(self, x):
        """[.., 16] fp32 head output: 15 logits then the value."""
        return self.head(self.body(x)).float()


def _split_heads(logits):
    return torch.split(logits, HEADS, dim=-1)


def sample_actions(logits, gen: Optional[torch.Generator] = None):
    """Gumbel-max sample of the six heads; returns (int8 [.., 6], logp [..])."""
    acts, logp = [], 0.0
    for lg in _split_heads(logits):
        lsm = F.log_softmax(lg, dim=-1)
        u = torch.rand(lg.shape, device=lg.device, generator=gen).clamp_(1e-20, 1.0)
        a = torch.argmax(lsm - torch.log(-torch.log(u)), dim=-1)
        acts.append(a)
        logp = logp + lsm.gather(-1, a.unsqueeze(-1)).squeeze(-1)
    return torch.stack(acts, dim=-1).to(torch.int8), logp


def sample_actions_hip(logits, seed, step, actions_out, logp_out):
    """HIP sampler (include/masurvival.h mas_sample_actions): logits [M, >=15]
    fp32 with unit column stride; writes actions_out int8 [M, 6], logp_out [M]."""
    lib = load_library()
    M = logits.shape[0]
    assert logits.is_cuda and logits.dtype == torch.float32 and logits.stride(1) == 1
    assert actions_out.is_contiguous() and logp_out.is_contiguous()
    check(lib.mas_sample_actions(M, ctypes.c_void_p(logits.data_ptr()), logits.stride(0), seed, step,
                                 ctypes.c_void_p(actions_out.data_ptr()), ctypes.c_void_p(logp_out.data_ptr()),
                                 ctypes.c_void_p(torch.cuda.current_stream(logits.device).cuda_stream)))


def evaluate_actions(logits, actions):
    """log-prob and entropy of given actions [.., 6]."""
    logp, ent = 0.0, 0.0
    a = actions.long()
    for k, lg in enumerate(_split_heads(logits)):
        lsm = F.log_softmax(lg, dim=-1)
        logp = logp + lsm.gather(-1, a[..., k:k + 1]).squeeze(-1)
        ent = ent - (lsm.exp() * lsm).sum(-1)
    return logp, ent


def gae_scratch(n_columns, device):
    """The partial-sum scratch one mas_gae call needs (mas_gae_scratch_doubles)."""
    n = load_library().mas_gae_scratch_doubles(int(n_columns))
    return torch.empty((n,), device=device, dtype=torch.float64)


def gae(rewards, values, dones, gamma, lam, adv_out, ret_out, sums_out, n_agents, stream=None, scratch=None):
    """HIP GAE over [T, N*A] columns (include/masurvival.h mas_gae).  scratch:
    float64 device tensor of mas_gae_scratch_doubles(N*A) (allocated here when
    None); concurrent calls need their own scratch and outputs."""
    lib = load_library()
    T = rewards.shape[0]
    M = rewards[0].numel()
    for t in (rewards, values, adv_out, ret_out):
        assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
    assert values.shape[0] == T + 1 and dones.shape[0] == T and dones.dtype == torch.uint8
    assert dones[0].numel() * n_agents == M and sums_out.dtype == torch.float64
    if scratch is None:
        scratch = gae_scratch(M, rewards.device)
    assert scratch.is_cuda and scratch.dtype == torch.float64 and scratch.numel() >= lib.mas_gae_scratch_doubles(M)
    s = stream if stream is not None else torch.cuda.current_stream(rewards.device).cuda_stream
    check(lib.mas_gae(T, M, n_agents, ctypes.c_void_p(rewards.data_ptr()), ctypes.c_void_p(values.data_ptr()),
                      ctypes.c_void_p(dones.data_ptr()), float(gamma), float(lam),
                      ctypes.c_void_p(adv_out.data_ptr()), ctypes.c_void_p(ret_out.data_ptr()),
                      ctypes.c_void_p(sums_out.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
                      ctypes.c_void_p(s)))


def adv_normalize(adv, stats, stream=None):
    """adv (DEVICE fp32, contiguous) normalised in place from stats = fp64
    [sum, sum of squares, count] (include/masurvival.h mas_adv_normalize):
    adv.sub_(mean.float()).div_(var.sqrt().float() + 1e-8), one launch."""
    assert adv.is_cuda and adv.dtype == torch.float32 and adv.is_contiguous()
    assert stats.dtype == torch.float64 and stats.numel() == 3 and stats.is_contiguous()
    lib = load_library()
    st = stream if stream is not None else torch.cuda.current_stream(adv.device).cuda_stream
    check(lib.mas_adv_normalize(adv.numel(), ctypes.c_void_p(adv.data_ptr()), ctypes.c_void_p(stats.data_ptr()),
                                ctypes.c_void_p(st)))


def gae_reference(rewards, values, dones, gamma, lam, n_agents):
    """Plain torch fp32 restatement of mas_gae (the numerics test's reference)."""
    T = rewards.shape[0]
    r = rewards.reshape(T, -1)
    v = values.reshape(T + 1, -1)
    nt = 1.0 - dones.reshape(T, -1).float().repeat_interleave(n_agents, dim=1)
    adv = torch.zeros_like(r)
    a = torch.zeros_like(r[0])
    for t in range(T - 1, -1, -1):
        delta = r[t] + gamma * v[t + 1] * nt[t] - v[t]
        a = delta + gamma * lam * nt[t] * a
        adv[t] = a
    return adv.reshape(rewards.shape), (adv + v[:T]).reshape(rewards.shape)


def gae_reference_into(rewards, values, dones, gamma, lam, adv_out, ret_out, sums_out, n_agents, stream=None,
                       scratch=None):
    """Same contract as gae() on host tensors -- test double for the CPU
    multi-process tests only (the product trainer always runs the HIP kernel)."""
    adv, ret = gae_reference(rewards, values, dones, gamma, lam, n_agents)
    adv_out.copy_(adv)
    ret_out.copy_(ret)
    sums_out[0] = adv.double().sum()
    sums_out[1] = (adv.double() ** 2).sum()


# MAS_POL_DW: the policy layers ('2', '3') whose weight gradients come from
# the mas_policy_dw kernel (LDS-staged split-K MFMA, k_dw_lds) instead of the
# split-K GEMMs (e.g. '23', '2', '0').  Per 4.2M-row minibatch (r02p7): layer
# 2 1.14 ms against 1.28 for its GEMM, layer 3 0.54 against 0.52 + the GEMM
# path's split-K sum; the update 30.3 ms with '2', 29.5 with '23'.
_DW_LAYERS = os.environ.get('MAS_POL_DW', '23')
# MAS_ACT_PAD: extra columns of the feature-major activation buffers (row
# stride M + pad; 0 = the power-of-two stride: dW2 kernel 1.21 vs 0.85 ms)
_ACT_PAD = int(os.environ.get('MAS_ACT_PAD', '64'))
# MAS_POL_LAYOUT: activation layout of the update ('fm' feature-major
# [F][rows] with the DPP row pairing and the mas_policy_dw kernels, 'rm'
# row-major [rows][F] written as plain 16-B stores, weight gradients as
# row-sum GEMMs)
_POL_LAYOUT = os.environ.get('MAS_POL_LAYOUT', 'fm')
_RM_LDH = 264  # row stride of the row-major h1 / h2 (column 256: ones)
# MAS_FUSED_ADAM=0: the torch clip_grad_norm_ + Adam step in the fused trainer
_FUSED_ADAM = os.environ.get('MAS_FUSED_ADAM', '1') != '0'


def _splitk_nt(a, b):
    """a [F, K] @ b[G, K]^T in fp32 for a huge K, as a batched GEMM over K
    chunks (bf16 in, partial sums reduced in fp32; rows may be strided)."""
    F_, K = a.shape
    G = b.shape[0]
    c = _split_k(K)
    pa = a.unflatten(1, (c, K // c)).permute(1, 0, 2)
    pb = b.unflatten(1, (c, K // c)).permute(1, 2, 0)
    return torch.bmm(pa, pb).sum(0, dtype=torch.float32)


def _splitk_tn(a, b):
    """a [K, F]^T @ b [K, G] in fp32 for a huge K (both row-major, any row
    stride): the row-sum GEMM of the row-major activations."""
    K = a.shape[0]
    c = _split_k(K)
    pa = a.unflatten(0, (c, K // c)).transpose(1, 2)
    pb = b.unflatten(0, (c, K // c))
    return torch.bmm(pa, pb).sum(0, dtype=torch.float32)


def _splitk_nn(a, x):
    """a [F, K] @ x [K, G] in fp32 for a huge K (x row-major, any row stride)."""
    F_, K = a.shape
    c = _split_k(K)
    pa = a.unflatten(1, (c, K // c)).permute(1, 0, 2)
    px = x.reshape(c, K // c, x.shape[1]) if x.is_contiguous() else x.unflatten(0, (c, K // c))
    return torch.bmm(pa, px).sum(0, dtype=torch.float32)


class FusedPolicy:
    """The HIP policy kernels (include/masurvival.h mas_policy_*) over a
    PolicyMLP's fp32 parameters: ``pack()`` after every optimizer step, ``act``
    for the rollout, ``grads`` for one PPO minibatch.  Hidden width 256."""

    def __init__(self, policy: 'PolicyMLP', obs_dim: int, device):
        self.lib = load_library()
        self.policy, self.D, self.device = policy, int(obs_dim), device
        self.Dp = 16 * ((self.D + 15) // 16)      # columns the kernels read / write
        self.Dx = 16 * ((self.D + 1 + 15) // 16)  # row stride of x: room for the bias column at index D
        w1, w2 = policy.body[0].weight, policy.body[2].weight
        assert w1.shape == (256, self.D) and w2.shape == (256, 256) and policy.head.weight.shape == (16, 256)
        self.packed = torch.empty((int(self.lib.mas_policy_packed_bytes(self.D)),), dtype=torch.uint8, device=device)
        self._bufs = None
        self._dwbuf = {}
        self.layout = _POL_LAYOUT
        if self.layout == 'rm':
            perm = [int(self.lib.mas_policy_rm_feature(c)) for c in range(256)]  # stored column -> feature
            q = [0] * 256
            for c, f in enumerate(perm):
                q[f] = c
            self._rm_q = torch.tensor(q, dtype=torch.long, device=device)  # feature -> stored column

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @torch.no_grad()
    def pack(self):
        p = self.policy
        ts = [p.body[0].weight, p.body[0].bias, p.body[2].weight, p.body[2].bias, p.head.weight, p.head.bias]
        ts = [t.detach().float().contiguous() for t in ts]
        check(self.lib.mas_policy_pack(self.D, *[ctypes.c_void_p(t.data_ptr()) for t in ts],
                                       ctypes.c_void_p(self.packed.data_ptr()), self._stream()))

    def x_buffer(self, *shape):
        """bf16 policy-input rows [*shape, Dx] with the bias column (index D) = 1."""
        x = torch.zeros((*shape, self.Dx), dtype=torch.bfloat16, device=self.device)
        x[..., self.D] = 1.0
        return x

    @torch.no_grad()
    def act(self, obs, seed, step, actions, logp, value, xb=None, first_row=0):
        """obs [M, D] fp32 rows -> actions int8 [M, 6], logp, value [M];
        xb [M, Dx] bf16 (optional, from x_buffer) receives the rows as the
        update reads them.  first_row: index of obs[0] in the whole batch when
        the batch is launched in shards (the sampling RNG is keyed by it)."""
        M = obs.shape[0]
        assert obs.is_contiguous() and obs.dtype == torch.float32 and obs.shape[1] == self.D
        assert actions.is_contiguous() and logp.is_contiguous() and value.is_contiguous()
        xp = ctypes.c_void_p(xb.data_ptr()) if xb is not None else None
        check(self.lib.mas_policy_act_rows(ctypes.c_void_p(self.packed.data_ptr()), self.D, M, int(first_row),
                                           ctypes.c_void_p(obs.data_ptr()), xp, self.Dx, int(seed), int(step),
                                           ctypes.c_void_p(actions.data_ptr()), ctypes.c_void_p(logp.data_ptr()),
                                           ctypes.c_void_p(value.data_ptr()), self._stream()))

    @torch.no_grad()
    def act_x(self, xb, seed, step, actions, logp, value, first_row=0):
        """act over bf16 input rows xb [M, Dx] (x_buffer layout, e.g. written by
        mas_step_x): the same actions, log-probs and values as act on the fp32
        rows they were rounded from; xb is not written."""
        M = xb.shape[0]
        assert xb.is_contiguous() and xb.dtype == torch.bfloat16 and xb.shape[1] == self.Dx
        assert actions.is_contiguous() and logp.is_contiguous() and value.is_contiguous()
        check(self.lib.mas_policy_act_x(ctypes.c_void_p(self.packed.data_ptr()), self.D, M, int(first_row),
                                        ctypes.c_void_p(xb.data_ptr()), self.Dx, int(seed), int(step),
                                        ctypes.c_void_p(actions.data_ptr()), ctypes.c_void_p(logp.data_ptr()),
                                        ctypes.c_void_p(value.data_ptr()), self._stream()))

    def _buffers_rm(self, M):
        if self._bufs is None or self._bufs['M'] != M:
            bf = dict(dtype=torch.bfloat16, device=self.device)
            nb = int(self.lib.mas_policy_blocks(M))
            h1 = torch.zeros((M, _RM_LDH), **bf)
            h2 = torch.zeros((M, _RM_LDH), **bf)
            h1[:, 256] = 1.0
            h2[:, 256] = 1.0
            self._bufs = {'M': M, 'h1': h1, 'h2': h2, 'da1': torch.empty((M, 256), **bf),
                          'da2': torch.empty((M, 256), **bf), 'dz': torch.empty((M, 16), **bf),
                          'part': torch.empty((nb, 4), dtype=torch.float32, device=self.device)}
        return self._bufs

    def _grads_rm(self, xb, actions, old_logp, adv, ret, cfg):
        M = xb.shape[0]
        B = self._buffers_rm(M)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        check(self.lib.mas_policy_train_rm(ptr(self.packed), self.D, M, ptr(xb), self.Dx, ptr(actions),
                                           ptr(old_logp), ptr(adv), ptr(ret), cfg.clip, cfg.vf_coef, cfg.ent_coef,
                                           1.0 / M, ptr(B['h1']), ptr(B['h2']), _RM_LDH, ptr(B['da1']),
                                           ptr(B['da2']), ptr(B['dz']), ptr(B['part']), self._stream()))
        q = self._rm_q
        g3 = _splitk_tn(B['dz'], B['h2'][:, :257])               # [16, 257], columns stored order
        g2 = _splitk_tn(B['da2'], B['h1'][:, :257])              # [256, 257]
        g1 = _splitk_tn(B['da1'], xb[:, :self.D + 1])            # [256, D + 1]
        g2 = g2.index_select(0, q)
        p = self.policy
        l1, l2, l3 = p.body[0], p.body[2], p.head
        grads = {l3.weight: g3[:, :256].index_select(1, q), l3.bias: g3[:, 256],
                 l2.weight: g2[:, :256].index_select(1, q), l2.bias: g2[:, 256],
                 l1.weight: g1.index_select(0, q)[:, :self.D], l1.bias: g1[:, self.D].index_select(0, q)}
        for prm, g in grads.items():
            if prm.grad is None:
                prm.grad = g.to(prm.dtype).clone(memory_format=torch.contiguous_format)
            else:
                prm.grad.copy_(g)
        s = B['part'].sum(0) / M
        pg, v, ent, clipfrac = s[0], s[1], s[2], s[3]
        return pg + cfg.vf_coef * v - cfg.ent_coef * ent, pg, v, ent, clipfrac

    def _buffers(self, M):
        if self._bufs is None or self._bufs['M'] != M:
            bf = dict(dtype=torch.bfloat16, device=self.device)
            nb = int(self.lib.mas_policy_blocks(M))
            # h1 / h2 carry a row of ones (row 256): dW @ [h; 1]^T yields the bias gradient as its last column.
            # Row stride ld = M + _ACT_PAD: a power-of-two stride (the 4.2M-row minibatch) puts every
            # feature row on the same HBM channels (mas_policy_train_ld)
            ld = M + _ACT_PAD
            h1, h2 = torch.empty((257, ld), **bf), torch.empty((257, ld), **bf)
            h1[256] = 1.0
            h2[256] = 1.0
            self._bufs = {'M': M, 'ld': ld, 'h1': h1, 'h2': h2,
                          'da1': torch.empty((256, ld), **bf), 'da2': torch.empty((256, ld), **bf),
                          'dz': torch.empty((16, ld), **bf),
                          'part': torch.empty((nb, 4), dtype=torch.float32, device=self.device)}
        return self._bufs

    def _dw(self, a, h, F, M, into=None):
        """(a[:, :M] @ h[:256, :M]^T, a.sum(1)) in fp32 via mas_policy_dw.
        into: (weight, bias) fp32 tensors that are one contiguous span of
        F * 256 + F floats (the flat gradient buffer of FusedAdam): the sums
        land there directly and (None, None) is returned."""
        key = ('dw', F, M)
        if key not in self._dwbuf:
            n = int(self.lib.mas_policy_dw_scratch(F, 256, M))
            self._dwbuf[key] = (torch.empty((n,), dtype=torch.float32, device=self.device),
                                torch.empty((F * 256 + F,), dtype=torch.float32, device=self.device))
        scratch, out = self._dwbuf[key]
        optr = into[0].data_ptr() if into is not None else out.data_ptr()
        check(self.lib.mas_policy_dw(F, 256, M, ctypes.c_void_p(a.data_ptr()), a.stride(0), ctypes.c_void_p(h.data_ptr()),
                                     h.stride(0), ctypes.c_void_p(optr), ctypes.c_void_p(scratch.data_ptr()),
                                     self._stream()))
        if into is not None:
            return None, None
        return out[:F * 256].view(F, 256), out[F * 256:]

    @staticmethod
    def _grad_span(w, b):
        """(w.grad, b.grad) when they are one contiguous fp32 span, weight then
        bias (FusedAdam's flat buffer), else None."""
        gw, gb = w.grad, b.grad
        if gw is None or gb is None or gw.dtype != torch.float32 or gb.dtype != torch.float32:
            return None
        if not (gw.is_contiguous() and gb.is_contiguous()):
            return None
        if gw.untyped_storage().data_ptr() != gb.untyped_storage().data_ptr():
            return None
        if gb.data_ptr() != gw.data_ptr() + 4 * gw.numel():
            return None
        return gw, gb

    def grads(self, xb, actions, old_logp, adv, ret, cfg: 'PPOConfig', stats: bool = True):
        """Sets .grad of the policy parameters to the gradient of the PPO loss
        (mean over the M rows) and returns (loss, pg, v, entropy, clipfrac);
        stats=False skips those reductions (the update keeps only the last
        minibatch's) and returns None."""
        M = xb.shape[0]
        assert xb.dtype == torch.bfloat16 and xb.shape[1] == self.Dx and xb.is_contiguous()
        for t in (actions, old_logp, adv, ret):
            assert t.is_contiguous()
        if self.layout == 'rm':
            return self._grads_rm(xb, actions, old_logp, adv, ret, cfg)
        B = self._buffers(M)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        check(self.lib.mas_policy_train_ld(ptr(self.packed), self.D, M, ptr(xb), self.Dx, ptr(actions),
                                           ptr(old_logp), ptr(adv), ptr(ret), cfg.clip, cfg.vf_coef, cfg.ent_coef,
                                           1.0 / M, ptr(B['h1']), ptr(B['h2']), ptr(B['da1']), ptr(B['da2']),
                                           ptr(B['dz']), B['ld'], ptr(B['part']), self._stream()))
        B = {k: (v[:, :M] if k in ('h1', 'h2', 'da1', 'da2', 'dz') else v) for k, v in B.items()}
        p = self.policy
        l1, l2, l3 = p.body[0], p.body[2], p.head
        # layers 2 / 3: the split-K MFMA kernel (mas_policy_dw) where enabled,
        # else the split-K GEMM over the ones-row trick; layer 1 reads x
        # row-major: a GEMM.  With FusedAdam's flat gradient buffer the dW
        # kernels' sums land in .grad directly (no copy launches)
        if '3' in _DW_LAYERS and M % 32 == 0:
            g3w, g3b = self._dw(B['dz'], B['h2'], 16, M, into=self._grad_span(l3.weight, l3.bias))
        else:
            g3 = _splitk_nt(B['dz'], B['h2'])          # [16, 257]
            g3w, g3b = g3[:, :256], g3[:, 256]
        if '2' in _DW_LAYERS and M % 32 == 0:
            g2w, g2b = self._dw(B['da2'], B['h1'], 256, M, into=self._grad_span(l2.weight, l2.bias))
        else:
            g2 = _splitk_nt(B['da2'], B['h1'])         # [256, 257]
            g2w, g2b = g2[:, :256], g2[:, 256]
        g1 = _splitk_nn(B['da1'], xb[:, :self.D + 1])  # [256, D + 1]
        grads = {l3.weight: g3w, l3.bias: g3b, l2.weight: g2w, l2.bias: g2b,
                 l1.weight: g1[:, :self.D], l1.bias: g1[:, self.D]}
        for prm, g in grads.items():
            if g is None:
                continue  # written in place above
            if prm.grad is None:
                prm.grad = g.to(prm.dtype).clone(memory_format=torch.contiguous_format)
            else:
                prm.grad.copy_(g)
        if not stats:
            return None
        s = B['part'].sum(0) / M
        pg, v, ent, clipfrac = s[0], s[1], s[2], s[3]
        return pg + cfg.vf_coef * v - cfg.ent_coef * ent, pg, v, ent, clipfrac


def policy_loss_reference(policy, x, actions, old_logp, adv, ret, cfg: 'PPOConfig'):
    """Plain torch fp32 restatement of the PPO loss the fused kernels
    differentiate (the numerics tests' reference): x fp32 rows [M, D]."""
    logits, v = policy(x)
    lp, ent = evaluate_actions(logits, actions)
    ratio = torch.exp(lp - old_logp)
    pg = -torch.min(ratio * adv, ratio.clamp(1 - cfg.clip, 1 + cfg.clip) * adv).mean()
    vl = F.mse_loss(v, ret)
    return pg + cfg.vf_coef * vl - cfg.ent_coef * ent.mean(), pg, vl, ent.mean()


class FusedAdam:
    """clip_grad_norm_ + torch.optim.Adam.step() for the fused trainer as one
    HIP launch pair (include/masurvival.h mas_policy_adam).  The parameters,
    their gradients and both Adam moments become views into four flat fp32
    buffers; the torch.optim.Adam object keeps holding them as its state, so
    its state_dict (checkpoints) is unchanged.  bind_state() re-points that
    state after Adam.load_state_dict replaced it.

    Used only for the plain form it restates (supports()): one param group,
    a float lr, no weight decay, amsgrad, maximize or capturable state; any
    other optimizer setup stays on torch.  After step(), ``.grad`` of each
    parameter holds the raw summed minibatch gradient the kernel read (the
    1 / world scale and the clip are applied inside the kernel, not written
    back), unlike torch's clip_grad_norm_, which scales .grad in place."""

    @staticmethod
    def supports(opt) -> bool:
        if not isinstance(opt, torch.optim.Adam) or len(opt.param_groups) != 1:
            return False
        g = opt.param_groups[0]
        return (not g.get('weight_decay', 0) and not g.get('amsgrad', False) and not g.get('maximize', False)
                and not g.get('capturable', False) and not g.get('differentiable', False)
                and not isinstance(g['lr'], torch.Tensor))

    def __init__(self, params, opt: torch.optim.Adam, lib, device):
        self.params, self.opt, self.lib, self.device = list(params), opt, lib, device
        n = sum(p.numel() for p in self.params)
        f = dict(dtype=torch.float32, device=device)
        self.p, self.g = torch.empty((n,), **f), torch.zeros((n,), **f)
        self.m, self.v = torch.zeros((n,), **f), torch.zeros((n,), **f)
        self.scratch = torch.empty((int(lib.mas_policy_adam_scratch()),), **f)
        self.spans = []
        off = 0
        with torch.no_grad():
            for prm in self.params:
                k = prm.numel()
                self.p[off:off + k].copy_(prm.detach().reshape(-1))
                prm.data = self.p[off:off + k].view_as(prm)
                prm.grad = self.g[off:off + k].view_as(prm)
                self.spans.append((off, k))
                off += k
        self.bind_state()

    @torch.no_grad()
    def bind_state(self):
        for prm, (off, k) in zip(self.params, self.spans):
            st = self.opt.state[prm]
            if 'exp_avg' in st:
                self.m[off:off + k].copy_(st['exp_avg'].reshape(-1))
                self.v[off:off + k].copy_(st['exp_avg_sq'].reshape(-1))
            else:
                self.m[off:off + k].zero_()
                self.v[off:off + k].zero_()
                st['step'] = torch.tensor(0.0)
            st['exp_avg'] = self.m[off:off + k].view_as(prm)
            st['exp_avg_sq'] = self.v[off:off + k].view_as(prm)

    def step(self, max_norm: float, grad_scale: float = 1.0):
        grp = self.opt.param_groups[0]
        steps = [self.opt.state[prm]['step'] for prm in self.params]
        for t in steps:
            t += 1  # CPU scalars, as torch.optim.Adam keeps them
        b1, b2 = grp['betas']
        check(self.lib.mas_policy_adam(self.p.numel(), ctypes.c_void_p(self.p.data_ptr()),
                                       ctypes.c_void_p(self.g.data_ptr()), ctypes.c_void_p(self.m.data_ptr()),
                                       ctypes.c_void_p(self.v.data_ptr()), float(grad_scale), float(max_norm),
                                       float(grp['lr']), float(b1), float(b2), float(grp['eps']),
                                       int(steps[0].item()), ctypes.c_void_p(self.scratch.data_ptr()),
                                       ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))


class RolloutBuffer:
    def __init__(self, T, N, A, D, device):
        self.T, self.N, self.A, self.D = T, N, A, D
        f = dict(device=device, dtype=torch.float32)
        self.obs = torch.zeros((T + 1, N, A, D), **f)
        self.actions = torch.zeros((T, N, A, 6), device=device, dtype=torch.int8)
        self.logp = torch.zeros((T, N, A), **f)
        self.values = torch.zeros((T + 1, N, A), **f)
        self.rewards = torch.zeros((T, N, A), **f)
        self.dones = torch.zeros((T, N), device=device, dtype=torch.uint8)
        self.adv = torch.zeros((T, N, A), **f)
        self.ret = torch.zeros((T, N, A), **f)
        # [sum, sum of squares, count] of the advantages: mas_gae writes the
        # sums into the first two (adv_sums is that view), the count is set
        # here (no host copy per iteration)
        self.adv_stats = torch.zeros((3,), device=device, dtype=torch.float64)
        self.adv_stats[2] = float(T * N * A)
        self.adv_sums = self.adv_stats[:2]
        self.gae_scratch = None  # mas_gae's partial sums (made at the first HIP GAE call)
        self.xb = None  # fused path: bf16 policy-input rows [T (+1 with x_obs), N*A, Dx] (mas_policy_act / mas_step_x)


def _allreduce_grads(params, world, group=None):
    """One flat bucket (~0.5 MB for the 2x256 MLP): a single RCCL ring
    all-reduce per minibatch instead of one per parameter tensor."""
    grads = [p.grad for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    flat.div_(world)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


class PPOTrainer:
    """Collect T steps of every env on this rank, GAE on device, PPO update.

    Fused path (GPU, hidden 256, the default there): the rollout step is ONE
    HIP kernel (mas_policy_act: MLP forward + sampling, also storing the bf16
    policy input for the update); each PPO minibatch is one HIP kernel
    (mas_policy_train: forward, loss gradient, backward data path) plus three
    split-K weight-gradient GEMMs.  Minibatches are contiguous time chunks of
    the rollout (T/minibatches steps of every env), visited in a random order
    each epoch: no row gather.  The torch path (random row minibatches,
    autograd) serves the CPU tests and is the numerics reference."""

    def __init__(self, env, cfg: PPOConfig = PPOConfig(), seed: int = 0, group=None):
        self.env, self.cfg = env, cfg
        self.device = env.device
        self.group = group
        self.world = dist.get_world_size(group) if group is not None or dist.is_initialized() else 1
        self.collectives = self.world > 1 if cfg.allreduce is None else bool(cfg.allreduce)
        if self.collectives and not (group is not None or dist.is_initialized()):
            raise ValueError('PPOConfig.allreduce=True needs an initialised torch.distributed process group')
        torch.manual_seed(seed)  # identical init on every rank
        self.policy = PolicyMLP(env.obs_dim, cfg.hidden).to(self.device)
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=cfg.lr, eps=1e-5)
        self.buf = RolloutBuffer(cfg.horizon, env.n_envs, env.n_agents, env.obs_dim, self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 7919 + (dist.get_rank() if dist.is_initialized() else 0))
        self.buf.obs[0].copy_(env.reset())
        self.last_stats = {}
        self.gae_impl = gae  # the HIP kernel; CPU tests inject gae_reference_into
        self.seed = int(seed) * 1000003 + (dist.get_rank() if dist.is_initialized() else 0)
        self.steps_taken = 0
        self._rollout_policy = None
        fused = cfg.fused
        if fused is None:
            fused = self.device.type == 'cuda' and cfg.hidden == 256
        self.fused = None
        self.fused_opt = None
        self.x_obs = False
        if fused:
            self.fused = FusedPolicy(self.policy, env.obs_dim, self.device)
            b = self.buf
            xo = cfg.x_obs
            if xo is None:
                # MAS_X_OBS=0 in the environment: the fp32 obs path (A/B runs)
                xo = (os.environ.get('MAS_X_OBS', '1') != '0' and hasattr(env, 'supports_step_x')
                      and env.supports_step_x())
            self.x_obs = bool(xo)
            # x_obs: rows T + 1 (the env writes step t's next rows into t + 1)
            self.buf.xb = self.fused.x_buffer(b.T + (1 if self.x_obs else 0), b.N * b.A)
            if self.x_obs:
                self._set_x0(self.buf.obs[0])
            M = b.N * b.A
            self._boot = (torch.empty((M, 6), dtype=torch.int8, device=self.device),
                          torch.empty((M,), dtype=torch.float32, device=self.device))
            self.fused.pack()
            if _FUSED_ADAM and FusedAdam.supports(self.opt):
                self.fused_opt = FusedAdam(self.policy.parameters(), self.opt, self.fused.lib, self.device)
        else:
            self._sync_rollout_policy()

    @torch.no_grad()
    def _set_x0(self, obs):
        """x_obs: the first rollout rows from fp32 obs [N, A, D] (a reset's,
        or a checkpoint's): rounded to bf16 as the kernels round."""
        b = self.buf
        b.xb[0][:, :b.D].copy_(obs.reshape(-1, b.D).to(torch.bfloat16))

    def _fwd(self, x):
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.cfg.autocast_bf16):
            return self.policy(x)

    @torch.no_grad()
    def _sync_rollout_policy(self):
        """bf16 copy of the policy for the rollout forward (refreshed after each
        update): no per-step weight casts under autocast."""
        if self.cfg.autocast_bf16 and self.device.type == 'cuda':
            if self._rollout_policy is None:
                import copy
                self._rollout_policy = copy.deepcopy(self.policy).to(torch.bfloat16)
            for d, s_ in zip(self._rollout_policy.parameters(), self.policy.parameters()):
                d.copy_(s_)

    @torch.no_grad()
    def rollout_step(self, t):
        b = self.buf
        if self.fused is not None and hasattr(self.env, 'shard_slices'):
            # sharded env (vec_env.ShardedVecMaSurvival): each shard's policy
            # forward + env step on its own stream, so one shard's act
            # overlaps the others' env kernels; rows keep their global RNG key
            A, D = b.A, b.D
            self.env.fork()
            for e, s, lo, hi in self.env.shard_slices():
                with torch.cuda.stream(s):
                    r0, r1 = lo * A, hi * A
                    if self.x_obs:
                        self.fused.act_x(b.xb[t][r0:r1], self.seed, self.steps_taken,
                                         b.actions[t].view(-1, 6)[r0:r1], b.logp[t].view(-1)[r0:r1],
                                         b.values[t].view(-1)[r0:r1], first_row=r0)
                        e.step_x(b.actions[t][lo:hi], b.xb[t + 1][r0:r1], b.rewards[t][lo:hi], b.dones[t][lo:hi])
                        continue
                    self.fused.act(b.obs[t].view(-1, D)[r0:r1], self.seed, self.steps_taken,
                                   b.actions[t].view(-1, 6)[r0:r1], b.logp[t].view(-1)[r0:r1],
                                   b.values[t].view(-1)[r0:r1], xb=b.xb[t][r0:r1], first_row=r0)
                    e.step(b.actions[t][lo:hi], out=(b.obs[t + 1][lo:hi], b.rewards[t][lo:hi], b.dones[t][lo:hi]))
            self.env.join()
            self.steps_taken += 1
            return
        if self.x_obs:
            # the env wrote these rows (bf16) at the last step; it writes the
            # next ones into row block t + 1
            self.fused.act_x(b.xb[t], self.seed, self.steps_taken, b.actions[t].view(-1, 6), b.logp[t].view(-1),
                             b.values[t].view(-1))
            self.steps_taken += 1
            self.env.step_x(b.actions[t], b.xb[t + 1], b.rewards[t], b.dones[t])
            return
        if self.fused is not None:
            self.fused.act(b.obs[t].view(-1, b.D), self.seed, self.steps_taken, b.actions[t].view(-1, 6),
                           b.logp[t].view(-1), b.values[t].view(-1), xb=b.xb[t])
        elif self.device.type == 'cuda':
            if self._rollout_policy is not None:
                h = self._rollout_policy.forward_raw(b.obs[t].to(torch.bfloat16))  # [N, A, 16] fp32
            else:
                h = self.policy.forward_raw(b.obs[t])
            h2 = h.reshape(-1, N_LOGITS + 1)
            sample_actions_hip(h2, self.seed, self.steps_taken, b.actions[t].view(-1, 6), b.logp[t].view(-1))
            b.values[t].copy_(h[..., N_LOGITS])
        else:  # CPU stand-in tests
            logits, v = self._fwd(b.obs[t])
            a, lp = sample_actions(logits, self.gen)
            b.actions[t].copy_(a)
            b.logp[t].copy_(lp)
            b.values[t].copy_(v)
        self.steps_taken += 1
        self.env.step(b.actions[t], out=(b.obs[t + 1], b.rewards[t], b.dones[t]))

    @torch.no_grad()
    def finish_rollout(self):
        b, c = self.buf, self.cfg
        if self.x_obs:
            self.fused.act_x(b.xb[c.horizon], self.seed, 0, self._boot[0], self._boot[1], b.values[c.horizon].view(-1))
        elif self.fused is not None:
            self.fused.act(b.obs[c.horizon].view(-1, b.D), self.seed, 0, self._boot[0], self._boot[1],
                           b.values[c.horizon].view(-1))
        else:
            _, v = self._fwd(b.obs[c.horizon])
            b.values[c.horizon].copy_(v)
        if self.gae_impl is gae and b.gae_scratch is None:
            b.gae_scratch = gae_scratch(b.N * b.A, self.device)
        self.gae_impl(b.rewards, b.values, b.dones, c.gamma, c.lam, b.adv, b.ret, b.adv_sums, self.env.n_agents,
                      scratch=b.gae_scratch)
        stats = b.adv_stats  # (b.adv_sums is its first two entries)
        if self.collectives:
            stats[2].fill_(float(b.adv.numel()))  # the all-reduce below sums the counts in place
            dist.all_reduce(stats, group=self.group)
        if self.gae_impl is gae and b.adv.is_cuda:
            # one launch (include/masurvival.h mas_adv_normalize), the roundings of the expression below
            adv_normalize(b.adv, stats)
        else:
            mean = stats[0] / stats[2]
            var = (stats[1] / stats[2] - mean * mean).clamp_min(0.0)
            b.adv.sub_(mean.float()).div_(var.sqrt().float() + 1e-8)

    def _update_fused(self):
        b, c = self.buf, self.cfg
        assert c.horizon % c.minibatches == 0, 'fused update: horizon must split into whole time chunks'
        tc = c.horizon // c.minibatches
        params = list(self.policy.parameters())
        for ep in range(c.epochs):
            order = torch.randperm(c.minibatches, generator=torch.Generator().manual_seed(self.steps_taken))
            for n, k in enumerate(order.tolist()):
                sl = slice(k * tc, (k + 1) * tc)
                xb = b.xb[sl].reshape(-1, self.fused.Dx)
                M = xb.shape[0]
                # last_stats keeps the last minibatch's loss terms: only it reduces them
                last = ep == c.epochs - 1 and n == c.minibatches - 1
                st = self.fused.grads(xb, b.actions[sl].reshape(M, 6), b.logp[sl].reshape(M),
                                      b.adv[sl].reshape(M), b.ret[sl].reshape(M), c, stats=last)
                if last:
                    loss, pg, vl, ent, cf = st
                if self.fused_opt is not None:
                    # flat gradient buffer: one all-reduce, the 1 / world folded into the step
                    if self.collectives:
                        dist.all_reduce(self.fused_opt.g, group=self.group)
                    self.fused_opt.step(c.max_grad_norm, 1.0 / self.world if self.collectives else 1.0)
                else:
                    if self.collectives:
                        _allreduce_grads(params, self.world, self.group)
                    nn.utils.clip_grad_norm_(params, c.max_grad_norm)
                    self.opt.step()
                self.fused.pack()
        self.last_stats = {'loss': loss.detach(), 'pg': pg.detach(), 'v': vl.detach(), 'entropy': ent.detach(),
                           'clipfrac': cf.detach()}
        if self.x_obs:
            b.xb[0].copy_(b.xb[c.horizon])
        else:
            b.obs[0].copy_(b.obs[c.horizon])

    def update(self):
        if self.fused is not None:
            return self._update_fused()
        b, c = self.buf, self.cfg
        M = c.horizon * b.N * b.A
        obs = b.obs[:c.horizon].reshape(M, b.D)
        acts = b.actions.reshape(M, 6)
        old_lp, adv, ret = b.logp.reshape(M), b.adv.reshape(M), b.ret.reshape(M)
        params = list(self.policy.parameters())
        mb = M // c.minibatches
        for _ in range(c.epochs):
            perm = torch.randperm(M, device=self.device, generator=self.gen)
            for k in range(c.minibatches):
                idx = perm[k * mb:(k + 1) * mb]
                logits, v = self._fwd(obs[idx])
                lp, ent = evaluate_actions(logits, acts[idx])
                ratio = torch.exp(lp - old_lp[idx])
                a = adv[idx]
                pg = -torch.min(ratio * a, ratio.clamp(1 - c.clip, 1 + c.clip) * a).mean()
                vl = F.mse_loss(v, ret[idx])
                loss = pg + c.vf_coef * vl - c.ent_coef * ent.mean()
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.collectives:
                    _allreduce_grads(params, self.world, self.group)
                nn.utils.clip_grad_norm_(params, c.max_grad_norm)
                self.opt.step()
        self.last_stats = {'loss': loss.detach(), 'pg': pg.detach(), 'v': vl.detach()}
        self._sync_rollout_policy()
        b.obs[0].copy_(b.obs[c.horizon])

    # -- checkpoint / resume ------------------------------------------------
    # The reference has no trainer (SURVEY.md §5 lists checkpointing as an
    # auxiliary); this keeps what a resumed run needs to continue the same
    # trajectory: fp32 master weights, Adam moments, the sampling counters and
    # generator, the next rollout's first observation and, when the env exposes
    # mas_get_state (VecMaSurvival), the whole batched env state.  Only tensors
    # and plain numbers, so torch.load(weights_only=True) reads it back.

    def state_dict(self):
        sd = {'policy': self.policy.state_dict(), 'opt': self.opt.state_dict(),
              'steps_taken': int(self.steps_taken), 'seed': int(self.seed),
              'gen': self.gen.get_state(), 'obs0': self.buf.obs[0].detach().clone()}
        if self.x_obs:
            sd['xb0'] = self.buf.xb[0].detach().clone()  # (x_obs: the next rollout's rows; obs0 is the reset's)
        if hasattr(self.env, 'get_state'):
            sd['env'] = self.env.get_state().detach().clone()
            if hasattr(self.env, 'state_meta'):
                sd['env_meta'] = self.env.state_meta()
        elif hasattr(self.env, 'n_envs') and self.env.__class__.__module__.startswith('masurvival'):
            raise ValueError(f'{type(self.env).__name__} cannot export its env state (no get_state): '
                             'a checkpoint without it would not resume the same trajectory')
        return sd

    @torch.no_grad()
    def load_state_dict(self, sd):
        self.policy.load_state_dict(sd['policy'])
        self.opt.load_state_dict(sd['opt'])
        if self.fused_opt is not None:
            self.fused_opt.bind_state()
        self.steps_taken = int(sd['steps_taken'])
        self.seed = int(sd['seed'])
        self.gen.set_state(sd['gen'].cpu())  # generator states are CPU ByteTensors (map_location moves them)
        if 'env' in sd:
            if not hasattr(self.env, 'set_state'):
                raise ValueError('checkpoint holds an env state but this env has no set_state')
            want = sd.get('env_meta')
            have = self.env.state_meta() if hasattr(self.env, 'state_meta') else None
            if want is not None and have is not None:
                # a state image only means something for the same config,
                # capacity class, env count and shard split
                diff = {k: (want.get(k), have.get(k)) for k in have if want.get(k) != have.get(k)}
                if diff:
                    raise ValueError(f'checkpoint env state does not match this env: {diff}')
            self.env.set_state(sd['env'].to(self.device))
        self.buf.obs[0].copy_(sd['obs0'])
        if self.x_obs:
            if 'xb0' in sd:
                self.buf.xb[0].copy_(sd['xb0'])
            else:
                self._set_x0(self.buf.obs[0])
        if self.fused is not None:
            self.fused.pack()
        else:
            self._sync_rollout_policy()

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))

    def iteration(self):
        with _phase('mas.rollout'):
            for t in range(self.cfg.horizon):
                self.rollout_step(t)
        with _phase('mas.gae'):
            self.finish_rollout()
        with _phase('mas.update'):
            self.update()
