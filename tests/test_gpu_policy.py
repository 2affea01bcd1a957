"""Fused HIP policy kernels (include/masurvival.h mas_policy_*) against a
plain torch fp32 restatement of the same MLP and PPO loss.

The kernels compute in bf16 MFMA with fp32 accumulation: the reference uses
the same bf16-rounded weights and inputs in fp32 arithmetic, so the
remaining differences are the bf16 rounding of the two hidden activations
and the accumulation order.  Tolerances (written per assertion below):
value/log-prob |d| <= 0.03 + 0.03 |ref|; gradients: cosine >= 0.999 and
relative norm error <= 3 % per parameter tensor; the bf16 input copy is
exact."""
import copy
import ctypes

import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival import ppo as ppo_mod  # noqa: E402
from masurvival.ppo import (FusedPolicy, PolicyMLP, PPOConfig, evaluate_actions,  # noqa: E402
                            policy_loss_reference, sample_actions_hip)


def _policy(D, seed=0, scale=1.0):
    torch.manual_seed(seed)
    p = PolicyMLP(D, 256).cuda()
    with torch.no_grad():
        for prm in p.parameters():
            prm.mul_(scale)
    return p


def _bf16_ref(p):
    r = copy.deepcopy(p)
    with torch.no_grad():
        for prm in r.parameters():
            prm.copy_(prm.bfloat16().float())
    return r


@pytest.mark.parametrize('D,M', [(160, 4096), (138, 1000 + 13), (468, 777), (160, 32)])
def test_policy_act_matches_reference(D, M):
    p = _policy(D, seed=D)
    fp = FusedPolicy(p, D, torch.device('cuda'))
    fp.pack()
    g = torch.Generator(device='cuda').manual_seed(M)
    obs = torch.randn((M, D), device='cuda', generator=g) * 3.0
    acts = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), device='cuda')
    v = torch.empty((M,), device='cuda')
    xb = torch.full((M, fp.Dx), 7.0, dtype=torch.bfloat16, device='cuda')
    fp.act(obs, 11, 5, acts, lp, v, xb=xb)
    # the bf16 copy of the rows is exact; written columns [0, Dp): the row,
    # then the bias column (1.0 at index D) when it falls inside, then zeros
    assert torch.equal(xb[:, :D], obs.bfloat16())
    if D < fp.Dp:
        assert bool((xb[:, D] == 1).all()) and bool((xb[:, D + 1:fp.Dp] == 0).all())
    assert bool((xb[:, fp.Dp:] == 7).all())
    ref = _bf16_ref(p)
    with torch.no_grad():
        raw = ref.forward_raw(xb[:, :D].float())
    # value and log-prob of the drawn actions: |d| <= 0.03 + 0.03 |ref|
    torch.testing.assert_close(v, raw[:, 15], atol=0.03, rtol=0.03)
    ref_lp, _ = evaluate_actions(raw[:, :15], acts)
    torch.testing.assert_close(lp, ref_lp, atol=0.03, rtol=0.03)
    # the same RNG stream as mas_sample_actions: on the reference logits the
    # draws agree except where two Gumbel scores are within the logit error
    a2 = torch.empty_like(acts)
    lp2 = torch.empty_like(lp)
    sample_actions_hip(raw.contiguous(), 11, 5, a2, lp2)
    agree = (a2 == acts).all(1).float().mean().item()
    assert agree > 0.97, agree


@pytest.mark.parametrize('D,M,first_row', [(160, 262144, 0), (138, 1000 + 13, 77), (160, 32 * 3 + 5, 1 << 20)])
def test_policy_act_split_sampler_is_bit_identical(D, M, first_row, monkeypatch):
    """The heads sampled on both half-waves (default) against the one-half
    loop (MAS_ACT_SPLIT=0): the same actions, log-probs and values, bit for
    bit, for the fp32-row and the bf16-row (act_x) forms and a shard offset."""
    p = _policy(D, seed=D + 1)
    fp = FusedPolicy(p, D, torch.device('cuda'))
    fp.pack()
    g = torch.Generator(device='cuda').manual_seed(M)
    obs = torch.randn((M, D), device='cuda', generator=g) * 3.0
    xb = fp.x_buffer(M)
    out = {}
    for split in ('1', '0'):
        monkeypatch.setenv('MAS_ACT_SPLIT', split)
        a = torch.empty((M, 6), dtype=torch.int8, device='cuda')
        lp = torch.empty((M,), device='cuda')
        v = torch.empty((M,), device='cuda')
        fp.act(obs, 5, 123, a, lp, v, xb=xb, first_row=first_row)
        ax = torch.empty_like(a)
        lpx = torch.empty_like(lp)
        vx = torch.empty_like(v)
        fp.act_x(xb, 5, 124, ax, lpx, vx, first_row=first_row)
        torch.cuda.synchronize()
        out[split] = (a, lp, v, ax, lpx, vx)
    for x, y in zip(out['1'], out['0']):
        assert torch.equal(x.view(torch.uint8) if x.dtype == torch.int8 else x.view(torch.int32),
                           y.view(torch.uint8) if y.dtype == torch.int8 else y.view(torch.int32))


def test_policy_act_action_distribution():
    D, M = 160, 100000
    p = _policy(D, seed=1, scale=0.0)  # zero weights: the heads' logits are the biases
    with torch.no_grad():
        p.head.bias.copy_(torch.linspace(-1.0, 1.0, 16))
    fp = FusedPolicy(p, D, torch.device('cuda'))
    fp.pack()
    obs = torch.randn((M, D), device='cuda')
    acts = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), device='cuda')
    v = torch.empty((M,), device='cuda')
    fp.act(obs, 3, 9, acts, lp, v)
    b = p.head.bias.detach().bfloat16().float()
    torch.testing.assert_close(v, b[15].expand(M), atol=0, rtol=0)
    off = 0
    for h, n in enumerate((3, 3, 3, 2, 2, 2)):
        pr = torch.softmax(b[off:off + n], dim=0)
        freq = torch.bincount(acts[:, h].long(), minlength=n).float() / M
        assert int(acts[:, h].min()) >= 0 and int(acts[:, h].max()) < n
        assert torch.allclose(freq, pr, atol=0.01), (h, freq, pr)
        off += n


def _cos(a, b):
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-30))


@pytest.mark.parametrize('D,M,off64,layout', [(160, 8192, False, 'fm'), (138, 2000 + 7, False, 'fm'),
                                              (160, 8192, True, 'fm'), (160, 8192, False, 'rm'),
                                              (138, 2000 + 7, False, 'rm')])
def test_policy_train_gradients_match_reference(D, M, off64, layout, monkeypatch):
    # off64: the 64-bit store-offset instantiation of k_policy_train, which only
    # activation buffers over 4 GB select (mas_policy.hip, MAS_POL_FORCE_OFF64);
    # layout 'rm': row-major activations (mas_policy_train_rm) and the row-sum
    # GEMMs with the stored-column permutation undone on the host
    if off64:
        monkeypatch.setenv('MAS_POL_FORCE_OFF64', '1')
    monkeypatch.setattr(ppo_mod, '_POL_LAYOUT', layout)
    p = _policy(D, seed=D + 1)
    cfg = PPOConfig()
    fp = FusedPolicy(p, D, torch.device('cuda'))
    fp.pack()
    g = torch.Generator(device='cuda').manual_seed(7)
    obs = torch.randn((M, D), device='cuda', generator=g) * 2.0
    xb = fp.x_buffer(M)
    acts = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), device='cuda')
    v = torch.empty((M,), device='cuda')
    fp.act(obs, 1, 2, acts, lp, v, xb=xb)
    # a policy that has moved since the rollout: some ratios leave the clip range
    old_lp = lp + 0.3 * torch.randn((M,), device='cuda', generator=g)
    adv = torch.randn((M,), device='cuda', generator=g)
    ret = v + torch.randn((M,), device='cuda', generator=g)
    loss, pg, vl, ent, cf = fp.grads(xb, acts, old_lp, adv, ret, cfg)
    ref = _bf16_ref(p)
    rl, rpg, rvl, rent = policy_loss_reference(ref, xb[:, :D].float(), acts, old_lp, adv, ret, cfg)
    ref.zero_grad()
    rl.backward()
    # loss terms: |d| <= 0.02 + 0.02 |ref|
    for a, b in ((loss, rl), (pg, rpg), (vl, rvl), (ent, rent)):
        assert abs(float(a) - float(b)) <= 0.02 + 0.02 * abs(float(b)), (float(a), float(b))
    assert 0.0 < float(cf) < 1.0
    for (name, a), b in zip(p.named_parameters(), ref.parameters()):
        ga, gb = a.grad.float(), b.grad
        assert _cos(ga, gb) >= 0.999, (name, _cos(ga, gb))
        assert float((ga.norm() - gb.norm()).abs() / gb.norm()) <= 0.03, name


@pytest.mark.parametrize('F,K', [(256, 65536 + 64 * 37), (256, 65536 + 32 * 37), (16, 65536 + 64 * 5), (16, 32 * 1001),
                                 (256, 64)])
def test_policy_dw_matches_fp32(F, K):
    """mas_policy_dw (split-K MFMA weight + bias gradients) against torch fp32
    on the same bf16 operands, row strides wider than K as in the trainer's
    [257][M] activation buffers (F = 256 with K % 64 == 0: the LDS-staged
    kernel; otherwise the direct one)."""
    from masurvival.abi import check, load_library
    lib = load_library()
    g = torch.Generator(device='cuda').manual_seed(F + K)
    a = torch.randn((F, K + 64), device='cuda', generator=g).to(torch.bfloat16)
    h = torch.randn((257, K + 64), device='cuda', generator=g).to(torch.bfloat16)
    n = int(lib.mas_policy_dw_scratch(F, 256, K))
    assert n > 0
    scratch = torch.empty((n,), device='cuda')
    out = torch.empty((F * 256 + F,), device='cuda')
    check(lib.mas_policy_dw(F, 256, K, ctypes.c_void_p(a.data_ptr()), a.stride(0), ctypes.c_void_p(h.data_ptr()),
                            h.stride(0), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(scratch.data_ptr()), None))
    torch.cuda.synchronize()
    af, hf = a[:, :K].float(), h[:256, :K].float()
    ref_w, ref_b = af @ hf.T, af.sum(1)
    # fp32 sums of K bf16 products in another order: |d| <= 1e-5 * sum |a||h|
    bound_w = 1e-5 * (af.abs() @ hf.abs().T) + 1e-6
    bound_b = 1e-5 * af.abs().sum(1) + 1e-6
    assert bool(((out[:F * 256].view(F, 256) - ref_w).abs() <= bound_w).all())
    assert bool(((out[F * 256:] - ref_b).abs() <= bound_b).all())
    # bad shapes are refused
    assert lib.mas_policy_dw(F, 256, K + 16, ctypes.c_void_p(a.data_ptr()), a.stride(0), ctypes.c_void_p(h.data_ptr()),
                             h.stride(0), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
                             None) != 0


def test_fused_trainer_iteration_on_env():
    from masurvival.config import C3_CONFIG
    from masurvival.ppo import PPOTrainer
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(C3_CONFIG, n_envs=1024, auto_reset=True)
    # (fp32 obs rows: the last check compares them with the update's bf16 rows)
    tr = PPOTrainer(env, PPOConfig(horizon=16, x_obs=False), seed=0)
    assert tr.fused is not None
    before = [q.detach().clone() for q in tr.policy.parameters()]
    for _ in range(2):
        tr.iteration()
    for k in ('loss', 'pg', 'v', 'entropy', 'clipfrac'):
        assert torch.isfinite(tr.last_stats[k]), k
    assert all(not torch.equal(a, b) for a, b in zip(before, tr.policy.parameters()))
    b = tr.buf
    assert bool(torch.isfinite(b.adv).all()) and bool(torch.isfinite(b.values).all())
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device='cuda', dtype=torch.int8)
    assert bool(((b.actions >= 0) & (b.actions < hi)).all())
    # the stored update input is the bf16 image of the observations the policy saw
    assert torch.equal(b.xb[3].view(b.N, b.A, -1)[..., :b.D], b.obs[3].bfloat16())
    env.close()


@pytest.mark.parametrize('max_norm,grad_scale', [(0.5, 1.0), (1e9, 0.5)])
def test_fused_adam_matches_torch(max_norm, grad_scale):
    """mas_policy_adam (FusedAdam) against clip_grad_norm_ + torch.optim.Adam
    over five steps of random gradients: one clipped regime, one unclipped
    with the all-reduce 1 / world scale.  fp32 in both; the bound covers the
    different summation order of the norm: |d| <= 1e-6 + 1e-5 |p|."""
    from masurvival.ppo import FusedAdam
    p_ref = _policy(160, seed=3)
    p_fus = _policy(160, seed=3)
    opt_ref = torch.optim.Adam(p_ref.parameters(), lr=3e-4, eps=1e-5)
    opt_fus = torch.optim.Adam(p_fus.parameters(), lr=3e-4, eps=1e-5)
    fa = FusedAdam(p_fus.parameters(), opt_fus, FusedPolicy(p_fus, 160, torch.device('cuda')).lib, torch.device('cuda'))
    g = torch.Generator(device='cuda').manual_seed(11)
    for _ in range(5):
        grads = [torch.randn(q.shape, device='cuda', generator=g) * 0.3 for q in p_ref.parameters()]
        for q, gr in zip(p_ref.parameters(), grads):
            q.grad = gr * grad_scale
        torch.nn.utils.clip_grad_norm_(list(p_ref.parameters()), max_norm)
        opt_ref.step()
        for q, gr in zip(p_fus.parameters(), grads):
            q.grad.copy_(gr)
        fa.step(max_norm, grad_scale)
    torch.cuda.synchronize()
    for (name, a), b in zip(p_fus.named_parameters(), p_ref.parameters()):
        assert bool(((a - b).abs() <= 1e-6 + 1e-5 * b.abs()).all()), name
        st_a, st_b = opt_fus.state[a], opt_ref.state[b]
        assert float(st_a['step']) == float(st_b['step']) == 5.0
        assert torch.allclose(st_a['exp_avg'], st_b['exp_avg'], rtol=1e-5, atol=1e-7), name
        assert torch.allclose(st_a['exp_avg_sq'], st_b['exp_avg_sq'], rtol=1e-5, atol=1e-9), name
    # the optimizer's state_dict round-trips into a fresh FusedAdam
    sd = opt_fus.state_dict()
    p2 = _policy(160, seed=4)
    opt2 = torch.optim.Adam(p2.parameters(), lr=3e-4, eps=1e-5)
    fa2 = FusedAdam(p2.parameters(), opt2, fa.lib, torch.device('cuda'))
    opt2.load_state_dict(sd)
    fa2.bind_state()
    assert torch.equal(fa2.m, fa.m) and torch.equal(fa2.v, fa.v)


@pytest.mark.parametrize('D,M', [(160, 8192 + 70), (138, 256 * 300 + 130), (468, 4096 + 2), (160, 128)])
def test_counted_wait_train_kernel_is_bit_identical(D, M, monkeypatch):
    """k_policy_train_db (the PPO update's default for 32-bit store offsets
    and obs_dim in (128, 160]: persistent 8-wave workgroups, double-buffered
    weight stages, full 256-row blocks; the partial last block on
    k_policy_train) and k_policy_train_cw (the other obs_dims) only reorder
    k_policy_train's loads, copies and activation stores: the gradients of a
    minibatch are bit-identical with MAS_POL_DB=0 MAS_POL_CW=0, the loss terms
    equal up to the order of the per-block partial sums -- full blocks plus a
    partial last block (M = 8262 and 76930: 32 / 300 full blocks + 70 / 130
    rows, D = 160 and 138: 10 and 9 layer-1 k-steps), the generic layer-1
    k-loop (D = 468) and a single block (M = 128)."""
    monkeypatch.setattr(ppo_mod, '_POL_LAYOUT', 'fm')
    cfg = PPOConfig()
    out = []
    for cw in ('1', '0'):
        monkeypatch.setenv('MAS_POL_CW', cw)
        monkeypatch.setenv('MAS_POL_DB', cw)
        p = _policy(D, seed=D + 3)
        fp = FusedPolicy(p, D, torch.device('cuda'))
        fp.pack()
        g = torch.Generator(device='cuda').manual_seed(11)
        obs = torch.randn((M, D), device='cuda', generator=g) * 2.0
        xb = fp.x_buffer(M)
        acts = torch.empty((M, 6), dtype=torch.int8, device='cuda')
        lp = torch.empty((M,), device='cuda')
        v = torch.empty((M,), device='cuda')
        fp.act(obs, 1, 2, acts, lp, v, xb=xb)
        old_lp = lp + 0.3 * torch.randn((M,), device='cuda', generator=g)
        adv = torch.randn((M,), device='cuda', generator=g)
        ret = v + torch.randn((M,), device='cuda', generator=g)
        terms = [float(t) for t in fp.grads(xb, acts, old_lp, adv, ret, cfg)]
        out.append((terms, [q.grad.detach().clone() for q in p.parameters()]))
    (t1, g1), (t0, g0) = out
    for a, b in zip(t1, t0):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(b)), (t1, t0)
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)
