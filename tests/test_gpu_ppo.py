"""HIP GAE kernel vs the plain torch fp32 restatement, and one PPO iteration
on the real env (GPU).  Tolerance: |adv - ref| <= 1e-5 + 1e-5*|ref| -- the
kernel folds gamma*lambda in fp32 while the reference multiplies by the
Python double product, so the last ulps may differ."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival.config import C3_CONFIG  # noqa: E402
from masurvival.ppo import PPOConfig, PPOTrainer, adv_normalize, gae, gae_reference  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


@pytest.mark.parametrize('scan', ['0', '1'])
@pytest.mark.parametrize('T,N,A', [(64, 1000, 4), (13, 37, 2), (1, 5, 3), (64, 65536, 4), (150, 300, 4)])
def test_gae_kernel_matches_reference(T, N, A, scan, monkeypatch):
    """Both forms of mas_gae: the per-column walk (default) and the
    wavefront scan over time (MAS_GAE_SCAN=1; T = 150 spans three 64-step
    chunks, so the carries between chunks are covered)."""
    monkeypatch.setenv('MAS_GAE_SCAN', scan)
    g = torch.Generator(device='cuda').manual_seed(T * 1000 + N)
    r = torch.randn((T, N, A), device='cuda', generator=g)
    v = torch.randn((T + 1, N, A), device='cuda', generator=g)
    d = (torch.rand((T, N), device='cuda', generator=g) < 0.05).to(torch.uint8)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    sums = torch.empty(2, device='cuda', dtype=torch.float64)
    gae(r, v, d, 0.99, 0.95, adv, ret, sums, A)
    ra, rr = gae_reference(r, v, d, 0.99, 0.95, A)
    torch.testing.assert_close(adv, ra, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ret, rr, atol=1e-5, rtol=1e-5)
    assert np.isclose(float(sums[0]), float(adv.double().sum()), rtol=1e-9, atol=1e-6)
    assert np.isclose(float(sums[1]), float((adv.double() ** 2).sum()), rtol=1e-9)


@pytest.mark.parametrize('n,shift', [(65536 * 4 * 20, 0.0), (1001, 3.0), (3, -2.0), (4096, 1e4)])
def test_adv_normalize_matches_torch_bit_exactly(n, shift):
    """mas_adv_normalize against the torch expression it replaces, on the
    same fp64 statistics: identical bits (n not a multiple of 4 covers the
    tail lanes; shift 1e4 makes sum_sq / n - mean^2 cancel)."""
    g = torch.Generator(device='cuda').manual_seed(n)
    adv = torch.randn((n,), device='cuda', generator=g) * 3.0 + shift
    stats = torch.stack([adv.double().sum(), (adv.double() ** 2).sum(),
                         torch.tensor(float(n), device='cuda', dtype=torch.float64)])
    mean = stats[0] / stats[2]
    var = (stats[1] / stats[2] - mean * mean).clamp_min(0.0)
    ref = adv.clone().sub_(mean.float()).div_(var.sqrt().float() + 1e-8)
    out = adv.clone()
    adv_normalize(out, stats)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))


def test_adv_normalize_zero_variance_clamps():
    """Negative rounding of the variance clamps to 0: (adv - mean) / 1e-8."""
    adv = torch.full((8,), 2.0, device='cuda')
    stats = torch.tensor([16.0, 32.0 - 1e-9, 8.0], device='cuda', dtype=torch.float64)
    adv_normalize(adv, stats)
    torch.cuda.synchronize()
    assert torch.equal(adv, torch.zeros_like(adv))


@pytest.mark.parametrize('scan', ['0', '1'])
def test_gae_concurrent_calls_on_two_streams(scan, monkeypatch):
    """Two mas_gae calls in flight at once on two streams, each with its own
    scratch and outputs, both checked against the torch restatement; the
    sums are also bit-stable from call to call (fixed summation order)."""
    monkeypatch.setenv('MAS_GAE_SCAN', scan)
    from masurvival.ppo import gae_scratch
    T, N, A = 64, 65536, 4
    cases = []
    for k in range(2):
        g = torch.Generator(device='cuda').manual_seed(77 + k)
        r = torch.randn((T, N, A), device='cuda', generator=g)
        v = torch.randn((T + 1, N, A), device='cuda', generator=g)
        d = (torch.rand((T, N), device='cuda', generator=g) < 0.05).to(torch.uint8)
        cases.append(dict(r=r, v=v, d=d, adv=torch.empty_like(r), ret=torch.empty_like(r),
                          sums=torch.empty(2, device='cuda', dtype=torch.float64),
                          scratch=gae_scratch(N * A, 'cuda'), stream=torch.cuda.Stream()))
    torch.cuda.synchronize()
    for rep in range(3):
        for c in cases:  # interleaved launches: both streams' kernels overlap
            gae(c['r'], c['v'], c['d'], 0.99, 0.95, c['adv'], c['ret'], c['sums'], A,
                stream=c['stream'].cuda_stream, scratch=c['scratch'])
        torch.cuda.synchronize()
        for c in cases:
            ra, rr = gae_reference(c['r'], c['v'], c['d'], 0.99, 0.95, A)
            torch.testing.assert_close(c['adv'], ra, atol=1e-5, rtol=1e-5)
            torch.testing.assert_close(c['ret'], rr, atol=1e-5, rtol=1e-5)
            assert np.isclose(float(c['sums'][0]), float(c['adv'].double().sum()), rtol=1e-9, atol=1e-6)
            assert np.isclose(float(c['sums'][1]), float((c['adv'].double() ** 2).sum()), rtol=1e-9)
            if rep == 0:
                c['first'] = c['sums'].clone()
            else:
                assert torch.equal(c['sums'], c['first'])


def test_ppo_iteration_on_env():
    env = VecMaSurvival(C3_CONFIG, n_envs=512, auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(horizon=16), seed=0)
    for _ in range(2):
        tr.iteration()
    assert torch.isfinite(tr.last_stats['loss'])
    assert bool(torch.isfinite(tr.buf.adv).all()) and bool(torch.isfinite(tr.buf.obs).all())


def test_hip_sampler_logp_and_distribution():
    from masurvival.ppo import evaluate_actions, sample_actions_hip
    g = torch.Generator(device='cuda').manual_seed(3)
    M = 200000
    row = torch.randn((1, 16), device='cuda', generator=g) * 1.5
    logits = row.repeat(M, 1).contiguous()
    acts = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), dtype=torch.float32, device='cuda')
    sample_actions_hip(logits, 1234, 7, acts, lp)
    ref_lp, _ = evaluate_actions(logits[:, :15], acts)
    torch.testing.assert_close(lp, ref_lp, atol=1e-5, rtol=1e-5)
    off = 0
    for h, n in enumerate((3, 3, 3, 2, 2, 2)):
        p = torch.softmax(row[0, off:off + n], dim=0)
        freq = torch.bincount(acts[:, h].long(), minlength=n).float() / M
        assert int(acts[:, h].max()) < n and int(acts[:, h].min()) >= 0
        assert torch.allclose(freq, p, atol=0.01), (h, freq, p)
        off += n
    # different step -> different draws, same step -> same draws
    acts2 = torch.empty_like(acts)
    sample_actions_hip(logits, 1234, 8, acts2, lp)
    assert not torch.equal(acts, acts2)
    acts3 = torch.empty_like(acts)
    sample_actions_hip(logits, 1234, 7, acts3, lp)
    assert torch.equal(acts, acts3)


@pytest.mark.parametrize('x_obs', [False, True])
def test_sharded_rollout_matches_one_handle(x_obs):
    """ShardedVecMaSurvival (3 handles on 3 streams, per-shard act with the
    global row key) fills the rollout buffer bit-identically to one handle
    (x_obs: each shard writes its bf16 policy rows, mas_step_x)."""
    from masurvival.vec_env import ShardedVecMaSurvival
    n, T = 4096, 6
    tr = []
    for env in (VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n)),
                ShardedVecMaSurvival(C3_CONFIG, n_envs=n, shards=3, seeds=range(n))):
        t_ = PPOTrainer(env, PPOConfig(horizon=8, x_obs=x_obs), seed=0)
        assert t_.x_obs == x_obs
        for t in range(T):
            t_.rollout_step(t)
        tr.append(t_)
    torch.cuda.synchronize()
    b1, b2 = tr[0].buf, tr[1].buf
    for name in ('obs', 'values'):
        assert torch.equal(getattr(b1, name)[:T + 1], getattr(b2, name)[:T + 1]), name
    for name in ('actions', 'logp', 'rewards', 'dones'):
        assert torch.equal(getattr(b1, name)[:T], getattr(b2, name)[:T]), name
    assert torch.equal(b1.xb[:T + (1 if x_obs else 0)], b2.xb[:T + (1 if x_obs else 0)])
    for t_ in tr:
        t_.env.close()


def _vec(n, seeds, shards):
    if shards == 1:
        return VecMaSurvival(C3_CONFIG, n_envs=n, seeds=seeds, auto_reset=True)
    from masurvival.vec_env import ShardedVecMaSurvival
    return ShardedVecMaSurvival(C3_CONFIG, n_envs=n, shards=shards, seeds=seeds, auto_reset=True)


@pytest.mark.parametrize('shards,x_obs', [(1, False), (2, False), (1, True), (2, True)])
def test_checkpoint_resume_on_env(tmp_path, shards, x_obs):
    """PPOTrainer.save after an iteration, load into a fresh trainer on a fresh
    env: the next rollout (fused act kernel + env kernels) is bit-identical to
    the run that never stopped -- policy, env state and sampling counters all
    restored.  shards=2: the env is a ShardedVecMaSurvival, whose state image
    is its shards' images concatenated."""
    n, T = 1024, 8
    trs = []
    env = _vec(n, list(range(n)), shards)
    tr = PPOTrainer(env, PPOConfig(horizon=T, x_obs=x_obs), seed=0)
    tr.iteration()
    path = str(tmp_path / 'ckpt.pt')
    tr.save(path)
    env2 = _vec(n, list(range(1000, 1000 + n)), shards)
    tr2 = PPOTrainer(env2, PPOConfig(horizon=T, x_obs=x_obs), seed=5)
    tr2.load(path)
    for t_ in (tr, tr2):
        for t in range(T):
            t_.rollout_step(t)
        trs.append(t_)
    torch.cuda.synchronize()
    b1, b2 = trs[0].buf, trs[1].buf
    # values[T] is the previous rollout's bootstrap value (finish_rollout),
    # which only the uninterrupted trainer has computed
    assert torch.equal(b1.obs, b2.obs) and torch.equal(b1.values[:T], b2.values[:T])
    assert torch.equal(b1.xb, b2.xb)
    for name in ('actions', 'logp', 'rewards', 'dones'):
        assert torch.equal(getattr(b1, name), getattr(b2, name)), name
    env.close()
    env2.close()


def test_x_obs_trainer_matches_fp32_obs_trainer():
    """PPOConfig.x_obs: the env writes the policy's bf16 input rows
    (mas_step_x) and the act kernel reads them (mas_policy_act_x), instead of
    fp32 obs rows that mas_policy_act rounds to bf16 itself.  Two trainers from
    the same seeds, two PPO iterations each with auto-reset: every rollout
    array, the update's input rows and the trained parameters are
    bit-identical."""
    n, T = 2048, 8
    trs = []
    for xo in (False, True):
        env = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n), auto_reset=True)
        tr = PPOTrainer(env, PPOConfig(horizon=T, x_obs=xo), seed=0)
        assert tr.x_obs == xo
        for _ in range(2):
            tr.iteration()
        trs.append(tr)
    torch.cuda.synchronize()
    b1, b2 = trs[0].buf, trs[1].buf
    for name in ('actions', 'logp', 'values', 'rewards', 'dones', 'adv', 'ret'):
        assert torch.equal(getattr(b1, name), getattr(b2, name)), name
    # the update's input rows (row block 0 of the x path already holds the next rollout's)
    assert torch.equal(b1.xb[1:T], b2.xb[1:T])
    # the fp32 path's last rows, rounded, are the x path's next rollout's first rows
    assert torch.equal(b2.xb[0].view(n, -1, b2.xb.shape[-1])[..., :b2.D], b1.obs[0].bfloat16())
    for p1, p2 in zip(trs[0].policy.parameters(), trs[1].policy.parameters()):
        assert torch.equal(p1, p2)
    for tr in trs:
        tr.env.close()


def test_checkpoint_env_mismatch_is_refused(tmp_path):
    """A checkpoint's env state only loads into an env with the same config,
    env count and shard split (same image size is not enough)."""
    n, T = 256, 4
    env = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n))
    tr = PPOTrainer(env, PPOConfig(horizon=T), seed=0)
    tr.iteration()
    path = str(tmp_path / 'ckpt.pt')
    tr.save(path)
    sb = env.state_bytes()
    env.close()
    # same capacity class (2v2) and N, hence the same image size, other config
    other = dict(C3_CONFIG, melee={'range': 3, 'damage': 20, 'cooldown': 40, 'drift': True})
    env2 = VecMaSurvival(other, n_envs=n, seeds=range(n))
    assert env2.state_bytes() == sb
    tr2 = PPOTrainer(env2, PPOConfig(horizon=T), seed=0)
    with pytest.raises(ValueError, match='does not match'):
        tr2.load(path)
    env2.close()
    env3 = _vec(n, list(range(n)), 2)
    tr3 = PPOTrainer(env3, PPOConfig(horizon=T), seed=0)
    with pytest.raises(ValueError, match='does not match'):
        tr3.load(path)
    env3.close()
