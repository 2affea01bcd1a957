"""HIP path == C oracle, bit for bit, on the same seeds and actions.

Parity bar: every observation float, reward and done flag identical
(np.array_equal) -- the kernels restate the oracle's float op order with
-ffp-contract=off, so the fp32 tolerance is 0.  Cases: every golden episode
replayed through VecMaSurvival (n_envs=1), and batched seeded episodes with
auto-reset compared env-by-env against oracle instances."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import golden_replay as gr  # noqa: E402
from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import C3_CONFIG, C5_CONFIG, ResolvedConfig, pcg64_state  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402
from oracle import OracleEnv  # noqa: E402


def make_vec(cfg, n, seeds, auto_reset):
    try:
        return VecMaSurvival(cfg, n_envs=n, seeds=seeds, auto_reset=auto_reset)
    except abi.MasError as e:
        class_missing(e)


@pytest.mark.parametrize('name', gr.golden_files())
def test_golden_episode_on_gpu(name):
    d, cfg = gr.load(name)
    env = make_vec(cfg, 1, [int(d['env_seed'])], False)
    obs = env.reset().cpu().numpy()[0]
    assert np.array_equal(obs, d['obs'][0]), gr.diff(obs, d['obs'][0])
    acts = torch.as_tensor(d['actions'], device=env.device)
    for t in range(len(d['done'])):
        o, r, dn, _ = env.step(acts[t:t + 1])
        o = o.cpu().numpy()[0]
        assert np.array_equal(o, d['obs'][t + 1]), (t, gr.diff(o, d['obs'][t + 1]))
        assert np.array_equal(r.cpu().numpy()[0], d['rewards'][t]), t
        assert bool(dn.cpu().numpy()[0]) == bool(d['done'][t]), t
    stats = env.flush_stats().cpu().numpy()[0]
    bad, ora_stats = gr.replay(name)
    assert bad is None
    assert np.array_equal(stats, ora_stats), (stats, ora_stats)


@pytest.mark.parametrize('cfg,n,T', [(None, 64, 400), (C3_CONFIG, 128, 300), (C5_CONFIG, 32, 200)])
def test_batched_autoreset_matches_oracle(cfg, n, T):
    rc = ResolvedConfig(cfg)
    seeds = list(range(1000, 1000 + n))
    env = make_vec(cfg, n, seeds, True)
    ors = [OracleEnv(rc.to_struct(), pcg64_state(s)) for s in seeds]
    obs = env.reset().cpu().numpy()
    for e in range(n):
        assert np.array_equal(obs[e], ors[e].reset()), e
    rng = np.random.default_rng(7)
    resets = 0
    for t in range(T):
        a = rng.integers(0, [3, 3, 3, 2, 2, 2], size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o.cpu().numpy(), r.cpu().numpy(), dn.cpu().numpy()
        for e in range(n):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
                resets += 1
            assert bool(dn[e]) == dd, (t, e)
            assert np.array_equal(r[e], rr), (t, e)
            assert np.array_equal(o[e], oo), (t, e, gr.diff(o[e], oo))
    assert T < 400 or resets > 0


def test_full_size_sampled_envs_match_oracle():
    """BASELINE size (2v2, N=65536): every env steps on the GPU; a sample of
    envs (incl. the first / last lanes and wave boundaries) is replayed by
    the oracle from the same seeds and actions."""
    rc = ResolvedConfig(C3_CONFIG)
    n, T = 65536, 40
    env = make_vec(C3_CONFIG, n, range(n), True)
    sample = [0, 1, 63, 64, 4095, 12345, 40000, 65535]
    ors = {e: OracleEnv(rc.to_struct(), pcg64_state(e)) for e in sample}
    obs = env.reset().cpu().numpy()
    for e in sample:
        assert np.array_equal(obs[e], ors[e].reset()), e
    rng = np.random.default_rng(11)
    for t in range(T):
        a = rng.integers(0, [3, 3, 3, 2, 2, 2], size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o.cpu().numpy(), r.cpu().numpy(), dn.cpu().numpy()
        for e in sample:
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
            assert bool(dn[e]) == dd and np.array_equal(r[e], rr) and np.array_equal(o[e], oo), (t, e)


def test_masked_reset_and_state_roundtrip():
    """auto_reset=False + mas_reset(mask) reproduces the oracle's reset of
    finished envs; get_state/set_state restores an exact checkpoint (the
    replay after a restore is bit-identical, RNG streams included)."""
    rc = ResolvedConfig(C3_CONFIG)
    n = 96
    env = make_vec(C3_CONFIG, n, range(500, 500 + n), False)
    ors = [OracleEnv(rc.to_struct(), pcg64_state(500 + e)) for e in range(n)]
    env.reset()
    for e in range(n):
        ors[e].reset()
    rng = np.random.default_rng(5)
    acts = [rng.integers(0, [3, 3, 3, 2, 2, 2], size=(n, rc.n_agents, 6)).astype(np.int8) for _ in range(60)]
    snap = None
    for t in range(60):
        if t == 30:
            snap = env.get_state().clone()
            snap_obs = env.obs.clone()
        o, r, dn, _ = env.step(torch.as_tensor(acts[t], device=env.device))
        dn_h = dn.cpu().numpy().astype(bool)
        o = o.cpu().numpy()
        for e in range(n):
            oo, rr, dd = ors[e].step(acts[t][e])
            assert dd == dn_h[e] and np.array_equal(o[e], oo), (t, e)
        if dn_h.any():
            ro = env.reset(mask=torch.as_tensor(dn_h.astype(np.uint8), device=env.device)).cpu().numpy()
            for e in np.nonzero(dn_h)[0]:
                assert np.array_equal(ro[e], ors[e].reset()), (t, e)
    # replay 30..59 from the checkpoint: identical trajectory
    env.set_state(snap)
    env.obs.copy_(snap_obs)
    env2_obs = []
    for t in range(30, 60):
        o, r, dn, _ = env.step(torch.as_tensor(acts[t], device=env.device))
        env2_obs.append(o.cpu().numpy().copy())
        dn_h = dn.cpu().numpy().astype(bool)
        if dn_h.any():
            env.reset(mask=torch.as_tensor(dn_h.astype(np.uint8), device=env.device))
    # compare with a fresh oracle replay of steps 30..59
    ors2 = [OracleEnv(rc.to_struct(), pcg64_state(500 + e)) for e in range(n)]
    for e in range(n):
        ors2[e].reset()
    for t in range(60):
        for e in range(n):
            oo, rr, dd = ors2[e].step(acts[t][e])
            if t >= 30:
                assert np.array_equal(env2_obs[t - 30][e], oo), (t, e)
            if dd:
                ors2[e].reset()
