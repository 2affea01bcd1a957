"""HIP path == C oracle in the regimes the benchmark times (bit-exact).

* per-GPU shard sizes of SURVEY.md 8(d): C2 1v1 x4096, the C4 shard 2v2
  x32768 and the C5 shard FFA4 (heals + randomized boxes) x16384 -- every
  env steps on the GPU, a sample (wave boundaries, first / last lanes, random
  envs) is replayed by the oracle from the same seeds and actions;
* the PPO regime: three PPO iterations of the fused trainer at the headline
  size (2v2 x65536).  The envs that left the contact-free fast path most often
  (general physics, contacts, TOI events up to the sub-step cap) are replayed
  through the oracle with the recorded policy actions and auto-reset;
* the xl capacity class (6 agents), the invalid-action counter and the
  MaSurvival facade's per-key dict observations against a golden fixture.

Parity bar: np.array_equal on every obs float, reward and done flag."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import golden_replay as gr  # noqa: E402
import oracle  # noqa: E402
from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import C1_CONFIG, C3_CONFIG, C5_CONFIG, ResolvedConfig, pcg64_state  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402
from oracle import OracleEnv  # noqa: E402

HI = np.array([3, 3, 3, 2, 2, 2])


def make_vec(cfg, n, seeds, auto_reset=True):
    try:
        return VecMaSurvival(cfg, n_envs=n, seeds=seeds, auto_reset=auto_reset)
    except abi.MasError as e:
        class_missing(e)


def _sample(n, k_random, seed):
    s = {0, 1, 63, 64, 65, 127, n // 2, n - 65, n - 64, n - 1}
    s |= set(np.random.default_rng(seed).choice(n, size=k_random, replace=False).tolist())
    return sorted(e for e in s if 0 <= e < n)


@pytest.mark.parametrize('name,cfg,n,T', [('C2 1v1', C1_CONFIG, 4096, 150),
                                          ('C4 2v2 shard', C3_CONFIG, 32768, 100),
                                          ('C5 ffa4 shard', C5_CONFIG, 16384, 100)])
def test_shard_size_sampled_envs_match_oracle(name, cfg, n, T):
    rc = ResolvedConfig(cfg)
    env = make_vec(cfg, n, range(n))
    sample = _sample(n, 40, n)
    ors = {e: OracleEnv(rc.to_struct(), pcg64_state(e)) for e in sample}
    obs = env.reset().cpu().numpy()
    for e in sample:
        assert np.array_equal(obs[e], ors[e].reset()), e
    rng = np.random.default_rng(n + 1)
    resets = 0
    for t in range(T):
        a = rng.integers(0, HI, size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        idx = torch.as_tensor(sample, device=env.device)
        o, r, dn = o[idx].cpu().numpy(), r[idx].cpu().numpy(), dn[idx].cpu().numpy()
        for k, e in enumerate(sample):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
                resets += 1
            assert bool(dn[k]) == dd and np.array_equal(r[k], rr), (name, t, e)
            assert np.array_equal(o[k], oo), (name, t, e, gr.diff(o[k], oo))
    assert env.invalid_actions() == 0
    env.close()


def test_ppo_regime_policy_actions_match_oracle():
    """Policy-driven parity at the headline size: 4 fused-PPO iterations
    (2v2 x65536, horizon 64) record every action and, per env, the GPU's
    general-path steps and SolveTOI events / sub-step-cap hits.  The envs
    that hit the cap, those with the most TOI events and the most
    general-path steps, plus fixed and random envs, are replayed through the
    oracle with those actions (auto-reset): bit-exact obs / reward / done,
    and the oracle must hit the cap on exactly the same envs."""
    from masurvival.ppo import PPOConfig, PPOTrainer
    rc = ResolvedConfig(C3_CONFIG)
    n, H, iters = 65536, 64, 4
    env = make_vec(C3_CONFIG, n, range(n))
    tr = PPOTrainer(env, PPOConfig(horizon=H), seed=0)
    assert tr.fused is not None
    gen_cnt = torch.zeros((n,), dtype=torch.int32, device=env.device)
    toi_cnt = torch.zeros((n,), dtype=torch.int32, device=env.device)
    env.set_toi_counter(toi_cnt)
    flags = torch.empty((n,), dtype=torch.uint8, device=env.device)
    acts, rews, dones = [], [], []
    for _ in range(iters):
        for t in range(H):
            tr.rollout_step(t)
            gen_cnt += (env.gen_flags(flags) != 0).to(torch.int32)  # 2: the slow list
        acts.append(tr.buf.actions.cpu().numpy())
        rews.append(tr.buf.rewards.cpu().numpy())
        dones.append(tr.buf.dones.cpu().numpy())
        tr.finish_rollout()
        tr.update()
    acts = np.concatenate(acts)    # [iters*H, N, A, 6]
    rews = np.concatenate(rews)    # [iters*H, N, A]
    dones = np.concatenate(dones)  # [iters*H, N]
    assert env.invalid_actions() == 0
    gen = gen_cnt.cpu().numpy()
    toi = toi_cnt.cpu().numpy()
    env.set_toi_counter(None)
    env.close()
    del tr
    caps, events = toi >> 16, toi & 0xffff
    assert caps.sum() > 0, 'no SolveTOI reached the sub-step cap in the PPO regime'
    # replay: the envs whose SolveTOI hit the cap, then the most TOI events,
    # then the most general-path steps, plus fixed / random envs
    pick = set(np.argsort(-caps, kind='stable')[:min(64, int((caps > 0).sum()))].tolist())
    pick |= set(np.argsort(-events, kind='stable')[:64].tolist())
    pick |= set(np.argsort(-gen, kind='stable')[:128].tolist())
    cands = sorted(pick | set(_sample(n, 8, 3)))
    # second pass: the same actions through a fresh handle, gathering the
    # candidates' observations (the env is deterministic given seeds + actions)
    env2 = make_vec(C3_CONFIG, n, range(n))
    idx = torch.as_tensor(cands, device=env2.device)
    obs0 = env2.reset()[idx].cpu().numpy()
    obs_c = []
    for t in range(acts.shape[0]):
        o, r, d, _ = env2.step(torch.as_tensor(acts[t], device=env2.device))
        assert np.array_equal(r.cpu().numpy(), rews[t]) and np.array_equal(d.cpu().numpy(), dones[t]), t
        obs_c.append(o[idx].cpu().numpy())
    env2.close()

    oracle.counters(True)
    per_env = {}
    for k, e in enumerate(cands):
        ora = OracleEnv(rc.to_struct(), pcg64_state(e))
        assert np.array_equal(obs0[k], ora.reset()), e
        for t in range(acts.shape[0]):
            oo, rr, dd = ora.step(acts[t, e])
            if dd:
                oo = ora.reset()
            assert bool(dones[t, e]) == dd and np.array_equal(rews[t, e], rr), (t, e)
            assert np.array_equal(obs_c[t][k], oo), (t, e, gr.diff(obs_c[t][k], oo))
        per_env[e] = oracle.counters(True)
    tot = {k: sum(c[k] for c in per_env.values()) for k in oracle.COUNTER_NAMES}
    capped = sorted(((c['toi_cap'], c['toi_event'], e) for e, c in per_env.items()), reverse=True)
    print('ppo-regime replay: %d envs; general-path steps max %d; GPU SolveTOI events max %d, capped envs %d; '
          'oracle counters over the replay %s; most capped env %s' % (
              len(cands), gen.max(), events.max(), int((caps > 0).sum()), json.dumps(tot), capped[:3]))
    # the oracle sees the same cap hits as the GPU on every replayed env
    for e in cands:
        assert (per_env[e]['toi_cap'] > 0) == (caps[e] > 0), (e, per_env[e], toi[e])
    dump = os.environ.get('MAS_DUMP_DIR')
    if dump:
        os.makedirs(dump, exist_ok=True)
        e = capped[0][2]
        np.savez_compressed(os.path.join(dump, 'ppo_regime_env.npz'), env_seed=e, actions=acts[:, e],
                            dones=dones[:, e], toi_cap=capped[0][0], toi_event=capped[0][1])
    assert tot['toi_event'] > 0 and tot['aa_contact'] > 0 and tot['island_contacts'] > 0, tot
    assert tot['toi_cap'] > 0, tot


def test_xl_class_six_agents_match_oracle():
    """A 6-agent FFA config needs the xl capacity class (> 4 agents)."""
    cfg = {'agents': {'n_agents': 6, 'agent_size': 1}, 'spawn_grid': {'grid_size': 4, 'floor_size': 20},
           'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}
    rc = ResolvedConfig(cfg)
    n, T = 48, 250
    env = make_vec(cfg, n, range(200, 200 + n))
    ors = [OracleEnv(rc.to_struct(), pcg64_state(200 + e)) for e in range(n)]
    obs = env.reset().cpu().numpy()
    for e in range(n):
        assert np.array_equal(obs[e], ors[e].reset()), e
    rng = np.random.default_rng(9)
    for t in range(T):
        a = rng.integers(0, HI, size=(n, 6, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o.cpu().numpy(), r.cpu().numpy(), dn.cpu().numpy()
        for e in range(n):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
            assert bool(dn[e]) == dd and np.array_equal(r[e], rr) and np.array_equal(o[e], oo), (t, e)
    env.close()


def test_invalid_actions_counted_and_rejected():
    env = make_vec(C3_CONFIG, 64, range(64))
    env.reset()
    a = torch.ones((64, 4, 6), dtype=torch.int8, device=env.device)
    env.step(a)
    assert env.invalid_actions() == 0
    a[5, 2, 3] = 2   # attack head is binary
    a[9, 0, 0] = -1
    env.step(a)
    assert env.invalid_actions() == 2
    with pytest.raises(AssertionError):
        env.step(a, validate=True)
    with pytest.raises(ValueError):
        env.step(a[:10])
    env.close()


@pytest.mark.parametrize('name', ['c3_2v2_script_s3.npz', 'nonomni_lastalive_s7.npz', 'c5_ffa4_script_s5.npz'])
def test_facade_dict_obs_match_golden(name):
    """The reference-shaped MaSurvival facade returns the fixture's dict keys,
    and each key's array equals the fixture row sliced by the layout."""
    from masurvival.envs.masurvival_env import MaSurvival
    d, cfg = gr.load(name)
    keys = json.loads(str(d['keys']))
    try:
        env = MaSurvival(cfg)
    except abi.MasError as e:
        class_missing(e)
    env.np_random = np.random.default_rng(int(d['env_seed']))
    obs = env.reset()
    assert sorted(obs.keys()) == keys

    def flat(o):
        return np.concatenate([o[k].reshape(env.n_agents, -1) for k in keys], axis=1)
    assert np.array_equal(flat(obs), d['obs'][0])
    for t in range(min(len(d['done']), 120)):
        obs, rew, done, info = env.step(tuple(d['actions'][t]))
        assert np.array_equal(flat(obs), d['obs'][t + 1]), t
        assert rew.dtype == np.float32 and np.array_equal(rew, d['rewards'][t]) and done == bool(d['done'][t])
        assert info == {}
    env.close()
