"""The C4 and C5 workloads at their configured env counts on one GPU
(BASELINE.json configs[3], configs[4]).

The 8-GPU runs shard these over ranks (the driver's scaling bench); one
MI355X holds each whole: 2v2 x262144 and FFA4 (heals + randomized boxes)
x131072.  Every env steps on the GPU; a sample -- the first and last waves,
the 2^17 boundary and random envs -- is replayed by the oracle from the same
seeds and actions with auto-reset (bit-exact).  One fused PPO iteration at
2v2 x262144 drives the policy kernels at a real 16.8M-row minibatch, beyond
the 32-bit store-offset range (k_policy_train's 64-bit path)."""
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

HI = np.array([3, 3, 3, 2, 2, 2])


def _sample(n, k_random, seed):
    s = {0, 1, 63, 64, 65, 127, (1 << 17) - 1, 1 << 17, (1 << 17) + 1, n // 2, n - 65, n - 64, n - 2, n - 1}
    s |= set(np.random.default_rng(seed).choice(n, size=k_random, replace=False).tolist())
    return sorted(e for e in s if 0 <= e < n)


@pytest.mark.parametrize('name,cfg,n,T', [('C4 2v2', C3_CONFIG, 262144, 30),
                                          ('C5 ffa4', C5_CONFIG, 131072, 25)])
def test_full_config_sampled_envs_match_oracle(name, cfg, n, T):
    rc = ResolvedConfig(cfg)
    try:
        env = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)
    sample = _sample(n, 24, n)
    ors = {e: OracleEnv(rc.to_struct(), pcg64_state(e)) for e in sample}
    obs = env.reset()
    idx = torch.as_tensor(sample, device=env.device)
    o0 = obs[idx].cpu().numpy()
    for k, e in enumerate(sample):
        assert np.array_equal(o0[k], ors[e].reset()), (name, e)
    rng = np.random.default_rng(n + 3)
    general = 0
    for t in range(T):
        a = rng.integers(0, HI, size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o[idx].cpu().numpy(), r[idx].cpu().numpy(), dn[idx].cpu().numpy()
        for k, e in enumerate(sample):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
            assert bool(dn[k]) == dd and np.array_equal(r[k], rr), (name, t, e)
            assert np.array_equal(o[k], oo), (name, t, e, gr.diff(o[k], oo))
        general += env.debug_counters()['phys_general_envs']
    assert general > 0
    assert env.invalid_actions() == 0
    assert env.debug_guards()['list_overflow'] == 0
    env.close()


def test_ppo_iteration_full_c4_size():
    """One fused PPO iteration (rollout of 64 steps, GAE, 4 minibatches of
    16.8M rows) at 2v2 x262144: the losses and the updated parameters are
    finite and the parameters moved."""
    from masurvival.ppo import PPOConfig, PPOTrainer
    n = 262144
    env = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n), auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(), seed=0)
    assert tr.fused is not None
    before = [p.detach().clone() for p in tr.policy.parameters()]
    tr.iteration()
    torch.cuda.synchronize()
    stats = {k: float(v) for k, v in tr.last_stats.items()}
    assert all(np.isfinite(v) for v in stats.values()), stats
    moved = 0.0
    for p, q in zip(tr.policy.parameters(), before):
        assert bool(torch.isfinite(p).all())
        moved += float((p.detach() - q).abs().sum())
    assert moved > 0.0
    assert env.debug_guards()['list_overflow'] == 0
    del tr
    env.close()
