"""PPO rollout side: GAE restatement, the trainer's
host logic on CPU with a stand-in env, and the multi-rank path (gloo,
world_size 2): identical parameters on every rank after an update and
advantage normalisation over the global statistics."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from masurvival.ppo import (PPOConfig, PPOTrainer, evaluate_actions, gae_reference, gae_reference_into,
                            sample_actions)


class StandInEnv:
    """Deterministic CPU env with VecMaSurvival's step/reset surface (test double)."""

    def __init__(self, n_envs=8, n_agents=4, obs_dim=12, seed=0):
        self.n_envs, self.n_agents, self.obs_dim = n_envs, n_agents, obs_dim
        self.device = torch.device('cpu')
        self.g = torch.Generator().manual_seed(seed)
        self.t = 0
        self.obs = torch.zeros((n_envs, n_agents, obs_dim))

    def reset(self):
        self.obs = torch.randn((self.n_envs, self.n_agents, self.obs_dim), generator=self.g)
        return self.obs

    def step(self, actions, out=None):
        self.t += 1
        o, r, d = out
        o.copy_(torch.randn(o.shape, generator=self.g))
        r.copy_((actions[..., 0].float() - 1.0) * 0.5 + (actions[..., 3].float()))
        d.copy_(((torch.arange(self.n_envs) + self.t) % 5 == 0).to(torch.uint8))
        return o, r, d, {}


def test_gae_reference_known_answer():
    # one column, T=3, gamma=0.5, lam=1: hand-computed
    r = torch.tensor([[1.0], [0.0], [2.0]])
    v = torch.tensor([[0.0], [1.0], [0.0], [4.0]])
    d = torch.tensor([[0], [1], [0]], dtype=torch.uint8)
    adv, ret = gae_reference(r, v, d, 0.5, 1.0, 1)
    # t=2: delta = 2 + .5*4 - 0 = 4 ; A2 = 4
    # t=1: done -> delta = 0 - 1 = -1 ; A1 = -1
    # t=0: delta = 1 + .5*1 - 0 = 1.5 ; A0 = 1.5 + .5*(-1) = 1.0
    assert torch.equal(adv[:, 0], torch.tensor([1.0, -1.0, 4.0]))
    assert torch.equal(ret, adv + v[:3])


def test_sampling_and_logprob_consistent():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn((512, 15), generator=g)
    a, lp = sample_actions(logits, g)
    assert a.dtype == torch.int8 and a.shape == (512, 6)
    hi = torch.tensor([3, 3, 3, 2, 2, 2])
    assert bool(((a >= 0) & (a.long() < hi)).all())
    lp2, ent = evaluate_actions(logits, a)
    assert torch.allclose(lp, lp2, atol=1e-6)
    assert bool((ent > 0).all())


def _trainer(env, minibatches=2):
    tr = PPOTrainer(env, PPOConfig(horizon=6, hidden=32, minibatches=minibatches, autocast_bf16=False), seed=3)
    tr.gae_impl = gae_reference_into
    return tr


def test_trainer_iteration_cpu():
    env = StandInEnv()
    tr = _trainer(env)
    before = [p.detach().clone() for p in tr.policy.parameters()]
    tr.iteration()
    assert torch.isfinite(tr.last_stats['loss'])
    assert any(not torch.equal(a, b) for a, b in zip(before, tr.policy.parameters()))
    adv = tr.buf.adv
    assert abs(float(adv.mean())) < 1e-4 and abs(float(adv.std(unbiased=False)) - 1) < 1e-3
    assert torch.equal(tr.buf.obs[0], tr.buf.obs[-1])


def _rank_main(rank, world, init_file, out_dir):
    dist.init_process_group('gloo', init_method=f'file://{init_file}', rank=rank, world_size=world)
    torch.set_num_threads(1)
    env = StandInEnv(seed=100 + rank)  # different data per rank
    tr = _trainer(env)
    tr.iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in tr.policy.parameters()])
    adv = tr.buf.adv.reshape(-1).double()
    torch.save({'flat': flat, 's1': float(adv.sum()), 's2': float((adv ** 2).sum()), 'n': adv.numel()},
               os.path.join(out_dir, f'rank{rank}.pt'))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_update(tmp_path):
    ctx = mp.get_context('spawn')
    init_file = str(tmp_path / 'rdzv')
    ps = [ctx.Process(target=_rank_main, args=(r, 2, init_file, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(150)
        assert p.exitcode == 0
    res = [torch.load(str(tmp_path / f'rank{r}.pt'), weights_only=True) for r in range(2)]
    assert torch.equal(res[0]['flat'], res[1]['flat']), 'ranks diverged after the gradient all-reduce'
    s1 = res[0]['s1'] + res[1]['s1']
    s2 = res[0]['s2'] + res[1]['s2']
    n = res[0]['n'] + res[1]['n']
    # normalised with the global (all-reduced) statistics: global mean 0, var 1,
    # while each rank alone is not exactly centred
    assert abs(s1 / n) < 1e-5 and abs(s2 / n - 1) < 1e-3
    assert abs(res[0]['s1'] / res[0]['n']) > 1e-4


def test_split_k_linear_matches_nn_linear():
    from masurvival.ppo import LinearSplitK
    torch.manual_seed(0)
    a = torch.nn.Linear(24, 16)
    b = LinearSplitK(24, 16)
    b.load_state_dict(a.state_dict())
    x = torch.randn(8192 * 4, 24, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    ya, yb = a(x), b(x2)
    torch.testing.assert_close(ya, yb)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(a.weight.grad, b.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(a.bias.grad, b.bias.grad, rtol=1e-4, atol=1e-3)


class StatefulStandInEnv(StandInEnv):
    """StandInEnv with VecMaSurvival's get_state/set_state (a flat uint8 buffer)."""

    def get_state(self):
        return torch.cat([self.g.get_state(), torch.tensor([self.t], dtype=torch.int64).view(torch.uint8)])

    def set_state(self, buf):
        self.g.set_state(buf[:-8].clone())
        self.t = int(buf[-8:].clone().view(torch.int64)[0])


def test_checkpoint_resume_continues_the_same_trajectory(tmp_path):
    """save() after one iteration, then a fresh trainer load()s it: its next
    iteration ends with the same parameters, Adam moments and obs as the run
    that never stopped (policy + Adam + sampling generator + env state)."""
    env = StatefulStandInEnv()
    tr = _trainer(env)
    tr.iteration()
    path = str(tmp_path / 'ckpt.pt')
    tr.save(path)
    tr.iteration()
    env2 = StatefulStandInEnv(seed=99)  # different state until the load
    tr2 = _trainer(env2)
    tr2.load(path)
    tr2.iteration()
    for a, b in zip(tr.policy.parameters(), tr2.policy.parameters()):
        assert torch.equal(a, b)
    s1, s2 = tr.opt.state_dict()['state'], tr2.opt.state_dict()['state']
    for k in s1:
        assert torch.equal(s1[k]['exp_avg'], s2[k]['exp_avg'])
        assert torch.equal(s1[k]['exp_avg_sq'], s2[k]['exp_avg_sq'])
    assert torch.equal(tr.buf.obs[0], tr2.buf.obs[0]) and tr.steps_taken == tr2.steps_taken


def test_fused_adam_only_for_plain_adam():
    """FusedAdam restates clip + torch.optim.Adam for one plain param group
    only; any other optimizer setup stays on torch."""
    import torch
    from masurvival.ppo import FusedAdam
    w = [torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2))]
    assert FusedAdam.supports(torch.optim.Adam(w, lr=1e-3, eps=1e-5))
    assert not FusedAdam.supports(torch.optim.Adam([{'params': w[:1]}, {'params': w[1:]}], lr=1e-3))
    assert not FusedAdam.supports(torch.optim.Adam(w, lr=1e-3, maximize=True))
    assert not FusedAdam.supports(torch.optim.Adam(w, lr=1e-3, weight_decay=0.1))
    assert not FusedAdam.supports(torch.optim.Adam(w, lr=1e-3, amsgrad=True))
    assert not FusedAdam.supports(torch.optim.Adam(w, lr=torch.tensor(1e-3)))
    assert not FusedAdam.supports(torch.optim.SGD(w, lr=1e-3))
