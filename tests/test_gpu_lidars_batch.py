"""Lidars (`simulation.py:357-392`, opt-in 'lidars' key) at batch scale on the
GPU against the C oracle (bit-exact).

`k_lidar` runs one lane per (env, agent, laser) ray, so several envs share a
wave (2v2 with 8 lasers: 32 rays per env, 2 envs per wave; FFA4 with 16
lasers: 64 rays per env, one env per wave).  These tests put many envs
through the kernel at once, with auto-reset and with `mas_reset(mask)`
(`launch_reset` -> `k_obs` with a mask -> `k_lidar` with the same mask), and
replay a sample that holds the first and last envs and the wave boundaries
through the oracle with the same seeds and actions.

A short safe zone (cooldown 12, damage 6) makes every episode end inside the
horizon, so the auto-reset step (`k_obs` resetting the done envs of its block,
then `k_lidar` over the fresh bodies) is covered many times.
Parity bar: np.array_equal on every obs float (the lidar columns included),
reward and done flag."""
import math

import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import golden_replay as gr  # noqa: E402
from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import ResolvedConfig, pcg64_state  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402
from oracle import OracleEnv  # noqa: E402

HI = np.array([3, 3, 3, 2, 2, 2])
MELEE = {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}
SHORT_ZONE = {'phases': 5, 'cooldown': 12, 'damage': 6, 'radiuses': [10, 5, 2.5, 1], 'centers': 'random'}

LID_2V2 = {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True}, 'melee': MELEE,
           'safe_zone': SHORT_ZONE, 'lidars': {'n_lasers': 8, 'fov': 0.5 * math.pi, 'depth': 6}}
LID_FFA4 = {
    'agents': {'n_agents': 4, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 20},
    'heals': {'reset_spawns': {'n_items': 16, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': False,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
              'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
    'melee': MELEE, 'safe_zone': SHORT_ZONE,
    'lidars': {'n_lasers': 16, 'fov': 2.0 * math.pi * 15 / 16, 'depth': 5.5}}


def _sample(n, rays_per_env, k_random, seed):
    """first / last envs, the envs on both sides of every 4th wave boundary
    of k_lidar's ray grid, and random envs"""
    epw = max(1, 64 // rays_per_env)
    s = {0, 1, n - 2, n - 1, n // 2}
    for w in range(0, n // epw, max(1, n // epw // 16)):
        s |= {w * epw - 1, w * epw, w * epw + epw - 1}
    s |= set(np.random.default_rng(seed).choice(n, size=k_random, replace=False).tolist())
    return sorted(e for e in s if 0 <= e < n)


def _make(cfg, n):
    try:
        return VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)


def _run(cfg, n, T, reset_every, seed):
    rc = ResolvedConfig(cfg)
    nl = rc.lidars['n_lasers']
    env = _make(cfg, n)
    lid_off, lid_shape = env.layout['lidars']
    assert lid_shape == (nl,)
    sample = _sample(n, rc.n_agents * nl, 24, seed)
    idx = torch.as_tensor(sample, device=env.device)
    ors = {e: OracleEnv(rc.to_struct(), pcg64_state(e)) for e in sample}
    last = {}
    obs = env.reset()[idx].cpu().numpy()
    for k, e in enumerate(sample):
        last[e] = ors[e].reset()
        assert np.array_equal(obs[k], last[e]), e
    rng = np.random.default_rng(seed)
    resets = masked = hits = 0
    for t in range(T):
        if reset_every and t % reset_every == reset_every - 1:
            # mas_reset(mask): only the masked envs are reset (their obs rows
            # and lidar columns rewritten); the other rows keep the last step's
            mask = rng.random(n) < 0.3
            mask[sample[::3]] = True
            o = env.reset(torch.as_tensor(mask.astype(np.uint8), device=env.device))[idx].cpu().numpy()
            for k, e in enumerate(sample):
                if mask[e]:
                    last[e] = ors[e].reset()
                    masked += 1
                assert np.array_equal(o[k], last[e]), ('masked reset', t, e, gr.diff(o[k], last[e]))
        a = rng.integers(0, HI, size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o[idx].cpu().numpy(), r[idx].cpu().numpy(), dn[idx].cpu().numpy()
        for k, e in enumerate(sample):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
                resets += 1
            last[e] = oo
            assert bool(dn[k]) == dd and np.array_equal(r[k], rr), (t, e)
            assert np.array_equal(o[k], oo), (t, e, gr.diff(o[k], oo))
            hits += int((oo[:, lid_off:lid_off + nl] < 1.0).sum())
    env.close()
    return resets, masked, hits


def test_lidars_2v2_batched_auto_reset_matches_oracle():
    """2v2, 8 lasers, 4096 envs (2 envs per 64-ray wave), 150 steps, auto-reset."""
    resets, _, hits = _run(LID_2V2, 4096, 150, 0, 41)
    assert resets > 0 and hits > 0, (resets, hits)


def test_lidars_ffa4_batched_auto_reset_matches_oracle():
    """FFA4 with 16 heals + 16 randomized boxes, 16 lasers, 1024 envs, 150 steps."""
    resets, _, hits = _run(LID_FFA4, 1024, 150, 0, 42)
    assert resets > 0 and hits > 0, (resets, hits)


LID_XXL = {
    'agents': {'n_agents': 8, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 22},
    'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 12, 'box_size': 1}, 'ownership': False,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
    'inventory': {'slots': 6},
    'melee': MELEE, 'safe_zone': SHORT_ZONE,
    'lidars': {'n_lasers': 12, 'fov': 1.5 * math.pi, 'depth': 7}}


def test_lidars_xxl_batched_auto_reset_matches_oracle():
    """The xxl class (8 agents, 20 heals, 12 boxes), 12 lasers, 512 envs, 150 steps."""
    resets, _, hits = _run(LID_XXL, 512, 150, 0, 44)
    assert resets > 0 and hits > 0, (resets, hits)


def test_lidars_masked_reset_matches_oracle():
    """mas_reset(mask) every 25 steps (launch_reset -> k_obs and k_lidar with the
    mask) between auto-reset steps: 2v2 8 lasers x1024."""
    resets, masked, hits = _run(LID_2V2, 1024, 100, 25, 43)
    assert masked > 0 and hits > 0, (masked, hits)
