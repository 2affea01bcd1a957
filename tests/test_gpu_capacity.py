"""Configs beyond the round-2 capacity classes (the reference takes any
n_agents / n_items / n_boxes / inventory slots, masurvival_env.py:166-169,
191-195, 210-221, bounded only by the spawn grid, semantics.py:59-79).

The `ffal` class (4 agents, 24 heals, 16 boxes, 8 inventory slots; 64 bodies,
the limit of the 64-bit body masks) takes the 4-agent configs of the paper's
media (8x8 grid, ~16-20 heals, ~8-12 randomized boxes, SURVEY.md section 2
row 8) and inventories larger than 4.  Parity: every env replayed by the
oracle with the same seeds and actions, bit-exact, with auto-reset.

The `xxl` class (8 agents, 20 heals, 16 boxes, 8 slots) takes the 5-8 agent
configs with the larger worlds (FFA8 and 4v4 below)."""
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

FFA4_BIG = {
    'agents': {'n_agents': 4, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 20},
    'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 12, 'box_size': 1}, 'ownership': False,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
              'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
    'inventory': {'slots': 6},
    'safe_zone': {'phases': 5, 'cooldown': 25, 'damage': 4, 'radiuses': [10, 5, 2.5, 1], 'centers': 'random'},
    'melee': MELEE}
TEAMS_BIG = {
    'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True},
    'spawn_grid': {'grid_size': 8, 'floor_size': 20},
    'heals': {'reset_spawns': {'n_items': 24, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': True,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
    'inventory': {'slots': 8},
    'safe_zone': {'phases': 5, 'cooldown': 25, 'damage': 4, 'radiuses': [10, 5, 2.5, 1], 'centers': 'random'},
    'melee': MELEE}
# the `xxl` class (8 agents, 20 heals, 16 boxes, 8 slots; 64 bodies)
FFA8_BIG = {
    'agents': {'n_agents': 8, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 24},
    'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': False,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
              'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
    'inventory': {'slots': 8},
    'safe_zone': {'phases': 5, 'cooldown': 25, 'damage': 4, 'radiuses': [12, 6, 3, 1], 'centers': 'random'},
    'melee': MELEE}
TEAMS8_BIG = {
    'agents': {'n_agents': 8, 'agent_size': 1}, 'teams': {'twoteams': True},
    'spawn_grid': {'grid_size': 7, 'floor_size': 20},
    'heals': {'reset_spawns': {'n_items': 16, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 12, 'box_size': 1}, 'ownership': True,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20},
    'inventory': {'slots': 6},
    'safe_zone': {'phases': 5, 'cooldown': 25, 'damage': 4, 'radiuses': [10, 5, 2.5, 1], 'centers': 'random'},
    'melee': MELEE}


@pytest.mark.parametrize('name,cfg,n,T', [('ffa4 20 heals 12 boxes 6 slots', FFA4_BIG, 256, 200),
                                          ('2v2 24 heals 16 owned boxes 8 slots', TEAMS_BIG, 128, 200),
                                          ('ffa8 20 heals 16 boxes 8 slots', FFA8_BIG, 128, 200),
                                          ('4v4 16 heals 12 owned boxes 6 slots', TEAMS8_BIG, 128, 200)])
def test_large_capacity_configs_match_oracle(name, cfg, n, T):
    rc = ResolvedConfig(cfg)
    try:
        env = VecMaSurvival(cfg, n_envs=n, seeds=range(500, 500 + n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)
    ors = [OracleEnv(rc.to_struct(), pcg64_state(500 + e)) for e in range(n)]
    obs = env.reset().cpu().numpy()
    for e in range(n):
        assert np.array_equal(obs[e], ors[e].reset()), e
    rng = np.random.default_rng(n)
    resets = 0
    for t in range(T):
        # collect-heavy actions: use and give often, so inventories fill past 4
        a = rng.integers(0, HI, size=(n, rc.n_agents, 6)).astype(np.int8)
        a[..., 4] &= (rng.random((n, rc.n_agents)) < 0.2).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        o, r, dn = o.cpu().numpy(), r.cpu().numpy(), dn.cpu().numpy()
        for e in range(n):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
                resets += 1
            assert bool(dn[e]) == dd and np.array_equal(r[e], rr), (name, t, e)
            assert np.array_equal(o[e], oo), (name, t, e, gr.diff(o[e], oo))
    assert resets > 0
    env.close()


def test_config_beyond_every_class_is_refused():
    """More than 8 agents (the widest class) is refused by mas_create with
    MAS_ERR_UNSUPPORTED and a message naming the compiled classes."""
    cfg = dict(FFA8_BIG, agents={'n_agents': 9, 'agent_size': 1})
    with pytest.raises(abi.MasError, match='no compiled capacity class'):
        VecMaSurvival(cfg, n_envs=8, seeds=range(8), auto_reset=True)
