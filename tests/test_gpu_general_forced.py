"""Every env on the general physics path (mas_debug_force_general), at the
per-GPU shard sizes, bit-exact against the oracle.

The contact-free fast path in k_pre appends each env it gives up on to the
general-path list (one wave-aggregated atomic per wave); k_gen_solve_g and
k_gen_toi then run over that list.  Round 2 recorded a GPU fault in a
variant of that list code on the ffa class.  Here
the list is driven to its maximum -- all N envs, every step -- on the ffa
class (C5 shard: FFA4, 16 heals, 16 randomized boxes, x16384) and on the 2v2
class, with auto-reset.  Checks: every step appends exactly N envs, the
append guard never fires (mas_debug_guards), and a sample of envs (first /
last, wave boundaries, random) replays bit-exactly through the oracle."""
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


# the xxl class (8 agents, 20 heals, 16 randomized boxes: 20 statics per
# agent, the widest general-path lane groups)
XXL_FFA8 = {
    'agents': {'n_agents': 8, 'agent_size': 1},
    'spawn_grid': {'grid_size': 8, 'floor_size': 22},
    'heals': {'reset_spawns': {'n_items': 20, 'item_size': 0.5}, 'heal': {'healing': 50}},
    'boxes': {'reset_spawns': {'n_boxes': 16, 'box_size': 1}, 'ownership': False,
              'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20,
              'randomized_shape': {'avg_w': 1.0, 'std_w': 0.5, 'avg_h': 1.0, 'std_h': 0.5}},
    'inventory': {'slots': 8},
    'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}


@pytest.mark.parametrize('name,cfg,n,T', [('C5 ffa4 shard', C5_CONFIG, 16384, 60),
                                          ('C3 2v2', C3_CONFIG, 8192, 60),
                                          ('xxl ffa8', XXL_FFA8, 4096, 60)])
def test_all_envs_on_general_path_match_oracle(name, cfg, n, T):
    rc = ResolvedConfig(cfg)
    try:
        env = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)
    env.force_general(True)
    s = {0, 1, 31, 32, 63, 64, n // 2, n - 33, n - 32, n - 2, n - 1}
    s |= set(np.random.default_rng(n).choice(n, size=24, replace=False).tolist())
    sample = sorted(s)
    idx = torch.as_tensor(sample, device=env.device)
    ors = {e: OracleEnv(rc.to_struct(), pcg64_state(e)) for e in sample}
    obs = env.reset()[idx].cpu().numpy()
    for k, e in enumerate(sample):
        assert np.array_equal(obs[k], ors[e].reset()), e
    rng = np.random.default_rng(n + 7)
    for t in range(T):
        a = rng.integers(0, HI, size=(n, rc.n_agents, 6)).astype(np.int8)
        o, r, dn, _ = env.step(torch.as_tensor(a, device=env.device))
        assert env.debug_counters()['phys_general_envs'] == n, t
        o, r, dn = o[idx].cpu().numpy(), r[idx].cpu().numpy(), dn[idx].cpu().numpy()
        for k, e in enumerate(sample):
            oo, rr, dd = ors[e].step(a[e])
            if dd:
                oo = ors[e].reset()
            assert bool(dn[k]) == dd and np.array_equal(r[k], rr), (name, t, e)
            assert np.array_equal(o[k], oo), (name, t, e, gr.diff(o[k], oo))
    assert env.debug_guards()['list_overflow'] == 0
    env.close()
