"""The reference-shaped surfaces above the C-ABI, checked against the oracle
and the reference-generated fixtures on the GPU:

* the ``MaSurvival`` facade (masurvival_env.py:32-135) replays golden
  episodes and returns the reference's observation dict key by key
  (fetch_observations :510-657, sorted ``spaces.Dict`` keys);
* a demo episode (``masurvival.demo.demo_env``, demo.py:84-157) from a JSON
  config (demo.py:174-176) ends with the stats the oracle computes for the
  same actions (flush_stats :471-508);
* ``mas_render_view`` (what the renderer draws) holds the oracle's bodies:
  agent pose / alive / health, box and heal positions, counts.
"""
import json

import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import golden_replay as gr  # noqa: E402
from masurvival import demo  # noqa: E402
from masurvival.config import C5_CONFIG, ResolvedConfig, pcg64_state  # noqa: E402
from masurvival.envs.masurvival_env import MaSurvival  # noqa: E402
from masurvival.layout import split_obs  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402
from oracle import OracleEnv  # noqa: E402


def _key_layout(keys, rc):
    from masurvival.layout import obs_layout
    n_lasers = rc.lidars['n_lasers'] if rc.lidars else 0
    D, lay = obs_layout(rc.n_agents, rc.n_heals, rc.n_boxes, rc.has_teams, n_lasers)
    assert list(lay) == keys
    return D, lay


@pytest.mark.parametrize('name', ['c3_2v2_random_s4.npz', 'c5_ffa4_script_s5.npz', 'lidars_ffa4_s13.npz'])
def test_facade_dict_obs_matches_golden(name):
    d, cfg = gr.load(name)
    keys = json.loads(str(d['keys']))
    rc = ResolvedConfig(cfg)
    D, lay = _key_layout(keys, rc)
    env = MaSurvival(config=cfg)
    assert list(env.observation_space.keys()) == keys

    def same(obs, flat, t):
        ref = split_obs(flat, lay)
        assert list(obs) == keys, t
        for k in keys:
            assert obs[k].dtype == np.float32 and obs[k].shape == ref[k].shape, (t, k)
            assert np.array_equal(obs[k], ref[k]), (t, k)
    same(env.reset(seed=int(d['env_seed'])), d['obs'][0], 0)
    for t in range(len(d['done'])):
        acts = tuple(np.asarray(a, dtype=np.int64) for a in d['actions'][t])
        obs, rew, done, info = env.step(acts)
        same(obs, d['obs'][t + 1], t + 1)
        assert np.array_equal(rew, d['rewards'][t]) and done == bool(d['done'][t]) and info == {}, t
    ref_stats = json.loads(str(d['stats']))
    assert env.flush_stats() == pytest.approx(ref_stats, abs=0)
    env.close()


class _Recorder(MaSurvival):
    def __init__(self, config):
        super().__init__(config=config)
        self.actions = []

    def step(self, actions):
        self.actions.append(np.stack([np.asarray(a) for a in actions]).astype(np.int8))
        return super().step(actions)


@pytest.mark.parametrize('cfg', [None, {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True},
                                         'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}])
def test_demo_episode_stats_match_oracle(tmp_path, cfg):
    path = None
    if cfg is not None:
        path = tmp_path / 'env.json'
        path.write_text(json.dumps(cfg))
        path = str(path)
    config = demo.load_config(path)
    env = _Recorder(config)
    stats, times = demo.demo_env(env, max_steps=300, seed=21)
    assert len(times) == len(env.actions) > 0
    rc = ResolvedConfig(config)
    ora = OracleEnv(rc.to_struct(), pcg64_state(21))
    ora.reset()
    for a in env.actions:
        _, _, done = ora.step(a)
    s = ora.flush_stats()
    R = 2 if rc.has_teams else rc.n_agents
    want = {f'reward{i}': float(s[i]) for i in range(R)}
    want.update({f'kills{i}': int(s[8 + i]) for i in range(R)})
    want.update(steps=int(s[16]), heals_used=int(s[17]), boxes_placed=int(s[18]))
    assert stats == want
    assert stats['steps'] == len(env.actions)


def test_render_view_matches_oracle_state():
    rc = ResolvedConfig(C5_CONFIG)
    n, T = 6, 120
    seeds = list(range(300, 300 + n))
    env = VecMaSurvival(C5_CONFIG, n_envs=n, seeds=seeds, auto_reset=False)
    ors = [OracleEnv(rc.to_struct(), pcg64_state(s)) for s in seeds]
    env.reset()
    obs_o = [o.reset() for o in ors]
    lay = env.layout
    rng = np.random.default_rng(5)
    done = np.zeros(n, dtype=bool)
    checked = 0
    for t in range(T + 1):
        if t % 20 == 0:
            for e in range(n):
                if done[e]:
                    continue
                v = env.render_view(e)
                ref = split_obs(obs_o[e], lay)
                ag = ref['agent']  # [A, 8]: id, health, x, y, angle, vx, vy, w
                # alive per the device; the oracle's row of a dead agent is
                # zeros (health can be <= 0 while alive: delayed zone deaths)
                alive = v['agents'][:, 3] == 1.0
                assert np.all(ag[~alive][:, 1:] == 0.0), (t, e)
                assert np.array_equal(v['agents'][alive][:, :3], ag[alive][:, 2:5]), (t, e)
                assert np.array_equal(v['agents'][alive][:, 4], ag[alive][:, 1]), (t, e)
                present = ref['boxes_mask'][0] == 0
                assert len(v['boxes']) == int(present.sum()), (t, e)
                assert np.array_equal(v['boxes'][:, :2], ref['boxes'][0][present][:, 8:10]), (t, e)
                hp = ref['heals_mask'][0] == 0
                assert np.array_equal(v['heals'], ref['heals'][0][hp]), (t, e)
                ip = ref['box_items_mask'][0] == 0
                assert np.array_equal(v['items'][:, :2], ref['box_items'][0][ip][:, 8:10]), (t, e)
                checked += 1
        if t == T:
            break
        a = rng.integers(0, [3, 3, 3, 2, 2, 2], size=(n, rc.n_agents, 6)).astype(np.int8)
        env.step(torch.as_tensor(a, device=env.device))
        for e in range(n):
            if not done[e]:
                obs_o[e], _, done[e] = ors[e].step(a[e])
    assert checked >= n * 3
    env.close()
