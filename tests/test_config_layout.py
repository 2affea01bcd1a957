"""Config front-end and observation layout follow the reference
(masurvival_env.py:49-56 merge, :309-312 melee switch, :391-447 spaces)."""
import numpy as np
import pytest

from masurvival.config import C3_CONFIG, C5_CONFIG, ResolvedConfig, merge_config
from masurvival.layout import obs_layout, split_obs


def test_merge_one_level_and_unknown_key():
    c = merge_config({'agents': {'n_agents': 3}})
    assert c['agents'] == {'n_agents': 3, 'agent_size': 1}
    with pytest.raises(KeyError):
        merge_config({'nonexistent': {}})


def test_nested_subdict_replaced_not_merged():
    # boxes.reset_spawns given partially -> box_size missing (reference KeyError at :348)
    rc = ResolvedConfig({'melee': {'range': 2, 'damage': 20, 'cooldown': 40},
                         'boxes': {'reset_spawns': {'n_boxes': 2}, 'ownership': False,
                                   'item': {'item_size': 0.5, 'offset': 0.75}, 'health': 20}})
    assert rc.config['boxes']['reset_spawns'] == {'n_boxes': 2}


def test_melee_switch_and_missing_melee():
    assert ResolvedConfig(None).continuous_melee is False
    assert ResolvedConfig({'melee': {'range': 2, 'damage': 20}}).continuous_melee is True
    assert ResolvedConfig({'melee': {'range': 2, 'damage': 20}}).to_struct().melee_cooldown == 0
    with pytest.raises(KeyError):
        ResolvedConfig({'agents': {'n_agents': 2, 'agent_size': 1}})


def test_invalid_sizes():
    with pytest.raises(ValueError):
        ResolvedConfig({'agents': {'n_agents': 1, 'agent_size': 1}, 'melee': {'range': 2, 'damage': 1}})
    with pytest.raises(IndexError):
        ResolvedConfig({'agents': {'n_agents': 9, 'agent_size': 1}, 'melee': {'range': 2, 'damage': 1,
                                                                             'cooldown': 1}})


@pytest.mark.parametrize('cfg,D', [(None, 138), (C3_CONFIG, 160), (C5_CONFIG, 468)])
def test_obs_dim_matches_survey(cfg, D):
    rc = ResolvedConfig(cfg)
    d, lay = obs_layout(rc.n_agents, rc.n_heals, rc.n_boxes, rc.has_teams)
    assert d == D
    assert list(lay) == sorted(lay)


def test_split_obs_roundtrip():
    rc = ResolvedConfig(C3_CONFIG)
    d, lay = obs_layout(rc.n_agents, rc.n_heals, rc.n_boxes, rc.has_teams)
    flat = np.arange(4 * d, dtype=np.float32).reshape(4, d)
    parts = split_obs(flat, lay)
    back = np.concatenate([parts[k].reshape(4, -1) for k in lay], axis=1)
    assert np.array_equal(back, flat)
    assert parts['others'].shape == (4, 3, 9)


def test_lidars_key_is_opt_in_and_sorted():
    base = ResolvedConfig(C3_CONFIG)
    d0, lay0 = obs_layout(base.n_agents, base.n_heals, base.n_boxes, base.has_teams)
    assert 'lidars' not in lay0 and base.lidars is None
    rc = ResolvedConfig(dict(C3_CONFIG, lidars={'n_lasers': 8, 'fov': 1.5, 'depth': 6}))
    s = rc.to_struct()
    assert (s.lidar_n_lasers, s.lidar_fov, s.lidar_depth) == (8, 1.5, 6.0)
    d, lay = obs_layout(rc.n_agents, rc.n_heals, rc.n_boxes, rc.has_teams, 8)
    assert d == d0 + 8 and list(lay) == sorted(lay)
    assert lay['lidars'] == (lay0['others'][0], (8,))
    for bad in (1, 33):
        with pytest.raises(ValueError):
            ResolvedConfig(dict(C3_CONFIG, lidars={'n_lasers': bad, 'fov': 1.0, 'depth': 5}))
