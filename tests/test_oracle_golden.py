"""The C oracle replays every golden episode bit-exactly.

The fixtures (tests/golden/*.npz) were produced by running the REFERENCE's
own simulation.py / semantics.py / masurvival_env.py over the test-only
Box2D/gym shim (tests/golden/make_golden.py); this pins the oracle's rules,
spawn/despawn order, RNG use, observation, reward, done and stats to the
reference code.  (Box2D arithmetic itself is the oracle's in both runs.)"""
import json

import numpy as np
import pytest

import golden_replay as gr
import oracle

FIXTURES = gr.golden_files()


def test_fixture_set_present():
    assert len(FIXTURES) >= 10


@pytest.mark.parametrize('name', FIXTURES)
def test_oracle_replays_golden_bit_exact(name):
    step, detail = gr.replay(name)
    assert step is None, f'{name}: first mismatch at step {step}: {detail}'
    d, _ = gr.load(name)
    ref = json.loads(str(d['stats']))
    stats = detail
    R = sum(1 for k in ref if k.startswith('reward'))
    for i in range(R):
        assert stats[i] == ref[f'reward{i}']
        assert stats[8 + i] == ref[f'kills{i}']
    assert stats[16] == ref['steps']
    assert stats[17] == ref['heals_used']
    assert stats[18] == ref['boxes_placed']


def test_golden_coverage():
    """The fixtures exercise every rule path the kernels implement."""
    oracle.counters(True)
    for name in FIXTURES:
        gr.replay(name)
    c = oracle.counters(True)
    for k in ['toi_event', 'sleep', 'box_broken', 'box_placed', 'item_picked', 'give_ok', 'give_lost',
              'drop_items', 'heal_used', 'aa_contact']:
        assert c[k] > 0, (k, c)


def test_ffal_fixtures_fill_past_four_slots():
    """The ffal-class fixtures (Inventory with slots > 4, more than 16 heals /
    4 boxes: semantics.py:165-245) hold inventories longer than the small
    classes' four slots, recorded from the reference's own Inventory."""
    names = [f for f in FIXTURES if f.startswith('ffal_')]
    assert len(names) >= 2
    for name in names:
        d, cfg = gr.load(name)
        assert int(d['max_inventory']) > 4, name
        assert int(d['max_inventory']) <= cfg['inventory']['slots'], name


def test_xxl_fixtures_exceed_the_xl_class():
    """The xxl-class fixtures (8 agents with more heals / boxes than the xl
    class's 8, up to 64 bodies) are configs no smaller class takes; the FFA8
    hoarders fill the eight inventory slots."""
    names = [f for f in FIXTURES if f.startswith('xxl_')]
    assert len(names) >= 2
    for name in names:
        d, cfg = gr.load(name)
        assert cfg['agents']['n_agents'] == 8, name
        assert cfg['heals']['reset_spawns']['n_items'] > 8 or cfg['boxes']['reset_spawns']['n_boxes'] > 8, name
    d, _ = gr.load('xxl_ffa8_s17.npz')
    assert int(d['max_inventory']) == 8
