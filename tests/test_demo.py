"""The demo CLI (`masurvival.demo`, the reference's `demo.py:164-293`
arguments): argument parsing, the JSON config loader and the unsupported
options on CPU; one random-policy episode and the batched mode on the GPU."""
import json

import numpy as np

import pytest

from masurvival import demo
from masurvival.config import ResolvedConfig


def test_parser_matches_reference_arguments():
    a = demo.build_parser().parse_args([])
    assert (a.policy, a.max_steps, a.env_config_fpath, a.render) == ('random', None, None, False)
    assert (a.screenshot_step, a.gif_record_interval, a.print_benchmark) == (0, 10, False)
    a = demo.build_parser().parse_args(['random', '--max-steps', '7', '-c', 'x.json', '--benchmark'])
    assert (a.max_steps, a.env_config_fpath, a.print_benchmark) == (7, 'x.json', True)
    with pytest.raises(SystemExit):
        demo.build_parser().parse_args(['greedy'])


def test_json_config_loads_and_resolves(tmp_path):
    cfg = {'agents': {'n_agents': 4}, 'teams': {'twoteams': True}, 'melee': {'cooldown': 40}}
    p = tmp_path / 'c3.json'
    p.write_text(json.dumps(cfg))
    loaded = demo.load_config(str(p))
    assert loaded == cfg
    rc = ResolvedConfig(loaded)
    assert rc.n_agents == 4 and rc.has_teams
    assert demo.load_config(None) is None


@pytest.mark.parametrize('argv', [['interactive'], ['-r']])
def test_unsupported_options_exit_with_a_message(argv):
    args = demo.build_parser().parse_args(argv)
    with pytest.raises(SystemExit, match='not available in the MI355X build'):
        demo.check_supported(args)


@pytest.mark.gpu
def test_demo_episode_and_benchmark_on_gpu(capsys):
    assert demo.main(['--max-steps', '30', '--benchmark', '--seed', '3']) == 0
    out = capsys.readouterr().out
    assert 'Episode complete' in out and 'Performance test results' in out and "'steps'" in out


def test_frames_are_saved(tmp_path):
    a = demo.build_parser().parse_args(['-s', str(tmp_path / 's.png'), '-g', str(tmp_path / 'e.gif')])
    f = np.zeros((8, 8, 3), dtype=np.uint8)
    demo.save_frames(a, {'screenshot': f, 'gif': [f, f + 50]})
    assert (tmp_path / 's.png').stat().st_size > 0 and (tmp_path / 'e.gif').stat().st_size > 0


@pytest.mark.gpu
def test_demo_screenshot_and_gif_on_gpu(tmp_path):
    assert demo.main(['--max-steps', '12', '-s', str(tmp_path / 's.png'), '--screenshot-step', '5',
                      '-g', str(tmp_path / 'e.gif'), '--gif-record-interval', '4']) == 0
    assert (tmp_path / 's.png').exists() and (tmp_path / 'e.gif').exists()


@pytest.mark.gpu
def test_demo_batched_on_gpu(capsys):
    assert demo.main(['--envs', '512', '--max-steps', '10']) == 0
    assert 'agent-env-steps/s' in capsys.readouterr().out
