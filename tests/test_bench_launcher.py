"""bench.py --gpus N starts its own torch.distributed.run child when no
launcher set WORLD_SIZE, relays rank 0's JSON line and reports the real
world size (MAS_BENCH_DRYRUN=1: the launcher, rendezvous, barrier and
max-over-ranks path over gloo on CPU, with no env)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ, MAS_BENCH_DRYRUN='1')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], capture_output=True, text=True,
                       env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    out = _run('--gpus', '2', '--steps', '5', '--warmup', '1')
    assert out['n_gpus'] == 2 and out['steps'] == 5 and out['warmup'] == 1


def test_bench_single_rank_default():
    out = _run('--steps', '3')
    assert out['n_gpus'] == 1
