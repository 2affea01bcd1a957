"""TEST INFRASTRUCTURE: replay a golden fixture through the C oracle."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

from masurvival.config import ResolvedConfig, pcg64_state  # noqa: E402
from oracle import OracleEnv  # noqa: E402

GOLDEN_DIR = os.path.join(ROOT, 'tests', 'golden')


def golden_files():
    return sorted(f for f in os.listdir(GOLDEN_DIR) if f.endswith('.npz'))


def load(name):
    d = np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False)
    cfg = json.loads(str(d['config']))
    return d, cfg


def replay(name, verbose=False):
    """Returns (first mismatching step or None, details)."""
    d, cfg = load(name)
    rc = ResolvedConfig(cfg)
    env = OracleEnv(rc.to_struct(), pcg64_state(int(d['env_seed'])))
    obs = env.reset()
    if not np.array_equal(obs, d['obs'][0]):
        return 0, diff(obs, d['obs'][0])
    for t in range(len(d['done'])):
        obs, rew, done = env.step(d['actions'][t])
        if not np.array_equal(obs, d['obs'][t + 1]):
            return t + 1, diff(obs, d['obs'][t + 1])
        if not np.array_equal(rew, d['rewards'][t]) or done != bool(d['done'][t]):
            return t + 1, ('rew/done', rew, d['rewards'][t], done, bool(d['done'][t]))
    stats = env.flush_stats()
    return None, stats


def diff(a, b):
    idx = np.argwhere(a != b)
    return [(tuple(i), float(a[tuple(i)]), float(b[tuple(i)])) for i in idx[:10]]


if __name__ == '__main__':
    for f in golden_files():
        print(f, replay(f))
