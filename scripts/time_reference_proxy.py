"""Labelled CPU proxy for the reference's own path: the
reference's Python env (masurvival_env.py + simulation.py + semantics.py from
/root/reference) stepped by demo.py's random policy (demo.py:119,135-141),
over the test-only Box2D/gym shim of tests/golden/shim, whose physics calls
the C oracle.  PyBox2D itself is absent from this image, so this is a PROXY:
Python dispatch, rules and obs assembly are the reference's; the Box2D calls
are the oracle's C (through ctypes).  Runs in THIS container (the reference
never travels to the GPU box); writes profiles/<out>.json.

usage: python scripts/time_reference_proxy.py [seconds_per_config] [out name]"""
import copy
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import make_golden as mg  # noqa: E402

CONFIGS = {
    '1v1': None,
    '2v2': {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True}, 'melee': mg.MELEE},
}


def time_config(name, cfg, budget):
    mod = mg.load_reference()
    env = mod.MaSurvival(config=copy.deepcopy(cfg) if cfg is not None else None)
    groups = env.simulation.groups
    mg.Box2D.CANONICAL_GROUPS[:] = list(groups.values())
    mg.Box2D.STATIC_GROUPS[:] = [groups['walls'], groups['boxes']]
    env.np_random = np.random.default_rng(0)
    env.reset()
    rng = np.random.default_rng(1)
    A = env.n_agents
    steps, episodes = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget:
        acts = tuple(rng.integers(0, [3, 3, 3, 2, 2, 2]) for _ in range(A))
        _, _, done, _ = env.step(acts)
        steps += 1
        if done:
            env.reset()
            episodes += 1
    dt = time.perf_counter() - t0
    return {'config': name, 'env_steps': steps, 'episodes_finished': episodes, 'seconds': dt,
            'env_steps_per_s': steps / dt, 'agent_env_steps_per_s': steps * A / dt}


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    out = sys.argv[2] if len(sys.argv) > 2 else 'r02_reference_proxy'
    cpu = subprocess.run(['lscpu'], capture_output=True, text=True).stdout
    model = next((ln.split(':', 1)[1].strip() for ln in cpu.splitlines() if ln.startswith('Model name')), '?')
    res = {'what': 'reference Python env (random policy, 1 process, 1 thread) over the test-only Box2D shim '
                   '(oracle C physics via ctypes); PROXY for PyBox2D, timed in the build container',
           'cpu_model': model, 'nproc': os.cpu_count(), 'python': platform.python_version(),
           'results': [time_config(k, v, budget) for k, v in CONFIGS.items()]}
    path = os.path.join(ROOT, 'profiles', out + '.json')
    json.dump(res, open(path, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
