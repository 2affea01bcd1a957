"""Demo / benchmark CLI with the reference's arguments (`demo.py:164-293`):
run one episode of `MaSurvival` with a random policy, print the episode
stats, and with --benchmark the per-step time (mean, std) as `demo.py:154-156`
does.  `--config` loads a JSON env config like `demo.py:174-176`.

Added for the batched build: `--envs N` runs N envs of `VecMaSurvival` on the
device (auto-reset, random actions drawn on the device) for --max-steps steps
and reports agent-env-steps/s.

Out of scope (they need pygame / a renderer, not on the step path): the
interactive policy and --render / --screenshot / --gif, which exit with an
error naming the missing feature.

usage: python -m masurvival.demo [random] [--max-steps N] [-c CONFIG.json]
                                 [--benchmark] [--envs N]"""
import argparse
import json
import pprint
import sys
import time
from typing import List, Optional

import numpy as np

ARGPARSE_DESC = ('Test the environment for one episode with a random policy '
                 '(MI355X build; interactive play and rendering are not available).')


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=ARGPARSE_DESC, formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument('policy', metavar='POLICY', type=str, default='random', nargs='?',
                    choices=['random', 'interactive'], help='The policy to use for testing.')
    ap.add_argument('--max-steps', dest='max_steps', metavar='STEPS', type=int, default=None,
                    help='Run only for the given amount of steps.')
    ap.add_argument('-c', '--config', dest='env_config_fpath', metavar='PATH', type=str, default=None,
                    help='Use the given JSON file as the env configuration.')
    ap.add_argument('-r', '--render', action='store_true', dest='render', default=False,
                    help='(not available in this build)')
    ap.add_argument('-s', '--screenshot', dest='screenshot_fpath', metavar='PATH', type=str, default=None,
                    help='(not available in this build)')
    ap.add_argument('--screenshot-step', dest='screenshot_step', metavar='STEP', type=int, default=0)
    ap.add_argument('-g', '--gif', dest='gif_fpath', metavar='PATH', type=str, default=None,
                    help='(not available in this build)')
    ap.add_argument('--gif-record-interval', dest='gif_record_interval', metavar='N', type=int, default=10)
    ap.add_argument('--benchmark', dest='print_benchmark', action='store_true', default=False,
                    help='Print benchmark information at the end of the episode.')
    ap.add_argument('--envs', dest='n_envs', metavar='N', type=int, default=None,
                    help='Batched mode: N device envs (auto-reset) for --max-steps steps (default 100).')
    ap.add_argument('--seed', dest='seed', type=int, default=None, help='Env seed (the reference ignores it).')
    return ap


def load_config(path: Optional[str]):
    """The JSON env config (`demo.py:174-176`), or None for the default."""
    if path is None:
        return None
    with open(path) as f:
        return json.load(f)


def check_supported(args) -> None:
    missing = []
    if args.policy == 'interactive':
        missing.append('the interactive policy (pygame)')
    if args.render or args.screenshot_fpath or args.gif_fpath:
        missing.append('rendering (--render / --screenshot / --gif)')
    if missing:
        raise SystemExit('not available in the MI355X build: ' + ', '.join(missing))


def demo_env(env, max_steps: Optional[int] = None, print_benchmark: bool = False, seed: Optional[int] = None):
    """One episode with a random policy (`demo.py:84-157`): until done or
    max_steps; returns (stats, step times)."""
    times: List[float] = []
    t, obs, done = 0, env.reset(seed=seed), False
    env.action_space.seed(seed)
    while not done:
        action = env.action_space.sample()
        t0 = time.perf_counter()
        obs, reward, done, info = env.step(action)  # returns host arrays: synchronous
        times.append(time.perf_counter() - t0)
        t += 1
        if max_steps is not None and t == max_steps:
            print(f'Maximum number of steps {t} reached, terminating episode.')
            break
    print('Episode complete. Stats printed below.')
    stats = env.flush_stats()
    env.close()
    pprint.PrettyPrinter().pprint(stats)
    if print_benchmark:
        a = np.array(times)
        print(f'Performance test results: {a.mean()}, {a.std()}')
    return stats, times


def demo_batched(config, n_envs: int, steps: int, seed: int = 0):
    """N device envs, random actions drawn on the device, auto-reset; prints
    and returns agent-env-steps/s."""
    import torch
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(config, n_envs=n_envs, seeds=range(seed, seed + n_envs), auto_reset=True)
    env.reset()
    dev = env.device
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    acts = torch.empty((n_envs, env.n_agents, 6), dtype=torch.int8, device=dev)

    def draw():
        acts.copy_((torch.rand((n_envs, env.n_agents, 6), generator=gen, device=dev) * hi).to(torch.int8))
    for _ in range(5):
        draw()
        env.step(acts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        draw()
        env.step(acts)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rate = n_envs * env.n_agents * steps / dt
    print(f'{n_envs} envs x {steps} steps: {1e3 * dt / steps:.3f} ms/step, {rate:.4g} agent-env-steps/s')
    env.close()
    return rate


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    check_supported(args)
    config = load_config(args.env_config_fpath)
    if args.n_envs is not None:
        demo_batched(config, args.n_envs, args.max_steps or 100, args.seed or 0)
        return 0
    from masurvival.envs.masurvival_env import MaSurvival
    env = MaSurvival(config=config)
    demo_env(env, args.max_steps, args.print_benchmark, args.seed)
    return 0


if __name__ == '__main__':
    sys.exit(main())
