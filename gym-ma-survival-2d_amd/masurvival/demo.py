"""Demo / benchmark CLI with the reference's arguments (`demo.py:164-293`):
run one episode of `MaSurvival` with a random policy, print the episode
stats, and with --benchmark the per-step time (mean, std) as `demo.py:154-156`
does.  `--config` loads a JSON env config like `demo.py:174-176`.

Added for the batched build: `--envs N` runs N envs of `VecMaSurvival` on the
device (auto-reset, random actions drawn on the device) for --max-steps steps
and reports agent-env-steps/s.

--screenshot / --gif record `render(mode='rgb_array')` frames (device state,
masurvival.render) as in `demo.py:178-209`, written with PIL instead of
imageio + gifsicle.  Out of scope (pygame): the interactive policy and
--render (a window); they exit with an error naming the missing feature.

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
                 '(MI355X build; interactive play and the pygame window are not available).')


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
                    help='Record a frame of the episode to the given file (--screenshot-step picks it).')
    ap.add_argument('--screenshot-step', dest='screenshot_step', metavar='STEP', type=int, default=0)
    ap.add_argument('-g', '--gif', dest='gif_fpath', metavar='PATH', type=str, default=None,
                    help='Record a GIF to the given file (one frame every --gif-record-interval steps).')
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
    if args.render:
        missing.append('rendering to a window (--render)')
    if missing:
        raise SystemExit('not available in the MI355X build: ' + ', '.join(missing))


def demo_env(env, max_steps: Optional[int] = None, print_benchmark: bool = False, seed: Optional[int] = None,
             record=None):
    """One episode with a random policy (`demo.py:84-157`): until done or
    max_steps; `record(t, frame)` gets an rgb_array frame after the reset
    and after each step; returns (stats, step times)."""
    times: List[float] = []
    t, obs, done = 0, env.reset(seed=seed), False
    env.action_space.seed(seed)
    if record is not None:
        record(t, env.render(mode='rgb_array'))
    while not done:
        action = env.action_space.sample()
        t0 = time.perf_counter()
        obs, reward, done, info = env.step(action)  # returns host arrays: synchronous
        times.append(time.perf_counter() - t0)
        t += 1
        if record is not None:
            record(t, env.render(mode='rgb_array'))
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
    rec = {'screenshot': None, 'gif': []}

    def record(t, frame):
        if args.screenshot_fpath is not None and t == args.screenshot_step:
            rec['screenshot'] = frame
        if args.gif_fpath is not None and t % args.gif_record_interval == 0:
            rec['gif'].append(frame)
    want = args.screenshot_fpath is not None or args.gif_fpath is not None
    demo_env(env, args.max_steps, args.print_benchmark, args.seed, record if want else None)
    save_frames(args, rec)
    return 0


def save_frames(args, rec) -> None:
    """The recorded screenshot (PNG) and GIF (`demo.py:201-209`), via PIL."""
    from PIL import Image
    if args.screenshot_fpath is not None and rec['screenshot'] is not None:
        print(f'Saving screenshot to {args.screenshot_fpath}.')
        Image.fromarray(rec['screenshot']).save(args.screenshot_fpath)
    if args.gif_fpath is not None and rec['gif']:
        frames = [Image.fromarray(f) for f in rec['gif']]
        frames[0].save(args.gif_fpath, save_all=True, append_images=frames[1:], duration=100, loop=0)


if __name__ == '__main__':
    sys.exit(main())
