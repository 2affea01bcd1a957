"""Per-phase wave time of the agent-lane kernels k_pre_lanes and k_post_lanes
from the profiling build (libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc
prof`; MAS_PROFILE marks in mas_lanes.h / mas_post_lanes.h).  Each wave's
first lane accumulates the 100 MHz constant-clock time between marks; we print
the mean per wave per step in microseconds (waves = ceil(N / envs per wave))
and each phase's share of its kernel.
usage: python profiles/prof_lanes.py [config] [n_envs] [steps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from masurvival import abi  # noqa: E402

KERNELS = {
    'k_pre_lanes': [(20, 'load groups + agent + actions'), (21, 'pend drop, motors, use, give'),
                    (22, 'melee rays + attacks'), (23, 'stores'), (24, 'fast physics (2 substeps)'),
                    (25, 'list appends')],
    'k_post_lanes': [(41, 'load groups + agent'), (42, 'box health + cameras'),
                     (43, 'deaths, pickup, zone, rewards, stats'), (44, 'stores + reset list'),
                     (45, 'obs rows')],
}


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else '2v2'
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS[cfg_name], n_envs=n, auto_reset=True)
    am = 1
    while am < env.n_agents:
        am *= 2
    waves = (n + 64 // am - 1) // (64 // am)
    buf = (ctypes.c_ulonglong * 64)()
    env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(0)
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
    acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
    for _ in range(5):
        env.step(acts())
    torch.cuda.synchronize()
    abi.check(lib.mas_prof_read(env._h, buf))
    for _ in range(steps):
        env.step(acts())
    torch.cuda.synchronize()
    abi.check(lib.mas_prof_read(env._h, buf))
    raw = np.array(buf[:], dtype=np.float64) * 0.01 / (waves * steps)  # us per wave-step
    print(f'# agent-lane kernel phase times, {cfg_name} N={n}, {waves} waves per launch, '
          f'mean per wave per step (us)')
    for k, marks in KERNELS.items():
        t = np.array([raw[s] for s, _ in marks])
        top = t.sum()
        print(f'{k}: {top:.1f} us per wave')
        for (s, name), v in zip(marks, t):
            print(f'  {name:40s} {v:9.2f} us  {100 * v / max(top, 1e-9):5.1f}%')


if __name__ == '__main__':
    main()
