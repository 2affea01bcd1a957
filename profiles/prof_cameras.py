"""Per-phase wave time of k_cameras from the profiling build (libmas_prof.so,
`make -C gym-ma-survival-2d_amd/csrc prof`): lane 0 of each wave adds the
100 MHz constant-clock time between marks (mas_kernels.inc k_cameras,
mas_step.h update_seen_cam).  Prints the mean per wave per step (us).
usage: python profiles/prof_cameras.py [n_envs] [steps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from masurvival import abi  # noqa: E402

PHASES = {8: 'state load', 9: 'box health', 10: 'fixture table', 13: 'cone query', 11: 'LOS rays',
          12: 'OR + pack'}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    buf = (ctypes.c_ulonglong * 64)()
    env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(0)
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
    acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
    for _ in range(5):
        env.step(acts())
    abi.check(lib.mas_prof_read(env._h, buf))
    for _ in range(steps):
        env.step(acts())
    abi.check(lib.mas_prof_read(env._h, buf))
    waves = (n * env.n_agents + 63) // 64
    tot = 0.0
    for k, name in PHASES.items():
        t = buf[k] * 0.01 / (waves * steps)
        tot += t
        print(f'{name:16s} {t:8.2f} us per wave-step')
    print(f'total {tot:.2f} us per wave-step, {waves} waves')


if __name__ == '__main__':
    main()
