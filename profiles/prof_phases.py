"""Per-phase wave time of k_step from the profiling build (libmas_prof.so,
`make -C gym-ma-survival-2d_amd/csrc prof`).  Each wave's lane 0 accumulates
the 100 MHz constant-clock time between marks; we print the mean per wave
per step in microseconds and the share of the kernel.
usage: python profiles/prof_phases.py [config] [n_envs] [steps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from masurvival import abi  # noqa: E402

# k_phys marks (mas_env.h ProfPhase): after the state load, per world_step
# after Collide / island Solve / SolveTOI, and after box health + store
PHASES = ['load', 'collide (x2 steps)', 'solve (x2)', 'toi (x2)', 'box health + store']


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else '2v2'
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS[cfg_name], n_envs=n, auto_reset=True)
    buf = (ctypes.c_ulonglong * 64)()
    env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(0)
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
    acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
    for _ in range(5):
        env.step(acts())
    abi.check(lib.mas_prof_read(env._h, buf))
    active_waves = 0
    for _ in range(steps):
        env.step(acts())
        active_waves += (env.debug_counters()['phys_general_envs'] + 63) // 64
    abi.check(lib.mas_prof_read(env._h, buf))
    waves = active_waves / steps  # k_phys (general path) runs only the envs that left the fast path
    t = np.array(buf[:len(PHASES)], dtype=np.float64) * 0.01 / (waves * steps)  # us per wave-step
    top = t.sum()
    print(f'# k_phys (general path) phase times, {cfg_name} N={n}, {waves:.1f} active waves/step, mean per active wave per step (us); total {top:.1f} us')
    for name, v in zip(PHASES, t):
        print(f'{name:32s} {v:9.2f} us  {100 * v / top:5.1f}%')


if __name__ == '__main__':
    main()
