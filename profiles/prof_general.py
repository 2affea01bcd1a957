"""Per-phase wave time of the general physics path (k_gen_solve, k_gen_toi)
from the profiling build (libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc
prof`).  Marks: mas_kernels.inc / mas_physics.h MAS_PROF; the first active
lane of each wave adds the 100 MHz constant-clock time since the previous
mark.  Prints the mean per ACTIVE wave per step (us).
With --ppo the env is driven by the PPO trainer (2 warm-up iterations,
then rollout steps of the trained policy): the regime of the headline bench.
usage: python profiles/prof_general.py [n_envs] [steps] [--ppo]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import torch  # noqa: E402

from masurvival import abi  # noqa: E402

SOLVE = {0: 'solve: state + contact load', 1: 'solve: collide', 2: 'solve: island solve', 3: 'solve: SolveTOI (fused)',
         4: 'solve: store'}
EPW = 8  # envs per wave of k_gen_solve_g for the 2v2 class (64 / SolveShape::G)
TOI = {20: 'toi: load + sweep', 21: 'toi: reject pre-tests', 22: 'toi: b2TimeOfImpact', 24: 'toi: TOI events',
       23: 'toi: min / exit'}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    n = int(args[0]) if len(args) > 0 else 65536
    steps = int(args[1]) if len(args) > 1 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    buf = (ctypes.c_ulonglong * 64)()
    if '--ppo' in sys.argv:
        from masurvival.ppo import PPOConfig, PPOTrainer
        tr = PPOTrainer(env, PPOConfig(), seed=0)
        for _ in range(2):
            tr.iteration()
        abi.check(lib.mas_prof_read(env._h, buf))
        gen_envs = 0
        for t in range(steps):
            tr.rollout_step(t)
            gen_envs += env.debug_counters()['phys_general_envs']
        abi.check(lib.mas_prof_read(env._h, buf))
        report(buf, gen_envs, steps)
        return
    env.reset()
    gen = torch.Generator(device=env.device)
    gen.manual_seed(0)
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
    acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
    for _ in range(150):  # let agents reach walls and each other
        env.step(acts())
    abi.check(lib.mas_prof_read(env._h, buf))
    gen_envs = 0
    for _ in range(steps):
        env.step(acts())
        gen_envs += env.debug_counters()['phys_general_envs']
    abi.check(lib.mas_prof_read(env._h, buf))
    report(buf, gen_envs, steps)


def report(buf, gen_envs, steps):
    g = gen_envs / steps
    ws, wt = 2 * (g + EPW - 1) // EPW, 2 * (4 * g + 63) // 64  # active waves per step (2 world steps)
    print(f'# general-path envs per step {g:.0f}; active waves per step: solve {ws:.0f}, toi {wt:.0f}')
    for tab, w in ((SOLVE, ws), (TOI, wt)):
        tot = 0.0
        for k, name in tab.items():
            t = buf[k] * 0.01 / (w * steps)
            tot += t
            print(f'{name:30s} {t:8.2f} us per active wave')
        print(f'{"total":30s} {tot:8.2f}')
    # k_gen_solve_g wave spans (MAS_PROF_SPAN): histogram in 10-us buckets, max
    hist = [buf[48 + b] for b in range(14)]
    if sum(hist):
        print(f'# k_gen_solve_g wave spans over {steps} steps: max {buf[62] * 0.01:.1f} us')
        for b, c in enumerate(hist):
            if c:
                print(f'  {10 * b:4d}-{10 * b + 10 if b < 13 else "":<4} us {c:8d} waves')


if __name__ == '__main__':
    main()
