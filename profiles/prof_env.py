"""Per-phase wave time of the env-step kernels from the profiling build
(libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc prof`; MAS_PROFILE marks,
mas_env.h).  Each wave accumulates the 100 MHz constant-clock time between
marks in LDS and adds it to its own record at its end (plain stores, no
atomics); printed: the mean per ACTIVE wave (us) of each phase, its share,
and the mean wave span, per kernel, over `steps` steps.
Regimes: --ppo (2 PPO iterations of pre-roll, then rollout steps of the
trained policy: the headline bench's regime) or random actions after 150
steps (default).
usage: python profiles/prof_env.py [config] [n_envs] [steps] [--ppo]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from masurvival import abi  # noqa: E402

PROF_HEAD, PROF_KERNELS, PROF_BLOCKS = 64, 6, 16384  # mas_env.h kProfHead / kProfKernels / kProfBlocks
PROF_WORDS = PROF_HEAD + PROF_KERNELS * PROF_BLOCKS * 16
GEN = [(0, 'ws1 load'), (1, 'ws1 collide'), (2, 'ws1 island solve'), (5, 'ws1 body shuffles + impulse-store fence'),
       (3, 'ws1 SolveTOI'), (4, 'ws1 stores'), (7, 'fence: ws1 stores complete'), (8, 'ws2 load'),
       (9, 'ws2 collide'), (10, 'ws2 island solve'), (13, 'ws2 body shuffles + impulse-store fence'),
       (11, 'ws2 SolveTOI'), (12, 'ws2 stores')]
POST = [(41, 'load groups + agent'), (42, 'box health + cameras'), (43, 'deaths, pickup, zone, rewards, stats'),
        (44, 'stores + auto-reset'), (45, 'obs rows')]
# (name, kid, base slot, [(slot, label)])
KERNELS = [
    ('k_pre_lanes', 1, 20, [(20, 'load groups + agent + actions'), (21, 'pend drop, motors, use, give'),
                            (22, 'melee rays + attacks'), (23, 'stores'), (24, 'fast physics (2 substeps)'),
                            (25, 'list appends')]),
    ('k_gen_solve_g (general-path list)', 0, 0, GEN),
    ('k_gen_solve_g (slow list, side stream)', 4, 0, GEN),
    ('k_post_lanes (all / main envs)', 2, 41, POST),
    ('k_post_lanes (slow list, side stream)', 5, 41, POST),
    ('k_obs', 3, 37, [(37, 'auto-reset'), (38, 'state load'), (39, 'row writer (windows)'), (40, 'tile stores')]),
]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    cfg_name = args[0] if len(args) > 0 else '2v2'
    n = int(args[1]) if len(args) > 1 else 65536
    steps = int(args[2]) if len(args) > 2 else 20
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS[cfg_name], n_envs=n, auto_reset=True)
    buf = (ctypes.c_ulonglong * PROF_WORDS)()
    gen_envs = 0
    if '--ppo' in sys.argv:
        from masurvival.ppo import PPOConfig, PPOTrainer
        tr = PPOTrainer(env, PPOConfig(), seed=0)
        for _ in range(2):
            tr.iteration()
        abi.check(lib.mas_prof_read(env._h, buf))
        for t in range(steps):
            tr.rollout_step(t)
            gen_envs += env.debug_counters()['phys_general_envs']
        regime = 'PPO regime (after 2 iterations)'
    else:
        env.reset()
        gen = torch.Generator(device=env.device)
        gen.manual_seed(0)
        hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
        acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
        for _ in range(150):
            env.step(acts())
        abi.check(lib.mas_prof_read(env._h, buf))
        for _ in range(steps):
            env.step(acts())
            gen_envs += env.debug_counters()['phys_general_envs']
        regime = 'random actions (after 150 steps)'
    torch.cuda.synchronize()
    abi.check(lib.mas_prof_read(env._h, buf))
    raw = np.frombuffer(buf, dtype=np.uint64)
    print(f'# {int(np.count_nonzero(raw))} nonzero words of {raw.size}')
    rec = raw[PROF_HEAD:].reshape(PROF_KERNELS, PROF_BLOCKS, 16).astype(np.float64)
    print(f'# env-step kernel phases, {cfg_name} N={n}, {regime}, {steps} steps; '
          f'general-path envs per step {gen_envs / steps:.0f}; mean per active wave (us)')
    for name, kid, base, marks in KERNELS:
        tot = rec[kid].sum(axis=0)
        waves = tot[15]
        if waves == 0:
            continue
        t = np.array([tot[s - base] for s, _ in marks]) * 0.01 / waves
        top = t.sum()
        print(f'{name}: {top:.1f} us per wave (span {tot[14] * 0.01 / waves:.1f}), {waves / steps:.0f} waves per step')
        for (s, label), v in zip(marks, t):
            print(f'  {label:44s} {v:9.2f} us  {100 * v / max(top, 1e-9):5.1f}%')


if __name__ == '__main__':
    main()
