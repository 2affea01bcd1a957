"""Per-phase wave time of the env-step kernels from the profiling build
(libmas_prof.so, `make -C gym-ma-survival-2d_amd/csrc prof`; MAS_PROFILE marks,
mas_env.h).  Each wave accumulates the 100 MHz constant-clock time between
marks in LDS and adds it to its own record at its end (plain stores, no
atomics); printed: the mean per ACTIVE wave (us) of each phase, its share,
and the mean wave span, per kernel, over `steps` steps.
Regimes: --ppo (2 PPO iterations of pre-roll, then rollout steps of the
trained policy: the headline bench's regime) or random actions after 150
steps (default).
With --waves: the records are read (and zeroed) after every step, so
each active wave's own span is known; printed per kernel: the span
percentiles per step (the launch lasts as long as its slowest wave) and the
phases of the slowest 1 % of waves beside the mean.
usage: python profiles/prof_env.py [config] [n_envs] [steps] [--ppo] [--waves]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from masurvival import abi  # noqa: E402

PROF_HEAD, PROF_KERNELS, PROF_BLOCKS = 64, 7, 16384  # mas_env.h kProfHead / kProfKernels / kProfBlocks
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
    ('k_obs (over a list)', 6, 37, [(37, 'auto-reset'), (38, 'state load'), (39, 'row writer (windows)'),
                                    (40, 'tile stores')]),
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
    per_step = []  # --waves: each step's records (differenced)
    prev = [None]
    total = [None]

    def snap():
        if '--waves' not in sys.argv:
            return
        torch.cuda.synchronize()
        abi.check(lib.mas_prof_read(env._h, buf))
        # (mas_prof_read returns the records since the last read and zeroes them)
        cur = np.frombuffer(buf, dtype=np.uint64).copy()
        if prev[0] is not None:
            per_step.append(cur[PROF_HEAD:].astype(np.float64).reshape(PROF_KERNELS, PROF_BLOCKS, 16))
            total[0] = cur if total[0] is None else total[0] + cur
        prev[0] = cur
    if '--ppo' in sys.argv:
        from masurvival.ppo import PPOConfig, PPOTrainer
        tr = PPOTrainer(env, PPOConfig(), seed=0)
        for _ in range(2):
            tr.iteration()
        snap()
        abi.check(lib.mas_prof_read(env._h, buf))
        for t in range(steps):
            tr.rollout_step(t)
            gen_envs += env.debug_counters()['phys_general_envs']
            snap()
        regime = 'PPO regime (after 2 iterations)'
    else:
        env.reset()
        gen = torch.Generator(device=env.device)
        gen.manual_seed(0)
        hi = torch.tensor([3, 3, 3, 2, 2, 2], device=env.device)
        acts = lambda: (torch.rand((n, env.n_agents, 6), generator=gen, device=env.device) * hi).to(torch.int8)  # noqa
        for _ in range(150):
            env.step(acts())
        snap()
        abi.check(lib.mas_prof_read(env._h, buf))
        for _ in range(steps):
            env.step(acts())
            gen_envs += env.debug_counters()['phys_general_envs']
            snap()
        regime = 'random actions (after 150 steps)'
    torch.cuda.synchronize()
    abi.check(lib.mas_prof_read(env._h, buf))
    raw = np.frombuffer(buf, dtype=np.uint64) if total[0] is None else total[0]
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
        if per_step:
            waves_report(per_step, kid, base, marks)


def waves_report(per_step, kid, base, marks):
    """Span percentiles of the active waves of each step, and the phases of
    the slowest 1 % of all waves against the mean of all."""
    pct = []
    rows = []
    for r in per_step:
        k = r[kid]
        act = k[:, 15] > 0
        if not act.any():
            continue
        sp = k[act, 14] * 0.01
        pct.append(np.percentile(sp, [50, 90, 99, 100]))
        rows.append(k[act])
    if not pct:
        return
    pct = np.array(pct).mean(axis=0)
    allw = np.concatenate(rows)
    sp = allw[:, 14]
    top = allw[sp >= np.percentile(sp, 99)]
    print(f'  waves per step: span p50 {pct[0]:.1f}, p90 {pct[1]:.1f}, p99 {pct[2]:.1f}, max {pct[3]:.1f} us '
          f'(mean over {len(per_step)} steps)')
    print(f'  {"phase (us per wave)":44s} {"all":>9s} {"slowest 1%":>11s}')
    for s, label in marks:
        print(f'  {label:44s} {allw[:, s - base].mean() * 0.01:9.2f} {top[:, s - base].mean() * 0.01:11.2f}')


if __name__ == '__main__':
    main()
