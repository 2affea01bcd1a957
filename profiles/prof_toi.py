"""Per-step SolveTOI work in the PPO regime (profiling build libmas_prof.so):
for each env step, the largest number of TOI events / b2TimeOfImpact calls /
TOI position iterations any (env, agent) lane ran in one k_gen_toi launch
(max over the step's two world steps), the event and call totals, and the
step's duration, and the largest per-lane time in each SolveTOI phase.  Explains the k_gen_toi launches that take ~10x the median.
usage: python profiles/prof_toi.py [n_envs] [iterations]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import torch  # noqa: E402

from masurvival import abi  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    lib = abi.load_library(os.path.join(os.path.dirname(abi.LIB_PATH), 'libmas_prof.so'))
    lib.mas_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    from masurvival.config import NAMED_CONFIGS
    from masurvival.ppo import PPOConfig, PPOTrainer
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(), seed=0)
    buf = (ctypes.c_ulonglong * 64)()
    env_step = env.step
    for it in range(iters):
        rows = []
        for t in range(tr.cfg.horizon):
            abi.check(lib.mas_prof_read(env._h, buf))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

            def timed(a, out=None):
                e0.record()
                r = env_step(a, out=out)
                e1.record()
                return r
            env.step = timed
            tr.rollout_step(t)
            env.step = env_step
            torch.cuda.synchronize()
            abi.check(lib.mas_prof_read(env._h, buf))
            rows.append((e0.elapsed_time(e1), buf[48], buf[49], buf[50], buf[51], buf[52],
                         env.debug_counters()['phys_general_envs'], [buf[53 + k] * 0.01 for k in range(5)]))
        tr.finish_rollout()
        tr.update()
        ms = [r[0] for r in rows]
        print(f'iter {it}: env step mean {sum(ms) / len(ms):.3f} ms, max {max(ms):.3f} ms', flush=True)
        for t, r in enumerate(rows):
            if r[0] > 1.5 * sorted(ms)[len(ms) // 2] or t % 16 == 0:
                print(f'  t={t:2d} {r[0]:.3f} ms  lane max: events {r[1]} toi calls {r[2]} pos iters {r[3]};'
                      f'  totals: events {r[4]} toi calls {r[5]}; general envs {r[6]}; lane max us: '
                      f'toi {r[7][0]:.1f} min+collide+gather {r[7][1]:.1f} position {r[7][2]:.1f} velocity {r[7][3]:.1f} integrate {r[7][4]:.1f}', flush=True)


if __name__ == '__main__':
    main()
