"""Time the pieces of one PPO rollout step and of the update separately
(HIP events on the current stream): policy forward + sample, env step,
finish_rollout (GAE), update.  usage: python scripts/ppo_breakdown.py [n_envs] [iterations]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.config import NAMED_CONFIGS  # noqa: E402
from masurvival.ppo import PPOConfig, PPOTrainer  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(), seed=0)
    T = tr.cfg.horizon
    env_step = env.step
    marks = []

    def timed_step(a, out=None):
        e1 = ev()
        e1.record()
        r = env_step(a, out=out)
        e2 = ev()
        e2.record()
        marks.append((e1, e2))
        return r
    env.step = timed_step
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for it in range(iters):
        marks.clear()
        e0 = ev(); e0.record()
        starts = []
        for t in range(T):
            s = ev(); s.record(); starts.append(s)
            tr.rollout_step(t)
        e_roll = ev(); e_roll.record()
        tr.finish_rollout()
        e_fin = ev(); e_fin.record()
        tr.update()
        e_upd = ev(); e_upd.record()
        torch.cuda.synchronize()
        env_ms = sum(a.elapsed_time(b) for a, b in marks)
        pol_ms = sum(s.elapsed_time(m[0]) for s, m in zip(starts, marks))
        print(f'iter {it}: rollout {e0.elapsed_time(e_roll):.2f} ms (policy fwd+sample {pol_ms:.2f}, env {env_ms:.2f}), '
              f'finish {e_roll.elapsed_time(e_fin):.2f} ms, update {e_fin.elapsed_time(e_upd):.2f} ms; '
              f'per step: policy {pol_ms / T:.3f} env {env_ms / T:.3f} update+finish '
              f'{e_roll.elapsed_time(e_upd) / T:.3f} ms; env step max {max(a.elapsed_time(b) for a, b in marks):.3f} ms, '
              f'general envs {env.debug_counters()["phys_general_envs"]}', flush=True)


if __name__ == '__main__':
    main()
