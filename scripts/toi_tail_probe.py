"""Who makes the general path's tail?  In the PPO regime of the headline
bench (2 trainer iterations, then rollout steps of the trained policy) this
records per env and per step the SolveTOI events (mas_debug_set_toi_counter:
events + 65536 per agent that hit the sub-step cap) and prints, per step, the
env step time, the general-path env count and the event distribution, then
how persistent the high-event envs are from one step to the next (could the
previous step's count pick the envs whose chains bound the general kernels?).
usage: python scripts/toi_tail_probe.py [n_envs] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.config import NAMED_CONFIGS  # noqa: E402
from masurvival.ppo import PPOConfig, PPOTrainer  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(), seed=0)
    for _ in range(2):
        tr.iteration()
    cnt = torch.zeros((n,), dtype=torch.int32, device=env.device)
    env.set_toi_counter(cnt)
    hist = []
    T = tr.cfg.horizon
    for t in range(steps):
        cnt.zero_()
        e1, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        env_step = env.step

        def timed(a, out=None, _s=env_step):
            e1.record()
            r = _s(a, out=out)
            e2.record()
            return r
        env.step = timed
        tr.rollout_step(t % T)
        env.step = env_step
        torch.cuda.synchronize()
        ev = (cnt & 0xffff).cpu()
        cap = (cnt >> 16).cpu()
        g = env.debug_counters()['phys_general_envs']
        hist.append(ev)
        print(f't={t:3d} env step {e1.elapsed_time(e2):.3f} ms  general {g:6d}  events>=1 {(ev >= 1).sum():6d} '
              f'>=2 {(ev >= 2).sum():5d} >=4 {(ev >= 4).sum():4d} >=8 {(ev >= 8).sum():4d} >=16 {(ev >= 16).sum():3d} '
              f'capped {(cap > 0).sum():3d}  max {int(ev.max()):3d}', flush=True)
    env.set_toi_counter(None)
    for k in (2, 4, 8, 16):
        prec, rec = [], []
        for a, b in zip(hist, hist[1:]):
            pa, pb = a >= k, b >= k
            if pa.sum():
                prec.append(float((pa & pb).sum()) / float(pa.sum()))
            if pb.sum():
                rec.append(float((pa & pb).sum()) / float(pb.sum()))
        mp = sum(prec) / len(prec) if prec else float('nan')
        mr = sum(rec) / len(rec) if rec else float('nan')
        print(f'events >= {k:2d}: of the envs over it at step t, {mp:.2f} are over it at t+1; '
              f'of those over it at t+1, {mr:.2f} were at t')
    # the envs holding the per-step maximum: over it at the previous step?
    hit = 0
    for a, b in zip(hist, hist[1:]):
        j = int(torch.argmax(b))
        hit += int(a[j] >= 4)
    print(f'step maximum env had >= 4 events the step before: {hit} of {len(hist) - 1}')


if __name__ == '__main__':
    main()
