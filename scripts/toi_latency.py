"""Serial latency of the general physics path on ONE env: replays the
PPO-regime env whose SolveTOI reaches the sub-step cap (profiles/
r02_wedged_env.npz, dumped by tests/test_gpu_parity_regimes.py) with n_envs=1,
so every kernel runs a single env and the step time is the env's own
dependent chain -- the tail that sets k_gen_toi's duration at 65536 envs.
Prints the per-step time of mas_step (HIP events), the steps above 2x the
median, and their sum.  A/B: --lib path/to/libmas_<variant>.so.
usage: python scripts/toi_latency.py [--lib LIB] [--reps R]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=None)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--data', default=os.path.join(ROOT, 'profiles', 'r02_wedged_env.npz'))
    a = ap.parse_args()
    from masurvival import abi
    if a.lib:
        abi.load_library(a.lib)
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    d = np.load(a.data)
    acts = torch.as_tensor(d['actions'], device='cuda').unsqueeze(1)  # [T, 1, A, 6]
    T = acts.shape[0]
    best = None
    for rep in range(a.reps):
        env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=1, seeds=[int(d['env_seed'])], auto_reset=True)
        env.reset()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(T)]
        dones = []
        for t in range(T):
            ev[t][0].record()
            _, _, dn, _ = env.step(acts[t])
            ev[t][1].record()
            dones.append(dn)
        torch.cuda.synchronize()
        ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
        dn = torch.stack(dones).cpu().numpy().reshape(-1)
        assert np.array_equal(dn, d['dones']), 'replay diverged from the recorded episode'
        env.close()
        best = ms if best is None else np.minimum(best, ms)
    med = float(np.median(best))
    slow = np.nonzero(best > 2 * med)[0]
    print(f'steps {T}: median {med * 1e3:.1f} us, mean {best.mean() * 1e3:.1f} us, total {best.sum():.2f} ms; '
          f'{len(slow)} steps > 2x median, sum {best[slow].sum():.2f} ms, max {best.max() * 1e3:.1f} us')
    print('slow steps:', ' '.join(f'{t}:{best[t] * 1e3:.0f}' for t in slow[:40]))


if __name__ == '__main__':
    main()
