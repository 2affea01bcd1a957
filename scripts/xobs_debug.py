"""Where the x_obs trainer's bf16 rows differ from the fp32-obs trainer's
(debugging tool for tests/test_gpu_ppo.py::test_x_obs_trainer_matches_fp32_obs_trainer)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.config import C3_CONFIG  # noqa: E402
from masurvival.ppo import PPOConfig, PPOTrainer  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402

n, T = 2048, 8
trs = []
for xo in (False, True):
    env = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n), auto_reset=True)
    tr = PPOTrainer(env, PPOConfig(horizon=T, x_obs=xo), seed=0)
    trs.append(tr)
b1, b2 = trs[0].buf, trs[1].buf
print('init xb0 equal', torch.equal(b1.xb[0], b2.xb[0]), 'dtype', b1.xb.dtype, b1.xb.shape, b2.xb.shape)
for it in range(2):
    for t in range(T):
        for tr in trs:
            tr.rollout_step(t)
        torch.cuda.synchronize()
        x1, x2 = b1.xb[t], b2.xb[t]
        d = (x1.view(torch.int16) != x2.view(torch.int16))
        if bool(d.any()):
            idx = d.nonzero()
            cols = torch.unique(idx[:, 1]).tolist()
            rows = torch.unique(idx[:, 0])
            print(f'it {it} t {t}: {int(d.sum())} differing bf16 words, {len(rows)} rows, columns {cols[:40]}')
            for r, c in idx[:8].tolist():
                print('   row', r, 'col', c, 'fp32-path', float(x1[r, c]), hex(int(x1[r, c].view(torch.int16)) & 0xffff),
                      'x-path', float(x2[r, c]), hex(int(x2[r, c].view(torch.int16)) & 0xffff))
        if t == 0 and it == 0:
            print('obs0 rows equal:', torch.equal(b1.xb[0], b2.xb[0]))
    for tr in trs:
        tr.finish_rollout()
        tr.update()
    torch.cuda.synchronize()
    print('after update', it, 'params equal', all(torch.equal(p, q) for p, q in zip(trs[0].policy.parameters(),
                                                                                  trs[1].policy.parameters())))
