"""A/B of the act kernel's head sampling (MAS_ACT_SPLIT, read per call by
mas_policy_act_x): 1 = both half-waves (default), 0 = one; the 2v2 rollout
batch (262144 bf16 rows), alternating blocks of 50 launches, HIP events.
usage: python scripts/act_split_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival import ppo  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    D, M = 160, 262144
    pol = ppo.PolicyMLP(D, 256).cuda()
    fp = ppo.FusedPolicy(pol, D, torch.device('cuda'))
    fp.pack()
    xb = fp.x_buffer(M)
    xb[:, :D] = torch.randn((M, D), device='cuda').to(torch.bfloat16)
    a = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), device='cuda')
    v = torch.empty((M,), device='cuda')
    res = {'1': [], '0': []}
    for r in range(rounds):
        for sv in ('1', '0'):
            os.environ['MAS_ACT_SPLIT'] = sv
            for i in range(5):
                fp.act_x(xb, 1, i, a, lp, v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(50):
                fp.act_x(xb, 1, i, a, lp, v)
            e1.record()
            torch.cuda.synchronize()
            res[sv].append(e0.elapsed_time(e1) / 50 * 1e3)
    for sv in ('1', '0'):
        print(f'MAS_ACT_SPLIT={sv}: act_x ' + ' '.join(f'{t:.1f}' for t in res[sv]) + ' us', flush=True)


if __name__ == '__main__':
    main()
