"""Feature-major ('fm') against row-major ('rm') update activations on one
4.2M-row PPO minibatch (2v2, D = 160): the train kernel alone, each
weight-gradient GEMM, and FusedPolicy.grads end to end (HIP events), plus the
largest relative difference between the two layouts' gradients.
usage: python scripts/policy_layout_probe.py [reps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival import abi, ppo  # noqa: E402


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.manual_seed(0)
    D, Mt = 160, 16 * 262144
    pol = ppo.PolicyMLP(D, 256).cuda()
    cfg = ppo.PPOConfig()
    fps = {}
    for lay in ('fm', 'rm'):
        ppo._POL_LAYOUT = lay
        fps[lay] = ppo.FusedPolicy(pol, D, torch.device('cuda'))
        fps[lay].pack()
    fp = fps['fm']
    xbt = fp.x_buffer(Mt)
    xbt[:, :D] = (0.5 * torch.randn((Mt, D), device='cuda')).to(torch.bfloat16)
    at = torch.randint(0, 2, (Mt, 6), device='cuda', dtype=torch.int8)
    olp = torch.randn((Mt,), device='cuda') - 5
    adv = torch.randn((Mt,), device='cuda')
    ret = torch.randn((Mt,), device='cuda')
    lib = fp.lib
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    grads = {}
    for lay, f in fps.items():
        t_grads = timed(lambda: f.grads(xbt, at, olp, adv, ret, cfg), reps)
        grads[lay] = [p.grad.detach().clone() for p in pol.parameters()]
        B = f._bufs
        if lay == 'fm':
            def train():
                abi.check(lib.mas_policy_train_ld(ptr(f.packed), D, Mt, ptr(xbt), f.Dx, ptr(at), ptr(olp), ptr(adv),
                                                  ptr(ret), 0.2, 0.5, 0.01, 1.0 / Mt, ptr(B['h1']), ptr(B['h2']),
                                                  ptr(B['da1']), ptr(B['da2']), ptr(B['dz']), B['ld'],
                                                  ptr(B['part']), f._stream()))
            Bv = {k: (v[:, :Mt] if k in ('h1', 'h2', 'da1', 'da2', 'dz') else v) for k, v in B.items()}
            gemms = {'dW3': lambda: f._dw(Bv['dz'], Bv['h2'], 16, Mt),
                     'dW2': lambda: f._dw(Bv['da2'], Bv['h1'], 256, Mt),
                     'dW1': lambda: ppo._splitk_nn(Bv['da1'], xbt[:, :D + 1])}
        else:
            def train():
                abi.check(lib.mas_policy_train_rm(ptr(f.packed), D, Mt, ptr(xbt), f.Dx, ptr(at), ptr(olp), ptr(adv),
                                                  ptr(ret), 0.2, 0.5, 0.01, 1.0 / Mt, ptr(B['h1']), ptr(B['h2']),
                                                  ppo._RM_LDH, ptr(B['da1']), ptr(B['da2']), ptr(B['dz']),
                                                  ptr(B['part']), f._stream()))
            gemms = {'dW3': lambda: ppo._splitk_tn(B['dz'], B['h2'][:, :257]),
                     'dW2': lambda: ppo._splitk_tn(B['da2'], B['h1'][:, :257]),
                     'dW1': lambda: ppo._splitk_tn(B['da1'], xbt[:, :D + 1])}
        t_train = timed(train, reps)
        parts = ', '.join(f'{k} {timed(g, reps):.3f}' for k, g in gemms.items())
        print(f'{lay}: train kernel {t_train:.3f} ms, {parts} ms, grads total {t_grads:.3f} ms ({Mt} rows)',
              flush=True)
        f._bufs = None
        torch.cuda.empty_cache()
    worst = 0.0
    for a, b in zip(grads['fm'], grads['rm']):
        worst = max(worst, float((a - b).norm() / a.norm().clamp_min(1e-30)))
    cos = [float(torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0))
           for a, b in zip(grads['fm'], grads['rm'])]
    print(f'fm vs rm gradients: max relative L2 difference {worst:.2e}, cosines {[round(c, 6) for c in cos]}')


if __name__ == '__main__':
    main()
