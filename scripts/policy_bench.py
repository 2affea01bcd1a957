"""Time the fused policy kernels alone (HIP events): mas_policy_act (fp32
rows) and mas_policy_act_x (bf16 rows) on the 2v2 rollout batch (65536 envs
x 4 agents) and mas_policy_train on one PPO
minibatch (16 steps x 262144 rows).  usage: policy_bench.py [lib.so ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival import abi  # noqa: E402


def run(lib_path):
    abi._lib = None
    lib = abi.load_library(lib_path)
    from masurvival import ppo
    ppo.load_library = lambda: lib
    D = 160
    pol = ppo.PolicyMLP(D, 256).cuda()
    fp = ppo.FusedPolicy(pol, D, torch.device('cuda'))
    fp.lib = lib
    fp.pack()
    M = 262144
    obs = torch.randn((M, D), device='cuda')
    xb = fp.x_buffer(M)
    a = torch.empty((M, 6), dtype=torch.int8, device='cuda')
    lp = torch.empty((M,), device='cuda')
    v = torch.empty((M,), device='cuda')
    for _ in range(5):
        fp.act(obs, 1, 0, a, lp, v, xb=xb)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(50):
        fp.act(obs, 1, i, a, lp, v, xb=xb)
    e1.record()
    torch.cuda.synchronize()
    t_act = e0.elapsed_time(e1) / 50
    # act_x: the rollout's path (bf16 rows mas_step_x wrote, nothing written back)
    for _ in range(5):
        fp.act_x(xb, 1, 0, a, lp, v)
    e0.record()
    for i in range(50):
        fp.act_x(xb, 1, i, a, lp, v)
    e1.record()
    torch.cuda.synchronize()
    t_actx = e0.elapsed_time(e1) / 50
    Mt = 16 * M
    xbt = fp.x_buffer(Mt)
    xbt[:, :D] = torch.randn((Mt, D), device='cuda').to(torch.bfloat16)
    at = torch.randint(0, 2, (Mt, 6), device='cuda', dtype=torch.int8)
    olp = torch.randn((Mt,), device='cuda') - 5
    adv = torch.randn((Mt,), device='cuda')
    ret = torch.randn((Mt,), device='cuda')
    cfg = ppo.PPOConfig()
    B = fp._buffers(Mt)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def train():
        abi.check(lib.mas_policy_train(ptr(fp.packed), D, Mt, ptr(xbt), fp.Dx, ptr(at), ptr(olp), ptr(adv), ptr(ret),
                                       0.2, 0.5, 0.01, 1.0 / Mt, ptr(B['h1']), ptr(B['h2']), ptr(B['da1']),
                                       ptr(B['da2']), ptr(B['dz']), ptr(B['part']), fp._stream()))
    train()
    fp.grads(xbt, at, olp, adv, ret, cfg)  # warm up the GEMM heuristics
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        train()
    e1.record()
    torch.cuda.synchronize()
    t_train = e0.elapsed_time(e1) / 5
    e0.record()
    for _ in range(5):
        fp.grads(xbt, at, olp, adv, ret, cfg)
    e1.record()
    torch.cuda.synchronize()
    t_grads = e0.elapsed_time(e1) / 5
    print(f'{os.path.basename(lib_path)}: act {t_act * 1e3:.1f} us, act_x {t_actx * 1e3:.1f} us (262144 rows), '
          f'train kernel {t_train:.3f} ms, '
          f'grads total {t_grads:.3f} ms ({Mt} rows)', flush=True)


if __name__ == '__main__':
    for p in sys.argv[1:] or [abi.LIB_PATH]:
        run(p)
