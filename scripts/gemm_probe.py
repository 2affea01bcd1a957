"""Operand order / width variants of the PPO weight-gradient GEMMs
(masurvival/ppo.py FusedPolicy.grads) at the headline minibatch size:
K = 4194304 rows, split-K batched over 64 chunks.  Prints ms per GEMM.
usage: python scripts/gemm_probe.py"""
import torch


def bench(fn, n=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    K, c, D, Dx = 4194304, 64, 160, 176
    bf = dict(device='cuda', dtype=torch.bfloat16)
    da2 = torch.randn((256, K), **bf)
    h1 = torch.randn((257, K), **bf)
    dz = torch.randn((16, K), **bf)
    da1 = torch.randn((256, K), **bf)
    xb = torch.randn((K, Dx), **bf)

    def nt(a, b):  # a [F, K] @ b [G, K]^T
        pa = a.view(a.shape[0], c, K // c).permute(1, 0, 2)
        pb = b.view(b.shape[0], c, K // c).permute(1, 2, 0)
        return torch.bmm(pa, pb).sum(0, dtype=torch.float32)

    def nt_swapped(a, b):  # (b a^T)^T
        pb = b.view(b.shape[0], c, K // c).permute(1, 0, 2)
        pa = a.view(a.shape[0], c, K // c).permute(1, 2, 0)
        return torch.bmm(pb, pa).sum(0, dtype=torch.float32).t()

    def nn(a, x):  # a [F, K] @ x [K, G]
        pa = a.view(a.shape[0], c, K // c).permute(1, 0, 2)
        px = x.unflatten(0, (c, K // c))
        return torch.bmm(pa, px).sum(0, dtype=torch.float32)

    def nn_swapped(a, x):  # (x^T a^T)^T
        pa = a.view(a.shape[0], c, K // c).permute(1, 2, 0)
        px = x.unflatten(0, (c, K // c)).transpose(1, 2)
        return torch.bmm(px, pa).sum(0, dtype=torch.float32).t()

    rows = [
        ('g2 da2 h1^T (N=257)', lambda: nt(da2, h1)),
        ('g2 swapped', lambda: nt_swapped(da2, h1)),
        ('g2 N=256 (no bias row)', lambda: nt(da2, h1[:256])),
        ('g3 dz h2^T', lambda: nt(dz, h1)),
        ('g3 swapped', lambda: nt_swapped(dz, h1)),
        ('g1 da1 x (N=161)', lambda: nn(da1, xb[:, :D + 1])),
        ('g1 N=176 (full rows)', lambda: nn(da1, xb)),
        ('g1 swapped (N=161)', lambda: nn_swapped(da1, xb[:, :D + 1])),
        ('g1 swapped full', lambda: nn_swapped(da1, xb)),
    ]
    for name, fn in rows:
        print(f'{name:28s} {bench(fn):.3f} ms', flush=True)

    # the three GEMMs of one minibatch back to back vs on three streams
    streams = [torch.cuda.Stream() for _ in range(3)]
    jobs = [lambda: nt(dz, h1), lambda: nt(da2, h1), lambda: nn(da1, xb[:, :D + 1])]

    def serial():
        for j in jobs:
            j()

    def concurrent():
        cur = torch.cuda.current_stream()
        for s_, j in zip(streams, jobs):
            s_.wait_stream(cur)
            with torch.cuda.stream(s_):
                j()
        for s_ in streams:
            cur.wait_stream(s_)
    print(f'{"g3+g2+g1 serial":28s} {bench(serial):.3f} ms', flush=True)
    print(f'{"g3+g2+g1 on 3 streams":28s} {bench(concurrent):.3f} ms', flush=True)


if __name__ == '__main__':
    main()
