"""GAE kernel time (mas_gae) at the bench's rollout shape: T=64, 65536 envs x 4 agents."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.ppo import gae, gae_scratch  # noqa: E402

T, N, A = 64, 65536, 4
g = torch.Generator(device='cuda').manual_seed(0)
r = torch.randn((T, N, A), device='cuda', generator=g)
v = torch.randn((T + 1, N, A), device='cuda', generator=g)
d = (torch.rand((T, N), device='cuda', generator=g) < 0.05).to(torch.uint8)
adv, ret = torch.empty_like(r), torch.empty_like(r)
sums = torch.empty(2, device='cuda', dtype=torch.float64)
sc = gae_scratch(N * A, 'cuda')
for _ in range(3):
    gae(r, v, d, 0.99, 0.95, adv, ret, sums, A, scratch=sc)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    gae(r, v, d, 0.99, 0.95, adv, ret, sums, A, scratch=sc)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / 20
nbytes = (3 * T + 1) * N * A * 4 + T * N
print(f'mas_gae T={T} N={N} A={A}: {us:.1f} us per call, {nbytes / us / 1e6:.2f} TB/s over {nbytes / 1e6:.0f} MB')
