"""Do independent env shards on separate HIP streams overlap?  Times the 2v2
env step (random actions, then policy act + env step as in the rollout) for
65536 envs as 1 handle, 2 handles x 32768 and 4 x 16384, each shard on its
own stream.  usage: python scripts/stream_probe.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.config import NAMED_CONFIGS  # noqa: E402
from masurvival.ppo import FusedPolicy, PolicyMLP  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


def run(k, steps, with_policy, warm=150):
    n = 65536 // k
    envs = [VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, seeds=range(j * n, (j + 1) * n), auto_reset=True)
            for j in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    A, D = envs[0].n_agents, envs[0].obs_dim
    dev = envs[0].device
    pol = PolicyMLP(D, 256).to(dev)
    fp = FusedPolicy(pol, D, dev)
    fp.pack()
    obs = [torch.zeros((n * A, D), device=dev) for _ in range(k)]
    acts = [torch.randint(0, 2, (n * A, 6), dtype=torch.int8, device=dev) for _ in range(k)]
    lp = [torch.empty(n * A, device=dev) for _ in range(k)]
    v = [torch.empty(n * A, device=dev) for _ in range(k)]
    rew = [torch.empty((n, A), device=dev) for _ in range(k)]
    done = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(k)]
    hi = torch.tensor([3, 3, 3, 2, 2, 2], device=dev)
    gens = [torch.Generator(device=dev) for _ in range(k)]
    for j, g in enumerate(gens):
        g.manual_seed(1234 + j)
    torch.cuda.synchronize()

    # the bench's env-mode workload in every variant: uniform random actions
    # drawn per step (the policy's actions, when timed, are overwritten)
    def step(t):
        for j in range(k):
            with torch.cuda.stream(streams[j]):
                if with_policy:
                    fp.act(obs[j], 1, t, acts[j], lp[j], v[j])
                u = torch.rand((n * A, 6), generator=gens[j], device=dev)
                acts[j].copy_((u * hi).to(torch.int8))
                envs[j].step(acts[j].view(n, A, 6), out=(obs[j].view(n, A, D), rew[j], done[j]))
    for t in range(warm):
        step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        step(warm + t)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    for e in envs:
        e.close()
    return dt * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    for with_policy in (False, True):
        for k in (1, 2, 4):
            ms = run(k, steps, with_policy)
            print(f'{"act+env" if with_policy else "env"} shards={k}: {ms:.3f} ms/step', flush=True)


if __name__ == '__main__':
    main()
