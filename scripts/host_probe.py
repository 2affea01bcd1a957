"""Host-submission probe: is the env step / rollout step bound by the host's
launch rate or by the GPU?  Prints, per mode, the host time to enqueue one
step (no sync), the wall time per step, and the wall time per step when the
env step is replayed from a captured HIP graph."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gym-ma-survival-2d_amd'))
import torch  # noqa: E402

from masurvival.config import NAMED_CONFIGS  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


def main():
    n = 65536
    env = VecMaSurvival(NAMED_CONFIGS['2v2'], n_envs=n, seeds=range(n), auto_reset=True)
    env.reset()
    dev = env.device
    acts = torch.randint(0, 2, (n, env.n_agents, 6), dtype=torch.int8, device=dev)
    for _ in range(20):
        env.step(acts)
    torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        env.step(acts)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'env eager: host enqueue {1e6 * (t1 - t0) / K:.1f} us/step, wall {1e6 * (t2 - t0) / K:.1f} us/step')

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        env.step(acts)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        env.step(acts)
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'env graph: host enqueue {1e6 * (t1 - t0) / K:.1f} us/step, wall {1e6 * (t2 - t0) / K:.1f} us/step')

    from masurvival.ppo import PPOConfig, PPOTrainer
    tr = PPOTrainer(env, PPOConfig(horizon=64), seed=0)
    for t in range(8):
        tr.rollout_step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(8, 64):
        tr.rollout_step(t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'ppo rollout: host enqueue {1e6 * (t1 - t0) / 56:.1f} us/step, wall {1e6 * (t2 - t0) / 56:.1f} us/step')
    t0 = time.perf_counter()
    tr.finish_rollout()
    tr.update()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'ppo finish+update (first): host {1e3 * (t1 - t0):.2f} ms, wall {1e3 * (t2 - t0):.2f} ms')
    for t in range(64):
        tr.rollout_step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.finish_rollout()
    tr.update()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'ppo finish+update: host {1e3 * (t1 - t0):.2f} ms, wall {1e3 * (t2 - t0):.2f} ms')


if __name__ == '__main__':
    main()
