"""Headline benchmark: agent-env-steps/sec for the 2v2 config.

A "step" is one rollout step of every env on this rank, all in HBM: the
shared policy MLP's forward on the current observations (bf16 autocast),
Gumbel-max sampling of the six action heads, the batched MaSurvival.step (the
HIP k_step kernel: actions -> 2 Box2D steps -> rules -> obs/rewards/done with
auto-reset, writing straight into the rollout buffer), and -- every
--horizon steps -- the GAE scan (HIP mas_gae) plus one PPO update (1 epoch,
4 minibatches, gradient all-reduce across ranks).  --mode env times the env
kernel alone under a device-RNG random policy.

Run: python bench.py [--gpus N --steps K --warmup W --config 2v2 --envs N_per_gpu]
For N>1 the driver launches one rank per GPU with torch.distributed.run; envs
shard with no data-path collective (weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def algorithmic_bytes_per_env_step(A, H, B, D):
    """Bstep = 8*S + 6A + 4*A*D + 4A + 1 with
    S = 27A + 14B + 3H + 17 + 2*(A(A-1)/2 + A(B+4)) + 4 persistent words."""
    S = 27 * A + 14 * B + 3 * H + 17 + 2 * (A * (A - 1) // 2 + A * (B + 4)) + 4
    return 8 * S + 6 * A + 4 * A * D + 4 * A + 1


def cpu_baseline(cfg, budget_s=12.0):
    """The C oracle (scalar restatement, 1 thread) on a bounded sample: round-robin
    over 64 envs of the same config with uniform random actions, until budget_s."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    from oracle import OracleEnv
    from masurvival.config import ResolvedConfig, pcg64_state
    rc = ResolvedConfig(cfg)
    n = 64
    envs = [OracleEnv(rc.to_struct(), pcg64_state(s)) for s in range(n)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(1)
    acts = rng.integers(0, [3, 3, 3, 2, 2, 2], size=(256, n, rc.n_agents, 6)).astype(np.int8)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        a = acts[(steps // n) % 256]
        for i, e in enumerate(envs):
            _, _, d = e.step(a[i])
            if d:
                e.reset()
        steps += n
    dt = time.perf_counter() - t0
    return {'value': steps * rc.n_agents / dt, 'unit': 'agent-env-steps/s', 'cores': 1, 'kind': 'port',
            'sample': f'{steps} env-steps ({n} envs round-robin, random actions, auto-reset) of the C oracle, '
                      f'1 thread, {dt:.1f}s incl. ctypes per-step call overhead'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=128, help='timed rollout steps (multiple of --horizon amortises the update)')
    ap.add_argument('--warmup', type=int, default=64)
    ap.add_argument('--config', default='2v2')
    ap.add_argument('--envs', type=int, default=None, help='envs per GPU (default 65536 for 2v2)')
    ap.add_argument('--mode', choices=['ppo', 'env'], default='ppo',
                    help='ppo: policy forward + env step + buffer, GAE + PPO update every horizon; env: random actions')
    ap.add_argument('--horizon', type=int, default=64)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--lib', default=None, help='alternative libmas*.so (A/B variants)')
    ap.add_argument('--shards', type=int, default=1,
                    help='env handles per GPU, each on its own HIP stream (vec_env.ShardedVecMaSurvival)')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # MAS_DIST_BACKEND=gloo and several ranks per GPU (local % devices) only
    # to rehearse the multi-rank path on a one-GPU box; the real run is RCCL
    backend = os.environ.get('MAS_DIST_BACKEND', 'nccl')
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)

    if args.lib:
        from masurvival import abi
        abi.load_library(args.lib)
    from masurvival.config import NAMED_CONFIGS
    from masurvival.vec_env import VecMaSurvival
    cfg = NAMED_CONFIGS[args.config]
    n = args.envs or {'1v1': 4096, '2v2': 65536, 'ffa4': 16384}[args.config]
    if args.shards > 1:
        from masurvival.vec_env import ShardedVecMaSurvival
        env = ShardedVecMaSurvival(cfg, n_envs=n, shards=args.shards, seeds=range(rank * n, rank * n + n),
                                   auto_reset=True)
    else:
        env = VecMaSurvival(cfg, n_envs=n, seeds=range(rank * n, rank * n + n), auto_reset=True)
    A, D = env.n_agents, env.obs_dim
    dev = env.device
    # the env kernel's launch duration, HIP events on the stream it runs on
    kev = []
    if args.shards > 1:
        # one mas_step launch group per shard, timed on the shard's stream
        for sub in env.envs:
            def timed_shard_step(a, out=None, _step=sub.step):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = _step(a, out=out)
                e1.record()
                kev.append((e0, e1))
                return r
            sub.step = timed_shard_step

    if args.mode == 'ppo':
        from masurvival.ppo import PPOConfig, PPOTrainer
        pcfg = PPOConfig(horizon=args.horizon)
        tr = PPOTrainer(env, pcfg, seed=0)
        env_step = env.step

        def timed_env_step(a, out=None):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = env_step(a, out=out)
            e1.record()
            kev.append((e0, e1))
            return r
        if args.shards == 1:
            env.step = timed_env_step
        state = {'t': 0, 'updates': 0}

        def one_step():
            tr.rollout_step(state['t'])
            state['t'] += 1
            if state['t'] == pcfg.horizon:
                tr.finish_rollout()
                tr.update()
                state['t'] = 0
                state['updates'] += 1
    else:
        env.reset()
        hi = torch.tensor([3, 3, 3, 2, 2, 2], device=dev, dtype=torch.int32)
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        acts = torch.empty((n, A, 6), dtype=torch.int8, device=dev)

        def one_step():
            u = torch.rand((n, A, 6), generator=gen, device=dev)
            acts.copy_((u * hi).to(torch.int8))
            if args.shards > 1:
                env.step(acts)
                return
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            env.step(acts)
            e1.record()
            kev.append((e0, e1))

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    kev.clear()
    if args.mode == 'ppo':
        state['updates'] = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    if world > 1:
        t = torch.tensor([dt, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kern_ms = float(t[0]), float(t[1])

    diag = env.debug_counters()
    total_agent_steps = world * n * A * args.steps
    b_env = algorithmic_bytes_per_env_step(A, env.rc.n_heals, env.rc.n_boxes, D)
    n_launch = n // args.shards  # envs per mas_step launch group (per shard when sharded)
    achieved = b_env * n_launch / (kern_ms * 1e-3) / 1e9
    workload = (f'{args.config} PPO rollout (policy MLP 2x256 bf16 fwd + sample + env step + buffer), '
                f'GAE + PPO update (1 epoch, 4 minibatches) every {args.horizon} steps'
                if args.mode == 'ppo' else f'{args.config} env step, random policy')
    line = {
        'metric': 'agent-env-steps/sec (whole node), %s N_envs=%d' % (args.config, n * world),
        'value': total_agent_steps / dt,
        'unit': 'agent-env-steps/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': dt * 1e3 / args.steps,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'f32', 'data': 'synthetic (seeded envs, on-device policy sampling)',
        'config': {'workload': workload, 'n_envs_per_gpu': n, 'n_agents': A, 'obs_dim': D,
                   'horizon': args.horizon if args.mode == 'ppo' else None,
                   'updates_in_timed_region': state['updates'] if args.mode == 'ppo' else 0,
                   'parallelism': f'env-shard x{world}',
                   'streams_per_gpu': args.shards,
                   'phys_general_envs_last_step': diag['phys_general_envs']},
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                     'kernel': 'k_step (mas_step)' if args.shards == 1 else
                     f'k_step (mas_step of one shard, {args.shards} shards on concurrent streams)',
                     'kernel_ms': kern_ms, 'bytes_per_env_step': b_env,
                     'bytes_per_launch': b_env * n_launch},
        'cpu_baseline': None,
    }
    # HBM traffic per mas_step from the committed rocprofv3 PMC passes of this
    # workload (profiles/pmc_traffic.py); null when none matches
    tname = 'r01_pmc_traffic.json' if args.mode == 'env' else 'r01_pmc_traffic_ppo.json'
    tpath = os.path.join(ROOT, 'profiles', tname)
    if os.path.exists(tpath):
        tr_ = json.load(open(tpath))
        if tr_.get('workload') == f'{args.config}:{n}' + ('' if args.mode == 'env' else ':ppo'):
            line['roofline']['traffic'] = tr_['traffic_bytes_per_step'] * n_launch / n
            line['roofline']['traffic_source'] = f'profiles/{tname} (FETCH_SIZE+WRITE_SIZE per mas_step)'
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline(cfg)
    if rank == 0:
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
