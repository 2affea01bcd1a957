"""Headline benchmark: agent-env-steps/sec for the 2v2 config.

A "step" is one rollout step of every env on this rank, all in HBM: the
fused policy kernel (MLP forward, bf16 MFMA with fp32 accumulation, plus
Gumbel-max sampling of the six action heads: mas_policy_act), the batched
MaSurvival.step (the HIP env kernels: actions -> 2 Box2D steps -> rules ->
obs/rewards/done with auto-reset, written straight into the rollout buffer),
and -- every --horizon steps -- the GAE scan (HIP mas_gae) plus one PPO update
(1 epoch, 4 minibatches, gradient all-reduce across ranks).

The timed window holds the work the metric names:
  * an untimed pre-roll of --preroll full PPO iterations first puts the envs
    and the policy in the training regime (general-path physics, contacts,
    TOI), not the episode-start regime;
  * after --warmup untimed steps, `align_steps` more untimed steps make the
    K timed steps END on a horizon boundary, so the window contains
    ceil(K / horizon) GAE + PPO updates (a short window is therefore
    pessimistic: it carries a whole update for fewer rollout steps).
--mode env times the env kernels alone under a device-RNG random policy.

Run: python bench.py [--gpus N --steps K --warmup W --config 2v2 --envs N_per_gpu]
--gpus N > 1 without a torch.distributed launcher: bench.py starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child
process (before touching the GPU), relays rank 0's JSON line and exits with
the child's return code.  Envs shard with no data-path collective (weak
scaling); n_gpus is the real world size.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
ENVS_DEFAULT = {'1v1': 4096, '2v2': 65536, 'ffa4': 16384}


def algorithmic_bytes_per_env_step(A, H, B, D, obs_bytes=4):
    """Bstep = 8*S + 6A + 4*A*D + 4A + 1 with
    S = 27A + 14B + 3H + 17 + 2*(A(A-1)/2 + A(B+4)) + 4 persistent words;
    obs_bytes = 2 when the step writes bf16 policy rows (mas_step_x: 2*A*D)."""
    S = 27 * A + 14 * B + 3 * H + 17 + 2 * (A * (A - 1) // 2 + A * (B + 4)) + 4
    return 8 * S + 6 * A + obs_bytes * A * D + 4 * A + 1


def cpu_info():
    model = '?'
    try:
        out = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        model = next((ln.split(':', 1)[1].strip() for ln in out.splitlines() if ln.startswith('Model name')), '?')
    except Exception:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count() or 1
    return model, avail


def cpu_baseline(config, leg_s=6.0, all_cores=False):
    """The C oracle (scalar restatement, oracle/ora_bench.c: the whole loop in
    C, no per-step ctypes call) on bounded samples, SURVEY.md 8(d):
      (i)   1v1 (C1), 1 env, 1 thread;
      (ii)  the bench config, 64 envs round-robin, 1 thread;
      (iii) the bench config, T threads (T = min(16, CPUs this process may use:
            the GPU box's per-GPU CPU share is 16)), 64 envs per thread;
      (iv)  the bench config on every CPU this process may use
            (len(os.sched_getaffinity(0))), 64 envs per
            thread -- only with all_cores (bench.py --cpu-all-cores): the
            GPU box's host is shared by the jobs of its 8 GPUs and each job's
            share is 16 CPUs, so the default run reports leg (iii) scaled
            linearly to all CPUs instead, labelled as an extrapolation.
    Uniform-random actions, auto-reset.  `value` is leg (iii)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    from masurvival.config import NAMED_CONFIGS, ResolvedConfig, pcg64_state
    model, avail = cpu_info()
    threads = max(1, min(16, avail))
    runs = [('c1_1env_1thread', '1v1', 1, 1),
            (f'{config}_64envs_1thread', config, 64, 1),
            (f'{config}_{64 * threads}envs_{threads}threads', config, 64 * threads, threads)]
    if all_cores and avail > threads:
        runs.append((f'{config}_{64 * avail}envs_{avail}threads_all_cores', config, 64 * avail, avail))
    legs = []
    for name, cfg_name, n, th in runs:
        rc = ResolvedConfig(NAMED_CONFIGS[cfg_name])
        st = np.stack([pcg64_state(s) for s in range(n)])
        steps, secs = oracle.bench_run(rc.to_struct(), st, th, leg_s)
        legs.append({'leg': name, 'threads': th, 'env_steps': steps, 'seconds': round(secs, 3),
                     'agent_env_steps_per_s': steps * rc.n_agents / secs})
    out = {'value': legs[2]['agent_env_steps_per_s'], 'unit': 'agent-env-steps/s', 'cores': threads,
           'kind': 'port',
           'sample': f'C oracle (oracle/ora_bench.c), {config}, {64 * threads} envs on {threads} threads, '
                     f'random actions + auto-reset, {legs[2]["seconds"]:.1f} s; other legs listed',
           'cpu_model': model, 'cpus_available': avail, 'legs': legs}
    if len(legs) == 3:
        out['all_cores_extrapolated'] = {
            'cpus': avail, 'agent_env_steps_per_s': legs[2]['agent_env_steps_per_s'] * avail / threads,
            'what': f'leg {legs[2]["leg"]} x {avail}/{threads} (linear; measure with bench.py --cpu-all-cores)'}
    proxy = os.path.join(ROOT, 'profiles', 'r02_reference_proxy.json')
    if os.path.exists(proxy):
        p = json.load(open(proxy))
        out['reference_proxy'] = {
            'what': 'reference Python env over the Box2D shim, 1 thread, timed in the build container '
                    '(profiles/r02_reference_proxy.json; PyBox2D absent: a labelled proxy)',
            'cpu_model': p.get('cpu_model'),
            'agent_env_steps_per_s': {r['config']: r['agent_env_steps_per_s'] for r in p['results']}}
    return out


def live_traffic(args, n, timeout_s=240):
    """HBM traffic per mas_step of this same workload, measured now: two
    child runs of this bench (same arguments, so the same seeds, regime and
    timed window) under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
    (separate passes: the two do not fit one, MI355X_MICROARCH.md), summed
    over the env-step kernels of each of the timed window's steps
    (profiles/pmc_traffic.py).  The children end with one mas_flush_stats
    (k_stats: 19 state words per env loaded and stored, 19 floats per env
    written -- 4-B lanes, the access width of the env kernels' state words)
    whose counters against those known bytes calibrate the raw counters for
    this access width (the guide calibrates 16-B lanes only).  Child
    processes, started after this run's timed region; returns a dict, or one
    with 'error' when rocprofv3 is missing or a pass fails."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, 'profiles'))
    import pmc_traffic
    prof = shutil.which('rocprofv3')
    if not prof:
        return {'error': 'rocprofv3 not found'}
    child, skip = [], False
    for a in sys.argv[1:]:  # (--lib passed on absolute: the children run in a scratch directory)
        if skip:
            skip = False
        elif a == '--lib':
            skip = True
        elif a != '--cpu-all-cores' and not a.startswith('--lib='):
            child.append(a)
    if args.lib:
        child += ['--lib', args.lib]
    child += ['--no-cpu-baseline', '--no-live-traffic', '--flush-stats']
    if not any(a.startswith('--horizon') for a in child):
        child += ['--horizon', str(args.horizon)]
    out, t0 = {}, time.perf_counter()
    with tempfile.TemporaryDirectory(prefix='mas_pmc_') as d:
        for c in ('FETCH_SIZE', 'WRITE_SIZE'):
            cmd = [prof, '--pmc', c, '--kernel-include-regex', 'mas::k_|k_stats', '--output-format', 'csv',
                   '-d', os.path.join(d, c), '-o', 'run', '--', sys.executable, os.path.abspath(__file__)] + child
            try:
                r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, timeout=timeout_s,
                                   env=dict(os.environ, MAS_BENCH_CHILD='1'))
            except subprocess.TimeoutExpired:
                return {'error': f'{c} pass timed out after {timeout_s} s'}
            csvs = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(d, c)) for f in fs
                    if f.endswith('counter_collection.csv')]
            if r.returncode != 0 or not csvs:
                return {'error': f'{c} pass failed (rc {r.returncode}): ' + (r.stderr or '')[-300:]}
            out[c] = csvs[0]
        f, nf = pmc_traffic.per_step(out['FETCH_SIZE'], 'FETCH_SIZE', args.steps)
        w, nw = pmc_traffic.per_step(out['WRITE_SIZE'], 'WRITE_SIZE', args.steps)
        cal = {c: pmc_traffic.kernel_bytes(out[c], c, 'k_stats') for c in out}
    fetch, write = sum(f.values()), sum(w.values())
    known = 19 * 4 * n  # k_stats: 19 words per env loaded (fetch); 19 stored + 19 floats written (write)
    res = {'fetch_bytes_per_step': fetch, 'write_bytes_per_step': write, 'traffic_bytes_per_step': fetch + write,
           'steps_profiled': min(nf, nw), 'per_kernel_fetch': dict(f), 'per_kernel_write': dict(w),
           'seconds': round(time.perf_counter() - t0, 1)}
    if cal.get('FETCH_SIZE') and cal.get('WRITE_SIZE'):
        kf, kw = cal['FETCH_SIZE'] / known, cal['WRITE_SIZE'] / (2 * known)
        res['calibration'] = {'kernel': 'k_stats (mas_flush_stats), 4-B lanes', 'fetch_counted_over_known': kf,
                              'write_counted_over_known': kw}
        res['traffic_bytes_per_step_calibrated'] = fetch / kf + write / kw
    return res


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """--gpus N > 1 without a launcher: run torch.distributed.run as a child
    process (nothing here has touched the GPU), relay its output, return its
    exit code."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MAS_BENCH_CHILD='1')
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    for ln in p.stdout.splitlines():
        if ln.startswith('{'):
            print(ln, flush=True)
        else:
            print(ln, file=sys.stderr, flush=True)
    return p.returncode


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=128, help='timed rollout steps')
    ap.add_argument('--warmup', type=int, default=16)
    ap.add_argument('--preroll', type=int, default=None,
                    help='untimed PPO iterations (ppo mode, default: enough for >= 128 steps, at least 2) or env '
                         'steps (env mode, default 128) before the warmup')
    ap.add_argument('--config', default='2v2')
    ap.add_argument('--envs', type=int, default=None, help='envs per GPU (default 65536 for 2v2)')
    ap.add_argument('--mode', choices=['ppo', 'env'], default='ppo',
                    help='ppo: policy forward + env step + buffer, GAE + PPO update every horizon; env: random actions')
    ap.add_argument('--horizon', type=int, default=None,
                    help='PPO rollout horizon; default: --steps when it is at most 64 (the timed window is then '
                         'exactly one PPO iteration), else 64')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-all-cores', action='store_true',
                    help='add the CPU-baseline leg on every CPU this process may use (cpu_baseline leg iv)')
    ap.add_argument('--lib', default=None, type=os.path.abspath,
                    help='alternative libmas*.so (A/B variants; made absolute: the PMC child runs start elsewhere)')
    ap.add_argument('--no-live-traffic', action='store_true',
                    help='skip the two rocprofv3 PMC child runs that measure roofline.traffic (live_traffic)')
    ap.add_argument('--flush-stats', action='store_true',
                    help='end with one mas_flush_stats (the PMC child runs: the counters\' calibration kernel)')
    ap.add_argument('--shards', type=int, default=1,
                    help='env handles per GPU, each on its own HIP stream (vec_env.ShardedVecMaSurvival)')
    return ap.parse_args()


def dry_run(args, world, rank):
    """MAS_BENCH_DRYRUN=1 (CPU tests of the launcher only): the rank set-up,
    barrier + max-over-ranks timing and the JSON relay, with no env."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group('gloo')
        dist.barrier()
    t0 = time.perf_counter()
    x = torch.zeros(1)
    for _ in range(args.steps):
        x += 1
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
        dist.barrier()
    if rank == 0:
        print(json.dumps({'metric': 'dry-run', 'value': 0.0, 'n_gpus': world, 'steps': args.steps,
                          'warmup': args.warmup, 'ms_per_step': dt * 1e3 / max(1, args.steps),
                          'data': 'dry-run (launcher test, no env)'}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse_args()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; n_gpus reports the world size',
              file=sys.stderr)
    if os.environ.get('MAS_BENCH_DRYRUN') == '1':
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist
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
    n = args.envs or ENVS_DEFAULT[args.config]
    if args.shards > 1:
        from masurvival.vec_env import ShardedVecMaSurvival
        env = ShardedVecMaSurvival(cfg, n_envs=n, shards=args.shards, seeds=range(rank * n, rank * n + n),
                                   auto_reset=True)
    else:
        env = VecMaSurvival(cfg, n_envs=n, seeds=range(rank * n, rank * n + n), auto_reset=True)
    A, D = env.n_agents, env.obs_dim
    dev = env.device
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    # the env kernels' launch-group duration, HIP events on the stream they run on
    kev = []

    def timed(step_fn):
        def f(a, out=None):
            e0, e1 = ev(), ev()
            e0.record()
            r = step_fn(a, out=out)
            e1.record()
            kev.append((e0, e1))
            return r
        return f

    def timed_x(step_fn):  # mas_step_x (the PPO trainer's bf16-row path)
        def f(*a):
            e0, e1 = ev(), ev()
            e0.record()
            r = step_fn(*a)
            e1.record()
            kev.append((e0, e1))
            return r
        return f

    if args.shards > 1:
        for sub in env.envs:
            sub.step = timed(sub.step)
            sub.step_x = timed_x(sub.step_x)
    else:
        env.step = timed(env.step)
        env.step_x = timed_x(env.step_x)

    rev, uev = [], []  # whole rollout step / whole GAE + update, on the current stream
    # the horizon: the timed window holds whole PPO iterations when it can
    # (--steps <= 64: one iteration of exactly --steps rollout steps and its
    # GAE + update), so ms_per_step is the training loop's steady-state cost
    # per step; a window shorter than the horizon would carry a whole update
    # of horizon steps' rows for fewer rollout steps
    if args.horizon is None:
        args.horizon = args.steps if args.steps <= 64 else 64
    if args.mode == 'ppo':
        from masurvival.ppo import PPOConfig, PPOTrainer
        pcfg = PPOConfig(horizon=args.horizon)
        tr = PPOTrainer(env, pcfg, seed=0)
        H = pcfg.horizon
        state = {'t': 0, 'updates': 0}

        # Every event record is a marker packet on the stream (~4-5 us of GPU
        # time between two kernels, r06m trace; events without the
        # system-scope fence measured the same), so the window records two per
        # rollout step: before k_pre and after the last env kernel (the env
        # step's pair, kev).  The rollout step runs from the previous boundary
        # event (the last env step's end, or the update's end) to this step's
        # env end, and the GAE + update from that env end to one event after
        # the update.
        shared = args.shards == 1
        state['edge'] = None

        def one_step():
            if shared:
                if state['edge'] is None:
                    state['edge'] = ev()
                    state['edge'].record()
                e0 = state['edge']
                tr.rollout_step(state['t'])
                e1 = kev[-1][1]  # the env step's end event (timed_x), the rollout step's last work
                state['edge'] = e1
            else:
                e0, e1 = ev(), ev()
                e0.record()
                tr.rollout_step(state['t'])
                e1.record()
            rev.append((e0, e1))
            state['t'] += 1
            if state['t'] == H:
                u0, u1 = (state['edge'], ev()) if shared else (ev(), ev())
                if not shared:
                    u0.record()
                tr.finish_rollout()
                tr.update()
                u1.record()
                uev.append((u0, u1))
                state['edge'] = u1
                state['t'] = 0
                state['updates'] += 1
        # >= 128 steps and >= 2 updates of pre-roll: the training regime
        # (general-path physics, contacts, TOI) whatever the horizon
        preroll = max(2, -(-128 // H)) if args.preroll is None else args.preroll
        for _ in range(preroll * H):
            one_step()
        for _ in range(args.warmup):
            one_step()
        align = (-(state['t'] + args.steps)) % H
        for _ in range(align):
            one_step()
    else:
        env.reset()
        hi = torch.tensor([3, 3, 3, 2, 2, 2], device=dev, dtype=torch.int32)
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        acts = torch.empty((n, A, 6), dtype=torch.int8, device=dev)

        def one_step():
            u = torch.rand((n, A, 6), generator=gen, device=dev)
            acts.copy_((u * hi).to(torch.int8))
            env.step(acts)
        preroll = 128 if args.preroll is None else args.preroll
        align = 0
        for _ in range(preroll + args.warmup):
            one_step()
    torch.cuda.synchronize()
    kev.clear()
    rev.clear()
    uev.clear()
    if args.mode == 'ppo':
        state['updates'] = 0
        state['edge'] = None  # the window's first rollout step starts at a fresh event
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
    if args.mode == 'ppo' and state['updates'] != math.ceil(args.steps / H):
        raise RuntimeError(f'timed window holds {state["updates"]} updates, expected {math.ceil(args.steps / H)}')
    mean_ms = lambda evs: float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else 0.0  # noqa: E731
    kern_ms, roll_ms, upd_ms = mean_ms(kev), mean_ms(rev), mean_ms(uev)
    if world > 1:
        t = torch.tensor([dt, kern_ms, roll_ms, upd_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kern_ms, roll_ms, upd_ms = (float(x) for x in t)

    diag = env.debug_counters()
    total_agent_steps = world * n * A * args.steps
    x_obs = args.mode == 'ppo' and tr.x_obs
    b_env = algorithmic_bytes_per_env_step(A, env.rc.n_heals, env.rc.n_boxes, D, obs_bytes=2 if x_obs else 4)
    n_launch = n // args.shards  # envs per mas_step launch group (per shard when sharded)
    achieved = b_env * n_launch / (kern_ms * 1e-3) / 1e9
    if args.mode == 'ppo':
        workload = (f'{args.config} PPO rollout (fused policy MLP 2x256 fwd + sample, env step into the rollout '
                    f'buffer), GAE + PPO update (1 epoch, 4 minibatches) every {args.horizon} steps')
    else:
        workload = f'{args.config} env step, random policy'
    line = {
        'metric': 'agent-env-steps/sec (whole node), %s N_envs=%d' % (args.config, n * world),
        'value': total_agent_steps / dt,
        'unit': 'agent-env-steps/s',
        'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': dt * 1e3 / args.steps,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'f32 env step; policy bf16 MFMA with f32 accumulate, f32 master weights + Adam'
                 if args.mode == 'ppo' else 'f32',
        'data': 'synthetic (seeded envs, on-device policy sampling)',
        'config': {'workload': workload, 'n_envs_per_gpu': n, 'n_agents': A, 'obs_dim': D,
                   'horizon': args.horizon if args.mode == 'ppo' else None,
                   'preroll': (f'{preroll} PPO iterations ({preroll * args.horizon} steps + {preroll} updates)'
                               if args.mode == 'ppo' else f'{preroll} env steps'),
                   'align_steps': align,
                   'updates_in_timed_region': state['updates'] if args.mode == 'ppo' else 0,
                   'window': (f'{args.steps} rollout steps = {args.steps / args.horizon:g} PPO iteration(s) of '
                              f'{args.horizon} steps, each with its GAE + update'
                              if args.mode == 'ppo' and args.steps % args.horizon == 0 else
                              (f'{args.steps} rollout steps + {state["updates"]} update(s) of {args.horizon} steps'
                               if args.mode == 'ppo' else None)),
                   'parallelism': f'env-shard x{world}',
                   'streams_per_gpu': args.shards,
                   'phys_general_envs_last_step': diag['phys_general_envs'],
                   'breakdown_ms': {'env_step': kern_ms,
                                    'rollout_step': roll_ms if args.mode == 'ppo' else None,
                                    'gae_plus_update': upd_ms if args.mode == 'ppo' else None,
                                    'amortised_step': (roll_ms + upd_ms / args.horizon)
                                    if args.mode == 'ppo' else None}},
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                     'kernel': 'mas_step launch group (k_pre_lanes, k_gen_solve_g, k_post_lanes with the auto-reset in place; the slow-list pair on the side stream)' if args.shards == 1 else
                     f'mas_step launch group of one shard ({args.shards} shards on concurrent streams)',
                     'kernel_ms': kern_ms, 'bytes_per_env_step': b_env,
                     'obs_rows': ('bf16 policy-input rows (mas_step_x)' if x_obs else 'fp32 obs rows (mas_step)'),
                     'bytes_per_launch': b_env * n_launch},
        'cpu_baseline': None,
    }
    # roofline.traffic: measured in this run only (live_traffic below); null
    # otherwise (committed PMC files of earlier trees are not this tree's bytes)
    if args.flush_stats:
        env.flush_stats()
        torch.cuda.synchronize()
    if rank == 0 and world == 1 and not args.no_live_traffic and os.environ.get('MAS_BENCH_CHILD') != '1':
        lt = live_traffic(args, n)
        line['roofline']['traffic_live'] = lt
        if 'traffic_bytes_per_step' in lt:
            # the guide's gfx950 correction (FETCH_SIZE counts half the bytes
            # read), confirmed for this access width by the k_stats
            # calibration of the same runs when it is present
            if 'traffic_bytes_per_step_calibrated' in lt:
                tb, how = lt['traffic_bytes_per_step_calibrated'], 'calibrated on k_stats (traffic_live.calibration)'
            else:
                tb, how = 2 * lt['fetch_bytes_per_step'] + lt['write_bytes_per_step'], 'FETCH_SIZE x 2 (guide)'
            line['roofline']['traffic'] = tb * n_launch / n
            line['roofline']['traffic_source'] = ('measured in this run: FETCH_SIZE + WRITE_SIZE per mas_step over '
                                                  'the timed window, two rocprofv3 --pmc child runs of this command, '
                                                  + how + '; raw counters in traffic_live')
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline(args.config, all_cores=args.cpu_all_cores)
    if rank == 0:
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
