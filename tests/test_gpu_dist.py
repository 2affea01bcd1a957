"""The multi-rank PPO path with the fused HIP policy kernels, world size 2.

The round-end driver runs bench.py over RCCL on 8 GPUs; a one-GPU box cannot,
so this runs two ranks on cuda:0 over gloo (which reduces CUDA tensors
through the host).  The collectives are the same calls the RCCL run makes:
the fp64 advantage-statistics all-reduce and one flat gradient all-reduce per
minibatch.  Checks: every rank ends an iteration with identical parameters,
and the advantages are normalised with the global statistics."""
import os

import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _rank_main(rank, world, init_file, out_dir):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    'gym-ma-survival-2d_amd'))
    from masurvival.config import C3_CONFIG
    from masurvival.ppo import PPOConfig, PPOTrainer
    from masurvival.vec_env import VecMaSurvival
    dist.init_process_group('gloo', init_method=f'file://{init_file}', rank=rank, world_size=world)
    n = 256
    env = VecMaSurvival(C3_CONFIG, n_envs=n, device='cuda:0', seeds=range(rank * n, rank * n + n))
    tr = PPOTrainer(env, PPOConfig(horizon=16), seed=0)
    assert tr.fused is not None
    tr.iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in tr.policy.parameters()]).cpu()
    adv = tr.buf.adv.reshape(-1).double()
    torch.save({'flat': flat, 's1': float(adv.sum()), 's2': float((adv ** 2).sum()), 'n': adv.numel()},
               os.path.join(out_dir, f'rank{rank}.pt'))
    dist.barrier()
    env.close()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_fused_ppo_iteration(tmp_path):
    ctx = mp.get_context('spawn')
    init_file = str(tmp_path / 'rdzv')
    ps = [ctx.Process(target=_rank_main, args=(r, 2, init_file, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(200)
        assert p.exitcode == 0
    res = [torch.load(str(tmp_path / f'rank{r}.pt'), weights_only=True) for r in range(2)]
    assert torch.equal(res[0]['flat'], res[1]['flat']), 'ranks diverged after the gradient all-reduce'
    s1 = res[0]['s1'] + res[1]['s1']
    s2 = res[0]['s2'] + res[1]['s2']
    n = res[0]['n'] + res[1]['n']
    assert abs(s1 / n) < 1e-5 and abs(s2 / n - 1) < 1e-3
