"""The RCCL code path of the multi-GPU bench on the one-GPU box.

bench.py's N-GPU run initialises torch.distributed with backend 'nccl' (RCCL
on ROCm) and the trainer all-reduces (sum adv, sum adv^2, count) once per
rollout and the flat gradient once per minibatch (`ppo.py` finish_rollout /
_allreduce_grads).  A one-GPU box cannot run 2 RCCL ranks, but a world of
one rank executes the same RCCL calls on device tensors: this test runs one
fused PPO iteration with the collectives forced on (PPOConfig.allreduce) over
an 'nccl' process group and requires the parameters to equal, bit for bit, a
run of the same seed without any process group (a one-rank sum and the
division by 1 are exact)."""
import os

import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

import torch.multiprocessing as mp  # noqa: E402


def _child(init_file, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    'gym-ma-survival-2d_amd'))
    import torch.distributed as dist
    from masurvival.config import C3_CONFIG
    from masurvival.ppo import PPOConfig, PPOTrainer
    from masurvival.vec_env import VecMaSurvival

    def one_iteration(cfg):
        env = VecMaSurvival(C3_CONFIG, n_envs=512, device='cuda:0', seeds=range(512))
        tr = PPOTrainer(env, cfg, seed=0)
        assert tr.fused is not None
        tr.iteration()
        flat = torch.cat([p.detach().reshape(-1) for p in tr.policy.parameters()]).cpu()
        adv = tr.buf.adv.detach().cpu()
        coll = tr.collectives
        env.close()
        return flat, adv, coll

    ref, ref_adv, coll0 = one_iteration(PPOConfig(horizon=16))
    assert not coll0
    dist.init_process_group('nccl', init_method=f'file://{init_file}', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    try:
        backend = dist.get_backend()
        x = torch.arange(4096, device='cuda:0', dtype=torch.float32)
        y = x.clone()
        dist.all_reduce(y)
        torch.cuda.synchronize()
        direct_ok = bool(torch.equal(x, y))
        got, got_adv, coll1 = one_iteration(PPOConfig(horizon=16, allreduce=True))
        assert coll1
        torch.save({'ref': ref, 'rccl': got, 'ref_adv': ref_adv, 'rccl_adv': got_adv, 'backend': backend,
                    'direct_ok': direct_ok}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world1_fused_ppo_iteration_matches_local(tmp_path):
    ctx = mp.get_context('spawn')
    out = str(tmp_path / 'rccl.pt')
    p = ctx.Process(target=_child, args=(str(tmp_path / 'rdzv'), out))
    p.start()
    p.join(240)
    assert p.exitcode == 0, p.exitcode
    r = torch.load(out, weights_only=True)
    assert r['backend'] == 'nccl' and r['direct_ok']
    assert torch.equal(r['ref_adv'], r['rccl_adv']), 'advantage normalisation differs through RCCL'
    assert torch.equal(r['ref'], r['rccl']), 'parameters differ after the RCCL gradient all-reduce'
