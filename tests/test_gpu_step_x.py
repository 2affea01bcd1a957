"""mas_step_x (include/masurvival.h): the env step writing the PPO consumer's
bf16 policy-input rows instead of fp32 obs rows.  Against mas_step on a twin
handle (same seeds, same actions, auto-reset on): rewards, done flags and the
state image bit-identical every step, and every written column the fp32 row
rounded to bf16 (round to nearest even, torch's float -> bfloat16, which is
also mas_policy_act's conversion); columns past obs_dim keep the caller's
values.  Configs cover both row sinks of k_post_lanes: the LDS-swapped
four-row form (QuadRowX: 4-agent classes filled exactly -- C3, C5) and the
per-lane form (SeqRowX: 1v1, 3 agents in the 4-agent class, 6 agents in xl)."""
import math

import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import C1_CONFIG, C3_CONFIG, C5_CONFIG  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402

HI = torch.tensor([3, 3, 3, 2, 2, 2])
SIX = {'agents': {'n_agents': 6, 'agent_size': 1}, 'spawn_grid': {'grid_size': 4, 'floor_size': 20},
       'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}
THREE = {'agents': {'n_agents': 3, 'agent_size': 1},
         'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True}}
SHORT_ZONE = {'phases': 5, 'cooldown': 12, 'damage': 6, 'radiuses': [10, 5, 2.5, 1], 'centers': 'random'}


@pytest.mark.parametrize('name,cfg,n,T', [
    ('C1 1v1 (SeqRowX)', C1_CONFIG, 512, 200),
    ('C3 2v2 (QuadRowX)', C3_CONFIG, 1024, 200),
    ('C5 ffa4 (QuadRowX)', dict(C5_CONFIG, safe_zone=SHORT_ZONE), 256, 120),
    ('3 agents in the 2v2 class (SeqRowX)', dict(THREE, safe_zone=SHORT_ZONE), 512, 160),
    ('6 agents, xl (SeqRowX)', dict(SIX, safe_zone=SHORT_ZONE), 128, 120)])
def test_step_x_rows_are_the_rounded_fp32_rows(name, cfg, n, T):
    try:
        ref = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
        xen = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)
    assert xen.supports_step_x()
    A, D = xen.n_agents, xen.obs_dim
    Dx = 8 * ((D + 1 + 7) // 8)  # room past obs_dim, a multiple of 4
    assert torch.equal(ref.reset(), xen.reset())
    x = torch.full((n * A, Dx), -7.0, dtype=torch.bfloat16, device=xen.device)  # sentinels past obs_dim
    rew = torch.empty((n, A), dtype=torch.float32, device=xen.device)
    dn = torch.empty((n,), dtype=torch.uint8, device=xen.device)
    gen = torch.Generator(device=xen.device)
    gen.manual_seed(n + 3)
    hi = HI.to(xen.device)
    dones = 0
    for t in range(T):
        a = (torch.rand((n, A, 6), generator=gen, device=xen.device) * hi).to(torch.int8)
        o, r, d, _ = ref.step(a)
        xen.step_x(a, x, rew, dn)
        assert torch.equal(d, dn), (name, t)
        assert torch.equal(r, rew), (name, t)
        want = o.reshape(n * A, D).to(torch.bfloat16)
        got = x[:, :D]
        assert torch.equal(got.view(torch.int16), want.view(torch.int16)), (name, t)  # bit for bit
        dones += int(d.sum())
    assert bool((x[:, D:] == -7.0).all()), name  # the caller's columns untouched
    assert dones > 0, name  # episodes ended and reset in place
    assert torch.equal(ref.get_state(), xen.get_state()), name
    ref.close()
    xen.close()


def test_step_x_refusals():
    lid = dict(C3_CONFIG, lidars={'n_lasers': 8, 'fov': 0.5 * math.pi, 'depth': 6})
    env = VecMaSurvival(lid, n_envs=64, seeds=range(64), auto_reset=True)
    assert not env.supports_step_x()  # k_lidar writes fp32 columns
    x = torch.zeros((64 * env.n_agents, 8 * ((env.obs_dim + 8) // 8)), dtype=torch.bfloat16, device=env.device)
    a = torch.zeros((64, env.n_agents, 6), dtype=torch.int8, device=env.device)
    rew = torch.empty((64, env.n_agents), device=env.device)
    dn = torch.empty((64,), dtype=torch.uint8, device=env.device)
    env.reset()
    with pytest.raises(abi.MasError, match='lidars'):
        env.step_x(a, x, rew, dn)
    env.close()
    env = VecMaSurvival(C3_CONFIG, n_envs=64, seeds=range(64), auto_reset=True)
    env.reset()
    lib, h = env._lib, env._h
    import ctypes
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    x = torch.zeros((64 * 4, 176), dtype=torch.bfloat16, device=env.device)
    for stride in (env.obs_dim - 4, 162):  # below obs_dim; not a multiple of 4
        assert lib.mas_step_x(h, p(a), p(x), stride, p(rew), p(dn), 1, None) == -1  # MAS_ERR_INVALID_ARG
    env.close()
