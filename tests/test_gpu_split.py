"""The split step (mas_debug_force_general bit 2 / MAS_SPLIT=1: the general
path and the general envs' k_cameras / k_post / k_obs on a side stream, the
other envs' on the caller's stream) against the one-stream order: two
handles on the same seeds and actions must give bit-identical obs, rewards,
done flags and state images, with auto-reset, in the contact-heavy regime
(random actions for 150 steps first), and with every env forced onto the
general path (the list-mode kernels then run every env)."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival import abi  # noqa: E402
from masurvival.config import C3_CONFIG, C5_CONFIG  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402

HI = torch.tensor([3, 3, 3, 2, 2, 2])


@pytest.mark.parametrize('name,cfg,n,T,forced', [('C3 2v2', C3_CONFIG, 8192, 220, False),
                                                 ('C5 ffa4', C5_CONFIG, 2048, 200, False),
                                                 ('C3 2v2 forced', C3_CONFIG, 4096, 40, True)])
def test_split_step_matches_one_stream(name, cfg, n, T, forced):
    try:
        one = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
        two = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        pytest.skip(str(e))
    two.split_step(True)
    if forced:
        one.force_general(True)
        two.force_general(True)
    assert torch.equal(one.reset(), two.reset())
    gen = torch.Generator(device=one.device)
    gen.manual_seed(n)
    hi = HI.to(one.device)
    general = 0
    for t in range(T):
        a = (torch.rand((n, one.n_agents, 6), generator=gen, device=one.device) * hi).to(torch.int8)
        o1, r1, d1, _ = one.step(a)
        o1, r1, d1 = o1.clone(), r1.clone(), d1.clone()
        o2, r2, d2, _ = two.step(a)
        assert torch.equal(d1, d2), (name, t)
        assert torch.equal(r1, r2), (name, t)
        assert torch.equal(o1, o2), (name, t)
        g1, g2 = one.debug_counters()['phys_general_envs'], two.debug_counters()['phys_general_envs']
        assert g1 == g2, (name, t)
        general += g1
    assert torch.equal(one.get_state(), two.get_state())
    assert general > 0
    assert one.debug_guards()['list_overflow'] == 0 and two.debug_guards()['list_overflow'] == 0
    one.close()
    two.close()
