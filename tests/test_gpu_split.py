"""The slow split against the one-stream order (mas_debug_force_general
bit 3, MAS_SPLIT): two handles on the same seeds and actions must give
bit-identical obs, rewards, done flags and state images, with auto-reset.

In the slow split only the envs whose previous general-path step was slow
(a SolveTOI at the sub-step cap, or >= MAS_SLOW_K TOI events) go to the
side stream.  MAS_SLOW_K=1 here, so that every env with a TOI event the step
before takes the side stream and the slow list is busy at these sizes (the
product default, 4, picks the few wedged envs of the PPO regime).

The contact-heavy regime is random actions (plus every env forced onto the
general path in one case: the list-mode kernels then run every env)."""
import math

import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import C3_CONFIG, C5_CONFIG  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402

HI = torch.tensor([3, 3, 3, 2, 2, 2])
# the Lidars run after the join, over every env (k_lidar reads the state the
# side stream wrote)
LID_2V2 = {'agents': {'n_agents': 4, 'agent_size': 1}, 'teams': {'twoteams': True},
           'melee': {'range': 2, 'damage': 20, 'cooldown': 40, 'drift': True},
           'lidars': {'n_lasers': 8, 'fov': 0.5 * math.pi, 'depth': 6}}


@pytest.mark.parametrize('name,cfg,n,T,mode,forced,ar', [
    ('C3 2v2 slow', C3_CONFIG, 8192, 220, None, False, True),
    ('C5 ffa4 slow', C5_CONFIG, 2048, 200, None, False, True),
    ('C3 2v2 slow forced', C3_CONFIG, 4096, 60, None, True, True),
    ('C3 2v2 slow no auto-reset', C3_CONFIG, 4096, 160, None, False, False),
    ('2v2 lidars slow', LID_2V2, 4096, 160, None, False, True)])
def test_split_step_matches_one_stream(name, cfg, n, T, mode, forced, ar, monkeypatch):
    monkeypatch.setenv('MAS_SLOW_K', '1')
    monkeypatch.delenv('MAS_SPLIT', raising=False)
    try:
        one = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=ar)
        two = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=ar)
    except abi.MasError as e:
        class_missing(e)
    one.split_step(0)
    two.split_step(mode)
    if forced:
        one.force_general(True)
        two.force_general(True)
    assert torch.equal(one.reset(), two.reset())
    gen = torch.Generator(device=one.device)
    gen.manual_seed(n)
    hi = HI.to(one.device)
    general = side = 0
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
        f1, f2 = one.gen_flags(), two.gen_flags()
        assert not bool((f1 == 2).any()), (name, t)  # no slow list on one stream
        assert torch.equal(f1 != 0, f2 != 0), (name, t)
        side += int((f2 == 2).sum())
    assert torch.equal(one.get_state(), two.get_state())
    assert general > 0
    assert side > 0, name  # the slow list ran
    assert one.debug_guards()['list_overflow'] == 0 and two.debug_guards()['list_overflow'] == 0
    one.close()
    two.close()
