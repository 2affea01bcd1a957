"""A graph-captured mas_step replays like eager steps (INTEGRATION.md
"Graph capture").

With the handle on one stream (MAS_SPLIT=0 / mas_debug_force_general bit 3)
mas_step keeps no host state between calls: the general-path list count is
zeroed on the device by the first post kernel after its last reader.  One
handle steps eagerly, a second replays a HIP graph of one captured step with
the same actions copied into its static action buffer; obs, rewards, done,
the general-path counts and the final state images must be identical, and no
list append may be refused (a count that grew across replays would re-step
stale entries and then overflow the list).

mas_step checks hipStreamIsCapturing: a step captured on a handle with the
default slow split while it is on (MAS_SLOW_K=1 and a warm-up that flags
slow envs, so the 8-step hold is active at capture) runs on one stream in
the graph and replays like eager steps of a one-stream handle."""
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu

from masurvival import abi  # noqa: E402
from gpu_util import class_missing  # noqa: E402
from masurvival.config import C3_CONFIG, C5_CONFIG  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402

HI = torch.tensor([3, 3, 3, 2, 2, 2])


@pytest.mark.parametrize('name,cfg,n,T,forced', [
    ('C3 2v2', C3_CONFIG, 4096, 120, False),
    ('C3 2v2 forced general', C3_CONFIG, 2048, 40, True),
    ('C5 ffa4', C5_CONFIG, 1024, 80, False)])
def test_captured_step_replays_like_eager(name, cfg, n, T, forced):
    try:
        eager = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
        graph = VecMaSurvival(cfg, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        class_missing(e)
    for e in (eager, graph):
        e.split_step(0)
        if forced:
            e.force_general(True)
    assert torch.equal(eager.reset(), graph.reset())
    act = torch.zeros((n, graph.n_agents, 6), dtype=torch.int8, device=graph.device)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        graph.step(act)
    gen = torch.Generator(device=graph.device)
    gen.manual_seed(n + 17)
    hi = HI.to(graph.device)
    general = 0
    for t in range(T):
        a = (torch.rand((n, graph.n_agents, 6), generator=gen, device=graph.device) * hi).to(torch.int8)
        act.copy_(a)
        g.replay()
        o1, r1, d1, _ = eager.step(a)
        assert torch.equal(d1, graph.dones), (name, t)
        assert torch.equal(r1, graph.rewards), (name, t)
        assert torch.equal(o1, graph.obs), (name, t)
        c1, c2 = eager.debug_counters()['phys_general_envs'], graph.debug_counters()['phys_general_envs']
        assert c1 == c2, (name, t, c1, c2)
        general += c1
    assert general > 0
    assert torch.equal(eager.get_state(), graph.get_state())
    assert eager.debug_guards()['list_overflow'] == 0
    assert graph.debug_guards()['list_overflow'] == 0
    del g
    eager.close()
    graph.close()


def test_captured_step_of_split_handle_replays_like_eager(monkeypatch):
    name, mode = 'slow split held at capture', None
    monkeypatch.setenv('MAS_SLOW_K', '1')
    monkeypatch.delenv('MAS_SPLIT', raising=False)
    n, T, warm = 4096, 100, 40
    try:
        eager = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n), auto_reset=True)
        graph = VecMaSurvival(C3_CONFIG, n_envs=n, seeds=range(n), auto_reset=True)
    except abi.MasError as e:
        pytest.fail(str(e))
    eager.split_step(0)
    graph.split_step(mode)
    assert torch.equal(eager.reset(), graph.reset())
    gen = torch.Generator(device=graph.device)
    gen.manual_seed(n + 29)
    hi = HI.to(graph.device)
    side = 0
    for t in range(warm):
        # eager warm-up on both: the graph handle's slow split turns on
        a = (torch.rand((n, graph.n_agents, 6), generator=gen, device=graph.device) * hi).to(torch.int8)
        o1, _, _, _ = eager.step(a)
        o2, _, _, _ = graph.step(a)
        assert torch.equal(o1, o2), (name, t)
        side += int((graph.gen_flags() == 2).sum())
    assert side > 0, name  # the slow list ran before the capture
    act = torch.zeros((n, graph.n_agents, 6), dtype=torch.int8, device=graph.device)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        graph.step(act)
    general = 0
    for t in range(T):
        a = (torch.rand((n, graph.n_agents, 6), generator=gen, device=graph.device) * hi).to(torch.int8)
        act.copy_(a)
        g.replay()
        o1, r1, d1, _ = eager.step(a)
        assert torch.equal(d1, graph.dones), (name, t)
        assert torch.equal(r1, graph.rewards), (name, t)
        assert torch.equal(o1, graph.obs), (name, t)
        assert not bool((graph.gen_flags() == 2).any()), (name, t)  # no slow list in the graph
        c1, c2 = eager.debug_counters()['phys_general_envs'], graph.debug_counters()['phys_general_envs']
        assert c1 == c2, (name, t, c1, c2)
        general += c1
    assert general > 0
    assert torch.equal(eager.get_state(), graph.get_state())
    # eager steps on the split handle after the replays:
    # the replays flagged slow envs, so the split turns on again and its first
    # step appends to a slow-list count slot the captured k_pre must have
    # zeroed (the host's slot parity did not move during the replays)
    side = 0
    for t in range(40):
        a = (torch.rand((n, graph.n_agents, 6), generator=gen, device=graph.device) * hi).to(torch.int8)
        o1, r1, d1, _ = eager.step(a)
        o2, r2, d2, _ = graph.step(a)
        assert torch.equal(d1, d2), (name, 'after replays', t)
        assert torch.equal(r1, r2), (name, 'after replays', t)
        assert torch.equal(o1, o2), (name, 'after replays', t)
        side += int((graph.gen_flags() == 2).sum())
    assert side > 0, name  # the slow list ran again after the replays
    assert torch.equal(eager.get_state(), graph.get_state())
    assert eager.debug_guards()['list_overflow'] == 0
    assert graph.debug_guards()['list_overflow'] == 0
    del g
    eager.close()
    graph.close()
