"""A/B of the general path's Collide + Solve kernels on a golden episode:
two n_envs = 1 handles replay the fixture's actions in lockstep, one with the
lane-group k_gen_solve_g (default), one with the one-lane k_gen_solve +
k_gen_toi (mas_debug_force_general bit 1; these kernels are only in the test
library libmas_ab.so, `make -C gym-ma-survival-2d_amd/csrc ab`).  After every step their mas_get_state
images are compared; at the first difference the differing words (index,
both values) and the step are printed and both images are saved.
usage: python scripts/ab_solve_golden.py <fixture.npz> [out.npz]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))
# the one-lane kernels live only in the test build (make -C .../csrc ab)
os.environ.setdefault('MAS_LIB', os.path.join(ROOT, 'gym-ma-survival-2d_amd', 'masurvival', '_lib', 'libmas_ab.so'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_replay as gr  # noqa: E402
from masurvival.config import pcg64_state  # noqa: E402
from masurvival.vec_env import VecMaSurvival  # noqa: E402


def main():
    name = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    d, cfg = gr.load(name)
    seed = int(d['env_seed'])
    envs = []
    for one_lane in (False, True):
        e = VecMaSurvival(cfg, n_envs=1, auto_reset=False)
        e.set_rng_states(pcg64_state(seed)[None])
        e.force_general(False, one_lane_solve=one_lane)
        e.reset()
        envs.append(e)
    prev = envs[0].get_state().cpu().numpy().view(np.uint32).copy()
    for t in range(len(d['done'])):
        a = torch.as_tensor(np.asarray(d['actions'][t], dtype=np.int8)[None], device=envs[0].device)
        for e in envs:
            e.step(a)
        sa = envs[0].get_state().cpu().numpy().view(np.uint32)
        sb = envs[1].get_state().cpu().numpy().view(np.uint32)
        if not np.array_equal(sa, sb):
            idx = np.nonzero(sa != sb)[0]
            print(f'first difference after step {t}: {len(idx)} words')
            for k in idx[:40]:
                print(f'  word {k}: lane-group {sa[k]:#010x} ({sa[k:k+1].view(np.float32)[0]!r})  '
                      f'one-lane {sb[k]:#010x} ({sb[k:k+1].view(np.float32)[0]!r})  before {prev[k]:#010x} '
                      f'({prev[k:k+1].view(np.float32)[0]!r})')
            if out:
                np.savez(out, step=t, before=prev, group=sa, one_lane=sb, actions=np.asarray(d['actions'][t]))
            return 1
        prev = sa.copy()
    print('identical over', len(d['done']), 'steps')
    return 0




def probe(name, npz):
    """Re-run the divergent step from the saved pre-step image on both
    variants and report the path the env took."""
    d, cfg = gr.load(name)
    s = np.load(npz)
    for one_lane in (False, True):
        e = VecMaSurvival(cfg, n_envs=1, auto_reset=False)
        e.force_general(False, one_lane_solve=one_lane)
        e.set_state(torch.as_tensor(s['before'].view(np.uint8), device=e.device))
        a = torch.as_tensor(np.asarray(s['actions'], dtype=np.int8)[None], device=e.device)
        e.step(a)
        st = e.get_state().cpu().numpy().view(np.uint32)
        f = st.view(np.float32)
        print('one_lane' if one_lane else 'group   ', 'general', e.debug_counters()['phys_general_envs'],
              'sleep words', f[6], f[13], 'awake', st[15], 'same as saved',
              np.array_equal(st, s['one_lane' if one_lane else 'group']))


if __name__ == '__main__':
    if len(sys.argv) > 3 and sys.argv[3] == 'probe':
        probe(sys.argv[1], sys.argv[2])
    elif sys.argv[1] == 'all':
        bad = 0
        for f in gr.golden_files():
            print(f, flush=True)
            sys.argv = [sys.argv[0], f]
            bad += main()
        sys.exit(1 if bad else 0)
    else:
        sys.exit(main())
