"""How often the Box2D Gauss-Seidel loops reach an exact fixed point (the
evidence behind the fixed-point exits in csrc/mas_physics.h, same_bits).

Builds an INSTRUMENTED COPY of the C oracle in a temp dir (the copy records,
per solver loop, the first iteration after which the state -- bodies'
position / velocity and the accumulated impulses -- is bit-identical to the
state before it; from there every later iteration repeats itself), replays
(a) the PPO-regime env whose SolveTOI reaches the sub-step cap
(profiles/r02_wedged_env.npz) and (b) 32 uniform-random 2v2 envs x 300
steps, and prints iterations run vs iterations needed.  Test tooling: the
oracle in oracle/ is not modified.
usage: python profiles/fixed_point_probe.py"""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, os.path.join(ROOT, 'gym-ma-survival-2d_amd'))

PATCHES = [
    ("""        for (int it = 0; it < vel_iters; ++it)
            for (int q = 0; q < nk; ++q) solve_vcon(w, &ks[q]);
        for (int q = 0; q < nk; ++q) {""",
     """        {
            int fixed_at = -1;
            for (int it = 0; it < vel_iters; ++it) {
                float snap[64]; int ns_ = 0;
                for (int m = 0; m < nm; ++m) { snap[ns_++] = w->v[members[m]].x; snap[ns_++] = w->v[members[m]].y; snap[ns_++] = w->w[members[m]]; }
                for (int q = 0; q < nk && ns_ < 62; ++q) { snap[ns_++] = ks[q].ni; snap[ns_++] = ks[q].ti; }
                for (int q = 0; q < nk; ++q) solve_vcon(w, &ks[q]);
                float now[64]; int nn = 0;
                for (int m = 0; m < nm; ++m) { now[nn++] = w->v[members[m]].x; now[nn++] = w->v[members[m]].y; now[nn++] = w->w[members[m]]; }
                for (int q = 0; q < nk && nn < 62; ++q) { now[nn++] = ks[q].ni; now[nn++] = ks[q].ti; }
                if (fixed_at < 0 && memcmp(snap, now, sizeof(float) * nn) == 0) fixed_at = it;
            }
            g_ins[0] += (long long)vel_iters * nk;
            g_ins[1] += (long long)(fixed_at < 0 ? vel_iters : fixed_at + 1) * nk;
        }
        for (int q = 0; q < nk; ++q) {"""),
    ("""        for (int it = 0; it < pos_iters; ++it) {
            float minSep = 0.0f;
            for (int q = 0; q < nk; ++q) minSep = b2min(minSep, solve_pcon(w, &ks[q], BAUMGARTE));
            if (minSep >= -3.0f * LINEAR_SLOP) { positionSolved = 1; break; }
        }""",
     """        {
            int fixed_at = -1, ran = 0;
            for (int it = 0; it < pos_iters; ++it) {
                float snap[48]; int ns_ = 0;
                for (int m = 0; m < nm; ++m) { snap[ns_++] = w->c[members[m]].x; snap[ns_++] = w->c[members[m]].y; snap[ns_++] = w->a[members[m]]; }
                float minSep = 0.0f;
                for (int q = 0; q < nk; ++q) minSep = b2min(minSep, solve_pcon(w, &ks[q], BAUMGARTE));
                ++ran;
                float now[48]; int nn = 0;
                for (int m = 0; m < nm; ++m) { now[nn++] = w->c[members[m]].x; now[nn++] = w->c[members[m]].y; now[nn++] = w->a[members[m]]; }
                if (fixed_at < 0 && memcmp(snap, now, sizeof(float) * nn) == 0) fixed_at = it;
                if (minSep >= -3.0f * LINEAR_SLOP) { positionSolved = 1; break; }
            }
            g_ins[2] += (long long)ran * nk;
            g_ins[3] += (long long)(fixed_at < 0 ? ran : fixed_at + 1) * nk;
        }"""),
    ("""        for (int it = 0; it < 20; ++it) {
            float minSep = 0.0f;
            for (int q = 0; q < ni; ++q) minSep = b2min(minSep, solve_pcon(w, &ks[q], TOI_BAUMGARTE));
            if (minSep >= -1.5f * LINEAR_SLOP) break;
        }""",
     """        {
            int f1 = -1, ran = 0;
            float h1[3] = {0, 0, 0};
            for (int it = 0; it < 20; ++it) {
                float minSep = 0.0f;
                for (int q = 0; q < ni; ++q) minSep = b2min(minSep, solve_pcon(w, &ks[q], TOI_BAUMGARTE));
                ++ran;
                float now[3] = {w->c[i].x, w->c[i].y, w->a[i]};
                if (it >= 1 && f1 < 0 && memcmp(now, h1, 12) == 0) f1 = it;
                memcpy(h1, now, 12);
                if (minSep >= -1.5f * LINEAR_SLOP) break;
            }
            g_ins[4] += (long long)ran * ni;
            g_ins[5] += (long long)(f1 < 0 ? ran : f1) * ni;
        }"""),
    ("""        for (int it = 0; it < vel_iters; ++it)
            for (int q = 0; q < ni; ++q) solve_vcon(w, &ks[q]);
        float h = (1.0f - minAlpha) * dt;""",
     """        {
            int fixed_at = -1;
            for (int it = 0; it < vel_iters; ++it) {
                float snap[3 + 2 * ORA_MAX_STAT]; int ns_ = 0;
                snap[ns_++] = w->v[i].x; snap[ns_++] = w->v[i].y; snap[ns_++] = w->w[i];
                for (int q = 0; q < ni; ++q) { snap[ns_++] = ks[q].ni; snap[ns_++] = ks[q].ti; }
                for (int q = 0; q < ni; ++q) solve_vcon(w, &ks[q]);
                float now[3 + 2 * ORA_MAX_STAT]; int nn = 0;
                now[nn++] = w->v[i].x; now[nn++] = w->v[i].y; now[nn++] = w->w[i];
                for (int q = 0; q < ni; ++q) { now[nn++] = ks[q].ni; now[nn++] = ks[q].ti; }
                if (fixed_at < 0 && memcmp(snap, now, sizeof(float) * nn) == 0) fixed_at = it;
            }
            g_ins[6] += (long long)vel_iters * ni;
            g_ins[7] += (long long)(fixed_at < 0 ? vel_iters : fixed_at + 1) * ni;
        }
        float h = (1.0f - minAlpha) * dt;"""),
]
HEADER = """
#include <string.h>
static long long g_ins[16];
void ora_instr(long long* o, int reset) { for (int k = 0; k < 16; ++k) { o[k] = g_ins[k]; if (reset) g_ins[k] = 0; } }
"""


def build(tmp):
    os.makedirs(os.path.join(tmp, 'oracle'))
    shutil.copytree(os.path.join(ROOT, 'include'), os.path.join(tmp, 'include'))
    for f in os.listdir(os.path.join(ROOT, 'oracle')):
        if f.endswith(('.c', '.h')):
            shutil.copy(os.path.join(ROOT, 'oracle', f), os.path.join(tmp, 'oracle', f))
    path = os.path.join(tmp, 'oracle', 'mas_oracle.c')
    s = open(path).read()
    i = s.index('/* World step: Box2D b2World::Step')
    s = s[:i] + HEADER + s[i:]
    for old, new in PATCHES:
        assert old in s, old[:60]
        s = s.replace(old, new, 1)
    open(path, 'w').write(s)
    so = os.path.join(tmp, 'libinstr.so')
    subprocess.check_call(['gcc', '-O2', '-std=gnu11', '-fPIC', '-ffp-contract=off', '-shared', '-o', so,
                           path, os.path.join(tmp, 'oracle', 'ora_bench.c'), '-lm', '-lpthread'])
    return so


def main():
    import oracle
    from masurvival.config import NAMED_CONFIGS, ResolvedConfig, pcg64_state
    with tempfile.TemporaryDirectory() as tmp:
        oracle.LIB = build(tmp)
        L = oracle.lib()
        L.ora_instr.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]

        def rd():
            o = (ctypes.c_longlong * 16)()
            L.ora_instr(o, 1)
            return list(o)

        def show(tag, o):
            print(f'{tag}: island velocity iterations x contacts run {o[0]} needed {o[1]} ({100 * o[1] / max(o[0], 1):.0f}%); '
                  f'island position run {o[2]} needed {o[3]}; SolveTOI position run {o[4]} needed {o[5]} '
                  f'({100 * o[5] / max(o[4], 1):.0f}%); SolveTOI velocity run {o[6]} needed {o[7]} '
                  f'({100 * o[7] / max(o[6], 1):.0f}%)')
        rc = ResolvedConfig(NAMED_CONFIGS['2v2'])
        d = np.load(os.path.join(ROOT, 'profiles', 'r02_wedged_env.npz'))
        env = oracle.OracleEnv(rc.to_struct(), pcg64_state(int(d['env_seed'])))
        env.reset()
        rd()
        for t in range(len(d['actions'])):
            if env.step(d['actions'][t])[2]:
                env.reset()
        show('PPO-regime env with the SolveTOI cap', rd())
        rng = np.random.default_rng(0)
        envs = [oracle.OracleEnv(rc.to_struct(), pcg64_state(s)) for s in range(32)]
        for e in envs:
            e.reset()
        rd()
        for _ in range(300):
            for e in envs:
                if e.step(rng.integers(0, [3, 3, 3, 2, 2, 2], size=(4, 6)))[2]:
                    e.reset()
        show('32 random 2v2 envs x 300 steps', rd())


if __name__ == '__main__':
    main()
