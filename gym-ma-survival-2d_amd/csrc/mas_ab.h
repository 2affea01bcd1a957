// mas_ab.h -- TEST BUILDS ONLY (MAS_AB_KERNELS=1, make ab -> libmas_ab.so):
// the one-lane-per-env general physics path (k_gen_solve: Collide + island
// Solve of a whole env on one lane; k_gen_toi: SolveTOI on a lane group per
// (env, agent)) that the lane-group kernel k_gen_solve_g (mas_gensolve.h)
// replaced.  scripts/ab_solve_golden.py replays every golden episode through
// both and compares the state images after every step; the product library
// does not contain this code.  Restates Box2D 2.3.x b2World::Solve /
// b2Island::Solve / b2World::SolveTOI as oracle/mas_oracle.c does.
#pragma once

#include "mas_physics.h"

namespace mas {

template <class C>
struct StepScratch {
    V2 c0[C::AM];
    float a0[C::AM];
};

// polygon(A = static S) vs circle(B = agent I); returns touching, manifold out
template <class C, class KT>
__device__ __forceinline__ bool update_as_g(EnvL<C>& L, const Params& P, const KT& K, int I, int S,
                                            const StaticG& g, V2& ln, V2& lp)
{
    uint32_t tm = K.ast(I);
    bool was = bit(tm, S);
    bool touching = collide_pc(g.poly, g.p, g.q, sel(L.c, I), kPolyRadius, P.agent_r, ln, lp);
    if (!(touching && was)) {
        K.set_asni(I, S, 0.0f);
        K.set_asti(I, S, 0.0f);
    }
    K.set_ast(I, touching ? (tm | (1u << S)) : (tm & ~(1u << S)));
    if (touching != was) wake(L, I);
    return touching;
}

template <class C>
struct Slots {
    int n;
    int key[C::KC];  // type<<16 | i<<8 | js   (type 0: agent-agent j; 1: agent-static s)
    VC k[C::KC];
    V2 ln[C::KC], lp[C::KC];
};

template <class C>
__device__ __forceinline__ void static_pq(const EnvL<C>& L, const Params& P, int s, V2& sp, Rot& sq)
{
    sp = opq(P.wall_pos[0]);
    sq = P.wall_q[0];
    sq.s = opq(sq.s);
    sq.c = opq(sq.c);
#pragma unroll
    for (int k = 1; k < kNumWalls; ++k)
        if (s == k) { sp = opq(P.wall_pos[k]); sq.s = opq(P.wall_q[k].s); sq.c = opq(P.wall_q[k].c); }
#pragma unroll
    for (int b = 0; b < C::BM; ++b)
        if (s == kNumWalls + b) { sp = opq(L.bp[b]); sq = kIdRot; }
}

// Islands over touching agent-agent contacts (Box2D DFS; statics do not
// propagate): label[i] = the smallest agent index of i's island; returns the
// solved agents (members of islands with an awake member).
template <class C, class KT>
__device__ __forceinline__ uint32_t island_labels(const EnvL<C>& L, const KT& K, int (&label)[C::AM])
{
    constexpr int AM = C::AM;
#pragma unroll
    for (int i = 0; i < AM; ++i) label[i] = i;
    // (agent-agent contacts are rare: the whole wave skips the propagation
    // when none of its envs has one)
#pragma unroll
    for (int pass = 0; pass < AM; ++pass) {
        if (!__any(K.aat() != 0u)) continue;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = i + 1; j < AM; ++j) {
                int p = aa_index<AM>(i, j);
                if (bit(L.alive_m, i) && bit(L.alive_m, j) && bit(K.aat(), p)) {
                    int l = label[i] < label[j] ? label[i] : label[j];
                    label[i] = l;
                    label[j] = l;
                }
            }
    }
    uint32_t solved = 0;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < AM; ++j)
            if (label[j] == label[i] && bit(L.alive_m, j) && bit(L.awake_m, j)) any = true;
        if (bit(L.alive_m, i) && any) solved |= 1u << i;
    }
    return solved;
}

// b2Island::Solve over the solved agents, restricted to `only` (k_gen: one
// island per call, its root's lane; islands share no body, so solving them
// apart is solving them together)
template <class C, class KT>
__device__ __forceinline__ void world_solve(EnvL<C>& L, const Params& P, const KT& K, StepScratch<C>& S, float h,
                                            float dtRatio, uint32_t only = ~0u)
{
    constexpr int AM = C::AM;
    const float m = P.inv_mass, I = P.inv_I;
    int label[AM];
    const uint32_t solved = island_labels(L, K, label) & only;
    if (solved == 0) return;
#pragma unroll
    for (int i = 0; i < AM; ++i)
        if (bit(solved, i)) wake(L, i);
    // sweep start + damping (Pade)
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        if (!bit(solved, i)) continue;
        S.c0[i] = L.c[i];
        S.a0[i] = L.a[i];
        float ld = 1.0f / (1.0f + h * P.lin_damp);
        L.v[i].x *= ld;
        L.v[i].y *= ld;
        float ad = 1.0f / (1.0f + h * P.ang_damp);
        L.w[i] *= ad;
    }
    // compact contact list (canonical order)
    Slots<C> sl;
    sl.n = 0;
    bool overflow = false;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = i + 1; j < AM; ++j) {
            int p = aa_index<AM>(i, j);
            if (bit(solved, i) && bit(solved, j) && bit(K.aat(), p)) {
                if (sl.n < C::KC) {
                    VC k = vc_init_aa(L.c[i], L.c[j], P.agent_r, m, I, m, I);
                    k.ni = dtRatio * K.aani(p);
                    k.ti = dtRatio * K.aati(p);
                    int key = (0 << 16) | (i << 8) | j;
#pragma unroll
                    for (int q = 0; q < C::KC; ++q)
                        if (q == sl.n) { sl.key[q] = key; sl.k[q] = k; }
                }
                sl.n++;
            }
        }
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        uint32_t t = bit(solved, i) ? K.ast(i) : 0u;
        // touching statics of agent i in canonical order (per-lane loop: the
        // trip count is the lane's contact count, usually 0)
#pragma unroll 1
        while (t) {
            const int s = __builtin_ctz(t);
            t &= t - 1;
            if (sl.n < C::KC) {
                StaticG g = static_geom_dyn(L, P, s);
                V2 ln = mk(0.0f, 0.0f), lp = mk(0.0f, 0.0f);
                collide_pc(g.poly, g.p, g.q, L.c[i], kPolyRadius, P.agent_r, ln, lp);
                VC k = vc_init_as(g.p, g.q, ln, lp, L.c[i], P.agent_r, m, I);
                k.ni = dtRatio * K.asni(i, s);
                k.ti = dtRatio * K.asti(i, s);
                int key = (1 << 16) | (i << 8) | s;
#pragma unroll
                for (int q = 0; q < C::KC; ++q)
                    if (q == sl.n) { sl.key[q] = key; sl.k[q] = k; sl.ln[q] = ln; sl.lp[q] = lp; }
            }
            sl.n++;
        }
    }
    overflow = sl.n > C::KC;
    if (!overflow) {
        // ---------------- fast path: compact slots ----------------
        // warm start (slot loops: the wave skips slots none of its envs uses)
#pragma unroll
        for (int q = 0; q < C::KC; ++q) {
            if (!__any(q < sl.n)) continue;
            if (q >= sl.n) continue;
            int key = sl.key[q];
            int i = slot_i(key), js = slot_js(key);
            V2 vB, vA = mk(0.0f, 0.0f);
            float wB, wA = 0.0f;
            if (slot_type(key) == 0) {
                vA = sel(L.v, i); wA = sel(L.w, i);
                vB = sel(L.v, js); wB = sel(L.w, js);
                vc_warm(sl.k[q], vA, wA, vB, wB, m, I, m, I);
                put(L.v, i, vA); put(L.w, i, wA);
                put(L.v, js, vB); put(L.w, js, wB);
            } else {
                vB = sel(L.v, i); wB = sel(L.w, i);
                vc_warm(sl.k[q], vA, wA, vB, wB, 0.0f, 0.0f, m, I);
                put(L.v, i, vB); put(L.w, i, wB);
            }
        }
        for (int it = 0; it < 10; ++it) {
            if (!__any(sl.n > 0)) break;
            V2 vp[AM];
            float wp[AM], qn[C::KC], qt[C::KC];
#pragma unroll
            for (int i = 0; i < AM; ++i) {
                vp[i] = L.v[i];
                wp[i] = L.w[i];
            }
#pragma unroll
            for (int q = 0; q < C::KC; ++q) {
                qn[q] = sl.k[q].ni;
                qt[q] = sl.k[q].ti;
            }
#pragma unroll
            for (int q = 0; q < C::KC; ++q) {
                if (!__any(q < sl.n)) continue;
                if (q >= sl.n) continue;
                int key = sl.key[q];
                int i = slot_i(key), js = slot_js(key);
                V2 vB, vA = mk(0.0f, 0.0f);
                float wB, wA = 0.0f;
                if (slot_type(key) == 0) {
                    vA = sel(L.v, i); wA = sel(L.w, i);
                    vB = sel(L.v, js); wB = sel(L.w, js);
                    vc_solve(sl.k[q], vA, wA, vB, wB, m, I, m, I);
                    put(L.v, i, vA); put(L.w, i, wA);
                    put(L.v, js, vB); put(L.w, js, wB);
                } else {
                    vB = sel(L.v, i); wB = sel(L.w, i);
                    vc_solve(sl.k[q], vA, wA, vB, wB, 0.0f, 0.0f, m, I);
                    put(L.v, i, vB); put(L.w, i, wB);
                }
            }
            // fixed point of the whole env (see same_bits): every lane of the wave
            bool same = true;
#pragma unroll
            for (int i = 0; i < AM; ++i) same = same && same_bits(L.v[i], vp[i]) && same_bits(L.w[i], wp[i]);
#pragma unroll
            for (int q = 0; q < C::KC; ++q)
                if (q < sl.n) same = same && same_bits(sl.k[q].ni, qn[q]) && same_bits(sl.k[q].ti, qt[q]);
            if (!__any(!same)) break;
        }
        // store impulses
#pragma unroll
        for (int q = 0; q < C::KC; ++q) {
            if (!__any(q < sl.n)) continue;
            if (q >= sl.n) continue;
            int key = sl.key[q];
            int i = slot_i(key), js = slot_js(key);
            if (slot_type(key) == 0) {
                K.set_aani(aa_index<AM>(i, js), sl.k[q].ni);
                K.set_aati(aa_index<AM>(i, js), sl.k[q].ti);
            } else {
                K.set_asni(i, js, sl.k[q].ni);
                K.set_asti(i, js, sl.k[q].ti);
            }
        }
    } else {
        // ---------------- slow path: every candidate pair, recomputed ----------------
        // (runtime loops, agent / static data through sel/put: this path only
        // runs for an env with more touching contacts than compact slots)
        V2 cpos[AM];
#pragma unroll
        for (int i = 0; i < AM; ++i) cpos[i] = L.c[i];
#pragma unroll 1
        for (int it = -2; it < 10; ++it) {  // -2: scale stored impulses, -1: warm start
#pragma unroll 1
            for (int i = 0; i < AM; ++i) {
#pragma unroll 1
                for (int j = i + 1; j < AM; ++j) {
                    int p = aa_index<AM>(i, j);
                    if (!(bit(solved, i) && bit(solved, j) && bit(K.aat(), p))) continue;
                    float ni = K.aani(p), ti = K.aati(p);
                    if (it == -2) {
                        K.set_aani(p, dtRatio * ni);
                        K.set_aati(p, dtRatio * ti);
                        continue;
                    }
                    VC k = vc_init_aa(sel(cpos, i), sel(cpos, j), P.agent_r, m, I, m, I);
                    k.ni = ni;
                    k.ti = ti;
                    V2 vA = sel(L.v, i), vB = sel(L.v, j);
                    float wA = sel(L.w, i), wB = sel(L.w, j);
                    if (it < 0) vc_warm(k, vA, wA, vB, wB, m, I, m, I);
                    else vc_solve(k, vA, wA, vB, wB, m, I, m, I);
                    put(L.v, i, vA); put(L.w, i, wA);
                    put(L.v, j, vB); put(L.w, j, wB);
                    K.set_aani(p, k.ni);
                    K.set_aati(p, k.ti);
                }
            }
#pragma unroll 1
            for (int i = 0; i < AM; ++i) {
                if (!bit(solved, i)) continue;
                uint32_t tm = K.ast(i);
#pragma unroll 1
                for (int s = 0; s < C::NS; ++s) {
                    if (!bit(tm, s)) continue;
                    float ni = K.asni(i, s), ti = K.asti(i, s);
                    if (it == -2) {
                        K.set_asni(i, s, dtRatio * ni);
                        K.set_asti(i, s, dtRatio * ti);
                        continue;
                    }
                    StaticG g = static_geom_dyn(L, P, s);
                    V2 ci = sel(cpos, i);
                    V2 ln = mk(0.0f, 0.0f), lp = mk(0.0f, 0.0f);
                    collide_pc(g.poly, g.p, g.q, ci, kPolyRadius, P.agent_r, ln, lp);
                    VC k = vc_init_as(g.p, g.q, ln, lp, ci, P.agent_r, m, I);
                    k.ni = ni;
                    k.ti = ti;
                    V2 vz = mk(0.0f, 0.0f), vB = sel(L.v, i);
                    float wz = 0.0f, wB = sel(L.w, i);
                    if (it < 0) vc_warm(k, vz, wz, vB, wB, 0.0f, 0.0f, m, I);
                    else vc_solve(k, vz, wz, vB, wB, 0.0f, 0.0f, m, I);
                    put(L.v, i, vB); put(L.w, i, wB);
                    K.set_asni(i, s, k.ni);
                    K.set_asti(i, s, k.ti);
                }
            }
        }
    }
    // integrate positions
#pragma unroll
    for (int i = 0; i < AM; ++i)
        if (bit(solved, i)) integrate(L.c[i], L.a[i], L.v[i], L.w[i], h);
    // position iterations with per-island early exit
    uint32_t done_isl = 0;  // bit per island root
    uint32_t solved_isl = 0;
    for (int it = 0; it < 10; ++it) {
        float minsep[AM];
#pragma unroll
        for (int r = 0; r < AM; ++r) minsep[r] = 0.0f;
        if (!overflow) {
#pragma unroll
            for (int q = 0; q < C::KC; ++q) {
                if (!__any(q < sl.n)) continue;
                if (q >= sl.n) continue;
                int key = sl.key[q];
                int i = slot_i(key), js = slot_js(key);
                int root = sel(label, i);
                if (bit(done_isl, root)) continue;
                float sep;
                if (slot_type(key) == 0) {
                    V2 cA = sel(L.c, i), cB = sel(L.c, js);
                    float aA = sel(L.a, i), aB = sel(L.a, js);
                    sep = pc_solve_aa(cA, aA, cB, aB, P.agent_r, m, I, kBaumgarte);
                    put(L.c, i, cA); put(L.a, i, aA);
                    put(L.c, js, cB); put(L.a, js, aB);
                } else {
                    V2 sp;
                    Rot sq;
                    static_pq(L, P, js, sp, sq);
                    V2 cB = sel(L.c, i);
                    float aB = sel(L.a, i);
                    sep = pc_solve_as(sp, sq, sl.ln[q], sl.lp[q], cB, aB, P.agent_r, m, I, kBaumgarte, P.inv_mass_rcp);
                    put(L.c, i, cB); put(L.a, i, aB);
                }
#pragma unroll
                for (int r = 0; r < AM; ++r)
                    if (r == root) minsep[r] = fmin_b2(minsep[r], sep);
            }
        } else {
#pragma unroll 1
            for (int i = 0; i < AM; ++i)
#pragma unroll 1
                for (int j = i + 1; j < AM; ++j) {
                    int p = aa_index<AM>(i, j);
                    if (!(bit(solved, i) && bit(solved, j) && bit(K.aat(), p))) continue;
                    int root = sel(label, i);
                    if (bit(done_isl, root)) continue;
                    V2 cA = sel(L.c, i), cB = sel(L.c, j);
                    float aA = sel(L.a, i), aB = sel(L.a, j);
                    float sep = pc_solve_aa(cA, aA, cB, aB, P.agent_r, m, I, kBaumgarte);
                    put(L.c, i, cA); put(L.a, i, aA);
                    put(L.c, j, cB); put(L.a, j, aB);
                    put(minsep, root, fmin_b2(sel(minsep, root), sep));
                }
#pragma unroll 1
            for (int i = 0; i < AM; ++i) {
                if (!bit(solved, i)) continue;
                uint32_t tm = K.ast(i);
                int root = sel(label, i);
#pragma unroll 1
                for (int s = 0; s < C::NS; ++s) {
                    if (!bit(tm, s) || bit(done_isl, root)) continue;
                    StaticG g = static_geom_dyn(L, P, s);
                    V2 ln = mk(0.0f, 0.0f), lp = mk(0.0f, 0.0f);
                    collide_pc(g.poly, g.p, g.q, sel(S.c0, i), kPolyRadius, P.agent_r, ln, lp);
                    V2 cB = sel(L.c, i);
                    float aB = sel(L.a, i);
                    float sep = pc_solve_as(g.p, g.q, ln, lp, cB, aB, P.agent_r, m, I, kBaumgarte, P.inv_mass_rcp);
                    put(L.c, i, cB); put(L.a, i, aB);
                    put(minsep, root, fmin_b2(sel(minsep, root), sep));
                }
            }
        }
        // islands whose minimum separation is acceptable are done
        uint32_t all_done = 1;
#pragma unroll
        for (int r = 0; r < AM; ++r) {
            bool is_root = false;
#pragma unroll
            for (int i = 0; i < AM; ++i)
                if (bit(solved, i) && label[i] == r) is_root = true;
            if (!is_root || bit(done_isl, r)) continue;
            if (minsep[r] >= -3.0f * kLinearSlop) {
                done_isl |= 1u << r;
                solved_isl |= 1u << r;
            } else {
                all_done = 0;
            }
        }
        if (all_done) break;
    }
    // sleep (per island)
    const float linTolSqr = kLinSleepTol * kLinSleepTol;
    const float angTolSqr = kAngSleepTol * kAngSleepTol;
    float minSleep[AM];
#pragma unroll
    for (int r = 0; r < AM; ++r) minSleep[r] = kMaxFloat;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        if (!bit(solved, i)) continue;
        int r = label[i];
        float ms = sel(minSleep, r);
        // branch-free selects, as world_step_fast / gen_solve_group
        const bool moving = (L.w[i] * L.w[i] > angTolSqr) | (dot(L.v[i], L.v[i]) > linTolSqr);
        const float acc = opq(L.sleep[i] + h);
        L.sleep[i] = moving ? 0.0f : acc;
        ms = moving ? 0.0f : fmin_b2(ms, acc);
        put(minSleep, r, ms);
    }
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        if (!bit(solved, i)) continue;
        int r = label[i];
        if (sel(minSleep, r) >= kTimeToSleep && bit(solved_isl, r)) {
            L.awake_m &= ~(1u << i);
            L.sleep[i] = 0.0f;
            L.v[i] = mk(0.0f, 0.0f);
            L.w[i] = 0.0f;
        }
    }
}

// b2World::SolveTOI for agent I (events of different agents are independent:
// statics never move and agent-agent pairs are not TOI pairs).
// Returns the number of TOI events, + 65536 when a contact reached
// b2_maxSubSteps (test diagnostics, Params::toi_diag).
template <class C, class KT>
__device__ __forceinline__ int toi_agent(EnvL<C>& L, const Params& P, const KT& K, const StepScratch<C>& S, int I,
                                         float dt)
{
    int events = 0;
    const float m = P.inv_mass, Ii = P.inv_I;
    Sweep sw;
    sw.c0 = sel(S.c0, I);
    sw.a0 = sel(S.a0, I);
    sw.c = sel(L.c, I);
    sw.a = sel(L.a, I);
    sw.alpha0 = 0.0f;
    const int ns = kNumWalls + L.nbox;
    float toi[C::NS];
    int cnt[C::NS];
#pragma unroll
    for (int s = 0; s < C::NS; ++s) { toi[s] = 1.0f; cnt[s] = 0; }
    uint32_t valid = 0, enabled = 0xffffffffu;
#ifdef MAS_PROFILE
    unsigned long long nev = 0, ntoi = 0, npos = 0, lt = wall_clock64(), tp[5] = {0, 0, 0, 0, 0};
#define MAS_LT(k)                                 \
    do {                                          \
        const unsigned long long n_ = wall_clock64(); \
        tp[k] += n_ - lt;                         \
        lt = n_;                                  \
    } while (0)
#else
#define MAS_LT(k) ((void)0)
#endif
    for (int guard = 0; guard < 9 * C::NS + 1; ++guard) {
        // (1) statics whose cached TOI is stale: the conservative pre-test
        //     settles most of them at alpha = 1 (unrolled, cheap)
        uint32_t need = 0;
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            if (s >= ns || !bit(enabled, s) || cnt[s] > 8 || bit(valid, s)) continue;
            StaticG g = static_geom(L, P, s);
            if (toi_reject(g, sw.c0, sw.c, P.agent_r)) {
                toi[s] = 1.0f;
                valid |= 1u << s;
            } else {
                need |= 1u << s;
            }
        }
        MAS_PROF(P, 21);
        MAS_LT(0);
        // (2) full b2TimeOfImpact for the rest (runtime loop: one code copy)
#pragma unroll 1
        while (need) {
            int s = __builtin_ctz(need);
            need &= need - 1;
            StaticG g = static_geom_dyn(L, P, s);
            const ToiPoly T = toi_poly(g.poly, g.p, g.angle);
            float beta;
#ifdef MAS_PROFILE
            ++ntoi;
#endif
            int st = time_of_impact(T, sw, P.agent_r, beta);
            float alpha = 1.0f;
            if (st == kToiTouching) alpha = fmin_b2(sw.alpha0 + (1.0f - sw.alpha0) * beta, 1.0f);
            put(toi, s, alpha);
            valid |= 1u << s;
        }
        MAS_PROF(P, 22);
        MAS_LT(1);
        // (3) minimum over the enabled contacts (ties: lowest canonical index)
        float minAlpha = 1.0f;
        int minS = -1;
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            if (s >= ns || !bit(enabled, s) || cnt[s] > 8) continue;
            if (toi[s] < minAlpha) {
                minAlpha = toi[s];
                minS = s;
            }
        }
        if (minS < 0 || 1.0f - 10.0f * kEps < minAlpha) break;
#ifdef MAS_PROFILE
        ++nev;
#endif
        Sweep backup = sw;
        {
            float beta = (minAlpha - sw.alpha0) / (1.0f - sw.alpha0);
            sw.c0 = add(sw.c0, scl(beta, sub(sw.c, sw.c0)));
            sw.a0 += beta * (sw.a - sw.a0);
            sw.alpha0 = minAlpha;
            sw.c = sw.c0;
            sw.a = sw.a0;
        }
        put(L.c, I, sw.c);
        put(L.a, I, sw.a);
        StaticG gm = static_geom_dyn(L, P, minS);
        V2 lnm = mk(0.0f, 0.0f), lpm = mk(0.0f, 0.0f);
        bool touching = update_as_g(L, P, K, I, minS, gm, lnm, lpm);
        valid &= ~(1u << minS);
#pragma unroll
        for (int s = 0; s < C::NS; ++s)
            if (s == minS) cnt[s] += 1;
        if (!touching) {
            enabled &= ~(1u << minS);
            sw = backup;
            put(L.c, I, sw.c);
            put(L.a, I, sw.a);
            continue;
        }
        wake(L, I);
        ++events;
        // island: the min contact first, then the agent's other touching statics
        uint32_t isl = 0;
        V2 iln[C::NS], ilp[C::NS];
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            iln[s] = mk(0.0f, 0.0f);
            ilp[s] = mk(0.0f, 0.0f);
            if (s >= ns || s == minS) continue;
            enabled |= 1u << s;
            StaticG g = static_geom(L, P, s);
            if (update_as_g(L, P, K, I, s, g, iln[s], ilp[s])) isl |= 1u << s;
        }
        MAS_LT(2);
        // b2Island::SolveTOI: position iterations (TOI Baumgarte) ...
        V2 cB = sel(L.c, I);
        float aB = sel(L.a, I);
        for (int it = 0; it < 20; ++it) {
#ifdef MAS_PROFILE
            ++npos;
#endif
            float minsep = 0.0f;
            minsep = fmin_b2(minsep, pc_solve_as(gm.p, gm.q, lnm, lpm, cB, aB, P.agent_r, m, Ii, kToiBaumgarte, P.inv_mass_rcp));
#pragma unroll
            for (int s = 0; s < C::NS; ++s) {
                if (!bit(isl, s)) continue;
                StaticG g = static_geom(L, P, s);
                minsep = fmin_b2(minsep, pc_solve_as(g.p, g.q, iln[s], ilp[s], cB, aB, P.agent_r, m, Ii, kToiBaumgarte, P.inv_mass_rcp));
            }
            if (minsep >= -1.5f * kLinearSlop) break;
        }
        MAS_LT(3);
        sw.c0 = cB;
        sw.a0 = aB;
        // ... then 10 velocity iterations without warm starting
        V2 vB = sel(L.v, I);
        float wB = sel(L.w, I);
        float nim = 0.0f, tim = 0.0f;
        float ni[C::NS], ti[C::NS];
#pragma unroll
        for (int s = 0; s < C::NS; ++s) { ni[s] = 0.0f; ti[s] = 0.0f; }
        for (int it = 0; it < 10; ++it) {
            {
                VC k = vc_init_as(gm.p, gm.q, lnm, lpm, cB, P.agent_r, m, Ii);
                k.ni = nim;
                k.ti = tim;
                V2 vz = mk(0.0f, 0.0f);
                float wz = 0.0f;
                vc_solve(k, vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                nim = k.ni;
                tim = k.ti;
            }
#pragma unroll
            for (int s = 0; s < C::NS; ++s) {
                if (!bit(isl, s)) continue;
                StaticG g = static_geom(L, P, s);
                VC k = vc_init_as(g.p, g.q, iln[s], ilp[s], cB, P.agent_r, m, Ii);
                k.ni = ni[s];
                k.ti = ti[s];
                V2 vz = mk(0.0f, 0.0f);
                float wz = 0.0f;
                vc_solve(k, vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                ni[s] = k.ni;
                ti[s] = k.ti;
            }
        }
        float h = (1.0f - minAlpha) * dt;
        integrate(cB, aB, vB, wB, h);
        put(L.c, I, cB);
        put(L.a, I, aB);
        put(L.v, I, vB);
        put(L.w, I, wB);
        sw.c = cB;
        sw.a = aB;
        valid = 0;
        MAS_PROF(P, 24);
        MAS_LT(4);
    }
    put(L.c, I, sw.c);
    put(L.a, I, sw.a);
#ifdef MAS_PROFILE
    // per-lane SolveTOI work: max events / b2TimeOfImpact calls / position
    // iterations over the launch's lanes, and the event total
    atomicMax(&P.prof[48], nev);
    atomicMax(&P.prof[49], ntoi);
    atomicMax(&P.prof[50], npos);
    atomicAdd(&P.prof[51], nev);
    atomicAdd(&P.prof[52], ntoi);
    for (int k = 0; k < 5; ++k) atomicMax(&P.prof[53 + k], tp[k]);
#endif
#undef MAS_LT
    bool capped = false;
#pragma unroll
    for (int s = 0; s < C::NS; ++s) capped = capped || (s < ns && bit(enabled, s) && cnt[s] > 8);
    return events + (capped ? 65536 : 0);
}


// b2World::Step(dt, 10, 10) up to SolveTOI: Collide + Solve.  S returns the
// sweep start (b2Sweep c0/a0) of every agent for SolveTOI, which runs as its
// own kernel, one lane per (env, agent) (k_gen_toi): TOI events of different
// agents are independent (statics never move, agent-agent pairs are not TOI
// pairs, and every agent SolveTOI touches is already awake).
template <class C, class KT>
__device__ __forceinline__ void world_step_solve(EnvL<C>& L, const Params& P, const KT& K, float dt,
                                                 StepScratch<C>& S)
{
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        S.c0[i] = L.c[i];
        S.a0[i] = L.a[i];
    }
    float inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
    float dtRatio = L.inv_dt0 * dt;
    // Collide: agent-agent pairs, then agent-static pairs (canonical order)
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
#pragma unroll
        for (int j = i + 1; j < C::AM; ++j) {
            if (!(bit(L.alive_m, i) && bit(L.alive_m, j))) continue;
            if (!(bit(L.awake_m, i) || bit(L.awake_m, j))) continue;
            int p = aa_index<C::AM>(i, j);
            const uint32_t at = K.aat();
            bool was = bit(at, p);
            V2 d = sub(L.c[j], L.c[i]);
            float dsq = dot(d, d);
            float rad = P.agent_r + P.agent_r;
            bool touching = !(dsq > rad * rad);
            if (!(touching && was)) {
                K.set_aani(p, 0.0f);
                K.set_aati(p, 0.0f);
            }
            K.set_aat(touching ? (at | (1u << p)) : (at & ~(1u << p)));
            if (touching != was) {
                wake(L, i);
                wake(L, j);
            }
        }
    // agent-static pairs: the exact b2CollidePolygonAndCircle runs only for
    // pairs a cheap test cannot rule out (circle vs the static's AABB, with a
    // margin): a pair beyond it has separation > radius, so the exact result
    // would be "not touching".  Those pairs are updated with mask arithmetic
    // (impulses reset, wake on a lost contact) -- the same state changes
    // b2Contact::Update makes -- and the survivors go through the exact update
    // in a per-lane loop whose trip count is the lane's survivor count.
    const int ns = kNumWalls + L.nbox;
    const float reach = P.agent_r + kPolyRadius + 1e-3f;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!(bit(L.alive_m, i) && bit(L.awake_m, i))) continue;
        const V2 ci = L.c[i];
        uint32_t cand = 0;
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            if (s >= ns) continue;
            V2 lo, hi;
            if (s < kNumWalls) {
                lo = P.wall_lo[s];
                hi = P.wall_hi[s];
            } else {
                const int b = s - kNumWalls;
                lo = mk(L.bp[b].x - L.bhx[b], L.bp[b].y - L.bhy[b]);
                hi = mk(L.bp[b].x + L.bhx[b], L.bp[b].y + L.bhy[b]);
            }
            const float dx = fmaxf(fmaxf(lo.x - ci.x, ci.x - hi.x), 0.0f);
            const float dy = fmaxf(fmaxf(lo.y - ci.y, ci.y - hi.y), 0.0f);
            if (dx * dx + dy * dy <= reach * reach) cand |= 1u << s;
        }
        const uint32_t lost = K.ast(i) & ~cand;
        if (lost) {
            wake(L, i);
#pragma unroll
            for (int s = 0; s < C::NS; ++s)
                if (bit(lost, s)) { K.set_asni(i, s, 0.0f); K.set_asti(i, s, 0.0f); }
            K.set_ast(i, K.ast(i) & cand);
        }
#pragma unroll 1
        while (cand) {
            const int s = __builtin_ctz(cand);
            cand &= cand - 1;
            StaticG g = static_geom_dyn(L, P, s);
            V2 ln, lp;
            update_as_g(L, P, K, i, s, g, ln, lp);
        }
    }
    MAS_PROF(P, kPfCollide);
    world_solve(L, P, K, S, dt, dtRatio);
    MAS_PROF(P, kPfSolve);
    L.inv_dt0 = inv_dt;
}

}  // namespace mas
