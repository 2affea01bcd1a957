// mas_gensolve.h -- b2World::Step Collide + island Solve of the general
// physics path on a lane group per env (k_gen_solve_g, mas_kernels.inc).
//
// Same state changes, bit for bit, as world_step_solve (mas_ab.h, test builds) --
// the one-lane-per-env form this replaces, itself the restatement of
// b2World::Step up to SolveTOI (Box2D 2.3.x b2World::Solve, b2Island::Solve,
// b2ContactSolver) that oracle/mas_oracle.c pins:
//
//   Collide   agent-agent pairs: few and order-dependent (a wake makes a
//             later pair of the same agent eligible), so every lane of the
//             group runs the short pair loop on the same values; lane p
//             writes pair p's impulse reset.  Agent-static pairs: lane s of
//             the group owns static s and updates (agent i, s) for every
//             awake agent i -- the AABB cull, b2CollidePolygonAndCircle and
//             the impulse reset on its lane; a wave ballot per agent gives
//             the new touching word.  (An agent-static update only wakes an
//             agent that is already awake, so these pairs are independent.)
//   Solve     every lane labels the islands (uniform).  The velocity
//             constraints are initialised in parallel, each on the lane that
//             owns the contact (lane p: agent pair p; lane s: agent-static
//             pairs of static s), and written to LDS at the contact's
//             canonical index (agent-agent i<j, then agent-static
//             agent-major, statics ascending: ballot + popcount prefix).
//             Lane r (agent r) then runs b2Island::Solve for the island it
//             roots: warm start, 10 velocity iterations, impulse store,
//             integration, <= 10 position iterations with the island's
//             early exit, sleep.  Islands share no body and no contact, so
//             solving them apart, each in canonical order, is solving them
//             together; the Gauss-Seidel loops stop at an exact fixed point
//             (same_bits, mas_physics.h), per island.
//
// A group is G lanes (G >= statics, agent pairs and agents), 64 / G envs per
// wave, over the compacted general-path list: where the one-lane kernel ran
// every flagged env's serial Collide (A x (B + 4) pairs) and whole-env solve
// on one lane, a wave here waits for its slowest island.
#pragma once

#include "mas_step.h"

namespace mas {

template <class C>
struct SolveShape {
    static constexpr int need0 = C::NS > C::NAA ? C::NS : C::NAA;
    static constexpr int need = need0 > C::AM ? need0 : C::AM;
    static constexpr int G = need <= 8 ? 8 : (need <= 16 ? 16 : 32);  // lanes per env
    static constexpr int EPW = kWG / G;                               // envs per wave
    static constexpr int KL = C::NAA + C::AM * C::NS;                 // contact records per env
    static constexpr int KR = C::KC < 4 ? C::KC : 4;                  // island contacts held in registers
    static_assert(need <= 32, "one lane per static / agent pair, 32-bit group ballots");
};

// contact record fields in LDS ([field][q][env of the wave])
enum {
    kRnx, kRny, kRax, kRay, kRbx, kRby, kRnm, kRtm,  // VC: normal, rA, rB, normal / tangent mass
    kRni, kRti,                                      // accumulated impulses (warm-started)
    kRkey,                                           // type << 16 | i << 8 | j-or-static (slot_* helpers)
    kRpnx, kRpny, kRppx, kRppy,                      // agent-static: world normal / plane point (position solve)
    kRecW
};

template <class C>
struct SolveRec {
    float* f;
    int slot;
    __device__ __forceinline__ float& at(int field, int q) const
    {
        return f[(field * SolveShape<C>::KL + q) * SolveShape<C>::EPW + slot];
    }
};

// ballot bits of this lane's group (group-relative lane order)
template <int G>
__device__ __forceinline__ uint32_t group_ballot(bool b)
{
    const int base = (int)(threadIdx.x & 63) & ~(G - 1);
    const uint64_t m = __ballot(b);
    return (uint32_t)((m >> base) & ((1ull << G) - 1ull));
}

template <int G>
__device__ __forceinline__ uint32_t group_or(uint32_t v)
{
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// static s's body (walls 0..3 from P, box s-4 from its state words) and its
// world AABB (world_step_solve's cull)
template <class C>
__device__ __forceinline__ void group_static(const Params& P, const uint32_t* __restrict__ state, int64_t N, int64_t e,
                                             bool load, int s, StaticG& g, V2& lo, V2& hi, float& bhx, float& bhy,
                                             int& bmeta)
{
    bhx = bhy = 0.0f;
    bmeta = 0;
    if (s < kNumWalls) {
        V2 wp = opq(P.wall_pos[0]), wl = opq(P.wall_lo[0]), wh = opq(P.wall_hi[0]);
        Rot wq = P.wall_q[0];
        float wa = P.wall_angle[0];
#pragma unroll
        for (int k = 1; k < kNumWalls; ++k)
            if (s == k) {
                wp = opq(P.wall_pos[k]);
                wl = opq(P.wall_lo[k]);
                wh = opq(P.wall_hi[k]);
                wq.s = opq(P.wall_q[k].s);
                wq.c = opq(P.wall_q[k].c);
                wa = opq(P.wall_angle[k]);
            }
        g.p = wp;
        g.q = wq;
        g.angle = wa;
        g.poly = P.wall_poly;
        lo = wl;
        hi = wh;
    } else {
        using TW = StateWords<C>;
        const int b = s - kNumWalls < C::BM ? s - kNumWalls : C::BM - 1;
        const int wb = TW::box + 1 + 6 * b;
        V2 bp = mk(0.0f, 0.0f);
        float hx = 0.0f, hy = 0.0f;
        int meta = 0;
        if (load) {
            bp = mk(__uint_as_float(state[state_index(wb, e, N)]), __uint_as_float(state[state_index(wb + 1, e, N)]));
            hx = __uint_as_float(state[state_index(wb + 2, e, N)]);
            hy = __uint_as_float(state[state_index(wb + 3, e, N)]);
            meta = (int)state[state_index(wb + 4, e, N)];
        }
        g.p = bp;
        g.q = kIdRot;
        g.angle = 0.0f;
        g.poly = box_poly(hx, hy, box_rot(meta), box_copied(meta));
        bhx = hx;
        bhy = hy;
        bmeta = meta;
        lo = mk(bp.x - hx, bp.y - hy);
        hi = mk(bp.x + hx, bp.y + hy);
    }
}

// b2Island::Solve of one island whose n <= KC contacts (record indices qi,
// canonical order) are held in registers: warm start, 10 velocity
// iterations (exact fixed-point exit), impulse store, integration, <= 10
// position iterations with the island's early exit, sleep.  The same
// operations in the same order as the LDS loops of gen_solve_group (and as
// world_solve, mas_ab.h).  new_awake: the members still awake.
template <class C, class KT>
__device__ __forceinline__ void island_solve_regs(const Params& P, const SolveRec<C>& R, const KT& K,
                                                  const int (&qi)[SolveShape<C>::KR], int n, uint32_t members, V2 (&c)[C::AM],
                                                  float (&a)[C::AM], V2 (&v)[C::AM], float (&w)[C::AM],
                                                  float (&sl)[C::AM], float dt, uint32_t& new_awake)
{
    constexpr int KC = SolveShape<C>::KR, AM = C::AM;
    const float m = P.inv_mass, Ii = P.inv_I;
    VC k[KC];
    int key[KC];
    V2 pn[KC], pp[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const int q = j < n ? qi[j] : 0;
        k[j].normal = mk(R.at(kRnx, q), R.at(kRny, q));
        k[j].rA = mk(R.at(kRax, q), R.at(kRay, q));
        k[j].rB = mk(R.at(kRbx, q), R.at(kRby, q));
        k[j].nm = R.at(kRnm, q);
        k[j].tm = R.at(kRtm, q);
        k[j].ni = R.at(kRni, q);
        k[j].ti = R.at(kRti, q);
        key[j] = __float_as_int(R.at(kRkey, q));
        pn[j] = mk(R.at(kRpnx, q), R.at(kRpny, q));
        pp[j] = mk(R.at(kRppx, q), R.at(kRppy, q));
    }
    // one contact's velocity step (warm start or solve) on the bodies
    auto vel = [&](int j, bool warm) {
        const int i = slot_i(key[j]), js = slot_js(key[j]);
        V2 vA = mk(0.0f, 0.0f), vB;
        float wA = 0.0f, wB;
        if (slot_type(key[j]) == 0) {
            vA = sel(v, i); wA = sel(w, i);
            vB = sel(v, js); wB = sel(w, js);
            if (warm) vc_warm(k[j], vA, wA, vB, wB, m, Ii, m, Ii);
            else vc_solve(k[j], vA, wA, vB, wB, m, Ii, m, Ii);
            put(v, i, vA); put(w, i, wA);
            put(v, js, vB); put(w, js, wB);
        } else {
            vB = sel(v, i); wB = sel(w, i);
            if (warm) vc_warm(k[j], vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
            else vc_solve(k[j], vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
            put(v, i, vB); put(w, i, wB);
        }
    };
#pragma unroll
    for (int j = 0; j < KC; ++j)
        if (j < n) vel(j, true);
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        V2 vp[AM];
        float wp[AM], qn[KC], qt[KC];
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            vp[j] = v[j];
            wp[j] = w[j];
        }
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            qn[j] = k[j].ni;
            qt[j] = k[j].ti;
        }
#pragma unroll
        for (int j = 0; j < KC; ++j)
            if (j < n) vel(j, false);
        bool same = true;
#pragma unroll
        for (int j = 0; j < AM; ++j) same = same && same_bits(v[j], vp[j]) && same_bits(w[j], wp[j]);
#pragma unroll
        for (int j = 0; j < KC; ++j)
            if (j < n) same = same && same_bits(k[j].ni, qn[j]) && same_bits(k[j].ti, qt[j]);
        if (same) break;
    }
    // store impulses
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= n) continue;
        const int i = slot_i(key[j]), js = slot_js(key[j]);
        if (slot_type(key[j]) == 0) {
            const int p = aa_index<AM>(i, js);
            K.set_aani(p, k[j].ni);
            K.set_aati(p, k[j].ti);
        } else {
            K.set_asni(i, js, k[j].ni);
            K.set_asti(i, js, k[j].ti);
        }
    }
#pragma unroll
    for (int j = 0; j < AM; ++j)
        if (bit(members, j)) integrate(c[j], a[j], v[j], w[j], dt);
    bool converged = false;
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        float minsep = 0.0f;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= n) continue;
            const int i = slot_i(key[j]), js = slot_js(key[j]);
            float sep;
            if (slot_type(key[j]) == 0) {
                V2 cA = sel(c, i), cB = sel(c, js);
                float aA = sel(a, i), aB = sel(a, js);
                sep = pc_solve_aa(cA, aA, cB, aB, P.agent_r, m, Ii, kBaumgarte);
                put(c, i, cA); put(a, i, aA);
                put(c, js, cB); put(a, js, aB);
            } else {
                V2 cB = sel(c, i);
                float aB = sel(a, i);
                sep = pc_solve_as_h(pn[j], pp[j], cB, aB, P.agent_r, m, Ii, kBaumgarte, P.inv_mass_rcp);
                put(c, i, cB); put(a, i, aB);
            }
            minsep = fmin_b2(minsep, sep);
        }
        if (minsep >= -3.0f * kLinearSlop) {
            converged = true;
            break;
        }
    }
    // sleep (branch-free: see gen_solve_group)
    const float linTolSqr = kLinSleepTol * kLinSleepTol;
    const float angTolSqr = kAngSleepTol * kAngSleepTol;
    float ms = kMaxFloat;
#pragma unroll
    for (int j = 0; j < AM; ++j) {
        const float ww = w[j] * w[j], vv = dot(v[j], v[j]);
        const bool moving = (ww > angTolSqr) | (vv > linTolSqr);
        const float acc = opq(sl[j] + dt);
        const bool mem = bit(members, j);
        sl[j] = mem ? (moving ? 0.0f : acc) : sl[j];
        ms = mem ? (moving ? 0.0f : fmin_b2(ms, acc)) : ms;
    }
    new_awake = members;
    if (ms >= kTimeToSleep && converged) {
        new_awake = 0;
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            if (!bit(members, j)) continue;
            sl[j] = 0.0f;
            v[j] = mk(0.0f, 0.0f);
            w[j] = 0.0f;
        }
    }
}

// MAS_ISLAND_K=0: every multi-body island through island_solve_regs (A/B).
// On for the classes with few statics only: the FFA classes' general kernel
// went 245 -> 256 VGPRs with it and measured 1.2 % slower (r06s), the 2v2
// class's 2 % faster
#ifndef MAS_ISLAND_K
#define MAS_ISLAND_K 1
#endif
template <class C>
constexpr bool kIslandK = MAS_ISLAND_K && C::AM > 2 && C::NS <= 8;
// island_solve_regs for an island of exactly NB (2 or 3) bodies: the members
// are gathered into NB compact slots (ascending agent index) and every
// contact's bodies re-indexed into them once, so each contact step selects
// out of NB registers instead of AM (one v_cndmask per component instead of
// AM - 1 to read, NB instead of AM to write back; the agent pair of a
// two-body island touches slots 0 and 1 with no selection at all).  The same
// operations on the same values in the same order: the contacts in
// canonical order, the fixed-point test over the members and the contacts
// (the other bodies never change), integration and sleep over the members
// ascending -- so the same bits.
template <class C, int NB, class KT>
__device__ __forceinline__ void island_solve_k(const Params& P, const SolveRec<C>& R, const KT& K,
                                               const int (&qi)[SolveShape<C>::KR], int n, uint32_t members,
                                               V2 (&c)[C::AM], float (&a)[C::AM], V2 (&v)[C::AM],
                                               float (&w)[C::AM], float (&sl)[C::AM], float dt, uint32_t& new_awake)
{
    constexpr int KC = SolveShape<C>::KR, AM = C::AM;
    static_assert(NB >= 1 && NB <= AM, "compact islands");  // (NB 1: a dead instantiation of the small classes)
    const float m = P.inv_mass, Ii = P.inv_I;
    // the members, ascending, into slots 0..NB-1
    int idx[NB];
    {
        uint32_t mm = members;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            idx[k] = __ffs(mm) - 1;
            mm &= mm - 1u;
        }
    }
    V2 cc[NB], vv[NB];
    float aa[NB], ww[NB], ss[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        cc[k] = sel(c, idx[k]);
        aa[k] = sel(a, idx[k]);
        vv[k] = sel(v, idx[k]);
        ww[k] = sel(w, idx[k]);
        ss[k] = sel(sl, idx[k]);
    }
    // slot of agent i among the members (i a member)
    auto slot_of = [&](int i) { return __popc(members & ((1u << i) - 1u)); };
    VC k[KC];
    int key[KC], si[KC], sj[KC];
    V2 pn[KC], pp[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const int q = j < n ? qi[j] : 0;
        k[j].normal = mk(R.at(kRnx, q), R.at(kRny, q));
        k[j].rA = mk(R.at(kRax, q), R.at(kRay, q));
        k[j].rB = mk(R.at(kRbx, q), R.at(kRby, q));
        k[j].nm = R.at(kRnm, q);
        k[j].tm = R.at(kRtm, q);
        k[j].ni = R.at(kRni, q);
        k[j].ti = R.at(kRti, q);
        key[j] = __float_as_int(R.at(kRkey, q));
        pn[j] = mk(R.at(kRpnx, q), R.at(kRpny, q));
        pp[j] = mk(R.at(kRppx, q), R.at(kRppy, q));
        si[j] = slot_of(slot_i(key[j]));
        sj[j] = slot_type(key[j]) == 0 ? slot_of(slot_js(key[j])) : 0;
    }
    // one contact's velocity step on the compact bodies
    auto vel = [&](int j, bool warm) {
        V2 vA = mk(0.0f, 0.0f), vB;
        float wA = 0.0f, wB;
        if (slot_type(key[j]) == 0) {
            if (NB == 2) {  // the pair is slots (0, 1)
                vA = vv[0]; wA = ww[0];
                vB = vv[1]; wB = ww[1];
            } else {
                vA = sel(vv, si[j]); wA = sel(ww, si[j]);
                vB = sel(vv, sj[j]); wB = sel(ww, sj[j]);
            }
            if (warm) vc_warm(k[j], vA, wA, vB, wB, m, Ii, m, Ii);
            else vc_solve(k[j], vA, wA, vB, wB, m, Ii, m, Ii);
            if (NB == 2) {
                vv[0] = vA; ww[0] = wA;
                vv[1] = vB; ww[1] = wB;
            } else {
                put(vv, si[j], vA); put(ww, si[j], wA);
                put(vv, sj[j], vB); put(ww, sj[j], wB);
            }
        } else {
            vB = sel(vv, si[j]); wB = sel(ww, si[j]);
            if (warm) vc_warm(k[j], vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
            else vc_solve(k[j], vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
            put(vv, si[j], vB); put(ww, si[j], wB);
        }
    };
#pragma unroll
    for (int j = 0; j < KC; ++j)
        if (j < n) vel(j, true);
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        V2 vp[NB];
        float wp[NB], qn[KC], qt[KC];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            vp[b] = vv[b];
            wp[b] = ww[b];
        }
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            qn[j] = k[j].ni;
            qt[j] = k[j].ti;
        }
#pragma unroll
        for (int j = 0; j < KC; ++j)
            if (j < n) vel(j, false);
        bool same = true;
#pragma unroll
        for (int b = 0; b < NB; ++b) same = same && same_bits(vv[b], vp[b]) && same_bits(ww[b], wp[b]);
#pragma unroll
        for (int j = 0; j < KC; ++j)
            if (j < n) same = same && same_bits(k[j].ni, qn[j]) && same_bits(k[j].ti, qt[j]);
        if (same) break;
    }
    // store impulses
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= n) continue;
        const int i = slot_i(key[j]), js = slot_js(key[j]);
        if (slot_type(key[j]) == 0) {
            const int p = aa_index<AM>(i, js);
            K.set_aani(p, k[j].ni);
            K.set_aati(p, k[j].ti);
        } else {
            K.set_asni(i, js, k[j].ni);
            K.set_asti(i, js, k[j].ti);
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) integrate(cc[b], aa[b], vv[b], ww[b], dt);
    bool converged = false;
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        float minsep = 0.0f;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= n) continue;
            float sep;
            if (slot_type(key[j]) == 0) {
                V2 cA, cB;
                float aA, aB;
                if (NB == 2) {
                    cA = cc[0]; aA = aa[0];
                    cB = cc[1]; aB = aa[1];
                } else {
                    cA = sel(cc, si[j]); aA = sel(aa, si[j]);
                    cB = sel(cc, sj[j]); aB = sel(aa, sj[j]);
                }
                sep = pc_solve_aa(cA, aA, cB, aB, P.agent_r, m, Ii, kBaumgarte);
                if (NB == 2) {
                    cc[0] = cA; aa[0] = aA;
                    cc[1] = cB; aa[1] = aB;
                } else {
                    put(cc, si[j], cA); put(aa, si[j], aA);
                    put(cc, sj[j], cB); put(aa, sj[j], aB);
                }
            } else {
                V2 cB = sel(cc, si[j]);
                float aB = sel(aa, si[j]);
                sep = pc_solve_as_h(pn[j], pp[j], cB, aB, P.agent_r, m, Ii, kBaumgarte, P.inv_mass_rcp);
                put(cc, si[j], cB); put(aa, si[j], aB);
            }
            minsep = fmin_b2(minsep, sep);
        }
        if (minsep >= -3.0f * kLinearSlop) {
            converged = true;
            break;
        }
    }
    // sleep (island_solve_regs' loop over the members, ascending)
    const float linTolSqr = kLinSleepTol * kLinSleepTol;
    const float angTolSqr = kAngSleepTol * kAngSleepTol;
    float ms = kMaxFloat;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const float ww2 = ww[b] * ww[b], vv2 = dot(vv[b], vv[b]);
        const bool moving = (ww2 > angTolSqr) | (vv2 > linTolSqr);
        const float acc = opq(ss[b] + dt);
        ss[b] = moving ? 0.0f : acc;
        ms = moving ? 0.0f : fmin_b2(ms, acc);
    }
    new_awake = members;
    if (ms >= kTimeToSleep && converged) {
        new_awake = 0;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            ss[b] = 0.0f;
            vv[b] = mk(0.0f, 0.0f);
            ww[b] = 0.0f;
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        put(c, idx[b], cc[b]);
        put(a, idx[b], aa[b]);
        put(v, idx[b], vv[b]);
        put(w, idx[b], ww[b]);
        put(sl, idx[b], ss[b]);
    }
}

// island_solve_regs for an island of ONE body (agent r) and n <= KC contacts,
// all agent-static: the body stays in scalars instead of being selected out
// of and put back into the AM-wide arrays around every contact of every
// iteration.  The same operations on the same values in the same order
// (the other bodies never change, so the fixed-point test over all of them
// reduces to body r and the contacts), so the same bits.
template <class C, class KT>
__device__ __forceinline__ void island_solve_one(const Params& P, const SolveRec<C>& R, const KT& K,
                                                 const int (&qi)[SolveShape<C>::KR], int n, int r, V2& c, float& a,
                                                 V2& v, float& w, float& sl, float dt, bool& asleep)
{
    constexpr int KC = SolveShape<C>::KR;
    const float m = P.inv_mass, Ii = P.inv_I;
    VC k[KC];
    V2 pn[KC], pp[KC];
    int js[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const int q = j < n ? qi[j] : 0;
        k[j].normal = mk(R.at(kRnx, q), R.at(kRny, q));
        k[j].rA = mk(R.at(kRax, q), R.at(kRay, q));
        k[j].rB = mk(R.at(kRbx, q), R.at(kRby, q));
        k[j].nm = R.at(kRnm, q);
        k[j].tm = R.at(kRtm, q);
        k[j].ni = R.at(kRni, q);
        k[j].ti = R.at(kRti, q);
        js[j] = slot_js(__float_as_int(R.at(kRkey, q)));
        pn[j] = mk(R.at(kRpnx, q), R.at(kRpny, q));
        pp[j] = mk(R.at(kRppx, q), R.at(kRppy, q));
    }
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= n) continue;
        V2 vA = mk(0.0f, 0.0f);
        float wA = 0.0f;
        vc_warm(k[j], vA, wA, v, w, 0.0f, 0.0f, m, Ii);
    }
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        const V2 vp = v;
        const float wp = w;
        float qn[KC], qt[KC];
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            qn[j] = k[j].ni;
            qt[j] = k[j].ti;
        }
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= n) continue;
            V2 vA = mk(0.0f, 0.0f);
            float wA = 0.0f;
            vc_solve(k[j], vA, wA, v, w, 0.0f, 0.0f, m, Ii);
        }
        bool same = same_bits(v, vp) && same_bits(w, wp);
#pragma unroll
        for (int j = 0; j < KC; ++j)
            if (j < n) same = same && same_bits(k[j].ni, qn[j]) && same_bits(k[j].ti, qt[j]);
        if (same) break;
    }
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (j >= n) continue;
        K.set_asni(r, js[j], k[j].ni);
        K.set_asti(r, js[j], k[j].ti);
    }
    integrate(c, a, v, w, dt);
    bool converged = false;
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        float minsep = 0.0f;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j >= n) continue;
            minsep = fmin_b2(minsep, pc_solve_as_h(pn[j], pp[j], c, a, P.agent_r, m, Ii, kBaumgarte, P.inv_mass_rcp));
        }
        if (minsep >= -3.0f * kLinearSlop) {
            converged = true;
            break;
        }
    }
    // sleep (island_solve_regs' loop for the one member)
    const float linTolSqr = kLinSleepTol * kLinSleepTol;
    const float angTolSqr = kAngSleepTol * kAngSleepTol;
    const bool moving = (w * w > angTolSqr) | (dot(v, v) > linTolSqr);
    const float acc = opq(sl + dt);
    sl = moving ? 0.0f : acc;
    const float ms = moving ? 0.0f : fmin_b2(kMaxFloat, acc);
    asleep = ms >= kTimeToSleep && converged;
    if (asleep) {
        sl = 0.0f;
        v = mk(0.0f, 0.0f);
        w = 0.0f;
    }
}

// One world step's Collide + Solve of env e on this lane's group (lane s of
// the group).  valid: the group holds an env (every lane of the wave runs the
// ballots and the barrier).  rec: this workgroup's contact records.
// TOI: also run b2World::SolveTOI of the step on the group (toi_agent_group,
// mas_physics.h: lane s owns static s) -- the fused general path, one launch
// per world step, no sweep buffer; else the sweep starts go to P.sweep for
// k_gen_toi.
// 1 (default): the SolveTOI agent loop runs by rank (each group's k-th TOI
// agent in round k); 0: by agent index
#ifndef MAS_TOI_BY_RANK
#define MAS_TOI_BY_RANK 1
#endif
template <class C, bool TOI>
__device__ __forceinline__ void gen_solve_group(const Params& P, uint32_t* __restrict__ state, int64_t N, int64_t e,
                                                bool valid, int s, float* rec_lds, int slot, int pf = 0)
{
    using SS = SolveShape<C>;
    using TW = StateWords<C>;
    constexpr int G = SS::G, AM = C::AM, NS = C::NS, NAA = C::NAA, KC = SS::KR;
    const float dt = (float)(1.0 / 60.0);
    const float m = P.inv_mass, Ii = P.inv_I;
    const Cont<C, ContGlbStore<C>> K{{state, N, e, P.w_cont}};
    const SolveRec<C> R{rec_lds, slot};

    // ---------------- load: the agents (every lane), this lane's static ----------------
    V2 c[AM], v[AM];
    float a[AM], w[AM], sl[AM];
    uint32_t alive = 0, awake = 0, aat0 = 0, ast0[AM];
    int nbox = 0;
    float inv_dt0 = 0.0f;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        c[i] = v[i] = mk(0.0f, 0.0f);
        a[i] = w[i] = sl[i] = 0.0f;
        ast0[i] = 0u;
    }
    if (valid) {
#pragma unroll
        for (int i = 0; i < AM; ++i) {
            c[i] = mk(__uint_as_float(state[state_index(7 * i, e, N)]), __uint_as_float(state[state_index(7 * i + 1, e, N)]));
            a[i] = __uint_as_float(state[state_index(7 * i + 2, e, N)]);
            v[i] = mk(__uint_as_float(state[state_index(7 * i + 3, e, N)]), __uint_as_float(state[state_index(7 * i + 4, e, N)]));
            w[i] = __uint_as_float(state[state_index(7 * i + 5, e, N)]);
            sl[i] = __uint_as_float(state[state_index(7 * i + 6, e, N)]);
        }
        alive = state[state_index(TW::alive, e, N)];
        awake = state[state_index(TW::awake, e, N)];
        nbox = (int)state[state_index(TW::box, e, N)];
        inv_dt0 = __uint_as_float(state[state_index(P.w_invdt, e, N)]);
        aat0 = K.aat();
#pragma unroll
        for (int i = 0; i < AM; ++i) ast0[i] = K.ast(i);
    }
    V2 cs[AM];  // sweep start (b2Sweep c0) = the positions before the solve
    float as_[AM];
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        cs[i] = c[i];
        as_[i] = a[i];
    }
    const int sc = s < NS ? s : NS - 1;
    StaticG g;
    V2 lo, hi;
    float bhx, bhy;
    int bmeta;
    group_static<C>(P, state, N, e, valid && s < NS && s >= kNumWalls, sc, g, lo, hi, bhx, bhy, bmeta);
    // the stored impulses of this lane's contacts that were touching
    // (agent-static pairs (i, s); agent pair p = s), fetched with the state:
    // Collide only zeroes contacts that leave the list, so these are the
    // values the velocity constraints start from
    float pni[AM], pti[AM], pan = 0.0f, pat = 0.0f;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        pni[i] = pti[i] = 0.0f;
        if (valid && s < NS && bit(ast0[i], s)) {
            pni[i] = K.asni(i, s);
            pti[i] = K.asti(i, s);
        }
    }
    if (valid && s < NAA && bit(aat0, s)) {
        pan = K.aani(s);
        pat = K.aati(s);
    }
    const float inv_dt = 1.0f / dt;
    const float dtRatio = inv_dt0 * dt;
    MAS_PROF(P, pf + kPfLoad);

    // ---------------- Collide: agent-agent pairs (serial on every lane) ----------------
    uint32_t aat = aat0, aa_eval = 0;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = i + 1; j < AM; ++j) {
            if (!(bit(alive, i) && bit(alive, j))) continue;
            if (!(bit(awake, i) || bit(awake, j))) continue;
            const int p = aa_index<AM>(i, j);
            const bool was = bit(aat, p);
            const V2 d = sub(c[j], c[i]);
            const float dsq = dot(d, d);
            const float rad = P.agent_r + P.agent_r;
            const bool touching = !(dsq > rad * rad);
            aa_eval |= 1u << p;
            // impulses reset (b2Contact::Update): a pair that stays out of
            // contact here; a new contact's reset is folded into its warm
            // start below (the solve writes its impulses)
            if (valid && s == p && !touching) {
                K.set_aani(p, 0.0f);
                K.set_aati(p, 0.0f);
            }
            aat = touching ? (aat | (1u << p)) : (aat & ~(1u << p));
            if (touching != was) {
                if (!bit(awake, i)) { awake |= 1u << i; sl[i] = 0.0f; }
                if (!bit(awake, j)) { awake |= 1u << j; sl[j] = 0.0f; }
            }
        }

    // ---------------- Collide: agent-static pairs, static s on lane s ----------------
    const int ns = kNumWalls + nbox;
    const float reach = P.agent_r + kPolyRadius + 1e-3f;
    uint32_t my_t = 0, my_lost = 0, my_new = 0;  // bit i: agent i's pair with this static
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        const bool ev = valid && s < ns && bit(alive, i) && bit(awake, i);
        const bool was = bit(ast0[i], s);
        const float dx = fmaxf(fmaxf(lo.x - c[i].x, c[i].x - hi.x), 0.0f);
        const float dy = fmaxf(fmaxf(lo.y - c[i].y, c[i].y - hi.y), 0.0f);
        const bool cand = dx * dx + dy * dy <= reach * reach;
        bool t = false;
        if (ev && cand) {
            V2 ln, lp;
            t = collide_pc(g.poly, g.p, g.q, c[i], kPolyRadius, P.agent_r, ln, lp);
        }
        if (ev && !t && (was || cand)) {
            K.set_asni(i, s, 0.0f);
            K.set_asti(i, s, 0.0f);
        }
        if (t) my_t |= 1u << i;
        if (ev && was && !cand) my_lost |= 1u << i;
        if (ev && t && !was) my_new |= 1u << i;
    }
    uint32_t ast[AM];
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        const uint32_t tb = group_ballot<G>(bit(my_t, i));
        const bool lost = group_ballot<G>(bit(my_lost, i)) != 0u;
        const uint32_t low = ns >= 32 ? 0xffffffffu : ((1u << ns) - 1u);
        const bool ev = bit(alive, i) && bit(awake, i);
        ast[i] = ev ? ((lost ? 0u : (ast0[i] & ~low)) | tb) : ast0[i];
    }
    MAS_PROF(P, pf + kPfCollide);

    // ---------------- Solve: islands (uniform), wake, damping ----------------
    int label[AM];
#pragma unroll
    for (int i = 0; i < AM; ++i) label[i] = i;
#pragma unroll
    for (int pass = 0; pass < AM; ++pass) {
        if (aat == 0u) break;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = i + 1; j < AM; ++j) {
                const int p = aa_index<AM>(i, j);
                if (bit(alive, i) && bit(alive, j) && bit(aat, p)) {
                    const int l = label[i] < label[j] ? label[i] : label[j];
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
            if (label[j] == label[i] && bit(alive, j) && bit(awake, j)) any = true;
        if (bit(alive, i) && any) solved |= 1u << i;
    }
    if (!valid) solved = 0;
#pragma unroll
    for (int i = 0; i < AM; ++i)
        if (bit(solved, i) && !bit(awake, i)) {
            awake |= 1u << i;
            sl[i] = 0.0f;
        }
    const uint32_t awake_pre = awake;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        if (!bit(solved, i)) continue;
        const float ld = 1.0f / (1.0f + dt * P.lin_damp);
        v[i].x *= ld;
        v[i].y *= ld;
        const float ad = 1.0f / (1.0f + dt * P.ang_damp);
        w[i] *= ad;
    }

    // ---------------- contact list: canonical index, velocity constraints ----------------
    uint32_t aa_list = 0;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = i + 1; j < AM; ++j)
            if (bit(solved, i) && bit(solved, j) && bit(aat, aa_index<AM>(i, j))) aa_list |= 1u << aa_index<AM>(i, j);
    const uint32_t nsmask = NS >= 32 ? 0xffffffffu : ((1u << NS) - 1u);
    int before[AM], nq = __popc(aa_list);
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        before[i] = nq;
        if (bit(solved, i)) nq += __popc(ast[i] & nsmask);
    }
    // agent-agent contact p on lane p
    if (s < NAA && bit(aa_list, s)) {
        int pi = 0, pj = 1;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = i + 1; j < AM; ++j)
                if (aa_index<AM>(i, j) == s) { pi = i; pj = j; }
        const bool reset = bit(aa_eval, s) && !bit(aat0, s);
        const float sni = reset ? 0.0f : pan, sti = reset ? 0.0f : pat;
        VC k = vc_init_aa(sel(c, pi), sel(c, pj), P.agent_r, m, Ii, m, Ii);
        k.ni = dtRatio * sni;
        k.ti = dtRatio * sti;
        const int q = __popc(aa_list & ((1u << s) - 1u));
        R.at(kRnx, q) = k.normal.x; R.at(kRny, q) = k.normal.y;
        R.at(kRax, q) = k.rA.x; R.at(kRay, q) = k.rA.y;
        R.at(kRbx, q) = k.rB.x; R.at(kRby, q) = k.rB.y;
        R.at(kRnm, q) = k.nm; R.at(kRtm, q) = k.tm;
        R.at(kRni, q) = k.ni; R.at(kRti, q) = k.ti;
        R.at(kRkey, q) = __int_as_float((0 << 16) | (pi << 8) | pj);
    }
    // agent-static contacts of static s on lane s
    if (s < NS) {
#pragma unroll
        for (int i = 0; i < AM; ++i) {
            if (!(bit(solved, i) && bit(ast[i], s))) continue;
            V2 ln = mk(0.0f, 0.0f), lp = mk(0.0f, 0.0f);
            collide_pc(g.poly, g.p, g.q, c[i], kPolyRadius, P.agent_r, ln, lp);
            VC k = vc_init_as(g.p, g.q, ln, lp, c[i], P.agent_r, m, Ii);
            const bool reset = bit(my_new, i);
            const float sni = reset ? 0.0f : pni[i], sti = reset ? 0.0f : pti[i];
            k.ni = dtRatio * sni;
            k.ti = dtRatio * sti;
            const int q = before[i] + __popc(ast[i] & ((1u << s) - 1u));
            const V2 pn = rmul(g.q, ln), pp = xmul(g.p, g.q, lp);
            R.at(kRnx, q) = k.normal.x; R.at(kRny, q) = k.normal.y;
            R.at(kRax, q) = k.rA.x; R.at(kRay, q) = k.rA.y;
            R.at(kRbx, q) = k.rB.x; R.at(kRby, q) = k.rB.y;
            R.at(kRnm, q) = k.nm; R.at(kRtm, q) = k.tm;
            R.at(kRni, q) = k.ni; R.at(kRti, q) = k.ti;
            R.at(kRkey, q) = __int_as_float((1 << 16) | (i << 8) | s);
            R.at(kRpnx, q) = pn.x; R.at(kRpny, q) = pn.y;
            R.at(kRppx, q) = pp.x; R.at(kRppy, q) = pp.y;
        }
    }
    wave_lds_sync();  // the records are in LDS (the workgroup is this wave)

    // ---------------- b2Island::Solve of the island agent s roots ----------------
    uint32_t new_awake = 0;  // this root's members' awake bits after sleep
    const bool root = s < AM && bit(solved, s) && sel(label, s) == s;
    if (root) {
        const int r = s;
        uint32_t members = 0;
#pragma unroll
        for (int j = 0; j < AM; ++j)
            if (label[j] == r && bit(solved, j)) members |= 1u << j;
        auto mine = [&](int q, int& key) {
            key = __float_as_int(R.at(kRkey, q));
            return sel(label, slot_i(key)) == r;
        };
        // the island's contacts (canonical order) into KR (<= 4) register
        // slots; more (rare) keeps them in LDS (the loops below)
        int qi[KC];
        int nqi = 0;
#pragma unroll
        for (int j = 0; j < KC; ++j) qi[j] = 0;
#pragma unroll 1
        for (int q = 0; q < nq; ++q) {
            int key;
            if (!mine(q, key)) continue;
#pragma unroll
            for (int j = 0; j < KC; ++j) qi[j] = opq(j == nqi ? q : qi[j]);
            ++nqi;
        }
        if (nqi <= KC && members == (1u << r)) {
            // one body (every contact agent-static): scalars, no selects
            V2 cr = sel(c, r), vr = sel(v, r);
            float ar = sel(a, r), wr = sel(w, r), slr = sel(sl, r);
            bool asleep;
            island_solve_one<C>(P, R, K, qi, nqi, r, cr, ar, vr, wr, slr, dt, asleep);
            put(c, r, cr);
            put(a, r, ar);
            put(v, r, vr);
            put(w, r, wr);
            put(sl, r, slr);
            new_awake = asleep ? 0u : members;
        } else if (nqi <= KC && kIslandK<C> && __popc(members) == 2) {
            island_solve_k<C, (AM > 2 ? 2 : 1)>(P, R, K, qi, nqi, members, c, a, v, w, sl, dt, new_awake);
        } else if (nqi <= KC) {
            island_solve_regs<C>(P, R, K, qi, nqi, members, c, a, v, w, sl, dt, new_awake);
        } else {
        auto load_vc = [&](int q) {
            VC k;
            k.normal = mk(R.at(kRnx, q), R.at(kRny, q));
            k.rA = mk(R.at(kRax, q), R.at(kRay, q));
            k.rB = mk(R.at(kRbx, q), R.at(kRby, q));
            k.nm = R.at(kRnm, q);
            k.tm = R.at(kRtm, q);
            k.ni = R.at(kRni, q);
            k.ti = R.at(kRti, q);
            return k;
        };
        // warm start
#pragma unroll 1
        for (int q = 0; q < nq; ++q) {
            int key;
            if (!mine(q, key)) continue;
            const VC k = load_vc(q);
            const int i = slot_i(key), js = slot_js(key);
            V2 vA = mk(0.0f, 0.0f), vB;
            float wA = 0.0f, wB;
            if (slot_type(key) == 0) {
                vA = sel(v, i); wA = sel(w, i);
                vB = sel(v, js); wB = sel(w, js);
                vc_warm(k, vA, wA, vB, wB, m, Ii, m, Ii);
                put(v, i, vA); put(w, i, wA);
                put(v, js, vB); put(w, js, wB);
            } else {
                vB = sel(v, i); wB = sel(w, i);
                vc_warm(k, vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
                put(v, i, vB); put(w, i, wB);
            }
        }
        // velocity iterations (exact fixed-point exit, per island)
#pragma unroll 1
        for (int it = 0; it < 10; ++it) {
            V2 vp[AM];
            float wp[AM];
#pragma unroll
            for (int j = 0; j < AM; ++j) {
                vp[j] = v[j];
                wp[j] = w[j];
            }
            bool same = true;
#pragma unroll 1
            for (int q = 0; q < nq; ++q) {
                int key;
                if (!mine(q, key)) continue;
                VC k = load_vc(q);
                const float ni0 = k.ni, ti0 = k.ti;
                const int i = slot_i(key), js = slot_js(key);
                V2 vA = mk(0.0f, 0.0f), vB;
                float wA = 0.0f, wB;
                if (slot_type(key) == 0) {
                    vA = sel(v, i); wA = sel(w, i);
                    vB = sel(v, js); wB = sel(w, js);
                    vc_solve(k, vA, wA, vB, wB, m, Ii, m, Ii);
                    put(v, i, vA); put(w, i, wA);
                    put(v, js, vB); put(w, js, wB);
                } else {
                    vB = sel(v, i); wB = sel(w, i);
                    vc_solve(k, vA, wA, vB, wB, 0.0f, 0.0f, m, Ii);
                    put(v, i, vB); put(w, i, wB);
                }
                same = same && same_bits(k.ni, ni0) && same_bits(k.ti, ti0);
                R.at(kRni, q) = k.ni;
                R.at(kRti, q) = k.ti;
            }
#pragma unroll
            for (int j = 0; j < AM; ++j) same = same && same_bits(v[j], vp[j]) && same_bits(w[j], wp[j]);
            if (same) break;
        }
        // store impulses
#pragma unroll 1
        for (int q = 0; q < nq; ++q) {
            int key;
            if (!mine(q, key)) continue;
            const int i = slot_i(key), js = slot_js(key);
            const float ni = R.at(kRni, q), ti = R.at(kRti, q);
            if (slot_type(key) == 0) {
                const int p = aa_index<AM>(i, js);
                K.set_aani(p, ni);
                K.set_aati(p, ti);
            } else {
                K.set_asni(i, js, ni);
                K.set_asti(i, js, ti);
            }
        }
        // integrate positions
#pragma unroll
        for (int j = 0; j < AM; ++j)
            if (bit(members, j)) integrate(c[j], a[j], v[j], w[j], dt);
        // position iterations, the island's early exit
        bool converged = false;
#pragma unroll 1
        for (int it = 0; it < 10; ++it) {
            float minsep = 0.0f;
#pragma unroll 1
            for (int q = 0; q < nq; ++q) {
                int key;
                if (!mine(q, key)) continue;
                const int i = slot_i(key), js = slot_js(key);
                float sep;
                if (slot_type(key) == 0) {
                    V2 cA = sel(c, i), cB = sel(c, js);
                    float aA = sel(a, i), aB = sel(a, js);
                    sep = pc_solve_aa(cA, aA, cB, aB, P.agent_r, m, Ii, kBaumgarte);
                    put(c, i, cA); put(a, i, aA);
                    put(c, js, cB); put(a, js, aB);
                } else {
                    const V2 pn = mk(R.at(kRpnx, q), R.at(kRpny, q)), pp = mk(R.at(kRppx, q), R.at(kRppy, q));
                    V2 cB = sel(c, i);
                    float aB = sel(a, i);
                    sep = pc_solve_as_h(pn, pp, cB, aB, P.agent_r, m, Ii, kBaumgarte, P.inv_mass_rcp);
                    put(c, i, cB); put(a, i, aB);
                }
                minsep = fmin_b2(minsep, sep);
            }
            if (minsep >= -3.0f * kLinearSlop) {
                converged = true;
                break;
            }
        }
        // sleep (per island)
        const float linTolSqr = kLinSleepTol * kLinSleepTol;
        const float angTolSqr = kAngSleepTol * kAngSleepTol;
        // (branch-free: the short-circuit if / else form of this loop was
        // miscompiled for the 1v1 class -- on the "w small, v large" path the
        // register holding sl[j] = 0 was reused for v.y^2 and stored as the
        // sleep time; scripts/ab_solve_golden.py found it)
        float ms = kMaxFloat;
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            const float ww = w[j] * w[j], vv = dot(v[j], v[j]);
            const bool moving = (ww > angTolSqr) | (vv > linTolSqr);
            const float acc = opq(sl[j] + dt);
            const bool mem = bit(members, j);
            sl[j] = mem ? (moving ? 0.0f : acc) : sl[j];
            ms = mem ? (moving ? 0.0f : fmin_b2(ms, acc)) : ms;
        }
        new_awake = members;
        if (ms >= kTimeToSleep && converged) {
            new_awake = 0;
#pragma unroll
            for (int j = 0; j < AM; ++j) {
                if (!bit(members, j)) continue;
                sl[j] = 0.0f;
                v[j] = mk(0.0f, 0.0f);
                w[j] = 0.0f;
            }
        }
        }  // more than KC island contacts
        if (!TOI) {
            // the island's bodies (b2Island::Solve writes back every member)
#pragma unroll
            for (int j = 0; j < AM; ++j) {
                if (!bit(members, j)) continue;
                const float out[7] = {c[j].x, c[j].y, a[j], v[j].x, v[j].y, w[j], sl[j]};
#pragma unroll
                for (int q = 0; q < 7; ++q) state[state_index(7 * j + q, e, N)] = __float_as_uint(out[q]);
            }
        }
    }
    MAS_PROF(P, pf + kPfSolve);
    const uint32_t awake_fin = (awake_pre & ~solved) | group_or<G>(new_awake);
    uint32_t toi_ran = 0;
    int toi_events = 0;  // TOI events of the env's agents, + 65536 per capped agent
    if (TOI) {
        // every lane takes the solved bodies from its island's root lane
        const int base = (int)(threadIdx.x & 63) & ~(G - 1);
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            if (!bit(solved, j)) continue;
            const int src = base + label[j];
            c[j] = mk(__shfl(c[j].x, src, 64), __shfl(c[j].y, src, 64));
            a[j] = __shfl(a[j], src, 64);
            v[j] = mk(__shfl(v[j].x, src, 64), __shfl(v[j].y, src, 64));
            w[j] = __shfl(w[j], src, 64);
            sl[j] = __shfl(sl[j], src, 64);
        }
        // the island solve's impulse stores are ordered before SolveTOI's
        // impulse resets (the same words, other lanes of this wave)
        __threadfence_block();
        MAS_PROF(P, pf + 5);  // the bodies' shuffles + the fence's wait for the impulse stores
        // ---------------- b2World::SolveTOI, agent by agent on the group ----------------
        // (TOI events of different agents are independent: statics never
        // move, agent-agent pairs are not TOI pairs.)  An agent whose sweep
        // every static's conservative pre-test rejects has no event and
        // SolveTOI changes nothing for it (toi_agent_group's first pass):
        // skipped.
        // the agents this env's SolveTOI runs (the group agrees on the mask)
        uint32_t need = 0;
#pragma unroll
        for (int i = 0; i < AM; ++i) {
            const bool act = valid && bit(alive, i) && bit(awake_fin, i);
            const bool keep = act && s < ns && !toi_reject(g, cs[i], c[i], P.agent_r);
            if (group_ballot<G>(keep) != 0u) need |= 1u << i;
        }
#if MAS_TOI_BY_RANK
        // Round k runs each group's k-th such agent (ascending index, the
        // serial order per env), so a wave runs as many rounds as its busiest
        // env has TOI agents; by agent index, agent i's round ran whenever
        // any env of the wave needed agent i (up to AM rounds for one agent
        // per env).  Agents' SolveTOI are independent (statics never move).
#pragma unroll 1
        for (int k = 0; k < AM; ++k) {
            if (!__any(need != 0u)) break;
            if (need == 0u) continue;
            const int i = __builtin_ctz(need);
            need &= need - 1u;
            const V2 ci = sel(c, i), vi = sel(v, i);
            const float ai = sel(a, i), wi = sel(w, i);
#else
#pragma unroll
        for (int i = 0; i < AM; ++i) {
            if (!bit(need, i)) continue;
            const V2 ci = c[i], vi = v[i];
            const float ai = a[i], wi = w[i];
#endif
            EnvL<C> L;
            L.alive_m = alive;
            L.awake_m = awake_fin;
            L.nbox = nbox;
#pragma unroll
            for (int k2 = 0; k2 < AM; ++k2) {
                L.c[k2] = ci;
                L.a[k2] = ai;
                L.v[k2] = vi;
                L.w[k2] = wi;
            }
#pragma unroll
            for (int k2 = 0; k2 < C::BM; ++k2) {
                L.bp[k2] = g.p;
                L.bhx[k2] = bhx;
                L.bhy[k2] = bhy;
                L.bmeta[k2] = bmeta;
            }
            const uint32_t asti = sel(ast, i);
            const ToiGroupOut o = toi_agent_group<C, G>(L, P, K, i, s, sel(cs, i), sel(as_, i), asti, dt);
            toi_events += o.events;
            put(c, i, o.c);
            put(a, i, o.a);
            put(v, i, o.v);
            put(w, i, o.w);
            const uint32_t keepm = ~((ns >= 32) ? 0xffffffffu : ((1u << ns) - 1u));
            put(ast, i, (asti & keepm) | o.touch);
            toi_ran |= 1u << i;
            if (P.toi_diag && o.events && s == 0 && valid) atomicAdd(P.toi_diag + e, o.events);
        }
        MAS_PROF(P, pf + kPfToi);
        // a slow env (sub-step cap, or many events) takes the slow list next
        // step (k_pre); the flag was cleared by this step's k_pre
        if (valid && s == 0 && P.slow_k > 0 && ((toi_events >> 16) != 0 || (toi_events & 0xffff) >= P.slow_k)) {
            P.slow_flag[e] = 1;
            // tell the host (mapped memory; a vector store): it turns the slow split on
            if (P.slow_sig) __hip_atomic_store(P.slow_sig, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (!valid) return;
    if (TOI && s < AM && ((solved | toi_ran) >> s & 1u)) {
        // agent s's body after the island solve and its SolveTOI
        const V2 cc = sel(c, s), vv = sel(v, s);
        const float out[7] = {cc.x, cc.y, sel(a, s), vv.x, vv.y, sel(w, s), sel(sl, s)};
#pragma unroll
        for (int q = 0; q < 7; ++q) state[state_index(7 * s + q, e, N)] = __float_as_uint(out[q]);
    }
    // touching words, awake mask, b2World's previous 1/dt, the sweep starts
    if (s == 0) {
        if (aat != aat0) K.set_aat(aat);
#pragma unroll
        for (int i = 0; i < AM; ++i)
            if (ast[i] != ast0[i]) K.set_ast(i, ast[i]);
        state[state_index(TW::awake, e, N)] = awake_fin;
        state[state_index(P.w_invdt, e, N)] = __float_as_uint(inv_dt);
    }
    // agents woken by Collide that no island holds cannot exist (a woken agent
    // is alive and awake, so its island is solved); the sweep of agent s
    if (!TOI && s < AM) {
        float* sw = P.sweep + e * (3 * AM) + 3 * s;
        const V2 c0s = sel(cs, s);
        sw[0] = c0s.x;
        sw[1] = c0s.y;
        sw[2] = sel(as_, s);
    }
    MAS_PROF(P, pf + kPfStore);
}

}  // namespace mas
