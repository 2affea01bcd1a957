// mas_lanes.h -- the pre-physics phase of the MaSurvival step on agent lanes
// (gfx950 HIP): lane (env slot j, agent i), C::AM consecutive lanes per env,
// kWG / C::AM envs per wave.
//
// Why: one lane per env gives one wave per SIMD at 65536 envs (2v2), and
// that wave's latency chain -- ~200 dependent state words per lane, the
// serial per-agent loops, the select chains over register arrays -- is the
// kernel's time.  Here each lane holds only its own agent (pose, velocity,
// health, inventory) in registers and the env's shared groups (boxes, box
// items, pending drops, heals) live in LDS, loaded cooperatively: a wave
// instruction moves C::AM state words of kWG / C::AM consecutive envs.  The
// per-agent work of the rules (motors, UseLast, the give and melee queries,
// the contact-free physics) runs on the agent's lane; the steps whose order
// the reference makes observable -- the give loop, the melee attacks, the
// box spawns of UseLast -- walk the agents in id order with the acting
// agent's values broadcast inside its env's lane group.  Same operations on
// the same values as step_pre + world_step_fast (mas_step.h, mas_physics.h),
// so the same bits.
//
// Reference: masurvival/semantics.py:300-370 (UseLast, GiveLast), 531-617
// (Melee / ContinuousMelee), 853-856 (Object.pre_step); simulation.py
// 394-424 (DynamicMotors); envs/masurvival_env.py:741-755 (queue_actions);
// Box2D 2.3.x b2World::Step for a contact-free world (world_step_fast).
#pragma once

#include "mas_gensolve.h"

namespace mas {

// first word of each state group (visit_state order; class_info checks it)
template <class C>
struct Lay {
    static constexpr int a4(int x) { return (x + 3) & ~3; }
    static constexpr int alive = 7 * C::AM, awake = 7 * C::AM + 1;
    static constexpr int rule = a4(7 * C::AM + 2), kRuleA = 4 + 3 * C::SM;  // words per agent
    static constexpr int box = a4(rule + C::AM * kRuleA), kBoxW = 1 + 6 * C::BM;
    static constexpr int item = a4(box + kBoxW), kItemW = 1 + 5 * C::BM;
    static constexpr int pend = a4(item + kItemW);
    static constexpr int heal = a4(pend + kItemW), kHealW = 1 + 2 * C::HM;
    static constexpr int zone = a4(heal + kHealW), kZoneW = 2 * kMaxPhases + 7;
    static constexpr int invdt = a4(zone + kZoneW);
    static constexpr int cont = a4(invdt + 1);
    static constexpr int rng = a4(cont + Cont<C>::kWords);
    static constexpr int stat = a4(rng + 10);
    static constexpr int seen = a4(stat + kStats);
};

// the env-shared groups of the wave's envs in LDS, [word][slot]
template <class C>
struct PreLds {
    static constexpr int S = kWG / C::AM;  // env slots per wave
    using LY = Lay<C>;
    uint32_t box[LY::kBoxW * S];
    uint32_t item[LY::kItemW * S];
    uint32_t pend[LY::kItemW * S];
    uint32_t heal[LY::kHealW * S];
    float ax[C::AM * S], ay[C::AM * S];  // agent positions (the give query)
    float tab[FixTab<C, S>::kWords * S];  // melee ray fixture tables
};

// slot j's view of PreLds
template <class C>
struct EnvV {
    static constexpr int S = kWG / C::AM;
    PreLds<C>* d;
    int j;
    __device__ uint32_t& bw(int w) const { return d->box[w * S + j]; }
    __device__ uint32_t& iw(int w) const { return d->item[w * S + j]; }
    __device__ uint32_t& pw(int w) const { return d->pend[w * S + j]; }
    __device__ uint32_t& hw(int w) const { return d->heal[w * S + j]; }
    __device__ int nbox() const { return (int)bw(0); }
    __device__ V2 bp(int b) const { return mk(__uint_as_float(bw(1 + 6 * b)), __uint_as_float(bw(2 + 6 * b))); }
    __device__ float bhx(int b) const { return __uint_as_float(bw(3 + 6 * b)); }
    __device__ float bhy(int b) const { return __uint_as_float(bw(4 + 6 * b)); }
    __device__ int bmeta(int b) const { return (int)bw(5 + 6 * b); }
    __device__ int nbi() const { return (int)iw(0); }
    __device__ V2 ip(int b) const { return mk(__uint_as_float(iw(1 + 5 * b)), __uint_as_float(iw(2 + 5 * b))); }
    __device__ int nheal() const { return (int)hw(0); }
    __device__ V2 hp(int h) const { return mk(__uint_as_float(hw(1 + 2 * h)), __uint_as_float(hw(2 + 2 * h))); }
    __device__ V2 agent(int k) const { return mk(d->ax[k * S + j], d->ay[k * S + j]); }
};

// this lane's agent (slot = IndexBodies id)
template <class C>
struct AgentL {
    V2 c, v;
    float a, w, sleep;
    int health, cause, cooldown, inv_n;
    int inv_meta[C::SM];
    float inv_hx[C::SM], inv_hy[C::SM];
};

// lanes of this lane's env group: group-relative bit masks and broadcasts
template <class C>
__device__ __forceinline__ uint32_t env_ballot(bool b)
{
    return group_ballot<C::AM>(b);
}
template <class C, class T>
__device__ __forceinline__ T env_bcast(T v, int src)
{
    return gshfl<C::AM>(v, src);
}

// the cooperative load / store of one state group's words for the wave's
// env slots: lane l moves word l / S of slot l % S, kWG / S words per
// instruction (each word's S envs are one contiguous row segment).  Unrolled
// over the group's kWG-word rounds with every load issued before the first
// LDS write: the rolled loop waited out one load latency per round (round
// r04h: 7 rounds for the 2v2 box group, four groups back to back).
// (split in two so that a kernel issues every group's loads -- and its
// per-lane state loads -- before the first LDS write: the compiler keeps
// global loads below earlier LDS stores it cannot prove disjoint)
template <int S, int NW>
struct GroupRows {
    static constexpr int T = (NW * S + kWG - 1) / kWG;
    uint32_t v[T];
    __device__ __forceinline__ void load(const uint32_t* __restrict__ state, int64_t N, int64_t e0, int w0)
    {
        const int lane = (int)threadIdx.x;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int i0 = lane + t * kWG;
            const int idx = i0 < NW * S ? i0 : NW * S - 1;  // (clamped: every load unconditional)
            const int w = idx / S, j = idx - w * S;
            const int64_t e = e0 + j < N ? e0 + j : N - 1;
            v[t] = state[state_index(w0 + w, e, N)];
        }
    }
    __device__ __forceinline__ void write(uint32_t* __restrict__ dst) const
    {
        const int lane = (int)threadIdx.x;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int idx = lane + t * kWG;
            if (idx < NW * S) dst[idx] = v[t];
        }
    }
    // load + write in chunks of 8 rounds (the big classes' groups: fewer live
    // registers, still 8 loads in flight)
    __device__ __forceinline__ static void copy(uint32_t* __restrict__ dst, const uint32_t* __restrict__ state,
                                                int64_t N, int64_t e0, int w0)
    {
        const int lane = (int)threadIdx.x;
#pragma unroll
        for (int c0 = 0; c0 < T; c0 += 8) {
            uint32_t u[8];
#pragma unroll
            for (int t = c0; t < c0 + 8 && t < T; ++t) {
                const int i0 = lane + t * kWG;
                const int idx = i0 < NW * S ? i0 : NW * S - 1;
                const int w = idx / S, j = idx - w * S;
                const int64_t e = e0 + j < N ? e0 + j : N - 1;
                u[t - c0] = state[state_index(w0 + w, e, N)];
            }
#pragma unroll
            for (int t = c0; t < c0 + 8 && t < T; ++t) {
                const int idx = lane + t * kWG;
                if (idx < NW * S) dst[idx] = u[t - c0];
            }
        }
    }
};
template <int S, int NW>
__device__ __forceinline__ void group_store(const uint32_t* __restrict__ src, uint32_t* __restrict__ state, int64_t N,
                                            int64_t e0, int w0, uint32_t slots)
{
    constexpr int T = (NW * S + kWG - 1) / kWG;
    const int lane = (int)threadIdx.x;
#pragma unroll
    for (int c0 = 0; c0 < T; c0 += 8) {  // chunks of 8 rounds: LDS reads, then stores
        uint32_t v[8];
#pragma unroll
        for (int t = c0; t < c0 + 8 && t < T; ++t) {
            const int i0 = lane + t * kWG;
            v[t - c0] = src[i0 < NW * S ? i0 : NW * S - 1];
        }
#pragma unroll
        for (int t = c0; t < c0 + 8 && t < T; ++t) {
            const int idx = lane + t * kWG;
            const int w = idx / S, j = idx - w * S;
            if (idx < NW * S && ((slots >> j) & 1u) && e0 + j < N) state[state_index(w0 + w, e0 + j, N)] = v[t - c0];
        }
    }
}

// Inventory.take into this lane's agent (semantics.py:179-187)
template <class C>
__device__ __forceinline__ void own_take(AgentL<C>& g, const Params& P, int meta, float hx, float hy)
{
    if (1 + g.inv_n > P.slots) return;
#pragma unroll
    for (int k = 0; k < C::SM; ++k)
        if (k == g.inv_n) {
            g.inv_meta[k] = meta;
            g.inv_hx[k] = hx;
            g.inv_hy[k] = hy;
        }
    g.inv_n += 1;
}

// pop this lane's agent's last item
template <class C>
__device__ __forceinline__ void own_pop(AgentL<C>& g, int& meta, float& hx, float& hy)
{
    const int n = g.inv_n - 1;
    meta = sel(g.inv_meta, n);
    hx = sel(g.inv_hx, n);
    hy = sel(g.inv_hy, n);
    g.inv_n = n;
}

// Health._change_health of this lane's agent (agent_damage, mas_step.h)
template <class C>
__device__ __forceinline__ void own_damage(AgentL<C>& g, bool alive, const Params& P, int i, int delta, int cause)
{
    if (!alive) return;
    if (P.teams && cause == kCauseBadge + team_of(P, i)) return;
    g.health += delta;
    g.cause = cause;
}

// box_damage on slot j's LDS box b (mas_step.h)
template <class C>
__device__ __forceinline__ void lds_box_damage(const EnvV<C>& V, int b, int delta, int cause)
{
    const int meta = V.bmeta(b);
    if (!box_hinit(meta)) return;  // not in Health.healths yet
    const int vuln = box_vuln(meta);
    if (vuln != kCauseNone && cause != vuln) return;  // OwnedObjectItem vulnerabilities
    V.bw(6 + 6 * b) = (uint32_t)((int)V.bw(6 + 6 * b) + delta);
    V.bw(5 + 6 * b) = (uint32_t)mk_boxmeta(box_rot(meta), box_copied(meta), 1, vuln, cause);
}

// build_fixtab (mas_step.h) of slot j from its LDS groups and agent positions
template <class C, int S>
__device__ __forceinline__ void build_fixtab_v(const EnvV<C>& V, const Params& P, const FixTab<C, S>& T,
                                               uint32_t alive_m)
{
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        const V2 p = V.bp(b);
        T.px(BIdx<C>::box + b) = p.x;
        T.py(BIdx<C>::box + b) = p.y;
        T.hx(b) = V.bhx(b);
        T.hy(b) = V.bhy(b);
        T.meta(b) = __int_as_float(V.bmeta(b));
        const V2 q = V.ip(b);
        T.px(BIdx<C>::bitem + b) = q.x;
        T.py(BIdx<C>::bitem + b) = q.y;
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h) {
        const V2 p = V.hp(h);
        T.px(BIdx<C>::heal + h) = p.x;
        T.py(BIdx<C>::heal + h) = p.y;
    }
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        T.px(BIdx<C>::wall + w) = P.wall_pos[w].x;
        T.py(BIdx<C>::wall + w) = P.wall_pos[w].y;
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        const V2 p = V.agent(i);
        T.px(BIdx<C>::agent + i) = p.x;
        T.py(BIdx<C>::agent + i) = p.y;
    }
    T.counts() = __int_as_float(V.nbox() | (V.nbi() << 8) | (V.nheal() << 16) | (int)(alive_m << 24));
}

// static s of slot j (walls from P, boxes from LDS): geometry and world AABB
template <class C>
__device__ __forceinline__ void static_v(const EnvV<C>& V, const Params& P, int s, V2& lo, V2& hi)
{
    if (s < kNumWalls) {
        V2 l = opq(P.wall_lo[0]), h = opq(P.wall_hi[0]);
#pragma unroll
        for (int k = 1; k < kNumWalls; ++k)
            if (s == k) { l = opq(P.wall_lo[k]); h = opq(P.wall_hi[k]); }
        lo = l;
        hi = h;
    } else {
        const int b = s - kNumWalls;
        const V2 p = V.bp(b);
        const float hx = V.bhx(b), hy = V.bhy(b);
        lo = mk(p.x - hx, p.y - hy);
        hi = mk(p.x + hx, p.y + hy);
    }
}
template <class C>
__device__ __forceinline__ StaticG static_geom_v(const EnvV<C>& V, const Params& P, int s)
{
    StaticG g;
    if (s < kNumWalls) {
        V2 wp = opq(P.wall_pos[0]);
        Rot wq = P.wall_q[0];
        float wa = P.wall_angle[0];
#pragma unroll
        for (int k = 1; k < kNumWalls; ++k)
            if (s == k) { wp = opq(P.wall_pos[k]); wq.s = opq(P.wall_q[k].s); wq.c = opq(P.wall_q[k].c); wa = opq(P.wall_angle[k]); }
        g.p = wp;
        g.q = wq;
        g.angle = wa;
        g.poly = P.wall_poly;
    } else {
        const int b = s - kNumWalls;
        const int meta = V.bmeta(b);
        g.p = V.bp(b);
        g.q = kIdRot;
        g.angle = 0.0f;
        g.poly = box_poly(V.bhx(b), V.bhy(b), box_rot(meta), box_copied(meta));
    }
    return g;
}

// One contact-free world.Step (world_step_fast, mas_physics.h) on agent
// lanes: each lane tests its own agent against the others and the statics,
// integrates and sleeps its own agent, and runs its own sweep's TOI reject.
// Returns false when any agent of the env needs the general path (the group
// then keeps its pre-step state); alive / awake: this lane's bits, awake is
// updated.
template <class C>
__device__ __forceinline__ bool world_step_fast_lane(AgentL<C>& g, bool alive, bool& awake, const EnvV<C>& V,
                                                     const Params& P, int i, float dt)
{
    const V2 c0 = g.c;
    bool bail = false;
    // Collide: any agent-agent pair at touching distance -> general path
    const uint32_t alive_m = env_ballot<C>(alive), awake_m = env_ballot<C>(awake);
#pragma unroll
    for (int k = 0; k < C::AM; ++k) {
        const V2 ck = mk(env_bcast<C>(g.c.x, k), env_bcast<C>(g.c.y, k));
        if (k == i) continue;
        if (!(alive && bit(alive_m, k))) continue;
        if (!(awake || bit(awake_m, k))) continue;
        // (the pair (min, max) is tested as world_step_fast does: d = c_hi - c_lo)
        const V2 d = k > i ? sub(ck, g.c) : sub(g.c, ck);
        const float rad = P.agent_r + P.agent_r;
        if (!(dot(d, d) > rad * rad)) bail = true;
    }
    // agent-static pairs: any narrowphase candidate -> general path.  (Over
    // the class maxima with the count as the guard: every static's index is
    // a constant -- a wall's bounds come straight from P, a box's LDS reads
    // issue up front -- instead of a runtime loop selecting among the walls;
    // the same tests, so the same decision.)
    const int ns = kNumWalls + V.nbox();
    const float reach = P.agent_r + kPolyRadius + 1e-3f;
    if (alive && awake) {
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            if (s >= ns) continue;
            V2 lo, hi;
            static_v(V, P, s, lo, hi);
            const float dx = fmaxf(fmaxf(lo.x - g.c.x, g.c.x - hi.x), 0.0f);
            const float dy = fmaxf(fmaxf(lo.y - g.c.y, g.c.y - hi.y), 0.0f);
            if (dx * dx + dy * dy <= reach * reach) bail = true;
        }
    }
    if (env_ballot<C>(bail) != 0u) return false;
    // Solve: every awake alive agent is its own island (damping, integrate,
    // per-island sleep; branch-free sleep block as world_step_fast)
    const float h = dt;
    if (alive && awake) {
        const float ld = 1.0f / (1.0f + h * P.lin_damp);
        g.v.x *= ld;
        g.v.y *= ld;
        const float ad = 1.0f / (1.0f + h * P.ang_damp);
        g.w *= ad;
        integrate(g.c, g.a, g.v, g.w, h);
        const float linTolSqr = kLinSleepTol * kLinSleepTol;
        const float angTolSqr = kAngSleepTol * kAngSleepTol;
        const bool moving = (g.w * g.w > angTolSqr) | (dot(g.v, g.v) > linTolSqr);
        const float acc = opq(g.sleep + h);
        g.sleep = moving ? 0.0f : acc;
        const float ms = moving ? 0.0f : fmin_b2(kMaxFloat, acc);
        if (ms >= kTimeToSleep) {
            awake = false;
            g.sleep = 0.0f;
            g.v = mk(0.0f, 0.0f);
            g.w = 0.0f;
        }
    }
    // SolveTOI: the sweep of an awake agent must be rejected by the cheap
    // test (the same world-AABB pre-filter as world_step_fast)
    if (alive && awake) {
        const float Rp =
            1.4143f * ((kPolyRadius + P.agent_r - 3.0f * kLinearSlop) + 0.25f * kLinearSlop + 0.02f) + 0.05f;
        const V2 slo = mk(fminf(c0.x, g.c.x) - Rp, fminf(c0.y, g.c.y) - Rp);
        const V2 shi = mk(fmaxf(c0.x, g.c.x) + Rp, fmaxf(c0.y, g.c.y) + Rp);
        // (the cull over the class maxima, constant indices; the exact
        // reject for the surviving statics, by runtime index)
        uint32_t near = 0;
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
            if (s >= ns) continue;
            V2 lo, hi;
            static_v(V, P, s, lo, hi);
            if (!(slo.x > hi.x || shi.x < lo.x || slo.y > hi.y || shi.y < lo.y)) near |= 1u << s;
        }
        while (near) {
            const int s = __builtin_ctz(near);
            near &= near - 1u;
            const StaticG sg = static_geom_v(V, P, s);
            if (!toi_reject(sg, c0, g.c, P.agent_r)) bail = true;
        }
    }
    return env_ballot<C>(bail) == 0u;
}

// 1: the agents' body words stored once, after the fast physics (the words
// before it when the fast path fails); 0: before it too
#ifndef MAS_PRE_BODY_ONCE
#define MAS_PRE_BODY_ONCE 1
#endif
// waves per SIMD the register budget of k_pre_lanes allows (4: 128 VGPRs, a
// 12-register spill for 2v2; 3: 168, none)
#ifndef MAS_PRE_OCC
#define MAS_PRE_OCC 4
#endif
// k_pre on agent lanes: queue_actions, Object drops, DynamicMotors, UseLast,
// GiveLast, Melee (step_pre order), the dirty stores, then the speculative
// contact-free 2 x world.Step and the general-path list append (fast_phys).
template <class C>
__global__ __launch_bounds__(kWG, MAS_PRE_OCC) void k_pre_lanes(Params P, uint32_t* __restrict__ state, int64_t N,
                                                      const int8_t* __restrict__ actions)
{
    using LY = Lay<C>;
    constexpr int S = kWG / C::AM, AM = C::AM;
    static_assert(kWG % AM == 0 && (AM & (AM - 1)) == 0, "agent lane groups must tile a wave");
    __shared__ PreLds<C> lds;
    MAS_PROF(P, -1);
    const int lane = (int)threadIdx.x;
    const int j = lane / AM, i = lane - j * AM;
    const int64_t e0 = xcd_block() * S, e = e0 + j;  // (XCD-aware block order)
    const bool valid = e < N;
    const int64_t ev = valid ? e : N - 1;
    const int A = P.A;
    // the slow list's count slot of the next step (mas_capi: two slots
    // alternate per step); the general-path list's count was zeroed by the
    // previous step's first post kernel
    if (blockIdx.x == 0 && lane == 0) {
        *P.slow_prev = 0;
        if (P.slow_zero2) *P.slow_zero2 = 0;
        P.reset_count[0] = 0;  // the auto-reset lists of this step (main and side stream)
        P.reset_count[1] = 0;
    }
    const EnvV<C> V{&lds, j};
    // ---- state: the env-shared groups into LDS, this lane's agent into registers
    GroupRows<S, LY::kBoxW> rbox;
    GroupRows<S, LY::kItemW> ritem, rpend;
    GroupRows<S, LY::kHealW> rheal;
    // all four groups' loads in flight at once when their registers fit
    // (2v2: 22 words per lane); the big classes (ffa: 76) write each group
    // as soon as its loads are issued
    constexpr bool kBatch = decltype(rbox)::T + 2 * decltype(ritem)::T + decltype(rheal)::T <= 24;
    if (kBatch) {
        rbox.load(state, N, e0, LY::box);
        ritem.load(state, N, e0, LY::item);
        rpend.load(state, N, e0, LY::pend);
        rheal.load(state, N, e0, LY::heal);
    } else {
        decltype(rbox)::copy(lds.box, state, N, e0, LY::box);
        decltype(ritem)::copy(lds.item, state, N, e0, LY::item);
        decltype(rpend)::copy(lds.pend, state, N, e0, LY::pend);
        decltype(rheal)::copy(lds.heal, state, N, e0, LY::heal);
    }
    AgentL<C> g;
    {
        float d[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) d[q] = __uint_as_float(state[state_index(7 * i + q, ev, N)]);
        g.c = mk(d[0], d[1]);
        g.a = d[2];
        g.v = mk(d[3], d[4]);
        g.w = d[5];
        g.sleep = d[6];
        const int wr = LY::rule + i * LY::kRuleA;
        g.health = (int)state[state_index(wr, ev, N)];
        g.cause = (int)state[state_index(wr + 1, ev, N)];
        g.cooldown = (int)state[state_index(wr + 2, ev, N)];
        g.inv_n = (int)state[state_index(wr + 3, ev, N)];
#pragma unroll
        for (int k = 0; k < C::SM; ++k) {
            g.inv_meta[k] = (int)state[state_index(wr + 4 + 3 * k, ev, N)];
            g.inv_hx[k] = __uint_as_float(state[state_index(wr + 5 + 3 * k, ev, N)]);
            g.inv_hy[k] = __uint_as_float(state[state_index(wr + 6 + 3 * k, ev, N)]);
        }
    }
    const uint32_t alive_m0 = state[state_index(LY::alive, ev, N)];
    const uint32_t awake_m0 = state[state_index(LY::awake, ev, N)];
    // contact memory (the touching words kAAT, kAST[i]): any -> general path
    const uint32_t touch_w = state[state_index(LY::cont + 1 + i, ev, N)] |
                             (i == 0 ? state[state_index(LY::cont, ev, N)] : 0u);
    const bool alive = bit(alive_m0, i);
    bool awake = bit(awake_m0, i);
    // queue_actions (masurvival_env.py:741-755): alive agents only; every
    // byte load unconditional (index clamped into the env's row)
    int ac[6];
    bool bad = false;
    {
        // (three 2-B loads, issued on every lane: a lane past A reads agent
        // A - 1's row and drops it)
        const uint16_t* ar = reinterpret_cast<const uint16_t*>(actions + (ev * A + (i < A ? i : A - 1)) * 6);
        const uint32_t a01 = ar[0], a23 = ar[1], a45 = ar[2];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t word = k < 2 ? a01 : (k < 4 ? a23 : a45);
            const int x = i < A ? (int)(int8_t)((word >> (8 * (k & 1))) & 0xffu) : 0;
            const int hi = k < 3 ? 2 : 1;
            bad = bad || x < 0 || x > hi;
            ac[k] = x < 0 ? 0 : (x > hi ? hi : x);
        }
    }
    {
        // the reference asserts action_space.contains (masurvival_env.py:80);
        // a kernel cannot raise: clamped, and the env-step counted once
        const bool env_bad = env_ballot<C>(bad) != 0u && valid && i == 0;
        const uint64_t m = __ballot(env_bad);
        if (m && lane == __ffsll((unsigned long long)m) - 1) atomicAdd(P.bad_actions, __popcll(m));
    }
    if (kBatch) {
        rbox.write(lds.box);
        ritem.write(lds.item);
        rpend.write(lds.pend);
        rheal.write(lds.heal);
    }
    lds.ax[i * S + j] = g.c.x;
    lds.ay[i * S + j] = g.c.y;
    wave_lds_sync();  // the wave's LDS groups are loaded (one-wave block)
    MAS_PROF(P, 20);
    uint32_t dirty = kGDyn;
    // ---------------- pre_step ----------------
    // boxes: Object.pre_step drops last step's queued box items
    // (semantics.py:853-856): appended to the box items in queue order, up to
    // the capacity (spawn_bitem)
    const int npend = (int)V.pw(0), nbi0 = V.nbi();
    if (npend > 0) dirty |= kGItem | kGPend;
    for (int k = i; k < C::BM; k += AM) {
        if (k < npend && nbi0 + k < C::BM) {
#pragma unroll
            for (int q = 0; q < 5; ++q) V.iw(1 + 5 * (nbi0 + k) + q) = V.pw(1 + 5 * k + q);
        }
    }
    wave_lds_sync();
    if (i == 0) {
        V.iw(0) = (uint32_t)(nbi0 + npend < C::BM ? nbi0 + npend : C::BM);
        V.pw(0) = 0u;
    }
    // agents: DynamicMotors (simulation.py:407-424).  qs / qc: the agent's
    // rotation, which Melee's from_polar reuses below
    float qs = 0.0f, qc = 1.0f;
    if (alive) {
        const Rot q = rot_of(g.a);
        qs = q.s;
        qc = q.c;
        const float par = (float)(ac[0] - 1) * P.imp0;
        const float nor = (float)(ac[1] - 1) * P.imp1;
        const V2 J = mk(q.c * par + (-q.s) * nor, q.s * par + q.c * nor);
        const float ang = (float)(ac[2] - 1) * P.imp2;
        if (!awake) {  // wake
            awake = true;
            g.sleep = 0.0f;
        }
        g.v = add(g.v, scl(P.inv_mass, J));
        g.w += P.inv_I * cross(sub(g.c, g.c), J);
        g.w += P.inv_I * ang;
    }
    // UseLast (semantics.py:300-309): Heal.use (:646-649) / ObjectItem.use
    // (:830-836); the placed boxes join the boxes group in agent order
    bool used = false, use_heal = false, use_box = false;
    int pmeta = 0;
    float phx = 0.0f, phy = 0.0f;
    if (alive && ac[4] && g.inv_n != 0) {
        own_pop(g, pmeta, phx, phy);
        used = true;
        if (it_kind(pmeta) == kItemHeal) {
            use_heal = true;
            own_damage(g, alive, P, i, P.healing, kCauseNone);
        } else if (it_kind(pmeta) == kItemBox) {
            use_box = true;
        }
    }
    if (used) dirty |= kGRule | kGStat | kGBox;
    const uint32_t boxers = env_ballot<C>(use_box);
    const int nbox0 = V.nbox();
    wave_lds_sync();  // every lane has read nbox (slot j) before lane 0 updates it
    if (use_box) {
        // spawn_box: the agent's rank among this step's box users
        const int b = nbox0 + __popc(boxers & ((1u << i) - 1u));
        if (b < C::BM) {
            const V2 off = from_polar(P.box_item_offset, g.a);
            const V2 pos = add(g.c, off);
            V.bw(1 + 6 * b) = __float_as_uint(pos.x);
            V.bw(2 + 6 * b) = __float_as_uint(pos.y);
            V.bw(3 + 6 * b) = __float_as_uint(phx);
            V.bw(4 + 6 * b) = __float_as_uint(phy);
            V.bw(5 + 6 * b) = (uint32_t)mk_boxmeta(it_rot(pmeta), it_copied(pmeta), 0,
                                                   P.ownership ? it_owner(pmeta) : kCauseNone, kCauseNone);
            V.bw(6 + 6 * b) = 0u;
        }
    }
    if (i == 0 && boxers) {
        const int nb = nbox0 + __popc(boxers);
        V.bw(0) = (uint32_t)(nb < C::BM ? nb : C::BM);
    }
    wave_lds_sync();
    // GiveLast (semantics.py:335-370): nearest body centre within the give
    // radius, then the gives in agent order (a later giver may pass on what
    // it was just given; a full inventory loses the item, quirk D3)
    int taker = -1;
    if (alive && ac[5]) {
        const V2 c = g.c;
        float mind = INFINITY;
        int best = -1;
        auto consider = [&](V2 oc, int id) {
            if (!circle_test_point(P.give_r, c, oc)) return;
            const float dd = len(sub(c, oc));
            if (dd < mind) { mind = dd; best = id; }
        };
        // (over the class maxima, the counts as guards: the LDS reads up front;
        // the same bodies in the same order)
        const int nb = V.nbox(), ni = V.nbi(), nh = V.nheal();
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < nb) consider(V.bp(b), BIdx<C>::box + b);
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < ni) consider(V.ip(b), BIdx<C>::bitem + b);
#pragma unroll
        for (int h = 0; h < C::HM; ++h)
            if (h < nh) consider(V.hp(h), BIdx<C>::heal + h);
#pragma unroll
        for (int w = 0; w < kNumWalls; ++w) consider(P.wall_pos[w], BIdx<C>::wall + w);
        const uint32_t alive_m = alive_m0;
#pragma unroll
        for (int k = 0; k < AM; ++k)
            if (k != i && bit(alive_m, k)) consider(V.agent(k), BIdx<C>::agent + k);
        taker = best;
    }
    {
        bool gave_any = false;
#pragma unroll
        for (int q = 0; q < AM; ++q) {
            // giver q of every env: its pop, then its taker's take
            bool give = false;
            int gm = 0;
            float gx = 0.0f, gy = 0.0f;
            int t = taker - BIdx<C>::agent;
            if (i == q && alive && ac[5] && taker >= BIdx<C>::agent && !(P.teams && team_of(P, t) != team_of(P, i)) &&
                g.inv_n != 0) {
                own_pop(g, gm, gx, gy);
                give = true;
            }
            const bool gb = env_bcast<C>((int)give, q) != 0;
            const int tb = env_bcast<C>(t, q);
            const int mb = env_bcast<C>(gm, q);
            const float xb = env_bcast<C>(gx, q), yb = env_bcast<C>(gy, q);
            if (gb && i == tb) own_take(g, P, mb, xb, yb);
            gave_any = gave_any || gb;
        }
        if (gave_any) dirty |= kGRule;
    }
    MAS_PROF(P, 21);
    // Melee / ContinuousMelee (semantics.py:531-554, 584-610): every ray
    // first (each lane casts its own agent's), then the attacks in agent
    // order; the cooldowns are those the attack loop sees
    {
        const bool on_cd = P.melee_cd > 0 && g.cooldown > 0;
        const bool need = valid && alive && ac[3] && !on_cd;
        int target = -1;
        if (__any(need)) {
            FixTab<C, S> T{lds.tab, j};
            if (i == 0) build_fixtab_v(V, P, T, alive_m0);
            wave_lds_sync();
            if (need) {
                // from_polar(range, angle) with the motors' rotation of the angle
                const V2 hand = mk(qc * P.melee_range + (-qs) * 0.0f, qs * P.melee_range + qc * 0.0f);
                target = ray_cast_fixtab(P, T, g.c, add(g.c, hand));
            }
        }
        const int cause_i = P.teams ? kCauseBadge + team_of(P, i) : i;
        bool hit_any = false;
#pragma unroll
        for (int q = 0; q < AM; ++q) {
            const bool att = i == q && alive && target >= 0 && ac[3] && !on_cd;
            const bool ab = env_bcast<C>((int)att, q) != 0;
            const int tg = env_bcast<C>(target, q);
            const int cz = env_bcast<C>(cause_i, q);
            if (ab) {
                if (tg >= BIdx<C>::agent) {
                    if (i == tg - BIdx<C>::agent) own_damage(g, alive, P, i, -P.melee_damage, cz);
                } else if (tg < BIdx<C>::bitem && i == q) {
                    lds_box_damage(V, tg, -P.melee_damage, cz);
                }
                hit_any = true;
            }
            wave_lds_sync();  // attacker q's box damage is visible to the next attacker
            if (att && P.melee_cd > 0) g.cooldown = P.melee_cd;
        }
        if (hit_any) dirty |= kGRule | kGBox;
        if (P.melee_cd > 0 && g.cooldown > 0) {
            g.cooldown -= 1;
            dirty |= kGRule;
        }
    }
    MAS_PROF(P, 22);
    // ---------------- stores: only the groups this step changed ----------------
    // (step_pre's dirty mask, ORed over the env's agents)
    uint32_t dirty_env = dirty;
#pragma unroll
    for (int o = 1; o < AM; o <<= 1) dirty_env |= (uint32_t)__shfl_xor((int)dirty_env, o, 64);
    const uint32_t awake_pre = env_ballot<C>(awake) | (awake_m0 & ~((AM >= 32) ? 0xffffffffu : ((1u << AM) - 1u)));
    // (every ballot in uniform control flow: a ballot counts active lanes only)
    const uint32_t heals_used = env_ballot<C>(use_heal), boxes_used = env_ballot<C>(use_box);
#if MAS_PRE_BODY_ONCE
    // the body words before the fast physics: stored below, once, only when
    // the fast path fails (the general path restarts from them)
    const float dpre[7] = {g.c.x, g.c.y, g.a, g.v.x, g.v.y, g.w, g.sleep};
#endif
    if (valid) {
#if !MAS_PRE_BODY_ONCE
        const float d[7] = {g.c.x, g.c.y, g.a, g.v.x, g.v.y, g.w, g.sleep};
#pragma unroll
        for (int q = 0; q < 7; ++q) state[state_index(7 * i + q, e, N)] = __float_as_uint(d[q]);
        if (i == 0) state[state_index(LY::awake, e, N)] = awake_pre;
#endif
        if (dirty_env & kGRule) {
            const int wr = LY::rule + i * LY::kRuleA;
            state[state_index(wr, e, N)] = (uint32_t)g.health;
            state[state_index(wr + 1, e, N)] = (uint32_t)g.cause;
            state[state_index(wr + 2, e, N)] = (uint32_t)g.cooldown;
            state[state_index(wr + 3, e, N)] = (uint32_t)g.inv_n;
#pragma unroll
            for (int k = 0; k < C::SM; ++k) {
                state[state_index(wr + 4 + 3 * k, e, N)] = (uint32_t)g.inv_meta[k];
                state[state_index(wr + 5 + 3 * k, e, N)] = __float_as_uint(g.inv_hx[k]);
                state[state_index(wr + 6 + 3 * k, e, N)] = __float_as_uint(g.inv_hy[k]);
            }
        }
        if ((dirty_env & kGStat) && i == 0) {
            // stats[17] += heals used, stats[18] += boxes placed (step_pre)
            float* st = reinterpret_cast<float*>(state);
            st[state_index(LY::stat + 17, e, N)] += (float)__popc(heals_used);
            st[state_index(LY::stat + 18, e, N)] += (float)__popc(boxes_used);
        }
    }
    // the env-shared groups from LDS, for the slots whose env changed them
    {
        const bool lead = i == 0;
        const uint64_t mb = __ballot(lead && (dirty_env & kGBox));
        const uint64_t mi = __ballot(lead && (dirty_env & kGItem));
        const uint64_t mp = __ballot(lead && (dirty_env & kGPend));
        // slot bits: lane j * AM of the wave is slot j's lead
        uint32_t sb = 0, si = 0, sp = 0;
#pragma unroll
        for (int q = 0; q < S; ++q) {
            sb |= (uint32_t)((mb >> (q * AM)) & 1ull) << q;
            si |= (uint32_t)((mi >> (q * AM)) & 1ull) << q;
            sp |= (uint32_t)((mp >> (q * AM)) & 1ull) << q;
        }
        if (sb) group_store<S, LY::kBoxW>(lds.box, state, N, e0, LY::box, sb);
        if (si) group_store<S, LY::kItemW>(lds.item, state, N, e0, LY::item, si);
        if (sp) group_store<S, LY::kItemW>(lds.pend, state, N, e0, LY::pend, sp);
    }
    MAS_PROF(P, 23);
    // ---------------- speculative contact-free physics (fast_phys) ----------------
    bool ok = touch_w == 0u;
    ok = env_ballot<C>(!ok) == 0u && !P.force_general;
    if (ok) {
        const float dt = (float)(1.0 / 60.0);
        bool aw = awake;
        ok = world_step_fast_lane(g, alive, aw, V, P, i, dt);
        if (ok) ok = world_step_fast_lane(g, alive, aw, V, P, i, dt);
        // (ok is the same on every lane of an env: the group's ballot is whole)
        const uint32_t awm = env_ballot<C>(aw) | (awake_m0 & ~((AM >= 32) ? 0xffffffffu : ((1u << AM) - 1u)));
        if (ok && valid) {
            const float d[7] = {g.c.x, g.c.y, g.a, g.v.x, g.v.y, g.w, g.sleep};
#pragma unroll
            for (int q = 0; q < 7; ++q) state[state_index(7 * i + q, e, N)] = __float_as_uint(d[q]);
            if (i == 0) {
                state[state_index(LY::awake, e, N)] = awm;
                state[state_index(LY::invdt, e, N)] = __float_as_uint(dt > 0.0f ? 1.0f / dt : 0.0f);
            }
        }
    }
#if MAS_PRE_BODY_ONCE
    if (!ok && valid) {
#pragma unroll
        for (int q = 0; q < 7; ++q) state[state_index(7 * i + q, e, N)] = __float_as_uint(dpre[q]);
        if (i == 0) state[state_index(LY::awake, e, N)] = awake_pre;
    }
#endif
    MAS_PROF(P, 24);
    // the general-path list append and the slow routing, one lane per env
    const bool lead = i == 0 && valid;
    bool slow = false;
    if (lead && P.slow_k > 0 && P.slow_flag[e]) {
        slow = P.slow_route && !ok;
        P.slow_flag[e] = 0;  // k_gen_solve_g sets it again if it still is
    }
    if (lead) P.gen_flag[e] = ok ? 0 : (slow ? 2 : 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const bool mine = lead && !ok && slow == (q == 1);
        const uint64_t m = __ballot(mine);
        if (m == 0ull) continue;
        // the general-path list: this block's shard (Params::list_shards):
        // with the XCD-aware order, shard s takes the s-th run of
        // ceil(blocks / shards) blocks (a contiguous env range: the general
        // kernel's XCD-mates then read the lines the range shares), else
        // every list_shards-th block; at most ceil(blocks / shards) blocks
        // either way (list_cap)
        const unsigned bps = (gridDim.x + (unsigned)P.list_shards - 1) / (unsigned)P.list_shards;
        const int sh = q ? 0 : (MAS_XCD_SWZ && MAS_LIST_XCD ? (int)(xcd_block() / bps) : (int)(blockIdx.x % (unsigned)P.list_shards));
        int* list = q ? P.slow_list : P.phys_list + (int64_t)sh * P.list_cap;
        int* count = q ? P.slow_count : P.phys_count + sh * kShardStride;
        const int64_t cap = q ? N : (int64_t)P.list_cap;
        const int leader = __ffsll((unsigned long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(count, __popcll(m));
        base = __shfl(base, leader, 64);
        if (mine) {
            const int64_t at = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
            if (at < cap) list[at] = (int)e;
            else atomicAdd(P.list_overflow, 1);
        }
    }
    MAS_PROF(P, 25);
    MAS_PROF_FLUSH(P, 1, 20);
}

}  // namespace mas
