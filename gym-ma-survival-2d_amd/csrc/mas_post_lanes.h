// mas_post_lanes.h -- the post-physics phases of the MaSurvival step in one
// launch on agent lanes (gfx950 HIP): the boxes' Health.post_step and
// despawn, Cameras.post_step, the agents' post_step (deaths + DeathDrop,
// AutoPickup, SafeZone), rewards, done, stats and the observation rows.
//
// Lane (env slot j, agent i) as in k_pre_lanes (mas_lanes.h): C::AM lanes
// per env, kWG / C::AM envs per wave.  The env's shared groups (boxes,
// pending drops, box items, heals, the zone) and a table of its agents'
// poses and healths live in LDS, loaded once per step by cooperative row
// loads; each lane holds its own agent's rule state.  This replaces three
// launches (k_cameras, k_post, k_obs) that each reloaded the same groups
// from HBM: the observation rows are built from the post-step state already
// in LDS.  Env-level steps whose order is observable (the box compaction,
// DeathDrop's RNG draws and spawns, the pickup compaction, the zone tick,
// the stats) run on the env's leader lane (agent 0) over LDS; per-agent
// steps (the camera cone queries, the pickup lists and takes, the zone
// damage, the rewards, the contact rows of a dead agent) on the agent's
// lane.  Same operations on the same values as box_health, update_seen_cam,
// step_post and write_obs_row (mas_step.h), so the same bits.
//
// Reference: masurvival/semantics.py:270-283 (AutoPickup), 387-396
// (DeathDrop), 403-506 (Health), 704-811 (SafeZone), 853-861 / 907-912
// (Object / OwnedObject despawn); simulation.py:314-354 (Cameras);
// envs/masurvival_env.py:510-739 (fetch_observations), 757-831 (rewards,
// is_done), 483-508 (stats).
#pragma once

#include "mas_lanes.h"

namespace mas {

constexpr int kPostObsW = 32;  // obs column window of the LDS tile (MAS_POST_OBS_SEQ=0)
// obs rows: 1 = each lane generates its own row once, in column order, and
// stores it with 16-B (8-B, 4-B when D is not a multiple of 4 / 2) stores
// (write_obs_row_seq); 0 = column windows of an LDS tile (write_obs_row_v)
#ifndef MAS_POST_OBS_SEQ
#define MAS_POST_OBS_SEQ 1
#endif

template <class C>
struct PostLds {
    static constexpr int S = kWG / C::AM;  // env slots per wave
    using LY = Lay<C>;
    static constexpr int kAgF = 7;                      // agent table: cx cy a vx vy w health
    static constexpr int kDropW = 3 + 3 * C::SM;        // a dying agent: cx cy n, then (meta hx hy) per slot
    uint32_t box[LY::kBoxW * S];
    uint32_t item[LY::kItemW * S];
    uint32_t heal[LY::kHealW * S];
    uint32_t zone[LY::kZoneW * S];
    float ag[kAgF * C::AM * S];  // [field][agent][slot]
    uint32_t seen[C::NB * S];    // camera-position mask byte per body (low 8 bits)
    int64_t eidx[S];             // env of each slot
    uint32_t misc[S];            // per slot: the despawn's kept mask | nbox before << 24 | any dead << 23
    uint32_t alivem[S];          // per slot: the alive mask the cameras see
    union {
        struct {
            uint16_t list[C::NB * kWG];  // the wave's (camera position, lane, body) ray list
        } cam;
        struct {
            uint32_t drop[kDropW * C::AM * S];  // [field][agent][slot]
            double ang[C::AM * C::SM * S];       // DeathDrop angles, [k][slot]
        } dd;
#if !MAS_POST_OBS_SEQ
        float tile[kWG * (kPostObsW + 1)];  // obs rows, one column window
#endif
    } u;
};

// slot j's view of PostLds
template <class C>
struct PostV {
    static constexpr int S = kWG / C::AM;
    PostLds<C>* d;
    int j;
    __device__ uint32_t& bw(int w) const { return d->box[w * S + j]; }
    __device__ uint32_t& iw(int w) const { return d->item[w * S + j]; }
    __device__ uint32_t& hw(int w) const { return d->heal[w * S + j]; }
    __device__ uint32_t& zw(int w) const { return d->zone[w * S + j]; }
    __device__ float& ag(int f, int k) const { return d->ag[(f * C::AM + k) * S + j]; }
    __device__ uint32_t& sn(int body) const { return d->seen[body * S + j]; }
    __device__ int nbox() const { return (int)bw(0); }
    __device__ V2 bp(int b) const { return mk(__uint_as_float(bw(1 + 6 * b)), __uint_as_float(bw(2 + 6 * b))); }
    __device__ float bhx(int b) const { return __uint_as_float(bw(3 + 6 * b)); }
    __device__ float bhy(int b) const { return __uint_as_float(bw(4 + 6 * b)); }
    __device__ int bmeta(int b) const { return (int)bw(5 + 6 * b); }
    __device__ int bhealth(int b) const { return (int)bw(6 + 6 * b); }
    __device__ int nbi() const { return (int)iw(0); }
    __device__ V2 ip(int b) const { return mk(__uint_as_float(iw(1 + 5 * b)), __uint_as_float(iw(2 + 5 * b))); }
    __device__ float ihx(int b) const { return __uint_as_float(iw(3 + 5 * b)); }
    __device__ float ihy(int b) const { return __uint_as_float(iw(4 + 5 * b)); }
    __device__ int imeta(int b) const { return (int)iw(5 + 5 * b); }
    __device__ int nheal() const { return (int)hw(0); }
    __device__ V2 hp(int h) const { return mk(__uint_as_float(hw(1 + 2 * h)), __uint_as_float(hw(2 + 2 * h))); }
    __device__ V2 agent(int k) const { return mk(ag(0, k), ag(1, k)); }
    // zone words (visit_state: zc[9] (x, y), phase, t_cd, t_sh, endgame, zpos, zrad)
    __device__ V2 zc(int k) const { return mk(__uint_as_float(zw(2 * k)), __uint_as_float(zw(2 * k + 1))); }
    static constexpr int kZPhase = 2 * kMaxPhases, kZCd = kZPhase + 1, kZSh = kZPhase + 2, kZEnd = kZPhase + 3,
                         kZPx = kZPhase + 4, kZPy = kZPhase + 5, kZRad = kZPhase + 6;
};

// env-slot table versions of the cooperative row loads / stores (the slots'
// envs need not be consecutive: the slow list); unrolled like group_load
template <int S, int NW>
struct SlotRows {
    static constexpr int T = (NW * S + kWG - 1) / kWG;
    uint32_t v[T];
    __device__ __forceinline__ void load(const uint32_t* __restrict__ state, int64_t N, const int64_t* eidx, int w0)
    {
        const int lane = (int)threadIdx.x;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int i0 = lane + t * kWG;
            const int idx = i0 < NW * S ? i0 : NW * S - 1;
            const int w = idx / S, j = idx - w * S;
            v[t] = state[state_index(w0 + w, eidx[j], N)];
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
    // load + write in chunks of 8 rounds (GroupRows::copy)
    __device__ __forceinline__ static void copy(uint32_t* __restrict__ dst, const uint32_t* __restrict__ state,
                                                int64_t N, const int64_t* eidx, int w0)
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
                u[t - c0] = state[state_index(w0 + w, eidx[j], N)];
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
__device__ __forceinline__ void slot_store(const uint32_t* __restrict__ src, uint32_t* __restrict__ state, int64_t N,
                                           const int64_t* eidx, int w0, uint32_t slots)
{
    constexpr int T = (NW * S + kWG - 1) / kWG;
    const int lane = (int)threadIdx.x;
    const int64_t ex = eidx[lane % S];  // (a round's lanes hold slots lane % S: kWG is a multiple of S)
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
            if (idx < NW * S && ((slots >> j) & 1u)) state[state_index(w0 + w, ex, N)] = v[t - c0];
        }
    }
}

// slots whose env-leader lane (agent 0) has b set
template <class C>
__device__ __forceinline__ uint32_t slot_mask(bool b)
{
    constexpr int S = kWG / C::AM;
    const uint64_t m = __ballot(b && ((int)threadIdx.x % C::AM) == 0);
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < S; ++q) r |= (uint32_t)((m >> (q * C::AM)) & 1ull) << q;
    return r;
}

// ray_cast_fixtab (mas_step.h) with every input read from slot j's LDS
// groups and agent table instead of a fixture table: the same broadphase
// cull and the same exact tests in the same canonical order, so the same
// first hit
template <class C>
__device__ __forceinline__ int ray_cast_pv(const Params& P, const PostV<C>& V, uint32_t alive, V2 p1, V2 p2)
{
    constexpr float m = 1e-3f;
    const V2 r = sub(p2, p1);
    const float rl = len(r);
    const V2 rn = rl > 0.0f ? scl(1.0f / rl, r) : mk(0.0f, 0.0f);
    const V2 v = mk(-rn.y, rn.x);
    const V2 av = mk(fabsf(v.x), fabsf(v.y));
    const float lox = fminf(p1.x, p2.x) - m, loy = fminf(p1.y, p2.y) - m;
    const float hix = fmaxf(p1.x, p2.x) + m, hiy = fmaxf(p1.y, p2.y) + m;
    auto keep = [&](V2 c, float ex, float ey) -> bool {
        if (c.x - ex > hix || c.x + ex < lox || c.y - ey > hiy || c.y + ey < loy) return false;
        return fabsf(dot(v, sub(p1, c))) - (av.x * ex + av.y * ey) <= m;
    };
    // (over the class maxima with the counts as guards: every LDS read of the
    // cull issued up front instead of one loop round trip per body)
    const int nbox = V.nbox(), nbi = V.nbi(), nheal = V.nheal();
    uint64_t mask = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b < nbox && keep(V.bp(b), V.bhx(b), V.bhy(b))) mask |= 1ull << (BIdx<C>::box + b);
        if (b < nbi && keep(V.ip(b), P.bitem_r, P.bitem_r)) mask |= 1ull << (BIdx<C>::bitem + b);
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h)
        if (h < nheal && keep(V.hp(h), P.heal_r, P.heal_r)) mask |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        const V2 c = scl(0.5f, add(P.wall_lo[w], P.wall_hi[w]));
        const V2 e = scl(0.5f, sub(P.wall_hi[w], P.wall_lo[w]));
        if (keep(c, e.x + m, e.y + m)) mask |= 1ull << (BIdx<C>::wall + w);
    }
#pragma unroll
    for (int k = 0; k < C::AM; ++k)
        if (bit(alive, k) && keep(V.agent(k), P.agent_r, P.agent_r)) mask |= 1ull << (BIdx<C>::agent + k);
    float maxf = 1.0f;
    int hit = -1;
    while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        float f;
        const bool is_box = k < BIdx<C>::bitem;
        const bool is_wall = k >= BIdx<C>::wall && k < BIdx<C>::agent;
        if (is_box || is_wall) {
            Poly4 poly;
            Rot q = kIdRot;
            V2 c;
            if (is_box) {
                const int meta = V.bmeta(k);
                poly = box_poly(V.bhx(k), V.bhy(k), box_rot(meta), box_copied(meta));
                c = V.bp(k);
            } else {
                poly = P.wall_poly;
                const int w = k - BIdx<C>::wall;
                c = opq(P.wall_pos[0]);
                q.s = opq(P.wall_q[0].s);
                q.c = opq(P.wall_q[0].c);
#pragma unroll
                for (int q2 = 1; q2 < kNumWalls; ++q2)
                    if (q2 == w) { c = opq(P.wall_pos[q2]); q.s = opq(P.wall_q[q2].s); q.c = opq(P.wall_q[q2].c); }
            }
            f = ray_poly(poly, c, q, p1, p2, maxf);
        } else {
            V2 c;
            float rad;
            if (k < BIdx<C>::heal) { c = V.ip(k - BIdx<C>::bitem); rad = P.bitem_r; }
            else if (k < BIdx<C>::wall) { c = V.hp(k - BIdx<C>::heal); rad = P.heal_r; }
            else { c = V.agent(k - BIdx<C>::agent); rad = P.agent_r; }
            f = ray_circle(rad, c, p1, p2, maxf);
        }
        if (f >= 0.0f) {
            hit = k;
            maxf = f;
            if (maxf == 0.0f) break;
        }
    }
    return hit;
}

// boxes: Health.post_step + Object / OwnedObject despawn (box_health,
// mas_step.h) of slot j on LDS, by its leader lane.  Returns whether the
// box / pending groups changed; kept, nb: the despawn compaction's kept
// boxes and nbox before it (any_dead: a compaction ran).
template <class C>
__device__ __forceinline__ bool box_health_v(const PostV<C>& V, const Params& P, bool& any_dead, uint32_t& kept,
                                             int& nb, uint32_t* __restrict__ state, int64_t N, int64_t e, bool store)
{
    using LY = Lay<C>;
    bool changed = false;
    any_dead = false;
    kept = 0;
    nb = V.nbox();
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b >= nb) continue;
        const int meta = V.bmeta(b);
        if (!box_hinit(meta)) {
            V.bw(5 + 6 * b) = (uint32_t)mk_boxmeta(box_rot(meta), box_copied(meta), 1, box_vuln(meta), box_cause(meta));
            V.bw(6 + 6 * b) = (uint32_t)P.box_health;
            changed = true;
        }
        if (V.bhealth(b) <= 0) any_dead = true;
        else kept |= 1u << b;
    }
    if (any_dead) {
        changed = true;
        // stable compaction; dead boxes queue (pos, copy_shape(proto), cause)
        int wi = 0;
        for (int b = 0; b < nb; ++b) {
            const V2 p = V.bp(b);
            const float hx = V.bhx(b), hy = V.bhy(b);
            const int meta = V.bmeta(b), hl = V.bhealth(b);
            if (hl <= 0) {
                const int rot = box_copy_rot(hx, hy, box_rot(meta));
                const int pm = mk_bimeta(rot, 1, box_cause(meta));
                // Object.next_spawns, straight to HBM (the pending group is
                // otherwise untouched here; k_pre drained it this step)
                const int np_ = (int)state[state_index(LY::pend, e, N)];
                if (store) {
                    if (np_ < C::BM) {
                        const uint32_t w5[5] = {__float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(hx),
                                                __float_as_uint(hy), (uint32_t)pm};
#pragma unroll
                        for (int q = 0; q < 5; ++q) state[state_index(LY::pend + 1 + 5 * np_ + q, e, N)] = w5[q];
                    }
                    state[state_index(LY::pend, e, N)] = (uint32_t)(np_ + 1);
                }
            } else {
                if (wi != b) {
#pragma unroll
                    for (int q = 1; q <= 6; ++q) V.bw(q + 6 * wi) = V.bw(q + 6 * b);
                }
                ++wi;
            }
        }
        V.bw(0) = (uint32_t)wi;
    }
    return changed;
}

// SafeZone.tick (zone_tick, mas_step.h) on slot j's LDS zone words
template <class C>
__device__ __forceinline__ void zone_tick_v(const PostV<C>& V, const Params& P)
{
    using PV = PostV<C>;
    int t_cd = (int)V.zw(PV::kZCd), t_sh = (int)V.zw(PV::kZSh), phase = (int)V.zw(PV::kZPhase);
    const int endgame = (int)V.zw(PV::kZEnd);
    if (t_cd == 0) {
        if (endgame) return;
        t_sh -= 1;
        V.zw(PV::kZSh) = (uint32_t)t_sh;
        if (t_sh > 0) {
            const double t = (double)t_sh / (double)P.zone_cooldown;
            double r1 = 0.0, r2 = 0.0;
#pragma unroll
            for (int k = 0; k + 1 < kMaxPhases; ++k)
                if (k == phase) { r1 = opq(P.zrad[k]); r2 = opq(P.zrad[k + 1]); }
            const V2 c1 = V.zc(phase), c2 = V.zc(phase + 1);
            const double radius = t * r1 + (1.0 - t) * r2;
            const float tf = (float)t, tf1 = (float)(1.0 - t);
            const V2 zp = add(scl(tf, c1), scl(tf1, c2));
            V.zw(PV::kZRad) = __float_as_uint((float)radius);
            V.zw(PV::kZPx) = __float_as_uint(zp.x);
            V.zw(PV::kZPy) = __float_as_uint(zp.y);
            return;
        }
        V.zw(PV::kZCd) = (uint32_t)P.zone_cooldown;
        phase += 1;
        V.zw(PV::kZPhase) = (uint32_t)phase;
        const V2 zp = V.zc(phase);
        V.zw(PV::kZPx) = __float_as_uint(zp.x);
        V.zw(PV::kZPy) = __float_as_uint(zp.y);
        float zr = __uint_as_float(V.zw(PV::kZRad));
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k == phase) zr = opq(P.zradf[k]);
        V.zw(PV::kZRad) = __float_as_uint(zr);
        if (phase == P.zone_phases - 1) V.zw(PV::kZEnd) = 1u;
    } else {
        t_cd -= 1;
        V.zw(PV::kZCd) = (uint32_t)t_cd;
        if (t_cd > 0) return;
        V.zw(PV::kZSh) = (uint32_t)P.zone_cooldown;
    }
}

// The obs row of agent i of slot j (write_obs_row, mas_step.h) from LDS:
// the agent table (post-step healths), the post-tick zone, the post-pickup
// heals, boxes and box items and their seen bytes; own: the lane's
// inventory's last item.  Sink: WinRow-like (column window).
struct WinRowP {
    float* p;
    int c0;
    __device__ void operator()(int k, float v)
    {
        const unsigned kk = (unsigned)(k - c0);
        p[kk < (unsigned)kPostObsW ? kk : (unsigned)kPostObsW] = v;
    }
    __device__ bool want(int off, int len) const { return off < c0 + kPostObsW && off + len > c0; }
};

template <class C, class Sink>
__device__ __forceinline__ void write_obs_row_v(const PostV<C>& V, const Params& P, uint32_t alive_m, int i,
                                                int lastmeta, float lhx, float lhy, Sink& row)
{
    using PV = PostV<C>;
    const int A = P.A, as_ = P.as_;
    const bool alive = bit(alive_m, i);
    const int pp = __popc(alive_m & ((1u << i) - 1u));  // post-despawn list position (quirk D1)
    // agent + others rows (_fetch_agents_observations :659-704)
    if (row.want(P.o_agent, as_) || row.want(P.o_oth, (A - 1) * as_) || row.want(P.o_othm, A - 1)) {
        for (int k = 0; k < A; ++k) {
            const bool ak = bit(alive_m, k);
            const int ok = k < i ? k : k - 1;
            int o = k == i ? P.o_agent : P.o_oth + ok * as_;
            if (!row.want(o, as_) && !(k != i && row.want(P.o_othm + ok, 1))) continue;
            row(o++, (float)k);
            if (P.teams) row(o++, (float)team_of(P, k));
            row(o++, ak ? V.ag(6, k) : 0.0f);
#pragma unroll
            for (int f = 0; f < 6; ++f) row(o++, ak ? V.ag(f, k) : 0.0f);
            if (k != i) {
                // others_mask: seen list at the post-despawn list index (quirk D1)
                float m = 1.0f;
                if (alive && ak && (V.sn(BIdx<C>::agent + k) >> pp) & 1u) m = 0.0f;
                row(P.o_othm + ok, m);
            }
        }
    }
    if (row.want(P.o_zone, 6)) {
        const int phase = (int)V.zw(PV::kZPhase);
        row(P.o_zone + 0, __uint_as_float(V.zw(PV::kZPx)));
        row(P.o_zone + 1, __uint_as_float(V.zw(PV::kZPy)));
        row(P.o_zone + 2, __uint_as_float(V.zw(PV::kZRad)));
        float z3 = 0.0f, z4 = 0.0f, z5 = 0.0f;
        if (phase < P.zone_phases - 1) {
            const V2 zn = V.zc(phase + 1);
            z3 = zn.x;
            z4 = zn.y;
#pragma unroll
            for (int k = 0; k < kMaxPhases; ++k)
                if (k == phase + 1) z5 = opq(P.zradf[k]);
        }
        row(P.o_zone + 3, z3);
        row(P.o_zone + 4, z4);
        row(P.o_zone + 5, z5);
    }
    if (P.H > 0 && (row.want(P.o_heal, 2 * P.H) || row.want(P.o_healm, P.H))) {
        const int nh = V.nheal();
        for (int h = 0; h < P.H; ++h) {
            if (!row.want(P.o_heal + 2 * h, 2) && !row.want(P.o_healm + h, 1)) continue;
            const bool present = h < nh;
            const V2 hp = V.hp(h);
            row(P.o_heal + 2 * h, present ? hp.x : 0.0f);
            row(P.o_heal + 2 * h + 1, present ? hp.y : 0.0f);
            float m;
            if (P.omniscient) m = present ? 0.0f : 1.0f;
            else m = (present && alive && ((V.sn(BIdx<C>::heal + h) >> pp) & 1u)) ? 0.0f : 1.0f;
            row(P.o_healm + h, m);
        }
    }
    if (P.B > 0 && (row.want(P.o_box, 11 * P.B) || row.want(P.o_boxm, P.B))) {
        const int nb = V.nbox();
        for (int b = 0; b < P.B; ++b) {
            const bool present = b < nb;
            if (row.want(P.o_box + 11 * b, 11)) {
                const int meta = V.bmeta(b);
                const Poly4 poly = box_poly(V.bhx(b), V.bhy(b), box_rot(meta), box_copied(meta));
                const V2 bp = V.bp(b);
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    row(P.o_box + 11 * b + 2 * v, present ? poly.v[v].x : 0.0f);
                    row(P.o_box + 11 * b + 2 * v + 1, present ? poly.v[v].y : 0.0f);
                }
                row(P.o_box + 11 * b + 8, present ? bp.x : 0.0f);
                row(P.o_box + 11 * b + 9, present ? bp.y : 0.0f);
                row(P.o_box + 11 * b + 10, 0.0f);  // box bodies always have angle 0
            }
            if (!row.want(P.o_boxm + b, 1)) continue;
            float m;
            if (P.omniscient) m = present ? 0.0f : 1.0f;
            else m = (present && alive && ((V.sn(BIdx<C>::box + b) >> pp) & 1u)) ? 0.0f : 1.0f;
            row(P.o_boxm + b, m);
        }
    }
    if (P.B > 0 && (row.want(P.o_bi, 10 * P.B) || row.want(P.o_bim, P.B))) {
        const int ni = V.nbi();
        for (int b = 0; b < P.B; ++b) {
            const bool present = b < ni;
            if (row.want(P.o_bi + 10 * b, 10)) {
                const float hx = V.ihx(b), hy = V.ihy(b);
                const int rot = bi_rot(V.imeta(b));
                const V2 ip = V.ip(b);
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const V2 cv = box_corner(hx, hy, rot + v);
                    row(P.o_bi + 10 * b + 2 * v, present ? cv.x : 0.0f);
                    row(P.o_bi + 10 * b + 2 * v + 1, present ? cv.y : 0.0f);
                }
                row(P.o_bi + 10 * b + 8, present ? ip.x : 0.0f);
                row(P.o_bi + 10 * b + 9, present ? ip.y : 0.0f);
            }
            if (!row.want(P.o_bim + b, 1)) continue;
            float m;
            if (P.omniscient) m = present ? 0.0f : 1.0f;
            else m = (present && alive && ((V.sn(BIdx<C>::bitem + b) >> pp) & 1u)) ? 0.0f : 1.0f;
            row(P.o_bim + b, m);
        }
    }
    // lidars: zeros here; k_lidar writes the columns afterwards
    if (P.n_lasers > 0 && row.want(P.o_lid, P.n_lasers)) {
        for (int k = 0; k < P.n_lasers; ++k) row(P.o_lid + k, 0.0f);
    }
    // usable inventory slots (:620-654)
    if (row.want(P.o_hs, 1) || row.want(P.o_hsm, 1) || row.want(P.o_bs, 8) || row.want(P.o_bsm, 1)) {
        if (P.H > 0) {
            const bool isheal = it_kind(lastmeta) == kItemHeal;
            row(P.o_hs, isheal ? (float)P.healing : 0.0f);
            row(P.o_hsm, isheal ? 0.0f : 1.0f);
        }
        if (P.B > 0) {
            const bool isbox = it_kind(lastmeta) == kItemBox;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const V2 cv = box_corner(lhx, lhy, it_rot(lastmeta) + v);
                row(P.o_bs + 2 * v, isbox ? cv.x : 0.0f);
                row(P.o_bs + 2 * v + 1, isbox ? cv.y : 0.0f);
            }
            row(P.o_bsm, isbox ? 0.0f : 1.0f);
        }
    }
}

// A lane's obs row in column order (the layout of build_layout, mas_capi.hip:
// the observation keys sorted by name), into a sink that packs consecutive
// columns into 16-B stores.  Same values as write_obs_row_v.
struct SeqRow {
    float* p;   // the row
    int vm1;    // store width in floats - 1 (3, 1 or 0; wave-uniform)
    int k = 0;  // next column (wave-uniform)
    float b0 = 0.0f, b1 = 0.0f, b2 = 0.0f, b3 = 0.0f;
    __device__ __forceinline__ void put(float v)
    {
        const int s = k & vm1;
        if (s == 0) b0 = v;
        else if (s == 1) b1 = v;
        else if (s == 2) b2 = v;
        else b3 = v;
        if (s == vm1) {
            float* q = p + (k - s);
            if (vm1 == 3) *reinterpret_cast<float4*>(q) = make_float4(b0, b1, b2, b3);
            else if (vm1 == 1) *reinterpret_cast<float2*>(q) = make_float2(b0, b1);
            else *q = b0;
        }
        ++k;
    }
    __device__ __forceinline__ void finish() {}
};

// The four rows of an env through LDS (A == C::AM == 4, D % 4 == 0, the
// compile-time column layout): each lane buffers 16 consecutive columns of its
// own row; at every 16-column boundary the env's four lanes swap them through
// LDS so that each store instruction writes one 64-B run of ONE row per env
// (lane i: floats 4i..4i+3 of the run) instead of 16 B of every lane's row --
// the 16-B pieces made the L2 write back partial 64-B halves (k_post_lanes
// WRITE_SIZE 295 vs 196 MB per 2v2 step, r04i vs r04e).  With the layout known
// at compile time every buffer slot and flush point is a constant (the same
// sink over run-time counts doubled the kernel's code).  stg: the env slot's
// [4 rows][4 float4] in LDS; every lane of the env calls it (on: store).
struct QuadRow {
    float* env;   // obs row 0 of the env
    float4* stg;  // LDS staging of the slot
    int i, D;     // this lane's row; the row length
    bool on;      // the env's rows are stored
    int k = 0;    // next column
    float b[16];
    __device__ __forceinline__ void put(float v)
    {
        const int s = k & 15;
        // (constant indices only: b stays in registers; s is a constant here)
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (s == q) b[q] = v;
        if (s == 15) flush(k - 15, 16);
        ++k;
    }
    __device__ __forceinline__ void finish()
    {
        if ((k & 15) != 0) flush(k - (k & 15), k & 15);
    }
    __device__ __forceinline__ void flush(int g0, int n)
    {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * q < n) stg[i * 4 + q] = make_float4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
        // (one wave: its LDS writes precede its reads, the previous group's
        // reads precede these writes)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 v = stg[r * 4 + i];
            if (on && 4 * i < n) *reinterpret_cast<float4*>(env + (int64_t)r * D + g0 + 4 * i) = v;
        }
    }
};

// bf16 rows for mas_step_x (the PPO consumer's policy input): the same
// columns, each rounded to bf16 (round to nearest even: the conversion the
// policy kernels apply to fp32 obs rows, so the policy sees the same bits).
__device__ __forceinline__ uint32_t bf16x2(float a, float b)
{
    const __bf16 x = (__bf16)a, y = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// QuadRow into bf16 rows (row stride ld elements, ld % 4 == 0, 8-B aligned
// base): the same LDS swap, each store writes 4 columns (8 B) of one row,
// a 32-B run of one row per env and instruction
struct QuadRowX {
    uint16_t* env;  // x row 0 of the env
    float4* stg;
    int i;
    int64_t ld;
    bool on;
    int k = 0;
    float b[16];
    __device__ __forceinline__ void put(float v)
    {
        const int s = k & 15;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (s == q) b[q] = v;
        if (s == 15) flush(k - 15, 16);
        ++k;
    }
    __device__ __forceinline__ void finish()
    {
        if ((k & 15) != 0) flush(k - (k & 15), k & 15);
    }
    __device__ __forceinline__ void flush(int g0, int n)
    {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * q < n) stg[i * 4 + q] = make_float4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 v = stg[r * 4 + i];
            if (on && 4 * i < n)
                *reinterpret_cast<uint2*>(env + (int64_t)r * ld + g0 + 4 * i) = make_uint2(bf16x2(v.x, v.y), bf16x2(v.z, v.w));
        }
    }
};

// SeqRow into one bf16 row: 8-B stores of 4 columns (ld % 4 == 0, 8-B
// aligned base), the last partial group column by column
struct SeqRowX {
    uint16_t* p;
    int k = 0;
    float b0 = 0.0f, b1 = 0.0f, b2 = 0.0f, b3 = 0.0f;
    __device__ __forceinline__ void put(float v)
    {
        const int s = k & 3;
        if (s == 0) b0 = v;
        else if (s == 1) b1 = v;
        else if (s == 2) b2 = v;
        else b3 = v;
        if (s == 3) *reinterpret_cast<uint2*>(p + (k - 3)) = make_uint2(bf16x2(b0, b1), bf16x2(b2, b3));
        ++k;
    }
    __device__ __forceinline__ void finish()
    {
        const int s = k & 3, g = k - s;
        const float v[3] = {b0, b1, b2};
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (q < s) p[g + q] = (uint16_t)(bf16x2(v[q], 0.0f) & 0xffffu);
    }
};

// EX: the config fills the class exactly (A, B, H at the class maxima, no
// lasers) with Teams = P.teams: every count is a compile-time constant, so
// the whole row unrolls and each column's index -- the sink's buffer slot and
// store offset -- is known at compile time (no per-column branch tree).
// Otherwise the counts come from P.  Either way every lane makes the same
// puts in the same order (the other agents by rank), so the column index is
// wave-uniform.
template <class C, bool EX, bool TEAMS, class Sink>
__device__ __forceinline__ void write_obs_row_seq(const PostV<C>& V, const Params& P, uint32_t alive_m, int i,
                                                  int lastmeta, float lhx, float lhy, Sink& o)
{
    using PV = PostV<C>;
    const int A = EX ? C::AM : P.A;
    const int B = EX ? C::BM : P.B;
    const int H = EX ? C::HM : P.H;
    const int NL = EX ? 0 : P.n_lasers;
    const bool teams = EX ? TEAMS : (P.teams != 0);
    const bool alive = bit(alive_m, i);
    const int pp = __popc(alive_m & ((1u << i) - 1u));  // post-despawn list position (quirk D1)
    auto agent_row = [&](int k) {
        const bool ak = bit(alive_m, k);
        o.put((float)k);
        if (teams) o.put((float)team_of(P, k));
        o.put(ak ? V.ag(6, k) : 0.0f);
#pragma unroll
        for (int f = 0; f < 6; ++f) o.put(ak ? V.ag(f, k) : 0.0f);
    };
    auto seen_mask = [&](bool present, int body) -> float {
        if (P.omniscient) return present ? 0.0f : 1.0f;
        return (present && alive && ((V.sn(body) >> pp) & 1u)) ? 0.0f : 1.0f;
    };
    // agent
    agent_row(i);
    if (B > 0) {
        // box_items, box_items_mask
        const int ni = V.nbi();
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const bool present = b < ni;
            const float hx = V.ihx(b), hy = V.ihy(b);
            const int rot = bi_rot(V.imeta(b));
            const V2 ip = V.ip(b);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const V2 cv = box_corner(hx, hy, rot + v);
                o.put(present ? cv.x : 0.0f);
                o.put(present ? cv.y : 0.0f);
            }
            o.put(present ? ip.x : 0.0f);
            o.put(present ? ip.y : 0.0f);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) o.put(seen_mask(b < ni, BIdx<C>::bitem + b));
        // box_slot, box_slot_mask
        const bool isbox = it_kind(lastmeta) == kItemBox;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const V2 cv = box_corner(lhx, lhy, it_rot(lastmeta) + v);
            o.put(isbox ? cv.x : 0.0f);
            o.put(isbox ? cv.y : 0.0f);
        }
        o.put(isbox ? 0.0f : 1.0f);
        // boxes, boxes_mask
        const int nb = V.nbox();
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const bool present = b < nb;
            const int meta = V.bmeta(b);
            const Poly4 poly = box_poly(V.bhx(b), V.bhy(b), box_rot(meta), box_copied(meta));
            const V2 bp = V.bp(b);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                o.put(present ? poly.v[v].x : 0.0f);
                o.put(present ? poly.v[v].y : 0.0f);
            }
            o.put(present ? bp.x : 0.0f);
            o.put(present ? bp.y : 0.0f);
            o.put(0.0f);  // box bodies always have angle 0
        }
#pragma unroll
        for (int b = 0; b < B; ++b) o.put(seen_mask(b < nb, BIdx<C>::box + b));
    }
    if (H > 0) {
        // heal_slot, heal_slot_mask
        const bool isheal = it_kind(lastmeta) == kItemHeal;
        o.put(isheal ? (float)P.healing : 0.0f);
        o.put(isheal ? 0.0f : 1.0f);
        // heals, heals_mask
        const int nh = V.nheal();
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const bool present = h < nh;
            const V2 hp = V.hp(h);
            o.put(present ? hp.x : 0.0f);
            o.put(present ? hp.y : 0.0f);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) o.put(seen_mask(h < nh, BIdx<C>::heal + h));
    }
    // lidars: zeros here; k_lidar writes the columns afterwards
    for (int k = 0; k < NL; ++k) o.put(0.0f);
    // others, others_mask: the other agents by rank (agent k skips i), the
    // seen list at the post-despawn list index
#pragma unroll
    for (int r = 0; r + 1 < A; ++r) agent_row(r < i ? r : r + 1);
#pragma unroll
    for (int r = 0; r + 1 < A; ++r) {
        const int k = r < i ? r : r + 1;
        const bool ak = bit(alive_m, k);
        o.put((alive && ak && ((V.sn(BIdx<C>::agent + k) >> pp) & 1u)) ? 0.0f : 1.0f);
    }
    // zone
    const int phase = (int)V.zw(PV::kZPhase);
    o.put(__uint_as_float(V.zw(PV::kZPx)));
    o.put(__uint_as_float(V.zw(PV::kZPy)));
    o.put(__uint_as_float(V.zw(PV::kZRad)));
    float z3 = 0.0f, z4 = 0.0f, z5 = 0.0f;
    if (phase < P.zone_phases - 1) {
        const V2 zn = V.zc(phase + 1);
        z3 = zn.x;
        z4 = zn.y;
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k == phase + 1) z5 = opq(P.zradf[k]);
    }
    o.put(z3);
    o.put(z4);
    o.put(z5);
    o.finish();
}

// Cameras._update_seen (simulation.py:336-354) on agent lanes: camera i of
// slot j.  slot_on: slot j takes part (its leader zeroes its seen rows and
// records the alive mask the rays see); cam_on: this lane's agent is a live
// camera of such a slot, at pos / angle ang; alive_m: the slot's alive mask.
// Every candidate of the cone test goes into one wave-wide list, and the line
// of sight rays are dealt over the 64 lanes (update_seen_dealt, mas_step.h:
// the same candidates, rays and first-hit test).  Every lane calls it.
template <class C>
__device__ __forceinline__ void cameras_v(PostLds<C>& lds, const PostV<C>& V, const Params& P, bool slot_on,
                                          bool cam_on, uint32_t alive_m, V2 pos, float ang, int i, int j, int lane)
{
    using PV = PostV<C>;
    constexpr int S = kWG / C::AM, AM = C::AM;
    if (i == 0 && slot_on) {
        lds.alivem[j] = alive_m;
#pragma unroll
        for (int k = 0; k < C::NB; ++k) V.sn(k) = 0u;
    }
    uint64_t cand = 0;  // bit per body in the cone
    int p = 0;
    if (cam_on) {
        p = __popc(alive_m & ((1u << i) - 1u));
        const Rot q = rot_of(ang);
        const int nb = V.nbox(), ni = V.nbi(), nh = V.nheal();
#pragma unroll
        for (int b = 0; b < C::BM; ++b) {
            if (b < nb && poly_test_point(P.cone, pos, q, V.bp(b))) cand |= 1ull << (BIdx<C>::box + b);
            if (b < ni && poly_test_point(P.cone, pos, q, V.ip(b))) cand |= 1ull << (BIdx<C>::bitem + b);
        }
#pragma unroll
        for (int h = 0; h < C::HM; ++h)
            if (h < nh && poly_test_point(P.cone, pos, q, V.hp(h))) cand |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
        for (int w = 0; w < kNumWalls; ++w)
            if (poly_test_point(P.cone, pos, q, P.wall_pos[w])) cand |= 1ull << (BIdx<C>::wall + w);
#pragma unroll
        for (int k = 0; k < AM; ++k)
            if (k != i && bit(alive_m, k) && poly_test_point(P.cone, pos, q, V.agent(k)))
                cand |= 1ull << (BIdx<C>::agent + k);
    }
    // the wave's rays dealt over its lanes (update_seen_cam)
    const int np = __popcll(cand);
    int incl = np;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int total = __shfl(incl, 63, 64);
    int at = incl - np;
    while (cand) {
        const int body = __builtin_ctzll(cand);
        cand &= cand - 1;
        lds.u.cam.list[at++] = (uint16_t)((p << 12) | (lane << 6) | body);
    }
    wave_lds_sync();  // the list, the agent table and the zeroed seen rows are visible
    const float eps1 = (float)(1.0 + 1e-6);
    for (int t = lane; t < total; t += 64) {
        const uint32_t en = lds.u.cam.list[t];
        const int body = (int)(en & 63u), o = (int)((en >> 6) & 63u), pc = (int)(en >> 12);
        const int so = o / AM, co = o - so * AM;  // the owner's slot and camera
        const PV Vo{&lds, so};
        const V2 opos = Vo.agent(co);
        V2 oc;
        if (body < BIdx<C>::bitem) oc = Vo.bp(body);
        else if (body < BIdx<C>::heal) oc = Vo.ip(body - BIdx<C>::bitem);
        else if (body < BIdx<C>::wall) oc = Vo.hp(body - BIdx<C>::heal);
        else if (body < BIdx<C>::agent) {
            const int w = body - BIdx<C>::wall;
            oc = opq(P.wall_pos[0]);
#pragma unroll
            for (int q2 = 1; q2 < kNumWalls; ++q2)
                if (q2 == w) oc = opq(P.wall_pos[q2]);
        } else oc = Vo.agent(body - BIdx<C>::agent);
        const V2 d = sub(oc, opos);
        const V2 end = add(opos, scl(eps1, d));
        if (ray_cast_pv(P, Vo, lds.alivem[so], opos, end) == body) atomicOr(&lds.seen[body * S + so], 1u << pc);
    }
    wave_lds_sync();  // the seen rows are complete
}

// BaseEnv.reset -> Simulation.reset (masurvival_env.py:59-74; env_reset,
// mas_step.h, the same draws in the same order) of slot j on its leader lane,
// into the slot's LDS groups: SpawnGrid.reset's shuffle of the grid cells
// (semantics.py:71-74, 987-992), RandomizeBoxShapes (:107-120) and the
// spawns (boxes, heals, agents from the end of the permutation), empty box
// items, the SafeZone's post_reset (:739-756).  The agent table gets the
// agents' spawn poses and full health.  R: the env's PCG64 stream; perm: the
// [grid cells][S] byte scratch.  Fisher-Yates from the top finalises cell i
// at step i and later steps touch only lower cells, so the swaps run only
// for the cells the spawns take (the draws of every step are still made).
template <class C>
__device__ __forceinline__ void reset_env_v(const PostV<C>& V, const Params& P, EnvL<C>& R, uint8_t* perm)
{
    using PV = PostV<C>;
    constexpr int S = PV::S;
    const int A = P.A, H = P.H, B = P.B;
    const int g = P.grid_size, n = g * g;
    auto pm = [&](int k) -> uint8_t& { return perm[k * S + V.j]; };
    const int used = A + H + B;  // <= n (mas_create)
    for (int k = 0; k < n; ++k) pm(k) = (uint8_t)k;
    for (int i = n - 1; i >= 1; --i) {
        const int jj = (int)pcg_interval32(R, (uint32_t)i);
        if (i >= n - used) {
            const uint8_t t = pm(i);
            pm(i) = pm(jj);
            pm(jj) = t;
        }
    }
    int top = n;
    auto cell = [&](int k) -> V2 {
        const int ii = k % g, jj = k / g;
        double ci = (double)ii / g + 0.5 / g;
        double cj = (double)jj / g + 0.5 / g;
        ci = P.floor_size * ci - P.floor_size / 2.0;
        cj = P.floor_size * cj - P.floor_size / 2.0;
        return mk((float)ci, (float)cj);
    };
    // boxes: sizes (RandomizeBoxShapes draws), then the spawn cells
    V.bw(0) = (uint32_t)B;  // (<= C::BM, mas_create)
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        float hx = 0.0f, hy = 0.0f;
        if (b < B) {
            hx = P.box_hx;
            hy = P.box_hy;
            if (P.randomized) {
                double wv = P.avg_w + P.std_w * pcg_normal(R);
                wv = P.min_w > wv ? P.min_w : wv;
                double hv = P.avg_h + P.std_h * pcg_normal(R);
                hv = P.min_h > hv ? P.min_h : hv;
                hx = (float)(wv / 2.0);
                hy = (float)(hv / 2.0);
            }
        }
        V.bw(3 + 6 * b) = __float_as_uint(hx);
        V.bw(4 + 6 * b) = __float_as_uint(hy);
    }
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        const V2 c = b < B ? cell(pm(--top)) : mk(0.0f, 0.0f);
        V.bw(1 + 6 * b) = __float_as_uint(c.x);
        V.bw(2 + 6 * b) = __float_as_uint(c.y);
        V.bw(5 + 6 * b) = (uint32_t)mk_boxmeta(0, 0, b < B ? 1 : 0, kCauseNone, kCauseNone);
        V.bw(6 + 6 * b) = (uint32_t)(b < B ? P.box_health : 0);
    }
    // box items: none
    V.iw(0) = 0u;
#pragma unroll
    for (int q = 1; q < Lay<C>::kItemW; ++q) V.iw(q) = 0u;
    // heals
    V.hw(0) = (uint32_t)H;
#pragma unroll
    for (int h = 0; h < C::HM; ++h) {
        const V2 c = h < H ? cell(pm(--top)) : mk(0.0f, 0.0f);
        V.hw(1 + 2 * h) = __float_as_uint(c.x);
        V.hw(2 + 2 * h) = __float_as_uint(c.y);
    }
    // agents: the agent table (pose, velocity 0, health)
#pragma unroll
    for (int k = 0; k < C::AM; ++k) {
        const V2 c = k < A ? cell(pm(--top)) : mk(0.0f, 0.0f);
        V.ag(0, k) = c.x;
        V.ag(1, k) = c.y;
#pragma unroll
        for (int f = 2; f < 6; ++f) V.ag(f, k) = 0.0f;
        V.ag(6, k) = k < A ? (float)P.agent_health : 0.0f;
    }
    // SafeZone.post_reset
    V2 zc[kMaxPhases];
#pragma unroll
    for (int k = 0; k < kMaxPhases; ++k) zc[k] = mk(0.0f, 0.0f);
    const int nr = P.zone_nr;
    if (P.zone_random) {
        for (int k = nr; k >= 0; --k) {
            double r = 0.0;
#pragma unroll
            for (int q = 0; q < kMaxPhases; ++q)
                if (q == k) r = opq(P.zrad[q]);
            const double Lz = P.floor_size - 2.0 * r;
            const double cx = (pcg_random(R) * Lz) - Lz / 2.0;
            const double cy = (pcg_random(R) * Lz) - Lz / 2.0;
            put(zc, k, mk((float)cx, (float)cy));
        }
    } else {
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k < nr) zc[k] = mk(P.zfix[k][0], P.zfix[k][1]);
    }
#pragma unroll
    for (int k = 0; k < kMaxPhases; ++k) {
        V.zw(2 * k) = __float_as_uint(zc[k].x);
        V.zw(2 * k + 1) = __float_as_uint(zc[k].y);
    }
    V.zw(PV::kZPhase) = 0u;
    V.zw(PV::kZCd) = (uint32_t)P.zone_cooldown;
    V.zw(PV::kZSh) = 0u;
    V.zw(PV::kZEnd) = 0u;
    V.zw(PV::kZPx) = __float_as_uint(zc[0].x);
    V.zw(PV::kZPy) = __float_as_uint(zc[0].y);
    V.zw(PV::kZRad) = __float_as_uint(P.zradf[0]);
}

// The auto-reset runs inside k_post_lanes (reset_in_post) when the spawn
// grid's permutation scratch fits the LDS union of its slots
template <class C>
constexpr int kPostUnionBytes = (int)sizeof(((PostLds<C>*)nullptr)->u);
template <class C>
inline bool reset_fits_post(const Params& P)
{
    return P.grid_size * P.grid_size * (kWG / C::AM) <= kPostUnionBytes<C>;
}

// The post-physics phases of one step on agent lanes (see the file comment),
// over env selection M (kAllEnvs / kMainEnvs on the caller's stream, the
// slow list's kGenEnvs on the side stream).  With the auto-reset (ar) the
// done envs are reset in place at the end (P.reset_in_post: their state and
// obs rows are the reset env's), or appended to the selection's reset list
// for the k_obs reset launch over that list (launch_post).
// waves per SIMD the register budget targets (3: <= 168 VGPRs)
#ifndef MAS_POST_OCC
#define MAS_POST_OCC 3
#endif
// test builds: MAS_POST_VGPR=n caps the kernel at n VGPRs for every class
// (the xl / ffa classes are LDS-bound and otherwise take ~230), to run the
// parity suites on a heavily spilling schedule
#ifdef MAS_POST_VGPR
#define MAS_POST_BOUNDS \
    __launch_bounds__(kWG, MAS_POST_OCC) __attribute__((amdgpu_waves_per_eu(512 / MAS_POST_VGPR, 512 / MAS_POST_VGPR)))
#else
#define MAS_POST_BOUNDS __launch_bounds__(kWG, MAS_POST_OCC)
#endif
template <class C, int M>
__global__ MAS_POST_BOUNDS void k_post_lanes(Params P, uint32_t* __restrict__ state, int64_t N,
                                                       float* __restrict__ obs, float* __restrict__ rew,
                                                       uint8_t* __restrict__ done, int ar)
{
    using LY = Lay<C>;
    using PV = PostV<C>;
    constexpr int S = kWG / C::AM, AM = C::AM;
    static_assert(kWG % AM == 0 && (AM & (AM - 1)) == 0, "agent lane groups must tile a wave");
    static_assert(C::NB <= 64 && AM <= 8, "16-bit camera list entries, 64-bit body masks");
    __shared__ PostLds<C> lds;
    MAS_PROF(P, -1);
    retire_phys_count<M>(P);
    const int lane = (int)threadIdx.x;
    const int j = lane / AM, i = lane - j * AM;
    const int A = P.A;
    // the env of slot j (lanes past the last env, or of an env the other
    // stream owns, stay for the wave's collectives and store nothing)
    // (a list's entries in launch order; the envs in the XCD-aware block order)
    const int64_t k0 = (M == kGenEnvs ? (int64_t)blockIdx.x : xcd_block()) * S;
    bool valid;
    int64_t e;
    if (M == kGenEnvs) {
        // the list's entries k0 .. k0 + S - 1 (a sharded list: list_pos)
        const ListPos lp = list_pos(P, N, k0, k0 + j);
        if (!lp.any) return;  // the whole workgroup (one wave)
        valid = lp.valid;
        e = valid ? lp.e : (int64_t)P.phys_list[0];
    } else {
        valid = k0 + j < N;
        e = valid ? k0 + j : N - 1;
    }
    if (valid && other_stream<M>(P, e)) valid = false;
    if (i == 0) lds.eidx[j] = e;
    wave_lds_sync();
    const PV V{&lds, j};
    // ---- state: the env-shared groups into LDS, this lane's agent into registers
    // every group's loads and this lane's agent loads first, then the LDS
    // writes (SlotRows)
    SlotRows<S, LY::kBoxW> rbox;
    SlotRows<S, LY::kItemW> ritem;
    SlotRows<S, LY::kHealW> rheal;
    SlotRows<S, LY::kZoneW> rzone;
    // (all in flight at once only when the registers fit the 3-wave budget)
    constexpr bool kBatch = decltype(rbox)::T + decltype(ritem)::T + decltype(rheal)::T + decltype(rzone)::T <= 16;
    if (kBatch) {
        rbox.load(state, N, lds.eidx, LY::box);
        ritem.load(state, N, lds.eidx, LY::item);
        rheal.load(state, N, lds.eidx, LY::heal);
        rzone.load(state, N, lds.eidx, LY::zone);
    } else {
        decltype(rbox)::copy(lds.box, state, N, lds.eidx, LY::box);
        decltype(ritem)::copy(lds.item, state, N, lds.eidx, LY::item);
        decltype(rheal)::copy(lds.heal, state, N, lds.eidx, LY::heal);
        decltype(rzone)::copy(lds.zone, state, N, lds.eidx, LY::zone);
    }
    AgentL<C> g;
    {
        float d[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) d[q] = __uint_as_float(state[state_index(7 * i + q, e, N)]);
        g.c = mk(d[0], d[1]);
        g.a = d[2];
        g.v = mk(d[3], d[4]);
        g.w = d[5];
        g.sleep = 0.0f;  // (not read here)
        const int wr = LY::rule + i * LY::kRuleA;
        g.health = (int)state[state_index(wr, e, N)];
        g.cause = (int)state[state_index(wr + 1, e, N)];
        g.cooldown = (int)state[state_index(wr + 2, e, N)];
        g.inv_n = (int)state[state_index(wr + 3, e, N)];
#pragma unroll
        for (int k = 0; k < C::SM; ++k) {
            g.inv_meta[k] = (int)state[state_index(wr + 4 + 3 * k, e, N)];
            g.inv_hx[k] = __uint_as_float(state[state_index(wr + 5 + 3 * k, e, N)]);
            g.inv_hy[k] = __uint_as_float(state[state_index(wr + 6 + 3 * k, e, N)]);
        }
    }
    uint32_t alive_m = state[state_index(LY::alive, e, N)];
    uint32_t awake_m = state[state_index(LY::awake, e, N)];
    bool alive = bit(alive_m, i);
    if (kBatch) {
        rbox.write(lds.box);
        ritem.write(lds.item);
        rheal.write(lds.heal);
        rzone.write(lds.zone);
    }
    V.ag(0, i) = g.c.x;
    V.ag(1, i) = g.c.y;
    V.ag(2, i) = g.a;
    V.ag(3, i) = g.v.x;
    V.ag(4, i) = g.v.y;
    V.ag(5, i) = g.w;
    wave_lds_sync();  // the wave's LDS groups are loaded (one-wave block)
    MAS_PROF(P, 41);
    // ---- boxes: Health.post_step + despawn (the first post_step hook, dict
    // order: the boxes group before the agents)
    bool bchanged = false;
    if (i == 0) {
        bool any_dead;
        uint32_t kept;
        int nb;
        bchanged = box_health_v(V, P, any_dead, kept, nb, state, N, e, valid);
        lds.misc[j] = kept | ((uint32_t)nb << 24) | (any_dead ? (1u << 23) : 0u);
    }
    wave_lds_sync();
    {
        // the agent-static contact rows follow the boxes (each agent's row on
        // its own lane: the rows are independent)
        const uint32_t mj = lds.misc[j];
        if (valid && (mj & (1u << 23))) {
            const Cont<C, ContGlbStore<C>> KG{{state, N, e, P.w_cont}};
            compact_cont_row<C>(KG, i, mj & 0x7fffffu, (int)(mj >> 24));
        }
    }
    // ---- Cameras.post_step (simulation.py:314-354): camera i of slot j
    cameras_v<C>(lds, V, P, true, valid && alive, alive_m, g.c, g.a, i, j, lane);
    MAS_PROF(P, 42);
    // ---------------- agents post_step (step_post, mas_step.h) ----------------
    uint32_t dirty = kGZone | kGStat;
    // Health.post_step -> despawn dead (id order): TrackDeaths, IndexBodies,
    // DeathDrop (semantics.py:387-396), Inventory, Health.pre_despawn -> TrackKills
    const bool dies = valid && alive && g.health <= 0;
    const uint32_t died = env_ballot<C>(dies);
    int kill_cause = kCauseNone;
    if (__any(died != 0u)) {
        // the dying agents' positions and inventories for the leader's DeathDrop
        constexpr int DW = PostLds<C>::kDropW;
        uint32_t* dr = lds.u.dd.drop;
        auto dref = [&](int f, int k) -> uint32_t& { return dr[(f * AM + k) * S + j]; };
        if (dies) {
            dref(0, i) = __float_as_uint(g.c.x);
            dref(1, i) = __float_as_uint(g.c.y);
            dref(2, i) = (uint32_t)g.inv_n;
#pragma unroll
            for (int k = 0; k < C::SM; ++k) {
                dref(3 + 3 * k, i) = (uint32_t)g.inv_meta[k];
                dref(4 + 3 * k, i) = __float_as_uint(g.inv_hx[k]);
                dref(5 + 3 * k, i) = __float_as_uint(g.inv_hy[k]);
            }
        }
        (void)DW;
        wave_lds_sync();
        if (i == 0 && died) {
            // numpy Generator(PCG64) of the env: angles = 2*pi*rng.random(total),
            // popped from the end per dying body (bodies in id order, items in
            // slot order)
            EnvL<C> R;
            {
                Loader ld{state, N, e, 0};
                visit_state(R, ld, kGRng);
            }
            int total = 0;
            for (int k = 0; k < AM; ++k)
                if (bit(died, k)) total += (int)dref(2, k);
            double* ang = lds.u.dd.ang;
            for (int k = 0; k < total; ++k) ang[k * S + j] = 6.283185307179586 * pcg_random(R);
            int top = total;
            for (int k = 0; k < AM; ++k) {
                if (!bit(died, k)) continue;
                const V2 ck = mk(__uint_as_float(dref(0, k)), __uint_as_float(dref(1, k)));
                const int n = (int)dref(2, k);
                for (int q = 0; q < n; ++q) {
                    --top;
                    const float a = (float)ang[top * S + j];
                    const V2 off = from_polar(P.dd_r, a);
                    const V2 pos = add(ck, off);
                    const int meta = (int)dref(3 + 3 * q, k);
                    if (it_kind(meta) == kItemHeal) {
                        const int nh = V.nheal();
                        if (nh < C::HM) {
                            V.hw(1 + 2 * nh) = __float_as_uint(pos.x);
                            V.hw(2 + 2 * nh) = __float_as_uint(pos.y);
                            V.hw(0) = (uint32_t)(nh + 1);
                        }
                    } else {
                        const int ni = V.nbi();
                        if (ni < C::BM) {
                            V.iw(1 + 5 * ni) = __float_as_uint(pos.x);
                            V.iw(2 + 5 * ni) = __float_as_uint(pos.y);
                            V.iw(3 + 5 * ni) = dref(4 + 3 * q, k);
                            V.iw(4 + 5 * ni) = dref(5 + 3 * q, k);
                            V.iw(5 + 5 * ni) = (uint32_t)mk_bimeta(it_rot(meta), it_copied(meta), it_owner(meta));
                            V.iw(0) = (uint32_t)(ni + 1);
                        }
                    }
                }
            }
            if (valid) {
                Storer st{state, N, e, 0};
                visit_state(R, st, kGRng);
            }
            // the agent-agent touching word: the pairs of the dead agents
            const Cont<C, ContGlbStore<C>> KG{{state, N, e, P.w_cont}};
            uint32_t aat = KG.aat();
            for (int k = 0; k < AM; ++k) {
                if (!bit(died, k)) continue;
                for (int m = 0; m < AM; ++m) {
                    if (m == k) continue;
                    const int pi = m < k ? aa_index<C::AM>(m, k) : aa_index<C::AM>(k, m);
                    aat &= ~(1u << pi);
                    if (valid) {
                        KG.set_aani(pi, 0.0f);
                        KG.set_aati(pi, 0.0f);
                    }
                }
            }
            if (valid) KG.set_aat(aat);
        }
        wave_lds_sync();
        if (dies) {
            kill_cause = g.cause;
            // the dead agent's contact rows (its own lane)
            const Cont<C, ContGlbStore<C>> KG{{state, N, e, P.w_cont}};
            KG.set_ast(i, 0u);
#pragma unroll
            for (int s = 0; s < C::NS; ++s) {
                KG.set_asni(i, s, 0.0f);
                KG.set_asti(i, s, 0.0f);
            }
            g.inv_n = 0;
        }
        alive_m &= ~died;
        awake_m &= ~died;
        alive = bit(alive_m, i);
        if (died) dirty |= kGDyn | kGRule | kGItem | kGHeal | kGSeen | kGRng;
    }
    // AutoPickup.post_step (semantics.py:278-283): every agent's list first,
    // then the takes in agent order (each agent's own inventory)
    {
        uint32_t lb = 0, lh = 0;
        if (alive) {
            const int ni = V.nbi(), nh = V.nheal();
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < ni && circle_test_point(P.pickup_r, g.c, V.ip(b))) lb |= 1u << b;
#pragma unroll
            for (int h = 0; h < C::HM; ++h)
                if (h < nh && circle_test_point(P.pickup_r, g.c, V.hp(h))) lh |= 1u << h;
        }
        uint32_t takenb = 0, takenh = 0;
        while (lb) {
            const int b = __builtin_ctz(lb);
            lb &= lb - 1;
            const int im = V.imeta(b);
            if (1 + g.inv_n <= P.slots) {
                own_take(g, P, mk_itmeta(kItemBox, bi_rot(im), bi_copied(im), bi_owner(im)), V.ihx(b), V.ihy(b));
                takenb |= 1u << b;
            }
        }
        while (lh) {
            const int h = __builtin_ctz(lh);
            lh &= lh - 1;
            if (1 + g.inv_n <= P.slots) {
                own_take(g, P, mk_itmeta(kItemHeal, 0, 0, kCauseNone), 0.0f, 0.0f);
                takenh |= 1u << h;
            }
        }
#pragma unroll
        for (int o = 1; o < AM; o <<= 1) {
            takenb |= (uint32_t)__shfl_xor((int)takenb, o, 64);
            takenh |= (uint32_t)__shfl_xor((int)takenh, o, 64);
        }
        if (takenb | takenh) dirty |= kGRule | kGItem | kGHeal | kGSeen;
        wave_lds_sync();  // every lane's pickup reads are done
        if (i == 0 && takenb) {
            const int ni = V.nbi();
            int wi = 0;
            for (int b = 0; b < ni; ++b) {
                if (bit(takenb, b)) continue;
                if (wi != b) {
#pragma unroll
                    for (int q = 1; q <= 5; ++q) V.iw(q + 5 * wi) = V.iw(q + 5 * b);
                }
                V.sn(BIdx<C>::bitem + wi) = V.sn(BIdx<C>::bitem + b);
                ++wi;
            }
            V.iw(0) = (uint32_t)wi;
        }
        if (i == 0 && takenh) {
            const int nh = V.nheal();
            int wi = 0;
            for (int h = 0; h < nh; ++h) {
                if (bit(takenh, h)) continue;
                if (wi != h) {
                    V.hw(1 + 2 * wi) = V.hw(1 + 2 * h);
                    V.hw(2 + 2 * wi) = V.hw(2 + 2 * h);
                }
                V.sn(BIdx<C>::heal + wi) = V.sn(BIdx<C>::heal + h);
                ++wi;
            }
            V.hw(0) = (uint32_t)wi;
        }
    }
    // SafeZone.post_step (semantics.py:758-768): damage outliers, then tick
    if (alive) {
        const V2 zp = mk(__uint_as_float(V.zw(PV::kZPx)), __uint_as_float(V.zw(PV::kZPy)));
        const float zr = __uint_as_float(V.zw(PV::kZRad));
        if (V.zw(PV::kZEnd) || !circle_test_point(zr, zp, g.c)) {
            own_damage(g, alive, P, i, -P.zone_damage, kCauseZone);
            dirty |= kGRule;
        }
    }
    wave_lds_sync();  // every lane has read the pre-tick zone
    if (i == 0) zone_tick_v(V, P);
    // ---------------- compute_rewards (masurvival_env.py:757-803) ----------------
    float r = 0.0f;
    int my_kills = 0, tkills0 = 0, tkills1 = 0;
    if (!P.teams) {
        int first_dead = -1;
        for (int k = AM - 1; k >= 0; --k)
            if (k < A && !bit(alive_m, k)) first_dead = k;
        r += bit(alive_m, i) ? P.r_alive : P.r_dead;
#pragma unroll
        for (int k = 0; k < AM; ++k) {
            const int c = env_bcast<C>(kill_cause, k);
            if (!bit(died, k)) continue;
            int idx = -1;
            if (c >= 0 && c < AM && bit(alive_m, c)) idx = c;
            else if (c == kCauseNone && first_dead >= 0) idx = first_dead;  // None in indexed_agents
            if (idx == i) {
                r += P.r_kill;
                my_kills += 1;
            }
        }
        if (bit(died, i)) r += P.r_death;
    } else {
        bool talive0 = false, talive1 = false;
        for (int k = 0; k < A; ++k)
            if (bit(alive_m, k)) (team_of(P, k) == 0 ? talive0 : talive1) = true;
        const int ti = team_of(P, i);
        if (i < A) r += (ti == 0 ? talive0 : talive1) ? P.r_alive : P.r_dead;
#pragma unroll
        for (int k = 0; k < AM; ++k) {
            const int c = env_bcast<C>(kill_cause, k);
            if (!bit(died, k)) continue;
            if (c != kCauseBadge && c != kCauseBadge + 1) continue;
            const int t = c - kCauseBadge;
            if (i < A && ti == t) r += P.r_kill;
            if (t == 0) tkills0 += 1;
            else tkills1 += 1;
        }
#pragma unroll
        for (int k = 0; k < AM; ++k) {
            if (!bit(died, k)) continue;
            if (i < A && ti == team_of(P, k)) r += P.r_death;
        }
    }
    if (valid && i < A) rew[e * A + i] = r;
    // ---------------- is_done (masurvival_env.py:810-831) ----------------
    int n_alive = 0;
    if (P.teams) {
        bool t0 = false, t1 = false;
        for (int k = 0; k < A; ++k) {
            if (!bit(alive_m, k)) continue;
            if (team_of(P, k) == 0) t0 = true;
            else t1 = true;
        }
        n_alive = (t0 ? 1 : 0) + (t1 ? 1 : 0);
    } else {
        n_alive = __popc(alive_m);
    }
    const bool is_done = P.gameover == 1 ? (n_alive <= 1) : (n_alive == 0);
    // ---------------- _update_stats (masurvival_env.py:483-508) ----------------
    {
        const int R = P.teams ? 2 : A;
        float rq[8];
        int kq[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int jq = P.teams ? (q == 0 ? 0 : A / 2) : q;
            rq[q] = env_bcast<C>(r, jq < AM ? jq : 0);
            kq[q] = P.teams ? (q == 0 ? tkills0 : tkills1) : env_bcast<C>(my_kills, q < AM ? q : 0);
        }
        if (valid && i == 0) {
            done[e] = is_done ? 1 : 0;
            float* st = reinterpret_cast<float*>(state);
            // every word's load issued before any add (the per-word
            // read-modify-write under q < R waited out one load latency each);
            // only the 2R + 1 words this step adds to are loaded
            float cur[17];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                cur[q] = q < R ? st[state_index(LY::stat + q, e, N)] : 0.0f;
                cur[8 + q] = q < R ? st[state_index(LY::stat + 8 + q, e, N)] : 0.0f;
            }
            cur[16] = st[state_index(LY::stat + 16, e, N)];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (q >= R) continue;
                st[state_index(LY::stat + q, e, N)] = cur[q] + rq[q];
                st[state_index(LY::stat + 8 + q, e, N)] = cur[8 + q] + (float)kq[q];
            }
            st[state_index(LY::stat + 16, e, N)] = cur[16] + 1.0f;
        }
    }
    MAS_PROF(P, 43);
    // the auto-reset in place (reset_in_post): a done env's post-step groups
    // are not stored, its reset state is (below)
    const bool rs = ar && P.reset_in_post && valid && is_done;
    const bool st_ok = valid && !rs;
    // ---------------- stores: the groups this step changed ----------------
    uint32_t dirty_env = dirty;
#pragma unroll
    for (int o = 1; o < AM; o <<= 1) dirty_env |= (uint32_t)__shfl_xor((int)dirty_env, o, 64);
    if (st_ok) {
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
        if ((dirty_env & kGDyn) && i == 0) {
            state[state_index(LY::alive, e, N)] = alive_m;
            state[state_index(LY::awake, e, N)] = awake_m;
        }
        if (i == 0) {
            // the seen bytes (recomputed every step by the cameras)
#pragma unroll
            for (int w = 0; w < kSeenWords<C>; ++w) {
                uint32_t x = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (4 * w + q < C::NB) x |= (V.sn(4 * w + q) & 0xffu) << (8 * q);
                state[state_index(LY::seen + w, e, N)] = x;
            }
        }
    }
    {
        const uint32_t sv = slot_mask<C>(st_ok);
        const uint32_t sb = slot_mask<C>(st_ok && bchanged);
        const uint32_t si = slot_mask<C>(st_ok && (dirty_env & kGItem));
        const uint32_t sh = slot_mask<C>(st_ok && (dirty_env & kGHeal));
        if (sb) slot_store<S, LY::kBoxW>(lds.box, state, N, lds.eidx, LY::box, sb);
        if (si) slot_store<S, LY::kItemW>(lds.item, state, N, lds.eidx, LY::item, si);
        if (sh) slot_store<S, LY::kHealW>(lds.heal, state, N, lds.eidx, LY::heal, sh);
        // the zone's mutable words only (phase, timers, endgame, the current
        // zone): the phase centres change only at a reset, whose path below
        // stores the whole group (saves 16 of 23 words per env and step)
        constexpr int kZM = PV::kZPhase;
        static_assert(LY::kZoneW - kZM == 7, "the zone's mutable words follow the centres");
        if (sv) slot_store<S, LY::kZoneW - kZM>(lds.zone + kZM * S, state, N, lds.eidx, LY::zone + kZM, sv);
    }
    // ---------------- auto-reset: the done envs ----------------
    if (ar && P.reset_in_post) {
        if (__any(rs)) {
            // BaseEnv.reset (masurvival_env.py:59-74) of the done envs in
            // place: the same state and obs rows as env_reset + update_seen
            // of the reset launch (k_obs), with the groups built in this
            // kernel's LDS.  The reset overwrites words this kernel stored for
            // the env from other lanes (DeathDrop, the contact rows): those
            // stores complete first (vmcnt counts stores on gfx9)
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            // (this block's state addresses from an opaque base: merged with
            // the kernel's other addresses they stayed live across it and spilled)
            uint32_t* const stR = opq_s(state);
            const int64_t NR = opq_s(N);
            if (rs && i == 0) {
                EnvL<C> R;
                Loader ld{stR, NR, e, 0};
                visit_state(R, ld, kGRng);  // (after the DeathDrop draws above)
                reset_env_v<C>(V, P, R, reinterpret_cast<uint8_t*>(&lds.u));
                Storer sr{stR, NR, e, 0};
                visit_state(R, sr, kGRng);
                P.slow_flag[e] = 0;  // a new episode: no slow-list history
            }
            wave_lds_sync();  // the reset groups and agent table are in LDS
            const uint32_t am_reset = (A >= 32) ? 0xffffffffu : ((1u << A) - 1u);
            if (rs) {
                // this lane's agent: its spawn pose, at rest, full health, empty inventory
                g.c = V.agent(i);
                g.a = 0.0f;
                g.v = mk(0.0f, 0.0f);
                g.w = 0.0f;
                g.sleep = 0.0f;
                g.health = i < A ? P.agent_health : 0;
                g.cause = kCauseNone;
                g.cooldown = 0;
                g.inv_n = 0;
#pragma unroll
                for (int k = 0; k < C::SM; ++k) {
                    g.inv_meta[k] = 0;
                    g.inv_hx[k] = 0.0f;
                    g.inv_hy[k] = 0.0f;
                }
                alive_m = am_reset;
                awake_m = am_reset;
                alive = i < A;
            }
            // Cameras.post_reset: the reset envs' cameras only
            cameras_v<C>(lds, V, P, rs, rs && alive, alive_m, g.c, g.a, i, j, lane);
            // every group but the stats (visit_state order, kResetSt)
            if (rs) {
                const float d[7] = {g.c.x, g.c.y, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int q = 0; q < 7; ++q) stR[state_index(7 * i + q, e, NR)] = __float_as_uint(d[q]);
                const int wr = LY::rule + i * LY::kRuleA;
                stR[state_index(wr, e, NR)] = (uint32_t)g.health;
                stR[state_index(wr + 1, e, NR)] = (uint32_t)g.cause;
                stR[state_index(wr + 2, e, NR)] = 0u;
                stR[state_index(wr + 3, e, NR)] = 0u;
#pragma unroll
                for (int k = 0; k < 3 * C::SM; ++k) stR[state_index(wr + 4 + k, e, NR)] = 0u;
                // the contact memory (a new b2World), dealt over the env's lanes
                for (int k = i; k < Cont<C>::kWords; k += AM) stR[state_index(P.w_cont + k, e, NR)] = 0u;
                if (i == 0) {
                    stR[state_index(LY::alive, e, NR)] = am_reset;
                    stR[state_index(LY::awake, e, NR)] = am_reset;
                    stR[state_index(LY::invdt, e, NR)] = 0u;
#pragma unroll
                    for (int q = 0; q < LY::kItemW; ++q) stR[state_index(LY::pend + q, e, NR)] = 0u;
#pragma unroll
                    for (int w = 0; w < kSeenWords<C>; ++w) {
                        uint32_t x = 0;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (4 * w + q < C::NB) x |= (V.sn(4 * w + q) & 0xffu) << (8 * q);
                        stR[state_index(LY::seen + w, e, NR)] = x;
                    }
                }
            }
            const uint32_t sr = slot_mask<C>(rs);
            slot_store<S, LY::kBoxW>(lds.box, stR, NR, lds.eidx, LY::box, sr);
            slot_store<S, LY::kItemW>(lds.item, stR, NR, lds.eidx, LY::item, sr);
            slot_store<S, LY::kHealW>(lds.heal, stR, NR, lds.eidx, LY::heal, sr);
            slot_store<S, LY::kZoneW>(lds.zone, stR, NR, lds.eidx, LY::zone, sr);
        }
    } else if (ar) {
        const bool mine = valid && i == 0 && is_done;
        const uint64_t m = __ballot(mine);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(P.reset_count, __popcll(m));
            base = __shfl(base, leader, 64);
            if (mine) {
                const int64_t at = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
                if (at < N) P.reset_list[at] = (int)e;
                else atomicAdd(P.list_overflow, 1);
            }
        }
    }
    MAS_PROF(P, 44);
    // ---------------- fetch_observations: rows from LDS ----------------
    V.ag(6, i) = (float)g.health;
    int lastmeta = 0;
    float lhx = 0.0f, lhy = 0.0f;
    if (alive && g.inv_n > 0) {
        lastmeta = sel(g.inv_meta, g.inv_n - 1);
        lhx = sel(g.inv_hx, g.inv_n - 1);
        lhy = sel(g.inv_hy, g.inv_n - 1);
    }
    wave_lds_sync();  // the agent table's healths and every LDS group are final
    const int D = P.D;
    const bool row_on = valid && i < A;
#if MAS_POST_OBS_SEQ
    const uintptr_t ob = reinterpret_cast<uintptr_t>(obs);
    const bool ex = A == C::AM && P.B == C::BM && P.H == C::HM && P.n_lasers == 0;
    if (P.xrow) {
        // mas_step_x: bf16 policy-input rows (x_ld % 4 == 0, 8-B aligned:
        // checked on the host), the same row writer
        if (C::AM == 4 && ex && (D & 3) == 0) {
            QuadRowX o{P.xrow + e * (int64_t)A * P.x_ld, reinterpret_cast<float4*>(&lds.u) + j * 16, i, P.x_ld, valid};
            if (P.teams) write_obs_row_seq<C, true, true>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
            else write_obs_row_seq<C, true, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
        } else if (row_on) {
            SeqRowX o{P.xrow + (e * A + i) * P.x_ld};
            if (ex && P.teams) write_obs_row_seq<C, true, true>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
            else if (ex) write_obs_row_seq<C, true, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
            else write_obs_row_seq<C, false, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
        }
    } else if (C::AM == 4 && ex && (D & 3) == 0 && (ob & 15) == 0) {
        // every lane (the swaps need the env's four), stores by `valid`
        static_assert(C::AM != 4 || sizeof(lds.u) >= sizeof(float4) * 16 * S, "the staging fits the union");
        QuadRow o{obs + e * (int64_t)(A * D), reinterpret_cast<float4*>(&lds.u) + j * 16, i, D, valid};
        if (P.teams) write_obs_row_seq<C, true, true>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
        else write_obs_row_seq<C, true, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
    } else if (row_on) {
        // 16-B stores when the rows are 16-B aligned (D % 4 == 0 and a 16-B
        // aligned buffer), else 8-B / 4-B
        const int vm1 = (D & 3) == 0 && (ob & 15) == 0 ? 3 : ((D & 1) == 0 && (ob & 7) == 0 ? 1 : 0);
        SeqRow o{obs + (e * A + i) * (int64_t)D, vm1};
        if (ex && P.teams) write_obs_row_seq<C, true, true>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
        else if (ex) write_obs_row_seq<C, true, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
        else write_obs_row_seq<C, false, false>(V, P, alive_m, i, lastmeta, lhx, lhy, o);
    }
#else
    const int trow = j * A + i;  // tile row (the wave's rows are consecutive unless kGenEnvs)
    const int64_t r0 = M == kGenEnvs ? 0 : k0 * A;
    const int64_t rr = e * A + i;  // this lane's obs row
    const uint64_t act = __ballot(row_on);
    float* row_tile = lds.u.tile + trow * (kPostObsW + 1);
    for (int c0 = 0; c0 < D; c0 += kPostObsW) {
        if (row_on) {
            WinRowP sink{row_tile, c0};
            write_obs_row_v(V, P, alive_m, i, lastmeta, lhx, lhy, sink);
        }
        wave_lds_sync();  // the tile's rows are in LDS
        // lane = (row parity, column): each store instruction writes two
        // 128-B row segments; 8 rows per lane per chunk, the LDS reads of a
        // chunk issued before its stores
        const int col = lane & (kPostObsW - 1), half = lane / kPostObsW;
        const bool col_ok = c0 + col < D;
        const int nrows = S * A;
        for (int q0 = 0; q0 < nrows; q0 += 16) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int q = q0 + 2 * k + half;
                v[k] = q < nrows ? lds.u.tile[q * (kPostObsW + 1) + col] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int q = q0 + 2 * k + half;
                const int sq = q / A, aq = q - sq * A;  // tile row q: slot q / A, agent q % A
                const bool on = q < nrows && ((act >> (sq * AM + aq)) & 1ull);
                if (on && col_ok) {
                    const int64_t orow = M == kGenEnvs ? lds.eidx[sq] * A + aq : r0 + q;
                    obs[orow * D + c0 + col] = v[k];
                }
            }
        }
        wave_lds_sync();  // the tile's reads are done before the next window's rows
    }
    (void)rr;
#endif
    MAS_PROF(P, 45);
    MAS_PROF_FLUSH(P, M == kGenEnvs ? 5 : 2, 41);
}

}  // namespace mas
