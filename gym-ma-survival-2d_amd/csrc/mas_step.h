// mas_step.h -- MaSurvival rules, observation, reward, done and reset for one
// env in registers (gfx950 HIP).  Reference: masurvival/semantics.py,
// simulation.py, envs/masurvival_env.py (cited per block); order of
// SURVEY.md Appendix A.  Per-thread transient lists (camera candidates,
// seen-by masks, the spawn-grid permutation) live in LDS, [k][64]-interleaved
// so that the 64 lanes of a wave hit 64 distinct banks.
#pragma once

#include "mas_physics.h"

namespace mas {

constexpr int kWG = 64;  // threads (= envs) per workgroup: one wave

// per-thread LDS scratch
template <class C, int S = kWG>  // S: columns ([k][S] interleaved)
struct Scr {
    uint16_t* pairs;  // [C::AM * C::NB][S] (camera, agent, candidate body) of update_seen
    uint32_t* seen;   // [C::NB][S] seen-by camera-position bitmask per body
    uint8_t* perm;    // [256][S] spawn-grid permutation
    int tid;          // this lane's column
    static constexpr int kPairs = C::AM * C::NB;
    __device__ uint16_t& pr(int k) { return pairs[k * S + tid]; }
    __device__ uint32_t& sn(int k) { return seen[k * S + tid]; }
    __device__ uint8_t& pm(int k) { return perm[k * S + tid]; }
};

// unified body index in canonical (dict, then list) order
template <class C> struct BIdx {
    static constexpr int box = 0;
    static constexpr int bitem = C::BM;
    static constexpr int heal = 2 * C::BM;
    static constexpr int wall = 2 * C::BM + C::HM;
    static constexpr int agent = 2 * C::BM + C::HM + kNumWalls;
};

template <class C>
__device__ __forceinline__ V2 body_pos(const EnvL<C>& L, const Params& P, int k)
{
    V2 r = mk(0.0f, 0.0f);
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (k == BIdx<C>::box + b) r = opq(L.bp[b]);
        if (k == BIdx<C>::bitem + b) r = opq(L.ip[b]);
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h)
        if (k == BIdx<C>::heal + h) r = opq(L.hp[h]);
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w)
        if (k == BIdx<C>::wall + w) r = opq(P.wall_pos[w]);
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (k == BIdx<C>::agent + i) r = opq(L.c[i]);
    return r;
}

// simulation.py:431-439 laser_scan + LaserRayCastCallback (:471-484): the
// closest fixture over ALL fixtures (sensors included); returns the body
// index or -1.  A report at fraction 0 ends the traversal (b2DynamicTree).
template <class C>
__device__ __forceinline__ int ray_cast(const EnvL<C>& L, const Params& P, V2 p1, V2 p2, float& maxf)
{
    maxf = 1.0f;
    int hit = -1;
    bool stop = false;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (stop || b >= L.nbox) continue;
        Poly4 poly = box_poly(L.bhx[b], L.bhy[b], box_rot(L.bmeta[b]), box_copied(L.bmeta[b]));
        float f = ray_poly(poly, L.bp[b], kIdRot, p1, p2, maxf);
        if (f >= 0.0f) { hit = BIdx<C>::box + b; maxf = f; stop = maxf == 0.0f; }
    }
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (stop || b >= L.nbi) continue;
        float f = ray_circle(P.bitem_r, L.ip[b], p1, p2, maxf);
        if (f >= 0.0f) { hit = BIdx<C>::bitem + b; maxf = f; stop = maxf == 0.0f; }
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h) {
        if (stop || h >= L.nheal) continue;
        float f = ray_circle(P.heal_r, L.hp[h], p1, p2, maxf);
        if (f >= 0.0f) { hit = BIdx<C>::heal + h; maxf = f; stop = maxf == 0.0f; }
    }
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        if (stop) continue;
        float f = ray_poly(P.wall_poly, P.wall_pos[w], P.wall_q[w], p1, p2, maxf);
        if (f >= 0.0f) { hit = BIdx<C>::wall + w; maxf = f; stop = maxf == 0.0f; }
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (stop || !bit(L.alive_m, i)) continue;
        float f = ray_circle(P.agent_r, L.c[i], p1, p2, maxf);
        if (f >= 0.0f) { hit = BIdx<C>::agent + i; maxf = f; stop = maxf == 0.0f; }
    }
    return hit;
}

template <class C>
__device__ __forceinline__ int ray_cast(const EnvL<C>& L, const Params& P, V2 p1, V2 p2)
{
    float f;
    return ray_cast(L, P, p1, p2, f);
}

// Lidars._update (simulation.py:377-392) for laser k of agent i: the
// Lidars module runs last in the agents group, so its scans see this step's
// final world -- the state k_obs reads.  The 'lidars' key (DESIGN.md
// section 2) holds the laser's relative depth (laser_scan :431-439), 1 when
// nothing is hit, 0 for a dead agent.
template <class C>
__device__ __forceinline__ float lidar_depth(const EnvL<C>& L, const Params& P, int i, int k)
{
    if (!bit(L.alive_m, i)) return 0.0f;
    const V2 org = sel(L.c, i);
    // Python float64: i*(fov/(n_lasers-1)) - fov/2. + orientation (:388-389)
    const float ang = (float)(P.lid_off[k] + (double)sel(L.a, i));
    const V2 end = add(org, from_polar(P.lid_depth, ang));
    float f;
    return ray_cast(L, P, org, end, f) < 0 ? 1.0f : f;
}

// Fixture table: per-lane LDS copy of what a ray test needs by runtime body
// index (positions of every body, box half-extents + meta), [field][kWG]
// interleaved so a wave's 64 lanes hit 64 distinct banks.
template <class C, int S = kWG>  // S: tables in the block ([field][S] interleaved)
struct FixTab {
    float* f;  // [2*NB + 3*BM + 1][S]
    int tid;   // this table's column
    static constexpr int kWords = 2 * C::NB + 3 * C::BM + 1;
    __device__ float& px(int k) const { return f[k * S + tid]; }
    __device__ float& py(int k) const { return f[(C::NB + k) * S + tid]; }
    __device__ float& hx(int b) const { return f[(2 * C::NB + b) * S + tid]; }
    __device__ float& hy(int b) const { return f[(2 * C::NB + C::BM + b) * S + tid]; }
    __device__ float& meta(int b) const { return f[(2 * C::NB + 2 * C::BM + b) * S + tid]; }
    // nbox | nbi << 8 | nheal << 16 | alive mask << 24
    __device__ float& counts() const { return f[(2 * C::NB + 3 * C::BM) * S + tid]; }
};

template <class C, int S>
__device__ __forceinline__ void build_fixtab(const EnvL<C>& L, const Params& P, const FixTab<C, S>& T)
{
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        T.px(BIdx<C>::box + b) = L.bp[b].x;
        T.py(BIdx<C>::box + b) = L.bp[b].y;
        T.hx(b) = L.bhx[b];
        T.hy(b) = L.bhy[b];
        T.meta(b) = __int_as_float(L.bmeta[b]);
        T.px(BIdx<C>::bitem + b) = L.ip[b].x;
        T.py(BIdx<C>::bitem + b) = L.ip[b].y;
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h) {
        T.px(BIdx<C>::heal + h) = L.hp[h].x;
        T.py(BIdx<C>::heal + h) = L.hp[h].y;
    }
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        T.px(BIdx<C>::wall + w) = P.wall_pos[w].x;
        T.py(BIdx<C>::wall + w) = P.wall_pos[w].y;
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        T.px(BIdx<C>::agent + i) = L.c[i].x;
        T.py(BIdx<C>::agent + i) = L.c[i].y;
    }
    T.counts() = __int_as_float(L.nbox | (L.nbi << 8) | (L.nheal << 16) | (int)(L.alive_m << 24));
}

// ray_cast with Box2D's own broadphase test in front: b2DynamicTree::RayCast
// only reports fixtures whose AABB the segment overlaps (segment AABB +
// separating axis).  The cull runs for every body with static indices; the
// exact b2Shape::RayCast then runs only over the surviving bodies, in
// canonical order, by runtime index from the fixture table.  A culled body
// cannot intersect the segment, so its exact test would have rejected it for
// any max fraction: the result is identical to ray_cast (the margin absorbs
// rounding).  Loop trips = the lane's survivors, not all NB bodies.
template <class C, int S>
__device__ __forceinline__ int ray_cast_tab(const EnvL<C>& L, const Params& P, const FixTab<C, S>& T, V2 p1, V2 p2)
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
    uint64_t mask = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b < L.nbox && keep(L.bp[b], L.bhx[b], L.bhy[b])) mask |= 1ull << (BIdx<C>::box + b);
        if (b < L.nbi && keep(L.ip[b], P.bitem_r, P.bitem_r)) mask |= 1ull << (BIdx<C>::bitem + b);
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h)
        if (h < L.nheal && keep(L.hp[h], P.heal_r, P.heal_r)) mask |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        V2 c = scl(0.5f, add(P.wall_lo[w], P.wall_hi[w]));
        V2 e = scl(0.5f, sub(P.wall_hi[w], P.wall_lo[w]));
        if (keep(c, e.x + m, e.y + m)) mask |= 1ull << (BIdx<C>::wall + w);
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (bit(L.alive_m, i) && keep(L.c[i], P.agent_r, P.agent_r)) mask |= 1ull << (BIdx<C>::agent + i);

    float maxf = 1.0f;
    int hit = -1;
    while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        const V2 c = mk(T.px(k), T.py(k));
        float f;
        const bool is_box = k < BIdx<C>::bitem;
        const bool is_wall = k >= BIdx<C>::wall && k < BIdx<C>::agent;
        if (is_box || is_wall) {
            Poly4 poly;
            Rot q = kIdRot;
            V2 pos = c;
            if (is_box) {
                const int meta = __float_as_int(T.meta(k));
                poly = box_poly(T.hx(k), T.hy(k), box_rot(meta), box_copied(meta));
            } else {
                poly = P.wall_poly;
                const int w = k - BIdx<C>::wall;
#pragma unroll
                for (int q2 = 0; q2 < kNumWalls; ++q2)
                    if (q2 == w) { q.s = opq(P.wall_q[q2].s); q.c = opq(P.wall_q[q2].c); }
            }
            f = ray_poly(poly, pos, q, p1, p2, maxf);
        } else {
            const float rad = k < BIdx<C>::heal ? P.bitem_r : (k < BIdx<C>::wall ? P.heal_r : P.agent_r);
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

// ray_cast_tab with every input read from a fixture table (the env of any
// lane of the block): the same broadphase cull and the same exact tests in
// the same canonical order, so the same first hit
template <class C, int S>
__device__ __forceinline__ int ray_cast_fixtab(const Params& P, const FixTab<C, S>& T, V2 p1, V2 p2)
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
    const int cnt = __float_as_int(T.counts());
    const int nbox = cnt & 0xff, nbi = (cnt >> 8) & 0xff, nheal = (cnt >> 16) & 0xff;
    const uint32_t alive = (uint32_t)cnt >> 24;
    uint64_t mask = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b < nbox && keep(mk(T.px(BIdx<C>::box + b), T.py(BIdx<C>::box + b)), T.hx(b), T.hy(b)))
            mask |= 1ull << (BIdx<C>::box + b);
        if (b < nbi && keep(mk(T.px(BIdx<C>::bitem + b), T.py(BIdx<C>::bitem + b)), P.bitem_r, P.bitem_r))
            mask |= 1ull << (BIdx<C>::bitem + b);
    }
#pragma unroll
    for (int h = 0; h < C::HM; ++h)
        if (h < nheal && keep(mk(T.px(BIdx<C>::heal + h), T.py(BIdx<C>::heal + h)), P.heal_r, P.heal_r))
            mask |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
    for (int w = 0; w < kNumWalls; ++w) {
        V2 c = scl(0.5f, add(P.wall_lo[w], P.wall_hi[w]));
        V2 e = scl(0.5f, sub(P.wall_hi[w], P.wall_lo[w]));
        if (keep(c, e.x + m, e.y + m)) mask |= 1ull << (BIdx<C>::wall + w);
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (bit(alive, i) && keep(mk(T.px(BIdx<C>::agent + i), T.py(BIdx<C>::agent + i)), P.agent_r, P.agent_r))
            mask |= 1ull << (BIdx<C>::agent + i);

    float maxf = 1.0f;
    int hit = -1;
    while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        const V2 c = mk(T.px(k), T.py(k));
        float f;
        const bool is_box = k < BIdx<C>::bitem;
        const bool is_wall = k >= BIdx<C>::wall && k < BIdx<C>::agent;
        if (is_box || is_wall) {
            Poly4 poly;
            Rot q = kIdRot;
            if (is_box) {
                const int meta = __float_as_int(T.meta(k));
                poly = box_poly(T.hx(k), T.hy(k), box_rot(meta), box_copied(meta));
            } else {
                poly = P.wall_poly;
                const int w = k - BIdx<C>::wall;
#pragma unroll
                for (int q2 = 0; q2 < kNumWalls; ++q2)
                    if (q2 == w) { q.s = opq(P.wall_q[q2].s); q.c = opq(P.wall_q[q2].c); }
            }
            f = ray_poly(poly, c, q, p1, p2, maxf);
        } else {
            const float rad = k < BIdx<C>::heal ? P.bitem_r : (k < BIdx<C>::wall ? P.heal_r : P.agent_r);
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

// Cameras._update_seen (simulation.py:336-354): camera list position p =
// rank among the alive agents; scr.sn(body) gets bit p when body is in the
// vision cone and the LOS ray to pos + (1+1e-6)*d hits it first.  All
// (camera, candidate) pairs of the env go into one list so a wave iterates
// max(pairs per env), not sum over cameras of max(candidates per camera).
template <class C, int S>
__device__ __forceinline__ void update_seen(const EnvL<C>& L, const Params& P, Scr<C, S>& scr, const FixTab<C, S>& T)
{
#pragma unroll
    for (int k = 0; k < C::NB; ++k) scr.sn(k) = 0u;
    int p = 0, np = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!bit(L.alive_m, i)) continue;
        const V2 pos = L.c[i];
        const Rot q = rot_of(L.a[i]);
        const uint32_t tag = ((uint32_t)p << 11) | ((uint32_t)i << 8);
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < L.nbox && poly_test_point(P.cone, pos, q, L.bp[b])) scr.pr(np++) = tag | (BIdx<C>::box + b);
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < L.nbi && poly_test_point(P.cone, pos, q, L.ip[b])) scr.pr(np++) = tag | (BIdx<C>::bitem + b);
#pragma unroll
        for (int h = 0; h < C::HM; ++h)
            if (h < L.nheal && poly_test_point(P.cone, pos, q, L.hp[h])) scr.pr(np++) = tag | (BIdx<C>::heal + h);
#pragma unroll
        for (int w = 0; w < kNumWalls; ++w)
            if (poly_test_point(P.cone, pos, q, P.wall_pos[w])) scr.pr(np++) = tag | (BIdx<C>::wall + w);
#pragma unroll
        for (int j = 0; j < C::AM; ++j)
            if (j != i && bit(L.alive_m, j) && poly_test_point(P.cone, pos, q, L.c[j]))
                scr.pr(np++) = tag | (BIdx<C>::agent + j);
        ++p;
    }
    const float eps1 = (float)(1.0 + 1e-6);
    for (int t = 0; t < np; ++t) {
        const uint32_t e = scr.pr(t);
        const int body = (int)(e & 0xffu), i = (int)((e >> 8) & 7u), cam = (int)(e >> 11);
        const V2 pos = mk(T.px(BIdx<C>::agent + i), T.py(BIdx<C>::agent + i));
        const V2 oc = mk(T.px(body), T.py(body));
        const V2 d = sub(oc, pos);
        const V2 end = add(pos, scl(eps1, d));
        if (ray_cast_tab(L, P, T, pos, end) == body) scr.sn(body) |= 1u << cam;
    }
}

// update_seen for the reset envs of a block, with the line-of-sight rays of
// all of them dealt over the block's lanes (one wave): each reset lane (mine)
// lists its (camera position, camera agent, candidate body) triples -- the
// cone test of update_seen, same order -- into `list` (at most S x AM x NB
// 16-bit entries: column, camera position, agent, body), then every lane
// casts list entries round-robin from the owner column's fixture table and
// sets the body's bit in the owner's seen row with an LDS atomicOr.  Same
// candidates, same rays, same first-hit test as update_seen; a block pays its
// mean ray count per lane instead of one env's rays in sequence.  Every lane
// of the block calls it (it holds two barriers).
template <class C, int S>
__device__ __forceinline__ void update_seen_dealt(const EnvL<C>& L, const Params& P, Scr<C, S>& scr,
                                                  const FixTab<C, S>& T, bool mine, uint16_t* list)
{
    static_assert(S <= 32 && C::AM <= 8 && C::NB <= 64 && S * C::AM <= 256, "16-bit list entries");
    constexpr int kB = C::NB <= 32 ? 5 : 6, kA = C::AM <= 2 ? 1 : (C::AM <= 4 ? 2 : 3),
                  kC = S <= 8 ? 3 : (S <= 16 ? 4 : 5);
    static_assert(kB + 2 * kA + kC <= 16, "16-bit list entries");
    const int lane = (int)threadIdx.x & 63;
    uint64_t cand[C::AM];
    int np = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) cand[i] = 0;
    if (mine) {
#pragma unroll
        for (int k = 0; k < C::NB; ++k) scr.sn(k) = 0u;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(L.alive_m, i)) continue;
            const V2 pos = L.c[i];
            const Rot q = rot_of(L.a[i]);
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbox && poly_test_point(P.cone, pos, q, L.bp[b])) cand[i] |= 1ull << (BIdx<C>::box + b);
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbi && poly_test_point(P.cone, pos, q, L.ip[b])) cand[i] |= 1ull << (BIdx<C>::bitem + b);
#pragma unroll
            for (int h = 0; h < C::HM; ++h)
                if (h < L.nheal && poly_test_point(P.cone, pos, q, L.hp[h])) cand[i] |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
            for (int w = 0; w < kNumWalls; ++w)
                if (poly_test_point(P.cone, pos, q, P.wall_pos[w])) cand[i] |= 1ull << (BIdx<C>::wall + w);
#pragma unroll
            for (int j = 0; j < C::AM; ++j)
                if (j != i && bit(L.alive_m, j) && poly_test_point(P.cone, pos, q, L.c[j]))
                    cand[i] |= 1ull << (BIdx<C>::agent + j);
            np += __popcll(cand[i]);
        }
    }
    int incl = np;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int total = __shfl(incl, 63, 64);
    int at = incl - np;
    if (mine) {
        int p = 0;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(L.alive_m, i)) continue;
            uint64_t c = cand[i];
            while (c) {
                const int body = __builtin_ctzll(c);
                c &= c - 1;
                list[at++] = (uint16_t)((((lane << kA | p) << kA | i) << kB) | body);
            }
            ++p;
        }
    }
    wave_lds_sync();  // the list and the fixture tables / zeroed seen rows are visible (one-wave block)
    const float eps1 = (float)(1.0 + 1e-6);
    for (int t = lane; t < total; t += 64) {
        const uint32_t en = list[t];
        const int body = (int)(en & ((1u << kB) - 1)), ia = (int)((en >> kB) & ((1u << kA) - 1)),
                  pc = (int)((en >> (kB + kA)) & ((1u << kA) - 1)), col = (int)(en >> (kB + 2 * kA));
        const FixTab<C, S> To{T.f, col};
        const V2 pos = mk(To.px(BIdx<C>::agent + ia), To.py(BIdx<C>::agent + ia));
        const V2 oc = mk(To.px(body), To.py(body));
        const V2 d = sub(oc, pos);
        const V2 end = add(pos, scl(eps1, d));
        if (ray_cast_fixtab(P, To, pos, end) == body) atomicOr(&scr.seen[body * S + col], 1u << pc);
    }
    wave_lds_sync();  // the LDS seen rows are complete (one-wave block)
}

// Cameras.seen <-> state bytes (kGSeen): byte k = camera-position mask of body k
template <class C, int S>
__device__ __forceinline__ void seen_pack(EnvL<C>& L, Scr<C, S>& scr)
{
#pragma unroll
    for (int w = 0; w < kSeenWords<C>; ++w) {
        uint32_t x = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * w + q < C::NB) x |= (scr.sn(4 * w + q) & 0xffu) << (8 * q);
        L.seenw[w] = x;
    }
}

template <class C>
__device__ __forceinline__ uint32_t seen_of(const EnvL<C>& L, int k)  // k static
{
    return (L.seenw[k >> 2] >> (8 * (k & 3))) & 0xffu;
}

// ---------------------------------------------------------------------------
// observation row writer: fetch_observations (masurvival_env.py:510-657)
// ---------------------------------------------------------------------------
template <class C, class Sink>
__device__ __forceinline__ void write_obs_row(const EnvL<C>& L, const Params& P, int i, Sink& row)
{
    const int A = P.A, as_ = P.as_;
    // the big classes' rows span several column windows: their entities are
    // tested one by one against the window (FFA x16384: k_obs 150 -> 130 us);
    // the small classes' sections fit a window or two (the tests cost more)
    constexpr bool fine = C::BM > 4;
    int post_pos[C::AM];
    int np = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        post_pos[i] = bit(L.alive_m, i) ? np : -1;
        np += bit(L.alive_m, i) ? 1 : 0;
    }
    float zone6[6];
    zone6[0] = L.zpos.x;
    zone6[1] = L.zpos.y;
    zone6[2] = L.zrad;
    zone6[3] = 0.0f;
    zone6[4] = 0.0f;
    zone6[5] = 0.0f;
    if (L.phase < P.zone_phases - 1) {
        int ph = L.phase + 1;
        zone6[3] = sel(L.zc, ph).x;
        zone6[4] = sel(L.zc, ph).y;
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k == ph) zone6[5] = opq(P.zradf[k]);
    }
    {
        bool alive = bit(L.alive_m, i);
        int pp = sel(post_pos, i);
        // agent + others rows (_fetch_agents_observations :659-704)
        // (sections outside the sink's column window are skipped: uniform test)
        const bool w_agents = row.want(P.o_agent, as_) || row.want(P.o_oth, (A - 1) * as_) ||
                              row.want(P.o_othm, A - 1);
#pragma unroll
        for (int j = 0; j < C::AM; ++j) {
            if (!w_agents) continue;
            if (j >= A) continue;
            bool aj = bit(L.alive_m, j);
            int o = j == i ? P.o_agent : P.o_oth + (j < i ? j : j - 1) * as_;
            // (per entity: rows of entities outside the window are skipped)
            if (fine && !row.want(o, as_) && !(j != i && row.want(P.o_othm + (j < i ? j : j - 1), 1))) continue;
            row(o++, (float)j);
            if (P.teams) row(o++, (float)team_of(P, j));
            row(o++, aj ? (float)L.health[j] : 0.0f);
            row(o++, aj ? L.c[j].x : 0.0f);
            row(o++, aj ? L.c[j].y : 0.0f);
            row(o++, aj ? L.a[j] : 0.0f);
            row(o++, aj ? L.v[j].x : 0.0f);
            row(o++, aj ? L.v[j].y : 0.0f);
            row(o++, aj ? L.w[j] : 0.0f);
            if (j != i) {
                // others_mask: seen list at the post-despawn list index (quirk D1)
                float m = 1.0f;
                if (alive && aj && (seen_of(L, BIdx<C>::agent + j) >> pp) & 1u) m = 0.0f;
                row(P.o_othm + (j < i ? j : j - 1), m);
            }
        }
        if (row.want(P.o_zone, 6)) {
#pragma unroll
            for (int q = 0; q < 6; ++q) row(P.o_zone + q, zone6[q]);
        }
        if (P.H > 0 && (row.want(P.o_heal, 2 * P.H) || row.want(P.o_healm, P.H))) {
#pragma unroll
            for (int h = 0; h < C::HM; ++h) {
                if (h >= P.H) continue;
                if (fine && !row.want(P.o_heal + 2 * h, 2) && !row.want(P.o_healm + h, 1)) continue;
                bool present = h < L.nheal;
                row(P.o_heal + 2 * h, present ? L.hp[h].x : 0.0f);
                row(P.o_heal + 2 * h + 1, present ? L.hp[h].y : 0.0f);
                float m;
                if (P.omniscient) m = present ? 0.0f : 1.0f;
                else m = (present && alive && ((seen_of(L, BIdx<C>::heal + h) >> pp) & 1u)) ? 0.0f : 1.0f;
                row(P.o_healm + h, m);
            }
        }
        if (P.B > 0 && (row.want(P.o_box, 11 * P.B) || row.want(P.o_boxm, P.B))) {
#pragma unroll
            for (int b = 0; b < C::BM; ++b) {
                if (b >= P.B) continue;
                bool present = b < L.nbox;
                if (!fine || row.want(P.o_box + 11 * b, 11)) {
                    Poly4 poly = box_poly(L.bhx[b], L.bhy[b], box_rot(L.bmeta[b]), box_copied(L.bmeta[b]));
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        row(P.o_box + 11 * b + 2 * v, present ? poly.v[v].x : 0.0f);
                        row(P.o_box + 11 * b + 2 * v + 1, present ? poly.v[v].y : 0.0f);
                    }
                    row(P.o_box + 11 * b + 8, present ? L.bp[b].x : 0.0f);
                    row(P.o_box + 11 * b + 9, present ? L.bp[b].y : 0.0f);
                    row(P.o_box + 11 * b + 10, 0.0f);  // box bodies always have angle 0
                }
                if (fine && !row.want(P.o_boxm + b, 1)) continue;
                float m;
                if (P.omniscient) m = present ? 0.0f : 1.0f;
                else m = (present && alive && ((seen_of(L, BIdx<C>::box + b) >> pp) & 1u)) ? 0.0f : 1.0f;
                row(P.o_boxm + b, m);
            }
        }
        if (P.B > 0 && (row.want(P.o_bi, 10 * P.B) || row.want(P.o_bim, P.B))) {
#pragma unroll
            for (int b = 0; b < C::BM; ++b) {
                if (b >= P.B) continue;
                bool present = b < L.nbi;
                if (!fine || row.want(P.o_bi + 10 * b, 10)) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        V2 cv = box_corner(L.ihx[b], L.ihy[b], bi_rot(L.imeta[b]) + v);
                        row(P.o_bi + 10 * b + 2 * v, present ? cv.x : 0.0f);
                        row(P.o_bi + 10 * b + 2 * v + 1, present ? cv.y : 0.0f);
                    }
                    row(P.o_bi + 10 * b + 8, present ? L.ip[b].x : 0.0f);
                    row(P.o_bi + 10 * b + 9, present ? L.ip[b].y : 0.0f);
                }
                if (fine && !row.want(P.o_bim + b, 1)) continue;
                float m;
                if (P.omniscient) m = present ? 0.0f : 1.0f;
                else m = (present && alive && ((seen_of(L, BIdx<C>::bitem + b) >> pp) & 1u)) ? 0.0f : 1.0f;
                row(P.o_bim + b, m);
            }
        }
        // lidars: zeros here; k_lidar (one lane per ray) writes the columns
        // after k_obs, so this row writer keeps its register budget
        if (P.n_lasers > 0 && row.want(P.o_lid, P.n_lasers)) {
#pragma unroll 1
            for (int k = 0; k < P.n_lasers; ++k) row(P.o_lid + k, 0.0f);
        }
        // usable inventory slots (:620-654)
        int lastmeta = 0;
        float lhx = 0.0f, lhy = 0.0f;
        const int ninv = sel(L.inv_n, i);
        const bool w_slots = row.want(P.o_hs, 1) || row.want(P.o_hsm, 1) || row.want(P.o_bs, 8) ||
                             row.want(P.o_bsm, 1);
        if (w_slots && alive && ninv > 0) {
            lastmeta = sel2(L.inv_meta, i, ninv - 1);
            lhx = sel2(L.inv_hx, i, ninv - 1);
            lhy = sel2(L.inv_hy, i, ninv - 1);
        }
        if (w_slots && P.H > 0) {
            bool isheal = it_kind(lastmeta) == kItemHeal;
            row(P.o_hs, isheal ? (float)P.healing : 0.0f);
            row(P.o_hsm, isheal ? 0.0f : 1.0f);
        }
        if (w_slots && P.B > 0) {
            bool isbox = it_kind(lastmeta) == kItemBox;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                V2 cv = box_corner(lhx, lhy, it_rot(lastmeta) + v);
                row(P.o_bs + 2 * v, isbox ? cv.x : 0.0f);
                row(P.o_bs + 2 * v + 1, isbox ? cv.y : 0.0f);
            }
            row(P.o_bsm, isbox ? 0.0f : 1.0f);
        }
    }
}

// ---------------------------------------------------------------------------
// reset: BaseEnv.reset (masurvival_env.py:59-74) -> Simulation.reset
// ---------------------------------------------------------------------------
template <class C, int S>
__device__ __forceinline__ void env_reset(EnvL<C>& L, const Params& P, Scr<C, S>& scr)
{
    const int A = P.A, H = P.H, B = P.B;
    const int g = P.grid_size;
    const int n = g * g;
    // SpawnGrid.reset: shuffle(square_grid) (semantics.py:71-74, 987-992)
    for (int k = 0; k < n; ++k) scr.pm(k) = (uint8_t)k;
    for (int i = n - 1; i >= 1; --i) {
        int j = (int)pcg_interval32(L, (uint32_t)i);
        uint8_t t = scr.pm(i);
        scr.pm(i) = scr.pm(j);
        scr.pm(j) = t;
    }
    int top = n;
    auto cell = [&](int k) -> V2 {
        int ii = k % g, jj = k / g;
        double ci = (double)ii / g + 0.5 / g;
        double cj = (double)jj / g + 0.5 / g;
        ci = P.floor_size * ci - P.floor_size / 2.0;
        cj = P.floor_size * cj - P.floor_size / 2.0;
        return mk((float)ci, (float)cj);
    };
    // new b2World: no contacts (k_reset zeroes the contact memory), inv_dt0 = 0
    L.inv_dt0 = 0.0f;
    // boxes: RandomizeBoxShapes (semantics.py:107-120), ResetSpawns, Health
    L.nbox = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        L.bp[b] = mk(0.0f, 0.0f);
        L.bhx[b] = 0.0f;
        L.bhy[b] = 0.0f;
        L.bmeta[b] = mk_boxmeta(0, 0, 0, kCauseNone, kCauseNone);
        L.bhealth[b] = 0;
        if (b >= B) continue;
        float hx = P.box_hx, hy = P.box_hy;
        if (P.randomized) {
            double wv = P.avg_w + P.std_w * pcg_normal(L);
            wv = P.min_w > wv ? P.min_w : wv;
            double hv = P.avg_h + P.std_h * pcg_normal(L);
            hv = P.min_h > hv ? P.min_h : hv;
            hx = (float)(wv / 2.0);
            hy = (float)(hv / 2.0);
        }
        L.bhx[b] = hx;
        L.bhy[b] = hy;
    }
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b >= B) continue;
        L.bp[b] = cell(scr.pm(--top));
        L.bmeta[b] = mk_boxmeta(0, 0, 1, kCauseNone, kCauseNone);
        L.bhealth[b] = P.box_health;
        L.nbox = b + 1;
    }
    L.nbi = 0;
    L.npend = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        L.ip[b] = mk(0.0f, 0.0f); L.ihx[b] = 0.0f; L.ihy[b] = 0.0f; L.imeta[b] = 0;
        L.pp[b] = mk(0.0f, 0.0f); L.phx[b] = 0.0f; L.phy[b] = 0.0f; L.pmeta[b] = 0;
    }
    L.nheal = 0;
#pragma unroll
    for (int h = 0; h < C::HM; ++h) {
        L.hp[h] = mk(0.0f, 0.0f);
        if (h >= H) continue;
        L.hp[h] = cell(scr.pm(--top));
        L.nheal = h + 1;
    }
    L.alive_m = 0;
    L.awake_m = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        L.c[i] = mk(0.0f, 0.0f);
        L.a[i] = 0.0f;
        L.v[i] = mk(0.0f, 0.0f);
        L.w[i] = 0.0f;
        L.sleep[i] = 0.0f;
        L.health[i] = 0;
        L.cause[i] = kCauseNone;
        L.cooldown[i] = 0;
        L.inv_n[i] = 0;
#pragma unroll
        for (int k = 0; k < C::SM; ++k) { L.inv_meta[i][k] = 0; L.inv_hx[i][k] = 0.0f; L.inv_hy[i][k] = 0.0f; }
        if (i >= A) continue;
        L.c[i] = cell(scr.pm(--top));
        L.alive_m |= 1u << i;
        L.awake_m |= 1u << i;
        L.health[i] = P.agent_health;
    }
    // SafeZone.post_reset (semantics.py:739-756)
    const int nr = P.zone_nr;
#pragma unroll
    for (int k = 0; k < kMaxPhases; ++k) L.zc[k] = mk(0.0f, 0.0f);
    if (P.zone_random) {
        for (int k = nr; k >= 0; --k) {
            double r = 0.0;
#pragma unroll
            for (int q = 0; q < kMaxPhases; ++q)
                if (q == k) r = opq(P.zrad[q]);
            double Lz = P.floor_size - 2.0 * r;
            double cx = (pcg_random(L) * Lz) - Lz / 2.0;
            double cy = (pcg_random(L) * Lz) - Lz / 2.0;
            put(L.zc, k, mk((float)cx, (float)cy));
        }
    } else {
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k < nr) L.zc[k] = mk(P.zfix[k][0], P.zfix[k][1]);
    }
    L.t_cd = P.zone_cooldown;
    L.t_sh = 0;
    L.phase = 0;
    L.endgame = 0;
    L.zpos = L.zc[0];
    L.zrad = P.zradf[0];
}

// one agent's agent-static row of the contact memory (touching word and
// impulses) shifted with the box despawn compaction of box_health: the row is
// read once into registers, box slot k takes the row of the k-th kept box,
// the slots past the kept boxes are cleared, and the row is written back.
// `kept`: the boxes that stay (b < nbox, health > 0); nb: nbox before.
template <class C, class KT>
__device__ __forceinline__ void compact_cont_row(const KT& K, int i, uint32_t kept, int nb)
{
    uint32_t t = K.ast(i);
    float ni[C::BM], ti[C::BM];
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        ni[b] = K.asni(i, kNumWalls + b);
        ti[b] = K.asti(i, kNumWalls + b);
    }
    int wi = 0;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b >= nb || !bit(kept, b)) continue;
#pragma unroll
        for (int k = 0; k < C::BM; ++k) {
            if (k != wi || k > b) continue;
            const bool tb = bit(t, kNumWalls + b);
            t = tb ? (t | (1u << (kNumWalls + k))) : (t & ~(1u << (kNumWalls + k)));
            ni[k] = ni[b];
            ti[k] = ti[b];
        }
        ++wi;
    }
#pragma unroll
    for (int k = 0; k < C::BM; ++k) {
        if (k < wi) continue;
        t &= ~(1u << (kNumWalls + k));
        ni[k] = 0.0f;
        ti[k] = 0.0f;
    }
    K.set_ast(i, t);
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        K.set_asni(i, kNumWalls + b, ni[b]);
        K.set_asti(i, kNumWalls + b, ti[b]);
    }
}

}  // namespace mas
