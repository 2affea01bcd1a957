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

// update_seen for the single camera slot `cam` (k_cameras runs one lane per
// (env, camera) and ORs the lanes' masks).  Each lane's cone query appends
// its (camera position, lane, body) candidates to the wave's list in LDS; the
// line-of-sight rays of the whole wave are then dealt round-robin over its
// 64 lanes (each ray reads the owner lane's fixture table), so a wave costs
// its mean candidate count, not its maximum.  Same candidates, same rays,
// same first-hit test: the seen masks are unchanged.  One fixture table and
// one seen row per env of the wave (column = env slot = lane / AM); the seen
// row must be zero on entry; `list` holds kWG * NB entries; the block is one
// wave.
template <class C>
__device__ __forceinline__ void update_seen_cam(const EnvL<C>& L, const Params& P, uint32_t* seen,
                                                const FixTab<C, kWG / C::AM>& T, int cam, uint32_t* list, bool active)
{
    const int lane = (int)threadIdx.x & 63;
    static_assert(C::NB <= 64, "body bit masks are 64-bit");
    uint64_t cand = 0;  // bit per body in the cone
    int p = 0;
    V2 pos = mk(0.0f, 0.0f);
    if (active && bit(L.alive_m, cam)) {
        p = __popc(L.alive_m & ((1u << cam) - 1u));
        float ang = 0.0f;
#pragma unroll
        for (int i = 0; i < C::AM; ++i)
            if (i == cam) { pos = opq(L.c[i]); ang = opq(L.a[i]); }
        const Rot q = rot_of(ang);
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < L.nbox && poly_test_point(P.cone, pos, q, L.bp[b])) cand |= 1ull << (BIdx<C>::box + b);
#pragma unroll
        for (int b = 0; b < C::BM; ++b)
            if (b < L.nbi && poly_test_point(P.cone, pos, q, L.ip[b])) cand |= 1ull << (BIdx<C>::bitem + b);
#pragma unroll
        for (int h = 0; h < C::HM; ++h)
            if (h < L.nheal && poly_test_point(P.cone, pos, q, L.hp[h])) cand |= 1ull << (BIdx<C>::heal + h);
#pragma unroll
        for (int w = 0; w < kNumWalls; ++w)
            if (poly_test_point(P.cone, pos, q, P.wall_pos[w])) cand |= 1ull << (BIdx<C>::wall + w);
#pragma unroll
        for (int j = 0; j < C::AM; ++j)
            if (j != cam && bit(L.alive_m, j) && poly_test_point(P.cone, pos, q, L.c[j]))
                cand |= 1ull << (BIdx<C>::agent + j);
    }
    MAS_PROF(P, 13);
    // wave prefix sum of the candidate counts
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
        list[at++] = ((uint32_t)p << 16) | ((uint32_t)lane << 8) | (uint32_t)body;
    }
    wave_lds_sync();  // the block is this wave: the list and every fixture table are visible
    constexpr int S = kWG / C::AM;
    const float eps1 = (float)(1.0 + 1e-6);
    for (int j = lane; j < total; j += 64) {
        const uint32_t en = list[j];
        const int body = (int)(en & 0xffu), o = (int)((en >> 8) & 0xffu), pc = (int)(en >> 16);
        const FixTab<C, S> To{T.f, o / C::AM};
        const int ocam = o % C::AM;  // the owner lane's camera slot
        const V2 opos = mk(To.px(BIdx<C>::agent + ocam), To.py(BIdx<C>::agent + ocam));
        const V2 oc = mk(To.px(body), To.py(body));
        const V2 d = sub(oc, opos);
        const V2 end = add(opos, scl(eps1, d));
        if (ray_cast_fixtab(P, To, opos, end) == body) atomicOr(&seen[body * S + o / C::AM], 1u << pc);
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

// byte k (runtime) := v
template <class C>
__device__ __forceinline__ void seen_put(EnvL<C>& L, int k, uint32_t v)
{
#pragma unroll
    for (int w = 0; w < kSeenWords<C>; ++w)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * w + q == k) L.seenw[w] = (L.seenw[w] & ~(0xffu << (8 * q))) | ((v & 0xffu) << (8 * q));
}

// Health._change_health for agents (semantics.py:490-500); teammates are
// immune to their own badge (TwoTeams.post_reset :942-946)
template <class C>
__device__ __forceinline__ void agent_damage(EnvL<C>& L, const Params& P, int t, int delta, int cause)
{
    if (!bit(L.alive_m, t)) return;
    if (P.teams && cause == kCauseBadge + team_of(P, t)) return;
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (i == t) {
            L.health[i] += delta;
            L.cause[i] = cause;
        }
}

template <class C>
__device__ __forceinline__ void box_damage(EnvL<C>& L, int b, int delta, int cause)
{
#pragma unroll
    for (int k = 0; k < C::BM; ++k) {
        if (k != b) continue;
        int meta = L.bmeta[k];
        if (!box_hinit(meta)) continue;  // not in Health.healths yet
        int vuln = box_vuln(meta);
        if (vuln != kCauseNone && cause != vuln) continue;  // OwnedObjectItem vulnerabilities
        L.bhealth[k] += delta;
        L.bmeta[k] = mk_boxmeta(box_rot(meta), box_copied(meta), 1, vuln, cause);
    }
}

// Inventory.take of one item (semantics.py:179-187) into agent t (runtime)
template <class C>
__device__ __forceinline__ bool inv_take(EnvL<C>& L, const Params& P, int t, int meta, float hx, float hy)
{
    bool ok = false;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (i != t) continue;
        if (1 + L.inv_n[i] > P.slots) continue;
#pragma unroll
        for (int k = 0; k < C::SM; ++k)
            if (k == L.inv_n[i]) {
                L.inv_meta[i][k] = meta;
                L.inv_hx[i][k] = hx;
                L.inv_hy[i][k] = hy;
            }
        L.inv_n[i] += 1;
        ok = true;
    }
    return ok;
}

// pop the last inventory item of agent i (static i)
template <class C>
__device__ __forceinline__ void inv_pop(EnvL<C>& L, int i, int& meta, float& hx, float& hy)
{
    int n = L.inv_n[i] - 1;
    meta = sel(L.inv_meta[i], n);
    hx = sel(L.inv_hx[i], n);
    hy = sel(L.inv_hy[i], n);
    L.inv_n[i] = n;
}

template <class C>
__device__ __forceinline__ void spawn_box(EnvL<C>& L, const Params& P, V2 pos, float hx, float hy, int rot,
                                          int copied, int vuln)
{
    int nb = L.nbox;
    if (nb >= C::BM) return;
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        if (b != nb) continue;
        L.bp[b] = pos;
        L.bhx[b] = hx;
        L.bhy[b] = hy;
        L.bmeta[b] = mk_boxmeta(rot, copied, 0, vuln, kCauseNone);
        L.bhealth[b] = 0;
        // contact memory of static slot b is already zero: slots >= nbox are
        // cleared by the despawn compaction and by reset (invariant)
    }
    L.nbox = nb + 1;
}

template <class C>
__device__ __forceinline__ void spawn_bitem(EnvL<C>& L, V2 pos, float hx, float hy, int meta)
{
    int n = L.nbi;
    if (n >= C::BM) return;
#pragma unroll
    for (int b = 0; b < C::BM; ++b)
        if (b == n) {
            L.ip[b] = pos;
            L.ihx[b] = hx;
            L.ihy[b] = hy;
            L.imeta[b] = meta;
        }
    L.nbi = n + 1;
}

template <class C>
__device__ __forceinline__ void spawn_heal(EnvL<C>& L, V2 pos)
{
    int n = L.nheal;
    if (n >= C::HM) return;
#pragma unroll
    for (int h = 0; h < C::HM; ++h) L.hp[h] = opq(h == n ? pos : L.hp[h]);  // selects, see put()
    L.nheal = n + 1;
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

// SafeZone.tick (semantics.py:776-811)
template <class C>
__device__ __forceinline__ void zone_tick(EnvL<C>& L, const Params& P)
{
    if (L.t_cd == 0) {
        if (L.endgame) return;
        L.t_sh -= 1;
        if (L.t_sh > 0) {
            double t = (double)L.t_sh / (double)P.zone_cooldown;
            double r1 = 0.0, r2 = 0.0;
#pragma unroll
            for (int k = 0; k + 1 < kMaxPhases; ++k)
                if (k == L.phase) { r1 = opq(P.zrad[k]); r2 = opq(P.zrad[k + 1]); }
            V2 c1 = sel(L.zc, L.phase), c2 = sel(L.zc, L.phase + 1);
            double radius = t * r1 + (1.0 - t) * r2;
            float tf = (float)t, tf1 = (float)(1.0 - t);
            L.zrad = (float)radius;
            L.zpos = add(scl(tf, c1), scl(tf1, c2));
            return;
        }
        L.t_cd = P.zone_cooldown;
        L.phase += 1;
        L.zpos = sel(L.zc, L.phase);
#pragma unroll
        for (int k = 0; k < kMaxPhases; ++k)
            if (k == L.phase) L.zrad = opq(P.zradf[k]);
        if (L.phase == P.zone_phases - 1) L.endgame = 1;
    } else {
        L.t_cd -= 1;
        if (L.t_cd > 0) return;
        L.t_sh = P.zone_cooldown;
    }
}

// ---------------------------------------------------------------------------
// one env step: BaseEnv.step (masurvival_env.py:76-90), in three phases that
// run as separate kernels (mas_kernels.inc): step_pre (queue_actions + the
// pre_step hooks), step_phys (2 x world.Step + boxes Health.post_step), then
// Cameras (update_seen) and step_post (the rest of post_step, rewards, done).
// ---------------------------------------------------------------------------
// the wave's melee rays, dealt over its lanes (step_pre): ray j of the wave
// is (owner lane << 8 | agent), its segment, and its first hit
template <class C>
struct RayJobs {
    uint16_t who[kWG * C::AM];
    float x1[kWG * C::AM], y1[kWG * C::AM], x2[kWG * C::AM], y2[kWG * C::AM];
    int16_t hit[kWG * C::AM];
};

template <class C>
__device__ __forceinline__ void step_pre(EnvL<C>& L, const Params& P, const FixTab<C>& T,
                                         const int8_t* __restrict__ act, RayJobs<C>* __restrict__ rj, bool valid,
                                         uint32_t& dirty)
{
    const int A = P.A;
    // dirty: the state groups this step changed (k_pre stores only those):
    // the agents' velocities always, the rest when a module touches them
    dirty = kGDyn;
    if (L.npend > 0) dirty |= kGItem | kGPend;
    // queue_actions (masurvival_env.py:741-755): alive agents only
    int ac[C::AM][6];
    // every byte load unconditional (index clamped into the env's row): the
    // loads issue together instead of one branch + load + wait each
    int8_t raw[C::AM][6];
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
#pragma unroll
        for (int k = 0; k < 6; ++k) raw[i][k] = act[min(i, A - 1) * 6 + k];
    // the reference asserts action_space.contains (masurvival_env.py:80);
    // a kernel cannot raise: out-of-range entries are clamped and the env-step
    // is counted in P.bad_actions (mas_invalid_actions reads it)
    bool bad = false;
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            int x = i < A ? (int)raw[i][k] : 0;
            int hi = k < 3 ? 2 : 1;
            bad = bad || x < 0 || x > hi;
            ac[i][k] = x < 0 ? 0 : (x > hi ? hi : x);
        }
    if (bad && valid) atomicAdd(P.bad_actions, 1);
    MAS_PROF(P, 41);
    // ---------------- pre_step ----------------
    // boxes: Object.pre_step drops last step's queued box items (semantics.py:853-856)
#pragma unroll
    for (int k = 0; k < C::BM; ++k)
        if (k < L.npend) spawn_bitem(L, L.pp[k], L.phx[k], L.phy[k], L.pmeta[k]);
    L.npend = 0;
    // agents: DynamicMotors (simulation.py:407-424).  qs / qc: each agent's
    // rotation, which Melee's from_polar reuses below (no module of pre_step
    // turns a body, so it is the same rotation of the same angle)
    float qs[C::AM], qc[C::AM];
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        qs[i] = 0.0f;
        qc[i] = 1.0f;
        if (!bit(L.alive_m, i)) continue;
        Rot q = rot_of(L.a[i]);
        qs[i] = q.s;
        qc[i] = q.c;
        float par = (float)(ac[i][0] - 1) * P.imp0;
        float nor = (float)(ac[i][1] - 1) * P.imp1;
        V2 J = mk(q.c * par + (-q.s) * nor, q.s * par + q.c * nor);
        float ang = (float)(ac[i][2] - 1) * P.imp2;
        wake(L, i);
        L.v[i] = add(L.v[i], scl(P.inv_mass, J));
        L.w[i] += P.inv_I * cross(sub(L.c[i], L.c[i]), J);
        L.w[i] += P.inv_I * ang;
    }
    MAS_PROF(P, 42);
    // UseLast (semantics.py:300-309): Heal.use (:646-649) / ObjectItem.use (:830-836)
    int uses_heal = 0, uses_box = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!bit(L.alive_m, i) || !ac[i][4] || L.inv_n[i] == 0) continue;
        int meta;
        float hx, hy;
        inv_pop(L, i, meta, hx, hy);
        dirty |= kGRule | kGStat | kGBox;
        if (it_kind(meta) == kItemHeal) {
            uses_heal++;
            agent_damage(L, P, i, P.healing, kCauseNone);
        } else if (it_kind(meta) == kItemBox) {
            uses_box++;
            V2 off = from_polar(P.box_item_offset, L.a[i]);
            spawn_box(L, P, add(L.c[i], off), hx, hy, it_rot(meta), it_copied(meta),
                      P.ownership ? it_owner(meta) : kCauseNone);
        }
    }
    MAS_PROF(P, 43);
    // GiveLast (semantics.py:335-370): nearest body centre within the give radius
    {
        int taker[C::AM];
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            taker[i] = -1;
            // the taker query has no side effect and only a giving agent's is
            // read (the give loop below skips the others)
            if (!bit(L.alive_m, i) || !ac[i][5]) continue;
            V2 c = L.c[i];
            float mind = INFINITY;
            int best = -1;
            auto consider = [&](V2 oc, int id) {
                if (!circle_test_point(P.give_r, c, oc)) return;
                float dd = len(sub(c, oc));
                if (dd < mind) { mind = dd; best = id; }
            };
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbox) consider(L.bp[b], BIdx<C>::box + b);
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbi) consider(L.ip[b], BIdx<C>::bitem + b);
#pragma unroll
            for (int h = 0; h < C::HM; ++h)
                if (h < L.nheal) consider(L.hp[h], BIdx<C>::heal + h);
#pragma unroll
            for (int w = 0; w < kNumWalls; ++w) consider(P.wall_pos[w], BIdx<C>::wall + w);
#pragma unroll
            for (int j = 0; j < C::AM; ++j)
                if (j != i && bit(L.alive_m, j)) consider(L.c[j], BIdx<C>::agent + j);
            taker[i] = best;
        }
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(L.alive_m, i) || !ac[i][5] || taker[i] < BIdx<C>::agent) continue;
            int t = taker[i] - BIdx<C>::agent;
            if (P.teams && team_of(P, t) != team_of(P, i)) continue;  // strangers
            if (L.inv_n[i] == 0) continue;
            int meta;
            float hx, hy;
            inv_pop(L, i, meta, hx, hy);
            inv_take(L, P, t, meta, hx, hy);  // full inventory: the item is lost (quirk D3)
            dirty |= kGRule;
        }
    }
    MAS_PROF(P, 44);
    // Melee / ContinuousMelee (semantics.py:531-554, 584-610): all rays first.
    // A ray (laser_scan: no side effect) is cast only for an agent whose
    // target the attack loop reads -- attacking and off cooldown; the
    // cooldowns are those the attack loop sees (decremented after it)
    {
        int target[C::AM];
        uint32_t need = 0;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            target[i] = -1;
            const bool on_cd = P.melee_cd > 0 && L.cooldown[i] > 0;
            if (bit(L.alive_m, i) && ac[i][3] && !on_cd) need |= 1u << i;
        }
        if (!valid) need = 0;  // (a lane past the last env only joins the wave's collectives)
        // the rays of the whole wave are dealt round-robin over its 64
        // lanes (each reads its owner env's fixture table; the same culled
        // first-hit cast): a wave costs its mean ray count per lane, not the
        // four rays of its busiest env (k_cameras does the same)
        if (__any(need != 0u)) {
            if (need) build_fixtab(L, P, T);
            const int lane = (int)threadIdx.x & 63;
            const int nr = __popc(need);
            int incl = nr;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const int total = __shfl(incl, 63, 64);
            const int first = incl - nr;
            int at = first;
#pragma unroll
            for (int i = 0; i < C::AM; ++i) {
                if (!bit(need, i)) continue;
                // from_polar(range, angle) with the motors' rotation of the angle
                const V2 c = L.c[i];
                const V2 hand = mk(qc[i] * P.melee_range + (-qs[i]) * 0.0f, qs[i] * P.melee_range + qc[i] * 0.0f);
                const V2 e = add(c, hand);
                rj->who[at] = (uint16_t)((lane << 8) | i);
                rj->x1[at] = c.x;
                rj->y1[at] = c.y;
                rj->x2[at] = e.x;
                rj->y2[at] = e.y;
                ++at;
            }
            wave_lds_sync();  // the block is this wave: the job list and the fixture tables are visible
            MAS_PROF(P, 45);
            for (int j = lane; j < total; j += 64) {
                const FixTab<C> To{T.f, (int)(rj->who[j] >> 8)};
                rj->hit[j] = (int16_t)ray_cast_fixtab(P, To, mk(rj->x1[j], rj->y1[j]), mk(rj->x2[j], rj->y2[j]));
            }
            wave_lds_sync();
            MAS_PROF(P, 46);
            at = first;
#pragma unroll
            for (int i = 0; i < C::AM; ++i) {
                if (!bit(need, i)) continue;
                target[i] = rj->hit[at];
                ++at;
            }
        }
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(L.alive_m, i)) continue;
            bool on_cd = P.melee_cd > 0 && L.cooldown[i] > 0;
            if (target[i] >= 0 && ac[i][3] && !on_cd) {
                dirty |= kGRule | kGBox;
                int cause = P.teams ? kCauseBadge + team_of(P, i) : i;
                int tg = target[i];
                if (tg >= BIdx<C>::agent) agent_damage(L, P, tg - BIdx<C>::agent, -P.melee_damage, cause);
                else if (tg < BIdx<C>::bitem) box_damage(L, tg, -P.melee_damage, cause);
                if (P.melee_cd > 0) L.cooldown[i] = P.melee_cd;
            }
        }
        if (P.melee_cd > 0) {
#pragma unroll
            for (int i = 0; i < C::AM; ++i)
                if (L.cooldown[i] > 0) {
                    L.cooldown[i] -= 1;
                    dirty |= kGRule;
                }
        }
    }
    L.stats[17] += (float)uses_heal;
    L.stats[18] += (float)uses_box;
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

// boxes: Health.post_step + Object / OwnedObject despawn (semantics.py:429-435,
// 858-861, 907-912) -- the first post_step hook (dict order: boxes group
// before agents), run at the start of k_cameras.  Returns true when the box /
// pending groups changed.  KT: contact-memory accessor (despawn compaction
// shifts the agent-static contact rows).
template <class C, class KT>
__device__ __forceinline__ bool box_health(EnvL<C>& L, const Params& P, const KT& K, bool cont_owner = true)
{
    bool changed = false;
    {
        bool any_dead = false;
#pragma unroll
        for (int b = 0; b < C::BM; ++b) {
            if (b >= L.nbox) continue;
            int meta = L.bmeta[b];
            if (!box_hinit(meta)) {
                L.bmeta[b] = mk_boxmeta(box_rot(meta), box_copied(meta), 1, box_vuln(meta), box_cause(meta));
                L.bhealth[b] = P.box_health;
                changed = true;
            }
            if (L.bhealth[b] <= 0) any_dead = true;
        }
        if (any_dead) {
            changed = true;
            // the agent-static contact rows follow the boxes, one agent's row
            // at a time (the rows are independent)
            uint32_t kept = 0;
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbox && L.bhealth[b] > 0) kept |= 1u << b;
#pragma unroll 1
            for (int i = 0; i < C::AM; ++i)
                if (cont_owner) compact_cont_row<C>(K, i, kept, L.nbox);
            // stable compaction; dead boxes queue (pos, copy_shape(proto), cause)
            int wi = 0;
#pragma unroll
            for (int b = 0; b < C::BM; ++b) {
                if (b >= L.nbox) continue;
                V2 p = L.bp[b];
                float hx = L.bhx[b], hy = L.bhy[b];
                int meta = L.bmeta[b], hl = L.bhealth[b];
                if (hl <= 0) {
                    int rot = box_copy_rot(hx, hy, box_rot(meta));
                    int pm = mk_bimeta(rot, 1, box_cause(meta));
                    int np_ = L.npend;
#pragma unroll
                    for (int k = 0; k < C::BM; ++k)
                        if (k == np_) { L.pp[k] = p; L.phx[k] = hx; L.phy[k] = hy; L.pmeta[k] = pm; }
                    L.npend = np_ + 1;
                } else {
#pragma unroll
                    for (int k = 0; k < C::BM; ++k) {
                        if (k != wi || k > b) continue;
                        L.bp[k] = p; L.bhx[k] = hx; L.bhy[k] = hy; L.bmeta[k] = meta; L.bhealth[k] = hl;
                    }
                    ++wi;
                }
            }
            L.nbox = wi;
        }
    }
    return changed;
}

// (cont_owner: this lane moves the HBM contact rows; k_cameras runs
// box_health on every camera lane of an env, the first one owning them)

// agents: Cameras.post_step over the pre-despawn list runs between step_phys
// and step_post (k_cameras); step_post reads and compacts its bytes.
// K: the contact memory, touched only on deaths (k_post passes the HBM image
// directly).  rng_used: the PCG64 stream advanced (DeathDrop draws).
template <class C, class KT>
__device__ __forceinline__ bool step_post(EnvL<C>& L, const Params& P, const KT& K, float* rew, bool& rng_used,
                                          uint32_t& dirty)
{
    const int A = P.A;
    // dirty: the state groups this step changed (k_post stores only those):
    // the zone timers and the stats always; the rest on deaths, pickups and
    // zone damage
    dirty = kGZone | kGStat;
    // agents: Health.post_step -> despawn dead (id order): TrackDeaths, IndexBodies,
    // DeathDrop (semantics.py:387-396), Inventory, Health.pre_despawn -> TrackKills
    uint32_t died = 0;
    int kill_cause[C::AM];
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        kill_cause[i] = kCauseNone;
        if (bit(L.alive_m, i) && L.health[i] <= 0) died |= 1u << i;
    }
    rng_used = died != 0;
    if (died) {
        dirty |= kGDyn | kGRule | kGItem | kGHeal | kGSeen | kGRng;
        int total = 0;
#pragma unroll
        for (int i = 0; i < C::AM; ++i)
            if (bit(died, i)) total += L.inv_n[i];
        // angles = 2*pi*rng.random(total), popped from the end per dying body
        // (dead bodies in id order, items in slot order)
        double ang[C::AM * C::SM];
#pragma unroll
        for (int k = 0; k < C::AM * C::SM; ++k) {
            ang[k] = 0.0;
            if (k < total) ang[k] = 6.283185307179586 * pcg_random(L);
        }
        int top = total;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(died, i)) continue;
#pragma unroll
            for (int k = 0; k < C::SM; ++k) {
                if (k >= L.inv_n[i]) continue;
                --top;
                float a = (float)sel(ang, top);
                V2 off = from_polar(P.dd_r, a);
                V2 p = add(L.c[i], off);
                int meta = L.inv_meta[i][k];
                if (it_kind(meta) == kItemHeal) spawn_heal(L, p);
                else spawn_bitem(L, p, L.inv_hx[i][k], L.inv_hy[i][k],
                                 mk_bimeta(it_rot(meta), it_copied(meta), it_owner(meta)));
            }
            L.inv_n[i] = 0;
        }
        uint32_t aat = K.aat();  // one load: the agent-agent touching word
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (!bit(died, i)) continue;
            kill_cause[i] = L.cause[i];
            L.alive_m &= ~(1u << i);
            L.awake_m &= ~(1u << i);
            K.set_ast(i, 0u);
#pragma unroll
            for (int s = 0; s < C::NS; ++s) { K.set_asni(i, s, 0.0f); K.set_asti(i, s, 0.0f); }
#pragma unroll
            for (int j = 0; j < C::AM; ++j) {
                if (j == i) continue;
                int p = j < i ? aa_index<C::AM>(j, i) : aa_index<C::AM>(i, j);
                aat &= ~(1u << p);
                K.set_aani(p, 0.0f);
                K.set_aati(p, 0.0f);
            }
        }
        K.set_aat(aat);
    }
    // AutoPickup.post_step (semantics.py:278-283): every agent's list first
    {
        uint32_t lb[C::AM], lh[C::AM];
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            lb[i] = 0;
            lh[i] = 0;
            if (!bit(L.alive_m, i)) continue;
#pragma unroll
            for (int b = 0; b < C::BM; ++b)
                if (b < L.nbi && circle_test_point(P.pickup_r, L.c[i], L.ip[b])) lb[i] |= 1u << b;
#pragma unroll
            for (int h = 0; h < C::HM; ++h)
                if (h < L.nheal && circle_test_point(P.pickup_r, L.c[i], L.hp[h])) lh[i] |= 1u << h;
        }
        uint32_t takenb = 0, takenh = 0;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
#pragma unroll
            for (int b = 0; b < C::BM; ++b) {
                if (!bit(lb[i], b)) continue;
                int im = L.imeta[b];
                if (inv_take(L, P, i, mk_itmeta(kItemBox, bi_rot(im), bi_copied(im), bi_owner(im)), L.ihx[b], L.ihy[b]))
                    takenb |= 1u << b;
            }
#pragma unroll
            for (int h = 0; h < C::HM; ++h) {
                if (!bit(lh[i], h)) continue;
                if (inv_take(L, P, i, mk_itmeta(kItemHeal, 0, 0, kCauseNone), 0.0f, 0.0f)) takenh |= 1u << h;
            }
        }
        if (takenb | takenh) dirty |= kGRule | kGItem | kGHeal | kGSeen;
        if (takenb) {
            int wi = 0;
#pragma unroll
            for (int b = 0; b < C::BM; ++b) {
                if (b >= L.nbi || bit(takenb, b)) continue;
                V2 p = L.ip[b];
                float hx = L.ihx[b], hy = L.ihy[b];
                int m = L.imeta[b];
                uint32_t sb = seen_of(L, BIdx<C>::bitem + b);
#pragma unroll
                for (int k = 0; k < C::BM; ++k)
                    if (k == wi && k <= b) { L.ip[k] = p; L.ihx[k] = hx; L.ihy[k] = hy; L.imeta[k] = m; }
                seen_put(L, BIdx<C>::bitem + wi, sb);
                ++wi;
            }
            L.nbi = wi;
        }
        if (takenh) {
            int wi = 0;
#pragma unroll
            for (int h = 0; h < C::HM; ++h) {
                if (h >= L.nheal || bit(takenh, h)) continue;
                V2 p = L.hp[h];
                uint32_t sb = seen_of(L, BIdx<C>::heal + h);
#pragma unroll
                for (int k = 0; k < C::HM; ++k)
                    if (k == wi && k <= h) L.hp[k] = p;
                seen_put(L, BIdx<C>::heal + wi, sb);
                ++wi;
            }
            L.nheal = wi;
        }
    }
    // SafeZone.post_step (semantics.py:758-768): damage outliers, then tick
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!bit(L.alive_m, i)) continue;
        if (L.endgame || !circle_test_point(L.zrad, L.zpos, L.c[i])) {
            agent_damage(L, P, i, -P.zone_damage, kCauseZone);
            dirty |= kGRule;
        }
    }
    zone_tick(L, P);
    // ---------------- compute_rewards (masurvival_env.py:757-803) ----------------
    float r[C::AM];
    int last_kills[C::AM];
#pragma unroll
    for (int i = 0; i < C::AM; ++i) { r[i] = 0.0f; last_kills[i] = 0; }
    if (!P.teams) {
        int first_dead = -1;
#pragma unroll
        for (int i = C::AM - 1; i >= 0; --i)
            if (i < A && !bit(L.alive_m, i)) first_dead = i;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) r[i] += bit(L.alive_m, i) ? P.r_alive : P.r_dead;
#pragma unroll
        for (int k = 0; k < C::AM; ++k) {
            if (!bit(died, k)) continue;
            int c = kill_cause[k];
            int idx = -1;
            if (c >= 0 && c < C::AM && bit(L.alive_m, c)) idx = c;
            else if (c == kCauseNone && first_dead >= 0) idx = first_dead;  // None in indexed_agents
#pragma unroll
            for (int i = 0; i < C::AM; ++i)
                if (i == idx) { r[i] += P.r_kill; last_kills[i] += 1; }
        }
#pragma unroll
        for (int k = 0; k < C::AM; ++k)
            if (bit(died, k)) r[k] += P.r_death;
    } else {
        bool talive[2] = {false, false};
#pragma unroll
        for (int i = 0; i < C::AM; ++i)
            if (i < A && bit(L.alive_m, i)) talive[team_of(P, i)] = true;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < C::AM; ++i)
                if (i < A && team_of(P, i) == t) r[i] += talive[t] ? P.r_alive : P.r_dead;
#pragma unroll
        for (int k = 0; k < C::AM; ++k) {
            if (!bit(died, k)) continue;
            int c = kill_cause[k];
            if (c != kCauseBadge && c != kCauseBadge + 1) continue;
            int t = c - kCauseBadge;
#pragma unroll
            for (int i = 0; i < C::AM; ++i)
                if (i < A && team_of(P, i) == t) r[i] += P.r_kill;
            last_kills[t] += 1;
        }
#pragma unroll
        for (int k = 0; k < C::AM; ++k) {
            if (!bit(died, k)) continue;
            int t = team_of(P, k);
#pragma unroll
            for (int i = 0; i < C::AM; ++i)
                if (i < A && team_of(P, i) == t) r[i] += P.r_death;
        }
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i) rew[i] = r[i];
    // ---------------- is_done (masurvival_env.py:810-831) ----------------
    int n_alive = 0;
    if (P.teams) {
        bool t0 = false, t1 = false;
#pragma unroll
        for (int i = 0; i < C::AM; ++i) {
            if (i >= A || !bit(L.alive_m, i)) continue;
            if (team_of(P, i) == 0) t0 = true;
            else t1 = true;
        }
        n_alive = (t0 ? 1 : 0) + (t1 ? 1 : 0);
    } else {
        n_alive = __popc(L.alive_m);
    }
    bool done = P.gameover == 1 ? (n_alive <= 1) : (n_alive == 0);
    // ---------------- _update_stats (masurvival_env.py:483-508) ----------------
    const int R = P.teams ? 2 : A;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (q >= R) continue;
        int j = P.teams ? (q == 0 ? 0 : A / 2) : q;
        L.stats[q] += sel(r, j);
        L.stats[8 + q] += (float)last_kills[q];
    }
    L.stats[16] += 1.0f;
    return done;
}

}  // namespace mas
