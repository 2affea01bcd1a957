// mas_physics.h -- b2World::Step for one env in registers (gfx950 HIP).
//
// The world MaSurvival builds is: dynamic circles (agents), static polygons
// (4 walls + boxes), sensors (heals, box items: no contacts).  Every solver
// manifold is 1-point (circles or polygon-circle), so the Box2D 2.3.x step
// reduces to: Collide (narrowphase on every candidate pair, warm-start
// impulses matched by "touching at the previous update"), island Solve
// (damping, warm start, 10 sequential-impulse iterations, integrate, <=10
// position iterations with per-island early exit, sleep) and SolveTOI for
// agent-vs-static pairs (conservative advancement b2TimeOfImpact + TOI
// sub-step).  Contacts are kept in a compact per-env list of C::KC register
// slots in canonical order; an env whose touching-contact count exceeds the
// slots takes the slow path that walks every candidate pair and recomputes
// the constraint data each iteration -- same arithmetic, same result.
#pragma once

#include "mas_env.h"

namespace mas {

constexpr float kBaumgarte = 0.2f;
constexpr float kToiBaumgarte = 0.75f;
constexpr float kMaxLinearCorrection = 0.2f;
constexpr float kMaxTranslation = 2.0f;
constexpr float kMaxRotation = 0.5f * kPi;
constexpr float kTimeToSleep = 0.5f;
constexpr float kLinSleepTol = 0.01f;
constexpr float kAngSleepTol = 2.0f / 180.0f * kPi;

template <class C>
struct StepScratch {
    V2 c0[C::AM];
    float a0[C::AM];
};

// ---------------------------------------------------------------------------
// Collide: b2Contact::Update
// ---------------------------------------------------------------------------
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

// ---------------------------------------------------------------------------
// contact constraint (b2ContactSolver, 1-point manifold)
// ---------------------------------------------------------------------------
struct VC {
    V2 normal, rA, rB;
    float nm, tm, ni, ti;
};

// InitializeVelocityConstraints for agent-agent (circles, A = i, B = j)
MAS_HD VC vc_init_aa(V2 cA, V2 cB, float r, float mA, float iA, float mB, float iB)
{
    VC k;
    V2 normal = mk(1.0f, 0.0f);
    if (dist2(cA, cB) > kEps * kEps) {
        normal = sub(cB, cA);
        normalize(normal);
    }
    V2 wcA = add(cA, scl(r, normal));
    V2 wcB = sub(cB, scl(r, normal));
    V2 point = scl(0.5f, add(wcA, wcB));
    k.normal = normal;
    k.rA = sub(point, cA);
    k.rB = sub(point, cB);
    float rnA = cross(k.rA, normal), rnB = cross(k.rB, normal);
    float kn = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
    k.nm = kn > 0.0f ? 1.0f / kn : 0.0f;
    V2 t = cross_vs(normal, 1.0f);
    float rtA = cross(k.rA, t), rtB = cross(k.rB, t);
    float kt = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
    k.tm = kt > 0.0f ? 1.0f / kt : 0.0f;
    k.ni = 0.0f;
    k.ti = 0.0f;
    return k;
}

// InitializeVelocityConstraints for static polygon (A) - agent (B), e_faceA
MAS_HD VC vc_init_as(V2 sp, Rot sq, V2 ln, V2 lp, V2 cB, float rB, float mB, float iB)
{
    VC k;
    V2 normal = rmul(sq, ln);
    V2 planePoint = xmul(sp, sq, lp);
    V2 clip = cB;
    V2 wcA = add(clip, scl(kPolyRadius - dot(sub(clip, planePoint), normal), normal));
    V2 wcB = sub(clip, scl(rB, normal));
    V2 point = scl(0.5f, add(wcA, wcB));
    k.normal = normal;
    k.rA = sub(point, sp);
    k.rB = sub(point, cB);
    const float mA = 0.0f, iA = 0.0f;
    float rnA = cross(k.rA, normal), rnB = cross(k.rB, normal);
    float kn = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
    k.nm = kn > 0.0f ? 1.0f / kn : 0.0f;
    V2 t = cross_vs(normal, 1.0f);
    float rtA = cross(k.rA, t), rtB = cross(k.rB, t);
    float kt = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
    k.tm = kt > 0.0f ? 1.0f / kt : 0.0f;
    k.ni = 0.0f;
    k.ti = 0.0f;
    return k;
}

// b2ContactSolver::WarmStart for one contact
MAS_HD void vc_warm(const VC& k, V2& vA, float& wA, V2& vB, float& wB, float mA, float iA, float mB, float iB)
{
    V2 t = cross_vs(k.normal, 1.0f);
    V2 Pi = add(scl(k.ni, k.normal), scl(k.ti, t));
    wA -= iA * cross(k.rA, Pi);
    vA = sub(vA, scl(mA, Pi));
    wB += iB * cross(k.rB, Pi);
    vB = add(vB, scl(mB, Pi));
}

// b2ContactSolver::SolveVelocityConstraints for one 1-point contact
MAS_HD void vc_solve(VC& k, V2& vA, float& wA, V2& vB, float& wB, float mA, float iA, float mB, float iB)
{
    V2 t = cross_vs(k.normal, 1.0f);
    {
        V2 dv = sub(sub(add(vB, cross_sv(wB, k.rB)), vA), cross_sv(wA, k.rA));
        float vt = dot(dv, t) - 0.0f;
        float lambda = k.tm * (-vt);
        float maxF = 0.2f * k.ni;
        float ni = clamp_b2(k.ti + lambda, -maxF, maxF);
        lambda = ni - k.ti;
        k.ti = ni;
        V2 Pt = scl(lambda, t);
        vA = sub(vA, scl(mA, Pt));
        wA -= iA * cross(k.rA, Pt);
        vB = add(vB, scl(mB, Pt));
        wB += iB * cross(k.rB, Pt);
    }
    {
        V2 dv = sub(sub(add(vB, cross_sv(wB, k.rB)), vA), cross_sv(wA, k.rA));
        float vn = dot(dv, k.normal);
        float lambda = -k.nm * (vn - 0.0f);
        float ni = fmax_b2(k.ni + lambda, 0.0f);
        lambda = ni - k.ni;
        k.ni = ni;
        V2 Pn = scl(lambda, k.normal);
        vA = sub(vA, scl(mA, Pn));
        wA -= iA * cross(k.rA, Pn);
        vB = add(vB, scl(mB, Pn));
        wB += iB * cross(k.rB, Pn);
    }
}

// one position-constraint correction; returns the separation measured
MAS_HD float pc_solve_aa(V2& cA, float& aA, V2& cB, float& aB, float r, float m, float I, float baum)
{
    V2 normal = sub(cB, cA);
    normalize(normal);
    V2 point = scl(0.5f, add(cA, cB));
    float sep = dot(sub(cB, cA), normal) - r - r;
    V2 rA = sub(point, cA), rB = sub(point, cB);
    float Cc = clamp_b2(baum * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
    float rnA = cross(rA, normal), rnB = cross(rB, normal);
    float K = m + m + I * rnA * rnA + I * rnB * rnB;
    float imp = K > 0.0f ? -Cc / K : 0.0f;
    V2 Pp = scl(imp, normal);
    cA = sub(cA, scl(m, Pp));
    aA -= I * cross(rA, Pp);
    cB = add(cB, scl(m, Pp));
    aB += I * cross(rB, Pp);
    return sep;
}

// (-Cc) / K of an agent-vs-static position constraint.  There K = mA + m +
// iA rnA^2 + I rnB^2 with mA = iA = 0 and rB = point - cB = cB - cB = 0, so K
// is exactly m (the agent's inverse mass) for finite operands, and K > 0.
// The quotient is one float64 multiply by rm = 1 / (double)m, rounded once to
// float: its relative error is below 2^-52, while a quotient of two floats
// lies at least 2^-49 (relative) away from any float rounding midpoint, so
// the rounding is the correctly rounded x / m -- the same bits as the IEEE
// division, without its 12-instruction dependent chain (the hot loop of the
// TOI position iterations).
MAS_HD float div_by_m(float x, double rm) { return (float)((double)x * rm); }

// Fixed points of the Gauss-Seidel loops.  An iteration of the position or
// velocity solver is a deterministic function of the bodies' state and the
// accumulated impulses (the constraint data is fixed for the loop).  When an
// iteration leaves that state bit-identical, every later iteration repeats
// it -- same state, same separation, same exit test -- so the loop can stop
// there with exactly the result of running all its iterations.  (The
// reference oracle runs every iteration; parity checks the equivalence.)
MAS_HD bool same_bits(float a, float b) { return __float_as_uint(a) == __float_as_uint(b); }
MAS_HD bool same_bits(V2 a, V2 b) { return same_bits(a.x, b.x) && same_bits(a.y, b.y); }

MAS_HD float pc_solve_as(V2 sp, Rot sq, V2 ln, V2 lp, V2& cB, float& aB, float r, float m, float I, float baum,
                         double rm)
{
    V2 normal = rmul(sq, ln);
    V2 planePoint = xmul(sp, sq, lp);
    V2 clip = cB;
    float sep = dot(sub(clip, planePoint), normal) - kPolyRadius - r;
    V2 point = clip;
    V2 rB = sub(point, cB);
    float Cc = clamp_b2(baum * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
    float imp = div_by_m(-Cc, rm);  // K == m: see div_by_m
    V2 Pp = scl(imp, normal);
    cB = add(cB, scl(m, Pp));
    aB += I * cross(rB, Pp);
    return sep;
}

// b2Island::Solve integration with the translation / rotation clamp
MAS_HD void integrate(V2& c, float& a, V2& v, float& w, float h)
{
    V2 tr = scl(h, v);
    if (dot(tr, tr) > kMaxTranslation * kMaxTranslation) {
        float ratio = kMaxTranslation / len(tr);
        v.x *= ratio;
        v.y *= ratio;
    }
    float rot = h * w;
    if (rot * rot > kMaxRotation * kMaxRotation) {
        float ratio = kMaxRotation / fabsf(rot);
        w *= ratio;
    }
    c = add(c, scl(h, v));
    a += h * w;
}

// ---------------------------------------------------------------------------
// Solve: islands + compact contact list
// ---------------------------------------------------------------------------
template <class C>
struct Slots {
    int n;
    int key[C::KC];  // type<<16 | i<<8 | js   (type 0: agent-agent j; 1: agent-static s)
    VC k[C::KC];
    V2 ln[C::KC], lp[C::KC];
};

MAS_HD int slot_type(int key) { return key >> 16; }
MAS_HD int slot_i(int key) { return (key >> 8) & 0xff; }
MAS_HD int slot_js(int key) { return key & 0xff; }

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
        if (L.w[i] * L.w[i] > angTolSqr || dot(L.v[i], L.v[i]) > linTolSqr) {
            L.sleep[i] = 0.0f;
            ms = 0.0f;
        } else {
            L.sleep[i] += h;
            ms = fmin_b2(ms, L.sleep[i]);
        }
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

// ---------------------------------------------------------------------------
// b2TimeOfImpact: static polygon (A, sweep fixed) vs agent point (B)
// ---------------------------------------------------------------------------
struct Sweep {
    V2 c0, c;
    float a0, a, alpha0;
};

struct SVert {
    V2 wA, wB, w;
    float a;
    int iA;
};

struct ToiPoly {
    Poly4 P;
    V2 c;  // static position (c0 == c)
    float ang;
    Rot q0;  // rot_of(ang)
};

MAS_HD ToiPoly toi_poly(const Poly4& P, V2 c, float ang)
{
    ToiPoly T;
    T.P = P;
    T.c = c;
    T.ang = ang;
    T.q0 = rot_of(ang);
    return T;
}

// b2Sweep::GetTransform of the static: the interpolated angle is almost
// always bit-identical to ang (always for ang = 0), and then its rotation is
// q0 -- the same rot_of of the same bits, without the fp64 sincos
MAS_HD void sweep_static(const ToiPoly& T, float beta, V2& p, Rot& q)
{
    p = add(scl(1.0f - beta, T.c), scl(beta, T.c));
    float angle = (1.0f - beta) * T.ang + beta * T.ang;
    uint32_t ua, ub;
    memcpy(&ua, &angle, 4);
    memcpy(&ub, &T.ang, 4);
    if (ua == ub) q = T.q0;
    else q = rot_of(angle);
}

MAS_HD V2 sweep_point(const Sweep& B, float beta)
{
    V2 p = add(scl(1.0f - beta, B.c0), scl(beta, B.c));
    // xfB.p -= Mul(q, localCenter = 0); the point proxy vertex (0,0) through
    // the identity-rotation transform: (1*0 - 0*0) + p
    return mk((1.0f * 0.0f - 0.0f * 0.0f) + p.x, (0.0f * 0.0f + 1.0f * 0.0f) + p.y);
}

MAS_HD int support4(const Poly4& P, V2 d)
{
    int best = 0;
    float bv = dot(P.v[0], d);
    for (int i = 1; i < 4; ++i) {
        float val = dot(P.v[i], d);
        if (val > bv) { best = i; bv = val; }
    }
    return best;
}

MAS_HD V2 pv(const Poly4& P, int i)
{
    V2 r = opq(P.v[0]);
    for (int k = 1; k < 4; ++k)
        if (i == k) r = opq(P.v[k]);
    return r;
}

struct SCache {
    float metric;
    int count;
    int iA0, iA1;
};

MAS_HD float simplex_metric(int count, const SVert& v0, const SVert& v1)
{
    // count 3 never reaches the cache (overlap -> early exit)
    return count == 2 ? len(sub(v0.w, v1.w)) : 0.0f;
}

// b2Distance for polygon (A) vs point (B); returns the distance, updates the cache
MAS_HD float gjk(SCache& cache, const Poly4& P, V2 pA, Rot qA, V2 pB)
{
    SVert v[3];
    int count = cache.count;
    for (int k = 0; k < 2; ++k) {
        if (k < count) {
            int ia = k == 0 ? cache.iA0 : cache.iA1;
            v[k].iA = ia;
            v[k].wA = xmul(pA, qA, pv(P, ia));
            v[k].wB = pB;
            v[k].w = sub(v[k].wB, v[k].wA);
            v[k].a = 0.0f;
        }
    }
    if (count > 1) {
        float metric1 = cache.metric;
        float metric2 = simplex_metric(count, v[0], v[1]);
        if (metric2 < 0.5f * metric1 || 2.0f * metric1 < metric2 || metric2 < kEps) count = 0;
    }
    if (count == 0) {
        v[0].iA = 0;
        v[0].wA = xmul(pA, qA, P.v[0]);
        v[0].wB = pB;
        v[0].w = sub(v[0].wB, v[0].wA);
        v[0].a = 1.0f;
        count = 1;
    }
    int iter = 0;
    while (iter < 20) {
        int saveCount = count;
        int save0 = v[0].iA, save1 = v[1].iA, save2 = v[2].iA;
        if (count == 2) {
            V2 w1 = v[0].w, w2 = v[1].w;
            V2 e12 = sub(w2, w1);
            float d12_2 = -dot(w1, e12);
            if (d12_2 <= 0.0f) {
                v[0].a = 1.0f;
                count = 1;
            } else {
                float d12_1 = dot(w2, e12);
                if (d12_1 <= 0.0f) {
                    v[1].a = 1.0f;
                    count = 1;
                    v[0] = v[1];
                } else {
                    float inv = 1.0f / (d12_1 + d12_2);
                    v[0].a = d12_1 * inv;
                    v[1].a = d12_2 * inv;
                    count = 2;
                }
            }
        } else if (count == 3) {
            V2 w1 = v[0].w, w2 = v[1].w, w3 = v[2].w;
            V2 e12 = sub(w2, w1);
            float d12_1 = dot(w2, e12), d12_2 = -dot(w1, e12);
            V2 e13 = sub(w3, w1);
            float d13_1 = dot(w3, e13), d13_2 = -dot(w1, e13);
            V2 e23 = sub(w3, w2);
            float d23_1 = dot(w3, e23), d23_2 = -dot(w2, e23);
            float n123 = cross(e12, e13);
            float d123_1 = n123 * cross(w2, w3);
            float d123_2 = n123 * cross(w3, w1);
            float d123_3 = n123 * cross(w1, w2);
            if (d12_2 <= 0.0f && d13_2 <= 0.0f) {
                v[0].a = 1.0f;
                count = 1;
            } else if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
                float inv = 1.0f / (d12_1 + d12_2);
                v[0].a = d12_1 * inv;
                v[1].a = d12_2 * inv;
                count = 2;
            } else if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
                float inv = 1.0f / (d13_1 + d13_2);
                v[0].a = d13_1 * inv;
                v[2].a = d13_2 * inv;
                count = 2;
                v[1] = v[2];
            } else if (d12_1 <= 0.0f && d23_2 <= 0.0f) {
                v[1].a = 1.0f;
                count = 1;
                v[0] = v[1];
            } else if (d13_1 <= 0.0f && d23_1 <= 0.0f) {
                v[2].a = 1.0f;
                count = 1;
                v[0] = v[2];
            } else if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
                float inv = 1.0f / (d23_1 + d23_2);
                v[1].a = d23_1 * inv;
                v[2].a = d23_2 * inv;
                count = 2;
                v[0] = v[2];
            } else {
                float inv = 1.0f / (d123_1 + d123_2 + d123_3);
                v[0].a = d123_1 * inv;
                v[1].a = d123_2 * inv;
                v[2].a = d123_3 * inv;
                count = 3;
            }
        }
        if (count == 3) break;
        V2 d;
        if (count == 1) {
            d = neg(v[0].w);
        } else {
            V2 e12 = sub(v[1].w, v[0].w);
            float sgn = cross(e12, neg(v[0].w));
            d = sgn > 0.0f ? cross_sv(1.0f, e12) : cross_vs(e12, 1.0f);
        }
        if (len2(d) < kEps * kEps) break;
        SVert nv;
        nv.iA = support4(P, rmult(qA, neg(d)));
        nv.wA = xmul(pA, qA, pv(P, nv.iA));
        nv.wB = pB;
        nv.w = sub(nv.wB, nv.wA);
        nv.a = 0.0f;
        ++iter;
        bool dup = false;
        if (saveCount > 0 && nv.iA == save0) dup = true;
        if (saveCount > 1 && nv.iA == save1) dup = true;
        if (saveCount > 2 && nv.iA == save2) dup = true;
        if (dup) break;
        if (count == 1) v[1] = nv;
        else v[2] = nv;
        ++count;
    }
    V2 wpA, wpB;
    if (count == 1) {
        wpA = v[0].wA;
        wpB = v[0].wB;
    } else if (count == 2) {
        wpA = add(scl(v[0].a, v[0].wA), scl(v[1].a, v[1].wA));
        wpB = add(scl(v[0].a, v[0].wB), scl(v[1].a, v[1].wB));
    } else {
        wpA = add(add(scl(v[0].a, v[0].wA), scl(v[1].a, v[1].wA)), scl(v[2].a, v[2].wA));
        wpB = wpA;
    }
    cache.metric = count == 2 ? len(sub(v[0].w, v[1].w)) : 0.0f;
    cache.count = count;
    cache.iA0 = v[0].iA;
    cache.iA1 = v[1].iA;
    return len(sub(wpA, wpB));
}

enum { kToiFailed = 1, kToiOverlapped = 2, kToiTouching = 3, kToiSeparated = 4 };

struct SepFn {
    int type;  // 0 points, 1 faceA
    V2 axis, lp;
};

MAS_HD SepFn sep_init(const SCache& cache, const ToiPoly& T, const Sweep& B, float t1)
{
    SepFn f;
    V2 pA;
    Rot qA;
    sweep_static(T, t1, pA, qA);
    V2 pB = sweep_point(B, t1);
    if (cache.count == 1) {
        f.type = 0;
        V2 pa = xmul(pA, qA, pv(T.P, cache.iA0));
        f.axis = sub(pB, pa);
        normalize(f.axis);
        f.lp = mk(0.0f, 0.0f);
        return f;
    }
    f.type = 1;
    V2 a1 = pv(T.P, cache.iA0), a2 = pv(T.P, cache.iA1);
    f.axis = cross_vs(sub(a2, a1), 1.0f);
    normalize(f.axis);
    V2 normal = rmul(qA, f.axis);
    f.lp = scl(0.5f, add(a1, a2));
    V2 pa = xmul(pA, qA, f.lp);
    float sv = dot(sub(pB, pa), normal);
    if (sv < 0.0f) f.axis = neg(f.axis);
    return f;
}

MAS_HD float sep_find_min(const SepFn& f, const ToiPoly& T, const Sweep& B, int& iA, float t)
{
    V2 pA;
    Rot qA;
    sweep_static(T, t, pA, qA);
    V2 pB = sweep_point(B, t);
    if (f.type == 0) {
        V2 axisA = rmult(qA, f.axis);
        iA = support4(T.P, axisA);
        V2 pa = xmul(pA, qA, pv(T.P, iA));
        return dot(sub(pB, pa), f.axis);
    }
    V2 normal = rmul(qA, f.axis);
    V2 pa = xmul(pA, qA, f.lp);
    iA = -1;
    return dot(sub(pB, pa), normal);
}

MAS_HD float sep_eval(const SepFn& f, const ToiPoly& T, const Sweep& B, int iA, float t)
{
    V2 pA;
    Rot qA;
    sweep_static(T, t, pA, qA);
    V2 pB = sweep_point(B, t);
    if (f.type == 0) {
        V2 pa = xmul(pA, qA, pv(T.P, iA));
        return dot(sub(pB, pa), f.axis);
    }
    V2 normal = rmul(qA, f.axis);
    V2 pa = xmul(pA, qA, f.lp);
    return dot(sub(pB, pa), normal);
}

// b2TimeOfImpact (tMax = 1): static polygon core (radius 0.01) vs point of
// radius rB.  The static angle is 0 or pi/2, so b2Sweep::Normalize is the
// identity; the point's angle never reaches its position.
MAS_HD int time_of_impact(const ToiPoly& T, const Sweep& B, float rB, float& tout)
{
    tout = 1.0f;
    float totalRadius = kPolyRadius + rB;
    float target = fmax_b2(kLinearSlop, totalRadius - 3.0f * kLinearSlop);
    float tolerance = 0.25f * kLinearSlop;
    float t1 = 0.0f;
    int iter = 0;
    SCache cache;
    cache.count = 0;
    cache.metric = 0.0f;
    cache.iA0 = 0;
    cache.iA1 = 0;
    for (;;) {
        V2 pA;
        Rot qA;
        sweep_static(T, t1, pA, qA);
        V2 pB = sweep_point(B, t1);
        float distance = gjk(cache, T.P, pA, qA, pB);
        if (distance <= 0.0f) {
            tout = 0.0f;
            return kToiOverlapped;
        }
        if (distance < target + tolerance) {
            tout = t1;
            return kToiTouching;
        }
        SepFn f = sep_init(cache, T, B, t1);
        int state = 0;
        float t2 = 1.0f;
        int pushBackIter = 0;
        for (;;) {
            int iA;
            float s2 = sep_find_min(f, T, B, iA, t2);
            if (s2 > target + tolerance) {
                state = kToiSeparated;
                tout = 1.0f;
                break;
            }
            if (s2 > target - tolerance) {
                t1 = t2;
                break;
            }
            float s1 = sep_eval(f, T, B, iA, t1);
            if (s1 < target - tolerance) {
                state = kToiFailed;
                tout = t1;
                break;
            }
            if (s1 <= target + tolerance) {
                state = kToiTouching;
                tout = t1;
                break;
            }
            int rootIterCount = 0;
            float a1 = t1, a2 = t2;
            for (;;) {
                float t;
                if (rootIterCount & 1) t = a1 + (target - s1) * (a2 - a1) / (s2 - s1);
                else t = 0.5f * (a1 + a2);
                ++rootIterCount;
                float sv = sep_eval(f, T, B, iA, t);
                if (fabsf(sv - target) < tolerance) {
                    t2 = t;
                    break;
                }
                if (sv > target) {
                    a1 = t;
                    s1 = sv;
                } else {
                    a2 = t;
                    s2 = sv;
                }
                if (rootIterCount == 50) break;
            }
            ++pushBackIter;
            if (pushBackIter == 8) break;
        }
        ++iter;
        if (state != 0) return state;
        if (iter == 20) {
            tout = t1;
            return kToiFailed;
        }
    }
}

// Conservative pre-test (device only, changes no result): the sweep segment
// against the polygon core's local rectangle grown by target + tolerance +
// margin.  b2TimeOfImpact reports "touching" only where the core-to-point
// distance drops below target + tolerance, so a segment that misses the
// grown rectangle always yields alpha = 1.
MAS_HD bool toi_reject(const StaticG& g, V2 p0, V2 p1, float rB)
{
    const float R = (kPolyRadius + rB - 3.0f * kLinearSlop) + 0.25f * kLinearSlop + 0.02f;
    V2 l0 = xmult(g.p, g.q, p0), l1 = xmult(g.p, g.q, p1);
    float ex = 0.0f, ey = 0.0f;
    for (int k = 0; k < 4; ++k) {
        ex = fmaxf(ex, fabsf(g.poly.v[k].x));
        ey = fmaxf(ey, fabsf(g.poly.v[k].y));
    }
    ex += R;
    ey += R;
    // the segment's box against the grown rectangle first: no divisions, and
    // it settles the far statics (most of them); then the exact slab test
    if (fminf(l0.x, l1.x) > ex || fmaxf(l0.x, l1.x) < -ex || fminf(l0.y, l1.y) > ey || fmaxf(l0.y, l1.y) < -ey)
        return true;
    float tmin = 0.0f, tmax = 1.0f;
    V2 d = sub(l1, l0);
    if (fabsf(d.x) < 1e-12f) {
        if (fabsf(l0.x) > ex) return true;
    } else {
        float ta = (-ex - l0.x) / d.x, tb = (ex - l0.x) / d.x;
        tmin = fmaxf(tmin, fminf(ta, tb));
        tmax = fminf(tmax, fmaxf(ta, tb));
        if (tmin > tmax) return true;
    }
    if (fabsf(d.y) < 1e-12f) {
        if (fabsf(l0.y) > ey) return true;
    } else {
        float ta = (-ey - l0.y) / d.y, tb = (ey - l0.y) / d.y;
        tmin = fmaxf(tmin, fminf(ta, tb));
        tmax = fminf(tmax, fmaxf(ta, tb));
        if (tmin > tmax) return true;
    }
    return false;
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


// ---------------------------------------------------------------------------
// Lane-group b2World::SolveTOI (k_gen_toi): G lanes per (env, agent) and
// lane s of the group owns static s (walls 0..3, then the boxes).  What is
// independent per static runs on its own lane -- the conservative pre-test
// and b2TimeOfImpact against the agent's sweep, the narrowphase update of
// each contact (b2Contact::Update) when the island is built -- and the
// minimum TOI is a butterfly reduction over the group (ties: lowest static,
// as the serial scan's strict <).  The TOI island solve (position then
// velocity iterations) is Gauss-Seidel over the island's contacts in
// Box2D's order (the min contact, then the agent's other touching contacts);
// every lane of the group runs it on the same values, so the group stays
// uniform.  Each contact's constraint data (normal, plane point; the
// velocity constraint) is computed once per event instead of once per
// iteration -- the same operations on the same inputs, so the same bits.
// Same results as toi_agent / world_toi_agent (oracle/mas_oracle.c).
// ---------------------------------------------------------------------------
template <class C>
constexpr int kToiG = C::NS <= 8 ? 8 : (C::NS <= 16 ? 16 : 32);

// value of lane `src` (group-relative) of this lane's group
template <int G, class T>
__device__ __forceinline__ T gshfl(T v, int src)
{
    const int base = (int)(threadIdx.x & 63) & ~(G - 1);
    return __shfl(v, base + src, 64);
}

// pc_solve_as / vc_init_as with the contact's normal and plane point given
// (rmul(sq, ln), xmul(sp, sq, lp) hoisted by the caller): identical ops
MAS_HD float pc_solve_as_h(V2 normal, V2 planePoint, V2& cB, float& aB, float r, float m, float I, float baum,
                           double rm)
{
    V2 clip = cB;
    float sep = dot(sub(clip, planePoint), normal) - kPolyRadius - r;
    V2 point = clip;
    V2 rB = sub(point, cB);
    float Cc = clamp_b2(baum * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
    float imp = div_by_m(-Cc, rm);  // K == m: see div_by_m
    V2 Pp = scl(imp, normal);
    cB = add(cB, scl(m, Pp));
    aB += I * cross(rB, Pp);
    return sep;
}

MAS_HD VC vc_init_as_h(V2 normal, V2 planePoint, V2 sp, V2 cB, float rB, float mB, float iB)
{
    VC k;
    V2 clip = cB;
    V2 wcA = add(clip, scl(kPolyRadius - dot(sub(clip, planePoint), normal), normal));
    V2 wcB = sub(clip, scl(rB, normal));
    V2 point = scl(0.5f, add(wcA, wcB));
    k.normal = normal;
    k.rA = sub(point, sp);
    k.rB = sub(point, cB);
    const float mA = 0.0f, iA = 0.0f;
    float rnA = cross(k.rA, normal), rnB = cross(k.rB, normal);
    float kn = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
    k.nm = kn > 0.0f ? 1.0f / kn : 0.0f;
    V2 t = cross_vs(normal, 1.0f);
    float rtA = cross(k.rA, t), rtB = cross(k.rB, t);
    float kt = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
    k.tm = kt > 0.0f ? 1.0f / kt : 0.0f;
    k.ni = 0.0f;
    k.ti = 0.0f;
    return k;
}

// the position of static q (compile-time q): walls from P, boxes from L
template <class C>
MAS_HD V2 static_pos(const EnvL<C>& L, const Params& P, int q)
{
    return q < kNumWalls ? P.wall_pos[q] : L.bp[q - kNumWalls];
}

struct ToiGroupOut {
    V2 c, v;
    float a, w;
    uint32_t touch;  // touching bits of the group's statics (s < ns), final
    int events;      // TOI events, + 65536 if a contact reached b2_maxSubSteps
};

// SolveTOI of agent I (awake, alive) for lane s of its group.  c0/a0: the
// agent's sweep start (b2Sweep c0/a0 of this world step); L: the env after
// the island solve; K: the contact memory in HBM (impulse resets of this
// lane's contact are written there); t0: agent I's touching word.
// test builds: 1 sends every TOI island through the general (more contacts
// than compact slots) branch, so the parity tests cover it
#ifndef MAS_TOI_FORCE_FALLBACK
#define MAS_TOI_FORCE_FALLBACK 0
#endif
template <class C, int G, class KT>
__device__ __forceinline__ ToiGroupOut toi_agent_group(const EnvL<C>& L, const Params& P, const KT& K, int I, int s,
                                                       V2 c0, float a0, uint32_t t0, float dt)
{
    static_assert(G >= C::NS && G <= 64 && (G & (G - 1)) == 0, "one lane per static");
    const float r = P.agent_r, m = P.inv_mass, Ii = P.inv_I;
    const int ns = kNumWalls + L.nbox;
    const bool mine = s < ns;
    const StaticG g = static_geom_dyn(L, P, s < C::NS ? s : C::NS - 1);
    const ToiPoly T = toi_poly(g.poly, g.p, g.angle);
    Sweep sw;
    sw.c0 = c0;
    sw.a0 = a0;
    sw.c = sel(L.c, I);
    sw.a = sel(L.a, I);
    sw.alpha0 = 0.0f;
    V2 vB = sel(L.v, I);
    float wB = sel(L.w, I);
    bool touch = mine && ((t0 >> s) & 1u);
    bool en = true, val = false;
    int cnt = 0;
    float toi = 1.0f;
    int events = 0;
    const int lane = (int)(threadIdx.x & 63);
    const int base = lane & ~(G - 1);
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << base;
#ifdef MAS_PROFILE
    // per group: TOI calls, position iterations, phase times (constant clock)
    unsigned long long ntoi = 0, npos = 0, lt = wall_clock64(), tp[5] = {0, 0, 0, 0, 0};
#define MAS_GT(k)                                     \
    do {                                              \
        const unsigned long long n_ = wall_clock64(); \
        tp[k] += n_ - lt;                             \
        lt = n_;                                      \
    } while (0)
#else
#define MAS_GT(k) ((void)0)
#endif
    for (int guard = 0; guard < 9 * C::NS + 1; ++guard) {
        // (1) this lane's stale TOI: conservative pre-test, else b2TimeOfImpact
        if (mine && en && cnt <= 8 && !val) {
            float alpha = 1.0f;
            if (!toi_reject(g, sw.c0, sw.c, r)) {
                float beta;
#ifdef MAS_PROFILE
                ++ntoi;
#endif
                const int st = time_of_impact(T, sw, r, beta);
                if (st == kToiTouching) alpha = fmin_b2(sw.alpha0 + (1.0f - sw.alpha0) * beta, 1.0f);
            }
            toi = alpha;
            val = true;
        }
        MAS_GT(0);
        // (2) group minimum over the candidates with alpha < 1
        float ma = (mine && en && cnt <= 8 && toi < 1.0f) ? toi : 2.0f;
        int ms = s;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            const float oa = __shfl_xor(ma, o, 64);
            const int os = __shfl_xor(ms, o, 64);
            if (oa < ma || (oa == ma && os < ms)) {
                ma = oa;
                ms = os;
            }
        }
        if (ma >= 1.0f || 1.0f - 10.0f * kEps < ma) break;
        const int minS = ms;
        const float minAlpha = ma;
        const Sweep backup = sw;
        {
            const float beta = (minAlpha - sw.alpha0) / (1.0f - sw.alpha0);
            sw.c0 = add(sw.c0, scl(beta, sub(sw.c, sw.c0)));
            sw.a0 += beta * (sw.a - sw.a0);
            sw.alpha0 = minAlpha;
            sw.c = sw.c0;
            sw.a = sw.a0;
        }
        // (3) b2Contact::Update of the min contact on its lane
        V2 ln = mk(0.0f, 0.0f), lp = mk(0.0f, 0.0f);
        int tch = 0;
        if (s == minS) {
            const bool t = collide_pc(g.poly, g.p, g.q, sw.c, kPolyRadius, r, ln, lp);
            if (!(t && touch)) {
                K.set_asni(I, s, 0.0f);
                K.set_asti(I, s, 0.0f);
            }
            touch = t;
            tch = t ? 1 : 0;
            val = false;
            ++cnt;
        }
        if (!gshfl<G>(tch, minS)) {
            if (s == minS) en = false;
            sw = backup;
            continue;
        }
        ++events;
        // (4) the island: every other contact of the agent is updated (and re-enabled)
        if (mine && s != minS) {
            en = true;
            const bool t = collide_pc(g.poly, g.p, g.q, sw.c, kPolyRadius, r, ln, lp);
            if (!(t && touch)) {
                K.set_asni(I, s, 0.0f);
                K.set_asti(I, s, 0.0f);
            }
            touch = t;
        }
        const uint32_t isl = (uint32_t)((__ballot(mine && touch) & gmask) >> base);
        // (5) constraint data of every island contact, once per event: the
        // min contact, then the agent's other touching contacts in static
        // order in KT compact slots (gathered from their lanes); more than
        // KT (rare) takes the masked loop over every static
        const V2 nrm = rmul(g.q, ln), ppt = xmul(g.p, g.q, lp);
        const V2 nm = mk(gshfl<G>(nrm.x, minS), gshfl<G>(nrm.y, minS));
        const V2 pm = mk(gshfl<G>(ppt.x, minS), gshfl<G>(ppt.y, minS));
        const V2 sm = mk(gshfl<G>(g.p.x, minS), gshfl<G>(g.p.y, minS));
        constexpr int NSLOT = 2;
        uint32_t rest = isl & ~(1u << minS);
        const int nsl = __builtin_popcount(rest);
        V2 sn[NSLOT], spp[NSLOT], ssp[NSLOT];
#pragma unroll
        for (int j = 0; j < NSLOT; ++j) {
            const int q = rest ? __builtin_ctz(rest) : 0;
            rest &= rest - 1u;
            sn[j] = mk(gshfl<G>(nrm.x, q), gshfl<G>(nrm.y, q));
            spp[j] = mk(gshfl<G>(ppt.x, q), gshfl<G>(ppt.y, q));
            ssp[j] = mk(gshfl<G>(g.p.x, q), gshfl<G>(g.p.y, q));
        }
        MAS_GT(1);
        V2 cB = sw.c;
        float aB = sw.a;
        if (nsl <= NSLOT && !MAS_TOI_FORCE_FALLBACK) {
            // b2Island::SolveTOI: position iterations (TOI Baumgarte) ...
            for (int it = 0; it < 20; ++it) {
#ifdef MAS_PROFILE
                ++npos;
#endif
                const V2 cp = cB;
                const float ap = aB;
                float minsep = 0.0f;
                minsep = fmin_b2(minsep, pc_solve_as_h(nm, pm, cB, aB, r, m, Ii, kToiBaumgarte, P.inv_mass_rcp));
#pragma unroll
                for (int j = 0; j < NSLOT; ++j)
                    if (j < nsl)
                        minsep = fmin_b2(minsep, pc_solve_as_h(sn[j], spp[j], cB, aB, r, m, Ii, kToiBaumgarte,
                                                               P.inv_mass_rcp));
                if (minsep >= -1.5f * kLinearSlop) break;
                if (same_bits(cB, cp) && same_bits(aB, ap)) break;  // fixed point (see same_bits)
            }
            MAS_GT(2);
            sw.c0 = cB;
            sw.a0 = aB;
            // ... then 10 velocity iterations without warm starting
            VC km = vc_init_as_h(nm, pm, sm, cB, r, m, Ii);
            VC kq[NSLOT];
#pragma unroll
            for (int j = 0; j < NSLOT; ++j) kq[j] = vc_init_as_h(sn[j], spp[j], ssp[j], cB, r, m, Ii);
            for (int it = 0; it < 10; ++it) {
                const V2 vp = vB;
                const float wp = wB, mnp = km.ni, mtp = km.ti;
                float qn[NSLOT], qt[NSLOT];
#pragma unroll
                for (int j = 0; j < NSLOT; ++j) {
                    qn[j] = kq[j].ni;
                    qt[j] = kq[j].ti;
                }
                {
                    V2 vz = mk(0.0f, 0.0f);
                    float wz = 0.0f;
                    vc_solve(km, vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                }
#pragma unroll
                for (int j = 0; j < NSLOT; ++j) {
                    if (j >= nsl) continue;
                    V2 vz = mk(0.0f, 0.0f);
                    float wz = 0.0f;
                    vc_solve(kq[j], vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                }
                bool same = same_bits(vB, vp) && same_bits(wB, wp) && same_bits(km.ni, mnp) && same_bits(km.ti, mtp);
#pragma unroll
                for (int j = 0; j < NSLOT; ++j)
                    if (j < nsl) same = same && same_bits(kq[j].ni, qn[j]) && same_bits(kq[j].ti, qt[j]);
                if (same) break;  // fixed point (see same_bits)
            }
        } else {
            // more island contacts than compact slots (rare): every static's
            // normal, point and position stay on its lane and are fetched by
            // shuffle where used, and lane q keeps contact q's accumulated
            // impulses (the group runs the serial solve in lockstep, so every
            // lane holds the same result), so no per-static arrays live in
            // registers for the whole kernel
#pragma unroll 1
            for (int it = 0; it < 20; ++it) {
#ifdef MAS_PROFILE
                ++npos;
#endif
                const V2 cp = cB;
                const float ap = aB;
                float minsep = 0.0f;
                minsep = fmin_b2(minsep, pc_solve_as_h(nm, pm, cB, aB, r, m, Ii, kToiBaumgarte, P.inv_mass_rcp));
#pragma unroll 1
                for (int q = 0; q < C::NS; ++q) {
                    if (!bit(isl, q) || q == minS) continue;
                    const V2 nq = mk(gshfl<G>(nrm.x, q), gshfl<G>(nrm.y, q));
                    const V2 pq = mk(gshfl<G>(ppt.x, q), gshfl<G>(ppt.y, q));
                    minsep = fmin_b2(minsep, pc_solve_as_h(nq, pq, cB, aB, r, m, Ii, kToiBaumgarte, P.inv_mass_rcp));
                }
                if (minsep >= -1.5f * kLinearSlop) break;
                if (same_bits(cB, cp) && same_bits(aB, ap)) break;  // fixed point (see same_bits)
            }
            MAS_GT(2);
            sw.c0 = cB;
            sw.a0 = aB;
            VC km = vc_init_as_h(nm, pm, sm, cB, r, m, Ii);
            float ni_own = 0.0f, ti_own = 0.0f;
#pragma unroll 1
            for (int it = 0; it < 10; ++it) {
                {
                    V2 vz = mk(0.0f, 0.0f);
                    float wz = 0.0f;
                    vc_solve(km, vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                }
#pragma unroll 1
                for (int q = 0; q < C::NS; ++q) {
                    if (!bit(isl, q) || q == minS) continue;
                    const V2 nq = mk(gshfl<G>(nrm.x, q), gshfl<G>(nrm.y, q));
                    const V2 pq = mk(gshfl<G>(ppt.x, q), gshfl<G>(ppt.y, q));
                    const V2 sq = mk(gshfl<G>(g.p.x, q), gshfl<G>(g.p.y, q));
                    VC k = vc_init_as_h(nq, pq, sq, cB, r, m, Ii);
                    k.ni = gshfl<G>(ni_own, q);
                    k.ti = gshfl<G>(ti_own, q);
                    V2 vz = mk(0.0f, 0.0f);
                    float wz = 0.0f;
                    vc_solve(k, vz, wz, vB, wB, 0.0f, 0.0f, m, Ii);
                    if (s == q) {
                        ni_own = k.ni;
                        ti_own = k.ti;
                    }
                }
            }
        }
        MAS_GT(3);
        const float h = (1.0f - minAlpha) * dt;
        integrate(cB, aB, vB, wB, h);
        sw.c = cB;
        sw.a = aB;
        val = false;
        MAS_GT(4);
    }
    ToiGroupOut o;
    o.c = sw.c;
    o.a = sw.a;
    o.v = vB;
    o.w = wB;
    o.touch = (uint32_t)((__ballot(mine && touch) & gmask) >> base);
    const bool capped = (__ballot(mine && en && cnt > 8) & gmask) != 0ull;
    o.events = events + (capped ? 65536 : 0);
#ifdef MAS_PROFILE
    // same slots as toi_agent's profile (profiles/prof_toi.py): max per group
    // of events / TOI calls (summed over the group's lanes) / position
    // iterations, totals, and the longest time per phase (0 TOI, 1 min +
    // narrowphase + island gather, 2 position, 3 velocity, 4 integrate)
    unsigned long long gt = ntoi;
#pragma unroll
    for (int o2 = 1; o2 < G; o2 <<= 1) gt += __shfl_xor(gt, o2, 64);
    if (s == 0) {
        atomicMax(&P.prof[48], (unsigned long long)events);
        atomicMax(&P.prof[49], gt);
        atomicMax(&P.prof[50], npos);
        atomicAdd(&P.prof[51], (unsigned long long)events);
        atomicAdd(&P.prof[52], gt);
        for (int k = 0; k < 5; ++k) atomicMax(&P.prof[53 + k], tp[k]);
    }
#endif
#undef MAS_GT
    return o;
}

// ---------------------------------------------------------------------------
// One b2World::Step of the general path on a lane group of the env (k_gen):
// lane (I, s) = agent I, static s, G lanes per agent.  Same state changes, in
// the same order per body, as world_step_solve + toi_agent_group:
//   Collide   agent-agent pairs on every lane (same values; the env's lane 0
//             writes their memory); agent-static pair (I, s) on its own lane
//             (b2Contact::Update, impulse reset, wake on a touching change);
//   Solve     every lane labels the islands; the lane (root, 0) of each
//             solved island runs b2Island::Solve for that island alone
//             (islands share no body: solving them apart is solving them
//             together, in the canonical contact order within each);
//   SolveTOI  per awake agent on its G lanes (toi_agent_group).
// Every lane keeps the whole env in registers; the contact memory is in LDS
// (K); agent state crosses lanes through `ag` ([AM][kAgW] of this env) at the
// workgroup barriers, which every lane of the workgroup reaches.
// ---------------------------------------------------------------------------
constexpr int kAgW = 8;  // exchanged agent words: c.x c.y a v.x v.y w sleep awake

template <class C, int G, class KT>
__device__ __forceinline__ void gen_world_step(EnvL<C>& L, const Params& P, const KT& K, int I, int s, int lt,
                                               float (*ag)[kAgW], uint32_t* woken, float dt, int64_t diag_env)
{
    constexpr int AM = C::AM;
    const float inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
    const float dtRatio = L.inv_dt0 * dt;
    V2 c0[AM];
    float a0[AM];
#pragma unroll
    for (int i = 0; i < AM; ++i) {
        c0[i] = L.c[i];
        a0[i] = L.a[i];
    }
    // ---- Collide: agent-agent pairs (every lane computes; lane 0 stores) ----
    const uint32_t at0 = K.aat();
    uint32_t at = at0, aa_reset = 0;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = i + 1; j < AM; ++j) {
            if (!(bit(L.alive_m, i) && bit(L.alive_m, j))) continue;
            if (!(bit(L.awake_m, i) || bit(L.awake_m, j))) continue;
            const int p = aa_index<AM>(i, j);
            const bool was = bit(at, p);
            const V2 d = sub(L.c[j], L.c[i]);
            const float dsq = dot(d, d);
            const float rad = P.agent_r + P.agent_r;
            const bool touching = !(dsq > rad * rad);
            if (!(touching && was)) aa_reset |= 1u << p;
            at = touching ? (at | (1u << p)) : (at & ~(1u << p));
            if (touching != was) {
                wake(L, i);
                wake(L, j);
            }
        }
    // ---- Collide: agent-static pair (I, s) on its lane ----
    const int ns = kNumWalls + L.nbox;
    const bool act = bit(L.alive_m, I) && bit(L.awake_m, I);
    bool tch = false, ch = false;
    const uint32_t tm = K.ast(I);
    if (act && s < ns) {
        const bool was = bit(tm, s);
        const StaticG g = static_geom_dyn(L, P, s < C::NS ? s : C::NS - 1);
        const V2 ci = sel(L.c, I);
        const float reach = P.agent_r + kPolyRadius + 1e-3f;
        V2 lo, hi;
        if (s < kNumWalls) {
            lo = mk(opq(P.wall_lo[0].x), opq(P.wall_lo[0].y));
            hi = mk(opq(P.wall_hi[0].x), opq(P.wall_hi[0].y));
#pragma unroll
            for (int k = 1; k < kNumWalls; ++k)
                if (s == k) { lo = opq(P.wall_lo[k]); hi = opq(P.wall_hi[k]); }
        } else {
            const int b = s - kNumWalls;
            V2 bp = opq(L.bp[0]);
            float hx = opq(L.bhx[0]), hy = opq(L.bhy[0]);
#pragma unroll
            for (int k = 1; k < C::BM; ++k)
                if (b == k) { bp = opq(L.bp[k]); hx = opq(L.bhx[k]); hy = opq(L.bhy[k]); }
            lo = mk(bp.x - hx, bp.y - hy);
            hi = mk(bp.x + hx, bp.y + hy);
        }
        const float dx = fmaxf(fmaxf(lo.x - ci.x, ci.x - hi.x), 0.0f);
        const float dy = fmaxf(fmaxf(lo.y - ci.y, ci.y - hi.y), 0.0f);
        const bool cand = dx * dx + dy * dy <= reach * reach;
        if (cand) {
            V2 ln, lp;
            tch = collide_pc(g.poly, g.p, g.q, ci, kPolyRadius, P.agent_r, ln, lp);
            if (!(tch && was)) {
                K.set_asni(I, s, 0.0f);
                K.set_asti(I, s, 0.0f);
            }
        } else if (was) {
            K.set_asni(I, s, 0.0f);
            K.set_asti(I, s, 0.0f);
        }
        ch = tch != was;
    }
    {
        const int lane = (int)(threadIdx.x & 63);
        const int base = lane & ~(G - 1);
        const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << base;
        const uint32_t tb = (uint32_t)((__ballot(tch) & gmask) >> base);
        const bool any_ch = (__ballot(ch) & gmask) != 0ull;
        if (act && s == 0) {
            K.set_ast(I, tb);
            if (any_ch) atomicOr(woken, 1u << I);
        }
    }
    __syncthreads();  // (1) agent-static updates and wakes of every group are in LDS
    if (lt == 0) {
        K.set_aat(at);
#pragma unroll
        for (int p = 0; p < C::NAA; ++p)
            if (bit(aa_reset, p)) { K.set_aani(p, 0.0f); K.set_aati(p, 0.0f); }
    }
    {
        const uint32_t wk = *woken;
#pragma unroll
        for (int i = 0; i < AM; ++i)
            if (bit(wk, i)) wake(L, i);
    }
    __syncthreads();  // (2) agent-agent memory stored; every lane read `woken`
    if (lt == 0) *woken = 0u;
    // ---- Solve: one island per root lane ----
    int label[AM];
    const uint32_t solved = island_labels(L, K, label);
    if (s == 0 && bit(solved, I) && sel(label, I) == I) {
        uint32_t members = 0;
#pragma unroll
        for (int j = 0; j < AM; ++j)
            if (label[j] == I) members |= 1u << j;
        StepScratch<C> S;
        world_solve(L, P, K, S, dt, dtRatio, members & solved);
#pragma unroll
        for (int j = 0; j < AM; ++j) {
            if (!bit(members & solved, j)) continue;
            ag[j][0] = L.c[j].x; ag[j][1] = L.c[j].y; ag[j][2] = L.a[j];
            ag[j][3] = L.v[j].x; ag[j][4] = L.v[j].y; ag[j][5] = L.w[j];
            ag[j][6] = L.sleep[j]; ag[j][7] = bit(L.awake_m, j) ? 1.0f : 0.0f;
        }
    }
    __syncthreads();  // (3) solved agents' state in LDS
#pragma unroll
    for (int j = 0; j < AM; ++j) {
        if (!bit(solved, j)) continue;
        L.c[j] = mk(ag[j][0], ag[j][1]); L.a[j] = ag[j][2];
        L.v[j] = mk(ag[j][3], ag[j][4]); L.w[j] = ag[j][5];
        L.sleep[j] = ag[j][6];
        L.awake_m = ag[j][7] != 0.0f ? (L.awake_m | (1u << j)) : (L.awake_m & ~(1u << j));
    }
    L.inv_dt0 = inv_dt;
    // ---- SolveTOI: agent I on its G lanes ----
    const uint32_t toi_m = L.alive_m & L.awake_m;
    if (bit(toi_m, I)) {
        const uint32_t t0 = K.ast(I);
        const ToiGroupOut o = toi_agent_group<C, G>(L, P, K, I, s, sel(c0, I), sel(a0, I), t0, dt);
        if (s == 0) {
            const uint32_t keep = ~((kNumWalls + L.nbox >= 32) ? 0xffffffffu : ((1u << (kNumWalls + L.nbox)) - 1u));
            K.set_ast(I, (t0 & keep) | o.touch);
            float* a = ag[0];
#pragma unroll
            for (int j = 0; j < AM; ++j)
                if (j == I) a = ag[j];
            a[0] = o.c.x; a[1] = o.c.y; a[2] = o.a; a[3] = o.v.x; a[4] = o.v.y; a[5] = o.w;
            if (P.toi_diag && o.events && diag_env >= 0) atomicAdd(P.toi_diag + diag_env, o.events);
        }
    }
    __syncthreads();  // (4) SolveTOI results in LDS
#pragma unroll
    for (int j = 0; j < AM; ++j) {
        if (!bit(toi_m, j)) continue;
        L.c[j] = mk(ag[j][0], ag[j][1]); L.a[j] = ag[j][2];
        L.v[j] = mk(ag[j][3], ag[j][4]); L.w[j] = ag[j][5];
    }
}

// ---------------------------------------------------------------------------
// Contact-free fast path of one world.Step (speculative).  Valid while the
// env has no contact memory, no pair reaches touching distance and no TOI
// sweep can hit a static: then Box2D's step is damping + integrate + sleep
// per agent, which this function computes with the same operations in the
// same order as world_step / world_solve.  Anything else (a contact, a
// candidate narrowphase pair, a TOI sweep the cheap test cannot reject) sets
// `bail`: the caller discards the registers and the env is re-run by the
// general kernel.  Returns false on bail.
// ---------------------------------------------------------------------------
template <class C>
__device__ __forceinline__ bool world_step_fast(EnvL<C>& L, const Params& P, float dt)
{
    V2 c0[C::AM];
#pragma unroll
    for (int i = 0; i < C::AM; ++i) c0[i] = L.c[i];
    const float inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
    // Collide: any agent-agent pair at touching distance -> general path
    bool bail = false;
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
#pragma unroll
        for (int j = i + 1; j < C::AM; ++j) {
            if (!(bit(L.alive_m, i) && bit(L.alive_m, j))) continue;
            if (!(bit(L.awake_m, i) || bit(L.awake_m, j))) continue;
            V2 d = sub(L.c[j], L.c[i]);
            float rad = P.agent_r + P.agent_r;
            if (!(dot(d, d) > rad * rad)) bail = true;
        }
    // agent-static pairs: any narrowphase candidate -> general path
    const int ns = kNumWalls + L.nbox;
    const float reach = P.agent_r + kPolyRadius + 1e-3f;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!(bit(L.alive_m, i) && bit(L.awake_m, i))) continue;
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
            const float dx = fmaxf(fmaxf(lo.x - L.c[i].x, L.c[i].x - hi.x), 0.0f);
            const float dy = fmaxf(fmaxf(lo.y - L.c[i].y, L.c[i].y - hi.y), 0.0f);
            if (dx * dx + dy * dy <= reach * reach) bail = true;
        }
    }
    if (bail) return false;
    // Solve: every awake alive agent is its own island (world_solve with no
    // contacts: damping, integrate, one position pass that is already done,
    // per-island sleep)
    const float h = dt;
    uint32_t solved = 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (bit(L.alive_m, i) && bit(L.awake_m, i)) solved |= 1u << i;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!bit(solved, i)) continue;
        float ld = 1.0f / (1.0f + h * P.lin_damp);
        L.v[i].x *= ld;
        L.v[i].y *= ld;
        float ad = 1.0f / (1.0f + h * P.ang_damp);
        L.w[i] *= ad;
    }
#pragma unroll
    for (int i = 0; i < C::AM; ++i)
        if (bit(solved, i)) integrate(L.c[i], L.a[i], L.v[i], L.w[i], h);
    const float linTolSqr = kLinSleepTol * kLinSleepTol;
    const float angTolSqr = kAngSleepTol * kAngSleepTol;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!bit(solved, i)) continue;
        float ms;
        if (L.w[i] * L.w[i] > angTolSqr || dot(L.v[i], L.v[i]) > linTolSqr) {
            L.sleep[i] = 0.0f;
            ms = 0.0f;
        } else {
            L.sleep[i] += h;
            ms = fmin_b2(kMaxFloat, L.sleep[i]);
        }
        if (ms >= kTimeToSleep) {
            L.awake_m &= ~(1u << i);
            L.sleep[i] = 0.0f;
            L.v[i] = mk(0.0f, 0.0f);
            L.w[i] = 0.0f;
        }
    }
    // SolveTOI: every sweep of an awake agent must be rejected by the cheap test.
    // World-AABB pre-filter first (changes no result): a sweep whose box, grown
    // by sqrt(2) R plus a rounding margin, misses the static's world AABB lies
    // outside toi_reject's grown local rectangle under any rotation of the
    // static, so toi_reject would return true; it runs only for the statics
    // this filter keeps (agents near a wall or a box).
    const float Rp =
        1.4143f * ((kPolyRadius + P.agent_r - 3.0f * kLinearSlop) + 0.25f * kLinearSlop + 0.02f) + 0.05f;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        if (!(bit(L.alive_m, i) && bit(L.awake_m, i))) continue;
        const V2 slo = mk(fminf(c0[i].x, L.c[i].x) - Rp, fminf(c0[i].y, L.c[i].y) - Rp);
        const V2 shi = mk(fmaxf(c0[i].x, L.c[i].x) + Rp, fmaxf(c0[i].y, L.c[i].y) + Rp);
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
            if (slo.x > hi.x || shi.x < lo.x || slo.y > hi.y || shi.y < lo.y) continue;
            StaticG g = static_geom(L, P, s);
            if (!toi_reject(g, c0[i], L.c[i], P.agent_r)) bail = true;
        }
    }
    L.inv_dt0 = inv_dt;
    return !bail;
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
