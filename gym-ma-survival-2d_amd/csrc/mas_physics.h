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

// ---------------------------------------------------------------------------
// Collide: b2Contact::Update
// ---------------------------------------------------------------------------
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
MAS_HD int slot_type(int key) { return key >> 16; }
MAS_HD int slot_i(int key) { return (key >> 8) & 0xff; }
MAS_HD int slot_js(int key) { return key & 0xff; }

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
    for (int guard = 0; guard < 9 * C::NS + 1; ++guard) {
        // (1) this lane's stale TOI: conservative pre-test, else b2TimeOfImpact
        if (mine && en && cnt <= 8 && !val) {
            float alpha = 1.0f;
            if (!toi_reject(g, sw.c0, sw.c, r)) {
                float beta;
                const int st = time_of_impact(T, sw, r, beta);
                if (st == kToiTouching) alpha = fmin_b2(sw.alpha0 + (1.0f - sw.alpha0) * beta, 1.0f);
            }
            toi = alpha;
            val = true;
        }
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
        V2 cB = sw.c;
        float aB = sw.a;
        if (nsl <= NSLOT && !MAS_TOI_FORCE_FALLBACK) {
            // b2Island::SolveTOI: position iterations (TOI Baumgarte) ...
            for (int it = 0; it < 20; ++it) {
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
        const float h = (1.0f - minAlpha) * dt;
        integrate(cB, aB, vB, wB, h);
        sw.c = cB;
        sw.a = aB;
        val = false;
    }
    ToiGroupOut o;
    o.c = sw.c;
    o.a = sw.a;
    o.v = vB;
    o.w = wB;
    o.touch = (uint32_t)((__ballot(mine && touch) & gmask) >> base);
    const bool capped = (__ballot(mine && en && cnt > 8) & gmask) != 0ull;
    o.events = events + (capped ? 65536 : 0);
    return o;
}

}  // namespace mas
