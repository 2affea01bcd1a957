// mas_math.h -- float geometry for the MaSurvival HIP kernels (gfx950).
//
// Every routine restates the Box2D 2.3.x arithmetic PyBox2D runs for the
// reference (simulation.py call sites) in the same float operation order, so
// that the device path is bit-identical to the CPU oracle: the kernels are
// compiled with -ffp-contract=off and IEEE f32 division / square root.
// sin/cos is the shared double-precision kernel (mas_sincos) standing in for
// libm sinf/cosf inside b2Rot::Set / the b2Mat22 angle setter.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define MAS_HD __host__ __device__ __forceinline__
#else
#define MAS_HD inline
#endif

namespace mas {

constexpr float kPi = 3.14159265359f;          // b2_pi
constexpr float kEps = 1.1920928955078125e-07f; // FLT_EPSILON (b2_epsilon)
constexpr float kMaxFloat = 3.402823466e+38f;   // b2_maxFloat
constexpr float kLinearSlop = 0.005f;
constexpr float kPolyRadius = 2.0f * kLinearSlop;

struct V2 {
    float x, y;
};
struct Rot {
    float s, c;
};

MAS_HD V2 mk(float x, float y) { V2 r; r.x = x; r.y = y; return r; }

// Optimisation barrier for values picked out of register arrays by runtime
// index: keeps LLVM from rewriting `select(c, a[k], a[j])` into a load from a
// selected address, which would pin the whole array (the env state) in
// scratch memory instead of VGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
MAS_HD float opq(float x) { asm volatile("" : "+v"(x)); return x; }
MAS_HD int opq(int x) { asm volatile("" : "+v"(x)); return x; }
MAS_HD uint32_t opq(uint32_t x) { asm volatile("" : "+v"(x)); return x; }
MAS_HD double opq(double x) { asm volatile("" : "+v"(x)); return x; }
MAS_HD uint64_t opq(uint64_t x) { asm volatile("" : "+v"(x)); return x; }
// a wave-uniform value (SGPRs) the compiler cannot see through: addresses
// derived from it are not merged (CSE'd) with the kernel's other state
// addresses, whose live ranges would otherwise span the kernel and spill
MAS_HD int64_t opq_s(int64_t x) { asm volatile("" : "+s"(x)); return x; }
template <class T>
MAS_HD T* opq_s(T* p)
{
    asm volatile("" : "+s"(p));
    return p;
}
#else
MAS_HD float opq(float x) { return x; }
MAS_HD int opq(int x) { return x; }
MAS_HD uint32_t opq(uint32_t x) { return x; }
MAS_HD double opq(double x) { return x; }
MAS_HD uint64_t opq(uint64_t x) { return x; }
MAS_HD int64_t opq_s(int64_t x) { return x; }
template <class T>
MAS_HD T* opq_s(T* p)
{
    return p;
}
#endif
MAS_HD V2 opq(V2 v) { return mk(opq(v.x), opq(v.y)); }
MAS_HD V2 add(V2 a, V2 b) { return mk(a.x + b.x, a.y + b.y); }
MAS_HD V2 sub(V2 a, V2 b) { return mk(a.x - b.x, a.y - b.y); }
MAS_HD V2 neg(V2 a) { return mk(-a.x, -a.y); }
MAS_HD V2 scl(float s, V2 a) { return mk(s * a.x, s * a.y); }
MAS_HD float dot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
MAS_HD float cross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
MAS_HD V2 cross_vs(V2 a, float s) { return mk(s * a.y, -s * a.x); }
MAS_HD V2 cross_sv(float s, V2 a) { return mk(-s * a.y, s * a.x); }
MAS_HD V2 rmul(Rot q, V2 v) { return mk(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
MAS_HD V2 rmult(Rot q, V2 v) { return mk(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
MAS_HD V2 xmul(V2 p, Rot q, V2 v) { return mk((q.c * v.x - q.s * v.y) + p.x, (q.s * v.x + q.c * v.y) + p.y); }
MAS_HD V2 xmult(V2 p, Rot q, V2 v)
{
    float px = v.x - p.x, py = v.y - p.y;
    return mk(q.c * px + q.s * py, -q.s * px + q.c * py);
}
MAS_HD float len2(V2 a) { return a.x * a.x + a.y * a.y; }
MAS_HD float len(V2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
MAS_HD float dist2(V2 a, V2 b) { V2 c = sub(a, b); return c.x * c.x + c.y * c.y; }
MAS_HD float fmin_b2(float a, float b) { return a < b ? a : b; }
MAS_HD float fmax_b2(float a, float b) { return a > b ? a : b; }
MAS_HD float clamp_b2(float a, float lo, float hi) { return fmax_b2(lo, fmin_b2(a, hi)); }
// b2Vec2::Normalize
MAS_HD float normalize(V2& a)
{
    float l = len(a);
    if (l < kEps) return 0.0f;
    float inv = 1.0f / l;
    a.x *= inv;
    a.y *= inv;
    return l;
}

// shared sin/cos: Cody-Waite reduction + fdlibm kernels in double, rounded once
MAS_HD void sincos_d(double x, double& so, double& co)
{
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double fn = floor(x * invpio2 + 0.5);
    double y = (x - fn * pio2_1) - fn * pio2_1t;
    long long n = (long long)fn;
    double z = y * y;
    double s = y + y * z * (S1 + z * (S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))));
    double c = 1.0 - 0.5 * z + z * z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    int q = (int)(n & 3);
    so = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
    co = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
}

MAS_HD Rot rot_of(float angle)
{
    double s, c;
    sincos_d((double)angle, s, c);
    Rot r;
    r.s = (float)s;
    r.c = (float)c;
    return r;
}

// simulation.py:20-23 from_polar: R.angle = angle; R * b2Vec2(length, 0)
MAS_HD V2 from_polar(float length, float angle)
{
    Rot q = rot_of(angle);
    return mk(q.c * length + (-q.s) * 0.0f, q.s * length + q.c * 0.0f);
}

// ---------------------------------------------------------------------------
// Polygons.  A box shape is (hx, hy, rot, copied): its vertex k is
// kBoxCanon[(rot + k) & 3] scaled by (hx, hy) (b2PolygonShape::SetAsBox order
// rotated); a copied shape (copy_shape -> b2PolygonShape::Set) carries
// normals recomputed from its edges, SetAsBox shapes carry exact normals.
// ---------------------------------------------------------------------------
struct Poly4 {
    V2 v[4];
    V2 n[4];
};

MAS_HD V2 box_corner(float hx, float hy, int idx)
{
    idx &= 3;
    return mk(idx == 0 || idx == 3 ? -hx : hx, idx < 2 ? -hy : hy);
}

MAS_HD Poly4 box_poly(float hx, float hy, int rot, int copied)
{
    Poly4 p;
    for (int k = 0; k < 4; ++k) p.v[k] = box_corner(hx, hy, rot + k);
    if (!copied) {
        p.n[0] = mk(0.0f, -1.0f);
        p.n[1] = mk(1.0f, 0.0f);
        p.n[2] = mk(0.0f, 1.0f);
        p.n[3] = mk(-1.0f, 0.0f);
    } else {
        for (int k = 0; k < 4; ++k) {
            V2 e = sub(p.v[(k + 1) & 3], p.v[k]);
            p.n[k] = cross_vs(e, 1.0f);
            normalize(p.n[k]);
        }
    }
    return p;
}

// copy_shape (simulation.py:43-45) of a box: b2PolygonShape::Set starts the
// hull at the right-most point (ties: lowest y); a CCW rectangle keeps its
// cyclic order, so only the start index changes.
MAS_HD int box_copy_rot(float hx, float hy, int rot)
{
    int i0 = 0;
    V2 p0 = box_corner(hx, hy, rot);
    float x0 = p0.x;
    float y0 = p0.y;
    for (int i = 1; i < 4; ++i) {
        V2 p = box_corner(hx, hy, rot + i);
        if (p.x > x0 || (p.x == x0 && p.y < y0)) {
            i0 = i;
            x0 = p.x;
            y0 = p.y;
        }
    }
    return (rot + i0) & 3;
}

// b2PolygonShape::TestPoint (skin ignored)
MAS_HD bool poly_test_point(const Poly4& P, V2 xp, Rot xq, V2 pt)
{
    V2 pl = rmult(xq, sub(pt, xp));
    bool in = true;
    for (int k = 0; k < 4; ++k) {
        if (dot(P.n[k], sub(pl, P.v[k])) > 0.0f) in = false;
    }
    return in;
}

// b2CircleShape::TestPoint with the centre at the transform position
MAS_HD bool circle_test_point(float r, V2 center, V2 pt)
{
    V2 d = sub(pt, center);
    return dot(d, d) <= r * r;
}

// b2CircleShape::RayCast; returns the fraction or -1
MAS_HD float ray_circle(float r, V2 pos, V2 p1, V2 p2, float maxf)
{
    V2 s = sub(p1, pos);
    float b = dot(s, s) - r * r;
    V2 rr_ = sub(p2, p1);
    float c = dot(s, rr_);
    float rr = dot(rr_, rr_);
    float sigma = c * c - rr * b;
    if (sigma < 0.0f || rr < kEps) return -1.0f;
    float a = -(c + sqrtf(sigma));
    if (0.0f <= a && a <= maxf * rr) return a / rr;
    return -1.0f;
}

// b2PolygonShape::RayCast (4 edges); returns the fraction or -1
MAS_HD float ray_poly(const Poly4& P, V2 xp, Rot xq, V2 p1w, V2 p2w, float maxf)
{
    V2 p1 = rmult(xq, sub(p1w, xp));
    V2 p2 = rmult(xq, sub(p2w, xp));
    V2 d = sub(p2, p1);
    float lower = 0.0f, upper = maxf;
    int index = -1;
    bool miss = false;
    // unrolled (static edge indices keep the polygon in registers); the
    // iterations after a miss change nothing, as Box2D's early return
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (miss) continue;
        float num = dot(P.n[i], sub(P.v[i], p1));
        float den = dot(P.n[i], d);
        if (den == 0.0f) {
            if (num < 0.0f) miss = true;
        } else if (den < 0.0f && num < lower * den) {
            lower = num / den;
            index = i;
        } else if (den > 0.0f && num < upper * den) {
            upper = num / den;
        }
        if (!miss && upper < lower) miss = true;
    }
    if (miss || index < 0) return -1.0f;
    return lower;
}

// b2CollidePolygonAndCircle (polygon = A).  Returns touching; ln/lp = the
// manifold's local normal / local point (type e_faceA).
MAS_HD bool collide_pc(const Poly4& P, V2 xp, Rot xq, V2 c, float rP, float rC, V2& ln, V2& lp)
{
    V2 cl = xmult(xp, xq, c);
    int ni = 0;
    float sep = -kMaxFloat;
    float radius = rP + rC;
    bool out = false;
    for (int i = 0; i < 4; ++i) {
        float s = dot(P.n[i], sub(cl, P.v[i]));
        if (s > radius) out = true;
        if (!out && s > sep) {
            sep = s;
            ni = i;
        }
    }
    if (out) return false;
    int i2 = (ni + 1) & 3;
    V2 v1 = P.v[0], v2 = P.v[0], nrm = P.n[0];
    for (int i = 0; i < 4; ++i) {
        if (i == ni) { v1 = P.v[i]; nrm = P.n[i]; }
        if (i == i2) v2 = P.v[i];
    }
    if (sep < kEps) {
        ln = nrm;
        lp = scl(0.5f, add(v1, v2));
        return true;
    }
    float u1 = dot(sub(cl, v1), sub(v2, v1));
    float u2 = dot(sub(cl, v2), sub(v1, v2));
    if (u1 <= 0.0f) {
        if (dist2(cl, v1) > radius * radius) return false;
        ln = sub(cl, v1);
        normalize(ln);
        lp = v1;
        return true;
    }
    if (u2 <= 0.0f) {
        if (dist2(cl, v2) > radius * radius) return false;
        ln = sub(cl, v2);
        normalize(ln);
        lp = v2;
        return true;
    }
    V2 fc = scl(0.5f, add(v1, v2));
    float s2 = dot(sub(cl, fc), nrm);
    if (s2 > radius) return false;
    ln = nrm;
    lp = fc;
    return true;
}

}  // namespace mas
