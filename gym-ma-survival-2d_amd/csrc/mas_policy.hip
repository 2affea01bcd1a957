// mas_policy.hip -- the PPO consumer's shared-parameter policy MLP as fused
// gfx950 kernels (the reference ships no trainer).
//
//   obs [M][D] -> z1 = W1 x + b1 -> h1 = tanh(z1) (256)
//              -> z2 = W2 h1 + b2 -> h2 = tanh(z2) (256)
//              -> z3 = W3 h2 + b3 (16: the six heads' 15 logits, then the value)
//
// Everything is computed TRANSPOSED, features x rows: one wave owns 32 agent
// rows, which sit on the lanes (the column of every 32x32 MFMA tile), and the
// features sit in the registers.  The f32 result of one
// v_mfma_f32_32x32x16_bf16 is then, converted to bf16 in place, the B
// operand of the next layer's MFMA (a product that sums over the tile's ROW
// index needs no lane movement and no LDS; cdna_hip_programming.md section 3):
// the only price is a permuted k order inside every 16-deep k-step, which the
// host-side packing (k_pack) folds into the weights once per update.  Layer 3
// pads W3 to 32 rows and puts the 16 real outputs on the rows that lane half 0
// holds, so lanes 0..31 end with their agent row's 16 outputs in registers.
//
// Weights are read as pre-packed 1-KiB fragments (one 16-B load per lane per
// MFMA, fully coalesced) from the L2-resident packed image; x is read once.
//
// k_policy_act   rollout: forward + Gumbel-max sampling of the six heads (the
//                exact RNG of k_sample) -> actions, log-prob, value; also
//                writes the bf16 copy of x the update reads.
// k_policy_train update: forward, the PPO loss gradient per row
//                (clipped surrogate + value MSE - entropy bonus), and the
//                backward data path dz -> dA2 -> dA1 in the same registers;
//                writes h1, h2, dA1, dA2, dz feature-major ([F][M] bf16) for
//                the weight-gradient GEMMs and per-block loss partials.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdlib>

#include <cstdint>

namespace mas {
namespace pol {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kH = 256;   // hidden width
constexpr int kMT = 8;    // 32-row M-tiles of a hidden layer
constexpr int kO = 16;    // real outputs of layer 3 (15 logits + value)
constexpr float kTanhC = 2.8853900817779268f;  // 2 log2(e)
#ifndef MAS_POL_WAVES
#define MAS_POL_WAVES 4
#endif
constexpr int kWaves = MAS_POL_WAVES;  // waves per workgroup (4: one per SIMD, two workgroups per CU)
constexpr int kTWaves = kWaves;  // waves per workgroup of the train kernel
constexpr int kLdsFrag = 4608;  // 72 KiB LDS weight stage (16-B fragments): two workgroups per CU
constexpr int kKc = kLdsFrag / (kMT * 64);  // layer-1 k-steps per stage (9)
constexpr int kHalf = kMT / 2 * 16 + 8;     // fragment slots of one forward half stage: W2 4 M-tiles + W3 8 k-steps
static_assert(kHalf * 64 == kLdsFrag, "a forward half stage fills the LDS stage");
constexpr int kBk0 = 16;                    // backward stage 0: W3^T (8 M-tiles x 2 k-steps)
constexpr int kBk1 = kMT / 2 * 16;          // backward stages 1, 2: W2^T M-tiles 0..3, 4..7

// packed image, in fragment slots of 64 x 16 B (one per lane), then f32
// biases; every LDS stage is one contiguous range:
//   w1   [ks1][8]                      layer-1, k-step major
//   w23  [2][kHalf]                    half q: W2 M-tiles 4q..4q+3 (x16 k-steps), then W3 k-steps 8q..8q+7
//   wbk  [kBk0 + 2 kBk1]               W3^T (M-tile x 2 k-steps), then W2^T (M-tile x 16 k-steps)
struct Layout {
    int ks1;  // 16-deep k-steps of layer 1 (ceil(D / 16))
    __host__ __device__ int64_t w1() const { return 0; }
    __host__ __device__ int64_t w23() const { return w1() + (int64_t)ks1 * kMT * 64; }
    __host__ __device__ int64_t wbk() const { return w23() + 2 * kHalf * 64; }
    __host__ __device__ int64_t nfrag() const { return wbk() + (kBk0 + 2 * kBk1) * 64; }
    // biases (floats) after the fragments: b1p [8][2][16], b2p [8][2][16] (both x kTanhC), b3 [16]
    __host__ __device__ int64_t b1() const { return nfrag() * 4; }
    __host__ __device__ int64_t b2() const { return b1() + kMT * 2 * 16; }
    __host__ __device__ int64_t b3() const { return b2() + kMT * 2 * 16; }
    __host__ __device__ int64_t bytes() const { return (b3() + kO) * 4; }
};

// row of the 32x32 C tile held in register i by lane half h
__host__ __device__ inline int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
// row of X carried by element j of lane half h in k-step s of an
// accumulator-as-operand fragment (registers 8s..8s+7)
__host__ __device__ inline int prow(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }
// padded layer-3 row of real output o (lane half 0, register o)
__host__ __device__ inline int orow(int o) { return (o & 3) + 8 * (o >> 2); }

// One thread per packed element: bf16 fragments and permuted f32 biases from
// the torch fp32 parameters (W1 [256][D], W2 [256][256], W3 [16][256]).
__global__ void k_pack(int D, int ks1, const float* __restrict__ W1, const float* __restrict__ b1,
                       const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ W3,
                       const float* __restrict__ b3, uint8_t* __restrict__ out)
{
    const Layout L{ks1};
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    __bf16* frag = reinterpret_cast<__bf16*>(out);
    float* fb = reinterpret_cast<float*>(out);
    const int64_t nel = L.nfrag() * 8;
    if (t < nel) {
        const int64_t f = t >> 3;
        const int j = (int)(t & 7);
        const int l = (int)(f & 63), r = l & 31, h = l >> 5;
        const int64_t g = f >> 6;  // fragment index
        float v = 0.0f;
        if (f < L.w23()) {  // W1: g = ks * 8 + mt, natural k order
            const int ks = (int)(g / kMT), mt = (int)(g % kMT);
            const int k = 16 * ks + 8 * h + j;
            v = k < D ? W1[(int64_t)(32 * mt + r) * D + k] : 0.0f;
        } else if (f < L.wbk()) {
            const int q = (int)(g - L.w23() / 64);
            const int hf = q / kHalf, u = q % kHalf;
            if (u < kMT / 2 * 16) {  // W2 (mo, kk = 2 mt + s), k permuted
                const int mo = kMT / 2 * hf + u / 16, kk = u % 16;
                v = W2[(32 * mo + r) * kH + 32 * (kk >> 1) + prow(kk & 1, h, j)];
            } else {  // W3 padded to 32 rows, k-step kk
                const int kk = 8 * hf + (u - kMT / 2 * 16);
                int o = -1;
                for (int q2 = 0; q2 < kO; ++q2)
                    if (orow(q2) == r) o = q2;
                v = o >= 0 ? W3[o * kH + 32 * (kk >> 1) + prow(kk & 1, h, j)] : 0.0f;
            }
        } else {
            const int q = (int)(g - L.wbk() / 64);
            if (q < 16) {  // W3pad^T: (mo, s)
                const int mo = q / 2, sk = q % 2;
                const int pr = prow(sk, h, j);  // padded output row
                int o = -1;
                for (int q2 = 0; q2 < kO; ++q2)
                    if (orow(q2) == pr) o = q2;
                v = o >= 0 ? W3[o * kH + 32 * mo + r] : 0.0f;
            } else {  // W2^T: (mt, kk = 2 mo + s)
                const int mt = (q - 16) / 16, kk = (q - 16) % 16;
                v = W2[(32 * (kk >> 1) + prow(kk & 1, h, j)) * kH + 32 * mt + r];
            }
        }
        frag[t] = (__bf16)v;
        return;
    }
    const int64_t u = t - nel;  // biases
    if (u < 2 * kMT * 2 * 16) {
        const int which = (int)(u / (kMT * 2 * 16));
        const int rem = (int)(u % (kMT * 2 * 16));
        const int mt = rem / 32, h = (rem / 16) & 1, i = rem & 15;
        const float* b = which == 0 ? b1 : b2;
        // hidden biases pre-scaled for tanh_pre (2 log2(e) b)
        fb[(which == 0 ? L.b1() : L.b2()) + rem] = b[32 * mt + crow(i, h)] * kTanhC;
    } else if (u < 2 * kMT * 2 * 16 + kO) {
        const int o = (int)(u - 2 * kMT * 2 * 16);
        fb[L.b3() + o] = b3[o];
    }
}

// timing experiments only (results garbage): 1 no tanh, 2 no sampling, 4 no MFMA, 8 no x loads
#ifndef MAS_POL_OCC_ACT
#define MAS_POL_OCC_ACT 2
#endif
#ifndef MAS_POL_EXP
#define MAS_POL_EXP 0
#endif
// scheduling strategy hint for the MFMA + LDS-read loops (A/B builds)
#ifndef MAS_POL_IGLP
#define MAS_POL_IGLP -1
#endif
__device__ __forceinline__ void iglp()
{
#if MAS_POL_IGLP >= 0
    __builtin_amdgcn_iglp_opt(MAS_POL_IGLP);
#endif
}

__device__ __forceinline__ f16v mfma(bf8 a, bf8 b, f16v c)
{
    if (MAS_POL_EXP & 4) return c + (float)a[0];
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// tanh(a + b) from the pre-scaled bias bc = kTanhC b (the packed image holds
// it): 1 - 2 / (2^(kTanhC (a + b)) + 1), five instructions -- FMA, v_exp_f32,
// add, v_rcp_f32, FMA -- where (e - 1) / (e + 1) after a clamp took eight.
// No clamp needed: 2^(+large) = inf gives 1, 2^(-large) = 0 gives -1
// (~1 ulp each for exp / rcp; the result is rounded to bf16 anyway).
__device__ __forceinline__ float tanh_pre(float a, float bc)
{
    if (MAS_POL_EXP & 1) return a;
    const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(a, kTanhC, bc));
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}
// tanh'(z) = 1 - h^2 from the stored activation h
__device__ __forceinline__ float dtanh(float h) { return __builtin_fmaf(-h, h, 1.0f); }

__device__ __forceinline__ float exp_fast(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float log_fast(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }

__device__ __forceinline__ void load16(const float* __restrict__ p, float* v)
{
    const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 a = q[k];
        v[4 * k] = a.x;
        v[4 * k + 1] = a.y;
        v[4 * k + 2] = a.z;
        v[4 * k + 3] = a.w;
    }
}

// x fragment of k-step ks for this lane's row from fp32 obs [M][D], for
// D % 4 == 0 and a complete k-step: unconditional 16-B loads (row clamped
// into range by the caller), the row of an out-of-range lane zeroed after
__device__ __forceinline__ bf8 x_frag_f32_full(const float* __restrict__ obs, int64_t row, bool ok, int D, int k0)
{
    const float* p = obs + row * D + k0;
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    const float z = ok ? 1.0f : 0.0f;
    bf8 f;
    f[0] = (__bf16)(a.x * z); f[1] = (__bf16)(a.y * z); f[2] = (__bf16)(a.z * z); f[3] = (__bf16)(a.w * z);
    f[4] = (__bf16)(b.x * z); f[5] = (__bf16)(b.y * z); f[6] = (__bf16)(b.z * z); f[7] = (__bf16)(b.w * z);
    return f;
}

// x fragment of k-step ks for this lane's row from fp32 obs [M][D]
__device__ __forceinline__ bf8 x_frag_f32(const float* __restrict__ obs, int64_t row, bool ok, int D, int k0)
{
    bf8 f;
    if (MAS_POL_EXP & 8) {
        for (int j = 0; j < 8; ++j) f[j] = (__bf16)(float)(row + k0 + j);
        return f;
    }
    const float* p = obs + row * D + k0;
    if (ok && (D & 3) == 0 && k0 + 8 <= D) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        f[0] = (__bf16)a.x; f[1] = (__bf16)a.y; f[2] = (__bf16)a.z; f[3] = (__bf16)a.w;
        f[4] = (__bf16)b.x; f[5] = (__bf16)b.y; f[6] = (__bf16)b.z; f[7] = (__bf16)b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)  // column D = 1: the bias column of the update's dW1 GEMM (W1 is 0 there)
            f[j] = (__bf16)((ok && k0 + j < D) ? p[j] : (ok && k0 + j == D ? 1.0f : 0.0f));
    }
    return f;
}

// cooperative copy of n <= kLdsFrag fragments (n a multiple of 64) into the
// LDS stage by LDS-DMA (global_load_lds_dwordx4: no registers, every load of
// the stage in flight at once, one wait), between two block barriers
constexpr int kStagePer = kLdsFrag / (64 * kWaves);  // fragments per thread (18)
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void stage(bf8* __restrict__ wl, const bf8* __restrict__ src, int n)
{
    __syncthreads();  // every wave is done with the previous stage
    // the wave's first fragment in a scalar register and the lane's byte
    // offset in a 32-bit one: each copy is a uniform base + that offset
    const int w0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    const uint32_t loff = (threadIdx.x & 63) * 16u;
#pragma unroll
    for (int k = 0; k < kStagePer; ++k) {
        const int i0 = w0 + k * 64 * kWaves;  // the wave's first fragment
        if (i0 < n)  // wave-uniform
            __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const uint8_t*>(src + i0) + loff),
                                             (lds_void*)(wl + i0), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
}

// Stagers: a call S(src, n) returns the LDS buffer holding the weights the
// caller computes from next; every wave of the block makes the same calls.
// Stage1: one 72-KiB buffer, copied in and drained per call (stage()).
struct Stage1 {
    bf8* wl;
    __device__ __forceinline__ const bf8* operator()(const bf8* src, int n) const
    {
        stage(wl, src, n);
        return wl;
    }
};

// The packed biases (b1p, b2p, b3: kBiasF floats) copied into LDS once per
// workgroup (MAS_POL_LDSB=1): the per-M-tile bias reads of the layers become
// ds_read_b128 instead of global loads.  No gain measured (r04g: the A/B
// was within policy_bench's run-order bias -- the same train kernel timed
// 3.88 vs 3.52 ms as first vs second library of one process): the MFMA
// loops read a 1-KiB weight fragment from LDS per 32-cycle MFMA on every
// SIMD, the CU's whole 128 B/clk, so LDS bias reads compete with the weight
// reads, while the global bias loads the compiler issues early are mostly
// hidden.  Off by default (k_policy_train_db always stages them: its
// double-buffered layout has the room).  Ordered before every read by the
// first weight stage's drain + barrier.
#ifndef MAS_POL_LDSB
#define MAS_POL_LDSB 0
#endif
constexpr int kBiasF = 2 * kMT * 2 * 16 + kO;
__device__ __forceinline__ const float* bias_lds(float* __restrict__ bl, const float* __restrict__ fb_b1)
{
    for (int t = (int)threadIdx.x; t < kBiasF; t += (int)blockDim.x) bl[t] = fb_b1[t];
    return bl;
}


__device__ __forceinline__ void tanh_h1(const f16v (&acc)[kMT], const float* __restrict__ b1p, int h,
                                        bf8 (&h1)[kMT][2])
{
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt) {
        float b[16];
        load16(b1p + (mt * 2 + h) * 16, b);
#pragma unroll
        for (int i = 0; i < 16; ++i) h1[mt][i >> 3][i & 7] = (__bf16)tanh_pre(acc[mt][i], b[i]);
    }
}

// layer 1, x fragments already in registers (KS k-steps, KS <= kKc): one W1
// stage, 8 M-tile accumulators, then bias + tanh into the bf16 operand
// fragments h1[mt][s].  Every wave of the block calls it (barriers); `on` =
// the wave has rows.
template <int KS, class STG>
__device__ __forceinline__ void layer1_reg(STG& S, const bf8* __restrict__ W,
                                           const float* __restrict__ b1p, int l, bool on, const bf8 (&x)[KS],
                                           bf8 (&h1)[kMT][2])
{
    const int h = l >> 5;
    f16v acc[kMT];
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt) acc[mt] = f16v{};
#pragma unroll
    for (int k0 = 0; k0 < KS; k0 += kKc) {
        const int kn = KS - k0 < kKc ? KS - k0 : kKc;
        const bf8* wl = S(W + k0 * kMT * 64, kn * kMT * 64);
        if (on) {
#pragma unroll
            for (int ks = k0; ks < k0 + kn; ++ks) {
                const bf8* w = wl + (ks - k0) * kMT * 64 + l;
#pragma unroll
                for (int mt = 0; mt < kMT; ++mt) acc[mt] = mfma(w[mt * 64], x[ks], acc[mt]);
            }
        }
    }
    tanh_h1(acc, b1p, h, h1);
}

// layer 1 for any obs_dim: W1 staged through LDS in chunks of kKc k-steps, x
// fragments loaded per k-step by xf(ks)
template <class XF, class STG>
__device__ __forceinline__ void layer1(STG& S, const bf8* __restrict__ W, const float* __restrict__ b1p,
                                       int ks1, int l, bool on, XF xf, bf8 (&h1)[kMT][2])
{
    f16v acc[kMT];
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt) acc[mt] = f16v{};
    for (int k0 = 0; k0 < ks1; k0 += kKc) {
        const int kn = ks1 - k0 < kKc ? ks1 - k0 : kKc;
        const bf8* wl = S(W + (int64_t)k0 * kMT * 64, kn * kMT * 64);
        if (on) {
#pragma unroll 2
            for (int ks = 0; ks < kn; ++ks) {
                const bf8 x = xf(k0 + ks);
                const bf8* w = wl + ks * kMT * 64 + l;
#pragma unroll
                for (int mt = 0; mt < kMT; ++mt) acc[mt] = mfma(w[mt * 64], x, acc[mt]);
            }
        }
    }
    tanh_h1(acc, b1p, l >> 5, h1);
}

// layer 2 (by output M-tile) fused with layer 3, in two LDS half stages;
// h2 kept when KEEP.  Every wave of the block calls it (barriers).
template <bool KEEP, class STG>
__device__ __forceinline__ f16v layers23(STG& S, const bf8* __restrict__ W23,
                                         const float* __restrict__ b2p, int l, bool on, const bf8 (&h1)[kMT][2],
                                         bf8 (&h2)[kMT][2])
{
    const int h = l >> 5;
    f16v z3 = f16v{};
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        const bf8* wl = S(W23 + hf * kHalf * 64, kHalf * 64);
        if (!on) continue;
#pragma unroll
        for (int q = 0; q < kMT / 2; ++q) {
            const int mo = kMT / 2 * hf + q;
            f16v a = f16v{};
            const bf8* w = wl + q * 16 * 64 + l;
            iglp();
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) a = mfma(w[kk * 64], h1[kk >> 1][kk & 1], a);
            float b[16];
            load16(b2p + (mo * 2 + h) * 16, b);
            bf8 f[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) f[i >> 3][i & 7] = (__bf16)tanh_pre(a[i], b[i]);
            const bf8* w3 = wl + (kMT / 2 * 16 + 2 * q) * 64 + l;
            z3 = mfma(w3[0], f[0], z3);
            z3 = mfma(w3[64], f[1], z3);
            if (KEEP) {
                h2[mo][0] = f[0];
                h2[mo][1] = f[1];
            }
        }
    }
    return z3;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

constexpr int kHeadN[6] = {3, 3, 3, 2, 2, 2};
constexpr int kHeadOff[6] = {0, 3, 6, 9, 11, 13};

// The heads' Gumbel-max sampling on both half-waves (the default; the
// environment's MAS_ACT_SPLIT=0, read per call, selects the one-half loop): lane
// half 0 holds the rows' 16 outputs (layer 3's padded C tile); lane l + 32
// takes a copy of lane l's and samples heads 2, 4, 5 while lane l samples
// heads 0, 1, 3 -- in three slots of equal shape: (0 | 2), (1 | 4, its third
// logit -inf: it adds nothing to the max, +0 to the exp sum and never wins),
// (3 | 5) -- so the wave issues the sampling instructions of three heads
// instead of six.  Each head's max, log-sum-exp, draws (mix64(base + 4 hd +
// k)) and choice are the same operations on the same values as the one-half
// loop of k_policy_act, and lane l adds the six heads' terms to the log-prob
// in head order: the same bits.
__device__ __forceinline__ void act_sample_split(const f16v& z3, const float* __restrict__ b3, int l, bool ok,
                                                 int64_t row, uint64_t seed, uint64_t step, int64_t first_row,
                                                 int8_t* __restrict__ act, float* __restrict__ logp,
                                                 float* __restrict__ value)
{
    const bool hi = l >= 32;
    float z[kO];
#pragma unroll
    for (int o = 0; o < kO; ++o) z[o] = __shfl(z3[o], l & 31, 64) + b3[o];
    const uint64_t base = mix64(seed ^ mix64(step * 0x100000001B3ULL + (uint64_t)(first_row + row)));
    constexpr int kA[3] = {0, 1, 3}, kB[3] = {2, 4, 5};
    float t[3];
    int bst[3];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
        const int hd = hi ? kB[sl] : kA[sl];
        const int offA = kHeadOff[kA[sl]], offB = kHeadOff[kB[sl]];
        constexpr int nn = 3;
        float zz[nn];
#pragma unroll
        for (int k = 0; k < nn; ++k) {
            const float za = k < kHeadN[kA[sl]] ? z[offA + k] : -INFINITY;
            const float zb = k < kHeadN[kB[sl]] ? z[offB + k] : -INFINITY;
            zz[k] = hi ? zb : za;
        }
        const int n = hi ? kHeadN[kB[sl]] : kHeadN[kA[sl]];
        float mx = zz[0];
#pragma unroll
        for (int k = 1; k < nn; ++k)
            if (k < kHeadN[kA[sl]] || k < kHeadN[kB[sl]]) mx = k < n ? fmaxf(mx, zz[k]) : mx;
        float se = 0.0f;
#pragma unroll
        for (int k = 0; k < nn; ++k)
            if (k < kHeadN[kA[sl]] || k < kHeadN[kB[sl]]) se = k < n ? se + exp_fast(zz[k] - mx) : se;
        const float lse = mx + log_fast(se);
        int best = 0;
        float bv = -INFINITY, lb = zz[0];
#pragma unroll
        for (int k = 0; k < nn; ++k) {
            if (!(k < kHeadN[kA[sl]] || k < kHeadN[kB[sl]])) continue;
            const uint64_t r = mix64(base + (uint64_t)(hd * 4 + k));
            const float u = ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);
            const float g = zz[k] - log_fast(-log_fast(u));
            if (k < n && g > bv) {
                bv = g;
                best = k;
                lb = zz[k];
            }
        }
        t[sl] = lb - lse;
        bst[sl] = best;
    }
    // lane l gathers heads 2, 4, 5 from lane l + 32 (every lane takes part)
    const int src = (l & 31) + 32;
    const float t2 = __shfl(t[0], src, 64), t4 = __shfl(t[1], src, 64), t5 = __shfl(t[2], src, 64);
    const int bp = __shfl(bst[0] | (bst[1] << 8) | (bst[2] << 16), src, 64);
    if (hi || !ok) return;
    float lp = 0.0f;
    lp += t[0];
    lp += t[1];
    lp += t2;
    lp += t[2];
    lp += t4;
    lp += t5;
    const uint32_t pa0 = (uint32_t)bst[0] | ((uint32_t)bst[1] << 8) | ((uint32_t)(bp & 0xff) << 16) |
                         ((uint32_t)bst[2] << 24);
    const uint32_t pa1 = (uint32_t)((bp >> 8) & 0xff) | ((uint32_t)((bp >> 16) & 0xff) << 8);
    uint16_t* ap = reinterpret_cast<uint16_t*>(act + row * 6);
    ap[0] = (uint16_t)pa0;
    ap[1] = (uint16_t)(pa0 >> 16);
    ap[2] = (uint16_t)pa1;
    logp[row] = lp;
    value[row] = z[kO - 1];
}

// KS > 0: compile-time k-step count (obs_dim in (16 (KS-1), 16 KS]) with every
// x fragment loaded up front; KS == 0: any obs_dim, chunked layer 1.
// XIN: the input rows are bf16 rows xb [M][xb_stride] already (mas_step_x
// wrote them; columns past obs_dim hold the bias column and zeros, which meet
// W1's zero padding), read instead of fp32 obs and not written back
template <int KS, bool XIN, bool SPLIT = true>
__global__ __launch_bounds__(64 * kWaves, MAS_POL_OCC_ACT * 4 / kWaves) void k_policy_act(const uint8_t* __restrict__ packed, int D, int ks1,
                                                             int64_t M, const float* __restrict__ obs,
                                                             __bf16* __restrict__ xb, int64_t xb_stride,
                                                             uint64_t seed, uint64_t step, int64_t first_row,
                                                             int8_t* __restrict__ act, float* __restrict__ logp,
                                                             float* __restrict__ value)
{
    __shared__ bf8 wl[kLdsFrag];
    Stage1 S{wl};
    const Layout Lo{ks1};
    const bf8* F = reinterpret_cast<const bf8*>(packed);
    const float* FB = reinterpret_cast<const float*>(packed);
#if MAS_POL_LDSB
    __shared__ float bl[kBiasF];
    const float* B1 = bias_lds(bl, FB + Lo.b1());
#else
    const float* B1 = FB + Lo.b1();
#endif
    const int l = threadIdx.x & 63, h = l >> 5;
    const int64_t row0 = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * 32;
    const bool on = row0 < M;  // wave-uniform
    const int64_t row = row0 + (l & 31);
    const bool ok = row < M;
    bf8 h1[kMT][2], h2[kMT][2];
    if constexpr (XIN) {
        // bf16 rows: 16-B loads of the lane's 8 columns per k-step, an
        // out-of-range lane's row clamped into range and zeroed
        const int64_t rr = ok ? row : M - 1;
        const __bf16* xr = xb + rr * xb_stride + 8 * h;
        if constexpr (KS > 0) {
            bf8 x[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf8 v = *reinterpret_cast<const bf8*>(xr + 16 * ks);
                x[ks] = ok ? v : bf8{};
            }
            layer1_reg<KS>(S, F + Lo.w1(), B1, l, on, x, h1);
        } else {
            layer1(S, F + Lo.w1(), B1, ks1, l, on,
                   [&](int ks) {
                       const bf8 v = *reinterpret_cast<const bf8*>(xr + 16 * ks);
                       return ok ? v : bf8{};
                   },
                   h1);
        }
    } else if constexpr (KS > 0) {
        bf8 x[KS];
        if ((D & 3) == 0 && D == 16 * KS) {  // every k-step complete: branch-free loads
            const int64_t rr = ok ? row : M - 1;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) x[ks] = x_frag_f32_full(obs, rr, ok, D, 16 * ks + 8 * h);
        } else {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) x[ks] = x_frag_f32(obs, row, ok, D, 16 * ks + 8 * h);
        }
        if (xb != nullptr && ok) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<bf8*>(xb + row * xb_stride + 16 * ks + 8 * h) = x[ks];
        }
        layer1_reg<KS>(S, F + Lo.w1(), B1, l, on, x, h1);
    } else {
        layer1(S, F + Lo.w1(), B1, ks1, l, on,
               [&](int ks) {
                   const bf8 x = x_frag_f32(obs, row, ok, D, 16 * ks + 8 * h);
                   if (xb != nullptr && ok) *reinterpret_cast<bf8*>(xb + row * xb_stride + 16 * ks + 8 * h) = x;
                   return x;
               },
               h1);
    }
    const f16v z3 = layers23<false>(S, F + Lo.w23(), B1 + kMT * 2 * 16, l, on, h1, h2);  // last barrier
    if (!on) return;
    if constexpr (SPLIT) {
        if (!(MAS_POL_EXP & 2)) {
            act_sample_split(z3, B1 + 2 * kMT * 2 * 16, l, ok, row, seed, step, first_row, act, logp, value);
            return;
        }
    }
    if (h != 0 || !ok) return;
    if (MAS_POL_EXP & 2) {
        value[row] = z3[0] + z3[15];
        return;
    }
    float z[kO];
    const float* b3 = B1 + 2 * kMT * 2 * 16;
#pragma unroll
    for (int o = 0; o < kO; ++o) z[o] = z3[o] + b3[o];
    // Gumbel-max over each head; the RNG stream of k_sample (mas_capi.hip),
    // hardware exp2/log2 (the draws agree with k_sample up to ~1 ulp ties)
    // (keyed by the row's index in the whole batch: a shard launched with its
    // first_row draws what the unsharded launch draws for those rows)
    const uint64_t base = mix64(seed ^ mix64(step * 0x100000001B3ULL + (uint64_t)(first_row + row)));
    float lp = 0.0f;
    uint32_t packed_a[2] = {0u, 0u};
#pragma unroll
    for (int hd = 0; hd < 6; ++hd) {
        const int n = kHeadN[hd], off = kHeadOff[hd];
        float mx = z[off];
#pragma unroll
        for (int k = 1; k < n; ++k) mx = fmaxf(mx, z[off + k]);
        float se = 0.0f;
#pragma unroll
        for (int k = 0; k < n; ++k) se += exp_fast(z[off + k] - mx);
        const float lse = mx + log_fast(se);
        int best = 0;
        float bv = -INFINITY, lb = z[off];
#pragma unroll
        for (int k = 0; k < n; ++k) {
            const uint64_t r = mix64(base + (uint64_t)(hd * 4 + k));
            const float u = ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);
            const float g = z[off + k] - log_fast(-log_fast(u));
            if (g > bv) {
                bv = g;
                best = k;
                lb = z[off + k];
            }
        }
        lp += lb - lse;
        packed_a[hd >> 2] |= (uint32_t)best << (8 * (hd & 3));
    }
    // 6 int8 per row (2-B aligned): three 2-B stores
    uint16_t* ap = reinterpret_cast<uint16_t*>(act + row * 6);
    ap[0] = (uint16_t)packed_a[0];
    ap[1] = (uint16_t)(packed_a[0] >> 16);
    ap[2] = (uint16_t)packed_a[1];
    logp[row] = lp;
    value[row] = z[kO - 1];
}

struct TrainArgs {
    const uint8_t* packed;
    int ks1;
    int64_t M;              // rows of this minibatch
    const __bf16* xb;       // [M][xb_stride] bf16
    int64_t xb_stride;
    const int8_t* act;      // [M][6]
    const float* old_logp;  // [M]
    const float* adv;       // [M] (normalised)
    const float* ret;       // [M]
    float clip, vf_coef, ent_coef, scale;  // scale = 1 / rows of the minibatch
    __bf16 *h1, *h2, *da1, *da2, *dz;      // feature-major [256 | 16][ld], or row-major (RM)
    int64_t ld;             // feature-major: their row stride (>= M; a power of two costs HBM bandwidth);
                            // RM: the row stride of h1 / h2 (>= 257: column 256 holds the ones)
    float* partials;        // [gridDim.x][4]: sum pg, sum (v-ret)^2, sum entropy, clipped count
};

// Feature-major activation store of one 32-row M-tile fragment (16 features
// crow(i, h) of 32*mt.. for this lane's row).  Lanes l and l^1 hold rows r and
// r^1 of the same features: one DPP swap per feature pair lets each lane write
// two consecutive rows of one feature as a 4-B word (half the store
// instructions of 2-B stores, full 128-B segments per wave half).  Needs M even
// (then both rows of a pair are in range or neither is).
// MAS_POL_PAIR: rows per lane of the feature-major stores when M allows (1, 2, 4)
#ifndef MAS_POL_PAIR
#define MAS_POL_PAIR 2
#endif
// waves per SIMD of the train kernel (A/B: 1 = 512 registers, no spills)
#ifndef MAS_POL_OCC
#define MAS_POL_OCC 2
#endif
// feature-major activation buffers of at most 2^32 bytes (257 rows of ld
// bf16): the store offsets fit in 32 bits
constexpr int64_t kOff32Ld = ((int64_t)1 << 32) / (2 * 257);
template <bool OFF32>
__device__ __forceinline__ void store_rows2(__bf16* base, int64_t M, int64_t row, int mt, int h, const bf8 (&v)[2])
{
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const bool odd = row & 1;
    // feature crow(2j + odd, h) = K(j) + odd + 4 h with K(j) = 2 (j & 1) + 8 (j >> 1).
    // OFF32: the lane's byte offset (feature odd + 4 h, column row & ~1) plus
    // the wave-uniform K rows of M (a scalar multiply), from the buffer base:
    // one vector add per store instead of a 64-bit multiply-add
    uint32_t* dst = reinterpret_cast<uint32_t*>(base + (row & ~(int64_t)1));
    const uint32_t m2 = OFF32 ? __builtin_amdgcn_readfirstlane((uint32_t)(M * 2)) : 0u;
    const uint32_t lane_off = OFF32 ? ((uint32_t)((int)odd + 4 * h) * m2 + (uint32_t)(row & ~(int64_t)1) * 2u) : 0u;
    const u4 w[2] = {__builtin_bit_cast(u4, v[0]), __builtin_bit_cast(u4, v[1])};
    // byte selectors of v_perm_b32 over {partner word, own word} (own bytes
    // 0-3, partner's 4-7): even row: own feature 2j, then the partner's
    // (row + 1); odd row: the partner's feature 2j + 1 (row - 1), then its own
    const uint32_t psel = odd ? 0x03020706u : 0x05040100u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        // features 2j (low half) and 2j + 1 (high half) of this lane's row;
        // quad_perm [1, 0, 3, 2]: lane l reads lane l ^ 1's whole word
        const uint32_t own = w[j >> 2][j & 3];
        const uint32_t par = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0xB1, 0xF, 0xF, false);
        const uint32_t word = __builtin_amdgcn_perm(par, own, psel);
        if (OFF32) {
            const uint32_t K = (uint32_t)(32 * mt + 2 * (j & 1) + 8 * (j >> 1));
            *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(base) + (lane_off + K * m2)) = word;
        } else {
            const int64_t f = 32 * mt + crow(odd ? 2 * j + 1 : 2 * j, h);
            dst[(f * M) >> 1] = word;
        }
    }
}

// Same with four consecutive rows per lane (8-B stores): a 4 x 4 transpose of
// bf16 within each lane quad (rows r..r+3 x features crow(4g..4g+3)) in two
// DPP exchanges, after which lane q of the quad holds feature 4g + q of all
// four rows.  Needs M % 4 == 0.
__device__ __forceinline__ void store_rows4(__bf16* base, int64_t M, int64_t row, int mt, int h, const bf8 (&v)[2])
{
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int q = (int)(row & 3);
    const bool hi = q & 2, odd = q & 1;
    const u4 w[2] = {__builtin_bit_cast(u4, v[0]), __builtin_bit_cast(u4, v[1])};
    uint2* dst = reinterpret_cast<uint2*>(base + (row & ~(int64_t)3));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const uint32_t W0 = w[g >> 1][2 * (g & 1)], W1 = w[g >> 1][2 * (g & 1) + 1];  // features 4g+0,1 / 4g+2,3
        // quad_perm [2, 3, 0, 1]: rows q and q ^ 2 trade the feature pair the other keeps
        const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(hi ? W0 : W1), 0x4E, 0xF, 0xF, false);
        const uint32_t X = hi ? r1 : W0, Y = hi ? W1 : r1;  // rows (q & 1), (q & 1) + 2 of feature pair (q & 2)
        const uint32_t s2 = odd ? ((X & 0xffffu) | (Y << 16)) : ((X >> 16) | (Y & 0xffff0000u));
        // quad_perm [1, 0, 3, 2]: rows q and q ^ 1 trade halves
        const uint32_t r2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0xB1, 0xF, 0xF, false);
        uint2 o;
        if (odd) {
            o.x = (r2 & 0xffffu) | (X & 0xffff0000u);
            o.y = (r2 >> 16) | (Y & 0xffff0000u);
        } else {
            o.x = (X & 0xffffu) | (r2 << 16);
            o.y = (Y & 0xffffu) | (r2 & 0xffff0000u);
        }
        const int64_t f = 32 * mt + 8 * g + 4 * h + q;  // crow(4g + q, h)
        dst[(f * M) >> 2] = o;
    }
}

// Row-major activation store (RM): lane (row, h) writes its M-tile fragment as
// two 16-B chunks of its own row, at columns 32 mt + 8 h (registers 0..7) and
// 32 mt + 16 + 8 h (registers 8..15).  No lane exchange: stored column
// 32 mt + 16 c + 8 h + j holds feature 32 mt + crow(8 c + j, h) (rm_feature);
// the weight-gradient GEMMs sum over rows, so the host un-permutes their
// [256 x G] results instead of the activations.
__host__ __device__ inline int rm_feature(int col)
{
    const int t = col & 31;
    return (col & ~31) + crow(8 * (t >> 4) + (t & 7), (t >> 3) & 1);
}
__device__ __forceinline__ void store_rm(__bf16* base, int64_t ldr, int64_t row, int mt, int h, const bf8 (&v)[2])
{
    bf8* p = reinterpret_cast<bf8*>(base + row * ldr + 32 * mt + 8 * h);
    p[0] = v[0];
    p[2] = v[1];
}

template <int KS, bool OFF32, bool RM>
__global__ __launch_bounds__(64 * kTWaves, MAS_POL_OCC * 4 / kTWaves) void k_policy_train(TrainArgs A)
{
    const Layout Lo{A.ks1};
    const bf8* F = reinterpret_cast<const bf8*>(A.packed);
    const float* FB = reinterpret_cast<const float*>(A.packed);
    __shared__ bf8 wl[kLdsFrag];
    Stage1 S{wl};
    const int l = threadIdx.x & 63, h = l >> 5, wv = threadIdx.x >> 6;
    const int64_t M = A.M, LD = A.ld;
    const int64_t row0 = ((int64_t)blockIdx.x * kTWaves + wv) * 32;
    const int64_t row = row0 + (l & 31);
    const bool ok = row < M;
    float st[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool on = row0 < M;  // wave-uniform
    {
        bf8 h1[kMT][2], h2[kMT][2];
        // branch-free: an out-of-range lane reads the last row (its results are never stored)
        const int64_t rr = ok ? row : M - 1;
        auto xf = [&](int ks) { return *reinterpret_cast<const bf8*>(A.xb + rr * A.xb_stride + 16 * ks + 8 * h); };
        if constexpr (KS > 0) {
            bf8 x[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) x[ks] = xf(ks);
            layer1_reg<KS>(S, F + Lo.w1(), FB + Lo.b1(), l, on, x, h1);
        } else {
            layer1(S, F + Lo.w1(), FB + Lo.b1(), A.ks1, l, on, xf, h1);
        }
        const f16v z3 = layers23<true>(S, F + Lo.w23(), FB + Lo.b2(), l, on, h1, h2);
        const bf8* wb = S(F + Lo.wbk(), kBk0 * 64);  // W3^T
        // feature-major activations for the weight gradients
        // wave-uniform store mode: 4 rows per lane (M % 4 == 0), 2 rows (M even), 1 row
        const int rows_per_lane = !MAS_POL_PAIR ? 1 : ((M | LD) & 3) == 0 ? MAS_POL_PAIR : ((M | LD) & 1) == 0 ? 2 : 1;
        const bool pair = rows_per_lane > 1;
        auto store_rows = [&](__bf16* base, int t, const bf8 (&v)[2]) {
            if (RM) store_rm(base, base == A.h1 || base == A.h2 ? LD : kH, row, t, h, v);
            else if (rows_per_lane == 4) store_rows4(base, LD, row, t, h, v);
            else store_rows2<OFF32>(base, LD, row, t, h, v);
        };
        if (on && ok) {
            if (RM || pair) {
#pragma unroll
                for (int mt = 0; mt < kMT; ++mt) {
                    store_rows(A.h1, mt, h1[mt]);
                    store_rows(A.h2, mt, h2[mt]);
                }
            } else {
#pragma unroll
                for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int64_t f = 32 * mt + crow(i, h);
                        A.h1[f * LD + row] = h1[mt][i >> 3][i & 7];
                        A.h2[f * LD + row] = h2[mt][i >> 3][i & 7];
                    }
            }
        }
        // PPO loss gradient of this row (lane half 0 holds the 16 outputs)
        float dz[kO];
#pragma unroll
        for (int o = 0; o < kO; ++o) dz[o] = 0.0f;
        if (on && h == 0 && ok) {
            float z[kO];
            const float* b3 = FB + Lo.b3();
#pragma unroll
            for (int o = 0; o < kO; ++o) z[o] = z3[o] + b3[o];
            const int8_t* a = A.act + row * 6;
            float lsm[15], p[15], hent[6];
            float lp = 0.0f, ent = 0.0f;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                float mx = z[off];
#pragma unroll
                for (int k = 1; k < n; ++k) mx = fmaxf(mx, z[off + k]);
                float se = 0.0f;
#pragma unroll
                for (int k = 0; k < n; ++k) se += exp_fast(z[off + k] - mx);
                const float lse = mx + log_fast(se);
                float e = 0.0f;
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    lsm[off + k] = z[off + k] - lse;
                    p[off + k] = exp_fast(lsm[off + k]);
                    e -= p[off + k] * lsm[off + k];
                    if (k == ak) lp += lsm[off + k];
                }
                hent[hd] = e;
                ent += e;
            }
            const float adv = A.adv[row];
            const float ratio = exp_fast(lp - A.old_logp[row]);
            const float s1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.0f - A.clip), 1.0f + A.clip);
            const float s2 = rc * adv;
            // d(-min(s1, s2))/d lp: the surrogate is differentiable through
            // s1 where it is the minimum (ties included: then s1 == s2 with
            // the ratio inside the clip range)
            const float glp = s1 <= s2 ? -s1 : 0.0f;
            const float sc = A.scale;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const float oh = k == ak ? 1.0f : 0.0f;
                    dz[off + k] = sc * (glp * (oh - p[off + k]) + A.ent_coef * p[off + k] * (lsm[off + k] + hent[hd]));
                }
            }
            const float dv = z[kO - 1] - A.ret[row];
            dz[kO - 1] = sc * A.vf_coef * 2.0f * dv;
            st[0] = -fminf(s1, s2);
            st[1] = dv * dv;
            st[2] = ent;
            st[3] = fabsf(ratio - 1.0f) > A.clip ? 1.0f : 0.0f;
            if (!RM) {
#pragma unroll
                for (int o = 0; o < kO; ++o) A.dz[(int64_t)o * LD + row] = (__bf16)dz[o];
            }
        }
        bf8 dzf[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) dzf[i >> 3][i & 7] = (__bf16)dz[i];
        if (RM && on && h == 0 && ok) {  // dz row-major [M][16], natural output order
            bf8* pz = reinterpret_cast<bf8*>(A.dz + row * kO);
            pz[0] = dzf[0];
            pz[1] = dzf[1];
        }
        // dA2 = (W3^T dz) * (1 - h2^2), by M-tile of layer 2
        bf8 da2[kMT][2];
        const bf8* W3T = wb + l;
#pragma unroll
        for (int mo = 0; mo < kMT; ++mo) {
            f16v g = f16v{};
            g = mfma(W3T[(mo * 2) * 64], dzf[0], g);
            g = mfma(W3T[(mo * 2 + 1) * 64], dzf[1], g);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float hv = (float)h2[mo][i >> 3][i & 7];
                da2[mo][i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
            }
            if (ok) {
                if (RM || pair) {
                    store_rows(A.da2, mo, da2[mo]);
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) A.da2[(int64_t)(32 * mo + crow(i, h)) * LD + row] = da2[mo][i >> 3][i & 7];
                }
            }
        }
        // dA1 = (W2^T dA2) * (1 - h1^2), by M-tile of layer 1
        const bf8* W2T = wb + l;
#pragma unroll
        for (int mt = 0; mt < kMT; ++mt) {
            if (mt % (kMT / 2) == 0)  // W2^T M-tiles 0..3, then 4..7
                W2T = S(F + Lo.wbk() + (kBk0 + (mt / (kMT / 2)) * kBk1) * 64, kBk1 * 64) + l;
            f16v g = f16v{};
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) g = mfma(W2T[((mt % (kMT / 2)) * 16 + kk) * 64], da2[kk >> 1][kk & 1], g);
            if (ok) {
                bf8 d1[2];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float hv = (float)h1[mt][i >> 3][i & 7];
                    d1[i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
                }
                if (RM || pair) {
                    store_rows(A.da1, mt, d1);
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) A.da1[(int64_t)(32 * mt + crow(i, h)) * LD + row] = d1[i >> 3][i & 7];
                }
            }
        }
    }
    // per-block loss partials (through the LDS stage, after its last reader)
    __syncthreads();
    float* red = reinterpret_cast<float*>(wl);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float v = st[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (l == 0) red[wv * 4 + k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < kTWaves; ++w) v += red[w * 4 + threadIdx.x];
        A.partials[(int64_t)blockIdx.x * 4 + threadIdx.x] = v;
    }
}


// ---------------------------------------------------------------------------
// k_policy_train_cw: k_policy_train's feature-major pair-store path (the PPO
// update's: M and ld even, not row-major) with the activation stores moved
// off the weight-stage drains.  vmcnt counts loads, stores and LDS-DMA
// together in issue order, so stage()'s wait for the stage's LDS-DMA copies
// (s_waitcnt 0) also waited for every activation store the wave had issued
// before them: each of the six stage boundaries of a block drained the
// block's stores with the wave parked at the barrier.  Here each boundary
// issues the next stage's copies first and only then the stores of values
// the previous phase finished (kept in registers until then: h1, h2, dA2,
// half of dA1), and waits with vmcnt(n) for n <= the stores issued after the
// copies -- the copies are older than those stores, so they have landed --
// leaving the stores in flight through the next phase's MFMAs.  Same values,
// same addresses: only the issue order of the stores moves.
// ---------------------------------------------------------------------------
// dA2 M-tiles stored behind the first W2^T copies (8 stores each; more than
// two spill: the scheduler hoists the stage's LDS reads above the stores)
#ifndef MAS_POL_CW_DEFER
#define MAS_POL_CW_DEFER 3
#endif
// dA1 M-tiles of the first W2^T half stored behind the second half's copies
#ifndef MAS_POL_CW_DEFER1
#define MAS_POL_CW_DEFER1 3
#endif
// a bare workgroup barrier: __syncthreads()'s workgroup-scope fences (even
// restricted to LDS: the LDS-DMA copies are LDS writes counted by vmcnt) make
// the compiler wait vmcnt(0) for the wave's outstanding stores -- the drain
// this kernel exists to avoid.  The ordering they gave is explicit here: the
// callers' s_waitcnt retires the wave's LDS traffic and copies, and the empty
// asm statements keep the compiler from moving memory accesses across.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_s_waitcnt((0x3F & 0xF) | ((0x3F >> 4) << 14) | (0x7 << 4) | (0 << 8));  // lgkmcnt(0)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// LDS-DMA copy of a stage of N fragments (no wait): stage() without its
// drain.  N is a multiple of the workgroup's 64 kWaves lanes, so every wave
// issues the same N / (64 kWaves) copies: no wave-dependent branch, which
// would give the compiler's wait-count analysis a path without copies
template <int N>
__device__ __forceinline__ void stage_copy(bf8* __restrict__ wl, const bf8* __restrict__ src)
{
    static_assert(N % (64 * kWaves) == 0 && N <= kLdsFrag, "whole copy rounds");
    lds_barrier();  // every wave is done with the previous stage
    const int w0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    const uint32_t loff = (threadIdx.x & 63) * 16u;
#pragma unroll
    for (int k = 0; k < N / (64 * kWaves); ++k) {
        const int i0 = w0 + k * 64 * kWaves;
        __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const uint8_t*>(src + i0) + loff),
                                         (lds_void*)(wl + i0), 16, 0, 0);
    }
}
// the stage's copies have landed once at most NST of the wave's vector memory
// operations are outstanding, NST <= the stores issued after the copies (a
// wave without rows issued none: it waits for everything)
template <int NST>
__device__ __forceinline__ void stage_landed(bool issued)
{
    static_assert(NST >= 0 && NST <= 63, "vmcnt is 6 bits");
    // gfx9 s_waitcnt: vmcnt [3:0] + [15:14], expcnt [6:4] and lgkmcnt [11:8] at their maximum (no wait)
    constexpr int imm = (NST & 0xF) | ((NST >> 4) << 14) | (0x7 << 4) | (0xF << 8);
    if (issued) __builtin_amdgcn_s_waitcnt(imm);
    else __builtin_amdgcn_s_waitcnt(0);
    lds_barrier();  // every wave's copies have landed
}

// one block's rows; FULL: every row of the block is in range (all blocks
// but the last), so no store sits under a branch -- a path that skips stores
// would leave the copies the newest operations and force vmcnt(0) waits
template <int KS, bool OFF32, bool FULL>
__device__ __forceinline__ void train_cw_block(const TrainArgs& A, bf8* wl, const float* B1, float (&st)[4])
{
    const Layout Lo{A.ks1};
    const bf8* F = reinterpret_cast<const bf8*>(A.packed);
    const float* FB = reinterpret_cast<const float*>(A.packed);
    Stage1 S{wl};
    const int l = threadIdx.x & 63, h = l >> 5, wv = threadIdx.x >> 6;
    const int64_t M = A.M, LD = A.ld;
    const int64_t row0 = ((int64_t)blockIdx.x * kTWaves + wv) * 32;
    const int64_t row = row0 + (l & 31);
    const bool ok = FULL || row < M;
    const bool on = FULL || row0 < M;  // wave-uniform: the wave has rows (its stores are issued)
    // (M even: both rows of a lane pair are in range or neither)
    {
        bf8 h1[kMT][2], h2[kMT][2];
        const int64_t rr = ok ? row : M - 1;
        auto xf = [&](int ks) { return *reinterpret_cast<const bf8*>(A.xb + rr * A.xb_stride + 16 * ks + 8 * h); };
        if constexpr (KS > 0) {
            bf8 x[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) x[ks] = xf(ks);
            layer1_reg<KS>(S, F + Lo.w1(), B1, l, on, x, h1);
        } else {
            layer1(S, F + Lo.w1(), B1, A.ks1, l, on, xf, h1);
        }
        auto st2 = [&](__bf16* base, int t, const bf8 (&v)[2]) {
            if (ok) store_rows2<OFF32>(base, LD, row, t, h, v);
        };
        const f16v z3 = layers23<true>(S, F + Lo.w23(), B1 + kMT * 2 * 16, l, on, h1, h2);
        // the loss inputs of this row, loaded ahead of the activation stores
        // (a load issued after them would wait for them: vmcnt is in order);
        // the output biases through the scalar cache
        const int64_t rl = ok ? row : M - 1;
        const uint16_t* ap = reinterpret_cast<const uint16_t*>(A.act + rl * 6);  // 2-byte aligned
        const uint32_t a01 = ap[0], a23 = ap[1], a45 = ap[2];
        const float adv = A.adv[rl], old_lp = A.old_logp[rl], ret = A.ret[rl];
        typedef const __attribute__((address_space(4))) float cfloat;
        const cfloat* b3 = (const cfloat*)(FB + Lo.b3());
        // W3^T; h1 and h2 go out behind its copies
        stage_copy<kBk0 * 64>(wl, F + Lo.wbk());
        if (on) {
#pragma unroll
            for (int mt = 0; mt < kMT; ++mt) {  // 128 stores
                st2(A.h1, mt, h1[mt]);
                st2(A.h2, mt, h2[mt]);
            }
        }
        stage_landed<63>(on);
        const bf8* wb = wl;
        // PPO loss gradient of this row (lane half 0 holds the 16 outputs)
        float dz[kO];
#pragma unroll
        for (int o = 0; o < kO; ++o) dz[o] = 0.0f;
        if (on && h == 0 && ok) {
            float z[kO];
#pragma unroll
            for (int o = 0; o < kO; ++o) z[o] = z3[o] + b3[o];
            int a[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) a[k] = (int)(int8_t)(((k < 2 ? a01 : k < 4 ? a23 : a45) >> (8 * (k & 1))) & 0xffu);
            float lsm[15], p[15], hent[6];
            float lp = 0.0f, ent = 0.0f;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                float mx = z[off];
#pragma unroll
                for (int k = 1; k < n; ++k) mx = fmaxf(mx, z[off + k]);
                float se = 0.0f;
#pragma unroll
                for (int k = 0; k < n; ++k) se += exp_fast(z[off + k] - mx);
                const float lse = mx + log_fast(se);
                float e = 0.0f;
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    lsm[off + k] = z[off + k] - lse;
                    p[off + k] = exp_fast(lsm[off + k]);
                    e -= p[off + k] * lsm[off + k];
                    if (k == ak) lp += lsm[off + k];
                }
                hent[hd] = e;
                ent += e;
            }
            const float ratio = exp_fast(lp - old_lp);
            const float s1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.0f - A.clip), 1.0f + A.clip);
            const float s2 = rc * adv;
            const float glp = s1 <= s2 ? -s1 : 0.0f;
            const float sc = A.scale;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const float oh = k == ak ? 1.0f : 0.0f;
                    dz[off + k] = sc * (glp * (oh - p[off + k]) + A.ent_coef * p[off + k] * (lsm[off + k] + hent[hd]));
                }
            }
            const float dv = z[kO - 1] - ret;
            dz[kO - 1] = sc * A.vf_coef * 2.0f * dv;
            st[0] = -fminf(s1, s2);
            st[1] = dv * dv;
            st[2] = ent;
            st[3] = fabsf(ratio - 1.0f) > A.clip ? 1.0f : 0.0f;
#pragma unroll
            for (int o = 0; o < kO; ++o) A.dz[(int64_t)o * LD + row] = (__bf16)dz[o];
        }
        bf8 dzf[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) dzf[i >> 3][i & 7] = (__bf16)dz[i];
        // dA2 = (W3^T dz) * (1 - h2^2), by M-tile of layer 2 (kept in registers)
        bf8 da2[kMT][2];
        const bf8* W3T = wb + l;
#pragma unroll
        for (int mo = 0; mo < kMT; ++mo) {
            f16v g = f16v{};
            g = mfma(W3T[(mo * 2) * 64], dzf[0], g);
            g = mfma(W3T[(mo * 2 + 1) * 64], dzf[1], g);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float hv = (float)h2[mo][i >> 3][i & 7];
                da2[mo][i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
            }
            if (on && mo < kMT - MAS_POL_CW_DEFER) st2(A.da2, mo, da2[mo]);
        }
        // dA1 = (W2^T dA2) * (1 - h1^2), by M-tile of layer 1, in two half
        // stages; dA2 goes out behind the first half's copies (dA1 is stored
        // as computed: holding tiles 0..3 for the second boundary would spill)
        const bf8* W2T = nullptr;
        bf8 d1k[kMT / 2][2];  // the deferred tiles (MAS_POL_CW_DEFER1 of them)
#pragma unroll
        for (int mt = 0; mt < kMT; ++mt) {
            if (mt == 0) {
                stage_copy<kBk1 * 64>(wl, F + Lo.wbk() + kBk0 * 64);
                if (on) {
#pragma unroll
                    for (int mo = kMT - MAS_POL_CW_DEFER; mo < kMT; ++mo) st2(A.da2, mo, da2[mo]);
                }
                stage_landed<8 * MAS_POL_CW_DEFER>(on);
                W2T = wl + l;
            } else if (mt == kMT / 2) {
                stage_copy<kBk1 * 64>(wl, F + Lo.wbk() + (kBk0 + kBk1) * 64);
                if (on) {
#pragma unroll
                    for (int q = kMT / 2 - MAS_POL_CW_DEFER1; q < kMT / 2; ++q) st2(A.da1, q, d1k[q]);
                }
                stage_landed<8 * MAS_POL_CW_DEFER1>(on);
                W2T = wl + l;
            }
            f16v g = f16v{};
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) g = mfma(W2T[((mt % (kMT / 2)) * 16 + kk) * 64], da2[kk >> 1][kk & 1], g);
            bf8 d1[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float hv = (float)h1[mt][i >> 3][i & 7];
                d1[i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
            }
            if (mt >= kMT / 2 - MAS_POL_CW_DEFER1 && mt < kMT / 2) {
                d1k[mt][0] = d1[0];
                d1k[mt][1] = d1[1];
            } else if (on) {
                st2(A.da1, mt, d1);
            }
        }
    }
}

template <int KS, bool OFF32>
__global__ __launch_bounds__(64 * kTWaves, MAS_POL_OCC * 4 / kTWaves) void k_policy_train_cw(TrainArgs A)
{
    __shared__ bf8 wl[kLdsFrag];
    const float* FB = reinterpret_cast<const float*>(A.packed);
#if MAS_POL_LDSB
    __shared__ float bl[kBiasF];
    const float* B1 = bias_lds(bl, FB + Layout{A.ks1}.b1());
#else
    const float* B1 = FB + Layout{A.ks1}.b1();
#endif
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float st[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if ((int64_t)(blockIdx.x + 1) * kTWaves * 32 <= A.M)  // block-uniform
        train_cw_block<KS, OFF32, true>(A, wl, B1, st);
    else
        train_cw_block<KS, OFF32, false>(A, wl, B1, st);

    // per-block loss partials (through the LDS stage, after its last reader)
    __syncthreads();
    float* red = reinterpret_cast<float*>(wl);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float v = st[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (l == 0) red[wv * 4 + k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < kTWaves; ++w) v += red[w * 4 + threadIdx.x];
        A.partials[(int64_t)blockIdx.x * 4 + threadIdx.x] = v;
    }
}

// ---------------------------------------------------------------------------
// k_policy_train_db: the PPO update's train kernel as one persistent
// 8-wave workgroup per CU with DOUBLE-BUFFERED weight stages (2 x 72 KiB of
// the CU's 160 KiB LDS).  k_policy_train runs two 4-wave workgroups per CU on
// one 72-KiB stage each: every stage boundary (7 per 128-row block) drains
// the stage's LDS-DMA copies -- and, vmcnt being in issue order, every
// activation store before them -- with the waves parked at the barrier, and
// hopes the other workgroup computes meanwhile.  Here a boundary waits only
// for copies issued a whole phase earlier: phase p starts by issuing the
// copies of stage p + 1 into the other buffer (all waves are past phase p - 1,
// the buffer's last reader), then the stores of activations finished earlier,
// then computes from buffer p; the landing of stage p + 1 waits with
// vmcnt(n), n the wave's vector memory operations issued after those copies
// (counted per phase below, capped at 63: the counter saturates, so 63
// outstanding implies every older operation done).  8 waves share each
// stage: 256 rows per weight pass instead of 128.  Full 256-row blocks only
// (straight-line stores, exact counts); the partial last block goes to
// k_policy_train (policy_train).  Same operations in the same order per row:
// bit-identical to k_policy_train (test_counted_wait_train_kernel_is_bit_identical).
// ---------------------------------------------------------------------------
#ifndef MAS_POL_DB_SB
#define MAS_POL_DB_SB 1
#endif
constexpr int kDW = 8;                  // waves per workgroup
constexpr int kDRows = 32 * kDW;        // rows per block
constexpr int kDCopy = 64 * kDW;        // fragments one copy round moves (one per thread)
static_assert(kLdsFrag % kDCopy == 0 && (kBk0 * 64) % kDCopy == 0 && (kBk1 * 64) % kDCopy == 0, "copy rounds");

// LDS-DMA copy of n fragments (n a multiple of kDCopy, wave-uniform), no
// wait.  Written as inline asm (global_load_lds_dwordx4 with the wave's
// global base in SGPRs, the lane's 16-B offset in one VGPR, the LDS base in
// m0): with the builtin, the compiler's wait-count pass cannot tell the next
// stage's buffer from the current one and waits for these copies (vmcnt(0),
// every store before them included) at the phase's first LDS read -- the
// serialisation this kernel removes.  Invisible to that pass, the copies are
// ordered only by land_db's explicit counts; the pass's own waits for other
// loads can only over-wait (it does not count these).  The LDS base goes in
// as an m0 operand ("{m0}"): the compiler sets m0 itself and knows it is
// used (a clobber of the reserved m0 is not honoured).
__device__ __forceinline__ void copy_db(bf8* __restrict__ buf, const bf8* __restrict__ src, int n)
{
    const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    const uint32_t loff = (threadIdx.x & 63) * 16u;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(buf) + w0 * 16u;  // LDS byte offset
    const uint8_t* g0 = reinterpret_cast<const uint8_t*>(src) + w0 * 16u;
    for (int k = 0; k < n; k += kDCopy) {
        const uint32_t m0v = lds0 + (uint32_t)k * 16u;
        const uint8_t* gk = g0 + (int64_t)k * 16;
        asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(loff), "s"(gk), "{m0}"(m0v) : "memory");
    }
}
// the stage copied one phase ago has landed in every wave: NST = this wave's
// vector memory operations issued after those copies (a lower bound)
// (the s_movk_i32 of 0x7a00 + NST into a dead SGPR marks the wait in the ISA:
// scripts/check_policy_waits.py, run by __graft_entry__.build(), checks that
// at least min(NST, 63) vector memory instructions follow the last copy
// before every marker -- a count above the real one would stop waiting
// before the copies land)
template <int NST>
__device__ __forceinline__ void land_db()
{
    constexpr int n = NST > 63 ? 63 : NST;
    int mark;
    asm volatile("s_movk_i32 %0, %1" : "=s"(mark) : "n"(0x7a00 + n));
    __builtin_amdgcn_s_waitcnt((n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    lds_barrier();
}

template <int KS, bool OFF32>
__global__ __launch_bounds__(64 * kDW, 1) void k_policy_train_db(TrainArgs A, int64_t nblk)
{
    static_assert(KS > 0, "compile-time layer-1 depth");
    constexpr int NCH = (KS + kKc - 1) / kKc;  // layer-1 stages
    __shared__ bf8 wl[2 * kLdsFrag];
    __shared__ float bl[kBiasF];
    __shared__ float red[kDW * 4];
    const Layout Lo{A.ks1};
    const bf8* F = reinterpret_cast<const bf8*>(A.packed);
    const float* FB = reinterpret_cast<const float*>(A.packed);
    bias_lds(bl, FB + Lo.b1());
    const float* b1p = bl;
    const float* b2p = bl + kMT * 2 * 16;
    const float* b3 = bl + 2 * kMT * 2 * 16;
    const int l0 = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t LD = A.ld;
    float st[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int sc = 0;  // stages so far: the current one is in buffer sc & 1
    auto buf = [&](int k) { return wl + (k & 1) * kLdsFrag; };
    // (each tile's 8 stores fenced off from the scheduler: a burst of
    // interleaved tiles' pair shuffles would spill)
    auto st2 = [&](__bf16* base, int64_t row, int t, int h, const bf8 (&v)[2]) {
        // (row re-materialised per tile: CSE'd across the buffers, the 64
        // per-word store offsets stayed live from phase C to G and spilled)
        asm volatile("" : "+v"(row));
        store_rows2<OFF32>(base, LD, row, t, h, v);
#if MAS_POL_DB_SB
        __builtin_amdgcn_sched_barrier(0);
#endif
    };
    const int64_t b0 = blockIdx.x;
    // the prologue's copies land before the loop (the same order as landing
    // them in the first block's phase A), so the loop's phase-A wait is always
    // the counted one: no path reaches it with fewer VMEM ops after the
    // copies than it counts (scripts/check_policy_waits.py checks every path)
    if (b0 < nblk) {
        copy_db(buf(0), F + Lo.w1(), (KS < kKc ? KS : kKc) * kMT * 64);
        land_db<0>();
    }
    for (int64_t blk = b0; blk < nblk; blk += gridDim.x) {
        // the lane index made opaque per block: keeps the compiler from
        // hoisting the blocks' LDS and store addresses out of the loop (held
        // live across it they spilled)
        int l = l0;
        asm volatile("" : "+v"(l));
        const int h = l >> 5;
        const int64_t row = blk * kDRows + wv * 32 + (l & 31);
        bf8 h1[kMT][2], h2[kMT][2];
        // the loss inputs of the row (read in phase E)
        uint32_t aw0 = 0, aw1 = 0;  // the row's 6 action bytes: 0..3, 4..5
        float adv = 0.0f, old_lp = 0.0f, ret = 0.0f;
        // ---- layer 1: NCH stages of up to kKc k-steps
        {
            f16v acc[kMT];
#pragma unroll
            for (int mt = 0; mt < kMT; ++mt) acc[mt] = f16v{};
            bf8 x[KS];
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                if (c == 0) {
                    if (blk != b0) land_db<32>();  // phase G: 32 dA1 stores after them
                } else {
                    if (c == 1) land_db<KS>();  // chunk 0: the x loads after them
                    else land_db<0>();
                }
                const bf8* w = buf(sc);
                if (c + 1 < NCH) {
                    const int k1 = (c + 1) * kKc, kn = KS - k1 < kKc ? KS - k1 : kKc;
                    copy_db(buf(sc + 1), F + Lo.w1() + k1 * kMT * 64, kn * kMT * 64);
                } else {
                    copy_db(buf(sc + 1), F + Lo.w23(), kHalf * 64);
                }
                if (c == 0) {
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
                        x[ks] = *reinterpret_cast<const bf8*>(A.xb + row * A.xb_stride + 16 * ks + 8 * h);
                }
                const int kn = KS - c * kKc < kKc ? KS - c * kKc : kKc;
#pragma unroll
                for (int q = 0; q < kn; ++q) {
                    const bf8* wk = w + q * kMT * 64 + l;
#pragma unroll
                    for (int mt = 0; mt < kMT; ++mt) acc[mt] = mfma(wk[mt * 64], x[c * kKc + q], acc[mt]);
                }
                ++sc;
            }
            tanh_h1(acc, b1p, h, h1);
        }
        // ---- layers 2 + 3: two half stages (C, D)
        f16v z3 = f16v{};
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            if (hf == 0) land_db<NCH == 1 ? KS : 0>();
            else land_db<64>();  // phase C: 64 h1 stores after them
            const bf8* wl2 = buf(sc);
            if (hf == 0) {
                copy_db(buf(sc + 1), F + Lo.w23() + kHalf * 64, kHalf * 64);
#pragma unroll
                for (int mt = 0; mt < kMT; ++mt) st2(A.h1, row, mt, h, h1[mt]);  // 64 stores
            } else {
                copy_db(buf(sc + 1), F + Lo.wbk(), kBk0 * 64);
                // the loss inputs of the row (read in phase E)
                const uint16_t* ap = reinterpret_cast<const uint16_t*>(A.act + row * 6);
                aw0 = (uint32_t)ap[0] | ((uint32_t)ap[1] << 16);
                aw1 = ap[2];
                adv = A.adv[row];
                old_lp = A.old_logp[row];
                ret = A.ret[row];
#pragma unroll
                for (int mt = 0; mt < kMT / 2; ++mt) st2(A.h2, row, mt, h, h2[mt]);  // 32 stores
            }
#pragma unroll
            for (int q = 0; q < kMT / 2; ++q) {
                const int mo = kMT / 2 * hf + q;
                f16v a = f16v{};
                const bf8* w = wl2 + q * 16 * 64 + l;
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) a = mfma(w[kk * 64], h1[kk >> 1][kk & 1], a);
                float b[16];
                load16(b2p + (mo * 2 + h) * 16, b);
#pragma unroll
                for (int i = 0; i < 16; ++i) h2[mo][i >> 3][i & 7] = (__bf16)tanh_pre(a[i], b[i]);
                const bf8* w3 = wl2 + (kMT / 2 * 16 + 2 * q) * 64 + l;
                z3 = mfma(w3[0], h2[mo][0], z3);
                z3 = mfma(w3[64], h2[mo][1], z3);
            }
            ++sc;
        }
        // the loss inputs consumed on every lane here, at the end of phase D:
        // their wait then sits in straight-line code (read only inside the
        // lane-half branch, they would stay pending in the compiler's
        // wait-count state on the branch-skipping path, around the block loop,
        // and force a full vmcnt(0) at the next reuse of their registers)
        // (a memory clobber anchors it after the phase's LDS reads and stores)
        // (in-out operands: nothing derived from them is computed before)
        asm volatile("" : "+v"(aw0), "+v"(aw1), "+v"(adv), "+v"(old_lp), "+v"(ret)::"memory");
        // ---- E: W3^T; the loss gradient, dA2
        // phase D: the 32 h2 stores after them (plus the loss-input loads, not
        // counted: the compiler may combine the six 2-B / 4-B loads into fewer
        // instructions, and a count above the real one would stop waiting too
        // early; counting fewer only over-waits)
        land_db<32>();
        const bf8* wb = buf(sc);
        copy_db(buf(sc + 1), F + Lo.wbk() + kBk0 * 64, kBk1 * 64);
#pragma unroll
        for (int mt = kMT / 2; mt < kMT; ++mt) st2(A.h2, row, mt, h, h2[mt]);  // 32 stores
        float dz[kO];
#pragma unroll
        for (int o = 0; o < kO; ++o) dz[o] = 0.0f;
        if (h == 0) {
            float z[kO];
#pragma unroll
            for (int o = 0; o < kO; ++o) z[o] = z3[o] + b3[o];
            int a[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) a[k] = (int)(int8_t)(((k < 4 ? aw0 : aw1) >> (8 * (k & 3))) & 0xffu);
            // (log-softmax and probabilities recomputed in the gradient loop
            // from the heads' lse: the same values, 30 fewer live registers)
            float lse[6], hent[6];
            float lp = 0.0f, ent = 0.0f;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                float mx = z[off];
#pragma unroll
                for (int k = 1; k < n; ++k) mx = fmaxf(mx, z[off + k]);
                float se = 0.0f;
#pragma unroll
                for (int k = 0; k < n; ++k) se += exp_fast(z[off + k] - mx);
                lse[hd] = mx + log_fast(se);
                float e = 0.0f;
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const float lsm = z[off + k] - lse[hd];
                    const float p = exp_fast(lsm);
                    e -= p * lsm;
                    if (k == ak) lp += lsm;
                }
                hent[hd] = e;
                ent += e;
            }
            const float ratio = exp_fast(lp - old_lp);
            const float s1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.0f - A.clip), 1.0f + A.clip);
            const float s2 = rc * adv;
            const float glp = s1 <= s2 ? -s1 : 0.0f;
            const float sc_ = A.scale;
#pragma unroll
            for (int hd = 0; hd < 6; ++hd) {
                const int n = kHeadN[hd], off = kHeadOff[hd];
                const int ak = a[hd];
#pragma unroll
                for (int k = 0; k < n; ++k) {
                    const float oh = k == ak ? 1.0f : 0.0f;
                    const float lsm = z[off + k] - lse[hd];
                    const float p = exp_fast(lsm);
                    dz[off + k] = sc_ * (glp * (oh - p) + A.ent_coef * p * (lsm + hent[hd]));
                }
            }
            const float dv = z[kO - 1] - ret;
            dz[kO - 1] = sc_ * A.vf_coef * 2.0f * dv;
            st[0] += -fminf(s1, s2);
            st[1] += dv * dv;
            st[2] += ent;
            st[3] += fabsf(ratio - 1.0f) > A.clip ? 1.0f : 0.0f;
#pragma unroll
            for (int o = 0; o < kO; ++o) A.dz[(int64_t)o * LD + row] = (__bf16)dz[o];
        }
        bf8 dzf[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) dzf[i >> 3][i & 7] = (__bf16)dz[i];
        bf8 da2[kMT][2];
#pragma unroll
        for (int mo = 0; mo < kMT; ++mo) {
            f16v g = f16v{};
            g = mfma(wb[(mo * 2) * 64 + l], dzf[0], g);
            g = mfma(wb[(mo * 2 + 1) * 64 + l], dzf[1], g);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float hv = (float)h2[mo][i >> 3][i & 7];
                da2[mo][i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
            }
            st2(A.da2, row, mo, h, da2[mo]);  // 64 stores
        }
        ++sc;
        // ---- F, G: W2^T halves; dA1
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            if (hf == 0) land_db<96>();  // phase E: 32 h2 + 64 dA2 stores (+ 16 dz) after them
            else land_db<32>();          // phase F: 32 dA1 stores
            const bf8* W2T = buf(sc);
            if (hf == 0) copy_db(buf(sc + 1), F + Lo.wbk() + (kBk0 + kBk1) * 64, kBk1 * 64);
            else if (blk + gridDim.x < nblk) copy_db(buf(sc + 1), F + Lo.w1(), (KS < kKc ? KS : kKc) * kMT * 64);
#pragma unroll
            for (int q = 0; q < kMT / 2; ++q) {
                const int mt = kMT / 2 * hf + q;
                f16v g = f16v{};
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) g = mfma(W2T[(q * 16 + kk) * 64 + l], da2[kk >> 1][kk & 1], g);
                bf8 d1[2];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float hv = (float)h1[mt][i >> 3][i & 7];
                    d1[i >> 3][i & 7] = (__bf16)(g[i] * dtanh(hv));
                }
                st2(A.da1, row, mt, h, d1);  // 8 stores
            }
            ++sc;
        }
    }
    const int l = l0;
    // per-workgroup loss partials: row 2 b0 (this workgroup's first block), zeros in the
    // other rows of its blocks (two 128-row partial rows per 256-row block)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float v = st[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (l == 0) red[wv * 4 + k] = v;
    }
    __syncthreads();
    for (int64_t blk = b0; blk < nblk; blk += gridDim.x) {
        if (threadIdx.x < 8) {
            const int k = (int)threadIdx.x & 3;
            float v = 0.0f;
            if (blk == b0 && threadIdx.x < 4) {
#pragma unroll
                for (int w = 0; w < kDW; ++w) v += red[w * 4 + k];
            }
            A.partials[(2 * blk + (threadIdx.x >> 2)) * 4 + k] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// Weight gradients of one minibatch, dW = A B^T and db = row sums of A, over
// the minibatch rows K: A [F][K] (dA2 or dz) and B [G][K] (h1 or h2) are the
// feature-major bf16 activations mas_policy_train writes (K contiguous, row
// strides lda / ldb), accumulated in fp32.  Split K: workgroup b takes rows
// [b kc, (b + 1) kc) and writes a partial record [F][G] + [F] (dW, db);
// k_dw_reduce sums the records.  Four waves per workgroup, wave (wf, wg)
// owning FT x GT 32x32 output tiles (MFMA accumulators, one wave per SIMD).
// The MFMA operands come straight from global memory: lane (r, h) of a
// 32x32x16 bf16 fragment holds 8 consecutive k of one row (16 B) for both A
// (row f) and B (row g), so no LDS staging is needed, and a row's 32 B per
// k-step and the next three k-steps' bytes share one 128-B line.  Each
// activation byte is read from HBM once.  Measured slower than the hipBLASLt
// split-K GEMMs it was meant to replace (dW2 2.86 vs 1.28 ms per 4.2M-row
// minibatch): a load instruction touches 32 rows 8 MB apart for 32 B each;
// it remains for K not a multiple of 64; the trainer runs k_dw_lds below.
template <int WF, int WGN, int FT, int GT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_dw_nt(
    int F, int G, int64_t K, const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
    int64_t kc, float* __restrict__ part)
{
    static_assert(WF * WGN == 4, "four waves");
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63), r = lane & 31, h = lane >> 5;
    const int wf = wave / WGN, wg = wave % WGN;
    const int64_t k0 = (int64_t)blockIdx.x * kc;
    const int64_t k1 = k0 + kc < K ? k0 + kc : K;
    f16v acc[FT][GT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < GT; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;
    float bs[FT];
    const __bf16* pa[FT];
    bool va[FT];
#pragma unroll
    for (int t = 0; t < FT; ++t) {
        const int f = (wf * FT + t) * 32 + r;
        va[t] = f < F;
        pa[t] = A + (int64_t)(va[t] ? f : 0) * lda + 8 * h;
        bs[t] = 0.0f;
    }
    const __bf16* pb[GT];
#pragma unroll
    for (int t = 0; t < GT; ++t) pb[t] = B + (int64_t)((wg * GT + t) * 32 + r) * ldb + 8 * h;
    const bf8 zero = {};
    // two k-steps per iteration, the next iteration's fragments loaded first
    bf8 a0[FT], a1[FT], b0[GT], b1[GT];
#pragma unroll
    for (int t = 0; t < FT; ++t) {
        a0[t] = va[t] ? *(const bf8*)(pa[t] + k0) : zero;
        a1[t] = va[t] ? *(const bf8*)(pa[t] + k0 + 16) : zero;
    }
#pragma unroll
    for (int t = 0; t < GT; ++t) {
        b0[t] = *(const bf8*)(pb[t] + k0);
        b1[t] = *(const bf8*)(pb[t] + k0 + 16);
    }
    for (int64_t k = k0; k < k1; k += 32) {
        const int64_t kn = k + 32 < k1 ? k + 32 : k;
        bf8 c0[FT], c1[FT], d0[GT], d1[GT];
#pragma unroll
        for (int t = 0; t < FT; ++t) {
            c0[t] = va[t] ? *(const bf8*)(pa[t] + kn) : zero;
            c1[t] = va[t] ? *(const bf8*)(pa[t] + kn + 16) : zero;
        }
#pragma unroll
        for (int t = 0; t < GT; ++t) {
            d0[t] = *(const bf8*)(pb[t] + kn);
            d1[t] = *(const bf8*)(pb[t] + kn + 16);
        }
#pragma unroll
        for (int i = 0; i < FT; ++i)
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[i][j] = mfma(a0[i], b0[j], acc[i][j]);
#pragma unroll
        for (int i = 0; i < FT; ++i)
#pragma unroll
            for (int j = 0; j < GT; ++j) acc[i][j] = mfma(a1[i], b1[j], acc[i][j]);
        if (wg == 0) {
#pragma unroll
            for (int t = 0; t < FT; ++t)
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[t] += (float)a0[t][e] + (float)a1[t][e];
        }
#pragma unroll
        for (int t = 0; t < FT; ++t) {
            a0[t] = c0[t];
            a1[t] = c1[t];
        }
#pragma unroll
        for (int t = 0; t < GT; ++t) {
            b0[t] = d0[t];
            b1[t] = d1[t];
        }
    }
    float* rec = part + (int64_t)blockIdx.x * ((int64_t)F * G + F);
#pragma unroll
    for (int i = 0; i < FT; ++i) {
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            const int g = (wg * GT + j) * 32 + r;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int f = (wf * FT + i) * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (f < F) rec[(int64_t)f * G + g] = acc[i][j][q];
            }
        }
    }
    if (wg == 0) {
#pragma unroll
        for (int t = 0; t < FT; ++t) {
            const float v = bs[t] + __shfl_xor(bs[t], 32, 64);
            if (h == 0 && va[t]) rec[(int64_t)F * G + (wf * FT + t) * 32 + r] = v;
        }
    }
}

// dW = A B^T for F = G = 256 through LDS (the faster form of k_dw_nt): per
// K-tile of kDwKT rows, both operand tiles [256][kDwKT] bf16 land in LDS by
// LDS-DMA (global_load_lds_dwordx4; the lanes of one row read its bytes of
// the tile contiguously), in a ring of kDwStages stages: kDwStages - 1 tiles'
// loads are in flight while one feeds the MFMAs (each wave waits with vmcnt
// for its oldest tile only, then a bare block barrier).  Row r's 16-B chunk c
// sits in slot c ^ ((r / RS) % CH) of its row, so a fragment read (32 rows,
// one chunk) is conflict-free per 16 lanes.  Thread t also sums row t of the
// A tile (db).  Measured (4.2M-row minibatch, dW2): 64-row tiles in 2 stages
// 1.13 ms, 32-row tiles in 4 stages 1.63 ms, the hipBLASLt GEMM 1.28 ms.
constexpr int kDwKT = 64;                  // K rows per tile
constexpr int kDwStages = 2;
constexpr int kDwRowB = kDwKT * 2;         // bytes of a row in a tile
constexpr int kDwCH = kDwKT / 8;           // 16-B chunks per row
constexpr int kDwRS = 128 / kDwKT;         // rows per 64 banks
constexpr int kDwRPI = 64 / kDwCH;         // rows per load instruction
constexpr int kDwIPW = 256 / kDwRPI / 4;   // load instructions per wave per operand
constexpr int kDwTileB = 256 * kDwRowB;    // bytes per operand tile
__device__ __forceinline__ int dw_off(int row, int c)
{
    return row * kDwRowB + 16 * (c ^ ((row / kDwRS) & (kDwCH - 1)));
}
template <int N>
__device__ __forceinline__ void wait_vm()
{
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt(((N >> 4) << 14) | (N & 15) | 0xF70);  // vmcnt(N), no expcnt / lgkmcnt wait
}

// FR = 256 (dW2: waves 2 x 2, 128 f x 128 g each) or 16 (dW3: the A tile's
// rows 16..31 stay zero, waves 1 x 4, 32 f x 64 g each); ST stages.
template <int FR, int ST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_dw_lds(
    int64_t K, const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb, int64_t kc,
    float* __restrict__ part)
{
    static_assert(FR == 256 || FR == 16, "F");
    constexpr int FA = FR == 256 ? 256 : 32;  // A tile rows (16..31 zero for FR = 16)
    constexpr int FT = FR == 256 ? 4 : 1, GT = FR == 256 ? 4 : 2;
    constexpr int AIPW = FR == 256 ? kDwIPW : 1;  // A load instructions per loading wave
    // one array, stage st = [A tile | B tile]: with two arrays the compiler
    // put a vmcnt(0) before the fragment reads (the next tiles' LDS-DMA could
    // not be told apart from them), which serialised loads and MFMAs
    constexpr int kA = FA * kDwRowB, kStB = kA + kDwTileB;
    __shared__ __attribute__((aligned(16))) uint8_t lds[ST][kStB];
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63), r = lane & 31, h = lane >> 5;
    const int wf = FR == 256 ? wave >> 1 : 0, wg = FR == 256 ? wave & 1 : wave;
    const int64_t k0 = (int64_t)blockIdx.x * kc;
    const int64_t k1 = k0 + kc < K ? k0 + kc : K;
    const int nt = (int)((k1 - k0) / kDwKT);
    const int lrow = lane / kDwCH, lslot = lane % kDwCH;
    if (FR < FA) {
        // the padding rows of every stage's A tile, once
        for (int i = (int)threadIdx.x; i < ST * (FA - FR) * kDwRowB / 16; i += 256) {
            const int st = i / ((FA - FR) * kDwRowB / 16), o = i % ((FA - FR) * kDwRowB / 16);
            *(uint4*)(&lds[st][FR * kDwRowB + 16 * o]) = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();
    }
    auto issue = [&](int t) {
        const int st = t % ST;
        const int64_t kt = k0 + (int64_t)t * kDwKT;
#pragma unroll
        for (int i = 0; i < kDwIPW; ++i) {
            const int R0 = (wave * kDwIPW + i) * kDwRPI;
            const int row = R0 + lrow;
            const int ch = lslot ^ ((row / kDwRS) & (kDwCH - 1));
            if (FR == 256)  // A and B rows interleaved (measured faster than B then A)
                __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)row * lda + kt + 8 * ch),
                                                 (lds_void*)(&lds[st][R0 * kDwRowB]), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(B + (int64_t)row * ldb + kt + 8 * ch),
                                             (lds_void*)(&lds[st][kA + R0 * kDwRowB]), 16, 0, 0);
        }
        if (FR < 256 && wave * AIPW * kDwRPI < FR) {  // wave-uniform
#pragma unroll
            for (int i = 0; i < AIPW; ++i) {
                const int R0 = (wave * AIPW + i) * kDwRPI;
                const int row = R0 + lrow;
                const int ch = lslot ^ ((row / kDwRS) & (kDwCH - 1));
                __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)row * lda + kt + 8 * ch),
                                                 (lds_void*)(&lds[st][R0 * kDwRowB]), 16, 0, 0);
            }
        }
    };
    f16v acc[FT][GT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < GT; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;
    float bsum = 0.0f;
#pragma unroll
    for (int t = 0; t < ST - 1; ++t)
        if (t < nt) issue(t);
    // the fewest load instructions a wave issues per tile (a wave that also
    // loads A rows waits a little longer than it must: still correct)
    constexpr int kPer = kDwIPW + (FR == 256 ? kDwIPW : 0);
    for (int t = 0; t < nt; ++t) {
        // this wave's loads of tile t have landed once at most the later
        // tiles' loads are outstanding
        const int later = nt - 1 - t < ST - 2 ? nt - 1 - t : ST - 2;
        if (ST > 3 && later >= 2) wait_vm<(ST > 3 ? 2 * kPer : 0)>();
        else if (ST > 2 && later == 1) wait_vm<(ST > 2 ? kPer : 0)>();
        else wait_vm<0>();
        // every wave's loads of tile t landed (each waited for its own);
        // tile t - 1's stage is free.  A bare s_barrier: __syncthreads()'s
        // fence would wait for the later tiles' loads too
        __builtin_amdgcn_s_barrier();
        if (t + ST - 1 < nt) issue(t + ST - 1);
        const uint8_t* la = lds[t % ST];
        const uint8_t* lb = lds[t % ST] + kA;
#pragma unroll
        for (int s = 0; s < kDwKT / 16; ++s) {
            const int c = 2 * s + h;
            bf8 a[FT], b[GT];
#pragma unroll
            for (int i = 0; i < FT; ++i) a[i] = *(const bf8*)(la + dw_off((wf * FT + i) * 32 + r, c));
#pragma unroll
            for (int j = 0; j < GT; ++j) b[j] = *(const bf8*)(lb + dw_off((wg * GT + j) * 32 + r, c));
#pragma unroll
            for (int i = 0; i < FT; ++i)
#pragma unroll
                for (int j = 0; j < GT; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
        }
        // db: thread t sums row t of the A tile
        if ((int)threadIdx.x < FR) {
#pragma unroll
            for (int c = 0; c < kDwCH; ++c) {
                const bf8 v = *(const bf8*)(la + dw_off((int)threadIdx.x, c));
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum += (float)v[e];
            }
        }
    }
    float* rec = part + (int64_t)blockIdx.x * (FR * 256 + FR);
#pragma unroll
    for (int i = 0; i < FT; ++i) {
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            const int g = (wg * GT + j) * 32 + r;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int f = (wf * FT + i) * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (f < FR) rec[(int64_t)f * 256 + g] = acc[i][j][q];
            }
        }
    }
    if ((int)threadIdx.x < FR) rec[FR * 256 + threadIdx.x] = bsum;
}

// out[i] = sum over the nb partial records of part[b][i], i < n
__global__ __launch_bounds__(256) void k_dw_reduce(int64_t n, int nb, const float* __restrict__ part,
                                                   float* __restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float a = 0.0f;
#pragma unroll 16
    for (int b = 0; b < nb; ++b) a += part[(int64_t)b * n + i];
    out[i] = a;
}
}  // namespace pol

// ---------------------------------------------------------------------------
// launchers (argument checks are in the C-ABI wrappers, mas_capi.hip)
// ---------------------------------------------------------------------------
int64_t policy_packed_bytes(int D) { return pol::Layout{(D + 15) / 16}.bytes(); }

hipError_t policy_pack(int D, const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                       const float* b3, void* packed, hipStream_t s)
{
    const pol::Layout L{(D + 15) / 16};
    const int64_t n = L.nfrag() * 8 + 2 * pol::kMT * 2 * 16 + pol::kO;
    hipLaunchKernelGGL(pol::k_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, D, L.ks1, W1, b1, W2, b2, W3,
                       b3, (uint8_t*)packed);
    return hipGetLastError();
}

int policy_rm_feature(int col) { return pol::rm_feature(col); }

// ---------------------------------------------------------------------------
// The PPO optimizer step over the policy's flat fp32 parameters (the trainer
// keeps parameters, gradients and both Adam moments as views into four flat
// buffers): torch.nn.utils.clip_grad_norm_ followed by torch.optim.Adam (no
// weight decay, no amsgrad) as two launches -- a split sum of squares, then
// every block re-sums the partials and updates its share -- instead of the
// ~20 foreach / norm / copy launches of the torch step per minibatch.
namespace pol {
constexpr int kAdamBlocks = 128;  // partial sums of the gradient norm
__device__ __forceinline__ float block_sum256(float v, float* red)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ __launch_bounds__(256) void k_adam_sqsum(int64_t n, const float* __restrict__ g, float scale,
                                                    float* __restrict__ part)
{
    __shared__ float red[4];
    float s = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float x = g[i] * scale;
        s += x * x;
    }
    s = block_sum256(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_adam_update(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     const float* __restrict__ part, float scale, float max_norm,
                                                     float b2, float w1, float w2, float step_size, float sqrt_bc2,
                                                     float eps)
{
    __shared__ float red[4];
    const float s = block_sum256(threadIdx.x < kAdamBlocks ? part[threadIdx.x] : 0.0f, red);
    // clip_grad_norm_: coef = max_norm / (norm + 1e-6), clamped to 1 (applied even when it is 1)
    const float coef = max_norm > 0.0f ? fminf(max_norm / (sqrtf(s) + 1e-6f), 1.0f) : 1.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float gi = (g[i] * scale) * coef;
        float mi = m[i];
        mi = mi + w1 * (gi - mi);                     // exp_avg.lerp_(grad, w1 = 1 - beta1)
        const float vi = v[i] * b2 + w2 * (gi * gi);  // exp_avg_sq.mul_(beta2).addcmul_(g, g, w2 = 1 - beta2)
        const float den = sqrtf(vi) / sqrt_bc2 + eps;
        p[i] = p[i] + (-step_size) * (mi / den);
        m[i] = mi;
        v[i] = vi;
    }
}
}  // namespace pol

int64_t policy_adam_scratch() { return pol::kAdamBlocks; }

hipError_t policy_adam(int64_t n, float* p, const float* g, float* m, float* v, float grad_scale, float max_norm,
                       double lr, double b1, double b2, double eps, int64_t step, float* scratch, hipStream_t s)
{
    // torch.optim.Adam's scalars are Python floats (double) rounded once to
    // float by the foreach kernels: the bias corrections, lr / bc1, and the
    // lerp / addcmul weights 1 - beta (1 - 0.999f in float would be 1.3e-5 off)
    const double bc1 = 1.0 - std::pow(b1, (double)step), bc2 = 1.0 - std::pow(b2, (double)step);
    const float step_size = (float)(lr / bc1), sqrt_bc2 = (float)std::sqrt(bc2);
    hipLaunchKernelGGL(pol::k_adam_sqsum, dim3(pol::kAdamBlocks), dim3(256), 0, s, n, g, grad_scale, scratch);
    const int64_t nb = (n + 255) / 256 < 512 ? (n + 255) / 256 : 512;
    hipLaunchKernelGGL(pol::k_adam_update, dim3((unsigned)nb), dim3(256), 0, s, n, p, g, m, v, scratch, grad_scale,
                       max_norm, (float)b2, (float)(1.0 - b1), (float)(1.0 - b2), step_size, sqrt_bc2, (float)eps);
    return hipGetLastError();
}


// workgroups of the train kernel (= its partial records) and of the act kernel
int64_t policy_blocks(int64_t M) { return (M + 32 * pol::kTWaves - 1) / (32 * pol::kTWaves); }
static int64_t act_blocks(int64_t M) { return (M + 32 * pol::kWaves - 1) / (32 * pol::kWaves); }

hipError_t policy_act(const void* packed, int D, int64_t M, const float* obs, void* xb, int64_t xb_stride,
                      uint64_t seed, uint64_t step, int64_t first_row, int8_t* act, float* logp, float* value,
                      hipStream_t s)
{
    const int ks1 = (D + 15) / 16;
    // obs == nullptr: the bf16 rows in xb are the input (mas_policy_act_x)
    const bool xin = obs == nullptr;
    // the heads' sampling on both half-waves; MAS_ACT_SPLIT=0 (read per call): on one
    const char* sv = getenv("MAS_ACT_SPLIT");
    const bool split = !(sv && sv[0] == '0');
    auto k = split ? (xin ? (ks1 == 10 ? pol::k_policy_act<10, true> : ks1 == 9 ? pol::k_policy_act<9, true>
                                                                              : pol::k_policy_act<0, true>)
                          : (ks1 == 10 ? pol::k_policy_act<10, false> : ks1 == 9 ? pol::k_policy_act<9, false>
                                                                               : pol::k_policy_act<0, false>))
                   : (xin ? (ks1 == 10 ? pol::k_policy_act<10, true, false> : ks1 == 9 ? pol::k_policy_act<9, true, false>
                                                                              : pol::k_policy_act<0, true, false>)
                          : (ks1 == 10 ? pol::k_policy_act<10, false, false>
                                       : ks1 == 9 ? pol::k_policy_act<9, false, false> : pol::k_policy_act<0, false, false>));
    hipLaunchKernelGGL(k, dim3((unsigned)act_blocks(M)), dim3(64 * pol::kWaves), 0, s, (const uint8_t*)packed, D,
                       ks1, M, obs, (__bf16*)xb, xb_stride, seed, step, first_row, act, logp, value);
    return hipGetLastError();
}

hipError_t policy_train(const void* packed, int D, int64_t M, const void* xb, int64_t xb_stride, const int8_t* act,
                        const float* old_logp, const float* adv, const float* ret, float clip, float vf_coef,
                        float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                        int64_t ld, float* partials, hipStream_t s, bool rm)
{
    pol::TrainArgs A;
    A.ld = ld;
    A.packed = (const uint8_t*)packed;
    A.ks1 = (D + 15) / 16;
    A.M = M;
    A.xb = (const __bf16*)xb;
    A.xb_stride = xb_stride;
    A.act = act;
    A.old_logp = old_logp;
    A.adv = adv;
    A.ret = ret;
    A.clip = clip;
    A.vf_coef = vf_coef;
    A.ent_coef = ent_coef;
    A.scale = scale;
    A.h1 = (__bf16*)h1;
    A.h2 = (__bf16*)h2;
    A.da1 = (__bf16*)da1;
    A.da2 = (__bf16*)da2;
    A.dz = (__bf16*)dz;
    A.partials = partials;
    // MAS_POL_FORCE_OFF64=1 (test hook, read per call): the 64-bit store
    // offsets that only buffers over 4 GB take, on any size
    const char* f64 = getenv("MAS_POL_FORCE_OFF64");
    const bool o32 = ld <= pol::kOff32Ld && !(f64 && f64[0] == '1');
    // the persistent double-buffered kernel for the full 256-row blocks of the
    // PPO update's store mode (feature-major, two rows per lane, 32-bit
    // offsets, compile-time layer-1 depth), k_policy_train for the rest;
    // MAS_POL_DB=0: k_policy_train_cw / k_policy_train only
    const char* db = getenv("MAS_POL_DB");
    const int64_t nfull = M / pol::kDRows;
    if (!rm && o32 && (A.ks1 == 10 || A.ks1 == 9) && ((M | ld) & 1) == 0 && nfull > 0 && !(db && db[0] == '0')) {
        static int ncu = 0;
        if (ncu == 0) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
                ncu = 256;
        }
        const int64_t grid = nfull < ncu ? nfull : ncu;
        auto kd = A.ks1 == 10 ? pol::k_policy_train_db<10, true> : pol::k_policy_train_db<9, true>;
        hipLaunchKernelGGL(kd, dim3((unsigned)grid), dim3(64 * pol::kDW), 0, s, A, nfull);
        const int64_t r0 = nfull * pol::kDRows;
        if (r0 < M) {  // the partial last block: k_policy_train on offset buffers
            pol::TrainArgs T = A;
            T.M = M - r0;
            T.xb = A.xb + r0 * A.xb_stride;
            T.act = A.act + r0 * 6;
            T.old_logp = A.old_logp + r0;
            T.adv = A.adv + r0;
            T.ret = A.ret + r0;
            T.h1 = A.h1 + r0;
            T.h2 = A.h2 + r0;
            T.da1 = A.da1 + r0;
            T.da2 = A.da2 + r0;
            T.dz = A.dz + r0;
            T.partials = A.partials + 2 * nfull * 4;
            auto kt = A.ks1 == 10 ? pol::k_policy_train<10, true, false> : pol::k_policy_train<9, true, false>;
            hipLaunchKernelGGL(kt, dim3((unsigned)policy_blocks(T.M)), dim3(64 * pol::kTWaves), 0, s, T);
        }
        return hipGetLastError();
    }
    // the counted-wait kernel for the PPO update's store mode (feature-major,
    // two rows per lane: M and ld even) with 32-bit store offsets; its 64-bit
    // offset and 9-k-step layer-1 builds spill (compiler resource report), so
    // those keep k_policy_train.  MAS_POL_CW=0: k_policy_train everywhere
    const char* cw = getenv("MAS_POL_CW");
    if (!rm && o32 && A.ks1 != 9 && ((M | ld) & 1) == 0 && !(cw && cw[0] == '0')) {
        auto kc = A.ks1 == 10 ? pol::k_policy_train_cw<10, true> : pol::k_policy_train_cw<0, true>;
        hipLaunchKernelGGL(kc, dim3((unsigned)policy_blocks(M)), dim3(64 * pol::kTWaves), 0, s, A);
        return hipGetLastError();
    }
    auto k = rm ? (A.ks1 == 10 ? pol::k_policy_train<10, false, true>
                   : A.ks1 == 9 ? pol::k_policy_train<9, false, true> : pol::k_policy_train<0, false, true>)
           : A.ks1 == 10 ? (o32 ? pol::k_policy_train<10, true, false> : pol::k_policy_train<10, false, false>)
           : A.ks1 == 9 ? (o32 ? pol::k_policy_train<9, true, false> : pol::k_policy_train<9, false, false>)
                        : (o32 ? pol::k_policy_train<0, true, false> : pol::k_policy_train<0, false, false>);
    hipLaunchKernelGGL(k, dim3((unsigned)policy_blocks(M)), dim3(64 * pol::kTWaves), 0, s, A);
    return hipGetLastError();
}

// dW = A B^T, db = row sums of A over K rows (F in {16, 256}, G = 256): the
// split-K records go to `scratch` (policy_dw_scratch floats), the sums to
// out [F * G + F] (dW row-major, then db)
// Split-K blocks: one workgroup per CU (256) whenever each still gets >= 2048
// rows (32 tiles: its 263-KB dW2 record is then an eighth of the 2 MB it
// streams).  The old rule (16384 rows per block) gave a 1.31M-row minibatch
// 80 blocks -- a third of the CUs: dW2 681 us against 859 for 4.19M rows
// (r06g).
static int dw_blocks(int64_t K)
{
    const int64_t b = K / 2048;
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}
int64_t policy_dw_scratch(int F, int G, int64_t K) { return (int64_t)dw_blocks(K) * ((int64_t)F * G + F); }

hipError_t policy_dw(int F, int G, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb, float* out,
                     float* scratch, hipStream_t s)
{
    const int nb = dw_blocks(K);
    int64_t kc = (K + nb - 1) / nb;
    kc = (kc + pol::kDwKT - 1) / pol::kDwKT * pol::kDwKT;
    const int nbu = (int)((K + kc - 1) / kc);
    if (F == 256 && G == 256 && K % pol::kDwKT == 0 && kc % pol::kDwKT == 0)
        hipLaunchKernelGGL((pol::k_dw_lds<256, pol::kDwStages>), dim3((unsigned)nbu), dim3(256), 0, s, K,
                           (const __bf16*)A, lda, (const __bf16*)B, ldb, kc, scratch);
    else if (F == 16 && G == 256 && K % pol::kDwKT == 0 && kc % pol::kDwKT == 0)
        hipLaunchKernelGGL((pol::k_dw_lds<16, 4>), dim3((unsigned)nbu), dim3(256), 0, s, K, (const __bf16*)A, lda,
                           (const __bf16*)B, ldb, kc, scratch);
    else if (F == 256)
        hipLaunchKernelGGL((pol::k_dw_nt<2, 2, 4, 4>), dim3((unsigned)nbu), dim3(256), 0, s, F, G, K,
                           (const __bf16*)A, lda, (const __bf16*)B, ldb, kc, scratch);
    else
        hipLaunchKernelGGL((pol::k_dw_nt<1, 4, 1, 2>), dim3((unsigned)nbu), dim3(256), 0, s, F, G, K,
                           (const __bf16*)A, lda, (const __bf16*)B, ldb, kc, scratch);
    const int64_t n = (int64_t)F * G + F;
    hipLaunchKernelGGL(pol::k_dw_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, nbu, scratch, out);
    return hipGetLastError();
}

}  // namespace mas

