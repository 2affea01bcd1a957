// mas_capi.hip -- host side of the C-ABI declared in include/masurvival.h:
// config validation, capacity-class dispatch, Params (walls, vision cone, body
// masses, observation layout) computed once per handle, HBM state
// allocation, and the small seed / stats kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "../../include/masurvival.h"
#include "mas_env.h"

#ifndef MAS_CLASS_LIST
#define MAS_CLASS_LIST "?"
#endif

using namespace mas;

namespace mas {
struct ClassInfo {
    int words, w_rng, w_has32, w_stats, w_cont, w_invdt, lds_bytes;
    int am, post_union;  // agent slots; k_post_lanes' LDS union bytes (the in-place reset's permutation scratch)
};
#define MAS_DECLARE(NAME)                                                                                     \
    ClassInfo class_info_##NAME();                                                                          \
    void launch_step_##NAME(dim3, hipStream_t, const Params&, uint32_t*, int64_t, const int8_t*, float*, float*, \
                            uint8_t*, int, const StepSplit*);                                               \
    void launch_reset_##NAME(dim3, hipStream_t, const Params&, uint32_t*, int64_t, const uint8_t*, float*); \
    void launch_view_##NAME(hipStream_t, const Params&, const uint32_t*, int64_t, int64_t, float*);
#ifdef MAS_HAVE_1v1
MAS_DECLARE(1v1)
#endif
#ifdef MAS_HAVE_2v2
MAS_DECLARE(2v2)
#endif
#ifdef MAS_HAVE_ffa
MAS_DECLARE(ffa)
#endif
#ifdef MAS_HAVE_ffal
MAS_DECLARE(ffal)
#endif
#ifdef MAS_HAVE_xl
MAS_DECLARE(xl)
#endif
#ifdef MAS_HAVE_xxl
MAS_DECLARE(xxl)
#endif
// fused policy MLP of the PPO consumer (mas_policy.hip)
int64_t policy_packed_bytes(int D);
int64_t policy_blocks(int64_t M);
hipError_t policy_pack(int D, const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                       const float* b3, void* packed, hipStream_t s);
hipError_t policy_act(const void* packed, int D, int64_t M, const float* obs, void* xb, int64_t xb_stride,
                      uint64_t seed, uint64_t step, int64_t first_row, int8_t* act, float* logp, float* value,
                      hipStream_t s);
hipError_t policy_train(const void* packed, int D, int64_t M, const void* xb, int64_t xb_stride, const int8_t* act,
                        const float* old_logp, const float* adv, const float* ret, float clip, float vf_coef,
                        float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                        int64_t ld, float* partials, hipStream_t s, bool rm);
int policy_rm_feature(int col);
int64_t policy_adam_scratch();
hipError_t policy_adam(int64_t n, float* p, const float* g, float* m, float* v, float grad_scale, float max_norm,
                       double lr, double b1, double b2, double eps, int64_t step, float* scratch, hipStream_t s);
int64_t policy_dw_scratch(int F, int G, int64_t K);
hipError_t policy_dw(int F, int G, int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb, float* out,
                     float* scratch, hipStream_t s);
}  // namespace mas

namespace {

constexpr int kWG = 64;  // threads per workgroup of k_step / k_reset (mas_step.h)
// mas_step's default use of the side streams (MAS_SPLIT, mas_handle::split)
constexpr int kSplitDefault = 2;

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(x)                                                                                       \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) return fail(MAS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

__global__ void k_seed(uint32_t* __restrict__ state, int64_t N, const uint64_t* __restrict__ st6, int w_rng,
                       int w_has32)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    // st_hi, st_lo, inc_hi, inc_lo as (lo, hi) word pairs, then has32, u32
    for (int k = 0; k < 4; ++k) {
        uint64_t x = st6[e * 6 + k];
        state[state_index(w_rng + 2 * k, e, N)] = (uint32_t)(x & 0xffffffffULL);
        state[state_index(w_rng + 2 * k + 1, e, N)] = (uint32_t)(x >> 32);
    }
    state[state_index(w_has32, e, N)] = (uint32_t)st6[e * 6 + 4];
    state[state_index(w_has32 + 1, e, N)] = (uint32_t)st6[e * 6 + 5];
}

__global__ void k_stats(uint32_t* __restrict__ state, int64_t N, int w_stats, float* __restrict__ out)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    for (int k = 0; k < kStats; ++k) {
        uint32_t u = state[state_index(w_stats + k, e, N)];
        float f;
        __builtin_memcpy(&f, &u, 4);
        out[e * kStats + k] = f;
        state[state_index(w_stats + k, e, N)] = 0u;
    }
}


// generic Box2D b2PolygonShape::Set (weld, gift wrap, normals) for the cone
Poly4 poly_set4(const V2* in)
{
    V2 ps[4];
    int n = 0;
    for (int i = 0; i < 4; ++i) {
        bool uniq = true;
        for (int j = 0; j < n; ++j)
            if (dist2(in[i], ps[j]) < 0.5f * kLinearSlop) uniq = false;
        if (uniq) ps[n++] = in[i];
    }
    int i0 = 0;
    float x0 = ps[0].x;
    for (int i = 1; i < n; ++i) {
        float x = ps[i].x;
        if (x > x0 || (x == x0 && ps[i].y < ps[i0].y)) {
            i0 = i;
            x0 = x;
        }
    }
    int hull[8], m = 0, ih = i0;
    for (;;) {
        hull[m] = ih;
        int ie = 0;
        for (int j = 1; j < n; ++j) {
            if (ie == ih) {
                ie = j;
                continue;
            }
            V2 r = sub(ps[ie], ps[hull[m]]);
            V2 v = sub(ps[j], ps[hull[m]]);
            float c = cross(r, v);
            if (c < 0.0f) ie = j;
            if (c == 0.0f && len2(v) > len2(r)) ie = j;
        }
        ++m;
        ih = ie;
        if (ie == i0 || m >= 8) break;
    }
    Poly4 P{};
    for (int i = 0; i < 4 && i < m; ++i) P.v[i] = ps[hull[i]];
    for (int i = 0; i < 4 && i < m; ++i) {
        V2 e = sub(P.v[(i + 1) % m], P.v[i]);
        P.n[i] = cross_vs(e, 1.0f);
        normalize(P.n[i]);
    }
    return P;
}


// ---------------------------------------------------------------------------
// Rollout-side: GAE(gamma, lambda) over an on-device rollout buffer
// (not in the reference) as a segmented wavefront scan.
// The recurrence A_t = delta_t + c_t A_{t+1} (c_t = gamma lambda (1 - done_t),
// zero at an episode end: the segments) composes affine maps x -> a + b x, so
// a wave scans 64 time steps of one column at once: lane q holds step q's map
// and six shuffle rounds (Kogge-Stone, suffix order) give every lane the
// composition of its map with all later ones in the chunk; the chunk's
// carry-in is the later chunk's A at its first step.  A workgroup owns 64
// consecutive columns (= env*A + agent): their [64 steps][64 columns] tiles of
// rewards, values and done flags land in LDS with coalesced row loads and the
// advantages / returns leave the same way; each wave scans 16 of the columns.
// The fp64 partial sums (sum adv, sum adv^2) feed the advantage
// normalisation that the trainer all-reduces across ranks: each workgroup
// stores its pair into its own slot of the caller's scratch (no atomics, no
// library-global state, so concurrent calls on other streams are
// independent and the sums are deterministic), and k_gae_sums adds the slots
// in a fixed order.
constexpr int kGaeCols = 64;  // columns per workgroup; time chunk = one wave's 64 lanes
constexpr int kGaeWalkCols = 256;  // columns per workgroup of k_gae_walk

// a 256-thread workgroup's (s1, s2) into part[2 * blockIdx.x ..]: wave
// butterflies, then the four waves in order (one plain store pair)
__device__ __forceinline__ void gae_block_part(double s1, double s2, double* __restrict__ part)
{
    for (int off = 32; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
    }
    __shared__ double ws[4][2];
    const int w = (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) {
        ws[w][0] = s1;
        ws[w][1] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = ws[0][0] + ws[1][0] + ws[2][0] + ws[3][0];
        part[2 * blockIdx.x + 1] = ws[0][1] + ws[1][1] + ws[2][1] + ws[3][1];
    }
}

__global__ __launch_bounds__(256) void k_gae(int T, int64_t M, int A, const float* __restrict__ rew,
                                             const float* __restrict__ val, const uint8_t* __restrict__ done,
                                             float gamma, float lam, float* __restrict__ adv,
                                             float* __restrict__ ret, double* __restrict__ part)
{
    __shared__ float sr[64][kGaeCols + 1];   // rewards, then the advantages
    __shared__ float sv[65][kGaeCols + 1];   // values (the chunk's and the next step's)
    __shared__ float sn[64][kGaeCols + 1];   // 1 - done, then the returns
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int64_t c0 = (int64_t)blockIdx.x * kGaeCols;
    const int64_t m = c0 + lane;  // this lane's column in the load / store phases
    const bool mok = m < M;
    const int64_t E = M / A;
    const int64_t e = mok ? m / A : 0;
    const float gl = gamma * lam;
    float carry[kGaeCols / 4];  // per column of this wave: A at the first step of the later chunk
#pragma unroll
    for (int k = 0; k < kGaeCols / 4; ++k) carry[k] = 0.0f;
    double s1 = 0.0, s2 = 0.0;
    for (int t_hi = T; t_hi > 0; t_hi -= 64) {
        const int t_lo = t_hi > 64 ? t_hi - 64 : 0, n = t_hi - t_lo;
        // the chunk's rows (and the value row after it), coalesced over the
        // columns: every load of the wave's 17 rows issued before the first
        // LDS write
        {
            float lr[17], lv[17];
            uint8_t ld[17];
#pragma unroll
            for (int k = 0; k < 17; ++k) {
                const int q = w + 4 * k;
                const int64_t t = t_lo + (q <= n ? q : n);
                lv[k] = mok && q <= n ? val[t * M + m] : 0.0f;
                lr[k] = mok && q < n ? rew[t * M + m] : 0.0f;
                ld[k] = mok && q < n ? done[t * E + e] : (uint8_t)1;
            }
#pragma unroll
            for (int k = 0; k < 17; ++k) {
                const int q = w + 4 * k;
                if (q <= n) sv[q][lane] = lv[k];
                if (q < n) {
                    sr[q][lane] = lr[k];
                    sn[q][lane] = ld[k] ? 0.0f : 1.0f;
                }
            }
        }
        __syncthreads();
        // the scan: lane = step q of the chunk, one column at a time
        const bool qok = lane < n;
#pragma unroll
        for (int k = 0; k < kGaeCols / 4; ++k) {
            const int cc = w * (kGaeCols / 4) + k;
            float a = 0.0f, b = 1.0f;  // (past the chunk: the identity)
            if (qok) {
                const float nt = sn[lane][cc], v = sv[lane][cc];
                a = sr[lane][cc] + gamma * sv[lane + 1][cc] * nt - v;
                b = gl * nt;
            }
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const float a2 = __shfl_down(a, off, 64), b2 = __shfl_down(b, off, 64);
                if (lane + off < 64) {
                    a = a + b * a2;
                    b = b * b2;
                }
            }
            const float At = a + b * carry[k];
            carry[k] = __shfl(At, 0, 64);
            if (qok) {
                const float v = sv[lane][cc];
                sr[lane][cc] = At;
                sn[lane][cc] = At + v;
                if (c0 + cc < M) {
                    s1 += (double)At;
                    s2 += (double)At * (double)At;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int q = w + 4 * k;
            if (q < n && mok) {
                const int64_t t = t_lo + q;
                adv[t * M + m] = sr[q][lane];
                ret[t * M + m] = sn[q][lane];
            }
        }
        __syncthreads();  // (the next chunk's loads reuse the tiles)
    }
    // the workgroup's partial sums (wave butterflies, then its 4 waves) into
    // its own slot of the caller's scratch (round 4's one-address atomics
    // serialised, ~20 ns each; round 5's 256 shared slots made concurrent
    // calls race: DESIGN.md 4.3.10)
    gae_block_part(s1, s2, part);
}

// The default form: one thread per column walking t = T-1..0, every
// load / store coalesced across the wavefront ([t][m] rows), rows prefetched
// kGaeChunk steps ahead so the recurrence does not wait on HBM each step;
// the same partial-sum slots as k_gae
constexpr int kGaeChunk = 8;

__global__ __launch_bounds__(256) void k_gae_walk(int T, int64_t M, int A, const float* __restrict__ rew,
                                             const float* __restrict__ val, const uint8_t* __restrict__ done,
                                             float gamma, float lam, float* __restrict__ adv,
                                             float* __restrict__ ret, double* __restrict__ part)
{
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t E = M / A;
    double s1 = 0.0, s2 = 0.0;
    if (m < M) {
        const int64_t e = m / A;
        float a = 0.0f;
        float vnext = val[(int64_t)T * M + m];
        int t = T - 1;
        for (; t >= kGaeChunk - 1; t -= kGaeChunk) {
            float r[kGaeChunk], v[kGaeChunk], nt[kGaeChunk];
#pragma unroll
            for (int k = 0; k < kGaeChunk; ++k) {
                const int64_t row = t - k;
                r[k] = rew[row * M + m];
                v[k] = val[row * M + m];
                nt[k] = done[row * E + e] ? 0.0f : 1.0f;
            }
#pragma unroll
            for (int k = 0; k < kGaeChunk; ++k) {
                const float delta = r[k] + gamma * vnext * nt[k] - v[k];
                a = delta + gamma * lam * nt[k] * a;
                const int64_t row = t - k;
                adv[row * M + m] = a;
                ret[row * M + m] = a + v[k];
                s1 += (double)a;
                s2 += (double)a * (double)a;
                vnext = v[k];
            }
        }
        for (; t >= 0; --t) {
            const float r = rew[(int64_t)t * M + m], v = val[(int64_t)t * M + m];
            const float nt = done[(int64_t)t * E + e] ? 0.0f : 1.0f;
            const float delta = r + gamma * vnext * nt - v;
            a = delta + gamma * lam * nt * a;
            adv[(int64_t)t * M + m] = a;
            ret[(int64_t)t * M + m] = a + v;
            s1 += (double)a;
            s2 += (double)a * (double)a;
            vnext = v;
        }
    }
    // the workgroup's partial sums into its slot (k_gae)
    gae_block_part(s1, s2, part);
}

// the slots' sum into adv_sums (fixed order: thread k adds slots k, k + 256,
// ..., then a butterfly and the four waves in order)
__global__ __launch_bounds__(256) void k_gae_sums(const double* __restrict__ part, int nblocks,
                                                  double* __restrict__ sums)
{
    const int k = (int)threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    for (int b = k; b < nblocks; b += 256) {
        s1 += part[2 * b];
        s2 += part[2 * b + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
    }
    __shared__ double ws[4][2];
    if ((k & 63) == 0) {
        ws[k >> 6][0] = s1;
        ws[k >> 6][1] = s2;
    }
    __syncthreads();
    if (k == 0) {
        sums[0] = ws[0][0] + ws[1][0] + ws[2][0] + ws[3][0];
        sums[1] = ws[0][1] + ws[1][1] + ws[2][1] + ws[3][1];
    }
}


// ---------------------------------------------------------------------------
// Policy action sampling for the rollout (the reference's RandomPolicy /
// MultiAgentPolicy.act, demo.py:14-22, batched): one lane per agent row, six
// categorical heads (MultiDiscrete [3,3,3,2,2,2]) over a row of 15 logits,
// Gumbel-max with a counter-based hash RNG keyed by (seed, step, row, head),
// plus the row's log-probability of the drawn actions.  Replaces ~40 small
// torch kernels per step with one.
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_sample(int64_t M, const float* __restrict__ logits, int64_t stride,
                                                uint64_t seed, uint64_t step, int8_t* __restrict__ act,
                                                float* __restrict__ logp)
{
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const float* x = logits + m * stride;
    float l[15];
#pragma unroll
    for (int k = 0; k < 15; ++k) l[k] = x[k];
    const int n[6] = {3, 3, 3, 2, 2, 2};
    const uint64_t base = mix64(seed ^ mix64(step * 0x100000001B3ULL + (uint64_t)m));
    float lp = 0.0f;
    int off = 0;
#pragma unroll
    for (int h = 0; h < 6; ++h) {
        float mx = l[off];
#pragma unroll
        for (int k = 1; k < 3; ++k)
            if (k < n[h]) mx = fmaxf(mx, l[off + k]);
        float se = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < n[h]) se += expf(l[off + k] - mx);
        const float lse = mx + logf(se);
        int best = 0;
        float bv = -INFINITY;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= n[h]) continue;
            const uint64_t r = mix64(base + (uint64_t)(h * 4 + k));
            const float u = ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
            const float g = l[off + k] - logf(-logf(u));
            if (g > bv) { bv = g; best = k; }
        }
        float lb = l[off];
#pragma unroll
        for (int k = 1; k < 3; ++k)
            if (k < n[h] && k == best) lb = l[off + k];
        lp += lb - lse;
        act[m * 6 + h] = (int8_t)best;
        off += n[h];
    }
    logp[m] = lp;
}

}  // namespace

struct Ops {
    ClassInfo info;
    void (*step)(dim3, hipStream_t, const Params&, uint32_t*, int64_t, const int8_t*, float*, float*, uint8_t*, int,
                 const StepSplit*);
    void (*reset)(dim3, hipStream_t, const Params&, uint32_t*, int64_t, const uint8_t*, float*);
    void (*view)(hipStream_t, const Params&, const uint32_t*, int64_t, int64_t, float*);
};

struct mas_handle {
    mas_config cfg;
    Params P;
    Ops ops;
    int64_t N;
    int device;
    uint32_t* state;
    uint64_t* seedbuf;
    int* phys;  // the general-path list (k_pre -> general path, sharded) + [1] (unused) + [1] invalid-action count
                // + [1] last count + [1] list guard, then the list's shard counts (Params::list_shards)
    uint8_t* gen_flag;  // [N] env left the fast path this step
    float* sweep;       // A/B builds only (MAS_AB_KERNELS): k_gen_solve -> k_gen_toi
    mas_obs_layout layout;
    // the slow split (launch_step): side stream + fork / join events, made at
    // the first mas_step that splits, on the handle's device.  split: 0 the
    // one-stream order, 2 (default) the slow list on the side stream;
    // MAS_SPLIT=0/2 in the environment at mas_create (any other value is
    // refused), or mas_debug_force_general bit 3 (one stream)
    StepSplit sp;
    bool sp_made;
    int split, split_default;
    int* resetl;        // [2][N] auto-reset lists (main, side stream) + [2] counts
    int* slow;          // [N] slow list + [2] count slots
    uint8_t* slow_flag; // [N]
    int* slow_sig;      // host-mapped signal (P.slow_sig): a step flagged a slow env
    int slow_hold;      // steps left of the slow split since the last signal
    int par;  // which of the two slow-list count slots the next mas_step appends to
};

static void build_layout(mas_handle* h)
{
    const mas_config& c = h->cfg;
    int A = c.n_agents, H = c.n_heals, B = c.n_boxes, as_ = 8 + (c.teams ? 1 : 0);
    mas_obs_layout& L = h->layout;
    memset(&L, 0, sizeof(L));
    L.n_agents = A;
    struct K { const char* name; int ndim, s0, s1; bool on; int* off; };
    Params& P = h->P;
    K keys[] = {
        {"agent", 1, as_, 0, true, &P.o_agent},
        {"box_items", 2, B, 10, B > 0, &P.o_bi},
        {"box_items_mask", 1, B, 0, B > 0, &P.o_bim},
        {"box_slot", 2, 1, 8, B > 0, &P.o_bs},
        {"box_slot_mask", 1, 1, 0, B > 0, &P.o_bsm},
        {"boxes", 2, B, 11, B > 0, &P.o_box},
        {"boxes_mask", 1, B, 0, B > 0, &P.o_boxm},
        {"heal_slot", 2, 1, 1, H > 0, &P.o_hs},
        {"heal_slot_mask", 1, 1, 0, H > 0, &P.o_hsm},
        {"heals", 2, H, 2, H > 0, &P.o_heal},
        {"heals_mask", 1, H, 0, H > 0, &P.o_healm},
        {"lidars", 1, c.lidar_n_lasers, 0, c.lidar_n_lasers > 0, &P.o_lid},
        {"others", 2, A - 1, as_, true, &P.o_oth},
        {"others_mask", 1, A - 1, 0, true, &P.o_othm},
        {"zone", 1, 6, 0, true, &P.o_zone},
    };
    int off = 0, nk = 0;
    for (auto& k : keys) {
        *k.off = -1;
        if (!k.on) continue;
        *k.off = off;
        snprintf(L.key_name[nk], 24, "%s", k.name);
        L.key_offset[nk] = off;
        L.key_ndim[nk] = k.ndim;
        L.key_shape[nk][0] = k.s0;
        L.key_shape[nk][1] = k.ndim > 1 ? k.s1 : 0;
        off += k.s0 * (k.ndim > 1 ? k.s1 : 1);
        ++nk;
    }
    L.n_keys = nk;
    L.obs_dim = off;
    P.D = off;
}

static int build_params(mas_handle* h)
{
    const mas_config& c = h->cfg;
    Params& P = h->P;
    memset(&P, 0, sizeof(P));
    P.A = c.n_agents;
    P.H = c.n_heals;
    P.B = c.n_boxes;
    P.slots = c.slots;
    P.teams = c.teams;
    P.ownership = c.ownership;
    P.melee_cd = c.melee_cooldown;
    P.omniscient = c.omniscient;
    P.gameover = c.gameover_mode;
    P.as_ = 8 + (c.teams ? 1 : 0);
    P.r_alive = c.r_alive;
    P.r_dead = c.r_dead;
    P.r_kill = c.r_kill;
    P.r_death = c.r_death;
    P.imp0 = c.impulse[0];
    P.imp1 = c.impulse[1];
    P.imp2 = c.impulse[2];
    P.agent_health = c.agent_health;
    P.melee_range = c.melee_range;
    P.melee_damage = c.melee_damage;
    P.box_health = c.box_health;
    P.box_hx = (float)(c.box_size / 2.0);
    P.box_hy = (float)(c.box_size / 2.0);
    P.randomized = c.randomized_boxes;
    P.avg_w = c.avg_w;
    P.std_w = c.std_w;
    P.avg_h = c.avg_h;
    P.std_h = c.std_h;
    P.min_w = c.min_w;
    P.min_h = c.min_h;
    P.agent_r = (float)(c.agent_size / 2.0);
    P.bitem_r = (float)(c.box_item_size / 2.0);
    P.heal_r = (float)(c.heal_size / 2.0);
    P.box_item_offset = c.box_item_offset;
    P.healing = c.healing;
    P.pickup_r = c.pickup_radius;
    P.give_r = c.give_radius;
    P.dd_r = c.deathdrop_radius;
    P.zone_phases = c.zone_phases;
    P.zone_cooldown = c.zone_cooldown;
    P.zone_damage = c.zone_damage;
    P.zone_nr = c.zone_n_radii;
    P.zone_random = c.zone_random_centers;
    for (int k = 0; k < kMaxPhases; ++k) {
        P.zrad[k] = k < c.zone_n_radii ? c.zone_radii[k] : 0.0;
        P.zradf[k] = (float)P.zrad[k];
        if (k < MAS_MAX_ZONE_PHASES && k < c.zone_n_radii) {
            P.zfix[k][0] = c.zone_centers[k][0];
            P.zfix[k][1] = c.zone_centers[k][1];
        }
    }
    P.floor_size = c.floor_size;
    P.grid_size = c.grid_size;
    // b2CircleShape::ComputeMass + b2Body::ResetMassData (density 1)
    {
        float r = P.agent_r;
        float mass = 1.0f * kPi * r * r;
        float I = mass * (0.5f * r * r + 0.0f);
        float m = 0.0f + mass;
        float bI = 0.0f + I;
        P.inv_mass = 1.0f / m;
        bI -= m * 0.0f;
        P.inv_I = 1.0f / bI;
        P.inv_mass_rcp = 1.0 / (double)P.inv_mass;
    }
    P.lin_damp = 0.8f;  // simulation.py:114 default_damping
    P.ang_damp = 0.8f;
    // ThickRoomWalls (semantics.py:685-695)
    {
        double height = c.floor_size, width = height / c.wall_aspect_ratio;
        P.wall_poly = box_poly((float)(width / 2.0), (float)(height / 2.0), 0, 0);
        double off = c.floor_size / 2.0;
        P.wall_pos[0] = mk((float)(-off), 0.0f);
        P.wall_pos[1] = mk(0.0f, (float)off);
        P.wall_pos[2] = mk((float)off, 0.0f);
        P.wall_pos[3] = mk(0.0f, (float)(-off));
        P.wall_angle[0] = 0.0f;
        P.wall_angle[1] = (float)(3.14159265358979323846 / 2.0);
        P.wall_angle[2] = 0.0f;
        P.wall_angle[3] = (float)(3.14159265358979323846 / 2.0);
        for (int k = 0; k < kNumWalls; ++k) P.wall_q[k] = rot_of(P.wall_angle[k]);
        for (int k = 0; k < kNumWalls; ++k) {
            V2 lo = mk(3.4e38f, 3.4e38f), hi = mk(-3.4e38f, -3.4e38f);
            for (int v = 0; v < 4; ++v) {
                V2 w = xmul(P.wall_pos[k], P.wall_q[k], P.wall_poly.v[v]);
                lo = mk(w.x < lo.x ? w.x : lo.x, w.y < lo.y ? w.y : lo.y);
                hi = mk(w.x > hi.x ? w.x : hi.x, w.y > hi.y ? w.y : hi.y);
            }
            P.wall_lo[k] = lo;
            P.wall_hi[k] = hi;
        }
    }
    // Cameras vision cone (simulation.py:321-328)
    {
        V2 left = from_polar(c.cam_depth, (float)(c.cam_fov / 2.0));
        V2 center = mk(c.cam_depth, 0.0f);
        V2 right = from_polar(c.cam_depth, (float)(-c.cam_fov / 2.0));
        V2 vs[4] = {mk(0.0f, 0.0f), left, center, right};
        P.cone = poly_set4(vs);
    }
    // Lidars._endpoints (simulation.py:385-392): per-laser angle offsets, float64
    P.n_lasers = c.lidar_n_lasers;
    P.lid_depth = c.lidar_depth;
    for (int k = 0; k < P.n_lasers; ++k)
        P.lid_off[k] = (double)k * (c.lidar_fov / (double)(P.n_lasers - 1)) - c.lidar_fov / 2.0;
    build_layout(h);
    return MAS_OK;
}

extern "C" {

const char* mas_last_error(void) { return g_err.c_str(); }
int32_t mas_abi_version(void) { return MAS_ABI_VERSION; }

int mas_create(const mas_config* cfg, int64_t n_envs, int32_t device, mas_handle** out)
{
    if (!cfg || !out || n_envs <= 0) return fail(MAS_ERR_INVALID_ARG, "mas_create: null argument or n_envs <= 0");
    const mas_config& c = *cfg;
    if (c.n_agents < 2 || c.n_heals < 0 || c.n_boxes < 0 || c.slots < 0)
        return fail(MAS_ERR_INVALID_ARG, "mas_create: n_agents must be >= 2 and counts non-negative");
    if (c.grid_size * c.grid_size > 256 || c.n_agents + c.n_heals + c.n_boxes > c.grid_size * c.grid_size)
        return fail(MAS_ERR_INVALID_ARG, "mas_create: spawn grid too large (>256 cells) or too small for the spawns");
    if (c.zone_phases < 1 || c.zone_n_radii + 1 > kMaxPhases || c.zone_phases > c.zone_n_radii + 1)
        return fail(MAS_ERR_INVALID_ARG, "mas_create: unsupported safe-zone phases");
    if (c.lidar_n_lasers != 0 && (c.lidar_n_lasers < 2 || c.lidar_n_lasers > MAS_MAX_LASERS))
        return fail(MAS_ERR_INVALID_ARG, "mas_create: lidar n_lasers must be 0 or in [2, MAS_MAX_LASERS]");
    // MAS_SPLIT: how mas_step uses the side streams (mas_handle::split)
    int split_mode = kSplitDefault;
    if (const char* v = getenv("MAS_SPLIT"); v && v[0]) {
        if (!strcmp(v, "0")) split_mode = 0;
        else if (!strcmp(v, "2")) split_mode = 2;
        else
            return fail(MAS_ERR_INVALID_ARG, "mas_create: MAS_SPLIT must be 0 (one stream) or 2 (the slow split); "
                                             "modes 1 and 3 were removed (DESIGN.md 4.1.1)");
    }
    mas_handle* h = new (std::nothrow) mas_handle();
    if (!h) return fail(MAS_ERR_OOM, "mas_create: out of host memory");
    h->cfg = c;
    h->N = n_envs;
    h->device = device;
    auto fits = [&](int AM, int HM, int BM, int SM) {
        return c.n_agents <= AM && c.n_heals <= HM && c.n_boxes <= BM && c.slots <= SM;
    };
    // capacity classes: (agents, heals, boxes, slots) -- see mas_k_<class>.hip
    bool ok = false;
#ifdef MAS_HAVE_1v1
    if (!ok && fits(2, 4, 4, 4)) { h->ops = Ops{class_info_1v1(), launch_step_1v1, launch_reset_1v1, launch_view_1v1}; ok = true; }
#endif
#ifdef MAS_HAVE_2v2
    if (!ok && fits(4, 4, 4, 4)) { h->ops = Ops{class_info_2v2(), launch_step_2v2, launch_reset_2v2, launch_view_2v2}; ok = true; }
#endif
#ifdef MAS_HAVE_ffa
    if (!ok && fits(4, 16, 16, 4)) { h->ops = Ops{class_info_ffa(), launch_step_ffa, launch_reset_ffa, launch_view_ffa}; ok = true; }
#endif
#ifdef MAS_HAVE_ffal
    if (!ok && fits(4, 24, 16, 8)) { h->ops = Ops{class_info_ffal(), launch_step_ffal, launch_reset_ffal, launch_view_ffal}; ok = true; }
#endif
#ifdef MAS_HAVE_xl
    if (!ok && fits(8, 8, 8, 4)) { h->ops = Ops{class_info_xl(), launch_step_xl, launch_reset_xl, launch_view_xl}; ok = true; }
#endif
#ifdef MAS_HAVE_xxl
    if (!ok && fits(8, 20, 16, 8)) { h->ops = Ops{class_info_xxl(), launch_step_xxl, launch_reset_xxl, launch_view_xxl}; ok = true; }
#endif
    if (!ok) {
        delete h;
        return fail(MAS_ERR_UNSUPPORTED, "mas_create: no compiled capacity class fits this config (classes: " MAS_CLASS_LIST ")");
    }
    if (h->ops.info.words <= 0) {
        delete h;
        return fail(MAS_ERR_UNSUPPORTED, "mas_create: state layout check failed (StateWords vs visit_state)");
    }
    build_params(h);
    h->P.w_cont = h->ops.info.w_cont;
    h->P.w_invdt = h->ops.info.w_invdt;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&h->state, (size_t)h->ops.info.words * (size_t)state_stride(n_envs) * 4);
    if (e == hipSuccess) e = hipMemset(h->state, 0, (size_t)h->ops.info.words * (size_t)state_stride(n_envs) * 4);
    if (e == hipSuccess) e = hipMalloc(&h->seedbuf, (size_t)n_envs * 6 * 8);
    h->P.prof = nullptr;
    h->phys = nullptr;
    // [N + kListSlack] the general-path list (its shards), [8] counters, then
    // the kListShards shard counts kShardStride ints apart (256-B aligned)
    const size_t list_ints = (size_t)n_envs + kListSlack;
    const size_t shard_at = (list_ints + 8 + kShardStride - 1) / kShardStride * kShardStride;
    const size_t phys_ints = shard_at + (size_t)kListShards * kShardStride;
    if (e == hipSuccess) e = hipMalloc(&h->phys, phys_ints * sizeof(int));
    if (e == hipSuccess) e = hipMemset(h->phys, 0, phys_ints * sizeof(int));
    h->sweep = nullptr;
#if MAS_AB_KERNELS
    if (e == hipSuccess) e = hipMalloc(&h->sweep, (size_t)n_envs * 3 * kSweepAgents * sizeof(float));
#endif
    h->P.sweep = h->sweep;
    h->gen_flag = nullptr;
    if (e == hipSuccess) e = hipMalloc(&h->gen_flag, (size_t)n_envs);
    if (e == hipSuccess) e = hipMemset(h->gen_flag, 0, (size_t)n_envs);
    h->P.gen_flag = h->gen_flag;
    h->P.phys_list = h->phys;
    h->P.phys_count = h->phys ? h->phys + shard_at : nullptr;
    h->P.list_shards = 1;  // (launch_step sets the step's sharding)
    h->P.list_cap = (int)n_envs;
    h->P.bad_actions = h->phys ? h->phys + list_ints + 1 : nullptr;
    h->P.phys_last = h->phys ? h->phys + list_ints + 2 : nullptr;
    h->par = 0;
    h->sp_made = false;
    {
        h->split = h->split_default = split_mode;
        const char* k = getenv("MAS_SLOW_K");
        h->P.slow_k = k ? atoi(k) : 4;  // TOI events of an env's step that make it slow (the cap always does)
    }
    h->P.list_overflow = h->phys ? h->phys + list_ints + 3 : nullptr;
    h->slow = nullptr;
    h->slow_flag = nullptr;
    if (e == hipSuccess) e = hipMalloc(&h->slow, ((size_t)n_envs + 4) * sizeof(int));
    if (e == hipSuccess) e = hipMemset(h->slow, 0, ((size_t)n_envs + 4) * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&h->slow_flag, (size_t)n_envs);
    if (e == hipSuccess) e = hipMemset(h->slow_flag, 0, (size_t)n_envs);
    h->P.slow_list = h->slow;
    h->P.slow_count = h->slow ? h->slow + n_envs : nullptr;
    h->P.slow_prev = h->slow ? h->slow + n_envs + 1 : nullptr;
    h->P.slow_flag = h->slow_flag;
    h->slow_sig = nullptr;
    h->slow_hold = 0;
    h->P.slow_sig = nullptr;
    h->P.slow_route = 0;
    h->resetl = nullptr;
    if (e == hipSuccess) e = hipMalloc(&h->resetl, ((size_t)2 * n_envs + 2) * sizeof(int));
    if (e == hipSuccess) e = hipMemset(h->resetl, 0, ((size_t)2 * n_envs + 2) * sizeof(int));
    h->P.reset_list = h->resetl;
    h->P.reset_count = h->resetl ? h->resetl + 2 * n_envs : nullptr;
    h->P.gen_sparse = 0;
    if (e == hipSuccess) e = hipHostMalloc((void**)&h->slow_sig, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        *h->slow_sig = 0;
        e = hipHostGetDevicePointer((void**)&h->P.slow_sig, h->slow_sig, 0);
    }
    h->P.force_general = 0;
    h->P.solve_one_lane = 0;
    h->P.toi_diag = nullptr;
#ifdef MAS_PROFILE
    if (e == hipSuccess) e = hipMalloc(&h->P.prof, kProfWords * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(h->P.prof, 0, kProfWords * sizeof(unsigned long long));
#endif
    if (e != hipSuccess) {
        std::string msg = std::string("mas_create: ") + hipGetErrorString(e);
        mas_destroy(h);
        return fail(MAS_ERR_HIP, msg);
    }
    *out = h;
    return MAS_OK;
}

int mas_destroy(mas_handle* h)
{
    if (!h) return MAS_OK;
    if (h->state) (void)hipFree(h->state);
    if (h->seedbuf) (void)hipFree(h->seedbuf);
    if (h->P.prof) (void)hipFree(h->P.prof);
    if (h->phys) (void)hipFree(h->phys);
    if (h->sweep) (void)hipFree(h->sweep);
    if (h->gen_flag) (void)hipFree(h->gen_flag);
    if (h->slow) (void)hipFree(h->slow);
    if (h->resetl) (void)hipFree(h->resetl);
    if (h->slow_flag) (void)hipFree(h->slow_flag);
    if (h->slow_sig) (void)hipHostFree(h->slow_sig);
    if (h->sp_made) {
        (void)hipStreamDestroy(h->sp.side);
        (void)hipEventDestroy(h->sp.fork);
        (void)hipEventDestroy(h->sp.join);
    }
    delete h;
    return MAS_OK;
}

#ifdef MAS_PROFILE
// profiling build only (not part of the ABI): copy out and clear the per-wave
// phase records, kProfWords 8-B words (mas_env.h; units: 10 ns ticks of the
// 100 MHz constant clock).
int mas_prof_read(mas_handle* h, unsigned long long* host64)
{
    if (!h || !host64 || !h->P.prof) return fail(MAS_ERR_INVALID_ARG, "mas_prof_read: not a profiling build");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(host64, h->P.prof, kProfWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(h->P.prof, 0, kProfWords * sizeof(unsigned long long)));
    return MAS_OK;
}
#endif

int mas_get_obs_layout(const mas_handle* h, mas_obs_layout* out)
{
    if (!h || !out) return fail(MAS_ERR_INVALID_ARG, "mas_get_obs_layout: null argument");
    *out = h->layout;
    return MAS_OK;
}

int64_t mas_num_envs(const mas_handle* h) { return h ? h->N : -1; }

int mas_seed(mas_handle* h, const uint64_t* host_rng_states, void* stream)
{
    if (!h || !host_rng_states) return fail(MAS_ERR_INVALID_ARG, "mas_seed: null argument");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(h->seedbuf, host_rng_states, (size_t)h->N * 6 * 8, hipMemcpyHostToDevice, s));
    dim3 g((unsigned)((h->N + 255) / 256));
    hipLaunchKernelGGL(k_seed, g, dim3(256), 0, s, h->state, h->N, h->seedbuf, h->ops.info.w_rng, h->ops.info.w_has32);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));  // host buffer may be released after return
    return MAS_OK;
}

int mas_reset(mas_handle* h, const uint8_t* env_mask, float* obs, void* stream)
{
    if (!h) return fail(MAS_ERR_INVALID_ARG, "mas_reset: null handle");
    dim3 g((unsigned)((h->N + kWG - 1) / kWG));
    h->ops.reset(g, (hipStream_t)stream, h->P, h->state, h->N, env_mask, obs);
    HIP_TRY(hipGetLastError());
    return MAS_OK;
}

// mas_step / mas_step_x: xrow non-null writes bf16 policy-input rows instead
// of the fp32 obs rows
static int step_impl(mas_handle* h, const int8_t* actions, float* obs, uint16_t* xrow, int64_t x_ld, float* rewards,
                     uint8_t* done, int32_t auto_reset, void* stream)
{
    dim3 g((unsigned)((h->N + kWG - 1) / kWG));
    if (h->split && !h->sp_made) {
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur));
        HIP_TRY(hipSetDevice(h->device));
        // the side stream at the highest priority (MAS_SIDE_PRIO=0: default
        // priority): its few waves carry the step's longest chain
        int lo = 0, hi = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        const char* pv = getenv("MAS_SIDE_PRIO");
        const bool prio = !(pv && pv[0] == '0');
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&h->sp.side, hipStreamNonBlocking, prio ? hi : lo);
        // fork / join order work between two streams of this device only: a
        // device-scope release (no system-scope cache writeback + invalidate
        // at each record, which a default event carries)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->sp.fork, hipEventDisableTiming | hipEventReleaseToDevice);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->sp.join, hipEventDisableTiming | hipEventReleaseToDevice);
        (void)hipSetDevice(cur);
        HIP_TRY(e);
        h->sp_made = true;
    }
    // The general-path list's count is zeroed on the device after its last
    // reader (launch_step), so a one-stream step can be graph-captured and
    // replayed.  The slow list's two count slots alternate per step (this
    // step appends to one, its k_pre zeroes the other) and the slow split is a
    // host decision per step: neither may be captured, so while the caller's
    // stream is capturing (hipStreamIsCapturing) the step runs on one stream.
    Params P = h->P;
    P.xrow = xrow;
    P.x_ld = x_ld;
    if (h->par) std::swap(P.slow_count, P.slow_prev);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing((hipStream_t)stream, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    // a captured step appends nothing to the slow list (slow_route 0).  Its
    // k_pre zeroes BOTH count slots on every replay: the host's slot parity
    // flips once at capture time but not per replay, so the eager step after
    // the replays may take either slot, and the slot it takes must not hold
    // the count of the last eager step before the capture (its
    // side stream would re-run those stale entries beside the main stream).
    // mas_debug_counters then reads 0 for the captured step, whichever slot.
    P.slow_zero2 = capturing ? P.slow_count : nullptr;
    // the slow split runs while the general kernels keep flagging slow envs
    // (the signal lags the device by the steps in flight: slow envs persist
    // for many steps); without any, no slow chain
    const StepSplit* sp = nullptr;
    if (h->split == 2 && !capturing) {
        if (__atomic_load_n(h->slow_sig, __ATOMIC_RELAXED)) {
            __atomic_store_n(h->slow_sig, 0, __ATOMIC_RELAXED);
            h->slow_hold = 8;
        }
        if (h->slow_hold > 0) {
            --h->slow_hold;
            sp = &h->sp;
        }
    }
    if (h->split != 2) P.slow_k = 0;  // no slow flags, no signal
    h->ops.step(g, (hipStream_t)stream, P, h->state, h->N, actions, obs, rewards, done, auto_reset, sp);
    HIP_TRY(hipGetLastError());
    h->par ^= 1;
    return MAS_OK;
}

int mas_step(mas_handle* h, const int8_t* actions, float* obs, float* rewards, uint8_t* done, int32_t auto_reset,
             void* stream)
{
    if (!h || !actions || !obs || !rewards || !done) return fail(MAS_ERR_INVALID_ARG, "mas_step: null argument");
    return step_impl(h, actions, obs, nullptr, 0, rewards, done, auto_reset, stream);
}

// why mas_step_x cannot run this handle (nullptr: it can)
static const char* step_x_refusal(const mas_handle* h, int32_t auto_reset)
{
    const mas_config& c = h->cfg;
    if (c.lidar_n_lasers != 0) return "mas_step_x: the lidars key (k_lidar writes fp32 columns): use mas_step";
    const int am = h->ops.info.am > 0 ? h->ops.info.am : 1;
    if (auto_reset && c.grid_size * c.grid_size * (64 / am) > h->ops.info.post_union)
        return "mas_step_x: this config's auto-reset runs in the fp32 reset launch (spawn grid too large for the "
               "in-place reset): use mas_step";
    return nullptr;
}

int mas_step_x_supported(const mas_handle* h, int32_t auto_reset)
{
    if (!h) return fail(MAS_ERR_INVALID_ARG, "mas_step_x_supported: null handle");
    return step_x_refusal(h, auto_reset) ? 0 : 1;
}

int mas_step_x(mas_handle* h, const int8_t* actions, void* x_bf16, int64_t x_stride, float* rewards, uint8_t* done,
               int32_t auto_reset, void* stream)
{
    if (!h || !actions || !x_bf16 || !rewards || !done) return fail(MAS_ERR_INVALID_ARG, "mas_step_x: null argument");
    if (x_stride < h->P.D || (x_stride % 4) != 0 || (reinterpret_cast<uintptr_t>(x_bf16) & 7))
        return fail(MAS_ERR_INVALID_ARG, "mas_step_x: x_stride must be a multiple of 4 >= obs_dim, x 8-B aligned");
    if (const char* why = step_x_refusal(h, auto_reset)) return fail(MAS_ERR_UNSUPPORTED, why);
    return step_impl(h, actions, nullptr, reinterpret_cast<uint16_t*>(x_bf16), x_stride, rewards, done, auto_reset,
                     stream);
}

int mas_flush_stats(mas_handle* h, float* stats, void* stream)
{
    if (!h || !stats) return fail(MAS_ERR_INVALID_ARG, "mas_flush_stats: null argument");
    dim3 g((unsigned)((h->N + 255) / 256));
    hipLaunchKernelGGL(k_stats, g, dim3(256), 0, (hipStream_t)stream, h->state, h->N, h->ops.info.w_stats, stats);
    HIP_TRY(hipGetLastError());
    return MAS_OK;
}

int mas_render_view(mas_handle* h, int64_t env, float* out)
{
    if (!h || !out || env < 0 || env >= h->N) return fail(MAS_ERR_INVALID_ARG, "mas_render_view: bad argument");
    float* d = nullptr;
    HIP_TRY(hipMalloc(&d, MAS_RENDER_VIEW_FLOATS * sizeof(float)));
    HIP_TRY(hipMemset(d, 0, MAS_RENDER_VIEW_FLOATS * sizeof(float)));
    HIP_TRY(hipDeviceSynchronize());
    h->ops.view(nullptr, h->P, h->state, h->N, env, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, d, MAS_RENDER_VIEW_FLOATS * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIP_TRY(e);
    // host-side header: floor size and the four walls (centre, angle, half extents)
    out[10] = (float)h->P.floor_size;
    float ex = 0.0f, ey = 0.0f;
    for (int v = 0; v < 4; ++v) {
        ex = std::max(ex, std::fabs(h->P.wall_poly.v[v].x));
        ey = std::max(ey, std::fabs(h->P.wall_poly.v[v].y));
    }
    for (int k = 0; k < kNumWalls; ++k) {
        float* w = out + 12 + 5 * k;
        w[0] = h->P.wall_pos[k].x;
        w[1] = h->P.wall_pos[k].y;
        w[2] = h->P.wall_angle[k];
        w[3] = ex;
        w[4] = ey;
    }
    return MAS_OK;
}

int64_t mas_state_bytes(const mas_handle* h) { return h ? (int64_t)h->ops.info.words * state_stride(h->N) * 4 : -1; }

int mas_get_state(mas_handle* h, void* dst, void* stream)
{
    if (!h || !dst) return fail(MAS_ERR_INVALID_ARG, "mas_get_state: null argument");
    HIP_TRY(hipMemcpyAsync(dst, h->state, (size_t)mas_state_bytes(h), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return MAS_OK;
}

int mas_set_state(mas_handle* h, const void* src, void* stream)
{
    if (!h || !src) return fail(MAS_ERR_INVALID_ARG, "mas_set_state: null argument");
    HIP_TRY(hipMemcpyAsync(h->state, src, (size_t)mas_state_bytes(h), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    // the slow-list routing hints belong to the replaced trajectories
    HIP_TRY(hipMemsetAsync(h->slow_flag, 0, (size_t)h->N, (hipStream_t)stream));
    return MAS_OK;
}

namespace {
// the advantages normalised in place (mas_adv_normalize): the statistics in
// double, the scale in float, with the roundings of the torch expression
// adv.sub_(mean.float()).div_(var.sqrt().float() + 1e-8) it replaces
__global__ __launch_bounds__(256) void k_adv_norm(int64_t n, float* __restrict__ adv, const double* __restrict__ st)
{
    const double mean = st[0] / st[2];
    const double v = st[1] / st[2] - mean * mean;
    const float m = (float)mean;
    const float sd = (float)sqrt(v > 0.0 ? v : 0.0) + 1e-8f;
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 + 3 < n) {
        float4 a = *reinterpret_cast<const float4*>(adv + i0);
        a.x = (a.x - m) / sd;
        a.y = (a.y - m) / sd;
        a.z = (a.z - m) / sd;
        a.w = (a.w - m) / sd;
        *reinterpret_cast<float4*>(adv + i0) = a;
    } else {
        for (int64_t i = i0; i < n; ++i) adv[i] = (adv[i] - m) / sd;
    }
}
}  // namespace

int mas_adv_normalize(int64_t n, float* adv, const double* stats, void* stream)
{
    if (n <= 0 || !adv || !stats) return fail(MAS_ERR_INVALID_ARG, "mas_adv_normalize: need n > 0 and non-null pointers");
    if (reinterpret_cast<uintptr_t>(adv) & 15)
        return fail(MAS_ERR_INVALID_ARG, "mas_adv_normalize: adv must be 16-B aligned");
    const int64_t blocks = (n + 1023) / 1024;
    if (blocks > 0x7fffffff) return fail(MAS_ERR_INVALID_ARG, "mas_adv_normalize: n too large");
    hipLaunchKernelGGL(k_adv_norm, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, adv, stats);
    HIP_TRY(hipGetLastError());
    return MAS_OK;
}

int64_t mas_gae_scratch_doubles(int64_t n_columns)
{
    return n_columns > 0 ? 2 * ((n_columns + kGaeCols - 1) / kGaeCols) : -1;
}

int mas_gae(int32_t T, int64_t n_columns, int32_t n_agents, const float* rewards, const float* values,
            const uint8_t* done, float gamma, float lam, float* advantages, float* returns, double* adv_sums,
            double* scratch, void* stream)
{
    if (T <= 0 || n_columns <= 0 || n_agents <= 0 || n_columns % n_agents)
        return fail(MAS_ERR_INVALID_ARG, "mas_gae: need T > 0 and n_columns a positive multiple of n_agents");
    if (!rewards || !values || !done || !advantages || !returns || !adv_sums || !scratch)
        return fail(MAS_ERR_INVALID_ARG, "mas_gae: null argument");
    if ((n_columns + kGaeCols - 1) / kGaeCols > 0x7fffffff)
        return fail(MAS_ERR_INVALID_ARG, "mas_gae: n_columns too large");
    hipStream_t s = (hipStream_t)stream;
    // the per-column walk (default); MAS_GAE_SCAN=1: the wavefront scan over
    // time (measured 135 vs 61.5 us at T = 64, 65536 x 4 columns)
    const char* scan_env = getenv("MAS_GAE_SCAN");
    int nblocks;
    if (scan_env && scan_env[0] == '1') {
        nblocks = (int)((n_columns + kGaeCols - 1) / kGaeCols);
        hipLaunchKernelGGL(k_gae, dim3((unsigned)nblocks), dim3(256), 0, s, (int)T, (int64_t)n_columns, (int)n_agents,
                           rewards, values, done, gamma, lam, advantages, returns, scratch);
    } else {
        nblocks = (int)((n_columns + kGaeWalkCols - 1) / kGaeWalkCols);
        hipLaunchKernelGGL(k_gae_walk, dim3((unsigned)nblocks), dim3(256), 0, s, (int)T, (int64_t)n_columns,
                           (int)n_agents, rewards, values, done, gamma, lam, advantages, returns, scratch);
    }
    hipLaunchKernelGGL(k_gae_sums, dim3(1), dim3(256), 0, s, (const double*)scratch, nblocks, adv_sums);
    HIP_TRY(hipGetLastError());
    return MAS_OK;
}

int mas_debug_counters(mas_handle* h, int64_t* host_out)
{
    if (!h || !host_out) return fail(MAS_ERR_INVALID_ARG, "mas_debug_counters: null argument");
    int c = 0, c2 = 0;
    HIP_TRY(hipDeviceSynchronize());
    // the last step's general-path count (kept by its first post kernel) and
    // the slow-list slot it appended to (kept until the next k_pre)
    HIP_TRY(hipMemcpy(&c, h->P.phys_last, sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&c2, h->par ? h->P.slow_count : h->P.slow_prev, sizeof(int), hipMemcpyDeviceToHost));
    host_out[0] = (int64_t)c + c2;
    return MAS_OK;
}

int mas_debug_guards(mas_handle* h, int64_t* host_out)
{
    if (!h || !host_out) return fail(MAS_ERR_INVALID_ARG, "mas_debug_guards: null argument");
    int c = 0;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&c, h->P.list_overflow, sizeof(int), hipMemcpyDeviceToHost));
    host_out[0] = c;
    return MAS_OK;
}

int mas_debug_force_general(mas_handle* h, int32_t on)
{
    if (!h) return fail(MAS_ERR_INVALID_ARG, "mas_debug_force_general: null handle");
#if !MAS_AB_KERNELS
    if (on & 2) return fail(MAS_ERR_UNSUPPORTED, "mas_debug_force_general: the one-lane kernels are in libmas_ab.so only");
#endif
    if (on & 4) return fail(MAS_ERR_INVALID_ARG, "mas_debug_force_general: bit 2 (the general split) was removed");
    h->P.force_general = (on & 1) ? 1 : 0;
    h->P.solve_one_lane = (on & 2) ? 1 : 0;
    h->split = (on & 8) ? 0 : h->split_default;
    return MAS_OK;
}

int mas_invalid_actions(mas_handle* h, int64_t* host_count, int32_t reset)
{
    if (!h || !host_count) return fail(MAS_ERR_INVALID_ARG, "mas_invalid_actions: null argument");
    int c = 0;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&c, h->P.bad_actions, sizeof(int), hipMemcpyDeviceToHost));
    if (reset) HIP_TRY(hipMemset(h->P.bad_actions, 0, sizeof(int)));
    *host_count = c;
    return MAS_OK;
}

int mas_debug_set_toi_counter(mas_handle* h, int32_t* counts)
{
    if (!h) return fail(MAS_ERR_INVALID_ARG, "mas_debug_set_toi_counter: null handle");
    h->P.toi_diag = counts;
    return MAS_OK;
}

int mas_debug_gen_flags(mas_handle* h, uint8_t* flags, void* stream)
{
    if (!h || !flags) return fail(MAS_ERR_INVALID_ARG, "mas_debug_gen_flags: null argument");
    HIP_TRY(hipMemcpyAsync(flags, h->gen_flag, (size_t)h->N, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return MAS_OK;
}

int mas_sample_actions(int64_t n_rows, const float* logits, int64_t row_stride, uint64_t seed, uint64_t step,
                       int8_t* actions, float* logp, void* stream)
{
    if (n_rows <= 0 || row_stride < 15 || !logits || !actions || !logp)
        return fail(MAS_ERR_INVALID_ARG, "mas_sample_actions: bad argument");
    dim3 g((unsigned)((n_rows + 255) / 256));
    hipLaunchKernelGGL(k_sample, g, dim3(256), 0, (hipStream_t)stream, n_rows, logits, row_stride, seed, step,
                       actions, logp);
    HIP_TRY(hipGetLastError());
    return MAS_OK;
}

int64_t mas_policy_packed_bytes(int32_t obs_dim) { return obs_dim > 0 ? policy_packed_bytes(obs_dim) : -1; }

int64_t mas_policy_blocks(int64_t n_rows) { return n_rows > 0 ? policy_blocks(n_rows) : 0; }

int mas_policy_pack(int32_t obs_dim, const float* w1, const float* b1, const float* w2, const float* b2,
                    const float* w3, const float* b3, void* packed, void* stream)
{
    if (obs_dim <= 0 || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !packed)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_pack: bad argument");
    HIP_TRY(policy_pack(obs_dim, w1, b1, w2, b2, w3, b3, packed, (hipStream_t)stream));
    return MAS_OK;
}

static bool policy_x_ok(int32_t obs_dim, int64_t x_stride)
{
    return x_stride >= ((obs_dim + 15) / 16) * 16 && x_stride % 8 == 0;
}

int mas_policy_act_rows(const void* packed, int32_t obs_dim, int64_t n_rows, int64_t first_row, const float* obs,
                        void* x_bf16, int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp,
                        float* value, void* stream)
{
    if (!packed || obs_dim <= 0 || n_rows <= 0 || first_row < 0 || !obs || !actions || !logp || !value)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_act: bad argument");
    if (x_bf16 && !policy_x_ok(obs_dim, x_stride))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_act: x_stride must be a multiple of 8 >= 16*ceil(obs_dim/16)");
    if ((reinterpret_cast<uintptr_t>(obs) & 15) || (reinterpret_cast<uintptr_t>(actions) & 1) ||
        (x_bf16 && (reinterpret_cast<uintptr_t>(x_bf16) & 15)))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_act: misaligned buffer (obs/x 16 B, actions 2 B)");
    HIP_TRY(policy_act(packed, obs_dim, n_rows, obs, x_bf16, x_stride, seed, step, first_row, actions, logp, value,
                       (hipStream_t)stream));
    return MAS_OK;
}

int mas_policy_act_x(const void* packed, int32_t obs_dim, int64_t n_rows, int64_t first_row, const void* x_bf16,
                     int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp, float* value,
                     void* stream)
{
    if (!packed || obs_dim <= 0 || n_rows <= 0 || first_row < 0 || !x_bf16 || !actions || !logp || !value)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_act_x: bad argument");
    if (!policy_x_ok(obs_dim, x_stride) || (reinterpret_cast<uintptr_t>(x_bf16) & 15) ||
        (reinterpret_cast<uintptr_t>(actions) & 1))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_act_x: x 16-B aligned with a padded row stride (a multiple "
                                         "of 8 >= 16*ceil(obs_dim/16)), actions 2-B aligned");
    HIP_TRY(policy_act(packed, obs_dim, n_rows, nullptr, const_cast<void*>(x_bf16), x_stride, seed, step, first_row,
                       actions, logp, value, (hipStream_t)stream));
    return MAS_OK;
}

int mas_policy_act(const void* packed, int32_t obs_dim, int64_t n_rows, const float* obs, void* x_bf16,
                   int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp, float* value,
                   void* stream)
{
    return mas_policy_act_rows(packed, obs_dim, n_rows, 0, obs, x_bf16, x_stride, seed, step, actions, logp, value,
                               stream);
}

int mas_policy_train(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                     const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                     float vf_coef, float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                     float* partials, void* stream)
{
    if (!packed || obs_dim <= 0 || n_rows <= 0 || !x_bf16 || !actions || !old_logp || !adv || !ret || !h1 || !h2 ||
        !da1 || !da2 || !dz || !partials)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train: bad argument");
    if (!policy_x_ok(obs_dim, x_stride) || (reinterpret_cast<uintptr_t>(x_bf16) & 15))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train: x must be 16-B aligned with a padded row stride");
    HIP_TRY(policy_train(packed, obs_dim, n_rows, x_bf16, x_stride, actions, old_logp, adv, ret, clip, vf_coef,
                         ent_coef, scale, h1, h2, da1, da2, dz, n_rows, partials, (hipStream_t)stream, false));
    return MAS_OK;
}

int mas_policy_train_ld(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                        const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                        float vf_coef, float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                        int64_t ld, float* partials, void* stream)
{
    if (!packed || obs_dim <= 0 || n_rows <= 0 || !x_bf16 || !actions || !old_logp || !adv || !ret || !h1 || !h2 ||
        !da1 || !da2 || !dz || !partials || ld < n_rows)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train_ld: bad argument");
    if (!policy_x_ok(obs_dim, x_stride) || (reinterpret_cast<uintptr_t>(x_bf16) & 15))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train_ld: x must be 16-B aligned with a padded row stride");
    HIP_TRY(policy_train(packed, obs_dim, n_rows, x_bf16, x_stride, actions, old_logp, adv, ret, clip, vf_coef,
                         ent_coef, scale, h1, h2, da1, da2, dz, ld, partials, (hipStream_t)stream, false));
    return MAS_OK;
}

int mas_policy_train_rm(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                        const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                        float vf_coef, float ent_coef, float scale, void* h1, void* h2, int64_t ld_h, void* da1,
                        void* da2, void* dz, float* partials, void* stream)
{
    const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!packed || obs_dim <= 0 || n_rows <= 0 || !x_bf16 || !actions || !old_logp || !adv || !ret || !h1 || !h2 ||
        !da1 || !da2 || !dz || !partials || ld_h < 257 || (ld_h % 8) != 0)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train_rm: bad argument (ld_h >= 257, a multiple of 8)");
    if (!al16(h1) || !al16(h2) || !al16(da1) || !al16(da2) || !al16(dz))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train_rm: activation buffers must be 16-B aligned");
    if (!policy_x_ok(obs_dim, x_stride) || !al16(x_bf16))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_train_rm: x must be 16-B aligned with a padded row stride");
    HIP_TRY(policy_train(packed, obs_dim, n_rows, x_bf16, x_stride, actions, old_logp, adv, ret, clip, vf_coef,
                         ent_coef, scale, h1, h2, da1, da2, dz, ld_h, partials, (hipStream_t)stream, true));
    return MAS_OK;
}

int32_t mas_policy_rm_feature(int32_t col) { return col >= 0 && col < 256 ? policy_rm_feature(col) : -1; }

int64_t mas_policy_adam_scratch(void) { return policy_adam_scratch(); }

int mas_policy_adam(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float grad_scale,
                    float max_norm, double lr, double beta1, double beta2, double eps, int64_t step, float* scratch,
                    void* stream)
{
    if (n <= 0 || !params || !grads || !exp_avg || !exp_avg_sq || !scratch || step < 1 || !(lr >= 0.0f) ||
        !(beta1 >= 0.0f && beta1 < 1.0f) || !(beta2 >= 0.0f && beta2 < 1.0f) || !(eps >= 0.0f))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_adam: bad argument (n > 0, step >= 1, 0 <= beta < 1)");
    HIP_TRY(policy_adam(n, params, grads, exp_avg, exp_avg_sq, grad_scale, max_norm, lr, beta1, beta2, eps, step,
                        scratch, (hipStream_t)stream));
    return MAS_OK;
}

int64_t mas_policy_dw_scratch(int32_t f, int32_t g, int64_t k)
{
    return (f == 16 || f == 256) && g == 256 && k > 0 ? policy_dw_scratch(f, g, k) : -1;
}

int mas_policy_dw(int32_t f, int32_t g, int64_t k, const void* a, int64_t lda, const void* b, int64_t ldb, float* out,
                  float* scratch, void* stream)
{
    const auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!(f == 16 || f == 256) || g != 256 || k <= 0 || (k % 32) != 0 || !a || !b || !out || !scratch)
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_dw: F in {16, 256}, G = 256, K a positive multiple of 32");
    if (lda < k || ldb < k || (lda % 8) != 0 || (ldb % 8) != 0 || !al16(a) || !al16(b))
        return fail(MAS_ERR_INVALID_ARG, "mas_policy_dw: rows must be 16-B aligned (strides a multiple of 8)");
    HIP_TRY(policy_dw(f, g, k, a, lda, b, ldb, out, scratch, (hipStream_t)stream));
    return MAS_OK;
}

}  // extern "C"
