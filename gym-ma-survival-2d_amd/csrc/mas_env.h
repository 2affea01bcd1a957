// mas_env.h -- one MaSurvival env step per thread (gfx950 HIP).
//
// Layout: env state is struct-of-arrays in HBM (word w of env e at
// state[w * N + e]): a wave loads / stores 64 consecutive envs' copies of a
// field with one coalesced 256-B access.  Inside the kernel the env lives in
// VGPRs (`EnvL`, every array statically indexed; runtime indices go through
// the select helpers sel/put), so the whole step -- pre_step rules, two
// Box2D-equivalent Steps, post_step rules, observation, reward, done and the
// optional auto-reset -- runs without touching memory between the state
// load and the state/obs store.
//
// Reference order is preserved exactly; every block
// cites the reference lines it restates.  Canonical orders where Box2D's is
// an implementation detail: queries/rays iterate groups in dict
// order (boxes, box_items, heals, walls, agents), contacts are solved in
// (agent-agent i<j, then agent-static agent-major) order.
#pragma once

#include "mas_math.h"
#include "ziggurat_tables.h"

// 1: test builds (make ab -> libmas_ab.so) with the one-lane general-path
// kernels of mas_ab.h (scripts/ab_solve_golden.py); 0: the product library
#ifndef MAS_AB_KERNELS
#define MAS_AB_KERNELS 0
#endif

namespace mas {

// damage causes (Health.causes values, semantics.py:490-500)
constexpr int kCauseNone = -1;
constexpr int kCauseBadge = 64;  // + team id (TeamBadge, semantics.py:917-920)
constexpr int kCauseZone = 96;   // SafeZone module instance

constexpr int kItemNone = 0, kItemHeal = 1, kItemBox = 2;
constexpr int kNumWalls = 4;
constexpr int kMaxPhases = 9;   // zone radii incl. the appended 0
constexpr int kStats = 19;      // MAS_STATS_WIDTH
constexpr int kMaxLasers = 32;  // MAS_MAX_LASERS
constexpr int kSweepAgents = 8;  // agents per env of the A/B builds' sweep buffer (mas_create)

template <int AM_, int HM_, int BM_, int SM_, int KC_>
struct Cap {
    static constexpr int AM = AM_;  // agents
    static constexpr int HM = HM_;  // heals
    static constexpr int BM = BM_;  // boxes (= box items = pending drops)
    static constexpr int SM = SM_;  // inventory slots
    static constexpr int NS = kNumWalls + BM_;            // static bodies
    static constexpr int NAA = AM_ * (AM_ - 1) / 2;       // agent-agent pairs
    static constexpr int KC = KC_;                         // compact contact slots
    static constexpr int NB = BM_ + BM_ + HM_ + kNumWalls + AM_;  // all bodies
};

// Per-config constants (host-computed, passed by value).
struct Params {
    int A, H, B, slots, teams, ownership, melee_cd, omniscient, gameover, D, as_;
    float r_alive, r_dead, r_kill, r_death;
    float imp0, imp1, imp2;
    int agent_health;
    float melee_range;
    int melee_damage, box_health;
    float box_hx, box_hy;
    int randomized;
    double avg_w, std_w, avg_h, std_h, min_w, min_h;
    float agent_r, bitem_r, heal_r, box_item_offset;
    int healing;
    float pickup_r, give_r, dd_r;
    int zone_phases, zone_cooldown, zone_damage, zone_nr, zone_random;
    double zrad[kMaxPhases];
    float zradf[kMaxPhases];
    float zfix[kMaxPhases][2];
    double floor_size;
    int grid_size;
    float inv_mass, inv_I, lin_damp, ang_damp;
    double inv_mass_rcp;  // 1 / (double)inv_mass (div_by_m, mas_physics.h)
    int w_cont;  // first state word of the contact memory (kGCont)
    int w_invdt;  // state word of inv_dt0 (b2World's previous 1/dt)
    Poly4 wall_poly;
    V2 wall_pos[kNumWalls];
    float wall_angle[kNumWalls];
    Rot wall_q[kNumWalls];
    Poly4 cone;
    V2 wall_lo[kNumWalls], wall_hi[kNumWalls];  // world AABBs of the walls (ray-cast culling)
    // observation key offsets (sorted-key layout); -1 when absent
    int o_agent, o_bi, o_bim, o_bs, o_bsm, o_box, o_boxm, o_hs, o_hsm, o_heal, o_healm, o_oth, o_othm, o_zone, o_lid;
    // Lidars (simulation.py:357-392; 0 lasers = off): laser k's angle offset
    // i*(fov/(n_lasers-1)) - fov/2. in float64 as Python computes it (:388)
    int n_lasers;
    float lid_depth;
    double lid_off[kMaxLasers];
    int* phys_list;   // envs that left the contact-free fast path this step (k_pre -> general path)
    int* phys_count;  // number of them: appended by k_pre, zeroed by the first post kernel on the caller's
                      // stream once the general path (its only reader) is done (graph-replay safe)
    // The general-path list in list_shards shards (kListShards, or 1): k_pre
    // block b appends to shard xcd_block() / ceil(blocks / list_shards)
    // (b % list_shards with MAS_XCD_SWZ=0) -- its entries at
    // phys_list[shard * list_cap ..], its count at phys_count[shard *
    // kShardStride] -- so that no single counter takes every wave's atomic
    // (memory-side atomics on one address serialise: round 4's one counter
    // cost k_pre ~17 us per wave in the PPO regime, profiles/r05e_prof_env_ppo.txt)
    int list_shards, list_cap;
    int* phys_last;   // the last step's count, copied there before the zeroing (mas_debug_counters)
    int* list_overflow;  // appends to phys_list / slow_list / reset_list refused by their bounds (mas_debug_guards)
    int* reset_list;     // [N] the done envs of this step's post kernel (auto-reset; the side stream: its own list)
    int* reset_count;    // their count: zeroed by k_pre, appended by k_post_lanes, read by the reset launch
    int reset_in_post;   // the auto-reset runs inside k_post_lanes (no reset list, no reset launch)
    int force_general;   // test diagnostics (mas_debug_force_general): every env takes the general physics path
    int solve_one_lane;  // A/B builds only (MAS_AB_KERNELS): the one-lane k_gen_solve + k_gen_toi
    uint8_t* gen_flag;  // [N] 1 = env e left the fast path this step (2: on the slow list)
    float* sweep;     // A/B builds only: [env][3 * agent slots] b2Sweep c0.x, c0.y, a0 (k_gen_solve -> k_gen_toi)
    int* toi_diag;    // test diagnostics (mas_debug_set_toi_counter): per env, TOI events + 65536 per capped SolveTOI
    int* bad_actions; // env-steps whose actions fell outside MultiDiscrete([3,3,3,2,2,2]) (clamped; mas_invalid_actions)
    // the slow split (launch_step): envs whose last general-path step had a
    // SolveTOI that hit the sub-step cap, or >= slow_k TOI events, go to
    // their own list, run on the side stream (k_pre routes, gen_flag 2)
    int* slow_list;      // [N]
    int* slow_count;     // its count slot this step: two slots alternate per split step (the split is
                         // decided on the host per mas_step, so it is never graph-captured)
    int* slow_prev;      // the other slot: k_pre zeroes it
    int* slow_zero2;     // non-null in a graph-captured step: k_pre zeroes this slot too (both slots), so the
                         // eager step after the replays appends to an empty slot whichever it takes
    uint8_t* slow_flag;  // [N] set by k_gen_solve_g, read and cleared by k_pre (cleared by resets)
    int slow_k;          // 0: no slow flags
    int slow_route;      // this step routes the flagged envs to the slow list (the slow split is on)
    int* slow_sig;       // host-mapped: set to 1 when k_gen_solve_g flags an env (the host turns the split on)
    int gen_sparse;      // k_gen_solve_g maps list entry p to (block p % grid, slot p / grid): one env per wave
                         // while the list is shorter than the grid (the slow list: the divergent SolveTOI
                         // chains of two slow envs in one wave would run one after the other)
    unsigned long long* prof;  // MAS_PROFILE builds only: per-phase wave time accumulators
    // mas_step_x: the observation rows go out as bf16 policy-input rows
    // (xrow[(e * A + i) * x_ld + c], columns c < D; nullptr: f32 obs rows)
    uint16_t* xrow;
    int64_t x_ld;
};

constexpr int kListShards = 64;   // shards of the general-path list (Params::list_shards)
constexpr int kShardStride = 64;  // ints between two shard counters (256 B: their own lines)
constexpr int kListSlack = kListShards * 64;  // list entries allocated past N (the shards' rounding)

// The slow split (launch_step): a second stream of the handle for the slow
// list's general path and post phases, forked from and joined back into the
// caller's stream by two events.  Null: the one-stream order.
struct StepSplit {
    hipStream_t side;
    hipEvent_t fork, join;
};

// Phase timing for the profiling build (make prof -> libmas_prof.so): the
// first active lane of each wave adds the constant-clock (100 MHz) time since
// the previous mark to its workgroup's LDS accumulator of phase k (every env
// kernel's workgroup is one wave); MAS_PROF_FLUSH(P, kid, base) at the
// kernel's end adds the wave's phases base .. base + 13 to its own record,
// P.prof[kProfHead + (kid * kProfBlocks + block) * 16 + q], with plain loads
// and stores (slot 14: the wave's span since MAS_PROF(P, -1), slot 15: the
// wave count); the host sums the records (profiles/prof_env.py).  Launches
// that can run at the same time (the two streams of the slow split) use
// different kids.  No atomics: round 4's marks added to one
// global counter per phase at every mark, and those contended memory-side
// atomics sat inside the timed phases.  Marks sit only at wave-convergent
// points.  Phase slots: 0-5, 7 / 8-13 the general path's world steps 1 / 2
// (kid 0; the slow list's, gen_sparse, kid 4); 20-25 k_pre_lanes (kid 1);
// 41-45 k_post_lanes (kid 2; over a list, kid 5); 37-40 k_obs (kid 3; over a
// list, kid 6).
constexpr int kProfHead = 64, kProfKernels = 7, kProfBlocks = 16384;
constexpr int kProfWords = kProfHead + kProfKernels * kProfBlocks * 16;  // 8-B words of P.prof
#ifdef MAS_PROFILE
constexpr int kProfSlots = 48;
struct ProfLds {
    unsigned long long t_last, t0;
    unsigned long long acc[kProfSlots];
};
__device__ __forceinline__ ProfLds& prof_lds()
{
    __shared__ ProfLds s;
    return s;
}
__device__ __forceinline__ bool prof_lead() { return (int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1; }
__device__ __forceinline__ void prof_mark(const Params& P, int k)
{
    const unsigned long long t = wall_clock64();
    ProfLds& s = prof_lds();
    if (prof_lead()) {
        if (k < 0) {
            for (int q = 0; q < kProfSlots; ++q) s.acc[q] = 0ull;
            s.t0 = t;
        } else {
            s.acc[k] += t - s.t_last;
        }
        s.t_last = t;
    }
}
__device__ __forceinline__ void prof_flush(const Params& P, int kid, int base)
{
    const unsigned long long t = wall_clock64();
    ProfLds& s = prof_lds();
    if (prof_lead() && blockIdx.x < (unsigned)kProfBlocks) {
        unsigned long long* rec = P.prof + kProfHead + ((int64_t)kid * kProfBlocks + blockIdx.x) * 16;
        for (int q = 0; q < 14; ++q) rec[q] += base + q < kProfSlots ? s.acc[base + q] : 0ull;
        rec[14] += t - s.t0;
        rec[15] += 1ull;
    }
}
#define MAS_PROF(P, k) ::mas::prof_mark(P, k)
#define MAS_PROF_FLUSH(P, kid, base) ::mas::prof_flush(P, kid, base)
#else
#define MAS_PROF(P, k) ((void)0)
#define MAS_PROF_FLUSH(P, kid, base) ((void)0)
#endif
enum ProfPhase { kPfLoad, kPfCollide, kPfSolve, kPfToi, kPfStore, kPfCount };

// LDS ordering inside a one-wave workgroup (every env kernel's workgroup is
// one wave): a wave's DS instructions execute in program order, so only the
// compiler must not move LDS accesses across this point (AMDGPU memory model:
// wavefront-scope fences emit nothing).  __syncthreads would also wait for
// the wave's outstanding global stores (s_waitcnt vmcnt(0)) -- in k_obs's
// column-window loop, each window's tile stores.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-aware block order of the agent-lane kernels (speed only, never
// correctness).  A one-wave block owns kWG / AM consecutive envs, so with
// AM >= 4 one 128-B line of a state word row ([word][env], 4-B words) spans
// two or more blocks; the dispatcher deals blocks round-robin over the 8
// XCDs (blocks b and b + 8 share one, MI355X_MICROARCH.md), so neighbouring
// blocks sit on different L2s and each fetches the whole line.  The
// bijective remap gives every group of XCD-mates one contiguous run of
// blocks (cdna_hip_programming.md T1).  MAS_XCD_SWZ=0: the plain order.
#ifndef MAS_XCD_SWZ
#define MAS_XCD_SWZ 1
#endif
__device__ __forceinline__ int64_t xcd_block()
{
    const int64_t b = blockIdx.x;
    if (!MAS_XCD_SWZ) return b;
    const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}
// the general-path list in XCD-aware order too: contiguous k_pre shards,
// the general kernel in runs of 16 waves (MAS_LIST_XCD=0: round 6's r06p order)
#ifndef MAS_LIST_XCD
#define MAS_LIST_XCD 1
#endif
// the same in runs of K consecutive blocks per XCD, dealt round-robin (a
// grid whose first blocks alone have work -- the general kernel over its
// list -- keeps every XCD busy); the last nb % 8K blocks keep their order
template <int K>
__device__ __forceinline__ int64_t xcd_block_run()
{
    const int64_t b = blockIdx.x;
    if (!MAS_XCD_SWZ || !MAS_LIST_XCD) return b;
    const int64_t nb = gridDim.x, full = nb - nb % (8 * K);
    if (b >= full) return b;
    const int64_t x = b % 8, i = b / 8;
    return (i / K) * (8 * K) + x * K + i % K;
}

// ---------------------------------------------------------------------------
// select helpers for runtime indices into register arrays
// ---------------------------------------------------------------------------
template <int N, class T>
MAS_HD T sel(const T (&a)[N], int i)
{
    T r = opq(a[0]);
#pragma unroll
    for (int k = 1; k < N; ++k) r = (i == k) ? opq(a[k]) : r;
    return r;
}
// every element is re-selected behind opq(): LLVM would otherwise fold the
// unrolled compare-and-store into one store at a runtime index and demote
// the whole array to scratch (each later read a memory round trip)
template <int N, class T>
MAS_HD void put(T (&a)[N], int i, T v)
{
#pragma unroll
    for (int k = 0; k < N; ++k) a[k] = opq(i == k ? v : a[k]);
}

template <int N, int M, class T>
MAS_HD T sel2(const T (&a)[N][M], int i, int j)
{
    T r = opq(a[0][0]);
#pragma unroll
    for (int p = 0; p < N; ++p)
#pragma unroll
        for (int q = 0; q < M; ++q) r = (i == p && j == q) ? opq(a[p][q]) : r;
    return r;
}
template <int N, int M, class T>
MAS_HD void put2(T (&a)[N][M], int i, int j, T v)
{
#pragma unroll
    for (int p = 0; p < N; ++p)
#pragma unroll
        for (int q = 0; q < M; ++q)
            if (i == p && j == q) a[p][q] = v;
}

// ---------------------------------------------------------------------------
// env state in registers
// ---------------------------------------------------------------------------
template <class C>
constexpr int kSeenWords = (C::NB + 3) / 4;

constexpr int kLanes = 64;  // one wave per workgroup in every env kernel

// Contact memory of one env (b2Contact: touching flag + the manifold point's
// accumulated normal / tangent impulse) for the agent-agent pairs (i<j,
// aa_index order) and the agent-static pairs (agent-major, statics = walls
// then boxes).  Kept in LDS, [word][kLanes], by the kernels that touch it
// (k_phys, k_post, k_reset): every access is by runtime pair index at LDS
// cost instead of a select over the whole table in registers.  The HBM image
// holds the same words in the same order (state group kGCont).
// env stride of the state image: N + MAS_STATE_PAD envs (a padded stride
// keeps the word rows of a power-of-two N off the same HBM channels; measured
// no change on the latency-bound env kernels, r02q1, so 0 by default -- the
// policy activations, which are bandwidth-bound, do pad: ppo.py _ACT_PAD)
#ifndef MAS_STATE_PAD
#define MAS_STATE_PAD 0
#endif
MAS_HD int64_t state_stride(int64_t N) { return N + MAS_STATE_PAD; }
MAS_HD int64_t state_index(int w, int64_t e, int64_t N) { return (int64_t)w * state_stride(N) + e; }

template <class C>
struct ContLdsStore {  // [word][kLanes] in LDS
    uint32_t* u;
    int tid;
    MAS_HD uint32_t& w(int k) const { return u[k * kLanes + tid]; }
};

template <class C>
struct ContGlbStore {  // the kGCont words of the HBM image (rare paths)
    uint32_t* st;
    int64_t N, e;
    int w0;
    MAS_HD uint32_t& w(int k) const { return st[state_index(w0 + k, e, N)]; }
};

template <class C, int S>
struct ContEnvLds {  // one env's words in LDS shared by the env's lanes, [word][S] (S envs per workgroup)
    uint32_t* u;     // this env's column
    MAS_HD uint32_t& w(int k) const { return u[k * S]; }
};

template <class C, class S = ContLdsStore<C>>
struct Cont : S {
    static constexpr int kNAA = C::NAA > 0 ? C::NAA : 1;
    static constexpr int kAAT = 0, kAST = 1, kAANI = 1 + C::AM, kAATI = kAANI + kNAA, kASNI = kAATI + kNAA,
                         kASTI = kASNI + C::AM * C::NS, kWords = kASTI + C::AM * C::NS;
    using S::w;
    MAS_HD uint32_t aat() const { return w(kAAT); }
    MAS_HD void set_aat(uint32_t v) const { w(kAAT) = v; }
    MAS_HD uint32_t ast(int i) const { return w(kAST + i); }
    MAS_HD void set_ast(int i, uint32_t v) const { w(kAST + i) = v; }
    MAS_HD float aani(int p) const { return bits_f(w(kAANI + p)); }
    MAS_HD float aati(int p) const { return bits_f(w(kAATI + p)); }
    MAS_HD void set_aani(int p, float v) const { w(kAANI + p) = f_bits(v); }
    MAS_HD void set_aati(int p, float v) const { w(kAATI + p) = f_bits(v); }
    MAS_HD float asni(int i, int s) const { return bits_f(w(kASNI + i * C::NS + s)); }
    MAS_HD float asti(int i, int s) const { return bits_f(w(kASTI + i * C::NS + s)); }
    MAS_HD void set_asni(int i, int s, float v) const { w(kASNI + i * C::NS + s) = f_bits(v); }
    MAS_HD void set_asti(int i, int s, float v) const { w(kASTI + i * C::NS + s) = f_bits(v); }
    MAS_HD static float bits_f(uint32_t u)
    {
        float f;
        __builtin_memcpy(&f, &u, 4);
        return f;
    }
    MAS_HD static uint32_t f_bits(float f)
    {
        uint32_t u;
        __builtin_memcpy(&u, &f, 4);
        return u;
    }
};



template <class C>
struct EnvL {
    // agents (slot = IndexBodies id)
    V2 c[C::AM];
    float a[C::AM];
    V2 v[C::AM];
    float w[C::AM];
    float sleep[C::AM];
    uint32_t alive_m, awake_m;
    int health[C::AM], cause[C::AM], cooldown[C::AM], inv_n[C::AM];
    int inv_meta[C::AM][C::SM];  // kind | rot<<2 | copied<<4 | (owner+1)<<8
    float inv_hx[C::AM][C::SM], inv_hy[C::AM][C::SM];
    // boxes group (list order); meta = rot | copied<<2 | hinit<<3 | (vuln+1)<<8 | (cause+1)<<16
    int nbox;
    V2 bp[C::BM];
    float bhx[C::BM], bhy[C::BM];
    int bmeta[C::BM], bhealth[C::BM];
    // box_items group; meta = rot | copied<<2 | (owner+1)<<8
    int nbi;
    V2 ip[C::BM];
    float ihx[C::BM], ihy[C::BM];
    int imeta[C::BM];
    // Object.next_spawns (dropped at the next pre_step)
    int npend;
    V2 pp[C::BM];
    float phx[C::BM], phy[C::BM];
    int pmeta[C::BM];
    // heals group
    int nheal;
    V2 hp[C::HM];
    // SafeZone
    V2 zc[kMaxPhases];
    int phase, t_cd, t_sh, endgame;
    V2 zpos;
    float zrad;
    // contact memory (touching flags + accumulated impulses) is not here: it
    // lives in LDS inside the kernels that use it (Cont below, kGCont)
    float inv_dt0;
    // numpy Generator(PCG64) state
    uint64_t st_hi, st_lo, inc_hi, inc_lo;
    uint32_t has32, u32v;
    float stats[kStats];
    // Cameras.seen as bytes: byte k of the packed words = bitmask over camera
    // positions (rank among alive agents) that see body k (BIdx order)
    uint32_t seenw[kSeenWords<C>];
};

// State groups: each phase kernel loads the groups it reads and stores the
// groups it writes (kernels in mas_kernels.inc), so a kernel's register
// footprint is its working set, not the whole env.
enum : uint32_t {
    kGDyn = 1u << 0,    // agent pose / velocity / sleep, alive & awake masks
    kGRule = 1u << 1,   // health, cause, cooldown, inventories
    kGBox = 1u << 2,    // boxes group
    kGItem = 1u << 3,   // box_items group
    kGPend = 1u << 4,   // Object.next_spawns
    kGHeal = 1u << 5,   // heals group
    kGZone = 1u << 6,   // SafeZone
    kGCont = 1u << 7,   // contact memory
    kGRng = 1u << 8,    // PCG64 stream
    kGStat = 1u << 9,   // flush_stats accumulators
    kGSeen = 1u << 10,  // camera seen-by bytes (Cameras.seen, consumed by the obs kernel)
    kGAll = (1u << 11) - 1,
};

// visit every persistent word in a fixed order; f.on gates the groups not in
// `mask` (the word cursor still advances, so offsets never depend on it).
// Groups start on 4-word boundaries: HBM image is AoSoA, word w of env e at
// state[((w / 4) * N + e) * 4 + w % 4], so a lane moves 4 words with one
// 16-B access and a wave's access is 1 KiB contiguous (state_index below).
template <class C, class F>
MAS_HD void visit_state(EnvL<C>& L, F& f, uint32_t mask = kGAll)
{
    f.on = (mask & kGDyn) != 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        f.io(L.c[i].x); f.io(L.c[i].y); f.io(L.a[i]); f.io(L.v[i].x); f.io(L.v[i].y); f.io(L.w[i]);
        f.io(L.sleep[i]);
    }
    f.io(L.alive_m); f.io(L.awake_m);
    f.align4();
    f.on = (mask & kGRule) != 0;
#pragma unroll
    for (int i = 0; i < C::AM; ++i) {
        f.io(L.health[i]); f.io(L.cause[i]); f.io(L.cooldown[i]); f.io(L.inv_n[i]);
#pragma unroll
        for (int k = 0; k < C::SM; ++k) { f.io(L.inv_meta[i][k]); f.io(L.inv_hx[i][k]); f.io(L.inv_hy[i][k]); }
    }
    f.align4();
    f.on = (mask & kGBox) != 0;
    f.io(L.nbox);
#pragma unroll
    for (int b = 0; b < C::BM; ++b) {
        f.io(L.bp[b].x); f.io(L.bp[b].y); f.io(L.bhx[b]); f.io(L.bhy[b]); f.io(L.bmeta[b]); f.io(L.bhealth[b]);
    }
    f.align4();
    f.on = (mask & kGItem) != 0;
    f.io(L.nbi);
#pragma unroll
    for (int b = 0; b < C::BM; ++b) { f.io(L.ip[b].x); f.io(L.ip[b].y); f.io(L.ihx[b]); f.io(L.ihy[b]); f.io(L.imeta[b]); }
    f.align4();
    f.on = (mask & kGPend) != 0;
    f.io(L.npend);
#pragma unroll
    for (int b = 0; b < C::BM; ++b) { f.io(L.pp[b].x); f.io(L.pp[b].y); f.io(L.phx[b]); f.io(L.phy[b]); f.io(L.pmeta[b]); }
    f.align4();
    f.on = (mask & kGHeal) != 0;
    f.io(L.nheal);
#pragma unroll
    for (int h = 0; h < C::HM; ++h) { f.io(L.hp[h].x); f.io(L.hp[h].y); }
    f.align4();
    f.on = (mask & kGZone) != 0;
#pragma unroll
    for (int k = 0; k < kMaxPhases; ++k) { f.io(L.zc[k].x); f.io(L.zc[k].y); }
    f.io(L.phase); f.io(L.t_cd); f.io(L.t_sh); f.io(L.endgame); f.io(L.zpos.x); f.io(L.zpos.y); f.io(L.zrad);
    f.align4();
    f.on = (mask & kGDyn) != 0;
    f.io(L.inv_dt0);
    f.align4();
    f.on = (mask & kGCont) != 0;
    f.cont(Cont<C>::kWords);
    f.align4();
    f.on = (mask & kGRng) != 0;
    f.io64(L.st_hi); f.io64(L.st_lo); f.io64(L.inc_hi); f.io64(L.inc_lo);
    f.io(L.has32); f.io(L.u32v);
    f.align4();
    f.on = (mask & kGStat) != 0;
#pragma unroll
    for (int k = 0; k < kStats; ++k) f.io(L.stats[k]);
    f.align4();
    f.on = (mask & kGSeen) != 0;
#pragma unroll
    for (int k = 0; k < kSeenWords<C>; ++k) f.io(L.seenw[k]);
    f.align4();
}

// compile-time word indices of the fields the light loaders read (visit_state
// order above; class_info checks them against it)
template <class C>
struct StateWords {
    static constexpr int alive = 7 * C::AM, awake = 7 * C::AM + 1;
    static constexpr int rule = (7 * C::AM + 2 + 3) & ~3;
    static constexpr int box = (rule + C::AM * (4 + 3 * C::SM) + 3) & ~3;  // nbox; box b: box + 1 + 6 b ..
};

struct WordCounter {
    int n = 0;
    bool on = true;
    MAS_HD void cont(int k) { n += k; }
    MAS_HD void align4() { n = (n + 3) & ~3; }
    template <class T> MAS_HD void io(T&) { n += 1; }
    template <class T> MAS_HD void io64(T&) { n += 2; }
};

template <class C>
inline int state_words()
{
    EnvL<C> L;
    WordCounter wc;
    visit_state(L, wc);
    return wc.n;
}

// ---------------------------------------------------------------------------
// numpy Generator(PCG64): next64 / next32 / random / random_interval / normal
// ---------------------------------------------------------------------------
template <class C>
MAS_HD uint64_t pcg_next64(EnvL<C>& L)
{
    const uint64_t mhi = 0x2360ED051FC65DA4ULL, mlo = 0x4385DF649FCCF645ULL;
    uint64_t lo = L.st_lo * mlo;
#ifdef __HIP_DEVICE_COMPILE__
    uint64_t hi = __umul64hi(L.st_lo, mlo);
#else
    uint64_t hi = (uint64_t)(((unsigned __int128)L.st_lo * mlo) >> 64);
#endif
    hi += L.st_lo * mhi + L.st_hi * mlo;
    uint64_t nlo = lo + L.inc_lo;
    uint64_t carry = nlo < lo ? 1ULL : 0ULL;
    L.st_lo = nlo;
    L.st_hi = hi + L.inc_hi + carry;
    uint64_t x = L.st_hi ^ L.st_lo;
    unsigned r = (unsigned)(L.st_hi >> 58);
    return (x >> r) | (x << ((64u - r) & 63u));
}

template <class C>
MAS_HD uint32_t pcg_next32(EnvL<C>& L)
{
    if (L.has32) {
        L.has32 = 0;
        return L.u32v;
    }
    uint64_t n = pcg_next64(L);
    L.has32 = 1;
    L.u32v = (uint32_t)(n >> 32);
    return (uint32_t)(n & 0xffffffffULL);
}

template <class C>
MAS_HD double pcg_random(EnvL<C>& L)
{
    return (double)(pcg_next64(L) >> 11) * (1.0 / 9007199254740992.0);
}

template <class C>
MAS_HD uint32_t pcg_interval32(EnvL<C>& L, uint32_t max)
{
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    do {
        v = pcg_next32(L) & mask;
    } while (v > max);
    return v;
}

template <class C>
__device__ __forceinline__ double pcg_normal(EnvL<C>& L)
{
    for (;;) {
        uint64_t r = pcg_next64(L);
        int idx = (int)(r & 0xff);
        r >>= 8;
        int sign = (int)(r & 1);
        uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
        double x = (double)rabs * mas_wi_double[idx];
        if (sign & 1) x = -x;
        if (rabs < mas_ki_double[idx]) return x;
        if (idx == 0) {
            for (;;) {
                double xx = -MAS_ZIGGURAT_NOR_INV_R * log1p(-pcg_random(L));
                double yy = -log1p(-pcg_random(L));
                if (yy + yy > xx * xx)
                    return ((rabs >> 8) & 1) ? -(MAS_ZIGGURAT_NOR_R + xx) : MAS_ZIGGURAT_NOR_R + xx;
            }
        } else {
            if (((mas_fi_double[idx - 1] - mas_fi_double[idx]) * pcg_random(L) + mas_fi_double[idx]) <
                exp(-0.5 * x * x))
                return x;
        }
    }
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
MAS_HD bool bit(uint32_t m, int i) { return (m >> i) & 1u; }
MAS_HD int team_of(const Params& P, int id) { return id < P.A / 2 ? 0 : 1; }
MAS_HD int box_rot(int meta) { return meta & 3; }
MAS_HD int box_copied(int meta) { return (meta >> 2) & 1; }
MAS_HD int box_hinit(int meta) { return (meta >> 3) & 1; }
MAS_HD int box_vuln(int meta) { return ((meta >> 8) & 0xff) - 1; }
MAS_HD int box_cause(int meta) { return ((meta >> 16) & 0xff) - 1; }
MAS_HD int mk_boxmeta(int rot, int copied, int hinit, int vuln, int cause)
{
    return rot | (copied << 2) | (hinit << 3) | ((vuln + 1) << 8) | ((cause + 1) << 16);
}
MAS_HD int it_kind(int meta) { return meta & 3; }
MAS_HD int it_rot(int meta) { return (meta >> 2) & 3; }
MAS_HD int it_copied(int meta) { return (meta >> 4) & 1; }
MAS_HD int it_owner(int meta) { return ((meta >> 8) & 0xff) - 1; }
MAS_HD int mk_itmeta(int kind, int rot, int copied, int owner)
{
    return kind | (rot << 2) | (copied << 4) | ((owner + 1) << 8);
}
// box-item / pending meta: rot | copied<<2 | (owner+1)<<8
MAS_HD int bi_rot(int meta) { return meta & 3; }
MAS_HD int bi_copied(int meta) { return (meta >> 2) & 1; }
MAS_HD int bi_owner(int meta) { return ((meta >> 8) & 0xff) - 1; }
MAS_HD int mk_bimeta(int rot, int copied, int owner) { return rot | (copied << 2) | ((owner + 1) << 8); }

constexpr Rot kIdRot = {0.0f, 1.0f};

template <int N>
MAS_HD int aa_index(int i, int j)
{
    // pair (i<j) index in row-major upper-triangle order
    return i * N - (i * (i + 1)) / 2 + (j - i - 1);
}

// wake (b2Body::SetAwake(true))
template <class C>
MAS_HD void wake(EnvL<C>& L, int i)
{
    if (!bit(L.awake_m, i)) {
        L.awake_m |= 1u << i;
        put(L.sleep, i, 0.0f);
    }
}

// ---------------------------------------------------------------------------
// static body geometry (walls 0..3, then boxes in list order)
// ---------------------------------------------------------------------------
struct StaticG {
    V2 p;
    Rot q;
    float angle;
    Poly4 poly;
};

template <class C>
MAS_HD StaticG static_geom(const EnvL<C>& L, const Params& P, int s)
{
    StaticG g;
    if (s < kNumWalls) {
        g.p = P.wall_pos[s];
        g.q = P.wall_q[s];
        g.angle = P.wall_angle[s];
        g.poly = P.wall_poly;
    } else {
        int b = s - kNumWalls;
        g.p = L.bp[b];
        g.q = kIdRot;
        g.angle = 0.0f;
        g.poly = box_poly(L.bhx[b], L.bhy[b], box_rot(L.bmeta[b]), box_copied(L.bmeta[b]));
    }
    return g;
}

// runtime static index -> geometry (select)
template <class C>
MAS_HD StaticG static_geom_dyn(const EnvL<C>& L, const Params& P, int s)
{
    // runtime s: select the raw inputs, then build the polygon once
    StaticG g;
    V2 wp = opq(P.wall_pos[0]);
    Rot wq = P.wall_q[0];
    float wa = P.wall_angle[0];
#pragma unroll
    for (int k = 1; k < kNumWalls; ++k)
        if (s == k) { wp = opq(P.wall_pos[k]); wq.s = opq(P.wall_q[k].s); wq.c = opq(P.wall_q[k].c); wa = opq(P.wall_angle[k]); }
    const int b = s - kNumWalls;
    V2 bp = opq(L.bp[0]);
    float hx = opq(L.bhx[0]), hy = opq(L.bhy[0]);
    int meta = opq(L.bmeta[0]);
#pragma unroll
    for (int k = 1; k < C::BM; ++k)
        if (b == k) { bp = opq(L.bp[k]); hx = opq(L.bhx[k]); hy = opq(L.bhy[k]); meta = opq(L.bmeta[k]); }
    if (s < kNumWalls) {
        g.p = wp;
        g.q = wq;
        g.angle = wa;
        g.poly = P.wall_poly;
    } else {
        g.p = bp;
        g.q = kIdRot;
        g.angle = 0.0f;
        g.poly = box_poly(hx, hy, box_rot(meta), box_copied(meta));
    }
    return g;
}

}  // namespace mas
