// K6 — the DRQN update (train_step_rnn, scripts/train_rnn_iterative.py:400-531) on the device.
//
// Four launches per update, every matrix product on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32):
//
//   k_dq_embed  (grads 1/3) the batch through the feature layers and the LSTM input projection for
//               all three streams (modelB on obs, modelB on next, targetB on next): per (stream,
//               32-column tile, time step) F1 = ReLU(W1 x + b1), F2 = ReLU(W2 F1 + b2) and
//               Zx = Wih F2 + bih + bhh, Zx written in the accumulator layout the recurrence starts
//               from; the obs stream's F1 / F2 kept for the weight gradients.
//   k_dq_recur  (grads 2/3) the whole recurrence, persistent: every (stream, column tile) is a group
//               of 16 workgroups, workgroup m owning LSTM units 8m..8m+7 (all four gates: one 32-row
//               MFMA tile, its Whh rows in registers, K split over the 4 waves). Per time step the
//               group exchanges h through write-through (sc1) stores + a per-workgroup step flag
//               (MI355X_MICROARCH.md hand-off table, row 1), the cell state never leaves registers.
//               Then the heads: each workgroup computes its 8 rows of the shared head and their
//               partial V / A; the obs stream's group gathers all three streams' partial Q, forms the
//               double-DQN target, smooth-L1 and dQ, the head gradients of its rows, and starts BPTT
//               from dh_T = W_S^T dS; per BPTT step dz in registers (gates and c saved by the
//               forward), dh_{t-1} = Whh^T dz as per-workgroup partials exchanged the same way.
//   k_dq_wgrad  (grads 3/3) the weight gradients: dWih = dZ F2^T, dWhh = dZ H^T and the biases over
//               all T*B columns (one workgroup per 32x32 output tile, K split over 16 waves); per
//               32-column tile dF2 = Wih^T dZ -> ReLU mask -> dW2 / db2 partials -> dF1 = W2^T dP2
//               -> dW1 / db1 partials, summed in a fixed order by the last tile to finish (arrival
//               ticket); the head gradient partials of the column tiles summed likewise.
//   k_drqn_apply (pm_drqn_apply) the NoisyLinear sigma gradients (mu gradient x epsilon), the global-
//               norm clip (fp64 partials met on an arrival ticket, summed in block order) and torch's
//               Adam, target sync: four launches per update in all.
//
// Every reduction runs in a fixed order and nothing sums through atomics, so an update is
// bit-reproducible run to run (the arrival ticket only picks which workgroup does the final sum).
#include "pm_host.h"
#include "pm_rnn.h"

namespace pm {
namespace {

constexpr int kG = 16;           // workgroups per recurrence group (8 LSTM units each)
constexpr int kNormBlocks = 256;  // k_drqn_apply blocks (fp64 norm partials, summed in block order)
constexpr int kWgA = 128;        // k_dq_wgrad: dWih / dWhh output tiles
constexpr int kWgC = 4;          // k_dq_wgrad: head-partial reduce workgroups
constexpr int kLowN = 8832;      // grad [0, kLowN): W1, b1, W2, b2 (the column-tile partials)
// per-column-tile head gradient partials (floats)
enum : int { HP_WS = 0, HP_BS = 16384, HP_V = 16512, HP_VB = 16640, HP_A = 16641, HP_AB = 17025, HP_N = 17028 };
constexpr int kHpStride = 17088;  // HP_N rounded up to 64

struct DqArgs {
    int B, T, nct, C0;
    const float *params, *target;
    float* grad;
    const float *obs, *next;
    const int32_t* act;
    const float* rew;
    const uint8_t* done;
    pm_drqn_stats* stats;
    const int32_t* enable;
    float gamma;
    float *ZX;   // [3][nct][T][16][1024]     Zx in the recurrence's accumulator layout
    float *HS;   // [3][nct][T+1][32][128] x2 h_t granules {value, tag} (the hand-off slots; slot 0 unused)
    float *F1T;  // [64][C0]                  obs stream F1 (column c = t*B + b)
    float *F2T;  // [128][C0]                 obs stream F2
    float *H;    // [128][C0]                 obs stream h_t, the input hidden of step t
    float *GS;   // [nct][T][16][64][16]      obs stream activated gates, wave-0 lane layout
    float *CS;   // [nct][T][16][64][4]       obs stream c_{t+1}
    float *dZ;   // [512][C0]
    float *QP;   // [3][nct][16][32][4] x2    partial (V, A0, A1, A2) granules of each workgroup's 8 head rows
    float *DHP;  // [nct][T][16][32][128] x2  slot t: per-workgroup partial granules of dh_{t+1}
    float *HP;   // [nct][kHpStride]          head gradient partials per column tile
    float *LP;   // [nct][4]                  loss / q sums per column tile
    float *W2P;  // [C0 / 32][kLowN]          W1 / b1 / W2 / b2 gradient partials per column tile
    double* part;
    int64_t* tstep;
    int32_t* flags;  // [0] update epoch (the granule tag base), [1] k_dq_wgrad's ticket, [2] k_drqn_apply's
    int poll_limit;  // polls per hand-off wait (pm_drqn.poll_limit: 0 = 2^20; < 0 = none, a test hook)
};
__device__ __forceinline__ int hand_limit(int pl) { return pl == 0 ? (1 << 20) : (pl < 0 ? 0 : pl); }

// workspace carve-up, 64-float aligned pieces
struct DqLayout {
    int64_t total = 0;
    int64_t add(int64_t floats) {
        const int64_t o = total;
        total += (floats + 63) / 64 * 64;
        return o;
    }
};

inline int64_t dq_layout(int B, int T, DqArgs* a, void* work) {
    const int64_t nct = B / 32, C0 = (int64_t)T * B;
    DqLayout L;
    const int64_t oZX = L.add(3 * nct * T * 16 * 1024), oHS = L.add(3 * nct * (T + 1) * 8192), oF1 = L.add(64 * C0),
                  oF2 = L.add(128 * C0), oH = L.add(128 * C0), oGS = L.add(nct * T * 16 * 1024),
                  oCS = L.add(nct * T * 16 * 256), odZ = L.add(512 * C0), oQP = L.add(3 * nct * 16 * 256),
                  oDHP = L.add(nct * T * 16 * 8192), oHP = L.add(nct * kHpStride), oLP = L.add(nct * 4),
                  oW2P = L.add(C0 / 32 * kLowN), oPart = L.add(2 * kNormBlocks), oTs = L.add(4),
                  oFl = L.add(4);
    if (a && work) {
        float* w = static_cast<float*>(work);
        a->B = B; a->T = T; a->nct = (int)nct; a->C0 = (int)C0;
        a->ZX = w + oZX; a->HS = w + oHS; a->F1T = w + oF1; a->F2T = w + oF2; a->H = w + oH; a->GS = w + oGS;
        a->CS = w + oCS; a->dZ = w + odZ; a->QP = w + oQP; a->DHP = w + oDHP; a->HP = w + oHP; a->LP = w + oLP;
        a->W2P = w + oW2P; a->part = reinterpret_cast<double*>(w + oPart);
        a->tstep = reinterpret_cast<int64_t*>(w + oTs); a->flags = reinterpret_cast<int32_t*>(w + oFl);
    }
    return L.total * 4;
}


// diagnostic builds: thread 0 of a chosen block stamps s_memrealtime (100 MHz) at phase boundaries
#ifdef PM_DIAG
#define DQ_STAMP(slot, cond)                                                                    \
    do {                                                                                        \
        if (threadIdx.x == 0 && (cond)) pm_diag_buf[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define DQ_STAMP(slot, cond) \
    do {                     \
    } while (0)
#endif
__device__ __forceinline__ bool skipped(const DqArgs& a) { return a.enable && *a.enable == 0; }

// ---------------------------------------------------------------- hand-off primitives
// In-launch hand-offs move data-tagged granules (MI355X_MICROARCH.md, R2 / handoff-1to1): each
// 8-byte granule is {value, tag} and the data IS the signal — the producer writes it with a
// write-through (sc1) 16-byte store (two granules), the consumer polls the granules themselves with
// sc1 loads until every tag matches, so no flag, no drain and no barrier sits between them. Tags
// carry the update's epoch (k_dq_embed bumps it), so a slot left by an earlier update never matches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
struct HandoffCtl {
    pm_drqn_stats* st;
    float* vflag;  // grad + PM_RNN_NPARAM + 1
    int limit;     // polls per hand-off before it counts as timed out
};
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// 4-byte write-through store / L2-coherent load (sc1), for the column-tile partials handed to the
// workgroups that sum them within the same launch (hand-off table row 1: sc1 on both sides)
__device__ __forceinline__ void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_wt(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
// two granules {v0, tag}, {v1, tag} with one 16-byte write-through store
__device__ __forceinline__ void st_g2(__amdgpu_buffer_rsrc_t r, int byte_off, float v0, float v1, uint32_t tag) {
    const u32x4 q = {__float_as_uint(v0), tag, __float_as_uint(v1), tag};
    __builtin_amdgcn_raw_buffer_store_b128(q, r, byte_off, 0, 16 /* sc1 */);
}
// Poll the granule pairs at byte offsets off[i] (16-B aligned, from base) until every tag equals
// `tag`; v[2i], v[2i+1] get the values. The polls are 8-byte agent-scope atomic loads (sc1): a
// plain or volatile-flagged buffer load is loop-invariant to the compiler and gets hoisted out of
// the poll. Wave-wide; bounded by hc.limit polls. On a timeout the values are garbage, so the update
// is voided (void_update): status bit 1 latched, and grad[PM_RNN_NPARAM + 1] (the void count) set.
// That slot rides the gradient all-reduce, so every rank's k_drqn_apply sees it and skips the Adam
// step and the target sync of that update: the parameters stay untouched and the replicas identical.
__device__ __forceinline__ void void_update(const HandoffCtl& hc) {
    atomicOr(&hc.st->status, 2);
    __hip_atomic_store(hc.vflag, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N, bool SLEEP = false>
__device__ __forceinline__ void gather(const void* base, const int (&off)[N], uint32_t tag, float (&v)[2 * N],
                                       const HandoffCtl& hc) {
    const char* b = static_cast<const char*>(base);
    for (int it = 0;; ++it) {
        uint64_t q[2 * N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const uint64_t* p = reinterpret_cast<const uint64_t*>(b + off[i]);
            q[2 * i] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            q[2 * i + 1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 2 * N; ++i) {
            ok = ok && (uint32_t)(q[i] >> 32) == tag;
            v[i] = __uint_as_float((uint32_t)q[i]);
        }
        if (__all(ok)) return;
        if (it >= hc.limit) {
            if ((threadIdx.x & 63) == 0) void_update(hc);
            return;
        }
        // (a sleep here with N > 8 makes the compiler keep the callers' arrays live across the loop:
        // thousands of spilled registers; the re-issued loads' round trip paces those polls instead)
        if constexpr (SLEEP) __builtin_amdgcn_s_sleep(2);
    }
}


// Lanes [0, n) of one wave poll one granule each (byte offset soff) until its tag equals `tag`: the
// wait for n producers costs one 8-byte load per producer per poll instead of a whole slot sweep by
// every wave (sweeping pollers congested the fabric: ~5 us per hop). Bounded like gather.
__device__ __forceinline__ void poll_tags(const void* base, int soff, int n, uint32_t tag, const HandoffCtl& hc) {
    const char* b = static_cast<const char*>(base);
    bool ok = (int)(threadIdx.x & 63) >= n;
    for (int it = 0; it < hc.limit; ++it) {
        if (!ok)
            ok = (uint32_t)(__hip_atomic_load(reinterpret_cast<const uint64_t*>(b + soff), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) >> 32) == tag;
        if (__all(ok)) return;
        __builtin_amdgcn_s_sleep(1);
    }
    if ((threadIdx.x & 63) == 0) void_update(hc);
}

// ---------------------------------------------------------------- 1: embedding + input projection
// grid: 3 streams x nct column tiles x T steps x 4 row quarters; wave w computes the Zx tile of
// recurrence workgroup m = 4 * quarter + w. Tile rows: row r' of workgroup m is gate r' >> 3 of LSTM
// unit 8m + (r' & 7), i.e. Wih / Whh row 128 (r' >> 3) + 8m + (r' & 7).
__global__ __launch_bounds__(256) void k_dq_embed(DqArgs a) {
    const int nct = a.nct, T = a.T, B = a.B;
    int bid = blockIdx.x;
    const int rq = bid & 3;
    bid >>= 2;
    const int t = bid % T;
    bid /= T;
    const int ct = bid % nct, s = bid / nct;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    if (blockIdx.x == 0 && tid == 0) {  // a new tag epoch for k_dq_recur's hand-offs; the wgrad ticket
        a.flags[0] = a.flags[0] + 1;
        a.flags[1] = 0;
        a.flags[2] = 0;  // k_drqn_apply's arrival counter (monotonic within an apply, generation-based)
    }
    if (skipped(a)) {  // this replica contributes nothing to the all-reduce
        for (int i = blockIdx.x * 256 + tid; i < PM_RNN_NPARAM + 4; i += gridDim.x * 256) a.grad[i] = 0.f;
        return;
    }
    if (blockIdx.x == 0 && tid == 0) {
        a.grad[PM_RNN_NPARAM] = 1.0f;      // this replica contributes
        a.grad[PM_RNN_NPARAM + 1] = 0.0f;  // no hand-off has timed out (yet) in this update
    }
    __shared__ __attribute__((aligned(16))) float F2s[32][132];
    DQ_STAMP(220, blockIdx.x == 0);
    const float* P = s == 2 ? a.target : a.params;
    const int b = ct * 32 + col;
    const int64_t c = (int64_t)t * B + b;
    float xs[4];
    tile_inputs((s == 0 ? a.obs : a.next) + ((int64_t)b * T + t) * 7, h, xs);
    // every weight operand of the wave is loaded up front: the Zx A fragments (64 registers) land
    // while F1 / F2 compute instead of after the F2 barrier
    const int m = 4 * rq + w;
    const float* wr = P + R_P_WIH + (int64_t)(128 * (col >> 3) + 8 * m + (col & 7)) * 128 + 4 * h;
    float4 av[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) av[j] = *reinterpret_cast<const float4*>(wr + 8 * j);
    float4 w2v[8];
    {
        const float* w2 = P + R_P_F2W + (32 * w + col) * 64 + 4 * h;
#pragma unroll
        for (int i = 0; i < 8; ++i) w2v[i] = *reinterpret_cast<const float4*>(w2 + 32 * (i >> 2) + 8 * (i & 3));
    }
    // F1 (both 32-row tiles, every wave): input k' = 2 s4 + h, k' = 0 the constant 1 (weight: b1)
    f32x16 c1[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
        const int row = 32 * jt + col;
        c1[jt] = f32x16{};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int kk = 2 * s4 + h;
            const float wv = kk == 0 ? P[R_P_F1B + row] : P[R_P_F1W + row * 7 + kk - 1];
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, xs[s4], c1[jt], 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
    }
    // F2 tile w: rows 32w + rho(r) + 4h; K = 64 over the two F1 tiles (k = 32 t2 + rho(r) + 4h)
    f32x16 f2;
#pragma unroll
    for (int r = 0; r < 16; ++r) f2[r] = P[R_P_F2B + 32 * w + rho(r) + 4 * h];
    {
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = w2v[4 * t2 + i];
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, c1[t2][4 * i + 0], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, c1[t2][4 * i + 1], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, c1[t2][4 * i + 2], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, c1[t2][4 * i + 3], f2, 0, 0, 0);
            }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) f2[r] = relu(f2[r]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(&F2s[col][32 * w + 8 * i + 4 * h]) =
            make_float4(f2[4 * i], f2[4 * i + 1], f2[4 * i + 2], f2[4 * i + 3]);
    if (s == 0 && rq == 0) {  // the obs stream's features for the weight gradients, [unit][column]
        const int64_t C0 = a.C0;
#pragma unroll
        for (int r = 0; r < 16; ++r) a.F2T[(int64_t)(32 * w + rho(r) + 4 * h) * C0 + c] = f2[r];
        if (w < 2)
#pragma unroll
            for (int r = 0; r < 16; ++r) a.F1T[(int64_t)(32 * w + rho(r) + 4 * h) * C0 + c] = c1[w][r];
    }
    __syncthreads();
    // Zx tile of recurrence workgroup m: K = 128 with k = 8j + 4h + e for k-step (j, e)
    f32x16 z;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rr = rho(r) + 4 * h;
        const int g = 128 * (rr >> 3) + 8 * m + (rr & 7);
        z[r] = P[R_P_BIH + g] + P[R_P_BHH + g];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(&F2s[col][8 * j + 4 * h]);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].x, bv.x, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].y, bv.y, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].z, bv.z, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].w, bv.w, z, 0, 0, 0);
    }
    float4* zx = reinterpret_cast<float4*>(a.ZX + ((((int64_t)s * nct + ct) * T + t) * 16 + m) * 1024) + lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) zx[64 * i] = make_float4(z[4 * i], z[4 * i + 1], z[4 * i + 2], z[4 * i + 3]);
    DQ_STAMP(222, blockIdx.x == 0);
}

// ---------------------------------------------------------------- 2: the recurrence (persistent)
struct RecurSmem {
    float red[2][4][16][64];  // the waves' partial accumulators, by step parity: a wave gathers its next
                              // h from other workgroups and may write a step ahead of a slower wave's read
    __attribute__((aligned(16))) float dzs[4][64][4];  // BPTT: wave 0's dz fragments for the other waves
    __attribute__((aligned(16))) float hT[32][132];  // h_T of this column tile [column][unit]
    float dS[8][32];                                 // dS of this workgroup's 8 shared-head rows
    float ws[8][128];                                // those rows of the effective W_S
    __attribute__((aligned(16))) float qs[3][32][4]; // the three streams' summed V / A per column
    __attribute__((aligned(16))) float dhs[4][64][4];  // BPTT: each wave's sum of 4 producers' dh partials
};

__device__ __forceinline__ float eff_w(const float* P, int mu, int sg, int ep, bool noisy) {
    return noisy ? P[mu] + P[sg] * P[ep] : P[mu];  // NoisyLinear: mu + sigma * epsilon (train), mu (eval)
}

// Slot layouts (granules, 8 B each):
//   HS  [grp][T+1][32 col][128 unit]   h_t of a (stream, column tile) group, tag E + t
//   QP  [grp][16 m][32 col][4]         the V / A partials of workgroup m's 8 shared-head rows, tag E + 1
//   DHP [ct][T][16 m][32 col][128]     workgroup m's partial of dh_{t+1} (slot t), tag E + t + 1
__global__ __launch_bounds__(256) void k_dq_recur(DqArgs a) {
    if (skipped(a)) return;
    __shared__ RecurSmem sm;
    const int nct = a.nct, T = a.T, B = a.B;
    int bid = blockIdx.x;
    const int m = bid & 15;
    bid >>= 4;
    const int ct = bid % nct, so = bid / nct;
    const int s = so == 2 ? 0 : so + 1;  // the next-state streams first: the obs stream's group waits for them
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const bool noisy = s != 2;  // modelB in train mode, targetB in eval mode
    const float* P = s == 2 ? a.target : a.params;
    const int64_t C0 = a.C0;
    const int bcol = ct * 32 + col;
    const int grp = s * nct + ct;
    const uint32_t E = (uint32_t)a.flags[0] << 7;  // this update's tag base (T + 1 < 128)
    const HandoffCtl hc{a.stats, a.grad + PM_RNN_NPARAM + 1, hand_limit(a.poll_limit)};
    [[maybe_unused]] const bool so0 = s == 0 && ct == 0 && m == 0, s10 = blockIdx.x == 0;  // stamping blocks (diag)
    DQ_STAMP(1, so0);
    DQ_STAMP(111, s10);
    float* HSg = a.HS + (int64_t)grp * (T + 1) * 8192;
    // this wave's Whh fragments: row 128 q + 8m + j of lane row col (q = col >> 3, j = col & 7), K quarter w
    float wa[16];
    {
        const float* wr = P + R_P_WHH + (int64_t)(128 * (col >> 3) + 8 * m + (col & 7)) * 128 + 32 * w + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 v = *reinterpret_cast<const float4*>(wr + 8 * j);
            wa[4 * j] = v.x; wa[4 * j + 1] = v.y; wa[4 * j + 2] = v.z; wa[4 * j + 3] = v.w;
        }
    }
    if (s == 0)  // the obs stream's rows of modelB's effective W_S (for dh_T), published by a later barrier
        for (int k = tid; k < 8 * 128; k += 256) {
            const int u = 8 * m + (k >> 7), kk = k & 127, o = u * 128 + kk;
            sm.ws[k >> 7][kk] = eff_w(a.params, R_P_SWMU + o, R_P_SWSG + o, R_P_SWEP + o, true);
        }
    // the K-quarter slot offsets of this lane: units 32w + 8j + 4h + {0..3} of column col
    int hoff[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        hoff[2 * j] = (col * 128 + 32 * w + 8 * j + 4 * h) * 8;
        hoff[2 * j + 1] = hoff[2 * j] + 16;
    }
    // Zx of this wave's unit e = w (registers 4q + w of the tile, one float of each float4 chunk q)
    const float* zx = a.ZX + ((int64_t)grp * T * 16 + m) * 1024 + lane * 4 + w;
    float c1 = 0.f;  // c of unit 8m + 4h + w, column col (each wave owns one unit per lane half)
    float zn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) zn[q] = zx[q * 256];
    // ---------------- forward
    for (int t = 0; t < T; ++t) {
        float z[4] = {zn[0], zn[1], zn[2], zn[3]};
        if (t + 1 < T)
#pragma unroll
            for (int q = 0; q < 4; ++q) zn[q] = zx[(int64_t)(t + 1) * 16 * 1024 + q * 256];
        if (t > 0) {
            float hv[16];
            int off[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) off[i] = hoff[i] + t * 32 * 128 * 8;
            // lanes 0..3 wait for the last granule of this wave's 4 producers, then the K quarter is read once
            poll_tags(HSg, ((t * 32 + 31) * 128 + 8 * (4 * w + (lane & 3)) + 7) * 8, 4, E + t, hc);
            gather<8, false>(HSg, off, E + t, hv, hc);  // h_t of the group, this wave's K quarter
            DQ_STAMP(160 + t, so0 && t < 10);
            f32x16 acc = {};
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[k], hv[k], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) sm.red[t & 1][w][r][lane] = acc[r];
            __syncthreads();
            DQ_STAMP(170 + t, so0 && t < 10);
            // unit e = w: gate q is register 4q + w of every wave's partial
#pragma unroll
            for (int q = 0; q < 4; ++q)
                z[q] = (((z[q] + sm.red[t & 1][0][4 * q + w][lane]) + sm.red[t & 1][1][4 * q + w][lane]) +
                        sm.red[t & 1][2][4 * q + w][lane]) + sm.red[t & 1][3][4 * q + w][lane];
        }
        // the cell of unit 8m + 4h + w (v_exp_f32 / v_rcp_f32 activations, a few ulp)
        const float gi = sig_hw(z[0]), gf = sig_hw(z[1]), gg = tanh_hw(z[2]), go = sig_hw(z[3]);
        c1 = gf * c1 + gi * gg;  // cy = forgetgate * cx + ingate * cellgate
        const float hn = go * tanh_hw(c1);
        __hip_atomic_store(reinterpret_cast<uint64_t*>(HSg) + ((t + 1) * 32 + col) * 128 + 8 * m + 4 * h + w,
                           ((uint64_t)(E + t + 1) << 32) | __float_as_uint(hn), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        DQ_STAMP(10 + t, so0 && t < 30);
        DQ_STAMP(120 + t, s10 && t < 30);
        if (s == 0) {  // what BPTT and the weight gradients need of the obs stream (plain stores)
            float* g = a.GS + (((int64_t)ct * T + t) * 16 + m) * 1024 + lane * 4 + w;
            g[0] = gi; g[256] = gf; g[512] = gg; g[768] = go;
            a.CS[(((int64_t)ct * T + t) * 16 + m) * 256 + lane * 4 + w] = c1;
            float* hr = a.H + (int64_t)(8 * m + 4 * h + w) * C0 + bcol;
            if (t + 1 < T) hr[(int64_t)(t + 1) * B] = hn;
            if (t == 0) hr[0] = 0.f;
        }
    }
    // ---------------- heads: rows 8m .. 8m+7 of the shared head (A rows duplicated x4 in the tile)
    // the shared head's A fragments (row 8m + (col & 7), duplicated x4; K quarter w), loaded while h_T is polled
    float wsf[16];
    {
        const int o = (8 * m + (col & 7)) * 128 + 32 * w + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = o + 8 * j + e;
                wsf[4 * j + e] = eff_w(P, R_P_SWMU + k, R_P_SWSG + k, R_P_SWEP + k, noisy);
            }
    }
    // wave 0's head weights of S rows 8m + 4h + e: bias, V, A0..2 (effective), loaded while h_T is polled
    float hw5[4][5];
    if (w == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int u = 8 * m + 4 * h + e;
            hw5[e][0] = eff_w(P, R_P_SBMU + u, R_P_SBSG + u, R_P_SBEP + u, noisy);
            hw5[e][1] = eff_w(P, R_P_VWMU + u, R_P_VWSG + u, R_P_VWEP + u, noisy);
            hw5[e][2] = eff_w(P, R_P_AWMU + u, R_P_AWSG + u, R_P_AWEP + u, noisy);
            hw5[e][3] = eff_w(P, R_P_AWMU + 128 + u, R_P_AWSG + 128 + u, R_P_AWEP + 128 + u, noisy);
            hw5[e][4] = eff_w(P, R_P_AWMU + 256 + u, R_P_AWSG + 256 + u, R_P_AWEP + 256 + u, noisy);
        }
    f32x16 sacc = {};
    {
        float hv[16];
        int off[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) off[i] = hoff[i] + T * 32 * 128 * 8;
        poll_tags(HSg, ((T * 32 + 31) * 128 + 8 * (4 * w + (lane & 3)) + 7) * 8, 4, E + T, hc);
        gather<8, false>(HSg, off, E + T, hv, hc);  // h_T
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *reinterpret_cast<float4*>(&sm.hT[col][32 * w + 8 * j + 4 * h]) =
                make_float4(hv[4 * j], hv[4 * j + 1], hv[4 * j + 2], hv[4 * j + 3]);
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(wsf[k], hv[k], sacc, 0, 0, 0);
    }
    if (w > 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.red[T & 1][w][r][lane] = sacc[r];
    __syncthreads();
    // wave 0: S rows u_e = 8m + 4h + e (registers r = e), their V / A partials
    float sv[4], sr[4];
    if (w == 0) {
        float pv = 0.f, pa0 = 0.f, pa1 = 0.f, pa2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = ((sacc[e] + sm.red[T & 1][1][e][lane]) + sm.red[T & 1][2][e][lane]) + sm.red[T & 1][3][e][lane];
            sv[e] = z + hw5[e][0];
            sr[e] = relu(sv[e]);
            pv = fmaf(hw5[e][1], sr[e], pv);
            pa0 = fmaf(hw5[e][2], sr[e], pa0);
            pa1 = fmaf(hw5[e][3], sr[e], pa1);
            pa2 = fmaf(hw5[e][4], sr[e], pa2);
        }
        pv += __shfl_xor(pv, 32);
        pa0 += __shfl_xor(pa0, 32);
        pa1 += __shfl_xor(pa1, 32);
        pa2 += __shfl_xor(pa2, 32);
        if (h == 0) {
            const __amdgpu_buffer_rsrc_t rq = rsrc(a.QP + (int64_t)grp * 16 * 256);
            st_g2(rq, (m * 32 + col) * 32, pv, pa0, E + 1);
            st_g2(rq, (m * 32 + col) * 32 + 16, pa1, pa2, E + 1);
        }
    }
    DQ_STAMP(50, so0);
    DQ_STAMP(150, s10);
    if (s != 0) return;  // block-uniform: the next-state streams are done
    // ---------------- the loss and the head gradients (obs stream)
    if (w < 3) {  // wave st gathers stream st's 16 partials of this column tile (8 per lane half)
        const int st = w;
        const float* QPs = a.QP + (int64_t)(st * nct + ct) * 16 * 256;
        float p[32];
#pragma unroll
        for (int k0 = 0; k0 < 8; k0 += 4) {
            int off[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                off[2 * k] = ((8 * h + k0 + k) * 32 + col) * 32;
                off[2 * k + 1] = off[2 * k] + 16;
            }
            float pp[16];
            gather<8, true>(QPs, off, E + 1, pp, hc);
#pragma unroll
            for (int k = 0; k < 16; ++k) p[4 * k0 + k] = pp[k];
        }
        float v = 0.f, x0 = 0.f, x1 = 0.f, x2 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) { v += p[4 * k]; x0 += p[4 * k + 1]; x1 += p[4 * k + 2]; x2 += p[4 * k + 3]; }
        v += __shfl_xor(v, 32);  // + the other half (commutative: both halves agree bit for bit)
        x0 += __shfl_xor(x0, 32);
        x1 += __shfl_xor(x1, 32);
        x2 += __shfl_xor(x2, 32);
        if (h == 0) *reinterpret_cast<float4*>(&sm.qs[st][col][0]) = make_float4(v, x0, x1, x2);
    }
    __syncthreads();
    float dV = 0.f, dA[3] = {0.f, 0.f, 0.f};
    if (w == 0) {
        float q[3][3];
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            const float4 qv = *reinterpret_cast<const float4*>(&sm.qs[st][col][0]);
            float v = qv.x, x0 = qv.y, x1 = qv.z, x2 = qv.w;
            const float* Pst = st == 2 ? a.target : a.params;
            const bool nz = st != 2;
            v += eff_w(Pst, R_P_VBMU, R_P_VBSG, R_P_VBEP, nz);
            x0 += eff_w(Pst, R_P_ABMU + 0, R_P_ABSG + 0, R_P_ABEP + 0, nz);
            x1 += eff_w(Pst, R_P_ABMU + 1, R_P_ABSG + 1, R_P_ABEP + 1, nz);
            x2 += eff_w(Pst, R_P_ABMU + 2, R_P_ABSG + 2, R_P_ABEP + 2, nz);
            const float mean = ((x0 + x1) + x2) / 3.0f;  // A.mean(dim=1)
            q[st][0] = v + (x0 - mean);
            q[st][1] = v + (x1 - mean);
            q[st][2] = v + (x2 - mean);
        }
        DQ_STAMP(51, so0);
        const int64_t jl = (int64_t)bcol * T + T - 1;  // the sequence's last step
        const int ac = a.act[jl];
        const float rl = a.rew[jl], dl = a.done[jl] ? 1.f : 0.f;
        const float qa = ac == 0 ? q[0][0] : (ac == 1 ? q[0][1] : q[0][2]);
        const int as = argmax3(q[1]);  // argmax Q_B(next) (first max)
        const float y = rl + a.gamma * q[2][as] * (1.0f - dl);
        const float d = qa - y, ad = fabsf(d);
        float lv = ad < 1.0f ? 0.5f * d * d : ad - 0.5f;  // smooth_l1, beta 1
        const float gq = fminf(fmaxf(d, -1.0f), 1.0f) / (float)B;
        dV = gq;
#pragma unroll
        for (int k = 0; k < 3; ++k) dA[k] = (k == ac ? gq : 0.f) - gq / 3.0f;
        if (m == 0) {  // loss / q sums of this column tile (lanes of half 0)
            float qs = qa;
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) { lv += __shfl_xor(lv, o); qs += __shfl_xor(qs, o); }
            if (lane == 0) { a.LP[ct * 4 + 0] = lv; a.LP[ct * 4 + 1] = qs; }
        }
        // dS of rows u_e (modelB's effective V / A weights), the head gradients of those rows
        float* HPc = a.HP + (int64_t)ct * kHpStride;
        float gv[4], ga[3][4], gb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float ds = hw5[e][1] * dV + hw5[e][2] * dA[0] + hw5[e][3] * dA[1] + hw5[e][4] * dA[2];
            const float dsm = sv[e] > 0.f ? ds : 0.f;
            sm.dS[4 * h + e][col] = dsm;
            gv[e] = dV * sr[e];
            ga[0][e] = dA[0] * sr[e];
            ga[1][e] = dA[1] * sr[e];
            ga[2][e] = dA[2] * sr[e];
            gb[e] = dsm;
        }
        // sums over the 32 columns of the half (fixed butterfly)
#pragma unroll
        for (int o = 16; o > 0; o >>= 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                gv[e] += __shfl_xor(gv[e], o);
                ga[0][e] += __shfl_xor(ga[0][e], o);
                ga[1][e] += __shfl_xor(ga[1][e], o);
                ga[2][e] += __shfl_xor(ga[2][e], o);
                gb[e] += __shfl_xor(gb[e], o);
            }
        if (col == 0)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int u = 8 * m + 4 * h + e;
                HPc[HP_V + u] = gv[e];
                HPc[HP_A + u] = ga[0][e];
                HPc[HP_A + 128 + u] = ga[1][e];
                HPc[HP_A + 256 + u] = ga[2][e];
                HPc[HP_BS + u] = gb[e];
            }
        if (m == 0) {
            float sb = dV, sa0 = dA[0], sa1 = dA[1], sa2 = dA[2];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) {
                sb += __shfl_xor(sb, o); sa0 += __shfl_xor(sa0, o); sa1 += __shfl_xor(sa1, o); sa2 += __shfl_xor(sa2, o);
            }
            if (lane == 0) { HPc[HP_VB] = sb; HPc[HP_AB] = sa0; HPc[HP_AB + 1] = sa1; HPc[HP_AB + 2] = sa2; }
        }
    }
    __syncthreads();  // dS (h_T and ws: earlier barriers)
    const float* DHc = a.DHP + (int64_t)ct * T * 16 * 8192;
    const __amdgpu_buffer_rsrc_t rDH = rsrc(DHc);
    {   // dh_T partial over this workgroup's 8 rows: thread (column, 16 units) -> slot T - 1
        const int c2 = tid >> 3, u0 = (tid & 7) * 16;
        float o16[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) o16[k] = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float ds = sm.dS[r][c2];
#pragma unroll
            for (int k = 0; k < 16; ++k) o16[k] = fmaf(sm.ws[r][u0 + k], ds, o16[k]);
        }
        const int base = ((((T - 1) * 16 + m) * 32 + c2) * 128 + u0) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) st_g2(rDH, base + 16 * i, o16[2 * i], o16[2 * i + 1], E + T);
    }
    {   // dW_S rows (partial over this column tile): thread (k', row half)
        const int kk = tid & 127, hr = tid >> 7;
        float g4[4] = {0.f, 0.f, 0.f, 0.f};
        for (int c2 = 0; c2 < 32; ++c2) {
            const float hv = sm.hT[c2][kk];
#pragma unroll
            for (int e = 0; e < 4; ++e) g4[e] = fmaf(sm.dS[4 * hr + e][c2], hv, g4[e]);
        }
        float* HPc = a.HP + (int64_t)ct * kHpStride;
#pragma unroll
        for (int e = 0; e < 4; ++e) HPc[HP_WS + (8 * m + 4 * hr + e) * 128 + kk] = g4[e];
    }
    DQ_STAMP(52, so0);
    // ---------------- BPTT
    // Whh^T fragments of this wave's output tile (units u' = 32w + col): k-step r covers gate rows
    // rho(r) + 4h of this workgroup's tile, i.e. Whh row 128 (r >> 2) + 8m + (r & 3) + 4h
    float wt[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
        wt[r] = a.params[R_P_WHH + (int64_t)(128 * (r >> 2) + 8 * m + (r & 3) + 4 * h) * 128 + 32 * w + col];
    float dc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = T - 1; t >= 0; --t) {
        float dz[16];
        float gt[16], cT[4], cP[4];  // wave 0: this step's gates and cells, loaded ahead of the dh wait
        if (w == 0) {
            const float4* g4 = reinterpret_cast<const float4*>(a.GS + (((int64_t)ct * T + t) * 16 + m) * 1024) + lane;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = g4[64 * i];
                gt[4 * i] = v.x; gt[4 * i + 1] = v.y; gt[4 * i + 2] = v.z; gt[4 * i + 3] = v.w;
            }
            const float4 cn = reinterpret_cast<const float4*>(a.CS + (((int64_t)ct * T + t) * 16 + m) * 256)[lane];
            const float4 cp = t > 0 ? reinterpret_cast<const float4*>(a.CS + (((int64_t)ct * T + t - 1) * 16 + m) * 256)[lane]
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
            cT[0] = cn.x; cT[1] = cn.y; cT[2] = cn.z; cT[3] = cn.w;
            cP[0] = cp.x; cP[1] = cp.y; cP[2] = cp.z; cP[3] = cp.w;
        }
        {   // every wave gathers 4 producers' partials of dh_{t+1} for this workgroup's units
            int off[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                off[2 * k] = ((((t * 16 + 4 * w + k) * 32) + col) * 128 + 8 * m + 4 * h) * 8;
                off[2 * k + 1] = off[2 * k] + 16;
            }
            float p[16];
            poll_tags(DHc, (((t * 16 + 4 * w + (lane & 3)) * 32 + 31) * 128 + 32 * (m >> 2) + 31) * 8, 4, E + t + 1,
                      hc);
            gather<8, false>(DHc, off, E + t + 1, p, hc);
            float d4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                d4[0] += p[4 * k]; d4[1] += p[4 * k + 1]; d4[2] += p[4 * k + 2]; d4[3] += p[4 * k + 3];
            }
            *reinterpret_cast<float4*>(&sm.dhs[w][lane][0]) = make_float4(d4[0], d4[1], d4[2], d4[3]);
        }
        DQ_STAMP(60 + t, so0 && t < 30);
        __syncthreads();  // the four waves' dh sums (dhs is rewritten only after every wave published)
        if (w == 0) {
            float dh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // the 16 producers' partials, in producer order
                const float4 v = *reinterpret_cast<const float4*>(&sm.dhs[k][lane][0]);
                dh[0] += v.x; dh[1] += v.y; dh[2] += v.z; dh[3] += v.w;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float gi = gt[e], gf = gt[4 + e], gg = gt[8 + e], go = gt[12 + e];
                const float tc = tanh_hw(cT[e]);
                const float dcc = dc[e] + dh[e] * go * (1.0f - tc * tc);
                dz[e] = dcc * gg * (gi * (1.0f - gi));
                dz[4 + e] = dcc * cP[e] * (gf * (1.0f - gf));
                dz[8 + e] = dcc * gi * (1.0f - gg * gg);
                dz[12 + e] = dh[e] * tc * (go * (1.0f - go));
                dc[e] = dcc * gf;
            }
            if (t > 0)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    *reinterpret_cast<float4*>(&sm.dzs[i][lane][0]) = make_float4(dz[4 * i], dz[4 * i + 1], dz[4 * i + 2], dz[4 * i + 3]);
        }
        const int64_t cc = (int64_t)t * B + bcol;
        if (t == 0) {  // dh_0 (the zero initial state) is not needed
            if (w == 0)
#pragma unroll
                for (int r = 0; r < 16; ++r) a.dZ[(int64_t)(128 * (r >> 2) + 8 * m + 4 * h + (r & 3)) * C0 + cc] = dz[r];
            break;
        }
        __syncthreads();  // dz fragments (reused at the next step only after every wave has published)
        if (w != 0)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = *reinterpret_cast<const float4*>(&sm.dzs[i][lane][0]);
                dz[4 * i] = v.x; dz[4 * i + 1] = v.y; dz[4 * i + 2] = v.z; dz[4 * i + 3] = v.w;
            }
        f32x16 acc = {};
        // r-th k-step: this workgroup's gate rows rho(r) + 4h (the accumulator layout of dz)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt[r], dz[r], acc, 0, 0, 0);
        const int base = ((((t - 1) * 16 + m) * 32 + col) * 128 + 32 * w + 4 * h) * 8;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            st_g2(rDH, base + 64 * i, acc[4 * i], acc[4 * i + 1], E + t);
            st_g2(rDH, base + 64 * i + 16, acc[4 * i + 2], acc[4 * i + 3], E + t);
        }
        if (w == 0)  // for the weight gradients, behind the hand-off stores in this wave's queue
#pragma unroll
            for (int r = 0; r < 16; ++r) a.dZ[(int64_t)(128 * (r >> 2) + 8 * m + 4 * h + (r & 3)) * C0 + cc] = dz[r];
        DQ_STAMP(90 + t, so0 && t < 30);
    }
    DQ_STAMP(2, so0);
}

// ---------------------------------------------------------------- 3: weight gradients
struct WgSmem {
    union {
        float red[16][16][64];          // type A: per-wave partial tiles
        struct {
            union {
                float dZs[512][32];     // type B: this column tile's dZ block (the dF2 B operands)
                float red2[4][128][33]; // type B: dF2 K-quarter partials, later dF1 partials
            };
            float dP2[128][33];
            float dP1[64][33];
            float F1s[64][33];
        } b;
    };
    float rs[16][64];
    float Xs[7][32];
    int last;
};

__global__ __launch_bounds__(1024) void k_dq_wgrad(DqArgs a) {
    if (skipped(a)) return;
    __shared__ WgSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const int64_t C0 = a.C0;
    const int B = a.B, T = a.T, nct = a.nct;
    const int nB = a.C0 / 32;
    int bid = blockIdx.x;
    DQ_STAMP(210, bid == 0);
    DQ_STAMP(200, bid == kWgA);
    if (bid < kWgA) {
        // ---- dWih (mat 0) / dWhh (mat 1) tile: rows g in [32 gt, +32), columns k' in [32 kt, +32)
        const int mat = bid >> 6, gt = (bid >> 2) & 15, kt = bid & 3;
        const float* Ar = a.dZ + (int64_t)(32 * gt + col) * C0 + 4 * h;
        const float* Br = (mat == 0 ? a.F2T : a.H) + (int64_t)(32 * kt + col) * C0 + 4 * h;
        f32x16 acc = {};
        float rsum = 0.f;
        const int nch = (int)(C0 / 8);  // 8-column chunks, round robin over the waves, 4 in flight
        for (int kc0 = w; kc0 < nch; kc0 += 64) {
            float4 av[4], bv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kc = min(kc0 + 16 * j, nch - 1);
                av[j] = *reinterpret_cast<const float4*>(Ar + 8 * kc);
                bv[j] = *reinterpret_cast<const float4*>(Br + 8 * kc);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (kc0 + 16 * j >= nch) break;  // wave-uniform
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].x, bv[j].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].y, bv[j].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].z, bv[j].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].w, bv[j].w, acc, 0, 0, 0);
                rsum += ((av[j].x + av[j].y) + av[j].z) + av[j].w;
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sm.red[w][r][lane] = acc[r];
        sm.rs[w][lane] = rsum;
        __syncthreads();
        if (w == 0) {
            float* G = a.grad + (mat == 0 ? R_P_WIH : R_P_WHH);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = sm.red[0][r][lane];
                for (int k = 1; k < 16; ++k) v += sm.red[k][r][lane];
                G[(int64_t)(32 * gt + rho(r) + 4 * h) * 128 + 32 * kt + col] = v;
            }
            DQ_STAMP(211, bid == 0);
            if (mat == 0 && kt == 0) {  // db_ih = db_hh = row sums of dZ
                float v = sm.rs[0][lane];
                for (int k = 1; k < 16; ++k) v += sm.rs[k][lane];
                v += __shfl_xor(v, 32);
                if (h == 0) { a.grad[R_P_BIH + 32 * gt + col] = v; a.grad[R_P_BHH + 32 * gt + col] = v; }
            }
        }
        return;
    }
    bid -= kWgA;
    if (bid < nB) {
        // ---- column tile: columns [c0, c0 + 32) (one time step t, batch rows b0 .. b0 + 31)
        const int64_t c0 = (int64_t)bid * 32;
        const int t = (int)(c0 / B), b0 = (int)(c0 % B);
        // the dZ block of the tile (512 rows x 128 B) global -> LDS, 8 rows per wave instruction
        for (int k = w; k < 64; k += 16) {
            const int row = 8 * k + (lane >> 3);
            __builtin_amdgcn_global_load_lds((const void*)(a.dZ + (int64_t)row * C0 + c0 + 4 * (lane & 7)),
                                             (lds_void*)&sm.b.dZs[8 * k][0], 16, 0, 0);
        }
        // dF2 = Wih^T dZ: wave (out tile ot = w & 3, K quarter kq = w >> 2), k = g = 128 kq + 2p + h
        {
            const int ot = w & 3, kq = w >> 2;
            f32x16 acc = {};
            const float* Wc = a.params + R_P_WIH + 32 * ot + col;
            float wa64[64];  // this wave's Wih^T operands, all in flight while the dZ block lands
#pragma unroll
            for (int p = 0; p < 64; ++p) wa64[p] = Wc[(int64_t)(128 * kq + 2 * p + h) * 128];
            drain();
            __syncthreads();  // the dZ block (global_load_lds) from every wave
#pragma unroll
            for (int p = 0; p < 64; ++p)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa64[p], sm.b.dZs[128 * kq + 2 * p + h][col], acc, 0, 0, 0);
            __syncthreads();  // dZs is overlaid by red2
#pragma unroll
            for (int r = 0; r < 16; ++r) sm.b.red2[kq][32 * ot + rho(r) + 4 * h][col] = acc[r];
        }
        for (int k = tid; k < 64 * 32; k += 1024) sm.b.F1s[k >> 5][k & 31] = a.F1T[(int64_t)(k >> 5) * C0 + c0 + (k & 31)];
        if (tid < 224) sm.Xs[tid % 7][tid / 7] = a.obs[((int64_t)(b0 + tid / 7) * T + t) * 7 + tid % 7];  // x of the 32 columns
        __syncthreads();
        DQ_STAMP(201, bid == 0);
        for (int k = tid; k < 128 * 32; k += 1024) {
            const int u = k >> 5, c2 = k & 31;
            const float v = ((sm.b.red2[0][u][c2] + sm.b.red2[1][u][c2]) + sm.b.red2[2][u][c2]) + sm.b.red2[3][u][c2];
            sm.b.dP2[u][c2] = a.F2T[(int64_t)u * C0 + c0 + c2] > 0.f ? v : 0.f;  // through the ReLU
        }
        __syncthreads();
        float* Wp = a.W2P + (int64_t)bid * kLowN;
        if (w < 8) {  // dW2 partial [k'][j] = sum_c dP2[k'][c] F1[j][c]: wave -> tile (k' tile w & 3, j tile w >> 2)
            const int rt = w & 3, jt = w >> 2;
            f32x16 acc = {};
#pragma unroll
            for (int p = 0; p < 16; ++p)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sm.b.dP2[32 * rt + col][2 * p + h], sm.b.F1s[32 * jt + col][2 * p + h],
                                                          acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) st_wt(&Wp[R_P_F2W + (32 * rt + rho(r) + 4 * h) * 64 + 32 * jt + col], acc[r]);
        } else if (tid < 512 + 128) {  // db2 partial
            const int u = tid - 512;
            float sb = 0.f;
            for (int c2 = 0; c2 < 32; ++c2) sb += sm.b.dP2[u][c2];
            st_wt(&Wp[R_P_F2B + u], sb);
        }
        {   // dF1 = W2^T dP2: wave (out tile jt = w & 1, K eighth ke = w >> 1), k = k' = 16 ke + 2p + h
            const int jt = w & 1, ke = w >> 1;
            f32x16 acc = {};
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int k = 16 * ke + 2 * p + h;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.params[R_P_F2W + k * 64 + 32 * jt + col], sm.b.dP2[k][col], acc, 0, 0, 0);
            }
            __syncthreads();  // red2 is free again (the dP2 pass is done)
#pragma unroll
            for (int r = 0; r < 16; ++r) sm.b.red2[ke >> 1][(ke & 1) * 64 + 32 * jt + rho(r) + 4 * h][col] = acc[r];
        }
        __syncthreads();
        for (int k = tid; k < 64 * 32; k += 1024) {
            const int j = k >> 5, c2 = k & 31;
            float v = 0.f;
#pragma unroll
            for (int ke = 0; ke < 8; ++ke) v += sm.b.red2[ke >> 1][(ke & 1) * 64 + j][c2];
            sm.b.dP1[j][c2] = sm.b.F1s[j][c2] > 0.f ? v : 0.f;
        }
        __syncthreads();
        DQ_STAMP(204, bid == 0);
        if (tid < 448) {  // dW1 partial [j][i] = sum_c dP1[j][c] x_i[c]
            const int j = tid / 7, i = tid % 7;
            float v = 0.f;
            for (int c2 = 0; c2 < 32; ++c2) v = fmaf(sm.b.dP1[j][c2], sm.Xs[i][c2], v);
            st_wt(&Wp[R_P_F1W + j * 7 + i], v);
        } else if (tid < 512) {
            const int j = tid - 448;
            float v = 0.f;
            for (int c2 = 0; c2 < 32; ++c2) v += sm.b.dP1[j][c2];
            st_wt(&Wp[R_P_F1B + j], v);
        }
        // arrival ticket: the last R column tiles to finish wait for the rest, then each sums a
        // quarter of the partials in tile order (the earlier arrivers are done, so the wait is short)
        const int R = min(4, nB);
        drain();
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            drain();
            const int k = atomicAdd(a.flags + 1, 1);
            int slot = k - (nB - R);
            if (slot >= 0) {
                const HandoffCtl hc{a.stats, a.grad + PM_RNN_NPARAM + 1, 4 * hand_limit(a.poll_limit)};
                for (int it = 0;; ++it) {
                    if (__hip_atomic_load(a.flags + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nB) break;
                    if (it >= hc.limit) { void_update(hc); slot = -1; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                drain();
            }
            sm.last = slot;
        }
        __syncthreads();
        DQ_STAMP(206, bid == 0);
        DQ_STAMP(207, sm.last == 0);
        if (sm.last < 0) return;
        const int per = (kLowN / R + 3) & ~3, lo = sm.last * per, hi = min(kLowN, lo + per);
        for (int i0 = lo + tid; i0 < hi; i0 += 4 * 1024) {  // 4 elements x 8 tiles = 32 loads in flight
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            for (int k = 0; k < nB; k += 8) {
                float x[4][8];
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int i = min(i0 + e * 1024, hi - 1);
                        x[e][j] = k + j < nB ? ld_wt(&a.W2P[(int64_t)(k + j) * kLowN + i]) : 0.f;
                    }
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (k + j < nB) v[e] += x[e][j];  // in tile order
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (i0 + e * 1024 < hi) a.grad[i0 + e * 1024] = v[e];
        }
        DQ_STAMP(208, true);
        return;
    }
    bid -= nB;
    // ---- head partials: sum over column tiles in order
    const int per = (HP_N + kWgC - 1) / kWgC, lo = bid * per, hi = min(HP_N, lo + per);
    for (int i = lo + tid; i < hi; i += 1024) {
        float v = 0.f;
        for (int k = 0; k < nct; ++k) v += a.HP[(int64_t)k * kHpStride + i];
        int dst;
        if (i < HP_BS) dst = R_P_SWMU + i;
        else if (i < HP_V) dst = R_P_SBMU + i - HP_BS;
        else if (i < HP_VB) dst = R_P_VWMU + i - HP_V;
        else if (i == HP_VB) dst = R_P_VBMU;
        else if (i < HP_AB) dst = R_P_AWMU + i - HP_A;
        else dst = R_P_ABMU + i - HP_AB;
        a.grad[dst] = v;
    }
    if (bid == 0 && tid == 0) {
        float ls = 0.f, qs = 0.f;
        for (int k = 0; k < nct; ++k) { ls += a.LP[k * 4]; qs += a.LP[k * 4 + 1]; }
        a.stats->loss = ls / (float)B;
        a.stats->q_mean = qs / (float)B;
    }
}

// NoisyLinear sigma gradients: d sigma = dW * epsilon (NoisyLinear.forward :45-46). Linear in the
// mu gradient with the same epsilon on every rank, so it is formed after the all-reduce (apply).
__device__ __forceinline__ int sigma_source(int i, int& ep) {
    if (i >= R_P_SWSG && i < R_P_SWSG + 16384) { ep = R_P_SWEP + i - R_P_SWSG; return R_P_SWMU + i - R_P_SWSG; }
    if (i >= R_P_SBSG && i < R_P_SBSG + 128) { ep = R_P_SBEP + i - R_P_SBSG; return R_P_SBMU + i - R_P_SBSG; }
    if (i >= R_P_VWSG && i < R_P_VWSG + 128) { ep = R_P_VWEP + i - R_P_VWSG; return R_P_VWMU + i - R_P_VWSG; }
    if (i == R_P_VBSG) { ep = R_P_VBEP; return R_P_VBMU; }
    if (i >= R_P_AWSG && i < R_P_AWSG + 384) { ep = R_P_AWEP + i - R_P_AWSG; return R_P_AWMU + i - R_P_AWSG; }
    if (i >= R_P_ABSG && i < R_P_ABSG + 3) { ep = R_P_ABEP + i - R_P_ABSG; return R_P_ABMU + i - R_P_ABSG; }
    return -1;
}

// ---------------------------------------------------------------- clip + Adam
struct AdamK {
    double lr, beta1, beta2, eps, max_norm;
    int64_t interval;
};

// One launch for the apply (round 3): every block forms its slice's sigma gradients and fp64 sum of
// squares, arrives on a monotonic ticket and waits for the other blocks (kNormBlocks = 256, one per
// CU: all resident), sums the 256 partials in block order — the same order in every block, so every
// block derives the identical clip coefficient — and runs Adam on its slice of the parameters.
__global__ __launch_bounds__(256) void k_drqn_apply(DqArgs a, AdamK k, float* params, float* target, float* m_,
                                                    float* v_) {
    constexpr int kPer = (PM_RNN_NP + kNormBlocks - 1) / kNormBlocks, kEl = (kPer + 255) / 256;
    __shared__ double red[256];
    __shared__ float cf[3];
    __shared__ int64_t ts_s;
    __shared__ int late;
    const float ranks = a.grad[PM_RNN_NPARAM];  // replicas that contributed (summed by the all-reduce)
    if (!(ranks > 0.f)) return;                 // grid-uniform
    if (a.grad[PM_RNN_NPARAM + 1] != 0.f) {     // a hand-off timed out on some rank: the update is void
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.stats->status, 8);
        return;                                 // grid-uniform: no Adam, no target sync, no step count
    }
    const float inv_world = 1.0f / ranks;
    const int64_t ts = a.stats->steps + 1, at = a.stats->adam_t + 1;  // read before any block's arrival
    // one slice per block for both phases, every operand loaded up front (kEl elements per thread):
    // the sigma gradients a block forms are the ones its Adam reads
    const int plo = blockIdx.x * kPer, phi = min(PM_RNN_NP, plo + kPer);
    float g[kEl], mm[kEl], vv[kEl], pr[kEl];
    double sq = 0.0;
#pragma unroll
    for (int e = 0; e < kEl; ++e) {
        const int i = plo + threadIdx.x + 256 * e;
        g[e] = 0.f; mm[e] = 0.f; vv[e] = 0.f; pr[e] = 0.f;
        if (i < phi) pr[e] = params[i];
        if (i < min(phi, PM_RNN_NPARAM)) {
            int ep;
            const int src = i >= R_P_SWSG ? sigma_source(i, ep) : -1;
            float graw = src >= 0 ? a.grad[src] * a.params[ep] : a.grad[i];
            mm[e] = m_[i];
            vv[e] = v_[i];
            if (src >= 0) a.grad[i] = graw;
            g[e] = graw * inv_world;
            sq += (double)g[e] * (double)g[e];
        }
    }
    red[threadIdx.x] = sq;
    __syncthreads();
    for (int kk = 128; kk > 0; kk >>= 1) {
        if (threadIdx.x < kk) red[threadIdx.x] += red[threadIdx.x + kk];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.part + blockIdx.x, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        drain();
        const uint32_t tk = atomicAdd(reinterpret_cast<unsigned*>(a.flags + 2), 1u);
        const uint32_t goal = (tk / kNormBlocks + 1) * kNormBlocks;  // this update's generation complete
        late = 0;
        for (int it = 0;; ++it) {
            if ((uint32_t)__hip_atomic_load(a.flags + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - goal < 0x80000000u)
                break;
            if (it >= (1 << 22)) {  // the norm would be partial: this block leaves its slice untouched
                atomicOr(&a.stats->status, 4);
                late = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (late) return;  // block-uniform
    red[threadIdx.x] = __hip_atomic_load(a.part + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (int kk = 128; kk > 0; kk >>= 1) {  // the same fixed tree in every block
        if (threadIdx.x < kk) red[threadIdx.x] += red[threadIdx.x + kk];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double ss = red[0];
        const float norm = (float)sqrt(ss);
        const float coef = (float)(k.max_norm / ((double)norm + 1e-6));  // clip_coef
        const double bc1 = 1.0 - pow(k.beta1, (double)at), bc2 = 1.0 - pow(k.beta2, (double)at);
        cf[0] = coef < 1.0f ? coef : 1.0f;  // clamp(clip_coef, max=1)
        cf[1] = (float)(k.lr / bc1);
        cf[2] = (float)sqrt(bc2);
        ts_s = ts;
        if (blockIdx.x == 0) {
            a.stats->norm = norm;
            a.stats->steps = ts;
            a.stats->adam_t = at;
        }
    }
    __syncthreads();
    const float coef = cf[0], step_size = cf[1], bc2s = cf[2];
    const bool sync = ts_s % k.interval == 0;  // targetB.load_state_dict(modelB.state_dict()) (:529-530)
#pragma unroll
    for (int e = 0; e < kEl; ++e) {
        const int i = plo + threadIdx.x + 256 * e;
        if (i >= phi) continue;
        if (i < PM_RNN_NPARAM) {
            const float gc = g[e] * coef;
            float m = mm[e], v = vv[e], p = pr[e];
            m = m + (float)(1.0 - k.beta1) * (gc - m);                  // exp_avg.lerp_(grad, 1-beta1)
            v = v * (float)k.beta2 + (float)(1.0 - k.beta2) * gc * gc;  // mul_(beta2).addcmul_(g, g, 1-beta2)
            const float denom = sqrtf(v) / bc2s + (float)k.eps;
            p = p - step_size * (m / denom);
            params[i] = p;
            m_[i] = m;
            v_[i] = v;
            if (sync) target[i] = p;
        } else if (sync) {
            target[i] = pr[e];  // the epsilon buffers
        }
    }
}

int check(const pm_drqn* d) {
    PM_REQUIRE(d, PM_E_ARG, "pm_drqn: null descriptor");
    PM_REQUIRE(d->params && d->target && d->adam_m && d->adam_v && d->grad && d->work && d->stats, PM_E_ARG,
               "pm_drqn: null buffer");
    PM_REQUIRE(d->batch >= 32 && d->batch <= 256 && d->batch % 32 == 0, PM_E_SIZE,
               "pm_drqn: batch %d (multiple of 32 in [32, 256])", d->batch);
    PM_REQUIRE(d->T >= 1 && d->T <= 64, PM_E_SIZE, "pm_drqn: T %d (1..64)", d->T);
    PM_REQUIRE(d->target_update_interval >= 1, PM_E_ARG, "pm_drqn: target_update_interval");
    PM_REQUIRE(((((uintptr_t)d->params) | ((uintptr_t)d->target) | ((uintptr_t)d->grad) | ((uintptr_t)d->work)) & 15) == 0,
               PM_E_ARG, "pm_drqn: params / target / grad / work must be 16-byte aligned");
    return PM_OK;
}

}  // namespace
}  // namespace pm

using namespace pm;

#ifdef PM_DIAG
extern "C" int pm_diag_read_drqn(uint64_t* out) {  // [256] stamps of the DRQN kernels
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_buf), sizeof(uint64_t) * 256);
}
extern "C" int pm_diag_clear_drqn(void) {
    static const unsigned long long z[256] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(pm_diag_buf), z, sizeof(z));
}
#endif

extern "C" int64_t pm_drqn_work_bytes(int32_t batch, int32_t T) {
    if (batch < 32 || batch % 32 || T < 1) return -1;
    return dq_layout(batch, T, nullptr, nullptr);
}

extern "C" int pm_drqn_grads(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    PM_REQUIRE(d->obs && d->next && d->act && d->rew && d->done, PM_E_ARG, "pm_drqn_grads: null batch");
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats; a.enable = d->enable;
    a.obs = d->obs; a.next = d->next; a.act = d->act; a.rew = d->rew; a.done = d->done;
    a.gamma = (float)d->gamma;
    a.poll_limit = d->poll_limit;
    hipLaunchKernelGGL(k_dq_embed, dim3(3 * a.nct * a.T * 4), dim3(256), 0, st, a);
    PM_LAUNCHED("k_dq_embed");
    pm_launch(PM_TIMER_DRQN, k_dq_recur, dim3(3 * a.nct * kG), dim3(256), st, a);
    PM_LAUNCHED("k_dq_recur");
    hipLaunchKernelGGL(k_dq_wgrad, dim3(kWgA + a.C0 / 32 + kWgC), dim3(1024), 0, st, a);
    PM_LAUNCHED("k_dq_wgrad");
    return PM_OK;
}

extern "C" int pm_drqn_apply(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats;
    AdamK k{d->lr, d->beta1, d->beta2, d->adam_eps, d->max_norm, d->target_update_interval};
    hipLaunchKernelGGL(k_drqn_apply, dim3(kNormBlocks), dim3(256), 0, st, a, k, d->params, d->target, d->adam_m,
                       d->adam_v);
    PM_LAUNCHED("k_drqn_apply");
    return PM_OK;
}

extern "C" int pm_drqn_update(const pm_drqn* d, void* stream) {
    if (int rc = pm_drqn_grads(d, stream)) return rc;
    return pm_drqn_apply(d, stream);
}
