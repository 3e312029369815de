// K6 — the DRQN update (train_step_rnn, scripts/train_rnn_iterative.py:400-531) on the device.
//
// Four launches per update; the batched products on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32), the
// per-sequence recurrence on the f32 VALU (same 32 fmaf / cycle / SIMD as the f32 MFMA on gfx950):
//
//   k_dq_embed  (grads 1/3) the batch through the feature layers and the LSTM input projection for
//               all three streams (modelB on obs, modelB on next, targetB on next): per (stream,
//               32-column tile, time step) F1 = ReLU(W1 x + b1), F2 = ReLU(W2 F1 + b2) and
//               Zx = Wih F2 + bih + bhh, Zx written [stream][t][gate row][sequence]; the obs stream's
//               F1 / F2 kept for the weight gradients; the effective head weights of modelB (train
//               mode) and targetB (eval mode) for the recurrence's heads.
//   k_dq_recur  (grads 2/3) the recurrence, one 1024-thread workgroup per sequence (modelB: obs and
//               next as two columns; targetB: two sequences' next), Whh in registers, no per-step
//               hand-off between CUs: forward, heads, the double-DQN target (targetB's Q(s_T) is the
//               one granule hand-off), smooth-L1 and dQ, dS, dh_T = W_S^T dS and BPTT with
//               dh_{t-1} = Whh^T dz summed in a fixed order through LDS.
//   k_dq_wgrad  (grads 3/3) the weight gradients: dWih = dZ F2^T, dWhh = dZ H^T and the biases over
//               all T*B columns, dW_S = dS h_T^T and db_S over the B sequences (one workgroup per
//               32x32 output tile, K split over 16 waves); per 32-column tile dF2 = Wih^T dZ -> ReLU
//               mask -> dW2 / db2 partials -> dF1 = W2^T dP2 -> dW1 / db1 partials (the dF2 trailer
//               of k_dq_recur forms dP2 / dP1); the V / A head gradients summed over the sequences in
//               order; on one replica each tile's fp64 share of the clip norm.
//   k_drqn_apply (pm_drqn_apply) the NoisyLinear sigma gradients (mu gradient x epsilon), the global-
//               norm clip (the tiles' shares in a fixed tree; replicas that all-reduce get the same
//               shares of the summed gradient from k_dq_norm) and torch's Adam, target sync: four
//               launches per update in all.
//
// Every reduction runs in a fixed order and nothing sums through atomics, so an update is
// bit-reproducible run to run.
#include "pm_host.h"
#include "pm_rnn.h"

namespace pm {
namespace {

constexpr int kRecThreads = 1024;  // k_dq_recur workgroup: thread 8u + kg = (LSTM unit u, K eighth kg)
constexpr int kNormBlocks = 256;  // k_drqn_apply blocks (fp64 norm partials, summed in block order)
constexpr int kWsStride = 132;   // row stride (floats) of the effective shared-head W image (WSE, LDS)
constexpr int kHwN = 704;        // HWE per net: b_S, w_V, w_A (3 x 128), b_V, b_A (3), padded
enum : int { HW_BS = 0, HW_V = 128, HW_A = 256, HW_VB = 640, HW_AB = 641 };
enum : int { SC_DV = 0, SC_DA = 1, SC_LOSS = 4, SC_Q = 5 };  // SC [B][8]: per-sequence head scalars

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
    float *ZX;   // [3][T][512][B]            Zx = Wih F2 + bih + bhh per (stream, step, gate row, sequence)
    float *F1T;  // [64][C0]                  obs stream F1 (column c = t*B + b)
    float *F2T;  // [128][C0]                 obs stream F2
    float *H;    // [128][C0]                 obs stream h_t, the input hidden of step t
    float *GC;   // [B][T][5][128]            obs stream activated gates i, f, g, o and c_{t+1} (BPTT scratch)
    float *dZ;   // [512][C0]
    float *QT;   // [B][4] x2                 targetB's Q(s_T) per sequence, granules {value, tag}
    float *DS;   // [128][B]                  obs stream dS (ReLU-masked shared-head gradient)
    float *SR;   // [128][B]                  obs stream ReLU(S)
    float *HT;   // [128][B]                  obs stream h_T
    float *SC;   // [B][8]                    dV, dA0..2, loss, Q(s, a)
    float *WSE;  // [2][128][kWsStride]       effective W_S of modelB (train mode) and targetB (eval)
    float *HWE;  // [2][kHwN]                 their effective head vectors
    float *DZH;  // [B][T][128][4] x2         obs stream dz granules {value, tag}, BPTT -> the dF2 trailer
    float *dP2;  // [128][C0]                 dF2 through F2's ReLU
    float *dP1;  // [64][C0]                  dF1 through F1's ReLU
    float *XT;   // [32][C0]                  obs stream inputs x^T (rows 7..31 zero)
    double* part;
    double* NP;      // [kWgTiles + 1] per-block sums of squares of the final gradient (local_norm)
    int64_t* tstep;  // [2] steps, adam_t as k_dq_wgrad found them (the apply's counters)
    int32_t* flags;  // [0] update epoch (the granule tag base); [1], [2] unused since round 6
    int poll_limit;  // polls per hand-off wait (pm_drqn.poll_limit: 0 = 2^20; < 0 = none, a test hook)
    int local_norm;  // 1: one replica (pm_drqn_update): k_dq_wgrad's blocks sum the clip norm's squares
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
    const int64_t oZX = L.add(3 * C0 * 512), oF1 = L.add(64 * C0), oF2 = L.add(128 * C0), oH = L.add(128 * C0),
                  oGC = L.add(C0 * 5 * 128), odZ = L.add(512 * C0), oQT = L.add((int64_t)B * 8),
                  oDS = L.add(128 * (int64_t)B), oSR = L.add(128 * (int64_t)B), oHT = L.add(128 * (int64_t)B),
                  oSC = L.add((int64_t)B * 8), oWSE = L.add(2 * 128 * kWsStride), oHWE = L.add(2 * kHwN),
                  oDZH = L.add(C0 * 1024), odP2 = L.add(128 * C0), odP1 = L.add(64 * C0),
                  oXT = L.add(32 * C0), oPart = L.add(2 * kNormBlocks), oNP = L.add(2 * 256), oTs = L.add(4),
                  oFl = L.add(4);
    if (a && work) {
        float* w = static_cast<float*>(work);
        a->B = B; a->T = T; a->nct = (int)nct; a->C0 = (int)C0;
        a->ZX = w + oZX; a->F1T = w + oF1; a->F2T = w + oF2; a->H = w + oH; a->GC = w + oGC; a->dZ = w + odZ;
        a->QT = w + oQT; a->DS = w + oDS; a->SR = w + oSR; a->HT = w + oHT; a->SC = w + oSC; a->WSE = w + oWSE;
        a->HWE = w + oHWE; a->DZH = w + oDZH; a->dP2 = w + odP2; a->dP1 = w + odP1; a->XT = w + oXT; a->part = reinterpret_cast<double*>(w + oPart); a->NP = reinterpret_cast<double*>(w + oNP);
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
__device__ __forceinline__ float eff_w(const float* P, int mu, int sg, int ep, bool noisy) {
    return noisy ? P[mu] + P[sg] * P[ep] : P[mu];  // NoisyLinear: mu + sigma * epsilon (train), mu (eval)
}

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
// grid: 3 streams x nct column tiles x T steps x 4 row quarters (main blocks, 8 waves), then
// kEmbEff blocks for the effective head weights. In a main block waves 0..3 compute F2 tile w (every
// wave of the four computes F1 first); then wave w computes half the K of Zx tile m = 4 quarter +
// (w & 3) (K half w >> 2: 32 MFMAs instead of 64 on one wave), the halves meeting in LDS. Tile rows:
// row r' of tile m is gate r' >> 3 of LSTM unit 8m + (r' & 7), i.e. Wih row 128 (r' >> 3) + 8m + (r' & 7).
constexpr int kEmbEff = 16;
__global__ __launch_bounds__(512) void k_dq_embed(DqArgs a) {
    const int nct = a.nct, T = a.T, B = a.B;
    const int nMain = 3 * nct * T * 4;
    int bid = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    if (blockIdx.x == 0 && tid == 0) a.flags[0] = a.flags[0] + 1;  // a new tag epoch for k_dq_recur's hand-offs
    if (skipped(a)) {  // this replica contributes nothing to the all-reduce
        for (int i = blockIdx.x * 512 + tid; i < PM_RNN_NPARAM + 4; i += gridDim.x * 512) a.grad[i] = 0.f;
        return;
    }
    if (blockIdx.x == 0 && tid == 0) {
        a.grad[PM_RNN_NPARAM] = 1.0f;      // this replica contributes
        a.grad[PM_RNN_NPARAM + 1] = 0.0f;  // no hand-off has timed out (yet) in this update
    }
    if (bid >= nMain) {
        // the effective head weights the recurrence's workgroups read (modelB in train mode: mu + sigma
        // * epsilon; targetB in eval mode: mu), W_S in the padded row image k_dq_recur copies to LDS
        for (int i = (bid - nMain) * 512 + tid; i < 2 * (16384 + 644); i += kEmbEff * 512) {
            const int n = i >= 16384 + 644, j = i - n * (16384 + 644);
            const float* Pn = n ? a.target : a.params;
            if (j < 16384) {
                a.WSE[(n * 128 + (j >> 7)) * kWsStride + (j & 127)] = eff_w(Pn, R_P_SWMU + j, R_P_SWSG + j, R_P_SWEP + j, !n);
            } else {
                const int v = j - 16384;  // b_S 128 | w_V 128 | w_A 384 | b_V | b_A 3
                int mu, sg, ep;
                if (v < 128) { mu = R_P_SBMU + v; sg = R_P_SBSG + v; ep = R_P_SBEP + v; }
                else if (v < 256) { mu = R_P_VWMU + v - 128; sg = R_P_VWSG + v - 128; ep = R_P_VWEP + v - 128; }
                else if (v < 640) { mu = R_P_AWMU + v - 256; sg = R_P_AWSG + v - 256; ep = R_P_AWEP + v - 256; }
                else if (v == 640) { mu = R_P_VBMU; sg = R_P_VBSG; ep = R_P_VBEP; }
                else { mu = R_P_ABMU + v - 641; sg = R_P_ABSG + v - 641; ep = R_P_ABEP + v - 641; }
                a.HWE[n * kHwN + v] = eff_w(Pn, mu, sg, ep, !n);
            }
        }
        return;
    }
    const int rq = bid & 3;
    bid >>= 2;
    const int t = bid % T;
    bid /= T;
    const int ct = bid % nct, s = bid / nct;
    __shared__ __attribute__((aligned(16))) float F2s[32][132];
    __shared__ float zp[4][16][64];  // the K-half-1 partials of the four Zx tiles
    DQ_STAMP(220, blockIdx.x == 0);
    const float* P = s == 2 ? a.target : a.params;
    const int b = ct * 32 + col;
    const int64_t c = (int64_t)t * B + b;
    const int m = 4 * rq + (w & 3), kh = w >> 2;
    DQ_STAMP(227, blockIdx.x == 0 && s == 0);
    // every load of the block is issued here, before any MFMA (one round trip instead of four):
    // the Zx A fragments of this wave's K half (all waves); x, W1 / b1, W2, b2 (F waves 0..3); the
    // Zx bias of tile m (waves 4..7, which form the final sum)
    const float* wr = P + R_P_WIH + (int64_t)(128 * (col >> 3) + 8 * m + (col & 7)) * 128 + 4 * h + 64 * kh;
    float4 av[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = *reinterpret_cast<const float4*>(wr + 8 * j);
    float xs[4], f1w[2][4], zb[16];
    float4 w2v[8];
    f32x16 f2;
    if (w < 4) {
        tile_inputs((s == 0 ? a.obs : a.next) + ((int64_t)b * T + t) * 7, h, xs);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int row = 32 * jt + col, kk = 2 * s4 + h;
                f1w[jt][s4] = P[kk == 0 ? R_P_F1B + row : R_P_F1W + row * 7 + kk - 1];
            }
        const float* w2 = P + R_P_F2W + (32 * w + col) * 64 + 4 * h;
#pragma unroll
        for (int i = 0; i < 8; ++i) w2v[i] = *reinterpret_cast<const float4*>(w2 + 32 * (i >> 2) + 8 * (i & 3));
#pragma unroll
        for (int r = 0; r < 16; ++r) f2[r] = P[R_P_F2B + 32 * w + rho(r) + 4 * h];
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rr = rho(r) + 4 * h;
            const int g = 128 * (rr >> 3) + 8 * m + (rr & 7);
            zb[r] = P[R_P_BIH + g] + P[R_P_BHH + g];
        }
    }
#ifdef PM_DIAG
    drain();
    DQ_STAMP(228, blockIdx.x == 0);
#endif
    if (w < 4) {
        // F1 (both 32-row tiles): input k' = 2 s4 + h, k' = 0 the constant 1 (weight: b1)
        f32x16 c1[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            c1[jt] = f32x16{};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(f1w[jt][s4], xs[s4], c1[jt], 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
        }
        // F2 tile w: rows 32w + rho(r) + 4h; K = 64 over the two F1 tiles (k = 32 t2 + rho(r) + 4h)
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
#pragma unroll
        for (int r = 0; r < 16; ++r) f2[r] = relu(f2[r]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<float4*>(&F2s[col][32 * w + 8 * i + 4 * h]) =
                make_float4(f2[4 * i], f2[4 * i + 1], f2[4 * i + 2], f2[4 * i + 3]);
        if (s == 0 && rq == 0) {  // the obs stream's features and inputs for the weight gradients, [unit][column]
            const int64_t C0 = a.C0;
            if (w == 0) {  // x^T from the tile operands: half 1 holds x0, x2, x4, x6, half 0 x1, x3, x5
                if (h) a.XT[c] = xs[0];
#pragma unroll
                for (int i = 1; i < 4; ++i) a.XT[(int64_t)(2 * i - 1 + h) * C0 + c] = xs[i];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a.F2T[(int64_t)(32 * w + rho(r) + 4 * h) * C0 + c] = f2[r];
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
                if (w == jt)  // static register index (c1[w] would be a 32-way select per element)
#pragma unroll
                    for (int r = 0; r < 16; ++r) a.F1T[(int64_t)(32 * jt + rho(r) + 4 * h) * C0 + c] = c1[jt][r];
        }
    }
    DQ_STAMP(223, blockIdx.x == 0);
    __syncthreads();
    DQ_STAMP(224, blockIdx.x == 0);
    // Zx tile m, K half kh: k = 64 kh + 8j + 4h + e for k-step (j, e)
    f32x16 z = {};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(&F2s[col][64 * kh + 8 * j + 4 * h]);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].x, bv.x, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].y, bv.y, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].z, bv.z, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].w, bv.w, z, 0, 0, 0);
    }
    DQ_STAMP(225, blockIdx.x == 0);
    if (kh == 0)
#pragma unroll
        for (int r = 0; r < 16; ++r) zp[w][r][lane] = z[r];
    __syncthreads();
    DQ_STAMP(226, blockIdx.x == 0);
    if (kh == 0) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = (zp[w & 3][r][lane] + z[r]) + zb[r];  // (K half 0 + K half 1) + bias
    // Zx[s][t][gate row][sequence]: a register's 32 columns are 128 contiguous bytes
    float* zx = a.ZX + ((int64_t)s * T + t) * 512 * B + b;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rr = rho(r) + 4 * h;
        zx[(int64_t)(128 * (rr >> 3) + 8 * m + (rr & 7)) * B] = z[r];
    }
    PM_STAMP_T(222, 256);
}

// ---------------------------------------------------------------- 2: the recurrence (sequence-private)
// One workgroup of 1024 threads owns whole sequences: the recurrence h_{t+1} = f(Zx_t + Whh h_t) of a
// sequence never leaves its CU, so no step waits on another CU (round 3 split the 512 gate rows over
// 16 workgroups and paid a cross-CU hand-off per step: 2T + 3 hops of ~3 us). Whh (512 x 128, 256 KB)
// lives in the workgroup's registers: thread 8u + kg holds rows 128q + u (the four gates of LSTM unit
// u) x columns 16kg .. 16kg + 15, 64 floats. On gfx950 the f32 VALU issues 32 fmaf per cycle per
// SIMD, the same rate as the f32 MFMA, so a matrix-vector step on the VALU loses nothing to the
// matrix cores and needs no 16- or 32-column tile.
//   forward  per step: 16 fmaf per gate per column from h in LDS, the K eighths summed by a DPP
//            butterfly (every lane of the unit ends with the sums), the cell on the lanes of its
//            column, h back to LDS: one barrier per step.
//   heads    S = W_S h_T (W_S rows in registers from an LDS image), V / A, Q.
//   BPTT     per step: dz from the saved gates, dh_{t-1} = Whh^T dz as 16 partials per thread, summed
//            over the wave's unit pairs (DPP row_ror 8), then over the 64 (wave, row) sets through LDS
//            in a fixed order: one barrier per step.
// Workgroups [0, B/2): targetB on `next`, sequences 2j and 2j + 1 (two columns); [B/2, B/2 + B):
// modelB on `obs` (column 0, the one BPTT runs on) and on `next` (column 1) of sequence b;
// [3B/2, 5B/2): the dF2 trailer of sequence b. The forward's one cross-workgroup hand-off is targetB's
// Q(s_T) (a granule pair per sequence, tag E + 1). A workgroup only ever waits on lower-indexed ones,
// which the dispatcher has placed before it, so the launch cannot deadlock whatever is resident.
constexpr int kGcLds = (2 * 128 * 68) / 768;  // T up to which the obs workgroup keeps its gate scratch in LDS
static_assert(128 * kWsStride <= 2 * 128 * 68, "W_S image in ws");
struct RecurSmem {
    // effective W_S (DMA image of WSE); once the heads hold it in registers, the obs workgroup's BPTT
    // reduction buffer (same shape as part) when part holds the forward's gate scratch
    __attribute__((aligned(16))) float ws[2 * 128 * 68];
    __attribute__((aligned(16))) float part[2][128][68];     // W^T dz partials [k][set, swizzled], by parity
    __attribute__((aligned(16))) float hs[2][288];           // h [unit][column], 4 floats of pad per 16 units
    float sr[2][128];                                        // ReLU(S) per column
    float qv[2][4];                                          // V, A0..2 per column
    float dva[4];                                            // dV, dA0..2
};

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over the 8 lanes of a unit (lanes 8i .. 8i + 7): quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror; every step adds two equal-order partial sums, so all 8 lanes get the same bits
__device__ __forceinline__ float sum8(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    return v;
}
__device__ __forceinline__ int hidx(int k) { return 2 * k + 4 * (k >> 4); }  // hs[.][hidx(k) + column]

// p[j] (this thread's partial of output k = 16 kg + j over its unit) summed over all 128 units; the
// caller's thread (u, kg) gets output u. Wave w's lanes hold units 8w .. 8w + 7 (lane 8i + kg); row r
// of the wave (16 lanes) holds units 2r, 2r + 1, summed by row_ror 8, giving set 4w + r of 64. The
// set is stored at column (set + 4 (k >> 4)) & 63 of row k: conflict-free stores, and a reader's 8
// sets stay two aligned float4s.
__device__ __forceinline__ float reduce_units(float (&p)[16], float (*part)[68], int lane, int w, int u, int kg) {
#pragma unroll
    for (int j = 0; j < 16; ++j) p[j] += dppf<0x128>(p[j]);
    if ((lane & 8) == 0) {
        const int col = (4 * w + (lane >> 4) + 4 * kg) & 63;
#pragma unroll
        for (int j = 0; j < 16; ++j) part[16 * kg + j][col] = p[j];
    }
    __syncthreads();
    const int sw = 4 * (u >> 4);
    const float4 v0 = *reinterpret_cast<const float4*>(&part[u][(8 * kg + sw) & 63]);
    const float4 v1 = *reinterpret_cast<const float4*>(&part[u][(8 * kg + 4 + sw) & 63]);
    const float d = ((((((v0.x + v0.y) + v0.z) + v0.w) + v1.x) + v1.y) + v1.z) + v1.w;
    return sum8(d);
}

// The dF2 trailer (workgroups [3B/2, 5B/2), one per sequence): the feature layers' backward of the obs
// stream, dF2_t = Wih^T dz_t, dP2 = dF2 (F2 > 0), then dF1 = W2^T dP2, dP1 = dF1 (F1 > 0) (k_dq_wgrad
// forms dW2 = dP2 F1^T and dW1 = dP1 x^T as tiles). Wih sits in registers in Whh's fragment layout,
// so dF2_t is BPTT's dh product on another matrix; each dz_t arrives from the sequence's obs
// workgroup as granules (tag E + 2 + t) while that workgroup moves on, so the pass trails BPTT by a
// hand-off instead of following it. It waits only on lower-indexed workgroups (dispatched first).
__device__ __forceinline__ void dq_df2(const DqArgs& a, RecurSmem& sm, int b, uint32_t E, const HandoffCtl& hc) {
    const int T = a.T, B = a.B;
    const int64_t C0 = a.C0;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, u = tid >> 3, kg = tid & 7;
    DQ_STAMP(8, b == 0);
    float wr[4][16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4* src = reinterpret_cast<const float4*>(a.params + R_P_WIH + (int64_t)(128 * q + u) * 128 + 16 * kg);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 v = src[i];
            wr[q][4 * i] = v.x; wr[q][4 * i + 1] = v.y; wr[q][4 * i + 2] = v.z; wr[q][4 * i + 3] = v.w;
        }
    }
    float* p2s = sm.ws;  // [T][128] dP2 of the sequence (row t read by the dF1 pass one step later)
    const char* dzh = reinterpret_cast<const char*>(a.DZH) + (int64_t)b * T * 128 * 32;
    const int j1 = tid >> 4, k16 = tid & 15;  // dF1: row j1, F2 rows 8 k16 .. 8 k16 + 7
    float w2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w2[i] = a.params[R_P_F2W + (8 * k16 + i) * 64 + j1];
    // dF1 of step t from the LDS dP2 row, summed over the 16 lanes of the row; lane k16 = 0 stores dP1
    auto df1_row = [&](int t, float f1m) {
        const float4 p0 = *reinterpret_cast<const float4*>(&p2s[t * 128 + 8 * k16]);
        const float4 p1 = *reinterpret_cast<const float4*>(&p2s[t * 128 + 8 * k16 + 4]);
        float v = w2[0] * p0.x;
        v = fmaf(w2[1], p0.y, v);
        v = fmaf(w2[2], p0.z, v);
        v = fmaf(w2[3], p0.w, v);
        v = fmaf(w2[4], p1.x, v);
        v = fmaf(w2[5], p1.y, v);
        v = fmaf(w2[6], p1.z, v);
        v = fmaf(w2[7], p1.w, v);
        v = sum8(v);
        v += dppf<0x128>(v);  // + the other 8 lanes of the 16-lane row
        if (k16 == 0) a.dP1[(int64_t)j1 * C0 + (int64_t)t * B + b] = f1m > 0.f ? v : 0.f;
    };
    float f1p = 0.f;
    for (int t = T - 1; t >= 0; --t) {
        const int64_t cc = (int64_t)t * B + b;
        const float f2 = a.F2T[(int64_t)u * C0 + cc];
        const float f1 = a.F1T[(int64_t)j1 * C0 + cc];
        const uint32_t tag = E + 2 + (uint32_t)t;
        const int off[2] = {(t * 128 + u) * 32, (t * 128 + u) * 32 + 16};
        float dz[4];
        {   // one read of the unit's granules first: when the trailer runs behind BPTT they are there;
            // otherwise lane 0 waits on the last granule of the wave's units (one store instruction of
            // the producer's wave w) and the wave reads them again
            bool ok = true;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint64_t* p = reinterpret_cast<const uint64_t*>(dzh + off[i]);
                const uint64_t q0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t q1 = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = ok && (uint32_t)(q0 >> 32) == tag && (uint32_t)(q1 >> 32) == tag;
                dz[2 * i] = __uint_as_float((uint32_t)q0);
                dz[2 * i + 1] = __uint_as_float((uint32_t)q1);
            }
            if (!__all(ok)) {
                poll_tags(dzh, ((t * 128 + 8 * w + 7) * 4 + 3) * 8, 1, tag, hc);
                gather<2, false>(dzh, off, tag, dz, hc);
            }
        }
        float p[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) p[j] = fmaf(wr[3][j], dz[3], fmaf(wr[2][j], dz[2], fmaf(wr[1][j], dz[1], wr[0][j] * dz[0])));
        const float d = reduce_units(p, sm.part[t & 1], lane, w, u, kg);  // its barrier publishes p2s row t + 1
        DQ_STAMP(180 + t, b == 0 && t < 20);
        if (t + 1 < T) df1_row(t + 1, f1p);
        f1p = f1;
        const float d2 = f2 > 0.f ? d : 0.f;
        if (kg == 0) {
            a.dP2[(int64_t)u * C0 + cc] = d2;
            p2s[t * 128 + u] = d2;
        }
    }
    __syncthreads();
    df1_row(0, f1p);
    DQ_STAMP(7, b == 0);
}

__global__ __launch_bounds__(kRecThreads) void k_dq_recur(DqArgs a) {
    if (skipped(a)) return;
    __shared__ RecurSmem sm;
    const int T = a.T, B = a.B;
    const int64_t C0 = a.C0;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, u = tid >> 3, kg = tid & 7, myc = kg & 1;
    // [0, B/2) targetB on next (sequences 2j, 2j + 1 as the two columns), [B/2, 3B/2) modelB on obs and
    // next of sequence b, [3B/2, 5B/2) the dF2 trailer of sequence b
    const int nT = B >> 1, bx = (int)blockIdx.x;
    const int role = bx < nT ? 0 : (bx < nT + B ? 1 : 2);
    const int b = role == 0 ? 2 * bx : (role == 1 ? bx - nT : bx - nT - B);  // column 0's sequence
    const uint32_t E = (uint32_t)a.flags[0] << 7;  // this update's tag base
    const HandoffCtl hc{a.stats, a.grad + PM_RNN_NPARAM + 1, hand_limit(a.poll_limit)};
    [[maybe_unused]] const bool so0 = bx == nT, s10 = bx == 0;  // stamping blocks (diag)
    if (role == 2) {
        dq_df2(a, sm, b, E, hc);
        return;
    }
    const bool tgt = role == 0;
    const int sc0 = tgt ? 2 : 0, sc1 = tgt ? 2 : 1, bc1 = tgt ? b + 1 : b;  // (stream, sequence) of column 1
    const float* P = tgt ? a.target : a.params;
    const int net = tgt ? 1 : 0;
    DQ_STAMP(1, so0);
    DQ_STAMP(111, s10);
    // Zx of step 0 first (step 0 needs no Whh: h_0 = 0), then Whh: the loads complete in issue
    // order, so step 0's cell runs while Whh is still in flight
    // Zx of this lane's column (the cell runs on the lanes of its column only)
    const float* zx = a.ZX + (int64_t)(myc ? sc1 : sc0) * T * 512 * B + (int64_t)u * B + (myc ? bc1 : b);
    float zn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) zn[q] = zx[(int64_t)q * 128 * B];
    // Whh rows 128q + u, columns 16kg .. 16kg + 15
    float wr[4][16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4* src = reinterpret_cast<const float4*>(P + R_P_WHH + (int64_t)(128 * q + u) * 128 + 16 * kg);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 v = src[i];
            wr[q][4 * i] = v.x; wr[q][4 * i + 1] = v.y; wr[q][4 * i + 2] = v.z; wr[q][4 * i + 3] = v.w;
        }
    }
    // ---------------- forward
    const bool gl_lds = !tgt && T <= kGcLds;  // block-uniform
    float* gl = &sm.part[0][0][0];
    float cst = 0.f;  // c of (unit u, column myc)
    // the cell of unit u, column myc (v_exp_f32 / v_rcp_f32 activations, a few ulp), then h to LDS
    // and the obs column's scratch; one barrier
    auto cell = [&](int t, const float (&g4)[4]) {
        const float gi = sig_hw(g4[0]), gf = sig_hw(g4[1]), gg = tanh_hw(g4[2]), go = sig_hw(g4[3]);
        cst = gf * cst + gi * gg;  // cy = forgetgate * cx + ingate * cellgate
        const float hn = go * tanh_hw(cst);
        if (kg < 2) sm.hs[(t + 1) & 1][hidx(u) + kg] = hn;
        if (!tgt && gl_lds) {  // the obs column (kg even): BPTT's scratch and h in LDS, [t][6][128]
            float* g = gl + t * 768 + u;
            if (kg == 0) { g[0] = gi; g[128] = gf; g[512] = cst; g[640] = hn; }
            else if (kg == 2) { g[256] = gg; g[384] = go; }
        } else if (!tgt) {  // the same in global memory (long sequences)
            float* gc = a.GC + ((int64_t)b * T + t) * 640 + u;
            if (kg == 0) {
                gc[0] = gi; gc[128] = gf; gc[512] = cst;
                float* hr = a.H + (int64_t)u * C0 + b;
                if (t + 1 < T) hr[(int64_t)(t + 1) * B] = hn;
                if (t == 0) hr[0] = 0.f;
            } else if (kg == 2) {
                gc[256] = gg; gc[384] = go;
            }
        }
        __syncthreads();
        DQ_STAMP(10 + t, so0 && t < 30);
        DQ_STAMP(120 + t, s10 && t < 30);
    };
    {   // step 0, outside the loop (h_0 = 0: the gates are Zx alone), so its wait covers Zx only
        float z[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) z[q] = zn[q];
        if (T > 1)
#pragma unroll
            for (int q = 0; q < 4; ++q) zn[q] = zx[(int64_t)512 * B + (int64_t)q * 128 * B];
        cell(0, z);
        // the effective W_S image -> LDS (global_load_lds, 1 KB per wave instruction), issued after
        // step 0 (issued before it, the copy made step 0's Zx wait a vmcnt(0) behind Whh and itself);
        // it lands beside Whh, which step 1 waits for anyway. kWsPieces per wave, the last clamped.
        {
            constexpr int kPieces = 128 * kWsStride / 256, kWsPieces = (kPieces + 15) / 16;
            const float* src = a.WSE + (int64_t)net * 128 * kWsStride;
#pragma unroll
            for (int j = 0; j < kWsPieces; ++j) {
                const int k = min(w + 16 * j, kPieces - 1);
                __builtin_amdgcn_global_load_lds((const void*)(src + 256 * k + 4 * lane), (lds_void*)&sm.ws[256 * k], 16, 0, 0);
            }
        }
    }
    for (int t = 1; t < T; ++t) {
        float z[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) z[q] = zn[q];
        if (t + 1 < T) {
            const int64_t o = (int64_t)(t + 1) * 512 * B;
#pragma unroll
            for (int q = 0; q < 4; ++q) zn[q] = zx[o + (int64_t)q * 128 * B];
        }
        float acc[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) { acc[q][0] = 0.f; acc[q][1] = 0.f; }
        const float* hp = &sm.hs[t & 1][36 * kg];  // units 16kg .. 16kg + 15, both columns
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 hv = *reinterpret_cast<const float4*>(hp + 4 * i);  // (k, c0) (k, c1) (k+1, c0) (k+1, c1)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc[q][0] = fmaf(wr[q][2 * i], hv.x, acc[q][0]);
                acc[q][1] = fmaf(wr[q][2 * i], hv.y, acc[q][1]);
                acc[q][0] = fmaf(wr[q][2 * i + 1], hv.z, acc[q][0]);
                acc[q][1] = fmaf(wr[q][2 * i + 1], hv.w, acc[q][1]);
            }
        }
        float g4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc[q][0] = sum8(acc[q][0]);
            acc[q][1] = sum8(acc[q][1]);
            g4[q] = z[q] + (myc ? acc[q][1] : acc[q][0]);
        }
        cell(t, g4);
    }
    // ---------------- heads: S = W_S h_T + b_S, V / A, Q for both columns
    drain();
    __syncthreads();  // every wave's share of the W_S image has landed
    float wsr[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(&sm.ws[u * kWsStride + 16 * kg + 4 * i]);
        wsr[4 * i] = v.x; wsr[4 * i + 1] = v.y; wsr[4 * i + 2] = v.z; wsr[4 * i + 3] = v.w;
    }
    const float* HW = a.HWE + net * kHwN;
    float sv0;  // S + b_S of row u, column 0
    {
        float s2[2] = {0.f, 0.f};
        const float* hp = &sm.hs[T & 1][36 * kg];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 hv = *reinterpret_cast<const float4*>(hp + 4 * i);
            s2[0] = fmaf(wsr[2 * i], hv.x, s2[0]);
            s2[1] = fmaf(wsr[2 * i], hv.y, s2[1]);
            s2[0] = fmaf(wsr[2 * i + 1], hv.z, s2[0]);
            s2[1] = fmaf(wsr[2 * i + 1], hv.w, s2[1]);
        }
        const float bs = HW[HW_BS + u];
        sv0 = sum8(s2[0]) + bs;
        const float sv1 = sum8(s2[1]) + bs;
        if (kg < 2) sm.sr[kg][u] = relu(kg ? sv1 : sv0);
    }
    __syncthreads();
    if (w == 0) {  // lane: output o (0 V, 1..3 A), column c, rows 16 pp .. 16 pp + 15
        const int o = lane & 3, c = (lane >> 2) & 1, pp = lane >> 3;
        const float* wo = HW + (o == 0 ? HW_V : HW_A + 128 * (o - 1)) + 16 * pp;
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = fmaf(wo[r], sm.sr[c][16 * pp + r], acc);
        acc += __shfl_xor(acc, 8);
        acc += __shfl_xor(acc, 16);
        acc += __shfl_xor(acc, 32);
        if (pp == 0) sm.qv[c][o] = acc + (o == 0 ? HW[HW_VB] : HW[HW_AB + o - 1]);
    }
    __syncthreads();
    float q[2][3];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float v = sm.qv[c][0], x0 = sm.qv[c][1], x1 = sm.qv[c][2], x2 = sm.qv[c][3];
        const float mean = ((x0 + x1) + x2) / 3.0f;  // A.mean(dim=1)
        q[c][0] = v + (x0 - mean);
        q[c][1] = v + (x1 - mean);
        q[c][2] = v + (x2 - mean);
    }
    if (tgt) {  // publish Q_target(s_T)
        if (tid < 2) {  // column tid = sequence b + tid
            const __amdgpu_buffer_rsrc_t rq = rsrc(a.QT);
            st_g2(rq, (b + tid) * 32, q[tid][0], q[tid][1], E + 1);
            st_g2(rq, (b + tid) * 32 + 16, q[tid][2], 0.f, E + 1);
        }
        DQ_STAMP(150, s10);
        return;
    }
    DQ_STAMP(50, so0);
    if (gl_lds)  // the weight gradients' H [unit][t * B + b]: h_t, the input hidden of step t (h_0 = 0)
        for (int t = kg; t < T; t += 8) a.H[(int64_t)u * C0 + (int64_t)t * B + b] = t == 0 ? 0.f : gl[(t - 1) * 768 + 640 + u];
    // BPTT's reduction buffer: ws once every wave holds its W_S rows (the heads' barriers), part otherwise
    float (*const red)[128][68] = gl_lds ? reinterpret_cast<float (*)[128][68]>(sm.ws) : sm.part;
    // ---------------- the loss and dQ (obs column), wave 0
    if (w == 0) {
        poll_tags(a.QT, b * 32 + 24, 1, E + 1, hc);
        const int off[2] = {b * 32, b * 32 + 16};
        float qt[4];
        gather<2, false>(a.QT, off, E + 1, qt, hc);
        const int64_t jl = (int64_t)b * T + T - 1;  // the sequence's last step
        const int ac = a.act[jl];
        const float rl = a.rew[jl], dl = a.done[jl] ? 1.f : 0.f;
        const float qa = ac == 0 ? q[0][0] : (ac == 1 ? q[0][1] : q[0][2]);
        const int as = argmax3(q[1]);  // argmax Q_B(next) (first max)
        const float y = rl + a.gamma * qt[as] * (1.0f - dl);
        const float d = qa - y, ad = fabsf(d);
        const float lv = ad < 1.0f ? 0.5f * d * d : ad - 0.5f;  // smooth_l1, beta 1
        const float gq = fminf(fmaxf(d, -1.0f), 1.0f) / (float)B;
        if (lane < 4) {
            const float dv = lane == 0 ? gq : (lane - 1 == ac ? gq : 0.f) - gq / 3.0f;
            sm.dva[lane] = dv;
            a.SC[b * 8 + SC_DV + lane] = dv;
        } else if (lane == 4) {
            a.SC[b * 8 + SC_LOSS] = lv;
            a.SC[b * 8 + SC_Q] = qa;
        }
        DQ_STAMP(51, so0);
    }
    __syncthreads();
    // dS of row u (modelB's effective V / A weights), through the ReLU; dh_T = W_S^T dS
    float dh;
    {
        const float ds = HW[HW_V + u] * sm.dva[0] + HW[HW_A + u] * sm.dva[1] + HW[HW_A + 128 + u] * sm.dva[2] +
                         HW[HW_A + 256 + u] * sm.dva[3];
        const float dsm = sv0 > 0.f ? ds : 0.f;
        if (kg == 0) {
            a.DS[(int64_t)u * B + b] = dsm;
            a.SR[(int64_t)u * B + b] = sm.sr[0][u];
            a.HT[(int64_t)u * B + b] = sm.hs[T & 1][hidx(u)];
        }
        float p[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) p[j] = wsr[j] * dsm;
        dh = reduce_units(p, red[T & 1], lane, w, u, kg);
    }
    DQ_STAMP(52, so0);
    // ---------------- BPTT (obs column)
    // the saved gates of step t: LDS [t][6][128] or global [t][5][128] (stride sg per step)
    const float* gcb = gl_lds ? gl + u : a.GC + (int64_t)b * T * 640 + u;
    const int sg = gl_lds ? 768 : 640;
    float gn[6];  // gi gf gg go c_t c_{t-1} of the next step down
    {
        const float* g = gcb + (int64_t)(T - 1) * sg;
#pragma unroll
        for (int v = 0; v < 5; ++v) gn[v] = g[128 * v];
        gn[5] = T > 1 ? g[512 - sg] : 0.f;
    }
    float dc = 0.f;
    const __amdgpu_buffer_rsrc_t rdz = rsrc(a.DZH);
    for (int t = T - 1; t >= 0; --t) {
        const float gi = gn[0], gf = gn[1], gg = gn[2], go = gn[3], cT = gn[4], cP = gn[5];
        if (t > 0) {
            const float* g = gcb + (int64_t)(t - 1) * sg;
#pragma unroll
            for (int v = 0; v < 5; ++v) gn[v] = g[128 * v];
            gn[5] = t > 1 ? g[512 - sg] : 0.f;
        }
        const float tc = tanh_hw(cT);
        const float dcc = dc + dh * go * (1.0f - tc * tc);
        const float dz0 = dcc * gg * (gi * (1.0f - gi));
        const float dz1 = dcc * cP * (gf * (1.0f - gf));
        const float dz2 = dcc * gi * (1.0f - gg * gg);
        const float dz3 = dh * tc * (go * (1.0f - go));
        dc = dcc * gf;
        if (kg < 4) {
            const float dzk = kg == 0 ? dz0 : (kg == 1 ? dz1 : (kg == 2 ? dz2 : dz3));
            a.dZ[(int64_t)(128 * kg + u) * C0 + (int64_t)t * B + b] = dzk;
        }
        if (kg == 0) {  // dz of unit u to the dF2 trailer: granules {dz_q, tag}, tag E + 2 + t
            const int o = (((int)b * T + t) * 128 + u) * 32;
            st_g2(rdz, o, dz0, dz1, E + 2 + t);
            st_g2(rdz, o + 16, dz2, dz3, E + 2 + t);
        }
        if (t == 0) break;
        float p[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) p[j] = fmaf(wr[3][j], dz3, fmaf(wr[2][j], dz2, fmaf(wr[1][j], dz1, wr[0][j] * dz0)));
        dh = reduce_units(p, red[t & 1], lane, w, u, kg);
        DQ_STAMP(90 + t, so0 && t < 30);
    }
    DQ_STAMP(2, so0);
}

// ---------------------------------------------------------------- 3: weight gradients
struct WgSmem {
    float red[16][16][64];  // per-wave partial tiles
    float rs[16][64];
};

// One 32 x 32 output tile per workgroup, K split over the 16 waves (8-column chunks round robin, 4 in
// flight), summed in wave order; the tile's row sums (the bias gradients) ride along.
//   mat 0: dWih = dZ F2^T (16 x 4 tiles, K = T*B)        row sums -> db_ih = db_hh
//   mat 1: dWhh = dZ H^T  (16 x 4)
//   mat 2: dW_S = dS h_T^T (4 x 4, K = B)                row sums -> db_S
//   mat 3: dW2 = dP2 F1^T (4 x 2, K = T*B)               row sums -> db2
//   mat 4: dW1 = dP1 x^T  (2 x 1; x^T rows 7..31 zero)    row sums -> db1
// then one workgroup for the V / A head gradients, the loss and mean Q.
constexpr int kWgTiles = 64 + 64 + 16 + 8 + 2;

__global__ __launch_bounds__(1024) void k_dq_wgrad(DqArgs a) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the step counters the apply steps from (tstep): only the
        a.tstep[0] = a.stats->steps;            // apply's block 0 advances them, so its other blocks must
        a.tstep[1] = a.stats->adam_t;           // not read stats themselves (a late block would see ts + 1)
    }
    if (skipped(a)) return;
    __shared__ WgSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const int64_t C0 = a.C0;
    const int B = a.B;
    const int bid = blockIdx.x;
    DQ_STAMP(210, bid == 0);
    if (bid < kWgTiles) {
        int mat, gt, kt;
        if (bid < 128) { mat = bid >> 6; gt = (bid >> 2) & 15; kt = bid & 3; }
        else if (bid < 144) { mat = 2; gt = (bid - 128) >> 2; kt = bid & 3; }
        else if (bid < 152) { mat = 3; gt = (bid - 144) >> 1; kt = bid & 1; }
        else { mat = 4; gt = bid - 152; kt = 0; }
        const int64_t ld = mat == 2 ? (int64_t)B : C0;
        const float* A = mat <= 1 ? a.dZ : (mat == 2 ? a.DS : (mat == 3 ? a.dP2 : a.dP1));
        const float* Bm = mat == 0 ? a.F2T : (mat == 1 ? a.H : (mat == 2 ? a.HT : (mat == 3 ? a.F1T : a.XT)));
        const float* Ar = A + (int64_t)(32 * gt + col) * ld + 4 * h;
        const float* Br = Bm + (int64_t)(32 * kt + col) * ld + 4 * h;
        f32x16 acc = {};
        float rsum = 0.f;
        const int nch = (int)(ld / 8);
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
            const int ldg = mat <= 2 ? 128 : (mat == 3 ? 64 : 7);
            float* G = a.grad + (mat == 0 ? R_P_WIH : (mat == 1 ? R_P_WHH : (mat == 2 ? R_P_SWMU : (mat == 3 ? R_P_F2W : R_P_F1W))));
            double sq = 0.0;  // this tile's share of the clip norm (local_norm), sigma gradients (mu x epsilon) included
            if (32 * kt + col < ldg)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float v = sm.red[0][r][lane];
                    for (int k = 1; k < 16; ++k) v += sm.red[k][r][lane];
                    const int e = (32 * gt + rho(r) + 4 * h) * ldg + 32 * kt + col;
                    G[e] = v;
                    sq += (double)v * (double)v;
                    if (mat == 2) {
                        const float gs = v * a.params[R_P_SWEP + e];
                        sq += (double)gs * (double)gs;
                    }
                }
            DQ_STAMP(211, bid == 0);
            if (mat != 1 && kt == 0) {  // the bias gradients: row sums
                float v = sm.rs[0][lane];
                for (int k = 1; k < 16; ++k) v += sm.rs[k][lane];
                v += __shfl_xor(v, 32);
                const int row = 32 * gt + col;
                if (h == 0) {
                    if (mat == 0) { a.grad[R_P_BIH + row] = v; a.grad[R_P_BHH + row] = v; }
                    else if (mat == 2) a.grad[R_P_SBMU + row] = v;
                    else if (mat == 3) a.grad[R_P_F2B + row] = v;
                    else a.grad[R_P_F1B + row] = v;
                    sq += (mat == 0 ? 2.0 : 1.0) * ((double)v * (double)v);
                    if (mat == 2) {
                        const float gs = v * a.params[R_P_SBEP + row];
                        sq += (double)gs * (double)gs;
                    }
                }
            }
            if (a.local_norm) {
                sq = wave_sum(sq);  // DPP reduction (pm_dev.h): xor-1-first association of the fp64 sum
                if (lane == 0) a.NP[bid] = sq;
            }
        }
        return;
    }
    // ---- the V / A head gradients: dw_o[r] = sum_b dQ_o[b] ReLU(S)[r][b] (o = V, A0..2) and their biases,
    // the loss and mean Q, each summed over the sequences in order
    double sq = 0.0;
    // the per-sequence scalars -> LDS once (coalesced), beside each thread's ReLU(S) row loads
    float* scs = &sm.red[0][0][0];  // [B][8]
    for (int i = tid; i < B * 8; i += 1024) scs[i] = a.SC[i];
    __syncthreads();
    if (tid < 512) {
        const int o = tid >> 7, r = tid & 127;
        const float4* sr = reinterpret_cast<const float4*>(a.SR + (int64_t)r * B);
        float v = 0.f;
        for (int b0 = 0; b0 < B; b0 += 64) {  // 16 float4 loads in flight, then the fmaf in sequence order
            float4 x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = b0 + 4 * i < B ? sr[b0 / 4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (b0 + 4 * i >= B) break;
                const int b = b0 + 4 * i;
                v = fmaf(scs[b * 8 + SC_DV + o], x[i].x, v);
                v = fmaf(scs[(b + 1) * 8 + SC_DV + o], x[i].y, v);
                v = fmaf(scs[(b + 2) * 8 + SC_DV + o], x[i].z, v);
                v = fmaf(scs[(b + 3) * 8 + SC_DV + o], x[i].w, v);
            }
        }
        const int e = o == 0 ? r : 128 * (o - 1) + r;
        a.grad[(o == 0 ? R_P_VWMU : R_P_AWMU) + e] = v;
        const float gs = v * a.params[(o == 0 ? R_P_VWEP : R_P_AWEP) + e];
        sq = (double)v * (double)v + (double)gs * (double)gs;
    } else if (tid < 518) {
        const int o = tid - 512;  // dV, dA0..2, loss, Q(s, a)
        float v = 0.f;
        for (int b = 0; b < B; ++b) v += scs[b * 8 + o];
        if (o == 0) a.grad[R_P_VBMU] = v;
        else if (o < 4) a.grad[R_P_ABMU + o - 1] = v;
        else if (o == SC_LOSS) a.stats->loss = v / (float)B;
        else a.stats->q_mean = v / (float)B;
        if (o < 4) {
            const float gs = v * a.params[o == 0 ? R_P_VBEP : R_P_ABEP + o - 1];
            sq = (double)v * (double)v + (double)gs * (double)gs;
        }
    }
    if (a.local_norm) {  // the block's squares, summed in a fixed tree
        double* red = reinterpret_cast<double*>(&sm.red[0][0][0]) + 1024;  // past scs ([B][8] <= 8 KB)
        red[tid] = sq;
        __syncthreads();
        for (int k = 512; k > 0; k >>= 1) {
            if (tid < k) red[tid] += red[tid + k];
            __syncthreads();
        }
        if (tid == 0) a.NP[kWgTiles] = red[0];
    }
}

// The clip norm's shares of replicas that all-reduce (pm_drqn_apply after pm_drqn_grads and the
// SUM), summed exactly as k_dq_wgrad's tiles sum them on the single-replica path (pm_drqn_update): the
// same elements per workgroup in the same order, the same DPP wave sum and head-block tree, over the
// values the apply steps with (the summed gradient over the rank count; a sigma gradient is mu
// gradient x epsilon, then over the rank count, as the apply forms it). With one rank every share,
// the clip coefficient and so every parameter are bit-identical to pm_drqn_update's, clip active or
// not; with more ranks it is the norm of the averaged gradient, as before.
__global__ __launch_bounds__(1024) void k_dq_norm(DqArgs a) {
    const float ranks = a.grad[PM_RNN_NPARAM];
    if (!(ranks > 0.f) || a.grad[PM_RNN_NPARAM + 1] != 0.f) return;  // grid-uniform: the apply does nothing
    const float inv_world = 1.0f / ranks;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const int bid = blockIdx.x;
    const float* G = a.grad;
    if (bid < kWgTiles) {
        if (w != 0) return;
        int mat, gt, kt;
        if (bid < 128) { mat = bid >> 6; gt = (bid >> 2) & 15; kt = bid & 3; }
        else if (bid < 144) { mat = 2; gt = (bid - 128) >> 2; kt = bid & 3; }
        else if (bid < 152) { mat = 3; gt = (bid - 144) >> 1; kt = bid & 1; }
        else { mat = 4; gt = bid - 152; kt = 0; }
        const int ldg = mat <= 2 ? 128 : (mat == 3 ? 64 : 7);
        const int gbase = mat == 0 ? R_P_WIH : (mat == 1 ? R_P_WHH : (mat == 2 ? R_P_SWMU : (mat == 3 ? R_P_F2W : R_P_F1W)));
        double sq = 0.0;
        if (32 * kt + col < ldg)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int e = (32 * gt + rho(r) + 4 * h) * ldg + 32 * kt + col;
                const float v = G[gbase + e] * inv_world;
                sq += (double)v * (double)v;
                if (mat == 2) {
                    const float gs = (G[gbase + e] * a.params[R_P_SWEP + e]) * inv_world;
                    sq += (double)gs * (double)gs;
                }
            }
        if (mat != 1 && kt == 0 && h == 0) {  // the bias rows (k_dq_wgrad's row sums)
            const int row = 32 * gt + col;
            const int bi = mat == 0 ? R_P_BIH : (mat == 2 ? R_P_SBMU : (mat == 3 ? R_P_F2B : R_P_F1B));
            const float v = G[bi + row] * inv_world;
            sq += (mat == 0 ? 2.0 : 1.0) * ((double)v * (double)v);
            if (mat == 2) {
                const float gs = (G[bi + row] * a.params[R_P_SBEP + row]) * inv_world;
                sq += (double)gs * (double)gs;
            }
        }
        sq = wave_sum(sq);
        if (lane == 0) a.NP[bid] = sq;
        return;
    }
    // the V / A heads and their biases, k_dq_wgrad's last workgroup's thread mapping and tree
    __shared__ double red[1024];
    double sq = 0.0;
    if (tid < 512) {
        const int o = tid >> 7, r = tid & 127, e = o == 0 ? r : 128 * (o - 1) + r;
        const int mu = (o == 0 ? R_P_VWMU : R_P_AWMU) + e, ep = (o == 0 ? R_P_VWEP : R_P_AWEP) + e;
        const float v = G[mu] * inv_world, gs = (G[mu] * a.params[ep]) * inv_world;
        sq = (double)v * (double)v + (double)gs * (double)gs;
    } else if (tid < 516) {
        const int o = tid - 512;
        const int mu = o == 0 ? R_P_VBMU : R_P_ABMU + o - 1, ep = o == 0 ? R_P_VBEP : R_P_ABEP + o - 1;
        const float v = G[mu] * inv_world, gs = (G[mu] * a.params[ep]) * inv_world;
        sq = (double)v * (double)v + (double)gs * (double)gs;
    }
    red[tid] = sq;
    __syncthreads();
    for (int kk = 512; kk > 0; kk >>= 1) {
        if (tid < kk) red[tid] += red[tid + kk];
        __syncthreads();
    }
    if (tid == 0) a.NP[kWgTiles] = red[0];
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

// One launch for the apply: every block forms its slice's sigma gradients, sums the norm's shares
// (NP: k_dq_wgrad's tiles on one replica, k_dq_norm's after an all-reduce, the same order) in one
// fixed tree — the same in every block, so every block derives the identical clip coefficient — and
// runs Adam on its slice of the parameters. The step counters come from k_dq_wgrad's snapshot
// (tstep): block 0 advances stats, so no block reads stats itself (no arrival, no ticket).
__global__ __launch_bounds__(256) void k_drqn_apply(DqArgs a, AdamK k, float* params, float* target, float* m_,
                                                    float* v_) {
    constexpr int kPer = (PM_RNN_NP + kNormBlocks - 1) / kNormBlocks, kEl = (kPer + 255) / 256;
    __shared__ double red[256];
    __shared__ float cf[3];
    __shared__ int64_t ts_s;
    const float ranks = a.grad[PM_RNN_NPARAM];  // replicas that contributed (summed by the all-reduce)
    if (!(ranks > 0.f)) return;                 // grid-uniform
    if (a.grad[PM_RNN_NPARAM + 1] != 0.f) {     // a hand-off timed out on some rank: the update is void
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.stats->status, 8);
        return;                                 // grid-uniform: no Adam, no target sync, no step count
    }
    const float inv_world = 1.0f / ranks;
    const int64_t ts = a.tstep[0] + 1, at = a.tstep[1] + 1;  // k_dq_wgrad's snapshot of the counters
    // one slice per block for both phases, every operand loaded up front (kEl elements per thread):
    // the sigma gradients a block forms are the ones its Adam reads
    const int plo = blockIdx.x * kPer, phi = min(PM_RNN_NP, plo + kPer);
    float g[kEl], mm[kEl], vv[kEl], pr[kEl];
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
        }
    }
    // the clip norm's shares: k_dq_wgrad's tiles (one replica) or k_dq_norm (replicas that all-reduce),
    // in the same order either way
    static_assert(kWgTiles + 1 <= 256, "norm partials");
    red[threadIdx.x] = (int)threadIdx.x <= kWgTiles ? a.NP[threadIdx.x] : 0.0;
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

static int drqn_grads(const pm_drqn* d, void* stream, int local_norm) {
    if (int rc = check(d)) return rc;
    PM_REQUIRE(d->obs && d->next && d->act && d->rew && d->done, PM_E_ARG, "pm_drqn_grads: null batch");
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats; a.enable = d->enable;
    a.obs = d->obs; a.next = d->next; a.act = d->act; a.rew = d->rew; a.done = d->done;
    a.gamma = (float)d->gamma;
    a.poll_limit = d->poll_limit;
    a.local_norm = local_norm;
    hipLaunchKernelGGL(k_dq_embed, dim3(3 * a.nct * a.T * 4 + kEmbEff), dim3(512), 0, st, a);
    PM_LAUNCHED("k_dq_embed");
    pm_launch(PM_TIMER_DRQN, k_dq_recur, dim3(a.B / 2 + 2 * a.B), dim3(kRecThreads), st, a);
    PM_LAUNCHED("k_dq_recur");
    hipLaunchKernelGGL(k_dq_wgrad, dim3(kWgTiles + 1), dim3(1024), 0, st, a);
    PM_LAUNCHED("k_dq_wgrad");
    return PM_OK;
}

static int drqn_apply(const pm_drqn* d, void* stream, int local_norm) {
    if (int rc = check(d)) return rc;
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.local_norm = local_norm;
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats;
    AdamK k{d->lr, d->beta1, d->beta2, d->adam_eps, d->max_norm, d->target_update_interval};
    if (!local_norm) {  // replicas: the shares of the summed gradient's norm, in k_dq_wgrad's order
        hipLaunchKernelGGL(k_dq_norm, dim3(kWgTiles + 1), dim3(1024), 0, st, a);
        PM_LAUNCHED("k_dq_norm");
    }
    hipLaunchKernelGGL(k_drqn_apply, dim3(kNormBlocks), dim3(256), 0, st, a, k, d->params, d->target, d->adam_m,
                       d->adam_v);
    PM_LAUNCHED("k_drqn_apply");
    return PM_OK;
}

extern "C" int pm_drqn_init(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    const int64_t bytes = dq_layout(d->batch, d->T, nullptr, nullptr);
    PM_REQUIRE(hipMemsetAsync(d->work, 0, (size_t)bytes, pm_stream(stream)) == hipSuccess, PM_E_LAUNCH,
               "pm_drqn_init: hipMemsetAsync failed");
    return PM_OK;
}

extern "C" int pm_drqn_grads(const pm_drqn* d, void* stream) { return drqn_grads(d, stream, 0); }
extern "C" int pm_drqn_apply(const pm_drqn* d, void* stream) { return drqn_apply(d, stream, 0); }

// One replica: the weight-gradient blocks sum the clip norm's shares as they store the gradient
// (replicas that all-reduce call pm_drqn_grads / pm_drqn_apply, whose k_dq_norm forms the same shares
// of the summed gradient: with one rank the two paths are bit-identical, clip active or not).
extern "C" int pm_drqn_update(const pm_drqn* d, void* stream) {
    if (int rc = drqn_grads(d, stream, 1)) return rc;
    return drqn_apply(d, stream, 1);
}
