// K5 — QNetRNN (models/qnet_rnn.py:58-152) for acting: features 7 -> 64 -> 128 (ReLU), one LSTM step
// (128 -> 128, torch gate order i, f, g, o), NoisyLinear shared head 128 -> 128 (ReLU), dueling V / A,
// on the matrix cores with the exact f32 MFMA (v_mfma_f32_32x32x2_f32), one 32-arena tile per wave.
//
// Same orientation as pm_mfma.h: every layer computes H^T = W X^T; a 32x32 accumulator holds column
// `lane & 31` (the arena) and rows (r&3) + 8(r>>2) + 4(lane>>5) (units) in register r, which is the
// B operand of the next layer's k-step r over those unit pairs. The LSTM gates are computed per
// 32-unit hidden block, all four gates together, so the cell update c' = s(f) c + s(i) tanh(g),
// h' = s(o) tanh(c') runs on the accumulators and h' lands directly in the head layer's B layout.
// (h, c) per arena live in HBM [n][128], read and written as float4 in that same unit order.
//
// The effective-weight block (PM_RNN_NW floats) is pre-arranged in fragment order: 615 KB per net,
// streamed through a block-shared LDS ring (see rnn_group).
#pragma once
#include "pm_mfma.h"

namespace pm {

// packed parameter block (PM_RNN_NP floats): the state_dict tensors in modelB.parameters() order,
// then the NoisyLinear epsilon buffers
enum : int {
    R_P_F1W = 0, R_P_F1B = 448, R_P_F2W = 512, R_P_F2B = 8704,
    R_P_WIH = 8832, R_P_WHH = 74368, R_P_BIH = 139904, R_P_BHH = 140416,
    R_P_SWMU = 140928, R_P_SBMU = 157312, R_P_SWSG = 157440, R_P_SBSG = 173824,
    R_P_VWMU = 173952, R_P_VBMU = 174080, R_P_VWSG = 174081, R_P_VBSG = 174209,
    R_P_AWMU = 174210, R_P_ABMU = 174594, R_P_AWSG = 174597, R_P_ABSG = 174981,
    R_P_NPARAM = 174984,
    R_P_SWEP = 174984, R_P_SBEP = 191368, R_P_VWEP = 191496, R_P_VBEP = 191624, R_P_AWEP = 191625,
    R_P_ABEP = 192009, R_P_SIZE = 192012,
};
// effective weights, fragment order (floats)
enum : int {
    R_F1 = 0,         // [jt 2][lane 64][s 4]: k' = 2s + (l>>5); k' = 0 -> b1 (input 1.0), else W1[32jt+(l&31)][k'-1]
    R_F2 = 512,       // [mt 4][t 2][rq 4][lane 64][e 4]: W2[32mt + (l&31)][32t + rho(4rq+e) + 4(l>>5)]
    R_B2 = 8704,      // [mt 4][h 2][r 16]: b2[32mt + rho(r) + 4h]
    R_G = 8832,       // [q 4][m 4][t 8][rq 4][lane 64][e 4]: [Wih|Whh][128q + 32m + (l&31)][32t + rho(4rq+e) + 4(l>>5)]
    R_BG = 139904,    // [q 4][m 4][h 2][r 16]: (bih + bhh)[128q + 32m + rho(r) + 4h]
    R_S = 140416,     // [mt 4][t 4][rq 4][lane 64][e 4]: folded shared-head W
    R_BS = 156800,    // [mt 4][h 2][r 16]
    R_H = 156928,     // [h 2][t 4][r 16][c 4]: heads W[c][32t + rho(r) + 4h], c = 0 V, 1..3 A
    R_BH = 157440,    // [c 4] + 12 pad
    R_NW = 157456,
};
static_assert(R_P_SIZE == PM_RNN_NP && R_NW == PM_RNN_NW, "QNetRNN block sizes");
constexpr int R_NOISE = 128 + 128 + 128 + 1 + 128 + 3;  // eps_in / eps_out of S, V, A (516)

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Hardware-rate activations for the acting path (v_exp_f32, v_rcp_f32: ~1 ulp each, a few ulp
// composed; the accurate forms above cost ~6x the VALU, which the f32 MFMA stream serialises with).
__device__ __forceinline__ float sig_hw(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float tanh_hw(float x) { return 2.0f * sig_hw(2.0f * x) - 1.0f; }

__device__ __forceinline__ void load_acc_bias(const float* __restrict__ b, f32x16& acc) {
    const float4* p = reinterpret_cast<const float4*>(b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 v = p[j];
        acc[4 * j] = v.x; acc[4 * j + 1] = v.y; acc[4 * j + 2] = v.z; acc[4 * j + 3] = v.w;
    }
}

// ---------------------------------------------------------------- the weight ring
// A workgroup of 4 waves runs 4 tiles (128 arenas) of the same net in lockstep. The weights stream
// through a double-buffered LDS ring in 16 KB stages, each stage four 4 KB pieces (one gate, or one
// 32-row tile of a layer) loaded by one wave each with global_load_lds (no registers) while the
// previous stage computes; every wave's MFMA A operands then come from LDS (ds_read_b128), its B
// operands from registers. Per 128 arenas: F2 in 2 stages, then per 32-unit hidden block m the 8
// K-steps of its four gates (t = 0..3: features, 4..7: h_prev) and the shared head's k-tile m.
constexpr int kStageFloats = 4096;  // 16 KB
constexpr int kRingStages = 2 + 4 * 9;

#ifdef PM_DIAG
// diagnostic builds: s_memrealtime after each ring barrier of a block's first group (blocks < 1024)
static __device__ unsigned long long pm_diag_stage[64][1024];  // [0, 48) rnn_group, [48, 64) rnn_tile_split
#define PM_STG(k)                                                                                   \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 1024 && g == 0) pm_diag_stage[(k)][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// shader-clock counter (s_memtime) beside the 100 MHz one: slots 40 (begin) and 47 (end)
#define PM_STG_CLK(k)                                                                               \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 1024 && g == 0) pm_diag_stage[(k)][blockIdx.x] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// split tiles: slot 48 + k of the block, thread 0 (blocks < 1024)
#define PM_SSTG(k)                                                                                  \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 1024) pm_diag_stage[48 + (k)][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PM_SSTG(k) \
    do {           \
    } while (0)
#define PM_STG(k) \
    do {          \
    } while (0)
#define PM_STG_CLK(k) \
    do {              \
    } while (0)
#endif

__device__ __forceinline__ const float* stage_piece(const float* __restrict__ w, int s, int piece) {
    if (s < 2) return w + R_F2 + (piece * 2 + s) * 4 * 256;  // F2: [mt][t = s]
    s -= 2;
    const int m = s / 9, t = s - 9 * m;
    if (t < 8) return w + R_G + ((piece * 4 + m) * 8 + t) * 4 * 256;  // gate q = piece, block m, K-step t
    return w + R_S + (piece * 4 + m) * 4 * 256;                         // shared head tile mt = piece, k-tile m
}

// Issue stage s into `slot`: wave w loads piece w (4 KB = 4 wave instructions of 1 KB). Landed at
// the caller's next __syncthreads() (which waits vmcnt(0)).
__device__ __forceinline__ void stage_issue(const float* __restrict__ w, int s, float* slot) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float4* src = reinterpret_cast<const float4*>(stage_piece(w, s, wv)) + lane;
    float4* dst = reinterpret_cast<float4*>(slot) + wv * 256;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_global_load_lds((const void*)(src + 64 * k), (lds_void*)(dst + 64 * k), 16, 0, 0);
}

// 64 MFMAs of one stage: acc[p] += piece p (A, LDS) x b[4 rq + e] (B, registers).
__device__ __forceinline__ void stage_mfma(const float* slot, const float (&b)[16], f32x16 (&acc)[4], int lane) {
    const float4* a4 = reinterpret_cast<const float4*>(slot) + lane;
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
        float4 a[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) a[p] = a4[(p * 4 + rq) * 64];
        // the four accumulator chains interleaved: consecutive MFMAs never depend on each other
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p].x, b[4 * rq + 0], acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p].y, b[4 * rq + 1], acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p].z, b[4 * rq + 2], acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p].w, b[4 * rq + 3], acc[p], 0, 0, 0);
    }
}

// F2 stage t: one K half (32 units) of all four 32-row feature tiles: b = the layer-1 tile t.
__device__ __forceinline__ void stage_mfma_f2(const float* slot, const f32x16& c1t, f32x16 (&acc)[4], int lane) {
    float b[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) b[r] = c1t[r];
    stage_mfma(slot, b, acc, lane);
}

// Block-shared LDS copy of the small per-net tables: heads (R_H .. R_H + 516) then the biases of
// F2 (R_B2, 128), the gates (R_BG, 512) and the shared head (R_BS, 128).
constexpr int kHwHeads = 0, kHwB2 = 528, kHwBG = kHwB2 + 128, kHwBS = kHwBG + 512, kHwFloats = kHwBS + 128;

__device__ __forceinline__ void stage_tables(const float* __restrict__ w, float* hw) {
    for (int k = threadIdx.x; k < kHwFloats; k += blockDim.x) {
        float v = 0.f;
        if (k < 516) v = w[R_H + k];
        else if (k >= kHwB2 && k < kHwBG) v = w[R_B2 + k - kHwB2];
        else if (k >= kHwBG && k < kHwBS) v = w[R_BG + k - kHwBG];
        else if (k >= kHwBS) v = w[R_BS + k - kHwBS];
        hw[k] = v;
    }
}

__device__ __forceinline__ void add_bias_lds(const float* b, f32x16& acc) {
    const float4* p = reinterpret_cast<const float4*>(b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 v = p[j];
        acc[4 * j] += v.x; acc[4 * j + 1] += v.y; acc[4 * j + 2] += v.z; acc[4 * j + 3] += v.w;
    }
}

// One acting step of QNetRNN for group g of a block's arena list (tiles 4g .. 4g+3, one per wave):
// q values out through `out`, (h, c) rows updated in HBM. Block-wide (all 4 waves, barriers).
// (h, c) are read from hin / cin (null: hst / cst, in place) and written to hst / cst.
template <typename Out>
__device__ __forceinline__ void rnn_group(const float* __restrict__ w, float* ring, const float* hw,
                                          const float* __restrict__ obs, float* hst, float* cst,
                                          const uint8_t* __restrict__ reset, const int* list, int count, int g,
                                          const Out& out, const float* hin = nullptr, const float* cin = nullptr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
    const int row = (4 * g + wave) * 32 + (lane & 31);
    const bool valid = row < count;
    const int arena = list[min(row, count - 1)];
    float* hs = hst + (size_t)arena * 128;
    float* cs = cst + (size_t)arena * 128;
    const float* hr = (hin ? hin : hst) + (size_t)arena * 128;
    const float* cr = (cin ? cin : cst) + (size_t)arena * 128;
    const bool zero = reset != nullptr && reset[arena] != 0;
    PM_STG(0);
    PM_STG_CLK(40);
    stage_issue(w, 0, ring);  // F2 first half lands while the prologue runs
    // ---- prologue: inputs, layer 1, biases, h_prev into the B-operand registers
    float xs[4];
    tile_inputs(obs + (size_t)arena * 7, h, xs);
    float xb[8][16];  // gate K-steps t = 0..7: B operands (features 0..3, h_prev 4..7)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const float4 v = zero ? make_float4(0.f, 0.f, 0.f, 0.f)
                                  : *reinterpret_cast<const float4*>(hr + 32 * t + 8 * rq + 4 * h);
            xb[4 + t][4 * rq] = v.x; xb[4 + t][4 * rq + 1] = v.y; xb[4 + t][4 * rq + 2] = v.z; xb[4 + t][4 * rq + 3] = v.w;
        }
    f32x16 c1[2];
    {
        const f32x16 zero16 = {};
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const float4 a = reinterpret_cast<const float4*>(w + R_F1)[jt * 64 + lane];
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, xs[0], zero16, 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, xs[1], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, xs[2], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, xs[3], c1[jt], 0, 0, 0);
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
    }
    f32x16 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x16{};
    __syncthreads();
    PM_STG(1);
    // ---- F2 (stages 0, 1)
    stage_issue(w, 1, ring + kStageFloats);
    stage_mfma_f2(ring, c1[0], acc, lane);
    __syncthreads();
    PM_STG(2);
    stage_issue(w, 2, ring);
    stage_mfma_f2(ring + kStageFloats, c1[1], acc, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        add_bias_lds(hw + kHwB2 + (mt * 2 + h) * 16, acc[mt]);
#pragma unroll
        for (int r = 0; r < 16; ++r) xb[mt][r] = relu(acc[mt][r]);
    }
    f32x16 sacc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) sacc[mt] = f32x16{};
    __syncthreads();
    PM_STG(3);
    // ---- LSTM: stage s = 2 + 9m + t lives in slot s & 1 = (m + t) & 1
#pragma unroll 1
    for (int m = 0; m < 4; ++m) {
        float4 cp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cp[j] = zero ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(cr + 32 * m + 8 * j + 4 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = f32x16{};
        const int s0 = 2 + 9 * m;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int s = s0 + t;
            stage_issue(w, s + 1, ring + ((s + 1) & 1) * kStageFloats);
            stage_mfma(ring + (s & 1) * kStageFloats, xb[t], acc, lane);
            __syncthreads();
            PM_STG(s + 2);
        }
        // cell update: c' = s(f) c + s(i) tanh(g), h' = s(o) tanh(c') (torch gate order i, f, g, o)
#pragma unroll
        for (int q = 0; q < 4; ++q) add_bias_lds(hw + kHwBG + ((q * 4 + m) * 2 + h) * 16, acc[q]);
        float hb[16];
        {
            float cn[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float cprev = (&cp[r >> 2].x)[r & 3];
                const float ig = sig_hw(acc[0][r]), fg = sig_hw(acc[1][r]);
                const float gg = tanh_hw(acc[2][r]), og = sig_hw(acc[3][r]);
                cn[r] = fg * cprev + ig * gg;
                hb[r] = og * tanh_hw(cn[r]);
            }
            if (valid) {  // h_prev is in registers: the rows can take the new state now
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    *reinterpret_cast<float4*>(cs + 32 * m + 8 * j + 4 * h) =
                        make_float4(cn[4 * j], cn[4 * j + 1], cn[4 * j + 2], cn[4 * j + 3]);
                    *reinterpret_cast<float4*>(hs + 32 * m + 8 * j + 4 * h) =
                        make_float4(hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
                }
            }
        }
        // shared head k-tile m (stage s0 + 8): sacc[mt] += W_S[32mt.., 32m + rho(r) + 4h] h'
        {
            const int s = s0 + 8;
            if (s + 1 < kRingStages) stage_issue(w, s + 1, ring + ((s + 1) & 1) * kStageFloats);
            PM_STG(42 + m);  // cell update done
            stage_mfma(ring + (s & 1) * kStageFloats, hb, sacc, lane);
            __syncthreads();
            PM_STG(s + 2);
        }
    }
    // ---- ReLU(shared head) and the dueling heads (VALU, weights from LDS)
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        add_bias_lds(hw + kHwBS + (mt * 2 + h) * 16, sacc[mt]);
        const float4* hw4 = reinterpret_cast<const float4*>(hw + kHwHeads) + (h * 4 + mt) * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float x = relu(sacc[mt][r]);
            const float4 wv = hw4[r];
            v = fmaf(wv.x, x, v);
            a0 = fmaf(wv.y, x, a0);
            a1 = fmaf(wv.z, x, a1);
            a2 = fmaf(wv.w, x, a2);
        }
    }
    v += __shfl_xor(v, 32);
    a0 += __shfl_xor(a0, 32);
    a1 += __shfl_xor(a1, 32);
    a2 += __shfl_xor(a2, 32);
    v += hw[512];
    a0 += hw[513];
    a1 += hw[514];
    a2 += hw[515];
    const float mean = ((a0 + a1) + a2) / 3.0f;
    const float q[3] = {v + (a0 - mean), v + (a1 - mean), v + (a2 - mean)};
    out(arena, valid && h == 0, q);
    PM_STG(46);
    PM_STG_CLK(47);
}

// ---------------------------------------------------------------- the split tile (side A's tail)
// One 32-arena tile on a whole 4-wave block, for the side-A groups a one-tile-per-wave round would
// leave to a second ~97 us round (round 6). Wave p computes only piece p of every ring stage — the
// F2 output tile p, gate p of each hidden block, the shared head's output tile p — with the same
// MFMA sequence per accumulator as rnn_group (so every result is bit-identical to it), its A
// operands streamed straight into registers four stages ahead (its own 4 KB piece per stage: no
// LDS ring, no barrier per stage). The pieces meet in LDS (xch) where a layer needs all of them:
// the four F2 tiles (the gates' feature K-steps), the four gates of a hidden block (the cell, which
// every wave then evaluates identically, so each holds h' as the head stage's B operand), and the
// four shared-head tiles (the dueling heads, wave 0). 38 stages of 16 MFMAs instead of 64.
#ifndef PM_SPLIT_AHEAD
#define PM_SPLIT_AHEAD 4
#endif
constexpr int kSplitAhead = PM_SPLIT_AHEAD;  // stages of A operands in flight per wave
__device__ __forceinline__ void piece_load(const float* __restrict__ w, int s, int lane, float4 (&a)[4]) {
    const float4* src = reinterpret_cast<const float4*>(stage_piece(w, s, threadIdx.x >> 6)) + lane;
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) a[rq] = src[64 * rq];
}
// piece p's 16 MFMAs of one stage, in stage_mfma's order for acc[p]
__device__ __forceinline__ void piece_mfma(const float4 (&a)[4], const float (&b)[16], f32x16& acc) {
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rq].x, b[4 * rq + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rq].y, b[4 * rq + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rq].z, b[4 * rq + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rq].w, b[4 * rq + 3], acc, 0, 0, 0);
    }
}
struct SplitX {
    float v[2][4][16][64];  // [buffer][wave][register][lane]: 32 KB
};
__device__ __forceinline__ void xch_put(SplitX& x, int buf, int p, int lane, const f32x16& acc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) x.v[buf][p][r][lane] = acc[r];
}

template <typename Out>
__device__ __forceinline__ void rnn_tile_split(const float* __restrict__ w, SplitX& x, const float* hw,
                                               const float* __restrict__ obs, float* hst, float* cst,
                                               const uint8_t* __restrict__ reset, const int* list, int count,
                                               int tile, const Out& out, const float* hin = nullptr,
                                               const float* cin = nullptr) {
    const int lane = threadIdx.x & 63, p = threadIdx.x >> 6, h = lane >> 5;
    const int row = tile * 32 + (lane & 31);
    const bool valid = row < count;
    const int arena = list[min(row, count - 1)];
    float* hs = hst + (size_t)arena * 128;
    float* cs = cst + (size_t)arena * 128;
    const float* hr = (hin ? hin : hst) + (size_t)arena * 128;
    const float* cr = (cin ? cin : cst) + (size_t)arena * 128;
    const bool zero = reset != nullptr && reset[arena] != 0;
    PM_SSTG(0);
    float4 pa[kSplitAhead][4];  // stage s's A operands in pa[s % kSplitAhead] (static after unrolling)
#pragma unroll
    for (int s = 0; s < kSplitAhead; ++s) piece_load(w, s, lane, pa[s]);
    // ---- prologue (rnn_group's): inputs, layer 1, h_prev into the B-operand registers
    float xs[4];
    tile_inputs(obs + (size_t)arena * 7, h, xs);
    float xb[8][16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const float4 v = zero ? make_float4(0.f, 0.f, 0.f, 0.f)
                                  : *reinterpret_cast<const float4*>(hr + 32 * t + 8 * rq + 4 * h);
            xb[4 + t][4 * rq] = v.x; xb[4 + t][4 * rq + 1] = v.y; xb[4 + t][4 * rq + 2] = v.z; xb[4 + t][4 * rq + 3] = v.w;
        }
    f32x16 c1[2];
    {
        const f32x16 zero16 = {};
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const float4 a = reinterpret_cast<const float4*>(w + R_F1)[jt * 64 + lane];
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, xs[0], zero16, 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, xs[1], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, xs[2], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, xs[3], c1[jt], 0, 0, 0);
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
    }
    // ---- F2 (stages 0, 1): output tile p
    f32x16 acc = {};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
        float b[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) b[r] = c1[t2][r];
        piece_mfma(pa[t2], b, acc);
        piece_load(w, t2 + kSplitAhead, lane, pa[t2]);
    }
    add_bias_lds(hw + kHwB2 + (p * 2 + h) * 16, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r]);
    PM_SSTG(1);
    xch_put(x, 0, p, lane, acc);
    __syncthreads();
    PM_SSTG(2);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) xb[mt][r] = x.v[0][mt][r][lane];
    f32x16 sacc = {};
    // ---- LSTM: hidden block m, gate p (stages 2 + 9m .. 2 + 9m + 7), then the shared head (2 + 9m + 8)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float4 cp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cp[j] = zero ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(cr + 32 * m + 8 * j + 4 * h);
        acc = f32x16{};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int s = 2 + 9 * m + t;
            piece_mfma(pa[s % kSplitAhead], xb[t], acc);
            if (s + kSplitAhead < kRingStages) piece_load(w, s + kSplitAhead, lane, pa[s % kSplitAhead]);
        }
        add_bias_lds(hw + kHwBG + ((p * 4 + m) * 2 + h) * 16, acc);
        const int buf = (m + 1) & 1;
        PM_SSTG(3 + 2 * m);
        xch_put(x, buf, p, lane, acc);
        __syncthreads();
        PM_SSTG(4 + 2 * m);
        float hb[16];
        {
            float cn[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float cprev = (&cp[r >> 2].x)[r & 3];
                const float ig = sig_hw(x.v[buf][0][r][lane]), fg = sig_hw(x.v[buf][1][r][lane]);
                const float gg = tanh_hw(x.v[buf][2][r][lane]), og = sig_hw(x.v[buf][3][r][lane]);
                cn[r] = fg * cprev + ig * gg;
                hb[r] = og * tanh_hw(cn[r]);
            }
            if (p == 0 && valid) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    *reinterpret_cast<float4*>(cs + 32 * m + 8 * j + 4 * h) =
                        make_float4(cn[4 * j], cn[4 * j + 1], cn[4 * j + 2], cn[4 * j + 3]);
                    *reinterpret_cast<float4*>(hs + 32 * m + 8 * j + 4 * h) =
                        make_float4(hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
                }
            }
        }
        {
            const int s = 2 + 9 * m + 8;
            piece_mfma(pa[s % kSplitAhead], hb, sacc);
            if (s + kSplitAhead < kRingStages) piece_load(w, s + kSplitAhead, lane, pa[s % kSplitAhead]);
        }
    }
    // ---- the dueling heads from the four shared-head tiles, in rnn_group's chain order (wave 0)
    add_bias_lds(hw + kHwBS + (p * 2 + h) * 16, sacc);
    PM_SSTG(11);
    xch_put(x, 1, p, lane, sacc);
    __syncthreads();
    PM_SSTG(12);
    if (p != 0) return;
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        const float4* hw4 = reinterpret_cast<const float4*>(hw + kHwHeads) + (h * 4 + mt) * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float xv = relu(x.v[1][mt][r][lane]);
            const float4 wv = hw4[r];
            v = fmaf(wv.x, xv, v);
            a0 = fmaf(wv.y, xv, a0);
            a1 = fmaf(wv.z, xv, a1);
            a2 = fmaf(wv.w, xv, a2);
        }
    }
    v += __shfl_xor(v, 32);
    a0 += __shfl_xor(a0, 32);
    a1 += __shfl_xor(a1, 32);
    a2 += __shfl_xor(a2, 32);
    v += hw[512];
    a0 += hw[513];
    a1 += hw[514];
    a2 += hw[515];
    const float mean = ((a0 + a1) + a2) / 3.0f;
    const float q[3] = {v + (a0 - mean), v + (a1 - mean), v + (a2 - mean)};
    out(arena, valid && h == 0, q);
    PM_SSTG(13);
}

}  // namespace pm
