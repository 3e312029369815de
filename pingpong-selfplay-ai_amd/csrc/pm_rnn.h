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
// streamed from L2 by each wave (one float4 per lane = 1 KB per 4 MFMAs), one step ahead.
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

__device__ __forceinline__ void load_acc_bias(const float* __restrict__ b, f32x16& acc) {
    const float4* p = reinterpret_cast<const float4*>(b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 v = p[j];
        acc[4 * j] = v.x; acc[4 * j + 1] = v.y; acc[4 * j + 2] = v.z; acc[4 * j + 3] = v.w;
    }
}

constexpr int kXStride = 260;  // LDS row (one arena) of the gate input [features 128 | h_prev 128] + pad

// One acting step of QNetRNN for the 32 arenas of this wave's tile (column = lane & 31).
// xs: layer-1 B operands (tile_inputs); hs/cs: this arena's (h, c) rows [128] (read, then written
// with the new state when `valid`); zero_state: start from h = c = 0 (episode start). xl: this
// wave's LDS gate-input rows [32][kXStride]; hw_lds: heads (R_H.. R_BH) staged in LDS. q: Q values.
__device__ __forceinline__ void rnn_tile(const float* __restrict__ w, const float (&xs)[4], float* hs, float* cs,
                                         bool zero_state, bool valid, const float* hw_lds, float* xl, int lane,
                                         float (&q)[3]) {
    const int h = lane >> 5, col = lane & 31;
    float* xrow = xl + col * kXStride;  // this lane's arena: units [0,128) features, [128,256) h_prev
    // ---- features 7 -> 64 -> 128
    {
        f32x16 c1[2];
        const f32x16 zero = {};
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const float4 a = reinterpret_cast<const float4*>(w + R_F1)[jt * 64 + lane];
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, xs[0], zero, 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, xs[1], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, xs[2], c1[jt], 0, 0, 0);
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, xs[3], c1[jt], 0, 0, 0);
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
        const float4* w2 = reinterpret_cast<const float4*>(w + R_F2) + lane;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            f32x16 acc;
            load_acc_bias(w + R_B2 + (mt * 2 + h) * 16, acc);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const float4 a = w2[((mt * 2 + t) * 4 + rq) * 64];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, c1[t][4 * rq + 0], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, c1[t][4 * rq + 1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, c1[t][4 * rq + 2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, c1[t][4 * rq + 3], acc, 0, 0, 0);
                }
            // units 32mt + 8j + 4h + e live in register 4j + e
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<float4*>(xrow + 32 * mt + 8 * j + 4 * h) =
                    make_float4(relu(acc[4 * j]), relu(acc[4 * j + 1]), relu(acc[4 * j + 2]), relu(acc[4 * j + 3]));
        }
    }
    // h_prev into the same rows
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u = 32 * t + 8 * j + 4 * h;
            const float4 v = zero_state ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(hs + u);
            *reinterpret_cast<float4*>(xrow + 128 + u) = v;
        }
    // the wave's rows are written by all its lanes: wave-level LDS visibility before the reads
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    // ---- LSTM gates per 32-unit hidden block m (the four gates interleaved), cell update in place;
    // the shared head's k-tile m consumes that block's h' right away (its K runs over the same blocks)
    f32x16 sacc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) load_acc_bias(w + R_BS + (mt * 2 + h) * 16, sacc[mt]);
    const float4* g4 = reinterpret_cast<const float4*>(w + R_G) + lane;
    const float4* s4 = reinterpret_cast<const float4*>(w + R_S) + lane;
#pragma unroll 1
    for (int m = 0; m < 4; ++m) {
        float4 cp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cp[j] = zero_state ? make_float4(0.f, 0.f, 0.f, 0.f)
                               : *reinterpret_cast<const float4*>(cs + 32 * m + 8 * j + 4 * h);
        f32x16 acc[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) load_acc_bias(w + R_BG + ((gq * 4 + m) * 2 + h) * 16, acc[gq]);
        // weights for (t, rq): g4[(((gq*4 + m)*8 + t)*4 + rq)*64]; software-pipelined one rq-step ahead
        float4 a[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) a[gq] = g4[(((gq * 4 + m) * 8 + 0) * 4 + 0) * 64];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const int nt = rq < 3 ? t : t + 1, nrq = rq < 3 ? rq + 1 : 0;
                float4 an[4];
                if (nt < 8) {
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) an[gq] = g4[(((gq * 4 + m) * 8 + nt) * 4 + nrq) * 64];
                }
                // B operands: units 32t + 8rq + 4h + (0..3) of this arena (k-steps 4rq .. 4rq+3)
                const float4 b = *reinterpret_cast<const float4*>(xrow + 32 * t + 8 * rq + 4 * h);
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    acc[gq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[gq].x, b.x, acc[gq], 0, 0, 0);
                    acc[gq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[gq].y, b.y, acc[gq], 0, 0, 0);
                    acc[gq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[gq].z, b.z, acc[gq], 0, 0, 0);
                    acc[gq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[gq].w, b.w, acc[gq], 0, 0, 0);
                }
                if (nt < 8) {
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) a[gq] = an[gq];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        float hb[16], cn[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float cprev = (&cp[r >> 2].x)[r & 3];
            const float ig = sigmoidf_(acc[0][r]), fg = sigmoidf_(acc[1][r]);
            const float gg = tanhf(acc[2][r]), og = sigmoidf_(acc[3][r]);
            cn[r] = fg * cprev + ig * gg;
            hb[r] = og * tanhf(cn[r]);
        }
        if (valid) {  // h_prev was copied to LDS: the global rows can take the new state now
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                *reinterpret_cast<float4*>(cs + 32 * m + 8 * j + 4 * h) =
                    make_float4(cn[4 * j], cn[4 * j + 1], cn[4 * j + 2], cn[4 * j + 3]);
                *reinterpret_cast<float4*>(hs + 32 * m + 8 * j + 4 * h) =
                    make_float4(hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
            }
        }
        // shared head, k-tile m: sacc[mt] += W_S[32mt.., 32m + rho(r) + 4h] * h'
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const float4 a4 = s4[((mt * 4 + m) * 4 + rq) * 64];
                sacc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, hb[4 * rq + 0], sacc[mt], 0, 0, 0);
                sacc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, hb[4 * rq + 1], sacc[mt], 0, 0, 0);
                sacc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, hb[4 * rq + 2], sacc[mt], 0, 0, 0);
                sacc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, hb[4 * rq + 3], sacc[mt], 0, 0, 0);
            }
    }
    // ---- ReLU(shared head) and the dueling heads (VALU, weights from LDS)
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        const f32x16& acc = sacc[mt];
        const float4* hw = reinterpret_cast<const float4*>(hw_lds) + (h * 4 + mt) * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float x = relu(acc[r]);
            const float4 wv = hw[r];
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
    v += hw_lds[512];
    a0 += hw_lds[513];
    a1 += hw_lds[514];
    a2 += hw_lds[515];
    const float mean = ((a0 + a1) + a2) / 3.0f;
    q[0] = v + (a0 - mean);
    q[1] = v + (a1 - mean);
    q[2] = v + (a2 - mean);
    __builtin_amdgcn_wave_barrier();  // this wave may overwrite its rows for the next tile
}

}  // namespace pm
