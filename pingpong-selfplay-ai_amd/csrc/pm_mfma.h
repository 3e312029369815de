// K2 on the matrix cores: QNet.forward (models/qnet.py:71-75) for 32 rows at a time with the exact
// f32 MFMA v_mfma_f32_32x32x2_f32 (D = A*B + C, bit-for-bit a k-ordered fmaf chain).
//
// Orientation: every layer computes H^T = W * X^T, weights as the A operand (rows = output units),
// activations as the B operand (columns = the 32 arenas of the tile). The accumulator of a 32x32
// tile holds column `lane & 31` and rows (r&3) + 8(r>>2) + 4(lane>>5) in register r, which is
// exactly the B-operand fragment the next layer needs for a k-step covering those two rows — so
// layer 1 -> ReLU -> layer 2 runs on registers with no LDS round trip or lane shuffle. Per tile:
// 8 MFMAs (7->64, K padded to 8) + 64 MFMAs (64->64); the 4 head outputs (V, A0..2) are 128 VALU
// FMAs per lane + one cross-half add, overlapped with the next tile's MFMAs.
//
// Weights are stored pre-arranged in "fragment order" (PM_QNET_NW block, after the plain part) so a
// wave reads each operand with one conflict-free ds_read_b128 per 4 MFMAs after a block stages the
// 20 KB fragment image into LDS.
#pragma once
#include "pm_dev.h"

namespace pm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;  // LDS destination of global_load_lds

constexpr int PLAIN = 4936;  // plain effective weights (4932) padded to 16 B
// fragment image (floats, from w + PLAIN)
enum : int {
    F_W1 = 0,      // [jt 2][lane 64][s 4]            k' = 2s + (l>>5): k' = 0 -> b1[32jt + (l&31)],
                   //                                 else W1[32jt + (l&31)][k' - 1] (input k' = 0 is 1.0)
    F_W2 = 512,    // [jt 2][t 2][rq 4][lane 64][e 4] W2[32jt + (l&31)][32t + rho(4rq+e) + 4(l>>5)]
    F_B1 = 4608,   // [jt 2][h 2][r 16]               b1[32jt + rho(r) + 4h]
    F_B2 = 4672,   // [jt 2][h 2][r 16]               b2[32jt + rho(r) + 4h]
    F_H = 4736,    // [h 2][t 2][r 16][c 4]           Wh[c][32t + rho(r) + 4h]
    F_BH = 4992,   // [c 4] + 12 pad                  bh[c]
    F_SIZE = 5008,
};
static_assert(PLAIN + F_SIZE == PM_QNET_NW, "effective weight block size");

__device__ __forceinline__ int rho(int r) { return (r & 3) + 8 * (r >> 2); }

// ReLU as one v_max_i32 on the float's bits: every negative float (sign bit set) is a negative
// int and becomes +0, every non-negative float is unchanged. fmaxf(x, 0) costs two VALU ops in
// IEEE mode (a canonicalize per max), and VALU time adds to MFMA time on a gfx950 SIMD.
__device__ __forceinline__ float relu(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

// ----------------------------------------------------------------------------- fragment writers
// Feature fragments (W1, W2, b1, b2) + the plain feature copy, from a parameter block. Block-wide.
__device__ __forceinline__ void write_feature_frags(const float* __restrict__ p, float* __restrict__ w) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int k = t; k < PM_QNET_HEAD_OFF; k += nt) w[k] = p[k];
    float* f = w + PLAIN;
    for (int k = t; k < 512; k += nt) {  // W1
        const int jt = k >> 8, lane = (k >> 2) & 63, s = k & 3;
        const int row = 32 * jt + (lane & 31), kk = 2 * s + (lane >> 5);
        f[F_W1 + k] = kk == 0 ? p[B1 + row] : p[W1 + row * 7 + kk - 1];  // bias rides input k' = 0
    }
    for (int k = t; k < 4096; k += nt) {  // W2
        const int e = k & 3, lane = (k >> 2) & 63, rq = (k >> 8) & 3, tt = (k >> 10) & 1, jt = k >> 11;
        const int row = 32 * jt + (lane & 31), col = 32 * tt + rho(4 * rq + e) + 4 * (lane >> 5);
        f[F_W2 + k] = p[W2 + row * 64 + col];
    }
    for (int k = t; k < 64; k += nt) {  // b1, b2
        const int r = k & 15, h = (k >> 4) & 1, jt = k >> 5;
        f[F_B1 + k] = p[B1 + 32 * jt + rho(r) + 4 * h];
        f[F_B2 + k] = p[B2 + 32 * jt + rho(r) + 4 * h];
    }
}

// Head fragments + plain head slice from 260 folded head values (Wh [4][64] | bh [4]). Block-wide.
__device__ __forceinline__ void write_head_frags(const float* heads, float* __restrict__ w) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int k = t; k < 260; k += nt) w[WH + k] = heads[k];
    float* f = w + PLAIN;
    for (int k = t; k < 256; k += nt) {
        const int c = k & 3, r = (k >> 2) & 15, tt = (k >> 6) & 1, h = k >> 7;
        f[F_H + k] = heads[c * 64 + 32 * tt + rho(r) + 4 * h];
    }
    if (t < 16) f[F_BH + t] = t < 4 ? heads[256 + t] : 0.f;
}

// ----------------------------------------------------------------------------- block helpers
constexpr int kLwChunks = (F_SIZE / 4 + 63) / 64;  // 1 KB chunks of the fragment image (20)
constexpr int kLwFloats = kLwChunks * 256;          // LDS image size: whole 1 KB wave chunks

// Copy n floats global -> LDS with global_load_lds (4 B per lane, one wave instruction per 64
// floats, no registers); dst must hold n rounded up to a multiple of 64 (the tail re-reads the
// last element). Block-wide; published by the caller's __syncthreads().
template <int N>
__device__ __forceinline__ void copy_lds_f32(const float* __restrict__ src, float* dst) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int c = wv; c * 64 < N; c += nw) {
        const int k = min(c * 64 + lane, N - 1);
        __builtin_amdgcn_global_load_lds((const void*)(src + k), (lds_void*)(dst + c * 64), 4, 0, 0);
    }
}
constexpr int pad64(int n) { return (n + 63) / 64 * 64; }
// The same copy as 16-byte lanes (1 KB per wave instruction, a quarter of the instructions): src and
// dst 16-byte aligned, N a multiple of 4, dst holding N rounded up to 256 floats. The 4-byte form
// was the last thing to land in the learner's load phase (~2 us after its plain loads).
template <int N>
__device__ __forceinline__ void copy_lds_f32x4(const float* __restrict__ src, float* dst) {
    static_assert(N % 4 == 0, "whole float4s");
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int c = wv; c * 256 < N; c += nw) {
        const int k = min(c * 64 + lane, N / 4 - 1);
        __builtin_amdgcn_global_load_lds((const void*)(s4 + k), (lds_void*)(dst + c * 256), 16, 0, 0);
    }
}
constexpr int pad256(int n) { return (n + 255) / 256 * 256; }

// Stage one net's fragment image global -> LDS directly (global_load_lds: 1 KB per wave
// instruction, no registers, no wait until the caller's barrier). `lw` holds kLwFloats floats.
// Chunk order starts at `rot` so concurrent blocks reading the same image spread over L2 channels.
// Block-wide; the caller's __syncthreads() (which waits vmcnt(0)) publishes the image.
__device__ __forceinline__ void stage_frags_lds(const float* __restrict__ w, float* lw, int rot) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const float4* src = reinterpret_cast<const float4*>(w + PLAIN);
    float4* lw4 = reinterpret_cast<float4*>(lw);
    rot %= kLwChunks;
    for (int c0 = wv; c0 < kLwChunks; c0 += nw) {
        const int c = c0 + rot < kLwChunks ? c0 + rot : c0 + rot - kLwChunks;
        const int k = min(c * 64 + lane, F_SIZE / 4 - 1);  // the pad tail re-reads the last float4
        __builtin_amdgcn_global_load_lds((const void*)(src + k), (lds_void*)(lw4 + c * 64), 16, 0, 0);
    }
}

// Per-env-block opponent lists. Per 256-arena block: its arenas grouped by opponent net for the
// next act (ascending within a net), and (offset << 16 | count) per net, so the act kernel's
// opponent tiles read their rows with two small loads instead of compacting ids next to MFMA waves
// (VALU there waits for the matrix cores). Block-wide (kListBlock threads); more than kListNets
// nets: no lists (the act kernel compacts).
constexpr int kListNets = 64;
constexpr int kListBlock = 256;
struct OppListSmem {
    int woff[kListBlock / 64][kListNets];  // per-wave count, then per-wave offset within the net
    int noff[kListNets], ncnt[kListNets];
};
__device__ __forceinline__ void write_opp_lists(int nn, int32_t* opp_list, int32_t* opp_cnt, OppListSmem& sm, int blk,
                                                int i, bool valid, int net) {
    if (nn > kListNets) return;  // uniform
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int rank = 0;
    for (int k = 0; k < nn; ++k) {
        const bool m = valid && net == k;
        const unsigned long long b = __ballot(m);
        if (m) rank = __popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) sm.woff[wv][k] = __popcll(b);
    }
    __syncthreads();
    if (wv == 0) {  // lane k < nn: per-wave offsets within net k, then an exclusive scan over nets
        int acc = 0;
        if (lane < nn) {
            for (int w = 0; w < kListBlock / 64; ++w) {
                const int c = sm.woff[w][lane];
                sm.woff[w][lane] = acc;
                acc += c;
            }
        }
        const int inc = wave_incl_scan_i32(acc);  // inclusive scan of the net counts across the wave (nn <= 64)
        if (lane < nn) { sm.ncnt[lane] = acc; sm.noff[lane] = inc - acc; }
    }
    __syncthreads();
    if (valid) opp_list[(size_t)blk * kListBlock + sm.noff[net] + sm.woff[wv][net] + rank] = i;
    if ((int)threadIdx.x < nn) opp_cnt[(size_t)blk * nn + threadIdx.x] = (sm.noff[threadIdx.x] << 16) | sm.ncnt[threadIdx.x];
}

// Compaction of the arenas i in [lo, hi) with id[i] == net, in ascending order, into an LDS list.
// Thread t owns ids [lo + 16 t, lo + 16 t + 16): compact_load issues its loads (four int4 when
// aligned; the caller overlaps them with other loads), compact_scan counts matches and places them
// with one block-wide exclusive scan. hi - lo <= 16 * blockDim.x (kListMax at 256 threads);
// `wtot` = LDS scratch of blockDim.x / 64 ints; *count = total. Block-wide.
__device__ __forceinline__ void compact_load(const int32_t* __restrict__ id, int lo, int hi, int (&v)[16]) {
    const int base = lo + 16 * (int)threadIdx.x;
    if (base + 16 <= hi && (reinterpret_cast<uintptr_t>(id + base) & 15) == 0) {
        const int4* p4 = reinterpret_cast<const int4*>(id + base);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 x = p4[q];
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = base + r < hi ? id[base + r] : -1;
    }
}
__device__ __forceinline__ void compact_scan(const int (&v)[16], int net, int lo, int* list, int* count, int* wtot) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = blockDim.x >> 6;
    const int base = lo + 16 * t;
    unsigned mask = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) mask |= (v[r] == net ? 1u : 0u) << r;
    const int c = __popc(mask);
    const int incl = wave_incl_scan_i32(c);
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int off = 0, total = 0;
    for (int w = 0; w < nw; ++w) {
        off += w < wv ? wtot[w] : 0;
        total += wtot[w];
    }
    int p = off + incl - c;
    while (mask) {
        const int r = __ffs(mask) - 1;
        mask &= mask - 1;
        list[p++] = base + r;
    }
    if (t == 0) *count = total;
}

struct TileOut {
    int8_t* act;     // [n] action (argmax, or eps-greedy when eps >= 0)
    float* q;        // [n][3] Q values (nullable)
    double eps;      // < 0: greedy
    uint64_t seed, ctr;
};

// Plain folded heads (Wh [4][64] | bh [4]) -> the F_H/F_BH fragment order (260 floats). Block-wide.
__device__ __forceinline__ void heads_to_frags(const float* heads, float* hf) {
    for (int k = threadIdx.x; k < 260; k += blockDim.x) {
        if (k < 256) {
            const int c = k & 3, r = (k >> 2) & 15, tt = (k >> 6) & 1, h = k >> 7;
            hf[k] = heads[c * 64 + 32 * tt + rho(r) + 4 * h];
        } else {
            hf[k] = heads[k];
        }
    }
}

// Layer 1 (7 -> 64) + ReLU + layer 2 (64 -> 64, pre-ReLU) for one 32-row tile on the matrix cores.
// xs: this lane's layer-1 B operands, input k' = 2s + (lane>>5) with k' = 0 the constant 1.0 (its
// weight column is b1) and k' = 1..7 the observation. The fma chain per output is b1 + W·x in
// k order, as with a bias-initialised accumulator. lw: staged fragments.
__device__ __forceinline__ void tile_hidden(const float* lw, const float (&xs)[4], int lane, f32x16 (&c2)[2]) {
    const int h = lane >> 5;
    f32x16 c1[2];
    const f32x16 zero = {};
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
        const float4 w = reinterpret_cast<const float4*>(lw + F_W1)[jt * 64 + lane];
        c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.x, xs[0], zero, 0, 0, 0);
        c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.y, xs[1], c1[jt], 0, 0, 0);
        c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.z, xs[2], c1[jt], 0, 0, 0);
        c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.w, xs[3], c1[jt], 0, 0, 0);
    }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
    // layer 2: the layer-1 accumulators are the B operands. Operand fragments are read one group
    // (4 MFMAs = 256 cycles) ahead; sched_barrier keeps the scheduler from hoisting all 16 reads
    // (64 registers) to the top.
    const float4* w2 = reinterpret_cast<const float4*>(lw + F_W2) + lane;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
        const float4* b = reinterpret_cast<const float4*>(lw + F_B2 + (jt * 2 + h) * 16);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const float4 v = b[q4];
            c2[jt][4 * q4 + 0] = v.x; c2[jt][4 * q4 + 1] = v.y; c2[jt][4 * q4 + 2] = v.z; c2[jt][4 * q4 + 3] = v.w;
        }
    }
    float4 wcur = w2[0];
#pragma unroll
    for (int g8 = 0; g8 < 16; ++g8) {  // g8 = (jt * 2 + t) * 4 + rq
        const int jt = g8 >> 3, t = (g8 >> 2) & 1, rq = g8 & 3;
        const float4 wnext = w2[((g8 + 1) & 15) * 64];
        c2[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.x, c1[t][4 * rq + 0], c2[jt], 0, 0, 0);
        c2[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.y, c1[t][4 * rq + 1], c2[jt], 0, 0, 0);
        c2[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.z, c1[t][4 * rq + 2], c2[jt], 0, 0, 0);
        c2[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.w, c1[t][4 * rq + 3], c2[jt], 0, 0, 0);
        wcur = wnext;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Dueling heads (VALU) on ReLU(c2): this lane holds 32 of the 64 hidden rows of its column; the two
// lane halves are summed with one cross-half add. hf: F_H/F_BH-ordered heads (260 floats).
// Q = V + (A - mean(A)) in every lane.
__device__ __forceinline__ void tile_heads(const float* hf, const f32x16 (&c2)[2], int lane, float (&q)[3]) {
    const int h = lane >> 5;
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    const float4* hw = reinterpret_cast<const float4*>(hf + h * 128);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float x = relu(c2[t][r]);
            const float4 w = hw[t * 16 + r];
            v = fmaf(w.x, x, v);
            a0 = fmaf(w.y, x, a0);
            a1 = fmaf(w.z, x, a1);
            a2 = fmaf(w.w, x, a2);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    v += __shfl_xor(v, 32);
    a0 += __shfl_xor(a0, 32);
    a1 += __shfl_xor(a1, 32);
    a2 += __shfl_xor(a2, 32);
    v += hf[256];
    a0 += hf[257];
    a1 += hf[258];
    a2 += hf[259];
    const float mean = ((a0 + a1) + a2) / 3.0f;  // A.mean(dim=1)
    q[0] = v + (a0 - mean);
    q[1] = v + (a1 - mean);
    q[2] = v + (a2 - mean);
}

// Layer 1 (both 32-row tiles) and layer-2 tile jt of tile_hidden (pm_mfma.h), MFMA for MFMA in the same
// order: the two layer-2 tiles are independent accumulator chains, so a wave computing one of them
// produces exactly the registers tile_hidden gives for it.
template <typename F>
__device__ __forceinline__ void hidden_half(const float* lw, const float (&xs)[4], int lane, int jt, f32x16& c2,
                                            F&& valu) {
    const int h = lane >> 5;
    f32x16 c1[2];
    const f32x16 zero = {};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const float4 w = reinterpret_cast<const float4*>(lw + F_W1)[t * 64 + lane];
        c1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.x, xs[0], zero, 0, 0, 0);
        c1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.y, xs[1], c1[t], 0, 0, 0);
        c1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.z, xs[2], c1[t], 0, 0, 0);
        c1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.w, xs[3], c1[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) c1[t][r] = relu(c1[t][r]);
    {
        const float4* b = reinterpret_cast<const float4*>(lw + F_B2 + (jt * 2 + h) * 16);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const float4 v = b[q4];
            c2[4 * q4 + 0] = v.x; c2[4 * q4 + 1] = v.y; c2[4 * q4 + 2] = v.z; c2[4 * q4 + 3] = v.w;
        }
    }
    const float4* w2 = reinterpret_cast<const float4*>(lw + F_W2) + lane + jt * 8 * 64;
    float4 wcur = w2[0];
#pragma unroll
    for (int g = 0; g < 8; ++g) {  // g = t * 4 + rq (tile_hidden's g8 for this jt)
        const int t = g >> 2, rq = g & 3;
        const float4 wnext = w2[((g + 1) & 7) * 64];
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.x, c1[t][4 * rq + 0], c2, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.y, c1[t][4 * rq + 1], c2, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.z, c1[t][4 * rq + 2], c2, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(wcur.w, c1[t][4 * rq + 3], c2, 0, 0, 0);
        valu(g);  // independent VALU work, scheduled between this group's dependent MFMAs
        wcur = wnext;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// tile_heads' fmaf chains over the rows of one layer-2 tile (t = the tile), continuing from acc.
__device__ __forceinline__ void heads_half(const float* hf, const f32x16& c2, int lane, int t, float (&acc)[4]) {
    const float4* hw = reinterpret_cast<const float4*>(hf + (lane >> 5) * 128) + t * 16;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float x = relu(c2[r]);
        const float4 w = hw[r];
        acc[0] = fmaf(w.x, x, acc[0]);
        acc[1] = fmaf(w.y, x, acc[1]);
        acc[2] = fmaf(w.z, x, acc[2]);
        acc[3] = fmaf(w.w, x, acc[3]);
    }
}

// tile_heads' tail after the chains (heads_half over both layer-2 tiles): the cross-half add, the
// biases and Q = V + (A - mean(A)).
__device__ __forceinline__ void heads_finish(const float (&acc)[4], const float* hf, float (&q)[3]) {
    float v = acc[0], a0 = acc[1], a1 = acc[2], a2 = acc[3];
    v += __shfl_xor(v, 32);
    a0 += __shfl_xor(a0, 32);
    a1 += __shfl_xor(a1, 32);
    a2 += __shfl_xor(a2, 32);
    v += hf[256];
    a0 += hf[257];
    a1 += hf[258];
    a2 += hf[259];
    const float mean = ((a0 + a1) + a2) / 3.0f;  // A.mean(dim=1)
    q[0] = v + (a0 - mean);
    q[1] = v + (a1 - mean);
    q[2] = v + (a2 - mean);
}

// layer-1 B operands of this lane for observation row o: input k' = 2s + h, k' = 0 -> 1.0 (bias),
// k' >= 1 -> o[k' - 1]
__device__ __forceinline__ void tile_inputs(const float* __restrict__ o, int h, float (&xs)[4]) {
    xs[0] = h ? o[0] : 1.0f;
    xs[1] = o[1 + h];
    xs[2] = o[3 + h];
    xs[3] = o[5 + h];
}

// The first tile's layer-1 operands when the caller could load them before its staging barrier
// (rows lo + k, no list needed): the observation load then shares the weight staging's round trip.
struct TilePre {
    bool have;
    float xs[4];
};

// QNet forward + action for `count` arenas listed in LDS `list` (arena indices), weights staged in
// LDS `lw`. Each wave takes tiles wave, wave + nwaves, ... Wave-uniform control flow throughout.
__device__ __forceinline__ void run_tiles(const float* lw, const float* __restrict__ obs, const int* list, int count,
                                          const TileOut& out, const TilePre pre) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int ntiles = (count + 31) >> 5;
    int tl = wave;
    if (tl >= ntiles) return;  // wave-uniform
    int arena = list[min(tl * 32 + col, count - 1)];
    float xs[4];
    if (pre.have) {
#pragma unroll
        for (int k = 0; k < 4; ++k) xs[k] = pre.xs[k];
    } else {
        tile_inputs(obs + (size_t)arena * 7, h, xs);
    }
    for (; tl < ntiles; tl += nw) {
        const int row = tl * 32 + col;
        const bool valid = row < count;
        // prefetch the next tile's observations: their loads land during this tile's MFMAs
        const int tn = tl + nw;
        int arena_n = arena;
        float xn[4] = {xs[0], xs[1], xs[2], xs[3]};
        if (tn < ntiles) {
            arena_n = list[min(tn * 32 + col, count - 1)];
            tile_inputs(obs + (size_t)arena_n * 7, h, xn);
        }
        f32x16 c2[2];
#ifdef PM_DIAG
        if (tl == wave) {  // first tile: operands in registers
            __builtin_amdgcn_s_waitcnt(0);
            PM_BLK(5);
        }
#endif
        tile_hidden(lw, xs, lane, c2);
#ifdef PM_DIAG
        if (tl == wave) PM_BLK(6);
#endif
        float q[3];
        tile_heads(lw + F_H, c2, lane, q);
#ifdef PM_DIAG
        if (tl == wave) PM_BLK(7);
#endif
        int a = argmax3(q);
        if (out.eps >= 0.0) {  // random.random() < eps ? randint(0,2) : argmax (train_iterative.py:126-130)
            const U4 rr = philox64((uint32_t)arena, TAG_ACT, out.ctr, out.seed);
            if (u53(rr.x, rr.y) < out.eps) a = below(rr.z, 3u);
        }
        if (h == 0 && valid) {
            if (out.act) out.act[arena] = (int8_t)a;
            if (out.q) {
                out.q[(size_t)arena * 3 + 0] = q[0];
                out.q[(size_t)arena * 3 + 1] = q[1];
                out.q[(size_t)arena * 3 + 2] = q[2];
            }
        }
        arena = arena_n;
#pragma unroll
        for (int k = 0; k < 4; ++k) xs[k] = xn[k];
    }
}

// ----------------------------------------------------------------------------- grouped act grid
// Block -> work: [0, nB) chunks of kChunkB arenas for side B (one net: w_B); then side A: net 0 in
// chunks of chunk0 arenas, nets 1..n_opp-1 in chunks of chunk1 arenas each, rows compacted by
// opponent id so every tile has uniform weights.
constexpr int kChunkB = 256;  // side-B rows per block: 8 tiles, two per wave (A-side chunks aim at ~96-128 rows)

struct ActGrid {
    int n, n_opp, chunk0, chunk1, side_b;
    __host__ __device__ int nb() const { return side_b ? (n + kChunkB - 1) / kChunkB : 0; }
    __host__ __device__ int na0() const { return (n + chunk0 - 1) / chunk0; }
    __host__ __device__ int na1() const { return (n + chunk1 - 1) / chunk1; }
    __host__ __device__ int blocks() const { return nb() + na0() + (n_opp - 1) * na1(); }
};

constexpr int kActBlock = 256;
constexpr int kListMax = 4096;        // max chunk size (the act kernels' 256-thread blocks)
constexpr int kListMaxLearn = 16384;  // k_learn's 1024-thread side-A blocks (16 ids per thread)

template <int LIST>
struct ActSharedT {
    static constexpr int kList = LIST;
    float lw[kLwFloats];  // fragment image, padded to whole 1 KB wave chunks
    int list[LIST];
    int count;
    int wtot[16];  // one per wave: up to 1024-thread blocks (k_learn's side-A act blocks)
    int lpre[LIST / 256], loff[LIST / 256], lcnt[LIST / 256];  // per 256-arena segment of the env kernel's lists
};
using ActShared = ActSharedT<kListMax>;
using ActSharedLearn = ActSharedT<kListMaxLearn>;
static_assert(kListMaxLearn / 256 <= 64, "one lane per list segment in act_block's scan");

// Block-wide body of the grouped act kernel for grid block b (blockDim.x == kActBlock). side B:
// eps-greedy on obsB with w_B; side A: greedy on obsA with w_opp[net]. opp == nullptr -> every
// arena plays net 0.
template <class Sh>
__device__ __forceinline__ void act_block(Sh& sh, const ActGrid& g, const float* __restrict__ w_opp,
                                          const int32_t* __restrict__ opp, const float* __restrict__ w_B,
                                          const float* __restrict__ obsA, const float* __restrict__ obsB,
                                          TileOut outA, TileOut outB, int b,
                                          const int32_t* __restrict__ opp_list = nullptr,
                                          const int32_t* __restrict__ opp_cnt = nullptr) {
    const float* w;
    const float* obs;
    TileOut out;
    int net, lo, hi;
    bool compact;
    if (b < g.nb()) {
        w = w_B; obs = obsB; out = outB; net = -1; lo = b * kChunkB; hi = min(lo + kChunkB, g.n); compact = false;
    } else {
        b -= g.nb();
        if (b < g.na0()) { net = 0; lo = b * g.chunk0; hi = min(lo + g.chunk0, g.n); }
        else { b -= g.na0(); net = 1 + b / g.na1(); lo = (b % g.na1()) * g.chunk1; hi = min(lo + g.chunk1, g.n); }
        w = w_opp + (size_t)net * PM_QNET_NW; obs = obsA; out = outA;
        compact = opp != nullptr;
        if (!compact && net != 0) return;  // block-uniform
    }
    // prologue: the fragment image (20 KB) goes global -> LDS directly (global_load_lds, 1 KB per
    // wave instruction, no registers) while this block's opponent ids load into registers: one
    // memory round trip. Each block starts at a different 1 KB chunk so concurrent blocks reading
    // the same image spread over L2 channels. Staging / compaction run at raised priority (their
    // VALU/LDS work loses arbitration to co-resident waves' f32 MFMA streams), the tiles at normal.
    __builtin_amdgcn_s_setprio(2);
    stage_frags_lds(w, sh.lw, b);
    // opponent rows: from the env kernel's per-block lists when the chunk is whole 256-arena blocks
    const bool lists = compact && opp_list != nullptr && (lo & 255) == 0 && (((hi - lo) & 255) == 0 || hi == g.n);
    int ids[16];
    if (compact && !lists) compact_load(opp, lo, hi, ids);
    PM_BLK(4);
    if (lists) {
        const int g0 = lo >> 8, G = (hi - lo + 255) >> 8;  // <= Sh::kList / 256 segments (<= 64)
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            const int v = lane < G ? opp_cnt[(size_t)(g0 + lane) * g.n_opp + net] : 0;
            const int c = v & 0xFFFF;
            const int incl = wave_incl_scan_i32(c);
            if (lane < G) { sh.lpre[lane] = incl - c; sh.loff[lane] = v >> 16; sh.lcnt[lane] = c; }
            if (lane == 63) sh.count = incl;
        }
        __syncthreads();
        const int j0 = threadIdx.x & 15;  // 16 threads per segment
        for (int seg = threadIdx.x >> 4; seg < G; seg += blockDim.x >> 4) {
            const int c = sh.lcnt[seg], dst = sh.lpre[seg];
            const int32_t* src = opp_list + (size_t)(g0 + seg) * 256 + sh.loff[seg];
            int v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = j0 + 16 * r < c ? src[j0 + 16 * r] : 0;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (j0 + 16 * r < c) sh.list[dst + j0 + 16 * r] = v[r];
        }
    } else if (compact) {
        compact_scan(ids, net, lo, sh.list, &sh.count, sh.wtot);
    } else {
        if (threadIdx.x == 0) sh.count = hi - lo;
        for (int k = threadIdx.x; k < hi - lo; k += blockDim.x) sh.list[k] = lo + k;
    }
    // rows lo + k (side B, or a single opponent net): this wave's first tile of observations loads
    // now, in the same round trip as the weight staging (the barrier below waits for both)
    TilePre pre{false, {0.f, 0.f, 0.f, 0.f}};
    if (!compact && !lists) {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, cnt = hi - lo;
        if (wave * 32 < cnt) {  // wave-uniform
            pre.have = true;
            tile_inputs(obs + (size_t)(lo + min(wave * 32 + (lane & 31), cnt - 1)) * 7, lane >> 5, pre.xs);
        }
    }
    __syncthreads();
    PM_BLK(1);
    __builtin_amdgcn_s_setprio(0);
    run_tiles(sh.lw, obs, sh.list, sh.count, out, pre);
}

// modelB's hidden features for the NEXT vector step, computed ahead of the update (the features
// 7 -> 64 -> 64 are frozen, models/qnet.py:62 with train_iterative.py:97: only the dueling heads
// train, so they depend on the observations alone). Tiles [t0, t1) of 32 arenas of obs, one per wave
// at a time: the pre-ReLU layer-2 accumulators c2 of tile_hidden, stored so that the act reads them
// with coalesced float4 loads: tile T, piece k (0..3: c2[0][4k..4k+3], 4..7: c2[1][4(k-4)..]), lane l
// at feat4[(T * 8 + k) * 64 + l]. Bit-identical to computing the tile in the act. Block-wide; lw:
// kLwFloats of LDS for the fragment image of w.
constexpr int kFeatTileFloats = 8 * 64 * 4;
// 16-B store with sc1 (write-through: the line leaves this XCD's L2 instead of staying dirty there
// until the kernel's end-of-launch write-back; the features are read by the next launch only).
__device__ __forceinline__ void store_f4_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v) {
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&v), r, byte_off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void feat_tiles(float* lw, const float* __restrict__ w, const float* __restrict__ obs, int n,
                                           int t0, int t1, float* __restrict__ feat) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    stage_frags_lds(w, lw, t0);
    int tl = t0 + wave;
    float xs[4] = {0.f, 0.f, 0.f, 0.f};
    if (tl < t1) tile_inputs(obs + (size_t)min(tl * 32 + (lane & 31), n - 1) * 7, lane >> 5, xs);
    __syncthreads();
    for (; tl < t1; tl += nw) {  // wave-uniform
        const int tn = tl + nw;
        float xn[4] = {xs[0], xs[1], xs[2], xs[3]};
        if (tn < t1) tile_inputs(obs + (size_t)min(tn * 32 + (lane & 31), n - 1) * 7, lane >> 5, xn);
        f32x16 c2[2];
        tile_hidden(lw, xs, lane, c2);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(feat, (short)0, 0x7fffffff, 0x00020000);
        const int off = (tl * 8 * 64 + lane) * 16;  // bytes; < 2 GB for n < 2^23 arenas
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            store_f4_sc1(rs, off + k * 64 * 16, make_float4(c2[0][4 * k], c2[0][4 * k + 1], c2[0][4 * k + 2], c2[0][4 * k + 3]));
            store_f4_sc1(rs, off + (4 + k) * 64 * 16,
                         make_float4(c2[1][4 * k], c2[1][4 * k + 1], c2[1][4 * k + 2], c2[1][4 * k + 3]));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) xs[k] = xn[k];
    }
}
// One tile's features as feat_tiles stored them.
__device__ __forceinline__ void feat_load(const float* __restrict__ feat, int tile, int lane, f32x16 (&c2)[2]) {
    const float4* src = reinterpret_cast<const float4*>(feat) + (size_t)tile * 8 * 64 + lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 a = src[k * 64], b = src[(4 + k) * 64];
        c2[0][4 * k] = a.x; c2[0][4 * k + 1] = a.y; c2[0][4 * k + 2] = a.z; c2[0][4 * k + 3] = a.w;
        c2[1][4 * k] = b.x; c2[1][4 * k + 1] = b.y; c2[1][4 * k + 2] = b.z; c2[1][4 * k + 3] = b.w;
    }
}

}  // namespace pm
