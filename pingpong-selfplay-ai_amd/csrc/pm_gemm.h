// Small fp32 GEMMs on the matrix cores (exact v_mfma_f32_32x32x2_f32), several independent problems
// per launch — the DRQN update's layer GEMMs (forward embedding, heads, weight gradients).
//
//   C(m, n) = epi( sum_k A(m, k) B(k, n) ),  A(m, k) = A[m*sam + k*sak], B(k, n) = B[k*sbk + n*sbn]
//
// One 256-thread workgroup per 32x32 tile of C; the 4 waves split K into quarters (multiples of 8)
// and their accumulators are summed through LDS in a fixed order (deterministic). Within a wave the
// k-slot of each lane half is permuted so that lane (r, h) of MFMA e covers k = kb + 4h + e: an
// operand that is contiguous along k is one float4 per lane per 4 MFMAs; one contiguous along m / n
// is 4 coalesced scalar loads. Epilogue: (+C) (+bias[m]) (+bias2[m]) (ReLU) (x [mask(m, n) > 0]).
#pragma once
#include "pm_dev.h"

namespace pm {

typedef float gemm_f32x16 __attribute__((ext_vector_type(16)));

enum : int { GF_RELU = 1, GF_ACCUM = 2, GF_AVEC = 4, GF_BVEC = 8 };

struct GemmProb {
    const float* A;
    const float* B;
    float* C;
    const float* bias;
    const float* bias2;
    const float* mask;
    int64_t sam, sak, sbk, sbn, scm, scn, smm, smn;
    int M, N, K, flags;
    int tn, blk0;  // tiles along n; first workgroup of this problem (set by gemm_launch)
};

constexpr int kGemmMax = 6;
struct GemmBatch {
    GemmProb p[kGemmMax];
    const int32_t* enable;  // nullable device flag: 0 = skip the whole launch
    int np, nblk;
};

__device__ __forceinline__ void gemm_tile(const GemmProb& P, int tile, float (*red)[16][64]) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5;
    const int m0 = (tile / P.tn) * 32, n0 = (tile % P.tn) * 32;
    const int M = P.M, N = P.N, K = P.K;
    const int kq = ((K + 31) / 32) * 8;
    const int kbeg = w * kq, kend = min(K, kbeg + kq);
    const int m = m0 + r32, n = n0 + r32;
    const bool mv = m < M, nv = n < N;
    const float* __restrict__ Ar = P.A + (int64_t)(mv ? m : 0) * P.sam;
    const float* __restrict__ Bc = P.B + (int64_t)(nv ? n : 0) * P.sbn;
    const bool avec = P.flags & GF_AVEC, bvec = P.flags & GF_BVEC;
    gemm_f32x16 acc = {};
    // chunks of 4 k-steps (32 k): every operand load of the chunk is issued before its 16 MFMAs
    for (int kc = kbeg; kc < kend; kc += 32) {
        float a[16], b[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k0 = kc + 8 * j + 4 * h;
            const bool kin = k0 < kend;
            if (avec) {
                const float4 v = (mv && kin) ? *reinterpret_cast<const float4*>(Ar + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
                a[4 * j] = v.x; a[4 * j + 1] = v.y; a[4 * j + 2] = v.z; a[4 * j + 3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) a[4 * j + e] = (mv && k0 + e < kend) ? Ar[(int64_t)(k0 + e) * P.sak] : 0.f;
            }
            if (bvec) {
                const float4 v = (nv && kin) ? *reinterpret_cast<const float4*>(Bc + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
                b[4 * j] = v.x; b[4 * j + 1] = v.y; b[4 * j + 2] = v.z; b[4 * j + 3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) b[4 * j + e] = (nv && k0 + e < kend) ? Bc[(int64_t)(k0 + e) * P.sbk] : 0.f;
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // the chunk's loads stay ahead of its MFMAs
#pragma unroll
        for (int e = 0; e < 16; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], b[e], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][r][lane] = acc[r];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = threadIdx.x + 256 * j, r = e >> 6, ln = e & 63;
        const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5), nn = n0 + (ln & 31);
        if (mm >= M || nn >= N) continue;
        float v = ((red[0][r][ln] + red[1][r][ln]) + red[2][r][ln]) + red[3][r][ln];
        float* c = P.C + (int64_t)mm * P.scm + (int64_t)nn * P.scn;
        if (P.flags & GF_ACCUM) v = *c + v;
        if (P.bias) v = v + P.bias[mm];
        if (P.bias2) v = v + P.bias2[mm];
        if (P.flags & GF_RELU) v = v > 0.f ? v : 0.f;
        if (P.mask && !(P.mask[(int64_t)mm * P.smm + (int64_t)nn * P.smn] > 0.f)) v = 0.f;
        *c = v;
    }
}

__global__ __launch_bounds__(256) void k_gemm(GemmBatch g) {
    __shared__ float red[4][16][64];
    if (g.enable && *g.enable == 0) return;
    int pi = 0;
#pragma unroll
    for (int j = 1; j < kGemmMax; ++j)
        if (j < g.np && (int)blockIdx.x >= g.p[j].blk0) pi = j;
    // block-uniform problem select without dynamic indexing into the kernel argument
    GemmProb P = g.p[0];
#pragma unroll
    for (int j = 1; j < kGemmMax; ++j)
        if (pi == j) P = g.p[j];
    gemm_tile(P, blockIdx.x - P.blk0, red);
}

// Host side: a problem with the vector flags derived from strides / alignment.
inline GemmProb gemm_prob(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
                          int64_t scm, int64_t scn, int M, int N, int K, int flags = 0, const float* bias = nullptr,
                          const float* bias2 = nullptr, const float* mask = nullptr, int64_t smm = 0,
                          int64_t smn = 0) {
    GemmProb p{};
    p.A = A; p.B = B; p.C = C; p.bias = bias; p.bias2 = bias2; p.mask = mask;
    p.sam = sam; p.sak = sak; p.sbk = sbk; p.sbn = sbn; p.scm = scm; p.scn = scn; p.smm = smm; p.smn = smn;
    p.M = M; p.N = N; p.K = K; p.flags = flags;
    auto al = [](const float* q) { return (((uintptr_t)q) & 15) == 0; };
    if (sak == 1 && (K & 3) == 0 && (M == 1 || (sam & 3) == 0) && al(A)) p.flags |= GF_AVEC;
    if (sbk == 1 && (K & 3) == 0 && (N == 1 || (sbn & 3) == 0) && al(B)) p.flags |= GF_BVEC;
    return p;
}

// Launch up to kGemmMax problems as one grid.
inline hipError_t gemm_launch(const GemmProb* probs, int np, hipStream_t st, const int32_t* enable = nullptr) {
    GemmBatch g{};
    g.np = np;
    g.enable = enable;
    int blk = 0;
    for (int i = 0; i < np; ++i) {
        g.p[i] = probs[i];
        g.p[i].tn = (probs[i].N + 31) / 32;
        g.p[i].blk0 = blk;
        blk += ((probs[i].M + 31) / 32) * g.p[i].tn;
    }
    g.nblk = blk;
    if (blk == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gemm, dim3(blk), dim3(256), 0, st, g);
    return hipGetLastError();
}

}  // namespace pm
