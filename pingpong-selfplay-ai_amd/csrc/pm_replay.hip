// K4 — prioritized replay on the device (scripts/train_iterative.py:49-76).
//
// Proportional sampling exactly as np.random.choice(p=...) does it (cdf = running sum of
// p_i = prio_i^alpha, first index whose running sum exceeds u * total: searchsorted 'right'),
// restructured for HBM: one streaming pass writes per-1024-entry block sums (fp64), then one wave
// per sample walks block sums and its block with wave-wide inclusive scans. Every reduction has a
// fixed order, so a sample is a pure function of (priorities, u) — no atomics anywhere.
#include "pm_dev.h"
#include "pm_host.h"
#include "pm_per.h"

using namespace pm;

namespace {

__global__ __launch_bounds__(256) void k_per_reduce(const float* __restrict__ prios, PerSize sz, float alpha,
                                                    double* __restrict__ bsum) {
    __shared__ double part[4];
    const int64_t size = sz.get();
    const int64_t nb = (size + PER_CHUNK - 1) / PER_CHUNK;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        double s = 0.0;
        const int64_t base = b * PER_CHUNK;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t e = base + t + k * 256;
            if (e < size) s += (double)powf(prios[e], alpha);
        }
        s = wave_sum(s);
        if (lane == 0) part[wv] = s;
        __syncthreads();
        if (t == 0) bsum[b] = ((part[0] + part[1]) + part[2]) + part[3];
        __syncthreads();
    }
}

}  // namespace


namespace {

__global__ __launch_bounds__(256) void k_per_sample(const float* __restrict__ prios, PerSize sz, float alpha,
                                                    double beta, const double* __restrict__ u, uint64_t seed,
                                                    uint64_t counter, const double* __restrict__ bsum,
                                                    int64_t* __restrict__ idx, float* __restrict__ w, int bs) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= bs) return;  // wave-uniform
    const int64_t size = sz.get();
    double uj;
    if (u) uj = u[j];
    else { const U4 r = philox64((uint32_t)j, TAG_PER, counter, seed); uj = u53(r.x, r.y); }
    int64_t i;
    float wr;
    per_sample_one(prios, size, bsum, alpha, beta, uj, i, wr);
    if ((threadIdx.x & 63) == 0) { idx[j] = i; w[j] = wr; }
}

__global__ __launch_bounds__(1024) void k_per_normalize(float* __restrict__ w, int bs) {
    __shared__ float red[16];
    float m = 0.f;
    for (int j = threadIdx.x; j < bs; j += 1024) m = fmaxf(m, w[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    float mx = red[0];
    for (int k = 1; k < 16; ++k) mx = fmaxf(mx, red[k]);
    for (int j = threadIdx.x; j < bs; j += 1024) w[j] = w[j] / mx;
}

__global__ __launch_bounds__(256) void k_per_update(float* __restrict__ prios, const int64_t* __restrict__ idx,
                                                    const float* __restrict__ err, int bs) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= bs) return;
    const int64_t i = idx[j];
    for (int k = j + 1; k < bs; ++k)
        if (idx[k] == i) return;  // a later duplicate wins (sequential update order)
    prios[i] = fabsf(err[j]) + 1e-6f;
}

}  // namespace

extern "C" int64_t pm_per_work_bytes(int64_t cap) { return per_work_bytes(cap); }

namespace pm {
int per_launch_reduce(const float* prios, PerSize sz, int64_t cap, float alpha, double* bsum, hipStream_t st) {
    const int64_t nb = (cap + PER_CHUNK - 1) / PER_CHUNK;
    const unsigned grid = (unsigned)(nb < 4096 ? (nb > 0 ? nb : 1) : 4096);
    hipLaunchKernelGGL(k_per_reduce, dim3(grid), dim3(256), 0, st, prios, sz, alpha, bsum);
    PM_LAUNCHED("k_per_reduce");
    return PM_OK;
}
int per_launch_update(float* prios, const int64_t* idx, const float* err, int bs, hipStream_t st) {
    hipLaunchKernelGGL(k_per_update, dim3(pm_blocks(bs, 256)), dim3(256), 0, st, prios, idx, err, bs);
    PM_LAUNCHED("k_per_update");
    return PM_OK;
}
}  // namespace pm

extern "C" int pm_per_sample(const float* prios, int64_t size, float alpha, float beta, const double* u, uint64_t seed,
                             uint64_t counter, int64_t* idx, float* w, int32_t bs, void* work, void* stream) {
    PM_REQUIRE(prios && idx && w && work, PM_E_ARG, "pm_per_sample: null buffer");
    PM_REQUIRE(size > 0 && bs > 0, PM_E_SIZE, "pm_per_sample: size=%lld bs=%d", (long long)size, bs);
    hipStream_t st = pm_stream(stream);
    double* bsum = reinterpret_cast<double*>(work);
    PerSize sz{size, nullptr, 0, 0};
    int rc = per_launch_reduce(prios, sz, size, alpha, bsum, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_per_sample, dim3(pm_blocks(bs, 4)), dim3(256), 0, st, prios, sz, alpha, (double)beta, u, seed,
                       counter, bsum, idx, w, bs);
    PM_LAUNCHED("k_per_sample");
    hipLaunchKernelGGL(k_per_normalize, dim3(1), dim3(1024), 0, st, w, bs);
    PM_LAUNCHED("k_per_normalize");
    return PM_OK;
}

extern "C" int pm_per_update(float* prios, const int64_t* idx, const float* err, int32_t bs, void* stream) {
    PM_REQUIRE(prios && idx && err, PM_E_ARG, "pm_per_update: null buffer");
    PM_REQUIRE(bs > 0, PM_E_SIZE, "pm_per_update: bs=%d", bs);
    return per_launch_update(prios, idx, err, bs, pm_stream(stream));
}
