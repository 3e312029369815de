// K4 — prioritized replay on the device (scripts/train_iterative.py:49-76).
//
// Proportional sampling as np.random.choice(p=...) does it (cdf = running sum of p_i = prio_i^alpha,
// first index whose running sum exceeds u * total: searchsorted 'right'), restructured for HBM: a
// streaming pass builds the sum tree of pm_per.h (fp32 leaves, 64- and 1024-entry fp64 nodes), then
// a 256-thread block per 64 samples descends it (one block-wide prefix of the chunk sums, then 4
// lanes per sample). Every reduction has a fixed order,
// so a sample is a pure function of (priorities, u) — no atomics anywhere.
#include "pm_dev.h"
#include "pm_host.h"
#include "pm_per.h"

using namespace pm;

namespace {

// Pending push range from the device control block (selfplay: a captured graph needs no host
// round trip), or none.
__device__ __forceinline__ PushRange push_range(const pm_ctrl* ctrl, int64_t n_push, int64_t cap, float alpha) {
    if (!ctrl) return PushRange{0, 0, cap, 0.f};
    return PushRange{ctrl->pos, n_push, cap, prio_pow(ctrl->size == 0 ? 1.0f : ctrl->max_prio, alpha)};
}

__global__ __launch_bounds__(256) void k_per_leaves(const float* __restrict__ prios, int64_t cap, float alpha,
                                                    float* __restrict__ leaf) {
    for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < cap; e += (int64_t)gridDim.x * 256)
        leaf[e] = prio_pow(prios[e], alpha);
}

// Four lanes per level-1 node (per_sub_sum4: lane & 3 sums one 16-leaf quarter, the same combine as
// per_sub_sum), so a wave reads 16 nodes' 4 KB of leaves contiguously instead of 64 scattered 256-B
// rows. The loop bound is block-uniform: every lane of a group of four reaches the shuffles.
__global__ __launch_bounds__(256) void k_per_subs(int64_t cap, float alpha, const pm_ctrl* ctrl, int64_t n_push,
                                                  PerTree tr) {
    const PushRange pr = push_range(ctrl, n_push, cap, alpha);
    for (int64_t t0 = (int64_t)blockIdx.x * 256; t0 < tr.nsub * 4; t0 += (int64_t)gridDim.x * 256) {
        const int64_t t = t0 + threadIdx.x, sb = t >> 2;
        const double v = per_sub_sum4(tr.leaf, sb < tr.nsub ? sb : tr.nsub - 1, pr);
        if ((t & 3) == 0 && sb < tr.nsub) tr.sub[sb] = v;
    }
}

// Both node levels in one launch: a block computes 64 level-1 nodes (four lanes each, as k_per_subs)
// into HBM and LDS, then four of its threads sum their 16-node groups into the level-2 nodes in
// per_chunk_sum's order (same values: the 16 loads per_chunk_sum would issue come from LDS).
__global__ __launch_bounds__(256) void k_per_nodes(int64_t cap, float alpha, const pm_ctrl* ctrl, int64_t n_push,
                                                   PerTree tr) {
    __shared__ double subl[64];
    const PushRange pr = push_range(ctrl, n_push, cap, alpha);
    const int64_t sb = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
    const double v = per_sub_sum4(tr.leaf, sb < tr.nsub ? sb : tr.nsub - 1, pr);
    if ((threadIdx.x & 3) == 0) {
        subl[threadIdx.x >> 2] = sb < tr.nsub ? v : 0.0;
        if (sb < tr.nsub) tr.sub[sb] = v;
    }
    __syncthreads();
    const int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x;
    if (threadIdx.x < 4 && c < tr.nchunk) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < PER_FAN; ++k) acc += subl[threadIdx.x * PER_FAN + k];
        tr.chunk[c] = acc;
    }
}

__global__ __launch_bounds__(256) void k_per_chunks(PerTree tr) {
    for (int64_t c = blockIdx.x * 256 + threadIdx.x; c < tr.nchunk; c += (int64_t)gridDim.x * 256)
        tr.chunk[c] = per_chunk_sum(tr, c);
}

__global__ __launch_bounds__(256) void k_per_sample(int64_t size, double beta, const double* __restrict__ u, uint64_t seed,
                                                    uint64_t counter, PerTree tr, int64_t* __restrict__ idx,
                                                    float* __restrict__ w, int bs) {
    __shared__ PerSampleSmem sm;
    per_sample_block(
        true, size, tr, PushRange{0, 0, size, 0.f}, beta, (int)blockIdx.x * PER_BS, bs, sm,
        [&](int j) {
            if (u) return u[j];
            const U4 r = philox64((uint32_t)j, TAG_PER, counter, seed);
            return u53(r.x, r.y);
        },
        [&](int j, int64_t i, float wr) { idx[j] = i; w[j] = wr; });
}

__global__ __launch_bounds__(1024) void k_per_normalize(float* __restrict__ w, int bs) {
    __shared__ float red[16];
    float m = 0.f;
    for (int j = threadIdx.x; j < bs; j += 1024) m = fmaxf(m, w[j]);
    m = wave_max(m);
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
int per_launch_build(const float* prios, int64_t cap, float alpha, const pm_ctrl* ctrl, int64_t n_push, void* work,
                     hipStream_t st) {
    const PerTree tr = per_tree(work, cap);
    const auto grid = [](int64_t n) {
        const int64_t b = (n + 255) / 256;
        return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
    };
    hipLaunchKernelGGL(k_per_leaves, dim3(grid(cap)), dim3(256), 0, st, prios, cap, alpha, tr.leaf);
    PM_LAUNCHED("k_per_leaves");
    hipLaunchKernelGGL(k_per_subs, dim3(grid(tr.nsub * 4)), dim3(256), 0, st, cap, alpha, ctrl, n_push, tr);
    PM_LAUNCHED("k_per_subs");
    hipLaunchKernelGGL(k_per_chunks, dim3(grid(tr.nchunk)), dim3(256), 0, st, tr);
    PM_LAUNCHED("k_per_chunks");
    return PM_OK;
}
int per_launch_nodes(void* work, int64_t cap, hipStream_t st) {
    const PerTree tr = per_tree(work, cap);
    hipLaunchKernelGGL(k_per_nodes, dim3((unsigned)((tr.nsub + 63) / 64)), dim3(256), 0, st, cap, 0.f,
                       (const pm_ctrl*)nullptr, (int64_t)0, tr);
    PM_LAUNCHED("k_per_nodes");
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
    const PerTree tr = per_tree(work, size);
    PM_REQUIRE(((uintptr_t)work & 15) == 0, PM_E_ARG, "pm_per_sample: work must be 16-byte aligned");
    int rc = per_launch_build(prios, size, alpha, nullptr, 0, work, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_per_sample, dim3(pm_blocks(bs, PER_BS)), dim3(256), 0, st, size, (double)beta, u, seed, counter, tr,
                       idx, w, bs);
    PM_LAUNCHED("k_per_sample");
    hipLaunchKernelGGL(k_per_normalize, dim3(1), dim3(1024), 0, st, w, bs);
    PM_LAUNCHED("k_per_normalize");
    return PM_OK;
}

extern "C" int pm_per_build(const float* prios, int64_t cap, float alpha, void* work, void* stream) {
    PM_REQUIRE(prios && work, PM_E_ARG, "pm_per_build: null buffer");
    PM_REQUIRE(cap > 0, PM_E_SIZE, "pm_per_build: cap=%lld", (long long)cap);
    PM_REQUIRE(((uintptr_t)work & 15) == 0, PM_E_ARG, "pm_per_build: work must be 16-byte aligned");
    return per_launch_build(prios, cap, alpha, nullptr, 0, work, pm_stream(stream));
}

extern "C" int pm_per_update(float* prios, const int64_t* idx, const float* err, int32_t bs, void* stream) {
    PM_REQUIRE(prios && idx && err, PM_E_ARG, "pm_per_update: null buffer");
    PM_REQUIRE(bs > 0, PM_E_SIZE, "pm_per_update: bs=%d", bs);
    return per_launch_update(prios, idx, err, bs, pm_stream(stream));
}
