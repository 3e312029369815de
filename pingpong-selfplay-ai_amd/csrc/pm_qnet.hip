// K2 — QNet acting for both players (models/qnet.py:52-75, scripts/train_iterative.py:124-130,240).
//
// One row per lane; the effective weights of a network are read through a wave-uniform pointer, so
// the 4 800 MACs of a forward are 4 800 v_fmac_f32 with a scalar-register weight operand (scalar
// loads through the K$, no LDS traffic, no per-lane weight loads). FP32-VALU bound: 9 600 FLOP
// per row and network.
#include "pm_dev.h"
#include "pm_host.h"

using namespace pm;

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void k_fold(const float* params, float* params_out, int mode, uint64_t seed,
                                                 uint64_t counter, const uint64_t* __restrict__ counter_dev,
                                                 float* __restrict__ w_eff) {
    __shared__ float noise[132];
    const float* pb = params + (size_t)blockIdx.x * PM_QNET_NP;
    float* po = params_out ? params_out + (size_t)blockIdx.x * PM_QNET_NP : nullptr;
    float* wb = w_eff + (size_t)blockIdx.x * PM_QNET_NW;
    for (int k = threadIdx.x; k < PM_QNET_HEAD_OFF; k += kBlock) wb[k] = pb[k];  // features: W1 b1 W2 b2
    const uint64_t ctr = counter + (counter_dev ? *counter_dev : 0ull);
    fold_heads(pb, po, mode, seed, TAG_NOISE_ACT, ctr + blockIdx.x, wb + WH, noise);
}

__global__ __launch_bounds__(kBlock) void k_qnet_q(const float* __restrict__ w, const float* __restrict__ x,
                                                   float* __restrict__ q, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const int ii = i < n ? i : n - 1;
    float xi[7], qi[3];
#pragma unroll
    for (int k = 0; k < 7; ++k) xi[k] = x[(size_t)ii * 7 + k];
    qnet_q(w, xi, qi);
    if (i < n) {
#pragma unroll
        for (int k = 0; k < 3; ++k) q[(size_t)i * 3 + k] = qi[k];
    }
}

__global__ __launch_bounds__(kBlock) void k_act(const float* __restrict__ w_opp, const int32_t* __restrict__ opp_id,
                                                const float* __restrict__ w_B, const float* __restrict__ obsA,
                                                const float* __restrict__ obsB, float epsilon,
                                                const double* __restrict__ eps_dev, uint64_t seed, uint64_t counter,
                                                const uint64_t* __restrict__ counter_dev, int8_t* __restrict__ aA,
                                                int8_t* __restrict__ aB, float* __restrict__ qA,
                                                float* __restrict__ qB, int n_opp, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const bool valid = i < n;
    const int ii = valid ? i : n - 1;
    float oa[7], ob[7], qa[3], qb[3];
#pragma unroll
    for (int k = 0; k < 7; ++k) { oa[k] = obsA[(size_t)ii * 7 + k]; ob[k] = obsB[(size_t)ii * 7 + k]; }
    const int id = opp_id ? min(max(opp_id[ii], 0), n_opp - 1) : 0;
    qnet_q_grouped(w_opp, id, oa, qa, valid);
    qnet_q(w_B, ob, qb);
    const double eps = eps_dev ? *eps_dev : (double)epsilon;
    const uint64_t ctr = counter + (counter_dev ? *counter_dev : 0ull);
    const U4 r = philox64((uint32_t)ii, TAG_ACT, ctr, seed);
    const int b = u53(r.x, r.y) < eps ? below(r.z, 3u) : argmax3(qb);
    if (valid) {
        aA[i] = (int8_t)argmax3(qa);
        aB[i] = (int8_t)b;
        if (qA) for (int k = 0; k < 3; ++k) qA[(size_t)i * 3 + k] = qa[k];
        if (qB) for (int k = 0; k < 3; ++k) qB[(size_t)i * 3 + k] = qb[k];
    }
}

}  // namespace

extern "C" int pm_qnet_fold(const float* params, float* params_out, int32_t mode, uint64_t seed, uint64_t counter,
                            const uint64_t* counter_dev, float* w_eff, int32_t count, void* stream) {
    PM_REQUIRE(params && w_eff, PM_E_ARG, "pm_qnet_fold: null buffer");
    PM_REQUIRE(mode >= PM_FOLD_EVAL && mode <= PM_FOLD_TRAIN_FRESH, PM_E_ARG, "pm_qnet_fold: mode %d", mode);
    PM_REQUIRE(count >= 0 && count <= 65535, PM_E_SIZE, "pm_qnet_fold: count=%d", count);
    if (count == 0) return PM_OK;
    hipLaunchKernelGGL(k_fold, dim3(count), dim3(kBlock), 0, pm_stream(stream), params, params_out, mode, seed, counter,
                       counter_dev, w_eff);
    PM_LAUNCHED("k_fold");
    return PM_OK;
}

extern "C" int pm_qnet_q(const float* w_eff, const float* x, float* q, int32_t n, void* stream) {
    PM_REQUIRE(n >= 0, PM_E_SIZE, "pm_qnet_q: n=%d", n);
    if (n == 0) return PM_OK;
    PM_REQUIRE(w_eff && x && q, PM_E_ARG, "pm_qnet_q: null buffer");
    hipLaunchKernelGGL(k_qnet_q, dim3(pm_blocks(n, kBlock)), dim3(kBlock), 0, pm_stream(stream), w_eff, x, q, n);
    PM_LAUNCHED("k_qnet_q");
    return PM_OK;
}

extern "C" int pm_qnet_act(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B,
                           const float* obsA, const float* obsB, float epsilon, const double* eps_dev, uint64_t seed,
                           uint64_t counter, const uint64_t* counter_dev, int8_t* aA, int8_t* aB, float* qA, float* qB,
                           int32_t n, void* stream) {
    PM_REQUIRE(n >= 0 && n_opp >= 1, PM_E_SIZE, "pm_qnet_act: n=%d n_opp=%d", n, n_opp);
    if (n == 0) return PM_OK;
    PM_REQUIRE(w_opp && w_B && obsA && obsB && aA && aB, PM_E_ARG, "pm_qnet_act: null buffer");
    hipLaunchKernelGGL(k_act, dim3(pm_blocks(n, kBlock)), dim3(kBlock), 0, pm_stream(stream), w_opp, opp_id, w_B, obsA,
                       obsB, epsilon, eps_dev, seed, counter, counter_dev, aA, aB, qA, qB, n_opp, n);
    PM_LAUNCHED("k_act");
    return PM_OK;
}
