// K2 — QNet folding and acting (models/qnet.py:6-75, scripts/train_iterative.py:124-130,240).
//
//   k_fold      NoisyLinear fold (eval / train / reset_noise + train) of the dueling heads, plus
//               the MFMA fragment image of the whole net (pm_mfma.h)
//   k_act       both players' QNet forward on the matrix cores, 32-arena tiles, rows grouped by
//               opponent net (ActGrid), epsilon-greedy for B, argmax (first index) for both
//   k_act(q)    QNet.forward only (same tiles, one net)
#include "pm_host.h"
#include "pm_mfma.h"

using namespace pm;

namespace {

__global__ __launch_bounds__(256) void k_fold(const float* params, float* params_out, int mode, uint64_t seed,
                                              uint64_t counter, const uint64_t* __restrict__ counter_dev,
                                              float* __restrict__ w_eff) {
    __shared__ float heads[260], noise[132];
    const float* pb = params + (size_t)blockIdx.x * PM_QNET_NP;
    float* po = params_out ? params_out + (size_t)blockIdx.x * PM_QNET_NP + PM_QNET_EPS_OFF : nullptr;
    float* wb = w_eff + (size_t)blockIdx.x * PM_QNET_NW;
    write_feature_frags(pb, wb);
    const uint64_t ctr = counter + (counter_dev ? *counter_dev : 0ull);
    fold_heads(pb, po, mode, seed, TAG_NOISE_ACT, ctr + blockIdx.x, heads, noise);
    __syncthreads();
    write_head_frags(heads, wb);
}

__global__ __launch_bounds__(kActBlock, 4) void k_act(ActGrid g, const float* __restrict__ w_opp,
                                                   const int32_t* __restrict__ opp, const float* __restrict__ w_B,
                                                   const float* __restrict__ obsA, const float* __restrict__ obsB,
                                                   TileOut outA, TileOut outB, const double* __restrict__ eps_dev,
                                                   const uint64_t* __restrict__ counter_dev) {
    __shared__ __attribute__((aligned(16))) ActShared sh;
    if (eps_dev) outB.eps = *eps_dev;
    if (counter_dev) outB.ctr += *counter_dev;
    act_block(sh, g, w_opp, opp, w_B, obsA, obsB, outA, outB, blockIdx.x);
}

}  // namespace

extern "C" int pm_qnet_fold(const float* params, float* params_out, int32_t mode, uint64_t seed, uint64_t counter,
                            const uint64_t* counter_dev, float* w_eff, int32_t count, void* stream) {
    PM_REQUIRE(mode >= PM_FOLD_EVAL && mode <= PM_FOLD_TRAIN_FRESH, PM_E_ARG, "pm_qnet_fold: mode %d", mode);
    PM_REQUIRE(count >= 0 && count <= 65535, PM_E_SIZE, "pm_qnet_fold: count=%d", count);
    if (count == 0) return PM_OK;
    PM_REQUIRE(params && w_eff, PM_E_ARG, "pm_qnet_fold: null buffer");
    PM_REQUIRE(((uintptr_t)w_eff & 15) == 0, PM_E_ARG, "pm_qnet_fold: w_eff must be 16-byte aligned");
    hipLaunchKernelGGL(k_fold, dim3(count), dim3(256), 0, pm_stream(stream), params, params_out, mode, seed, counter,
                       counter_dev, w_eff);
    PM_LAUNCHED("k_fold");
    return PM_OK;
}

extern "C" int pm_qnet_q(const float* w_eff, const float* x, float* q, int32_t n, void* stream) {
    PM_REQUIRE(n >= 0, PM_E_SIZE, "pm_qnet_q: n=%d", n);
    if (n == 0) return PM_OK;
    PM_REQUIRE(w_eff && x && q, PM_E_ARG, "pm_qnet_q: null buffer");
    PM_REQUIRE(((uintptr_t)w_eff & 15) == 0, PM_E_ARG, "pm_qnet_q: w_eff must be 16-byte aligned");
    ActGrid g{n, 1, 256, 256, 0};
    TileOut out{nullptr, q, -1.0, 0, 0};
    hipLaunchKernelGGL(k_act, dim3(g.blocks()), dim3(kActBlock), 0, pm_stream(stream), g, w_eff, nullptr, w_eff, x,
                       x, out, out, nullptr, nullptr);
    PM_LAUNCHED("k_act(q)");
    return PM_OK;
}

extern "C" int pm_qnet_act(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B,
                           const float* obsA, const float* obsB, float epsilon, const double* eps_dev, uint64_t seed,
                           uint64_t counter, const uint64_t* counter_dev, int8_t* aA, int8_t* aB, float* qA, float* qB,
                           int32_t n, int32_t chunk0, int32_t chunk1, void* stream) {
    PM_REQUIRE(n >= 0 && n_opp >= 1 && n_opp <= 4097, PM_E_SIZE, "pm_qnet_act: n=%d n_opp=%d", n, n_opp);
    if (n == 0) return PM_OK;
    PM_REQUIRE(w_opp && w_B && obsA && obsB && aA && aB, PM_E_ARG, "pm_qnet_act: null buffer");
    PM_REQUIRE((((uintptr_t)w_opp | (uintptr_t)w_B) & 15) == 0, PM_E_ARG, "pm_qnet_act: weights must be 16-B aligned");
    if (chunk0 <= 0) chunk0 = 256;
    if (chunk1 <= 0) chunk1 = kListMax;
    PM_REQUIRE(chunk0 <= kListMax && chunk1 <= kListMax, PM_E_SIZE, "pm_qnet_act: chunk > %d", kListMax);
    ActGrid g{n, opp_id ? n_opp : 1, chunk0, chunk1, 1};
    TileOut outA{aA, qA, -1.0, 0, 0};
    TileOut outB{aB, qB, (double)epsilon, seed, counter};
    hipLaunchKernelGGL(k_act, dim3(g.blocks()), dim3(kActBlock), 0, pm_stream(stream), g, w_opp, opp_id, w_B, obsA,
                       obsB, outA, outB, eps_dev, counter_dev);
    PM_LAUNCHED("k_act");
    return PM_OK;
}
