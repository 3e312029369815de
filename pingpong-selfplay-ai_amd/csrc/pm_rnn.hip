// K5 — QNetRNN acting (models/qnet_rnn.py, scripts/train_rnn_iterative.py:371-389) on the matrix
// cores: fold (NoisyLinear mu + sigma * eps into the fragment-ordered block), single-net step
// (pm_rnn_q: parity / the drop-in module's forward) and the fused two-player act (pm_rnn_act).
#include <stdlib.h>

#include <algorithm>

#include "pm_host.h"
#include "pm_rnn.h"

using namespace pm;

namespace {

constexpr int kRnnBlock = 256;  // 4 waves, one 32-arena tile each at a time
constexpr int kRnnRows = 128;   // arenas per block on the ungrouped side

// reset_noise() (models/qnet_rnn.py:33-41) for fc_shared_head.0, fc_V, fc_A after _scale_noise:
// [0,128) f(eps_in) S | [128,256) f(eps_out) S | [256,384) f(eps_in) V | [384] f(eps_out) V |
// [385,513) f(eps_in) A | [513,516) f(eps_out) A. Philox(seed) counter (index, tag, ctr).
__device__ __forceinline__ void rnn_noise(uint64_t seed, uint64_t ctr, float* noise) {
    for (int k = threadIdx.x; k < R_NOISE; k += blockDim.x) {
        uint32_t layer, which, e;
        if (k < 256) { layer = 0; which = k >= 128; e = (uint32_t)(k & 127); }
        else if (k < 385) { layer = 1; which = k >= 384; e = which ? 0u : (uint32_t)(k - 256); }
        else { layer = 2; which = k >= 513; e = which ? (uint32_t)(k - 513) : (uint32_t)(k - 385); }
        const U4 r = philox64(e, TAG_NOISE_RNN | (layer << 8) | (which << 12), ctr, seed);
        noise[k] = scale_noise(normal(r.x, r.y));
    }
}

// NoisyLinear weight / bias as the forward uses them (qnet_rnn.py:43-50), torch float32 order.
struct RnnFold {
    const float* p;
    const float* noise;  // fresh draws (mode FRESH) or nullptr
    int mode;
    // layer: 0 S (128 x 128), 1 V (1 x 128), 2 A (3 x 128)
    __device__ __forceinline__ float weight(int layer, int row, int k) const {
        const int wmu = layer == 0 ? R_P_SWMU : layer == 1 ? R_P_VWMU : R_P_AWMU;
        const int wsg = layer == 0 ? R_P_SWSG : layer == 1 ? R_P_VWSG : R_P_AWSG;
        const int wep = layer == 0 ? R_P_SWEP : layer == 1 ? R_P_VWEP : R_P_AWEP;
        const int idx = row * 128 + k;
        if (mode == PM_FOLD_EVAL) return p[wmu + idx];
        float eps;
        if (mode == PM_FOLD_TRAIN) {
            eps = p[wep + idx];
        } else {
            const int in0 = layer == 0 ? 0 : layer == 1 ? 256 : 385;
            const int out0 = layer == 0 ? 128 : layer == 1 ? 384 : 513;
            eps = noise[out0 + row] * noise[in0 + k];  // eps_out.ger(eps_in)
        }
        return p[wmu + idx] + p[wsg + idx] * eps;
    }
    __device__ __forceinline__ float bias(int layer, int row) const {
        const int bmu = layer == 0 ? R_P_SBMU : layer == 1 ? R_P_VBMU : R_P_ABMU;
        const int bsg = layer == 0 ? R_P_SBSG : layer == 1 ? R_P_VBSG : R_P_ABSG;
        const int bep = layer == 0 ? R_P_SBEP : layer == 1 ? R_P_VBEP : R_P_ABEP;
        if (mode == PM_FOLD_EVAL) return p[bmu + row];
        const float eps = mode == PM_FOLD_TRAIN ? p[bep + row]
                                                : noise[(layer == 0 ? 128 : layer == 1 ? 384 : 513) + row];
        return p[bmu + row] + p[bsg + row] * eps;
    }
};

constexpr int kFoldBlock = 1024;  // one noise draw per thread (516 draws), one element per thread
__global__ __launch_bounds__(kFoldBlock) void k_rnn_fold(const float* __restrict__ params, float* __restrict__ params_out,
                                                  int mode, uint64_t seed, uint64_t counter,
                                                  const uint64_t* __restrict__ counter_dev, float* __restrict__ w_eff) {
    __shared__ float noise[R_NOISE];
    const int net = blockIdx.y;
    const float* p = params + (size_t)net * PM_RNN_NP;
    float* w = w_eff + (size_t)net * PM_RNN_NW;
    // the fresh draws only where they are read: the shared head / head elements [R_S, ...) and block
    // 0 (modelB's epsilon buffers); the feature and LSTM blocks skip the Box-Muller work (block-uniform)
    const bool need = (blockIdx.x + 1) * blockDim.x > R_S || blockIdx.x == 0;
    if (mode == PM_FOLD_TRAIN_FRESH && need) {
        rnn_noise(seed, counter + (counter_dev ? *counter_dev : 0ull) + (uint64_t)net * 0x10000ull, noise);
        __syncthreads();
    }
    const RnnFold F{p, noise, mode};
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < PM_RNN_NW; e += gridDim.x * blockDim.x) {
        float v;
        if (e < R_F2) {
            const int k = e - R_F1, s = k & 3, lane = (k >> 2) & 63, jt = k >> 8;
            const int row = 32 * jt + (lane & 31), kk = 2 * s + (lane >> 5);
            v = kk == 0 ? p[R_P_F1B + row] : p[R_P_F1W + row * 7 + kk - 1];
        } else if (e < R_B2) {
            const int k = e - R_F2, ee = k & 3, lane = (k >> 2) & 63, rq = (k >> 8) & 3, t = (k >> 10) & 1, mt = k >> 11;
            v = p[R_P_F2W + (32 * mt + (lane & 31)) * 64 + 32 * t + rho(4 * rq + ee) + 4 * (lane >> 5)];
        } else if (e < R_G) {
            const int k = e - R_B2, r = k & 15, h = (k >> 4) & 1, mt = k >> 5;
            v = p[R_P_F2B + 32 * mt + rho(r) + 4 * h];
        } else if (e < R_BG) {
            const int k = e - R_G, ee = k & 3, lane = (k >> 2) & 63, rq = (k >> 8) & 3, t = (k >> 10) & 7;
            const int m = (k >> 13) & 3, gq = k >> 15;
            const int row = 128 * gq + 32 * m + (lane & 31), kk = 32 * (t & 3) + rho(4 * rq + ee) + 4 * (lane >> 5);
            v = t < 4 ? p[R_P_WIH + row * 128 + kk] : p[R_P_WHH + row * 128 + kk];
        } else if (e < R_S) {
            const int k = e - R_BG, r = k & 15, h = (k >> 4) & 1, m = (k >> 5) & 3, gq = k >> 7;
            const int row = 128 * gq + 32 * m + rho(r) + 4 * h;
            v = p[R_P_BIH + row] + p[R_P_BHH + row];
        } else if (e < R_BS) {
            const int k = e - R_S, ee = k & 3, lane = (k >> 2) & 63, rq = (k >> 8) & 3, t = (k >> 10) & 3, mt = k >> 12;
            v = F.weight(0, 32 * mt + (lane & 31), 32 * t + rho(4 * rq + ee) + 4 * (lane >> 5));
        } else if (e < R_H) {
            const int k = e - R_BS, r = k & 15, h = (k >> 4) & 1, mt = k >> 5;
            v = F.bias(0, 32 * mt + rho(r) + 4 * h);
        } else if (e < R_BH) {
            const int k = e - R_H, c = k & 3, r = (k >> 2) & 15, t = (k >> 6) & 3, h = k >> 8;
            const int unit = 32 * t + rho(r) + 4 * h;
            v = c == 0 ? F.weight(1, 0, unit) : F.weight(2, c - 1, unit);
        } else {
            const int c = e - R_BH;
            v = c == 0 ? F.bias(1, 0) : c < 4 ? F.bias(2, c - 1) : 0.f;
        }
        w[e] = v;
    }
    if (mode == PM_FOLD_TRAIN_FRESH && params_out && blockIdx.x == 0) {  // reset_noise leaves the buffers
        float* po = params_out + (size_t)net * PM_RNN_NP;
        for (int k = threadIdx.x; k < 128 * 128; k += blockDim.x) po[R_P_SWEP + k] = noise[128 + (k >> 7)] * noise[k & 127];
        for (int k = threadIdx.x; k < 128; k += blockDim.x) {
            po[R_P_SBEP + k] = noise[128 + k];
            po[R_P_VWEP + k] = noise[384] * noise[256 + k];
            for (int a = 0; a < 3; ++a) po[R_P_AWEP + a * 128 + k] = noise[513 + a] * noise[385 + k];
        }
        if (threadIdx.x < 3) po[R_P_ABEP + threadIdx.x] = noise[513 + threadIdx.x];
        if (threadIdx.x == 0) po[R_P_VBEP] = noise[384];
    }
}

// Action selection and stores for one row: argmax (first max), then the epsilon branch
// (random.random() < eps ? randint(0, 2); the forward still advanced (h, c), :376-380).
struct RowOut {
    int8_t* act;
    float* q;
    double eps;
    uint64_t seed, ctr;
    __device__ __forceinline__ void operator()(int arena, bool store, const float (&qv)[3]) const {
        int a = argmax3(qv);
        if (eps >= 0.0) {
            const U4 rr = philox64((uint32_t)arena, TAG_ACT, ctr, seed);
            if (u53(rr.x, rr.y) < eps) a = below(rr.z, 3u);
        }
        if (store) {
            if (act) act[arena] = (int8_t)a;
            if (q) {
                q[(size_t)arena * 3 + 0] = qv[0];
                q[(size_t)arena * 3 + 1] = qv[1];
                q[(size_t)arena * 3 + 2] = qv[2];
            }
        }
    }
};

constexpr int kRnnList = 2048;  // max arenas per grouped chunk

struct RnnShared {
    float ring[2 * kStageFloats];  // the weight ring (32 KB)
    float hw[kHwFloats];           // heads + biases (stage_tables)
    int list[kRnnList];
    int count;
    int wtot[kRnnBlock / 64];
    int tot[kListNets], gpre[kListNets + 1], scan[kRnnBlock], net;
};

// Side A from the env kernel's per-block opponent lists (write_opp_lists): every net's arenas are
// packed globally into 128-row groups, block b taking group b of the concatenation over nets (only
// each net's last group is partial). Fills sh.list / sh.count; returns the net, or -1 past the end.
// Block-wide; LDS scratch: sh.tot / gpre / scan, sh.list[kRnnRows ..] for the env-block prefix.
constexpr int kMaxEnvBlocks = kRnnList - kRnnRows - 1;  // n <= kMaxEnvBlocks * kListBlock
__device__ __forceinline__ int packed_rows(const int32_t* __restrict__ opp_list, const int32_t* __restrict__ opp_cnt,
                                           int n, int nn, int b, RnnShared& sh) {
    const int t = threadIdx.x, neb = (n + kListBlock - 1) / kListBlock;
    if (t < nn) sh.tot[t] = 0;
    __syncthreads();
    for (int idx = t; idx < neb * nn; idx += blockDim.x) atomicAdd(&sh.tot[idx % nn], opp_cnt[idx] & 0xFFFF);
    __syncthreads();
    if (t == 0) {
        int acc = 0, k = -1;
        for (int j = 0; j < nn; ++j) {
            sh.gpre[j] = acc;
            if (b >= acc) k = j;
            acc += (sh.tot[j] + kRnnRows - 1) / kRnnRows;
        }
        sh.gpre[nn] = acc;
        sh.net = b < acc ? k : -1;
        while (sh.net >= 0 && sh.tot[sh.net] == 0) --sh.net;  // skip nets without arenas
    }
    __syncthreads();
    const int k = sh.net;
    if (k < 0) return -1;
    const int g = b - sh.gpre[k];
    // exclusive prefix over env blocks of net k's counts: pre[e] in sh.list[kRnnRows + e]
    int* pre = sh.list + kRnnRows;
    const int per = (neb + blockDim.x - 1) / blockDim.x, e0 = min(neb, t * per), e1 = min(neb, e0 + per);
    int cnt = 0;
    for (int e = e0; e < e1; ++e) cnt += opp_cnt[(size_t)e * nn + k] & 0xFFFF;
    sh.scan[t] = cnt;
    __syncthreads();
    for (int s = 1; s < (int)blockDim.x; s <<= 1) {
        const int v = t >= s ? sh.scan[t - s] : 0;
        __syncthreads();
        sh.scan[t] += v;
        __syncthreads();
    }
    int acc = sh.scan[t] - cnt;
    for (int e = e0; e < e1; ++e) {
        pre[e] = acc;
        acc += opp_cnt[(size_t)e * nn + k] & 0xFFFF;
    }
    if (t == 0) pre[neb] = sh.tot[k];
    __syncthreads();
    const int count = min(kRnnRows, sh.tot[k] - g * kRnnRows);
    for (int j = t; j < count; j += blockDim.x) {
        const int r = g * kRnnRows + j;
        int lo = 0, hi = neb;  // pre[lo] <= r < pre[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (pre[mid] <= r) lo = mid; else hi = mid;
        }
        const int v = opp_cnt[(size_t)lo * nn + k];
        sh.list[j] = opp_list[(size_t)lo * kListBlock + (v >> 16) + (r - pre[lo])];
    }
    if (t == 0) sh.count = count;
    __syncthreads();
    return k;
}

// All rows of the block's list, 128 per group (block-uniform loop: every wave takes every barrier).
__device__ __forceinline__ void rnn_rows(const float* __restrict__ w, RnnShared& sh, const float* __restrict__ obs,
                                         float* hst, float* cst, const uint8_t* __restrict__ reset, int count,
                                         const RowOut& out, const float* hin = nullptr, const float* cin = nullptr) {
    for (int g = 0; g * kRnnRows < count; ++g)
        rnn_group(w, sh.ring, sh.hw, obs, hst, cst, reset, sh.list, count, g, out, hin, cin);
}

__global__ __launch_bounds__(kRnnBlock, 1) void k_rnn_q(const float* __restrict__ w, const float* __restrict__ x,
                                                        float* h, float* c, const uint8_t* __restrict__ reset,
                                                        float* __restrict__ q, int n) {
    __shared__ RnnShared sh;
    const int lo = blockIdx.x * kRnnRows, hi = min(lo + kRnnRows, n);
    stage_tables(w, sh.hw);
    for (int k = threadIdx.x; k < hi - lo; k += blockDim.x) sh.list[k] = lo + k;
    __syncthreads();
    rnn_rows(w, sh, x, h, c, reset, hi - lo, RowOut{nullptr, q, -1.0, 0, 0});
}

struct RnnActArgs {
    const float* w_opp;
    const int32_t* opp;
    const int32_t *opp_list, *opp_cnt;  // per-env-block lists (packed side A) or null
    const float* w_B;
    const float *obsA, *obsB;
    float *hA, *cA, *hB, *cB;
    const float *hA_in, *cA_in;  // side A's (h, c) source (null: hA / cA in place)
    const uint8_t* reset;
    int8_t *aA, *aB;
    float *qA, *qB;
    double eps;
    const double* eps_dev;
    uint64_t seed, counter;
    const uint64_t* counter_dev;
};

// Block b of the act grid: ActGrid (pm_mfma.h) with kRnnRows-arena chunks on side B (b < nb); side A
// grouped by opponent net (b >= nb). Block-wide. split >= 0 (packed side A only): side-A blocks
// [split, ...) are split tiles, four per group from group `split` on (rnn_tile_split: one 32-arena
// tile per block, its stages spread over the four waves), so the groups past the first round finish
// in ~a quarter of a group's time on the CUs the first round frees.
__device__ __forceinline__ void rnn_act_block(const ActGrid& g, const RnnActArgs& A, int b, RnnShared& sh, int split,
                                              SplitX& sx) {
    const int nb = (g.n + kRnnRows - 1) / kRnnRows;
    const float* w;
    int net = -1, lo, hi;
    bool compact = false;
    if (b >= nb && A.opp_list) {  // side A packed over the env kernel's lists
        const int sb = b - nb;
        const bool tail = split >= 0 && sb >= split;
        const int grp = tail ? split + (sb - split) / 4 : sb, tile = tail ? (sb - split) % 4 : 0;
        const int k = packed_rows(A.opp_list, A.opp_cnt, g.n, g.n_opp, grp, sh);
        if (k < 0) return;                      // block-uniform: past the last group
        if (tail && 32 * tile >= sh.count) return;  // block-uniform: the group has no such tile
        w = A.w_opp + (size_t)k * PM_RNN_NW;
        stage_tables(w, sh.hw);
        __syncthreads();
        const RowOut out{A.aA, A.qA, -1.0, 0, 0};
        if (tail)
            rnn_tile_split(w, sx, sh.hw, A.obsA, A.hA, A.cA, A.reset, sh.list, sh.count, tile, out, A.hA_in, A.cA_in);
        else
            rnn_rows(w, sh, A.obsA, A.hA, A.cA, A.reset, sh.count, out, A.hA_in, A.cA_in);
        return;
    }
    if (b < nb) {
        w = A.w_B; lo = b * kRnnRows; hi = min(lo + kRnnRows, g.n);
    } else {
        b -= nb;
        if (b < g.na0()) { net = 0; lo = b * g.chunk0; hi = min(lo + g.chunk0, g.n); }
        else { b -= g.na0(); net = 1 + b / g.na1(); lo = (b % g.na1()) * g.chunk1; hi = min(lo + g.chunk1, g.n); }
        w = A.w_opp + (size_t)net * PM_RNN_NW;
        compact = A.opp != nullptr;
        if (!compact && net != 0) return;  // block-uniform
    }
    stage_tables(w, sh.hw);
    int ids[16];
    if (compact) compact_load(A.opp, lo, hi, ids);
    if (compact) {
        compact_scan(ids, net, lo, sh.list, &sh.count, sh.wtot);
    } else {
        if (threadIdx.x == 0) sh.count = hi - lo;
        for (int k = threadIdx.x; k < hi - lo; k += blockDim.x) sh.list[k] = lo + k;
    }
    __syncthreads();
    const uint64_t ctr = A.counter + (A.counter_dev ? *A.counter_dev : 0ull);
    const int count = sh.count;
    if (net < 0) {
        const double eps = A.eps_dev ? *A.eps_dev : A.eps;
        rnn_rows(w, sh, A.obsB, A.hB, A.cB, A.reset, count, RowOut{A.aB, A.qB, eps, A.seed, ctr});
    } else {
        rnn_rows(w, sh, A.obsA, A.hA, A.cA, A.reset, count, RowOut{A.aA, A.qA, -1.0, 0, 0}, A.hA_in, A.cA_in);
    }
}

// Blocks [b0, b1) of the act grid, gridDim.x of them at a time (a grid smaller than b1 - b0 loops:
// the overlapped QNetRNN step runs side A on part of the chip beside the DRQN update).
__global__ __launch_bounds__(kRnnBlock, 1) void k_rnn_act(ActGrid g, RnnActArgs A, int b0, int b1, int split) {
    __shared__ RnnShared sh;
    __shared__ SplitX sx;
    for (int b = b0 + (int)blockIdx.x; b < b1; b += (int)gridDim.x) {
        __syncthreads();  // the previous block's LDS tables / lists are dead
        rnn_act_block(g, A, b, sh, split, sx);
    }
}

// The split tail of the packed side-A launch (round 6): PONGMI_RNN_SPLIT=0 turns it off (every group
// on whole blocks, the grid looping); PONGMI_RNN_SPLIT_R=r forces the first split group (tests: 0 =
// every group split). Read per launch.
int split_first(int max_blocks, int groups) {
    const char* e = getenv("PONGMI_RNN_SPLIT");
    if (e && *e && atoi(e) == 0) return -1;
    const char* r = getenv("PONGMI_RNN_SPLIT_R");
    if (r && *r) return std::max(0, std::min(atoi(r), groups));
    return max_blocks > 0 && max_blocks < groups ? max_blocks : -1;
}

}  // namespace

extern "C" int pm_rnn_fold(const float* params, float* params_out, int32_t mode, uint64_t seed, uint64_t counter,
                           const uint64_t* counter_dev, float* w_eff, int32_t count, void* stream) {
    if (count == 0) return PM_OK;
    PM_REQUIRE(params && w_eff && count > 0, PM_E_ARG, "pm_rnn_fold: null buffer or count");
    PM_REQUIRE(mode >= PM_FOLD_EVAL && mode <= PM_FOLD_TRAIN_FRESH, PM_E_ARG, "pm_rnn_fold: mode %d", mode);
    PM_REQUIRE((((uintptr_t)w_eff) & 15) == 0, PM_E_ARG, "pm_rnn_fold: w_eff must be 16-byte aligned");
    hipLaunchKernelGGL(k_rnn_fold, dim3(pm_blocks(PM_RNN_NW, kFoldBlock), count), dim3(kFoldBlock), 0, pm_stream(stream), params,
                       params_out, mode, seed, counter, counter_dev, w_eff);
    PM_LAUNCHED("k_rnn_fold");
    return PM_OK;
}

extern "C" int pm_rnn_q(const float* w_eff, const float* x, float* h, float* c, const uint8_t* reset, float* q,
                        int32_t n, void* stream) {
    if (n == 0) return PM_OK;
    PM_REQUIRE(w_eff && x && h && c && q && n > 0, PM_E_ARG, "pm_rnn_q: null buffer or n");
    PM_REQUIRE(((((uintptr_t)w_eff) | ((uintptr_t)h) | ((uintptr_t)c)) & 15) == 0, PM_E_ARG,
               "pm_rnn_q: w_eff / h / c must be 16-byte aligned");
    hipLaunchKernelGGL(k_rnn_q, dim3(pm_blocks(n, kRnnRows)), dim3(kRnnBlock), 0, pm_stream(stream), w_eff, x, h, c,
                       reset, q, n);
    PM_LAUNCHED("k_rnn_q");
    return PM_OK;
}

int pm_rnn_act_part(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B, const float* obsA,
                    const float* obsB, float* hA, float* cA, float* hB, float* cB, const uint8_t* reset, float epsilon,
                    const double* eps_dev, uint64_t seed, uint64_t counter, const uint64_t* counter_dev, int8_t* aA,
                    int8_t* aB, float* qA, float* qB, int32_t n, int32_t chunk0, int32_t chunk1,
                    const int32_t* opp_list, const int32_t* opp_cnt, int32_t part, int32_t max_blocks, void* stream,
                    const float* hA_in, const float* cA_in) {
    if (n == 0) return PM_OK;
    PM_REQUIRE(!hA_in == !cA_in && (((uintptr_t)hA_in | (uintptr_t)cA_in) & 15) == 0, PM_E_ARG,
               "pm_rnn_act: hA_in / cA_in both set (16-B aligned) or both null");
    PM_REQUIRE(w_opp && w_B && obsA && obsB && hA && cA && hB && cB && aA && aB && n > 0 && n_opp >= 1, PM_E_ARG,
               "pm_rnn_act: null buffer or size");
    PM_REQUIRE(((((uintptr_t)w_opp) | ((uintptr_t)w_B) | ((uintptr_t)hA) | ((uintptr_t)cA) | ((uintptr_t)hB) |
                 ((uintptr_t)cB)) & 15) == 0,
               PM_E_ARG, "pm_rnn_act: weights and hidden states must be 16-byte aligned");
    PM_REQUIRE(part == PM_ACT_ALL || part == PM_ACT_B || part == PM_ACT_A, PM_E_ARG, "pm_rnn_act: part=%d", part);
    if (chunk0 <= 0) chunk0 = 256;
    if (chunk1 <= 0) chunk1 = kRnnList;
    PM_REQUIRE(chunk0 <= kRnnList && chunk1 <= kRnnList, PM_E_SIZE, "pm_rnn_act: chunk > %d", kRnnList);
    const bool lists = opp_list && opp_cnt && opp_id && n_opp <= kListNets;
    PM_REQUIRE(!lists || (n + kListBlock - 1) / kListBlock <= kMaxEnvBlocks, PM_E_SIZE,
               "pm_rnn_act: n %d too large for opponent lists", n);
    const ActGrid g{n, opp_id ? n_opp : 1, chunk0, chunk1, 0};
    const int nb = (n + kRnnRows - 1) / kRnnRows;
    const RnnActArgs a{w_opp, opp_id, lists ? opp_list : nullptr, lists ? opp_cnt : nullptr, w_B, obsA, obsB, hA, cA,
                       hB, cB, hA_in, cA_in, reset, aA, aB, qA, qB, (double)epsilon, eps_dev, seed, counter,
                       counter_dev};
    const int na = lists ? nb + n_opp : g.blocks();  // packed: sum over nets of ceil(rows / 128) <= nb + nets
    const int b0 = part == PM_ACT_A ? nb : 0;
    int b1 = part == PM_ACT_B ? nb : nb + na;
    // side A alone from the lists, on a capped grid (the overlapped step): the groups past the cap run
    // as split tiles, every block once (grid = whole-group blocks + 4 per remaining group)
    const int split = part == PM_ACT_A && lists ? split_first(max_blocks, na) : -1;
    if (split >= 0) b1 = nb + split + 4 * (na - split);
    int grid = b1 - b0;
    if (split < 0 && max_blocks > 0 && grid > max_blocks) grid = max_blocks;
    pm_launch(PM_TIMER_RNN_ACT, k_rnn_act, dim3(grid), dim3(kRnnBlock), pm_stream(stream), g, a, b0, b1, split);
    PM_LAUNCHED("k_rnn_act");
    return PM_OK;
}

extern "C" int pm_rnn_act(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B,
                          const float* obsA, const float* obsB, float* hA, float* cA, float* hB, float* cB,
                          const uint8_t* reset, float epsilon, const double* eps_dev, uint64_t seed, uint64_t counter,
                          const uint64_t* counter_dev, int8_t* aA, int8_t* aB, float* qA, float* qB, int32_t n,
                          int32_t chunk0, int32_t chunk1, const int32_t* opp_list, const int32_t* opp_cnt,
                          void* stream) {
    return pm_rnn_act_part(w_opp, opp_id, n_opp, w_B, obsA, obsB, hA, cA, hB, cB, reset, epsilon, eps_dev, seed,
                           counter, counter_dev, aA, aB, qA, qB, n, chunk0, chunk1, opp_list, opp_cnt, PM_ACT_ALL, 0,
                           stream, nullptr, nullptr);
}

#ifdef PM_DIAG
extern "C" int pm_diag_read_rnn(uint64_t* out) {  // [64][1024] ring-stage stamps (48.. split tiles)
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_stage), sizeof(pm_diag_stage));
}
extern "C" int pm_diag_clear_rnn(void) {
    static unsigned long long z[64][1024];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(pm_diag_stage), z, sizeof(z));
}
#endif
