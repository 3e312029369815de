// K8 — the match megakernel: whole greedy episodes in one launch.
//
// The evaluators (scripts/train_iterative.py:171-196 eval_vs_model / eval_vs_pool), the round-robin
// tournament (tests/test_round_robin.py:290-330) and the arena (tests/arena.py:294-320) play
// episodes with frozen nets: reset with a given serve, both players greedy, tick until a score
// reaches max_score. Stepping that as act + env launches per tick moves the fp64 state through HBM
// and pays ~6 launches per tick for a few thousand arenas; here every arena lives in registers for
// its whole episode:
//
//   block = 4 waves = 4 tiles of 32 columns over a range of arenas that share one (net A, net B)
//   pair (the host groups arenas by pair and splits each group into block ranges); both nets'
//   fragment images (2 x 20 KB) are staged into LDS once; then each wave loops: observe -> QNet
//   forward of player A and of player B on the matrix cores (pm_mfma.h tile_hidden / tile_heads,
//   exact f32) -> argmax -> PongEnv2P.step (pm_dev.h tick, fp64). A column whose episode ends
//   takes the next arena of the block's range (lane refill), so the matrix cores keep working on
//   live episodes instead of finished ones; the wave leaves when its range is exhausted and its
//   columns are done, or at max_steps.
//
// Both 32-lane halves of a wave hold the same arena (the MFMA tile layout gives column lane & 31 to
// both halves), so the tick runs duplicated at no cost in a 64-wide wave. Net id -1 is
// HardcodedBallFollower (tests/test_round_robin.py:207-228): move toward the ball x beyond a 0.01
// float32 tolerance. Outputs per arena: final scores, episode length and the sign of rB - rA on the
// last tick (the evaluators' win test, train_iterative.py:180). No barrier after the staging one,
// so each wave leaves on its own; every wave exits by max_steps (arenas still running then, or
// never started, are counted in *status).
#include "pm_host.h"
#include "pm_mfma.h"

using namespace pm;

namespace {

constexpr int kPlayBlock = 256;
constexpr int kPlayArenas = kPlayBlock / 2;  // columns per block: 4 tiles of 32
constexpr int kMaxSlots = 1024;              // slots per block range (staged in LDS)

// 2 x 20 KB weight images + the block's slot table: 68 KB, two blocks per CU
struct PlayShared {
    float lw[2][kLwFloats];
    double sv[kMaxSlots * 3];  // serves of the block's slots (vx, vy, spin)
    int ord[kMaxSlots];        // arena of each slot
    int next;                  // next unclaimed slot
};

// n dwords global -> LDS with global_load_lds (4 B per lane, no registers); published by the
// caller's __syncthreads(). The tail of the last wave instruction re-reads the last dword.
__device__ __forceinline__ void copy_lds_dwords(const void* __restrict__ src, void* dst, int n) {
    if (n <= 0) return;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const uint32_t* s = static_cast<const uint32_t*>(src);
    uint32_t* d = static_cast<uint32_t*>(dst);
    for (int c = wv; c * 64 < n; c += nw) {
        const int k = min(c * 64 + lane, n - 1);
        __builtin_amdgcn_global_load_lds((const void*)(s + k), (lds_void*)(d + c * 64), 4, 0, 0);
    }
}

// layer-1 B operands from register-resident observations (tile_inputs with a register array)
__device__ __forceinline__ void inputs_of(const float (&o)[7], int h, float (&xs)[4]) {
    xs[0] = h ? o[0] : 1.0f;
    xs[1] = h ? o[2] : o[1];
    xs[2] = h ? o[4] : o[3];
    xs[3] = h ? o[6] : o[5];
}

__device__ __forceinline__ int follower(const float (&o)[7]) {  // obs: ball_x [0], own paddle x [4]
    const float tol = 0.01f;
    return o[0] < o[4] - tol ? 0 : (o[0] > o[4] + tol ? 2 : 1);
}

__device__ __forceinline__ int greedy(const float* lw, const float (&o)[7], int lane) {
    float xs[4];
    inputs_of(o, lane >> 5, xs);
    f32x16 c2[2];
    tile_hidden(lw, xs, lane, c2);
    float q[3];
    tile_heads(lw + F_H, c2, lane, q);
    return argmax3(q);
}

// Column c of a wave (both lane halves) plays slots of its block's range one after another: slot
// c first, then the next unclaimed slot (LDS counter) whenever its episode ends. The slot table
// (arena + serve per slot) is staged in LDS with the weights, so a refill is an LDS read.
__global__ __launch_bounds__(kPlayBlock) void k_play(const pm_env_params p, const float* __restrict__ w, int n_nets,
                                                     const int32_t* __restrict__ blk_nets,
                                                     const int32_t* __restrict__ blk_range,
                                                     const int32_t* __restrict__ order,
                                                     const double* __restrict__ serves, int n, int max_steps,
                                                     int32_t* __restrict__ scoreA, int32_t* __restrict__ scoreB,
                                                     int32_t* __restrict__ length, int8_t* __restrict__ last,
                                                     int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) PlayShared sm;
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane & 31;
    int netA = blk_nets[2 * b], netB = blk_nets[2 * b + 1];
    const int start = blk_range[2 * b], count = blk_range[2 * b + 1];
    const bool bad_net = netA < -1 || netA >= n_nets || netB < -1 || netB >= n_nets;
    const bool bad_range = count < 0 || count > kMaxSlots || start < 0;
    const int live = (bad_net || bad_range) ? 0 : count;  // block-uniform; a bad block plays nothing
    if (live > 0) {
        if (netA >= 0) stage_frags_lds(w + (size_t)netA * PM_QNET_NW, sm.lw[0], b);
        if (netB >= 0) stage_frags_lds(w + (size_t)netB * PM_QNET_NW, sm.lw[1], b + kLwChunks / 2);
        copy_lds_dwords(serves + (size_t)start * 3, sm.sv, live * 6);
        copy_lds_dwords(order + start, sm.ord, live);
    }
    if (threadIdx.x == 0) sm.next = kPlayArenas;
    __syncthreads();  // images and slot table in LDS (waits vmcnt(0)); `next` set

    const int s0 = wv * 32 + col;  // this column's first slot
    int slot = s0 < live ? s0 : -1;
    int arena = -1, bad = 0, len = 0;
    Arena a;
    serve(a, 0.0, 0.0, 0.0);
    bool done = true;
    for (int t = 0;; ++t) {
        // (re)fill: a column with no live episode takes its next slot (reset() with the host-drawn
        // serve, envs/my_pong_env_2p.py:83-114); columns that ended claim the next unclaimed one
        if (done && slot >= 0) {  // identical in both halves of a column
            arena = sm.ord[slot];
            serve(a, sm.sv[slot * 3 + 0], sm.sv[slot * 3 + 1], sm.sv[slot * 3 + 2]);
            len = 0;
            done = false;
            if (arena < 0 || arena >= n) { bad += 1; done = true; arena = -1; }
            slot = -2;  // claim another when this episode ends
        }
        if (__ballot(done && slot == -2) != 0) {  // wave-uniform
            int k = live;
            if (done && slot == -2 && lane < 32) k = atomicAdd(&sm.next, 1);
            k = __shfl(k, col);
            if (done && slot == -2) slot = k < live ? k : -1;
            if (__ballot(done && slot >= 0) != 0) continue;  // start the claimed slots before stepping
        }
        if (__ballot(!done) == 0 || t >= max_steps) break;  // wave-uniform
        float oA[7], oB[7];
        observe(a, oA, oB);
        const int aA = netA >= 0 ? greedy(sm.lw[0], oA, lane) : follower(oA);
        const int aB = netB >= 0 ? greedy(sm.lw[1], oB, lane) : follower(oB);
        if (!done) {
            float rA, rB;
            const int d = tick(p, a, aA, aB, rA, rB);
            ++len;
            if (d) {
                if (lane < 32) {
                    scoreA[arena] = a.sA;
                    scoreB[arena] = a.sB;
                    length[arena] = len;
                    last[arena] = (int8_t)(rB > rA ? 1 : (rA > rB ? -1 : 0));
                }
                done = true;
            }
        }
    }
    if (lane < 32) {
        // cut by max_steps: the running episode, and this column's claimed slot if any
        const int lost = (!done && arena >= 0 ? 1 : 0) + bad + (slot >= 0 ? 1 : 0);
        if (lost) atomicAdd(status, lost);
        if ((bad_net || bad_range) && lane == 0 && wv == 0) atomicAdd(status, 1);
    }
}

}  // namespace

extern "C" int pm_play(const pm_env_params* p, const float* w_nets, int32_t n_nets, const int32_t* blk_nets,
                       const int32_t* blk_range, int32_t n_blocks, const int32_t* order, const double* serves,
                       int32_t n, int32_t max_steps, int32_t* scoreA, int32_t* scoreB, int32_t* length, int8_t* last,
                       int32_t* status, void* stream) {
    PM_REQUIRE(n >= 0 && n_blocks >= 0 && n_nets >= 0 && max_steps >= 0, PM_E_SIZE,
               "pm_play: n=%d n_blocks=%d n_nets=%d max_steps=%d", n, n_blocks, n_nets, max_steps);
    if (n_blocks == 0) return PM_OK;
    PM_REQUIRE(p && blk_nets && blk_range && order && serves && scoreA && scoreB && length && last && status,
               PM_E_ARG, "pm_play: null buffer");
    PM_REQUIRE(n_nets == 0 || (w_nets && (((uintptr_t)w_nets) & 15) == 0), PM_E_ARG,
               "pm_play: w_nets must be non-null and 16-byte aligned");
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "pm_play: speed_scale_every must be > 0");
    hipLaunchKernelGGL(k_play, dim3(n_blocks), dim3(kPlayBlock), 0, pm_stream(stream), *p, w_nets, n_nets, blk_nets,
                       blk_range, order, serves, n, max_steps, scoreA, scoreB, length, last, status);
    PM_LAUNCHED("k_play");
    return PM_OK;
}
