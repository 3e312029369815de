// K8 — the match megakernel: whole greedy episodes in one launch.
//
// The evaluators (scripts/train_iterative.py:171-196 eval_vs_model / eval_vs_pool), the round-robin
// tournament (tests/test_round_robin.py:290-330) and the arena (tests/arena.py:294-320) play
// episodes with frozen nets: reset with a given serve, both players greedy, tick until a score
// reaches max_score. Stepping that as act + env launches per tick moves the fp64 state through HBM
// and pays ~6 launches per tick for a few thousand arenas; here every arena lives in registers for
// its whole episode:
//
//   block = 4 waves = 4 tiles of 32 arenas that share one (net A, net B) pair (the host groups
//   arenas by pair and pads groups to whole blocks); both nets' fragment images (2 x 20 KB) are
//   staged into LDS once; then each wave loops: observe -> QNet forward of player A and of player
//   B on the matrix cores (pm_mfma.h tile_hidden / tile_heads, 32 arenas per tile, exact f32) ->
//   argmax -> PongEnv2P.step (pm_dev.h tick, fp64) -> until all 32 arenas are done or max_steps.
//
// Both 32-lane halves of a wave hold the same arena (the MFMA tile layout gives column lane & 31 to
// both halves), so the tick runs duplicated at no cost in a 64-wide wave. Net id -1 is
// HardcodedBallFollower (tests/test_round_robin.py:207-228): move toward the ball x beyond a 0.01
// float32 tolerance. Outputs per arena: final scores, episode length and the sign of rB - rA on the
// last tick (the evaluators' win test, train_iterative.py:180). No barrier after the staging one,
// so each wave leaves on its own; every wave exits by max_steps.
#include "pm_host.h"
#include "pm_mfma.h"

using namespace pm;

namespace {

constexpr int kPlayBlock = 256;
constexpr int kPlayArenas = kPlayBlock / 2;  // 4 tiles of 32

struct PlayShared {
    float lw[2][kLwFloats];
};

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

__global__ __launch_bounds__(kPlayBlock) void k_play(const pm_env_params p, const float* __restrict__ w, int n_nets,
                                                     const int32_t* __restrict__ blk_nets,
                                                     const int32_t* __restrict__ arenas,
                                                     const double* __restrict__ serves, int n, int max_steps,
                                                     int32_t* __restrict__ scoreA, int32_t* __restrict__ scoreB,
                                                     int32_t* __restrict__ length, int8_t* __restrict__ last,
                                                     int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) PlayShared sm;
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int netA = blk_nets[2 * b], netB = blk_nets[2 * b + 1];
    const bool bad_net = netA < -1 || netA >= n_nets || netB < -1 || netB >= n_nets;
    if (bad_net) netA = netB = -1;  // block-uniform; reported below
    if (netA >= 0) stage_frags_lds(w + (size_t)netA * PM_QNET_NW, sm.lw[0], b);
    if (netB >= 0) stage_frags_lds(w + (size_t)netB * PM_QNET_NW, sm.lw[1], b + kLwChunks / 2);
    int arena = arenas[(size_t)b * kPlayArenas + wv * 32 + (lane & 31)];
    const bool bad_arena = arena >= n;
    if (bad_arena || bad_net) arena = -1;
    Arena a;
    {
        double vx = 0.0, vy = 0.0, sp = 0.0;
        if (arena >= 0) {
            vx = serves[(size_t)arena * 3 + 0];
            vy = serves[(size_t)arena * 3 + 1];
            sp = serves[(size_t)arena * 3 + 2];
        }
        serve(a, vx, vy, sp);  // reset() with the host-drawn serve (envs/my_pong_env_2p.py:83-114)
    }
    __syncthreads();  // the images are in LDS (waits vmcnt(0))

    bool done = arena < 0;
    int len = 0;
    float lastA = 0.f, lastB = 0.f;
    for (int t = 0; t < max_steps; ++t) {
        if (__ballot(!done) == 0) break;  // wave-uniform
        float oA[7], oB[7];
        observe(a, oA, oB);
        const int aA = netA >= 0 ? greedy(sm.lw[0], oA, lane) : follower(oA);
        const int aB = netB >= 0 ? greedy(sm.lw[1], oB, lane) : follower(oB);
        if (!done) {
            float rA, rB;
            const int d = tick(p, a, aA, aB, rA, rB);
            ++len;
            if (d) { done = true; lastA = rA; lastB = rB; }
        }
    }
    if (lane < 32) {
        if (arena >= 0) {
            scoreA[arena] = a.sA;
            scoreB[arena] = a.sB;
            length[arena] = done ? len : -1;
            last[arena] = (int8_t)(lastB > lastA ? 1 : (lastA > lastB ? -1 : 0));
        }
        if ((arena >= 0 && !done) || bad_arena || (bad_net && lane == 0 && wv == 0)) atomicAdd(status, 1);
    }
}

}  // namespace

extern "C" int pm_play(const pm_env_params* p, const float* w_nets, int32_t n_nets, const int32_t* blk_nets,
                       const int32_t* arenas, int32_t n_blocks, const double* serves, int32_t n, int32_t max_steps,
                       int32_t* scoreA, int32_t* scoreB, int32_t* length, int8_t* last, int32_t* status,
                       void* stream) {
    PM_REQUIRE(n >= 0 && n_blocks >= 0 && n_nets >= 0 && max_steps >= 0, PM_E_SIZE,
               "pm_play: n=%d n_blocks=%d n_nets=%d max_steps=%d", n, n_blocks, n_nets, max_steps);
    if (n_blocks == 0) return PM_OK;
    PM_REQUIRE(p && blk_nets && arenas && serves && scoreA && scoreB && length && last && status, PM_E_ARG,
               "pm_play: null buffer");
    PM_REQUIRE(n_nets == 0 || (w_nets && (((uintptr_t)w_nets) & 15) == 0), PM_E_ARG,
               "pm_play: w_nets must be non-null and 16-byte aligned");
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "pm_play: speed_scale_every must be > 0");
    hipLaunchKernelGGL(k_play, dim3(n_blocks), dim3(kPlayBlock), 0, pm_stream(stream), *p, w_nets, n_nets, blk_nets,
                       arenas, serves, n, max_steps, scoreA, scoreB, length, last, status);
    PM_LAUNCHED("k_play");
    return PM_OK;
}
