// K9 — inference-only self-play rollout, K vector steps per launch (BASELINE configs[1]).
//
// The rollout of scripts/train_iterative.py:239-242 without learning, for n arenas in lockstep: per
// vector step both players act — modelA greedy on its folded weights (:240; modelA keeps NoisyNet's
// frozen epsilon buffers), modelB NoisyNet with fresh noise per vector step shared by all arenas
// (reset_noise in select_action_B, :125) and epsilon-greedy (:126-130) — then PongEnv2P.step ticks
// every arena and finished ones are served again (the step-keyed Philox serve of pm_env_step's
// production autoreset). Stepped as launches, one vector step is three kernels (fold, act, env) that
// move the fp64 state and the observations through HBM; here every arena stays in registers for all
// K steps and only its final state leaves the CU.
//
// Two kernels per launch:
//   k_rollout_heads — one block per step folds modelB's heads with that step's noise (gen_noise +
//     fold_heads_from, exactly pm_qnet_fold FRESH) into the F_H/F_BH fragment order: 264 floats per
//     step in a caller workspace (PM_ROLL_HEADS);
//   k_rollout — a block of 4 waves (kRollBlock = 256) owns one tile of 32 arenas. Wave 2p + j works
//     for player p (0 = A, 1 = B) and computes layer-2 tile j of that player's forward (layer 1 in
//     both), so a forward is 40 dependent MFMAs on two SIMDs instead of 72 on one. The j = 0 wave runs
//     the head chains over its rows and hands the partial sums to the j = 1 wave through LDS (part[]),
//     which continues them in tile_heads' fmaf order and forms the action. Every wave keeps the same
//     fp64 arena in both lane halves (the MFMA tile layout gives column lane & 31 to both), the
//     actions meet in LDS behind the step's barriers and all four waves tick identically. Wave 3
//     streams the next step's heads global -> LDS (global_load_lds, 1 KB, double-buffered) while it
//     computes the current step, so the heads never cost a round trip on the step's critical path.
//
// Bit-identical to `steps` repetitions of pm_qnet_fold(paramsB, FRESH, seed_net, c) ->
// pm_qnet_act({wA}, NULL, w_B, obsA, obsB, epsilon, seed_env, c) -> pm_env_step(autoreset, seed_env,
// c) with c = counter0 + s (tests/test_gpu_rollout.py).
//
// pm_rollout_push (§8f3, the collecting rollout) runs the same launch and also writes every vector
// step's transitions straight from registers into the replay ring, as memory.push((oB, aB, rB, nB,
// done)) does in the training loop (train_iterative.py:242-243, :56-63): one 64-byte row (s[7], r,
// s'[7], bits(aB | done << 8)), its priority and its PER leaf, with ep_reward carried per arena
// (:238, :245) and the episodes' win / reward counts (:247-249). Wave 3 issues the step's three
// stores right after the tick; the vmcnt(0) it already waits on for the next step's heads retires
// them a full step later, so no store latency reaches the step's critical path.
#include <stdlib.h>

#include "pm_host.h"
#include "pm_mfma.h"
#include "pm_per.h"

using namespace pm;

namespace {

constexpr int kRollBlock = 256;  // waves 2p + j: player p (0 = A, 1 = B), layer-2 tile j; one tile of 32 arenas
constexpr int kHeadsBlock = 256;
static_assert(PM_ROLL_HEADS == 264, "heads workspace stride: 256 fragment floats + 4 biases + 4 pad");

__global__ __launch_bounds__(kHeadsBlock) void k_rollout_heads(const float* __restrict__ paramsB, uint64_t seed_net,
                                                               uint64_t counter0, float* __restrict__ ws) {
    __shared__ float noise[132];
    __shared__ float heads[260];
    gen_noise(seed_net, TAG_NOISE_ACT, counter0 + blockIdx.x, noise, threadIdx.x, blockDim.x);
    __syncthreads();
    fold_heads_from(paramsB + PM_QNET_HEAD_OFF, nullptr, noise, PM_FOLD_TRAIN_FRESH, heads, nullptr, threadIdx.x,
                    blockDim.x);
    __syncthreads();
    float* hf = ws + (size_t)blockIdx.x * PM_ROLL_HEADS;
    heads_to_frags(heads, hf);
    if (threadIdx.x < 4) hf[260 + threadIdx.x] = 0.f;
}

struct RollShared {
    float lw[kLwFloats];   // modelA's fragment image
    float lwB[kLwFloats];  // modelB's feature fragments (its heads come from hf)
    float hf[2][320];      // modelB's heads of the step (fragment order, 256 + biases), double-buffered
    __attribute__((aligned(16))) float part[2][2][64][4];  // [step & 1][player] head chains after c2[0]
    int act[2][2][32];     // [step & 1][player][column]
};

// Stream step t's heads (PM_ROLL_HEADS floats at ws + t * PM_ROLL_HEADS) into dst: one 16-byte and one
// 4-byte global_load_lds (the latter's tail lanes re-read the biases' pad). Wave-wide; completes at
// the issuing wave's next vmcnt(0).
__device__ __forceinline__ void fetch_heads(const float* __restrict__ ws, int t, float* dst, int lane) {
    const float* src = ws + (size_t)t * PM_ROLL_HEADS;
    __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const float4*>(src) + lane), (lds_void*)dst, 16,
                                     0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 256 + (lane & 7)), (lds_void*)(dst + 256), 4, 0, 0);
}

// fetch_heads for the loop: the same two LDS-DMA loads issued from inline asm. With the builtin the
// compiler cannot tell the DMA's LDS target from the weight image the next ds_reads hit and puts a
// vmcnt(0) right behind the fetch (measured in the ISA: the prefetch then overlapped nothing, and a
// collecting launch's replay stores were waited there too). Issued here, the only wait is the
// explicit vmcnt(0) wave 3 executes before the step's second barrier.
__device__ __forceinline__ void fetch_heads_async(const float* __restrict__ ws, int t, float* dst, int lane) {
    const float* src = ws + (size_t)t * PM_ROLL_HEADS;
    const uint32_t m0a = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
    const float4* g4 = reinterpret_cast<const float4*>(src) + lane;
    const float* g1 = src + 256 + (lane & 7);
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %3, off" ::"s"(m0a),
        "s"(m0a + 1024u), "v"(g4), "v"(g1)
        : "memory", "m0");
}

// serve_draw (pm_dev.h) for the step-keyed stream, split into four stages so that its integer and fp64
// work fills the gaps of the dependent MFMA chain: the same expressions in the same order, so the
// draw is bit-identical. Every lane draws, done or not (the select happens after the tick).
struct StagedServe {
    U4 r0, r1;
    ServeDraw d;
    __device__ __forceinline__ void stage(int g, const pm_env_params& p, uint32_t i, uint64_t ctr, uint64_t seed) {
        if (g == 0) r0 = philox(i, TAG_SERVE_STEP, (uint32_t)ctr, (uint32_t)(ctr >> 32), seed);
        if (g == 1) r1 = philox(i, TAG_SERVE_STEP | 0x100u, (uint32_t)ctr, (uint32_t)(ctr >> 32), seed);
        if (g == 2) {
            d.speed = p.speed_lo + (p.speed_hi - p.speed_lo) * u53(r0.x, r0.y);
            const bool first = u53(r0.z, r0.w) < 0.5;
            const double lo = first ? p.ang0_lo : p.ang1_lo, hi = first ? p.ang0_hi : p.ang1_hi;
            const double ang = lo + (hi - lo) * u53(r1.x, r1.y);
            d.rad = ang * (3.141592653589793 / 180.0);
            d.spin = p.spin_lo + (p.spin_hi - p.spin_lo) * u53(r1.z, r1.w);
        }
        if (g == 3) {
            double sn, cs;
            sincos_serve(d.rad, sn, cs);
            d.vx = d.speed * cs;
            d.vy = d.speed * sn;
        }
    }
};

// The collecting rollout's replay target (pm_roll_replay, device side).
struct RollPush {
    float* trans;
    float* prios;
    float* leaf;       // nullable: the PER leaves (prio^alpha) of pm_per_work_bytes(cap) work
    float* ep_reward;  // [n], carried
    int64_t pos, cap;  // ring slot of step 0's arena 0; steps * n <= cap, so no slot is written twice
    float prio, alpha;
};

// A block of 4 waves owns one tile of 32 arenas: wave 2 p + j computes layer-2 tile j of player p's
// forward (p = 0: A on modelA's image, p = 1: B on modelB's features + the step's heads), so each
// forward is 40 MFMAs deep instead of 72. Wave j = 0 runs the head chains over its tile's rows and
// hands the four partial sums per lane to wave j = 1 through LDS, which continues them over its rows:
// the same fmaf sequence as tile_heads, so every Q value and action is bit-identical to pm_qnet_act.
template <bool PUSH>
__device__ __forceinline__ void rollout_body(const pm_env_params& p, const pm_env_state& s, const float* __restrict__ wA,
                                             const float* __restrict__ wB, const float* __restrict__ ws, double eps,
                                             uint64_t seed_env, uint64_t counter0, int steps, float* __restrict__ obsA,
                                             float* __restrict__ obsB, long long* __restrict__ stats, int n,
                                             const RollPush& rp) {
    __shared__ __attribute__((aligned(16))) RollShared sm;
    const int lane = threadIdx.x & 63, col = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPRs, not VGPRs
    const int player = wv >> 1, half = wv & 1;
    const int i = blockIdx.x * 32 + col;
    const bool valid = i < n;
    stage_frags_lds(wA, sm.lw, blockIdx.x);  // block-wide: chunks spread over the waves
    stage_frags_lds(wB, sm.lwB, blockIdx.x + kLwChunks / 2);
    if (wv == 3) fetch_heads(ws, 0, sm.hf[0], lane);
    Arena a = load_arena(s, valid ? i : n - 1);
    const float* lw = player ? sm.lwB : sm.lw;
    int fin = 0, winB = 0, ptA = 0, ptB = 0, winE = 0, rsum = 0;  // per arena: |count| <= steps < 2^31
    float er = 0.f, leafv = 0.f;
    if constexpr (PUSH) {
        er = rp.ep_reward[valid ? i : n - 1];
        // memory.push's priority as a PER leaf (wave-uniform: kept in an SGPR)
        leafv = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(prio_pow(rp.prio, rp.alpha))));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // both images and step 0's heads in LDS
    for (int st = 0; st < steps; ++st) {
        const uint64_t ctr = counter0 + (uint64_t)st;
        if (wv == 3 && st + 1 < steps) fetch_heads_async(ws, st + 1, sm.hf[(st + 1) & 1], lane);  // lands during the MFMAs
        float oA[7], oB[7], o[7];
        observe(a, oA, oB);
#pragma unroll
        for (int k = 0; k < 7; ++k) o[k] = player ? oB[k] : oA[k];  // selects, not a pointer (no scratch)
        float xs[4];
        tile_inputs(o, lane >> 5, xs);
        f32x16 c2;
        StagedServe sv;
        hidden_half(lw, xs, lane, half, c2, [&](int g) { sv.stage(g, p, (uint32_t)i, ctr, seed_env); });
        const float* hf = player ? sm.hf[st & 1] : sm.lw + F_H;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        if (half == 0) {
            heads_half(hf, c2, lane, 0, acc);
            *reinterpret_cast<float4*>(&sm.part[st & 1][player][lane][0]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
        __syncthreads();  // the chains over layer-2 tile 0
        if (half == 1) {
            const float4 pa = *reinterpret_cast<const float4*>(&sm.part[st & 1][player][lane][0]);
            acc[0] = pa.x; acc[1] = pa.y; acc[2] = pa.z; acc[3] = pa.w;
            heads_half(hf, c2, lane, 1, acc);
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
            const float q[3] = {v + (a0 - mean), v + (a1 - mean), v + (a2 - mean)};
            int act = argmax3(q);
            if (player) {  // random.random() < eps ? randint(0, 2) : argmax (train_iterative.py:126-130)
                const U4 rr = philox64((uint32_t)i, TAG_ACT, ctr, seed_env);
                if (u53(rr.x, rr.y) < eps) act = (int)below(rr.z, 3u);
            }
            if (lane < 32) {
                sm.act[st & 1][player][col] = act;
            }
        }
        // wave 3: the next step's heads have landed (and, collecting, the previous step's replay stores)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // both players' actions
        const int aA = sm.act[st & 1][0][col], aB = sm.act[st & 1][1][col];
        float rA, rB;
        const int d = tick(p, a, aA, aB, rA, rB);
        ptA += rA > 0.f ? 1 : 0;
        ptB += rB > 0.f ? 1 : 0;
        if constexpr (PUSH) {
            er += rB;  // ep_reward += rB (:245)
            if (d) {
                winE += er > 0.f ? 1 : 0;
                rsum += (int)er;
            }
            if (wv == 3 && valid) {  // memory.push((oB, aB, rB, nB, done)): lanes < 32 s, lanes >= 32 s'
                float nA[7], nB[7];
                observe(a, nA, nB);  // the terminal observation, before the serve
                int64_t slot = rp.pos + (int64_t)st * n + i;
                if (slot >= rp.cap) slot -= rp.cap;
                float4* row = reinterpret_cast<float4*>(rp.trans + slot * PM_TRANS_F) + (lane >> 5) * 2;
                const bool hi = lane >= 32;
                st_f4<false>(row, hi ? make_float4(nB[0], nB[1], nB[2], nB[3]) : make_float4(oB[0], oB[1], oB[2], oB[3]));
                st_f4<false>(row + 1, hi ? make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8)))
                                         : make_float4(oB[4], oB[5], oB[6], rB));
                if (!hi) rp.prios[slot] = rp.prio;
                else if (rp.leaf) rp.leaf[slot] = leafv;
            }
            if (d) er = 0.f;
        }
        if (d) {  // env.reset() with K1's step-keyed production serve
            fin += 1;
            winB += rB > 0.f ? 1 : 0;
            serve_finish(sv.d);  // the rare |angle| >= 135 degree redo
            serve(a, sv.d.vx, sv.d.vy, sv.d.spin);
        }
    }
    if (wv == 0 && lane < 32 && valid) {  // wave 0 writes the arenas and their observations
        store_arena(s, i, a);
        float oA[7], oB[7];
        observe(a, oA, oB);
        store_row7(obsA + (size_t)i * 7, oA);
        store_row7(obsB + (size_t)i * 7, oB);
        if constexpr (PUSH) rp.ep_reward[i] = er;
    }
    if (!stats) return;  // block-uniform
    constexpr int NS = PUSH ? 6 : 4;
    const bool mine = wv == 0 && lane < 32 && valid;  // one lane per arena
    long long v[6] = {mine ? fin : 0, mine ? winB : 0, mine ? ptA : 0, mine ? ptB : 0, mine ? winE : 0,
                      mine ? rsum : 0};
#pragma unroll
    for (int k = 0; k < NS; ++k) v[k] = wave_sum(v[k]);
    long long mv = v[0];
#pragma unroll
    for (int k = 1; k < NS; ++k) mv = lane == k ? v[k] : mv;
    if (wv == 0 && lane < NS) atomicAdd(reinterpret_cast<unsigned long long*>(stats + lane), (unsigned long long)mv);
}

// rollout_body with the arena ticked once (round 5, the collecting launch's default): the four waves'
// forwards as above, but only wave 3 keeps the fp64 arena; it ticks, pushes, and publishes both
// players' next observations in LDS (a third barrier per step), and waves 0-1, idle during the tick,
// draw the next step's step-keyed serves and player B's epsilon branch into LDS (pure functions of
// arena, step and seed, as K9 does). rollout_body ticks every arena in all 8 half-waves and draws
// every serve in all four waves: at 65 536 arenas the launch is bound by that replicated VALU work.
// Bit-identical: the same tick, draws, forwards and head chains, in the same order.
struct Roll1Shared {
    RollShared r;
    float ob[2][32][8];       // [player][column]: the step's observations
    ServeDraw sdraw[2][32];   // [step & 1][column]
    int epsa[2][32];          // [step & 1][column]: -1 = argmax stands, else player B's random action
};
// PD: wave 0 draws the serve's two Philox blocks at once (lanes 0-31 the first tag, lanes 32-63 the
// second, for the same arenas) and hands the second to lanes 0-31 by v_permlane32_swap: one block's
// instruction stream instead of two in a row, the same bits.
template <bool PD = false>
__device__ __forceinline__ void roll1_draws(const pm_env_params& p, Roll1Shared& sm, int i, uint64_t ctr, int b,
                                            double eps, uint64_t seed, int wv, int lane) {
    const int col = lane & 31;
    if (PD && wv == 0) {
        const U4 r = philox((uint32_t)i, lane >= 32 ? (TAG_SERVE_STEP | 0x100u) : TAG_SERVE_STEP, (uint32_t)ctr,
                            (uint32_t)(ctr >> 32), seed);
        const auto sx = __builtin_amdgcn_permlane32_swap(r.x, r.x, false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(r.y, r.y, false, false);
        const auto sz = __builtin_amdgcn_permlane32_swap(r.z, r.z, false, false);
        const auto sw = __builtin_amdgcn_permlane32_swap(r.w, r.w, false, false);
        StagedServe sv;
        sv.r0 = U4{sx[0], sy[0], sz[0], sw[0]};  // lanes 0-31's block in both halves
        sv.r1 = U4{sx[1], sy[1], sz[1], sw[1]};  // lanes 32-63's
        sv.stage(2, p, (uint32_t)i, ctr, seed);
        sv.stage(3, p, (uint32_t)i, ctr, seed);
        if (lane < 32) sm.sdraw[b][col] = sv.d;
    } else if (!PD && wv == 0 && lane < 32) {
        StagedServe sv;
#pragma unroll
        for (int k = 0; k < 4; ++k) sv.stage(k, p, (uint32_t)i, ctr, seed);
        sm.sdraw[b][col] = sv.d;
    } else if (wv == 1 && lane < 32) {
        const U4 rr = philox64((uint32_t)i, TAG_ACT, ctr, seed);
        sm.epsa[b][col] = u53(rr.x, rr.y) < eps ? (int)below(rr.z, 3u) : -1;
    }
}
template <bool PUSH, bool PD = false>
__device__ __forceinline__ void rollout_body1(const pm_env_params& p, const pm_env_state& s, const float* __restrict__ wA,
                                              const float* __restrict__ wB, const float* __restrict__ ws, double eps,
                                              uint64_t seed_env, uint64_t counter0, int steps, float* __restrict__ obsA,
                                              float* __restrict__ obsB, long long* __restrict__ stats, int n,
                                              const RollPush& rp) {
    __shared__ __attribute__((aligned(16))) Roll1Shared sm;
    const int lane = threadIdx.x & 63, col = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int player = wv >> 1, half = wv & 1;
    const int i = blockIdx.x * 32 + col;
    const bool valid = i < n;
    stage_frags_lds(wA, sm.r.lw, blockIdx.x);
    stage_frags_lds(wB, sm.r.lwB, blockIdx.x + kLwChunks / 2);
    if (wv == 3) fetch_heads(ws, 0, sm.r.hf[0], lane);
    Arena a{};
    int fin = 0, winB = 0, ptA = 0, ptB = 0, winE = 0, rsum = 0;
    float er = 0.f, leafv = 0.f;
    if (wv == 3) {
        a = load_arena(s, valid ? i : n - 1);
        float oA[7], oB[7];
        observe(a, oA, oB);
        if (lane < 32)
#pragma unroll
            for (int k = 0; k < 7; ++k) { sm.ob[0][col][k] = oA[k]; sm.ob[1][col][k] = oB[k]; }
        if constexpr (PUSH) {
            er = rp.ep_reward[valid ? i : n - 1];
            leafv = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(prio_pow(rp.prio, rp.alpha))));
        }
    }
    roll1_draws<PD>(p, sm, i, counter0, 0, eps, seed_env, wv, lane);
    const float* lw = player ? sm.r.lwB : sm.r.lw;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // both images, step 0's heads, observations and draws in LDS
    for (int st = 0; st < steps; ++st) {
        const uint64_t ctr = counter0 + (uint64_t)st;
        if (wv == 3 && st + 1 < steps) fetch_heads_async(ws, st + 1, sm.r.hf[(st + 1) & 1], lane);
        float xs[4];
        tile_inputs(sm.ob[player][col], lane >> 5, xs);
        f32x16 c2;
        hidden_half(lw, xs, lane, half, c2, [](int) {});
        const float* hf = player ? sm.r.hf[st & 1] : sm.r.lw + F_H;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        if (half == 0) {
            heads_half(hf, c2, lane, 0, acc);
            *reinterpret_cast<float4*>(&sm.r.part[st & 1][player][lane][0]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
        __syncthreads();  // the chains over layer-2 tile 0
        if (half == 1) {
            const float4 pa = *reinterpret_cast<const float4*>(&sm.r.part[st & 1][player][lane][0]);
            acc[0] = pa.x; acc[1] = pa.y; acc[2] = pa.z; acc[3] = pa.w;
            heads_half(hf, c2, lane, 1, acc);
            float q[3];
            heads_finish(acc, hf, q);
            int act = argmax3(q);
            if (player) {  // random.random() < eps ? randint(0, 2) : argmax (train_iterative.py:126-130)
                const int ea = sm.epsa[st & 1][col];
                if (ea >= 0) act = ea;
            }
            if (lane < 32) sm.r.act[st & 1][player][col] = act;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 3: the next step's heads (and its stores)
        __syncthreads();  // both players' actions
        if (wv == 3) {
            const int aA = sm.r.act[st & 1][0][col], aB = sm.r.act[st & 1][1][col];
            float oB[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) oB[k] = sm.ob[1][col][k];  // the step's observation of B (push's s)
            float rA, rB;
            const int d = tick(p, a, aA, aB, rA, rB);
            ptA += rA > 0.f ? 1 : 0;
            ptB += rB > 0.f ? 1 : 0;
            if constexpr (PUSH) {
                er += rB;  // ep_reward += rB (:245)
                if (d) {
                    winE += er > 0.f ? 1 : 0;
                    rsum += (int)er;
                }
                if (valid) {  // memory.push((oB, aB, rB, nB, done)): lanes < 32 s, lanes >= 32 s'
                    float nA[7], nB[7];
                    observe(a, nA, nB);  // the terminal observation, before the serve
                    int64_t slot = rp.pos + (int64_t)st * n + i;
                    if (slot >= rp.cap) slot -= rp.cap;
                    float4* row = reinterpret_cast<float4*>(rp.trans + slot * PM_TRANS_F) + (lane >> 5) * 2;
                    const bool hi = lane >= 32;
                    st_f4<false>(row, hi ? make_float4(nB[0], nB[1], nB[2], nB[3]) : make_float4(oB[0], oB[1], oB[2], oB[3]));
                    st_f4<false>(row + 1, hi ? make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8)))
                                             : make_float4(oB[4], oB[5], oB[6], rB));
                    if (!hi) rp.prios[slot] = rp.prio;
                    else if (rp.leaf) rp.leaf[slot] = leafv;
                }
                if (d) er = 0.f;
            }
            if (d) {  // env.reset() with K1's step-keyed production serve
                fin += 1;
                winB += rB > 0.f ? 1 : 0;
                ServeDraw sd = sm.sdraw[st & 1][col];
                serve_finish(sd);  // the rare |angle| >= 135 degree redo
                serve(a, sd.vx, sd.vy, sd.spin);
            }
            float oA[7], nB2[7];
            observe(a, oA, nB2);
            if (lane < 32)
#pragma unroll
                for (int k = 0; k < 7; ++k) { sm.ob[0][col][k] = oA[k]; sm.ob[1][col][k] = nB2[k]; }
        } else if (st + 1 < steps) {
            roll1_draws<PD>(p, sm, i, ctr + 1, (st + 1) & 1, eps, seed_env, wv, lane);  // the next step's draws
        }
        __syncthreads();  // (C) the next observations
    }
    if (wv == 3 && lane < 32 && valid) {  // wave 3 writes the arenas and their observations
        store_arena(s, i, a);
        float oA[7], oB[7];
        observe(a, oA, oB);
        store_row7(obsA + (size_t)i * 7, oA);
        store_row7(obsB + (size_t)i * 7, oB);
        if constexpr (PUSH) rp.ep_reward[i] = er;
    }
    if (!stats) return;  // block-uniform
    constexpr int NS = PUSH ? 6 : 4;
    const bool mine = wv == 3 && lane < 32 && valid;  // one lane per arena
    long long v[6] = {mine ? fin : 0, mine ? winB : 0, mine ? ptA : 0, mine ? ptB : 0, mine ? winE : 0,
                      mine ? rsum : 0};
#pragma unroll
    for (int k = 0; k < NS; ++k) v[k] = wave_sum(v[k]);
    long long mv = v[0];
#pragma unroll
    for (int k = 1; k < NS; ++k) mv = lane == k ? v[k] : mv;
    if (wv == 3 && lane < NS) atomicAdd(reinterpret_cast<unsigned long long*>(stats + lane), (unsigned long long)mv);
}

// The inference launch keeps the compiler's own register budget (2 waves per SIMD with the MFMA
// accumulators in AGPRs: 3.14 us per vector step at 4 096 arenas). The collecting launch runs 65 536
// arenas, 16 blocks per CU queued: capped at 168 registers it fits 3 waves per SIMD, 19.9 against
// 21.0 us per vector step (same-box A/B, profiles/r3_roll_ab.txt); the same cap on the inference
// launch costs 15 % (3.61 us: no AGPR accumulators).
__global__ __launch_bounds__(kRollBlock) void k_rollout(const pm_env_params p, const pm_env_state s,
                                                        const float* __restrict__ wA, const float* __restrict__ wB,
                                                        const float* __restrict__ ws, double eps, uint64_t seed_env,
                                                        uint64_t counter0, int steps, float* __restrict__ obsA,
                                                        float* __restrict__ obsB, long long* __restrict__ stats,
                                                        int n) {
    rollout_body<false>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, RollPush{});
}

__global__ __launch_bounds__(kRollBlock) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_rollout_push(
    const pm_env_params p, const pm_env_state s, const float* __restrict__ wA, const float* __restrict__ wB,
    const float* __restrict__ ws, double eps, uint64_t seed_env, uint64_t counter0, int steps,
    float* __restrict__ obsA, float* __restrict__ obsB, long long* __restrict__ stats, int n, const RollPush rp) {
    rollout_body<true>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, rp);
}
// the one-tick bodies (rollout_body1)
template <bool PD>
__global__ __launch_bounds__(kRollBlock) void k_rollout1(const pm_env_params p, const pm_env_state s,
                                                         const float* __restrict__ wA, const float* __restrict__ wB,
                                                         const float* __restrict__ ws, double eps, uint64_t seed_env,
                                                         uint64_t counter0, int steps, float* __restrict__ obsA,
                                                         float* __restrict__ obsB, long long* __restrict__ stats,
                                                         int n) {
    rollout_body1<false, PD>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, RollPush{});
}
template <bool PD>
__global__ __launch_bounds__(kRollBlock) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_rollout_push1(
    const pm_env_params p, const pm_env_state s, const float* __restrict__ wA, const float* __restrict__ wB,
    const float* __restrict__ ws, double eps, uint64_t seed_env, uint64_t counter0, int steps,
    float* __restrict__ obsA, float* __restrict__ obsB, long long* __restrict__ stats, int n, const RollPush rp) {
    rollout_body1<true, PD>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, rp);
}

// ---------------------------------------------------------------------------------------------------
// K9 on 16-arena tiles (the inference launch): v_mfma_f32_16x16x4_f32 is, like the 32x32x2 form, a
// k-ordered fmaf chain bit for bit (tools/mfma_order_probe.hip: 0 of 102 400 outputs differ), so a
// QNet forward computed in 16-row / 16-column tiles over the SAME k sequences as tile_hidden /
// tile_heads gives the same bits. Half the tile width doubles the tiles: 4 096 arenas are 256 blocks,
// one per CU, instead of 128 blocks on half the chip, and each block's MFMA chain is half as long.
//
// Block = 8 waves, wave 4p + rt: player p, row tile rt (16 of the 64 units) of both layers.
//   layer 1 (K 8: bias + 7 inputs, 2 MFMAs) -> ReLU -> LDS in layer 2's k order (tile_hidden's pair
//   sequence (t, r) -> units 32t + rho(r) + {0, 4}) -> layer 2 (K 64, 16 MFMAs from the bias) -> ReLU
//   -> LDS in the head chains' order -> wave 0: both players' head chains (lanes 32p + 16h + col: half
//   h of column col, tile_heads' per-half fmaf chains and cross-half add), the actions, then the fp64
//   tick of the 16 arenas (kept in wave 0's registers, replicated over its four lane groups) and the
//   next observations into LDS. Three barriers per vector step (every wave computing all four layer-1
//   tiles into a slab of its own, to drop the first, ran 4.13 us per step against 2.69:
//   profiles/r4_roll16_ab.txt). Every LDS array a lane group reads as float4 runs keeps its 16 columns
//   side by side (conflict-free ds_read_b128; the first layout, [col][64], ran 3.67 us per step).
constexpr int kR16Block = 512;

#ifdef PM_DIAG
// k_rollout16's per-step phases (diagnostic build only): waves 0 (heads + tick) and 1 (a layer wave)
// of block 0 add the s_memtime cycles between phase points over every step of the launch.
static __device__ unsigned long long pm_diag_roll[2][8];
#define ROLL_T(k)                                                                 \
    do {                                                                          \
        if (diag) {                                                               \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime();         \
            dacc[(k)] += now_ - dprev;                                            \
            dprev = now_;                                                         \
        }                                                                         \
    } while (0)
#else
#define ROLL_T(k) \
    do {          \
    } while (0)
#endif

// layer 2's k order: sequence position of unit u, and the unit at position q
__device__ __forceinline__ int l2_pos(int u) {
    const int t = u >> 5, v = u & 31, b = (v >> 2) & 1, r = (v & 3) + 4 * (v >> 3);
    return 2 * (16 * t + r) + b;
}
__device__ __forceinline__ int l2_unit(int q) {
    const int i = q >> 1, b = q & 1;
    return 32 * (i >> 4) + rho(i & 15) + 4 * b;
}
// the head chains' order: unit u is element 16t + r of half (u >> 2) & 1's chain
__device__ __forceinline__ int head_pos(int u) {
    const int t = u >> 5, v = u & 31;
    return 16 * t + (v & 3) + 4 * (v >> 3);
}

typedef float f32x4v16 __attribute__((ext_vector_type(4)));

struct Roll16Shared {
    __attribute__((aligned(16))) float img2[2][4][4][64][4];  // [p][rt][s4][lane][e]: layer-2 A, instruction 4 s4 + e
    __attribute__((aligned(16))) float img1[2][4][64][2];     // [p][rt][lane][s]: layer-1 A
    __attribute__((aligned(16))) float b2v[2][4][4][4];       // [p][rt][g][r]: b2[16 rt + 4 g + r]
    __attribute__((aligned(16))) float hfA[264];              // modelA's heads (F_H / F_BH order)
    __attribute__((aligned(16))) float hfB[2][320];           // modelB's heads of the step, double-buffered
    // the two staging arrays are read as float4 runs whose 16 lanes per lane group sit side by side
    // (lane col at [..][col][4]): one ds_read_b128 pass per lane group, no bank conflict
    __attribute__((aligned(16))) float h1s[2][4][4][16][4];   // [p][g][s >> 2][col][s & 3]: layer-2 B of instruction s
    __attribute__((aligned(16))) float c2s[2][2][8][16][4];   // [p][h][q >> 2][col][q & 3]: ReLU(layer 2), chain order
    float ob[2][16][8];                                       // [p][col]: the observations of the step
    // the draws of step st (buffer st & 1), made by wave 1 during step st - 1's heads + tick (an idle
    // window of that wave): the step-keyed serve (used if the arena's episode ends) and player B's
    // epsilon branch (-1: the argmax stands, else the random action)
    ServeDraw sdraw[2][16];
    int epsa[2][16];
    // MH (heads on the matrix cores): the head weights by output, opw[set][h][j][q] = weight of output
    // j (V, A0, A1, A2) at chain position q of half h; set 0 = modelA (once), 1 + b = modelB of step
    // buffer b (rearranged from hfB by wave 7 while it is idle)
    __attribute__((aligned(16))) float opw[3][2][4][32];
};

// Head weights (F_H order, 260 floats) -> opw[set]: output-major per half (one wave).
__device__ __forceinline__ void roll16_opw(Roll16Shared& sm, int set, const float* hf) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int idx = it * 64 + lane, h = idx >> 7, j = (idx >> 5) & 3, q = idx & 31;
        sm.opw[set][h][j][q] = hf[(h * 32 + q) * 4 + j];
    }
}

// Step ctr's per-arena draws into buffer b (wave 1; lane group 0: the step-keyed serve, the same
// StagedServe stages as the stepped path; lane group 1: player B's epsilon branch, philox64 keyed
// as K1's act draw). Pure functions of (arena, step, seed): drawn a step ahead, bit-identical.
__device__ __forceinline__ void roll16_draws(const pm_env_params& p, Roll16Shared& sm, int i, uint64_t ctr, int b,
                                             double eps, uint64_t seed, int g) {
    const int col = threadIdx.x & 15;
    if (g == 0) {
        StagedServe sv;
#pragma unroll
        for (int k = 0; k < 4; ++k) sv.stage(k, p, (uint32_t)i, ctr, seed);
        sm.sdraw[b][col] = sv.d;
    } else if (g == 1) {
        const U4 rr = philox64((uint32_t)i, TAG_ACT, ctr, seed);
        sm.epsa[b][col] = u53(rr.x, rr.y) < eps ? (int)below(rr.z, 3u) : -1;
    }
}

// PL: the heads' cross-lane moves on the gfx950 row / half swaps instead of ds_bpermute round trips.
// xor16_sum: v + (v of lane ^ 16) as v_permlane16_swap (rows 0 <-> 1 and 2 <-> 3 exchanged between two
// copies), so each lane adds the same pair: the same bits as v + __shfl_xor(v, 16) (an IEEE add
// commutes). halves_bcast: lanes 0-31's value in both halves (lo) and lanes 32-63's (hi), one
// v_permlane32_swap for both.
__device__ __forceinline__ float xor16_sum(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ void halves_bcast(int v, int& lo, int& hi) {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    lo = (int)r[0];
    hi = (int)r[1];
}

// PL: the step's draws split so that neither outlasts wave 0's heads + tick (the single drawing wave,
// three Philox blocks in a row behind a lane-group branch, was the last to reach barrier C). Wave 1:
// the serve's two Philox blocks at once, lane group 0 on the first tag and group 1 on the second,
// group 1's block handed to group 0 by a row swap, then the serve's fp64 stages; wave 2: player B's
// epsilon branch. Same functions of the same counters, so the same bits.
__device__ __forceinline__ void roll16_serve(const pm_env_params& p, Roll16Shared& sm, int i, uint64_t ctr, int b,
                                             uint64_t seed, int g) {
    const U4 r = philox((uint32_t)i, g == 1 ? (TAG_SERVE_STEP | 0x100u) : TAG_SERVE_STEP, (uint32_t)ctr,
                        (uint32_t)(ctr >> 32), seed);
    const auto sx = __builtin_amdgcn_permlane16_swap(r.x, r.x, false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(r.y, r.y, false, false);
    const auto sz = __builtin_amdgcn_permlane16_swap(r.z, r.z, false, false);
    const auto sw = __builtin_amdgcn_permlane16_swap(r.w, r.w, false, false);
    StagedServe sv;
    sv.r0 = r;
    sv.r1 = U4{sx[1], sy[1], sz[1], sw[1]};  // rows 1 and 3's block in rows 0 and 2
    sv.stage(2, p, (uint32_t)i, ctr, seed);
    sv.stage(3, p, (uint32_t)i, ctr, seed);
    if (g == 0) sm.sdraw[b][threadIdx.x & 15] = sv.d;
}
__device__ __forceinline__ void roll16_eps(Roll16Shared& sm, int i, uint64_t ctr, int b, double eps, uint64_t seed,
                                           int g) {
    if (g == 0) {
        const U4 rr = philox64((uint32_t)i, TAG_ACT, ctr, seed);
        sm.epsa[b][threadIdx.x & 15] = u53(rr.x, rr.y) < eps ? (int)below(rr.z, 3u) : -1;
    }
}

template <bool PUSH, bool MH, bool W2R = false, bool PL = false>
__device__ __forceinline__ void rollout16_body(const pm_env_params& p, const pm_env_state& s, const float* __restrict__ wA,
                                               const float* __restrict__ wB, const float* __restrict__ ws, double eps,
                                               uint64_t seed_env, uint64_t counter0, int steps, float* __restrict__ obsA,
                                               float* __restrict__ obsB, long long* __restrict__ stats, int n,
                                               const RollPush& rp) {
    __shared__ Roll16Shared sm;
    const int t = threadIdx.x, lane = t & 63, col = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int player = wv >> 2, rt = wv & 3;
    const int i = blockIdx.x * 16 + col;
    const bool valid = i < n;
    // ---- operand images from the plain effective weights (once per launch; global reads hit L2)
    for (int k = t; k < 2 * 4 * 4 * 64 * 4; k += kR16Block) {
        const int pp = k >> 12, r2 = (k >> 10) & 3, s4 = (k >> 8) & 3, ln = (k >> 2) & 63, e = k & 3;
        const float* w = pp ? wB : wA;
        (&sm.img2[0][0][0][0][0])[k] = w[W2 + (16 * r2 + (ln & 15)) * 64 + l2_unit(4 * (4 * s4 + e) + (ln >> 4))];
    }
    for (int k = t; k < 2 * 4 * 64 * 2; k += kR16Block) {
        const int pp = k >> 9, r2 = (k >> 7) & 3, ln = (k >> 1) & 63, sx = k & 1;
        const float* w = pp ? wB : wA;
        const int row = 16 * r2 + (ln & 15), kk = 4 * sx + (ln >> 4);  // input k' = 0 is the constant 1 (b1)
        (&sm.img1[0][0][0][0])[k] = kk == 0 ? w[B1 + row] : w[W1 + row * 7 + kk - 1];
    }
    if (t < 128) {
        const int pp = t >> 6, r2 = (t >> 4) & 3, gg = (t >> 2) & 3, r = t & 3;
        (&sm.b2v[0][0][0][0])[t] = (pp ? wB : wA)[B2 + 16 * r2 + 4 * gg + r];
    }
    if (t < 260) sm.hfA[t] = t < 256 ? wA[PLAIN + F_H + t] : wA[PLAIN + F_BH + t - 256];
    if (wv == 7) fetch_heads(ws, 0, sm.hfB[0], lane);
    if (PL && wv == 1) roll16_serve(p, sm, i, counter0, 0, seed_env, g);
    if (PL && wv == 2) roll16_eps(sm, i, counter0, 0, eps, seed_env, g);
    if (!PL && wv == 1) roll16_draws(p, sm, i, counter0, 0, eps, seed_env, g);
    // ---- wave 0 keeps the 16 arenas (every lane group a copy) and ticks them
    Arena a{};
    int fin = 0, winB = 0, ptA = 0, ptB = 0, winE = 0, rsum = 0;
    float er = 0.f, leafv = 0.f;
    if (wv == 0) {
        a = load_arena(s, valid ? i : n - 1);
        float oA[7], oB[7];
        observe(a, oA, oB);
        if (g < 2)
#pragma unroll
            for (int k = 0; k < 7; ++k) sm.ob[g][col][k] = g ? oB[k] : oA[k];
        if constexpr (PUSH) {
            er = rp.ep_reward[valid ? i : n - 1];
            leafv = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(prio_pow(rp.prio, rp.alpha))));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MH && wv == 7) roll16_opw(sm, 1, sm.hfB[0]);  // its own fetch of hfB[0] has landed (same wave)
    if (MH && wv == 6) roll16_opw(sm, 0, wA + PLAIN + F_H);  // modelA's heads straight from global
    __syncthreads();
    const float4* im2 = reinterpret_cast<const float4*>(sm.img2[player][rt][0][lane]);
    // W2R: the wave's layer-1 and layer-2 A operands and layer-2 bias, constant over the launch, held in
    // registers (2 + 16 + 4) instead of read from LDS every step
    float4 w2r[4], b2r{};
    const float2 w1r = W2R ? *reinterpret_cast<const float2*>(sm.img1[player][rt][lane]) : float2{};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) w2r[s4] = W2R ? im2[s4 * 64] : float4{};
    if (W2R) b2r = *reinterpret_cast<const float4*>(sm.b2v[player][rt][g]);
#ifdef PM_DIAG
    const bool diag = blockIdx.x == 0 && wv < 2;
    unsigned long long dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dprev = __builtin_amdgcn_s_memtime();
#endif
    for (int st = 0; st < steps; ++st) {
        const uint64_t ctr = counter0 + (uint64_t)st;
        if (wv == 7 && st + 1 < steps) fetch_heads_async(ws, st + 1, sm.hfB[(st + 1) & 1], lane);  // lands during the step
        float hw4[32];  // MH, wave 0: lane 32 pp + 16 h + 4 cg + j's A operands, the weights of output j
        // of player pp's half h. PL: read at the step's start (wave 7 wrote this step's set before the
        // last barrier C), so the reads retire under the layers instead of holding wave 0 at barrier B
        auto read_hw4 = [&]() {
            const float* src = sm.opw[(lane >> 5) ? 1 + (st & 1) : 0][(lane >> 4) & 1][lane & 3];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 w = *reinterpret_cast<const float4*>(src + 4 * k);
                hw4[4 * k] = w.x; hw4[4 * k + 1] = w.y; hw4[4 * k + 2] = w.z; hw4[4 * k + 3] = w.w;
            }
        };
        if (PL && MH && wv == 0) read_hw4();
        // layer 1, the wave's row tile (K 8: bias + 7 inputs, input k' = 4 s + g) -> ReLU -> LDS
        {
            const float* o = sm.ob[player][col];
            // PL: both inputs read together (one LDS wait, not a masked read, a wait, a read, a wait)
            const float o0 = PL ? o[g == 0 ? 0 : g - 1] : 0.f;
            const float x0 = PL ? (g == 0 ? 1.0f : o0) : (g == 0 ? 1.0f : o[g - 1]), x1 = o[3 + g];
            const float2 w1 = W2R ? w1r : *reinterpret_cast<const float2*>(sm.img1[player][rt][lane]);
            const f32x4v16 zero = {0.f, 0.f, 0.f, 0.f};
            f32x4v16 c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.x, x0, zero, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1.y, x1, c1, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // unit 16 rt + 4 g + r -> its slot in layer 2's k order
                const int q = l2_pos(16 * rt + 4 * g + r), sq = q >> 2;
                sm.h1s[player][q & 3][sq >> 2][col][sq & 3] = relu(c1[r]);
            }
        }
        ROLL_T(0);        // step start (barrier C) -> layer 1 issued
        __syncthreads();  // (A) the player's layer 1
        ROLL_T(1);
        float bs[16];
        {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 v = *reinterpret_cast<const float4*>(sm.h1s[player][g][k][col]);
                bs[4 * k] = v.x; bs[4 * k + 1] = v.y; bs[4 * k + 2] = v.z; bs[4 * k + 3] = v.w;
            }
        }
        const float4 bi = W2R ? b2r : *reinterpret_cast<const float4*>(sm.b2v[player][rt][g]);
        f32x4v16 c2 = {bi.x, bi.y, bi.z, bi.w};

#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const float4 w = W2R ? w2r[s4] : im2[s4 * 64];
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, bs[4 * s4 + 0], c2, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, bs[4 * s4 + 1], c2, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, bs[4 * s4 + 2], c2, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, bs[4 * s4 + 3], c2, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int u = 16 * rt + 4 * g + r, q = head_pos(u);
            sm.c2s[player][(u >> 2) & 1][q >> 2][col][q & 3] = relu(c2[r]);
        }
        if (wv == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next step's heads landed
        if (!PL && MH && wv == 0) read_hw4();  // before barrier B: the latency hides under it
        ROLL_T(2);        // layer 2 + staging
        __syncthreads();  // (B) both players' layer 2
        ROLL_T(3);
        int aA = 0, aB = 0;
        ServeDraw sd_pre{};
        if (MH && wv == 0) {
            // heads on the matrix cores: one chain of 32 v_mfma_f32_4x4x1_16b_f32 (a k-ordered fmaf
            // chain bit for bit, tools/mfma4_probe.hip) covers every (player, half, column): block b =
            // lanes 4b..4b+3 = (pp, h, column group cg) multiplies the 4 outputs' weights (A: lane
            // 4b + j supplies output j) by 4 columns' ReLU(layer 2) (B: lane 4b + j supplies column
            // 4 cg + j), so lane 32 pp + 16 h + col ends with the four partial sums of tile_heads' half
            // chains for its column, in the VALU path's lanes and the same fmaf order
            const int hp = lane >> 5, hh = (lane >> 4) & 1;
            const float* hf = hp ? sm.hfB[st & 1] : sm.hfA;
            float xb[32];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 x = *reinterpret_cast<const float4*>(sm.c2s[hp][hh][k][col]);
                xb[4 * k] = x.x; xb[4 * k + 1] = x.y; xb[4 * k + 2] = x.z; xb[4 * k + 3] = x.w;
            }
            // PL: player B's epsilon branch read before the chain, not behind the argmax, and the step's
            // serve draw (applied to the arenas whose episode ends) before the tick, not inside its branch
            const int ea_pre = PL ? sm.epsa[st & 1][col] : 0;
            if constexpr (PL) sd_pre = sm.sdraw[st & 1][col];
            f32x4v16 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 32; ++q) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(hw4[q], xb[q], acc, 0, 0, 0);
            if constexpr (PL) {  // every operand read issued ahead of the chain (one wait per read, in order)
                __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);  // DS reads
                __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);  // the MFMAs
            }
            float v = acc[0], a0 = acc[1], a1 = acc[2], a2 = acc[3];
            if constexpr (PL) {  // + the other half (both lanes get the same bits)
                v = xor16_sum(v);
                a0 = xor16_sum(a0);
                a1 = xor16_sum(a1);
                a2 = xor16_sum(a2);
            } else {
                v += __shfl_xor(v, 16);
                a0 += __shfl_xor(a0, 16);
                a1 += __shfl_xor(a1, 16);
                a2 += __shfl_xor(a2, 16);
            }
            v += hf[256];
            a0 += hf[257];
            a1 += hf[258];
            a2 += hf[259];
            const float mean = ((a0 + a1) + a2) / 3.0f;  // A.mean(dim=1)
            const float qv[3] = {v + (a0 - mean), v + (a1 - mean), v + (a2 - mean)};
            int act = argmax3(qv);
            if (hp) {  // random.random() < eps ? randint(0, 2) : argmax (train_iterative.py:126-130)
                const int ea = PL ? ea_pre : sm.epsa[st & 1][col];
                if (ea >= 0) act = ea;
            }
            if constexpr (PL) {
                halves_bcast(act, aA, aB);  // rows 0 and 1 (2 and 3) hold the same actions
            } else {
                aA = __shfl(act, col);
                aB = __shfl(act, 32 + col);
            }
        }
        if (wv == 0) {
          if constexpr (!MH) {
            // heads: lane 32 hp + 16 hh + col runs half hh's four chains of player hp, column col
            const int hp = lane >> 5, hh = (lane >> 4) & 1;
            const float* hf = hp ? sm.hfB[st & 1] : sm.hfA;
            const float4* hw = reinterpret_cast<const float4*>(hf) + hh * 32;
            float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 x = *reinterpret_cast<const float4*>(sm.c2s[hp][hh][k][col]);
                const float xx[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float4 w = hw[4 * k + e];
                    v = fmaf(w.x, xx[e], v);
                    a0 = fmaf(w.y, xx[e], a0);
                    a1 = fmaf(w.z, xx[e], a1);
                    a2 = fmaf(w.w, xx[e], a2);
                }
            }
            v += __shfl_xor(v, 16);  // + the other half (both lanes get the same bits)
            a0 += __shfl_xor(a0, 16);
            a1 += __shfl_xor(a1, 16);
            a2 += __shfl_xor(a2, 16);
            v += hf[256];
            a0 += hf[257];
            a1 += hf[258];
            a2 += hf[259];
            const float mean = ((a0 + a1) + a2) / 3.0f;  // A.mean(dim=1)
            const float q[3] = {v + (a0 - mean), v + (a1 - mean), v + (a2 - mean)};
            int act = argmax3(q);
            if (hp) {  // random.random() < eps ? randint(0, 2) : argmax (train_iterative.py:126-130)
                const int ea = sm.epsa[st & 1][col];
                if (ea >= 0) act = ea;
            }
            aA = __shfl(act, col);
            aB = __shfl(act, 32 + col);
          }
            ROLL_T(4);    // heads + actions
            float sB[7];  // the step's observation of B (memory.push's s)
#pragma unroll
            for (int k = 0; k < 7; ++k) sB[k] = sm.ob[1][col][k];
            float rA, rB;
            const int d = tick(p, a, aA, aB, rA, rB);
            ptA += rA > 0.f ? 1 : 0;
            ptB += rB > 0.f ? 1 : 0;
            if constexpr (PUSH) {
                er += rB;  // ep_reward += rB (:245)
                if (d) {
                    winE += er > 0.f ? 1 : 0;
                    rsum += (int)er;
                }
                if (valid) {  // memory.push((oB, aB, rB, nB, done)): lane group g stores the row's float4 g
                    float nA[7], nB[7];
                    observe(a, nA, nB);  // the terminal observation, before the serve
                    int64_t slot = rp.pos + (int64_t)st * n + i;
                    if (slot >= rp.cap) slot -= rp.cap;
                    const float4 v = g == 0 ? make_float4(sB[0], sB[1], sB[2], sB[3])
                                   : g == 1 ? make_float4(sB[4], sB[5], sB[6], rB)
                                   : g == 2 ? make_float4(nB[0], nB[1], nB[2], nB[3])
                                            : make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8)));
                    st_f4<false>(reinterpret_cast<float4*>(rp.trans + slot * PM_TRANS_F) + g, v);
                    if (g == 0) rp.prios[slot] = rp.prio;
                    else if (g == 1 && rp.leaf) rp.leaf[slot] = leafv;
                }
                if (d) er = 0.f;
            }
            if (d) {  // env.reset() with K1's step-keyed production serve
                fin += 1;
                winB += rB > 0.f ? 1 : 0;
                ServeDraw sd = (PL && MH) ? sd_pre : sm.sdraw[st & 1][col];
                serve_finish(sd);
                serve(a, sd.vx, sd.vy, sd.spin);
            }
            float oA[7], oB[7];
            observe(a, oA, oB);
            if (g < 2)
#pragma unroll
                for (int k = 0; k < 7; ++k) sm.ob[g][col][k] = g ? oB[k] : oA[k];
            ROLL_T(5);    // tick (+ push) + next observations
        } else if (wv == 1 && st + 1 < steps) {  // the next step's draws
            if constexpr (PL) roll16_serve(p, sm, i, ctr + 1, (st + 1) & 1, seed_env, g);
            else roll16_draws(p, sm, i, ctr + 1, (st + 1) & 1, eps, seed_env, g);
        } else if (PL && wv == 2 && st + 1 < steps) {
            roll16_eps(sm, i, ctr + 1, (st + 1) & 1, eps, seed_env, g);
        } else if (MH && wv == 7 && st + 1 < steps) {
            roll16_opw(sm, 1 + ((st + 1) & 1), sm.hfB[(st + 1) & 1]);  // the next step's heads (landed before barrier B)
        }
        __syncthreads();  // (C) the next observations
        ROLL_T(6);
    }
#ifdef PM_DIAG
    if (diag && lane == 0)
#pragma unroll
        for (int k = 0; k < 8; ++k) pm_diag_roll[wv][k] = k < 7 ? dacc[k] : (unsigned long long)steps;
#endif
    if (wv == 0 && g == 0 && valid) {
        store_arena(s, i, a);
        float oA[7], oB[7];
        observe(a, oA, oB);
        store_row7(obsA + (size_t)i * 7, oA);
        store_row7(obsB + (size_t)i * 7, oB);
        if constexpr (PUSH) rp.ep_reward[i] = er;
    }
    if (!stats || wv != 0) return;
    constexpr int NS = PUSH ? 6 : 4;
    const bool mine = g == 0 && valid;  // one lane per arena
    long long v[6] = {mine ? fin : 0, mine ? winB : 0, mine ? ptA : 0, mine ? ptB : 0, mine ? winE : 0,
                      mine ? rsum : 0};
#pragma unroll
    for (int k = 0; k < NS; ++k) v[k] = wave_sum(v[k]);
    long long mv = v[0];
#pragma unroll
    for (int k = 1; k < NS; ++k) mv = lane == k ? v[k] : mv;
    if (lane < NS) atomicAdd(reinterpret_cast<unsigned long long*>(stats + lane), (unsigned long long)mv);
}

template <bool MH, bool W2R, bool PL>
__global__ __launch_bounds__(kR16Block) void k_rollout16(const pm_env_params p, const pm_env_state s,
                                                         const float* __restrict__ wA, const float* __restrict__ wB,
                                                         const float* __restrict__ ws, double eps, uint64_t seed_env,
                                                         uint64_t counter0, int steps, float* __restrict__ obsA,
                                                         float* __restrict__ obsB, long long* __restrict__ stats,
                                                         int n) {
    rollout16_body<false, MH, W2R, PL>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, RollPush{});
}
// the collecting launch runs 65 536 arenas (4 096 blocks): two blocks per CU (4 waves per SIMD) need
// <= 128 registers
template <bool MH>
__global__ __launch_bounds__(kR16Block) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_rollout16_push(
    const pm_env_params p, const pm_env_state s, const float* __restrict__ wA, const float* __restrict__ wB,
    const float* __restrict__ ws, double eps, uint64_t seed_env, uint64_t counter0, int steps,
    float* __restrict__ obsA, float* __restrict__ obsB, long long* __restrict__ stats, int n, const RollPush rp) {
    rollout16_body<true, MH>(p, s, wA, wB, ws, eps, seed_env, counter0, steps, obsA, obsB, stats, n, rp);
}

// 16-arena tiles: PONGMI_ROLL16 bit 0 = the inference launch, bit 1 = the collecting launch (A/B),
// bit 2 = the round-4 VALU head chains instead of the MFMA ones in the inference launch (A/B), bit 3 =
// the 32-arena-tile kernels with the replicated tick (rollout_body) instead of rollout_body1, bit 4 = the
// inference launch's layer-2 weights read from LDS every step (round 5) instead of held in registers, bit 5 =
// the MFMA heads' cross-lane moves through ds_bpermute (round 5) instead of the permlane swaps, bit 6 = the
// one-tick 32-arena bodies' serve draw as two Philox blocks in a row (round 5); default 1. Read at every
// launch (one getenv), so a test can cover every kernel in one process.
int roll16() {
    const char* e = getenv("PONGMI_ROLL16");
    return e && *e ? atoi(e) : 1;
}

}  // namespace

static int rollout_launch(const pm_env_params* p, const pm_env_state* s, const float* wA, const float* wB,
                          const float* paramsB, float epsilon, uint64_t seed_env, uint64_t seed_net, uint64_t counter0,
                          int32_t steps, float* heads_ws, float* obsA, float* obsB, const RollPush* rp, void* per_work,
                          int64_t* stats, int32_t n, void* stream) {
    const char* name = rp ? "pm_rollout_push" : "pm_rollout";
    PM_REQUIRE(n >= 0 && steps >= 0, PM_E_SIZE, "%s: n=%d steps=%d", name, n, steps);
    if (n == 0 || steps == 0) return PM_OK;
    PM_REQUIRE(p && s && s->x && s->y && s->vx && s->vy && s->spin && s->top && s->bot && s->scoreA && s->scoreB &&
                   s->bounces && wA && wB && paramsB && heads_ws && obsA && obsB,
               PM_E_ARG, "%s: null buffer", name);
    PM_REQUIRE((((uintptr_t)wA) | ((uintptr_t)wB) | ((uintptr_t)heads_ws)) % 16 == 0, PM_E_ARG,
               "%s: wA, wB and heads_ws must be 16-byte aligned", name);
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "%s: speed_scale_every must be > 0", name);
    hipStream_t st = pm_stream(stream);
    hipLaunchKernelGGL(k_rollout_heads, dim3(steps), dim3(kHeadsBlock), 0, st, paramsB, seed_net, counter0, heads_ws);
    PM_LAUNCHED("k_rollout_heads");
    const dim3 grid(pm_blocks(n, 32)), block(kRollBlock);
    const int r16 = roll16();
    if (rp && (r16 & 2)) {
        // VALU heads here: the MFMA heads' operands do not fit this kernel's 128-register cap (2 blocks per CU)
        pm_launch(PM_TIMER_ROLLOUT, k_rollout16_push<false>, dim3(pm_blocks(n, 16)),
                  dim3(kR16Block), st, *p, *s, wA, wB, (const float*)heads_ws, (double)epsilon, seed_env, counter0,
                  (int)steps, obsA, obsB, reinterpret_cast<long long*>(stats), n, *rp);
        PM_LAUNCHED("k_rollout16_push");
        if (per_work) return per_launch_nodes(per_work, rp->cap, st);
        return PM_OK;
    }
    if (rp) {
        pm_launch(PM_TIMER_ROLLOUT, (r16 & 8) ? k_rollout_push : ((r16 & 64) ? k_rollout_push1<false> : k_rollout_push1<true>),
                  grid, block, st, *p, *s, wA, wB,
                  (const float*)heads_ws, (double)epsilon, seed_env, counter0, (int)steps, obsA, obsB,
                  reinterpret_cast<long long*>(stats), n, *rp);
        PM_LAUNCHED("k_rollout_push");
        if (per_work) return per_launch_nodes(per_work, rp->cap, st);
        return PM_OK;
    }
    if (r16 & 1) {
        // bit 2: VALU heads (keeps the shuffles); bit 4: weights from LDS; bit 5: the heads' ds_bpermute moves
        const bool pl = !(r16 & 32);
        const auto kern = (r16 & 4) ? ((r16 & 16) ? k_rollout16<false, false, false> : k_rollout16<false, true, false>)
                        : (r16 & 16) ? (pl ? k_rollout16<true, false, true> : k_rollout16<true, false, false>)
                                     : (pl ? k_rollout16<true, true, true> : k_rollout16<true, true, false>);
        pm_launch(PM_TIMER_ROLLOUT, kern, dim3(pm_blocks(n, 16)),
                  dim3(kR16Block), st, *p, *s, wA, wB, (const float*)heads_ws, (double)epsilon, seed_env, counter0,
                  (int)steps, obsA, obsB, reinterpret_cast<long long*>(stats), n);
        PM_LAUNCHED("k_rollout16");
        return PM_OK;
    }
    pm_launch(PM_TIMER_ROLLOUT, (r16 & 8) ? k_rollout : ((r16 & 64) ? k_rollout1<false> : k_rollout1<true>), grid, block, st,
              *p, *s, wA, wB,
              (const float*)heads_ws, (double)epsilon, seed_env, counter0, (int)steps, obsA, obsB,
              reinterpret_cast<long long*>(stats), n);
    PM_LAUNCHED("k_rollout");
    return PM_OK;
}

#ifdef PM_DIAG
extern "C" int pm_diag_read_roll(uint64_t* out) {  // [2][8]: waves 0 / 1 of block 0, cycles per phase, [7] steps
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_roll), sizeof(pm_diag_roll));
}
#endif

extern "C" int pm_rollout(const pm_env_params* p, const pm_env_state* s, const float* wA, const float* wB,
                          const float* paramsB, float epsilon, uint64_t seed_env, uint64_t seed_net, uint64_t counter0,
                          int32_t steps, float* heads_ws, float* obsA, float* obsB, int64_t* stats, int32_t n,
                          void* stream) {
    return rollout_launch(p, s, wA, wB, paramsB, epsilon, seed_env, seed_net, counter0, steps, heads_ws, obsA, obsB,
                          nullptr, nullptr, stats, n, stream);
}

extern "C" int pm_rollout_push(const pm_env_params* p, const pm_env_state* s, const float* wA, const float* wB,
                               const float* paramsB, float epsilon, uint64_t seed_env, uint64_t seed_net,
                               uint64_t counter0, int32_t steps, float* heads_ws, float* obsA, float* obsB,
                               const pm_roll_replay* rp, int64_t* stats, int32_t n, void* stream) {
    PM_REQUIRE(rp && rp->trans && rp->prios && rp->ep_reward, PM_E_ARG, "pm_rollout_push: null replay buffer");
    PM_REQUIRE(rp->cap > 0 && rp->pos >= 0 && rp->pos < rp->cap, PM_E_SIZE, "pm_rollout_push: pos=%lld cap=%lld",
               (long long)rp->pos, (long long)rp->cap);
    PM_REQUIRE(n >= 0 && steps >= 0 && (int64_t)steps * n <= rp->cap, PM_E_SIZE,
               "pm_rollout_push: steps * n = %lld exceeds cap %lld (a slot would be written twice in one launch)",
               (long long)steps * n, (long long)rp->cap);
    PM_REQUIRE(((uintptr_t)rp->trans) % 16 == 0 && ((uintptr_t)rp->per_work) % 16 == 0, PM_E_ARG,
               "pm_rollout_push: trans and per_work must be 16-byte aligned");
    const RollPush d{rp->trans, rp->prios, rp->per_work ? per_tree(rp->per_work, rp->cap).leaf : nullptr,
                     rp->ep_reward, rp->pos, rp->cap, rp->prio, rp->alpha};
    return rollout_launch(p, s, wA, wB, paramsB, epsilon, seed_env, seed_net, counter0, steps, heads_ws, obsA, obsB,
                          &d, rp->per_work, stats, n, stream);
}
