// The batched self-play learner: one vector step of scripts/train_iterative.py:239-245 for n arenas,
// three kernels, nothing returns to the host:
//
//   k_act_sp (MFMA tiles)  both players' QNet forward + eps-greedy / argmax (pm_mfma.h); its first
//                          ceil(batch/64) blocks draw this step's PER sample (64 samples per block) off
//                          the sum tree, which already accounts for the push k_env is about to make
//   k_env    (n lanes)     env tick + replay push + episode bookkeeping + serves
//   k_learn  (1 WG, 1024)  Q_B(s), Q_B(s'), Q_T(s') on the matrix cores into LDS, double-DQN targets,
//                          IS-weighted MSE, priority scatter, sum-tree refresh (scattered sub-blocks +
//                          next push range), head grads [+ Adam / target sync / epsilon decay /
//                          counters / next weights when unsharded]
//   ----------------------- (sharded: RCCL all-reduce of sp.grad, then k_adam)
//
// Every loop counter lives in the device control block (pm_ctrl), so a whole vector step can be
// replayed from a captured graph.
#include <algorithm>
#include <cmath>

#include "pm_host.h"
#include "pm_mfma.h"
#include "pm_per.h"

using namespace pm;

#ifdef PM_DIAG
// k_env phase timeline (diagnostic build only): wave 0 of each env block. A stamp records when the
// wave's instruction stream reaches it (no drain: stores still in flight are not waited for);
// PM_ENV_STAMP_DRAIN first waits for every outstanding memory operation of the wave.
static __device__ unsigned long long pm_diag_env[8][1024];
// k_learn's side blocks: [0] begin, [1] after the act blocks' sleep, [2] end, [3] role | rows << 16
static __device__ unsigned long long pm_diag_side[4][1024];
#define PM_SIDE(k, sb, v)                                                        \
    do {                                                                         \
        if (threadIdx.x == 0 && (sb) < 1024) pm_diag_side[(k)][(sb)] = (v);      \
    } while (0)
#define PM_ENV_STAMP(k, blk)                                                                   \
    do {                                                                                       \
        asm volatile("" ::: "memory");                                                         \
        if (threadIdx.x == 0 && (blk) < 1024) pm_diag_env[(k)][(blk)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define PM_ENV_STAMP_DRAIN(k, blk)                                                             \
    do {                                                                                       \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                            \
        if (threadIdx.x == 0 && (blk) < 1024) pm_diag_env[(k)][(blk)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PM_SIDE(k, sb, v) \
    do {                  \
    } while (0)
#define PM_ENV_STAMP(k, blk) \
    do {                     \
    } while (0)
#define PM_ENV_STAMP_DRAIN(k, blk) \
    do {                           \
    } while (0)
#endif

namespace {

constexpr int kBlock = 256;
static_assert(kBlock == kRowBlock, "row staging assumes kRowBlock-thread blocks");
constexpr int kLearn = 1024;              // k_learn / k_adam / k_prepare block
constexpr int kGradN = PM_GRAD_EPISODES;  // grad[kGradN] = finished episodes, grad[kGradN + 1] = updated flag
static_assert(PM_GRAD_EPISODES == PM_QNET_NHEAD && PM_GRAD_UPDATED == kGradN + 1 && PM_GRAD_LEN >= kGradN + 2, "grad layout");
constexpr uint32_t kHashEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ bool learner_active(const pm_selfplay& sp) {
    const int64_t s = sp.ctrl->size + sp.n;
    return (s < sp.cap ? s : sp.cap) >= sp.batch;
}

__device__ __forceinline__ double beta_of(const pm_selfplay& sp, int64_t frame) {  // :137
    const double b = sp.beta_start + (double)frame * (1.0 - sp.beta_start) / (double)sp.beta_frames;
    return b < 1.0 ? b : 1.0;
}

// The push k_env makes this step: [pos, pos + n) mod cap at max(prios) (1.0 into an empty buffer, :57).
__device__ __forceinline__ float push_prio(int64_t size, float max_prio) { return size == 0 ? 1.0f : max_prio; }
__device__ __forceinline__ PushRange push_of(const pm_selfplay& sp, int64_t pos, int64_t size, float max_prio) {
    return PushRange{pos, sp.n, sp.cap, prio_pow(push_prio(size, max_prio), (float)sp.alpha)};
}
}  // namespace

// ------------------------------------------------------------------------------------ rollout
// PrioritizedReplay.sample (:64-73) for update samples [64 b, 64 b + 64): proportional draw + un-normalised
// IS weight, one 256-thread block per 64 samples (pm_per.h: per_sample_block). pending: the step's
// push has not landed yet (update 0, drawn beside k_env: the tree accounts for it and its leaves read
// as the pushed value); otherwise (updates 1..U-1) the replay is as k_env left it. The fill is the
// post-push one either way: pos/size advance only when the step commits.
// NS: samples per block (PER_BS, or 32 for the split forward of k_actenv's sampler blocks: lanes of the
// block's upper half then descend for samples no output is taken from).
template <int NS = PER_BS, class Hook = NoHook>
__device__ __forceinline__ void sample_block(const pm_selfplay& sp, int b, bool pending, PerSampleSmem& sm,
                                             int64_t* sidx = nullptr, Hook l2done = Hook()) {
    static_assert(NS == PER_BS || NS == PER_BS / 2, "64 or 32 samples per block");
    const pm_ctrl* c = sp.ctrl;
    const int64_t s = c->size + sp.n;
    const int64_t size = s < sp.cap ? s : sp.cap;
    const int64_t frame = c->frame_idx + 1;  // frame_idx += 1 before sampling (:136)
    const PushRange pr = pending ? push_of(sp, c->pos, c->size, c->max_prio) : PushRange{0, 0, sp.cap, 0.f};
    const uint64_t key = sp.seed_env;
    per_sample_block(
        size >= sp.batch, size, per_tree(sp.per_work, sp.cap), pr, beta_of(sp, frame), b * NS,
        min(sp.batch, b * NS + NS), sm,
        [&](int j) {
            const U4 r = philox64((uint32_t)j, TAG_PER, (uint64_t)frame, key);
            return u53(r.x, r.y);
        },
        [&](int j, int64_t idx, float w) {
            sp.idx[j] = idx;
            sp.isw[j] = w;
            if (sidx) sidx[j - b * NS] = idx;
        },
        l2done);
}

// Both players act (train_iterative.py:240-241) on the matrix cores: ActGrid blocks, modelB tiles
// with epsilon-greedy, opponent tiles grouped by net (modelA / pool) so weights are tile-uniform.
// Blocks [0, ceil(batch/64)) sample the update's batch instead (latency-bound, hidden under the act).
// part: PM_ACT_ALL (sample + side B + side A), PM_ACT_B (sample + side B), PM_ACT_A (side A only:
// the opponents' greedy actions depend on nothing the learner writes, so the overlapped step runs
// them for the next vector step beside k_learn).
union ActSpShared {
    ActShared act;
    PerSampleSmem per;
};
// Feature tiles per feature block: 8 (256-thread blocks, two tiles per wave) / 16 (k_learn's 1024).
constexpr int kFeatTilesAct = 8, kFeatTilesLearn = 16;
// The env blocks' replay rows, state and observation rows go out write-through (pm_dev.h st_out):
// none of it is re-read from this L2 before the kernel boundary. PM_ENV_WT=0 builds plain stores.
#ifndef PM_ENV_WT
#define PM_ENV_WT 6
#endif
constexpr bool kEnvWTRows = (PM_ENV_WT & 1) != 0, kEnvWTState = (PM_ENV_WT & 2) != 0, kEnvWTObs = (PM_ENV_WT & 4) != 0;
__host__ __device__ inline int feat_ntiles(int n) { return (n + 31) / 32; }

__global__ __launch_bounds__(kActBlock, 4) void k_act_sp(const pm_selfplay sp, int part) {
    __shared__ __attribute__((aligned(16))) ActSpShared sh;
    PM_BLK(0);
    const int nsb = part == PM_ACT_A ? 0 : (sp.batch + PER_BS - 1) / PER_BS;
    {   // parts A / ALL with featB: modelB's features for these observations, blocks after the act grid
        const ActGrid g{sp.n, sp.n_pool + 1, sp.chunk_A, sp.chunk_P, part == PM_ACT_A ? 0 : 1};
        const int fb = (int)blockIdx.x - nsb - g.blocks();
        if (fb >= 0) {  // block-uniform
            const int t0 = fb * kFeatTilesAct;
            feat_tiles(sh.act.lw, sp.w_B, sp.obsB, sp.n, t0, min(t0 + kFeatTilesAct, feat_ntiles(sp.n)), sp.featB);
            return;
        }
    }
    if ((int)blockIdx.x < nsb) {
        PM_STAMP(64);
        sample_block(sp, (int)blockIdx.x, true, sh.per);
        PM_STAMP(65);
        PM_BLK_END();
        return;
    }
    if ((int)blockIdx.x == nsb) PM_STAMP_ANY(70);
    const ActGrid g{sp.n, sp.n_pool + 1, sp.chunk_A, sp.chunk_P, part == PM_ACT_A ? 0 : 1};
    const TileOut outA{sp.aA, nullptr, -1.0, 0, 0};
    const TileOut outB{sp.aB, nullptr, -1.0, 0, 0};  // greedy here; k_env applies the epsilon draw
    act_block(sh.act, g, sp.w_opp, sp.n_pool > 0 ? sp.opp : nullptr, sp.w_B, sp.obsA, sp.obsB, outA, outB,
              (int)blockIdx.x - nsb, sp.n_pool + 1 <= kListNets ? sp.opp_list : nullptr, sp.opp_cnt);
    PM_BLK_END();
}

// The three QNet evaluations of train_step (:152-155) for one 32-row tile of the sampled batch on
// the matrix cores: row r < B is s of sample r, row r >= B is s' of sample r - B (the same replay
// row). This lane's row: trans row `id`, `nxt` selects s'. Returns the pre-ReLU features (MFMA
// accumulator layout) and Q_B / Q_T of the row (heads from learn_heads, staged in hf0 / hf1).
// Every output column depends only on its own row, so which tile or kernel computes a row never
// changes a bit of it. rb: the row's reward and action|done bits (trans slots 7 and 15), loaded with
// the operands (a load placed after the MFMAs costs its consumer one more round trip).
__device__ __forceinline__ void batch_row_fwd(const pm_selfplay& sp, const float* lw, const float* hf0, const float* hf1,
                                              int64_t id, bool nxt, int lane, f32x16 (&c2)[2], float (&qb)[3],
                                              float (&qt)[3], float (&rb)[2]) {
    float xs[4];
    const float* tr = sp.trans + id * PM_TRANS_F;
    tile_inputs(tr + (nxt ? 8 : 0), lane >> 5, xs);
    rb[0] = tr[7];
    rb[1] = tr[15];
    tile_hidden(lw, xs, lane, c2);
    tile_heads(hf0, c2, lane, qb);
    tile_heads(hf1, c2, lane, qt);
}

// Rows of the batch whose replay row is NOT in this step's push range are stable while the env tick
// runs: they are computed beside it (one tile per wave) into hfeat [B][80] (features of s | Q_B(s)
// 0..2, r at 3, Q_B(s') 4..6, action|done bits at 7, Q_T(s') 8..10 at 64..); k_learn computes the
// rest. Carrying r and the bits here spares k_learn a load that depends on idx.
template <bool WT = false>
__device__ __forceinline__ void store_hfeat(float* hfeat, int j, bool nxt, int lane, const f32x16 (&c2)[2],
                                            const float (&qb)[3], const float (&qt)[3], const float (&rb)[2]) {
    float* row = hfeat + (size_t)j * 80;
    const int h = lane >> 5;
    if (!nxt) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) st_out<WT>(&row[32 * t + rho(q) + 4 * h], relu(c2[t][q]));
    }
    if (h == 0) {
        if (!nxt) {
            st_out<WT>(&row[64], qb[0]); st_out<WT>(&row[65], qb[1]); st_out<WT>(&row[66], qb[2]);
            st_out<WT>(&row[67], rb[0]);  // reward
            st_out<WT>(&row[71], rb[1]);  // action | done << 8 (float bits)
        } else {
            st_out<WT>(&row[68], qb[0]); st_out<WT>(&row[69], qb[1]); st_out<WT>(&row[70], qb[2]);
            st_out<WT>(&row[72], qt[0]); st_out<WT>(&row[73], qt[1]); st_out<WT>(&row[74], qt[2]);
        }
    }
}

// k_env's last ceil(2B/128) blocks (plain step): rows f * 128 .. of the batch (s rows, then s').
// pending = false (updates 1..U-1, k_batch_fwd): no push is in flight, this block computes every row.
__device__ __forceinline__ void env_fwd_block(const pm_selfplay& sp, int f, bool pending = true) {
    __shared__ __attribute__((aligned(16))) float lw[kLwFloats];
    __shared__ __attribute__((aligned(16))) float hf[2][264];
    if (!learner_active(sp)) return;  // block-uniform
    stage_frags_lds(sp.w_B, lw, f * 5);
    for (int k = threadIdx.x; k < 2 * 264; k += blockDim.x) hf[k / 264][k % 264] = sp.learn_heads[k];
    __syncthreads();
    const int lane = threadIdx.x & 63, B = sp.batch;
    const int r0 = f * 128 + (int)(threadIdx.x >> 6) * 32;
    if (r0 >= 2 * B) return;  // wave-uniform
    const int r = min(r0 + (lane & 31), 2 * B - 1);
    const bool nxt = r >= B;
    const int j = nxt ? r - B : r;
    const int64_t id = sp.idx[j];
    const pm_ctrl* c = sp.ctrl;
    const bool mine = r0 + (lane & 31) < 2 * B && !(pending && push_of(sp, c->pos, c->size, c->max_prio).covers(id));
    f32x16 c2[2];
    float qb[3], qt[3];
    float rb[2];
    batch_row_fwd(sp, lw, hf[0], hf[1], id, nxt, lane, c2, qb, qt, rb);
    if (mine) store_hfeat(sp.hfeat, j, nxt, lane, c2, qb, qt, rb);
}

// The fused step's sampler blocks: block b draws samples [64 b, 64 b + 64) (per_sample_block) and then
// computes their stable rows' forward itself, one tile per wave (waves 0-1: s rows of the block's
// samples, waves 2-3: their s' rows): no other block waits for the sample. The weight image and the
// update's heads are staged while the sampler descends the tree.
struct SampleFwdSmem {
    PerSampleSmem per;
    float lw[kLwFloats];
    float hf[pad256(2 * 264)];  // modelB (update noise) [0, 264) | targetB (mu) [264, 528) head fragments
    int64_t sidx[PER_BS];
};
__device__ __forceinline__ void sample_fwd_block(const pm_selfplay& sp, int b, SampleFwdSmem& sm) {
    // the forward's weights are staged once the top level of the descent is done: LDS DMA in flight
    // makes hipcc wait vmcnt(0) at the next use of a plain load, which would put the 20 KB staging in
    // front of the chunk-sum round trip
    sample_block(sp, b, true, sm.per, sm.sidx, [&] {
        stage_frags_lds(sp.w_B, sm.lw, b * 5);
        copy_lds_f32x4<2 * 264>(sp.learn_heads, sm.hf);
    });
    if (!learner_active(sp)) return;  // block-uniform (sample_block returned before its first barrier)
    __syncthreads();  // sidx, staged weights
    PM_BLK(1);
    const int lane = threadIdx.x & 63, B = sp.batch;
    const int r = (int)(threadIdx.x >> 6) * 32 + (lane & 31);  // row of the block's 128: s rows, then s'
    const bool nxt = r >= PER_BS;
    const int js = nxt ? r - PER_BS : r;
    const int j = b * PER_BS + js;
    const int64_t id = sm.sidx[min(j, B - 1) - b * PER_BS];
    const pm_ctrl* c = sp.ctrl;
    const bool mine = j < B && !push_of(sp, c->pos, c->size, c->max_prio).covers(id);
    f32x16 c2[2];
    float qb[3], qt[3];
    float rb[2];
    batch_row_fwd(sp, sm.lw, sm.hf, sm.hf + 264, id, nxt, lane, c2, qb, qt, rb);
    if (mine) store_hfeat(sp.hfeat, j, nxt, lane, c2, qb, qt, rb);
}

// The split variant (PONGMI_SFB=32, the default): block b draws samples [32 b, 32 b + 32) and its 4 waves
// split the forward of the 2 tiles (s rows, s' rows) by layer-2 tile, as k_rollout16 does (pm_mfma.h
// hidden_half / heads_half): wave 2 k + jt computes layer-2 tile jt of tile k (24 MFMAs deep instead of
// 40); wave jt = 0 runs the head chains over its 32 units and hands the partial sums to wave jt = 1
// through LDS, which continues them in tile_heads' order. Every stored value is bit-identical to
// sample_fwd_block's. s rows need only Q_B (store_hfeat stores Q_T of s' rows only).
struct SampleFwd32Smem {
    PerSampleSmem per;
    float lw[kLwFloats];
    float hf[pad256(2 * 264)];
    int64_t sidx[PER_BS / 2];
    float part[2][64][8];  // [tile][lane]: Q_B chains 0..3, Q_T chains 4..7 after layer-2 tile 0
};
__device__ __forceinline__ void sample_fwd_block32(const pm_selfplay& sp, int b, SampleFwd32Smem& sm) {
    constexpr int NS = PER_BS / 2;
    sample_block<NS>(sp, b, true, sm.per, sm.sidx, [&] {
        stage_frags_lds(sp.w_B, sm.lw, b * 5);
        copy_lds_f32x4<2 * 264>(sp.learn_heads, sm.hf);
    });
    if (!learner_active(sp)) return;  // block-uniform
    __syncthreads();  // sidx, staged weights
    PM_BLK(1);
    const int lane = threadIdx.x & 63, B = sp.batch;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool nxt = (wv >> 1) != 0;  // wave-uniform: tile 0 = s rows, tile 1 = s' rows
    const int jt = wv & 1;
    const int j = b * NS + (lane & 31);
    const int64_t id = sm.sidx[min(j, B - 1) - b * NS];
    const pm_ctrl* c = sp.ctrl;
    const bool mine = j < B && !push_of(sp, c->pos, c->size, c->max_prio).covers(id);
    float xs[4];
    const float* tr = sp.trans + id * PM_TRANS_F;
    tile_inputs(tr + (nxt ? 8 : 0), lane >> 5, xs);
    const float rb0 = tr[7], rb1 = tr[15];
    f32x16 c2;
    hidden_half(sm.lw, xs, lane, jt, c2, [](int) {});
    const float* hf0 = sm.hf;
    const float* hf1 = sm.hf + 264;
    float ab[4] = {0.f, 0.f, 0.f, 0.f}, at[4] = {0.f, 0.f, 0.f, 0.f};
    float* row = sp.hfeat + (size_t)j * 80;
    const int h = lane >> 5;
    if (jt == 0) {
        heads_half(hf0, c2, lane, 0, ab);
        if (nxt) heads_half(hf1, c2, lane, 0, at);
        *reinterpret_cast<float4*>(&sm.part[nxt][lane][0]) = make_float4(ab[0], ab[1], ab[2], ab[3]);
        if (nxt) *reinterpret_cast<float4*>(&sm.part[nxt][lane][4]) = make_float4(at[0], at[1], at[2], at[3]);
    }
    if (mine && !nxt) {
#pragma unroll
        for (int q = 0; q < 16; ++q) row[32 * jt + rho(q) + 4 * h] = relu(c2[q]);
    }
    __syncthreads();  // the chains over layer-2 tile 0
    if (jt == 0) return;
    {
        const float4 pa = *reinterpret_cast<const float4*>(&sm.part[nxt][lane][0]);
        ab[0] = pa.x; ab[1] = pa.y; ab[2] = pa.z; ab[3] = pa.w;
    }
    heads_half(hf0, c2, lane, 1, ab);
    float qb[3], qt[3];
    heads_finish(ab, hf0, qb);
    if (nxt) {
        const float4 pt = *reinterpret_cast<const float4*>(&sm.part[nxt][lane][4]);
        at[0] = pt.x; at[1] = pt.y; at[2] = pt.z; at[3] = pt.w;
        heads_half(hf1, c2, lane, 1, at);
        heads_finish(at, hf1, qt);
    }
    if (mine && h == 0) {
        if (!nxt) {
            row[64] = qb[0]; row[65] = qb[1]; row[66] = qb[2];
            row[67] = rb0;  // reward
            row[71] = rb1;  // action | done << 8 (float bits)
        } else {
            row[68] = qb[0]; row[69] = qb[1]; row[70] = qb[2];
            row[72] = qt[0]; row[73] = qt[1]; row[74] = qt[2];
        }
    }
}

__device__ __forceinline__ void write_opp_lists(const pm_selfplay& sp, OppListSmem& sm, int blk, int i, bool valid,
                                                int net) {
    write_opp_lists(sp.n_pool + 1, sp.opp_list, sp.opp_cnt, sm, blk, i, valid, net);
}

struct EnvSmem {
    float lds[2][kBlock][7];
    long long red[kBlock / 64][6];
    OppListSmem ol;
};
struct ActEnvSmem {
    EnvSmem e;
    float lw[kLwFloats];  // modelB's acting fragment image
};

// env.step (:242) + memory.push (:243) + episode bookkeeping (:245-249) + next opponent (:235-236)
// and env.reset (:238) for finished arenas of env block blk; writes next step's observations.
// ACT (the fused step, k_actenv): modelB's greedy action for the block's 256 arenas is computed here
// first (select_action_B, :126-130, the argmax side), on the matrix cores: wave w takes the two
// 32-row tiles of its own 64 arenas, so lane l's action sits in lane l (tile 0 holds rows 0-31 in
// both lane halves, tile 1 rows 32-63), with no LDS exchange. The env's state loads are issued with
// the weight staging and land under it. Without ACT (k_env) the argmax comes from k_act_sp via aB.
template <bool ACT>
__device__ __forceinline__ void env_block(const pm_selfplay& sp, int blk, EnvSmem& sm, float* lw) {
    const int i0 = blk * kBlock;
    const int i = i0 + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool valid = i < sp.n;
    const int ii = valid ? i : sp.n - 1;
    const pm_ctrl* c = sp.ctrl;
    if (blk == 0) PM_STAMP_ANY(72);
    PM_ENV_STAMP(0, blk);
    float xs[2][4];
    f32x16 fc2[2][2];  // featB: this wave's two tiles of modelB's features (computed ahead)
    if (ACT && sp.featB) {
        // heads only: F_H .. F_BH of the acting image (65 float4) -> LDS; the features from featB
        if (threadIdx.x < 65)
            reinterpret_cast<float4*>(lw + F_H)[threadIdx.x] =
                reinterpret_cast<const float4*>(sp.w_B + PLAIN + F_H)[threadIdx.x];
#pragma unroll
        for (int k = 0; k < 2; ++k) feat_load(sp.featB, blk * 8 + 2 * wv + k, lane, fc2[k]);
    } else if (ACT) {
        stage_frags_lds(sp.w_B, lw, blk);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int row = min(i0 + 64 * wv + 32 * k + (lane & 31), sp.n - 1);
            tile_inputs(sp.obsB + (size_t)row * 7, lane >> 5, xs[k]);
        }
    }
    // Every per-arena load is issued here, in one basic block, before any branch (loads placed after
    // a branch were issued only after it, one more HBM round trip). The serve counter goes first:
    // the next episode's opponent and serve are drawn for every lane while the state loads are in
    // flight (lanes that finish use them; see k_env_step).
    // The control block is read before them (vmcnt retires in issue order: what only needs ns and
    // the control words can then run while the state is still in flight).
    const uint32_t ns = (uint32_t)__builtin_nontemporal_load(&sp.st.serves[ii]);
    const int64_t pos = c->pos, size = c->size;
    const float cmaxp = c->max_prio;
    const uint64_t cstep = c->step;
    const double ceps = c->epsilon;
    const int o = sp.opp[ii];
    const float er0 = sp.ep_reward[ii];
    Arena a = load_arena(sp.st, ii);
    const int aA = sp.aA[ii];
    int aB = ACT ? 0 : sp.aB[ii];
    __builtin_amdgcn_sched_barrier(0);
    const float maxp = push_prio(size, cmaxp);  // max(prios) if buffer else 1.0 (:57)
    float* leaf = per_tree(sp.per_work, sp.cap).leaf;
    const float pval = prio_pow(maxp, (float)sp.alpha);  // its PER leaf

    // Draws that need only the serve counter and the control block, pinned ahead of everything that
    // waits for the state loads:
    //   select_action_B (:126-130): random.random() < eps ? randint(0, 2) : argmax (the argmax is
    //   the act's; the draw is per-arena VALU work, cheaper here than beside the MFMAs);
    //   the next episode's opponent (:235-236) and serve (env.reset(), :238), used if this one ends.
    int onext, eps_a;
    bool eps_hit;
    double svx, svy, sspn;
    {
        const U4 rr = philox64((uint32_t)ii, TAG_ACT, cstep, sp.seed_env);
        eps_hit = u53(rr.x, rr.y) < ceps;
        eps_a = (int)below(rr.z, 3u);
        const U4 q = philox((uint32_t)ii, TAG_OPP, ns, 0u, sp.seed_env);
        onext = (sp.n_pool > 0 && u53(q.x, q.y) < sp.pool_ratio) ? 1 + below(q.z, (uint32_t)sp.n_pool) : 0;
        philox_serve(sp.env, (uint32_t)ii, ns, sp.seed_env, svx, svy, sspn);
        asm volatile("" ::"v"(onext), "v"(svx), "v"(svy), "v"(sspn), "v"(eps_hit), "v"(eps_a));
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ACT) {
        __syncthreads();  // the fragment image is staged (every load of the block has landed)
        PM_ENV_STAMP(7, blk);
        int act[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float q[3];
            if (sp.featB) {
                tile_heads(lw + F_H, fc2[k], lane, q);
            } else {
                f32x16 c2[2];
                tile_hidden(lw, xs[k], lane, c2);
                tile_heads(lw + F_H, c2, lane, q);
            }
            act[k] = argmax3(q);
            if (sp.featB && sp.frow) {  // k_learn_multi's features of s: ReLU(layer 2) of this push's rows
                const int ar = i0 + 64 * wv + 32 * k + (lane & 31);
                if (ar < sp.n) {
                    int64_t slot = pos + ar;
                    if (slot >= sp.cap) slot -= sp.cap;
                    float4* fr = reinterpret_cast<float4*>(sp.frow + slot * 64) + (lane >> 5);
#pragma unroll
                    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4)  // units 32 jt + 8 q4 + 4 h + 0..3
                            st_f4<kEnvWTRows>(fr + 8 * jt + 2 * q4,
                                              make_float4(relu(fc2[k][jt][4 * q4]), relu(fc2[k][jt][4 * q4 + 1]),
                                                          relu(fc2[k][jt][4 * q4 + 2]), relu(fc2[k][jt][4 * q4 + 3])));
                }
            }
        }
        aB = lane < 32 ? act[0] : act[1];
    }
    PM_ENV_STAMP(1, blk);
    if (eps_hit) aB = eps_a;
    float oA[7], oB[7];
    observe(a, oA, oB);  // the state the actions were chosen on (= obs of the previous env kernel)
    float rA, rB;
    const int d = tick(sp.env, a, aA, aB, rA, rB);
    float nA[7], nB[7];
    observe(a, nA, nB);
#ifdef PM_DIAG
    asm volatile("" ::"v"(nA[0]), "v"(nB[1]), "v"(d));
#endif
    PM_ENV_STAMP(2, blk);
    const float er = er0 + rB;  // ep_reward += rB (:245)
    const bool fin = valid && d;
    {   // per-block partials, no atomics (:247-249)
        const bool win = er > 0.f;
        const unsigned long long mf = __ballot(fin), mA = __ballot(fin && o == 0), mwA = __ballot(fin && o == 0 && win);
        const unsigned long long mP = __ballot(fin && o != 0), mwP = __ballot(fin && o != 0 && win);
        const int rs = wave_sum(fin ? (int)er : 0);
        if (lane == 0) {
            sm.red[wv][0] = __popcll(mf); sm.red[wv][1] = __popcll(mA); sm.red[wv][2] = __popcll(mwA);
            sm.red[wv][3] = __popcll(mP); sm.red[wv][4] = __popcll(mwP); sm.red[wv][5] = rs;
        }
    }
    int onew = o;
    if (valid) {
        // memory.push((oB, aB, rB, nB, done)) (:243, :56-63)
        int64_t slot = pos + i;  // pos < cap and i < n <= cap: one conditional subtract is the modulo
        if (slot >= sp.cap) slot -= sp.cap;  // (a per-lane 64-bit % is a ~100-instruction expansion)
        // write-through (pm_dev.h st_out): the ring is re-read only by later samples, and the state and
        // observation rows only by later launches, so none of it stays dirty in L2 for the boundary
        float4* row = reinterpret_cast<float4*>(sp.trans + slot * PM_TRANS_F);
        st_f4<kEnvWTRows>(row + 0, make_float4(oB[0], oB[1], oB[2], oB[3]));
        st_f4<kEnvWTRows>(row + 1, make_float4(oB[4], oB[5], oB[6], rB));
        st_f4<kEnvWTRows>(row + 2, make_float4(nB[0], nB[1], nB[2], nB[3]));
        st_f4<kEnvWTRows>(row + 3, make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8))));
        sp.prios[slot] = maxp;
        leaf[slot] = pval;
        float ernew = er;
        if (d) {  // next episode: the opponent and serve drawn above
            onew = onext;
            serve(a, svx, svy, sspn);
            sp.st.serves[i] = (int32_t)ns + 1;
            ernew = 0.f;
            observe(a, nA, nB);
        }
        store_arena<kEnvWTState>(sp.st, i, a);
        sp.opp[i] = onew;
        sp.aB[i] = (int8_t)aB;  // the action taken
        sp.ep_reward[i] = ernew;
    }
    PM_ENV_STAMP(3, blk);
#pragma unroll
    for (int k = 0; k < 7; ++k) { sm.lds[0][threadIdx.x][k] = nA[k]; sm.lds[1][threadIdx.x][k] = nB[k]; }
    __syncthreads();
    PM_ENV_STAMP(4, blk);
    if (threadIdx.x < 6) {
        long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += sm.red[w][threadIdx.x];
        sp.partials[(size_t)blk * 8 + threadIdx.x] = t;
    }
    write_opp_lists(sp, sm.ol, blk, i, valid, onew);
    PM_ENV_STAMP(5, blk);
    copy_rows7<kEnvWTObs>(sp.obsA, sm.lds[0], i0, sp.n);
    copy_rows7<kEnvWTObs>(sp.obsB, sm.lds[1], i0, sp.n);
    PM_ENV_STAMP_DRAIN(6, blk);
}

// The plain step's env kernel: env blocks first, then the learner-forward blocks (measured:
// dispatching the forward blocks first lengthens the kernel by ~1 us; last, they finish inside the
// env blocks' time).
__global__ __launch_bounds__(kBlock) void k_env(const pm_selfplay sp) {
    const int blk = (int)blockIdx.x;
    const int nenv = (sp.n + kBlock - 1) / kBlock;
    if (blk >= nenv) {
        env_fwd_block(sp, blk - nenv);
        return;
    }
    __shared__ __attribute__((aligned(16))) EnvSmem sm;
    env_block<false>(sp, blk, sm, nullptr);
}

// The fused step's first kernel (pm_selfplay_actenv): blocks [0, ceil(B/64)) sample the update's batch
// and compute its stable rows (sample_fwd_block); every other block acts for modelB and ticks its 256
// arenas (env_block<true>). Replaces k_act_sp(PM_ACT_B) + k_env of the overlapped step, bit for bit.
union ActEnvShared {
    ActEnvSmem ae;
    SampleFwdSmem sf;
    SampleFwd32Smem sf32;
};
// NS: samples per sampler block (64: sample_fwd_block, 32: sample_fwd_block32).
template <int NS>
__global__ __launch_bounds__(kBlock) void k_actenv(const pm_selfplay sp) {
    __shared__ __attribute__((aligned(16))) ActEnvShared sh;
    const int nsb = (sp.batch + NS - 1) / NS;
    if ((int)blockIdx.x < nsb) {
        PM_BLK(0);
        if constexpr (NS == PER_BS) sample_fwd_block(sp, (int)blockIdx.x, sh.sf);
        else sample_fwd_block32(sp, (int)blockIdx.x, sh.sf32);
        PM_BLK_END();
        return;
    }
    env_block<true>(sp, (int)blockIdx.x - nsb, sh.ae.e, sh.ae.lw);
}

// ------------------------------------------------------------------------------------ init
__global__ __launch_bounds__(kBlock) void k_sp_init(const pm_selfplay sp) {
    __shared__ __attribute__((aligned(16))) float lds[kBlock][7];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0};
    int net = 0;
    if (i < sp.n) {
        const uint32_t ns = (uint32_t)sp.st.serves[i];
        const U4 q = philox((uint32_t)i, TAG_OPP, ns, 0u, sp.seed_env);
        net = (sp.n_pool > 0 && u53(q.x, q.y) < sp.pool_ratio) ? 1 + below(q.z, (uint32_t)sp.n_pool) : 0;
        sp.opp[i] = net;
        Arena a;
        double vx, vy, spn;
        philox_serve(sp.env, (uint32_t)i, ns, sp.seed_env, vx, vy, spn);
        serve(a, vx, vy, spn);
        store_arena(sp.st, i, a);
        sp.st.serves[i] = (int32_t)ns + 1;
        sp.ep_reward[i] = 0.f;
        observe(a, oA, oB);
    }
    {
        __shared__ OppListSmem ol;
        write_opp_lists(sp, ol, blockIdx.x, i, i < sp.n, net);
    }
    store_rows7(sp.obsA, lds, oA, i0, sp.n);
    store_rows7(sp.obsB, lds, oB, i0, sp.n);
}

// ------------------------------------------------------------------------------------ learner
// ------------------------------------------------------------------------------------ apply
struct __attribute__((aligned(16))) ApplySmem {  // 520-float arrays padded to whole 1 KB (16-B lane) global_load_lds chunks
    float hp[pad256(PM_QNET_NHEAD)];   // modelB head parameters (after the optimizer step)
    float tmu[pad256(PM_QNET_NHEAD)];  // targetB head parameters (mu used)
    float m[pad256(PM_QNET_NHEAD)], v[pad256(PM_QNET_NHEAD)];  // Adam moments
    float g[PM_QNET_NHEAD + 2];                // shard-summed grads | finished episodes | updated flag
    float ak[2];                               // Adam step size lr / (1 - b1^t), sqrt(1 - b2^t)
    float nact[132], ntrain[132];
    float heads[3][260];                       // folded acting / next-update / target heads
    double eps_next;                           // fused learner: eps * decay^D, computed early
};

// torch.optim.Adam's bias corrections for update number ts, computed in fp64 as torch does (Python
// floats), once per block (two fp64 pow per thread cost ~3 us of VALU in a 1024-thread block).
__device__ __forceinline__ void adam_consts(const pm_selfplay& sp, int64_t ts, ApplySmem& sm) {
    const double bc1 = 1.0 - pow(sp.beta1, (double)ts);
    const double bc2 = 1.0 - pow(sp.beta2, (double)ts);
    sm.ak[0] = (float)(sp.lr / bc1);
    sm.ak[1] = (float)sqrt(bc2);
}
// The same two constants from two lanes of one wave (lane `which` = 0: step size, 1: sqrt(bc2)), so
// the two fp64 pow run side by side instead of back to back.
__device__ __forceinline__ void adam_const_lane(const pm_selfplay& sp, int64_t ts, ApplySmem& sm, int which) {
    const double bc = 1.0 - pow(which ? sp.beta2 : sp.beta1, (double)ts);
    sm.ak[which] = which ? (float)sqrt(bc) : (float)(sp.lr / bc);
}

// Block-wide: the optimizer's inputs global -> LDS directly (global_load_lds, no wait until the
// caller's barrier). g: from LDS already when fused.
__device__ __forceinline__ void load_apply_inputs(const pm_selfplay& sp, ApplySmem& sm, bool with_grad) {
    copy_lds_f32x4<PM_QNET_NHEAD>(sp.paramsB + PM_QNET_HEAD_OFF, sm.hp);
    copy_lds_f32x4<PM_QNET_NHEAD>(sp.paramsT + PM_QNET_HEAD_OFF, sm.tmu);
    copy_lds_f32x4<PM_QNET_NHEAD>(sp.adam_m, sm.m);
    copy_lds_f32x4<PM_QNET_NHEAD>(sp.adam_v, sm.v);
    if (with_grad)
        for (int k = threadIdx.x; k < PM_QNET_NHEAD + 2; k += blockDim.x) sm.g[k] = sp.grad[k];
}

// Everything that follows from the head parameters once they are final for this step, from LDS:
// acting weights for the next vector step (select_action_B -> reset_noise, :125; the noise lands
// in modelB's epsilon buffers), the next update's modelB heads with fresh noise (reset_noise, :142)
// and targetB heads (eval mode: mu, :100), both in MFMA fragment order in learn_heads, plus that
// update's noise. Block-wide; noise already in sm.nact / sm.ntrain.
__device__ __forceinline__ void derive_weights(const pm_selfplay& sp, ApplySmem& sm) {
    const int t = threadIdx.x;
    float* lh = sp.learn_heads;
    // the three folds are independent: one pass on three 260-thread groups, one barrier, then the
    // three fragment writes
    // (threads 256..1023: in the fused learner threads < 256 are still refreshing level-2 tree nodes)
    const int g = (t - 256) >> 8, u = (t - 256) & 255;
    if (t >= 256 && g == 0) {
        fold_heads_from(sm.hp, nullptr, sm.nact, PM_FOLD_TRAIN_FRESH, sm.heads[0], sp.paramsB + PM_QNET_EPS_OFF, u, 256);
    } else if (t >= 256 && g == 1) {
        fold_heads_from(sm.hp, nullptr, sm.ntrain, PM_FOLD_TRAIN_FRESH, sm.heads[1], lh + 528, u, 256);
    } else if (t >= 256 && g == 2) {
        fold_heads_from(sm.tmu, nullptr, nullptr, PM_FOLD_EVAL, sm.heads[2], nullptr, u, 256);
    }
    __syncthreads();
    write_head_frags(sm.heads[0], sp.w_B);
    heads_to_frags(sm.heads[1], lh);
    heads_to_frags(sm.heads[2], lh + 264);
}

// derive_weights for an update of k_learn_multi that is not the launch's last: only what the next
// update reads, from LDS to LDS — the next update's modelB heads (fresh noise) and targetB heads.
// The acting weights and every global copy follow from the last update alone.
__device__ __forceinline__ void derive_weights_lds(ApplySmem& sm) {
    const int t = threadIdx.x;
    const int g = (t - 256) >> 8, u = (t - 256) & 255;
    if (t >= 256 && g == 1) {
        fold_heads_from(sm.hp, nullptr, sm.ntrain, PM_FOLD_TRAIN_FRESH, sm.heads[1], nullptr, u, 256);
    } else if (t >= 256 && g == 2) {
        fold_heads_from(sm.tmu, nullptr, nullptr, PM_FOLD_EVAL, sm.heads[2], nullptr, u, 256);
    }
    __syncthreads();
}

// Both noise draws at once, half of the block each.
__device__ __forceinline__ void gen_both_noises(const pm_selfplay& sp, ApplySmem& sm, uint64_t act_ctr,
                                                uint64_t train_ctr) {
    const int t = threadIdx.x, half = blockDim.x / 2;
    if (t < half) gen_noise(sp.seed_net, TAG_NOISE_ACT, act_ctr, sm.nact, t, half);
    else gen_noise(sp.seed_net, TAG_NOISE_TRAIN, train_ctr, sm.ntrain, t - half, half);
}
// The same draws on threads [t0, t0 + 512) only (the fused learner's waves with slack in its load
// phase). Same values: every noise element depends only on (seed, tag, counter, index).
__device__ __forceinline__ void gen_both_noises_on(const pm_selfplay& sp, ApplySmem& sm, uint64_t act_ctr,
                                                   uint64_t train_ctr, int t0) {
    const int u = (int)threadIdx.x - t0;
    if (u < 0 || u >= 512) return;
    if (u < 256) gen_noise(sp.seed_net, TAG_NOISE_ACT, act_ctr, sm.nact, u, 256);
    else gen_noise(sp.seed_net, TAG_NOISE_TRAIN, train_ctr, sm.ntrain, u - 256, 256);
}

// optimizer.step() (:161) on the shard-summed grads, target sync (:166-168), epsilon decay (:261),
// replay / step counters, then derive_weights for the next step. All inputs in LDS (sm) and `cs`
// (the control block as the kernel found it); only stores go to global memory. Both noises are in
// sm.nact / sm.ntrain and sm.eps_next holds eps * decay^D already (drawn / computed by idle waves
// while the callers' loads were in flight). Two parts: apply_adam (per-thread, no barrier: the fused
// learner runs it beside the sum-tree's level-2 refresh) and apply_finish (behind a barrier).
// torch.optim.Adam (single-tensor path) on head parameter k with gradient g (summed over shards).
__device__ __forceinline__ void adam_one(const pm_selfplay& sp, ApplySmem& sm, int k, float gsum, bool store = true) {
    const float step_size = sm.ak[0], bc2s = sm.ak[1];  // adam_consts, published before a barrier
    const float g = gsum / (float)sp.world;
    float m = sm.m[k], v = sm.v[k], p = sm.hp[k];
    m = m + (float)(1.0 - sp.beta1) * (g - m);                  // exp_avg.lerp_(grad, 1-beta1)
    v = v * (float)sp.beta2 + (float)(1.0 - sp.beta2) * g * g;  // mul_(beta2).addcmul_(g, g, 1-beta2)
    const float denom = sqrtf(v) / bc2s + (float)sp.adam_eps;
    p = p - step_size * (m / denom);
    if (store) {  // k_learn_multi keeps all but its last update's state in LDS only
        sp.paramsB[PM_QNET_HEAD_OFF + k] = p;
        sp.adam_m[k] = m;
        sp.adam_v[k] = v;
    }
    sm.hp[k] = p;
    sm.m[k] = m;  // k_learn_multi runs the next update from LDS
    sm.v[k] = v;
}
__device__ __forceinline__ void apply_adam(const pm_selfplay& sp, ApplySmem& sm) {
    const int t = threadIdx.x, nt = blockDim.x;
    if (sm.g[kGradN + 1] > 0.5f)
        for (int k = t; k < PM_QNET_NHEAD; k += nt) adam_one(sp, sm, k, sm.g[k]);
}
// mode (PM_UPD_*): FIRST commits the epsilon decay of the step's finished episodes, LAST the replay
// and step counters (with U > 1 updates per step pm_selfplay_commit does that after the last one).
__device__ __forceinline__ void apply_finish(const pm_selfplay& sp, ApplySmem& sm, const pm_ctrl& cs, int mode) {
    const int t = threadIdx.x, nt = blockDim.x;
    const bool train = sm.g[kGradN + 1] > 0.5f;
    const int64_t ts = cs.train_steps + (train ? 1 : 0);
    const uint64_t step = cs.step;
    PM_STAMP(20);
    if (train && ts % sp.target_update_interval == 0) {  // targetB.load_state_dict(modelB) (:166-168)
        for (int k = t; k < PM_QNET_NHEAD; k += nt) sm.tmu[k] = sm.hp[k];
        for (int k = t; k < PM_QNET_NP; k += nt) {
            const int h = k - PM_QNET_HEAD_OFF;
            sp.paramsT[k] = (h >= 0 && h < PM_QNET_NHEAD) ? sm.hp[h] : sp.paramsB[k];
        }
        __syncthreads();
    }
    derive_weights(sp, sm);
    PM_STAMP(21);
    if (t == 0) {
        pm_ctrl* c = sp.ctrl;
        if (mode & PM_UPD_FIRST) {
            const double e = sm.eps_next;  // eps * decay^D, D = finished episodes (all shards) (:261)
            c->epsilon = e > sp.min_epsilon ? e : sp.min_epsilon;
        }
        if (train) { c->train_steps = ts; c->frame_idx = cs.frame_idx + 1; }
        if (mode & PM_UPD_LAST) {
            c->pos = (cs.pos + sp.n) % sp.cap;
            const int64_t s = cs.size + sp.n;
            c->size = s < sp.cap ? s : sp.cap;
            c->step = step + 1;
        }
    }
}

// ------------------------------------------------------------------------------------ learner
// ---- the push-range rows of an update's batch: the samples whose replay row this step's k_actenv
// wrote (its sampler blocks cannot read them), s rows then s' rows, one 32-row tile per wave, in
// plist order (pcnt: per-wave counts of the ballot that built plist; B <= 256: waves 0..3).
// emit(j, nxt, lane, c2, qb, qt, rb) runs for the lanes that hold a row.
template <typename Emit>
__device__ __forceinline__ void push_rows_fwd(const pm_selfplay& sp, const float* lw, const float* hf,
                                              const int64_t* sidx, const int* plist, const int* pcnt, int wv, int lane,
                                              Emit emit) {
    int pre[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < 4; ++w) pre[w + 1] = pre[w] + pcnt[w];
    const int np = pre[4];
    if (wv * 32 >= 2 * np) return;  // wave-uniform
    const int rr = min(wv * 32 + (lane & 31), 2 * np - 1);
    const bool nxt = rr >= np;
    const int k = nxt ? rr - np : rr;
    // selects, not pre[w]: a dynamically indexed array is a scratch store + load round trip
    const int w = k >= pre[3] ? 3 : k >= pre[2] ? 2 : k >= pre[1] ? 1 : 0;
    const int pw = k >= pre[3] ? pre[3] : k >= pre[2] ? pre[2] : k >= pre[1] ? pre[1] : 0;
    const int j = plist[w * 64 + k - pw];
    f32x16 c2[2];
    float qb[3], qt[3], rb[2];
    batch_row_fwd(sp, lw, hf, hf + 264, sidx[j], nxt, lane, c2, qb, qt, rb);
    if (wv * 32 + (lane & 31) < 2 * np) emit(j, nxt, lane, c2, qb, qt, rb);
}

// The push-row hand-off inside k_learn: block 1 computes the push rows beside the learner's load
// phase and publishes them in hfeat rows [B, 2B) (hfeat row layout), then the flag word at hfeat row
// 2B = ctrl.step + 1. Publication follows the cross-CU rules for write-through hand-offs: every
// payload store and the flag store sc1, every storing wave waits vmcnt(0), a workgroup barrier,
// then one lane stores the flag; the learner polls the flag with sc1 loads from one lane, joins a
// barrier, and reads the payload with sc1 loads only. Block 1 reads the control block unsynchronised,
// so in a FIRST update it ALWAYS publishes its token (at once, with no rows, when the update does not
// train) and a learner that commits the control block in this launch (fused apply) waits for that
// token before the commit even when it needed no rows: block 1 can then never see the next step's
// control block and publish the token the NEXT launch's learner polls for with rows built from this
// step's push range. Block 1 waits for nothing, so it always completes; the poll is
// bounded anyway (kPushPollMax, ~20 ms): a flag that never came sets ctrl.status bit 0, which the
// host reports as an error (pongmi.selfplay.SelfPlayLearner.check_status), and an update whose push
// rows never came is void: it trains nothing (no scatter, gradients, Adam or train-step count), as
// an update before the replay holds a batch.
constexpr int kPushPollMax = 20000;
constexpr int PM_CTRL_PUSH_TIMEOUT = 1;
constexpr int PM_CTRL_NAN_PRIO = 2;  // a NaN |TD error| was scattered (its PER leaf is 0: never sampled)
__device__ __forceinline__ bool push_handoff(int mode, bool train) { return (mode & PM_UPD_FIRST) && train; }
__device__ __forceinline__ int* push_flag(const pm_selfplay& sp) {
    return reinterpret_cast<int*>(sp.hfeat + (size_t)2 * sp.batch * 80);
}
__device__ __forceinline__ int push_token(const pm_ctrl& cs) { return (int)((uint32_t)cs.step + 1u); }
// the tree-refresh epoch (tree_block): word 1 of the flag row
__device__ __forceinline__ uint32_t* tr_epoch(const pm_selfplay& sp) {
    return reinterpret_cast<uint32_t*>(sp.hfeat + (size_t)2 * sp.batch * 80) + 1;
}
// The push rows as tagged 8-byte granules {tag, float bits} (round 5; tr bit 3, PONGMI_PUSHG): sample
// j's hfeat floats 0..74 at granule j * 76 + f of hfeat rows [2B + 8, 4B + 8) (ABI 22). The data is
// the flag: block 1 stores each granule once (sc1), with no drain, and the learner's loads of them are
// the poll, which saves the payload drain, the flag store's trip and the flag poll's (~2 us; MI355X
// guide: handoff-1to1 vs handoff-flag). The tag is this launch's tree-refresh epoch + 1 (tr_epoch:
// bumped by block 1 at the end of every launch with the tree block, so never reused by a later
// launch, checkpoint restores included). The flag word is still stored, right after block 1 read the
// control block: a learner that needed no rows waits for it before its commit; one that
// saw a granule of this launch's tag knows block 1 read this step's control block.
constexpr int kPushGF = 76;  // granule stride per sample (floats 0..74 used)
constexpr int kPushGN = 75;
__device__ __forceinline__ uint64_t* push_granules(const pm_selfplay& sp) {
    return reinterpret_cast<uint64_t*>(sp.hfeat + (size_t)(2 * sp.batch + 8) * 80);
}
__device__ __forceinline__ void push_publish(uint64_t* g, uint32_t tag, float v) {
    __hip_atomic_store(g, ((uint64_t)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane polls for block 1's token of this update (bounded). false: it never came (status bit 0 set).
__device__ __forceinline__ bool push_wait(const pm_selfplay& sp, const pm_ctrl& cs) {
    const int* flag = push_flag(sp);
    const int tok = push_token(cs);
    for (int it = 0; __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tok; ++it) {
        if (it == kPushPollMax) {
            sp.ctrl->status = cs.status | PM_CTRL_PUSH_TIMEOUT;
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

struct PushFwdSmem {
    float lw[kLwFloats];
    float hf[pad256(2 * 264)];
    int64_t sidx[PM_MAX_BATCH];
    int plist[PM_MAX_BATCH];
    int pcnt[16];
    float part[8][64][8];  // push_rows_fwd2: the head chains after layer-2 tile 0, per tile pair of waves
};

// push_rows_fwd on block 1's 16 waves, two per 32-row tile (hidden_half / heads_half, as
// sample_fwd_block32): wave 2k + jt computes layer-2 tile jt of tile 8 it + k (24 MFMAs deep instead
// of 40); wave jt = 0 runs the head chains over its 32 units and hands them to wave jt = 1 through
// LDS, which continues them in tile_heads' order. Bit-identical rows to push_rows_fwd.
__device__ __forceinline__ void push_rows_fwd2(const pm_selfplay& sp, PushFwdSmem& sm, int wv, int lane, float* pay,
                                               uint32_t gtag) {
    uint64_t* pg = push_granules(sp);
    // hfeat float f of sample j: a payload-row word (drained + flag) or a tagged granule
    auto put = [&](int j, int f, float v) {
        if (gtag) push_publish(pg + (size_t)j * kPushGF + f, gtag, v);
        else st_out<true>(pay + (size_t)j * 80 + f, v);
    };
    int pre[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < 4; ++w) pre[w + 1] = pre[w] + sm.pcnt[w];
    const int np = pre[4];
    const int ntile = (2 * np + 31) >> 5;
    const int jt = wv & 1, h = lane >> 5;
    const float* hf0 = sm.hf;
    const float* hf1 = sm.hf + 264;
    for (int it = 0; it * 8 < ntile; ++it) {  // block-uniform
        const int tile = it * 8 + (wv >> 1);
        const bool act = tile < ntile;  // wave-uniform
        f32x16 c2 = {};
        float ab[4] = {0.f, 0.f, 0.f, 0.f}, at[4] = {0.f, 0.f, 0.f, 0.f};
        float rb0 = 0.f, rb1 = 0.f;
        bool nxt = false, mine = false;
        int j = 0;
        if (act) {
            const int r0 = tile * 32 + (lane & 31);
            const int rr = min(r0, 2 * np - 1);
            nxt = rr >= np;
            const int k = nxt ? rr - np : rr;
            const int w = k >= pre[3] ? 3 : k >= pre[2] ? 2 : k >= pre[1] ? 1 : 0;
            const int pw = k >= pre[3] ? pre[3] : k >= pre[2] ? pre[2] : k >= pre[1] ? pre[1] : 0;
            j = sm.plist[w * 64 + k - pw];
            mine = r0 < 2 * np;
            const float* tr = sp.trans + sm.sidx[j] * PM_TRANS_F;
            float xs[4];
            tile_inputs(tr + (nxt ? 8 : 0), h, xs);
            rb0 = tr[7];
            rb1 = tr[15];
            hidden_half(sm.lw, xs, lane, jt, c2, [](int) {});
            if (mine && !nxt) {
#pragma unroll
                for (int q = 0; q < 16; ++q) put(j, 32 * jt + rho(q) + 4 * h, relu(c2[q]));
            }
            if (jt == 0) {
                heads_half(hf0, c2, lane, 0, ab);
                heads_half(hf1, c2, lane, 0, at);
                *reinterpret_cast<float4*>(&sm.part[wv >> 1][lane][0]) = make_float4(ab[0], ab[1], ab[2], ab[3]);
                *reinterpret_cast<float4*>(&sm.part[wv >> 1][lane][4]) = make_float4(at[0], at[1], at[2], at[3]);
            }
        }
        __syncthreads();  // the chains over layer-2 tile 0
        if (act && jt == 1) {
            const float4 pb = *reinterpret_cast<const float4*>(&sm.part[wv >> 1][lane][0]);
            const float4 pt = *reinterpret_cast<const float4*>(&sm.part[wv >> 1][lane][4]);
            ab[0] = pb.x; ab[1] = pb.y; ab[2] = pb.z; ab[3] = pb.w;
            at[0] = pt.x; at[1] = pt.y; at[2] = pt.z; at[3] = pt.w;
            heads_half(hf0, c2, lane, 1, ab);
            heads_half(hf1, c2, lane, 1, at);
            float qb[3], qt[3];
            heads_finish(ab, hf0, qb);
            heads_finish(at, hf1, qt);
            if (mine && h == 0) {
                if (!nxt) {
                    put(j, 64, qb[0]); put(j, 65, qb[1]); put(j, 66, qb[2]);
                    put(j, 67, rb0);  // reward
                    put(j, 71, rb1);  // action | done << 8 (float bits)
                } else {
                    put(j, 68, qb[0]); put(j, 69, qb[1]); put(j, 70, qb[2]);
                    put(j, 72, qt[0]); put(j, 73, qt[1]); put(j, 74, qt[2]);
                }
            }
        }
        if ((it + 1) * 8 < ntile) __syncthreads();  // block-uniform: part is reused
    }
}
// Returns the control block as block 1 read it (the tree refresh uses the same copy: the learner
// waits for block 1's token or granules, which follow this read, before it commits the next step's).
__device__ __forceinline__ pm_ctrl push_fwd_block(const pm_selfplay& sp, int mode, PushFwdSmem& sm, bool push2, bool pushg) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, B = sp.batch;
    PM_STAMP_ANY(50);
    stage_frags_lds(sp.w_B, sm.lw, 0);
    copy_lds_f32x4<2 * 264>(sp.learn_heads, sm.hf);
    const int64_t id = t < B ? sp.idx[t] : 0;
    const uint32_t gtag = pushg ? __hip_atomic_load(tr_epoch(sp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    __builtin_amdgcn_sched_barrier(0);
    const pm_ctrl cs = *sp.ctrl;
    const int64_t s_after = cs.size + sp.n < sp.cap ? cs.size + sp.n : sp.cap;
    if (!push_handoff(mode, s_after >= B)) {  // block-uniform: no rows to compute
        if ((mode & PM_UPD_FIRST) && t == 0) st_out<true>(push_flag(sp), push_token(cs));
        return cs;
    }
    if (pushg && t == 0) st_out<true>(push_flag(sp), push_token(cs));  // block 1 read the control block
    const bool ip = t < B && push_of(sp, cs.pos, cs.size, cs.max_prio).covers(id);
    const unsigned long long m = __ballot(ip);
    if (ip) sm.plist[wv * 64 + __popcll(m & ((1ull << lane) - 1ull))] = t;
    if (lane == 0) sm.pcnt[wv] = __popcll(m);
    if (t < B) sm.sidx[t] = id;
    __syncthreads();
    PM_STAMP_ANY(51);
    float* pay = sp.hfeat + (size_t)B * 80;
    if (push2)
        push_rows_fwd2(sp, sm, wv, lane, pay, gtag);
    else
        push_rows_fwd(sp, sm.lw, sm.hf, sm.sidx, sm.plist, sm.pcnt, wv, lane,
                      [&](int j, bool nxt, int ln, const f32x16 (&c2)[2], const float (&qb)[3], const float (&qt)[3],
                          const float (&rb)[2]) { store_hfeat<true>(pay, j, nxt, ln, c2, qb, qt, rb); });
    PM_STAMP_ANY(52);
    if (pushg) return cs;  // block-uniform: the granules need no drain, the flag is out
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's payload stores are complete
    __syncthreads();
    PM_STAMP_ANY(53);
    if (t == 0) st_out<true>(push_flag(sp), push_token(cs));
    return cs;
}

// ---- the sum-tree refresh block (round 5): block 1, after the push rows, refreshes every tree node
// the update changes, so the learner's chain ends with its gradients, Adam and the head folds.
// The learner refreshed them itself in two dependent global round trips behind its own stores
// (scatter stores acknowledged -> the touched level-1 nodes' leaves loaded -> level-1 stores
// acknowledged -> the touched level-2 nodes' children loaded: ~8 us of its ~24 us). Block 1 knows
// which nodes those are from the sample indices and the control block alone, so it loads their
// inputs into LDS long before the update's priorities exist:
//   - entries: the B sampled indices, plus (LAST) the next push range's segment ends (its partial
//     level-1 / level-2 nodes); one level-1 slot per distinct sub-block and one level-2 slot per
//     distinct chunk (LDS hash sets), a chunk's 16 positions mapped to the level-1 slots inside it;
//   - LDS DMA: the 64 leaves of every level-1 slot, the 16 level-1 nodes of every level-2 slot;
//   - the learner publishes, as tagged 8-byte granules (hfeat's hand-off rows, MI355X_MICROARCH.md
//     handoff-1to1: one sc1 store each, no flag, no fence), each sample's new leaf prio ** alpha, the
//     next push's max priority and whether the update scattered; block 1 applies the scatter's
//     winners (the last duplicate of an index, as the learner's hash) to its LDS leaves, sums every
//     level-1 slot from LDS with the pending push substituted (per_quarter's order), then every
//     level-2 slot from LDS with the refreshed / pushed children substituted (per_chunk_sum's order),
//     and writes the wholly pushed nodes as the learner did (constants).
// Same functions, same orders: the tree stays bit-identical to a rebuild
// (test_sum_tree_incremental_equals_rebuild). The granule tag is an epoch word block 1 bumps at
// its end (both blocks read it at their start; the next launch's tag is new). A poll that never
// completes (bounded) sets ctrl.status bit 2 and leaves the tree alone. PONGMI_TR=0 (A/B) keeps the
// refresh in the learner.
constexpr int kTrSlots = PM_MAX_BATCH + 8;  // distinct level-1 / level-2 nodes: samples + <= 4 push edges (x8 rows)
constexpr int kTrHash = 1024;                // open-addressing sets keyed by node id
constexpr uint32_t kTrEmpty = 0xFFFFFFFFu;
constexpr int kTrPollMax = 20000;
constexpr int PM_CTRL_TREE_TIMEOUT = 4;
constexpr int PM_CTRL_TREE_REPAIRED = 8;  // a stale tree was rebuilt by pm_selfplay_repair_tree
struct TreeRefreshSmem {
    __attribute__((aligned(16))) float lf[kTrSlots][PER_SUB];   // leaves of every level-1 slot (LDS DMA)
    __attribute__((aligned(16))) double ls[kTrSlots][PER_FAN];  // level-1 nodes of every level-2 slot (LDS DMA)
    double subv[kTrSlots];                                     // refreshed level-1 nodes
    uint32_t subid[kTrSlots], chid[kTrSlots];
    int16_t cmap[kTrSlots][PER_FAN];  // level-2 slot x position -> level-1 slot inside it (-1: none)
    uint32_t skey[kTrHash];
    int sslot[kTrHash];
    uint32_t ckey[kTrHash];
    int cslot[kTrHash];
    uint32_t ikey[512];  // sampled index -> winning sample (the last duplicate, as the learner's hash)
    int iwin[512];
    uint32_t eidx[kTrSlots];  // entries: sampled indices, then the push edges
    int esub[kTrSlots];
    float leaf_new[PM_MAX_BATCH];
    float maxp_next;
    int scattered, ok, nsub, nch;
};
__device__ __forceinline__ uint64_t* tr_granules(const pm_selfplay& sp) {
    return reinterpret_cast<uint64_t*>(sp.hfeat + (size_t)(2 * sp.batch + 1) * 80);
}
__device__ __forceinline__ void tr_publish(const pm_selfplay& sp, int k, uint32_t v, uint32_t tag) {
    __hip_atomic_store(tr_granules(sp) + k, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int tr_hash(uint32_t k, int bits) { return (int)((k * 2654435761u) >> (32 - bits)); }
__device__ __forceinline__ int tr_insert(uint32_t* key, uint32_t k, int bits) {
    const int mask = (1 << bits) - 1;
    int h = tr_hash(k, bits);
    for (;;) {
        const uint32_t old = atomicCAS(&key[h], kTrEmpty, k);
        if (old == kTrEmpty || old == k) return h;
        h = (h + 1) & mask;
    }
}
__device__ __forceinline__ int tr_lookup(const uint32_t* key, uint32_t k, int bits) {  // -1: absent
    const int mask = (1 << bits) - 1;
    for (int h = tr_hash(k, bits);; h = (h + 1) & mask) {
        const uint32_t v = key[h];
        if (v == k) return h;
        if (v == kTrEmpty) return -1;
    }
}

__device__ __forceinline__ void tree_block(const pm_selfplay& sp, int mode, TreeRefreshSmem& sm, const pm_ctrl& cs,
                                           int poll_max) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, B = sp.batch;
    PM_STAMP_ANY(55);
    const PerTree tree = per_tree(sp.per_work, sp.cap);
    const uint32_t tag = __hip_atomic_load(tr_epoch(sp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const bool last = mode & PM_UPD_LAST;
    const int64_t s_after = cs.size + sp.n < sp.cap ? cs.size + sp.n : sp.cap;
    const int ns = s_after >= B ? B : 0;  // an update that cannot train scatters nothing
    const int64_t npos = (cs.pos + sp.n) % sp.cap;
    const int64_t end1 = npos + sp.n < sp.cap ? npos + sp.n : sp.cap;
    const int64_t end2 = npos + sp.n - sp.cap;  // > 0: the wrapped part [0, end2)
    const int nedge = last ? (end2 > 0 ? 4 : 2) : 0;
    const int ne = ns + nedge;
    for (int k = t; k < kTrHash; k += kLearn) { sm.skey[k] = kTrEmpty; sm.ckey[k] = kTrEmpty; }
    for (int k = t; k < 512; k += kLearn) { sm.ikey[k] = kTrEmpty; sm.iwin[k] = -1; }
    for (int k = t; k < kTrSlots * PER_FAN; k += kLearn) (&sm.cmap[0][0])[k] = -1;
    if (t == 0) { sm.nsub = 0; sm.nch = 0; sm.ok = 1; }
    if (t < ne) {
        const int64_t e = t < ns ? sp.idx[t] : (t - ns == 0 ? npos : t - ns == 1 ? end1 - 1 : t - ns == 2 ? 0 : end2 - 1);
        sm.eidx[t] = (uint32_t)e;
    }
    __syncthreads();
    if (t < ne) {
        tr_insert(sm.skey, sm.eidx[t] / PER_SUB, 10);
        if (t < ns) atomicMax(&sm.iwin[tr_insert(sm.ikey, sm.eidx[t], 9)], t);
    }
    __syncthreads();
    if (t < kTrHash && sm.skey[t] != kTrEmpty) {  // compact: one level-1 slot per distinct sub-block
        const int s = atomicAdd(&sm.nsub, 1);
        sm.sslot[t] = s;
        sm.subid[s] = sm.skey[t];
    }
    __syncthreads();
    const int nsub = sm.nsub;
    if (t < ne) sm.esub[t] = sm.sslot[tr_lookup(sm.skey, sm.eidx[t] / PER_SUB, 10)];
    if (t < nsub) tr_insert(sm.ckey, sm.subid[t] / PER_FAN, 10);
    __syncthreads();
    if (t < kTrHash && sm.ckey[t] != kTrEmpty) {
        const int c = atomicAdd(&sm.nch, 1);
        sm.cslot[t] = c;
        sm.chid[c] = sm.ckey[t];
    }
    __syncthreads();
    const int nch = sm.nch;
    if (t < nsub) sm.cmap[sm.cslot[tr_lookup(sm.ckey, sm.subid[t] / PER_FAN, 10)]][sm.subid[t] % PER_FAN] = (int16_t)t;
    // LDS DMA: wave instruction i moves 1 KB: level-1 slots 4i .. 4i + 3 (64 leaves each) / level-2
    // slots 8i .. 8i + 7 (16 nodes each); lanes past the count re-read the last slot
    for (int i = wv; 4 * i < nsub; i += kLearn / 64) {
        const int s = min(4 * i + (lane >> 4), nsub - 1);
        __builtin_amdgcn_global_load_lds((const void*)(tree.leaf + (size_t)sm.subid[s] * PER_SUB + 4 * (lane & 15)),
                                         (lds_void*)&sm.lf[4 * i][0], 16, 0, 0);
    }
    for (int i = wv; 8 * i < nch; i += kLearn / 64) {
        const int c = min(8 * i + (lane >> 3), nch - 1);
        __builtin_amdgcn_global_load_lds((const void*)(tree.sub + (size_t)sm.chid[c] * PER_FAN + 2 * (lane & 7)),
                                         (lds_void*)&sm.ls[8 * i][0], 16, 0, 0);
    }
    PM_STAMP_ANY(56);
    // the learner's granules: [0, B) each sample's new leaf, B the next push's max priority, B + 1 flags
    if (t < B + 2) {
        uint64_t g = 0;
        bool got = false;
        for (int it = 0; it < poll_max; ++it) {
            g = __hip_atomic_load(tr_granules(sp) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(g >> 32) == tag) { got = true; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!got) sm.ok = 0;
        const uint32_t v = (uint32_t)g;
        if (t < B) sm.leaf_new[t] = __uint_as_float(v);
        else if (t == B) sm.maxp_next = __uint_as_float(v);
        else sm.scattered = (int)(v & 1u);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS DMA landed
    __syncthreads();
    PM_STAMP_ANY(57);
    if (!sm.ok) {  // block-uniform: the learner's granules never came; the tree is left as it was
        if (t == 0) {
            atomicOr(&sp.ctrl->status, PM_CTRL_TREE_TIMEOUT);
            __hip_atomic_store(tr_epoch(sp), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (sm.scattered && t < ns && sm.iwin[tr_lookup(sm.ikey, sm.eidx[t], 9)] == t)
        sm.lf[sm.esub[t]][sm.eidx[t] % PER_SUB] = sm.leaf_new[t];  // the scatter's winner (:74-76)
    const float pval = last ? prio_pow(push_prio(s_after, sm.maxp_next), (float)sp.alpha) : 0.f;
    const PushRange next = last ? PushRange{npos, sp.n, sp.cap, pval} : PushRange{0, 0, sp.cap, 0.f};
    // the next push in 32-bit bounds (cap < 2^31): entries [q1lo, q1hi) and [0, q2hi); wholly pushed
    // level-1 nodes [p1lo, p1hi) and [0, p2hi) — what per_leaf / per_sub_pushed decide, without
    // their 64-bit ring arithmetic per element
    const int cap32 = (int)sp.cap;
    const int q1lo = last ? (int)npos : 0, q1hi = last ? (int)end1 : 0, q2hi = last && end2 > 0 ? (int)end2 : 0;
    const int p1lo = (q1lo + PER_SUB - 1) / PER_SUB, p1hi = q1hi / PER_SUB, p2hi = q2hi / PER_SUB;
    PM_STAMP_ANY(60);
    __syncthreads();
    // level 1: 4 lanes per slot (one quarter each, per_quarter's order), combined as per_combine
    for (int base = 0; base < 4 * nsub; base += kLearn) {
        const int k = base + t, s = min(k >> 2, nsub - 1), q = k & 3;
        const int lo = (int)sm.subid[s] * PER_SUB + 16 * q;
        float v[16];  // the quarter's 16 leaves, read before any select (no load under a branch)
        const float4* l4 = reinterpret_cast<const float4*>(&sm.lf[s][16 * q]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 x = l4[j];
            v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(v[j]));
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int e = lo + i;
            const bool pushed = (e >= q1lo && e < q1hi) || e < q2hi;
            const double x = (double)(pushed ? pval : v[i]);
            acc += e < cap32 ? x : 0.0;  // past cap: no leaf
        }
        const double node = per_combine(quad_f64<0>(acc), quad_f64<1>(acc), quad_f64<2>(acc), quad_f64<3>(acc));
        if (q == 0 && k < 4 * nsub) {
            sm.subv[s] = node;
            tree.sub[sm.subid[s]] = node;
        }
    }
    PM_STAMP_ANY(61);
    const double csub = per_sub_pushed_sum(next);
    {   // the wholly pushed level-1 nodes of the next push: one constant
        const int n1 = p1hi > p1lo ? p1hi - p1lo : 0;
        for (int k = t; k < n1 + p2hi; k += kLearn) tree.sub[k < n1 ? p1lo + k : k - n1] = csub;
    }
    PM_STAMP_ANY(62);
    __syncthreads();
    PM_STAMP_ANY(58);
    // level 2: every chunk slot from LDS, its refreshed / pushed children substituted (per_chunk_sum)
    const int nsub_tree = (int)tree.nsub;
    static_assert(PER_FAN == 16, "one DPP row per level-2 node");
    // one 16-lane DPP row per chunk slot: lane k of the row reads child k (consecutive LDS words; a
    // thread per slot reading its 16 children strided 128 B apart was a 32-way bank conflict per
    // read), and the row's lane 0 folds the 16 terms in per_chunk_sum's order (row_shl:k)
    for (int base = wv * 4; base < nch; base += kLearn / 16) {  // wave-uniform
        const int slot = min(base + (lane >> 4), nch - 1), k = lane & 15;
        const int m = sm.cmap[slot][k];
        const double old = sm.ls[slot][k];
        const double fresh = sm.subv[m >= 0 ? m : 0];
        const int sb = (int)sm.chid[slot] * PER_FAN + k;
        const bool pushed = (sb >= p1lo && sb < p1hi) || sb < p2hi;
        const double v = m >= 0 ? fresh : (pushed ? csub : old);
        const double x = sb < nsub_tree ? v : 0.0;
        double acc = 0.0;
        acc += x;
        acc += dpp_f64<0x101>(x); acc += dpp_f64<0x102>(x); acc += dpp_f64<0x103>(x);
        acc += dpp_f64<0x104>(x); acc += dpp_f64<0x105>(x); acc += dpp_f64<0x106>(x);
        acc += dpp_f64<0x107>(x); acc += dpp_f64<0x108>(x); acc += dpp_f64<0x109>(x);
        acc += dpp_f64<0x10A>(x); acc += dpp_f64<0x10B>(x); acc += dpp_f64<0x10C>(x);
        acc += dpp_f64<0x10D>(x); acc += dpp_f64<0x10E>(x); acc += dpp_f64<0x10F>(x);
        if (k == 0 && base + (lane >> 4) < nch) tree.chunk[sm.chid[slot]] = acc;
    }
    PM_STAMP_ANY(63);
    if (last) {  // the next push's other level-2 nodes: inside a segment (every boundary chunk holds an
                 // edge entry, so it has a slot), all 16 children wholly pushed: one constant
        double cc = 0.0;
#pragma unroll
        for (int k = 0; k < PER_FAN; ++k) cc += csub;
        const int c1lo = q1lo / PER_CHUNK, c1hi = (q1hi - 1) / PER_CHUNK + 1;
        const int c2hi = q2hi > 0 ? (q2hi - 1) / PER_CHUNK + 1 : 0;
        const int n1 = c1hi > c1lo ? c1hi - c1lo : 0;
        for (int k = t; k < n1 + c2hi; k += kLearn) {
            const int ch = k < n1 ? c1lo + k : k - n1;
            if (tr_lookup(sm.ckey, (uint32_t)ch, 10) < 0) tree.chunk[ch] = cc;
        }
    }
    PM_STAMP_ANY(59);
    if (t == 0) __hip_atomic_store(tr_epoch(sp), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct LearnSmem {
    union {
        float gpart[16][256];  // gradient phase: per-wave partial sums
    } u;
    __attribute__((aligned(16))) float Hs[PM_MAX_BATCH][64];  // ReLU(features(s)) of the batch (LDS DMA rows)
    // hfeat row floats 64..75 of each sample as three float4 planes (LDS DMA: lane t's 16 B at
    // base + 16 t): Q_B(s) 0..2 | r 3 | Q_B(s') 4..6 | action|done bits 7 | Q_T(s') 8..10
    __attribute__((aligned(16))) float qv4[3][PM_MAX_BATCH][4];
    float coef[PM_MAX_BATCH][4]; // dL/d(V, A0, A1, A2) per sample
    float eps_tr[pad256(260)];    // the update's noise (eps section layout)
    int64_t sidx[PM_MAX_BATCH];
    uint32_t hkey[512];          // open-addressing set of sampled indices (last-duplicate-wins)
    int hwin[512];
    float red[16][8];
    long long cnt[16][6];        // per-wave episode counters of the rollout (phase 0)
    long long ctot[6];           // their sums (phase 1)
    int plist[PM_MAX_BATCH];     // samples whose row is in this step's push range, per wave slot
    int pcnt[16];
    int void_upd;                // the push-row hand-off timed out: this update trains nothing
    float loss_out;              // the update's loss, committed to the control block at the kernel's end
    ApplySmem ap;
};

// train_step (:134-168) for the batch k_act_sp sampled, plus the episode counters of the rollout and
// the sum-tree refresh. Single workgroup of 1024 threads; global loads are issued up front.
union LearnShared {
    LearnSmem learn;
    ActSharedLearn act;
    PushFwdSmem pf;
    TreeRefreshSmem tr;
};
static_assert(sizeof(LearnShared) <= 160 * 1024, "k_learn LDS");

// Block 0 is the learner. Blocks 1.. (pm_selfplay_learn_act) run the opponents' greedy act for the
// NEXT vector step (train_iterative.py:240, side A) on the observations k_env just wrote: those
// actions depend on nothing the learner changes, and the learner occupies one CU, so they ride in
// this launch on otherwise idle CUs instead of lengthening the next k_act_sp. act_block is
// block-size agnostic: a 1024-thread block stages, compacts and tiles a 4x larger chunk.
// mode (PM_UPD_*): FIRST = the update that follows this step's k_env (its batch may hold rows of the
// push k_env just made, which this kernel computes; it sums the rollout's episode counters); LAST =
// the step's last update (refreshes the sum tree for the next push, commits the step). U = 1: both.
// Block 1 is push_fwd_block; the side-A act blocks (launches with side blocks) follow it.
// A side block's start delay: n x s_sleep 16 (1 024 clocks each; n = 8 ~ the former s_sleep 127)
__device__ __forceinline__ void side_nap(int n) {
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(16);
}

// PG: the push rows as tagged granules (tr bit 3; a separate instantiation: the flag consumer's
// branch beside the granule sweep made the compiler wait for every granule load in turn).
template <bool PG>
__global__ __launch_bounds__(kLearn) void k_learn(const pm_selfplay sp, int chunkA, int chunkP, int mode, int tr, int ftiles, int sleepf) {
    __shared__ __attribute__((aligned(16))) LearnShared shm;
    // tr: bit 0 the tree-refresh block, bit 1 push_rows_fwd2, bit 2 the apply's noise in phase 2
    const bool push2 = (tr & 2) != 0, late_noise = (tr & 4) != 0;
    const int tr_poll = (tr & 16) ? 0 : kTrPollMax;  // bit 4: test hook, the refresh block's poll times out at once
    constexpr bool pushg = PG;
    tr &= 1;
    if (blockIdx.x > 0) {
        if (blockIdx.x == 1) {
            const pm_ctrl cs = push_fwd_block(sp, mode, shm.pf, push2, pushg);
            if (tr) {
                __syncthreads();  // the push rows' LDS is reused
                tree_block(sp, mode, shm.tr, cs, tr_poll);
            }
            return;
        }
        const int sb = (int)blockIdx.x - 2;  // side block index
        PM_SIDE(0, sb, __builtin_amdgcn_s_memrealtime());
        const ActGrid g{sp.n, sp.n_pool + 1, chunkA, chunkP, 0};
        const int fb = sb - g.blocks();
        if (fb >= 0) {  // block-uniform: modelB's features for the next step (sp.featB)
            if (sleepf & 2) side_nap(sleepf >> 8);
            const int t0 = fb * ftiles;
            feat_tiles(shm.act.lw, sp.w_B, sp.obsB, sp.n, t0, min(t0 + ftiles, feat_ntiles(sp.n)), sp.featB);
            PM_STAMP_MAX(67);
            PM_SIDE(2, sb, __builtin_amdgcn_s_memrealtime());
            PM_SIDE(3, sb, 1ull | ((unsigned long long)(min(t0 + ftiles, feat_ntiles(sp.n)) - t0) << 16));
            return;
        }
        // the learner's load phase is latency-bound under the side blocks' staging bursts: the role
        // with slack starts after its loads are in flight (side_sleep: the feature blocks by default)
        if (sleepf & 1) side_nap(sleepf >> 8);
        PM_SIDE(1, sb, __builtin_amdgcn_s_memrealtime());
        const TileOut outA{sp.aA, nullptr, -1.0, 0, 0};
        act_block(shm.act, g, sp.w_opp, sp.n_pool > 0 ? sp.opp : nullptr, nullptr, sp.obsA, nullptr, outA, outA,
                  sb, sp.n_pool + 1 <= kListNets ? sp.opp_list : nullptr, sp.opp_cnt);
        PM_STAMP_MAX(66);
        PM_SIDE(2, sb, __builtin_amdgcn_s_memrealtime());
        PM_SIDE(3, sb, 0ull | ((unsigned long long)shm.act.count << 16));
        return;
    }
    LearnSmem& sm = shm.learn;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int B = sp.batch;
    pm_ctrl* c = sp.ctrl;
    PM_STAMP(0);
    const pm_ctrl cs = *c;  // loop counters as the step found them (only this kernel / k_adam commit)
    const PerTree tree = per_tree(sp.per_work, sp.cap);
    const bool first = mode & PM_UPD_FIRST, last = mode & PM_UPD_LAST;

    // ---- phase 0: every independent load, issued before any use. LDS-bound arrays go global ->
    // LDS directly (global_load_lds); register loads are issued unconditionally (gating them on the
    // control block, or storing each to LDS right away, costs one round trip per load).
    const int nbr = (sp.n + kBlock - 1) / kBlock;
    copy_lds_f32x4<260>(sp.learn_heads + 528, sm.eps_tr);
    if (sp.fuse_apply) load_apply_inputs(sp, sm.ap, false);
    long long part[6] = {0, 0, 0, 0, 0, 0};
    if (first && t < nbr) {
#pragma unroll
        for (int k = 0; k < 6; ++k) part[k] = sp.partials[(size_t)t * 8 + k];
    }
    const float wraw_l = t < B ? sp.isw[t] : 0.f;
    const int64_t id_l = t < B ? sp.idx[t] : 0;
    const float eps_v = t < 260 ? sp.learn_heads[528 + t] : 0.f;
    const uint32_t tr_tag = tr ? __hip_atomic_load(tr_epoch(sp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    // the rows k_env's forward blocks computed (hfeat [B][80]): sample t's Q block (floats 64..75,
    // phase 2's operands) global -> LDS (qv4 planes) here; its 64 features go global -> LDS below.
    // (Round 4 loaded it to registers: the compiler kept the float4[3] in scratch, a store that
    // waited for the load's round trip at the top of the phase.)
    if (t < PM_MAX_BATCH) {  // wave-uniform: waves 0..3
        const float4* src = reinterpret_cast<const float4*>(sp.hfeat + (size_t)min(t, B - 1) * 80 + 64);
#pragma unroll
        for (int k = 0; k < 3; ++k)
            __builtin_amdgcn_global_load_lds((const void*)(src + k), (lds_void*)&sm.qv4[k][wv * 64][0], 16, 0, 0);
    }
    for (int b = t + kLearn; first && b < nbr; b += kLearn)  // n > 256 * 1024 arenas only
#pragma unroll
        for (int k = 0; k < 6; ++k) part[k] += sp.partials[(size_t)b * 8 + k];
    const int64_t s_after = cs.size + sp.n < sp.cap ? cs.size + sp.n : sp.cap;
    bool train = s_after >= B;  // cleared (block-uniformly) if the push rows never arrive: a void update
    const bool train0 = train;  // as phase 0 found it (the apply's noise counter)
    bool act = train && t < B;
    if (t == 0) sm.void_upd = 0;
    // fused: the optimizer's scalar prologue on waves with slack in this load phase (they are not
    // on the dependent idx -> replay-row path of waves 0-3): the Adam bias corrections (two fp64
    // pow) on the last thread, both NoisyNet draws of the apply on the upper half of the block
    PM_STAMP(35);
    if (sp.fuse_apply && !late_noise) {
        if (t >= kLearn - 2) adam_const_lane(sp, cs.train_steps + 1, sm.ap, t - (kLearn - 2));
        gen_both_noises_on(sp, sm.ap, cs.step + 1, (uint64_t)(cs.train_steps + (train ? 1 : 0)) + 1, kLearn / 2);
    }
    PM_STAMP(34);
    if (train && t < 260) sp.paramsB[PM_QNET_EPS_OFF + t] = eps_v;  // reset_noise leaves it in modelB
    const float wraw = act ? wraw_l : 0.f;
    const int64_t id = act ? id_l : 0;
    for (int k = t; k < 512; k += kLearn) { sm.hkey[k] = kHashEmpty; sm.hwin[k] = -1; }
    if (act) sm.sidx[t] = id;
    {   // samples whose replay row k_env was writing: computed here (phase 1)
        const bool ip = first && act && push_of(sp, cs.pos, cs.size, cs.max_prio).covers(id);
        const unsigned long long m = __ballot(ip);
        if (ip) sm.plist[wv * 64 + __popcll(m & ((1ull << lane) - 1ull))] = t;
        if (lane == 0) sm.pcnt[wv] = __popcll(m);
    }
    PM_STAMP(16);  // (NOWAIT build: wave 0 had idx and the control block)
#if defined(PM_DIAG) && !defined(PM_DIAG_NOWAIT)
    PM_STAMP(30);
    asm volatile("" ::"v"(wraw_l), "v"((int)id_l));
    PM_STAMP(31);
    PM_STAMP(32);
    PM_STAMP(33);
#endif
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const long long s = wave_sum(part[k]);
        if (lane == 0) sm.cnt[wv][k] = s;
    }
    PM_STAMP(17);  // (NOWAIT: the partials)
    {
        const float m = wave_max(wraw);
        if (lane == 0) sm.red[wv][0] = m;
    }
    PM_STAMP(18);  // (NOWAIT: isw)
    PM_STAMP_T(19, 960);  // the last wave reaches the DMA issue
    // ReLU(features(s)) of the batch: each hfeat row's 64 floats global -> LDS (4 rows per wave
    // instruction), issued after every register load of this phase so nothing here waits on them; the
    // first reader is phase 3 (drained before phase 2's barrier, or before the push-row copy)
    if (train)
        for (int ci = wv; 4 * ci < B; ci += kLearn / 64) {
            const int row = min(4 * ci + (lane >> 4), B - 1);
            __builtin_amdgcn_global_load_lds((const void*)(sp.hfeat + (size_t)row * 80 + 4 * (lane & 15)),
                                             (lds_void*)&sm.Hs[4 * ci][0], 16, 0, 0);
        }
#if defined(PM_DIAG) && !defined(PM_DIAG_NOWAIT)
    // (after the feature rows' DMA is issued, as in the product build: the stamps include it landing;
    // PM_DIAG_NOWAIT drops this wait, so the timeline's later phases run as in the product build)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // this wave's loads (incl. LDS DMA) landed
    PM_STAMP_T(40, 0); PM_STAMP_T(41, 256); PM_STAMP_T(42, 512); PM_STAMP_T(43, 960);
#endif
    __syncthreads();
    PM_STAMP(1);

    // ---- phase 1: counters; the batch forward on the matrix cores (one 32-row tile per wave)
    long long ep_fin = 0;
    bool waited = false;  // block-uniform: the push-row token was seen
    if (t < 6) {
        long long s = 0;
        for (int w = 0; w < 16; ++w) s += sm.cnt[w][t];
        sm.ctot[t] = s;  // read after the next barrier
    }
    if (sp.fuse_apply && first && !late_noise && t == kLearn - 1) {  // the per-episode epsilon decay (:261) beside the forward
        long long s = 0;                     // (same sum, same order as thread 0's ctot[0])
        for (int w = 0; w < 16; ++w) s += sm.cnt[w][0];
        sm.ap.eps_next = cs.epsilon * pow(sp.epsilon_decay, (double)(float)s);
        PM_STAMP_T(37, kLearn - 1);
    }
    if (train) {  // rows in the push range (s rows then s' rows)
        int pre[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < 4; ++w) pre[w + 1] = pre[w] + sm.pcnt[w];  // B <= 256: waves 0..3
        const int np = pre[4];
        if (np > 0 && push_handoff(mode, train)) {  // block-uniform: block 1 computes them
            waited = true;
            if constexpr (PG) {  // the granules: up to 4 per thread in flight, re-polled until their tags match
                const uint64_t* pg = push_granules(sp);
                const int tot = np * kPushGN;
                uint64_t g[4];
                int jf[4];
                auto issue = [&](int k0) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = k0 + u * kLearn;
                        g[u] = (uint64_t)tr_tag << 32;  // past the end: no load (reads as arrived)
                        jf[u] = 0;
                        if (k < tot) {
                            const int q = k / kPushGN, f = k - q * kPushGN;
                            const int w = q >= pre[3] ? 3 : q >= pre[2] ? 2 : q >= pre[1] ? 1 : 0;
                            const int pw = q >= pre[3] ? pre[3] : q >= pre[2] ? pre[2] : q >= pre[1] ? pre[1] : 0;
                            jf[u] = sm.plist[w * 64 + q - pw] * kPushGF + f;
                            g[u] = __hip_atomic_load(pg + jf[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                };
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the feature rows' DMA, before rows are overwritten
                issue(t);  // the first round trip rides under the barrier
                __syncthreads();
                PM_STAMP(54);
                for (int k0 = t; k0 < tot; k0 += 4 * kLearn) {
                    if (k0 != t) issue(k0);
                    for (int it = 0;; ++it) {
                        bool done = true;
#pragma unroll
                        for (int u = 0; u < 4; ++u) done &= (uint32_t)(g[u] >> 32) == tr_tag;
                        if (done) break;
                        if (it == kPushPollMax) {  // never came: this update trains nothing (status bit 0)
                            sm.void_upd = 1;
                            sp.ctrl->status = cs.status | PM_CTRL_PUSH_TIMEOUT;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if ((uint32_t)(g[u] >> 32) != tr_tag)
                                g[u] = __hip_atomic_load(pg + jf[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (k0 + u * kLearn >= tot) break;
                        const int j = jf[u] / kPushGF, f = jf[u] - j * kPushGF;
                        const float v = __uint_as_float((uint32_t)g[u]);
                        if (f < 64) sm.Hs[j][f] = v;
                        else sm.qv4[(f - 64) >> 2][j][f & 3] = v;
                    }
                }
                PM_STAMP_T(36, 0);
            } else {
            if (t == 0 && !push_wait(sp, cs)) sm.void_upd = 1;
            PM_STAMP_T(36, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the feature rows' DMA, before rows are overwritten
            __syncthreads();
            PM_STAMP(54);
            const float* pay = sp.hfeat + (size_t)B * 80;
            for (int k = t; k < np * 76; k += kLearn) {
                const int q = k / 76, f = k - q * 76;
                const int w = q >= pre[3] ? 3 : q >= pre[2] ? 2 : q >= pre[1] ? 1 : 0;
                const int j = sm.plist[w * 64 + q - pre[w]];
                const float v = __hip_atomic_load(pay + (size_t)j * 80 + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (f < 64) sm.Hs[j][f] = v;
                else sm.qv4[(f - 64) >> 2][j][f & 3] = v;
            }
            }
        }
    }
    float wmax = sm.red[0][0];
    for (int w = 1; w < 16; ++w) wmax = fmaxf(wmax, sm.red[w][0]);
    if (t < PM_MAX_BATCH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the qv4 DMA (waves 0..3)
    __syncthreads();
    PM_STAMP(2);
    if (sm.void_upd) train = act = false;  // block-uniform: the hand-off timed out
    ep_fin = sm.ctot[0];
    // the rollout bookkeeping (:245-249) is committed at the kernel's end (commit_counters): stored
    // here, wave 0's vmcnt(0) before phase 2's barrier waited for these stores' acknowledgements

    // ---- phase 2: double-DQN targets, loss, priorities, bias grads
    float lossp = 0.f, prio = 0.f;
    float cf[4] = {0.f, 0.f, 0.f, 0.f};
    int slot = 0;
    if (act) {
        const float4 v0 = *reinterpret_cast<const float4*>(sm.qv4[0][t]);
        const float4 v1 = *reinterpret_cast<const float4*>(sm.qv4[1][t]);
        const float4 v2 = *reinterpret_cast<const float4*>(sm.qv4[2][t]);
        const float rwd = v0.w;
        const int bits = __float_as_int(v1.w);
        const int a = bits & 0xff, dn = (bits >> 8) & 1;
        const float qs[3] = {v0.x, v0.y, v0.z};
        const float qn[3] = {v1.x, v1.y, v1.z};
        const float qt[3] = {v2.x, v2.y, v2.z};
        const float q = qs[a];                                            // modelB(s).gather(a)   (:152)
        const float nq = qt[argmax3(qn)];                                 // targetB(ns)[argmax modelB(ns)]
        const float tgt = rwd + (float)sp.gamma * nq * (dn ? 0.f : 1.f);  // r + gamma*nq*(~d)     (:156)
        const float diff = q - tgt;
        const float w = wraw / wmax;                                      // w /= w.max() (:72)
        lossp = w * (diff * diff);
        const float g = 2.f * w * diff / (float)B;  // d mean(w (q-t)^2) / dq
        cf[0] = g;
#pragma unroll
        for (int k = 0; k < 3; ++k) cf[1 + k] = g * ((k == a ? 1.f : 0.f) - 1.f / 3.f);
        *reinterpret_cast<float4*>(sm.coef[t]) = make_float4(cf[0], cf[1], cf[2], cf[3]);
        prio = fabsf(diff) + 1e-6f;  // |err| + 1e-6 (:76)
        // update_priorities runs sequentially (:74-76): the last duplicate of an index wins
        const uint32_t key = (uint32_t)id;
        slot = (int)((key * 2654435761u) >> 23);
        for (;;) {
            const uint32_t old = atomicCAS(&sm.hkey[slot], kHashEmpty, key);
            if (old == kHashEmpty || old == key) break;
            slot = (slot + 1) & 511;
        }
        atomicMax(&sm.hwin[slot], t);
    } else if (sp.fuse_apply && late_noise && t >= kLearn / 2) {
        // the apply's scalar prologue on waves this phase leaves idle (late_noise; else in phase 0):
        // Adam's bias corrections (two fp64 pow) and both NoisyNet draws, consumed from phase 4 on.
        // (the train-step counter: `train` as phase 1 settled it, as the phase-0 draw would have it
        // when no hand-off timed out)
        // (and the per-episode epsilon decay (:261), one fp64 pow per lane in one instruction stream:
        // lane 61 decay^D, lanes 62 / 63 the Adam corrections)
        if (t >= kLearn - 3) {
            const int which = t - (kLearn - 2);  // -1: the epsilon decay
            long long s = 0;                     // (same sum, same order as thread 0's ctot[0])
            for (int w = 0; w < 16; ++w) s += sm.cnt[w][0];
            const double base = which < 0 ? sp.epsilon_decay : which ? sp.beta2 : sp.beta1;
            const double ex = which < 0 ? (double)(float)s : (double)(cs.train_steps + 1);
            const double p = pow(base, ex);
            if (which < 0) {
                if (first) sm.ap.eps_next = cs.epsilon * p;
            } else {
                const double bc = 1.0 - p;
                sm.ap.ak[which] = which ? (float)sqrt(bc) : (float)(sp.lr / bc);
            }
        }
        gen_both_noises_on(sp, sm.ap, cs.step + 1, (uint64_t)(cs.train_steps + (train0 ? 1 : 0)) + 1, kLearn / 2);
    }
    {
        const float s = wave_sum(lossp), mp = wave_max(prio);
#pragma unroll
        for (int k = 0; k < 4; ++k) cf[k] = wave_sum(cf[k]);
        if (lane == 0) {
            sm.red[wv][1] = s; sm.red[wv][2] = mp;
#pragma unroll
            for (int k = 0; k < 4; ++k) sm.red[wv][3 + k] = cf[k];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of the feature rows (phase 3 reads them)
    __syncthreads();
    PM_STAMP(3);

    // ---- phase 3: priority scatter; head gradients (16 waves x 16 samples, fixed-order combine)
    float mpx = 0.f;
    if (train) {
        mpx = sm.red[0][2];
        for (int w = 1; w < 16; ++w) mpx = fmaxf(mpx, sm.red[w][2]);
    }
    const float leaf_v = act ? prio_pow(prio, (float)sp.alpha) : 0.f;
    if (tr) {  // the tree-refresh block's inputs (tree_block): every sample's leaf, the next push's max
               // priority and whether this update scatters, as tagged granules
        if (t < B) tr_publish(sp, t, __float_as_uint(leaf_v), tr_tag);
        if (t == B) tr_publish(sp, B, __float_as_uint(train ? fmaxf(cs.max_prio, mpx) : cs.max_prio), tr_tag);
        if (t == B + 1) tr_publish(sp, B + 1, train ? 1u : 0u, tr_tag);
    }
    if (train) {
        if (act && sm.hwin[slot] == t) {
            sp.prios[id] = prio;
            tree.leaf[id] = leaf_v;
            if (prio != prio) atomicOr(&sp.ctrl->status, PM_CTRL_NAN_PRIO);
        }
        if (t == 0) {
            float l = 0.f;
            for (int w = 0; w < 16; ++w) l += sm.red[w][1];
            sm.loss_out = l / (float)B;  // committed at the kernel's end, with the counters
        }
        const int col = t & 63;
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        const int j0 = wv * 16, j1 = min(j0 + 16, B);
        for (int j = j0; j < j1; ++j) {
            const float4 k4 = *reinterpret_cast<const float4*>(sm.coef[j]);
            const float h = sm.Hs[j][col];
            g[0] = fmaf(k4.x, h, g[0]);
            g[1] = fmaf(k4.y, h, g[1]);
            g[2] = fmaf(k4.z, h, g[2]);
            g[3] = fmaf(k4.w, h, g[3]);
        }
        // lw / hf are dead: the forward finished before the last barrier
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.u.gpart[wv][r * 64 + col] = g[r];
    }
    const float max_prio_next = train ? fmaxf(cs.max_prio, mpx) : cs.max_prio;
    if (!tr) __threadfence_block();  // phase 4 re-reads the scattered leaves (this workgroup: no L2 writeback)
    __syncthreads();
    PM_STAMP(4);

    // ---- phase 4: gradients out; sum tree: sub-blocks of the scatter and of the next push range
    // not the last update: no pending push (empty range: refreshed nodes are plain sums of the leaves)
    const PushRange next = last ? push_of(sp, (cs.pos + sp.n) % sp.cap, s_after, max_prio_next)
                                : PushRange{0, 0, sp.cap, 0.f};
    if (train) {
        if (t < 256) {  // dL/dW_mu = sum_j coef_j h_j; dL/dW_sigma = dL/dW_mu * eps (the update's noise)
            float g = 0.f;
#pragma unroll
            for (int w = 0; w < 16; ++w) g += sm.u.gpart[w][t];
            const int row = t >> 6, col = t & 63;
            float* gs = sm.ap.g;
            const int a = row - 1;  // fc_V.weight_mu / _sigma, or fc_A.weight_mu / _sigma (row a)
            const int kmu = row == 0 ? col : 130 + a * 64 + col, ksg = row == 0 ? 65 + col : 325 + a * 64 + col;
            const float gsg = g * sm.eps_tr[row == 0 ? P_VWEP - PM_QNET_EPS_OFF + col
                                                     : P_AWEP - PM_QNET_EPS_OFF + a * 64 + col];
            gs[kmu] = g;
            gs[ksg] = gsg;
            if (sp.fuse_apply) {  // the optimizer step on the two parameters this thread owns
                adam_one(sp, sm.ap, kmu, g);
                adam_one(sp, sm.ap, ksg, gsg);
            }
        } else if (t < 260) {  // dL/db_mu = sum_j coef_j
            const int k = t - 256;
            float g = 0.f;
            for (int w = 0; w < 16; ++w) g += sm.red[w][3 + k];
            float* gs = sm.ap.g;
            // fc_V.bias_mu / _sigma, or fc_A.bias_mu / _sigma (k - 1)
            const int kmu = k == 0 ? 64 : 322 + k - 1, ksg = k == 0 ? 129 : 517 + k - 1;
            const float gsg = g * sm.eps_tr[k == 0 ? P_VBEP - PM_QNET_EPS_OFF : P_ABEP - PM_QNET_EPS_OFF + k - 1];
            gs[kmu] = g;
            gs[ksg] = gsg;
            if (sp.fuse_apply) {
                adam_one(sp, sm.ap, kmu, g);
                adam_one(sp, sm.ap, ksg, gsg);
            }
        }
        PM_STAMP(8); PM_STAMP_T(9, 960);
        if (!tr) {  // level-1 nodes of the scatter: 4 lanes per sampled index (duplicates recompute the
                    // same node from the same leaves: identical values)
            const int j = min(t >> 2, B - 1);
            const int64_t sb = sm.sidx[j] / PER_SUB;
            const double v = per_sub_sum4(tree.leaf, sb, next);
            if ((t & 3) == 0) tree.sub[sb] = v;
        }
        PM_STAMP(10); PM_STAMP_T(11, 960);
    } else {
        for (int k = t; k < kGradN; k += kLearn) sm.ap.g[k] = 0.f;
    }
    if (t == 0) { sm.ap.g[kGradN] = (float)ep_fin; sm.ap.g[kGradN + 1] = train ? 1.f : 0.f; }
    if (!tr) {  // level-1 nodes of the next push: wholly pushed ones are one constant; the <= 4 partially
                // pushed ones at the segment ends are summed from the leaves by 4 lanes of wave 0 each
        const RingNodes rn = ring_nodes(next, PER_SUB);
        const double csub = per_sub_pushed_sum(next);
        for (int64_t k = t; k < rn.count(); k += kLearn) {
            const int64_t sb = rn.at(k);
            if (per_sub_pushed(sb, next)) tree.sub[sb] = csub;
        }
        PM_STAMP(12); PM_STAMP_T(13, 960);
        if (wv == 0) {
            const int g = lane >> 2;
            const bool ok = g < 4 && (g < 2 ? rn.na : rn.nb) > 0;
            const int64_t sb = !ok ? 0 : g == 0 ? rn.a0 : g == 1 ? rn.a0 + rn.na - 1 : g == 2 ? 0 : rn.nb - 1;
            const double v = per_sub_sum4(tree.leaf, sb, next);
            if (ok && (lane & 3) == 0 && !per_sub_pushed(sb, next)) tree.sub[sb] = v;
        }
    }
    PM_STAMP(14); PM_STAMP_T(15, 960);
    if (!tr) __threadfence_block();  // phase 5 re-reads the level-1 nodes (this workgroup: no L2 writeback)
    __syncthreads();
    PM_STAMP(5);
    for (int k = t; k < kGradN + 2; k += kLearn) sp.grad[k] = sm.ap.g[k];
    // ---- phase 5: level-2 nodes over the refreshed sub-blocks; beside them (fused) the target sync
    // and the three head folds of derive_weights, which run on threads 256.. (level 2's are < 256)
    if (!tr && act && sm.hwin[slot] == t) {
        const int64_t ch = id / PER_CHUNK;
        tree.chunk[ch] = per_chunk_sum(tree, ch);
    }
    if (!tr) {
        const RingNodes rn = ring_nodes(next, PER_CHUNK);
        for (int64_t k = t; k < rn.count(); k += kLearn) {
            const int64_t ch = rn.at(k);
            tree.chunk[ch] = per_chunk_sum(tree, ch);
        }
    }
    PM_STAMP(6);
    if (sp.fuse_apply && first && !waited) {  // block 1 read the control block before this launch commits it
        if (t == 0) push_wait(sp, cs);
        __syncthreads();
    }
    if (sp.fuse_apply) apply_finish(sp, sm.ap, cs, mode);  // unsharded: Adam ran with the gradients (phase 4)
    if (t == 0) {  // the counters, last: no store of theirs sits in front of a phase's vmcnt(0) wait
        if (first) {  // rollout bookkeeping (:245-249)
            c->ep_step = ep_fin;
            c->episodes = cs.episodes + ep_fin;
            c->ep_A = cs.ep_A + sm.ctot[1]; c->win_A = cs.win_A + sm.ctot[2];
            c->ep_P = cs.ep_P + sm.ctot[3]; c->win_P = cs.win_P + sm.ctot[4];
            c->reward_B = cs.reward_B + (double)sm.ctot[5];
        }
        if (train) {
            c->last_loss = sm.loss_out;
            c->max_prio = max_prio_next;  // n > batch pushes of max_prio survive the scatter
        }
    }
    PM_STAMP(7);
}

// ------------------------------------------------------------------------------------ Adam + commit
// The scalar prologue (both noises, the bias-correction and epsilon-decay pows) runs while the
// loads are in flight: every thread reads the all-reduced updated flag and episode count itself.
__global__ __launch_bounds__(kLearn) void k_adam(const pm_selfplay sp, int mode) {
    __shared__ ApplySmem sm;
    const int t = threadIdx.x;
    const pm_ctrl cs = *sp.ctrl;
    load_apply_inputs(sp, sm, true);
    const float D = sp.grad[kGradN], upd = sp.grad[kGradN + 1];  // finished episodes | updated flag (all shards)
    const int64_t ts = cs.train_steps + (upd > 0.5f ? 1 : 0);
    gen_both_noises_on(sp, sm, cs.step + 1, (uint64_t)ts + 1, kLearn / 2);
    if (t >= kLearn - 2) adam_const_lane(sp, cs.train_steps + 1, sm, t - (kLearn - 2));
    if (t == kLearn / 2 - 1) sm.eps_next = cs.epsilon * pow(sp.epsilon_decay, (double)D);  // as apply_update's D
    __syncthreads();
    apply_adam(sp, sm);
    __syncthreads();
    apply_finish(sp, sm, cs, mode);
}

// pm_selfplay_prepare: features + acting weights of the current step + next update's heads
__global__ __launch_bounds__(kLearn) void k_prepare(const pm_selfplay sp) {
    __shared__ ApplySmem sm;
    write_feature_frags(sp.paramsB, sp.w_B);
    load_apply_inputs(sp, sm, false);
    gen_both_noises(sp, sm, sp.ctrl->step, (uint64_t)sp.ctrl->train_steps + 1);
    __syncthreads();
    derive_weights(sp, sm);
}

// ------------------------------------------------------------------------------------ U > 1 updates
// Updates 1..U-1 of a vector step: the PER sample over the replay as this step's push left it (one
// wave per sample), then the batch forward of every row (no pending push: k_env's forward blocks'
// job, on their own launch).
__global__ __launch_bounds__(256) void k_resample(const pm_selfplay sp) {
    __shared__ PerSampleSmem sm;
    sample_block(sp, (int)blockIdx.x, false, sm);
}
__global__ __launch_bounds__(kBlock) void k_batch_fwd(const pm_selfplay sp) { env_fwd_block(sp, (int)blockIdx.x, false); }

// pm_selfplay_commit, pass 1: max(prios[0, size)) (memory.push: prios.max(), :57) as float bits into
// ctrl->max_bits (priorities are > 0, so the int order of the bits is the float order).
constexpr int kMaxBlocks = 512;
__global__ __launch_bounds__(256) void k_prio_max(const pm_selfplay sp) {
    __shared__ float red[4];
    const pm_ctrl* c = sp.ctrl;
    const int64_t s = c->size + sp.n;
    const int64_t size = s < sp.cap ? s : sp.cap;
    const int64_t n4 = size / 4;
    const float4* p4 = reinterpret_cast<const float4*>(sp.prios);
    float m = 0.f;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += (int64_t)gridDim.x * 256) {
        const float4 v = p4[k];
        m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    if (blockIdx.x == 0 && threadIdx.x < size - 4 * n4) m = fmaxf(m, sp.prios[4 * n4 + threadIdx.x]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        atomicMax(&sp.ctrl->max_bits, __float_as_int(m));
    }
}

// pm_selfplay_commit, pass 2 (one workgroup): max_prio = that maximum; the sum tree's level-1 then
// level-2 nodes over the next push range with the push substituted (as k_learn's LAST update does);
// pos / size / step advance.
__global__ __launch_bounds__(kLearn) void k_commit(const pm_selfplay sp) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    pm_ctrl* c = sp.ctrl;
    const pm_ctrl cs = *c;
    const PerTree tree = per_tree(sp.per_work, sp.cap);
    const int64_t s = cs.size + sp.n;
    const int64_t s_after = s < sp.cap ? s : sp.cap;
    const float mp = __int_as_float(cs.max_bits);
    const PushRange next = push_of(sp, (cs.pos + sp.n) % sp.cap, s_after, mp);
    {
        const RingNodes rn = ring_nodes(next, PER_SUB);
        const double csub = per_sub_pushed_sum(next);
        for (int64_t k = t; k < rn.count(); k += kLearn) {
            const int64_t sb = rn.at(k);
            if (per_sub_pushed(sb, next)) tree.sub[sb] = csub;
        }
        if (wv == 0) {  // the <= 4 partially pushed nodes at the segment ends, 4 lanes each
            const int g = lane >> 2;
            const bool ok = g < 4 && (g < 2 ? rn.na : rn.nb) > 0;
            const int64_t sb = !ok ? 0 : g == 0 ? rn.a0 : g == 1 ? rn.a0 + rn.na - 1 : g == 2 ? 0 : rn.nb - 1;
            const double v = per_sub_sum4(tree.leaf, sb, next);
            if (ok && (lane & 3) == 0 && !per_sub_pushed(sb, next)) tree.sub[sb] = v;
        }
    }
    __threadfence_block();
    __syncthreads();
    {
        const RingNodes rn = ring_nodes(next, PER_CHUNK);
        for (int64_t k = t; k < rn.count(); k += kLearn) {
            const int64_t ch = rn.at(k);
            tree.chunk[ch] = per_chunk_sum(tree, ch);
        }
    }
    if (t == 0) {
        c->max_prio = mp;
        c->max_bits = 0;
        c->pos = (cs.pos + sp.n) % sp.cap;
        c->size = s_after;
        c->step = cs.step + 1;
    }
}

// ------------------------------------------------------------------------------------ U > 1 in one launch
// k_learn_multi: updates 1..U-1 of a vector step (after update 0's k_learn, before pm_selfplay_commit)
// as ONE single-workgroup launch, instead of k_resample + k_batch_fwd + k_learn per update (three
// launches, two of them on other CUs, ~30 us per update). Bit-identical to that sequence: the same
// PER descent (the chunk-level prefix in per_round_prefix's order, per_group_find for levels 1 and
// 0), the same head chains as tile_heads, and k_learn's phases 2-5 and fused apply in the same
// arithmetic order. What makes one workgroup enough:
//   - the features are frozen (train_iterative.py:97), so the batch forward needs only the heads:
//     ReLU(features(s)) of every replay row is stored at push time (sp.frow, written by k_actenv from
//     featB), features(s') of row i is frow[(i + n) % cap] (the same arena's next push) or, for this
//     step's own push, featB; a done row's s' never enters the target (nq * (1 - done)), so the
//     post-reset features stand in for the terminal ones there;
//   - the sum tree's top level (<= 1024 chunk sums) lives in LDS for all the updates; tree reads go
//     around L1 (nontemporal loads), so the workgroup's own scatters and refreshes are always seen;
//   - head parameters, Adam moments, the update's noisy heads and the next noise stay in LDS; the
//     global copies are written as the sequence of launches would leave them.
constexpr int kMultiChunks = PER_ROUND;  // level-2 nodes kept in LDS (capacity <= 1 M entries)

struct MultiSmem {
    float Hs[PM_MAX_BATCH][68];   // ReLU(features(s)) of the batch (k_learn's Hs); 16-byte rows
    float qv[PM_MAX_BATCH][12];   // Q_B(s) 0..2 | r 3 | Q_B(s') 4..6 | action|done bits 7 | Q_T(s') 8..10
    float coef[PM_MAX_BATCH][4];
    float gpart[16][256];
    float hf[2][264];             // the update's modelB heads (fresh noise) | targetB heads, fragment order
    float eps_tr[pad256(260)];    // the update's noise (eps section layout)
    double chunk[kMultiChunks];   // level-2 nodes
    double incl[kMultiChunks];    // their inclusive prefix (per_round_prefix)
    double wsum[16];
    int64_t sidx[PM_MAX_BATCH];
    float sw[PM_MAX_BATCH];       // un-normalised IS weights
    uint32_t hkey[512];
    int hwin[512];
    float red[16][8];
    double total;
    double pa[PM_MAX_BATCH];      // the drawn leaf's value per sample (its IS weight's pow in a pass of its own)
    int64_t ts, frame;            // train_steps, frame_idx as the updates advance them
    float maxp, loss;
    ApplySmem ap;
    // the kernel's arguments, copied once: multi_update (not inlined) reads them through a reference,
    // which for the kernel-argument struct itself meant a private (scratch) copy read per use
    pm_selfplay sp;
};
static_assert(sizeof(MultiSmem) <= 160 * 1024, "k_learn_multi LDS");

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) { return __builtin_nontemporal_load(p); }
typedef float f32x4v __attribute__((ext_vector_type(4)));
// 16 consecutive floats [lo, lo + 16) around L1 (4 x 16-byte loads; scalar loads past cap read 0).
// 16-scalar-load sweeps of a 4-lane group per sample cost 15 us per level here (one request per lane
// and load), the 16-byte ones a tenth of that.
__device__ __forceinline__ void ld_nt16(const float* p, int64_t lo, int64_t cap, float (&v)[16]) {
    if (lo + 16 <= cap) {
        const f32x4v* p4 = reinterpret_cast<const f32x4v*>(p + lo);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4v x = __builtin_nontemporal_load(p4 + q);
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lo + i < cap ? ld_nt(p + lo + i) : 0.f;
    }
}

// per_quarter / per_sub_sum4 (no pending push) with loads around L1.
__device__ __forceinline__ double multi_quarter(const float* leaf, int64_t sb, int k, int64_t cap) {
    const int64_t lo = sb * PER_SUB + 16 * k;
    float v[16];
    ld_nt16(leaf, lo, cap, v);
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += lo + i < cap ? (double)v[i] : 0.0;
    return acc;
}
__device__ __forceinline__ double multi_sub_sum4(const float* leaf, int64_t sb, int64_t cap) {
    const int lane = threadIdx.x & 63;
    const double q = multi_quarter(leaf, sb, lane & 3, cap);
    return per_combine(quad_f64<0>(q), quad_f64<1>(q), quad_f64<2>(q), quad_f64<3>(q));
}
__device__ __forceinline__ double multi_chunk_sum(const PerTree& t, int64_t c) {
    typedef double f64x2v __attribute__((ext_vector_type(2)));
    double v[PER_FAN];
    if (c * PER_FAN + PER_FAN <= t.nsub) {  // sub is 256-byte aligned: 16-byte loads of the node's 16
        const f64x2v* p = reinterpret_cast<const f64x2v*>(t.sub + c * PER_FAN);
#pragma unroll
        for (int k = 0; k < PER_FAN / 2; ++k) {
            const f64x2v x = __builtin_nontemporal_load(p + k);
            v[2 * k] = x.x;
            v[2 * k + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < PER_FAN; ++k) v[k] = c * PER_FAN + k < t.nsub ? ld_nt(t.sub + c * PER_FAN + k) : 0.0;
    }
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < PER_FAN; ++k) acc += v[k];
    return acc;
}

// One lane half's share of tile_heads: the fmaf chains over this half's 32 units (32 tt + 8 q4 + 4 h
// + e, in tile_heads' (t, r) order with r = 4 q4 + e), x[16 tt + 4 q4 + e] = ReLU'd feature. The
// cross-half add and the rest follow in half_heads_finish (lanes t and t ^ 1 hold the two halves).
__device__ __forceinline__ void half_chains(const float* hf, int h, const float (&x)[32], float (&s)[4]) {
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    const float4* hw = reinterpret_cast<const float4*>(hf + h * 128);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const float4 w = hw[k];  // (t, r) = (k >> 4, k & 15): unit 32 t + rho(r) + 4 h
        v = fmaf(w.x, x[k], v);
        a0 = fmaf(w.y, x[k], a0);
        a1 = fmaf(w.z, x[k], a1);
        a2 = fmaf(w.w, x[k], a2);
    }
    s[0] = v; s[1] = a0; s[2] = a1; s[3] = a2;
}
// The same chains for two rows with one sweep of the weights (the sweep's LDS reads bound this phase).
__device__ __forceinline__ void half_chains2(const float* hf, int h, const float (&xa)[32], const float (&xb)[32],
                                             float (&sa)[4], float (&sb)[4]) {
    float v = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f, u = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
    const float4* hw = reinterpret_cast<const float4*>(hf + h * 128);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const float4 w = hw[k];
        v = fmaf(w.x, xa[k], v);
        a0 = fmaf(w.y, xa[k], a0);
        a1 = fmaf(w.z, xa[k], a1);
        a2 = fmaf(w.w, xa[k], a2);
        u = fmaf(w.x, xb[k], u);
        b0 = fmaf(w.y, xb[k], b0);
        b1 = fmaf(w.z, xb[k], b1);
        b2 = fmaf(w.w, xb[k], b2);
    }
    sa[0] = v; sa[1] = a0; sa[2] = a1; sa[3] = a2;
    sb[0] = u; sb[1] = b0; sb[2] = b1; sb[3] = b2;
}
__device__ __forceinline__ void half_heads_finish(const float* hf, const float (&s)[4], float (&q)[3]) {
    float v = s[0] + __shfl_xor(s[0], 1), a0 = s[1] + __shfl_xor(s[1], 1);  // v_h0 + v_h1 in either lane
    float a1 = s[2] + __shfl_xor(s[2], 1), a2 = s[3] + __shfl_xor(s[3], 1);
    v += hf[256];
    a0 += hf[257];
    a1 += hf[258];
    a2 += hf[259];
    const float mean = ((a0 + a1) + a2) / 3.0f;
    q[0] = v + (a0 - mean);
    q[1] = v + (a1 - mean);
    q[2] = v + (a2 - mean);
}

// Half h's 32 ReLU'd features of a replay row from frow (8 float4: units 32 tt + 8 q4 + 4 h + 0..3) ...
__device__ __forceinline__ void load_frow_half(const float* frow, int64_t slot, int h, float (&x)[32]) {
    const float4* p = reinterpret_cast<const float4*>(frow + slot * 64) + h;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 v = p[2 * k];
        x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
    }
}
// ... or of one arena from featB (feat_tiles' layout: tile a / 32, piece 4 tt + q4, lane half h,
// component e; pre-ReLU there).
__device__ __forceinline__ void load_featB_half(const float* featB, int a, int h, float (&x)[32]) {
    const float4* p = reinterpret_cast<const float4*>(featB) + (size_t)(a >> 5) * 8 * 64 + 32 * h + (a & 31);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 v = p[k * 64];
        x[4 * k] = relu(v.x); x[4 * k + 1] = relu(v.y); x[4 * k + 2] = relu(v.z); x[4 * k + 3] = relu(v.w);
    }
}

// per_group_find<16> over lv[k] = lo + k < size ? (double)f[k] : 0 with the leaves kept as floats.
__device__ __forceinline__ int group_find16f(const float (&f)[16], int64_t lo, int64_t size, double x, double& before,
                                             double& val) {
    const int lane = threadIdx.x & 63, q = lane & 3, g0 = lane & ~3;
    auto lv = [&](int e) { return lo + e < size ? (double)f[e] : 0.0; };
    double acc = 0.0;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc += lv(e);
    const double s0 = quad_f64<0>(acc), s1 = quad_f64<1>(acc), s2 = quad_f64<2>(acc);
    const double ex = q == 0 ? 0.0 : (q == 1 ? s0 : (q == 2 ? s0 + s1 : (s0 + s1) + s2));
    int hit = -1, nz = -1;
    double hb = 0.0, hv = 0.0, nb = 0.0, nv = 0.0, run = ex;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const double v = lv(e);
        if (hit < 0 && run + v > x) { hit = e; hb = run; hv = v; }
        if (v > 0.0) { nz = e; nb = run; nv = v; }
        run += v;
    }
    const unsigned gh = (unsigned)(__ballot(hit >= 0) >> g0) & 15u;
    const unsigned gn = (unsigned)(__ballot(nz >= 0) >> g0) & 15u;
    int src, k;
    if (gh) {
        src = __ffs(gh) - 1;
        k = hit;
    } else {
        src = gn ? 31 - __clz(gn) : 0;
        k = nz < 0 ? 0 : nz;
        hb = nz < 0 ? ex : nb;
        hv = nz < 0 ? 0.0 : nv;
    }
    const int kk = quad_sel_i32(k, src);
    before = quad_sel_f64(hb, src);
    val = quad_sel_f64(hv, src);
    return src * 16 + kk;
}

// The update's noise in eps-section layout from the FRESH fold's draws (what fold_heads_from writes
// to its eps_out), threads [0, 260).
__device__ __forceinline__ void noise_to_eps(const float* noise, float* eps) {
    const int k = threadIdx.x;
    if (k >= 260) return;
    const int row = k < 256 ? k >> 6 : k - 256, col = k & 63;
    const bool w = k < 256;
    float ep;
    int eo;
    if (row == 0) {
        ep = w ? noise[64] * noise[col] : noise[64];
        eo = w ? E_VWEP + col : E_VBEP;
    } else {
        const int a = row - 1;
        ep = w ? noise[129 + a] * noise[65 + col] : noise[129 + a];
        eo = w ? E_AWEP + a * 64 + col : E_ABEP + a;
    }
    eps[eo] = ep;
}

// One update of k_learn_multi. A function of its own (not inlined): inside the kernel's loop the
// compiler hoisted every loop-invariant address and kernel-argument load out of it and spilled them
// (~700 B of scratch per lane at the 128-VGPR cap of a 1024-thread workgroup). `sp` is the kernel's
// LDS copy (MultiSmem::sp): a reference to the kernel-argument struct itself made the compiler
// materialise it in scratch and read every field from there (720 -> 204 B of scratch per lane,
// 32.6 -> 34.3 M env-steps/s at U = 64, r5ai).
#ifndef PM_MULTI_INLINE
#define PM_MULTI_INLINE __noinline__
#endif
__device__ PM_MULTI_INLINE void multi_update(const pm_selfplay& sp, MultiSmem& sm, int64_t size, int64_t nb, int64_t c_pos,
                                          uint64_t c_step, bool final, bool early_pow) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, B = sp.batch;
    const PerTree tree = per_tree(sp.per_work, sp.cap);
    PM_STAMP(100);
    const int64_t ts = sm.ts, frame = sm.frame + 1;  // frame_idx += 1 before sampling (:136)
    for (int k = t; k < 512; k += kLearn) { sm.hkey[k] = kHashEmpty; sm.hwin[k] = -1; }
    PM_STAMP(119);
    // ---- PER sample (per_sample_block, no pending push): level 2 over the LDS chunk sums
    {
        double run[4] = {0.0, 0.0, 0.0, 0.0}, acc = 0.0, incl = 0.0;
        if (t < 256) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t ch = 4 * t + e;
                acc += ch < nb ? sm.chunk[ch] : 0.0;
                run[e] = acc;
            }
        }
        PM_STAMP(120);
        incl = wave_incl_scan(acc, lane);
        double excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0.0;
        if (lane == 63) sm.wsum[wv] = incl;
        PM_STAMP(121);
        __syncthreads();
        PM_STAMP(122);
        if (t < 256) {
            double wb = 0.0;
            for (int w = 0; w < wv; ++w) wb += sm.wsum[w];
            const double ex = wb + excl;
#pragma unroll
            for (int e = 0; e < 4; ++e) sm.incl[4 * t + e] = ex + run[e];
        }
        if (t == 0) sm.total = ((0.0 + sm.wsum[0]) + sm.wsum[1]) + sm.wsum[2] + sm.wsum[3];
        __syncthreads();
    }
    PM_STAMP(101);
    const double total = sm.total;
    {
        const int j = t >> 2, q = t & 3;
        const int n = (int)nb;
        double x = 0.0, before = 0.0;
        int64_t blk = 0;
        {
            const U4 r = philox64((uint32_t)j, TAG_PER, (uint64_t)frame, sp.seed_env);
            const double uu = j < B ? u53(r.x, r.y) : 0.0;
            x = uu * total;
            if (total > 0.0) {
                int lo = 0, hi = n;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sm.incl[mid] > x) hi = mid;
                    else lo = mid + 1;
                }
                if (lo < n) {
                    blk = lo;
                    before = lo ? sm.incl[lo - 1] : 0.0;
                } else {  // the last nonzero chunk: the first to reach the end value
                    int l2 = 0, h2 = n - 1;
                    while (l2 < h2) {
                        const int mid = (l2 + h2) >> 1;
                        if (sm.incl[mid] >= sm.incl[n - 1]) h2 = mid;
                        else l2 = mid + 1;
                    }
                    blk = l2;
                    before = l2 ? sm.incl[l2 - 1] : 0.0;
                }
            }
        }
        PM_STAMP(111);
        double sv[4];
        const int64_t s0 = blk * PER_FAN + 4 * q;
#pragma unroll
        for (int e = 0; e < 4; ++e) sv[e] = s0 + e < tree.nsub ? ld_nt(tree.sub + s0 + e) : 0.0;
        double b1, v1;
        const int64_t sb = blk * PER_FAN + per_group_find<4>(sv, x - before, b1, v1);
        PM_STAMP(112);
        float lf[16];
        const int64_t lo = sb * PER_SUB + 16 * q;
        ld_nt16(tree.leaf, lo, sp.cap, lf);
        double b0, pa;
        const int k = group_find16f(lf, lo, size, x - before - b1, b0, pa);
        PM_STAMP(113);
        // ---- the sample's three head evaluations on the same 4 lanes, each lane one sweep of one head
        // set's weights (those LDS reads bound this phase): lanes 0-1 (lane halves h) run Q_B(s) and
        // Q_B(s') on modelB's heads, lanes 2-3 Q_T(s') on targetB's. The row loads are issued as soon as
        // the descent has the index; lanes 0-1 keep the features of s for Hs, lane 1 loads the reward
        // and action|done bits, lane 0 forms the IS weight while the loads are in flight.
        const int64_t id = sb * PER_SUB + k;
        const int h = q & 1, set = q >> 1;
        float xs[32], xn[32];
        float rb[2] = {0.f, 0.f};
        {
            int64_t a = id - c_pos;
            if (a < 0) a += sp.cap;
            if (a < sp.n) {  // this step's push: s' = the observations featB holds
                load_featB_half(sp.featB, (int)a, h, xn);
            } else {
                int64_t nx = id + sp.n;
                if (nx >= sp.cap) nx -= sp.cap;
                load_frow_half(sp.frow, nx, h, xn);
            }
        }
        if (set == 0) {
            load_frow_half(sp.frow, id, h, xs);
            if (h) {
                const float* tr = sp.trans + id * PM_TRANS_F;
                rb[0] = tr[7];
                rb[1] = tr[15];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 32; ++e) xs[e] = xn[e];
        }
        // early_pow (PONGMI_MULTI_EARLYPOW): the sample's IS weight on its lane 0 here, while the row
        // loads are in flight, and the wave's max of them before the barrier below (instead of a pow
        // pass on the batch's waves after it, then a max, then a barrier)
        float wr = 0.f;
        if (early_pow && q == 0 && j < B) wr = (float)pow((double)size * (pa / total), -beta_of(sp, frame));
#ifdef PM_DIAG
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PM_STAMP(117);
#endif
        const float* hfs = sm.hf[set];
        float s1[4], s2[4], q1[3], q2[3];
        half_chains2(hfs, h, xs, xn, s1, s2);  // set 0: Q_B(s), Q_B(s'); set 1: Q_T(s') (twice)
        half_heads_finish(hfs, s1, q1);
        half_heads_finish(hfs, s2, q2);
        PM_STAMP(118);
        if (j < B) {
            if (set == 0) {
#pragma unroll
                for (int e = 0; e < 32; e += 4)  // units 32 tt + 8 q4 + 4 h + 0..3: one 16-byte store each
                    *reinterpret_cast<float4*>(&sm.Hs[j][32 * (e >> 4) + 8 * ((e >> 2) & 3) + 4 * h]) =
                        make_float4(xs[e], xs[e + 1], xs[e + 2], xs[e + 3]);
                if (h == 0) {
                    sm.qv[j][0] = q1[0]; sm.qv[j][1] = q1[1]; sm.qv[j][2] = q1[2];
                    sm.qv[j][4] = q2[0]; sm.qv[j][5] = q2[1]; sm.qv[j][6] = q2[2];
                    sm.sidx[j] = id;
                    sm.pa[j] = pa;
                    sm.sw[j] = wr;
                    if (final) sp.idx[j] = id;
                } else {
                    sm.qv[j][3] = rb[0];
                    sm.qv[j][7] = rb[1];
                }
            } else if (h == 0) {
                sm.qv[j][8] = q1[0]; sm.qv[j][9] = q1[1]; sm.qv[j][10] = q1[2];
            }
        }
        if (early_pow) {  // block-uniform
            const float m = wave_max(wr);
            if (lane == 0) sm.red[wv][0] = m;
        }
    }
    __syncthreads();
    PM_STAMP(102);
    // this update's noise is left in modelB's epsilon buffers by its phase 0 (reset_noise); the
    // target sync below copies it from there
    const bool act = t < B;
    // the IS weights (size * P(i))^-beta, one fp64 pow per lane on the batch's waves only (every
    // wave running it for its 16 samples cost ~3 us of VALU issue)
    float wraw;
    if (early_pow) {
        wraw = act ? sm.sw[t] : 0.f;
    } else {
        wraw = act ? (float)pow((double)size * (sm.pa[t] / total), -beta_of(sp, frame)) : 0.f;
        const float m = wave_max(wraw);
        if (lane == 0) sm.red[wv][0] = m;
        __syncthreads();
    }
    if (act && final) sp.isw[t] = wraw;
    const int64_t id = act ? sm.sidx[t] : 0;
    PM_STAMP(103);
    float wmax = sm.red[0][0];
    for (int w = 1; w < 16; ++w) wmax = fmaxf(wmax, sm.red[w][0]);
    // no barrier: the TD phase below writes sm.red[.][1..6], never the [.][0] just read
    PM_STAMP(104);
    // ---- k_learn phase 2: double-DQN targets, loss, priorities, bias grads
    float lossp = 0.f, prio = 0.f;
    float cf[4] = {0.f, 0.f, 0.f, 0.f};
    int slot = 0;
    if (act) {
        const float rwd = sm.qv[t][3];
        const int bits = __float_as_int(sm.qv[t][7]);
        const int a = bits & 0xff, dn = (bits >> 8) & 1;
        const float qs[3] = {sm.qv[t][0], sm.qv[t][1], sm.qv[t][2]};
        const float qn[3] = {sm.qv[t][4], sm.qv[t][5], sm.qv[t][6]};
        const float qt[3] = {sm.qv[t][8], sm.qv[t][9], sm.qv[t][10]};
        const float q = qs[a];
        const float nq = qt[argmax3(qn)];
        const float tgt = rwd + (float)sp.gamma * nq * (dn ? 0.f : 1.f);
        const float diff = q - tgt;
        const float w = wraw / wmax;
        lossp = w * (diff * diff);
        const float g = 2.f * w * diff / (float)B;
        cf[0] = g;
#pragma unroll
        for (int k = 0; k < 3; ++k) cf[1 + k] = g * ((k == a ? 1.f : 0.f) - 1.f / 3.f);
        *reinterpret_cast<float4*>(sm.coef[t]) = make_float4(cf[0], cf[1], cf[2], cf[3]);
        prio = fabsf(diff) + 1e-6f;
        const uint32_t key = (uint32_t)id;
        slot = (int)((key * 2654435761u) >> 23);
        for (;;) {
            const uint32_t old = atomicCAS(&sm.hkey[slot], kHashEmpty, key);
            if (old == kHashEmpty || old == key) break;
            slot = (slot + 1) & 511;
        }
        atomicMax(&sm.hwin[slot], t);
    } else if (t >= kLearn / 2) {  // the apply's scalar prologue on waves the TD phase leaves idle:
        if (t >= kLearn - 2) adam_const_lane(sp, ts + 1, sm.ap, t - (kLearn - 2));  // Adam's corrections
        gen_both_noises_on(sp, sm.ap, c_step + 1, (uint64_t)(ts + 1) + 1, kLearn / 2);  // both noises
    }
    {
        const float s = wave_sum(lossp), mp = wave_max(prio);
#pragma unroll
        for (int k = 0; k < 4; ++k) cf[k] = wave_sum(cf[k]);
        if (lane == 0) {
            sm.red[wv][1] = s; sm.red[wv][2] = mp;
#pragma unroll
            for (int k = 0; k < 4; ++k) sm.red[wv][3 + k] = cf[k];
        }
    }
    __syncthreads();
    PM_STAMP(105);
    // ---- phase 3: priority scatter; head gradient partials (16 waves x 16 samples)
    if (act && sm.hwin[slot] == t) {
        sp.prios[id] = prio;
        tree.leaf[id] = prio_pow(prio, (float)sp.alpha);
        if (prio != prio) atomicOr(&sp.ctrl->status, PM_CTRL_NAN_PRIO);
    }
    {
        float mpx = sm.red[0][2];
        for (int w = 1; w < 16; ++w) mpx = fmaxf(mpx, sm.red[w][2]);
        float l = 0.f;
        for (int w = 0; w < 16; ++w) l += sm.red[w][1];
        if (t == 0) {
            sm.loss = l / (float)B;
            sm.maxp = fmaxf(sm.maxp, mpx);
        }
        const int col = t & 63;
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        const int j0 = wv * 16, j1 = min(j0 + 16, B);
        for (int j = j0; j < j1; ++j) {
            const float4 k4 = *reinterpret_cast<const float4*>(sm.coef[j]);
            const float h = sm.Hs[j][col];
            g[0] = fmaf(k4.x, h, g[0]);
            g[1] = fmaf(k4.y, h, g[1]);
            g[2] = fmaf(k4.z, h, g[2]);
            g[3] = fmaf(k4.w, h, g[3]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.gpart[wv][r * 64 + col] = g[r];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the scatter's stores are in L2 before the
    __syncthreads();                                   // refresh's L1-bypassing loads
    PM_STAMP(106);
    // ---- phase 4: gradients + Adam on the thread that forms each; level-1 nodes of the scatter
    if (t < 256) {
        float g = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) g += sm.gpart[w][t];
        const int row = t >> 6, col = t & 63;
        float* gs = sm.ap.g;
        const int a = row - 1;
        const int kmu = row == 0 ? col : 130 + a * 64 + col, ksg = row == 0 ? 65 + col : 325 + a * 64 + col;
        const float gsg = g * sm.eps_tr[row == 0 ? P_VWEP - PM_QNET_EPS_OFF + col
                                                 : P_AWEP - PM_QNET_EPS_OFF + a * 64 + col];
        gs[kmu] = g;
        gs[ksg] = gsg;
        adam_one(sp, sm.ap, kmu, g, final);
        adam_one(sp, sm.ap, ksg, gsg, final);
    } else if (t < 260) {
        const int k = t - 256;
        float g = 0.f;
        for (int w = 0; w < 16; ++w) g += sm.red[w][3 + k];
        float* gs = sm.ap.g;
        const int kmu = k == 0 ? 64 : 322 + k - 1, ksg = k == 0 ? 129 : 517 + k - 1;
        const float gsg = g * sm.eps_tr[k == 0 ? P_VBEP - PM_QNET_EPS_OFF : P_ABEP - PM_QNET_EPS_OFF + k - 1];
        gs[kmu] = g;
        gs[ksg] = gsg;
        adam_one(sp, sm.ap, kmu, g, final);
        adam_one(sp, sm.ap, ksg, gsg, final);
    }
    PM_STAMP(115);
    {
        const int j = min(t >> 2, B - 1);
        const int64_t sb = sm.sidx[j] / PER_SUB;
        const double v = multi_sub_sum4(tree.leaf, sb, sp.cap);
        PM_STAMP(116);
        if ((t & 3) == 0) tree.sub[sb] = v;
    }
    if (t == 0) { sm.ap.g[kGradN] = 0.f; sm.ap.g[kGradN + 1] = 1.f; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // level-1 stores land before level 2 reads them
    __syncthreads();
    PM_STAMP(107);
    if (final)
        for (int k = t; k < kGradN + 2; k += kLearn) sp.grad[k] = sm.ap.g[k];
    // ---- phase 5: level-2 nodes of the scatter (global and the LDS copy)
    if (act && sm.hwin[slot] == t) {
        const int64_t ch = id / PER_CHUNK;
        const double v = multi_chunk_sum(tree, ch);
        tree.chunk[ch] = v;
        sm.chunk[ch] = v;
    }
    // ---- apply_finish (mode 0): target sync, next weights; counters at the end of the launch
    if (t == 0) { sm.ts = ts + 1; sm.frame = frame; }
    if ((ts + 1) % sp.target_update_interval == 0) {  // targetB.load_state_dict(modelB) (:166-168)
        for (int k = t; k < PM_QNET_NHEAD; k += kLearn) sm.ap.tmu[k] = sm.ap.hp[k];
        for (int k = t; k < PM_QNET_NP; k += kLearn) {
            const int h = k - PM_QNET_HEAD_OFF, e = k - PM_QNET_EPS_OFF;
            sp.paramsT[k] = (h >= 0 && h < PM_QNET_NHEAD) ? sm.ap.hp[h]
                            : (e >= 0 ? sm.eps_tr[e] : sp.paramsB[k]);  // eps: this update's noise
        }
        __syncthreads();
    }
    PM_STAMP(108);
    if (final) {
        derive_weights(sp, sm.ap);  // w_B, learn_heads (global), modelB's eps buffers <- the acting noise
        __syncthreads();
    } else {
        derive_weights_lds(sm.ap);
    }
    PM_STAMP(109);
    heads_to_frags(sm.ap.heads[1], sm.hf[0]);
    heads_to_frags(sm.ap.heads[2], sm.hf[1]);
    noise_to_eps(sm.ap.ntrain, sm.eps_tr);
    // no vmcnt(0) here: the next update's global reads (level-1 nodes, leaves) see stores that were
    // drained at phases 3 / 4; its LDS state is complete at this barrier
    __syncthreads();
    PM_STAMP(124);
}

__global__ __launch_bounds__(kLearn, 1) void k_learn_multi(const pm_selfplay sp, int updates, int mflags) {
    __shared__ __attribute__((aligned(16))) MultiSmem sm;
    const int t = threadIdx.x, B = sp.batch;
    const PerTree tree = per_tree(sp.per_work, sp.cap);
    pm_ctrl* c = sp.ctrl;
    const int64_t c_pos = c->pos, c_size = c->size;
    const uint64_t c_step = c->step;
    const int64_t s_all = c_size + sp.n;
    const int64_t size = s_all < sp.cap ? s_all : sp.cap;  // the replay as this step's push left it
    if (size < B) return;  // block-uniform: no update trains (each would only re-derive the same weights)
    const int64_t nb = (size + PER_CHUNK - 1) / PER_CHUNK;
    // ---- state into LDS
    for (int k = t; k < kMultiChunks; k += kLearn) sm.chunk[k] = k < tree.nchunk ? ld_nt(tree.chunk + k) : 0.0;
    for (int k = t; k < 2 * 264; k += kLearn) sm.hf[k / 264][k % 264] = sp.learn_heads[k];
    for (int k = t; k < 260; k += kLearn) sm.eps_tr[k] = sp.learn_heads[528 + k];
    load_apply_inputs(sp, sm.ap, false);
    if (t == 0) {  // loop-carried counters live in LDS (registers are the scarce resource here)
        sm.ts = c->train_steps;
        sm.frame = c->frame_idx;
        sm.maxp = c->max_prio;
        sm.loss = c->last_loss;
    }
    for (int k = t; k < (int)(sizeof(pm_selfplay) / 4); k += kLearn)
        reinterpret_cast<uint32_t*>(&sm.sp)[k] = reinterpret_cast<const uint32_t*>(&sp)[k];
    __syncthreads();

    for (int u = 1; u < updates; ++u) multi_update(sm.sp, sm, size, nb, c_pos, c_step, u == updates - 1, mflags & 1);
    if (t == 0) {
        c->train_steps = sm.ts;
        c->frame_idx = sm.frame;
        c->last_loss = sm.loss;
        c->max_prio = sm.maxp;
    }
}

namespace {
int check(const pm_selfplay* sp) {
    PM_REQUIRE(sp && sp->ctrl && sp->trans && sp->prios && sp->per_work && sp->idx && sp->isw && sp->grad &&
                   sp->partials && sp->hfeat && sp->w_opp && sp->paramsB && sp->paramsT && sp->w_B && sp->adam_m &&
                   sp->adam_v && sp->opp && sp->ep_reward,
               PM_E_ARG, "pm_selfplay: null buffer");
    PM_REQUIRE(sp->n > 0 && sp->batch >= 1 && sp->batch <= PM_MAX_BATCH && sp->n > sp->batch && sp->cap >= sp->n &&
                   sp->cap < 0xFFFFFFFFll,
               PM_E_SIZE, "pm_selfplay: n=%d batch=%d cap=%lld", sp->n, sp->batch, (long long)sp->cap);
    PM_REQUIRE(sp->n_pool >= 0 && sp->n_pool <= 4096 && sp->world >= 1, PM_E_SIZE, "pm_selfplay: n_pool/world");
    PM_REQUIRE(sp->obsA && sp->obsB && sp->aA && sp->aB && sp->learn_heads && sp->opp_list && sp->opp_cnt, PM_E_ARG,
               "pm_selfplay: null buffer");
    PM_REQUIRE(!sp->fuse_apply || sp->world == 1, PM_E_ARG, "pm_selfplay: fuse_apply needs world == 1");
    PM_REQUIRE(sp->chunk_A > 0 && sp->chunk_A <= kListMax && sp->chunk_P > 0 && sp->chunk_P <= kListMax, PM_E_SIZE,
               "pm_selfplay: chunk_A/chunk_P must be in [1, %d]", kListMax);
    PM_REQUIRE(((((uintptr_t)sp->w_opp) | ((uintptr_t)sp->w_B) | ((uintptr_t)sp->prios) | ((uintptr_t)sp->per_work) |
                 ((uintptr_t)sp->paramsB) | ((uintptr_t)sp->paramsT) | ((uintptr_t)sp->adam_m) | ((uintptr_t)sp->adam_v) |
                 ((uintptr_t)sp->learn_heads)) &
                15) == 0,
               PM_E_ARG, "pm_selfplay: w_opp / w_B / prios / per_work / paramsB / paramsT / adam_m / adam_v / "
                         "learn_heads must be 16-byte aligned");
    PM_REQUIRE(sp->env.speed_scale_every > 0 && sp->target_update_interval > 0 && sp->beta_frames > 0, PM_E_ARG,
               "pm_selfplay: zero interval");
    return PM_OK;
}
}  // namespace

// prepare: derived weights + a full rebuild of the PER sum tree (with the coming push substituted).
// Call after init and after any host-side change of parameters, priorities or counters.
extern "C" int pm_selfplay_prepare(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    hipLaunchKernelGGL(k_prepare, dim3(1), dim3(kLearn), 0, st, *sp);
    PM_LAUNCHED("k_prepare");
    return per_launch_build(sp->prios, sp->cap, (float)sp->alpha, sp->ctrl, sp->n, sp->per_work, st);
}

namespace {
__global__ void k_tree_repaired(pm_ctrl* c) {
    if (threadIdx.x == 0 && (c->status & PM_CTRL_TREE_TIMEOUT))
        c->status = (c->status & ~PM_CTRL_TREE_TIMEOUT) | PM_CTRL_TREE_REPAIRED;
}
}  // namespace

// After a tree-refresh timeout (ctrl.status bit 2: the sums disagree with the leaves the learner
// scattered): a full rebuild of the PER sum tree from prios + ctrl (the pending push substituted, as
// pm_selfplay_prepare), then status bit 2 -> bit 3. Nothing else is re-derived.
extern "C" int pm_selfplay_repair_tree(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    if ((rc = per_launch_build(sp->prios, sp->cap, (float)sp->alpha, sp->ctrl, sp->n, sp->per_work, st))) return rc;
    hipLaunchKernelGGL(k_tree_repaired, dim3(1), dim3(64), 0, st, sp->ctrl);
    PM_LAUNCHED("k_tree_repaired");
    return PM_OK;
}

extern "C" int pm_selfplay_init(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    hipLaunchKernelGGL(k_sp_init, dim3(pm_blocks(sp->n, kBlock)), dim3(kBlock), 0, st, *sp);
    PM_LAUNCHED("k_sp_init");
    return pm_selfplay_prepare(sp, stream);
}

namespace {
int launch_act(const pm_selfplay* sp, int part, hipStream_t st) {
    const ActGrid g{sp->n, sp->n_pool + 1, sp->chunk_A, sp->chunk_P, part == PM_ACT_A ? 0 : 1};
    const int nsb = part == PM_ACT_A ? 0 : (sp->batch + PER_BS - 1) / PER_BS;
    int blocks = part == PM_ACT_B ? nsb + g.nb() : nsb + g.blocks();
    if (part != PM_ACT_B && sp->featB) blocks += (feat_ntiles(sp->n) + kFeatTilesAct - 1) / kFeatTilesAct;
    hipLaunchKernelGGL(k_act_sp, dim3(blocks), dim3(kActBlock), 0, st, *sp, part);
    PM_LAUNCHED("k_act_sp");
    return PM_OK;
}

// The side-A act grid of k_learn's extra blocks (1024 threads: four act blocks' worth each).
// k_learn_multi's preconditions: features of every live replay row stored (frow_ready), the current
// observations' features in featB (the update-0 launch computes them), the fused apply, a sum tree
// whose top level fits LDS.
bool multi_ok(const pm_selfplay* sp) {
    return sp->frow && sp->frow_ready && sp->featB && sp->fuse_apply && sp->world == 1 &&
           (sp->cap + PER_CHUNK - 1) / PER_CHUNK <= kMultiChunks && ((uintptr_t)sp->frow & 15) == 0;
}

// k_learn's side blocks (launches with the next step's side-A act): one CU each (the launch's LDS), so
// they run in ONE round beside the learner only if they fit the CUs the learner and block 1 leave, and
// they end together only if their work is even. PONGMI_SIDE=1 (default) sizes them from the opponent
// draw's expected rows: each net's chunk (a multiple of 256 arenas, so the act reads the env kernel's
// lists) is expected to hold kSideRows rows (~15 full 32-row tiles for 16 waves), and the feature
// tiles are spread over the CUs left (>= 16 per block). At configs[2] (pool 8, ratio 0.33): 86 modelA
// blocks (768 arenas, ~515 rows), 48 pool blocks (11 776 arenas, ~486 rows), 114 feature blocks of 18
// tiles: 250 blocks. PONGMI_SIDE=0: the round-4 grid (4x the act kernel's chunks up to 4 096 arenas,
// 16 feature tiles: 64 + 128 + 128 side blocks, two rounds; measured r5m: modelA blocks of ~705 rows
// end 22 us after the learner starts, the second round's feature blocks 23.8 us, the learner ~19 us).
struct LearnGrid {
    ActGrid g;
    int ftiles;
};
constexpr int kSideRows = 480;
// Which side blocks start with a ~3.4 us s_sleep, so the learner's load phase is not queued behind
// their staging bursts (PONGMI_SIDE_SLEEP: bit 0 act blocks, bit 1 feature blocks). Default 2 since
// the one-round grid: the feature blocks have the slack (r5o, same box, two interleaved passes:
// 2 -> 1.79 / 1.81 G env-steps/s, 0 -> 1.81 / 1.77, 1 (round 4) -> 1.76 / 1.75, 3 -> 1.75 / 1.75).
// PONGMI_SIDE_NAP: the delay in units of 1 024 clocks (default 8, ~3.4 us), bits 8.. of the argument.
int side_sleep() {
    const char* e = getenv("PONGMI_SIDE_SLEEP");
    const char* n = getenv("PONGMI_SIDE_NAP");
    const int roles = e && *e ? atoi(e) : 2, nap = n && *n ? atoi(n) : 8;
    return (roles & 3) | (std::max(0, std::min(nap, 64)) << 8);
}
int side_mode() {
    static const int v = [] {
        const char* e = getenv("PONGMI_SIDE");
        return e && *e ? atoi(e) : 1;
    }();
    return v;
}
int device_cus() {
    static const int v = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus;
    }();
    return v;
}
int side_chunk(double p) {
    if (!(p > 0.0)) return kListMaxLearn;
    const double c = std::ceil(kSideRows / p / 256.0) * 256.0;
    return c >= kListMaxLearn ? kListMaxLearn : (c < 256.0 ? 256 : (int)c);
}
LearnGrid learn_grid(const pm_selfplay* sp) {
    const int ntiles = feat_ntiles(sp->n);
    if (side_mode() == 0)
        return LearnGrid{ActGrid{sp->n, sp->n_pool + 1, std::min(4 * sp->chunk_A, kListMax),
                                 std::min(4 * sp->chunk_P, kListMax), 0},
                         kFeatTilesLearn};
    const double pp = sp->n_pool > 0 ? sp->pool_ratio : 0.0;
    const ActGrid g{sp->n, sp->n_pool + 1, side_chunk(1.0 - pp), side_chunk(sp->n_pool > 0 ? pp / sp->n_pool : 0.0), 0};
    // the feature blocks take the CUs the act blocks leave; when (nearly) none are left (n well above
    // configs[2]'s 65 536: the act blocks alone fill the chip) they share the chip over the whole
    // device instead, so no block runs thousands of tiles in series
    const int left = device_cus() - 2 - g.blocks();
    const int slots = left >= 32 ? left : device_cus();
    int ft = (ntiles + slots - 1) / slots;
    ft = std::max(ft, kFeatTilesLearn);
    return LearnGrid{g, std::min(ft, std::max(ntiles, 1))};
}

// The sum-tree refresh in block 1 (tree_block) unless PONGMI_TR=0 (the learner's own refresh, A/B).
// Read per launch (a getenv per k_learn launch is host work beside the GPU's): the variants are
// bitwise equal (test_learner_variants_are_bitwise_identical switches them between launches).
int tree_refresh_block() {
    const int v = [] {
        const char* e = getenv("PONGMI_TR");
        const char* p = getenv("PONGMI_PUSH2");  // block 1's push rows on two waves per tile (default 1)
        const char* q = getenv("PONGMI_LATE_NOISE");  // the apply's noise / Adam constants in phase 2 (default 1)
        const char* g = getenv("PONGMI_PUSHG");  // push rows as tagged granules (default 1; needs TR and PUSH2)
        const int tr = e && *e ? (atoi(e) != 0) : 1, p2 = p && *p ? (atoi(p) != 0) : 1;
        const int pg = (g && *g ? (atoi(g) != 0) : 1) && tr && p2;
        const char* f = getenv("PONGMI_TR_FORCE_TIMEOUT");  // test hook: block 1's granule poll times out
        return tr | (p2 << 1) | ((q && *q ? (atoi(q) != 0) : 1) << 2) | (pg << 3) | ((f && *f && atoi(f) != 0) << 4);
    }();
    return v;
}

int launch_learn(const pm_selfplay* sp, bool with_act, hipStream_t st, int mode = PM_UPD_FIRST | PM_UPD_LAST) {
    const LearnGrid lg = learn_grid(sp);
    const ActGrid& g = lg.g;
    unsigned blocks = 2u + (with_act ? (unsigned)g.blocks() : 0u);  // learner, push-row block, side blocks
    if (with_act && sp->featB) blocks += (unsigned)((feat_ntiles(sp->n) + lg.ftiles - 1) / lg.ftiles);
    const int tr = tree_refresh_block();
    pm_launch(PM_TIMER_LEARN, (tr & 8) ? k_learn<true> : k_learn<false>, dim3(blocks), dim3(kLearn), st, *sp, g.chunk0,
              g.chunk1, mode, tr, lg.ftiles, side_sleep());
    PM_LAUNCHED("k_learn");
    return PM_OK;
}
}  // namespace

extern "C" int pm_selfplay_act(const pm_selfplay* sp, void* stream) {
    return pm_selfplay_act_part(sp, PM_ACT_ALL, stream);
}

extern "C" int pm_selfplay_act_part(const pm_selfplay* sp, int32_t part, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    PM_REQUIRE(part == PM_ACT_ALL || part == PM_ACT_B || part == PM_ACT_A, PM_E_ARG,
               "pm_selfplay_act_part: part=%d", part);
    return launch_act(sp, part, pm_stream(stream));
}

extern "C" int pm_selfplay_env(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    const unsigned nfwd = pm_blocks(2 * sp->batch, 128);  // batch rows not in the push range (env_fwd_block)
    hipLaunchKernelGGL(k_env, dim3(pm_blocks(sp->n, kBlock) + nfwd), dim3(kBlock), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_env");
    return PM_OK;
}

extern "C" int pm_selfplay_actenv(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    // PONGMI_SFB: samples per sampler block, 32 (split forward, default) or 64 (round-4 blocks)
    static const int sfb = [] {
        const char* e = getenv("PONGMI_SFB");
        return e && atoi(e) == 64 ? 64 : 32;
    }();
    const unsigned nsb = (unsigned)((sp->batch + sfb - 1) / sfb);
    if (sfb == 64)
        pm_launch(PM_TIMER_ACTENV, k_actenv<64>, dim3(nsb + pm_blocks(sp->n, kBlock)), dim3(kBlock), pm_stream(stream), *sp);
    else
        pm_launch(PM_TIMER_ACTENV, k_actenv<32>, dim3(nsb + pm_blocks(sp->n, kBlock)), dim3(kBlock), pm_stream(stream), *sp);
    PM_LAUNCHED("k_actenv");
    return PM_OK;
}

extern "C" int pm_selfplay_rollout(const pm_selfplay* sp, void* stream) {
    int rc = pm_selfplay_act(sp, stream);
    return rc ? rc : pm_selfplay_env(sp, stream);
}

extern "C" int pm_selfplay_learn(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    return rc ? rc : launch_learn(sp, false, pm_stream(stream));
}

extern "C" int pm_selfplay_learn_act(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    return rc ? rc : launch_learn(sp, true, pm_stream(stream));
}

extern "C" int pm_selfplay_apply(const pm_selfplay* sp, void* stream) {
    return pm_selfplay_apply_ex(sp, PM_UPD_FIRST | PM_UPD_LAST, stream);
}

extern "C" int pm_selfplay_apply_ex(const pm_selfplay* sp, int32_t mode, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    PM_REQUIRE(mode >= 0 && mode <= (PM_UPD_FIRST | PM_UPD_LAST), PM_E_ARG, "pm_selfplay_apply_ex: mode=%d", mode);
    if (sp->fuse_apply) return PM_OK;  // learn already applied (unsharded, fused)
    hipLaunchKernelGGL(k_adam, dim3(1), dim3(kLearn), 0, pm_stream(stream), *sp, (int)mode);
    PM_LAUNCHED("k_adam");
    return PM_OK;
}

extern "C" int pm_selfplay_learn_ex(const pm_selfplay* sp, int32_t mode, int32_t with_act, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    PM_REQUIRE(mode >= 0 && mode <= (PM_UPD_FIRST | PM_UPD_LAST), PM_E_ARG, "pm_selfplay_learn_ex: mode=%d", mode);
    return launch_learn(sp, with_act != 0, pm_stream(stream), (int)mode);
}

extern "C" int pm_selfplay_resample(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    hipLaunchKernelGGL(k_resample, dim3((sp->batch + PER_BS - 1) / PER_BS), dim3(256), 0, st, *sp);
    PM_LAUNCHED("k_resample");
    hipLaunchKernelGGL(k_batch_fwd, dim3(pm_blocks(2 * sp->batch, 128)), dim3(kBlock), 0, st, *sp);
    PM_LAUNCHED("k_batch_fwd");
    return PM_OK;
}

extern "C" int pm_selfplay_commit(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    const int64_t blocks = std::min<int64_t>(kMaxBlocks, std::max<int64_t>(1, (sp->cap + 4095) / 4096));
    hipLaunchKernelGGL(k_prio_max, dim3((unsigned)blocks), dim3(256), 0, st, *sp);
    PM_LAUNCHED("k_prio_max");
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(kLearn), 0, st, *sp);
    PM_LAUNCHED("k_commit");
    return PM_OK;
}

extern "C" int pm_selfplay_step_multi(const pm_selfplay* sp, int32_t updates, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    PM_REQUIRE(updates >= 1, PM_E_ARG, "pm_selfplay_step_multi: updates=%d", updates);
    PM_REQUIRE(sp->world == 1, PM_E_ARG, "pm_selfplay_step_multi: unsharded only (world=%d)", sp->world);
    if (updates == 1) return pm_selfplay_step_overlap(sp, stream);
    hipStream_t st = pm_stream(stream);
    if ((rc = pm_selfplay_actenv(sp, stream))) return rc;
    if ((rc = launch_learn(sp, true, st, PM_UPD_FIRST))) return rc;
    if ((rc = pm_selfplay_apply_ex(sp, PM_UPD_FIRST, stream))) return rc;
    if (multi_ok(sp)) {  // updates 1..U-1 in one single-workgroup launch
        const char* ep = getenv("PONGMI_MULTI_EARLYPOW");  // A/B, read per launch; bit-identical either way
        const int mflags = ep && *ep ? (atoi(ep) != 0) : 0;
        pm_launch(PM_TIMER_LEARN_MULTI, k_learn_multi, dim3(1), dim3(kLearn), st, *sp, (int)updates, mflags);
        PM_LAUNCHED("k_learn_multi");
        return pm_selfplay_commit(sp, stream);
    }
    for (int u = 1; u < updates; ++u) {
        if ((rc = pm_selfplay_resample(sp, stream))) return rc;
        if ((rc = launch_learn(sp, false, st, 0))) return rc;
        if ((rc = pm_selfplay_apply_ex(sp, 0, stream))) return rc;
    }
    return pm_selfplay_commit(sp, stream);
}

extern "C" int pm_selfplay_step(const pm_selfplay* sp, void* stream) {
    int rc = pm_selfplay_rollout(sp, stream);
    if (!rc) rc = pm_selfplay_learn(sp, stream);
    return rc ? rc : pm_selfplay_apply(sp, stream);
}

extern "C" int pm_selfplay_step_overlap(const pm_selfplay* sp, void* stream) {
    int rc = pm_selfplay_actenv(sp, stream);
    if (!rc) rc = pm_selfplay_learn_act(sp, stream);
    return rc ? rc : pm_selfplay_apply(sp, stream);
}

#ifdef PM_DIAG
extern "C" int pm_diag_read_side(uint64_t* out) {  // [4][1024]: k_learn side blocks (begin, after sleep, end, role | rows)
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_side), sizeof(uint64_t) * 4 * 1024);
}
extern "C" int pm_diag_read(uint64_t* out, int32_t n) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_buf), sizeof(uint64_t) * (n < 256 ? n : 256));
    return e == hipSuccess ? 0 : (int)e;
}
extern "C" int pm_diag_read_blk(uint64_t* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_blk), sizeof(uint64_t) * 8 * 4096);
}
extern "C" int pm_diag_read_env(uint64_t* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_diag_env), sizeof(uint64_t) * 8 * 1024);
}
extern "C" int pm_diag_clear(void) {
    static const unsigned long long z[256] = {0};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(pm_diag_buf), z, sizeof(z));
}
#endif
