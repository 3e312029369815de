// K7 — QNetRNN self-play: scripts/train_rnn_iterative.py's hot loop (:731-798) for n arenas.
//
// One vector step = one env step in every arena, on one stream:
//   pm_rnn_fold   modelB's NoisyLinear layers with fresh noise (select_action_for_model's
//                 reset_noise, :385), written back into modelB's epsilon buffers
//   pm_rnn_act    both players on the matrix cores, (h, c) carried per arena (K5)
//   k_rsp_env     env.step, SequenceReplayBuffer.push_step into the arena's transition ring,
//                 ep reward / length, next opponent + env.reset() for finished arenas (HBM-bound)
//   k_rsp_append  finished episodes of length >= T appended to the episode table in arena order
//                 (deque(maxlen=capacity).append, :114), counters, epsilon decay (:798)
//   k_rsp_sample  SequenceReplayBuffer.sample(64) (:118-173) into the DRQN batch, and the enable
//                 flag (len(memory) > batch * min_episodes_for_training_start, :768)
// then pm_drqn_update (K6). Transition rings are [depth][n] records of 64 B written by step
// (coalesced); an episode is (arena, first step, length), its steps read back from the ring.
#include <stdlib.h>

#include "pm_host.h"
#include "pm_mfma.h"

using namespace pm;

namespace {

constexpr int kBlock = 256;
static_assert(kBlock == kRowBlock, "row staging assumes kRowBlock-thread blocks");

__device__ __forceinline__ int draw_opponent(const pm_rnn_selfplay& sp, int i, uint32_t ns) {
    // use_pool_opponent = pool and random() < ratio; opponent = random.choice(pool) (:735-736)
    const U4 q = philox((uint32_t)i, TAG_OPP, ns, 0u, sp.seed_env);
    return (sp.n_pool > 0 && u53(q.x, q.y) < sp.pool_ratio) ? 1 + below(q.z, (uint32_t)sp.n_pool) : 0;
}

__global__ __launch_bounds__(kBlock) void k_rsp_init(const pm_rnn_selfplay sp) {
    __shared__ __attribute__((aligned(16))) float lds[kBlock][7];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0};
    if (i < sp.n) {
        const uint32_t ns = (uint32_t)sp.st.serves[i];
        sp.opp[i] = draw_opponent(sp, i, ns);
        Arena a;
        double vx, vy, spn;
        philox_serve(sp.env, (uint32_t)i, ns, sp.seed_env, vx, vy, spn);
        serve(a, vx, vy, spn);
        store_arena(sp.st, i, a);
        sp.st.serves[i] = (int32_t)ns + 1;
        sp.ep_reward[i] = 0.f;
        sp.ep_len[i] = 0;
        sp.ep_steps[i] = 0;
        sp.reset[i] = 1;  // init_hidden for both players (:744-746)
        observe(a, oA, oB);
    }
    {
        __shared__ OppListSmem ol;
        write_opp_lists(sp.n_pool + 1, sp.opp_list, sp.opp_cnt, ol, blockIdx.x, i, i < sp.n, i < sp.n ? sp.opp[i] : 0);
    }
    store_rows7(sp.obsA, lds, oA, i0, sp.n);
    store_rows7(sp.obsB, lds, oB, i0, sp.n);
}

__global__ __launch_bounds__(kBlock) void k_rsp_env(const pm_rnn_selfplay sp) {
    __shared__ __attribute__((aligned(16))) float lds[2][kBlock][7];
    __shared__ long long red[kBlock / 64][6];
    __shared__ int red_st[kBlock / 64];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    const bool valid = i < sp.n;
    const int ii = valid ? i : sp.n - 1;
    const uint64_t step = sp.ctrl->step;
    // serve counter first; the next opponent and serve are drawn while the state loads land
    const uint32_t ns = (uint32_t)__builtin_nontemporal_load(&sp.st.serves[ii]);
    __builtin_amdgcn_sched_barrier(0);
    Arena a = load_arena(sp.st, ii);
    const int aA = sp.aA[ii], aB = sp.aB[ii], o = sp.opp[ii];
    const int onext = draw_opponent(sp, ii, ns);
    double svx, svy, sspn;
    philox_serve(sp.env, (uint32_t)ii, ns, sp.seed_env, svx, svy, sspn);
    float oA[7], oB[7];
    observe(a, oA, oB);  // the observation the actions were chosen on
    float rA, rB;
    const int d = tick(sp.env, a, aA, aB, rA, rB);
    float nA[7], nB[7];
    observe(a, nA, nB);
    const float er = sp.ep_reward[ii] + rB;  // episode_reward_b += reward_B (:765)
    const int len = sp.ep_len[ii] + 1;       // the trajectory push_step is collecting (:107-110)
    const int steps = sp.ep_steps[ii] + 1;   // for step_in_episode in range(max_episode_steps) (:751)
    // the episode ends on done or at the step cut; the trajectory only on done (:111-116)
    const bool end = d || (sp.max_steps > 0 && steps >= sp.max_steps);
    const bool fin = valid && end;
    {   // per-block partials, no atomics: finished, vs-A, wins vs A, vs-pool, wins vs pool, reward
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const bool win = er > 0.f;  // win_flag = episode_reward_b > 0 (:783)
        const unsigned long long mf = __ballot(fin), mA = __ballot(fin && o == 0), mwA = __ballot(fin && o == 0 && win);
        const unsigned long long mP = __ballot(fin && o != 0), mwP = __ballot(fin && o != 0 && win);
        const int rs = wave_sum(fin ? (int)er : 0);
        if (lane == 0) {
            red[wv][0] = __popcll(mf); red[wv][1] = __popcll(mA); red[wv][2] = __popcll(mwA);
            red[wv][3] = __popcll(mP); red[wv][4] = __popcll(mwP); red[wv][5] = rs;
        }
    }
    int onew = o;
    if (valid) {
        // memory.push_step(obs_B, act_B, reward_B, next_obs_B, done) (:770, :107-110)
        float4* row = reinterpret_cast<float4*>(sp.trans + ((int64_t)(step % (uint64_t)sp.depth) * sp.n + i) * PM_TRANS_F);
        row[0] = make_float4(oB[0], oB[1], oB[2], oB[3]);
        row[1] = make_float4(oB[4], oB[5], oB[6], rB);
        row[2] = make_float4(nB[0], nB[1], nB[2], nB[3]);
        row[3] = make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8)));
        if (end) {  // episode over (done or cut): next opponent, env.reset() (:735-740)
            onew = onext;
            sp.opp[i] = onew;
            serve(a, svx, svy, sspn);
            sp.st.serves[i] = (int32_t)ns + 1;
            observe(a, nA, nB);
        }
        store_arena(sp.st, i, a);
        sp.ep_reward[i] = end ? 0.f : er;
        sp.ep_len[i] = d ? 0 : len;
        sp.ep_steps[i] = end ? 0 : steps;
        sp.reset[i] = (uint8_t)end;  // init_hidden for both players at the next episode (:744-746)
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) { lds[0][threadIdx.x][k] = nA[k]; lds[1][threadIdx.x][k] = nB[k]; }
    {   // episodes to store, ranked in arena order within the block -> the block's staging slots
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        // stored when len >= trace_length (:112-115) and short enough to stay in the ring (header)
        const bool st = valid && d && len >= sp.T && len <= sp.depth / 2;
        if (valid && d && len > sp.depth / 2) atomicOr(&sp.ctrl->status, 4);
        const unsigned long long m = __ballot(st);
        if (lane == 0) red_st[wv] = __popcll(m);
        __syncthreads();
        int rank = __popcll(m & ((1ull << lane) - 1ull));
        for (int w = 0; w < wv; ++w) rank += red_st[w];
        if (st) {
            int64_t* slot = sp.fin + 2 * ((int64_t)blockIdx.x * kBlock + rank);
            slot[0] = (int64_t)(uint32_t)i | ((int64_t)len << 32);
            slot[1] = (int64_t)step - len + 1;
        }
    }
    if (threadIdx.x < 7) {
        long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += threadIdx.x < 6 ? red[w][threadIdx.x] : red_st[w];
        sp.partials[(size_t)blockIdx.x * 8 + threadIdx.x] = t;
    }
    {   // the next act's per-block opponent lists
        __shared__ OppListSmem ol;
        write_opp_lists(sp.n_pool + 1, sp.opp_list, sp.opp_cnt, ol, blockIdx.x, i, valid, onew);
    }
    copy_rows7(sp.obsA, lds[0], i0, sp.n);  // staged before the ranking barrier
    copy_rows7(sp.obsB, lds[1], i0, sp.n);
}

constexpr int kAppend = 1024;  // one thread per env block: n <= kAppend * kBlock

// The env blocks' staged episodes appended to the table in arena order (block prefix sums), the
// bookkeeping partials summed, epsilon decayed once per finished episode, the step advanced.
__global__ __launch_bounds__(kAppend) void k_rsp_append(const pm_rnn_selfplay sp) {
    __shared__ int off[kAppend + 1];
    __shared__ long long wred[kAppend / 64][7];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    pm_rnn_ctrl* c = sp.ctrl;
    const int nblk = (sp.n + kBlock - 1) / kBlock;
    long long p[7] = {0, 0, 0, 0, 0, 0, 0};
    if (t < nblk) {
#pragma unroll
        for (int k = 0; k < 7; ++k) p[k] = sp.partials[(size_t)t * 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const long long v = wave_sum(p[k]);
        if (lane == 0) wred[wv][k] = v;
    }
    off[t + 1] = (int)p[6];  // stored episodes of env block t
    if (t == 0) off[0] = 0;
    __syncthreads();
    for (int s = 1; s <= kAppend; s <<= 1) {  // inclusive scan of off[1..kAppend]
        const int v = t + 1 > s ? off[t + 1 - s] : 0;
        __syncthreads();
        off[t + 1] += v;
        __syncthreads();
    }
    const int total = off[kAppend];
    const int64_t base = c->seq_count;
    for (int e = t; e < total; e += kAppend) {  // entry e: env block b with off[b] <= e < off[b + 1]
        int lo = 0, hi = kAppend;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (off[mid] <= e) lo = mid; else hi = mid;
        }
        const int64_t* src = sp.fin + 2 * ((int64_t)lo * kBlock + (e - off[lo]));
        const int64_t slot = (base + e) % sp.seq_cap;
        sp.seq_eps[2 * slot] = src[0];
        sp.seq_eps[2 * slot + 1] = src[1];
    }
    // the six counter sums, one thread each (one thread summing all 96 from LDS had its loads hoisted
    // into registers past the 128-VGPR cap: 324 B of scratch per lane)
    __shared__ long long tots[6];
    if (t < 6) {
        long long v = 0;
        for (int w = 0; w < kAppend / 64; ++w) v += wred[w][t];
        tots[t] = v;
    }
    __syncthreads();
    if (t == 0) {
        long long tot[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) tot[k] = tots[k];
        // deque(maxlen=seq_cap) keeps the newest seq_cap episodes; an episode that finished more than
        // depth / 2 steps ago also leaves (its steps are about to leave the ring): entries [0, E(s))
        // finished at or before step s, E(s) = seq_mark[s % depth] (header: ring safety)
        const uint64_t now = c->step;
        const int64_t count = base + total;
        sp.seq_mark[now % (uint64_t)sp.depth] = count;
        const int64_t h = sp.depth / 2;
        const int64_t by_cap = count > sp.seq_cap ? count - sp.seq_cap : 0;
        const int64_t by_age = (int64_t)now >= h + 1 ? sp.seq_mark[(now - h - 1) % (uint64_t)sp.depth] : 0;
        if (by_age > by_cap) c->status |= 2;
        c->seq_count = count;
        c->seq_size = count - (by_age > by_cap ? by_age : by_cap);
        c->episodes += tot[0];
        c->ep_A += tot[1]; c->win_A += tot[2]; c->ep_P += tot[3]; c->win_P += tot[4];
        c->reward_B += (double)tot[5];
        double eps = c->epsilon;
        for (long long q = 0; q < tot[0] && eps > sp.min_epsilon; ++q) {  // max(min_epsilon, eps * decay) per episode
            eps = eps * sp.epsilon_decay;
            if (eps < sp.min_epsilon) eps = sp.min_epsilon;
        }
        c->epsilon = eps;
        c->step = c->step + 1;
    }
}

struct SampleOut {
    float *obs, *next, *rew;
    int32_t* act;
    uint8_t* done;
    int B, T;
};

// u: the update of this vector step (0: the env call's draw; 1..U-1: pm_rnn_selfplay_sample).
__global__ __launch_bounds__(512) void k_rsp_sample(const pm_rnn_selfplay sp, SampleOut o, int u) {
    pm_rnn_ctrl* c = sp.ctrl;
    const int64_t size = c->seq_size;
    const bool en = size > sp.min_episodes && size > 0;
    if (threadIdx.x == 0) { *sp.enable = en; c->train = en; }
    if (!en) return;
    const uint64_t now = c->step;  // steps [0, now) written; slot s % depth holds the latest s
    const int64_t first = c->seq_count - size;
    for (int e = threadIdx.x; e < o.B * o.T; e += blockDim.x) {  // one (sequence, step) per thread
        const int b = e / o.T, tau = e % o.T;
        // np.random.choice(len(buffer), batch, replace=True), then randint(0, len - T + 1) (:131, :147)
        const U4 r = philox64((uint32_t)b, TAG_SEQ, now | ((uint64_t)u << 48), sp.seed_env);
        const int64_t j = below(r.x, (uint32_t)size);
        const int64_t slot = (first + j) % sp.seq_cap;
        const int64_t packed = sp.seq_eps[2 * slot];
        const int arena = (int)(packed & 0xffffffff), L = (int)(packed >> 32);
        const int64_t s = sp.seq_eps[2 * slot + 1] + below(r.y, (uint32_t)(L - o.T + 1)) + tau;
        if ((int64_t)now - 1 - s >= sp.depth) atomicOr(&c->status, 1);  // overwritten
        const float4* row =
            reinterpret_cast<const float4*>(sp.trans + ((s % sp.depth) * (int64_t)sp.n + arena) * PM_TRANS_F);
        const float4 r0 = row[0], r1 = row[1], r2 = row[2], r3 = row[3];
        float* ob = o.obs + (int64_t)e * 7;
        float* nx = o.next + (int64_t)e * 7;
        ob[0] = r0.x; ob[1] = r0.y; ob[2] = r0.z; ob[3] = r0.w; ob[4] = r1.x; ob[5] = r1.y; ob[6] = r1.z;
        nx[0] = r2.x; nx[1] = r2.y; nx[2] = r2.z; nx[3] = r2.w; nx[4] = r3.x; nx[5] = r3.y; nx[6] = r3.z;
        const int bits = __float_as_int(r3.w);
        o.rew[e] = r1.w;
        o.act[e] = bits & 0xff;
        o.done[e] = (uint8_t)(bits >> 8);
    }
}

int check(const pm_rnn_selfplay* sp) {
    PM_REQUIRE(sp, PM_E_ARG, "pm_rnn_selfplay: null descriptor");
    PM_REQUIRE(sp->n > 0 && sp->n_pool >= 0, PM_E_SIZE, "pm_rnn_selfplay: n %d, n_pool %d", sp->n, sp->n_pool);
    PM_REQUIRE(sp->T >= 1 && sp->depth > sp->T && sp->seq_cap >= 1, PM_E_SIZE, "pm_rnn_selfplay: T %d depth %d",
               sp->T, sp->depth);
    PM_REQUIRE(sp->opp && sp->ep_reward && sp->ep_len && sp->ep_steps && sp->seq_mark && sp->max_steps >= 0 && sp->reset && sp->w_opp && sp->paramsB && sp->w_B && sp->hA &&
                   sp->cA && sp->hB && sp->cB && sp->obsA && sp->obsB && sp->aA && sp->aB && sp->trans && sp->seq_eps &&
                   sp->fin && sp->partials && sp->opp_list && sp->opp_cnt && sp->enable && sp->ctrl,
               PM_E_ARG, "pm_rnn_selfplay: null buffer");
    PM_REQUIRE((((uintptr_t)sp->trans) & 15) == 0, PM_E_ARG, "pm_rnn_selfplay: trans must be 16-byte aligned");
    PM_REQUIRE(sp->n <= kAppend * kBlock, PM_E_SIZE, "pm_rnn_selfplay: n %d > %d", sp->n, kAppend * kBlock);
    return PM_OK;
}

}  // namespace

extern "C" int pm_rnn_selfplay_init(const pm_rnn_selfplay* sp, void* stream) {
    if (int rc = check(sp)) return rc;
    hipLaunchKernelGGL(k_rsp_init, dim3(pm_blocks(sp->n, kBlock)), dim3(kBlock), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_rsp_init");
    return PM_OK;
}

namespace {
int act_part(const pm_rnn_selfplay* sp, int part, int max_blocks, void* stream) {
    const uint64_t* ctr = &sp->ctrl->step;
    // modelB.reset_noise() then act (:385-387): one noise draw per vector step for all arenas
    if (part != PM_ACT_A)
        if (int rc = pm_rnn_fold(sp->paramsB, sp->paramsB, PM_FOLD_TRAIN_FRESH, sp->seed_net, 0, ctr, sp->w_B, 1, stream))
            return rc;
    return pm_rnn_act_part(sp->w_opp, sp->opp, 1 + sp->n_pool, sp->w_B, sp->obsA, sp->obsB, sp->hA, sp->cA, sp->hB,
                           sp->cB, sp->reset, 0.f, &sp->ctrl->epsilon, sp->seed_env, 0, ctr, sp->aA, sp->aB, sp->qA,
                           sp->qB, sp->n, sp->chunk_A, sp->chunk_P, sp->opp_list, sp->opp_cnt, part, max_blocks,
                           stream, sp->hA_in, sp->cA_in);
}

// Fork / join events of the overlapped step, one pair per device (created on first use).
int step_events(hipEvent_t& fork, hipEvent_t& join) {
    static hipEvent_t ev[64][2] = {};
    int dev = 0;
    PM_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, PM_E_LAUNCH, "hipGetDevice");
    for (int k = 0; k < 2; ++k)
        if (!ev[dev][k]) {
            const hipError_t e = hipEventCreateWithFlags(&ev[dev][k], hipEventDisableTiming);
            PM_REQUIRE(e == hipSuccess, (int)e, "hipEventCreate: %s", hipGetErrorString(e));
        }
    fork = ev[dev][0];
    join = ev[dev][1];
    return PM_OK;
}

// CUs left to the DRQN update while the opponents' act runs beside it: the act blocks hold a CU
// each (one wave per SIMD), so the act grid is capped at the CU count minus this reserve.
// PONGMI_RNN_RESERVE_CUS overrides the reserve (tuning).
constexpr int kDrqnReserveCUs = 64;
int side_a_blocks() {
    static int cus = 0, reserve = kDrqnReserveCUs;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                     hipSuccess)
            cus = 256;
        if (const char* e = getenv("PONGMI_RNN_RESERVE_CUS")) reserve = atoi(e);
    }
    return cus > 2 * reserve ? cus - reserve : (cus + 1) / 2;
}
}  // namespace

extern "C" int pm_rnn_selfplay_act(const pm_rnn_selfplay* sp, void* stream) {
    return pm_rnn_selfplay_act_part(sp, PM_ACT_ALL, stream);
}

extern "C" int pm_rnn_selfplay_act_part(const pm_rnn_selfplay* sp, int32_t part, void* stream) {
    if (int rc = check(sp)) return rc;
    PM_REQUIRE(part == PM_ACT_ALL || part == PM_ACT_B || part == PM_ACT_A, PM_E_ARG,
               "pm_rnn_selfplay_act_part: part=%d", part);
    return act_part(sp, part, 0, stream);
}

namespace {
int rsp_env_tick(const pm_rnn_selfplay* sp, hipStream_t st) {
    hipLaunchKernelGGL(k_rsp_env, dim3(pm_blocks(sp->n, kBlock)), dim3(kBlock), 0, st, *sp);
    PM_LAUNCHED("k_rsp_env");
    return PM_OK;
}
// the episode-table append and the update's batch sample (after k_rsp_env, same stream)
int rsp_append_sample(const pm_rnn_selfplay* sp, const pm_drqn* d, hipStream_t st) {
    hipLaunchKernelGGL(k_rsp_append, dim3(1), dim3(kAppend), 0, st, *sp);
    PM_LAUNCHED("k_rsp_append");
    if (d) {
        PM_REQUIRE(d->T == sp->T, PM_E_ARG, "pm_rnn_selfplay: learner T %d != %d", d->T, sp->T);
        const SampleOut o{const_cast<float*>(d->obs), const_cast<float*>(d->next), const_cast<float*>(d->rew),
                          const_cast<int32_t*>(d->act), const_cast<uint8_t*>(d->done), d->batch, d->T};
        hipLaunchKernelGGL(k_rsp_sample, dim3(1), dim3(512), 0, st, *sp, o, 0);
        PM_LAUNCHED("k_rsp_sample");
    }
    return PM_OK;
}
}  // namespace

extern "C" int pm_rnn_selfplay_env(const pm_rnn_selfplay* sp, const pm_drqn* d, void* stream) {
    if (int rc = check(sp)) return rc;
    hipStream_t st = pm_stream(stream);
    if (int rc = rsp_env_tick(sp, st)) return rc;
    return rsp_append_sample(sp, d, st);
}

extern "C" int pm_rnn_selfplay_sample(const pm_rnn_selfplay* sp, const pm_drqn* d, int32_t u, void* stream) {
    if (int rc = check(sp)) return rc;
    PM_REQUIRE(d && d->T == sp->T, PM_E_ARG, "pm_rnn_selfplay_sample: learner missing or T mismatch");
    PM_REQUIRE(u >= 0 && u < (1 << 15), PM_E_ARG, "pm_rnn_selfplay_sample: u=%d", u);
    const SampleOut o{const_cast<float*>(d->obs), const_cast<float*>(d->next), const_cast<float*>(d->rew),
                      const_cast<int32_t*>(d->act), const_cast<uint8_t*>(d->done), d->batch, d->T};
    hipLaunchKernelGGL(k_rsp_sample, dim3(1), dim3(512), 0, pm_stream(stream), *sp, o, (int)u);
    PM_LAUNCHED("k_rsp_sample");
    return PM_OK;
}

extern "C" int pm_rnn_selfplay_rollout(const pm_rnn_selfplay* sp, const pm_drqn* d, void* stream) {
    if (int rc = pm_rnn_selfplay_act(sp, stream)) return rc;
    return pm_rnn_selfplay_env(sp, d, stream);
}

extern "C" int pm_rnn_selfplay_step(const pm_rnn_selfplay* sp, const pm_drqn* d, void* stream) {
    PM_REQUIRE(d, PM_E_ARG, "pm_rnn_selfplay_step: null learner");
    if (int rc = pm_rnn_selfplay_rollout(sp, d, stream)) return rc;
    return pm_drqn_update(d, stream);
}

// The overlapped vector step. The opponents' act (modelA / pool nets in eval mode, :753-755) reads
// only what the env kernel writes (obs A, opponent ids, reset flags) and their own (h, c), never the
// DRQN update's parameters, so the NEXT step's side A runs on `side_stream` beside this step's update
// (on part of the chip: the update's kernels are a few dozen blocks each), and this step's act is
// modelB's side only. Results are bit-identical to pm_rnn_selfplay_step_multi.
// Contract: sp->aA holds the opponents' actions for the current observations (pm_rnn_selfplay_act_part
// with PM_ACT_A, or the previous overlapped step); on return `stream` has joined the side stream.
namespace {
// One DRQN update; sharded (comm): grads, the in-stream all-reduce of d->grad, apply.
int drqn_update(const pm_drqn* d, pm_comm* comm, void* stream) {
    if (!comm) return pm_drqn_update(d, stream);
    if (int rc = pm_drqn_grads(d, stream)) return rc;
    if (int rc = pm_comm_allreduce_f32(comm, d->grad, PM_RNN_NPARAM + 4, stream)) return rc;
    return pm_drqn_apply(d, stream);
}

// The overlapped step after modelB's act: env + sample, fork (the next step's opponent act on the
// side stream), the updates, join.
int finish_overlap(const pm_rnn_selfplay* sp, const pm_drqn* d, pm_comm* comm, int32_t updates, void* side_stream,
                   void* stream) {
    PM_REQUIRE(d, PM_E_ARG, "pm_rnn_selfplay_step_overlap: null learner");
    PM_REQUIRE(updates >= 1, PM_E_ARG, "pm_rnn_selfplay_step_overlap: updates=%d", updates);
    PM_REQUIRE(side_stream && side_stream != stream, PM_E_ARG, "pm_rnn_selfplay_step_overlap: needs a second stream");
    hipEvent_t fork, join;
    if (int rc = step_events(fork, join)) return rc;
    PM_REQUIRE(d->T == sp->T, PM_E_ARG, "pm_rnn_selfplay: learner T %d != %d", d->T, sp->T);  // before any launch
    hipStream_t st = pm_stream(stream), side = pm_stream(side_stream);
    // the fork follows the env tick: side A reads only what k_rsp_env writes (observations, opponent
    // ids, reset flags) and its own (h, c), so the episode-table append and the batch sample run
    // beside it instead of in front of it
    if (int rc = rsp_env_tick(sp, st)) return rc;
    hipError_t e = hipEventRecord(fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(side, fork, 0);
    PM_REQUIRE(e == hipSuccess, (int)e, "step_overlap fork: %s", hipGetErrorString(e));
    if (int rc = act_part(sp, PM_ACT_A, side_a_blocks(), side_stream)) return rc;
    e = hipEventRecord(join, side);
    PM_REQUIRE(e == hipSuccess, (int)e, "step_overlap join record: %s", hipGetErrorString(e));
    if (int rc = rsp_append_sample(sp, d, st)) return rc;
    for (int u = 0; u < updates; ++u) {
        if (u)
            if (int rc = pm_rnn_selfplay_sample(sp, d, u, stream)) return rc;
        if (int rc = drqn_update(d, comm, stream)) return rc;
    }
    e = hipStreamWaitEvent(st, join, 0);
    PM_REQUIRE(e == hipSuccess, (int)e, "step_overlap join: %s", hipGetErrorString(e));
    return PM_OK;
}
}  // namespace

// The overlapped vector step. The opponents' act (modelA / pool nets in eval mode, :753-755) reads
// only what the env kernel writes (obs A, opponent ids, reset flags) and their own (h, c), never the
// DRQN update's parameters, so the NEXT step's side A runs on `side_stream` beside this step's update
// (on part of the chip: the update's kernels are a few dozen blocks each), and this step's act is
// modelB's side only. Results are bit-identical to pm_rnn_selfplay_step_multi.
// Contract: sp->aA holds the opponents' actions for the current observations (pm_rnn_selfplay_act_part
// with PM_ACT_A, or the previous overlapped step); on return `stream` has joined the side stream.
extern "C" int pm_rnn_selfplay_step_overlap(const pm_rnn_selfplay* sp, const pm_drqn* d, int32_t updates,
                                            void* side_stream, void* stream) {
    if (int rc = check(sp)) return rc;
    if (int rc = act_part(sp, PM_ACT_B, 0, stream)) return rc;
    return finish_overlap(sp, d, nullptr, updates, side_stream, stream);
}

extern "C" int pm_rnn_selfplay_finish_overlap(const pm_rnn_selfplay* sp, const pm_drqn* d, int32_t updates,
                                              void* side_stream, void* stream) {
    if (int rc = check(sp)) return rc;
    return finish_overlap(sp, d, nullptr, updates, side_stream, stream);
}

// Sharded and overlapped: the same step with every update's gradient all-reduced in stream order.
extern "C" int pm_rnn_selfplay_step_sharded_overlap(const pm_rnn_selfplay* sp, const pm_drqn* d, pm_comm* comm,
                                                    int32_t updates, void* side_stream, void* stream) {
    if (int rc = check(sp)) return rc;
    PM_REQUIRE(comm, PM_E_ARG, "pm_rnn_selfplay_step_sharded_overlap: null comm");
    if (int rc = act_part(sp, PM_ACT_B, 0, stream)) return rc;
    return finish_overlap(sp, d, comm, updates, side_stream, stream);
}

extern "C" int pm_rnn_selfplay_step_multi(const pm_rnn_selfplay* sp, const pm_drqn* d, int32_t updates, void* stream) {
    PM_REQUIRE(updates >= 1, PM_E_ARG, "pm_rnn_selfplay_step_multi: updates=%d", updates);
    if (int rc = pm_rnn_selfplay_step(sp, d, stream)) return rc;
    for (int u = 1; u < updates; ++u) {
        if (int rc = pm_rnn_selfplay_sample(sp, d, u, stream)) return rc;
        if (int rc = pm_drqn_update(d, stream)) return rc;
    }
    return PM_OK;
}
