// The batched self-play learner: one vector step of scripts/train_iterative.py:239-245 for n arenas.
//
//   k_act_sp    (MFMA tiles)   both players' QNet forward + eps-greedy / argmax (pm_mfma.h)
//   k_env       (n lanes)      env tick + replay push + episode bookkeeping + serves
//   k_per_refresh              per-1024 block sums of prio^alpha for the blocks that changed
//   k_sp_sample (batch waves)  proportional sample + un-normalised IS weights
//   k_dqn_fwd   (MFMA tiles)   Q_B(s), Q_B(s'), Q_T(s') and features of s for the sampled batch
//   k_dqn       (1 WG)         double-DQN targets, IS-weighted MSE, head grads, priority update
//   ----------------------------- (sharded: RCCL all-reduce of sp.grad here)
//   k_adam      (1 WG)         Adam on the 520 head params, target sync, epsilon decay,
//                              replay/step counters, next step's acting noise and next update's
//                              heads (fused into k_dqn when unsharded)
//
// Nothing returns to the host: every loop counter lives in the device control block (pm_ctrl), so
// a whole vector step can be replayed from a captured graph.
#include "pm_host.h"
#include "pm_mfma.h"
#include "pm_per.h"

using namespace pm;

namespace {

constexpr int kBlock = 256;
constexpr int kGradN = PM_QNET_NHEAD;  // grad[520] = finished episodes, grad[521] = updated flag

__device__ __forceinline__ bool learner_active(const pm_selfplay& sp) {
    const int64_t s = sp.ctrl->size + sp.n;
    return (s < sp.cap ? s : sp.cap) >= sp.batch;
}

// ------------------------------------------------------------------------------------ rollout
// Both players act (train_iterative.py:240-241) on the matrix cores: ActGrid blocks, modelB tiles
// with epsilon-greedy, opponent tiles grouped by net (modelA / pool) so weights are tile-uniform.
__global__ __launch_bounds__(kActBlock, 2) void k_act_sp(const pm_selfplay sp) {
    __shared__ __attribute__((aligned(16))) ActShared sh;
    const ActGrid g{sp.n, sp.n_pool + 1, sp.chunk_A, sp.chunk_P, 1};
    const TileOut outA{sp.aA, nullptr, -1.0, 0, 0};
    const TileOut outB{sp.aB, nullptr, sp.ctrl->epsilon, sp.seed_env, sp.ctrl->step};
    act_block(sh, g, sp.w_opp, sp.n_pool > 0 ? sp.opp : nullptr, sp.w_B, sp.obsA, sp.obsB, outA, outB);
}

// env.step (:242) + memory.push (:243) + episode bookkeeping (:245-249) + next opponent (:235-236)
// and env.reset (:238) for finished arenas; writes next step's observations. HBM-bound.
__global__ __launch_bounds__(kBlock) void k_env(const pm_selfplay sp) {
    __shared__ float lds[kBlock][7];
    __shared__ long long red[kBlock / 64][6];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    const bool valid = i < sp.n;
    const int ii = valid ? i : sp.n - 1;
    const pm_ctrl* c = sp.ctrl;
    const int64_t pos = c->pos, size = c->size;
    const float maxp = size == 0 ? 1.0f : c->max_prio;  // max(prios) if buffer else 1.0 (:57)

    Arena a = load_arena(sp.st, ii);
    const int aA = sp.aA[ii], aB = sp.aB[ii];
    const int o = sp.opp[ii];
    float oA[7], oB[7];
    observe(a, oA, oB);  // the state the actions were chosen on (= obs of the previous env kernel)
    float rA, rB;
    const int d = tick(sp.env, a, aA, aB, rA, rB);
    float nA[7], nB[7];
    observe(a, nA, nB);
    const float er = sp.ep_reward[ii] + rB;  // ep_reward += rB (:245)
    const bool fin = valid && d;
    {   // per-block partials, no atomics (:247-249)
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const bool win = er > 0.f;
        const unsigned long long mf = __ballot(fin), mA = __ballot(fin && o == 0), mwA = __ballot(fin && o == 0 && win);
        const unsigned long long mP = __ballot(fin && o != 0), mwP = __ballot(fin && o != 0 && win);
        int rs = fin ? (int)er : 0;
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) rs += __shfl_xor(rs, s);
        if (lane == 0) {
            red[wv][0] = __popcll(mf); red[wv][1] = __popcll(mA); red[wv][2] = __popcll(mwA);
            red[wv][3] = __popcll(mP); red[wv][4] = __popcll(mwP); red[wv][5] = rs;
        }
    }
    if (valid) {
        // memory.push((oB, aB, rB, nB, done)) (:243, :56-63)
        const int64_t slot = (pos + i) % sp.cap;
        float4* row = reinterpret_cast<float4*>(sp.trans + slot * PM_TRANS_F);
        row[0] = make_float4(oB[0], oB[1], oB[2], oB[3]);
        row[1] = make_float4(oB[4], oB[5], oB[6], rB);
        row[2] = make_float4(nB[0], nB[1], nB[2], nB[3]);
        row[3] = make_float4(nB[4], nB[5], nB[6], __int_as_float(aB | (d << 8)));
        sp.prios[slot] = maxp;
        int onew = o;
        float ernew = er;
        if (d) {  // next episode: opponent draw then env.reset()
            const uint32_t ns = (uint32_t)sp.st.serves[i];
            const U4 q = philox((uint32_t)i, TAG_OPP, ns, 0u, sp.seed_env);
            onew = (sp.n_pool > 0 && u53(q.x, q.y) < sp.pool_ratio) ? 1 + below(q.z, (uint32_t)sp.n_pool) : 0;
            double vx, vy, spn;
            philox_serve(sp.env, (uint32_t)i, ns, sp.seed_env, vx, vy, spn);
            serve(a, vx, vy, spn);
            sp.st.serves[i] = (int32_t)ns + 1;
            ernew = 0.f;
            observe(a, nA, nB);
        }
        store_arena(sp.st, i, a);
        sp.opp[i] = onew;
        sp.ep_reward[i] = ernew;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w][threadIdx.x];
        sp.partials[(size_t)blockIdx.x * 8 + threadIdx.x] = t;
    }
    store_rows7(sp.obsA, lds, nA, i0, sp.n);
    store_rows7(sp.obsB, lds, nB, i0, sp.n);
}

// ------------------------------------------------------------------------------------ init
__global__ __launch_bounds__(kBlock) void k_sp_init(const pm_selfplay sp) {
    __shared__ float lds[kBlock][7];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0};
    if (i < sp.n) {
        const uint32_t ns = (uint32_t)sp.st.serves[i];
        const U4 q = philox((uint32_t)i, TAG_OPP, ns, 0u, sp.seed_env);
        sp.opp[i] = (sp.n_pool > 0 && u53(q.x, q.y) < sp.pool_ratio) ? 1 + below(q.z, (uint32_t)sp.n_pool) : 0;
        Arena a;
        double vx, vy, spn;
        philox_serve(sp.env, (uint32_t)i, ns, sp.seed_env, vx, vy, spn);
        serve(a, vx, vy, spn);
        store_arena(sp.st, i, a);
        sp.st.serves[i] = (int32_t)ns + 1;
        sp.ep_reward[i] = 0.f;
        observe(a, oA, oB);
    }
    store_rows7(sp.obsA, lds, oA, i0, sp.n);
    store_rows7(sp.obsB, lds, oB, i0, sp.n);
}

// ------------------------------------------------------------------------------------ learner
__device__ __forceinline__ double beta_of(const pm_selfplay& sp, int64_t frame) {  // :137
    const double b = sp.beta_start + (double)frame * (1.0 - sp.beta_start) / (double)sp.beta_frames;
    return b < 1.0 ? b : 1.0;
}

__global__ __launch_bounds__(256) void k_sp_sample(const pm_selfplay sp, const double* __restrict__ bsum) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= sp.batch || !learner_active(sp)) return;  // wave-uniform
    const int64_t s = sp.ctrl->size + sp.n;
    const int64_t size = s < sp.cap ? s : sp.cap;
    const int64_t frame = sp.ctrl->frame_idx + 1;  // frame_idx += 1 before sampling (:136)
    const U4 r = philox64((uint32_t)j, TAG_PER, (uint64_t)frame, sp.seed_env);
    int64_t idx;
    float wr;
    per_sample_one(sp.prios, size, bsum, (float)sp.alpha, beta_of(sp, frame), u53(r.x, r.y), idx, wr);
    if ((threadIdx.x & 63) == 0) { sp.idx[j] = idx; sp.isw[j] = wr; }
}

// Priority block sums, incremental: only the 1024-entry blocks this step's push wrote ([pos, pos+n)
// mod cap) and the blocks the previous update's priority scatter touched (sp.idx still holds its
// indices) changed since they were last summed. Each is recomputed from scratch in the same fixed
// order as a full pass (k_per_reduce), so the sums are identical to a full recompute.
__global__ __launch_bounds__(256) void k_per_refresh(const pm_selfplay sp, double* __restrict__ bsum) {
    __shared__ double part[4];
    if (!learner_active(sp)) return;
    const int64_t nbc = (sp.cap + PER_CHUNK - 1) / PER_CHUNK;
    const int64_t npush = (int64_t)(sp.n + PER_CHUNK - 1) / PER_CHUNK + 2;
    int64_t blk;
    if ((int64_t)blockIdx.x < npush) {
        const int64_t pos = sp.ctrl->pos;  // not yet committed: the push of this step started here
        const int64_t first = pos / PER_CHUNK, last = (pos + sp.n - 1) / PER_CHUNK;
        if (first + (int64_t)blockIdx.x > last) return;
        blk = (first + blockIdx.x) % nbc;
    } else {
        blk = sp.idx[blockIdx.x - npush] / PER_CHUNK;
    }
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const float alpha = (float)sp.alpha;
    double acc = 0.0;
    const int64_t base = blk * PER_CHUNK;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t e = base + t + k * 256;
        if (e < sp.cap) acc += (double)powf(sp.prios[e], alpha);
    }
    acc = wave_sum(acc);
    if (lane == 0) part[wv] = acc;
    __syncthreads();
    if (t == 0) bsum[blk] = ((part[0] + part[1]) + part[2]) + part[3];
}

// ------------------------------------------------------------------------------------ apply
struct ApplySmem {
    float hp[PM_QNET_NHEAD];   // modelB head parameters (after the optimizer step)
    float tmu[PM_QNET_NHEAD];  // targetB head parameters (mu used)
    float nact[132], ntrain[132];
    float heads[260];
};

// Everything that follows from the head parameters once they are final for this step, from LDS:
// acting weights for vector step `act_ctr` (select_action_B -> reset_noise, :125; the noise lands
// in modelB's epsilon buffers), the next update's modelB heads with fresh noise `train_ctr`
// (reset_noise, :142) and targetB heads (eval mode: mu, :100), both in MFMA fragment order in
// learn_heads, plus that update's noise. Block-wide; noise already in sm.nact / sm.ntrain.
__device__ __forceinline__ void derive_weights(const pm_selfplay& sp, ApplySmem& sm) {
    const int t = threadIdx.x, nt = blockDim.x;
    float* lh = sp.learn_heads;
    fold_heads_from(sm.hp, nullptr, sm.nact, PM_FOLD_TRAIN_FRESH, sm.heads, sp.paramsB + PM_QNET_EPS_OFF, t, nt);
    __syncthreads();
    write_head_frags(sm.heads, sp.w_B);
    __syncthreads();
    fold_heads_from(sm.hp, nullptr, sm.ntrain, PM_FOLD_TRAIN_FRESH, sm.heads, lh + 528, t, nt);
    __syncthreads();
    heads_to_frags(sm.heads, lh);
    __syncthreads();
    fold_heads_from(sm.tmu, nullptr, nullptr, PM_FOLD_EVAL, sm.heads, nullptr, t, nt);
    __syncthreads();
    heads_to_frags(sm.heads, lh + 264);
}

// Both noise draws at once, half of the block each.
__device__ __forceinline__ void gen_both_noises(const pm_selfplay& sp, ApplySmem& sm, uint64_t act_ctr,
                                                uint64_t train_ctr) {
    const int t = threadIdx.x, half = blockDim.x / 2;
    if (t < half) gen_noise(sp.seed_net, TAG_NOISE_ACT, act_ctr, sm.nact, t, half);
    else gen_noise(sp.seed_net, TAG_NOISE_TRAIN, train_ctr, sm.ntrain, t - half, half);
}

// optimizer.step() (:161) on the shard-summed grads, target sync (:166-168), epsilon decay (:261),
// replay / step counters, then derive_weights for the next step. One global load round trip:
// grads, Adam moments, modelB and targetB heads are read together; the rest runs from LDS.
__device__ __forceinline__ void apply_update(const pm_selfplay& sp, ApplySmem& sm) {
    const int t = threadIdx.x, nt = blockDim.x;
    pm_ctrl* c = sp.ctrl;
    const bool train = sp.grad[kGradN + 1] > 0.5f;
    const int64_t ts = c->train_steps + (train ? 1 : 0);
    const uint64_t step = c->step;
    const double bc1 = 1.0 - pow(sp.beta1, (double)ts);
    const double bc2 = 1.0 - pow(sp.beta2, (double)ts);
    const float step_size = (float)(sp.lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    for (int k = t; k < PM_QNET_NHEAD; k += nt) {  // torch.optim.Adam, single-tensor path
        float p = sp.paramsB[PM_QNET_HEAD_OFF + k];
        sm.tmu[k] = sp.paramsT[PM_QNET_HEAD_OFF + k];
        if (train) {
            const float g = sp.grad[k] / (float)sp.world;
            float m = sp.adam_m[k], v = sp.adam_v[k];
            m = m + (float)(1.0 - sp.beta1) * (g - m);                  // exp_avg.lerp_(grad, 1-beta1)
            v = v * (float)sp.beta2 + (float)(1.0 - sp.beta2) * g * g;  // mul_(beta2).addcmul_(g, g, 1-beta2)
            const float denom = sqrtf(v) / bc2s + (float)sp.adam_eps;
            p = p - step_size * (m / denom);
            sp.paramsB[PM_QNET_HEAD_OFF + k] = p;
            sp.adam_m[k] = m;
            sp.adam_v[k] = v;
        }
        sm.hp[k] = p;
    }
    gen_both_noises(sp, sm, step + 1, (uint64_t)ts + 1);
    __syncthreads();
    if (train && ts % sp.target_update_interval == 0) {  // targetB.load_state_dict(modelB) (:166-168)
        for (int k = t; k < PM_QNET_NHEAD; k += nt) sm.tmu[k] = sm.hp[k];
        for (int k = t; k < PM_QNET_NP; k += nt) {
            const int h = k - PM_QNET_HEAD_OFF;
            sp.paramsT[k] = (h >= 0 && h < PM_QNET_NHEAD) ? sm.hp[h] : sp.paramsB[k];
        }
    }
    __syncthreads();
    derive_weights(sp, sm);
    if (t == 0) {
        const double D = (double)sp.grad[kGradN];  // finished episodes (all shards)
        const double e = c->epsilon * pow(sp.epsilon_decay, D);  // per-episode decay (:261)
        c->epsilon = e > sp.min_epsilon ? e : sp.min_epsilon;
        if (train) { c->train_steps = ts; c->frame_idx += 1; }
        c->pos = (c->pos + sp.n) % sp.cap;
        const int64_t s = c->size + sp.n;
        c->size = s < sp.cap ? s : sp.cap;
        c->step = step + 1;
    }
}

// ------------------------------------------------------------------------------------ learner
// The three QNet evaluations of train_step (:152-155) for the sampled batch on the matrix cores:
// rows [0, B) are s, rows [B, 2B) are s'. Heads come precomputed in learn_heads (modelB with the
// update's fresh noise, targetB with mu). Writes h2 = ReLU(features(s)) for the gradient and, per
// sample j, q[j*16 + 0..2] = Q_B(s), [4..6] = Q_B(s'), [8..10] = Q_T(s'). One tile per wave.
__global__ __launch_bounds__(256) void k_dqn_fwd(const pm_selfplay sp) {
    __shared__ __attribute__((aligned(16))) float lw[F_SIZE];
    __shared__ __attribute__((aligned(16))) float hf[2][264];
    if (!learner_active(sp)) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, col = lane & 31;
    const int B = sp.batch;
    stage_frags(sp.w_B, lw);  // modelB.features fragments (frozen; == targetB.features)
    for (int k = threadIdx.x; k < 2 * 264; k += blockDim.x) hf[k / 264][k % 264] = sp.learn_heads[k];
    if (blockIdx.x == 0)  // the update's noise in modelB's epsilon buffers, as reset_noise leaves them
        for (int k = threadIdx.x; k < 260; k += blockDim.x) sp.paramsB[PM_QNET_EPS_OFF + k] = sp.learn_heads[528 + k];
    __syncthreads();
    const int tile = blockIdx.x * 4 + wave;
    if (tile * 32 >= 2 * B) return;  // wave-uniform
    const int g = tile * 32 + col;
    const bool valid = g < 2 * B;
    const int gg = valid ? g : 2 * B - 1;
    const bool nxt = gg >= B;
    const int j = nxt ? gg - B : gg;
    float xs[4];
    tile_inputs(sp.trans + sp.idx[j] * PM_TRANS_F + (nxt ? 8 : 0), h, xs);
    f32x16 c2[2];
    tile_hidden(lw, xs, lane, c2);
    float qb[3], qt[3];
    tile_heads(hf[0], c2, lane, qb);
    tile_heads(hf[1], c2, lane, qt);
    float* hs = sp.hfeat + (size_t)j * 64;
    float* q = sp.hfeat + (size_t)B * 64 + (size_t)j * 16;
    if (valid && !nxt) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) hs[32 * t + rho(r) + 4 * h] = fmaxf(c2[t][r], 0.f);
    }
    if (valid && h == 0) {
        if (!nxt) {
            q[0] = qb[0]; q[1] = qb[1]; q[2] = qb[2];
        } else {
            q[4] = qb[0]; q[5] = qb[1]; q[6] = qb[2];
            q[8] = qt[0]; q[9] = qt[1]; q[10] = qt[2];
        }
    }
}

__global__ __launch_bounds__(256) void k_dqn(const pm_selfplay sp) {
    __shared__ float Hs[PM_MAX_BATCH][65];
    __shared__ float coef[PM_MAX_BATCH][4];
    __shared__ int64_t sidx[PM_MAX_BATCH];
    __shared__ float red[4][2];
    __shared__ float red2[4][8];
    __shared__ long long cnt[4][6];
    __shared__ ApplySmem asm_;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    pm_ctrl* c = sp.ctrl;

    // ---- rollout partials -> episode counters: one block row per thread, then a fixed-order tree
    {
        const int nbr = (sp.n + kBlock - 1) / kBlock;
        long long v[6] = {0, 0, 0, 0, 0, 0};
        for (int b = t; b < nbr; b += 256)
#pragma unroll
            for (int k = 0; k < 6; ++k) v[k] += sp.partials[(size_t)b * 8 + k];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
            if (lane == 0) cnt[wv][k] = v[k];
        }
    }
    __syncthreads();
    const bool train = learner_active(sp);
    if (t == 0) {
        long long s[6];
        for (int k = 0; k < 6; ++k) s[k] = ((cnt[0][k] + cnt[1][k]) + cnt[2][k]) + cnt[3][k];
        c->ep_step = s[0];
        c->episodes += s[0];
        c->ep_A += s[1]; c->win_A += s[2];
        c->ep_P += s[3]; c->win_P += s[4];
        c->reward_B += (double)s[5];
        sp.grad[kGradN] = (float)s[0];
        sp.grad[kGradN + 1] = train ? 1.f : 0.f;
    }
    if (train) {
        const int B = sp.batch;
        const bool act = t < B;
        {   // features of s (k_dqn_fwd) -> LDS, coalesced
            const float4* src = reinterpret_cast<const float4*>(sp.hfeat);
            for (int k = t; k < B * 16; k += 256) {
                const float4 v = src[k];
                const int row = k >> 4, c4 = (k & 15) * 4;
                Hs[row][c4 + 0] = v.x; Hs[row][c4 + 1] = v.y; Hs[row][c4 + 2] = v.z; Hs[row][c4 + 3] = v.w;
            }
        }
        // ---- IS weights: w /= max(w) over the batch (:72)
        const float wraw = act ? sp.isw[t] : 0.f;
        float m = wraw;
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
        if (lane == 0) red[wv][0] = m;
        __syncthreads();
        const float wmax = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
        float lossp = 0.f, prio = 0.f;
        float cf[4] = {0.f, 0.f, 0.f, 0.f};
        if (act) {
            const int64_t id = sp.idx[t];
            sidx[t] = id;
            const float* tr = sp.trans + id * PM_TRANS_F;
            const float rwd = tr[7];
            const int bits = __float_as_int(tr[15]);
            const int a = bits & 0xff, dn = (bits >> 8) & 1;
            const float* qq = sp.hfeat + (size_t)B * 64 + (size_t)t * 16;
            const float qs[3] = {qq[0], qq[1], qq[2]};
            const float qn[3] = {qq[4], qq[5], qq[6]};
            const float qt[3] = {qq[8], qq[9], qq[10]};
            const float q = qs[a];                                            // modelB(s).gather(a)   (:152)
            const float nq = qt[argmax3(qn)];                                 // targetB(ns)[argmax modelB(ns)]
            const float tgt = rwd + (float)sp.gamma * nq * (dn ? 0.f : 1.f);  // r + gamma*nq*(~d)     (:156)
            const float diff = q - tgt;
            const float w = wraw / wmax;
            lossp = w * (diff * diff);
            const float g = 2.f * w * diff / (float)B;  // d mean(w (q-t)^2) / dq
            cf[0] = g;
#pragma unroll
            for (int k = 0; k < 3; ++k) cf[1 + k] = g * ((k == a ? 1.f : 0.f) - 1.f / 3.f);
#pragma unroll
            for (int k = 0; k < 4; ++k) coef[t][k] = cf[k];
            prio = fabsf(diff) + 1e-6f;  // |err| + 1e-6 (:76)
        }
        // loss, max priority and the 4 bias gradients (sum_j coef_j) as block reductions
        float s = lossp, mp = prio;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o);
            mp = fmaxf(mp, __shfl_xor(mp, o));
#pragma unroll
            for (int k = 0; k < 4; ++k) cf[k] += __shfl_xor(cf[k], o);
        }
        __syncthreads();
        if (lane == 0) {
            red[wv][0] = s; red[wv][1] = mp;
#pragma unroll
            for (int k = 0; k < 4; ++k) red2[wv][k] = cf[k];
        }
        __syncthreads();
        if (act) {  // update_priorities: sequential order, the last duplicate wins (:74-76)
            const int64_t mine = sidx[t];
            bool last = true;
#pragma unroll 8
            for (int k = 0; k < B; ++k) last &= !(k > t && sidx[k] == mine);  // uniform k: broadcast reads
            if (last) sp.prios[mine] = prio;
        }
        if (t == 0) {
            c->last_loss = (((red[0][0] + red[1][0]) + red[2][0]) + red[3][0]) / (float)B;
            const float mpx = fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1]));
            c->max_prio = fmaxf(c->max_prio, mpx);  // n > batch pushes of max_prio survive the scatter
        }
        // ---- head gradients: dL/dW_mu = sum_j coef_j h_j (one output per thread), dL/db_mu = sum_j
        // coef_j; dL/dW_sigma = dL/dW_mu * eps with the update's noise (learn_heads[528..])
        const float* ep = sp.learn_heads + 528;
        {
            const int row = t >> 6, col = t & 63;  // 256 weight outputs, row uniform per wave
            float g = 0.f;
#pragma unroll 8
            for (int j = 0; j < B; ++j) g = fmaf(coef[j][row], Hs[j][col], g);
            if (row == 0) {
                sp.grad[col] = g;                                                  // fc_V.weight_mu
                sp.grad[65 + col] = g * ep[P_VWEP - PM_QNET_EPS_OFF + col];          // fc_V.weight_sigma
            } else {
                const int a = row - 1;
                sp.grad[130 + a * 64 + col] = g;                                   // fc_A.weight_mu
                sp.grad[325 + a * 64 + col] = g * ep[P_AWEP - PM_QNET_EPS_OFF + a * 64 + col];  // fc_A.weight_sigma
            }
        }
        if (t < 4) {
            const float g = ((red2[0][t] + red2[1][t]) + red2[2][t]) + red2[3][t];
            if (t == 0) {
                sp.grad[64] = g;                                                   // fc_V.bias_mu
                sp.grad[129] = g * ep[P_VBEP - PM_QNET_EPS_OFF];                     // fc_V.bias_sigma
            } else {
                sp.grad[322 + t - 1] = g;                                          // fc_A.bias_mu
                sp.grad[517 + t - 1] = g * ep[P_ABEP - PM_QNET_EPS_OFF + t - 1];     // fc_A.bias_sigma
            }
        }
    } else {
        for (int k = t; k < kGradN; k += 256) sp.grad[k] = 0.f;
    }
    if (sp.fuse_apply) {  // unsharded: no all-reduce between the gradient and the optimizer step
        __threadfence_block();
        __syncthreads();
        apply_update(sp, asm_);
    }
}

// ------------------------------------------------------------------------------------ Adam + commit
__global__ __launch_bounds__(1024) void k_adam(const pm_selfplay sp) {
    __shared__ ApplySmem sm;
    apply_update(sp, sm);
}

// pm_selfplay_prepare: features + acting weights of the current step + next update's heads
__global__ __launch_bounds__(256) void k_prepare(const pm_selfplay sp) {
    __shared__ ApplySmem sm;
    write_feature_frags(sp.paramsB, sp.w_B);
    for (int k = threadIdx.x; k < PM_QNET_NHEAD; k += blockDim.x) {
        sm.hp[k] = sp.paramsB[PM_QNET_HEAD_OFF + k];
        sm.tmu[k] = sp.paramsT[PM_QNET_HEAD_OFF + k];
    }
    gen_both_noises(sp, sm, sp.ctrl->step, (uint64_t)sp.ctrl->train_steps + 1);
    __syncthreads();
    derive_weights(sp, sm);
}

int check(const pm_selfplay* sp) {
    PM_REQUIRE(sp && sp->ctrl && sp->trans && sp->prios && sp->per_work && sp->idx && sp->isw && sp->grad &&
                   sp->partials && sp->hfeat && sp->w_opp && sp->paramsB && sp->paramsT && sp->w_B && sp->adam_m &&
                   sp->adam_v && sp->opp && sp->ep_reward,
               PM_E_ARG, "pm_selfplay: null buffer");
    PM_REQUIRE(sp->n > 0 && sp->batch >= 1 && sp->batch <= PM_MAX_BATCH && sp->n > sp->batch && sp->cap >= sp->n,
               PM_E_SIZE, "pm_selfplay: n=%d batch=%d cap=%lld", sp->n, sp->batch, (long long)sp->cap);
    PM_REQUIRE(sp->n_pool >= 0 && sp->n_pool <= 4096 && sp->world >= 1, PM_E_SIZE, "pm_selfplay: n_pool/world");
    PM_REQUIRE(sp->obsA && sp->obsB && sp->aA && sp->aB && sp->learn_heads, PM_E_ARG, "pm_selfplay: null buffer");
    PM_REQUIRE(!sp->fuse_apply || sp->world == 1, PM_E_ARG, "pm_selfplay: fuse_apply needs world == 1");
    PM_REQUIRE(sp->chunk_A > 0 && sp->chunk_A <= kListMax && sp->chunk_P > 0 && sp->chunk_P <= kListMax, PM_E_SIZE,
               "pm_selfplay: chunk_A/chunk_P must be in [1, %d]", kListMax);
    PM_REQUIRE(((((uintptr_t)sp->w_opp) | ((uintptr_t)sp->w_B)) & 15) == 0, PM_E_ARG, "pm_selfplay: weights alignment");
    PM_REQUIRE(sp->env.speed_scale_every > 0 && sp->target_update_interval > 0 && sp->beta_frames > 0, PM_E_ARG,
               "pm_selfplay: zero interval");
    return PM_OK;
}

}  // namespace

extern "C" int pm_selfplay_prepare(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipLaunchKernelGGL(k_prepare, dim3(1), dim3(256), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_prepare");
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

extern "C" int pm_selfplay_act(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    const ActGrid g{sp->n, sp->n_pool + 1, sp->chunk_A, sp->chunk_P, 1};
    hipLaunchKernelGGL(k_act_sp, dim3(g.blocks()), dim3(kActBlock), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_act_sp");
    return PM_OK;
}

extern "C" int pm_selfplay_env(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipLaunchKernelGGL(k_env, dim3(pm_blocks(sp->n, kBlock)), dim3(kBlock), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_env");
    return PM_OK;
}

extern "C" int pm_selfplay_rollout(const pm_selfplay* sp, void* stream) {
    int rc = pm_selfplay_act(sp, stream);
    return rc ? rc : pm_selfplay_env(sp, stream);
}

extern "C" int pm_selfplay_learn(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    hipStream_t st = pm_stream(stream);
    double* bsum = reinterpret_cast<double*>(sp->per_work);
    const int npush = (sp->n + PER_CHUNK - 1) / PER_CHUNK + 2;
    hipLaunchKernelGGL(k_per_refresh, dim3(npush + sp->batch), dim3(256), 0, st, *sp, bsum);
    PM_LAUNCHED("k_per_refresh");
    hipLaunchKernelGGL(k_sp_sample, dim3(pm_blocks(sp->batch, 4)), dim3(256), 0, st, *sp, bsum);
    PM_LAUNCHED("k_sp_sample");
    hipLaunchKernelGGL(k_dqn_fwd, dim3(pm_blocks(2 * sp->batch, 128)), dim3(256), 0, st, *sp);
    PM_LAUNCHED("k_dqn_fwd");
    hipLaunchKernelGGL(k_dqn, dim3(1), dim3(256), 0, st, *sp);
    PM_LAUNCHED("k_dqn");
    return PM_OK;
}

extern "C" int pm_selfplay_apply(const pm_selfplay* sp, void* stream) {
    int rc = check(sp);
    if (rc) return rc;
    if (sp->fuse_apply) return PM_OK;  // learn already applied (unsharded, fused)
    hipLaunchKernelGGL(k_adam, dim3(1), dim3(1024), 0, pm_stream(stream), *sp);
    PM_LAUNCHED("k_adam");
    return PM_OK;
}

extern "C" int pm_selfplay_step(const pm_selfplay* sp, void* stream) {
    int rc = pm_selfplay_rollout(sp, stream);
    if (!rc) rc = pm_selfplay_learn(sp, stream);
    return rc ? rc : pm_selfplay_apply(sp, stream);
}
