// K6 — the DRQN update (train_step_rnn, scripts/train_rnn_iterative.py:400-531) on the device.
//
// Five launches per update, every matrix product on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32):
//
//   k_dq_embed  (grads 1/3) the batch through the feature layers and the LSTM input projection for
//               all three streams (modelB on obs, modelB on next, targetB on next): per (stream,
//               32-column tile, time step) F1 = ReLU(W1 x + b1), F2 = ReLU(W2 F1 + b2) and
//               Zx = Wih F2 + bih + bhh, Zx written in the accumulator layout the recurrence starts
//               from; the obs stream's F1 / F2 kept for the weight gradients.
//   k_dq_recur  (grads 2/3) the whole recurrence, persistent: every (stream, column tile) is a group
//               of 16 workgroups, workgroup m owning LSTM units 8m..8m+7 (all four gates: one 32-row
//               MFMA tile, its Whh rows in registers, K split over the 4 waves). Per time step the
//               group exchanges h through write-through (sc1) stores + a per-workgroup step flag
//               (MI355X_MICROARCH.md hand-off table, row 1), the cell state never leaves registers.
//               Then the heads: each workgroup computes its 8 rows of the shared head and their
//               partial V / A; the obs stream's group gathers all three streams' partial Q, forms the
//               double-DQN target, smooth-L1 and dQ, the head gradients of its rows, and starts BPTT
//               from dh_T = W_S^T dS; per BPTT step dz in registers (gates and c saved by the
//               forward), dh_{t-1} = Whh^T dz as per-workgroup partials exchanged the same way.
//   k_dq_wgrad  (grads 3/3) the weight gradients: dWih = dZ F2^T, dWhh = dZ H^T and the biases over
//               all T*B columns (one workgroup per 32x32 output tile, K split over 16 waves); per
//               32-column tile dF2 = Wih^T dZ -> ReLU mask -> dW2 / db2 partials -> dF1 = W2^T dP2
//               -> dW1 / db1 partials, summed in a fixed order by the last tile to finish (arrival
//               ticket); the head gradient partials of the column tiles summed likewise.
//   k_drqn_norm, k_drqn_adam  (pm_drqn_apply) the NoisyLinear sigma gradients (mu gradient x epsilon),
//               the global-norm clip (fp64 partials, fixed order) and torch's Adam, target sync.
//
// Every reduction runs in a fixed order and nothing sums through atomics, so an update is
// bit-reproducible run to run (the arrival ticket only picks which workgroup does the final sum).
#include "pm_host.h"
#include "pm_rnn.h"

namespace pm {
namespace {

constexpr int kG = 16;           // workgroups per recurrence group (8 LSTM units each)
constexpr int kNormBlocks = 256;  // k_drqn_norm blocks (fp64 partials, summed in order by k_drqn_adam)
constexpr int kWgA = 128;        // k_dq_wgrad: dWih / dWhh output tiles
constexpr int kWgC = 4;          // k_dq_wgrad: head-partial reduce workgroups
constexpr int kLowN = 8832;      // grad [0, kLowN): W1, b1, W2, b2 (the column-tile partials)
// per-column-tile head gradient partials (floats)
enum : int { HP_WS = 0, HP_BS = 16384, HP_V = 16512, HP_VB = 16640, HP_A = 16641, HP_AB = 17025, HP_N = 17028 };
constexpr int kHpStride = 17088;  // HP_N rounded up to 64

struct DqArgs {
    int B, T, nct, C0;
    const float *params, *target;
    float* grad;
    const float *obs, *next;
    const int32_t* act;
    const float* rew;
    const uint8_t* done;
    pm_drqn_stats* stats;
    const int32_t* enable;
    float gamma;
    float *ZX;   // [3][nct][T][16][1024]     Zx in the recurrence's accumulator layout
    float *HS;   // [3][nct][T+1][32][128]    h_t per column (the hand-off slots; slot 0 unused)
    float *F1T;  // [64][C0]                  obs stream F1 (column c = t*B + b)
    float *F2T;  // [128][C0]                 obs stream F2
    float *H;    // [128][C0]                 obs stream h_t, the input hidden of step t
    float *GS;   // [nct][T][16][64][16]      obs stream activated gates, wave-0 lane layout
    float *CS;   // [nct][T][16][64][4]       obs stream c_{t+1}
    float *dZ;   // [512][C0]
    float *QP;   // [3][nct][16][32][4]       partial (V, A0, A1, A2) of each workgroup's 8 head rows
    float *DHP;  // [nct][T][16][32][128]     slot t: per-workgroup partials of dh_{t+1}
    float *HP;   // [nct][kHpStride]          head gradient partials per column tile
    float *LP;   // [nct][4]                  loss / q sums per column tile
    float *W2P;  // [C0 / 32][kLowN]          W1 / b1 / W2 / b2 gradient partials per column tile
    double* part;
    int64_t* tstep;
    int32_t* flags;  // [3][nct][16] forward | [3][nct][16] Q | [nct][16] backward | ticket
};

// workspace carve-up, 64-float aligned pieces
struct DqLayout {
    int64_t total = 0;
    int64_t add(int64_t floats) {
        const int64_t o = total;
        total += (floats + 63) / 64 * 64;
        return o;
    }
};

inline int64_t dq_layout(int B, int T, DqArgs* a, void* work) {
    const int64_t nct = B / 32, C0 = (int64_t)T * B;
    DqLayout L;
    const int64_t oZX = L.add(3 * nct * T * 16 * 1024), oHS = L.add(3 * nct * (T + 1) * 4096), oF1 = L.add(64 * C0),
                  oF2 = L.add(128 * C0), oH = L.add(128 * C0), oGS = L.add(nct * T * 16 * 1024),
                  oCS = L.add(nct * T * 16 * 256), odZ = L.add(512 * C0), oQP = L.add(3 * nct * 16 * 128),
                  oDHP = L.add(nct * T * 16 * 4096), oHP = L.add(nct * kHpStride), oLP = L.add(nct * 4),
                  oW2P = L.add(C0 / 32 * kLowN), oPart = L.add(2 * kNormBlocks), oTs = L.add(4),
                  oFl = L.add(7 * nct * 16 + 4);
    if (a && work) {
        float* w = static_cast<float*>(work);
        a->B = B; a->T = T; a->nct = (int)nct; a->C0 = (int)C0;
        a->ZX = w + oZX; a->HS = w + oHS; a->F1T = w + oF1; a->F2T = w + oF2; a->H = w + oH; a->GS = w + oGS;
        a->CS = w + oCS; a->dZ = w + odZ; a->QP = w + oQP; a->DHP = w + oDHP; a->HP = w + oHP; a->LP = w + oLP;
        a->W2P = w + oW2P; a->part = reinterpret_cast<double*>(w + oPart);
        a->tstep = reinterpret_cast<int64_t*>(w + oTs); a->flags = reinterpret_cast<int32_t*>(w + oFl);
    }
    return L.total * 4;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ bool skipped(const DqArgs& a) { return a.enable && *a.enable == 0; }

// ---------------------------------------------------------------- hand-off primitives
// Write-through (sc1) 16-byte stores and loads through a buffer resource (MI355X_MICROARCH.md,
// hand-off table row 1: every byte of a hand-off stored and loaded sc1, the flag an sc1 store by one
// lane after the storing wave's vmcnt(0), the consumer's poll an sc1 load).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
    typedef __attribute__((ext_vector_type(4))) float f4v;
    const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v) { store_f4_sc1(r, byte_off, v); }
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void flag_set(int32_t* f, int v) {
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Lanes [0, n) of the calling wave poll flags f[lane] (sc1 loads) until every one is >= need.
// Bounded: a wait that never completes sets status bit 1 and returns (the update is then void).
__device__ __forceinline__ void wait_flags(const int32_t* f, int n, int need, int lane, pm_drqn_stats* st) {
    bool ok = lane >= n;
    for (int it = 0; it < (1 << 21); ++it) {
        if (!ok) ok = __hip_atomic_load(f + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need;
        if (__all(ok)) return;
        __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) atomicOr(&st->status, 2);
}

// ---------------------------------------------------------------- 1: embedding + input projection
// grid: 3 streams x nct column tiles x T steps x 4 row quarters; wave w computes the Zx tile of
// recurrence workgroup m = 4 * quarter + w. Tile rows: row r' of workgroup m is gate r' >> 3 of LSTM
// unit 8m + (r' & 7), i.e. Wih / Whh row 128 (r' >> 3) + 8m + (r' & 7).
__global__ __launch_bounds__(256) void k_dq_embed(DqArgs a) {
    const int nct = a.nct, T = a.T, B = a.B;
    int bid = blockIdx.x;
    const int rq = bid & 3;
    bid >>= 2;
    const int t = bid % T;
    bid /= T;
    const int ct = bid % nct, s = bid / nct;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    if (blockIdx.x == 0)
        for (int i = tid; i < 7 * nct * 16 + 4; i += 256) a.flags[i] = 0;
    if (skipped(a)) {  // this replica contributes nothing to the all-reduce
        for (int i = blockIdx.x * 256 + tid; i < PM_RNN_NPARAM + 4; i += gridDim.x * 256) a.grad[i] = 0.f;
        return;
    }
    if (blockIdx.x == 0 && tid == 0) a.grad[PM_RNN_NPARAM] = 1.0f;
    __shared__ __attribute__((aligned(16))) float F2s[32][132];
    const float* P = s == 2 ? a.target : a.params;
    const int b = ct * 32 + col;
    const int64_t c = (int64_t)t * B + b;
    float xs[4];
    tile_inputs((s == 0 ? a.obs : a.next) + ((int64_t)b * T + t) * 7, h, xs);
    // F1 (both 32-row tiles, every wave): input k' = 2 s4 + h, k' = 0 the constant 1 (weight: b1)
    f32x16 c1[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
        const int row = 32 * jt + col;
        c1[jt] = f32x16{};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int kk = 2 * s4 + h;
            const float wv = kk == 0 ? P[R_P_F1B + row] : P[R_P_F1W + row * 7 + kk - 1];
            c1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, xs[s4], c1[jt], 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) c1[jt][r] = relu(c1[jt][r]);
    }
    // F2 tile w: rows 32w + rho(r) + 4h; K = 64 over the two F1 tiles (k = 32 t2 + rho(r) + 4h)
    f32x16 f2;
#pragma unroll
    for (int r = 0; r < 16; ++r) f2[r] = P[R_P_F2B + 32 * w + rho(r) + 4 * h];
    {
        const float* w2 = P + R_P_F2W + (32 * w + col) * 64 + 4 * h;
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = *reinterpret_cast<const float4*>(w2 + 32 * t2 + 8 * i);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, c1[t2][4 * i + 0], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, c1[t2][4 * i + 1], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, c1[t2][4 * i + 2], f2, 0, 0, 0);
                f2 = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, c1[t2][4 * i + 3], f2, 0, 0, 0);
            }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) f2[r] = relu(f2[r]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(&F2s[col][32 * w + 8 * i + 4 * h]) =
            make_float4(f2[4 * i], f2[4 * i + 1], f2[4 * i + 2], f2[4 * i + 3]);
    if (s == 0 && rq == 0) {  // the obs stream's features for the weight gradients, [unit][column]
        const int64_t C0 = a.C0;
#pragma unroll
        for (int r = 0; r < 16; ++r) a.F2T[(int64_t)(32 * w + rho(r) + 4 * h) * C0 + c] = f2[r];
        if (w < 2)
#pragma unroll
            for (int r = 0; r < 16; ++r) a.F1T[(int64_t)(32 * w + rho(r) + 4 * h) * C0 + c] = c1[w][r];
    }
    __syncthreads();
    // Zx tile of recurrence workgroup m: K = 128 with k = 8j + 4h + e for k-step (j, e)
    const int m = 4 * rq + w;
    f32x16 z;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rr = rho(r) + 4 * h;
        const int g = 128 * (rr >> 3) + 8 * m + (rr & 7);
        z[r] = P[R_P_BIH + g] + P[R_P_BHH + g];
    }
    const float* wr = P + R_P_WIH + (int64_t)(128 * (col >> 3) + 8 * m + (col & 7)) * 128 + 4 * h;
    float4 av[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) av[j] = *reinterpret_cast<const float4*>(wr + 8 * j);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(&F2s[col][8 * j + 4 * h]);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].x, bv.x, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].y, bv.y, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].z, bv.z, z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j].w, bv.w, z, 0, 0, 0);
    }
    float4* zx = reinterpret_cast<float4*>(a.ZX + ((((int64_t)s * nct + ct) * T + t) * 16 + m) * 1024) + lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) zx[64 * i] = make_float4(z[4 * i], z[4 * i + 1], z[4 * i + 2], z[4 * i + 3]);
}

// ---------------------------------------------------------------- 2: the recurrence (persistent)
struct RecurSmem {
    float red[3][16][64];                            // partial accumulators of waves 1..3
    __attribute__((aligned(16))) float dzs[4][64][4];  // BPTT: wave 0's dz fragments for the other waves
    __attribute__((aligned(16))) float hT[32][132];  // h_T of this column tile [column][unit]
    float dS[8][32];                                 // dS of this workgroup's 8 shared-head rows
    float ws[8][128];                                // those rows of the effective W_S
};

__device__ __forceinline__ float eff_w(const float* P, int mu, int sg, int ep, bool noisy) {
    return noisy ? P[mu] + P[sg] * P[ep] : P[mu];  // NoisyLinear: mu + sigma * epsilon (train), mu (eval)
}

__global__ __launch_bounds__(256) void k_dq_recur(DqArgs a) {
    if (skipped(a)) return;
    __shared__ RecurSmem sm;
    const int nct = a.nct, T = a.T, B = a.B;
    int bid = blockIdx.x;
    const int m = bid & 15;
    bid >>= 4;
    const int ct = bid % nct, so = bid / nct;
    const int s = so == 2 ? 0 : so + 1;  // streams 1 and 2 first: the obs stream's group waits for them
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const bool noisy = s != 2;  // modelB in train mode, targetB in eval mode
    const float* P = s == 2 ? a.target : a.params;
    const int64_t C0 = a.C0;
    const int bcol = ct * 32 + col;
    const int grp = s * nct + ct;
    float* HSg = a.HS + (int64_t)grp * (T + 1) * 4096;
    const __amdgpu_buffer_rsrc_t rHS = rsrc(HSg);
    int32_t* fl = a.flags + grp * 16;
    // this wave's Whh fragments: row 128 q + 8m + j of lane row col (q = col >> 3, j = col & 7), K quarter w
    float wa[16];
    {
        const float* wr = P + R_P_WHH + (int64_t)(128 * (col >> 3) + 8 * m + (col & 7)) * 128 + 32 * w + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 v = *reinterpret_cast<const float4*>(wr + 8 * j);
            wa[4 * j] = v.x; wa[4 * j + 1] = v.y; wa[4 * j + 2] = v.z; wa[4 * j + 3] = v.w;
        }
    }
    const float4* zx = reinterpret_cast<const float4*>(a.ZX + ((int64_t)grp * T * 16 + m) * 1024) + lane;
    float cst[4] = {0.f, 0.f, 0.f, 0.f};  // wave 0: c of units 8m + 4h + e, column col
    float4 zn[4];
    if (w == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) zn[i] = zx[64 * i];
    // ---------------- forward
    for (int t = 0; t < T; ++t) {
        f32x16 acc = {};
        if (w == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { acc[4 * i] = zn[i].x; acc[4 * i + 1] = zn[i].y; acc[4 * i + 2] = zn[i].z; acc[4 * i + 3] = zn[i].w; }
            if (t + 1 < T)
#pragma unroll
                for (int i = 0; i < 4; ++i) zn[i] = zx[(int64_t)(t + 1) * 16 * 256 + 64 * i];
        }
        if (t > 0) {
            if (w == 0) wait_flags(fl, 16, t, lane, a.stats);
            __syncthreads();  // h_t published by the whole group
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 hv = ld_sc1(rHS, ((t * 32 + col) * 128 + 32 * w + 8 * j + 4 * h) * 4);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * j + 0], hv.x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * j + 1], hv.y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * j + 2], hv.z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * j + 3], hv.w, acc, 0, 0, 0);
            }
            if (w > 0)
#pragma unroll
                for (int r = 0; r < 16; ++r) sm.red[w - 1][r][lane] = acc[r];
            __syncthreads();
        }
        if (w != 0) continue;
        // wave 0: the cell of units 8m + 4h + e (gate q in register 4q + e), column col
        float hn[4], gt[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float z = acc[r];
            if (t > 0) z = ((z + sm.red[0][r][lane]) + sm.red[1][r][lane]) + sm.red[2][r][lane];
            gt[r] = (r >> 2) == 2 ? tanhf(z) : sigm(z);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            cst[e] = gt[4 + e] * cst[e] + gt[e] * gt[8 + e];  // cy = forgetgate * cx + ingate * cellgate
            hn[e] = gt[12 + e] * tanhf(cst[e]);
        }
        st_sc1(rHS, (((t + 1) * 32 + col) * 128 + 8 * m + 4 * h) * 4, make_float4(hn[0], hn[1], hn[2], hn[3]));
        if (s == 0) {  // what BPTT and the weight gradients need of the obs stream
            float4* g4 = reinterpret_cast<float4*>(a.GS + (((int64_t)ct * T + t) * 16 + m) * 1024) + lane;
#pragma unroll
            for (int i = 0; i < 4; ++i) g4[64 * i] = make_float4(gt[4 * i], gt[4 * i + 1], gt[4 * i + 2], gt[4 * i + 3]);
            reinterpret_cast<float4*>(a.CS + (((int64_t)ct * T + t) * 16 + m) * 256)[lane] =
                make_float4(cst[0], cst[1], cst[2], cst[3]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float* hr = a.H + (int64_t)(8 * m + 4 * h + e) * C0 + bcol;
                if (t + 1 < T) hr[(int64_t)(t + 1) * B] = hn[e];
                if (t == 0) hr[0] = 0.f;
            }
        }
        drain();
        if (lane == 0) flag_set(fl + m, t + 1);
    }
    // ---------------- heads: rows 8m .. 8m+7 of the shared head (A rows duplicated x4 in the tile)
    if (w == 0) wait_flags(fl, 16, T, lane, a.stats);
    __syncthreads();  // h_T published
    f32x16 sacc = {};
    {
        const int u = 8 * m + (col & 7);  // S row of lane row col
        const int kb = 32 * w + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 hv = ld_sc1(rHS, ((T * 32 + col) * 128 + kb + 8 * j) * 4);
            *reinterpret_cast<float4*>(&sm.hT[col][kb + 8 * j]) = hv;
            const int k0 = u * 128 + kb + 8 * j;
            float wv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) wv[e] = eff_w(P, R_P_SWMU + k0 + e, R_P_SWSG + k0 + e, R_P_SWEP + k0 + e, noisy);
            sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[0], hv.x, sacc, 0, 0, 0);
            sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[1], hv.y, sacc, 0, 0, 0);
            sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[2], hv.z, sacc, 0, 0, 0);
            sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[3], hv.w, sacc, 0, 0, 0);
        }
    }
    if (w > 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.red[w - 1][r][lane] = sacc[r];
    __syncthreads();
    // wave 0: S rows u_e = 8m + 4h + e (registers r = e), their V / A partials
    float sv[4], sr[4];
    float* QPs = a.QP + (int64_t)grp * 16 * 128;
    if (w == 0) {
        float pv = 0.f, pa0 = 0.f, pa1 = 0.f, pa2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int u = 8 * m + 4 * h + e;
            const float z = ((sacc[e] + sm.red[0][e][lane]) + sm.red[1][e][lane]) + sm.red[2][e][lane];
            sv[e] = z + eff_w(P, R_P_SBMU + u, R_P_SBSG + u, R_P_SBEP + u, noisy);
            sr[e] = relu(sv[e]);
            pv = fmaf(eff_w(P, R_P_VWMU + u, R_P_VWSG + u, R_P_VWEP + u, noisy), sr[e], pv);
            pa0 = fmaf(eff_w(P, R_P_AWMU + u, R_P_AWSG + u, R_P_AWEP + u, noisy), sr[e], pa0);
            pa1 = fmaf(eff_w(P, R_P_AWMU + 128 + u, R_P_AWSG + 128 + u, R_P_AWEP + 128 + u, noisy), sr[e], pa1);
            pa2 = fmaf(eff_w(P, R_P_AWMU + 256 + u, R_P_AWSG + 256 + u, R_P_AWEP + 256 + u, noisy), sr[e], pa2);
        }
        pv += __shfl_xor(pv, 32);
        pa0 += __shfl_xor(pa0, 32);
        pa1 += __shfl_xor(pa1, 32);
        pa2 += __shfl_xor(pa2, 32);
        if (h == 0) st_sc1(rsrc(QPs), (m * 32 + col) * 16, make_float4(pv, pa0, pa1, pa2));
        drain();
        if (lane == 0) flag_set(a.flags + 3 * nct * 16 + grp * 16 + m, 1);
    }
    if (s != 0) return;  // block-uniform: the next-state streams are done
    // ---------------- the loss and the head gradients (obs stream), on wave 0
    float dV = 0.f, dA[3] = {0.f, 0.f, 0.f};
    if (w == 0) {
        const int32_t* fq = a.flags + 3 * nct * 16;
        // lanes [0, 48): stream (lane >> 4), workgroup (lane & 15) of this column tile
        {
            const int sl = lane >> 4;
            bool ok = lane >= 48;
            for (int it = 0; it < (1 << 21); ++it) {
                if (!ok) ok = __hip_atomic_load(fq + (sl * nct + ct) * 16 + (lane & 15), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) >= 1;
                if (__all(ok)) break;
                __builtin_amdgcn_s_sleep(1);
                if (it == (1 << 21) - 1 && lane == 0) atomicOr(&a.stats->status, 2);
            }
        }
        float q[3][3];
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            const float* QPst = a.QP + (int64_t)(st * nct + ct) * 16 * 128;
            const __amdgpu_buffer_rsrc_t rq = rsrc(QPst);
            float v = 0.f, x0 = 0.f, x1 = 0.f, x2 = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {  // this lane half's 8 workgroups, in order
                const float4 p = ld_sc1(rq, ((8 * h + k) * 32 + col) * 16);
                v += p.x; x0 += p.y; x1 += p.z; x2 += p.w;
            }
            v += __shfl_xor(v, 32);  // + the other half (commutative: both halves agree bit for bit)
            x0 += __shfl_xor(x0, 32);
            x1 += __shfl_xor(x1, 32);
            x2 += __shfl_xor(x2, 32);
            const float* Pst = st == 2 ? a.target : a.params;
            const bool nz = st != 2;
            v += eff_w(Pst, R_P_VBMU, R_P_VBSG, R_P_VBEP, nz);
            x0 += eff_w(Pst, R_P_ABMU + 0, R_P_ABSG + 0, R_P_ABEP + 0, nz);
            x1 += eff_w(Pst, R_P_ABMU + 1, R_P_ABSG + 1, R_P_ABEP + 1, nz);
            x2 += eff_w(Pst, R_P_ABMU + 2, R_P_ABSG + 2, R_P_ABEP + 2, nz);
            const float mean = ((x0 + x1) + x2) / 3.0f;  // A.mean(dim=1)
            q[st][0] = v + (x0 - mean);
            q[st][1] = v + (x1 - mean);
            q[st][2] = v + (x2 - mean);
        }
        const int64_t jl = (int64_t)bcol * T + T - 1;  // the sequence's last step
        const int ac = a.act[jl];
        const float rl = a.rew[jl], dl = a.done[jl] ? 1.f : 0.f;
        const float qa = ac == 0 ? q[0][0] : (ac == 1 ? q[0][1] : q[0][2]);
        const int as = argmax3(q[1]);  // argmax Q_B(next) (first max)
        const float y = rl + a.gamma * q[2][as] * (1.0f - dl);
        const float d = qa - y, ad = fabsf(d);
        float lv = ad < 1.0f ? 0.5f * d * d : ad - 0.5f;  // smooth_l1, beta 1
        const float gq = fminf(fmaxf(d, -1.0f), 1.0f) / (float)B;
        dV = gq;
#pragma unroll
        for (int k = 0; k < 3; ++k) dA[k] = (k == ac ? gq : 0.f) - gq / 3.0f;
        if (m == 0) {  // loss / q sums of this column tile (lanes of half 0)
            float qs = qa;
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) { lv += __shfl_xor(lv, o); qs += __shfl_xor(qs, o); }
            if (lane == 0) { a.LP[ct * 4 + 0] = lv; a.LP[ct * 4 + 1] = qs; }
        }
        // dS of rows u_e (modelB's effective V / A weights), the head gradients of those rows
        float* HPc = a.HP + (int64_t)ct * kHpStride;
        float gv[4], ga[3][4], gb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int u = 8 * m + 4 * h + e;
            const float* Q = a.params;
            const float ds = eff_w(Q, R_P_VWMU + u, R_P_VWSG + u, R_P_VWEP + u, true) * dV +
                             eff_w(Q, R_P_AWMU + u, R_P_AWSG + u, R_P_AWEP + u, true) * dA[0] +
                             eff_w(Q, R_P_AWMU + 128 + u, R_P_AWSG + 128 + u, R_P_AWEP + 128 + u, true) * dA[1] +
                             eff_w(Q, R_P_AWMU + 256 + u, R_P_AWSG + 256 + u, R_P_AWEP + 256 + u, true) * dA[2];
            const float dsm = sv[e] > 0.f ? ds : 0.f;
            sm.dS[4 * h + e][col] = dsm;
            gv[e] = dV * sr[e];
            ga[0][e] = dA[0] * sr[e];
            ga[1][e] = dA[1] * sr[e];
            ga[2][e] = dA[2] * sr[e];
            gb[e] = dsm;
        }
        // sums over the 32 columns of the half (fixed butterfly)
#pragma unroll
        for (int o = 16; o > 0; o >>= 1)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                gv[e] += __shfl_xor(gv[e], o);
                ga[0][e] += __shfl_xor(ga[0][e], o);
                ga[1][e] += __shfl_xor(ga[1][e], o);
                ga[2][e] += __shfl_xor(ga[2][e], o);
                gb[e] += __shfl_xor(gb[e], o);
            }
        if (col == 0)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int u = 8 * m + 4 * h + e;
                HPc[HP_V + u] = gv[e];
                HPc[HP_A + u] = ga[0][e];
                HPc[HP_A + 128 + u] = ga[1][e];
                HPc[HP_A + 256 + u] = ga[2][e];
                HPc[HP_BS + u] = gb[e];
            }
        if (m == 0) {
            float sb = dV, sa0 = dA[0], sa1 = dA[1], sa2 = dA[2];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) {
                sb += __shfl_xor(sb, o); sa0 += __shfl_xor(sa0, o); sa1 += __shfl_xor(sa1, o); sa2 += __shfl_xor(sa2, o);
            }
            if (lane == 0) { HPc[HP_VB] = sb; HPc[HP_AB] = sa0; HPc[HP_AB + 1] = sa1; HPc[HP_AB + 2] = sa2; }
        }
    }
    // this workgroup's rows of modelB's effective W_S (for dh_T)
    for (int k = tid; k < 8 * 128; k += 256) {
        const int u = 8 * m + (k >> 7), kk = k & 127, o = u * 128 + kk;
        sm.ws[k >> 7][kk] = eff_w(a.params, R_P_SWMU + o, R_P_SWSG + o, R_P_SWEP + o, true);
    }
    __syncthreads();  // dS, h_T, ws
    {   // dW_S rows (partial over this column tile): thread (k', row half)
        const int kk = tid & 127, hr = tid >> 7;
        float g4[4] = {0.f, 0.f, 0.f, 0.f};
        for (int c2 = 0; c2 < 32; ++c2) {
            const float hv = sm.hT[c2][kk];
#pragma unroll
            for (int e = 0; e < 4; ++e) g4[e] = fmaf(sm.dS[4 * hr + e][c2], hv, g4[e]);
        }
        float* HPc = a.HP + (int64_t)ct * kHpStride;
#pragma unroll
        for (int e = 0; e < 4; ++e) HPc[HP_WS + (8 * m + 4 * hr + e) * 128 + kk] = g4[e];
    }
    const __amdgpu_buffer_rsrc_t rDH = rsrc(a.DHP + (int64_t)ct * T * 16 * 4096);
    {   // dh_T partial over this workgroup's 8 rows: thread (column, 16 units)
        const int c2 = tid >> 3, u0 = (tid & 7) * 16;
        float o16[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) o16[k] = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float ds = sm.dS[r][c2];
#pragma unroll
            for (int k = 0; k < 16; ++k) o16[k] = fmaf(sm.ws[r][u0 + k], ds, o16[k]);
        }
        const int base = (((T - 1) * 16 + m) * 32 + c2) * 128 + u0;
#pragma unroll
        for (int i = 0; i < 4; ++i) st_sc1(rDH, (base + 4 * i) * 4, make_float4(o16[4 * i], o16[4 * i + 1], o16[4 * i + 2], o16[4 * i + 3]));
    }
    drain();
    __syncthreads();
    int32_t* fb = a.flags + 6 * nct * 16 + ct * 16;
    if (tid == 0) flag_set(fb + m, 1);
    // ---------------- BPTT
    // Whh^T fragments of this wave's output tile (units u' = 32w + col): k-step r covers gate rows
    // rho(r) + 4h of this workgroup's tile, i.e. Whh row 128 (r >> 2) + 8m + (r & 3) + 4h
    float wt[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
        wt[r] = a.params[R_P_WHH + (int64_t)(128 * (r >> 2) + 8 * m + (r & 3) + 4 * h) * 128 + 32 * w + col];
    float dc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = T - 1; t >= 0; --t) {
        float dz[16];
        if (w == 0) {
            const float4* g4 = reinterpret_cast<const float4*>(a.GS + (((int64_t)ct * T + t) * 16 + m) * 1024) + lane;
            float gt[16];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = g4[64 * i];
                gt[4 * i] = v.x; gt[4 * i + 1] = v.y; gt[4 * i + 2] = v.z; gt[4 * i + 3] = v.w;
            }
            const float4 cn = reinterpret_cast<const float4*>(a.CS + (((int64_t)ct * T + t) * 16 + m) * 256)[lane];
            const float4 cp = t > 0 ? reinterpret_cast<const float4*>(a.CS + (((int64_t)ct * T + t - 1) * 16 + m) * 256)[lane]
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
            const float cT[4] = {cn.x, cn.y, cn.z, cn.w}, cP[4] = {cp.x, cp.y, cp.z, cp.w};
            wait_flags(fb, 16, T - t, lane, a.stats);
            float dh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 16; ++k) {  // the 16 workgroups' partials of dh_{t+1}, in order
                const float4 p = ld_sc1(rDH, (((t * 16 + k) * 32 + col) * 128 + 8 * m + 4 * h) * 4);
                dh[0] += p.x; dh[1] += p.y; dh[2] += p.z; dh[3] += p.w;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float gi = gt[e], gf = gt[4 + e], gg = gt[8 + e], go = gt[12 + e];
                const float tc = tanhf(cT[e]);
                const float dcc = dc[e] + dh[e] * go * (1.0f - tc * tc);
                dz[e] = dcc * gg * (gi * (1.0f - gi));
                dz[4 + e] = dcc * cP[e] * (gf * (1.0f - gf));
                dz[8 + e] = dcc * gi * (1.0f - gg * gg);
                dz[12 + e] = dh[e] * tc * (go * (1.0f - go));
                dc[e] = dcc * gf;
            }
            const int64_t cc = (int64_t)t * B + bcol;
#pragma unroll
            for (int r = 0; r < 16; ++r) a.dZ[(int64_t)(128 * (r >> 2) + 8 * m + 4 * h + (r & 3)) * C0 + cc] = dz[r];
            if (t > 0)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    *reinterpret_cast<float4*>(&sm.dzs[i][lane][0]) = make_float4(dz[4 * i], dz[4 * i + 1], dz[4 * i + 2], dz[4 * i + 3]);
        }
        if (t == 0) break;  // dh_0 (the zero initial state) is not needed
        __syncthreads();  // dz fragments
        if (w != 0)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = *reinterpret_cast<const float4*>(&sm.dzs[i][lane][0]);
                dz[4 * i] = v.x; dz[4 * i + 1] = v.y; dz[4 * i + 2] = v.z; dz[4 * i + 3] = v.w;
            }
        f32x16 acc = {};
        // r-th k-step: this workgroup's gate rows rho(r) + 4h (the accumulator layout of dz)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt[r], dz[r], acc, 0, 0, 0);
        const int base = (((t - 1) * 16 + m) * 32 + col) * 128 + 32 * w + 4 * h;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            st_sc1(rDH, (base + 8 * i) * 4, make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]));
        drain();
        __syncthreads();
        if (tid == 0) flag_set(fb + m, T - t + 1);
    }
}

// ---------------------------------------------------------------- 3: weight gradients
struct WgSmem {
    union {
        float red[16][16][64];          // type A: per-wave partial tiles
        struct {
            float red2[4][128][33];     // type B: dF2 K-quarter partials, later dF1 partials
            float dP2[128][33];
            float dP1[64][33];
            float F1s[64][33];
        } b;
    };
    float rs[16][64];
    int last;
};

__global__ __launch_bounds__(1024) void k_dq_wgrad(DqArgs a) {
    if (skipped(a)) return;
    __shared__ WgSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
    const int64_t C0 = a.C0;
    const int B = a.B, T = a.T, nct = a.nct;
    const int nB = a.C0 / 32;
    int bid = blockIdx.x;
    if (bid < kWgA) {
        // ---- dWih (mat 0) / dWhh (mat 1) tile: rows g in [32 gt, +32), columns k' in [32 kt, +32)
        const int mat = bid >> 6, gt = (bid >> 2) & 15, kt = bid & 3;
        const float* Ar = a.dZ + (int64_t)(32 * gt + col) * C0 + 4 * h;
        const float* Br = (mat == 0 ? a.F2T : a.H) + (int64_t)(32 * kt + col) * C0 + 4 * h;
        f32x16 acc = {};
        float rsum = 0.f;
        for (int kc = w; kc * 8 < C0; kc += 16) {  // 8-column chunks, round robin over the waves
            const float4 av = *reinterpret_cast<const float4*>(Ar + 8 * kc);
            const float4 bv = *reinterpret_cast<const float4*>(Br + 8 * kc);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc, 0, 0, 0);
            rsum += ((av.x + av.y) + av.z) + av.w;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sm.red[w][r][lane] = acc[r];
        sm.rs[w][lane] = rsum;
        __syncthreads();
        if (w == 0) {
            float* G = a.grad + (mat == 0 ? R_P_WIH : R_P_WHH);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = sm.red[0][r][lane];
                for (int k = 1; k < 16; ++k) v += sm.red[k][r][lane];
                G[(int64_t)(32 * gt + rho(r) + 4 * h) * 128 + 32 * kt + col] = v;
            }
            if (mat == 0 && kt == 0) {  // db_ih = db_hh = row sums of dZ
                float v = sm.rs[0][lane];
                for (int k = 1; k < 16; ++k) v += sm.rs[k][lane];
                v += __shfl_xor(v, 32);
                if (h == 0) { a.grad[R_P_BIH + 32 * gt + col] = v; a.grad[R_P_BHH + 32 * gt + col] = v; }
            }
        }
        return;
    }
    bid -= kWgA;
    if (bid < nB) {
        // ---- column tile: columns [c0, c0 + 32) (one time step t, batch rows b0 .. b0 + 31)
        const int64_t c0 = (int64_t)bid * 32;
        const int t = (int)(c0 / B), b0 = (int)(c0 % B);
        // dF2 = Wih^T dZ: wave (out tile ot = w & 3, K quarter kq = w >> 2), k = g = 128 kq + 2p + h
        {
            const int ot = w & 3, kq = w >> 2;
            f32x16 acc = {};
            const float* Wc = a.params + R_P_WIH + 32 * ot + col;
            const float* Zc = a.dZ + c0 + col;
#pragma unroll 8
            for (int p = 0; p < 64; ++p) {
                const int g = 128 * kq + 2 * p + h;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Wc[(int64_t)g * 128], Zc[(int64_t)g * C0], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) sm.b.red2[kq][32 * ot + rho(r) + 4 * h][col] = acc[r];
        }
        for (int k = tid; k < 64 * 32; k += 1024) sm.b.F1s[k >> 5][k & 31] = a.F1T[(int64_t)(k >> 5) * C0 + c0 + (k & 31)];
        __syncthreads();
        for (int k = tid; k < 128 * 32; k += 1024) {
            const int u = k >> 5, c2 = k & 31;
            const float v = ((sm.b.red2[0][u][c2] + sm.b.red2[1][u][c2]) + sm.b.red2[2][u][c2]) + sm.b.red2[3][u][c2];
            sm.b.dP2[u][c2] = a.F2T[(int64_t)u * C0 + c0 + c2] > 0.f ? v : 0.f;  // through the ReLU
        }
        __syncthreads();
        float* Wp = a.W2P + (int64_t)bid * kLowN;
        {   // dW2 partial [k'][j] = sum_c dP2[k'][c] F1[j][c]; db2 partial
            const int u = tid >> 3, j0 = (tid & 7) * 8;
            float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int c2 = 0; c2 < 32; ++c2) {
                const float d = sm.b.dP2[u][c2];
#pragma unroll
                for (int k = 0; k < 8; ++k) o8[k] = fmaf(d, sm.b.F1s[j0 + k][c2], o8[k]);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) Wp[R_P_F2W + u * 64 + j0 + k] = o8[k];
            if ((tid & 7) == 0) {
                float sb = 0.f;
                for (int c2 = 0; c2 < 32; ++c2) sb += sm.b.dP2[u][c2];
                Wp[R_P_F2B + u] = sb;
            }
        }
        {   // dF1 = W2^T dP2: wave (out tile jt = w & 1, K eighth ke = w >> 1), k = k' = 16 ke + 2p + h
            const int jt = w & 1, ke = w >> 1;
            f32x16 acc = {};
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                const int k = 16 * ke + 2 * p + h;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.params[R_P_F2W + k * 64 + 32 * jt + col], sm.b.dP2[k][col], acc, 0, 0, 0);
            }
            __syncthreads();  // red2 is free again (the dP2 pass is done)
#pragma unroll
            for (int r = 0; r < 16; ++r) sm.b.red2[ke >> 1][(ke & 1) * 64 + 32 * jt + rho(r) + 4 * h][col] = acc[r];
        }
        __syncthreads();
        for (int k = tid; k < 64 * 32; k += 1024) {
            const int j = k >> 5, c2 = k & 31;
            float v = 0.f;
#pragma unroll
            for (int ke = 0; ke < 8; ++ke) v += sm.b.red2[ke >> 1][(ke & 1) * 64 + j][c2];
            sm.b.dP1[j][c2] = sm.b.F1s[j][c2] > 0.f ? v : 0.f;
        }
        __syncthreads();
        if (tid < 448) {  // dW1 partial [j][i] = sum_c dP1[j][c] x_i[c]
            const int j = tid / 7, i = tid % 7;
            float v = 0.f;
            for (int c2 = 0; c2 < 32; ++c2) v = fmaf(sm.b.dP1[j][c2], a.obs[((int64_t)(b0 + c2) * T + t) * 7 + i], v);
            Wp[R_P_F1W + j * 7 + i] = v;
        } else if (tid < 512) {
            const int j = tid - 448;
            float v = 0.f;
            for (int c2 = 0; c2 < 32; ++c2) v += sm.b.dP1[j][c2];
            Wp[R_P_F1B + j] = v;
        }
        // arrival ticket: the last column tile sums every tile's partials in tile order
        drain();
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            drain();
            const int k = atomicAdd(a.flags + 7 * nct * 16, 1);
            sm.last = k == nB - 1;
            if (sm.last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            drain();
        }
        __syncthreads();
        if (!sm.last) return;
        for (int i = tid; i < kLowN; i += 1024) {
            float v = 0.f;
            for (int k = 0; k < nB; ++k) v += a.W2P[(int64_t)k * kLowN + i];
            a.grad[i] = v;
        }
        return;
    }
    bid -= nB;
    // ---- head partials: sum over column tiles in order
    const int per = (HP_N + kWgC - 1) / kWgC, lo = bid * per, hi = min(HP_N, lo + per);
    for (int i = lo + tid; i < hi; i += 1024) {
        float v = 0.f;
        for (int k = 0; k < nct; ++k) v += a.HP[(int64_t)k * kHpStride + i];
        int dst;
        if (i < HP_BS) dst = R_P_SWMU + i;
        else if (i < HP_V) dst = R_P_SBMU + i - HP_BS;
        else if (i < HP_VB) dst = R_P_VWMU + i - HP_V;
        else if (i == HP_VB) dst = R_P_VBMU;
        else if (i < HP_AB) dst = R_P_AWMU + i - HP_A;
        else dst = R_P_ABMU + i - HP_AB;
        a.grad[dst] = v;
    }
    if (bid == 0 && tid == 0) {
        float ls = 0.f, qs = 0.f;
        for (int k = 0; k < nct; ++k) { ls += a.LP[k * 4]; qs += a.LP[k * 4 + 1]; }
        a.stats->loss = ls / (float)B;
        a.stats->q_mean = qs / (float)B;
    }
}

// NoisyLinear sigma gradients: d sigma = dW * epsilon (NoisyLinear.forward :45-46). Linear in the
// mu gradient with the same epsilon on every rank, so it is formed after the all-reduce (apply).
__device__ __forceinline__ int sigma_source(int i, int& ep) {
    if (i >= R_P_SWSG && i < R_P_SWSG + 16384) { ep = R_P_SWEP + i - R_P_SWSG; return R_P_SWMU + i - R_P_SWSG; }
    if (i >= R_P_SBSG && i < R_P_SBSG + 128) { ep = R_P_SBEP + i - R_P_SBSG; return R_P_SBMU + i - R_P_SBSG; }
    if (i >= R_P_VWSG && i < R_P_VWSG + 128) { ep = R_P_VWEP + i - R_P_VWSG; return R_P_VWMU + i - R_P_VWSG; }
    if (i == R_P_VBSG) { ep = R_P_VBEP; return R_P_VBMU; }
    if (i >= R_P_AWSG && i < R_P_AWSG + 384) { ep = R_P_AWEP + i - R_P_AWSG; return R_P_AWMU + i - R_P_AWSG; }
    if (i >= R_P_ABSG && i < R_P_ABSG + 3) { ep = R_P_ABEP + i - R_P_ABSG; return R_P_ABMU + i - R_P_ABSG; }
    return -1;
}

// ---------------------------------------------------------------- clip + Adam
__global__ __launch_bounds__(256) void k_drqn_norm(DqArgs a) {
    __shared__ double red[256];
    const float ranks = a.grad[PM_RNN_NPARAM];  // replicas that contributed (summed by the all-reduce)
    if (!(ranks > 0.f)) return;
    const float inv_world = 1.0f / ranks;
    const int n = PM_RNN_NPARAM, per = (n + kNormBlocks - 1) / kNormBlocks;
    const int lo = blockIdx.x * per, hi = min(n, lo + per);
    double s = 0.0;
#pragma unroll 4
    for (int i = lo + threadIdx.x; i < hi; i += 256) {
        int ep;
        const int src = i >= R_P_SWSG ? sigma_source(i, ep) : -1;
        float graw = a.grad[i];
        if (src >= 0) {
            graw = a.grad[src] * a.params[ep];
            a.grad[i] = graw;
        }
        const float g = graw * inv_world;
        s += (double)g * (double)g;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.part[blockIdx.x] = red[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // tstep[0]: train step (target sync), tstep[1]: Adam t
        const int64_t ts = a.stats->steps + 1, at = a.stats->adam_t + 1;
        a.tstep[0] = ts;
        a.tstep[1] = at;
        a.stats->steps = ts;
        a.stats->adam_t = at;
    }
}

struct AdamK {
    double lr, beta1, beta2, eps, max_norm;
    int64_t interval;
};

__global__ __launch_bounds__(256) void k_drqn_adam(DqArgs a, AdamK k, float* params, float* target, float* m_,
                                                   float* v_) {
    __shared__ float cf[3];
    __shared__ int64_t ts_s;
    const float ranks = a.grad[PM_RNN_NPARAM];
    if (!(ranks > 0.f)) return;
    const float inv_world = 1.0f / ranks;
    __shared__ double ps[kNormBlocks];
    if (threadIdx.x < kNormBlocks) ps[threadIdx.x] = a.part[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        double ss = 0.0;
        for (int j = 0; j < kNormBlocks; ++j) ss += ps[j];
        const float norm = (float)sqrt(ss);
        const float coef = (float)(k.max_norm / ((double)norm + 1e-6));  // clip_coef
        const int64_t ts = a.tstep[0], at = a.tstep[1];
        const double bc1 = 1.0 - pow(k.beta1, (double)at), bc2 = 1.0 - pow(k.beta2, (double)at);
        cf[0] = coef < 1.0f ? coef : 1.0f;  // clamp(clip_coef, max=1)
        cf[1] = (float)(k.lr / bc1);
        cf[2] = (float)sqrt(bc2);
        ts_s = ts;
        if (blockIdx.x == 0) a.stats->norm = norm;
    }
    __syncthreads();
    const float coef = cf[0], step_size = cf[1], bc2s = cf[2];
    const bool sync = ts_s % k.interval == 0;  // targetB.load_state_dict(modelB.state_dict()) (:529-530)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < PM_RNN_NP; i += gridDim.x * blockDim.x) {
        if (i < PM_RNN_NPARAM) {
            const float g = (a.grad[i] * inv_world) * coef;
            float m = m_[i], v = v_[i], p = params[i];
            m = m + (float)(1.0 - k.beta1) * (g - m);                 // exp_avg.lerp_(grad, 1-beta1)
            v = v * (float)k.beta2 + (float)(1.0 - k.beta2) * g * g;  // mul_(beta2).addcmul_(g, g, 1-beta2)
            const float denom = sqrtf(v) / bc2s + (float)k.eps;
            p = p - step_size * (m / denom);
            params[i] = p;
            m_[i] = m;
            v_[i] = v;
            if (sync) target[i] = p;
        } else if (sync) {
            target[i] = params[i];  // the epsilon buffers
        }
    }
}

int check(const pm_drqn* d) {
    PM_REQUIRE(d, PM_E_ARG, "pm_drqn: null descriptor");
    PM_REQUIRE(d->params && d->target && d->adam_m && d->adam_v && d->grad && d->work && d->stats, PM_E_ARG,
               "pm_drqn: null buffer");
    PM_REQUIRE(d->batch >= 32 && d->batch <= 256 && d->batch % 32 == 0, PM_E_SIZE,
               "pm_drqn: batch %d (multiple of 32 in [32, 256])", d->batch);
    PM_REQUIRE(d->T >= 1 && d->T <= 64, PM_E_SIZE, "pm_drqn: T %d (1..64)", d->T);
    PM_REQUIRE(d->target_update_interval >= 1, PM_E_ARG, "pm_drqn: target_update_interval");
    PM_REQUIRE(((((uintptr_t)d->params) | ((uintptr_t)d->target) | ((uintptr_t)d->grad) | ((uintptr_t)d->work)) & 15) == 0,
               PM_E_ARG, "pm_drqn: params / target / grad / work must be 16-byte aligned");
    return PM_OK;
}

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" int64_t pm_drqn_work_bytes(int32_t batch, int32_t T) {
    if (batch < 32 || batch % 32 || T < 1) return -1;
    return dq_layout(batch, T, nullptr, nullptr);
}

extern "C" int pm_drqn_grads(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    PM_REQUIRE(d->obs && d->next && d->act && d->rew && d->done, PM_E_ARG, "pm_drqn_grads: null batch");
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats; a.enable = d->enable;
    a.obs = d->obs; a.next = d->next; a.act = d->act; a.rew = d->rew; a.done = d->done;
    a.gamma = (float)d->gamma;
    hipLaunchKernelGGL(k_dq_embed, dim3(3 * a.nct * a.T * 4), dim3(256), 0, st, a);
    PM_LAUNCHED("k_dq_embed");
    pm_launch(PM_TIMER_DRQN, k_dq_recur, dim3(3 * a.nct * kG), dim3(256), st, a);
    PM_LAUNCHED("k_dq_recur");
    hipLaunchKernelGGL(k_dq_wgrad, dim3(kWgA + a.C0 / 32 + kWgC), dim3(1024), 0, st, a);
    PM_LAUNCHED("k_dq_wgrad");
    return PM_OK;
}

extern "C" int pm_drqn_apply(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    hipStream_t st = pm_stream(stream);
    DqArgs a{};
    dq_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats;
    hipLaunchKernelGGL(k_drqn_norm, dim3(kNormBlocks), dim3(256), 0, st, a);
    PM_LAUNCHED("k_drqn_norm");
    AdamK k{d->lr, d->beta1, d->beta2, d->adam_eps, d->max_norm, d->target_update_interval};
    hipLaunchKernelGGL(k_drqn_adam, dim3(pm_blocks(PM_RNN_NP, 256)), dim3(256), 0, st, a, k, d->params, d->target,
                       d->adam_m, d->adam_v);
    PM_LAUNCHED("k_drqn_adam");
    return PM_OK;
}

extern "C" int pm_drqn_update(const pm_drqn* d, void* stream) {
    if (int rc = pm_drqn_grads(d, stream)) return rc;
    return pm_drqn_apply(d, stream);
}
