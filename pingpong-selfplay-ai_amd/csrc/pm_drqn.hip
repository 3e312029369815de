// K6 — the DRQN update (train_step_rnn, scripts/train_rnn_iterative.py:400-531) on the device.
//
// One update is a fixed chain of launches on one stream, every GEMM on the exact-f32 MFMA:
//   prep        plain effective heads (modelB train: mu + sigma*eps; targetB eval: mu), the batch
//               gathered feature-major X[7][2*T*B] (column t*B + b; obs then next), last-step a/r/done
//   embed x3    F1 = ReLU(W1 X + b1), F2 = ReLU(W2 F1 + b2), Zx = Wih F2 + bih + bhh — modelB on
//               obs and next, targetB on next (three streams of T*B columns)
//   fwd   xT    one LSTM step for all three streams (gate pre-activations Zx_t + Whh h_{t-1}; the
//               four gates of a 32-unit block land in one workgroup, cell update in its epilogue);
//               the obs stream keeps h, c and the gate activations for BPTT
//   heads x3    S = ReLU(W_S h_T + b_S) (GEMM); Q, double-DQN target, smooth-L1, dQ -> V/A grads,
//               dS (one workgroup); dW_S, db_S, dh_T = W_S^T dS (GEMM)
//   bwd   xT    one BPTT step: dz_t from (dh_t, dc_t, the cached gates) into LDS, dh_{t-1} = Whh^T dz_t
//   wgrad x3    dWih = dZ F2^T, dWhh = dZ H_{t-1}^T, db = rowsum dZ, dF2 = Wih^T dZ (masked by the
//               ReLU) -> dW2, db2, dF1 -> dW1, db1
//   (apply)     NoisyLinear sigma grads = mu grads * epsilon, formed in the norm pass
// then (pm_drqn_apply) the global-norm clip (fp64 partials, fixed order) and torch's Adam.
// Nothing uses atomics: the update is bit-reproducible run to run.
#include "pm_gemm.h"
#include "pm_host.h"
#include "pm_rnn.h"

namespace pm {
namespace {

constexpr int kNormBlocks = 64;
// plain effective head block (floats)
enum : int { E_S = 0, E_SB = 16384, E_V = 16512, E_VB = 16640, E_A = 16644, E_AB = 17028, E_N = 17040 };

struct DrqnArgs {
    int B, T, C0, ldh;  // C0 = T*B columns per stream; ldh = (T+1)*B (h / c histories)
    const float *params, *target;
    float *grad;
    float *X, *F1B, *F1T, *F2B, *F2T, *ZxB, *ZxT;
    float *Hp0, *Hp1, *Hp2, *Cs0, *Cs1, *Cs2;
    float *G0, *S0, *S1, *S2, *dS, *dH0, *dH1, *dC0, *dC1, *dZ, *dP2, *dP1;
    float *effB, *effT;
    int32_t *a_last;
    float *r_last, *d_last, *one;
    double *part;
    int64_t *tstep;
    const float *obs, *next;
    const int32_t *act;
    const float *rew;
    const uint8_t *done;
    pm_drqn_stats *stats;
    const int32_t* enable;
    float gamma;
};

// workspace carve-up (floats unless noted), 64-float aligned pieces
struct DrqnLayout {
    int64_t off[40];
    int n = 0;
    int64_t total = 0;
    int64_t add(int64_t floats) {
        off[n++] = total;
        total += (floats + 63) / 64 * 64;
        return off[n - 1];
    }
};

inline int64_t drqn_layout(int B, int T, DrqnArgs* a, void* work) {
    const int64_t C0 = (int64_t)T * B, ldh = (int64_t)(T + 1) * B;
    DrqnLayout L;
    const int64_t oX = L.add(7 * 2 * C0), oF1B = L.add(64 * 2 * C0), oF1T = L.add(64 * C0), oF2B = L.add(128 * 2 * C0),
                  oF2T = L.add(128 * C0), oZxB = L.add(512 * 2 * C0), oZxT = L.add(512 * C0);
    int64_t oHp[3], oCs[3];
    for (int s = 0; s < 3; ++s) { oHp[s] = L.add(128 * ldh); oCs[s] = L.add(128 * ldh); }
    const int64_t oG0 = L.add(512 * C0), oS0 = L.add(128 * B), oS1 = L.add(128 * B), oS2 = L.add(128 * B),
                  odS = L.add(128 * B), odH0 = L.add(128 * B), odH1 = L.add(128 * B), odC0 = L.add(128 * B),
                  odC1 = L.add(128 * B), odZ = L.add(512 * C0), odP2 = L.add(128 * C0), odP1 = L.add(64 * C0),
                  oEB = L.add(E_N), oET = L.add(E_N), oA = L.add(B), oR = L.add(B), oD = L.add(B), oOne = L.add(4),
                  oPart = L.add(2 * kNormBlocks), oTs = L.add(4);
    const int64_t bytes = L.total * 4;
    if (a && work) {
        float* w = static_cast<float*>(work);
        a->B = B; a->T = T; a->C0 = (int)C0; a->ldh = (int)ldh;
        a->X = w + oX; a->F1B = w + oF1B; a->F1T = w + oF1T; a->F2B = w + oF2B; a->F2T = w + oF2T;
        a->ZxB = w + oZxB; a->ZxT = w + oZxT;
        a->Hp0 = w + oHp[0]; a->Hp1 = w + oHp[1]; a->Hp2 = w + oHp[2];
        a->Cs0 = w + oCs[0]; a->Cs1 = w + oCs[1]; a->Cs2 = w + oCs[2];
        a->G0 = w + oG0; a->S0 = w + oS0; a->S1 = w + oS1; a->S2 = w + oS2; a->dS = w + odS;
        a->dH0 = w + odH0; a->dH1 = w + odH1; a->dC0 = w + odC0; a->dC1 = w + odC1;
        a->dZ = w + odZ; a->dP2 = w + odP2; a->dP1 = w + odP1; a->effB = w + oEB; a->effT = w + oET;
        a->a_last = reinterpret_cast<int32_t*>(w + oA); a->r_last = w + oR; a->d_last = w + oD; a->one = w + oOne;
        a->part = reinterpret_cast<double*>(w + oPart); a->tstep = reinterpret_cast<int64_t*>(w + oTs);
    }
    return bytes;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------- prep
__device__ __forceinline__ bool skipped(const DrqnArgs& a) { return a.enable && *a.enable == 0; }

__global__ __launch_bounds__(256) void k_drqn_prep(DrqnArgs a) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    if (skipped(a)) {  // this replica contributes nothing to the all-reduce
        for (int i = tid; i < PM_RNN_NPARAM + 4; i += nt) a.grad[i] = 0.f;
        return;
    }
    if (tid == 0) a.grad[PM_RNN_NPARAM] = 1.0f;
    // effective heads: modelB train (mu + sigma * eps, NoisyLinear.forward :44-46), targetB eval (mu)
    for (int i = tid; i < 2 * E_N; i += nt) {
        const bool T = i >= E_N;
        const int k = T ? i - E_N : i;
        const float* p = T ? a.target : a.params;
        int mu = -1, sg = 0, ep = 0;
        if (k < E_SB) { mu = R_P_SWMU + k; sg = R_P_SWSG + k; ep = R_P_SWEP + k; }
        else if (k < E_V) { mu = R_P_SBMU + k - E_SB; sg = R_P_SBSG + k - E_SB; ep = R_P_SBEP + k - E_SB; }
        else if (k < E_VB) { mu = R_P_VWMU + k - E_V; sg = R_P_VWSG + k - E_V; ep = R_P_VWEP + k - E_V; }
        else if (k == E_VB) { mu = R_P_VBMU; sg = R_P_VBSG; ep = R_P_VBEP; }
        else if (k >= E_A && k < E_AB) { mu = R_P_AWMU + k - E_A; sg = R_P_AWSG + k - E_A; ep = R_P_AWEP + k - E_A; }
        else if (k >= E_AB && k < E_AB + 3) { mu = R_P_ABMU + k - E_AB; sg = R_P_ABSG + k - E_AB; ep = R_P_ABEP + k - E_AB; }
        float v = 0.f;
        if (mu >= 0) v = T ? p[mu] : p[mu] + p[sg] * p[ep];
        (T ? a.effT : a.effB)[k] = v;
    }
    // the batch, feature-major: X[i][t*B + b] = obs[b][t][i], X[i][C0 + t*B + b] = next[b][t][i]
    const int B = a.B, Tn = a.T, C0 = a.C0;
    for (int e = tid; e < 2 * C0 * 7; e += nt) {
        const int i = e / (2 * C0), col = e % (2 * C0);
        const int nx = col >= C0, cc = col - nx * C0, t = cc / B, b = cc % B;
        a.X[e] = (nx ? a.next : a.obs)[((int64_t)b * Tn + t) * 7 + i];
    }
    for (int b = tid; b < B; b += nt) {
        const int64_t j = (int64_t)b * Tn + Tn - 1;
        a.a_last[b] = a.act[j];
        a.r_last[b] = a.rew[j];
        a.d_last[b] = a.done[j] ? 1.f : 0.f;
    }
    if (tid == 0) a.one[0] = 1.0f;
}

// ---------------------------------------------------------------- forward LSTM step
// grid: 3 streams x (B/32) column tiles x 4 hidden blocks; wave q = gate q (torch order i, f, g, o)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_drqn_fwd(DrqnArgs a, int t) {
    if (skipped(a)) return;
    __shared__ float gate[4][32][33];
    const int B = a.B, C0 = a.C0, ldh = a.ldh, nct = B / 32;
    const int mb = blockIdx.x & 3, ct = (blockIdx.x >> 2) % nct, s = blockIdx.x / (4 * nct);
    const float* P = s == 2 ? a.target : a.params;
    const float* Zx = s == 2 ? a.ZxT : a.ZxB;
    const int64_t ldz = s == 2 ? C0 : 2 * C0;
    const int zc = (s == 1 ? C0 : 0) + t * B + ct * 32;
    float* Hp = s == 0 ? a.Hp0 : (s == 1 ? a.Hp1 : a.Hp2);
    float* Cs = s == 0 ? a.Cs0 : (s == 1 ? a.Cs1 : a.Cs2);
    const int q = threadIdx.x >> 6, lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5;
    const int g0 = q * 128 + 32 * mb;
    gemm_f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = Zx[(int64_t)(g0 + (r & 3) + 8 * (r >> 2) + 4 * h) * ldz + zc + r32];
    if (t > 0) {  // + Whh h_{t-1}: all 16 + 64 operand loads of the wave issued before the 64 MFMAs
        const float* __restrict__ Wr = P + R_P_WHH + (int64_t)(g0 + r32) * 128;
        const float* __restrict__ Hc = Hp + t * B + ct * 32 + r32;
        float4 w4[16];
        float hb[64];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int k0 = 8 * j + 4 * h;
            w4[j] = *reinterpret_cast<const float4*>(Wr + k0);
#pragma unroll
            for (int e = 0; e < 4; ++e) hb[4 * j + e] = Hc[(int64_t)(k0 + e) * ldh];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the MFMA chain
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w4[j].x, hb[4 * j], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w4[j].y, hb[4 * j + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w4[j].z, hb[4 * j + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w4[j].w, hb[4 * j + 3], acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float v = acc[r];
        gate[q][(r & 3) + 8 * (r >> 2) + 4 * h][r32] = q == 2 ? tanhf(v) : sigm(v);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) {
        const int u = e >> 5, c = e & 31, U = 32 * mb + u, col = ct * 32 + c;
        const float gi = gate[0][u][c], gf = gate[1][u][c], gg = gate[2][u][c], go = gate[3][u][c];
        const float cp = t > 0 ? Cs[(int64_t)U * ldh + t * B + col] : 0.f;
        const float c2 = gf * cp + gi * gg;  // cy = forgetgate * cx + ingate * cellgate
        const float h2 = go * tanhf(c2);
        Cs[(int64_t)U * ldh + (t + 1) * B + col] = c2;
        Hp[(int64_t)U * ldh + (t + 1) * B + col] = h2;
        if (t == 0) { Cs[(int64_t)U * ldh + col] = 0.f; Hp[(int64_t)U * ldh + col] = 0.f; }
        if (s == 0) {
            const int64_t gc = (int64_t)t * B + col;
            a.G0[(int64_t)U * C0 + gc] = gi;
            a.G0[(int64_t)(128 + U) * C0 + gc] = gf;
            a.G0[(int64_t)(256 + U) * C0 + gc] = gg;
            a.G0[(int64_t)(384 + U) * C0 + gc] = go;
        }
    }
}

// ---------------------------------------------------------------- heads: Q, TD target, loss, dQ
__global__ __launch_bounds__(256) void k_drqn_q(DrqnArgs a) {
    if (skipped(a)) return;
    __shared__ float Q[3][256][3];
    __shared__ float dV[256], dA[256][3], lv[256], qv[256];
    const int B = a.B, tid = threadIdx.x;
    for (int e = tid; e < 3 * B; e += 256) {
        const int s = e / B, b = e % B;
        const float* eff = s == 2 ? a.effT : a.effB;
        const float* S = s == 0 ? a.S0 : (s == 1 ? a.S1 : a.S2);
        float v = 0.f, x0 = 0.f, x1 = 0.f, x2 = 0.f;
#pragma unroll 16
        for (int u = 0; u < 128; ++u) {
            const float su = S[u * B + b];
            v += eff[E_V + u] * su;
            x0 += eff[E_A + u] * su;
            x1 += eff[E_A + 128 + u] * su;
            x2 += eff[E_A + 256 + u] * su;
        }
        v += eff[E_VB];
        x0 += eff[E_AB]; x1 += eff[E_AB + 1]; x2 += eff[E_AB + 2];
        const float mean = ((x0 + x1) + x2) / 3.0f;  // A.mean(dim=1)
        Q[s][b][0] = v + (x0 - mean);
        Q[s][b][1] = v + (x1 - mean);
        Q[s][b][2] = v + (x2 - mean);
    }
    __syncthreads();
    if (tid < B) {
        const int b = tid, ac = a.a_last[b];
        const float q = Q[0][b][ac];
        const int as = argmax3(Q[1][b]);  // argmax Q_B(next) (first max)
        const float y = a.r_last[b] + a.gamma * Q[2][b][as] * (1.0f - a.d_last[b]);
        const float d = q - y, ad = fabsf(d);
        lv[b] = ad < 1.0f ? 0.5f * d * d : ad - 0.5f;  // smooth_l1, beta 1
        qv[b] = q;
        const float gq = fminf(fmaxf(d, -1.0f), 1.0f) / (float)B;
        dV[b] = gq;
#pragma unroll
        for (int k = 0; k < 3; ++k) dA[b][k] = (k == ac ? gq : 0.f) - gq / 3.0f;
    }
    __syncthreads();
    float* g = a.grad;
    if (tid == 0) {
        float ls = 0.f, qs = 0.f;
        for (int b = 0; b < B; ++b) { ls += lv[b]; qs += qv[b]; }
        a.stats->loss = ls / (float)B;
        a.stats->q_mean = qs / (float)B;
    }
    if (tid < 128) {
        const int u = tid;
        float gv = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll 16
        for (int b = 0; b < B; ++b) {
            const float su = a.S0[u * B + b];
            gv += dV[b] * su; g0 += dA[b][0] * su; g1 += dA[b][1] * su; g2 += dA[b][2] * su;
        }
        g[R_P_VWMU + u] = gv;
        g[R_P_AWMU + u] = g0; g[R_P_AWMU + 128 + u] = g1; g[R_P_AWMU + 256 + u] = g2;
    } else if (tid < 132) {
        const int k = tid - 128;
        float sacc = 0.f;
        for (int b = 0; b < B; ++b) sacc += k == 0 ? dV[b] : dA[b][k - 1];
        g[k == 0 ? R_P_VBMU : R_P_ABMU + k - 1] = sacc;
    }
    const float* eff = a.effB;
    for (int e = tid; e < 128 * B; e += 256) {
        const int u = e / B, b = e % B;
        const float ds = eff[E_V + u] * dV[b] + eff[E_A + u] * dA[b][0] + eff[E_A + 128 + u] * dA[b][1] +
                         eff[E_A + 256 + u] * dA[b][2];
        a.dS[e] = a.S0[e] > 0.f ? ds : 0.f;
    }
}

// ---------------------------------------------------------------- one BPTT step
// grid: 4 unit tiles x (B/32) column tiles. dz_t for all 512 gate rows of the block's columns in
// LDS; the block writes dz_t / dc_{t-1} for its own 32 units and dh_{t-1} = Whh^T dz_t for them.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_drqn_bwd(DrqnArgs a, int t) {
    if (skipped(a)) return;
    __shared__ float dz[512][33];
    __shared__ float red[4][16][64];
    const int B = a.B, C0 = a.C0, ldh = a.ldh, Tn = a.T;
    const int mu = blockIdx.x & 3, ct = blockIdx.x >> 2;
    const float* dHin = ((Tn - 1 - t) & 1) ? a.dH1 : a.dH0;
    float* dHout = ((Tn - t) & 1) ? a.dH1 : a.dH0;
    const float* dCin = ((Tn - 1 - t) & 1) ? a.dC1 : a.dC0;
    float* dCout = ((Tn - t) & 1) ? a.dC1 : a.dC0;
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const float* __restrict__ Wc = a.params + R_P_WHH + 32 * mu + (ln & 31);  // A(m = u_out, k = g) = Whh[g][u_out]
    float wa[64];  // this wave's K quarter of the Whh column, loaded before the elementwise pass
    if (t > 0) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) wa[4 * j + e] = Wc[(int64_t)(128 * wv + 8 * j + 4 * (ln >> 5) + e) * 128];
    }
    __builtin_amdgcn_sched_barrier(0);
    // 16 (unit, column) pairs per thread in two halves: the 8 operand loads of 8 pairs are issued
    // before any of their stores (the workspace pointers may alias, so the compiler would not)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        float v[8][8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * (8 * half + q);
            const int u = e >> 5, col = ct * 32 + (e & 31);
            const int64_t gc = (int64_t)t * B + col;
            v[q][0] = dHin[u * B + col];
            v[q][1] = t == Tn - 1 ? 0.f : dCin[u * B + col];
            v[q][2] = a.G0[(int64_t)u * C0 + gc];
            v[q][3] = a.G0[(int64_t)(128 + u) * C0 + gc];
            v[q][4] = a.G0[(int64_t)(256 + u) * C0 + gc];
            v[q][5] = a.G0[(int64_t)(384 + u) * C0 + gc];
            v[q][6] = a.Cs0[(int64_t)u * ldh + (t + 1) * B + col];
            v[q][7] = a.Cs0[(int64_t)u * ldh + t * B + col];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = threadIdx.x + 256 * (8 * half + q);
            const int u = e >> 5, c = e & 31, col = ct * 32 + c;
            const int64_t gc = (int64_t)t * B + col;
            const float dh = v[q][0], dcc = v[q][1], gi = v[q][2], gf = v[q][3], gg = v[q][4], go = v[q][5];
            const float cT = v[q][6], cp = v[q][7];
            const float tc = tanhf(cT);
            const float dc = dcc + dh * go * (1.0f - tc * tc);
            const float dzi = dc * gg * (gi * (1.0f - gi));
            const float dzf = dc * cp * (gf * (1.0f - gf));
            const float dzg = dc * gi * (1.0f - gg * gg);
            const float dzo = dh * tc * (go * (1.0f - go));
            dz[u][c] = dzi; dz[128 + u][c] = dzf; dz[256 + u][c] = dzg; dz[384 + u][c] = dzo;
            if ((u >> 5) == mu) {
                a.dZ[(int64_t)u * C0 + gc] = dzi;
                a.dZ[(int64_t)(128 + u) * C0 + gc] = dzf;
                a.dZ[(int64_t)(256 + u) * C0 + gc] = dzg;
                a.dZ[(int64_t)(384 + u) * C0 + gc] = dzo;
                dCout[u * B + col] = dc * gf;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (t == 0) return;  // dh_{-1} is not needed
    const int w = wv, lane = ln, r32 = lane & 31, h = lane >> 5;
    gemm_f32x16 acc = {};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int k0 = 128 * w + 8 * j + 4 * h;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[4 * j + e], dz[k0 + e][r32], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][r][lane] = acc[r];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256) {
        const int r = e >> 6, ln = e & 63;
        const int m = (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5), n = ln & 31;
        dHout[(32 * mu + m) * B + ct * 32 + n] = ((red[0][r][ln] + red[1][r][ln]) + red[2][r][ln]) + red[3][r][ln];
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
__global__ __launch_bounds__(256) void k_drqn_norm(DrqnArgs a) {
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

__global__ __launch_bounds__(256) void k_drqn_adam(DrqnArgs a, AdamK k, float* params, float* target, float* m_,
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
    if (batch < 1 || T < 1) return -1;
    return drqn_layout(batch, T, nullptr, nullptr);
}

extern "C" int pm_drqn_grads(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    PM_REQUIRE(d->obs && d->next && d->act && d->rew && d->done, PM_E_ARG, "pm_drqn_grads: null batch");
    hipStream_t st = pm_stream(stream);
    DrqnArgs a{};
    drqn_layout(d->batch, d->T, &a, d->work);
    a.params = d->params; a.target = d->target; a.grad = d->grad; a.stats = d->stats; a.enable = d->enable;
    a.obs = d->obs; a.next = d->next; a.act = d->act; a.rew = d->rew; a.done = d->done;
    a.gamma = (float)d->gamma;
    const int B = a.B, C0 = a.C0, ldh = a.ldh, T = a.T, nct = B / 32;
    const float *PB = d->params, *PT = d->target;
    float* g = d->grad;
    hipLaunchKernelGGL(k_drqn_prep, dim3(64), dim3(256), 0, st, a);
    PM_LAUNCHED("k_drqn_prep");
    // embedding: modelB on [obs | next] (2*C0 columns), targetB on next (C0 columns)
    GemmProb p[kGemmMax];
    p[0] = gemm_prob(PB + R_P_F1W, 7, 1, a.X, 2 * C0, 1, a.F1B, 2 * C0, 1, 64, 2 * C0, 7, GF_RELU, PB + R_P_F1B);
    p[1] = gemm_prob(PT + R_P_F1W, 7, 1, a.X + C0, 2 * C0, 1, a.F1T, C0, 1, 64, C0, 7, GF_RELU, PT + R_P_F1B);
    PM_REQUIRE(gemm_launch(p, 2, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (F1)");
    p[0] = gemm_prob(PB + R_P_F2W, 64, 1, a.F1B, 2 * C0, 1, a.F2B, 2 * C0, 1, 128, 2 * C0, 64, GF_RELU, PB + R_P_F2B);
    p[1] = gemm_prob(PT + R_P_F2W, 64, 1, a.F1T, C0, 1, a.F2T, C0, 1, 128, C0, 64, GF_RELU, PT + R_P_F2B);
    PM_REQUIRE(gemm_launch(p, 2, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (F2)");
    p[0] = gemm_prob(PB + R_P_WIH, 128, 1, a.F2B, 2 * C0, 1, a.ZxB, 2 * C0, 1, 512, 2 * C0, 128, 0, PB + R_P_BIH,
                     PB + R_P_BHH);
    p[1] = gemm_prob(PT + R_P_WIH, 128, 1, a.F2T, C0, 1, a.ZxT, C0, 1, 512, C0, 128, 0, PT + R_P_BIH, PT + R_P_BHH);
    PM_REQUIRE(gemm_launch(p, 2, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (Zx)");
    for (int t = 0; t < T; ++t) {
        hipLaunchKernelGGL(k_drqn_fwd, dim3(3 * nct * 4), dim3(256), 0, st, a, t);
        PM_LAUNCHED("k_drqn_fwd");
    }
    // shared head on h_T (column T*B of the histories)
    const int64_t hT = (int64_t)T * B;
    p[0] = gemm_prob(a.effB + E_S, 128, 1, a.Hp0 + hT, ldh, 1, a.S0, B, 1, 128, B, 128, GF_RELU, a.effB + E_SB);
    p[1] = gemm_prob(a.effB + E_S, 128, 1, a.Hp1 + hT, ldh, 1, a.S1, B, 1, 128, B, 128, GF_RELU, a.effB + E_SB);
    p[2] = gemm_prob(a.effT + E_S, 128, 1, a.Hp2 + hT, ldh, 1, a.S2, B, 1, 128, B, 128, GF_RELU, a.effT + E_SB);
    PM_REQUIRE(gemm_launch(p, 3, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (S)");
    hipLaunchKernelGGL(k_drqn_q, dim3(1), dim3(256), 0, st, a);
    PM_LAUNCHED("k_drqn_q");
    p[0] = gemm_prob(a.dS, B, 1, a.Hp0 + hT, 1, ldh, g + R_P_SWMU, 128, 1, 128, 128, B);  // dW_S = dS h_T^T
    p[1] = gemm_prob(a.dS, B, 1, a.one, 0, 0, g + R_P_SBMU, 1, 0, 128, 1, B);             // db_S
    p[2] = gemm_prob(a.effB + E_S, 1, 128, a.dS, B, 1, a.dH0, B, 1, 128, B, 128);          // dh_T = W_S^T dS
    PM_REQUIRE(gemm_launch(p, 3, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (dS)");
    for (int t = T - 1; t >= 0; --t) {
        hipLaunchKernelGGL(k_drqn_bwd, dim3(4 * nct), dim3(256), 0, st, a, t);
        PM_LAUNCHED("k_drqn_bwd");
    }
    // weight gradients over all T*B columns of the obs stream
    p[0] = gemm_prob(a.dZ, C0, 1, a.F2B, 1, 2 * C0, g + R_P_WIH, 128, 1, 512, 128, C0);  // dWih = dZ F2^T
    p[1] = gemm_prob(a.dZ, C0, 1, a.Hp0, 1, ldh, g + R_P_WHH, 128, 1, 512, 128, C0);     // dWhh = dZ H_{t-1}^T
    p[2] = gemm_prob(a.dZ, C0, 1, a.one, 0, 0, g + R_P_BIH, 1, 0, 512, 1, C0);           // db_ih
    p[3] = gemm_prob(a.dZ, C0, 1, a.one, 0, 0, g + R_P_BHH, 1, 0, 512, 1, C0);           // db_hh
    p[4] = gemm_prob(PB + R_P_WIH, 1, 128, a.dZ, C0, 1, a.dP2, C0, 1, 128, C0, 512, 0, nullptr, nullptr, a.F2B,
                     2 * C0, 1);  // dF2 = Wih^T dZ, through the ReLU
    PM_REQUIRE(gemm_launch(p, 5, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (dZ)");
    p[0] = gemm_prob(a.dP2, C0, 1, a.F1B, 1, 2 * C0, g + R_P_F2W, 64, 1, 128, 64, C0);  // dW2
    p[1] = gemm_prob(a.dP2, C0, 1, a.one, 0, 0, g + R_P_F2B, 1, 0, 128, 1, C0);         // db2
    p[2] = gemm_prob(PB + R_P_F2W, 1, 64, a.dP2, C0, 1, a.dP1, C0, 1, 64, C0, 128, 0, nullptr, nullptr, a.F1B, 2 * C0,
                     1);  // dF1 = W2^T dF2, through the ReLU
    PM_REQUIRE(gemm_launch(p, 3, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (dP2)");
    p[0] = gemm_prob(a.dP1, C0, 1, a.X, 1, 2 * C0, g + R_P_F1W, 7, 1, 64, 7, C0);  // dW1
    p[1] = gemm_prob(a.dP1, C0, 1, a.one, 0, 0, g + R_P_F1B, 1, 0, 64, 1, C0);     // db1
    PM_REQUIRE(gemm_launch(p, 2, st, d->enable) == hipSuccess, PM_E_LAUNCH, "k_gemm (dP1)");
    return PM_OK;
}

extern "C" int pm_drqn_apply(const pm_drqn* d, void* stream) {
    if (int rc = check(d)) return rc;
    hipStream_t st = pm_stream(stream);
    DrqnArgs a{};
    drqn_layout(d->batch, d->T, &a, d->work);
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
