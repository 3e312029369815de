// v_mfma_f32_4x4x1_16b_f32 on gfx950: operand / accumulator lane layout, whether a chain of them is a
// k-ordered fmaf chain bit for bit (as the 16x16x4 / 32x32x2 forms are: tools/mfma_order_probe.hip),
// and its issue cost beside the 16x16x4 form (s_memtime around chains of 4 interleaved accumulators).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mfma4_probe.hip -o tools/mfma4_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// layout: one MFMA with lane-coded operands; D[l][r] for the 4 accumulator registers
__global__ void k_layout(const float* a, const float* b, float* d) {
    const int l = threadIdx.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

// chain: `steps` MFMAs, step s uses a[s][l], b[s][l]; starts from c[l][r]
__global__ void k_chain(const float* a, const float* b, const float* c, float* d, int steps) {
    const int l = threadIdx.x;
    f32x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[l * 4 + r];
    for (int s = 0; s < steps; ++s) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[s * 64 + l], b[s * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

// cost: 4 interleaved accumulator chains of 8 (16x16x4) or 32 (4x4x1) steps, cycles by s_memtime
template <int KIND>
__global__ void k_cost(const float* a, float* d, unsigned long long* cyc) {
    const int l = threadIdx.x;
    f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    float x[32];
    for (int s = 0; s < 32; ++s) x[s] = a[s * 64 + l];
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (KIND == 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[4 * s + c], x[s], acc[c], 0, 0, 0);
    } else {
#pragma unroll
        for (int s = 0; s < 32; ++s)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c == 0) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(x[s], x[(s + 1) & 31], acc[c], 0, 0, 0);
        // (one chain of 32: the heads' per-player work is one 4x4x1 chain covering all 16 blocks)
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) d[(c * 64 + l) * 4 + r] = acc[c][r];
    if (l == 0) cyc[KIND] = t1 - t0;
}

static float rnd() {
    const float m = (float)rand() / RAND_MAX - 0.5f;
    return ldexpf(m, rand() % 24 - 12);
}

int main() {
    srand(11);
    float *a, *b, *c, *d;
    unsigned long long* cyc;
    const int S = 32;
    hipMallocManaged(&a, S * 64 * 4); hipMallocManaged(&b, S * 64 * 4);
    hipMallocManaged(&c, 64 * 4 * 4); hipMallocManaged(&d, 4 * 64 * 4 * 4);
    hipMallocManaged(&cyc, 2 * 8);
    // layout: A = lane + 1, B = 1 -> which A lane feeds D[l][r]; then A = 1, B = lane + 1
    int srcA[64][4], srcB[64][4];
    for (int l = 0; l < 64; ++l) { a[l] = (float)(l + 1); b[l] = 1.f; }
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, a, b, d);
    hipDeviceSynchronize();
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) srcA[l][r] = (int)d[l * 4 + r] - 1;
    for (int l = 0; l < 64; ++l) { a[l] = 1.f; b[l] = (float)(l + 1); }
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, a, b, d);
    hipDeviceSynchronize();
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) srcB[l][r] = (int)d[l * 4 + r] - 1;
    printf("{\"layout\": [");
    for (int l = 0; l < 64; ++l)
        printf("%s[%d,%d,%d,%d,%d,%d,%d,%d]", l ? "," : "", srcA[l][0], srcB[l][0], srcA[l][1], srcB[l][1], srcA[l][2],
               srcB[l][2], srcA[l][3], srcB[l][3]);
    printf("]}\n");
    // exactness: D[l][r] = fmaf chain over s of a[s][srcA] * b[s][srcB] from c[l][r]
    int bad_seq = 0, bad_pair = 0, total = 0;
    for (int trial = 0; trial < 200; ++trial) {
        for (int i = 0; i < S * 64; ++i) { a[i] = rnd(); b[i] = rnd(); }
        for (int i = 0; i < 256; ++i) c[i] = trial & 1 ? 0.f : rnd();
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, a, b, c, d, S);
        hipDeviceSynchronize();
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
                float seq = c[l * 4 + r], pair = c[l * 4 + r];
                for (int s = 0; s < S; ++s) {
                    const float x = a[s * 64 + srcA[l][r]], y = b[s * 64 + srcB[l][r]];
                    seq = fmaf(x, y, seq);
                    pair = pair + x * y;  // (-ffp-contract=off: product rounded, then the add)
                }
                bad_seq += d[l * 4 + r] != seq;
                bad_pair += d[l * 4 + r] != pair;
                ++total;
            }
    }
    printf("{\"mfma\": \"4x4x1_16b\", \"steps\": %d, \"outputs\": %d, \"differ_from_sequential_fmaf\": %d, "
           "\"differ_from_mul_then_add\": %d}\n", S, total, bad_seq, bad_pair);
    for (int i = 0; i < S * 64; ++i) a[i] = rnd();
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_cost<0>, dim3(1), dim3(64), 0, 0, a, d, cyc);
        hipLaunchKernelGGL(k_cost<1>, dim3(1), dim3(64), 0, 0, a, d, cyc);
        hipDeviceSynchronize();
        printf("{\"cycles_4_chains_x8_16x16x4\": %llu, \"cycles_1_chain_x32_4x4x1\": %llu}\n", cyc[0], cyc[1]);
    }
    return 0;
}
