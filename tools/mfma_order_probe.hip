// Accumulation-order probe for the exact-f32 matrix instructions on gfx950: does
// v_mfma_f32_16x16x4_f32 (and 32x32x2) equal k-ordered fmaf chains bit for bit? Random operands with
// wide exponent spread (so orders differ visibly); every output compared against several host orders.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mfma_order_probe.hip -o tools/mfma_order_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// one wave: K-step chain of `steps` 16x16x4 MFMAs; A [16][4*steps], B [4*steps][16], C [16][16]
__global__ void k16(const float* A, const float* B, const float* C, float* D, int steps) {
    const int l = threadIdx.x;  // 64 lanes
    f32x4 acc;
    // accumulator layout (16x16, 4 regs): lane l holds D[4*(l>>4) + r][l & 15], r = 0..3
    for (int r = 0; r < 4; ++r) acc[r] = C[(4 * (l >> 4) + r) * 16 + (l & 15)];
    for (int s = 0; s < steps; ++s) {
        const float a = A[(l & 15) * (4 * steps) + 4 * s + (l >> 4)];  // A[m = l & 15][k = l >> 4]
        const float b = B[(4 * s + (l >> 4)) * 16 + (l & 15)];          // B[k = l >> 4][n = l & 15]
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

__global__ void k32(const float* A, const float* B, const float* C, float* D, int steps) {
    const int l = threadIdx.x;
    f32x16 acc;
    // 32x32 accumulator: lane l, reg r -> row 8*(r>>2) + 4*(l>>5) + (r&3), column l & 31
    for (int r = 0; r < 16; ++r) acc[r] = C[(8 * (r >> 2) + 4 * (l >> 5) + (r & 3)) * 32 + (l & 31)];
    for (int s = 0; s < steps; ++s) {
        const float a = A[(l & 31) * (2 * steps) + 2 * s + (l >> 5)];  // A[m][k = l >> 5]
        const float b = B[(2 * s + (l >> 5)) * 32 + (l & 31)];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) D[(8 * (r >> 2) + 4 * (l >> 5) + (r & 3)) * 32 + (l & 31)] = acc[r];
}

static float rnd() {
    const float m = (float)rand() / RAND_MAX - 0.5f;
    return ldexpf(m, rand() % 24 - 12);
}

static int run(int N, int kper, int steps) {
    const int K = kper * steps;
    float *A, *B, *C, *D;
    hipMallocManaged(&A, N * K * 4); hipMallocManaged(&B, K * N * 4);
    hipMallocManaged(&C, N * N * 4); hipMallocManaged(&D, N * N * 4);
    int bad_seq = 0, bad_pair = 0, bad_exact = 0, total = 0;
    for (int trial = 0; trial < 200; ++trial) {
        for (int i = 0; i < N * K; ++i) { A[i] = rnd(); B[i] = rnd(); }
        for (int i = 0; i < N * N; ++i) C[i] = rnd();
        if (N == 16) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, C, D, steps);
        else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, C, D, steps);
        hipDeviceSynchronize();
        for (int m = 0; m < N; ++m)
            for (int n = 0; n < N; ++n) {
                float seq = C[m * N + n], pair = C[m * N + n];
                double ex = C[m * N + n];
                for (int s = 0; s < steps; ++s) {
                    double blk = 0.0;
                    for (int k = 0; k < kper; ++k) {
                        const int kk = kper * s + k;
                        seq = fmaf(A[m * K + kk], B[kk * N + n], seq);
                        blk += (double)A[m * K + kk] * (double)B[kk * N + n];
                    }
                    // one rounding per instruction: C + exact block sum (double is exact enough here)
                    pair = (float)((double)pair + blk);
                    ex += blk;
                }
                const float d = D[m * N + n];
                bad_seq += d != seq; bad_pair += d != pair; bad_exact += d != (float)ex; ++total;
            }
    }
    printf("{\"mfma\": \"%dx%dx%d\", \"steps\": %d, \"outputs\": %d, \"differ_from_sequential_fmaf\": %d, "
           "\"differ_from_round_per_instruction\": %d, \"differ_from_exact_sum\": %d}\n",
           N, N, kper, steps, total, bad_seq, bad_pair, bad_exact);
    return 0;
}

int main() {
    srand(7);
    run(32, 2, 16);
    run(16, 4, 16);
    run(16, 4, 1);
    return 0;
}
