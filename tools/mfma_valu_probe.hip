// Probe: how much VALU issue does a wave get on a SIMD whose partner wave streams
// v_mfma_f32_32x32x2_f32 back to back? One workgroup of 512 threads (8 waves): waves w and w + 4
// share SIMD w % 4. Waves 0-3 run an MFMA chain (or idle), waves 4-7 run a dependent-free VALU
// loop (or idle); each wave records its s_memtime span. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512) void probe(int mode, int n_mfma, int n_valu, unsigned long long* span, float* sink) {
    const int wave = threadIdx.x >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < 4) {
        if (mode == 4) {  // one wave: MFMA chain with 8 own VALU fmas between consecutive MFMAs
            f32x16 c = {};
            float a = threadIdx.x * 1e-3f, b = 1.0f;
            float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
            for (int i = 0; i < n_mfma; ++i) {
                c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
                x0 = fmaf(x0, 0.999f, 0.5f); x1 = fmaf(x1, 0.999f, 0.5f); x2 = fmaf(x2, 0.999f, 0.5f); x3 = fmaf(x3, 0.999f, 0.5f);
                x4 = fmaf(x4, 0.999f, 0.5f); x5 = fmaf(x5, 0.999f, 0.5f); x6 = fmaf(x6, 0.999f, 0.5f); x7 = fmaf(x7, 0.999f, 0.5f);
            }
            float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
            for (int r = 0; r < 16; ++r) s += c[r];
            sink[threadIdx.x] = s;
        } else if (mode & 1) {
            f32x16 c = {};
            float a = threadIdx.x * 1e-3f, b = 1.0f;
            for (int i = 0; i < n_mfma; ++i) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
            float s = 0.f;
            for (int r = 0; r < 16; ++r) s += c[r];
            sink[threadIdx.x] = s;
        }
    } else if (mode & 2) {
        if (mode & 8) __builtin_amdgcn_s_setprio(3);
        float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
        for (int i = 0; i < n_valu; ++i) {  // 8 independent fma chains
            x0 = fmaf(x0, 0.999f, 0.5f); x1 = fmaf(x1, 0.999f, 0.5f); x2 = fmaf(x2, 0.999f, 0.5f); x3 = fmaf(x3, 0.999f, 0.5f);
            x4 = fmaf(x4, 0.999f, 0.5f); x5 = fmaf(x5, 0.999f, 0.5f); x6 = fmaf(x6, 0.999f, 0.5f); x7 = fmaf(x7, 0.999f, 0.5f);
        }
        sink[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) span[wave] = t1 - t0;
}

int main() {
    unsigned long long* d_span;
    float* d_sink;
    hipMalloc(&d_span, 8 * sizeof(unsigned long long));
    hipMalloc(&d_sink, 512 * sizeof(float));
    const int n_mfma = 2000, n_valu = 2000;  // 2000 MFMA x 64 cyc = 128k cyc; 16000 VALU x 4 cyc = 64k cyc
    const char* names[12] = {"idle", "mfma only", "valu only", "mfma + valu", "interleaved", "", "", "", "",
                             "", "", "mfma + valu prio"};
    const int modes[5] = {1, 2, 3, 11, 4};
    for (int mi = 0; mi < 5; ++mi) {
        const int mode = modes[mi];
        for (int rep = 0; rep < 3; ++rep) probe<<<1, 512>>>(mode, n_mfma, n_valu, d_span, d_sink);
        hipDeviceSynchronize();
        unsigned long long span[8];
        hipMemcpy(span, d_span, sizeof(span), hipMemcpyDeviceToHost);
        printf("%-12s mfma waves %8llu cyc (%5.1f cyc/mfma) | valu waves %8llu cyc (%5.2f cyc/valu op)\n", names[mode],
               span[0], (mode & 1) ? (double)span[0] / n_mfma : 0.0, span[4],
               (mode & 2) ? (double)span[4] / (8.0 * n_valu) : 0.0);
        if (mode == 4) printf("             (interleaved: 8 fma per mfma inside wave 0; valu-only time for 16000 fma = 105k cyc)\n");
    }
    return 0;
}
