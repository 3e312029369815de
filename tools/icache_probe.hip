// Instruction-fetch probe: one workgroup runs a straight-line block of ~N KB of VALU code twice
// (cold, then warm instruction cache) and stamps s_memrealtime (100 MHz) around each pass. If the
// cold pass is much slower, single-workgroup kernels with large code (k_learn) pay for fetching
// their code every launch.
//   hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o tools/icache_probe && ./tools/icache_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int N>
__device__ __forceinline__ float body(float x, float y) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        x = __builtin_fmaf(x, y, (float)k);
        asm volatile("" : "+v"(x));  // one v_fma per step, nothing folded
    }
    return x;
}

template <int N>
__global__ __launch_bounds__(256) void k_probe(float* out, unsigned long long* ts, int waves) {
    float x = threadIdx.x, y = 0.999f;
    unsigned long long t[5];
    t[0] = __builtin_amdgcn_s_memrealtime();
    for (int pass = 0; pass < 4; ++pass) {
        x = body<N>(x, y);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t[pass + 1] = __builtin_amdgcn_s_memrealtime();
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0)
        for (int k = 0; k < 5; ++k) ts[blockIdx.x * 5 + k] = t[k];
}

template <int N>
void run(float* out, unsigned long long* ts, int threads) {
    unsigned long long h[5];
    double acc[4] = {0, 0, 0, 0};
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_probe<N>, dim3(1), dim3(threads), 0, 0, out, ts, threads / 64);
        hipDeviceSynchronize();
        hipMemcpy(h, ts, sizeof(h), hipMemcpyDeviceToHost);
        for (int k = 0; k < 4; ++k) acc[k] += (h[k + 1] - h[k]) * 10.0;  // ns
    }
    printf("{\"fma_per_pass\": %d, \"code_kb\": %.1f, \"threads\": %d, \"pass_ns\": [%.0f, %.0f, %.0f, %.0f]}\n", N,
           N * 8 / 1024.0, threads, acc[0] / reps, acc[1] / reps, acc[2] / reps, acc[3] / reps);
}

int main() {
    float* out;
    unsigned long long* ts;
    hipMalloc(&out, 4 * 1024);
    hipMalloc(&ts, 8 * 64);
    run<512>(out, ts, 64);
    run<2048>(out, ts, 64);
    run<4096>(out, ts, 64);
    run<4096>(out, ts, 256);
    return 0;
}
