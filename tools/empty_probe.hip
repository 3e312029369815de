// Launch floor probe: an empty 256-block kernel launched back to back, timed (1) by HIP events around
// the whole sequence and (2) from each launch's own dispatch (hipExtLaunchKernel begin/end events, the
// interval rocprofv3's kernel trace reports). Run it bare and under rocprofv3 --kernel-trace to see
// what the profiler adds to a kernel's recorded duration (DESIGN.md, K1 measurement).
//   hipcc --offload-arch=gfx950 -O3 tools/empty_probe.hip -o tools/empty_probe && ./tools/empty_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1023) p[0] = 1;  // never true: keeps the kernel from being elided
}

int main() {
    const int reps = 2000, blocks[2] = {256, 1024};
    for (int bi = 0; bi < 2; ++bi) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int k = 0; k < 200; ++k) hipLaunchKernelGGL(k_empty, dim3(blocks[bi]), dim3(256), 0, 0, nullptr);
        CK(hipEventRecord(a, 0));
        for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(k_empty, dim3(blocks[bi]), dim3(256), 0, 0, nullptr);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        double disp = 0.0;
        const int nd = 200;
        for (int k = 0; k < nd; ++k) {
            hipEvent_t s0, s1;
            CK(hipEventCreate(&s0));
            CK(hipEventCreate(&s1));
            hipExtLaunchKernelGGL(k_empty, dim3(blocks[bi]), dim3(256), 0, 0, s0, s1, 0, (int*)nullptr);
            CK(hipEventSynchronize(s1));
            float d = 0.f;
            CK(hipEventElapsedTime(&d, s0, s1));
            disp += d;
            CK(hipEventDestroy(s0));
            CK(hipEventDestroy(s1));
        }
        printf("{\"blocks\": %d, \"back_to_back_us\": %.3f, \"dispatch_us\": %.3f}\n", blocks[bi], ms * 1e3 / reps,
               disp * 1e3 / nd);
    }
    return 0;
}
