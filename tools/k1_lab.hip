// K1 lab: variants of the batched PongEnv2P step (k_env_step) timed side by side on one device.
// Not the product: used to choose the product kernel's structure. Every variant is
// checked bit-for-bit against the base variant after K steps from the same state and actions.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//         -Iinclude -Ipingpong-selfplay-ai_amd/csrc tools/k1_lab.hip -o tools/k1_lab && ./tools/k1_lab [n...]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "pm_dev.h"

using namespace pm;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));

struct Out {
    float *obsA, *obsB, *rA, *rB, *tA, *tB;
    uint8_t* done;
};

__device__ __forceinline__ void serve_sincos(const pm_env_params& p, uint32_t i, uint32_t nserve, uint64_t seed,
                                             double& vx, double& vy, double& spin) {
    const U4 r0 = philox(i, TAG_SERVE, nserve, 0u, seed);
    const U4 r1 = philox(i, TAG_SERVE | 0x100u, nserve, 0u, seed);
    const double speed = p.speed_lo + (p.speed_hi - p.speed_lo) * u53(r0.x, r0.y);
    double ang;
    if (u53(r0.z, r0.w) < 0.5) ang = p.ang0_lo + (p.ang0_hi - p.ang0_lo) * u53(r1.x, r1.y);
    else ang = p.ang1_lo + (p.ang1_hi - p.ang1_lo) * u53(r1.x, r1.y);
    const double rad = ang * (3.141592653589793 / 180.0);
    double s, c;
    sincos(rad, &s, &c);
    vx = speed * c;
    vy = speed * s;
    spin = p.spin_lo + (p.spin_hi - p.spin_lo) * u53(r1.z, r1.w);
}

// STORE: 0 = store_rows7 per output (two barriers each), 1 = all rows staged, one barrier,
//        2 = direct per-lane 28-B rows (dwordx4 + dwordx3)
// SPEC:  serves loaded first and the next serve drawn for every lane while the state loads land
// TRIG:  0 = cos + sin, 1 = sincos
template <int BLOCK, int STORE, bool SPEC, int TRIG, int TERM = 0, int SKEL = 0>
__global__ __launch_bounds__(BLOCK) void k_var(pm_env_params p, pm_env_state s, const int8_t* __restrict__ aA,
                                               const int8_t* __restrict__ aB, Out o, uint64_t seed, int n) {
    __shared__ __attribute__((aligned(16))) float lds[STORE == 1 || STORE == 3 ? 4 : 1][BLOCK][7];
    const int i0 = blockIdx.x * BLOCK;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0}, tA[7] = {0}, tB[7] = {0};
    if (i < n) {
        int32_t ns = 0;
        double svx = 0, svy = 0, ssp = 0;
        if (SPEC) {
            ns = __builtin_nontemporal_load(&s.serves[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
        Arena a = load_arena(s, i);
        const int xa = aA[i], xb = aB[i];
        if (SPEC) {
            if (TRIG) serve_sincos(p, (uint32_t)i, (uint32_t)ns, seed, svx, svy, ssp);
            else philox_serve(p, (uint32_t)i, (uint32_t)ns, seed, svx, svy, ssp);
        }
        float ra = 0.f, rb = 0.f;
        int d = 0;
        if (SKEL) { ra = (float)xa; rb = (float)xb; } else d = tick(p, a, xa, xb, ra, rb);
        observe(a, oA, oB);
#pragma unroll
        for (int k = 0; k < 7; ++k) { tA[k] = oA[k]; tB[k] = oB[k]; }
        if (d) {
            if (!SPEC) {
                ns = s.serves[i];
                if (TRIG) serve_sincos(p, (uint32_t)i, (uint32_t)ns, seed, svx, svy, ssp);
                else philox_serve(p, (uint32_t)i, (uint32_t)ns, seed, svx, svy, ssp);
            }
            serve(a, svx, svy, ssp);
            s.serves[i] = ns + 1;
            observe(a, oA, oB);
            if (TERM) {
                float* r = o.tA + (size_t)i * 7;
                float* q = o.tB + (size_t)i * 7;
#pragma unroll
                for (int k = 0; k < 7; ++k) { r[k] = tA[k]; q[k] = tB[k]; }
            }
        }
        store_arena(s, i, a);
        o.rA[i] = ra;
        o.rB[i] = rb;
        o.done[i] = (uint8_t)d;
    }
    if (STORE == 0) {
        store_rows7(o.obsA, lds[0], oA, i0, n);
        store_rows7(o.obsB, lds[0], oB, i0, n);
        if (!TERM) {
            store_rows7(o.tA, lds[0], tA, i0, n);
            store_rows7(o.tB, lds[0], tB, i0, n);
        }
    } else if (STORE == 1) {
        const int t = threadIdx.x;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            lds[0][t][k] = oA[k]; lds[1][t][k] = oB[k];
            if (!TERM) { lds[2][t][k] = tA[k]; lds[3][t][k] = tB[k]; }
        }
        __syncthreads();
        const int rows = min(BLOCK, n - i0);
        float* dsts[4] = {o.obsA, o.obsB, o.tA, o.tB};
        if (rows == BLOCK) {
#pragma unroll
            for (int q = 0; q < (TERM ? 2 : 4); ++q) {
                float4* d4 = reinterpret_cast<float4*>(dsts[q] + (size_t)i0 * 7);
                const float4* s4 = reinterpret_cast<const float4*>(&lds[q][0][0]);
                for (int f = t; f < BLOCK * 7 / 4; f += BLOCK) d4[f] = s4[f];
            }
        } else {
            for (int q = 0; q < (TERM ? 2 : 4); ++q)
                for (int f = t; f < rows * 7; f += BLOCK) dsts[q][(size_t)i0 * 7 + f] = (&lds[q][0][0])[f];
        }
    } else if (STORE == 3) {
        // per-wave staging: each wave writes its own 64 rows and reads them back (LDS ops of one wave
        // complete in order), so no block barrier
        const int t = threadIdx.x, lane = t & 63, w0 = t & ~63;
        const int nq = TERM ? 2 : 4;
        float* dsts[4] = {o.obsA, o.obsB, o.tA, o.tB};
        const float* v[4] = {oA, oB, tA, tB};
        const int wrows = min(64, n - (i0 + w0));
        for (int q = 0; q < nq; ++q) {
#pragma unroll
            for (int k = 0; k < 7; ++k) lds[q][t][k] = v[q][k];
        }
        __builtin_amdgcn_wave_barrier();
        if (wrows == 64) {
            for (int q = 0; q < nq; ++q) {
                float4* d4 = reinterpret_cast<float4*>(dsts[q] + (size_t)(i0 + w0) * 7);
                const float4* s4 = reinterpret_cast<const float4*>(&lds[q][w0][0]);
                d4[lane] = s4[lane];
                if (lane < 48) d4[64 + lane] = s4[64 + lane];
            }
        } else if (wrows > 0) {
            for (int q = 0; q < nq; ++q)
                for (int f = lane; f < wrows * 7; f += 64) dsts[q][(size_t)(i0 + w0) * 7 + f] = (&lds[q][w0][0])[f];
        }
    } else {
        if (i < n) {
            float* rows[4] = {o.obsA, o.obsB, o.tA, o.tB};
            const float* v[4] = {oA, oB, tA, tB};
#pragma unroll
            for (int q = 0; q < (TERM ? 2 : 4); ++q) {
                float* r = rows[q] + (size_t)i * 7;
                *reinterpret_cast<f4u*>(r) = f4u{v[q][0], v[q][1], v[q][2], v[q][3]};
                *reinterpret_cast<f3u*>(r + 4) = f3u{v[q][4], v[q][5], v[q][6]};
            }
        }
    }
}


// Timeline of one wave per block (lane 0 stores): s_memtime at phase boundaries of the
// onebar + spec + sincos + termdone variant.
__global__ __launch_bounds__(256) void k_stamp(pm_env_params p, pm_env_state s, const int8_t* __restrict__ aA,
                                               const int8_t* __restrict__ aB, Out o, uint64_t seed, int n,
                                               unsigned long long* stamps) {
    __shared__ float lds[2][256][7];
    unsigned long long ts[8];
    ts[0] = __builtin_amdgcn_s_memtime();
    const int i0 = blockIdx.x * 256;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0}, tA[7] = {0}, tB[7] = {0};
    int32_t ns = __builtin_nontemporal_load(&s.serves[i]);
    __builtin_amdgcn_sched_barrier(0);
    Arena a = load_arena(s, i);
    const int xa = aA[i], xb = aB[i];
    double svx = 0, svy = 0, ssp = 0;
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    ts[1] = __builtin_amdgcn_s_memtime();
    serve_sincos(p, (uint32_t)i, (uint32_t)ns, seed, svx, svy, ssp);
    asm volatile("" :: "v"(svx), "v"(svy), "v"(ssp));
    ts[2] = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ts[3] = __builtin_amdgcn_s_memtime();
    float ra = 0.f, rb = 0.f;
    const int d = tick(p, a, xa, xb, ra, rb);
    asm volatile("" :: "v"(a.x), "v"(a.y), "v"(a.vx), "v"(a.vy), "v"(d));
    ts[4] = __builtin_amdgcn_s_memtime();
    observe(a, oA, oB);
#pragma unroll
    for (int k = 0; k < 7; ++k) { tA[k] = oA[k]; tB[k] = oB[k]; }
    if (d) {
        serve(a, svx, svy, ssp);
        s.serves[i] = ns + 1;
        observe(a, oA, oB);
        float* r = o.tA + (size_t)i * 7;
        float* q = o.tB + (size_t)i * 7;
#pragma unroll
        for (int k = 0; k < 7; ++k) { r[k] = tA[k]; q[k] = tB[k]; }
    }
    store_arena(s, i, a);
    o.rA[i] = ra;
    o.rB[i] = rb;
    o.done[i] = (uint8_t)d;
    ts[5] = __builtin_amdgcn_s_memtime();
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 7; ++k) { lds[0][t][k] = oA[k]; lds[1][t][k] = oB[k]; }
    __syncthreads();
    ts[6] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        float4* d4 = reinterpret_cast<float4*>((q ? o.obsB : o.obsA) + (size_t)i0 * 7);
        const float4* s4 = reinterpret_cast<const float4*>(&lds[q][0][0]);
        for (int f = t; f < 256 * 7 / 4; f += 256) d4[f] = s4[f];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ts[7] = __builtin_amdgcn_s_memtime();
    if ((t & 63) == 0) {
        unsigned long long* dst = stamps + ((size_t)blockIdx.x * 4 + (t >> 6)) * 8;
        for (int k = 0; k < 8; ++k) dst[k] = ts[k];
    }
}

struct Bufs {
    double* f64;
    int32_t* i32;
    pm_env_state st;
    Out o;
    int8_t *aA, *aB;
};

static Bufs alloc(int n) {
    Bufs b;
    CK(hipMalloc(&b.f64, sizeof(double) * 7 * n));
    CK(hipMalloc(&b.i32, sizeof(int32_t) * 4 * n));
    b.st = {b.f64, b.f64 + n, b.f64 + 2 * (size_t)n, b.f64 + 3 * (size_t)n, b.f64 + 4 * (size_t)n,
            b.f64 + 5 * (size_t)n, b.f64 + 6 * (size_t)n, b.i32, b.i32 + n, b.i32 + 2 * (size_t)n,
            b.i32 + 3 * (size_t)n};
    float* f;
    CK(hipMalloc(&f, sizeof(float) * (size_t)n * 30));
    b.o = {f, f + 7 * (size_t)n, f + 14 * (size_t)n, f + 15 * (size_t)n, f + 16 * (size_t)n, f + 23 * (size_t)n,
           nullptr};
    CK(hipMalloc(&b.o.done, n));
    CK(hipMalloc(&b.aA, n));
    CK(hipMalloc(&b.aB, n));
    return b;
}

typedef void (*Launch)(const pm_env_params&, Bufs&, uint64_t, int, hipStream_t);

__global__ void k_empty(int n) {}
static void launch_empty(const pm_env_params& p, Bufs& b, uint64_t seed, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_empty, dim3((n + 255) / 256), dim3(256), 0, st, n);
}

template <int BLOCK, int STORE, bool SPEC, int TRIG, int TERM = 0, int SKEL = 0>
static void launch(const pm_env_params& p, Bufs& b, uint64_t seed, int n, hipStream_t st) {
    hipLaunchKernelGGL((k_var<BLOCK, STORE, SPEC, TRIG, TERM, SKEL>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, p, b.st,
                       b.aA, b.aB, b.o, seed, n);
}

struct Var {
    const char* name;
    Launch fn;
};

int main(int argc, char** argv) {
    std::vector<int> ns;
    for (int k = 1; k < argc; ++k) ns.push_back(atoi(argv[k]));
    if (ns.empty()) ns = {65536, 262144, 1048576};
    pm_env_params p = {};
    p.paddle_width = 0.2; p.paddle_speed = 0.03; p.magnus_factor = 0.025; p.restitution = 1.0; p.friction = 0.6;
    p.ball_mass = 1.0; p.radius = 0.03; p.speed_lo = 0.03; p.speed_hi = 0.05; p.spin_lo = -5; p.spin_hi = 5;
    p.ang0_lo = -60; p.ang0_hi = -30; p.ang1_lo = 30; p.ang1_hi = 60; p.half_width = 0.1;
    p.speed_scale = 1.0 + 0.1; p.inertia = 0.4 * 1.0 * 0.03 * 0.03; p.jt_coef = (2.0 * 1.0) / 7.0;
    p.max_score = 3; p.speed_scale_every = 1; p.enable_spin = 1;
    Var vars[] = {
        {"base256", launch<256, 0, false, 0>},   {"onebar256", launch<256, 1, false, 0>},
        {"direct256", launch<256, 2, false, 0>}, {"direct256_spec", launch<256, 2, true, 0>},
        {"direct256_spec_sincos", launch<256, 2, true, 1>}, {"direct256_sincos", launch<256, 2, false, 1>},
        {"onebar256_spec_sincos", launch<256, 1, true, 1>}, {"direct128_spec_sincos", launch<128, 2, true, 1>},
        {"direct64_spec_sincos", launch<64, 2, true, 1>},
        {"onebar256_spec_sincos_termdone", launch<256, 1, true, 1, 1>},
        {"onebar256_skeleton_termdone", launch<256, 1, false, 0, 1, 1>},
        {"onebar256_skeleton", launch<256, 1, false, 0, 0, 1>},
        {"empty256", launch_empty},
        {"wave256_spec_sincos_termdone", launch<256, 3, true, 1, 1>},
        {"wave256_spec_sincos", launch<256, 3, true, 1, 0>},
    };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t seed = 77;

    if (getenv("K1_STAMP")) {
        const int n = 65536;
        Bufs b = alloc(n);
        std::vector<double> f0(7 * (size_t)n);
        std::vector<int32_t> i0(4 * (size_t)n, 0);
        std::vector<int8_t> ha(n), hb(n);
        for (int k = 0; k < n; ++k) {
            ha[k] = rand() % 3; hb[k] = rand() % 3;
            f0[k] = 0.5; f0[n + k] = 0.5; f0[2 * (size_t)n + k] = 0.02; f0[3 * (size_t)n + k] = 0.035;
            f0[4 * (size_t)n + k] = (k % 11) - 5; f0[5 * (size_t)n + k] = 0.5; f0[6 * (size_t)n + k] = 0.5;
        }
        CK(hipMemcpy(b.aA, ha.data(), n, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.aB, hb.data(), n, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.f64, f0.data(), 8 * f0.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(b.i32, i0.data(), 4 * i0.size(), hipMemcpyHostToDevice));
        unsigned long long* dst;
        const int nw = n / 64;
        CK(hipMalloc(&dst, sizeof(unsigned long long) * 8 * nw));
        std::vector<unsigned long long> h(8 * (size_t)nw);
        std::vector<std::vector<double>> acc(8);
        for (int t = 0; t < 300; ++t) {
            hipLaunchKernelGGL(k_stamp, dim3(n / 256), dim3(256), 0, st, p, b.st, b.aA, b.aB, b.o, seed, n, dst);
            if (t >= 100 && t % 10 == 0) {
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(h.data(), dst, 8 * h.size(), hipMemcpyDeviceToHost));
                unsigned long long t0 = ~0ull, tend = 0;
                for (int w = 0; w < nw; ++w) { t0 = std::min(t0, h[w * 8]); tend = std::max(tend, h[w * 8 + 7]); }
                for (int w = 0; w < nw; ++w) {
                    acc[0].push_back((double)(h[w * 8] - t0));
                    for (int k = 1; k < 8; ++k) acc[k].push_back((double)(h[w * 8 + k] - h[w * 8 + k - 1]));
                }
                acc[0].push_back(-1.0 * (double)(tend - t0));  // span marker (negative)
            }
        }
        const char* names[8] = {"start offset", "serves load", "serve draw", "rest of loads", "tick", "serve+state stores", "lds+barrier", "obs stores drained"};
        for (int k = 0; k < 8; ++k) {
            std::vector<double> v;
            double span = 0; int ns_ = 0;
            for (double x : acc[k]) { if (x < 0) { span += -x; ns_++; } else v.push_back(x); }
            std::sort(v.begin(), v.end());
            printf("%-22s median %8.0f  p90 %8.0f cycles\n", names[k], v[v.size() / 2], v[v.size() * 9 / 10]);
            if (k == 0) printf("%-22s mean %8.0f cycles\n", "span (first start->last end)", span / ns_);
        }
        return 0;
    }
    for (int n : ns) {
        Bufs b = alloc(n), ref = alloc(n);
        // realistic state: serve every arena, then 300 base steps with random actions
        std::vector<int8_t> ha(n), hb(n);
        srand(1);
        for (int k = 0; k < n; ++k) { ha[k] = rand() % 3; hb[k] = rand() % 3; }
        CK(hipMemcpy(b.aA, ha.data(), n, hipMemcpyHostToDevice));
        CK(hipMemcpy(b.aB, hb.data(), n, hipMemcpyHostToDevice));
        std::vector<double> f0(7 * (size_t)n);
        std::vector<int32_t> i0(4 * (size_t)n, 0);
        for (int k = 0; k < n; ++k) {
            f0[k] = 0.5; f0[n + k] = 0.5; f0[2 * (size_t)n + k] = 0.02; f0[3 * (size_t)n + k] = 0.035;
            f0[4 * (size_t)n + k] = (k % 11) - 5; f0[5 * (size_t)n + k] = 0.5; f0[6 * (size_t)n + k] = 0.5;
        }
        CK(hipMemcpy(b.f64, f0.data(), 8 * f0.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(b.i32, i0.data(), 4 * i0.size(), hipMemcpyHostToDevice));
        for (int t = 0; t < 300; ++t) {
            for (int k = 0; k < n; k += 997) { ha[k] = (ha[k] + 1) % 3; }
            vars[0].fn(p, b, seed, n, st);
        }
        CK(hipStreamSynchronize(st));
        std::vector<double> snap_f(7 * (size_t)n), out_f(7 * (size_t)n), ref_f(7 * (size_t)n);
        std::vector<int32_t> snap_i(4 * (size_t)n), out_i(4 * (size_t)n), ref_i(4 * (size_t)n);
        std::vector<float> out_o(30 * (size_t)n), ref_o(30 * (size_t)n);
        CK(hipMemcpy(snap_f.data(), b.f64, 8 * snap_f.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(snap_i.data(), b.i32, 4 * snap_i.size(), hipMemcpyDeviceToHost));
        for (int v = 0; v < NV; ++v) {
            // correctness: 40 steps from the snapshot, compare with the base variant
            CK(hipMemcpy(b.f64, snap_f.data(), 8 * snap_f.size(), hipMemcpyHostToDevice));
            CK(hipMemcpy(b.i32, snap_i.data(), 4 * snap_i.size(), hipMemcpyHostToDevice));
            for (int t = 0; t < 40; ++t) vars[v].fn(p, b, seed, n, st);
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(out_f.data(), b.f64, 8 * out_f.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(out_i.data(), b.i32, 4 * out_i.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(out_o.data(), b.o.obsA, 4 * out_o.size(), hipMemcpyDeviceToHost));
            if (v == 0) { ref_f = out_f; ref_i = out_i; ref_o = out_o; }
            const bool same = !memcmp(out_f.data(), ref_f.data(), 8 * ref_f.size()) &&
                              !memcmp(out_i.data(), ref_i.data(), 4 * ref_i.size()) &&
                              !memcmp(out_o.data(), ref_o.data(), 4 * ref_o.size());
            // timing: 200 back-to-back launches
            for (int t = 0; t < 10; ++t) vars[v].fn(p, b, seed, n, st);
            const int R = 200;
            if (getenv("K1_GRAPH")) {
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
                for (int t = 0; t < 50; ++t) vars[v].fn(p, b, seed, n, st);
                CK(hipStreamEndCapture(st, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGraphLaunch(ge, st));
                CK(hipEventRecord(e0, st));
                for (int t = 0; t < R / 50; ++t) CK(hipGraphLaunch(ge, st));
                CK(hipEventRecord(e1, st));
            } else {
                CK(hipEventRecord(e0, st));
                for (int t = 0; t < R; ++t) vars[v].fn(p, b, seed, n, st);
                CK(hipEventRecord(e1, st));
            }
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / R;
            printf("{\"n\": %d, \"variant\": \"%s\", \"us\": %.2f, \"GBs_259B\": %.0f, \"bitexact_vs_base\": %s}\n", n,
                   vars[v].name, us, (double)n * 259 / (us * 1e-6) / 1e9, same ? "true" : "false");
            fflush(stdout);
        }
    }
    return 0;
}
