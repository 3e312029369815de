// K1 — batched PongEnv2P reset / step over struct-of-arrays fp64 arenas, one arena per lane.
//
// HBM-bound: per env-step 203 algorithmic bytes (fp64 state 7x8 read + write, int32 scores /
// bounces 12 read + write, actions 2, obs 56, rewards 8, done 1). Observations leave the kernel
// through an LDS transpose so every store is a full 16-byte-per-lane coalesced write.
#include <stdlib.h>

#include "pm_dev.h"
#include "pm_host.h"

using namespace pm;

namespace {

constexpr int kBlock = 256;
static_assert(kBlock == kRowBlock, "row staging assumes kRowBlock-thread blocks");

__device__ __forceinline__ void do_serve(const pm_env_params& p, const pm_env_state& s, Arena& a, int i,
                                         const double* __restrict__ inject, int inject_cap, uint64_t seed,
                                         int32_t* status) {
    const int32_t ns = s.serves[i];
    double vx, vy, sp;
    if (inject) {
        const double* r = inject + ((size_t)i * inject_cap + (ns % inject_cap)) * 3;
        vx = r[0]; vy = r[1]; sp = r[2];
    } else {
        philox_serve(p, (uint32_t)i, (uint32_t)ns, seed, vx, vy, sp);
    }
    serve(a, vx, vy, sp);
    s.serves[i] = ns + 1;
}

__global__ __launch_bounds__(kBlock) void k_env_reset(pm_env_params p, pm_env_state s, const uint8_t* __restrict__ mask,
                                                      const double* __restrict__ inject, int inject_cap, uint64_t seed,
                                                      float* __restrict__ obsA, float* __restrict__ obsB,
                                                      int32_t* status, int n) {
    __shared__ __attribute__((aligned(16))) float lds[kBlock][7];
    const int i0 = blockIdx.x * kBlock;
    const int i = i0 + threadIdx.x;
    float oA[7] = {0}, oB[7] = {0};
    if (i < n) {
        Arena a = load_arena(s, i);
        if (!mask || mask[i]) {
            do_serve(p, s, a, i, inject, inject_cap, seed, status);
            store_arena(s, i, a);
        }
        observe(a, oA, oB);
    }
    if (obsA) store_rows7(obsA, lds, oA, i0, n);
    if (obsB) store_rows7(obsB, lds, oB, i0, n);
}

#ifdef PM_DIAG
// K1 per-wave timeline (diagnostic build only): lane 0 of every wave stamps s_memtime at the phase
// boundaries of k_env_step; pm_k1_diag_read copies [8][4096] out.
static __device__ unsigned long long pm_k1_diag[8][4096];
#define K1_STAMP(k)                                                                             \
    do {                                                                                        \
        const unsigned w_ = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);                    \
        if ((threadIdx.x & 63) == 0 && w_ < 4096) pm_k1_diag[(k)][w_] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define K1_DRAIN() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define K1_STAMP(k) \
    do {            \
    } while (0)
#define K1_DRAIN() \
    do {           \
    } while (0)
#endif

// One lane per arena, one wave per SIMD at 65 536 arenas: the kernel is a single load -> tick ->
// store pass, so its time is the serial latency of that pass. What keeps it short:
//   - the production serve (two Philox draws + sincos) is keyed by (arena, env-step counter), a
//     kernel argument (ABI 15), so every lane draws it while its state loads are in flight: the
//     draw no longer waits for a loaded per-arena serve counter, and that counter's 8 bytes per
//     arena are neither read nor written (round 2 keyed it by the serve count and drew it beside the
//     tick);
//   - tick() is branch-free, with one shared collide path and reciprocal-multiply division;
//   - the production reset is branch-free too: every lane forms the served arena and done lanes
//     select it, so the state stores follow the tick directly, and the term rows of done lanes
//     leave last, after the block's observation rows;
//   - every observation row of the block is staged in LDS once, behind one barrier, and leaves as
//     full float4 stores;
//   - the autoreset mode and parity-mode injection are template parameters, so no uniform branch
//     splits the hot block.
// AR (autoreset): 0 none, 1 reset + full term rows (term row = the step's pre-reset observation),
// 2 reset + term rows written for done arenas only (the other rows are left as they were).
// WT: write-through outputs (pm_dev.h st_out), chosen by the arena count at launch.
//
// k_env_step_w (round 5, the default): the same tick with WAVE-level observation staging. Every wave
// stages its own 64 rows in a private LDS slice and reads them back as float4s (the LDS operations of
// one wave complete in issue order), so no workgroup barrier sits between a wave's tick and its
// stores and each wave's serial chain is its own: load -> draw + tick -> LDS row staging -> one store
// burst (observation float4s, state, rewards, done). The block variant above waited at
// __syncthreads for the block's slowest wave (median 416, p90 1 332 cycles) between its state stores
// and its observation stores (profiles/r4_k1_experiments.txt). PONGMI_K1_STG=0 selects it (A/B).
template <int AR, bool INJ, bool WT>
__global__ __launch_bounds__(kBlock) void k_env_step_w(pm_env_params p, pm_env_state s, const int8_t* __restrict__ aA,
                                                       const int8_t* __restrict__ aB, float* __restrict__ obsA,
                                                       float* __restrict__ obsB, float* __restrict__ rA,
                                                       float* __restrict__ rB, uint8_t* __restrict__ done,
                                                       float* __restrict__ tobsA, float* __restrict__ tobsB,
                                                       const double* __restrict__ inject, int inject_cap,
                                                       uint64_t seed, uint64_t ctr, int32_t* status, int n) {
    __shared__ __attribute__((aligned(16))) float lds[4][kBlock][7];
    constexpr bool DRAW = AR && !INJ;
    const int t = threadIdx.x;
    const int lane = t & 63, w0 = t & ~63;
    const int iw = blockIdx.x * kBlock + w0;  // first arena of this wave
    if (iw >= n) return;                      // whole wave past the end (no barrier in this kernel)
    const int i = iw + lane;
    const int wrows = min(64, n - iw);
    const bool full_term = tobsA && AR != 2;
    float oA[7] = {0}, oB[7] = {0}, tA[7], tB[7];
    int d = 0;
    Arena a{};
    float ra = 0.f, rb = 0.f;
    K1_STAMP(0);
    if (i < n) {
        int32_t ns = 0;
        ServeDraw sv{};
        if (INJ) ns = __builtin_nontemporal_load(&s.serves[i]);
        a = load_arena(s, i);
        const int xa = aA[i], xb = aB[i];
        if (DRAW) {
            sv = serve_draw(p, (uint32_t)i, (uint32_t)ctr, seed, TAG_SERVE_STEP, (uint32_t)(ctr >> 32));
            asm volatile("" ::"v"(sv.vx), "v"(sv.vy), "v"(sv.spin), "v"(sv.rad));
        }
#ifdef PM_DIAG
        K1_DRAIN();
        K1_STAMP(1);
#endif
        d = tick(p, a, xa, xb, ra, rb);
        K1_STAMP(2);
        observe(a, oA, oB);
        if (full_term) {
#pragma unroll
            for (int k = 0; k < 7; ++k) { lds[2][t][k] = oA[k]; lds[3][t][k] = oB[k]; }
        }
        if constexpr (DRAW) {
#pragma unroll
            for (int k = 0; k < 7; ++k) { tA[k] = oA[k]; tB[k] = oB[k]; }
            serve_finish(sv);  // the rare |angle| >= 135 degree redo
            Arena r = a;
            serve(r, sv.vx, sv.vy, sv.spin);
            a.x = d ? r.x : a.x; a.y = d ? r.y : a.y; a.vx = d ? r.vx : a.vx; a.vy = d ? r.vy : a.vy;
            a.spin = d ? r.spin : a.spin; a.top = d ? r.top : a.top; a.bot = d ? r.bot : a.bot;
            a.sA = d ? 0 : a.sA; a.sB = d ? 0 : a.sB; a.bounces = d ? 0 : a.bounces;
            observe(a, oA, oB);
        } else if (AR && d) {
            if (AR == 2 && tobsA) {
                store_row7(tobsA + (size_t)i * 7, oA);
                store_row7(tobsB + (size_t)i * 7, oB);
            }
            const double* r = inject + ((size_t)i * inject_cap + (ns % inject_cap)) * 3;
            serve(a, r[0], r[1], r[2]);
            s.serves[i] = ns + 1;
            observe(a, oA, oB);
        }
    }
    K1_STAMP(3);
    // the wave's rows: LDS slice [w0, w0 + 64) of each staging array, 1 792 B, 16-B aligned
#pragma unroll
    for (int k = 0; k < 7; ++k) { lds[0][t][k] = oA[k]; lds[1][t][k] = oB[k]; }
    // wave-scope ordering only: the rows are read back by lanes of the same wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    K1_STAMP(4);
    const int nq = full_term ? 4 : 2;
    float* const dsts[4] = {obsA, obsB, tobsA, tobsB};
    const size_t rowoff = (size_t)iw * 7;
    bool vec = wrows == 64;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (q < nq) vec = vec && ((((uintptr_t)(dsts[q] + rowoff)) & 15) == 0);
    if (vec) {
        // read every float4 first, then one burst of stores: observations, state, rewards, done
        float4 f[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < nq) {
                const float4* s4 = reinterpret_cast<const float4*>(&lds[q][w0][0]);
                f[q][0] = s4[lane];
                if (lane < 48) f[q][1] = s4[64 + lane];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < nq) {
                float4* d4 = reinterpret_cast<float4*>(dsts[q] + rowoff);
                st_f4<WT>(d4 + lane, f[q][0]);
                if (lane < 48) st_f4<WT>(d4 + 64 + lane, f[q][1]);
            }
        }
    } else {
        for (int q = 0; q < nq; ++q)
            for (int e = lane; e < wrows * 7; e += 64) dsts[q][rowoff + e] = (&lds[q][w0][0])[e];
    }
    if (i < n) {
        store_arena<WT>(s, i, a);
        st_out<WT>(&rA[i], ra);
        st_out<WT>(&rB[i], rb);
        done[i] = (uint8_t)d;
        if (DRAW && AR == 2 && tobsA && d) {
            store_row7(tobsA + (size_t)i * 7, tA);
            store_row7(tobsB + (size_t)i * 7, tB);
        }
    }
    K1_STAMP(5);
    K1_DRAIN();
    K1_STAMP(6);
}

template <int AR, bool INJ, bool WT>
__global__ __launch_bounds__(kBlock) void k_env_step(pm_env_params p, pm_env_state s, const int8_t* __restrict__ aA,
                                                     const int8_t* __restrict__ aB, float* __restrict__ obsA,
                                                     float* __restrict__ obsB, float* __restrict__ rA,
                                                     float* __restrict__ rB, uint8_t* __restrict__ done,
                                                     float* __restrict__ tobsA, float* __restrict__ tobsB,
                                                     const double* __restrict__ inject, int inject_cap,
                                                     uint64_t seed, uint64_t ctr, int32_t* status, int n) {
    __shared__ __attribute__((aligned(16))) float lds[4][kBlock][7];
    constexpr bool DRAW = AR && !INJ;
    const int i0 = blockIdx.x * kBlock;
    const int t = threadIdx.x;
    const int i = i0 + t;
    const bool full_term = tobsA && AR != 2;  // tobsA and tobsB are both set or both null
    float oA[7] = {0}, oB[7] = {0}, tA[7], tB[7];
    int tdone = 0;
    K1_STAMP(0);
    if (i < n) {
        int32_t ns = 0;
        ServeDraw sv{};
        if (INJ) ns = __builtin_nontemporal_load(&s.serves[i]);
        Arena a = load_arena(s, i);
        const int xa = aA[i], xb = aB[i];
        // the step-keyed draw depends on no load: it runs while the state is in flight, and is
        // pinned complete ahead of the tick (the compiler would sink it into the done lanes' path)
        if (DRAW) {
            sv = serve_draw(p, (uint32_t)i, (uint32_t)ctr, seed, TAG_SERVE_STEP, (uint32_t)(ctr >> 32));
            asm volatile("" ::"v"(sv.vx), "v"(sv.vy), "v"(sv.spin), "v"(sv.rad));
        }
#ifdef PM_DIAG
        K1_DRAIN();
        K1_STAMP(1);
#endif
        float ra, rb;
        const int d = tick(p, a, xa, xb, ra, rb);
        K1_STAMP(2);
        observe(a, oA, oB);
        if (full_term) {
#pragma unroll
            for (int k = 0; k < 7; ++k) { lds[2][t][k] = oA[k]; lds[3][t][k] = oB[k]; }
        }
        if constexpr (DRAW) {
#pragma unroll
            for (int k = 0; k < 7; ++k) { tA[k] = oA[k]; tB[k] = oB[k]; }
            serve_finish(sv);  // the rare |angle| >= 135 degree redo (a branch no lane normally takes)
            Arena r = a;
            serve(r, sv.vx, sv.vy, sv.spin);
            a.x = d ? r.x : a.x; a.y = d ? r.y : a.y; a.vx = d ? r.vx : a.vx; a.vy = d ? r.vy : a.vy;
            a.spin = d ? r.spin : a.spin; a.top = d ? r.top : a.top; a.bot = d ? r.bot : a.bot;
            a.sA = d ? 0 : a.sA; a.sB = d ? 0 : a.sB; a.bounces = d ? 0 : a.bounces;
            observe(a, oA, oB);
        } else if (AR && d) {  // parity mode: the injected serve of done arenas
            if (AR == 2 && tobsA) {
                store_row7(tobsA + (size_t)i * 7, oA);
                store_row7(tobsB + (size_t)i * 7, oB);
            }
            const double* r = inject + ((size_t)i * inject_cap + (ns % inject_cap)) * 3;
            serve(a, r[0], r[1], r[2]);
            s.serves[i] = ns + 1;
            observe(a, oA, oB);
        }
        store_arena<WT>(s, i, a);
        st_out<WT>(&rA[i], ra);
        st_out<WT>(&rB[i], rb);
        done[i] = (uint8_t)d;
        tdone = d;
    }
    K1_STAMP(3);
#pragma unroll
    for (int k = 0; k < 7; ++k) { lds[0][t][k] = oA[k]; lds[1][t][k] = oB[k]; }
    __syncthreads();
    K1_STAMP(4);
    copy_rows7<WT>(obsA, lds[0], i0, n);
    copy_rows7<WT>(obsB, lds[1], i0, n);
    if (full_term) {
        copy_rows7<WT>(tobsA, lds[2], i0, n);
        copy_rows7<WT>(tobsB, lds[3], i0, n);
    }
    if (DRAW && AR == 2 && tobsA && tdone) {
        store_row7(tobsA + (size_t)i * 7, tA);
        store_row7(tobsB + (size_t)i * 7, tB);
    }
    K1_STAMP(5);
    K1_DRAIN();
    K1_STAMP(6);
}

__global__ __launch_bounds__(kBlock) void k_collide(const double* __restrict__ in, const double* __restrict__ inertia,
                                                    double* __restrict__ out, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double* r = in + (size_t)i * 8;
    pm_env_params p = {};
    p.restitution = r[4]; p.friction = r[5]; p.ball_mass = r[6]; p.radius = r[7];
    p.inertia = inertia[i];
    p.jt_coef = (2.0 * r[6]) / 7.0;
    p.inv_mass = 1.0 / r[6];
    p.inv_inertia = 1.0 / p.inertia;
    double vn2, vt2, om2;
    collide(p, r[0], r[1], r[2], r[3], vn2, vt2, om2);
    out[(size_t)i * 3 + 0] = vn2;
    out[(size_t)i * 3 + 1] = vt2;
    out[(size_t)i * 3 + 2] = om2;
}

// Write-through K1 outputs up to kK1WtMax arenas (latency-bound sizes); PONGMI_K1_WT=0/1 forces
// the choice (experiments).
constexpr int32_t kK1WtMax = 131072;
int k1_write_through(int32_t n) {
    static const int forced = [] {
        const char* e = getenv("PONGMI_K1_WT");
        return e && *e ? atoi(e) : -1;
    }();
    return forced >= 0 ? (forced != 0) : (n <= kK1WtMax);
}

// Wave-level observation staging (k_env_step_w) unless PONGMI_K1_STG=0 (the block-barrier A/B).
int k1_wave_staging() {
    static const int v = [] {
        const char* e = getenv("PONGMI_K1_STG");
        return e && *e ? (atoi(e) != 0) : 1;
    }();
    return v;
}

bool state_ok(const pm_env_state* s) {
    return s && s->x && s->y && s->vx && s->vy && s->spin && s->top && s->bot && s->scoreA && s->scoreB &&
           s->bounces && s->serves;
}

}  // namespace

extern "C" int pm_env_reset(const pm_env_params* p, const pm_env_state* s, const uint8_t* mask, const double* inject,
                            int32_t inject_cap, uint64_t seed, float* obsA, float* obsB, int32_t* status, int32_t n,
                            void* stream) {
    PM_REQUIRE(n >= 0, PM_E_SIZE, "pm_env_reset: n=%d", n);
    if (n == 0) return PM_OK;
    PM_REQUIRE(p && state_ok(s), PM_E_ARG, "pm_env_reset: null params/state");
    PM_REQUIRE(!inject || inject_cap > 0, PM_E_ARG, "pm_env_reset: inject without capacity");
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "pm_env_reset: speed_scale_every must be > 0");
    if (n == 0) return PM_OK;
    hipLaunchKernelGGL(k_env_reset, dim3(pm_blocks(n, kBlock)), dim3(kBlock), 0, pm_stream(stream), *p, *s, mask,
                       inject, inject_cap, seed, obsA, obsB, status, n);
    PM_LAUNCHED("k_env_reset");
    return PM_OK;
}

extern "C" int pm_env_step(const pm_env_params* p, const pm_env_state* s, const int8_t* aA, const int8_t* aB,
                           float* obsA, float* obsB, float* rA, float* rB, uint8_t* done, float* term_obsA,
                           float* term_obsB, int32_t autoreset, const double* inject, int32_t inject_cap,
                           uint64_t seed, uint64_t counter, int32_t* status, int32_t n, void* stream) {
    PM_REQUIRE(n >= 0, PM_E_SIZE, "pm_env_step: n=%d", n);
    if (n == 0) return PM_OK;
    PM_REQUIRE(p && state_ok(s), PM_E_ARG, "pm_env_step: null params/state");
    PM_REQUIRE(aA && aB && obsA && obsB && rA && rB && done, PM_E_ARG, "pm_env_step: null buffer");
    PM_REQUIRE(!term_obsA == !term_obsB, PM_E_ARG, "pm_env_step: term_obsA and term_obsB must both be set or both NULL");
    PM_REQUIRE(autoreset >= 0 && autoreset <= 2, PM_E_ARG, "pm_env_step: autoreset=%d not in {0,1,2}", autoreset);
    PM_REQUIRE(!inject || inject_cap > 0, PM_E_ARG, "pm_env_step: inject without capacity");
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "pm_env_step: speed_scale_every must be > 0");
    using K = decltype(&k_env_step<0, false, false>);
    static const K kernels[2][2][3][2] = {
        {{{k_env_step<0, false, false>, k_env_step<0, true, false>},
          {k_env_step<1, false, false>, k_env_step<1, true, false>},
          {k_env_step<2, false, false>, k_env_step<2, true, false>}},
         {{k_env_step<0, false, true>, k_env_step<0, true, true>},
          {k_env_step<1, false, true>, k_env_step<1, true, true>},
          {k_env_step<2, false, true>, k_env_step<2, true, true>}}},
        {{{k_env_step_w<0, false, false>, k_env_step_w<0, true, false>},
          {k_env_step_w<1, false, false>, k_env_step_w<1, true, false>},
          {k_env_step_w<2, false, false>, k_env_step_w<2, true, false>}},
         {{k_env_step_w<0, false, true>, k_env_step_w<0, true, true>},
          {k_env_step_w<1, false, true>, k_env_step_w<1, true, true>},
          {k_env_step_w<2, false, true>, k_env_step_w<2, true, true>}}}};
    pm_launch(PM_TIMER_ENV_STEP, kernels[k1_wave_staging()][k1_write_through(n)][autoreset][inject != nullptr],
              dim3(pm_blocks(n, kBlock)),
              dim3(kBlock), pm_stream(stream), *p, *s, aA, aB, obsA, obsB, rA, rB, done, term_obsA, term_obsB, inject,
              inject_cap, seed, counter, status, n);
    PM_LAUNCHED("k_env_step");
    return PM_OK;
}

#ifdef PM_DIAG
extern "C" int pm_k1_diag_read(uint64_t* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pm_k1_diag), sizeof(pm_k1_diag), 0, hipMemcpyDeviceToHost);
}
#endif

extern "C" int pm_collide(const double* in, const double* inertia, double* out, int32_t n, void* stream) {
    PM_REQUIRE(n >= 0, PM_E_SIZE, "pm_collide: n=%d", n);
    if (n == 0) return PM_OK;
    PM_REQUIRE(in && inertia && out, PM_E_ARG, "pm_collide: null buffer");
    hipLaunchKernelGGL(k_collide, dim3(pm_blocks(n, kBlock)), dim3(kBlock), 0, pm_stream(stream), in, inertia, out, n);
    PM_LAUNCHED("k_collide");
    return PM_OK;
}
