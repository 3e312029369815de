// K1 — batched PongEnv2P reset / step over struct-of-arrays fp64 arenas, one arena per lane.
//
// HBM-bound: per env-step 203 algorithmic bytes (fp64 state 7x8 read + write, int32 scores /
// bounces 12 read + write, actions 2, obs 56, rewards 8, done 1). Observations leave the kernel
// through an LDS transpose so every store is a full 16-byte-per-lane coalesced write.
#include <stdlib.h>
#include <string.h>

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
// PRO (round 5, the default): the prologue is ordered for latency. Every lane loads from a clamped
// index (i < n ? i : n - 1), so no bounds branch splits the kernel-argument loads into two dependent
// scalar rounds (bound n first, then the pointers: ~2 scalar-cache round trips before the first
// vector load), and a scheduling barrier keeps every state / action load ahead of the serve draw —
// without it the compiler interleaved ~100 Philox instructions in front of the state loads and ~200
// in front of the score loads. Stores stay guarded by i < n. PONGMI_K1_PRO=0 selects the round-4
// prologue (A/B). Round-5 measurements that were NOT kept (profiles/r5_k1_experiments.txt): wave-level
// observation staging without the workgroup barrier (one store burst 4.25 us, state stores first
// 4.19 us, against 4.11 us with the barrier), and 16-B per-lane state accesses (field pairs / quads per
// instruction: the copy skeleton 4.12 against 3.53 us).
template <int AR, bool INJ, bool WT, int PRO>
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
    if ((PRO & 1) || i < n) {
        const int il = (PRO & 1) ? (i < n ? i : n - 1) : i;  // the loads' index (clamped: no bounds branch)
        int32_t ns = 0;
        ServeDraw sv{};
        if (INJ) ns = __builtin_nontemporal_load(&s.serves[il]);
        Arena a = load_arena(s, il);
        const int xa = aA[il], xb = aB[il];
        if (PRO & 2) __builtin_amdgcn_sched_barrier(0);  // every load issued before the draw's first instruction
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
            if (AR == 2 && tobsA && i < n) {
                store_row7(tobsA + (size_t)i * 7, oA);
                store_row7(tobsB + (size_t)i * 7, oB);
            }
            const double* r = inject + ((size_t)il * inject_cap + (ns % inject_cap)) * 3;
            serve(a, r[0], r[1], r[2]);
            if (i < n) s.serves[i] = ns + 1;
            observe(a, oA, oB);
        }
        if (i < n) {
            store_arena<WT>(s, i, a);
            st_out<WT>(&rA[i], ra);
            st_out<WT>(&rB[i], rb);
            done[i] = (uint8_t)d;
            tdone = d;
        }
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

// The scalar drop-in's fast path (PongEnv2P, one arena: envs/my_pong_env_2p.py:83-225). One lane
// steps / serves arena 0 with the same tick / serve / observe as K1 (so its results are K1's for
// n = 1 bit for bit), writes obsA[7] obsB[7] rA rB done to `out` and then `seq` to out word 17 with
// a system-scope release: `out` is normally host-mapped memory (pm_host_mapped_alloc), which the
// host polls, so one call costs one launch and no copy or stream synchronisation.
__device__ __forceinline__ void emit1(float* out, const float (&oA)[7], const float (&oB)[7], float ra, float rb,
                                      float dn, uint32_t seq) {
#pragma unroll
    for (int k = 0; k < 7; ++k) { out[k] = oA[k]; out[7 + k] = oB[k]; }
    out[14] = ra; out[15] = rb; out[16] = dn;
    __hip_atomic_store(reinterpret_cast<uint32_t*>(out + 17), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(64) void k_env_step1(pm_env_params p, pm_env_state s, int xa, int xb, float* out,
                                                  uint32_t seq) {
    if (threadIdx.x != 0) return;
    Arena a = load_arena(s, 0);
    float ra, rb, oA[7], oB[7];
    const int d = tick(p, a, xa, xb, ra, rb);
    store_arena(s, 0, a);
    observe(a, oA, oB);
    emit1(out, oA, oB, ra, rb, (float)d, seq);
}
__global__ __launch_bounds__(64) void k_env_reset1(pm_env_state s, double vx, double vy, double spin, float* out,
                                                   uint32_t seq) {
    if (threadIdx.x != 0) return;
    Arena a;
    serve(a, vx, vy, spin);
    store_arena(s, 0, a);
    s.serves[0] = s.serves[0] + 1;
    float oA[7], oB[7];
    observe(a, oA, oB);
    emit1(out, oA, oB, 0.f, 0.f, 0.f, seq);
}
__global__ __launch_bounds__(64) void k_collide1(double vn, double vt, double u, double om, double e, double mu,
                                                 double m, double R, double inertia, double* out, uint32_t seq) {
    if (threadIdx.x != 0) return;
    pm_env_params p = {};
    p.restitution = e; p.friction = mu; p.ball_mass = m; p.radius = R;
    p.inertia = inertia;
    p.jt_coef = (2.0 * m) / 7.0;
    p.inv_mass = 1.0 / m;
    p.inv_inertia = 1.0 / inertia;
    collide(p, vn, vt, u, om, out[0], out[1], out[2]);
    __hip_atomic_store(reinterpret_cast<uint32_t*>(out + 3), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

// K1 prologue (PONGMI_K1_PRO, A/B; bit 0 clamped loads, bit 1 loads ahead of the draw): 3 (default)
// both, 0 round 4's.
int k1_prologue() {
    static const int v = [] {
        const char* e = getenv("PONGMI_K1_PRO");
        const int x = e && *e ? atoi(e) : 3;
        return x >= 0 && x <= 3 ? x : 3;
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
    using K = decltype(&k_env_step<0, false, false, 3>);
#define PM_K1_SET(PRO)                                                                               \
    {{{k_env_step<0, false, false, PRO>, k_env_step<0, true, false, PRO>},                           \
      {k_env_step<1, false, false, PRO>, k_env_step<1, true, false, PRO>},                           \
      {k_env_step<2, false, false, PRO>, k_env_step<2, true, false, PRO>}},                          \
     {{k_env_step<0, false, true, PRO>, k_env_step<0, true, true, PRO>},                             \
      {k_env_step<1, false, true, PRO>, k_env_step<1, true, true, PRO>},                             \
      {k_env_step<2, false, true, PRO>, k_env_step<2, true, true, PRO>}}}
    static const K kernels[4][2][3][2] = {PM_K1_SET(0), PM_K1_SET(1), PM_K1_SET(2), PM_K1_SET(3)};
#undef PM_K1_SET
    pm_launch(PM_TIMER_ENV_STEP, kernels[k1_prologue()][k1_write_through(n)][autoreset][inject != nullptr],
              dim3(pm_blocks(n, kBlock)),
              dim3(kBlock), pm_stream(stream), *p, *s, aA, aB, obsA, obsB, rA, rB, done, term_obsA, term_obsB, inject,
              inject_cap, seed, counter, status, n);
    PM_LAUNCHED("k_env_step");
    return PM_OK;
}

extern "C" int pm_env_step1(const pm_env_params* p, const pm_env_state* s, int32_t aA, int32_t aB, float* out,
                            uint32_t seq, void* stream) {
    PM_REQUIRE(p && state_ok(s) && out, PM_E_ARG, "pm_env_step1: null params/state/out");
    PM_REQUIRE(aA >= 0 && aA <= 2 && aB >= 0 && aB <= 2, PM_E_ARG, "pm_env_step1: actions (%d, %d)", aA, aB);
    PM_REQUIRE(p->speed_scale_every > 0, PM_E_ARG, "pm_env_step1: speed_scale_every must be > 0");
    hipLaunchKernelGGL(k_env_step1, dim3(1), dim3(64), 0, pm_stream(stream), *p, *s, (int)aA, (int)aB, out, seq);
    PM_LAUNCHED("k_env_step1");
    return PM_OK;
}

extern "C" int pm_env_reset1(const pm_env_state* s, double vx, double vy, double spin, float* out, uint32_t seq,
                             void* stream) {
    PM_REQUIRE(state_ok(s) && out, PM_E_ARG, "pm_env_reset1: null state/out");
    hipLaunchKernelGGL(k_env_reset1, dim3(1), dim3(64), 0, pm_stream(stream), *s, vx, vy, spin, out, seq);
    PM_LAUNCHED("k_env_reset1");
    return PM_OK;
}

extern "C" int pm_collide1(const double* row, double inertia, double* out, uint32_t seq, void* stream) {
    PM_REQUIRE(row && out, PM_E_ARG, "pm_collide1: null row/out");
    hipLaunchKernelGGL(k_collide1, dim3(1), dim3(64), 0, pm_stream(stream), row[0], row[1], row[2], row[3], row[4],
                       row[5], row[6], row[7], inertia, out, seq);
    PM_LAUNCHED("k_collide1");
    return PM_OK;
}

extern "C" void* pm_host_mapped_alloc(int64_t bytes, void** dev) {
    void* h = nullptr;
    if (bytes <= 0 || !dev) return nullptr;
    if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    memset(h, 0, (size_t)bytes);
    if (hipHostGetDevicePointer(dev, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return nullptr;
    }
    return h;
}

extern "C" int pm_host_mapped_free(void* host) {
    if (!host) return PM_OK;
    const hipError_t e = hipHostFree(host);
    return e == hipSuccess ? PM_OK : pm_fail((int)e, "pm_host_mapped_free: %s", hipGetErrorString(e));
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
