// Device-side building blocks shared by the libpongmi kernels (gfx950 / CDNA4, wave64).
//
//   philox()        counter-based RNG (Philox4x32-10): every draw is a pure function of
//                   (seed, index, purpose, step) -> results never depend on launch geometry.
//   Arena/tick()    one PongEnv2P.step on a register-resident arena (envs/my_pong_env_2p.py:116-232,
//                   envs/physics.py:3-23), IEEE binary64 in the reference's evaluation order.
//                   The library is compiled with -ffp-contract=off: no FMA is ever formed here.
//   fold_heads()    NoisyLinear folding / reset_noise (models/qnet.py:33-50) of the two dueling heads.
//   (the MFMA QNet forward lives in pm_mfma.h)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pongmi.h"

#ifdef PM_DIAG
// TU-local (no -fgpu-rdc): only pm_selfplay.hip stamps, and it exports the reader.
static __device__ unsigned long long pm_diag_buf[256];
#define PM_STAMP(slot)                                                                 \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x == 0) pm_diag_buf[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define PM_STAMP_ANY(slot)                                                             \
    do {                                                                               \
        if (threadIdx.x == 0) pm_diag_buf[(slot)] = __builtin_amdgcn_s_memrealtime();  \
    } while (0)
// per-block timeline of one kernel: [0] begin, [1] ready (inputs staged), [2] end (all waves),
// [3] placement: CU id (__smid) | XCC id << 16, [4..7] kernel-specific mid points
static __device__ unsigned long long pm_diag_blk[8][4096];
#define PM_BLK_END()                                                                              \
    do {                                                                                          \
        __syncthreads();                                                                          \
        PM_BLK(2);                                                                                \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                                \
            pm_diag_blk[3][blockIdx.x] =                                                          \
                (unsigned long long)__smid() | ((unsigned long long)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15) << 16); \
    } while (0)
#define PM_BLK(k)                                                                                  \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 4096) pm_diag_blk[(k)][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// latest end over the blocks of one role (block-wide: a barrier, then thread 0's atomic max)
#define PM_STAMP_MAX(slot)                                                                              \
    do {                                                                                                \
        __syncthreads();                                                                                \
        if (threadIdx.x == 0) atomicMax(&pm_diag_buf[(slot)], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#define PM_STAMP_T(slot, tid)                                                                            \
    do {                                                                                                 \
        if (threadIdx.x == (tid) && blockIdx.x == 0) pm_diag_buf[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PM_BLK(k) \
    do {          \
    } while (0)
#define PM_BLK_END() \
    do {             \
    } while (0)
#define PM_STAMP_T(slot, tid) \
    do {                      \
    } while (0)
#define PM_STAMP_MAX(slot) \
    do {                   \
    } while (0)
#define PM_STAMP_ANY(slot) \
    do {                   \
    } while (0)
#define PM_STAMP(slot) \
    do {               \
    } while (0)
#endif

namespace pm {

// ----------------------------------------------------------------------------- wave reductions
// A wave's butterfly reduction `for (o = 32; o; o >>= 1) v = op(v, __shfl_xor(v, o))` on the DPP
// and scalar paths instead of six ds_bpermute round trips (~2 us for six int64 chains in the learner's
// phase 0). After the xor-1 / xor-2 steps (quad_perm) every quad holds one value, so the half-row /
// row mirrors pair each lane with a lane holding its xor-4 / xor-8 partner's value; the last two steps
// are (a0 + a16) + (a32 + a48) from four readlanes. The pairing runs xor-1 first, the reverse of the
// loop above (xor-32 first), so the result equals the loop's bit for bit only for an associative op
// (integer sums, max, min); a float sum is the same 63 additions in a different association (ADVICE
// r5) and is covered by the tolerance tests of its callers, not by bit-identity. Full waves only
// (every lane active). Result wave-uniform.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(dpp_i32<CTRL>(__float_as_int(v)));
}
template <int CTRL>
__device__ __forceinline__ long long dpp_i64(long long v) {
    const int lo = dpp_i32<CTRL>((int)(unsigned long long)v), hi = dpp_i32<CTRL>((int)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    return __longlong_as_double(dpp_i64<CTRL>(__double_as_longlong(v)));
}
__device__ __forceinline__ int lane_i32(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float lane_f32(float v, int l) { return __int_as_float(lane_i32(__float_as_int(v), l)); }
__device__ __forceinline__ long long lane_i64(long long v, int l) {
    const unsigned lo = (unsigned)lane_i32((int)(unsigned long long)v, l);
    const unsigned hi = (unsigned)lane_i32((int)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double lane_f64(double v, int l) { return __longlong_as_double(lane_i64(__double_as_longlong(v), l)); }
#define PM_WAVE_RED(T, SUF, OP)                                                                   \
    __device__ __forceinline__ T wave_##OP(T v) {                                                 \
        v = pm_op_##OP(v, dpp_##SUF<0xB1>(v));  /* quad_perm [1,0,3,2]: xor 1 */                   \
        v = pm_op_##OP(v, dpp_##SUF<0x4E>(v));  /* quad_perm [2,3,0,1]: xor 2 */                   \
        v = pm_op_##OP(v, dpp_##SUF<0x141>(v)); /* row_half_mirror: = xor 4 here */                \
        v = pm_op_##OP(v, dpp_##SUF<0x140>(v)); /* row_mirror: = xor 8 here */                     \
        return pm_op_##OP(pm_op_##OP(lane_##SUF(v, 0), lane_##SUF(v, 16)),                        \
                          pm_op_##OP(lane_##SUF(v, 32), lane_##SUF(v, 48)));                      \
    }
template <class T>
__device__ __forceinline__ T pm_op_sum(T a, T b) { return a + b; }
__device__ __forceinline__ float pm_op_max(float a, float b) { return fmaxf(a, b); }
PM_WAVE_RED(long long, i64, sum)
PM_WAVE_RED(int, i32, sum)
PM_WAVE_RED(float, f32, sum)
PM_WAVE_RED(double, f64, sum)
PM_WAVE_RED(float, f32, max)
#undef PM_WAVE_RED
// Quad broadcasts on DPP (quad_perm [I,I,I,I]): lane (lane & ~3) + I's value in every lane of the
// quad, as __shfl(v, (lane & ~3) + I) without the LDS crossbar. quad_sel: the quad-uniform lane src's.
// Full waves only.
template <int I>
__device__ __forceinline__ double quad_f64(double v) { return dpp_f64<I * 0x55>(v); }
template <int I>
__device__ __forceinline__ int quad_i32(int v) { return dpp_i32<I * 0x55>(v); }
__device__ __forceinline__ double quad_sel_f64(double v, int src) {
    const double a = quad_f64<0>(v), b = quad_f64<1>(v), c = quad_f64<2>(v), d = quad_f64<3>(v);
    return src == 0 ? a : src == 1 ? b : src == 2 ? c : d;
}
__device__ __forceinline__ int quad_sel_i32(int v, int src) {
    const int a = quad_i32<0>(v), b = quad_i32<1>(v), c = quad_i32<2>(v), d = quad_i32<3>(v);
    return src == 0 ? a : src == 1 ? b : src == 2 ? c : d;
}
// Inclusive prefix sum of a full wave on DPP: Hillis-Steele within each 16-lane row (row_shr 1/2/4/8,
// lanes shifted in from outside the row read 0), then the row carries (row_bcast:15 into rows 1 and 3,
// row_bcast:31 into rows 2 and 3). Integers only (the association differs from a lane-serial scan).
__device__ __forceinline__ int wave_incl_scan_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

// ----------------------------------------------------------------------------- RNG
enum : uint32_t { TAG_SERVE = 1, TAG_ACT = 2, TAG_OPP = 3, TAG_NOISE_ACT = 4, TAG_PER = 5, TAG_NOISE_TRAIN = 6, TAG_NOISE_RNN = 7, TAG_SEQ = 8,
                  TAG_SERVE_STEP = 9 };

struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t key) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of mul_hi + mul_lo: the
        // 32-bit integer multiplies are quarter-rate, and this halves them (same bits)
        const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

__device__ __forceinline__ U4 philox64(uint32_t index, uint32_t tag, uint64_t ctr, uint64_t key) {
    return philox(index, tag, (uint32_t)ctr, (uint32_t)(ctr >> 32), key);
}

// uniform double in [0, 1) with 53 random bits (like CPython's random.random())
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
    return (double)v * 0x1.0p-53;
}
// uniform integer in [0, n) (randint(0, n-1)); bias <= n / 2^32
__device__ __forceinline__ int32_t below(uint32_t r, uint32_t n) {
    return (int32_t)(((uint64_t)r * n) >> 32);
}
// One N(0,1) float by Box-Muller (cos branch) from two u32: the torch.randn stand-in (distribution
// parity with the reference). Evaluated in double with +, -, *, /, sqrt only — a fixed polynomial
// log (atanh series on m in [sqrt(1/2), sqrt(2))) and cos (Taylor on the octant-reduced angle) —
// then rounded once to float. Every step is a correctly rounded IEEE operation (this file builds with
// -ffp-contract=off), so the oracle's numpy restatement (oracle.normal_f32) reproduces every draw bit
// for bit: the noise, and with it every NoisyNet forward, is pinned exactly, not to an ulp band.
// Accuracy: log and cos within ~1e-16 relative, far below the float the result is rounded to.
__device__ __forceinline__ double det_ln_u1(uint32_t k) {  // ln(k * 2^-24), k in [1, 2^24]
    int e = 31 - __builtin_clz(k);                        // k = m 2^e, m in [1, 2)
    double m = (double)k / (double)(1u << e);             // exact
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;  // ln m = 2 atanh(s)
    const double p = s2 * (0.66666666666666663 + s2 * (0.40000000000000002 + s2 * (0.28571428571428570 +
                     s2 * (0.22222222222222221 + s2 * (0.18181818181818182 + s2 * (0.15384615384615385 +
                     s2 * (0.13333333333333333 + s2 * (0.11764705882352941 + s2 * (0.10526315789473684 +
                     s2 * 0.09523809523809523)))))))));
    return (double)(e - 24) * 0.69314718055994531 + (2.0 * s + s * p);
}
__device__ __forceinline__ double det_cos_turn(double t) {  // cos(2 pi t), t in [0, 1) (24-bit grid)
    const double q = floor(4.0 * t + 0.5);                 // octant-centred quadrant 0..4
    const double th = 6.2831853071795862 * (t - 0.25 * q);  // [-pi/4, pi/4]
    const double z = th * th;
    const double c = 1.0 + z * (-0.5 + z * (0.041666666666666664 + z * (-0.0013888888888888889 +
                     z * (2.4801587301587302e-05 + z * (-2.755731922398589e-07 + z * (2.0876756987868100e-09 +
                     z * -1.1470745597729725e-11))))));
    const double s = th * (1.0 + z * (-0.16666666666666666 + z * (0.0083333333333333332 + z * (-0.00019841269841269841 +
                     z * (2.7557319223985893e-06 + z * (-2.5052108385441720e-08 + z * (1.6059043836821613e-10 +
                     z * -7.6471637318198164e-13)))))));
    const int qi = (int)q & 3;
    return qi == 0 ? c : (qi == 1 ? -s : (qi == 2 ? -c : s));
}
__device__ __forceinline__ float normal(uint32_t a, uint32_t b) {
    const double r = sqrt(-2.0 * det_ln_u1((a >> 8) + 1u));  // u1 = ((a >> 8) + 1) 2^-24 in (0, 1]
    return (float)(r * det_cos_turn((double)(b >> 8) * 0x1.0p-24));  // u2 in [0, 1)
}
// NoisyLinear._scale_noise (models/qnet.py:35-36): sign(x) * sqrt(|x|), the root correctly rounded
__device__ __forceinline__ float scale_noise(float x) {
    const float s = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    return s * (float)sqrt((double)fabsf(x));
}

// ----------------------------------------------------------------------------- environment
struct Arena {
    double x, y, vx, vy, spin, top, bot;
    int32_t sA, sB, bounces;
};

__device__ __forceinline__ Arena load_arena(const pm_env_state& s, int i) {
    Arena a;
    a.x = s.x[i]; a.y = s.y[i]; a.vx = s.vx[i]; a.vy = s.vy[i];
    a.spin = s.spin[i]; a.top = s.top[i]; a.bot = s.bot[i];
    a.sA = s.scoreA[i]; a.sB = s.scoreB[i]; a.bounces = s.bounces[i];
    return a;
}

// Output stores. WT = write-through (sc1): the line leaves this XCD's L2 with the store instead of
// staying dirty there until the kernel-end write-back, which the next dependent launch waits for
// (≈ dirty bytes / 6 TB/s). Worth it where a kernel is latency-bound and its outputs are not re-read
// from this L2 soon (measured: K1 at 65 536 arenas 4.50 -> 4.41 us; at 262 144, store-throughput
// bound, 9.4 -> 10.5 us, since narrow sc1 stores are separate fabric writes).
template <bool WT, typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
typedef float pm_f4v __attribute__((ext_vector_type(4)));
template <bool WT>
__device__ __forceinline__ void st_f4(float4* p, float4 v) {
    if constexpr (WT) {
        const pm_f4v x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
    } else {
        *p = v;
    }
}

template <bool WT = false>
__device__ __forceinline__ void store_arena(const pm_env_state& s, int i, const Arena& a) {
    st_out<WT>(&s.x[i], a.x); st_out<WT>(&s.y[i], a.y); st_out<WT>(&s.vx[i], a.vx); st_out<WT>(&s.vy[i], a.vy);
    st_out<WT>(&s.spin[i], a.spin); st_out<WT>(&s.top[i], a.top); st_out<WT>(&s.bot[i], a.bot);
    st_out<WT>(&s.scoreA[i], a.sA); st_out<WT>(&s.scoreB[i], a.sB); st_out<WT>(&s.bounces[i], a.bounces);
}

// _get_obs_for_A / _get_obs_for_B (envs/my_pong_env_2p.py:235-257): fp64 -> f32 round-to-nearest
__device__ __forceinline__ void observe(const Arena& a, float* oA, float* oB) {
    oA[0] = (float)a.x; oA[1] = (float)(1.0 - a.y); oA[2] = (float)a.vx; oA[3] = (float)(-a.vy);
    oA[4] = (float)a.top; oA[5] = (float)a.bot; oA[6] = (float)a.spin;
    oB[0] = (float)a.x; oB[1] = (float)a.y; oB[2] = (float)a.vx; oB[3] = (float)a.vy;
    oB[4] = (float)a.bot; oB[5] = (float)a.top; oB[6] = (float)a.spin;
}

// Row staging for [n][7] f32 outputs. Every kernel that stages rows runs kRowBlock-thread blocks and
// declares its staging array 16-byte aligned, so a block's rows leave LDS as ds_read_b128 and reach
// HBM as full global_store_dwordx4 (BLOCK * 7 / 4 float4s, two per thread), with no runtime trip
// count (a row-per-lane store of 28-byte rows would be seven 4-byte stores per lane).
constexpr int kRowBlock = 256;

// The copy-out of rows the caller already staged in LDS (and fenced with a barrier): several outputs
// can share one barrier. No barrier inside.
template <bool WT = false>
__device__ __forceinline__ void copy_rows7(float* __restrict__ dst, const float (*lds)[7], int i0, int n) {
    const int t = threadIdx.x;
    const int rows = min(kRowBlock, n - i0);
    float* base = dst + (size_t)i0 * 7;
    const float* src = &lds[0][0];
    if (rows == kRowBlock && (((uintptr_t)base) & 15) == 0) {
        float4* d4 = reinterpret_cast<float4*>(base);
        const float4* s4 = reinterpret_cast<const float4*>(__builtin_assume_aligned(src, 16));
#pragma unroll
        for (int f = t; f < kRowBlock * 7 / 4; f += kRowBlock) st_f4<WT>(d4 + f, s4[f]);
    } else {
        for (int f = t; f < rows * 7; f += kRowBlock) base[f] = src[f];
    }
}

// Stage one row per thread in LDS and copy the block's rows out. Block-wide, two barriers.
__device__ __forceinline__ void store_rows7(float* __restrict__ dst, float (*lds)[7], const float* row, int i0,
                                            int n) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 7; ++k) lds[t][k] = row[k];
    __syncthreads();
    copy_rows7(dst, lds, i0, n);
    __syncthreads();
}

// One 28-byte row written by its own lane as dwordx4 + dwordx3 (4-byte aligned: gfx950 global
// stores take unaligned addresses), for scattered rows that are not worth an LDS round trip.
typedef float pm_f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float pm_f3u __attribute__((ext_vector_type(3), aligned(4)));
__device__ __forceinline__ void store_row7(float* __restrict__ dst, const float* v) {
    *reinterpret_cast<pm_f4u*>(dst) = pm_f4u{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<pm_f3u*>(dst + 4) = pm_f3u{v[4], v[5], v[6]};
}

// reset() (:83-114) with a given serve (vx, vy, spin)
__device__ __forceinline__ void serve(Arena& a, double vx, double vy, double spin) {
    a.sA = 0; a.sB = 0; a.bounces = 0;
    a.top = 0.5; a.bot = 0.5; a.x = 0.5; a.y = 0.5;
    a.vx = vx; a.vy = vy; a.spin = spin;
}

// sin and cos of x for |x| < 3*pi/4 (serve angles are within +-135 degrees for any sane config;
// the caller falls back to OCML otherwise), straight-line: one Cody-Waite step by pi/2 with a
// two-part constant (fdlibm __ieee754_rem_pio2's first case) and fdlibm's __kernel_sin /
// __kernel_cos polynomials on the reduced pair (y0, y1), the quadrant applied by selects. Error
// < 1 ulp, as OCML's sincos; no branch, so the draw schedules together with the env tick.
__device__ __forceinline__ void sincos_serve(double x, double& s, double& c) {
    const double pio4 = 7.85398163397448278999e-01;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const int n = x > pio4 ? 1 : (x < -pio4 ? -1 : 0);
    const double z0 = n > 0 ? x - pio2_1 : x + pio2_1;
    const double t = n > 0 ? pio2_1t : -pio2_1t;
    double y0 = z0 - t;
    double y1 = (z0 - y0) - t;
    y0 = n == 0 ? x : y0;
    y1 = n == 0 ? 0.0 : y1;
    // __kernel_sin(y0, y1, 1)
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = y0 * y0, v = z * y0;
    const double rs = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double ks = y0 - ((z * (0.5 * y1 - v * rs) - y1) - v * S1);
    // __kernel_cos(y0, y1): |y0| <= pi/4 < 0.78125, fdlibm's plain branch
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double kc = w + (((1.0 - w) - hz) + (z * rc - y0 * y1));
    s = n == 0 ? ks : (n > 0 ? kc : -kc);
    c = n == 0 ? kc : (n > 0 ? -ks : ks);
}

// Production serve draws from Philox: speed = U(lo,hi), coin < 0.5 picks the angle interval,
// angle = U(interval) degrees -> radians (math.radians: deg * (pi/180)), spin = U(lo,hi).
// serve_draw is straight-line (hot kernels draw it for every lane beside the tick); serve_finish
// redoes the rare |angle| >= 135 degree case with OCML's sincos, where the serve is applied.
struct ServeDraw {
    double speed, rad, vx, vy, spin;
};
// Counter (i, tag, c2, c3): (i, TAG_SERVE, serve number, 0) for the serve-count stream, (i,
// TAG_SERVE_STEP, step lo, step hi) for K1's step-keyed production stream.
__device__ __forceinline__ ServeDraw serve_draw(const pm_env_params& p, uint32_t i, uint32_t nserve, uint64_t seed,
                                                uint32_t tag = TAG_SERVE, uint32_t c3 = 0u) {
    const U4 r0 = philox(i, tag, nserve, c3, seed);
    const U4 r1 = philox(i, tag | 0x100u, nserve, c3, seed);
    ServeDraw d;
    d.speed = p.speed_lo + (p.speed_hi - p.speed_lo) * u53(r0.x, r0.y);
    const bool first = u53(r0.z, r0.w) < 0.5;
    const double lo = first ? p.ang0_lo : p.ang1_lo, hi = first ? p.ang0_hi : p.ang1_hi;
    const double ang = lo + (hi - lo) * u53(r1.x, r1.y);
    d.rad = ang * (3.141592653589793 / 180.0);
    double sn, cs;
    sincos_serve(d.rad, sn, cs);
    d.vx = d.speed * cs;
    d.vy = d.speed * sn;
    d.spin = p.spin_lo + (p.spin_hi - p.spin_lo) * u53(r1.z, r1.w);
    return d;
}
__device__ __forceinline__ void serve_finish(ServeDraw& d) {
    if (!(fabs(d.rad) < 2.35619449019234483700)) {
        double sn, cs;
        sincos(d.rad, &sn, &cs);
        d.vx = d.speed * cs;
        d.vy = d.speed * sn;
    }
}
__device__ __forceinline__ void philox_serve(const pm_env_params& p, uint32_t i, uint32_t nserve, uint64_t seed,
                                             double& vx, double& vy, double& spin) {
    ServeDraw d = serve_draw(p, i, nserve, seed);
    serve_finish(d);
    vx = d.vx; vy = d.vy; spin = d.spin;
}

__device__ __forceinline__ double clip01(double v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); }

// a / b for a divisor b with correctly rounded reciprocal inv = RN(1/b): q = RN(a*inv) is within an
// ulp of a/b, and one FMA residual step q + RN(a - b*q)*inv rounds correctly (Markstein's theorem,
// for results clear of under/overflow; checked against IEEE division on 2.4e8 random operands for
// the divisors the configs produce). Zero dividends keep their sign, as a/b does.
__device__ __forceinline__ double div_by(double a, double b, double inv) {
    const double q = a * inv;
    const double r = __builtin_fma(-q, b, a);
    const double q2 = __builtin_fma(r, inv, q);
    return a == 0.0 ? q : q2;
}

// collide_sphere_with_moving_plane (envs/physics.py:3-23)
__device__ __forceinline__ void collide(const pm_env_params& p, double vn, double vt, double u, double om,
                                        double& vn2, double& vt2, double& om2) {
    const double e = p.restitution, m = p.ball_mass, R = p.radius;
    vn2 = (-e) * vn;
    const double Jn = (m * (1.0 + e)) * fabs(vn);
    const double Jt_star = p.jt_coef * ((u + R * om) - vt);
    const double mf = p.friction * Jn;
    const double vrel = (vt - u) - R * om;  // used only when sliding (|Jt*| > mu Jn)
    const double Jt = fabs(Jt_star) <= mf ? Jt_star : (-mf) * copysign(1.0, vrel);
    vt2 = vt + div_by(Jt, m, p.inv_mass);
    om2 = om - div_by(R * Jt, p.inertia, p.inv_inertia);
}

// One PongEnv2P.step. Returns done; rewards are exactly -1/0/+1.
// Straight-line code: every branch of the reference is evaluated and the taken side selected
// (v_cndmask), so the whole tick is one basic block the scheduler can interleave with other
// independent work (the next serve's draw) and no lane waits on another lane's side of a branch.
// Every selected value is computed by the reference's own expression in its order, so selection
// changes no bit. A paddle hit at the top (y < 0, player A) and at the bottom (y > 1, player B)
// share one collide evaluation: the bottom case is the top case with vn = -vy and vy' = -vn' (exact
// negations). `bounces % every == 0` is true for every == 1, as the reference's `every == 1 or`.
__device__ __forceinline__ int tick(const pm_env_params& p, Arena& a, int aA, int aB, float& rA, float& rB) {
    // paddle: top - ps == top + (-ps) exactly, and top + 0.0 == top for the paddle's range (never
    // -0.0: it starts at 0.5 and x - x rounds to +0.0), so one add of a selected step is the
    // reference's if/elif
    const double ps = p.paddle_speed;
    a.top = clip01(a.top + (aA == 0 ? -ps : (aA == 2 ? ps : 0.0)));
    a.bot = clip01(a.bot + (aB == 0 ? -ps : (aB == 2 ? ps : 0.0)));

    double vx = p.enable_spin ? a.vx + (p.magnus_factor * a.spin) * a.vy : a.vx;
    double x = a.x + vx;
    const double y = a.y + a.vy;
    const bool wl = x < 0.0, wr = x > 1.0;
    x = wl ? -x : (wr ? 2.0 - x : x);
    vx = (wl || wr) ? -vx : vx;

    const bool low = y < 0.0, high = y > 1.0;
    const double pad = low ? a.top : a.bot;
    const bool inside = (pad - p.half_width) <= x && x <= (pad + p.half_width);
    const bool hit = (low || high) && inside;
    const int act = low ? aA : aB;
    const double u = act == 0 ? -ps : (act == 2 ? ps : 0.0);
    double vn2, vt2, om2;
    collide(p, low ? a.vy : -a.vy, vx, u, a.spin, vn2, vt2, om2);
    // materialise the impulse for every lane here: otherwise the compiler sinks it into a branch
    // on `hit`, which splits the tick into separately scheduled blocks
    asm volatile("" : "+v"(vn2), "+v"(vt2), "+v"(om2));
    const int nb = a.bounces + 1;
    const bool scale = nb % p.speed_scale_every == 0;
    const double hvy = low ? vn2 : -vn2;
    a.x = x;
    a.vx = hit ? (scale ? vt2 * p.speed_scale : vt2) : vx;
    a.vy = hit ? (scale ? hvy * p.speed_scale : hvy) : a.vy;
    a.spin = hit ? om2 : a.spin;
    a.y = hit ? (low ? 0.0 : 1.0) : y;
    a.bounces = hit ? nb : a.bounces;

    const bool missA = low && !inside, missB = high && !inside;  // A defends y < 0, B defends y > 1
    a.sB += missA ? 1 : 0;
    a.sA += missB ? 1 : 0;
    rA = missA ? -1.f : (missB ? 1.f : 0.f);
    rB = missA ? 1.f : (missB ? -1.f : 0.f);
    return missA ? (a.sB >= p.max_score) : (missB ? (a.sA >= p.max_score) : 0);
}

// ----------------------------------------------------------------------------- QNet
enum : int { W1 = 0, B1 = 448, W2 = 512, B2 = 4608, WH = 4672, BH = 4928 };  // effective-weight offsets
static_assert(BH + 4 == 4932, "plain effective weight layout");

// Parameter-block offsets (pongmi.h PM_QNET_NP layout): heads at PM_QNET_HEAD_OFF, eps at PM_QNET_EPS_OFF
enum : int {
    P_VWMU = PM_QNET_HEAD_OFF + 0, P_VBMU = P_VWMU + 64, P_VWSG = P_VBMU + 1, P_VBSG = P_VWSG + 64,
    P_AWMU = P_VBSG + 1, P_ABMU = P_AWMU + 192, P_AWSG = P_ABMU + 3, P_ABSG = P_AWSG + 192,
    P_VWEP = PM_QNET_EPS_OFF + 0, P_VBEP = P_VWEP + 64, P_AWEP = P_VBEP + 1, P_ABEP = P_AWEP + 192,
};
static_assert(P_ABSG + 3 == PM_QNET_EPS_OFF, "head layout");
static_assert(P_ABEP + 3 == PM_QNET_NP, "eps layout");

// torch argmax: first maximal index
__device__ __forceinline__ int argmax3(const float* q) {
    int b = 0;
    if (q[1] > q[b]) b = 1;
    if (q[2] > q[b]) b = 2;
    return b;
}

// ----------------------------------------------------------------------------- NoisyNet fold
// Head-section offsets (relative to PM_QNET_HEAD_OFF) and eps-section offsets (relative to
// PM_QNET_EPS_OFF) of a parameter block.
enum : int {
    H_VWMU = 0, H_VBMU = 64, H_VWSG = 65, H_VBSG = 129, H_AWMU = 130, H_ABMU = 322, H_AWSG = 325, H_ABSG = 517,
    E_VWEP = 0, E_VBEP = 64, E_AWEP = 65, E_ABEP = 257,
};

// reset_noise() draws (models/qnet.py:33-41) for both heads from Philox(seed, tag, ctr), after
// _scale_noise: noise[0,64) f(eps_in) fc_V | [64] f(eps_out) fc_V | [65,129) f(eps_in) fc_A |
// [129,132) f(eps_out) fc_A. Threads [tid0, tid0 + nt) of the block take part.
__device__ __forceinline__ void gen_noise(uint64_t seed, uint32_t tag, uint64_t ctr, float* noise, int tid, int nt) {
    for (int k = tid; k < 132; k += nt) {
        const uint32_t layer = k < 65 ? 0u : 1u;
        const uint32_t kk = layer ? (uint32_t)(k - 65) : (uint32_t)k;
        const uint32_t which = kk < 64 ? 0u : 1u;
        const uint32_t e = which ? kk - 64 : kk;
        const U4 r = philox64(e, tag | (layer << 8) | (which << 12), ctr, seed);
        noise[k] = scale_noise(normal(r.x, r.y));
    }
}

// Fold the heads (NoisyLinear.forward, models/qnet.py:43-50) into heads[0,260) = Wh [4][64] | bh [4]:
//   EVAL: W = mu;  TRAIN: W = mu + sigma*eps with eps from `eps` (eps-section layout);
//   FRESH: eps = f(eps_out) (x) f(eps_in) from `noise` (gen_noise), also written to eps_out (nullable).
// hp = the 520-float head section (global or LDS). Threads [tid, tid + nt) take part.
__device__ __forceinline__ void fold_heads_from(const float* hp, const float* eps, const float* noise, int mode,
                                                float* heads, float* eps_out, int tid, int nt) {
    for (int k = tid; k < 260; k += nt) {
        // k in [0,256): weight row k/64 (0 = V, 1..3 = A), column k%64; [256,260): biases
        const int row = k < 256 ? k >> 6 : k - 256, col = k & 63;
        const bool w = k < 256;
        float mu, sg, ep = 0.f;
        int eo;
        if (row == 0) {
            mu = w ? hp[H_VWMU + col] : hp[H_VBMU];
            sg = w ? hp[H_VWSG + col] : hp[H_VBSG];
            eo = w ? E_VWEP + col : E_VBEP;
            if (mode == PM_FOLD_TRAIN_FRESH) ep = w ? noise[64] * noise[col] : noise[64];
        } else {
            const int a = row - 1;
            mu = w ? hp[H_AWMU + a * 64 + col] : hp[H_ABMU + a];
            sg = w ? hp[H_AWSG + a * 64 + col] : hp[H_ABSG + a];
            eo = w ? E_AWEP + a * 64 + col : E_ABEP + a;
            if (mode == PM_FOLD_TRAIN_FRESH) ep = w ? noise[129 + a] * noise[65 + col] : noise[129 + a];
        }
        if (mode == PM_FOLD_TRAIN) ep = eps[eo];
        heads[w ? k : 256 + row] = mode == PM_FOLD_EVAL ? mu : mu + sg * ep;  // torch: mu + (sigma*eps)
        if (mode == PM_FOLD_TRAIN_FRESH && eps_out) eps_out[eo] = ep;
    }
}

// One parameter block, block-wide (generates the noise first in FRESH mode). `noise` is LDS
// scratch of >= 132 floats; eps_out (nullable) is the block's eps section to write.
__device__ __forceinline__ void fold_heads(const float* params, float* eps_out, int mode, uint64_t seed, uint32_t tag,
                                           uint64_t ctr, float* heads, float* noise) {
    if (mode == PM_FOLD_TRAIN_FRESH) {
        gen_noise(seed, tag, ctr, noise, threadIdx.x, blockDim.x);
        __syncthreads();
    }
    fold_heads_from(params + PM_QNET_HEAD_OFF, params + PM_QNET_EPS_OFF, noise, mode, heads, eps_out, threadIdx.x,
                    blockDim.x);
}

}  // namespace pm
