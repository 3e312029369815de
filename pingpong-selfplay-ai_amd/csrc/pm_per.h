// PER pieces shared between pm_replay.hip and pm_selfplay.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pongmi.h"
#include "pm_dev.h"

namespace pm {

// Sum tree over the leaves prio^alpha (fp32 leaf array, fp64 nodes), two node levels:
//   leaf[e]  = powf(prio[e], alpha), kept next to the priorities (push and scatter write both)
//   sub[s]   = ((q0 + q1) + q2) + q3, q_k = sequential fp64 sum of leaves [64 s + 16 k, +16)  (level 1)
//   chunk[c] = sequential fp64 sum of sub[16 c .. 16 c + 16)                                  (level 2)
// Every node is always computed by the same functions in the same order, so a node recomputed
// after an incremental change is bit-identical to a full rebuild. The stored leaves mean a node
// refresh is loads + adds (no pow), and 4 threads share a level-1 node (one quarter each).
constexpr int PER_SUB = 64;
constexpr int PER_FAN = 16;
constexpr int PER_CHUNK = PER_SUB * PER_FAN;

__host__ __device__ inline int64_t per_pad(int64_t n_doubles) { return ((n_doubles * 8 + 255) / 256) * 256; }

struct PerTree {
    double* chunk;  // [nchunk]
    double* sub;    // [nsub]
    float* leaf;    // [cap]
    int64_t nchunk, nsub;
};

__host__ __device__ inline PerTree per_tree(void* work, int64_t cap) {
    PerTree t;
    t.nsub = (cap + PER_SUB - 1) / PER_SUB;
    t.nchunk = (cap + PER_CHUNK - 1) / PER_CHUNK;
    char* w = reinterpret_cast<char*>(work);
    t.chunk = reinterpret_cast<double*>(w);
    t.sub = reinterpret_cast<double*>(w + per_pad(t.nchunk));
    t.leaf = reinterpret_cast<float*>(w + per_pad(t.nchunk) + per_pad(t.nsub));
    return t;
}

inline int64_t per_work_bytes(int64_t cap) {
    return per_pad((cap + PER_CHUNK - 1) / PER_CHUNK) + per_pad((cap + PER_SUB - 1) / PER_SUB) +
           ((cap * 4 + 255) / 256) * 256;
}

// The replay push that is about to land (or landing concurrently): entries [pos, pos + n) mod cap
// hold leaf value `pval` = powf(max(prios), alpha) (memory.push stores max(prios),
// train_iterative.py:57) as far as the tree and the sampler are concerned. n = 0: none.
struct PushRange {
    int64_t pos, n, cap;
    float pval;
    __device__ __forceinline__ int64_t dist(int64_t e) const {
        const int64_t d = e - pos;
        return d < 0 ? d + cap : d;
    }
    __device__ __forceinline__ bool covers(int64_t e) const { return dist(e) < n; }
};

__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    return v;
}

// Tree nodes of granularity g (entries per node) overlapping the ring range [pos, pos + n) mod cap:
// ids a0 .. a0 + na - 1 (the part up to cap) then 0 .. nb - 1 (the wrapped part). Overlaps between
// the two segments only repeat a node (same value written twice).
struct RingNodes {
    int64_t a0, na, nb;
    __device__ __forceinline__ int64_t count() const { return na + nb; }
    __device__ __forceinline__ int64_t at(int64_t k) const { return k < na ? a0 + k : k - na; }
};
__device__ __forceinline__ RingNodes ring_nodes(const PushRange& pr, int64_t g) {
    RingNodes r{pr.pos / g, 0, 0};
    if (pr.n <= 0) return r;
    const int64_t end1 = pr.pos + pr.n < pr.cap ? pr.pos + pr.n : pr.cap;
    r.na = (end1 - 1) / g - r.a0 + 1;
    const int64_t end2 = pr.pos + pr.n - pr.cap;
    r.nb = end2 > 0 ? (end2 - 1) / g + 1 : 0;
    return r;
}

// prio ** alpha, PrioritizedReplay's leaf (train_iterative.py:67: prios ** alpha in float32). Formed
// in double from +, -, *, / and exact scalings only — ln p by the atanh series on m in
// [sqrt(1/2), sqrt(2)), exp by a Cody-Waite split and its Taylor series — then rounded once to float:
// within an ulp of numpy's powf (the reference's arithmetic), and a fixed sequence of correctly
// rounded operations, so the oracle (oracle.det_pow_f32) restates every leaf bit for bit; equal to
// the correctly rounded pow on every input and within 1 ulp of numpy's float32 power
// (tests/test_oracle_golden.py::test_det_pow_within_one_ulp_of_numpy_power). Non-positive and NaN
// priorities give a 0 leaf (never sampled); the learner latches pm_ctrl.status bit 1 for a NaN one,
// where the reference's numpy would carry the NaN into np.random.choice (which raises).
__device__ __forceinline__ float prio_pow(float p, float alpha) {
    if (!(p > 0.f)) return 0.f;
    int e;
    double m = 2.0 * frexp((double)p, &e);  // p = m 2^(e - 1), m in [1, 2): exact
    e = e - 1;
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    const double q = s2 * (0.66666666666666663 + s2 * (0.40000000000000002 + s2 * (0.28571428571428570 +
                     s2 * (0.22222222222222221 + s2 * (0.18181818181818182 + s2 * (0.15384615384615385 +
                     s2 * (0.13333333333333333 + s2 * (0.11764705882352941 + s2 * (0.10526315789473684 +
                     s2 * 0.09523809523809523)))))))));
    const double y = (double)alpha * ((double)e * 0.69314718055994531 + (2.0 * s + s * q));
    const double k = floor(y * 1.4426950408889634 + 0.5);
    const double r = (y - k * 6.93147180369123816490e-01) - k * 1.90821492927058770002e-10;  // |r| <= ln2 / 2
    const double ex = 1.0 + r * (1.0 + r * (0.5 + r * (0.16666666666666666 + r * (0.041666666666666664 +
                      r * (0.008333333333333333 + r * (0.001388888888888889 + r * (0.0001984126984126984 +
                      r * (2.48015873015873e-05 + r * (2.7557319223985893e-06 + r * (2.755731922398589e-07 +
                      r * (2.505210838544172e-08 + r * (2.08767569878681e-09 + r * 1.6059043836821613e-10))))))))))));
    return (float)ldexp(ex, (int)k);
}

// Leaf e as the tree sees it: pushed value inside the pending push range, 0 past cap.
__device__ __forceinline__ float per_leaf(const float* __restrict__ leaf, int64_t e, const PushRange& pr) {
    return pr.covers(e) ? pr.pval : (e < pr.cap ? leaf[e] : 0.f);
}

// Quarter k of level-1 node sb: sequential fp64 sum of its 16 leaves (loads issued together).
__device__ __forceinline__ double per_quarter(const float* __restrict__ leaf, int64_t sb, int k, const PushRange pr) {
    const int64_t lo = sb * PER_SUB + 16 * k;
    float v[16];
    if (lo + 16 <= pr.cap) {
        const float4* p4 = reinterpret_cast<const float4*>(leaf + lo);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 x = p4[q];
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lo + i < pr.cap ? leaf[lo + i] : 0.f;
    }
    const int64_t d0 = pr.dist(lo);  // covers(lo + i) without a 64-bit op per leaf
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int64_t d = d0 + i;
        if (d >= pr.cap) d -= pr.cap;
        acc += lo + i < pr.cap ? (double)(d < pr.n ? pr.pval : v[i]) : 0.0;  // past cap: no leaf
    }
    return acc;
}
__device__ __forceinline__ double per_combine(double q0, double q1, double q2, double q3) {
    return ((q0 + q1) + q2) + q3;
}
// Level-1 node, one thread (rebuilds and rare paths).
__device__ __forceinline__ double per_sub_sum(const float* __restrict__ leaf, int64_t sb, const PushRange pr) {
    const double q0 = per_quarter(leaf, sb, 0, pr), q1 = per_quarter(leaf, sb, 1, pr);
    const double q2 = per_quarter(leaf, sb, 2, pr), q3 = per_quarter(leaf, sb, 3, pr);
    return per_combine(q0, q1, q2, q3);
}
// Level-1 node by 4 consecutive lanes (lane & 3 = quarter); the node lands in every lane of the group.
__device__ __forceinline__ double per_sub_sum4(const float* __restrict__ leaf, int64_t sb, const PushRange pr) {
    const int lane = threadIdx.x & 63;
    const double q = per_quarter(leaf, sb, lane & 3, pr);
    return per_combine(quad_f64<0>(q), quad_f64<1>(q), quad_f64<2>(q), quad_f64<3>(q));
}

// A level-1 node wholly inside the push range: the same sums over 16 copies of the pushed leaf.
__device__ __forceinline__ bool per_sub_pushed(int64_t sb, const PushRange pr) {
    const int64_t lo = sb * PER_SUB;
    return lo + PER_SUB <= pr.cap && pr.dist(lo) + PER_SUB <= pr.n;
}
__device__ __forceinline__ double per_sub_pushed_sum(const PushRange pr) {
    double q = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) q += (double)pr.pval;
    return per_combine(q, q, q, q);
}

// Level-2 node c from its 16 level-1 nodes. One thread.
__device__ __forceinline__ double per_chunk_sum(const PerTree& t, int64_t c) {
    double v[PER_FAN];
#pragma unroll
    for (int k = 0; k < PER_FAN; ++k) v[k] = c * PER_FAN + k < t.nsub ? t.sub[c * PER_FAN + k] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < PER_FAN; ++k) acc += v[k];
    return acc;
}

// ----------------------------------------------------------------------------- block sampler
// PrioritizedReplay.sample (scripts/train_iterative.py:64-73): np.random.choice(p) picks the first
// index whose running sum of p exceeds u (searchsorted 'right'). Here a 256-thread block draws
// PER_BS = 64 samples at once, descending the tree in three dependent load round trips:
//   level 2: the block loads every chunk sum once (4 per thread), forms their inclusive prefix in LDS
//            (one block scan) and each sample binary-searches it for t = u * total;
//   level 1: 4 lanes per sample read the chosen chunk's 16 sub sums (4 each), a 4-lane scan finds
//            the sub-block;
//   level 0: the same 4 lanes read its 64 leaves (16 each, one float4 x4 load) and find the entry.
// Compared with one wave per sample, the block does the top-level scan once for 64 samples: the
// wave-wide scans of <= 1024 chunk sums per sample were VALU work that starved beside the act's MFMA
// streams. Every sum has a fixed order, so a sample is a pure function of (tree, u). When rounding
// leaves the target at or past a node's running total, the last nonzero child is taken (as before).
constexpr int PER_BS = 64;       // samples per 256-thread block
constexpr int PER_ROUND = 1024;  // chunk sums per prefix round (capacities <= 1M: one round)

struct PerSampleSmem {
    double incl[PER_ROUND];  // inclusive prefix of the round's chunk sums (plus the earlier rounds)
    double wsum[4];
};

// The round's inclusive prefix of chunk sums [c0, c0 + 1024) into sm.incl, offset by base; returns
// the running total after the round. v: this thread's 4 chunk sums (chunks c0 + 4t .. 4t + 3).
__device__ inline double per_round_prefix(const double (&v)[4], double base, PerSampleSmem& sm) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    double run[4], acc = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) { acc += v[e]; run[e] = acc; }
    const double incl = wave_incl_scan(acc, lane);
    double excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0.0;
    if (lane == 63) sm.wsum[wv] = incl;
    __syncthreads();
    double wb = base;
    for (int w = 0; w < wv; ++w) wb += sm.wsum[w];
    const double ex = wb + excl;
#pragma unroll
    for (int e = 0; e < 4; ++e) sm.incl[4 * t + e] = ex + run[e];
    const double tot = ((base + sm.wsum[0]) + sm.wsum[1]) + sm.wsum[2] + sm.wsum[3];
    __syncthreads();
    return tot;
}

// First k in [0, n) with sm.incl[k] > x (n if none).
__device__ __forceinline__ int per_lds_search(const PerSampleSmem& sm, int n, double x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sm.incl[mid] > x) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// 4-lane group search over the group's 4 x NV values (lane q of the group holds values
// [NV q, NV q + NV) in v, in order): the first value whose running sum exceeds x, else the last
// nonzero one. Returns its index in [0, 4 NV) (every lane of the group), `before` = running sum in
// front of it, `val` = the value.
template <int NV>
__device__ __forceinline__ int per_group_find(const double (&v)[NV], double x, double& before, double& val) {
    const int lane = threadIdx.x & 63, q = lane & 3, g0 = lane & ~3;
    double acc = 0.0;
#pragma unroll
    for (int e = 0; e < NV; ++e) acc += v[e];
    const double s0 = quad_f64<0>(acc), s1 = quad_f64<1>(acc), s2 = quad_f64<2>(acc);
    const double ex = q == 0 ? 0.0 : (q == 1 ? s0 : (q == 2 ? s0 + s1 : (s0 + s1) + s2));
    int hit = -1, nz = -1;
    double hb = 0.0, hv = 0.0, nb = 0.0, nv = 0.0, run = ex;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
        if (hit < 0 && run + v[e] > x) { hit = e; hb = run; hv = v[e]; }
        if (v[e] > 0.0) { nz = e; nb = run; nv = v[e]; }
        run += v[e];
    }
    const unsigned gh = (unsigned)(__ballot(hit >= 0) >> g0) & 15u;
    const unsigned gn = (unsigned)(__ballot(nz >= 0) >> g0) & 15u;
    int src, k;
    if (gh) {
        src = __ffs(gh) - 1;
        k = hit;
    } else {
        src = gn ? 31 - __clz(gn) : 0;
        k = nz < 0 ? 0 : nz;
        hb = nz < 0 ? ex : nb;
        hv = nz < 0 ? 0.0 : nv;
    }
    // every lane computed its candidate; take lane src's (the branch above is group-uniform)
    const int kk = quad_sel_i32(k, src);
    before = quad_sel_f64(hb, src);
    val = quad_sel_f64(hv, src);
    return src * NV + kk;
}

// Block-wide (256 threads, block-uniform arguments): samples j0 .. j0 + 63 (those < bs) with uniforms
// ufn(j), un-normalised IS weights (size * P(i))^-beta. Leaves inside the pending push range read as
// pr.pval (the push kernel may be writing them). out(j, idx, w) is called once per sample. For
// capacities <= 1M the chunk sums are loaded before `active` is tested (the caller's control-block
// read and these loads share one round trip); !active returns with nothing written.
struct NoHook {
    __device__ void operator()() const {}
};
// l2done(): called by every thread once the level-2 search is done (before the level-1 loads), where
// a caller issues work whose loads must not delay the chunk-sum round trip.
template <class UFn, class OutFn, class Hook = NoHook>
__device__ inline void per_sample_block(bool active, int64_t size, const PerTree& tr, const PushRange& pr, double beta,
                                        int j0, int bs, PerSampleSmem& sm, UFn ufn, OutFn out, Hook l2done = Hook()) {
    const int t = threadIdx.x, q = t & 3;
    const int j = j0 + (t >> 2);
    const bool one_round = tr.nchunk <= PER_ROUND;  // kernel-argument uniform
    double vc[4] = {0.0, 0.0, 0.0, 0.0};
    if (one_round) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t c = 4 * t + e;
            vc[e] = c < tr.nchunk ? tr.chunk[c] : 0.0;
        }
        asm volatile("" ::"v"(vc[0]), "v"(vc[1]), "v"(vc[2]), "v"(vc[3]));
    }
    if (!active) return;  // block-uniform
    const int64_t nb = (size + PER_CHUNK - 1) / PER_CHUNK;
    const double u = j < bs ? ufn(j) : 0.0;
    // level 2
    double total = 0.0;
    if (nb > PER_ROUND) {  // capacities > 1M: the total first, one pass over the rounds
        for (int64_t c0 = 0; c0 < nb; c0 += PER_ROUND) {
            double v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t c = c0 + 4 * t + e;
                v[e] = c < nb ? tr.chunk[c] : 0.0;
            }
            total = per_round_prefix(v, total, sm);
        }
    }
    int64_t blk = -1, lastnz = 0;
    double before = 0.0, lastbef = 0.0, x = 0.0, run = 0.0;
    for (int64_t c0 = 0; c0 < nb; c0 += PER_ROUND) {
        double v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t c = c0 + 4 * t + e;
            v[e] = c < nb ? (one_round ? vc[e] : tr.chunk[c]) : 0.0;
        }
        const double end = per_round_prefix(v, run, sm);
        if (nb <= PER_ROUND) total = end;
        x = u * total;
        const int n = (int)(nb - c0 < PER_ROUND ? nb - c0 : PER_ROUND);
        if (blk < 0 && end > run) {
            const int k = per_lds_search(sm, n, x);
            if (k < n) {
                blk = c0 + k;
                before = k ? sm.incl[k - 1] : run;
            } else {  // last nonzero chunk of the round: the first to reach the round's end value
                int lo = 0, hi = n - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sm.incl[mid] >= sm.incl[n - 1]) hi = mid;
                    else lo = mid + 1;
                }
                lastnz = c0 + lo;
                lastbef = lo ? sm.incl[lo - 1] : run;
            }
        }
        run = end;
        __syncthreads();  // sm.incl is rewritten by the next round
    }
    if (blk < 0) { blk = lastnz; before = lastbef; }
    PM_BLK(4);
    l2done();
    // level 1: the chunk's 16 sub sums, 4 per lane of the sample's group
    double sv[4];
    const int64_t s0 = blk * PER_FAN + 4 * q;
#pragma unroll
    for (int e = 0; e < 4; ++e) sv[e] = s0 + e < tr.nsub ? tr.sub[s0 + e] : 0.0;
    double b1, v1;
    const int64_t sb = blk * PER_FAN + per_group_find<4>(sv, x - before, b1, v1);
    PM_BLK(5);
    // level 0: the sub-block's 64 leaves, 16 per lane
    double lv[16];
    {
        const int64_t lo = sb * PER_SUB + 16 * q;
        float f[16];
        if (lo + 16 <= pr.cap) {
            const float4* p4 = reinterpret_cast<const float4*>(tr.leaf + lo);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 a = p4[k];
                f[4 * k] = a.x; f[4 * k + 1] = a.y; f[4 * k + 2] = a.z; f[4 * k + 3] = a.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) f[k] = lo + k < pr.cap ? tr.leaf[lo + k] : 0.f;
        }
        const int64_t d0 = pr.dist(lo);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            int64_t d = d0 + k;
            if (d >= pr.cap) d -= pr.cap;
            lv[k] = lo + k < size ? (double)(d < pr.n ? pr.pval : f[k]) : 0.0;
        }
    }
    double b0, pa;
    const int k = per_group_find<16>(lv, x - before - b1, b0, pa);
    PM_BLK(6);
    if (q == 0 && j < bs) out(j, sb * PER_SUB + k, (float)pow((double)size * (pa / total), -beta));
    PM_BLK(7);
}

// Full rebuild over prios[0, cap): leaves, then level-1 and level-2 nodes with the pending push
// range substituted (from ctrl when non-null, else none).
int per_launch_build(const float* prios, int64_t cap, float alpha, const pm_ctrl* ctrl, int64_t n_push, void* work,
                     hipStream_t st);
int per_launch_update(float* prios, const int64_t* idx, const float* err, int bs, hipStream_t st);
// Level-1 and level-2 nodes over leaves already written (no pending push range).
int per_launch_nodes(void* work, int64_t cap, hipStream_t st);

}  // namespace pm
