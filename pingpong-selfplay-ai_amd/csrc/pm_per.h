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

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

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

__device__ __forceinline__ float prio_pow(float p, float alpha) { return powf(p, alpha); }

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
        acc += (double)(d < pr.n ? pr.pval : v[i]);
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
    const int lane = threadIdx.x & 63, base = lane & ~3;
    const double q = per_quarter(leaf, sb, lane & 3, pr);
    return per_combine(__shfl(q, base), __shfl(q, base + 1), __shfl(q, base + 2), __shfl(q, base + 3));
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

// One value per lane: the first lane whose running sum exceeds t (searchsorted 'right'); if rounding
// leaves t at or past the wave's total, the last nonzero lane. `before` = running sum in front of it.
__device__ inline int lane_find(double v, double t, int lane, double& before, double& val) {
    const double incl = wave_incl_scan(v, lane);
    double excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0.0;
    const unsigned long long hit = __ballot(incl > t);
    int L;
    if (hit) {
        L = __ffsll((long long)hit) - 1;
    } else {
        const unsigned long long nz = __ballot(v > 0.0);
        L = nz ? 63 - __clzll((long long)nz) : 0;
    }
    before = __shfl(excl, L);
    val = __shfl(v, L);
    return L;
}

// Level-2 search helpers: 16 chunk sums per lane (one load round trip per 1024 chunks).
__device__ inline int chunk_find(const double (&vals)[16], double part, double incl, double run, double t, int lane,
                                 double& before) {
    const unsigned long long hit = __ballot(run + incl > t);
    if (!hit) return -1;
    const int L = __ffsll((long long)hit) - 1;
    double base = run + (incl - part), bef = base, lastbef = base;
    int found = -1, lastnz = -1;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (found < 0 && base + vals[e] > t) { found = e; bef = base; }
        if (vals[e] > 0.0) { lastnz = e; lastbef = base; }
        base += vals[e];
    }
    if (found < 0) { found = lastnz; bef = lastbef; }  // rounding: lane sum fell short of its scan
    found = __shfl(found, L);
    before = __shfl(bef, L);
    return found < 0 ? -1 : L * 16 + found;
}

// One wave per sample: idx and the un-normalised IS weight (size * P(i))^-beta for the uniform u.
// Descends chunk sums (scan of <= 1024 per round trip) -> the chunk's 16 level-1 sums -> the 64
// leaves of one sub-block: three dependent load round trips for capacities up to 1M.
// Leaves inside the pending push range read as pr.pval (the push kernel may be writing them).
__device__ inline void per_sample_one(int64_t size, const PerTree& tr, const PushRange& pr, double beta, double u,
                                      int64_t& idx_out, float& wraw_out) {
    const int lane = threadIdx.x & 63;
    const int64_t nb = (size + PER_CHUNK - 1) / PER_CHUNK;
    // level 2: totals and the chunk
    double total, before = 0.0, t;
    int64_t blk = -1;
    if (nb <= 1024) {  // capacity <= 1M: one round trip, totals and search from the same registers
        double vals[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t c = (int64_t)lane * 16 + e;
            vals[e] = c < nb ? tr.chunk[c] : 0.0;
        }
        double part = 0.0;
#pragma unroll
        for (int e = 0; e < 16; ++e) part += vals[e];
        const double incl = wave_incl_scan(part, lane);
        total = __shfl(incl, 63);
        t = u * total;
        blk = chunk_find(vals, part, incl, 0.0, t, lane, before);
        PM_BLK(4);
    } else {
        total = 0.0;
        for (int64_t c0 = 0; c0 < nb; c0 += 1024) {
            double part = 0.0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t c = c0 + (int64_t)lane * 16 + e;
                part += c < nb ? tr.chunk[c] : 0.0;
            }
            total += wave_sum(part);
        }
        t = u * total;
        double run = 0.0;
        for (int64_t c0 = 0; c0 < nb && blk < 0; c0 += 1024) {
            double vals[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t c = c0 + (int64_t)lane * 16 + e;
                vals[e] = c < nb ? tr.chunk[c] : 0.0;
            }
            double part = 0.0;
#pragma unroll
            for (int e = 0; e < 16; ++e) part += vals[e];
            const double incl = wave_incl_scan(part, lane);
            const double tot = __shfl(incl, 63);
            if (run + tot > t) {
                double b;
                const int k = chunk_find(vals, part, incl, run, t, lane, b);
                if (k >= 0) { blk = c0 + k; before = b; }
            }
            run += tot;
        }
    }
    if (blk < 0) {  // u * total rounded up to the total: the last nonzero chunk (rare)
        for (int64_t c0 = ((nb - 1) / 64) * 64; c0 >= 0 && blk < 0; c0 -= 64) {
            const int64_t c = c0 + lane;
            const unsigned long long nz = __ballot(c < nb && tr.chunk[c] > 0.0);
            if (nz) blk = c0 + 63 - __clzll((long long)nz);
        }
        if (blk < 0) blk = 0;
        before = 0.0;
        for (int64_t c = 0; c < blk; ++c) before += tr.chunk[c];
    }
    // level 1: the chunk's 16 sub-block sums
    double b1, v1;
    const int64_t s0 = blk * PER_FAN;
    const double sv = (lane < PER_FAN && s0 + lane < tr.nsub) ? tr.sub[s0 + lane] : 0.0;
    const int64_t sb = s0 + lane_find(sv, t - before, lane, b1, v1);
    PM_BLK(5);
    // level 0: 64 leaves
    const int64_t e = sb * PER_SUB + lane;
    const double pv = e < size ? (double)per_leaf(tr.leaf, e, pr) : 0.0;
    double b0, pa;
    const int k = lane_find(pv, t - before - b1, lane, b0, pa);
    PM_BLK(6);
    idx_out = sb * PER_SUB + k;
    wraw_out = (float)pow((double)size * (pa / total), -beta);
#ifdef PM_DIAG
    asm volatile("" ::"v"(wraw_out));
#endif
    PM_BLK(7);
}

// Full rebuild over prios[0, cap): leaves, then level-1 and level-2 nodes with the pending push
// range substituted (from ctrl when non-null, else none).
int per_launch_build(const float* prios, int64_t cap, float alpha, const pm_ctrl* ctrl, int64_t n_push, void* work,
                     hipStream_t st);
int per_launch_update(float* prios, const int64_t* idx, const float* err, int bs, hipStream_t st);

}  // namespace pm
