// PER pieces shared between pm_replay.hip and pm_selfplay.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pongmi.h"
#include "pm_dev.h"

namespace pm {

constexpr int PER_CHUNK = 1024;  // priorities per level-1 block sum

// Replay fill seen by a kernel: a host value, or (selfplay) min(ctrl->size + n_push, cap) read on
// the device so a captured graph needs no host round trip.
struct PerSize {
    int64_t host;
    const pm_ctrl* ctrl;
    int64_t n_push;
    int64_t cap;
    __device__ __forceinline__ int64_t get() const {
        if (!ctrl) return host;
        const int64_t s = ctrl->size + n_push;
        return s < cap ? s : cap;
    }
};

inline int64_t per_work_bytes(int64_t cap) {
    const int64_t nb = (cap + PER_CHUNK - 1) / PER_CHUNK;
    return ((nb * 8 + 255) / 256) * 256;
}

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

// Values accessor for the two search levels.
struct BlockSums {
    const double* s;
    int64_t n;
    __device__ double operator()(int64_t k) const { return k < n ? s[k] : 0.0; }
};
struct PowPrios {
    const float* p;
    int64_t lo, hi;
    float alpha;
    __device__ double operator()(int64_t k) const {
        const int64_t e = lo + k;
        return e < hi ? (double)powf(p[e], alpha) : 0.0;
    }
};

// Within one loaded chunk (16 values per lane, `part` their sum, `incl` the wave's inclusive scan of
// parts, `run` the running sum in front of the chunk): the first element whose running sum exceeds
// t. Returns the in-chunk index (lane*16 + e) or -1; `before` / `val` get its prefix and value.
__device__ inline int chunk_find(const double (&vals)[16], double part, double incl, double run, double t, int lane,
                                 double& before, double& val) {
    const unsigned long long hit = __ballot(run + incl > t);
    if (!hit) return -1;
    const int L = __ffsll((long long)hit) - 1;
    // every lane resolves its own 16 values; lane L's answer is the one broadcast
    double base = run + (incl - part), bef = base, lastbef = base, v = 0.0, lastv = 0.0;
    int found = -1, lastnz = -1;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (found < 0 && base + vals[e] > t) { found = e; bef = base; v = vals[e]; }
        if (vals[e] > 0.0) { lastnz = e; lastbef = base; lastv = vals[e]; }
        base += vals[e];
    }
    if (found < 0) { found = lastnz; bef = lastbef; v = lastv; }  // rounding: lane sum fell short of its scan
    found = __shfl(found, L);
    before = __shfl(bef, L);
    val = __shfl(v, L);
    return found < 0 ? -1 : L * 16 + found;
}

// First k in [0, m) with (sum_{j<=k} v(j)) > t, scanning in chunks of 1024 (16 per lane). Each
// chunk's 16 values per lane are loaded together into registers before any compare, so a search
// costs one memory round trip per chunk. Returns -1 if none. Wave-uniform result.
template <class V>
__device__ inline int64_t wave_search(const V& v, int64_t m, double t, double& before, double& val, int lane) {
    double run = 0.0;
    for (int64_t c0 = 0; c0 < m; c0 += 1024) {
        const int64_t b = c0 + (int64_t)lane * 16;
        double vals[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) vals[e] = v(b + e);
        double part = 0.0;
#pragma unroll
        for (int e = 0; e < 16; ++e) part += vals[e];
        const double incl = wave_incl_scan(part, lane);
        const double tot = __shfl(incl, 63);
        if (run + tot > t) {  // wave-uniform
            const int k = chunk_find(vals, part, incl, run, t, lane, before, val);
            if (k >= 0) return c0 + k;
        }
        run += tot;
    }
    return -1;
}

// last k in [0, m) with v(k) > 0 (u*total rounding past the end)
template <class V>
__device__ inline int64_t wave_last_nonzero(const V& v, int64_t m, int lane) {
    for (int64_t c0 = ((m - 1) / 64) * 64; c0 >= 0; c0 -= 64) {
        const int64_t k = c0 + lane;
        const unsigned long long nz = __ballot(k < m && v(k) > 0.0);
        if (nz) return c0 + 63 - __clzll((long long)nz);
    }
    return 0;
}

// One wave per sample (called by the selfplay learner too). Writes idx and the un-normalised IS
// weight (size * P(i))^-beta. With <= 1024 block sums (capacity <= 1M) the totals, the block
// search and the element search take one load round trip each.
__device__ inline void per_sample_one(const float* __restrict__ prios, int64_t size, const double* __restrict__ bsum,
                                      float alpha, double beta, double u, int64_t& idx_out, float& wraw_out) {
    const int lane = threadIdx.x & 63;
    const int64_t nb = (size + PER_CHUNK - 1) / PER_CHUNK;
    BlockSums bs{bsum, nb};
    double total, t, before = 0.0, bval = 0.0;
    int64_t blk;
    if (nb <= 1024) {
        double vals[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) vals[e] = bs((int64_t)lane * 16 + e);
        double part = 0.0;
#pragma unroll
        for (int e = 0; e < 16; ++e) part += vals[e];
        const double incl = wave_incl_scan(part, lane);
        total = __shfl(incl, 63);
        t = u * total;
        blk = chunk_find(vals, part, incl, 0.0, t, lane, before, bval);
    } else {
        total = 0.0;
        for (int64_t c0 = 0; c0 < nb; c0 += 1024) {
            double part = 0.0;
            const int64_t b = c0 + (int64_t)lane * 16;
#pragma unroll
            for (int e = 0; e < 16; ++e) part += bs(b + e);
            total += wave_sum(part);
        }
        t = u * total;
        blk = wave_search(bs, nb, t, before, bval, lane);
    }
    if (blk < 0) { blk = wave_last_nonzero(bs, nb, lane); before = 0.0; }
    const int64_t lo = blk * PER_CHUNK, hi = min(lo + (int64_t)PER_CHUNK, size);
    PowPrios pp{prios, lo, hi, alpha};
    double before0 = 0.0, pa = 0.0;
    int64_t k = wave_search(pp, hi - lo, t - before, before0, pa, lane);
    if (k < 0) { k = wave_last_nonzero(pp, hi - lo, lane); pa = (double)powf(prios[lo + k], alpha); }
    idx_out = lo + k;
    wraw_out = (float)pow((double)size * (pa / total), -beta);
}

int per_launch_reduce(const float* prios, PerSize sz, int64_t cap, float alpha, double* bsum, hipStream_t st);
int per_launch_update(float* prios, const int64_t* idx, const float* err, int bs, hipStream_t st);

}  // namespace pm
