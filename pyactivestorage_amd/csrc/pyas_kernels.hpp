// pyas_kernels.hpp — gfx950 kernels of the chunk-reduction backend (templates).
// Instantiated once per dtype by pyas_inst.hip (one object per dtype, so the
// build runs in parallel); dispatched by dtype in pyas_kernels.hip.
//
// k_reduce        : the hot path.  One workgroup per (chunk, tile); streams the
//                   chunk's selected bytes from HBM with 16-B loads, undoes the
//                   HDF5 shuffle in registers (v_perm byte transposes), swaps
//                   byte order, applies the compiled mask and reduces to
//                   {sum, count, min, max}.  Replaces storage.py:51-100 per chunk.
// k_finish / k_combine : fixed-order combine of partials
//                   (active.py:575-598), no atomics => deterministic.
// k_reduce_axes   : partial-axis reduction (storage.py:98-100, axis ⊂ dims).
// k_select        : method=None path (storage.py:95-96, returns data + mask).
// (k_unshuffle, the standalone filter reversal, lives in pyas_kernels.hip.)
#pragma once
#include <hip/hip_runtime.h>

#include "pyas_device.hpp"
#include "pyas_internal.hpp"

namespace pyas {

// Debug progress marks (tools/dbg harnesses only: -DPYAS_DBG): each thread
// writes its last mark to host-mapped memory the host can poll while a
// kernel runs.  Empty in the library build.
#ifdef PYAS_DBG
__device__ int *pyas_dbg_mark;
#define PYAS_MARK(v)                                                                              \
    do {                                                                                          \
        if (pyas_dbg_mark)                                                                        \
            __hip_atomic_store(pyas_dbg_mark + blockIdx.x * kBlock + threadIdx.x, (int)(v),        \
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                      \
    } while (0)
#else
#define PYAS_MARK(v) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// vector un-shuffle: 16 consecutive elements from ES byte planes
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t word(const uint4 &v, int j) {
    return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
// a,b,c,d hold byte 0,1,2,3 of four consecutive elements; returns the four
// little-endian 32-bit words (8 v_perm_b32).
__device__ __forceinline__ void transpose4(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                           uint32_t e[4]) {
    const uint32_t t0 = perm(b, a, 0x05010400u), t1 = perm(b, a, 0x07030602u);
    const uint32_t u0 = perm(d, c, 0x05010400u), u1 = perm(d, c, 0x07030602u);
    e[0] = perm(u0, t0, 0x05040100u);
    e[1] = perm(u0, t0, 0x07060302u);
    e[2] = perm(u1, t1, 0x05040100u);
    e[3] = perm(u1, t1, 0x07060302u);
}

template <typename T, bool BSWAP>
__device__ __forceinline__ void unshuffle16(const uint4 *pl, T out[16]) {
    constexpr int ES = sizeof(T);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if constexpr (ES == 2) {
            const uint32_t a = word(pl[BSWAP ? 1 : 0], j), b = word(pl[BSWAP ? 0 : 1], j);
            const uint32_t w0 = perm(b, a, 0x05010400u), w1 = perm(b, a, 0x07030602u);
            out[4 * j + 0] = bits_to<T>((uint16_t)(w0 & 0xffffu));
            out[4 * j + 1] = bits_to<T>((uint16_t)(w0 >> 16));
            out[4 * j + 2] = bits_to<T>((uint16_t)(w1 & 0xffffu));
            out[4 * j + 3] = bits_to<T>((uint16_t)(w1 >> 16));
        } else if constexpr (ES == 4) {
            uint32_t e[4];
            if (BSWAP) transpose4(word(pl[3], j), word(pl[2], j), word(pl[1], j), word(pl[0], j), e);
            else transpose4(word(pl[0], j), word(pl[1], j), word(pl[2], j), word(pl[3], j), e);
#pragma unroll
            for (int k = 0; k < 4; ++k) out[4 * j + k] = bits_to<T>(e[k]);
        } else if constexpr (ES == 8) {
            uint32_t lo[4], hi[4];
            if (BSWAP) {
                transpose4(word(pl[7], j), word(pl[6], j), word(pl[5], j), word(pl[4], j), lo);
                transpose4(word(pl[3], j), word(pl[2], j), word(pl[1], j), word(pl[0], j), hi);
            } else {
                transpose4(word(pl[0], j), word(pl[1], j), word(pl[2], j), word(pl[3], j), lo);
                transpose4(word(pl[4], j), word(pl[5], j), word(pl[6], j), word(pl[7], j), hi);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                out[4 * j + k] = bits_to<T>(((uint64_t)hi[k] << 32) | (uint64_t)lo[k]);
        }
    }
}

// Streaming 16-B load; PYAS_NT=1 marks it non-temporal (read-once data).
#ifndef PYAS_UNROLL
#define PYAS_UNROLL 4
#endif
#ifndef PYAS_NT
#define PYAS_NT 1   // measured: +7 % (C2) / +5 % (C3) over default-policy loads
#endif
__device__ __forceinline__ uint4 ldg16(const uint4 *p) {
#if PYAS_NT
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(r.x, r.y, r.z, r.w);
#else
    return *p;
#endif
}

// A load through the constant address space: with a wave-uniform address the
// compiler issues s_load (counted by lgkmcnt), so waiting for it never waits
// for the wave's vector loads in flight.  For read-only tables only (chunk and output
// offsets: a vector load of one at a chunk boundary used to stall the column
// walks' ring of loads with vmcnt(0)).
template <typename V>
__device__ __forceinline__ V sload(const V *p) {
    return *(const __attribute__((address_space(4))) V *)p;
}

// Raw 16 bytes of the plain layout -> 16/ES values
template <typename T, bool BSWAP>
__device__ __forceinline__ void unpack16(const uint4 &r, T *x) {
    using U = typename TT<T>::U;
    constexpr int N = 16 / sizeof(T);
    U w[N];
    __builtin_memcpy(w, &r, 16);
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = bits_to<T>(BSWAP ? bswap(w[k]) : w[k]);
}

template <typename T, bool BSWAP, int MASKED, bool CONV>
__device__ __forceinline__ void consume16(const uint4 &r, TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    T x[N];
    unpack16<T, BSWAP>(r, x);
    acc.template add_n<N, MASKED, CONV>(x, mk);
}

// U vectors, one NaN ballot for all of them
template <typename T, bool BSWAP, int MASKED, bool CONV, int U>
__device__ __forceinline__ void consume16_u(const uint4 *r, TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        T x[N];
        unpack16<T, BSWAP>(r[u], x);
        bad |= acc.template add_lazy<N, MASKED, CONV>(x, mk);
    }
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            T x[N];
            unpack16<T, BSWAP>(r[u], x);
            acc.template check_nan<N>(x);
        }
    }
}

// ---------------------------------------------------------------------------
// contiguous runs
// ---------------------------------------------------------------------------
// Plain layout, memory elements [m0, m1) of the chunk at `base`.  The body is
// 16-B global loads, U per lane per step, register double-buffered so the
// next step's loads are in flight while the current step is reduced.
template <typename T, bool BSWAP, int MASKED>
__device__ void run_plain(const uint8_t *base, int64_t m0, int64_t m1, TileAcc<T> &acc,
                          const MaskT<T> &mk) {
    constexpr int ES = sizeof(T);
    const int tid = threadIdx.x;
    const int64_t b0 = m0 * ES, b1 = m1 * ES;               // byte range in the chunk
    const int64_t mis = (int64_t)((uintptr_t)base & 15);
    const int64_t a0 = ((b0 + mis + 15) & ~(int64_t)15) - mis;  // first 16-B aligned byte
    const int64_t a1 = ((b1 + mis) & ~(int64_t)15) - mis;
    if (a0 >= a1) {
        for (int64_t i = m0 + tid; i < m1; i += kBlock) {
            const T v = load_plain<T, BSWAP>(base, i);
            acc.template add_n<1, MASKED, false>(&v, mk);
        }
        if (!MASKED) {} // counts of unmasked tiles are added by the caller
        return;
    }
    const int64_t nhead = (a0 - b0) / ES, ntail = (b1 - a1) / ES;
    if (tid < nhead) {
        const T v = load_plain<T, BSWAP>(base, m0 + tid);
        acc.template add_n<1, MASKED, false>(&v, mk);
    }
    if (tid < ntail) {
        const T v = load_plain<T, BSWAP>(base, m1 - ntail + tid);
        acc.template add_n<1, MASKED, false>(&v, mk);
    }
    const uint4 *v = reinterpret_cast<const uint4 *>(base + a0);  // keeps global provenance
    const int64_t nvec = (a1 - a0) / 16;
    constexpr int U = PYAS_UNROLL;
    constexpr int64_t STEP = (int64_t)U * kBlock;
    const int64_t nsteps = nvec / STEP;
    if (nsteps > 0) {
        uint4 cur[U], nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = ldg16(v + tid + u * kBlock);
        for (int64_t s = 0; s + 1 < nsteps; ++s) {
            // the next step's loads are in flight while this step is reduced
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ldg16(v + (s + 1) * STEP + tid + u * kBlock);
            consume16_u<T, BSWAP, MASKED, true, U>(cur, acc, mk);
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
        consume16_u<T, BSWAP, MASKED, true, U>(cur, acc, mk);
    }
    for (int64_t k = nsteps * STEP + tid; k < nvec; k += kBlock)
        consume16<T, BSWAP, MASKED, false>(ldg16(v + k), acc, mk);
}

// Shuffled layout, chunk elements [i0, i1); n = elements in the chunk.
template <typename T, bool BSWAP, int MASKED>
__device__ void run_shuffled(const uint8_t *base, int64_t n, int64_t i0, int64_t i1,
                             TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int ES = sizeof(T);
    const int tid = threadIdx.x;
    const bool vec_ok = (((uintptr_t)base & 15) == 0) && ((n & 15) == 0);
    const int64_t g0 = (i0 + 15) & ~(int64_t)15, g1 = i1 & ~(int64_t)15;
    if (!vec_ok || g0 >= g1) {
        for (int64_t i = i0 + tid; i < i1; i += kBlock) {
            const T v = load_shuffled<T, BSWAP>(base, n, i);
            acc.template add_n<1, MASKED, false>(&v, mk);
        }
        return;
    }
    if (tid < g0 - i0) {
        const T v = load_shuffled<T, BSWAP>(base, n, i0 + tid);
        acc.template add_n<1, MASKED, false>(&v, mk);
    }
    if (tid < i1 - g1) {
        const T v = load_shuffled<T, BSWAP>(base, n, g1 + tid);
        acc.template add_n<1, MASKED, false>(&v, mk);
    }
    const int64_t ng = (g1 - g0) / 16;
    const int64_t nfull = ng / kBlock * kBlock;
    for (int64_t g = tid; g < ng; g += kBlock) {
        const int64_t i = g0 + g * 16;
        uint4 pl[ES];
#pragma unroll
        for (int b = 0; b < ES; ++b) pl[b] = ldg16(reinterpret_cast<const uint4 *>(base + (int64_t)b * n + i));
        T x[16];
        unshuffle16<T, BSWAP>(pl, x);
        if (g < nfull) acc.template add_n<16, MASKED, false>(x, mk);
        else acc.template add_n<16, MASKED, false>(x, mk);
    }
}

// ---------------------------------------------------------------------------
// generic (strided / listed / table-masked) selections
// ---------------------------------------------------------------------------
struct Decomp {
    int64_t mem;
    int64_t v[2];
};

// Decompose position e (row-major over the dims whose bit is in dmask) into
// chunk memory index and table indices.
__device__ __forceinline__ void decompose(const Sel &s, const int32_t *pool, const int64_t *cstride,
                                          const MaskTab &tab, int ndim, uint32_t dmask,
                                          int64_t e, Decomp &o) {
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < ndim && ((dmask >> d) & 1u)) {
            const int64_t cd = s.cnt[d];
            const int64_t q = e / cd, k = e - q * cd;
            e = q;
            o.mem += sel_index(s, pool, d, k) * cstride[d];
            o.v[0] += k * tab.stride[0][d];
            o.v[1] += k * tab.stride[1][d];
        }
    }
}

template <typename T>
__device__ __forceinline__ bool all_masked(const MaskT<T> &mk, const MaskTab &tab, const Decomp &o, T x) {
    bool m = mk.masked(x);
    if (tab.on[0]) m |= tab_masked<T>(tab, 0, o.v[0], x);
    if (tab.on[1]) m |= tab_masked<T>(tab, 1, o.v[1], x);
    return m;
}

// Mixed-radix position counter over the selected box (innermost dim
// fastest).  Divisions happen once per thread; every step of `stride`
// elements is then a carry-propagating add per dim (no division).
struct RadixCounter {
    uint32_t idx[PYAS_MAX_DIMS], inc[PYAS_MAX_DIMS], cnt[PYAS_MAX_DIMS];
    __device__ __forceinline__ void init(const Sel &s, int ndim, uint32_t dmask, uint64_t start,
                                         uint64_t stride) {
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            const bool on = d < ndim && ((dmask >> d) & 1u);
            const uint32_t c = on ? (uint32_t)s.cnt[d] : 1u;
            cnt[d] = c;
            idx[d] = (uint32_t)(start % c);
            start /= c;
            inc[d] = (uint32_t)(stride % c);
            stride /= c;
        }
    }
    __device__ __forceinline__ void advance() {
        uint32_t carry = 0;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            const uint32_t x = idx[d] + inc[d] + carry;
            carry = x >= cnt[d] ? 1u : 0u;
            idx[d] = carry ? x - cnt[d] : x;
        }
    }
    __device__ __forceinline__ void locate(const Sel &s, const int32_t *pool, const int64_t *cstride,
                                           const MaskTab &tab, int ndim, uint32_t dmask,
                                           Decomp &o) const {
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
            if (d < ndim && ((dmask >> d) & 1u)) {
                o.mem += sel_index(s, pool, d, idx[d]) * cstride[d];
                o.v[0] += (int64_t)idx[d] * tab.stride[0][d];
                o.v[1] += (int64_t)idx[d] * tab.stride[1][d];
            }
        }
    }
};

template <typename T, bool SHUF, bool BSWAP, int MASKED>
__device__ void run_generic(const ReduceArgs &a, const uint8_t *base, const Sel &s, int64_t e0,
                            int64_t e1, TileAcc<T> &acc, const MaskT<T> &mk) {
    const uint32_t all = (1u << a.ndim) - 1u;
    RadixCounter rc;
    rc.init(s, a.ndim, all, (uint64_t)(e0 + threadIdx.x), (uint64_t)kBlock);
    for (int64_t e = e0 + threadIdx.x; e < e1; e += kBlock) {
        Decomp o{0, {0, 0}};
        rc.locate(s, a.pool, a.cstride, a.tab, a.ndim, all, o);
        const T x = load_elem<T, SHUF, BSWAP>(base, a.chunk_elems, o.mem);
        acc.add_one(x, MASKED ? all_masked(mk, a.tab, o, x) : false);
        rc.advance();
    }
}

// Box-like selections whose innermost part is a contiguous run of L
// elements (dims > k full, dim k unit step): stream each run as 16-B vectors.
// Work items are (outer index of dims < k, vector within the run), walked by
// a radix counter, U independent 16-B loads in flight per lane.
template <typename T, bool BSWAP, int MASKED>
__device__ void run_rows(const ReduceArgs &a, const uint8_t *base, const Sel &s, int k, int64_t L,
                         int64_t e0, int64_t e1, TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    const int64_t V = L / N;                       // vectors per run
    const int64_t q0 = e0 / N, q1 = e1 / N;        // vector range of this tile
    // radix over (dims 0..k-1, vector) with the vector as the fastest digit
    Sel rs = s;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d == k) rs.cnt[d] = (int32_t)V;
        else if (d > k) rs.cnt[d] = 1;
    }
    const uint32_t dm = (2u << k) - 1u;            // dims 0..k
    int64_t inner0 = 0;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d == k) inner0 = (int64_t)s.start[d] * a.cstride[d];
    RadixCounter rc;
    rc.init(rs, a.ndim, dm, (uint64_t)(q0 + threadIdx.x), (uint64_t)kBlock);
    auto addr = [&](const RadixCounter &r) -> const uint4 * {
        int64_t mem = inner0;
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d)
            if (d < k) mem += sel_index(s, a.pool, d, r.idx[d]) * a.cstride[d];
        uint32_t v = 0;
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d)
            if (d == k) v = r.idx[d];
        return reinterpret_cast<const uint4 *>(base + (mem + (int64_t)v * N) * (int64_t)sizeof(T));
    };
    constexpr int U = 4;
    int64_t q = q0 + threadIdx.x;
    // converged part: every lane has U full items
    const int64_t nfull = ((q1 - q0) / (U * kBlock)) * (U * kBlock);
    for (int64_t it = 0; it < nfull; it += U * kBlock) {
        const uint4 *p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { p[u] = addr(rc); rc.advance(); }
        uint4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = ldg16(p[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) consume16<T, BSWAP, MASKED, true>(r[u], acc, mk);
        q += U * kBlock;
    }
    for (; q < q1; q += kBlock) {
        consume16<T, BSWAP, MASKED, false>(ldg16(addr(rc)), acc, mk);
        rc.advance();
    }
}

// run_rows for runs at any alignment and of any length (a hyperslab cutting
// an f32 row at element 1: [1:64] of a 64-element row).  Work items are
// (outer index, group j of N consecutive positions of the run); a group
// wholly inside the tile is one 16-B load at its element address (unaligned
// global loads are allowed), a short group (the run's last, or one cut by
// the tile's range [e0, e1)) reads its elements one by one.  The positions
// taken are exactly [e0, e1), so the caller's unmasked count holds.
template <typename T, bool BSWAP, int MASKED>
__device__ void run_rows_any(const ReduceArgs &a, const uint8_t *base, const Sel &s, int k, int64_t L,
                             int64_t e0, int64_t e1, TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    const int64_t Vr = (L + N - 1) / N;               // groups per run
    const int64_t r0 = e0 / L, r1 = (e1 + L - 1) / L;  // runs touching [e0, e1)
    const int64_t g0 = r0 * Vr, g1 = r1 * Vr;
    const int64_t cut0 = e0 - r0 * L, cut1 = e1 - (r1 - 1) * L;   // first run from, last run to
    Sel rs = s;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d == k) rs.cnt[d] = (int32_t)Vr;
        else if (d > k) rs.cnt[d] = 1;
    }
    const uint32_t dm = (2u << k) - 1u;               // dims 0..k
    int64_t inner0 = 0;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d == k) inner0 = (int64_t)s.start[d] * a.cstride[d];
    // the digits of item g (dims 0..k-1, then the group j at dim k) and its
    // run's memory offset, both stepped by kBlock items per iteration without
    // multiplies: ud[d] = the offset of one index of dim d (< k), incu/cntu
    // = ud times the digit's increment / count (32-bit: chunks < 2^31 elems)
    RadixCounter rc;
    rc.init(rs, a.ndim, dm, (uint64_t)(g0 + threadIdx.x), (uint64_t)kBlock);
    int32_t ud[PYAS_MAX_DIMS], incu[PYAS_MAX_DIMS], cntu[PYAS_MAX_DIMS];
    int64_t mem64 = inner0;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        ud[d] = d < k ? (int32_t)((int64_t)s.step[d] * a.cstride[d]) : 0;
        incu[d] = (int32_t)rc.inc[d] * ud[d];
        cntu[d] = (int32_t)rc.cnt[d] * ud[d];
        if (d < k) mem64 += sel_index(s, a.pool, d, rc.idx[d]) * a.cstride[d];
    }
    int32_t mem = (int32_t)mem64;
    // U items per lane per step: their 16-B loads are issued together (8
    // measured worse: 176 VGPRs cut k_reduce_u's occupancy, C3 [1:1023]^3
    // 1.37 -> 2.17 ms and C5 86.9 -> 70.5 %)
    constexpr int U = 4;
    for (int64_t g = g0 + threadIdx.x; g < g1; g += U * kBlock) {
        int32_t at[U], elo[U], ehi[U];
        bool full[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t gu = g + (int64_t)u * kBlock;
            int32_t j = 0;
#pragma unroll
            for (int d = 0; d < PYAS_MAX_DIMS; ++d)
                if (d == k) j = (int32_t)rc.idx[d];
            const int32_t lo = j * N, hi = lo + N < L ? lo + N : (int32_t)L;
            int32_t el = lo, eh = gu < g1 ? hi : lo;   // past the tile: nothing
            if (gu < g0 + Vr && cut0 > el) el = (int32_t)cut0;
            if (gu >= g1 - Vr && cut1 < eh) eh = (int32_t)cut1;
            if (eh < el) eh = el;
            at[u] = mem + lo;
            full[u] = eh - el == N;
            elo[u] = mem + el;
            ehi[u] = mem + eh;
            // next item: kBlock further (carry-propagating, offset kept in step)
            uint32_t carry = 0;
#pragma unroll
            for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
                const uint32_t x = rc.idx[d] + rc.inc[d] + carry;
                const uint32_t c2 = x >= rc.cnt[d] ? 1u : 0u;
                rc.idx[d] = c2 ? x - rc.cnt[d] : x;
                mem += incu[d] + (carry ? ud[d] : 0) - (c2 ? cntu[d] : 0);
                carry = c2;
            }
        }
        // every load of the step is issued before anything is consumed: a
        // short group (nearly every step has some: one per run) loads its
        // elements at clamped addresses beside the 16-B loads (a dependent
        // load per element made the step wait on each)
        uint4 r[U];
        T xs[U][N];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (full[u]) {
                __builtin_memcpy(&r[u], base + (int64_t)at[u] * (int64_t)sizeof(T), 16);
            } else if (ehi[u] > elo[u]) {
#pragma unroll
                for (int t = 0; t < N; ++t) {
                    const int32_t i = elo[u] + t < ehi[u] ? elo[u] + t : ehi[u] - 1;
                    xs[u][t] = load_plain<T, BSWAP>(base, i);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (full[u]) {
                consume16<T, BSWAP, MASKED, false>(r[u], acc, mk);
            } else {
#pragma unroll
                for (int t = 0; t < N; ++t)
                    if (elo[u] + t < ehi[u]) acc.template add_n<1, MASKED, false>(&xs[u][t], mk);
            }
        }
    }
}

// 16 bytes at any element-aligned address (AL: 16-B aligned -> one load)
template <bool AL>
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    if constexpr (AL) {
        return ldg16(reinterpret_cast<const uint4 *>(p));
    } else {
        uint4 r;
        __builtin_memcpy(&r, p, 16);
        return r;
    }
}

// One byte-plane piece of a shuffled vector: W bytes at q (AL: W-aligned)
#ifndef PYAS_PLANE_NT
#define PYAS_PLANE_NT 1   // plane pieces loaded non-temporal (0: plain loads, a tuning variant)
#endif
template <typename W, bool AL, bool NT = true>
__device__ __forceinline__ W ldp(const uint8_t *q) {
    if constexpr (AL && NT && PYAS_PLANE_NT) {
        return __builtin_nontemporal_load(reinterpret_cast<const W *>(q));
    } else if constexpr (AL) {
        return *reinterpret_cast<const W *>(q);
    } else {
        W r;
        __builtin_memcpy(&r, q, sizeof(W));
        return r;
    }
}

// 16 bytes = N = 16/ES consecutive elements of the plain layout, addressed
// by `p` in the plain layout of the chunk at `base` (n elements).  With SHUF
// the chunk is HDF5-shuffled (byte b of element e at b*n + e), so those
// elements are N consecutive bytes of each of the ES byte planes: ES loads
// of N bytes (f32: 4 dwords, 256 contiguous bytes per plane per wave),
// reassembled into the plain bytes with v_perm; the caller's unpack16 then
// applies the byte order as for plain chunks.  AL: see ldv_aligned.
// NT = false: plain loads for the plane pieces (the lean fold's walk over
// rows whose plane pieces share 128-B lines, measured faster there).
template <typename T, bool SHUF, bool AL, bool NT = true>
__device__ __forceinline__ uint4 ldv(const uint8_t *base, const uint8_t *p, int64_t n) {
    constexpr int ES = sizeof(T);
    if constexpr (!SHUF || ES == 1) {
        return ld16<AL>(p);
    } else {
        const uint8_t *q = base + ((uint64_t)(p - base) / ES);
        if constexpr (ES == 4) {          // 4 planes x 4 bytes
            uint32_t w[4], e[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) w[b] = ldp<uint32_t, AL, NT>(q + b * n);
            transpose4(w[0], w[1], w[2], w[3], e);
            return make_uint4(e[0], e[1], e[2], e[3]);
        } else if constexpr (ES == 2) {   // 2 planes x 8 bytes
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 a = ldp<u32x2, AL, NT>(q), b = ldp<u32x2, AL, NT>(q + n);
            return make_uint4(perm(b.x, a.x, 0x05010400u), perm(b.x, a.x, 0x07030602u),
                              perm(b.y, a.y, 0x05010400u), perm(b.y, a.y, 0x07030602u));
        } else {                          // 8 planes x 2 bytes
            uint32_t h[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) h[b] = ldp<uint16_t, AL, NT>(q + b * n);
            const uint32_t x01 = h[0] | (h[1] << 16), x23 = h[2] | (h[3] << 16);
            const uint32_t x45 = h[4] | (h[5] << 16), x67 = h[6] | (h[7] << 16);
            return make_uint4(perm(x23, x01, 0x06040200u), perm(x67, x45, 0x06040200u),
                              perm(x23, x01, 0x07050301u), perm(x67, x45, 0x07050301u));
        }
    }
}

// Whether ldv<T, SHUF, true> may be used on the chunk at `base` of n elements:
// plain: base 16-B aligned; shuffled: every plane piece W = 16/ES-aligned
// (vector offsets are multiples of N elements in every dense layout).
template <typename T, bool SHUF>
__device__ __forceinline__ bool ldv_aligned(const uint8_t *base, int64_t n) {
    constexpr int ES = sizeof(T), N = 16 / ES;
    if constexpr (!SHUF || ES == 1) return ((uintptr_t)base & 15) == 0;
    else return (((uintptr_t)base | (uint64_t)n) & (N - 1)) == 0;
}

// A load unit of the row layouts: VPL = (SHUF ? ES : 1) consecutive 16-B
// vectors of the plain layout.  Shuffled, that is 16 consecutive elements =
// one 16-B load from each of the ES byte planes (a wave reads 1 KiB of a
// plane per instruction when its lanes' units are adjacent), transposed
// into ES plain vectors with v_perm; the caller's unpack16 applies the byte
// order as for plain chunks.  AL: see ldu_aligned.
template <typename T, bool SHUF>
struct Unit {
    static constexpr int VPL = (SHUF && sizeof(T) > 1) ? (int)sizeof(T) : 1;
};

template <typename T, bool SHUF, bool AL>
__device__ __forceinline__ void ldu(const uint8_t *base, const uint8_t *p, int64_t n,
                                    uint4 v[Unit<T, SHUF>::VPL]) {
    constexpr int ES = sizeof(T);
    if constexpr (Unit<T, SHUF>::VPL == 1) {
        v[0] = ld16<AL>(p);
    } else {
        const uint8_t *q = base + ((uint64_t)(p - base) / ES);
        uint4 pl[ES];
#pragma unroll
        for (int b = 0; b < ES; ++b) pl[b] = ld16<AL>(q + b * n);
        if constexpr (ES == 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t e[4];
                transpose4(word(pl[0], j), word(pl[1], j), word(pl[2], j), word(pl[3], j), e);
                v[j] = make_uint4(e[0], e[1], e[2], e[3]);
            }
        } else if constexpr (ES == 2) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t a0 = word(pl[0], 2 * j), b0 = word(pl[1], 2 * j);
                const uint32_t a1 = word(pl[0], 2 * j + 1), b1 = word(pl[1], 2 * j + 1);
                v[j] = make_uint4(perm(b0, a0, 0x05010400u), perm(b0, a0, 0x07030602u),
                                  perm(b1, a1, 0x05010400u), perm(b1, a1, 0x07030602u));
            }
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t lo[4], hi[4];
                transpose4(word(pl[0], w), word(pl[1], w), word(pl[2], w), word(pl[3], w), lo);
                transpose4(word(pl[4], w), word(pl[5], w), word(pl[6], w), word(pl[7], w), hi);
                v[2 * w] = make_uint4(lo[0], hi[0], lo[1], hi[1]);
                v[2 * w + 1] = make_uint4(lo[2], hi[2], lo[3], hi[3]);
            }
        }
    }
}

// Whether ldu<T, SHUF, true> may be used on the chunk at `base` of n
// elements (unit offsets are multiples of 16 elements when shuffled).
template <typename T, bool SHUF>
__device__ __forceinline__ bool ldu_aligned(const uint8_t *base, int64_t n) {
    if constexpr (Unit<T, SHUF>::VPL == 1) return ((uintptr_t)base & 15) == 0;
    else return (((uintptr_t)base | (uint64_t)n) & 15) == 0;
}

// ---------------------------------------------------------------------------
// spans with a per-lane predicate (cut chunks of hyperslabs, strides, lists)
// ---------------------------------------------------------------------------
// A selection is read as spans: the dims < kk are enumerated (each selected
// index tuple is one span, any step or an index list), the dims >= kk are
// inside the span: a run of `ext` chunk elements starting `m_in` elements
// into the span's outer row, of which those at multiples of `istep` are
// selected (istep > 1 only for a strided innermost dim).  When every span
// starts at the same offset `off` from a 16-B boundary (16-element boundary
// when shuffled), a span is G aligned groups and a lane keeps ONE group
// position j for the whole tile: its in-span predicate (which of its group's
// elements are selected) is computed once, and every group is one aligned
// 16-B load (ES plane loads when shuffled) -- no element loads, no per-item
// bookkeeping beyond the span address.  The groups at either end of a span
// read a few unselected bytes of the same 16-B line; those never cross a
// page (a page boundary is 16-B aligned) and sit in 128-B lines the span's
// own bytes already fetch.
struct SpanPlan {
    int kk;              // dims < kk: enumerated; dims >= kk: inside a span
    int32_t m_in;        // memory offset of a span's first element in its outer row
    int32_t ext;         // memory extent of a span (elements)
    int32_t istep;       // in-span step (1, or the innermost dim's |step|)
    int32_t off;         // elements from the group boundary to a span's first element
    int32_t G, P;        // aligned groups per span; spans per block pass (P * G <= kBlock)
    int64_t nspans;      // spans in the chunk's selection
    int64_t per_span;    // selected elements per span
};

template <typename T, bool SHUF>
__device__ __forceinline__ bool span_plan(const ReduceArgs &a, const uint8_t *base, const Sel &s,
                                          SpanPlan &sp) {
    constexpr int ES = sizeof(T);
    constexpr bool SH = SHUF && ES > 1;
    constexpr int NU = SH ? 16 : 16 / ES;   // elements per aligned group
    if (a.tab.on[0] || a.tab.on[1] || a.chunk_elems >= (int64_t(1) << 31)) return false;
    if (SH && ((((uintptr_t)base) | (uint64_t)a.chunk_elems) & 15) != 0) return false;
    // innermost dim that is not whole
    int k = -1;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d)
        if (d < a.ndim && k < 0 &&
            !(s.step[d] == 1 && s.start[d] == 0 && (int64_t)s.cnt[d] == a.shape[d]))
            k = d;
    if (k < 0) return false;
    int64_t cs_k = 1, sk = 1, st_k = 0, cn_k = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d == k) { cs_k = a.cstride[d]; sk = s.step[d]; st_k = s.start[d]; cn_k = s.cnt[d]; }
    if (sk < 0) { st_k += (cn_k - 1) * sk; sk = -sk; }   // same elements, ascending
    // three span forms (written as selects: a branch-per-form version of this
    // lost the `ext` of the last form at -O1 and above, ROCm 7.2 hipcc)
    // a run of whole inner rows -- unless it would exceed one block pass
    // (> 4 KiB): then dim k is enumerated too and a span is one inner block
    // (C3 [:, 1:64, :]: 63 spans of 256 B, not one of 15.75 KiB)
    const bool run = sk == 1 && (cn_k * cs_k + NU - 1) / NU + 1 <= kBlock;
    const bool strided = !run && sk > 1 && k == a.ndim - 1;   // strided innermost dim
    // otherwise: a list, or strided with inner rows -> dim k enumerated too
    sp.kk = (run || strided) ? k : k + 1;
    const int64_t m_in = run ? st_k * cs_k : strided ? st_k : 0;
    const int64_t ext = run ? cn_k * cs_k : strided ? (cn_k - 1) * sk + 1 : cs_k;
    sp.m_in = (int32_t)m_in;
    sp.ext = (int32_t)ext;
    sp.istep = strided ? (int32_t)sk : 1;
    sp.per_span = run ? cn_k * cs_k : strided ? cn_k : cs_k;
    // every span must start at the same offset from a group boundary
    int64_t m0 = sp.m_in, nsp = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d < sp.kk) {
            nsp *= s.cnt[d];
            if (s.cnt[d] > 0) m0 += sel_index(s, a.pool, d, 0) * a.cstride[d];
            if (s.cnt[d] > 1) {
                // SpanWalk: an index list only as the last span dim
                if (s.step[d] == 0 && d < sp.kk - 1) return false;
                const int64_t delta = (s.step[d] != 0 ? (int64_t)s.step[d] : 1) * a.cstride[d];
                if (SH ? (delta & 15) != 0 : ((delta * ES) & 15) != 0) return false;
            }
        }
    }
    sp.nspans = nsp;
    sp.off = SH ? (int32_t)(m0 & 15) : (int32_t)((((uintptr_t)base + (uint64_t)(m0 * ES)) & 15) / ES);
    const int64_t G = (sp.off + (int64_t)sp.ext + NU - 1) / NU;
    if (G < 1 || G > kBlock) return false;
    sp.G = (int32_t)G;
    sp.P = (int32_t)(kBlock / G);
    return true;
}

// The spans of one lane group, walked in order, for span dims that are all
// slices (any step): the digits of the current span and its first group's
// element offset.  The next span adds the last span dim's memory step; only
// a carry out of that dim (every cnt[kk-1] spans) walks the outer digits.
// (A block-strided walk advanced every digit with a carry chain per item:
// ~40 VALU ops per 16-B group, C3 [1:1023]^3's cut chunks at 39 % of 8 TB/s.)
constexpr int kSpanPool = 512;   // index-list entries run_spans copies to LDS
struct SpanWalk {
    int32_t ix[PYAS_MAX_DIMS];   // digits of the dims < last
    int32_t xl;                  // digit of the last span dim
    int32_t mem;                 // element offset of this lane's group in the current span
    // lp: the last span dim's index list (its first entry at lp[0]; an LDS
    // copy, run_spans), unused when that dim is a slice
    __device__ __forceinline__ void init(const ReduceArgs &a, const Sel &s, int kk, int64_t q, int32_t gofs,
                                         const int32_t *lp) {
        uint32_t r = (uint32_t)q;
        int32_t m = gofs;
        xl = 0;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            ix[d] = 0;
            if (d < kk) {
                const uint32_t c = (uint32_t)s.cnt[d], qq = r / c;
                const int32_t dig = (int32_t)(r - qq * c);
                r = qq;
                const int32_t idx = (d == kk - 1 && s.step[d] == 0) ? lp[dig] : (int32_t)sel_index(s, a.pool, d, dig);
                m += idx * (int32_t)a.cstride[d];
                if (d == kk - 1) xl = dig;
                else ix[d] = dig;
            }
        }
        mem = m;
    }
    // one more span along the last span dim; an index list there costs an
    // LDS read per span
    __device__ __forceinline__ void next(const ReduceArgs &a, const Sel &s, int kk, const int32_t *lp) {
        int32_t cl = 1, sk = 0, cs = 0;
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d)
            if (d == kk - 1) { cl = s.cnt[d]; sk = s.step[d]; cs = (int32_t)a.cstride[d]; }
        const int32_t x0 = xl;
        if (__builtin_expect(++xl < cl, 1)) {
            mem += sk != 0 ? sk * cs : (lp[xl] - lp[x0]) * cs;
            return;
        }
        // carry into the outer span dims (rare; slices or single indices,
        // span_plan's rule: affine in the digits)
        xl = 0;
        mem -= sk != 0 ? x0 * sk * cs : (lp[x0] - lp[0]) * cs;
        bool carry = true;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            if (carry && d < kk - 1) {
                const int32_t dd = s.step[d] * (int32_t)a.cstride[d];
                mem += dd;
                if (++ix[d] >= s.cnt[d]) {
                    ix[d] = 0;
                    mem -= s.cnt[d] * dd;
                } else {
                    carry = false;
                }
            }
        }
    }
};

// Spans [q0, q1) of the chunk at `base` (plan sp).  Lane group p (P of
// them, G lanes each) walks the spans [q0 + p*M, q0 + (p+1)*M) in order, lane
// j of a group reading group j of each span; U groups per lane in flight.
// Counts: masked tiles count through ballots, unmasked ones are counted by
// the caller ((q1 - q0) * per_span).
template <typename T, bool SHUF, bool BSWAP, int MASKED>
__device__ void run_spans(const ReduceArgs &a, const uint8_t *base, const Sel &s, const SpanPlan &sp,
                          int64_t q0, int64_t q1, TileAcc<T> &acc, const MaskT<T> &mk) {
    constexpr int ES = sizeof(T);
    constexpr bool SH = SHUF && ES > 1;
    constexpr int N = 16 / ES;                // elements per plain 16-B vector
    constexpr int VPL = SH ? ES : 1;          // plain vectors per group
    constexpr int NU = N * VPL;               // elements per group
    const int tid = threadIdx.x;
    const int p = tid / sp.G, j = tid - p * sp.G;
    uint32_t bits = 0;                        // this lane's selected group elements
    if (p < sp.P) {
#pragma unroll
        for (int t = 0; t < NU; ++t) {
            const int32_t x = j * NU - sp.off + t;
            if (x >= 0 && x < sp.ext && x % sp.istep == 0) bits |= 1u << t;
        }
    }
    const int64_t M = (q1 - q0 + sp.P - 1) / sp.P;   // spans per lane group
    const int64_t qa = q0 + (int64_t)p * M;
    const int64_t qb = qa + M < q1 ? qa + M : q1;
    const int kk = sp.kk;
    // an index list as the last span dim: its entries copied to LDS once,
    // so a span's address never waits on a global pool read (C3 [:, list64,
    // :] walked 256 spans per chunk, two dependent global reads each: 20 %)
    __shared__ int32_t spool[kSpanPool];
    const int32_t *lp = spool;
    {
        int32_t lst = 0, lsk = 1, lcnt = 0;
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d)
            if (d == kk - 1) { lst = s.start[d]; lsk = s.step[d]; lcnt = s.cnt[d]; }
        if (lsk == 0) {   // block-uniform
            if (lcnt <= kSpanPool) {
                __syncthreads();   // a previous tile's walk may still read it
                for (int i = tid; i < lcnt; i += kBlock) spool[i] = a.pool[lst + i];
                __syncthreads();
            } else {
                lp = a.pool + lst;
            }
        }
    }
    SpanWalk w;
    // span-independent part of a group's address (elements; may be -off < 0)
    w.init(a, s, kk, qa < q1 ? qa : q0, j * NU - sp.off + sp.m_in, lp);
    // groups in flight per lane: 4, or 8 plain vectors' worth when shuffled
    // (f64: one group = 8 vectors; 4 of them took k_reduce_u to ~300 VGPRs)
#ifndef PYAS_SPANS_U
#define PYAS_SPANS_U 2   // plain groups in flight per lane (4 took k_reduce_u f32 to 248 VGPRs + scratch)
#endif
    constexpr int U = VPL == 1 ? PYAS_SPANS_U : (8 / VPL > 0 ? 8 / VPL : 1);
    int64_t q = qa;
    for (int64_t it = 0; it < M; it += U) {   // uniform trip count
        uint4 r[U][VPL];
        bool on[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            on[u] = bits != 0 && q < qb;
#pragma unroll
            for (int v = 0; v < VPL; ++v) r[u][v] = make_uint4(0u, 0u, 0u, 0u);
            if (on[u]) {
                if constexpr (SH) {
                    ldu<T, true, true>(base, base + (int64_t)w.mem * ES, a.chunk_elems, r[u]);
                } else {
                    r[u][0] = ldg16(reinterpret_cast<const uint4 *>(base + (int64_t)w.mem * ES));
                }
                if (q + 1 < qb) w.next(a, s, kk, lp);
            }
            ++q;
        }
        bool bad = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t b = on[u] ? bits : 0u;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                T x[N];
                unpack16<T, BSWAP>(r[u][v], x);
                bad |= acc.template add_pred<N, MASKED>(x, b >> (v * N), mk);
            }
        }
        if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t b = on[u] ? bits : 0u;
#pragma unroll
                for (int v = 0; v < VPL; ++v) {
                    T x[N];
                    unpack16<T, BSWAP>(r[u][v], x);
#pragma unroll
                    for (int t = 0; t < N; ++t)
                        if ((b >> (v * N + t)) & 1u) acc.template check_nan<1>(&x[t]);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// combines (fixed order)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ typename TT<T>::Acc sum_of(const pyas_scalar &s, bool round) {
    using A = typename TT<T>::Acc;
    if constexpr (TT<T>::kind == 0) return round ? (A)(T)s.f : (A)s.f;
    else if constexpr (TT<T>::kind == 1) return round ? (A)(T)s.i : (A)s.i;
    else return round ? (A)(T)s.u : (A)s.u;
}

template <typename T>
__device__ __forceinline__ void merge(WAcc<T> &acc, const pyas_partial &p, bool round) {
    acc.sum += sum_of<T>(p.sum, round);
    if (p.count > 0) {
        acc.count += p.count;
        acc.mn = pmin(acc.mn, TT<T>::from(p.min));
        acc.mx = pmax(acc.mx, TT<T>::from(p.max));
    }
}

// ---------------------------------------------------------------------------
// compact per-output records (pyas.h PYAS_REC_*): one method's value in the
// variable dtype (the sum rounded as sum_of(round) rounds it) + int32 count
// ---------------------------------------------------------------------------
template <typename T> struct Rec {
    static constexpr int kBytes = sizeof(T) <= 4 ? 8 : 16;
};

template <typename T>
__device__ __forceinline__ int64_t out_bytes(int rec) {
    return rec ? (int64_t)Rec<T>::kBytes : (int64_t)sizeof(pyas_partial);
}

// p as record `rec` (the first Rec<T>::kBytes bytes of the result)
template <typename T>
__device__ __forceinline__ uint4 rec_of(const pyas_partial &p, int rec) {
    // every field converted, then values selected: a field picked by a
    // runtime index would put p in scratch memory
    const T vs = (T)sum_of<T>(p.sum, true), vmin = TT<T>::from(p.min), vmax = TT<T>::from(p.max);
    const T v = rec == PYAS_REC_SUM ? vs : rec == PYAS_REC_MIN ? vmin : vmax;
    uint4 r = {0u, 0u, 0u, 0u};
    if constexpr (sizeof(T) <= 4) {
        __builtin_memcpy(&r.x, &v, sizeof(T));
        r.y = (uint32_t)p.count;
    } else {
        __builtin_memcpy(&r.x, &v, 8);
        r.z = (uint32_t)p.count;
    }
    return r;
}

// A <= 4-byte type's record (value word, count word) as a pyas_partial.
template <typename T>
__device__ __forceinline__ pyas_partial part_raw(uint2 r, int rec) {
    static_assert(sizeof(T) <= 4, "8-byte records are 16 B");
    pyas_partial p;
    T v;
    __builtin_memcpy(&v, &r.x, sizeof(T));
    p.count = (int64_t)(int32_t)r.y;
    pyas_scalar sv, mv;
    if constexpr (TT<T>::kind == 0) sv.f = (double)v;
    else if constexpr (TT<T>::kind == 1) sv.i = (int64_t)v;
    else sv.u = (uint64_t)v;
    TT<T>::put(mv, v);
    p.sum.u = rec == PYAS_REC_SUM ? sv.u : 0u;
    p.min.u = rec == PYAS_REC_MIN ? mv.u : 0u;
    p.max.u = rec == PYAS_REC_MAX ? mv.u : 0u;
    return p;
}

// Entry i of a partial array of form `rec` as a pyas_partial (the fields a
// record does not carry are 0: neutral for the method that reads it).
template <typename T>
__device__ __forceinline__ pyas_partial part_at(const void *base, int64_t i, int rec) {
    if (rec == 0) return reinterpret_cast<const pyas_partial *>(base)[i];
    if constexpr (sizeof(T) <= 4) {
        return part_raw<T>(reinterpret_cast<const uint2 *>(base)[i], rec);
    } else {
        pyas_partial p;
        T v;
        const uint4 r = reinterpret_cast<const uint4 *>(base)[i];
        __builtin_memcpy(&v, &r.x, 8);
        p.count = (int64_t)(int32_t)r.z;
        pyas_scalar sv, mv;
        if constexpr (TT<T>::kind == 0) sv.f = (double)v;
        else if constexpr (TT<T>::kind == 1) sv.i = (int64_t)v;
        else sv.u = (uint64_t)v;
        TT<T>::put(mv, v);
        p.sum.u = rec == PYAS_REC_SUM ? sv.u : 0u;
        p.min.u = rec == PYAS_REC_MIN ? mv.u : 0u;
        p.max.u = rec == PYAS_REC_MAX ? mv.u : 0u;
        return p;
    }
}

// Output o of the per-chunk partial-axis kernels in the caller's form
template <typename T>
__device__ __forceinline__ void put_out(const AxesArgs &a, int64_t o, const pyas_partial &p) {
    if (a.rec == 0) {
        a.out[o] = p;
        return;
    }
    const uint4 r = rec_of<T>(p, a.rec);
    uint8_t *dst = reinterpret_cast<uint8_t *>(a.out) + o * Rec<T>::kBytes;
    if constexpr (Rec<T>::kBytes == 8) *reinterpret_cast<uint2 *>(dst) = make_uint2(r.x, r.y);
    else *reinterpret_cast<uint4 *>(dst) = r;
}

// Staged writes of a tile's outputs: slot k of the LDS stage (uint4 array)
// holds output k in the caller's form; stage_flush copies n of them to
// outputs o0.. as consecutive non-temporal stores (16-B pieces where the
// destination allows, else 8-B records).
template <typename T>
__device__ __forceinline__ void stage_put(const AxesArgs &a, uint4 *stage, int k, const pyas_partial &p) {
    if (a.rec == 0) {   // the 32-byte partial as two 16-B words, from its fields
        stage[k * 2] = make_uint4((uint32_t)p.sum.u, (uint32_t)(p.sum.u >> 32), (uint32_t)(uint64_t)p.count,
                                  (uint32_t)((uint64_t)p.count >> 32));
        stage[k * 2 + 1] = make_uint4((uint32_t)p.min.u, (uint32_t)(p.min.u >> 32), (uint32_t)p.max.u,
                                      (uint32_t)(p.max.u >> 32));
    } else if constexpr (Rec<T>::kBytes == 16) {
        stage[k] = rec_of<T>(p, a.rec);
    } else {
        const uint4 r = rec_of<T>(p, a.rec);
        reinterpret_cast<uint2 *>(stage)[k] = make_uint2(r.x, r.y);
    }
}

template <typename T>
__device__ __forceinline__ void stage_flush(const AxesArgs &a, const uint4 *stage, int64_t o0, int64_t n,
                                            int tid, int nthr) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int64_t rb = out_bytes<T>(a.rec);
    uint8_t *dst = reinterpret_cast<uint8_t *>(a.out) + o0 * rb;
    if (rb == 8 && ((o0 & 1) || (n & 1))) {      // odd record boundaries: 8-B pieces
        const uint2 *s2 = reinterpret_cast<const uint2 *>(stage);
        u32x2 *d2 = reinterpret_cast<u32x2 *>(dst);
        for (int64_t q = tid; q < n; q += nthr) {
            const uint2 h = s2[q];
            u32x2 v = {h.x, h.y};
            __builtin_nontemporal_store(v, d2 + q);
        }
        return;
    }
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
    const int64_t nq = n * rb / 16;
    for (int64_t q = tid; q < nq; q += nthr) {
        const uint4 h = stage[q];
        u32x4 v = {h.x, h.y, h.z, h.w};
        __builtin_nontemporal_store(v, d4 + q);
    }
}

// n partials -> one per block (contiguous segments), fixed order
template <typename T>
__global__ __launch_bounds__(kBlock) void k_combine(const pyas_partial *in, int64_t n, int64_t seg,
                                                    uint32_t flags, pyas_partial *out) {
    const int64_t lo = (int64_t)blockIdx.x * seg;
    const int64_t hi = lo + seg < n ? lo + seg : n;
    const bool round = (flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    WAcc<T> acc;
    acc.init();
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) merge(acc, in[i], round);
    block_reduce_w(acc);
    if (threadIdx.x == 0) store_wpartial(out + blockIdx.x, acc);
}

// ---------------------------------------------------------------------------
// k_finish: tiles -> chunks -> groups -> total in ONE launch
// ---------------------------------------------------------------------------
// Block g owns chunks [g*kCombineSeg, ...), one thread per chunk:
//   chunk partial = sequential fold of the chunk's tiles in tile order
//                   (written to chunk_out when requested);
//   group partial = k_combine's fixed order over the block's chunks, with the
//                   chunk sums rounded to the variable dtype if asked
//                   (active.py:512,585 store partials into `out` of that dtype).
// The total is the fold of the group partials in group order, done by the
// block that arrives last on a device-scope counter (cnt != NULL; the counter
// is left at zero again), or by a separate k_combine launch (cnt == NULL).
// Only one arrival per BLOCK of this small kernel: the hot kernel's
// 16k workgroups never wait on each other (an arrival per reduce workgroup
// costs ~3 us of store/atomic latency each and was measured 6 % slower).
// Hand-off (HIP's scoped C++ memory model, LLVM AMDGPU memory model for
// gfx950): each block stores its group partial, then increments the counter
// with an agent-scope acq_rel fetch_add.  Its release half orders the
// partial's stores before the increment; the increments form one release
// sequence, so the block whose fetch_add returns ng-1 acquires every earlier
// block's partial.  That block's thread 0 publishes the fact through LDS and
// a workgroup barrier, and every thread then issues its own agent-scope
// acquire fence before reading the partials.  (One release per finish
// block, ng = n_chunks/256 of them, not per reduce workgroup: the L2
// write-back a gfx950 agent release costs is paid 16 times for C3.)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_finish(FinishArgs f) {
    const int64_t lo = (int64_t)blockIdx.x * kCombineSeg;
    const int64_t hi = lo + kCombineSeg < f.n_chunks ? lo + kCombineSeg : f.n_chunks;
    const bool round = (f.flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    WAcc<T> acc;
    acc.init();
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
        pyas_partial cp;
        if (f.tpc == 1) {
            cp = f.tiles[i];
        } else {
            WAcc<T> ch;
            ch.init();
            for (int64_t t = 0; t < f.tpc; ++t) merge(ch, f.tiles[i * f.tpc + t], false);
            TT<T>::put_acc(cp.sum, ch.sum);
            cp.count = (int64_t)ch.count;
            TT<T>::put(cp.min, ch.mn);
            TT<T>::put(cp.max, ch.mx);
        }
        if (f.chunk_out) f.chunk_out[i] = cp;
        merge(acc, cp, round);
    }
    if (!f.total) return;
    block_reduce_w(acc);
    const int64_t ng = (f.n_chunks + kCombineSeg - 1) / kCombineSeg;
    if (ng == 1 && f.cnt) {
        if (threadIdx.x == 0) store_wpartial(f.total, acc);
        return;
    }
    __shared__ uint32_t s_last;
    if (threadIdx.x == 0) {
        store_wpartial_agent(f.gtmp + blockIdx.x, acc);
        bool last = false;
        if (f.cnt) {
            const uint32_t old = __hip_atomic_fetch_add(f.cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = old == (uint32_t)ng - 1u;
            if (last) __hip_atomic_store(f.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    WAcc<T> tot;   // = k_combine over the group partials (already rounded)
    tot.init();
    for (int64_t i = threadIdx.x; i < ng; i += kBlock) merge(tot, load_partial_agent(f.gtmp + i), false);
    block_reduce_w(tot);
    if (threadIdx.x == 0) store_wpartial(f.total, tot);
}

// Is the selection one contiguous run of chunk memory?  (innermost non-full
// dim has unit step; every dim outside it picks one index; no mask tables)
// *m0 = the memory index of its first element.
__device__ __forceinline__ bool sel_contiguous(const ReduceArgs &a, const Sel &s, int64_t *m0) {
    bool contig = !(a.tab.on[0] || a.tab.on[1]);
    bool seen_partial = false;
    int64_t m = 0;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < a.ndim) {
            const bool full = s.step[d] == 1 && s.start[d] == 0 && (int64_t)s.cnt[d] == a.shape[d];
            if (seen_partial) {
                if (s.cnt[d] > 1) contig = false;
            } else if (!full) {
                seen_partial = true;
                if (s.cnt[d] > 1 && s.step[d] != 1) contig = false;
            }
            if (s.cnt[d] > 0) m += sel_index(s, a.pool, d, 0) * a.cstride[d];
        }
    }
    *m0 = m;
    return contig;
}

// Rows of 16-B vectors (run_rows)?  No shuffle or tables, unit-step
// innermost partial dim *k, every run (*L elements) 16-B aligned.
template <typename T, bool SHUF>
__device__ __forceinline__ bool rows_aligned(const ReduceArgs &a, const uint8_t *base, const Sel &s,
                                             int *kp, int64_t *Lp) {
    constexpr int64_t ES = sizeof(T);
    int k = -1;
    int64_t L = 1;
    bool rows = !SHUF && !(a.tab.on[0] || a.tab.on[1]) && ((uintptr_t)base & 15) == 0;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < a.ndim) {
            if (k < 0) {
                const bool full = s.step[d] == 1 && s.start[d] == 0 && (int64_t)s.cnt[d] == a.shape[d];
                if (!full) {
                    k = d;
                    if (s.step[d] != 1) rows = false;
                    if (((int64_t)s.start[d] * a.cstride[d] * ES) % 16 != 0) rows = false;
                    L *= s.cnt[d];
                } else {
                    L *= a.shape[d];
                }
            } else if ((a.cstride[d] * ES) % 16 != 0) {
                rows = false;  // an outer dim whose rows start unaligned
            }
        }
    }
    if (k < 0 || (L * ES) % 16 != 0) rows = false;
    *kp = k;
    *Lp = L;
    return rows;
}

// The predicate stream (run_spans) for cut chunks; ReduceArgs::spans picks
// where it runs at run time (1: not on chunks whose aligned runs run_rows
// streams); PYAS_SPANS=0 builds it out.
#ifndef PYAS_SPANS
#define PYAS_SPANS 1
#endif

// ---------------------------------------------------------------------------
// the hot kernel
// ---------------------------------------------------------------------------
// SEL = false: every chunk fully selected (batch.sel == NULL) -> a lean
// streaming-only kernel (no selection state, high occupancy).
template <typename T, bool SHUF, bool BSWAP, int MASKED, bool SEL>
__device__ __forceinline__ void reduce_body(const ReduceArgs &a) {
    const int64_t b = blockIdx.x;
    const int64_t c = b / a.tpc;
    const int64_t t = b - c * a.tpc;
    pyas_partial *const tout = a.out + b;
    const uint8_t *base = a.data + a.offsets[c];
    MaskT<T> mk;
    if constexpr (MASKED) mk.init(a.mask);
    TileAcc<T> acc;
    acc.init();
    if constexpr (!SEL) {
        int64_t per = (a.chunk_elems + a.tpc - 1) / a.tpc;
        per = (per + 63) & ~(int64_t)63;
        const int64_t e0 = t * per, e1 = e0 + per < a.chunk_elems ? e0 + per : a.chunk_elems;
        if (e0 < e1) {
            if constexpr (SHUF && sizeof(T) > 1)
                run_shuffled<T, BSWAP, MASKED>(base, a.chunk_elems, e0, e1, acc, mk);
            else
                run_plain<T, BSWAP, MASKED>(base, e0, e1, acc, mk);
        }
        tile_finish(acc, (!MASKED && e0 < e1) ? (uint64_t)(e1 - e0) : 0u, tout);
        return;
    }
    Sel s;
    load_sel(s, a.sel, c, a.ndim, a.shape);
    int64_t total = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) total *= (int64_t)s.cnt[d];
#if PYAS_SPANS
    // cut chunks whose spans fit one block pass: the predicate stream,
    // tiled by whole spans (unless the selection is one contiguous run,
    // which run_plain / run_shuffled stream at the whole-chunk rate)
    int64_t m0s = 0;
    int ks = -1;
    int64_t Ls = 1;
    if (a.spans && total > 0 && !sel_contiguous(a, s, &m0s)) {
        SpanPlan sp;
        if (span_plan<T, SHUF>(a, base, s, sp) && (a.spans == 2 || !rows_aligned<T, SHUF>(a, base, s, &ks, &Ls))) {
            // (tiles sized by the bytes the spans read instead -- fewer, longer
            // lane-group walks -- measured slower: C3 [:, list64, :] 21 -> 12 %,
            // [:, 0:1024:3, :] 61 -> 41 % of 8 TB/s; the walk is latency-bound)
            const int64_t per = (sp.nspans + a.tpc - 1) / a.tpc;
            const int64_t q0 = t * per < sp.nspans ? t * per : sp.nspans;
            const int64_t q1 = q0 + per < sp.nspans ? q0 + per : sp.nspans;
            if (q0 < q1) run_spans<T, SHUF, BSWAP, MASKED>(a, base, s, sp, q0, q1, acc, mk);
            tile_finish(acc, (!MASKED && q0 < q1) ? (uint64_t)((q1 - q0) * sp.per_span) : 0u, tout);
            return;
        }
    }
#endif
    int64_t per = (total + a.tpc - 1) / a.tpc;
    per = (per + 63) & ~(int64_t)63;
    const int64_t e0 = t * per, e1 = e0 + per < total ? e0 + per : total;
    bool generic = false;
    if (e0 < e1) {
        int64_t m0 = 0;
        if (sel_contiguous(a, s, &m0)) {
            if constexpr (SHUF && sizeof(T) > 1)
                run_shuffled<T, BSWAP, MASKED>(base, a.chunk_elems, m0 + e0, m0 + e1, acc, mk);
            else
                run_plain<T, BSWAP, MASKED>(base, m0 + e0, m0 + e1, acc, mk);
        } else {
            int k = -1;
            int64_t L = 1;
            const bool rows = rows_aligned<T, SHUF>(a, base, s, &k, &L);
            // any unit-step innermost partial dim, no shuffle or tables: runs
            // of L contiguous elements at any alignment (run_rows_any)
            bool runs = !SHUF && !(a.tab.on[0] || a.tab.on[1]) && k >= 0 && a.chunk_elems < (int64_t(1) << 31);
#pragma unroll
            for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
                if (d == k && s.step[d] != 1) runs = false;
                if (d < k && s.step[d] == 0) runs = false;   // an index list: the generic walk
            }
            // (aligned rows stay on run_rows: through run_rows_any they measured
            // slower, C3 [4:1020]^3 0.96 -> 1.08 ms and C5 86.9 -> 66.7 %)
            if (rows) {
                run_rows<T, BSWAP, MASKED>(a, base, s, k, L, e0, e1, acc, mk);
            } else if (runs) {
                run_rows_any<T, BSWAP, MASKED>(a, base, s, k, L, e0, e1, acc, mk);
            } else {
                generic = true;
                run_generic<T, SHUF, BSWAP, MASKED>(a, base, s, e0, e1, acc, mk);
            }
        }
    }
    // unmasked contiguous tiles count every element; the generic path counts itself
    const uint64_t extra = (!MASKED && !generic && e0 < e1) ? (uint64_t)(e1 - e0) : 0u;
    tile_finish(acc, extra, tout);
}

// Every chunk whole (batch.sel == NULL), 4-/8-byte dtypes: the lean
// streaming kernel.  Its registers are capped for >= PYAS_WAVES waves per SIMD (measured on C3,
// masked f32: 83 -> 60 VGPRs, 5 -> 8 waves, 0.698 -> 0.635 ms, no spills).
#ifndef PYAS_WAVES
#define PYAS_WAVES 8
#endif
#if PYAS_WAVES
#define PYAS_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(PYAS_WAVES, 8)))
#else
#define PYAS_WAVES_ATTR
#endif
template <typename T, bool SHUF, bool BSWAP, int MASKED>
__global__ __launch_bounds__(kBlock) PYAS_WAVES_ATTR void k_reduce(ReduceArgs a) {
    reduce_body<T, SHUF, BSWAP, MASKED, false>(a);
}

// Uncapped: per-chunk selections (hyperslabs, strides, lists), where the cap
// spills (C5 measured 46 % slower), and 1-/2-byte dtypes (16 or 8 values per
// 16-B load also spill under the cap).  Keeps the compiler's allocation.
template <typename T, bool SHUF, bool BSWAP, int MASKED, bool SEL>
__global__ __launch_bounds__(kBlock) void k_reduce_u(ReduceArgs a) {
    reduce_body<T, SHUF, BSWAP, MASKED, SEL>(a);
}

// LDS writes of a wave visible to its other lanes (no block barrier)
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// segmented combine: one thread per output segment, sequential fixed order
template <typename T>
__global__ __launch_bounds__(kBlock) void k_combine_segments(const pyas_partial *in, const int64_t *index,
                                                             const int64_t *seg, int64_t n_seg,
                                                             uint32_t flags, pyas_partial *out) {
    const int64_t sidx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (sidx >= n_seg) return;
    const bool round = (flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    WAcc<T> acc;
    acc.init();
    const int rec = (int)((flags >> 4) & 3u);   // PYAS_COMBINE_REC
    for (int64_t k = seg[sidx]; k < seg[sidx + 1]; ++k) merge(acc, part_at<T>(in, index[k], rec), round);
    store_wpartial(out + sidx, acc);
}

// NumPy's zero sign (defined with the tie passes below; key layout there)
constexpr uint64_t kTieWNone = ~0ull;
constexpr int kTieOffBits = 24;
constexpr uint32_t kTieRemRank = 127;
__device__ __forceinline__ void tie_keys(int64_t e, uint64_t sg, const TieCall &c, const TieRule &t, bool lanes,
                                         uint64_t &k1, uint64_t &w, uint64_t &ka);
__device__ __forceinline__ int tie_finalize(uint64_t k1, uint64_t w, uint64_t ka, const TieCall &c,
                                            const TieRule &t);
__device__ __forceinline__ void tie_keys32(uint32_t e, uint64_t sg, const TieCall &c, const TieRule &t,
                                           const uint8_t *rank, const uint8_t *arank, bool lanes, uint64_t &k1,
                                           uint64_t &w, uint64_t &ka);

// box-query combine (pyas_combine_grid): one thread per final output element,
// chunk layers folded in C order of the reduced dims' coordinates
template <typename T, bool KEY>
__global__ __launch_bounds__(kBlock) void k_combine_grid(const pyas_partial *in, pyas_grid g, CombineTie ct,
                                                         int64_t n_out, int64_t n_layers,
                                                         uint32_t flags, pyas_partial *out) {
    const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    // KEY: the level-2 keys depend on the layer's position alone, so up to
    // kKeyTab layers they are worked out once per workgroup (sign bit 0; a
    // zero's sign is OR-ed in), not per output and zero layer
    constexpr int kKeyTab = KEY ? 512 : 1;
    __shared__ uint64_t ktab1[kKeyTab], ktabw[kKeyTab];
    const bool ktab = KEY && n_layers <= kKeyTab;
    if constexpr (KEY) {
        if (ktab) {   // uniform over the workgroup
            for (int e = (int)threadIdx.x; e < (int)n_layers; e += kBlock) {
                uint64_t x1, xw, xa;
                tie_keys32((uint32_t)e, 0u, ct.c, ct.t, ct.t.rank, ct.t.acc_rank, true, x1, xw, xa);
                ktab1[e] = x1;
                ktabw[e] = xw;
            }
            __syncthreads();
        }
    }
    if (f >= n_out) return;
    const bool round = (flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    int64_t gstride[PYAS_MAX_DIMS];
    int64_t j = 0, jstride = 1, st = 1, nk = 0;   // nk: the chunk position of the kept coordinates
    // (outputs under 2^32 -- every practical grid -- decode f in 32-bit
    // divisions: 64-bit ones are a long software sequence per kept dim)
    const bool narrow = (uint64_t)n_out <= 0xFFFFFFFFull;
    int64_t rest = f;
    uint32_t rest32 = (uint32_t)f;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        gstride[d] = st;
        if (d < g.ndim) {
            if (!((g.axes_mask >> d) & 1u)) {
                int64_t p;
                if (narrow) {
                    const uint32_t e = (uint32_t)g.out_extent[d], q = rest32 / e;
                    p = rest32 - q * e;
                    rest32 = q;
                } else {
                    const int64_t e = g.out_extent[d];
                    p = rest % e;
                    rest /= e;
                }
                const int64_t ad = g.pos_coord[d][p];
                nk += ad * st;
                j += (int64_t)g.pos_local[d][p] * jstride;
                jstride *= g.coord_count[d][ad];
            }
            st *= g.n_coords[d];
        }
    }
    // Layers in C order over the reduced dims: a radix counter walks the
    // chunk positions (no division per layer), and U layers' offset and
    // partial loads are issued before they are merged (in the same order, so
    // the result does not change): with few outputs and many layers (C3
    // axes (0,1): 1024 outputs x 256 layers) the fold is latency-bound.
    WAcc<T> acc;
    acc.init();
    int64_t digit[PYAS_MAX_DIMS];
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) digit[d] = 0;
    int64_t n = nk;
    // PYAS_FOLD_ZERO_SIGN_* (flags bits 8-9; the records carry level 1): the
    // sign of the last layer whose min (max) is a zero (elementwise `out`
    // calls), or (KEY) NumPy's level-2 keys over the zero layers at their
    // positions in the `out` call, as k_tie_grid_t would take them
    const uint32_t zs = (flags >> 8) & 3u;
    bool zneg = false;
    uint64_t zk1 = 0, zkw = kTieWNone;
    const int rec = (int)((flags >> 4) & 3u);
    // U layers' offsets, then their U partials, in flight before the merges;
    // compact records of <= 4-byte types (RAW) load as 8-B words, so 16
    // layers fit the registers 8 full partials took
    auto layers = [&](auto u_c, auto raw_c) {
        constexpr int U = decltype(u_c)::value;
        constexpr bool RAW = decltype(raw_c)::value;
        for (int64_t l0 = 0; l0 < n_layers; l0 += U) {
            int64_t off[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                off[u] = 0;
                if (l0 + u < n_layers) {
                    off[u] = g.chunk_out_offsets[n];
                    bool carry = true;
#pragma unroll
                    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
                        if (carry && d < g.ndim && ((g.axes_mask >> d) & 1u)) {
                            n += gstride[d];
                            if (++digit[d] == g.n_coords[d]) {
                                digit[d] = 0;
                                n -= g.n_coords[d] * gstride[d];
                            } else {
                                carry = false;
                            }
                        }
                    }
                }
            }
            using LT = typename std::conditional<RAW, uint2, pyas_partial>::type;
            LT ld[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (l0 + u < n_layers) {
                    if constexpr (RAW) ld[u] = reinterpret_cast<const uint2 *>(in)[off[u] + j];
                    else ld[u] = part_at<T>(in, off[u] + j, rec);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (l0 + u < n_layers) {
                    pyas_partial pu;
                    if constexpr (RAW) pu = part_raw<T>(ld[u], rec);
                    else pu = ld[u];
                    merge(acc, pu, round);
                    if constexpr (TT<T>::kind == 0) {
                        if (zs && pu.count > 0) {
                            const double v = zs == 1 ? pu.min.f : pu.max.f;
                            if (v == 0.0) {
                                zneg = __builtin_signbit(v) != 0;
                                if constexpr (KEY) {
                                    uint64_t x1, xw, xa;
                                    if (ktab) {
                                        const uint64_t sg = zneg ? 1u : 0u;
                                        x1 = ktab1[l0 + u];
                                        x1 = x1 ? x1 | sg : 0u;
                                        xw = ktabw[l0 + u] | sg;
                                    } else {
                                        // 32-bit keys (a layer's position is < 2^31): the
                                        // 64-bit divisions of tie_keys cost the combine ~2x
                                        tie_keys32((uint32_t)(l0 + u), zneg ? 1u : 0u, ct.c, ct.t, ct.t.rank,
                                                   ct.t.acc_rank, true, x1, xw, xa);
                                    }
                                    zk1 = x1 > zk1 ? x1 : zk1;
                                    zkw = xw < zkw ? xw : zkw;
                                }
                            }
                        }
                    }
                }
            }
        }
    };
    if constexpr (sizeof(T) <= 4) {
        if (rec) layers(std::integral_constant<int, 16>(), std::true_type());
        else layers(std::integral_constant<int, 8>(), std::false_type());
    } else {
        layers(std::integral_constant<int, 8>(), std::false_type());
    }
    if constexpr (TT<T>::kind == 0) {
        if (zs && (zs == 1 ? acc.mn : acc.mx) == (T)0) {
            bool neg = zneg;
            if constexpr (KEY) {
                const int sg = tie_finalize(zk1, zkw, 0, ct.c, ct.t);
                neg = sg > 0;
                if (sg < 0) neg = __builtin_signbit(zs == 1 ? acc.mn : acc.mx) != 0;
            }
            if (zs == 1) acc.mn = neg ? (T)-0.0 : (T)0.0;
            else acc.mx = neg ? (T)-0.0 : (T)0.0;
        }
    }
    store_wpartial(out + f, acc);
}

// k_combine_grid for few outputs with many layers each (C3 axes (0,1)/(1,2)/
// (0,2): 1024 outputs x 256 layers, where one thread per output leaves 16
// waves on the device, each waiting on its layers' loads in turn): one wave
// per output, lane t holding layer l0 + t of a 64-layer tile, up to kCwTiles
// tiles' loads in flight per lane.  Per tile:
//  - count, min and max go through an in-order butterfly (the lower lane
//    block is the left operand): merge's min/max keep the earlier of equal
//    values and the later NaN, and the count guard makes an empty layer the
//    identity, so this operator is associative and the tree equals the
//    sequential fold;
//  - each lane rounds its layer's sum (sum_of) and lane 0 adds the 64 sums
//    from LDS in layer order, the only sequential chain left.
// Same values as k_combine_grid's merges, in the same order: bit-identical.
constexpr int kCombineWaveMinLayers = 32;   // below this the per-thread form is used
// Above this many outputs the per-thread form has enough waves to hide its
// loads (>= 8 per CU) and reads each layer's partials coalesced across
// adjacent outputs, where the wave form reads 32 B per lane from 64 chunks
constexpr int64_t kCombineWaveMaxOut = int64_t(1) << 17;
constexpr int kCwTiles = 4;                 // 64-layer tiles in flight per lane

template <typename T>
__device__ __forceinline__ void cw_combine(int64_t &c, T &mn, T &mx, int64_t c2, T mn2, T mx2) {
    c += c2;
    mn = pmin(mn, mn2);   // (left, right)
    mx = pmax(mx, mx2);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_combine_grid_wave(const pyas_partial *in, pyas_grid g,
                                                              int64_t n_out, int64_t n_layers,
                                                              uint32_t flags, pyas_partial *out) {
    using A = typename TT<T>::Acc;
    __shared__ A s_sum[kBlock / kWave][kWave];
    const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int64_t f = (int64_t)blockIdx.x * (kBlock / kWave) + w;
    if (f >= n_out) return;   // wave-uniform; only wave-level syncs below
    const bool round = (flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    int64_t gstride[PYAS_MAX_DIMS];
    int64_t j = 0, jstride = 1, rest = f, st = 1, nk = 0;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        gstride[d] = st;
        if (d < g.ndim) {
            st *= g.n_coords[d];
            if (!((g.axes_mask >> d) & 1u)) {
                const int64_t e = g.out_extent[d];
                const int64_t p = rest % e;
                rest /= e;
                const int64_t c = g.pos_coord[d][p];
                nk += c * gstride[d];
                j += (int64_t)g.pos_local[d][p] * jstride;
                jstride *= g.coord_count[d][c];
            }
        }
    }
    auto offset = [&](int64_t l) {   // layer l (< 2^31, host) -> its chunk's partial array
        int64_t n = nk;
        uint32_t rr = (uint32_t)l;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            if (d < g.ndim && ((g.axes_mask >> d) & 1u)) {
                const uint32_t nc = (uint32_t)g.n_coords[d], q = rr / nc;
                n += (int64_t)(rr - q * nc) * gstride[d];
                rr = q;
            }
        }
        return g.chunk_out_offsets[n];
    };
    WAcc<T> acc;
    acc.init();
    for (int64_t l0 = 0; l0 < n_layers; l0 += kCwTiles * kWave) {   // wave-uniform
        pyas_partial p[kCwTiles];
        int64_t off[kCwTiles];
#pragma unroll
        for (int u = 0; u < kCwTiles; ++u) {
            const int64_t l = l0 + u * kWave + lane;
            off[u] = l < n_layers ? offset(l) : 0;
        }
#pragma unroll
        for (int u = 0; u < kCwTiles; ++u) {
            const int64_t l = l0 + u * kWave + lane;
            if (l < n_layers) p[u] = part_at<T>(in, off[u] + j, (int)((flags >> 4) & 3u));
        }
#pragma unroll
        for (int u = 0; u < kCwTiles; ++u) {
            const int64_t t0 = l0 + u * kWave;
            if (t0 >= n_layers) break;
            const bool live = t0 + lane < n_layers;
            int64_t c = 0;
            T mn = TT<T>::highest(), mx = TT<T>::lowest();
            A sm = 0;
            if (live) {
                sm = sum_of<T>(p[u].sum, round);
                if (p[u].count > 0) {
                    c = p[u].count;
                    mn = TT<T>::from(p[u].min);
                    mx = TT<T>::from(p[u].max);
                }
            }
#pragma unroll
            for (int m = 1; m < kWave; m <<= 1) {
                const int64_t c2 = shfl_xor(c, m);
                const T mn2 = shfl_xor(mn, m), mx2 = shfl_xor(mx, m);
                if (lane & m) {            // partner block is the earlier one
                    int64_t cl = c2;
                    T lmn = mn2, lmx = mx2;
                    cw_combine(cl, lmn, lmx, c, mn, mx);
                    c = cl; mn = lmn; mx = lmx;
                } else {
                    cw_combine(c, mn, mx, c2, mn2, mx2);
                }
            }
            s_sum[w][lane] = sm;
            wave_sync_lds();
            if (lane == 0) {
                const int m = (int)(n_layers - t0 < kWave ? n_layers - t0 : kWave);
                A x = acc.sum;
                if (m == kWave) {
#pragma unroll 16
                    for (int k = 0; k < kWave; ++k) x += s_sum[w][k];
                } else {
                    for (int k = 0; k < m; ++k) x += s_sum[w][k];
                }
                acc.sum = x;
                acc.count += c;
                acc.mn = pmin(acc.mn, mn);
                acc.mx = pmax(acc.mx, mx);
            }
            wave_sync_lds();   // lane 0's reads before the next tile's writes
        }
    }
    if (lane == 0) store_wpartial(out + f, acc);
}

// ---------------------------------------------------------------------------
// partial-axis reduction (axis ⊂ dims), one thread per output element
// ---------------------------------------------------------------------------
// Two layouts, chosen by the host:
//  column (a.row == false; innermost selected dim kept): a workgroup holds
//    OT = 256/S outputs x S splits of the reduced range; lanes with the same
//    split hold consecutive outputs (consecutive addresses); the S partials of
//    an output are folded through LDS in split order (deterministic);
//  row (a.row; innermost dim reduced): G lanes per output (G a power of two,
//    about 8 elements per lane), 64/G outputs per wave, lanes of a group read
//    consecutive addresses, then a segmented shuffle reduce inside the group.
// Both walk index spaces with radix counters (no per-element division) and
// keep 4 independent loads in flight per lane.
template <typename T, int U, bool SHUF, bool BSWAP>
__device__ __forceinline__ void axes_walk(const ReduceArgs &r, const uint8_t *base, const Sel &s,
                                          uint32_t red, const Decomp &base_o, RadixCounter &rc,
                                          int64_t q0, int64_t n_red, int64_t stride, bool tabs,
                                          const MaskT<T> &mk, TileAcc<T> &acc) {
    int64_t q = q0;
    const int64_t nfull = q0 + ((n_red - q0 + stride - 1) / stride) / U * U * stride;
    for (; q < nfull; q += U * stride) {
        Decomp od[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            od[u] = base_o;
            rc.locate(s, r.pool, r.cstride, r.tab, r.ndim, red, od[u]);
            rc.advance();
        }
        T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = load_elem<T, SHUF, BSWAP>(base, r.chunk_elems, od[u].mem);
#pragma unroll
        for (int u = 0; u < U; ++u) acc.add_one(x[u], tabs ? all_masked(mk, r.tab, od[u], x[u]) : mk.masked(x[u]));
    }
    for (; q < n_red; q += stride) {
        Decomp od = base_o;
        rc.locate(s, r.pool, r.cstride, r.tab, r.ndim, red, od);
        const T x = load_elem<T, SHUF, BSWAP>(base, r.chunk_elems, od.mem);
        acc.add_one(x, tabs ? all_masked(mk, r.tab, od, x) : mk.masked(x));
        rc.advance();
    }
}

// Same walk with the reduced-index -> element-offset map precomputed in LDS
// (no tables): per element one LDS read, one add, one load; U in flight.
template <typename T, int U, bool SHUF, bool BSWAP>
__device__ __forceinline__ void axes_walk_lds(const uint8_t *base, int64_t chunk_elems,
                                              const int32_t *roff, int64_t base_mem, int64_t q0,
                                              int64_t n_red, int64_t stride, const MaskT<T> &mk,
                                              TileAcc<T> &acc) {
    int64_t q = q0;
    const int64_t nfull = q0 + ((n_red - q0 + stride - 1) / stride) / U * U * stride;
    for (; q < nfull; q += U * stride) {
        T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[u] = load_elem<T, SHUF, BSWAP>(base, chunk_elems, base_mem + roff[q + u * stride]);
#pragma unroll
        for (int u = 0; u < U; ++u) acc.add_one(x[u], mk.masked(x[u]));
    }
    for (; q < n_red; q += stride) {
        const T x = load_elem<T, SHUF, BSWAP>(base, chunk_elems, base_mem + roff[q]);
        acc.add_one(x, mk.masked(x));
    }
}


// Fold the S split partials of each of OT outputs through LDS in split order
// (deterministic); thread (ol, sp=0) ends with the folded value.
// fold_splits for the N accumulators of a lane at once: one barrier pair
// per pass instead of one per output.  `lds`: fold_lds_bytes<T, N>() bytes.
template <typename T, int N>
constexpr int fold_lds_bytes() {
    return N * kBlock * (int)(sizeof(typename TT<T>::Acc) + sizeof(uint32_t) + 2 * sizeof(T) + 1);
}
template <typename T, int N>
__device__ __forceinline__ void fold_splits_n(TileAcc<T> *acc, int S, int OT, int ol, int sp, void *lds) {
    using A = typename TT<T>::Acc;
    A *l_sum = reinterpret_cast<A *>(lds);
    uint32_t *l_cnt = reinterpret_cast<uint32_t *>(l_sum + N * kBlock);
    T *l_mn = reinterpret_cast<T *>(l_cnt + N * kBlock);
    T *l_mx = l_mn + N * kBlock;
    uint8_t *l_nan = reinterpret_cast<uint8_t *>(l_mx + N * kBlock);
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        l_sum[k * kBlock + t] = acc[k].sum;
        l_cnt[k * kBlock + t] = acc[k].count;
        l_mn[k * kBlock + t] = acc[k].mn;
        l_mx[k * kBlock + t] = acc[k].mx;
        l_nan[k * kBlock + t] = acc[k].nan ? 1 : 0;
    }
    __syncthreads();
    if (sp == 0) {
        for (int q = 1; q < S; ++q) {
            const int u = q * OT + ol;
#pragma unroll
            for (int k = 0; k < N; ++k) {
                acc[k].sum += l_sum[k * kBlock + u];
                acc[k].count += l_cnt[k * kBlock + u];
                acc[k].mn = tmin(acc[k].mn, l_mn[k * kBlock + u]);
                acc[k].mx = tmax(acc[k].mx, l_mx[k * kBlock + u]);
                acc[k].nan = acc[k].nan || l_nan[k * kBlock + u];
            }
        }
    }
    __syncthreads();
}

template <typename T>
__device__ __forceinline__ void fold_splits(TileAcc<T> &acc, int S, int OT, int ol, int sp) {
    __shared__ typename TT<T>::Acc l_sum[kBlock];
    __shared__ uint32_t l_cnt[kBlock];
    __shared__ T l_mn[kBlock], l_mx[kBlock];
    __shared__ uint8_t l_nan[kBlock];
    const int t = threadIdx.x;
    l_sum[t] = acc.sum; l_cnt[t] = acc.count; l_mn[t] = acc.mn; l_mx[t] = acc.mx;
    l_nan[t] = acc.nan ? 1 : 0;
    __syncthreads();
    if (sp == 0) {
        for (int k = 1; k < S; ++k) {
            const int u = k * OT + ol;
            acc.sum += l_sum[u];
            acc.count += l_cnt[u];
            acc.mn = tmin(acc.mn, l_mn[u]);
            acc.mx = tmax(acc.mx, l_mx[u]);
            acc.nan = acc.nan || l_nan[u];
        }
    }
    __syncthreads();
}

template <typename T, bool SHUF, bool BSWAP>
__device__ void axes_block(const AxesArgs &a, int64_t c, int64_t j, const uint8_t *base,
                           const Sel &s, uint32_t red, uint32_t keep, int64_t n_out, int64_t n_red,
                           const MaskT<T> &mk, int32_t *roff) {
    const ReduceArgs &r = a.r;
    constexpr int ES = sizeof(T), N = 16 / ES;
    const bool tabs = r.tab.on[0] || r.tab.on[1];
    const bool use_lds = !tabs && n_red <= a.roff_cap;   // roff holds a.roff_cap entries
    // 16-B vector modes: the last chunk dim is a unit-step, 16-B aligned run
    const int last = r.ndim - 1;
    int64_t cnt_last = 1, start_last = 0, step_last = 1, shape_last = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d == last) { cnt_last = s.cnt[d]; start_last = s.start[d]; step_last = s.step[d]; shape_last = r.shape[d]; }
    const bool vec_ok = use_lds && !SHUF && ES >= 4 && step_last == 1 && ((uintptr_t)base & 15) == 0 &&
                        (cnt_last * ES) % 16 == 0 && (start_last * ES) % 16 == 0 && (shape_last * ES) % 16 == 0;
    const bool row_vec = a.row && a.vec && vec_ok;
    const bool col_vec = !a.row && a.vec && vec_ok;
    if (use_lds) {   // reduced-index -> element offset, once per workgroup
        const int64_t nq = row_vec ? n_red / N : n_red;
        const uint64_t m = row_vec ? N : 1;
        RadixCounter t;   // one decomposition per thread, then digit adds
        t.init(s, r.ndim, red, threadIdx.x * m, kBlock * m);
        for (int64_t q = threadIdx.x; q < nq; q += kBlock) {
            Decomp d{0, {0, 0}};
            t.locate(s, r.pool, r.cstride, r.tab, r.ndim, red, d);
            roff[q] = (int32_t)d.mem;
            t.advance();
        }
        __syncthreads();
    }
    if (!a.row) {
        int S = a.split;
        // 16-B column walks: the host sized the split for the chunk's whole
        // kept extent; a chunk whose selection keeps fewer vectors (a strided
        // kept dim: [:, ::3, :] over (0,) keeps a third) splits its reduced
        // rows over the lanes that would otherwise idle (block-uniform: per
        // chunk), keeping >= 8 rows per lane
        if (col_vec) {
            const int64_t nvec = n_out / N;
            while (S * 2 <= kBlock && nvec * S * 2 <= a.bpc * kBlock && n_red / (S * 2) >= 8) S *= 2;
        }
        const int OT = kBlock / S;
        const int ol = threadIdx.x % OT, sp = threadIdx.x / OT;
        const int64_t n_items = col_vec ? n_out / N : n_out;   // outputs or N-output vectors
        const uint64_t m = col_vec ? N : 1;
        RadixCounter ko;   // kept-index counter stepping with the loop
        ko.init(s, r.ndim, keep, (uint64_t)(j * OT + ol) * m, (uint64_t)(a.bpc * OT) * m);
        for (int64_t o0 = j * OT; o0 < n_items; o0 += a.bpc * OT) {   // block-uniform loop
            const int64_t oi = o0 + ol;
            Decomp base_o{0, {0, 0}};
            if (oi < n_items) ko.locate(s, r.pool, r.cstride, r.tab, r.ndim, keep, base_o);
            ko.advance();
            if (col_vec) {
                TileAcc<T> acc[N];
#pragma unroll
                for (int k = 0; k < N; ++k) acc[k].init();
                if (oi < n_items) {
                    // U rows in flight per lane; output k's U values summed
                    // in groups of 4 (widened once per group, as the dense
                    // column walk), one NaN ballot per U rows
                    const uint8_t *bo = base + base_o.mem * ES;
                    constexpr int U = 8;
                    int64_t q = sp;
                    const int64_t nfull = sp + ((n_red - sp + S - 1) / S) / U * U * S;
                    for (; q < nfull; q += U * S) {
                        uint4 v[U];
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            v[u] = ldg16(reinterpret_cast<const uint4 *>(bo + (int64_t)roff[q + u * S] * ES));
                        T xs[N][U];
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            T x[N];
                            unpack16<T, BSWAP>(v[u], x);
#pragma unroll
                            for (int k = 0; k < N; ++k) xs[k][u] = x[k];
                        }
                        bool bad = false;
#pragma unroll
                        for (int k = 0; k < N; ++k) bad |= acc[k].template add_lazy<U, kMaskAll, false>(xs[k], mk);
                        if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
                            for (int k = 0; k < N; ++k) acc[k].template check_nan<U>(xs[k]);
                        }
                    }
                    for (; q < n_red; q += S) {
                        T x[N];
                        unpack16<T, BSWAP>(ldg16(reinterpret_cast<const uint4 *>(bo + (int64_t)roff[q] * ES)), x);
#pragma unroll
                        for (int k = 0; k < N; ++k) acc[k].add_one(x[k], mk.masked(x[k]));
                    }
                }
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    if (S > 1) fold_splits(acc[k], S, OT, ol, sp);
                    if (sp == 0 && oi < n_items) {
                        pyas_partial pp;
                        tile_store_lane(acc[k], &pp);
                        put_out<T>(a, a.out_offsets[c] + oi * N + k, pp);
                    }
                }
                continue;
            }
            TileAcc<T> acc;
            acc.init();
            if (oi < n_items) {
                if (use_lds) {
                    axes_walk_lds<T, 8, SHUF, BSWAP>(base, r.chunk_elems, roff, base_o.mem, sp, n_red, S, mk, acc);
                } else {
                    RadixCounter rc;
                    rc.init(s, r.ndim, red, (uint64_t)sp, (uint64_t)S);
                    axes_walk<T, 4, SHUF, BSWAP>(r, base, s, red, base_o, rc, sp, n_red, S, tabs, mk, acc);
                }
            }
            if (S > 1) fold_splits(acc, S, OT, ol, sp);
            if (sp == 0 && oi < n_items) {
                pyas_partial pp;
                tile_store_lane(acc, &pp);
                put_out<T>(a, a.out_offsets[c] + oi, pp);
            }
        }
    } else {
        // G lanes per output (host-sized for element or 16-B vector walks)
        const int G = a.group;
        const int lane = threadIdx.x & (kWave - 1);
        const int gl = lane & (G - 1);
        const int64_t per_wave = kWave / G;
        const int64_t wave = (int64_t)j * (kBlock / kWave) + threadIdx.x / kWave;
        const int64_t nwaves = (int64_t)a.bpc * (kBlock / kWave);
        RadixCounter ko;   // kept-index counter stepping with the loop
        ko.init(s, r.ndim, keep, (uint64_t)(wave * per_wave + lane / G), (uint64_t)(nwaves * per_wave));
        for (int64_t o0 = wave * per_wave; o0 < n_out; o0 += nwaves * per_wave) {  // wave-uniform
            const int64_t o = o0 + lane / G;
            TileAcc<T> acc;
            acc.init();
            Decomp base_o{0, {0, 0}};
            if (o < n_out) ko.locate(s, r.pool, r.cstride, r.tab, r.ndim, keep, base_o);
            ko.advance();
            if (o < n_out) {
                if (row_vec) {
                    const uint8_t *bo = base + base_o.mem * ES;
                    const int64_t nv = n_red / N;
                    constexpr int U = 4;
                    int64_t q = gl;
                    const int64_t nfull = gl + ((nv - gl + G - 1) / G) / U * U * G;
                    for (; q < nfull; q += U * G) {
                        uint4 v[U];
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            v[u] = ldg16(reinterpret_cast<const uint4 *>(bo + (int64_t)roff[q + u * G] * ES));
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            T x[N];
                            unpack16<T, BSWAP>(v[u], x);
                            acc.template add_n<N, true, false>(x, mk);
                        }
                    }
                    for (; q < nv; q += G) {
                        T x[N];
                        unpack16<T, BSWAP>(ldg16(reinterpret_cast<const uint4 *>(bo + (int64_t)roff[q] * ES)), x);
                        acc.template add_n<N, true, false>(x, mk);
                    }
                } else if (use_lds) {
                    axes_walk_lds<T, 8, SHUF, BSWAP>(base, r.chunk_elems, roff, base_o.mem, gl, n_red, G, mk, acc);
                } else {
                    RadixCounter rc;
                    rc.init(s, r.ndim, red, (uint64_t)gl, (uint64_t)G);
                    axes_walk<T, 4, SHUF, BSWAP>(r, base, s, red, base_o, rc, gl, n_red, G, tabs, mk, acc);
                }
            }
            pyas_partial pp;
            group_finish(acc, G, (o < n_out && gl == 0) ? &pp : nullptr);
            if (o < n_out && gl == 0) put_out<T>(a, a.out_offsets[c] + o, pp);
        }
    }
}

// ---------------------------------------------------------------------------
// dense partial-axis reduction: a fully selected, unshuffled chunk without
// index tables.  The host merges the chunk dims into the canonical form
// (RO, KO, RI, KI) = (reduced outer, kept outer, reduced inner, kept inner):
// element (ro, ko, ri, ki) at ((ro*KO + ko)*RI + ri)*KI + ki, output
// ko*KI + ki, reduced row ro*RI + ri.  No offset maps, no radix counters:
// addresses advance by constant strides.
//  column (KI*ES % 16 == 0): a lane owns one 16-B vector of N outputs, the
//    reduced rows are split over S lane sets (folded in split order);
//    a wave reads whole 16-B runs of the same row (1 KiB when KI >= 64 N);
//  row (KI == 1): G lanes per output read consecutive 16-B vectors of its
//    runs (a wave reads 64/G adjacent runs = 1 KiB), DPP butterfly per group;
//    with one vector per lane per output each lane keeps 4 outputs in flight.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool chunk_is_full(const Sel &s, const int64_t *shape, int ndim) {
    bool full = true;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d)
        if (d < ndim) full = full && s.start[d] == 0 && s.step[d] == 1 && s.cnt[d] == shape[d];
    return full;
}

template <int CTRL, typename V>
__device__ __forceinline__ V dpp_mov(V v) {
    if constexpr (sizeof(V) <= 4) {
        int w = 0;
        __builtin_memcpy(&w, &v, sizeof(V));
        w = __builtin_amdgcn_update_dpp(0, w, CTRL, 0xf, 0xf, false);
        V r;
        __builtin_memcpy(&r, &w, sizeof(V));
        return r;
    } else {
        int w[2];
        __builtin_memcpy(w, &v, 8);
        w[0] = __builtin_amdgcn_update_dpp(0, w[0], CTRL, 0xf, 0xf, false);
        w[1] = __builtin_amdgcn_update_dpp(0, w[1], CTRL, 0xf, 0xf, false);
        V r;
        __builtin_memcpy(&r, w, 8);
        return r;
    }
}

// Butterfly over aligned groups of G lanes (G power of two <= 64, wave-
// uniform): quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror
// (each pairs uniform halves of the group so far), then xor 16 / 32.
// Every lane of a group ends with the group's combined partial.
template <typename T>
__device__ __forceinline__ void group_reduce(TileAcc<T> &a, int G, uint32_t &cnt, uint32_t &nan) {
    cnt = a.count;
    nan = a.nan ? 1u : 0u;
#define PYAS_DPP_STEP(CTRL)                                   \
    do {                                                      \
        a.sum += dpp_mov<CTRL>(a.sum);                        \
        cnt += dpp_mov<CTRL>(cnt);                            \
        a.mn = tmin(a.mn, dpp_mov<CTRL>(a.mn));               \
        a.mx = tmax(a.mx, dpp_mov<CTRL>(a.mx));               \
        nan |= dpp_mov<CTRL>(nan);                            \
    } while (0)
    if (G >= 2) PYAS_DPP_STEP(0xB1);
    if (G >= 4) PYAS_DPP_STEP(0x4E);
    if (G >= 8) PYAS_DPP_STEP(0x141);
    if (G >= 16) PYAS_DPP_STEP(0x140);
#undef PYAS_DPP_STEP
    for (int m = 16; m < G; m <<= 1) {
        a.sum += shfl_xor(a.sum, m);
        cnt += shfl_xor(cnt, m);
        a.mn = tmin(a.mn, shfl_xor(a.mn, m));
        a.mx = tmax(a.mx, shfl_xor(a.mx, m));
        nan |= shfl_xor(nan, m);
    }
}

template <typename T>
__device__ __forceinline__ void store_group(const TileAcc<T> &a, uint32_t cnt, uint32_t nan,
                                            pyas_partial *out) {
    pyas_partial p;
    TT<T>::put_acc(p.sum, a.sum);
    p.count = (int64_t)cnt;
    T mn = a.mn, mx = a.mx;
    if constexpr (TT<T>::kind == 0) {
        if (nan) { mn = (T)__builtin_nan(""); mx = mn; }
    }
    TT<T>::put(p.min, mn);
    TT<T>::put(p.max, mx);
    *out = p;
}

#ifndef PYAS_COL_U
#define PYAS_COL_U 4      // 16-B loads per step per lane (column layout; measured 4 >= 8)
#endif
// Occupancy floors (waves per SIMD; 0 = none) of the partial-axis kernels,
// per layout: column / row / LDS-row per-chunk kernels, column / LDS-row
// in-kernel folds.  A floor caps VGPRs at 512 / waves (minus granularity).
#ifndef PYAS_COL_WAVES
#define PYAS_COL_WAVES 0
#endif
#ifndef PYAS_ROW_WAVES
#define PYAS_ROW_WAVES 0
#endif
#ifndef PYAS_LDS_WAVES
#define PYAS_LDS_WAVES 0
#endif
#ifndef PYAS_STREAM_WAVES
#define PYAS_STREAM_WAVES 0
#endif
#ifndef PYAS_FOLD_COL_WAVES
#define PYAS_FOLD_COL_WAVES 0
#endif
#ifndef PYAS_FOLD_ROW_WAVES
#define PYAS_FOLD_ROW_WAVES 0
#endif
#define PYAS_WAVES_FLOOR_(W) __attribute__((amdgpu_waves_per_eu(W, 8)))
#define PYAS_WAVES_FLOOR(W) PYAS_WAVES_FLOOR_##W
#define PYAS_WAVES_FLOOR_0
#define PYAS_WAVES_FLOOR_1 PYAS_WAVES_FLOOR_(1)
#define PYAS_WAVES_FLOOR_2 PYAS_WAVES_FLOOR_(2)
#define PYAS_WAVES_FLOOR_3 PYAS_WAVES_FLOOR_(3)
#define PYAS_WAVES_FLOOR_4 PYAS_WAVES_FLOOR_(4)
#define PYAS_WAVES_FLOOR_5 PYAS_WAVES_FLOOR_(5)
#define PYAS_WAVES_FLOOR_6 PYAS_WAVES_FLOOR_(6)
#define PYAS_WAVES_FLOOR_7 PYAS_WAVES_FLOOR_(7)
#define PYAS_WAVES_FLOOR_8 PYAS_WAVES_FLOOR_(8)
#define PYAS_XATTR(W) PYAS_WAVES_FLOOR(W)

// ---------------------------------------------------------------------------
// cut chunks in the dense kernels
// ---------------------------------------------------------------------------
// A chunk cut by a box selection (a hyperslab's edge: unit steps, at least
// half the chunk selected) is read by the dense kernels as its whole chunk:
// the reduced elements outside the box are excluded (a per-row bit from an
// LDS map in the column layouts, per-element bits in the row layouts) and
// the outputs outside it are not written; those inside go to their place in
// the chunk's partial array (C order over the box's kept extents).  The
// bytes outside the box are still read: at most half the chunk by the
// eligibility rule, ~1.6 % per cut dim at a [1:1023] edge of 64^3 chunks.
struct CutBox {
    int32_t lo[PYAS_MAX_DIMS], hi[PYAS_MAX_DIMS];   // the box, chunk coordinates
    int64_t ost[PYAS_MAX_DIMS];                    // kept dims: output strides; reduced: 0
};

// Whether the dense launch (a.cuts) takes this cut chunk; identical in the
// dense kernels and k_reduce_axes, which leaves it to them.
__device__ __forceinline__ bool cut_eligible(const AxesArgs &a, const Sel &s) {
    if (!a.cuts) return false;
    int64_t sel = 1, all = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d < a.r.ndim) {
            if (s.step[d] != 1 && s.cnt[d] != 1) return false;   // a box: unit steps (or one index)
            if (s.cnt[d] < 1) return false;
            sel *= s.cnt[d];
            all *= a.r.shape[d];
        }
    }
    return 2 * sel >= all;
}

__device__ __forceinline__ void cut_box(const AxesArgs &a, const Sel &s, CutBox &cb) {
    int64_t st = 1;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        cb.lo[d] = 0;
        cb.hi[d] = 1;
        cb.ost[d] = 0;
        if (d < a.r.ndim) {
            cb.lo[d] = (int32_t)sel_index(s, a.r.pool, d, 0);
            cb.hi[d] = cb.lo[d] + s.cnt[d];
            if (!((a.axes >> d) & 1u)) {
                cb.ost[d] = st;
                st *= s.cnt[d];
            }
        }
    }
}

// Kept index f (C order over the kept dims, whole-chunk extents) -> its
// place in the cut chunk's partial array, or -1 outside the box.  32-bit
// arithmetic (a.cuts needs chunks under 2^31 elements).
__device__ __forceinline__ int64_t cut_out(const AxesArgs &a, const CutBox &cb, int64_t fi) {
    uint32_t f = (uint32_t)fi;
    int64_t o = 0;
    bool in = true;
#pragma unroll
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < a.r.ndim && !((a.axes >> d) & 1u)) {
            const uint32_t n = (uint32_t)a.r.shape[d], q = f / n, c = f - q * n;
            f = q;
            in = in && (int32_t)c >= cb.lo[d] && (int32_t)c < cb.hi[d];
            o += ((int64_t)c - cb.lo[d]) * cb.ost[d];
        }
    }
    return in ? o : -1;
}

// The kept coordinates of consecutive kept indices f0, f0 + 1, ... (a
// column item's N outputs): one decomposition, then carry-propagating steps.
struct CutWalk {
    int32_t c[PYAS_MAX_DIMS];
    __device__ __forceinline__ void init(const AxesArgs &a, int64_t f0) {
        uint32_t f = (uint32_t)f0;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            c[d] = 0;
            if (d < a.r.ndim && !((a.axes >> d) & 1u)) {
                const uint32_t n = (uint32_t)a.r.shape[d], q = f / n;
                c[d] = (int32_t)(f - q * n);
                f = q;
            }
        }
    }
    // place of the current index in the cut chunk's array, or -1
    __device__ __forceinline__ int64_t out(const AxesArgs &a, const CutBox &cb) const {
        int64_t o = 0;
        bool in = true;
#pragma unroll
        for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
            if (d < a.r.ndim && !((a.axes >> d) & 1u)) {
                in = in && c[d] >= cb.lo[d] && c[d] < cb.hi[d];
                o += (int64_t)(c[d] - cb.lo[d]) * cb.ost[d];
            }
        }
        return in ? o : -1;
    }
    __device__ __forceinline__ void step(const AxesArgs &a) {
        bool carry = true;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            if (carry && d < a.r.ndim && !((a.axes >> d) & 1u)) {
                ++c[d];
                carry = c[d] >= (int32_t)a.r.shape[d];
                if (carry) c[d] = 0;
            }
        }
    }
};

// Bit map over the reduced positions r (C order over the reduced dims,
// whole-chunk extents; the column layouts' row r = ro * RI + ri, the row
// layouts' element ro * RI + x): bit r set iff r lies in the box.  Built by
// the whole block; nr <= 32 * kCutMapWords (host-checked).
__device__ __forceinline__ void cut_map(const AxesArgs &a, const CutBox &cb, int64_t nr, uint32_t *map) {
    // one position per lane, 64 per wave step, words from a ballot (a
    // word per thread, 32 serial decompositions each, made the LDS row
    // layout's small workgroups wait ~2k cycles on threads 0-1: C3
    // [1:1023]^3 (2,) 1.30 ms)
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int64_t nw = (nr + 31) / 32;
    for (int64_t r0 = (int64_t)wv * kWave; r0 < nr; r0 += kBlock) {   // wave-uniform
        uint32_t r = (uint32_t)(r0 + lane);
        bool in = (int64_t)r < nr;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            if (d < a.r.ndim && ((a.axes >> d) & 1u)) {
                const uint32_t n = (uint32_t)a.r.shape[d], q = r / n, c = r - q * n;
                r = q;
                in = in && (int32_t)c >= cb.lo[d] && (int32_t)c < cb.hi[d];
            }
        }
        const uint64_t b = __ballot(in);
        if (lane == 0) map[r0 / 32] = (uint32_t)b;
        if (lane == 0 && r0 / 32 + 1 < nw) map[r0 / 32 + 1] = (uint32_t)(b >> 32);
    }
    if (threadIdx.x == 0) map[nw] = 0;   // cut_bits may read one word past the end
    __syncthreads();
}

// Bits [r, r + n) of the map (n <= 32), bit 0 = position r.
__device__ __forceinline__ uint32_t cut_bits(const uint32_t *map, int64_t r, int n) {
    const int64_t w = r >> 5;
    const int sh = (int)(r & 31);
    uint64_t v = map[w];
    if (sh + n > 32) v |= (uint64_t)map[w + 1] << 32;
    const uint64_t m = n >= 32 ? 0xffffffffull : ((1ull << n) - 1);
    return (uint32_t)((v >> sh) & m);
}

// U rows of N outputs (16-B vectors w[u]) into acc[N]: output k's U rows as
// groups of 4 (sums widened once per group, one mask test per element,
// per-lane counts), one NaN ballot for all of them.
template <typename T, bool BSWAP, int MASKED, int U>
__device__ __forceinline__ void col_consume(const uint4 *w, TileAcc<T> *acc, const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    static_assert(U % 4 == 0, "PYAS_COL_U: a multiple of the 4-row sum groups");
    T xs[N][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        T x[N];
        unpack16<T, BSWAP>(w[u], x);
#pragma unroll
        for (int k = 0; k < N; ++k) xs[k][u] = x[k];
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < N; ++k) bad |= acc[k].template add_lazy<U, MASKED, false>(xs[k], mk);
    if (__builtin_expect(__ballot(bad) != 0, 0)) {   // a NaN (or inf - inf) somewhere
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k].template check_nan<U>(xs[k]);
    }
}

// col_consume for a cut chunk: only rows whose bit is set in `rows` (bit u =
// row u of the step) count; per-lane counts, masked or not.
template <typename T, bool BSWAP, int MASKED, int U>
__device__ __forceinline__ void col_consume_p(const uint4 *w, TileAcc<T> *acc, const MaskT<T> &mk, uint32_t rows) {
    constexpr int N = 16 / sizeof(T);
    T xs[N][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        T x[N];
        unpack16<T, BSWAP>(w[u], x);
#pragma unroll
        for (int k = 0; k < N; ++k) xs[k][u] = x[k];
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < N; ++k) bad |= acc[k].template add_pred<U, MASKED, 1>(xs[k], rows, mk);
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
        for (int k = 0; k < N; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((rows >> u) & 1u) acc[k].template check_nan<1>(&xs[k][u]);
    }
}

// NumPy's sign of a zero min/max per column output (elementwise level-1
// calls: the chunk's innermost non-1 dim kept, so every later zero wins).
// ZT 1 (splits, S > 1: rows interleave across lanes): zt[k] = ((r + 1) << 1)
// | sign of the last zero of output k this lane read (row r in visiting
// order), max-combined across splits.  ZT 2 (S == 1: one lane walks every
// row in order): zt[k] = the high word of the last zero read (1: none), a
// compare and a select per element; zt_final turns it into ZT 1's form.
// rows: the step's rows in the box (bit u = row r0 + u * S).  Zeros are
// masked all or none (value rules), so a masked zero never decides.
template <typename T, bool BSWAP, int U, int ZT>
__device__ __forceinline__ void col_track_zeros(const uint4 *w, uint32_t *zt, uint32_t rows, int64_t r0, int S) {
    constexpr int N = 16 / sizeof(T);
    using Ub = typename TT<T>::U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        T x[N];
        unpack16<T, BSWAP>(w[u], x);
        const bool in = (rows >> u) & 1u;
        if constexpr (ZT == 2) {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const uint32_t hi = (uint32_t)(bits_to<Ub>(x[k]) >> (8 * sizeof(T) - 32));
                zt[k] = (in && x[k] == (T)0) ? hi : zt[k];
            }
        } else {
            const uint32_t key = (uint32_t)(r0 + (int64_t)u * S + 1) << 1;
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const uint32_t sg = (uint32_t)(bits_to<Ub>(x[k]) >> (8 * sizeof(T) - 1));
                if (in && x[k] == (T)0) zt[k] = key | sg;
            }
        }
    }
}
__device__ __forceinline__ uint32_t zt_final(uint32_t z) { return z == 1u ? 0u : (2u | (z >> 31)); }

// One pass of the column layout over one chunk: lane (il, sp) folds split
// sp of the reduced rows of vector item i (N consecutive kept outputs) into
// acc[N], PYAS_COL_U 16-B loads in flight.
template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, bool CUT = false, int ZT = 0>
__device__ __forceinline__ void col_rows(const AxesDense &d, const uint8_t *base, int64_t n, int64_t i,
                                         int sp, const MaskT<T> &mk, TileAcc<T> *acc,
                                         const uint32_t *rmap = nullptr, uint32_t *zt = nullptr) {
    constexpr int ES = sizeof(T), N = 16 / ES;
    const int S = d.split;
    const int64_t KIV = d.KI / N, R = d.RO * d.RI;
    const int64_t sRO = d.KO * d.RI * d.KI;                    // elements per ro step
    const int64_t dq = S / d.RI, dr = S - dq * d.RI;            // row step S = dq*RI + dr
    const int64_t step_off = (dq * sRO + dr * d.KI) * ES;       // bytes
    const int64_t wrap_off = (sRO - d.RI * d.KI) * ES;          // ri wrapped past RI
    const int64_t ko = i / KIV, v = i - ko * KIV;
    int64_t ro = sp / d.RI, ri = sp - ro * d.RI;
    const uint8_t *p = base + ((ro * d.KO + ko) * d.RI * d.KI + ri * d.KI + v * N) * ES;
    const int64_t nt = (R - sp + S - 1) / S;
    auto next = [&]() {
        p += step_off;
        ri += dr;
        if (ri >= d.RI) { ri -= d.RI; p += wrap_off; }
    };
    constexpr int U = PYAS_COL_U;
    int64_t t = 0;
    for (; t + U <= nt; t += U) {
        uint4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { w[u] = ldv<T, SHUF, AL>(base, p, n); next(); }
        uint32_t rb = (1u << U) - 1u;
        if constexpr (CUT) {
            rb = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) rb |= cut_bits(rmap, sp + (t + u) * S, 1) << u;
            col_consume_p<T, BSWAP, MASKED, U>(w, acc, mk, rb);
        } else {
            col_consume<T, BSWAP, MASKED, U>(w, acc, mk);
        }
        if constexpr (ZT) col_track_zeros<T, BSWAP, U, ZT>(w, zt, rb, sp + t * S, S);
    }
    for (; t < nt; ++t) {
        const uint4 wv = ldv<T, SHUF, AL>(base, p, n);
        T x[N];
        unpack16<T, BSWAP>(wv, x);
        next();
        uint32_t rb = 1u;
        if constexpr (CUT) {
            rb = cut_bits(rmap, sp + t * S, 1);
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (acc[k].template add_pred<1, MASKED, 1>(x + k, rb, mk)) acc[k].template check_nan<1>(x + k);
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) acc[k].template add_n<1, MASKED, false>(x + k, mk);
        }
        if constexpr (ZT) col_track_zeros<T, BSWAP, 1, ZT>(&wv, zt, rb, sp + t * S, S);
    }
    if constexpr (!MASKED && !CUT) {   // add_n counts only in masked mode
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k].count += (uint32_t)nt;
    }
}

// col_rows over 16-B aligned vectors with two 4-row load groups in flight
// while the oldest is consumed (col_rows waits for each group before issuing
// the next).  Same 4-row groups and tail as col_rows: bit-identical.
#ifndef PYAS_COL_RING
#define PYAS_COL_RING 1
#endif
template <typename T, bool SHUF, bool BSWAP, int MASKED, bool CUT = false, int ZT = 0>
__device__ __forceinline__ void col_rows_ring(const AxesDense &d, const uint8_t *base, int64_t n, int64_t i,
                                              int sp, const MaskT<T> &mk, TileAcc<T> *acc,
                                              const uint32_t *rmap = nullptr, uint32_t *zt = nullptr) {
    constexpr int ES = sizeof(T), N = 16 / ES, U = PYAS_COL_U;
    const int S = d.split;
    const int64_t KIV = d.KI / N, R = d.RO * d.RI;
    const int64_t sRO = d.KO * d.RI * d.KI;
    const int64_t dq = S / d.RI, dr = S - dq * d.RI;
    const int64_t step_off = (dq * sRO + dr * d.KI) * ES;
    const int64_t wrap_off = (sRO - d.RI * d.KI) * ES;
    const int64_t ko = i / KIV, v = i - ko * KIV;
    int64_t ro = sp / d.RI, ri = sp - ro * d.RI;
    const uint8_t *p = base + ((ro * d.KO + ko) * d.RI * d.KI + ri * d.KI + v * N) * ES;
    const int64_t nt = (R - sp + S - 1) / S, ng = nt / U;
    auto fetch = [&](uint4 *b) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            b[u] = ldv<T, SHUF, true>(base, p, n);
            p += step_off;
            ri += dr;
            if (ri >= d.RI) { ri -= d.RI; p += wrap_off; }
        }
    };
    // rows of group g: sp + (g * U + u) * S (CUT: their bits from the map)
    auto rbits = [&](int64_t g) -> uint32_t {
        uint32_t rb = 0;
        if (S == 1) {
            rb = cut_bits(rmap, sp + g * U, U);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) rb |= cut_bits(rmap, sp + (g * U + u) * S, 1) << u;
        }
        return rb;
    };
    uint4 buf[2][U];
    if (ng > 0) fetch(buf[0]);
    if (ng > 1) fetch(buf[1]);
    for (int64_t g = 0; g < ng; g += 2) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if (g + s < ng) {
                uint4 cur[U];
#pragma unroll
                for (int u = 0; u < U; ++u) cur[u] = buf[s][u];
                if (g + s + 2 < ng) fetch(buf[s]);
                uint32_t rb = (1u << U) - 1u;
                if constexpr (CUT) {
                    rb = rbits(g + s);
                    col_consume_p<T, BSWAP, MASKED, U>(cur, acc, mk, rb);
                } else {
                    col_consume<T, BSWAP, MASKED, U>(cur, acc, mk);
                }
                if constexpr (ZT) col_track_zeros<T, BSWAP, U, ZT>(cur, zt, rb, sp + (g + s) * U * S, S);
            }
        }
    }
    for (int64_t t = ng * U; t < nt; ++t) {   // p is at row ng * U
        const uint4 wv = ldv<T, SHUF, true>(base, p, n);
        T x[N];
        unpack16<T, BSWAP>(wv, x);
        p += step_off;
        ri += dr;
        if (ri >= d.RI) { ri -= d.RI; p += wrap_off; }
        uint32_t rb = 1u;
        if constexpr (CUT) {
            rb = cut_bits(rmap, sp + t * S, 1);
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (acc[k].template add_pred<1, MASKED, 1>(x + k, rb, mk)) acc[k].template check_nan<1>(x + k);
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) acc[k].template add_n<1, MASKED, false>(x + k, mk);
        }
        if constexpr (ZT) col_track_zeros<T, BSWAP, 1, ZT>(&wv, zt, rb, sp + t * S, S);
    }
    if constexpr (!MASKED && !CUT) {
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k].count += (uint32_t)nt;
    }
}


// Shuffled column layout in load units (ES >= 4): the G = ES lanes of an
// item group (consecutive items of one kept run) each load ONE unit -- 16
// elements = G vectors, one 16-B piece from each byte plane -- of a
// different row, and exchange them through the wave's LDS area (a G x G
// transpose, row stride 65 vectors: conflict-free writes and reads), after
// which each lane holds its own item's vectors for G rows, consumed in row
// order like col_rows' steps.  A wave's plane loads are then 16 B per lane
// (up to 1 KiB per plane per instruction) instead of N-byte pieces, which
// fetched half cache lines.  col_units_ok() is the block-uniform guard;
// `xch` holds kBlock / kWave * G * 65 vectors.
template <typename T>
__device__ __forceinline__ bool col_units_ok(const AxesDense &d) {
    constexpr int ES = sizeof(T), N = 16 / ES, G = ES;
    if constexpr (ES < 4) {
        return false;
    } else {
        const int64_t R = d.RO * d.RI;
        return d.it % G == 0 && (d.KI / N) % G == 0 && R % d.split == 0 && (R / d.split) % G == 0;
    }
}
template <typename T>
constexpr int col_units_lds() { return (kBlock / kWave) * (int)sizeof(T) * 65; }   // vectors

template <typename T, bool BSWAP, int MASKED>
__device__ void col_rows_units(const AxesDense &d, const uint8_t *base, int64_t n, int64_t i, int sp,
                               const MaskT<T> &mk, TileAcc<T> *acc, uint4 *xch) {
    constexpr int ES = sizeof(T), N = 16 / ES, G = ES;
    const int S = d.split;
    const int lane = threadIdx.x & (kWave - 1), j = lane & (G - 1), gl = lane - j;
    const int64_t KIV = d.KI / N, R = d.RO * d.RI;
    const int64_t gi = i - j;                       // the group's first item
    const int64_t ko = gi / KIV, v = gi - ko * KIV;
    const int64_t SG = (int64_t)S * G;              // a lane's row step
    const int64_t sRO = d.KO * d.RI * d.KI;
    const int64_t dq = SG / d.RI, dr = SG - dq * d.RI;
    const int64_t step_off = (dq * sRO + dr * d.KI) * ES, wrap_off = (sRO - d.RI * d.KI) * ES;
    const int64_t r0 = sp + (int64_t)j * S;         // this lane's first row
    int64_t ro = r0 / d.RI, ri = r0 - ro * d.RI;
    const uint8_t *p = base + ((ro * d.KO + ko) * d.RI * d.KI + ri * d.KI + v * N) * ES;
    const int64_t steps = R / SG;
    uint4 *wx = xch + (threadIdx.x / kWave) * (G * 65);
    auto adv = [&]() {
        p += step_off;
        ri += dr;
        if (ri >= d.RI) { ri -= d.RI; p += wrap_off; }
    };
    uint4 nx[G];   // the next step's unit is in flight while this one is consumed
    if (steps > 0) { ldu<T, true, true>(base, p, n, nx); adv(); }
    for (int64_t t = 0; t < steps; ++t) {
        uint4 u[G];
#pragma unroll
        for (int k = 0; k < G; ++k) u[k] = nx[k];
        if (t + 1 < steps) { ldu<T, true, true>(base, p, n, nx); adv(); }
        // u[k]: row t*G + j of item gi + k  ->  area[j][gl + k]
#pragma unroll
        for (int k = 0; k < G; ++k) wx[j * 65 + gl + k] = u[k];
        wave_sync_lds();
        uint4 w[G];
#pragma unroll
        for (int r = 0; r < G; ++r) w[r] = wx[r * 65 + lane];
        wave_sync_lds();
        col_consume<T, BSWAP, MASKED, G>(w, acc, mk);
    }
    if constexpr (!MASKED) {
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k].count += (uint32_t)(R / S);
    }
}

// NumPy's sign on a zero min/max partial (ZT, a.zs = 1 min / 2 max): the
// sign of the last zero the output's column walk saw (col_track_zeros).
template <typename T>
__device__ __forceinline__ void zs_apply(const AxesArgs &a, pyas_partial &pp, uint32_t z) {
    if (!z) return;
    const double sg = (z & 1u) ? -0.0 : 0.0;
    if (a.zs == 1 && pp.min.f == 0.0) pp.min.f = sg;
    if (a.zs == 2 && pp.max.f == 0.0) pp.max.f = sg;
}

template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, bool CUT = false, bool ZT = false>
__device__ void dense_col(const AxesArgs &a, int64_t c, int64_t j, const uint8_t *base,
                          const MaskT<T> &mk, uint4 *stage, const CutBox *cb = nullptr,
                          const uint32_t *rmap = nullptr) {
    constexpr int ES = sizeof(T), N = 16 / ES;
    const AxesDense &d = a.d;
    const int IT = d.it, S = d.split;
    const int il = threadIdx.x & (IT - 1), sp = threadIdx.x / IT;
    const int64_t items = d.KO * (d.KI / N);
    const int64_t ob = sload(a.out_offsets + c);
    // aligned chunks: the ring walk (measured faster than the shuffled unit
    // exchange too); PYAS_COL_RING=0 builds the earlier walks
    constexpr bool ring = PYAS_COL_RING && AL;
    const bool units = !CUT && !ZT && !ring && SHUF && AL && col_units_ok<T>(d) &&
                       ldu_aligned<T, SHUF>(base, a.r.chunk_elems);
    // ZT: the splits' zero trackers meet here (max of the keys)
    __shared__ uint32_t zfold[ZT ? N * kBlock : 1];
    for (int64_t i0 = j * IT; i0 < items; i0 += d.bpc * IT) {   // block-uniform
        const int64_t i = i0 + il;
        TileAcc<T> acc[N];
        uint32_t zt[N];
#pragma unroll
        for (int k = 0; k < N; ++k) { acc[k].init(); zt[k] = 0; }
        if constexpr (ZT) {   // one lane per column (S == 1): the compare-and-select tracker
            if (S == 1) {
#pragma unroll
                for (int k = 0; k < N; ++k) zt[k] = 1u;
            }
        }
        if constexpr (ring) {
            if (i < items && sp < S && sp < d.RO * d.RI) {
                if constexpr (ZT) {
                    if (S == 1) col_rows_ring<T, SHUF, BSWAP, MASKED, CUT, 2>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
                    else col_rows_ring<T, SHUF, BSWAP, MASKED, CUT, 1>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
                } else {
                    col_rows_ring<T, SHUF, BSWAP, MASKED, CUT>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
                }
            }
        } else if constexpr (SHUF && sizeof(T) >= 4 && !CUT && !ZT) {
            if (units) {
                if (i < items && sp < S) col_rows_units<T, BSWAP, MASKED>(d, base, a.r.chunk_elems, i, sp, mk, acc, stage);
                __syncthreads();   // the exchange area is reused below
            } else if (i < items && sp < S && sp < d.RO * d.RI) {
                col_rows<T, SHUF, BSWAP, MASKED, AL>(d, base, a.r.chunk_elems, i, sp, mk, acc);
            }
        } else if (i < items && sp < S && sp < d.RO * d.RI) {
            if constexpr (ZT) {
                if (S == 1) col_rows<T, SHUF, BSWAP, MASKED, AL, CUT, 2>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
                else col_rows<T, SHUF, BSWAP, MASKED, AL, CUT, 1>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
            } else {
                col_rows<T, SHUF, BSWAP, MASKED, AL, CUT>(d, base, a.r.chunk_elems, i, sp, mk, acc, rmap, zt);
            }
        }
        if constexpr (ZT) {
            if (S == 1) {
#pragma unroll
                for (int k = 0; k < N; ++k) zt[k] = zt_final(zt[k]);
            } else {   // the latest zero over the splits (rows interleave: the largest key)
#pragma unroll
                for (int k = 0; k < N; ++k) zfold[k * kBlock + threadIdx.x] = zt[k];
                __syncthreads();
                if (sp == 0) {
                    for (int q = 1; q < S; ++q) {
#pragma unroll
                        for (int k = 0; k < N; ++k) {
                            const uint32_t o = zfold[k * kBlock + q * IT + il];
                            zt[k] = o > zt[k] ? o : zt[k];
                        }
                    }
                }
                __syncthreads();
            }
        }
        if constexpr (CUT) {
            PYAS_MARK(3);
            // outputs inside the box only, each at its place in the cut
            // chunk's partial array (not a contiguous range: direct stores)
            if constexpr (N <= 4) {
                if (S > 1) fold_splits_n<T, N>(acc, S, IT, il, sp, stage);
            }
            CutWalk cw;
            cw.init(a, i * N);   // kept index ko * KI + v * N of the item's first output
#pragma unroll
            for (int k = 0; k < N; ++k) {
                if constexpr (N > 4) {
                    if (S > 1) fold_splits(acc[k], S, IT, il, sp);
                }
                if (sp == 0 && i < items) {
                    const int64_t o = cw.out(a, *cb);
                    if (o >= 0) {
                        pyas_partial pp;
                        tile_store_lane(acc[k], &pp);
                        if constexpr (ZT) zs_apply<T>(a, pp, zt[k]);
                        put_out<T>(a, ob + o, pp);
                    }
                }
                cw.step(a);
            }
            PYAS_MARK(4);
        } else if constexpr (N <= 4) {
            // Stage the pass's IT*N partials (<= 32 KiB) in LDS, then write
            // them as consecutive 16-B stores (a lane's own N partials are
            // 32*N bytes apart from its neighbours').  The split fold uses
            // the same LDS first (fold_lds_bytes <= 32 KiB for N <= 4).
            static_assert(fold_lds_bytes<T, N>() <= kBlock * 4 * 2 * 16, "fold scratch exceeds the stage");
            if (S > 1) fold_splits_n<T, N>(acc, S, IT, il, sp, stage);
#pragma unroll
            for (int k = 0; k < N; ++k) {
                if (sp == 0) {
                    pyas_partial pp;
                    tile_store_lane(acc[k], &pp);
                    if constexpr (ZT) zs_apply<T>(a, pp, zt[k]);
                    stage_put<T>(a, stage, il * N + k, pp);
                }
            }
            __syncthreads();
            stage_flush<T>(a, stage, ob + i0 * N, ((items - i0 < IT) ? items - i0 : IT) * N, threadIdx.x, kBlock);
            __syncthreads();
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                if (S > 1) fold_splits(acc[k], S, IT, il, sp);
                if (sp == 0 && i < items) {
                    pyas_partial pp;
                    tile_store_lane(acc[k], &pp);
                    if constexpr (ZT) zs_apply<T>(a, pp, zt[k]);
                    put_out<T>(a, ob + i * N + k, pp);
                }
            }
        }
    }
}

// U units of VPL vectors into acc, the elements of unit u selected by bits
// ub[u] (bit e = element e of the unit): a cut chunk's row layouts.
template <typename T, bool BSWAP, int MASKED, int U, int VPL>
__device__ __forceinline__ void consume_units_p(const uint4 *w, const uint32_t *ub, TileAcc<T> &acc,
                                                const MaskT<T> &mk) {
    constexpr int N = 16 / sizeof(T);
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
            T x[N];
            unpack16<T, BSWAP>(w[u * VPL + v], x);
            bad |= acc.template add_pred<N, MASKED, 1>(x, ub[u] >> (v * N), mk);
        }
    }
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                T x[N];
                unpack16<T, BSWAP>(w[u * VPL + v], x);
#pragma unroll
                for (int t = 0; t < N; ++t)
                    if ((ub[u] >> (v * N + t)) & 1u) acc.template check_nan<1>(&x[t]);
            }
        }
    }
}

template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, int UO, bool CUT = false>
__device__ void dense_row(const AxesArgs &a, int64_t c, int64_t j, const uint8_t *base,
                          const MaskT<T> &mk, const CutBox *cb = nullptr, const uint32_t *rmap = nullptr) {
    const int64_t n = a.r.chunk_elems;
    constexpr int ES = sizeof(T), N = 16 / ES, VPL = Unit<T, SHUF>::VPL;
    constexpr int NU = N * VPL;                      // elements per load unit
    const AxesDense &d = a.d;
    const int G = d.group, P = kWave / G;
    const int lane = threadIdx.x & (kWave - 1), gl = lane & (G - 1), pg = lane / G;
    const int64_t VG = d.RI / N / VPL / G;           // load units per lane per run
    const int64_t Q = d.RO * VG;                     // load units per lane per output
    const int64_t wave = j * (kBlock / kWave) + threadIdx.x / kWave;
    const int64_t nwaves = d.bpc * (kBlock / kWave);
    const int64_t vstep = (int64_t)G * N * VPL * ES;             // bytes (plain layout)
    const int64_t wrap = (d.KO - 1) * d.RI * ES;                 // next run of the output
    const int64_t ob = sload(a.out_offsets + c);
    for (int64_t o0 = wave * P * UO; o0 < d.KO; o0 += nwaves * P * UO) {   // wave-uniform
        TileAcc<T> acc[UO];
#pragma unroll
        for (int u = 0; u < UO; ++u) acc[u].init();
        if constexpr (UO > 1) {
            // one unit per lane per output (RO == 1, RI == G*N*VPL): UO outputs in flight
            uint4 w[UO][VPL];
#pragma unroll
            for (int u = 0; u < UO; ++u) {
                const int64_t o = o0 + u * P + pg;
                if (o < d.KO) ldu<T, SHUF, AL>(base, base + (o * d.RI + gl * N * VPL) * ES, n, w[u]);
            }
            uint32_t ub = 0;
            if constexpr (CUT) ub = cut_bits(rmap, (int64_t)gl * NU, NU);
#pragma unroll
            for (int u = 0; u < UO; ++u) {
                const int64_t o = o0 + u * P + pg;
                if (o < d.KO) {
                    if constexpr (CUT) {
                        consume_units_p<T, BSWAP, MASKED, 1, VPL>(w[u], &ub, acc[u], mk);
                    } else {
                        consume16_u<T, BSWAP, MASKED, false, VPL>(w[u], acc[u], mk);
                        if constexpr (!MASKED) acc[u].count += N * VPL;
                    }
                }
            }
        } else {
            const int64_t o = o0 + pg;
            if (o < d.KO) {
                const uint8_t *p = base + (o * d.RI + gl * N * VPL) * ES;
                int64_t vc = 0, ro = 0;
                auto next = [&]() {
                    p += vstep;
                    if (++vc == VG) { vc = 0; ++ro; p += wrap; }
                };
                // units in flight: 4 plain vectors, or 2 (f32) / 1 (f64) shuffled units
                constexpr int U = VPL == 1 ? 4 : (VPL >= 8 ? 1 : 8 / VPL);
                int64_t t = 0;
                for (; t + U <= Q; t += U) {
                    uint4 w[U * VPL];
                    uint32_t ub[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if constexpr (CUT) ub[u] = cut_bits(rmap, ro * d.RI + (vc * G + gl) * NU, NU);
                        ldu<T, SHUF, AL>(base, p, n, w + u * VPL);
                        next();
                    }
                    if constexpr (CUT) consume_units_p<T, BSWAP, MASKED, U, VPL>(w, ub, acc[0], mk);
                    else consume16_u<T, BSWAP, MASKED, false, U * VPL>(w, acc[0], mk);
                }
                for (; t < Q; ++t) {
                    uint4 w[VPL];
                    uint32_t ub = 0;
                    if constexpr (CUT) ub = cut_bits(rmap, ro * d.RI + (vc * G + gl) * NU, NU);
                    ldu<T, SHUF, AL>(base, p, n, w);
                    next();
                    if constexpr (CUT) consume_units_p<T, BSWAP, MASKED, 1, VPL>(w, &ub, acc[0], mk);
                    else consume16_u<T, BSWAP, MASKED, false, VPL>(w, acc[0], mk);
                }
                if constexpr (!MASKED && !CUT) acc[0].count += (uint32_t)(Q * N * VPL);
            }
        }
#pragma unroll
        for (int u = 0; u < UO; ++u) {
            uint32_t cnt, nan;
            group_reduce(acc[u], G, cnt, nan);
            const int64_t o = o0 + u * P + pg;
            if (gl == 0 && o < d.KO) {
                int64_t oo = o;
                if constexpr (CUT) oo = cut_out(a, *cb, o);
                if (oo >= 0) {
                    pyas_partial pp;
                    store_group(acc[u], cnt, nan, &pp);
                    put_out<T>(a, ob + oo, pp);
                }
            }
        }
    }
}

// Row layout through LDS (RO == 1, KI == 1, runs of V <= 16 16-B vectors;
// e.g. axis (2,) of 64^3 f32): a wave loads kWave/H consecutive runs with
// coalesced 16-B loads (1 KiB per instruction), writes them to its own LDS
// tile (run stride V + 1 vectors: b128 reads and writes are bank-conflict
// free), then H lanes per output fold the run from LDS.  No butterfly for
// H == 1, log2(H) DPP steps otherwise.  The next tile's loads are issued before
// the current tile is folded.
constexpr int kRowLdsStride = 17;   // 16-B vectors per LDS run (V <= 16, + 1 pad)


// ZT (a.zs: 1 min, 2 max; floats): each output row is ONE contiguous NumPy
// call over the box's run along the innermost dim (storage.py:99-100; the
// reduced group is that dim alone when the chunk is cut).  A row whose
// min/max is a zero keys NumPy's winning zero from the tile still in LDS, as
// k_axes_fold_row does (the K1/W keys of tie_keys on bit masks of the call's
// positions, row_zs_masks): the last remainder zero if any, else the later of
// the last seed/top-lane zero and, unless the seed is a zero, the last zero of
// the lowest lane-rank class holding one.  Its sign goes into the record.
// Zero-free tiles cost one ballot.
__device__ __forceinline__ int msb64(uint64_t v) { return 63 - __builtin_clzll(v); }   // v != 0
constexpr int kRowZsRank = 4 + 64;        // then each position's lane rank, one byte each (255: not a lane)
constexpr int kRowZsWords = kRowZsRank + 8;   // rem, top, vec, box run, the rank classes, the ranks

// The masks ZT reads (LDS, zm[kRowZsWords]) for a call of L positions e
// (e = 0 the seed, then m = L - 1 elements: the first nv in t.lanes lanes, the
// rest remainder): built by wave 0 with ballots, once per workgroup.
__device__ __forceinline__ void row_zs_masks(const TieRule &t, int L, uint64_t *zm) {
    if (threadIdx.x >= kWave) return;
    const int e = threadIdx.x, lanes = t.lanes;
    const int m = L - 1, nv = m - m % lanes;
    const bool vec = e >= 1 && e <= nv;
    const int rk = vec ? (int)t.rank[(e - 1) % lanes] : -1;
    const uint64_t rem = __ballot(e > nv && e < L), top = __ballot(vec && rk == 0), vm = __ballot(vec);
    const uint64_t run = __ballot(e < L);
    for (int k = 0; k < lanes && k < 64; ++k) {
        const uint64_t cm = __ballot(rk == k);
        if (e == 0) zm[4 + k] = cm;
    }
    reinterpret_cast<uint8_t *>(zm + kRowZsRank)[e] = vec ? (uint8_t)rk : (uint8_t)255;
    if (e == 0) {
        zm[0] = rem;
        zm[1] = top;
        zm[2] = vm;
        zm[3] = run;
    }
}

// The winning zero of a row call (box positions Z, bit e = position e).
// A few lane zeros: their ranks from the per-position byte table, the loads
// independent (at 2 % zeros a zero row holds one or two, and the class
// search below waited on one LDS mask per class until the zero's class);
// more: the class search, which then stops early.  (Round 6 measured a
// table pick from lane-class sets -- two LDS lookups -- slower than the
// search: 1.40 vs 1.20-1.32 ms on the C3 slab (2,), profiles/r06/zeros.)
__device__ __forceinline__ int row_zs_pick(uint64_t Z, const uint64_t *zm, int lanes) {
    const uint64_t zr = Z & zm[0];
    if (zr) return msb64(zr);
    const uint64_t sig = Z & (zm[1] | 1u);
    const int e1 = sig ? msb64(sig) : -1;
    int ew = -1;
    const uint64_t Zv = Z & zm[2];   // the zeros in the lanes
    if (!(Z & 1u) && Zv) {
        if (__builtin_popcountll(Zv) <= 8) {
            // latest first, strictly lower rank replaces: the last zero of the lowest rank
            const uint8_t *zr = reinterpret_cast<const uint8_t *>(zm + kRowZsRank);
            uint32_t best = 256u;
            for (uint64_t b = Zv; b;) {
                const int e = msb64(b);
                b &= ~(1ull << e);
                const uint32_t r = zr[e];
                if (r < best) {
                    best = r;
                    ew = e;
                }
            }
        } else {
            for (int k = 0; k < lanes; ++k) {
                const uint64_t cz = Z & zm[4 + k];
                if (cz) {
                    ew = msb64(cz);
                    break;
                }
            }
        }
    }
    return ew > e1 ? ew : e1;
}

template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, int H, bool CUT = false, bool ZT = false>
__device__ void dense_row_lds(const AxesArgs &a, int64_t c, int64_t j, const uint8_t *base,
                              const MaskT<T> &mk, uint4 *tile, const CutBox *cb = nullptr,
                              const uint32_t *rmap = nullptr, const uint64_t *zm = nullptr, int zs0 = 0) {
    const int64_t n = a.r.chunk_elems;
    constexpr int ES = sizeof(T), N = 16 / ES, RPW = kWave / H, VPL = Unit<T, SHUF>::VPL;
    // load units per lane per tile (64 * UL * VPL >= the tile's RPW * 16 vectors)
    constexpr int UL = 16 / H / VPL > 0 ? 16 / H / VPL : 1;
    const AxesDense &d = a.d;
    const int V = (int)(d.RI / N);                  // vectors per run, V % H == 0, V % VPL == 0
    const int VH = V / H;                           // vectors per lane
    const int lane = threadIdx.x & (kWave - 1), r = lane / H, h = lane - r * H;
    uint4 *t = tile + (threadIdx.x / kWave) * RPW * kRowLdsStride;
    const int64_t wave = j * (kBlock / kWave) + threadIdx.x / kWave;
    const int64_t nwaves = d.bpc * (kBlock / kWave);
    const int64_t ob = sload(a.out_offsets + c);
    // tile unit q = u * kWave + lane: vectors q*VPL .. +VPL-1, in run q*VPL / V
    int lidx[UL];   // the unit's place in the wave's LDS tile (run q / V, vector q % V)
#pragma unroll
    for (int u = 0; u < UL; ++u) {
        const int q = (u * kWave + lane) * VPL, lr = q / V;
        lidx[u] = lr * kRowLdsStride + (q - lr * V);
    }
    uint4 w[UL][VPL];
    auto load = [&](int64_t o0) {
        const int64_t nvec = (d.KO - o0 < RPW ? d.KO - o0 : RPW) * V;
        const uint8_t *src = base + o0 * d.RI * ES;
#pragma unroll
        for (int u = 0; u < UL; ++u)
            if ((u * kWave + lane) * VPL < nvec)
                ldu<T, SHUF, AL>(base, src + (int64_t)(u * kWave + lane) * VPL * 16, n, w[u]);
    };
    // CUT: this lane's VH * N run positions inside the box (the same for
    // every row: RO == 1), read from the map once
    uint64_t lbits = 0;
    if constexpr (CUT) {
        const int64_t p0 = (int64_t)h * VH * N;
        const int nb = VH * N;
        lbits = cut_bits(rmap, p0, nb < 32 ? nb : 32);
        if (nb > 32) lbits |= (uint64_t)cut_bits(rmap, p0 + 32, nb - 32 < 32 ? nb - 32 : 32) << 32;
    }
    int64_t o0 = wave * RPW;
    if (o0 < d.KO) load(o0);
    for (; o0 < d.KO; o0 += nwaves * RPW) {   // wave-uniform
        const int64_t nvec = (d.KO - o0 < RPW ? d.KO - o0 : RPW) * V;
#pragma unroll
        for (int u = 0; u < UL; ++u)
            if ((u * kWave + lane) * VPL < nvec) {
#pragma unroll
                for (int i = 0; i < VPL; ++i) t[lidx[u] + i] = w[u][i];
            }
        wave_sync_lds();
        if (o0 + nwaves * RPW < d.KO) load(o0 + nwaves * RPW);
        TileAcc<T> acc;
        acc.init();
        const uint4 *row = t + r * kRowLdsStride + h * VH;
        // ZT: the lane's zero bits (its first element highest), gathered as
        // the fold reads the tile -- a second pass over the tile held
        // registers next to the loads in flight (a wave per SIMD: 1.28 ms vs
        // 0.92) -- and only for vectors after which the lane's running
        // min/max is exactly zero: before that every element was of one sign
        // (no zero), and once it is past zero the row is not a zero row.
        // Zero-free rows pay a compare and a branch per vector.
        using ZW = typename std::conditional<H == 1, uint64_t, uint32_t>::type;
        ZW zl = 0;
        for (int i = 0; i < VH; ++i) {
            T x[N];
            unpack16<T, BSWAP>(row[i], x);
            if constexpr (CUT) {   // the run's elements inside the box (RO == 1: position = element)
                const uint32_t b = (uint32_t)(lbits >> (i * N)) & (uint32_t)((1ull << N) - 1);
                if (acc.template add_pred<N, MASKED, 1>(x, b, mk)) {
#pragma unroll
                    for (int q = 0; q < N; ++q)
                        if ((b >> q) & 1u) acc.template check_nan<1>(&x[q]);
                }
            } else {
                acc.template add_n<N, MASKED, false>(x, mk);
            }
            if constexpr (ZT) {
                const T ext = a.zs == 1 ? acc.mn : acc.mx;
                if (ext == (T)0) {
                    uint32_t b = 0;
#pragma unroll
                    for (int k = 0; k < N; ++k) b |= (x[k] == (T)0 ? 1u : 0u) << (N - 1 - k);
                    zl |= (ZW)b << (VH * N - N * (i + 1));
                }
            }
        }
        if constexpr (!MASKED && !CUT) acc.count += (uint32_t)(VH * N);
        uint32_t cnt, nan;
        group_reduce(acc, H, cnt, nan);
        int zsg = -1;   // ZT: the row's NumPy zero sign bit (-1: not a zero row)
        if constexpr (ZT) {
            const T v = a.zs == 1 ? acc.mn : acc.mx;
            const bool zrow = o0 + r < d.KO && cnt > 0 && !nan && v == (T)0;   // the row's H lanes agree
            if (__ballot(zrow)) {
                uint64_t Z = 0;
                if (zrow) {   // the lane's zero bits reversed to element order at its offset
                    const int J = VH * N;
                    if constexpr (H == 1) Z = __builtin_bitreverse64(zl) >> (64 - J);
                    else Z = (uint64_t)(__builtin_bitreverse32(zl) >> (32 - J)) << (h * J);
                }
#pragma unroll
                for (int mm = H / 2; mm >= 1; mm >>= 1) Z |= shfl_xor(Z, mm);
                if (zrow && h == 0) {
                    // the box's run along the innermost dim: positions from its start zs0
                    const int e = row_zs_pick((Z >> zs0) & zm[3], zm, a.t.lanes);
                    if (e >= 0) {
                        const int x = zs0 + e;
                        T xe[N];
                        unpack16<T, BSWAP>(t[r * kRowLdsStride + x / N], xe);
                        T we = xe[0];
#pragma unroll
                        for (int k = 1; k < N; ++k) we = (x % N) == k ? xe[k] : we;
                        zsg = __builtin_signbit(we) ? 1 : 0;
                    }
                }
            }
        }
        auto row_out = [&](pyas_partial &pp) {
            store_group(acc, cnt, nan, &pp);
            if constexpr (ZT) {
                if (zsg >= 0) {
                    const T zz = zsg ? -(T)0 : (T)0;
                    if (a.zs == 1) TT<T>::put(pp.min, zz);
                    else TT<T>::put(pp.max, zz);
                }
            }
        };
        if constexpr (CUT) {   // rows inside the box only, at their place in the cut chunk's array
            if (h == 0 && o0 + r < d.KO) {
                const int64_t oo = cut_out(a, *cb, o0 + r);
                if (oo >= 0) {
                    pyas_partial pp;
                    row_out(pp);
                    put_out<T>(a, ob + oo, pp);
                }
            }
            wave_sync_lds();   // the tile's reads before the next tile's writes
            continue;
        }
        // the tile's partials go out as consecutive 16-B non-temporal stores,
        // staged in the (now read) tile area, instead of store_group's
        // per-lane 32-B writes that half fill each store instruction's span
        // (C3 (2,): plain unchanged at 0.85 ms, shuffled 0.85 -> 0.84 ms)
        wave_sync_lds();
        if (h == 0) {
            pyas_partial pp;
            row_out(pp);
            stage_put<T>(a, t, r, pp);
        }
        wave_sync_lds();
        stage_flush<T>(a, t, ob + o0, nvec / V, lane, kWave);
        wave_sync_lds();
    }
}

// Which kernel owns chunk c: the dense one when the chunk is fully selected,
// or (a.cuts) a box covering at least half of it.
__device__ __forceinline__ bool dense_owns(const AxesArgs &a, const Sel &s) {
    return a.d.mode != 0 && (chunk_is_full(s, a.r.shape, a.r.ndim) || cut_eligible(a, s));
}

// ZS (a.zs set; float types, MODE 1 or >= 4; kernels of their own, so the
// keying's registers never cost the other launches occupancy): the walk keys
// NumPy's sign of a zero min/max of every chunk it takes, whole or cut.
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE, bool CUTS, bool ZS = false>
__device__ __forceinline__ void axes_dense_body(const AxesArgs &a) {
    static_assert(!ZS || (CUTS && TT<T>::kind == 0 && (MODE == 1 || MODE >= 4)), "zero-sign keying: float column/LDS rows");
    const int64_t c = blockIdx.x / a.d.bpc;
    const int64_t j = blockIdx.x - c * a.d.bpc;
    const ReduceArgs &r = a.r;
    Sel s;
    load_sel(s, r.sel, c, r.ndim, r.shape);
    if (!dense_owns(a, s)) return;   // the generic kernel takes this chunk
    const uint8_t *base = r.data + r.offsets[c];
    MaskT<T> mk;
    mk.init(r.mask);
    const bool al = MODE == 1 ? ldv_aligned<T, SHUF>(base, r.chunk_elems) : ldu_aligned<T, SHUF>(base, r.chunk_elems);
    // LDS: dense_col's store stage (32 KiB; also the shuffled unit exchange
    // area, col_units_lds <= 2080 vectors, and the split-fold scratch), or
    // the LDS row layout's tile; CUTS: the cut chunks' reduced-position map
    constexpr int H = MODE == 4 ? 1 : MODE == 5 ? 2 : 4;
    constexpr int kLds = MODE == 1 ? (sizeof(T) >= 4 ? (kBlock * 8 > col_units_lds<T>() ? kBlock * 8 : col_units_lds<T>()) : 1)
                        : MODE >= 4 ? (kBlock / kWave) * (kWave / H) * kRowLdsStride : 1;
    __shared__ uint4 lds[kLds];
    // ZS row layouts: the masks of the row call's positions (row_zs_masks)
    constexpr bool kRowZs = ZS && MODE >= 4;
    __shared__ uint64_t zm[kRowZs ? kRowZsWords : 1];
    if constexpr (CUTS) {
        // a cut chunk (a.cuts launches): read as its whole chunk, the box
        // applied through the reduced-position map and the output remap
        if (!chunk_is_full(s, r.shape, r.ndim)) {
            __shared__ uint32_t cmap[kCutMapWords + 1];
            CutBox cb;
            PYAS_MARK(1);
            cut_box(a, s, cb);
            cut_map(a, cb, a.d.RO * a.d.RI, cmap);
            int zs0 = 0;   // kRowZs: the box's run along the innermost dim (static indices:
            int zL = 1;    // a runtime index would put the box in scratch memory)
            if constexpr (kRowZs) {
#pragma unroll
                for (int dd = 0; dd < PYAS_MAX_DIMS; ++dd) {
                    if (dd == r.ndim - 1) {
                        zs0 = cb.lo[dd];
                        zL = cb.hi[dd] - cb.lo[dd];
                    }
                }
                row_zs_masks(a.t, zL, zm);
                __syncthreads();
            }
            PYAS_MARK(2);
            if constexpr (MODE == 1) {
                if (al) dense_col<T, SHUF, BSWAP, MASKED, true, true, ZS>(a, c, j, base, mk, lds, &cb, cmap);
                else dense_col<T, SHUF, BSWAP, MASKED, false, true, ZS>(a, c, j, base, mk, lds, &cb, cmap);
            } else if constexpr (MODE >= 4) {
                if (al) dense_row_lds<T, SHUF, BSWAP, MASKED, true, H, true, ZS>(a, c, j, base, mk, lds, &cb, cmap, zm, zs0);
                else dense_row_lds<T, SHUF, BSWAP, MASKED, false, H, true, ZS>(a, c, j, base, mk, lds, &cb, cmap, zm, zs0);
            } else {
                constexpr int UO = MODE == 2 ? 1 : 4;
                if (al) dense_row<T, SHUF, BSWAP, MASKED, true, UO, true>(a, c, j, base, mk, &cb, cmap);
                else dense_row<T, SHUF, BSWAP, MASKED, false, UO, true>(a, c, j, base, mk, &cb, cmap);
            }
            PYAS_MARK(5);
            return;
        }
    }
    if constexpr (MODE == 1) {
        if (al) dense_col<T, SHUF, BSWAP, MASKED, true, false, ZS>(a, c, j, base, mk, lds);
        else dense_col<T, SHUF, BSWAP, MASKED, false, false, ZS>(a, c, j, base, mk, lds);
    } else if constexpr (MODE >= 4) {
        if constexpr (kRowZs) {
            row_zs_masks(a.t, (int)a.d.RI, zm);
            __syncthreads();
        }
        if (al) dense_row_lds<T, SHUF, BSWAP, MASKED, true, H, false, ZS>(a, c, j, base, mk, lds, nullptr, nullptr, zm);
        else dense_row_lds<T, SHUF, BSWAP, MASKED, false, H, false, ZS>(a, c, j, base, mk, lds, nullptr, nullptr, zm);
    } else if constexpr (MODE == 2) {
        if (al) dense_row<T, SHUF, BSWAP, MASKED, true, 1>(a, c, j, base, mk);
        else dense_row<T, SHUF, BSWAP, MASKED, false, 1>(a, c, j, base, mk);
    } else {
        if (al) dense_row<T, SHUF, BSWAP, MASKED, true, 4>(a, c, j, base, mk);
        else dense_row<T, SHUF, BSWAP, MASKED, false, 4>(a, c, j, base, mk);
    }
}

// One kernel per layout family, so each carries its own occupancy floor.
// The *_cut kernels also take the batch's cut chunks (AxesArgs::cuts).
#ifndef PYAS_LDS_CUT_WAVES
#define PYAS_LDS_CUT_WAVES 4   // the cut path must not cost whole chunks a wave: 137 VGPRs (3 per SIMD)
#endif
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_COL_WAVES) void k_axes_dense_col(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, false>(a);
}
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_ROW_WAVES) void k_axes_dense_row(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, false>(a);
}
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_LDS_WAVES) void k_axes_dense_lds(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, false>(a);
}
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_COL_WAVES) void k_axes_dense_col_cut(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, true>(a);
}
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_ROW_WAVES) void k_axes_dense_row_cut(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, true>(a);
}
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_LDS_CUT_WAVES) void k_axes_dense_lds_cut(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, true>(a);
}
// Zero-sign keying (a.zs): column and LDS row layouts, whole and cut chunks
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_COL_WAVES) void k_axes_dense_col_zs(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, true, true>(a);
}
#ifndef PYAS_LDS_ZS_WAVES
#define PYAS_LDS_ZS_WAVES 4   // the row kernel is latency-bound: 3 waves cost C3 [1:1023]^3 (2,) min 0.92 -> 1.28 ms
#endif
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_LDS_ZS_WAVES) void k_axes_dense_lds_zs(AxesArgs a) {
    axes_dense_body<T, SHUF, BSWAP, MASKED, MODE, true, true>(a);
}

// Whole-chunk box query, column layout, chunk layers folded in the kernel
// (pyas_reduce_axes_grid).  Block (col, j) owns the kept-dims chunk column
// `col` and items j, j + bpc, ... of it; for each layer (the column's chunks
// along the reduced dims, in C order) it runs dense_col's pass and merges
// the per-chunk partial (tile_store_lane, then k_combine_grid's merge with
// the same rounding) into a running WAcc per output.  The arithmetic is
// k_axes_dense + k_combine_grid's, operation for operation, so the result is
// bit-identical; the per-chunk partial arrays are never written.
template <typename T, bool SHUF, bool BSWAP, int MASKED>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_FOLD_COL_WAVES) void k_axes_fold(AxesArgs a, FoldGrid g) {
    constexpr int N = 16 / sizeof(T);
    const AxesDense &d = a.d;
    const ReduceArgs &r = a.r;
    const int64_t col = blockIdx.x / d.bpc;
    const int64_t j = blockIdx.x - col * d.bpc;
    const uint32_t red = a.axes;
    int64_t ac[PYAS_MAX_DIMS], gstride[PYAS_MAX_DIMS];
    int64_t rest = col, st = 1, nk = 0;
#pragma unroll
    for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
        ac[dd] = 0;
        gstride[dd] = st;
        if (dd < r.ndim) {
            st *= g.n_coords[dd];
            if (!((red >> dd) & 1u)) {
                const int64_t q = rest / g.n_coords[dd];
                ac[dd] = rest - q * g.n_coords[dd];
                rest = q;
                nk += ac[dd] * gstride[dd];
            }
        }
    }
    MaskT<T> mk;
    mk.init(r.mask);
    const int IT = d.it, S = d.split;
    const int il = threadIdx.x & (IT - 1), sp = threadIdx.x / IT;
    const int64_t items = d.KO * (d.KI / N);
    const bool round = (g.flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    // split-fold area; for shuffled chunks also the unit exchange area
    // (col_rows_units), the two separated by barriers
    constexpr int kFoldLds = fold_lds_bytes<T, N>() > col_units_lds<T>() * 16 ? fold_lds_bytes<T, N>()
                                                                               : col_units_lds<T>() * 16;
    __shared__ __attribute__((aligned(16))) uint8_t fold_lds[kFoldLds];
    auto layer_base = [&](int64_t l) {
        int64_t n = nk, rr = l;
#pragma unroll
        for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
            if (dd < r.ndim && ((red >> dd) & 1u)) {
                const int64_t q = rr / g.n_coords[dd];
                n += (rr - q * g.n_coords[dd]) * gstride[dd];
                rr = q;
            }
        }
        return r.data + sload(r.offsets + n);
    };
    // Pipelined walk (block-uniform choice): every lane has the same rows per
    // layer, a multiple of U, and every layer is aligned, so the walk is
    // one stream of U-row steps whose next step's loads -- across a layer
    // boundary too -- are in flight while the current step is consumed.
    constexpr int U = PYAS_COL_U, ES = sizeof(T);
    const int64_t R = d.RO * d.RI;
    bool pipe = R % S == 0 && (R / S) % U == 0;
    for (int64_t l = 0; pipe && l < g.n_layers; ++l) pipe = ldv_aligned<T, SHUF>(layer_base(l), r.chunk_elems);
    // shuffled chunks outside the pipelined walk: unit loads + LDS exchange
    // per layer when the geometry admits it (measured on C3 (0,)/(1,): the
    // pipelined dword-piece walk 0.78/0.90 ms, the unit exchange 0.80-0.82/
    // 0.97-0.98 ms, so the pipeline wins where it applies)
    bool units = SHUF && !pipe && col_units_ok<T>(d);
    for (int64_t l = 0; units && l < g.n_layers; ++l) units = ldu_aligned<T, SHUF>(layer_base(l), r.chunk_elems);
    const int64_t KIV = d.KI / N, sRO = d.KO * d.RI * d.KI;
    const int64_t dq = S / d.RI, dr = S - dq * d.RI;
    const int64_t step_off = (dq * sRO + dr * d.KI) * ES, wrap_off = (sRO - d.RI * d.KI) * ES;
    for (int64_t i0 = j * IT; i0 < items; i0 += d.bpc * IT) {   // block-uniform
        const int64_t i = i0 + il;
        WAcc<T> w[N];
#pragma unroll
        for (int k = 0; k < N; ++k) w[k].init();
        const bool act = i < items && sp < S && sp < R;
        if (pipe) {
            const int64_t ntu = R / S;
            const int64_t ko = i / KIV, v = i - ko * KIV, ro0 = sp / d.RI, ri0 = sp - ro0 * d.RI;
            const int64_t off0 = ((ro0 * d.KO + ko) * d.RI * d.KI + ri0 * d.KI + v * N) * ES;
            int64_t off = off0, ri = ri0;
            const uint8_t *b = layer_base(0);
            uint4 nx[U];
            auto fetch = [&]() {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    nx[u] = ldv<T, SHUF, true>(b, b + off, r.chunk_elems);
                    off += step_off;
                    ri += dr;
                    if (ri >= d.RI) { ri -= d.RI; off += wrap_off; }
                }
            };
            if (act) fetch();
            for (int64_t l = 0; l < g.n_layers; ++l) {
                TileAcc<T> acc[N];
#pragma unroll
                for (int k = 0; k < N; ++k) acc[k].init();
                for (int64_t t = 0; t < ntu; t += U) {
                    uint4 cur[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) cur[u] = nx[u];
                    if (act) {
                        if (t + U < ntu) {
                            fetch();
                        } else if (l + 1 < g.n_layers) {   // the next layer's first step
                            b = layer_base(l + 1);
                            off = off0;
                            ri = ri0;
                            fetch();
                        }
                        col_consume<T, BSWAP, MASKED, U>(cur, acc, mk);
                    }
                }
                if constexpr (!MASKED) {
                    if (act) {
#pragma unroll
                        for (int k = 0; k < N; ++k) acc[k].count += (uint32_t)ntu;
                    }
                }
                if (S > 1) fold_splits_n<T, N>(acc, S, IT, il, sp, fold_lds);
                if (sp == 0) {
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        pyas_partial pp;
                        tile_store_lane(acc[k], &pp);
                        merge(w[k], pp, round);
                    }
                }
            }
        } else {
            for (int64_t l = 0; l < g.n_layers; ++l) {
                const uint8_t *base = layer_base(l);
                TileAcc<T> acc[N];
#pragma unroll
                for (int k = 0; k < N; ++k) acc[k].init();
                if (units) {
                    if constexpr (SHUF && sizeof(T) >= 4) {
                        if (act)
                            col_rows_units<T, BSWAP, MASKED>(d, base, r.chunk_elems, i, sp, mk, acc,
                                                             reinterpret_cast<uint4 *>(fold_lds));
                    }
                    __syncthreads();   // the exchange area is the split-fold area
                } else if (act) {
                    if (ldv_aligned<T, SHUF>(base, r.chunk_elems))
                        col_rows<T, SHUF, BSWAP, MASKED, true>(d, base, r.chunk_elems, i, sp, mk, acc);
                    else
                        col_rows<T, SHUF, BSWAP, MASKED, false>(d, base, r.chunk_elems, i, sp, mk, acc);
                }
                if (S > 1) fold_splits_n<T, N>(acc, S, IT, il, sp, fold_lds);
                if (sp == 0) {
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        pyas_partial pp;
                        tile_store_lane(acc[k], &pp);
                        merge(w[k], pp, round);
                    }
                }
            }
        }
        if (sp == 0 && i < items) {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                int64_t loc = i * N + k, f = 0;   // kept-dims index in the chunk -> final element
#pragma unroll
                for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
                    if (dd < r.ndim && !((red >> dd) & 1u)) {
                        const int64_t q = loc / r.shape[dd];
                        f += (ac[dd] * r.shape[dd] + (loc - q * r.shape[dd])) * g.ostride[dd];
                        loc = q;
                    }
                }
                store_wpartial(a.out + f, w[k]);
            }
        }
    }
}

#ifndef PYAS_LEAN_DEPTH
#define PYAS_LEAN_DEPTH 2   // 4-row load groups in flight per lane (k_axes_fold_lean)
#endif
#ifndef PYAS_LEAN_WAVES
#define PYAS_LEAN_WAVES 4   // occupancy floor: <= 128 VGPRs, 16 waves per CU
#endif

// One lane's row walk over a run of layers (chunks) that share one column
// geometry: groups of 4 rows (the two-step path's PYAS_COL_U grouping, so
// the sums are bit-identical), DEPTH groups of 16-B loads in flight while
// the oldest is consumed.  The fetch cursor runs ahead of the consume cursor
// across layer boundaries, so a layer's first loads are in flight while the
// previous layer's last group is summed.  The walk covers layers
// [l0, l0 + n_layers) at layer_base(l) + off0; when a layer's last group has
// been consumed, layer_end(cl, acc) runs (cl = layers done before it) with
// the layer's sum / min / max in acc[] (counts: masked mode counts per
// element; unmasked, the walk adds the layer's R rows first).
// NV > 1: the lane walks NV items at once (row-0 byte offsets offs[s],
// partials in acc[s * N ...]), so a wave's loads of one row cover NV KiB
// when its items are adjacent.
struct NoGroupHook {
    __device__ void operator()(const uint4 *) const {}
};

template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, int DEPTH, bool NT, int NV, typename LB,
          typename LE, typename OG = NoGroupHook>
__device__ __forceinline__ void col_walk_layers(const AxesDense &d, int64_t n, const int64_t *offs, int64_t l0,
                                                int64_t n_layers, const MaskT<T> &mk, const LB &layer_base,
                                                TileAcc<T> *acc, const LE &layer_end,
                                                const OG &on_group = OG{}) {
    constexpr int N = 16 / sizeof(T), ES = sizeof(T), U = 4;
    const int64_t R = d.RO * d.RI;                      // rows per layer, a multiple of U
    const int64_t step = d.KI * ES;                     // next ri
    const int64_t wrap = (d.KO * d.RI * d.KI - d.RI * d.KI) * ES;   // ri wrapped: next ro
    const int64_t gpl = R / U, total = n_layers * gpl;  // groups per layer, in all
    // fetch cursor
    const uint8_t *fb = layer_base(l0);
    int64_t foff = 0, fl = 0;   // row offset from the items' row 0
    int64_t fri = 0, fg = 0;
    auto fetch = [&](uint4 *buf) {   // buf[v * U + u]: item set v, row u of the group
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int v = 0; v < NV; ++v) buf[v * U + u] = ldv<T, SHUF, AL, NT>(fb, fb + offs[v] + foff, n);
            foff += step;
            if (++fri == d.RI) { fri = 0; foff += wrap; }
        }
        if (++fg == gpl) {   // next layer (wave-uniform)
            fg = 0;
            if (++fl < n_layers) {
                fb = layer_base(l0 + fl);
                foff = 0;
                fri = 0;
            }
        }
    };
    int64_t cg = 0, cl = 0;   // consumed groups of the current layer, consumed layers
    auto consume = [&](const uint4 *buf) {
#pragma unroll
        for (int v = 0; v < NV; ++v) col_consume<T, BSWAP, MASKED, U>(buf + v * U, acc + v * N, mk);
        on_group(buf);   // rows u = 0..U-1 of the group, in order (item set 0)
        if (++cg == gpl) {
            cg = 0;
            if constexpr (!MASKED) {
#pragma unroll
                for (int k = 0; k < NV * N; ++k) acc[k].count += (uint32_t)R;
            }
            layer_end(cl, acc);
            ++cl;
        }
    };
    uint4 buf[DEPTH][NV * U];
#pragma unroll
    for (int s = 0; s < DEPTH; ++s)
        if (s < total) fetch(buf[s]);
    for (int64_t t = 0; t < total; t += DEPTH) {   // wave-uniform
#pragma unroll
        for (int s = 0; s < DEPTH; ++s) {
            if (t + s < total) {
                uint4 cur[NV * U];
#pragma unroll
                for (int u = 0; u < NV * U; ++u) cur[u] = buf[s][u];
                if (t + s + DEPTH < total) fetch(buf[s]);
                consume(cur);
            }
        }
    }
}

// k_axes_fold_lean's walk over every layer of its column: each layer's
// partial is merged into w[] when its last group is consumed (tile_store_lane
// + merge, as k_combine_grid would).  With `sink` set, each layer's rounded
// sum is stored at sink[(layer - l0) * sstride + k * IB] instead of being
// added to w[k].sum (the second half of a split column, added in order by
// the first half's lane).
// ZS: zs[k] tracks output k's last zero in (layer, row) order: the word of
// that zero holding its sign bit, kZsNone while none (the elementwise rule
// both NumPy reductions follow when the innermost dim is kept;
// k_axes_fold_lean writes it to a zero min/max).
constexpr uint32_t kZsNone = 1u;   // no zero seen (a zero's sign word is 0 or 0x80000000)

template <typename T, bool SHUF, bool BSWAP, int MASKED, bool AL, int DEPTH, bool SINK, bool NT, bool ZS,
          typename LB>
__device__ __forceinline__ void lean_walk(const AxesDense &d, int64_t n, int64_t off0, int64_t l0,
                                          int64_t n_layers, bool round, const MaskT<T> &mk,
                                          const LB &layer_base, WAcc<T> *w,
                                          typename TT<T>::Acc *sink, int sstride, int IB, uint32_t *zs) {
    constexpr int N = 16 / sizeof(T);
    // acc[k]: the current layer's sum / min / max; its count and NaN flag run
    // over every layer (merge adds counts, and a NaN layer min/max stays NaN
    // through pmin/pmax).  A layer's sum is rounded and added to w[k].sum and
    // its min/max folded into w[k] with merge's pmin/pmax, in layer order; an
    // empty layer's +-inf (or integer extremes) leave w[k] unchanged, as
    // merge's count > 0 guard does.  (Fewer live registers than a full
    // TileAcc -> pyas_partial -> merge per layer, same results.)
    TileAcc<T> acc[N];
#pragma unroll
    for (int k = 0; k < N; ++k) acc[k].init();
    auto merge_layer = [&](int64_t cl, TileAcc<T> *ac) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            pyas_scalar s;
            TT<T>::put_acc(s, ac[k].sum);
            if constexpr (SINK) sink[cl * sstride + k * IB] = sum_of<T>(s, round);
            else w[k].sum += sum_of<T>(s, round);
            w[k].mn = pmin(w[k].mn, ac[k].mn);
            w[k].mx = pmax(w[k].mx, ac[k].mx);
            ac[k].sum = 0;
            ac[k].mn = TT<T>::highest();
            ac[k].mx = TT<T>::lowest();
        }
    };
    if constexpr (ZS) {
        // a zero's maskedness is one fact per query (value-based rules), so
        // the trackers take every zero; a masked zero never makes the min
        // or max a zero, and only a zero min/max reads them
        auto track = [&](const uint4 *buf) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                T x[N];
                unpack16<T, BSWAP>(buf[u], x);
#pragma unroll
                for (int k = 0; k < N; ++k) {   // a compare and a select per element
                    uint32_t hi;                   // the word holding the sign bit
                    if constexpr (sizeof(T) == 4) {
                        __builtin_memcpy(&hi, &x[k], 4);
                    } else {
                        uint64_t b;
                        __builtin_memcpy(&b, &x[k], 8);
                        hi = (uint32_t)(b >> 32);
                    }
                    zs[k] = x[k] == (T)0 ? hi : zs[k];
                }
            }
        };
        col_walk_layers<T, SHUF, BSWAP, MASKED, AL, DEPTH, NT, 1>(d, n, &off0, l0, n_layers, mk, layer_base, acc,
                                                                 merge_layer, track);
    } else {
        col_walk_layers<T, SHUF, BSWAP, MASKED, AL, DEPTH, NT, 1>(d, n, &off0, l0, n_layers, mk, layer_base, acc,
                                                                 merge_layer);
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        w[k].count = (int64_t)acc[k].count;   // host: n_layers * rows < 2^31
        if constexpr (TT<T>::kind == 0) {
            if (acc[k].nan) {
                w[k].mn = (T)__builtin_nan("");
                w[k].mx = w[k].mn;
            }
        }
    }
}

// Whole-chunk box query, column layout, one lane per item and no split of
// the reduced rows (dense_geometry's split == 1, rows per chunk a multiple
// of 4): the lean form of k_axes_fold.  No barrier inside the walk; each
// lane streams its item's rows through the layers of its column with
// PYAS_LEAN_DEPTH x 4 loads in flight, under 128 VGPRs (16 waves per CU;
// k_axes_fold carries 146-173 VGPRs, 12 waves, and folds its split rows
// through LDS behind a barrier per layer).
// g.lean == 2 splits each column's layers in two halves walked by two lanes
// of the block (twice the waves, each half as long: measured on C3 (0,)
// 6.1 -> 6.8 TB/s with tools/colwalk_probe.hip).  The second half stores
// its per-layer sums in LDS, and the first half's lane adds them after its
// own, in layer order, and folds in the second half's min/max (pmin/pmax,
// earlier half first), count and NaN.  Either way the arithmetic is
// k_axes_dense (split 1) + k_combine_grid's: bit-identical.
// ZS (g.zs = which: 1 min, 2 max; the host checks that both NumPy reductions
// are elementwise, pyas.h PYAS_FOLD_ZERO_SIGN_*): each lane also tracks its
// outputs' last zero, in layer order then row order, and a zero min/max of
// the result takes that zero's sign -- what storage.py:99-100 and
// active.py:594 return when every later zero wins -- so the zero-sign passes
// (pyas_tie_chunk_flags + pyas_tie_grid) need not re-read the chunks.
template <typename T, bool SHUF, bool BSWAP, int MASKED, bool ZS>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_LEAN_WAVES) void k_axes_fold_lean(AxesArgs a, FoldGrid g) {
    constexpr int N = 16 / sizeof(T), ES = sizeof(T), IB2 = kBlock / 2;
    using A = typename TT<T>::Acc;
    const AxesDense &d = a.d;
    const ReduceArgs &r = a.r;
    const int LS = g.lean;                             // 1 or 2 (host)
    const int IB = kBlock / LS;                        // items per block
    const int half = threadIdx.x / IB, il = threadIdx.x - half * IB;   // wave-uniform half
    const int64_t col = blockIdx.x / d.bpc;
    const int64_t j = blockIdx.x - col * d.bpc;
    const int64_t items = d.KO * (d.KI / N);
    const int64_t i = j * IB + il;
    const bool act = i < items;
    if (LS == 1 && !act) return;   // unsplit: no barrier below
    const uint32_t red = a.axes;
    int64_t ac[PYAS_MAX_DIMS], gstride[PYAS_MAX_DIMS];
    int64_t rest = col, st = 1, nk = 0;
#pragma unroll
    for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
        ac[dd] = 0;
        gstride[dd] = st;
        if (dd < r.ndim) {
            st *= g.n_coords[dd];
            if (!((red >> dd) & 1u)) {
                const int64_t q = rest / g.n_coords[dd];
                ac[dd] = rest - q * g.n_coords[dd];
                rest = q;
                nk += ac[dd] * gstride[dd];
            }
        }
    }
    auto layer_base = [&](int64_t l) {
        int64_t cn = nk, rr = l;
#pragma unroll
        for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
            if (dd < r.ndim && ((red >> dd) & 1u)) {
                const int64_t q = rr / g.n_coords[dd];
                cn += (rr - q * g.n_coords[dd]) * gstride[dd];
                rr = q;
            }
        }
        return r.data + sload(r.offsets + cn);
    };
    MaskT<T> mk;
    mk.init(r.mask);
    const bool round = (g.flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    const int64_t KIV = d.KI / N, ko = i / KIV, v = i - ko * KIV;
    const int64_t off0 = (ko * d.RI * d.KI + v * N) * ES;   // row 0 of item i
    bool al = true;   // block-uniform: every layer's plane pieces aligned
    for (int64_t l = 0; al && l < g.n_layers; ++l) al = ldv_aligned<T, SHUF>(layer_base(l), r.chunk_elems);
    const int64_t hA = LS == 2 ? (g.n_layers + 1) / 2 : g.n_layers;   // host: n_layers - hA <= kLeanMaxB
    const int64_t l0 = half ? hA : 0, nl = half ? g.n_layers - hA : hA;
    __shared__ A s_sum[kLeanMaxB * N * IB2];      // second half: per-layer sums [layer][k][item]
    __shared__ T s_mn[N * IB2], s_mx[N * IB2];
    __shared__ uint32_t s_cnt[N * IB2];
    __shared__ uint32_t s_zs[ZS ? N * IB2 : 1];
    A *sink = half ? s_sum + il : nullptr;
    WAcc<T> w[N];
    uint32_t zs[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        w[k].init();
        zs[k] = kZsNone;
    }
    // AL_ / NT_: compile-time aligned walk / non-temporal plane loads
    auto walk = [&](auto al_c, auto nt_c) {
        constexpr bool AL_ = decltype(al_c)::value, NT_ = decltype(nt_c)::value;
        constexpr int DEP = AL_ ? PYAS_LEAN_DEPTH : 1;
        if (half)
            lean_walk<T, SHUF, BSWAP, MASKED, AL_, DEP, true, NT_, ZS>(d, r.chunk_elems, off0, l0, nl, round,
                                                                     mk, layer_base, w, sink, N * IB, IB, zs);
        else
            lean_walk<T, SHUF, BSWAP, MASKED, AL_, DEP, false, NT_, ZS>(d, r.chunk_elems, off0, l0, nl, round,
                                                                      mk, layer_base, w, sink, N * IB, IB, zs);
    };
    if (act) {
        bool done = false;
        if constexpr (SHUF) {
            // rows under 128 elements: a row's plane piece shares its 128-B
            // line with the next row's, read by the lane's next load; plain
            // loads keep the line for it (C3 shuffled (1,): 64-B pieces,
            // 0.785 -> 0.751 ms; (0,)'s 4-KiB pieces stay non-temporal)
            if (al && d.KI < 128) {
                walk(std::true_type{}, std::false_type{});
                done = true;
            }
        }
        if (!done) {
            if (al) walk(std::true_type{}, std::true_type{});
            else walk(std::false_type{}, std::true_type{});
        }
    }
    if (LS == 2) {
        if (half && act) {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                s_mn[k * IB + il] = w[k].mn;
                s_mx[k * IB + il] = w[k].mx;
                s_cnt[k * IB + il] = (uint32_t)w[k].count;
                if constexpr (ZS) s_zs[k * IB + il] = zs[k];
            }
        }
        __syncthreads();
        if (half || !act) return;
        for (int64_t l = 0; l < g.n_layers - hA; ++l) {
#pragma unroll
            for (int k = 0; k < N; ++k) w[k].sum += s_sum[(l * N + k) * IB + il];
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
            w[k].mn = pmin(w[k].mn, s_mn[k * IB + il]);
            w[k].mx = pmax(w[k].mx, s_mx[k * IB + il]);
            w[k].count += (int64_t)s_cnt[k * IB + il];
            if constexpr (ZS) {   // the second half's layers come later
                const uint32_t z2 = s_zs[k * IB + il];
                zs[k] = z2 != kZsNone ? z2 : zs[k];
            }
        }
    }
    if constexpr (ZS) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const T z = (zs[k] >> 31) ? -(T)0 : (T)0;
            if (zs[k] != kZsNone && w[k].count > 0) {
                if ((g.zs & 1u) && w[k].mn == (T)0) w[k].mn = z;
                if ((g.zs & 2u) && w[k].mx == (T)0) w[k].mx = z;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        int64_t loc = i * N + k, f = 0;   // kept-dims index in the chunk -> final element
#pragma unroll
        for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
            if (dd < r.ndim && !((red >> dd) & 1u)) {
                const int64_t q = loc / r.shape[dd];
                f += (ac[dd] * r.shape[dd] + (loc - q * r.shape[dd])) * g.ostride[dd];
                loc = q;
            }
        }
        store_wpartial(a.out + f, w[k]);
    }
}


// Per-chunk column layout streamed over several chunks (pyas_reduce_axes
// with every chunk whole, dense_geometry's split 1, rows per chunk a
// multiple of 4).  Block (g, j) owns items j * kBlock * NV ... of chunks
// g * cpb ... g * cpb + cpb - 1 and walks them as ONE ring of loads
// (col_walk_layers: a chunk's first rows are in flight while the previous
// chunk's last group is summed), instead of one short walk per chunk with a
// fill and a drain each (dense_col: 64 KiB per wave on C3).  When a chunk's
// last group is in, each wave stages its lanes' partials in its own 8-KiB
// LDS area and writes them as consecutive 16-B stores (no block barrier).
// Same 4-row groups, order and count as col_rows_ring: bit-identical to
// dense_col.  A block whose chunks are not all 16-B aligned runs dense_col
// per chunk instead (block-uniform).
// NV items per lane, kWave apart: with adjacent items (a kept inner run of
// >= NV KiB, C3 axis (0,)) a wave's loads of one row cover NV KiB; NV > 1
// keeps one 4-row group in flight per item instead of two.
template <typename T, bool SHUF, bool BSWAP, int MASKED, int NV>
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_STREAM_WAVES) void k_axes_col_stream(AxesArgs a) {
    constexpr int N = 16 / sizeof(T);
    const AxesDense &d = a.d;
    const ReduceArgs &r = a.r;
    const int64_t g = blockIdx.x / d.bpc;
    const int64_t j = blockIdx.x - g * d.bpc;
    const int64_t c0 = g * d.cpb;
    const int64_t nc = d.n_chunks - c0 < d.cpb ? d.n_chunks - c0 : d.cpb;
    auto layer_base = [&](int64_t l) { return r.data + sload(r.offsets + c0 + l); };
    MaskT<T> mk;
    mk.init(r.mask);
    __shared__ uint4 stage[kBlock * 2 * N > col_units_lds<T>() ? kBlock * 2 * N : col_units_lds<T>()];
    bool al = true;   // block-uniform
    for (int64_t l = 0; al && l < nc; ++l) al = ldv_aligned<T, SHUF>(layer_base(l), r.chunk_elems);
    if (!al) {
        for (int64_t l = 0; l < nc; ++l)
            dense_col<T, SHUF, BSWAP, MASKED, false>(a, c0 + l, j, layer_base(l), mk, stage);
        return;
    }
    // wave w of block j owns items j * kBlock * NV + w * kWave * NV + v * kWave + lane, v < NV
    constexpr int DEPTH = NV == 1 ? 2 : 1;
    const int64_t items = d.KO * (d.KI / N);
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t iw = j * kBlock * NV + (threadIdx.x / kWave) * (kWave * NV);   // the wave's first item
    if (iw + lane >= items) return;                   // no block barrier below
    const int nv = (int)(items - iw < kWave ? items - iw : kWave);   // active lanes (a prefix)
    uint4 *ws = stage + (threadIdx.x / kWave) * (kWave * 2 * N);
    const int64_t KIV = d.KI / N;
    int64_t offs[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {   // row 0 of each item; a missing item re-reads item set 0's
        const int64_t it = iw + v * kWave + lane < items ? iw + v * kWave + lane : iw + lane;
        const int64_t ko = it / KIV, vv = it - ko * KIV;
        offs[v] = (ko * d.RI * d.KI + vv * N) * sizeof(T);
    }
    auto chunk_end = [&](int64_t cl, TileAcc<T> *acc) {
        const int64_t cob = sload(a.out_offsets + c0 + cl);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t iv = iw + v * kWave;
            const int64_t nvv = items - iv < kWave ? items - iv : kWave;   // items of set v (may be <= 0)
#pragma unroll
            for (int k = 0; k < N; ++k) {
                pyas_partial pp;
                tile_store_lane(acc[v * N + k], &pp);
                stage_put<T>(a, ws, lane * N + k, pp);
                acc[v * N + k].init();
            }
            wave_sync_lds();
            stage_flush<T>(a, ws, cob + iv * N, nvv * N, lane, nv);
            wave_sync_lds();   // the area is rewritten next
        }
    };
    TileAcc<T> acc[NV * N];
#pragma unroll
    for (int k = 0; k < NV * N; ++k) acc[k].init();
    // shuffled rows under 128 elements: plain plane loads (k_axes_fold_lean's rule)
    if (SHUF && d.KI < 128)
        col_walk_layers<T, SHUF, BSWAP, MASKED, true, DEPTH, false, NV>(
            d, r.chunk_elems, offs, 0, nc, mk, layer_base, acc, chunk_end);
    else
        col_walk_layers<T, SHUF, BSWAP, MASKED, true, DEPTH, true, NV>(
            d, r.chunk_elems, offs, 0, nc, mk, layer_base, acc, chunk_end);
}

// Shuffled chunks whose reduced rows sit inside each kept-outer block (dense
// form RO == 1, e.g. axis (1,) of a 64^3 chunk): the block of kept-outer
// index ko is RI x KI elements, contiguous in every byte plane (RI*KI bytes
// per plane, 4 KiB for C3).  A wave streams one such slab (or RB rows of it)
// with 16-B loads -- every load instruction reads 1 KiB of one plane, and
// the slab's planes are 4 contiguous 4 KiB runs -- transposes each lane's
// 16 elements out of the byte planes in registers (v_perm, as ldu does) and
// writes them to its LDS tile in the plain layout; each lane then walks the
// rows of its output columns ki = lane + 64 q from LDS in 4-row groups,
// exactly col_rows_ring's arithmetic (same groups, order and counts), so the
// partials equal dense_col's bit for bit.  The next slab's plane loads are
// issued piece by piece as this slab's pieces are transposed (one rolling
// register buffer), and are in flight while it is reduced from LDS.  Waves
// are persistent: wave gw of TW takes units (chunk, ko) gw, gw + TW, ...
// (adjacent waves read adjacent slabs).  Round 3's dword-plane walks ran this
// geometry at 58 % of 8 TB/s: their loads are 64-B pieces of 4 rows.
template <typename T, bool BSWAP, int MASKED, int KPL>
__global__ __launch_bounds__(kBlock) void k_axes_shuf_slab(AxesArgs a) {
    constexpr int ES = sizeof(T), MM = kSlabBytes / 1024 / ES;   // load steps per plane (max)
    using U = typename TT<T>::U;
    __shared__ uint4 tiles[kBlock / kWave][kSlabBytes / 16];
    const AxesDense &d = a.d;
    const ReduceArgs &r = a.r;
    // wave-uniform unit indices in SGPRs: the chunk offsets and output
    // offsets then come with scalar loads, which never wait on the vector
    // loads of the next slab in flight (a vector load of out_offsets[c] at a
    // unit's end made the wave wait for those with vmcnt(0))
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
    const int64_t gw = (int64_t)blockIdx.x * (kBlock / kWave) + w;
    const int64_t TW = (int64_t)gridDim.x * (kBlock / kWave);
    const int64_t KI = d.KI, RI = d.RI, RB = d.rb, NS = RI / RB;
    const int64_t n = r.chunk_elems;
    const int M = (int)(RB * KI / 1024);                 // 16-B loads per lane per plane
    const int64_t units = d.n_chunks * d.KO;
    uint4 *tile = tiles[w];
    const T *tv = reinterpret_cast<const T *>(tile);
    MaskT<T> mk;
    mk.init(r.mask);
    // One rolling register buffer: as soon as piece m of a slab has been
    // transposed into LDS, the next slab's piece m is loaded into the same
    // registers, so a wave keeps (MM - 1) x ES loads in flight through the
    // transposes and all MM x ES of the next slab through the reduction.
    // (Round 4's first form issued the next slab only after the whole
    // transpose, leaving the wave without loads in flight meanwhile.)
    uint4 pl[MM][ES];
    // wave-uniform base of sub-slab s of unit u (scalar registers) and its
    // alignment; a lane adds its 16-B offset and an immediate per piece
    auto slab_base = [&](int64_t u, int64_t s) {
        const int64_t c = u / d.KO, ko = u - c * d.KO;
        return r.data + sload(r.offsets + c) + (ko * RI + s * RB) * KI;
    };
    const uint32_t lo = 16u * (uint32_t)lane;
    // piece m's ES plane loads (pieces m >= M re-read piece 0, never used:
    // every path issues the same loads, so each wait leaves exactly the
    // younger ones in flight)
    // (one load form for aligned and unaligned chunks: a branch per piece
    // made the compiler's waits drain every load in flight)
    auto load_piece = [&](const uint8_t *sb, int m) {
        const int mm = m < M ? m : 0;
#pragma unroll
        for (int b = 0; b < ES; ++b) pl[m][b] = ld16<false>(sb + b * n + lo + mm * 1024);
    };
    TileAcc<T> acc[KPL];
#pragma unroll
    for (int q = 0; q < KPL; ++q) acc[q].init();
    int64_t u = gw, s = 0;
    if (u < units) {
        const uint8_t *sb0 = slab_base(u, 0);
#pragma unroll
        for (int m = 0; m < MM; ++m) load_piece(sb0, m);
    }
    while (u < units) {   // wave-uniform
        const int64_t cu = u, cs = s;
        if (++s == NS) {
            s = 0;
            u += TW;
        }
        // the next sub-slab (past the last unit: this one again, never used)
        const uint8_t *sbn = u < units ? slab_base(u, s) : slab_base(cu, cs);
        // plane bytes -> plain elements (raw byte order) -> LDS, piece by
        // piece (pieces m >= M too: rows past RB of the tile, never read --
        // no branch, so the waits stay exact)
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            {
                uint4 v[ES];
                if constexpr (ES == 4) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        uint32_t e[4];
                        transpose4(word(pl[m][0], j), word(pl[m][1], j), word(pl[m][2], j), word(pl[m][3], j), e);
                        v[j] = make_uint4(e[0], e[1], e[2], e[3]);
                    }
                } else if constexpr (ES == 2) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const uint32_t a0 = word(pl[m][0], 2 * j), b0 = word(pl[m][1], 2 * j);
                        const uint32_t a1 = word(pl[m][0], 2 * j + 1), b1 = word(pl[m][1], 2 * j + 1);
                        v[j] = make_uint4(perm(b0, a0, 0x05010400u), perm(b0, a0, 0x07030602u),
                                          perm(b1, a1, 0x05010400u), perm(b1, a1, 0x07030602u));
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        uint32_t lo4[4], hi4[4];
                        transpose4(word(pl[m][0], j), word(pl[m][1], j), word(pl[m][2], j), word(pl[m][3], j), lo4);
                        transpose4(word(pl[m][4], j), word(pl[m][5], j), word(pl[m][6], j), word(pl[m][7], j), hi4);
                        v[2 * j] = make_uint4(lo4[0], hi4[0], lo4[1], hi4[1]);
                        v[2 * j + 1] = make_uint4(lo4[2], hi4[2], lo4[3], hi4[3]);
                    }
                }
#pragma unroll
                for (int b = 0; b < ES; ++b) tile[(m * 64 + lane) * ES + b] = v[b];
            }
            // piece m of the next sub-slab, into the freed registers; the
            // scheduling fences keep the pieces' loads in this order (the
            // scheduler would otherwise regroup them and the waits with them)
            __builtin_amdgcn_sched_barrier(0);
            load_piece(sbn, m);
            __builtin_amdgcn_sched_barrier(0);
        }
        wave_sync_lds();
        // rows of this sub-slab, output columns ki = lane + 64 q, 4-row groups
        int64_t rr = 0;
        for (; rr + 4 <= RB; rr += 4) {
            bool bad = false;
#pragma unroll
            for (int q = 0; q < KPL; ++q) {
                T x[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    U raw;
                    const T y = tv[(rr + k) * KI + q * 64 + lane];
                    __builtin_memcpy(&raw, &y, ES);
                    if (BSWAP) raw = bswap(raw);
                    x[k] = bits_to<T>(raw);
                }
                bad |= acc[q].template add_lazy<4, MASKED, false>(x, mk);
            }
            if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
                for (int q = 0; q < KPL; ++q) {
                    T x[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        U raw;
                        const T y = tv[(rr + k) * KI + q * 64 + lane];
                        __builtin_memcpy(&raw, &y, ES);
                        if (BSWAP) raw = bswap(raw);
                        x[k] = bits_to<T>(raw);
                    }
                    acc[q].template check_nan<4>(x);
                }
            }
        }
        for (; rr < RB; ++rr) {   // a row tail (RB % 4): single rows, as col_rows does
#pragma unroll
            for (int q = 0; q < KPL; ++q) {
                U raw;
                const T y = tv[rr * KI + q * 64 + lane];
                __builtin_memcpy(&raw, &y, ES);
                if (BSWAP) raw = bswap(raw);
                const T x = bits_to<T>(raw);
                acc[q].template add_n<1, MASKED, false>(&x, mk);
            }
        }
        if (cs == NS - 1) {   // the unit's last rows: its KPL * 64 outputs
            const int64_t c = cu / d.KO, ko = cu - c * d.KO;
            const int64_t ob = sload(a.out_offsets + c) + ko * KI;
#pragma unroll
            for (int q = 0; q < KPL; ++q) {
                if constexpr (!MASKED) acc[q].count += (uint32_t)RI;
                pyas_partial pp;
                tile_store_lane(acc[q], &pp);
                put_out<T>(a, ob + q * 64 + lane, pp);
                acc[q].init();
            }
        }
        wave_sync_lds();   // the tile is rewritten next
    }
}




// A position's place in a contiguous call, stepped one position at a time
// (l = q * lr + k * piece + kpos): tie_keys(l, sign 0) without a division,
// for a walk over consecutive positions (the fold's layers).
struct TiePos {
    uint32_t q = 0, k = 0, pos = 0, kpos = 0;
    __device__ void next(const TieCall &c, const TieRule &t) {
        if (++pos == (uint32_t)c.lr) {
            pos = kpos = k = 0;
            ++q;
        } else if (++kpos == (uint32_t)t.piece) {
            kpos = 0;
            ++k;
        }
    }
    __device__ void keys(int64_t l, const TieCall &c, const TieRule &t, uint64_t &k1, uint64_t &w) const {
        if (l == 0) {   // the seed
            k1 = 2u;
            w = 0u;
            return;
        }
        const uint32_t P = (uint32_t)t.piece, lr = (uint32_t)c.lr, L = (uint32_t)t.lanes;
        const uint32_t s0 = (q == 0 && k == 0) ? 1u : k * P;
        const uint32_t e1 = (k + 1) * P < lr ? (k + 1) * P : lr;
        const uint32_t m = e1 - s0, off = pos - s0;
        const bool vec = off < (m & ~(L - 1u));
        const uint32_t rk = vec ? (uint32_t)t.rank[off & (L - 1u)] : kTieRemRank;
        k1 = (!vec || rk == 0) ? (((uint64_t)l + 1) << 1) : 0u;
        w = (((uint64_t)q * (uint64_t)c.npr + k + 1) << 32) | ((uint64_t)rk << 25) |
            ((uint64_t)(((uint32_t)1 << kTieOffBits) - 1 - off) << 1);
    }
};

// Whole-chunk box query, LDS row layout (modes 4/5/6), chunk layers folded
// in the kernel (pyas_reduce_axes_grid).  Block (col, j), wave w owns the
// output tiles j*4 + w, + 4*bpc, ... of kept-dims chunk column `col`; for
// each layer (the column's chunks along the reduced dims, in C order) it
// stages the layer chunk's runs through LDS and folds them as dense_row_lds
// does, then merges the partial store_group would write into a running WAcc
// (k_combine_grid's merge, same rounding).  Bit-identical to k_axes_dense +
// k_combine_grid; the next layer's tile is loaded while this one is folded.
// ZS (g.zs = which: 1 min, 2 max): NumPy's sign of a zero min/max fused in.
// Each output row of a chunk is ONE contiguous reduce call of NumPy's
// (storage.py:99-100 over a C-ordered chunk whose trailing reduced group is
// the row; tie rule g.t).  When a layer's row min/max is a zero, the row's
// lane 0 finds the winning zero from the tile still in LDS, by the host's
// masks of the row's positions (the K1/W keys of tie_keys, evaluated on
// bits): the last remainder zero if any (read backwards from the row's end:
// one or two vectors on zero-heavy data); else, from the row's whole zero
// mask, the later of the last seed/top-lane zero (K1) and, unless the seed
// is a zero, the last zero of the lowest lane-rank class holding one (W).
// The winner's sign is read back from LDS and keyed at position l of the
// `out` array's call g.c2 (active.py:594; the position's keys are
// wave-uniform, worked out once per layer); the output's zero min/max takes
// the sign those level-2 keys give.  Zero-free layers cost one ballot.
// (Building the zero mask in the main pass instead cost every min/max query
// 21 %: C3 (2,) 0.70 -> 0.85 ms.)
template <typename T, bool SHUF, bool BSWAP, int MASKED, int H, bool ZS>
// (Holding the ZS kernel to 128 VGPRs, the non-ZS kernel's 4 waves per SIMD,
// made it slower: C3 (2,) 0.77 -> 1.0-1.06 ms, profiles/r04/zeros7.)
__global__ __launch_bounds__(kBlock) PYAS_XATTR(PYAS_FOLD_ROW_WAVES) void k_axes_fold_row(AxesArgs a, FoldGrid g) {
    constexpr int ES = sizeof(T), N = 16 / ES, RPW = kWave / H, VPL = Unit<T, SHUF>::VPL;
    constexpr int UL = 16 / H / VPL > 0 ? 16 / H / VPL : 1;   // load units per lane per tile
    __shared__ uint4 tile[(kBlock / kWave) * RPW * kRowLdsStride];
    // ZS: lane-class sets -> rank sets, per byte of the class set (entries
    // 256 h + byte: the ranks of lanes 8 h + i for the byte's bits i), and
    // rank -> lane
    __shared__ uint16_t s_pt[ZS ? 512 : 1];
    __shared__ uint8_t s_ord[ZS ? 64 : 1];
    if constexpr (ZS) {
        for (int x = threadIdx.x; x < 512; x += kBlock) {
            const int hh = x >> 8, byte = x & 255;
            uint32_t m = 0;
            for (int i = 0; i < 8; ++i)
                if (((byte >> i) & 1) && 8 * hh + i < g.t.lanes) m |= 1u << g.t.rank[8 * hh + i];
            s_pt[x] = (uint16_t)m;
        }
        if ((int)threadIdx.x < g.t.lanes) s_ord[g.t.rank[threadIdx.x]] = (uint8_t)threadIdx.x;
        __syncthreads();
    }
    const AxesDense &d = a.d;
    const ReduceArgs &r = a.r;
    const int64_t col = blockIdx.x / d.bpc;
    const int64_t j = blockIdx.x - col * d.bpc;
    const uint32_t red = a.axes;
    int64_t ac[PYAS_MAX_DIMS], gstride[PYAS_MAX_DIMS];
    int64_t rest = col, st = 1, nk = 0;
#pragma unroll
    for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
        ac[dd] = 0;
        gstride[dd] = st;
        if (dd < r.ndim) {
            st *= g.n_coords[dd];
            if (!((red >> dd) & 1u)) {
                const int64_t q = rest / g.n_coords[dd];
                ac[dd] = rest - q * g.n_coords[dd];
                rest = q;
                nk += ac[dd] * gstride[dd];
            }
        }
    }
    auto layer_base = [&](int64_t l) {
        int64_t n = nk, rr = l;
#pragma unroll
        for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
            if (dd < r.ndim && ((red >> dd) & 1u)) {
                const int64_t q = rr / g.n_coords[dd];
                n += (rr - q * g.n_coords[dd]) * gstride[dd];
                rr = q;
            }
        }
        return r.data + sload(r.offsets + n);
    };
    MaskT<T> mk;
    mk.init(r.mask);
    const bool round = (g.flags & PYAS_COMBINE_ROUND_TO_VAR) != 0;
    const int V = (int)(d.RI / N), VH = V / H;
    const int lane = threadIdx.x & (kWave - 1), rw = lane / H, h = lane - rw * H;
    uint4 *t = tile + (threadIdx.x / kWave) * RPW * kRowLdsStride;
    const int64_t wave = j * (kBlock / kWave) + threadIdx.x / kWave;
    const int64_t nwaves = d.bpc * (kBlock / kWave);
    int lrow[UL], lcol[UL];
#pragma unroll
    for (int u = 0; u < UL; ++u) {
        const int q = (u * kWave + lane) * VPL;
        lrow[u] = q / V;
        lcol[u] = q - lrow[u] * V;
    }
    uint4 w[UL][VPL];
    auto load = [&](const uint8_t *base, int64_t o0, int64_t nvec) {
        const uint8_t *src = base + o0 * d.RI * ES;
        if (ldu_aligned<T, SHUF>(SHUF ? base : src, r.chunk_elems)) {
#pragma unroll
            for (int u = 0; u < UL; ++u)
                if ((u * kWave + lane) * VPL < nvec)
                    ldu<T, SHUF, true>(base, src + (int64_t)(u * kWave + lane) * VPL * 16, r.chunk_elems, w[u]);
        } else {
#pragma unroll
            for (int u = 0; u < UL; ++u)
                if ((u * kWave + lane) * VPL < nvec)
                    ldu<T, SHUF, false>(base, src + (int64_t)(u * kWave + lane) * VPL * 16, r.chunk_elems, w[u]);
        }
    };
    for (int64_t o0 = wave * RPW; o0 < d.KO; o0 += nwaves * RPW) {   // wave-uniform
        const int64_t nvec = (d.KO - o0 < RPW ? d.KO - o0 : RPW) * V;
        WAcc<T> wacc;
        wacc.init();
        uint64_t zk1 = 0, zkw = kTieWNone;   // ZS: level-2 keys of the row's zero layers
        TiePos l2;                           // ZS: layer l's place in the `out` call
        load(layer_base(0), o0, nvec);
        for (int64_t l = 0; l < g.n_layers; ++l) {
#pragma unroll
            for (int u = 0; u < UL; ++u)
                if ((u * kWave + lane) * VPL < nvec) {
#pragma unroll
                    for (int i = 0; i < VPL; ++i) t[lrow[u] * kRowLdsStride + lcol[u] + i] = w[u][i];
                }
            wave_sync_lds();
            if (l + 1 < g.n_layers) load(layer_base(l + 1), o0, nvec);
            TileAcc<T> acc;
            acc.init();
            const uint4 *row = t + rw * kRowLdsStride + h * VH;
            // ZS: the lane's zero bits (its first element highest), gathered
            // only for vectors after which its running min/max is exactly
            // zero (before, no zero was read; past zero, not a zero row):
            // zero-free rows pay a compare and a branch per vector.  (The
            // whole mask built unconditionally cost every min/max query 21 %;
            // re-reading the tile for zero rows cost 2 %-zero data +29 %.)
            using ZW = typename std::conditional<H == 1, uint64_t, uint32_t>::type;
            ZW zl = 0;
            for (int i = 0; i < VH; ++i) {
                T x[N];
                unpack16<T, BSWAP>(row[i], x);
                acc.template add_n<N, MASKED, false>(x, mk);
                if constexpr (ZS) {
                    const T ext = (g.zs & 1u) ? acc.mn : acc.mx;
                    if (ext == (T)0) {
                        uint32_t b = 0;
#pragma unroll
                        for (int k = 0; k < N; ++k) b |= (x[k] == (T)0 ? 1u : 0u) << (N - 1 - k);
                        zl |= (ZW)b << (VH * N - N * (i + 1));
                    }
                }
            }
            if constexpr (!MASKED) acc.count += (uint32_t)(VH * N);
            uint32_t cnt, nan;
            group_reduce(acc, H, cnt, nan);   // every lane of the row holds the row's result
            if constexpr (ZS) {
                const T v = (g.zs & 1u) ? acc.mn : acc.mx;
                // the rows whose min/max is a zero find their winning zero e
                // from the tile, all H lanes of a row together (a masked zero
                // never makes the min/max a zero -- value rules mask zeros all
                // or none -- so every zero element counts)
                const bool zrow = cnt > 0 && !nan && v == (T)0;   // the row's H lanes agree
                if (__ballot(zrow)) {
                    const uint4 *trow = t + rw * kRowLdsStride;
                    int e = -1;
                    // the row's zero mask Z (lane h: its VH vectors, reversed
                    // to element order at its offset), then: the last
                    // remainder zero, if any, wins (K1; W is never later);
                    // else the later of the last seed/top-lane zero (K1) and,
                    // unless the seed is a zero, the last zero of the lowest
                    // lane-rank class holding one (W)
                    uint64_t Z = 0;
                    if (zrow) {
                        const int J = VH * N;
                        if constexpr (H == 1) Z = __builtin_bitreverse64(zl) >> (64 - J);
                        else Z = (uint64_t)(__builtin_bitreverse32(zl) >> (32 - J)) << (h * J);
                    }
#pragma unroll
                    for (int mm = H / 2; mm >= 1; mm >>= 1) Z |= shfl_xor(Z, mm);
                    if (zrow && h == 0 && Z) {
                        const uint64_t zr = Z & g.zrow_rem;
                        if (zr) {
                            e = msb64(zr);
                        } else {
                            const uint64_t sig = Z & (g.zrow_top | 1u);
                            const int e1 = sig ? msb64(sig) : -1;
                            int ew = -1;
                            const uint64_t Zv = Z & g.zrow_vec;   // the zeros in the lanes
                            if (!(Z & 1u) && Zv) {   // (a zero seed is W itself, at 0)
                                const int L = g.t.lanes;
                                if (L <= 16) {
                                    // the lane classes holding a zero (bit j: lane j),
                                    // through the rank tables: the lowest rank's class
                                    uint32_t C = 0;
                                    for (int bb = 0; 1 + bb * L < 64; ++bb)
                                        C |= (uint32_t)(Zv >> (1 + bb * L)) & ((1u << L) - 1u);
                                    const uint32_t P = (uint32_t)s_pt[C & 0xFFu] | (uint32_t)s_pt[256 + (C >> 8)];
                                    const int jj = s_ord[__builtin_ctz(P)];
                                    ew = msb64(Zv & (g.zrow_rep << (1 + jj)));
                                } else {
                                    for (int rk = 0; rk < L; ++rk) {
                                        const uint64_t cz = Z & g.zrow_cm[rk];
                                        if (cz) {
                                            ew = msb64(cz);
                                            break;
                                        }
                                    }
                                }
                            }
                            e = ew > e1 ? ew : e1;
                        }
                    }
                    // level-2 keys of position l (sign 0; wave-uniform, from
                    // the incremental position state: no division)
                    uint64_t lk1, lkw;
                    l2.keys(l, g.c2, g.t, lk1, lkw);
                    if (zrow && h == 0 && e >= 0) {
                        T xe[N];
                        unpack16<T, BSWAP>(trow[e / N], xe);
                        T we = xe[0];
#pragma unroll
                        for (int k = 1; k < N; ++k) we = (e % N) == k ? xe[k] : we;
                        const uint64_t sg = __builtin_signbit(we) ? 1u : 0u;
                        const uint64_t x1 = lk1 ? (lk1 | sg) : 0u, xw = lkw | sg;
                        zk1 = x1 > zk1 ? x1 : zk1;
                        zkw = xw < zkw ? xw : zkw;
                    }
                }
                l2.next(g.c2, g.t);
            }
            if (h == 0) {
                pyas_partial pp;
                store_group(acc, cnt, nan, &pp);
                merge(wacc, pp, round);
            }
            wave_sync_lds();
        }
        if constexpr (ZS) {
            if (h == 0 && wacc.count > 0 && (zk1 != 0 || zkw != kTieWNone)) {
                const int sg = tie_finalize(zk1, zkw, 0, g.c2, g.t);
                const T zz = sg == 1 ? -(T)0 : (T)0;
                if ((g.zs & 1u) && wacc.mn == (T)0) wacc.mn = zz;
                if ((g.zs & 2u) && wacc.mx == (T)0) wacc.mx = zz;
            }
        }
        if (h == 0 && o0 + rw < d.KO) {
            int64_t loc = o0 + rw, f = 0;   // kept-dims index in the chunk -> final element
#pragma unroll
            for (int dd = PYAS_MAX_DIMS - 1; dd >= 0; --dd) {
                if (dd < r.ndim && !((red >> dd) & 1u)) {
                    const int64_t q = loc / r.shape[dd];
                    f += (ac[dd] * r.shape[dd] + (loc - q * r.shape[dd])) * g.ostride[dd];
                    loc = q;
                }
            }
            store_wpartial(a.out + f, wacc);
        }
    }
}

template <typename T, bool SHUF, bool BSWAP>
__global__ __launch_bounds__(kBlock) void k_reduce_axes(AxesArgs a) {
    // the reduced-offset map, sized by the host to the chunk's reduced extent
    // (a.roff_cap entries): a fixed 32 KiB array held 4 workgroups per CU
    extern __shared__ int32_t roff[];
    const int64_t c = blockIdx.x / a.bpc;
    const int64_t j = blockIdx.x - c * a.bpc;
    const ReduceArgs &r = a.r;
    Sel s;
    load_sel(s, r.sel, c, r.ndim, r.shape);
    if (dense_owns(a, s)) return;    // k_axes_dense took this chunk
    const uint8_t *base = r.data + r.offsets[c];
    MaskT<T> mk;
    mk.init(r.mask);
    const uint32_t all = (1u << r.ndim) - 1u;
    const uint32_t red = a.axes & all, keep = all & ~red;
    int64_t n_out = 1, n_red = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d < r.ndim) {
            if ((red >> d) & 1u) n_red *= s.cnt[d];
            else n_out *= s.cnt[d];
        }
    }
    axes_block<T, SHUF, BSWAP>(a, c, j, base, s, red, keep, n_out, n_red, mk, roff);
}

// ---------------------------------------------------------------------------
// method=None: select + mask into dense outputs
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_select(SelectArgs a) {
    const int64_t c = blockIdx.x / a.bpc;
    const int64_t j = blockIdx.x - c * a.bpc;
    const ReduceArgs &r = a.r;
    const uint8_t *base = r.data + r.offsets[c];
    MaskT<T> mk;
    mk.init(r.mask);
    Sel s;
    load_sel(s, r.sel, c, r.ndim, r.shape);
    int64_t total = 1;
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) total *= s.cnt[d];
    const uint32_t all = (1u << r.ndim) - 1u;
    const bool scatter = a.scatter_pos != nullptr;
    T *vals = reinterpret_cast<T *>(a.values) + (scatter ? 0 : a.out_offsets[c]);
    uint8_t *msk = a.mask_out ? a.mask_out + (scatter ? 0 : a.out_offsets[c]) : nullptr;
    const int32_t *cb = scatter ? a.scatter_base + c * r.ndim : nullptr;
    for (int64_t e = j * kBlock + threadIdx.x; e < total; e += a.bpc * kBlock) {
        Decomp o{0, {0, 0}};
        decompose(s, r.pool, r.cstride, r.tab, r.ndim, all, e, o);
        const T x = load_elem_rt<T>(base, r.chunk_elems, o.mem, a.shuf, a.bswap);
        int64_t out = e;
        if (scatter) {   // block-uniform
            out = 0;
            int64_t rem = e;
#pragma unroll
            for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
                if (d < r.ndim) {
                    const int64_t cd = s.cnt[d];
                    const int64_t q = rem / cd, k = rem - q * cd;
                    rem = q;
                    out += a.scatter_pos[cb[d] + k] * a.ostride[d];
                }
            }
        }
        vals[out] = x;
        if (msk) msk[out] = all_masked(mk, r.tab, o, x) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// NumPy's sign of a zero min/max (pyas.h pyas_tie_*; zerosign.py restates
// the same arithmetic and documents the measured NumPy behaviour)
// ---------------------------------------------------------------------------
// Key layouts (order-free: K1 combines by max, W by min):
//   K1, contiguous loop : (e + 1) << 1 | sign of the seed, top-lane and
//                         remainder zeros (0: none)
//   W                   : (row + 1) << 32 | lane rank << 25 | (2^24-1-off) << 1 | sign
//                         (the seed: sign alone; none: kTieWNone)
//   K1, strided loop    : (call + 1) << 33 | remainder << 32 | acc priority << 25 | off << 1 | sign
//                         (the seed: 2 | sign)
// (kTieWNone, kTieOffBits, kTieRemRank: defined above k_axes_fold_row)

// Call structure (zerosign.call_structure): cnt/vstride per dim in elements,
// perm = iteration order (outer -> inner).  lr = 1: elementwise calls.  A
// strided call (acc) whose first buffer fill spans more than one kept
// iteration dim: the first n_copy runs are copied, i.e. contiguous calls;
// `block` = those kept dims.
__device__ __forceinline__ TieCall tie_call(const int64_t *cnt, const int64_t *vstride, uint32_t red,
                                            const int32_t *perm, int nd, bool buffered, int64_t piece) {
    TieCall c;
    c.acc = 0;
    c.lr = 1;
    c.npr = 1;
    c.n_copy = 0;
    c.block = 0;
    int64_t lr = 1, prev_stride = 0, prev_cnt = 0, inner_stride = 0, first = 0, kb = 1;
    bool one = true, any = false, chain = true;
    int state = 0;   // 0 trailing reduced group, 1 kept block, 2 done
#pragma unroll
    for (int i = PYAS_MAX_DIMS - 1; i >= 0; --i) {
        if (i < nd && state < 2) {
            const int d = perm[i];
            if (cnt[d] != 1) {
                const bool r = (red >> d) & 1u;
                if (state == 0 && r) {
                    if (!any) inner_stride = vstride[d];
                    else if (vstride[d] != prev_stride * prev_cnt) one = false;
                    any = true;
                    lr *= cnt[d];
                } else if (!any || r) {
                    state = 2;
                } else {
                    if (state == 0) {
                        state = 1;
                        first = cnt[d];
                    } else if (chain && vstride[d] == prev_stride * prev_cnt) {
                        first *= cnt[d];
                    } else {
                        chain = false;
                    }
                    c.block |= 1u << d;
                    kb *= cnt[d];
                }
                prev_stride = vstride[d];
                prev_cnt = cnt[d];
            }
        }
    }
    if (!any) {
        c.block = 0;
        return c;
    }
    c.lr = lr;
    c.npr = (lr + piece - 1) / piece;
    c.acc = (one && !buffered && inner_stride != 1) ? 1 : 0;
    // only a non-empty kept block right outside the group can be copied
    // (call_structure's `if block and piece`)
    const int64_t n1 = c.acc && c.block && lr < piece ? (piece / lr < kb ? piece / lr : kb) : 0;
    if (n1 > first) c.n_copy = n1;
    else c.block = 0;
    return c;
}

// Keys of a zero at reduced position e (sg = its sign bit): k1/w for a
// contiguous call, ka for a strided one (lanes: a copied strided call).
__device__ __forceinline__ void tie_keys(int64_t e, uint64_t sg, const TieCall &c, const TieRule &t, bool lanes,
                                         uint64_t &k1, uint64_t &w, uint64_t &ka) {
    k1 = 0;
    w = kTieWNone;
    ka = 0;
    const bool acc = c.acc && !lanes;
    if (e == 0) {
        if (acc) ka = 2u | sg;
        else {
            k1 = 2u | sg;
            w = sg;
        }
        return;
    }
    const int64_t P = t.piece;
    const int64_t q = e / c.lr, pos = e - q * c.lr;
    const int64_t k = pos / P;
    const int64_t s0 = (q == 0 && k == 0) ? 1 : k * P;
    const int64_t e1 = (k + 1) * P < c.lr ? (k + 1) * P : c.lr;
    const int64_t m = e1 - s0, off = pos - s0;
    const uint64_t row1 = (uint64_t)(q * c.npr + k + 1);
    if (acc) {
        const int64_t nv = m - m % t.acc;
        const bool vec = off < nv;
        const uint64_t prio = vec ? (uint64_t)(t.acc - 1 - t.acc_rank[off % t.acc]) : 0u;
        ka = (row1 << 33) | ((uint64_t)(vec ? 0 : 1) << 32) | (prio << 25) | ((uint64_t)off << 1) | sg;
        return;
    }
    const int64_t nv = m - m % t.lanes;
    const bool vec = off < nv;
    const uint32_t rank = vec ? (uint32_t)t.rank[off % t.lanes] : kTieRemRank;
    k1 = (!vec || rank == 0) ? ((((uint64_t)e + 1) << 1) | sg) : 0u;
    w = (row1 << 32) | ((uint64_t)rank << 25) | ((uint64_t)(((int64_t)1 << kTieOffBits) - 1 - off) << 1) | sg;
}

// Reduced position of the zero behind a contiguous call's W key.
__device__ __forceinline__ int64_t tie_w_pos(uint64_t w, const TieCall &c, const TieRule &t) {
    if (w < 2) return 0;
    const int64_t row = (int64_t)(w >> 32) - 1;
    const int64_t off = (((int64_t)1 << kTieOffBits) - 1) - (int64_t)((w >> 1) & ((1u << kTieOffBits) - 1));
    const int64_t q = row / c.npr, k = row - q * c.npr;
    const int64_t s0 = (q == 0 && k == 0) ? 1 : k * (int64_t)t.piece;
    return q * c.lr + s0 + off;
}

// Sign bit from an output's combined keys; -1 when it holds no zero.
__device__ __forceinline__ int tie_finalize(uint64_t k1, uint64_t w, uint64_t ka, const TieCall &c,
                                            const TieRule &t) {
    if (ka) return (int)(ka & 1u);   // a strided call's zero is later than a copied first call's
    if (k1 == 0 && w == kTieWNone) return -1;
    if (k1 == 0) return (int)(w & 1u);
    if (w == kTieWNone) return (int)(k1 & 1u);
    const int64_t e1 = (int64_t)(k1 >> 1) - 1;
    return tie_w_pos(w, c, t) > e1 ? (int)(w & 1u) : (int)(k1 & 1u);
}

template <typename T>
__device__ __forceinline__ bool tie_zero(const pyas_partial &p, uint32_t which) {
    return p.count > 0 && (((which & 1u) && TT<T>::from(p.min) == (T)0) ||
                           ((which & 2u) && TT<T>::from(p.max) == (T)0));
}

template <typename T>
__device__ __forceinline__ void tie_put(pyas_partial *p, uint32_t which, int sg) {
    const T z = sg ? -(T)0 : (T)0;
    if ((which & 1u) && TT<T>::from(p->min) == (T)0) TT<T>::put(p->min, z);
    if ((which & 2u) && TT<T>::from(p->max) == (T)0) TT<T>::put(p->max, z);
}

// The form of level-1 partial arrays: PYAS_TIE_REC in `which` = records of
// the queried method (pyas_reduce_axes_ex), else 32-byte partials.
__device__ __forceinline__ int tie_rec(uint32_t which) {
    return (which & PYAS_TIE_REC) ? ((which & 1u) ? PYAS_REC_MIN : PYAS_REC_MAX) : 0;
}

// tie_put on entry i of a partial array of form `rec` (a record's value is
// the queried min or max itself)
template <typename T>
__device__ __forceinline__ void tie_put_at(void *parts, int64_t i, int rec, uint32_t which, int sg) {
    if (rec == 0) {
        tie_put<T>(reinterpret_cast<pyas_partial *>(parts) + i, which, sg);
        return;
    }
    T *v = reinterpret_cast<T *>(reinterpret_cast<uint8_t *>(parts) + i * Rec<T>::kBytes);
    if (*v == (T)0) *v = sg ? -(T)0 : (T)0;
}

// Group reductions over G consecutive lanes of a wave (G = 1: none; 16 or
// 64: DPP/bpermute butterflies that never leave the group).
template <int G>
__device__ __forceinline__ uint64_t grp_max_u64(uint64_t v) {
    static_assert(G == 1 || G == 16 || G == kWave, "lanes per output: 1, 16 or a wave");
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor(v, m);
        v = o > v ? o : v;
    }
    return v;
}

template <int G>
__device__ __forceinline__ uint64_t grp_min_u64(uint64_t v) {
    return ~grp_max_u64<G>(~v);
}

// tie_keys in 32-bit arithmetic: every position, call length and piece of a
// chunk output is < 2^31 (pyas_tie_chunks checks the reduced count).  The
// rule's priority tables are read from LDS (rank / arank).
__device__ __forceinline__ void tie_keys32(uint32_t e, uint64_t sg, const TieCall &c, const TieRule &t,
                                           const uint8_t *rank, const uint8_t *arank, bool lanes, uint64_t &k1,
                                           uint64_t &w, uint64_t &ka) {
    k1 = 0;
    w = kTieWNone;
    ka = 0;
    const bool acc = c.acc && !lanes;
    if (e == 0) {
        if (acc) ka = 2u | sg;
        else {
            k1 = 2u | sg;
            w = sg;
        }
        return;
    }
    const uint32_t P = (uint32_t)t.piece, lr = (uint32_t)c.lr;
    const uint32_t q = e / lr, pos = e - q * lr;
    const uint32_t k = pos / P;
    const uint32_t s0 = (q == 0 && k == 0) ? 1u : k * P;
    const uint32_t e1 = (k + 1) * P < lr ? (k + 1) * P : lr;
    const uint32_t m = e1 - s0, off = pos - s0;
    const uint64_t row1 = (uint64_t)q * (uint64_t)c.npr + k + 1;
    if (acc) {
        const uint32_t A = (uint32_t)t.acc;
        const uint32_t nv = m - m % A;
        const bool vec = off < nv;
        const uint64_t prio = vec ? (uint64_t)(t.acc - 1 - arank[off % A]) : 0u;
        ka = (row1 << 33) | ((uint64_t)(vec ? 0 : 1) << 32) | (prio << 25) | ((uint64_t)off << 1) | sg;
        return;
    }
    const uint32_t L = (uint32_t)t.lanes;
    const uint32_t nv = m - m % L;
    const bool vec = off < nv;
    const uint32_t rk = vec ? (uint32_t)rank[off % L] : kTieRemRank;
    k1 = (!vec || rk == 0) ? ((((uint64_t)e + 1) << 1) | sg) : 0u;
    w = (row1 << 32) | ((uint64_t)rk << 25) | ((uint64_t)(((uint32_t)1 << kTieOffBits) - 1 - off) << 1) | sg;
}

// Per-chunk state of the level-1 scan, worked out once by one lane and
// shared through LDS: the call structure, the reduced dims in visiting
// order (scan slots, innermost first) and the kept dims (innermost first).
struct TieSetup {
    TieCall call;
    int64_t n_out, R, base_red, data_off, out_base;
    int32_t nr, nk;
    uint32_t rc[PYAS_MAX_DIMS];
    int32_t rst[PYAS_MAX_DIMS], rsp[PYAS_MAX_DIMS], rcs[PYAS_MAX_DIMS];
    int64_t rt0[PYAS_MAX_DIMS], rt1[PYAS_MAX_DIMS];
    uint32_t kc[PYAS_MAX_DIMS];
    int32_t kst[PYAS_MAX_DIMS], ksp[PYAS_MAX_DIMS], kcs[PYAS_MAX_DIMS];
    int64_t kbw[PYAS_MAX_DIMS], kt0[PYAS_MAX_DIMS], kt1[PYAS_MAX_DIMS];
    uint32_t kin;                     // bit j: kept slot j lies in NumPy's copied first fill
};

__device__ void tie_setup(const TieChunkArgs &a, int64_t c, TieSetup &S) {
    const ReduceArgs &r = a.r;
    Sel s;
    load_sel(s, r.sel, c, r.ndim, r.shape);
    int64_t cnt[PYAS_MAX_DIMS];
    int64_t n_out = 1, R = 1;
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        cnt[d] = d < r.ndim ? (int64_t)s.cnt[d] : 1;
        if ((a.axes >> d) & 1u) R *= cnt[d];
        else n_out *= cnt[d];
    }
    S.n_out = n_out;
    S.R = R;
    S.data_off = r.offsets[c];
    S.out_base = a.out_offsets ? a.out_offsets[c] : c;
    int64_t vstride[PYAS_MAX_DIMS];
    int64_t st = 1;
    for (int i = r.ndim - 1; i >= 0; --i) {
        const int d = a.g.perm[i];
        vstride[d] = st;
        st *= cnt[d];
    }
    if (a.g.flags & PYAS_TIE_VIEW)
        for (int d = 0; d < r.ndim; ++d) vstride[d] = (int64_t)s.step[d] * r.cstride[d];
    S.call = tie_call(cnt, vstride, a.axes, a.g.perm, r.ndim, (a.g.flags & PYAS_TIE_BUFFERED) != 0, a.t.piece);
    int64_t bw[PYAS_MAX_DIMS];   // kept-block weights (NumPy's copied first fill), inner first
    st = 1;
    for (int i = r.ndim - 1; i >= 0; --i) {
        const int d = a.g.perm[i];
        bw[d] = ((S.call.block >> d) & 1u) ? st : 0;
        if ((S.call.block >> d) & 1u) st *= cnt[d];
    }
    int nr = 0;
    S.base_red = 0;
    for (int i = r.ndim - 1; i >= 0; --i) {
        const int d = a.g.perm[i];
        if (!((a.axes >> d) & 1u)) continue;
        if (cnt[d] == 1) {   // one selected index: an offset, not a scan slot
            S.base_red += sel_index(s, r.pool, d, 0) * r.cstride[d];
            continue;
        }
        S.rc[nr] = (uint32_t)cnt[d];
        S.rst[nr] = s.start[d];
        S.rsp[nr] = s.step[d];
        S.rcs[nr] = (int32_t)r.cstride[d];
        S.rt0[nr] = r.tab.stride[0][d];
        S.rt1[nr] = r.tab.stride[1][d];
        ++nr;
    }
    S.nr = nr;
    int nk = 0;
    S.kin = 0;
    for (int d = r.ndim - 1; d >= 0; --d) {   // outputs are C-ordered over the kept dims
        if ((a.axes >> d) & 1u) continue;
        S.kc[nk] = (uint32_t)cnt[d];
        S.kst[nk] = s.start[d];
        S.ksp[nk] = s.step[d];
        S.kcs[nk] = (int32_t)r.cstride[d];
        S.kbw[nk] = bw[d];
        S.kt0[nk] = r.tab.stride[0][d];
        S.kt1[nk] = r.tab.stride[1][d];
        if ((S.call.block >> d) & 1u) S.kin |= 1u << nk;
        ++nk;
    }
    S.nk = nk;
}

// Level 1 (storage.py:99-100 over chunk[sel]): the sign NumPy gives each zero
// min/max output of a chunk, from ONE backward scan over the output's reduced
// positions e (its visiting order) that stops early.  Every key combines by
// max except W, and:
//  - a significant zero of a contiguous call (the seed aside: a top-lane or
//    remainder zero, K1 != 0) at e1 decides the output on its own: W's zero is
//    never later than e1 (it sits in e1's row or an earlier one, and in e1's
//    row it has rank 0 (then it is e1) or precedes the remainder);
//  - a strided call's zero (KA) in row r beats every zero of earlier rows and
//    every copied (contiguous) call; the rest of row r decides among them.
// So the scan walks e downwards in steps of G*V elements and stops after the
// step holding the first significant zero, or once it has finished the row of
// the first strided zero; only an output with neither is scanned to e = 0, and
// then its keys are complete.  tie_finalize of the scanned suffix's keys
// equals that of all keys (zerosign.predict_scan; tests compare with NumPy).
// G lanes share an output (1: one output per lane, for elementwise calls,
// where adjacent lanes hold adjacent outputs).  A workgroup takes one chunk
// and loops over its outputs, kBlock / G at a time; when every chunk has one
// output (a full reduction) each wave takes a chunk (a.cpw = 4 chunks per
// workgroup).  The chunk's setup is worked out once, by one lane, into LDS
// (TieSetup); the scan reads it as wave-uniform values.  Rewrite mode
// (parts): outputs whose min/max is a zero get NumPy's sign.  Flag mode
// (flags): one byte per chunk output, bit 0 an unmasked zero, bit 1 the
// winning zero's sign; skipped when *gate == 0.
template <typename T, int G>
__global__ __launch_bounds__(kBlock) void k_tie_scan(TieChunkArgs a) {
    constexpr int NG = kBlock / G;
    constexpr int V = G == 16 ? 1 : 4;        // elements per lane per step (8 measured slower for
                                              // a wave: C3 full min 34.7 -> 47.6 us at 50 % zeros)
    constexpr int NW = kBlock / kWave;
    __shared__ TieSetup setups[NW];
    __shared__ uint8_t rank[64], arank[64];
    const ReduceArgs &r = a.r;
    if (a.gate && *a.gate == 0u) return;
    const int grp = (int)threadIdx.x / G, gl = (int)threadIdx.x % G;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
    if (threadIdx.x < 64) {
        rank[threadIdx.x] = a.t.rank[threadIdx.x];
        arank[threadIdx.x] = a.t.acc_rank[threadIdx.x];
    }
    int64_t c, o_first, o_step;
    int slot;
    if (a.cpw > 1) {   // one output per chunk, a wave per chunk (host: G == kWave)
        c = (int64_t)blockIdx.x * a.cpw + wv;
        if (a.pick) {      // only the chunks the level-2 keys can pick: wave 0 K1's, wave 1 W's
            const uint64_t k1 = a.pick[0], kw = a.pick[1];
            const int64_t c1 = k1 ? (int64_t)(k1 >> 1) - 1 - a.pick_base : -1;
            const int64_t cw = kw != kTieWNone ? tie_w_pos(kw, a.pick_call, a.t) - a.pick_base : -1;
            c = wv == 0 ? c1 : (wv == 1 && cw != c1) ? cw : -1;
        }
        o_first = 0;
        o_step = 1;
        slot = wv;
        if (c >= 0 && c < a.n_chunks && lane == 0) tie_setup(a, c, setups[slot]);
    } else {
        c = blockIdx.x;
        o_first = grp;
        o_step = NG;
        slot = 0;
        if (threadIdx.x == 0) tie_setup(a, c, setups[0]);
    }
    __syncthreads();
    if (c < 0 || c >= a.n_chunks) return;   // wave-uniform
    const TieSetup &S = setups[slot];
    const int rec = tie_rec(a.which);
    const int64_t n_out = S.n_out, R = S.R;
    if (n_out == 0 || R == 0) return;
    const TieCall call = S.call;
    const int nr = S.nr, nk = S.nk;
    const bool tabs = r.tab.on[0] || r.tab.on[1];
    uint32_t rc[PYAS_MAX_DIMS];
    int32_t rst[PYAS_MAX_DIMS], rsp[PYAS_MAX_DIMS], rcs[PYAS_MAX_DIMS];
#pragma unroll
    for (int i = 0; i < PYAS_MAX_DIMS; ++i) {   // wave-uniform: scalar registers
        rc[i] = __builtin_amdgcn_readfirstlane(i < nr ? S.rc[i] : 1u);
        rst[i] = __builtin_amdgcn_readfirstlane(i < nr ? S.rst[i] : 0);
        rsp[i] = __builtin_amdgcn_readfirstlane(i < nr ? S.rsp[i] : 0);
        rcs[i] = __builtin_amdgcn_readfirstlane(i < nr ? S.rcs[i] : 0);
    }
    MaskT<T> mk;
    mk.init(r.mask);
    const uint8_t *data = r.data + S.data_off;
    const int64_t obase = S.out_base;
    for (int64_t ol = o_first; ol < n_out; ol += o_step) {   // group-uniform
        const int64_t ob = obase + ol;
        if (a.parts && !tie_zero<T>(part_at<T>(a.parts, ob, rec), a.which)) continue;
        // the output's kept coordinates: memory / table base, and whether its
        // first run is a copied (contiguous) call of a strided reduction
        Decomp base{S.base_red, {0, 0}};
        bool olanes = false;
        {
            uint32_t oo = (uint32_t)ol;
            int64_t bidx = 0;
            bool beyond = false;   // a kept coordinate outside the block is non-zero
#pragma unroll
            for (int j = 0; j < PYAS_MAX_DIMS; ++j) {
                if (j < nk) {
                    const uint32_t kcj = S.kc[j], q = j + 1 < nk ? oo / kcj : 0u, k = oo - q * kcj;
                    oo = q;   // (the last kept slot needs no division: oo < its count)
                    if ((S.kin >> j) & 1u) bidx += (int64_t)k * S.kbw[j];
                    else beyond |= k != 0;
                    const int64_t idx = S.ksp[j] != 0 ? (int64_t)S.kst[j] + (int64_t)k * S.ksp[j]
                                                      : (int64_t)r.pool[(int64_t)S.kst[j] + k];
                    base.mem += idx * S.kcs[j];
                    if (tabs) {
                        base.v[0] += (int64_t)k * S.kt0[j];
                        base.v[1] += (int64_t)k * S.kt1[j];
                    }
                }
            }
            olanes = call.n_copy && !beyond && bidx < call.n_copy;
        }
        uint64_t k1 = 0, kw = kTieWNone, ka = 0, stop1 = 0;   // stop1 = scan floor + 1 (0: none yet)
        int64_t hi = R;
        while (hi > 0 && (int64_t)stop1 - 1 < hi) {           // group-uniform
            const int64_t lo = hi - (int64_t)G * V;
            T x[V];
            Decomp o[V];
#pragma unroll
            for (int j = 0; j < V; ++j) {   // lanes of a load adjacent in e
                const int64_t e = lo + (int64_t)j * G + gl;
                o[j] = base;
                x[j] = (T)1;
                if (e >= 0) {
                    uint32_t rr = (uint32_t)e;
#pragma unroll
                    for (int i = 0; i < PYAS_MAX_DIMS; ++i) {
                        if (i < nr) {
                            const uint32_t q = i + 1 < nr ? rr / rc[i] : 0u, k = rr - q * rc[i];
                            rr = q;   // (the last slot needs no division: rr < its count)
                            const int64_t idx = rsp[i] != 0 ? (int64_t)rst[i] + (int64_t)k * rsp[i]
                                                            : (int64_t)r.pool[(int64_t)rst[i] + k];
                            o[j].mem += idx * rcs[i];
                            if (tabs) {
                                o[j].v[0] += (int64_t)k * S.rt0[i];
                                o[j].v[1] += (int64_t)k * S.rt1[i];
                            }
                        }
                    }
                    x[j] = load_elem_rt<T>(data, r.chunk_elems, o[j].mem, a.shuf, a.bswap);
                }
            }
            uint64_t thr1 = 0;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int64_t e = lo + (int64_t)j * G + gl;
                if (e >= 0 && x[j] == (T)0 && !all_masked(mk, r.tab, o[j], x[j])) {
                    const bool lanes = olanes && e < call.lr;
                    uint64_t x1, xw, xa;
                    tie_keys32((uint32_t)e, __builtin_signbit(x[j]) ? 1u : 0u, call, a.t, rank, arank, lanes, x1,
                               xw, xa);
                    k1 = x1 > k1 ? x1 : k1;
                    kw = xw < kw ? xw : kw;
                    ka = xa > ka ? xa : ka;
                    int64_t thr = -1;
                    if (call.acc && !lanes) {          // finish this zero's row
                        const uint32_t ue = (uint32_t)e, lr = (uint32_t)call.lr, P = (uint32_t)a.t.piece;
                        const uint32_t q = ue / lr, pos = ue - q * lr;
                        thr = (int64_t)q * lr + (pos / P) * P;
                    } else if (x1 != 0 && e > 0) {     // a significant zero decides
                        thr = e;
                    }
                    const uint64_t t1 = (uint64_t)(thr + 1);
                    thr1 = t1 > thr1 ? t1 : thr1;
                }
            }
            thr1 = thr1 > stop1 ? thr1 : stop1;
            stop1 = grp_max_u64<G>(thr1);
            hi = lo;
        }
        k1 = grp_max_u64<G>(k1);
        kw = grp_min_u64<G>(kw);
        ka = grp_max_u64<G>(ka);
        if (gl == 0) {
            const int sg = tie_finalize(k1, kw, ka, call, a.t);
            if (a.parts) {
                if (sg >= 0) tie_put_at<T>(a.parts, ob, rec, a.which, sg);
            } else {
                a.flags[ob] = sg < 0 ? (uint8_t)0 : (uint8_t)(1u | ((unsigned)sg << 1));
            }
        }
    }
}

// Is any final output's min/max a zero (the fold path's level-1 gate)?
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tie_gate(const pyas_partial *fin, int64_t n, uint32_t which,
                                                     uint32_t *gate) {
    int hit = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        hit |= tie_zero<T>(fin[i], which) ? 1 : 0;
    if (__syncthreads_or(hit) && threadIdx.x == 0) atomicOr(gate, 1u);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor(v, m);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor(v, m);
        v = o < v ? o : v;
    }
    return v;
}

// Level-2 keys by position alone of a full reduction's chunk partials
// (positions base + l of the `out` call; which zero wins does not depend on
// the signs): keys[0] = max K1, keys[1] = min W over the zero partials, one
// atomic each per workgroup.  The winner is one of the two chunks, so only
// they need the level-1 scan (pyas_tie_chunks_total).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tie_pick(const pyas_partial *parts, int64_t n, uint32_t which,
                                                     int64_t base, TieCall call, TieRule t, uint64_t *keys) {
    __shared__ uint64_t s1[kBlock / kWave], sw[kBlock / kWave];
    const int rec = tie_rec(which);
    uint64_t k1 = 0, kw = kTieWNone;
    for (int64_t l = (int64_t)blockIdx.x * kBlock + threadIdx.x; l < n; l += (int64_t)gridDim.x * kBlock) {
        if (!tie_zero<T>(part_at<T>(parts, l, rec), which)) continue;
        uint64_t x1, xw, xa;
        tie_keys(base + l, 0u, call, t, true, x1, xw, xa);
        k1 = x1 > k1 ? x1 : k1;
        kw = xw < kw ? xw : kw;
    }
    k1 = wave_max_u64(k1);
    kw = wave_min_u64(kw);
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        s1[w] = k1;
        sw[w] = kw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kBlock / kWave; ++i) {
            k1 = s1[i] > k1 ? s1[i] : k1;
            kw = sw[i] < kw ? sw[i] : kw;
        }
        if (k1) atomicMax(reinterpret_cast<unsigned long long *>(keys), (unsigned long long)k1);
        if (kw != kTieWNone) atomicMin(reinterpret_cast<unsigned long long *>(keys + 1), (unsigned long long)kw);
    }
}

// Level 2 (active.py:594 over the `out` array): one wave per (final output,
// slice of its chunk layers).  Layer l of output f comes from the grid
// tables (kind 0, pyas_combine_grid's walk), a segment list (kind 1,
// pyas_combine_segments') or parts[l] itself (kind 2, one output); its
// reduced position is layer_base + l.  keys == NULL: the output's sign is
// written to fin[f] (one slice per output); else the wave's keys are folded
// into keys[f] (max) / keys[n_out + f] (min).
// Keys of layers [lb, le) of final output f, lanes l0, l0 + ls, ... (the
// callers: a wave per output slice, or a thread per output).
template <typename T>
__device__ __forceinline__ void tie_grid_keys(const TieGridArgs &a, int64_t f, int64_t sl, int l0, int ls,
                                              uint64_t &k1, uint64_t &kw) {
    const pyas_grid &g = a.g;
    int64_t gstride[PYAS_MAX_DIMS];
    int64_t j = 0, nk = 0, l_lo = 0, l_n = a.n_layers;
    if (a.kind == 0) {
        int64_t jstride = 1, rest = f, st = 1;
#pragma unroll
        for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
            gstride[d] = st;
            if (d < g.ndim) {
                st *= g.n_coords[d];
                if (!((g.axes_mask >> d) & 1u)) {
                    const int64_t ext = g.out_extent[d];
                    const int64_t p = rest % ext;
                    rest /= ext;
                    const int64_t cc = g.pos_coord[d][p];
                    nk += cc * gstride[d];
                    j += (int64_t)g.pos_local[d][p] * jstride;
                    jstride *= g.coord_count[d][cc];
                }
            }
        }
    } else if (a.kind == 1) {
        l_lo = a.seg[f];
        l_n = a.seg[f + 1] - l_lo;
    }
    const int64_t per = (l_n + a.slices - 1) / a.slices;
    const int64_t lb = sl * per, le = (lb + per) < l_n ? (lb + per) : l_n;
    const int rec = tie_rec(a.which);
    k1 = 0;
    kw = kTieWNone;
    for (int64_t l = lb + l0; l < le; l += ls) {
        int64_t idx;
        if (a.kind == 0) {
            int64_t n = nk;
            uint32_t rr = (uint32_t)l;
#pragma unroll
            for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
                if (d < g.ndim && ((g.axes_mask >> d) & 1u)) {
                    const uint32_t nc = (uint32_t)g.n_coords[d], q = rr / nc;
                    n += (int64_t)(rr - q * nc) * gstride[d];
                    rr = q;
                }
            }
            idx = g.chunk_out_offsets[n] + j;
        } else if (a.kind == 1) {
            idx = a.index ? a.index[l_lo + l] : l_lo + l;
        } else {
            idx = l;
        }
        bool zero;
        uint64_t sg;
        if (a.flags) {
            const uint8_t b = a.flags[idx];
            zero = (b & 1u) != 0;
            sg = (b >> 1) & 1u;
        } else {
            const pyas_partial p = part_at<T>(a.parts, idx, rec);
            const T v = TT<T>::from((a.which & 1u) ? p.min : p.max);
            zero = p.count > 0 && v == (T)0;
            sg = __builtin_signbit(v) ? 1u : 0u;
        }
        if (zero) {
            uint64_t x1, xw, xa;
            tie_keys(a.layer_base + l, sg, a.call, a.t, true, x1, xw, xa);
            k1 = x1 > k1 ? x1 : k1;
            kw = xw < kw ? xw : kw;
        }
    }
}

template <typename T>
__device__ __forceinline__ void tie_grid_out(const TieGridArgs &a, int64_t f, uint64_t k1, uint64_t kw) {
    if (a.keys) {
        if (k1) atomicMax(reinterpret_cast<unsigned long long *>(a.keys + f), (unsigned long long)k1);
        if (kw != kTieWNone)
            atomicMin(reinterpret_cast<unsigned long long *>(a.keys + a.n_out + f), (unsigned long long)kw);
    } else {
        const int sg = tie_finalize(k1, kw, 0, a.call, a.t);
        if (sg >= 0) tie_put<T>(a.fin + f, a.which, sg);
    }
}

// Level 2 (active.py:594 over the `out` array): one wave per (final output,
// slice of its chunk layers).  Layer l of output f comes from the grid
// tables (kind 0, pyas_combine_grid's walk), a segment list (kind 1,
// pyas_combine_segments') or parts[l] itself (kind 2, one output); its
// reduced position is layer_base + l.  keys == NULL: the output's sign is
// written to fin[f] (one slice per output); else the wave's keys are folded
// into keys[f] (max) / keys[n_out + f] (min).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tie_grid(TieGridArgs a) {
    const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int64_t gw = (int64_t)blockIdx.x * (kBlock / kWave) + w;
    const int64_t f = gw / a.slices, sl = gw - f * a.slices;
    if (f >= a.n_out) return;   // wave-uniform
    if (!tie_zero<T>(a.fin[f], a.which)) return;
    uint64_t k1, kw;
    tie_grid_keys<T>(a, f, sl, lane, kWave, k1, kw);
    k1 = wave_max_u64(k1);
    kw = wave_min_u64(kw);
    if (lane == 0) tie_grid_out<T>(a, f, k1, kw);
}

// Level 2 with a thread per final output (one slice): many outputs with few
// layers each (C3 partial axes: 2^20 outputs x 16 layers), where a wave per
// output would leave most lanes idle.  Adjacent threads read adjacent flags
// or partials of the same chunk.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tie_grid_t(TieGridArgs a) {
    const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (f >= a.n_out || !tie_zero<T>(a.fin[f], a.which)) return;
    uint64_t k1, kw;
    tie_grid_keys<T>(a, f, 0, 0, 1, k1, kw);
    tie_grid_out<T>(a, f, k1, kw);
}

// Keys of n_sets slices or ranks ([K1[n_out], W[n_out]] each) -> fin's signs.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tie_finalize(const uint64_t *keys, int64_t n_out, int32_t n_sets,
                                                         TieCall call, TieRule t, uint32_t which,
                                                         pyas_partial *fin) {
    const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (f >= n_out || !tie_zero<T>(fin[f], which)) return;
    uint64_t k1 = 0, kw = kTieWNone;
    for (int32_t s = 0; s < n_sets; ++s) {
        const uint64_t x1 = keys[(int64_t)s * 2 * n_out + f], xw = keys[(int64_t)s * 2 * n_out + n_out + f];
        k1 = x1 > k1 ? x1 : k1;
        kw = xw < kw ? xw : kw;
    }
    const int sg = tie_finalize(k1, kw, 0, call, t);
    if (sg >= 0) tie_put<T>(fin + f, which, sg);
}

template <typename T>
hipError_t launch_tie_chunks_t(const TieChunkArgs &a, int64_t grid, hipStream_t st) {
    if constexpr (TT<T>::kind != 0) {
        return hipSuccess;
    } else {
        switch (a.group) {
        case 1: hipLaunchKernelGGL((k_tie_scan<T, 1>), dim3((unsigned)grid), dim3(kBlock), 0, st, a); break;
        case 16: hipLaunchKernelGGL((k_tie_scan<T, 16>), dim3((unsigned)grid), dim3(kBlock), 0, st, a); break;
        case 64: hipLaunchKernelGGL((k_tie_scan<T, 64>), dim3((unsigned)grid), dim3(kBlock), 0, st, a); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
}

template <typename T>
hipError_t launch_tie_gate_t(const pyas_partial *fin, int64_t n, uint32_t which, uint32_t *gate, hipStream_t st) {
    if constexpr (TT<T>::kind != 0) {
        return hipSuccess;
    } else {
        int64_t blocks = (n + kBlock - 1) / kBlock;
        blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
        hipLaunchKernelGGL((k_tie_gate<T>), dim3((unsigned)blocks), dim3(kBlock), 0, st, fin, n, which, gate);
        return hipGetLastError();
    }
}

template <typename T>
hipError_t launch_tie_pick_t(const pyas_partial *parts, int64_t n, uint32_t which, int64_t base, const TieCall &call,
                             const TieRule &t, uint64_t *keys, hipStream_t st) {
    if constexpr (TT<T>::kind != 0) {
        return hipSuccess;
    } else {
        int64_t blocks = (n + kBlock - 1) / kBlock;
        blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
        hipLaunchKernelGGL((k_tie_pick<T>), dim3((unsigned)blocks), dim3(kBlock), 0, st, parts, n, which, base,
                           call, t, keys);
        return hipGetLastError();
    }
}

template <typename T>
hipError_t launch_tie_grid_t(const TieGridArgs &a, hipStream_t st) {
    if constexpr (TT<T>::kind != 0) {
        return hipSuccess;
    } else {
        if (a.per_thread) {
            const int64_t blocks = (a.n_out + kBlock - 1) / kBlock;
            hipLaunchKernelGGL((k_tie_grid_t<T>), dim3((unsigned)blocks), dim3(kBlock), 0, st, a);
            return hipGetLastError();
        }
        const int64_t waves = a.n_out * a.slices;
        const int64_t blocks = (waves + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((k_tie_grid<T>), dim3((unsigned)blocks), dim3(kBlock), 0, st, a);
        return hipGetLastError();
    }
}

template <typename T>
hipError_t launch_tie_finalize_t(const uint64_t *keys, int64_t n_out, int32_t n_sets, const TieCall &call,
                                 const TieRule &t, uint32_t which, pyas_partial *fin, hipStream_t st) {
    if constexpr (TT<T>::kind != 0) {
        return hipSuccess;
    } else {
        const int64_t blocks = (n_out + kBlock - 1) / kBlock;
        hipLaunchKernelGGL((k_tie_finalize<T>), dim3((unsigned)blocks), dim3(kBlock), 0, st, keys, n_out, n_sets,
                           call, t, which, fin);
        return hipGetLastError();
    }
}

// ---------------------------------------------------------------------------
// per-dtype launchers (declared in pyas_internal.hpp)
// ---------------------------------------------------------------------------
// Kernel mask mode for the scalar rules left in m (prepare() has dropped
// equality rules a threshold already covers): 0 unmasked, kMaskRange
// thresholds only, kMaskNoEq1 one equality interval + thresholds, kMaskAll.
inline int mask_mode(const pyas_mask &m, bool masked) {
    if (!masked) return 0;
    const uint32_t f = m.flags;
    if (f & (PYAS_MASK_TAB0 | PYAS_MASK_TAB1)) return kMaskAll;
    if (!(f & (PYAS_MASK_EQ0 | PYAS_MASK_EQ1))) return kMaskRange;
    if (!(f & PYAS_MASK_EQ1)) return kMaskNoEq1;
    return kMaskAll;
}

template <typename T, bool SEL>
static void launch_reduce_ts(const ReduceArgs &a, bool shuf, bool bsw, bool masked, dim3 g,
                             hipStream_t st) {
    const dim3 blk(kBlock);
#define PYAS_L(S, B, M)                                                                \
    do {                                                                               \
        if constexpr (SEL || sizeof(T) < 4)                                            \
            hipLaunchKernelGGL((k_reduce_u<T, S, B, M, SEL>), g, blk, 0, st, a);       \
        else hipLaunchKernelGGL((k_reduce<T, S, B, M>), g, blk, 0, st, a);             \
    } while (0)
    // the lean kernel also has variants with fewer rules (mask_mode)
    const int mm = mask_mode(a.mask, masked);
    if constexpr (sizeof(T) == 1) {
        if (masked) PYAS_L(false, false, kMaskAll);
        else PYAS_L(false, false, 0);
    } else if constexpr (sizeof(T) >= 4) {
        // the trimmed mask modes for the selection kernel too (a cut
        // chunk's predicate stream with all six compares was VALU-bound:
        // C3 [1:1023]^3 k_reduce_u 1.11 ms)
#define PYAS_LM(S, B)                                                 \
        do {                                                          \
            if (!mm) PYAS_L(S, B, 0);                                 \
            else if (mm == kMaskRange) PYAS_L(S, B, kMaskRange);      \
            else if (mm == kMaskNoEq1) PYAS_L(S, B, kMaskNoEq1);      \
            else PYAS_L(S, B, kMaskAll);                              \
        } while (0)
        if (shuf) { if (bsw) PYAS_LM(true, true); else PYAS_LM(true, false); }
        else { if (bsw) PYAS_LM(false, true); else PYAS_LM(false, false); }
#undef PYAS_LM
    } else {
        (void)mm;
        if (shuf) {
            if (bsw) { if (masked) PYAS_L(true, true, kMaskAll); else PYAS_L(true, true, 0); }
            else { if (masked) PYAS_L(true, false, kMaskAll); else PYAS_L(true, false, 0); }
        } else {
            if (bsw) { if (masked) PYAS_L(false, true, kMaskAll); else PYAS_L(false, true, 0); }
            else { if (masked) PYAS_L(false, false, kMaskAll); else PYAS_L(false, false, 0); }
        }
    }
#undef PYAS_L
}

template <typename T>
hipError_t launch_reduce_t(const ReduceArgs &a, bool shuf, bool bsw, bool masked, int64_t grid,
                           hipStream_t st) {
    const dim3 g((unsigned)grid);
    // vector fill/missing tables are applied by the selection-aware path only
    // (a NULL table there means every chunk whole)
    const bool sel = a.sel || a.tab.on[0] || a.tab.on[1];
    if (sel) {
        launch_reduce_ts<T, true>(a, shuf, bsw, masked, g, st);
    } else {
        launch_reduce_ts<T, false>(a, shuf, bsw, masked, g, st);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_finish_t(const FinishArgs &f, hipStream_t st) {
    const int64_t ng = (f.n_chunks + kCombineSeg - 1) / kCombineSeg;
    hipLaunchKernelGGL((k_finish<T>), dim3((unsigned)ng), dim3(kBlock), 0, st, f);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_combine_t(const pyas_partial *in, int64_t n, int64_t seg, int64_t nblocks,
                            uint32_t flags, pyas_partial *out, hipStream_t st) {
    hipLaunchKernelGGL((k_combine<T>), dim3((unsigned)nblocks), dim3(kBlock), 0, st, in, n, seg,
                       flags, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_combine_segments_t(const pyas_partial *in, const int64_t *index,
                                     const int64_t *seg, int64_t n_seg, uint32_t flags,
                                     pyas_partial *out, hipStream_t st) {
    const dim3 g((unsigned)((n_seg + kBlock - 1) / kBlock)), blk(kBlock);
    hipLaunchKernelGGL((k_combine_segments<T>), g, blk, 0, st, in, index, seg, n_seg, flags, out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_combine_grid_t(const pyas_partial *in, const pyas_grid &g, const CombineTie &ct, int64_t n_out,
                                 int64_t n_layers, uint32_t flags, pyas_partial *out,
                                 hipStream_t st) {
    const dim3 blk(kBlock);
    if (n_layers >= kCombineWaveMinLayers && n_layers < (int64_t(1) << 31) && n_out <= kCombineWaveMaxOut &&
        !(flags & kCombineThreadOnly)) {   // (the wave form decodes layer ids in 32 bits)
        constexpr int64_t wpb = kBlock / kWave;
        const dim3 grid((unsigned)((n_out + wpb - 1) / wpb));
        hipLaunchKernelGGL((k_combine_grid_wave<T>), grid, blk, 0, st, in, g, n_out, n_layers, flags, out);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((n_out + kBlock - 1) / kBlock));
    // the keyed form only when level 2 is keyed: its keys cost the plain
    // combine 49 -> 71 us on the C3 slab (2,) (profiles/r06/zeros2)
    if (ct.on) hipLaunchKernelGGL((k_combine_grid<T, true>), grid, blk, 0, st, in, g, ct, n_out, n_layers, flags, out);
    else hipLaunchKernelGGL((k_combine_grid<T, false>), grid, blk, 0, st, in, g, ct, n_out, n_layers, flags, out);
    return hipGetLastError();
}

// Mask modes: all four for little-endian >= 4-byte data, {0, kMaskAll}
// for byte-swapped or narrow data (fewer instantiations; same results).
template <typename T, bool SHUF, bool BSWAP, int MASKED, int MODE>
static void launch_dense_k(const AxesArgs &a, dim3 g, hipStream_t st) {
    const dim3 blk(kBlock);
    if constexpr (TT<T>::kind == 0 && (MODE == 1 || MODE >= 4)) {
        if (a.zs) {   // the host admits zero-sign keying for these layouts only
            if constexpr (MODE == 1) hipLaunchKernelGGL((k_axes_dense_col_zs<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
            else hipLaunchKernelGGL((k_axes_dense_lds_zs<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
            return;
        }
    }
    if (a.cuts) {   // the batch's cut chunks too (every mask mode: kMaskAll cost C3 (2,) ~2x)
        if constexpr (MODE == 1) hipLaunchKernelGGL((k_axes_dense_col_cut<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
        else if constexpr (MODE >= 4) hipLaunchKernelGGL((k_axes_dense_lds_cut<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
        else hipLaunchKernelGGL((k_axes_dense_row_cut<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
        return;
    }
    if constexpr (MODE == 1) hipLaunchKernelGGL((k_axes_dense_col<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
    else if constexpr (MODE >= 4) hipLaunchKernelGGL((k_axes_dense_lds<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
    else hipLaunchKernelGGL((k_axes_dense_row<T, SHUF, BSWAP, MASKED, MODE>), g, blk, 0, st, a);
}

template <typename T, bool SHUF, int MODE>
static void launch_dense_ms(const AxesArgs &a, bool masked, dim3 g, hipStream_t st) {
    const int mm = mask_mode(a.r.mask, masked);
    if (a.bswap && sizeof(T) > 1) {
        if (mm) launch_dense_k<T, SHUF, true, kMaskAll, MODE>(a, g, st);
        else launch_dense_k<T, SHUF, true, 0, MODE>(a, g, st);
        return;
    }
    if constexpr (sizeof(T) >= 4) {
        if (mm == kMaskRange) { launch_dense_k<T, SHUF, false, kMaskRange, MODE>(a, g, st); return; }
        if (mm == kMaskNoEq1) { launch_dense_k<T, SHUF, false, kMaskNoEq1, MODE>(a, g, st); return; }
    }
    if (mm) launch_dense_k<T, SHUF, false, kMaskAll, MODE>(a, g, st);
    else launch_dense_k<T, SHUF, false, 0, MODE>(a, g, st);
}

template <typename T, int MODE>
static void launch_dense_m(const AxesArgs &a, bool masked, dim3 g, hipStream_t st) {
    if constexpr (sizeof(T) > 1) {
        if (a.shuf) { launch_dense_ms<T, true, MODE>(a, masked, g, st); return; }
    }
    launch_dense_ms<T, false, MODE>(a, masked, g, st);
}

template <typename T, bool SHUF, int NV>
static void launch_col_stream(const AxesArgs &a, bool masked, dim3 gr, hipStream_t st) {
    const dim3 blk(kBlock);
    const int mm = mask_mode(a.r.mask, masked);
    if (a.bswap) {
        if (mm) hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, true, kMaskAll, NV>), gr, blk, 0, st, a);
        else hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, true, 0, NV>), gr, blk, 0, st, a);
    } else if (mm == kMaskRange) {
        hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, false, kMaskRange, NV>), gr, blk, 0, st, a);
    } else if (mm == kMaskNoEq1) {
        hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, false, kMaskNoEq1, NV>), gr, blk, 0, st, a);
    } else {
        if (mm) hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, false, kMaskAll, NV>), gr, blk, 0, st, a);
        else hipLaunchKernelGGL((k_axes_col_stream<T, SHUF, false, 0, NV>), gr, blk, 0, st, a);
    }
}

template <typename T, int KPL>
static void launch_shuf_slab(const AxesArgs &a, bool masked, dim3 gr, hipStream_t st) {
    const dim3 blk(kBlock);
    const int mm = mask_mode(a.r.mask, masked);
    if (a.bswap) {
        if (mm) hipLaunchKernelGGL((k_axes_shuf_slab<T, true, kMaskAll, KPL>), gr, blk, 0, st, a);
        else hipLaunchKernelGGL((k_axes_shuf_slab<T, true, 0, KPL>), gr, blk, 0, st, a);
    } else if (mm == kMaskRange) {
        hipLaunchKernelGGL((k_axes_shuf_slab<T, false, kMaskRange, KPL>), gr, blk, 0, st, a);
    } else if (mm == kMaskNoEq1) {
        hipLaunchKernelGGL((k_axes_shuf_slab<T, false, kMaskNoEq1, KPL>), gr, blk, 0, st, a);
    } else {
        if (mm) hipLaunchKernelGGL((k_axes_shuf_slab<T, false, kMaskAll, KPL>), gr, blk, 0, st, a);
        else hipLaunchKernelGGL((k_axes_shuf_slab<T, false, 0, KPL>), gr, blk, 0, st, a);
    }
}

template <typename T>
hipError_t launch_axes_dense_t(const AxesArgs &a, bool masked, int64_t grid, hipStream_t st) {
    const dim3 g((unsigned)grid);
    if constexpr (sizeof(T) >= 2) {
        if (a.d.mode == 1 && a.d.rb > 0 && a.shuf) {   // k_axes_shuf_slab (host: RO == 1, whole chunks)
            if (a.d.KI == 64) launch_shuf_slab<T, 1>(a, masked, g, st);
            else launch_shuf_slab<T, 2>(a, masked, g, st);
            return hipGetLastError();
        }
    }
    if constexpr (sizeof(T) >= 4) {
        if (a.d.mode == 1 && a.d.cpb > 0) {   // k_axes_col_stream (host: split 1, whole chunks)
            // host: shuffled chunks stream with one item per lane, plain
            // ones with 2 or 4
            if (a.shuf) launch_col_stream<T, true, 1>(a, masked, g, st);
            else if (a.d.nv == 4) launch_col_stream<T, false, 4>(a, masked, g, st);
            else launch_col_stream<T, false, 2>(a, masked, g, st);
            return hipGetLastError();
        }
    }
    if (a.d.mode == 1) launch_dense_m<T, 1>(a, masked, g, st);
    else return launch_axes_dense_rows_t<T>(a, masked, grid, st);   // separate object (build time)
    return hipGetLastError();
}

// The row layouts (modes 2-6) of launch_axes_dense_t, instantiated in their
// own object per dtype so the build runs them in parallel.
template <typename T>
hipError_t launch_axes_dense_rows_t(const AxesArgs &a, bool masked, int64_t grid, hipStream_t st) {
    const dim3 g((unsigned)grid);
    if (a.d.mode == 2) launch_dense_m<T, 2>(a, masked, g, st);
    else if (a.d.mode == 4) launch_dense_m<T, 4>(a, masked, g, st);
    else if (a.d.mode == 5) launch_dense_m<T, 5>(a, masked, g, st);
    else if (a.d.mode == 6) launch_dense_m<T, 6>(a, masked, g, st);
    else launch_dense_m<T, 3>(a, masked, g, st);
    return hipGetLastError();
}

template <typename T, bool SHUF, int H, bool ZS>
static void launch_fold_row_s(const AxesArgs &a, const FoldGrid &g, bool masked, dim3 gr, hipStream_t st) {
    const dim3 blk(kBlock);
    const int mm = mask_mode(a.r.mask, masked);
    if (a.bswap) {
        if (mm) hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, true, kMaskAll, H, ZS>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, true, 0, H, ZS>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskRange) {
        hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, false, kMaskRange, H, ZS>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskNoEq1) {
        hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, false, kMaskNoEq1, H, ZS>), gr, blk, 0, st, a, g);
    } else {
        if (mm) hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, false, kMaskAll, H, ZS>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold_row<T, SHUF, false, 0, H, ZS>), gr, blk, 0, st, a, g);
    }
}

template <typename T, int H>
static void launch_fold_row(const AxesArgs &a, const FoldGrid &g, bool masked, dim3 gr, hipStream_t st) {
    if constexpr (TT<T>::kind == 0) {   // signed zeros: floats only
        if (g.zs) {
            if (a.shuf) launch_fold_row_s<T, true, H, true>(a, g, masked, gr, st);
            else launch_fold_row_s<T, false, H, true>(a, g, masked, gr, st);
            return;
        }
    }
    if (a.shuf) launch_fold_row_s<T, true, H, false>(a, g, masked, gr, st);
    else launch_fold_row_s<T, false, H, false>(a, g, masked, gr, st);
}

template <typename T, bool SHUF, bool ZS>
static void launch_fold_lean_z(const AxesArgs &a, const FoldGrid &g, bool masked, dim3 gr, hipStream_t st) {
    const dim3 blk(kBlock);
    const int mm = mask_mode(a.r.mask, masked);
    if (a.bswap) {
        if (mm) hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, true, kMaskAll, ZS>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, true, 0, ZS>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskRange) {
        hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, false, kMaskRange, ZS>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskNoEq1) {
        hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, false, kMaskNoEq1, ZS>), gr, blk, 0, st, a, g);
    } else {
        if (mm) hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, false, kMaskAll, ZS>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold_lean<T, SHUF, false, 0, ZS>), gr, blk, 0, st, a, g);
    }
}

template <typename T, bool SHUF>
static void launch_fold_lean(const AxesArgs &a, const FoldGrid &g, bool masked, dim3 gr, hipStream_t st) {
    if constexpr (TT<T>::kind == 0) {   // signed zeros: floats only
        if (g.zs) {
            launch_fold_lean_z<T, SHUF, true>(a, g, masked, gr, st);
            return;
        }
    }
    launch_fold_lean_z<T, SHUF, false>(a, g, masked, gr, st);
}

template <typename T, bool SHUF>
static void launch_fold_col(const AxesArgs &a, const FoldGrid &g, bool masked, dim3 gr, hipStream_t st) {
    const dim3 blk(kBlock);
    const int mm = mask_mode(a.r.mask, masked);
    if (g.lean) {
        launch_fold_lean<T, SHUF>(a, g, masked, gr, st);
    } else if (a.bswap) {
        if (mm) hipLaunchKernelGGL((k_axes_fold<T, SHUF, true, kMaskAll>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold<T, SHUF, true, 0>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskRange) {
        hipLaunchKernelGGL((k_axes_fold<T, SHUF, false, kMaskRange>), gr, blk, 0, st, a, g);
    } else if (mm == kMaskNoEq1) {
        hipLaunchKernelGGL((k_axes_fold<T, SHUF, false, kMaskNoEq1>), gr, blk, 0, st, a, g);
    } else {
        if (mm) hipLaunchKernelGGL((k_axes_fold<T, SHUF, false, kMaskAll>), gr, blk, 0, st, a, g);
        else hipLaunchKernelGGL((k_axes_fold<T, SHUF, false, 0>), gr, blk, 0, st, a, g);
    }
}

template <typename T>
hipError_t launch_axes_fold_t(const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                              hipStream_t st) {
    const dim3 gr((unsigned)grid);
    if constexpr (sizeof(T) < 4) {
        return hipErrorInvalidValue;     // dense_geometry: >= 4-byte elements only
    } else if (a.d.mode >= 4) {
        return launch_axes_fold_rows_t<T>(a, g, masked, grid, st);   // separate object (build time)
    } else {
        if (a.shuf) launch_fold_col<T, true>(a, g, masked, gr, st);
        else launch_fold_col<T, false>(a, g, masked, gr, st);
    }
    return hipGetLastError();
}

// The LDS row fold (modes 4-6) of launch_axes_fold_t, in its own object.
template <typename T>
hipError_t launch_axes_fold_rows_t(const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                                   hipStream_t st) {
    const dim3 gr((unsigned)grid);
    if constexpr (sizeof(T) < 4) {
        return hipErrorInvalidValue;
    } else {
        if (a.d.mode == 4) launch_fold_row<T, 1>(a, g, masked, gr, st);
        else if (a.d.mode == 5) launch_fold_row<T, 2>(a, g, masked, gr, st);
        else launch_fold_row<T, 4>(a, g, masked, gr, st);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_axes_t(const AxesArgs &a, int64_t grid, hipStream_t st) {
    const dim3 g((unsigned)grid), blk(kBlock);
    const int cap = a.roff_cap < 0 ? 0 : (a.roff_cap > kAxesLds ? kAxesLds : a.roff_cap);
    AxesArgs b = a;
    b.roff_cap = cap;
    const size_t lds = (size_t)(cap > 0 ? cap : 1) * sizeof(int32_t);
    if constexpr (sizeof(T) == 1) {
        hipLaunchKernelGGL((k_reduce_axes<T, false, false>), g, blk, lds, st, b);
    } else {
        if (a.shuf && a.bswap) hipLaunchKernelGGL((k_reduce_axes<T, true, true>), g, blk, lds, st, b);
        else if (a.shuf) hipLaunchKernelGGL((k_reduce_axes<T, true, false>), g, blk, lds, st, b);
        else if (a.bswap) hipLaunchKernelGGL((k_reduce_axes<T, false, true>), g, blk, lds, st, b);
        else hipLaunchKernelGGL((k_reduce_axes<T, false, false>), g, blk, lds, st, b);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_select_t(const SelectArgs &a, int64_t grid, hipStream_t st) {
    hipLaunchKernelGGL((k_select<T>), dim3((unsigned)grid), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// result formatting (pyas_format_partials): active.py:591-630 on the device
// ---------------------------------------------------------------------------
// One thread per combined partial.  values receives what Active._format puts
// in the masked result, mask one byte per element (1 = masked):
//   M_SUM  : the sum in the variable dtype (floats) or int64/uint64 (ints);
//   M_MIN/M_MAX: the value in the variable dtype;
//   M_MEAN : np.ma's `out / n` (_DomainedBinaryOperation with
//            _DomainSafeDivide): r = f64(out) / f64(n); masked where n == 0,
//            r is not finite, or |out| * finfo(float).tiny >= |n|; a masked
//            element holds 0.0 + f64(out) (np.copyto 0, then += m * out).
template <typename T, int M>
__global__ __launch_bounds__(kBlock) void k_format(const pyas_partial *in, int64_t n, void *values,
                                                   uint8_t *mask, int64_t *counts) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    using S = typename std::conditional<TT<T>::kind == 0, T,
              typename std::conditional<TT<T>::kind == 1, int64_t, uint64_t>::type>::type;
    const pyas_partial p = in[i];
    const int64_t cnt = p.count;
    if (counts) counts[i] = cnt;
    bool m = cnt == 0;
    if constexpr (M == PYAS_FORMAT_MIN || M == PYAS_FORMAT_MAX) {
        static_cast<T *>(values)[i] = TT<T>::from(M == PYAS_FORMAT_MIN ? p.min : p.max);
    } else {
        S v;
        if constexpr (TT<T>::kind == 0) v = (T)p.sum.f;
        else if constexpr (TT<T>::kind == 1) v = p.sum.i;
        else v = p.sum.u;
        if constexpr (M == PYAS_FORMAT_SUM) {
            static_cast<S *>(values)[i] = v;
        } else {
            const double da = (double)v;
            double r = da / (double)cnt;
            double av;                                   // np.absolute(out) as f64
            if constexpr (TT<T>::kind == 0) av = __builtin_fabs(da);
            else if constexpr (TT<T>::kind == 1) av = (double)(v < 0 ? (int64_t)(0ull - (uint64_t)v) : v);
            else av = da;
            const double tiny = 2.2250738585072014e-308;
            m = m || !__builtin_isfinite(r) || av * tiny >= (double)(cnt < 0 ? -cnt : cnt);
            if (m) r = 0.0 + da;
            static_cast<double *>(values)[i] = r;
        }
    }
    mask[i] = m ? 1 : 0;
}

template <typename T>
hipError_t launch_format_t(const pyas_partial *in, int64_t n, int32_t method, void *values,
                           uint8_t *mask, int64_t *counts, hipStream_t st) {
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock)), blk(kBlock);
    switch (method) {
        case PYAS_FORMAT_SUM:
            hipLaunchKernelGGL((k_format<T, PYAS_FORMAT_SUM>), grid, blk, 0, st, in, n, values, mask, counts);
            break;
        case PYAS_FORMAT_MIN:
            hipLaunchKernelGGL((k_format<T, PYAS_FORMAT_MIN>), grid, blk, 0, st, in, n, values, mask, counts);
            break;
        case PYAS_FORMAT_MAX:
            hipLaunchKernelGGL((k_format<T, PYAS_FORMAT_MAX>), grid, blk, 0, st, in, n, values, mask, counts);
            break;
        case PYAS_FORMAT_MEAN:
            hipLaunchKernelGGL((k_format<T, PYAS_FORMAT_MEAN>), grid, blk, 0, st, in, n, values, mask, counts);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Explicit instantiation of every launcher for one dtype (pyas_inst.hip), in
// three parts compiled as separate objects (the build runs them in parallel):
// 1 the streaming reduce, combines, select, format and the generic axes
// kernel; 2 the dense partial-axis kernels; 3 the in-kernel layer folds.
#define PYAS_INSTANTIATE_PART1(T)                                                              \
    template hipError_t launch_reduce_t<T>(const ReduceArgs &, bool, bool, bool, int64_t,     \
                                           hipStream_t);                                      \
    template hipError_t launch_finish_t<T>(const FinishArgs &, hipStream_t);                  \
    template hipError_t launch_combine_t<T>(const pyas_partial *, int64_t, int64_t, int64_t,  \
                                            uint32_t, pyas_partial *, hipStream_t);           \
    template hipError_t launch_combine_segments_t<T>(const pyas_partial *, const int64_t *,   \
                                                     const int64_t *, int64_t, uint32_t,     \
                                                     pyas_partial *, hipStream_t);           \
    template hipError_t launch_axes_t<T>(const AxesArgs &, int64_t, hipStream_t);             \
    template hipError_t launch_combine_grid_t<T>(const pyas_partial *, const pyas_grid &,     \
                                                 const CombineTie &,                          \
                                                 int64_t, int64_t, uint32_t, pyas_partial *,  \
                                                 hipStream_t);                               \
    template hipError_t launch_select_t<T>(const SelectArgs &, int64_t, hipStream_t);         \
    template hipError_t launch_format_t<T>(const pyas_partial *, int64_t, int32_t, void *,    \
                                           uint8_t *, int64_t *, hipStream_t);                \
    template hipError_t launch_tie_chunks_t<T>(const TieChunkArgs &, int64_t, hipStream_t);      \
    template hipError_t launch_tie_gate_t<T>(const pyas_partial *, int64_t, uint32_t, uint32_t *,  \
                                             hipStream_t);                                       \
    template hipError_t launch_tie_grid_t<T>(const TieGridArgs &, hipStream_t);                   \
    template hipError_t launch_tie_pick_t<T>(const pyas_partial *, int64_t, uint32_t, int64_t,     \
                                             const TieCall &, const TieRule &, uint64_t *, hipStream_t); \
    template hipError_t launch_tie_finalize_t<T>(const uint64_t *, int64_t, int32_t, const TieCall &, \
                                                 const TieRule &, uint32_t, pyas_partial *, hipStream_t);
#define PYAS_INSTANTIATE_PART2(T)                                                              \
    extern template hipError_t launch_axes_dense_rows_t<T>(const AxesArgs &, bool, int64_t,     \
                                                           hipStream_t); /* part 4 */         \
    template hipError_t launch_axes_dense_t<T>(const AxesArgs &, bool, int64_t, hipStream_t);
#define PYAS_INSTANTIATE_PART3(T)                                                              \
    extern template hipError_t launch_axes_fold_rows_t<T>(const AxesArgs &, const FoldGrid &,   \
                                                          bool, int64_t, hipStream_t); /* part 5 */ \
    template hipError_t launch_axes_fold_t<T>(const AxesArgs &, const FoldGrid &, bool, int64_t, \
                                              hipStream_t);
#define PYAS_INSTANTIATE_PART4(T)                                                              \
    template hipError_t launch_axes_dense_rows_t<T>(const AxesArgs &, bool, int64_t, hipStream_t);
#define PYAS_INSTANTIATE_PART5(T)                                                              \
    template hipError_t launch_axes_fold_rows_t<T>(const AxesArgs &, const FoldGrid &, bool, int64_t, \
                                                   hipStream_t);

}  // namespace pyas
