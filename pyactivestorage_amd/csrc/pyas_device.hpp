// pyas_device.hpp — device-side building blocks of the gfx950 chunk reducer.
//
// The per-element pipeline restated from the reference (storage.py:55-100):
//   raw bytes --(un-shuffle, storage.py:121-122 / numcodecs Shuffle.decode)-->
//   element bits --(byte order from dtype, storage.py:59 .view(dtype))-->
//   value --(mask_missing, storage.py:126-153)--> (sum, count, min, max).
// All of it happens in registers: the chunk bytes are read from HBM once.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pyas.h"

namespace pyas {

constexpr int kBlock = 256;   // 4 wave64 per workgroup
constexpr int kWave = 64;

// Type-generic lane exchange: moves the bits as 32-bit words (ds_swizzle /
// DPP under the hood), so 1/2/4/8-byte values all take the same path.
template <typename V>
__device__ __forceinline__ V shfl_xor(V v, int m) {
    if constexpr (sizeof(V) <= 4) {
        uint32_t w = 0;
        __builtin_memcpy(&w, &v, sizeof(V));
        w = (uint32_t)__shfl_xor((int)w, m, kWave);
        V r;
        __builtin_memcpy(&r, &w, sizeof(V));
        return r;
    } else {
        uint32_t w[2];
        __builtin_memcpy(w, &v, 8);
        w[0] = (uint32_t)__shfl_xor((int)w[0], m, kWave);
        w[1] = (uint32_t)__shfl_xor((int)w[1], m, kWave);
        V r;
        __builtin_memcpy(&r, w, 8);
        return r;
    }
}


// ---------------------------------------------------------------------------
// dtype traits
// ---------------------------------------------------------------------------
template <typename T> struct TT;
#define PYAS_INT_TRAITS(TYPE, UTYPE, ACC, KIND, LO, HI)                        \
    template <> struct TT<TYPE> {                                              \
        using U = UTYPE;                                                       \
        using Acc = ACC;                                                       \
        static constexpr int kind = KIND; /* 1 signed, 2 unsigned */           \
        __device__ static TYPE lowest() { return LO; }                         \
        __device__ static TYPE highest() { return HI; }                        \
        __device__ static TYPE from(pyas_scalar s) {                           \
            return KIND == 1 ? (TYPE)s.i : (TYPE)s.u;                          \
        }                                                                      \
        __device__ static void put(pyas_scalar &s, TYPE v) {                   \
            if (KIND == 1) s.i = (int64_t)v; else s.u = (uint64_t)v;           \
        }                                                                      \
        __device__ static void put_acc(pyas_scalar &s, ACC v) {                \
            if (KIND == 1) s.i = (int64_t)v; else s.u = (uint64_t)v;           \
        }                                                                      \
    };
PYAS_INT_TRAITS(int8_t, uint8_t, int64_t, 1, INT8_MIN, INT8_MAX)
PYAS_INT_TRAITS(uint8_t, uint8_t, uint64_t, 2, 0, UINT8_MAX)
PYAS_INT_TRAITS(int16_t, uint16_t, int64_t, 1, INT16_MIN, INT16_MAX)
PYAS_INT_TRAITS(uint16_t, uint16_t, uint64_t, 2, 0, UINT16_MAX)
PYAS_INT_TRAITS(int32_t, uint32_t, int64_t, 1, INT32_MIN, INT32_MAX)
PYAS_INT_TRAITS(uint32_t, uint32_t, uint64_t, 2, 0, UINT32_MAX)
PYAS_INT_TRAITS(int64_t, uint64_t, int64_t, 1, INT64_MIN, INT64_MAX)
PYAS_INT_TRAITS(uint64_t, uint64_t, uint64_t, 2, 0, UINT64_MAX)
#undef PYAS_INT_TRAITS

template <> struct TT<float> {
    using U = uint32_t;
    using Acc = double;
    static constexpr int kind = 0;
    __device__ static float lowest() { return -__builtin_inff(); }
    __device__ static float highest() { return __builtin_inff(); }
    __device__ static float from(pyas_scalar s) { return (float)s.f; }
    __device__ static void put(pyas_scalar &s, float v) { s.f = (double)v; }
    __device__ static void put_acc(pyas_scalar &s, double v) { s.f = v; }
};
template <> struct TT<double> {
    using U = uint64_t;
    using Acc = double;
    static constexpr int kind = 0;
    __device__ static double lowest() { return -__builtin_inf(); }
    __device__ static double highest() { return __builtin_inf(); }
    __device__ static double from(pyas_scalar s) { return s.f; }
    __device__ static void put(pyas_scalar &s, double v) { s.f = v; }
    __device__ static void put_acc(pyas_scalar &s, double v) { s.f = v; }
};

__device__ __forceinline__ uint8_t bswap(uint8_t x) { return x; }
__device__ __forceinline__ uint16_t bswap(uint16_t x) { return __builtin_bswap16(x); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap(uint64_t x) { return __builtin_bswap64(x); }

template <typename T, typename U>
__device__ __forceinline__ T bits_to(U u) {
    static_assert(sizeof(T) == sizeof(U), "size");
    T t;
    __builtin_memcpy(&t, &u, sizeof(T));
    return t;
}

// ---------------------------------------------------------------------------
// element loaders
// ---------------------------------------------------------------------------
// Plain layout: element i at base + i*ES (offset is ES-aligned by contract).
template <typename T, bool BSWAP>
__device__ __forceinline__ T load_plain(const uint8_t *base, int64_t i) {
    using U = typename TT<T>::U;
    U u = *reinterpret_cast<const U *>(base + i * (int64_t)sizeof(T));
    if (BSWAP) u = bswap(u);
    return bits_to<T>(u);
}

// HDF5 shuffle layout (numcodecs Shuffle, elementsize == sizeof(T)):
// byte b of element i lives at base + b*n + i, n = elements in the chunk.
template <typename T, bool BSWAP>
__device__ __forceinline__ T load_shuffled(const uint8_t *base, int64_t n, int64_t i) {
    using U = typename TT<T>::U;
    constexpr int ES = sizeof(T);
    U u = 0;
#pragma unroll
    for (int b = 0; b < ES; ++b) {
        const U byte = (U)base[(int64_t)b * n + i];
        const int sh = BSWAP ? 8 * (ES - 1 - b) : 8 * b;
        u |= byte << sh;
    }
    return bits_to<T>(u);
}

template <typename T, bool SHUF, bool BSWAP>
__device__ __forceinline__ T load_elem(const uint8_t *base, int64_t n, int64_t i) {
    if constexpr (SHUF && sizeof(T) > 1) return load_shuffled<T, BSWAP>(base, n, i);
    else return load_plain<T, BSWAP>(base, i);
}

// Runtime-flagged loader for the non-hot kernels (axis / select).
template <typename T>
__device__ __forceinline__ T load_elem_rt(const uint8_t *base, int64_t n, int64_t i,
                                          bool shuf, bool bsw) {
    if (shuf) return bsw ? load_shuffled<T, true>(base, n, i) : load_shuffled<T, false>(base, n, i);
    return bsw ? load_plain<T, true>(base, i) : load_plain<T, false>(base, i);
}

// ---------------------------------------------------------------------------
// mask (compiled mask_missing, storage.py:126-153)
// ---------------------------------------------------------------------------
constexpr int kMaskAll = 1, kMaskNoEq1 = 2, kMaskRange = 3;

template <typename T> struct MaskT {
    T lo0, hi0, lo1, hi1, gt, lt;
    __device__ void init(const pyas_mask &m) {
        const T big = TT<T>::highest(), small = TT<T>::lowest();
        if (m.flags & PYAS_MASK_EQ0) { lo0 = TT<T>::from(m.eq_lo[0]); hi0 = TT<T>::from(m.eq_hi[0]); }
        else { lo0 = big; hi0 = small; }
        if (m.flags & PYAS_MASK_EQ1) { lo1 = TT<T>::from(m.eq_lo[1]); hi1 = TT<T>::from(m.eq_hi[1]); }
        else { lo1 = big; hi1 = small; }
        gt = (m.flags & PYAS_MASK_GT) ? TT<T>::from(m.gt) : big;
        lt = (m.flags & PYAS_MASK_LT) ? TT<T>::from(m.lt) : small;
    }
    // Branch-free: every rule evaluated with neutral thresholds when disabled.
    // NaN compares false everywhere, so it is never masked (np.ma semantics).
    __device__ __forceinline__ bool masked(T x) const {
        const bool e0 = (x >= lo0) & (x <= hi0);
        const bool e1 = (x >= lo1) & (x <= hi1);
        return e0 | e1 | (x > gt) | (x < lt);
    }
    // Kernel-level mask mode M (the MASKED template argument): 0 none,
    // kMaskAll every rule, kMaskNoEq1 without the second equality rule
    // (_FillValue inside the valid range: 4 fewer ops), kMaskRange the two
    // thresholds only (no equality rule left after mask_mode's trimming,
    // e.g. C3's _FillValue below valid_min: 2 compares per element).
    template <int M>
    __device__ __forceinline__ bool masked_m(T x) const {
        if constexpr (M == kMaskRange) return (x > gt) | (x < lt);
        else if constexpr (M == kMaskNoEq1) return ((x >= lo0) & (x <= hi0)) | (x > gt) | (x < lt);
        else return masked(x);
    }
};

// Vector fill/missing tables (broadcast equality, storage.py:133-143)
struct MaskTab {
    const pyas_scalar *lo[2];
    const pyas_scalar *hi[2];
    int64_t stride[2][PYAS_MAX_DIMS];
    bool on[2];
};

template <typename T>
__device__ __forceinline__ bool tab_masked(const MaskTab &t, int k, int64_t vidx, T x) {
    const T lo = TT<T>::from(t.lo[k][vidx]);
    const T hi = TT<T>::from(t.hi[k][vidx]);
    return (x >= lo) & (x <= hi);
}

// ---------------------------------------------------------------------------
// accumulator: sum / count / NaN-propagating min & max (np.ma.sum/min/max)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T pmin(T a, T x) {
    // NaN propagates: once a is NaN it stays; a NaN x replaces a.
    return (x < a || x != x) ? x : a;
}
template <typename T>
__device__ __forceinline__ T pmax(T a, T x) {
    return (x > a || x != x) ? x : a;
}

// C = uint32_t inside a tile (<= 2^31 elements), int64_t for combines.
template <typename T, typename C> struct AccT {
    typename TT<T>::Acc sum;
    C count;
    T mn, mx;
    __device__ void init() {
        sum = 0;
        count = 0;
        mn = TT<T>::highest();
        mx = TT<T>::lowest();
    }
    __device__ __forceinline__ void add_valid(T x) {
        sum += (typename TT<T>::Acc)x;
        count += 1;
        mn = pmin(mn, x);
        mx = pmax(mx, x);
    }
    // Select-based (no branch): a masked element contributes nothing.
    __device__ __forceinline__ void add_flag(T x, bool is_masked) {
        const bool v = !is_masked;
        sum += v ? (typename TT<T>::Acc)x : (typename TT<T>::Acc)0;
        count += v ? (C)1 : (C)0;
        mn = v ? pmin(mn, x) : mn;
        mx = v ? pmax(mx, x) : mx;
    }
    template <int MASKED>
    __device__ __forceinline__ void add(T x, const MaskT<T> &mk) {
        if constexpr (!MASKED) add_valid(x);
        else add_flag(x, mk.template masked_m<MASKED>(x));
    }
};
template <typename T> using Acc = AccT<T, uint32_t>;
template <typename T> using WAcc = AccT<T, int64_t>;

// ---------------------------------------------------------------------------
// Streaming-kernel accumulator.  Per lane: sum, NaN-free min/max (native
// v_min/v_max; a NaN is remembered in `nan` and forces min = max = NaN at
// the end, exactly np.ma.min/max's NaN propagation), count.  In converged
// code (every lane runs the same trip count) counts come from a 64-lane
// ballot popcount on the scalar unit (`ucount`, wave-uniform).
// ---------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ T tmin(T a, T b) {
    if constexpr (TT<T>::kind == 0) return __builtin_fmin(a, b);
    else return b < a ? b : a;
}
template <> __device__ __forceinline__ float tmin<float>(float a, float b) { return __builtin_fminf(a, b); }
template <typename T> __device__ __forceinline__ T tmax(T a, T b) {
    if constexpr (TT<T>::kind == 0) return __builtin_fmax(a, b);
    else return b > a ? b : a;
}
template <> __device__ __forceinline__ float tmax<float>(float a, float b) { return __builtin_fmaxf(a, b); }

// Type used to sum one 16-byte group before widening (exact for ints: at
// most 16 int8 / 8 int16 values; float32 groups of 4 add one f32 rounding
// per group, far inside the 1e-6 parity bound).
template <typename T> struct GroupSum { using type = typename TT<T>::Acc; };
template <> struct GroupSum<float> { using type = float; };
template <> struct GroupSum<int8_t> { using type = int32_t; };
template <> struct GroupSum<uint8_t> { using type = uint32_t; };
template <> struct GroupSum<int16_t> { using type = int32_t; };
template <> struct GroupSum<uint16_t> { using type = uint32_t; };

template <typename T> struct TileAcc {
    using S = typename TT<T>::Acc;
    S sum;
    T mn, mx;
    uint32_t count, ucount;
    bool nan;
    __device__ void init() {
        sum = 0;
        mn = TT<T>::highest();
        mx = TT<T>::lowest();
        count = 0;
        ucount = 0;
        nan = false;
    }
    // N values in groups of at most 4; CONV: all 64 lanes execute this call
    // (uniform trip count).  Floats: the NaN flag is taken from the group
    // sum, not per element: an unmasked NaN (NaN is never masked) makes the
    // group sum NaN, so only when some lane's group sum is NaN (a NaN, or
    // +inf + -inf) does the wave test that group's elements one by one.
    template <int N, int MASKED, bool CONV>
    __device__ __forceinline__ void add_n(const T *x, const MaskT<T> &mk) {
        if (__builtin_expect(__ballot(add_lazy<N, MASKED, CONV>(x, mk)) != 0, 0))   // wave-uniform, rare
            check_nan<N>(x);
    }
    // add_n without the NaN test: returns whether this lane must run
    // check_nan on x (the caller batches one ballot over several calls)
    template <int N, int MASKED, bool CONV>
    __device__ __forceinline__ bool add_lazy(const T *x, const MaskT<T> &mk) {
        constexpr int GS = N < 4 ? N : 4;
        static_assert(N % GS == 0, "add_n: N must be a multiple of the group size");
        bool bad = false;
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += GS) bad |= add_group<GS, MASKED, CONV>(x + k0, mk);
        return bad;
    }
    template <int N>
    __device__ __forceinline__ void check_nan(const T *x) {
        if constexpr (TT<T>::kind == 0) {
#pragma unroll
            for (int k = 0; k < N; ++k) nan |= (x[k] != x[k]);
        }
    }
    template <int N, int MASKED, bool CONV>
    __device__ __forceinline__ bool add_group(const T *x, const MaskT<T> &mk) {
        using G = typename GroupSum<T>::type;
        G g = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const T v = x[k];
            if constexpr (MASKED) {
                const bool ok = !mk.template masked_m<MASKED>(v);
                if constexpr (TT<T>::kind == 0) {
                    const T y = ok ? v : (T)__builtin_nan("");  // v_min/v_max skip NaN
                    mn = tmin(mn, y);
                    mx = tmax(mx, y);
                } else {
                    mn = tmin(mn, ok ? v : TT<T>::highest());
                    mx = tmax(mx, ok ? v : TT<T>::lowest());
                }
                g += ok ? (G)v : (G)0;
                if constexpr (CONV) ucount += (uint32_t)__builtin_popcountll(__ballot(ok));
                else count += ok ? 1u : 0u;
            } else {
                mn = tmin(mn, v);
                mx = tmax(mx, v);
                g += (G)v;
            }
        }
        sum += (S)g;
        if constexpr (TT<T>::kind == 0) return g != g;
        else return false;
    }
    // N values of which only those whose bit is set in `sel` are selected
    // (run_spans' in-span predicate, the dense kernels' cut chunks).  CNT:
    // 0 the caller counts (unmasked tiles), 1 per-lane counts, 2 ballot
    // counts (converged code only).  Returns whether this lane must run
    // check_nan on its selected values.
    template <int N, int MASKED, int CNT = (MASKED ? 2 : 0)>
    __device__ __forceinline__ bool add_pred(const T *x, uint32_t sel, const MaskT<T> &mk) {
        using G = typename GroupSum<T>::type;
        constexpr int GS = N < 4 ? N : 4;
        bool bad = false;
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += GS) {
            G g = 0;
#pragma unroll
            for (int k = k0; k < k0 + GS; ++k) {
                const T v = x[k];
                bool ok = ((sel >> k) & 1u) != 0;
                if constexpr (MASKED) ok = ok && !mk.template masked_m<MASKED>(v);
                if constexpr (TT<T>::kind == 0) {
                    const T y = ok ? v : (T)__builtin_nan("");
                    mn = tmin(mn, y);
                    mx = tmax(mx, y);
                } else {
                    mn = tmin(mn, ok ? v : TT<T>::highest());
                    mx = tmax(mx, ok ? v : TT<T>::lowest());
                }
                g += ok ? (G)v : (G)0;
                if constexpr (CNT == 2) ucount += (uint32_t)__builtin_popcountll(__ballot(ok));
                else if constexpr (CNT == 1) count += ok ? 1u : 0u;
            }
            sum += (S)g;
            if constexpr (TT<T>::kind == 0) bad |= g != g;
        }
        return bad;
    }
    // one element with an externally computed mask bit (generic path)
    __device__ __forceinline__ void add_one(T v, bool is_masked) {
        if constexpr (TT<T>::kind == 0) nan |= (v != v);
        const bool ok = !is_masked;
        if constexpr (TT<T>::kind == 0) {
            const T y = ok ? v : (T)__builtin_nan("");
            mn = tmin(mn, y);
            mx = tmax(mx, y);
        } else {
            mn = tmin(mn, ok ? v : TT<T>::highest());
            mx = tmax(mx, ok ? v : TT<T>::lowest());
        }
        sum += ok ? (S)v : (S)0;
        count += ok ? 1u : 0u;
    }
};

// One lane's TileAcc -> pyas_partial (no cross-lane work).
template <typename T>
__device__ __forceinline__ void tile_store_lane(const TileAcc<T> &a, pyas_partial *out) {
    pyas_partial p;
    TT<T>::put_acc(p.sum, a.sum);
    p.count = (int64_t)a.count + (int64_t)a.ucount;
    T mn = a.mn, mx = a.mx;
    if constexpr (TT<T>::kind == 0) {
        if (a.nan) { mn = (T)__builtin_nan(""); mx = mn; }
    }
    TT<T>::put(p.min, mn);
    TT<T>::put(p.max, mx);
    *out = p;
}

// Wave reduction of TileAcc (every lane participates) -> lane 0 stores.
template <typename T>
__device__ __forceinline__ void wave_finish(TileAcc<T> &a, pyas_partial *out) {
    uint64_t c = (uint64_t)a.count;
    uint32_t nan = a.nan ? 1u : 0u;
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) {
        a.sum += shfl_xor(a.sum, m);
        c += shfl_xor(c, m);
        a.mn = tmin(a.mn, shfl_xor(a.mn, m));
        a.mx = tmax(a.mx, shfl_xor(a.mx, m));
        nan |= shfl_xor(nan, m);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) {
        a.count = (uint32_t)0;
        a.ucount = 0;
        a.nan = nan != 0;
        pyas_partial p;
        TT<T>::put_acc(p.sum, a.sum);
        p.count = (int64_t)c;
        T mn = a.mn, mx = a.mx;
        if constexpr (TT<T>::kind == 0) {
            if (nan) { mn = (T)__builtin_nan(""); mx = mn; }
        }
        TT<T>::put(p.min, mn);
        TT<T>::put(p.max, mx);
        *out = p;
    }
}

// Segmented reduction over aligned groups of G lanes (G power of two <= 64);
// the lane given a non-null `out` stores its group's partial.
template <typename T>
__device__ __forceinline__ void group_finish(TileAcc<T> &a, int G, pyas_partial *out) {
    uint64_t c = (uint64_t)a.count;
    uint32_t nan = a.nan ? 1u : 0u;
    for (int m = G / 2; m >= 1; m >>= 1) {   // uniform trip count
        a.sum += shfl_xor(a.sum, m);
        c += shfl_xor(c, m);
        a.mn = tmin(a.mn, shfl_xor(a.mn, m));
        a.mx = tmax(a.mx, shfl_xor(a.mx, m));
        nan |= shfl_xor(nan, m);
    }
    if (out) {
        pyas_partial p;
        TT<T>::put_acc(p.sum, a.sum);
        p.count = (int64_t)c;
        T mn = a.mn, mx = a.mx;
        if constexpr (TT<T>::kind == 0) {
            if (nan) { mn = (T)__builtin_nan(""); mx = mn; }
        }
        TT<T>::put(p.min, mn);
        TT<T>::put(p.max, mx);
        *out = p;
    }
}

// Partials handed between workgroups of ONE launch (the chained combine) are
// written and read with agent-scope relaxed atomics: on gfx950 these are
// sc1 accesses at the device-coherent level, so no agent-scope fence (a whole
// L2 write-back / invalidate per XCD) is needed to publish or observe them.
__device__ __forceinline__ void store_partial_agent(pyas_partial *out, const pyas_partial &p) {
    uint64_t w[4];
    __builtin_memcpy(w, &p, sizeof(w));
    uint64_t *o = reinterpret_cast<uint64_t *>(out);
#pragma unroll
    for (int k = 0; k < 4; ++k) __hip_atomic_store(o + k, w[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ pyas_partial load_partial_agent(const pyas_partial *in) {
    uint64_t w[4];
    const uint64_t *i = reinterpret_cast<const uint64_t *>(in);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = __hip_atomic_load(const_cast<uint64_t *>(i + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pyas_partial p;
    __builtin_memcpy(&p, w, sizeof(w));
    return p;
}

// Block reduction of TileAcc -> one pyas_partial (thread 0 stores).
// `extra_count` is added once (unmasked tiles: the element count).
template <typename T>
__device__ void tile_finish(TileAcc<T> &a, uint64_t extra_count, pyas_partial *out) {
    using S = typename TT<T>::Acc;
    const int lane = threadIdx.x & (kWave - 1);
    uint64_t c = (uint64_t)a.count + (lane == 0 ? (uint64_t)a.ucount : 0u);
    uint32_t nan = a.nan ? 1u : 0u;
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) {
        a.sum += shfl_xor(a.sum, m);
        c += shfl_xor(c, m);
        a.mn = tmin(a.mn, shfl_xor(a.mn, m));
        a.mx = tmax(a.mx, shfl_xor(a.mx, m));
        nan |= shfl_xor(nan, m);
    }
    __shared__ S s_sum[kBlock / kWave];
    __shared__ uint64_t s_cnt[kBlock / kWave];
    __shared__ T s_mn[kBlock / kWave];
    __shared__ T s_mx[kBlock / kWave];
    __shared__ uint32_t s_nan[kBlock / kWave];
    const int w = threadIdx.x / kWave;
    if (lane == 0) {
        s_sum[w] = a.sum; s_cnt[w] = c; s_mn[w] = a.mn; s_mx[w] = a.mx; s_nan[w] = nan;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 1; k < kBlock / kWave; ++k) {
            a.sum += s_sum[k];
            c += s_cnt[k];
            a.mn = tmin(a.mn, s_mn[k]);
            a.mx = tmax(a.mx, s_mx[k]);
            nan |= s_nan[k];
        }
        c += extra_count;
        pyas_partial p;
        TT<T>::put_acc(p.sum, a.sum);
        p.count = (int64_t)c;
        if constexpr (TT<T>::kind == 0) {
            if (nan) { a.mn = (T)__builtin_nan(""); a.mx = a.mn; }
        }
        TT<T>::put(p.min, a.mn);
        TT<T>::put(p.max, a.mx);
        *out = p;
    }
}

template <typename T, typename C>
__device__ __forceinline__ void merge_acc(AccT<T, C> &a, const typename TT<T>::Acc s, C c, T mn, T mx) {
    a.sum += s;
    a.count += c;
    a.mn = pmin(a.mn, mn);
    a.mx = pmax(a.mx, mx);
}

// Wave64 butterfly; every lane ends with the wave total (fixed order).
template <typename T, typename C>
__device__ __forceinline__ void wave_reduce(AccT<T, C> &a) {
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1)
        merge_acc(a, shfl_xor(a.sum, m), shfl_xor(a.count, m), shfl_xor(a.mn, m), shfl_xor(a.mx, m));
}

// Wave reduction, then one LDS exchange across the 4 waves.  Result valid in
// thread 0.  Fixed order => deterministic.
template <typename T, typename C>
__device__ void block_reduce(AccT<T, C> &a) {
    using A = typename TT<T>::Acc;
    wave_reduce(a);
    __shared__ A s_sum[kBlock / kWave];
    __shared__ C s_cnt[kBlock / kWave];
    __shared__ T s_mn[kBlock / kWave];
    __shared__ T s_mx[kBlock / kWave];
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        s_sum[w] = a.sum; s_cnt[w] = a.count; s_mn[w] = a.mn; s_mx[w] = a.mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 1; k < kBlock / kWave; ++k) merge_acc(a, s_sum[k], s_cnt[k], s_mn[k], s_mx[k]);
    }
}
template <typename T>
__device__ void block_reduce_w(WAcc<T> &a) { block_reduce(a); }

template <typename T, typename C>
__device__ __forceinline__ void store_partial(pyas_partial *out, const AccT<T, C> &a) {
    pyas_partial p;
    TT<T>::put_acc(p.sum, a.sum);
    p.count = (int64_t)a.count;
    TT<T>::put(p.min, a.mn);
    TT<T>::put(p.max, a.mx);
    *out = p;
}
template <typename T>
__device__ __forceinline__ void store_wpartial(pyas_partial *out, const WAcc<T> &a) { store_partial(out, a); }
template <typename T>
__device__ __forceinline__ void store_wpartial_agent(pyas_partial *out, const WAcc<T> &a) {
    pyas_partial p;
    TT<T>::put_acc(p.sum, a.sum);
    p.count = (int64_t)a.count;
    TT<T>::put(p.min, a.mn);
    TT<T>::put(p.max, a.mx);
    store_partial_agent(out, p);
}

// ---------------------------------------------------------------------------
// selection of one chunk (storage.py:95 chunk[chunk_selection])
// ---------------------------------------------------------------------------
struct Sel {
    int32_t start[PYAS_MAX_DIMS], step[PYAS_MAX_DIMS], cnt[PYAS_MAX_DIMS];
};

__device__ __forceinline__ void load_sel(Sel &s, const int32_t *sel, int64_t c, int ndim,
                                         const int64_t *shape) {
#pragma unroll
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) {
        if (d < ndim) {
            if (sel) {
                const int32_t *p = sel + ((int64_t)c * PYAS_MAX_DIMS + d) * 3;
                s.start[d] = p[0]; s.step[d] = p[1]; s.cnt[d] = p[2];
            } else {
                s.start[d] = 0; s.step[d] = 1; s.cnt[d] = (int32_t)shape[d];
            }
        } else {
            s.start[d] = 0; s.step[d] = 1; s.cnt[d] = 1;
        }
    }
}

__device__ __forceinline__ int64_t sel_index(const Sel &s, const int32_t *pool, int d, int64_t k) {
    return s.step[d] != 0 ? (int64_t)s.start[d] + k * (int64_t)s.step[d]
                          : (int64_t)pool[(int64_t)s.start[d] + k];
}

}  // namespace pyas
