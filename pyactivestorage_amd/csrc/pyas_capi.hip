// pyas_capi.hip — the extern "C" boundary declared in include/pyas.h.
//
// Host-side responsibilities: argument validation (mirroring the reference's
// error behaviour: ValueError -> PYAS_EINVAL, NotImplementedError ->
// PYAS_ENOTSUP), geometry (tiles per chunk), per-stream scratch for tile
// partials, launching the kernel chain on the caller's stream, and optional
// HIP-event timing of the hot kernel for bench.py.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "pyas.h"
#include "pyas_internal.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(e == hipErrorOutOfMemory ? PYAS_ENOMEM : PYAS_EDEVICE, "%s: %s", what,
                hipGetErrorString(e));
}

#define PYAS_HIP(call)                                  \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

constexpr int64_t kDefaultTileBytes = 256 * 1024;

int elem_size(int dtype) {
    switch (dtype) {
        case PYAS_I8: case PYAS_U8: return 1;
        case PYAS_I16: case PYAS_U16: return 2;
        case PYAS_I32: case PYAS_U32: case PYAS_F32: return 4;
        case PYAS_I64: case PYAS_U64: case PYAS_F64: return 8;
        default: return 0;
    }
}

struct Scratch {
    void *ptr = nullptr;
    size_t bytes = 0;
    uint32_t *cnt = nullptr;   // chained-combine arrival counters, zero between launches
    int64_t n_cnt = 0;
};

}  // namespace

struct pyas_ctx {
    int device = 0;
    int64_t tile_bytes = kDefaultTileBytes;
    int32_t inflate_wbits = 13;   // LDS history ring of pyas_inflate: 2^13 B per stream
    bool chained = true;          // k_finish folds the total itself (arrival counter)
    int64_t fold_min_blocks = 2048;   // pyas_reduce_axes_grid: fewest workgroups worth folding
    int32_t n_cu = 256;               // compute units (hipDeviceProp_t; sizes k_axes_col_stream's grid)
    pyas::TieRule tie[2];             // NumPy's zero-sign rule for f32, f64 (lanes 0: unset)
    pyas::Ingest *ingest = nullptr;   // pinned staging ring of pyas_read_ranges (lazy)
    std::mutex mu;
    std::unordered_map<void *, Scratch> scratch;  // keyed by stream
    std::unordered_map<void *, Scratch> tie_scratch;  // gate word / keys of the tie passes
    // timing
    std::vector<hipEvent_t> ev0, ev1;
    int32_t timing_n = 0;
};

namespace {

int ensure_scratch(pyas_ctx *ctx, void *stream, size_t bytes, void **out) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    Scratch &s = ctx->scratch[stream];
    if (s.bytes < bytes) {
        if (s.ptr) {
            // the stream may still use the old buffer
            PYAS_HIP(hipStreamSynchronize((hipStream_t)stream));
            PYAS_HIP(hipFree(s.ptr));
            s.ptr = nullptr;
            s.bytes = 0;
        }
        const size_t want = bytes < 4096 ? 4096 : bytes;
        PYAS_HIP(hipMalloc(&s.ptr, want));
        s.bytes = want;
    }
    *out = s.ptr;
    return PYAS_OK;
}

// Zeroed arrival counters of the chained combine for `stream` (the kernel
// leaves them zero again, so only a new allocation is cleared).
int ensure_counters(pyas_ctx *ctx, void *stream, int64_t n, uint32_t **out) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    Scratch &s = ctx->scratch[stream];
    if (s.n_cnt < n) {
        if (s.cnt) {
            PYAS_HIP(hipStreamSynchronize((hipStream_t)stream));
            PYAS_HIP(hipFree(s.cnt));
            s.cnt = nullptr;
            s.n_cnt = 0;
        }
        const int64_t want = n < 1024 ? 1024 : n;
        PYAS_HIP(hipMalloc((void **)&s.cnt, (size_t)want * sizeof(uint32_t)));
        PYAS_HIP(hipMemsetAsync(s.cnt, 0, (size_t)want * sizeof(uint32_t), (hipStream_t)stream));
        s.n_cnt = want;
    }
    *out = s.cnt;
    return PYAS_OK;
}

// An equality interval [lo, hi] wholly below the `< lt` threshold or wholly
// above the `> gt` one masks nothing the threshold does not already mask, so
// it is dropped (C3/C4: _FillValue -999 under valid_min 1000) and the kernels
// run a mode with fewer compares (mask_mode).  A lone second interval moves
// to slot 0.  The set of masked values is unchanged.
void trim_mask(pyas_mask &m, int dtype) {
    auto lt = [dtype](const pyas_scalar &x, const pyas_scalar &y) {
        if (dtype == PYAS_F32 || dtype == PYAS_F64) return x.f < y.f;
        if (dtype == PYAS_U8 || dtype == PYAS_U16 || dtype == PYAS_U32 || dtype == PYAS_U64) return x.u < y.u;
        return x.i < y.i;
    };
    for (int k = 0; k < 2; ++k) {
        const uint32_t bit = k == 0 ? PYAS_MASK_EQ0 : PYAS_MASK_EQ1;
        if (!(m.flags & bit)) continue;
        const bool below = (m.flags & PYAS_MASK_LT) && lt(m.eq_hi[k], m.lt);
        const bool above = (m.flags & PYAS_MASK_GT) && lt(m.gt, m.eq_lo[k]);
        if (below || above) m.flags &= ~bit;
    }
    if (!(m.flags & PYAS_MASK_EQ0) && (m.flags & PYAS_MASK_EQ1)) {
        m.eq_lo[0] = m.eq_lo[1];
        m.eq_hi[0] = m.eq_hi[1];
        m.flags = (m.flags & ~PYAS_MASK_EQ1) | PYAS_MASK_EQ0;
    }
}

// Validate the batch and fill the kernel argument block.
int prepare(const pyas_ctx *ctx, const pyas_batch *b, const pyas_mask *m, pyas::ReduceArgs &a,
            int &es, bool &shuf, bool &bsw, bool &masked) {
    if (!b) return fail(PYAS_EINVAL, "batch is NULL");
    es = elem_size(b->dtype);
    if (es == 0) return fail(PYAS_ENOTSUP, "unsupported dtype code %d", b->dtype);
    if (b->ndim < 1 || b->ndim > PYAS_MAX_DIMS)
        return fail(PYAS_EINVAL, "chunk rank %d outside 1..%d", b->ndim, PYAS_MAX_DIMS);
    if (b->n_chunks < 0) return fail(PYAS_EINVAL, "negative chunk count");
    int64_t elems = 1;
    for (int d = 0; d < b->ndim; ++d) {
        if (b->chunk_shape[d] <= 0) return fail(PYAS_EINVAL, "chunk_shape[%d] = %lld", d, (long long)b->chunk_shape[d]);
        elems *= b->chunk_shape[d];
        if (elems >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "chunk has >= 2^31 elements");
    }
    if (b->shuffle > 1 && b->shuffle != es)
        return fail(PYAS_ENOTSUP, "shuffle elementsize %d != dtype itemsize %d", b->shuffle, es);
    if (b->n_chunks > 0 && (!b->data || !b->offsets))
        return fail(PYAS_EINVAL, "data/offsets pointer is NULL");
    shuf = b->shuffle > 1 && es > 1;
    bsw = b->byteswap != 0 && es > 1;
    std::memset(&a, 0, sizeof(a));
    a.data = (const uint8_t *)b->data;
    a.offsets = b->offsets;
    a.sel = b->sel;
    a.pool = b->index_pool;
    a.ndim = b->ndim;
    a.chunk_elems = elems;
    {   // PYAS_SPANS (per call: tests and benches switch it): 0 off, 1 not on
        // the aligned runs run_rows streams, unset / 2 every cut chunk a span
        // plan fits (C3 [4:1020]^3 0.726 -> 0.708 ms; C5 level)
        const char *e = getenv("PYAS_SPANS");
        a.spans = e && *e ? atoi(e) : 2;
    }
    int64_t stride = 1;
    for (int d = PYAS_MAX_DIMS - 1; d >= 0; --d) {
        if (d < b->ndim) {
            a.shape[d] = b->chunk_shape[d];
            a.cstride[d] = stride;
            stride *= b->chunk_shape[d];
        } else {
            a.shape[d] = 1;
            a.cstride[d] = 0;
        }
    }
    masked = false;
    if (m) {
        a.mask = *m;
        const uint32_t known = PYAS_MASK_EQ0 | PYAS_MASK_EQ1 | PYAS_MASK_GT | PYAS_MASK_LT |
                               PYAS_MASK_TAB0 | PYAS_MASK_TAB1;
        if (m->flags & ~known) return fail(PYAS_EINVAL, "unknown mask flags 0x%x", m->flags);
        for (int k = 0; k < 2; ++k) {
            const uint32_t bit = k == 0 ? PYAS_MASK_TAB0 : PYAS_MASK_TAB1;
            if (m->flags & bit) {
                if (!m->tab_lo[k] || !m->tab_hi[k] || m->tab_len[k] <= 0)
                    return fail(PYAS_EINVAL, "mask table %d enabled but empty", k);
                a.tab.on[k] = true;
                a.tab.lo[k] = m->tab_lo[k];
                a.tab.hi[k] = m->tab_hi[k];
                for (int d = 0; d < PYAS_MAX_DIMS; ++d) a.tab.stride[k][d] = m->tab_stride[k][d];
            }
        }
        masked = m->flags != 0;
        trim_mask(a.mask, b->dtype);
    }
    (void)ctx;
    return PYAS_OK;
}

int64_t tiles_per_chunk(const pyas_ctx *ctx, int64_t chunk_bytes) {
    const int64_t tb = ctx->tile_bytes > 0 ? ctx->tile_bytes : kDefaultTileBytes;
    int64_t t = (chunk_bytes + tb - 1) / tb;
    return t < 1 ? 1 : t;
}

// Fixed-order combine of n partials into out[0]; may use scratch at `tmp`
// (room for n / kSeg + 1 partials).
constexpr int64_t kSeg = pyas::kCombineSeg;

int combine_into(int dtype, const pyas_partial *in, int64_t n, uint32_t flags, pyas_partial *tmp,
                 pyas_partial *out, hipStream_t st) {
    if (n <= 0) {
        PYAS_HIP(hipMemsetAsync(out, 0, sizeof(pyas_partial), st));
        return PYAS_OK;
    }
    const int64_t nblocks = (n + kSeg - 1) / kSeg;
    if (nblocks == 1) {
        PYAS_HIP(pyas::launch_combine(dtype, in, n, kSeg, 1, flags, out, st));
        return PYAS_OK;
    }
    PYAS_HIP(pyas::launch_combine(dtype, in, n, kSeg, nblocks, flags, tmp, st));
    PYAS_HIP(pyas::launch_combine(dtype, tmp, nblocks, nblocks, 1, 0u, out, st));
    return PYAS_OK;
}

}  // namespace

namespace pyas {

int set_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int ctx_device(const pyas_ctx *ctx) { return ctx->device; }

}  // namespace pyas

extern "C" {

int pyas_abi_version(void) { return PYAS_ABI_VERSION; }

const char *pyas_last_error(void) { return g_err.c_str(); }

int pyas_device_count(int *count) {
    if (!count) return fail(PYAS_EINVAL, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = n;
    return PYAS_OK;
}

int pyas_ctx_create(int device, pyas_ctx **out) {
    if (!out) return fail(PYAS_EINVAL, "out is NULL");
    int n = 0;
    PYAS_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(PYAS_EINVAL, "device %d not in [0, %d)", device, n);
    PYAS_HIP(hipSetDevice(device));
    pyas_ctx *c = new pyas_ctx();
    c->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->n_cu = cus;
    *out = c;
    return PYAS_OK;
}

int pyas_ctx_destroy(pyas_ctx *ctx) {
    if (!ctx) return PYAS_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto &kv : ctx->scratch)
    {
        if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        if (kv.second.cnt) (void)hipFree(kv.second.cnt);
    }
    for (auto &kv : ctx->tie_scratch)
        if (kv.second.ptr) (void)hipFree(kv.second.ptr);
    if (ctx->ingest) pyas::ingest_destroy(ctx->ingest);
    for (auto e : ctx->ev0) (void)hipEventDestroy(e);
    for (auto e : ctx->ev1) (void)hipEventDestroy(e);
    delete ctx;
    return PYAS_OK;
}

int pyas_ctx_set_tile_bytes(pyas_ctx *ctx, int64_t tile_bytes) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (tile_bytes < 0) return fail(PYAS_EINVAL, "tile_bytes < 0");
    ctx->tile_bytes = tile_bytes == 0 ? kDefaultTileBytes : tile_bytes;
    return PYAS_OK;
}

static pyas::Ingest *ingest_of(pyas_ctx *ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->ingest) ctx->ingest = pyas::ingest_create(ctx->device);
    return ctx->ingest;
}

int pyas_ctx_set_ingest_slots(pyas_ctx *ctx, int32_t n_slots, int64_t slot_bytes) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    std::string msg;
    const int rc = pyas::ingest_configure(ingest_of(ctx), n_slots, slot_bytes, msg);
    return rc ? fail(rc, "%s", msg.c_str()) : PYAS_OK;
}

int pyas_read_ranges(pyas_ctx *ctx, int fd, int64_t n, const int64_t *file_offsets,
                     const int64_t *sizes, void *dst, const int64_t *dst_offsets, int32_t threads,
                     void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    std::string msg;
    const int rc = pyas::ingest_read(ingest_of(ctx), fd, n, file_offsets, sizes, (uint8_t *)dst,
                                     dst_offsets, threads, (hipStream_t)stream, msg);
    return rc ? fail(rc, "%s", msg.c_str()) : PYAS_OK;
}

int pyas_read_ranges_zlib(pyas_ctx *ctx, int fd, int64_t n, const int64_t *file_offsets,
                          const int64_t *sizes, void *dst, const int64_t *dst_offsets, int64_t out_bytes,
                          int32_t *status, int32_t threads, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (out_bytes <= 0) return fail(PYAS_EINVAL, "out_bytes must be > 0");
    std::string msg;
    const int rc = pyas::ingest_read(ingest_of(ctx), fd, n, file_offsets, sizes, (uint8_t *)dst,
                                     dst_offsets, threads, (hipStream_t)stream, msg, out_bytes, status);
    return rc ? fail(rc, "%s", msg.c_str()) : PYAS_OK;
}

int pyas_ctx_set_tie_rule(pyas_ctx *ctx, int32_t dtype, const pyas_tie_rule *rule) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (dtype != PYAS_F32 && dtype != PYAS_F64) return fail(PYAS_EINVAL, "tie rules are for f32/f64");
    pyas::TieRule &t = ctx->tie[dtype == PYAS_F64 ? 1 : 0];
    std::memset(&t, 0, sizeof(t));
    if (!rule) return PYAS_OK;
    if (rule->lanes < 1 || rule->lanes > 64 || rule->piece < 1 || rule->piece >= (1 << 24) || rule->acc < 1 ||
        rule->acc > 64)
        return fail(PYAS_EINVAL, "tie rule: lanes %d, piece %d, acc %d", rule->lanes, rule->piece, rule->acc);
    auto perm_ok = [](const uint8_t *rank, int n) {
        bool seen[64] = {false};
        for (int l = 0; l < n; ++l) {
            if (rank[l] >= n || seen[rank[l]]) return false;
            seen[rank[l]] = true;
        }
        return true;
    };
    if (!perm_ok(rule->rank, rule->lanes) || !perm_ok(rule->acc_rank, rule->acc))
        return fail(PYAS_EINVAL, "tie rule: a rank table is not a permutation");
    t.lanes = rule->lanes;
    t.piece = rule->piece;
    t.acc = rule->acc;
    std::memcpy(t.rank, rule->rank, sizeof(t.rank));
    std::memcpy(t.acc_rank, rule->acc_rank, sizeof(t.acc_rank));
    return PYAS_OK;
}

namespace {

const pyas::TieRule *tie_of(const pyas_ctx *ctx, int32_t dtype) {
    if (dtype != PYAS_F32 && dtype != PYAS_F64) return nullptr;
    const pyas::TieRule &t = ctx->tie[dtype == PYAS_F64 ? 1 : 0];
    return t.lanes ? &t : nullptr;
}

pyas::TieCall grid_call(const pyas::TieRule &t, int64_t lr) {
    pyas::TieCall c;
    c.acc = 0;
    c.block = 0;
    c.n_copy = 0;
    c.lr = lr < 1 ? 1 : lr;
    c.npr = (c.lr + t.piece - 1) / t.piece;
    return c;
}

int check_geom(const pyas_tie_geom *g, int ndim) {
    if (!g) return fail(PYAS_EINVAL, "tie geometry is NULL");
    uint32_t seen = 0;
    for (int i = 0; i < ndim; ++i) {
        const int d = g->perm[i];
        if (d < 0 || d >= ndim || ((seen >> d) & 1u)) return fail(PYAS_EINVAL, "tie geometry: perm is not a permutation");
        seen |= 1u << d;
    }
    if (g->flags & ~(PYAS_TIE_VIEW | PYAS_TIE_BUFFERED)) return fail(PYAS_EINVAL, "tie geometry: unknown flags");
    return PYAS_OK;
}

// Level 1 shared by pyas_tie_chunks / pyas_tie_chunk_flags.
// pick (full reductions): device keys of pyas_tie_chunks_total's pick pass;
// only the two chunks they name are scanned, one workgroup.
int tie_chunks(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask, const pyas_tie_geom *geom,
               uint32_t axes_mask, uint32_t which, const int64_t *out_offsets, pyas_partial *partials,
               uint8_t *flags, const uint32_t *gate, hipStream_t st, const uint64_t *pick = nullptr,
               int64_t pick_base = 0, int64_t pick_lr = 1) {
    pyas::TieChunkArgs a;
    std::memset(&a, 0, sizeof(a));
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, a.r, es, shuf, bsw, masked);
    if (rc) return rc;
    if ((rc = check_geom(geom, batch->ndim))) return rc;
    const pyas::TieRule *t = tie_of(ctx, batch->dtype);
    if ((which & PYAS_TIE_REC) && (which & 3u) != 1u && (which & 3u) != 2u)
        return fail(PYAS_EINVAL, "PYAS_TIE_REC needs which 1 (min) or 2 (max)");
    if (!t || batch->n_chunks == 0 || (which & 3u) == 0) return PYAS_OK;
    const uint32_t full = (1u << batch->ndim) - 1u;
    if ((axes_mask & ~full) != 0) return fail(PYAS_EINVAL, "axes_mask 0x%x outside the chunk rank", axes_mask);
    if ((axes_mask & full) != full && !out_offsets)
        return fail(PYAS_EINVAL, "out_offsets is NULL for a partial-axis reduction");
    int64_t kept = 1, red = 1;
    for (int d = 0; d < batch->ndim; ++d) {
        if (!((axes_mask >> d) & 1u)) kept *= batch->chunk_shape[d];
        else red *= batch->chunk_shape[d];
    }
    if (red >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "tie pass: 2^31 or more reduced elements per output");
    // lanes per output of the backward scan (k_tie_scan): one when the
    // innermost visited dim is kept (elementwise calls: adjacent lanes hold
    // adjacent outputs, and each lane stops at its last zero), else by the
    // reduced count per output
    int inner_kept = -1;
    for (int i = batch->ndim - 1; i >= 0 && inner_kept < 0; --i) {
        const int d = geom->perm[i];
        if (batch->chunk_shape[d] != 1) inner_kept = ((axes_mask >> d) & 1u) ? 0 : 1;
    }
    // (a full reduction: a wave per chunk, four chunks per workgroup)
    // short calls (< 256 reduced elements, e.g. C3 (2,): 64) take a lane per
    // output too, 4 positions per step: a group of 16 per output walked the
    // chunk's 4096 outputs 4 at a time per wave, one chain of dependent loads
    // each (13 ms per C3 query at 50 % zeros)
    int group = kept == 1 ? pyas::kWave : inner_kept == 1 ? 1 : red >= 1024 ? pyas::kWave : red >= 256 ? 16 : 1;
    const char *e_group = getenv("PYAS_TIE_GROUP");   // per call: tests force each layout
    if (e_group && *e_group) {
        const int g = atoi(e_group);
        if (g == 1 || g == 16 || g == pyas::kWave) group = g;
    }
    if (pick) group = pyas::kWave;   // the picked chunks: a wave each
    a.group = group;
    a.n_chunks = batch->n_chunks;
    a.cpw = (kept == 1 && group == pyas::kWave) ? pyas::kBlock / pyas::kWave : 1;
    a.t = *t;
    a.g = *geom;
    a.axes = axes_mask;
    a.which = which & (3u | PYAS_TIE_REC);
    a.shuf = shuf;
    a.bswap = bsw;
    a.out_offsets = out_offsets;
    a.parts = partials;
    a.flags = flags;
    a.gate = gate;
    int64_t grid = (batch->n_chunks + a.cpw - 1) / a.cpw;   // a workgroup per chunk (or per cpw)
    if (pick) {
        if (kept != 1 || a.cpw < 2) return fail(PYAS_EINVAL, "the picked tie scan needs a full reduction");
        a.pick = pick;
        a.pick_call = grid_call(*t, pick_lr);
        a.pick_base = pick_base;
        grid = 1;
    }
    if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "tie grid too large");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_tie_chunks(batch->dtype, a, grid, st));
    return PYAS_OK;
}

// Per-stream gate word and key scratch of the tie passes.
// Growing swaps the pointer under the context lock; the old buffer is freed
// after the stream's queued work is done, outside the lock, so
// other threads never wait on this stream.
int tie_scratch(pyas_ctx *ctx, void *stream, size_t bytes, void **out) {
    void *old = nullptr;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        Scratch &s = ctx->tie_scratch[stream];
        if (s.bytes < bytes) {
            const size_t want = bytes < 4096 ? 4096 : bytes;
            void *p = nullptr;
            PYAS_HIP(hipMalloc(&p, want));
            old = s.ptr;
            s.ptr = p;
            s.bytes = want;
        }
        *out = s.ptr;
    }
    if (old) {
        PYAS_HIP(hipStreamSynchronize((hipStream_t)stream));
        PYAS_HIP(hipFree(old));
    }
    return PYAS_OK;
}

// Level 2: one wave per (output, layer slice); several slices per output
// fold their keys through `keys` (or an internal buffer + finalize).
int tie_level2(pyas_ctx *ctx, int32_t dtype, pyas::TieGridArgs &a, int64_t max_layers, uint64_t *keys,
               hipStream_t st) {
    const pyas::TieRule *t = tie_of(ctx, dtype);
    if (!t || a.n_out <= 0 || max_layers <= 0) return PYAS_OK;
    a.t = *t;
    // few outputs with many layers: split the layers over waves
    int64_t slices = 1;
    if (a.n_out < 4096 && max_layers > 4 * pyas::kWave) {
        slices = max_layers / (4 * pyas::kWave);
        const int64_t cap = 8192 / a.n_out > 1 ? 8192 / a.n_out : 1;
        if (slices > cap) slices = cap;
    }
    a.slices = slices;
    // few layers per output (<= 64) and many outputs: a thread per output
    a.per_thread = (max_layers <= pyas::kWave && a.n_out >= 4096) ? 1 : 0;
    if ((a.n_out * slices) / (pyas::kBlock / pyas::kWave) >= (int64_t(1) << 31))
        return fail(PYAS_ENOTSUP, "tie grid too large");
    PYAS_HIP(hipSetDevice(ctx->device));
    uint64_t *own = nullptr;
    if (!keys && slices > 1) {
        void *p = nullptr;
        int rc = tie_scratch(ctx, st, (size_t)a.n_out * 16, &p);
        if (rc) return rc;
        own = (uint64_t *)p;
        PYAS_HIP(hipMemsetAsync(own, 0, (size_t)a.n_out * 8, st));
        PYAS_HIP(hipMemsetAsync(own + a.n_out, 0xff, (size_t)a.n_out * 8, st));
    }
    a.keys = keys ? keys : own;
    PYAS_HIP(pyas::launch_tie_grid(dtype, a, st));
    if (own) PYAS_HIP(pyas::launch_tie_finalize(dtype, own, a.n_out, 1, a.call, a.t, a.which, a.fin, st));
    return PYAS_OK;
}

}  // namespace

int pyas_tie_chunks(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask, const pyas_tie_geom *geom,
                    uint32_t axes_mask, uint32_t which, const int64_t *out_offsets, pyas_partial *partials,
                    void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!partials && batch && batch->n_chunks > 0) return fail(PYAS_EINVAL, "partials is NULL");
    return tie_chunks(ctx, batch, mask, geom, axes_mask, which, out_offsets, partials, nullptr, nullptr,
                      (hipStream_t)stream);
}

int pyas_tie_chunks_total(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask, const pyas_tie_geom *geom,
                          uint32_t which, pyas_partial *partials, int64_t layer_base, int64_t lr, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!batch) return fail(PYAS_EINVAL, "batch is NULL");
    if ((which & ~PYAS_TIE_REC) != 1u && (which & ~PYAS_TIE_REC) != 2u)
        return fail(PYAS_EINVAL, "which must be 1 (min) or 2 (max), optionally | PYAS_TIE_REC");
    if (layer_base < 0 || lr < 1) return fail(PYAS_EINVAL, "layer_base < 0 or lr < 1");
    const pyas::TieRule *t = tie_of(ctx, batch->dtype);
    if (!t || batch->n_chunks == 0) return PYAS_OK;
    if (!partials) return fail(PYAS_EINVAL, "partials is NULL");
    void *p = nullptr;
    int rc = tie_scratch(ctx, stream, 16, &p);
    if (rc) return rc;
    uint64_t *keys = (uint64_t *)p;
    hipStream_t st = (hipStream_t)stream;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipMemsetAsync(keys, 0, 8, st));
    PYAS_HIP(hipMemsetAsync(keys + 1, 0xff, 8, st));
    PYAS_HIP(pyas::launch_tie_pick(batch->dtype, partials, batch->n_chunks, which, layer_base, grid_call(*t, lr), *t,
                                   keys, st));
    return tie_chunks(ctx, batch, mask, geom, (1u << batch->ndim) - 1u, which, nullptr, partials, nullptr, nullptr,
                      st, keys, layer_base, lr);
}

int pyas_tie_chunk_flags(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask, const pyas_tie_geom *geom,
                         uint32_t axes_mask, uint32_t which, const int64_t *out_offsets, const pyas_partial *final_,
                         int64_t n_final, uint8_t *flags, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!batch) return fail(PYAS_EINVAL, "batch is NULL");
    if (which != 1u && which != 2u) return fail(PYAS_EINVAL, "which must be 1 (min) or 2 (max)");
    if (!tie_of(ctx, batch->dtype) || batch->n_chunks == 0 || n_final <= 0) return PYAS_OK;
    if (!final_ || !flags) return fail(PYAS_EINVAL, "NULL argument");
    void *p = nullptr;
    int rc = tie_scratch(ctx, stream, 16, &p);
    if (rc) return rc;
    uint32_t *gate = (uint32_t *)p;
    hipStream_t st = (hipStream_t)stream;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipMemsetAsync(gate, 0, 4, st));
    PYAS_HIP(pyas::launch_tie_gate(batch->dtype, final_, n_final, which, gate, st));
    return tie_chunks(ctx, batch, mask, geom, axes_mask, which, out_offsets, nullptr, flags, gate, st);
}

int pyas_tie_grid(pyas_ctx *ctx, int32_t dtype, const pyas_grid *grid, const pyas_partial *parts,
                  const uint8_t *flags, int64_t lr, uint32_t which, pyas_partial *final_, uint64_t *keys,
                  void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!grid || !final_ || (!parts && !flags) || !grid->chunk_out_offsets)
        return fail(PYAS_EINVAL, "NULL argument");
    if ((which & ~PYAS_TIE_REC) != 1u && (which & ~PYAS_TIE_REC) != 2u)
        return fail(PYAS_EINVAL, "which must be 1 (min) or 2 (max), optionally | PYAS_TIE_REC");
    if (grid->ndim < 1 || grid->ndim > PYAS_MAX_DIMS) return fail(PYAS_EINVAL, "grid rank %d", grid->ndim);
    const pyas::TieRule *t = tie_of(ctx, dtype);
    if (!t) return PYAS_OK;
    int64_t n_out = 1, n_layers = 1;
    for (int d = 0; d < grid->ndim; ++d) {
        if ((grid->axes_mask >> d) & 1u) n_layers *= grid->n_coords[d];
        else n_out *= grid->out_extent[d];
    }
    if (n_layers >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "more than 2^31 chunk layers");
    pyas::TieGridArgs a;
    std::memset(&a, 0, sizeof(a));
    a.g = *grid;
    a.kind = 0;
    a.parts = parts;
    a.flags = flags;
    a.fin = final_;
    a.n_out = n_out;
    a.n_layers = n_layers;
    a.call = grid_call(*t, lr);
    a.which = which;
    return tie_level2(ctx, dtype, a, n_layers, keys, (hipStream_t)stream);
}

int pyas_tie_segments(pyas_ctx *ctx, int32_t dtype, const pyas_partial *parts, const int64_t *index,
                      const int64_t *seg, int64_t n_seg, int64_t n_layers, int64_t layer_base, int64_t lr,
                      uint32_t which, pyas_partial *final_, uint64_t *keys, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!parts || !final_) return fail(PYAS_EINVAL, "NULL argument");
    if ((which & ~PYAS_TIE_REC) != 1u && (which & ~PYAS_TIE_REC) != 2u)
        return fail(PYAS_EINVAL, "which must be 1 (min) or 2 (max), optionally | PYAS_TIE_REC");
    if (!seg && (index || n_seg != 1)) return fail(PYAS_EINVAL, "seg NULL needs index NULL and one segment");
    if (n_layers < 0 || layer_base < 0) return fail(PYAS_EINVAL, "negative layer count or base");
    const pyas::TieRule *t = tie_of(ctx, dtype);
    if (!t) return PYAS_OK;
    pyas::TieGridArgs a;
    std::memset(&a, 0, sizeof(a));
    a.kind = seg ? 1 : 2;
    a.index = index;
    a.seg = seg;
    a.parts = parts;
    a.fin = final_;
    a.n_out = n_seg;
    a.n_layers = n_layers;
    a.layer_base = layer_base;
    a.call = grid_call(*t, lr);
    a.which = which;
    // segment lengths live on the device: the caller's n_layers bounds them
    return tie_level2(ctx, dtype, a, n_layers, keys, (hipStream_t)stream);
}

int pyas_tie_keys_reset(pyas_ctx *ctx, uint64_t *keys, int64_t n_out, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n_out <= 0) return PYAS_OK;
    if (!keys) return fail(PYAS_EINVAL, "keys is NULL");
    hipStream_t st = (hipStream_t)stream;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipMemsetAsync(keys, 0, (size_t)n_out * 8, st));
    PYAS_HIP(hipMemsetAsync(keys + n_out, 0xff, (size_t)n_out * 8, st));
    return PYAS_OK;
}

int pyas_tie_finalize(pyas_ctx *ctx, int32_t dtype, const uint64_t *keys, int64_t n_out, int32_t n_sets,
                      int64_t lr, uint32_t which, pyas_partial *final_, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (which != 1u && which != 2u) return fail(PYAS_EINVAL, "which must be 1 (min) or 2 (max)");
    const pyas::TieRule *t = tie_of(ctx, dtype);
    if (!t || n_out <= 0 || n_sets <= 0) return PYAS_OK;
    if (!keys || !final_) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_tie_finalize(dtype, keys, n_out, n_sets, grid_call(*t, lr), *t, which, final_,
                                       (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_ctx_set_fold_min_blocks(pyas_ctx *ctx, int64_t n) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n < 0) return fail(PYAS_EINVAL, "fold_min_blocks < 0");
    ctx->fold_min_blocks = n == 0 ? 2048 : n;
    return PYAS_OK;
}

int pyas_ctx_set_chained_combine(pyas_ctx *ctx, int32_t on) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    ctx->chained = on != 0;
    return PYAS_OK;
}

int pyas_ctx_set_inflate_window_bits(pyas_ctx *ctx, int32_t wbits) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (wbits < 13 || wbits > 15) return fail(PYAS_EINVAL, "inflate window bits %d not in [13, 15]", wbits);
    ctx->inflate_wbits = wbits;
    return PYAS_OK;
}

int pyas_malloc(pyas_ctx *ctx, size_t nbytes, void **dptr) {
    if (!ctx || !dptr) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    *dptr = nullptr;
    PYAS_HIP(hipMalloc(dptr, nbytes ? nbytes : 1));
    return PYAS_OK;
}

int pyas_free(pyas_ctx *ctx, void *dptr) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!dptr) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipFree(dptr));
    return PYAS_OK;
}

int pyas_host_alloc(pyas_ctx *ctx, size_t nbytes, void **hptr) {
    if (!ctx || !hptr) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    *hptr = nullptr;
    PYAS_HIP(hipHostMalloc(hptr, nbytes ? nbytes : 1, hipHostMallocDefault));
    return PYAS_OK;
}

int pyas_host_free(pyas_ctx *ctx, void *hptr) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!hptr) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipHostFree(hptr));
    return PYAS_OK;
}

int pyas_memcpy_h2d(pyas_ctx *ctx, void *dst, const void *src, size_t n, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n == 0) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_memcpy_d2h(pyas_ctx *ctx, void *dst, const void *src, size_t n, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n == 0) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_stream_create(pyas_ctx *ctx, void **stream) {
    if (!ctx || !stream) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    hipStream_t s;
    PYAS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void *)s;
    return PYAS_OK;
}

int pyas_stream_destroy(pyas_ctx *ctx, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!stream) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipStreamSynchronize((hipStream_t)stream));
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        auto it = ctx->scratch.find(stream);
        if (it != ctx->scratch.end()) {
            if (it->second.ptr) (void)hipFree(it->second.ptr);
            if (it->second.cnt) (void)hipFree(it->second.cnt);
            ctx->scratch.erase(it);
        }
        auto jt = ctx->tie_scratch.find(stream);
        if (jt != ctx->tie_scratch.end()) {
            if (jt->second.ptr) (void)hipFree(jt->second.ptr);
            ctx->tie_scratch.erase(jt);
        }
    }
    PYAS_HIP(hipStreamDestroy((hipStream_t)stream));
    return PYAS_OK;
}

int pyas_stream_synchronize(pyas_ctx *ctx, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(hipStreamSynchronize((hipStream_t)stream));
    return PYAS_OK;
}

int pyas_stream_wait(pyas_ctx *ctx, void *waiter, void *waitee) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (waiter == waitee) return PYAS_OK;
    PYAS_HIP(hipSetDevice(ctx->device));
    hipEvent_t ev;
    PYAS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, (hipStream_t)waitee);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)waiter, ev, 0);
    (void)hipEventDestroy(ev);   // released once the wait is satisfied
    if (e != hipSuccess) return hip_fail(e, "pyas_stream_wait");
    return PYAS_OK;
}

int pyas_reduce_chunks(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                       pyas_partial *chunk_out, pyas_partial *total, uint32_t combine_flags,
                       void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!chunk_out && !total) return fail(PYAS_EINVAL, "neither chunk_out nor total given");
    if (combine_flags & ~PYAS_COMBINE_ROUND_TO_VAR)
        return fail(PYAS_EINVAL, "unknown combine flags 0x%x", combine_flags);
    pyas::ReduceArgs a;
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, a, es, shuf, bsw, masked);
    if (rc) return rc;
    PYAS_HIP(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = batch->n_chunks;
    if (n == 0) {
        if (total) PYAS_HIP(hipMemsetAsync(total, 0, sizeof(pyas_partial), st));
        return PYAS_OK;
    }
    const int64_t tpc = tiles_per_chunk(ctx, a.chunk_elems * es);
    const int64_t grid = n * tpc;
    if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid of %lld workgroups", (long long)grid);
    a.tpc = tpc;
    // k_reduce writes one partial per workgroup: straight into chunk_out when a
    // chunk is one tile, else into scratch; k_finish folds tiles -> chunks ->
    // groups -> total in one launch.
    // scratch layout: [tile partials (unless they go to chunk_out)] [group partials]
    const bool direct = tpc == 1 && chunk_out;
    const size_t tiles_b = direct ? 0 : (size_t)grid * sizeof(pyas_partial);
    const int64_t ng = (n + kSeg - 1) / kSeg;
    const size_t tmp_b = (size_t)(ng + 1) * sizeof(pyas_partial);
    void *scr = nullptr;
    rc = ensure_scratch(ctx, stream, tiles_b + tmp_b, &scr);
    if (rc) return rc;
    a.out = direct ? chunk_out : (pyas_partial *)scr;
    pyas::FinishArgs f;
    f.tiles = a.out;
    f.tpc = tpc;
    f.n_chunks = n;
    f.chunk_out = direct ? nullptr : chunk_out;
    f.gtmp = (pyas_partial *)((char *)scr + tiles_b);
    f.total = total;
    f.cnt = nullptr;
    f.flags = combine_flags;
    if (total && ctx->chained) {
        rc = ensure_counters(ctx, stream, 1, &f.cnt);
        if (rc) return rc;
    }

    const bool timed = ctx->timing_n < (int32_t)ctx->ev0.size();
    if (timed) PYAS_HIP(hipEventRecord(ctx->ev0[ctx->timing_n], st));
    PYAS_HIP(pyas::launch_reduce(batch->dtype, a, shuf, bsw, masked, grid, st));
    if (timed) {
        PYAS_HIP(hipEventRecord(ctx->ev1[ctx->timing_n], st));
        ctx->timing_n++;
    }
    if (direct && !total) return PYAS_OK;
    PYAS_HIP(pyas::launch_finish(batch->dtype, f, st));
    if (total && !f.cnt)   // unchained: fold the group partials in a second launch
        PYAS_HIP(pyas::launch_combine(batch->dtype, f.gtmp, ng, ng, 1, 0u, total, st));
    return PYAS_OK;
}

// Dense partial-axis geometry: merge the chunk dims into runs of reduced /
// kept dims and fit them to (RO, KO, RI, KI); pick the column layout (a
// kept inner run of whole 16-B vectors) or the row layout (a reduced inner
// run of whole 16-B vectors, >= 4 lanes per output).  mode 0 = not dense.
// Shuffled chunks (vpl = es) load the row layouts in units of 16 elements
// (one 16-B piece per byte plane = vpl vectors), so a run must hold whole
// units.
static void dense_geometry(pyas::AxesDense &d, const pyas_batch *b, uint32_t axes_mask, int es,
                           int vpl, bool excluded) {
    std::memset(&d, 0, sizeof(d));
    if (excluded || axes_mask == 0) return;
    int64_t ext[PYAS_MAX_DIMS];
    int kind[PYAS_MAX_DIMS], nr = 0;
    for (int dd = 0; dd < b->ndim; ++dd) {
        const int k = (axes_mask >> dd) & 1u;
        if (nr && kind[nr - 1] == k) ext[nr - 1] *= b->chunk_shape[dd];
        else { kind[nr] = k; ext[nr++] = b->chunk_shape[dd]; }
    }
    int64_t v[4] = {1, 1, 1, 1};   // slots RO (reduced), KO (kept), RI (reduced), KI (kept)
    int slot = 3;
    for (int q = nr - 1; q >= 0; --q) {
        while (slot >= 0 && (slot % 2 == 1 ? 0 : 1) != kind[q]) --slot;
        if (slot < 0) return;      // more than 4 alternating runs
        v[slot--] = ext[q];
    }
    d.RO = v[0]; d.KO = v[1]; d.RI = v[2]; d.KI = v[3];
    const int64_t nv = 16 / es, chunk_bytes = d.RO * d.KO * d.RI * d.KI * es;
    auto pow2_ceil = [](int64_t x) { int64_t p = 1; while (p < x) p *= 2; return p; };
    if (d.KI > 1) {
        if ((d.KI * es) % 16) return;
        const int64_t items = d.KO * (d.KI / nv), rows = d.RO * d.RI;
        int64_t it = pow2_ceil(items < pyas::kBlock ? items : pyas::kBlock);
        int64_t sp = pyas::kBlock / it;
        while (sp > 1 && rows < sp * 4) sp >>= 1;   // >= 4 rows per split
        d.mode = 1;
        d.it = (int32_t)it;
        d.split = (int32_t)sp;
        d.bpc = (items + it - 1) / it;
    } else {
        if ((d.RI * es) % 16) return;
        const int64_t V = d.RI / nv;
        if (V % vpl) return;       // shuffled: whole 16-element units per run
        // Short single runs (RO == 1, <= 256 B): through LDS, 1, 2 or 4 lanes
        // per output (PYAS_ROW_LDS: 0 off, else the most lanes allowed; default 2)
        const char *e_lds = getenv("PYAS_ROW_LDS");     // per call: tests switch it
        const int row_lds = e_lds ? atoi(e_lds) : 2;
        // tiles per wave: 2 measured best in round 1; with the staged partial
        // stores (round 3) 1 is: C3 (2,) 0.80-0.81 ms against 0.82 (4: 0.87,
        // 8: 0.89; profiles/r03/axes_row_tpw.txt)
        const char *e_tpw = getenv("PYAS_ROW_LDS_TPW");
        const int64_t row_tpw = e_tpw && atoi(e_tpw) > 0 ? (int64_t)atoi(e_tpw) : (int64_t)1;
        if (row_lds && d.RO == 1 && V <= 16) {
            int h = 1;
            while (h < row_lds && h < 4 && V % (h * 2) == 0) h *= 2;
            d.mode = h == 1 ? 4 : h == 2 ? 5 : 6;
            d.group = h;
            const int64_t per_pass = (pyas::kBlock / pyas::kWave) * (pyas::kWave / h);
            const int64_t bpc = (d.KO + row_tpw * per_pass - 1) / (row_tpw * per_pass);   // tiles per wave
            d.bpc = bpc < 1 ? 1 : bpc;
            return;
        }
        // G lanes per output: the largest power of two dividing V (<= 64)
        // that still leaves each lane >= row_vecs vectors per run
        static const int64_t row_vecs = [] {
            const char *e = getenv("PYAS_ROW_VECS");
            return e ? (int64_t)atoi(e) : (int64_t)2;   // measured: 2 beats 1 and 4 on (2,)
        }();
        const int64_t Vu = V / vpl, min_units = vpl > 1 ? 1 : row_vecs;   // load units per run
        int64_t g = 1;
        while (g < pyas::kWave && Vu % (g * 2) == 0 && Vu / (g * 2) >= min_units) g *= 2;
        if (g < 4) return;         // too few lanes per output to coalesce
        const int64_t per_lane = d.RO * (Vu / g);
        const int64_t uo = per_lane == 1 ? 4 : 1;
        d.mode = uo == 4 ? 3 : 2;
        d.group = (int32_t)g;
        const int64_t per_pass = (pyas::kBlock / pyas::kWave) * (pyas::kWave / g) * uo;
        int64_t bpc = (d.KO + per_pass - 1) / per_pass;
        const int64_t by_bytes = chunk_bytes >> 16;   // >= ~64 KiB per workgroup
        if (bpc > by_bytes) bpc = by_bytes;
        d.bpc = bpc < 1 ? 1 : bpc;
    }
}

int pyas_reduce_axes(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                     uint32_t axes_mask, const int64_t *out_offsets, pyas_partial *out,
                     void *stream) {
    return pyas_reduce_axes_ex(ctx, batch, mask, axes_mask, PYAS_REC_FULL, out_offsets, out, stream);
}

int pyas_reduce_axes_ex(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                        uint32_t axes_mask, int32_t rec, const int64_t *out_offsets, void *out,
                        void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    const bool want_zs = (rec & PYAS_REC_ZERO_SIGN) != 0;
    // PYAS_REC_DENSE_ONLY (and PYAS_REC_ZERO_SIGN, which makes the same
    // promise): every chunk is whole or a box the dense launch takes
    const bool dense_only = (rec & (PYAS_REC_DENSE_ONLY | PYAS_REC_ZERO_SIGN)) != 0;
    // PYAS_REC_GENERIC_ONLY: no chunk is the dense launch's (none is made)
    const bool generic_only = (rec & PYAS_REC_GENERIC_ONLY) != 0;
    if (dense_only && generic_only) return fail(PYAS_EINVAL, "PYAS_REC_DENSE_ONLY and PYAS_REC_GENERIC_ONLY together");
    rec &= ~(PYAS_REC_ZERO_SIGN | PYAS_REC_DENSE_ONLY | PYAS_REC_GENERIC_ONLY);
    if (rec < PYAS_REC_FULL || rec > PYAS_REC_MAX) return fail(PYAS_EINVAL, "unknown record form %d", rec);
    pyas::AxesArgs x;
    std::memset(&x, 0, sizeof(x));
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, x.r, es, shuf, bsw, masked);
    if (rc) return rc;
    if (axes_mask >> batch->ndim) return fail(PYAS_EINVAL, "axes mask 0x%x beyond rank %d", axes_mask, batch->ndim);
    if (batch->n_chunks == 0) return PYAS_OK;
    if (!out_offsets || !out) return fail(PYAS_EINVAL, "out/out_offsets is NULL");
    PYAS_HIP(hipSetDevice(ctx->device));
    // Geometry from the full chunk extents (selections only shrink them).
    int64_t keep_elems = 1, red_elems = 1;
    for (int d = 0; d < batch->ndim; ++d) {
        if ((axes_mask >> d) & 1u) red_elems *= batch->chunk_shape[d];
        else keep_elems *= batch->chunk_shape[d];
    }
    if (rec != PYAS_REC_FULL && red_elems >= (int64_t(1) << 31))
        return fail(PYAS_ENOTSUP, "records count in int32: 2^31 or more reduced elements per output");
    x.rec = rec;
    // k_reduce_axes' LDS offset map: one entry per reduced position of a
    // whole chunk (a selection never reduces more; one that does, e.g. a
    // repeated index list, takes the radix walk)
    x.roff_cap = red_elems <= pyas::kAxesLds ? (int32_t)red_elems : 0;
    x.row = ((axes_mask >> (batch->ndim - 1)) & 1u) != 0;
    // 16-B vector walks: >= 4-byte unshuffled elements, no index tables, the
    // reduced offsets fit the LDS map and the last dim is whole 16-B vectors.
    const int64_t last_bytes = (int64_t)batch->chunk_shape[batch->ndim - 1] * es;
    x.vec = es >= 4 && !shuf && !x.r.tab.on[0] && !x.r.tab.on[1] && red_elems <= pyas::kAxesLds &&
            last_bytes % 16 == 0;
    const int64_t nv = 16 / es;   // elements per vector
    auto pow2_floor = [](int64_t v) { int64_t p = 1; while (p * 2 <= v) p *= 2; return p; };
    int64_t per_block, keep_items = keep_elems;
    if (x.row) {   // about 8 reduced elements (or 4 vectors) per lane, G in [1, 64]
        const int64_t per_lane_units = x.vec ? red_elems / nv / 4 : red_elems / 8;
        int64_t g = pow2_floor(per_lane_units > 0 ? per_lane_units : 1);
        x.group = (int32_t)(g > pyas::kWave ? pyas::kWave : g);
        x.split = 1;
        per_block = (pyas::kBlock / pyas::kWave) * (pyas::kWave / x.group);
    } else {       // split the reduced range when a chunk has few outputs (or vectors of them)
        if (x.vec && keep_elems % nv == 0) keep_items = keep_elems / nv;
        else x.vec = false;
        int64_t sp = 1;
        while (sp < pyas::kBlock && keep_items * sp * 2 <= pyas::kBlock && red_elems / (sp * 2) >= 8) sp *= 2;
        x.split = (int32_t)sp;
        x.group = 1;
        per_block = pyas::kBlock / sp;
    }
    // workgroups per chunk: enough to cover the outputs once, but each
    // streaming at least ~128 KiB so the per-workgroup offset map amortises
    int64_t bpc = (keep_items + per_block - 1) / per_block;
    const int64_t by_bytes = (x.r.chunk_elems * es) >> 17;
    if (bpc > by_bytes) bpc = by_bytes;
    if (bpc > 64) bpc = 64;
    if (bpc < 1) bpc = 1;
    x.axes = axes_mask;
    x.bpc = bpc;
    x.out_offsets = out_offsets;
    x.out = reinterpret_cast<pyas_partial *>(out);
    x.shuf = shuf;
    x.bswap = bsw;
    dense_geometry(x.d, batch, axes_mask, es, shuf ? es : 1, x.r.tab.on[0] || x.r.tab.on[1]);
    // Fully selected chunks go to k_axes_dense, the rest to k_reduce_axes
    // (each kernel skips the other's chunks); sel == NULL means all full.
    // With selections, the dense launch also takes the cut chunks whose box
    // covers at least half the chunk (cut_eligible: a hyperslab's edges),
    // read whole with the box applied per row / element; the reduced
    // positions' bit map must fit LDS.  PYAS_AXES_CUTS=0 leaves every cut
    // chunk to k_reduce_axes.
    {
        const char *e = getenv("PYAS_AXES_CUTS");   // per call: tests and benches switch it
        x.cuts = batch->sel && x.d.mode != 0 && !(e && *e == '0') &&
                 x.d.RO * x.d.RI <= 32 * (int64_t)pyas::kCutMapWords &&
                 x.r.chunk_elems < (int64_t(1) << 31);   // 32-bit index arithmetic
    }
    // PYAS_REC_ZERO_SIGN: the column walk keys NumPy's sign of a zero
    // min/max itself (the level-1 calls are elementwise: the innermost dim
    // kept, so the last zero in row order wins), instead of pyas_tie_chunks
    // scanning the chunks again.  Every chunk must then be walked by the
    // dense kernel: whole, or a cut box it takes (the caller's promise).
    if (want_zs) {
        if (rec != PYAS_REC_MIN && rec != PYAS_REC_MAX)
            return fail(PYAS_EINVAL, "PYAS_REC_ZERO_SIGN needs PYAS_REC_MIN or PYAS_REC_MAX");
        if (batch->dtype != PYAS_F32 && batch->dtype != PYAS_F64)
            return fail(PYAS_ENOTSUP, "zero sign: float dtypes only");
        if (batch->sel && !x.cuts) return fail(PYAS_ENOTSUP, "zero sign in the per-chunk walk: cut chunks not taken");
        const pyas::TieRule *t = tie_of(ctx, batch->dtype);
        if (!t) return fail(PYAS_ENOTSUP, "zero sign: no tie rule set for this dtype");
        if (x.d.mode == 1) {
            if ((axes_mask >> (batch->ndim - 1)) & 1u)
                return fail(PYAS_ENOTSUP, "zero sign in the column walk: innermost dim reduced");
        } else if (x.d.mode >= 4) {
            // LDS row layout: each output row is one contiguous NumPy call (of
            // the box's run along the innermost dim for a cut chunk, so the
            // reduced group must be that dim alone), keyed with the rule
            if (batch->sel && x.d.RI != batch->chunk_shape[batch->ndim - 1])
                return fail(PYAS_ENOTSUP, "zero sign in the row walk: a cut chunk's reduced group spans dims");
            if (x.d.RI > 64 || x.d.RI - 1 >= t->piece)
                return fail(PYAS_ENOTSUP, "zero sign in the row walk: rows over 64 elements or NumPy's buffer");
            if (t->lanes < 1 || t->lanes > 64 || (t->lanes & (t->lanes - 1)))
                return fail(PYAS_ENOTSUP, "zero sign in the row walk: a lane count that is not a power of two");
            x.t = *t;
        } else {
            return fail(PYAS_ENOTSUP, "zero sign in the per-chunk walk: column or LDS row layouts only");
        }
        x.zs = rec == PYAS_REC_MIN ? 1 : 2;
    }
    // LDS row layout, whole chunks or the zero-sign kernel: two tiles per
    // wave (C3 (2,) records 0.77-0.79 -> 0.73 ms, 4 tiles 0.74, 3 0.75;
    // the cut kernel's slab (2,) mean measured slower at 2: 1.16 -> 1.23 ms,
    // gpurun_out/r05/rowlds2); PYAS_ROW_LDS_TPW overrides both
    if (x.d.mode >= 4 && (!batch->sel || x.zs) && !getenv("PYAS_ROW_LDS_TPW")) {
        const int64_t per_pass = (pyas::kBlock / pyas::kWave) * (pyas::kWave / x.d.group);
        const int64_t bpc = (x.d.KO + 2 * per_pass - 1) / (2 * per_pass);
        x.d.bpc = bpc < 1 ? 1 : bpc;
    }
    // Streamed column layout (k_axes_col_stream): every chunk whole, one
    // lane per item column (split 1), rows in whole 4-row groups; each
    // workgroup walks cpb chunks as one ring of loads.  Measured on C3
    // (tools/bench_axes.py, profiles/r03/axes_stream_sweep.txt), per
    // geometry:
    //  - plain, kept inner run >= 4 KiB (axis (0,)): 4 items per lane, about
    //    1024 workgroups (0.884 -> 0.795 ms);
    //  - plain otherwise (axis (1,)): 2 items per lane, about 256 workgroups
    //    (0.90 -> 0.805 ms);
    //  - shuffled, kept inner run under 128 elements (axis (1,)): 1 item per
    //    lane, about 512 workgroups (0.975 -> 0.927 ms); other shuffled
    //    geometries measured slower streamed ((0,): 0.846 -> 0.88-1.0 ms) and
    //    keep dense_col.
    // PYAS_COL_STREAM: 0 off, N > 0 forces N chunks per workgroup wherever
    // the kernel can run (tests), unset auto.
    const int64_t col_items = x.d.mode == 1 ? x.d.KO * (x.d.KI / (16 / es)) : 0;
    if (x.d.mode == 1 && !batch->sel && !x.zs && es >= 4 && x.d.split == 1 && x.d.it == pyas::kBlock &&
        (x.d.RO * x.d.RI) % 4 == 0) {
        const char *e = getenv("PYAS_COL_STREAM");   // per call: tests and benches switch it
        const int64_t forced = e ? atoll(e) : -1;
        const int64_t kiv = x.d.KI / (16 / es);     // vectors per kept inner run
        const int nv = shuf ? 1 : (kiv % 256 == 0 && col_items >= 4 * pyas::kBlock) ? 4 : 2;
        // workgroups per CU aimed at (C3: 1024 / 256 / 512 on 256 CUs).  The
        // chunks per workgroup are rounded up, so the grid never exceeds the
        // target: one workgroup past a round of the CUs would take a second
        // round nearly alone (C3 (1,) at 24 or 48 chunks per workgroup:
        // 0.86-0.89 ms against 0.79 at 32; profiles/r03/axes_stream_cpb.txt)
        const int64_t target = (int64_t)ctx->n_cu * (shuf ? 2 : nv == 4 ? 4 : 1);
        // auto: the measured geometries, with every lane's NV items present
        const bool auto_ok = shuf ? x.d.KI < 128 : col_items >= nv * pyas::kBlock;
        const int64_t bpc = (col_items + nv * pyas::kBlock - 1) / (nv * pyas::kBlock);
        int64_t cpb = forced >= 0 ? forced : auto_ok ? (batch->n_chunks * bpc + target - 1) / target : 0;
        if (cpb > batch->n_chunks) cpb = batch->n_chunks;
        if (cpb >= 2 || forced > 0) {
            x.d.cpb = cpb;
            x.d.nv = nv;
            x.d.n_chunks = batch->n_chunks;
            x.d.bpc = bpc;
        }
    }
    // Shuffled chunks whose reduced rows lie inside each kept-outer block
    // (RO == 1, e.g. C3 axis (1,)): k_axes_shuf_slab stages each block's
    // byte-plane runs (RI x KI bytes per plane, whole 1 KiB loads) through
    // LDS.  KI of 64 or 128 output columns, RB rows per 16 KiB tile.
    // PYAS_SHUF_SLAB=0 (or a forced PYAS_COL_STREAM) keeps the column walks.
    // Split 1 only (one lane set walks all rows): the same 4-row groups in the
    // same order as dense_col / k_axes_col_stream / k_axes_fold_lean, so the
    // partials stay bit-identical to theirs.
    if (x.d.mode == 1 && shuf && !batch->sel && !x.zs && es >= 2 && x.d.RO == 1 && (x.d.KI == 64 || x.d.KI == 128) &&
        x.d.split == 1 && !x.r.tab.on[0] && !x.r.tab.on[1]) {
        const char *e = getenv("PYAS_SHUF_SLAB");   // per call: tests and benches switch it
        int64_t rb = pyas::kSlabBytes / (x.d.KI * es);
        if (rb > x.d.RI) rb = x.d.RI;
        rb -= rb % 4;
        const char *e_cs = getenv("PYAS_COL_STREAM");   // a forced column walk keeps that walk
        if (!(e && *e == '0') && !(e_cs && *e_cs) && rb >= 4 && x.d.RI % rb == 0 && (rb * x.d.KI) % 1024 == 0) {
            x.d.rb = rb;
            x.d.cpb = 0;
            x.d.n_chunks = batch->n_chunks;
            // persistent waves: two 4-wave workgroups per CU (64 KiB of LDS each)
            const int64_t units = batch->n_chunks * x.d.KO;
            int64_t wgs = (int64_t)ctx->n_cu * 2;
            if (wgs * (pyas::kBlock / pyas::kWave) > units) wgs = (units + 3) / 4;
            PYAS_HIP(pyas::launch_axes_dense(batch->dtype, x, masked, wgs, (hipStream_t)stream));
            return PYAS_OK;
        }
    }
    if (x.d.mode && !(generic_only && batch->sel)) {
        const int64_t g = (x.d.cpb > 0 ? (batch->n_chunks + x.d.cpb - 1) / x.d.cpb : batch->n_chunks) * x.d.bpc;
        if (g >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
        PYAS_HIP(pyas::launch_axes_dense(batch->dtype, x, masked, g, (hipStream_t)stream));
    }
    if (!x.d.mode || (batch->sel && !(dense_only && x.cuts))) {
        // with cut chunks in the dense launch, the generic kernel keeps only
        // boxes under half a chunk and non-box selections: one workgroup per
        // chunk (most of its workgroups only find their chunk taken; at 8 per
        // chunk that empty launch cost C3 [1:1023]^3 (2,) 74 us, at one 13 us;
        // with the caller's PYAS_REC_DENSE_ONLY it is not launched)
        if (x.cuts) x.bpc = 1;
        const int64_t grid = batch->n_chunks * x.bpc;
        if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
        PYAS_HIP(pyas::launch_reduce_axes(batch->dtype, x, grid, (hipStream_t)stream));
    }
    return PYAS_OK;
}

int pyas_reduce_axes_grid(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                          const pyas_grid *g, uint32_t combine_flags, pyas_partial *out,
                          void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!g || !out) return fail(PYAS_EINVAL, "NULL argument");
    pyas::AxesArgs x;
    std::memset(&x, 0, sizeof(x));
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, x.r, es, shuf, bsw, masked);
    if (rc) return rc;
    if (combine_flags & ~(PYAS_COMBINE_ROUND_TO_VAR | PYAS_FOLD_ZERO_SIGN_MIN | PYAS_FOLD_ZERO_SIGN_MAX))
        return fail(PYAS_EINVAL, "unknown combine flags 0x%x", combine_flags);
    if (g->ndim != batch->ndim) return fail(PYAS_EINVAL, "grid rank %d != batch rank %d", g->ndim, batch->ndim);
    const uint32_t axes_mask = g->axes_mask;
    if (axes_mask == 0 || (axes_mask >> batch->ndim))
        return fail(PYAS_EINVAL, "axes mask 0x%x for rank %d", axes_mask, batch->ndim);
    if (batch->sel) return fail(PYAS_ENOTSUP, "the in-kernel layer fold needs whole chunks (sel == NULL)");
    pyas::FoldGrid fg;
    std::memset(&fg, 0, sizeof(fg));
    // NumPy's zero sign fused into the lean column fold (floats; the caller
    // has checked that both reductions are elementwise)
    fg.zs = (batch->dtype == PYAS_F32 || batch->dtype == PYAS_F64) ? (combine_flags >> 8) & 3u : 0u;
    combine_flags &= ~(PYAS_FOLD_ZERO_SIGN_MIN | PYAS_FOLD_ZERO_SIGN_MAX);
    int64_t n_pos = 1, ost = 1;
    fg.n_layers = 1;
    fg.n_cols = 1;
    for (int d = batch->ndim - 1; d >= 0; --d) {
        if (g->n_coords[d] < 1) return fail(PYAS_EINVAL, "n_coords[%d] = %lld", d, (long long)g->n_coords[d]);
        fg.n_coords[d] = g->n_coords[d];
        n_pos *= g->n_coords[d];
        if ((axes_mask >> d) & 1u) {
            fg.n_layers *= g->n_coords[d];
        } else {
            if (g->out_extent[d] != g->n_coords[d] * batch->chunk_shape[d])
                return fail(PYAS_EINVAL, "out_extent[%d] = %lld is not n_coords x chunk extent", d,
                            (long long)g->out_extent[d]);
            fg.n_cols *= g->n_coords[d];
            fg.ostride[d] = ost;
            ost *= g->out_extent[d];
        }
    }
    if (n_pos != batch->n_chunks)
        return fail(PYAS_EINVAL, "%lld chunks for a grid of %lld", (long long)batch->n_chunks, (long long)n_pos);
    fg.flags = combine_flags;
    dense_geometry(x.d, batch, axes_mask, es, shuf ? es : 1, x.r.tab.on[0] || x.r.tab.on[1]);
    if ((x.d.mode != 1 && x.d.mode < 4) || es < 4)
        return fail(PYAS_ENOTSUP, "the in-kernel layer fold needs the dense column or LDS row layout");
    // Each workgroup walks every layer of its column, so the grid is only
    // n_cols x bpc: trade items per pass for splits of the reduced rows
    // until the launch fills the chip (>= 8 workgroups per CU by default).
    const int64_t min_blocks = ctx->fold_min_blocks;
    // Lean column fold (k_axes_fold_lean): the split-1 geometry the two-step
    // path uses (so bit-identical), whole 4-row groups, and enough lanes in
    // the grid that no split is needed (PYAS_FOLD_LEAN=0 turns it off).
    // Split each column's layers in two halves (twice the lanes) when the
    // unsplit grid is under two rounds of 1024 workgroups and the second half
    // fits the LDS sums.  PYAS_FOLD_LEAN: 0 off, 1 unsplit, 2 split, unset auto.
    const char *e_lean = getenv("PYAS_FOLD_LEAN");   // per call: tests and benches switch it
    const int lean_env = e_lean ? atoi(e_lean) : -1;
    const int64_t lean_items = x.d.mode == 1 ? x.d.KO * (x.d.KI / (16 / es)) : 0;
    const int64_t lean_bpc1 = (lean_items + pyas::kBlock - 1) / pyas::kBlock;
    const bool can_split = fg.n_layers >= 2 && fg.n_layers - (fg.n_layers + 1) / 2 <= pyas::kLeanMaxB;
    if (lean_env != 0 && x.d.mode == 1 && x.d.split == 1 && (x.d.RO * x.d.RI) % 4 == 0 &&
        fg.n_layers * x.d.RO * x.d.RI < (int64_t(1) << 31) &&   // per-lane uint32 counts
        fg.n_cols * lean_bpc1 >= min_blocks / 2) {
        // auto: only where the rows of a chunk sit inside a kept-outer run
        // (RI > 1, e.g. C3 axis (1,): 0.71 -> 0.67 ms); with RO rows 16 KiB+
        // apart (axis (0,)) the split measured 0.71 -> 0.73 ms
        const bool split = can_split && (lean_env == 2 ||
                                         (lean_env < 0 && x.d.RI > 1 && fg.n_cols * lean_bpc1 < 2048));
        fg.lean = split ? 2 : 1;
        x.d.bpc = (lean_items + pyas::kBlock / fg.lean - 1) / (pyas::kBlock / fg.lean);
    } else if (x.d.mode >= 4) {   // LDS row layout: one output tile per wave
        const int64_t rpw = pyas::kWave / x.d.group, per_block = (pyas::kBlock / pyas::kWave) * rpw;
        x.d.bpc = (x.d.KO + per_block - 1) / per_block;
    } else {
        const int64_t items = x.d.KO * (x.d.KI / (16 / es)), rows = x.d.RO * x.d.RI;
        while (fg.n_cols * x.d.bpc < min_blocks && x.d.it > 32 && rows >= (int64_t)x.d.split * 2 * 4 &&
               x.d.split * 2 <= pyas::kBlock / (x.d.it / 2)) {
            x.d.it /= 2;
            x.d.split *= 2;
            x.d.bpc = (items + x.d.it - 1) / x.d.it;
        }
    }
    if (fg.n_cols * x.d.bpc < min_blocks / 4)
        return fail(PYAS_ENOTSUP, "in-kernel layer fold: %lld workgroups are too few to fill the device",
                    (long long)(fg.n_cols * x.d.bpc));
    if (fg.zs) {
        // level 2: the `out` array (C-ordered, active.py:512) reduced over the
        // chunk-grid dims -- its call is the trailing reduced group
        // (zerosign.grid_lr)
        int64_t lr2 = 1;
        for (int d = batch->ndim - 1; d >= 0; --d) {
            const bool red = (axes_mask >> d) & 1u;
            const int64_t ext = red ? g->n_coords[d] : g->out_extent[d];
            if (ext == 1) continue;
            if (!red) break;
            lr2 *= ext;
        }
        if (fg.lean) {
            // the lean fold tracks "the last zero wins": both reductions
            // elementwise (the chunk's innermost non-1 dim kept, lr2 == 1)
            bool inner_kept = false;
            for (int d = batch->ndim - 1; d >= 0; --d) {
                if (batch->chunk_shape[d] == 1) continue;
                inner_kept = !((axes_mask >> d) & 1u);
                break;
            }
            if (!inner_kept || lr2 != 1)
                return fail(PYAS_ENOTSUP, "zero sign in the lean column fold: a reduction is not elementwise");
            // the sign is NumPy's only where a tie rule was derived and
            // validated for this dtype on this host (pyas.h: ENOTSUP otherwise)
            if (!tie_of(ctx, batch->dtype))
                return fail(PYAS_ENOTSUP, "zero sign in the lean column fold: no tie rule set for this dtype");
        } else if (x.d.mode >= 4) {
            // LDS row layout: each output row (RI elements, RO == KI == 1) is
            // one contiguous NumPy call; the rule comes from the context
            const pyas::TieRule *t = tie_of(ctx, batch->dtype);
            if (!t) return fail(PYAS_ENOTSUP, "zero sign in the row fold: no tie rule set for this dtype");
            if (fg.zs == 3u) return fail(PYAS_ENOTSUP, "zero sign in the row fold: min or max, not both");
            if (x.d.RI - 1 >= t->piece || lr2 >= (int64_t(1) << 31))
                return fail(PYAS_ENOTSUP, "zero sign in the row fold: call longer than NumPy's buffer");
            if (x.d.RI > 64) return fail(PYAS_ENOTSUP, "zero sign in the row fold: rows over 64 elements");
            if (t->lanes & (t->lanes - 1))
                return fail(PYAS_ENOTSUP, "zero sign in the row fold: a lane count that is not a power of two");
            fg.t = *t;
            fg.c2 = grid_call(*t, lr2);
            // the row call's positions as bit masks: e = 0 the seed, then
            // m = RI - 1 elements, the first nv in L lanes, the rest remainder
            const int64_t m = x.d.RI - 1, L = t->lanes, nv = m - m % L;
            for (int64_t e = nv + 1; e < x.d.RI; ++e) fg.zrow_rem |= uint64_t(1) << e;
            for (int64_t e = 1; e <= nv; ++e) {
                const int r = t->rank[(e - 1) % L];
                fg.zrow_cm[r] |= uint64_t(1) << e;
                fg.zrow_vec |= uint64_t(1) << e;
                if (r == 0) fg.zrow_top |= uint64_t(1) << e;
            }
            for (int64_t b = 0; b * L < 64; ++b) fg.zrow_rep |= uint64_t(1) << (b * L);
        } else {
            return fail(PYAS_ENOTSUP, "the zero sign is fused into the lean column and the row folds only (this "
                                      "geometry takes k_axes_fold)");
        }
    }
    x.axes = axes_mask;
    x.out = out;
    x.shuf = shuf;
    x.bswap = bsw;
    const int64_t grid = fg.n_cols * x.d.bpc;
    if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_axes_fold(batch->dtype, x, fg, masked, grid, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_select_chunks(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                       const int64_t *out_offsets, void *values, uint8_t *mask_out,
                       void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    pyas::SelectArgs x;
    std::memset(&x, 0, sizeof(x));
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, x.r, es, shuf, bsw, masked);
    if (rc) return rc;
    if (batch->n_chunks == 0) return PYAS_OK;
    if (!out_offsets || !values) return fail(PYAS_EINVAL, "values/out_offsets is NULL");
    PYAS_HIP(hipSetDevice(ctx->device));
    int64_t bpc = (x.r.chunk_elems + pyas::kBlock - 1) / pyas::kBlock;
    if (bpc > 64) bpc = 64;
    x.bpc = bpc;
    x.out_offsets = out_offsets;
    x.values = values;
    x.mask_out = mask_out;
    x.shuf = shuf;
    x.bswap = bsw;
    const int64_t grid = batch->n_chunks * bpc;
    if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
    PYAS_HIP(pyas::launch_select(batch->dtype, x, grid, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_select_scatter(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                        const pyas_scatter *scatter, void *values, uint8_t *mask_out,
                        void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (!scatter || !scatter->pos || !scatter->chunk_base)
        return fail(PYAS_EINVAL, "scatter tables are NULL");
    pyas::SelectArgs x;
    std::memset(&x, 0, sizeof(x));
    int es;
    bool shuf, bsw, masked;
    int rc = prepare(ctx, batch, mask, x.r, es, shuf, bsw, masked);
    if (rc) return rc;
    if (batch->n_chunks == 0) return PYAS_OK;
    if (!values) return fail(PYAS_EINVAL, "values is NULL");
    PYAS_HIP(hipSetDevice(ctx->device));
    int64_t bpc = (x.r.chunk_elems + pyas::kBlock - 1) / pyas::kBlock;
    if (bpc > 64) bpc = 64;
    x.bpc = bpc;
    x.values = values;
    x.mask_out = mask_out;
    x.shuf = shuf;
    x.bswap = bsw;
    x.scatter_pos = scatter->pos;
    x.scatter_base = scatter->chunk_base;
    for (int d = 0; d < PYAS_MAX_DIMS; ++d) x.ostride[d] = scatter->out_stride[d];
    const int64_t grid = batch->n_chunks * bpc;
    if (grid >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
    PYAS_HIP(pyas::launch_select(batch->dtype, x, grid, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_combine_partials(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in, int64_t n,
                          uint32_t combine_flags, pyas_partial *out, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (elem_size(dtype) == 0) return fail(PYAS_ENOTSUP, "unsupported dtype code %d", dtype);
    if (!out || (n > 0 && !in)) return fail(PYAS_EINVAL, "NULL partials");
    if (combine_flags & ~PYAS_COMBINE_ROUND_TO_VAR)
        return fail(PYAS_EINVAL, "unknown combine flags 0x%x", combine_flags);
    PYAS_HIP(hipSetDevice(ctx->device));
    void *scr = nullptr;
    int rc = ensure_scratch(ctx, stream, ((size_t)(n / kSeg) + 2) * sizeof(pyas_partial), &scr);
    if (rc) return rc;
    return combine_into(dtype, in, n, combine_flags, (pyas_partial *)scr, out, (hipStream_t)stream);
}

int pyas_combine_segments(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in,
                          const int64_t *index, const int64_t *seg_offsets, int64_t n_segments,
                          uint32_t combine_flags, pyas_partial *out, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (elem_size(dtype) == 0) return fail(PYAS_ENOTSUP, "unsupported dtype code %d", dtype);
    if (n_segments < 0) return fail(PYAS_EINVAL, "negative segment count");
    if (n_segments == 0) return PYAS_OK;
    if (!in || !index || !seg_offsets || !out) return fail(PYAS_EINVAL, "NULL argument");
    // PYAS_COMBINE_REC: `in` holds compact records (pyas_reduce_axes_ex)
    if (combine_flags & ~(PYAS_COMBINE_ROUND_TO_VAR | PYAS_COMBINE_REC(3)))
        return fail(PYAS_EINVAL, "unknown combine flags 0x%x", combine_flags);
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_combine_segments(dtype, in, index, seg_offsets, n_segments, combine_flags,
                                           out, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_combine_grid(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in, const pyas_grid *g,
                      uint32_t combine_flags, pyas_partial *out, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (elem_size(dtype) == 0) return fail(PYAS_ENOTSUP, "unsupported dtype code %d", dtype);
    if (!g) return fail(PYAS_EINVAL, "grid is NULL");
    if (g->ndim < 1 || g->ndim > PYAS_MAX_DIMS)
        return fail(PYAS_EINVAL, "grid rank %d outside 1..%d", g->ndim, PYAS_MAX_DIMS);
    if (g->axes_mask >> g->ndim) return fail(PYAS_EINVAL, "axes mask 0x%x beyond rank %d", g->axes_mask, g->ndim);
    // PYAS_COMBINE_REC: `in` holds compact records (pyas_reduce_axes_ex)
    if (combine_flags & ~(PYAS_COMBINE_ROUND_TO_VAR | PYAS_COMBINE_REC(3) | PYAS_FOLD_ZERO_SIGN_MIN |
                          PYAS_FOLD_ZERO_SIGN_MAX))
        return fail(PYAS_EINVAL, "unknown combine flags 0x%x", combine_flags);
    // PYAS_FOLD_ZERO_SIGN_*: `in` carries level 1's signs (PYAS_REC_ZERO_SIGN);
    // the combine keys level 2 itself: when the `out` array's calls are
    // elementwise (its trailing non-1 dims kept) the last zero layer wins,
    // else the keys over each call's zero layers decide (tie_keys)
    pyas::CombineTie ct;
    std::memset(&ct, 0, sizeof(ct));
    if (combine_flags & (PYAS_FOLD_ZERO_SIGN_MIN | PYAS_FOLD_ZERO_SIGN_MAX)) {
        if ((combine_flags & (PYAS_FOLD_ZERO_SIGN_MIN | PYAS_FOLD_ZERO_SIGN_MAX)) ==
            (PYAS_FOLD_ZERO_SIGN_MIN | PYAS_FOLD_ZERO_SIGN_MAX))
            return fail(PYAS_EINVAL, "zero sign: min or max, not both");
        if (dtype != PYAS_F32 && dtype != PYAS_F64) return fail(PYAS_ENOTSUP, "zero sign: float dtypes only");
        if (!tie_of(ctx, dtype)) return fail(PYAS_ENOTSUP, "zero sign: no tie rule set for this dtype");
        int64_t lr2 = 1;
        for (int d = g->ndim - 1; d >= 0; --d) {
            const bool red = (g->axes_mask >> d) & 1u;
            const int64_t ext = red ? g->n_coords[d] : g->out_extent[d];
            if (ext == 1) continue;
            if (!red) break;
            lr2 *= ext;
        }
        // calls of lr2 > 1 layers: the keys of NumPy's reduce over each call
        // (k_tie_grid_t's, in the same pass instead of a second launch)
        if (lr2 != 1) {
            ct.on = 1;
            ct.t = *tie_of(ctx, dtype);
            ct.c = grid_call(ct.t, lr2);
        }
        combine_flags |= pyas::kCombineThreadOnly;   // the per-thread form keys it
    }
    int64_t n_out = 1, n_layers = 1;
    for (int d = 0; d < g->ndim; ++d) {
        if (g->n_coords[d] < 1) return fail(PYAS_EINVAL, "n_coords[%d] = %lld", d, (long long)g->n_coords[d]);
        if ((g->axes_mask >> d) & 1u) {
            n_layers *= g->n_coords[d];
        } else {
            if (g->out_extent[d] < 1) return fail(PYAS_EINVAL, "out_extent[%d] = %lld", d, (long long)g->out_extent[d]);
            if (!g->pos_coord[d] || !g->pos_local[d] || !g->coord_count[d])
                return fail(PYAS_EINVAL, "kept dim %d has a NULL table", d);
            n_out *= g->out_extent[d];
        }
    }
    if (!in || !out || !g->chunk_out_offsets) return fail(PYAS_EINVAL, "NULL argument");
    if (ct.on && n_layers >= (int64_t(1) << 31))   // the keyed combine's 32-bit layer positions
        return fail(PYAS_ENOTSUP, "zero sign: more than 2^31 chunk layers");
    PYAS_HIP(hipSetDevice(ctx->device));
    // PYAS_COMBINE_WAVE=0 (read per call: tests switch it) keeps the
    // per-thread fold for every layer count
    const char *e_wave = getenv("PYAS_COMBINE_WAVE");
    if (e_wave && std::strcmp(e_wave, "0") == 0) combine_flags |= pyas::kCombineThreadOnly;
    PYAS_HIP(pyas::launch_combine_grid(dtype, in, *g, ct, n_out, n_layers, combine_flags, out,
                                       (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_format_partials(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in, int64_t n,
                         int32_t method, void *values, uint8_t *mask, int64_t *counts,
                         void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (elem_size(dtype) == 0) return fail(PYAS_ENOTSUP, "unsupported dtype code %d", dtype);
    if (method < PYAS_FORMAT_SUM || method > PYAS_FORMAT_MEAN)
        return fail(PYAS_EINVAL, "unknown format method %d", method);
    if (n < 0) return fail(PYAS_EINVAL, "negative partial count");
    if (n == 0) return PYAS_OK;
    if (n >= (int64_t(1) << 40)) return fail(PYAS_ENOTSUP, "too many partials");
    if (!in || !values || !mask) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_format(dtype, in, n, method, values, mask, counts, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_unshuffle(pyas_ctx *ctx, const void *src, void *dst, int64_t n_bytes, int32_t elementsize,
                   void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n_bytes < 0 || elementsize < 1) return fail(PYAS_EINVAL, "bad size/elementsize");
    if (n_bytes == 0) return PYAS_OK;
    if (!src || !dst) return fail(PYAS_EINVAL, "NULL buffer");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_unshuffle(src, dst, n_bytes, elementsize, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_unshuffle_chunks(pyas_ctx *ctx, const void *src, const int64_t *src_offsets, void *dst,
                          const int64_t *dst_offsets, int64_t n_chunks, int64_t chunk_bytes,
                          int32_t elementsize, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n_chunks < 0 || chunk_bytes < 0) return fail(PYAS_EINVAL, "bad n_chunks/chunk_bytes");
    if (elementsize != 2 && elementsize != 4 && elementsize != 8)
        return fail(PYAS_ENOTSUP, "pyas_unshuffle_chunks: elementsize %d (2, 4 or 8)", elementsize);
    if (n_chunks == 0 || chunk_bytes == 0) return PYAS_OK;
    if (!src || !dst || !src_offsets || !dst_offsets) return fail(PYAS_EINVAL, "NULL buffer");
    if (n_chunks * ((chunk_bytes + 4095) / 4096) >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "grid too large");
    PYAS_HIP(hipSetDevice(ctx->device));
    PYAS_HIP(pyas::launch_unshuffle_chunks(src, src_offsets, dst, dst_offsets, n_chunks, chunk_bytes,
                                           elementsize, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_inflate(pyas_ctx *ctx, const uint8_t *src, const int64_t *src_offsets,
                 const int64_t *src_sizes, int64_t n, uint8_t *dst,
                 const int64_t *dst_offsets, const int64_t *dst_capacity,
                 int64_t *out_sizes, int32_t *status, void *stream) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (n < 0) return fail(PYAS_EINVAL, "negative stream count");
    if (n == 0) return PYAS_OK;
    if (!src || !src_offsets || !src_sizes || !dst || !dst_offsets || !dst_capacity || !out_sizes || !status)
        return fail(PYAS_EINVAL, "NULL array");
    if (n >= (int64_t(1) << 31)) return fail(PYAS_ENOTSUP, "too many streams");
    PYAS_HIP(hipSetDevice(ctx->device));
    pyas::InflateArgs x{src, src_offsets, src_sizes, dst, dst_offsets, dst_capacity, out_sizes, status};
    PYAS_HIP(pyas::launch_inflate(x, n, ctx->inflate_wbits, (hipStream_t)stream));
    return PYAS_OK;
}

int pyas_timing_enable(pyas_ctx *ctx, int32_t max_launches) {
    if (!ctx) return fail(PYAS_EINVAL, "ctx is NULL");
    if (max_launches < 0) return fail(PYAS_EINVAL, "max_launches < 0");
    PYAS_HIP(hipSetDevice(ctx->device));
    for (auto e : ctx->ev0) (void)hipEventDestroy(e);
    for (auto e : ctx->ev1) (void)hipEventDestroy(e);
    ctx->ev0.assign(max_launches, nullptr);
    ctx->ev1.assign(max_launches, nullptr);
    for (int i = 0; i < max_launches; ++i) {
        PYAS_HIP(hipEventCreate(&ctx->ev0[i]));
        PYAS_HIP(hipEventCreate(&ctx->ev1[i]));
    }
    ctx->timing_n = 0;
    return PYAS_OK;
}

int pyas_timing_read(pyas_ctx *ctx, float *ms, int32_t cap, int32_t *n) {
    if (!ctx || !n) return fail(PYAS_EINVAL, "NULL argument");
    PYAS_HIP(hipSetDevice(ctx->device));
    const int32_t m = ctx->timing_n < cap ? ctx->timing_n : cap;
    for (int i = 0; i < m; ++i) {
        PYAS_HIP(hipEventSynchronize(ctx->ev1[i]));
        PYAS_HIP(hipEventElapsedTime(&ms[i], ctx->ev0[i], ctx->ev1[i]));
    }
    *n = m;
    return PYAS_OK;
}

}  // extern "C"
