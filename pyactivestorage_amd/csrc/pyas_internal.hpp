// pyas_internal.hpp — kernel argument blocks and launcher prototypes shared by
// pyas_kernels.hip (device code) and pyas_capi.hip (the extern "C" boundary).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "pyas.h"
#include "pyas_device.hpp"

namespace pyas {

// Passed by value in the kernarg segment (a few hundred bytes).
struct ReduceArgs {
    const uint8_t *data;
    const int64_t *offsets;
    const int32_t *sel;
    const int32_t *pool;
    int64_t shape[PYAS_MAX_DIMS];
    int64_t cstride[PYAS_MAX_DIMS];   // row-major element strides of a chunk
    int64_t chunk_elems;
    int64_t tpc;                      // tiles (workgroups) per chunk
    int32_t ndim;
    int32_t spans;                    // run_spans: 0 off, 1 cut chunks run_rows cannot stream, 2 every cut chunk
    pyas_mask mask;
    MaskTab tab;
    pyas_partial *out;                // one partial per workgroup (tile b of chunk b / tpc)
};

// Chunks per first-level combine group: one k_finish block, one thread per
// chunk (k_combine uses the same segments, so both orders agree).
constexpr int64_t kCombineSeg = kBlock;

// k_finish: tile partials -> chunk partials -> group partials -> total
struct FinishArgs {
    const pyas_partial *tiles;        // n_chunks * tpc, chunk-major
    int64_t tpc, n_chunks;
    pyas_partial *chunk_out;          // may be NULL
    pyas_partial *gtmp;               // n_chunks / kCombineSeg + 1 group partials
    pyas_partial *total;              // may be NULL (chunk partials only)
    uint32_t *cnt;                    // zeroed arrival counter; NULL: the host folds gtmp
    uint32_t flags;                   // PYAS_COMBINE_*
};

constexpr int kCutMapWords = 512;   // cut chunks' reduced-position bit map in LDS (16384 positions; + 1 pad word)
constexpr int kAxesLds = 8192;   // reduced-index offsets kept in LDS (int32, 32 KiB)

// Dense partial-axis geometry (k_axes_dense): the chunk dims merged into
// (RO, KO, RI, KI) = (reduced outer, kept outer, reduced inner, kept inner).
constexpr int kSlabBytes = 16384;     // k_axes_shuf_slab: LDS tile per wave (plain elements)

struct AxesDense {
    int32_t mode;                     // 0 off, 1 column, 2 row, 3 row with 4 outputs per lane,
                                      // 4/5/6 row through LDS with 1/2/4 lanes per output
    int32_t it, split;                // column: items per pass (power of 2), row splits
    int32_t group;                    // row: lanes per output (power of 2)
    int64_t RO, KO, RI, KI;
    int64_t bpc;                      // workgroups per chunk of the dense launch
    int64_t cpb;                      // column layout: chunks per workgroup of k_axes_col_stream (0: off)
    int32_t nv;                       // k_axes_col_stream: items per lane (1, 2 or 4)
    int64_t n_chunks;                 // k_axes_col_stream / k_axes_shuf_slab: chunks in the batch
    int64_t rb;                       // k_axes_shuf_slab: rows per LDS tile (0: off)
};

// NumPy's sign of a zero min/max (pyas_tie_*); float types only
struct TieRule {
    int32_t lanes, piece, acc;        // lanes 0: no rule set
    uint8_t rank[64], acc_rank[64];
};
struct AxesArgs {
    ReduceArgs r;
    AxesDense d;
    uint32_t axes;
    int64_t bpc;                      // workgroups per chunk
    const int64_t *out_offsets;
    pyas_partial *out;
    bool shuf, bswap;
    bool row;                         // innermost dim reduced: G lanes per output
    int32_t group;                    // row layout: lanes per output (power of 2)
    int32_t split;                    // column layout: splits of the reduced range
    bool vec;                         // geometry admits 16-B vector walks (kernel re-checks per chunk)
    int32_t rec;                      // per-chunk outputs: 0 pyas_partial, else a PYAS_REC_* record
    bool cuts;                        // dense launch also takes cut chunks (box, >= half the chunk)
    int32_t zs;                       // the walk keys NumPy's sign of a zero min (1) / max (2)
    TieRule t;                        // zs in the LDS row layout: the host's rule (rows are calls)
    int32_t roff_cap;                 // k_reduce_axes: entries of its LDS offset map (dynamic LDS, <= kAxesLds)
};

// pyas_reduce_axes_grid: the chunk layers of a whole-chunk box query folded
// inside the dense column kernel (no per-chunk partial arrays)
// pyas_combine_grid: internal combine flag (PYAS_COMBINE_WAVE=0) keeping the
// per-thread fold (k_combine_grid) for every layer count
constexpr uint32_t kCombineThreadOnly = 1u << 31;
constexpr int kLeanMaxB = 8;         // k_axes_fold_lean: layers of a split column's second half (LDS sums)
struct FoldGrid;                     // below, after the tie structs it carries


struct InflateArgs {
    const uint8_t *src;
    const int64_t *src_offsets, *src_sizes;
    uint8_t *dst;
    const int64_t *dst_offsets, *dst_capacity;
    int64_t *out_sizes;
    int32_t *status;
};

struct SelectArgs {
    ReduceArgs r;
    int64_t bpc;
    const int64_t *out_offsets;
    void *values;
    uint8_t *mask_out;
    bool shuf, bswap;
    // scatter mode (pyas_select_scatter): element k of chunk c's selection
    // lands at sum_d pos[base[c][d] + k_d] * ostride[d] of the output array
    const int64_t *scatter_pos;
    const int32_t *scatter_base;
    int64_t ostride[PYAS_MAX_DIMS];
};

// Per-dtype launchers: defined in pyas_kernels.hpp, instantiated per dtype by
// pyas_inst.hip.
template <typename T>
hipError_t launch_reduce_t(const ReduceArgs &a, bool shuf, bool bsw, bool masked, int64_t grid,
                           hipStream_t st);
template <typename T>
hipError_t launch_finish_t(const FinishArgs &f, hipStream_t st);
template <typename T>
hipError_t launch_combine_t(const pyas_partial *in, int64_t n, int64_t seg, int64_t nblocks,
                            uint32_t flags, pyas_partial *out, hipStream_t st);
template <typename T>
hipError_t launch_combine_segments_t(const pyas_partial *in, const int64_t *index,
                                     const int64_t *seg, int64_t n_seg, uint32_t flags,
                                     pyas_partial *out, hipStream_t st);
template <typename T>
hipError_t launch_axes_t(const AxesArgs &a, int64_t grid, hipStream_t st);
struct CombineTie;   // below, after the tie structs it carries
template <typename T>
hipError_t launch_combine_grid_t(const pyas_partial *in, const pyas_grid &g, const CombineTie &ct, int64_t n_out,
                                 int64_t n_layers, uint32_t flags, pyas_partial *out,
                                 hipStream_t st);
template <typename T>
hipError_t launch_axes_dense_t(const AxesArgs &a, bool masked, int64_t grid, hipStream_t st);
template <typename T>
hipError_t launch_axes_dense_rows_t(const AxesArgs &a, bool masked, int64_t grid, hipStream_t st);
template <typename T>
hipError_t launch_axes_fold_t(const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                              hipStream_t st);
template <typename T>
hipError_t launch_axes_fold_rows_t(const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                                   hipStream_t st);
template <typename T>
hipError_t launch_select_t(const SelectArgs &a, int64_t grid, hipStream_t st);
struct TieCall {
    int32_t acc;                      // 1: strided reduce loop (accumulator keys)
    uint32_t block;                   // acc: kept dims of NumPy's copied first buffer fill
    int64_t lr, npr;                  // call length (1: elementwise), pieces per call
    int64_t n_copy;                   // acc: runs of that fill (contiguous calls), 0: none
};
// k_combine_grid keying level 2 of NumPy's zero sign itself for `out` calls
// of any length (on = 1): the call and the host's rule
struct CombineTie {
    TieCall c;
    TieRule t;
    int32_t on;
};
struct FoldGrid {
    int64_t n_coords[PYAS_MAX_DIMS];  // chunk coordinates per dim (chunk n = C-order position)
    int64_t ostride[PYAS_MAX_DIMS];   // final-output element strides (kept dims)
    int64_t n_layers, n_cols;         // chunks along the reduced dims / kept dims
    uint32_t flags;                   // PYAS_COMBINE_*
    int32_t lean;                     // column layout: k_axes_fold_lean (split 1, rows % 4 == 0),
                                      // 1 = one lane per column item, 2 = layers split over two
    uint32_t zs;                      // NumPy's zero sign fused for min (1) / max (2)
    TieRule t;                        // zs in k_axes_fold_row: the host's rule,
    TieCall c2;                       //   the `out` array's call (level 2), and masks over a
    uint64_t zrow_rem, zrow_top;      //   row's positions e (RI <= 64): remainder, top-priority lane,
    uint64_t zrow_vec, zrow_rep;      //   all lane positions, lane 0's positions (from e = 1),
    uint64_t zrow_cm[64];             //   lane-rank classes (zrow_cm[r]: the lane of rank r)
};
struct TieChunkArgs {
    ReduceArgs r;
    TieRule t;
    pyas_tie_geom g;
    uint32_t axes, which;
    bool shuf, bswap;
    const int64_t *out_offsets;       // NULL: one output per chunk, at index c
    pyas_partial *parts;              // rewrite mode, or NULL and:
    uint8_t *flags;                   //   flag mode (one byte per chunk output)
    const uint32_t *gate;             //   flag mode: skip when *gate == 0
    int64_t n_chunks;
    int32_t cpw;                      // chunks per workgroup: 1, or a wave per chunk (one output each)
    int32_t group;                    // lanes per output: 1, 16 or 64 (k_tie_scan)
    const uint64_t *pick;             // non-NULL (full reductions): only the chunks of the level-2
    TieCall pick_call;                //   K1 / W keys pick[0] / pick[1] (positions pick_base + c
    int64_t pick_base;                //   of the `out` call pick_call), a wave each
};
struct TieGridArgs {
    pyas_grid g;                      // kind 0: layers from the grid tables
    const int64_t *index, *seg;       // kind 1: segments (index NULL: identity)
    int32_t kind;                     // 2: one output, layer l = entry l
    const pyas_partial *parts;        // level-1 partials, or
    const uint8_t *flags;             //   level-1 flag bytes
    pyas_partial *fin;
    uint64_t *keys;
    int64_t n_out, n_layers, layer_base, slices;
    int32_t per_thread;               // k_tie_grid_t: a thread per output (few layers, many outputs)
    TieCall call;
    TieRule t;
    uint32_t which;
};
template <typename T>
hipError_t launch_tie_chunks_t(const TieChunkArgs &a, int64_t grid, hipStream_t st);
template <typename T>
hipError_t launch_tie_gate_t(const pyas_partial *fin, int64_t n, uint32_t which, uint32_t *gate, hipStream_t st);
template <typename T>
hipError_t launch_tie_grid_t(const TieGridArgs &a, hipStream_t st);
template <typename T>
hipError_t launch_tie_pick_t(const pyas_partial *parts, int64_t n, uint32_t which, int64_t base, const TieCall &call,
                             const TieRule &t, uint64_t *keys, hipStream_t st);
template <typename T>
hipError_t launch_tie_finalize_t(const uint64_t *keys, int64_t n_out, int32_t n_sets, const TieCall &call,
                                 const TieRule &t, uint32_t which, pyas_partial *fin, hipStream_t st);
template <typename T>
hipError_t launch_format_t(const pyas_partial *in, int64_t n, int32_t method, void *values,
                           uint8_t *mask, int64_t *counts, hipStream_t st);

// dtype dispatch (pyas_kernels.hip)
hipError_t launch_reduce(int dtype, const ReduceArgs &a, bool shuf, bool bsw, bool masked,
                         int64_t grid, hipStream_t st);
hipError_t launch_finish(int dtype, const FinishArgs &f, hipStream_t st);
hipError_t launch_combine(int dtype, const pyas_partial *in, int64_t n, int64_t seg,
                          int64_t nblocks, uint32_t flags, pyas_partial *out, hipStream_t st);
hipError_t launch_combine_segments(int dtype, const pyas_partial *in, const int64_t *index,
                                   const int64_t *seg, int64_t n_seg, uint32_t flags,
                                   pyas_partial *out, hipStream_t st);
hipError_t launch_reduce_axes(int dtype, const AxesArgs &a, int64_t grid, hipStream_t st);
hipError_t launch_combine_grid(int dtype, const pyas_partial *in, const pyas_grid &g, const CombineTie &ct,
                               int64_t n_out, int64_t n_layers, uint32_t flags,
                               pyas_partial *out, hipStream_t st);
hipError_t launch_axes_dense(int dtype, const AxesArgs &a, bool masked, int64_t grid, hipStream_t st);
hipError_t launch_axes_fold(int dtype, const AxesArgs &a, const FoldGrid &g, bool masked, int64_t grid,
                            hipStream_t st);
hipError_t launch_inflate(const InflateArgs &x, int64_t n, int wbits, hipStream_t st);
hipError_t launch_select(int dtype, const SelectArgs &a, int64_t grid, hipStream_t st);
hipError_t launch_tie_chunks(int dtype, const TieChunkArgs &a, int64_t grid, hipStream_t st);
hipError_t launch_tie_gate(int dtype, const pyas_partial *fin, int64_t n, uint32_t which, uint32_t *gate,
                           hipStream_t st);
hipError_t launch_tie_grid(int dtype, const TieGridArgs &a, hipStream_t st);
hipError_t launch_tie_pick(int dtype, const pyas_partial *parts, int64_t n, uint32_t which, int64_t base,
                           const TieCall &call, const TieRule &t, uint64_t *keys, hipStream_t st);
hipError_t launch_tie_finalize(int dtype, const uint64_t *keys, int64_t n_out, int32_t n_sets, const TieCall &call,
                               const TieRule &t, uint32_t which, pyas_partial *fin, hipStream_t st);
hipError_t launch_format(int dtype, const pyas_partial *in, int64_t n, int32_t method, void *values,
                         uint8_t *mask, int64_t *counts, hipStream_t st);
// host ingest (pyas_ingest.hip): pread ring -> pinned slots -> H2D
struct Ingest;
Ingest *ingest_create(int device);
void ingest_destroy(Ingest *g);
int ingest_configure(Ingest *g, int32_t n_slots, int64_t slot_bytes, std::string &msg);
// zlib_out > 0: every range is a zlib stream inflated on the reader thread
// into exactly zlib_out bytes of its staging slot (status[i] != 0 when it is
// not: a pyas_inflate_status, or PYAS_INFLATE_OVERFLOW for a short output).
int ingest_read(Ingest *g, int fd, int64_t n, const int64_t *file_offsets, const int64_t *sizes,
                uint8_t *dst, const int64_t *dst_offsets, int32_t threads, hipStream_t st,
                std::string &msg, int64_t zlib_out = 0, int32_t *status = nullptr);
// zlib.decompress of one stream (RFC 1950) into at most `cap` bytes of dst;
// a pyas_inflate_status, n_out = bytes written (pyas_ingest.hip).
int host_inflate(const uint8_t *src, int64_t n_src, uint8_t *dst, int64_t cap, int64_t &n_out);

// pyas_capi.hip: the thread-local pyas_last_error() message, and the device a
// context is bound to (for runtime pieces in other translation units)
int set_error(int code, const char *fmt, ...);
int ctx_device(const pyas_ctx *ctx);

hipError_t launch_unshuffle_chunks(const void *src, const int64_t *soff, void *dst, const int64_t *doff,
                                   int64_t n_chunks, int64_t nbytes, int64_t es, hipStream_t st);
hipError_t launch_unshuffle(const void *src, void *dst, int64_t nbytes, int64_t es,
                            hipStream_t st);

}  // namespace pyas
