/*
 * pyas.h — C ABI of the MI355X (gfx950) chunk-reduction backend.
 *
 * Drop-in boundary for PyActiveStorage's local chunk reducer.  Every entry
 * point below names the reference interface it replaces (paths relative to
 * the NCAS-CMS/PyActiveStorage repository):
 *
 *   reference                                       | replaced by
 *   ------------------------------------------------+---------------------------
 *   activestorage/storage.py:8-104  reduce_chunk    | pyas_reduce_chunks (batch,
 *     (one call per chunk, NumPy)                   |   method != None)
 *   activestorage/storage.py:95-96  chunk[sel] +    | pyas_select_chunks
 *     mask_missing  (method=None branch, :102-103)  |
 *   activestorage/storage.py:98-100 np.ma.count +   | pyas_reduce_axes (partial
 *     method(axis=..., keepdims=True), axis ⊂ dims  |   axis reductions)
 *   activestorage/storage.py:107-123 filter_pipeline| fused into the kernels
 *     + numcodecs.Shuffle.decode (hdf2numcodec:37)  |   (pyas_batch.shuffle) and
 *                                                   |   pyas_unshuffle
 *   activestorage/storage.py:119-120 compression.   | pyas_inflate (zlib streams,
 *     decode = numcodecs.Zlib (hdf2numcodec:34-35)  |   one wave per chunk)
 *   activestorage/storage.py:126-153 mask_missing   | pyas_mask (thresholds are
 *                                                   |   pre-compiled on the host)
 *   activestorage/storage.py:51-53,156-162 open +   | pyas_read_ranges (pread
 *     read_block, once per chunk                    |   ring -> pinned -> H2D)
 *   activestorage/active.py:557-598 thread-pool     | pyas_reduce_chunks with a
 *     fan-out + out[...] assembly + method(out)     |   `total` output, and
 *                                                   |   pyas_combine_partials
 *
 * Conventions
 *   - Plain C types only; every pointer documented as "device" must be a HIP
 *     device (or managed) pointer on the context's device.  `stream` is a
 *     hipStream_t passed as void* (NULL = the null stream).
 *   - Every function returns a pyas_status; on failure pyas_last_error()
 *     returns a thread-local message.  Launch functions do not synchronise
 *     and allocate nothing after the first call with a given geometry, so a
 *     caller may capture them into a hipGraph after one warm call.
 *   - Results are deterministic: no floating-point atomics anywhere; partials
 *     are combined in a fixed order.
 */
#ifndef PYAS_H
#define PYAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PYAS_ABI_VERSION 2
#define PYAS_MAX_DIMS 8

typedef enum {
    PYAS_OK = 0,
    PYAS_EINVAL = 1,      /* bad argument (reference: ValueError)            */
    PYAS_ENOTSUP = 2,     /* unsupported dtype/filter (NotImplementedError)  */
    PYAS_EDEVICE = 3,     /* HIP runtime / launch failure                    */
    PYAS_ENOMEM = 4,      /* device allocation failed                        */
    PYAS_EINDEX = 5,      /* selection out of the chunk (IndexError)         */
    PYAS_EIO = 6          /* file read failed or ended early (OSError)       */
} pyas_status;

/* netCDF-4 numeric types (the 10 the format defines) */
typedef enum {
    PYAS_I8 = 0, PYAS_U8 = 1, PYAS_I16 = 2, PYAS_U16 = 3, PYAS_I32 = 4,
    PYAS_U32 = 5, PYAS_I64 = 6, PYAS_U64 = 7, PYAS_F32 = 8, PYAS_F64 = 9
} pyas_dtype;

/* One 8-byte value in the data's class: f for floats, i for signed, u for
 * unsigned integers.  Float data values (f32 too) are carried exactly as f64. */
typedef union {
    double f;
    int64_t i;
    uint64_t u;
} pyas_scalar;

/* Partial result of a masked reduction over a set of elements (32 bytes).
 * sum  : floats accumulate in f64; signed ints in int64, unsigned in uint64,
 *        both wrapping modulo 2^64 exactly as NumPy's int64/uint64 sums do.
 * count: unmasked elements (np.ma.count, storage.py:98).
 * min/max: NaN-propagating like np.ma.min/max; meaningless when count == 0
 *        (the reference returns `masked` there, storage.py:99-100). */
typedef struct {
    pyas_scalar sum;
    int64_t count;
    pyas_scalar min;
    pyas_scalar max;
} pyas_partial;

/* Compiled form of mask_missing (storage.py:126-153).  All thresholds are
 * values OF THE DATA TYPE (already converted by the host so that the device
 * comparison in the data type is exactly NumPy's comparison in the promoted
 * type).  An element x is masked iff
 *     (eq_lo[0] <= x <= eq_hi[0]) || (eq_lo[1] <= x <= eq_hi[1])
 *  || x > gt || x < lt  || (vector tables, below).
 * Disabled rules use neutral values (empty interval lo > hi; gt = +inf or
 * type max; lt = -inf or type min) and their bit is clear in `flags`.
 * Vector _FillValue / missing_value (storage.py:133-143, broadcast equality)
 * use device tables of intervals indexed by sum_d idx_d * tab_stride[k][d],
 * idx_d = position inside the chunk's selection along chunk dim d. */
#define PYAS_MASK_EQ0 1u
#define PYAS_MASK_EQ1 2u
#define PYAS_MASK_GT 4u
#define PYAS_MASK_LT 8u
#define PYAS_MASK_TAB0 16u
#define PYAS_MASK_TAB1 32u

typedef struct {
    uint32_t flags;
    int32_t tab_len[2];
    pyas_scalar eq_lo[2];
    pyas_scalar eq_hi[2];
    pyas_scalar gt;
    pyas_scalar lt;
    const pyas_scalar *tab_lo[2];           /* device, tab_len[k] entries */
    const pyas_scalar *tab_hi[2];
    int64_t tab_stride[2][PYAS_MAX_DIMS];
} pyas_mask;

/* A batch of chunks of ONE variable resident in device memory.
 * Chunk c occupies bytes [offsets[c], offsets[c] + chunk_nbytes) of `data`
 * (uncompressed; byte-shuffled when `shuffle` > 1; big-endian when
 * `byteswap`).  offsets[c] must be a multiple of the element size.
 * Selection (storage.py:95 chunk[chunk_selection]) per chunk and chunk dim:
 *   sel[(c*PYAS_MAX_DIMS + d)*3 + {0,1,2}] = {start, step, count}
 *   step != 0 : indices start + k*step, k < count   (slices; step may be < 0)
 *   step == 0 : indices index_pool[start + k], k < count (integer lists)
 * sel == NULL selects every chunk completely. */
typedef struct {
    int32_t dtype;                     /* pyas_dtype */
    int32_t byteswap;                  /* 1: stored non-native (big-endian) */
    int32_t shuffle;                   /* HDF5 shuffle element size, 0/1 = off */
    int32_t ndim;                      /* chunk rank, 1..PYAS_MAX_DIMS */
    int64_t chunk_shape[PYAS_MAX_DIMS];
    int64_t n_chunks;
    const void *data;                  /* device */
    const int64_t *offsets;            /* device [n_chunks] */
    const int32_t *sel;                /* device [n_chunks*PYAS_MAX_DIMS*3] or NULL */
    const int32_t *index_pool;         /* device, used by step == 0 dims */
} pyas_batch;

/* combine flags */
#define PYAS_COMBINE_ROUND_TO_VAR 1u   /* round each input sum to the variable
                                          dtype first (Active stores partials in
                                          an `out` array of the var dtype,
                                          active.py:512,585) */

typedef struct pyas_ctx pyas_ctx;

/* ---- library / context -------------------------------------------------- */
int pyas_abi_version(void);
const char *pyas_last_error(void);
int pyas_device_count(int *count);
int pyas_ctx_create(int device, pyas_ctx **out);
int pyas_ctx_destroy(pyas_ctx *ctx);
/* Tile size (bytes of selected data per workgroup); 0 restores the default. */
int pyas_ctx_set_tile_bytes(pyas_ctx *ctx, int64_t tile_bytes);
/* LDS history ring of pyas_inflate, 2^wbits bytes per stream, wbits in
 * [13, 15] (default 13).  Smaller rings run more streams per CU; matches
 * reaching past the ring read the already-written output.  Results do not
 * depend on it. */
int pyas_ctx_set_inflate_window_bits(pyas_ctx *ctx, int32_t wbits);
/* on != 0 (default): pyas_reduce_chunks folds tiles -> chunks -> groups ->
 * total in one finishing launch (the last group to finish folds the total,
 * in group order); 0: the total is folded by a second launch.  Results are
 * bit-identical either way. */
int pyas_ctx_set_chained_combine(pyas_ctx *ctx, int32_t on);
/* pyas_reduce_axes_grid launches n_cols x (workgroups per column); it splits
 * the reduced rows further until the launch has >= n workgroups, and refuses
 * (PYAS_ENOTSUP, two-step path) below n / 4.  0 restores the default 2048. */
int pyas_ctx_set_fold_min_blocks(pyas_ctx *ctx, int64_t n);

/* ---- NumPy's sign of a zero min/max -------------------------------------
 * storage.py:99-100 returns np.ma.min/max(chunk[sel], axis, keepdims=True),
 * and active.py:594 reduces the `out` array of per-chunk results the same
 * way.  When an extreme is zero and +0.0 and -0.0 both occur, the zero NumPy
 * returns is decided by the order its reduction visits the elements
 * (pyactivestorage_amd/zerosign.py states the measured rules): the iterator
 * walks the reduced array in memory order; every run of the trailing
 * reduced dims is one call of the reduce loop, cut into pieces of
 * np.getbufsize() elements; a contiguous call keeps one accumulator per SIMD
 * lane seeded with the running result (later wins in a lane, lanes folded
 * in a fixed priority, then a scalar remainder); a strided call keeps `acc`
 * accumulators seeded with its first elements; an elementwise loop (kept
 * innermost dim) lets every later zero win.  The lane counts and priorities
 * depend on the SIMD target NumPy dispatches on the host, so the host derives
 * them from NumPy and sets them per float dtype:
 *   lanes 1..64, piece 1..2^24, rank[lane] = priority (0 wins every tie),
 *   acc 1..64 accumulators of the strided loop, acc_rank likewise. */
typedef struct {
    int32_t lanes;
    int32_t piece;
    int32_t acc;
    uint8_t rank[64];
    uint8_t acc_rank[64];
} pyas_tie_rule;
/* dtype PYAS_F32 or PYAS_F64; rule NULL clears it (no sign rewriting). */
int pyas_ctx_set_tie_rule(pyas_ctx *ctx, int32_t dtype, const pyas_tie_rule *rule);

/* How NumPy walks chunk[sel] (after mask_missing) for one query:
 * perm = chunk dims (the batch's dim order) from outer to inner in memory;
 * PYAS_TIE_VIEW: the array is the chunk[sel] view itself (no mask attribute
 * and slices only), so its strides are step * chunk stride; otherwise it is
 * a copy, contiguous in perm order; PYAS_TIE_BUFFERED: non-native byte
 * order (NumPy reduces through a contiguous buffer). */
#define PYAS_TIE_VIEW 1u
#define PYAS_TIE_BUFFERED 2u
typedef struct {
    int32_t perm[PYAS_MAX_DIMS];
    uint32_t flags;
} pyas_tie_geom;

/* Level 1, per chunk (storage.py:99-100): for every output of every chunk of
 * `batch` (the chunk's selection reduced over the dims in axes_mask; outputs
 * row-major over the kept selected dims, at partials[out_offsets[c] + o], or
 * partials[c] when out_offsets is NULL) whose partial has count > 0 and a
 * zero min (which bit 0) / max (bit 1): rewrite that zero's sign as NumPy's
 * (masked elements never tie).  Float dtypes only; a no-op without a rule. */
int pyas_tie_chunks(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                    const pyas_tie_geom *geom, uint32_t axes_mask, uint32_t which,
                    const int64_t *out_offsets, pyas_partial *partials, void *stream);
/* Level 1 of a FULL reduction (every dim reduced, one partial per chunk, the
 * chunks at positions layer_base + c of the `out` array's call of length lr,
 * active.py:594), done only where it can matter: which zero the level-2 keys
 * pick depends on positions alone, so a pick pass keys the zero partials
 * with sign 0, and only the chunk holding the K1 winner and the chunk
 * holding the W winner are scanned (pyas_tie_chunks' scan, one wave each).
 * pyas_tie_segments over the same partials then gives the same result as
 * after pyas_tie_chunks over every chunk (a group of ranks: each rank's keys
 * name its own two chunks, and the exchange picks among them).  Replaces
 * pyas_tie_chunks for storage.py:99-100 + active.py:594 full reductions. */
int pyas_tie_chunks_total(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                          const pyas_tie_geom *geom, uint32_t which, pyas_partial *partials,
                          int64_t layer_base, int64_t lr, void *stream);
/* Level 1 for a result folded without per-chunk partials
 * (pyas_reduce_axes_grid): when any of the n_final partials in `final_`
 * has a zero min/max (which: 1 or 2), write one byte per chunk output to
 * flags[out_offsets[c] + o] (bit 0: the output holds an unmasked zero, bit
 * 1: the sign NumPy's reduction of it returns); otherwise write nothing. */
int pyas_tie_chunk_flags(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                         const pyas_tie_geom *geom, uint32_t axes_mask, uint32_t which,
                         const int64_t *out_offsets, const pyas_partial *final_, int64_t n_final,
                         uint8_t *flags, void *stream);
/* ---- memory helpers (so a non-torch host can drive the ABI) ------------- */
int pyas_malloc(pyas_ctx *ctx, size_t nbytes, void **dptr);
int pyas_free(pyas_ctx *ctx, void *dptr);
/* Pinned (page-locked) host memory: H2D copies from it are DMA, without the
 * runtime's pageable staging.  The per-chunk drop-in reads each chunk
 * (storage.py:51-53 read_block) straight into a per-thread pinned buffer. */
int pyas_host_alloc(pyas_ctx *ctx, size_t nbytes, void **hptr);
int pyas_host_free(pyas_ctx *ctx, void *hptr);
int pyas_memcpy_h2d(pyas_ctx *ctx, void *dst, const void *src, size_t n, void *stream);
int pyas_memcpy_d2h(pyas_ctx *ctx, void *dst, const void *src, size_t n, void *stream);
int pyas_stream_create(pyas_ctx *ctx, void **stream);
int pyas_stream_destroy(pyas_ctx *ctx, void *stream);
int pyas_stream_synchronize(pyas_ctx *ctx, void *stream);
/* Work queued on `waiter` after this call starts only once everything queued
 * on `waitee` so far has finished (an event recorded on waitee, waited on by
 * waiter; no host synchronisation).  Lets ingest copies on one stream
 * overlap device inflate on another (Active's compressed-chunk pipeline). */
int pyas_stream_wait(pyas_ctx *ctx, void *waiter, void *waitee);

/* ---- hot path ------------------------------------------------------------ */
/* Fused un-shuffle -> byte-swap -> select -> mask -> sum/count/min/max for
 * every chunk of the batch.  chunk_out (device, n_chunks entries, may be
 * NULL) receives one partial per chunk (storage.py:98-100 with axis = all
 * dims); total (device, 1 entry, may be NULL) receives the combine of all
 * chunk partials under `combine_flags` (active.py:594-598). */
int pyas_reduce_chunks(pyas_ctx *ctx, const pyas_batch *batch,
                       const pyas_mask *mask, pyas_partial *chunk_out,
                       pyas_partial *total, uint32_t combine_flags,
                       void *stream);

/* Partial-axis reduction: for chunk c the selected block is reduced over the
 * chunk dims whose bit is set in axes_mask; outputs (row-major over the
 * remaining selected dims, keepdims) start at out[out_offsets[c]]. */
int pyas_reduce_axes(pyas_ctx *ctx, const pyas_batch *batch,
                     const pyas_mask *mask, uint32_t axes_mask,
                     const int64_t *out_offsets, pyas_partial *out,
                     void *stream);

/* Compact per-output records (pyas_reduce_axes_ex): what storage.py:98-100
 * returns per chunk for ONE method, with the sum rounded to the variable
 * dtype as Active stores it in its `out` array (active.py:512,585).  A
 * record is a value in the variable dtype -- the sum (PYAS_REC_SUM, for sum
 * and mean; an integer sum wraps to the variable dtype), the min
 * (PYAS_REC_MIN) or the max (PYAS_REC_MAX) -- and an int32 count:
 * PYAS_REC_BYTES(itemsize) bytes, 8 for 1/2/4-byte dtypes (value in the low
 * bytes of the first 4, count in the next 4), 16 for 8-byte dtypes (value,
 * count, 4 zero bytes).  An all-zero record is neutral (count 0).  The
 * combines read them with PYAS_COMBINE_REC(rec) in combine_flags, the
 * zero-sign passes with PYAS_TIE_REC in `which`; their results are
 * bit-identical to the 32-byte path with PYAS_COMBINE_ROUND_TO_VAR. */
#define PYAS_REC_FULL 0    /* the 32-byte pyas_partial */
#define PYAS_REC_SUM 1
#define PYAS_REC_MIN 2
#define PYAS_REC_MAX 3
#define PYAS_REC_BYTES(itemsize) ((itemsize) <= 4 ? 8 : 16)
#define PYAS_COMBINE_REC(rec) ((uint32_t)(rec) << 4)
#define PYAS_TIE_REC 4u    /* which: parts are PYAS_REC_MIN (which 1) / _MAX (which 2) records */
/* OR'ed into pyas_reduce_axes_ex's rec (PYAS_REC_MIN / PYAS_REC_MAX of a
 * float variable): the per-chunk walk writes NumPy's sign of a zero min/max
 * itself (storage.py:99-100), so pyas_tie_chunks need not run.  Column
 * layout (innermost chunk dim kept): the calls are elementwise and the last
 * zero wins.  LDS row layout (innermost dim reduced, rows <= 64 elements, the
 * reduced group that dim alone when chunks are cut): each row is one
 * contiguous call, keyed with the context's tie rule
 * (pyas_ctx_set_tie_rule).  The caller promises every chunk is whole or a unit-step box
 * covering at least half the chunk with more than one index in the
 * innermost dim; PYAS_ENOTSUP when the launch cannot key the sign (another
 * layout, no tie rule, cut chunks it would not take). */
#define PYAS_REC_ZERO_SIGN 0x100
/* OR'ed into pyas_reduce_axes_ex's rec: the caller promises what
 * PYAS_REC_ZERO_SIGN's caller promises (every chunk whole or a unit-step box
 * covering at least half the chunk with more than one index in the innermost
 * dim), so the generic per-element walk is not launched for the chunks the
 * dense launch leaves (there are none).  A broken promise leaves those
 * chunks' outputs unwritten. */
#define PYAS_REC_DENSE_ONLY 0x200
/* The opposite promise: no chunk is whole or such a box (e.g. a strided or
 * listed selection in every chunk), so the dense launch, which would find no
 * chunk of its own, is not made.  A broken promise leaves the whole and box
 * chunks' outputs unwritten. */
#define PYAS_REC_GENERIC_ONLY 0x400
/* pyas_reduce_axes writing `rec` records (PYAS_REC_*; PYAS_REC_FULL is
 * pyas_reduce_axes itself): out[out_offsets[c] + o] in record units.  A
 * chunk's outputs must count < 2^31 elements each. */
int pyas_reduce_axes_ex(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                        uint32_t axes_mask, int32_t rec, const int64_t *out_offsets, void *out,
                        void *stream);

/* method=None: decode + select + mask into dense row-major outputs.
 * values (device) receives native-endian elements, mask_out (device, may be
 * NULL) one byte per element (1 = masked); chunk c starts at element
 * out_offsets[c]. */
int pyas_select_chunks(pyas_ctx *ctx, const pyas_batch *batch,
                       const pyas_mask *mask, const int64_t *out_offsets,
                       void *values, uint8_t *mask_out, void *stream);

/* method=None for a whole orthogonal query (Active._select, active.py:
 * 483-485 -> storage.py:95-103 per chunk, then the reference places each
 * chunk's selection at its out_selection): element k = (k_0..k_{n-1}) of
 * chunk c's selection (C order over the selection counts) is written to
 * values/mask_out at  sum_d pos[chunk_base[c*ndim + d] + k_d] * out_stride[d]
 * (an element index of the caller's output array).  pos (int64) and
 * chunk_base (int32) are device arrays; dims dropped by an integer index use
 * out_stride 0. */
typedef struct {
    const int64_t *pos;
    const int32_t *chunk_base;
    int64_t out_stride[PYAS_MAX_DIMS];
} pyas_scatter;

int pyas_select_scatter(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                        const pyas_scatter *scatter, void *values, uint8_t *mask_out,
                        void *stream);

/* Fixed-order combine of n partials (device) into *out (device).  Used for
 * the per-chunk -> total step and for the cross-GPU combine of per-rank
 * partials after an RCCL all-gather. */
int pyas_combine_partials(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in,
                          int64_t n, uint32_t combine_flags, pyas_partial *out,
                          void *stream);

/* ---- several GPUs in one process (active.py:557-598 across devices) ------
 * Each of the ndev contexts (distinct devices) reduces its own batch of the
 * SAME variable on its own stream (pyas_reduce_chunks, combine_flags as
 * there); the per-device totals then travel in ONE RCCL all-gather over
 * xGMI (communicators over the listed devices, created with
 * ncclCommInitAll on first use of a device list and kept until
 * pyas_shard_release) and every device folds them in list order.
 * out[k] (device memory of ctx[k], ndev + 1 partials): out[k][0] receives
 * the global total, identical on every device; out[k][1 + j] the total of
 * device j.  mask may be NULL (unmasked) or hold one mask per device.
 * Asynchronous like every launch: synchronise streams[k] before reading.
 * Bounded wait: with the environment variable PYAS_SHARD_TIMEOUT_MS set to
 * a number >= 0 the call instead waits for the exchange up to that many
 * milliseconds (0: one poll), polling the streams and ncclCommGetAsyncError.
 * On an RCCL or stream error, or on expiry once every device has reached
 * its collectives (a stalled peer), it aborts the device list's
 * communicators (ncclCommAbort), drops them from the cache and returns
 * PYAS_EDEVICE naming the devices that had not finished; the streams and
 * out buffers of that call are then to be discarded.  On expiry while a
 * device is still reducing (its collectives queued, not started) it keeps
 * the communicators -- aborting would free them under queued RCCL kernels
 * -- and returns PYAS_EDEVICE naming the busy devices; the exchange then
 * completes on the streams.  Verified on hardware at ndev = 1.
 * Thread safety: calls on the same device list are serialised from group
 * start to group end (RCCL allows one group on a communicator at a time);
 * pyas_shard_release waits for a call still using a set.
 * Zero sign: this entry returns the combined partial as the devices reduce
 * it; pyas_reduce_sharded_tie below applies storage.py/active.py's
 * +0.0/-0.0 rule (as pyactivestorage_amd.distributed does).
 * RCCL is resolved from the process first (an RCCL already mapped, e.g.
 * torch's), then librccl.so.1.
 * The multi-process equivalent (one process per GPU) is
 * pyactivestorage_amd.distributed over torch.distributed. */
int pyas_reduce_sharded(pyas_ctx *const *ctx, const pyas_batch *const *per_dev,
                        const pyas_mask *const *mask, int32_t ndev, uint32_t combine_flags,
                        pyas_partial *const *out, void *const *streams);
/* pyas_reduce_sharded with NumPy's sign of a zero min (which = 1) or max
 * (which = 2) of a float variable (storage.py:99-100 per chunk, active.py:594
 * over the per-chunk results): device k's chunks are positions
 * [sum of earlier devices' n_chunks, + n_chunks) of the query's chunk order
 * (the `out` array); each device keeps its per-chunk partials (per-call
 * scratch), keys its two candidate chunks (pyas_tie_chunks_total) and its
 * total (pyas_tie_segments), the 16-byte keys travel in the same RCCL group
 * as the totals, and every device applies pyas_tie_finalize to out[k][0].
 * The tie rule of the dtype must be set on every ctx
 * (pyas_ctx_set_tie_rule); without one, and for integer dtypes or which = 0,
 * this is pyas_reduce_sharded.  `geom` as for pyas_tie_chunks. */
int pyas_reduce_sharded_tie(pyas_ctx *const *ctx, const pyas_batch *const *per_dev,
                            const pyas_mask *const *mask, int32_t ndev, uint32_t combine_flags,
                            const pyas_tie_geom *geom, uint32_t which,
                            pyas_partial *const *out, void *const *streams);
/* Destroy the cached RCCL communicators of pyas_reduce_sharded (waits for a
 * call still using them). */
int pyas_shard_release(void);

/* Segmented fixed-order combine: out[s] = fold of in[index[k]] for k in
 * [seg_offsets[s], seg_offsets[s+1]) in order (device arrays).  This is the
 * partial-axis form of the Active combine (active.py:575-598): `in` holds
 * per-chunk partial arrays, each segment lists the partials that fall on one
 * output element along the reduced axes. */
int pyas_combine_segments(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in,
                          const int64_t *index, const int64_t *seg_offsets,
                          int64_t n_segments, uint32_t combine_flags,
                          pyas_partial *out, void *stream);

/* Box-query form of the partial-axis combine (active.py:487-516,591-598:
 * each chunk's partial array is placed at its out_selection in `out`, then
 * method(out, axis) folds the chunk layers).  For an orthogonal selection the
 * chunks are the C-ordered product of per-dim chunk-coordinate lists, so the
 * segments of pyas_combine_segments follow from small per-dim tables and no
 * per-output index list is built on the host.  Output element f (C order
 * over out_extent) folds, in C order over the reduced dims' coordinates,
 * in[chunk_out_offsets[n] + j] where n is the chunk's position in the
 * product and j the element's index in that chunk's kept-dims partial array
 * (C order over the chunk's selected counts, reduced dims of extent 1). */
typedef struct {
    int32_t ndim;
    uint32_t axes_mask;                          /* reduced dims */
    int64_t n_coords[PYAS_MAX_DIMS];             /* chunk coordinates per dim */
    int64_t out_extent[PYAS_MAX_DIMS];           /* kept dims: final extent; reduced: 1 */
    const int32_t *pos_coord[PYAS_MAX_DIMS];     /* kept dims (device): position -> coordinate index */
    const int32_t *pos_local[PYAS_MAX_DIMS];     /* kept dims (device): position -> index in that chunk's selection */
    const int32_t *coord_count[PYAS_MAX_DIMS];   /* kept dims (device): coordinate index -> selected count */
    const int64_t *chunk_out_offsets;            /* device [prod n_coords] (pyas_reduce_axes's out_offsets) */
} pyas_grid;

int pyas_combine_grid(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in,
                      const pyas_grid *grid, uint32_t combine_flags, pyas_partial *out,
                      void *stream);

/* pyas_reduce_axes + pyas_combine_grid in ONE launch, for a box query whose
 * chunks are all whole (batch->sel == NULL) and laid out in the grid's C
 * order (chunk n = grid position n, prod n_coords chunks), each kept dim's
 * final extent being n_coords x the chunk extent.  The chunk layers along the
 * reduced dims are folded inside the reduction kernel, in the same order and
 * with the same rounding as pyas_combine_grid, so `out` (device, one partial
 * per final element) is bit-identical to the two-step result while the
 * per-chunk partial arrays are never written.  Only grid->ndim, axes_mask,
 * n_coords and out_extent are read.  Returns PYAS_ENOTSUP (nothing launched)
 * when the geometry does not admit it (element size < 4 bytes, shuffled
 * bytes, vector mask tables, or a reduced innermost dim): the caller then
 * takes the two-step path. */
int pyas_reduce_axes_grid(pyas_ctx *ctx, const pyas_batch *batch, const pyas_mask *mask,
                          const pyas_grid *grid, uint32_t combine_flags, pyas_partial *out,
                          void *stream);
/* combine_flags of pyas_reduce_axes_grid: NumPy's sign of a zero min (MIN)
 * or max (MAX), fused into the fold, so pyas_tie_chunk_flags and
 * pyas_tie_grid are not needed.  The caller checks that the chunks are
 * C-ordered (NumPy reduces chunk[sel] in memory order, storage.py:99-100);
 * the library derives both NumPy calls from the geometry:
 *  - lean column fold (innermost dim kept): valid where both reductions are
 *    elementwise (the chunks' innermost non-1 dim and the `out` array's,
 *    active.py:594, are kept) -- every later zero wins, and each lane tracks
 *    its outputs' last zero (layer order, then row order);
 *  - LDS row fold (modes 4-6, each output row one contiguous call): the
 *    context's tie rule (pyas_ctx_set_tie_rule) keys the zeros of a row
 *    whose min/max is a zero, and the row's sign is keyed at its layer's
 *    position in the `out` array's call (MIN or MAX, not both).
 * Float dtypes; PYAS_ENOTSUP (nothing launched) when the geometry takes
 * another fold kernel, a reduction the kernel cannot key, or no rule is set:
 * fold without the flag and run the zero-sign passes then.
 * pyas_combine_grid takes the same flags over records that already carry
 * level 1's signs (pyas_reduce_axes_ex with PYAS_REC_ZERO_SIGN) and keys
 * level 2 itself, so pyas_tie_grid is not needed: where the `out` array's
 * calls are elementwise (its innermost non-1 dim kept) each output takes the
 * sign of its last layer whose min (max) is a zero; where they run over the
 * trailing reduced dims (calls of lr layers), the context's tie rule keys the
 * zero layers at their positions in the call (pyas_tie_grid's keys). */
#define PYAS_FOLD_ZERO_SIGN_MIN 0x100u
#define PYAS_FOLD_ZERO_SIGN_MAX 0x200u

/* ---- NumPy's sign of a zero min/max, level 2 (see pyas_tie_chunks) ---- */
/* Level 2, across chunks (active.py:594): every final output f (partials
 * final_, device) whose min (which 1) / max (which 2) is a zero gets the sign
 * NumPy's reduction of the `out` array returns.  The chunk layers of f are
 * walked as pyas_combine_grid walks them; layer l's value comes from the
 * level-1 partials (`parts`, pyas_reduce_axes layout) or flag bytes
 * (`flags`).  lr: the length of one reduce call over `out` (the product of
 * its trailing reduced extents, 1 when its innermost non-1 dim is kept).
 * keys NULL: the sign is written to final_; else K1 keys are folded into
 * keys[f] (max) and W keys into keys[n_out + f] (min), for ranks of a group
 * to combine with pyas_tie_finalize (keys set up by pyas_tie_keys_reset). */
int pyas_tie_grid(pyas_ctx *ctx, int32_t dtype, const pyas_grid *grid, const pyas_partial *parts,
                  const uint8_t *flags, int64_t lr, uint32_t which, pyas_partial *final_,
                  uint64_t *keys, void *stream);
/* Level 2 over segments (pyas_combine_segments' layout: layer k of output s
 * is parts[index[seg[s] + k]]), or, with index == seg == NULL, one output
 * whose layers are parts[0 .. n_layers) (a full reduction; n_seg == 1).
 * Layer k sits at reduced position layer_base + k (a rank's first chunk). */
int pyas_tie_segments(pyas_ctx *ctx, int32_t dtype, const pyas_partial *parts, const int64_t *index,
                      const int64_t *seg, int64_t n_seg, int64_t n_layers, int64_t layer_base,
                      int64_t lr, uint32_t which, pyas_partial *final_, uint64_t *keys, void *stream);
/* keys (device, 2 * n_out): K1 = 0, W = all ones. */
int pyas_tie_keys_reset(pyas_ctx *ctx, uint64_t *keys, int64_t n_out, void *stream);
/* Combine n_sets key arrays (device, n_sets x [K1[n_out], W[n_out]]) and
 * write the signs into final_'s zero min/max. */
int pyas_tie_finalize(pyas_ctx *ctx, int32_t dtype, const uint64_t *keys, int64_t n_out, int32_t n_sets,
                      int64_t lr, uint32_t which, pyas_partial *final_, void *stream);

/* Result formatting on the device: the last step of Active._from_storage
 * (active.py:591-630) applied to n combined partials (device), so that only
 * the result's values and mask cross PCIe (9-16 bytes per output instead of
 * the 32-byte partial).  `values` (device) receives
 *   PYAS_FORMAT_SUM : the sum in the variable dtype for floats (the partial's
 *                     f64 rounded, as `out` of that dtype stores it), int64
 *                     for signed and uint64 for unsigned ints;
 *   PYAS_FORMAT_MIN / PYAS_FORMAT_MAX: the value in the variable dtype;
 *   PYAS_FORMAT_MEAN: float64, bit-identical to np.ma's `out / n`
 *                     (active.py:630): masked where n == 0, where the
 *                     quotient is not finite, or where np.ma's safe-divide
 *                     domain |out| * finfo(float).tiny >= |n| holds; a
 *                     masked element holds 0.0 + f64(out) as np.ma leaves it.
 * mask (device) receives one byte per element (1 = masked); counts (device,
 * may be NULL) the partials' counts as int64 (the `n` of components mode). */
enum { PYAS_FORMAT_SUM = 0, PYAS_FORMAT_MIN = 1, PYAS_FORMAT_MAX = 2, PYAS_FORMAT_MEAN = 3 };
int pyas_format_partials(pyas_ctx *ctx, int32_t dtype, const pyas_partial *in, int64_t n,
                         int32_t method, void *values, uint8_t *mask, int64_t *counts,
                         void *stream);

/* Standalone HDF5/numcodecs byte un-shuffle (storage.py:121-122), device to
 * device; n_bytes % elementsize trailing bytes are copied through. */
int pyas_unshuffle(pyas_ctx *ctx, const void *src, void *dst, int64_t n_bytes,
                   int32_t elementsize, void *stream);

/* Batched un-shuffle of n_chunks whole chunks of chunk_bytes each, device to
 * device: chunk i from src + src_offsets[i] to dst + dst_offsets[i] (both
 * offset arrays in device memory); elementsize 2, 4 or 8 (PYAS_ENOTSUP
 * otherwise); trailing chunk_bytes % elementsize bytes are copied through.
 * Resident variables keep their chunks un-shuffled this way, so later
 * queries take the dense kernels (storage.py:121-122 once per chunk). */
int pyas_unshuffle_chunks(pyas_ctx *ctx, const void *src, const int64_t *src_offsets, void *dst,
                          const int64_t *dst_offsets, int64_t n_chunks, int64_t chunk_bytes,
                          int32_t elementsize, void *stream);

/* ---- zlib inflate (row f3) ------------------------------------------------- */
/* Per-stream outcome of pyas_inflate, mirroring zlib inflate()'s failures
 * (zlib.error from zlib.decompress in the reference, storage.py:119-120). */
typedef enum {
    PYAS_INFLATE_OK = 0,
    PYAS_INFLATE_BAD_HEADER = 1,    /* "incorrect header check" / bad method  */
    PYAS_INFLATE_NEED_DICT = 2,     /* preset dictionary (FDICT)              */
    PYAS_INFLATE_BAD_BLOCK = 3,     /* "invalid block type"                   */
    PYAS_INFLATE_BAD_STORED = 4,    /* "invalid stored block lengths"         */
    PYAS_INFLATE_BAD_CODE = 5,      /* invalid code lengths / tree            */
    PYAS_INFLATE_BAD_SYMBOL = 6,    /* invalid literal/length/distance code   */
    PYAS_INFLATE_BAD_DISTANCE = 7,  /* "invalid distance too far back"        */
    PYAS_INFLATE_TRUNCATED = 8,     /* "incomplete or truncated stream"       */
    PYAS_INFLATE_BAD_CHECKSUM = 9,  /* "incorrect data check" (Adler-32)      */
    PYAS_INFLATE_OVERFLOW = 10      /* output larger than dst_capacity        */
} pyas_inflate_status;

/* Inflate n independent zlib (RFC 1950) streams, device to device
 * (replaces numcodecs.Zlib.decode -> zlib.decompress at storage.py:119-120;
 * built by hdf2numcodec.py:34-35).  Stream c is src[src_offsets[c] ..
 * + src_sizes[c]) and inflates into dst[dst_offsets[c] .. + dst_capacity[c]);
 * out_sizes[c] receives the inflated length and status[c] a
 * pyas_inflate_status.  All arrays are device arrays.  Bytes after the
 * Adler-32 trailer are ignored, as zlib.decompress does.  A dst offset that is
 * 16-byte aligned gets 1 KiB coalesced writes. */
int pyas_inflate(pyas_ctx *ctx, const uint8_t *src, const int64_t *src_offsets,
                 const int64_t *src_sizes, int64_t n, uint8_t *dst,
                 const int64_t *dst_offsets, const int64_t *dst_capacity,
                 int64_t *out_sizes, int32_t *status, void *stream);

/* ---- host ingest (row f2) ------------------------------------------------ */
/* Positioned reads of n byte ranges of an open file straight into device
 * memory.  Replaces the reference's per-chunk open + read_block
 * (storage.py:51-53, :156-162) run on active.py:557's 30-thread pool.
 * Range i is file[file_offsets[i] .. + sizes[i]) and lands at
 * dst + dst_offsets[i] (dst: device).  `threads` reader threads pread(2)
 * into a ring of pinned staging slots; each filled slot is copied H2D on
 * `stream` while the next slots are read.  Returns once every copy is
 * enqueued on `stream`: work queued after it on that stream sees the data.
 * A read error or end of file before a range ends -> PYAS_EIO.  The offset
 * and size arrays are host arrays. */
int pyas_read_ranges(pyas_ctx *ctx, int fd, int64_t n, const int64_t *file_offsets,
                     const int64_t *sizes, void *dst, const int64_t *dst_offsets,
                     int32_t threads, void *stream);
/* pyas_read_ranges for zlib-compressed chunks inflated on the HOST: each
 * range is one zlib stream (storage.py:119-120 through numcodecs.Zlib,
 * hdf2numcodec.py:34-35) that the reader thread preads and inflates
 * straight into its pinned staging slot; the inflated out_bytes are copied
 * H2D to dst + dst_offsets[i].  status (host, n entries) receives a
 * pyas_inflate_status per stream (PYAS_INFLATE_OVERFLOW also for an output
 * shorter or longer than out_bytes); a failed stream's bytes in dst are
 * undefined and the caller raises (re-running zlib gives zlib's message).
 * Few streams inflate faster here than with pyas_inflate, whose per-stream
 * rate is one serial DEFLATE decoder; Active picks the side per query. */
int pyas_read_ranges_zlib(pyas_ctx *ctx, int fd, int64_t n, const int64_t *file_offsets,
                          const int64_t *sizes, void *dst, const int64_t *dst_offsets,
                          int64_t out_bytes, int32_t *status, int32_t threads, void *stream);
/* Staging ring of pyas_read_ranges: n_slots x slot_bytes of pinned host
 * memory (default 16 x 64 MiB; each slot is pinned on first use). */
int pyas_ctx_set_ingest_slots(pyas_ctx *ctx, int32_t n_slots, int64_t slot_bytes);

/* ---- per-chunk drop-in, coalesced across threads ------------------------- */
/* The reference's Active._from_storage calls reduce_chunk once per chunk from
 * a 30-thread pool (active.py:556-589 -> :765-776 -> storage.py:8-104), each
 * call opening the file and reading its chunk (storage.py:51-53,156-162).
 * pyas_coalesced_reduce is that per-chunk call, thread-safe and blocking: the
 * calling thread preads its chunk into a pinned ring shared by all callers,
 * and a dispatcher thread reduces every chunk whose read has completed in one
 * H2D copy, one zlib-inflate launch and one reduce launch per (layout, mask,
 * axes) group, then wakes the callers.  Same per-chunk results as
 * pyas_reduce_chunks / pyas_reduce_axes on that chunk. */
typedef struct {
    int32_t dtype;                     /* pyas_dtype */
    int32_t byteswap;                  /* 1: stored non-native (big-endian) */
    int32_t shuffle;                   /* fused HDF5 shuffle (== itemsize) or 0 */
    int32_t ndim;
    int64_t chunk_shape[PYAS_MAX_DIMS];
    int32_t zlib;                      /* 1: the file bytes are one zlib stream
                                          (hdf2numcodec.py:34-35, storage.py:119-120) */
    uint32_t axes_mask;                /* chunk dims reduced (all dims: one partial) */
    uint32_t tie_which;                /* NumPy's zero sign for min (1) / max (2): pyas_tie_chunks */
    pyas_tie_geom tie;
} pyas_chunk_desc;

typedef struct pyas_coalescer pyas_coalescer;

/* ring_bytes: pinned host ring + device mirror (0 = 256 MiB); max_batch:
 * most chunks per dispatch (0 = 4096).  Starts the dispatcher thread. */
int pyas_coalescer_create(pyas_ctx *ctx, int64_t ring_bytes, int32_t max_batch,
                          pyas_coalescer **out);
int pyas_coalescer_destroy(pyas_coalescer *c);
/* stats (int64[8]): batches dispatched, chunks reduced, largest batch,
 * dispatcher busy ns (launching), callers' file-read ns, callers'
 * wait-for-batch ns, device-queue ns (per batch: from its launch, or the
 * previous batch's completion if later, to its completion), requests
 * handed back to the per-call path */
int pyas_coalescer_stats(pyas_coalescer *c, int64_t *stats);
/* Reduce file `path` bytes [offset, offset + size) as one chunk described by
 * desc/mask (mask without vector tables), selection `sel` (host
 * [PYAS_MAX_DIMS*3] as in pyas_batch, NULL = whole chunk) with `pool`
 * (host, pool_len entries) for listed dims.  `out` (host) receives n_out
 * partials (n_out must equal the kept selected extents' product, 1 when
 * every dim is reduced).  info (host int64[3]): bytes read (or -errno if the
 * open failed), inflate status, inflated size.  Returns PYAS_OK, or
 * PYAS_EIO for an open/read failure, short read or failed/mis-sized inflate,
 * PYAS_ENOTSUP for what the coalescer does not take (vector mask tables, a
 * chunk larger than the ring, uncompressed size != chunk bytes): the caller
 * then runs the per-call path, which raises the reference's exact error. */
int pyas_coalesced_reduce(pyas_coalescer *c, const char *path, int64_t offset, int64_t size,
                          const pyas_chunk_desc *desc, const pyas_mask *mask,
                          const int32_t *sel, const int32_t *pool, int32_t pool_len,
                          int64_t n_out, pyas_partial *out, int64_t *info);

/* ---- measurement ---------------------------------------------------------- */
/* When enabled, the main reduce kernel of each pyas_reduce_chunks call is
 * bracketed by HIP events on the launch stream (up to max_launches calls). */
int pyas_timing_enable(pyas_ctx *ctx, int32_t max_launches);
/* Synchronises the recorded events; writes up to cap durations (ms). */
int pyas_timing_read(pyas_ctx *ctx, float *ms, int32_t cap, int32_t *n);

#ifdef __cplusplus
}
#endif
#endif /* PYAS_H */
