// pyas_coalesce.hip — batching runtime behind the per-chunk drop-in.
//
// The reference calls reduce_chunk once per chunk from a 30-thread pool
// (activestorage/active.py:556-589 -> _process_chunk :765-776 ->
// storage.py:8-104), and every call opens the file and reads its chunk
// (storage.py:51-53, read_block :156-162).  Run one by one on the GPU, each
// such call pays its own H2D copy, launches, D2H copy and stream sync: the
// device would sit idle between tiny launches.
//
// Here concurrent calls are coalesced without changing the calling pattern:
//   caller thread  : open + pread(2) of its chunk straight into a pinned host
//                    ring (ctypes released the GIL), then sleep;
//   dispatcher     : take the longest prefix of the ring's unsubmitted
//                    requests whose reads are done, copy it H2D in one or two
//                    copies (a wrapped ring), inflate every zlib stream of the
//                    batch in one launch, reduce every chunk in one launch per
//                    (layout, mask, axes) group, copy every partial back in one
//                    copy, record the batch's event -- and go on to the next
//                    batch without waiting (up to `depth` batches in flight,
//                    each with its own scratch slot);
//   completer      : wait on the oldest batch's event, hand each caller its
//                    partials, wake exactly those callers, free their ring
//                    space.
// Batches grow with load (callers keep filling the ring while earlier
// batches run) and there are no timers.  Only the launches are serial: the
// device round trip of one batch overlaps the next batch's launch, and the
// batches in flight run side by side (one stream per slot; a zlib batch's
// inflate is one wave per chunk, latency-bound).  The chunk bytes go H2D on
// a copy stream; the batch meta and the partials stay in coherent host
// memory that the kernels read and write directly.  Anything the batch cannot express —
// vector mask tables, a chunk larger than the ring, a short read, a zlib
// failure — is handed back to the caller (PYAS_ENOTSUP / PYAS_EIO / info[])
// so that the per-call path raises the reference's exact exception.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdlib.h>
#include <fcntl.h>
#include <unistd.h>

#include <zlib.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pyas.h"
#include "pyas_internal.hpp"
#include "pyas_queue.hpp"

namespace {

constexpr int64_t kAlign = 256;
constexpr int64_t kDefaultRing = int64_t(256) << 20;

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int es_of(int dtype) {
    switch (dtype) {
        case PYAS_I8: case PYAS_U8: return 1;
        case PYAS_I16: case PYAS_U16: return 2;
        case PYAS_I32: case PYAS_U32: case PYAS_F32: return 4;
        case PYAS_I64: case PYAS_U64: case PYAS_F64: return 8;
        default: return 0;
    }
}

constexpr int SKIP = pyas::kSkip, SUBMITTED = pyas::kSubmitted;

// What one launch group shares; compared bytewise (zero-initialised).
struct Key {
    pyas_chunk_desc desc;
    pyas_mask mask;
};

// ring_off / span / state / cv: pyas::QItem (pyas_queue.hpp)
struct Req : pyas::QItem {
    Key key;
    int32_t sel[PYAS_MAX_DIMS * 3];
    bool has_sel = false;
    const int32_t *pool = nullptr;  // caller memory, valid while it waits
    int32_t pool_len = 0;
    int64_t nbytes = 0;
    int64_t n_out = 0;
    int64_t chunk_bytes = 0;        // decoded bytes
    pyas_partial *out = nullptr;    // caller memory
    int64_t *info = nullptr;
    int rc = PYAS_OK;
    std::string err;
};

struct Group {
    Key key;
    std::vector<Req *> reqs;
};

struct GMeta { int64_t off, sel_off, pool_off, n, pool_len, out_base, dec_base, inf_base; bool any_sel; };

template <typename T>
struct DevBuf {
    T *p = nullptr;
    int64_t n = 0;
    hipError_t ensure(int64_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        int64_t m = want < 1024 ? 1024 : want + want / 2;
        hipError_t e = hipMalloc((void **)&p, (size_t)m * sizeof(T));
        if (e == hipSuccess) n = m;
        return e;
    }
};

// Pinned host memory; `coherent` = uncached fine-grained memory the kernels
// read and write directly over PCIe (the zero-copy batch meta and partials).
template <typename T>
struct HostBuf {
    T *p = nullptr;
    int64_t n = 0;
    bool coherent = false;
    hipError_t ensure(int64_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        int64_t m = want < 1024 ? 1024 : want + want / 2;
        hipError_t e = hipHostMalloc((void **)&p, (size_t)m * sizeof(T),
                                     coherent ? hipHostMallocCoherent : hipHostMallocDefault);
        if (e == hipSuccess) n = m;
        return e;
    }
};

}  // namespace

namespace {
// Scratch of one in-flight batch (the dispatcher fills it, the completer
// drains it); reused once the batch has completed.
struct Slot {
    HostBuf<uint8_t> hmeta;
    DevBuf<uint8_t> dmeta;
    DevBuf<uint8_t> ddecode;
    DevBuf<pyas_partial> dout;
    HostBuf<pyas_partial> hout;
    HostBuf<int64_t> hinf;      // inflate out_sizes + status, copied back
    hipStream_t st = nullptr;   // this slot's kernels: batches in flight run side by side
    hipEvent_t ev = nullptr;
    hipEvent_t ev_copy = nullptr;   // the batch's H2D copies are done (copy stream)
    bool ev_ok = false;         // the event was recorded behind the batch
    std::vector<Req *> batch;
    std::vector<Group> groups;
    std::vector<GMeta> gm;
    int64_t n_inf = 0;
    int64_t inf_off = 0;        // inflate out_sizes + status: offset in the meta block
    int64_t t_launched = 0;     // launch_batch returned
};
}  // namespace

struct pyas_coalescer {
    pyas_ctx *ctx = nullptr;
    int device = 0;
    int64_t ring_bytes = 0;
    int32_t max_batch = 4096;
    uint8_t *hring = nullptr;   // pinned
    uint8_t *dring = nullptr;   // device mirror (same offsets)
    pyas::BatchQueue<Req, Slot> *q = nullptr;   // ring, FIFO and hand-offs; its mutex guards the stats
    std::thread disp, comp;
    hipStream_t cst = nullptr;   // H2D chunk copies (callers' in caller-copy mode; the
                                 // dispatcher's unless PYAS_COALESCE_COPYSTREAM=0)
    bool copy_stream = true;
    bool zero_copy = true;       // meta read / partials written in coherent host memory (PYAS_COALESCE_ZEROCOPY)
    // batches in flight (PYAS_COALESCE_DEPTH).  Measured on the box
    // (profiles/r02/dropin_*knobs.jsonl): uncompressed 21.5k chunks/s at 1
    // and 2, 21.4k at 4; zlib 1,063 chunks/s at 1, 760 at 4, 604 at 8 (more
    // batches in flight are smaller, and each zlib batch is bounded by one
    // stream's inflate latency), so one batch runs while the next gathers.
    int32_t depth = 1;
    // Where a zlib chunk is inflated (PYAS_COALESCE_INFLATE=host|device).
    // The device inflates one stream per wave at ~55 MB/s, so a batch of the
    // pool's <= 30 streams takes ~20 ms; a caller thread inflates its own
    // stream with zlib at several hundred MB/s, and the 30 callers do so in
    // parallel.  The device wins only with thousands of streams in flight
    // (Active's batched path, pyas_inflate), which the per-chunk pattern never
    // has: the callers inflate, the device reduces.
    bool host_inflate = true;
    std::vector<Slot *> slots;
    // Measured on the box (tools/bench_dropin.py): with 30 reader threads on a
    // 16-CPU host share, the dispatcher copying the batch's prefix and
    // sleeping on its completion event leaves the most CPU to the readers.
    bool caller_copy = false;   // PYAS_COALESCE_COPY=caller: each caller copies its own chunk
    bool blocking_sync = true;  // PYAS_COALESCE_SYNC=spin: the dispatcher spins on the batch
    int64_t n_batches = 0, n_chunks = 0, max_seen = 0;
    int64_t busy_ns = 0, read_ns = 0, wait_ns = 0;   // dispatcher launching; callers reading; callers waiting
    int64_t gpu_ns = 0, t_last_done = 0;   // completion-to-completion time of back-to-back batches
    int64_t n_back = 0;          // requests handed back to the per-call path (rc != OK)
};

namespace {

// Host bounds check of one selection row (the device trusts it).
bool sel_ok(const pyas_chunk_desc &d, const int32_t *sel, const int32_t *pool, int32_t pool_len,
            int64_t &n_sel_out, uint32_t axes) {
    int64_t n_out = 1;
    for (int k = 0; k < PYAS_MAX_DIMS; ++k) {
        const int64_t ext = k < d.ndim ? d.chunk_shape[k] : 1;
        const int64_t start = sel ? sel[k * 3 + 0] : 0;
        const int64_t step = sel ? sel[k * 3 + 1] : 1;
        const int64_t cnt = sel ? sel[k * 3 + 2] : ext;
        if (cnt < 0) return false;
        if (cnt > 0) {
            if (step != 0) {
                const int64_t last = start + (cnt - 1) * step;
                if (start < 0 || start >= ext || last < 0 || last >= ext) return false;
            } else {
                if (!pool || start < 0 || start + cnt > pool_len) return false;
                for (int64_t i = 0; i < cnt; ++i)
                    if (pool[start + i] < 0 || pool[start + i] >= ext) return false;
            }
        }
        if (k < d.ndim && !((axes >> k) & 1u)) n_out *= cnt;
    }
    n_sel_out = n_out;
    return true;
}

// Enqueue one batch on its slot's stream (no lock held) and record its event; requests
// that cannot run get their rc here.  The completer finishes the batch.
void launch_batch(pyas_coalescer *c, Slot *sl) {
    std::vector<Req *> &batch = sl->batch;
    std::vector<Group> &groups = sl->groups;
    groups.clear();
    sl->ev_ok = false;
    sl->n_inf = 0;
    // groups of identical keys, in first-seen order
    for (Req *r : batch) {
        if (r->state == SKIP) continue;
        Group *g = nullptr;
        for (auto &x : groups)
            if (std::memcmp(&x.key, &r->key, sizeof(Key)) == 0) { g = &x; break; }
        if (!g) {
            groups.push_back(Group{r->key, {}});
            g = &groups.back();
        }
        g->reqs.push_back(r);
    }
    auto fail_all = [&](int rc, const std::string &msg) {
        for (Req *r : batch)
            if (r->state != SKIP) { r->rc = rc; r->err = msg; }
    };
    if (groups.empty()) return;
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) { fail_all(PYAS_EDEVICE, hipGetErrorString(e)); return; }

    // host meta block: per group [offsets n][out_offsets n][src_off n][src_size n]
    // [dst_off n][dst_cap n] (int64) [sel n*24][pool] (int32); partial bases
    int64_t meta_bytes = 0, total_out = 0, decode_bytes = 0, n_inf = 0;
    std::vector<GMeta> &gm = sl->gm;
    gm.assign(groups.size(), GMeta{});
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        Group &g = groups[gi];
        GMeta &m = gm[gi];
        m.n = (int64_t)g.reqs.size();
        m.off = meta_bytes;
        meta_bytes += 6 * m.n * 8;
        m.any_sel = false;
        m.pool_len = 0;
        for (Req *r : g.reqs) { m.any_sel |= r->has_sel; m.pool_len += r->pool_len; }
        m.sel_off = meta_bytes;
        if (m.any_sel) meta_bytes += m.n * PYAS_MAX_DIMS * 3 * 4;
        m.pool_off = meta_bytes;
        meta_bytes = align_up(meta_bytes + (m.pool_len > 0 ? m.pool_len : 1) * 4, 16);
        m.out_base = total_out;
        for (Req *r : g.reqs) total_out += r->n_out;
        m.dec_base = decode_bytes;
        m.inf_base = n_inf;
        if (g.key.desc.zlib) {
            for (Req *r : g.reqs) decode_bytes += align_up(r->chunk_bytes, kAlign);
            n_inf += m.n;
        }
    }
    sl->n_inf = n_inf;
    if ((e = sl->hmeta.ensure(meta_bytes)) != hipSuccess || (e = sl->dmeta.ensure(meta_bytes)) != hipSuccess ||
        (e = sl->dout.ensure(total_out > 0 ? total_out : 1)) != hipSuccess ||
        (e = sl->hout.ensure(total_out > 0 ? total_out : 1)) != hipSuccess ||
        (e = sl->hinf.ensure(2 * (n_inf > 0 ? n_inf : 1))) != hipSuccess ||
        (decode_bytes > 0 && (e = sl->ddecode.ensure(decode_bytes)) != hipSuccess)) {
        fail_all(e == hipErrorOutOfMemory ? PYAS_ENOMEM : PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    // inflate out_sizes + status: a device-only region after the meta block
    const int64_t inf_dev_off = align_up(meta_bytes, 16);
    sl->inf_off = inf_dev_off;
    if (n_inf > 0 && (e = sl->dmeta.ensure(inf_dev_off + 2 * n_inf * 8)) != hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    if (n_inf > 0 && c->zero_copy && (e = sl->hmeta.ensure(inf_dev_off + 2 * n_inf * 8)) != hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    uint8_t *hm = sl->hmeta.p;
    uint8_t *dm = c->zero_copy ? sl->hmeta.p : sl->dmeta.p;   // the kernels read the meta from here
    pyas_partial *dout = c->zero_copy ? sl->hout.p : sl->dout.p;
    int64_t dec_cursor = 0;
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        Group &g = groups[gi];
        GMeta &m = gm[gi];
        int64_t *offs = (int64_t *)(hm + m.off);
        int64_t *oofs = offs + m.n;
        int64_t *soff = oofs + m.n, *ssz = soff + m.n, *doff = ssz + m.n, *dcap = doff + m.n;
        int32_t *sel = (int32_t *)(hm + m.sel_off);
        int32_t *pool = (int32_t *)(hm + m.pool_off);
        int64_t ob = m.out_base, pp = 0;
        for (int64_t i = 0; i < m.n; ++i) {
            Req *r = g.reqs[i];
            if (g.key.desc.zlib) {
                soff[i] = r->ring_off;
                ssz[i] = r->nbytes;
                doff[i] = dec_cursor;
                dcap[i] = r->chunk_bytes;
                offs[i] = dec_cursor;
                dec_cursor += align_up(r->chunk_bytes, kAlign);
            } else {
                offs[i] = r->ring_off;
                soff[i] = ssz[i] = doff[i] = dcap[i] = 0;
            }
            oofs[i] = ob;
            ob += r->n_out;
            if (m.any_sel) {
                int32_t *row = sel + i * PYAS_MAX_DIMS * 3;
                if (r->has_sel) {
                    std::memcpy(row, r->sel, sizeof(r->sel));
                    for (int k = 0; k < PYAS_MAX_DIMS; ++k)
                        if (row[k * 3 + 1] == 0) row[k * 3 + 0] += (int32_t)pp;   // pool offset
                    if (r->pool_len > 0) std::memcpy(pool + pp, r->pool, (size_t)r->pool_len * 4);
                    pp += r->pool_len;
                } else {
                    for (int k = 0; k < PYAS_MAX_DIMS; ++k) {
                        row[k * 3 + 0] = 0;
                        row[k * 3 + 1] = 1;
                        row[k * 3 + 2] = k < g.key.desc.ndim ? (int32_t)g.key.desc.chunk_shape[k] : 1;
                    }
                }
            }
        }
        if (m.pool_len == 0) pool[0] = 0;
    }
    // 1. the chunk bytes: copy the prefix here, one copy per contiguous run
    //    (two when the ring wrapped; gaps are alignment padding or skipped
    //    reads of the same prefix) -- or, with PYAS_COALESCE_COPY=caller,
    //    each caller already enqueued its own H2D copy on sl->st right after
    //    its read, before it marked the request FILLED, so the launches
    //    below are ordered after them
    hipStream_t cs = c->copy_stream ? c->cst : sl->st;   // where the chunk bytes are copied
    if (!c->caller_copy) {
        int64_t run_a = -1, run_b = -1;
        for (Req *r : batch) {
            if (r->state == SKIP) continue;
            if (run_a >= 0 && r->ring_off >= run_b) {
                run_b = r->ring_off + r->nbytes;
                continue;
            }
            if (run_a >= 0 &&
                (e = hipMemcpyAsync(c->dring + run_a, c->hring + run_a, (size_t)(run_b - run_a),
                                    hipMemcpyHostToDevice, cs)) != hipSuccess) {
                fail_all(PYAS_EDEVICE, hipGetErrorString(e));
                return;
            }
            run_a = r->ring_off;
            run_b = r->ring_off + r->nbytes;
        }
        if (run_a >= 0 &&
            (e = hipMemcpyAsync(c->dring + run_a, c->hring + run_a, (size_t)(run_b - run_a),
                                hipMemcpyHostToDevice, cs)) != hipSuccess) {
            fail_all(PYAS_EDEVICE, hipGetErrorString(e));
            return;
        }
    }
    // the kernels wait for the copy stream's copies (the callers' too, in
    // caller-copy mode: they were enqueued before the requests were FILLED)
    if ((c->copy_stream || c->caller_copy) &&
        ((e = hipEventRecord(sl->ev_copy, c->cst)) != hipSuccess ||
         (e = hipStreamWaitEvent(sl->st, sl->ev_copy, 0)) != hipSuccess)) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    // 2. meta H2D (zero-copy: the kernels read it from coherent host memory)
    if (!c->zero_copy &&
        (e = hipMemcpyAsync(dm, hm, (size_t)meta_bytes, hipMemcpyHostToDevice, sl->st)) != hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    int64_t *dinf = (int64_t *)(dm + inf_dev_off);   // [out_sizes n_inf][status n_inf (int32 in 8 B slots)]
    // 3. per group: inflate, reduce
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        Group &g = groups[gi];
        GMeta &m = gm[gi];
        const int64_t *d_offs = (const int64_t *)(dm + m.off);
        const int64_t *d_oofs = d_offs + m.n;
        const int64_t *d_soff = d_oofs + m.n, *d_ssz = d_soff + m.n, *d_doff = d_ssz + m.n,
                      *d_dcap = d_doff + m.n;
        int rc = PYAS_OK;
        if (g.key.desc.zlib) {
            rc = pyas_inflate(c->ctx, c->dring, d_soff, d_ssz, m.n, sl->ddecode.p, d_doff, d_dcap,
                              dinf + m.inf_base, (int32_t *)(dinf + n_inf) + m.inf_base, sl->st);
        }
        pyas_batch b;
        std::memset(&b, 0, sizeof(b));
        b.dtype = g.key.desc.dtype;
        b.byteswap = g.key.desc.byteswap;
        b.shuffle = g.key.desc.shuffle;
        b.ndim = g.key.desc.ndim;
        for (int k = 0; k < PYAS_MAX_DIMS; ++k) b.chunk_shape[k] = g.key.desc.chunk_shape[k];
        b.n_chunks = m.n;
        b.data = g.key.desc.zlib ? (const void *)sl->ddecode.p : (const void *)c->dring;
        b.offsets = d_offs;
        b.sel = m.any_sel ? (const int32_t *)(dm + m.sel_off) : nullptr;
        b.index_pool = (const int32_t *)(dm + m.pool_off);
        const uint32_t full = (g.key.desc.ndim >= 32) ? 0xffffffffu : ((1u << g.key.desc.ndim) - 1u);
        if (rc == PYAS_OK) {
            // NumPy's sign of a zero min/max, for min/max call shapes only
            const uint32_t tw = g.key.desc.tie_which;
            if ((g.key.desc.axes_mask & full) == full) {
                rc = pyas_reduce_chunks(c->ctx, &b, &g.key.mask, dout + m.out_base, nullptr, 0u, sl->st);
                if (rc == PYAS_OK && tw)
                    rc = pyas_tie_chunks(c->ctx, &b, &g.key.mask, &g.key.desc.tie, full, tw, nullptr,
                                         dout + m.out_base, sl->st);
            } else {
                rc = pyas_reduce_axes(c->ctx, &b, &g.key.mask, g.key.desc.axes_mask, d_oofs, dout, sl->st);
                if (rc == PYAS_OK && tw)
                    rc = pyas_tie_chunks(c->ctx, &b, &g.key.mask, &g.key.desc.tie, g.key.desc.axes_mask, tw,
                                         d_oofs, dout, sl->st);
            }
        }
        if (rc != PYAS_OK) {
            const std::string msg = pyas_last_error();
            for (Req *r : g.reqs) { r->rc = rc; r->err = msg; }
        }
    }
    // 4. partials (and inflate results) back; the completer waits on the event
    if (!c->zero_copy && total_out > 0 &&
        (e = hipMemcpyAsync(sl->hout.p, sl->dout.p, (size_t)total_out * sizeof(pyas_partial),
                            hipMemcpyDeviceToHost, sl->st)) != hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    if (!c->zero_copy && n_inf > 0 &&
        (e = hipMemcpyAsync(sl->hinf.p, dinf, (size_t)(2 * n_inf) * 8, hipMemcpyDeviceToHost, sl->st)) !=
            hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    if ((e = hipEventRecord(sl->ev, sl->st)) != hipSuccess) {
        fail_all(PYAS_EDEVICE, hipGetErrorString(e));
        return;
    }
    sl->ev_ok = true;
}

// After the batch's event (no lock held): the partials and inflate results
// to each caller's memory.
void finish_batch(pyas_coalescer *c, Slot *sl) {
    std::vector<Req *> &batch = sl->batch;
    if (sl->ev_ok) {
        const hipError_t e = hipEventSynchronize(sl->ev);
        if (e != hipSuccess) {
            for (Req *r : batch)
                if (r->state != SKIP) { r->rc = PYAS_EDEVICE; r->err = hipGetErrorString(e); }
            return;
        }
    } else {
        // launch_batch failed part-way (every live request carries its rc):
        // drain what it did enqueue before the slot is reused
        (void)hipStreamSynchronize(sl->st);
        return;
    }
    const int64_t n_inf = sl->n_inf;
    // inflate out_sizes + status: copied back, or written in place (zero-copy)
    const int64_t *inf = sl->hinf.p;
    if (c->zero_copy && n_inf > 0) inf = (const int64_t *)(sl->hmeta.p + sl->inf_off);
    for (size_t gi = 0; gi < sl->groups.size(); ++gi) {
        Group &g = sl->groups[gi];
        GMeta &m = sl->gm[gi];
        int64_t ob = m.out_base;
        for (int64_t i = 0; i < m.n; ++i) {
            Req *r = g.reqs[i];
            if (g.key.desc.zlib) {
                const int64_t osz = inf[m.inf_base + i];
                const int32_t stt = ((const int32_t *)(inf + n_inf))[m.inf_base + i];
                r->info[1] = stt;
                r->info[2] = osz;
                if (r->rc == PYAS_OK && (stt != PYAS_INFLATE_OK || osz != r->chunk_bytes)) {
                    r->rc = PYAS_EIO;   // the caller re-runs the per-call path for zlib's exact error
                    r->err = "inflate failed or size mismatch";
                }
            }
            if (r->rc == PYAS_OK)
                std::memcpy(r->out, sl->hout.p + ob, (size_t)r->n_out * sizeof(pyas_partial));   // both modes
            ob += r->n_out;
        }
    }
}

void dispatcher(pyas_coalescer *c) {
    (void)hipSetDevice(c->device);
    Slot *sl = nullptr;
    while (c->q->next_batch(sl)) {
        const int64_t t0 = now_ns();
        launch_batch(c, sl);
        const int64_t t1 = now_ns();
        sl->t_launched = t1;
        c->q->launched(sl, [&] { c->busy_ns += t1 - t0; });
    }
    c->q->dispatcher_done();
}

void completer(pyas_coalescer *c) {
    (void)hipSetDevice(c->device);
    Slot *sl = nullptr;
    while (c->q->next_done(sl)) {
        finish_batch(c, sl);
        const int64_t t_done = now_ns();
        c->q->complete(sl, [&] {
            // time this batch held the device queue: from its launch (or the
            // previous batch's completion, if later) to its completion
            c->gpu_ns += t_done - (sl->t_launched > c->t_last_done ? sl->t_launched : c->t_last_done);
            c->t_last_done = t_done;
            int64_t nch = 0;
            for (Req *r : sl->batch) {
                if (r->state == SUBMITTED) ++nch;
                if (r->rc != PYAS_OK) ++c->n_back;
            }
            c->n_batches += 1;
            c->n_chunks += nch;
            if (nch > c->max_seen) c->max_seen = nch;
        });
    }
}

}  // namespace

extern "C" {

int pyas_coalescer_create(pyas_ctx *ctx, int64_t ring_bytes, int32_t max_batch, pyas_coalescer **out) {
    if (!ctx || !out) return pyas::set_error(PYAS_EINVAL, "NULL argument");
    if (ring_bytes < 0 || max_batch < 0) return pyas::set_error(PYAS_EINVAL, "negative ring size or batch");
    pyas_coalescer *c = new pyas_coalescer();
    c->ctx = ctx;
    c->device = pyas::ctx_device(ctx);
    c->ring_bytes = align_up(ring_bytes > 0 ? ring_bytes : kDefaultRing, kAlign);
    c->max_batch = max_batch > 0 ? max_batch : 4096;
    c->q = new pyas::BatchQueue<Req, Slot>(c->ring_bytes, c->max_batch);
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->hring, (size_t)c->ring_bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void **)&c->dring, (size_t)c->ring_bytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking);
    if (const char *v = getenv("PYAS_COALESCE_COPY")) c->caller_copy = std::strcmp(v, "caller") == 0;
    if (const char *v = getenv("PYAS_COALESCE_SYNC")) c->blocking_sync = std::strcmp(v, "spin") != 0;
    if (const char *v = getenv("PYAS_COALESCE_DEPTH")) c->depth = atoi(v) > 0 ? atoi(v) : 1;
    if (const char *v = getenv("PYAS_COALESCE_ZEROCOPY")) c->zero_copy = std::strcmp(v, "0") != 0;
    if (const char *v = getenv("PYAS_COALESCE_INFLATE")) c->host_inflate = std::strcmp(v, "device") != 0;
    if (const char *v = getenv("PYAS_COALESCE_COPYSTREAM")) c->copy_stream = std::strcmp(v, "0") != 0;
    for (int i = 0; e == hipSuccess && i < c->depth; ++i) {
        Slot *sl = new Slot();
        sl->hmeta.coherent = sl->hout.coherent = c->zero_copy;
        e = hipEventCreateWithFlags(&sl->ev, hipEventDisableTiming |
                                                 (c->blocking_sync ? hipEventBlockingSync : 0u));
        if (e == hipSuccess) e = hipEventCreateWithFlags(&sl->ev_copy, hipEventDisableTiming);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&sl->st, hipStreamNonBlocking);
        c->slots.push_back(sl);
        c->q->add_slot(sl);
    }
    if (e != hipSuccess) {
        for (Slot *sl : c->slots) {
            if (sl->ev) (void)hipEventDestroy(sl->ev);
            if (sl->ev_copy) (void)hipEventDestroy(sl->ev_copy);
            if (sl->st) (void)hipStreamDestroy(sl->st);
            delete sl;
        }
        if (c->cst) (void)hipStreamDestroy(c->cst);
        if (c->hring) (void)hipHostFree(c->hring);
        if (c->dring) (void)hipFree(c->dring);
        delete c->q;
        delete c;
        return pyas::set_error(e == hipErrorOutOfMemory ? PYAS_ENOMEM : PYAS_EDEVICE, hipGetErrorString(e));
    }
    c->disp = std::thread(dispatcher, c);
    c->comp = std::thread(completer, c);
    *out = c;
    return PYAS_OK;
}

int pyas_coalescer_destroy(pyas_coalescer *c) {
    if (!c) return PYAS_OK;
    c->q->stop();
    if (c->disp.joinable()) c->disp.join();
    if (c->comp.joinable()) c->comp.join();
    (void)hipSetDevice(c->device);
    if (c->cst) (void)hipStreamSynchronize(c->cst);
    if (c->cst) (void)hipStreamDestroy(c->cst);
    for (Slot *sl : c->slots) {
        if (sl->st) (void)hipStreamSynchronize(sl->st);
        if (sl->st) (void)hipStreamDestroy(sl->st);
        if (sl->ev) (void)hipEventDestroy(sl->ev);
        if (sl->ev_copy) (void)hipEventDestroy(sl->ev_copy);
        if (sl->hmeta.p) (void)hipHostFree(sl->hmeta.p);
        if (sl->hout.p) (void)hipHostFree(sl->hout.p);
        if (sl->hinf.p) (void)hipHostFree(sl->hinf.p);
        if (sl->dmeta.p) (void)hipFree(sl->dmeta.p);
        if (sl->ddecode.p) (void)hipFree(sl->ddecode.p);
        if (sl->dout.p) (void)hipFree(sl->dout.p);
        delete sl;
    }
    (void)hipHostFree(c->hring);
    (void)hipFree(c->dring);
    delete c->q;
    delete c;
    return PYAS_OK;
}

int pyas_coalescer_stats(pyas_coalescer *c, int64_t *stats) {
    if (!c || !stats) return pyas::set_error(PYAS_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->q->mu);
    stats[0] = c->n_batches;
    stats[1] = c->n_chunks;
    stats[2] = c->max_seen;
    stats[3] = c->busy_ns;
    stats[4] = c->read_ns;
    stats[5] = c->wait_ns;
    stats[6] = c->gpu_ns;
    stats[7] = c->n_back;
    return PYAS_OK;
}

int pyas_coalesced_reduce(pyas_coalescer *c, const char *path, int64_t offset, int64_t size,
                          const pyas_chunk_desc *desc, const pyas_mask *mask, const int32_t *sel,
                          const int32_t *pool, int32_t pool_len, int64_t n_out, pyas_partial *out,
                          int64_t *info) {
    if (!c || !path || !desc || !mask || !out || !info) return pyas::set_error(PYAS_EINVAL, "NULL argument");
    info[0] = info[1] = info[2] = 0;
    const int es = es_of(desc->dtype);
    if (es == 0) return pyas::set_error(PYAS_ENOTSUP, "unsupported dtype code %d", desc->dtype);
    if (desc->ndim < 1 || desc->ndim > PYAS_MAX_DIMS) return pyas::set_error(PYAS_EINVAL, "bad chunk rank");
    if (mask->flags & (PYAS_MASK_TAB0 | PYAS_MASK_TAB1))
        return pyas::set_error(PYAS_ENOTSUP, "vector mask tables are not coalesced");
    if (desc->axes_mask >> desc->ndim) return pyas::set_error(PYAS_EINVAL, "axes beyond the chunk rank");
    if (offset < 0 || size < 0) return pyas::set_error(PYAS_EINVAL, "negative offset/size");
    Req r;
    std::memset(&r.key, 0, sizeof(r.key));
    std::memcpy(&r.key.desc, desc, sizeof(*desc));
    std::memcpy(&r.key.mask, mask, sizeof(*mask));
    int64_t elems = 1;
    for (int k = 0; k < desc->ndim; ++k) {
        if (desc->chunk_shape[k] <= 0) return pyas::set_error(PYAS_EINVAL, "bad chunk shape");
        elems *= desc->chunk_shape[k];
    }
    for (int k = desc->ndim; k < PYAS_MAX_DIMS; ++k) r.key.desc.chunk_shape[k] = 0;
    r.chunk_bytes = elems * es;
    if (!desc->zlib && size != r.chunk_bytes)
        return pyas::set_error(PYAS_ENOTSUP, "size %lld is not the chunk's %lld bytes", (long long)size,
                               (long long)r.chunk_bytes);
    int64_t n_sel_out = 0;
    if (!sel_ok(*desc, sel, pool, pool_len, n_sel_out, desc->axes_mask))
        return pyas::set_error(PYAS_EINDEX, "selection reaches outside the chunk");
    if (n_sel_out != n_out) return pyas::set_error(PYAS_EINVAL, "n_out %lld != selection's %lld",
                                                   (long long)n_out, (long long)n_sel_out);
    if (sel) {
        r.has_sel = true;
        std::memcpy(r.sel, sel, sizeof(r.sel));
    }
    r.pool = pool;
    r.pool_len = sel ? pool_len : 0;
    r.n_out = n_out;
    r.out = out;
    r.info = info;
    r.nbytes = size;
    // a zlib chunk inflated by this thread lands decoded in the ring and joins
    // the uncompressed requests of its layout
    const bool inflate_here = desc->zlib && c->host_inflate;
    if (inflate_here) {
        r.key.desc.zlib = 0;
        r.nbytes = r.chunk_bytes;
    }
    r.span = align_up(r.nbytes > 0 ? r.nbytes : 1, kAlign);
    if (r.span > c->ring_bytes) return pyas::set_error(PYAS_ENOTSUP, "chunk larger than the coalescing ring");

    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
        info[0] = -errno;
        return pyas::set_error(PYAS_EIO, "open failed: %s", strerror(errno));
    }
    if (!c->q->reserve(&r)) {
        close(fd);
        return pyas::set_error(PYAS_EDEVICE, "coalescer stopped");
    }
    const int64_t off = r.ring_off;

    const int64_t t_read = now_ns();
    int64_t got = 0;
    int read_errno = 0;
    thread_local std::vector<uint8_t> zbuf;   // this caller's compressed bytes
    if (inflate_here && (int64_t)zbuf.size() < size) zbuf.resize((size_t)size);
    uint8_t *const dst = inflate_here ? zbuf.data() : c->hring + off;
    while (got < size) {
        const ssize_t k = pread(fd, dst + got, (size_t)(size - got), (off_t)(offset + got));
        if (k < 0) {
            if (errno == EINTR) continue;
            read_errno = errno;
            break;
        }
        if (k == 0) break;
        got += k;
    }
    close(fd);
    info[0] = got;
    bool inflated = true;
    if (inflate_here && got == size && !read_errno) {
        int64_t n_dec = 0;
        const int zst = pyas::host_inflate(zbuf.data(), size, c->hring + off, r.chunk_bytes, n_dec);
        info[1] = zst;
        info[2] = n_dec;
        inflated = zst == PYAS_INFLATE_OK && n_dec == r.chunk_bytes;
        if (!inflated) r.err = "inflate failed or size mismatch";
    }
    hipError_t ce = hipSuccess;
    if (c->caller_copy && got == size && !read_errno && inflated && r.nbytes > 0) {
        // this chunk's H2D copy, issued by the caller so that copies overlap
        // other callers' reads; ordered before the batch's launches by its ev_copy
        ce = hipSetDevice(c->device);
        if (ce == hipSuccess)
            ce = hipMemcpyAsync(c->dring + off, c->hring + off, (size_t)r.nbytes, hipMemcpyHostToDevice, c->cst);
    }

    const int64_t t_wait = now_ns();
    const bool ok = got == size && !read_errno && inflated && ce == hipSuccess;
    if (!ok) r.rc = ce == hipSuccess ? PYAS_EIO : PYAS_EDEVICE;
    if (ce != hipSuccess) r.err = hipGetErrorString(ce);
    c->q->finish(&r, ok, [&] {
        c->read_ns += t_wait - t_read;
        c->wait_ns += now_ns() - t_wait;
    });
    if (r.rc != PYAS_OK) {
        if (r.err.empty()) r.err = read_errno ? strerror(read_errno) : "short read";
        return pyas::set_error(r.rc, "%s", r.err.c_str());
    }
    return PYAS_OK;
}

}  // extern "C"
