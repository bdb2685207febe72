// pyas_ingest.hip — host ingest (row f2): positioned file reads straight into
// device memory through a ring of pinned staging slots.
//
// The reference opens the file and reads each chunk on its own, once per
// chunk, from a 30-thread pool (activestorage/storage.py:51-53 open +
// read_block at :156-162; pool at activestorage/active.py:557-572), then
// NumPy works on the host copy.  Here a query's chunk byte ranges are read by
// `threads` workers with pread(2) into pinned slots; every filled slot is
// copied H2D with hipMemcpyAsync on the caller's stream while the workers
// fill the next slots, so disk/page-cache reads, PCIe and the device work
// queued behind the copies overlap.  Slot reuse waits on the event recorded
// after that slot's previous copy.
#include <errno.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pyas_internal.hpp"

namespace pyas {

// zlib.decompress of one stream (storage.py:119-120 through numcodecs.Zlib,
// hdf2numcodec.py:34-35) into at most `cap` bytes of dst: a
// pyas_inflate_status.  Bytes after the stream's end are ignored, as
// zlib.decompress does; the caller re-runs a failed stream through zlib to
// raise zlib's own error.
int host_inflate(const uint8_t *src, int64_t n_src, uint8_t *dst, int64_t cap, int64_t &n_out) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    n_out = 0;
    if (inflateInit(&zs) != Z_OK) return PYAS_INFLATE_BAD_HEADER;
    zs.next_in = const_cast<Bytef *>(src);
    zs.avail_in = (uInt)n_src;
    zs.next_out = dst;
    zs.avail_out = (uInt)cap;
    const int r = inflate(&zs, Z_FINISH);
    n_out = (int64_t)zs.total_out;
    int st = PYAS_INFLATE_OK;
    if (r == Z_NEED_DICT) st = PYAS_INFLATE_NEED_DICT;
    else if (r == Z_DATA_ERROR) st = PYAS_INFLATE_BAD_CODE;
    else if (r != Z_STREAM_END) st = zs.avail_out == 0 ? PYAS_INFLATE_OVERFLOW : PYAS_INFLATE_TRUNCATED;
    inflateEnd(&zs);
    return st;
}

namespace {

struct Piece {
    int64_t file_off, size, dst_off, slot_off;
};

struct Group {   // what one staging slot carries: consecutive pieces
    size_t first, count;
    int64_t bytes;
};

}  // namespace

// Default ring: 16 x 64 MiB.  Measured on MI355X (tools/bench_ingest.py, 4 GiB
// page-cache-hot file, 1 MiB chunks): what matters is the bytes in flight —
// 256 MiB rings reach 25-36 GB/s, 512 MiB 48-52 GB/s, 1 GiB 51-55 GB/s (the
// PCIe Gen5 x16 copy rate is ~56 GB/s).  Slots are pinned lazily, one at a
// time, so a small query pins only the slots it uses.
struct Ingest {
    int device = 0;
    int32_t n_slots = 16;
    int64_t slot_bytes = 64 << 20;
    std::vector<uint8_t *> slot;     // hipHostMalloc'd on first use
    std::vector<hipEvent_t> done;    // recorded after each slot's latest copy
    std::mutex call_mu;              // one pyas_read_ranges at a time per context

    ~Ingest() { release(); }

    void release() {
        for (size_t s = 0; s < slot.size(); ++s) {
            if (slot[s]) {
                (void)hipEventSynchronize(done[s]);
                (void)hipHostFree(slot[s]);
            }
        }
        for (auto e : done) (void)hipEventDestroy(e);
        slot.clear();
        done.clear();
    }

    hipError_t ensure(int used) {
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return e;
        if (done.empty()) {
            slot.assign((size_t)n_slots, nullptr);
            done.resize((size_t)n_slots);
            for (auto &ev : done) {
                e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
                if (e != hipSuccess) return e;
            }
        }
        for (int s = 0; s < used; ++s) {
            if (slot[s]) continue;
            e = hipHostMalloc((void **)&slot[s], (size_t)slot_bytes, hipHostMallocDefault);
            if (e != hipSuccess) { slot[s] = nullptr; return e; }
        }
        return hipSuccess;
    }
};

Ingest *ingest_create(int device) {
    Ingest *g = new Ingest;
    g->device = device;
    return g;
}

void ingest_destroy(Ingest *g) { delete g; }

int ingest_configure(Ingest *g, int32_t n_slots, int64_t slot_bytes, std::string &msg) {
    std::lock_guard<std::mutex> lk(g->call_mu);
    if (n_slots < 2 || n_slots > 256) { msg = "ingest slots must be in [2, 256]"; return PYAS_EINVAL; }
    if (slot_bytes < (1 << 16) || slot_bytes > (int64_t(1) << 31)) {
        msg = "ingest slot size must be in [64 KiB, 2 GiB]";
        return PYAS_EINVAL;
    }
    g->release();
    g->n_slots = n_slots;
    g->slot_bytes = slot_bytes;
    return PYAS_OK;
}

// pread the whole range (restarting on EINTR and short reads); returns 0 or errno,
// ENODATA for end of file before `size` bytes.
static int pread_full(int fd, uint8_t *dst, int64_t size, int64_t off) {
    while (size > 0) {
        const ssize_t r = ::pread(fd, dst, (size_t)std::min<int64_t>(size, int64_t(1) << 30), (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (r == 0) return ENODATA;
        dst += r;
        off += r;
        size -= r;
    }
    return 0;
}

int ingest_read(Ingest *g, int fd, int64_t n, const int64_t *file_offsets, const int64_t *sizes,
                uint8_t *dst, const int64_t *dst_offsets, int32_t threads, hipStream_t st,
                std::string &msg, int64_t zlib_out, int32_t *status) {
    std::lock_guard<std::mutex> lk(g->call_mu);
    if (n < 0 || (n > 0 && (!file_offsets || !sizes || !dst || !dst_offsets))) {
        msg = "read_ranges: NULL array or negative count";
        return PYAS_EINVAL;
    }
    if (fd < 0) { msg = "read_ranges: invalid file descriptor"; return PYAS_EINVAL; }
    if (zlib_out < 0 || (zlib_out > 0 && !status)) { msg = "read_ranges: zlib output size or status"; return PYAS_EINVAL; }
    if (zlib_out > g->slot_bytes) {
        msg = "read_ranges: inflated chunk larger than a staging slot (pyas_ctx_set_ingest_slots)";
        return PYAS_ENOTSUP;
    }
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    // ranges -> pieces of at most one slot -> groups (one slot each)
    std::vector<Piece> pieces;
    pieces.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        if (sizes[i] < 0 || file_offsets[i] < 0 || dst_offsets[i] < 0) {
            msg = "read_ranges: negative offset or size at range " + std::to_string(i);
            return PYAS_EINVAL;
        }
        if (zlib_out) {   // one piece per stream: its inflated bytes fill the slot space
            status[i] = PYAS_INFLATE_OK;
            pieces.push_back({file_offsets[i], sizes[i], dst_offsets[i], 0});
            continue;
        }
        for (int64_t p = 0; p < sizes[i]; p += g->slot_bytes)
            pieces.push_back({file_offsets[i] + p, std::min(g->slot_bytes, sizes[i] - p), dst_offsets[i] + p, 0});
    }
    auto footprint = [&](const Piece &pc) { return zlib_out ? zlib_out : pc.size; };
    if (pieces.empty()) return PYAS_OK;
    // a group fills one slot; in zlib mode the inflating is the work, so
    // the streams are spread over as many groups as can be in flight at once
    // (one per slot, one reader thread each)
    int64_t group_cap = g->slot_bytes;
    if (zlib_out) {
        const int64_t lanes = std::max<int64_t>(1, std::min<int64_t>(threads, g->n_slots));
        const int64_t per = (n + lanes - 1) / lanes;
        group_cap = std::min<int64_t>(g->slot_bytes, std::max<int64_t>(1, per) * zlib_out);
    }
    std::vector<Group> groups;
    {
        Group cur{0, 0, 0};
        for (size_t k = 0; k < pieces.size(); ++k) {
            if (cur.count && cur.bytes + footprint(pieces[k]) > group_cap) {
                groups.push_back(cur);
                cur = Group{k, 0, 0};
            }
            pieces[k].slot_off = cur.bytes;
            cur.bytes += footprint(pieces[k]);
            cur.count++;
        }
        groups.push_back(cur);
    }
    const int K = g->n_slots;
    const int64_t G = (int64_t)groups.size();
    hipError_t he = g->ensure((int)std::min<int64_t>(K, G));
    if (he != hipSuccess) { msg = std::string("pinned staging: ") + hipGetErrorString(he); return PYAS_ENOMEM; }

    std::atomic<int64_t> next{0};
    std::atomic<int> err_code{0};
    std::mutex mu;
    std::condition_variable cv;
    // enq[s]: index of the last group whose copy from slot s is enqueued (-1 none)
    std::vector<int64_t> enq(K, -1);
    // a slot's first use in this call still waits for the previous call's copy
    std::string err_msg;

    auto worker = [&]() {
        (void)hipSetDevice(g->device);
        std::vector<uint8_t> zbuf;   // this thread's compressed bytes (zlib mode)
        for (;;) {
            const int64_t gi = next.fetch_add(1);
            if (gi >= G || err_code.load()) break;
            const int s = (int)(gi % K);
            {   // the previous group of this slot must have enqueued its copy
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return enq[s] == gi - K || (gi < K && enq[s] == -1) || err_code.load(); });
                if (err_code.load()) break;
            }
            if (hipEventSynchronize(g->done[s]) != hipSuccess) {   // ... and that copy has landed
                std::lock_guard<std::mutex> l(mu);
                err_code = PYAS_EDEVICE;
                err_msg = "staging event";
                cv.notify_all();
                break;
            }
            uint8_t *slot = g->slot[(size_t)s];
            const Group &gr = groups[(size_t)gi];
            int rc = 0;
            size_t bad = 0;
            for (size_t k = gr.first; k < gr.first + gr.count && !rc; ++k) {
                bad = k;
                if (!zlib_out) {
                    rc = pread_full(fd, slot + pieces[k].slot_off, pieces[k].size, pieces[k].file_off);
                    continue;
                }
                // zlib: pread the stream, inflate it on this thread straight
                // into the pinned slot
                if ((int64_t)zbuf.size() < pieces[k].size) zbuf.resize((size_t)pieces[k].size);
                rc = pread_full(fd, zbuf.data(), pieces[k].size, pieces[k].file_off);
                if (rc) break;
                int64_t n_out = 0;
                int zs = host_inflate(zbuf.data(), pieces[k].size, slot + pieces[k].slot_off, zlib_out, n_out);
                if (zs == PYAS_INFLATE_OK && n_out != zlib_out) zs = PYAS_INFLATE_OVERFLOW;
                status[k] = zs;   // pieces are the streams, in order
            }
            std::lock_guard<std::mutex> l(mu);
            if (rc) {
                err_code = PYAS_EIO;
                err_msg = std::string(rc == ENODATA ? "short read (end of file)" : std::strerror(rc)) +
                          " at file offset " + std::to_string(pieces[bad].file_off) + " (" +
                          std::to_string(pieces[bad].size) + " bytes)";
                cv.notify_all();
                break;
            }
            // contiguous destination runs -> one copy each
            hipError_t e = hipSuccess;
            size_t k = gr.first;
            while (k < gr.first + gr.count && e == hipSuccess) {
                size_t j = k + 1;
                int64_t len = footprint(pieces[k]);
                while (j < gr.first + gr.count && pieces[j].dst_off == pieces[k].dst_off + len &&
                       pieces[j].slot_off == pieces[k].slot_off + len) {
                    len += footprint(pieces[j]);
                    ++j;
                }
                e = hipMemcpyAsync(dst + pieces[k].dst_off, slot + pieces[k].slot_off, (size_t)len,
                                   hipMemcpyHostToDevice, st);
                k = j;
            }
            if (e == hipSuccess) e = hipEventRecord(g->done[s], st);
            if (e != hipSuccess) {
                err_code = PYAS_EDEVICE;
                err_msg = std::string("H2D copy: ") + hipGetErrorString(e);
            }
            enq[s] = gi;
            cv.notify_all();
            if (e != hipSuccess) break;
        }
    };
    const int nt = (int)std::min<int64_t>(threads, G);
    std::vector<std::thread> pool;
    pool.reserve((size_t)nt);
    for (int t = 0; t < nt; ++t) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
    if (err_code.load()) {
        msg = err_msg;
        return err_code.load();
    }
    return PYAS_OK;
}

}  // namespace pyas
