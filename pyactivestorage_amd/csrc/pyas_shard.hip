// pyas_shard.hip — one process driving several GPUs (pyas_reduce_sharded).
//
// The reference's only parallelism is a thread pool over chunks
// (activestorage/active.py:557-572) followed by one combine of the
// per-chunk results (active.py:594-598).  Across the GPUs of a node the
// chunks shard with no data movement: each device reduces its own batch
// from its own HBM, and the per-device 32-byte totals travel in ONE RCCL
// all-gather (xGMI), after which every device folds them in device order,
// so the answer does not depend on arrival order.  This is the same
// exchange pyactivestorage_amd/distributed.py makes with torch.distributed
// (one process per GPU); here a non-Python host that holds every device in
// one process gets it through the C ABI.
#include <dlfcn.h>
#include <link.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pyas.h"
#include "pyas_internal.hpp"

namespace {

// RCCL is opened on first use, not linked: a process that never shards does
// not load it, and a process that already holds an RCCL (torch's
// torch/lib/librccl.so, loaded by `import torch` as a dependency of a
// RTLD_LOCAL extension, so its symbols are not in the global scope) shares
// that copy instead of loading a second one.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

// The path of an RCCL already mapped into the process (any file name
// containing "librccl"), or "" if none.
std::string loaded_rccl_path() {
    std::string found;
    dl_iterate_phdr(
        [](struct dl_phdr_info *info, size_t, void *data) -> int {
            const char *n = info->dlpi_name;
            if (n && std::strstr(n, "librccl")) {
                *static_cast<std::string *>(data) = n;
                return 1;
            }
            return 0;
        },
        &found);
    return found;
}

bool bind(void *h, Rccl &r) {
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.comm_abort = (decltype(r.comm_abort))dlsym(h, "ncclCommAbort");
    r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    return r.comm_init_all && r.comm_destroy && r.comm_abort && r.async_error && r.group_start &&
           r.group_end && r.all_gather && r.error_string;
}

int rccl(const Rccl *&out) {
    static std::once_flag once;
    static Rccl r;
    static bool ok = false;
    std::call_once(once, [] {
        // 1. symbols already in the global scope; 2. an RCCL mapped by
        // someone else (torch's copy); 3. the system RCCL
        if (dlsym(RTLD_DEFAULT, "ncclCommInitAll") && bind(RTLD_DEFAULT, r)) { ok = true; return; }
        const std::string mapped = loaded_rccl_path();
        void *h = mapped.empty() ? nullptr : dlopen(mapped.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        ok = h && bind(h, r);
    });
    if (!ok) return pyas::set_error(PYAS_ENOTSUP, "RCCL (librccl.so.1) could not be loaded");
    out = &r;
    return PYAS_OK;
}

// One communicator set per device list.  `mu` serialises its users: RCCL
// does not allow two group-start..group-end sequences on the same
// communicators at once, and pyas_shard_release must not destroy them while
// a call is still using them.
struct CommSet {
    std::mutex mu;
    std::vector<ncclComm_t> comms;   // comms[k] drives devices[k]
    bool dead = false;               // aborted or released: do not use
};

std::mutex g_mu;   // guards g_comms (the map), never held across RCCL calls
std::map<std::vector<int>, std::shared_ptr<CommSet>> g_comms;   // keyed by the device list, in order

int nccl_fail(const Rccl *x, ncclResult_t r, const char *what) {
    return pyas::set_error(PYAS_EDEVICE, "%s: %s", what, x->error_string(r));
}

// Communicators over `devs` (ncclCommInitAll: one rank per listed device,
// rank k = devs[k]); created once per device list and kept until
// pyas_shard_release() (or until a timed-out exchange aborts them).
int comms_for(const Rccl *x, const std::vector<int> &devs, std::shared_ptr<CommSet> &out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        auto cs = std::make_shared<CommSet>();
        cs->comms.resize(devs.size());
        ncclResult_t r = x->comm_init_all(cs->comms.data(), (int)devs.size(), devs.data());
        if (r != ncclSuccess) return nccl_fail(x, r, "ncclCommInitAll");
        it = g_comms.emplace(devs, std::move(cs)).first;
    }
    out = it->second;
    return PYAS_OK;
}

// Drop a communicator set from the cache (it was aborted).
void forget(const std::vector<int> &devs, const std::shared_ptr<CommSet> &cs) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(devs);
    if (it != g_comms.end() && it->second == cs) g_comms.erase(it);
}

// PYAS_SHARD_TIMEOUT_MS: when set (>= 0), pyas_reduce_sharded waits for the
// exchange up to that many milliseconds instead of returning at once.
long shard_timeout_ms() {
    const char *e = std::getenv("PYAS_SHARD_TIMEOUT_MS");
    if (!e || !*e) return -1;
    char *end = nullptr;
    const long v = std::strtol(e, &end, 10);
    return (end && *end == 0 && v >= 0) ? v : -1;
}

void abort_set(const Rccl *x, CommSet &cs) {
    for (ncclComm_t c : cs.comms) x->comm_abort(c);
    cs.dead = true;
}

// Wait for every stream to drain, watching the communicators for
// asynchronous errors, until `ms` have passed.  `pre[k]` was recorded on
// streams[k] just before its collectives were enqueued.
//   * an RCCL async error or a stream error: abort the set (its
//     communicators may be mid-collective) and report the device;
//   * expiry with every pre[k] reached: the collectives are running and a
//     peer is stalled -- abort the set so it cannot hang later users;
//   * expiry with some pre[k] not reached: that device is still reducing and
//     its collectives have not started, so aborting would free the
//     communicators under queued RCCL kernels.  The set is kept (the exchange
//     completes once the device catches up) and PYAS_EDEVICE names the
//     devices still busy.
// Caller holds cs.mu.
int bounded_wait(const Rccl *x, CommSet &cs, const std::vector<int> &devs, void *const *streams,
                 const std::vector<hipEvent_t> &pre, long ms) {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
    const size_t n = devs.size();
    std::vector<char> done(n, 0);
    for (;;) {
        size_t ndone = 0;
        for (size_t k = 0; k < n; ++k) {
            if (!done[k]) {
                ncclResult_t ae = ncclSuccess;
                if (x->async_error(cs.comms[k], &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                    abort_set(x, cs);
                    return pyas::set_error(PYAS_EDEVICE, "RCCL all-gather on device %d failed: %s", devs[k],
                                           x->error_string(ae));
                }
                const hipError_t q = hipStreamQuery((hipStream_t)streams[k]);
                if (q == hipSuccess) {
                    done[k] = 1;
                } else if (q != hipErrorNotReady) {
                    abort_set(x, cs);
                    return pyas::set_error(PYAS_EDEVICE, "device %d stream: %s; the RCCL communicators were "
                                           "aborted", devs[k], hipGetErrorString(q));
                }
            }
            ndone += done[k] ? 1 : 0;
        }
        if (ndone == n) return PYAS_OK;
        if (std::chrono::steady_clock::now() >= t_end) break;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    std::string late, busy;
    for (size_t k = 0; k < n; ++k) {
        if (done[k]) continue;
        late += (late.empty() ? "" : ",") + std::to_string(devs[k]);
        if (hipEventQuery(pre[k]) == hipErrorNotReady) busy += (busy.empty() ? "" : ",") + std::to_string(devs[k]);
    }
    if (!busy.empty())
        return pyas::set_error(PYAS_EDEVICE,
                               "sharded reduce: device(s) %s did not finish within %ld ms; device(s) %s had not "
                               "reached the exchange, so the communicators were kept and the exchange stays "
                               "queued (synchronise the streams before reading out)",
                               late.c_str(), ms, busy.c_str());
    abort_set(x, cs);
    return pyas::set_error(PYAS_EDEVICE,
                           "sharded reduce: device(s) %s did not finish within %ld ms; the RCCL "
                           "communicators were aborted (the next call creates new ones)",
                           late.c_str(), ms);
}

// Per-call device scratch of one device (stream-ordered allocation).
struct Scratch {
    void *p = nullptr;
    hipStream_t st = nullptr;
    int dev = 0;
    ~Scratch() {
        if (p) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(dev);
            (void)hipFreeAsync(p, st);
            (void)hipSetDevice(cur);
        }
    }
};

}  // namespace

extern "C" {

int pyas_reduce_sharded_tie(pyas_ctx *const *ctx, const pyas_batch *const *per_dev, const pyas_mask *const *mask,
                            int32_t ndev, uint32_t combine_flags, const pyas_tie_geom *geom, uint32_t which,
                            pyas_partial *const *out, void *const *streams) {
    if (ndev < 1) return pyas::set_error(PYAS_EINVAL, "ndev must be >= 1 (got %d)", ndev);
    if (!ctx || !per_dev || !out || !streams) return pyas::set_error(PYAS_EINVAL, "NULL argument");
    if (which > 2u) return pyas::set_error(PYAS_EINVAL, "which must be 0, 1 (min) or 2 (max) (got %u)", which);
    if (which && !geom) return pyas::set_error(PYAS_EINVAL, "zero sign (which != 0) needs the tie geometry");
    std::vector<int> devs((size_t)ndev);
    int32_t dtype = -1;
    for (int k = 0; k < ndev; ++k) {
        if (!ctx[k] || !per_dev[k] || !out[k]) return pyas::set_error(PYAS_EINVAL, "NULL entry for device %d", k);
        devs[k] = pyas::ctx_device(ctx[k]);
        for (int j = 0; j < k; ++j)
            if (devs[j] == devs[k])
                return pyas::set_error(PYAS_EINVAL, "device %d appears twice (entries %d and %d)", devs[k], j, k);
        if (k == 0) dtype = per_dev[k]->dtype;
        else if (per_dev[k]->dtype != dtype)
            return pyas::set_error(PYAS_EINVAL, "entry %d has dtype %d, entry 0 has %d", k, per_dev[k]->dtype,
                                   dtype);
    }
    if (which && dtype != PYAS_F32 && dtype != PYAS_F64) which = 0u;   // integers have no signed zero
    // device k's chunks sit at positions base[k] .. base[k] + n_chunks of the
    // query's chunk order (the `out` array of active.py:594, one call of lr)
    std::vector<int64_t> base((size_t)ndev);
    int64_t lr = 0;
    for (int k = 0; k < ndev; ++k) {
        base[k] = lr;
        lr += per_dev[k]->n_chunks;
    }
    // 1. each device: its batch -> its total, written where the in-place
    //    all-gather expects rank k's piece (out[k][1 + k]).  With the zero
    //    sign, the per-chunk partials are kept (scratch) for level 1 of the
    //    sign (pyas_tie_chunks_total, storage.py:99-100), level 2 keys this
    //    device's total (pyas_tie_segments), and the keys of every device
    //    travel with the totals to pyas_tie_finalize (active.py:594).
    std::vector<Scratch> scratch((size_t)ndev);
    std::vector<uint64_t *> keys((size_t)ndev, nullptr);
    for (int k = 0; k < ndev; ++k) {
        pyas_partial *parts = nullptr;
        if (which) {
            const size_t nparts = (size_t)std::max<int64_t>(per_dev[k]->n_chunks, 1);
            const size_t nbytes = nparts * sizeof(pyas_partial) + (size_t)ndev * 2 * sizeof(uint64_t);
            Scratch &sc = scratch[(size_t)k];
            sc.dev = devs[k];
            sc.st = (hipStream_t)streams[k];
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(devs[k]);
            const hipError_t e = hipMallocAsync(&sc.p, nbytes, sc.st);
            (void)hipSetDevice(cur);
            if (e != hipSuccess) {
                sc.p = nullptr;
                return pyas::set_error(PYAS_ENOMEM, "device %d scratch: %s", devs[k], hipGetErrorString(e));
            }
            parts = static_cast<pyas_partial *>(sc.p);
            keys[k] = reinterpret_cast<uint64_t *>(parts + nparts);
        }
        const pyas_mask *mk = mask ? mask[k] : nullptr;
        int rc0 = pyas_reduce_chunks(ctx[k], per_dev[k], mk, parts, out[k] + 1 + k, combine_flags, streams[k]);
        if (rc0) return rc0;
        if (which) {
            rc0 = pyas_tie_keys_reset(ctx[k], keys[k] + 2 * k, 1, streams[k]);   // this device's [K1, W]
            if (!rc0 && per_dev[k]->n_chunks > 0) {
                rc0 = pyas_tie_chunks_total(ctx[k], per_dev[k], mk, geom, which, parts, base[k], lr, streams[k]);
                if (!rc0)
                    rc0 = pyas_tie_segments(ctx[k], dtype, parts, nullptr, nullptr, 1, per_dev[k]->n_chunks, base[k],
                                            lr, which, out[k] + 1 + k, keys[k] + 2 * k, streams[k]);
            }
            if (rc0) return rc0;
        }
    }
    // 2. ONE exchange over xGMI, in place: the 32-byte totals (and the 16-byte
    //    keys) in one RCCL group; the communicator set is held from group
    //    start to group end (and through the optional bounded wait), so
    //    concurrent callers on the same device list take turns
    const Rccl *x = nullptr;
    int rc = rccl(x);
    if (rc) return rc;
    std::shared_ptr<CommSet> cs;
    rc = comms_for(x, devs, cs);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(cs->mu);
        if (cs->dead) return pyas::set_error(PYAS_EDEVICE, "the RCCL communicators were released during the call");
        const long ms = shard_timeout_ms();
        std::vector<hipEvent_t> pre;
        if (ms >= 0) {   // where each stream reaches its collectives
            pre.assign((size_t)ndev, nullptr);
            for (int k = 0; k < ndev; ++k) {
                int cur = 0;
                (void)hipGetDevice(&cur);
                (void)hipSetDevice(devs[k]);
                hipError_t e = hipEventCreateWithFlags(&pre[k], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventRecord(pre[k], (hipStream_t)streams[k]);
                (void)hipSetDevice(cur);
                if (e != hipSuccess) {
                    for (hipEvent_t ev : pre) if (ev) (void)hipEventDestroy(ev);
                    return pyas::set_error(PYAS_EDEVICE, "device %d event: %s", devs[k], hipGetErrorString(e));
                }
            }
        }
        ncclResult_t r = x->group_start();
        if (r != ncclSuccess) return nccl_fail(x, r, "ncclGroupStart");
        for (int k = 0; k < ndev && r == ncclSuccess; ++k) {
            r = x->all_gather(out[k] + 1 + k, out[k] + 1, sizeof(pyas_partial), ncclUint8, cs->comms[k],
                              (hipStream_t)streams[k]);
            if (r == ncclSuccess && which)
                r = x->all_gather(keys[k] + 2 * k, keys[k], 2 * sizeof(uint64_t), ncclUint8, cs->comms[k],
                                  (hipStream_t)streams[k]);
        }
        if (r != ncclSuccess) {
            x->group_end();
            for (hipEvent_t ev : pre) (void)hipEventDestroy(ev);
            return nccl_fail(x, r, "ncclAllGather");
        }
        r = x->group_end();
        if (r != ncclSuccess) {
            for (hipEvent_t ev : pre) (void)hipEventDestroy(ev);
            return nccl_fail(x, r, "ncclGroupEnd");
        }
        if (ms >= 0) {
            rc = bounded_wait(x, *cs, devs, streams, pre, ms);
            for (hipEvent_t ev : pre) (void)hipEventDestroy(ev);
            if (rc) {
                if (cs->dead) forget(devs, cs);
                return rc;
            }
        }
    }
    // 3. every device folds the totals in device order (the per-chunk sums
    //    were already rounded to the variable dtype under combine_flags),
    //    then gives a zero min/max NumPy's sign from every device's keys
    for (int k = 0; k < ndev; ++k) {
        rc = pyas_combine_partials(ctx[k], dtype, out[k] + 1, ndev, 0u, out[k], streams[k]);
        if (rc) return rc;
        if (which) {
            rc = pyas_tie_finalize(ctx[k], dtype, keys[k], 1, ndev, lr, which, out[k], streams[k]);
            if (rc) return rc;
        }
    }
    return PYAS_OK;
}

int pyas_reduce_sharded(pyas_ctx *const *ctx, const pyas_batch *const *per_dev, const pyas_mask *const *mask,
                        int32_t ndev, uint32_t combine_flags, pyas_partial *const *out, void *const *streams) {
    return pyas_reduce_sharded_tie(ctx, per_dev, mask, ndev, combine_flags, nullptr, 0u, out, streams);
}

int pyas_shard_release(void) {
    std::map<std::vector<int>, std::shared_ptr<CommSet>> sets;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        sets.swap(g_comms);
    }
    if (sets.empty()) return PYAS_OK;
    const Rccl *x = nullptr;
    int rc = rccl(x);
    if (rc) return rc;
    for (auto &kv : sets) {
        std::lock_guard<std::mutex> lk(kv.second->mu);   // waits for a call still using the set
        if (kv.second->dead) continue;
        kv.second->dead = true;
        for (ncclComm_t c : kv.second->comms) {
            ncclResult_t r = x->comm_destroy(c);
            if (r != ncclSuccess && rc == PYAS_OK) rc = nccl_fail(x, r, "ncclCommDestroy");
        }
    }
    return rc;
}

}  // extern "C"
