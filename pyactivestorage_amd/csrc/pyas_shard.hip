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
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <mutex>
#include <vector>

#include "pyas.h"
#include "pyas_internal.hpp"

namespace {

// RCCL is opened on first use, not linked: a process that never shards does
// not load it, and a process that already holds an RCCL (torch's, loaded by
// `import torch`) shares that copy instead of loading a second one.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

int rccl(const Rccl *&out) {
    static std::once_flag once;
    static Rccl r;
    static bool ok = false;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);   // already loaded?
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.all_gather && r.error_string;
    });
    if (!ok) return pyas::set_error(PYAS_ENOTSUP, "RCCL (librccl.so.1) could not be loaded");
    out = &r;
    return PYAS_OK;
}

struct CommSet {
    std::vector<ncclComm_t> comms;   // comms[k] drives devices[k]
};

std::mutex g_mu;
std::map<std::vector<int>, CommSet> g_comms;   // keyed by the device list, in order

int nccl_fail(const Rccl *x, ncclResult_t r, const char *what) {
    return pyas::set_error(PYAS_EDEVICE, "%s: %s", what, x->error_string(r));
}

// Communicators over `devs` (ncclCommInitAll: one rank per listed device,
// rank k = devs[k]); created once per device list and kept until
// pyas_shard_release().
int comms_for(const Rccl *x, const std::vector<int> &devs, std::vector<ncclComm_t> &out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        CommSet cs;
        cs.comms.resize(devs.size());
        ncclResult_t r = x->comm_init_all(cs.comms.data(), (int)devs.size(), devs.data());
        if (r != ncclSuccess) return nccl_fail(x, r, "ncclCommInitAll");
        it = g_comms.emplace(devs, std::move(cs)).first;
    }
    out = it->second.comms;
    return PYAS_OK;
}

}  // namespace

extern "C" {

int pyas_reduce_sharded(pyas_ctx *const *ctx, const pyas_batch *const *per_dev, const pyas_mask *const *mask,
                        int32_t ndev, uint32_t combine_flags, pyas_partial *const *out, void *const *streams) {
    if (ndev < 1) return pyas::set_error(PYAS_EINVAL, "ndev must be >= 1 (got %d)", ndev);
    if (!ctx || !per_dev || !out || !streams) return pyas::set_error(PYAS_EINVAL, "NULL argument");
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
    // 1. each device: its batch -> its total, written where the in-place
    //    all-gather expects rank k's piece (out[k][1 + k])
    for (int k = 0; k < ndev; ++k) {
        int rc = pyas_reduce_chunks(ctx[k], per_dev[k], mask ? mask[k] : nullptr, nullptr, out[k] + 1 + k,
                                    combine_flags, streams[k]);
        if (rc) return rc;
    }
    // 2. ONE all-gather of the 32-byte totals over xGMI, in place
    const Rccl *x = nullptr;
    int rc = rccl(x);
    if (rc) return rc;
    std::vector<ncclComm_t> comms;
    rc = comms_for(x, devs, comms);
    if (rc) return rc;
    ncclResult_t r = x->group_start();
    if (r != ncclSuccess) return nccl_fail(x, r, "ncclGroupStart");
    for (int k = 0; k < ndev; ++k) {
        r = x->all_gather(out[k] + 1 + k, out[k] + 1, sizeof(pyas_partial), ncclUint8, comms[k],
                          (hipStream_t)streams[k]);
        if (r != ncclSuccess) {
            x->group_end();
            return nccl_fail(x, r, "ncclAllGather");
        }
    }
    r = x->group_end();
    if (r != ncclSuccess) return nccl_fail(x, r, "ncclGroupEnd");
    // 3. every device folds the totals in device order (the per-chunk sums
    //    were already rounded to the variable dtype under combine_flags)
    for (int k = 0; k < ndev; ++k) {
        rc = pyas_combine_partials(ctx[k], dtype, out[k] + 1, ndev, 0u, out[k], streams[k]);
        if (rc) return rc;
    }
    return PYAS_OK;
}

int pyas_shard_release(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_comms.empty()) return PYAS_OK;
    const Rccl *x = nullptr;
    int rc = rccl(x);
    if (rc) return rc;
    for (auto &kv : g_comms)
        for (ncclComm_t c : kv.second.comms) {
            ncclResult_t r = x->comm_destroy(c);
            if (r != ncclSuccess && rc == PYAS_OK) rc = nccl_fail(x, r, "ncclCommDestroy");
        }
    g_comms.clear();
    return rc;
}

}  // extern "C"
