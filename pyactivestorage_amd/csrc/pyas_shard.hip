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
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <mutex>
#include <vector>

#include "pyas.h"
#include "pyas_internal.hpp"

namespace {

struct CommSet {
    std::vector<ncclComm_t> comms;   // comms[k] drives devices[k]
};

std::mutex g_mu;
std::map<std::vector<int>, CommSet> g_comms;   // keyed by the device list, in order

int nccl_fail(ncclResult_t r, const char *what) {
    return pyas::set_error(PYAS_EDEVICE, "%s: %s", what, ncclGetErrorString(r));
}

// Communicators over `devs` (ncclCommInitAll: one rank per listed device,
// rank k = devs[k]); created once per device list and kept until
// pyas_shard_release().
int comms_for(const std::vector<int> &devs, std::vector<ncclComm_t> &out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        CommSet cs;
        cs.comms.resize(devs.size());
        ncclResult_t r = ncclCommInitAll(cs.comms.data(), (int)devs.size(), devs.data());
        if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitAll");
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
    std::vector<ncclComm_t> comms;
    int rc = comms_for(devs, comms);
    if (rc) return rc;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (int k = 0; k < ndev; ++k) {
        r = ncclAllGather(out[k] + 1 + k, out[k] + 1, sizeof(pyas_partial), ncclUint8, comms[k],
                          (hipStream_t)streams[k]);
        if (r != ncclSuccess) {
            ncclGroupEnd();
            return nccl_fail(r, "ncclAllGather");
        }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
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
    int rc = PYAS_OK;
    for (auto &kv : g_comms)
        for (ncclComm_t c : kv.second.comms) {
            ncclResult_t r = ncclCommDestroy(c);
            if (r != ncclSuccess && rc == PYAS_OK) rc = nccl_fail(r, "ncclCommDestroy");
        }
    g_comms.clear();
    return rc;
}

}  // extern "C"
