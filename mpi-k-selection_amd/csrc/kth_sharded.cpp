// kth_sharded.cpp -- single-process multi-GPU selection (include/kth.h
// kth_sharded_*, kth_select_i32_sharded).
//
// Replaces the whole CGM driver of the reference (TODO-kth-problem-cgm.c:81-278:
// block partition + Scatterv, ~12 weighted-median rounds of Gather / Bcast /
// Allreduce, final Gatherv + rank-0 sort) for a caller that holds one shard per
// GPU in ONE process: the same per-rank device steps as the one-process-per-GPU
// protocol (kth_dist_*), driven here for every device in turn, with the
// collectives as grouped RCCL calls over communicators from ncclCommInitAll:
//
//   per device: begin, sample           -> ncclAllGather of the samples
//   per device: window, scan            -> ncclAllReduce of the counts slot
//                                          (+ the candidates' first digit)
//   per device: level l (usually one)   -> ncclAllReduce of the histogram slot
//   per device: result                  -> every device holds the same answer
//
// Each device's work is enqueued on its own ctx stream, the collectives on the
// same streams; the host waits once before the second level call (for level
// 0's DistStatus: how many levels follow, while the device still has the
// all-reduce after level 0 queued) and once at the end to read the answer.  RCCL is resolved at first use (dlopen of the
// librccl.so.1 already in the process, e.g. torch's, or the system one), so
// libkth.so itself does not depend on it.
//
// Local transport: a handle whose shards all live on ONE device (the same
// device id repeated, e.g. 8 shards x 2^30 keys on one MI355X) runs the same
// per-shard steps with no RCCL: every shard's ctx enqueues on one shared
// stream (so each step sees the previous step of every shard complete), the
// samples are written straight into one gathered buffer at their offsets (the
// all-gather), and each all-reduce is one small kernel that sums the shards'
// slot words and writes the sum back to every shard's slot
// (kth_internal_slots_sum) -- the arithmetic RCCL's ncclSum performs.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kth.h"
#include "kth_internal.h"

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
};

const Rccl &rccl() {
    static const Rccl r = [] {
        Rccl x;
        void *h = nullptr;
        // prefer a copy already loaded (torch's), then the system one
        const char *names[] = {"librccl.so.1", "librccl.so"};
        for (const char *nm : names)
            if (!h) h = dlopen(nm, RTLD_NOW | RTLD_NOLOAD);
        const char *env = getenv("KTH_RCCL_LIB");
        if (!h && env) h = dlopen(env, RTLD_NOW);
        for (const char *nm : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
            if (!h) h = dlopen(nm, RTLD_NOW);
        if (!h) return x;
        x.CommInitAll = reinterpret_cast<decltype(x.CommInitAll)>(dlsym(h, "ncclCommInitAll"));
        x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
        x.AllReduce = reinterpret_cast<decltype(x.AllReduce)>(dlsym(h, "ncclAllReduce"));
        x.AllGather = reinterpret_cast<decltype(x.AllGather)>(dlsym(h, "ncclAllGather"));
        x.Broadcast = reinterpret_cast<decltype(x.Broadcast)>(dlsym(h, "ncclBroadcast"));
        x.GroupStart = reinterpret_cast<decltype(x.GroupStart)>(dlsym(h, "ncclGroupStart"));
        x.GroupEnd = reinterpret_cast<decltype(x.GroupEnd)>(dlsym(h, "ncclGroupEnd"));
        x.ok = x.CommInitAll && x.CommDestroy && x.AllReduce && x.AllGather && x.Broadcast && x.GroupStart && x.GroupEnd;
        return x;
    }();
    return r;
}

#define TRY(x)                           \
    do {                                 \
        int r_ = (x);                    \
        if (r_ < 0) return r_;           \
    } while (0)
#define HIPT(x)                                  \
    do {                                         \
        if ((x) != hipSuccess) {                 \
            (void)hipGetLastError();             \
            return KTH_EHIP;                     \
        }                                        \
    } while (0)
#define NCCLT(x)                                 \
    do {                                         \
        if ((x) != ncclSuccess) return KTH_ECOMM; \
    } while (0)

constexpr int64_t SMALL_PER_GPU = 64;  // fewer keys on some GPU: gather to device 0

struct Dev {
    int device = 0;
    kth_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    bool own_stream = false;  // local transport: shard 0 owns the shared stream
    ncclComm_t comm = nullptr;
    uint64_t *slots = nullptr;  // 3 * KTH_STATS_WORDS
    uint32_t *sample = nullptr, *gathered = nullptr;
    int64_t sample_cap = 0, gathered_cap = 0;
    int32_t *out = nullptr;
    int32_t *staging = nullptr;  // device 0: the union, small / unbalanced inputs
    int64_t staging_cap = 0;
    int32_t *d_status = nullptr;  // the handle's host status words, as this device addresses them
};

int grow(int device, void **p, int64_t *cap, int64_t bytes) {
    if (*cap >= bytes) return KTH_OK;
    HIPT(hipSetDevice(device));
    HIPT(hipDeviceSynchronize());
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, (size_t)bytes) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return KTH_ENOMEM;
    }
    *cap = bytes;
    return KTH_OK;
}

}  // namespace

struct kth_sharded {
    std::vector<Dev> d;
    bool local = false;           // every shard on one device: the local transport (no RCCL)
    uint32_t *lgathered = nullptr;  // local transport: the gathered sample (every shard's at its offset)
    int64_t lgathered_cap = 0;
    int32_t *h_status = nullptr;  // per shard [answer, error], host-visible (pinned, mapped, portable)
    int32_t *d_status = nullptr;  // ... its device address
    double enqueue_us = 0;  // host time of the last select up to its last enqueue (kth_sharded_enqueue_us)
};

namespace {

// All shards copied next to each other on device 0, then one single-GPU select
// (cf. the reference's final Gatherv + rank-0 solve, TODO-kth-problem-cgm.c:242-278).
int select_gathered(kth_sharded *h, const int32_t *const *shards, const int64_t *shard_n, int64_t n_total, int64_t k,
                    int32_t *out) {
    Dev &d0 = h->d[0];
    TRY(grow(d0.device, reinterpret_cast<void **>(&d0.staging), &d0.staging_cap, std::max<int64_t>(n_total, 1) * 4));
    HIPT(hipSetDevice(d0.device));
    for (Dev &x : h->d) HIPT(hipStreamSynchronize(x.stream));  // the handle's earlier work on the shards
    int64_t off = 0;
    for (size_t i = 0; i < h->d.size(); ++i) {
        if (shard_n[i] > 0 && h->d[i].device == d0.device)
            HIPT(hipMemcpyAsync(d0.staging + off, shards[i], (size_t)shard_n[i] * 4, hipMemcpyDeviceToDevice,
                                d0.stream));
        else if (shard_n[i] > 0)
            HIPT(hipMemcpyPeerAsync(d0.staging + off, d0.device, shards[i], h->d[i].device, (size_t)shard_n[i] * 4,
                                    d0.stream));
        off += shard_n[i];
    }
    return kth_select_i32_ctx(d0.ctx, d0.staging, n_total, k, out);
}

}  // namespace

extern "C" {

int kth_sharded_destroy(kth_sharded *h) {
    if (!h) return KTH_EINVAL;
    for (Dev &x : h->d) {
        (void)hipSetDevice(x.device);
        if (x.stream) (void)hipStreamSynchronize(x.stream);
        if (x.comm && rccl().ok) (void)rccl().CommDestroy(x.comm);
        if (x.slots) (void)hipFree(x.slots);
        if (x.sample) (void)hipFree(x.sample);
        if (x.gathered) (void)hipFree(x.gathered);
        if (x.out) (void)hipFree(x.out);
        if (x.staging) (void)hipFree(x.staging);
        if (x.ctx) (void)kth_ctx_destroy(x.ctx);  // before its stream: it synchronises on it
    }
    for (Dev &x : h->d)  // (local transport: one stream, owned by shard 0)
        if (x.stream && x.own_stream) {
            (void)hipSetDevice(x.device);
            (void)hipStreamDestroy(x.stream);
        }
    if (h->lgathered) {
        (void)hipSetDevice(h->d[0].device);
        (void)hipFree(h->lgathered);
    }
    if (h->h_status) (void)hipHostFree(h->h_status);
    delete h;
    return KTH_OK;
}

int kth_sharded_create(const int *devices, int ngpu, kth_sharded **out) {
    if (!out) return KTH_EINVAL;
    *out = nullptr;
    if (!devices || ngpu < 1) return KTH_EINVAL;
    const int ndev = kth_device_count();
    if (ndev <= 0) return KTH_ENODEV;
    // distinct devices: RCCL, one rank per device; the same device repeated:
    // the local transport (any other repetition is refused)
    bool all_same = true, distinct = true;
    for (int i = 0; i < ngpu; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev) return KTH_EINVAL;
        all_same = all_same && devices[i] == devices[0];
        for (int j = 0; j < i; ++j) distinct = distinct && devices[j] != devices[i];
    }
    const bool local = ngpu > 1 && all_same;
    if (!local && !distinct) return KTH_EINVAL;
    if (local && ngpu > KTH_LOCAL_MAX_SHARDS) return KTH_EINVAL;
    if (!local && !rccl().ok) return KTH_ECOMM;
    kth_sharded *h = new kth_sharded();
    h->local = local;
    h->d.resize((size_t)ngpu);
    int rc = KTH_OK;
    std::vector<ncclComm_t> comms((size_t)ngpu, nullptr);
    for (int i = 0; i < ngpu && rc == KTH_OK; ++i) {
        Dev &x = h->d[(size_t)i];
        x.device = devices[i];
        if ((rc = kth_ctx_create(x.device, &x.ctx)) != KTH_OK) break;
        if (hipSetDevice(x.device) != hipSuccess) {
            rc = KTH_EHIP;
            break;
        }
        if (local && i > 0) {
            x.stream = h->d[0].stream;  // one stream for every shard of the device
        } else if (hipStreamCreateWithFlags(&x.stream, hipStreamNonBlocking) != hipSuccess) {
            rc = KTH_EHIP;
            break;
        } else {
            x.own_stream = true;
        }
        if ((rc = kth_ctx_set_stream(x.ctx, x.stream)) != KTH_OK) break;
        if (hipMalloc(reinterpret_cast<void **>(&x.slots), 3 * (size_t)KTH_STATS_WORDS * 8) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&x.out), 4) != hipSuccess) {
            rc = KTH_ENOMEM;
            break;
        }
    }
    if (rc == KTH_OK) {  // the answers' read-back buffer
        if (hipSetDevice(devices[0]) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&h->h_status), 2 * (size_t)ngpu * sizeof(int32_t),
                          hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void **>(&h->d_status), h->h_status, 0) != hipSuccess)
            rc = KTH_ENOMEM;
        // each device's own mapping of the (portable) words: no reliance on
        // one address serving every device
        for (size_t i = 0; rc == KTH_OK && i < h->d.size(); ++i) {
            Dev &x = h->d[i];
            if (hipSetDevice(x.device) != hipSuccess ||
                hipHostGetDevicePointer(reinterpret_cast<void **>(&x.d_status), h->h_status, 0) != hipSuccess)
                rc = KTH_EHIP;
        }
    }
    if (rc == KTH_OK && !local) {
        if (rccl().CommInitAll(comms.data(), ngpu, devices) != ncclSuccess)
            rc = KTH_ECOMM;
        else
            for (int i = 0; i < ngpu; ++i) h->d[(size_t)i].comm = comms[(size_t)i];
    }
    (void)hipGetLastError();
    if (rc != KTH_OK) {
        kth_sharded_destroy(h);
        return rc;
    }
    *out = h;
    return KTH_OK;
}

int64_t kth_sharded_sample_split(const int64_t *shard_n, int P, int64_t *s_dev) {
    if (!shard_n || !s_dev || P < 1) return KTH_EINVAL;
    int64_t n_total = 0;
    for (int i = 0; i < P; ++i) {
        if (shard_n[i] < 0) return KTH_EINVAL;
        n_total += shard_n[i];
    }
    if (n_total < 1) return KTH_EINVAL;
    // ~kth_dist_sample_size(n_total) sample keys in all, split over the shards
    // in proportion to their sizes (a multiple of 64 each, at least 64, at
    // most the shard rounded down to 64): the gathered sample is then ~uniform
    // over the union also for unbalanced shards, so the window is as good a
    // guess as one GPU's
    const int64_t s_want = kth_dist_sample_size(n_total);
    int64_t s_total = 0;
    for (int i = 0; i < P; ++i) {
        const double share = (double)s_want * (double)shard_n[i] / (double)n_total;
        int64_t si = std::max<int64_t>(64, (int64_t)share & ~int64_t(63));
        si = std::min<int64_t>(si, shard_n[i] & ~int64_t(63));
        s_dev[i] = si;
        s_total += si;
    }
    return s_total;
}

int kth_sharded_select_i32(kth_sharded *h, const int32_t *const *shards, const int64_t *shard_n, int64_t k,
                           int32_t *out) {
    if (!h || !shards || !shard_n || !out) return KTH_EINVAL;
    const int P = (int)h->d.size();
    int64_t n_total = 0, n_min = INT64_MAX;
    for (int i = 0; i < P; ++i) {
        if (shard_n[i] < 0 || (shard_n[i] > 0 && !shards[i])) return KTH_EINVAL;
        n_total += shard_n[i];
        n_min = std::min(n_min, shard_n[i]);
    }
    if (k < 1 || k > n_total) return KTH_EINVAL;
    if (n_min < SMALL_PER_GPU) return select_gathered(h, shards, shard_n, n_total, k, out);
    const auto t0 = std::chrono::steady_clock::now();

    // per-shard sample sizes (kth_sharded_sample_split); balanced shards give
    // every shard the same count and one all-gather, unequal counts are
    // gathered as one group of broadcasts (a gatherv) over RCCL
    std::vector<int64_t> s_dev((size_t)P), s_off((size_t)P + 1, 0);
    const int64_t s_total = kth_sharded_sample_split(shard_n, P, s_dev.data());
    TRY(s_total);
    bool equal = true;
    for (int i = 0; i < P; ++i) {
        s_off[(size_t)i + 1] = s_off[(size_t)i] + s_dev[(size_t)i];
        equal = equal && s_dev[(size_t)i] == s_dev[0];
    }
    if (h->local) {
        TRY(grow(h->d[0].device, reinterpret_cast<void **>(&h->lgathered), &h->lgathered_cap, s_total * 4));
    } else {
        for (int i = 0; i < P; ++i) {
            Dev &x = h->d[(size_t)i];
            TRY(grow(x.device, reinterpret_cast<void **>(&x.sample), &x.sample_cap, s_dev[(size_t)i] * 4));
            TRY(grow(x.device, reinterpret_cast<void **>(&x.gathered), &x.gathered_cap, s_total * 4));
        }
    }
    std::vector<uint64_t *> slot_bufs((size_t)P);
    for (int i = 0; i < P; ++i) slot_bufs[(size_t)i] = h->d[(size_t)i].slots;
    auto allreduce = [&](int slot) -> int {
        if (h->local) {  // one stream: every shard's step is complete before the sum runs
            HIPT(hipSetDevice(h->d[0].device));
            return kth_internal_slots_sum(slot_bufs.data(), P, slot, h->d[0].stream);
        }
        const Rccl &R = rccl();  // (the local transport never loads RCCL)
        NCCLT(R.GroupStart());
        for (Dev &x : h->d) {
            uint64_t *p = x.slots + (size_t)slot * KTH_STATS_WORDS;
            if (R.AllReduce(p, p, KTH_STATS_WORDS, ncclUint64, ncclSum, x.comm, x.stream) != ncclSuccess) {
                (void)R.GroupEnd();
                return KTH_ECOMM;
            }
        }
        NCCLT(R.GroupEnd());
        return KTH_OK;
    };
    // the samples: local -> straight into the shared gathered buffer at each
    // shard's offset; RCCL -> the shard's buffer, then an all-gather (or a
    // gatherv of broadcasts)
    for (int i = 0; i < P; ++i) {
        Dev &x = h->d[(size_t)i];
        uint32_t *dst = h->local ? h->lgathered + s_off[(size_t)i] : x.sample;
        TRY(kth_dist_begin(x.ctx, x.slots, n_total, k));
        TRY(kth_dist_sample(x.ctx, shards[i], shard_n[i], dst, s_dev[(size_t)i]));
    }
    if (!h->local) {
        const Rccl &R = rccl();
        NCCLT(R.GroupStart());
        for (int i = 0; i < P; ++i) {
            Dev &x = h->d[(size_t)i];
            ncclResult_t r = ncclSuccess;
            if (equal) {
                r = R.AllGather(x.sample, x.gathered, (size_t)s_dev[0], ncclUint32, x.comm, x.stream);
            } else {
                // (every rank passes its own sample as the send buffer; only the root's is read)
                for (int root = 0; root < P && r == ncclSuccess; ++root)
                    r = R.Broadcast(x.sample, x.gathered + s_off[(size_t)root], (size_t)s_dev[(size_t)root], ncclUint32,
                                    root, x.comm, x.stream);
            }
            if (r != ncclSuccess) {
                (void)R.GroupEnd();
                return KTH_ECOMM;
            }
        }
        NCCLT(R.GroupEnd());
    }
    // the window: on one device computed once and shared (every shard would
    // derive the same one from the same gathered sample)
    bool shared = false;
    if (h->local) {
        TRY(kth_dist_window(h->d[0].ctx, h->lgathered, s_total));
        std::vector<kth_ctx *> rest;
        for (int i = 1; i < P; ++i) rest.push_back(h->d[(size_t)i].ctx);
        const int r = kth_internal_dist_window_share(h->d[0].ctx, rest.data(), P - 1);
        TRY(r);
        shared = r == KTH_OK;
    }
    int slot = -1;
    for (int i = 0; i < P; ++i) {
        Dev &x = h->d[(size_t)i];
        if (!(shared || (h->local && i == 0)))
            TRY(kth_dist_window(x.ctx, h->local ? h->lgathered : x.gathered, s_total));
        const int r = kth_dist_scan(x.ctx, shards[i], shard_n[i]);
        TRY(r);
        slot = r;
    }
    TRY(allreduce(slot));
    // the levels, until every shard says KTH_DIST_DONE (they agree: the same
    // reduced slots); usually one level, so two all-reduces in all
    for (int l = 0;; ++l) {
        for (int i = 0; i < P; ++i) {
            const int r = kth_dist_level(h->d[(size_t)i].ctx, shards[i], shard_n[i], l);
            TRY(r);
            if (i > 0 && r != slot) return KTH_EINTERNAL;
            slot = r;
        }
        if (slot == KTH_DIST_DONE) break;
        TRY(allreduce(slot));
    }
    for (Dev &x : h->d) TRY(kth_dist_result(x.ctx, x.out));
    // every shard's [answer, error] to the host in one gather per device and
    // one wait each (a per-shard stats read and copy took ~2 round trips a shard)
    if (h->local) {
        std::vector<kth_ctx *> ctxs;
        for (Dev &x : h->d) ctxs.push_back(x.ctx);
        TRY(kth_internal_status_gather(ctxs.data(), P, h->d_status, h->d[0].stream));
    } else {
        for (int i = 0; i < P; ++i) {
            Dev &x = h->d[(size_t)i];
            TRY(kth_internal_status_gather(&x.ctx, 1, x.d_status + 2 * i, x.stream));
        }
    }
    h->enqueue_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    for (Dev &x : h->d) {
        if (h->local && &x != &h->d[0]) continue;  // (one shared stream)
        HIPT(hipSetDevice(x.device));
        HIPT(hipStreamSynchronize(x.stream));
    }
    // every shard must hold the same answer (they picked the same digits from
    // the same reduced histograms); the per-shard error words must be clear
    const volatile int32_t *hs = h->h_status;
    for (int i = 0; i < P; ++i) {
        if (hs[2 * i + 1] != 0) return KTH_EINTERNAL;
        if (hs[2 * i] != hs[0]) return KTH_EINTERNAL;
    }
    *out = hs[0];
    return KTH_OK;
}

double kth_sharded_enqueue_us(const kth_sharded *h) { return h ? h->enqueue_us : -1.0; }

// One-shot form: shard i's device from its pointer; the handle (RCCL
// communicators, per-device ctx and scratch) is kept per host thread and
// reused while the device list stays the same.
int kth_select_i32_sharded(const int32_t *const *dev_shards, const int64_t *shard_n, int ngpu, int64_t k,
                           int32_t *out) {
    static thread_local kth_sharded *cached = nullptr;
    static thread_local std::vector<int> cached_devs;
    if (!dev_shards || !shard_n || !out || ngpu < 1) return KTH_EINVAL;
    if (kth_device_count() <= 0) return KTH_ENODEV;
    std::vector<int> devs((size_t)ngpu);
    for (int i = 0; i < ngpu; ++i) {
        if (!dev_shards[i]) return KTH_EINVAL;
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, dev_shards[i]) != hipSuccess) {
            (void)hipGetLastError();
            return KTH_EINVAL;
        }
        if (at.type != hipMemoryTypeDevice) return KTH_EINVAL;  // device memory only
        devs[(size_t)i] = at.device;
    }
    if (!cached || cached_devs != devs) {
        if (cached) kth_sharded_destroy(cached);
        cached = nullptr;
        cached_devs.clear();
        TRY(kth_sharded_create(devs.data(), ngpu, &cached));
        cached_devs = devs;
    }
    return kth_sharded_select_i32(cached, dev_shards, shard_n, k, out);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// One sharded selection over the caller's RCCL communicator, one call: the
// kth_dist_* steps of this rank with the collectives in between, all on the
// ctx stream.  A scripted caller (kselect.dist) paid one host round trip per
// step through its bindings -- ~18 us of device idle a select at world size
// 1, the host's path from its wait on level 0 to the next select's first
// launch (profiles/r5_dist_early_result.txt) -- which this call removes.
extern "C" int kth_dist_select_rccl(kth_ctx *ctx, void *nccl_all_reduce, void *nccl_all_gather, void *nccl_comm,
                                    int world, const int32_t *d_keys, int64_t n_local, int64_t n_total, int64_t k,
                                    uint64_t *d_slots, uint32_t *d_sample, uint32_t *d_gathered, int64_t s_local,
                                    int32_t *d_out, int early) {
    using AllReduceFn = ncclResult_t (*)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                         hipStream_t);
    using AllGatherFn = ncclResult_t (*)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    if (!ctx || !nccl_all_reduce || !nccl_all_gather || !nccl_comm || world < 1 || !d_keys || !d_slots ||
        !d_sample || !d_gathered || !d_out || s_local < 64)
        return KTH_EINVAL;
    const auto all_reduce = reinterpret_cast<AllReduceFn>(nccl_all_reduce);
    const auto all_gather = reinterpret_cast<AllGatherFn>(nccl_all_gather);
    const auto comm = reinterpret_cast<ncclComm_t>(nccl_comm);
    const auto stream = reinterpret_cast<hipStream_t>(kth_internal_ctx_stream(ctx));
    auto reduce = [&](int slot) -> int {
        uint64_t *p = d_slots + (size_t)slot * KTH_STATS_WORDS;
        NCCLT(all_reduce(p, p, KTH_STATS_WORDS, ncclUint64, ncclSum, comm, stream));
        return KTH_OK;
    };
    TRY(kth_dist_begin(ctx, d_slots, n_total, k));
    TRY(kth_dist_sample(ctx, d_keys, n_local, d_sample, s_local));
    NCCLT(all_gather(d_sample, d_gathered, (size_t)s_local, ncclUint32, comm, stream));
    TRY(kth_dist_window(ctx, d_gathered, s_local * world));
    int slot = kth_dist_scan(ctx, d_keys, n_local);
    TRY(slot);
    TRY(reduce(slot));
    for (int l = 0;; ++l) {  // usually one level: two all-reduces in all
        if (l > KTH_DIST_MAX_LEVELS) return KTH_EINTERNAL;
        if (l == 1 && early) TRY(kth_dist_result_early(ctx, d_out));  // before level 1 waits for level 0
        slot = kth_dist_level(ctx, d_keys, n_local, l);
        TRY(slot);
        if (slot == KTH_DIST_DONE) break;
        TRY(reduce(slot));
    }
    return kth_dist_result(ctx, d_out);
}
