// bloom_capi.cpp — the C ABI of include/bloomhip.h: filter handles, stream
// ordering, host staging, strategy selection and per-kernel timing around
// the gfx950 kernels of bloom_kernels.hip.
//
// Reference surface replaced (jackdent/cs265-lsm-tree):
//   BloomFilter(long)      src/bloom_filter.h:12      -> bloomhip_create
//   set(KEY_t)             src/bloom_filter.cpp:49-53 -> bloomhip_set_batch / bloomhip_set
//   is_set(KEY_t) const    src/bloom_filter.cpp:55-59 -> bloomhip_test_batch / bloomhip_is_set
//   Run::Run sizing        src/run.cpp:13-15          -> bloomhip_m_bits
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <utility>
#include <vector>

#include "../../include/bloomhip.h"
#include "bloom_kernels.h"
#include "bloom_merge.h"

using namespace bloomhip;

namespace {

thread_local std::string g_last_error;

// One spin-wait step of the host polls below: the x86 pause hint, the
// AArch64 yield hint, nothing elsewhere.
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#elif defined(__aarch64__)
    __builtin_arm_yield();
#endif
}

int fail_hip(hipError_t e, const char *what) {
    g_last_error = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    if (e == hipErrorOutOfMemory) return BLOOMHIP_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return BLOOMHIP_ENODEV;
    return BLOOMHIP_EIO;
}

#define HIP_TRY(expr)                                       \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return fail_hip(_e, #expr);   \
    } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == dev) {  // common case: nothing to switch or restore
            prev = -1;
            ok = true;
            return;
        }
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

enum ProfSlot {
    SLOT_CLEAR = 0,
    SLOT_ATOMIC = 1,
    SLOT_LDS = 2,
    SLOT_PART_BIN = 3,
    SLOT_PART_APPLY = 4,
    SLOT_PROBE = 5,
    SLOT_PROBE_PART = 6,
    SLOT_COPY = 7,
    SLOT_PROBE_LDS = 8,
    SLOT_PROBE_STACK = 9,
    SLOT_PROBE_STACK_ROUTE = 10,  // a stacked probe with GET routing fused into its combine
    SLOT_ROUTE = 11,              // k_route after the probes (routing not fused)
};
const char *kSlotNames[BLOOMHIP_PROF_SLOTS] = {
    "clear(memset)", "k_build_atomic", "k_build_lds",       "k_part_bin", "k_part_apply",
    "k_probe",       "probe_partitioned", "copy",           "k_probe_lds",  "probe_stacked",
    "probe_stacked+route", "k_route",
};

struct PendingTiming {
    int slot;
    hipEvent_t a, b;
};

}  // namespace

struct bloomhip_filter {
    int device = 0;
    uint64_t m = 0;
    uint64_t nwords64 = 0;
    uint32_t *d_words = nullptr;
    hipStream_t stream = nullptr;
    ModParams mp{};
    int strategy = BLOOMHIP_BUILD_AUTO;
    int probe_strategy = BLOOMHIP_PROBE_AUTO;
    bool known_zero = true;      // host-side knowledge that every bit is 0
    bool pending_clear = false;  // cleared, but the memset is not issued yet

    std::mutex mu;  // guards staging, workspace and profiling state
    void *d_stage = nullptr;
    size_t stage_bytes = 0;
    void *d_out_stage = nullptr;
    size_t out_stage_bytes = 0;

    // run metadata (§8f rows 1, 4): d_meta[0] = max key, d_meta[1..nfences]
    // = fence pointers; set by bloomhip_set_batch_run / bloomhip_set_run_meta
    int32_t *d_meta = nullptr;
    size_t meta_bytes = 0;
    uint32_t nfences = 0;
    void *d_route_stage = nullptr;  // first/page staging for host outputs
    size_t route_stage_bytes = 0;
    // bloomhip_is_set's answer: a pinned host word mapped into the device
    // (allocated on the first scalar call)
    uint32_t *h_hit = nullptr;
    uint32_t *d_hit = nullptr;

    bool prof = false;
    uint64_t prof_launches[BLOOMHIP_PROF_SLOTS] = {};
    double prof_ms[BLOOMHIP_PROF_SLOTS] = {};
    std::vector<PendingTiming> pending;
    std::vector<hipEvent_t> spare_events;
};

namespace {

// Locks the distinct handles of a multi-filter call in one global order (by
// address) and releases them in reverse, so concurrent calls over the same
// filters in different orders ([a, b] and [b, a]) cannot deadlock.
class HandleLocks {
   public:
    HandleLocks(const bloomhip_filter *const *fs, int n) {
        for (int i = 0; i < n; i++) hs_.push_back(const_cast<bloomhip_filter *>(fs[i]));
        std::sort(hs_.begin(), hs_.end(), std::less<bloomhip_filter *>());
        hs_.erase(std::unique(hs_.begin(), hs_.end()), hs_.end());
        for (bloomhip_filter *h : hs_) h->mu.lock();
    }
    ~HandleLocks() {
        for (auto it = hs_.rbegin(); it != hs_.rend(); ++it) (*it)->mu.unlock();
    }
    HandleLocks(const HandleLocks &) = delete;
    HandleLocks &operator=(const HandleLocks &) = delete;

   private:
    std::vector<bloomhip_filter *> hs_;
};

// NULL is HIP's default (null) stream, as everywhere in HIP: work given no
// stream is ordered with the caller's other default-stream work (e.g. a torch
// copy on its default stream).
hipStream_t pick_stream(const bloomhip_filter *, void *stream) {
    return reinterpret_cast<hipStream_t>(stream);
}

hipError_t grow(void **ptr, size_t *have, size_t need) {
    if (*have >= need) return hipSuccess;
    if (*ptr) {
        hipError_t e = hipFree(*ptr);
        if (e != hipSuccess) return e;
        *ptr = nullptr;
        *have = 0;
    }
    size_t sz = std::max<size_t>(need, 1 << 20);
    hipError_t e = hipMalloc(ptr, sz);
    if (e == hipSuccess) *have = sz;
    return e;
}

// Grows *ptr to >= need bytes; a fresh allocation is written once on `s` so
// its pages are mapped before a kernel's first touch (a first build on fresh
// 200 MB of workspace otherwise ran 100x slower).
hipError_t grow_touched(void **ptr, size_t *have, size_t need, hipStream_t s) {
    if (*have >= need) return hipSuccess;
    hipError_t e = grow(ptr, have, need);
    if (e == hipSuccess) e = hipMemsetAsync(*ptr, 0, *have, s);
    return e;
}

// Scratch of the partition build / partitioned probe.  Shared by every handle
// that runs on the same (device, stream): work on one stream is ordered, so
// one set of buffers serves all of it, allocated (and first touched) once.
// Lock order everywhere: filter handle(s) first, then a workspace; g_ws_mu
// (the map) is only ever held alone (workspace_for, bloomhip_trim), never
// while a workspace lock is taken, so a compaction that holds its workspace
// across the build of its output run's filter cannot deadlock with trim.  The
// workspace lock is recursive: that build takes it again (run_partition).
// Callers hold a shared_ptr, so a workspace that bloomhip_trim drops from
// the map stays alive until its last user is done with it; trim frees its
// buffers under its lock and marks it retired, and a caller that locks a
// retired workspace (it looked it up before trim took the map) looks up the
// current one instead (LockedWorkspace), so no buffer is ever regrown in a
// workspace that has left the map (it would never be freed).
struct Workspace {
    std::recursive_mutex mu;  // held while work using the buffers is enqueued
    bool retired = false;     // dropped from the map by bloomhip_trim (mu held)
    uint64_t *pos = nullptr;  // tile-sorted packed entries
    size_t pos_bytes = 0;
    uint32_t *runs = nullptr;  // run starts: tile-major rows, then segment-major
    size_t runs_bytes = 0;
    uint8_t *res = nullptr;  // partitioned probe: result byte per sorted entry
    size_t res_bytes = 0;
    uint16_t *slots = nullptr;  // partitioned probe: sorted slot per (key, hash)
    size_t slots_bytes = 0;
    void *mbuf[2] = {nullptr, nullptr};  // compaction: merge rounds ping-pong
    size_t mbuf_bytes[2] = {0, 0};
    uint64_t *msplit = nullptr;  // compaction: merge-path splits
    size_t msplit_bytes = 0;
    uint32_t *mcount = nullptr;  // compaction: block counts / offsets
    size_t mcount_bytes = 0;
    int32_t *mkeys = nullptr;  // compaction: the merged run's kept keys, packed
    size_t mkeys_bytes = 0;
    void *kway = nullptr;  // one-pass compaction: samples, partition bounds, look-back state
    size_t kway_bytes = 0;
    uint32_t *h_kept = nullptr;  // one-pass compaction: kept count, pinned + mapped (coherent)
    uint32_t *d_kept = nullptr;  // its device address
};

std::mutex g_ws_mu;
std::map<std::pair<int, hipStream_t>, std::shared_ptr<Workspace>> g_ws;

std::shared_ptr<Workspace> workspace_for(int device, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto &w = g_ws[{device, s}];
    if (!w) w = std::make_shared<Workspace>();
    return w;
}

// The (device, stream) workspace, locked and live: a workspace that
// bloomhip_trim retired between the lookup and the lock is let go and the
// lookup repeated (trim has replaced the map by then, so this terminates).
struct LockedWorkspace {
    std::shared_ptr<Workspace> w;
    std::unique_lock<std::recursive_mutex> lk;
    LockedWorkspace(int device, hipStream_t s) {
        for (;;) {
            w = workspace_for(device, s);
            lk = std::unique_lock<std::recursive_mutex>(w->mu);
            if (!w->retired) return;
            lk.unlock();
        }
    }
    Workspace *operator->() const { return w.get(); }
    Workspace *get() const { return w.get(); }
};

// Frees a workspace's buffers (its lock held by the caller; the stream's
// queued work that uses them is waited for first).
void free_workspace_buffers(int device, hipStream_t s, Workspace *w) {
    DeviceGuard g(device);
    (void)hipStreamSynchronize(s);
    for (void **p : {(void **)&w->pos, (void **)&w->runs, (void **)&w->res, (void **)&w->slots,
                     &w->mbuf[0], &w->mbuf[1], (void **)&w->msplit, (void **)&w->mcount,
                     (void **)&w->mkeys, &w->kway}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    if (w->h_kept) (void)hipHostFree(w->h_kept);
    w->h_kept = w->d_kept = nullptr;
    w->pos_bytes = w->runs_bytes = w->res_bytes = w->slots_bytes = 0;
    w->mbuf_bytes[0] = w->mbuf_bytes[1] = w->msplit_bytes = w->mcount_bytes = w->mkeys_bytes = 0;
    w->kway_bytes = 0;
}

hipEvent_t take_event(bloomhip_filter *f) {
    if (!f->spare_events.empty()) {
        hipEvent_t e = f->spare_events.back();
        f->spare_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Runs `launch` on `s`, bracketed by events when profiling is enabled.
template <class F>
hipError_t timed(bloomhip_filter *f, int slot, hipStream_t s, F &&launch) {
    if (!f->prof) return launch();
    hipEvent_t a = take_event(f), b = take_event(f);
    if (!a || !b) return launch();
    (void)hipEventRecord(a, s);
    hipError_t e = launch();
    (void)hipEventRecord(b, s);
    f->pending.push_back({slot, a, b});
    return e;
}

int harvest_profile(bloomhip_filter *f) {
    for (auto &p : f->pending) {
        HIP_TRY(hipEventSynchronize(p.b));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
        f->prof_ms[p.slot] += ms;
        f->prof_launches[p.slot] += 1;
        f->spare_events.push_back(p.a);
        f->spare_events.push_back(p.b);
    }
    f->pending.clear();
    return BLOOMHIP_OK;
}

int classify_keys(const void *keys, size_t stride, int *layout) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(keys);
    if (stride < 4 || stride % 4 != 0 || (a & 3)) return BLOOMHIP_EINVAL;
    if (stride == 4 && (a & 15) == 0) *layout = KEYS_PACKED;
    else if (stride == 8 && (a & 15) == 0) *layout = KEYS_ENTRY;
    else *layout = KEYS_STRIDED;
    return BLOOMHIP_OK;
}

// Device-resident view of `n` keys: the caller's buffer, or a copy of a host
// buffer into the handle's staging area (enqueued on s).
int device_keys(bloomhip_filter *f, const void *keys, size_t n, size_t stride, int on_device,
                hipStream_t s, KeySpan *out) {
    int layout = 0;
    if (n && !keys) return BLOOMHIP_EINVAL;
    if (stride < 4 || stride % 4) return BLOOMHIP_EINVAL;
    const void *dev = keys;
    if (!on_device && n) {
        const size_t bytes = (n - 1) * stride + 4;
        HIP_TRY(grow(&f->d_stage, &f->stage_bytes, bytes));
        int rc = timed(f, SLOT_COPY, s, [&] {
            return hipMemcpyAsync(f->d_stage, keys, bytes, hipMemcpyHostToDevice, s);
        });
        if (rc != hipSuccess) return fail_hip((hipError_t)rc, "hipMemcpyAsync(keys H2D)");
        dev = f->d_stage;
    }
    if (n) {
        int rc = classify_keys(dev, stride, &layout);
        if (rc) return rc;
    }
    *out = KeySpan{reinterpret_cast<const char *>(dev), n, stride, layout};
    return BLOOMHIP_OK;
}

bool partition_able(const bloomhip_filter *f) {
    PartitionWorkspace ws{};
    return plan_segments(f->m, device_cu_count(), &ws);
}

int resolve_strategy(const bloomhip_filter *f, size_t n) {
    if (f->strategy != BLOOMHIP_BUILD_AUTO) return f->strategy;
    const uint64_t bytes = (f->m + 7) / 8;
    if (bytes <= kLdsBitmapBytes) {
        // Worth a private LDS copy once the batch outweighs the merge.
        return n >= (size_t)(f->m / 64) ? BLOOMHIP_BUILD_LDS : BLOOMHIP_BUILD_ATOMIC;
    }
    // The partition build pays two passes over 8 B/key; below ~64K keys a
    // direct atomic build is cheaper.
    if (n >= (1u << 16) && partition_able(f)) return BLOOMHIP_BUILD_PARTITION;
    return BLOOMHIP_BUILD_ATOMIC;
}

int strategy_supported(const bloomhip_filter *f, int strategy) {
    switch (strategy) {
        case BLOOMHIP_BUILD_ATOMIC: return 1;
        case BLOOMHIP_BUILD_LDS: return f->mp.fast && (f->m + 7) / 8 <= kLdsBitmapBytes;
        case BLOOMHIP_BUILD_PARTITION: return partition_able(f);
        default: return 0;
    }
}

// A partition pass over n keys with the segment geometry in *ws (from
// plan_segments / plan_stack): the position/run buffers of `w` grown to fit.
int partition_buffers(Workspace *w, size_t n, hipStream_t s, PartitionWorkspace *ws_inout) {
    PartitionWorkspace ws = *ws_inout;
    if (ws.tile_keys == 0) ws.tile_keys = choose_tile_keys(ws.nbins);
    ws.ntiles = (n + ws.tile_keys - 1) / ws.tile_keys;
    HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->pos), &w->pos_bytes,
                         ws.ntiles * (size_t)ws.tile_keys * 8, s));
    const size_t table = ws.ntiles * (ws.nbins + 1);  // run starts, both layouts
    HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->runs), &w->runs_bytes, table * 2 * 4, s));
    ws.pos = w->pos;
    ws.run_rows = w->runs;
    ws.run_starts = w->runs + table;
    *ws_inout = ws;
    return BLOOMHIP_OK;
}

// Geometry of a partition pass over n keys for filter size m, with the
// position/run buffers of `w` grown to fit.
int partition_workspace(Workspace *w, uint64_t m, size_t n, hipStream_t s,
                        PartitionWorkspace *out, bool build = false) {
    PartitionWorkspace ws{};
    if (!(build ? plan_build(m, device_cu_count(), &ws) : plan_segments(m, device_cu_count(), &ws)))
        return BLOOMHIP_ERANGE;
    *out = ws;
    return partition_buffers(w, n, s, out);
}

// The partitioned probe's result bytes and slots, grown to fit ws.
int probe_buffers(Workspace *w, const PartitionWorkspace &ws, hipStream_t s) {
    HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->res), &w->res_bytes,
                         ws.ntiles * (size_t)ws.tile_keys * 3, s));
    HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->slots), &w->slots_bytes,
                         ws.ntiles * 3 * (size_t)ws.tile_keys * sizeof(uint16_t), s));
    return BLOOMHIP_OK;
}

bool lds_probe_able(const bloomhip_filter *f) {
    return f->mp.fast && f->nwords64 * 8 <= kLdsBitmapBytes;
}

// How filter f is probed in a batch of n keys: its own strategy, else the
// batch owner's, else AUTO.  A strategy that cannot apply to f (LDS for a
// filter larger than LDS, PARTITION for m >= 2^32) falls back to gathers.
int probe_kind(const bloomhip_filter *f, int owner_strategy, size_t n) {
    const int st = f->probe_strategy != BLOOMHIP_PROBE_AUTO ? f->probe_strategy : owner_strategy;
    if (st == BLOOMHIP_PROBE_PARTITION)
        return partition_able(f) ? BLOOMHIP_PROBE_PARTITION : BLOOMHIP_PROBE_GATHER;
    if (st == BLOOMHIP_PROBE_LDS)
        return lds_probe_able(f) ? BLOOMHIP_PROBE_LDS : BLOOMHIP_PROBE_GATHER;
    if (st == BLOOMHIP_PROBE_GATHER) return BLOOMHIP_PROBE_GATHER;
    // AUTO (and STACKED for a filter no stack took) (tools/probe_sweep.py): LDS-sized filters from LDS
    // once the batch amortises the staging; gathers while the filter mostly
    // hits in L2 / MALL; beyond that the partitioned probe.
    if (lds_probe_able(f) && n >= kProbeLdsMinKeys) return BLOOMHIP_PROBE_LDS;
    if (partition_able(f) && (f->m + 7) / 8 > kProbeGatherMaxBytes &&
        n >= kProbePartitionMinKeys)
        return BLOOMHIP_PROBE_PARTITION;
    return BLOOMHIP_PROBE_GATHER;
}

// Issues a clear() that was deferred (see bloomhip_clear) on stream s.
int materialize_clear(bloomhip_filter *f, hipStream_t s) {
    if (!f->pending_clear) return BLOOMHIP_OK;
    hipError_t e = timed(f, SLOT_CLEAR, s,
                         [&] { return hipMemsetAsync(f->d_words, 0, f->nwords64 * 8, s); });
    if (e != hipSuccess) return fail_hip(e, "hipMemsetAsync(bitmap)");
    f->pending_clear = false;
    return BLOOMHIP_OK;
}

int run_partition(bloomhip_filter *f, const KeySpan &ks, hipStream_t s) {
    const LockedWorkspace w(f->device, s);
    PartitionWorkspace ws{};
    int rc = partition_workspace(w.get(), f->m, ks.n, s, &ws, /*build=*/true);
    if (rc) return rc;
    hipError_t e = timed(f, SLOT_PART_BIN, s, [&] { return launch_part_bin(ks, f->mp, ws, s); });
    if (e != hipSuccess) return fail_hip(e, "k_part_bin");
    const int merge = f->known_zero ? 0 : 1;
    e = timed(f, SLOT_PART_APPLY, s,
              [&] { return launch_part_apply(f->mp, f->d_words, ws, merge, s); });
    if (e != hipSuccess) return fail_hip(e, "k_part_apply");
    return BLOOMHIP_OK;
}

}  // namespace

extern "C" {

int bloomhip_abi_version(void) { return BLOOMHIP_ABI_VERSION; }

#ifndef BLOOMHIP_KERNEL_SHA
#define BLOOMHIP_KERNEL_SHA "unknown"
#endif
const char *bloomhip_kernel_sha(void) { return BLOOMHIP_KERNEL_SHA; }

const char *bloomhip_strerror(int status) {
    switch (status) {
        case BLOOMHIP_OK: return "ok";
        case BLOOMHIP_EIO: return "HIP runtime error";
        case BLOOMHIP_ENOMEM: return "out of device memory";
        case BLOOMHIP_ENODEV: return "no such device";
        case BLOOMHIP_EINVAL: return "invalid argument";
        case BLOOMHIP_ERANGE: return "size out of supported range";
        default: return "unknown status";
    }
}

const char *bloomhip_last_error(void) { return g_last_error.c_str(); }

int bloomhip_device_count(int *count) {
    g_last_error.clear();
    if (!count) return BLOOMHIP_EINVAL;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail_hip(e, "hipGetDeviceCount");
    }
    *count = n;
    return BLOOMHIP_OK;
}

int bloomhip_m_bits(int64_t max_size, float bits_per_entry, uint64_t *m_out) {
    g_last_error.clear();
    // Run::Run: bloom_filter(max_size * bf_bits_per_entry) — long * float is a
    // float product, truncated to long by BloomFilter(long).  src/run.cpp:13-15
    if (!m_out) return BLOOMHIP_EINVAL;
    const float f = (float)max_size * bits_per_entry;
    if (std::isnan(f) || f < 1.0f) return BLOOMHIP_EINVAL;  // reference: m==0 -> SIGFPE
    if (f >= 9.2233720368547758e18f) return BLOOMHIP_ERANGE;
    *m_out = (uint64_t)(int64_t)f;
    return BLOOMHIP_OK;
}

int bloomhip_create(int device, uint64_t m_bits, bloomhip_filter **out) {
    g_last_error.clear();
    if (!out || m_bits == 0) return BLOOMHIP_EINVAL;
    *out = nullptr;
    if (m_bits > (1ull << 46)) return BLOOMHIP_ERANGE;  // 8 TiB of bits: beyond one GPU
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return BLOOMHIP_ENODEV;
    DeviceGuard g(device);
    if (!g.ok) return fail_hip(hipErrorInvalidDevice, "hipSetDevice");
    auto *f = new bloomhip_filter();
    f->device = device;
    f->m = m_bits;
    f->nwords64 = (m_bits + 63) / 64;
    f->mp = make_mod_params(m_bits);
    hipError_t e = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&f->d_words, f->nwords64 * 8);
    if (e == hipSuccess) e = hipMemsetAsync(f->d_words, 0, f->nwords64 * 8, f->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
    if (e != hipSuccess) {
        int rc = fail_hip(e, "bloomhip_create");
        if (f->d_words) (void)hipFree(f->d_words);
        if (f->stream) (void)hipStreamDestroy(f->stream);
        delete f;
        return rc;
    }
    *out = f;
    return BLOOMHIP_OK;
}

int bloomhip_destroy(bloomhip_filter *f) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    (void)hipStreamSynchronize(f->stream);
    for (auto &p : f->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : f->spare_events) (void)hipEventDestroy(e);
    if (f->d_words) (void)hipFree(f->d_words);
    if (f->d_stage) (void)hipFree(f->d_stage);
    if (f->d_out_stage) (void)hipFree(f->d_out_stage);
    if (f->d_meta) (void)hipFree(f->d_meta);
    if (f->d_route_stage) (void)hipFree(f->d_route_stage);
    if (f->h_hit) (void)hipHostFree(f->h_hit);
    (void)hipStreamDestroy(f->stream);
    delete f;
    return BLOOMHIP_OK;
}

int bloomhip_size(const bloomhip_filter *f, uint64_t *m_out) {
    g_last_error.clear();
    if (!f || !m_out) return BLOOMHIP_EINVAL;
    *m_out = f->m;
    return BLOOMHIP_OK;
}

int bloomhip_nwords(const bloomhip_filter *f, uint64_t *nwords_out) {
    g_last_error.clear();
    if (!f || !nwords_out) return BLOOMHIP_EINVAL;
    *nwords_out = f->nwords64;
    return BLOOMHIP_OK;
}

int bloomhip_device(const bloomhip_filter *f, int *device_out) {
    g_last_error.clear();
    if (!f || !device_out) return BLOOMHIP_EINVAL;
    *device_out = f->device;
    return BLOOMHIP_OK;
}

int bloomhip_device_words(const bloomhip_filter *f, void **dptr_out) {
    g_last_error.clear();
    if (!f || !dptr_out) return BLOOMHIP_EINVAL;
    {
        // A deferred clear is issued on the default stream before the raw
        // pointer is handed out.
        bloomhip_filter *fm = const_cast<bloomhip_filter *>(f);
        DeviceGuard g(f->device);
        std::lock_guard<std::mutex> lk(fm->mu);
        int rc = materialize_clear(fm, nullptr);
        if (rc) return rc;
    }
    *dptr_out = f->d_words;
    return BLOOMHIP_OK;
}

int bloomhip_stream(const bloomhip_filter *f, void **stream_out) {
    g_last_error.clear();
    if (!f || !stream_out) return BLOOMHIP_EINVAL;
    *stream_out = f->stream;
    return BLOOMHIP_OK;
}

int bloomhip_clear(bloomhip_filter *f, void *stream) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    std::lock_guard<std::mutex> lk(f->mu);
    (void)stream;
    // Deferred: a partition build overwrites every segment, so a clear that
    // is followed by one needs no memset.  Anything else that touches the
    // bitmap first issues the memset on its own stream (materialize_clear).
    f->pending_clear = true;
    f->known_zero = true;
    return BLOOMHIP_OK;
}

namespace {

// The build of keys ks into f on stream s (f->mu held).
int build_locked(bloomhip_filter *f, const KeySpan &ks, size_t n, hipStream_t s) {
    const int strategy = resolve_strategy(f, n);
    if (!strategy_supported(f, strategy)) return BLOOMHIP_EINVAL;
    int rc;
    if (strategy == BLOOMHIP_BUILD_PARTITION && f->pending_clear) {
        f->pending_clear = false;  // pass 2 writes every word with merge = 0
    } else {
        rc = materialize_clear(f, s);
        if (rc) return rc;
    }
    hipError_t e = hipSuccess;
    switch (strategy) {
        case BLOOMHIP_BUILD_LDS:
            e = timed(f, SLOT_LDS, s, [&] { return launch_build_lds(ks, f->mp, f->d_words, s); });
            break;
        case BLOOMHIP_BUILD_PARTITION:
            rc = run_partition(f, ks, s);
            if (rc) return rc;
            break;
        default:
            e = timed(f, SLOT_ATOMIC, s,
                      [&] { return launch_build_atomic(ks, f->mp, f->d_words, s); });
            break;
    }
    if (e != hipSuccess) return fail_hip(e, "build kernel launch");
    f->known_zero = false;
    return BLOOMHIP_OK;
}

// Room for a run's metadata: max key + ceil(n / kFenceStride) fences.
int meta_reserve(bloomhip_filter *f, size_t nfences) {
    return grow(reinterpret_cast<void **>(&f->d_meta), &f->meta_bytes, (nfences + 1) * 4) ==
                   hipSuccess
               ? BLOOMHIP_OK
               : fail_hip(hipErrorOutOfMemory, "run metadata allocation");
}

}  // namespace

int bloomhip_set_batch(bloomhip_filter *f, const void *keys, size_t n, size_t stride_bytes,
                       int keys_on_device, void *stream) {
    if (!f) return BLOOMHIP_EINVAL;
    if (n == 0) return BLOOMHIP_OK;
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    hipStream_t s = pick_stream(f, stream);
    KeySpan ks{};
    int rc = device_keys(f, keys, n, stride_bytes, keys_on_device, s, &ks);
    if (rc) return rc;
    rc = build_locked(f, ks, n, s);
    if (rc) return rc;
    if (!keys_on_device) HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

namespace {

// bloomhip_set_batch_run with f->mu held and f's device current.
// sorted: the caller guarantees keys ascending (a compaction's output), so the
// max key is the last one and only the fence keys need reading.
int set_batch_run_locked(bloomhip_filter *f, const void *keys, size_t n, size_t stride_bytes,
                         int keys_on_device, hipStream_t s, bool sorted = false) {
    KeySpan ks{};
    int rc = device_keys(f, keys, n, stride_bytes, keys_on_device, s, &ks);
    if (rc) return rc;
    if (n) {
        rc = build_locked(f, ks, n, s);
        if (rc) return rc;
    }
    const size_t nf = (n + kFenceStride - 1) / kFenceStride;
    if (nf > 0xFFFFFFFFull) return BLOOMHIP_ERANGE;
    rc = meta_reserve(f, nf);
    if (rc) return rc;
    hipError_t e = sorted ? launch_run_meta_sorted(ks, f->d_meta, s) : launch_run_meta(ks, f->d_meta, s);
    if (e != hipSuccess) return fail_hip(e, "k_run_meta launch");
    f->nfences = (uint32_t)nf;
    if (!keys_on_device) HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

}  // namespace

int bloomhip_set_batch_run(bloomhip_filter *f, const void *keys, size_t n, size_t stride_bytes,
                           int keys_on_device, void *stream) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    return set_batch_run_locked(f, keys, n, stride_bytes, keys_on_device, pick_stream(f, stream));
}

int bloomhip_set_run_meta(bloomhip_filter *f, const int32_t *fences, size_t nfences,
                          int32_t max_key) {
    g_last_error.clear();
    if (!f || (nfences && !fences) || nfences > 0xFFFFFFFFull) return BLOOMHIP_EINVAL;
    for (size_t i = 1; i < nfences; i++)
        if (fences[i] < fences[i - 1]) return BLOOMHIP_EINVAL;  // a run is written sorted
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    int rc = meta_reserve(f, nfences);
    if (rc) return rc;
    std::vector<int32_t> h(nfences + 1);
    h[0] = max_key;
    for (size_t i = 0; i < nfences; i++) h[1 + i] = fences[i];
    HIP_TRY(hipMemcpy(f->d_meta, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    f->nfences = (uint32_t)nfences;
    return BLOOMHIP_OK;
}

int bloomhip_get_run_meta(const bloomhip_filter *f, int32_t *fences, size_t cap,
                          size_t *nfences_out, int32_t *max_key_out) {
    g_last_error.clear();
    if (!f || !nfences_out) return BLOOMHIP_EINVAL;
    bloomhip_filter *fm = const_cast<bloomhip_filter *>(f);
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(fm->mu);
    *nfences_out = f->nfences;
    if (!f->d_meta) {
        if (max_key_out) *max_key_out = INT32_MIN;
        return BLOOMHIP_OK;
    }
    if (fences && cap < f->nfences) return BLOOMHIP_ERANGE;
    std::vector<int32_t> h(f->nfences + 1);
    HIP_TRY(hipDeviceSynchronize());  // the metadata may come from any stream
    HIP_TRY(hipMemcpy(h.data(), f->d_meta, h.size() * 4, hipMemcpyDeviceToHost));
    if (max_key_out) *max_key_out = h[0];
    if (fences)
        for (size_t i = 0; i < f->nfences; i++) fences[i] = h[1 + i];
    return BLOOMHIP_OK;
}

namespace {

// Device time of probing one filter alone, and of one stacked pass, in us
// per 2^24 keys on MI355X (C3's level filters, tools/probe_sweep.py): what
// AUTO weighs before stacking a group.
constexpr double kCostLds = 70, kCostGatherL2 = 125, kCostGatherFar = 530, kCostPartition = 250,
                 kCostStacked = 230, kCostLadder = 170;

double probe_cost_alone(const bloomhip_filter *f, size_t n) {
    switch (probe_kind(f, BLOOMHIP_PROBE_AUTO, n)) {
        case BLOOMHIP_PROBE_LDS: return kCostLds;
        case BLOOMHIP_PROBE_PARTITION: return kCostPartition;
        default: return (f->m + 7) / 8 <= kProbeGatherMaxBytes ? kCostGatherL2 : kCostGatherFar;
    }
}

int effective_probe_strategy(const bloomhip_filter *f, int owner_strategy) {
    return f->probe_strategy != BLOOMHIP_PROBE_AUTO ? f->probe_strategy : owner_strategy;
}

// Stacked probes (BLOOMHIP_PROBE_STACKED, kernels.h StackTable) for the
// groups of filters that take one; marks their rows in `done`.  Largest
// filter first: its group is every not-yet-taken filter whose m divides its
// m (largest first, <= kMaxStack).  A group with an explicit STACKED member
// always runs; an AUTO group runs when it beats its members' own probes.
// route (optional): GET routing to fuse into the combine of a stack that
// takes every filter of the call (bloomhip_route_gets); *routed says whether
// it was.
struct FusedRoute {
    const RouteTable *rt;
    RouteOut out;
    bool routed;
};

int probe_stacks(bloomhip_filter *f0, const bloomhip_filter *const *filters, int nf,
                 const KeySpan &ks, size_t n, uint64_t *dout, hipStream_t s,
                 std::vector<char> &done, FusedRoute *route = nullptr) {
    std::vector<int> cand;
    for (int j = 0; j < nf; j++) {
        const int st = effective_probe_strategy(filters[j], f0->probe_strategy);
        if (filters[j]->mp.fast && (st == BLOOMHIP_PROBE_AUTO || st == BLOOMHIP_PROBE_STACKED))
            cand.push_back(j);
    }
    std::stable_sort(cand.begin(), cand.end(),
                     [&](int a, int b) { return filters[a]->m > filters[b]->m; });
    const int ncu = device_cu_count();
    const size_t nw = (n + 63) / 64;
    for (size_t a = 0; a < cand.size(); a++) {
        const int h = cand[a];
        if (done[h]) continue;
        const uint64_t mh = filters[h]->m;
        std::vector<int> mem{h};
        for (size_t b = a + 1; b < cand.size() && mem.size() < (size_t)kMaxStack; b++)
            if (!done[cand[b]] && mh % filters[cand[b]]->m == 0) mem.push_back(cand[b]);
        bool explicit_stack = false;
        uint64_t g = 0, mmin = ~0ull;
        double alone = 0;
        for (int j : mem) {
            mmin = std::min(mmin, filters[j]->m);
            explicit_stack |= effective_probe_strategy(filters[j], f0->probe_strategy) ==
                              BLOOMHIP_PROBE_STACKED;
            g = std::gcd(g, filters[j]->m);
            alone += probe_cost_alone(filters[j], n);
        }
        // A ladder (members d << t_j: an LSM's levels at a power-of-two
        // fanout) bins by hash bits, else segments of m_max.
        PartitionWorkspace ws{};
        StackTable st{};
        uint64_t msz[kMaxStack];
        for (size_t k = 0; k < mem.size(); k++) msz[k] = filters[mem[k]]->m;
        const bool ladder = plan_ladder(msz, (int)mem.size(), ncu, &st, &ws);
        if (!ladder && !plan_stack(mh, g, mmin, (int)mem.size(), ncu, &ws)) continue;
        if (!explicit_stack && (mem.size() < 2 || n < kProbePartitionMinKeys ||
                                ws.nbins < (size_t)ncu ||
                                alone <= (ladder ? kCostLadder : kCostStacked)))
            continue;
        st.nf = (int)mem.size();
        for (int k = 0; k < st.nf; k++) {
            st.words[k] = filters[mem[k]]->d_words;
            st.mwords[k] = (uint32_t)(filters[mem[k]]->m / 32);
            st.row[k] = mem[k];
        }
        // every filter of a routing call in this one stack: the routing runs
        // in its combine (k_probe_combine_route), not in k_route afterwards
        const bool fuse = route && (int)mem.size() == nf && route->rt->nruns == nf &&
                          (size_t)route->rt->total_fences * 4 <= kRouteLdsFenceBytesMax;
        // (The fused combine on super-tiles stages 48 KiB of result bytes per
        // tile, which with the f = 10 tree's fences leaves one workgroup per
        // CU; round 5 routed such stacks on 8192-key tiles instead, 0.351
        // against 0.387 ms. Since the combine's range check reads one window
        // per member (round 6), super-tiles route that tree faster: 0.3126 ->
        // 0.3093 ms, profiles/r06/route_super_tiles/.)
        const LockedWorkspace w(f0->device, s);
        int rc = partition_buffers(w.get(), n, s, &ws);
        if (rc) return rc;
        rc = probe_buffers(w.get(), ws, s);
        if (rc) return rc;
        hipError_t e = timed(f0, fuse ? SLOT_PROBE_STACK_ROUTE : SLOT_PROBE_STACK, s, [&] {
            return fuse ? launch_probe_stacked(ks, filters[h]->mp, st, ws, w->res, w->slots, dout, nw, s,
                                               route->rt, route->out)
                        : launch_probe_stacked(ks, filters[h]->mp, st, ws, w->res, w->slots, dout, nw, s);
        });
        if (fuse && e == hipSuccess) route->routed = true;
        if (e != hipSuccess) return fail_hip(e, "stacked probe launch");
        for (int j : mem) done[j] = 1;
    }
    return BLOOMHIP_OK;
}

// is_set rows of every filter for keys ks into dout (nf x ceil(n/64)), on s
// (f0->mu held, clears materialised).
int probe_rows(bloomhip_filter *f0, const bloomhip_filter *const *filters, int nf,
               const KeySpan &ks, size_t n, uint64_t *dout, hipStream_t s,
               FusedRoute *route = nullptr) {
    const size_t nw = (n + 63) / 64;
    // Groups of stacked levels first: one partitioned pass each.
    std::vector<char> done((size_t)nf, 0);
    int rc = probe_stacks(f0, filters, nf, ks, n, dout, s, done, route);
    if (rc) return rc;
    // Then, one filter at a time: small filters from LDS, large ones
    // partitioned; the rest: gathers, up to kMaxProbeFilters per launch.
    std::vector<int> gather_idx;
    for (int j = 0; j < nf; j++) {
        if (done[j]) continue;
        const int kind = probe_kind(filters[j], f0->probe_strategy, n);
        if (kind == BLOOMHIP_PROBE_GATHER) {
            gather_idx.push_back(j);
            continue;
        }
        if (kind == BLOOMHIP_PROBE_LDS) {
            hipError_t e = timed(f0, SLOT_PROBE_LDS, s, [&] {
                return launch_probe_lds(ks, filters[j]->mp, filters[j]->d_words,
                                        dout + (size_t)j * nw, nw, s);
            });
            if (e != hipSuccess) return fail_hip(e, "k_probe_lds launch");
            continue;
        }
        const LockedWorkspace w(f0->device, s);
        PartitionWorkspace ws{};
        rc = partition_workspace(w.get(), filters[j]->m, n, s, &ws);
        if (rc) return rc;
        rc = probe_buffers(w.get(), ws, s);
        if (rc) return rc;
        hipError_t e = timed(f0, SLOT_PROBE_PART, s, [&] {
            return launch_probe_partitioned(ks, filters[j]->mp, filters[j]->d_words, ws, w->res,
                                            w->slots, dout + (size_t)j * nw, s);
        });
        if (e != hipSuccess) return fail_hip(e, "partitioned probe launch");
    }
    for (size_t j0 = 0; j0 < gather_idx.size();) {
        // one launch per run of consecutive output rows (<= kMaxProbeFilters)
        ProbeTable t{};
        const int row0 = gather_idx[j0];
        size_t j1 = j0;
        while (j1 < gather_idx.size() && j1 - j0 < (size_t)kMaxProbeFilters &&
               gather_idx[j1] == row0 + (int)(j1 - j0)) {
            t.words[j1 - j0] = filters[gather_idx[j1]]->d_words;
            t.mp[j1 - j0] = filters[gather_idx[j1]]->mp;
            j1++;
        }
        t.nf = (int)(j1 - j0);
        hipError_t e = timed(f0, SLOT_PROBE, s,
                             [&] { return launch_probe(ks, t, dout + (size_t)row0 * nw, nw, s); });
        if (e != hipSuccess) return fail_hip(e, "k_probe launch");
        j0 = j1;
    }
    return BLOOMHIP_OK;
}

// Deferred clears of every filter, issued on s (every handle's lock held).
int materialize_all(const bloomhip_filter *const *filters, int nf, hipStream_t s) {
    for (int j = 0; j < nf; j++) {
        int rc = materialize_clear(const_cast<bloomhip_filter *>(filters[j]), s);
        if (rc) return rc;
    }
    return BLOOMHIP_OK;
}

}  // namespace

int bloomhip_test_batch(const bloomhip_filter *const *filters, int nf, const void *keys, size_t n,
                        size_t stride_bytes, int keys_on_device, uint64_t *out_packed,
                        int out_on_device, void *stream) {
    if (!filters || nf <= 0 || !out_packed) return BLOOMHIP_EINVAL;
    for (int j = 0; j < nf; j++)
        if (!filters[j] || filters[j]->device != filters[0]->device) return BLOOMHIP_EINVAL;
    if (n == 0) return BLOOMHIP_OK;
    // Staging and profiling state live on the first handle.
    bloomhip_filter *f0 = const_cast<bloomhip_filter *>(filters[0]);
    DeviceGuard g(f0->device);
    HandleLocks locks(filters, nf);
    hipStream_t s = pick_stream(f0, stream);
    KeySpan ks{};
    int rc = device_keys(f0, keys, n, stride_bytes, keys_on_device, s, &ks);
    if (rc) return rc;
    rc = materialize_all(filters, nf, s);
    if (rc) return rc;
    const size_t nw = (n + 63) / 64;
    const size_t out_bytes = (size_t)nf * nw * 8;
    uint64_t *dout = out_packed;
    if (!out_on_device) {
        HIP_TRY(grow(&f0->d_out_stage, &f0->out_stage_bytes, out_bytes));
        dout = reinterpret_cast<uint64_t *>(f0->d_out_stage);
    }
    rc = probe_rows(f0, filters, nf, ks, n, dout, s);
    if (rc) return rc;
    if (!out_on_device) {
        hipError_t e = timed(f0, SLOT_COPY, s, [&] {
            return hipMemcpyAsync(out_packed, dout, out_bytes, hipMemcpyDeviceToHost, s);
        });
        if (e != hipSuccess) return fail_hip(e, "hipMemcpyAsync(results D2H)");
    }
    if (!keys_on_device || !out_on_device) HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

namespace {

// bloomhip_route_gets and bloomhip_route_gets_packed: the candidate rows and
// either first / page or their packed form (each output optional).
int route_impl(const bloomhip_filter *const *runs, int nruns, const void *keys, size_t n,
               size_t stride_bytes, int keys_on_device, uint64_t *cand_packed, int32_t *first_run,
               int32_t *page, uint32_t *packed, int out_on_device, void *stream) {
    g_last_error.clear();
    if (!runs || nruns <= 0 || nruns > kMaxRouteRuns) return BLOOMHIP_EINVAL;
    if (packed && nruns > kRoutePackedMaxRuns) return BLOOMHIP_EINVAL;
    for (int j = 0; j < nruns; j++)
        if (!runs[j] || runs[j]->device != runs[0]->device) return BLOOMHIP_EINVAL;
    if (n == 0) return BLOOMHIP_OK;
    bloomhip_filter *f0 = const_cast<bloomhip_filter *>(runs[0]);
    DeviceGuard g(f0->device);
    HandleLocks locks(runs, nruns);
    hipStream_t s = pick_stream(f0, stream);
    KeySpan ks{};
    int rc = device_keys(f0, keys, n, stride_bytes, keys_on_device, s, &ks);
    if (rc) return rc;
    rc = materialize_all(runs, nruns, s);
    if (rc) return rc;
    RouteTable t{};
    t.nruns = nruns;
    uint32_t off = 0;
    for (int j = 0; j < nruns; j++) {
        bloomhip_filter *fj = const_cast<bloomhip_filter *>(runs[j]);
        if (!fj->d_meta) {  // no metadata: never a candidate
            rc = meta_reserve(fj, 0);
            if (rc) return rc;
            fj->nfences = 0;
        }
        t.meta[j] = fj->d_meta;
        t.nfences[j] = fj->nfences;
        t.fence_off[j] = off;
        off += fj->nfences;
    }
    t.total_fences = off;
    const size_t nw = (n + 63) / 64;
    const size_t cand_bytes = (size_t)nruns * nw * 8;
    uint64_t *dcand = out_on_device ? cand_packed : nullptr;
    if (!dcand) {
        HIP_TRY(grow(&f0->d_out_stage, &f0->out_stage_bytes, cand_bytes));
        dcand = reinterpret_cast<uint64_t *>(f0->d_out_stage);
    }
    RouteOut ro{};
    if (out_on_device) {
        ro = RouteOut{first_run, page, packed};
    } else if (first_run || page || packed) {
        HIP_TRY(grow(&f0->d_route_stage, &f0->route_stage_bytes, n * 8));
        int32_t *stage = reinterpret_cast<int32_t *>(f0->d_route_stage);
        ro.first = first_run ? stage : nullptr;
        ro.page = page ? stage + n : nullptr;
        ro.packed = packed ? reinterpret_cast<uint32_t *>(stage) : nullptr;
    }
    FusedRoute fr{&t, ro, false};
    rc = probe_rows(f0, runs, nruns, ks, n, dcand, s, &fr);
    if (rc) return rc;
    if (!fr.routed) {  // the filters were probed apart: route over their rows
        hipError_t e = timed(f0, SLOT_ROUTE, s, [&] { return launch_route(ks, t, dcand, nw, ro, s); });
        if (e != hipSuccess) return fail_hip(e, "k_route launch");
    }
    if (!out_on_device) {
        if (cand_packed)
            HIP_TRY(hipMemcpyAsync(cand_packed, dcand, cand_bytes, hipMemcpyDeviceToHost, s));
        if (first_run)
            HIP_TRY(hipMemcpyAsync(first_run, ro.first, n * 4, hipMemcpyDeviceToHost, s));
        if (page) HIP_TRY(hipMemcpyAsync(page, ro.page, n * 4, hipMemcpyDeviceToHost, s));
        if (packed) HIP_TRY(hipMemcpyAsync(packed, ro.packed, n * 4, hipMemcpyDeviceToHost, s));
    }
    if (!keys_on_device || !out_on_device) HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

}  // namespace

int bloomhip_route_gets(const bloomhip_filter *const *runs, int nruns, const void *keys, size_t n,
                        size_t stride_bytes, int keys_on_device, uint64_t *cand_packed,
                        int32_t *first_run, int32_t *page, int out_on_device, void *stream) {
    return route_impl(runs, nruns, keys, n, stride_bytes, keys_on_device, cand_packed, first_run, page,
                      nullptr, out_on_device, stream);
}

int bloomhip_route_gets_packed(const bloomhip_filter *const *runs, int nruns, const void *keys,
                               size_t n, size_t stride_bytes, int keys_on_device,
                               uint64_t *cand_packed, uint32_t *route, int out_on_device,
                               void *stream) {
    return route_impl(runs, nruns, keys, n, stride_bytes, keys_on_device, cand_packed, nullptr,
                      nullptr, route, out_on_device, stream);
}

int bloomhip_set(bloomhip_filter *f, int32_t key) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    hipStream_t s = nullptr;  // HIP's default stream, ordered with the caller's other work
    int rc = materialize_clear(f, s);
    if (rc) return rc;
    hipError_t e = launch_set1(f->d_words, f->mp, key, s);
    if (e != hipSuccess) return fail_hip(e, "k_set1 launch");
    f->known_zero = false;
    HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

int bloomhip_is_set(const bloomhip_filter *fc, int32_t key, int *hit_out) {
    g_last_error.clear();
    if (!fc || !hit_out) return BLOOMHIP_EINVAL;
    bloomhip_filter *f = const_cast<bloomhip_filter *>(fc);
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    if (!f->h_hit) {
        // fine-grained (coherent) and mapped: the kernel's system-scope store
        // is visible to the host spin below without a stream synchronisation
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&f->h_hit), 64,
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&f->d_hit), f->h_hit, 0));
    }
    hipStream_t s = nullptr;
    int rc = materialize_clear(f, s);
    if (rc) return rc;
    *reinterpret_cast<volatile uint32_t *>(f->h_hit) = 2u;  // overwritten by the kernel
    hipError_t e = launch_is_set1(f->d_words, f->mp, key, f->d_hit, s);
    if (e != hipSuccess) return fail_hip(e, "k_is_set1 launch");
    // The kernel's last act is the answer's system-scope store, so once the
    // word changes the kernel is done: spin on it (cheaper than the stream
    // synchronisation's wake-up) for up to kIsSetSpin, then synchronise,
    // which also reports a kernel that failed.
    constexpr std::chrono::microseconds kIsSetSpin{1000};
    volatile uint32_t *hv = reinterpret_cast<volatile uint32_t *>(f->h_hit);
    const auto t0 = std::chrono::steady_clock::now();
    while (*hv == 2u && std::chrono::steady_clock::now() - t0 < kIsSetSpin) cpu_relax();
    // (A hipStreamQuery after a successful spin, to report a kernel fault at
    // once, made the call 12.0 us median against 8.7 without it, bench
    // scalar_is_set; a fault is sticky and surfaces at the next synchronising
    // call on this filter instead.)
    if (*hv == 2u) HIP_TRY(hipStreamSynchronize(s));
    const uint32_t v = *hv;
    if (v > 1u) return fail_hip(hipErrorUnknown, "k_is_set1 result not visible");
    *hit_out = (int)v;
    return BLOOMHIP_OK;
}

int bloomhip_download(const bloomhip_filter *f, uint64_t *words, size_t nwords, void *stream) {
    g_last_error.clear();
    if (!f || !words || nwords != f->nwords64) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    hipStream_t s = pick_stream(f, stream);
    {
        bloomhip_filter *fm = const_cast<bloomhip_filter *>(f);
        std::lock_guard<std::mutex> lk(fm->mu);
        int rc = materialize_clear(fm, s);
        if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(words, f->d_words, nwords * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return BLOOMHIP_OK;
}

int bloomhip_upload(bloomhip_filter *f, const uint64_t *words, size_t nwords, void *stream) {
    g_last_error.clear();
    if (!f || !words || nwords != f->nwords64) return BLOOMHIP_EINVAL;
    const unsigned tail = (unsigned)(f->m % 64);
    if (tail && (words[nwords - 1] >> tail) != 0) return BLOOMHIP_EINVAL;  // bits >= m
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    hipStream_t s = pick_stream(f, stream);
    HIP_TRY(hipMemcpyAsync(f->d_words, words, nwords * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    f->pending_clear = false;
    f->known_zero = false;
    return BLOOMHIP_OK;
}

int bloomhip_clone(const bloomhip_filter *src, int device, bloomhip_filter **out) {
    g_last_error.clear();
    if (!src || !out) return BLOOMHIP_EINVAL;
    *out = nullptr;
    bloomhip_filter *f = nullptr;
    int rc = bloomhip_create(device, src->m, &f);
    if (rc) return rc;
    bloomhip_filter *sm = const_cast<bloomhip_filter *>(src);
    {
        DeviceGuard gs(src->device);
        std::lock_guard<std::mutex> lk(sm->mu);
        // the source's queued work may be on any stream: wait for the device
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess && !sm->pending_clear) {
            // xGMI peer copy between devices, a D2D copy on one device
            e = src->device == device
                    ? hipMemcpy(f->d_words, src->d_words, src->nwords64 * 8,
                                hipMemcpyDeviceToDevice)
                    : hipMemcpyPeer(f->d_words, device, src->d_words, src->device,
                                    src->nwords64 * 8);
        }
        if (e == hipSuccess && src->d_meta) {
            std::vector<int32_t> h(src->nfences + 1);
            e = hipMemcpy(h.data(), src->d_meta, h.size() * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess) {
                f->known_zero = sm->pending_clear || sm->known_zero;
                f->strategy = src->strategy;
                f->probe_strategy = src->probe_strategy;
                rc = bloomhip_set_run_meta(f, h.data() + 1, src->nfences, h[0]);
            }
        } else if (e == hipSuccess) {
            f->known_zero = sm->pending_clear || sm->known_zero;
            f->strategy = src->strategy;
            f->probe_strategy = src->probe_strategy;
        }
        if (e != hipSuccess) rc = fail_hip(e, "bloomhip_clone copy");
    }
    if (rc) {
        (void)bloomhip_destroy(f);
        return rc;
    }
    if (!f->known_zero) {
        DeviceGuard gd(device);
        HIP_TRY(hipDeviceSynchronize());
    }
    *out = f;
    return BLOOMHIP_OK;
}

int bloomhip_sync(const bloomhip_filter *f, void *stream) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    HIP_TRY(hipStreamSynchronize(pick_stream(f, stream)));
    return BLOOMHIP_OK;
}

int bloomhip_set_strategy(bloomhip_filter *f, int strategy) {
    g_last_error.clear();
    if (!f || strategy < BLOOMHIP_BUILD_AUTO || strategy > BLOOMHIP_BUILD_PARTITION)
        return BLOOMHIP_EINVAL;
    if (strategy != BLOOMHIP_BUILD_AUTO && !strategy_supported(f, strategy)) return BLOOMHIP_EINVAL;
    std::lock_guard<std::mutex> lk(f->mu);
    f->strategy = strategy;
    return BLOOMHIP_OK;
}

int bloomhip_set_probe_strategy(bloomhip_filter *f, int strategy) {
    g_last_error.clear();
    if (!f || strategy < BLOOMHIP_PROBE_AUTO || strategy > BLOOMHIP_PROBE_STACKED)
        return BLOOMHIP_EINVAL;
    std::lock_guard<std::mutex> lk(f->mu);
    f->probe_strategy = strategy;
    return BLOOMHIP_OK;
}

int bloomhip_resolve_strategy(const bloomhip_filter *f, size_t n, int *strategy_out) {
    g_last_error.clear();
    if (!f || !strategy_out) return BLOOMHIP_EINVAL;
    *strategy_out = resolve_strategy(f, n);
    return BLOOMHIP_OK;
}

int bloomhip_profile_enable(bloomhip_filter *f, int enable) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    std::lock_guard<std::mutex> lk(f->mu);
    f->prof = enable != 0;
    return BLOOMHIP_OK;
}

int bloomhip_profile_read(bloomhip_filter *f, int slot, const char **name_out,
                          uint64_t *launches_out, double *ms_out) {
    if (!f || slot < 0 || slot >= BLOOMHIP_PROF_SLOTS) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    int rc = harvest_profile(f);
    if (rc) return rc;
    if (name_out) *name_out = kSlotNames[slot];
    if (launches_out) *launches_out = f->prof_launches[slot];
    if (ms_out) *ms_out = f->prof_ms[slot];
    return BLOOMHIP_OK;
}

int bloomhip_profile_reset(bloomhip_filter *f) {
    g_last_error.clear();
    if (!f) return BLOOMHIP_EINVAL;
    DeviceGuard g(f->device);
    std::lock_guard<std::mutex> lk(f->mu);
    int rc = harvest_profile(f);
    for (int i = 0; i < BLOOMHIP_PROF_SLOTS; i++) {
        f->prof_ms[i] = 0.0;
        f->prof_launches[i] = 0;
    }
    return rc;
}

int bloomhip_trim(void) {
    g_last_error.clear();
    // Take the map's entries out under g_ws_mu alone, then free each
    // workspace's buffers under its own lock (the global lock order: never
    // a workspace lock inside g_ws_mu).  A call that already holds one of
    // them finishes first; one that starts later gets a fresh workspace.
    std::map<std::pair<int, hipStream_t>, std::shared_ptr<Workspace>> taken;
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        taken.swap(g_ws);
    }
    for (auto &kv : taken) {
        Workspace *w = kv.second.get();
        std::lock_guard<std::recursive_mutex> wl(w->mu);
        free_workspace_buffers(kv.first.first, kv.first.second, w);
        w->retired = true;  // a late user looks up the map's current one
    }
    return BLOOMHIP_OK;
}

constexpr uint32_t kKeptPending = 0xFFFFFFFFu;  // never a count: total < 2^32 - 1

int bloomhip_compact(const void *const *runs, const size_t *nentries, int nruns,
                     int runs_on_device, int drop_tombstones, void *out_entries, size_t *n_out,
                     int out_on_device, bloomhip_filter *f, int device, void *stream) {
    g_last_error.clear();
    if (nruns < 0 || (nruns && (!runs || !nentries)) || !n_out || (f && f->device != device))
        return BLOOMHIP_EINVAL;
    uint64_t total = 0;
    for (int r = 0; r < nruns; r++) {
        if (nentries[r] && !runs[r]) return BLOOMHIP_EINVAL;
        total += nentries[r];
    }
    if (total >= 0xFFFFFFFFull) return BLOOMHIP_ERANGE;  // 32-bit block offsets
    if (total && !out_entries) return BLOOMHIP_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return BLOOMHIP_ENODEV;
    if (device < 0 || device >= ndev) return BLOOMHIP_EINVAL;
    DeviceGuard g(device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint64_t kept = 0;
    {
        // The merged run lives in the shared workspace (mbuf) until its filter
        // is built and it is copied out, so the workspace stays locked until
        // then (filter first, then workspace: the global lock order).
        std::unique_lock<std::mutex> flk;
        if (f) flk = std::unique_lock<std::mutex>(f->mu);
        const LockedWorkspace w(device, s);
        // + one entry of padding per run: merge outputs start 16-B aligned
        const size_t bytes = (std::max<uint64_t>(total, 1) + (uint64_t)nruns + 2) * 8;
        for (int i = 0; i < 2; i++) HIP_TRY(grow_touched(&w->mbuf[i], &w->mbuf_bytes[i], bytes, s));
        HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->msplit), &w->msplit_bytes,
                             merge_split_words(total) * 8, s));
        HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->mcount), &w->mcount_bytes,
                             compact_count_words(total) * 4 + 4, s));
        if (f)
            HIP_TRY(grow_touched(reinterpret_cast<void **>(&w->mkeys), &w->mkeys_bytes,
                                 std::max<uint64_t>(total, 1) * 4, s));
        // the runs, newest first; host runs are staged into mbuf[0]
        std::vector<std::pair<const char *, uint64_t>> list;
        uint64_t off = 0;
        for (int r = 0; r < nruns; r++) {
            if (!nentries[r]) continue;
            if (runs_on_device) {
                list.push_back({static_cast<const char *>(runs[r]), nentries[r]});
            } else {
                char *dst = static_cast<char *>(w->mbuf[0]) + off * 8;
                HIP_TRY(hipMemcpyAsync(dst, runs[r], nentries[r] * 8, hipMemcpyHostToDevice, s));
                list.push_back({dst, nentries[r]});
                off += nentries[r];
            }
        }
        if (!list.empty() && list.size() <= (size_t)kKwayMaxRuns) {
            // one pass: merge + newest-wins dedup + tombstones + packed keys
            // (bloom_merge.hip k_kway_*), into the caller's buffer or mbuf[1]
            const void *rp[kKwayMaxRuns];
            uint64_t rn[kKwayMaxRuns];
            const int k = (int)list.size();
            for (int r = 0; r < k; r++) {
                rp[r] = list[r].first;
                rn[r] = list[r].second;
            }
            HIP_TRY(grow_touched(&w->kway, &w->kway_bytes, kway_workspace_bytes(rn, k), s));
            if (!w->h_kept) {
                HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&w->h_kept), 64,
                                      hipHostMallocMapped | hipHostMallocCoherent));
                HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&w->d_kept), w->h_kept, 0));
            }
            volatile uint32_t *hk = w->h_kept;
            *hk = kKeptPending;  // overwritten by the merge's last partition
            void *dst = out_on_device ? out_entries : w->mbuf[1];
            hipError_t e = launch_compact_kway(rp, rn, k, drop_tombstones, dst, f ? w->mkeys : nullptr,
                                               w->kway, w->d_kept, s);
            if (e != hipSuccess) return fail_hip(e, "k-way compaction launch");
            // The kept count sizes the filter build.  The last partition
            // stores it (system scope) once every kept count before it is
            // known, while the merge may still be writing entries: the build
            // is enqueued on the same stream, so it runs after the merge
            // anyway, and the GPU does not idle through a copy + synchronise
            // round trip (0.457 ms per bench call with it).  The spin is
            // bounded (kKeptSpin, with a pause per poll): when the stream has
            // more queued ahead of the merge than that, the stream is
            // synchronised instead of holding a core (this also reports a
            // failed kernel).
            constexpr std::chrono::microseconds kKeptSpin{2000};
            const auto t0 = std::chrono::steady_clock::now();
            while (*hk == kKeptPending && std::chrono::steady_clock::now() - t0 < kKeptSpin)
                cpu_relax();
            if (*hk == kKeptPending) HIP_TRY(hipStreamSynchronize(s));
            kept = *hk;
            if (kept > total) return fail_hip(hipErrorUnknown, "k-way compaction count not visible");
            if (f) {
                int rc = kept ? set_batch_run_locked(f, w->mkeys, (size_t)kept, 4, 1, s, true)
                              : set_batch_run_locked(f, dst, 0, 8, 1, s, true);
                if (rc) return rc;
            }
            if (!out_on_device && kept)
                HIP_TRY(hipMemcpyAsync(out_entries, dst, kept * 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            *n_out = (size_t)kept;
            return BLOOMHIP_OK;
        }
        // more than kKwayMaxRuns runs: pairwise merge rounds, the left (newer)
        // input winning ties; round outputs alternate between the two
        // buffers, never the round's input; then the dedup pass
        int dst_buf = runs_on_device ? 0 : 1;
        while (list.size() > 1) {
            std::vector<std::pair<const char *, uint64_t>> next;
            char *base = static_cast<char *>(w->mbuf[dst_buf]);
            uint64_t o = 0;
            // the round's merges go out together (one split + one tile
            // launch per kMaxMergePairs pairs)
            std::vector<MergePairArgs> pairs;
            for (size_t i = 0; i < list.size(); i += 2) {
                char *dst = base + o * 8;
                if (i + 1 < list.size()) {
                    pairs.push_back({list[i].first, list[i].second, list[i + 1].first,
                                     list[i + 1].second, dst});
                    next.push_back({dst, list[i].second + list[i + 1].second});
                } else {
                    HIP_TRY(hipMemcpyAsync(dst, list[i].first, list[i].second * 8,
                                           hipMemcpyDeviceToDevice, s));
                    next.push_back({dst, list[i].second});
                }
                o += (next.back().second + 1) & ~1ull;  // every output 16-B aligned
            }
            for (size_t p0 = 0; p0 < pairs.size(); p0 += kMaxMergePairs) {
                const int np = (int)std::min<size_t>(kMaxMergePairs, pairs.size() - p0);
                hipError_t e = launch_merge_round(pairs.data() + p0, np, w->msplit, s);
                if (e != hipSuccess) return fail_hip(e, "merge launch");
            }
            list.swap(next);
            dst_buf ^= 1;
        }
        // newest entry per key, tombstones dropped on request
        const char *merged = list.empty() ? nullptr : list[0].first;
        void *dst = out_on_device ? out_entries : w->mbuf[merged == w->mbuf[0] ? 1 : 0];
        if (merged) {
            // with a filter to build, the kept keys also go out packed: the
            // build's pass 1 then reads 4 B per key, not the 8-B entries
            hipError_t e = launch_dedup(merged, total, drop_tombstones, dst, w->mcount, s,
                                        f ? w->mkeys : nullptr);
            if (e != hipSuccess) return fail_hip(e, "dedup launch");
            uint32_t cnt = 0;
            HIP_TRY(hipMemcpyAsync(&cnt, w->mcount + compact_count_words(total) - 1, 4,
                                   hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            kept = cnt;
        }
        if (f) {
            // the merged run is sorted by key: fences and max key directly
            int rc = kept ? set_batch_run_locked(f, w->mkeys, (size_t)kept, 4, 1, s, true)
                          : set_batch_run_locked(f, dst, 0, 8, 1, s, true);
            if (rc) return rc;
        }
        if (!out_on_device && kept)
            HIP_TRY(hipMemcpyAsync(out_entries, dst, kept * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *n_out = (size_t)kept;
    return BLOOMHIP_OK;
}

int bloomhip_host_positions(uint64_t m, const int32_t *keys, size_t n, uint64_t *out) {
    g_last_error.clear();
    if (m == 0 || (n && (!keys || !out))) return BLOOMHIP_EINVAL;
    const ModParams mp = make_mod_params(m);
    for (size_t i = 0; i < n; i++) positions3(keys[i], mp, out + 3 * i);
    return BLOOMHIP_OK;
}

}  // extern "C"
