/*
 * bloomhip.h — C ABI of the MI355X (gfx950) Bloom-filter engine.
 *
 * Drop-in for the set/test surface of jackdent/cs265-lsm-tree
 * src/bloom_filter.{h,cpp}:
 *
 *   class BloomFilter {                       src/bloom_filter.h:6-15
 *       boost::dynamic_bitset<> table;        src/bloom_filter.h:7
 *       uint64_t hash_1/2/3(KEY_t) const;     src/bloom_filter.h:8-10, .cpp:8-47
 *     public:
 *       BloomFilter(long length);             src/bloom_filter.h:12
 *       void set(KEY_t);                      src/bloom_filter.cpp:49-53
 *       bool is_set(KEY_t) const;             src/bloom_filter.cpp:55-59
 *   };
 *
 * and for its sizing in Run::Run (src/run.cpp:13-15).  Results are bit-exact
 * with the reference: the same bitmap (dynamic_bitset block layout, bit i in
 * 64-bit block i/64 at bit i%64) after the same keys are set, and the same
 * is_set booleans.  k = 3 with the reference's three fixed hashes.
 *
 * Conventions
 *   - Plain C types only; `void *stream` is a hipStream_t, NULL meaning HIP's
 *     default (null) stream as in every HIP API.  No HIP or torch headers are
 *     needed to bind this ABI.
 *   - Every entry point returns an int status: 0 on success, a negative
 *     errno-style code on failure; nothing throws across the ABI.  The
 *     reference has no error path at all (m == 0 is a SIGFPE there,
 *     src/bloom_filter.cpp:19); here m == 0 is rejected with BLOOMHIP_EINVAL.
 *   - A handle owns one device bitmap on one device.  Calls on a handle are
 *     ordered on the stream they are given; different handles may be driven
 *     from different host threads (one per GPU for per-run sharding).
 *   - Device-resident calls (keys_on_device = 1, out_on_device = 1) are
 *     asynchronous.  A call given any HOST buffer synchronises the stream
 *     before it returns, so host buffers may be reused immediately (the
 *     reference's calls are synchronous, src/run.cpp:93,162).
 *   - Keys are KEY_t = int32_t (src/types.h:4) read at `stride_bytes`
 *     (4 for a packed key vector, 8 for entry_t runs, src/types.h:14-22).
 */
#ifndef BLOOMHIP_H
#define BLOOMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLOOMHIP_ABI_VERSION 1

#define BLOOMHIP_OK 0
#define BLOOMHIP_EIO (-5)     /* HIP runtime error; see bloomhip_last_error() */
#define BLOOMHIP_ENOMEM (-12) /* device allocation failed */
#define BLOOMHIP_ENODEV (-19) /* no such device / no GPU */
#define BLOOMHIP_EINVAL (-22) /* bad argument (m == 0, NULL, bad stride...) */
#define BLOOMHIP_ERANGE (-34) /* size out of supported range */

/* Build strategies for bloomhip_set_batch (bloomhip_set_strategy). */
#define BLOOMHIP_BUILD_AUTO 0      /* pick by m and n (default) */
#define BLOOMHIP_BUILD_ATOMIC 1    /* one pass, global atomicOr per bit */
#define BLOOMHIP_BUILD_LDS 2       /* private LDS bitmap per workgroup (m/8 <= LDS) */
#define BLOOMHIP_BUILD_PARTITION 3 /* hash+bin pass, then LDS segment pass */

/* Probe strategies for bloomhip_test_batch (bloomhip_set_probe_strategy). */
#define BLOOMHIP_PROBE_AUTO 0      /* LDS for LDS-sized filters, gather up to 8 MiB, else partition */
#define BLOOMHIP_PROBE_GATHER 1    /* per-key gathers of the 3 bits */
#define BLOOMHIP_PROBE_PARTITION 2 /* bin positions by segment, test in LDS */
#define BLOOMHIP_PROBE_LDS 3       /* whole filter staged in each workgroup's LDS (m/8 <= 160 KiB) */
/* One partitioned pass for up to 8 filters whose sizes all divide the largest
 * one's (x % m_j == (x % m_max) % m_j): an LSM's stacked levels, where run
 * capacities grow by the fanout (src/lsm_tree.cpp:36-41).  AUTO picks it for
 * such groups when it beats probing the members one by one. */
#define BLOOMHIP_PROBE_STACKED 4

typedef struct bloomhip_filter bloomhip_filter;

int bloomhip_abi_version(void);
/* Digest of the kernel sources this library was compiled from (first 16 hex
 * digits of SHA-256 over csrc/bloom_kernels.hip, bloom_kernels.h,
 * bloom_math.h): measurement tools tie profiles to the kernels that ran. */
const char *bloomhip_kernel_sha(void);
const char *bloomhip_strerror(int status);
/* Text of the last HIP error seen by this host thread ("" if none). */
const char *bloomhip_last_error(void);
int bloomhip_device_count(int *count);

/* m = (long)((float)max_size * bits_per_entry): Run::Run's sizing of its
 * filter, evaluated in float exactly as src/run.cpp:13-15 does. */
int bloomhip_m_bits(int64_t max_size, float bits_per_entry, uint64_t *m_out);

/* BloomFilter(long length): an all-zero filter of m_bits bits on `device`.
 * src/bloom_filter.h:12.  m_bits must be >= 1. */
int bloomhip_create(int device, uint64_t m_bits, bloomhip_filter **out);
int bloomhip_destroy(bloomhip_filter *f);

/* table.size() (src/bloom_filter.cpp:19) and the number of 64-bit blocks. */
int bloomhip_size(const bloomhip_filter *f, uint64_t *m_out);
int bloomhip_nwords(const bloomhip_filter *f, uint64_t *nwords_out);
int bloomhip_device(const bloomhip_filter *f, int *device_out);
/* Device address of the bitmap (ceil(m/64) uint64 blocks), for zero-copy
 * interop.  Valid until bloomhip_destroy.  A deferred clear is issued on the
 * default stream first. */
int bloomhip_device_words(const bloomhip_filter *f, void **dptr_out);
/* A non-blocking stream owned by the handle, for callers that want the
 * filter's work off the default stream (pass it as `stream`). */
int bloomhip_stream(const bloomhip_filter *f, void **stream_out);

/* Reset every bit to 0.  The memset is deferred: a following partition
 * build overwrites every word anyway, and any other use of the bitmap issues
 * it first on that use's stream. */
int bloomhip_clear(bloomhip_filter *f, void *stream);

/* BloomFilter::set for keys[0..n): src/bloom_filter.cpp:49-53, as called per
 * written entry by Run::put (src/run.cpp:162) during a flush
 * (src/lsm_tree.cpp:127-129) or compaction (src/lsm_tree.cpp:81-88). */
int bloomhip_set_batch(bloomhip_filter *f, const void *keys, size_t n, size_t stride_bytes,
                       int keys_on_device, void *stream);

/* BloomFilter::is_set of every key against each of nf filters
 * (src/bloom_filter.cpp:55-59; Run::get's probe, src/run.cpp:93, over the
 * runs a GET visits, src/lsm_tree.cpp:180-212).  All filters must live on
 * one device.  Result bit i%64 of out_packed[j*ceil(n/64) + i/64] is
 * is_set(key i) for filters[j]; bits past n in the last word are 0. */
int bloomhip_test_batch(const bloomhip_filter *const *filters, int nf, const void *keys,
                        size_t n, size_t stride_bytes, int keys_on_device,
                        uint64_t *out_packed, int out_on_device, void *stream);

/* --- run metadata and batched GET routing ------
 *
 * bloomhip_set_batch_run: a whole run written at once (a flush,
 * src/lsm_tree.cpp:124-129, or a compaction's output, :74-88): set() of every
 * key as bloomhip_set_batch, plus the run's metadata that Run::put builds in
 * the same pass (src/run.cpp:158-174): a fence pointer = the key of every
 * entry whose index is a multiple of 4096 (getpagesize(), :164-166), and the
 * max key (:170; the reference leaves max_key uninitialised, src/run.h:13 —
 * here it starts at INT32_MIN).  Replaces the previous metadata. */
int bloomhip_set_batch_run(bloomhip_filter *f, const void *keys, size_t n, size_t stride_bytes,
                           int keys_on_device, void *stream);
/* Metadata of a run restored from disk (fences ascending).  Synchronous. */
int bloomhip_set_run_meta(bloomhip_filter *f, const int32_t *fences, size_t nfences,
                          int32_t max_key);
/* Metadata back to the host: *nfences_out always; fences (if non-NULL,
 * capacity cap) and *max_key_out.  Synchronous. */
int bloomhip_get_run_meta(const bloomhip_filter *f, int32_t *fences, size_t cap,
                          size_t *nfences_out, int32_t *max_key_out);

/* Batched GET routing over nruns <= 64 runs, runs[0] the newest
 * (LSMTree::get_run order, src/lsm_tree.cpp:141-151).  Run r is a candidate
 * for key i when Run::get would read a page for it (src/run.cpp:94-96):
 *     fence_r[0] <= key <= max_key_r  &&  is_set_r(key)
 * (a run without metadata is never a candidate).  Outputs, each optional
 * (NULL to skip):
 *   cand_packed  nruns x ceil(n/64) u64, bit i%64 of row r word i/64;
 *   first_run[i] the newest candidate (the run LSMTree::get settles on when
 *                the key is there, src/lsm_tree.cpp:195-201), -1 if none;
 *   page[i]      that run's page index, upper_bound(fences, key) - 1
 *                (src/run.cpp:97-99), -1 if none.
 * Reading the page and checking the key stays with the caller. */
int bloomhip_route_gets(const bloomhip_filter *const *runs, int nruns, const void *keys,
                        size_t n, size_t stride_bytes, int keys_on_device,
                        uint64_t *cand_packed, int32_t *first_run, int32_t *page,
                        int out_on_device, void *stream);
/* The same routing with first_run and page packed into one u32 per GET, half
 * the output bytes of the two int32 arrays (the GET's whole answer for
 * Run::get, src/run.cpp:93-99, in one word):
 *   route[i] = first_run[i] << 28 | page[i]   when key i has a candidate run,
 *              BLOOMHIP_ROUTE_NONE            when it has none.
 * nruns <= 16.  cand_packed as above; each output optional (NULL to skip). */
#define BLOOMHIP_ROUTE_NONE 0xFFFFFFFFu
#define BLOOMHIP_ROUTE_PAGE_BITS 28
int bloomhip_route_gets_packed(const bloomhip_filter *const *runs, int nruns, const void *keys,
                               size_t n, size_t stride_bytes, int keys_on_device,
                               uint64_t *cand_packed, uint32_t *route, int out_on_device,
                               void *stream);

/* --- persistence beside the run -------------------------
 * The reference keeps a run's entries in an mmap'd file (src/run.cpp:34-72)
 * and its filter only in memory (src/run.h:11).  bloomhip_save writes the
 * bitmap (dynamic_bitset blocks) and the run metadata to `path` (written to
 * path.tmp, then renamed); bloomhip_load creates a filter on `device` from
 * such a file (BLOOMHIP_EINVAL for a file that is not one, or is damaged:
 * the file ends with an FNV-1a 64 checksum).  bloomhip_build_from_run_file
 * maps a run file of entry_t {key, val} records (src/types.h:14-22), sizes
 * the filter as Run::Run does (m = (long)((float)max_size * bpe),
 * src/run.cpp:13-15) and builds it and the run metadata from its first
 * n_entries records.  All synchronous. */
int bloomhip_save(const bloomhip_filter *f, const char *path);
int bloomhip_load(const char *path, int device, bloomhip_filter **out);
int bloomhip_build_from_run_file(const char *path, uint64_t n_entries, int64_t max_size,
                                 float bits_per_entry, int device, bloomhip_filter **out);

/* --- compaction fused with the new run's filter build ----
 * LSMTree::merge_down (src/lsm_tree.cpp:48-95) through MergeContext
 * (src/merge.cpp:6-39): a k-way merge of nruns key-sorted runs of entry_t
 * {key, val} records (src/types.h:14-22), runs[0] the newest (precedence 0),
 * releasing for each distinct key only the newest run's entry; with
 * drop_tombstones (merging into the last level, src/lsm_tree.cpp:84-86)
 * entries whose val is VAL_TOMBSTONE (INT32_MIN) are dropped.  The merged run
 * (ascending keys) goes to out_entries (capacity: the sum of nentries; must
 * not alias an input) and its length to *n_out.  When f is not NULL the new
 * run's filter and metadata are built from the merged keys in the same call
 * (bloomhip_set_batch_run on the device copy).  Runs and output are host
 * buffers unless runs_on_device / out_on_device; everything runs on
 * `device` (f's device when given).  Synchronous (the output length is
 * returned). */
int bloomhip_compact(const void *const *runs, const size_t *nentries, int nruns,
                     int runs_on_device, int drop_tombstones, void *out_entries, size_t *n_out,
                     int out_on_device, bloomhip_filter *f, int device, void *stream);

/* Scalar compatibility entry points (one key; synchronous), for
 * BloomFilter::set (src/bloom_filter.cpp:49-53) and is_set (:55-59) called
 * once per key.  Low-latency path: the key travels as a kernel argument (no
 * host-to-device copy), one single-lane kernel on HIP's default stream, and
 * is_set's answer is written straight into a pinned, mapped host word of the
 * handle: one launch + one stream synchronisation per call (bench.py
 * `scalar_is_set` measures it).  Calls on one handle serialise on its lock;
 * batch callers should use bloomhip_set_batch / bloomhip_test_batch. */
int bloomhip_set(bloomhip_filter *f, int32_t key);
int bloomhip_is_set(const bloomhip_filter *f, int32_t key, int *hit_out);

/* Persistence: copy the bitmap out/in as ceil(m/64) uint64 blocks in the
 * reference's dynamic_bitset layout.  Host buffers; synchronous.  Upload
 * rejects blocks with bits set at positions >= m. */
int bloomhip_download(const bloomhip_filter *f, uint64_t *words, size_t nwords, void *stream);
int bloomhip_upload(bloomhip_filter *f, const uint64_t *words, size_t nwords, void *stream);

/* A copy of filter src (bitmap, run metadata, strategies) on `device`: a
 * peer copy over xGMI between GPUs, a device-to-device copy on one GPU.  The
 * probe side of per-run sharding: each GPU holds replicas of the
 * runs' filters and probes its own slice of the GET keys.  Synchronous. */
int bloomhip_clone(const bloomhip_filter *src, int device, bloomhip_filter **out);

/* Wait for all work queued on `stream` (NULL: the default stream). */
int bloomhip_sync(const bloomhip_filter *f, void *stream);

/* Build strategy override (BLOOMHIP_BUILD_*); AUTO by default. */
int bloomhip_set_strategy(bloomhip_filter *f, int strategy);
/* Probe strategy (BLOOMHIP_PROBE_*) for this filter; AUTO by default.  In a
 * test_batch the first filter's setting applies to filters left on AUTO. */
int bloomhip_set_probe_strategy(bloomhip_filter *f, int strategy);
/* Strategy AUTO resolved for a batch of n keys on this filter. */
int bloomhip_resolve_strategy(const bloomhip_filter *f, size_t n, int *strategy_out);

/* Per-kernel device timing.  While enabled, every kernel the handle launches
 * is bracketed by HIP events on its stream; bloomhip_profile_read returns,
 * for kernel slot `slot` (0..BLOOMHIP_PROF_SLOTS-1), its name, launch count
 * and summed device milliseconds (it synchronises the stream). */
#define BLOOMHIP_PROF_SLOTS 12
int bloomhip_profile_enable(bloomhip_filter *f, int enable);
int bloomhip_profile_read(bloomhip_filter *f, int slot, const char **name_out,
                          uint64_t *launches_out, double *ms_out);
int bloomhip_profile_reset(bloomhip_filter *f);

/* Free the scratch the partition build / partitioned probe cache per
 * (device, stream).  Waits for those streams; call when no build is queued. */
int bloomhip_trim(void);

/* Self-test hook (no GPU needed): the engine's own position arithmetic —
 * the same inline functions the kernels run — evaluated on the host.
 * out[3*i + j] = hash_{j+1}(keys[i]) % m. */
int bloomhip_host_positions(uint64_t m, const int32_t *keys, size_t n, uint64_t *out);

#ifdef __cplusplus
}
#endif

#endif /* BLOOMHIP_H */
