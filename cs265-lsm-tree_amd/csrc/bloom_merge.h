// bloom_merge.h — compaction kernels; see bloom_merge.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bloomhip {

// Stable merge of two key-sorted entry_t arrays (a wins ties) into out
// (na + nb entries; a, b 8-B aligned, out 16-B aligned).  split_ws:
// merge_split_words(na + nb) u64.
hipError_t launch_merge2(const void *a, uint64_t na, const void *b, uint64_t nb, void *out,
                         uint64_t *split_ws, hipStream_t stream);
// Up to kMaxMergePairs such merges in one pair of launches (a merge round);
// split_ws: merge_split_words(total entries of the round) u64.
constexpr int kMaxMergePairs = 8;
struct MergePairArgs {
    const void *a;
    uint64_t na;
    const void *b;
    uint64_t nb;
    void *out;
};
hipError_t launch_merge_round(const MergePairArgs *pairs, int np, uint64_t *split_ws,
                              hipStream_t stream);
uint64_t merge_split_words(uint64_t total);

// Keeps the first entry of each key of a key-sorted array (dropping entries
// whose value is VAL_TOMBSTONE when drop_tombstones), packed into out; the
// kept count lands in counts_ws[ceil(n / tile)] (compact_count_words(n) u32).
// keys_out (optional, n int32): the kept keys, packed.
hipError_t launch_dedup(const void *in, uint64_t n, int drop_tombstones, void *out,
                        uint32_t *counts_ws, hipStream_t stream, int32_t *keys_out = nullptr);
uint64_t compact_count_words(uint64_t n);

// One-pass k-way compaction (bloom_merge.hip k_kway_*): the runs (newest
// first, each key-sorted, non-empty, 8-B aligned; k <= kKwayMaxRuns) merged
// in (key, run, index) order, the first entry of every key kept (tombstones
// dropped on request) and written packed to out (+ the kept keys to keys_out
// when non-null); the kept count lands in *count_out (device u32).  ws:
// kway_workspace_bytes(n, k), 16-B aligned.
constexpr int kKwayMaxRuns = 8;
uint64_t kway_workspace_bytes(const uint64_t *n, int k);
hipError_t launch_compact_kway(const void *const *runs, const uint64_t *n, int k, int drop,
                               void *out, int32_t *keys_out, void *ws, uint32_t *count_out,
                               hipStream_t stream);

}  // namespace bloomhip
