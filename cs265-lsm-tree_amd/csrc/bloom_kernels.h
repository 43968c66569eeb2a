// bloom_kernels.h — internal launch interface between the C ABI
// (bloom_capi.cpp) and the gfx950 kernels (bloom_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "bloom_math.h"

namespace bloomhip {

// Layout of the key vector handed to a kernel.
enum KeyLayout : int {
    KEYS_PACKED = 0,  // int32 keys at stride 4, base 16-byte aligned
    KEYS_ENTRY = 1,   // entry_t {key, val} at stride 8, base 8-byte aligned (src/types.h:14-22)
    KEYS_STRIDED = 2, // any stride (multiple of 4)
};

struct KeySpan {
    const char *base;
    size_t n;
    size_t stride;  // bytes
    int layout;
};

constexpr int kMaxProbeFilters = 16;

struct ProbeTable {
    const uint32_t *words[kMaxProbeFilters];
    ModParams mp[kMaxProbeFilters];
    int nf;
};

// LDS bytes a private-bitmap workgroup may use (m/8 must fit).
constexpr size_t kLdsBitmapBytes = 64 * 1024;

// Partition build geometry: one LDS segment = 2^kSegBits bits.
constexpr int kSegBits = 19;  // 64 KiB of bitmap per segment workgroup
constexpr size_t kPartTileKeys = 4096;
constexpr size_t kPartMaxBins = 2048;  // m <= 2^30 bits

struct PartitionWorkspace {
    uint32_t *bins;        // [nbins * cap] segment-local offsets
    uint32_t *counts;      // [nbins] fill counters
    size_t cap;            // capacity per bin (entries)
    size_t nbins;
};

// Kernels enqueued on `stream`; all return hipSuccess or the launch error.
hipError_t launch_build_atomic(const KeySpan &keys, const ModParams &mp, uint32_t *words,
                               hipStream_t stream);
hipError_t launch_build_lds(const KeySpan &keys, const ModParams &mp, uint32_t *words,
                            hipStream_t stream);
hipError_t launch_part_bin(const KeySpan &keys, const ModParams &mp, uint32_t *words,
                           const PartitionWorkspace &ws, hipStream_t stream);
// merge_existing: OR into the current bitmap instead of overwriting segments.
hipError_t launch_part_apply(const ModParams &mp, uint32_t *words, const PartitionWorkspace &ws,
                             int merge_existing, hipStream_t stream);
hipError_t launch_probe(const KeySpan &keys, const ProbeTable &t, uint64_t *out, size_t nwords_out,
                        hipStream_t stream);

}  // namespace bloomhip
