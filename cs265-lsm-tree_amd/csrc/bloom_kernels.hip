// bloom_kernels.hip — gfx950 kernels for Bloom-filter build (set) and probe
// (is_set).  Bit-exact restatement of jackdent/cs265-lsm-tree
// src/bloom_filter.cpp:49-59 over batches of int32 keys.
//
// Bitmap: the reference's dynamic_bitset<unsigned long> block layout (bit i in
// 64-bit block i/64, bit i%64).  On little-endian that is the same bytes as a
// 32-bit word view (word i>>5, bit i&31), which is what the kernels address,
// so 32-bit atomicOr / LDS words produce the reference's blocks directly.
//
// Build strategies:
//   atomic    — one pass, 3 global atomicOr per key (any m).
//   lds       — m/8 <= 64 KiB: every workgroup builds a private copy of the
//               whole filter in LDS with ds_or, then ORs its non-zero words
//               into the global bitmap.
//   partition — m <= 2^30: pass 1 hashes a tile of keys, counting-sorts the
//               3 positions by 2^19-bit segment in LDS and appends each
//               segment's run to that segment's bin; pass 2 gives every
//               segment to one workgroup, which ORs its bin into a 64 KiB
//               LDS image and writes the segment out with coalesced stores.
#include "bloom_kernels.h"

namespace bloomhip {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int32_t load_key(const KeySpan &ks, size_t i) {
    return *reinterpret_cast<const int32_t *>(ks.base + i * ks.stride);
}

__device__ __forceinline__ uint32_t pos32(uint64_t raw, const ModParams &mp) {
    return mod_fast(raw, mp);
}

__device__ __forceinline__ void global_or(uint32_t *words, uint64_t p) {
    __hip_atomic_fetch_or(words + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void set3_global(uint32_t *words, int32_t k, const ModParams &mp) {
    if (mp.fast) {
        global_or(words, pos32(raw_hash1(k), mp));
        global_or(words, pos32(raw_hash2(k), mp));
        global_or(words, pos32(raw_hash3(k), mp));
    } else {
        global_or(words, raw_hash1(k) % mp.m);
        global_or(words, raw_hash2(k) % mp.m);
        global_or(words, raw_hash3(k) % mp.m);
    }
}

// ---------------------------------------------------------------------------
// atomic: 4 keys per thread per iteration (one 16-B load for packed keys).
// ---------------------------------------------------------------------------
template <int LAYOUT>
__global__ void __launch_bounds__(kBlock) k_build_atomic(KeySpan ks, ModParams mp,
                                                         uint32_t *__restrict__ words) {
    const size_t nthreads = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nquads = ks.n / 4;
    for (size_t q = tid; q < nquads; q += nthreads) {
        int32_t k0, k1, k2, k3;
        if constexpr (LAYOUT == KEYS_PACKED) {
            const int4 v = reinterpret_cast<const int4 *>(ks.base)[q];
            k0 = v.x; k1 = v.y; k2 = v.z; k3 = v.w;
        } else if constexpr (LAYOUT == KEYS_ENTRY) {
            const int4 a = reinterpret_cast<const int4 *>(ks.base)[2 * q];
            const int4 b = reinterpret_cast<const int4 *>(ks.base)[2 * q + 1];
            k0 = a.x; k1 = a.z; k2 = b.x; k3 = b.z;
        } else {
            k0 = load_key(ks, 4 * q); k1 = load_key(ks, 4 * q + 1);
            k2 = load_key(ks, 4 * q + 2); k3 = load_key(ks, 4 * q + 3);
        }
        set3_global(words, k0, mp);
        set3_global(words, k1, mp);
        set3_global(words, k2, mp);
        set3_global(words, k3, mp);
    }
    // tail (< 4 keys)
    const size_t t = nquads * 4 + tid;
    if (t < ks.n) set3_global(words, load_key(ks, t), mp);
}

// ---------------------------------------------------------------------------
// lds: private LDS copy of the whole filter per workgroup (m/8 <= 64 KiB).
// ---------------------------------------------------------------------------
template <int LAYOUT>
__global__ void __launch_bounds__(kBlock) k_build_lds(KeySpan ks, ModParams mp,
                                                      uint32_t *__restrict__ words,
                                                      uint32_t nw32, size_t keys_per_block) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_bits[];
    for (uint32_t i = threadIdx.x; i < nw32; i += blockDim.x) lds_bits[i] = 0;
    __syncthreads();

    const size_t begin = (size_t)blockIdx.x * keys_per_block;
    const size_t end = min(ks.n, begin + keys_per_block);
    for (size_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
        int32_t k;
        if constexpr (LAYOUT == KEYS_PACKED) k = reinterpret_cast<const int32_t *>(ks.base)[i];
        else k = load_key(ks, i);
        const uint32_t p1 = pos32(raw_hash1(k), mp);
        const uint32_t p2 = pos32(raw_hash2(k), mp);
        const uint32_t p3 = pos32(raw_hash3(k), mp);
        atomicOr(&lds_bits[p1 >> 5], 1u << (p1 & 31));
        atomicOr(&lds_bits[p2 >> 5], 1u << (p2 & 31));
        atomicOr(&lds_bits[p3 >> 5], 1u << (p3 & 31));
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nw32; i += blockDim.x) {
        const uint32_t w = lds_bits[i];
        if (w) __hip_atomic_fetch_or(words + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// partition pass 1: hash a tile, counting-sort its positions by segment in
// LDS, reserve each segment's run in its bin, write the runs out.
// ---------------------------------------------------------------------------
constexpr int kMaxBins = 2048;
constexpr int kTilePos = (int)kPartTileKeys * 3;
constexpr int kKeysPerThread = (int)kPartTileKeys / kBlock;  // 16

template <int LAYOUT>
__global__ void __launch_bounds__(kBlock) k_part_bin(KeySpan ks, ModParams mp,
                                                     uint32_t *__restrict__ words,
                                                     PartitionWorkspace ws) {
    __shared__ uint32_t s_sorted[kTilePos];   // 48 KiB
    __shared__ uint32_t s_hist[kMaxBins];     // counts, then run starts in s_sorted
    __shared__ uint32_t s_base[kMaxBins];     // reserved start of the run in the bin
    __shared__ uint32_t s_wave_sum[kBlock / 64];

    const int nbins = (int)ws.nbins;
    const size_t tile0 = (size_t)blockIdx.x * kPartTileKeys;
    const int tid = threadIdx.x;

    for (int b = tid; b < nbins; b += kBlock) s_hist[b] = 0;
    __syncthreads();

    // 1. positions + rank within segment (LDS atomics).
    uint32_t pos[kKeysPerThread * 3];
    uint32_t rank[kKeysPerThread * 3];
    int nvalid = 0;
#pragma unroll
    for (int j = 0; j < kKeysPerThread; j++) {
        const size_t i = tile0 + (size_t)j * kBlock + tid;
        if (i < ks.n) {
            int32_t k;
            if constexpr (LAYOUT == KEYS_PACKED) k = reinterpret_cast<const int32_t *>(ks.base)[i];
            else k = load_key(ks, i);
            pos[3 * j + 0] = pos32(raw_hash1(k), mp);
            pos[3 * j + 1] = pos32(raw_hash2(k), mp);
            pos[3 * j + 2] = pos32(raw_hash3(k), mp);
            nvalid = j + 1;
        }
    }
#pragma unroll
    for (int j = 0; j < kKeysPerThread * 3; j++) {
        if (j < nvalid * 3) rank[j] = atomicAdd(&s_hist[pos[j] >> kSegBits], 1u);
    }
    __syncthreads();

    // 2. exclusive scan of the histogram (block-wide) -> run starts; reserve
    //    each non-empty run in its bin with one global atomic.
    constexpr int kPer = kMaxBins / kBlock;  // 8 bins per thread
    uint32_t local[kPer];
    uint32_t tsum = 0;
#pragma unroll
    for (int q = 0; q < kPer; q++) {
        const int b = tid * kPer + q;
        local[q] = b < nbins ? s_hist[b] : 0u;
        tsum += local[q];
    }
    // wave-level inclusive scan of tsum
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t incl = tsum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_wave_sum[wave] = incl;
    __syncthreads();
    uint32_t wave_off = 0;
    for (int w = 0; w < wave; w++) wave_off += s_wave_sum[w];
    uint32_t run = wave_off + incl - tsum;
#pragma unroll
    for (int q = 0; q < kPer; q++) {
        const int b = tid * kPer + q;
        if (b < nbins) {
            const uint32_t c = local[q];
            s_hist[b] = run;  // run start inside s_sorted
            s_base[b] = c ? atomicAdd(&ws.counts[b], c) : 0u;
            run += c;
        }
    }
    __syncthreads();

    // 3. scatter into the LDS image sorted by segment.
#pragma unroll
    for (int j = 0; j < kKeysPerThread * 3; j++) {
        if (j < nvalid * 3) s_sorted[s_hist[pos[j] >> kSegBits] + rank[j]] = pos[j];
    }
    __syncthreads();

    // 4. copy runs out: consecutive threads take consecutive sorted entries,
    //    so each wave writes one or two contiguous runs.
    const size_t tile_keys = min((size_t)kPartTileKeys, ks.n - tile0);
    const int npos = (int)tile_keys * 3;
    const uint32_t segmask = (1u << kSegBits) - 1u;
    for (int e = tid; e < npos; e += kBlock) {
        const uint32_t p = s_sorted[e];
        const uint32_t b = p >> kSegBits;
        const uint32_t dst = s_base[b] + (uint32_t)e - s_hist[b];
        if (dst < ws.cap) {
            ws.bins[(size_t)b * ws.cap + dst] = p & segmask;
        } else {
            // bin full (only for adversarial key sets): set the bit directly.
            __hip_atomic_fetch_or(words + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------
// partition pass 2: one workgroup per 2^19-bit segment.
// ---------------------------------------------------------------------------
constexpr int kSegWords = (1 << kSegBits) / 32;  // 16384 u32 = 64 KiB

__global__ void __launch_bounds__(1024) k_part_apply(uint32_t *__restrict__ words, uint64_t nw32,
                                                     PartitionWorkspace ws, int merge_existing) {
    extern __shared__ __attribute__((aligned(16))) uint32_t seg[];
    const uint32_t b = blockIdx.x;
    for (int i = threadIdx.x; i < kSegWords; i += blockDim.x) seg[i] = 0;
    __syncthreads();

    const uint32_t total = ws.counts[b];
    const uint32_t cnt = min((uint32_t)ws.cap, total);
    // A full bin spilled positions straight into this segment with atomics.
    const bool merge = merge_existing || total > (uint32_t)ws.cap;
    const uint32_t *src = ws.bins + (size_t)b * ws.cap;
    const uint32_t nq = cnt / 4;
    const uint4 *src4 = reinterpret_cast<const uint4 *>(src);  // cap is a multiple of 4
    for (uint32_t q = threadIdx.x; q < nq; q += blockDim.x) {
        const uint4 v = src4[q];
        atomicOr(&seg[v.x >> 5], 1u << (v.x & 31));
        atomicOr(&seg[v.y >> 5], 1u << (v.y & 31));
        atomicOr(&seg[v.z >> 5], 1u << (v.z & 31));
        atomicOr(&seg[v.w >> 5], 1u << (v.w & 31));
    }
    for (uint32_t e = nq * 4 + threadIdx.x; e < cnt; e += blockDim.x) {
        const uint32_t v = src[e];
        atomicOr(&seg[v >> 5], 1u << (v & 31));
    }
    __syncthreads();

    const uint64_t w0 = (uint64_t)b * kSegWords;
    const uint64_t wend = min(nw32, w0 + kSegWords);
    const int nseg = (int)(wend - w0);
    uint32_t *dst = words + w0;
    if (nseg == kSegWords) {
        uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
        const uint4 *seg4 = reinterpret_cast<const uint4 *>(seg);
        for (int q = threadIdx.x; q < kSegWords / 4; q += blockDim.x) {
            uint4 v = seg4[q];
            if (merge) {
                const uint4 o = dst4[q];
                v.x |= o.x; v.y |= o.y; v.z |= o.z; v.w |= o.w;
            }
            dst4[q] = v;
        }
    } else {
        for (int i = threadIdx.x; i < nseg; i += blockDim.x) {
            uint32_t v = seg[i];
            if (merge) v |= dst[i];
            dst[i] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// probe: one key per lane; the three raw hashes are computed once and reduced
// modulo each filter's m; per filter the AND of the three bit tests (with the
// reference's short-circuit) is packed with a 64-lane ballot into one u64.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool test_bit(const uint32_t *w, uint64_t p) {
    return (w[p >> 5] >> (p & 31)) & 1u;
}

template <int LAYOUT>
__global__ void __launch_bounds__(kBlock) k_probe(KeySpan ks, ProbeTable t,
                                                  uint64_t *__restrict__ out, size_t nw_out) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t w = wave; w < nw_out; w += nwaves) {
        const size_t i = w * 64 + lane;
        const bool valid = i < ks.n;
        int32_t k = 0;
        if (valid) {
            if constexpr (LAYOUT == KEYS_PACKED) k = reinterpret_cast<const int32_t *>(ks.base)[i];
            else k = load_key(ks, i);
        }
        const uint64_t h1 = raw_hash1(k), h2 = raw_hash2(k), h3 = raw_hash3(k);
        for (int f = 0; f < t.nf; f++) {
            const ModParams &mp = t.mp[f];
            const uint32_t *fw = t.words[f];
            bool hit = false;
            if (valid) {
                if (mp.fast) {
                    hit = test_bit(fw, pos32(h1, mp)) && test_bit(fw, pos32(h2, mp)) &&
                          test_bit(fw, pos32(h3, mp));
                } else {
                    hit = test_bit(fw, h1 % mp.m) && test_bit(fw, h2 % mp.m) &&
                          test_bit(fw, h3 % mp.m);
                }
            }
            const uint64_t ballot = __ballot(hit);
            if (lane == 0) out[(size_t)f * nw_out + w] = ballot;
        }
    }
}

inline unsigned grid_for(size_t work_items, unsigned per_block, unsigned cap) {
    size_t g = (work_items + per_block - 1) / per_block;
    if (g == 0) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_build_atomic(const KeySpan &ks, const ModParams &mp, uint32_t *words,
                               hipStream_t stream) {
    if (ks.n == 0) return hipSuccess;
    const unsigned grid = grid_for((ks.n + 3) / 4, kBlock, 16384);
    switch (ks.layout) {
        case KEYS_PACKED:
            k_build_atomic<KEYS_PACKED><<<grid, kBlock, 0, stream>>>(ks, mp, words); break;
        case KEYS_ENTRY:
            k_build_atomic<KEYS_ENTRY><<<grid, kBlock, 0, stream>>>(ks, mp, words); break;
        default:
            k_build_atomic<KEYS_STRIDED><<<grid, kBlock, 0, stream>>>(ks, mp, words); break;
    }
    return hipGetLastError();
}

hipError_t launch_build_lds(const KeySpan &ks, const ModParams &mp, uint32_t *words,
                            hipStream_t stream) {
    if (ks.n == 0) return hipSuccess;
    const uint32_t nw32 = (uint32_t)((mp.m + 31) / 32);
    const size_t lds = (size_t)nw32 * 4;
    // Enough keys per block that the merge (nw32 words) stays a small share.
    size_t kpb = (size_t)nw32 * 2;
    if (kpb < 4096) kpb = 4096;
    unsigned grid = (unsigned)((ks.n + kpb - 1) / kpb);
    if (grid > 1024) {
        grid = 1024;
        kpb = (ks.n + grid - 1) / grid;
    }
    if (ks.layout == KEYS_PACKED)
        k_build_lds<KEYS_PACKED><<<grid, kBlock, lds, stream>>>(ks, mp, words, nw32, kpb);
    else
        k_build_lds<KEYS_STRIDED><<<grid, kBlock, lds, stream>>>(ks, mp, words, nw32, kpb);
    return hipGetLastError();
}

hipError_t launch_part_bin(const KeySpan &ks, const ModParams &mp, uint32_t *words,
                           const PartitionWorkspace &ws, hipStream_t stream) {
    if (ks.n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((ks.n + kPartTileKeys - 1) / kPartTileKeys);
    if (ks.layout == KEYS_PACKED)
        k_part_bin<KEYS_PACKED><<<grid, kBlock, 0, stream>>>(ks, mp, words, ws);
    else
        k_part_bin<KEYS_STRIDED><<<grid, kBlock, 0, stream>>>(ks, mp, words, ws);
    return hipGetLastError();
}

hipError_t launch_part_apply(const ModParams &mp, uint32_t *words, const PartitionWorkspace &ws,
                             int merge_existing, hipStream_t stream) {
    const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
    k_part_apply<<<(unsigned)ws.nbins, 1024, kSegWords * 4, stream>>>(words, nw32, ws,
                                                                    merge_existing);
    return hipGetLastError();
}

hipError_t launch_probe(const KeySpan &ks, const ProbeTable &t, uint64_t *out, size_t nw_out,
                        hipStream_t stream) {
    if (nw_out == 0) return hipSuccess;
    const unsigned grid = grid_for(nw_out, kBlock / 64, 16384);
    if (ks.layout == KEYS_PACKED)
        k_probe<KEYS_PACKED><<<grid, kBlock, 0, stream>>>(ks, t, out, nw_out);
    else
        k_probe<KEYS_STRIDED><<<grid, kBlock, 0, stream>>>(ks, t, out, nw_out);
    return hipGetLastError();
}

}  // namespace bloomhip
