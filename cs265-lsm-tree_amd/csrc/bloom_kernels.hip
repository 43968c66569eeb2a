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
//   lds       — m/8 <= 160 KiB: every workgroup builds a private copy of the
//               whole filter in LDS with ds_or, then ORs its non-zero words
//               into the global bitmap.
//   partition — m <= 2^33: pass 1 hashes a tile of keys (4096 or 8192) and
//               counting-sorts its 3 positions by segment in LDS (segments of
//               up to 160 KiB, a multiple of the CU count where possible),
//               writing the sorted tile as 21-bit entries packed three per
//               u64 and its per-segment run starts; pass 2 gives every
//               segment to one workgroup, which walks that segment's run in
//               every tile, ORs it into an LDS image of the segment and
//               writes the segment out with coalesced stores.  No global
//               atomics.
// Probe strategies: gather, LDS, partitioned (pass 1 with slots, pass 2 tests
// the segment's bits, k_probe_combine) and stacked (several filters in one
// partitioned pass).
//
// This unit: the atomic and LDS builds, the gather and LDS probes, run
// metadata and GET routing, the scalar calls, and the geometry planners.
// The partition kernels are in bloom_device.h (one translation unit per
// instantiation family: bloom_pass1_*.hip, bloom_pass2.hip, bloom_probe*.hip).
#include "bloom_device.h"

#include <stdlib.h>

namespace bloomhip {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t pos32(uint64_t raw, const ModParams &mp) {
    return mod_32(raw, mp);
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
        global_or(words, mod_wide(raw_hash1(k), mp));
        global_or(words, mod_wide(raw_hash2(k), mp));
        global_or(words, mod_wide(raw_hash3(k), mp));
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
            k0 = load_key<LAYOUT>(ks, 4 * q); k1 = load_key<LAYOUT>(ks, 4 * q + 1);
            k2 = load_key<LAYOUT>(ks, 4 * q + 2); k3 = load_key<LAYOUT>(ks, 4 * q + 3);
        }
        set3_global(words, k0, mp);
        set3_global(words, k1, mp);
        set3_global(words, k2, mp);
        set3_global(words, k3, mp);
    }
    // tail (< 4 keys)
    const size_t t = nquads * 4 + tid;
    if (t < ks.n) set3_global(words, load_key<LAYOUT>(ks, t), mp);
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
        else k = load_key<LAYOUT>(ks, i);
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

// Every load of the tile is issued before any LDS store, at clamped (always
// valid) addresses so that no load sits under a branch: C4's 161 MB table
// 86.3 -> 63.9 us (3.7 -> 5.0 TB/s, tools/ubench.py transpose).
__global__ void __launch_bounds__(kTransposeBlock) k_runs_transpose(
    const uint32_t *__restrict__ rows, uint32_t *__restrict__ cols, size_t ntiles, int width) {
    __shared__ uint32_t t[kTransposeTile][kTransposeTile + 1];
    constexpr int kRowsPerPass = kTransposeBlock / 64, kPer = kTransposeTile / kRowsPerPass;
    const int b0 = blockIdx.x * kTransposeTile;           // first segment column
    const size_t t0 = (size_t)blockIdx.y * kTransposeTile;  // first tile row
    const int x = threadIdx.x & 63, y0 = threadIdx.x >> 6;
    const int bx = min(b0 + x, width - 1);
    uint32_t v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; i++) {
        const size_t tile = min(t0 + y0 + kRowsPerPass * i, ntiles - 1);
        v[i] = rows[tile * width + bx];
    }
#pragma unroll
    for (int i = 0; i < kPer; i++) t[y0 + kRowsPerPass * i][x] = v[i];
    __syncthreads();
    const size_t tile = t0 + x;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
        const int y = y0 + kRowsPerPass * i;
        if (tile < ntiles && b0 + y < width) cols[(size_t)(b0 + y) * ntiles + tile] = t[x][y];
    }
}

// ---------------------------------------------------------------------------
// probe: one key per lane; the three raw hashes are computed once and reduced
// modulo each filter's m; per filter the AND of the three bit tests (with the
// reference's short-circuit) is packed with a 64-lane ballot into one u64.
// ---------------------------------------------------------------------------
constexpr int kProbeGroup = 4;  // filters whose gathers a lane has in flight together

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
            else k = load_key<LAYOUT>(ks, i);
        }
        const uint64_t h[3] = {raw_hash1(k), raw_hash2(k), raw_hash3(k)};
        for (int g = 0; g < t.nf; g += kProbeGroup) {
            // Round r tests hash r of every still-alive (key, filter) pair of
            // the group: the reference's short-circuit && per filter, with the
            // group's gathers of one round in flight together.
            bool alive[kProbeGroup];
#pragma unroll
            for (int q = 0; q < kProbeGroup; q++) alive[q] = valid && g + q < t.nf;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                uint32_t word[kProbeGroup], bit[kProbeGroup];
#pragma unroll
                for (int q = 0; q < kProbeGroup; q++) {
                    if (alive[q]) {
                        const ModParams &mp = t.mp[g + q];
                        const uint64_t p = mod_any(h[r], mp);
                        word[q] = t.words[g + q][p >> 5];
                        bit[q] = (uint32_t)p & 31u;
                    }
                }
#pragma unroll
                for (int q = 0; q < kProbeGroup; q++)
                    if (alive[q]) alive[q] = (word[q] >> bit[q]) & 1u;
            }
#pragma unroll
            for (int q = 0; q < kProbeGroup; q++) {
                const uint64_t ballot = __ballot(alive[q]);
                if (lane == 0 && g + q < t.nf) out[(size_t)(g + q) * nw_out + w] = ballot;
            }
        }
    }
}

// LDS probe (k_probe_lds): filters of at most kLdsBitmapBytes are staged
// whole into each workgroup's LDS (one 1024-thread workgroup per CU), then
// every key of the grid-stride loop tests its three bits there: random LDS
// reads run ~10x the L2 gather rate.  All three bits are
// read (branch-free; an LDS read costs less than the divergence), the AND is
// the reference's && result.
constexpr int kProbeLdsBlock = 1024;

template <int LAYOUT, bool P2>
__global__ void __launch_bounds__(kProbeLdsBlock) k_probe_lds(KeySpan ks, const uint32_t *words,
                                                             ModParams mp, uint32_t nw32,
                                                             uint64_t *__restrict__ out,
                                                             size_t nw_out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t filt[];
    const uint2 *src = reinterpret_cast<const uint2 *>(words);  // nw32 is even
    for (uint32_t q = threadIdx.x; q < nw32 / 2; q += kProbeLdsBlock)
        reinterpret_cast<uint2 *>(filt)[q] = src[q];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    constexpr int kWaves = kProbeLdsBlock / 64;
    for (size_t w = (size_t)blockIdx.x * kWaves + (threadIdx.x >> 6); w < nw_out;
         w += (size_t)gridDim.x * kWaves) {
        const size_t i = w * 64 + lane;
        const bool valid = i < ks.n;
        int32_t k = 0;
        if (valid) {
            if constexpr (LAYOUT == KEYS_PACKED) k = reinterpret_cast<const int32_t *>(ks.base)[i];
            else k = load_key<LAYOUT>(ks, i);
        }
        const uint32_t p1 = P2 ? mod_p2(raw_hash1(k), mp) : mod_fast(raw_hash1(k), mp);
        const uint32_t p2 = P2 ? mod_p2(raw_hash2(k), mp) : mod_fast(raw_hash2(k), mp);
        const uint32_t p3 = P2 ? mod_p2(raw_hash3(k), mp) : mod_fast(raw_hash3(k), mp);
        const uint32_t hit = (filt[p1 >> 5] >> (p1 & 31)) & (filt[p2 >> 5] >> (p2 & 31)) &
                             (filt[p3 >> 5] >> (p3 & 31)) & 1u;
        const uint64_t ballot = __ballot(valid && hit);
        if (lane == 0) out[w] = ballot;
    }
}

// ---------------------------------------------------------------------------
// §8f rows 1 and 4: run metadata and batched GET routing.
// k_run_meta: the fence pointers of a run written in key order (the key of
// every entry whose index is a multiple of kFenceStride, src/run.cpp:164-166)
// and its max key (src/run.cpp:170), built beside the filter.
// k_route: per key, which runs Run::get would read (range check against the
// run's first fence and max key, then the filter bit, src/run.cpp:94-96), the
// newest such run (src/lsm_tree.cpp:141-151,195-201) and its page index
// (upper_bound over its fences - 1, src/run.cpp:97-99).  The filter bits come
// from the probe kernels (any strategy) in the packed rows `cand`, which are
// rewritten in place with the range check applied.  All runs' fences are
// staged in LDS when they fit, so the page search costs LDS reads only.
// ---------------------------------------------------------------------------
constexpr int kMetaBlock = 256;

template <int LAYOUT>
__global__ void __launch_bounds__(kMetaBlock) k_run_meta(KeySpan ks, int32_t *__restrict__ meta) {
    int32_t *fences = meta + 1;
    __shared__ int32_t s_max[kMetaBlock / 64];
    int32_t mx = INT32_MIN;
    // Packed keys and entry_t runs: 4 consecutive keys per lane per step (one
    // 16-B load, or four 8-B entry loads), two steps in flight; a fence is
    // always the first key of a step (kFenceStride % 4 == 0).
    constexpr bool VEC = LAYOUT == KEYS_PACKED || LAYOUT == KEYS_ENTRY;
    const size_t nthreads = (size_t)gridDim.x * kMetaBlock;
    const size_t tid = (size_t)blockIdx.x * kMetaBlock + threadIdx.x;
    size_t done = 0;
    if constexpr (VEC) {
        static_assert(kFenceStride % 4 == 0, "fences at step starts");
        const size_t nq = ks.n / 4;
        const bool a16 = (reinterpret_cast<uintptr_t>(ks.base) & 15) == 0;
        auto quad = [&](size_t q) -> int4 {
            if constexpr (LAYOUT == KEYS_PACKED) return reinterpret_cast<const int4 *>(ks.base)[q];
            if (a16) {  // two entries per 16-B load
                const int4 *e = reinterpret_cast<const int4 *>(ks.base) + 2 * q;
                const int4 u = e[0], w = e[1];
                return make_int4(u.x, u.z, w.x, w.z);
            }
            const int2 *e = reinterpret_cast<const int2 *>(ks.base) + 4 * q;
            return make_int4(e[0].x, e[1].x, e[2].x, e[3].x);
        };
        auto take = [&](size_t q, const int4 &v) {
            if ((4 * q) % kFenceStride == 0) fences[4 * q / kFenceStride] = v.x;
            mx = max(mx, max(max(v.x, v.y), max(v.z, v.w)));
        };
        size_t q = tid;
        for (; q + nthreads < nq; q += 2 * nthreads) {
            const int4 a = quad(q), c = quad(q + nthreads);
            take(q, a);
            take(q + nthreads, c);
        }
        if (q < nq) take(q, quad(q));
        done = nq * 4;
    }
    for (size_t i = done + tid; i < ks.n; i += nthreads) {
        const int32_t k = load_key<LAYOUT>(ks, i);
        if (i % kFenceStride == 0) fences[i / kFenceStride] = k;
        mx = max(mx, k);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kMetaBlock / 64; w++) mx = max(mx, s_max[w]);
        atomicMax(meta, mx);  // meta[0] starts at INT32_MIN
    }
}

constexpr int kRouteBlock = 256;

// this lane's value becomes `r` where bit `lane` of the wave mask is set
__device__ __forceinline__ int32_t select_by_mask(uint64_t mask, int32_t r, int32_t v) {
    int32_t out;
    asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(out) : "v"(v), "v"(r), "s"(mask));
    return out;
}

// One wave handles 64 consecutive keys per step, fetched one step ahead with
// the step's candidate words (lane r < nruns loads run r's word; the
// range-checked words leave the same way, one store per run from lane r).
// Per run the candidate test is wave-mask work: the filter word (read from
// lane r) AND the ballot of the range check; the newest candidate run is
// picked with a mask select.  NR > 0 fixes the run count at compile time (the
// run loop unrolls; the kernel is instruction-issue bound, PMC: ~160 VALU +
// ~125 SALU per step before).  Page search (upper_bound over the run's fences,
// staged in LDS): one interpolation guess from the run's first and last
// fence places a window of kRouteWindow fences; two reads check that the
// answer lies in it, and a branchless 4-step search finds it there.  When
// the check fails, a binary search over the whole run does (exact either
// way, only slower).

template <int LAYOUT, bool LDS_FENCES, int NR>
__global__ void __launch_bounds__(kRouteBlock) k_route(KeySpan ks, RouteTable t,
                                                      uint64_t *__restrict__ cand, size_t nw,
                                                      int32_t *__restrict__ first,
                                                      int32_t *__restrict__ page,
                                                      uint32_t *__restrict__ packed) {
    extern __shared__ int32_t s_fences[];
    __shared__ int32_t s_lo[kMaxRouteRuns], s_hi[kMaxRouteRuns];
    __shared__ uint32_t s_nf[kMaxRouteRuns], s_off[kMaxRouteRuns];
    __shared__ float s_scale[kMaxRouteRuns];
    const int nruns = NR > 0 ? NR : t.nruns;
    for (int r = threadIdx.x; r < nruns; r += kRouteBlock) {
        const uint32_t nf = t.nfences[r];
        const int32_t f0 = nf ? t.meta[r][1] : 0, fl = nf ? t.meta[r][nf] : 0;
        s_hi[r] = nf ? t.meta[r][0] : INT32_MIN;  // no fences: never in range
        s_lo[r] = nf ? f0 : INT32_MAX;
        s_nf[r] = nf;
        s_off[r] = t.fence_off[r];
        s_scale[r] = (nf > 1 && fl > f0) ? (float)(nf - 1) / ((float)fl - (float)f0) : 0.0f;
    }
    if constexpr (LDS_FENCES) {
        // eight independent loads in flight per thread per batch
        constexpr int kBatch = 8;
        for (int r = 0; r < nruns; r++) {
            const uint32_t nf = t.nfences[r];
            const int32_t *src = t.meta[r] + 1;
            int32_t *dst = s_fences + t.fence_off[r];
            for (uint32_t b = 0; b < nf; b += kBatch * kRouteBlock) {
                int32_t v[kBatch];
#pragma unroll
                for (int q = 0; q < kBatch; q++) {
                    const uint32_t i = b + q * kRouteBlock + threadIdx.x;
                    v[q] = i < nf ? src[i] : 0;
                }
#pragma unroll
                for (int q = 0; q < kBatch; q++) {
                    const uint32_t i = b + q * kRouteBlock + threadIdx.x;
                    if (i < nf) dst[i] = v[q];
                }
            }
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const size_t wstep = ((size_t)gridDim.x * kRouteBlock) >> 6;
    size_t w = __builtin_amdgcn_readfirstlane(
        (uint32_t)(((size_t)blockIdx.x * kRouteBlock + threadIdx.x) >> 6));
    // Unconditional (clamped) loads: a load under a branch makes the
    // compiler's wait counting fall back to waiting for everything.
    auto load_key_at = [&](size_t ww) -> int32_t {
        const size_t i = min(min(ww, nw - 1) * 64 + lane, ks.n - 1);  // ks.n >= 1 here
        if constexpr (LAYOUT == KEYS_PACKED) return reinterpret_cast<const int32_t *>(ks.base)[i];
        else return load_key<LAYOUT>(ks, i);
    };
    auto load_cand_at = [&](size_t ww) -> uint64_t {
        return cand[(size_t)min(lane, nruns - 1) * nw + min(ww, nw - 1)];
    };
    // One step of 64 keys.  The loop below runs two steps per iteration on
    // two register sets, each set's loads issued a whole step ahead (a
    // single loop-carried set made the compiler wait for the prefetch
    // right away, at the copy).
    auto step = [&](size_t w, int32_t k, uint64_t cw) {
        const size_t i = w * 64 + lane;
        const bool valid = i < ks.n;
        int32_t fr = -1;
        uint64_t newc = 0, open = ~0ull;  // open: lanes without a candidate run yet
#pragma unroll
        for (int r = 0; r < (NR > 0 ? NR : kMaxRouteRuns); r++) {
            if (NR == 0 && r >= nruns) break;
            // (readlane returns int: through uint32_t, or the low half sign-extends)
            const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cw, r);
            const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cw >> 32), r);
            const uint64_t b = (((uint64_t)bhi << 32) | blo) &
                               __ballot(valid && k >= s_lo[r] && k <= s_hi[r]);
            if (lane == r) newc = b;
            fr = select_by_mask(b & open, r, fr);
            open &= ~b;
        }
        if (lane < nruns) cand[(size_t)lane * nw + w] = newc;
        int32_t pg = -1;
        if (fr >= 0) {
            // upper_bound(fences, k); k >= fences[0] (range check), so the
            // answer is in [1, n].
            const int n = (int)s_nf[fr];
            int lo;
            if constexpr (LDS_FENCES) {
                lo = route_page(s_fences + s_off[fr], n, k, (float)s_lo[fr], s_scale[fr]) + 1;
            } else {
                // fences beyond the LDS budget: binary search in global memory
                const int32_t *fz = t.meta[0];
                for (int r = 0; r < nruns; r++)  // this lane's run (kernarg pointers)
                    if (r == fr) fz = t.meta[r] + 1;
                int l = 1, h = n;
                while (l < h) {
                    const int mid = (l + h) >> 1;
                    if (fz[mid] <= k) l = mid + 1;
                    else h = mid;
                }
                lo = l;
            }
            pg = lo - 1;
        }
        if (valid) {
            if (first) first[i] = fr;
            if (page) page[i] = pg;
            if (packed) packed[i] = route_pack(fr, pg);
        }
    };
    int32_t ka = load_key_at(w);
    uint64_t ca = load_cand_at(w);
    while (w < nw) {
        const int32_t kb = load_key_at(w + wstep);
        const uint64_t cb = load_cand_at(w + wstep);
        step(w, ka, ca);
        w += wstep;
        if (w >= nw) break;
        ka = load_key_at(w + wstep);
        ca = load_cand_at(w + wstep);
        step(w, kb, cb);
        w += wstep;
    }
}

// Scalar set / is_set (bloomhip_set / bloomhip_is_set): the key is a kernel
// argument and lane 0 does the reference's work for it
// (src/bloom_filter.cpp:49-53 / :55-59, all three bits read).
__global__ void __launch_bounds__(64) k_set1(uint32_t *__restrict__ words, ModParams mp,
                                             int32_t k) {
    if (threadIdx.x == 0) set3_global(words, k, mp);
}

__global__ void __launch_bounds__(64) k_is_set1(const uint32_t *__restrict__ words, ModParams mp,
                                                int32_t k, uint32_t *__restrict__ hit) {
    if (threadIdx.x != 0) return;
    const uint64_t p1 = mod_any(raw_hash1(k), mp), p2 = mod_any(raw_hash2(k), mp),
                   p3 = mod_any(raw_hash3(k), mp);
    const uint32_t v = (words[p1 >> 5] >> (p1 & 31)) & (words[p2 >> 5] >> (p2 & 31)) &
                       (words[p3 >> 5] >> (p3 & 31)) & 1u;
    // system scope: the host spins on this (mapped, fine-grained) word
    __hip_atomic_store(hit, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
    const size_t lds = ((size_t)nw32 * 4 + 15) & ~(size_t)15;
    if (lds > kLdsBitmapBytes) return hipErrorInvalidValue;
    // Keys per block: enough that the merge (nw32 atomics) stays a small
    // share, few enough that the grid covers the chip.
    size_t kpb = (size_t)nw32 / 4;
    if (kpb < 2048) kpb = 2048;
    unsigned grid = (unsigned)((ks.n + kpb - 1) / kpb);
    if (grid > 1024) {
        grid = 1024;
        kpb = (ks.n + grid - 1) / grid;
    }
    static const bool attr_set = [] {  // > 64 KiB of dynamic LDS must be opted into
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_build_lds<KEYS_PACKED>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBitmapBytes);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_build_lds<KEYS_STRIDED>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBitmapBytes);
        return true;
    }();
    (void)attr_set;
    if (ks.layout == KEYS_PACKED)
        k_build_lds<KEYS_PACKED><<<grid, kBlock, lds, stream>>>(ks, mp, words, nw32, kpb);
    else
        k_build_lds<KEYS_STRIDED><<<grid, kBlock, lds, stream>>>(ks, mp, words, nw32, kpb);
    return hipGetLastError();
}

int device_cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (cus[dev] == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            c <= 0)
            c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}

// The multiply-high divisor of SegMap: magic = ceil(2^31 / g), accepted only
// when mulhi(x, magic) == (x >> 1) / g for every x < 2 * nsub.  g = 1 gives
// 2^31, i.e. x >> 1.
// x M / 2^32 = x / 2g + x e / (g 2^32) with e = M g - 2^31 < g: the floor is
// x / 2g's whenever x e < 2^31 (the fraction of x / 2g is at most 1 - 1/2g).
// Every planned geometry passes that bound; the brute-force check (one
// division per value, ~80 us per plan at 2 nsub = 32768, on the host path of
// every partition call) is only the fallback, and only over SegMap's
// original domain (nsub <= kPartMaxSub).
static bool seg_magic(uint32_t g, uint64_t nsub, uint32_t *magic) {
    if (g == 0 || nsub == 0 || 2 * nsub > (1ull << 32)) return false;
    const uint32_t M = (uint32_t)(((1ull << 31) + g - 1) / g);
    const uint64_t e = (uint64_t)M * g - (1ull << 31);
    if ((2 * nsub - 1) * e >= (1ull << 31)) {
        if (nsub > kPartMaxSub) return false;
        for (uint32_t x = 0; x < 2 * nsub; x++)
            if ((uint32_t)(((uint64_t)x * M) >> 32) != (x >> 1) / g) return false;
    }
    *magic = M;
    return true;
}

bool plan_segments(uint64_t m, int ncu, PartitionWorkspace *ws) {
    if (m == 0 || ncu <= 0) return false;
    // Pass-2 segments: a multiple W of the CU count, each fitting in LDS.
    // Segment images up to all 160 KiB of a CU's LDS (pass 2 has no static
    // LDS): C5 gets 512 segments instead of 768, runs 1.5x longer.
    const uint64_t seg_max = kStackMaxBits;
    const uint64_t per_round = (uint64_t)ncu * seg_max;
    const uint64_t W = ((m + per_round - 1) / per_round) * (uint64_t)ncu;
    // q = p >> s: the smallest power of two 2^s with at most kPartMaxSub
    // values, then g = ceil(nsub / W) per segment, while g << s fits LDS.
    uint32_t s = 5;  // >= one 32-bit word
    while ((((m - 1) >> s) + 1) > kPartMaxSub) s++;
    uint64_t nsub = ((m - 1) >> s) + 1;
    uint64_t g = (nsub + W - 1) / W;
    while (g > 1 && (g << s) > seg_max) g--;
    if ((g << s) > seg_max) return false;  // m > kPartMaxSub * 2^20 (nbins caps it lower)
    // 128-B aligned segments for the 16-B segment stores.
    while (((g << s) % 1024) != 0) g++;
    if ((g << s) > seg_max) return false;
    const uint64_t nbins = (nsub + g - 1) / g;
    if (nbins > kPartMaxBinsBig || (nbins > kPartMaxBins && choose_tile_keys(nbins) == kPartTileKeys))
        return false;
    uint32_t magic = 0;
    if (!seg_magic((uint32_t)g, (uint32_t)nsub, &magic)) return false;
    ws->sub_shift = s;
    ws->group = (uint32_t)g;
    ws->nsub = (uint32_t)nsub;
    ws->seg_bits = (uint32_t)(g << s);
    ws->nbins = (size_t)nbins;
    ws->magic = magic;
    return true;
}

bool plan_build(uint64_t m, int ncu, PartitionWorkspace *ws) {
    if (!plan_segments(m, ncu, ws)) return false;
    if (m <= 0xFFFFFFFFull && ws->nbins >= kSuperMinBins && ws->nbins <= kSuperMaxBins)
        ws->tile_keys = (uint32_t)kSuperTileKeys;  // many short runs: super-tiles (k_part_bin2)
    uint32_t d = 0, t = 0;
    if (!p2_form(m, &d, &t)) return true;
    uint32_t u = 0;
    while (((size_t)1 << u) < ws->nbins) u++;
    if (((size_t)1 << u) != ws->nbins || t < u + 7) return true;
    const uint32_t sl = t - u;
    uint32_t dbits = 0;
    while ((1u << dbits) < d) dbits++;
    if (sl + dbits > kEntryBits || ((uint64_t)d << sl) > kStackMaxBits || ((d << sl) % 1024) != 0)
        return true;
    ws->lad_s = sl;
    ws->lad_u = u;
    ws->lad_hb = 0;
    ws->seg_bits = d << sl;  // the bin's image: d blocks of 2^s bits
    ws->tile_keys = 0;       // the ladder build keeps k_part_bin's tiles
    return true;
}

bool plan_stack(uint64_t m_max, uint64_t gcd_m, uint64_t m_min, int nf, int ncu,
                PartitionWorkspace *ws) {
    if (m_max == 0 || m_max > 0xFFFFFFFFull || nf < 1 || nf > kMaxStack || gcd_m == 0 ||
        m_max % gcd_m != 0 || gcd_m % 128 != 0 || m_min < gcd_m)
        return false;
    // Segment widths w = g << s: w | m_max, so the segments tile the largest
    // member, and w <= m_min, so member j's window of a segment, the w bits
    // from (b * w) mod m_j on, wraps at most once (pass 2 stages it with the
    // wrap; 128 | m_j keeps every 16-B vector on one side of it); all
    // members' windows in the pass-2 workgroup's LDS (160 KiB: the kernel
    // has no static LDS).  The segment map b = mulhi(p >> (s - 1),
    // ceil(2^31 / g)) must be exact over m_max (seg_magic): any s whose 2^s
    // divides m_max, so sizes with a large odd part (the f = 10 tree's
    // 5,120,000 * 10^i = 2^(13+i) * 625 * 5^i) stack too.
    const uint64_t wmax = kStackMaxBits / (uint64_t)nf;
    uint64_t best_w = 0;
    uint32_t best_s = 0, best_magic = 0;
    // The segment count sets the run length per tile (tile entries / nbins),
    // w only the LDS image: the widest w that still gives every CU a segment,
    // else (small m_max) the narrowest, for the most segments.
    auto better = [&](uint64_t w) {
        if (best_w == 0) return true;
        const bool a = m_max / w >= (uint64_t)ncu, b = m_max / best_w >= (uint64_t)ncu;
        if (a != b) return a;
        return a ? w > best_w : w < best_w;
    };
    // Only w that are multiples of 128 bits count, so below s = 7 g steps by
    // 2^(7 - s); and g falls, so the scan of an s ends where w leaves more
    // than kPartMaxBinsBig segments (a few hundred candidates per call, not
    // the ~wmax a unit step visits)
    for (uint32_t s = 1; s < 32 && (1ull << s) <= wmax; s++) {
        if (m_max % (1ull << s)) break;  // larger s cannot divide either
        const uint64_t gstep = s < 7 ? 1ull << (7 - s) : 1ull;
        for (uint64_t g = (wmax >> s) / gstep * gstep; g >= 1; g -= gstep) {
            const uint64_t w = g << s;
            if (m_max / w > kPartMaxBinsBig) break;  // and for every smaller g
            if (w % 128 || m_max % w || w > m_min) continue;
            if (!(better(w) || (w == best_w && s > best_s))) continue;
            uint32_t magic = 0;
            if (!seg_magic((uint32_t)g, m_max >> s, &magic)) continue;
            best_w = w;
            best_s = s;
            best_magic = magic;
        }
    }
    if (best_w == 0) return false;
    ws->sub_shift = best_s;
    ws->group = (uint32_t)(best_w >> best_s);
    ws->nsub = (uint32_t)(m_max >> best_s);
    ws->seg_bits = (uint32_t)best_w;
    ws->nbins = (size_t)(m_max / best_w);
    ws->magic = best_magic;
    // many short runs (the f = 10 tree: 1,250 segments, ~20 entries per
    // 8192-key tile): pass 1 on super-tiles (k_part_bin2 with the slot plane)
    ws->tile_keys = ws->nbins >= kSuperMinBins && ws->nbins <= kSuperMaxBins ? (uint32_t)kSuperTileKeys : 0u;
    return true;
}

// Ladder geometry (kernels.h LadderTable).  Of the (s, k) that fit -- the
// entry (s bits + member 0's block index) in 21 bits; images + table (one
// 32-bit LDS byte address per direct member 1.. and for the packed tuple, rs
// words per row) + tuple map in 160 KiB, or the images alone when the tuple
// is computed (k = 1, LadderTable::ctup) -- the fewest LDS reads per entry
// (k direct members, one packed word, one table row unless computed), then
// the smallest image, then the widest blocks.  Pass 1 tiles of 8192 keys: runs of ~96 entries per bin.
constexpr uint32_t kLadderTileKeys = 2 * (uint32_t)kPartTileKeys;

bool plan_ladder(const uint64_t *m, int nf, int ncu, StackTable *st, PartitionWorkspace *ws,
                 bool allow_computed) {
    if (nf < 2 || nf > kMaxStack) return false;
    uint32_t d = 0, t[kMaxStack];
    for (int j = 0; j < nf; j++) {
        uint32_t dj = 0, tj = 0;
        if (!p2_form(m[j], &dj, &tj) || (j > 0 && (dj != d || tj > t[j - 1]))) return false;
        d = dj;
        t[j] = tj;
    }
    const uint32_t tmax = t[0], tmin = t[nf - 1];
    uint32_t u = 1;
    while ((1u << u) < (uint32_t)(ncu > 2 ? ncu : 2)) u++;
    if (u > 12 || tmax < u + 7) return false;
    auto pow2mod = [&](uint32_t e) {
        uint32_t pm = 1 % d;
        for (uint32_t q = 0; q < e; q++) pm = (pm * 2) % d;
        return pm;
    };
    LadderTable best{};
    size_t best_bytes = 0;
    uint32_t best_reads = ~0u;
    for (uint32_t s = 7; s <= tmin && s + u <= tmax; s++) {
        for (uint32_t kc = 0; kc <= (uint32_t)nf; kc++) {
            // kc = 0: one direct member with the packed tuple computed
            // (LadderTable::ctup, no table); kc >= 1: kc direct members
            const uint32_t k = kc == 0 ? 1 : kc;
            const bool ct = kc == 0;
            if (k > 3 && k < (uint32_t)nf) continue;  // the compiled-in direct counts
            if (ct && (!allow_computed || nf < 2 || t[1] < s + u)) continue;  // member 1's block = hi mod nblk[1]
            LadderTable L{};
            L.s = s;
            L.u = u;
            L.hb = tmax - s - u;
            L.d = d;
            L.k = k;
            if (L.hb > 16) continue;
            L.ne = d << L.hb;
            uint32_t ebits = 0;
            while ((1u << ebits) < L.ne) ebits++;
            if (s + ebits > kEntryBits) continue;
            uint32_t nb = 0;
            for (int j = 0; j < nf; j++) {
                L.t[j] = t[j];
                L.nblk[j] = t[j] >= s + u ? d << (t[j] - s - u) : d;
                L.pmod[j] = pow2mod(tmax - t[j]);
                L.pmodk[j] = (uint32_t)j >= k ? pow2mod(t[k] - t[j]) : 0u;
                if ((uint32_t)j < k) {
                    L.base[j] = nb;
                    nb += L.nblk[j];
                }
            }
            L.img_words = nb << (s - 5);
            if (k < (uint32_t)nf) {
                L.bpp = nf - (int)k <= 4 ? 4 : 8;
                const uint32_t tuple_words = L.bpp << (s - 5);
                L.pk_words = (L.img_words + tuple_words - 1) / tuple_words * tuple_words;
                L.img_words = L.pk_words + L.nblk[k] * tuple_words;
            }
            const uint32_t rw = (k - 1) + (k < (uint32_t)nf ? 1 : 0);
            L.rs = rw <= 1 ? 1 : rw <= 2 ? 2 : rw <= 4 ? 4 : 8;
            uint32_t reads = k + (k < (uint32_t)nf) + (k > 1 || k < (uint32_t)nf);
            if (ct) {
                // hi mod nblk[1] as hi - mulhi(hi, M) * nblk[1], exact for
                // every entry high part hi < ne (checked here)
                const uint32_t nb1 = L.nblk[1];
                const uint32_t M = (uint32_t)(((1ull << 32) + nb1 - 1) / nb1);
                bool exact = nb1 < (1u << 23);
                // exact for hi e < 2^32, e = M nb1 - 2^32 < nb1 (as seg_magic's
                // bound); the loop only when that bound does not cover ne
                const uint64_t e = (uint64_t)M * nb1 - (1ull << 32);
                if (exact && L.ne && (uint64_t)(L.ne - 1) * e >= (1ull << 32))
                    for (uint32_t hi = 0; exact && hi < L.ne; hi++)
                        exact = (uint32_t)(((uint64_t)hi * M) >> 32) == hi / nb1;
                if (!exact) continue;
                L.ctup = 1;
                L.tmagic = M;
                L.rs = 0;
                reads = 2;  // member 0's word and the packed word
            }
            const size_t bytes = ladder_lds_bytes(L);
            if (bytes > kStackMaxBits / 8) continue;
            if (reads < best_reads || (reads == best_reads && bytes <= best_bytes)) {
                best = L;  // ascending s: ties keep the wider blocks
                best_bytes = bytes;
                best_reads = reads;
            }
        }
    }
    if (best_bytes == 0) return false;
    st->ladder = 1;
    st->lad = best;
    ws->nbins = (size_t)1 << u;
    ws->lad_s = best.s;
    ws->lad_u = best.u;
    ws->lad_hb = best.hb;
    ws->seg_bits = 0;
    ws->tile_keys = kLadderTileKeys;
    return true;
}

hipError_t launch_runs_transpose(const PartitionWorkspace &ws, hipStream_t stream) {
    const int width = (int)ws.nbins;
    const dim3 grid((unsigned)((width + kTransposeTile - 1) / kTransposeTile),
                    (unsigned)((ws.ntiles + kTransposeTile - 1) / kTransposeTile));
    if (grid.y > 65535u) return hipErrorInvalidValue;  // > 2^28 keys per batch
    k_runs_transpose<<<grid, kTransposeBlock, 0, stream>>>(ws.run_rows, ws.run_starts, ws.ntiles,
                                                           width);
    return hipGetLastError();
}

bool runs_as_columns(const PartitionWorkspace &ws) {
    return ws.ntiles * ws.nbins * 4 <= kColumnTableMaxBytes;
}

hipError_t launch_part_bin(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                           hipStream_t stream) {
    if (ks.n == 0) return hipSuccess;
    return launch_bin<false>(ks, mp, ws, nullptr, stream);
}

hipError_t launch_probe_lds(const KeySpan &ks, const ModParams &mp, const uint32_t *words,
                            uint64_t *out, size_t nw_out, hipStream_t stream) {
    if (nw_out == 0) return hipSuccess;
    const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
    if (!mp.fast || nw32 * 4 > kLdsBitmapBytes) return hipErrorInvalidValue;
    static const bool attr_set = [] {
        for (const void *fn : {reinterpret_cast<const void *>(&k_probe_lds<KEYS_PACKED, false>),
                               reinterpret_cast<const void *>(&k_probe_lds<KEYS_STRIDED, false>),
                               reinterpret_cast<const void *>(&k_probe_lds<KEYS_PACKED, true>),
                               reinterpret_cast<const void *>(&k_probe_lds<KEYS_STRIDED, true>)})
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kLdsBitmapBytes);
        return true;
    }();
    (void)attr_set;
    // each workgroup stages the filter once: give it >= 64 waves of keys;
    // two workgroups per CU when two copies fit the CU's LDS
    const size_t lds = (size_t)nw32 * 4;
    const unsigned per_cu = lds * 2 <= kLdsBitmapBytes ? 2u : 1u;
    const unsigned grid =
        grid_for(nw_out, 64 * (kProbeLdsBlock / 64), per_cu * (unsigned)device_cu_count());
#define PROBE_LDS(L, P)                                                                  \
    k_probe_lds<L, P><<<grid, kProbeLdsBlock, lds, stream>>>(ks, words, mp, (uint32_t)nw32, \
                                                             out, nw_out)
    if (ks.layout == KEYS_PACKED) {
        if (mp.p2) PROBE_LDS(KEYS_PACKED, true); else PROBE_LDS(KEYS_PACKED, false);
    } else {
        if (mp.p2) PROBE_LDS(KEYS_STRIDED, true); else PROBE_LDS(KEYS_STRIDED, false);
    }
#undef PROBE_LDS
    return hipGetLastError();
}

// A run known to be sorted by key (a compaction's output): its max key is
// the last key, and only the fence keys are read (src/run.cpp:164-170 give the
// same values for a run written in key order).
template <int LAYOUT>
__global__ void __launch_bounds__(kMetaBlock) k_run_meta_sorted(KeySpan ks, size_t nf,
                                                                int32_t *__restrict__ meta) {
    const size_t i = (size_t)blockIdx.x * kMetaBlock + threadIdx.x;
    if (i < nf) meta[1 + i] = load_key<LAYOUT>(ks, i * kFenceStride);
    if (i == 0) meta[0] = load_key<LAYOUT>(ks, ks.n - 1);
}

hipError_t launch_run_meta_sorted(const KeySpan &ks, int32_t *meta, hipStream_t stream) {
    if (ks.n == 0)
        return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(meta), (int)INT32_MIN, 1, stream);
    const size_t nf = (ks.n + kFenceStride - 1) / kFenceStride;
    const unsigned grid = (unsigned)((nf + kMetaBlock - 1) / kMetaBlock);
    if (ks.layout == KEYS_PACKED)
        k_run_meta_sorted<KEYS_PACKED><<<grid, kMetaBlock, 0, stream>>>(ks, nf, meta);
    else if (ks.layout == KEYS_ENTRY)
        k_run_meta_sorted<KEYS_ENTRY><<<grid, kMetaBlock, 0, stream>>>(ks, nf, meta);
    else
        k_run_meta_sorted<KEYS_STRIDED><<<grid, kMetaBlock, 0, stream>>>(ks, nf, meta);
    return hipGetLastError();
}

hipError_t launch_run_meta(const KeySpan &ks, int32_t *meta, hipStream_t stream) {
    hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(meta), (int)INT32_MIN, 1,
                                     stream);
    if (e != hipSuccess || ks.n == 0) return e;
    const unsigned grid = grid_for(ks.n, kMetaBlock * 32, 2048);
    if (ks.layout == KEYS_PACKED)
        k_run_meta<KEYS_PACKED><<<grid, kMetaBlock, 0, stream>>>(ks, meta);
    else if (ks.layout == KEYS_ENTRY)
        k_run_meta<KEYS_ENTRY><<<grid, kMetaBlock, 0, stream>>>(ks, meta);
    else
        k_run_meta<KEYS_STRIDED><<<grid, kMetaBlock, 0, stream>>>(ks, meta);
    return hipGetLastError();
}

hipError_t launch_route(const KeySpan &ks, const RouteTable &t, uint64_t *cand, size_t nw,
                        const RouteOut &ro, hipStream_t stream) {
    if (ro.packed && t.nruns > kRoutePackedMaxRuns) return hipErrorInvalidValue;
    if (nw == 0) return hipSuccess;
    const size_t lds = (size_t)t.total_fences * 4;
    // Fences from LDS beat L2 reads.  The grid is what fits on the chip at
    // once (the staged fences bound the workgroups per CU), and every wave
    // walks many 64-key steps, so each workgroup stages the fences once.
    const bool in_lds = lds <= kRouteLdsFenceBytesMax;
    const size_t per_block = (in_lds ? lds : 0) + 2048;
    int per_cu = (int)(kLdsBitmapBytes / per_block);
    per_cu = per_cu < 1 ? 1 : per_cu > 8 ? 8 : per_cu;  // 8 x 256 threads = 32 waves per CU
    const unsigned grid = grid_for(nw, kRouteBlock / 64, (unsigned)(device_cu_count() * per_cu));
#define ROUTE_LAUNCH(L, F, R) \
    k_route<L, F, R><<<grid, kRouteBlock, F ? lds : 0, stream>>>(ks, t, cand, nw, ro.first, ro.page, ro.packed)
#define ROUTE_NR(L, F)                                                          \
    switch (t.nruns) {                                                          \
        case 1: ROUTE_LAUNCH(L, F, 1); break;                                   \
        case 2: ROUTE_LAUNCH(L, F, 2); break;                                   \
        case 3: ROUTE_LAUNCH(L, F, 3); break;                                   \
        case 4: ROUTE_LAUNCH(L, F, 4); break;                                   \
        case 5: ROUTE_LAUNCH(L, F, 5); break;                                   \
        case 6: ROUTE_LAUNCH(L, F, 6); break;                                   \
        case 7: ROUTE_LAUNCH(L, F, 7); break;                                   \
        case 8: ROUTE_LAUNCH(L, F, 8); break;                                   \
        default: ROUTE_LAUNCH(L, F, 0); break;                                  \
    }
    if (ks.layout == KEYS_PACKED) {
        if (in_lds) ROUTE_NR(KEYS_PACKED, true) else ROUTE_LAUNCH(KEYS_PACKED, false, 0);
    } else {
        if (in_lds) ROUTE_NR(KEYS_STRIDED, true) else ROUTE_LAUNCH(KEYS_STRIDED, false, 0);
    }
#undef ROUTE_NR
#undef ROUTE_LAUNCH
    return hipGetLastError();
}

hipError_t launch_set1(uint32_t *words, const ModParams &mp, int32_t key, hipStream_t stream) {
    k_set1<<<1, 64, 0, stream>>>(words, mp, key);
    return hipGetLastError();
}

hipError_t launch_is_set1(const uint32_t *words, const ModParams &mp, int32_t key, uint32_t *hit,
                          hipStream_t stream) {
    k_is_set1<<<1, 64, 0, stream>>>(words, mp, key, hit);
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
