// bloom_device.h — the partition kernels (pass 1 k_part_bin, pass 2
// k_part_apply, the probe's k_probe_combine) and their host-side launch
// templates, shared by the kernel translation units (bloom_pass1_*.hip,
// bloom_pass2.hip, bloom_probe*.hip) and the micro-benchmarks.  Each product
// instantiation lives in exactly one translation unit (the exported wrappers
// declared at the end), so the units compile in parallel.
//
// Bit-exact restatement of jackdent/cs265-lsm-tree src/bloom_filter.cpp:49-59
// over batches of int32 keys; the bitmap is dynamic_bitset<unsigned long>'s
// block layout (src/bloom_filter.h:7), addressed as 32-bit words.
#pragma once

#include <stdlib.h>

#include <algorithm>
#include <numeric>

#include "bloom_kernels.h"

namespace bloomhip {

namespace {

// Key i of a span.  The layout is a template argument wherever the kernel
// has one, so entry_t runs (stride 8) address as base + 8i instead of a
// runtime 64-bit stride multiply.
template <int LAYOUT = KEYS_STRIDED>
__device__ __forceinline__ int32_t load_key(const KeySpan &ks, size_t i) {
    if constexpr (LAYOUT == KEYS_PACKED) return reinterpret_cast<const int32_t *>(ks.base)[i];
    else if constexpr (LAYOUT == KEYS_ENTRY) return reinterpret_cast<const int2 *>(ks.base)[i].x;
    else return *reinterpret_cast<const int32_t *>(ks.base + i * ks.stride);
}

// ---------------------------------------------------------------------------
// partition pass 1 (k_part_bin): persistent workgroups of TB threads walk
// tiles of TB * kPartKPT keys.  Each thread hashes kPartKPT keys; the tile's
// 3 positions per key are counting-sorted by segment in LDS (an LDS atomic
// gives each its rank in its segment, a scan gives the segment offsets) and
// the sorted tile goes out packed: the low kEntryBits bits of each position,
// three per u64, 8 B per key-hash triple instead of 12.
// Column `tile` of the segment-major run table gets each segment's run of
// the tile, [start, end) in entries packed start | end << 16 (one u32 per
// (tile, segment): pass 2 reads the table once).  No global atomics.
//
// The next tile's keys are loaded while the current tile is sorted, and the
// workgroup barriers wait only for LDS (lgkmcnt), so the sorted tile's
// stores drain under the next tile's hashing.
//
// MK (how a position is reduced mod m): kModFast, the general remainder for
// m < 2^32 kept scaled by 2^l; kModWide, m >= 2^32 (64-bit positions,
// mod_wide; the entries are the same); kModP2, m = d << t with d | 255 and
// t >= kEntryBits (bloom_math.h mod_p2_hi): the entry is the key hash's own
// low 21 bits and p >> shift = (x >> t) % d << (t - shift) | bits shift..t-1
// of x, so only the 5-instruction (x >> t) % d is left of the remainder.
// SLOTS (partitioned probe): also write, per key and hash, the index its
// position got in the sorted tile: slots[(tile*3 + h)*tile_keys + key].
// ---------------------------------------------------------------------------

// Inclusive prefix sum across the 64 lanes of a wave in DPP steps (no LDS):
// row_shr 1/2/4/8 inside each row of 16 lanes (a lane with no source keeps
// the old value 0), then row_bcast:15 (row r's last lane into row r + 1,
// rows 1 and 3) and row_bcast:31 (lane 31 into rows 2 and 3).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// (a << S) | b in one instruction.
template <typename S>
__device__ __forceinline__ uint32_t lshl_or(uint32_t a, S sh, uint32_t b) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(sh), "v"(b));
    return r;
}

// (a << s) | b in one instruction, s in an SGPR.
__device__ __forceinline__ uint32_t lshl_or_s(uint32_t a, uint32_t sh, uint32_t b) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(sh), "v"(b));
    return r;
}

// Workgroup barrier that waits for this wave's LDS operations only.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS word at an absolute byte address.  Pass 2 has no static LDS, so its
// dynamic image starts at LDS address 0 (launch_apply_g checks that once per
// kernel) and image offsets are addresses: a pointer formed from the image's
// generic pointer costs a v_add of its relocated address (0) per access.
__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) {
    return *(const __attribute__((address_space(3))) uint32_t *)(size_t)byte_addr;
}
typedef uint32_t lds_v2u __attribute__((ext_vector_type(2)));
typedef uint32_t lds_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 lds_word2(uint32_t byte_addr) {
    const lds_v2u v = *(const __attribute__((address_space(3))) lds_v2u *)(size_t)byte_addr;
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint4 lds_word4(uint32_t byte_addr) {
    const lds_v4u v = *(const __attribute__((address_space(3))) lds_v4u *)(size_t)byte_addr;
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

// The keys of thread tid in a pass-1 tile: the kPartKPT consecutive keys
// tile0 + kPartKPT * tid + j, so a whole tile is read as 16-B vectors (two per
// thread for packed keys, four for entry_t runs); a short last tile by guarded
// scalar loads.  Which thread hashes which key does not matter to the sort,
// and the probe's slots are indexed by the key's place in the tile.
template <int LAYOUT, int TB>
__device__ __forceinline__ void load_tile_keys(const KeySpan &ks, size_t tile, int tid,
                                               int32_t (&k)[kPartKPT]) {
    static_assert(kPartKPT == 8, "two int4 / four entry pairs per thread");
    const size_t i0 = tile * (size_t)(TB * kPartKPT) + (size_t)kPartKPT * tid;
    const bool full = (tile + 1) * (size_t)(TB * kPartKPT) <= ks.n;  // uniform per workgroup
    if constexpr (LAYOUT == KEYS_PACKED) {
        if (full) {
            const int4 *v = reinterpret_cast<const int4 *>(ks.base) + i0 / 4;
            const int4 a = v[0], b = v[1];
            k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
            k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
            return;
        }
    } else if constexpr (LAYOUT == KEYS_ENTRY) {  // 16-B aligned entry_t run
        if (full) {
            const int4 *v = reinterpret_cast<const int4 *>(ks.base) + i0 / 2;
            const int4 a = v[0], b = v[1], c = v[2], d = v[3];
            k[0] = a.x; k[1] = a.z; k[2] = b.x; k[3] = b.z;
            k[4] = c.x; k[5] = c.z; k[6] = d.x; k[7] = d.z;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < kPartKPT; j++) {
        const size_t i = i0 + j;
        k[j] = i < ks.n ? load_key<LAYOUT>(ks, i) : 0;
    }
}

// Bijective block -> work-unit map that gives each XCD a contiguous range of
// units (cdna_hip_programming.md §5.5 T1, bijective form for n % 8 != 0).
__device__ __forceinline__ unsigned xcd_remap(unsigned x, unsigned n) {
    constexpr unsigned kXcds = 8;
    const unsigned q = n / kXcds, r = n % kXcds;
    const unsigned xcd = x % kXcds, idx = x / kXcds;
    // XCD xcd owns units [start, start + q + (xcd < r)).
    const unsigned start = xcd * q + min(xcd, r);
    return start + idx;
}

// Pass-1 tile of persistent block x in round k: each round covers the next
// gridDim.x tiles, dealt so that every XCD takes a contiguous range of them
// (segment-major run-start stores then fill whole lines in one L2).  ntiles
// when the block has no tile in that round.
__device__ __forceinline__ size_t part_tile(size_t k, size_t ntiles) {
    const size_t base = k * gridDim.x;
    if (base >= ntiles) return ntiles;
    const size_t nr = min((size_t)gridDim.x, ntiles - base);
    return blockIdx.x < nr ? base + xcd_remap(blockIdx.x, (unsigned)nr) : ntiles;
}

// The segment of position p (SegMap: a shift, then an exact multiply-high
// division, checked on the host for every shifted value): two instructions,
// no branch.
template <typename P>
__device__ __forceinline__ uint32_t seg_of(P p, const SegMap &sm) {
    return __umulhi((uint32_t)(p >> sm.shift), sm.magic);
}

// A pass-1 histogram bin b starts at b << kBinShift and counts in steps of 4,
// so the rank atomic returns (b << kBinShift) + 4 * rank: (that >> 17) is the
// byte address 4b of the bin's offset (4 * rank < 4 * 3 * 8192 < 2^17), and
// no VALU touches the atomic's result before the scatter (its wait sits at the
// barrier).  After the scan bin b holds its BYTE offset into the sorted image
// minus b << kBinShift, so bin + rank value is the entry's byte slot.
constexpr uint32_t kBinShift = 19;  // 8192 segments << 19 < 2^32

// Outputs: pos_out[tile * kTileKeys ..] (u64), the tile's entries sorted by
// segment, packed three per u64; segment b's run of the tile (start | end
// << 16, b = 0..nbins-1): COLS = true: straight into the segment-major table
// runs[b * ntiles + tile]; COLS = false: into the tile-major
// runs[tile * nbins + b], for k_runs_transpose (large tables).
constexpr int kModFast = 0, kModWide = 1, kModP2 = 2, kModLadder = 3, kModLadder0 = 4;
// plan_build's one-member ladder with the block relabelled to (x >> 24) % d
// (bloom_math.h mod_p2_hi24; ladder0_relabel): C2 and C5
constexpr int kModLadder0R = 5;

// The bin (segment) of one raw hash and its pass-1 entry (the position's low
// kEntryBits bits, or the ladder's packed form), by reduction MK: pass 1's
// whole per-position arithmetic after the hash (tools/ubench.py prices it
// alone as the compute ceiling of pass 1).
template <int MK, int MINW>
__device__ __forceinline__ void bin_entry(uint64_t raw, const ModParams &mp, const SegMap &sm,
                                          uint32_t &b, uint32_t &ent) {
    if constexpr (MK == kModWide) {
        const uint64_t p = mod_wide(raw, mp);
        b = seg_of(p, sm);
        ent = (uint32_t)p & kEntryMask;
    } else if constexpr (MK == kModLadder) {
        // ladder stack (StackTable::lad): bin = hash bits
        // [s, s+u), entry = (a_max << hb | bits [s+u, t_max))
        // << s | bits [0, s) with a_max = (x >> t_max) % d
        const uint32_t xl = (uint32_t)raw;
        const uint32_t a = mod_p2_hi(raw, mp);
        b = __builtin_amdgcn_ubfe(xl, sm.shift, sm.lad_u);
        const uint32_t ehi =
            (a << sm.lad_hb) + __builtin_amdgcn_ubfe(xl, sm.scaled_shift, sm.lad_hb);
        ent = (ehi << sm.shift) | __builtin_amdgcn_ubfe(xl, 0, sm.shift);
    } else if constexpr (MK == kModLadder0) {
        // one-member ladder (plan_build): bin = hash bits
        // [s, t), entry = a << s | bits [0, s)
        const uint32_t xl = (uint32_t)raw;
        if constexpr (MINW >= 6) {
            // at the 80-VGPR cap of three workgroups per CU
            // the plain form spilled 50 VGPRs
            const uint32_t lo = __builtin_amdgcn_ubfe(xl, 0, sm.shift);
            b = __builtin_amdgcn_ubfe(xl, sm.shift, sm.lad_u);
            ent = lshl_or_s(mod_p2_hi(raw, mp), sm.shift, lo);
        } else {
            // (C5's pass 1: 229 us, against 256 for the pinned
            // form above and for segments)
            const uint32_t a = mod_p2_hi(raw, mp);
            b = __builtin_amdgcn_ubfe(xl, sm.shift, sm.lad_u);
            ent = (a << sm.shift) | __builtin_amdgcn_ubfe(xl, 0, sm.shift);
        }
    } else if constexpr (MK == kModLadder0R) {
        // as kModLadder0 with a' = (x >> 24) % d for a = (x >> t) % d: one
        // shift and one v_sad_u8 instead of an alignbit, a shift and the sad
        // (pass 2 maps image block a' back to a, ladder0_block)
        const uint32_t xl = (uint32_t)raw;
        if constexpr (MINW >= 6) {
            const uint32_t lo = __builtin_amdgcn_ubfe(xl, 0, sm.shift);
            b = __builtin_amdgcn_ubfe(xl, sm.shift, sm.lad_u);
            ent = lshl_or_s(mod_p2_hi24(raw, mp), sm.shift, lo);
        } else {
            const uint32_t a = mod_p2_hi24(raw, mp);
            b = __builtin_amdgcn_ubfe(xl, sm.shift, sm.lad_u);
            ent = (a << sm.shift) | __builtin_amdgcn_ubfe(xl, 0, sm.shift);
        }
    } else if constexpr (MK == kModP2) {
        const uint32_t xl = (uint32_t)raw;
        const uint32_t r = mod_p2_hi(raw, mp);
        const uint32_t q = (r << sm.p2_hi_shift) |
                           __builtin_amdgcn_ubfe(xl, sm.shift, sm.p2_hi_shift);
        b = __umulhi(q, sm.magic);
        ent = xl & kEntryMask;
    } else {
        // the remainder still scaled by 2^l: the entry is a
        // bit-field of it, and one shift reaches the segment
        const uint32_t ru = mod_fast_scaled(raw, mp);
        b = __umulhi(ru >> sm.scaled_shift, sm.magic);
        ent = __builtin_amdgcn_ubfe(ru, mp.l, kEntryBits);
    }
}

// A 16-B non-temporal store (pass 1's sorted tiles beyond the Infinity Cache).
__device__ __forceinline__ void nt_store16(uint4 *p, const uint4 &v) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(p));
}

// ABL (micro-benchmarks only, tools/ubench.py p1abl: the pass's cost by
// stage): 0 the whole tile; 1 hash + bin and entry only; 2 + the rank
// atomics; 3 + the scan and the run table; 4 + the scatter; 5 + the packing,
// without the sorted tile's stores.  A stage's unconsumed results go to one
// store that only an impossible value takes.
template <int LAYOUT, bool SLOTS, bool COLS, int TB, int MK, int MAXB = 0, int MINW = 4,
          int ABL = 0, bool NT = false>
__global__ void __launch_bounds__(TB, MINW) k_part_bin(KeySpan ks, ModParams mp,
                                                       uint64_t *__restrict__ pos_out,
                                                       uint32_t *__restrict__ runs, SegMap sm,
                                                       size_t ntiles, uint16_t *__restrict__ slots) {
    constexpr int kTileKeys = TB * kPartKPT;
    constexpr int kTilePos = 3 * kTileKeys;
    constexpr int kMaxB = MAXB ? MAXB : TB >= 1024 ? (int)kPartMaxBinsBig : (int)kPartMaxBins;
    constexpr int kScanPer = (kMaxB + 1 + TB - 1) / TB;  // scan entries per thread, at most
    static_assert(4 * kTilePos <= (1 << 17) && kTilePos < (1 << 16) &&
                      ((uint64_t)(kMaxB - 1) << kBinShift) < (1ull << 32),
                  "packed rank fields (bin nbins, never incremented, may wrap to 0)");
    // static LDS even for the 96 KiB of an 8192-key tile (gfx950 takes it);
    // dynamic LDS or a pointer to it made the compiler spill registers here
    __shared__ __attribute__((aligned(16))) uint32_t s_sorted[kTilePos];
    __shared__ uint32_t s_hist[kMaxB + 1];
    __shared__ uint32_t s_wsum[TB / 64];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int nb = (int)sm.nbins;
    const int per = (nb + 1 + TB - 1) / TB;  // this launch's scan entries per thread
    int32_t kcur[kPartKPT], knext[kPartKPT];

    // One tile.  FULL (every tile but a short last one) makes the key count a
    // constant: no per-key guards, and a fixed number of vector-memory ops
    // after the next tile's key loads, so the wait for those keys at the top
    // of the next tile is vmcnt(#stores) instead of a drain of every store.
    // Those loads are issued after the run-start stores for that reason.
    auto do_tile = [&](auto full_c, size_t tile, size_t next) {
        constexpr bool FULL = decltype(full_c)::value;
        const size_t tile0 = tile * kTileKeys;
        const int tile_keys = FULL ? (int)kTileKeys : (int)min((size_t)kTileKeys, ks.n - tile0);
        auto live = [&](int j) { return FULL || kPartKPT * tid + j < tile_keys; };
#pragma clang loop unroll(disable) vectorize(disable)
        for (int b = tid; b <= nb; b += TB) s_hist[b] = (uint32_t)b << kBinShift;
        lds_barrier();  // also: the previous tile's s_sorted reads are done

        // 1. positions -> (segment, rank in segment) and the entry; the ranks
        //    are not consumed before the barrier, so all 24 LDS atomics of a
        //    thread stay in flight behind the hashing.
        uint32_t br[kPartKPT * 3];   // (segment << kBinShift) + 4 * rank
        uint32_t ent[kPartKPT * 3];  // low kEntryBits bits of the position
#pragma unroll
        for (int j = 0; j < kPartKPT; j++) {
            if (live(j)) {
                const int32_t k = kcur[j];
#pragma unroll
                for (int h = 0; h < 3; h++) {
                    const uint64_t raw = h == 0 ? raw_hash1(k) : h == 1 ? raw_hash2(k) : raw_hash3(k);
                    uint32_t b, e;
                    bin_entry<MK, MINW>(raw, mp, sm, b, e);
                    ent[3 * j + h] = e;
                    if constexpr (ABL == 1) br[3 * j + h] = b;
                    else br[3 * j + h] = atomicAdd(&s_hist[b], 4u);
                }
            } else {
#pragma unroll
                for (int h = 0; h < 3; h++) br[3 * j + h] = ent[3 * j + h] = 0;
            }
        }
        lds_barrier();
        // (ablation: the stage's results consumed by one impossible store)
        auto consume = [&]() {
            uint32_t x = 0;
#pragma unroll
            for (int q = 0; q < 3 * kPartKPT; q++) x ^= br[q] + ent[q];
            if (x == 0x9E3779B9u) reinterpret_cast<uint32_t *>(pos_out)[tile * kTileKeys + tid] = x;
        };
        if constexpr (ABL == 1 || ABL == 2) {
            if (next < ntiles) load_tile_keys<LAYOUT, TB>(ks, next, tid, knext);
            consume();
            return;
        }

        // 2. exclusive scan of the nbins+1 counts (the extra slot is 0 and
        //    receives the tile total); thread t owns [t*per, t*per + per).
        //    Waves that own no bin (C2: waves 5-7 of 8) skip it: nobody
        //    reads their wave sums, which come after every live bin.
        const bool scan_wave = wave * 64 * per <= nb;  // uniform per wave
        uint32_t local[kScanPer];  // 4 * count of bin b
        uint32_t tsum = 0, incl = 0;
        if (scan_wave) {
#pragma unroll
            for (int q = 0; q < kScanPer; q++) {
                const int b = tid * per + q;
                local[q] = (q < per && b <= nb) ? s_hist[b] - ((uint32_t)b << kBinShift) : 0u;
                tsum += local[q];
            }
            incl = wave_incl_scan(tsum);
            if (lane == 63) s_wsum[wave] = incl;
        }
        lds_barrier();
        if (scan_wave) {
            uint32_t run = incl - tsum;
            for (int w = 0; w < wave; w++) run += s_wsum[w];
#pragma unroll
            for (int q = 0; q < kScanPer; q++) {
                const int b = tid * per + q;
                if (q < per && b <= nb) {
                    // biased by -(b << kBinShift): bin + rank value = byte slot
                    s_hist[b] = run - ((uint32_t)b << kBinShift);
                    // segment b's run of this tile, [start, end) in entries,
                    // packed start | end << 16 (both < 3 * 8192), straight
                    // from the scan's registers: segment-major column or
                    // tile-major row
                    const uint32_t pk = (run >> 2) | (((run + local[q]) >> 2) << 16);
                    if (b < nb) {
                        if constexpr (COLS) runs[(size_t)b * ntiles + tile] = pk;
                        else runs[tile * (size_t)nb + b] = pk;
                    }
                    run += local[q];
                }
            }
        }
        lds_barrier();
        if (next < ntiles) load_tile_keys<LAYOUT, TB>(ks, next, tid, knext);
        if constexpr (ABL == 3) {
            consume();
            return;
        }

        // 3. scatter into the LDS image sorted by segment, one hash at a time:
        //    its kPartKPT offset reads first (one wait), then the writes.
        //    Byte addresses throughout (the histogram holds byte offsets).
        const char *hist_b = reinterpret_cast<const char *>(s_hist);
        char *sorted_b = reinterpret_cast<char *>(s_sorted);
#pragma unroll
        for (int h = 0; h < 3; h++) {
            uint32_t slot[kPartKPT];  // byte offset in the sorted image
#pragma unroll
            for (int j = 0; j < kPartKPT; j++)
                slot[j] = *reinterpret_cast<const uint32_t *>(hist_b + (br[3 * j + h] >> 17)) +
                          br[3 * j + h];
#pragma unroll
            for (int j = 0; j < kPartKPT; j++)
                if (live(j)) *reinterpret_cast<uint32_t *>(sorted_b + slot[j]) = ent[3 * j + h];
            if constexpr (SLOTS) {
                // key kPartKPT*tid + j's sorted index, one 16-B store per hash
                uint16_t *sl = slots + (tile * 3 + h) * kTileKeys + kPartKPT * tid;
                if (FULL) {
                    uint32_t w[kPartKPT / 2];
#pragma unroll
                    for (int q = 0; q < kPartKPT / 2; q++)  // slots are byte offsets: 4 | slot
                        w[q] = lshl_or(slot[2 * q + 1], 14, slot[2 * q] >> 2);
                    // non-temporal: the slots are read once, by the combine
                    // after pass 2, and kept out of the caches they leave the
                    // sorted entries pass 2 is about to read (C3 pass 1
                    // 108 -> 96 us, the whole probe 283 -> 262 us)
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u wv = {w[0], w[1], w[2], w[3]};
                    __builtin_nontemporal_store(wv, reinterpret_cast<v4u *>(sl));
                } else {
#pragma unroll
                    for (int j = 0; j < kPartKPT; j++)
                        if (live(j)) sl[j] = (uint16_t)(slot[j] >> 2);
                }
            }
        }
        lds_barrier();
        if constexpr (ABL == 4) return;
        // 4. the sorted tile goes out packed, three entries per u64, as 16-B
        //    stores: thread t packs entries 6v .. 6v+5 for its vectors v.  In
        //    a short tile the entries past its end are stale, masked so they
        //    cannot spill into a neighbour field (pass 2 never uses them).
        uint4 *dst = reinterpret_cast<uint4 *>(pos_out + tile * (size_t)kTileKeys);
        constexpr int kVecs = kTileKeys / 2;  // 16-B vectors per tile
        constexpr int kStores = kVecs / TB;
        static_assert(kStores * TB == kVecs, "whole vectors per thread");
        uint4 v[kStores];
#pragma unroll
        for (int r = 0; r < kStores; r++) {
            const uint2 *src = reinterpret_cast<const uint2 *>(s_sorted + 6 * (r * TB + tid));
            const uint2 a = src[0], b = src[1], c = src[2];
            uint32_t e[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
            if constexpr (!FULL) {
                // past the tile's positions: 0, not stale (the ladder probe's
                // pass 2 reads with every entry of a vector, its run's or not)
#pragma unroll
                for (int q = 0; q < 6; q++) e[q] = 6 * (r * TB + tid) + q < 3 * tile_keys ? e[q] & kEntryMask : 0u;
            }
            // (a << s) | b is one v_lshl_or_b32; the compiler emitted a shift
            // and an or for each (5 instead of 3 per u64)
            v[r] = make_uint4(lshl_or(e[1], 21, e[0]), lshl_or(e[2], 10, e[1] >> 11),
                              lshl_or(e[4], 21, e[3]), lshl_or(e[5], 10, e[4] >> 11));
        }
        if constexpr (ABL == 0) {
            if constexpr (NT) {
                // sorted tiles beyond the Infinity Cache (C5: 512 MiB): stored
                // non-temporal, so they do not evict what pass 2 can use
                // there (C5 build 0.419 -> 0.406 ms; below it, C2's 128 MiB,
                // pass 2 reads them from the cache: 35 us, 48 from HBM; a
                // runtime choice in the kernel spilled 3-4 VGPRs)
#pragma unroll
                for (int r = 0; r < kStores; r++) nt_store16(dst + r * TB + tid, v[r]);
            } else {
#pragma unroll
                for (int r = 0; r < kStores; r++) dst[r * TB + tid] = v[r];
            }
        } else {
            // keep the packing: a store only when an impossible value shows
#pragma unroll
            for (int r = 0; r < kStores; r++)
                if (v[r].x == 0xFFFFFFFFu && v[r].y == 0xFFFFFFFFu) dst[r * TB + tid] = v[r];
        }
    };

    // Full tiles in the loop; the short last tile (index ntiles - 1, always
    // in a block's final round) after it, so the loop sees only FULL.
    const size_t nfull = ks.n / kTileKeys;
    size_t tile = part_tile(0, ntiles);
    if (tile < ntiles) load_tile_keys<LAYOUT, TB>(ks, tile, tid, kcur);
    size_t round = 0;
    for (; tile < nfull; round++) {
        const size_t next = part_tile(round + 1, ntiles);
        do_tile(BoolC<true>{}, tile, next);
#pragma unroll
        for (int j = 0; j < kPartKPT; j++) kcur[j] = knext[j];
        tile = next;
    }
    if (tile < ntiles) do_tile(BoolC<false>{}, tile, ntiles);
}

// ---------------------------------------------------------------------------
// pass 1 on super-tiles (k_part_bin2, builds with many short runs: C4): one
// 1024-thread workgroup sorts a tile of kSuperTileKeys = 16,384 keys, two
// halves of 8,192 (A, B), so each segment's run of a tile is twice as long
// as k_part_bin's (C4: ~20 entries against ~10) and there are half as many
// (tile, segment) pairs for pass 2 to walk and half the run table.  Neither
// the sorted tile (49,152 entries, 192 KiB as u32) nor every position's
// entry and rank in registers fit (96 live values per thread spilled ~100
// VGPRs at the 128 of 4 waves per SIMD), so:
//   1. A's positions: bin + entry (bin_entry), rank in the JOINT histogram
//      (the rank atomic's return stays in a register), the key's three
//      entries packed into one u64 of an LDS stash (64 KiB, the thread's own
//      column: conflict-free);
//   2. B's positions: the same, entries kept in registers;
//   3. one scan of the joint counts: segment b's run of the super-tile is
//      [off(b), off(b + 1)), written to the run table;
//   4. every entry's index in the sorted super-tile, f = off(b) + rank (one
//      LDS read);
//   5. two phases of 24,576 sorted entries each: the entries whose f falls
//      in the phase (A's taken from the stash) are written to the 96 KiB LDS
//      image at f - phase base, which goes out packed as k_part_bin's.
// The histogram and the scan's wave sums live in the image's space (both
// are dead before the first phase writes): stash + image = all 160 KiB.
// Ranks reach 49,151, so the rank field is 18 bits: bins at << 20 (at most
// 4,095 bins), the bin's byte address is (rank value) >> 18.
// ---------------------------------------------------------------------------
constexpr uint32_t kBinShift2 = 20;
constexpr int kSuperBlock = 1024;

template <int LAYOUT>
__device__ __forceinline__ void load_half_keys(const KeySpan &ks, size_t tile, int half, int tid,
                                               int32_t (&k)[kPartKPT]) {
    constexpr size_t kHalf = (size_t)kSuperBlock * kPartKPT;
    const size_t i0 = tile * kSuperTileKeys + half * kHalf + (size_t)kPartKPT * tid;
    const bool full = tile * kSuperTileKeys + (half + 1) * kHalf <= ks.n;  // uniform per workgroup
    if constexpr (LAYOUT == KEYS_PACKED) {
        if (full) {
            const int4 *v = reinterpret_cast<const int4 *>(ks.base) + i0 / 4;
            const int4 a = v[0], b = v[1];
            k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
            k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
            return;
        }
    } else if constexpr (LAYOUT == KEYS_ENTRY) {
        if (full) {
            const int4 *v = reinterpret_cast<const int4 *>(ks.base) + i0 / 2;
            const int4 a = v[0], b = v[1], c = v[2], d = v[3];
            k[0] = a.x; k[1] = a.z; k[2] = b.x; k[3] = b.z;
            k[4] = c.x; k[5] = c.z; k[6] = d.x; k[7] = d.z;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < kPartKPT; j++) {
        const size_t i = i0 + j;
        k[j] = i < ks.n ? load_key<LAYOUT>(ks, i) : 0;
    }
}

// SLOTS (the stacked probe's pass 1 on super-tiles): also each key's sorted
// index per hash, u16 (< 49,152), in the slot plane [tile][hash][key] the
// combine reads.
template <int LAYOUT, bool COLS, int MK, int MAXB, bool SLOTS = false>
__global__ void __launch_bounds__(kSuperBlock, 4) k_part_bin2(KeySpan ks, ModParams mp,
                                                              uint64_t *__restrict__ pos_out,
                                                              uint32_t *__restrict__ runs, SegMap sm,
                                                              size_t ntiles, uint16_t *__restrict__ slots) {
    constexpr int TB = kSuperBlock;
    constexpr int kHalfKeys = TB * kPartKPT;          // 8192
    constexpr int kTileKeys = 2 * kHalfKeys;          // 16384
    constexpr int kTilePos = 3 * kTileKeys;           // 49152
    constexpr int kPhasePos = kTilePos / 2;           // 24576 entries: 96 KiB
    constexpr uint32_t kPhaseBytes = 4u * kPhasePos;
    constexpr int kScanPer = (MAXB + 1 + TB - 1) / TB;
    constexpr int kPer = 3 * kPartKPT;                // positions per thread and half
    constexpr int kStashWords = 2 * kHalfKeys;        // one u64 per key of half A
    static_assert(4 * kTilePos <= (1 << 18) && kTilePos < (1 << 16) &&
                      ((uint64_t)MAXB << kBinShift2) < (1ull << 32),
                  "rank fields (the bin nbins, never incremented, included)");
    static_assert(kSuperTileKeys == (size_t)kTileKeys, "super-tile size");
    static_assert(MAXB + 1 + TB / 64 <= kPhasePos, "histogram and wave sums inside the image");
    // [image: kPhasePos][stash: kStashWords], histogram + wave sums at the
    // image's start until the phases.  The image first: an entry's slot is
    // then its LDS byte address (no add per write), and the stash is reached
    // through the offset field
    __shared__ __attribute__((aligned(16))) uint32_t s_pool[kPhasePos + kStashWords];
    uint32_t *img = s_pool;
    uint2 *stash = reinterpret_cast<uint2 *>(s_pool + kPhasePos);
    uint32_t *s_hist = img;
    uint32_t *s_wsum = img + MAXB + 1;
    char *img_b = reinterpret_cast<char *>(img);
    const char *hist_b = reinterpret_cast<const char *>(s_hist);

    const int nb = (int)sm.nbins;
    const int per = (nb + 1 + TB - 1) / TB;
    int32_t kA[kPartKPT], kB[kPartKPT];

    auto do_tile = [&](auto full_c, size_t tile, size_t next) {
        constexpr bool FULL = decltype(full_c)::value;
        // The thread index, opaque per tile: what derives from it (the scan's
        // bins and run-table pointers, stash and image addresses) is formed
        // in the tile, not hoisted out of the tile loop into ~30 registers
        // that the 128-VGPR cap then spilled.
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, wave = tid >> 6;
        const size_t tile0 = tile * kTileKeys;
        const int tile_keys = FULL ? kTileKeys : (int)min((size_t)kTileKeys, ks.n - tile0);
        auto live = [&](int half, int j) { return FULL || half * kHalfKeys + kPartKPT * tid + j < tile_keys; };
        // B's keys load under A's hashing (needed only after it)
        load_half_keys<LAYOUT>(ks, tile, 1, tid, kB);
        lds_barrier();  // the previous tile's image and stash reads are done
#pragma clang loop unroll(disable) vectorize(disable)
        for (int b = tid; b <= nb; b += TB) s_hist[b] = (uint32_t)b << kBinShift2;
        lds_barrier();

        // 1. A: rank in the joint histogram, the key's entries to the stash
        uint32_t brA[kPer], brB[kPer], eB[2 * kPartKPT];
#pragma unroll
        for (int j = 0; j < kPartKPT; j++) {
            uint32_t e[3];
#pragma unroll
            for (int h = 0; h < 3; h++) {
                const int q = 3 * j + h;
                e[h] = 0;
                if (live(0, j)) {
                    const uint64_t raw = h == 0 ? raw_hash1(kA[j]) : h == 1 ? raw_hash2(kA[j]) : raw_hash3(kA[j]);
                    uint32_t b;
                    bin_entry<MK, 4>(raw, mp, sm, b, e[h]);
                    brA[q] = atomicAdd(&s_hist[b], 4u);
                } else {
                    brA[q] = 0;
                }
            }
            stash[j * TB + tid] = make_uint2(lshl_or(e[1], 21, e[0]), lshl_or(e[2], 10, e[1] >> 11));
            __builtin_amdgcn_sched_barrier(0);
        }
        // 2. B: the same, the key's entries kept packed (two registers for
        //    three entries: the unpacked 24 spilled)
#pragma unroll
        for (int j = 0; j < kPartKPT; j++) {
            uint32_t e[3];
#pragma unroll
            for (int h = 0; h < 3; h++) {
                const int q = 3 * j + h;
                e[h] = 0;
                if (live(1, j)) {
                    const uint64_t raw = h == 0 ? raw_hash1(kB[j]) : h == 1 ? raw_hash2(kB[j]) : raw_hash3(kB[j]);
                    uint32_t b;
                    bin_entry<MK, 4>(raw, mp, sm, b, e[h]);
                    brB[q] = atomicAdd(&s_hist[b], 4u);
                } else {
                    brB[q] = 0;
                }
            }
            eB[2 * j] = lshl_or(e[1], 21, e[0]);
            eB[2 * j + 1] = lshl_or(e[2], 10, e[1] >> 11);
            __builtin_amdgcn_sched_barrier(0);
        }
        lds_barrier();

        // 3. exclusive scan of the joint counts (k_part_bin step 2)
        const bool scan_wave = wave * 64 * per <= nb;
        uint32_t local[kScanPer];
        uint32_t tsum = 0, incl = 0;
        if (scan_wave) {
#pragma unroll
            for (int q = 0; q < kScanPer; q++) {
                const int b = tid * per + q;
                local[q] = (q < per && b <= nb) ? s_hist[b] - ((uint32_t)b << kBinShift2) : 0u;
                tsum += local[q];
            }
            incl = wave_incl_scan(tsum);
            if (lane == 63) s_wsum[wave] = incl;
        }
        lds_barrier();
        if (scan_wave) {
            uint32_t run = incl - tsum;
            for (int w = 0; w < wave; w++) run += s_wsum[w];
#pragma unroll
            for (int q = 0; q < kScanPer; q++) {
                const int b = tid * per + q;
                if (q < per && b <= nb) {
                    s_hist[b] = run - ((uint32_t)b << kBinShift2);
                    const uint32_t pk = (run >> 2) | (((run + local[q]) >> 2) << 16);
                    if (b < nb) {
                        if constexpr (COLS) runs[(size_t)b * ntiles + tile] = pk;
                        else runs[tile * (size_t)nb + b] = pk;
                    }
                    run += local[q];
                }
            }
        }
        lds_barrier();
        if (next < ntiles) load_half_keys<LAYOUT>(ks, next, 0, tid, kA);

        // 4. every entry's byte slot in the sorted super-tile (dead: ~0, in
        //    no phase); in groups of 6 (the scheduler would otherwise issue
        //    all 48 reads first, into 48 more registers)
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            const uint32_t fa = *reinterpret_cast<const uint32_t *>(hist_b + (brA[q] >> 18)) + brA[q];
            const uint32_t fb = *reinterpret_cast<const uint32_t *>(hist_b + (brB[q] >> 18)) + brB[q];
            brA[q] = live(0, q / 3) ? fa : ~0u;
            brB[q] = live(1, q / 3) ? fb : ~0u;
            // formed here: the compiler otherwise defers the add into both
            // phases and keeps the read offset and the rank value apart
            // (two registers per entry instead of one)
            asm volatile("" : "+v"(brA[q]), "+v"(brB[q]));
            if (q % 6 == 5) __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (SLOTS) {
            // key 8 tid + j of half A and 8192 + 8 tid + j of half B: their
            // sorted index per hash, one non-temporal 16-B store per half and
            // hash (read once, by the combine, after pass 2)
            uint16_t *sl = slots + tile * 3 * (size_t)kTileKeys + kPartKPT * tid;
            if constexpr (FULL) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int h = 0; h < 3; h++) {
                    // byte slots: 4 | slot, so (odd << 14) | (even >> 2)
                    const v4u wa = {lshl_or(brA[3 + h], 14, brA[h] >> 2), lshl_or(brA[9 + h], 14, brA[6 + h] >> 2),
                                    lshl_or(brA[15 + h], 14, brA[12 + h] >> 2),
                                    lshl_or(brA[21 + h], 14, brA[18 + h] >> 2)};
                    const v4u wb = {lshl_or(brB[3 + h], 14, brB[h] >> 2), lshl_or(brB[9 + h], 14, brB[6 + h] >> 2),
                                    lshl_or(brB[15 + h], 14, brB[12 + h] >> 2),
                                    lshl_or(brB[21 + h], 14, brB[18 + h] >> 2)};
                    __builtin_nontemporal_store(wa, reinterpret_cast<v4u *>(sl + h * kTileKeys));
                    __builtin_nontemporal_store(wb, reinterpret_cast<v4u *>(sl + h * kTileKeys + kHalfKeys));
                }
            } else {
#pragma unroll
                for (int j = 0; j < kPartKPT; j++) {
#pragma unroll
                    for (int h = 0; h < 3; h++) {
                        if (live(0, j)) sl[h * kTileKeys + j] = (uint16_t)(brA[3 * j + h] >> 2);
                        if (live(1, j)) sl[h * kTileKeys + kHalfKeys + j] = (uint16_t)(brB[3 * j + h] >> 2);
                    }
                }
            }
        }
        lds_barrier();  // the histogram is read: the image is free

        // 5. two phases of kPhasePos sorted entries through the LDS image
        uint4 *dst = reinterpret_cast<uint4 *>(pos_out + tile * (size_t)kTileKeys);
        constexpr int kVecs = kPhasePos / 6;  // 16-B vectors per phase
        constexpr int kStores = kVecs / TB;
        static_assert(kStores * TB == kVecs, "whole vectors per thread");
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const uint32_t base = ph * kPhaseBytes;
            // the stash words of all 8 keys first (one wait), then the
            // conditional writes: a read inside each branch waited for the
            // LDS round trip once per entry
            uint2 w[kPartKPT];
#pragma unroll
            for (int j = 0; j < kPartKPT; j++) w[j] = stash[j * TB + tid];
#pragma unroll
            for (int j = 0; j < kPartKPT; j++) {
#pragma unroll
                for (int h = 0; h < 3; h++) {
                    const uint32_t la = brA[3 * j + h] - base;
                    if (la < kPhaseBytes) {
                        const uint32_t e = h == 0 ? w[j].x & kEntryMask
                                         : h == 1 ? __builtin_amdgcn_alignbit(w[j].y, w[j].x, 21) & kEntryMask
                                                  : w[j].y >> 10;
                        *reinterpret_cast<uint32_t *>(img_b + la) = e;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kPartKPT; j++) {
#pragma unroll
                for (int h = 0; h < 3; h++) {
                    const uint32_t lb = brB[3 * j + h] - base;
                    if (lb < kPhaseBytes) {
                        const uint32_t lo = eB[2 * j], hi = eB[2 * j + 1];
                        const uint32_t e = h == 0 ? lo & kEntryMask
                                         : h == 1 ? __builtin_amdgcn_alignbit(hi, lo, 21) & kEntryMask
                                                  : hi >> 10;
                        *reinterpret_cast<uint32_t *>(img_b + lb) = e;
                    }
                }
            }
            lds_barrier();
#pragma unroll
            for (int r = 0; r < kStores; r++) {
                const uint2 *src = reinterpret_cast<const uint2 *>(img + 6 * (r * TB + tid));
                const uint2 a = src[0], b = src[1], c = src[2];
                uint32_t e[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
                if constexpr (!FULL) {
#pragma unroll
                    for (int z = 0; z < 6; z++) e[z] &= kEntryMask;
                }
                // (plain stores: non-temporal ones, as k_part_bin's at C5, made
                // C4's pass 1 slower, 1.299 -> 1.317 ms, more than pass 2 gained)
                dst[ph * kVecs + r * TB + tid] =
                    make_uint4(lshl_or(e[1], 21, e[0]), lshl_or(e[2], 10, e[1] >> 11),
                               lshl_or(e[4], 21, e[3]), lshl_or(e[5], 10, e[4] >> 11));
            }
            if (ph == 0) lds_barrier();  // phase 0's image is read before phase 1 writes
        }
    };

    const size_t nfull = ks.n / kTileKeys;
    size_t tile = part_tile(0, ntiles);
    if (tile < ntiles) load_half_keys<LAYOUT>(ks, tile, 0, (int)threadIdx.x, kA);
    size_t round = 0;
    for (; tile < nfull; round++) {
        const size_t next = part_tile(round + 1, ntiles);
        do_tile(BoolC<true>{}, tile, next);
        tile = next;
    }
    if (tile < ntiles) do_tile(BoolC<false>{}, tile, ntiles);
}

// ---------------------------------------------------------------------------
// run-table transpose: pass 1 writes one row of nbins packed runs per tile
// (contiguous, cheap); pass 2 wants, per segment, its run bounds of all tiles
// contiguous.  A 64 x 64 LDS-tiled transpose: 256-B coalesced reads and
// writes, the LDS tile padded one word per row against bank conflicts.
// Small tables are written straight from pass 1 as columns (COLS): at C2
// (4 MiB) that costs ~2 us against ~6 us for a transpose launch.  Large ones
// go through the transpose: at C4 (805 MB) the column stores cost ~2.1 ms
// (partial-line write-backs), the transpose 0.39 ms (tools/ubench.py part*).
// ---------------------------------------------------------------------------
constexpr size_t kColumnTableMaxBytes = 16u << 20;  // larger run tables: rows + transpose
constexpr int kTransposeTile = 64;
constexpr int kTransposeBlock = 256;

// ---------------------------------------------------------------------------
// partition pass 2 (k_part_apply): workgroup b ORs segment b's run of every
// tile into an LDS image of the segment (S bits), then writes the segment
// out with plain 16-B stores (OR-merged with the old bitmap when that may be
// non-zero).  Segments never overlap, so no atomics leave the CU.
// ---------------------------------------------------------------------------

constexpr int kApplyBlock = 1024;
// pass 2's prologue: loads per thread in flight while an LDS image is staged
constexpr int kStageBatch = 4;
constexpr int kApplyDepth = 2;  // lane-group loads per wave per batch

// Lanes per tile for pass 2, from the average run length L = tile entries /
// nbins: a step reads 6G entries of a tile (G lanes x one 16-B vector);
// runs longer than a step finish in the wave-uniform tail loop.  Measured
// (tools/ubench.py part*, G x depth sweep): G = 4 wins from runs of 8 (C4)
// to 48 entries (C2, C5): C2 38 us vs 66 at G = 8 and 47 at G = 2.
inline int apply_lanes_per_tile(size_t nbins, size_t tile_pos = kPartTilePos) {
    const size_t L = tile_pos / (nbins ? nbins : 1);
    if (L < 96) return 4;
    if (L < 192) return 8;
    if (L < 384) return 16;
    return 32;
}

// MODE kApplyBuild: OR every entry into the zeroed LDS image, write the
// segment.  kApplyProbe: the LDS image is the filter's segment; each entry's
// bit is written as one result byte at the entry's own index in the sorted
// tile (res[tile*kTilePos + index]), so the result stores follow the runs
// like the loads.  kApplyStack: LDS holds bits [b*w, (b+1)*w) mod m_j of
// every stack member j (StackTable), the result byte carries member j's bit
// at bit j.
//
// The walk: G consecutive lanes share one tile and read its run as 16-B
// vectors (two packed u64 = six entries), lane j of the group taking the
// vector that holds the run's first entry + j, so one load instruction
// covers 64/G tiles x 6G entries.  An entry is this segment's exactly when
// its index lies in [run start, run end) (the bounds are already in the
// lane's registers); its offset is (entry - b*S) mod 2^21.  Lanes of tiles
// past the end re-read the last tile, which ORs / writes the same values
// twice.  A wave owns batches of kApplyDepth load groups; the next batch's
// run bounds are loaded while the current one is applied, and the rare tile
// whose run outlasts the first step is finished by a wave-uniform loop.
constexpr int kApplyBuild = 0, kApplyProbe = 1, kApplyStack = 2, kApplyLadder = 3;
// kApplyBuildL: a build on plan_build's one-member ladder (bins = hash bits):
// the entry is the image offset itself, and the image's d blocks go to
// a << t | b << s (StackTable::lad's s, t[0], d).
constexpr int kApplyBuildL = 4;

template <int MODE, int G, int TILE_KEYS, int BLOCK = kApplyBlock, int DEPTH = kApplyDepth,
          int WALK = 0, int NF = 0, int LK = 0>
__global__ void __launch_bounds__(BLOCK) k_part_apply(
    const uint64_t *__restrict__ pos, const uint32_t *__restrict__ run_starts, int ntiles,
    int nbins, uint32_t seg_bits, uint64_t m, uint32_t *__restrict__ words, uint64_t nw32,
    int merge_existing, uint8_t *__restrict__ res, StackTable st) {
    constexpr bool PROBE = MODE != kApplyBuild && MODE != kApplyBuildL;
    static_assert(G >= 1 && G <= 64 && (64 % G) == 0, "G lanes per tile");
    constexpr int kTilePos = 3 * TILE_KEYS;
    constexpr int kTPI = 64 / G;                 // tiles per load instruction
    constexpr int kBatchTiles = kTPI * DEPTH;   // tiles per wave batch
    constexpr uint32_t kLastVec = TILE_KEYS / 2 - 1;

    const uint32_t seg_words = seg_bits / 32;
    extern __shared__ __attribute__((aligned(16))) uint32_t seg[];
    // Neighbouring segments' runs share 128-B lines of every sorted tile and
    // of the run-start rows, so give consecutive segments to workgroups on one
    // XCD (blocks are dealt round-robin over the 8 XCDs): a bijection on
    // [0, nbins); placement only affects speed.
    // One segment b per workgroup, or (the stacked probe with a segment
    // stride S, StackTable::seg_stride; a compile-time 0 for every other
    // mode) segments c, c + S, c + 2S, ...: members whose windows repeat with
    // a period dividing S (StackTable::keep_mask) are staged for the first
    // of them only.  Only at G = 4 (short runs, many segments) and up to 7
    // compiled-in members: the loop took 64 -> 68 VGPRs at 8 members and
    // 62 -> 65 at G = 8 with 5, which leaves one 1024-lane workgroup per CU.
    constexpr bool kStrided = MODE == kApplyStack && NF < 8 && G == 4;
    const int seg_stride = kStrided ? st.seg_stride : 0;
    uint32_t stage_mask = ~0u;
    for (int b = (int)xcd_remap(blockIdx.x, seg_stride ? (unsigned)seg_stride : (unsigned)nbins);;) {
    {
    // the thread index laundered per segment in the strided loop, which
    // otherwise hoists thread-dependent addresses out of it (52 -> 61 VGPRs)
    uint32_t tix = threadIdx.x;
    if constexpr (kStrided) asm volatile("" : "+v"(tix));
    const uint64_t w0 = (uint64_t)b * seg_words;
    const int nseg = (int)(min(nw32, w0 + seg_words) - w0);  // last segment may be short
    const uint64_t base = (uint64_t)b * seg_bits;
    const uint32_t base21 = (uint32_t)base & kEntryMask;
    if constexpr (MODE == kApplyStack) {
        // member j's bits (b*w + o) mod m_j for o < w: the w bits from
        // (b*w) mod m_j on, wrapping at m_j (w <= m_j; w and m_j are
        // multiples of 128 bits, so no 16-B vector straddles the wrap)
        // Word-interleaved image: member j's word p at seg[p * nf + j], so an
        // entry's nf words sit together and one address (+ immediate offsets)
        // reaches all of them.
        const int nf = NF ? NF : st.nf;  // NF: the member count as a compile-time constant
        for (int j = 0; j < nf; j++) {
            if (!((stage_mask >> j) & 1u)) continue;  // its window is already in LDS
            const uint32_t mw = st.mwords[j];
            const uint32_t start = (uint32_t)(((uint64_t)b * seg_words) % mw);
            const uint4 *src = reinterpret_cast<const uint4 *>(st.words[j]);
            const int nvec = (int)seg_words / 4;
            // kStageBatch vectors per thread in flight before their LDS
            // stores; past the end a lane reloads its own first vector (no
            // load under a branch, and no one address every lane hits); a
            // load-store loop waited for each load in turn
            for (int i0 = tix; i0 < nvec; i0 += kStageBatch * BLOCK) {
                uint4 v[kStageBatch];
#pragma unroll
                for (int k = 0; k < kStageBatch; k++) {
                    const int ik = i0 + k * BLOCK;
                    uint32_t wi = start + 4u * (uint32_t)(ik < nvec ? ik : i0);
                    if (wi >= mw) wi -= mw;
                    v[k] = src[wi / 4];
                }
#pragma unroll
                for (int k = 0; k < kStageBatch; k++) {
                    const int i = i0 + k * BLOCK;
                    if (i < nvec) {
                        uint32_t *dst = seg + (size_t)(4 * i) * nf + j;
                        dst[0] = v[k].x;
                        dst[nf] = v[k].y;
                        dst[2 * nf] = v[k].z;
                        dst[3 * nf] = v[k].w;
                    }
                }
            }
        }
    } else if constexpr (MODE == kApplyLadder) {
        // bin b's blocks of the direct members (StackTable::lad), block q at
        // LDS word q << (s - 5); the table: row e (member 0's block, the
        // entry's bits above s) holds rs words, one 32-bit LDS byte address
        // each: the other direct members' blocks and the packed image's
        // tuple; the tuple map: per tuple, the first bit of each packed
        // member's block; then the packed image, bpp bits per position and
        // tuple.  With a computed tuple (LK = 0) there is no table, and the
        // tuple map lives in member 0's area until member 0 is staged.
        const LadderTable &L = st.lad;
        // direct members (L.k, compiled in); LK = 0: one, and the packed
        // tuple computed from the entry (LadderTable::ctup: no table)
        constexpr uint32_t K = LK == 0 ? 1 : LK;
        constexpr bool CT = LK == 0;
        constexpr uint32_t BPP = (uint32_t)NF - K <= 4 ? 4u : 8u;
        const uint32_t bv = L.s - 7;  // log2 of 16-B vectors per block
        const uint32_t bin = (uint32_t)b;
        // first bit of block i of member j for this bin
        auto first_bit = [&](uint32_t j, uint32_t i) -> uint32_t {
            const uint32_t tj = L.t[j];
            if (tj >= L.s + L.u) {
                const uint32_t hj = tj - L.s - L.u;
                return ((i >> hj) << tj) + ((i & ((1u << hj) - 1u)) << (L.s + L.u)) + (bin << L.s);
            }
            return (i << tj) + ((bin & ((1u << (tj - L.s)) - 1u)) << L.s);
        };
        // block of member j given a = (x >> t_j) % d and xs = hash bits [s, t)
        // for some t >= t_j (bits [s + u, t_j) of x are bits [u, t_j - s) of xs)
        auto block_of = [&](uint32_t j, uint32_t aj, uint32_t xs) -> uint32_t {
            const uint32_t tj = L.t[j];
            if (tj < L.s + L.u) return aj;
            const uint32_t hj = tj - L.s - L.u;
            return (aj << hj) | ((xs >> L.u) & ((1u << hj) - 1u));
        };
        // (one load per iteration: batching these loads, as the segment
        // stack's staging does, made C3's probe 0.170 -> 0.180 ms)
        auto stage_direct = [&]() {
            for (uint32_t j = 0; j < K; j++) {
                const uint4 *src = reinterpret_cast<const uint4 *>(st.words[j]);
                uint4 *dst = reinterpret_cast<uint4 *>(seg) + ((size_t)L.base[j] << bv);
                for (uint32_t q = tix; q < (L.nblk[j] << bv); q += BLOCK)
                    dst[q] = src[(first_bit(j, q >> bv) >> 7) + (q & ((1u << bv) - 1u))];
            }
        };
        if constexpr (!CT) stage_direct();
        uint32_t *tbl = seg + L.img_words;
        // the tuple map follows the table; with a computed tuple (no table,
        // the images fill the LDS) it sits where member 0's blocks go, which
        // are staged after the packed image is built from it
        uint32_t *tmap = CT ? seg : tbl + L.ne * L.rs;
        constexpr uint32_t kTupleShift = BPP == 4 ? 0u : 1u;  // tuple words = 2^(s-3+this)
        for (uint32_t e = CT ? L.ne : tix; e < L.ne; e += BLOCK) {
            const uint32_t amax = e >> L.hb;
            const uint32_t xs = ((e & ((1u << L.hb) - 1u)) << L.u) | bin;  // hash bits [s, t_max)
            for (uint32_t j = 1; j < (uint32_t)NF && j <= K; j++) {
                const uint32_t tj = L.t[j];
                const uint32_t aj = (amax * L.pmod[j] + (xs >> (tj - L.s)) % L.d) % L.d;
                const uint32_t ij = block_of(j, aj, xs);
                // direct member j: its block's LDS byte address; member K:
                // the packed tuple's
                tbl[e * L.rs + (j - 1)] = j < K ? (L.base[j] + ij) << (L.s - 3)
                                                : (L.pk_words + (ij << (L.s - 3 + kTupleShift))) << 2;
            }
        }
        if constexpr (K < (uint32_t)NF) {
            const uint32_t tk = L.t[K < (uint32_t)kMaxStack ? K : 0], ntup = L.nblk[K];
            for (uint32_t tp = tix; tp < ntup; tp += BLOCK) {
                // tuple tp = member K's block: a_K and hash bits [s, t_K)
                uint32_t ak, xs;
                if (tk >= L.s + L.u) {
                    const uint32_t hk = tk - L.s - L.u;
                    ak = tp >> hk;
                    xs = ((tp & ((1u << hk) - 1u)) << L.u) | bin;
                } else {
                    ak = tp;
                    xs = bin & ((1u << (tk - L.s)) - 1u);
                }
                for (uint32_t j = K; j < (uint32_t)NF; j++) {
                    const uint32_t aj = (ak * L.pmodk[j] + (xs >> (L.t[j] - L.s)) % L.d) % L.d;
                    tmap[8 * tp + (j - K)] = first_bit(j, block_of(j, aj, xs));
                }
            }
        }
        __syncthreads();
        if constexpr (K < (uint32_t)NF) {
            // packed image: thread task = (tuple, 32 positions): one 32-bit
            // read per packed member, spread to bpp-bit fields
            const uint32_t cps = 1u << (L.s - 5);  // 32-position chunks per tuple
            const uint32_t ntask = L.nblk[K] * cps;
            uint32_t *pk = seg + L.pk_words;
            for (uint32_t q = tix; q < ntask; q += BLOCK) {
                const uint32_t tp = q >> (L.s - 5), c = q & (cps - 1u);
                uint32_t w[NF];
#pragma unroll
                for (int j = 0; j < NF; j++)
                    w[j] = (uint32_t)j >= K ? st.words[j][(tmap[8 * tp + (j - K)] >> 5) + c] : 0u;
                uint32_t *dst = pk + q * BPP;
                if constexpr (BPP == 4) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        uint32_t o = 0;
#pragma unroll
                        for (int j = 0; j < NF; j++) {
                            if ((uint32_t)j < K) continue;
                            uint32_t x = (w[j] >> (8 * r)) & 0xFFu;  // positions 8r .. 8r+7
                            x = (x | (x << 12)) & 0x000F000Fu;
                            x = (x | (x << 6)) & 0x03030303u;
                            x = (x | (x << 3)) & 0x11111111u;  // bit i at 4i
                            o |= x << (j - K);
                        }
                        dst[r] = o;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 8; r++) {
                        uint32_t o = 0;
#pragma unroll
                        for (int j = 0; j < NF; j++) {
                            if ((uint32_t)j < K) continue;
                            uint32_t x = (w[j] >> (4 * r)) & 0xFu;  // positions 4r .. 4r+3
                            x = (x | (x << 14)) & 0x00030003u;
                            x = (x | (x << 7)) & 0x01010101u;  // bit i at 8i
                            o |= x << (j - K);
                        }
                        dst[r] = o;
                    }
                }
            }
        }
        if constexpr (CT) {
            __syncthreads();  // the tuple map's last reads
            stage_direct();
        }
    } else if constexpr (MODE == kApplyProbe) {
        for (int i = tix; i < (int)seg_words; i += BLOCK)
            seg[i] = i < nseg ? words[w0 + i] : 0u;
    } else {
        for (int i = tix; i < (int)seg_words / 4; i += BLOCK)
            reinterpret_cast<uint4 *>(seg)[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();

    const int lane = tix & 63;
    const int wave = tix >> 6;
    const uint32_t sub = (uint32_t)(lane % G);  // this lane's vector in its tile's step
    const int tl = lane / G;                    // this lane's tile in a load group
    const int nbatch = (ntiles + kBatchTiles - 1) / kBatchTiles;

    // Run bounds travel packed (start | end << 16) until they are used: a
    // decode right after the prefetching load makes the compiler wait for
    // it there, i.e. for every load issued before it, the entry-vector
    // prefetch included (that wait made the packed table slower than two
    // u32 columns: C2 pass 2 36 -> 41 us, C4 1.22 -> 1.56 ms).
    auto dec = [](uint32_t pk) { return make_uint2(pk & 0xFFFFu, pk >> 16); };
    // The walk visits tiles last to first (data tile rt(t) for walk step t):
    // pass 1 wrote them first to last, so the most recently written sorted
    // tiles -- the ones still in the Infinity Cache -- are read first (C5
    // pass 2 205 -> 197.5 us, C2 unchanged, profiles/r04/reverse_walk/).
    auto rt = [&](int t) -> int { return ntiles - 1 - t; };
    auto bounds = [&](int j, uint32_t (&r)[DEPTH]) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            const int t = j * kBatchTiles + d * kTPI + tl;
            r[d] = t < ntiles ? run_starts[(size_t)b * ntiles + rt(t)] : 0u;
        }
    };
    // Vector vi of tile t; lanes past the tile's last vector load that one
    // but keep their own vi, so none of its entries counts for them (a
    // clamped index would make up to G-1 lanes OR the same words, and those
    // same-address LDS atomics serialise the segments at a tile's end).
    auto load = [&](int t, uint32_t vi) -> uint4 {
        return reinterpret_cast<const uint4 *>(pos + (size_t)rt(t) * TILE_KEYS)[min(vi, kLastVec)];
    };
    // The vector a lane loads for its step at vector vi of a run ending at
    // entry `end`, group base vector vb.  WALK 2 (short runs): a lane whose
    // vector lies past the run's end loads the group's first vector instead
    // -- a line the group reads anyway, so the wave instruction touches fewer
    // distinct lines (C4's ~10-entry runs span 2-3 of a group's 4 vectors:
    // pass 2 1190 -> 1158 us).  The lane keeps its own vi for the entry
    // mask, so none of what it loaded counts.  Longer runs keep the plain
    // load: there the vector past a run's end starts the neighbour
    // segment's run, which an XCD neighbour reads next from the same L2
    // (C2 pass 2 35.5 -> 39.5 us with the redirect, profiles/r05/redirect/).
    auto vload = [&](uint32_t vi, uint32_t vb, uint32_t end) -> uint32_t {
        if constexpr (WALK >= 2) return 6 * vi < end ? vi : vb;
        return vi;
    };
    // The six entries of vector vi of tile t; run = [r.x, r.y).
    auto apply6 = [&](const uint4 &v, int t, uint32_t vi, const uint2 &r) {
        const uint32_t e[6] = {v.x & kEntryMask, __builtin_amdgcn_alignbit(v.y, v.x, 21) & kEntryMask,
                               v.y >> 10,        v.z & kEntryMask,
                               __builtin_amdgcn_alignbit(v.w, v.z, 21) & kEntryMask, v.w >> 10};
        const uint32_t i0 = 6 * vi - r.x, len = r.y - r.x;  // entry k is in the run iff i0 + k < len
        if constexpr (!PROBE) {
            // Branch-free: the run's entries among the six form the 6-bit
            // mask vm; an entry outside the run ORs 0.  The word's LDS byte
            // address is ((e - base) mod 2^21) / 32 * 4 (the segment image
            // starts at LDS address 0: the kernel has no static LDS, which
            // launch_apply_g checks before the first launch; an address
            // taken from seg's pointer costs a v_add of the image's
            // relocated address, 0, per entry) and the
            // bit index the low 5 bits of e - base, which the shift takes as
            // they are.
            const int s0 = (int)(6 * vi) - (int)r.x;          // entry 0's place in the run
            const int lo = max(-s0, 0), hi = min(max((int)r.y - (int)(6 * vi), 0), 6);
            const uint32_t vm = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            // WALK 3 (super-tiles): a lane whose vector holds none of the
            // run's entries (a redirected load past the run's end: about half
            // of them at C4's ~20-entry runs) issues no atomics, so the
            // segment image's banks serve only the lanes with bits to set
            if (WALK < 1 || vm != 0) {
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const uint32_t d = MODE == kApplyBuildL ? e[k] : e[k] - base21;
                    const uint32_t addr = (d >> 3) & ((kEntryMask >> 3) & ~3u);
                    const uint32_t bit = __builtin_amdgcn_ubfe(vm, k, 1) << (d & 31);
                    __attribute__((address_space(3))) uint32_t *w =
                        (__attribute__((address_space(3))) uint32_t *)(size_t)addr;
                    __hip_atomic_fetch_or(w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        } else {
            // the run's entries among the six, as the build's 6-bit mask
            // (round 6: once per vector instead of a compare and an OR per entry)
            const int s0 = (int)(6 * vi) - (int)r.x;
            const int lo = max(-s0, 0), hi = min(max((int)r.y - (int)(6 * vi), 0), 6);
            const uint32_t mask = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            (void)i0;
            (void)len;
            uint32_t bits[6];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const uint32_t ok = __builtin_amdgcn_ubfe(mask, k, 1);
                if constexpr (MODE == kApplyLadder) {
                    // member 0's block is the entry's high part (its blocks
                    // come first at LDS 0, 2^(s-3) bytes each), so its word's
                    // byte address is (e >> 3) & ~3; the table row gives the
                    // other direct members' block addresses and the packed
                    // tuple's (block and tuple bases are aligned, so the
                    // offsets OR in).  Bit extracts take the entry itself
                    // as the shift: v_bfe_u32 uses its low 5 bits.
                    const LadderTable &L = st.lad;
                    constexpr int K = LK == 0 ? 1 : LK;  // direct members, compiled in
                    constexpr bool CT = LK == 0;          // packed tuple computed, no table
                    // An entry outside the run is another run's (or 0 past a
                    // short tile's end: k_part_bin writes zeros there), so
                    // its high part is a block this bin stages and its reads
                    // stay in the image; its result bits are not stored
                    // (round 6: the select cost a VALU per entry)
                    const uint32_t ee = e[k];
                    (void)ok;
                    const uint32_t a0 = (ee >> 3) & ~3u;
                    uint32_t acc = __builtin_amdgcn_ubfe(lds_word(a0), ee, 1u);
                    if constexpr (CT) {
                        // tuple = member 1's block = hi mod nblk[1] (LadderTable::ctup)
                        const uint32_t hi = ee >> L.s;
                        const uint32_t tup =
                            (uint32_t)((int)hi + __mul24((int)__umulhi(hi, L.tmagic), -(int)L.nblk[1]));
                        uint32_t pa, psh;
                        if constexpr (NF - 1 <= 4) {  // 8 positions per word, tuples of 2^(s-1) bytes
                            pa = ((ee >> 1) & ((1u << (L.s - 1)) - 4u)) | ((tup << (L.s - 1)) + 4 * L.pk_words);
                            psh = ee << 2;
                        } else {  // 4 positions per word, tuples of 2^s bytes
                            pa = (ee & ((1u << L.s) - 4u)) | ((tup << L.s) + 4 * L.pk_words);
                            psh = ee << 3;
                        }
                        acc |= __builtin_amdgcn_ubfe(lds_word(pa), psh, (uint32_t)(NF - 1)) << 1;
                    } else if constexpr (K > 1 || K < NF) {
                        constexpr int RW = (K - 1) + (K < NF ? 1 : 0);  // row words used
                        constexpr int RS = RW <= 1 ? 1 : RW <= 2 ? 2 : RW <= 4 ? 4 : 8;  // = L.rs
                        const uint32_t row = L.img_words * 4 + (ee >> L.s) * (4 * RS);  // byte address
                        uint32_t rw[RW];
                        if constexpr (RW == 1) {
                            rw[0] = lds_word(row);
                        } else if constexpr (RW == 2) {
                            const uint2 v2 = lds_word2(row);
                            rw[0] = v2.x;
                            rw[1] = v2.y;
                        } else {
#pragma unroll
                            for (int q = 0; q < RW; q += 4) {
                                const uint4 v4 = lds_word4(row + 4 * q);
                                const uint32_t vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                                for (int r = 0; r < 4; r++)
                                    if (q + r < RW) rw[q + r] = vv[r];
                            }
                        }
                        const uint32_t wmask = (1u << (L.s - 3)) - 4u;  // word offset in a block
#pragma unroll
                        for (int j = 1; j < K; j++) {
                            const uint32_t wj = lds_word((a0 & wmask) | rw[j - 1]);
                            acc |= __builtin_amdgcn_ubfe(wj, ee, 1u) << j;
                        }
                        if constexpr (K < NF) {
                            uint32_t pa, psh;
                            if constexpr (NF - K <= 4) {  // 8 positions per word: (lo >> 3) words
                                pa = ((ee >> 1) & ((1u << (L.s - 1)) - 4u)) | rw[K - 1];
                                psh = ee << 2;
                            } else {  // 4 positions per word: (lo >> 2) words
                                pa = (ee & ((1u << L.s) - 4u)) | rw[K - 1];
                                psh = ee << 3;
                            }
                            const uint32_t pw = lds_word(pa);
                            acc |= __builtin_amdgcn_ubfe(pw, psh, (uint32_t)(NF - K)) << K;
                        }
                    }
                    bits[k] = acc;
                    continue;
                }
                const uint32_t o = ok ? (e[k] - base21) & kEntryMask : 0u;  // reads stay in the image
                if constexpr (MODE == kApplyStack) {
                    const uint32_t sh = o & 31;
                    uint32_t acc = 0;
                    if constexpr (NF > 0) {  // straight-line: NF reads at immediate offsets
                        const uint32_t *wp = seg + (o >> 5) * (uint32_t)NF;
#pragma unroll
                        for (int j = 0; j < NF; j++) acc |= __builtin_amdgcn_ubfe(wp[j], sh, 1u) << j;
                    } else {
                        const uint32_t *wp = seg + __umul24(o >> 5, (uint32_t)st.nf);
#pragma unroll
                        for (int j = 0; j < kMaxStack; j++)  // member j's word at immediate offset 4j
                            if (j < st.nf) acc |= __builtin_amdgcn_ubfe(wp[j], sh, 1u) << j;
                    }
                    bits[k] = acc;
                } else {
                    bits[k] = (seg[o >> 5] >> (o & 31)) & 1u;
                }
            }
            // six result bytes at 6*vi (2-byte aligned): whole pairs as
            // 2-byte stores, a run's edge byte by byte
            uint8_t *p = res + (size_t)rt(t) * kTilePos + 6 * vi;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const uint32_t mq = (mask >> (2 * q)) & 3u;
                if (mq == 3u) {
                    *reinterpret_cast<uint16_t *>(p + 2 * q) =
                        (uint16_t)(bits[2 * q] | (bits[2 * q + 1] << 8));
                } else if (mq == 1u) {
                    p[2 * q] = (uint8_t)bits[2 * q];
                } else if (mq == 2u) {
                    p[2 * q + 1] = (uint8_t)bits[2 * q + 1];
                }
            }
        }
    };

    if constexpr (WALK >= 4 && WALK <= 6) {
        // WALK 1 / 3 / 2's walks for builds (round 6: WALK 4 / 5 / 6),
        // restated for fewer instructions per step: unrolled over two
        // register sets (the old loops copy their carried state at the
        // back-edge: seven moves a step), the vector and run-bound loads
        // addressed from uniform bases by 32-bit byte offsets (the sorted
        // tiles span < 4 GiB: the launchers check), so a step forms a load
        // address in two instructions instead of eight 64-bit ones, and a
        // run's end kept in vectors (the step test multiplies nothing).
        // Lanes past the last tile hold an empty run (r = 0).  NV vectors
        // per lane and step (WALK 5: two, for super-tiles' ~20-entry runs);
        // REDIR (WALK 5, 6: short runs): a lane whose vector lies past the
        // run's end loads the group's first vector instead (WALK 2's note).
        // Not launched: WALK 4 against WALK 1 was 1 % faster in the pass-2
        // micro-benchmark but 4 % slower in the bench (C2 35.2 -> 36.7 us,
        // profiles/r06/rejected/walk4_bench/), WALK 5 against WALK 3 on C4's
        // super-tiles 806 against 796 us (profiles/r06/rejected/walk5_c4/).
        static_assert(!PROBE, "builds");
        constexpr int NV = WALK == 5 ? 2 : 1;
        constexpr bool REDIR = WALK >= 5;
        constexpr int kGroupsPerWave = 64 / G;
        const int Q = kGroupsPerWave * (BLOCK / 64);
        constexpr uint32_t kVecShift = __builtin_ctz((unsigned)TILE_KEYS / 2);  // vectors per tile, log2
        const char *pos_b = reinterpret_cast<const char *>(pos);
        const char *col_b = reinterpret_cast<const char *>(run_starts + (size_t)b * ntiles);
        auto bnd = [&](int tt) -> uint32_t {
            return tt < ntiles ? *reinterpret_cast<const uint32_t *>(col_b + ((uint32_t)rt(tt) << 2)) : 0u;
        };
        auto vec = [&](uint32_t tv, uint32_t vi) -> uint4 {
            return *reinterpret_cast<const uint4 *>(pos_b + ((tv + min(vi, kLastVec)) << 4));
        };
        auto tvec = [&](int t) -> uint32_t { return (uint32_t)rt(min(t, ntiles - 1)) << kVecShift; };
        auto ceil6 = [](uint32_t x) { return (x + 5u) / 6u; };
        struct St {
            int t;        // walk step: tile rt(t)
            uint32_t r;   // its run, start | end << 16 (0: none)
            uint32_t rn;  // the run of tile t + Q
            uint32_t vb;  // the group's first vector of this step
            uint32_t ev;  // the run's end in vectors, ceil(end / 6)
            uint32_t tv;  // the tile's first vector
            uint4 v[NV];  // this lane's vectors of the step: vb + sub + G k
        };
        auto loads = [&](St &s) {
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const uint32_t vi = s.vb + sub + G * k;
                s.v[k] = vec(s.tv, REDIR && vi >= s.ev ? s.vb : vi);
            }
        };
        St A, B;
        A.t = wave * kGroupsPerWave + tl;
        A.r = bnd(A.t);
        A.rn = bnd(A.t + Q);
        A.vb = (A.r & 0xFFFFu) / 6u;
        A.ev = ceil6(A.r >> 16);
        A.tv = tvec(A.t);
        loads(A);
        // the step after c into n (its loads issued first), then c applied
        auto step = [&](const St &c, St &n) {
            const uint32_t vb2 = c.vb + NV * G;
            const bool adv = vb2 >= c.ev;
            n.t = adv ? c.t + Q : c.t;
            n.r = adv ? c.rn : c.r;
            n.vb = adv ? (c.rn & 0xFFFFu) / 6u : vb2;
            n.ev = adv ? ceil6(c.rn >> 16) : c.ev;
            n.tv = adv ? tvec(c.t + Q) : c.tv;
            n.rn = c.rn;
            if (adv) n.rn = bnd(c.t + 2 * Q);
            loads(n);
            if (c.vb < c.ev) {
#pragma unroll
                for (int k = 0; k < NV; k++) apply6(c.v[k], c.t, c.vb + sub + G * k, dec(c.r));
            }
        };
        while (true) {
            if (__ballot(A.t < ntiles) == 0) break;
            step(A, B);
            if (__ballot(B.t < ntiles) == 0) break;
            step(B, A);
        }
    } else if constexpr (WALK == 1 || WALK == 2) {
        // Independent lane groups: group q (G lanes) walks tiles q, q + Q,
        // q + 2Q, ... one step (G vectors) per iteration, moving to its next
        // tile as soon as its run ends, so no group waits for the longest run
        // of a batch.  The next step's vector is loaded before the current
        // one is applied, and the next tile's run bounds one tile ahead.
        constexpr int kGroupsPerWave = 64 / G;
        const int Q = kGroupsPerWave * (BLOCK / 64);
        auto bnd = [&](int tt) -> uint32_t {  // packed; 0 = empty past the end
            return tt < ntiles ? run_starts[(size_t)b * ntiles + rt(tt)] : 0u;
        };
        // the current and the next tile's bounds both stay packed (a decode
        // of the next one as it becomes current would sit between its load
        // and its register: a copy, hence a wait)
        int t = wave * kGroupsPerWave + tl;
        uint32_t r = bnd(t), rn = bnd(t + Q);
        uint32_t vb = (r & 0xFFFFu) / 6u;  // the group's step base (vector index)
        uint4 v = load(min(t, ntiles - 1), vload(vb + sub, vb, r >> 16));
        while (__ballot(t < ntiles) != 0) {
            // state after this step: advance within the run or to the next
            // tile.  On a tile change the new lookahead bounds are loaded
            // straight into their loop register, before the next step's
            // vector, so the wait before the apply (vmcnt 1) leaves only that
            // vector in flight
            int t2 = t;
            uint32_t r2 = r, vb2 = vb + G;
            const bool adv = 6 * vb2 >= (r >> 16);
            if (adv) {
                t2 += Q;
                r2 = rn;
                vb2 = (r2 & 0xFFFFu) / 6u;
            }
            uint32_t rn2 = rn;
            if (adv) rn2 = bnd(t2 + Q);
            const uint4 v2 = load(min(t2, ntiles - 1), vload(vb2 + sub, vb2, r2 >> 16));
            if (t < ntiles && 6 * vb < (r >> 16)) apply6(v, t, vb + sub, dec(r));
            t = t2; r = r2; rn = rn2; vb = vb2; v = v2;
        }
    } else if constexpr (WALK >= 7) {
        // WALK 3 on two interleaved chains per lane group (round 6): chain c
        // walks the group's tiles q + c Q, q + (2 + c) Q, ..., both chains'
        // next vectors in flight together, so a lane holds four 16-B loads
        // and two run-bound loads in flight instead of two and one (C4's
        // entries come from HBM, not the Infinity Cache: its pass 2 waits on
        // load latency, one (tile, segment) pair per group step).  WALK 10:
        // WALK 1 (one vector per lane, no redirect) on two chains.
        constexpr int kGroupsPerWave = 64 / G;
        const int Q = kGroupsPerWave * (BLOCK / 64);
        constexpr int NC = WALK == 10 ? 2 : WALK - 5;  // WALK 7: 2 chains (launched), 8: 3, 9: 4 (slower)
        constexpr int NV = WALK == 10 ? 1 : 2;          // vectors per lane and step
        auto vl = [&](uint32_t vi, uint32_t vb, uint32_t end) -> uint32_t {
            if constexpr (WALK == 10) return vi;
            return vload(vi, vb, end);
        };
        auto bnd = [&](int tt) -> uint32_t {
            return tt < ntiles ? run_starts[(size_t)b * ntiles + rt(tt)] : 0u;
        };
        int t[NC];
        uint32_t r[NC], rn[NC], vb[NC];
        uint4 v[NC][NV];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            t[c] = wave * kGroupsPerWave + tl + c * Q;
            r[c] = bnd(t[c]);
            rn[c] = bnd(t[c] + NC * Q);
            vb[c] = (r[c] & 0xFFFFu) / 6u;
#pragma unroll
            for (int k = 0; k < NV; k++)
                v[c][k] = load(min(t[c], ntiles - 1), vl(vb[c] + k * G + sub, vb[c], r[c] >> 16));
        }
        auto live = [&]() {
            bool any = false;
#pragma unroll
            for (int c = 0; c < NC; c++) any |= t[c] < ntiles;
            return any;
        };
        while (__ballot(live()) != 0) {
            int t2[NC];
            uint32_t r2[NC], rn2[NC], vb2[NC];
            uint4 v2[NC][NV];
#pragma unroll
            for (int c = 0; c < NC; c++) {
                t2[c] = t[c];
                r2[c] = r[c];
                vb2[c] = vb[c] + NV * G;
                const bool adv = 6 * vb2[c] >= (r[c] >> 16);
                if (adv) {
                    t2[c] += NC * Q;
                    r2[c] = rn[c];
                    vb2[c] = (r2[c] & 0xFFFFu) / 6u;
                }
                rn2[c] = rn[c];
                if (adv) rn2[c] = bnd(t2[c] + NC * Q);
            }
#pragma unroll
            for (int c = 0; c < NC; c++)
#pragma unroll
                for (int k = 0; k < NV; k++)
                    v2[c][k] = load(min(t2[c], ntiles - 1), vl(vb2[c] + k * G + sub, vb2[c], r2[c] >> 16));
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (t[c] < ntiles && 6 * vb[c] < (r[c] >> 16)) {
#pragma unroll
                    for (int k = 0; k < NV; k++) apply6(v[c][k], t[c], vb[c] + k * G + sub, dec(r[c]));
                }
            }
#pragma unroll
            for (int c = 0; c < NC; c++) {
                t[c] = t2[c]; r[c] = r2[c]; rn[c] = rn2[c]; vb[c] = vb2[c];
#pragma unroll
                for (int k = 0; k < NV; k++) v[c][k] = v2[c][k];
            }
        }
    } else if constexpr (WALK == 3) {
        // The same walk with two vectors per lane per step (vectors vb + sub
        // and vb + G + sub: a step covers 12G entries), loads past a run's
        // end redirected as at WALK 2: runs a little longer than one G-vector
        // step (super-tiles: ~20 entries, 4-5 vectors) take one step.
        constexpr int kGroupsPerWave = 64 / G;
        const int Q = kGroupsPerWave * (BLOCK / 64);
        auto bnd = [&](int tt) -> uint32_t {
            return tt < ntiles ? run_starts[(size_t)b * ntiles + rt(tt)] : 0u;
        };
        int t = wave * kGroupsPerWave + tl;
        uint32_t r = bnd(t), rn = bnd(t + Q);
        uint32_t vb = (r & 0xFFFFu) / 6u;
        uint4 v = load(min(t, ntiles - 1), vload(vb + sub, vb, r >> 16));
        uint4 w = load(min(t, ntiles - 1), vload(vb + G + sub, vb, r >> 16));
        while (__ballot(t < ntiles) != 0) {
            int t2 = t;
            uint32_t r2 = r, vb2 = vb + 2 * G;
            const bool adv = 6 * vb2 >= (r >> 16);
            if (adv) {
                t2 += Q;
                r2 = rn;
                vb2 = (r2 & 0xFFFFu) / 6u;
            }
            uint32_t rn2 = rn;
            if (adv) rn2 = bnd(t2 + Q);
            const uint4 v2 = load(min(t2, ntiles - 1), vload(vb2 + sub, vb2, r2 >> 16));
            const uint4 w2 = load(min(t2, ntiles - 1), vload(vb2 + G + sub, vb2, r2 >> 16));
            if (t < ntiles && 6 * vb < (r >> 16)) {
                apply6(v, t, vb + sub, dec(r));
                apply6(w, t, vb + G + sub, dec(r));
            }
            t = t2; r = r2; rn = rn2; vb = vb2; v = v2; w = w2;
        }
    } else {
    uint32_t rp[DEPTH];  // this batch's bounds, packed
    if (wave < nbatch) bounds(wave, rp);
    for (int j = wave; j < nbatch; j += (BLOCK / 64)) {
        int t[DEPTH];
        uint32_t vi[DEPTH];
        uint4 v[DEPTH];
        uint2 r[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            r[d] = dec(rp[d]);
            t[d] = min(j * kBatchTiles + d * kTPI + tl, ntiles - 1);
            vi[d] = r[d].x / 6u + sub;
            v[d] = load(t[d], vload(vi[d], vi[d] - sub, r[d].y));
        }
        uint32_t rn[DEPTH];
        const int jn = j + (BLOCK / 64);
        if (jn < nbatch) bounds(jn, rn);
#pragma unroll
        for (int d = 0; d < DEPTH; d++) apply6(v[d], t[d], vi[d], r[d]);
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            for (uint32_t vn = r[d].x / 6u + sub + G; __ballot(6 * vn < r[d].y) != 0; vn += G)
                apply6(load(t[d], vload(vn, vn - sub, r[d].y)), t[d], vn, r[d]);
        }
#pragma unroll
        for (int d = 0; d < DEPTH; d++) rp[d] = rn[d];
    }
    }
    if constexpr (PROBE) {
        if constexpr (kStrided) goto segment_done;
        return;
    }
    __syncthreads();

    if constexpr (MODE == kApplyBuildL) {
        // block a of the image (2^s bits) is the bitmap's bits a << t | b << s;
        // with the relabelled pass 1 (LadderTable::rinv != 0) image block a'
        // is the bitmap's block ladder0_block(a', b)
        const uint32_t ls = st.lad.s, lt = st.lad.t[0];
        const uint32_t vpb = 1u << (ls - 7);  // 16-B vectors per block
        const uint4 *seg4 = reinterpret_cast<const uint4 *>(seg);
        uint4 *w4 = reinterpret_cast<uint4 *>(words);
        auto block = [&](uint32_t q) -> uint4 * {
            uint32_t a = q >> (ls - 7);
            const uint32_t i = q & (vpb - 1u);
            if (st.lad.rinv) a = ladder0_block(a, (uint32_t)b, ls, st.lad.d, st.lad.rinv);
            return w4 + (((size_t)a << (lt - 7)) + ((size_t)b << (ls - 7)) + i);
        };
        // (two loops: one loop with both stores under a branch had its
        // stores merged into one plain store; the segments' note below)
        if (merge_existing) {
            for (uint32_t q = tix; q < st.lad.d * vpb; q += BLOCK) {
                uint4 *dq = block(q);
                uint4 v = seg4[q];
                const uint4 o = *dq;
                v.x |= o.x; v.y |= o.y; v.z |= o.z; v.w |= o.w;
                *dq = v;
            }
        } else {
            for (uint32_t q = tix; q < st.lad.d * vpb; q += BLOCK) nt_store16(block(q), seg4[q]);
        }
        return;
    }

    uint32_t *dst = words + w0;
    if (nseg == (int)seg_words) {  // seg_words % 4 == 0 and w0 is 16-B aligned
        uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
        const uint4 *seg4 = reinterpret_cast<const uint4 *>(seg);
        if (merge_existing) {
            for (int q = tix; q < (int)seg_words / 4; q += BLOCK) {
                uint4 v = seg4[q];
                const uint4 o = dst4[q];
                v.x |= o.x; v.y |= o.y; v.z |= o.z; v.w |= o.w;
                dst4[q] = v;
            }
        } else {
            // a fresh filter's finished segment: stored non-temporal, for
            // later probes, not this build (the L2 and Infinity Cache keep the
            // keys and sorted tiles: C2 188.6 -> 191.3, C4 129.1 -> 130.3
            // Gkeys/s in the bench A/B); a merge stores plainly what it has
            // just read (re-reading a non-temporal bitmap in repeated merges
            // cost C2 0.0909 -> 0.0917 ms)
            for (int q = tix; q < (int)seg_words / 4; q += BLOCK) nt_store16(dst4 + q, seg4[q]);
        }
    } else {
        for (int i = tix; i < nseg; i += BLOCK) {
            uint32_t v = seg[i];
            if (merge_existing) v |= dst[i];
            dst[i] = v;
        }
    }
    }
    segment_done:
        if (!seg_stride) return;
        b += seg_stride;
        if (b >= nbins) return;
        stage_mask = ~st.keep_mask;
        __syncthreads();  // the walk's last image reads, before the next staging
    }
}

// Partitioned / stacked probe, last step (k_probe_combine): one workgroup per
// tile stages the tile's result bytes (sorted order) in LDS; thread t takes the
// 8 consecutive keys 8t .. 8t+7, reads their slots as one 16-B vector per hash
// (8-byte-per-lane loads of round 1 took the address unit 24 instructions per
// thread), ANDs each key's three bytes (bit j of the AND is filter j's is_set)
// and writes, per filter j, the byte of its 8 answers: key 8t + i at bit i of
// byte t of the tile's part of row rows.row[j] (the packed rows' bit order:
// bit i % 64 of word i / 64 is key i).  A wave's bytes are 64 contiguous bytes
// per row.  The bits of filter j are gathered out of the 8 AND bytes by two
// multiplies: with bytes b0..b3 (0/1 at bits 0, 8, 16, 24),
// (b * 0x01020408) >> 24 puts b_i at bit i and every other partial product
// below bit 24 or above bit 31 (no carries: those bits are distinct).
constexpr int kCombineKeys = 8;  // keys per thread (and pass: super-tiles take two)
template <int TILE_KEYS, int kCombineBlock>
__global__ void __launch_bounds__(kCombineBlock) k_probe_combine(
    const uint8_t *__restrict__ res, const uint16_t *__restrict__ slots, size_t n,
    uint64_t *__restrict__ out, size_t nw, StackTable rows) {
    constexpr int kTilePos = 3 * TILE_KEYS;
    constexpr int kPasses = TILE_KEYS / (kCombineBlock * kCombineKeys);
    static_assert(kPasses * kCombineBlock * kCombineKeys == TILE_KEYS, "8 keys per thread and pass");
    __shared__ __attribute__((aligned(16))) uint8_t s_r[kTilePos];
    const size_t tile = blockIdx.x;
    const size_t tile0 = tile * TILE_KEYS;
    const int tile_keys = (int)min((size_t)TILE_KEYS, n - tile0);
    uint4 va[kPasses], vb[kPasses], vc[kPasses];
#pragma unroll
    for (int ps = 0; ps < kPasses; ps++) {
        const int k0 = kCombineKeys * ((int)threadIdx.x + ps * kCombineBlock);
        const uint4 *sl = reinterpret_cast<const uint4 *>(slots + tile * 3 * TILE_KEYS + k0);
        va[ps] = sl[0];
        vb[ps] = sl[TILE_KEYS / 8];
        vc[ps] = sl[2 * (TILE_KEYS / 8)];
    }
    // the tile's result bytes: every load issued before any LDS store, at
    // clamped indices (no load under a branch; a load-store loop waited for
    // each load in turn)
    const uint4 *src = reinterpret_cast<const uint4 *>(res + tile * (size_t)kTilePos);
    constexpr int kResVec = kTilePos / 16, kResPer = (kResVec + kCombineBlock - 1) / kCombineBlock;
    uint4 rv[kResPer];
#pragma unroll
    for (int j = 0; j < kResPer; j++) rv[j] = src[min((int)threadIdx.x + j * kCombineBlock, kResVec - 1)];
#pragma unroll
    for (int j = 0; j < kResPer; j++)
        if ((int)threadIdx.x + j * kCombineBlock < kResVec)
            reinterpret_cast<uint4 *>(s_r)[threadIdx.x + j * kCombineBlock] = rv[j];
    __syncthreads();
#pragma unroll
    for (int ps = 0; ps < kPasses; ps++) {
        const int k0 = kCombineKeys * ((int)threadIdx.x + ps * kCombineBlock);  // this pass's first key
        // live keys of a short last tile; past them the slots are stale
        const uint32_t a[4] = {va[ps].x, va[ps].y, va[ps].z, va[ps].w},
                       b[4] = {vb[ps].x, vb[ps].y, vb[ps].z, vb[ps].w},
                       c[4] = {vc[ps].x, vc[ps].y, vc[ps].z, vc[ps].w};
        uint32_t hit[kCombineKeys];
#pragma unroll
        for (int i = 0; i < kCombineKeys; i++) {
            const int sh = 16 * (i & 1);
            const uint32_t sa = (a[i / 2] >> sh) & 0xFFFFu, sb = (b[i / 2] >> sh) & 0xFFFFu,
                           sc = (c[i / 2] >> sh) & 0xFFFFu;
            hit[i] = k0 + i < tile_keys ? (uint32_t)(s_r[min(sa, (uint32_t)kTilePos - 1)] &
                                                     s_r[min(sb, (uint32_t)kTilePos - 1)] &
                                                     s_r[min(sc, (uint32_t)kTilePos - 1)])
                                        : 0u;
        }
        // bytes of the tile's rows that hold keys: whole 64-key words, so the
        // last word of a short tile gets its zero bits too
        if (k0 >= ((tile_keys + 63) & ~63)) continue;
        const uint32_t lo = hit[0] | (hit[1] << 8) | (hit[2] << 16) | (hit[3] << 24);
        const uint32_t hi = hit[4] | (hit[5] << 8) | (hit[6] << 16) | (hit[7] << 24);
        const size_t byte0 = tile0 / 8 + threadIdx.x + ps * kCombineBlock;
#pragma unroll
        for (int j = 0; j < kMaxStack; j++) {
            if (j < rows.nf) {
                const uint32_t bl = ((lo >> j) & 0x01010101u) * 0x01020408u;
                const uint32_t bh = ((hi >> j) & 0x01010101u) * 0x01020408u;
                const uint32_t byte = (bl >> 24) | ((bh >> 20) & 0xF0u);
                reinterpret_cast<uint8_t *>(out + (size_t)rows.row[j] * nw)[byte0] = (uint8_t)byte;
            }
        }
    }
}

// The page of key k in a run (src/run.cpp:97-99): upper_bound over the run's
// n >= 1 fences (staged in LDS at fz) minus 1, for k >= fences[0] (the range
// check passed).  One interpolation guess from the run's first fence (f0) and
// fence spacing (scale = (n - 1) / (last - first)) places a window of
// kRouteWindow fences; two reads check that the answer is inside it, and 4
// branchless halving steps find it there; when the check fails, a binary
// search over the whole run does (exact either way, only slower).
constexpr int kRouteWindow = 15;  // fences; answers a .. a + 15: 4 halving steps
// A page guess is clamped to [0, 2^24] in float before it becomes an int
// (exact in float; a run has < 2^24 fences: n < 2^32 / kFenceStride).
constexpr float kGuessMax = 16777216.0f;

__device__ __forceinline__ int route_page(const int32_t *fz, int n, int32_t k, float f0, float scale) {
    int a = 0;
    bool ok = true;
    if (n > kRouteWindow) {
        const float gf = ((float)k - f0) * scale;
        // clamped in float first: a float-to-int conversion out of int range
        // is undefined (tight fences make the product huge); any guess past
        // the run's end is clamped to the last window below anyway
        const int g = (int)fminf(fmaxf(gf, 0.0f), kGuessMax);
        a = min(max(g - kRouteWindow / 2, 0), n - kRouteWindow);
        // the answer is in [a, a + 15] iff fences[a - 1] <= k and
        // fences[a + 15] > k (a window at either end passes that side)
        const int32_t fl = fz[max(a - 1, 0)], fh = fz[min(a + kRouteWindow, n - 1)];
        ok = (a == 0 || fl <= k) && (a + kRouteWindow >= n || fh > k);
    }
    int lo = a;
#pragma unroll
    for (int st = 8; st >= 1; st >>= 1) {  // fences at index >= n count as > k
        const int idx = lo + st - 1;
        if (idx < n && fz[min(idx, n - 1)] <= k) lo += st;
    }
    if (!ok) {  // the guess missed (rare): binary search the whole run
        int l = 1, h = n;
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (fz[mid] <= k) l = mid + 1;
            else h = mid;
        }
        lo = l;
    }
    return lo - 1;
}

// Routing fused into the stacked probe's combine (§8f row 1, Run::get's test
// src/run.cpp:93-99 over the runs LSMTree::get visits, src/lsm_tree.cpp:
// 141-216), when every run of the call is a member of one stack: each key's
// member bits (the combine's AND byte) are range-checked against its runs'
// [first fence, max key] right here, the newest candidate run is the lowest
// set bit, its page comes from the fences staged in LDS, and the candidate
// rows leave range-checked -- the rows are not written by the combine and
// read back by k_route.  Persistent workgroups stage the runs' fences once.
// Member j is run rows.row[j]; the RouteTable is indexed by run.
// The fused page search's window: 7 fences and 3 halving steps (one
// dependent LDS read fewer than k_route's 15; the guess from the run's first
// and last fence lands within a fence or two for C3's keys).
constexpr int kFusedWindow = 7;

template <int TILE_KEYS, int BLOCK, int LAYOUT>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8))) k_probe_combine_route(
    const uint8_t *__restrict__ res, const uint16_t *__restrict__ slots, KeySpan ks,
    uint64_t *__restrict__ out, size_t nw, StackTable rows, RouteTable rt,
    int32_t *__restrict__ first, int32_t *__restrict__ page, uint32_t *__restrict__ packed,
    size_t ntiles) {
    constexpr int kTilePos = 3 * TILE_KEYS;
    constexpr int kPasses = TILE_KEYS / (BLOCK * kCombineKeys);  // super-tiles: two
    static_assert(kPasses * BLOCK * kCombineKeys == TILE_KEYS, "8 keys per thread and pass");
    extern __shared__ int32_t s_fences[];
    __shared__ __attribute__((aligned(16))) uint8_t s_r[kTilePos];
    // per run: its fences' LDS offset and count, first fence and fence
    // spacing (one 16-B read per routed key); per member: its run's key
    // range as a window, k - lo <= span in u32 (one broadcast read per member
    // and pass of 8 keys)
    __shared__ __attribute__((aligned(16))) uint4 s_rec[kMaxStack];
    __shared__ __attribute__((aligned(8))) uint2 s_win[kMaxStack];
    __shared__ int s_run_of[kMaxStack];
    const int nf = rows.nf;
    for (int r = threadIdx.x; r < nf; r += BLOCK) {
        const uint32_t n = rt.nfences[r];
        const int32_t f0 = n ? rt.meta[r][1] : 0, fl = n ? rt.meta[r][n] : 0;
        const float scale = (n > 1 && fl > f0) ? (float)(n - 1) / ((float)fl - (float)f0) : 0.0f;
        s_rec[r] = make_uint4(rt.fence_off[r], n, __float_as_uint((float)f0), __float_as_uint(scale));
        s_run_of[r] = rows.row[r];
        const int rr = rows.row[r];  // member r's run: [first fence, max key]
        const uint32_t nr = rt.nfences[rr];
        const int32_t lo = nr ? rt.meta[rr][1] : 0, hi = nr ? rt.meta[rr][0] : 0;
        s_win[r] = make_uint2((uint32_t)lo, (uint32_t)hi - (uint32_t)lo);  // (a dead window: live below)
    }
    // members whose run has keys in range at all (no fences, or max key
    // below the first fence: never in range), and whether member j is run j
    uint32_t live = 0;
    bool ident = true;
#pragma unroll
    for (int j = 0; j < kMaxStack; j++) {
        if (j < nf) {
            const int r = rows.row[j];
            const uint32_t n = rt.nfences[r];
            if (n && rt.meta[r][0] >= rt.meta[r][1]) live |= 1u << j;
            ident &= r == j;
        }
    }
    const uint32_t live4 = live * 0x01010101u;
    {
        // every run's fences, contiguous in LDS (fence_off is the prefix of
        // the counts), 8 loads in flight per thread (a load-then-store loop
        // per run waited for each load: ~12 us before the first tile)
        constexpr int kBatch = 8;
        const uint32_t total = rt.total_fences;
        for (uint32_t b = 0; b < total; b += kBatch * BLOCK) {
            int32_t v[kBatch];
#pragma unroll
            for (int q = 0; q < kBatch; q++) {
                const uint32_t g = b + q * BLOCK + threadIdx.x;
                // g's run, by compile-time indices (a runtime index into the
                // kernel-argument arrays went through scratch memory)
                const int32_t *src = rt.meta[0] + 1;
                uint32_t off = 0;
#pragma unroll
                for (int rr = 1; rr < kMaxStack; rr++) {
                    if (rr < nf && rt.fence_off[rr] <= g) {
                        src = rt.meta[rr] + 1;
                        off = rt.fence_off[rr];
                    }
                }
                v[q] = g < total ? src[g - off] : 0;
            }
#pragma unroll
            for (int q = 0; q < kBatch; q++) {
                const uint32_t g = b + q * BLOCK + threadIdx.x;
                if (g < total) s_fences[g] = v[q];
            }
        }
    }
    const int kt = kCombineKeys * (int)threadIdx.x;  // this thread's first key in a tile's pass
    const bool vec_out = ((reinterpret_cast<uintptr_t>(first) | reinterpret_cast<uintptr_t>(page) |
                           reinterpret_cast<uintptr_t>(packed)) & 15) == 0;
    for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const size_t tile0 = tile * TILE_KEYS;
        const int tile_keys = (int)min((size_t)TILE_KEYS, ks.n - tile0);
        // pass ps's keys: 8 tid + 8 BLOCK ps .. + 7; their slots and the keys
        // (pass 0's loads in flight across the staging below)
        const uint4 *sl = reinterpret_cast<const uint4 *>(slots + tile * 3 * TILE_KEYS + kt);
        uint4 va = sl[0], vb = sl[TILE_KEYS / 8], vc = sl[2 * (TILE_KEYS / 8)];
        int32_t key[kCombineKeys];
        auto load_keys = [&](int k0) {
            if (LAYOUT == KEYS_PACKED && tile_keys == TILE_KEYS) {
                const int4 *kv = reinterpret_cast<const int4 *>(ks.base) + (tile0 + k0) / 4;
                const int4 x = kv[0], y = kv[1];
                key[0] = x.x; key[1] = x.y; key[2] = x.z; key[3] = x.w;
                key[4] = y.x; key[5] = y.y; key[6] = y.z; key[7] = y.w;
            } else {
#pragma unroll
                for (int i = 0; i < kCombineKeys; i++)
                    key[i] = k0 + i < tile_keys ? load_key<LAYOUT>(ks, tile0 + k0 + i) : 0;
            }
        };
        load_keys(kt);
        __syncthreads();  // the previous tile's result bytes are no longer read
        // the tile's result bytes: every load issued before any LDS store (a
        // load-store loop waited for each; loaded before the barrier, they
        // spilled under the 64-VGPR cap), clamped so no load sits under a branch
        constexpr int kResVec = kTilePos / 16, kResPer = (kResVec + BLOCK - 1) / BLOCK;
        const uint4 *src = reinterpret_cast<const uint4 *>(res + tile * (size_t)kTilePos);
        uint4 rv[kResPer];
#pragma unroll
        for (int j = 0; j < kResPer; j++) rv[j] = src[min((int)threadIdx.x + j * BLOCK, kResVec - 1)];
#pragma unroll
        for (int j = 0; j < kResPer; j++)
            if ((int)threadIdx.x + j * BLOCK < kResVec) reinterpret_cast<uint4 *>(s_r)[threadIdx.x + j * BLOCK] = rv[j];
        __syncthreads();
        // (unrolled: a loop over the two passes of a super-tile spilled 44
        // VGPRs; the 512-lane strided-key variant spills 2 either way)
#pragma unroll
        for (int ps = 0; ps < kPasses; ps++) {
        const int k0 = kt + ps * kCombineKeys * BLOCK;  // this pass's first key
        if (ps > 0) {
            const uint4 *sp = sl + ps * BLOCK;  // 8 u16 per thread: BLOCK vectors per pass
            va = sp[0];
            vb = sp[TILE_KEYS / 8];
            vc = sp[2 * (TILE_KEYS / 8)];
            load_keys(k0);
        }
        const uint32_t a[4] = {va.x, va.y, va.z, va.w}, b[4] = {vb.x, vb.y, vb.z, vb.w},
                       c[4] = {vc.x, vc.y, vc.z, vc.w};
        // byte i: key i's member bits, then its candidate runs (bit r: filter and range)
        uint32_t cand_lo = 0, cand_hi = 0, in_lo = 0, in_hi = 0;
        int32_t fr[kCombineKeys], pg[kCombineKeys];
#pragma unroll
        for (int i = 0; i < kCombineKeys; i++) {
            const int sh = 16 * (i & 1);
            const uint32_t sa = (a[i / 2] >> sh) & 0xFFFFu, sb = (b[i / 2] >> sh) & 0xFFFFu,
                           sc = (c[i / 2] >> sh) & 0xFFFFu;
            const uint32_t hit = k0 + i < tile_keys ? (uint32_t)(s_r[min(sa, (uint32_t)kTilePos - 1)] &
                                                                 s_r[min(sb, (uint32_t)kTilePos - 1)] &
                                                                 s_r[min(sc, (uint32_t)kTilePos - 1)])
                                                    : 0u;
            if (i < 4) cand_lo |= hit << (8 * i);
            else cand_hi |= hit << (8 * (i - 4));
        }
        // the range checks, member by member over the 8 keys (k - lo <= span)
#pragma unroll
        for (int j = 0; j < kMaxStack; j++) {
            if (j < nf) {
                const uint2 w = s_win[j];
#pragma unroll
                for (int i = 0; i < kCombineKeys; i++) {
                    const uint32_t in = (uint32_t)key[i] - w.x <= w.y ? 1u << (8 * (i & 3) + j) : 0u;
                    if (i < 4) in_lo |= in;
                    else in_hi |= in;
                }
            }
        }
        cand_lo &= in_lo & live4;
        cand_hi &= in_hi & live4;
        if (!ident) {  // member j is run rows.row[j]: move its bits
            const uint32_t ml = cand_lo, mh = cand_hi;
            cand_lo = cand_hi = 0;
#pragma unroll
            for (int j = 0; j < kMaxStack; j++) {
                if (j < nf) {
                    const int sh = s_run_of[j] - j;
                    const uint32_t bl = ml & (0x01010101u << j), bh = mh & (0x01010101u << j);
                    cand_lo |= sh >= 0 ? bl << sh : bl >> -sh;
                    cand_hi |= sh >= 0 ? bh << sh : bh >> -sh;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kCombineKeys; i++) {
            const uint32_t m = ((i < 4 ? cand_lo : cand_hi) >> (8 * (i & 3))) & 0xFFu;
            fr[i] = m ? __builtin_ctz(m) : -1;  // runs newest first: the lowest bit
        }
        // The pages of the lane's keys, two searched side by side (their LDS
        // reads independent; all 8 at once took 89 VGPRs, which left one
        // 1024-lane workgroup per CU, and 4 spilled under the 64-VGPR cap
        // that fits two): the window guess and its check, 4 halving steps,
        // and the whole-run binary search for the rare key whose guess missed.
        constexpr int kSide = 2;
#pragma unroll
        for (int h = 0; h < kCombineKeys; h += kSide) {
            int base_[kSide], n_[kSide], lo_[kSide];
            bool ok_[kSide];
#pragma unroll
            for (int u = 0; u < kSide; u++) {
                const int i = h + u;
                const uint4 rec = s_rec[max(fr[i], 0)];
                base_[u] = (int)rec.x;
                n_[u] = fr[i] >= 0 ? (int)rec.y : 0;
                int a = 0;
                ok_[u] = true;
                if (n_[u] > kFusedWindow) {
                    const int g = (int)fminf(fmaxf(((float)key[i] - __uint_as_float(rec.z)) * __uint_as_float(rec.w), 0.0f),
                                             kGuessMax);
                    a = min(max(g - kFusedWindow / 2, 0), n_[u] - kFusedWindow);
                    const int32_t fl = s_fences[base_[u] + max(a - 1, 0)];
                    const int32_t fh = s_fences[base_[u] + min(a + kFusedWindow, n_[u] - 1)];
                    ok_[u] = (a == 0 || fl <= key[i]) && (a + kFusedWindow >= n_[u] || fh > key[i]);
                }
                lo_[u] = a;
            }
#pragma unroll
            for (int st = (kFusedWindow + 1) / 2; st >= 1; st >>= 1) {
#pragma unroll
                for (int u = 0; u < kSide; u++) {
                    const int idx = lo_[u] + st - 1;
                    const int32_t f = s_fences[base_[u] + min(idx, max(n_[u] - 1, 0))];
                    if (idx < n_[u] && f <= key[h + u]) lo_[u] += st;
                }
            }
#pragma unroll
            for (int u = 0; u < kSide; u++) {
                const int i = h + u;
                if (!ok_[u]) {  // the guess missed (rare): binary search the whole run
                    const int32_t *fz = s_fences + base_[u];
                    int l = 1, hh = n_[u];
                    while (l < hh) {
                        const int mid = (l + hh) >> 1;
                        if (fz[mid] <= key[i]) l = mid + 1;
                        else hh = mid;
                    }
                    lo_[u] = l;
                }
                pg[i] = fr[i] >= 0 ? lo_[u] - 1 : -1;
            }
        }
        // first / page (or their packed form) of the live keys
        if (vec_out && tile_keys == TILE_KEYS) {
            int4 *f4 = reinterpret_cast<int4 *>(first + tile0 + k0);
            int4 *p4 = reinterpret_cast<int4 *>(page + tile0 + k0);
            if (first) {
                f4[0] = make_int4(fr[0], fr[1], fr[2], fr[3]);
                f4[1] = make_int4(fr[4], fr[5], fr[6], fr[7]);
            }
            if (page) {
                p4[0] = make_int4(pg[0], pg[1], pg[2], pg[3]);
                p4[1] = make_int4(pg[4], pg[5], pg[6], pg[7]);
            }
            if (packed) {
                uint4 *q4 = reinterpret_cast<uint4 *>(packed + tile0 + k0);
                q4[0] = make_uint4(route_pack(fr[0], pg[0]), route_pack(fr[1], pg[1]),
                                   route_pack(fr[2], pg[2]), route_pack(fr[3], pg[3]));
                q4[1] = make_uint4(route_pack(fr[4], pg[4]), route_pack(fr[5], pg[5]),
                                   route_pack(fr[6], pg[6]), route_pack(fr[7], pg[7]));
            }
        } else {
#pragma unroll
            for (int i = 0; i < kCombineKeys; i++) {
                if (k0 + i < tile_keys) {
                    if (first) first[tile0 + k0 + i] = fr[i];
                    if (page) page[tile0 + k0 + i] = pg[i];
                    if (packed) packed[tile0 + k0 + i] = route_pack(fr[i], pg[i]);
                }
            }
        }
        // candidate rows: bytes of the tile's rows that hold keys (whole
        // 64-key words), run r's byte = bit r of the 8 keys' masks
        if (k0 < ((tile_keys + 63) & ~63)) {
            const uint32_t lo = cand_lo, hi = cand_hi;
            const size_t byte0 = tile0 / 8 + threadIdx.x + ps * BLOCK;
#pragma unroll
            for (int r = 0; r < kMaxStack; r++) {
                if (r < nf) {
                    const uint32_t bl = ((lo >> r) & 0x01010101u) * 0x01020408u;
                    const uint32_t bh = ((hi >> r) & 0x01010101u) * 0x01020408u;
                    const uint32_t byte = (bl >> 24) | ((bh >> 20) & 0xF0u);
                    reinterpret_cast<uint8_t *>(out + (size_t)r * nw)[byte0] = (uint8_t)byte;
                }
            }
        }
        }  // passes
    }
}

}  // namespace

// Exported by the kernel translation units (one instantiation family each).
hipError_t launch_runs_transpose(const PartitionWorkspace &ws, hipStream_t stream);  // bloom_kernels.hip
bool runs_as_columns(const PartitionWorkspace &ws);                                  // bloom_kernels.hip
// pass 1: build / probe (slots) at 512 or 1024 threads (bloom_pass1_*.hip)
hipError_t launch_bin_build512(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               hipStream_t stream);
hipError_t launch_bin_build1024(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                                hipStream_t stream);
hipError_t launch_bin_probe512(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               uint16_t *slots, hipStream_t stream);
// pass 1 of a build on super-tiles (bloom_pass1_super.hip)
hipError_t launch_bin_super(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                            hipStream_t stream);
hipError_t launch_bin_super_probe(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                                  uint16_t *slots, hipStream_t stream);  // bloom_pass1_super_probe.hip
hipError_t launch_bin_probe1024(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                                uint16_t *slots, hipStream_t stream);
// pass 2 of the probes (bloom_probe.hip, bloom_probe_ladder.hip) and the combine
hipError_t launch_apply_stack(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                              const StackTable &st, hipStream_t stream);
hipError_t launch_apply_ladder(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                               const StackTable &st, hipStream_t stream);
hipError_t launch_combine(const PartitionWorkspace &ws, const uint8_t *res, const uint16_t *slots,
                          size_t n, uint64_t *out, size_t nw, const StackTable &rows,
                          hipStream_t stream);

namespace {

// One pass-1 launch: MAXB is the histogram capacity the kernel is compiled
// for (its scan loop and registers follow it, so a small capacity is cheaper:
// C2's 256 segments at MAXB 511 run pass 1 in 74.5 us against 87 at 4096,
// tools/ubench.py part with UB_P1).  Only the packed / entry_t fast paths get
// the small capacities; strided keys and m >= 2^32 use the largest.
// Workgroups of pass 1 resident per CU: the 4096-key build tile with a
// histogram of <= 511 bins takes 50 KiB of LDS, so three fit a CU when the
// registers are capped for 6 waves per SIMD (80 VGPRs, 2 spilled): C2 pass 1
// 59.5 -> 58.1 us (tools/ubench.py p1ab, variant 5003).  Everything else:
// two 512-thread or one 1024-thread workgroup per CU.
template <int TB, bool SLOTS, int MAXB>
constexpr int part_bin_wgs_per_cu() {
    return TB >= 1024 ? 1 : (!SLOTS && MAXB > 0 && MAXB <= 511) ? 3 : 2;
}

template <int L, bool SLOTS, int TB, int MK, int MAXB>
void bin_launch(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                uint32_t *runs, const SegMap &sm, bool cols, uint16_t *slots, hipStream_t stream) {
    constexpr int kWgs = part_bin_wgs_per_cu<TB, SLOTS, MAXB>();
    constexpr int kMinW = kWgs * TB / 256;  // waves per SIMD the registers must allow
    const size_t g = (size_t)device_cu_count() * kWgs;
    const unsigned grid = (unsigned)(ws.ntiles < g ? ws.ntiles : g);
    if constexpr (!SLOTS && TB >= 1024 && MAXB == 1023) {
        // builds whose sorted tiles exceed the Infinity Cache (C5): stored
        // non-temporal (k_part_bin's NT)
        if (ws.ntiles * (uint64_t)(TB * kPartKPT) * 8 > kInfinityCacheBytes) {
            if (cols)
                k_part_bin<L, SLOTS, true, TB, MK, MAXB, kMinW, 0, true><<<grid, TB, 0, stream>>>(
                    ks, mp, ws.pos, runs, sm, ws.ntiles, slots);
            else
                k_part_bin<L, SLOTS, false, TB, MK, MAXB, kMinW, 0, true><<<grid, TB, 0, stream>>>(
                    ks, mp, ws.pos, runs, sm, ws.ntiles, slots);
            return;
        }
    }
    if (cols)
        k_part_bin<L, SLOTS, true, TB, MK, MAXB, kMinW><<<grid, TB, 0, stream>>>(
            ks, mp, ws.pos, runs, sm, ws.ntiles, slots);
    else
        k_part_bin<L, SLOTS, false, TB, MK, MAXB, kMinW><<<grid, TB, 0, stream>>>(
            ks, mp, ws.pos, runs, sm, ws.ntiles, slots);
}

template <int L, bool SLOTS, int TB, int MK>
void bin_launch_fast(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                     uint32_t *runs, const SegMap &sm, bool cols, uint16_t *slots,
                     hipStream_t stream) {
    const size_t nb = ws.nbins;
    if constexpr (TB >= 1024) {
        if (nb <= 1023) bin_launch<L, SLOTS, TB, MK, 1023>(ks, mp, ws, runs, sm, cols, slots, stream);
        else if (nb <= 2047) bin_launch<L, SLOTS, TB, MK, 2047>(ks, mp, ws, runs, sm, cols, slots, stream);
        else if (nb <= 4095) bin_launch<L, SLOTS, TB, MK, 4095>(ks, mp, ws, runs, sm, cols, slots, stream);
        else bin_launch<L, SLOTS, TB, MK, (int)kPartMaxBinsBig>(ks, mp, ws, runs, sm, cols, slots, stream);
    } else {
        if (nb <= 511) bin_launch<L, SLOTS, TB, MK, 511>(ks, mp, ws, runs, sm, cols, slots, stream);
        else bin_launch<L, SLOTS, TB, MK, (int)kPartMaxBins>(ks, mp, ws, runs, sm, cols, slots, stream);
    }
}

// Whether pass 1 may take the p2 reduction (kModP2) for this geometry: the
// entry must be the hash's low kEntryBits bits (t >= 21) and p >> shift must
// reach bit t (shift <= t).
inline bool p2_pass1(const ModParams &mp, const SegMap &sm) {
    return mp.fast && mp.p2 && mp.p2t >= kEntryBits && sm.shift <= mp.p2t && mp.p2t - sm.shift < 32;
}

// Pass 1's reduction kind (kMod*) and segment map for a batch on geometry
// ws, as k_part_bin is launched with them; -1 when the geometry is not one
// pass 1 takes.  (tools/ubench.py prices bin_entry with these alone.)
inline int pass1_plan(const ModParams &mp, const PartitionWorkspace &ws, bool slots, SegMap *out) {
    SegMap sm = seg_map_of(ws);
    const bool wide = !mp.fast;
    if (!wide) {  // the fast path shifts the remainder scaled by 2^l
        sm.scaled_shift = sm.shift + mp.l;
        if (sm.scaled_shift > 31) {  // m < 2^(32-l) <= 2^shift: every p is in segment 0
            sm.scaled_shift = 0;
            sm.magic = 0;
        }
    }
    int mk;
    if (ws.lad_u) {  // ladder stack: bins are hash bits [s, s + u) (plan_ladder)
        if (!mp.fast || !mp.p2 || sm.shift + sm.lad_u + sm.lad_hb != mp.p2t) return -1;
        sm.scaled_shift = sm.shift + sm.lad_u;
        // plan_build's one-member ladder, relabelled where 24 lies in [s, t]
        mk = sm.lad_hb == 0 && !slots ? (ladder0_relabel(mp, ws) ? kModLadder0R : kModLadder0) : kModLadder;
    } else if (wide) {
        mk = kModWide;
    } else if (p2_pass1(mp, sm)) {
        sm.p2_hi_shift = mp.p2t - sm.shift;
        mk = kModP2;
    } else {
        mk = kModFast;
    }
    *out = sm;
    return mk;
}

template <bool SLOTS, int TB, int MK>
void bin_launch_layout(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                       uint32_t *runs, const SegMap &sm, bool cols, uint16_t *slots,
                       hipStream_t stream) {
    constexpr int kCap = TB >= 1024 ? (int)kPartMaxBinsBig : (int)kPartMaxBins;
    const bool entry16 =
        ks.layout == KEYS_ENTRY && (reinterpret_cast<uintptr_t>(ks.base) & 15) == 0;
    // only the packed / entry_t fast paths get the small histogram
    // capacities; strided keys and m >= 2^32 use the largest
    if constexpr (MK != kModWide) {
        if (ks.layout == KEYS_PACKED)
            bin_launch_fast<KEYS_PACKED, SLOTS, TB, MK>(ks, mp, ws, runs, sm, cols, slots, stream);
        else if (entry16)
            bin_launch_fast<KEYS_ENTRY, SLOTS, TB, MK>(ks, mp, ws, runs, sm, cols, slots, stream);
        else
            bin_launch<KEYS_STRIDED, SLOTS, TB, MK, kCap>(ks, mp, ws, runs, sm, cols, slots, stream);
    } else {
        if (ks.layout == KEYS_PACKED)
            bin_launch<KEYS_PACKED, SLOTS, TB, MK, kCap>(ks, mp, ws, runs, sm, cols, slots, stream);
        else if (entry16)
            bin_launch<KEYS_ENTRY, SLOTS, TB, MK, kCap>(ks, mp, ws, runs, sm, cols, slots, stream);
        else
            bin_launch<KEYS_STRIDED, SLOTS, TB, MK, kCap>(ks, mp, ws, runs, sm, cols, slots, stream);
    }
}

template <bool SLOTS, int TB>
hipError_t launch_bin_tb(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                         uint16_t *slots, hipStream_t stream) {
    constexpr int kCap = TB >= 1024 ? (int)kPartMaxBinsBig : (int)kPartMaxBins;
    if (ws.nbins > (size_t)kCap) return hipErrorInvalidValue;
    const bool cols = runs_as_columns(ws);
    uint32_t *runs = cols ? ws.run_starts : ws.run_rows;
    SegMap sm{};
    switch (pass1_plan(mp, ws, SLOTS, &sm)) {
        case kModLadder0:
            if constexpr (!SLOTS) {
                bin_launch_layout<SLOTS, TB, kModLadder0>(ks, mp, ws, runs, sm, cols, slots, stream);
                break;
            } else {
                return hipErrorInvalidValue;
            }
        case kModLadder0R:
            if constexpr (!SLOTS) {
                bin_launch_layout<SLOTS, TB, kModLadder0R>(ks, mp, ws, runs, sm, cols, slots, stream);
                break;
            } else {
                return hipErrorInvalidValue;
            }
        case kModLadder: bin_launch_layout<SLOTS, TB, kModLadder>(ks, mp, ws, runs, sm, cols, slots, stream); break;
        case kModWide: bin_launch_layout<SLOTS, TB, kModWide>(ks, mp, ws, runs, sm, cols, slots, stream); break;
        case kModP2: bin_launch_layout<SLOTS, TB, kModP2>(ks, mp, ws, runs, sm, cols, slots, stream); break;
        case kModFast: bin_launch_layout<SLOTS, TB, kModFast>(ks, mp, ws, runs, sm, cols, slots, stream); break;
        default: return hipErrorInvalidValue;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || cols) return e;
    return launch_runs_transpose(ws, stream);
}


// Pass 1 on super-tiles (k_part_bin2): builds whose geometry plan_build gave
// kSuperTileKeys (segments of m < 2^32, more than kSuperMinBins of them).
template <int MK, bool SLOTS>
hipError_t launch_bin_super_mk(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               const SegMap &sm, uint16_t *slots, hipStream_t stream) {
    const bool cols = runs_as_columns(ws);
    uint32_t *runs = cols ? ws.run_starts : ws.run_rows;
    const size_t g = (size_t)device_cu_count();
    const unsigned grid = (unsigned)(ws.ntiles < g ? ws.ntiles : g);
    const bool entry16 = ks.layout == KEYS_ENTRY && (reinterpret_cast<uintptr_t>(ks.base) & 15) == 0;
#define SUPER_L(L, C) \
    k_part_bin2<L, C, MK, (int)kSuperMaxBins, SLOTS><<<grid, kSuperBlock, 0, stream>>>(ks, mp, ws.pos, runs, sm, \
                                                                                     ws.ntiles, slots)
    if (ks.layout == KEYS_PACKED) {
        if (cols) SUPER_L(KEYS_PACKED, true); else SUPER_L(KEYS_PACKED, false);
    } else if (entry16) {
        if (cols) SUPER_L(KEYS_ENTRY, true); else SUPER_L(KEYS_ENTRY, false);
    } else {
        if (cols) SUPER_L(KEYS_STRIDED, true); else SUPER_L(KEYS_STRIDED, false);
    }
#undef SUPER_L
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || cols) return e;
    return launch_runs_transpose(ws, stream);
}

template <bool SLOTS>
hipError_t launch_bin_super_impl(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                                 uint16_t *slots, hipStream_t stream) {
    if (ws.nbins > kSuperMaxBins || (SLOTS && !slots)) return hipErrorInvalidValue;
    SegMap sm{};
    switch (pass1_plan(mp, ws, SLOTS, &sm)) {
        case kModP2: return launch_bin_super_mk<kModP2, SLOTS>(ks, mp, ws, sm, slots, stream);
        case kModFast: return launch_bin_super_mk<kModFast, SLOTS>(ks, mp, ws, sm, slots, stream);
        default: return hipErrorInvalidValue;
    }
}

// Pass 1 for a build (SLOTS = false) or a probe (SLOTS = true), then the
// run-start transpose when the table is large: the exported instantiation
// for the batch's tile size.
template <bool SLOTS>
hipError_t launch_bin(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                      uint16_t *slots, hipStream_t stream) {
    const bool big = tile_keys_of(ws) == 2 * kPartTileKeys;
    if constexpr (SLOTS) {
        if (tile_keys_of(ws) == kSuperTileKeys) return launch_bin_super_probe(ks, mp, ws, slots, stream);
        return big ? launch_bin_probe1024(ks, mp, ws, slots, stream)
                   : launch_bin_probe512(ks, mp, ws, slots, stream);
    } else {
        if (tile_keys_of(ws) == kSuperTileKeys) return launch_bin_super(ks, mp, ws, stream);
        return big ? launch_bin_build1024(ks, mp, ws, stream) : launch_bin_build512(ks, mp, ws, stream);
    }
}

// The segment stack's pass 2 on persistent workgroups (round 5): member j's
// window of segment b starts at word (b * sw) mod mw_j, periodic in b with
// period P_j = mw_j / gcd(sw, mw_j) (the f = 10 tree at w = 409,600 bits:
// 25 for level 0, 125 for level 1, every segment for level 2).  With S
// resident workgroups, S a multiple of the periods of a set of members,
// workgroup c takes segments c, c + S, c + 2S, ... and stages those members'
// windows once (the f = 10 tree: 150 KiB staged per segment -> 50 KiB for
// four of a workgroup's five).  Sets st.seg_stride = 0 when no member
// repeats within the resident workgroups or each segment has its own anyway.
inline void stack_stride(size_t nbins, uint32_t seg_words, size_t lds, StackTable &st) {
    st.seg_stride = 0;
    st.keep_mask = 0;
    const size_t per_cu = std::max<size_t>(1, std::min<size_t>(2048 / kApplyBlock, kLdsBitmapBytes / std::max<size_t>(lds, 1)));
    const uint64_t cap = (uint64_t)device_cu_count() * per_cu;
    if (nbins <= cap || st.nf < 1 || st.nf > kMaxStack) return;
    uint64_t P[kMaxStack];
    int ord[kMaxStack];
    for (int j = 0; j < st.nf; j++) {
        P[j] = st.mwords[j] / std::gcd<uint64_t>(seg_words, st.mwords[j]);
        ord[j] = j;
    }
    std::sort(ord, ord + st.nf, [&](int a, int c) { return P[a] < P[c]; });
    uint64_t L = 1;
    uint32_t mask = 0;
    for (int q = 0; q < st.nf; q++) {
        const int j = ord[q];
        if (P[j] >= nbins) continue;  // no repeat among the segments
        const uint64_t l2 = std::lcm<uint64_t>(L, P[j]);
        if (l2 > cap) continue;
        L = l2;
        mask |= 1u << j;
    }
    if (!mask) return;
    const uint64_t S = L * (cap / L);
    if (S >= nbins) return;
    st.seg_stride = (int)S;
    st.keep_mask = mask;
}

// Launches pass 2 (build or probe) with S/8 bytes of dynamic LDS (> 64 KiB
// must be opted into per kernel).
template <int MODE, int G, int TK, int DEPTH = kApplyDepth, int WALK = 0, int NF = 0, int LK = 0>
hipError_t launch_apply_g(const PartitionWorkspace &ws, uint64_t m, uint32_t *words,
                          uint64_t nw32, int merge, uint8_t *res, const StackTable &st,
                          hipStream_t stream) {
    if (NF && st.nf != NF) return hipErrorInvalidValue;
    // The build's walk addresses the segment image by absolute LDS byte
    // address, which is right only while the dynamic image starts at LDS
    // address 0, i.e. while the kernel has no static LDS: checked once per
    // instantiation from the code object, and the launch refused otherwise.
    static const bool lds_ok = [] {
        const void *fn =
            reinterpret_cast<const void *>(&k_part_apply<MODE, G, TK, kApplyBlock, DEPTH, WALK, NF, LK>);
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kStackMaxBits / 8));
        hipFuncAttributes fa{};
        return hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.sharedSizeBytes == 0;
    }();
    if (!lds_ok) return hipErrorInvalidDeviceFunction;
    const size_t lds = MODE == kApplyLadder ? ladder_lds_bytes(st.lad)
                                            : (size_t)ws.seg_bits / 8 * (MODE == kApplyStack ? st.nf : 1);
    if (lds > kStackMaxBits / 8) return hipErrorInvalidValue;
    StackTable sk = st;
    sk.seg_stride = 0;
    sk.keep_mask = 0;
    if (MODE == kApplyStack && NF < 8 && G == 4) stack_stride(ws.nbins, ws.seg_bits / 32, lds, sk);
    const unsigned grid = sk.seg_stride ? (unsigned)sk.seg_stride : (unsigned)ws.nbins;
    k_part_apply<MODE, G, TK, kApplyBlock, DEPTH, WALK, NF, LK><<<grid, kApplyBlock, lds, stream>>>(
        ws.pos, ws.run_starts, (int)ws.ntiles, (int)ws.nbins, ws.seg_bits, m, words, nw32, merge,
        res, sk);
    return hipGetLastError();
}

// The stacked pass 2 with the member count compiled in (straight-line member
// reads instead of a guarded loop over up to kMaxStack), G lanes per tile.
template <int G, int TK, int WALK = 0>
hipError_t launch_stack_nf(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                           const StackTable &st, hipStream_t stream) {
    switch (st.nf) {
#define STACK_NF(N) \
    case N: return launch_apply_g<kApplyStack, G, TK, kApplyDepth, WALK, N>(ws, m, nullptr, 0, 0, res, st, stream);
        STACK_NF(2) STACK_NF(3) STACK_NF(4) STACK_NF(5) STACK_NF(6) STACK_NF(7) STACK_NF(8)
#undef STACK_NF
        default: return launch_apply_g<kApplyStack, G, TK, kApplyDepth, WALK>(ws, m, nullptr, 0, 0, res, st, stream);
    }
}

// The ladder's pass 2 with the member count and the direct members (plan_ladder:
// 1, 2, 3 or all of them) compiled in.
template <int G, int TK, int WALK, int N, int D = kApplyDepth>
hipError_t launch_ladder_k(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                           const StackTable &st, hipStream_t stream) {
    switch (st.lad.k) {
        case 1:
            if (st.lad.ctup)  // the packed tuple computed (LadderTable::ctup)
                return launch_apply_g<kApplyLadder, G, TK, D, WALK, N, 0>(ws, m, nullptr, 0, 0, res, st, stream);
            return launch_apply_g<kApplyLadder, G, TK, D, WALK, N, 1>(ws, m, nullptr, 0, 0, res, st, stream);
        case 2: return launch_apply_g<kApplyLadder, G, TK, D, WALK, N, 2>(ws, m, nullptr, 0, 0, res, st, stream);
        case 3:
            if constexpr (N >= 3)
                return launch_apply_g<kApplyLadder, G, TK, D, WALK, N, 3>(ws, m, nullptr, 0, 0, res, st, stream);
            else
                return hipErrorInvalidValue;
        default:
            if (st.lad.k != (uint32_t)N) return hipErrorInvalidValue;
            return launch_apply_g<kApplyLadder, G, TK, D, WALK, N, N>(ws, m, nullptr, 0, 0, res, st, stream);
    }
}

template <int G, int TK, int WALK = 1, int D = kApplyDepth>
hipError_t launch_ladder_nf(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                            const StackTable &st, hipStream_t stream) {
    switch (st.nf) {
        case 2: return launch_ladder_k<G, TK, WALK, 2, D>(ws, m, res, st, stream);
        case 3: return launch_ladder_k<G, TK, WALK, 3, D>(ws, m, res, st, stream);
        case 4: return launch_ladder_k<G, TK, WALK, 4, D>(ws, m, res, st, stream);
        case 5: return launch_ladder_k<G, TK, WALK, 5, D>(ws, m, res, st, stream);
        case 6: return launch_ladder_k<G, TK, WALK, 6, D>(ws, m, res, st, stream);
        case 7: return launch_ladder_k<G, TK, WALK, 7, D>(ws, m, res, st, stream);
        case 8: return launch_ladder_k<G, TK, WALK, 8, D>(ws, m, res, st, stream);
        default: return hipErrorInvalidValue;
    }
}

template <int MODE, int TK>
hipError_t launch_apply_tk(const PartitionWorkspace &ws, uint64_t m, uint32_t *words,
                           uint64_t nw32, int merge, uint8_t *res, const StackTable &st,
                           hipStream_t stream) {
    if constexpr (MODE == kApplyLadder) {
        // batch walk at G = 8 (C3, 5 levels at 96-entry runs: 75.6 us against
        // 84.2 for independent groups at G = 4 and 78.5 at G = 8)
        return launch_ladder_nf<8, TK, 0>(ws, m, res, st, stream);
    } else if constexpr (MODE == kApplyStack) {
        // independent lane groups at G = 4 (C3, 5 levels: 108 -> 102 us; 4 levels: equal)
        if (apply_lanes_per_tile(ws.nbins, 3 * TK) <= 4) {
            if (3 * TK / ws.nbins < 24)  // short runs: loads past a run's end redirected
                return launch_stack_nf<4, TK, 2>(ws, m, res, st, stream);
            return launch_stack_nf<4, TK, 1>(ws, m, res, st, stream);
        }
        return launch_stack_nf<8, TK>(ws, m, res, st, stream);
    } else {
        switch (apply_lanes_per_tile(ws.nbins, 3 * TK)) {
            case 4:  // builds: independent lane groups (C2 pass 2 39.5 -> 34.4 us, C4 1.39 -> 1.36 ms),
                     // runs shorter than a group's step: loads past a run's end redirected
                if constexpr (MODE == kApplyBuild || MODE == kApplyBuildL) {
                    if (3 * TK / ws.nbins < 24)
                        return launch_apply_g<MODE, 4, TK, 1, 2>(ws, m, words, nw32, merge, res, st, stream);
                    // entries beyond the Infinity Cache (C5: 512 MiB, read
                    // from HBM): two vectors per lane and step, so a ~48-entry
                    // run is one step with twice the loads in flight (C5 pass 2
                    // 192.5 -> 173.6 us, tools/ubench.py p2ab_c5; C2's 128 MiB
                    // equal either way, so it keeps WALK 1)
                    if ((uint64_t)ws.ntiles * TK * 8 > kInfinityCacheBytes)
                        return launch_apply_g<MODE, 4, TK, 1, 3>(ws, m, words, nw32, merge, res, st, stream);
                    // (round 6's restated walk, WALK 4, was 1 % faster in
                    // tools/ubench.py p2ab but slower in the bench, where pass 2
                    // follows pass 1: C2 pass 2 35.2 -> 36.7 us, value 187.6 ->
                    // 184.6, profiles/r06/rejected/walk4_bench/; not launched)
                    return launch_apply_g<MODE, 4, TK, 1, 1>(ws, m, words, nw32, merge, res, st, stream);
                } else
                    return launch_apply_g<MODE, 4, TK>(ws, m, words, nw32, merge, res, st, stream);
            case 8: return launch_apply_g<MODE, 8, TK>(ws, m, words, nw32, merge, res, st, stream);
            case 16: return launch_apply_g<MODE, 16, TK>(ws, m, words, nw32, merge, res, st, stream);
            default: return launch_apply_g<MODE, 32, TK>(ws, m, words, nw32, merge, res, st, stream);
        }
    }
}

template <int MODE>
hipError_t launch_apply(const PartitionWorkspace &ws, uint64_t m, uint32_t *words, uint64_t nw32,
                        int merge, uint8_t *res, const StackTable &st, hipStream_t stream) {
    if constexpr (MODE == kApplyBuild) {
        if (tile_keys_of(ws) == kSuperTileKeys) {
            // super-tiles: >= kSuperMinBins segments, runs of at most 48
            // entries on average: independent groups of 4 lanes
            constexpr int TK = (int)kSuperTileKeys;
            // short runs: two vectors per lane, on two interleaved chains per
            // lane group (WALK 7: C4 pass 2 795 -> 764 us; three chains 875,
            // four 916, profiles/r06/c4_two_chains/)
            if (3 * TK / ws.nbins < 24)
                return launch_apply_g<MODE, 4, TK, 1, 7>(ws, m, words, nw32, merge, res, st, stream);
            return launch_apply_g<MODE, 4, TK, 1, 1>(ws, m, words, nw32, merge, res, st, stream);
        }
    } else if constexpr (MODE == kApplyStack) {
        // a segment stack on super-tiles (plan_stack: 1,024-4,095 segments,
        // runs of 12-48 entries): four lanes per tile, two vectors per lane
        if (tile_keys_of(ws) == kSuperTileKeys) return launch_stack_nf<4, (int)kSuperTileKeys, 3>(ws, m, res, st, stream);
    }
    return tile_keys_of(ws) == 2 * kPartTileKeys
               ? launch_apply_tk<MODE, 2 * (int)kPartTileKeys>(ws, m, words, nw32, merge, res, st,
                                                               stream)
               : launch_apply_tk<MODE, (int)kPartTileKeys>(ws, m, words, nw32, merge, res, st,
                                                           stream);
}

}  // namespace

}  // namespace bloomhip
