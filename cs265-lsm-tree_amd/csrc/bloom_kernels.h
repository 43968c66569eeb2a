// bloom_kernels.h — internal launch interface between the C ABI
// (bloom_capi.cpp) and the gfx950 kernels (bloom_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

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

// Run metadata and GET routing (§8f rows 1, 4).
constexpr size_t kFenceStride = 4096;  // getpagesize() entries per fence, src/run.cpp:164
constexpr int kMaxRouteRuns = 64;
// Routing stages every run's fences in LDS up to this (k_route, and the
// combine with routing fused in, which runs one workgroup per CU instead of
// two above ~56 KB): the f = 10 tree's three runs have 13,875 fences, 55 KB,
// and a binary search in global memory took 0.59 ms for its 16.8M GETs.
// Dynamic LDS within 64 KiB needs no opt-in.
constexpr size_t kRouteLdsFenceBytesMax = 60u << 10;
// Packed route output (bloomhip_route_gets_packed): one u32 per GET, the
// newest candidate run in bits 28-31 and its page in bits 0-27, or
// kRouteNone; half the bytes of the two int32 arrays first / page.
constexpr uint32_t kRouteNone = 0xFFFFFFFFu;
constexpr int kRoutePackedMaxRuns = 16;
constexpr uint32_t kRoutePageBits = 28;
__host__ __device__ __forceinline__ uint32_t route_pack(int32_t run, int32_t page) {
    return run >= 0 ? ((uint32_t)run << kRoutePageBits) | (uint32_t)page : kRouteNone;
}
// The route outputs of a routing call, each optional (null to skip).
struct RouteOut {
    int32_t *first;
    int32_t *page;
    uint32_t *packed;
};
// LDS of one workgroup of the combine with routing fused in
// (k_probe_combine_route): the runs' fences (dynamic), the tile's result
// bytes (3 per key, static) and the per-run tables (static, < 1 KiB).  The
// launch and probe_stacks' tile choice both size from this one helper.
inline size_t combine_route_lds_bytes(uint32_t total_fences, size_t tile_keys) {
    return (size_t)total_fences * 4 + 3 * tile_keys + 1024;
}

// Run metadata on the device: meta[0] = max key, meta[1 .. nfences] = the
// fence pointers, ascending (a run is written sorted).
struct RouteTable {
    const int32_t *meta[kMaxRouteRuns];
    uint32_t nfences[kMaxRouteRuns];
    uint32_t fence_off[kMaxRouteRuns];  // offset of run r's fences in the LDS copy
    uint32_t total_fences;
    int nruns;
};

// LDS bytes a private-bitmap workgroup may use (m/8 must fit): 160 KiB per
// CU on gfx950, one such workgroup per CU.
constexpr size_t kLdsBitmapBytes = 160 * 1024;

// Partition build geometry.  Pass 1 counting-sorts a tile's 3 positions per
// key by SEGMENT (b = p / S, S = seg_bits <= 160 KiB of bits, so a segment
// fits one workgroup's LDS), computed as (p >> sub_shift) / group with a
// host-verified multiply-high (SegMap).  Pass 2 gives each segment to one
// workgroup.  plan_segments picks (sub_shift, group) so that the number of
// segments is a multiple of the CU count: every CU of pass 2 gets the same
// share.
// Pass 2 has no static LDS: segment images may use all 160 KiB (plan_segments).
constexpr uint32_t kStackMaxBits = 160u * 1024u * 8u;
constexpr int kPartBlock = 512;
constexpr int kPartKPT = 8;  // keys per thread in pass 1
constexpr size_t kPartTileKeys = (size_t)kPartBlock * kPartKPT;  // 4096
constexpr int kPartTilePos = (int)kPartTileKeys * 3;
constexpr size_t kPartMaxBins = 4096;     // segments of a 4096-key tile (512 threads)
constexpr size_t kPartMaxBinsBig = 8192;  // segments of an 8192-key tile (1024 threads)
constexpr size_t kPartMaxSub = 16384;     // p >> sub_shift below this (SegMap's domain)

// Sorted-tile entries: the low kEntryBits bits of each position, three per
// u64 (bits 0-20, 21-41, 42-62).  A segment has at most kStackMaxBits <
// 2^21 bits, so within segment b's run (known by index from the run table)
// the offset is exactly (entry - b*S) mod 2^21.  8 B per 3 entries instead of
// 12, and the same format for any m (2^46 included).
constexpr uint32_t kEntryBits = 21;
constexpr uint32_t kEntryMask = (1u << kEntryBits) - 1u;
static_assert(kStackMaxBits <= (1u << kEntryBits), "segment offsets fit an entry");

// p -> segment, branch-free: x = p >> (sub_shift - 1) (< 2 * kPartMaxSub),
// b = mulhi(x, magic) = (x >> 1) / group.  magic = ceil(2^31 / group) (2^31
// for group 1), checked exact for every x < 2 * nsub when planned.
struct SegMap {
    uint32_t shift;  // sub_shift - 1 (ladder: s, the bin's lowest hash bit)
    uint32_t magic;
    uint32_t nbins;
    uint32_t scaled_shift;  // shift + l: the same map on a remainder scaled by 2^l (mod_fast_scaled)
    uint32_t p2_hi_shift;   // t - shift: where (x >> t) % d lands in p >> shift (m = d << t)
    uint32_t lad_u;         // ladder: log2(nbins), the bin's hash bits [s, s + u)
    uint32_t lad_hb;        // ladder: t_max - s - u, hash bits [s + u, t_max) kept in the entry
};

struct PartitionWorkspace {
    uint64_t *pos;         // [ntiles * tile_keys] packed sorted entries (3 per u64)
    uint32_t *run_rows;    // [ntiles * nbins], pass-1 runs (start | end << 16), tile-major
    uint32_t *run_starts;  // [nbins * ntiles], the same segment-major (pass 2)
    size_t ntiles;
    size_t nbins;          // segments
    uint32_t sub_shift;    // q = pos >> sub_shift
    uint32_t group;        // q's per segment
    uint32_t nsub;         // number of q values
    uint32_t seg_bits;     // S = group << sub_shift
    uint32_t tile_keys;    // keys per pass-1 tile: kPartTileKeys, or twice that (0 = default)
    uint32_t magic;        // SegMap::magic
    uint32_t lad_s;        // ladder stack (StackTable::lad): bins are hash bits [s, s + u);
    uint32_t lad_u;        //   0 for every other partition pass
    uint32_t lad_hb;
};


// Whether a build on plan_build's one-member ladder (bins = hash bits
// [s, t), m = d << t) takes the relabelled block a' = (x >> 24) % d in pass 1
// (bloom_math.h mod_p2_hi24: one instruction less per position) and pass 2
// maps it back (ladder0_block): when s <= 24 <= t, so the hash bits [24, t)
// are bin bits (C2: s = 17, t = 25; C5: s = 18, t = 27).
inline bool ladder0_relabel(const ModParams &mp, const PartitionWorkspace &ws) {
    return ws.lad_u && ws.lad_hb == 0 && mp.p2 && ws.lad_s <= 24 && mp.p2t >= 24;
}
// 2^-(t-24) mod d (d odd) for ladder0_block.
inline uint32_t ladder0_inv(const ModParams &mp) {
    uint32_t p = 1;
    for (uint32_t i = 24; i < mp.p2t; i++) p = p * 2 % mp.p2d;
    for (uint32_t v = 1; v < mp.p2d; v++)
        if (p * v % mp.p2d == 1) return v;
    return 1;  // d = 1 (not a p2 form)
}

inline SegMap seg_map_of(const PartitionWorkspace &ws) {
    if (ws.lad_u) return SegMap{ws.lad_s, 0, (uint32_t)ws.nbins, 0, 0, ws.lad_u, ws.lad_hb};
    return SegMap{ws.sub_shift - 1, ws.magic, (uint32_t)ws.nbins, 0, 0, 0, 0};
}

// Keys per pass-1 tile for a batch sorted into nbins segments: short runs
// make pass 2 line-bound, so batches with more than 256 segments (under 48
// entries per segment of a 4096-key tile) sort 8192-key tiles (one
// 1024-thread workgroup per CU) and get runs twice as long: C3, C4 and C5,
// while C2's 256 segments keep 4096-key tiles.  More than kPartMaxBins
// segments always need the 8192-key tile (its histogram holds 8192).
inline uint32_t choose_tile_keys(size_t nbins) {
    return nbins > 256 ? 2 * (uint32_t)kPartTileKeys : (uint32_t)kPartTileKeys;
}
// Builds on many short runs (segments of m < 2^32, at least kSuperMinBins of
// them: C4's 2,458) sort super-tiles of two 8192-key halves in pass 1
// (k_part_bin2): runs twice as long, half the (tile, segment) pairs.
constexpr size_t kSuperTileKeys = 4 * kPartTileKeys;  // 16384
constexpr size_t kSuperMinBins = 1024;
constexpr size_t kSuperMaxBins = 4095;                // the rank fields: bins << 20
inline size_t tile_keys_of(const PartitionWorkspace &ws) {
    return ws.tile_keys ? ws.tile_keys : kPartTileKeys;
}


// Geometry of a stacked probe (seg_bits = w): false when no w = g << s with
// w | m_max, w <= m_min (the smallest member), nf * w bits <= kStackMaxBits
// and <= kPartMaxBinsBig segments exists.  Prefers the widest w that still
// gives >= ncu segments.  gcd_m: gcd of the members' sizes (a multiple of
// 128 bits).
bool plan_stack(uint64_t m_max, uint64_t gcd_m, uint64_t m_min, int nf, int ncu,
                PartitionWorkspace *ws);

// CUs of the current device (cached).
int device_cu_count();
// Fills the geometry fields of ws for a filter of m bits; false when the
// partition path does not apply (more than kPartMaxBinsBig segments of at
// most 160 KiB: m above about 2^33.3 bits).
bool plan_segments(uint64_t m, int ncu, PartitionWorkspace *ws);
// Build geometry: plan_segments, then, when m = d << t (the p2 form) and the
// segment count is a power of two 2^u, the same bins taken as hash bits
// [t - u, t) (a one-member ladder, kernels.h LadderTable): bin b holds the d
// blocks a << t | b << s (s = t - u) of 2^s bits, its entry is a << s | the
// hash's low s bits, so pass 1 takes the bin with one bit-field extract
// instead of a shift and multiply-high and pass 2 addresses the image with
// the entry itself.  C2 (5 << 25: 256 bins of 80 KiB) and C5 (5 << 27: 512
// of 160 KiB) take it; C4 (3 << 30, 2,458 segments) keeps segments.
bool plan_build(uint64_t m, int ncu, PartitionWorkspace *ws);

// Probe: filters up to this size are gathered directly; larger ones use the
// partitioned probe when the batch has at least kProbePartitionMinKeys keys.
// Measured at C3 (16.8M GET keys, tools/probe_sweep.py): gather 134 us vs
// partition 247 us for the 5 MiB level-3 filter, 531 vs 259 us for the
// 20 MiB level 4 (gathers then miss the 4 MiB per-XCD L2 on most probes).
constexpr size_t kProbeGatherMaxBytes = 8u << 20;
// Filters of at most kLdsBitmapBytes are probed from LDS (k_probe_lds) once
// the batch has this many keys (each workgroup stages the whole filter).
constexpr size_t kProbeLdsMinKeys = 1u << 16;
constexpr size_t kProbePartitionMinKeys = 1u << 18;

// Stacked probe (BLOOMHIP_PROBE_STACKED): up to kMaxStack filters whose sizes
// all divide the largest one, m_max, probed in ONE partitioned pass.  For
// m_j | m_max, x % m_j == (x % m_max) % m_j, so the positions modulo m_max
// alone place every member's bits: with a segment width w dividing every
// m_j, bit p (< m_max) of segment b = p / w at offset o = p % w lands in
// member j's segment b % (m_j / w) at the same offset o.  Pass 2 holds the w-bit
// segment of every member in LDS and writes one result byte per sorted entry
// (bit j = member j's bit); the combine ANDs each key's three bytes.
// MI355X's Infinity Cache (MALL): a pass-2 input larger than this comes from HBM
constexpr uint64_t kInfinityCacheBytes = 256ull << 20;
constexpr int kMaxStack = 8;

// Ladder stack: every member is m_j = d << t_j with the same odd d | 255
// (the p2 form of bloom_math.h) -- an LSM's levels at a power-of-two fanout
// (C3: d = 5, t_j = 17, 19, ..., 25).  Then x % m_j = a_j << t_j | (x mod
// 2^t_j) with a_j = (x >> t_j) % d, and a_j follows from the largest
// member's a_max and the hash bits between: a_j = (a_max * 2^(t_max - t_j) +
// bits [t_j, t_max) of x) % d.  Pass 1 bins positions by hash bits [s, s+u)
// (2^u = 256 bins, one per CU, s <= t_min, s + u <= t_max) and keeps the
// entry e = (a_max << hb | bits [s+u, t_max)) << s | bits [0, s), hb =
// t_max - s - u.  For bin b every member's bits that such an entry can
// reach are whole blocks of 2^s bits: member j's block i is
//   t_j >= s+u: a = i >> (t_j-s-u), h = i mod 2^(t_j-s-u): bits from
//               a << t_j | h << (s+u) | b << s,
//   t_j <  s+u: a = i: bits from a << t_j | (b mod 2^(t_j - s)) << s,
// (d << max(0, t_j - s - u) blocks).  Members 0 .. k-1 ("direct") have
// their blocks staged in LDS (block q at LDS word q * 2^(s-5)); the smaller
// members k .. nf-1 ("packed") are merged into one image of bpp (4 or 8)
// bits per position: for each block i of member k (a "tuple": every smaller
// member's block follows from it and the bin), position p holds bit j - k =
// member j's bit, so one LDS read answers all packed members.  A table
// from e >> s (member 0's block) gives the LDS byte addresses of the other
// direct members' blocks and of the packed image's tuple (one word each, rs
// words per row).  Runs are as long as the build's (256 bins
// instead of the segment stack's 1,280 at C3) and each member bit is staged
// once per bin.
struct LadderTable {
    uint32_t s, u, hb, d;       // geometry as above
    uint32_t ne;                // d << hb: entry high parts (table rows)
    uint32_t k;                 // direct members (1 .. nf)
    uint32_t bpp;               // packed bits per position: 4 or 8 (0: none, k == nf)
    uint32_t pk_words;          // LDS word where the packed image starts (tuple-aligned)
    uint32_t img_words;         // LDS words of the direct blocks + packed image (the table follows)
    uint32_t rs;                // table row stride in words: 1, 2, 4 or 8
    uint32_t t[kMaxStack];      // member j is d << t[j] (member 0 the largest)
    uint32_t nblk[kMaxStack];   // member j's blocks per bin (packed members: tuples = nblk[k])
    uint32_t base[kMaxStack];   // direct member j's first block in the image
    uint32_t pmod[kMaxStack];   // 2^(t_max - t_j) % d
    uint32_t pmodk[kMaxStack];  // 2^(t_k - t_j) % d (packed members j > k)
    // Computed tuple (k = 1, ctup = 1): no table.  Member 1's block for an
    // entry with high part hi = e >> s is hi mod nblk[1] (t_1 >= s + u: the
    // ladder identity on x >> (s + u)), i.e. hi - mulhi(hi, tmagic) * nblk[1]
    // (tmagic = ceil(2^32 / nblk[1]), checked exact for every hi < ne), so an
    // entry costs two LDS reads (member 0's word, the packed word) and the
    // images may fill all of the LDS.
    uint32_t ctup;
    uint32_t tmagic;
    // plan_build's one-member ladder (a build's pass 2, kApplyBuildL) after
    // the relabelled pass 1 (ladder0_relabel): 2^-(t-24) mod d, else 0
    uint32_t rinv;
};

struct StackTable {
    const uint32_t *words[kMaxStack];  // member bitmaps (32-bit word view)
    uint32_t mwords[kMaxStack];        // m_j / 32: member j's size in words (m_j % 128 == 0)
    int row[kMaxStack];                // output row of member j
    int nf;
    int ladder;                        // 1: lad holds a ladder geometry (plan_ladder)
    LadderTable lad;
    // Segment-stack pass 2 only, set at its launch (stack_stride): 0, or the
    // stride S of the persistent workgroups' segments (b, b + S, ...), and
    // the members whose windows are the same for all of them (bit j).
    int seg_stride;
    uint32_t keep_mask;
};

// Ladder geometry for members m[0] >= m[1] >= ... (all d << t_j with one d):
// fills st->lad / st->ladder and the workspace's bins; false when the members
// do not form a ladder or no (s, u) fits the LDS image, the entry's 21 bits
// and the table.  ncu sets u (2^u >= ncu bins).
// allow_computed = false: only the table forms (A/B of LadderTable::ctup).
bool plan_ladder(const uint64_t *m, int nf, int ncu, StackTable *st, PartitionWorkspace *ws,
                 bool allow_computed = true);
// LDS bytes of a ladder pass 2: the images, the table, and the tuple map
// (tuple -> packed members' blocks) used while the packed image is built.
inline size_t ladder_lds_bytes(const LadderTable &l) {
    if (l.ctup) return (size_t)l.img_words * 4;
    return (size_t)l.img_words * 4 + (size_t)l.ne * l.rs * 4 + (l.bpp ? (size_t)l.nblk[l.k] * 32 : 0);
}


// Kernels enqueued on `stream`; all return hipSuccess or the launch error.
hipError_t launch_build_atomic(const KeySpan &keys, const ModParams &mp, uint32_t *words,
                               hipStream_t stream);
hipError_t launch_build_lds(const KeySpan &keys, const ModParams &mp, uint32_t *words,
                            hipStream_t stream);
hipError_t launch_part_bin(const KeySpan &keys, const ModParams &mp, const PartitionWorkspace &ws,
                           hipStream_t stream);
// merge_existing: OR into the current bitmap instead of overwriting segments.
hipError_t launch_part_apply(const ModParams &mp, uint32_t *words, const PartitionWorkspace &ws,
                             int merge_existing, hipStream_t stream);
// Probe of one filter with m/8 <= kLdsBitmapBytes staged in LDS; out[w]
// packs keys 64w .. 64w+63.
hipError_t launch_probe_lds(const KeySpan &keys, const ModParams &mp, const uint32_t *words,
                            uint64_t *out, size_t nw_out, hipStream_t stream);
hipError_t launch_probe(const KeySpan &keys, const ProbeTable &t, uint64_t *out, size_t nwords_out,
                        hipStream_t stream);
// Scalar set / is_set of one key passed by value (one lane); is_set writes 0/1
// to *hit (a mapped host word or device memory).
hipError_t launch_set1(uint32_t *words, const ModParams &mp, int32_t key, hipStream_t stream);
hipError_t launch_is_set1(const uint32_t *words, const ModParams &mp, int32_t key, uint32_t *hit,
                          hipStream_t stream);
// meta[0] = max key, meta[1 ..] = the ceil(n / kFenceStride) fences of a run.
hipError_t launch_run_meta(const KeySpan &keys, int32_t *meta, hipStream_t stream);
// The same for keys known sorted ascending: fences read directly, max = last key.
hipError_t launch_run_meta_sorted(const KeySpan &keys, int32_t *meta, hipStream_t stream);
// Applies the range checks to the probe rows `cand` in place and writes the
// newest candidate run and its page index per key (first/page may be null).
hipError_t launch_route(const KeySpan &keys, const RouteTable &t, uint64_t *cand, size_t nw,
                        const RouteOut &ro, hipStream_t stream);
// Partitioned probe of one filter (nbins as plan_segments): bin the
// keys' positions by segment (recording each position's sorted slot), test
// each segment in LDS writing one result byte per sorted entry, then AND each
// key's three bytes into out[ceil(n/64)].  Workspace: res holds
// ntiles*kPartTilePos bytes, slots ntiles*3*kPartTileKeys u16.
// Stacked probe of st.nf members (see StackTable) whose largest has
// ModParams mp_max; ws from plan_stack, res/slots as for the partitioned
// probe.  Row st.row[j] of out (nw words per row) gets member j's results.
// rt (GET routing fused into the combine, k_probe_combine_route): every run
// of the routing call is a member (rt->nruns == st.nf, st.row a permutation)
// and their fences fit kRouteLdsFenceBytesMax; out then gets the range-checked
// candidate rows and the route outputs (each may be null) what k_route writes.
hipError_t launch_probe_stacked(const KeySpan &keys, const ModParams &mp_max, const StackTable &st,
                                const PartitionWorkspace &ws, uint8_t *res, uint16_t *slots,
                                uint64_t *out, size_t nw, hipStream_t stream,
                                const RouteTable *rt = nullptr, const RouteOut &ro = RouteOut{});
hipError_t launch_probe_partitioned(const KeySpan &keys, const ModParams &mp, const uint32_t *words,
                                    const PartitionWorkspace &ws, uint8_t *res, uint16_t *slots,
                                    uint64_t *out, hipStream_t stream);

}  // namespace bloomhip
