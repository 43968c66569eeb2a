// bloom_merge.hip — SURVEY §8f row 3: the compaction that produces a run's
// keys, fused with that run's filter build.
//
// Reference: MergeContext (src/merge.h:8-37, src/merge.cpp:6-39) pops the
// smallest (key, precedence) head of k sorted runs — precedence = the order
// runs were added, newest first (LSMTree::merge_down iterates a level's
// runs front to back, src/lsm_tree.cpp:74-76, and runs are emplace_front'ed,
// :78,125) — and releases only the newest entry of each key; merge_down drops
// entries whose value is VAL_TOMBSTONE when writing the last level
// (src/lsm_tree.cpp:81-88).  Run::put then sets the filter bits and fences.
//
// On the GPU: a tree of stable 2-way merges (merge path: per 2048-output tile
// a binary search on the cross diagonal picks each input's share, the tile is
// staged in LDS and each lane merges 8 outputs), left input always the newer,
// so equal keys come out newest first; then one compaction pass keeps the
// first entry of each key (dropping tombstones on request) with a block scan
// and a scan over the block counts.  Every pass streams entries through HBM
// with coalesced 16-B accesses; the filter build runs on the merged keys in
// place (stride 8).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_merge.h"

namespace bloomhip {
namespace {

constexpr int kMergeBlock = 256;
constexpr int kMergeIpt = 8;                          // outputs per lane
constexpr int kMergeTile = kMergeBlock * kMergeIpt;  // outputs per workgroup
constexpr int32_t kTombstone = INT32_MIN;            // VAL_TOMBSTONE, src/types.h:12

struct Entry {
    int32_t key, val;
};

// Number of A entries among the first d outputs of the stable merge (A wins
// ties): the largest i with A[i-1] before B[d-i].
template <typename GetA, typename GetB>
__device__ __forceinline__ uint64_t merge_path(GetA a_key, uint64_t na, GetB b_key, uint64_t nb,
                                               uint64_t d) {
    uint64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a_key(mid) <= b_key(d - 1 - mid)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One thread per tile boundary, a binary merge-path search.  (Wider searches
// were slower: a 64-ary search by one wave per boundary 31 vs 22 us, its 128
// scattered loads per round missing where the serial searches' first levels
// share cached lines; a 16-ary search by one thread, 15 probes per round,
// 79 vs 23 us: 30 scattered loads per round and thread queue in the address
// units of the few CUs the 33 workgroups occupy.)
// The pairs of one merge round, launched together (their tiles and split
// searches share one grid: a round of fan-in 4 pays one split latency, not
// two).  Pair p's tiles are [tile0[p], tile0[p + 1]); its splits sit at
// split_ws[tile0[p] + p ..] (ntiles_p + 1 of them).
struct MergeRound {
    const Entry *a[kMaxMergePairs];
    const Entry *b[kMaxMergePairs];
    Entry *out[kMaxMergePairs];
    uint64_t na[kMaxMergePairs], nb[kMaxMergePairs];
    uint64_t tile0[kMaxMergePairs + 1];
    int np;
};

__global__ void k_merge_split(MergeRound R, uint64_t *__restrict__ split) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= R.tile0[R.np] + (uint64_t)R.np) return;
    int p = 0;
    for (int q = 1; q < R.np; q++)
        if (R.tile0[q] + (uint64_t)q <= t) p = q;
    const uint64_t lt = t - (R.tile0[p] + (uint64_t)p);  // boundary lt of pair p
    const Entry *a = R.a[p], *b = R.b[p];
    const uint64_t na = R.na[p], nb = R.nb[p];
    const uint64_t d = min(lt * (uint64_t)kMergeTile, na + nb);
    split[t] = merge_path([&](uint64_t i) { return a[i].key; }, na,
                          [&](uint64_t j) { return b[j].key; }, nb, d);
}

// A merge tile: the tile's share of A and of B staged in LDS, one merge-path
// search per lane in LDS, 8 outputs per lane, the tile written back.  Global
// traffic moves in 16-B vectors: a share is copied in the 16-B-aligned
// vectors (by address) that cover it and lands at the same parity in LDS;
// a vector that reaches outside its array is copied entry by entry.  The
// output tile starts at an even entry of a 16-B-aligned output (launch_merge2
// checks) and leaves as 16-B stores.
// Entries s0 .. s0+cnt-1 of src go to dst[par + k], par = the address parity
// of src + s0 (in entries); dst is 16-B aligned.
__device__ __forceinline__ void stage_share(const Entry *__restrict__ src, uint64_t n,
                                            uint64_t s0, int cnt, int par, Entry *dst) {
    if (cnt <= 0) return;
    const int nv = (par + cnt + 1) / 2;
    int4 *d4 = reinterpret_cast<int4 *>(dst);
    for (int v = threadIdx.x; v < nv; v += kMergeBlock) {
        const int64_t e = (int64_t)s0 - par + 2 * (int64_t)v;  // the vector's first entry
        if (e >= 0 && (uint64_t)e + 1 < n) {
            d4[v] = *reinterpret_cast<const int4 *>(src + e);
        } else {
            if (e >= 0 && (uint64_t)e < n) dst[2 * v] = src[e];
            if (e + 1 >= 0 && (uint64_t)(e + 1) < n) dst[2 * v + 1] = src[e + 1];
        }
    }
}

__global__ void __launch_bounds__(kMergeBlock) k_merge_tile(MergeRound R,
                                                            const uint64_t *__restrict__ splits) {
    __shared__ __attribute__((aligned(16))) Entry s_in[kMergeTile + 4];
    __shared__ __attribute__((aligned(16))) Entry s_out[kMergeTile];
    int p = 0;
    for (int q = 1; q < R.np; q++)
        if (R.tile0[q] <= blockIdx.x) p = q;
    const Entry *__restrict__ a = R.a[p];
    const Entry *__restrict__ b = R.b[p];
    Entry *__restrict__ out = R.out[p];
    const uint64_t na = R.na[p], nb = R.nb[p];
    const uint64_t *split = splits + R.tile0[p] + p;
    const uint64_t t = blockIdx.x - R.tile0[p];
    const uint64_t d0 = t * kMergeTile, d1 = min(d0 + kMergeTile, na + nb);
    const uint64_t a0 = split[t], a1 = split[t + 1];
    const uint64_t b0 = d0 - a0, b1 = d1 - a1;
    const int ta = (int)(a1 - a0), tb = (int)(b1 - b0);
    const int pa = (int)((reinterpret_cast<uintptr_t>(a + a0) >> 3) & 1);  // A at s_in[pa]
    const int pbp = (int)((reinterpret_cast<uintptr_t>(b + b0) >> 3) & 1);
    const int bb = (pa + ta + 1) & ~1;  // B's vectors from here
    const int pb = bb + pbp;            // B at s_in[pb]
    stage_share(a, na, a0, ta, pa, s_in);
    stage_share(b, nb, b0, tb, pbp, s_in + bb);
    __syncthreads();
    const int d = threadIdx.x * kMergeIpt;
    const int total = ta + tb;
    if (d < total) {
        const Entry *sa = s_in + pa, *sb = s_in + pb;
        int ia = (int)merge_path([&](uint64_t i) { return sa[i].key; }, (uint64_t)ta,
                                 [&](uint64_t j) { return sb[j].key; }, (uint64_t)tb, (uint64_t)d);
        int ib = d - ia;
        const int n = min(kMergeIpt, total - d);
        for (int k = 0; k < n; k++) {
            const bool take_a = ia < ta && (ib >= tb || sa[ia].key <= sb[ib].key);
            s_out[d + k] = take_a ? sa[ia++] : sb[ib++];
        }
    }
    __syncthreads();
    int4 *o4 = reinterpret_cast<int4 *>(out + d0);  // d0 even, out 16-B aligned
    const int4 *s4 = reinterpret_cast<const int4 *>(s_out);
    for (int i = threadIdx.x; i < total / 2; i += kMergeBlock) o4[i] = s4[i];
    if ((total & 1) && threadIdx.x == 0) out[d0 + total - 1] = s_out[total - 1];
}

// Keep entry i when it is the first (newest) of its key, and not a dropped
// tombstone.  A dedup tile is kCompactRounds rounds of kCompactBlock lanes x 2
// entries: lane l of round r owns entries 2l, 2l + 1 of the round's 512, read
// as one 16-B vector (coalesced), plus the key before them.
constexpr int kCompactBlock = 256;
constexpr int kCompactRounds = 8;
constexpr int kCompactTile = kCompactBlock * 2 * kCompactRounds;  // 4096 entries

struct Pair {
    Entry e0, e1;
    uint32_t k0, k1;  // keep flags
};

__device__ __forceinline__ Pair load_pair(const Entry *__restrict__ e, uint64_t n, uint64_t i,
                                          int drop) {
    Pair p{};
    if (i + 1 < n) {
        const int4 v = *reinterpret_cast<const int4 *>(e + i);  // i even: 16-B aligned
        p.e0 = Entry{v.x, v.y};
        p.e1 = Entry{v.z, v.w};
    } else if (i < n) {
        p.e0 = e[i];
    }
    const int32_t prev = i > 0 && i < n ? e[i - 1].key : 0;
    p.k0 = i < n && (i == 0 || prev != p.e0.key) && !(drop && p.e0.val == kTombstone);
    p.k1 = i + 1 < n && p.e1.key != p.e0.key && !(drop && p.e1.val == kTombstone);
    return p;
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *s_w,
                                                         uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t base = 0, all = 0;
    for (int w = 0; w < (int)(blockDim.x / 64); w++) {
        if (w < wave) base += s_w[w];
        all += s_w[w];
    }
    __syncthreads();
    if (total) *total = all;
    return base + incl - v;
}

__global__ void __launch_bounds__(kCompactBlock) k_compact_count(const Entry *__restrict__ e,
                                                                 uint64_t n, int drop,
                                                                 uint32_t *__restrict__ counts) {
    __shared__ uint32_t s_w[kCompactBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kCompactTile + 2 * (uint64_t)threadIdx.x;
    Pair p[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; r++)  // every load issued before any is used
        p[r] = load_pair(e, n, base + (uint64_t)r * 2 * kCompactBlock, drop);
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kCompactRounds; r++) c += p[r].k0 + p[r].k1;
    uint32_t total;
    (void)block_exclusive_scan(c, s_w, &total);
    if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

// Exclusive scan of the block counts in place (one workgroup), total in
// counts[nblocks].
__global__ void __launch_bounds__(1024) k_scan_counts(uint32_t *__restrict__ counts,
                                                      uint64_t nblocks) {
    __shared__ uint32_t s_w[1024 / 64];
    __shared__ uint64_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nblocks; b0 += 1024) {
        const uint64_t i = b0 + threadIdx.x;
        const uint32_t v = i < nblocks ? counts[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, s_w, &total);
        if (i < nblocks) counts[i] = (uint32_t)(s_carry + ex);
        __syncthreads();
        if (threadIdx.x == 0) s_carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[nblocks] = (uint32_t)s_carry;
}

// Kept entries leave in input order: per round, an exclusive scan of the
// lanes' kept counts places them, so a wave's stores cover one contiguous
// range of the output.
// keys_out (optional): the kept keys again, packed (stride 4), for the new
// run's filter build (pass 1 reads 4 B per key instead of 8).
__global__ void __launch_bounds__(kCompactBlock) k_compact_write(
    const Entry *__restrict__ e, uint64_t n, int drop, const uint32_t *__restrict__ offsets,
    Entry *__restrict__ out, int32_t *__restrict__ keys_out) {
    __shared__ uint32_t s_w[kCompactBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kCompactTile + 2 * (uint64_t)threadIdx.x;
    Pair p[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; r++)
        p[r] = load_pair(e, n, base + (uint64_t)r * 2 * kCompactBlock, drop);
    uint64_t run = offsets[blockIdx.x];
#pragma unroll
    for (int r = 0; r < kCompactRounds; r++) {
        uint32_t total;
        const uint64_t pos = run + block_exclusive_scan(p[r].k0 + p[r].k1, s_w, &total);
        if (p[r].k0) out[pos] = p[r].e0;
        if (p[r].k1) out[pos + p[r].k0] = p[r].e1;
        if (keys_out) {
            if (p[r].k0) keys_out[pos] = p[r].e0.key;
            if (p[r].k1) keys_out[pos + p[r].k0] = p[r].e1.key;
        }
        run += total;
    }
}

}  // namespace

hipError_t launch_merge_round(const MergePairArgs *pairs, int np, uint64_t *split_ws,
                              hipStream_t stream) {
    if (np < 1 || np > kMaxMergePairs) return hipErrorInvalidValue;
    MergeRound R{};
    R.np = np;
    uint64_t tiles = 0;
    for (int p = 0; p < np; p++) {
        // inputs 8-B aligned (entries), the output 16-B aligned (vector stores)
        if (((reinterpret_cast<uintptr_t>(pairs[p].a) | reinterpret_cast<uintptr_t>(pairs[p].b)) &
             7) ||
            (reinterpret_cast<uintptr_t>(pairs[p].out) & 15))
            return hipErrorInvalidValue;
        R.a[p] = reinterpret_cast<const Entry *>(pairs[p].a);
        R.b[p] = reinterpret_cast<const Entry *>(pairs[p].b);
        R.out[p] = reinterpret_cast<Entry *>(pairs[p].out);
        R.na[p] = pairs[p].na;
        R.nb[p] = pairs[p].nb;
        R.tile0[p] = tiles;
        tiles += (pairs[p].na + pairs[p].nb + kMergeTile - 1) / kMergeTile;
    }
    R.tile0[np] = tiles;
    if (tiles == 0) return hipSuccess;
    const uint64_t nsplit = tiles + (uint64_t)np;
    k_merge_split<<<(unsigned)((nsplit + 255) / 256), 256, 0, stream>>>(R, split_ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_merge_tile<<<(unsigned)tiles, kMergeBlock, 0, stream>>>(R, split_ws);
    return hipGetLastError();
}

hipError_t launch_merge2(const void *a, uint64_t na, const void *b, uint64_t nb, void *out,
                         uint64_t *split_ws, hipStream_t stream) {
    const MergePairArgs p{a, na, b, nb, out};
    return launch_merge_round(&p, 1, split_ws, stream);
}

uint64_t merge_split_words(uint64_t total) { return total / kMergeTile + 2 * kMaxMergePairs + 2; }
uint64_t compact_count_words(uint64_t n) { return (n + kCompactTile - 1) / kCompactTile + 1; }

hipError_t launch_dedup(const void *in, uint64_t n, int drop_tombstones, void *out,
                        uint32_t *counts_ws, hipStream_t stream, int32_t *keys_out) {
    const uint64_t nblocks = (n + kCompactTile - 1) / kCompactTile;
    const Entry *e = reinterpret_cast<const Entry *>(in);
    if (nblocks) {
        k_compact_count<<<(unsigned)nblocks, kCompactBlock, 0, stream>>>(e, n, drop_tombstones,
                                                                          counts_ws);
        hipError_t err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    k_scan_counts<<<1, 1024, 0, stream>>>(counts_ws, nblocks);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || nblocks == 0) return err;
    k_compact_write<<<(unsigned)nblocks, kCompactBlock, 0, stream>>>(
        e, n, drop_tombstones, counts_ws, reinterpret_cast<Entry *>(out), keys_out);
    return hipGetLastError();
}

}  // namespace bloomhip
