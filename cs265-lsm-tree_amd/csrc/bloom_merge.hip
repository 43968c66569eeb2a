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

// ---------------------------------------------------------------------------
// One-pass k-way compaction (k <= kKwayMaxRuns): merge, newest-wins dedup,
// tombstone drop and the packed kept keys in ONE pass over the entries.
//
// Total order of all entries: (key, run, index) -- run 0 is the newest, so
// among equal keys the newest run's first entry comes first, exactly the
// entry MergeContext releases (src/merge.cpp:17-35); an entry is kept when its
// key differs from its predecessor's in this order (and it is not a dropped
// tombstone).
//
// Partitions: every kKwayS-th entry of every run is a sample; the samples'
// ranks in the total order (k_kway_split: binary searches over the other
// runs' samples) pick every q-th sample as a partition start, and the
// start's position in each run is found by a binary search between two of
// that run's samples.  A partition holds exactly q samples, so at most
// (q + k) * kKwayS entries: with q = kKwayCap / kKwayS - k it fits one
// workgroup's LDS whatever the key distribution or duplicates (q fixed at 8
// for every k left a fan-in-4 partition half full on average: twice the
// partitions, each paying the ticket, bounds and look-back latencies).  k_kway_merge merges a partition's k shares in
// LDS (log2 k rounds of stable merge-path merges, the newer list on the
// left), flags the kept entries, and places them with a decoupled look-back
// over the partitions' kept counts (partitions taken in ticket order, so
// every partition waits only on ones already running).
// ---------------------------------------------------------------------------
constexpr int kKwayS = 256;                                    // sample stride
constexpr int kKwayCap = 32 * kKwayS;                          // entries per partition, at most (64 KiB)
static_assert(kKwayCap / kKwayS > kKwayMaxRuns, "at least one sample per partition");
constexpr int kKwayBlock = 1024;
constexpr int kKwayIpt = kKwayCap / kKwayBlock;                // outputs per lane per round
static_assert(kKwayIpt * kKwayBlock == kKwayCap, "whole outputs per lane");

struct KwayRuns {
    const Entry *run[kKwayMaxRuns];
    uint64_t n[kKwayMaxRuns];
    uint64_t soff[kKwayMaxRuns + 1];  // run r's samples at skeys[soff[r] .. soff[r + 1])
    int k;
    uint32_t q;  // samples per partition (kway_q)
};

// Also zeroes the look-back state and the ticket (np <= samples: a launch
// of its own cost more than the stores).
__global__ void __launch_bounds__(256) k_kway_samples(KwayRuns R, int32_t *__restrict__ skeys,
                                                      uint64_t *__restrict__ status, uint32_t np,
                                                      uint32_t *__restrict__ ticket) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g < np) status[g] = 0;
    if (g == 0) *ticket = 0;
    if (g >= R.soff[R.k]) return;
    int r = 0;
    while (r + 1 < R.k && R.soff[r + 1] <= g) r++;
    skeys[g] = R.run[r][(g - R.soff[r]) * kKwayS].key;
}

// Entries of run rr before (x, r) in the total order: key < x, or key == x
// and rr < r (a newer run's equal keys come first).
__device__ __forceinline__ bool kway_before(int32_t key, int32_t x, int rr, int r) {
    return key < x || (key == x && rr < r);
}

// Thread per sample: its rank; a rank that is a multiple of R.q starts a
// partition, whose bounds in every run this thread writes.
__global__ void __launch_bounds__(256) k_kway_split(KwayRuns R, const int32_t *__restrict__ skeys,
                                                   uint32_t *__restrict__ bounds, uint32_t nparts) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const int k = R.k;
    if (g == 0) {
        for (int rr = 0; rr < k; rr++) {
            bounds[rr] = 0;
            bounds[(size_t)nparts * kKwayMaxRuns + rr] = (uint32_t)R.n[rr];
        }
    }
    if (g >= R.soff[k]) return;
    int r = 0;
    while (r + 1 < k && R.soff[r + 1] <= g) r++;
    const uint64_t j = g - R.soff[r];
    const int32_t x = skeys[g];
    // samples of every other run before (x, r): k - 1 lower bounds, their
    // loads interleaved (one dependent step for all runs at a time)
    uint32_t lo[kKwayMaxRuns], hi[kKwayMaxRuns];
    uint32_t maxlen = 0;
#pragma unroll
    for (int rr = 0; rr < kKwayMaxRuns; rr++) {
        lo[rr] = 0;
        hi[rr] = rr < k && rr != r ? (uint32_t)(R.soff[rr + 1] - R.soff[rr]) : 0u;
        maxlen = max(maxlen, hi[rr]);
    }
    for (uint32_t span = maxlen; span > 0; span >>= 1) {
#pragma unroll
        for (int rr = 0; rr < kKwayMaxRuns; rr++) {
            if (lo[rr] < hi[rr]) {
                const uint32_t mid = (lo[rr] + hi[rr]) >> 1;
                if (kway_before(skeys[R.soff[rr] + mid], x, rr, r)) lo[rr] = mid + 1;
                else hi[rr] = mid;
            }
        }
    }
    uint64_t rank = j;
#pragma unroll
    for (int rr = 0; rr < kKwayMaxRuns; rr++)
        if (rr < k && rr != r) rank += lo[rr];
    if (rank == 0 || rank % R.q != 0) return;
    const uint64_t p = rank / R.q;
    // the partition start's position in run rr: c samples of rr come before
    // it, so it lies in ((c - 1) * S, c * S]; a lower bound in that window
    uint32_t a[kKwayMaxRuns], b[kKwayMaxRuns];
    uint32_t wmax = 0;
#pragma unroll
    for (int rr = 0; rr < kKwayMaxRuns; rr++) {
        const uint32_t c = lo[rr];
        a[rr] = c > 0 ? (c - 1) * kKwayS + 1 : 0u;
        b[rr] = rr < k && rr != r ? (uint32_t)min((uint64_t)c * kKwayS, R.n[rr]) : 0u;
        if (rr >= k || rr == r) a[rr] = b[rr];
        wmax = max(wmax, b[rr] - a[rr]);
    }
    for (uint32_t span = wmax; span > 0; span >>= 1) {
#pragma unroll
        for (int rr = 0; rr < kKwayMaxRuns; rr++) {
            if (a[rr] < b[rr]) {
                const uint32_t mid = (a[rr] + b[rr]) >> 1;
                if (kway_before(R.run[rr][mid].key, x, rr, r)) a[rr] = mid + 1;
                else b[rr] = mid;
            }
        }
    }
#pragma unroll
    for (int rr = 0; rr < kKwayMaxRuns; rr++)
        if (rr < k) bounds[p * kKwayMaxRuns + rr] = rr == r ? (uint32_t)(j * kKwayS) : a[rr];
}

// Look-back status of a partition: flag in bits 62-63 (1 = its own kept
// count, 2 = the inclusive prefix of kept counts), value below.
constexpr uint64_t kKwayAgg = 1ull << 62, kKwayIncl = 2ull << 62, kKwayVal = (1ull << 62) - 1;

// One workgroup per partition (taken in ticket order).  One LDS buffer: each
// merge round's outputs are computed into registers (kKwayIpt entries per
// lane), then written back over the round's input after a barrier, so a
// 1024-lane workgroup takes 64 KiB and two fit a CU (two buffers halved
// that: the kernel is latency-bound).  Partitions of up to 8192 entries on
// 1024 lanes: 189 us at fan-in 4 against 210 for 4096 on 512 lanes (four per
// CU; each partition pays the ticket, its bounds and the look-back) and 260
// for 16384 on 1024 lanes (one per CU).  Persistent workgroups that took the next ticket
// and loaded the next bounds during a partition's merge were slower (292 us
// against 221 at fan-in 4, rocprofv3): they spilled at 4 workgroups per CU,
// and a workgroup held in the look-back held its later partitions too.
__global__ void __launch_bounds__(kKwayBlock, 2) k_kway_merge(
    KwayRuns R, const uint32_t *__restrict__ bounds, uint32_t nparts, int drop,
    uint64_t *__restrict__ status, uint32_t *__restrict__ ticket, Entry *__restrict__ out,
    int32_t *__restrict__ keys_out, uint32_t *__restrict__ count_out) {
    __shared__ __attribute__((aligned(16))) Entry s_buf[kKwayCap];
    __shared__ uint32_t s_off[kKwayMaxRuns + 1];
    __shared__ uint32_t s_lo[kKwayMaxRuns];
    __shared__ uint32_t s_w[kKwayBlock / 64];
    __shared__ uint64_t s_im[kKwayBlock / 64], s_zm[kKwayBlock / 64];
    __shared__ uint32_t s_p;
    __shared__ uint64_t s_base;
    __shared__ int32_t s_pred;
    __shared__ int s_has_pred;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, k = R.k;
    if (tid == 0) s_p = atomicAdd(ticket, 1u);  // ticket order: predecessors are running
    __syncthreads();
    const uint32_t p = s_p;
    // the shares and the entry just before the partition (its predecessor):
    // lane r of the first wave reads run r's bounds
    if (tid < 64) {
        const int r = tid;
        uint32_t lo = 0, c = 0;
        if (r < k) {
            lo = bounds[(size_t)p * kKwayMaxRuns + r];
            c = bounds[(size_t)(p + 1) * kKwayMaxRuns + r] - lo;
        }
        // exclusive prefix of the share sizes over lanes 0..k-1 (k <= 8)
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < kKwayMaxRuns; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off, 64);
            if (r >= off) incl += o;
        }
        if (r < k) {
            s_lo[r] = lo;
            s_off[r] = incl - c;
        }
        if (r == k - 1) s_off[k] = incl;
    }
    __syncthreads();
    const int total = (int)s_off[k];
    // every load of the partition in flight at once: this lane's kKwayIpt
    // positions of the concatenated shares (strided, so each load instruction
    // is coalesced), and (lanes 0..k-1) the key just before run r's share; a
    // load-then-store loop per run waited for each run's loads in turn
    const int d0 = tid * kKwayIpt;  // this lane's outputs of the merge: [d0, d0 + kKwayIpt)
    Entry mine[kKwayIpt];
    {
        int r = 0;
#pragma unroll
        for (int i = 0; i < kKwayIpt; i++) {
            const int d = tid + i * kKwayBlock;
            if (d < total) {
                while ((int)s_off[r + 1] <= d) r++;
                mine[i] = R.run[r][s_lo[r] + (uint32_t)(d - (int)s_off[r])];
            }
        }
    }
    int32_t pkey = INT32_MIN;
    const bool phas = tid < k && s_lo[tid] > 0;
    if (phas) pkey = R.run[tid][s_lo[tid] - 1].key;
    {
        // the total order's last entry before the partition: the largest key
        const uint64_t hm = __ballot(phas);
        int32_t mk = phas ? pkey : INT32_MIN;
        if (tid < 64) {
#pragma unroll
            for (int off = 4; off >= 1; off >>= 1) mk = max(mk, __shfl_xor(mk, off, 64));
            if (tid == 0) {
                s_has_pred = hm != 0;
                s_pred = mk;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < kKwayIpt; i++)
        if (tid + i * kKwayBlock < total) s_buf[tid + i * kKwayBlock] = mine[i];
    __syncthreads();
    if (k == 1) {  // no merge round: this lane's outputs straight from the staged run
#pragma unroll
        for (int i = 0; i < kKwayIpt; i++) mine[i] = d0 + i < total ? s_buf[d0 + i] : Entry{0, 0};
    }
    // merge rounds: lists L_q = [ofs[q], ofs[q + 1]); pairs (0,1), (2,3), ...
    // go out at the same offsets (adjacent lists merge in place of both).
    // The list bounds live in LDS (s_off, updated between rounds): a private
    // array indexed by the lane's pair went to scratch memory.
    const uint32_t *ofs = s_off;
    int nl = k;
    while (nl > 1) {
        const int np = (nl + 1) / 2;
        // this lane's outputs of the round, into registers: one merge-path
        // search where the lane enters a pair, then a sequential merge with
        // both lists' head entries held in registers (one 8-B LDS read per
        // output, for the entry that replaces the one taken; reading both
        // heads' keys and then the taken entry per output was three)
        int a1 = 0, b1 = -1, ia = 0, ib = 0;
        Entry ea{0, 0}, eb{0, 0};
#pragma unroll
        for (int i = 0; i < kKwayIpt; i++) {
            const int d = d0 + i;
            if (d < total) {
                if (d >= b1) {
                    // the pair holding output d (pairs are consecutive output ranges)
                    int q = 0;
                    while (q + 1 < np && (int)ofs[min(2 * (q + 1), nl)] <= d) q++;
                    const int a0 = (int)ofs[2 * q];
                    a1 = (int)ofs[min(2 * q + 1, nl)];
                    b1 = (int)ofs[min(2 * q + 2, nl)];
                    const int na = a1 - a0, nb = b1 - a1, dd = d - a0;
                    // A entries among the pair's first dd outputs (A wins ties)
                    int lo = dd > nb ? dd - nb : 0, hi = dd < na ? dd : na;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (s_buf[a0 + mid].key <= s_buf[a1 + dd - 1 - mid].key) lo = mid + 1;
                        else hi = mid;
                    }
                    ia = a0 + lo;       // absolute LDS indices of the next A and B entries
                    ib = a1 + dd - lo;
                    ea = s_buf[min(ia, kKwayCap - 1)];  // past a list's end: never taken
                    eb = s_buf[min(ib, kKwayCap - 1)];
                }
                const bool take_a = ia < a1 && (ib >= b1 || ea.key <= eb.key);
                mine[i] = take_a ? ea : eb;
                const int nx = take_a ? ++ia : ++ib;
                const Entry e = s_buf[min(nx, kKwayCap - 1)];
                if (take_a) ea = e;
                else eb = e;
            }
        }
        __syncthreads();  // every lane's reads of this round's lists and bounds
#pragma unroll
        for (int i = 0; i < kKwayIpt; i++)
            if (d0 + i < total) s_buf[d0 + i] = mine[i];
        // the merged lists' bounds: list q of the next round is pair q
        if (tid == 0)
            for (int q = 1; q <= np; q++) s_off[q] = s_off[min(2 * q, nl)];
        nl = np;
        __syncthreads();
    }
    // kept flags of this lane's outputs, in order
    uint32_t keep = 0, c = 0;
#pragma unroll
    for (int i = 0; i < kKwayIpt; i++) {
        const int d = d0 + i;
        if (d < total) {
            const Entry e = mine[i];
            const int32_t pkey = i > 0 ? mine[i - 1].key : d > 0 ? s_buf[d - 1].key : s_pred;
            const bool first = d > 0 ? pkey != e.key : (!s_has_pred || s_pred != e.key);
            const bool kk = first && !(drop && e.val == kTombstone);
            keep |= (uint32_t)kk << i;
            c += kk;
        }
    }
    uint32_t ctot;
    const uint32_t excl = block_exclusive_scan(c, s_w, &ctot);
    // Decoupled look-back over the partitions' kept counts, the whole block
    // reading 512 predecessors' states per step (one wave's 64 per step took
    // 8 dependent steps to cross the 512 partitions running at once); the
    // nearest inclusive prefix ends it.  Relaxed agent-scope atomics (only
    // the counts travel).
    if (p == 0) {
        if (tid == 0) {
            __hip_atomic_store(&status[0], kKwayIncl | ctot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_base = 0;
        }
    } else {
        if (tid == 0) {
            __hip_atomic_store(&status[p], kKwayAgg | ctot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // wait for the nearest predecessor alone (one load per try) before
            // reading the window: 512 loads per try while it runs would load
            // the memory system for every other workgroup
            while (__hip_atomic_load(&status[p - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();
        uint64_t base = 0;
        for (int64_t q0 = (int64_t)p - 1;;) {
            const int64_t q = q0 - tid;  // thread 0 reads the nearest predecessor
            const uint64_t v = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : kKwayIncl;  // before partition 0: an empty prefix
            const uint64_t im = __ballot((v & kKwayIncl) != 0), zm = __ballot(v == 0);
            if (lane == 0) {
                s_im[wave] = im;
                s_zm[wave] = zm;
            }
            __syncthreads();
            // the nearest inclusive prefix: thread index F (kKwayBlock: none)
            int F = kKwayBlock;
            bool waiting = false;
            for (int w = 0; w < kKwayBlock / 64; w++) {
                const uint64_t iw = s_im[w], zw = s_zm[w];
                if (iw) {
                    const int fi = __builtin_ctzll(iw);
                    waiting = (zw & (fi < 63 ? (2ull << fi) - 1 : ~0ull)) != 0;
                    F = w * 64 + fi;
                    break;
                }
                if (zw) {
                    waiting = true;
                    break;
                }
            }
            __syncthreads();  // s_im / s_zm read by all before the next step writes them
            if (waiting) {  // a predecessor has not published yet: read again
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t tsum;
            (void)block_exclusive_scan(tid <= F ? (uint32_t)(v & kKwayVal) : 0u, s_w, &tsum);
            base += tsum;
            if (F < kKwayBlock) break;
            q0 -= kKwayBlock;
        }
        if (tid == 0) {
            __hip_atomic_store(&status[p], kKwayIncl | (base + ctot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            s_base = base;
        }
    }
    // system scope: the host may spin on this word (pinned, mapped) to size
    // the next launch before the merge has drained
    if (tid == 0 && p + 1 == nparts)
        __hip_atomic_store(count_out, (uint32_t)(s_base + ctot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();  // every lane's reads of s_buf above are done
    // kept entries packed in place in LDS (they only move down), then written out coalesced
    uint32_t w = excl;
#pragma unroll
    for (int i = 0; i < kKwayIpt; i++)
        if ((keep >> i) & 1u) s_buf[w++] = mine[i];
    __syncthreads();
    const uint64_t base = s_base;
    for (int i = tid; i < (int)ctot; i += kKwayBlock) {
        const Entry e = s_buf[i];
        out[base + i] = e;
        if (keys_out) keys_out[base + i] = e.key;
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

namespace bloomhip {

namespace {
uint32_t kway_q(int k) { return (uint32_t)(kKwayCap / kKwayS - k); }
}  // namespace

uint64_t kway_parts(const uint64_t *n, int k) {
    uint64_t ns = 0;
    for (int r = 0; r < k; r++) ns += (n[r] + kKwayS - 1) / kKwayS;
    return ns ? (ns - 1) / kway_q(k) + 1 : 0;
}

uint64_t kway_workspace_bytes(const uint64_t *n, int k) {
    uint64_t ns = 0;
    for (int r = 0; r < k; r++) ns += (n[r] + kKwayS - 1) / kKwayS;
    const uint64_t np = kway_parts(n, k);
    // samples | bounds (np + 1 rows) | status (np) + ticket + count
    return ((ns * 4 + 15) & ~15ull) + (np + 1) * kKwayMaxRuns * 4 + 16 + np * 8 + 16;
}

hipError_t launch_compact_kway(const void *const *runs, const uint64_t *n, int k, int drop,
                               void *out, int32_t *keys_out, void *ws, uint32_t *count_out,
                               hipStream_t stream) {
    if (k < 1 || k > kKwayMaxRuns) return hipErrorInvalidValue;
    KwayRuns R{};
    R.k = k;
    R.q = kway_q(k);
    uint64_t ns = 0;
    for (int r = 0; r < k; r++) {
        if (n[r] == 0 || (reinterpret_cast<uintptr_t>(runs[r]) & 7)) return hipErrorInvalidValue;
        R.run[r] = reinterpret_cast<const Entry *>(runs[r]);
        R.n[r] = n[r];
        R.soff[r] = ns;
        ns += (n[r] + kKwayS - 1) / kKwayS;
    }
    R.soff[k] = ns;
    const uint64_t np = kway_parts(n, k);
    if (np == 0 || np >= (1ull << 31)) return hipErrorInvalidValue;
    char *b = reinterpret_cast<char *>(ws);
    int32_t *skeys = reinterpret_cast<int32_t *>(b);
    b += (ns * 4 + 15) & ~15ull;
    uint32_t *bounds = reinterpret_cast<uint32_t *>(b);
    b += (np + 1) * kKwayMaxRuns * 4;
    b = reinterpret_cast<char *>((reinterpret_cast<uintptr_t>(b) + 15) & ~(uintptr_t)15);
    uint64_t *status = reinterpret_cast<uint64_t *>(b);
    uint32_t *ticket = reinterpret_cast<uint32_t *>(status + np);
    const unsigned gs = (unsigned)((ns + 255) / 256);
    if ((uint64_t)gs * 256 < np) return hipErrorInvalidValue;  // the samples launch zeroes status
    k_kway_samples<<<gs, 256, 0, stream>>>(R, skeys, status, (uint32_t)np, ticket);
    k_kway_split<<<gs, 256, 0, stream>>>(R, skeys, bounds, (uint32_t)np);
    k_kway_merge<<<(unsigned)np, kKwayBlock, 0, stream>>>(R, bounds, (uint32_t)np, drop, status, ticket,
                                                  reinterpret_cast<Entry *>(out), keys_out, count_out);
    return hipGetLastError();
}

}  // namespace bloomhip
