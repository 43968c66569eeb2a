// ubench.hip — micro-benchmarks that price the primitives the Bloom kernels
// are built from on gfx950: random 4-B global atomicOr (agent vs workgroup
// scope), random 4-B gathers, random LDS ds_or, and the exact hash+mod
// arithmetic alone.  Not part of the product path; used by
// tools/ubench.py to pick build strategies.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_kernels.hip"  // the product kernels, for ablation timing builds

using namespace bloomhip;

namespace {

__device__ __forceinline__ uint32_t xorshift(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

template <int SCOPE>
__global__ void ub_atomic_or(uint32_t *words, uint32_t nwords, int iters) {
    uint32_t s = 0x9E3779B9u ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    for (int i = 0; i < iters; i++) {
        const uint32_t r = xorshift(s);
        const uint32_t w = (uint32_t)(((uint64_t)r * nwords) >> 32);
        __hip_atomic_fetch_or(words + w, 1u << (r & 31), __ATOMIC_RELAXED, SCOPE);
    }
}

__global__ void ub_gather(const uint32_t *words, uint32_t nwords, int iters, uint32_t *sink) {
    uint32_t s = 0x9E3779B9u ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t r = xorshift(s);
        const uint32_t w = (uint32_t)(((uint64_t)r * nwords) >> 32);
        acc += words[w];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void ub_lds_or(int iters, uint32_t *sink) {
    extern __shared__ uint32_t seg[];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) seg[i] = 0;
    __syncthreads();
    uint32_t s = 0x9E3779B9u ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    for (int i = 0; i < iters; i++) {
        const uint32_t r = xorshift(s);
        atomicOr(&seg[r >> 18], 1u << (r & 31));
    }
    __syncthreads();
    if (seg[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

__global__ void ub_hash(ModParams mp, int iters, uint32_t *sink) {
    uint32_t acc = 0;
    int32_t k = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    for (int i = 0; i < iters; i++) {
        acc ^= mod_fast(raw_hash1(k), mp) + mod_fast(raw_hash2(k), mp) + mod_fast(raw_hash3(k), mp);
        k += 0x9E3779B9;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void ub_rawhash(int iters, uint32_t *sink) {
    uint64_t acc = 0;
    int32_t k = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    for (int i = 0; i < iters; i++) {
        acc ^= raw_hash1(k) + raw_hash2(k) + raw_hash3(k);
        k += 0x9E3779B9;
    }
    if (acc == 0x12345678u) sink[0] = (uint32_t)acc;
}

// VALU / LDS overlap probe: waves of the first `valu_waves` of each 16-wave
// workgroup run the hash+mod loop, the others random LDS ds_add_rtn (mode 0:
// both, 1: hash waves only (others exit), 2: LDS waves only).
template <int OP>  // LDS op of the non-hashing waves: 0 ds_add_rtn, 1 ds_write, 2 ds_read
__global__ void __launch_bounds__(1024) ub_mixed(ModParams mp, int valu_waves, int mode,
                                                 int hash_iters, int lds_iters, uint32_t *sink) {
    extern __shared__ uint32_t seg[];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) seg[i] = 0;
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    if (wave < valu_waves) {
        if (mode == 2) return;
        uint32_t acc = 0;
        int32_t k = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
        for (int i = 0; i < hash_iters; i++) {
            acc ^= mod_fast(raw_hash1(k), mp) + mod_fast(raw_hash2(k), mp) + mod_fast(raw_hash3(k), mp);
            k += 0x9E3779B9;
        }
        if (acc == 0x12345678u) sink[0] = acc;
    } else {
        if (mode == 1) return;
        uint32_t s = 0x9E3779B9u ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
        uint32_t acc = 0;
        for (int i = 0; i < lds_iters; i++) {
            s += 0x9E3779B9u;  // 1 VALU per op (a Weyl sequence), so the LDS waves stay LDS-bound
            const uint32_t r = s;
            if constexpr (OP == 0) acc += atomicAdd(&seg[r >> 18], 1u);  // pass 1's ranks
            else if constexpr (OP == 1) seg[r >> 18] = r;                  // the scatter
            else acc += seg[r >> 18];                                      // offset reads
        }
        if (acc == 0x12345678u) sink[0] = acc;
    }
}

__global__ void ub_stream(const uint4 *buf, size_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

}  // namespace

extern "C" int ubench_run(int which, void *dbuf, size_t bytes, uint64_t m, int grid, int block,
                          int iters, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t *w = reinterpret_cast<uint32_t *>(dbuf);
    const uint32_t nwords = (uint32_t)(bytes / 4 - 1);  // last word is the sink
    uint32_t *sink = w + nwords;
    switch (which) {
        case 0: ub_atomic_or<__HIP_MEMORY_SCOPE_AGENT><<<grid, block, 0, s>>>(w, nwords, iters); break;
        case 1: ub_atomic_or<__HIP_MEMORY_SCOPE_WORKGROUP><<<grid, block, 0, s>>>(w, nwords, iters); break;
        case 2: ub_gather<<<grid, block, 0, s>>>(w, nwords, iters, sink); break;
        case 3: ub_lds_or<<<grid, block, 65536, s>>>(iters, sink); break;
        case 4: ub_hash<<<grid, block, 0, s>>>(make_mod_params(m), iters, sink); break;
        case 5: ub_rawhash<<<grid, block, 0, s>>>(iters, sink); break;
        case 6: ub_stream<<<grid, block, 0, s>>>(reinterpret_cast<const uint4 *>(dbuf), bytes / 16 - 1, sink); break;
        case 10: case 11: case 12:  // block = waves doing VALU (of 16), iters = hash iters
            ub_mixed<0><<<grid, 1024, 65536, s>>>(make_mod_params(167772160), block, which - 10,
                                                  iters, iters * 6, sink);
            break;
        case 20: case 21: case 22:
            ub_mixed<1><<<grid, 1024, 65536, s>>>(make_mod_params(167772160), block, which - 20,
                                                  iters, iters * 6, sink);
            break;
        case 30: case 31: case 32:
            ub_mixed<2><<<grid, 1024, 65536, s>>>(make_mod_params(167772160), block, which - 30,
                                                  iters, iters * 6, sink);
            break;
        default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Pass 1 of the partition build: 0 = the product's launch, 1..3 = pass 1
// with phases removed (ABLATE), 4 = pass 1 writing run-start columns, 5 =
// pass 1 writing rows, 6 = the row -> column transpose alone.
extern "C" int ubench_part_bin(int ablate, const void *keys, size_t n, uint64_t m, uint32_t *pos,
                               uint32_t *run_starts, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const KeySpan ks{reinterpret_cast<const char *>(keys), n, 4, KEYS_PACKED};
    const ModParams mp = make_mod_params(m);
    PartitionWorkspace ws{};
    if (!plan_segments(m, device_cu_count(), &ws)) return -34;
    const int nbins = (int)ws.nbins;
    const size_t ntiles = (n + kPartTileKeys - 1) / kPartTileKeys;
    const unsigned grid = part_bin_grid(ntiles);
    const int nsub = (int)ws.nsub, ssh = (int)ws.sub_shift, grp = (int)ws.group;
    // run_starts holds both layouts: segment-major first, the pass-1 rows after
    ws.ntiles = ntiles;
    ws.run_starts = run_starts;
    ws.run_rows = run_starts + ntiles * (ws.nbins + 1);
    uint32_t *rows = ws.run_rows;
    switch (ablate) {
        case 0:
            ws.pos = pos;
            if (launch_part_bin(ks, mp, ws, s) != hipSuccess) return -5;
            break;
        case 1: k_part_bin<KEYS_PACKED, 1><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, rows, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 2: k_part_bin<KEYS_PACKED, 2><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, rows, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 3: k_part_bin<KEYS_PACKED, 3><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, rows, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 4: k_part_bin<KEYS_PACKED, 0, false, true><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, run_starts, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 5: k_part_bin<KEYS_PACKED, 0, false, false><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, rows, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 6: if (launch_runs_transpose(ws, s) != hipSuccess) return -5; break;
        case 7:  // pass 1 (columns) with one workgroup per CU, leaving LDS for a concurrent pass 2
            k_part_bin<KEYS_PACKED, 0, false, true><<<(unsigned)device_cu_count(), kPartBlock, 0, s>>>(ks, mp, pos, run_starts, nbins, nsub, ssh, grp, ntiles, nullptr);
            break;
        // 8..10: the product's pass 1 with the second half of the grid
        // started 1..3 x 8K cycles late (do the two workgroups of a CU run
        // their VALU and LDS phases in step?)
        case 8: k_part_bin<KEYS_PACKED, 0, false, true, kPartBlock, 1><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, run_starts, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 9: k_part_bin<KEYS_PACKED, 0, false, true, kPartBlock, 2><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, run_starts, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        case 10: k_part_bin<KEYS_PACKED, 0, false, true, kPartBlock, 3><<<grid, kPartBlock, 0, s>>>(ks, mp, pos, run_starts, nbins, nsub, ssh, grp, ntiles, nullptr); break;
        default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Pass 2 of the partition build on the positions of ubench_part_bin ablate 0:
// variant G in {2..64} = the product walk with G lanes per tile, 100 + G =
// the same with the LDS ORs skipped (loads only), 0 = the product's choice.
extern "C" int ubench_part_apply(int variant, const uint32_t *pos, const uint32_t *run_starts,
                                 size_t n, uint64_t m, uint32_t *words, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    PartitionWorkspace ws{};
    if (!plan_segments(m, device_cu_count(), &ws)) return -34;
    const int nbins = (int)ws.nbins;
    const int ntiles = (int)((n + kPartTileKeys - 1) / kPartTileKeys);
    const uint64_t nw32 = ((m + 63) / 64) * 2;
    const uint32_t sb = ws.seg_bits;
    if (variant == 0) variant = apply_lanes_per_tile(ws.nbins);
#define UB_APPLY(G, A) UB_APPLYD(G, A, kApplyDepth)
#define UB_APPLYD(G, A, D)                                                                    \
    do {                                                                                      \
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_part_apply<kApplyBuild, G, A, kApplyBlock, D>), \
                                  hipFuncAttributeMaxDynamicSharedMemorySize,                 \
                                  (int)(kSegMaxBits / 8));                                    \
        k_part_apply<kApplyBuild, G, A, kApplyBlock, D><<<nbins, kApplyBlock, sb / 8, s>>>(         \
            pos, run_starts, ntiles, nbins, sb, m, words, nw32, 0, nullptr, StackTable{});    \
    } while (0)
    switch (variant) {
        case 2: UB_APPLY(2, 0); break;
        case 4: UB_APPLY(4, 0); break;
        case 8: UB_APPLY(8, 0); break;
        case 16: UB_APPLY(16, 0); break;
        case 32: UB_APPLY(32, 0); break;
        case 64: UB_APPLY(64, 0); break;
        case 402: UB_APPLYD(2, 0, 2); break;   // 400 + G: depth 2, 500 + G: depth 1
        case 404: UB_APPLYD(4, 0, 2); break;
        case 408: UB_APPLYD(8, 0, 2); break;
        case 416: UB_APPLYD(16, 0, 2); break;
        case 502: UB_APPLYD(2, 0, 1); break;
        case 504: UB_APPLYD(4, 0, 1); break;
        case 508: UB_APPLYD(8, 0, 1); break;
        case 516: UB_APPLYD(16, 0, 1); break;
        case 102: UB_APPLY(2, 1); break;
        case 104: UB_APPLY(4, 1); break;
        case 108: UB_APPLY(8, 1); break;
        case 116: UB_APPLY(16, 1); break;
        case 132: UB_APPLY(32, 1); break;
        default: return -22;
    }
#undef UB_APPLY
#undef UB_APPLYD
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The stacked probe (C3 by default) by phase: 0 = the product's three
// launches, 1 = pass 1 (with slots), 2 = pass 2 alone (G from
// apply_lanes_per_tile), 3 = pass 2 without its result stores, 4 = pass 2
// reading only member 0's image, 5 = the combine; 100 + G = pass 2 with G
// lanes per tile.  Buffers sized by the caller for plan_stack's geometry
// (ubench_stack_geometry; runs: both layouts).  Members must divide the
// largest, so their gcd is the smallest.
namespace {
bool ub_stack_plan(int nf, const uint64_t *ms, uint64_t *mmax, PartitionWorkspace *ws) {
    uint64_t g = 0;
    *mmax = 0;
    for (int j = 0; j < nf; j++) {
        *mmax = ms[j] > *mmax ? ms[j] : *mmax;
        g = g == 0 || ms[j] < g ? ms[j] : g;
    }
    return plan_stack(*mmax, g, g, nf, device_cu_count(), ws);
}
}  // namespace

extern "C" int ubench_stack_geometry(int nf, const uint64_t *ms, uint64_t *nbins_out,
                                     uint64_t *seg_bits_out) {
    uint64_t mmax = 0;
    PartitionWorkspace ws{};
    if (!ub_stack_plan(nf, ms, &mmax, &ws)) return -34;
    *nbins_out = ws.nbins;
    *seg_bits_out = ws.seg_bits;
    return 0;
}

extern "C" int ubench_stack(int variant, const void *keys, size_t n, int nf, const uint64_t *ms,
                            void *const *words, uint32_t *pos, uint32_t *runs, uint8_t *res,
                            uint16_t *slots, uint64_t *out, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const KeySpan ks{reinterpret_cast<const char *>(keys), n, 4, KEYS_PACKED};
    uint64_t mmax = 0;
    PartitionWorkspace ws{};
    if (!ub_stack_plan(nf, ms, &mmax, &ws)) return -34;
    ws.tile_keys = choose_tile_keys(ws.nbins);
    ws.ntiles = (n + ws.tile_keys - 1) / ws.tile_keys;
    ws.pos = pos;
    ws.run_rows = runs;
    ws.run_starts = runs + ws.ntiles * (ws.nbins + 1);
    StackTable st{};
    st.nf = nf;
    for (int j = 0; j < nf; j++) {
        st.words[j] = reinterpret_cast<const uint32_t *>(words[j]);
        st.mwords[j] = (uint32_t)(ms[j] / 32);
        st.row[j] = j;
    }
    const ModParams mp = make_mod_params(mmax);
    const size_t nw = (n + 63) / 64;
    const size_t lds = (size_t)ws.seg_bits / 8 * nf;
#define UB_STACK(G, A, T) UB_STACKB(G, A, T, kApplyBlock)
#define UB_STACKT(G, A, T, B, TP)                                                                  \
    do {                                                                                           \
        (void)hipFuncSetAttribute(                                                                 \
            reinterpret_cast<const void *>(&k_part_apply<kApplyStack, G, A, B, kApplyDepth, TP>),  \
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kStackMaxBits / 8));                 \
        k_part_apply<kApplyStack, G, A, B, kApplyDepth, TP><<<(unsigned)ws.nbins, B, lds, s>>>(    \
            ws.pos, ws.run_starts, (int)ws.ntiles, (int)ws.nbins, ws.seg_bits, mmax, nullptr, 0,   \
            0, res, T);                                                                            \
    } while (0)
#define UB_STACKD(G, D)                                                                            \
    do {                                                                                           \
        if (ws.tile_keys == 2 * kPartTileKeys) {                                                   \
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(                              \
                &k_part_apply<kApplyStack, G, 0, kApplyBlock, D, 2 * kPartTilePos>),               \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kStackMaxBits / 8));             \
            k_part_apply<kApplyStack, G, 0, kApplyBlock, D, 2 * kPartTilePos>                      \
                <<<(unsigned)ws.nbins, kApplyBlock, lds, s>>>(ws.pos, ws.run_starts,               \
                (int)ws.ntiles, (int)ws.nbins, ws.seg_bits, mmax, nullptr, 0, 0, res, st);         \
        } else {                                                                                   \
            return -22;                                                                            \
        }                                                                                          \
    } while (0)
#define UB_STACKB(G, A, T, B)                                                                      \
    do {                                                                                           \
        if (ws.tile_keys == 2 * kPartTileKeys) UB_STACKT(G, A, T, B, 2 * kPartTilePos);            \
        else UB_STACKT(G, A, T, B, kPartTilePos);                                                  \
    } while (0)
    const int G = apply_lanes_per_tile(ws.nbins, 3 * tile_keys_of(ws));
    StackTable one = st;
    one.nf = 1;
    switch (variant) {
        case 0: return launch_probe_stacked(ks, mp, st, ws, res, slots, out, nw, s) == hipSuccess ? 0 : -5;
        case 1: return launch_bin<true>(ks, mp, ws, slots, s) == hipSuccess ? 0 : -5;
        case 2: return launch_apply<kApplyStack>(ws, mmax, nullptr, 0, 0, res, st, s) == hipSuccess ? 0 : -5;
        case 3:
            if (G == 4) UB_STACK(4, 2, st); else if (G == 8) UB_STACK(8, 2, st); else return -22;
            break;
        case 4:
            if (G == 4) UB_STACK(4, 0, one); else if (G == 8) UB_STACK(8, 0, one); else return -22;
            break;
        case 5:
            return launch_combine(ws, res, slots, n, out, nw, st, s) == hipSuccess ? 0 : -5;
            break;
        case 6:
            if (G == 4) UB_STACK(4, 3, st); else if (G == 8) UB_STACK(8, 3, st); else return -22;
            break;
        case 8:
            if (G == 4) UB_STACKB(4, 0, st, 512); else if (G == 8) UB_STACKB(8, 0, st, 512); else return -22;
            break;
        case 10:
            if (G == 4) UB_STACKB(4, 2, st, 512); else if (G == 8) UB_STACKB(8, 2, st, 512); else return -22;
            break;
        case 11:  // image staging only
            if (G == 8) UB_STACK(8, 4, st); else return -22;
            break;
        case 201: UB_STACKD(8, 1); break;
        case 203: UB_STACKD(8, 3); break;
        case 204: UB_STACKD(8, 4); break;
        case 102: UB_STACK(2, 0, st); break;
        case 104: UB_STACK(4, 0, st); break;
        case 108: UB_STACK(8, 0, st); break;
        case 116: UB_STACK(16, 0, st); break;
        default: return -22;
    }
#undef UB_STACK
#undef UB_STACKB
#undef UB_STACKT
#undef UB_STACKD
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
