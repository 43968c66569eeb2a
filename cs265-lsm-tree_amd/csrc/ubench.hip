// ubench.hip — micro-benchmarks that price the primitives the Bloom kernels
// are built from on gfx950: random 4-B global atomicOr (agent vs workgroup
// scope), random 4-B gathers, random LDS ds_or, and the exact hash+mod
// arithmetic alone.  Not part of the product path; used by
// tools/ubench.py to pick build strategies.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <numeric>

#include "bloom_device.h"  // the product kernels and launch templates, for ablation builds
#include "bloom_merge.h"

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

// Random ds_or with half the lanes idle in five ways (round 6: what pass 2's
// out-of-run entries cost the LDS): 0 every lane a random word; 1 odd lanes
// OR 0 into one word shared by the group; 2 odd lanes masked off; 3 odd lanes
// OR 0 into a private word each; 4 odd lanes OR 0 into a random word (pass
// 2's branch-free masking).
template <int MODE>
__global__ void __launch_bounds__(1024) ub_lds_or_idle(int iters, uint32_t *sink) {
    extern __shared__ uint32_t seg[];
    for (int i = threadIdx.x; i < 16384 + 64; i += blockDim.x) seg[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const bool idle = MODE != 0 && (lane & 1);
    uint32_t s = 0x9E3779B9u ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    for (int i = 0; i < iters; i++) {
        const uint32_t r = xorshift(s);
        uint32_t w = r >> 18, v = 1u << (r & 31);
        if (idle) {
            v = 0;
            if constexpr (MODE == 1) w = 16384;
            if constexpr (MODE == 3) w = 16384 + lane;
        }
        if constexpr (MODE == 2) {
            if (!idle) atomicOr(&seg[w], v);
        } else {
            atomicOr(&seg[w], v);
        }
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

// hash3 + the p2 remainder (m = d << t, d | 255: bloom_math.h mod_p2), the
// remainder the C2-C5 filters take
__global__ void ub_hash_p2(ModParams mp, int iters, uint32_t *sink) {
    uint32_t acc = 0;
    int32_t k = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    for (int i = 0; i < iters; i++) {
        acc ^= mod_p2(raw_hash1(k), mp) + mod_p2(raw_hash2(k), mp) + mod_p2(raw_hash3(k), mp);
        k += 0x9E3779B9;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Pass 1's whole per-key arithmetic, without its loads, sort or stores: the
// three hashes and, per hash, the bin and entry exactly as k_part_bin forms
// them (bin_entry with the product's reduction MK and segment map for the
// batch's geometry): the VALU ceiling of a build's or probe's pass 1.
template <int MK>
__global__ void ub_pass1_arith(ModParams mp, SegMap sm, int iters, uint32_t *sink) {
    uint32_t acc = 0;
    int32_t k = (int32_t)((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    for (int i = 0; i < iters; i++) {
        uint32_t b0, e0, b1, e1, b2, e2;
        bin_entry<MK, 4>(raw_hash1(k), mp, sm, b0, e0);
        bin_entry<MK, 4>(raw_hash2(k), mp, sm, b1, e1);
        bin_entry<MK, 4>(raw_hash3(k), mp, sm, b2, e2);
        acc ^= (b0 + e0) ^ (b1 + e1) ^ (b2 + e2);
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
        case 7: {
            const ModParams mp = make_mod_params(m);
            if (!mp.p2) return -22;
            ub_hash_p2<<<grid, block, 0, s>>>(mp, iters, sink);
            break;
        }
        case 6: ub_stream<<<grid, block, 0, s>>>(reinterpret_cast<const uint4 *>(dbuf), bytes / 16 - 1, sink); break;
        case 40: ub_lds_or_idle<0><<<grid, 1024, 66 * 1024, s>>>(iters, sink); break;
        case 41: ub_lds_or_idle<1><<<grid, 1024, 66 * 1024, s>>>(iters, sink); break;
        case 42: ub_lds_or_idle<2><<<grid, 1024, 66 * 1024, s>>>(iters, sink); break;
        case 43: ub_lds_or_idle<3><<<grid, 1024, 66 * 1024, s>>>(iters, sink); break;
        case 44: ub_lds_or_idle<4><<<grid, 1024, 66 * 1024, s>>>(iters, sink); break;
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

// Pass 1's per-key arithmetic (ub_pass1_arith) for the product's geometry:
// a build of a filter of ms[0] bits (nf = 1, plan_build), or a stacked probe
// of nf members (plan_ladder, else plan_stack).  *mk_out: the reduction kind.
extern "C" int ubench_pass1_arith(int nf, const uint64_t *ms, int grid, int block, int iters,
                                  void *dbuf, void *stream, int *mk_out) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t *sink = reinterpret_cast<uint32_t *>(dbuf);
    PartitionWorkspace ws{};
    StackTable st{};
    uint64_t mmax = 0, g = 0, mmin = ~0ull;
    for (int j = 0; j < nf; j++) {
        mmax = std::max(mmax, ms[j]);
        mmin = std::min(mmin, ms[j]);
        g = g == 0 ? ms[j] : std::gcd(g, ms[j]);
    }
    const int ncu = device_cu_count();
    if (nf == 1) {
        if (!plan_build(mmax, ncu, &ws)) return -34;
    } else if (!plan_ladder(ms, nf, ncu, &st, &ws) && !plan_stack(mmax, g, mmin, nf, ncu, &ws)) {
        return -34;
    }
    const ModParams mp = make_mod_params(mmax);
    SegMap sm{};
    const int mk = pass1_plan(mp, ws, nf > 1, &sm);
    *mk_out = mk;
    switch (mk) {
        case kModFast: ub_pass1_arith<kModFast><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        case kModWide: ub_pass1_arith<kModWide><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        case kModP2: ub_pass1_arith<kModP2><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        case kModLadder: ub_pass1_arith<kModLadder><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        case kModLadder0: ub_pass1_arith<kModLadder0><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        case kModLadder0R: ub_pass1_arith<kModLadder0R><<<grid, block, 0, s>>>(mp, sm, iters, sink); break;
        default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Geometry of the product's partition build of n keys into m bits
// (tools/ubench.py sizes its buffers from it): segments, segment bits, tile
// keys and tiles.
// out4: segments, segment bits, tile keys, tiles.
// out4: the larger of plan_build's and plan_segments' segment counts, the
// product's segment bits, the smallest tile of the two plans and the tiles
// at that size: buffers sized from these hold every variant of ubench_part.
extern "C" int ubench_part_geometry(size_t n, uint64_t m, uint64_t *out4) {
    PartitionWorkspace ws{}, sg{};
    if (!plan_build(m, device_cu_count(), &ws) || !plan_segments(m, device_cu_count(), &sg)) return -34;
    const size_t tk = std::min<size_t>(ws.tile_keys ? ws.tile_keys : choose_tile_keys(ws.nbins),
                                       choose_tile_keys(sg.nbins));
    out4[0] = std::max(ws.nbins, sg.nbins);
    out4[1] = ws.seg_bits;
    out4[2] = tk;
    out4[3] = (n + tk - 1) / tk;
    return 0;
}

// Phases of the product's partition build (tools/ubench.py part, p1ab):
// 0 = pass 1 as the product launches it, 1 = pass 2 as the product launches
// it over variant 0's output; 5001 / 5003 = pass-1 shapes (MINW waves per
// SIMD, NWG workgroups per CU).  runs: both table layouts.
extern "C" int ubench_part(int variant, const void *keys, size_t n, uint64_t m, uint64_t *pos,
                           uint32_t *runs, uint32_t *words, void *stream, size_t pos_cap,
                           size_t runs_cap) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const KeySpan ks{reinterpret_cast<const char *>(keys), n, 4, KEYS_PACKED};
    const ModParams mp = make_mod_params(m);
    PartitionWorkspace ws{};
    // 20 / 21: pass 1 / pass 2 on plan_segments' segments (the round-2
    // geometry); everything else on the product's plan_build
    const bool seg = variant == 20 || variant == 21;
    if (!(seg ? plan_segments(m, device_cu_count(), &ws) : plan_build(m, device_cu_count(), &ws)))
        return -34;
    if (!ws.tile_keys) ws.tile_keys = choose_tile_keys(ws.nbins);  // plan_build's super-tiles kept
    ws.ntiles = (n + ws.tile_keys - 1) / ws.tile_keys;
    // the caller's buffers must hold this plan's tiles (pos, in u64) and
    // both run-table layouts (runs, in u32): refused, not overrun
    if (ws.ntiles * ws.tile_keys > pos_cap || 2 * ws.ntiles * (ws.nbins + 1) > runs_cap) return -28;
    ws.pos = pos;
    ws.run_rows = runs;
    ws.run_starts = runs + ws.ntiles * (ws.nbins + 1);
    hipError_t e = hipSuccess;
    switch (variant) {
        case 0: case 20: e = launch_part_bin(ks, mp, ws, s); break;
        case 1: case 21: e = launch_part_apply(mp, words, ws, 0, s); break;
        // pass-1 shapes with the p2 remainder (MINW, NWG)
#define UB_P2(V, TB, MAXB, MINW, NWG)                                                             \
    case V: {                                                                                    \
        if (ws.nbins > MAXB || ws.tile_keys != TB * kPartKPT || !mp.p2) return -22;             \
        SegMap sm = seg_map_of(ws);                                                              \
        sm.p2_hi_shift = mp.p2t - sm.shift;                                                      \
        const unsigned g = (unsigned)std::min<size_t>(ws.ntiles, (size_t)device_cu_count() * NWG); \
        k_part_bin<KEYS_PACKED, false, true, TB, kModP2, MAXB, MINW>                             \
            <<<g, TB, 0, s>>>(ks, mp, ws.pos, ws.run_starts, sm, ws.ntiles, nullptr);            \
        e = hipGetLastError();                                                                   \
        break;                                                                                   \
    }
        UB_P2(5001, 512, 511, 4, 2) UB_P2(5003, 512, 511, 6, 3)
#undef UB_P2
        // 2500 / 2503: pass 2 of a super-tile build (C4) on the round-6
        // walk with two vectors per lane (WALK 5) / the product's WALK 3
        case 2500: case 2503: case 2523: case 2522: case 2507: case 2508: case 2509: case 2511: {
            // 2523 / 2522: WALK 3 at G = 2 lanes per tile (24 entries a step
            // for C4's ~20-entry runs) / WALK 2 (one vector) at G = 4
            if (ws.lad_u || tile_keys_of(ws) != kSuperTileKeys) return -22;
            const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
            constexpr int TK = (int)kSuperTileKeys;
            if (variant == 2500)
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 5>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2503)
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 3>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2507)
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 7>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2508)
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 8>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2509)
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 9>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2523)
                e = launch_apply_g<kApplyBuild, 2, TK, 1, 3>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else if (variant == 2511)  // two chains of one redirected vector per lane
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 11>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            else
                e = launch_apply_g<kApplyBuild, 4, TK, 1, 2>(ws, mp.m, words, nw32, 0, nullptr, StackTable{}, s);
            break;
        }
        // 2400 / 2401: pass 2 of plan_build's one-member ladder (C2, C5) on
        // the round-6 build walk (WALK 4) / the product's WALK 1, over
        // variant 0's output
        case 2400: case 2401: case 2410: case 2413: case 2417: {
            if (!ws.lad_u || ws.lad_hb != 0 || !mp.p2) return -22;
            StackTable st{};
            st.lad.s = ws.lad_s;
            st.lad.u = ws.lad_u;
            st.lad.d = mp.p2d;
            st.lad.t[0] = mp.p2t;
            st.lad.rinv = ladder0_relabel(mp, ws) ? ladder0_inv(mp) : 0u;
            const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
            const size_t tk = tile_keys_of(ws);
            if (tk == 4096)
                e = variant == 2400 ? launch_apply_g<kApplyBuildL, 4, 4096, 1, 4>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2410 ? launch_apply_g<kApplyBuildL, 4, 4096, 1, 10>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2413 ? launch_apply_g<kApplyBuildL, 4, 4096, 1, 3>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2417 ? launch_apply_g<kApplyBuildL, 4, 4096, 1, 7>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                                    : launch_apply_g<kApplyBuildL, 4, 4096, 1, 1>(ws, mp.m, words, nw32, 0, nullptr, st, s);
            else if (tk == 8192)
                e = variant == 2400 ? launch_apply_g<kApplyBuildL, 4, 8192, 1, 4>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2410 ? launch_apply_g<kApplyBuildL, 4, 8192, 1, 10>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2413 ? launch_apply_g<kApplyBuildL, 4, 8192, 1, 3>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                  : variant == 2417 ? launch_apply_g<kApplyBuildL, 4, 8192, 1, 7>(ws, mp.m, words, nw32, 0, nullptr, st, s)
                                    : launch_apply_g<kApplyBuildL, 4, 8192, 1, 1>(ws, mp.m, words, nw32, 0, nullptr, st, s);
            else
                return -22;
            break;
        }
        // 5100 + ABL: the product's C2 pass 1 (plan_build's one-member
        // ladder, 4096-key tiles, three workgroups per CU) cut after a
        // stage (k_part_bin's ABL): the ablation ladder of tools/ubench.py p1abl
#define UB_ABL(A)                                                                                 \
    case 5100 + A: {                                                                             \
        SegMap sm{};                                                                             \
        if (pass1_plan(mp, ws, false, &sm) != kModLadder0R || ws.tile_keys != 4096 ||           \
            ws.nbins > 511 || !runs_as_columns(ws))                                              \
            return -22;                                                                          \
        const unsigned g = (unsigned)std::min<size_t>(ws.ntiles, (size_t)device_cu_count() * 3); \
        k_part_bin<KEYS_PACKED, false, true, 512, kModLadder0R, 511, 6, A>                       \
            <<<g, 512, 0, s>>>(ks, mp, ws.pos, ws.run_starts, sm, ws.ntiles, nullptr);           \
        e = hipGetLastError();                                                                   \
        break;                                                                                   \
    }
        UB_ABL(0) UB_ABL(1) UB_ABL(2) UB_ABL(3) UB_ABL(4) UB_ABL(5)
#undef UB_ABL
        default: return -22;
    }
    return e == hipSuccess ? 0 : -5;
}

// The stacked probe (C3 by default) by phase: 0 = the product's three
// launches, 1 = pass 1 (with slots), 2 = pass 2, 5 = the combine; 100 + G =
// pass 2 with G lanes per tile.  Buffers sized by the caller for plan_stack's
// geometry (ubench_stack_geometry; runs: both layouts).  Members must divide
// the largest, so their gcd is the smallest.
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
                            void *const *words, uint64_t *pos, uint32_t *runs, uint8_t *res,
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
    hipError_t e = hipSuccess;
    switch (variant) {
        case 0: e = launch_probe_stacked(ks, mp, st, ws, res, slots, out, nw, s); break;
        case 1: e = launch_bin<true>(ks, mp, ws, slots, s); break;
        case 2: e = launch_apply_stack(ws, mmax, res, st, s); break;
        case 5: e = launch_combine(ws, res, slots, n, out, nw, st, s); break;
        default: return -22;
    }
    return e == hipSuccess ? 0 : -5;
}

// Ladder stack (plan_ladder) on the product kernels, tile_keys 4096 or 8192:
// 0 the whole probe, 1 pass 1, 2 pass 2 (product walk), 5 combine,
// 20 + G pass 2 at G lanes per tile (independent groups), 30 + G batch walk,
// 41 / 44 batch walk G = 8 at one / four load groups per wave.
extern "C" int ubench_ladder(int variant, int tile_keys, const void *keys, size_t n, int nf,
                             const uint64_t *ms, void *const *words, uint64_t *pos,
                             uint32_t *runs, uint8_t *res, uint16_t *slots, uint64_t *out,
                             void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const KeySpan ks{reinterpret_cast<const char *>(keys), n, 4, KEYS_PACKED};
    PartitionWorkspace ws{};
    StackTable st{};
    // variants >= 100: the same phase (variant - 100) on the table planner
    // (no computed tuple, LadderTable::ctup = 0), for A/B
    const bool table = variant >= 100 && variant < 200;
    if (table) variant -= 100;
    if (!plan_ladder(ms, nf, device_cu_count(), &st, &ws, !table)) return -34;
    if (tile_keys) ws.tile_keys = (uint32_t)tile_keys;
    ws.ntiles = (n + ws.tile_keys - 1) / ws.tile_keys;
    ws.pos = pos;
    ws.run_rows = runs;
    ws.run_starts = runs + ws.ntiles * (ws.nbins + 1);
    st.nf = nf;
    for (int j = 0; j < nf; j++) {
        st.words[j] = reinterpret_cast<const uint32_t *>(words[j]);
        st.mwords[j] = (uint32_t)(ms[j] / 32);
        st.row[j] = j;
    }
    const ModParams mp = make_mod_params(ms[0]);
    const size_t nw = (n + 63) / 64;
    hipError_t e = hipSuccess;
    switch (variant) {
        case 0: e = launch_probe_stacked(ks, mp, st, ws, res, slots, out, nw, s); break;
        case 1: e = launch_bin<true>(ks, mp, ws, slots, s); break;
        case 2: e = launch_apply_ladder(ws, ms[0], res, st, s); break;
        case 5: e = launch_combine(ws, res, slots, n, out, nw, st, s); break;
        case 11: case 12: {
            // pass 1 of the product's geometry WITHOUT the slot stores (11:
            // the sorted tile and runs as the product writes them; 12: also
            // no sorted-tile stores): what the slot plane and the tile's
            // write-out cost C3's pass 1
            SegMap sm{};
            if (pass1_plan(mp, ws, true, &sm) != kModLadder || ws.tile_keys != 8192) return -22;
            const bool cols = runs_as_columns(ws);
            uint32_t *rt = cols ? ws.run_starts : ws.run_rows;
            const unsigned g = (unsigned)std::min<size_t>(ws.ntiles, (size_t)device_cu_count());
            if (variant == 11) {
                if (cols) k_part_bin<KEYS_PACKED, false, true, 1024, kModLadder, 1023, 4><<<g, 1024, 0, s>>>(ks, mp, ws.pos, rt, sm, ws.ntiles, nullptr);
                else k_part_bin<KEYS_PACKED, false, false, 1024, kModLadder, 1023, 4><<<g, 1024, 0, s>>>(ks, mp, ws.pos, rt, sm, ws.ntiles, nullptr);
            } else {
                if (cols) k_part_bin<KEYS_PACKED, false, true, 1024, kModLadder, 1023, 4, 5><<<g, 1024, 0, s>>>(ks, mp, ws.pos, rt, sm, ws.ntiles, nullptr);
                else k_part_bin<KEYS_PACKED, false, false, 1024, kModLadder, 1023, 4, 5><<<g, 1024, 0, s>>>(ks, mp, ws.pos, rt, sm, ws.ntiles, nullptr);
            }
            e = hipGetLastError();
            if (e == hipSuccess && !cols) e = launch_runs_transpose(ws, s);
            break;
        }
        default: return -22;
    }
    return e == hipSuccess ? 0 : -5;
}

extern "C" int ubench_ladder_geometry(int nf, const uint64_t *ms, uint64_t *out6) {
    PartitionWorkspace ws{};
    StackTable st{};
    if (!plan_ladder(ms, nf, device_cu_count(), &st, &ws)) return -34;
    out6[0] = ws.nbins;
    out6[1] = st.lad.s;
    out6[2] = st.lad.hb;
    out6[3] = ladder_lds_bytes(st.lad);
    out6[4] = st.lad.k;
    out6[5] = st.lad.bpp;
    return 0;
}

// ---- rocprofv3 counter calibration (tools/ubench.py cal) --------------------
// Kernels that request a known number of bytes in the access shapes the
// product issues, so FETCH_SIZE / WRITE_SIZE can be read against them
// (MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced reads).
// Reads (each requested byte once):
//   0  coalesced 16-B vectors, a wave's 64 vectors contiguous (1 KiB)
//   1  the first 64 B of every 128-B line, coalesced over lines
//   2  one 16-B vector of every 128-B line
//   3  pass 2's walk: the buffer as tiles x nseg runs of R vectors; block b
//      reads segment b's run of every tile, 4 lanes per run (lane i the
//      run's vectors i, i + 4, ...), each group of 4 its own tiles
// Writes (each byte once):
//   10 coalesced 16-B vector stores
//   11 2-byte stores, three per lane at 6i, 6i + 2, 6i + 4 (the probe's
//      result bytes along sorted runs)
//   12 one 4-B store per 128-B line, column-major into a row-major table
//      (pass 1's segment-major run-table columns)
__global__ void __launch_bounds__(1024) ub_cal(uint4 *buf, size_t nv, int shape, int R, int nseg,
                                               uint32_t *sink) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nth = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    if (shape == 0) {
        for (size_t i = tid; i < nv; i += nth) {
            const uint4 v = buf[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    } else if (shape == 1) {
        for (size_t i = tid; i < nv / 2; i += nth) {  // vector i of the half lines
            const uint4 v = buf[(i / 4) * 8 + (i % 4)];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    } else if (shape == 2) {
        for (size_t i = tid; i < nv / 8; i += nth) {
            const uint4 v = buf[i * 8];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    } else if (shape == 3) {
        const size_t ntiles = nv / ((size_t)nseg * R);
        const int g = threadIdx.x / 4, gl = threadIdx.x % 4, ng = blockDim.x / 4;
        for (int b = blockIdx.x; b < nseg; b += gridDim.x)
            for (size_t t = g; t < ntiles; t += ng) {
                const uint4 *run = buf + (t * nseg + b) * R;
                for (int i = gl; i < R; i += 4) {
                    const uint4 v = run[i];
                    acc ^= v.x ^ v.y ^ v.z ^ v.w;
                }
            }
    } else if (shape == 10) {
        for (size_t i = tid; i < nv; i += nth) buf[i] = make_uint4((uint32_t)i, 1, 2, 3);
    } else if (shape == 11) {
        uint16_t *b16 = reinterpret_cast<uint16_t *>(buf);
        for (size_t i = tid; i < nv * 16 / 6; i += nth) {
            b16[3 * i] = (uint16_t)i;
            b16[3 * i + 1] = (uint16_t)(i >> 1);
            b16[3 * i + 2] = (uint16_t)(i >> 2);
        }
    } else if (shape == 12) {
        uint32_t *b32 = reinterpret_cast<uint32_t *>(buf);
        const size_t rows = nv * 4 / 32, cols = 32;  // 128-B rows of 32 words
        for (size_t i = tid; i < rows * cols; i += nth) b32[(i % rows) * cols + i / rows] = (uint32_t)i;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Bytes each calibration shape requests from a buffer of nv vectors.
extern "C" uint64_t ubench_cal_bytes(int shape, size_t nv, int R, int nseg) {
    switch (shape) {
        case 0: case 10: return (uint64_t)nv * 16;
        case 1: return (uint64_t)nv * 8;
        case 2: return (uint64_t)nv * 2;
        case 3: return (uint64_t)(nv / ((size_t)nseg * R)) * nseg * R * 16;
        case 11: return (uint64_t)(nv * 16 / 6) * 6;
        case 12: return (uint64_t)nv * 16;
        default: return 0;
    }
}

extern "C" int ubench_cal(int shape, void *buf, size_t nv, int R, int nseg, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t *sink = reinterpret_cast<uint32_t *>(buf);  // never written for these inputs
    const unsigned grid = shape == 3 ? (unsigned)nseg : (unsigned)(device_cu_count() * 2);
    ub_cal<<<grid, 1024, 0, s>>>(reinterpret_cast<uint4 *>(buf), nv, shape, R, nseg, sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The run-table transpose with a configurable column stride (>= ntiles):
// rows [ntiles][width] -> cols[b * cstride + tile].  VEC = 1: the product's
// 64 x 64 LDS tile, 4-B accesses; VEC = 4: rows read as 16-B vectors when
// width % 4 == 0.  (tools/ubench.py transpose: does the 64 KiB column stride
// of C4's 16,384 super-tiles cost the write side?)
namespace {
__global__ void __launch_bounds__(256) ub_transpose(const uint32_t *__restrict__ rows,
                                                    uint32_t *__restrict__ cols, size_t ntiles,
                                                    int width, size_t cstride) {
    __shared__ uint32_t t[64][65];
    const int b0 = blockIdx.x * 64;
    const size_t t0 = (size_t)blockIdx.y * 64;
    const int x = threadIdx.x & 63, y0 = threadIdx.x >> 6;
    for (int y = y0; y < 64; y += 4) {
        const size_t tile = t0 + y;
        if (tile < ntiles && b0 + x < width) t[y][x] = rows[tile * width + b0 + x];
    }
    __syncthreads();
    for (int y = y0; y < 64; y += 4) {
        const size_t tile = t0 + x;
        if (tile < ntiles && b0 + y < width) cols[(size_t)(b0 + y) * cstride + tile] = t[x][y];
    }
}
}  // namespace

// variant 2: every load of the tile issued before any LDS store (clamped
// addresses, no load under a branch), the stores likewise; TR tile rows.
template <int TR>
__global__ void __launch_bounds__(256) ub_transpose2(const uint32_t *__restrict__ rows,
                                                     uint32_t *__restrict__ cols, size_t ntiles,
                                                     int width, size_t cstride) {
    __shared__ uint32_t t[TR][65];
    constexpr int kPer = TR / 4;
    const int b0 = blockIdx.x * 64;
    const size_t t0 = (size_t)blockIdx.y * TR;
    const int x = threadIdx.x & 63, y0 = threadIdx.x >> 6;
    uint32_t v[kPer];
    const int bx = min(b0 + x, width - 1);
#pragma unroll
    for (int i = 0; i < kPer; i++) {
        const size_t tile = min(t0 + y0 + 4 * i, ntiles - 1);
        v[i] = rows[tile * width + bx];
    }
#pragma unroll
    for (int i = 0; i < kPer; i++) t[y0 + 4 * i][x] = v[i];
    __syncthreads();
    // writes: lane x takes tile t0 + x (+ 64 per half for TR = 128), row b0 + y
#pragma unroll
    for (int h = 0; h < TR / 64; h++) {
        const size_t tile = t0 + h * 64 + x;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int y = y0 + 4 * i;
            if (tile < ntiles && b0 + y < width) cols[(size_t)(b0 + y) * cstride + tile] = t[h * 64 + x][y];
        }
    }
}

extern "C" int ubench_transpose(const void *rows, void *cols, size_t ntiles, int width,
                                size_t cstride, void *stream) {
    if (cstride < ntiles) return -22;
    const dim3 grid((unsigned)((width + 63) / 64), (unsigned)((ntiles + 63) / 64));
    ub_transpose<<<grid, 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        reinterpret_cast<const uint32_t *>(rows), reinterpret_cast<uint32_t *>(cols), ntiles, width,
        cstride);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int ubench_transpose2(int tr, const void *rows, void *cols, size_t ntiles, int width,
                                 size_t cstride, void *stream) {
    if (cstride < ntiles || (tr != 64 && tr != 128)) return -22;
    const dim3 grid((unsigned)((width + 63) / 64), (unsigned)((ntiles + tr - 1) / tr));
    auto r = reinterpret_cast<const uint32_t *>(rows);
    auto c = reinterpret_cast<uint32_t *>(cols);
    auto s = reinterpret_cast<hipStream_t>(stream);
    if (tr == 64) ub_transpose2<64><<<grid, 256, 0, s>>>(r, c, ntiles, width, cstride);
    else ub_transpose2<128><<<grid, 256, 0, s>>>(r, c, ntiles, width, cstride);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
