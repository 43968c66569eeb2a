// bloom_probe.hip — the partitioned and stacked probes: pass 2 in probe and
// segment-stack modes, the combine, and the launch sequences (bloom_device.h).
#include "bloom_device.h"

namespace bloomhip {

// The combine for the batch's tile size (1024 threads: 42 us at C3 against
// 45 for 512 and 53 for 256).
hipError_t launch_combine(const PartitionWorkspace &ws, const uint8_t *res, const uint16_t *slots,
                          size_t n, uint64_t *out, size_t nw, const StackTable &rows,
                          hipStream_t stream) {
    constexpr int kBig = 2 * (int)kPartTileKeys, kSmall = (int)kPartTileKeys, kSuper = (int)kSuperTileKeys;
    if (tile_keys_of(ws) == kSuperTileKeys)  // super-tiles: two passes of 8 keys per thread
        k_probe_combine<kSuper, 1024><<<(unsigned)ws.ntiles, 1024, 0, stream>>>(res, slots, n, out, nw, rows);
    else if (tile_keys_of(ws) == 2 * kPartTileKeys)
        k_probe_combine<kBig, kBig / kCombineKeys>
            <<<(unsigned)ws.ntiles, kBig / kCombineKeys, 0, stream>>>(res, slots, n, out, nw, rows);
    else
        k_probe_combine<kSmall, kSmall / kCombineKeys>
            <<<(unsigned)ws.ntiles, kSmall / kCombineKeys, 0, stream>>>(res, slots, n, out, nw, rows);
    return hipGetLastError();
}

hipError_t launch_apply_stack(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                              const StackTable &st, hipStream_t stream) {
    return launch_apply<kApplyStack>(ws, m, nullptr, 0, 0, res, st, stream);
}

hipError_t launch_probe_partitioned(const KeySpan &ks, const ModParams &mp, const uint32_t *words,
                                    const PartitionWorkspace &ws, uint8_t *res, uint16_t *slots,
                                    uint64_t *out, hipStream_t stream) {
    if (ks.n == 0) return hipSuccess;
    hipError_t e = launch_bin<true>(ks, mp, ws, slots, stream);
    if (e != hipSuccess) return e;
    const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
    uint32_t *w = const_cast<uint32_t *>(words);  // read-only in PROBE mode
    e = launch_apply<kApplyProbe>(ws, mp.m, w, nw32, 0, res, StackTable{}, stream);
    if (e != hipSuccess) return e;
    StackTable rows{};
    rows.nf = 1;
    return launch_combine(ws, res, slots, ks.n, out, (ks.n + 63) / 64, rows, stream);
}

// The combine with GET routing fused in (k_probe_combine_route), when every
// run of the routing call is a member of this stack and the runs' fences fit
// in LDS; else hipErrorInvalidValue before anything is launched.
hipError_t launch_combine_route(const PartitionWorkspace &ws, const uint8_t *res,
                                const uint16_t *slots, const KeySpan &ks, uint64_t *out, size_t nw,
                                const StackTable &rows, const RouteTable &rt, const RouteOut &ro,
                                hipStream_t stream) {
    if (rt.nruns != rows.nf || (size_t)rt.total_fences * 4 > kRouteLdsFenceBytesMax) return hipErrorInvalidValue;
    if (ro.packed && rt.nruns > kRoutePackedMaxRuns) return hipErrorInvalidValue;
    unsigned seen = 0;
    for (int j = 0; j < rows.nf; j++) {
        if (rows.row[j] < 0 || rows.row[j] >= rows.nf) return hipErrorInvalidValue;
        seen |= 1u << rows.row[j];
    }
    if (seen != (1u << rows.nf) - 1u) return hipErrorInvalidValue;
    constexpr int kBig = 2 * (int)kPartTileKeys, kSmall = (int)kPartTileKeys;
    const size_t lds = (size_t)rt.total_fences * 4;
    // persistent workgroups, as many as are resident at once: two per CU
    // while two copies of the fences and the tile's result bytes fit the
    // LDS, else one (a second round of workgroups would start only when the
    // first has walked all of its tiles)
    const size_t per_wg = combine_route_lds_bytes(rt.total_fences, tile_keys_of(ws));
    const size_t cap = (size_t)device_cu_count() * (2 * per_wg <= kLdsBitmapBytes ? 2 : 1);
    const unsigned grid = (unsigned)(ws.ntiles < cap ? ws.ntiles : cap);
#define COMBINE_ROUTE(TK, L)                                                                      \
    k_probe_combine_route<TK, TK / kCombineKeys, L><<<grid, TK / kCombineKeys, lds, stream>>>(    \
        res, slots, ks, out, nw, rows, rt, ro.first, ro.page, ro.packed, ws.ntiles)
    const bool big = tile_keys_of(ws) == 2 * kPartTileKeys, super = tile_keys_of(ws) == kSuperTileKeys;
    constexpr int kSuper = (int)kSuperTileKeys;
#define COMBINE_ROUTE_SUPER(L)                                                                    \
    k_probe_combine_route<kSuper, 1024, L><<<grid, 1024, lds, stream>>>(                          \
        res, slots, ks, out, nw, rows, rt, ro.first, ro.page, ro.packed, ws.ntiles)
    if (ks.layout == KEYS_PACKED) {
        if (super) COMBINE_ROUTE_SUPER(KEYS_PACKED);
        else if (big) COMBINE_ROUTE(kBig, KEYS_PACKED); else COMBINE_ROUTE(kSmall, KEYS_PACKED);
    } else {
        if (super) COMBINE_ROUTE_SUPER(KEYS_STRIDED);
        else if (big) COMBINE_ROUTE(kBig, KEYS_STRIDED); else COMBINE_ROUTE(kSmall, KEYS_STRIDED);
    }
#undef COMBINE_ROUTE_SUPER
#undef COMBINE_ROUTE
    return hipGetLastError();
}

hipError_t launch_probe_stacked(const KeySpan &ks, const ModParams &mp_max, const StackTable &st,
                                const PartitionWorkspace &ws, uint8_t *res, uint16_t *slots,
                                uint64_t *out, size_t nw, hipStream_t stream, const RouteTable *rt,
                                const RouteOut &ro) {
    if (ks.n == 0) return hipSuccess;
    if (rt && (rt->nruns != st.nf || (size_t)rt->total_fences * 4 > kRouteLdsFenceBytesMax))
        return hipErrorInvalidValue;
    auto combine = [&]() {
        return rt ? launch_combine_route(ws, res, slots, ks, out, nw, st, *rt, ro, stream)
                  : launch_combine(ws, res, slots, ks.n, out, nw, st, stream);
    };
    if (st.ladder) {  // plan_ladder's geometry
        const LadderTable &L = st.lad;
        if (st.nf < 2 || st.nf > kMaxStack || !mp_max.fast || !mp_max.p2 || !ws.lad_u ||
            ws.lad_s != L.s || ws.lad_u != L.u || ws.lad_hb != L.hb || ws.nbins != (1u << L.u) ||
            L.t[0] != mp_max.p2t || L.d != mp_max.p2d || L.s < 7 ||
            ladder_lds_bytes(L) > kStackMaxBits / 8)
            return hipErrorInvalidValue;
        if (L.k < 1 || L.k > (uint32_t)st.nf || (L.k < (uint32_t)st.nf) != (L.bpp != 0) ||
            (L.bpp != 0 && L.bpp != 4 && L.bpp != 8) || (L.bpp == 4 && st.nf - (int)L.k > 4))
            return hipErrorInvalidValue;
        for (int j = 0; j < st.nf; j++)
            if ((uint64_t)st.mwords[j] * 32 != ((uint64_t)L.d << L.t[j]) || L.t[j] < L.s)
                return hipErrorInvalidValue;
        if (L.ctup ? (L.k != 1 || L.rs != 0 || L.tmagic == 0 || L.t[1] < L.s + L.u)
                   : (L.rs != 1 && L.rs != 2 && L.rs != 4 && L.rs != 8))
            return hipErrorInvalidValue;
        if (L.base[0] != 0) return hipErrorInvalidValue;
        hipError_t e = launch_bin<true>(ks, mp_max, ws, slots, stream);
        if (e != hipSuccess) return e;
        e = launch_apply_ladder(ws, mp_max.m, res, st, stream);
        if (e != hipSuccess) return e;
        return combine();
    }
    if (st.nf < 1 || st.nf > kMaxStack || !mp_max.fast || ws.seg_bits % 128 != 0 ||
        (uint64_t)ws.nbins * ws.seg_bits != mp_max.m)
        return hipErrorInvalidValue;
    for (int j = 0; j < st.nf; j++)
        if (st.mwords[j] % 4 != 0 || (uint64_t)st.mwords[j] * 32 < ws.seg_bits ||
            mp_max.m % ((uint64_t)st.mwords[j] * 32) != 0)
            return hipErrorInvalidValue;
    hipError_t e = launch_bin<true>(ks, mp_max, ws, slots, stream);
    if (e != hipSuccess) return e;
    e = launch_apply_stack(ws, mp_max.m, res, st, stream);
    if (e != hipSuccess) return e;
    return combine();
}

}  // namespace bloomhip
