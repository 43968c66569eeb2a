// bloom_pass2.hip — pass 2 of the partition build (k_part_apply in build
// modes, bloom_device.h): segments or plan_build's one-member ladder.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_part_apply(const ModParams &mp, uint32_t *words, const PartitionWorkspace &ws,
                             int merge_existing, hipStream_t stream) {
    if (ws.ntiles == 0) return hipSuccess;
    const uint64_t nw32 = ((mp.m + 63) / 64) * 2;
    if (ws.lad_u) {  // plan_build's one-member ladder
        if (!mp.p2 || ws.lad_hb != 0 || ws.lad_s + ws.lad_u != mp.p2t || ws.lad_s < 7 ||
            ws.seg_bits != (mp.p2d << ws.lad_s) || ws.nbins != ((size_t)1 << ws.lad_u))
            return hipErrorInvalidValue;
        StackTable st{};
        st.lad.s = ws.lad_s;
        st.lad.u = ws.lad_u;
        st.lad.d = mp.p2d;
        st.lad.t[0] = mp.p2t;
        st.lad.rinv = ladder0_relabel(mp, ws) ? ladder0_inv(mp) : 0u;
        return launch_apply<kApplyBuildL>(ws, mp.m, words, nw32, merge_existing, nullptr, st,
                                          stream);
    }
    return launch_apply<kApplyBuild>(ws, mp.m, words, nw32, merge_existing, nullptr, StackTable{},
                                     stream);
}

}  // namespace bloomhip
