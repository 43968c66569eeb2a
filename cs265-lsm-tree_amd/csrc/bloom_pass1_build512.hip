// bloom_pass1_build512.hip — pass 1 of the partition build (no slots) at
// 512 threads per workgroup (4096-key tiles): every key layout and
// remainder kind of k_part_bin (bloom_device.h), in one translation unit.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_build512(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               hipStream_t stream) {
    return launch_bin_tb<false, 512>(ks, mp, ws, nullptr, stream);
}

}  // namespace bloomhip
