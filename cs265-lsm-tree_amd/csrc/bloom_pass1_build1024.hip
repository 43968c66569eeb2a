// bloom_pass1_build1024.hip — pass 1 of the partition build (no slots) at
// 1024 threads per workgroup (8192-key tiles): every key layout and
// remainder kind of k_part_bin (bloom_device.h), in one translation unit.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_build1024(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               hipStream_t stream) {
    return launch_bin_tb<false, 1024>(ks, mp, ws, nullptr, stream);
}

}  // namespace bloomhip
