// bloom_pass1_super.hip — pass 1 of the partition build on super-tiles of
// 16,384 keys (k_part_bin2, bloom_device.h): builds with many short runs.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_super(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                            hipStream_t stream) {
    return launch_bin_super_impl<false>(ks, mp, ws, nullptr, stream);
}

}  // namespace bloomhip
