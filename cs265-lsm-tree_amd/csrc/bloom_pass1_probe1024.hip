// bloom_pass1_probe1024.hip — pass 1 of the partition probe (with the probe's slots) at
// 1024 threads per workgroup (8192-key tiles): every key layout and
// remainder kind of k_part_bin (bloom_device.h), in one translation unit.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_probe1024(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               uint16_t *slots, hipStream_t stream) {
    return launch_bin_tb<true, 1024>(ks, mp, ws, slots, stream);
}

}  // namespace bloomhip
