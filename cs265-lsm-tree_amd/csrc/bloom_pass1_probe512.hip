// bloom_pass1_probe512.hip — pass 1 of the partition probe (with the probe's slots) at
// 512 threads per workgroup (4096-key tiles): every key layout and
// remainder kind of k_part_bin (bloom_device.h), in one translation unit.
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_probe512(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                               uint16_t *slots, hipStream_t stream) {
    return launch_bin_tb<true, 512>(ks, mp, ws, slots, stream);
}

}  // namespace bloomhip
