// bloom_pass1_super_probe.hip — pass 1 of the stacked probe on super-tiles
// of 16,384 keys (k_part_bin2 with the slot plane, bloom_device.h): segment
// stacks with many short runs (the f = 10 tree's 1,250 segments).
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_bin_super_probe(const KeySpan &ks, const ModParams &mp, const PartitionWorkspace &ws,
                                  uint16_t *slots, hipStream_t stream) {
    return launch_bin_super_impl<true>(ks, mp, ws, slots, stream);
}

}  // namespace bloomhip
