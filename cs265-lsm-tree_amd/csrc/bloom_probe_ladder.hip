// bloom_probe_ladder.hip — pass 2 of the ladder stack (k_part_apply in
// kApplyLadder mode for every member count and direct count, bloom_device.h).
#include "bloom_device.h"

namespace bloomhip {

hipError_t launch_apply_ladder(const PartitionWorkspace &ws, uint64_t m, uint8_t *res,
                               const StackTable &st, hipStream_t stream) {
    return launch_apply<kApplyLadder>(ws, m, nullptr, 0, 0, res, st, stream);
}

}  // namespace bloomhip
