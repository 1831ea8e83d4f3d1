// Normal-region kernels for CodecC records with uint8_t packed results.
#include "rl_region_k.hpp"

namespace rl {
template hipError_t chains_launch_t<CodecC, uint8_t>(const RegionArgs&, hipStream_t, hipStream_t, hipEvent_t);
template hipError_t region_launch_t<CodecC, uint8_t>(const RegionArgs&, hipStream_t, hipStream_t, hipEvent_t);
}  // namespace rl
