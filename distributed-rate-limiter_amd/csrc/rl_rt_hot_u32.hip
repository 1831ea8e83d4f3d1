// Hot-chain kernels for CodecC records with uint32_t packed results.
#include "rl_hot.hpp"

namespace rl {
template hipError_t hot_chains_t<CodecC, uint32_t>(const RegionArgs&, hipStream_t);
template hipError_t hot_fill_t<CodecC, uint32_t>(const RegionArgs&, hipStream_t);
}  // namespace rl
