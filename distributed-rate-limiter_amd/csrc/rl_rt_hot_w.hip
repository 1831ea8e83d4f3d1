// Hot-chain kernels for CodecW records with uint64_t packed results.
#include "rl_hot.hpp"

namespace rl {
template hipError_t hot_chains_t<CodecW, uint64_t>(const RegionArgs&, hipStream_t);
template hipError_t hot_fill_t<CodecW, uint64_t>(const RegionArgs&, hipStream_t);
}  // namespace rl
