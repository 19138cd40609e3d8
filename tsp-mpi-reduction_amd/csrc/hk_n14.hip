// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 14.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<14>(const LaunchArgs &, int);
}  // namespace tspgpu
