// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 12, 13.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<12>(const LaunchArgs &, int);
template hipError_t launch_threads<13>(const LaunchArgs &, int);
}  // namespace tspgpu
