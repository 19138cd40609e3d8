// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 16, 17.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<16>(const LaunchArgs &, int);
template hipError_t launch_threads<17>(const LaunchArgs &, int);
}  // namespace tspgpu
