// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 15.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<15>(const LaunchArgs &, int);
}  // namespace tspgpu
