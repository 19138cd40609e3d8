// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 18, 19.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<18>(const LaunchArgs &, int);
template hipError_t launch_threads<19>(const LaunchArgs &, int);
}  // namespace tspgpu
