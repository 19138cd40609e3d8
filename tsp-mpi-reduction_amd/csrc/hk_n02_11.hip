// Explicit instantiations of the K1 kernels (heldkarp_impl.h) for N = 2, 3, 4, 5, 6, 7, 8, 9, 10, 11.
#include "heldkarp_impl.h"

namespace tspgpu {
template hipError_t launch_threads<2>(const LaunchArgs &, int);
template hipError_t launch_threads<3>(const LaunchArgs &, int);
template hipError_t launch_threads<4>(const LaunchArgs &, int);
template hipError_t launch_threads<5>(const LaunchArgs &, int);
template hipError_t launch_threads<6>(const LaunchArgs &, int);
template hipError_t launch_threads<7>(const LaunchArgs &, int);
template hipError_t launch_threads<8>(const LaunchArgs &, int);
template hipError_t launch_threads<9>(const LaunchArgs &, int);
template hipError_t launch_threads<10>(const LaunchArgs &, int);
template hipError_t launch_threads<11>(const LaunchArgs &, int);
}  // namespace tspgpu
