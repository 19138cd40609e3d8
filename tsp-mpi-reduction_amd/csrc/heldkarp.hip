// K1 dispatch: picks the layer kernel (heldkarp_impl.h launch_threads) and the
// n == 2 kernel.  Every layer kernel is compiled in its own unit under k1l/
// (tools/gen_hk_units.py; declared extern here), so a process loads only the
// code objects of the kernels it launches.  Kernel design and the
// bit-exactness argument: heldkarp_impl.h.
#include "heldkarp_impl.h"
#include "k1l/hkl_units.h"

namespace tspgpu {

#define TSPGPU_INST(NN) template hipError_t launch_threads<NN>(const LaunchArgs &, int);
TSPGPU_INST(2) TSPGPU_INST(3) TSPGPU_INST(4) TSPGPU_INST(5) TSPGPU_INST(6) TSPGPU_INST(7)
TSPGPU_INST(8) TSPGPU_INST(9) TSPGPU_INST(10) TSPGPU_INST(11) TSPGPU_INST(12) TSPGPU_INST(13)
TSPGPU_INST(14) TSPGPU_INST(15) TSPGPU_INST(16) TSPGPU_INST(17) TSPGPU_INST(18) TSPGPU_INST(19)
#undef TSPGPU_INST

// n == 2: tsp.cpp:483-502 with cityNums = {1}: key(empty,1) is default-inserted
// with cost 0, so cost = 0 + d[1][0] and the path is [1, 0].
template <typename V>
__global__ void two_city_kernel(const V *__restrict__ dist, int nblocks, V *__restrict__ cost_out,
                                int32_t *__restrict__ tour_out)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    cost_out[b] = V(0) + dist[(size_t)b * 4 + 2];
    tour_out[(size_t)b * 3 + 0] = 1;
    tour_out[(size_t)b * 3 + 1] = 0;
    tour_out[(size_t)b * 3 + 2] = -1;
}

int threads_for(int N, bool lds_table, int requested)
{
    if (lds_table) return lds_table_threads(N);
    if (N >= 12 && N <= 15 && (requested == 512 || requested == 1024)) return requested;
    return 256;
}

size_t lds_bytes_for(int N, bool lds_table, int threads, bool compact, int vbytes)
{
    return N >= 2 && N <= kMaxN ? lds_bytes(N, lds_table, threads, compact, vbytes) : 0;
}

hipError_t launch_heldkarp(const LaunchArgs &a, int grid)
{
    if (a.nblocks <= 0) return hipSuccess;
    const int N = a.n - 1;
    if (N == 1) {
        if (a.vbytes == 4)
            hipLaunchKernelGGL(two_city_kernel<int32_t>, dim3((a.nblocks + 255) / 256), dim3(256), 0, a.stream,
                               static_cast<const int32_t *>(a.dist), a.nblocks, static_cast<int32_t *>(a.cost),
                               a.tour);
        else
            hipLaunchKernelGGL(two_city_kernel<double>, dim3((a.nblocks + 255) / 256), dim3(256), 0, a.stream,
                               static_cast<const double *>(a.dist), a.nblocks, static_cast<double *>(a.cost), a.tour);
        return hipGetLastError();
    }
    switch (N) {
    case 2: return launch_threads<2>(a, grid);
    case 3: return launch_threads<3>(a, grid);
    case 4: return launch_threads<4>(a, grid);
    case 5: return launch_threads<5>(a, grid);
    case 6: return launch_threads<6>(a, grid);
    case 7: return launch_threads<7>(a, grid);
    case 8: return launch_threads<8>(a, grid);
    case 9: return launch_threads<9>(a, grid);
    case 10: return launch_threads<10>(a, grid);
    case 11: return launch_threads<11>(a, grid);
    case 12: return launch_threads<12>(a, grid);
    case 13: return launch_threads<13>(a, grid);
    case 14: return launch_threads<14>(a, grid);
    case 15: return launch_threads<15>(a, grid);
    case 16: return launch_threads<16>(a, grid);
    case 17: return launch_threads<17>(a, grid);
    case 18: return launch_threads<18>(a, grid);
    case 19: return launch_threads<19>(a, grid);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace tspgpu
