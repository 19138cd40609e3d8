// K1 variant 5 (sub-cube tiled, hk_tiled.h) configurations, one per
// instantiation file hkt_c<id>.hip (compiled in parallel):
//   X(id, value type, N, L, threads per workgroup, distance copies R, workgroups per CU)
// Regenerate the hkt_c*.hip files with tools/gen_tiled_cfgs.py after editing.
#pragma once
#include "hk_tiled.h"

#define TSPGPU_TILED_CFGS(X) \
    X(14, double, 15, 10, 256, 1, 6) \
    X(20, int32_t, 15, 10, 256, 1, 8) \
    X(22, double, 14, 10, 256, 1, 6) \
    X(23, double, 13, 10, 256, 1, 6) \
    X(12, double, 15, 10, 256, 1, 5) \
    X(2, double, 15, 11, 256, 1, 3) \
    X(0, double, 15, 11, 512, 1, 2) \
    X(1, double, 15, 10, 256, 1, 4) \
    X(3, double, 15, 10, 512, 1, 2) \
    X(4, double, 15, 11, 512, 2, 2) \
    X(5, double, 14, 11, 512, 1, 2) \
    X(6, double, 14, 10, 256, 1, 4) \
    X(7, int32_t, 15, 11, 256, 1, 4) \
    X(8, int32_t, 15, 11, 512, 1, 2) \
    X(9, int32_t, 14, 11, 256, 1, 4) \
    X(10, double, 13, 10, 256, 1, 4) \
    X(11, double, 15, 10, 128, 1, 6) \
    X(13, double, 15, 10, 192, 1, 5) \
    X(15, double, 15, 9, 256, 1, 6) \
    X(16, double, 15, 9, 256, 1, 7) \
    X(17, double, 15, 10, 256, 2, 5) \
    X(18, double, 15, 10, 256, 1, 7) \
    X(19, int32_t, 15, 10, 256, 1, 6) \
    X(21, int32_t, 15, 11, 256, 1, 5) \
    X(24, int32_t, 14, 10, 256, 1, 6) \
    X(26, double, 12, 10, 256, 1, 6) \
    X(25, double, 12, 9, 256, 1, 8) \
    X(27, int32_t, 14, 10, 256, 1, 8) \
    X(28, int32_t, 13, 10, 256, 1, 8)

namespace tspgpu {
struct TiledCfg {
    int id, vbytes, N, L, threads, R, wg;
    hipError_t (*launch)(const TiledArgs &);
};
#define TSPGPU_TILED_EXTERN(ID, V, N, L, T, R, W) \
    extern template hipError_t launch_tiled_n<V, N, L, T, R, W>(const TiledArgs &);
TSPGPU_TILED_CFGS(TSPGPU_TILED_EXTERN)
#undef TSPGPU_TILED_EXTERN
// every configuration (tspgpu.cpp picks by n, value type and TSPGPU_TILED_CFG)
inline const TiledCfg *tiled_cfgs(int *count)
{
#define TSPGPU_TILED_ROW(ID, V, N, L, T, R, W) {ID, (int)sizeof(V), N, L, T, R, W, &launch_tiled_n<V, N, L, T, R, W>},
    static const TiledCfg t[] = {TSPGPU_TILED_CFGS(TSPGPU_TILED_ROW)};
#undef TSPGPU_TILED_ROW
    *count = (int)(sizeof(t) / sizeof(t[0]));
    return t;
}
}  // namespace tspgpu
