// K1 variant 5 instantiation 28 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<int32_t, 13, 10, 256, 1, 8>(const TiledArgs &);
}  // namespace tspgpu
