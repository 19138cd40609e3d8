// K1 variant 5 instantiation 21 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<int32_t, 15, 11, 256, 1, 5>(const TiledArgs &);
}  // namespace tspgpu
