// K1 variant 5 instantiation 17 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 15, 10, 256, 2, 5>(const TiledArgs &);
}  // namespace tspgpu
