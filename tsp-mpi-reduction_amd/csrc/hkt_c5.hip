// K1 variant 5 instantiation 5 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 14, 11, 512, 1, 2>(const TiledArgs &);
}  // namespace tspgpu
