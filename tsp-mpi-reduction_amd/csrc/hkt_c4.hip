// K1 variant 5 instantiation 4 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 15, 11, 512, 2, 2>(const TiledArgs &);
}  // namespace tspgpu
