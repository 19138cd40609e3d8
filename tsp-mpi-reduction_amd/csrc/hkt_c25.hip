// K1 variant 5 instantiation 25 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 12, 9, 256, 1, 8>(const TiledArgs &);
}  // namespace tspgpu
