// K1 variant 5 instantiation 26 (table: hkt_cfg.h)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 12, 10, 256, 1, 6>(const TiledArgs &);
}  // namespace tspgpu
