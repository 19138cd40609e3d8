// K1 variant 5 configuration 14 (k1_cfg.h, tools/gen_k1_cfgs.py)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 15, 10, 256, 1, 6>(const TiledArgs &);
}  // namespace tspgpu
