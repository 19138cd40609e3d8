// K1 variant 5 configuration 2 (k1_cfg.h, tools/gen_k1_cfgs.py)
#include "hk_tiled.h"
namespace tspgpu {
template hipError_t launch_tiled_n<double, 15, 11, 256, 1, 3>(const TiledArgs &);
}  // namespace tspgpu
