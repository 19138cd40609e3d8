// K1 variant 6 configuration 69 (k1_cfg.h, tools/gen_k1_cfgs.py)
#include "hk_sub.h"
namespace tspgpu {
template hipError_t launch_sub_n<int32_t, 13, 10, 256, 8>(const SubArgs &);
}  // namespace tspgpu
