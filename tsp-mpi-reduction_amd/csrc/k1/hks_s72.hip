// K1 variant 6 configuration 72 (k1_cfg.h, tools/gen_k1_cfgs.py)
#include "hk_sub.h"
namespace tspgpu {
template hipError_t launch_sub_n<int32_t, 15, 9, 128, 12>(const SubArgs &);
}  // namespace tspgpu
