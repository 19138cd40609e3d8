// K1 variant 6 configuration 62 (k1_cfg.h, tools/gen_k1_cfgs.py)
#include "hk_sub.h"
namespace tspgpu {
template hipError_t launch_sub_n<double, 14, 10, 256, 6>(const SubArgs &);
}  // namespace tspgpu
