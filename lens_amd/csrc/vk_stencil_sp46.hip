// Stage-split pass variants 46 / 47 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(46, 10, 16, 2, 5, 0)   // 16 rows prefetched
VK_SP_DEFINE(47, 10, 12, 2, 10, 0)   // one stage per wave
