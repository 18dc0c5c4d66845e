// Stage-split pass variants 44 / 45 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(44, 10, 8, 2, 5, 0)   // 8 rows prefetched by wave 0
VK_SP_DEFINE(45, 10, 12, 2, 5, 0)   // 12 rows prefetched
