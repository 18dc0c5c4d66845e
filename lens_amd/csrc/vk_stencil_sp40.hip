// Stage-split pass variants 40 / 41 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(40, 10, 4, 2, 5, 0)   // C = 2, 5 waves, barrier per iteration
VK_SP_DEFINE(41, 10, 4, 2, 2, 0)   // C = 2, 2 waves
