// Stage-split pass variants 50 / 51 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(50, 10, 4, 2, 2, vk_sp::SP_FLAGS)   // C = 2, 2 waves, ring
VK_SP_DEFINE(51, 10, 4, 2, 10, vk_sp::SP_FLAGS)   // C = 2, 10 waves, ring
