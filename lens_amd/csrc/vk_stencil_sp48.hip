// Stage-split pass variants 48 / 49 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(48, 10, 4, 2, 5, vk_sp::SP_FLAGS)   // C = 2, 5 waves, counter-guarded ring (no barrier)
VK_SP_DEFINE(49, 10, 4, 4, 5, vk_sp::SP_FLAGS)   // C = 4, 5 waves, ring
