// Stage-split pass variants 42 / 43 (vk_stencil_sp.h; dispatch: vk_stencil_sp.hip).
#include "vk_stencil_sp.h"

VK_SP_DEFINE(42, 10, 4, 4, 5, 0)   // C = 4 (256-column tiles), 5 waves
VK_SP_DEFINE(43, 10, 4, 4, 2, 0)   // C = 4, 2 waves
