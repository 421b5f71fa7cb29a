// ek_tpl_grp.hip — instantiations of the grouping walk k_grp_walk (ek_keymajor.h) and its launcher.
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void launch_grp_walk(bool sort, bool isf, int rdep, dim3 grid, dim3 block, size_t lds, hipStream_t s, DPlan* p,
                     const GrpDesc& g, const Results& res) {
#define EK_GW(S, F, R) hipLaunchKernelGGL((k_grp_walk<S, F, R>), grid, block, lds, s, p, g, res)
#define EK_GW_R(S, F) if (rdep == 8) EK_GW(S, F, 8); else if (rdep == 12) EK_GW(S, F, 12); else EK_GW(S, F, 16)
    if (isf) { if (sort) { EK_GW_R(true, true); } else { EK_GW_R(false, true); } }
    else { if (sort) { EK_GW_R(true, false); } else { EK_GW_R(false, false); } }
#undef EK_GW_R
#undef EK_GW
}

}  // namespace ek
