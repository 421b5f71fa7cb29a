// ek_tpl_grp.hip — instantiations of the grouping walk k_grp_walk (ek_keymajor.h) and its launcher.
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void launch_grp_walk(bool sort, bool isf, int rdep, bool having, dim3 grid, dim3 block, size_t lds, hipStream_t s, DPlan* p,
                     const GrpDesc& g, const Results& res) {
#define EK_GW(S, F, R, H) hipLaunchKernelGGL((k_grp_walk<S, F, R, H>), grid, block, lds, s, p, g, res)
#define EK_GW_R(S, F, H) if (rdep == 8) EK_GW(S, F, 8, H); else if (rdep == 12) EK_GW(S, F, 12, H); else EK_GW(S, F, 16, H)
#define EK_GW_H(S, F) if (having) { EK_GW_R(S, F, true); } else { EK_GW_R(S, F, false); }
    if (isf) { if (sort) { EK_GW_H(true, true) } else { EK_GW_H(false, true) } }
    else { if (sort) { EK_GW_H(true, false) } else { EK_GW_H(false, false) } }
#undef EK_GW_H
#undef EK_GW_R
#undef EK_GW
}

}  // namespace ek
