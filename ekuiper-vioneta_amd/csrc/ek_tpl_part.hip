// ek_tpl_part.hip — instantiations of k_part<MODE, WHERE, NVC> (MODE 0-3) (the pane-mode partition, ek_kernels.h) and its
// launcher (ek_launch.h). Units of their own so the device compile runs as parallel jobs.
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void launch_part(int mode, bool where, int nvc, dim3 grid, size_t lds, hipStream_t s, DPlan* p, const DBatch& db,
                 const PaneGrid& g, const GroupDesc& gd, const uint8_t* acc, const Staging& st, uint32_t* ctab, int ls,
                 int64_t rs, int32_t* pane_err) {
#define EK_PART(M, W, N) hipLaunchKernelGGL((k_part<M, W, N>), grid, dim3(kPartBlock), lds, s, p, db, g, gd, acc, st, ctab, ls, rs, pane_err)
#define EK_PART_N(M, W) switch (nvc) { case 1: EK_PART(M, W, 1); break; case 2: EK_PART(M, W, 2); break; \
                                       case 3: EK_PART(M, W, 3); break; default: EK_PART(M, W, 4); break; }
#define EK_PART_W(M) if (where) { EK_PART_N(M, true) } else { EK_PART_N(M, false) }
    if (mode == 0) { EK_PART_W(0) } else if (mode == 1) { EK_PART_W(1) } else if (mode == 2) { EK_PART_W(2) } else { EK_PART_N(3, false) }   // (MODE 3: no WHERE plans, fz_eligible)
#undef EK_PART_W
#undef EK_PART_N
#undef EK_PART
}

}  // namespace ek
