// ek_tpl_small.hip — instantiations of k_small_win (one wave per small range window, ek_range.h) and its launcher:
// the rules without WHERE here, those with WHERE in ek_tpl_small_w.hip (two parallel jobs).
#ifndef EK_SW_WHERE
#define EK_SW_WHERE false
#define EK_SW_FN launch_small_win_nowhere
#endif
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void EK_SW_FN(int nvc, int rm, bool hs, int grid, int nwin, size_t lds, hipStream_t s, DPlan* p, const DBatch& src,
              const int64_t* ab, const int32_t* wl, const int32_t* slot, const int64_t* ob, const Results& res,
              const SwArith& ar, const SwRedo& rd) {
#define EK_SW(N, R, H) hipLaunchKernelGGL((k_small_win<N, EK_SW_WHERE, R, H>), dim3(grid), dim3(kSwLanes), lds, s, p, src, ab, wl, slot, ob, res, nwin, ar, rd)
#define EK_SW_N(R, H) switch (nvc) { case 1: EK_SW(1, R, H); break; case 2: EK_SW(2, R, H); break; \
                                     case 3: EK_SW(3, R, H); break; default: EK_SW(4, R, H); break; }
    if (hs) {
        if (rm <= 16) { EK_SW_N(16, true) } else { EK_SW_N(kSwRows, true) }
    } else {
        if (rm <= 16) { EK_SW_N(16, false) } else { EK_SW_N(kSwRows, false) }
    }
#undef EK_SW_N
#undef EK_SW
}

#if !EK_SW_WHERE
void launch_small_win_where(int nvc, int rm, bool hs, int grid, int nwin, size_t lds, hipStream_t s, DPlan* p,
                            const DBatch& src, const int64_t* ab, const int32_t* wl, const int32_t* slot, const int64_t* ob,
                            const Results& res, const SwArith& ar, const SwRedo& rd);
void launch_small_win(int nvc, bool where, int rm, bool hs, int grid, int nwin, size_t lds, hipStream_t s, DPlan* p,
                      const DBatch& src, const int64_t* ab, const int32_t* wl, const int32_t* slot, const int64_t* ob,
                      const Results& res, const SwArith& ar, const SwRedo& rd) {
    if (where) launch_small_win_where(nvc, rm, hs, grid, nwin, lds, s, p, src, ab, wl, slot, ob, res, ar, rd);
    else launch_small_win_nowhere(nvc, rm, hs, grid, nwin, lds, s, p, src, ab, wl, slot, ob, res, ar, rd);
}
#endif

}  // namespace ek
