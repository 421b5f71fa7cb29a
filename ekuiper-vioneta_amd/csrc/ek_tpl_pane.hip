// ek_tpl_pane.hip — instantiations of k_agg, k_finalize / k_finalize_merge and k_ung_tile (pane mode, ek_kernels.h)
// and their launchers (ek_launch.h).
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void launch_agg(int nvc, bool sort, bool having, bool small, dim3 grid, size_t lds, hipStream_t s, DPlan* p, const GroupDesc& gd,
                const LdsLayout& lay, const uint32_t* ctab, int ls, int64_t rs, const Staging& st, const DState& ds,
                const Results& res, const int32_t* pane_err, const int64_t* pbase, uint64_t* scratch, int64_t scr_stride) {
#define EK_AGG(N, S, H, U) do { if constexpr (!(S) && !(U)) { if (small) { hipLaunchKernelGGL((k_agg<N, S, H, U, 4>), grid, dim3(kAggBlock), lds, s, p, gd, lay, ctab, ls, rs, st, ds, res, pane_err, pbase, scratch, scr_stride); break; } } \
                                hipLaunchKernelGGL((k_agg<N, S, H, U>), grid, dim3(kAggBlock), lds, s, p, gd, lay, ctab, ls, rs, st, ds, res, pane_err, pbase, scratch, scr_stride); } while (0)
#define EK_AGG_N(S, H, U) switch (nvc) { case 1: EK_AGG(1, S, H, U); break; case 2: EK_AGG(2, S, H, U); break; \
                                         case 3: EK_AGG(3, S, H, U); break; default: EK_AGG(4, S, H, U); break; }
    // (no staged validity: the fold's instantiation without per-row validity registers; the sort path keeps one)
    const bool nul = st.nullable_mask != 0 || (gd.pad2 & 8);   // EKGPU_VARIANT bit 3: the nullable instantiation always
    if (sort) { if (having) { EK_AGG_N(true, true, true) } else { EK_AGG_N(true, false, true) } }
    else if (nul) { if (having) { EK_AGG_N(false, true, true) } else { EK_AGG_N(false, false, true) } }
    else { if (having) { EK_AGG_N(false, true, false) } else { EK_AGG_N(false, false, false) } }
#undef EK_AGG_N
#undef EK_AGG
}

void launch_fin(int nvc, bool merge, dim3 grid, hipStream_t s, DPlan* p, const WinDesc* w, const DState& ds,
                int32_t ring, const int32_t* pane_err, const Results& res) {
#define EK_FIN(N) if (merge) hipLaunchKernelGGL(k_finalize_merge<N>, dim3(grid.y), dim3(kBlock), 0, s, p, w, ds, ring, pane_err, res); \
                  else hipLaunchKernelGGL(k_finalize<N>, grid, dim3(kBlock), 0, s, p, w, ds, ring, pane_err, res)
    switch (nvc) { case 1: EK_FIN(1); break; case 2: EK_FIN(2); break; case 3: EK_FIN(3); break; default: EK_FIN(4); break; }
#undef EK_FIN
}

void launch_fin_ring(int r, bool vc, bool hv, int part, dim3 grid, hipStream_t s, DPlan* p, const WinDesc* w, int32_t nwin,
                     int32_t cw, const DState& ds, int32_t ring, const int32_t* pane_err, const Results& res, uint32_t* gbase) {
#define EK_FR(R, V, H, P) hipLaunchKernelGGL((k_finalize_ring<R, V, H, P>), grid, dim3(kBlock), 0, s, p, w, nwin, cw, ds, ring, pane_err, res, gbase)
#define EK_FR_R(V, H, P) if (r <= 4) EK_FR(4, V, H, P); else if (r <= 8) EK_FR(8, V, H, P); else if (r <= 12) EK_FR(12, V, H, P); else EK_FR(16, V, H, P)
    if (part == 1) { if (vc) { EK_FR_R(true, false, 1); } else { EK_FR_R(false, false, 1); } return; }
    if (part == 2) { if (vc) { EK_FR_R(true, false, 2); } else { EK_FR_R(false, false, 2); } return; }
    if (vc) { if (hv) { EK_FR_R(true, true, 0); } else { EK_FR_R(true, false, 0); } }
    else { if (hv) { EK_FR_R(false, true, 0); } else { EK_FR_R(false, false, 0); } }
#undef EK_FR_R
#undef EK_FR
}

void launch_ung(int nvc, bool where, dim3 grid, hipStream_t s, DPlan* p, const DBatch& db, const GroupDesc& gd,
                const uint8_t* acc, const DState& ds, int64_t tile, int32_t* pane_err) {
#define EK_UNG(N, W) hipLaunchKernelGGL((k_ung_tile<N, W>), grid, dim3(kUngBlock), 0, s, p, db, gd, acc, ds, tile, pane_err)
#define EK_UNG_N(W) switch (nvc) { case 1: EK_UNG(1, W); break; case 2: EK_UNG(2, W); break; case 3: EK_UNG(3, W); break; default: EK_UNG(4, W); break; }
    if (where) { EK_UNG_N(true) } else { EK_UNG_N(false) }
#undef EK_UNG_N
#undef EK_UNG
}

}  // namespace ek
