// ek_launch.h — host launchers of the engine's big template kernel families.
//
// Each family is instantiated in a unit of its own (ek_tpl_pane.hip, ek_tpl_small.hip, ek_tpl_km.hip) so the
// gfx950 device compile of the engine runs as parallel jobs; the engine (ek_engine.hip) calls these launchers with
// the runtime choices (value columns, WHERE, mode) and the launch geometry. Arguments are the kernels' own.
#pragma once
#include "ek_kernels.h"
#include "ek_range.h"
#include "ek_keymajor.h"

namespace ek {

// pane mode (ek_kernels.h): k_part<MODE, WHERE, NVC>, k_agg<NVC, SORT, HAVING, NULLABLE>, k_finalize / k_finalize_merge<NVC>,
// k_ung_tile<NVC, WHERE>
void launch_part(int mode, bool where, int nvc, dim3 grid, size_t lds, hipStream_t s, DPlan* p, const DBatch& db,
                 const PaneGrid& g, const GroupDesc& gd, const uint8_t* acc, const Staging& st, uint32_t* ctab, int ls,
                 int64_t rs, int32_t* pane_err);
void launch_agg(int nvc, bool sort, bool having, bool small, dim3 grid, size_t lds, hipStream_t s, DPlan* p, const GroupDesc& gd,
                const LdsLayout& lay, const uint32_t* ctab, int ls, int64_t rs, const Staging& st, const DState& ds,
                const Results& res, const int32_t* pane_err, const int64_t* pbase, uint64_t* scratch, int64_t scr_stride);
void launch_fin(int nvc, bool merge, dim3 grid, hipStream_t s, DPlan* p, const WinDesc* w, const DState& ds,
                int32_t ring, const int32_t* pane_err, const Results& res);
// k_finalize_ring<R, VC, HV>: R = ring slots (4 / 8 / 12 / 16, >= the panes of a window), VC: the value column's
// non-nil count, HV: a HAVING; grid (key blocks, window chunks)
void launch_fin_ring(int r, bool vc, bool hv, int part, dim3 grid, hipStream_t s, DPlan* p, const WinDesc* w, int32_t nwin,
                     int32_t cw, const DState& ds, int32_t ring, const int32_t* pane_err, const Results& res, uint32_t* gbase);
void launch_ung(int nvc, bool where, dim3 grid, hipStream_t s, DPlan* p, const DBatch& db, const GroupDesc& gd,
                const uint8_t* acc, const DState& ds, int64_t tile, int32_t* pane_err);

// small range windows (ek_range.h): k_small_win<NVC, WHERE, RM, HS>, RM = rows per lane (16: windows up to 1024 rows),
// HS = HAVING absent or over count(*) alone (table-decided); `grid` persistent waves over `nwin` windows, rd: the
// candidate cap and redo list
void launch_small_win(int nvc, bool where, int rm, bool hs, int grid, int nwin, size_t lds, hipStream_t s, DPlan* p,
                      const DBatch& src, const int64_t* ab, const int32_t* wl, const int32_t* slot, const int64_t* ob,
                      const Results& res, const SwArith& ar, const SwRedo& rd);

// key-major walks (ek_keymajor.h): k_km_walk<NVC, SORT, WRITE, ONE, HS>, k_grp_walk<SORT, ISF, R, HV>; hs: HAVING absent
// or over count(*) alone with every key run shorter than kHStarTab (ignored with sort)
void launch_km_walk(int nvc, bool sort, bool write, bool one, bool hs, int nblk, size_t lds, hipStream_t s, DPlan* p,
                    const KmDesc& d, const Results& res);
void launch_grp_walk(bool sort, bool isf, int rdep, bool having, dim3 grid, dim3 block, size_t lds, hipStream_t s, DPlan* p,
                     const GrpDesc& g, const Results& res);

}  // namespace ek
