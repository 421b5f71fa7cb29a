// ek_stream.hip — instantiation and launch of the XCD-resident streaming kernel (ek_stream.h), compiled as its
// own translation unit so the engine's other kernels do not rebuild with it.
#include <hip/hip_runtime.h>

#define EK_NT_KERNEL static   // the shared headers' other kernels belong to ek_engine.hip
#include "ek_stream.h"

namespace ek {

template <int N, bool WH>
static void launch_t(int grid, size_t lds, hipStream_t s, DPlan* p, const DBatch& db, const StreamDesc& sd,
                     const LdsLayout& lay, const DState& ds, const Results& rv, int32_t* perr) {
    hipLaunchKernelGGL((k_stream<N, WH>), dim3(grid), dim3(kSBlock), lds, s, p, db, sd, lay, ds, rv, perr);
}

void launch_stream_kernel(int nvc, bool where, int grid, size_t lds, hipStream_t s, DPlan* p, const DBatch& db,
                          const StreamDesc& sd, const LdsLayout& lay, const DState& ds, const Results& rv, int32_t* perr) {
    switch (nvc) {
    case 1: where ? launch_t<1, true>(grid, lds, s, p, db, sd, lay, ds, rv, perr) : launch_t<1, false>(grid, lds, s, p, db, sd, lay, ds, rv, perr); break;
    default: where ? launch_t<2, true>(grid, lds, s, p, db, sd, lay, ds, rv, perr) : launch_t<2, false>(grid, lds, s, p, db, sd, lay, ds, rv, perr); break;
    }
}

}  // namespace ek
