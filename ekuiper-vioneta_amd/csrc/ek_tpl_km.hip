// ek_tpl_km.hip — instantiations of the key-major walk k_km_walk (ek_keymajor.h) and its launcher.
#define EK_NO_PLAIN_KERNELS
#include "ek_launch.h"

namespace ek {

void launch_km_walk(int nvc, bool sort, bool write, bool one, bool hs, int nblk, size_t lds, hipStream_t s, DPlan* p,
                    const KmDesc& d, const Results& res) {
#define EK_KM(N, S, W, O, H) hipLaunchKernelGGL((k_km_walk<N, S, W, O, H>), dim3(nblk), dim3(kKmBlock), lds, s, p, d, res)
#define EK_KM_H(N, W, O) if (hs) EK_KM(N, false, W, O, true); else EK_KM(N, false, W, O, false);
#define EK_KM_SW(N) if (one) { if (sort) EK_KM(N, true, true, true, false); else { EK_KM_H(N, true, true) } } \
                    else if (sort) { if (write) EK_KM(N, true, true, false, false); else EK_KM(N, true, false, false, false); } \
                    else { if (write) { EK_KM_H(N, true, false) } else { EK_KM_H(N, false, false) } }
    switch (nvc) { case 1: EK_KM_SW(1) break; case 2: EK_KM_SW(2) break; case 3: EK_KM_SW(3) break; default: EK_KM_SW(4) break; }
#undef EK_KM_SW
#undef EK_KM_H
#undef EK_KM
}

}  // namespace ek
