// bf16 instantiations of the Flat-IP top-K kernel (see topk_impl.h).
#include "topk_impl.h"

namespace rt {
namespace topk {

int launch_bf16(const Args& a, const Plan& p, hipStream_t st) {
    const int s = (a.d + 16 - 1) / 16;  // MFMA k-steps
    if (s <= 2) return launch_S<__hip_bfloat16, 2>(a, p, st);
    if (s <= 4) return launch_S<__hip_bfloat16, 4>(a, p, st);
    if (s <= 8) return launch_S<__hip_bfloat16, 8>(a, p, st);
    if (s <= 16) return launch_S<__hip_bfloat16, 16>(a, p, st);
    return RT_ERR_UNSUPPORTED;
}

}  // namespace topk
}  // namespace rt
