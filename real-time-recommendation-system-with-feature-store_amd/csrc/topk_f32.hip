// f32 instantiations of the Flat-IP top-K kernel (see topk_impl.h).
#include "topk_impl.h"

namespace rt {
namespace topk {

int launch_f32(const Args& a, const Plan& p, hipStream_t st) {
    const int s = (a.d + 2 - 1) / 2;  // MFMA k-steps
    if (s <= 16) return launch_S<float, 16>(a, p, st);
    if (s <= 32) return launch_S<float, 32>(a, p, st);
    if (s <= 64) return launch_S<float, 64>(a, p, st);
    return RT_ERR_UNSUPPORTED;
}

}  // namespace topk
}  // namespace rt
