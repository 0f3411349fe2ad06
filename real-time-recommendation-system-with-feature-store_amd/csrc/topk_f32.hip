// f32 instantiations of the Flat-IP top-K kernel (see topk_impl.h).
#include "topk_impl.h"

namespace rt {
namespace topk {

// MFMA k-steps (2 per instruction) padded to 16 / 32 / 64 / 128 (d <= 32 / 64 / 128 / 256)
static int s_f32(int d) {
    const int s = (d + 1) / 2;
    return s <= 16 ? 16 : s <= 32 ? 32 : s <= 64 ? 64 : s <= 128 ? 128 : 0;
}

int launch_f32(const Args& a, const Plan& p, hipStream_t st) {
    switch (s_f32(a.d)) {
        case 16: return launch_S<float, 16>(a, p, st);
        case 32: return launch_S<float, 32>(a, p, st);
        case 64: return launch_S<float, 64>(a, p, st);
        case 128: return launch_S<float, 128>(a, p, st);
        default: return RT_ERR_UNSUPPORTED;
    }
}

Shape shape_f32(int d, int k) {
    switch (s_f32(d)) {
        case 16: return shape_S<float, 16>(k);
        case 32: return shape_S<float, 32>(k);
        case 64: return shape_S<float, 64>(k);
        default: return shape_S<float, 128>(k);
    }
}

}  // namespace topk
}  // namespace rt
