// bf16 instantiations of the Flat-IP top-K kernel (see topk_impl.h).
#include "topk_impl.h"

namespace rt {
namespace topk {

// MFMA k-steps (16 per instruction) padded to 4 / 8 / 16 (d <= 64 / 128 / 256)
static int s_bf16(int d) {
    const int s = (d + 15) / 16;
    return s <= 4 ? 4 : s <= 8 ? 8 : s <= 16 ? 16 : 0;
}

int launch_bf16(const Args& a, const Plan& p, hipStream_t st) {
    switch (s_bf16(a.d)) {
        case 4: return launch_S<__hip_bfloat16, 4>(a, p, st);
        case 8: return launch_S<__hip_bfloat16, 8>(a, p, st);
        case 16: return launch_S<__hip_bfloat16, 16>(a, p, st);
        default: return RT_ERR_UNSUPPORTED;
    }
}

// one v4 scan launch in a given mode (the sharded-search entry points)
int v4_scan_bf16(const Args& a, const Plan& p, int stride, int rank, int mode, hipStream_t st) {
    switch (s_bf16(a.d)) {
        case 4: return v4::launch_scan<__hip_bfloat16, 4, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, stride, rank, a.meta,
                                                          mode, a.fail, st);
        case 8: return v4::launch_scan<__hip_bfloat16, 8, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, stride, rank, a.meta,
                                                          mode, a.fail, st);
        default: return RT_ERR_UNSUPPORTED;
    }
}

Shape shape_bf16(int d, int k) {
    switch (s_bf16(d)) {
        case 4: return shape_S<__hip_bfloat16, 4>(k);
        case 8: return shape_S<__hip_bfloat16, 8>(k);
        default: return shape_S<__hip_bfloat16, 16>(k);
    }
}

}  // namespace topk
}  // namespace rt
