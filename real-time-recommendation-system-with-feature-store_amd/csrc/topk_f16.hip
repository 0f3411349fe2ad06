// f16 instantiations of the Flat-IP top-K kernel (see topk_impl.h).
#include "topk_impl.h"

namespace rt {
namespace topk {

// MFMA k-steps (16 per instruction) padded to 4 / 8 / 16 (d <= 64 / 128 / 256)
static int s_f16(int d) {
    const int s = (d + 15) / 16;
    return s <= 4 ? 4 : s <= 8 ? 8 : s <= 16 ? 16 : 0;
}

int launch_f16(const Args& a, const Plan& p, hipStream_t st) {
    switch (s_f16(a.d)) {
        case 4: return launch_S<__half, 4>(a, p, st);
        case 8: return launch_S<__half, 8>(a, p, st);
        case 16: return launch_S<__half, 16>(a, p, st);
        default: return RT_ERR_UNSUPPORTED;
    }
}

// one v4 scan launch in a given mode (the sharded-search entry points)
int v4_scan_f16(const Args& a, const Plan& p, int stride, int rank, int mode, hipStream_t st) {
    switch (s_f16(a.d)) {
        case 4: return v4::launch_scan<__half, 4, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, stride, rank, a.meta,
                                                          mode, a.fail, st);
        case 8: return v4::launch_scan<__half, 8, v4::kQS>(a, p.q_tiles, p.splits, p.items_per_split, stride, rank, a.meta,
                                                          mode, a.fail, st);
        default: return RT_ERR_UNSUPPORTED;
    }
}

Shape shape_f16(int d, int k) {
    switch (s_f16(d)) {
        case 4: return shape_S<__half, 4>(k);
        case 8: return shape_S<__half, 8>(k);
        default: return shape_S<__half, 16>(k);
    }
}

}  // namespace topk
}  // namespace rt

#ifdef RT_TOPK_PROBE_TIMING
extern "C" void* rt_topk_probe_cycles_f16() { return rt::topk::v3::probe_cycles_addr(); }
#endif
