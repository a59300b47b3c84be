// Wide-net kernel variants (df_wide_impl.h): one per chain mode (MODE_LOGPDF in df_wide_lp.hip).
#include "df_wide_impl.h"

namespace df {

void* wide_ptr_logpdf(bool split);  // df_wide_lp.hip

namespace {
template <bool SPLIT>
void* wide_ptr_t(int mode) {
    switch (mode) {
        case MODE_FWD: return reinterpret_cast<void*>(&wide_kernel<MODE_FWD, SPLIT>);
        case MODE_FWD_INPLACE: return reinterpret_cast<void*>(&wide_kernel<MODE_FWD_INPLACE, SPLIT>);
        case MODE_BWD: return reinterpret_cast<void*>(&wide_kernel<MODE_BWD, SPLIT>);
        default: return wide_ptr_logpdf(SPLIT);
    }
}
void* wide_ptr(int mode, bool split = false) { return split ? wide_ptr_t<true>(mode) : wide_ptr_t<false>(mode); }
}  // namespace

hipError_t launch_wide(int mode, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st, bool split) {
    void* args[] = {const_cast<ChainArgs*>(&a)};
    return hipLaunchKernel(wide_ptr(mode, split), dim3(grid), dim3(split ? wide::kSplitWaves * 64 : wide::kThreads),
                           args, lds, st);
}

hipError_t set_wide_lds_limit(size_t lds, bool split) {
    for (int mode = 0; mode < 4; ++mode) {
        hipError_t e =
            hipFuncSetAttribute(wide_ptr(mode, split), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace df
