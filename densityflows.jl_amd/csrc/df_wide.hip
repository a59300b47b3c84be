// Wide-net kernel variants (df_wide_impl.h): one per chain mode.
#include "df_wide_impl.h"

namespace df {

namespace {
void* wide_ptr(int mode) {
    switch (mode) {
        case MODE_FWD: return reinterpret_cast<void*>(&wide_kernel<MODE_FWD>);
        case MODE_FWD_INPLACE: return reinterpret_cast<void*>(&wide_kernel<MODE_FWD_INPLACE>);
        case MODE_BWD: return reinterpret_cast<void*>(&wide_kernel<MODE_BWD>);
        default: return reinterpret_cast<void*>(&wide_kernel<MODE_LOGPDF>);
    }
}
}  // namespace

hipError_t launch_wide(int mode, const ChainArgs& a, unsigned grid, size_t lds, hipStream_t st) {
    void* args[] = {const_cast<ChainArgs*>(&a)};
    return hipLaunchKernel(wide_ptr(mode), dim3(grid), dim3(wide::kThreads), args, lds, st);
}

hipError_t set_wide_lds_limit(size_t lds) {
    for (int mode = 0; mode < 4; ++mode) {
        hipError_t e = hipFuncSetAttribute(wide_ptr(mode), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace df
