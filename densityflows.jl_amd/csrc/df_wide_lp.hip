// Wide-net kernel, MODE_LOGPDF (logpdf, the NLL and the training inverse pass with its
// snapshots): a unit of its own so that it is scheduled apart from the forward modes
// (Makefile: FLAGS_df_wide_lp vs FLAGS_df_wide).
#include "df_wide_impl.h"

namespace df {

void* wide_ptr_logpdf(bool split) {
    return split ? reinterpret_cast<void*>(&wide_kernel<MODE_LOGPDF, true>)
                 : reinterpret_cast<void*>(&wide_kernel<MODE_LOGPDF, false>);
}

}  // namespace df
