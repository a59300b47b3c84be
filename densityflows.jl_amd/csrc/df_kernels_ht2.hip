// Generic kernel variant: hidden width <= 32 (HT = 2 row tiles of 16).
#include "df_chain_impl.h"

namespace df {
template hipError_t launch_chain_ht<2>(int, bool, const ChainArgs&, unsigned, size_t, hipStream_t);
template hipError_t set_lds_limit_ht<2>(size_t);
template hipError_t chain_occupancy_ht<2>(int, bool, size_t, int*);
}  // namespace df
