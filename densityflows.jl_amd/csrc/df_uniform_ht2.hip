// Specialised kernel variant: default conditioner shape, hidden width 32.
#include "df_uniform_impl.h"

namespace df {
template hipError_t launch_uniform_ht<2>(int, int, const ChainArgs&, unsigned, size_t, hipStream_t);
template hipError_t set_uniform_lds_limit_ht<2>(size_t);
template hipError_t uniform_occupancy_ht<2>(int, int, size_t, int*);
}  // namespace df
