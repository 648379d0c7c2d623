// vrt_sort.hip -- stable device radix sort of (uint32 key, uint32 value)
// pairs for the light-map accumulation (hipCUB / rocPRIM onesweep).  Kept
// in its own translation unit: hipCUB's templates dominate compile time.
#include <hipcub/hipcub.hpp>

#include "vrt_internal.h"

namespace vrt {

hipError_t sort_pairs_u32(void *temp, size_t *temp_bytes, const uint32_t *keys_in, uint32_t *keys_out,
                          const uint32_t *vals_in, uint32_t *vals_out, int64_t n, int bits, hipStream_t st)
{
        return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                  (int)n, 0, bits, st);
}

}  // namespace vrt
