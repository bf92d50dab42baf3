// Key/value radix sort used by the spatial index (spatial.hpp): Hilbert keys
// of the particles (or of the evaluation points) with their indices.  Kept
// in its own translation unit so that rocPRIM's templates compile once
// (declared in spatial.hpp).
#include <hipcub/hipcub.hpp>

#include <cstdint>

namespace abc {

size_t sort_pairs_temp_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(
      nullptr, bytes, static_cast<const uint64_t*>(nullptr),
      static_cast<uint64_t*>(nullptr), static_cast<const int32_t*>(nullptr),
      static_cast<int32_t*>(nullptr), static_cast<int>(n > 0 ? n : 1), 0, 64,
      hipStream_t{});
  return bytes;
}

hipError_t sort_pairs(void* temp, size_t temp_bytes, const uint64_t* keys_in,
                      uint64_t* keys_out, const int32_t* vals_in,
                      int32_t* vals_out, int64_t n, int end_bit,
                      hipStream_t st) {
  size_t b = temp_bytes;
  return hipcub::DeviceRadixSort::SortPairs(temp, b, keys_in, keys_out, vals_in,
                                            vals_out, static_cast<int>(n), 0,
                                            end_bit, st);
}

}  // namespace abc
