// tables.hpp -- launch helper shared by the comb-table builders (ecdsa_impl.hpp, ed25519.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace jgk {
// Comb-table entry builds of `total` entries per key (x tn keys): one launch,
// or -- `sliced`, for builds beside running verification -- launches of
// TABLE_SLICE entries with the stream synchronised after each, so a build
// holds a hardware queue it may share with a verify lane for one slice
// (~20-60 ms) instead of a whole table (~1.1 s for a P-256 W = 26 key).
constexpr int TABLE_SLICE = 1 << 23;
template <class Launch>
inline void table_slices(int total, int tn, bool sliced, hipStream_t s, Launch&& launch) {
  const int step = sliced ? TABLE_SLICE : total;
  for (int e0 = 0; e0 < total; e0 += step) {
    const int e1 = total - e0 < step ? total : e0 + step;
    launch(e0, e1, dim3((unsigned)((e1 - e0 + 63) / 64), (unsigned)tn));
    if (sliced) (void)hipStreamSynchronize(s);
  }
}

}  // namespace jgk
