// CPU build of the device SHA-2 code (cap_amd/csrc/kernels/sha2.hpp) for
// tests/test_sha2_host.py: the same compression functions and padding the
// prep / hash / PSS kernels run, checked against hashlib on the CPU.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../cap_amd/csrc/kernels/sha2.hpp"

extern "C" int sha2_host(int bits, const uint8_t* msg, uint32_t len, const uint8_t* prefix64, uint8_t* out) {
  // the device reads aligned words around the string: give it slack
  std::vector<uint32_t> buf((len + 3) / 4 + 64, 0);
  std::memcpy(buf.data(), msg, len);
  sha2::MemString m{buf.data(), 0, len};
  if (bits == 256) {
    uint32_t h[8];
    sha2::sha256_mem(h, m);
    for (int k = 0; k < 8; ++k)
      for (int b = 0; b < 4; ++b) out[4 * k + b] = (uint8_t)(h[k] >> (24 - 8 * b));
    return 32;
  }
  uint32_t pre[16];
  for (int k = 0; k < 16 && prefix64; ++k)
    pre[k] = (uint32_t)prefix64[4 * k] << 24 | (uint32_t)prefix64[4 * k + 1] << 16 | (uint32_t)prefix64[4 * k + 2] << 8 |
             prefix64[4 * k + 3];
  uint64_t h[8];
  sha2::sha512_mem(h, bits == 384, m, pre, prefix64 ? 64 : 0);
  const int nw = bits == 384 ? 6 : 8;
  for (int k = 0; k < nw; ++k)
    for (int b = 0; b < 8; ++b) out[8 * k + b] = (uint8_t)(h[k] >> (56 - 8 * b));
  return nw * 8;
}
