// host_mont.hpp -- RSA key constants on the host at key staging: R^2 mod n
// for the device's Montgomery radix R = 2^(28 L) (kernels/rsa.hip works on L
// 28-bit limbs) and n' = -n^-1 mod 2^28.
//
// Round 3 computed R^2 on the device by 56 L modular doublings, one thread per
// key: ~8 k dependent doublings of a 148-limb number for an RSA-4096 key, the
// ~200 ms that every jg_keys_load of the 32-kid bench set spent in key prep
// (profiles/r04_s1_keyload_trace.log).  Here: Montgomery arithmetic on 32-bit
// words (R32 = 2^(32 w)), 2^(56 L) mod n by square-and-double from R32 mod n
// -- about log2(56 L) Montgomery squarings, ~0.2 ms per RSA-4096 key.
// Plain C++ (no HIP): tests/test_host_mont.py builds it alone against Python
// big integers.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace hostmont {

// n as little-endian 32-bit words, top word nonzero, n odd
class Mont {
 public:
  explicit Mont(std::vector<uint32_t> n) : n_(std::move(n)), w_(n_.size()) {
    uint32_t inv = 1;                                   // n^-1 mod 2^32 (Newton)
    for (int k = 0; k < 5; ++k) inv *= 2u - n_[0] * inv;
    n0inv_ = 0u - inv;                                  // -n^-1 mod 2^32
  }
  size_t words() const { return w_; }

  // r = a b / R32 mod n (a, b < n); r may alias a or b
  void mul(uint32_t* r, const uint32_t* a, const uint32_t* b) const {
    std::vector<uint32_t> t(w_ + 2, 0);
    for (size_t i = 0; i < w_; ++i) {
      uint64_t c = 0;
      for (size_t j = 0; j < w_; ++j) {
        const uint64_t s = (uint64_t)t[j] + (uint64_t)a[j] * b[i] + c;
        t[j] = (uint32_t)s;
        c = s >> 32;
      }
      uint64_t s = (uint64_t)t[w_] + c;
      t[w_] = (uint32_t)s;
      t[w_ + 1] = (uint32_t)(s >> 32);
      const uint32_t m = t[0] * n0inv_;
      c = ((uint64_t)t[0] + (uint64_t)m * n_[0]) >> 32;
      for (size_t j = 1; j < w_; ++j) {
        s = (uint64_t)t[j] + (uint64_t)m * n_[j] + c;
        t[j - 1] = (uint32_t)s;
        c = s >> 32;
      }
      s = (uint64_t)t[w_] + c;
      t[w_ - 1] = (uint32_t)s;
      t[w_] = t[w_ + 1] + (uint32_t)(s >> 32);
    }
    reduce_once(t.data(), t[w_]);
    for (size_t j = 0; j < w_; ++j) r[j] = t[j];
  }

  // x = 2 x mod n (x < n)
  void dbl(uint32_t* x) const {
    uint32_t carry = 0;
    for (size_t j = 0; j < w_; ++j) {
      const uint32_t v = x[j];
      x[j] = (v << 1) | carry;
      carry = v >> 31;
    }
    reduce_once(x, carry);
  }

  // 2^e mod n
  std::vector<uint32_t> pow2(uint64_t e) const {
    std::vector<uint32_t> x(w_, 0);
    // R32 mod n: 2^b - n (n has b bits, so it is < n), doubled 32 w - b times
    const int b = bitlen();
    std::vector<uint32_t> top(w_ + 1, 0);
    top[b / 32] |= 1u << (b % 32);
    int64_t br = 0;
    for (size_t j = 0; j < w_; ++j) {
      const int64_t v = (int64_t)top[j] - (int64_t)n_[j] + br;
      x[j] = (uint32_t)v;
      br = v < 0 ? -1 : 0;
    }
    for (int k = b; k < (int)(32 * w_); ++k) dbl(x.data());
    if (e == 0) {                                       // Mont(1) -> 1
      std::vector<uint32_t> one(w_, 0), r(w_);
      one[0] = 1;
      mul(r.data(), x.data(), one.data());
      return r;
    }
    // Mont(2^e) by square-and-double from Mont(2), then out of the domain
    dbl(x.data());
    int hb = 63;
    while (!((e >> hb) & 1)) --hb;
    for (int k = hb - 1; k >= 0; --k) {
      mul(x.data(), x.data(), x.data());
      if ((e >> k) & 1) dbl(x.data());
    }
    std::vector<uint32_t> one(w_, 0), r(w_);
    one[0] = 1;
    mul(r.data(), x.data(), one.data());
    return r;
  }

 private:
  int bitlen() const {
    int b = 32 * (int)w_;
    uint32_t t = n_[w_ - 1];
    int z = 0;
    while (z < 32 && !(t & 0x80000000u)) { t <<= 1; ++z; }
    return b - z;
  }
  // t (w words + a carry word) < 2n -> t mod n in place
  void reduce_once(uint32_t* t, uint32_t carry) const {
    std::vector<uint32_t> d(w_);
    int64_t br = 0;
    for (size_t j = 0; j < w_; ++j) {
      const int64_t v = (int64_t)t[j] - (int64_t)n_[j] + br;
      d[j] = (uint32_t)v;
      br = v < 0 ? -1 : 0;
    }
    if (carry || br == 0)
      for (size_t j = 0; j < w_; ++j) t[j] = d[j];
  }
  std::vector<uint32_t> n_;
  size_t w_;
  uint32_t n0inv_;
};

// n as L 28-bit limbs (the key blob's layout) -> R^2 mod n, R = 2^(28 L), as
// L 28-bit limbs; *np = -n^-1 mod 2^28.  n must be odd and its limbs < 2^28.
inline void rsa_key_constants(const uint32_t* n28, int L, uint32_t* rr28, uint32_t* np) {
  std::vector<uint32_t> w((28 * (size_t)L + 31) / 32, 0);
  for (int i = 0; i < L; ++i) {
    const uint64_t v = (uint64_t)n28[i] << ((28 * i) % 32);
    const size_t q = (28 * (size_t)i) / 32;
    w[q] |= (uint32_t)v;
    if (q + 1 < w.size()) w[q + 1] |= (uint32_t)(v >> 32);
  }
  while (w.size() > 1 && w.back() == 0) w.pop_back();
  const Mont m(w);
  const std::vector<uint32_t> r = m.pow2(56ull * (uint64_t)L);
  for (int i = 0; i < L; ++i) {
    const size_t bit = 28 * (size_t)i, q = bit / 32, s = bit % 32;
    uint64_t v = q < r.size() ? r[q] : 0;
    if (q + 1 < r.size()) v |= (uint64_t)r[q + 1] << 32;
    rr28[i] = (uint32_t)(v >> s) & 0x0fffffffu;
  }
  uint32_t inv = 1;
  for (int k = 0; k < 5; ++k) inv *= 2u - n28[0] * inv;
  *np = (0u - inv) & 0x0fffffffu;
}

}  // namespace hostmont
