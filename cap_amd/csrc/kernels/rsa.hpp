// rsa.hpp -- launch interface of the RSA kernels (rsa.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct RsaArgs {
  const jgk::JobDev* jobs;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // decoded signature integer, LE words, SoA rows
  const uint32_t* dig;        // digest rows
  uint32_t* xmw;              // x*R mod n, limb rows (generic-e path)
  uint32_t* xlr;              // x, limb rows
  uint32_t* yw;               // s^e mod n rows (LE words)
  uint8_t* status;
  const uint16_t* siglen;
  uint8_t* verdict_pad;
  uint8_t* pss_scratch;       // 2 KiB per token of the class range
  int32_t has_pss;            // the range holds PS* tokens (else the PKCS#1-only pad kernel)
  int64_t npad, begin, end;
};

// RSA-2048 layout: JG_RSA2K_G lanes per token, H limbs per lane
#ifndef JG_RSA2K_G
#define JG_RSA2K_G 2
#endif
constexpr int RSA2K_G = JG_RSA2K_G;
constexpr int RSA2K_H = RSA2K_G == 2 ? 37 : 19;
constexpr int rsa_limbs(int cls) {
  return cls == jgk::CLS_RSA2K ? RSA2K_G * RSA2K_H : cls == jgk::CLS_RSA3K ? 112 : 148;
}
// rows of the signature scratch each RSA class reads: the modexp's limb loads
// touch words up to (28 L - 1) / 32 + 1 (load_limbs_from_words), so those
// rows must be zeroed by prep
constexpr int rsa_sig_rows(int cls) {
  return (28 * rsa_limbs(cls) - 1) / 32 + 2;
}
static_assert(rsa_sig_rows(jgk::CLS_RSA4K) <= jgk::SIGW_ROWS, "RSA-4K signature rows exceed the scratch");

void launch_rsa(int cls, const RsaArgs& a, hipStream_t s, const jgk::Marker& mk);
void launch_rsa_keyprep(jgk::DevKey* keys, uint32_t* blob, int nkeys, hipStream_t s);
