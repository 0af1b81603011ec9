// rsa.hpp -- launch interface of the RSA kernels (rsa.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct RsaArgs {
  const jg_tok_dev* toks;
  const int32_t* perm;
  const int32_t* wave_key;
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

// rows of the signature scratch each RSA class reads
constexpr int rsa_sig_rows(int cls) {
  return cls == jgk::CLS_RSA2K ? 66 : cls == jgk::CLS_RSA3K ? 99 : 128;
}
constexpr int rsa_limbs(int cls) {
  return cls == jgk::CLS_RSA2K ? 74 : cls == jgk::CLS_RSA3K ? 112 : 148;
}

void launch_rsa(int cls, const RsaArgs& a, hipStream_t s, const jgk::Marker& mk);
void launch_rsa_keyprep(jgk::DevKey* keys, uint32_t* blob, int nkeys, hipStream_t s);
