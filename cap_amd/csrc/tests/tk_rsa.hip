// tk_rsa.hip -- TEST INFRASTRUCTURE (libcapjwt_tk.so only, never the product
// path): the raw RSA public operation y = s^e mod n through the production
// k_rsa_modexp kernel and the key constants of host_mont.hpp (as jg_keys_load
// stages them), so tests/test_gpu_rsa.py can compare
// every output word with Python's pow() -- the EM compare of k_rsa_pad only
// tells accept from reject.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <initializer_list>
#include <vector>

#include "../host_mont.hpp"
#include "../kernels/rsa.hip"   // kernels in an anonymous namespace: this TU's own copy

namespace {

template <class T>
T* dev_upload(const std::vector<T>& h) {
  T* d = nullptr;
  if (hipMalloc(&d, h.size() * sizeof(T) + 16) != hipSuccess) return nullptr;
  (void)hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
  return d;
}

}  // namespace

// cls: CLS_RSA2K/3K/4K.  n_le: the modulus as n_words little-endian 32-bit
// words (odd, bit length within the class).  s_le: ntok signature integers,
// n_words words each.  Out: y_le (ntok x n_words words), ok[i] = 1 when the
// kernel accepted s_i (s_i < n).  Returns 0, or -1 on bad arguments / HIP errors.
extern "C" int tk_rsa_modexp(int cls, const uint32_t* n_le, int n_words, uint64_t e, const uint32_t* s_le, int ntok,
                             uint32_t* y_le, uint8_t* ok) {
  if (cls < CLS_RSA2K || cls > CLS_RSA4K || ntok <= 0 || n_words <= 0 || n_words > SIGW_ROWS) return -1;
  const int64_t np = (ntok + WAVE - 1) / WAVE * WAVE;
  int bits = 0;
  for (int q = n_words - 1; q >= 0 && !bits; --q)
    if (n_le[q]) bits = 32 * q + 32 - __builtin_clz(n_le[q]);
  // the RSA-4K+ class picks its layout (148 / 296 / 592 limbs) by the key size
  const int L = cls == CLS_RSA4K ? rsa4k_limbs_for_bits(bits) : rsa_limbs(cls);
  if (bits == 0 || L == 0 || bits > 28 * L - 2 || !(n_le[0] & 1)) return -1;

  // key blob: n as 28-bit limbs, then R^2 (host_mont.hpp, as jg_keys_load stages it)
  std::vector<uint32_t> blob(2 * (size_t)L, 0);
  for (int j = 0; j < L; ++j) {
    const int bit = 28 * j, q = bit >> 5, sh = bit & 31;
    const uint64_t w0 = q < n_words ? n_le[q] : 0, w1 = q + 1 < n_words ? n_le[q + 1] : 0;
    blob[j] = (uint32_t)(((w1 << 32) | w0) >> sh) & 0x0fffffffu;
  }
  DevKey K{};
  hostmont::rsa_key_constants(blob.data(), L, blob.data() + L, &K.np);
  K.kind = 1;
  K.cls = cls;
  K.valid = 1;
  K.kbytes = (bits + 7) / 8;
  K.e_lo = (uint32_t)e;
  K.e_hi = (uint32_t)(e >> 32);
  K.nlimbs = (uint32_t)L;
  K.n_off = 0;
  K.rr_off = (uint64_t)L;
  K.embits = bits - 1;

  std::vector<uint32_t> sigw((size_t)SIGW_ROWS * np, 0);
  for (int p = 0; p < ntok; ++p)
    for (int q = 0; q < n_words; ++q) sigw[(size_t)q * np + p] = s_le[(size_t)p * n_words + q];
  std::vector<JobDev> jobs(np);
  for (int64_t p = 0; p < np; ++p) jobs[p] = JobDev{0, 0, 0, job_pack(0, p < ntok ? 1u : JOB_PAD, 0)};
  std::vector<uint16_t> siglen(np, (uint16_t)K.kbytes);
  std::vector<uint8_t> status(np, ST_OK);

  DevKey* dk = dev_upload(std::vector<DevKey>{K});
  uint32_t* dblob = dev_upload(blob);
  uint32_t* dsig = dev_upload(sigw);
  JobDev* djobs = dev_upload(jobs);
  uint16_t* dlen = dev_upload(siglen);
  uint8_t* dst = dev_upload(status);
  std::vector<uint32_t> zero((size_t)(2 * L + SIGW_ROWS) * np, 0);
  uint32_t* rows = dev_upload(zero);
  int rc = (dk && dblob && dsig && djobs && dlen && dst && rows) ? 0 : -1;
  if (rc == 0) {
    RsaArgs a{};
    a.jobs = djobs; a.keys = dk; a.keyblob = dblob; a.sigw = dsig;
    a.xmw = rows; a.xlr = rows + (size_t)L * np; a.yw = rows + (size_t)2 * L * np;
    a.status = dst; a.siglen = dlen; a.npad = np; a.begin = 0; a.end = np;
    const unsigned waves = (unsigned)(np / WAVE);
    switch (cls) {   // the launch shapes of launch_rsa, without the padding check
      case CLS_RSA2K: hipLaunchKernelGGL((k_rsa_modexp<RSA2K_H, RSA2K_G, 8>), dim3(waves * RSA2K_G), dim3(WAVE), 0, 0, a); break;
      case CLS_RSA3K: hipLaunchKernelGGL((k_rsa_modexp<RSA3K_H, RSA3K_G, RSA3K_U>), dim3(waves * RSA3K_G), dim3(WAVE), 0, 0, a); break;
      default:
        if (L == rsa4k_layout_limbs(0)) hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 4, 8>), dim3(waves * 4), dim3(WAVE), 0, 0, a);
        else if (L == rsa4k_layout_limbs(1)) hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 8, 8>), dim3(waves * 8), dim3(WAVE), 0, 0, a);
        else hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 16, 8>), dim3(waves * 16), dim3(WAVE), 0, 0, a);
        break;
    }
    if (hipDeviceSynchronize() != hipSuccess) rc = -1;
  }
  if (rc == 0) {
    std::vector<uint32_t> yw((size_t)SIGW_ROWS * np);
    (void)hipMemcpy(yw.data(), rows + (size_t)2 * L * np, yw.size() * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipMemcpy(status.data(), dst, status.size(), hipMemcpyDeviceToHost);
    for (int p = 0; p < ntok; ++p) {
      ok[p] = status[p] == ST_OK;
      for (int q = 0; q < n_words; ++q) y_le[(size_t)p * n_words + q] = yw[(size_t)q * np + p];
    }
  }
  for (void* ptr : {(void*)dk, (void*)dblob, (void*)dsig, (void*)djobs, (void*)dlen, (void*)dst, (void*)rows})
    if (ptr) (void)hipFree(ptr);
  return rc;
}
