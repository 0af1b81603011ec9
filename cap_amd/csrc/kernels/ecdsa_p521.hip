// ecdsa_p521.hip -- the P521 instantiations of ecdsa_impl.hpp: the verify
// chain, key staging and generator table for every key-table width.
#define JG_EC_SCALAR_ATTR __attribute__((amdgpu_waves_per_eu(2)))
#include "ecdsa_impl.hpp"
#include "ec_small.hpp"

void launch_ec_p521(const EcArgs& a, hipStream_t s, const Marker& mk) {
  if (a.wq == 20) launch_chain<CurveP521W<20>>(a, s, mk);
  else if (a.wq == 18) launch_chain<CurveP521W<18>>(a, s, mk);
  else launch_chain<CurveP521W<16>>(a, s, mk);
}

void launch_ec_keyprep_p521(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  keyprep_chain<CurveP521W<16>>(keys, blob, idx, n, s);
}

void launch_ec_keytables_p521(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced) {
  if (wq == 20) keytables_chain<CurveP521W<20>>(keys, blob, tidx, tn, s, sliced);
  else if (wq == 18) keytables_chain<CurveP521W<18>>(keys, blob, tidx, tn, s, sliced);
  else keytables_chain<CurveP521W<16>>(keys, blob, tidx, tn, s, sliced);
}

void launch_ec_gtable_p521(uint32_t* tab, hipStream_t s) { gtable_chain<CurveP521W<16>>(tab, s); }

void launch_ec_small_p521(const EcSmallArgs& a, int wq, hipStream_t s) {
  if (wq == 20) small_launch<CurveP521W<20>>(a, s);
  else if (wq == 18) small_launch<CurveP521W<18>>(a, s);
  else small_launch<CurveP521W<16>>(a, s);
}
