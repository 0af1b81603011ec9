// ecdsa_p256.hip -- the P256 instantiations of ecdsa_impl.hpp: the verify
// chain, key staging and generator table for every key-table width.
#include "ecdsa_impl.hpp"
#include "ec_small.hpp"

void launch_ec_p256(const EcArgs& a, hipStream_t s, const Marker& mk) {
  if (a.wq == 26) launch_chain<CurveP256W<26>>(a, s, mk);
  else if (a.wq == 24) launch_chain<CurveP256W<24>>(a, s, mk);
  else if (a.wq == 22) launch_chain<CurveP256W<22>>(a, s, mk);
  else launch_chain<CurveP256W<20>>(a, s, mk);
}

void launch_ec_keyprep_p256(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  keyprep_chain<CurveP256W<20>>(keys, blob, idx, n, s);
}

void launch_ec_keytables_p256(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced) {
  if (wq == 26) keytables_chain<CurveP256W<26>>(keys, blob, tidx, tn, s, sliced);
  else if (wq == 24) keytables_chain<CurveP256W<24>>(keys, blob, tidx, tn, s, sliced);
  else if (wq == 22) keytables_chain<CurveP256W<22>>(keys, blob, tidx, tn, s, sliced);
  else keytables_chain<CurveP256W<20>>(keys, blob, tidx, tn, s, sliced);
}

void launch_ec_gtable_p256(uint32_t* tab, hipStream_t s) { gtable_chain<CurveP256W<20>>(tab, s); }

void launch_ec_small_p256(const EcSmallArgs& a, int wq, hipStream_t s) {
  if (wq == 26) small_launch<CurveP256W<26>>(a, s);
  else if (wq == 24) small_launch<CurveP256W<24>>(a, s);
  else if (wq == 22) small_launch<CurveP256W<22>>(a, s);
  else small_launch<CurveP256W<20>>(a, s);
}
