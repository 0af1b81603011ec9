// ecdsa_p384.hip -- the P384 instantiations of ecdsa_impl.hpp: the verify
// chain, key staging and generator table for every key-table width.
#include "ecdsa_impl.hpp"
#include "ec_small.hpp"

void launch_ec_p384(const EcArgs& a, hipStream_t s, const Marker& mk) {
  if (a.wq == 24) launch_chain<CurveP384W<24>>(a, s, mk);
  else if (a.wq == 20) launch_chain<CurveP384W<20>>(a, s, mk);
  else if (a.wq == 18) launch_chain<CurveP384W<18>>(a, s, mk);
  else launch_chain<CurveP384W<16>>(a, s, mk);
}

void launch_ec_keyprep_p384(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  keyprep_chain<CurveP384W<16>>(keys, blob, idx, n, s);
}

void launch_ec_keytables_p384(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced) {
  if (wq == 24) keytables_chain<CurveP384W<24>>(keys, blob, tidx, tn, s, sliced);
  else if (wq == 20) keytables_chain<CurveP384W<20>>(keys, blob, tidx, tn, s, sliced);
  else if (wq == 18) keytables_chain<CurveP384W<18>>(keys, blob, tidx, tn, s, sliced);
  else keytables_chain<CurveP384W<16>>(keys, blob, tidx, tn, s, sliced);
}

void launch_ec_gtable_p384(uint32_t* tab, hipStream_t s) { gtable_chain<CurveP384W<16>>(tab, s); }

void launch_ec_small_p384(const EcSmallArgs& a, int wq, hipStream_t s) {
  if (wq == 24) small_launch<CurveP384W<24>>(a, s);
  else if (wq == 20) small_launch<CurveP384W<20>>(a, s);
  else if (wq == 18) small_launch<CurveP384W<18>>(a, s);
  else small_launch<CurveP384W<16>>(a, s);
}
