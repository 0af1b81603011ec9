// ecdsa.hip -- ECDSA launch interface (ecdsa.hpp): dispatch by curve to the
// per-curve translation units (ecdsa_p256.hip, ecdsa_p384.hip, ecdsa_p521.hip),
// which instantiate the device code of ecdsa_impl.hpp.
#include <hip/hip_runtime.h>

#include "ecdsa.hpp"

using namespace jgk;

void launch_ec_p256(const EcArgs& a, hipStream_t s, const Marker& mk);
void launch_ec_p384(const EcArgs& a, hipStream_t s, const Marker& mk);
void launch_ec_p521(const EcArgs& a, hipStream_t s, const Marker& mk);
void launch_ec_keyprep_p256(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
void launch_ec_keytables_p256(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced);
void launch_ec_keyprep_p384(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
void launch_ec_keytables_p384(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced);
void launch_ec_keyprep_p521(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
void launch_ec_keytables_p521(int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                              bool sliced);
void launch_ec_gtable_p256(uint32_t* tab, hipStream_t s);
void launch_ec_gtable_p384(uint32_t* tab, hipStream_t s);
void launch_ec_gtable_p521(uint32_t* tab, hipStream_t s);
void launch_ec_small_p256(const EcSmallArgs& a, int wq, hipStream_t s);
void launch_ec_small_p384(const EcSmallArgs& a, int wq, hipStream_t s);
void launch_ec_small_p521(const EcSmallArgs& a, int wq, hipStream_t s);

void launch_ec(int cls, const EcArgs& a, hipStream_t s, const Marker& mk) {
  if (a.end <= a.begin) return;
  switch (cls) {
    case CLS_P256: launch_ec_p256(a, s, mk); break;
    case CLS_P384: launch_ec_p384(a, s, mk); break;
    case CLS_P521: launch_ec_p521(a, s, mk); break;
    default: break;
  }
}

void launch_ec_keyprep(int cls, DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  if (n <= 0) return;
  switch (cls) {
    case CLS_P256: launch_ec_keyprep_p256(keys, blob, idx, n, s); break;
    case CLS_P384: launch_ec_keyprep_p384(keys, blob, idx, n, s); break;
    case CLS_P521: launch_ec_keyprep_p521(keys, blob, idx, n, s); break;
    default: break;
  }
}

void launch_ec_keytables(int cls, int wq, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                         bool sliced) {
  if (tn <= 0) return;
  switch (cls) {
    case CLS_P256: launch_ec_keytables_p256(wq, keys, blob, tidx, tn, s, sliced); break;
    case CLS_P384: launch_ec_keytables_p384(wq, keys, blob, tidx, tn, s, sliced); break;
    case CLS_P521: launch_ec_keytables_p521(wq, keys, blob, tidx, tn, s, sliced); break;
    default: break;
  }
}

void launch_ec_gtable(int cls, uint32_t* tab, hipStream_t s) {
  switch (cls) {
    case CLS_P256: launch_ec_gtable_p256(tab, s); break;
    case CLS_P384: launch_ec_gtable_p384(tab, s); break;
    case CLS_P521: launch_ec_gtable_p521(tab, s); break;
    default: break;
  }
}

void launch_ec_small(int cls, int wq, const EcSmallArgs& a, hipStream_t s) {
  if (a.n == 0) return;
  switch (cls) {
    case CLS_P256: launch_ec_small_p256(a, wq, s); break;
    case CLS_P384: launch_ec_small_p384(a, wq, s); break;
    case CLS_P521: launch_ec_small_p521(a, wq, s); break;
    default: break;
  }
}
