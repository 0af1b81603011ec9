// CPU harness for cap_amd/csrc/host_mont.hpp (tests/test_host_mont.py)
#include <cstdint>

#include "../../cap_amd/csrc/host_mont.hpp"

extern "C" void host_rsa_key_constants(const uint32_t* n28, int L, uint32_t* rr28, uint32_t* np) {
  hostmont::rsa_key_constants(n28, L, rr28, np);
}
