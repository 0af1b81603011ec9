// tk.hip -- device unit-test kernels for the multi-precision core (test
// infrastructure: built into libcapjwt_tk.so, used only by tests/).
// Each entry point runs one primitive over n lanes: inputs and outputs are
// arrays of 28-bit limbs, lane-major ([lane][L]).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../kernels/mp.hpp"
#include "../kernels/fe25519.hpp"
#include "../kernels/ecdsa_impl.hpp"   // EC device functions (anonymous namespace) for point-level tests

#include <type_traits>

namespace {

template <class F>
__global__ void k_op(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  constexpr int L = F::L;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[L], y[L], r[L];
#pragma unroll
  for (int j = 0; j < L; ++j) { x[j] = a[i * L + j]; y[j] = b[i * L + j]; }
  switch (op) {
    case 0: mp::mul<F>(r, x, y); break;
    case 1: mp::sqr<F>(r, x); break;
    case 2: mp::inv<F>(r, x); break;
    case 3: mp::to_mont<F>(r, x); break;
    case 4: mp::from_mont<F>(r, x); break;
    case 5: mp::sub<F>(r, x, y); mp::norm<F>(r); break;
    case 6: mp::csub<F>(r); break;
    case 7: mp::mulf<F>(r, x, y); break;      // hot-loop products (P-384: special-form reduction)
    case 8: mp::sqrf<F>(r, x); break;
    default: break;
  }
  if (op == 6) {
#pragma unroll
    for (int j = 0; j < L; ++j) r[j] = x[j];
    mp::csub<F>(r);
  }
#pragma unroll
  for (int j = 0; j < L; ++j) out[i * L + j] = r[j];
}

template <class F>
__global__ void k_fold(const uint32_t* a, uint32_t* out, int n, int canon) {
  constexpr int L = F::L;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[L];
#pragma unroll
  for (int j = 0; j < L; ++j) x[j] = a[i * L + j];
  if (canon) mp::canon<F>(x); else mp::freduce<F>(x);
#pragma unroll
  for (int j = 0; j < L; ++j) out[i * L + j] = x[j];
}

template <class F, class = void> struct has_fold : std::false_type {};
template <class F> struct has_fold<F, std::void_t<decltype(F::FOLD_S)>> : std::true_type {};

template <class F>
int run_op(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  const size_t bytes = sizeof(uint32_t) * F::L * (size_t)n;
  uint32_t *da, *db, *dout;
  if (hipMalloc(&da, bytes) || hipMalloc(&db, bytes) || hipMalloc(&dout, bytes)) return -1;
  (void)hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  if (op >= 100) {
    if constexpr (has_fold<F>::value)
      hipLaunchKernelGGL(k_fold<F>, dim3((n + 63) / 64), dim3(64), 0, 0, da, dout, n, op - 100);
  } else hipLaunchKernelGGL(k_op<F>, dim3((n + 63) / 64), dim3(64), 0, 0, op, da, db, dout, n);
  const hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
  return e == hipSuccess ? 0 : -2;
}

}  // namespace

extern "C" int tk_field_op(int field, int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  switch (field) {
    case 0: return run_op<P256P>(op, a, b, out, n);
    case 1: return run_op<P256N>(op, a, b, out, n);
    case 2: return run_op<P384P>(op, a, b, out, n);
    case 3: return run_op<P384N>(op, a, b, out, n);
    case 4: return run_op<P521P>(op, a, b, out, n);
    case 5: return run_op<P521N>(op, a, b, out, n);
    case 6: return run_op<ED25519P>(op, a, b, out, n);
    case 7: return run_op<ED25519L>(op, a, b, out, n);
    default: return -1;
  }
}

// ---------------------------------------------------------------- EC level
namespace {

template <class CV, bool Z1>
__global__ void k_tk_madd(const uint32_t* in, uint32_t* out, int n) {
  // in per lane: X Y Z x2 y2 (5L words); out: X Y Z (3L)
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t X[L], Y[L], Z[L], x2[L], y2[L];
  const uint32_t* s = in + (size_t)i * 5 * L;
  for (int j = 0; j < L; ++j) { X[j] = s[j]; Y[j] = s[L + j]; Z[j] = s[2 * L + j]; x2[j] = s[3 * L + j]; y2[j] = s[4 * L + j]; }
  if (Z1) madd_z1<Fp>(X, Y, Z, x2, y2);       // Z must be Montgomery 1
  else madd<Fp>(X, Y, Z, x2, y2);
  uint32_t* o = out + (size_t)i * 3 * L;
  for (int j = 0; j < L; ++j) { o[j] = X[j]; o[L + j] = Y[j]; o[2 * L + j] = Z[j]; }
}

template <class CV>
__global__ void k_tk_entry(const int* wd, uint32_t* out, int n) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t gx[L], gy[L];
  mp::set_const<Fp>(gx, CV::C::GX_M); mp::set_const<Fp>(gy, CV::C::GY_M);
  uint32_t base[2 * L], ent[2 * L];
  constexpr int W = ec_comb_w(CV::CLS, true);
  window_base<CV, W>(base, gx, gy, wd[2 * i]);
  table_entry<CV, W>(ent, base, wd[2 * i + 1]);
  load_entry<CV>(ent, out + (size_t)i * 2 * L, out + (size_t)i * 2 * L + L);   // table format -> x, y limbs
}

template <class CV>
int run_ec(int what, const void* in, size_t in_bytes, uint32_t* out, size_t out_bytes, int n) {
  void *din, *dout;
  if (hipMalloc(&din, in_bytes) || hipMalloc(&dout, out_bytes)) return -1;
  (void)hipMemcpy(din, in, in_bytes, hipMemcpyHostToDevice);
  if (what == 0) hipLaunchKernelGGL((k_tk_madd<CV, false>), dim3((n + 63) / 64), dim3(64), 0, 0, (const uint32_t*)din, (uint32_t*)dout, n);
  else if (what == 2) hipLaunchKernelGGL((k_tk_madd<CV, true>), dim3((n + 63) / 64), dim3(64), 0, 0, (const uint32_t*)din, (uint32_t*)dout, n);
  else hipLaunchKernelGGL(k_tk_entry<CV>, dim3((n + 63) / 64), dim3(64), 0, 0, (const int*)din, (uint32_t*)dout, n);
  const hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, out_bytes, hipMemcpyDeviceToHost);
  (void)hipFree(din); (void)hipFree(dout);
  return e == hipSuccess ? 0 : -2;
}

}  // namespace

// what: 0 madd (in: n x 5L words), 2 madd with Z1 = 1, 1 generator table entry (in: n x (w, d) ints)
extern "C" int tk_ec(int curve, int what, const void* in, size_t in_bytes, uint32_t* out, size_t out_bytes, int n) {
  switch (curve) {
    case 1: return run_ec<CurveP256>(what, in, in_bytes, out, out_bytes, n);
    case 2: return run_ec<CurveP384>(what, in, in_bytes, out, out_bytes, n);
    case 3: return run_ec<CurveP521>(what, in, in_bytes, out, out_bytes, n);
    default: return -1;
  }
}

// ---------------------------------------------------------------- radix-2^25.5 GF(2^255 - 19)
namespace {
__global__ void k_fe(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[fe::L], y[fe::L], r[fe::L];
  for (int j = 0; j < fe::L; ++j) { x[j] = a[i * fe::L + j]; y[j] = b[i * fe::L + j]; }
  if (op == 0) {
    fe::mul(r, x, y);
  } else {
    fe::copy(r, x);
    fe::canon(r);
  }
  for (int j = 0; j < fe::L; ++j) out[i * fe::L + j] = r[j];
}
}  // namespace

// op 0: fe::mul(a, b), 1: fe::canon(a); arrays of n x 10 limbs (lane-major)
extern "C" int tk_fe25519(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, int n) {
  const size_t bytes = sizeof(uint32_t) * fe::L * (size_t)n;
  uint32_t *da, *db, *dout;
  if (hipMalloc(&da, bytes) || hipMalloc(&db, bytes) || hipMalloc(&dout, bytes)) return -1;
  (void)hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_fe, dim3((n + 63) / 64), dim3(64), 0, 0, op, da, db, dout, n);
  const hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dout);
  return e == hipSuccess ? 0 : -2;
}
