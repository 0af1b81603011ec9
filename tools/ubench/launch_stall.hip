// Host-side launch latency on a few streams: find periodic blocking launches
// in the HIP runtime (pattern of the verify pipeline: per chunk ~8 kernels +
// 1 event on one of 3 streams, round robin).  Measurement only.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spin(unsigned* p, int iters) {
  unsigned v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0x12345u) p[0] = v;
}

int main(int argc, char** argv) {
  const int nstreams = argc > 1 ? atoi(argv[1]) : 3;
  const int kpc = argc > 2 ? atoi(argv[2]) : 8;       // kernels per chunk
  const int evflag = argc > 3 ? atoi(argv[3]) : hipEventDisableTiming;
  std::vector<hipStream_t> st(nstreams);
  for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  std::vector<hipEvent_t> ev(8);
  for (auto& e : ev) hipEventCreateWithFlags(&e, evflag);
  unsigned* d;
  hipMalloc(&d, 4);
  for (int it = 0; it < 3; ++it) {
    std::vector<std::pair<int, double>> slow;
    const auto t0 = std::chrono::steady_clock::now();
    for (int c = 0; c < 64; ++c) {
      hipStream_t s = st[c % nstreams];
      const auto c0 = std::chrono::steady_clock::now();
      for (int k = 0; k < kpc; ++k) hipLaunchKernelGGL(k_spin, dim3(512), dim3(256), 0, s, d, 2000);
      hipEventRecord(ev[c % 8], s);
      if (c >= 8) hipEventSynchronize(ev[(c - 8) % 8]);     // 8 chunks in flight, as the pipeline's slots
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
      if (ms > 0.3) slow.emplace_back(c, ms);
    }
    hipDeviceSynchronize();
    const double tot = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("streams %d kernels/chunk %d evflag %d iter %d: %.2f ms total; slow chunks:", nstreams, kpc, evflag, it, tot);
    for (auto& x : slow) printf(" %d:%.2f", x.first, x.second);
    printf("\n");
  }
  return 0;
}
