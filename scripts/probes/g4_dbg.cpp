// Debug harness: gemm4w at var 32 / 64 on small shapes vs a CPU fp32 reference (build against any gemm4w.hip
// with -I <dir>: scripts/probes/g4_dbg.cpp -> g4_dbg_*).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>
#include "gemm4w.hip"
static uint16_t f2b(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
static float b2f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; std::memcpy(&f, &u, 4); return f; }
int main() {
  const int shapes[][3] = {{256, 256, 128}, {256, 256, 256}, {256, 256, 512}, {512, 512, 1024}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    std::vector<uint16_t> a(M * K), w(N * K), c(M * N);
    uint32_t x = 12345;
    auto rnd = [&]() { x = x * 1664525u + 1013904223u; return ((x >> 8) & 0xffff) / 32768.f - 1.f; };
    for (auto& v : a) v = f2b(rnd());
    for (auto& v : w) v = f2b(rnd() / 16.f);
    void *da, *dw, *dc;
    (void)hipMalloc(&da, a.size() * 2); (void)hipMalloc(&dw, w.size() * 2); (void)hipMalloc(&dc, c.size() * 2);
    (void)hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    for (int var : {32, 64}) {
      (void)hipMemset(dc, 0, c.size() * 2);
      int rc = lwc_gemm4w(da, dw, dc, nullptr, M, N, K, K, N, 0, 256, nullptr, 0, 0, 1, 1e-5f, var, 8, 1, 0, nullptr, nullptr, 0);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(c.data(), dc, c.size() * 2, hipMemcpyDeviceToHost);
      double maxe = 0;
      for (int i = 0; i < M; i += 7)
        for (int j = 0; j < N; j += 5) {
          double s = 0;
          for (int k = 0; k < K; ++k) s += (double)b2f(a[i * K + k]) * b2f(w[j * K + k]);
          maxe = std::max(maxe, std::fabs(s - b2f(c[i * N + j])));
        }
      printf("M=%d N=%d K=%d var=%d rc=%d max err %.4f\n", M, N, K, var, rc, maxe);
    }
    (void)hipFree(da); (void)hipFree(dw); (void)hipFree(dc);
  }
  return 0;
}
