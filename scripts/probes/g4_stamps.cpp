// Where a gemm4w tile's time goes: a diagnostic build of csrc/kernels/gemm4w.hip with LWC_G4_STAMPS, whose
// wave 0 of every workgroup records s_memrealtime at up to eight points of each persistent round (s_memtime
// at the first and last):
//   S0 tile start, S1 first K tiles landed (prologue wait + barrier), S2 main loop + drain + block barrier
//   done, S7 epilogue done; the wave-local (VAR 64) epilogue also S3 next tile's DMA issued, S4 / S5 / S6
//   m-tiles 0 / 0-3 / 0-7 staged and stored.
// Per shape: the call time (events, 20 back-to-back calls after ~1.5 s of warm-up launches on random
// operands), the in-kernel clock (memtime / realtime x 100 MHz) and, per round, the median over workgroups of
// prologue (S1 - S0), main loop (S2 - S1), epilogue (S7 - S2) and the hand-off to the next round (next S0 - S7);
// for VAR 64 the epilogue's parts.  (The stamped build of the residual epilogue may spill a few VGPRs: compare
// those arms by call time.)
//
// Build (CPU container): hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLWC_G4_STAMPS -I csrc/kernels \
//   scripts/probes/g4_stamps.cpp -o scripts/probes/g4_stamps
// Run (GPU box): timeout -k 10 120 scripts/probes/g4_stamps
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "gemm4w.hip"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void fill_rand(uint16_t* x, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float f = ((h & 0xffffff) / 16777216.0f) * 2.f - 1.f;  // [-1, 1)
    x[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

struct Shape {
  const char* name;
  int M, N, K, epi, var;
};

static double med(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const Shape shapes[] = {
      {"gate_up+swiglu 4096x28672x4096 VAR64", 4096, 28672, 4096, 2, 64},
      {"lm_head 4096x128256x4096 VAR64", 4096, 128256, 4096, 0, 64},
      {"o+res 4096x4096x4096 VAR64", 4096, 4096, 4096, 1, 64},
      {"down+res 4096x4096x14336 VAR64", 4096, 4096, 14336, 1, 64},
      {"enc o+bias 524288x768x768 VAR64", 524288, 768, 768, 3, 64},
      {"enc FFN1+bias+GELU 524288x3072x768 VAR64", 524288, 3072, 768, 4, 64},
  };
  const int blocks = lwc::g4w::device_cus();
  unsigned long long* dst = nullptr;
  CK(hipMalloc(&dst, (size_t)blocks * 64 * 16 * sizeof(unsigned long long)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lwc::g4w::g4_stamps), &dst, sizeof(dst)));
  for (const Shape& sh : shapes) {
    uint16_t *A, *W, *C, *R = nullptr;
    CK(hipMalloc(&A, (size_t)sh.M * sh.K * 2));
    CK(hipMalloc(&W, (size_t)sh.N * sh.K * 2));
    CK(hipMalloc(&C, (size_t)sh.M * sh.N * 2));
    fill_rand<<<1024, 256>>>(A, (size_t)sh.M * sh.K, 1);
    fill_rand<<<1024, 256>>>(W, (size_t)sh.N * sh.K, 2);
    if (sh.epi == 1 || sh.epi == 3 || sh.epi == 4) {  // residual [M, N] / bias [N]
      const size_t nr = sh.epi == 1 ? (size_t)sh.M * sh.N : (size_t)sh.N;
      CK(hipMalloc(&R, nr * 2));
      fill_rand<<<1024, 256>>>(R, nr, 3);
    }
    CK(hipDeviceSynchronize());
    auto call = [&]() {
      return lwc_gemm4w(A, W, C, R, sh.M, sh.N, sh.K, sh.K, sh.epi == 2 ? sh.N / 2 : sh.N, sh.epi, 256, nullptr, 0, 0,
                        1, 1e-5f, sh.var, 0, 1, 0, nullptr, nullptr, 0);
    };
    if (call() != 0) {
      fprintf(stderr, "%s: launch refused\n", sh.name);
      return 1;
    }
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 1.5) {
      for (int i = 0; i < 10; ++i) call();
      CK(hipDeviceSynchronize());
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) call();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // the last call's stamps
    std::vector<unsigned long long> h((size_t)blocks * 64 * 16);
    CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
    const int tiles = ((sh.M + 255) / 256) * ((sh.N + 255) / 256);
    const int rounds = (tiles + blocks - 1) / blocks;
    auto at = [&](int b, int r, int k, int which) { return h[((size_t)b * 64 + r) * 16 + 2 * k + which]; };
    std::vector<double> clk;
    for (int b = 0; b < blocks; ++b) {
      const int last = std::min(rounds, 64) - 1;
      const double dc = (double)(at(b, last, 7, 0) - at(b, 0, 0, 0));
      const double dt = (double)(at(b, last, 7, 1) - at(b, 0, 0, 1));
      if (dt > 0 && at(b, last, 7, 1) >= at(b, 0, 0, 1)) clk.push_back(dc / dt * 100.0);  // MHz
    }
    printf("== %s: %.1f us/call, %d tiles, %d rounds, in-kernel clock %.0f MHz (median over workgroups)\n", sh.name,
           ms * 1e3 / 20, tiles, rounds, med(clk));
    printf("   round | prologue | main loop | epilogue [DMA issue, m-tile 0, m-tiles 1-3, 4-7, tail] | hand-off | loop us/K tile\n");
    double sp = 0, sm = 0, se = 0, sh_ = 0;
    for (int r = 0; r < std::min(rounds, 64); ++r) {
      std::vector<double> p, m, e, o, d[5];
      for (int b = 0; b < blocks; ++b) {
        const int tile = r * blocks + (b & 7) * (blocks / 8) + (b >> 3);
        if (tile >= tiles) continue;
        auto us = [&](int k1, int k0) { return ((double)at(b, r, k1, 1) - (double)at(b, r, k0, 1)) * 0.01; };
        p.push_back(us(1, 0));
        m.push_back(us(2, 1));
        e.push_back(us(7, 2));
        if (sh.var == 64)
          for (int k = 0; k < 5; ++k) d[k].push_back(us(k + 3, k + 2));
        const int nt = (r + 1) * blocks + (b & 7) * (blocks / 8) + (b >> 3);
        if (r + 1 < std::min(rounds, 64) && nt < tiles)
          o.push_back(((double)at(b, r + 1, 0, 1) - (double)at(b, r, 7, 1)) * 0.01);
      }
      sp += med(p), sm += med(m), se += med(e), sh_ += med(o);
      if (r < 3 || r + 2 >= rounds)
        printf("   %5d | %8.2f | %9.2f | %8.2f [%5.2f %5.2f %5.2f %5.2f %5.2f] | %8.2f | %.3f\n", r, med(p), med(m),
               med(e), med(d[0]), med(d[1]), med(d[2]), med(d[3]), med(d[4]), med(o), med(m) / (sh.K / 64));
    }
    printf("   sum   | %8.2f | %9.2f | %8.2f | %8.2f\n", sp, sm, se, sh_);
    // dispatch skew and tail: first / last workgroup start (round 0 S0) and first / last end (last round S7),
    // relative to the first start
    {
      const int last = std::min(rounds, 64) - 1;
      double s0min = 1e30, s0max = 0, s7min = 1e30, s7max = 0;
      for (int b = 0; b < blocks; ++b) {
        const double a0 = (double)at(b, 0, 0, 1);
        int lr = last;
        while (lr > 0 && (lr * blocks + (b & 7) * (blocks / 8) + (b >> 3)) >= tiles) --lr;
        const double a7 = (double)at(b, lr, 7, 1);
        s0min = std::min(s0min, a0), s0max = std::max(s0max, a0);
        s7min = std::min(s7min, a7), s7max = std::max(s7max, a7);
      }
      printf("   starts %.2f .. %.2f us, ends %.2f .. %.2f us (from the first start)\n", 0.0, (s0max - s0min) * 0.01,
             (s7min - s0min) * 0.01, (s7max - s0min) * 0.01);
      // per XCD group (blockIdx % 8: the blocks that share an XCD's L2 under round-robin dispatch): the ends'
      // spread inside the group, and the group's last end — how much a per-XCD work queue could balance
      printf("   per XCD group: ");
      for (int x = 0; x < 8; ++x) {
        double lo = 1e30, hi = 0;
        for (int b = x; b < blocks; b += 8) {
          int lr = last;
          while (lr > 0 && (lr * blocks + (b & 7) * (blocks / 8) + (b >> 3)) >= tiles) --lr;
          const double a7 = (double)at(b, lr, 7, 1);
          lo = std::min(lo, a7), hi = std::max(hi, a7);
        }
        printf("[%.0f..%.0f] ", (lo - s0min) * 0.01, (hi - s0min) * 0.01);
      }
      printf("\n");
    }
    CK(hipFree(A));
    CK(hipFree(W));
    CK(hipFree(C));
    if (R) CK(hipFree(R));
  }
  CK(hipFree(dst));
  return 0;
}
