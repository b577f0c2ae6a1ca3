// Packed-fp32 GELU polynomial on gfx950: does v_pk_fma_f32 with broadcast (op_sel_hi = 0) scalar / constant
// operands compute what the source says?  Three forms over x in [-10, 10] against a host float reference:
// 0 packed float2 (as gemm4w's epilogue wrote it), 1 packed with every coefficient forced into VGPRs, 2 scalar.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/pkfma_probe.cpp -o scripts/probes/pkfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

typedef float float2v __attribute__((ext_vector_type(2)));
__constant__ float kC[8] = {-1.58077310e-09f, 1.21710387e-07f, -4.10085086e-06f, 8.06672293e-05f,
                            -1.04820350e-03f, 9.66487196e-03f, -6.61753780e-02f, 3.98847515e-01f};

template <int MODE>
__global__ void k(const float* x, float* y, int n) {
  const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (i + 1 >= n) return;
  if constexpr (MODE == 2) {
    for (int e = 0; e < 2; ++e) {
      const float v = x[i + e], xc = __builtin_amdgcn_fmed3f(v, -4.f, 4.f), s = xc * xc;
      float p = kC[0];
      for (int c = 1; c < 8; ++c) p = __builtin_fmaf(p, s, kC[c]);
      y[i + e] = __builtin_fmaf(v, xc * p, v * 0.5f);
    }
  } else {
    const float2v v = {x[i], x[i + 1]};
    const float2v xc = {__builtin_amdgcn_fmed3f(v.x, -4.f, 4.f), __builtin_amdgcn_fmed3f(v.y, -4.f, 4.f)};
    const float2v s = xc * xc;
    float2v c[8];
    for (int j = 0; j < 8; ++j) {
      float cj = kC[j];
      if constexpr (MODE == 1) asm volatile("" : "+v"(cj));
      c[j] = float2v{cj, cj};
    }
    float2v p = c[0];
    for (int j = 1; j < 8; ++j) p = __builtin_elementwise_fma(p, s, c[j]);
    const float2v r = __builtin_elementwise_fma(v, xc * p, v * 0.5f);
    y[i] = r.x;
    y[i + 1] = r.y;
  }
}

int main() {
  const int n = 1 << 16;
  std::vector<float> hx(n), hy(n);
  for (int i = 0; i < n; ++i) hx[i] = -10.f + 20.f * i / (n - 1);
  float *dx, *dy;
  (void)hipMalloc(&dx, n * 4);
  (void)hipMalloc(&dy, n * 4);
  (void)hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    if (mode == 0) k<0><<<n / 512, 256>>>(dx, dy, n);
    if (mode == 1) k<1><<<n / 512, 256>>>(dx, dy, n);
    if (mode == 2) k<2><<<n / 512, 256>>>(dx, dy, n);
    (void)hipMemcpy(hy.data(), dy, n * 4, hipMemcpyDeviceToHost);
    double worst = 0;
    int wi = 0;
    for (int i = 0; i < n; ++i) {
      const double ref = 0.5 * hx[i] * (1.0 + std::erf(hx[i] / std::sqrt(2.0)));
      const double e = std::fabs(hy[i] - ref);
      if (!(e <= worst)) worst = e, wi = i;
    }
    printf("mode %d: max |err| %.3g at x = %.4f (got %.6g)\n", mode, worst, hx[wi], hy[wi]);
  }
  return 0;
}
