// K6 dense projection GEMM, C[M, N] = A[M, K] . W[N, K]^T (bf16 in, fp32 accumulate), 256 x 256 tiles
// for the decode-batch shapes of the Llama/Mixtral layers (M = decode batch 512..4096, N, K >= 4096).
//
//   workgroup : 8 waves (512 threads) as 2 (M) x 4 (N); wave tile 128 x 64 = 8 x 4 MFMA 16x16 tiles,
//               mfma_f32_16x16x32_bf16, 128 accumulator registers per lane.
//   K step    : BK = 64 (128 B per row).  A and W tiles (32 KiB each) are staged global -> LDS by
//               LDS-DMA (global_load_lds_dwordx4, no VGPR staging), double-buffered (128 KiB LDS):
//               the DMA of step t+1 is issued before the fragment reads / MFMAs of step t.
//   LDS image : lane-linear (DMA writes base + lane*16), 16 B chunk c of row r stored at chunk
//               c ^ (r & 7): the swizzle is applied to the DMA SOURCE address and to the fragment
//               read (ds_read_b128 lane groups hit 16 distinct bank quads: conflict-free).
//   grid      : 1-D, XCD-aware (bijective remap): the tiles one XCD runs at a time share their W
//               panel (m fastest within an n panel), so weights stream from HBM ~once.
//   epilogue  : accumulators -> bf16 through LDS (freed after the K loop) -> 16 B row stores;
//               optional fused residual add (C = A W^T + R) for the o / down projections.
#include "common.h"

namespace lwc {

typedef __bf16 g256bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kT = 256;          // tile M = N
constexpr int kBKB = 128;        // bytes of K per tile row (64 bf16)
constexpr int kTileB = kT * kBKB;  // 32 KiB per operand tile
constexpr int kStageB = 2 * kTileB;

struct Gemm256Params {
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  const bf16_t* R;  // optional residual [M, N] (row stride ldc)
  int M, N, K, lda, ldc;
  int tiles_m, tiles_n;
};

LWC_DEVICE float4v mfma_16x16x32(const uint4v& a, const uint4v& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(g256bf16x8, a), __builtin_bit_cast(g256bf16x8, b),
                                                 c, 0, 0, 0);
}

__global__ void __launch_bounds__(512) gemm256_kernel(Gemm256Params p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wm = wid >> 2, wn = wid & 3;

  // tile id: XCD-aware remap, then m fastest inside an n panel
  const int nwg = p.tiles_m * p.tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tm = t % p.tiles_m, tn = t / p.tiles_m;
  const int m0 = tm * kT, n0 = tn * kT;
  const int KT = p.K / 64;

  // ---- LDS-DMA staging: each thread moves 4 chunks of A and 4 of W per K step ----
  // unit u = i*512 + tid (i = 0..3) -> row u>>3, LDS chunk u&7 (lane-linear image)
  const bf16_t* asrc[4];
  const bf16_t* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = i * 512 + tid;
    const int row = u >> 3, pch = u & 7;
    const int ch = pch ^ (row & 7);  // global chunk that belongs at LDS chunk pch
    const int ar = min(m0 + row, p.M - 1);  // rows past M are clamped (their outputs are not stored)
    const int wr = min(n0 + row, p.N - 1);
    asrc[i] = p.A + (size_t)ar * p.lda + ch * 8;
    wsrc[i] = p.W + (size_t)wr * p.K + ch * 8;
  }
  auto stage = [&](int buf, int kt) {
    uint8_t* base = smem + buf * kStageB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint8_t* da = base + (i * 512 + wid * 64) * 16;
      uint8_t* dw = base + kTileB + (i * 512 + wid * 64) * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(asrc[i] + kt * 64),
                                       (__attribute__((address_space(3))) void*)da, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * 64),
                                       (__attribute__((address_space(3))) void*)dw, 16, 0, 0);
    }
  };

  float4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) stage(cur ^ 1, kt + 1);
    const uint8_t* As = smem + cur * kStageB;
    const uint8_t* Ws = As + kTileB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // two k-steps of 32 in the 64-wide K tile
      const int ch = 4 * s + q;
      uint4v bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + r16;
        bfr[j] = *reinterpret_cast<const uint4v*>(Ws + r * kBKB + ((ch ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wm * 128 + i * 16 + r16;
        const uint4v af = *reinterpret_cast<const uint4v*>(As + r * kBKB + ((ch ^ (r & 7)) << 4));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_16x16x32(af, bfr[j], acc[i][j]);
      }
    }
    __syncthreads();  // waits the DMA of step kt+1 (vmcnt) and every wave's reads of `cur`
  }

  // ---- epilogue: per wave 128 x 64 bf16 through LDS, then 16 B stores ----
  bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * 64;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + 4 * q + r, col = j * 16 + r16;
        ot[row * 64 + (col ^ ((row & 7) << 3))] = f2bf(acc[i][j][r]);
      }
  __syncthreads();
  // 128 rows x 8 chunks of 16 B per wave; lane covers rows lane/8 + 8k, chunk lane%8
  const int cch = lane & 7;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int row = (lane >> 3) + 8 * k;
    const int gm = m0 + wm * 128 + row;
    const int gn = n0 + wn * 64 + cch * 8;
    if (gm < p.M && gn < p.N) {
      uint4v v = *reinterpret_cast<const uint4v*>(ot + row * 64 + ((cch * 8) ^ ((row & 7) << 3)));
      if (p.R) {
        float a[8], b[8];
        unpack8(v, a);
        unpack8(*reinterpret_cast<const uint4v*>(p.R + (size_t)gm * p.ldc + gn), b);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += b[e];
        v = pack8(a);
      }
      *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) = v;
    }
  }
}

}  // namespace lwc

// C = A W^T (+ R).  Requires K % 64 == 0, N % 8 == 0, 16-byte aligned rows (lda, ldc % 8 == 0).
extern "C" int lwc_gemm256(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda, int ldc,
                           hipStream_t s) {
  using namespace lwc;
  if (K % 64 != 0 || N % 8 != 0 || lda % 8 != 0 || ldc % 8 != 0) return -1;
  if (M == 0 || N == 0) return 0;
  Gemm256Params p{(const bf16_t*)A, (const bf16_t*)W, (bf16_t*)C, (const bf16_t*)R, M, N, K, lda, ldc,
                  (M + kT - 1) / kT, (N + kT - 1) / kT};
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm256_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kStageB);
    attr = true;
  }
  gemm256_kernel<<<p.tiles_m * p.tiles_n, 512, 2 * kStageB, s>>>(p);
  return (int)hipGetLastError();
}
