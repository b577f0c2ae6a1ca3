// K6 skinny projection GEMM for decode-sized row counts (M <= 64): C[M, N] (+ R) = A[M, K] . W[N, K]^T, bf16
// in / out, fp32 accumulation.
//
// At a serving decode step (a few to 64 sequences) every projection is a weight stream: o (N = K = 4096)
// reads 33.5 MB of W for 0.5 MFLOP per weight row.  The 256 x 256-tile cores (gemm4w / gemm8p) leave all
// but M / 256 of their tile idle and run one tile per 256 W rows (16 workgroups for o: 10x the library's
// time), and hipBLASLt's kernels at these shapes read W at 1.7-2.5 TB/s (o / qkv at M <= 64,
// `scripts/serve_load.py` planner table).  Here the weight stream is the whole design:
//
//   * one workgroup per 16 W rows (N / 16 workgroups: 256 for o, 384 for qkv), 8 waves each owning 1/8 of K
//     (split-K inside the workgroup: no atomics, no second pass, a fixed summation order);
//   * per wave, batches of U k-steps of 32: U 16-byte W loads (lane (r16, g): row r16, k 8g..8g+7 of the
//     step) and U x MT activation loads (A is a few KB-MB, L2-resident) issued back to back, then U x MT
//     `v_mfma_f32_16x16x32_bf16` with W as the A operand and the activations as the B operand, so the
//     accumulator of lane (r16, q) holds output row 16 mt + r16, columns n0 + 4q .. 4q + 3 (4 consecutive
//     output columns: one 8-byte store, one 8-byte residual load);
//   * the 8 waves' partial tiles meet in LDS (8 x MT x 1 KiB) and MT waves finish: sum in wave order,
//     + residual (or SwiGLU of the gate and up tiles, EPI 2), bf16, store.
// Rows past M read zeros (buffer offsets past the activation resource's end) and are not stored.
//
// Requires K % 2048 == 0 (8 waves x an even number of 4-step batches of 32), N % 16 == 0, M <= 64, lda / ldc % 4 == 0; the
// planner (ops/gemm_plan.py, backend "gv") times it against hipBLASLt per decode bucket.
#include "common.h"

namespace lwc {
namespace skinny {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KS = 8;  // waves per workgroup (split-K)

LWC_DEVICE float4v mfma(const uint4v& a, const uint4v& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

struct Params {
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  const bf16_t* R;  // residual [M, ldc] (EPI 1) — may alias C
  int M, N, K, lda, ldc;
};

// NW weight tiles of 16 rows per workgroup, on the same activation fragments: EPI 2 (SwiGLU, W = [gate; up]
// interleaved in blocks of 32 rows, ops.swiglu_interleave) takes its 16 output columns' gate rows 64 (x / 2) +
// 16 (x % 2) + [0, 16) and the up rows 32 further (NW = 2); the plain / residual forms take 16 (NW = 1) or 32
// adjacent output columns (NW = 2: half the workgroups, so half the activation re-reads from L2 — past 16
// rows those loads, M / 16 times the weight bytes, are what limits the NW = 1 form)
template <int MT, int EPI, int NW>
__global__ void __launch_bounds__(512) skinny_kernel(Params p) {
  constexpr int U = 4;  // k-steps per load batch: nb = K / 1024 batches, even for K % 2048 == 0
  static_assert(EPI != 2 || NW == 2, "SwiGLU pairs a gate and an up tile");
  constexpr int TS = EPI == 2 ? 32 : 16;  // W rows between the NW tiles
  __shared__ float4v red[KS][NW][MT][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (EPI == 2 ? 16 : 16 * NW);  // first output column
  const int wrow = EPI == 2 ? 64 * (blockIdx.x >> 1) + 16 * (blockIdx.x & 1) : n0;  // first W row
  const int Kw = p.K / KS;          // this wave's K range [w Kw, (w + 1) Kw)
  const int nb = Kw / (32 * U);     // load batches
  const __amdgpu_buffer_rsrc_t rW = uniform_rsrc(p.W + (size_t)wrow * p.K, (16 + TS * (NW - 1)) * p.K * 2);
  const __amdgpu_buffer_rsrc_t rA = uniform_rsrc(p.A, p.M * p.lda * 2);
  uint32_t voW[NW];
#pragma unroll
  for (int t = 0; t < NW; ++t) voW[t] = (uint32_t)(((r16 + TS * t) * p.K + w * Kw + 8 * g) * 2);
  uint32_t voA[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) voA[mt] = (uint32_t)(((mt * 16 + r16) * p.lda + w * Kw + 8 * g) * 2);

  float4v acc[NW][MT];
#pragma unroll
  for (int t = 0; t < NW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = float4v{0.f, 0.f, 0.f, 0.f};
  // two register sets: batch b + 1's loads go out before batch b's MFMAs (sched_barrier keeps the compiler
  // from interleaving them into load / wait / MFMA triples, which drained the queue every batch)
  uint4v wf[2][U][NW], af[2][U][MT];
  auto load = [&](int b, uint4v(&wb)[U][NW], uint4v(&ab)[U][MT]) {
#pragma unroll
    for (int s = 0; s < U; ++s) {
      const int so = (b * U + s) * 64;  // 32 k of bf16 per step (wave-uniform: soffset)
#pragma unroll
      for (int t = 0; t < NW; ++t)
        wb[s][t] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rW, voW[t], so, 0));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        ab[s][mt] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rA, voA[mt], so, 0));
    }
  };
  auto compute = [&](const uint4v(&wb)[U][NW], const uint4v(&ab)[U][MT]) {
#pragma unroll
    for (int s = 0; s < U; ++s)
#pragma unroll
      for (int t = 0; t < NW; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[t][mt] = mfma(wb[s][t], ab[s][mt], acc[t][mt]);
  };
  // straight-line pairs (no conditional loads: a load under a branch made the wait before every compute a
  // vmcnt(0)); nb is even
  load(0, wf[0], af[0]);
  for (int b = 0; b + 2 < nb; b += 2) {
    load(b + 1, wf[1], af[1]);
    __builtin_amdgcn_sched_barrier(0);
    compute(wf[0], af[0]);
    __builtin_amdgcn_sched_barrier(0);
    load(b + 2, wf[0], af[0]);
    __builtin_amdgcn_sched_barrier(0);
    compute(wf[1], af[1]);
    __builtin_amdgcn_sched_barrier(0);
  }
  load(nb - 1, wf[1], af[1]);
  __builtin_amdgcn_sched_barrier(0);
  compute(wf[0], af[0]);
  __builtin_amdgcn_sched_barrier(0);
  compute(wf[1], af[1]);
#pragma unroll
  for (int t = 0; t < NW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[w][t][mt][lane] = acc[t][mt];
  __syncthreads();
  if (w < MT) {  // wave w finishes m-tile w: the 8 partials in wave order
    float4v sum[NW];
#pragma unroll
    for (int t = 0; t < NW; ++t) {
      sum[t] = red[0][t][w][lane];
#pragma unroll
      for (int k = 1; k < KS; ++k) sum[t] += red[k][t][w][lane];
    }
    constexpr int NO = EPI == 2 ? 1 : NW;  // 16-column output groups
    if constexpr (EPI == 2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sum[0][e] = sum[0][e] * __builtin_amdgcn_rcpf(1.f + __expf(-sum[0][e])) * sum[1][e];
    }
    const int m = w * 16 + r16;
    if (m < p.M) {
#pragma unroll
      for (int t = 0; t < NO; ++t) {
        const size_t off = (size_t)m * p.ldc + n0 + 16 * t + 4 * g;
        float v[4] = {sum[t][0], sum[t][1], sum[t][2], sum[t][3]};
        if constexpr (EPI == 1) {
          const uint2 rr = *reinterpret_cast<const uint2*>(p.R + off);
          v[0] += __uint_as_float(rr.x << 16);
          v[1] += __uint_as_float(rr.x & 0xffff0000u);
          v[2] += __uint_as_float(rr.y << 16);
          v[3] += __uint_as_float(rr.y & 0xffff0000u);
        }
        uint2 o;
        o.x = pack_bf16x2(v[0], v[1]);
        o.y = pack_bf16x2(v[2], v[3]);
        *reinterpret_cast<uint2*>(p.C + off) = o;
      }
    }
  }
}

template <int EPI, int NW>
int launch_nw(const Params& p, hipStream_t s) {
  const int mt = (p.M + 15) / 16;
  const dim3 grid(EPI == 2 ? p.N / 32 : p.N / (16 * NW));  // SwiGLU: N / 2 output columns, 16 per workgroup
  switch (mt) {
    case 1: skinny_kernel<1, EPI, NW><<<grid, 512, 0, s>>>(p); break;
    case 2: skinny_kernel<2, EPI, NW><<<grid, 512, 0, s>>>(p); break;
    case 3:
    case 4: skinny_kernel<4, EPI, NW><<<grid, 512, 0, s>>>(p); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// plain / residual: 32 output columns per workgroup past 16 rows when that still leaves >= 192 workgroups
// (M / 16 activation re-reads halved: qkv at M = 32 23.9 -> 17.9 us), else 16 (o, N = 4096: 128 workgroups
// of 32 columns ran 17.6 us against 13.8 with 256 of 16 — too little of the weight stream in flight)
template <int EPI>
int launch(const Params& p, hipStream_t s) {
  if constexpr (EPI == 2) {
    return launch_nw<2, 2>(p, s);
  } else {
    if (p.M > 16 && p.N % 32 == 0 && p.N / 32 >= 192) return launch_nw<EPI, 2>(p, s);
    return launch_nw<EPI, 1>(p, s);
  }
}

}  // namespace skinny
}  // namespace lwc

// C = A . W^T (epi 0), R + A . W^T (epi 1; R may be C) or silu(A . Wg^T) * (A . Wu^T) over a 32-row gate/up
// interleaved W [N, K] (epi 2, C [M, N / 2]) for M <= 64 rows.  -1: shape not taken.
extern "C" int lwc_skinny_gemm(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda,
                               int ldc, int epi, hipStream_t s) {
  using namespace lwc::skinny;
  const int NC = epi == 2 ? N / 2 : N;
  if (M < 0 || M > 64 || K % 2048 != 0 || N % (epi == 2 ? 64 : 16) != 0 || lda % 4 != 0 || ldc % 4 != 0 ||
      lda < K || ldc < NC)
    return -1;
  if (epi < 0 || epi > 2) return -1;
  if (epi == 1 && R == nullptr) return -1;
  if ((long long)48 * K * 2 >= (1LL << 31) || (long long)M * lda * 2 >= (1LL << 31)) return -1;
  if (M == 0 || N == 0) return 0;
  Params p{(const lwc::bf16_t*)A, (const lwc::bf16_t*)W, (lwc::bf16_t*)C, (const lwc::bf16_t*)R, M, N, K, lda, ldc};
  return epi == 1 ? launch<1>(p, s) : (epi == 2 ? launch<2>(p, s) : launch<0>(p, s));
}
