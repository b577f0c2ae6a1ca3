// K11 Mixture-of-experts plumbing (Mixtral-8x7B, BASELINE config 5) + fp8 activation quantisation.
//
//   moe_router  : h [T, d] . router^T (the router GEMV, wave-per-TPW-tokens, reduce-scatter) fused with
//                 the top-k: experts per token and their softmax weights (Mixtral: softmax over all E,
//                 keep top-k, renormalise == softmax over the top-k logits); then
//   moe_permute : per-expert segments row_off[E+1] and the dispatch permutation
//                   src_row[pos] = token of expert-sorted row pos,   inv[t*k + j] = pos of (t, j)
//                 (one workgroup: counts in LDS, prefix, slots by LDS atomics).
//   moe_route   : the same from precomputed logits [T, E] (thread-per-token top-k + moe_permute).
//                 Everything stays on the device (graph-capturable).
//   moe_combine : out[t] = sum_j w[t, j] * Y[inv[t*k + j]]   (expert outputs back to token order)
//   quant_fp8_rows : per-row dynamic e4m3 (OCP) quantisation: scale = amax / 448.
// The expert GEMMs themselves are the grouped MFMA GEMM (gemm.hip) reading A through src_row.
#include "common.h"

namespace lwc {

constexpr int kMaxExperts = 64;
constexpr int kMaxTopK = 8;

// Repeated arg-max top-k (ties -> lower expert id) + softmax over the selected logits of one token.
// lv[EM]: the token's logits (experts >= E already -inf).  Writes ids / weights of (t, 0..k-1).
template <int EM, int KM>
LWC_DEVICE void route_token(const float (&lv)[EM], int E, int k, int t, int* __restrict__ topk_ids,
                            float* __restrict__ topk_w) {
  bool taken[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) taken[e] = e >= E;
  int ids[KM];
  float vals[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    if (j >= k) break;
    int best = 0;
    float bv = -INFINITY;
    bool found = false;
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      if (!taken[e] && (!found || lv[e] > bv)) {
        best = e;
        bv = lv[e];
        found = true;
      }
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) taken[e] |= e == best;
    ids[j] = best;
    vals[j] = bv;
  }
  // softmax over the selected logits (vals[0] is the largest; read it once — the loop overwrites vals[0])
  const float vmax = vals[0];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    if (j >= k) break;
    vals[j] = __expf(vals[j] - vmax);
    sum += vals[j];
  }
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    if (j >= k) break;
    topk_ids[t * k + j] = ids[j];
    topk_w[t * k + j] = vals[j] / sum;
  }
}

// top-k of precomputed router logits [T, E] bf16: one thread per token, many workgroups
template <int EM, int KM>
__global__ void __launch_bounds__(256) moe_topk_kernel(const bf16_t* __restrict__ logits, int T, int E, int k,
                                                       int* __restrict__ topk_ids, float* __restrict__ topk_w) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  float lv[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) lv[e] = e < E ? bf2f(logits[(size_t)t * E + e]) : -INFINITY;
  route_token<EM, KM>(lv, E, k, t, topk_ids, topk_w);
}

// Wave reduce-scatter: the step with xor mask M keeps half of the N live partials (the lane's half by its
// bit M, the partner's other half added through one ds_bpermute each).  Recursion by template, so every
// index is a compile-time constant: as a loop nest the compiler kept the step sizes dynamic and indexed the
// 32 partials by v_cmp / v_cndmask chains (~4700 instructions, 39 us at 4096 tokens).
template <int N, int M, int NV>
LWC_DEVICE void reduce_scatter(float (&acc)[NV], int lane) {
  if constexpr (N > 1) {
    const bool up = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float keep = up ? acc[i + N / 2] : acc[i];
      const float send = up ? acc[i] : acc[i + N / 2];
      acc[i] = keep + __shfl_xor(send, M);
    }
    reduce_scatter<N / 2, M / 2, NV>(acc, lane);
  }
}

// Router GEMV fused with the top-k (K11a): logits[t, e] = <h[t, :], router[e, :]> for the TPW tokens of a
// workgroup.  The 4 waves split the row (wave w takes 16-byte chunks w*64 + lane + 256 i), each lane keeps
// EM x TPW fp32 partials, issuing all of its h / router loads of an iteration before the FMAs.  A wave then
// reduce-SCATTERS its partials (each xor step trades half of the remaining values with the partner lane),
// so after log2(EM*TPW) steps lane l holds the wave sum of value (l >> (6 - log2(EM*TPW))) — 31 shuffles
// for 32 sums instead of 6 per sum — and the 4 wave sums meet in LDS.  The logit is rounded to bf16 as the
// unfused F.linear (bf16 out) would hold it, so both paths pick the same experts.  The router rows (E x d
// bf16, 64 KB for Mixtral) are L2-resident; h is read once.
template <int EM, int KM, int TPW>
__global__ void __launch_bounds__(256) moe_router_kernel(const bf16_t* __restrict__ h, int ldh,
                                                         const bf16_t* __restrict__ router, int T, int E, int d,
                                                         int k, int* __restrict__ topk_ids,
                                                         float* __restrict__ topk_w, bf16_t* __restrict__ logits) {
  constexpr int NV = EM * TPW;
  static_assert(NV <= 64 && (NV & (NV - 1)) == 0, "EM * TPW must be a power of two <= 64");
  __shared__ float s_part[4][NV];
  __shared__ float s_l[NV];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int t0 = blockIdx.x * TPW;
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  const int nc = d >> 3;
  // rows past T / experts past E read a clamped (valid) row; their sums are never used
  const bf16_t* hrow[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) hrow[j] = h + (size_t)min(t0 + j, T - 1) * ldh;
  const bf16_t* rrow[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) rrow[e] = router + (size_t)min(e, E - 1) * d;
#pragma unroll 2
  for (int c = wv * 64 + lane; c < nc; c += 256) {
    uint4v hr[TPW], rr[EM];
#pragma unroll
    for (int j = 0; j < TPW; ++j) hr[j] = *reinterpret_cast<const uint4v*>(hrow[j] + c * 8);
#pragma unroll
    for (int e = 0; e < EM; ++e) rr[e] = *reinterpret_cast<const uint4v*>(rrow[e] + c * 8);
    float hv[TPW][8];
#pragma unroll
    for (int j = 0; j < TPW; ++j) unpack8(hr[j], hv[j]);
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      float rv[8];
      unpack8(rr[e], rv);
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int x = 0; x < 8; ++x) acc[j * EM + e] = fmaf(hv[j][x], rv[x], acc[j * EM + e]);
    }
  }
  reduce_scatter<NV, 32>(acc, lane);
  constexpr int SH = 64 / NV;  // lanes sharing one value after the scatter: finish with a plain xor-sum
#pragma unroll
  for (int m = SH / 2; m >= 1; m >>= 1) acc[0] += __shfl_xor(acc[0], m);
  if (lane % SH == 0) s_part[wv][lane / SH] = acc[0];  // value index = token * EM + expert
  __syncthreads();
  if (threadIdx.x < NV) {
    const int v = threadIdx.x;  // fixed summation order over the waves: deterministic
    s_l[v] = bf2f(f2bf(((s_part[0][v] + s_part[1][v]) + s_part[2][v]) + s_part[3][v]));
  }
  __syncthreads();
  if (threadIdx.x < TPW && t0 + (int)threadIdx.x < T) {
    const int j = threadIdx.x, t = t0 + j;
    float lv[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      lv[e] = e < E ? s_l[j * EM + e] : -INFINITY;
      if (logits != nullptr && e < E) logits[(size_t)t * E + e] = f2bf(lv[e]);
    }
    route_token<EM, KM>(lv, E, k, t, topk_ids, topk_w);
  }
}

// Expert segments + dispatch permutation from topk_ids (one workgroup: LDS counts, prefix, LDS cursors).
// Row order inside an expert segment is arbitrary (atomics), but every row is computed independently, so
// results are deterministic.
__global__ void __launch_bounds__(1024) moe_permute_kernel(const int* __restrict__ topk_ids, int n, int k, int E,
                                                           int* __restrict__ row_off, int* __restrict__ src_row,
                                                           int* __restrict__ inv) {
  __shared__ int s_count[kMaxExperts];
  __shared__ int s_cursor[kMaxExperts];
  constexpr int PT = 8;  // n <= 8192 (the decode batches): every id read once, into registers
  const int tid = threadIdx.x;
  const bool held = n <= 1024 * PT;
  int ids[PT];
  if (tid < E) s_count[tid] = 0;
  if (held) {
#pragma unroll
    for (int i = 0; i < PT; ++i) ids[i] = tid + 1024 * i < n ? topk_ids[tid + 1024 * i] : -1;
  }
  __syncthreads();
  if (held) {
#pragma unroll
    for (int i = 0; i < PT; ++i)
      if (ids[i] >= 0) atomicAdd(&s_count[ids[i]], 1);
  } else {
    for (int i = tid; i < n; i += 1024) atomicAdd(&s_count[topk_ids[i]], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      row_off[e] = acc;
      s_cursor[e] = acc;
      acc += s_count[e];
    }
    row_off[E] = acc;
  }
  __syncthreads();
  if (held) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      if (ids[i] >= 0) {
        const int idx = tid + 1024 * i;
        const int pos = atomicAdd(&s_cursor[ids[i]], 1);
        src_row[pos] = idx / k;
        inv[idx] = pos;
      }
    }
  } else {
    for (int i = tid; i < n; i += 1024) {
      const int pos = atomicAdd(&s_cursor[topk_ids[i]], 1);
      src_row[pos] = i / k;
      inv[i] = pos;
    }
  }
}

// one workgroup per token; d % 8 == 0
__global__ void __launch_bounds__(256) moe_combine_kernel(const bf16_t* __restrict__ Y, const int* __restrict__ inv,
                                                          const float* __restrict__ w, int k, int d,
                                                          bf16_t* __restrict__ out) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = w[t * k + j];
      float y[8];
      unpack8(*reinterpret_cast<const uint4v*>(Y + (size_t)inv[t * k + j] * d + c), y);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += wj * y[e];
    }
    *reinterpret_cast<uint4v*>(out + (size_t)t * d + c) = pack8(acc);
  }
}

// one workgroup per row; d % 8 == 0.  q = x / scale as e4m3 (OCP fn), scale = amax / 448.
__global__ void __launch_bounds__(256) quant_fp8_rows_kernel(const bf16_t* __restrict__ x, int d,
                                                             uint8_t* __restrict__ q, float* __restrict__ scale) {
  __shared__ float red[8];
  const int r = blockIdx.x;
  const bf16_t* row = x + (size_t)r * d;
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4v*>(row + c), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / 448.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[r] = s;
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4v*>(row + c), v);
    uint32_t lo = 0, hi = 0;
    // v_cvt_pk_fp8_f32: two f32 -> two e4m3 bytes in the low / high word half
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
    *reinterpret_cast<uint2*>(q + (size_t)r * d + c) = make_uint2(lo, hi);
  }
}

// SwiGLU + per-row e4m3 quantisation in one pass (the MoE expert FFN between its two fp8 GEMMs):
// gu [rows, 2F] (gate | up, or interleaved in blocks of blk) -> q [rows, F] e4m3 + scale [rows].  One
// workgroup per row keeps silu(g)*u in registers across the row-max reduction, so the bf16 activation is
// never written or re-read (F <= 8 * 256 * kMaxC; larger rows take the recompute loop).
constexpr int kSqMaxC = 8;
// x * sigmoid(x) with v_rcp_f32 (1 ulp) instead of the IEEE division sequence (v_div_scale x2, v_div_fmas,
// v_div_fixup around an rcp: ~9 VALU per element in an epilogue of 256 per lane); the result is rounded
// to bf16 (or e4m3) anyway.  x -> -inf: rcp(inf) = 0, x * 0 = -0 as the division gives
LWC_DEVICE float silu_q(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__global__ void __launch_bounds__(256) silu_mul_quant_fp8_kernel(const bf16_t* __restrict__ gu, int F, int blk,
                                                                 uint8_t* __restrict__ q, float* __restrict__ scale) {
  __shared__ float red[8];
  const int r = blockIdx.x;
  const bf16_t* row = gu + (size_t)r * 2 * F;
  const int nchunk = F >> 3;
  const bool hold = nchunk <= 256 * kSqMaxC;
  float act[kSqMaxC][8];
  auto compute = [&](int c, float (&o)[8]) {
    const bf16_t* src = row + (c / blk) * 2 * blk + c % blk;
    float g[8], u[8];
    unpack8(*reinterpret_cast<const uint4v*>(src), g);
    unpack8(*reinterpret_cast<const uint4v*>(src + blk), u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bf2f(f2bf(silu_q(g[e]) * u[e]));  // the value the bf16 path would hold
  };
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < kSqMaxC; ++i) {
    const int ci = threadIdx.x + 256 * i;
    if (hold && ci < nchunk) {
      compute(ci * 8, act[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(act[i][e]));
    }
  }
  if (!hold) {
    for (int ci = threadIdx.x; ci < nchunk; ci += 256) {
      float o[8];
      compute(ci * 8, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(o[e]));
    }
  }
  amax = block_max(amax, red);
  const float sc = fmaxf(amax, 1e-12f) / 448.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) scale[r] = sc;
  auto store = [&](int c, const float (&v)[8]) {
    uint32_t lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
    *reinterpret_cast<uint2*>(q + (size_t)r * F + c) = make_uint2(lo, hi);
  };
  if (hold) {
#pragma unroll
    for (int i = 0; i < kSqMaxC; ++i) {
      const int ci = threadIdx.x + 256 * i;
      if (ci < nchunk) store(ci * 8, act[i]);
    }
  } else {
    for (int ci = threadIdx.x; ci < nchunk; ci += 256) {
      float o[8];
      compute(ci * 8, o);
      store(ci * 8, o);
    }
  }
}

}  // namespace lwc

extern "C" int lwc_silu_mul_quant_fp8(const void* gu, int rows, int F, int blk, void* q, float* scale, hipStream_t s) {
  using namespace lwc;
  if (blk <= 0) blk = F;
  if (F % 8 != 0 || blk % 8 != 0 || F % blk != 0) return -1;
  if (rows == 0) return 0;
  silu_mul_quant_fp8_kernel<<<rows, 256, 0, s>>>((const bf16_t*)gu, F, blk, (uint8_t*)q, scale);
  return (int)hipGetLastError();
}

extern "C" int lwc_moe_route(const void* logits, int T, int E, int k, int* topk_ids, float* topk_w, int* row_off,
                             int* src_row, int* inv, hipStream_t s) {
  using namespace lwc;
  if (E > kMaxExperts || k > kMaxTopK || k > E || k < 1) return -1;
  if (T == 0) {
    (void)hipMemsetAsync(row_off, 0, sizeof(int) * (E + 1), s);
    return (int)hipGetLastError();
  }
  const dim3 grid((T + 255) / 256);
  const bf16_t* lg = (const bf16_t*)logits;
  if (E <= 8 && k <= 2)
    moe_topk_kernel<8, 2><<<grid, 256, 0, s>>>(lg, T, E, k, topk_ids, topk_w);
  else if (E <= 16)
    moe_topk_kernel<16, kMaxTopK><<<grid, 256, 0, s>>>(lg, T, E, k, topk_ids, topk_w);
  else
    moe_topk_kernel<kMaxExperts, kMaxTopK><<<grid, 256, 0, s>>>(lg, T, E, k, topk_ids, topk_w);
  moe_permute_kernel<<<1, 1024, 0, s>>>(topk_ids, T * k, k, E, row_off, src_row, inv);
  return (int)hipGetLastError();
}

// Router GEMV + top-k + permutation: h [T, d] bf16 (row stride ldh), router [E, d] bf16.  logits (optional,
// [T, E] bf16) receives the rounded logits.  E <= 16; d % 8 == 0.
extern "C" int lwc_moe_router(const void* h, int ldh, const void* router, int T, int E, int d, int k, int* topk_ids,
                              float* topk_w, int* row_off, int* src_row, int* inv, void* logits, hipStream_t s) {
  using namespace lwc;
  if (E > 16 || k > kMaxTopK || k > E || k < 1 || d % 8 != 0 || ldh % 8 != 0) return -1;
  if (T == 0) {
    (void)hipMemsetAsync(row_off, 0, sizeof(int) * (E + 1), s);
    return (int)hipGetLastError();
  }
  const bf16_t* hp = (const bf16_t*)h;
  const bf16_t* rp = (const bf16_t*)router;
  if (E <= 8 && k <= 2)
    moe_router_kernel<8, 2, 4><<<(T + 3) / 4, 256, 0, s>>>(hp, ldh, rp, T, E, d, k, topk_ids, topk_w,
                                                                (bf16_t*)logits);
  else if (E <= 8)
    moe_router_kernel<8, kMaxTopK, 4><<<(T + 3) / 4, 256, 0, s>>>(hp, ldh, rp, T, E, d, k, topk_ids, topk_w,
                                                                       (bf16_t*)logits);
  else
    moe_router_kernel<16, kMaxTopK, 4><<<(T + 3) / 4, 256, 0, s>>>(hp, ldh, rp, T, E, d, k, topk_ids, topk_w,
                                                                        (bf16_t*)logits);
  moe_permute_kernel<<<1, 1024, 0, s>>>(topk_ids, T * k, k, E, row_off, src_row, inv);
  return (int)hipGetLastError();
}

extern "C" int lwc_moe_combine(const void* Y, const int* inv, const float* w, int T, int k, int d, void* out,
                               hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0) return -1;
  if (T == 0) return 0;
  moe_combine_kernel<<<T, 256, 0, s>>>((const bf16_t*)Y, inv, w, k, d, (bf16_t*)out);
  return (int)hipGetLastError();
}

extern "C" int lwc_quant_fp8_rows(const void* x, int rows, int d, void* q, float* scale, hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0) return -1;
  if (rows == 0) return 0;
  quant_fp8_rows_kernel<<<rows, 256, 0, s>>>((const bf16_t*)x, d, (uint8_t*)q, scale);
  return (int)hipGetLastError();
}
