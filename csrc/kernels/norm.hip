// K1 rmsnorm_fused_residual and K9a layernorm(+residual) for gfx950.
//
// One workgroup per row; every thread owns up to kMaxVec 16-byte vectors (8 bf16) of the row in
// registers, so the row is read from HBM exactly once and written once (residual stream update and
// normalised output in the same pass).  Memory-bound: the only levers are 16 B/lane accesses
// (Guideline 13) and a single pass.
//
// Reference behaviour served: decoder layers for `LlmBase.model` (reference
// src/score/llm/mod.rs:10) and the embeddings encoder (`WeightTrainingTableEmbeddings.model`,
// src/score/model/mod.rs:309-314).
#include "common.h"

namespace lwc {

constexpr int kMaxVec = 4;  // rows up to 4 * 8 * 1024 = 32768 elements

// y = rmsnorm(x [+ residual]) * w ; if residual != nullptr: residual <- x + residual (pre-norm sum)
template <bool kResidual>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                      const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                      int d, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const uint4v* xr = reinterpret_cast<const uint4v*>(x + (size_t)row * d);
  uint4v* rr = reinterpret_cast<uint4v*>(residual + (size_t)row * d);
  const uint4v* wr = reinterpret_cast<const uint4v*>(w);
  uint4v* yr = reinterpret_cast<uint4v*>(y + (size_t)row * d);
  float v[kMaxVec][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxVec; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < nvec) {
      unpack8(xr[i], v[k]);
      if (kResidual) {
        float r[8];
        unpack8(rr[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r[j];
        rr[i] = pack8(v[k]);
        // the normalised value is computed from the bf16-rounded sum, as the residual stream holds it
        unpack8(rr[i], v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
#pragma unroll
  for (int k = 0; k < kMaxVec; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < nvec) {
      float wf[8], o[8];
      unpack8(wr[i], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * inv * wf[j];
      yr[i] = pack8(o);
    }
  }
}

// Wave-per-row RMSNorm for the decode rows (d = 64 * 8 * VPL, e.g. 4096 -> VPL = 8): a wave owns a whole
// row, each lane VPL 16-byte vectors (lane-interleaved, so every load / store instruction moves 1 KiB
// contiguous), all loads issued before the first use, and the reduction is a wave reduction — no LDS, no
// workgroup barrier.  The workgroup-per-row kernel above spends most of a 4096-wide row's time in its two
// barriers and a single 16 B load per lane (4.4 TB/s at [4096, 4096]).
// kQuant: the normalised row is also quantised per row to OCP e4m3 for the fp8 projection that consumes it
// (config 5's dense fp8 layers): scale = max|bf16(y)| / 448 over the row, q = e4m3(bf16(y) / scale) —
// exactly quant_fp8_rows(rmsnorm(x)) without writing and re-reading the bf16 row (y may be null then).
template <int VPL, bool kResidual, bool kQuant = false>
__global__ void __launch_bounds__(256) rmsnorm_wave_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
                                                           const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                           int rows, int d, float eps, uint8_t* __restrict__ q = nullptr,
                                                           float* __restrict__ qscale = nullptr) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole waves exit; no barrier below
  const int lane = threadIdx.x & 63;
  const uint4v* xr = reinterpret_cast<const uint4v*>(x + (size_t)row * d);
  uint4v* rr = reinterpret_cast<uint4v*>(residual + (size_t)row * d);
  const uint4v* wr = reinterpret_cast<const uint4v*>(w);
  uint4v* yr = reinterpret_cast<uint4v*>(y + (size_t)row * d);
  uint4v raw[VPL];
#pragma unroll
  for (int k = 0; k < VPL; ++k) raw[k] = xr[lane + 64 * k];
  if (kResidual) {
    uint4v res[VPL];
#pragma unroll
    for (int k = 0; k < VPL; ++k) res[k] = rr[lane + 64 * k];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      float a[8], b[8];
      unpack8(raw[k], a);
      unpack8(res[k], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
      raw[k] = pack8(a);  // the normalised value is computed from the bf16-rounded sum, as the stream holds it
      rr[lane + 64 * k] = raw[k];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    float a[8];
    unpack8(raw[k], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
  const float inv = rsqrtf(wave_sum(ss) / (float)d + eps);
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    float a[8], wf[8], o[8];
    unpack8(raw[k], a);
    unpack8(wr[lane + 64 * k], wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = a[j] * inv * wf[j];
    const uint4v packed = pack8(o);
    if (!kQuant || y != nullptr) yr[lane + 64 * k] = packed;
    if (kQuant) {
      raw[k] = packed;  // keep bf16(y) for the quantisation pass
      float b[8];
      unpack8(packed, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(b[j]));
    }
  }
  if (kQuant) {
    amax = wave_max(amax);
    const float sc = fmaxf(amax, 1e-12f) / 448.f;
    const float qi = 1.f / sc;
    if (lane == 0) qscale[row] = sc;
    uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * d);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      float v[8];
      unpack8(raw[k], v);
      uint32_t lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * qi, v[1] * qi, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * qi, v[3] * qi, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * qi, v[5] * qi, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * qi, v[7] * qi, hi, true);
      qr[lane + 64 * k] = make_uint2(lo, hi);
    }
  }
}

template <int VPL>
static void launch_rmsnorm_wave(const void* x, void* residual, const void* w, void* y, int rows, int d, float eps,
                                hipStream_t s) {
  const dim3 grid((rows + 3) / 4);
  if (residual)
    rmsnorm_wave_kernel<VPL, true><<<grid, 256, 0, s>>>((const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w,
                                                        (bf16_t*)y, rows, d, eps);
  else
    rmsnorm_wave_kernel<VPL, false><<<grid, 256, 0, s>>>((const bf16_t*)x, nullptr, (const bf16_t*)w, (bf16_t*)y,
                                                         rows, d, eps);
}

template <int VPL>
static void launch_rmsnorm_wave_q(const void* x, void* residual, const void* w, void* y, int rows, int d, float eps,
                                  void* q, float* qscale, hipStream_t s) {
  const dim3 grid((rows + 3) / 4);
  if (residual)
    rmsnorm_wave_kernel<VPL, true, true><<<grid, 256, 0, s>>>((const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w,
                                                              (bf16_t*)y, rows, d, eps, (uint8_t*)q, qscale);
  else
    rmsnorm_wave_kernel<VPL, false, true><<<grid, 256, 0, s>>>((const bf16_t*)x, nullptr, (const bf16_t*)w, (bf16_t*)y,
                                                               rows, d, eps, (uint8_t*)q, qscale);
}

// LayerNorm with affine: y = (h - mean)/sqrt(var+eps) * g + b, h = x (+ residual);
// residual (if given) is NOT updated: BERT post-norm writes y back as the new stream.
// pb (optional): a pre-norm bias, h = x (+ residual) + pb — the residual projection's bias when its GEMM
// fused the residual add instead (x then already holds the stream).
template <bool kResidual>
__global__ void __launch_bounds__(1024) layernorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ residual,
                                                        const bf16_t* __restrict__ pb, const bf16_t* __restrict__ g,
                                                        const bf16_t* __restrict__ b, bf16_t* __restrict__ y, int d,
                                                        float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const uint4v* xr = reinterpret_cast<const uint4v*>(x + (size_t)row * d);
  const uint4v* rr = reinterpret_cast<const uint4v*>(residual + (size_t)row * d);
  const uint4v* gr = reinterpret_cast<const uint4v*>(g);
  const uint4v* br = reinterpret_cast<const uint4v*>(b);
  uint4v* yr = reinterpret_cast<uint4v*>(y + (size_t)row * d);
  float v[kMaxVec][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxVec; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < nvec) {
      unpack8(xr[i], v[k]);
      if (kResidual) {
        float r[8];
        unpack8(rr[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r[j];
      }
      if (pb) {
        float c[8];
        unpack8(reinterpret_cast<const uint4v*>(pb)[i], c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += c[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    }
  }
  const float mean = block_sum(s, scratch) / (float)d;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxVec; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = v[k][j] - mean;
        s2 += c * c;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, scratch) / (float)d + eps);
#pragma unroll
  for (int k = 0; k < kMaxVec; ++k) {
    const int i = threadIdx.x + k * blockDim.x;
    if (i < nvec) {
      float gf[8], bf[8], o[8];
      unpack8(gr[i], gf);
      unpack8(br[i], bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * inv * gf[j] + bf[j];
      yr[i] = pack8(o);
    }
  }
}

// LayerNorm for rows of at most 1024 elements (bge-base 768, bge-large 1024): one wave per row, lane l owning
// the row's 16-byte vectors l and l + 64, four rows per 256-thread workgroup, wave shuffles for the two sums
// (no LDS, no block barriers: the one-workgroup-per-row kernel ran 768-wide rows at ~4.9 TB/s).  x and y may
// be the same tensor (every lane loads its vectors before the first shuffle).
template <bool kResidual>
__global__ void __launch_bounds__(256) layernorm_wave_kernel(const bf16_t* x, const bf16_t* __restrict__ residual,
                                                             const bf16_t* __restrict__ pb, const bf16_t* __restrict__ g,
                                                             const bf16_t* __restrict__ b, bf16_t* y, int rows, int d,
                                                             float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nvec = d >> 3;
  const uint4v* xr = reinterpret_cast<const uint4v*>(x + (size_t)row * d);
  const uint4v* rr = reinterpret_cast<const uint4v*>(residual + (size_t)row * d);
  float v[2][8];
  uint4v raw[2], rraw[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      raw[k] = xr[i];
      if (kResidual) rraw[k] = rr[i];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      unpack8(raw[k], v[k]);
      if (kResidual) {
        float r[8];
        unpack8(rraw[k], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r[j];
      }
      if (pb) {
        float c[8];
        unpack8(reinterpret_cast<const uint4v*>(pb)[i], c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += c[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)d;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (lane + 64 * k < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = v[k][j] - mean;
        s2 += c * c;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
  const float inv = rsqrtf(s2 / (float)d + eps);
  uint4v* yr = reinterpret_cast<uint4v*>(y + (size_t)row * d);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      float gf[8], bf[8], o[8];
      unpack8(reinterpret_cast<const uint4v*>(g)[i], gf);
      unpack8(reinterpret_cast<const uint4v*>(b)[i], bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * inv * gf[j] + bf[j];
      yr[i] = pack8(o);
    }
  }
}

// ss[r] = sum(x[r]^2), one wave per row: the (single) partial row sum of squares an RMSNorm folded into the
// next projection (gemm4w RS 1) reads for rows no residual epilogue produced partials for (the embedding rows)
__global__ void __launch_bounds__(256) rms_rowsumsq_kernel(const bf16_t* __restrict__ x, float* __restrict__ ss, int rows,
                                                           int d) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const uint4v* xr = reinterpret_cast<const uint4v*>(x + (size_t)row * d);
  float s = 0.f;
  for (int i = lane; i < (d >> 3); i += 64) {
    float v[8];
    unpack8(xr[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) ss[row] = s;
}

static int norm_threads(int d) {
  // one 16-byte vector per thread when the row allows it (shortest latency per row)
  int nvec = d / 8;
  int t = ((nvec + 63) / 64) * 64;
  if (t < 64) t = 64;
  if (t > 1024) t = 1024;
  return t;
}

}  // namespace lwc

extern "C" int lwc_rmsnorm(const void* x, void* residual, const void* w, void* y, int rows, int d, float eps,
                           hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0 || d > kMaxVec * 8 * 1024) return -1;
  if (rows == 0) return 0;
  if (rows >= 256 && (d == 4096 || d == 2048 || d == 8192)) {  // decode / prefill rows: a wave per row
    if (d == 2048) launch_rmsnorm_wave<4>(x, residual, w, y, rows, d, eps, s);
    else if (d == 4096) launch_rmsnorm_wave<8>(x, residual, w, y, rows, d, eps, s);
    else launch_rmsnorm_wave<16>(x, residual, w, y, rows, d, eps, s);
    return (int)hipGetLastError();
  }
  const int t = norm_threads(d);
  if (residual)
    rmsnorm_kernel<true><<<rows, t, 0, s>>>((const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, (bf16_t*)y, d, eps);
  else
    rmsnorm_kernel<false><<<rows, t, 0, s>>>((const bf16_t*)x, nullptr, (const bf16_t*)w, (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

// RMSNorm (+ residual) with the per-row e4m3 quantisation of its output fused (wave per row; d in
// {2048, 4096, 8192}); y (bf16 output) is optional.  Returns -1 for other widths (the caller runs the two
// kernels).
extern "C" int lwc_rmsnorm_quant_fp8(const void* x, void* residual, const void* w, void* y, int rows, int d, float eps,
                                     void* q, float* qscale, hipStream_t s) {
  using namespace lwc;
  if (d != 2048 && d != 4096 && d != 8192) return -1;
  if (rows == 0) return 0;
  if (d == 2048) launch_rmsnorm_wave_q<4>(x, residual, w, y, rows, d, eps, q, qscale, s);
  else if (d == 4096) launch_rmsnorm_wave_q<8>(x, residual, w, y, rows, d, eps, q, qscale, s);
  else launch_rmsnorm_wave_q<16>(x, residual, w, y, rows, d, eps, q, qscale, s);
  return (int)hipGetLastError();
}

extern "C" int lwc_layernorm(const void* x, const void* residual, const void* pre_bias, const void* g, const void* b,
                             void* y, int rows, int d, float eps, hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0 || d > kMaxVec * 8 * 1024) return -1;
  if (rows == 0) return 0;
  const bf16_t* pb = (const bf16_t*)pre_bias;
  if (d <= 1024) {
    const int grid = (rows + 3) / 4;
    if (residual)
      layernorm_wave_kernel<true><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)residual, pb, (const bf16_t*)g,
                                                       (const bf16_t*)b, (bf16_t*)y, rows, d, eps);
    else
      layernorm_wave_kernel<false><<<grid, 256, 0, s>>>((const bf16_t*)x, nullptr, pb, (const bf16_t*)g,
                                                        (const bf16_t*)b, (bf16_t*)y, rows, d, eps);
    return (int)hipGetLastError();
  }
  if (x == y) return -1;  // the workgroup-per-row kernel is not in-place safe across its vector loop
  const int t = norm_threads(d);
  if (residual)
    layernorm_kernel<true><<<rows, t, 0, s>>>((const bf16_t*)x, (const bf16_t*)residual, pb, (const bf16_t*)g,
                                              (const bf16_t*)b, (bf16_t*)y, d, eps);
  else
    layernorm_kernel<false><<<rows, t, 0, s>>>((const bf16_t*)x, nullptr, pb, (const bf16_t*)g, (const bf16_t*)b,
                                               (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

extern "C" int lwc_rms_rowsumsq(const void* x, float* ss, int rows, int d, hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0) return -1;
  if (rows == 0) return 0;
  rms_rowsumsq_kernel<<<(rows + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ss, rows, d);
  return (int)hipGetLastError();
}
