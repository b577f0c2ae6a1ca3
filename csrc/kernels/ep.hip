// C4 expert-parallel dispatch / combine around the all-to-all (parallel/expert.py, padded mode).
//
// The MoE layer under EP: this rank routes its tokens (moe_route: expert-sorted rows, expert segments
// row_off[E+1]); rank r owns experts [r*El, (r+1)*El), so the sorted rows are also destination-sorted.
// Exchange buffer [W][C + 1 slots][RB bytes] (C = the capacity every rank agrees on):
//   slot 0 of chunk r = header: El int32 row counts, one per expert of rank r;
//   slots 1..C        = rows: payload (row_bytes, bf16 or e4m3 bytes) then, with scales, the row's f32
//                       scale at byte row_bytes; RB = round16(row_bytes + 4 * has_scale).
// One exchange moves rows, fp8 scales and counts together (no separate count all-to-all, no host sync).
//
//   ep_pack       : chunk r <- the sorted rows of rank r's experts, gathered straight from the token rows
//                   through src_row (no separate gather), header = counts, unused slots zeroed.
//   (all-to-all)
//   ep_unpack     : received (source s, slot i) -> expert-major position among this rank's rows: a row of
//                   local expert e from source s lands after every row of experts < e (all sources) and
//                   after expert e's rows from sources < s.  Writes the expert-major rows (+ scales), the
//                   local segments row_off_local[El+1] the grouped GEMM reads, and map[s*C+i] (its
//                   position, -1 for an unused slot).  Counts that cannot be real (a peer that never
//                   arrived poisons its chunk with all-ones bytes: -1) zero that source's chunk, so no index
//                   leaves the buffers; its CommFailure comes from the all-to-all's error word.
//   (grouped expert GEMMs)
//   ep_back       : back[s][i] = expert output of received (s, i) (zero for unused slots).
//   (all-to-all)
//   ep_combine    : out[t] = sum_j w[t, j] * ret[owner(p) * C + p - base(owner)], p = inv[t*k + j]: the
//                   MoE weighted combine reading the returned rows in place (no un-permute copy).
// Six launches besides the GEMMs (pack, exchange, unpack, back, exchange, combine) where the torch glue
// they replace issued ~20 index / scatter / searchsorted kernels per layer.
#include "common.h"

namespace lwc {

constexpr int kEpMaxCounts = 64;  // W * El (e.g. 8 ranks x 8 experts)

struct EpGeo {
  int W, El, C, RB, row_bytes, has_scale;
};

LWC_DEVICE void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int n) {
  for (int c = threadIdx.x * 16; c < n; c += blockDim.x * 16)
    *reinterpret_cast<uint4v*>(dst + c) = *reinterpret_cast<const uint4v*>(src + c);
}

LWC_DEVICE void zero_bytes(uint8_t* __restrict__ dst, int n) {
  for (int c = threadIdx.x * 16; c < n; c += blockDim.x * 16) *reinterpret_cast<uint4v*>(dst + c) = uint4v{0, 0, 0, 0};
}

// grid (C + 1, W)
__global__ void __launch_bounds__(256) ep_pack_kernel(const uint8_t* __restrict__ x, const float* __restrict__ xs,
                                                      const int* __restrict__ src, const int* __restrict__ row_off,
                                                      EpGeo g, uint8_t* __restrict__ send) {
  const int slot = blockIdx.x, r = blockIdx.y;
  uint8_t* dst = send + ((size_t)r * (g.C + 1) + slot) * g.RB;
  const int base = row_off[r * g.El], n = row_off[(r + 1) * g.El] - base;
  if (slot == 0) {
    zero_bytes(dst, g.RB);
    __syncthreads();
    for (int e = threadIdx.x; e < g.El; e += blockDim.x)
      reinterpret_cast<int*>(dst)[e] = row_off[r * g.El + e + 1] - row_off[r * g.El + e];
    return;
  }
  const int j = slot - 1;
  if (j >= n) {
    zero_bytes(dst, g.RB);
    return;
  }
  const int p = base + j;
  const int row = src != nullptr ? src[p] : p;
  copy_bytes(dst, x + (size_t)row * g.row_bytes, g.row_bytes);
  if (g.has_scale && threadIdx.x == 0) *reinterpret_cast<float*>(dst + g.row_bytes) = xs[row];
}

// Per-(source, expert) counts of the received headers, sanitised, with the expert-major and chunk-internal
// offsets (every block recomputes them: W * El <= 64 values).
struct EpCounts {
  int cnt[kEpMaxCounts], em[kEpMaxCounts], cum[kEpMaxCounts], tot[8 * kEpMaxCounts / 8];
};

LWC_DEVICE void ep_counts(const uint8_t* __restrict__ recv, const EpGeo& g, EpCounts& s) {
  const int n = g.W * g.El;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const int src = t / g.El, e = t % g.El;
    s.cnt[t] = reinterpret_cast<const int*>(recv + (size_t)src * (g.C + 1) * g.RB)[e];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int src = 0; src < g.W; ++src) {
      long long sum = 0;
      bool bad = false;
      for (int e = 0; e < g.El; ++e) {
        const int c = s.cnt[src * g.El + e];
        bad |= c < 0;
        sum += c;
      }
      bad |= sum > g.C;
      int acc = 0;
      for (int e = 0; e < g.El; ++e) {
        if (bad) s.cnt[src * g.El + e] = 0;
        s.cum[src * g.El + e] = acc;
        acc += s.cnt[src * g.El + e];
      }
      s.tot[src] = acc;
    }
    int acc = 0;  // expert-major: expert e's rows from source 0, 1, ... after every row of experts < e
    for (int e = 0; e < g.El; ++e)
      for (int src = 0; src < g.W; ++src) {
        s.em[src * g.El + e] = acc;
        acc += s.cnt[src * g.El + e];
      }
  }
  __syncthreads();
}

// grid (C, W): block = received (source blockIdx.y, row slot blockIdx.x)
__global__ void __launch_bounds__(256) ep_unpack_kernel(const uint8_t* __restrict__ recv, EpGeo g,
                                                        uint8_t* __restrict__ x_local, float* __restrict__ s_local,
                                                        int* __restrict__ map, int* __restrict__ row_off_local) {
  __shared__ EpCounts s;
  ep_counts(recv, g, s);
  const int i = blockIdx.x, src = blockIdx.y;
  if (i == 0 && src == 0 && threadIdx.x == 0) {
    int acc = 0;
    row_off_local[0] = 0;
    for (int e = 0; e < g.El; ++e) {
      for (int q = 0; q < g.W; ++q) acc += s.cnt[q * g.El + e];
      row_off_local[e + 1] = acc;
    }
  }
  if (i >= s.tot[src]) {
    if (threadIdx.x == 0) map[src * g.C + i] = -1;
    return;
  }
  int e = 0;
  while (e + 1 < g.El && i >= s.cum[src * g.El + e + 1]) ++e;
  const int dest = s.em[src * g.El + e] + (i - s.cum[src * g.El + e]);
  const uint8_t* row = recv + ((size_t)src * (g.C + 1) + 1 + i) * g.RB;
  copy_bytes(x_local + (size_t)dest * g.row_bytes, row, g.row_bytes);
  if (threadIdx.x == 0) {
    map[src * g.C + i] = dest;
    if (g.has_scale) s_local[dest] = *reinterpret_cast<const float*>(row + g.row_bytes);
  }
}

// grid (C, W): back[src][i] = y_local[map[src*C+i]] (out_bytes per row), zeros for unused slots
__global__ void __launch_bounds__(256) ep_back_kernel(const uint8_t* __restrict__ y_local, const int* __restrict__ map,
                                                      int C, int out_bytes, uint8_t* __restrict__ back) {
  const int i = blockIdx.x, src = blockIdx.y;
  const int m = map[src * C + i];
  uint8_t* dst = back + ((size_t)src * C + i) * out_bytes;
  if (m < 0)
    zero_bytes(dst, out_bytes);
  else
    copy_bytes(dst, y_local + (size_t)m * out_bytes, out_bytes);
}

// one workgroup per token; ret [W*C, d] bf16 (rows as this rank sent them, returned with expert outputs)
__global__ void __launch_bounds__(256) ep_combine_kernel(const bf16_t* __restrict__ ret, const int* __restrict__ row_off,
                                                         const int* __restrict__ inv, const float* __restrict__ w,
                                                         int E, int El, int C, int k, int d, bf16_t* __restrict__ out) {
  const int t = blockIdx.x;
  __shared__ size_t s_row[8];
  if (threadIdx.x < k) {
    const int p = inv[t * k + threadIdx.x];
    int e = 0;
    while (e + 1 < E && p >= row_off[e + 1]) ++e;
    const int r = e / El;
    s_row[threadIdx.x] = (size_t)r * C + (p - row_off[r * El]);
  }
  __syncthreads();
  for (int c = threadIdx.x * 8; c < d; c += blockDim.x * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = w[t * k + j];
      float y[8];
      unpack8(*reinterpret_cast<const uint4v*>(ret + s_row[j] * d + c), y);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * y[q];
    }
    *reinterpret_cast<uint4v*>(out + (size_t)t * d + c) = pack8(acc);
  }
}

}  // namespace lwc

namespace {
bool ep_geo_ok(int W, int El, int C, int RB, int row_bytes, int has_scale) {
  return W >= 1 && W <= 8 && El >= 1 && W * El <= lwc::kEpMaxCounts && C >= 1 && row_bytes % 16 == 0 && RB % 16 == 0 &&
         RB >= row_bytes + 4 * has_scale && RB >= El * 4;
}
}  // namespace

extern "C" int lwc_ep_pack(const void* x, const float* xs, const int* src, const int* row_off, int W, int El, int C,
                           int RB, int row_bytes, void* send, hipStream_t s) {
  if (!ep_geo_ok(W, El, C, RB, row_bytes, xs != nullptr)) return -1;
  lwc::EpGeo g{W, El, C, RB, row_bytes, xs != nullptr};
  lwc::ep_pack_kernel<<<dim3(C + 1, W), 256, 0, s>>>((const uint8_t*)x, xs, src, row_off, g, (uint8_t*)send);
  return (int)hipGetLastError();
}

extern "C" int lwc_ep_unpack(const void* recv, int W, int El, int C, int RB, int row_bytes, int has_scale,
                             void* x_local, float* s_local, int* map, int* row_off_local, hipStream_t s) {
  if (!ep_geo_ok(W, El, C, RB, row_bytes, has_scale) || (has_scale && !s_local)) return -1;
  lwc::EpGeo g{W, El, C, RB, row_bytes, has_scale};
  lwc::ep_unpack_kernel<<<dim3(C, W), 256, 0, s>>>((const uint8_t*)recv, g, (uint8_t*)x_local, s_local, map,
                                                   row_off_local);
  return (int)hipGetLastError();
}

extern "C" int lwc_ep_back(const void* y_local, const int* map, int W, int C, int out_bytes, void* back,
                           hipStream_t s) {
  if (W < 1 || C < 1 || out_bytes % 16 != 0) return -1;
  lwc::ep_back_kernel<<<dim3(C, W), 256, 0, s>>>((const uint8_t*)y_local, map, C, out_bytes, (uint8_t*)back);
  return (int)hipGetLastError();
}

extern "C" int lwc_ep_combine(const void* ret, const int* row_off, const int* inv, const float* w, int T, int E,
                              int El, int C, int k, int d, void* out, hipStream_t s) {
  if (k < 1 || k > 8 || d % 8 != 0 || El < 1 || E % El != 0) return -1;
  if (T == 0) return 0;
  lwc::ep_combine_kernel<<<T, 256, 0, s>>>((const lwc::bf16_t*)ret, row_off, inv, w, E, El, C, k, d,
                                           (lwc::bf16_t*)out);
  return (int)hipGetLastError();
}
