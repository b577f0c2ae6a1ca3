// Scoring kernels (gfx950):
//   K9d  pool_l2norm        : CLS / mean / last-token pooling of encoder states + L2 normalisation;
//   K10a cosine_consensus    : S = E E^T on MFMA (16x16 tiles, one wave each) followed by a row-reduce
//                              + softmax kernel -> per-candidate centrality and consensus weights.
//   K10c knn_topk           : training-table neighbour search — cosine of one query against every table row
//                              and the `top` best rows: per 256-row slab a wave-per-row dot
//                              product into LDS and a block top-k, then the slab winners are merged level by
//                              level (up to 4096 candidates per merging workgroup).
//   K10b vote_tally          : the voter tally of the reference (src/score/completions/client.rs:384-455)
//                              for R requests at once — one workgroup per request, fp64 like the host
//                              tally and in the same summation order, so the results are bitwise equal to
//                              the C++ consensus core.  A single request (~L x C <= 128 x 20 multiply-adds)
//                              stays on the host (a launch costs more than the arithmetic); the serving
//                              path batches the tallies of concurrent requests (score/tally_batch.py).
#include "common.h"

namespace lwc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// hidden: [T, d] (row stride ld); cu_seqlens: [nseq+1]; out_f32: [nseq, d]; out_bf16: [nseq, d] (optional)
// mode: 0 = CLS (first token), 1 = mean, 2 = last token
__global__ void __launch_bounds__(256) pool_l2norm_kernel(const bf16_t* __restrict__ hidden, int ld,
                                                         const int* __restrict__ cu, int d, int mode,
                                                         float* __restrict__ out_f32, bf16_t* __restrict__ out_bf16) {
  __shared__ float scratch[16];
  __shared__ float pooled[4096];
  const int s = blockIdx.x;
  const int t0 = cu[s], t1 = cu[s + 1];
  const int len = t1 - t0;
  float ss = 0.f;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float acc = 0.f;
    if (len > 0) {
      if (mode == 0)
        acc = bf2f(hidden[(size_t)t0 * ld + c]);
      else if (mode == 2)
        acc = bf2f(hidden[(size_t)(t1 - 1) * ld + c]);
      else {
        for (int t = t0; t < t1; ++t) acc += bf2f(hidden[(size_t)t * ld + c]);
        acc /= (float)len;
      }
    }
    pooled[c] = acc;
    ss += acc * acc;
  }
  ss = block_sum(ss, scratch);
  const float inv = ss > 0.f ? rsqrtf(ss) : 0.f;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    const float v = pooled[c] * inv;
    out_f32[(size_t)s * d + c] = v;
    if (out_bf16) out_bf16[(size_t)s * d + c] = f2bf(v);
  }
}

// E: [R, n, d] bf16 (rows L2-normalised); S: [R, n_pad, n_pad] f32, n_pad = round_up(n, 16)
__global__ void __launch_bounds__(64) cosine_tiles_kernel(const bf16_t* __restrict__ E, int n, int d,
                                                          float* __restrict__ S, int n_pad) {
  const int ti = blockIdx.x, tj = blockIdx.y, r = blockIdx.z;
  const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
  const bf16_t* Er = E + (size_t)r * n * d;
  const int ri = ti * 16 + r16, rj = tj * 16 + r16;
  float4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < d; k0 += 32) {
    short8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ri < n) a = *reinterpret_cast<const short8*>(Er + (size_t)ri * d + k0 + 8 * g);
    if (rj < n) b = *reinterpret_cast<const short8*>(Er + (size_t)rj * d + k0 + 8 * g);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
  }
  float* Sr = S + (size_t)r * n_pad * n_pad;
#pragma unroll
  for (int q = 0; q < 4; ++q) Sr[(size_t)(ti * 16 + 4 * g + q) * n_pad + tj * 16 + r16] = acc[q];
}

// per request: centrality_i = mean_{j != i} S_ij ; weights = softmax(centrality / tau); best = argmax
__global__ void __launch_bounds__(256) consensus_reduce_kernel(const float* __restrict__ S, int n, int n_pad,
                                                              float inv_tau, float* __restrict__ centrality,
                                                              float* __restrict__ weights, int* __restrict__ best) {
  __shared__ float scratch[16];
  __shared__ float cen[1024];
  const int r = blockIdx.x;
  const float* Sr = S + (size_t)r * n_pad * n_pad;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < n; ++j) s += (j == i) ? 0.f : Sr[(size_t)i * n_pad + j];
    const float c = n > 1 ? s / (float)(n - 1) : 1.f;
    cen[i] = c;
    centrality[(size_t)r * n + i] = c;
    mx = fmaxf(mx, c * inv_tau);
  }
  mx = block_max(mx, scratch);
  float se = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) se += __expf(cen[i] * inv_tau - mx);
  se = block_sum(se, scratch);
  for (int i = threadIdx.x; i < n; i += blockDim.x) weights[(size_t)r * n + i] = __expf(cen[i] * inv_tau - mx) / se;
  if (threadIdx.x == 0) {
    int bi = 0;
    for (int i = 1; i < n; ++i)
      if (cen[i] > cen[bi]) bi = i;
    best[r] = bi;
  }
}

// ---- K10c: top-k rows of E [n, d] f32 by dot product with q [d] --------------------------------------
constexpr int kKnnRows = 256;  // rows per slab (one workgroup)
constexpr int kKnnMaxK = 64;

// The k largest of vals[0..m) (LDS), in order, ties to the lower index; consumed entries become -inf.
// Writes (value, index from idx[] or the position) to out_v / out_i.  256 threads.
LWC_DEVICE void block_topk(float* vals, const int* idx, int m, int k, float* out_v, int* out_i, float* red_v,
                           int* red_i) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int r = 0; r < k; ++r) {
    float bv = -INFINITY;
    int bp = 0x7fffffff;
    for (int i = tid; i < m; i += 256) {
      const float v = vals[i];
      if (v > bv) {  // strided walk: the first hit of a value is this thread's lowest position
        bv = v;
        bp = i;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int op = __shfl_xor(bp, o, 64);
      if (ov > bv || (ov == bv && op < bp)) {
        bv = ov;
        bp = op;
      }
    }
    if (lane == 0) {
      red_v[wid] = bv;
      red_i[wid] = bp;
    }
    __syncthreads();
    if (tid == 0) {
      float v = red_v[0];
      int pidx = red_i[0];
      for (int w = 1; w < 4; ++w)
        if (red_v[w] > v || (red_v[w] == v && red_i[w] < pidx)) {
          v = red_v[w];
          pidx = red_i[w];
        }
      out_v[r] = v;
      out_i[r] = pidx < m ? (idx ? idx[pidx] : pidx) : -1;
      if (pidx < m) vals[pidx] = -INFINITY;
    }
    __syncthreads();
  }
}

// slab s: rows [256 s, 256 s + 256): one wave per row at a time, float4 loads along d
__global__ void __launch_bounds__(256) knn_slab_kernel(const float* __restrict__ E, int n, int d,
                                                       const float* __restrict__ q, int k, float* __restrict__ part_v,
                                                       int* __restrict__ part_i) {
  __shared__ float sims[kKnnRows];
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  const int s = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r0 = s * kKnnRows;
  for (int rr = wid; rr < kKnnRows; rr += 4) {
    const int row = r0 + rr;
    float acc = 0.f;
    if (row < n) {
      const float4v* e = reinterpret_cast<const float4v*>(E + (size_t)row * d);
      const float4v* qq = reinterpret_cast<const float4v*>(q);
      for (int c = lane; c < d / 4; c += 64) {
        const float4v a = e[c], b = qq[c];
        acc += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
      }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sims[rr] = row < n ? acc : -INFINITY;
  }
  __syncthreads();
  __shared__ float out_v[kKnnMaxK];
  __shared__ int out_i[kKnnMaxK];
  block_topk(sims, nullptr, kKnnRows, k, out_v, out_i, red_v, red_i);
  for (int r = threadIdx.x; r < k; r += 256) {
    part_v[(size_t)s * k + r] = out_v[r];
    part_i[(size_t)s * k + r] = out_i[r] >= 0 ? r0 + out_i[r] : -1;
  }
}

// merge: each workgroup takes the winners of `group` consecutive lists of k (list-major = row order, so
// ties still resolve to the lower row) and writes its k best; the host repeats until one list is left
constexpr int kKnnMergeMax = 4096;  // entries per merging workgroup (32 KiB of LDS)
__global__ void __launch_bounds__(256) knn_merge_kernel(const float* __restrict__ in_v, const int* __restrict__ in_i,
                                                        int m, int k, int group, float* __restrict__ out_vals,
                                                        int* __restrict__ out_rows) {
  __shared__ float v[kKnnMergeMax];
  __shared__ int ix[kKnnMergeMax];
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  __shared__ float out_v[kKnnMaxK];
  __shared__ int out_i[kKnnMaxK];
  const int base = blockIdx.x * group * k;
  const int cnt = min(group * k, m - base);
  for (int i = threadIdx.x; i < cnt; i += 256) {
    v[i] = in_i[base + i] >= 0 ? in_v[base + i] : -INFINITY;
    ix[i] = in_i[base + i];
  }
  __syncthreads();
  block_topk(v, ix, cnt, k, out_v, out_i, red_v, red_i);
  for (int r = threadIdx.x; r < k; r += 256) {
    out_vals[(size_t)blockIdx.x * k + r] = out_v[r];
    out_rows[(size_t)blockIdx.x * k + r] = out_i[r];
  }
}

// ---- K10b: batched vote tally ---------------------------------------------------------------------
// V: [R, L, C] f64 (padded choices are 0), w: [R, L] f64, valid: [R, L] u8 (0 = the voter has no vote:
// errored or padding).  cw / conf: [R, C], vconf: [R, L] (NaN where !valid).
// cw[c] = sum_l w_l V[l, c] (l ascending); conf = cw / sum_c cw (0 when the sum is not > 0);
// vconf[l] = sum_c conf[c] V[l, c] (c ascending) — the host tally's order, term for term.
constexpr int kTallyMaxC = 1024;
__global__ void __launch_bounds__(256) vote_tally_kernel(const double* __restrict__ V, const double* __restrict__ w,
                                                         const unsigned char* __restrict__ valid, int L, int C,
                                                         double* __restrict__ cw, double* __restrict__ conf,
                                                         double* __restrict__ vconf) {
#pragma clang fp contract(off)  // separate multiply and add roundings, as the host tally computes them
  __shared__ double s_cw[kTallyMaxC];
  __shared__ double s_sum;
  const int r = blockIdx.x;
  const double* Vr = V + (size_t)r * L * C;
  const double* wr = w + (size_t)r * L;
  const unsigned char* ok = valid + (size_t)r * L;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double acc = 0.0;
    for (int l = 0; l < L; ++l)
      if (ok[l]) acc += Vr[(size_t)l * C + c] * wr[l];
    s_cw[c] = acc;
    cw[(size_t)r * C + c] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int c = 0; c < C; ++c) s += s_cw[c];
    s_sum = s;
  }
  __syncthreads();
  const double sum = s_sum;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const double v = sum > 0.0 ? s_cw[c] / sum : 0.0;
    conf[(size_t)r * C + c] = v;
    s_cw[c] = v;  // each thread touches only its own entries: no barrier before this overwrite
  }
  __syncthreads();
  for (int l = threadIdx.x; l < L; l += blockDim.x) {
    double a = __builtin_nan("");
    if (ok[l]) {
      a = 0.0;
      for (int c = 0; c < C; ++c) a += s_cw[c] * Vr[(size_t)l * C + c];
    }
    vconf[(size_t)r * L + l] = a;
  }
}

}  // namespace lwc

extern "C" int lwc_vote_tally(const double* V, const double* w, const unsigned char* valid, int R, int L, int C,
                              double* cw, double* conf, double* vconf, hipStream_t s) {
  using namespace lwc;
  if (C < 1 || C > kTallyMaxC || L < 0) return -1;
  if (R == 0) return 0;
  vote_tally_kernel<<<R, 256, 0, s>>>(V, w, valid, L, C, cw, conf, vconf);
  return (int)hipGetLastError();
}

// part_v / part_i: scratch of 2 * slabs * k entries (ping-pong between merge levels)
extern "C" int lwc_knn_topk(const float* E, int n, int d, const float* q, int k, float* part_v, int* part_i,
                            float* vals, int* rows, hipStream_t s) {
  using namespace lwc;
  if (d % 4 != 0 || k < 1 || k > kKnnMaxK || k > n) return -1;
  const int slabs = (n + kKnnRows - 1) / kKnnRows;
  int m = slabs * k;
  knn_slab_kernel<<<slabs, 256, 0, s>>>(E, n, d, q, k, part_v, part_i);
  const int group = kKnnMergeMax / k;  // >= 64 lists per merging workgroup
  float* src_v = part_v;
  int* src_i = part_i;
  float* dst_v = part_v + (size_t)slabs * k;
  int* dst_i = part_i + (size_t)slabs * k;
  while (true) {
    const int lists = m / k;
    const int blocks = (lists + group - 1) / group;
    float* ov = blocks == 1 ? vals : dst_v;
    int* oi = blocks == 1 ? rows : dst_i;
    knn_merge_kernel<<<blocks, 256, 0, s>>>(src_v, src_i, m, k, group, ov, oi);
    if (blocks == 1) break;
    m = blocks * k;
    float* tv = src_v;
    int* ti = src_i;
    src_v = dst_v;
    src_i = dst_i;
    dst_v = tv;
    dst_i = ti;
  }
  return (int)hipGetLastError();
}

extern "C" int lwc_pool_l2norm(const void* hidden, int ld, const int* cu, int nseq, int d, int mode, float* out_f32,
                               void* out_bf16, hipStream_t s) {
  using namespace lwc;
  if (d > 4096) return -1;
  if (nseq == 0) return 0;
  pool_l2norm_kernel<<<nseq, 256, 0, s>>>((const bf16_t*)hidden, ld, cu, d, mode, out_f32, (bf16_t*)out_bf16);
  return (int)hipGetLastError();
}

extern "C" int lwc_cosine_consensus(const void* E, int R, int n, int d, float* S, float inv_tau, float* centrality,
                                    float* weights, int* best, hipStream_t s) {
  using namespace lwc;
  if (d % 32 != 0 || n > 1024) return -1;
  if (R == 0 || n == 0) return 0;
  const int nt = (n + 15) / 16, n_pad = nt * 16;
  cosine_tiles_kernel<<<dim3(nt, nt, R), 64, 0, s>>>((const bf16_t*)E, n, d, S, n_pad);
  consensus_reduce_kernel<<<R, 256, 0, s>>>(S, n, n_pad, inv_tau, centrality, weights, best);
  return (int)hipGetLastError();
}

