// Element-wise / data-movement kernels for gfx950:
//   K2  rope_kv_write   : rotate-half RoPE on q and k (in place in the fused qkv buffer) and scatter
//                          k, v into the paged KV cache in the same pass;
//   K5  silu_mul        : SwiGLU  out = silu(gate) * up  over a fused [T, 2F] gate_up buffer;
//   K7  embedding_gather: token ids -> hidden rows;
//   K12 kv_block_copy   : copy-on-write fork of whole KV blocks (all layers, K and V).
// All of them move 16 B per lane (Guideline 13); trig comes from a host-built cos/sin table
// (Appendix B "Element-wise": on-device sin/cos turns RoPE VALU-bound).
#include "common.h"

namespace lwc {

constexpr int kRopeVMax = 4096;  // V row elements staged in LDS (Hkv * D; Llama-3-8B: 1024)

// qkv: [T, (Hq + 2*Hkv) * D]; cos/sin: [max_pos, D/2] f32; K cache [NB, Hkv, BS, D];
// V cache [NB, Hkv, BS/4, D, 4] (4-token interleaved)
__global__ void __launch_bounds__(512) rope_kv_write_kernel(bf16_t* __restrict__ qkv, const int* __restrict__ positions,
                                                           const int* __restrict__ slots, const float* __restrict__ cos_t,
                                                           const float* __restrict__ sin_t, bf16_t* __restrict__ kc,
                                                           bf16_t* __restrict__ vc, int Hq, int Hkv, int D, int BS,
                                                           int rope_q) {
  const int t = blockIdx.x;
  const int half = D >> 1;
  const int vec_per_head_rot = half >> 3;  // threads per head for rotation (8 dims each half)
  const int n_rot = (Hq + Hkv) * vec_per_head_rot;
  const int row_len = (Hq + 2 * Hkv) * D;
  bf16_t* row = qkv + (size_t)t * row_len;
  const int pos = positions[t];
  const int slot = slots ? slots[t] : -1;
  const int blk = slot >= 0 ? slot / BS : 0, off = slot >= 0 ? slot % BS : 0;
  // rope_q = 0 (pure decode steps): q stays un-rotated in qkv — the decode attention kernels rotate it as
  // they load it — and only the k heads are rotated and cached
  for (int i = threadIdx.x + (rope_q ? 0 : Hq * vec_per_head_rot); i < n_rot; i += blockDim.x) {
    const int h = i / vec_per_head_rot;      // 0..Hq+Hkv-1 (q heads then k heads)
    const int c = (i % vec_per_head_rot) * 8;  // first-half dim offset
    bf16_t* hp = row + h * D;
    uint4v* p1 = reinterpret_cast<uint4v*>(hp + c);
    uint4v* p2 = reinterpret_cast<uint4v*>(hp + c + half);
    float x1[8], x2[8], o1[8], o2[8];
    unpack8(*p1, x1);
    unpack8(*p2, x2);
    const float4* cp = reinterpret_cast<const float4*>(cos_t + (size_t)pos * half + c);
    const float4* sp = reinterpret_cast<const float4*>(sin_t + (size_t)pos * half + c);
    float cs[8], sn[8];
    *reinterpret_cast<float4*>(cs) = cp[0];
    *reinterpret_cast<float4*>(cs + 4) = cp[1];
    *reinterpret_cast<float4*>(sn) = sp[0];
    *reinterpret_cast<float4*>(sn + 4) = sp[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = x1[j] * cs[j] - x2[j] * sn[j];
      o2[j] = x2[j] * cs[j] + x1[j] * sn[j];
    }
    const uint4v n1 = pack8(o1), n2 = pack8(o2);
    if (rope_q || slot < 0) {  // k-only (pure decode) steps read k from the cache only: no write-back
      *p1 = n1;
      *p2 = n2;
    }
    if (h >= Hq && slot >= 0) {
      const int kh = h - Hq;
      bf16_t* dst = kc + (((size_t)blk * Hkv + kh) * BS + off) * D;
      *reinterpret_cast<uint4v*>(dst + c) = n1;
      *reinterpret_cast<uint4v*>(dst + c + half) = n2;
    }
  }
  // V is cached 4-token interleaved per block ([NB, Hkv, BS/4, D, 4]) so the decode kernels' P.V MFMA
  // reads 4 consecutive tokens of a dim as one 8 B load (see attention_decode.hip).  One element per
  // thread, consecutive threads = consecutive dims: a wave's 64 stores cover 16 32-byte sectors.
  // The row's V comes in through LDS: 16 B loads (one per 8 dims), then the 2 B stores with consecutive threads
  // on consecutive dims (2 B global loads took 8x the load instructions).
  if (slot >= 0) {
    const bf16_t* vsrc = row + (Hq + Hkv) * D;
    __shared__ uint4v vrow[kRopeVMax / 8];
    const int nv = Hkv * D;
    if (nv <= kRopeVMax) {
      for (int i = threadIdx.x; i < (nv >> 3); i += blockDim.x) vrow[i] = reinterpret_cast<const uint4v*>(vsrc)[i];
      __syncthreads();
    }
    const bf16_t* vl = nv <= kRopeVMax ? reinterpret_cast<const bf16_t*>(vrow) : vsrc;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
      const int vh = i / D, d = i - vh * D;
      vc[((size_t)blk * Hkv + vh) * D * BS + ((off >> 2) * D + d) * 4 + (off & 3)] = vl[i];
    }
  }
}

// x * sigmoid(x) with v_rcp_f32 (1 ulp) instead of the IEEE division sequence (v_div_scale x2, v_div_fmas,
// v_div_fixup around an rcp: ~9 VALU per element in an epilogue of 256 per lane); the result is rounded
// to bf16 (or e4m3) anyway.  x -> -inf: rcp(inf) = 0, x * 0 = -0 as the division gives
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// in: [T, 2F] = [gate | up]; out: [T, F]
// gate of output column c at input column (c / blk) * 2 * blk + c % blk, up at + blk (blk = F: [gate | up]
// halves; blk = 32: the gate/up interleaved weight layout of gemm8p's SwiGLU epilogue)
__global__ void silu_mul_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out, int T, int F, int blk) {
  const int fv = F >> 3;
  const size_t total = (size_t)T * fv;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t t = i / fv;
    const int c = (int)(i % fv) * 8;
    const bf16_t* r = in + t * 2 * F + (c / blk) * 2 * blk + c % blk;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const uint4v*>(r), g);
    unpack8(*reinterpret_cast<const uint4v*>(r + blk), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
    *reinterpret_cast<uint4v*>(out + t * F + c) = pack8(o);
  }
}

// table: [V, d]; ids: [T] (int32); out: [T, d]
__global__ void embedding_gather_kernel(const bf16_t* __restrict__ table, const int* __restrict__ ids,
                                        bf16_t* __restrict__ out, int d, int V) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const uint4v* src = reinterpret_cast<const uint4v*>(table + (size_t)id * d);
  uint4v* dst = reinterpret_cast<uint4v*>(out + (size_t)t * d);
  for (int i = threadIdx.x; i < (d >> 3); i += blockDim.x) dst[i] = src[i];
}

// cache: [L, 2, NB, block_elems]; pairs: [P, 2] (src, dst) int32
__global__ void kv_block_copy_kernel(bf16_t* __restrict__ cache, const int* __restrict__ pairs, int NB,
                                     int64_t block_elems) {
  const int p = blockIdx.x, lk = blockIdx.y;
  const int src = pairs[2 * p], dst = pairs[2 * p + 1];
  bf16_t* base = cache + (size_t)lk * NB * block_elems;
  const uint4v* s = reinterpret_cast<const uint4v*>(base + (size_t)src * block_elems);
  uint4v* d = reinterpret_cast<uint4v*>(base + (size_t)dst * block_elems);
  for (int64_t i = threadIdx.x; i < (block_elems >> 3); i += blockDim.x) d[i] = s[i];
}

// Paged cache rows -> contiguous [n, Hkv*D] K and V (cached-prefix prefill).  One thread per (token, head,
// 8 dims): K is one 16 B load; V (4-token interleaved, 8 B per dim-quad) is 8 x 8 B loads whose token lane
// is extracted.  Neighbouring tokens of a quad share their 32 B sectors through the cache.
__global__ void kv_gather_kernel(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                 const int64_t* __restrict__ slots, bf16_t* __restrict__ ko, bf16_t* __restrict__ vo,
                                 int n, int Hkv, int D, int BS) {
  const int chunks = D >> 3;
  const size_t total = (size_t)n * Hkv * chunks;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % chunks);
    const int h = (int)((i / chunks) % Hkv);
    const size_t t = i / ((size_t)chunks * Hkv);
    const int64_t sl = slots[t];
    const int64_t blk = sl / BS;
    const int off = (int)(sl % BS);
    const size_t head = ((size_t)blk * Hkv + h) * BS * D;  // element offset of (block, head)
    const size_t orow = t * (size_t)Hkv * D + (size_t)h * D + c * 8;
    *reinterpret_cast<uint4v*>(ko + orow) = *reinterpret_cast<const uint4v*>(kc + head + (size_t)off * D + c * 8);
    const bf16_t* vq = vc + head + (size_t)(off >> 2) * D * 4 + (off & 3);  // dim d at vq[4 d]
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)vq[4 * (c * 8 + 2 * e)] | ((uint32_t)vq[4 * (c * 8 + 2 * e + 1)] << 16);
    *reinterpret_cast<uint4v*>(vo + orow) = uint4v{w[0], w[1], w[2], w[3]};
  }
}

static int ew_grid(size_t work, int threads) {
  size_t g = (work + threads - 1) / threads;
  if (g > 4096) g = 4096;  // grid-stride beyond ~16 waves/CU (Guideline 11)
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace lwc

extern "C" int lwc_rope_kv_write(void* qkv, const int* positions, const int* slots, const float* cos_t,
                                 const float* sin_t, void* kc, void* vc, int T, int Hq, int Hkv, int D, int BS,
                                 int rope_q, hipStream_t s) {
  using namespace lwc;
  if (D % 16 != 0 || T <= 0) return T == 0 ? 0 : -1;
  // (320 threads — every rotated pair of a Llama-3 token in one round — measured 27.9 vs 26.3 us at T = 4096;
  // a wave per token with 8 dims per lane, 2 B V stores 32 B apart across lanes, 23.4 vs 10.7 us k-only at
  // T = 3072: the V scatter wants consecutive lanes on consecutive dims)
  // k only: Hkv * D/16 rotations (64 for Llama-3) + the V scatter, 128 threads
  rope_kv_write_kernel<<<T, rope_q ? 256 : 128, 0, s>>>((bf16_t*)qkv, positions, slots, cos_t, sin_t, (bf16_t*)kc,
                                                        (bf16_t*)vc, Hq, Hkv, D, BS, rope_q);
  return (int)hipGetLastError();
}

extern "C" int lwc_silu_mul(const void* in, void* out, int T, int F, int blk, hipStream_t s) {
  using namespace lwc;
  if (blk <= 0) blk = F;
  if (F % 8 != 0 || blk % 8 != 0 || F % blk != 0) return -1;
  if (T == 0) return 0;
  silu_mul_kernel<<<ew_grid((size_t)T * F / 8, 256), 256, 0, s>>>((const bf16_t*)in, (bf16_t*)out, T, F, blk);
  return (int)hipGetLastError();
}

extern "C" int lwc_embedding_gather(const void* table, const int* ids, void* out, int T, int d, int V,
                                    hipStream_t s) {
  using namespace lwc;
  if (d % 8 != 0) return -1;
  if (T == 0) return 0;
  embedding_gather_kernel<<<T, 128, 0, s>>>((const bf16_t*)table, ids, (bf16_t*)out, d, V);
  return (int)hipGetLastError();
}

extern "C" int lwc_kv_gather(const void* kc, const void* vc, const long long* slots, void* ko, void* vo, int n,
                             int Hkv, int D, int BS, hipStream_t s) {
  using namespace lwc;
  if (D % 8 != 0 || BS % 4 != 0) return -1;
  if (n == 0) return 0;
  kv_gather_kernel<<<ew_grid((size_t)n * Hkv * (D / 8), 256), 256, 0, s>>>(
      (const bf16_t*)kc, (const bf16_t*)vc, (const int64_t*)slots, (bf16_t*)ko, (bf16_t*)vo, n, Hkv, D, BS);
  return (int)hipGetLastError();
}

extern "C" int lwc_kv_block_copy(void* cache, const int* pairs, int P, int LK, int NB, long long block_elems,
                                 hipStream_t s) {
  using namespace lwc;
  if (block_elems % 8 != 0) return -1;
  if (P == 0) return 0;
  kv_block_copy_kernel<<<dim3(P, LK), 256, 0, s>>>((bf16_t*)cache, pairs, NB, block_elems);
  return (int)hipGetLastError();
}
