// K3 paged_attn_decode: one query token per sequence against a paged bf16 KV cache, GQA
// (G = Hq/Hkv query heads per KV head, G <= 16), split-K (flash-decoding) over the context.
//
// Layout (all bf16):
//   q        : [B, q_stride] — head hq at q + b*q_stride + hq*D (q lives inside the fused qkv row)
//   k_cache  : [NB, Hkv, BS, D]          (token-major rows of D)
//   v_cache  : [NB, Hkv, D, BS]          (TRANSPOSED: a column of V = BS contiguous tokens)
//   block_tables [B, max_blocks] int32, ctx_lens [B] int32
//
// MFMA design (mfma_f32_16x16x32_bf16, one wave = 64 lanes, lane l: r16 = l & 15, g = l >> 4):
//   S^T = K Q^T per 16-token block, 4 k-steps over D=128:
//     A (K)  : lane holds K[tok r16][32s + 8g + j]        -> one 16 B load straight from the cache
//     B (Q^T): lane holds Q[head r16][32s + 8g + j]       -> kept in registers for the whole kernel
//     C      : lane reg r = S^T[tok 4g + r][head r16]
//   O = P V per 32 tokens (a PAIR of blocks A,B), k permuted as {A: 4g+0..3, B: 4g+0..3}:
//     A (P)  : exactly the softmaxed S^T_A, S^T_B accumulator registers (no data movement)
//     B (V)  : lane holds V[those 8 tokens][dim 16n + r16] -> two 8 B loads from the transposed cache
//     C      : lane reg r = O[head 4g + r][dim 16n + r16]
// Only the first G of the 16 MFMA rows are real heads: the chip is HBM-bound here (≈25x more
// bytes than MFMA cycles per CU), so the idle rows cost nothing and VALU stays free for the softmax.
#include "common.h"

namespace lwc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

LWC_DEVICE float4v mfma16(const short8& a, const short8& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

constexpr int kD = 128;
constexpr int kBS = 16;
constexpr int kWaves = 4;
constexpr float kLog2e = 1.4426950408889634f;

struct DecodeParams {
  const bf16_t* q;
  const bf16_t* kc;
  const bf16_t* vc;
  const int* block_tables;
  const int* ctx_lens;
  bf16_t* out;          // [B, Hq, D]   (used when num_splits == 1)
  float* part_o;        // [B, Hq, S, D] (num_splits > 1)
  float* part_lse;      // [B, Hq, S]
  int q_stride, Hq, Hkv, G, max_blocks, num_splits;
  float scale;
};

__global__ void __launch_bounds__(256) paged_decode_kernel(DecodeParams p) {
  const int b = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int ctx = p.ctx_lens[b];
  const int nblk_total = (ctx + kBS - 1) / kBS;
  const int per_split = (nblk_total + p.num_splits - 1) / p.num_splits;
  const int blk_begin = split * per_split;
  const int blk_end = min(nblk_total, blk_begin + per_split);
  const int* bt = p.block_tables + (size_t)b * p.max_blocks;

  // Q^T operand (B) for the 4 k-steps; heads >= G are zero rows.
  short8 qf[4];
  {
    const bool valid = r16 < p.G;
    const bf16_t* qh = p.q + (size_t)b * p.q_stride + (size_t)(kvh * p.G + (valid ? r16 : 0)) * kD;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      short8 v = *reinterpret_cast<const short8*>(qh + 32 * s + 8 * g);
      qf[s] = valid ? v : short8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const float sl2 = p.scale * kLog2e;

  float4v o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = float4v{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;  // running max / sum (log2 domain) for head r16

  const size_t kv_head_stride = (size_t)kBS * kD;  // elements per (block, head)
  for (int pair = blk_begin + 2 * wid; pair < blk_end; pair += 2 * kWaves) {
    const int blkA = pair, blkB = pair + 1;
    const bool hasB = blkB < blk_end;
    const int physA = bt[blkA];
    const int physB = hasB ? bt[blkB] : physA;
    const bf16_t* kA = p.kc + ((size_t)physA * p.Hkv + kvh) * kv_head_stride;
    const bf16_t* kB = p.kc + ((size_t)physB * p.Hkv + kvh) * kv_head_stride;
    const bf16_t* vA = p.vc + ((size_t)physA * p.Hkv + kvh) * kv_head_stride;
    const bf16_t* vB = p.vc + ((size_t)physB * p.Hkv + kvh) * kv_head_stride;
    // issue all loads of the pair up front (K: 8 x 16 B, V: 16 x 8 B per lane)
    short8 ka[4], kb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ka[s] = *reinterpret_cast<const short8*>(kA + r16 * kD + 32 * s + 8 * g);
      kb[s] = *reinterpret_cast<const short8*>(kB + r16 * kD + 32 * s + 8 * g);
    }
    short4v va[8], vb[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      va[n] = *reinterpret_cast<const short4v*>(vA + (16 * n + r16) * kBS + 4 * g);
      vb[n] = *reinterpret_cast<const short4v*>(vB + (16 * n + r16) * kBS + 4 * g);
    }
    float4v sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sa = mfma16(ka[s], qf[s], sa);
      sb = mfma16(kb[s], qf[s], sb);
    }
    // scale into the log2 domain + mask tokens past the context
    float pa[4], pb[4];
    float mx = -1e30f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ta = blkA * kBS + 4 * g + r, tb = blkB * kBS + 4 * g + r;
      pa[r] = ta < ctx ? sa[r] * sl2 : -INFINITY;
      pb[r] = (hasB && tb < ctx) ? sb[r] * sl2 : -INFINITY;
      mx = fmaxf(mx, fmaxf(pa[r], pb[r]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = exp2f(m - m_new);
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[r] = exp2f(pa[r] - m_new);
      pb[r] = exp2f(pb[r] - m_new);
      rs += pa[r] + pb[r];
    }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
    // rescale O: O row (4g + r) belongs to head 4g+r, whose alpha lives in lane 4g+r
    float al[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) al[r] = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= al[r];
    // P operand (A): k order {A: 4g+0..3, B: 4g+0..3}
    short8 pf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = (short)f2bf(pa[r]);
      pf[4 + r] = (short)f2bf(pb[r]);
    }
    // cache slots past the context may hold stale/uninitialised bits (possibly NaN): P = 0 there,
    // but 0 * NaN = NaN, so those V elements are zeroed by select, not by arithmetic.
    bool okA[4], okB[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      okA[r] = blkA * kBS + 4 * g + r < ctx;
      okB[r] = hasB && (blkB * kBS + 4 * g + r < ctx);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      short8 vf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vf[r] = okA[r] ? va[n][r] : (short)0;
        vf[4 + r] = okB[r] ? vb[n][r] : (short)0;
      }
      o[n] = mfma16(pf, vf, o[n]);
    }
  }

  // ---- combine the 4 waves through LDS ----
  __shared__ float s_m[kWaves][16], s_l[kWaves][16];
  __shared__ float s_o[kWaves][16][kD + 4];
  if (g == 0) {
    s_m[wid][r16] = m;
    s_l[wid][r16] = l;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[wid][4 * g + r][16 * n + r16] = o[n][r];
  __syncthreads();
  // thread t: head h = t / 16 (< G), dims 8*(t%16) .. +8
  const int t = threadIdx.x;
  const int h = t >> 4, dc = (t & 15) * 8;
  if (h < p.G) {
    float M = -1e30f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, s_m[w][h]);
    float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float f = exp2f(s_m[w][h] - M);
      L += f * s_l[w][h];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f * s_o[w][h][dc + j];
    }
    const int hq = kvh * p.G + h;
    const float inv = L > 0.f ? 1.f / L : 0.f;
    if (p.num_splits == 1) {
      float outv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) outv[j] = acc[j] * inv;
      *reinterpret_cast<uint4v*>(p.out + ((size_t)b * p.Hq + hq) * kD + dc) = pack8(outv);
    } else {
      float* po = p.part_o + (((size_t)b * p.Hq + hq) * p.num_splits + split) * kD + dc;
#pragma unroll
      for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
      if ((t & 15) == 0)
        p.part_lse[((size_t)b * p.Hq + hq) * p.num_splits + split] = L > 0.f ? M + log2f(L) : -INFINITY;
    }
  }
}

// Combine split-K partials: out[b, hq, :] = sum_s 2^(lse_s - LSE) o_s
__global__ void __launch_bounds__(128) paged_decode_reduce_kernel(const float* __restrict__ part_o,
                                                                  const float* __restrict__ part_lse,
                                                                  bf16_t* __restrict__ out, int S) {
  const int bh = blockIdx.x;  // b * Hq + hq
  const int d = threadIdx.x;  // 0..127
  const float* lse = part_lse + (size_t)bh * S;
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, lse[s]);
  float L = 0.f, acc = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < S; ++s) {
      const float f = exp2f(lse[s] - M);
      L += f;
      acc += f * part_o[((size_t)bh * S + s) * kD + d];
    }
  }
  out[(size_t)bh * kD + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

}  // namespace lwc

extern "C" int lwc_paged_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                                const int* ctx_lens, void* out, float* part_o, float* part_lse, int B, int Hq,
                                int Hkv, int D, int BS, int max_blocks, int num_splits, float scale, hipStream_t s) {
  using namespace lwc;
  if (D != kD || BS != kBS || Hq % Hkv != 0 || Hq / Hkv > 16 || num_splits < 1) return -1;
  if (num_splits > 1 && (!part_o || !part_lse)) return -2;
  if (B == 0) return 0;
  DecodeParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, ctx_lens, (bf16_t*)out,
                 part_o, part_lse, q_stride, Hq, Hkv, Hq / Hkv, max_blocks, num_splits, scale};
  paged_decode_kernel<<<dim3(B, Hkv, num_splits), 256, 0, s>>>(p);
  if (num_splits > 1) paged_decode_reduce_kernel<<<B * Hq, kD, 0, s>>>(part_o, part_lse, (bf16_t*)out, num_splits);
  return (int)hipGetLastError();
}
