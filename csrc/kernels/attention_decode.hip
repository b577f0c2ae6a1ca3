// K3 paged_attn_decode: one query token per sequence against a paged bf16 KV cache, GQA
// (G = Hq/Hkv query heads per KV head, G <= 16), split-K (flash-decoding) over the context, and a
// PREFIX-SHARED (cascade) mode for sequences forked from one prompt.
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
//     B (Q^T): lane holds Q[row r16][32s + 8g + j]        -> kept in registers for the whole kernel
//     C      : lane reg r = S^T[tok 4g + r][row r16]
//   O = P V per 32 tokens (a PAIR of blocks A,B), k permuted as {A: 4g+0..3, B: 4g+0..3}:
//     A (P)  : exactly the softmaxed S^T_A, S^T_B accumulator registers (no data movement)
//     B (V)  : lane holds V[those 8 tokens][dim 16n + r16] -> two 8 B loads from the transposed cache
//     C      : lane reg r = O[row 4g + r][dim 16n + r16]
// The 16 MFMA rows are "query rows".  Plain decode: row = a query head of ONE sequence (only G of 16
// rows are real — the op is HBM-bound so idle rows cost nothing).  Prefix mode: the n sequences that
// share a prompt are packed 16/G per wave-tile, row = (sequence, head), and the shared prompt blocks
// are read ONCE per tile instead of once per sequence: for N candidates of one prompt this removes
// (N-1)/N of the prompt's KV traffic and finally uses the MFMA rows.  The suffix pass (each
// sequence's own blocks) merges the prefix partial (o, lse) in its epilogue.
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
  bf16_t* out;          // [B, Hq, D]   (suffix/plain with num_splits == 1)
  float* part_o;        // [B, Hq, S, D] (num_splits > 1)
  float* part_lse;      // [B, Hq, S]
  // prefix sharing
  const int* tiles;     // [max_tiles, 3] (row_start, nseq, prefix_blocks); prefix pass only
  const int* start_blk; // [B] first block of the suffix pass (0 = no prefix partial to merge)
  float* pre_o;         // [B, Hq, D] normalised prefix partial
  float* pre_lse;       // [B, Hq]    its log2-sum-exp
  int q_stride, Hq, Hkv, G, max_blocks, num_splits, num_tiles;
  float scale;
};

// PREFIX=true : blockIdx.x = tile;  PREFIX=false: blockIdx.x = sequence
template <bool PREFIX>
__global__ void __launch_bounds__(256) paged_decode_kernel(DecodeParams p) {
  const int item = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;

  int row_seq0, nrows, blk_begin, blk_end, ctx;
  if (PREFIX) {
    if (item >= p.num_tiles) return;
    const int* t = p.tiles + 3 * item;
    row_seq0 = t[0];
    nrows = t[1] * p.G;
    blk_begin = 0;
    blk_end = t[2];
    ctx = blk_end * kBS;
  } else {
    row_seq0 = item;
    nrows = p.G;
    ctx = p.ctx_lens[item];
    const int nblk_total = (ctx + kBS - 1) / kBS;
    const int b0 = p.start_blk ? p.start_blk[item] : 0;
    const int per_split = (nblk_total - b0 + p.num_splits - 1) / p.num_splits;
    blk_begin = b0 + split * per_split;
    blk_end = min(nblk_total, blk_begin + per_split);
  }
  // row -> (sequence, query head)
  auto row_seq = [&](int row) { return PREFIX ? row_seq0 + row / p.G : row_seq0; };
  auto row_head = [&](int row) { return kvh * p.G + (PREFIX ? row % p.G : row); };
  const int* bt = p.block_tables + (size_t)row_seq0 * p.max_blocks;  // prefix blocks are shared by the tile

  // Q^T operand (B) for the 4 k-steps; rows >= nrows are zero.
  short8 qf[4];
  {
    const bool valid = r16 < nrows;
    const int rr = valid ? r16 : 0;
    const bf16_t* qh = p.q + (size_t)row_seq(rr) * p.q_stride + (size_t)row_head(rr) * kD;
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
  float m = -1e30f, l = 0.f;  // running max / sum (log2 domain) for row r16

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
    // rescale O: O row (4g + r) belongs to row 4g+r, whose alpha lives in lane 4g+r
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
  __shared__ float s_m[kWaves + 1][16], s_l[kWaves + 1][16];
  __shared__ float s_o[kWaves + 1][16][kD + 4];
  if (g == 0) {
    s_m[wid][r16] = m;
    s_l[wid][r16] = l;
  }
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[wid][4 * g + r][16 * n + r16] = o[n][r];
  __syncthreads();
  // thread t: row h = t / 16 (< nrows), dims 8*(t%16) .. +8
  const int t = threadIdx.x;
  const int h = t >> 4, dc = (t & 15) * 8;
  if (h < nrows) {
    const int seq = row_seq(h), hq = row_head(h);
    int nparts = kWaves;
    // suffix/plain pass with one split: the prefix partial joins as a 5th "wave" (m = lse, l = 1)
    const bool merge_prefix = !PREFIX && p.num_splits == 1 && p.start_blk && p.start_blk[seq] > 0;
    if (merge_prefix) {
      s_m[kWaves][h] = p.pre_lse[(size_t)seq * p.Hq + hq];
      s_l[kWaves][h] = 1.f;
      const float* po = p.pre_o + ((size_t)seq * p.Hq + hq) * kD + dc;
#pragma unroll
      for (int j = 0; j < 8; ++j) s_o[kWaves][h][dc + j] = po[j];
      nparts = kWaves + 1;
    }
    float M = -1e30f;
    for (int w = 0; w < nparts; ++w) M = fmaxf(M, s_m[w][h]);
    float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < nparts; ++w) {
      const float f = exp2f(s_m[w][h] - M);
      L += f * s_l[w][h];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f * s_o[w][h][dc + j];
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    if (PREFIX) {
      float* po = p.pre_o + ((size_t)seq * p.Hq + hq) * kD + dc;
#pragma unroll
      for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
      if ((t & 15) == 0) p.pre_lse[(size_t)seq * p.Hq + hq] = L > 0.f ? M + log2f(L) : -INFINITY;
    } else if (p.num_splits == 1) {
      float outv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) outv[j] = acc[j] * inv;
      *reinterpret_cast<uint4v*>(p.out + ((size_t)seq * p.Hq + hq) * kD + dc) = pack8(outv);
    } else {
      float* po = p.part_o + (((size_t)seq * p.Hq + hq) * p.num_splits + split) * kD + dc;
#pragma unroll
      for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
      if ((t & 15) == 0)
        p.part_lse[((size_t)seq * p.Hq + hq) * p.num_splits + split] = L > 0.f ? M + log2f(L) : -INFINITY;
    }
  }
}

// Combine split-K partials (+ the prefix partial): out[b, hq, :] = sum_s 2^(lse_s - LSE) o_s
__global__ void __launch_bounds__(128) paged_decode_reduce_kernel(const float* __restrict__ part_o,
                                                                  const float* __restrict__ part_lse,
                                                                  const int* __restrict__ start_blk,
                                                                  const float* __restrict__ pre_o,
                                                                  const float* __restrict__ pre_lse,
                                                                  bf16_t* __restrict__ out, int S, int Hq) {
  const int bh = blockIdx.x;  // b * Hq + hq
  const int d = threadIdx.x;  // 0..127
  const bool pre = start_blk && start_blk[bh / Hq] > 0;
  const float* lse = part_lse + (size_t)bh * S;
  float M = pre ? pre_lse[bh] : -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, lse[s]);
  float L = 0.f, acc = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < S; ++s) {
      const float f = exp2f(lse[s] - M);
      L += f;
      acc += f * part_o[((size_t)bh * S + s) * kD + d];
    }
    if (pre) {
      const float f = exp2f(pre_lse[bh] - M);
      L += f;
      acc += f * pre_o[(size_t)bh * kD + d];
    }
  }
  out[(size_t)bh * kD + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

}  // namespace lwc

// Plain / suffix decode.  start_blk, pre_o, pre_lse may be null (no prefix sharing).
extern "C" int lwc_paged_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                                const int* ctx_lens, void* out, float* part_o, float* part_lse, int B, int Hq,
                                int Hkv, int D, int BS, int max_blocks, int num_splits, float scale,
                                const int* start_blk, const float* pre_o, const float* pre_lse, hipStream_t s) {
  using namespace lwc;
  if (D != kD || BS != kBS || Hq % Hkv != 0 || Hq / Hkv > 16 || num_splits < 1) return -1;
  if (num_splits > 1 && (!part_o || !part_lse)) return -2;
  if (start_blk && (!pre_o || !pre_lse)) return -3;
  if (B == 0) return 0;
  DecodeParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, ctx_lens, (bf16_t*)out,
                 part_o, part_lse, nullptr, start_blk, (float*)pre_o, (float*)pre_lse, q_stride, Hq, Hkv, Hq / Hkv,
                 max_blocks, num_splits, 0, scale};
  paged_decode_kernel<false><<<dim3(B, Hkv, num_splits), 256, 0, s>>>(p);
  if (num_splits > 1)
    paged_decode_reduce_kernel<<<B * Hq, kD, 0, s>>>(part_o, part_lse, start_blk, pre_o, pre_lse, (bf16_t*)out,
                                                     num_splits, Hq);
  return (int)hipGetLastError();
}

// Prefix pass: one workgroup per (tile, kv head); tiles = [max_tiles, 3] (row_start, nseq, prefix_blocks),
// the first `num_tiles` valid; nseq * G <= 16.  Writes pre_o / pre_lse for the tiles' rows.
extern "C" int lwc_paged_decode_prefix(const void* q, int q_stride, const void* kc, const void* vc,
                                       const int* block_tables, const int* tiles, const int* num_tiles_dev,
                                       int max_tiles, float* pre_o, float* pre_lse, int B, int Hq, int Hkv, int D,
                                       int BS, int max_blocks, float scale, hipStream_t s) {
  using namespace lwc;
  (void)num_tiles_dev;
  if (D != kD || BS != kBS || Hq % Hkv != 0 || Hq / Hkv > 16) return -1;
  if (max_tiles == 0) return 0;
  DecodeParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, nullptr, nullptr, nullptr,
                 nullptr, tiles, nullptr, pre_o, pre_lse, q_stride, Hq, Hkv, Hq / Hkv, max_blocks, 1, max_tiles, scale};
  paged_decode_kernel<true><<<dim3(max_tiles, Hkv, 1), 256, 0, s>>>(p);
  return (int)hipGetLastError();
}
