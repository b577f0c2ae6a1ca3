// K3 paged_attn_decode: one query token per sequence against a paged bf16 KV cache, GQA
// (G = Hq/Hkv query heads per KV head, G <= 16), split-K (flash-decoding) over the context, and a
// PREFIX-SHARED (cascade) mode for sequences forked from one prompt.
//
// Layout (all bf16):
//   q        : [B, q_stride] — head hq at q + b*q_stride + hq*D (q lives inside the fused qkv row)
//   k_cache  : [NB, Hkv, BS, D]          (token-major rows of D)
//   v_cache  : [NB, Hkv, BS/4, D, 4]     (4-token INTERLEAVED: 4 consecutive tokens of one dim are
//                                         8 contiguous bytes = one lane's PV B-operand slice; a token's
//                                         row is written with 8 B stride, 4 dims per 32 B sector)
//   block_tables [B, max_blocks] int32, ctx_lens [B] int32
//
// MFMA design (mfma_f32_16x16x32_bf16, one wave = 64 lanes, lane l: r16 = l & 15, g = l >> 4):
//   S^T = K Q^T per 16-token block, 4 k-steps over D=128:
//     A (K)  : lane holds K[tok r16][32s + 8g + j]        -> one 16 B load straight from the cache
//     B (Q^T): lane holds Q[row r16][32s + 8g + j]        -> kept in registers for the whole kernel
//     C      : lane reg r = S^T[tok 4g + r][row r16]
//   O = P V per 32 tokens (a PAIR of blocks A,B), k permuted as {A: 4g+0..3, B: 4g+0..3}:
//     A (P)  : exactly the softmaxed S^T_A, S^T_B accumulator registers (no data movement)
//     B (V)  : lane holds V[those 8 tokens][dim 16n + r16] -> two 8 B loads from the interleaved cache
//     C      : lane reg r = O[row 4g + r][dim 16n + r16]
// The 16 MFMA rows are "query rows".  Plain decode: row = a query head of ONE sequence (only G of 16
// rows are real — the op is HBM-bound so idle rows cost nothing).  Cascade kernel: the n sequences
// that share a prompt are packed 16/G per wave-tile, row = (sequence, head), and the shared prompt
// blocks are read ONCE per tile instead of once per sequence: for N candidates of one prompt this
// removes (N-1)/N of the prompt's KV traffic and finally uses the MFMA rows; each sequence's own
// blocks follow in the same launch, softmax states merged in registers.
#include <cstdlib>

#include "common.h"

namespace lwc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t uint2v __attribute__((ext_vector_type(2)));

// K = 16 form for PV: one block's 4 tokens per lane group (operands are 8-byte halves of the 16 B V loads)
LWC_DEVICE float4v mfma16k16(const uint2v& a, const uint2v& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(short4v, a), __builtin_bit_cast(short4v, b), c,
                                                   0, 0, 0);
}

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
  int q_stride, Hq, Hkv, G, max_blocks, num_splits;
  float scale;
  // q rotation at load (pure decode steps: rope_kv_write left q un-rotated): rotate-half RoPE with the
  // model's [max_pos, D/2] fp32 tables at positions[row]; null = q already rotated
  const float* rope_cos;
  const float* rope_sin;
  const int* positions;
};

// K and V registers of one PAIR of 16-token blocks for one wave (K: 8 x 16 B, V: 16 x 8 B per lane).
struct PairRegs {
  short8 ka[4], kb[4];
  // PV operands, loaded in place: va[m] (vb[m]) = block A's (B's) tokens 4g..4g+3 of dims 32m + 2 r16 (low
  // 8 B: n-tile 2m) and 32m + 2 r16 + 1 (high 8 B: n-tile 2m+1) — one 16 B load each
  uint4v va[4], vb[4];
};


// Token rows at or past `ctx` (the tail of a sequence's last block, or a pair without a B block) are
// not fetched: each (block, head) segment is addressed through a 4 KiB buffer resource and the lanes
// that own such rows use an offset past its end, so the hardware returns zeros without a memory request.
// (Branch-free: the exec-masked form of the same loads made the compiler wrap every load in its own
// branch and insert a vmcnt(0) inside one of them, draining the two-pair pipeline every pair.)
// Their scores are masked to -inf and their V elements selected away (pair_softmax / pair_values), so
// the values never matter; zeros only keep the registers defined.  At the bench's decode shape the
// suffix's last block is on average half empty: ~10 % of the suffix bytes.
constexpr int kOOB = 0x40000000;  // an offset past any segment's num_records

LWC_DEVICE __amdgpu_buffer_rsrc_t seg_rsrc(const bf16_t* seg) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)seg, (short)0, kBS * kD * 2, 0x00020000);
}

LWC_DEVICE void load_pair_k(PairRegs& r, const DecodeParams& p, const int* bt, int kvh, int blkA, bool hasB, int r16,
                            int g, int ctx = 0x7fffffff) {
  const size_t kv_head_stride = (size_t)kBS * kD;  // elements per (block, head)
  const int physA = bt[blkA];
  const int physB = hasB ? bt[blkA + 1] : physA;
  const __amdgpu_buffer_rsrc_t rA = seg_rsrc(p.kc + ((size_t)physA * p.Hkv + kvh) * kv_head_stride);
  const __amdgpu_buffer_rsrc_t rB = seg_rsrc(p.kc + ((size_t)physB * p.Hkv + kvh) * kv_head_stride);
  const bool okA = blkA * kBS + r16 < ctx;
  const bool okB = hasB && (blkA + 1) * kBS + r16 < ctx;
  const int base = (r16 * kD + 8 * g) * 2;
  const int oA = okA ? base : kOOB, oB = okB ? base : kOOB;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    r.ka[s] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rA, oA + 64 * s, 0, 0));
    r.kb[s] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rB, oB + 64 * s, 0, 0));
  }
}

// Output dimension of accumulator n in lane r16: n-tiles pair up (2m, 2m+1) over 32 dims, the lane owning
// two ADJACENT dims of each pair, so a lane's V operands for both tiles are ONE 16 B load per block (the
// [BS/4][D][4] layout stores a token group's adjacent dims contiguously; the PV MFMA is the K = 16 form per
// block, whose 8-byte B operands are the halves of that load): 8 full-line 16 B loads per pair instead of
// 16 half-width 8 B ones.  Every epilogue writes o[n] to odim(n, r16).
LWC_DEVICE int odim(int n, int r16) { return 32 * (n >> 1) + 2 * r16 + (n & 1); }

LWC_DEVICE void load_pair_v(PairRegs& r, const DecodeParams& p, const int* bt, int kvh, int blkA, bool hasB, int r16,
                            int g, int ctx = 0x7fffffff) {
  const size_t kv_head_stride = (size_t)kBS * kD;
  const int physA = bt[blkA];
  const int physB = hasB ? bt[blkA + 1] : physA;
  const __amdgpu_buffer_rsrc_t rA = seg_rsrc(p.vc + ((size_t)physA * p.Hkv + kvh) * kv_head_stride);
  const __amdgpu_buffer_rsrc_t rB = seg_rsrc(p.vc + ((size_t)physB * p.Hkv + kvh) * kv_head_stride);
  const bool okA = blkA * kBS + 4 * g < ctx;  // lane group g holds tokens 4g..4g+3
  const bool okB = hasB && (blkA + 1) * kBS + 4 * g < ctx;
  const int base = (g * kD + 2 * r16) * 8;  // tokens 4g..4g+3 of dims 32m + 2 r16, +1: [BS/4][D][4] layout
  const int oA = okA ? base : kOOB, oB = okB ? base : kOOB;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    r.va[m] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rA, oA + 256 * m, 0, 0));
    r.vb[m] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rB, oB + 256 * m, 0, 0));
  }
}

LWC_DEVICE void load_pair(PairRegs& r, const DecodeParams& p, const int* bt, int kvh, int blkA, bool hasB, int r16,
                          int g, int ctx = 0x7fffffff) {
  load_pair_k(r, p, bt, kvh, blkA, hasB, r16, g, ctx);
  load_pair_v(r, p, bt, kvh, blkA, hasB, r16, g, ctx);
}

// S^T for the pair's two blocks (C layout: lane reg i = S^T[tok 4g+i][row r16]).
LWC_DEVICE void pair_scores(const PairRegs& r, const short8 (&qf)[4], float4v& sa, float4v& sb) {
  sa = float4v{0.f, 0.f, 0.f, 0.f};
  sb = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    sa = mfma16(r.ka[s], qf[s], sa);
    sb = mfma16(r.kb[s], qf[s], sb);
  }
}

// Online-softmax update (log2 domain) for the pair; rescales O and returns the P operand.
// Lazy rescaling threshold (log2 units): the running max is only raised — and O rescaled — when
// some row's new scores exceed it by more than this, so P <= 2^8 and most pairs skip the rescale.
constexpr float kLazyRescale = 8.f;

// Online-softmax update (log2 domain) for the pair; rescales O when needed and returns the P operand.
// `row_on` = false leaves this lane's query row untouched (p = 0): used when one wave carries rows
// of several sequences and a pass covers only one of them.
LWC_DEVICE void pair_softmax(const float4v& sa, const float4v& sb, int blkA, bool hasB, int ctx, bool row_on,
                             float sl2, int g, float4v (&o)[8], float& m, float& l, short8& pf) {
  const int blkB = blkA + 1;
  float pa[4], pb[4];
  float mx = -1e30f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ta = blkA * kBS + 4 * g + i, tb = blkB * kBS + 4 * g + i;
    pa[i] = (row_on && ta < ctx) ? sa[i] * sl2 : -INFINITY;
    pb[i] = (row_on && hasB && tb < ctx) ? sb[i] * sl2 : -INFINITY;
    mx = fmaxf(mx, fmaxf(pa[i], pb[i]));
  }
  mx = row_max4(mx);
  if (__any(mx > m + kLazyRescale)) {  // wave-uniform
    const float m_new = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - m_new);
    l *= alpha;
    m = m_new;
    // O row (4g + i) belongs to query row 4g+i, whose alpha lives in lane 4g+i
    float al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) al[i] = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= al[i];
  }
  float rs = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pa[i] = __builtin_amdgcn_exp2f(pa[i] - m);
    pb[i] = __builtin_amdgcn_exp2f(pb[i] - m);
    rs += pa[i] + pb[i];
  }
  l += row_sum4(rs);
  // P operand (A): k order {A: 4g+0..3, B: 4g+0..3}
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pf[i] = (short)f2bf(pa[i]);
    pf[4 + i] = (short)f2bf(pb[i]);
  }
}

// O += P V for the pair: per n-tile pair m, four K = 16 MFMAs (block A's and block B's 4 tokens per lane
// group, dims 2m / 2m+1 of the lane's 16 B loads; the P operand halves are the A / B score registers).
// Cache slots past the context may hold stale/uninitialised bits (possibly NaN): P = 0 there, but
// 0 * NaN = NaN, so in a pair that reaches past the context those V elements are zeroed by select, not
// arithmetic.  Pairs fully inside take the select-free path.
LWC_DEVICE uint2v lo2(const uint4v& v) { return uint2v{v[0], v[1]}; }
LWC_DEVICE uint2v hi2(const uint4v& v) { return uint2v{v[2], v[3]}; }

LWC_DEVICE void pv_mfmas(const short8& pf, const uint4v (&va)[4], const uint4v (&vb)[4], float4v (&o)[8]) {
  const uint4v pw = __builtin_bit_cast(uint4v, pf);
  const uint2v pa = lo2(pw), pb = hi2(pw);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    o[2 * m] = mfma16k16(pa, lo2(va[m]), o[2 * m]);
    o[2 * m + 1] = mfma16k16(pa, hi2(va[m]), o[2 * m + 1]);
    o[2 * m] = mfma16k16(pb, lo2(vb[m]), o[2 * m]);
    o[2 * m + 1] = mfma16k16(pb, hi2(vb[m]), o[2 * m + 1]);
  }
}

LWC_DEVICE void pair_values(const PairRegs& r, const short8& pf, int blkA, bool hasB, int ctx, int g,
                            float4v (&o)[8]) {
  const int blkB = blkA + 1;
  if (hasB && (blkB + 1) * kBS <= ctx) {  // wave-uniform
    pv_mfmas(pf, r.va, r.vb, o);
    return;
  }
  // tokens of this lane's 4-token groups inside the context: a bit mask per 16-bit element (both dims of a
  // 16 B load share the tokens), applied with ANDs (NaN bits become +0)
  const int nA = min(max(ctx - (blkA * kBS + 4 * g), 0), 4);
  const int nB = hasB ? min(max(ctx - (blkB * kBS + 4 * g), 0), 4) : 0;
  const unsigned long long mA = nA >= 4 ? ~0ull : ((1ull << (16 * nA)) - 1);
  const unsigned long long mB = nB >= 4 ? ~0ull : ((1ull << (16 * nB)) - 1);
  const uint4v qa{(uint32_t)mA, (uint32_t)(mA >> 32), (uint32_t)mA, (uint32_t)(mA >> 32)};
  const uint4v qb{(uint32_t)mB, (uint32_t)(mB >> 32), (uint32_t)mB, (uint32_t)(mB >> 32)};
  uint4v va[4], vb[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    va[m] = r.va[m] & qa;
    vb[m] = r.vb[m] & qb;
  }
  pv_mfmas(pf, va, vb, o);
}

// One whole pair: scores, softmax, values.
LWC_DEVICE void attend_pair(const PairRegs& r, int blkA, bool hasB, int ctx, const short8 (&qf)[4], float sl2, int g,
                            float4v (&o)[8], float& m, float& l) {
  float4v sa, sb;
  pair_scores(r, qf, sa, sb);
  short8 pf;
  pair_softmax(sa, sb, blkA, hasB, ctx, true, sl2, g, o, m, l, pf);
  pair_values(r, pf, blkA, hasB, ctx, g, o);
}

// Q^T operand (B) for the 4 k-steps of one wave; rows >= nrows are zero.
template <bool PREFIX>
LWC_DEVICE void load_q(short8 (&qf)[4], const DecodeParams& p, int row_seq0, int nrows, int kvh, int r16, int g) {
  const bool valid = r16 < nrows;
  const int rr = valid ? r16 : 0;
  // lanes past the wave's rows read sequence 0 (then zeroed): in the cascade kernel a wave of a short
  // super-tile can own no sequence at all, and row_seq0 then lies past the batch — reading q there went
  // out of bounds (it faulted only when q ended a mapped region)
  const int seq = !valid ? 0 : (PREFIX ? row_seq0 + rr / p.G : row_seq0);
  const int hq = kvh * p.G + (PREFIX ? rr % p.G : rr);
  const bf16_t* qh = p.q + (size_t)seq * p.q_stride + (size_t)hq * kD;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    short8 v = *reinterpret_cast<const short8*>(qh + 32 * s + 8 * g);
    qf[s] = valid ? v : short8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  if (p.rope_cos) {
    // the lane's dims are 32 s + 8 g + e: dim d < 64 (s = 0, 1) and its rotate-half partner d + 64 sit in
    // qf[s] and qf[s + 2] of the SAME lane, so the rotation is register-local (rounded to bf16 as
    // rope_kv_write rounds the q it writes back)
    const int pos = p.positions[seq];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 32 * s + 8 * g;
      const float4 c0 = *reinterpret_cast<const float4*>(p.rope_cos + (size_t)pos * (kD / 2) + c);
      const float4 c1 = *reinterpret_cast<const float4*>(p.rope_cos + (size_t)pos * (kD / 2) + c + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(p.rope_sin + (size_t)pos * (kD / 2) + c);
      const float4 s1 = *reinterpret_cast<const float4*>(p.rope_sin + (size_t)pos * (kD / 2) + c + 4);
      const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x1 = bf2f((bf16_t)qf[s][e]), x2 = bf2f((bf16_t)qf[s + 2][e]);
        qf[s][e] = (short)f2bf(x1 * cs[e] - x2 * sn[e]);
        qf[s + 2][e] = (short)f2bf(x2 * cs[e] + x1 * sn[e]);
      }
    }
  }
}

// blockIdx.x = sequence.  4 waves split the sequence's block pairs and combine through LDS: the
// long-context / small-batch path.
__global__ void __launch_bounds__(256)
    paged_decode_kernel(DecodeParams p, const int* __restrict__ block_tables, const int* __restrict__ ctx_lens) {
  const int item = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  // wid through readfirstlane: the compiler then knows everything derived from it (sequence, block
  // indices) is wave-uniform and loads block tables / ctx lens with SCALAR loads — as vector loads each
  // one needed an s_waitcnt vmcnt(0) that drained the K/V loads in flight (the pipeline collapsed)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g = lane >> 4;

  const int nrows = p.G;
  const int ctx = ctx_lens[item];
  const int nblk_total = (ctx + kBS - 1) / kBS;
  const int per_split = (nblk_total + p.num_splits - 1) / p.num_splits;
  const int blk_begin = split * per_split;
  const int blk_end = min(nblk_total, blk_begin + per_split);
  const int* bt = block_tables + (size_t)item * p.max_blocks;

  short8 qf[4];
  load_q<false>(qf, p, item, nrows, kvh, r16, g);
  const float sl2 = p.scale * kLog2e;

  float4v o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = float4v{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;  // running max / sum (log2 domain) for row r16

  for (int pair = blk_begin + 2 * wid; pair < blk_end; pair += 2 * kWaves) {
    PairRegs r;
    const bool hasB = pair + 1 < blk_end;
    load_pair(r, p, bt, kvh, pair, hasB, r16, g, ctx);
    attend_pair(r, pair, hasB, ctx, qf, sl2, g, o, m, l);
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
    for (int r = 0; r < 4; ++r) s_o[wid][4 * g + r][odim(n, r16)] = o[n][r];
  __syncthreads();
  // thread t: row h = t / 16 (< nrows), dims 8*(t%16) .. +8
  const int t = threadIdx.x;
  const int h = t >> 4, dc = (t & 15) * 8;
  if (h < nrows) {
    const int hq = kvh * p.G + h;
    float M = -1e30f;
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, s_m[w][h]);
    float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < kWaves; ++w) {
      const float f = exp2f(s_m[w][h] - M);
      L += f * s_l[w][h];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f * s_o[w][h][dc + j];
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    if (p.num_splits == 1) {
      float outv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) outv[j] = acc[j] * inv;
      *reinterpret_cast<uint4v*>(p.out + ((size_t)item * p.Hq + hq) * kD + dc) = pack8(outv);
    } else {
      float* po = p.part_o + (((size_t)item * p.Hq + hq) * p.num_splits + split) * kD + dc;
#pragma unroll
      for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
      if ((t & 15) == 0)
        p.part_lse[((size_t)item * p.Hq + hq) * p.num_splits + split] = L > 0.f ? M + log2f(L) : -INFINITY;
    }
  }
}

// One WAVE per item, kWaves independent items per workgroup, no LDS and no barriers: the
// large-batch path (B * Hkv * splits >= kWaveKernelMinItems).  Item = (sequence, split).  The block-pair
// loop is software-pipelined in registers (the loads of pair i+1 are in flight while pair i is on the
// MFMAs), and the epilogue writes straight from the accumulator layout.
__global__ void __launch_bounds__(256) paged_decode_wave_kernel(DecodeParams p, int num_items,
                                                                const int* __restrict__ block_tables,
                                                                const int* __restrict__ ctx_lens) {
  // wid through readfirstlane: the compiler then knows everything derived from it (sequence, block
  // indices) is wave-uniform and loads block tables / ctx lens with SCALAR loads — as vector loads each
  // one needed an s_waitcnt vmcnt(0) that drained the K/V loads in flight (the pipeline collapsed)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int item = blockIdx.x * kWaves + wid, kvh = blockIdx.y;
  if (item >= num_items) return;  // the whole wave leaves; nothing below synchronises
  const int r16 = lane & 15, g = lane >> 4;

  const int seq = item / p.num_splits;
  const int split = item - seq * p.num_splits;
  const int nrows = p.G;
  const int ctx = ctx_lens[seq];
  const int nblk_total = (ctx + kBS - 1) / kBS;
  const int per_split = (nblk_total + p.num_splits - 1) / p.num_splits;
  const int blk_begin = split * per_split;
  const int blk_end = min(nblk_total, blk_begin + per_split);
  const int* bt = block_tables + (size_t)seq * p.max_blocks;

  short8 qf[4];
  load_q<false>(qf, p, seq, nrows, kvh, r16, g);
  const float sl2 = p.scale * kLog2e;

  float4v o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = float4v{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;

  // Rolling one-set pipeline: the K registers are refilled with pair i+1 as soon as the S MFMAs
  // of pair i have consumed them, the V registers right after the PV MFMAs — a pair's loads are in
  // flight under the previous pair's softmax / PV work at ~1/2 the registers of a double buffer.
  PairRegs r;
  int pair = blk_begin;
  if (pair < blk_end) {
    load_pair_k(r, p, bt, kvh, pair, pair + 1 < blk_end, r16, g, ctx);
    load_pair_v(r, p, bt, kvh, pair, pair + 1 < blk_end, r16, g, ctx);
  }
  while (pair < blk_end) {
    const bool hasB = pair + 1 < blk_end;
    const int nxt = pair + 2;
    float4v sa, sb;
    pair_scores(r, qf, sa, sb);
    if (nxt < blk_end) load_pair_k(r, p, bt, kvh, nxt, nxt + 1 < blk_end, r16, g, ctx);
    short8 pf;
    pair_softmax(sa, sb, pair, hasB, ctx, true, sl2, g, o, m, l, pf);
    pair_values(r, pf, pair, hasB, ctx, g, o);
    if (nxt < blk_end) load_pair_v(r, p, bt, kvh, nxt, nxt + 1 < blk_end, r16, g, ctx);
    pair = nxt;
  }

  // epilogue: lane (g, r16) owns rows 4g+i, dims 16n+r16; row stats live in lane (row)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int R = 4 * g + i;
    const float li = __shfl(l, R, 64), mi = __shfl(m, R, 64);
    if (R >= nrows) continue;
    const size_t bh = (size_t)seq * p.Hq + kvh * p.G + R;
    const float inv = li > 0.f ? 1.f / li : 0.f;
    if (p.num_splits > 1) {
      float* dst = p.part_o + (bh * p.num_splits + split) * kD;
#pragma unroll
      for (int n = 0; n < 8; ++n) dst[odim(n, r16)] = o[n][i] * inv;
      if (r16 == 0) p.part_lse[bh * p.num_splits + split] = li > 0.f ? mi + log2f(li) : -INFINITY;
    } else {
      bf16_t* dst = p.out + bh * kD;
#pragma unroll
      for (int n = 0; n < 8; ++n) dst[odim(n, r16)] = f2bf(o[n][i] * inv);
    }
  }
}

// B * Hkv * splits at/above which the wave-per-item kernel runs (tests lower it to cover both paths)
static int g_wave_min_items = 2048;

// ---------------------------------------------------------------------------------------------
// CASCADE kernel: the shared-prompt pass and every sequence's own suffix in ONE launch, no partials.
//
// Workgroup = kCWaves waves = one SUPER-TILE (row_start, nseq, prefix_blocks) x one KV head; wave w
// owns sequences row_start + w*per .. (+per), per = 16/G, as its 16 MFMA query rows (seq, head).
//  phase 1 (prefix): the super-tile's sequences share their first `prefix_blocks` blocks.  The WG
//    stages kCPairs block pairs at a time into LDS (K rows XOR-swizzled by 16 B chunk, V^T linear),
//    and every wave runs the pair loop for its 16 rows out of LDS: the prompt's KV is read from HBM
//    once per (super-tile, head) — 32 sequences for Llama-3's G=4 — instead of once per sequence.
//  phase 2 (suffix): each wave walks its sequences' own blocks from global memory (rolling register
//    pipeline that crosses sequence boundaries), masking the rows of the other sequences
//    (row_on), so the prefix and suffix softmax states merge in registers.
//  epilogue: bf16 output straight from the accumulator layout.
// Super-tiles with prefix_blocks = 0 are plain decode for up to kCWaves*per unrelated sequences.
constexpr int kCWaves = 8;
constexpr int kCPairsMax = 8;                      // pairs staged per LDS chunk (<= 128 KiB)
constexpr int kCRounds = 1024 / (kCWaves * 64);     // 16 B loads per thread per pair
constexpr int kPairBytes = 4 * kBS * kD * 2;        // K_A, K_B, V_A^T, V_B^T = 16 KiB
constexpr int kSegBytes = kBS * kD * 2;             // 4 KiB

struct CascadeParams {
  const bf16_t* q;
  const bf16_t* kc;
  const bf16_t* vc;
  const int* block_tables;
  const int* ctx_lens;
  const int* tiles;  // [max_tiles, 3]
  bf16_t* out;       // [B, Hq, D]
  int q_stride, Hq, Hkv, G, max_blocks;
  float scale;
  const float* rope_cos;  // as DecodeParams
  const float* rope_sin;
  const int* positions;
  // MX output (the fp8 o projection's A operand): e4m3 rows [B, Hq * D] + e8m0 scales [Hq][mx_rows][4], one per
  // 32 dims of a head (out is then unused)
  uint8_t* out8;
  uint8_t* mx;
  int mx_rows;
};

// The index tables come in as const __restrict__ kernel arguments (not through the params struct): with
// uniform addresses the compiler may then use SCALAR loads for them (no possible clobber by the output
// stores).  As vector loads every block-table / ctx-len read needed an s_waitcnt vmcnt(0), which drained
// the K/V loads in flight and serialised both phases.
template <int kCPairs>
__global__ void __launch_bounds__(kCWaves * 64)
    paged_decode_cascade_kernel(CascadeParams p, const int* __restrict__ block_tables, const int* __restrict__ ctx_lens,
                                const int* __restrict__ tiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // heads are the fast grid dimension: the real tiles (a prefix of the table) are dispatched first,
  // the graph-capture slack (nseq = 0 entries) last
  const int tile = blockIdx.y, kvh = blockIdx.x;
  const int* t = tiles + 3 * tile;
  const int row_start = t[0], nseq = t[1], pblk = t[2];
  if (nseq <= 0) return;  // uniform for the whole workgroup, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // see above
  const int r16 = lane & 15, g = lane >> 4;
  const int per = 16 / p.G;
  const int s0 = row_start + wid * per;
  const int nseq_w = max(0, min(per, nseq - wid * per));
  const int nrows = nseq_w * p.G;
  const float sl2 = p.scale * kLog2e;
  const size_t kv_head_stride = (size_t)kBS * kD;

  short8 qf[4];
  DecodeParams qp{};
  qp.q = p.q;
  qp.q_stride = p.q_stride;
  qp.G = p.G;
  qp.rope_cos = p.rope_cos;
  qp.rope_sin = p.rope_sin;
  qp.positions = p.positions;
  load_q<true>(qf, qp, s0, nrows, kvh, r16, g);

  float4v o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = float4v{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;

  // ---- phase 1: shared prefix through LDS ----
  const int* bt0 = block_tables + (size_t)row_start * p.max_blocks;
  const int pctx = pblk * kBS;
  // LDS-DMA of prefix chunk c0 (kCPairs block pairs; global_load_lds_dwordx4): wave-instruction (pair, round)
  // writes 1 KiB contiguously, lane-linear; the K image's XOR swizzle is applied to the SOURCE address.
  auto issue_chunk = [&](int c0) {
    const int npairs = min(kCPairs, (pblk - c0 + 1) / 2);
#pragma unroll
    for (int pi = 0; pi < kCPairs; ++pi) {
#pragma unroll
      for (int rd = 0; rd < kCRounds; ++rd) {
        // 16 B unit u = rd*512 + tid of the pair's 16 KiB image: segment (K_A, K_B, V_A, V_B) u >> 8 is
        // wave-uniform (rd*2 + wid/4), the position inside it is (wid%4)*64 + lane
        const int seg = rd * 2 + (wid >> 2), pos = ((wid & 3) << 6) + lane;
        const int blk = c0 + 2 * pi + (seg & 1);
        if (pi < npairs && blk < pblk) {  // wave-uniform: a wave's 64 units lie in one segment
          const int phys = bt0[blk];
          const unsigned char* src =
              reinterpret_cast<const unsigned char*>(((seg < 2) ? p.kc : p.vc) +
                                                     ((size_t)phys * p.Hkv + kvh) * kv_head_stride);
          if (seg < 2) {  // K [16 tok][256 B]: 16 B chunk XOR row
            const int row = pos >> 4, pch = pos & 15;
            src += row * 256 + ((pch ^ row) << 4);
          } else {  // V [4 token groups][128 dim][8 B], linear: the 16 B reads (dims 2 r16, +1 of a group)
            src += pos << 4;  // of one lane group span 256 contiguous bytes = every bank once
          }
          unsigned char* dst = smem + pi * kPairBytes + (rd * (kCWaves * 64) + wid * 64) * 16;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
      }
    }
  };
  // prefix pair pi of the chunk at c0, out of LDS, into `r` (a free register set) and onto the state
  auto attend_lds = [&](PairRegs& r, int c0, int pi) {
    const int blkA = c0 + 2 * pi;
    const bool hasB = blkA + 1 < pblk;
    const unsigned char* pb = smem + pi * kPairBytes;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ch = ((4 * s + g) ^ r16) << 4;
      r.ka[s] = *reinterpret_cast<const short8*>(pb + r16 * 256 + ch);
      r.kb[s] = *reinterpret_cast<const short8*>(pb + kSegBytes + r16 * 256 + ch);
    }
#pragma unroll
    for (int m2 = 0; m2 < 4; ++m2) {
      const int off = (g * kD + 32 * m2 + 2 * r16) << 3;
      r.va[m2] = *reinterpret_cast<const uint4v*>(pb + 2 * kSegBytes + off);
      r.vb[m2] = *reinterpret_cast<const uint4v*>(pb + 3 * kSegBytes + off);
    }
    attend_pair(r, blkA, hasB, pctx, qf, sl2, g, o, m, l);
  };
  auto phase1 = [&]() {
    for (int c0 = 0; c0 < pblk; c0 += 2 * kCPairs) {
      const int npairs = min(kCPairs, (pblk - c0 + 1) / 2);
      __syncthreads();  // previous chunk fully consumed
      issue_chunk(c0);
      __syncthreads();
      if (nrows > 0) {
        for (int pi = 0; pi < npairs; ++pi) {
          PairRegs r;
          attend_lds(r, c0, pi);
        }
      }
    }
  };

  // ---- phase 2: each sequence's own blocks, two pairs in flight per wave ----
  // Positions walk (sequence j of the wave, block pair) across the wave's sequences.  Two register
  // sets alternate (unrolled by two, so no register copies of in-flight loads): while one pair is on
  // the MFMAs the next pair's K and V are already loading — two pairs (32 KiB) in flight per wave.
  DecodeParams lp{};
  lp.kc = p.kc;
  lp.vc = p.vc;
  lp.Hkv = p.Hkv;
  struct Pos {
    int j, pair, end, ctx;
  };
  auto seq_pos = [&](int j) {  // first suffix pair of sequence j (or beyond), skipping empty suffixes
    Pos q{j, pblk, 0, 0};
    while (q.j < nseq_w) {
      q.ctx = ctx_lens[s0 + q.j];
      q.end = (q.ctx + kBS - 1) / kBS;
      if (q.pair < q.end) break;
      ++q.j;
    }
    return q;
  };
  auto next = [&](Pos q) {
    q.pair += 2;
    return q.pair < q.end ? q : seq_pos(q.j + 1);
  };
  auto load = [&](PairRegs& r, const Pos& q) {
    const int* bt = block_tables + (size_t)(s0 + q.j) * p.max_blocks;
    load_pair_k(r, lp, bt, kvh, q.pair, q.pair + 1 < q.end, r16, g, q.ctx);
    load_pair_v(r, lp, bt, kvh, q.pair, q.pair + 1 < q.end, r16, g, q.ctx);
  };
  auto attend = [&](const PairRegs& r, const Pos& q) {
    const bool row_on = r16 < nrows && r16 / p.G == q.j;
    float4v sa, sb;
    pair_scores(r, qf, sa, sb);
    short8 pf;
    pair_softmax(sa, sb, q.pair, q.pair + 1 < q.end, q.ctx, row_on, sl2, g, o, m, l, pf);
    pair_values(r, pf, q.pair, q.pair + 1 < q.end, q.ctx, g, o);
  };

  if (pblk > 2 * kCPairs) {
    // long shared prompt (several LDS chunks): the chunked prefix pass, then the suffixes
    phase1();
    if (nrows > 0) {
      PairRegs ra, rb;
      Pos p0 = seq_pos(0);
      if (p0.j < nseq_w) {
        Pos p1 = next(p0);
        load(ra, p0);
        if (p1.j < nseq_w) load(rb, p1);
        while (true) {
          attend(ra, p0);
          if (p1.j >= nseq_w) break;
          const Pos p2 = next(p1);
          if (p2.j < nseq_w) load(ra, p2);
          attend(rb, p1);
          if (p2.j >= nseq_w) break;
          const Pos p3 = next(p2);
          if (p3.j < nseq_w) load(rb, p3);
          p0 = p2;
          p1 = p3;
        }
      }
    }
  } else {
    // The whole shared prompt fits one LDS chunk (the common case: a few hundred prompt tokens).  Its
    // LDS-DMA is issued first and lands while the first two suffix pairs load (both streams in flight
    // together — the serial DMA-then-compute prefix pass left the CU's memory pipe idle: one workgroup per
    // CU, VGPR-bound); then every prefix pair is attended out of LDS in the register set a suffix pair
    // has just released, between the suffix pairs, while the other set's loads are in flight.  Online
    // softmax merges in any order.
    const int npre = (pblk + 1) / 2;
    int pre = 0;
    issue_chunk(0);
    PairRegs ra, rb;
    Pos p0{nseq_w, 0, 0, 0}, p1{nseq_w, 0, 0, 0};
    if (nrows > 0) {
      p0 = seq_pos(0);
      if (p0.j < nseq_w) {
        p1 = next(p0);
        load(ra, p0);
        if (p1.j < nseq_w) load(rb, p1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's prefix DMA (and both suffix pairs) landed
    __syncthreads();                                  // every wave's prefix DMA landed: LDS chunk readable
    if (nrows > 0) {
      if (p0.j < nseq_w) {
        while (true) {
          attend(ra, p0);
          if (pre < npre) attend_lds(ra, 0, pre++);
          if (p1.j >= nseq_w) break;
          const Pos p2 = next(p1);
          if (p2.j < nseq_w) load(ra, p2);
          attend(rb, p1);
          if (pre < npre) attend_lds(rb, 0, pre++);
          if (p2.j >= nseq_w) break;
          const Pos p3 = next(p2);
          if (p3.j < nseq_w) load(rb, p3);
          p0 = p2;
          p1 = p3;
        }
      }
      while (pre < npre) attend_lds(ra, 0, pre++);
    }
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int R = 4 * g + i;
    const float li = __shfl(l, R, 64);
    if (R >= nrows) continue;
    const int seq = s0 + R / p.G;
    const int hq = kvh * p.G + R % p.G;
    const float inv = li > 0.f ? 1.f / li : 0.f;
    if (p.out8) {
      // block b = dims [32b, 32b + 32) = o[2b], o[2b + 1] of the 16 lanes of this DPP row (odim)
      uint8_t* dst = p.out8 + ((size_t)seq * p.Hq + hq) * kD;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float v0 = o[2 * b][i] * inv, v1 = o[2 * b + 1][i] * inv;
        const int e = mx_exp(row16_max(fmaxf(fabsf(v0), fabsf(v1))));
        const float sc = __builtin_amdgcn_ldexpf(1.f, -e);
        const uint32_t pk = __builtin_amdgcn_cvt_pk_fp8_f32(v0 * sc, v1 * sc, 0, false);
        *reinterpret_cast<uint16_t*>(dst + odim(2 * b, r16)) = (uint16_t)pk;
        if (r16 == 0) p.mx[((size_t)hq * p.mx_rows + seq) * 4 + b] = (uint8_t)(e + 127);
      }
    } else {
      bf16_t* dst = p.out + ((size_t)seq * p.Hq + hq) * kD;
#pragma unroll
      for (int n = 0; n < 8; ++n) dst[odim(n, r16)] = f2bf(o[n][i] * inv);
    }
  }
}

// Combine split-K partials: out[b, hq, :] = sum_s 2^(lse_s - LSE) o_s / sum_s 2^(lse_s - LSE)
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

extern "C" int lwc_set_decode_wave_min_items(int n) {
  const int old = lwc::g_wave_min_items;
  lwc::g_wave_min_items = n;
  return old;
}

// Plain split-K paged decode (the small-batch / no-shared-prompt path; the engine's large batches with
// forked prompts use the cascade kernel below).
extern "C" int lwc_paged_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                                const int* ctx_lens, void* out, float* part_o, float* part_lse, int B, int Hq,
                                int Hkv, int D, int BS, int max_blocks, int num_splits, float scale,
                                const float* rope_cos, const float* rope_sin, const int* positions, hipStream_t s) {
  using namespace lwc;
  if (D != kD || BS != kBS || Hq % Hkv != 0 || Hq / Hkv > 16 || num_splits < 1) return -1;
  if (num_splits > 1 && (!part_o || !part_lse)) return -2;
  if (B == 0) return 0;
  DecodeParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, ctx_lens, (bf16_t*)out,
                 part_o, part_lse, q_stride, Hq, Hkv, Hq / Hkv, max_blocks, num_splits, scale,
                 rope_cos, rope_sin, positions};
  if ((long)B * Hkv * num_splits >= g_wave_min_items) {
    const int items = B * num_splits;
    paged_decode_wave_kernel<<<dim3((items + kWaves - 1) / kWaves, Hkv), 256, 0, s>>>(p, items, block_tables,
                                                                                      ctx_lens);
  } else {
    paged_decode_kernel<<<dim3(B, Hkv, num_splits), 256, 0, s>>>(p, block_tables, ctx_lens);
  }
  if (num_splits > 1) paged_decode_reduce_kernel<<<B * Hq, kD, 0, s>>>(part_o, part_lse, (bf16_t*)out, num_splits);
  return (int)hipGetLastError();
}

// Cascade decode (shared prefix + suffix in one launch); tiles = [max_tiles, 3] super-tiles
// (row_start, nseq <= kCWaves*16/G, prefix_blocks), unused entries nseq = 0.
extern "C" int lwc_paged_decode_cascade(const void* q, int q_stride, const void* kc, const void* vc,
                                        const int* block_tables, const int* ctx_lens, const int* tiles, int max_tiles,
                                        void* out, int Hq, int Hkv, int D, int BS, int max_blocks, float scale,
                                        const float* rope_cos, const float* rope_sin, const int* positions,
                                        void* out8, void* mx, int mx_rows, hipStream_t s) {
  using namespace lwc;
  if (D != kD || BS != kBS || Hq % Hkv != 0 || 16 % (Hq / Hkv) != 0) return -1;
  if ((out8 == nullptr) != (mx == nullptr)) return -1;
  if (max_tiles == 0) return 0;
  CascadeParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, block_tables, ctx_lens, tiles,
                  (bf16_t*)out, q_stride, Hq, Hkv, Hq / Hkv, max_blocks, scale, rope_cos, rope_sin, positions,
                  (uint8_t*)out8, (uint8_t*)mx, mx_rows};
  static int pairs = 0;
  if (pairs == 0) {
    const char* e = getenv("LWC_CASCADE_PAIRS");
    pairs = e ? atoi(e) : 8;
    for (int k : {2, 4, 8})
      (void)hipFuncSetAttribute(k == 2 ? (const void*)paged_decode_cascade_kernel<2>
                                       : k == 4 ? (const void*)paged_decode_cascade_kernel<4>
                                                : (const void*)paged_decode_cascade_kernel<8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, k * kPairBytes);
  }
  {
    const char* e = getenv("LWC_CASCADE_PAIRS");  // experiment knob, re-read per launch
    if (e) pairs = atoi(e);
  }
  const dim3 grid(Hkv, max_tiles);
  if (pairs == 2)
    paged_decode_cascade_kernel<2><<<grid, kCWaves * 64, 2 * kPairBytes, s>>>(p, block_tables, ctx_lens, tiles);
  else if (pairs == 4)
    paged_decode_cascade_kernel<4><<<grid, kCWaves * 64, 4 * kPairBytes, s>>>(p, block_tables, ctx_lens, tiles);
  else
    paged_decode_cascade_kernel<8><<<grid, kCWaves * 64, 8 * kPairBytes, s>>>(p, block_tables, ctx_lens, tiles);
  return (int)hipGetLastError();
}

extern "C" int lwc_cascade_rows_per_tile(int G) { return lwc::kCWaves * (16 / G); }
