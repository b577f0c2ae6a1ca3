// K8a+K8b+K8c+K8d fused: logits processing, raw log-softmax + top-k logprobs, and top-k / top-p /
// min-p / top-a filtered multinomial sampling (or greedy argmax) in ONE pass over each logits row.
//
// One 1024-thread workgroup per row.  The row (bf16, V <= 8*1024*SLOTS) is loaded ONCE from HBM into
// registers as packed bf16 (16 B per load, SLOTS loads per thread) and every later phase — raw max and
// log-sum-exp, the top-K selection for `top_logprobs`, penalties/bias/grammar mask, the filter
// thresholds and the inverse-CDF draw — works on those registers plus block reductions.
// Element index of (thread t, slot j, lane-element e) = (j*1024 + t)*8 + e.
//
// Thresholds are found by exact binary search over the 16-bit order-preserving key of the bf16 value
// (16 block-reduction rounds), so top-p / top-k are exact (ties at the threshold are kept, as in the
// usual "keep >= threshold" convention).  Randomness: Philox4x32-10 keyed by the per-sequence seed,
// counter = per-sequence step — reproducible per (seed, step) independent of batch composition.
//
// Reference fields served: temperature/top_p/min_p/top_a/top_k/frequency_penalty/presence_penalty/
// repetition_penalty/logit_bias (src/score/llm/mod.rs:39-72, validation :376-406,:490-508),
// top_logprobs <= 20 (:455-467) feeding the vote extractor (src/score/completions/client.rs:1721-1793),
// and constrained output modes (json_schema / tool_call, src/score/llm/mod.rs:690-696).
#include "common.h"

namespace lwc {

constexpr int kSampT = 1024;
constexpr int kMaxTopK = 20;
constexpr int kCollect = 64;

struct SampleParams {
  const bf16_t* logits;  // [B, ld]
  int ld, V;
  const float* temperature;  // [B]  (<= 0 -> greedy)
  const float* top_p;        // [B]  (>= 1 -> off)
  const int* top_k;          // [B]  (<= 0 -> off)
  const float* min_p;        // [B]  (<= 0 -> off)
  const float* top_a;        // [B]  (<= 0 -> off)
  const float* freq_pen;     // [B] or null
  const float* pres_pen;     // [B] or null
  const float* rep_pen;      // [B] or null
  uint16_t* counts;          // [B, V] generated-token counts (or null); updated with the sample
  const int* count_rows;     // [B] row of `counts` for each batch row (or null = identity)
  const float* bias;         // [NBT, V] dense logit bias rows (or null)
  const int* bias_rows;      // [B] row of `bias` (-1 = none)
  const uint32_t* mask;      // [NMT, V/32] allowed-token bitmasks (or null)
  const int* mask_rows;      // [B] row of `mask` (-1 = none)
  const unsigned long long* seeds;    // [B]
  const unsigned long long* offsets;  // [B] (step counter)
  int num_logprobs;          // K for top logprobs (0..20)
  int mask_logprobs;         // 1: rows with a grammar mask report logprobs over the MASKED distribution
                             //    (the restricted softmax over the allowed tokens — the vote fast path)
  int need_logprob;          // 0: no caller reads out_logprob (and K == 0): the raw log-sum-exp is not
                             //    computed and out_logprob is NaN
  int* out_token;            // [B]
  float* out_logprob;        // [B]  raw logprob of the sampled token
  int* out_topk_ids;         // [B, K]
  float* out_topk_lp;        // [B, K]
};

// ---- Philox4x32-10 ----
LWC_DEVICE void philox4x32(uint32_t (&ctr)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = 0xD2511F53u * ctr[0], hi0 = __umulhi(0xD2511F53u, ctr[0]);
    const uint32_t lo1 = 0xCD9E8D57u * ctr[2], hi1 = __umulhi(0xCD9E8D57u, ctr[2]);
    const uint32_t n0 = hi1 ^ ctr[1] ^ k0, n2 = hi0 ^ ctr[3] ^ k1;
    ctr[0] = n0;
    ctr[1] = lo1;
    ctr[2] = n2;
    ctr[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

LWC_DEVICE uint32_t f2key(float f) {  // order-preserving 16-bit key of the bf16-rounded value
  const uint32_t b = __float_as_uint(f) >> 16;
  return (b & 0x8000u) ? (~b & 0xffffu) : (b | 0x8000u);
}
LWC_DEVICE float key2f(uint32_t k) {
  const uint32_t b = (k & 0x8000u) ? (k & 0x7fffu) : (~k & 0xffffu);
  return __uint_as_float(b << 16);
}

// Keep the packed row opaque at the top of every pass: otherwise LICM hoists the 8*SLOTS unpacked
// floats (or their keys) out of the binary-search loops and the kernel spills (1024 threads leave
// 128 VGPRs per lane; the packed row alone is 4*SLOTS of them).
#define OPAQUE_ROW(row)                                   \
  _Pragma("unroll") for (int _j = 0; _j < SLOTS; ++_j) { \
    asm volatile("" : "+v"(row[_j]));                     \
  }

// value of element e (0..7) of the row vector held in slot j (compile-time j, e: stays in VGPRs)
#define GET(row, j, e) \
  (((e)&1) ? __uint_as_float((row)[j][(e) >> 1] & 0xffff0000u) : __uint_as_float((row)[j][(e) >> 1] << 16))

// fp16 helpers for the probability form of the row (u in [0,1] as packed fp16)
LWC_DEVICE uint16_t h2bits(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
#define KEYU(row, j, e) ((((e)&1) ? ((row)[j][(e) >> 1] >> 16) : ((row)[j][(e) >> 1] & 0xffffu)))
#define GETU(row, j, e) ((float)__builtin_bit_cast(_Float16, (uint16_t)KEYU(row, j, e)))

// Packed selection over the probability form (two non-negative fp16 u per register: their bit patterns
// order like the values).  Per pair: a saturating 16-bit subtract against (threshold - 1) is >= 1 exactly
// where key >= threshold, min(., 1) makes that a 0/1 mask, and either a packed add counts it or a packed
// multiply by 0x3C00 turns it into fp16 0 / 1.0 for a v_dot2 that sums the kept u in fp32 — 2 VALU per
// element instead of unpack + compare + select + add (+ the SDWA hazard nops) per element.
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
LWC_DEVICE half2v as_h2(uint32_t w) { return __builtin_bit_cast(half2v, w); }
LWC_DEVICE void count2(uint32_t& c2, uint32_t w0, uint32_t w1, uint32_t thr1x2, uint32_t one2) {
  uint32_t t0, t1;
  asm("v_pk_sub_u16 %1, %3, %5 clamp\n\t"
      "v_pk_sub_u16 %2, %4, %5 clamp\n\t"
      "v_pk_min_u16 %1, %1, %6\n\t"
      "v_pk_min_u16 %2, %2, %6\n\t"
      "v_pk_add_u16 %0, %0, %1\n\t"
      "v_pk_add_u16 %0, %0, %2"
      : "+v"(c2), "=&v"(t0), "=&v"(t1)
      : "v"(w0), "v"(w1), "v"(thr1x2), "v"(one2));
}
// Two registers (four u) per block, the whole chain in one asm block: the compiler puts a hazard nop
// after every inline-asm result a compiled instruction reads, so the dot stays inside.  Ordering keeps
// each v_dot2c >= 1 instruction after the multiply that feeds it (VALU write -> DOT read) and the dots
// back to back on one accumulator (same-DOT srcC forwarding, no wait); the accumulator's final reader
// waits through dot_read().
LWC_DEVICE void mass2(float& acc, uint32_t w0, uint32_t w1, uint32_t thr1x2, uint32_t one2, uint32_t h1x2) {
  uint32_t t0, t1;
  asm("v_pk_sub_u16 %1, %3, %5 clamp\n\t"
      "v_pk_sub_u16 %2, %4, %5 clamp\n\t"
      "v_pk_min_u16 %1, %1, %6\n\t"
      "v_pk_min_u16 %2, %2, %6\n\t"
      "v_pk_mul_lo_u16 %1, %1, %7\n\t"
      "v_pk_mul_lo_u16 %2, %2, %7\n\t"
      "v_dot2c_f32_f16 %0, %3, %1\n\t"
      "v_dot2c_f32_f16 %0, %4, %2"
      : "+v"(acc), "=&v"(t0), "=&v"(t1)
      : "v"(w0), "v"(w1), "v"(thr1x2), "v"(one2), "v"(h1x2));
}
// DOT write -> VALU read needs 3 wait states
LWC_DEVICE float dot_read(float acc) {
  float r;
  asm("s_nop 2\n\tv_mov_b32 %0, %1" : "=v"(r) : "v"(acc));
  return r;
}
LWC_DEVICE uint32_t thr1x2(uint32_t key) { return ((key - 1u) & 0xffffu) * 0x10001u; }  // key >= 1

LWC_DEVICE int block_sum_i(int v, int* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  int r = lane < (kSampT / 64) ? scratch[lane] : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
  return r;
}

template <int SLOTS>
__global__ void __launch_bounds__(kSampT) sample_kernel(SampleParams p) {
  __shared__ float sred[32];
  __shared__ int sredi[32];
  __shared__ float s_cval[kCollect];
  __shared__ int s_cidx[kCollect];
  __shared__ int s_ccount;
  __shared__ float s_scan[kSampT / 64];
  __shared__ uint32_t s_tkey[kSampT];
  __shared__ uint32_t s_lb, s_fkey;
  __shared__ uint32_t s_own[SLOTS * 4];
  __shared__ float s_oexcl;
  __shared__ int s_found;

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const bf16_t* lrow = p.logits + (size_t)b * p.ld;
  const int nvec = p.V >> 3;

  // ---- load the raw row once ----
  uint4v row[SLOTS];
  const uint32_t* lmask =
      (p.mask_logprobs && p.mask && p.mask_rows[b] >= 0) ? p.mask + (size_t)p.mask_rows[b] * (p.V >> 5) : nullptr;
#pragma unroll
  for (int j = 0; j < SLOTS; ++j) {
    const int vi = j * kSampT + t;
    row[j] = vi < nvec ? *reinterpret_cast<const uint4v*>(lrow + (size_t)vi * 8) : uint4v{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};
    if (lmask && vi < nvec) {  // constrained logprobs: disallowed tokens are -inf from the start
      const uint32_t bits = (lmask[vi >> 2] >> ((vi & 3) * 8)) & 0xffu;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t lo = (bits >> (2 * c)) & 1u ? (row[j][c] & 0xffffu) : 0xff80u;
        const uint32_t hi = (bits >> (2 * c + 1)) & 1u ? (row[j][c] >> 16) : 0xff80u;
        row[j][c] = lo | (hi << 16);
      }
    }
  }
  // ---- raw max (+ each thread's own max key: the top-K search bound) and log-sum-exp ----
  float mx = -INFINITY;
OPAQUE_ROW(row);
#pragma unroll
  for (int j = 0; j < SLOTS; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) mx = fmaxf(mx, GET(row, j, e));
  const uint32_t my_maxkey = f2key(mx);
  const float raw_max = block_max(mx, sred);
  const int lane = t & 63, wid = t >> 6;
  const int K = p.num_logprobs;
  // The raw log-sum-exp (the denominator of every reported logprob) is only computed when some output
  // needs it, and its exp sum rides along in a pass that runs anyway: the processed-row pass, or the
  // sampling pass's exp when the row is unprocessed (then its max IS the raw max).  Only a greedy
  // unprocessed row pays a pass of its own.
  const bool need_lse = p.need_logprob || K > 0;
  float se = 0.f;

  // ---- raw top-K (for top_logprobs): candidates collected here, ranked and written once the
  // log-sum-exp is known ----
  if (K > 0) {
    // Bound first: the K largest per-thread maxima are K distinct elements, so the K-th largest element
    // of the row is >= the K-th largest thread max (lb).  One wave finds lb over the 1024 thread maxima
    // (no block barriers inside the search); the elements >= lb — rarely more than a few dozen — are
    // then collected in one pass.  Only if they overflow the collection buffer does the exact 16-round
    // search over the whole row run (starting from lb).  Masked (-inf, key 0x7f) entries are never
    // candidates: a row with < K finite values returns fewer (rest: id -1).
    if (t == 0) s_ccount = 0;
    s_tkey[t] = my_maxkey;
    __syncthreads();
    if (t < 64) {
      uint32_t lo = 0x80u, hi = 0xffffu;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        float c = 0.f;
#pragma unroll
        for (int i = 0; i < kSampT / 64; ++i) c += s_tkey[i * 64 + t] >= mid ? 1.f : 0.f;
        if (wave_sum(c) >= (float)K)
          lo = mid;
        else
          hi = mid - 1;
      }
      if (t == 0) s_lb = lo;
    }
    __syncthreads();
    uint32_t lo = s_lb;
#pragma unroll 1
    for (int attempt = 0; attempt < 2; ++attempt) {
      if (attempt == 1) {  // overflow: exact search for the K-th largest key, then collect again
        uint32_t hi = 0xffffu;
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          int c = 0;
OPAQUE_ROW(row);
#pragma unroll
          for (int j = 0; j < SLOTS; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) c += f2key(GET(row, j, e)) >= mid;
          if (block_sum_i(c, sredi) >= K)
            lo = mid;
          else
            hi = mid - 1;
        }
        __syncthreads();
        if (t == 0) s_ccount = 0;
        __syncthreads();
      }
      // candidates are sparse (a few dozen of 128k): one float compare per element and a wave-uniform
      // branch on its ballot; only an element position where some lane of the wave hits runs the exact
      // key test and the LDS append (key2f(lo) is the smallest value with key >= lo, so the float test
      // passes a superset: -0 next to +0)
      const float thr = key2f(lo);
OPAQUE_ROW(row);
#pragma unroll
      for (int j = 0; j < SLOTS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = GET(row, j, e);
          const bool h = v >= thr;
          if (__builtin_amdgcn_ballot_w64(h)) {
            const int idx = (j * kSampT + t) * 8 + e;
            if (h && f2key(v) >= lo) {  // padding past V holds -inf (key 0x7f < lo): never collected
              const int slot = atomicAdd(&s_ccount, 1);
              if (slot < kCollect) {
                s_cval[slot] = v;
                s_cidx[slot] = idx;
              }
            }
          }
        }
      __syncthreads();
      if (s_ccount <= kCollect) break;  // block-uniform
    }
  }

  // ---- processed values y = raw + bias - penalties (masked -> -inf), stored back as bf16 ----
  const float* brow = (p.bias && p.bias_rows[b] >= 0) ? p.bias + (size_t)p.bias_rows[b] * p.V : nullptr;
  const uint32_t* mrow = (p.mask && p.mask_rows[b] >= 0) ? p.mask + (size_t)p.mask_rows[b] * (p.V >> 5) : nullptr;
  const int crow_i = p.counts ? (p.count_rows ? p.count_rows[b] : b) : -1;
  const uint16_t* crow = crow_i >= 0 ? p.counts + (size_t)crow_i * p.V : nullptr;
  const float fpen = p.freq_pen ? p.freq_pen[b] : 0.f, ppen = p.pres_pen ? p.pres_pen[b] : 0.f;
  const float rpen = p.rep_pen ? p.rep_pen[b] : 1.f;
  const bool use_pen = crow && (fpen != 0.f || ppen != 0.f || rpen != 1.f);
  const bool processed = brow || mrow || use_pen;
  if (processed) {
OPAQUE_ROW(row);
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const int vi = j * kSampT + t;
      if (vi >= nvec) continue;
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = GET(row, j, e);
      if (need_lse) {
#pragma unroll
        for (int e = 0; e < 8; ++e) se += __expf(y[e] - raw_max);
      }
      if (brow) {
        const float4 b0 = reinterpret_cast<const float4*>(brow + (size_t)vi * 8)[0];
        const float4 b1 = reinterpret_cast<const float4*>(brow + (size_t)vi * 8)[1];
        y[0] += b0.x; y[1] += b0.y; y[2] += b0.z; y[3] += b0.w;
        y[4] += b1.x; y[5] += b1.y; y[6] += b1.z; y[7] += b1.w;
      }
      if (use_pen) {
        const uint4v c4 = *reinterpret_cast<const uint4v*>(crow + (size_t)vi * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t c = (c4[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
          if (c) {
            y[e] = y[e] > 0.f ? y[e] / rpen : y[e] * rpen;
            y[e] -= fpen * (float)c + ppen;
          }
        }
      }
      if (mrow) {
        const uint32_t m = (mrow[vi >> 2] >> ((vi & 3) * 8)) & 0xffu;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (!((m >> e) & 1u)) y[e] = -INFINITY;
      }
      row[j] = pack8(y);
    }
  }

  const float T = p.temperature[b];
  int token = 0;
  float raw_lse = __builtin_nanf("");
  if (T <= 0.f) {
    if (need_lse) {
      if (!processed) {
OPAQUE_ROW(row);
#pragma unroll
        for (int j = 0; j < SLOTS; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) se += __expf(GET(row, j, e) - raw_max);
      }
      raw_lse = raw_max + __logf(block_sum(se, sred));
    }
    // ---- greedy: argmax (lowest index on ties).  The row maximum is known (the raw max; a processed row
    // takes one max pass), so the argmax is the lowest index holding it — instead of a value-and-index
    // compare chain with a branch per element.  (Padding past V holds -inf: it can only match
    // a row that is -inf everywhere, whose answer, index 0, is found first.)
    float gm = raw_max;
    if (processed) {
      float ym = -INFINITY;
OPAQUE_ROW(row);
#pragma unroll
      for (int j = 0; j < SLOTS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) ym = fmaxf(ym, GET(row, j, e));
      gm = block_max(ym, sred);
    }
    // the thread's elements visited from its highest index down, the last match wins: its lowest index,
    // one compare + one select per element, no branch
    int bi = 0x7fffffff;
OPAQUE_ROW(row);
#pragma unroll
    for (int j = SLOTS - 1; j >= 0; --j)
#pragma unroll
      for (int e = 7; e >= 0; --e) {
        bi = GET(row, j, e) == gm ? (j * kSampT + t) * 8 + e : bi;
      }
    int cand = bi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    __syncthreads();
    if ((t & 63) == 0) sredi[t >> 6] = cand;
    __syncthreads();
    cand = (t & 63) < (kSampT / 64) ? sredi[t & 63] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    token = cand == 0x7fffffff ? 0 : cand;
  } else {
    const float invT = 1.f / T;
    float ymax = raw_max;  // unprocessed row: the processed max IS the raw max (no extra pass)
    if (processed) {
      float ym = -INFINITY;
OPAQUE_ROW(row);
#pragma unroll
      for (int j = 0; j < SLOTS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) ym = fmaxf(ym, GET(row, j, e));
      ymax = block_max(ym, sred);
    }
    if (!(ymax > -INFINITY)) ymax = 0.f;  // every token masked: all u = 0 (the argmax fallback below)
    const uint32_t kOne2 = 0x00010001u, kH1 = 0x3C003C00u;
    // ---- one exp per element: the row becomes u_i = exp((y_i - ymax)/T) in [0, 1] as packed fp16.
    // Non-negative fp16 bit patterns are order-preserving, so every later threshold search compares
    // raw 16-bit keys and sums fp16 values: no transcendental inside the searches.  The same pass
    // sums this thread's share of Z (over the ROUNDED values, as every later mass is).
    float zloc = 0.f;
    // unprocessed row + logprobs wanted: the raw exp sum needs its own pass over the raw values (fusing
    // it into the pass below doubles that pass's live values and the SLOTS=16 instance spills)
    if (need_lse && !processed) {
OPAQUE_ROW(row);
#pragma unroll
      for (int j = 0; j < SLOTS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) se += __expf(GET(row, j, e) - raw_max);
    }
    // u = 2^(y * c1 + c0), c1 = log2(e) / T, c0 ~ -ymax * c1 rounded so that the exponent of y = ymax is
    // >= 0: with v_cvt_pkrtz (round toward zero) the max element is exactly 1.0 (0x3C00) and every other
    // element (at least one bf16 ulp below it, far above the fp32 rounding of c0) below 1; y = -inf gives
    // exactly 0.  One fma + one exp per element, two values per pack, their (rounded) sum by one v_dot2
    // against (1, 1)
    const float c1 = invT * 1.4426950408889634f;
    float c0 = -ymax * c1;
    if (__builtin_fmaf(ymax, c1, c0) < 0.f)  // one ulp toward +inf (c0 != 0 here)
      c0 = __uint_as_float(__float_as_uint(c0) + (c0 > 0.f ? 1u : 0xffffffffu));
    const half2v ones2 = {(_Float16)1.f, (_Float16)1.f};
OPAQUE_ROW(row);
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float y0 = GET(row, j, 2 * c), y1 = GET(row, j, 2 * c + 1);
        const auto h = __builtin_amdgcn_cvt_pkrtz(__builtin_amdgcn_exp2f(__builtin_fmaf(y0, c1, c0)),
                                                  __builtin_amdgcn_exp2f(__builtin_fmaf(y1, c1, c0)));
        const uint32_t w = __builtin_bit_cast(uint32_t, h);
        zloc = __builtin_amdgcn_fdot2(as_h2(w), ones2, zloc, false);
        row[j][c] = w;
      }
    }
    float Z;
    if (need_lse) {  // both sums in one block reduction
      const float zw = wave_sum(zloc), sw = wave_sum(se);
      __syncthreads();
      if (lane == 0) {
        sred[wid] = zw;
        sred[16 + wid] = sw;
      }
      __syncthreads();
      Z = wave_sum(lane < kSampT / 64 ? sred[lane] : 0.f);
      raw_lse = raw_max + __logf(wave_sum(lane < kSampT / 64 ? sred[16 + lane] : 0.f));
    } else {
      Z = block_sum(zloc, sred);
    }
    // mass of the elements with key >= KEY (macro, not a lambda: a by-reference capture of `row`
    // makes it addressable and sends it to scratch)
#define MASS_LOCAL(KEY, OUT)                                                           \
  do {                                                                                 \
    OPAQUE_ROW(row);                                                                   \
    const uint32_t _t2 = thr1x2(KEY);                                                  \
    float _s = 0.f;                                                                    \
    _Pragma("unroll") for (int j = 0; j < SLOTS; ++j) {                                \
      mass2(_s, row[j][0], row[j][1], _t2, kOne2, kH1);                                \
      mass2(_s, row[j][2], row[j][3], _t2, kOne2, kH1);                                \
    }                                                                                  \
    OUT = dot_read(_s);                                                                \
  } while (0)
#define MASS_GE(KEY, OUT)        \
  do {                           \
    float _l;                    \
    MASS_LOCAL(KEY, _l);         \
    OUT = block_sum(_l, sred);   \
  } while (0)
    uint32_t tau_k = 0;  // top-k: keep elements with key >= tau_k
    const int k = p.top_k[b];
    if (k > 0) {
      uint32_t lo = 0, hi = 0x3C00u;  // keys of [0, 1.0]
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        const uint32_t t2 = thr1x2(mid);
        uint32_t c2 = 0u;
OPAQUE_ROW(row);
#pragma unroll
        for (int j = 0; j < SLOTS; ++j) {
          count2(c2, row[j][0], row[j][1], t2, kOne2);
          count2(c2, row[j][2], row[j][3], t2, kOne2);
        }
        if (block_sum_i((int)((c2 & 0xffffu) + (c2 >> 16)), sredi) >= k)
          lo = mid;
        else
          hi = mid - 1;
      }
      tau_k = lo;
    }
    // the filters other than top-p are plain lower bounds on the key
    uint32_t L0 = tau_k;
    const float mp = p.min_p[b];
    if (mp > 0.f) L0 = max(L0, (uint32_t)h2bits(mp));        // u_i >= min_p  (u_max = 1)
    const float ta = p.top_a[b];
    if (ta > 0.f) L0 = max(L0, (uint32_t)h2bits(fminf(ta / Z, 1.f)));  // p_i >= top_a p_max^2 <=> u_i >= top_a / Z
    if (L0 > 0x3C00u) L0 = 0x3C00u;                            // never filter out the argmax (u = 1)
    if (L0 == 0u) L0 = 1u;                                     // zero-mass elements are never kept
    // ---- top-p by rejection first (exact): draw s from the distribution over {key >= L0}; s is in the
    // nucleus {key >= tau_p} iff the mass strictly above it is < top_p * mass(top-k set).  Accepted
    // (probability >= top_p), s is exactly a draw from the nucleus-and-filters distribution.  Rejected,
    // tau_p > key_s is known: the exact search for tau_p starts there and a fresh uniform is drawn
    // over {key >= max(tau_p, L0)} — the result is again exactly distributed (the fallback does not
    // depend on the rejected draw).  Saves the ~14 block-wide passes of a threshold search per row in
    // the common case.
    const float tp = p.top_p[b];
    float target = 0.f;
    if (tp < 1.f) {
      float mk = Z;
      if (tau_k > 0u) MASS_GE(tau_k, mk);
      target = tp * mk;
    }
    uint32_t ctr[4] = {(uint32_t)p.offsets[b], (uint32_t)(p.offsets[b] >> 32), 0u, 0u};
    philox4x32(ctr, (uint32_t)p.seeds[b], (uint32_t)(p.seeds[b] >> 32));
    uint32_t tau = L0;
    bool check = tp < 1.f;
    int found = 0;
#pragma unroll 1
    for (int attempt = 0; attempt < 2; ++attempt) {
      // ---- inverse-CDF draw over {key >= tau} (order: thread-major, then slot, then element) ----
      float local = 0.f;
      if (tau <= 1u)
        local = zloc;  // every positive element is kept: the thread's share of Z
      else
        MASS_LOCAL(tau, local);
      // exclusive scan of `local` over threads
      float incl = local;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float n = __shfl_up(incl, o, 64);
        if (lane >= o) incl += n;
      }
      __syncthreads();
      if (lane == 63) s_scan[wid] = incl;
      __syncthreads();
      float wave_off = 0.f, total = 0.f;
      for (int w = 0; w < kSampT / 64; ++w) {
        const float sw = s_scan[w];
        if (w < wid) wave_off += sw;
        total += sw;
      }
      const float excl = wave_off + incl - local;
      const float u01 = (((attempt == 0 ? ctr[0] : ctr[1]) >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float u = u01 * total;
      // The owner: the lowest thread whose [excl, excl + local) holds u — or, when rounding put u at or
      // past the end, the last thread with mass (its last kept element is taken).  Its packed u go to
      // LDS and ONE wave walks them (two elements per dword, an exclusive scan over the lanes) instead
      // of a single lane stepping through 8 * SLOTS elements with a branch each.
      int cand = (local > 0.f && u >= excl && u < excl + local) ? t : 0x7fffffff;
      int lastt = local > 0.f ? t : -1;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        cand = min(cand, __shfl_xor(cand, o, 64));
        lastt = max(lastt, __shfl_xor(lastt, o, 64));
      }
      __syncthreads();
      if (lane == 0) {
        sredi[wid] = cand;
        sredi[16 + wid] = lastt;
      }
      __syncthreads();
      cand = lane < (kSampT / 64) ? sredi[lane] : 0x7fffffff;
      lastt = lane < (kSampT / 64) ? sredi[16 + lane] : -1;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        cand = min(cand, __shfl_xor(cand, o, 64));
        lastt = max(lastt, __shfl_xor(lastt, o, 64));
      }
      const bool past_end = cand == 0x7fffffff;
      const int owner = past_end ? lastt : cand;  // block-uniform
      found = 0x7fffffff;
      if (owner >= 0) {
        if (t == owner) {
#pragma unroll
          for (int j = 0; j < SLOTS; ++j)
#pragma unroll
            for (int c = 0; c < 4; ++c) s_own[j * 4 + c] = row[j][c];
          s_oexcl = excl;
        }
        __syncthreads();
        if (t < 64) {
          constexpr int ND = SLOTS * 4, P = (ND + 63) / 64;  // lane: dwords [lane*P, lane*P + P)
          float v[2 * P];
          float sl = 0.f;
#pragma unroll
          for (int q = 0; q < P; ++q) {
            const int d = lane * P + q;
            const uint32_t w = d < ND ? s_own[d] : 0u;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t kk = h ? (w >> 16) : (w & 0xffffu);
              // tau >= 1: zero-mass elements are never kept
              v[2 * q + h] = kk >= tau ? (float)__builtin_bit_cast(_Float16, (uint16_t)kk) : 0.f;
              sl += v[2 * q + h];
            }
          }
          float incl = sl;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const float n = __shfl_up(incl, o, 64);
            if (lane >= o) incl += n;
          }
          float acc = s_oexcl + incl - sl;
          int mine = -1, lastk = -1;
#pragma unroll
          for (int e = 0; e < 2 * P; ++e)
            if (v[e] > 0.f) {
              acc += v[e];
              lastk = e;
              if (mine < 0 && u < acc) mine = e;
            }
          const unsigned long long hit = __ballot(mine >= 0 && !past_end);
          int sel_lane, sel_e;
          if (hit) {
            sel_lane = __ffsll((long long)hit) - 1;
            sel_e = __shfl(mine, sel_lane, 64);
          } else {  // rounding at the owner's top edge, or u past the end: its last kept element
            const unsigned long long any = __ballot(lastk >= 0);
            sel_lane = 63 - __clzll((long long)any);
            sel_e = __shfl(lastk, sel_lane, 64);
          }
          if (lane == sel_lane) {
            const int d = lane * P + (sel_e >> 1);
            const uint32_t w = s_own[d];
            s_found = ((d >> 2) * kSampT + owner) * 8 + 2 * (d & 3) + (sel_e & 1);
            s_fkey = (sel_e & 1) ? (w >> 16) : (w & 0xffffu);
          }
        }
        __syncthreads();
        found = s_found;
      }
      if (found == 0x7fffffff) {
        // u landed past the last kept element through rounding: fall back to argmax (key 0x3C00: always
        // inside the nucleus)
        float bv = -INFINITY;
        int bi = 0x7fffffff;
OPAQUE_ROW(row);
#pragma unroll
        for (int j = 0; j < SLOTS; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = GETU(row, j, e);
            const int idx = (j * kSampT + t) * 8 + e;
            if (v > bv || (v == bv && idx < bi)) {  // padding past V has u = 0 < u_max = 1
              bv = v;
              bi = idx;
            }
          }
        const float gm = block_max(bv, sred);
        int cand = (bv == gm) ? bi : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
        __syncthreads();
        if (lane == 0) sredi[wid] = cand;
        __syncthreads();
        cand = lane < (kSampT / 64) ? sredi[lane] : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
        found = cand == 0x7fffffff ? 0 : cand;
        break;
      }
      if (!check) break;
      // ---- nucleus test of the draw (s_fkey: the drawn element's key, written by the walk) ----
      const uint32_t ks = s_fkey;
      float above;
      MASS_GE(ks + 1u, above);
      if (above < target) break;  // accepted (block-uniform)
      // rejected: tau_p > ks.  Exact search for the largest key with mass(>= key) >= target.
      uint32_t lo = ks + 1u, hi = 0x3C00u;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        float mm;
        MASS_GE(mid, mm);
        if (mm >= target)
          lo = mid;
        else
          hi = mid - 1;
      }
      tau = max(lo, L0);
      check = false;
    }
#undef MASS_GE
    token = found;
  }
  if (K > 0 && t < 64) {  // one wave: rank-sort the collected top-K candidates (value desc, index asc)
    const int n = min(s_ccount, kCollect);
    for (int r = n + t; r < K; r += 64) {  // fewer finite values than K: empty slots
      p.out_topk_ids[(size_t)b * K + r] = -1;
      p.out_topk_lp[(size_t)b * K + r] = -INFINITY;
    }
    if (t < n) {
      const float v = s_cval[t];
      const int ix = s_cidx[t];
      int rank = 0;
      for (int u = 0; u < n; ++u) {
        const float w = s_cval[u];
        rank += (w > v) || (w == v && s_cidx[u] < ix);
      }
      if (rank < K) {
        p.out_topk_ids[(size_t)b * K + rank] = ix;
        p.out_topk_lp[(size_t)b * K + rank] = v - raw_lse;
      }
    }
  }
  if (t == 0) {
    p.out_token[b] = token;
    p.out_logprob[b] = bf2f(lrow[token]) - raw_lse;
    if (p.counts && crow_i >= 0) {
      uint16_t* c = p.counts + (size_t)crow_i * p.V + token;
      if (*c < 0xffffu) *c += 1;
    }
  }
}

}  // namespace lwc

extern "C" int lwc_sample(const void* logits, int ld, int V, int B, const float* temperature, const float* top_p,
                          const int* top_k, const float* min_p, const float* top_a, const float* freq_pen,
                          const float* pres_pen, const float* rep_pen, void* counts, const int* count_rows,
                          const float* bias, const int* bias_rows, const unsigned int* mask, const int* mask_rows,
                          const unsigned long long* seeds, const unsigned long long* offsets, int num_logprobs,
                          int mask_logprobs, int need_logprob, int* out_token, float* out_logprob, int* out_topk_ids,
                          float* out_topk_lp, hipStream_t s) {
  using namespace lwc;
  if (V % 32 != 0 || num_logprobs < 0 || num_logprobs > kMaxTopK) return -1;
  if (B == 0) return 0;
  SampleParams p{(const bf16_t*)logits, ld, V, temperature, top_p, top_k, min_p, top_a, freq_pen, pres_pen, rep_pen,
                 (uint16_t*)counts, count_rows, bias, bias_rows, mask, mask_rows, seeds, offsets, num_logprobs,
                 mask_logprobs, need_logprob, out_token, out_logprob, out_topk_ids, out_topk_lp};
  const int nvec = V / 8;
  const int slots = (nvec + kSampT - 1) / kSampT;
  if (slots <= 4)
    sample_kernel<4><<<B, kSampT, 0, s>>>(p);
  else if (slots <= 8)
    sample_kernel<8><<<B, kSampT, 0, s>>>(p);
  else if (slots <= 16)
    sample_kernel<16><<<B, kSampT, 0, s>>>(p);
  else if (slots <= 20)
    sample_kernel<20><<<B, kSampT, 0, s>>>(p);
  else
    return -1;
  return (int)hipGetLastError();
}
