// K4 prefill_attn_varlen (causal, GQA) and K9c encoder_attn (bidirectional) — one flash-attention
// forward for packed variable-length sequences (cu_seqlens), head_dim 32 (bge-small), 64 or 128,
// bf16 in/out.
//
// Workgroup = 4 waves = 64 query rows of one (sequence, query head); each wave owns 16 rows and
// walks 32-key tiles that all 4 waves share through a double-buffered, XOR-swizzled LDS image
// (register-staged: next tile's global loads are issued before the current tile's MFMAs and written
// to LDS after them — cdna_hip_programming.md T14).
//
// Per wave and key tile (mfma_f32_16x16x32_bf16; lane l: r16 = l & 15, g = l >> 4):
//   S^T = K Q^T :  A = K rows from LDS (ds_read_b128, chunk XOR row swizzle: T2),
//                  B = Q^T held in registers for the whole kernel;
//                  C: lane reg r = S^T[key 4g + r][query r16]   (two 16-key subtiles)
//   O  += P V   :  A = the softmaxed S^T registers themselves (k permuted {4g+0..3, 16+4g+0..3}),
//                  B = V columns by ds_read_b64_tr_b16 (T10 hardware transpose), same permutation;
//                  C: lane reg r = O[query 4g + r][dim 16n + r16]
// so P never leaves registers.  Online softmax in the log2 domain; rows are finite-initialised
// (-1e30) so fully-masked tiles cannot produce NaN.
//
// PAGED mode (mixed chunked prefill, engine/engine.py): the keys / values of sequence s are read straight
// from the paged cache through its block table — K [NB, Hkv, 16, D] token-major, V [NB, Hkv, 4, D, 4]
// 4-token interleaved (the decode layout) — with key positions [0, k_lens[s]) and the sequence's queries
// the last len_q of them (a prompt chunk after its earlier chunks, or after a cached prefix).  A 32-key
// tile is exactly two blocks: each operand tile is two contiguous 4 KiB segments.  K is staged into the
// same swizzled row image; V keeps the interleaved layout in LDS (odd token groups XOR byte bit 7), where
// one ds_read_b64 returns a lane's 4 consecutive keys of one dim — the PV B operand without a transpose.
// V elements of keys past k_lens (the tail of the last block, stale bytes) are zeroed: P is 0 there, but
// 0 x a stale Inf / NaN would not be.  No per-layer gather of the cached keys into contiguous buffers.
#include <type_traits>

#include "common.h"

namespace lwc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short4v lds_short4;

LWC_DEVICE float4v mfma16p(const short8& a, const short8& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

constexpr int kQT = 64;  // query rows per workgroup
constexpr float kLazyRescale = 8.f;
constexpr int kKT = 32;  // keys per tile

struct PrefillParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* out;
  const int* cu_seqlens;
  const int* cu_seqlens_k;  // null: keys = queries; else sequence s attends keys [cu_k[s], cu_k[s+1]) and its
                            // queries are the LAST len_q of those positions (cached-prefix prefill)
  int q_stride, k_stride, v_stride, o_stride;  // elements per token row
  int Hq, Hkv, nseq, max_tiles;
  float scale;
  int causal;
  // PAGED: block tables [nseq, bt_stride] of the key cache; k_lens [nseq] key positions per sequence
  const int* block_tables;
  const int* k_lens;
  int bt_stride;
  // MX output (D = 128; the fp8 o projection's A operand, as the decode cascade kernel writes it): e4m3 rows
  // out8 [T, Hq * D] (row stride o_stride bytes) + e8m0 scales mx [Hq][mx_rows][4], one per 32 dims
  uint8_t* out8;
  uint8_t* mx;
  int mx_rows;
};

// The block tables come in as a const __restrict__ kernel argument (not through the params struct): the
// compiler may then read them with SCALAR loads.  As vector loads each block id needed an s_waitcnt
// vmcnt(0) — which also waits for the LDS-DMA of the tiles in flight and serialises the pipeline.
template <int D, bool PAGED>
__global__ void __launch_bounds__(256) prefill_attn_kernel(PrefillParams p, const int* __restrict__ block_tables) {
  constexpr int CPR = D / 8;                // 16-byte chunks per row
  constexpr int KS = D / 32;                // k-steps for S
  constexpr int NS = D / 16;                // n-subtiles for O
  constexpr int TILE_BYTES = kKT * D * 2;   // one K or V tile
  constexpr int NST = 3;                    // LDS stages: tiles t (computing), t+1 and t+2 (in flight)
  constexpr int INSTR = TILE_BYTES / 1024;  // 1 KiB LDS-DMA wave-instructions per operand tile
  constexpr int PER_WAVE = 2 * INSTR / 4;   // K + V wave-instructions each of the 4 waves issues per tile
  constexpr int RPI = 1024 / (2 * D);       // tile rows per wave-instruction
  static_assert(PER_WAVE >= 1 && (2 * INSTR) % 4 == 0, "tile must split evenly over 4 waves");
  __shared__ __attribute__((aligned(16))) char smem[NST * 2 * TILE_BYTES];  // [stage][K|V]

  const int seq = blockIdx.x / p.max_tiles, qtile = blockIdx.x % p.max_tiles;
  const int hq = blockIdx.y, kvh = hq / (p.Hq / p.Hkv);
  const int s0 = p.cu_seqlens[seq], len = p.cu_seqlens[seq + 1] - s0;
  const int q0 = qtile * kQT;
  if (q0 >= len) return;  // whole workgroup exits together (uniform)
  // keys: the sequence's own rows, or (cached prefix / PAGED) a longer key range whose last len rows are
  // the queries
  const int ks0 = PAGED ? 0 : p.cu_seqlens_k ? p.cu_seqlens_k[seq] : s0;
  // wave-uniform by construction; readfirstlane lets the compiler keep the DMA buffer resources in SGPRs
  const int klen = __builtin_amdgcn_readfirstlane(PAGED ? p.k_lens[seq]
                                                        : p.cu_seqlens_k ? p.cu_seqlens_k[seq + 1] - ks0 : len);
  const int* bt = PAGED ? block_tables + (size_t)seq * p.bt_stride : nullptr;
  const int qoff = klen - len;  // key position of query row 0
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int qrow = q0 + wid * 16 + r16;  // this lane's query (as B-operand column)

  short8 qf[KS];
  {
    const int qr = qrow < len ? qrow : len - 1;
    const bf16_t* qp = p.q + (size_t)(s0 + qr) * p.q_stride + hq * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const short8*>(qp + 32 * s + 8 * g);
  }
  const float sl2 = p.scale * 1.4426950408889634f;

  const int q_last = min(len, q0 + kQT) - 1;
  const int kv_end = p.causal ? q_last + 1 + qoff : klen;
  const int ntiles = (kv_end + kKT - 1) / kKT;

  // ---- LDS-DMA staging (buffer loads straight into LDS, 16 B per lane, no register round trip) ----
  // Wave-instruction j of a tile (j < INSTR: K image, else V image) writes the image's bytes
  // [1 KiB * (j % INSTR), +1 KiB) lane-linearly; the image's swizzle is applied to the SOURCE address.  Keys
  // at or past klen are out of the buffer resource's range: the hardware writes zeros, no request.
  //  K (and non-paged V) image: row r (key in tile), 16 B chunk c at ((r * CPR) + (c ^ (r % CPR))) * 16.
  //  Paged V image: the tile's two interleaved block segments [4 token groups][D][4], odd groups' bytes
  //  XOR bit 7 (the layout the ds_read_b64 PV operand reads conflict-free).
  const int lrow = lane / CPR, lpc = lane % CPR;
  auto issue = [&](int tile, int stage) {
    char* kb = smem + stage * 2 * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int j = wid + 4 * i;  // wave-uniform
      const bool isv = j >= INSTR;
      const int jj = isv ? j - INSTR : j;
      char* dst = kb + (isv ? TILE_BYTES : 0) + jj * 1024;
      if constexpr (PAGED) {
        // the instruction's 1 KiB lies in one block segment: K rows jj*RPI.. or V bytes jj*1024..
        const int half = isv ? (jj * 1024) / 4096 : (jj * RPI) / 16;
        const int blk = bt[__builtin_amdgcn_readfirstlane(2 * tile + half)];
        const int valid = min(max(klen - (tile * kKT + half * 16), 0), 16);  // keys of this block in range
        const bf16_t* segp = (isv ? p.v : p.k) + ((size_t)blk * p.Hkv + kvh) * 16 * D;
        uint32_t vo, nrec;
        if (!isv) {
          const int r = jj * RPI + lrow;  // key in tile
          vo = (uint32_t)(((r % 16) * CPR + (lpc ^ (r % CPR))) * 16);
          nrec = (uint32_t)(valid * D * 2);
        } else {
          const int P = jj * 1024 + lane * 16;                     // byte of the V image
          const int bsrc = (P ^ (((P / (D * 8)) & 1) << 7)) % 4096;  // byte in the block segment
          vo = (uint32_t)bsrc;
          nrec = (uint32_t)(((valid + 3) / 4) * D * 8);  // whole token groups; a partial group is fixed up
        }
        // readfirstlane: uniform already, but the compiler may compute it on the VALU (then every DMA became a
        // waterfall loop over "divergent" resources)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)segp, (short)0, __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, vo, 0, 0, 0);
      } else {
        const int r = jj * RPI + lrow;
        const int key = tile * kKT + r;
        const int stride = isv ? p.v_stride : p.k_stride;
        const bf16_t* base = (isv ? p.v : p.k) + (size_t)ks0 * stride + kvh * D;
        const uint32_t vo = (uint32_t)(key * stride * 2 + ((lpc ^ (r % CPR)) * 16));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)base, (short)0, (uint32_t)(klen * stride * 2), 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, vo, 0, 0, 0);
      }
    }
  };

  float4v o[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) o[n] = float4v{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;

  issue(0, 0);
  if (ntiles > 1) issue(1, 1);
  // loop-invariant LDS read offsets of this lane (the stage base is a compile-time immediate below)
  int kofs[KS], vofs[NS];
#pragma unroll
  for (int s = 0; s < KS; ++s) kofs[s] = (r16 * CPR + ((4 * s + g) ^ (r16 & (CPR - 1)))) * 16;
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    if constexpr (PAGED) {
      vofs[n] = ((g * D + 16 * n + r16) << 3) ^ ((g & 1) << 7);
    } else {
      const int qq = r16 >> 2, pp = r16 & 3;
      const int rowA = 4 * g + qq, chunk = 2 * n + (pp >> 1);
      vofs[n] = (rowA * CPR + (chunk ^ (rowA & (CPR - 1)))) * 16 + (pp & 1) * 8;
    }
  }
  auto tile_step = [&](const int t, auto stage) {
    constexpr int buf = decltype(stage)::value;
    // own DMA of tile t landed (tile t+1's may stay in flight), then every wave's (barrier); the barrier also
    // ends every wave's reads of tile t-1, whose stage tile t+2 now refills
    if (t + 1 < ntiles)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < ntiles) issue(t + 2, (t + 2) % NST);
    if constexpr (PAGED) {
      // the last tile's partially valid token group holds stale V bytes of keys >= klen (P is 0 there, but
      // 0 x a stale Inf / NaN would not be): zero them (uniform branch: the last tile only)
      const int tk = klen - t * kKT;  // keys of this tile in range
      if (tk < kKT && (tk & 3)) {
        char* vimg = smem + buf * 2 * TILE_BYTES + TILE_BYTES;
        const int half = tk / 16, grp = (tk % 16) / 4;
        if (threadIdx.x < D) {
          for (int r = tk & 3; r < 4; ++r) {
            const int bsrc = half * 4096 + grp * D * 8 + threadIdx.x * 8 + r * 2;
            *reinterpret_cast<bf16_t*>(vimg + (bsrc ^ (((bsrc / (D * 8)) & 1) << 7))) = 0;
          }
        }
        __syncthreads();
      }
    }
    const char* kb = smem + buf * 2 * TILE_BYTES;  // compile-time stage: LDS reads take immediate offsets
    const char* vb = kb + TILE_BYTES;
    // ---- S^T for the two 16-key subtiles ----
    float4v sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const short8 ka = *reinterpret_cast<const short8*>(kb + kofs[s]);
      const short8 kbv = *reinterpret_cast<const short8*>(kb + kofs[s] + 16 * CPR * 16);  // keys 16..31
      sa = mfma16p(ka, qf[s], sa);
      sb = mfma16p(kbv, qf[s], sb);
    }
    // ---- mask + online softmax (per query r16) ----
    float pa[4], pb[4];
    float mx = -1e30f;
    // interior tile (every key in range and, causal, at or before the wave's first query): no mask
    const int tlast = t * kKT + kKT - 1;
    if (tlast < klen && (!p.causal || tlast <= q0 + wid * 16 + qoff)) {  // wave-uniform
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pa[r] = sa[r] * sl2;
        pb[r] = sb[r] * sl2;
        mx = fmaxf(mx, fmaxf(pa[r], pb[r]));
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ka_ = t * kKT + 4 * g + r, kb_ = ka_ + 16;
        const bool va = ka_ < klen && (!p.causal || ka_ <= qrow + qoff);
        const bool vbk = kb_ < klen && (!p.causal || kb_ <= qrow + qoff);
        pa[r] = va ? sa[r] * sl2 : -INFINITY;
        pb[r] = vbk ? sb[r] * sl2 : -INFINITY;
        mx = fmaxf(mx, fmaxf(pa[r], pb[r]));
      }
    }
    mx = row_max4(mx);
    // lazy rescale (log2 domain): the running max only moves — and O / l are rescaled — when some row's new
    // scores exceed it by more than kLazyRescale, so P <= 2^8 and most tiles skip the cross-lane alpha
    // shuffles and the O multiplies
    if (__any(mx > m + kLazyRescale)) {  // wave-uniform
      const float m_new = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - m_new);
      l *= alpha;
      m = m_new;
      float al[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) al[r] = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
      for (int n = 0; n < NS; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[n][r] *= al[r];
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[r] = __builtin_amdgcn_exp2f(pa[r] - m);  // raw v_exp_f32: -inf -> 0, arguments <= 8
      pb[r] = __builtin_amdgcn_exp2f(pb[r] - m);
      rs += pa[r] + pb[r];
    }
    l += row_sum4(rs);
    short8 pf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = (short)f2bf(pa[r]);
      pf[4 + r] = (short)f2bf(pb[r]);
    }
    // ---- O += P V, V columns via the hardware transpose read ----
    if constexpr (PAGED) {
      // lane: keys 4g..4g+3 (block A half) and 16+4g..16+4g+3 (block B half) of dim 16n + r16, 8 B each
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        const int off = vofs[n];
        const short4v va4 = *reinterpret_cast<const short4v*>(vb + off);
        const short4v vb4 = *reinterpret_cast<const short4v*>(vb + TILE_BYTES / 2 + off);
        short8 vf;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          vf[r] = va4[r];
          vf[4 + r] = vb4[r];
        }
        o[n] = mfma16p(pf, vf, o[n]);
      }
    } else
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int offA = vofs[n], offB = vofs[n] + 16 * CPR * 16;  // rows 4g+qq and 16+4g+qq: same swizzle
      const short4v va4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(vb + offA));
      const short4v vb4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(vb + offB));
      short8 vf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vf[r] = va4[r];
        vf[4 + r] = vb4[r];
      }
      o[n] = mfma16p(pf, vf, o[n]);
    }
  };
  for (int t = 0; t < ntiles; t += NST) {  // unrolled by the stage count: every stage base is a constant
    tile_step(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile_step(t + 1, std::integral_constant<int, 1>{});
    if (t + 2 < ntiles) tile_step(t + 2, std::integral_constant<int, 2>{});
  }

  // ---- epilogue: normalise, stage the wave's 16 x D tile through LDS, 16 B stores ----
  float linv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float lr = __shfl(l, 4 * g + r, 64);
    linv[r] = lr > 0.f ? 1.f / lr : 0.f;
  }
  __syncthreads();
  bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 16 * D;
#pragma unroll
  for (int n = 0; n < NS; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) ot[(4 * g + r) * D + 16 * n + r16] = f2bf(o[n][r] * linv[r]);
  __syncthreads();
  if constexpr (D == 128) {
    if (p.out8 != nullptr) {  // uniform
      // lane: row lane / 4 of the wave's 16, 32-dim block lane % 4 -> 32 e4m3 bytes + one e8m0 scale
      const int row = lane >> 2, b = lane & 3;
      const int qr = q0 + wid * 16 + row;
      float v[32];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4v*>(ot + row * D + 32 * b + 8 * c), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[8 * c + j] = f[j];
      }
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
      const int e = mx_exp(amax);
      const float sc = __builtin_amdgcn_ldexpf(1.f, -e);
      uint32_t w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i] * sc, v[4 * i + 1] * sc, 0, false);
        w[i] = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2] * sc, v[4 * i + 3] * sc, x, true);
      }
      if (qr < len) {
        uint8_t* dst = p.out8 + (size_t)(s0 + qr) * p.o_stride + hq * D + 32 * b;
        *reinterpret_cast<uint4v*>(dst) = uint4v{w[0], w[1], w[2], w[3]};
        *reinterpret_cast<uint4v*>(dst + 16) = uint4v{w[4], w[5], w[6], w[7]};
        p.mx[((size_t)hq * p.mx_rows + s0 + qr) * 4 + b] = (uint8_t)(e + 127);
      }
      return;
    }
  }
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int row = c / CPR, ch = c % CPR;
    const int qr = q0 + wid * 16 + row;
    if (qr < len)
      *reinterpret_cast<uint4v*>(p.out + (size_t)(s0 + qr) * p.o_stride + hq * D + ch * 8) =
          *reinterpret_cast<const uint4v*>(ot + row * D + ch * 8);
  }
}

}  // namespace lwc

extern "C" int lwc_prefill_attention(const void* q, const void* k, const void* v, void* out, const int* cu_seqlens,
                                     const int* cu_seqlens_k, int nseq, int max_seqlen, int q_stride, int k_stride, int v_stride, int o_stride,
                                     int Hq, int Hkv, int D, float scale, int causal, hipStream_t s) {
  using namespace lwc;
  if (Hq % Hkv != 0) return -1;
  if (nseq == 0 || max_seqlen == 0) return 0;
  const int max_tiles = (max_seqlen + kQT - 1) / kQT;
  PrefillParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)out, cu_seqlens, cu_seqlens_k,
                  q_stride, k_stride,
                  v_stride, o_stride, Hq, Hkv, nseq, max_tiles, scale, causal, nullptr, nullptr, 0,
                  nullptr, nullptr, 0};
  dim3 grid(nseq * max_tiles, Hq);
  if (D == 128)
    prefill_attn_kernel<128, false><<<grid, 256, 0, s>>>(p, nullptr);
  else if (D == 64)
    prefill_attn_kernel<64, false><<<grid, 256, 0, s>>>(p, nullptr);
  else if (D == 32)
    prefill_attn_kernel<32, false><<<grid, 256, 0, s>>>(p, nullptr);
  else
    return -1;
  return (int)hipGetLastError();
}

// The same with the output in MX form (D = 128, keys = queries): out8 [T, Hq * 128] e4m3 (row stride o8_stride
// bytes), mx [Hq][mx_rows >= T][4] e8m0 — what the fp8 o projection's block-scaled MFMAs read, so the bf16
// output and its row quantisation pass are gone.
extern "C" int lwc_prefill_attention_mx(const void* q, const void* k, const void* v, void* out8, void* mx,
                                        int mx_rows, const int* cu_seqlens, int nseq, int max_seqlen, int q_stride,
                                        int k_stride, int v_stride, int o8_stride, int Hq, int Hkv, float scale,
                                        int causal, hipStream_t s) {
  using namespace lwc;
  if (Hq % Hkv != 0 || o8_stride % 16 != 0) return -1;
  if (nseq == 0 || max_seqlen == 0) return 0;
  const int max_tiles = (max_seqlen + kQT - 1) / kQT;
  PrefillParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, nullptr, cu_seqlens, nullptr, q_stride,
                  k_stride, v_stride, o8_stride, Hq, Hkv, nseq, max_tiles, scale, causal, nullptr, nullptr, 0,
                  (uint8_t*)out8, (uint8_t*)mx, mx_rows};
  dim3 grid(nseq * max_tiles, Hq);
  prefill_attn_kernel<128, false><<<grid, 256, 0, s>>>(p, nullptr);
  return (int)hipGetLastError();
}

// Causal prefill of query chunks against a PAGED KV cache (D = 128, block size 16): sequence s has queries
// cu_seqlens[s]..cu_seqlens[s+1] = its key positions [k_lens[s] - len_q, k_lens[s]); its keys come from
// kc / vc through block_tables[s] (bt_stride entries per row, covering ceil(k_lens[s] / 16) blocks).
extern "C" int lwc_prefill_attention_paged(const void* q, const void* kc, const void* vc, void* out,
                                           const int* cu_seqlens, const int* block_tables, const int* k_lens,
                                           int bt_stride, int nseq, int max_seqlen, int q_stride, int o_stride, int Hq,
                                           int Hkv, int D, float scale, hipStream_t s) {
  using namespace lwc;
  if (Hq % Hkv != 0 || D != 128) return -1;
  if (nseq == 0 || max_seqlen == 0) return 0;
  const int max_tiles = (max_seqlen + kQT - 1) / kQT;
  PrefillParams p{(const bf16_t*)q, (const bf16_t*)kc, (const bf16_t*)vc, (bf16_t*)out, cu_seqlens, nullptr,
                  q_stride, 0, 0, o_stride, Hq, Hkv, nseq, max_tiles, scale, 1, block_tables, k_lens, bt_stride,
                  nullptr, nullptr, 0};
  dim3 grid(nseq * max_tiles, Hq);
  prefill_attn_kernel<128, true><<<grid, 256, 0, s>>>(p, block_tables);
  return (int)hipGetLastError();
}
