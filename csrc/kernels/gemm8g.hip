// K6g' grouped fp8 GEMM on the 8-phase 256x256 schedule (the MoE expert FFNs of config 5):
//   C[r, :] = (A[a_rows[r], :] . W_g^T) * a_scale[a_rows[r]] * w_scale[g, :]   for rows r of group g
// with groups = the experts' contiguous row segments row_off[g]..row_off[g+1] (device table, no host
// sync, graph-capturable) and A gathered through a_rows (MoE dispatch without a permute copy).
//
// Why a second grouped kernel: the 128x128 register-staged kernel (gemm.hip) pays two barriers and a
// full LDS rewrite per 128-byte K step for 16 block-scaled MFMAs per wave — latency-bound at ~1.0-1.3
// PF/s fp8 (profiles/moe_r32.md: MFMA busy ~20 %).  Large decode batches give every expert >= 2 full
// 256-row tiles (T = 2048 tokens, top-2, 8 experts: 512 rows each), which is the dense 8-phase template's
// regime (csrc/kernels/gemm8p.hip, cdna_hip_programming.md §5 "The 256² 8-phase template"):
//   * 8 waves = 2 (M) x 4 (N), wave tile 128 x 64; K tile = 128 BYTES (= 128 e4m3), four 16 KiB LDS
//     units A0 A1 B0 B1 per K tile, two K-tile buffers (128 KiB), LDS-DMA (buffer_load ... lds) staging
//     with the swizzle on the SOURCE address, 4 phases per K tile with counted vmcnt, raw s_barrier and
//     the two wave rows staggered by one barrier — byte for byte the gemm8p pipeline;
//   * MFMA: the block-scaled mfma_scale_f32_16x16x128_f8f6f4 with unit e8m0 scales: a lane's two 16 B
//     fragments (k-chunks q and 4+q of the 128-byte slice) form one 32-byte operand, so a phase issues
//     8 MFMAs of twice the bf16 cycle count — the same MFMA cycles per phase as gemm8p at 2x the FLOPs;
//   * A rows: per-lane DMA source offsets from a_rows (rows past the group's end load a valid row of
//     the group and are masked at the store); W: the group's [N, K] slab through its own descriptor;
//   * epilogue: fp32 accumulators x activation row scale x weight channel scale -> bf16 -> LDS -> 16 B
//     row stores (rows < the group's end only).
// Work distribution: one 256 x 256 tile per workgroup; workgroup ids are dealt round-robin to the 8
// XCDs, and XCD x walks the n-tiles n = x (mod 8) with all m-tiles of an n-tile consecutive, so the
// weight tile of an expert is read from HBM once per XCD and reused from its L2 by the expert's other
// m-tiles.  Surplus slots (routing decides the m-tile count at run time) exit immediately.
#include "common.h"

namespace lwc {
namespace g8g {

typedef int v8i32 __attribute__((ext_vector_type(8)));

constexpr int kUnitB = 128 * 128;   // 128 rows x 128 B
constexpr int kBufB = 4 * kUnitB;   // one K tile: A0 A1 B0 B1
constexpr int kLdsB = 2 * kBufB;    // 128 KiB
constexpr int kUA0 = 0, kUA1 = kUnitB, kUB0 = 2 * kUnitB, kUB1 = 3 * kUnitB;

struct Params {
  const uint8_t* A;       // [rows_a, K] e4m3
  const uint8_t* W;       // [G][N, K] e4m3
  bf16_t* C;              // [rows, ldc]
  const int* row_off;     // [G + 1]
  const int* a_rows;      // [rows] or null
  const float* a_scale;   // [rows_a]
  const float* w_scale;   // [G][N]
  int G, N, K, lda, ldc;  // K in elements (= bytes), lda in elements
  int rows_a;             // rows of A (DMA bounds)
  int slots, n_tiles;     // m-tile slots per n-tile, n-tiles
  int rows_c;             // output rows when row_off is null (dense: G = 1)
  int gn;                 // grouped: n-tiles an XCD walks per m-slot before the next slot (>= 1)
  int skip_empty;         // skip the MFMAs of empty 64-row blocks (LWC_G8G_SKIP=0: A/B off)
  // MX activations (kMxOut producer / kMxA consumer): e8m0 block scales [K / 128][s_rows][4] bytes, block b
  // of a 128-byte K slice = its bytes [32b, 32b + 32).  (The block-scaled MFMA takes a lane's two 16-byte
  // fragments as K [16q, 16q + 16) and [64 + 16q, ...) of its 128 and scales K block b by the byte lane
  // group b supplies — measured, scripts/mx_probe.py.)
  const uint8_t* a_mx;    // kMxA: scales of A (a_scale unused)
  uint8_t* mx_out;        // kMxOut: scales of the e4m3 output (C is then e4m3 [rows, ldc bytes])
  int s_rows;             // rows of the scale planes
};

// kernel modes: output / A operand handling
constexpr int kPlain = 0;   // bf16 out, A per-row scaled
constexpr int kSwiglu = 1;  // SwiGLU epilogue, bf16 out
constexpr int kMxOut = 2;   // SwiGLU epilogue, e4m3 out with MX block scales (feeds a kMxA GEMM)
constexpr int kMxA = 3;     // bf16 out, A carries MX block scales
constexpr int kMxLds = 4096;  // kMxA: the two K buffers' scale tiles (256 rows x 4 blocks, twice: see the DMA)

// A block-scaled: the lane's e8m0 scale is byte OP of sa (its row's scale for the lane's K block)
template <int OP>
LWC_DEVICE float4v mfma8s(const uint4v& a0, const uint4v& a1, const uint4v& b0, const uint4v& b1, const float4v& c,
                          int sa) {
  const v8i32 av = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  const v8i32 bv = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, OP, sa, 0, 127);
}

// max over each quad of lanes
LWC_DEVICE float quad_max(float x) {
  x = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false)));  // ^1
  return fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false)));  // ^2
}

LWC_DEVICE float4v mfma8(const uint4v& a0, const uint4v& a1, const uint4v& b0, const uint4v& b1, const float4v& c) {
  const v8i32 av = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  const v8i32 bv = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
}

// grouped default: an XCD takes all of its n-tiles for one m-slot before the next slot (gn = n-tiles per XCD).
// Config 5's routed shapes at 4096 tokens, one MI355X, medians of 5 interleaved rounds (scripts/g8g_order_ab.py):
// gate|up + SwiGLU 908.1 -> 893.4 us, down 474.3 -> 466.7 us vs gn = 1 (the n-tile-major order); with the
// empty-block MFMA skip below as well 878.0 / 443.9 us.  LWC_G8G_GN overrides.
constexpr int kDefaultGn = 1 << 20;

LWC_DEVICE float silu8(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// SWIGLU: W's rows are gate / up interleaved in blocks of 32 (ops.swiglu_interleave per expert), so each
// wave's 64 columns are one gate block and its up block; the epilogue applies the scales, then
// silu(gate) * up, and writes [rows, N / 2] bf16 — the [rows, N] gate|up intermediate never reaches HBM.
template <int MODE>
__global__ void __launch_bounds__(512) gemm8g_kernel(Params p) {
  constexpr bool SWIGLU = MODE == kSwiglu || MODE == kMxOut;
  constexpr bool MXA = MODE == kMxA;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // ---- work item: XCD-grouped (n-tile, m-slot), then (group, m-tile) of the slot ----
  const int id = blockIdx.x, xcd = id & 7, local = id >> 3;
  int g = 0, m_begin = 0, m_end = 0, ntile = 0;
  if (p.row_off == nullptr) {
    // dense (G = 1, rows [0, rows_c), slots = m-tiles): XCD x runs a contiguous range of the GROUPED tile
    // order (8 m-tiles x every n-tile, m fastest), so the workgroups resident on an XCD at once share a
    // few A and W panels in its L2 instead of each streaming its own A panel from HBM (at the embedder's
    // 266k-row prefill the expert-style n-major order re-read A once per n-tile)
    const int T = p.slots * p.n_tiles, per = (T + 7) / 8, t = xcd * per + local;
    if (local >= per || t >= T) return;  // uniform
    const int group = 8 * p.n_tiles, first_m = (t / group) * 8, gsz = min(p.slots - first_m, 8), in = t % group;
    m_begin = (first_m + in % gsz) * 256;
    m_end = p.rows_c;
    ntile = in / gsz;
  } else {
    // an XCD owns n-tiles xcd, xcd + 8, ...; it walks them in windows of gn: every m-slot (the experts'
    // row tiles back to back) takes the window's gn n-tiles in a row, so the workgroups resident at once
    // hold ~32/gn consecutive row tiles x gn weight panels (each expert's panel still read once, every A
    // tile once per window instead of once per n-tile)
    const int w = p.slots * p.gn, in = local % w;
    ntile = ((local / w) * p.gn + in % p.gn) * 8 + xcd;
    int slot = in / p.gn;
    if (ntile >= p.n_tiles) return;  // uniform
    for (; g < p.G; ++g) {
      const int r0 = p.row_off[g], r1 = p.row_off[g + 1];
      const int nt = (r1 - r0 + 255) / 256;
      if (slot < nt) {
        m_begin = r0 + slot * 256;
        m_end = r1;
        break;
      }
      slot -= nt;
    }
    if (g >= p.G) return;  // surplus slot (uniform)
  }
  const int n0 = ntile * 256;
  const int KT = p.K / 128;

  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int wr = wid >> 2, wc = wid & 3;

  // per-thread DMA geometry: unit u, instruction i -> unit row ru = i*64 + tid/8 at LDS chunk tid%8, holding
  // global chunk chk of that row (swizzle on the source).  A rows are gathered: source row of tile row t.
  const int chk = ((tid & 7) ^ ((tid >> 4) & 7)) * 16;
  uint32_t voA[2][2], voW[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int r = m_begin + i * 128 + h * 64 + (tid >> 3);
      if (r >= m_end) r = m_begin;  // a valid row of the group; its outputs are never stored
      const int src = p.a_rows ? p.a_rows[r] : r;
      voA[h][i] = (uint32_t)(src * p.lda + chk);
      voW[h][i] = (uint32_t)(((2 * i + (tid >> 8)) * 64 + h * 32 + ((tid >> 3) & 31)) * p.K + chk);
    }
  const int dst_lane0 = wid * 64 * 16;
  const int sw = (r16 >> 1) & 7;
  const int off0 = r16 * 128 + ((q ^ sw) << 4), off1 = r16 * 128 + (((4 + q) ^ sw) << 4);

  // kMxA: the tile's scales ([row][4 blocks], one dword per row) DMA'd with unit A0, one dword piece per thread
  // (an LDS-DMA lands every lane's piece on a 4-byte slot, so no narrower piece packs): threads 256..511 load
  // a second copy, keeping every wave's vmcnt count equal; a lane then reads its 8 fragments' bytes
  uint32_t voS = 0u;
  if constexpr (MXA) {
    int r = m_begin + (tid & 255);
    if (r >= m_end) r = m_begin;
    voS = (uint32_t)(r * 4);
  }
  const __amdgpu_buffer_rsrc_t rS = uniform_rsrc(p.a_mx, MXA ? (p.K / 128) * p.s_rows * 4 : 0);
  const __amdgpu_buffer_rsrc_t rA = uniform_rsrc(p.A, p.rows_a * p.lda);
  const __amdgpu_buffer_rsrc_t rW = uniform_rsrc(p.W + ((size_t)g * p.N + n0) * p.K, min(p.N - n0, 256) * p.K);
  auto stage = [&](int u, uint8_t* buf, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      auto* dst = (__attribute__((address_space(3))) void*)(buf + u * kUnitB + i * 512 * 16 + dst_lane0);
      if (u < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, voA[u][i], kt * 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, dst, 16, voW[u - 2][i], kt * 128, 0, 0);
    }
    if constexpr (MXA) {
      if (u == 0) {
        auto* dst = (__attribute__((address_space(3))) void*)(smem + kLdsB + (kt & 1) * 2048 + (wid >> 2) * 1024 +
                                                              (wid & 3) * 256);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rS, dst, 4, voS, kt * p.s_rows * 4, 0, 0);
      }
    }
  };
  auto rd = [&](const uint8_t* u, int row0, uint4v& f0, uint4v& f1) {
    f0 = *reinterpret_cast<const uint4v*>(u + row0 * 128 + off0);
    f1 = *reinterpret_cast<const uint4v*>(u + row0 * 128 + off1);
  };

  float4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = float4v{0.f, 0.f, 0.f, 0.f};

  uint4v a[4][2], b0[2][2], b1[2][2];
  int sc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // kMxA: this K tile's scale (block q) of the lane's 8 row fragments
  auto mma = [&](int i0, int j0, const uint4v (&bb)[2][2]) {
    if constexpr (MXA) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[i0 + i][j0 + jj] = mfma8s<0>(a[i][0], a[i][1], bb[jj][0], bb[jj][1], acc[i0 + i][j0 + jj], sc[i0 + i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[i0 + i][j0 + jj] = mfma8(a[i][0], a[i][1], bb[jj][0], bb[jj][1], acc[i0 + i][j0 + jj]);
    }
  };
  auto rdA = [&](const uint8_t* buf, int u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) rd(buf + u, wr * 64 + i * 16, a[i][0], a[i][1]);
  };
  auto rdB = [&](const uint8_t* buf, int u, uint4v (&bb)[2][2]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) rd(buf + u, wc * 32 + jj * 16, bb[jj][0], bb[jj][1]);
  };

#define G8_BAR() __builtin_amdgcn_s_barrier()
  // rows of this wave row that hold data (wave-uniform): a ragged last tile of an expert (on average half of
  // it) skips the MFMAs of its empty 64-row blocks — the barriers, LDS reads and DMA stay, so the two wave
  // rows keep their schedule
  const int live = p.skip_empty ? __builtin_amdgcn_readfirstlane(m_end - m_begin - wr * 128) : 256;
#define G8_MFMA(i0, j0, bb)                          \
  G8_BAR();                                          \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_s_setprio(1);                     \
  if ((i0) * 16 < live) mma(i0, j0, bb);             \
  __builtin_amdgcn_s_setprio(0);                     \
  G8_BAR()
#define G8_STAGE(U, R) stage(U, smem + ((R) & 1) * kBufB, (R))
#define G8_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
  // kMxA stages 1 more piece with unit A0: the waits after A0 / B0 of the next tile leave 5 in flight, not 4
#define G8_VMX() \
  if constexpr (MXA) G8_VM(5); \
  else G8_VM(4)
#define G8_TILE(R, ST1, ST2, ST3, ST4, W1, W2, W4) \
  {                                                \
    uint8_t* cb = smem + ((R) & 1) * kBufB;        \
    rdB(cb, kUB0, b0);                             \
    __builtin_amdgcn_sched_barrier(0);             \
    rdA(cb, kUA0);                                 \
    if constexpr (MXA) {                           \
      const uint8_t* st = smem + kLdsB + ((R) & 1) * 2048 + (wr * 128 + r16) * 4 + q; \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) sc[i] = st[i * 64]; \
    }                                              \
    ST1;                                           \
    W1;                                            \
    G8_MFMA(0, 0, b0);                             \
    rdB(cb, kUB1, b1);                             \
    ST2;                                           \
    W2;                                            \
    G8_MFMA(0, 2, b1);                             \
    rdA(cb, kUA1);                                 \
    ST3;                                           \
    G8_MFMA(4, 2, b1);                             \
    ST4;                                           \
    W4;                                            \
    G8_MFMA(4, 0, b0);                             \
  }
  // the same unit lead / vmcnt schedule as gemm8p: tile r stages tile r+1 (A0 B0 B1 A1 in P1..P4)
  G8_STAGE(0, 0); G8_STAGE(2, 0); G8_STAGE(3, 0); G8_STAGE(1, 0);
  G8_VM(4);
  G8_BAR();
  if (wr == 1) G8_BAR();  // stagger the two wave rows by one barrier
  int r = 0;
  for (; r < KT - 1; ++r)
    G8_TILE(r, G8_STAGE(0, r + 1), G8_STAGE(2, r + 1), G8_STAGE(3, r + 1), G8_STAGE(1, r + 1), G8_VMX(), G8_VMX(),
            G8_VM(4))
  G8_TILE(r, , , , , G8_VM(2), G8_VM(0), )
#undef G8_TILE
#undef G8_VMX
#undef G8_VM
#undef G8_STAGE
  if (wr == 0) G8_BAR();  // re-align the wave rows
#undef G8_MFMA
#undef G8_BAR
  __syncthreads();  // every wave is done reading the K buffers: LDS is reused by the epilogue

  // ---- epilogue: scales in registers, per wave 128 rows x 64 bf16 columns through LDS, 16 B stores ----
  // (row loop outermost: one activation scale live at a time — hoisting all 32 of them spills)
  __builtin_amdgcn_sched_barrier(0);
  float ws[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int col = n0 + wc * 64 + jj * 16 + r16;
    ws[jj] = col < p.N ? p.w_scale[(size_t)g * p.N + col] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      int row = m_begin + wr * 128 + i * 16 + 4 * q + rr;
      if (row >= m_end) row = m_begin;
      const float as = MXA ? 1.f : p.a_scale[p.a_rows ? p.a_rows[row] : row];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj][rr] *= as * ws[jj];
      __builtin_amdgcn_sched_barrier(0);  // one scale load in flight at a time: no 32-load VGPR burst
    }
  if constexpr (SWIGLU) {
    // columns jj 0, 1 of the wave are gate, jj 2, 3 the matching up columns: 32 outputs per row
    constexpr int CW = 32;
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * CW;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int row = i * 16 + 4 * q + rr, col = jj * 16 + r16;
          ot[row * CW + (col ^ ((row & 3) << 3))] = f2bf(silu8(acc[i][jj][rr]) * acc[i][jj + 2][rr]);
        }
    __syncthreads();
    const int cch = lane % 4, nout = p.N / 2;
    if constexpr (MODE == kMxOut) {
      // e4m3 rows with one e8m0 scale per (row, MX block): the wave's 32 outputs of a row are exactly block wc of
      // the workgroup's 128 (= one K slice of the down GEMM), held by one quad of lanes (8 each)
      uint8_t* q8 = reinterpret_cast<uint8_t*>(p.C);
#pragma unroll 4
      for (int k = 0; k < 8; ++k) {
        const int row = lane / 4 + 16 * k;
        const int gm = m_begin + wr * 128 + row;
        const int gn = n0 / 2 + wc * 32 + cch * 8;
        float v[8];
        unpack8(*reinterpret_cast<const uint4v*>(ot + row * CW + ((cch * 8) ^ ((row & 3) << 3))), v);
        float m = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
        const int e = mx_exp(quad_max(m));
        const float inv = __builtin_amdgcn_ldexpf(1.f, -e);
        uint32_t lo = 0, hi = 0;
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
        if (gm < m_end && gn < nout) {
          *reinterpret_cast<uint2*>(q8 + (size_t)gm * p.ldc + gn) = uint2{lo, hi};
          if (cch == 0) p.mx_out[((size_t)(n0 / 256) * p.s_rows + gm) * 4 + wc] = (uint8_t)(e + 127);
        }
      }
    } else {
#pragma unroll 4
      for (int k = 0; k < 8; ++k) {
        const int row = lane / 4 + 16 * k;
        const int gm = m_begin + wr * 128 + row;
        const int gn = n0 / 2 + wc * 32 + cch * 8;
        if (gm < m_end && gn < nout)
          *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) =
              *reinterpret_cast<const uint4v*>(ot + row * CW + ((cch * 8) ^ ((row & 3) << 3)));
      }
    }
  } else {
    constexpr int CW = 64;
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * CW;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int row = i * 16 + 4 * q + rr, col = jj * 16 + r16;
          ot[row * CW + (col ^ ((row & 7) << 3))] = f2bf(acc[i][jj][rr]);
        }
    __syncthreads();
    const int cch = lane % 8;
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int row = lane / 8 + 8 * k;
      const int gm = m_begin + wr * 128 + row;
      const int gn = n0 + wc * 64 + cch * 8;
      if (gm < m_end && gn < p.N)
        *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) =
            *reinterpret_cast<const uint4v*>(ot + row * CW + ((cch * 8) ^ ((row & 7) << 3)));
    }
  }
}

}  // namespace g8g
}  // namespace lwc

// Grouped fp8 GEMM on the 8-phase schedule.  Requires K % 128 == 0, N % 8 == 0, lda / ldc % 16 == 0 (bytes
// / elements: 16-byte rows), rows_a * lda < 2^31 and 256 * K < 2^31 (32-bit buffer offsets); max_slots >=
// sum_g ceil(M_g / 256) (ceil(rows / 256) + G always is).  row_off == null: dense, G = 1, rows [0, rows_c).
// mode: 0 plain, 1 SwiGLU epilogue (bf16 out), 2 SwiGLU epilogue with e4m3 + MX block-scale output (C is
// e4m3 [rows_c, ldc bytes], mx_out [N / 256][s_rows][4]); a_mx != null: A carries MX block scales
// [K / 128][s_rows][4] (mode 0 only; a_scale unused).
extern "C" int lwc_gemm8g_fp8(const void* A, const void* W, void* C, const int* row_off, const int* a_rows,
                              const float* a_scale, const float* w_scale, int G, int max_slots, int N, int K, int lda,
                              int ldc, int rows_a, int rows_c, int mode, const void* a_mx, void* mx_out, int s_rows,
                              hipStream_t s) {
  using namespace lwc::g8g;
  if (K % 128 != 0 || K < 128 || N % 8 != 0 || lda % 16 != 0 || ldc % 8 != 0 || G < 1) return -1;
  if ((long long)rows_a * lda >= (1LL << 31) || 256LL * K >= (1LL << 31)) return -1;
  const int swiglu = mode == 1 || mode == 2;
  if (mode < 0 || mode > 2 || !w_scale || (!a_scale && !a_mx)) return -2;
  if (swiglu && N % 64 != 0) return -1;  // whole gate / up block pairs per wave
  if (mode == 2 && (N % 256 != 0 || !mx_out || s_rows < rows_c || ldc % 16 != 0)) return -1;
  if (a_mx && (mode != 0 || a_rows || s_rows < rows_a || (long long)(K / 128) * s_rows * 4 >= (1LL << 31))) return -1;
  if (max_slots <= 0) return 0;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8g_kernel<kPlain>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsB);
    (void)hipFuncSetAttribute((const void*)gemm8g_kernel<kSwiglu>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsB);
    (void)hipFuncSetAttribute((const void*)gemm8g_kernel<kMxOut>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsB);
    (void)hipFuncSetAttribute((const void*)gemm8g_kernel<kMxA>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLdsB + kMxLds);
    attr = true;
  }
  const int n_tiles = (N + 255) / 256;
  const char* gv = getenv("LWC_G8G_GN");
  const int nj = (n_tiles + 7) / 8, gn = std::max(1, std::min(gv ? atoi(gv) : kDefaultGn, nj));
  Params p{(const uint8_t*)A, (const uint8_t*)W, (lwc::bf16_t*)C, row_off, a_rows, a_scale, w_scale,
           G, N, K, lda, ldc, rows_a, max_slots, n_tiles, rows_c, gn, 1,
           (const uint8_t*)a_mx, (uint8_t*)mx_out, s_rows};
  if (const char* sv = getenv("LWC_G8G_SKIP")) p.skip_empty = atoi(sv);
  // dense: 8 XCD ranges of ceil(tiles / 8) grouped tiles; grouped: per XCD, windows of gn n-tiles x
  // max_slots m-slots
  const unsigned grid = row_off ? (unsigned)(((nj + gn - 1) / gn) * gn * max_slots * 8)
                                : (unsigned)(8 * ((n_tiles * max_slots + 7) / 8));
  if (a_mx)
    gemm8g_kernel<kMxA><<<grid, 512, kLdsB + kMxLds, s>>>(p);
  else if (mode == 2)
    gemm8g_kernel<kMxOut><<<grid, 512, kLdsB, s>>>(p);
  else if (mode == 1)
    gemm8g_kernel<kSwiglu><<<grid, 512, kLdsB, s>>>(p);
  else
    gemm8g_kernel<kPlain><<<grid, 512, kLdsB, s>>>(p);
  return (int)hipGetLastError();
}
