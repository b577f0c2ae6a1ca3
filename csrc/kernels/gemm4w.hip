// K6 dense projection GEMM, 4-wave interleaved schedule: C = A . W^T with fused epilogues.
//
//   C[M, N]   = A[M, K] . W[N, K]^T (+ R)             EPI_PLAIN / EPI_RESIDUAL
//   H[M, N/2] = silu(A . Wg^T) * (A . Wu^T)            EPI_SWIGLU (W rows gate/up interleaved in blocks of 32)
//   C         = A . W^T + bias (then GELU: exact erf on VAR 32, the tanh form on VAR 64)   EPI_BIAS / _GELU
//
// Why a second core next to gemm8p: gemm8p pairs two waves per SIMD and hands the matrix pipe back and
// forth across s_barriers (compute segment of one wave || load segment of its partner).  Its load
// segments (2 LDS-DMA pieces + fragment reads) outlast the 16-MFMA compute segment, so the matrix pipe
// idles at every hand-off (profiles/gemm8p.md: SQ_WAIT_ANY 30 %, +16-37 % when the staging is removed).
// Here ONE wave per SIMD owns a 128 x (16 NT) slice of the 256 x BN tile (BN = 16 NT x 2; NT = 8: 256
// fp32 accumulators per lane, held in the AGPR half of gfx950's unified 512-entry register file) and
// keeps its matrix pipe fed by itself: every load instruction sits between MFMAs (a 16x16x32 MFMA holds
// the wave's vector issue for 8 of its 16 cycles; the other 8 issue one ds_read or one LDS-DMA piece).
//
// Per K tile (BK = 64) and wave: 16 NT MFMAs (8 m x NT n tiles x 2 k-steps of 32), 2 (8 + NT)
// ds_read_b128 fragment reads, 8 + NT LDS-DMA pieces of 1 KiB (the workgroup moves the A | W tile).  LDS
// holds two K tiles.  Register fragments are double-buffered by k-step: X = k-step 0, Y = k-step 1.  The main
// loop (G4_TILE_H, hipBLASLt's MT256x256x64 segment shape, disassembled): seg A = the Y reads of tile R, one
// per k-step-0 MFMA, lgkmcnt(0), barrier; seg B = the rest of k-step 0 and most of k-step 1, carrying tile
// R+2's DMA pieces one per ~5 MFMAs at raised wave priority, counted vmcnt, barrier; seg C = the last
// k-step-1 MFMAs with the X reads of tile R+1.  vmcnt never reaches 0 inside the loop except for the last
// two tiles.
//   hazards: WAR — tile R+2 overwrites buffer R & 1 only after every wave's reads of tile R completed
//            (lgkmcnt(0) + barrier closing seg A).  RAW — tile R+1 is read in seg C after every wave's
//            counted vmcnt wait for it (tile R+2's pieces, the youngest, stay in flight) + the barrier
//            closing seg B.
//   interleave: each load is followed by its share of the segment's MFMAs, pinned by sched_barrier(0).
//   MFMA: inline asm with the accumulator tied IN PLACE in an AGPR quad.  The builtin lets the register
//         allocator pick the untied form (dst != srcC); with every AGPR live it then rotates the
//         accumulators through VGPRs — ~300 v_accvgpr moves per K tile, measured in the .s.  The compiler
//         cannot see the asm's latency: llm_weighted_consensus_amd/_isa_guard.py checks the built code
//         object for accumulator moves / reads of in-flight MFMA results and fails the build on one.
// Two schedules share that loop (the planner picks per shape, ops/gemm_plan.py): VAR 32 with the block-
// staged epilogue (accumulators -> LDS image -> 16 B row stores), and VAR 64 — the wave-local epilogue on
// the transposed accumulator layout (TR / TRR below), with the next persistent tile's first two K tiles
// DMA'd inside this tile's last two iterations (even K tile counts).
//
// LDS image (per operand, per K tile): rows x 128 B, lane-linear DMA image; 16 B chunk c of row r is
// stored at chunk c ^ ((r >> 1) & 7) (swizzle applied to the DMA source address and to the read: the 16
// lanes of a ds_read_b128 group hit 16 distinct bank quads — gemm8p's image, SQ_LDS_BANK_CONFLICT 0).
//
// Work distribution: data-parallel, persistent (one workgroup per CU), tiles in rounds of 8 x wpx with
// XCD x taking wpx consecutive tiles of the grouped (gm m-tiles) order, so its tiles share operand panels
// in its L2.  No stream-K: the planner (ops/gemm_plan.py) gives shapes with a ragged last round to
// gemm8p's stream-K or picks BN = 192 (qkv at M = 4096: 512 tiles = 2 whole rounds instead of 1.5).
// Epilogue: accumulators -> bf16 (SwiGLU / bias / GELU in fp32 registers) -> LDS -> 16 B row stores (+
// residual read in the same pass).
//
// RMSNorm folded into the projections (the decode chain, models/llama.py): rmsnorm(x) . W^T =
// diag(1/rms(x)) . (x . (W diag(g))^T), so with the norm weight g folded into W once at load, a
// projection of the raw residual stream only needs its accumulator rows scaled by r = 1/rms(x) — the
// norm pass (a read and a write of every row) disappears.
//   RS 2 (producer: the o / down projections' residual epilogue): each wave sums the squares of its 128
//        output columns (the bf16-rounded new residual stream) per row, the two waves sharing rows add
//        theirs through LDS, and the tile stores ONE partial per row: ss[tn][row] (tiles_n partials, fixed
//        order, no atomics, no cross-workgroup hand-off).
//   RS 1 (consumer: qkv, gate|up, lm_head): the P partials of the tile's 256 rows arrive in LDS by P LDS-DMA
//        pieces (1 KiB each) issued before the tile's first K-tile pieces (the prologue's counted wait
//        retires them); after the prologue barrier thread t adds row t's partials in order and keeps
//        r = rsqrt(sum / K + eps) in LDS; the epilogue scales its rows before SwiGLU / the store.  The
//        first projection of a chain reads P = 1 partial from rms_rowsumsq (norm.hip).  VAR 64: from the
//        second persistent tile on, the tile's partials were DMA'd under the previous tile's main loop.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace lwc {
namespace g4w {

constexpr int kOpA = 256 * 128;  // A operand's K tile: 256 rows x 128 B
// buffer load / store cache policy sc1 (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16): write-through stores, L1-bypassing loads
constexpr int kSC1 = 16;

enum Epi { EPI_PLAIN = 0, EPI_RESIDUAL = 1, EPI_SWIGLU = 2, EPI_BIAS = 3, EPI_BIAS_GELU = 4 };

struct Params {
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  const bf16_t* R;  // EPI_RESIDUAL: residual [M, ldc]; EPI_BIAS*: bias [N]
  int M, N, K, lda, ldc;
  int tiles_m, tiles_n, KT;
  int gm;
  int wpx, tiles;
  float* ss;        // RS 1: row sum-of-squares partials [P][ssld] (read); RS 2: [tiles_n][ssld] (written)
  int P;            // RS 1: partials per row (<= 16)
  int ssld;         // floats between partials (a multiple of 4: 16-byte aligned LDS-DMA sources)
  float eps;        // RS 1
  // split-K (VAR 64): tiles [0, full) run whole; every tile t >= full runs as S units over K ranges of KT / S
  // K tiles.  The first S - 1 arrivers (a ticket from cnt[t]) store their fp32 accumulators into part, then
  // count themselves in done[t]; the last arriver waits for those (they already run: no deadlock), adds
  // the partials and runs the epilogue.  cnt / done are zero between calls (zeroed once, reset by each
  // tile's last arriver).
  int full, S, units;
  float* part;      // [(tiles - full) * (S - 1)][8 NT][256] float4
  int* cnt;         // [tiles]
  int* done;        // [tiles]
};

template <int NT>
struct Geo {
  static constexpr int BN = 32 * NT;            // W rows per tile
  static constexpr int OpB = BN * 128;          // W operand's K tile
  static constexpr int Buf = kOpA + OpB;        // one K tile
  static constexpr int Lds = 2 * Buf;           // two K tiles
  static constexpr int Pieces = 8 + NT;         // LDS-DMA pieces per wave per K tile
  static constexpr int Reads = 8 + NT;          // fragment reads per wave per k-step
};

LWC_DEVICE void mfma(float4v& d, const uint4v& a, const uint4v& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
}
// TR: operands swapped — the MFMA computes the tile transposed (A operand = W rows, B = activation rows), so
// a lane's accumulator quad holds 4 consecutive OUTPUT COLUMNS of one output row instead of 4 rows of one
// column; the wave-local epilogue then packs rows in registers (no LDS staging), see TR below
template <bool TR>
LWC_DEVICE void mfma2(float4v& d, const uint4v& a, const uint4v& b) {
  if constexpr (TR)
    mfma(d, b, a);
  else
    mfma(d, a, b);
}
// the first non-MFMA read of an accumulator after the last (opaque) MFMA: 16 wait states
#define G4_MFMA_DRAIN() asm volatile("s_nop 15" ::: "memory")
#define G4_BAR() __builtin_amdgcn_s_barrier()
#define G4_VM(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")
#define G4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
// the wave-local epilogue's accumulators of m-tile I into AV[NT] (VGPRs): the tile's own, plus the partial
// sums of the other split-K units when this workgroup is a split tile's last arriver (nsl slabs behind the
// resource pslab, read with sc1 loads: L2, never a stale L1 line).  The first slab's values come from PP,
// loaded one m-tile ahead (G4_ACC_PREFETCH0 before the loop; each G4_ACC_LOAD issues the next m-tile's), so
// the loads of m-tile i + 1 are in flight under m-tile i's epilogue.  The residual epilogue (TRR) prefetches;
// the TR epilogues load each m-tile's partials in place (G4_ACC_LOAD_SYNC: 32 more live VGPRs made them spill)
#define G4_SLAB(U, I, G) \
  __builtin_bit_cast(float4v, __builtin_amdgcn_raw_buffer_load_b128(pslab, (((I) * NT + (G)) * 256 + tid) * 16, \
                                                                    (U) * (8 * NT * 256 * 16), kSC1))
#define G4_ACC_PREFETCH0(PP)                                      \
  do {                                                            \
    if (SK && nsl > 0) {                                          \
      _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) PP[g_] = G4_SLAB(0, 0, g_); \
    }                                                             \
  } while (0)
#define G4_ACC_LOAD_SYNC(AV, I)                                                  \
  do {                                                                           \
    _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) AV[g_] = acc[I][g_];       \
    for (int u_ = 0; SK && u_ < nsl; ++u_) {                                     \
      _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) AV[g_] += G4_SLAB(u_, I, g_); \
    }                                                                            \
  } while (0)
#define G4_ACC_LOAD(AV, PP, I)                                                   \
  do {                                                                           \
    _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) AV[g_] = acc[I][g_];       \
    if (SK && nsl > 0) {                                                         \
      _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) AV[g_] += PP[g_];        \
      if ((I) + 1 < 8) {                                                         \
        _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) PP[g_] = G4_SLAB(0, (I) + 1, g_); \
      }                                                                          \
      for (int u_ = 1; u_ < nsl; ++u_) {                                         \
        _Pragma("unroll") for (int g_ = 0; g_ < NT; ++g_) AV[g_] += G4_SLAB(u_, I, g_); \
      }                                                                          \
    }                                                                            \
  } while (0)

// Diagnostic build only (scripts/probes/g4_stamps.cpp defines LWC_G4_STAMPS): wave 0 of every workgroup
// records s_memrealtime at up to eight points of each persistent round (and s_memtime at the first and last)
// into g4_stamps[block][round][8] with vector stores (points: scripts/probes/g4_stamps.cpp); the product build has no stamp code at all.
#ifdef LWC_G4_STAMPS
__device__ unsigned long long* g4_stamps;
#define G4_STAMP(round, k)                                                                  \
  do {                                                                                      \
    if (threadIdx.x == 0 && (round) < 64) {                                                 \
      unsigned long long* sp_ = g4_stamps + ((size_t)blockIdx.x * 64 + (round)) * 16 + 2 * (k); \
      if ((k) == 0 || (k) == 7) sp_[0] = __builtin_amdgcn_s_memtime();                      \
      sp_[1] = __builtin_amdgcn_s_memrealtime();                                            \
    }                                                                                       \
  } while (0)
#else
#define G4_STAMP(round, k) ((void)0)
#endif

// x * sigmoid(x) with v_rcp_f32 (1 ulp) instead of the IEEE division sequence (v_div_scale x2, v_div_fmas,
// v_div_fixup around an rcp: ~9 VALU per element in an epilogue of 256 per lane); the result is rounded
// to bf16 (or e4m3) anyway.  x -> -inf: rcp(inf) = 0, x * 0 = -0 as the division gives
LWC_DEVICE float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
LWC_DEVICE float erf_as(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * a);  // v_rcp_f32 (1 ulp): __frcp_rn is a full division sequence
  const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.f - y * __expf(-a * a), x);
}
LWC_DEVICE float gelu_erf(float x) { return 0.5f * x * (1.f + erf_as(x * 0.70710678118654752f)); }
// GELU in the tanh form, x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) — the form hipBLASLt's bias+GELU
// epilogue computes (the library arm the planner times against): 2 transcendentals + 4 VALU instead of
// erf_as's 2 + ~12, within 8.1e-3 of the erf form at the bge-large FFN1 shape, the bf16 output's own rounding
// being 7.8e-3 (ops/gemm_plan.py linear_bias).  The VAR 64 epilogue uses it; the other schedules keep erf.
// (A degree-7 polynomial of the erf form, clamped at |x| = 4 — no transcendental, 12 VALU — ran FFN1 + GELU
// 3.5 % slower at config 2's shape; its packed-fp32 form miscompiled inside this epilogue:
// profiles/round6_ab.md, scripts/probes/pkfma_probe.cpp.)
LWC_DEVICE float gelu_tanh(float x) {
  const float z = x * (1.5957691216f + 0.0713548163f * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-z));
}

// work unit u -> (tile, first K tile, K tile count): whole tiles first, then the split tiles' S units each
// (consecutive: one tile's units land on one XCD's wpx consecutive units, its partials stay in that L2)
template <bool SK>
LWC_DEVICE void unit_tile(const Params& p, int u, int& t, int& kt0, int& nkt) {
  if (!SK || u < p.full) {
    t = u, kt0 = 0, nkt = p.KT;
  } else {
    // (unit s of S: K tile pairs [s * H / S, (s + 1) * H / S) of the tile's H = KT / 2 — S need not divide KT)
    const int v = u - p.full, s = v % p.S, h = p.KT >> 1;
    t = p.full + v / p.S, kt0 = 2 * (s * h / p.S), nkt = 2 * ((s + 1) * h / p.S) - kt0;
  }
}

LWC_DEVICE void tile_mn(const Params& p, int t, int& m, int& n) {
  const int group = p.gm * p.tiles_n;
  const int first_m = (t / group) * p.gm;
  const int gsz = min(p.tiles_m - first_m, p.gm);
  const int in = t % group;
  m = first_m + in % gsz;
  n = in / gsz;
}

// Epilogue LDS image column of (row, col) for a CW-wide bf16 row: XOR swizzle by 8-column chunks (keeps
// every 16 B chunk contiguous); CW = 96 swizzles its last 32 columns among themselves.
template <int CW>
LWC_DEVICE int swz(int row, int col) {
  if constexpr (CW == 96) return col < 64 ? col ^ ((row & 7) << 3) : col ^ ((row & 3) << 3);
  return col ^ (((row & 7) << 3) % CW);
}

// LDS bytes: the two K tiles, then the RS area (RS 1: P x 256 partials + 256 row scales; RS 2: row sums)
template <int NT, int RS>
constexpr int lds_bytes() {
  return Geo<NT>::Lds + (RS == 1 ? 16384 + 1024 : (RS == 2 ? 2048 : 0)) + 16;  // (+ the split-K ticket word)
}

// SK: the split-K build (VAR 64; chosen per call only when the call splits): the other builds carry none of
// its code (its epilogue paths cost the unsplit VAR 64 kernels ~1 % at the serving shapes when they did)
template <int EPI, int NT, int VAR, int RS, bool SK>
__global__ void __launch_bounds__(256, 1) gemm4w_kernel(Params p) {
  using G = Geo<NT>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int KT = p.KT;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  static_assert(VAR == 32 || VAR == 64, "gemm4w schedules: 32 (block-staged epilogue), 64 (wave-local)");
  static_assert(!SK || VAR == 64, "split-K runs on the VAR 64 schedule");
  // VAR 64: the wave-local epilogue ("prefetch across persistent tiles") on the transposed accumulator layout
  // (mfma2): plain / SwiGLU / bias / GELU (TR; RS 0, and the row-scaled consumers RS 1) and residual (TRR,
  // RS 0 / 2)
  constexpr bool PAP = VAR == 64;
  constexpr bool TR = PAP && RS != 2 && EPI != EPI_RESIDUAL;
  constexpr bool TRR = PAP && EPI == EPI_RESIDUAL;
  constexpr bool TRL = TR || TRR;
  static_assert(!PAP || TRL, "the wave-local epilogue runs on the transposed layout");
  // RS 1: the P x 256 partials (16 KiB) and the 256 row scales (1 KiB) after the K buffers; RS 2: the four
  // waves' 128 row sums (2 KiB) at the same place
  constexpr int RSOFF = G::Lds, RSV = RSOFF + 16384;
  constexpr int SKOFF = lds_bytes<NT, RS>() - 16;  // split-K: the workgroup's arrival ticket
  // LDS-DMA piece k (64 lanes x 16 B = 256 rows x fp32) of partial k of m-tile rows [m, m + 256)
  auto ss_dma = [&](int m, int k) {
    const __amdgpu_buffer_rsrc_t rR = uniform_rsrc(p.ss + (size_t)k * p.ssld + m, (p.M - m) * 4);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rR, (__attribute__((address_space(3))) void*)(smem + RSOFF + k * 1024),
                                             16, (uint32_t)((threadIdx.x & 63) * 16), 0, 0, 0);
  };

  for (int round = 0;; ++round) {
    const int unit = round * 8 * p.wpx + xcd * p.wpx + j;
    if (unit >= p.units) break;
    int tile, kt0, nkt;
    unit_tile<SK>(p, unit, tile, kt0, nkt);
    int tm, tn;
    tile_mn(p, tile, tm, tn);
    const int m0 = tm * 256, n0 = tn * G::BN;
    G4_STAMP(round, 0);
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int wm = wid >> 1, wn = wid & 1;

    // DMA: piece i of wave wid covers operand rows i*32 + wid*8 + lane/8, LDS chunk lane%8, which holds
    // global chunk (lane%8) ^ ((row >> 1) & 7); (row >> 1) & 7 does not depend on i.
    const int drow = wid * 8 + (lane >> 3);
    const int dchk = ((lane & 7) ^ ((drow >> 1) & 7)) * 8;
    const uint32_t voA = (uint32_t)((drow * p.lda + dchk) * 2);
    const uint32_t voW = (uint32_t)((drow * p.K + dchk) * 2);
    const int sA = 32 * p.lda * 2, sW = 32 * p.K * 2;  // bytes between pieces
    const int dst0 = wid * 1024;
    // (a split unit's K range starts kt0 K tiles in: the resources start there.  A's resource spans only the
    // tile's own 256 rows, so A of any size takes one launch: the 32-bit range is per tile)
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.A + (size_t)m0 * p.lda + kt0 * 64), (short)0, min(p.M - m0, 256) * p.lda * 2 - kt0 * 128,
        0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.W + (size_t)n0 * p.K + kt0 * 64), (short)0, min(p.N - n0, G::BN) * p.K * 2 - kt0 * 128, 0x00020000);
    // LDS-DMA piece k of one K tile (k < 8: A rows, else W rows)
    auto piece = [&](uint8_t* buf, int kt, int k) {
      if (k < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rA, (__attribute__((address_space(3))) void*)(buf + k * 4096 + dst0), 16, voA, k * sA + kt * 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rW, (__attribute__((address_space(3))) void*)(buf + kOpA + (k - 8) * 4096 + dst0), 16, voW,
            (k - 8) * sW + kt * 128, 0, 0);
    };
    auto stage = [&](uint8_t* buf, int kt) {
#pragma unroll
      for (int k = 0; k < G::Pieces; ++k) piece(buf, kt, k);
    };
    // VAR 64: the next persistent tile (its first two K tiles are DMA'd inside the last two main-loop
    // iterations of this one).  Past the last tile the pieces re-read this tile's first two K tiles into
    // the freed buffers instead: every piece a real memory request — pieces past a resource's end complete
    // out of order with the real ones before them, and a counted vmcnt wait then passes too early
    // (measured: wrong results at every K tile count past 2)
    const int nunit = (round + 1) * 8 * p.wpx + xcd * p.wpx + j;
    const bool pf = PAP && nunit < p.units;
    int um = tm, un = tn, ukt0 = kt0;
    if (pf) {
      int ut, unkt;
      unit_tile<SK>(p, nunit, ut, ukt0, unkt);
      tile_mn(p, ut, um, un);
    }
    const __amdgpu_buffer_rsrc_t nA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.A + (size_t)um * 256 * p.lda + ukt0 * 64), (short)0,
        min(p.M - um * 256, 256) * p.lda * 2 - ukt0 * 128, 0x00020000);
    const __amdgpu_buffer_rsrc_t nW = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.W + (size_t)un * G::BN * p.K + ukt0 * 64), (short)0,
        min(p.N - un * G::BN, G::BN) * p.K * 2 - ukt0 * 128, 0x00020000);
    auto npiece = [&](uint8_t* buf, int kt, int k) {  // piece k of the NEXT tile's K tile kt
      if (k < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            nA, (__attribute__((address_space(3))) void*)(buf + k * 4096 + dst0), 16, voA, k * sA + kt * 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            nW, (__attribute__((address_space(3))) void*)(buf + kOpA + (k - 8) * 4096 + dst0), 16, voW,
            (k - 8) * sW + kt * 128, 0, 0);
    };
    // fragment reads: m-tile / n-tile i adds i * 16 rows = i * 2048 B; the swizzle only depends on r16
    const int sw = (r16 >> 1) & 7;
    const int offA0 = (wm * 128 + r16) * 128 + ((q ^ sw) << 4);
    const int offA1 = (wm * 128 + r16) * 128 + (((4 + q) ^ sw) << 4);
    const int offB0 = kOpA + (wn * 16 * NT + r16) * 128 + ((q ^ sw) << 4);
    const int offB1 = kOpA + (wn * 16 * NT + r16) * 128 + (((4 + q) ^ sw) << 4);

    float4v acc[8][NT];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < NT; ++jj) acc[i][jj] = float4v{0.f, 0.f, 0.f, 0.f};
    uint4v xa[8], xb[NT], ya[8], yb[NT];
    // fragment read k of a k-step (k < NT: W n-tile k, else A m-tile k - NT)
    auto rd1 = [&](const uint8_t* buf, int oa, int ob, uint4v(&fa)[8], uint4v(&fb)[NT], int k) {
      if (k < NT)
        fb[k] = *reinterpret_cast<const uint4v*>(buf + ob + k * 2048);
      else
        fa[k - NT] = *reinterpret_cast<const uint4v*>(buf + oa + (k - NT) * 2048);
    };

    // (VAR 64 takes even K tile counts only — the host falls back to VAR 32 — so the next tile's first
    // two K tiles, DMA'd inside the last two iterations, land in buffers 0 and 1)
    const int nt = nkt;  // (a split unit: its share of the K tiles; even, like every VAR 64 count)
    (void)KT;
    // VAR 64 ("prefetch across persistent tiles"): from the second tile on, this tile's first two K tiles
    // were issued by the previous tile right after its main loop, under its epilogue; the waits below then
    // also cover the previous epilogue's memory ops issued after them (stricter, still exact for the data)
    // (the residual epilogue takes this path too — TRR: residual chunks loaded two m-tiles ahead, not all up
    // front, which spilled — and so does its RS 2 form: no block barriers between the adds and the stores)
    if (!PAP || round == 0) {
      if constexpr (RS == 1) {  // the oldest VMEM ops of each wave: the counted wait below retires them
        for (int k = wid; k < p.P; k += 4) ss_dma(m0, k);
      }
      stage(smem, 0);
      if (nt > 1) stage(smem + G::Buf, 1);
    }
    if (nt > 1) {
      G4_VM(G::Pieces);
    } else {
      G4_VM(0);
    }
    G4_BAR();
    G4_STAMP(round, 1);
    if constexpr (RS == 1) {
      // row tid's scale from its partials (the main loop's first barrier publishes it to the epilogues)
      const float* part = reinterpret_cast<const float*>(smem + RSOFF);
      float sum = 0.f;
      if constexpr (PAP) {
        // (the accumulators and the fragment registers are live here: a few partials in flight at a time)
#pragma unroll 4
        for (int k = 0; k < p.P; ++k) sum += part[k * 256 + tid];  // fixed order: deterministic
      } else {
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = part[k * 256 + tid];  // all 16 in flight (the region is always 16 KiB)
#pragma unroll
        for (int k = 0; k < 16; ++k) sum += k < p.P ? v[k] : 0.f;  // fixed order: deterministic
      }
      reinterpret_cast<float*>(smem + RSV)[tid] = rsqrtf(sum / (float)p.K + p.eps);
      if constexpr (PAP) {
        // the NEXT persistent tile's partials go out now, under this tile's main loop (its prologue is the
        // previous tile's tail, which issues no partials): every thread has read this tile's first, then the
        // DMA overwrites the region.  The oldest VMEM ops of the loop: its first counted wait retires them.
        G4_LGKM0();
        G4_BAR();
        __builtin_amdgcn_sched_barrier(0);
        if (pf) {
          for (int k = wid; k < p.P; k += 4) ss_dma(um * 256, k);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < G::Reads; ++k) rd1(smem, offA0, offB0, xa, xb, k);

    constexpr int M1 = 8 * NT;  // MFMAs of one k-step
    // VAR 32: the library kernel's segment shape (hipBLASLt's MT256x256x64 DTL loop, disassembled: the same
    // 128 MFMA / 32 ds_read_b128 / 16 LDS-DMA per K tile, two barriers).  seg A: the Y reads of tile R back
    // to back, one per k-step-0 MFMA, then a few more MFMAs, lgkmcnt(0), barrier; seg B: the long middle —
    // the rest of k-step 0 and most of k-step 1 — carrying the tile R+2 DMA pieces one per ~5 MFMAs at raised
    // wave priority (s_setprio 3), vmcnt, barrier; seg C: the last k-step-1 MFMAs with the X reads of tile
    // R+1 one per MFMA.  Waits land after sections with no loads of their own in flight behind them.
    constexpr int HA = G::Reads + M1 / 6;        // seg A MFMAs (k-step 0)
    constexpr int HC = G::Reads + M1 / 8;        // seg C MFMAs (k-step 1)
    constexpr int HB = 2 * M1 - HA - HC;          // seg B MFMAs (k-step 0 rest, then k-step 1)
#define G4_TILE_H(R, STAGE, NEXT)                                                                   \
  {                                                                                                 \
    uint8_t* cur = smem + ((R) & 1) * G::Buf;                                                       \
    uint8_t* nxt = smem + (((R) + 1) & 1) * G::Buf;                                                 \
    _Pragma("unroll") for (int m = 0; m < HA; ++m) {                                                \
      if (m < G::Reads) rd1(cur, offA1, offB1, ya, yb, m);                                          \
      mfma2<TRL>(acc[m / NT][m % NT], xa[m / NT], xb[m % NT]);                                            \
      __builtin_amdgcn_sched_barrier(0);                                                            \
    }                                                                                               \
    G4_LGKM0();                                                                                     \
    G4_BAR();                                                                                       \
    if constexpr ((STAGE) != 0) __builtin_amdgcn_s_setprio(3);                                      \
    _Pragma("unroll") for (int q = 0; q < HB; ++q) {                                                \
      if constexpr ((STAGE) == 1) {                                                                 \
        if (q * G::Pieces / HB != (q + 1) * G::Pieces / HB) piece(cur, (R) + 2, q * G::Pieces / HB); \
      } else if constexpr ((STAGE) == 2) {                                                          \
        if (q * G::Pieces / HB != (q + 1) * G::Pieces / HB) npiece(cur, (R) + 2 - nt, q * G::Pieces / HB); \
      }                                                                                             \
      const int m = HA + q;                                                                         \
      if (m < M1)                                                                                   \
        mfma2<TRL>(acc[m / NT][m % NT], xa[m / NT], xb[m % NT]);                                          \
      else                                                                                          \
        mfma2<TRL>(acc[(m - M1) / NT][(m - M1) % NT], ya[(m - M1) / NT], yb[(m - M1) % NT]);              \
      __builtin_amdgcn_sched_barrier(0);                                                            \
    }                                                                                               \
    if constexpr ((STAGE) != 0) {                                                                   \
      __builtin_amdgcn_s_setprio(0);                                                                \
      G4_VM(G::Pieces);                                                                             \
    } else {                                                                                        \
      G4_VM(0);                                                                                     \
    }                                                                                               \
    G4_BAR();                                                                                       \
    _Pragma("unroll") for (int c = 0; c < HC; ++c) {                                                \
      if constexpr (NEXT) {                                                                         \
        if (c < G::Reads) rd1(nxt, offA0, offB0, xa, xb, c);                                        \
      }                                                                                             \
      const int m = M1 - HC + c;                                                                    \
      mfma2<TRL>(acc[m / NT][m % NT], ya[m / NT], yb[m % NT]);                                            \
      __builtin_amdgcn_sched_barrier(0);                                                            \
    }                                                                                               \
  }
    int r = 0;
    {
      // VAR 64 (TAIL 2): the last two K tiles carry the NEXT tile's first two (into the buffers they
      // free: buffer 0, then 1, as the prologue's stage(0) / stage(1) — KT is even for these variants): seg B
      // pieces as in the steady state, no DMA burst left for the epilogue.  (The same control flow as the
      // other variants' tail: a differently shaped tail made the register allocator rotate the accumulators
      // through v_accvgpr_mov copies that read in-flight inline-asm MFMA results.)
      constexpr int TAIL = PAP ? 2 : 0;
      for (; r + 2 < nt; ++r) G4_TILE_H(r, 1, true)
      if (nt >= 2) {
        G4_TILE_H(r, TAIL, true)
        ++r;
      }
      G4_TILE_H(r, TAIL, false)
    }
#undef G4_TILE_H
    // accumulators are read by VALU / stores from here on.  The MFMAs are opaque inline asm, so the compiler
    // takes their results as ready at once: without a barrier it hoisted v_accvgpr_read of the last MFMAs'
    // accumulators above the drain (the row-scaled variant read stale e = 2, 3 values).  The drain, then an
    // empty asm "writing" every accumulator: no read can move above it.
    __builtin_amdgcn_sched_barrier(0);
    G4_MFMA_DRAIN();
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < NT; ++jj) asm volatile("" : "+a"(acc[i][jj]));
    // VAR 32: every wave is done with the K buffers, which the block-staged epilogue reuses.  VAR 64's
    // wave-local epilogue touches no K buffer (its LDS use, the RS areas, is ordered by the main loop's
    // barriers and the next tile's prologue barrier), so no block barrier here: a __syncthreads() would also
    // drain vmcnt(0) — the next tile's K-tile DMA issued in the last iteration — before the epilogue starts
    if constexpr (!PAP) __syncthreads();
    G4_STAMP(round, 2);
    int nsl = 0;  // split-K last arriver: partial slabs to add in the epilogue
    __amdgpu_buffer_rsrc_t pslab = __builtin_amdgcn_make_buffer_rsrc(nullptr, (short)0, 0, 0x00020000);
    if constexpr (SK) {
      // split-K (tile >= full, wave-uniform): arrival ticket; the first S - 1 arrivers publish their partial
      // sums and leave, the last one adds them and runs the epilogue.  Hand-off (MI355X_MICROARCH.md,
      // inter-workgroup visibility, the sc1 table's first row): every slab byte is stored write-through (sc1,
      // 16 B) and loaded sc1 (L2, bypassing L1), every storing wave waits vmcnt(0), a block barrier, then one
      // lane's agent-scope add to done[tile]; the last arriver's lane 0 polls done[tile] with sc1 loads and the
      // block barrier releases the other waves.  No release / acquire fences: a release fence writes back the
      // whole XCD L2 — here 256 KB of fresh partials per workgroup — and cost ~30 us per call
      if (tile >= p.full) {
        int* tk = reinterpret_cast<int*>(smem + SKOFF);
        if (tid == 0) tk[0] = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int ticket = __builtin_amdgcn_readfirstlane(tk[0]);
        pslab = uniform_rsrc(p.part + (size_t)(tile - p.full) * (p.S - 1) * (8 * NT * 256 * 4),
                             (p.S - 1) * (8 * NT * 256 * 16));
        if (ticket < p.S - 1) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int jj = 0; jj < NT; ++jj)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, acc[i][jj]), pslab,
                                                     ((i * NT + jj) * 256 + tid) * 16, ticket * (8 * NT * 256 * 16),
                                                     kSC1);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) __hip_atomic_fetch_add(p.done + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          continue;  // this unit's work is in the partial: no epilogue
        }
        if (tid == 0) {
          // the units waited for hold earlier tickets: they are running and wait on nothing.  Bounded anyway
          // (~0.3 s), so a broken hand-off cannot hang the GPU
          for (int it = 0; it < (1 << 21); ++it) {
            if (__hip_atomic_load(p.done + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= p.S - 1) break;
            __builtin_amdgcn_s_sleep(2);
          }
          // every unit of this tile has counted itself: reset for the next call
          __hip_atomic_store(p.done + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        // the partials are added where the epilogue reads the accumulators (G4_ACC_LOAD): the accumulators
        // stay as the MFMAs left them (rewriting them here made the register allocator rotate all of them
        // through v_accvgpr_mov copies, caught by the build's ISA guard)
        nsl = p.S - 1;
      }
    }

    constexpr int CW = EPI == EPI_SWIGLU ? 8 * NT : 16 * NT;
    if constexpr (PAP) {
      // ---- epilogue, wave-local: per m-tile (16 rows), no block barrier; rows packed in registers (TR, TRR)
      const int ncol0 = EPI == EPI_SWIGLU ? n0 / 2 + wn * 8 * NT : n0 + wn * 16 * NT;
      const int ncols = EPI == EPI_SWIGLU ? p.N / 2 : p.N;
      const int row0 = __builtin_amdgcn_readfirstlane(m0 + wm * 128);  // uniform: buffer resources in SGPRs, no waterfall loops
      // stores branch-free through a buffer resource over this wave's rows: a lane whose chunk lies past
      // the last column takes an offset past the resource's end, so the hardware drops it (no exec-masked
      // store branches between the epilogue's memory operations)
      const int rows_c = max(0, min(p.M - row0, 128));
      const __amdgpu_buffer_rsrc_t rC = uniform_rsrc(p.C + (size_t)row0 * p.ldc, rows_c * p.ldc * 2);
      // TR: the bias of the lane's 4 consecutive columns 16 g + 4 q .. + 3 of each n-tile g (8 B loads; N % 8
      // == 0, so a group lies wholly inside or past the last column)
      // (kept packed, 2 VGPRs per group, unpacked per use; the column base is made opaque so the loads are not
      // hoisted above the main loop, where 32 live floats made this kernel spill)
      uint2 tbias[NT];
      if constexpr (TR && (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU)) {
        int cb = n0 + wn * 16 * NT + 4 * q;
        asm volatile("" : "+v"(cb));
#pragma unroll
        for (int g = 0; g < NT; ++g) {
          const int col = cb + g * 16;
          tbias[g] = col < p.N ? *reinterpret_cast<const uint2*>(p.R + col) : uint2{0u, 0u};
        }
      }
      // TR / TRR: the lane's 16 B chunk of column pair g2 of an m-tile (the layout of the TR stores below):
      // the column part per lane (past the last column: an offset past the resource's end, dropped), the
      // m-tile's row offset wave-uniform in soffset
      uint32_t tr_vo[NT / 2];
#pragma unroll
      for (int g2 = 0; g2 < NT / 2; ++g2) {
        const int gn = ncol0 + g2 * 32 + (q & 1) * 16 + (q >> 1) * 8;
        tr_vo[g2] = gn < ncols ? (uint32_t)((r16 * p.ldc + gn) * 2) : 0x80000000u;
      }
      auto tr_so = [&](int i) { return i * 32 * p.ldc; };  // (kernel argument x constant: SALU)
      const __amdgpu_buffer_rsrc_t rR =
          uniform_rsrc(EPI == EPI_RESIDUAL ? p.R + (size_t)row0 * p.ldc : p.A, EPI == EPI_RESIDUAL ? rows_c * p.ldc * 2 : 0);
      uint4v rv[2][NT / 2];  // TRR: residual chunks of m-tiles i and i + 1 (two m-tiles ahead of the adds)
      if constexpr (TRR) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int g2 = 0; g2 < NT / 2; ++g2)
            rv[i][g2] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rR, tr_vo[g2], tr_so(i), 0));
      }
      float4v pp[NT];  // split-K (TRR): the first partial slab's values of the next m-tile
      if constexpr (TRR && SK) G4_ACC_PREFETCH0(pp);
      G4_STAMP(round, 3);
      if constexpr (TRR) {
        // residual on the TR layout: per column pair the fp32 accumulators swap halves by v_permlane16_swap
        // (4 per pair), the lane adds its 16 B residual chunk (loaded two m-tiles ahead) to 8 consecutive
        // columns and stores them in place; RS 2: the row's squares over the wave's 128 columns meet across
        // the 4 lanes of the row (xor 16, 32)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float4v av[NT];  // the m-tile's accumulators (+ the split-K partials of the other units)
          G4_ACC_LOAD(av, pp, i);
          uint4v res[NT / 2];
#pragma unroll
          for (int g2 = 0; g2 < NT / 2; ++g2) res[g2] = rv[i & 1][g2];
          if (i + 2 < 8) {
#pragma unroll
            for (int g2 = 0; g2 < NT / 2; ++g2)
              rv[i & 1][g2] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rR, tr_vo[g2], tr_so(i + 2), 0));
          }
          float sq = 0.f;
#pragma unroll
          for (int g2 = 0; g2 < NT / 2; ++g2) {
            float x[8], y[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(av[2 * g2][e]),
                                                              __float_as_uint(av[2 * g2 + 1][e]), false, false);
              x[e] = __uint_as_float(r[0]);
              x[e + 4] = __uint_as_float(r[1]);
            }
            unpack8(res[g2], y);
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] += y[e];
            const uint4v v = pack8(x);
            if constexpr (RS == 2) {  // the bf16-rounded values the stream now holds
              float z[8];
              unpack8(tr_vo[g2] != 0x80000000u ? v : uint4v{0u, 0u, 0u, 0u}, z);
#pragma unroll
              for (int e = 0; e < 8; ++e) sq += z[e] * z[e];
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rC, tr_vo[g2], tr_so(i), 0);
          }
          if constexpr (RS == 2) {
            sq += __shfl_xor(sq, 16);
            sq += __shfl_xor(sq, 32);
            if (q == 0) reinterpret_cast<float*>(smem + RSOFF)[wid * 128 + i * 16 + r16] = sq;
          }
          __builtin_amdgcn_sched_barrier(0);
          if (i == 0) G4_STAMP(round, 4);
          if (i == 3) G4_STAMP(round, 5);
          if (i == 7) G4_STAMP(round, 6);
        }
        if constexpr (RS == 2) {
          __syncthreads();  // both waves of each row half wrote their row sums
          if (wn == 0) {
            const float* rsum = reinterpret_cast<const float*>(smem + RSOFF);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int row = lane + 64 * h, gm = m0 + wm * 128 + row;
              if (gm < p.M) p.ss[(size_t)tn * p.ssld + gm] = rsum[wid * 128 + row] + rsum[(wid + 1) * 128 + row];
            }
          }
        }
        G4_STAMP(round, 7);
        continue;
      }
      if constexpr (TR) {
        // TR layout: lane (r16, q) holds output row i * 16 + r16, columns g * 16 + 4 q + e of output group g
        // (g = n-tile for the plain / bias output, h * 2 + jj for SwiGLU's h-th 32-column block).  Per m-tile:
        // SwiGLU / bias (+ GELU) / bf16 packing in registers (v_cvt_pk_bf16_f32 pairs), then groups (2 g2, 2 g2 + 1) pair up
        // by v_permlane16_swap: row-of-16-lanes q keeps group 2 g2 + (q & 1), columns (q >> 1) * 8 .. + 7 —
        // 16 contiguous bytes — and stores them with ONE buffer_store_dwordx4.  No LDS staging, no LDS waits
        // (the block-staged image cost 16-32 ds_write_b16 + 2-4 ds_read_b128 + 2 lgkmcnt(0) per m-tile).
        constexpr int NO = EPI == EPI_SWIGLU ? NT / 2 : NT;  // 16-column output groups
        static_assert(NO % 2 == 0, "TR pairs output groups");
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          uint32_t o[NO][2];
          float4v av[NT];  // the m-tile's accumulators (+ the split-K partials of the other units)
          G4_ACC_LOAD_SYNC(av, i);
          // RS 1 (folded RMSNorm consumer): every value of the lane's row i * 16 + r16 takes the row's 1/rms
          float sc = 1.f;
          if constexpr (RS == 1) sc = reinterpret_cast<const float*>(smem + RSV)[wm * 128 + i * 16 + r16];
#pragma unroll
          for (int g = 0; g < NO; ++g) {
            float v[4];
            if constexpr (EPI == EPI_SWIGLU) {
              const int gate = (g >> 1) * 4 + (g & 1);  // n-tile of the gate half; the up half is 2 further
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if constexpr (RS == 1)
                  v[e] = silu(av[gate][e] * sc) * (av[gate + 2][e] * sc);
                else
                  v[e] = silu(av[gate][e]) * av[gate + 2][e];
              }
            } else if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
              const float tb[4] = {__uint_as_float(tbias[g].x << 16), __uint_as_float(tbias[g].x & 0xffff0000u),
                                   __uint_as_float(tbias[g].y << 16), __uint_as_float(tbias[g].y & 0xffff0000u)};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float y = av[g][e] + tb[e];
                v[e] = EPI == EPI_BIAS_GELU ? gelu_tanh(y) : y;
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = RS == 1 ? av[g][e] * sc : av[g][e];
            }
            o[g][0] = pack_bf16x2(v[0], v[1]);
            o[g][1] = pack_bf16x2(v[2], v[3]);
          }
#pragma unroll
          for (int g2 = 0; g2 < NO / 2; ++g2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const auto r = __builtin_amdgcn_permlane16_swap(o[2 * g2][d], o[2 * g2 + 1][d], false, false);
              o[2 * g2][d] = r[0];
              o[2 * g2 + 1][d] = r[1];
            }
            const uint4v v = {o[2 * g2][0], o[2 * g2][1], o[2 * g2 + 1][0], o[2 * g2 + 1][1]};
            __builtin_amdgcn_raw_buffer_store_b128(v, rC, tr_vo[g2], tr_so(i), 0);
          }
          __builtin_amdgcn_sched_barrier(0);  // one m-tile's accumulators in flight at a time
          if (i == 0) G4_STAMP(round, 4);
          if (i == 3) G4_STAMP(round, 5);
          if (i == 7) G4_STAMP(round, 6);
        }
        G4_STAMP(round, 7);
        continue;  // no block barrier: the next tile's first wait + barrier orders everything
      }
    }

    // ---- epilogue: per wave 128 rows x CW bf16 columns through LDS, then 16 B stores
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * CW;
    constexpr int CPR_ = CW / 8;
    constexpr int kIt_ = 128 * CPR_ / 64;                                   // residual chunks per lane
    constexpr int kGrp_ = kIt_ % 16 == 0 ? 16 : (kIt_ % 12 == 0 ? 12 : 8);  // whole groups only
    // residual: the first group's loads go out before the accumulators are staged (into registers the main
    // loop's fragments held), so their HBM round trip overlaps the staging instead of following it
    uint4v rv0[EPI == EPI_RESIDUAL ? kGrp_ : 1];
    const int erow0 = __builtin_amdgcn_readfirstlane(m0 + wm * 128);  // uniform: buffer resources in SGPRs
    const int encol0 = EPI == EPI_SWIGLU ? n0 / 2 + wn * 8 * NT : n0 + wn * 16 * NT;
    // (a valid pointer and an empty range for the epilogues without a residual operand)
    const __amdgpu_buffer_rsrc_t rRes =
        EPI == EPI_RESIDUAL ? uniform_rsrc(p.R + (size_t)erow0 * p.ldc, max(0, min(p.M - erow0, 128)) * p.ldc * 2)
                            : uniform_rsrc(p.A, 0);
    if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
      for (int u = 0; u < kGrp_; ++u) {
        const int c = lane + 64 * u;
        const int row = c / CPR_, gn = encol0 + (c % CPR_) * 8;
        rv0[u] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rRes, (row * p.ldc + gn) * 2, 0, 0));
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4v t[NT];
#pragma unroll
      for (int jj = 0; jj < NT; ++jj) t[jj] = acc[i][jj];
      if constexpr (RS == 1) {
        const float4v sc = *reinterpret_cast<const float4v*>(smem + RSV + (wm * 128 + i * 16 + 4 * q) * 4);
#pragma unroll
        for (int jj = 0; jj < NT; ++jj) t[jj] *= sc;
      }
      if constexpr (EPI == EPI_SWIGLU) {
        // n-tiles of the wave: W rows wn*128 + jj*16; 32-row blocks alternate gate / up, so gate tiles
        // {0,1,4,5} pair with up tiles {2,3,6,7}
#pragma unroll
        for (int h = 0; h < NT / 4; ++h)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
#pragma unroll
            for (int e = 0; e < 4; ++e) t[h * 4 + jj][e] = silu(t[h * 4 + jj][e]) * t[h * 4 + jj + 2][e];
      }
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
        // bias re-read per m-tile (L1 hits): loaded once before the K loop it would pin NT VGPRs through it
        int bcol = n0 + wn * 16 * NT + r16;
        asm volatile("" : "+v"(bcol));
#pragma unroll
        for (int jj = 0; jj < NT; ++jj) {
          const int col = bcol + jj * 16;
          const float bv = col < p.N ? bf2f(p.R[col]) : 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float y = t[jj][e] + bv;
            t[jj][e] = EPI == EPI_BIAS_GELU ? gelu_erf(y) : y;
          }
        }
      }
#pragma unroll
      for (int jj = 0; jj < NT; ++jj) {
        if constexpr (EPI == EPI_SWIGLU) {
          if ((jj & 3) >= 2) continue;
        }
        const int oc = EPI == EPI_SWIGLU ? (jj >> 2) * 32 + (jj & 1) * 16 : jj * 16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = i * 16 + 4 * q + e, col = oc + r16;
          ot[row * CW + swz<CW>(row, col)] = f2bf(t[jj][e]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one m-tile's values live at a time
    }
    __syncthreads();
    constexpr int CPR = CW / 8;  // 16 B chunks per row
    const int ncol0 = EPI == EPI_SWIGLU ? n0 / 2 + wn * 8 * NT : n0 + wn * 16 * NT;
    const int ncols = EPI == EPI_SWIGLU ? p.N / 2 : p.N;
    if constexpr (EPI == EPI_RESIDUAL) {
      // Residual loads branch-free through a buffer resource over this wave's rows (rows past M read zeros
      // without a request; columns past N are never stored), kGrp of them in flight per lane before the
      // first add: loaded inside the store's bounds branch, every chunk waited its own HBM round trip
      // (vmcnt(0) per 16 B, the epilogue's whole latency).
      const int row0 = erow0;
      const __amdgpu_buffer_rsrc_t rR = rRes;
      constexpr int kIt = kIt_;                                   // chunks per lane: 32 (bn 256), 24 (bn 192)
      constexpr int kGrp = kGrp_;
      static_assert(kIt % kGrp == 0, "residual epilogue groups must tile the wave's chunks");
#pragma unroll 1
      for (int g0 = 0; g0 < kIt; g0 += kGrp) {
        uint4v rv[kGrp];
        if (g0 == 0) {
#pragma unroll
          for (int u = 0; u < kGrp; ++u) rv[u] = rv0[u];
        } else {
#pragma unroll
          for (int u = 0; u < kGrp; ++u) {
            const int c = lane + 64 * (g0 + u);
            const int row = c / CPR, gn = ncol0 + (c % CPR) * 8;
            rv[u] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rR, (row * p.ldc + gn) * 2, 0, 0));
          }
        }
#pragma unroll
        for (int u = 0; u < kGrp; ++u) {
          const int c = lane + 64 * (g0 + u);
          const int row = c / CPR, cch = c % CPR;
          const int gm = row0 + row, gn = ncol0 + cch * 8;
          float x[8], y[8];
          unpack8(*reinterpret_cast<const uint4v*>(ot + row * CW + swz<CW>(row, cch * 8)), x);
          unpack8(rv[u], y);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += y[e];
          const uint4v v = pack8(x);
          if (gm < p.M && gn < ncols) *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) = v;
          if constexpr (RS == 2) {
            // the row's squares over this wave's CW columns (of the rounded values the stream now holds):
            // the CPR lanes sharing a row are lanes 16 r' .. 16 r' + 15 (CPR = 16), a 4-step xor tree
            static_assert(CPR == 16, "RS 2 takes 256-wide tiles");
            float z[8];
            unpack8(gn < ncols ? v : uint4v{0u, 0u, 0u, 0u}, z);
            float sq = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sq += z[e] * z[e];
            sq += __shfl_xor(sq, 8);
            sq += __shfl_xor(sq, 4);
            sq += __shfl_xor(sq, 2);
            sq += __shfl_xor(sq, 1);
            if ((lane & 15) == 0) reinterpret_cast<float*>(smem + RSOFF)[wid * 128 + row] = sq;
          }
        }
      }
    } else {
#pragma unroll 4
      for (int c = lane; c < 128 * CPR; c += 64) {
        const int row = c / CPR, cch = c % CPR;
        const int gm = m0 + wm * 128 + row;
        const int gn = ncol0 + cch * 8;
        if (gm < p.M && gn < ncols)
          *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) =
              *reinterpret_cast<const uint4v*>(ot + row * CW + swz<CW>(row, cch * 8));
      }
    }
    __syncthreads();  // LDS free for the next tile
    if constexpr (RS == 2) {
      // the two waves of each 128-row half add their row sums (written before the barrier above) in a fixed
      // order and store the tile's partial; the next tile's epilogue rewrites them only after its main loop
      if (wn == 0) {
        const float* rsum = reinterpret_cast<const float*>(smem + RSOFF);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = lane + 64 * h, gm = m0 + wm * 128 + row;
          if (gm < p.M) p.ss[(size_t)tn * p.ssld + gm] = rsum[wid * 128 + row] + rsum[(wid + 1) * 128 + row];
        }
      }
    }
    G4_STAMP(round, 7);
  }
  // (VAR 64 / 96: the last tile's loop issued pieces nothing waited for; retire them before the
  // workgroup's LDS is released)
  if constexpr (PAP) G4_VM(0);
}

template <int EPI, int NT, int VAR, int RS, bool SK = false>
int launch3(const Params& p, hipStream_t s) {
  constexpr int lds = lds_bytes<NT, RS>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm4w_kernel<EPI, NT, VAR, RS, SK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  gemm4w_kernel<EPI, NT, VAR, RS, SK><<<8 * p.wpx, 256, lds, s>>>(p);
  return (int)hipGetLastError();
}

template <int EPI, int NT>
int launch(const Params& p, hipStream_t s, int var, int rs) {
  // schedule: 32 = the library-shaped main loop with the block-staged epilogue, 64 = the same loop with the
  // wave-local transposed-layout epilogue and the next persistent tile's first K tiles DMA'd inside this
  // one's last two iterations (even K tile counts only: odd ones run 32).  The planner picks per shape
  // (ops/gemm_plan.py).  rs: 1 = row-scaled epilogue (plain / SwiGLU), 2 = residual + row sums of squares.
  if (var != 64 || (p.KT & 1)) var = 32;
  if (p.S > 1) {
    // split-K builds: bn 256; plain / SwiGLU (RS 0, or 1: the row-scaled consumers of the folded chain, e.g.
    // the vocabulary projection's ragged last round) and residual (RS 0, or 2: the chain's producers)
    if constexpr (NT == 8 && (EPI == EPI_PLAIN || EPI == EPI_SWIGLU)) {
      if (rs == 0) return launch3<EPI, NT, 64, 0, true>(p, s);
      if (rs == 1) return launch3<EPI, NT, 64, 1, true>(p, s);
    }
    if constexpr (NT == 8 && EPI == EPI_RESIDUAL) {
      if (rs == 0) return launch3<EPI, NT, 64, 0, true>(p, s);
      if (rs == 2) return launch3<EPI, NT, 64, 2, true>(p, s);
    }
    return -1;
  }
  if (rs == 1) {
    if constexpr (EPI == EPI_PLAIN || EPI == EPI_SWIGLU) {
      return var == 64 ? launch3<EPI, NT, 64, 1>(p, s) : launch3<EPI, NT, 32, 1>(p, s);
    }
    return -1;
  }
  if (rs == 2) {
    if constexpr (EPI == EPI_RESIDUAL && NT == 8) {
      return var == 64 ? launch3<EPI, NT, 64, 2>(p, s) : launch3<EPI, NT, 32, 2>(p, s);
    }
    return -1;
  }
  return var == 64 ? launch3<EPI, NT, 64, 0>(p, s) : launch3<EPI, NT, 32, 0>(p, s);
}

template <int NT>
int dispatch(const Params& p, int epi, hipStream_t s, int var, int rs) {
  switch (epi) {
    case EPI_PLAIN: return launch<EPI_PLAIN, NT>(p, s, var, rs);
    case EPI_RESIDUAL: return launch<EPI_RESIDUAL, NT>(p, s, var, rs);
    case EPI_BIAS: return rs ? -1 : launch<EPI_BIAS, NT>(p, s, var, 0);
    case EPI_BIAS_GELU: return rs ? -1 : launch<EPI_BIAS_GELU, NT>(p, s, var, 0);
    case EPI_SWIGLU:
      if constexpr (NT == 8) return launch<EPI_SWIGLU, NT>(p, s, var, rs);
      return -1;
  }
  return -1;
}

int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8) cus = 256;
  }
  return cus;
}

}  // namespace g4w
}  // namespace lwc

// C = A . W^T (epilogue epi as lwc_gemm8p: 0 plain, 1 + residual, 2 SwiGLU over 32-row gate/up interleaved W,
// 3 + bias, 4 gelu(. + bias)); bn = 256 or 192 (W rows per tile; SwiGLU needs 256).  Requires K % 64 == 0,
// N % 8 == 0, lda / ldc % 8 == 0.  Folded RMSNorm (file head): ss [P][ssld] with P >= 1 partial row sums of
// squares (epi 0 / 2) scales the accumulator rows by rsqrt(sum / K + eps); ss [N/256][ssld] (epi 1, bn 256)
// makes the residual epilogue write those partials of its output.  var: schedule, 64 or 32 (anything else).
// gm: m-tiles per group of the grouped tile order (an XCD's consecutive tiles run gm m-tiles down each n column).
// splits / split_from / part / cnt: split-K of the tiles from split_from on (VAR 64; see Params).
extern "C" int lwc_gemm4w(const void* A, const void* W, void* C, const void* R, int M, int N, int K, int lda, int ldc,
                          int epi, int bn, float* ss, int ssld, int rs_mode, int P, float eps, int var, int gm,
                          int splits, int split_from, float* part, int* cnt, hipStream_t s) {
  using namespace lwc::g4w;
  if (K % 64 != 0 || K < 64 || N % 8 != 0 || lda % 8 != 0 || ldc % 8 != 0) return -1;
  if (bn != 256 && bn != 192) return -1;
  // (A: every buffer resource spans one tile's 256 rows, so any M; W: one tile's bn rows)
  if ((long long)256 * lda * 2 >= (1LL << 31) || (long long)bn * K * 2 >= (1LL << 31)) return -1;
  if (epi == EPI_SWIGLU && (N % 64 != 0 || bn != 256)) return -1;
  if ((epi == EPI_RESIDUAL || epi == EPI_BIAS || epi == EPI_BIAS_GELU) && R == nullptr) return -1;
  if (rs_mode < 0 || rs_mode > 2 || (rs_mode && (ss == nullptr || ssld < M || ssld % 4 != 0))) return -1;
  if (rs_mode == 1 && ((epi != EPI_PLAIN && epi != EPI_SWIGLU) || P < 1 || P > 16)) return -1;
  if (rs_mode == 2 && (epi != EPI_RESIDUAL || bn != 256)) return -1;
  if (M == 0 || N == 0) return 0;
  const int tiles_m = (M + 255) / 256, tiles_n = (N + bn - 1) / bn, tiles = tiles_m * tiles_n;
  // split-K (VAR 64 only): tiles [split_from, tiles) run as `splits` units of about K / splits each (an even K
  // tile count, like every VAR 64 unit: KT even, KT / 2 >= splits); workspace part [(tiles - split_from) * (splits - 1) * 256 * bn] fp32,
  // cnt [2 * tiles] int32 zeroed once
  const int KT = K / 64;
  if (splits > 1) {
    if (var != 64 || KT % 2 != 0 || KT / 2 < splits || part == nullptr || cnt == nullptr) return -1;
  } else {
    splits = 1;
  }
  const int full = splits > 1 ? std::max(0, std::min(split_from, tiles)) : tiles;
  const int units = full + (tiles - full) * splits;
  const int wpx = std::min(device_cus() / 8, (units + 7) / 8);
  // grouped tile order: an XCD's wpx consecutive tiles run gm m-tiles down each n column.  Auto (gm <= 0): 4
  // for the decode projections (up to 128 n-tiles: o / down / qkv / gate|up at M = 4096 read 1-4 % faster
  // than with 8 in scripts/microbench.py g4ab, G4_GMS), 8 for the vocabulary projection's 501 n-tiles
  if (gm <= 0) gm = tiles_n > 128 ? 8 : 4;
  Params p{(const lwc::bf16_t*)A, (const lwc::bf16_t*)W, (lwc::bf16_t*)C, (const lwc::bf16_t*)R, M, N, K, lda, ldc,
           tiles_m, tiles_n, KT, std::max(1, gm), wpx, tiles, ss, P, ssld, eps, full, splits, units, part, cnt,
           cnt ? cnt + tiles : nullptr};
  return bn == 256 ? dispatch<8>(p, epi, s, var, rs_mode) : dispatch<6>(p, epi, s, var, rs_mode);
}
