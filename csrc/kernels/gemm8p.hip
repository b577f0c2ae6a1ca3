// K6 dense projection GEMM, 8-phase schedule + stream-K tail: C = A . W^T for the decode-batch projections
// (M = decode batch 512..4096; N, K >= 4096), with fused epilogues.
//
//   C[M, N]  = A[M, K] . W[N, K]^T  (+ R)            EPI_PLAIN / EPI_RESIDUAL
//   H[M, N/2] = silu(A . Wg^T) * (A . Wu^T)          EPI_SWIGLU, W rows gate/up interleaved in blocks of 32
//                                                     (ops.swiglu_interleave), so one tile holds both halves
//
// Tile pipeline (cdna_hip_programming.md §5 "The 256² 8-phase template", written for this kernel's operand split):
//   workgroup : 8 waves (512 threads) = 2 (M) x 4 (N); wave tile 128 x 64 = 8 x 4 MFMA 16x16 tiles,
//               mfma_f32_16x16x32_bf16, 128 fp32 accumulators per lane.
//   K tile    : BK = 64 (128 B per row), staged global -> LDS by LDS-DMA (global_load_lds_dwordx4) in four
//               16 KiB UNITS, each of which is exactly what one compute phase reads:
//                 A0 = rows {0..63, 128..191}   (quadrant mi=0 of both wave rows)
//                 A1 = rows {64..127, 192..255} (mi=1)
//                 B0 = W rows {0..31, 64..95, 128..159, 192..223} (ni=0 of the 4 wave columns)
//                 B1 = the other 128 W rows (ni=1)
//               Two K-tile buffers (128 KiB LDS).
//   phases    : 4 per K tile, one C quadrant (4 x 2 MFMA tiles x K 64 = 16 MFMAs) each:
//                 P1 reads B0 + A0 -> acc[0..3][0..1]     stage A0(t+1)  vmcnt(4) (retires B1(t))
//                 P2 reads B1      -> acc[0..3][2..3]     stage B0(t+1)  vmcnt(4) (retires A1(t))
//                 P3 reads A1      -> acc[4..7][2..3]     stage B1(t+1)
//                 P4 (registers)   -> acc[4..7][0..1]     stage A1(t+1)  vmcnt(4) (retires A0, B0 (t+1))
//               Each phase: ds_reads, 2 x glds, counted vmcnt, s_barrier, MFMA cluster at raised priority,
//               s_barrier.  vmcnt never reaches 0 inside the loop: 2-3 units stay in flight across the
//               barriers.  The two wave rows run one barrier apart (wr == 1 passes an extra barrier first),
//               so on every SIMD one wave issues MFMAs while its partner reads LDS and issues loads.
//   hazards   : RAW - a unit is read in the phase after the wait that retired it (every wave waits for its
//               own DMAs, then the barrier).  WAR - a unit buffer is re-staged 4-5 phases after its last read
//               (>= 2 needed with the staggered wave rows).
//   LDS image : lane-linear DMA image, 16 B chunk c of unit row r stored at chunk c ^ ((r >> 1) & 7): the
//               16 lanes of a ds_read_b128 group (16 consecutive rows, same chunk) hit 16 distinct bank quads.
//               The swizzle is applied to the DMA SOURCE address and to the read (both sides).
//
// Work distribution (persistent, one workgroup per CU, grid = 8 XCDs x wpx):
//   The decode shapes do not divide into whole rounds of 256 tiles (qkv at M=3072: 288 tiles = 1.1 rounds;
//   o / down: 192 = 0.75; gate_up: 1344 = 5.25), so a plain one-tile-per-workgroup grid idles 12-44 % of the
//   chip in its last round.  Here the first `sk_tiles` tiles (the remainder plus one full round) are split
//   by K iterations (stream-K): each XCD owns a contiguous, tile-aligned share of them and its wpx workgroups
//   split that share's K iterations evenly.  The remaining tiles run data-parallel, one per workgroup per
//   round, XCD x taking wpx consecutive tiles (m fastest: the XCD's tiles share W panels in its L2).
//   A tile cut between workgroups is finished by the one holding its last K iteration (the finaliser),
//   which adds the fp32 partials the others wrote to the workspace.  Each workgroup walks its stream-K
//   range backwards, so it publishes its partial (range end) first and finalises (range start) last, and
//   a finaliser only waits on LOWER block ids of its own XCD — workgroups dispatched earlier, hence
//   resident: no co-residency assumption, no deadlock.  Partial hand-off: plain stores, vmcnt(0), barrier,
//   agent-scope release + flag store; the reader polls the flag, agent-scope acquire, resets the flag for
//   the next launch (flags start zeroed), barrier, plain loads.
//   epilogue  : accumulators -> bf16 (SwiGLU / residual applied in registers) -> LDS -> 16 B row stores.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace lwc {
namespace g8p {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kUnitB = 128 * 128;   // 128 rows x 128 B
constexpr int kBufB = 4 * kUnitB;   // one K tile: A0 A1 B0 B1
constexpr int kLdsB = 2 * kBufB;    // 128 KiB
constexpr int kUA0 = 0, kUA1 = kUnitB, kUB0 = 2 * kUnitB, kUB1 = 3 * kUnitB;
constexpr int kPartialF = 256 * 256;  // fp32 partial tile per workgroup

enum Epi { EPI_PLAIN = 0, EPI_RESIDUAL = 1, EPI_SWIGLU = 2, EPI_BIAS = 3, EPI_BIAS_GELU = 4 };

struct Params {
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  const bf16_t* R;     // EPI_RESIDUAL: residual [M, ldc]; EPI_BIAS / EPI_BIAS_GELU: bias [N]
  float* ws;    // [8 * wpx, kPartialF] partial tiles
  int* flags;   // [8 * wpx] partial-ready flags (zero between launches)
  int M, N, K, lda, ldc;  // N = rows of W
  int tiles_m, tiles_n, KT;
  int gm;  // tile order: groups of gm m-tiles, n fastest across a group (32 consecutive tiles ~ 4 x 8)
  int wpx, sk_tiles, dp_rounds;
};

LWC_DEVICE float4v mfma(const uint4v& a, const uint4v& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// x * sigmoid(x) with v_rcp_f32 (1 ulp) instead of the IEEE division sequence (v_div_scale x2, v_div_fmas,
// v_div_fixup around an rcp: ~9 VALU per element in an epilogue of 256 per lane); the result is rounded
// to bf16 (or e4m3) anyway.  x -> -inf: rcp(inf) = 0, x * 0 = -0 as the division gives
LWC_DEVICE float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// erf by Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below bf16's resolution): one exp, one rcp and a
// 5-term polynomial — the libm erff's branches made the fused epilogue cost more than a separate pass.
LWC_DEVICE float erf_as(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * a);  // v_rcp_f32 (1 ulp): __frcp_rn is a full division sequence
  const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.f - y * __expf(-a * a), x);
}
LWC_DEVICE float gelu_erf(float x) { return 0.5f * x * (1.f + erf_as(x * 0.70710678118654752f)); }

// K-iteration range [a, e) of stream-K workgroup j (of wpx) on XCD x.
LWC_DEVICE void sk_range(const Params& p, int x, int j, int& a, int& e) {
  const int t0 = p.sk_tiles * x / 8, t1 = p.sk_tiles * (x + 1) / 8;
  const int ix = (t1 - t0) * p.KT;
  a = t0 * p.KT + (int)((long long)ix * j / p.wpx);
  e = t0 * p.KT + (int)((long long)ix * (j + 1) / p.wpx);
}

// Tile t -> (m, n): grouped order, gm m-tiles per group, m fastest inside the group, so the wpx
// consecutive tiles an XCD runs in one round form a ~gm x (wpx / gm) block whose A and W panels its
// L2 shares (a plain m-fastest order spans every m-tile of the matrix: 1.5x the L2 misses at 4096^3).
LWC_DEVICE void tile_mn(const Params& p, int t, int& m, int& n) {
  const int group = p.gm * p.tiles_n;
  const int first_m = (t / group) * p.gm;
  const int gsz = min(p.tiles_m - first_m, p.gm);
  const int in = t % group;
  m = first_m + in % gsz;
  n = in / gsz;
}

template <int EPI>
__global__ void __launch_bounds__(512) gemm8p_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int KT = p.KT;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;

  int sk_a = 0, sk_e = 0;
  if (p.sk_tiles > 0) sk_range(p, xcd, j, sk_a, sk_e);
  int it = sk_e, round = 0;

  while (true) {
    // ---- next work item: stream-K segments (backwards), then data-parallel tiles ----
    int tile, klo, khi;
    if (it > sk_a) {
      tile = (it - 1) / KT;
      const int seg = max(sk_a, tile * KT);
      klo = seg - tile * KT;
      khi = it - tile * KT;
      it = seg;
    } else if (round < p.dp_rounds) {
      tile = p.sk_tiles + round * 8 * p.wpx + xcd * p.wpx + j;
      klo = 0;
      khi = KT;
      ++round;
    } else {
      break;
    }
    int tm, tn;
    tile_mn(p, tile, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    // Lane geometry is re-derived per item from an opaque copy of threadIdx.x: hoisted out of the
    // item loop, the ~100 epilogue / fragment addresses it feeds would stay live and spill.
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int wr = wid >> 2, wc = wid & 3;

    // per-thread DMA geometry (byte offsets from the tile's buffer base): unit u, instruction i -> unit row
    // ru = i*64 + tid/8 at LDS chunk tid%8, which holds global chunk chk of that row (swizzle on the source)
    const int chk = ((tid & 7) ^ ((tid >> 4) & 7)) * 8;
    uint32_t voA[2][2], voW[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        voA[h][i] = (uint32_t)(((i * 128 + h * 64 + (tid >> 3)) * p.lda + chk) * 2);
        voW[h][i] = (uint32_t)((((2 * i + (tid >> 8)) * 64 + h * 32 + ((tid >> 3) & 31)) * p.K + chk) * 2);
      }
    const int dst_lane0 = wid * 64 * 16;  // wave-uniform LDS destination of instruction 0 inside a unit
    const int sw = (r16 >> 1) & 7;
    const int off0 = r16 * 128 + ((q ^ sw) << 4), off1 = r16 * 128 + (((4 + q) ^ sw) << 4);

    // buffer descriptors of the tile's A rows / W rows: rows past M / N fall outside num_records and
    // load as zeros (their outputs are not stored)
    const __amdgpu_buffer_rsrc_t rA = uniform_rsrc(p.A + (size_t)m0 * p.lda, (p.M - m0) * p.lda * 2);
    const __amdgpu_buffer_rsrc_t rW = uniform_rsrc(p.W + (size_t)n0 * p.K, min(p.N - n0, 256) * p.K * 2);
    auto stage = [&](int u, uint8_t* buf, int kt) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        auto* dst = (__attribute__((address_space(3))) void*)(buf + u * kUnitB + i * 512 * 16 + dst_lane0);
        if (u < 2)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, voA[u][i], kt * 128, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, dst, 16, voW[u - 2][i], kt * 128, 0, 0);
      }
    };
    auto rd = [&](const uint8_t* u, int row0, uint4v& f0, uint4v& f1) {
      f0 = *reinterpret_cast<const uint4v*>(u + row0 * 128 + off0);
      f1 = *reinterpret_cast<const uint4v*>(u + row0 * 128 + off1);
    };

    // acc[i][jj] = 16 x 16 tile (i, jj) of the wave's 128 x 64 (lane: rows 4q..4q+3 of column r16).
    // (The 32x32x16 MFMA with the same units and phases measured ~10 % slower on every shape.)
    float4v acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = float4v{0.f, 0.f, 0.f, 0.f};

    uint4v a[4][2], b0[2][2], b1[2][2];
    auto mma = [&](int i0, int j0, const uint4v (&bb)[2][2]) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) acc[i0 + i][j0 + jj] = mfma(a[i][s], bb[jj][s], acc[i0 + i][j0 + jj]);
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
#define G8_MFMA(i0, j0, bb)                          \
  G8_BAR();                                          \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_s_setprio(1);                     \
  mma(i0, j0, bb);                                   \
  __builtin_amdgcn_s_setprio(0);                     \
  G8_BAR()

    const int nt = khi - klo;  // K tiles of this item; tile r lives in LDS buffer r & 1
#define G8_STAGE(U, R) stage(U, smem + ((R) & 1) * kBufB, klo + (R))
#define G8_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
#define G8_TILE(R, ST1, ST2, ST3, ST4, W1, W2, W4) \
  {                                                \
    uint8_t* cb = smem + ((R) & 1) * kBufB;        \
    rdB(cb, kUB0, b0);                             \
    __builtin_amdgcn_sched_barrier(0);             \
    rdA(cb, kUA0);                                 \
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
    // unit issue runs 4 units ahead of consumption: tile r stages tile r+1 (A0 B0 B1 A1 in P1..P4), 2 units
    // in flight at each wait.  (A 6-unit lead — B1, A1 of r+1 and A0, B0 of r+2, vmcnt(8) — measured the
    // same at 4096^3 and on the decode shapes: the DMA latency is covered, the cost is in the barriers.)
    G8_STAGE(0, 0); G8_STAGE(2, 0); G8_STAGE(3, 0); G8_STAGE(1, 0);
    G8_VM(4);
    G8_BAR();
    if (wr == 1) G8_BAR();  // stagger the two wave rows by one barrier
    int r = 0;
    for (; r < nt - 1; ++r)
      G8_TILE(r, G8_STAGE(0, r + 1), G8_STAGE(2, r + 1), G8_STAGE(3, r + 1), G8_STAGE(1, r + 1), G8_VM(4), G8_VM(4),
              G8_VM(4))
    G8_TILE(r, , , , , G8_VM(2), G8_VM(0), )
#undef G8_TILE
#undef G8_VM
#undef G8_STAGE
    if (wr == 0) G8_BAR();  // re-align the wave rows
#undef G8_MFMA
#undef G8_BAR

    // ---- stream-K hand-off ----
    if (khi < KT) {  // contributor: publish the fp32 partial, no store of C
      float4v* wsp = reinterpret_cast<float4v*>(p.ws + (size_t)blockIdx.x * kPartialF);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) wsp[(wid * 32 + i * 4 + jj) * 64 + lane] = acc[i][jj];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(p.flags + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;  // the next item's prologue only touches LDS after this item's last barrier
    }
    if (klo > 0) {  // finaliser: add the partials of the lower workgroups of this XCD covering [0, klo)
      const int tile_begin = tile * KT;
      for (int jp = j - 1; jp >= 0; --jp) {
        int pa, pe;
        sk_range(p, xcd, jp, pa, pe);
        if (pe <= tile_begin) break;
        if (pa == pe) continue;  // empty range: no partial
        const int blk = jp * 8 + xcd;
        if (tid == 0) {
          while (__hip_atomic_load(p.flags + blk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            __builtin_amdgcn_s_sleep(1);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(p.flags + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const float4v* wsq = reinterpret_cast<const float4v*>(p.ws + (size_t)blk * kPartialF);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[i][jj] += wsq[(wid * 32 + i * 4 + jj) * 64 + lane];
          __builtin_amdgcn_sched_barrier(0);  // 4 loads in flight at a time: no 128-VGPR load burst
        }
        if (pa <= tile_begin) break;
      }
    }

    __syncthreads();  // every wave is done reading the K buffers: LDS is reused by the epilogue

    // ---- epilogue: per wave 128 rows x CW bf16 columns through LDS, then 16 B stores ----
    constexpr int CW = EPI == EPI_SWIGLU ? 32 : 64;
    constexpr int NJ = CW / 16;
    if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][jj][r] = silu(acc[i][jj][r]) * acc[i][jj + 2][r];
    }
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
      // bias (+ exact erf GELU) on the fp32 accumulators, before the one bf16 rounding: the encoder's
      // FFN1 needs no separate bias_gelu pass over [M, ffn]
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int col = n0 + wc * 64 + jj * 16 + r16;
        const float bv = col < p.N ? bf2f(p.R[col]) : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = acc[i][jj][r] + bv;
            acc[i][jj][r] = EPI == EPI_BIAS_GELU ? gelu_erf(y) : y;
          }
      }
    }
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * CW;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + 4 * q + r, col = jj * 16 + r16;
          ot[row * CW + (col ^ (((row & 7) << 3) % CW))] = f2bf(acc[i][jj][r]);
        }
    __syncthreads();
    constexpr int CPR = CW / 8;    // 16 B chunks per row
    constexpr int RPI = 64 / CPR;  // rows per store instruction
    const int cch = lane % CPR;
    const int ncol0 = EPI == EPI_SWIGLU ? n0 / 2 + wc * 32 : n0 + wc * 64;
    const int ncols = EPI == EPI_SWIGLU ? p.N / 2 : p.N;
    if constexpr (EPI == EPI_RESIDUAL) {
      // residual rows through a buffer resource (rows past M read zeros, no request), all of a group's loads
      // in flight before the first add — inside the store's bounds branch each 16 B load waited its own
      // HBM round trip
      const int row0 = m0 + wr * 128;
      const int rows_here = max(0, min(p.M - row0, 128));
      const __amdgpu_buffer_rsrc_t rR = uniform_rsrc(p.R + (size_t)row0 * p.ldc, rows_here * p.ldc * 2);
      const int gn = ncol0 + cch * 8;
      constexpr int kIt = 128 / RPI, kGrp = kIt < 16 ? kIt : 16;
      static_assert(kIt % kGrp == 0, "residual epilogue groups must tile the wave's rows");
#pragma unroll 1
      for (int k0 = 0; k0 < kIt; k0 += kGrp) {
        uint4v rv[kGrp];
#pragma unroll
        for (int u = 0; u < kGrp; ++u) {
          const int row = lane / CPR + RPI * (k0 + u);
          rv[u] = __builtin_bit_cast(uint4v, __builtin_amdgcn_raw_buffer_load_b128(rR, (row * p.ldc + gn) * 2, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < kGrp; ++u) {
          const int row = lane / CPR + RPI * (k0 + u);
          float x[8], y[8];
          unpack8(*reinterpret_cast<const uint4v*>(ot + row * CW + ((cch * 8) ^ (((row & 7) << 3) % CW))), x);
          unpack8(rv[u], y);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += y[e];
          if (row0 + row < p.M && gn < ncols) *reinterpret_cast<uint4v*>(p.C + (size_t)(row0 + row) * p.ldc + gn) = pack8(x);
        }
      }
    } else {
#pragma unroll 4
      for (int k = 0; k < 128 / RPI; ++k) {
        const int row = lane / CPR + RPI * k;
        const int gm = m0 + wr * 128 + row;
        const int gn = ncol0 + cch * 8;
        if (gm < p.M && gn < ncols)
          *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) =
              *reinterpret_cast<const uint4v*>(ot + row * CW + ((cch * 8) ^ (((row & 7) << 3) % CW)));
      }
    }
    __syncthreads();  // LDS free for the next item's prologue
  }
}

template <int EPI>
int launch(const Params& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsB);
    attr = true;
  }
  gemm8p_kernel<EPI><<<8 * p.wpx, 512, kLdsB, s>>>(p);
  return (int)hipGetLastError();
}

// Experiment knob (A/B in one process, scripts/microbench.py g8ab): LWC_G8_GM, the tile group height
// (default 8; 1 = plain m-fastest order).
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
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

}  // namespace g8p
}  // namespace lwc

// Workgroups the kernel launches (= partial slots / flags the workspace must hold): 8 x (CUs / 8).
extern "C" int lwc_gemm8p_slots() { return 8 * (lwc::g8p::device_cus() / 8); }

// epi 0: C = A W^T; 1: C = A W^T + R; 2: C[:, :N/2] = silu(gate) * up over 32-row interleaved W (N % 64 == 0);
// 3: C = A W^T + bias (R = bias [N]); 4: C = gelu(A W^T + bias) (exact erf GELU).
// Requires K % 64 == 0, N % 8 == 0, lda / ldc % 8 == 0 (16-byte rows); ws >= slots * 65536 floats,
// flags >= slots ints, zero on the first call (the kernel leaves them zero).
extern "C" int lwc_gemm8p(const void* A, const void* W, void* C, const void* R, float* ws, int* flags, int M, int N,
                          int K, int lda, int ldc, int epi, hipStream_t s) {
  using namespace lwc::g8p;
  if (K % 64 != 0 || K < 64 || N % 8 != 0 || lda % 8 != 0 || ldc % 8 != 0) return -1;
  if ((long long)M * lda * 2 >= (1LL << 31) || 256LL * K * 2 >= (1LL << 31)) return -1;  // 32-bit buffer offsets
  if (epi == EPI_SWIGLU && N % 64 != 0) return -1;
  if ((epi == EPI_RESIDUAL || epi == EPI_BIAS || epi == EPI_BIAS_GELU) && R == nullptr) return -1;
  if (M == 0 || N == 0) return 0;
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256, tiles = tiles_m * tiles_n, KT = K / 64;
  int wpx = device_cus() / 8;
  // at least ~8 K iterations per stream-K workgroup: shrink the grid for small problems
  const long long iters = (long long)tiles * KT;
  if (iters < 8LL * 8 * wpx) wpx = (int)std::max(1LL, iters / 64);
  const int G = 8 * wpx;
  int sk = 0, dp = tiles / G;
  if (tiles % G != 0) {
    dp = std::max(0, tiles / G - 1);
    sk = tiles - dp * G;
  }
  Params p{(const lwc::bf16_t*)A, (const lwc::bf16_t*)W, (lwc::bf16_t*)C, (const lwc::bf16_t*)R, ws, flags,
           M, N, K, lda, ldc, tiles_m, tiles_n, KT, std::max(1, env_int("LWC_G8_GM", 8)), wpx, sk, dp};
  switch (epi) {
    case EPI_PLAIN: return launch<EPI_PLAIN>(p, s);
    case EPI_RESIDUAL: return launch<EPI_RESIDUAL>(p, s);
    case EPI_SWIGLU: return launch<EPI_SWIGLU>(p, s);
    case EPI_BIAS: return launch<EPI_BIAS>(p, s);
    case EPI_BIAS_GELU: return launch<EPI_BIAS_GELU>(p, s);
  }
  return -1;
}
