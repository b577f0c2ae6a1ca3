// K6 dense fp8 (OCP e4m3) projection GEMM on the 4-wave schedule of gemm4w:
//
//   C[M, N] = (A[M, K] . W[N, K]^T) * a_scale[row] * w_scale[col]        (bf16 out)
//
// Why: gemm8g (8 waves = 2 per SIMD, wave tile 128 x 64) runs the fp8 projections at ~2.2-2.5 PF/s, about half
// of the e4m3 MFMA rate.  Its LDS traffic is the limit: per 32 cycles of one 16x16x128 MFMA a 128 x 64 wave
// tile reads 12 KiB of fragments per 32 MFMAs, i.e. 24 B/cycle per SIMD — 96 B/cycle for the CU's four busy
// waves plus 32 B/cycle of LDS-DMA writes, the LDS's whole 128 B/cycle.  gemm4w's layout (ONE wave per SIMD
// holding a 128 x 128 tile in 256 AGPRs) reads 32 KiB per 64 MFMAs = 16 B/cycle per SIMD: 64 + 32 B/cycle.
//
// fp8 mapping of gemm4w's K tile: the LDS image is byte for byte gemm4w's (rows x 128 B, 16 B chunk c of row r
// at chunk c ^ ((r >> 1) & 7), LDS-DMA with the swizzle on the source).  A K tile is 128 e4m3 = ONE
// v_mfma_f32_16x16x128_f8f6f4 per 16 x 16 output block, whose 32-byte operand of lane (r16, q) is K bytes
// [16q, 16q + 16) and [64 + 16q, 64 + 16q + 16) of row r16 (scripts/mx_probe.py): chunks q and 4 + q, which two
// ds_read_b128 land directly in the two halves of the operand's register octet.
//
// Schedule per K tile r (every MFMA needs both halves of its fragments, so gemm4w's k-step double buffer
// becomes: A fragments double-buffered by tile (2 x 8 octets), W fragments split by column half):
//   half 1: MFMAs of columns 0..3 (all 8 row blocks) on A_r, B_r[0..3]  || reads of B_r[4..7]
//           lgkmcnt(0), vmcnt(0) (tile r+1 landed), s_barrier   — every wave is done reading tile r's buffer
//   half 2: MFMAs of columns 4..7 on A_r, B_r[4..7]  || LDS-DMA of tile r+2 into tile r's buffer,
//                                                      reads of A_{r+1} (other set) and B_{r+1}[0..3]
// One barrier per K tile; the DMA of a tile has ~one K tile of lead.  The loop is unrolled by two (the A set
// is a compile-time index).  MFMAs are inline asm with the accumulator tied in place (see gemm4w.hip).
//
// Work distribution, epilogue staging and store: as gemm4w (persistent, XCD-grouped tile order; accumulators
// x row scale x column scale -> bf16 -> LDS -> 16 B row stores).
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace lwc {
namespace g4w {
int env_int(const char* name, int dflt);
int device_cus();
}  // namespace g4w

namespace g4w8 {

typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef int v4i32 __attribute__((ext_vector_type(4)));

constexpr int kOp = 256 * 128;  // one operand's K tile: 256 rows x 128 B
constexpr int kBuf = 2 * kOp;   // A | W
constexpr int kLds = 2 * kBuf;  // two K tiles: 128 KiB (the epilogue staging reuses all of it)
constexpr int kPieces = 16;     // LDS-DMA pieces (1 KiB) per wave per K tile: 8 of A, 8 of W

struct Params {
  const uint8_t* A;       // [M, lda] e4m3
  const uint8_t* W;       // [N, K] e4m3
  bf16_t* C;              // [M, ldc]
  const float* a_scale;   // [M]
  const float* w_scale;   // [N]
  int M, N, K, lda, ldc;  // K, lda in bytes (= elements)
  int tiles_m, tiles_n, KT, gm, wpx, tiles;
};

LWC_DEVICE void mfma8(float4v& d, const v8i32& a, const v8i32& b) {
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
}
// the first non-MFMA read of an accumulator after the last (opaque) MFMA: the 16x16x128 f8f6f4 MFMA runs twice
// the passes of the bf16 16x16x32 one, and gemm4w's single s_nop 15 let the epilogue read the last MFMA's block
// (rows 4k+2 / 4k+3 of acc[7][7]) before it was written (seen whenever no DMA wait preceded the drain)
#define G48_DRAIN() asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory")
#define G48_BAR() __builtin_amdgcn_s_barrier()
#define G48_VM(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")
#define G48_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

LWC_DEVICE void tile_mn(const Params& p, int t, int& m, int& n) {
  const int group = p.gm * p.tiles_n;
  const int first_m = (t / group) * p.gm;
  const int gsz = min(p.tiles_m - first_m, p.gm);
  const int in = t % group;
  m = first_m + in % gsz;
  n = in / gsz;
}

// epilogue staging column of (row, col) in a 128-wide bf16 row: XOR by 8-column chunks
LWC_DEVICE int swz(int row, int col) { return col ^ ((row & 7) << 3); }

__global__ void __launch_bounds__(256, 1) gemm4w8_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int KT = p.KT + (p.KT & 1);  // virtual K tiles (even; see piece)
  const int xcd = blockIdx.x & 7, jw = blockIdx.x >> 3;

  for (int round = 0;; ++round) {
    const int tile = round * 8 * p.wpx + xcd * p.wpx + jw;
    if (tile >= p.tiles) break;
    int tm, tn;
    tile_mn(p, tile, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int wm = wid >> 1, wn = wid & 1;

    // ---- LDS-DMA: piece k of wave wid covers operand rows k*32 + wid*8 + lane/8, LDS chunk lane%8 (holding
    // global chunk (lane%8) ^ ((row >> 1) & 7)) — gemm4w's pieces, in bytes
    const int drow = wid * 8 + (lane >> 3);
    const int dchk = ((lane & 7) ^ ((drow >> 1) & 7)) * 16;
    const uint32_t voA = (uint32_t)(drow * p.lda + dchk);
    const uint32_t voW = (uint32_t)(drow * p.K + dchk);
    const int sA = 32 * p.lda, sW = 32 * p.K;
    const int dst0 = wid * 1024;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.A + (size_t)m0 * p.lda), (short)0, (p.M - m0) * p.lda, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.W + (size_t)n0 * p.K), (short)0, min(p.N - n0, 256) * p.K, 0x00020000);
    // K tiles are counted VIRTUALLY: an odd count gets a leading all-zero tile (its DMA offsets lie past the
    // buffer ranges: the hardware writes zeros, no request; its MFMAs add 0), so the loop is one path of
    // tile PAIRS — two loop paths joined before the epilogue made the compiler copy accumulators at the join,
    // ahead of the MFMA drain.
    const int odd = p.KT & 1;
    auto piece = [&](uint8_t* buf, int v, int k) {
      const int kt = v - odd;  // real K tile (-1: the zero tile)
      if (k < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rA, (__attribute__((address_space(3))) void*)(buf + k * 4096 + dst0), 16, voA,
            kt < 0 ? (1 << 30) : k * sA + kt * 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rW, (__attribute__((address_space(3))) void*)(buf + kOp + (k - 8) * 4096 + dst0), 16, voW,
            kt < 0 ? (1 << 30) : (k - 8) * sW + kt * 128, 0, 0);
    };

    // ---- fragment reads: row / column block i adds i * 16 rows = i * 2048 B; the swizzle depends on r16 only
    const int sw = (r16 >> 1) & 7;
    const int offA0 = (wm * 128 + r16) * 128 + ((q ^ sw) << 4);
    const int offA1 = (wm * 128 + r16) * 128 + (((4 + q) ^ sw) << 4);
    const int offB0 = kOp + (wn * 128 + r16) * 128 + ((q ^ sw) << 4);
    const int offB1 = kOp + (wn * 128 + r16) * 128 + (((4 + q) ^ sw) << 4);

    float4v acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    v8i32 fa[2][8], fb[8];
    // read k (< 16) of an operand's fragments: block k / 2, half k % 2 (chunk q / chunk 4 + q).  The low half
    // starts a NEW octet (upper half undefined until the second read): inserting into the register's previous
    // value would keep that value — the fragment set of two tiles ago — alive, three A sets, and spill.
    auto lo8 = [](const v4i32& v) { return __builtin_shufflevector(v, v, 0, 1, 2, 3, -1, -1, -1, -1); };
    auto rdA = [&](const uint8_t* buf, v8i32(&f)[8], int k) {
      if (k & 1)
        f[k >> 1].s4567 = *reinterpret_cast<const v4i32*>(buf + offA1 + (k >> 1) * 2048);
      else
        f[k >> 1] = lo8(*reinterpret_cast<const v4i32*>(buf + offA0 + (k >> 1) * 2048));
    };
    auto rdB = [&](const uint8_t* buf, int k) {
      if (k & 1)
        fb[k >> 1].s4567 = *reinterpret_cast<const v4i32*>(buf + offB1 + (k >> 1) * 2048);
      else
        fb[k >> 1] = lo8(*reinterpret_cast<const v4i32*>(buf + offB0 + (k >> 1) * 2048));
    };

    // ---- prologue: tiles 0 and 1 in flight, wait for tile 0, its A fragments and B columns 0..3
#pragma unroll
    for (int k = 0; k < kPieces; ++k) piece(smem, 0, k);
    if (KT > 1) {
#pragma unroll
      for (int k = 0; k < kPieces; ++k) piece(smem + kBuf, 1, k);
      G48_VM(kPieces);
    } else {
      G48_VM(0);
    }
    G48_BAR();
#pragma unroll
    for (int k = 0; k < 16; ++k) rdA(smem, fa[0], k);
#pragma unroll
    for (int k = 0; k < 8; ++k) rdB(smem, k);

    // ---- one K tile (see the file head); S = the A set of tile r = r & 1 (compile time).  The K loop is
    // branch-free: the last two tiles still issue their "tile r+2" DMA, clamped to tile KT-1 (L2-resident bytes
    // written into a buffer nobody reads any more; the epilogue waits for it), and they read the idle buffer's
    // stale bytes as "tile r+1" fragments, never used.  Branches inside the loop (a flag per DMA piece, or
    // separate instantiations of the last tiles) made the register allocator rotate the accumulators through
    // VGPRs and spill at the joins.
    auto body = [&](const int r, auto s_) {
      constexpr int S = decltype(s_)::value;
      uint8_t* cur = smem + S * kBuf;        // compile-time buffer bases: every fragment read is one lane base
      uint8_t* nxt = smem + (S ^ 1) * kBuf;  // + an immediate offset
      const int kt2 = min(r + 2, KT - 1);
      // half 1: columns 0..3 || B_r[4..7]
#pragma unroll
      for (int m = 0; m < 32; ++m) {
        if ((m & 1) == 0 && m < 16) rdB(cur, 8 + (m >> 1));
        mfma8(acc[m & 7][m >> 3], fa[S][m & 7], fb[m >> 3]);
        __builtin_amdgcn_sched_barrier(0);
      }
      G48_LGKM0();
      G48_VM(0);  // tile r+1 landed (the only DMA in flight)
      G48_BAR();
      // half 2: columns 4..7 || DMA of tile r+2 into tile r's buffer, reads of A_{r+1} and B_{r+1}[0..3]
#pragma unroll
      for (int m = 0; m < 32; ++m) {
        if (m < 16)
          rdA(nxt, fa[S ^ 1], m);
        else if (m < 24)
          rdB(nxt, m - 16);
        if (m < kPieces) piece(cur, kt2, m);
        mfma8(acc[m & 7][4 + (m >> 3)], fa[S][m & 7], fb[4 + (m >> 3)]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // every pair ends with the MFMA drain: the register allocator may give the accumulators other AGPRs after
    // the loop (or in a peeled copy of it) and inserts the copies right behind the last MFMAs — opaque asm to
    // it, so without the drain those copies read blocks still being written (~1.6 % of the K loop)
    for (int r = 0; r < KT; r += 2) {
      body(r, I0{});
      body(r + 1, I1{});
      __builtin_amdgcn_sched_barrier(0);
      G48_DRAIN();
    }
    G48_VM(0);  // the last (clamped) DMA has landed before the epilogue reuses LDS
    // accumulators are read by VALU from here on.  The MFMAs are opaque inline asm, so the compiler takes their
    // results as ready at once: the drain, then an empty asm "writing" every accumulator (see gemm4w.hip)
    __builtin_amdgcn_sched_barrier(0);
    G48_DRAIN();
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
    __syncthreads();  // every wave is done with the K buffers: LDS is reused by the epilogue

    // ---- epilogue: x row scale x column scale -> bf16, per wave 128 x 128 through LDS, 16 B row stores
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem) + wid * 128 * 128;
    float cs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = n0 + wn * 128 + j * 16 + r16;
      cs[j] = col < p.N ? p.w_scale[col] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float rs[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * 128 + i * 16 + 4 * q + e;
        rs[e] = row < p.M ? p.a_scale[row] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4v t = acc[i][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = i * 16 + 4 * q + e, col = j * 16 + r16;
          ot[row * 128 + swz(row, col)] = f2bf(t[e] * rs[e] * cs[j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one row block's values live at a time
    }
    __syncthreads();
#pragma unroll 4
    for (int c = lane; c < 128 * 16; c += 64) {
      const int row = c >> 4, cch = c & 15;
      const int gm = m0 + wm * 128 + row;
      const int gn = n0 + wn * 128 + cch * 8;
      if (gm < p.M && gn < p.N)
        *reinterpret_cast<uint4v*>(p.C + (size_t)gm * p.ldc + gn) =
            *reinterpret_cast<const uint4v*>(ot + row * 128 + swz(row, cch * 8));
    }
    __syncthreads();  // LDS free for the next tile
  }
}

}  // namespace g4w8
}  // namespace lwc

// C[M, N] bf16 = (A . W^T) * a_scale[row] * w_scale[col]; A [M, lda] e4m3, W [N, K] e4m3.  K % 128 == 0,
// N % 8 == 0, lda % 16 == 0, ldc % 8 == 0, M * lda and 256 * K below 2^31 (32-bit buffer ranges).
extern "C" int lwc_gemm4w8(const void* A, const void* W, void* C, const float* a_scale, const float* w_scale, int M,
                           int N, int K, int lda, int ldc, hipStream_t s) {
  using namespace lwc::g4w8;
  if (K % 128 != 0 || K < 128 || N % 8 != 0 || lda % 16 != 0 || ldc % 8 != 0 || lda < K) return -1;
  if ((long long)M * lda >= (1LL << 31) || 256LL * K >= (1LL << 31)) return -1;
  if (M == 0 || N == 0) return 0;
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256, tiles = tiles_m * tiles_n;
  const int wpx = std::min(lwc::g4w::device_cus() / 8, (tiles + 7) / 8);
  Params p{(const uint8_t*)A, (const uint8_t*)W, (lwc::bf16_t*)C, a_scale, w_scale, M, N, K, lda, ldc,
           tiles_m, tiles_n, K / 128, std::max(1, lwc::g4w::env_int("LWC_G8_GM", 8)), wpx, tiles};
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm4w8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    attr = true;
  }
  gemm4w8_kernel<<<8 * wpx, 256, kLds, s>>>(p);
  return (int)hipGetLastError();
}
