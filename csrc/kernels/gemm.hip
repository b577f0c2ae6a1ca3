// K6g grouped GEMM on MFMA: C[rows, N] = A[rows, K] . W_g[N, K]^T for row groups g (MoE experts),
// with the group table on the DEVICE so a launch needs no host sync (graph-capturable), plus the
// fp8 (OCP e4m3) variant with per-row activation and per-channel weight scales (config 5).
//
//   groups : row_off[G+1] (device, int32): group g owns rows [row_off[g], row_off[g+1]) of A and C and
//            multiplies them by W + g * w_group_stride.  A plain GEMM is G = 1, row_off = {0, M}.
//            Optional a_rows[r] gathers A's row per output row (MoE dispatch without a permute copy).
//   grid   : x = m-tile SLOT (>= sum_g ceil(M_g / BM); surplus slots exit), y = n-tile.
//   tile   : BM x BN = 128 x 128, BK = 64; 4 waves as 2 x 2, each 64 x 64 = 4 x 4 MFMA 16x16 tiles.
//   K loop : register-staged, one LDS stage (next K-tile's global loads in flight under the current
//            tile's MFMAs, written to LDS after a barrier; 4 workgroups per CU hide each other's stalls),
//            16-byte chunks XOR-swizzled by row (conflict-free ds_read_b128 fragment reads).
//   MFMA   : bf16: mfma_f32_16x16x32_bf16 (lane: row r16, k-chunk g); fp8: the block-scaled
//            mfma_scale_f32_16x16x128_f8f6f4 with unit scales (32 e4m3 per lane, whole 128 B k-slice).
// Both operands are K-contiguous (torch.nn.functional.linear layout), so A and W tiles share one
// staging / fragment code path.
#include "common.h"

namespace lwc {

typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef int v8i32 __attribute__((ext_vector_type(8)));

constexpr int kGM = 128, kGN = 128;
constexpr int kGKBytes = 128;          // bytes of K per tile row (64 bf16 or 128 fp8)
constexpr int kGChunks = kGKBytes / 16;  // 16 B chunks per tile row
constexpr int kGTileBytes = kGM * kGKBytes;  // 16 KiB per operand tile

struct GemmParams {
  const uint8_t* A;     // [rows, K] (bf16 or fp8), row stride lda elements
  const uint8_t* W;     // [G][N, K]
  bf16_t* C;            // [rows, N], row stride ldc
  const int* row_off;   // [G + 1]
  const float* a_scale; // fp8: [rows] per-row activation scales
  const float* w_scale; // fp8: [G][N] per-channel weight scales
  const bf16_t* bias;   // optional [G][N]
  const int* a_rows;    // optional [rows]: A row of output row r is a_rows[r] (MoE dispatch gather)
  int G, N, K, lda, ldc;
  long long w_group_stride;  // elements
  float* C32;           // split-K (splits > 1): fp32 [rows, N] accumulation buffer (zeroed), C unused
  int splits;           // K split into `splits` ranges (grid z); partials added with fp32 atomics
  int slots;            // m-tile slots per n-tile (grid mapping below)
  int n_tiles;
  int xcd_group;        // 1: 1-D grid, the m-slots of one n-tile on ONE XCD back to back (see below)
};

LWC_DEVICE float4v mfma_bf16(const short8& a, const short8& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(gbf16x8, a), __builtin_bit_cast(gbf16x8, b), c, 0,
                                                 0, 0);
}

template <bool FP8>
__global__ void __launch_bounds__(256, 3) grouped_gemm_kernel(GemmParams p) {
  constexpr int ES = FP8 ? 1 : 2;  // element size
  // ONE LDS stage (32 KiB): the next K tile waits in registers.  Four workgroups fit a CU (LDS 4 x 32 KiB,
  // 128 VGPRs = 4 waves per SIMD), so while one workgroup stalls on its loads the others compute — the
  // small-M MoE decode launches are latency-bound, and occupancy buys more than a second LDS buffer.
  __shared__ __attribute__((aligned(16))) uint8_t smem[1][2][kGTileBytes];  // [stage][A|W]

  // ---- grid mapping ----
  // xcd_group = 0: x = m-slot, y = n-tile.  xcd_group = 1 (experts with several m-tiles, e.g. a large
  // MoE decode batch): workgroup ids are dealt round-robin to the 8 XCDs, so id = local * 8 + xcd, and
  // each XCD walks ITS n-tiles (j = xcd mod 8) with all m-slots of an n-tile consecutive: every m-tile
  // of an expert reuses the same weight tile from that XCD's L2 instead of streaming it again from HBM.
  int slot, ntile;
  if (p.xcd_group) {
    const int id = blockIdx.x, xcd = id & 7, local = id >> 3;
    ntile = (local / p.slots) * 8 + xcd;
    slot = local % p.slots;
    if (ntile >= p.n_tiles) return;  // uniform
  } else {
    slot = blockIdx.x;
    ntile = blockIdx.y;
  }
  // ---- locate (group, m-tile) of this slot ----
  int g = 0, m_begin = 0, m_end = 0;
  for (; g < p.G; ++g) {
    const int r0 = p.row_off[g], r1 = p.row_off[g + 1];
    const int nt = (r1 - r0 + kGM - 1) / kGM;
    if (slot < nt) {
      m_begin = r0 + slot * kGM;
      m_end = r1;
      break;
    }
    slot -= nt;
  }
  if (g >= p.G) return;  // surplus slot (uniform for the workgroup)
  const int n0 = ntile * kGN;
  const uint8_t* W = p.W + (size_t)g * p.w_group_stride * ES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wm = wid >> 1, wn = wid & 1;

  const int KT_all = p.K * ES / kGKBytes;  // K tiles (K * ES is a multiple of 128 B)
  // split-K: this workgroup's K-tile range
  const int kper = (KT_all + p.splits - 1) / p.splits;
  const int kt0 = blockIdx.z * kper, KT = min(KT_all, kt0 + kper) - kt0;
  if (KT <= 0) return;  // uniform
  // staging: 1024 chunks per operand tile, 4 per thread.  The A row pointers (MoE gather through
  // a_rows) are resolved ONCE: a per-iteration index load would put a dependent memory round trip in
  // front of every K tile's A loads.
  const uint8_t* arow[4];
  const uint8_t* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 3, ch = c & 7;
    const int ar = m_begin + row;
    arow[i] = ar < m_end ? p.A + (size_t)(p.a_rows ? p.a_rows[ar] : ar) * p.lda * ES + ch * 16 : nullptr;
    const int wr = n0 + row;
    wrow[i] = wr < p.N ? W + (size_t)wr * p.K * ES + ch * 16 : nullptr;
  }
  uint4v sa[4], sw[4];
  auto gload = [&](int kt) {
    const size_t kb = (size_t)(kt0 + kt) * kGKBytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sa[i] = arow[i] ? *reinterpret_cast<const uint4v*>(arow[i] + kb) : uint4v{0, 0, 0, 0};
      sw[i] = wrow[i] ? *reinterpret_cast<const uint4v*>(wrow[i] + kb) : uint4v{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int row = c >> 3, ch = c & 7;
      const int off = row * kGKBytes + ((ch ^ (row & 7)) << 4);
      *reinterpret_cast<uint4v*>(&smem[buf][0][off]) = sa[i];
      *reinterpret_cast<uint4v*>(&smem[buf][1][off]) = sw[i];
    }
  };

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  gload(0);
  for (int kt = 0; kt < KT; ++kt) {
    __syncthreads();  // everyone is done reading the previous tile
    lstore(0);
    __syncthreads();
    if (kt + 1 < KT) gload(kt + 1);  // in flight under this tile's MFMAs
    const uint8_t* As = smem[0][0];
    const uint8_t* Ws = smem[0][1];
    if constexpr (FP8) {
      // one block-scaled MFMA 16x16x128 (e4m3 x e4m3, unit e8m0 scales: the per-row / per-channel
      // scales stay in the epilogue) per 16x16 tile covers the whole 128-byte k-slice: twice the fp8
      // rate of four 16x16x32 MFMAs.  Lane group q holds the row's 16 B chunks q and 4+q for A and W
      // alike, so both operands see the same k permutation and the dot product is unchanged.
      uint4v b0[4], b1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rb = wn * 64 + j * 16 + r16;
        b0[j] = *reinterpret_cast<const uint4v*>(Ws + rb * kGKBytes + ((q ^ (rb & 7)) << 4));
        b1[j] = *reinterpret_cast<const uint4v*>(Ws + rb * kGKBytes + (((4 + q) ^ (rb & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra = wm * 64 + i * 16 + r16;
        const uint4v a0 = *reinterpret_cast<const uint4v*>(As + ra * kGKBytes + ((q ^ (ra & 7)) << 4));
        const uint4v a1 = *reinterpret_cast<const uint4v*>(As + ra * kGKBytes + (((4 + q) ^ (ra & 7)) << 4));
        const v8i32 av = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const v8i32 bv = {(int)b0[j].x, (int)b0[j].y, (int)b0[j].z, (int)b0[j].w,
                            (int)b1[j].x, (int)b1[j].y, (int)b1[j].z, (int)b1[j].w};
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc[i][j], 0, 0, 0, 127, 0, 127);
        }
      }
    } else {
      // two 16 B-chunk halves of the 128 B k-slice: 2 k-steps of 32 bf16 each
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + q;
        uint4v af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ra = wm * 64 + i * 16 + r16;
          af[i] = *reinterpret_cast<const uint4v*>(As + ra * kGKBytes + ((ch ^ (ra & 7)) << 4));
          const int rb = wn * 64 + i * 16 + r16;
          bfr[i] = *reinterpret_cast<const uint4v*>(Ws + rb * kGKBytes + ((ch ^ (rb & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma_bf16(__builtin_bit_cast(short8, af[i]), __builtin_bit_cast(short8, bfr[j]), acc[i][j]);
      }
    }
  }

  // ---- epilogue: scales, bias, bf16 store (lane reg r = C[row 4q + r][col r16] of each 16x16) ----
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + r16;
    if (col >= p.N) continue;
    const float ws = FP8 ? p.w_scale[(size_t)g * p.N + col] : 1.f;
    const float bv = p.bias && blockIdx.z == 0 ? bf2f(p.bias[(size_t)g * p.N + col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m_begin + wm * 64 + i * 16 + 4 * q + r;
        if (row < m_end) {
          const float as = FP8 ? p.a_scale[p.a_rows ? p.a_rows[row] : row] : 1.f;
          const float v = acc[i][j][r] * as * ws + bv;
          if (p.splits > 1)
            atomicAdd(p.C32 + (size_t)row * p.N + col, v);
          else
            p.C[(size_t)row * p.ldc + col] = f2bf(v);
        }
      }
  }
}

// split-K finalize: fp32 accumulation buffer -> bf16 C
__global__ void __launch_bounds__(256) f32_to_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                          long long n, int N, int ldc) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i * 4 >= n) return;
  const long long e = i * 4;  // N % 16 == 0: a 4-group never crosses a row
  const float4 v = *reinterpret_cast<const float4*>(src + e);
  bf16_t* o = dst + (e / N) * ldc + e % N;
  o[0] = f2bf(v.x);
  o[1] = f2bf(v.y);
  o[2] = f2bf(v.z);
  o[3] = f2bf(v.w);
}

}  // namespace lwc

// max_slots: grid x; must be >= sum_g ceil(M_g / 128) (sum_g <= ceil(M_total / 128) + G works for any split).
// splits > 1: split-K over grid z; `c32` = zeroed fp32 [rows, N] workspace (rows = max row index + 1),
// finalised into C (bf16) by a second kernel.
extern "C" int lwc_grouped_gemm(const void* A, const void* W, void* C, const int* row_off, const float* a_scale,
                                const float* w_scale, const void* bias, const int* a_rows, int G, int max_slots, int N,
                                int K, int lda, int ldc, long long w_group_stride, int fp8, float* c32, int splits,
                                long long rows, hipStream_t s) {
  using namespace lwc;
  const int es = fp8 ? 1 : 2;
  if ((K * es) % kGKBytes != 0 || N % 16 != 0 || G < 1 || splits < 1) return -1;
  if (fp8 && (!a_scale || !w_scale)) return -2;
  if (splits > 1 && !c32) return -3;
  if (max_slots == 0) return 0;
  const int n_tiles = (N + kGN - 1) / kGN;
  // several m-tiles per group on average (rows >= 2 * 128 * G): group each n-tile's m-slots on one XCD
  const int xcd_group = rows >= 2LL * kGM * G ? 1 : 0;
  GemmParams p{(const uint8_t*)A, (const uint8_t*)W, (bf16_t*)C, row_off, a_scale, w_scale, (const bf16_t*)bias,
               a_rows, G, N, K, lda, ldc, w_group_stride, c32, splits, max_slots, n_tiles, xcd_group};
  const dim3 grid = xcd_group ? dim3((unsigned)(((n_tiles + 7) / 8) * max_slots * 8), 1, splits)
                              : dim3(max_slots, n_tiles, splits);
  if (fp8)
    grouped_gemm_kernel<true><<<grid, 256, 0, s>>>(p);
  else
    grouped_gemm_kernel<false><<<grid, 256, 0, s>>>(p);
  if (splits > 1 && rows > 0) {
    const long long n = rows * N;
    f32_to_bf16_kernel<<<(unsigned)((n / 4 + 255) / 256), 256, 0, s>>>(c32, (bf16_t*)C, n, N, ldc);
  }
  return (int)hipGetLastError();
}
