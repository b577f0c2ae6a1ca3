// C3 tensor-parallel all-reduce over IPC-mapped peer buffers (xGMI), one-shot, hipGraph-capturable; and
// the C4 equal-split all-to-all of the expert-parallel MoE layers on the same regions and flag protocol.
//
// Why not only RCCL: a TP decode step all-reduces two [B, hidden] activations per layer.  An eager
// dist.all_reduce cannot sit inside the captured decode graph, so the TP path lost its hipGraph (every
// kernel of every layer became a host launch).  This kernel is an ordinary stream launch: the whole TP
// decode step is captured again, the all-reduce included.
//
// Memory: every rank owns one REGION (hipExtMallocWithFlags(hipDeviceMallocUncached): fine-grained,
// not cached in any L2, so bytes a peer wrote over xGMI are never served stale), exported with
// hipIpcGetMemHandle and opened by every peer (hipIpcOpenMemHandle).  Region layout:
//   [0, 32 KiB)      flags[kMaxRanks][kMaxBlocks] int32  — written by PEERS: flags[p][b] = epoch of the
//                                                          last call whose block b of rank p pushed here
//   [32 KiB, 64 KiB) epochs[kMaxBlocks] int32            — this rank's per-block call counter (local)
//   [64 KiB, ...)    data[2][W][cap] bytes                — slot (parity, p) receives rank p's payload
//
// One call, per block b (every rank launches the same grid; block b of every rank handles the same
// contiguous element range):
//   1. e = ++epochs[b]; parity = e & 1
//   2. PUSH: read this rank's range of x once, store it into data[parity][me] of every PEER region
//      (16 B vector stores over xGMI)
//   3. every storing wave drains its stores (vmcnt 0), workgroup barrier, one lane: system-scope
//      release fence, then flags[me][b] = e in every peer region (system-scope atomic store)
//   4. lanes 0..W-1 poll this rank's flags[p][b] until it is AT LEAST e (system-scope atomic loads,
//      bounded spin with s_sleep), workgroup barrier.  "At least", not "equal": a fast peer may finish
//      call e and publish call e+1's flag into this region before this rank's poller has read e — the
//      call-e data slot is still intact then (the peer's call-e+1 push goes to the other parity slot and
//      its call-e+2 push waits for this rank's call-e+1 flag).
//   5. SUM in RANK ORDER (p = 0..W-1, this rank's own term read from x) in fp32, bf16 result to out —
//      the same summation order on every rank, so all ranks hold bitwise-identical activations.
// Failure: a poller that exceeds the spin bound (a dead, hung or desynchronised peer) sets the sticky
// error word AND the block writes NaN over its whole output range instead of summing a slot that may
// hold stale data — downstream logits are poisoned, never silently wrong; the host reads the error word
// asynchronously one step later (parallel/allreduce.py) and fails the in-flight requests.
// Reuse safety: parity double-buffering.  Rank r writes slot (e&1) of call e only after its call e-1
// block b saw every peer's call-(e-1) flag, which each peer set after finishing ALL of call e-2 (stream
// order) — the last reads of that slot.  Flags are monotonic epochs: nothing is reset between calls.
#include <cstring>

#include "common.h"

namespace lwc {
namespace ar {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 1024;
constexpr size_t kFlagsOff = 0;
constexpr size_t kEpochOff = (size_t)kMaxRanks * kMaxBlocks * 4;  // 32 KiB
constexpr size_t kDataOff = 64 * 1024;
constexpr int kThreads = 512;
constexpr long long kDefaultSpinLimit = 1LL << 26;  // x s_sleep(2) (~60 ns): ~4 s, far past any healthy peer

struct Params {
  uint8_t* base[kMaxRanks];  // every rank's region as mapped in THIS process (base[me] = own)
  const bf16_t* x;           // this rank's input [n]
  bf16_t* out;               // result [n] (may alias x)
  int* err;                  // device error word (0 = ok; 1 = a peer never arrived)
  long long n;               // elements (multiple of 8)
  long long cap;             // bytes per data slot
  long long spin_limit;      // poll iterations (each ~60 ns) before a peer is declared missing
  int me, W;
};

LWC_DEVICE int* flags_of(uint8_t* region, int p, int b) {
  return reinterpret_cast<int*>(region + kFlagsOff) + p * kMaxBlocks + b;
}

__global__ void __launch_bounds__(kThreads) allreduce_kernel(Params p) {
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  const long long nvec = p.n >> 3;  // 16 B vectors
  const long long per = (nvec + nb - 1) / nb;
  const long long v0 = (long long)b * per, v1 = min(nvec, v0 + per);
  uint8_t* mine = p.base[p.me];
  int* epoch_p = reinterpret_cast<int*>(mine + kEpochOff) + b;
  const int e = __hip_atomic_load(epoch_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const int parity = e & 1;
  const uint4v* xv = reinterpret_cast<const uint4v*>(p.x);

  // 2. push this rank's range into every peer's slot (parity, me)
  for (long long v = v0 + t; v < v1; v += kThreads) {
    const uint4v val = xv[v];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) {
      if (q >= p.W) break;
      if (q == p.me) continue;
      uint4v* dst = reinterpret_cast<uint4v*>(p.base[q] + kDataOff + ((size_t)parity * p.W + p.me) * p.cap);
      dst[v] = val;
    }
  }
  // 3. publish: every wave's stores are complete before the barrier; one lane fences and signals
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    for (int q = 0; q < p.W; ++q)
      if (q != p.me) __hip_atomic_store(flags_of(p.base[q], p.me, b), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 4. wait for every peer's block b of this call (flags only grow: wait until flag >= e)
  __shared__ int missing;
  if (t == 0) missing = 0;
  __syncthreads();
  if (t < p.W && t != p.me) {
    const int* f = flags_of(mine, t, b);
    long long spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > p.spin_limit) {
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        missing = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (t == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  uint4v* ov = reinterpret_cast<uint4v*>(p.out);
  if (missing) {  // a peer never arrived: poison this block's range, never sum a possibly stale slot
    const uint32_t nan2 = 0x7FC07FC0u;  // two bf16 quiet NaNs
    for (long long v = v0 + t; v < v1; v += kThreads) ov[v] = uint4v{nan2, nan2, nan2, nan2};
    if (t == 0) __hip_atomic_store(epoch_p, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // 5. sum in rank order
  for (long long v = v0 + t; v < v1; v += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) {
      if (q >= p.W) break;
      const uint4v src = q == p.me ? xv[v]
                                   : reinterpret_cast<const uint4v*>(mine + kDataOff +
                                                                     ((size_t)parity * p.W + q) * p.cap)[v];
      float f[8];
      unpack8(src, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    ov[v] = pack8(acc);
  }
  if (t == 0) __hip_atomic_store(epoch_p, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- C4: equal-split all-to-all on the same regions and flag protocol (expert-parallel dispatch / combine)
// send = W chunks of `chunk` bytes (chunk q goes to rank q), recv = W chunks (chunk p came from rank p).
// Per block b (a contiguous range of every chunk): push send chunk q's range into slot (parity, me) of
// peer q's region, copy the own chunk locally, publish flags[me][b] = e in every peer, wait until every
// peer's flag here is at least e, then copy slot (parity, p) -> recv chunk p.  A peer that never arrives:
// sticky error word, and the block fills its recv ranges with all-ones bytes (NaN for bf16 / f32 / e4m3
// payloads, -1 for integer counts) instead of copying a possibly stale slot.
struct A2AParams {
  uint8_t* base[kMaxRanks];
  const uint8_t* send;
  uint8_t* recv;
  int* err;
  long long chunk;  // bytes per (source, destination) chunk, multiple of 16
  long long cap;    // bytes per data slot (>= chunk)
  long long spin_limit;
  int me, W;
};

__global__ void __launch_bounds__(kThreads) alltoall_kernel(A2AParams p) {
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  const long long nvec = p.chunk >> 4;
  const long long per = (nvec + nb - 1) / nb;
  const long long v0 = (long long)b * per, v1 = min(nvec, v0 + per);
  uint8_t* mine = p.base[p.me];
  int* epoch_p = reinterpret_cast<int*>(mine + kEpochOff) + b;
  const int e = __hip_atomic_load(epoch_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const int parity = e & 1;
  const uint4v* sv = reinterpret_cast<const uint4v*>(p.send);
  uint4v* rv = reinterpret_cast<uint4v*>(p.recv);
  for (long long v = v0 + t; v < v1; v += kThreads) {
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) {
      if (q >= p.W) break;
      const uint4v val = sv[(long long)q * nvec + v];
      if (q == p.me) {
        rv[(long long)q * nvec + v] = val;
      } else {
        uint4v* dst = reinterpret_cast<uint4v*>(p.base[q] + kDataOff + ((size_t)parity * p.W + p.me) * p.cap);
        dst[v] = val;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    for (int q = 0; q < p.W; ++q)
      if (q != p.me) __hip_atomic_store(flags_of(p.base[q], p.me, b), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __shared__ int missing;
  if (t == 0) missing = 0;
  __syncthreads();
  if (t < p.W && t != p.me) {
    const int* f = flags_of(mine, t, b);
    long long spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > p.spin_limit) {
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        missing = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (t == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  const uint32_t ones = 0xFFFFFFFFu;
  for (long long v = v0 + t; v < v1; v += kThreads) {
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) {
      if (q >= p.W) break;
      if (q == p.me) continue;
      rv[(long long)q * nvec + v] =
          missing ? uint4v{ones, ones, ones, ones}
                  : reinterpret_cast<const uint4v*>(mine + kDataOff + ((size_t)parity * p.W + q) * p.cap)[v];
    }
  }
  if (t == 0) __hip_atomic_store(epoch_p, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ar
}  // namespace lwc

// recv[p] = rank p's send chunk for this rank (W chunks of `chunk` bytes each, chunk % 16 == 0, chunk <= cap).
extern "C" int lwc_alltoall(void* const* bases, int me, int W, const void* send, void* recv, long long chunk,
                            long long cap, int* err, int blocks, long long spin_limit, hipStream_t s) {
  using namespace lwc::ar;
  if (W < 1 || W > kMaxRanks || me < 0 || me >= W || chunk % 16 != 0 || chunk > cap) return -1;
  if (blocks < 1 || blocks > kMaxBlocks) return -2;
  if (chunk == 0) return 0;
  A2AParams p{};
  for (int i = 0; i < W; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.send = static_cast<const uint8_t*>(send);
  p.recv = static_cast<uint8_t*>(recv);
  p.err = err;
  p.chunk = chunk;
  p.cap = cap;
  p.spin_limit = spin_limit > 0 ? spin_limit : kDefaultSpinLimit;
  p.me = me;
  p.W = W;
  alltoall_kernel<<<blocks, kThreads, 0, s>>>(p);
  return (int)hipGetLastError();
}

// Bytes of a region for W ranks and `cap` bytes per slot.
extern "C" long long lwc_ar_region_bytes(int W, long long cap) {
  return (long long)lwc::ar::kDataOff + 2LL * W * cap;
}

// Allocate + zero this rank's region; returns its IPC handle (64 bytes) in `handle`.
extern "C" int lwc_ar_alloc(long long bytes, void** ptr, void* handle) {
  hipError_t rc = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (rc != hipSuccess) return (int)rc;
  rc = hipMemset(*ptr, 0, (size_t)bytes);
  if (rc != hipSuccess) return (int)rc;
  rc = hipDeviceSynchronize();
  if (rc != hipSuccess) return (int)rc;
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), *ptr);
}

extern "C" int lwc_ar_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int lwc_ar_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }
extern "C" int lwc_ar_free(void* ptr) { return (int)hipFree(ptr); }
extern "C" int lwc_ar_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// out = sum over ranks of x (bf16 [n], n % 8 == 0, 2n <= cap); `bases` = W region pointers as mapped here.
// spin_limit <= 0: the default bound (~4 s).
extern "C" int lwc_allreduce(void* const* bases, int me, int W, const void* x, void* out, long long n, long long cap,
                             int* err, int blocks, long long spin_limit, hipStream_t s) {
  using namespace lwc::ar;
  if (W < 1 || W > kMaxRanks || me < 0 || me >= W || n % 8 != 0 || 2 * n > cap) return -1;
  if (blocks < 1 || blocks > kMaxBlocks) return -2;
  if (n == 0) return 0;
  Params p{};
  for (int i = 0; i < W; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.x = static_cast<const lwc::bf16_t*>(x);
  p.out = static_cast<lwc::bf16_t*>(out);
  p.err = err;
  p.n = n;
  p.cap = cap;
  p.spin_limit = spin_limit > 0 ? spin_limit : kDefaultSpinLimit;
  p.me = me;
  p.W = W;
  allreduce_kernel<<<blocks, kThreads, 0, s>>>(p);
  return (int)hipGetLastError();
}
