// One-shot IPC all-reduce over xGMI for latency-bound tensor-parallel messages
// (SURVEY §5.8 COMM-2; the reference has no collectives at all).
//
// Every rank owns ONE uncached device allocation (hipExtMallocWithFlags
// hipDeviceMallocUncached) that all peers map through hipIpc handles:
//
//   [ control (32 KiB): flag[2][128 blocks][8 ranks] u32 | flag2 (same) | epoch u32 | done u32 | err u32 ]
//   [ data parity 0 (cap bytes) ][ data parity 1 (cap bytes) ][ reduced parity 0 ][ reduced parity 1 ]
//
// Call e (e = epoch + 1, parity p = e & 1, the same for every block of the call):
//   1. block b copies its slice of the input into its OWN data[p];
//   2. system-scope release: flag[p][b][rank] = e stored into EVERY peer's control
//      block (each xGMI link carries one 4-byte write);
//   3. waits until all peers' flag[p][b][*] >= e in its own (local) control block;
//   4. reads the same slice of every peer's data[p] (7 links in parallel), sums in
//      fp32 in fixed rank order (bitwise identical on every rank), writes `out`.
// Double-buffering by parity makes an end barrier unnecessary: rank r can only
// rewrite data[p] at call e+2 after every peer passed call e+1's barrier, i.e.
// finished reading call e (kernels of one stream are ordered, so once ANY block of rank r's call
// e + 1 saw a peer's e + 1 flag, that peer's whole call-e kernel is done).  This needs every block
// of a call to use the same parity whatever partition the call uses (one-shot and two-shot slice
// the buffer differently, and the block count follows the message size): the epoch is ONE device
// counter per rank, advanced by the last block of each call to finish (per-block epochs
// diverged when consecutive calls used different block counts, so a block could reuse the parity
// a peer was still reading).  It lives in device memory, so the kernel takes no per-call arguments
// and a captured hipGraph replays it correctly.  Every spin has a bounded budget: a missing peer
// sets `err` and the kernel drains instead of hanging the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm.h"

namespace lumen {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void add_vec(float* acc, const u32x4v v, int is_bf16) {
  if (is_bf16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += __uint_as_float(v[i] << 16);
      acc[2 * i + 1] += __uint_as_float(v[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += __uint_as_float(v[i]);
  }
}

__device__ __forceinline__ uint32_t rne_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// The last block of a call to finish advances the rank's epoch (the next call is the next kernel on
// the stream: every one of its blocks reads the new value).
__device__ __forceinline__ void end_call(ArCtl* ctl, uint32_t e) {
  const uint32_t d = __hip_atomic_fetch_add(&ctl->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (d + 1u == gridDim.x) {
    __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctl->epoch, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// BF16 = 1: bf16 elements (8 per 16-byte vector); 0: fp32 (4 per vector).
template <int BF16>
__global__ void __launch_bounds__(512) custom_ar_kernel(const u32x4v* __restrict__ in, u32x4v* __restrict__ out,
                                                        ArPeers peers, int rank, int world, int64_t nvec,
                                                        int64_t vec_per_block, int64_t cap_bytes) {
  const int b = blockIdx.x;
  char* mine = peers.base[rank];
  ArCtl* ctl = reinterpret_cast<ArCtl*>(mine);
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int p = (int)(e & 1u);
  const int64_t lo = (int64_t)b * vec_per_block;
  const int64_t hi = lo + vec_per_block < nvec ? lo + vec_per_block : nvec;

  // 1. stage my slice into my own data[p]
  u32x4v* my_data = reinterpret_cast<u32x4v*>(mine + AR_CTL_BYTES + (int64_t)p * cap_bytes);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my_data[i] = in[i];
  __threadfence_system();
  __syncthreads();

  // 2. signal every peer (including myself), 3. wait for every peer
  if (threadIdx.x < (unsigned)world) {
    ArCtl* pc = reinterpret_cast<ArCtl*>(peers.base[threadIdx.x]);
    __hip_atomic_store(&pc->flag[p][b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = &ctl->flag[p][b][threadIdx.x];
    int spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > AR_SPIN_LIMIT) {
        __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 4. reduce the slice over all ranks in rank order
  const int64_t off = AR_CTL_BYTES + (int64_t)p * cap_bytes;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      const u32x4v v = reinterpret_cast<const u32x4v*>(peers.base[r] + off)[i];
      add_vec(acc, v, BF16);
    }
    u32x4v o;
    if (BF16) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rne_bf16(acc[2 * k]) | (rne_bf16(acc[2 * k + 1]) << 16);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(acc[k]);
    }
    out[i] = o;
  }
  __syncthreads();
  if (threadIdx.x == 0) end_call(ctl, e);
}

// Two-shot form for bandwidth-bound messages (a TP prefill all-reduce: 624 x 4096 bf16 = 5 MB per
// layer at Llama-3-8B), same buffers and epochs.  Block b owns vectors [lo, hi) on every rank and
// splits them into `world` sub-slices:
//   1. copy [lo, hi) of the input into my data[p]; signal flag[p][b] to every peer; wait for all;
//   2. reduce MY sub-slice over all ranks' data[p] (fp32, rank order) -> out and my red[p];
//   3. signal flag2[p][b] to every peer; wait for all;
//   4. copy every peer's reduced sub-slice from its red[p] into out.
// Each rank moves 2 (n-1)/n of the message over its links instead of (n-1) x (one-shot), so at
// n = 8 and MB-sized messages the links carry 4x less.  Reuse by parity is safe as in the one-shot
// form: a rank rewrites data[p] / red[p] at call e + 2 only after every peer signalled call
// e + 1 (or e + 2), i.e. finished reading call e.
template <int BF16>
__global__ void __launch_bounds__(512) custom_ar2_kernel(const u32x4v* __restrict__ in, u32x4v* __restrict__ out,
                                                         ArPeers peers, int rank, int world, int64_t nvec,
                                                         int64_t vec_per_block, int64_t cap_bytes) {
  const int b = blockIdx.x;
  char* mine = peers.base[rank];
  ArCtl* ctl = reinterpret_cast<ArCtl*>(mine);
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int p = (int)(e & 1u);
  const int64_t lo = (int64_t)b * vec_per_block;
  const int64_t hi = lo + vec_per_block < nvec ? lo + vec_per_block : nvec;
  const int64_t sub = (hi - lo + world - 1) / world;
  const int64_t doff = AR_CTL_BYTES + (int64_t)p * cap_bytes;         // data[p]
  const int64_t roff = AR_CTL_BYTES + (int64_t)(2 + p) * cap_bytes;   // red[p]

  // 1. stage [lo, hi) into my data[p], barrier 1
  u32x4v* my_data = reinterpret_cast<u32x4v*>(mine + doff);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my_data[i] = in[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < (unsigned)world) {
    ArCtl* pc = reinterpret_cast<ArCtl*>(peers.base[threadIdx.x]);
    __hip_atomic_store(&pc->flag[p][b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = &ctl->flag[p][b][threadIdx.x];
    int spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > AR_SPIN_LIMIT) {
        __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 2. reduce my sub-slice -> out, my red[p]
  u32x4v* my_red = reinterpret_cast<u32x4v*>(mine + roff);
  const int64_t s0 = lo + rank * sub, s1 = s0 + sub < hi ? s0 + sub : hi;
  for (int64_t i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) add_vec(acc, reinterpret_cast<const u32x4v*>(peers.base[r] + doff)[i], BF16);
    u32x4v o;
    if (BF16) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rne_bf16(acc[2 * k]) | (rne_bf16(acc[2 * k + 1]) << 16);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(acc[k]);
    }
    my_red[i] = o;
    out[i] = o;
  }
  __threadfence_system();
  __syncthreads();

  // 3. barrier 2: every rank's reduced sub-slice published
  if (threadIdx.x < (unsigned)world) {
    ArCtl* pc = reinterpret_cast<ArCtl*>(peers.base[threadIdx.x]);
    __hip_atomic_store(&pc->flag2[p][b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = &ctl->flag2[p][b][threadIdx.x];
    int spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > AR_SPIN_LIMIT) {
        __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 4. gather the peers' reduced sub-slices
  for (int r = 1; r < world; ++r) {
    const int q = (rank + r) % world;            // start at a different peer on every rank
    const int64_t q0 = lo + q * sub, q1 = q0 + sub < hi ? q0 + sub : hi;
    const u32x4v* src = reinterpret_cast<const u32x4v*>(peers.base[q] + roff);
    for (int64_t i = q0 + threadIdx.x; i < q1; i += blockDim.x) out[i] = src[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) end_call(ctl, e);
}

hipError_t custom_all_reduce_2shot(const void* in, void* out, const ArPeers& peers, int rank, int world,
                                   int64_t bytes, int is_bf16, int64_t cap_bytes, hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world) return hipErrorInvalidValue;
  if (bytes % 16 != 0 || bytes > cap_bytes) return hipErrorInvalidValue;
  const int64_t nvec = bytes / 16;
  if (nvec == 0) return hipSuccess;
  // >= 2 vectors per thread per sub-slice at n = 8: up to 128 workgroups keep more remote reads in
  // flight over the 7 links (a 5 MB prefill message: 128 x 40 KB)
  int64_t blocks = (nvec + 1023) / 1024;
  if (blocks > AR_MAX_BLOCKS) blocks = AR_MAX_BLOCKS;
  const int64_t per = (nvec + blocks - 1) / blocks;
  blocks = (nvec + per - 1) / per;
  if (is_bf16)
    hipLaunchKernelGGL(custom_ar2_kernel<1>, dim3((unsigned)blocks), dim3(512), 0, stream, (const u32x4v*)in,
                       (u32x4v*)out, peers, rank, world, nvec, per, cap_bytes);
  else
    hipLaunchKernelGGL(custom_ar2_kernel<0>, dim3((unsigned)blocks), dim3(512), 0, stream, (const u32x4v*)in,
                       (u32x4v*)out, peers, rank, world, nvec, per, cap_bytes);
  return hipGetLastError();
}

hipError_t custom_all_reduce(const void* in, void* out, const ArPeers& peers, int rank, int world, int64_t bytes,
                             int is_bf16, int64_t cap_bytes, hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world) return hipErrorInvalidValue;
  if (bytes % 16 != 0 || bytes > cap_bytes) return hipErrorInvalidValue;
  const int64_t nvec = bytes / 16;
  if (nvec == 0) return hipSuccess;
  int64_t blocks = (nvec + 511) / 512;
  if (blocks > AR_MAX_BLOCKS) blocks = AR_MAX_BLOCKS;
  const int64_t per = (nvec + blocks - 1) / blocks;
  blocks = (nvec + per - 1) / per;
  if (is_bf16)
    hipLaunchKernelGGL(custom_ar_kernel<1>, dim3((unsigned)blocks), dim3(512), 0, stream, (const u32x4v*)in,
                       (u32x4v*)out, peers, rank, world, nvec, per, cap_bytes);
  else
    hipLaunchKernelGGL(custom_ar_kernel<0>, dim3((unsigned)blocks), dim3(512), 0, stream, (const u32x4v*)in,
                       (u32x4v*)out, peers, rank, world, nvec, per, cap_bytes);
  return hipGetLastError();
}

}  // namespace lumen
