// Per-CU LDS-DMA intake probe: how many bytes per second can one CU pull into LDS with
// global_load_lds (16 B per lane), as a function of waves per workgroup, loads in flight per
// wave and the source footprint (L2-resident / Infinity-Cache-resident / HBM)?  No compute.
//   hipcc --offload-arch=gfx950 -O3 -o glds_intake glds_intake.hip && ./glds_intake
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* g_ptr_t;

template <int DEPTH>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory"); }

// each wave streams `iters` 1-KiB pieces from its own walk over src (wrapping at `mask`+1 bytes)
// into a private 16-slot LDS ring, keeping DEPTH pieces in flight
template <int DEPTH>
__global__ void intake(const char* __restrict__ src, size_t mask, int iters, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  char* ring = smem + wid * 16 * 1024;
  size_t off = ((size_t)blockIdx.x * 977 + wid * 131) * 1024;
  for (int i = 0; i < iters; ++i) {
    const char* p = src + ((off + (size_t)i * 1024 * 8) & mask) + lane * 16;   // stride 8 KiB: spread channels
    __builtin_amdgcn_global_load_lds((g_ptr_t)p, (lds_ptr_t)(ring + (i & 15) * 1024), 16, 0, 0);
    if (i >= DEPTH) vm_wait<DEPTH>();
  }
  vm_wait<0>();
  if (lane == 0 && ring[wid] == 123) sink[blockIdx.x] = 1;
}

// same through registers (global_load_dwordx4, DEPTH loads in flight, summed so nothing is dead)
template <int DEPTH>
__global__ void intake_reg(const char* __restrict__ src, size_t mask, int iters, unsigned* sink) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  size_t off = ((size_t)blockIdx.x * 977 + wid * 131) * 1024;
  uint4 acc = {0, 0, 0, 0};
  for (int i = 0; i < iters; i += DEPTH) {
    uint4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
      v[d] = *(const uint4*)(src + ((off + (size_t)(i + d) * 1024 * 8) & mask) + lane * 16);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) { acc.x ^= v[d].x; acc.y ^= v[d].y; acc.z ^= v[d].z; acc.w ^= v[d].w; }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[blockIdx.x] = 1;
}

template <typename K>
float run(K kern, int grid, int waves, size_t lds, const char* src, size_t bytes, int iters, unsigned* sink) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, 0, src, bytes - 1, iters, sink);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, 0, src, bytes - 1, iters, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 5;
}

int main() {
  const size_t big = (size_t)4 << 30;
  char* src;
  unsigned* sink;
  CHECK(hipMalloc(&src, big));
  CHECK(hipMemset(src, 1, big));
  CHECK(hipMalloc(&sink, 4096 * 4));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int iters = 4096;
  const size_t foots[] = {(size_t)2 << 20, (size_t)64 << 20, (size_t)4 << 30};
  const char* fname[] = {"L2(2MiB)", "MALL(64MiB)", "HBM(4GiB)"};
  for (int fi = 0; fi < 3; ++fi) {
    for (int waves : {1, 2, 4, 8}) {
      const size_t lds = (size_t)waves * 16 * 1024 > 65536 ? (size_t)waves * 16 * 1024 : 65536 + 1024;  // 1 WG per CU
      for (int depth : {2, 4, 8, 12}) {
        float ms;
        auto kern = depth == 2 ? intake<2> : depth == 4 ? intake<4> : depth == 8 ? intake<8> : intake<12>;
        ms = run(kern, cus, waves, lds, src, foots[fi], iters, sink);
        const double bytes = (double)cus * waves * iters * 1024;
        printf("{\"kind\":\"glds\",\"src\":\"%s\",\"waves\":%d,\"depth\":%d,\"us\":%.1f,\"GBps_per_CU\":%.1f,\"TBps\":%.2f}\n",
               fname[fi], waves, depth, ms * 1e3, bytes / cus / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e12);
      }
      for (int depth : {4, 8}) {
        auto kern = depth == 4 ? intake_reg<4> : intake_reg<8>;
        float ms = run(kern, cus, waves, 0, src, foots[fi], iters, sink);
        const double bytes = (double)cus * waves * iters * 1024;
        printf("{\"kind\":\"reg\",\"src\":\"%s\",\"waves\":%d,\"depth\":%d,\"us\":%.1f,\"GBps_per_CU\":%.1f,\"TBps\":%.2f}\n",
               fname[fi], waves, depth, ms * 1e3, bytes / cus / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
