// calib_fetch.hip — DIAGNOSTIC (not the product): known-byte kernels in k_run's own access
// widths, so that rocprofv3's FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md §HBM: calibrated
// there only for 16-B-per-lane streaming reads and stores) can be turned into bytes for each
// pattern k_run issues.  Every buffer is 1 GiB or more (past the 256 MiB Infinity Cache), and
// every kernel requests a known number of bytes, printed with its name; run it under
//   rocprofv3 --pmc FETCH_SIZE -- ./calib_fetch     and     rocprofv3 --pmc WRITE_SIZE -- ...
// and divide.  The patterns (tg_amd.hip):
//   dword      the twist's loads / stores: lane p reads word p of a 624-word generation, 64
//              lanes = 256 contiguous bytes per instruction (twist_load / twist_store)
//   x4         16 B per lane, contiguous across the wave (k_classify / the worklist records)
//   dma16_env  global_load_lds_dwordx4, each lane 16 B of a DIFFERENT env (stride 624 B: the
//              code window fill, RngCodes::fill)
//   x4_env     16-B loads / stores, each lane a different env (stride 16 B within a random
//              permutation: k_run's scattered st4 / ang stores of its listed envs)
//   x2_env     8-B loads / stores, each lane a different env (ep, a draw's two MT words)
//   code4      4-B stores, one per lane, contiguous (the twist's draw codes)
//   gen_stores k_regen's store stream without its compute: per job (a random env's half of
//              8 generations) 8 x 624 dword stores (256 B per instruction, generations 2,496 B
//              apart: every other one not 128-B aligned) and 8 x 312 code bytes (64 B per
//              instruction); gen_stores_aligned the same with generations 2,560 B apart.  Their
//              rocprofv3 durations are the store-bound ceiling of k_regen's pattern.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int BLOCK = 256;

__global__ void k_dword(const uint32_t* __restrict__ src, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK)
    acc ^= src[i];
  if (acc == 0x12345678u) sink[0] = acc;  // never true in practice; keeps the loads
}
__global__ void k_dword_store(uint32_t* __restrict__ dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK)
    dst[i] = (uint32_t)i;
}
__global__ void k_x4(const uint4* __restrict__ src, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// one 16-B chunk per lane from env perm[i] (env stride `stride` bytes), by LDS-DMA
__global__ void k_dma16_env(const uint8_t* __restrict__ base, const uint32_t* __restrict__ perm,
                            uint64_t n, uint32_t stride, uint32_t* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t win[BLOCK * 16];
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(win + (threadIdx.x & ~63u) * 16));
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const uint8_t* g = base + (uint64_t)perm[i] * stride + 16u * (uint32_t)(i % 13);
    uint32_t save;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(save)
        : "s"(m0), "v"(g)
        : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (win[threadIdx.x * 16] == 0xAB && win[threadIdx.x * 16 + 1] == 0xCD) sink[1] = 1;
}
template <class T>
__global__ void k_env_load(const uint8_t* __restrict__ base, const uint32_t* __restrict__ perm,
                           uint64_t n, uint32_t stride, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const T v = *reinterpret_cast<const T*>(base + (uint64_t)perm[i] * stride);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) acc ^= w[k];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
template <class T>
__global__ void k_env_store(uint8_t* __restrict__ base, const uint32_t* __restrict__ perm,
                            uint64_t n, uint32_t stride) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    T v;
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
    for (unsigned k = 0; k < sizeof(T) / 4; ++k) w[k] = (uint32_t)i + k;
    *reinterpret_cast<T*>(base + (uint64_t)perm[i] * stride) = v;
  }
}

// k_regen's stores alone (see the header): GSTRIDE words between generations
template <int GSTRIDE>
__global__ void k_gen_stores(uint32_t* __restrict__ mt, uint8_t* __restrict__ mc,
                             const uint32_t* __restrict__ jobs, int njobs) {
  const int lane = threadIdx.x & 63;
  const int w = (int)((blockIdx.x * (uint64_t)BLOCK + threadIdx.x) >> 6);
  const int nw = (int)(gridDim.x * (BLOCK / 64));
  for (int j = w; j < njobs; j += nw) {
    const uint32_t e = jobs[j];
    const uint64_t env = e & 0x7FFFFFFFu, half = e >> 31;
    uint32_t* const dst = mt + env * (16 * GSTRIDE) + half * (8 * GSTRIDE);
    uint8_t* const dc = mc + env * 4992 + half * 2496;
    for (int g = 0; g < 8; ++g) {
#pragma unroll
      for (int r = 0; r < 10; ++r) {
        const int p = r * 64 + lane;
        if (p < 624) dst[g * GSTRIDE + p] = (uint32_t)(p ^ j);
      }
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        const int d = r * 64 + lane;
        if (d < 312) dc[g * 312 + d] = (uint8_t)(d ^ j);
      }
    }
  }
}

int main() {
  const uint64_t GiB = 1ull << 30;
  const uint64_t nenv = 1ull << 20;  // k_run's batch
  uint8_t *buf = nullptr, *buf2 = nullptr;
  uint32_t *perm = nullptr, *sink = nullptr;
  CHECK(hipMalloc(&buf, 2 * GiB));
  CHECK(hipMalloc(&buf2, 2 * GiB));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 1, 2 * GiB));
  CHECK(hipMemset(buf2, 2, 2 * GiB));
  std::vector<uint32_t> p(nenv);
  for (uint64_t i = 0; i < nenv; ++i) p[i] = (uint32_t)i;
  srand(7);
  for (uint64_t i = nenv - 1; i > 0; --i) std::swap(p[i], p[(uint64_t)rand() % (i + 1)]);
  CHECK(hipMalloc(&perm, nenv * 4));
  CHECK(hipMemcpy(perm, p.data(), nenv * 4, hipMemcpyHostToDevice));
  const int grid = 8192;
  // each pattern once as a warm-up of its code, then REPS timed dispatches (rocprofv3 averages)
  const int REPS = 3;
  printf("{\"kernels\": {\n");
  for (int r = 0; r < REPS; ++r) {
    // the cache holds the previous kernel's lines: flush it with a 1 GiB store in between
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_dword, dim3(grid), dim3(BLOCK), 0, 0, (const uint32_t*)buf, GiB / 4, sink);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_x4, dim3(grid), dim3(BLOCK), 0, 0, (const uint4*)buf, GiB / 16, sink);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_dma16_env, dim3(grid), dim3(BLOCK), 0, 0, buf, perm, nenv, 624u, sink);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_env_load<uint4>, dim3(grid), dim3(BLOCK), 0, 0, buf, perm, nenv, 1024u, sink);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_env_load<uint2>, dim3(grid), dim3(BLOCK), 0, 0, buf, perm, nenv, 1024u, sink);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_env_store<uint4>, dim3(grid), dim3(BLOCK), 0, 0, buf, perm, nenv, 1024u);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_env_store<uint2>, dim3(grid), dim3(BLOCK), 0, 0, buf, perm, nenv, 1024u);
  }
  // k_regen's store stream: 52,800 jobs (a uniform 1M-env launch's halves) over 262,144 envs
  const int njobs = 52800;
  const uint64_t genv = 1ull << 18;
  uint32_t *gmt = nullptr, *gjobs = nullptr;
  uint8_t* gmc = nullptr;
  CHECK(hipMalloc(&gmt, genv * 16 * 640 * 4));
  CHECK(hipMalloc(&gmc, genv * 4992));
  {
    std::vector<uint32_t> jb(njobs);
    std::vector<char> used(genv, 0);
    for (int j = 0; j < njobs; ++j) {
      uint32_t v;
      do v = (uint32_t)(((uint64_t)rand() * 65536 + rand()) % genv); while (used[v]);
      used[v] = 1;
      jb[j] = v | ((rand() & 1) ? 0x80000000u : 0u);
    }
    CHECK(hipMalloc(&gjobs, njobs * 4));
    CHECK(hipMemcpy(gjobs, jb.data(), njobs * 4, hipMemcpyHostToDevice));
  }
  for (int r = 0; r < REPS; ++r) {
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_gen_stores<624>, dim3(2048), dim3(BLOCK), 0, 0, gmt, gmc, gjobs, njobs);
    hipLaunchKernelGGL(k_dword_store, dim3(grid), dim3(BLOCK), 0, 0, (uint32_t*)buf2, GiB / 4);
    hipLaunchKernelGGL(k_gen_stores<640>, dim3(2048), dim3(BLOCK), 0, 0, gmt, gmc, gjobs, njobs);
  }
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(gmt));
  CHECK(hipFree(gmc));
  CHECK(hipFree(gjobs));
  // bytes each dispatch requests (loads or stores)
  printf("  \"k_dword\": %llu,\n", (unsigned long long)GiB);
  printf("  \"k_dword_store\": %llu,\n", (unsigned long long)GiB);
  printf("  \"k_x4\": %llu,\n", (unsigned long long)GiB);
  printf("  \"k_dma16_env\": %llu,\n", (unsigned long long)(16 * nenv));
  printf("  \"k_env_load<uint4>\": %llu,\n", (unsigned long long)(16 * nenv));
  printf("  \"k_env_load<uint2>\": %llu,\n", (unsigned long long)(8 * nenv));
  printf("  \"k_env_store<uint4>\": %llu,\n", (unsigned long long)(16 * nenv));
  printf("  \"k_env_store<uint2>\": %llu,\n", (unsigned long long)(8 * nenv));
  printf("  \"k_gen_stores<624>\": %llu,\n", (unsigned long long)njobs * 8 * (2496 + 312));
  printf("  \"k_gen_stores<640>\": %llu\n", (unsigned long long)njobs * 8 * (2496 + 312));
  printf("}}\n");
  CHECK(hipFree(buf));
  CHECK(hipFree(buf2));
  CHECK(hipFree(perm));
  CHECK(hipFree(sink));
  return 0;
}
