// twist_bench.hip — DIAGNOSTIC (not the product): throughput of the whole-wave MT19937
// regeneration ("twist", tg_amd.hip twist_load / twist_store) in isolation, in variants, over a
// k_run-sized list of stale halves (random envs of a 1M-env batch, as the refill queue sees
// them).  Every variant's output (words and draw codes) is checked against variant A's.
//   A  words in VGPRs (24 loads per lane), one twist at a time      (k_gen_twist, round 2)
//   B  A, software-pipelined: twist j + 1's loads in flight during j   (k_run's queue, round 3)
//   C  the source generation by LDS-DMA (3 x 1 KB global_load_lds), one twist at a time
//   D  C with the next twist's source DMA'd into a second LDS buffer during this one
//   E  C, then G = 4 chained twists in LDS: 4 generations of draw codes per source load, only the
//      last generation's words written (a code ring of G generations per half; rate counted per
//      generation, HBM bytes (2 x 2,496 + G x 312) / G per generation)
//   F  E writing every generation's words (a ring of 2G generations per env: no reconstruction
//      for the draws that need the double), HBM bytes (2,496 / G + 2,496 + 312) per generation
//   G  F with the draw codes from integer thresholds on the 53-bit draw (no f64 work)
//   H  E with the integer codes
//   I  C with the integer codes (one twist per source load, as k_run's refill queue)
//   J  a half of 8 generations per job, twisted in place in one LDS buffer, every generation's
//      words and codes stored (the product's twist_chain, source by LDS-DMA)
//   K  J with TWO jobs per wave, their rounds interleaved (two independent dependency chains)
//   L  J with the rounds in groups {0,1,2} {3,4,5} {6,7,8} {9} (the product's twist_lds)
//   M  L without the draw-code pass;  N  L without the global stores (latency anatomy)
//   O  L with the draw codes from the top 27 bits (draw_code_words: one tempered word)
// Prints one JSON line: twists per microsecond and the HBM bytes rate (5,304 B per twist).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "../../gym-treasure-game_amd/csrc/tg_core.h"

using namespace tg;

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) uint32_t lds_u32;
constexpr int BLOCK = 256;
constexpr int ROUNDS = (MT_N + 63) / 64;

struct Regs {
  uint32_t a[ROUNDS], b[ROUNDS], c[4];
};
__device__ __forceinline__ void load_regs(const uint32_t* src, Regs& t) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const int p = r * 64 + lane;
    t.a[r] = p < MT_N ? src[p] : 0u;
    t.b[r] = p + 1 < MT_N ? src[p + 1] : 0u;
    if (r < 4) t.c[r] = p < MT_N - MT_M ? src[p + MT_M] : 0u;
  }
}
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void codes_out(lds_u32* nw, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < (MT_N / 2 + 63) / 64; ++r) {
    const int d = r * 64 + lane;
    if (d < MT_N / 2) {
      const lds_u32* w = nw + 2 * d;
      dst_c[d] = (uint8_t)draw_code(mt_double(w[0], w[1]));
    }
  }
}
__device__ __forceinline__ void store_regs(const Regs& t, uint32_t* dst, uint8_t* dst_c, lds_u32* nw) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const int p = r * 64 + lane;
    if (p < MT_N) {
      const uint32_t bb = p + 1 < MT_N ? t.b[r] : nw[0];
      const uint32_t cc = p < MT_N - MT_M ? t.c[r < 4 ? r : 0] : nw[p - (MT_N - MT_M)];
      const uint32_t w = mt_twist(t.a[r], bb, cc);
      nw[p] = w;
      dst[p] = w;
    }
    wave_fence();
  }
  codes_out(nw, dst_c);
}
struct Thr {
  uint64_t p1, p2, n1, n2, j, f;
};
__constant__ Thr kThr;
__device__ __forceinline__ uint32_t code_int(uint32_t w0, uint32_t w1) {
  const uint64_t k = ((uint64_t)(mt_temper(w0) >> 5) << 26) | (mt_temper(w1) >> 6);
  const uint32_t pos = (uint32_t)(k >= kThr.p1) + (uint32_t)(k >= kThr.p2);
  const uint32_t neg = (uint32_t)(k >= kThr.n1) + (uint32_t)(k >= kThr.n2);
  return pos | (neg << CODE_NEG_SHIFT) | (k >= kThr.j ? CODE_JUMP : 0u) | (k < kThr.f ? CODE_FLIP : 0u);
}
__device__ __forceinline__ void codes_int(lds_u32* nw, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < (MT_N / 2 + 63) / 64; ++r) {
    const int d = r * 64 + lane;
    if (d < MT_N / 2) {
      const lds_u32* w = nw + 2 * d;
      dst_c[d] = (uint8_t)code_int(w[0], w[1]);
    }
  }
}
// the source generation into LDS: 156 x 16 B chunks, lane l takes chunks l, l + 64, l + 128
__device__ __forceinline__ void dma_src(const uint32_t* src, lds_u32* s) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int ch = j * 64 + lane;
    if (ch < MT_N / 4) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(s + j * 256));
      const void* g = src + ch * 4;
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
  }
}
template <bool INT = false>
__device__ __forceinline__ void store_lds(const lds_u32* s, uint32_t* dst, uint8_t* dst_c, lds_u32* nw) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const int p = r * 64 + lane;
    if (p < MT_N) {
      const uint32_t a = s[p];
      const uint32_t bb = p + 1 < MT_N ? s[p + 1] : nw[0];
      const uint32_t cc = p < MT_N - MT_M ? s[p + MT_M] : nw[p - (MT_N - MT_M)];
      const uint32_t w = mt_twist(a, bb, cc);
      nw[p] = w;
      dst[p] = w;
    }
    wave_fence();
  }
  if (INT) codes_int(nw, dst_c); else codes_out(nw, dst_c);
}

// G twists chained in LDS from the source in s: codes of every generation, words of the last
// only (ALL = false) or of every generation (ALL: dst + g * MT_N)
template <int G, bool ALL = false, bool INT = false>
__device__ __forceinline__ void chain_lds(lds_u32* s, lds_u32* t, uint32_t* dst, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        const uint32_t a = s[p];
        const uint32_t bb = p + 1 < MT_N ? s[p + 1] : t[0];
        const uint32_t cc = p < MT_N - MT_M ? s[p + MT_M] : t[p - (MT_N - MT_M)];
        const uint32_t w = mt_twist(a, bb, cc);
        t[p] = w;
        if (ALL) dst[g * MT_N + p] = w;
        else if (g == G - 1) dst[p] = w;
      }
      wave_fence();
    }
    if (INT) codes_int(t, dst_c + g * (MT_N / 2));
    else codes_out(t, dst_c + g * (MT_N / 2));
    lds_u32* x = s; s = t; t = x;
  }
}

// in-place successor of the generation in s (the product's twist_lds), words + codes stored
__device__ __forceinline__ void inplace_round(lds_u32* s, int r, uint32_t* dst) {
  const int lane = threadIdx.x & 63;
  const int p = r * 64 + lane;
  if (p < MT_N) {
    const uint32_t a = s[p];
    const uint32_t b = s[p + 1 < MT_N ? p + 1 : 0];
    const uint32_t c = s[p < MT_N - MT_M ? p + MT_M : p - (MT_N - MT_M)];
    const uint32_t w = mt_twist(a, b, c);
    s[p] = w;
    dst[p] = w;
  }
}
template <int G>
__device__ __forceinline__ void chain1(lds_u32* s, uint32_t* dst, uint8_t* dst_c) {
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    wave_fence();
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
      inplace_round(s, r, dst + g * MT_N);
      wave_fence();
    }
    codes_out(s, dst_c + g * (MT_N / 2));
  }
}
template <int G>
__device__ __forceinline__ void chain2(lds_u32* s, uint32_t* dst, uint8_t* dst_c, lds_u32* s2, uint32_t* dst2,
                                       uint8_t* dst_c2) {
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    wave_fence();
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
      inplace_round(s, r, dst + g * MT_N);
      inplace_round(s2, r, dst2 + g * MT_N);
      wave_fence();
    }
    codes_out(s, dst_c + g * (MT_N / 2));
    codes_out(s2, dst_c2 + g * (MT_N / 2));
  }
}

// the product's grouped in-place twist (tg_amd.hip twist_lds), with parts switched off
__device__ __forceinline__ void codes_top27(lds_u32* nw, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < (MT_N / 2 + 63) / 64; ++r) {
    const int d = r * 64 + lane;
    if (d < MT_N / 2) {
      const lds_u32* w = nw + 2 * d;
      dst_c[d] = (uint8_t)draw_code_words(w[0], w[1]);
    }
  }
}
// CODES: 0 none, 1 draw_code(mt_double) (f64), 2 draw_code_words (the top 27 bits)
template <int CODES, bool STORES>
__device__ __forceinline__ void inplace_grouped(lds_u32* s, uint32_t* dst, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
  wave_fence();
#pragma unroll
  for (int r0 = 0; r0 < ROUNDS; r0 += 3) {
    uint32_t w[3];
#pragma unroll
    for (int r = r0; r < r0 + 3 && r < ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        const uint32_t a = s[p];
        const uint32_t b = s[p + 1 < MT_N ? p + 1 : 0];
        const uint32_t c = s[p < MT_N - MT_M ? p + MT_M : p - (MT_N - MT_M)];
        w[r - r0] = mt_twist(a, b, c);
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = r0; r < r0 + 3 && r < ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        s[p] = w[r - r0];
        if (STORES) dst[p] = w[r - r0];
      }
    }
    wave_fence();
  }
  if (CODES == 1) codes_out(s, dst_c);
  if (CODES == 2) codes_top27(s, dst_c);
}
template <int G, int CODES, bool STORES>
__device__ __forceinline__ void chain_g(lds_u32* s, uint32_t* dst, uint8_t* dst_c) {
#pragma unroll 1
  for (int g = 0; g < G; ++g) inplace_grouped<CODES, STORES>(s, dst + g * MT_N, dst_c + g * (MT_N / 2));
}

struct Job {
  uint32_t* mt;   // [envs][1248]
  uint8_t* mc;    // [envs][624]
  uint8_t* mc4;   // [envs][4 * 312] (variants E-G)
  uint32_t* mt4;  // [envs][4 * 624] (variants F, G)
  uint32_t* mt8;  // [envs][8 * 624] (variants J, K)
  uint8_t* mc8;   // [envs][8 * 312]
  const uint32_t* ent;  // env | src half << 31
  int n;
};
__device__ __forceinline__ void job_ptrs(const Job& J, uint32_t e, const uint32_t*& src, uint32_t*& dst,
                                         uint8_t*& dc) {
  const uint64_t env = e & 0x7FFFFFFFu;
  const uint32_t sh = (e >> 31) ? (uint32_t)MT_N : 0u;
  src = J.mt + env * MT_WORDS + sh;
  dst = J.mt + env * MT_WORDS + (MT_N - sh);
  dc = J.mc + env * MT_CODES + (MT_N - sh) / 2;
}

template <int V>
__global__ __launch_bounds__(BLOCK) void k_twist(Job J) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[BLOCK / 64][3 * MT_N];
  lds_u32* const base = (lds_u32*)lds[threadIdx.x >> 6];
  const int nw = (int)(gridDim.x * (BLOCK / 64));
  const int w = (int)((blockIdx.x * BLOCK + threadIdx.x) >> 6);
  const uint32_t *src;
  uint32_t* dst;
  uint8_t* dc;
  if constexpr (V == 0) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      Regs t;
      load_regs(src, t);
      store_regs(t, dst, dc, base);
    }
  } else if constexpr (V == 1) {
    int j = w;
    if (j >= J.n) return;
    Regs t;
    job_ptrs(J, J.ent[j], src, dst, dc);
    load_regs(src, t);
    while (true) {
      Regs u = t;
      uint32_t* d0 = dst;
      uint8_t* c0 = dc;
      const int jn = j + nw;
      if (jn < J.n) {
        job_ptrs(J, J.ent[jn], src, dst, dc);
        load_regs(src, t);
      }
      store_regs(u, d0, c0, base);
      if (jn >= J.n) break;
      j = jn;
    }
  } else if constexpr (V == 2) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous twist's LDS reads done
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_lds(base, dst, dc, base + MT_N);
    }
  } else if constexpr (V == 4) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      chain_lds<4>(base, base + MT_N, dst, J.mc4 + (uint64_t)(J.ent[j] & 0x7FFFFFFFu) * (4 * MT_N / 2));
    }
  } else if constexpr (V == 7) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      chain_lds<4, false, true>(base, base + MT_N, dst, J.mc4 + (uint64_t)(J.ent[j] & 0x7FFFFFFFu) * (4 * MT_N / 2));
    }
  } else if constexpr (V == 8) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_lds<true>(base, dst, dc, base + MT_N);
    }
  } else if constexpr (V == 9) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t env = J.ent[j] & 0x7FFFFFFFu;
      chain1<8>(base, J.mt8 + env * (8 * MT_N), J.mc8 + env * (8 * MT_N / 2));
    }
  } else if constexpr (V == 10) {
    for (int j = 2 * w; j < J.n; j += 2 * nw) {
      const uint32_t *src2;
      uint32_t* dst2;
      uint8_t* dc2;
      const bool two = j + 1 < J.n;
      job_ptrs(J, J.ent[j], src, dst, dc);
      job_ptrs(J, J.ent[two ? j + 1 : j], src2, dst2, dc2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      dma_src(src2, base + MT_N);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t env = J.ent[j] & 0x7FFFFFFFu, env2 = J.ent[two ? j + 1 : j] & 0x7FFFFFFFu;
      if (two)
        chain2<8>(base, J.mt8 + env * (8 * MT_N), J.mc8 + env * (8 * MT_N / 2), base + MT_N,
                  J.mt8 + env2 * (8 * MT_N), J.mc8 + env2 * (8 * MT_N / 2));
      else
        chain1<8>(base, J.mt8 + env * (8 * MT_N), J.mc8 + env * (8 * MT_N / 2));
    }
  } else if constexpr (V >= 11 && V <= 14) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t env = J.ent[j] & 0x7FFFFFFFu;
      chain_g<8, V == 12 ? 0 : V == 14 ? 2 : 1, V != 13>(base, J.mt8 + env * (8 * MT_N), J.mc8 + env * (8 * MT_N / 2));
    }
  } else if constexpr (V == 5 || V == 6) {
    for (int j = w; j < J.n; j += nw) {
      job_ptrs(J, J.ent[j], src, dst, dc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_src(src, base);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t env = J.ent[j] & 0x7FFFFFFFu;
      chain_lds<4, true, V == 6>(base, base + MT_N, J.mt4 + env * (4 * MT_N), J.mc4 + env * (4 * MT_N / 2));
    }
  } else {
    int j = w;
    if (j >= J.n) return;
    int buf = 0;
    job_ptrs(J, J.ent[j], src, dst, dc);
    dma_src(src, base);
    while (true) {
      uint32_t* d0 = dst;
      uint8_t* c0 = dc;
      const int jn = j + nw;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other buffer's reads done
      if (jn < J.n) {
        job_ptrs(J, J.ent[jn], src, dst, dc);
        dma_src(src, base + (buf ^ 1) * MT_N);
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // this twist's source (not the next's)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      store_lds(base + buf * MT_N, d0, c0, base + 2 * MT_N);
      if (jn >= J.n) break;
      j = jn;
      buf ^= 1;
    }
  }
}

__global__ void k_fill(uint32_t* mt, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    mt[i] = (uint32_t)(x ^ (x >> 31));
  }
}

int main(int argc, char** argv) {
  const uint64_t envs = 1ull << 20;
  const int njobs = argc > 1 ? atoi(argv[1]) : 130000;
  const int grid = argc > 2 ? atoi(argv[2]) : 1280;  // 5 waves per SIMD x 1024 SIMDs / 4
  uint32_t* mt;
  uint8_t* mc;
  uint32_t* ent;
  uint8_t* mc4;
  uint32_t* mt4;
  CHECK(hipMalloc(&mc4, envs * 4 * MT_N / 2));
  CHECK(hipMalloc(&mt4, envs * 4 * MT_N * 4));
  uint32_t* mt8;
  uint8_t* mc8;
  CHECK(hipMalloc(&mt8, envs * 8 * MT_N * 4));
  CHECK(hipMalloc(&mc8, envs * 8 * MT_N / 2));
  {  // integer thresholds of draw_code on k = r * 2^53 (each field is monotone in r)
    auto code_k = [](uint64_t k) { return draw_code((double)k * (1.0 / 9007199254740992.0)); };
    auto first = [&](auto pred) {  // smallest k in [0, 2^53] with pred(code_k(k))
      uint64_t lo = 0, hi = 1ull << 53;
      while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (pred(code_k(mid))) hi = mid; else lo = mid + 1;
      }
      return lo;
    };
    Thr t;
    t.p1 = first([](uint32_t c) { return (c & CODE_POS) >= 1; });
    t.p2 = first([](uint32_t c) { return (c & CODE_POS) >= 2; });
    t.n1 = first([](uint32_t c) { return ((c >> CODE_NEG_SHIFT) & 3u) >= 1; });
    t.n2 = first([](uint32_t c) { return ((c >> CODE_NEG_SHIFT) & 3u) >= 2; });
    t.j = first([](uint32_t c) { return (c & CODE_JUMP) != 0; });
    t.f = first([](uint32_t c) { return (c & CODE_FLIP) == 0; });
    // the thresholds reproduce draw_code around each boundary
    const uint64_t b[6] = {t.p1, t.p2, t.n1, t.n2, t.j, t.f};
    for (uint64_t x : b)
      for (int64_t d = -3; d <= 3; ++d) {
        const uint64_t k = x + d;
        const uint32_t c = (uint32_t)(k >= t.p1) + (uint32_t)(k >= t.p2) |
                           (((uint32_t)(k >= t.n1) + (uint32_t)(k >= t.n2)) << CODE_NEG_SHIFT) |
                           (k >= t.j ? CODE_JUMP : 0u) | (k < t.f ? CODE_FLIP : 0u);
        if (c != code_k(k)) { fprintf(stderr, "threshold mismatch at %llu\n", (unsigned long long)k); exit(1); }
      }
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(kThr), &t, sizeof t));
  }
  CHECK(hipMalloc(&mt, envs * MT_WORDS * 4));
  CHECK(hipMalloc(&mc, envs * MT_CODES));
  CHECK(hipMalloc(&ent, njobs * 4));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(BLOCK), 0, 0, mt, envs * MT_WORDS);
  CHECK(hipDeviceSynchronize());
  srand(1);
  std::vector<uint32_t> e(njobs);
  std::vector<char> used(envs, 0);
  for (int j = 0; j < njobs; ++j) {  // distinct envs (a half is listed once per step)
    uint32_t v;
    do v = (uint32_t)(((uint64_t)rand() * 65536 + rand()) % envs); while (used[v]);
    used[v] = 1;
    e[j] = v | ((rand() & 1) ? 0x80000000u : 0u);
  }
  CHECK(hipMemcpy(ent, e.data(), njobs * 4, hipMemcpyHostToDevice));
  const Job J{mt, mc, mc4, mt4, mt8, mc8, ent, njobs};
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<uint32_t> ref_w, ref_c, ref4_w, ref4_c, ref8_w, ref8_c;
  printf("{\"jobs\": %d, \"grid\": %d, \"variants\": {", njobs, grid);
  for (int v = 0; v < 15; ++v) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      // jobs name distinct envs and read one half, write the other: every run sees the same input
      CHECK(hipEventRecord(a));
      if (v == 0) hipLaunchKernelGGL(k_twist<0>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 1) hipLaunchKernelGGL(k_twist<1>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 2) hipLaunchKernelGGL(k_twist<2>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 3) hipLaunchKernelGGL(k_twist<3>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 4) hipLaunchKernelGGL(k_twist<4>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 5) hipLaunchKernelGGL(k_twist<5>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 6) hipLaunchKernelGGL(k_twist<6>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 7) hipLaunchKernelGGL(k_twist<7>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 8) hipLaunchKernelGGL(k_twist<8>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 9) hipLaunchKernelGGL(k_twist<9>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 10) hipLaunchKernelGGL(k_twist<10>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 11) hipLaunchKernelGGL(k_twist<11>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 12) hipLaunchKernelGGL(k_twist<12>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 13) hipLaunchKernelGGL(k_twist<13>, dim3(grid), dim3(BLOCK), 0, 0, J);
      if (v == 14) hipLaunchKernelGGL(k_twist<14>, dim3(grid), dim3(BLOCK), 0, 0, J);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    // output check: a sample of the regenerated halves against variant A
    std::vector<uint32_t> w(envs * MT_WORDS / 64), c(envs * MT_CODES / 64 / 4);
    CHECK(hipMemcpy(w.data(), mt, w.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c.data(), mc, c.size() * 4, hipMemcpyDeviceToHost));
    bool same = true;
    if (v == 0) ref_w = w, ref_c = c;
    else if (v < 4 || v == 8) same = (w == ref_w) && (c == ref_c);
    std::vector<uint32_t> w4(envs * 4 * MT_N / 64), c4(envs * 4 * MT_N / 2 / 64 / 4);
    std::vector<uint32_t> w8(envs * 8 * MT_N / 64), c8(envs * 8 * MT_N / 2 / 64 / 4);
    if ((v >= 9 && v <= 11) || v == 14) {
      CHECK(hipMemcpy(w8.data(), mt8, w8.size() * 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(c8.data(), mc8, c8.size() * 4, hipMemcpyDeviceToHost));
      if (v == 9) ref8_w = w8, ref8_c = c8;
      else same = (w8 == ref8_w) && (c8 == ref8_c);
    }
    if (v >= 5 && v <= 6) {
      CHECK(hipMemcpy(w4.data(), mt4, w4.size() * 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(c4.data(), mc4, c4.size() * 4, hipMemcpyDeviceToHost));
      if (v == 5) ref4_w = w4, ref4_c = c4;
      else same = (w4 == ref4_w) && (c4 == ref4_c);
    }
    const double us = best * 1e3;
    const int gens = v >= 4 && v <= 7 ? 4 : v >= 9 ? 8 : 1;
    // per-wave latency of one generation: waves busy x time / generations
    const int waves_busy = std::min(njobs / (v == 10 ? 2 : 1), grid * 4);
    const double bytes = v == 4 || v == 7 ? 2 * 2496.0 + 4 * 312.0
                         : v == 5 || v == 6 ? 5 * 2496.0 + 4 * 312.0
                         : v >= 9 ? 9 * 2496.0 + 8 * 312.0 : 5304.0;
    printf("%s\"%c\": {\"ms\": %.4f, \"twists_per_us\": %.1f, \"us_per_gen_per_wave\": %.2f, "
           "\"GBps\": %.0f, \"same_as_A\": %s}",
           v ? ", " : "", 'A' + v, best, njobs * gens / us, waves_busy * us / ((double)njobs * gens),
           njobs * bytes / us / 1e3,
           v == 4 || v == 5 || v == 7 || v == 9 || v == 12 || v == 13 ? "null" : same ? "true" : "false");
  }
  printf("}}\n");
  return 0;
}
