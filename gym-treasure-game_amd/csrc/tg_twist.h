// tg_twist.h — whole-wavefront MT19937 regeneration (device only): a half of the ring
// (MT_HALF_GENS generations, tg_core.h) twisted by the 64 lanes of one wave, the generations
// chained in the wave's LDS scratch, every generation's 312 draw codes and the even
// generations' 624 words stored (tg_core.h MT_STORE).
// Used by k_regen (the deferred regeneration, every 16 compact steps), k_gen_twist (tg_create,
// tg_write_state), k_reset and k_step (tg_amd.hip).  (The twist variants measured in isolation,
// DESIGN.md §3.3, are restated in scripts/calib/twist_bench.hip.)
//
// What bounds it: not HBM.  One generation is ~2.8 KB of stores, and the
// wave's VALU work per generation — 624 twists plus 312 draw codes — is what a k_regen launch
// spends its time on (8 waves per SIMD, every SIMD busy).  So the code pass is written for the
// fewest VALU instructions: one tempered word per draw, the outcome picked from a 4-entry table
// in a register by the draw's top 2 bits, no f64 except on the ~1-in-10^7 draws next to a
// threshold.
#pragma once
#include <hip/hip_runtime.h>

#include "tg_core.h"

namespace tg {

typedef __attribute__((address_space(1))) uint32_t glb_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;

// a ring store: plain, or non-temporal (NT: k_regen, whose words and codes are read steps later,
// not by this launch)
template <bool NT, class P, class T>
__device__ __forceinline__ void ring_store(P* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- draw codes: one tempered word per draw (tg_core.h top27_code) --------------------------
// A generation's 312 draw codes from its words in LDS: draw d = r * 64 + lane per round, its
// two words one 8-B LDS read (consecutive lanes, consecutive 8 B: no bank conflict, where a
// 4-B read of every other word conflicted 2-way), its code one byte of a coalesced 64-B store.
template <bool NT = false>
__device__ __forceinline__ void codes_from_lds(const lds_u32* w, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
  const lds_u64* const wl = reinterpret_cast<const lds_u64*>(w) + lane;
  uint8_t* const cl = dst_c + lane;
#pragma unroll
  for (int r = 0; r < (MT_N / 2 + 63) / 64; ++r) {
    if (r < MT_N / 2 / 64 || lane < MT_N / 2 - 64 * (MT_N / 2 / 64)) {
      const uint64_t p = wl[64 * r];  // words 128 r + 2 lane (low) and + 1
      const uint32_t w0 = (uint32_t)p, a = mt_temper(w0) >> 5;
      ring_store<NT>(cl + 64 * r,
                     (uint8_t)(__builtin_expect(top27_slow(a), 0) ? draw_code(mt_double(w0, (uint32_t)(p >> 32)))
                                                                  : top27_code(a)));
    }
  }
}

// ---- the twist --------------------------------------------------------------------------------
// genrand_uint32's twist of one word: y = upper bit of a | lower 31 bits of b; (y & 1) is b's
// low bit
__device__ __forceinline__ uint32_t twist_word(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & MT_UPPER) | (b & MT_LOWER);
  return c ^ (y >> 1) ^ ((0u - (b & 1u)) & 0x9908b0dfu);
}

// The whole-wave twist's inputs: 24 dwords per lane, loaded by twist_load, used by twist_store.
struct TwistIn {
  static constexpr int ROUNDS = (MT_N + 63) / 64;  // 10
  uint32_t a[ROUNDS], b[ROUNDS], c[4];
};
// the loads of a twist from a generation in HBM (issued, not waited for)
__device__ __forceinline__ void twist_load(const glb_u32* src, TwistIn& t) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < TwistIn::ROUNDS; ++r) {
    const int p = r * 64 + lane;
    t.a[r] = p < MT_N ? src[p] : 0u;
    t.b[r] = p + 1 < MT_N ? src[p + 1] : 0u;
    if (r < 4) t.c[r] = p < MT_N - MT_M ? src[p + MT_M] : 0u;
  }
}
// The rounds of a twist go in groups {0, 1, 2} {3, 4, 5} {6, 7, 8} {9}: round r reads new words
// p - 227 written by rounds r - 4 and r - 3 only, so a group needs nothing from itself, and its
// reads issue together (4 LDS round trips per generation instead of 10).
constexpr int TWIST_GROUP = 3;
// the generation after the one in t (registers), into scratch (LDS) and, unless null, dst
// (HBM), then, unless dst_c is null, its codes (dst / dst_c wave-uniform)
template <bool NT = false>
__device__ __forceinline__ void twist_store(const TwistIn& t, glb_u32* dst, uint8_t* dst_c,
                                            lds_u32* scratch) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r0 = 0; r0 < TwistIn::ROUNDS; r0 += TWIST_GROUP) {
#pragma unroll
    for (int r = r0; r < r0 + TWIST_GROUP && r < TwistIn::ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        const uint32_t bb = p + 1 < MT_N ? t.b[r] : scratch[0];
        const uint32_t cc = p < MT_N - MT_M ? t.c[r < 4 ? r : 0] : scratch[p - (MT_N - MT_M)];
        const uint32_t w = twist_word(t.a[r], bb, cc);
        scratch[p] = w;
        if (dst) ring_store<NT>(dst + p, w);
      }
    }
    // the group visible to later groups, whose lanes read what other lanes wrote: a
    // wavefront-scope fence orders the LDS accesses in the compiler (one wave's LDS operations
    // execute in order), without the hardware wait for the store's completion (A/B against
    // s_waitcnt lgkmcnt(0) after every round: 0.1322 vs 0.1340 ms)
    wave_fence();
  }
  if (dst_c) codes_from_lds<NT>(scratch, dst_c);
}
// The next generation in place in LDS (s: a generation -> its successor), stored to dst with
// its codes.  Round r reads words p + 1 (old: round r + 1 writes it, for lane 63), p + 397
// (old for p < 227: rounds >= 6 write them) or p - 227 (new: rounds r - 4 / r - 3), then
// writes p.  A group's reads are all issued before its writes (the compiler barrier: one
// wave's LDS operations execute in order), so round r + 1's write cannot overtake round r's
// read of word 64 (r + 1).  dst / dst_c as twist_store.  Must be reached by all 64 lanes.
template <bool NT = false>
__device__ __forceinline__ void twist_lds(lds_u32* s, glb_u32* dst, uint8_t* dst_c) {
  const int lane = threadIdx.x & 63;
  wave_fence();  // the previous codes pass's reads of s before this twist's writes
#pragma unroll
  for (int r0 = 0; r0 < TwistIn::ROUNDS; r0 += TWIST_GROUP) {
    uint32_t w[TWIST_GROUP];
#pragma unroll
    for (int r = r0; r < r0 + TWIST_GROUP && r < TwistIn::ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        const uint32_t a = s[p];
        const uint32_t b = s[p + 1 < MT_N ? p + 1 : 0];
        const uint32_t c = s[p < MT_N - MT_M ? p + MT_M : p - (MT_N - MT_M)];
        w[r - r0] = twist_word(a, b, c);
      }
    }
    asm volatile("" ::: "memory");  // the group's reads before its writes, in program order
#pragma unroll
    for (int r = r0; r < r0 + TWIST_GROUP && r < TwistIn::ROUNDS; ++r) {
      const int p = r * 64 + lane;
      if (p < MT_N) {
        s[p] = w[r - r0];
        if (dst) ring_store<NT>(dst + p, w[r - r0]);
      }
    }
    wave_fence();
  }
  if (dst_c) codes_from_lds<NT>(s, dst_c);
}
// `gens` generations in sequence after the one in t, ring generations g0, g0 + 1, ... of an env
// whose stored words start at w and codes at c: each one's codes, and the words of the even
// ones (tg_core.h mt_store_off).  With lead, one twist leads in first (t holds a stored
// generation 6; its successor, the other half's generation 7, is the chain's source: neither
// stored nor coded).  The first twist from registers, the rest chained in the wave's LDS
// scratch, so a half's regeneration reads one generation from HBM.  w / c wave-uniform; must
// be reached by all 64 lanes.
template <bool NT = false>
__device__ __forceinline__ void twist_chain(const TwistIn& t, glb_u32* w, uint8_t* c, int g0, int gens,
                                            bool lead, lds_u32* scratch) {
  auto wd = [&](int g) { return (g & 1) ? (glb_u32*)nullptr : w + mt_store_off((uint32_t)g); };
  if (lead) twist_store<NT>(t, nullptr, nullptr, scratch);
  else twist_store<NT>(t, wd(g0), c + g0 * (MT_N / 2), scratch);
  for (int j = lead ? 0 : 1; j < gens; ++j) twist_lds<NT>(scratch, wd(g0 + j), c + (g0 + j) * (MT_N / 2));
}
__device__ __forceinline__ void wave_twist_gens(const glb_u32* src, glb_u32* w, uint8_t* c, int g0,
                                                int gens, bool lead, lds_u32* scratch) {
  TwistIn t;
  twist_load(src, t);
  twist_chain(t, w, c, g0, gens, lead, scratch);
}
// stored word offset of the source of half dst's regeneration (dst: ring position 0 / MT_HALF):
// the other half's stored generation 6, whose twist (the lead-in) is that half's generation 7
__device__ __forceinline__ uint32_t regen_src_off(uint32_t dst) {
  return mt_store_off(((uint32_t)MT_HALF - dst) / (uint32_t)MT_N + (uint32_t)MT_HALF_GENS - 2u);
}

}  // namespace tg
