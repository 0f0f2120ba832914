// tg_amd.hip — MI355X (gfx950) batched Treasure Game: kernels + the C ABI of include/tg_amd.h.
//
// One wavefront lane per env.  Per launch every lane loads its env from struct-of-arrays
// HBM (16-B + 16-B + 8-B coalesced loads), runs the requested option to completion
// (_Option.run, OP/:20-36) over the level grid staged in LDS, writes obs / reward / valid /
// done, and stores the env back.  Auto-reset compacts completed episodes with a wavefront
// ballot + one atomic per wave.  No MFMA: the path is integer/branch work plus a handful of
// IEEE f64 ops (obs divisions, uniform/gauss), built with -ffp-contract=off.
//
// HBM layout per handle (N envs):
//   st4[N]  uint4   {pos = px | py<<16 (i16 pair), flags, objs = kx,ky,gx,gy (i8 x4), mt_pos}
//   ang[N]  double2 {handle0.angle, handle1.angle}
//   ep[N]   int2    {episode return, episode length}
//   mt[N][624] u32  env-major MT19937 words (2,496 B per env)
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <algorithm>
#include <chrono>
#include <mutex>
#include <cstdlib>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tg_amd.h"
#include "tg_core.h"
#include "tg_level.h"
#include "tg_batch.h"
#include "tg_twist.h"

#ifndef TG_FLOW_TU  // (tg_flow.hip includes this file for the device code only)
namespace tg {
thread_local std::string g_err;
}
#endif
using namespace tg;
namespace {
void srv_register(tg_batch* h, bool live);  // the exit-time server registry (below)
}

namespace {

constexpr int BLOCK = 256;
// k_run's workgroup: a workgroup holds its CU slot (LDS, wave slots) until its slowest wave
// ends, and k_run's waves differ in length by up to ~3x
#ifndef TG_RUN_BLOCK
#define TG_RUN_BLOCK 256
#endif
constexpr int RUN_BLOCK = TG_RUN_BLOCK;
static_assert(RUN_BLOCK % 64 == 0 && BLOCK % RUN_BLOCK == 0, "whole waves, whole k_classify blocks");
// issue priority of the option waves whose ticks are slow (ladders, drops, jumps), which share
// SIMDs with the go waves (0.153 vs 0.156 ms per step)
constexpr int PRIO_SLOW = 3;

// ------------------------------------------------------------------------------------------
// SoA pack / unpack
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void unpack_st4(const uint4 s, Env& e) {
  e.px = (int)(int16_t)(s.x & 0xFFFFu);
  e.py = (int)(int16_t)(s.x >> 16);
  e.f = s.y;
  e.kx = (int)(int8_t)(s.z & 0xFF);
  e.ky = (int)(int8_t)((s.z >> 8) & 0xFF);
  e.gx = (int)(int8_t)((s.z >> 16) & 0xFF);
  e.gy = (int)(int8_t)(s.z >> 24);
  e.mti = s.w;
}
__device__ __forceinline__ void unpack(const uint4 s, const double2 a, Env& e) {
  unpack_st4(s, e);
  e.ang0 = a.x;
  e.ang1 = a.y;
}
__device__ __forceinline__ uint4 pack(const Env& e) {
  uint4 s;
  s.x = ((uint32_t)e.px & 0xFFFFu) | ((uint32_t)e.py << 16);
  s.y = e.f;
  s.z = ((uint32_t)e.kx & 0xFF) | (((uint32_t)e.ky & 0xFF) << 8) | (((uint32_t)e.gx & 0xFF) << 16) |
        ((uint32_t)e.gy << 24);
  s.w = e.mti;
  return s;
}

// The level in LDS: the bordered cell grid (per-lane indexed probes) and the trigger table
// (indexed per lane by the cascade; kernel arguments indexed per lane would be vector loads
// from the kernarg segment).
struct LdsLevel {
  uint32_t trig[12];
  uint32_t grid[MAX_CELLS / 4];
};
TG_HD int grid_words(int W, int H) { return ((W + 2 * PAD) * (H + 2 * PAD) + 3) / 4; }
// grid words, trigger table and (masks: non-null) the level bitmasks into LDS; NT: the
// workgroup's threads
template <int NT = BLOCK>
__device__ __forceinline__ void stage_cells(uint32_t* lgrid, uint32_t* ltrig,
                                            const uint32_t* __restrict__ grid, const Level& L,
                                            uint32_t* masks = nullptr) {
  const int nwords = grid_words(L.W, L.H);
  for (int i = threadIdx.x; i < nwords; i += NT) lgrid[i] = grid[i];
  if (threadIdx.x < 12) ltrig[threadIdx.x] = L.trig[threadIdx.x >> 1][threadIdx.x & 1];
  if (masks && L.masks)
    for (int i = threadIdx.x; i < mk_words(L.W, L.H); i += NT) masks[i] = L.masks[i];
  __syncthreads();
}
__device__ __forceinline__ void stage_level(LdsLevel& lv, const uint32_t* __restrict__ grid,
                                            const Level& L) {
  stage_cells(lv.grid, lv.trig, grid, L);
}
#define LEVEL_IN_LDS()                   \
  __shared__ LdsLevel lv;                \
  stage_level(lv, grid, L);              \
  const uint32_t* const trig = lv.trig;  \
  const Map m{reinterpret_cast<const uint8_t*>(lv.grid), L.W, L.H}
// k_run's LDS: the waves' code windows (WIN_WAVE_BYTES each, at offset 0: 16-B aligned for the
// LDS-DMA), then the level's grid words and bitmasks (Map::mk).  (Sized at launch for the
// handle's level instead of the largest, with the rows' loads issued before the staging
// barrier, it measured ~4 % slower for the masked policy: DESIGN.md §3.1.)
#define RUN_LEVEL_IN_LDS()                                                                \
  __shared__ uint4 run_lds[((RUN_BLOCK / 64) * WIN_WAVE_BYTES + MAX_CELLS + 4 * MK_MAX_WORDS) / 16]; \
  __shared__ uint32_t ltrig[12];                                                          \
  uint8_t* const win = reinterpret_cast<uint8_t*>(run_lds);                                \
  uint32_t* const lgrid = reinterpret_cast<uint32_t*>(win + (RUN_BLOCK / 64) * WIN_WAVE_BYTES); \
  uint32_t* const lmk = lgrid + grid_words(L.W, L.H);                                     \
  stage_cells<RUN_BLOCK>(lgrid, ltrig, grid, L, lmk);                                     \
  const uint32_t* const trig = ltrig;                                                     \
  const Map m{reinterpret_cast<const uint8_t*>(lgrid), L.W, L.H, L.masks ? lmk : nullptr}

__device__ __forceinline__ void store_obs(double* out, int64_t i, const double o[9]) {
  double* p = out + i * 9;
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k] = o[k];
}

// ------------------------------------------------------------------------------------------
// CPython random for the option loops (k_run, k_step): tg::Rng's read-only consumption of the
// two pre-twisted generations, reading each draw's code byte (tg_core.h draw_code: its noisy /
// jump / flip outcomes) from a per-lane window in LDS.
//   Window: WIN_CHUNKS 16-B chunks (16 codes each) per lane, slot j of the wave's window at
//   m0 + j * 1 KB holding the lane's j-th chunk from where the window starts.  prime() fills
//   it with one LDS-DMA (global_load_lds_dwordx4) per slot: every lane's chunk j goes to slot
//   j, so M0 (which addresses the DMA's LDS destination and must be wave-uniform) is the same
//   for all of them and each slot costs ONE instruction.  The first draw waits for the DMAs
//   (s_waitcnt vmcnt(0), once per launch; k_run primes before the option's setup so the wait
//   is mostly covered); every later draw is an LDS byte read, issued one draw ahead.  The
//   window holds 112 draws, more than an option of the default level consumes in one step
//   (<= ~110); a lane that exhausts it refills it the same way (WAR: lgkmcnt(0) before the
//   DMAs; RAW: vmcnt(0) after) and pays one memory latency.  The DMAs are issued from inline
//   asm, invisible to the compiler's waitcnt pass, so no register copy of a loaded value is
//   waited for early (a register-held prefetch made the compiler wait at the load).
//   Position bookkeeping is deferred: the window start (pos) plus the draws taken since (n)
//   are folded into pos at a refill and at finish.
//   Stale halves: a window overlapping the half the lane is not in, while that half is stale
//   (crossed), is loaded only after the lane has regenerated that half itself (regen_half:
//   rare, > 312 draws since the refill; the refilling idle wave, if any, writes the same).
//   Draws that need the double (handle angles in a flip cascade, an auto-reset's uniform and
//   gauss) consume the code and read the position's two words (one 8-B load).
// ------------------------------------------------------------------------------------------
// code bytes per lane per LDS-DMA (global_load_lds_dwordx4).  The dword form (lane l's 4 B at
// M0 + 4l, no LDS bank conflicts) needs 4x the DMA instructions per fill and measured 7 %
// slower (profiles/r03/lds_window_ab.json)
constexpr int WIN_UNIT = 16;
constexpr int WIN_DRAWS = 64;                       // codes per lane in the window
constexpr int WIN_SLOTS = WIN_DRAWS / WIN_UNIT;     // DMA instructions per fill
constexpr int WIN_SLOT_BYTES = 64 * WIN_UNIT;       // one slot: every lane's unit
constexpr uint32_t CODE_UNITS = MT_CODES / WIN_UNIT;
static_assert(MT_CODES % WIN_UNIT == 0, "whole DMA units of codes per env");
constexpr int WIN_WAVE_BYTES = WIN_SLOTS * WIN_SLOT_BYTES;  // 4 KB per wave
constexpr int WAVE_SCRATCH = MT_N * 4;                       // wave_twist's scratch (aliases it)
static_assert(WIN_WAVE_BYTES >= WAVE_SCRATCH, "wave_refill reuses the window as scratch");
static_assert(WIN_DRAWS - WIN_UNIT + 1 >= (int)MAX_TICK_DRAWS, "a refilled window holds a tick's draws");

// LDS-DMA of one WIN_UNIT-byte unit per active lane into LDS [m0 + lane * WIN_UNIT]; M0 is
// saved/restored.  SC1: the load bypasses this CU's L1 (k_flow, whose codes another CU of the
// XCD may have rewritten in the same launch: tg_flow.h)
template <bool SC1 = false>
__device__ __forceinline__ void glds_unit(uint32_t m0, const void* gptr) {
  uint32_t save;
  if constexpr (SC1)
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off sc1\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(save)
        : "s"(__builtin_amdgcn_readfirstlane(m0)), "v"(gptr)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(save)
        : "s"(__builtin_amdgcn_readfirstlane(m0)), "v"(gptr)
        : "memory");
}

// the rare second crossing (RngCodes::fill), out of line so that the draw sites stay small, its
// generation loops out of line too: a callee's registers add to its caller's allocation (k_run
// 104 VGPRs, 4 waves per SIMD, with them inline)
__device__ __noinline__ void twist_gen_call(const uint32_t* src, uint32_t* dst) { twist_gen(src, dst); }
__device__ __noinline__ void gen_codes_call(const uint32_t* w, uint8_t* c) { gen_codes(w, c); }
struct GenCalls {
  __device__ void twist(const uint32_t* src, uint32_t* dst) const { twist_gen_call(src, dst); }
  __device__ void codes(const uint32_t* w, uint8_t* c) const { gen_codes_call(w, c); }
};
__device__ __noinline__ void regen_half(uint32_t* mt, uint8_t* mc, uint32_t h) {
  twist_half(mt, h, mc, false, GenCalls());
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
}
// k_flow's form: the half's source words may have been written by another CU of the XCD in the
// same launch (the env's previous item ran there), so this CU's L1 is invalidated first; the
// stores go through the L1 (write-through) to the XCD's L2, where the env's next item, on
// whichever CU of the XCD, reads them with L1-bypassing loads (tg_flow.h) once this wave's
// stores are complete.  No L2 writeback: nothing crosses XCDs (an agent-scope release's
// buffer_wbl2 here wrote back the XCD's whole L2 on every per-lane regeneration).
__device__ __noinline__ void regen_half_flow(uint32_t* mt, uint8_t* mc, uint32_t h) {
  asm volatile("buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
  twist_half(mt, h, mc, false, GenCalls());
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
}

// a stored MT word read past this CU's L1 (an agent-scope relaxed load: global_load sc1), for
// k_flow, where another CU of the XCD may have rewritten it in the same launch (tg_flow.h)
struct Sc1Ld {
  __device__ uint32_t operator()(const uint32_t* p) const {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};
__device__ __noinline__ WordPair mt_pair_ool_sc1(const uint32_t* mt, uint32_t p) {
  WordPair r;
  mt_pair(mt, p, r.w0, r.w1, Sc1Ld());
  return r;
}

template <bool FLOW = false>  // FLOW: k_flow's L1-bypassing loads (tg_flow.h)
struct RngCodesT {
  static constexpr uint32_t NONE = 0xFFFFFFFFu;
  uint32_t* mt;      // this env's MT_STORE stored words (HBM)
  uint8_t* mc;       // this env's MT_CODES code bytes (HBM)
  lds_u8* cell;      // this lane's unit in slot 0 of the wave's window
  uint32_t m0;       // LDS address of slot 0 of the wave's window (wave-uniform)
  uint32_t pos;      // word position of the window's first draw (even)
  uint32_t n;        // draws taken since then
  uint32_t rd;       // LDS offset of the next draw's code from cell: slot * 1 KB + byte
  uint32_t left;     // draws left in the window
  uint32_t nxc;      // the next draw's code (read one draw ahead)
  uint32_t stale;    // word offset (0 / 624) of the half that is two generations behind, or NONE
  uint32_t tag;      // the state word's MT_STALE | MT_LISTED bits on entry
  uint32_t draws;
  uint32_t regens;   // halves this lane regenerated itself (regen_half)
  bool primed, loaded, entered;  // entered: a half was entered in this launch (as tg::Rng)

  __device__ __forceinline__ RngCodesT(uint32_t* m, uint8_t* c, uint32_t state, lds_u8* wave_win)
      : mt(m), mc(c), cell(wave_win + (threadIdx.x & 63) * WIN_UNIT),
        m0(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)wave_win)),
        pos(state & MT_POS_MASK), n(0u), rd(0u), left(0u), nxc(0u),
        stale((state & MT_STALE) ? (uint32_t)MT_HALF - mt_half(state & MT_POS_MASK) : NONE),
        tag(state & (MT_STALE | MT_LISTED)),
        draws(0u), regens(0u), primed(false), loaded(false), entered(false) {}

  // fold the draws taken since the window start into pos (a window is < MT_HALF / 2 draws, so
  // at most one half boundary lies in between).  Entering a half that is stale (possible only
  // when the window ended exactly at the boundary, so nothing of it was read) regenerates it
  // first, from the half being left, which then becomes the stale one.
  __device__ __forceinline__ void sync() {
    const uint32_t d = pos >> 1, e = d + n;
    if (e / (MT_HALF / 2) != d / (MT_HALF / 2)) {
      const uint32_t left_half = mt_half(pos), entered_half = (uint32_t)MT_HALF - left_half;
      if (stale == entered_half) {
        if (FLOW) regen_half_flow(mt, mc, entered_half);
        else regen_half(mt, mc, entered_half);
        ++regens;
      }
      stale = left_half;
      entered = true;
    }
    pos = 2u * (e >= (uint32_t)MT_CODES ? e - (uint32_t)MT_CODES : e);
    n = 0u;
  }
  // DMA the window starting at pos (all lanes reaching it start at slot 0: one DMA per slot)
  __device__ __forceinline__ void fill() {
    const uint32_t d = pos >> 1, c0 = d / (uint32_t)WIN_UNIT;
    if (stale != NONE) {
      // the draws the window serves are words [pos, pos + 2 * left) (mod MT_WORDS; the bytes of
      // its first and last chunks outside that range are never read): regenerate the stale
      // half first if they overlap it
      const uint32_t w0 = pos, w1 = pos + 2u * ((uint32_t)WIN_DRAWS - d % (uint32_t)WIN_UNIT);
      if ((w0 < stale + (uint32_t)MT_HALF && stale < w1) ||
          (w1 > (uint32_t)MT_WORDS && stale < w1 - (uint32_t)MT_WORDS)) {
        if (FLOW) regen_half_flow(mt, mc, stale);
        else regen_half(mt, mc, stale);
        ++regens;
        stale = NONE;
      }
    }
#pragma unroll
    for (int j = 0; j < WIN_SLOTS; ++j) {
      const uint32_t c = c0 + j < CODE_UNITS ? c0 + j : c0 + j - CODE_UNITS;
      glds_unit<FLOW>(m0 + j * WIN_SLOT_BYTES, mc + c * (uint32_t)WIN_UNIT);
    }
    rd = d % (uint32_t)WIN_UNIT;
    left = (uint32_t)WIN_DRAWS - rd;
    loaded = false;
  }
  __device__ __forceinline__ uint32_t read() const {
    const uint32_t r = rd < (uint32_t)WIN_DRAWS ? rd : 0u;  // stay inside the window
    return cell[(r / WIN_UNIT) * WIN_SLOT_BYTES + r % WIN_UNIT];
  }
  __device__ __forceinline__ void prime() {
    fill();
    primed = true;
  }
  // at least k draws available in the window (the option loops call it once per tick: a tick
  // draws at most 6 times; an auto-reset 4); refilling is rare and has one site per loop
  __device__ __forceinline__ void reserve(uint32_t k) {
    if (!primed) prime();
    if (left < k) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // no read of the old window pending
      sync();
      fill();
    }
    if (!loaded) {  // the window's DMAs must have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      nxc = read();
      loaded = true;
    }
  }
  // at least k draws staged (no refill: the plain go loop's exit test)
  __device__ __forceinline__ bool has(uint32_t k) const { return left >= k; }
  // the code dword holding draws 4d .. 4d + 3 of the window (d < WIN_DRAWS / 4)
  __device__ __forceinline__ uint32_t dword(uint32_t d) const {
    return *reinterpret_cast<const lds_u32*>(cell + (4u * d / WIN_UNIT) * WIN_SLOT_BYTES +
                                             (4u * d) % WIN_UNIT);
  }
  // walk_ticks (tg_core.h) four draws per LDS read: the codes of a dword are applied one by one
  // (each tick checks the span, the staged draws and the cap at its start, as walk_ticks), so
  // the result is walk_ticks's; the next dword is read while this one is applied
  template <int DIR>
  __device__ __forceinline__ int walk(int& x, const int lim, const int cap) {
    int taken = 0;
    if (!((DIR > 0 ? x <= lim : x >= lim) && left >= TICK_DRAWS && cap > 0)) return 0;
    uint32_t w = dword(rd >> 2);
    while (true) {
      const uint32_t wn = dword((rd >> 2) + 1u);  // inside the window: left >= TICK_DRAWS here
      const int k = (int)(rd & 3u);
      int moved = 0;
      bool act = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int st = code_step((w >> (8 * i)) & 0xFFu, DIR < 0);
        act = act && (i >= k ? ((DIR > 0 ? x <= lim : x >= lim) &&
                                left - (uint32_t)moved >= TICK_DRAWS && taken + moved < cap)
                             : true);
        if (i >= k && act) {
          x += st;
          ++moved;
        }
      }
      taken += moved;
      rd += (uint32_t)moved;
      left -= (uint32_t)moved;
      n += (uint32_t)moved;
      draws += (uint32_t)moved;
      if (moved < 4 - k) break;  // the walk stopped inside this dword
      if (!((DIR > 0 ? x <= lim : x >= lim) && left >= TICK_DRAWS && taken < cap)) break;
      w = wn;
    }
    nxc = read();  // code() reads one draw ahead
    return taken;
  }
#ifdef TG_DIAG_STAMPS
  // DIAGNOSTIC BUILD ONLY: s_memtime per phase of the option loops (tg_core.h run_option_k):
  // ph[k] sums the time of the segments ending at stamp k (1 plain walk, 2 window refill,
  // 3 full tick); rounds counts stamp 0
  unsigned long long ph[4] = {0, 0, 0, 0}, last = 0;
  uint32_t rounds = 0;
  __device__ __forceinline__ void phase(int k) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if (last) ph[k] += now - last;
    last = now;
    rounds += k == 0;
  }
#else
  __device__ __forceinline__ void phase(int) {}
#endif
  // a draw was taken past the staged window (reserve's bound broken: flagged E_WINDOW)
  __device__ __forceinline__ bool overrun() const { return left > (uint32_t)WIN_DRAWS; }
  // one draw, consumed for its outcomes (draw_code); reserve() guarantees it is in the window
  __device__ __forceinline__ uint32_t code() {
    const uint32_t c = nxc;
    ++n;
    ++draws;
    ++rd;
    --left;
    nxc = read();  // the next draw's code, one draw ahead (a byte of the window when left = 0)
    return c;
  }
  // one draw as its double (rare): the code is consumed too, the value built from the words
  // (an odd generation's twisted from the stored one before it, tg_core.h mt_pair)
  __device__ __forceinline__ double random() {
    uint32_t p = (pos >> 1) + n;
    p = 2u * (p >= (uint32_t)MT_CODES ? p - (uint32_t)MT_CODES : p);
    (void)code();
    const WordPair w = FLOW ? mt_pair_ool_sc1(mt, p) : mt_pair_ool(mt, p);
    return mt_double(w.w0, w.w1);
  }
  __device__ __forceinline__ double uniform(double a, double b) { return a + (b - a) * random(); }
  // drain the DMAs (the window is reused as scratch); returns the state word to store: the
  // entry's stale half, still stale, keeps its bits (listed or not); a half left in this launch
  // is stale and not listed yet; none, if the lane regenerated the stale half itself
  __device__ __forceinline__ uint32_t finish() {
    if (primed) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    sync();
    primed = loaded = false;
    return pos | (stale == NONE ? 0u : entered ? MT_STALE : tag);
  }
};

using RngCodes = RngCodesT<false>;

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}
// For every lane in `need`: regenerate the stale half of its env (the one not holding the
// position in its state word), one env at a time, with the whole wave (wave_twist_gens: its
// MT_HALF_GENS generations from the other half's last).  Must be reached by all 64 lanes.
__device__ __forceinline__ void wave_refill(unsigned long long need, uint32_t* env_mt, uint8_t* env_mc,
                                            uint32_t state, lds_u32* scratch) {
  const uint32_t pos = state & MT_POS_MASK;
  const uint32_t dst = (uint32_t)MT_HALF - mt_half(pos);
  const uint64_t src_l = (uint64_t)(uintptr_t)(env_mt + regen_src_off(dst));
  const uint64_t w_l = (uint64_t)(uintptr_t)env_mt;
  const uint64_t c_l = (uint64_t)(uintptr_t)env_mc;
  const int g0_l = (int)(dst / (uint32_t)MT_N);
  while (need) {
    const int L = __ffsll((long long)need) - 1;
    need &= need - 1;
    wave_twist_gens((const glb_u32*)(uintptr_t)readlane64(src_l, L),
                    (glb_u32*)(uintptr_t)readlane64(w_l, L), (uint8_t*)(uintptr_t)readlane64(c_l, L),
                    __builtin_amdgcn_readlane(g0_l, L), MT_HALF_GENS, true, scratch);
  }
}

// 64-lane sum (wave64)
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

enum { ST_STEPS, ST_VALID, ST_TICKS, ST_DRAWS, ST_EPISODES, ST_EP_OVERFLOW, ST_REGENS, ST_WTICKS,
       ST_COUNT };

// 64-lane max (wave64)
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// In-kernel span stamps of the timed launches (tg_set_timing): each wave's lane 0 folds its
// start and end (s_memrealtime: the 100 MHz constant clock) into one of KST_SLOTS
// (min start, max end) pairs of the launch's record, with returnless atomics on 64 addresses;
// flush_timing reduces them to the launch's span, first wave start to last wave end.  Null
// record: not timed (a wave-uniform branch).
constexpr int KST_SLOTS = 64;
constexpr int KST_STRIDE = 16;  // u64 per slot: each slot's pair in a 128-B line of its own
__device__ __forceinline__ unsigned long long kst_begin(const unsigned long long* ks) {
  return ks ? __builtin_amdgcn_s_memrealtime() : 0ull;
}
__device__ __forceinline__ void kst_end(unsigned long long* ks, unsigned long long t0) {
  if (ks && (threadIdx.x & 63) == 0) {
    unsigned long long* const s = ks + KST_STRIDE * (blockIdx.x % KST_SLOTS);
    atomicMin(s, t0);
    atomicMax(s + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}
#ifndef TG_FLOW_TU  // (the other kernels: the main unit only; tg_flow.hip compiles k_flow alone)
__global__ void k_kst_init(unsigned long long* ks, int64_t slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < slots) {
    ks[KST_STRIDE * i] = ~0ull;
    ks[KST_STRIDE * i + 1] = 0ull;
  }
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
// random.seed(seed0 + i): init_by_array into half 0's last stored slot (tg_core.h init_mt);
// k_gen_twist then makes the ring's 2 x MT_HALF_GENS generations from it, and k_reset (mask NULL)
// performs the constructor's game build (_TreasureGameImpl.__init__, IM/:31-53: 4 draws) —
// tg_create.
__global__ __launch_bounds__(BLOCK) void k_create(Soa S, int64_t n, uint64_t seed0,
                                                   const uint32_t* __restrict__ genrand) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  seed_mt(S.mt + i * MT_STORE + MT_SEED_OFF, genrand, seed0 + (uint64_t)i);
  Env e{};
  e.mti = 0u;
  S.st4[i] = pack(e);
  S.ang[i] = make_double2(0.0, 0.0);
  S.ep[i] = make_int2(0, 0);
}
// `gens` generations for every env, in sequence after the stored words at offset src: ring
// generations g0, g0 + 1, ... (codes; words of the even ones; tg_create, tg_write_state)
__global__ __launch_bounds__(BLOCK) void k_gen_twist(Soa S, int64_t n, uint32_t src, int g0,
                                                     int gens) {
  __shared__ __attribute__((aligned(16))) uint32_t scratch[BLOCK / 64][MT_N];
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  unsigned long long need = __ballot(i < n);
  const int64_t i0 = i - (threadIdx.x & 63);
  while (need) {
    const int L = __ffsll((long long)need) - 1;
    need &= need - 1;
    const int64_t e = i0 + L;
    wave_twist_gens((const glb_u32*)(S.mt + e * MT_STORE + src), (glb_u32*)(S.mt + e * MT_STORE),
                    S.mc + e * MT_CODES, g0, gens, false, (lds_u32*)scratch[threadIdx.x >> 6]);
  }
}

// the draw codes of the ring's first generation (stored words [0, 624)) of every env (tg_write_state)
__global__ __launch_bounds__(BLOCK) void k_gen_codes(Soa S, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i < n) gen_codes(S.mt + i * MT_STORE, S.mc + i * MT_CODES);
}

__global__ __launch_bounds__(BLOCK) void k_reset(Soa S, int64_t n, Level L,
                                                  const uint8_t* __restrict__ mask,
                                                  double* __restrict__ obs, uint32_t tstep) {
  __shared__ __attribute__((aligned(16))) uint32_t scratch[BLOCK / 64][MT_N];
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = i < n;
  const bool reset = live && (!mask || mask[i]);
  Env e;
  e.mti = 0u;
  if (live) {
    unpack(S.st4[i], S.ang[i], e);
    if (reset) {
      Rng rng(S.mt + i * MT_STORE, e.mti, S.mc + i * MT_CODES);
      reset_env(L, e, rng);
      e.mti = rng.finish();
    }
    if (obs) {
      double o[9];
      observe(L, e, o);
      store_obs(obs, i, o);
    }
  }
  const bool stale = reset && (e.mti & MT_STALE);
  wave_refill(__ballot(stale), S.mt + (live ? i : 0) * MT_STORE, S.mc + (live ? i : 0) * MT_CODES, e.mti,
              (lds_u32*)scratch[threadIdx.x >> 6]);
  if (reset) {
    e.mti &= ~(MT_STALE | MT_LISTED);
    S.st4[i] = pack(e);
    S.ang[i] = make_double2(e.ang0, e.ang1);
    S.ep[i] = make_int2(0, (int32_t)tstep);  // the episode starts with the next step
  }
}

#endif  // TG_FLOW_TU

struct StepIO {
  int32_t* __restrict__ actions;   // input; with policy >= 0 the step's actions are written here
  double* __restrict__ obs;
  int32_t* __restrict__ reward;
  uint8_t* __restrict__ valid;
  uint8_t* __restrict__ done;
  double* __restrict__ final_obs;  // may be null
  int policy;                      // -1: actions given; else TG_POLICY_* evaluated in the step
                                   // (selects the kernels' POL instantiation)
  uint64_t a0;                     // the policy's action seed and step index
  int64_t t;
  uint32_t tstep;                  // this step's index in the handle's step count (launch_step):
                                   // an episode's length is tstep + 1 - its start step (S.ep.y)
};

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// the synthetic policies (tg_policy_actions): a[t, g] = h(a0, g, t) % 9, or the k-th set bit
// of available_mask with k = h % popcount (masked-uniform; h % 9 when nothing can run)
__device__ __forceinline__ int policy_action(const Level& L, const Map& m, const Env& e,
                                             int policy, uint64_t a0, int64_t g, int64_t t) {
  const uint64_t h = sm64(sm64(a0 ^ sm64((uint64_t)g)) ^ (uint64_t)t);
  int a = (int)(h % 9ull);
  if (policy == TG_POLICY_MASKED) {
    const uint32_t mk = available_mask(L, m, e);
    const int c = __popc(mk);
    if (c) {
      uint32_t k = (uint32_t)(h % (uint64_t)c);
      uint32_t mm = mk;
      while (k--) mm &= mm - 1u;
      a = __ffs(mm) - 1;
    }
  }
  return a;
}
struct EpQueue {
  tg_episode* __restrict__ eps;
  int32_t* count;
  int32_t cap;
};

// Completed episodes (auto-reset): wavefront ballot, popcount prefix, one atomic per wave.
// The queue is drained by tg_episodes; if nobody drains it, the count must not run away (an
// int32 that wraps would turn the bound check into an out-of-bounds store): a wave whose
// records do not all fit clamps the count back to cap (atomicMin) after its add.  Between an
// add and its clamp other waves can add, so the count stays below cap + the records of the
// waves in flight (<= cap + n < 2^31 with cap <= 2^28 and n < 2^30); slots are compared
// unsigned.  The records that do not fit are counted per wave in the wave's own block slot.
// Must be reached by every lane of the wave.
__device__ __forceinline__ void record_episodes(bool mine, int64_t g, int2& ep, uint32_t tstep,
                                                const EpQueue& q, unsigned long long* stats,
                                                int64_t sl) {  // sl: the wave's stats slot
  const unsigned long long b = __ballot(mine);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  const int first = __ffsll((long long)b) - 1;
  const int cnt = __popcll(b);
  int base = 0;
  if (lane == first) {
    base = atomicAdd(q.count, cnt);
    if ((uint32_t)base + (uint32_t)cnt > (uint32_t)q.cap) {
      atomicMin(q.count, q.cap);
      const uint32_t lost = (uint32_t)base >= (uint32_t)q.cap
                                ? (uint32_t)cnt : (uint32_t)base + (uint32_t)cnt - (uint32_t)q.cap;
      atomicAdd(&stats[(size_t)sl * ST_COUNT + ST_EP_OVERFLOW], (unsigned long long)lost);
    }
  }
  base = __shfl(base, first, 64);
  if (mine) {
    const uint32_t slot = (uint32_t)base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    if (slot < (uint32_t)q.cap) {
      tg_episode r;
      r.env = g;
      r.ret = ep.x;
      r.len = (int32_t)(tstep + 1u - (uint32_t)ep.y);
      q.eps[slot] = r;
    }
    ep = make_int2(0, (int32_t)(tstep + 1u));  // the next episode starts with the next step
  }
}

// Launch counters: every step kernel has a per-block slot of `part` ([grid][ST_COUNT]) and the
// host sums the slots on demand (one counter word per launch took ~32k same-line atomics:
// ~370 us at ~88 atomics/us).  Each wave's lane 0 adds its sums into its block's slot with
// returnless atomics (no contention across blocks; no barrier, so every wave exits as soon as
// it is done).  Must be reached by every lane of the wave.
// wave_ticks: the wave's longest lane's ticks (the tick loop's trip count, lane efficiency).
__device__ __forceinline__ void wave_stats(unsigned long long* __restrict__ part, int steps,
                                           int valid, int ticks, int draws, int episodes,
                                           int regens = 0, bool wave_ticks = false,
                                           int64_t sl = -1) {  // slot: blockIdx.x by default
  // a counter that is 0 on every lane (k_run's steps / valid, most waves' episodes) skips its
  // six cross-lane steps: the reductions sit in the option waves' epilogue, on the tail
  auto sum = [](int x) { return __ballot(x != 0) ? wave_sum(x) : 0; };
  const int v[5] = {sum(steps), sum(valid), sum(ticks), sum(draws), sum(episodes)};
  const int wt = wave_ticks ? wave_max(ticks) : 0;
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* const slot = part + (size_t)(sl < 0 ? (int64_t)blockIdx.x : sl) * ST_COUNT;
#pragma unroll
    for (int c = 0; c < 5; ++c)
      if (v[c]) atomicAdd(&slot[c], (unsigned long long)v[c]);
    if (regens) atomicAdd(&slot[ST_REGENS], (unsigned long long)regens);
    if (wt) atomicAdd(&slot[ST_WTICKS], (unsigned long long)wt);
  }
}

// wave_stats for a wave whose only live lane is lane 0 (k_py1, k_serve1): lane 0's own values,
// no cross-lane reductions (~0.5 us of a one-env call)
__device__ __forceinline__ void lane0_stats(unsigned long long* __restrict__ part, int steps,
                                            int valid, int ticks, int draws, int episodes,
                                            int regens = 0, bool wave_ticks = false) {
  if ((threadIdx.x & 63) != 0) return;
  unsigned long long* const slot = part + (size_t)blockIdx.x * ST_COUNT;
  const int v[5] = {steps, valid, ticks, draws, episodes};
#pragma unroll
  for (int c = 0; c < 5; ++c)
    if (v[c]) atomicAdd(&slot[c], (unsigned long long)v[c]);
  if (regens) atomicAdd(&slot[ST_REGENS], (unsigned long long)regens);
  if (wave_ticks && ticks) atomicAdd(&slot[ST_WTICKS], (unsigned long long)ticks);
}

// finish one env-step: obs/reward/valid/done rows, episode counters, optional auto-reset.
// keep != nullptr: the obs row is returned there instead of stored (the caller stores it).
// The option waves' epilogue computes its obs rows by f64 division: the quotient table
// (tg_core.h obs_div) is a global load on their tail, and by stamps the epilogue was ~4,000
// cycles shorter without it (profiles/r04/stamps_divq_uniform_r04k.log); k_classify, whose
// waves are not a tail, keeps the table
__device__ __forceinline__ Level level_div(const Level& L) {
  Level d = L;
  d.obs_q = nullptr;
  return d;
}
// VALID: the valid row is this call's (k_classify writes every env's valid row itself, coalesced:
// k_run's scattered byte store cost a 32-B write granule per listed env)
template <bool AUTORESET, bool FINAL, bool VALID = true, class R>
__device__ __forceinline__ void finish_step(const Level& L, Env& e, R& rng, int64_t i,
                                            const StepResult& r, int2& ep, const StepIO& io,
                                            double* keep = nullptr) {
  if (rng.overrun()) e.f |= E_WINDOW;
  double o[9];
  observe(L, e, o);  // get_state (TG/:94)
  io.reward[i] = r.reward;
  if (VALID) io.valid[i] = (uint8_t)r.ran;
  io.done[i] = (uint8_t)r.done;
  ep.x += r.reward;  // (ep.y, the episode's start step, stays: no store for a reward-None step)
  if (FINAL) store_obs(io.final_obs, i, o);
  if (AUTORESET && r.done) {
    reset_env(L, e, rng);
    observe(L, e, o);
  }
  if (keep) {
#pragma unroll
    for (int k = 0; k < 9; ++k) keep[k] = o[k];
  } else {
    store_obs(io.obs, i, o);
  }
}

// The obs rows of a wave's 64 consecutive envs (4,608 B) through LDS: lane l stores the
// 8-B words l, l+64, ... of the span, so each store instruction writes 512 contiguous bytes
// (a lane storing its own 72-B row touches ~36 cache lines per instruction).  Rows of envs
// not in `mask` are left alone.  Every lane of the wave must reach it.
__device__ __forceinline__ void store_obs_wave(double* __restrict__ out, int64_t wave_first,
                                               unsigned long long mask, const double o[9],
                                               double* __restrict__ stage) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 9; ++k) stage[lane * 9 + k] = o[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double* const dst = out + wave_first * 9;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int w = j * 64 + lane;
    if ((mask >> (w / 9)) & 1ull) __builtin_nontemporal_store(stage[w], dst + w);
  }
}

// ---- one-pass step: one lane per env, the option runs in place (TG_MODE_DIRECT) ----------
constexpr int POL_IMMEDIATE = -2;  // k_step's action is io.a0 (tg_step1), not an array entry
// POL: -1 actions given; POL_IMMEDIATE one action for all (tg_step1); else the TG_POLICY_*
// evaluated here (tg_rollout).  A template
// parameter, so the per-step kernels carry none of the policy's code or registers.
// One step of env i (lane i's; live iff i < n) with the level in LDS (trig, m) and the wave's
// code window wscr: k_step's body, also k_serve1's private-stream step.  Every lane of the wave
// must reach it.
template <bool AUTORESET, bool FINAL, int POL, bool ONE = false>  // ONE: only lane 0 live (k_serve1)
__device__ __forceinline__ StepResult step_env(const Soa& S, int64_t n, const Level& L,
                                         const uint32_t* trig, const Map& m, lds_u8* wscr,
                                         int64_t i, const StepIO& io, const EpQueue& q,
                                         int64_t g0, unsigned long long* __restrict__ stats,
                                         uint32_t* __restrict__ err_or) {
  const bool live = i < n;
  StepResult r{0, 0, 0, 0};
  uint32_t draws = 0;
  int lregen = 0;  // halves this lane regenerated in its option loop
  Env e;
  e.mti = 0u;
  int2 ep = make_int2(0, 0), ep_in = ep;
  if (live) {
    unpack(S.st4[i], S.ang[i], e);
    ep = S.ep[i];
    ep_in = ep;
    RngCodes rng(S.mt + i * MT_STORE, S.mc + i * MT_CODES, e.mti, wscr);
    int act;
    if constexpr (POL >= 0) {
      act = policy_action(L, m, e, POL, io.a0, g0 + i, io.t);
      if (io.actions) io.actions[i] = act;
    } else if constexpr (POL == POL_IMMEDIATE) {
      act = (int)(int64_t)io.a0;  // tg_step1: the action is a kernel argument
    } else {
      act = io.actions[i];
    }
    r = env_step(L, trig, m, e, act, rng);
    finish_step<AUTORESET, FINAL>(level_div(L), e, rng, i, r, ep, io);
    e.mti = rng.finish();
    draws = rng.draws;
    lregen = (int)rng.regens;
    if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
  }
  // one pass, no classify pass after it: regenerate the halves left in this launch now
  const unsigned long long need = __ballot(live && (e.mti & MT_STALE));
  wave_refill(need, S.mt + (live ? i : 0) * MT_STORE,
              S.mc + (live ? i : 0) * MT_CODES, e.mti,
              (lds_u32*)wscr);
  e.mti &= ~(MT_STALE | MT_LISTED);
  if (AUTORESET) record_episodes(live && r.done, g0 + i, ep, io.tstep, q, stats, blockIdx.x);
  if (live) {
    S.st4[i] = pack(e);
    S.ang[i] = make_double2(e.ang0, e.ang1);
    if (ep.x != ep_in.x || ep.y != ep_in.y) S.ep[i] = ep;  // a reward-None step changes nothing
  }
  if constexpr (ONE)
    lane0_stats(stats, live ? 1 : 0, r.ran, r.ticks, (int)draws, AUTORESET ? (live && r.done) : 0,
                __popcll(need) + lregen, true);
  else
    wave_stats(stats, live ? 1 : 0, r.ran, r.ticks, (int)draws, AUTORESET ? (live && r.done) : 0,
               __popcll(need) + wave_sum(lregen), true);
  return r;
}

template <bool AUTORESET, bool FINAL, int POL = -1>
__global__ __launch_bounds__(BLOCK) void k_step(Soa S, int64_t n, Level L,
                                                 const uint32_t* __restrict__ grid, StepIO io,
                                                 EpQueue q, int64_t g0,
                                                 unsigned long long* __restrict__ stats,
                                                 uint32_t* __restrict__ err_or,
                                                 unsigned long long* __restrict__ ks) {
  const unsigned long long kt0 = kst_begin(ks);
  __shared__ __attribute__((aligned(16))) uint8_t win[(BLOCK / 64) * WIN_WAVE_BYTES];
  LEVEL_IN_LDS();
  lds_u8* const wscr = (lds_u8*)win + (threadIdx.x >> 6) * WIN_WAVE_BYTES;
  step_env<AUTORESET, FINAL, POL>(S, n, L, trig, m, wscr, (int64_t)blockIdx.x * BLOCK + threadIdx.x,
                                  io, q, g0, stats, err_or);
  kst_end(ks, kt0);
}

// ---- two-pass compacted step (TG_MODE_COMPACT) -------------------------------------------
// Pass 1, k_classify: one lane per env (coalesced).  Evaluates option_list[a].can_run();
// envs whose option cannot run finish here (reward None, obs/done rows written, state
// unchanged); the rest are appended to per-option worklists.  Appends are aggregated per
// workgroup in LDS and the counters are sharded 8 ways (blockIdx % 8) across cache lines (one
// word alone saturates at ~88 atomics/us, MI355X_MICROARCH.md "dequeue").
// Pass 2, k_run: wave w runs chunk w (64 envs) of the worklists concatenated in run order
// (options in kOrder, each option's 8 shards).  Only the options are padded to whole chunks
// (round 2 padded every shard), so every wave holds ONE option: a wave-uniform k selects a loop
// specialised to that option's primitive actions.  (Round 3 also tried worklists per (option,
// predicted length class), which raised lane efficiency from 0.53 to 0.84 but ran 2-5 % slower:
// DESIGN.md §3.1.)
constexpr int SHARDS = 8;  // the stale-MT-half refill lists: one per XCD (k_regen's waves of XCD x drain list x)
// the worklists' shards (k_classify's workgroup b appends to shard b % WSHARDS): each
// (option, shard) counter takes one returning atomic per workgroup that lists an env of that
// option, so more shards spread a launch's ~4k x 10 atomics over more words
#ifndef TG_WSHARDS
#define TG_WSHARDS 8
#endif
constexpr int WSHARDS = TG_WSHARDS;
// Worklists: one per option, and one (L_RESET) of the envs whose option cannot run but which
// enter the step done with auto-reset on (stepped with auto-reset off until done, then on):
// k_run resets them (reward None, no option), so k_classify carries no reset path (the gauss
// pair's f64 library code held it at 79 VGPRs, 6 waves per SIMD; without it 58, 8 waves)
constexpr int L_RESET = O_COUNT;
constexpr int NLIST = O_COUNT + 1;
constexpr int kOrderH[NLIST] = {O_JUMP_LEFT, O_JUMP_RIGHT, O_GO_LEFT,     O_GO_RIGHT,
                                O_DOWN_LEFT, O_DOWN_RIGHT, O_UP_LADDER,   O_DOWN_LADDER,
                                O_INTERACT,  L_RESET};
struct RunPos {
  int of[NLIST];  // run position of list k (kOrder's inverse)
};
constexpr RunPos make_runpos() {
  RunPos r{};
  for (int j = 0; j < NLIST; ++j) r.of[kOrderH[j]] = j;
  return r;
}
constexpr RunPos kRunPos = make_runpos();
constexpr int NSEG = NLIST * WSHARDS;  // segment = run position * WSHARDS + shard
static_assert(NSEG <= 2 * RUN_BLOCK, "k_run's prefix: two segments per thread");
constexpr int NCTR = NSEG;      // the worklist counters
constexpr int CTR_STRIDE = 32;  // counters 128 B apart
struct Work {
  int32_t* __restrict__ lists;   // [NSEG][shard_cap], segment = run position * WSHARDS + shard
  // the listed envs' state, in worklist order (written by k_classify, which has loaded it
  // anyway): k_run reads its chunk's 64 records coalesced, in one round trip with the list
  // entries, instead of a dependent gather of 16 + 16 + 8 scattered bytes per lane
  uint4* __restrict__ wst4;      // [NSEG][shard_cap]
  double2* __restrict__ wang;
  int2* __restrict__ wep;
  int32_t* __restrict__ ctr;     // [NCTR * CTR_STRIDE], this step's counters
  int32_t* __restrict__ ctr_next;  // the other parity's, zeroed here for the next step
  // stale MT halves, one list per shard (= blockIdx.x % SHARDS, the XCD), appended across the
  // pending steps: list x at refill[x * rcap ..], its length at rcnt[x * CTR_STRIDE]
  uint32_t* __restrict__ refill;  // env | source half
  int32_t* __restrict__ rcnt;
  int64_t rcap;
  int64_t shard_cap;
};
// worklist order = the order the chunks' loads reach HBM at the kernel's start (all option
// waves are resident at once and issue their loads together): the jump waves first, whose
// ticks are the slowest in wall time (~2,100 cycles each) and which end the kernel, then the
// long go walks (mean 56 ticks), drops, ladders, interact.  A/B against go
// first: 0.1366 vs 0.1400 ms.
__constant__ int kOrder[NLIST] = {O_JUMP_LEFT, O_JUMP_RIGHT, O_GO_LEFT,     O_GO_RIGHT,
                                  O_DOWN_LEFT, O_DOWN_RIGHT, O_UP_LADDER,   O_DOWN_LADDER,
                                  O_INTERACT,  L_RESET};
__constant__ int kSegBase[NLIST] = {kRunPos.of[0] * WSHARDS, kRunPos.of[1] * WSHARDS,
                                      kRunPos.of[2] * WSHARDS, kRunPos.of[3] * WSHARDS,
                                      kRunPos.of[4] * WSHARDS, kRunPos.of[5] * WSHARDS,
                                      kRunPos.of[6] * WSHARDS, kRunPos.of[7] * WSHARDS,
                                      kRunPos.of[8] * WSHARDS, kRunPos.of[9] * WSHARDS};

// 8 waves per SIMD: its 98-106 SGPRs (the level, the step's pointers) held it to 7; forced, 32-55
// of them spill to VGPR lanes (no VGPR spills, 60 VGPRs).  A/B r04r: uniform 0.1246 vs 0.1258 ms
// per step in each of 4 rounds; masked within its spread
template <bool AUTORESET, bool FINAL, int POL = -1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_classify(
    Soa S, int64_t n, Level L, const uint32_t* __restrict__ grid, StepIO io, EpQueue q, Work w,
    int64_t g0, unsigned long long* __restrict__ stats, uint32_t* __restrict__ err_or,
    unsigned long long* __restrict__ ks) {
  const unsigned long long kt0 = kst_begin(ks);
  __shared__ int bcnt[NLIST], bbase[NLIST];
  __shared__ int rwc[BLOCK / 64], rbase;  // stale halves per wave; the workgroup's list range
  // the obs staging reuses the level's LDS: nothing reads the grid after the second barrier
  // below (finish_step / reset_env use only L), so 18.4 KB instead of 20.8 KB per workgroup
  __shared__ union {
    LdsLevel lv;
    double ostage[BLOCK * 9];
  } lds;
  LdsLevel& lv = lds.lv;
  double* const ostage = lds.ostage;
  double orow[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = i < n;
  const int lane = threadIdx.x & 63;
  // every load this lane may need, issued before the level staging and the barriers so their
  // latencies overlap (the angles / episode words only matter if the option cannot run)
  uint4 s4 = make_uint4(0, 0, 0, 0);
  int32_t act = 0;
  double2 a2 = make_double2(0.0, 0.0);
  int2 ep = make_int2(0, 0);
  if (live) {
    s4 = S.st4[i];
    if constexpr (POL < 0) act = io.actions[i];
    a2 = S.ang[i];
    ep = S.ep[i];
  }
  if (threadIdx.x < NLIST) bcnt[threadIdx.x] = 0;
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < NCTR; c += BLOCK) w.ctr_next[c * CTR_STRIDE] = 0;
  stage_level(lv, grid, L);  // includes the barrier
  const Map m{reinterpret_cast<const uint8_t*>(lv.grid), L.W, L.H};
  int k = -1;
  bool runs = false;
  Env e;
  e.mti = 0u;
  if (live) {
    unpack_st4(s4, e);
    if constexpr (POL >= 0) {  // the rollout's on-device policy (tg_rollout)
      act = policy_action(L, m, e, POL, io.a0, g0 + i, io.t);
      if (io.actions) io.actions[i] = act;
    }
    k = option_index(act);
    runs = k >= 0 && can_run(L, m, e, k);
    if (k < 0) e.f |= E_ACTION;
  }
  // every env's valid row, coalesced (reward None unless its option runs; k_run writes the
  // listed envs' other rows)
  if (live) io.valid[i] = (uint8_t)runs;
  // entering done with auto-reset on and no option to run: reset in k_run (L_RESET)
  const bool rst = AUTORESET && live && !runs && is_done(e);
  const int bk = runs ? k : rst ? L_RESET : -1;  // the env's worklist
  // halves left stale and not listed yet go on this step's refill list (MT_LISTED); k_regen
  // regenerates the lists of several steps at once (a lane that needs a half first does it
  // itself: the ring leaves >= ~2,400 draws of slack, launch_step)
  // (dense lists: a drain of a few steps' lists spreads one half per wave, where the per-wave
  // regions of round 4 left a wave with the few regions holding 3-4 halves for ~0.1 ms; one
  // atomic per workgroup, beside the worklists' below: per wave, ~2,000 returning atomics per
  // counter and step at the masked policy's rate serialised k_classify, 30.8 -> 39.2 us)
  const bool stale = live && (e.mti & (MT_STALE | MT_LISTED)) == MT_STALE;
  int srank = 0;
  {
    const unsigned long long b = __ballot(stale);
    srank = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) rwc[threadIdx.x >> 6] = __popcll(b);
    if (stale) e.mti |= MT_LISTED;
  }
  // workgroup-local slots: one LDS atomic per wave and option present in the wave (the
  // wave's lanes are matched option by option)
  int slot = 0;
  {
    unsigned long long pend = __ballot(bk >= 0);
    while (pend) {
      const int first = __ffsll((long long)pend) - 1;
      const int b0 = __builtin_amdgcn_readlane(bk, first);
      const unsigned long long b = __ballot(bk == b0);
      int base = 0;
      if (lane == first) base = atomicAdd(&bcnt[b0], __popcll(b));
      base = __shfl(base, first, 64);
      if (bk == b0) slot = base + __popcll(b & ((1ull << lane) - 1ull));
      pend &= ~b;
    }
  }
  __syncthreads();
  // the workgroup's worklist ranges: issue the global atomics now, use them after the
  // reward-None envs are finished (their latency overlaps that work)
  const int shard = blockIdx.x % SHARDS, wshard = blockIdx.x % WSHARDS;
  int my_base = 0;
  if (threadIdx.x < NLIST) {
    const int c = bcnt[threadIdx.x];
    my_base = c ? atomicAdd(&w.ctr[(kSegBase[threadIdx.x] + wshard) * CTR_STRIDE], c) : 0;
  } else if (threadIdx.x == 64) {  // (another wave than the worklists' atomics)
    int c = 0;
#pragma unroll
    for (int v = 0; v < BLOCK / 64; ++v) c += rwc[v];
    my_base = c ? atomicAdd(&w.rcnt[shard * CTR_STRIDE], c) : 0;
  }
  const uint4 s4w = pack(e);  // the state the worklist copy carries (listed half, E_ACTION)

  // envs whose option cannot run: reward None, state unchanged (TG/:91-96, OP/:22-23); not
  // done, or auto-reset off (the others are k_run's, L_RESET)
  const bool fin = live && !runs && !rst;
  if (fin) {
    e.ang0 = a2.x;
    e.ang1 = a2.y;
    Rng rng(S.mt + i * MT_STORE, e.mti, S.mc + i * MT_CODES);  // no draws without a reset
    StepResult r{0, 0, (int)is_done(e), 0};
    finish_step<false, FINAL, false>(L, e, rng, i, r, ep, io, orow);
    if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
  }
  const int2 ep_in = ep;
  store_obs_wave(io.obs, i - lane, __ballot(fin), orow, ostage + (threadIdx.x & ~63) * 9);
  if (fin) {
    const uint4 s4n = pack(e);
    if (s4n.x != s4.x || s4n.y != s4.y || s4n.z != s4.z || s4n.w != s4.w) {  // reset / flag
      S.st4[i] = s4n;
      S.ang[i] = make_double2(e.ang0, e.ang1);
    }
    // reward None: the return and the episode's start step are unchanged unless it ended
    if (ep.x != ep_in.x || ep.y != ep_in.y) S.ep[i] = ep;
  }
  if (threadIdx.x < NLIST) bbase[threadIdx.x] = my_base;
  if (threadIdx.x == 64) rbase = my_base;
  __syncthreads();
  if (stale) {
    int at = rbase + srank;
    for (int v = 0; v < (int)(threadIdx.x >> 6); ++v) at += rwc[v];
    w.refill[shard * w.rcap + at] = (uint32_t)i | (mt_half(e.mti & MT_POS_MASK) ? 0x80000000u : 0u);
  }
  if (bk >= 0) {
    const int64_t at = (int64_t)(kSegBase[bk] + wshard) * w.shard_cap + bbase[bk] + slot;
    w.lists[at] = (int32_t)i;
    w.wst4[at] = s4w;
    w.wang[at] = a2;
    w.wep[at] = ep;
  }
  wave_stats(stats, live ? 1 : 0, runs ? 1 : 0, 0, 0, 0);
  kst_end(ks, kt0);
}

#ifdef TG_DIAG_STAMPS
// DIAGNOSTIC BUILD ONLY (scripts/diag_stamps.py): per-wave s_memtime stamps of k_run
constexpr int NSTAMP = 11;
// per wave: 4 durations/counts, 100 MHz start and end, the option loop's phases (walk, refill,
// full tick: lane 0's sums) and rounds
constexpr int NSTAMP_WAVES = 1 << 17;
__device__ unsigned long long g_stamps[NSTAMP_WAVES * NSTAMP];
#define TG_STAMP(v) v = __builtin_amdgcn_s_memtime()
#else
#define TG_STAMP(v) (void)0
#endif

template <bool AUTORESET, bool FINAL>
__global__ __launch_bounds__(RUN_BLOCK) void k_run(Soa S, int64_t n, Level L,
                                                const uint32_t* __restrict__ grid, StepIO io,
                                                EpQueue q, Work w, int64_t g0,
                                                unsigned long long* __restrict__ stats,
                                                uint32_t* __restrict__ err_or,
                                                unsigned long long* __restrict__ ks) {
  const unsigned long long kt0 = kst_begin(ks);
  // the worklists in run order: pre[s] = envs listed before segment s (exclusive prefix of the
  // counters, two segments per thread), then per option (run order j) its first segment's
  // prefix and its start in the chunk space, where each option is padded to whole chunks
  __shared__ int pre[NSEG + 1];
  __shared__ int wtot[RUN_BLOCK / 64];
  __shared__ int ostart[NLIST + 1], oraw[NLIST + 1];
  {
    const int s0 = 2 * (int)threadIdx.x, ln = threadIdx.x & 63;
    const int c0 = s0 < NSEG ? w.ctr[s0 * CTR_STRIDE] : 0;
    const int c1 = s0 + 1 < NSEG ? w.ctr[(s0 + 1) * CTR_STRIDE] : 0;
    int v = c0 + c1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (ln >= o) v += y;
    }
    if (ln == 63) wtot[threadIdx.x >> 6] = v;
    __syncthreads();
    for (int wv = 0; wv < (int)(threadIdx.x >> 6); ++wv) v += wtot[wv];
    const int excl = v - c0 - c1;
    if (s0 < NSEG) pre[s0] = excl;
    if (s0 + 1 < NSEG) pre[s0 + 1] = excl + c0;
    if (threadIdx.x == RUN_BLOCK - 1) pre[NSEG] = v;
  }
  __syncthreads();
  // a workgroup past every listed chunk (the grid covers n envs, a uniform step lists ~1 in 5;
  // the options' padding adds < 64 each) leaves before it stages the level: ~3/4 of the grid
  if ((int)(blockIdx.x * RUN_BLOCK) >= pre[NSEG] + NLIST * 63) {
    kst_end(ks, kt0);
    return;
  }
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int j = 0; j < NLIST; ++j) {
      const int sb = j * WSHARDS, se = sb + WSHARDS;
      ostart[j] = acc;
      oraw[j] = pre[sb];
      acc += (pre[se] - pre[sb] + 63) & ~63;
    }
    ostart[NLIST] = acc;
    oraw[NLIST] = pre[NSEG];
  }
  RUN_LEVEL_IN_LDS();  // includes the barrier (ostart / oraw)
  const int total = ostart[NLIST];
  const int base = (blockIdx.x * RUN_BLOCK + threadIdx.x) & ~63;  // wave w runs chunk w
  int oj = 0;  // ostart[oj] <= base < ostart[oj + 1] (wave-uniform)
  while (oj + 1 < NLIST && ostart[oj + 1] <= base) ++oj;
  oj = __builtin_amdgcn_readfirstlane(oj);
  const int k = kOrder[oj];
  // this lane's place in option k's lists (the raw prefix's coordinates), and its segment
  const int qraw = oraw[oj] + base + (threadIdx.x & 63) - ostart[oj];
  const bool live = base < total && qraw < oraw[oj + 1];
  int seg = oj * WSHARDS;
  if (live) {
    int hi = seg + WSHARDS;  // pre[seg] <= qraw < pre[hi]
    while (hi - seg > 1) {
      const int mid = (seg + hi) >> 1;
      if (pre[mid] <= qraw) seg = mid; else hi = mid;
    }
  }
  const int idx = qraw - pre[seg];
  int64_t i = 0;
  StepResult r{0, 0, 0, 0};
  Env e;
  e.mti = 0u;
  int2 ep = make_int2(0, 0);
  uint32_t draws = 0;
  int regens = 0;  // wave-uniform
  int lregen = 0;  // halves this lane regenerated in its option loop
  lds_u8* const wscr = (lds_u8*)win + (threadIdx.x >> 6) * WIN_WAVE_BYTES;
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  TG_STAMP(t0);
#ifdef TG_DIAG_STAMPS
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  (void)t0; (void)t1; (void)t2; (void)t3;
#ifdef TG_DIAG_STAMPS
  unsigned long long ph1 = 0, ph2 = 0, ph3 = 0;
  uint32_t prounds = 0;
#endif
  if (live) {
    const int64_t at = (int64_t)seg * w.shard_cap + idx;
    i = w.lists[at];
    unpack(w.wst4[at], w.wang[at], e);
    ep = w.wep[at];
    RngCodes rng(S.mt + i * MT_STORE, S.mc + i * MT_CODES, e.mti, wscr);
    rng.prime();  // issue the code loads now; the first draw comes after the policy setup
    TG_STAMP(t1);
    if (k != O_GO_LEFT && k != O_GO_RIGHT && k != O_INTERACT) __builtin_amdgcn_s_setprio(PRIO_SLOW);
    // k is wave-uniform: one specialised loop; L_RESET's envs run none (reward None)
    if (k != L_RESET) run_option(L, trig, m, e, k, rng, r);
    TG_STAMP(t2);
#ifdef TG_DIAG_STAMPS
    ph1 = rng.ph[1], ph2 = rng.ph[2], ph3 = rng.ph[3], prounds = rng.rounds;
#endif
    r.done = is_done(e);
    finish_step<AUTORESET, FINAL, false>(level_div(L), e, rng, i, r, ep, io);  // valid: k_classify's
    e.mti = rng.finish();  // a half left here: MT_STALE, listed by the next k_classify
    draws = rng.draws;
    lregen = (int)rng.regens;
    if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
  }
  // (k_run's grid has BLOCK / RUN_BLOCK workgroups per stats slot, as wave_stats below)
  if (AUTORESET)
    record_episodes(live && r.done, g0 + i, ep, io.tstep, q, stats, (int64_t)blockIdx.x / (BLOCK / RUN_BLOCK));
  if (live) {
    S.st4[i] = pack(e);
    S.ang[i] = make_double2(e.ang0, e.ang1);
    S.ep[i] = ep;
  }
  __builtin_amdgcn_s_setprio(0);
  wave_stats(stats, 0, 0, r.ticks, (int)draws, AUTORESET ? (live && r.done) : 0,
             regens + (__ballot(lregen != 0) ? wave_sum(lregen) : 0), true,
             (int64_t)blockIdx.x / (BLOCK / RUN_BLOCK));
  kst_end(ks, kt0);
#ifdef TG_DIAG_STAMPS
  TG_STAMP(t3);
  {
    int mx = r.ticks;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    const int sum = wave_sum(r.ticks);
    const unsigned long long bl = __ballot(live);
    const int src = bl ? __ffsll((long long)bl) - 1 : 0;
    const unsigned long long a1 = __shfl(t1, src, 64);
    const unsigned long long a2 = __shfl(t2, src, 64);
    const int wv = (blockIdx.x * RUN_BLOCK + threadIdx.x) >> 6;
    const unsigned long long rt3 = __builtin_amdgcn_s_memrealtime();
    // the phases of the lane whose option loop ran longest (the wave's own time)
    int lmax = src;
    unsigned long long best = 0;
    for (int l = 0; l < 64; ++l) {
      const unsigned long long tl = __shfl(ph1 + ph2 + ph3, l, 64);
      if (((bl >> l) & 1ull) && tl > best) best = tl, lmax = l;
    }
    const unsigned long long p1 = __shfl(ph1, lmax, 64), p2 = __shfl(ph2, lmax, 64),
                             p3 = __shfl(ph3, lmax, 64);
    const uint32_t pr = __shfl(prounds, lmax, 64);
    if ((threadIdx.x & 63) == 0 && wv < NSTAMP_WAVES) {
      unsigned long long* const g = g_stamps + (size_t)wv * NSTAMP;
      // an idle wave (no listed chunk) is option 15 with 1 iteration
      g[0] = bl ? a1 - t0 : 0;
      g[1] = bl ? a2 - a1 : 0;
      g[2] = bl ? t3 - a2 : t3 - t0;
      g[3] = bl ? (unsigned long long)mx | ((unsigned long long)sum << 32) | ((unsigned long long)k << 56)
                : 1ull | (15ull << 56);
      g[4] = rt0;
      g[5] = rt3;
      g[6] = p1;
      g[7] = p2;
      g[8] = p3;
      g[9] = pr;
      g[10] = (unsigned long long)regens;  // halves this wave regenerated from the queue
    }
  }
#endif
}

// ---- deferred regeneration of the listed stale MT halves (k_regen) ----------------------------
// k_classify appends the halves the previous step left stale (MT_STALE) to its shard's refill
// list and marks them MT_LISTED; every REGEN_STEPS compact steps (and on tg_regenerate) k_regen
// regenerates every pending entry with a full-occupancy grid and no option loops beside it: the
// waves of XCD x (blockIdx.x % 8) take list x's entries, an even share each (the halves cost
// the same: MT_HALF_GENS twists), the rest from the list's counter.  An entry is regenerated iff
// its env's state word still says MT_STALE (its lane may have regenerated the half itself, or
// crossed again since): the half not holding the position, from the last generation of the one
// holding it.  The word loses MT_STALE | MT_LISTED by an atomic AND before the twist (the
// claim: of several entries for one env, one regenerates).  It runs alone on the stream, so
// nothing else touches the state meanwhile.
// Slack: a listed half is needed again only after the env consumes the rest of the half it is
// in, >= MT_HALF / 2 - (one step's draws) ~ 2,400 draws, more than REGEN_STEPS steps draw on the
// default level (<= ~110 per step); a lane that gets there first regenerates the half itself.
constexpr int REGEN_STEPS = 16;
// regen_ctr, per set: the 8 grab counters, then the 8 list lengths (k_classify's rcnt)
constexpr int RCTR_LIST = 8;
constexpr int RCTR_N = 16;
#ifndef TG_FLOW_TU  // (the other kernels: the main unit only; tg_flow.hip compiles k_flow alone)
// k_regen's ring stores: non-temporal (its words and codes are read steps later, not by this
// launch) with TG_REGEN_NT=1
#ifndef TG_REGEN_NT
#define TG_REGEN_NT 0
#endif
constexpr bool REGEN_NT = TG_REGEN_NT != 0;
__global__ __launch_bounds__(BLOCK) void k_regen(Soa S, const uint32_t* __restrict__ refill,
                                                 int64_t rcap, int32_t* __restrict__ ctr,
                                                 int32_t* __restrict__ ctr_next,
                                                 unsigned long long* __restrict__ stats,
                                                 int nstat, unsigned long long* __restrict__ ks) {
  const unsigned long long kt0 = kst_begin(ks);
  __shared__ __attribute__((aligned(16))) uint32_t scratch[BLOCK / 64][MT_N];
  lds_u32* const scr = (lds_u32*)scratch[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  const int xcd = (int)(blockIdx.x & 7u);
  const int64_t cnt = ctr[(RCTR_LIST + xcd) * CTR_STRIDE];
  if (blockIdx.x == 0 && threadIdx.x < RCTR_N) ctr_next[threadIdx.x * CTR_STRIDE] = 0;
  int32_t* const q = ctr + xcd * CTR_STRIDE;
  const uint32_t* const list = refill + xcd * rcap;
  uint32_t* const st_w = reinterpret_cast<uint32_t*>(S.st4);  // word 4i + 3: env i's MT word
  auto src_of = [&](uint32_t env, uint32_t s) {
    const uint32_t dst = (uint32_t)MT_HALF - mt_half(s & MT_POS_MASK);
    return (const glb_u32*)(S.mt + (int64_t)env * MT_STORE + regen_src_off(dst));
  };
  // this wave's index among its XCD's waves; the first grab is static (an even share, at most
  // 64: one entry per lane), the rest come from the counter, which starts past the static ones
  const int wx = (int)(blockIdx.x >> 3) * (BLOCK / 64) + (int)(threadIdx.x >> 6);
  const int64_t nwx = (int64_t)((gridDim.x - (unsigned)xcd + 7u) >> 3) * (BLOCK / 64);
  int64_t grab = (cnt + nwx - 1) / nwx;
  if (grab > 64) grab = 64;
  if (grab < 1) grab = 1;
  int halves = 0;
  bool first = true;
  while (true) {
    int64_t j0 = (int64_t)wx * grab;
    if (!first) {
      int g = 0;
      if (lane == 0) g = atomicAdd(q, (int)grab);
      j0 = nwx * grab + __builtin_amdgcn_readfirstlane(g);
    }
    first = false;
    if (j0 >= cnt) break;
    const int64_t m = cnt - j0 < grab ? cnt - j0 : grab;
    const uint32_t env_l = lane < m ? list[j0 + lane] & 0x7FFFFFFFu : 0u;
    // claim: clear MT_STALE | MT_LISTED and regenerate only if this lane's clear found
    // MT_STALE.  An env can be listed twice before a drain (its lane regenerated the listed
    // half itself, crossed again, and the next k_classify listed the new stale half): both
    // entries name the half not holding the position, and the second claim finds it clean
    // (round 4 regenerated such a half once per entry: 20,320 vs 15,360 halves on the corridor
    // level).  Entries of one grab for one env are serialised at the word's L2 channel.
    const uint32_t st_l = lane < m ? atomicAnd(&st_w[(int64_t)env_l * 4 + 3], ~(MT_STALE | MT_LISTED)) : 0u;
    unsigned long long need = __ballot(lane < m && (st_l & MT_STALE));
    // one half at a time: 52 VGPRs, 8 waves per SIMD (the next half's source loads pipelined
    // into this one's twist took 76 VGPRs, 6 waves, and measured no faster: DESIGN.md §3.3)
    while (need) {
      const int L = __ffsll((long long)need) - 1;
      need &= need - 1;
      const uint32_t env = __builtin_amdgcn_readlane(env_l, L), s = __builtin_amdgcn_readlane(st_l, L);
      const uint32_t dst = (uint32_t)MT_HALF - mt_half(s & MT_POS_MASK);
      TwistIn t;
      twist_load(src_of(env, s), t);
      twist_chain<REGEN_NT>(t, (glb_u32*)(S.mt + (int64_t)env * MT_STORE), S.mc + (int64_t)env * MT_CODES,
                            (int)(dst / (uint32_t)MT_N), MT_HALF_GENS, true, scr);
      ++halves;
    }
  }
  // the grid can exceed the stats slots (>= 8 workgroups, one per XCD counter, at small n)
  if (lane == 0 && halves)
    atomicAdd(&stats[(size_t)(blockIdx.x % (unsigned)nstat) * ST_COUNT + ST_REGENS],
              (unsigned long long)halves);
  kst_end(ks, kt0);
}

#endif  // TG_FLOW_TU

#include "tg_flow.h"

#ifndef TG_FLOW_TU  // (the other kernels: the main unit only; tg_flow.hip compiles k_flow alone)
__global__ __launch_bounds__(BLOCK) void k_mask(Soa S, int64_t n, Level L,
                                                 const uint32_t* __restrict__ grid,
                                                 uint16_t* __restrict__ out) {
  LEVEL_IN_LDS();
  (void)trig;
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  Env e;
  unpack(S.st4[i], S.ang[i], e);
  out[i] = (uint16_t)available_mask(L, m, e);
}

__global__ __launch_bounds__(BLOCK) void k_observe(Soa S, int64_t n, Level L,
                                                    double* __restrict__ obs) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  Env e;
  unpack(S.st4[i], S.ang[i], e);
  double o[9];
  observe(L, e, o);
  store_obs(obs, i, o);
}

// a[t, g] = h(a0, g, t) % 9, or the k-th set bit of available_mask (masked-uniform)
__global__ __launch_bounds__(BLOCK) void k_actions(Soa S, int64_t n, Level L,
                                                    const uint32_t* __restrict__ grid,
                                                    uint64_t a0, int64_t g0, int64_t t,
                                                    int policy, int32_t* __restrict__ out) {
  __shared__ LdsLevel lv;
  if (policy == TG_POLICY_MASKED) stage_level(lv, grid, L);  // uniform branch
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const Map m{reinterpret_cast<const uint8_t*>(lv.grid), L.W, L.H};
  Env e{};
  if (policy == TG_POLICY_MASKED) unpack(S.st4[i], S.ang[i], e);
  out[i] = policy_action(L, m, e, policy, a0, g0 + i, t);
}

// move up to `cap` completed-episode records to `out`, keep the rest queued (device only,
// so the per-step episode gather never waits on the host)
__global__ __launch_bounds__(BLOCK) void k_drain_episodes(tg_episode* __restrict__ eps,
                                                           int32_t* eps_count, int32_t eps_cap,
                                                           tg_episode* __restrict__ out,
                                                           int32_t* __restrict__ count,
                                                           int32_t cap) {
  int32_t n = *eps_count;
  if ((uint32_t)n > (uint32_t)eps_cap) n = eps_cap;  // see record_episodes: never above cap + n
  const int32_t m = n < cap ? n : cap;
  for (int32_t k = threadIdx.x; k < m; k += BLOCK) out[k] = eps[k];
  __syncthreads();
  for (int32_t base = m; base < n; base += BLOCK) {  // shift the remainder down in chunks
    const int32_t k = base + threadIdx.x;
    tg_episode r;
    if (k < n) r = eps[k];
    __syncthreads();
    if (k < n) eps[k - m] = r;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *eps_count = n - m;
    *count = m;
  }
}

// The six collision predicates (IM/:232-288) at every pixel of [x0, x1) x [y0, y1) with the
// doors closed per door_bits, bit order as the reference's predicate listing: up_clear, can_go_up,
// can_go_down, can_go_left, can_go_right, can_fall.  The device build of Map (mul24 / div48
// take the __umul24 path only here), pinned against the reference's F2 truth tables.
__global__ __launch_bounds__(BLOCK) void k_predicates(Level L, const uint32_t* __restrict__ grid,
                                                       int x0, int x1, int y0, int y1,
                                                       uint32_t door_bits,
                                                       uint8_t* __restrict__ out) {
  LEVEL_IN_LDS();
  (void)trig;
  const int64_t w = x1 - x0;
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= w * (int64_t)(y1 - y0)) return;
  Env e{};
  e.px = x0 + (int)(i % w);
  e.py = y0 + (int)(i / w);
  e.f = (door_bits & 7u) << F_OBJ;
  out[i] = (uint8_t)((unsigned)m.up_clear(e) | (unsigned)m.can_go_up(e) << 1 |
                     (unsigned)m.can_go_down(e) << 2 | (unsigned)m.can_go_side(e, -1) << 3 |
                     (unsigned)m.can_go_side(e, +1) << 4 | (unsigned)m.can_fall(e) << 5);
}

// tg_read_state's MT part: the generation holding each env's position (CPython's mt[]),
// envs [first, first + count) -> dst [count][624] (contiguous), 4 words per lane (an odd
// generation's twisted from the stored one before it)
__global__ __launch_bounds__(BLOCK) void k_gather_mt(Soa S, int64_t first, int64_t count,
                                                      uint32_t* __restrict__ dst) {
  constexpr int Q = MT_N / 4;  // 156 uint4 per generation
  const int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (t >= count * Q) return;
  const int64_t k = t / Q;
  const int q = (int)(t - k * Q);
  const int64_t i = first + k;
  const uint32_t g = (S.st4[i].w & MT_POS_MASK) / (uint32_t)MT_N;
  const uint32_t* const mt = S.mt + i * MT_STORE;
  uint4 v;
  if (g & 1u) {
    const uint32_t* const prev = mt + mt_store_off(g - 1u);
    v = make_uint4(twist_at(prev, 4 * q), twist_at(prev, 4 * q + 1), twist_at(prev, 4 * q + 2),
                   twist_at(prev, 4 * q + 3));
  } else {
    v = reinterpret_cast<const uint4*>(mt + mt_store_off(g))[q];
  }
  reinterpret_cast<uint4*>(dst)[t] = v;
}

// ---- the N=1 drop-in over a Python-level random stream (tg_step1_py / tg_reset1_py) ---------
// One wave.  The stream's generation (tg_pystate: random.getstate()'s 624 words + index) is read
// from pinned host memory into LDS with its two successors (twisted by the wave), lane 0 runs the
// step / reset with a PyRng over them, and the wave writes back the generation holding the
// stream's new position, so the caller's random.setstate continues exactly where CPython's
// would: any index, odd ones too (the twist is a recurrence on consecutive words, so words are
// read by absolute position across generations), and gauss_next carried in and out.
constexpr int PY_GENS = 3;  // generations held in LDS; a 4th+ is twisted in place by lane 0
struct PyRng {
  uint32_t* w;     // LDS: PY_GENS slots of MT_N words, generation g in slot (g + off) % PY_GENS
  uint32_t q;      // absolute word position (generation g holds positions [g*624, g*624 + 624))
  uint32_t lo;     // oldest generation held
  uint32_t draws;
  uint32_t off;    // the ring's rotation (k_serve1 keeps the ring in LDS across calls)
  // the generation holding the next word, its slot and the word's index there (set up at the
  // first draw; a draw crosses into the next generation only every 312 draws)
  uint32_t gc = 0u, qi = 0u;
  const uint32_t* cs = nullptr;
  __device__ __forceinline__ uint32_t* slot(uint32_t g) const { return w + ((g + off) % PY_GENS) * MT_N; }
  __device__ __forceinline__ const uint32_t* gen(uint32_t g) {
    while (g >= lo + PY_GENS) {  // > 2 generations in one call (long levels): twist in place
      twist_gen(slot(lo + PY_GENS - 1), slot(lo));
      ++lo;
    }
    return slot(g);
  }
  __device__ __forceinline__ uint32_t next_word() {
    if (qi == (uint32_t)MT_N) {
      cs = gen(++gc);
      qi = 0u;
    }
    return cs[qi++];
  }
  __device__ __forceinline__ double random() {
    if (!cs) {
      gc = q / MT_N;
      qi = q - gc * MT_N;
      cs = gen(gc);
    }
    uint32_t a, b;
    if (qi + 2u <= (uint32_t)MT_N) {  // both words in the current generation
      a = cs[qi];
      b = cs[qi + 1u];
      qi += 2u;
    } else {
      a = next_word();
      b = next_word();
    }
    q += 2;
    ++draws;
    return mt_double(a, b);
  }
  __device__ __forceinline__ double uniform(double a, double b) { return a + (b - a) * random(); }
  __device__ __forceinline__ uint32_t code() { return draw_code(random()); }
  __device__ __forceinline__ void reserve(uint32_t) {}
  __device__ __forceinline__ bool has(uint32_t) const { return true; }
  __device__ __forceinline__ bool overrun() const { return false; }
  __device__ __forceinline__ void phase(int) {}
  template <int DIR>
  __device__ __forceinline__ int walk(int& x, int lim, int cap) { return walk_ticks<DIR>(*this, x, lim, cap); }
};
// dst = twist_gen(src) with the 64 lanes of the (only) wave, both in LDS
__device__ __forceinline__ void lds_twist64(const uint32_t* src, uint32_t* dst) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int r = 0; r < (MT_N + 63) / 64; ++r) {
    const int p = r * 64 + lane;
    if (p < MT_N) {
      const uint32_t b = p + 1 < MT_N ? src[p + 1] : dst[0];
      const uint32_t c = p < MT_N - MT_M ? src[p + MT_M] : dst[p - (MT_N - MT_M)];
      dst[p] = mt_twist(src[p], b, c);
    }
    __syncthreads();
  }
}
// lane 0 runs the call (a step of `action`, or RESET) over the ring W, where generation j of the
// caller's stream (j = 0: the one tg_pystate holds; q0 its index) sits in slot (j + off) % 3.
// On return py holds the state after the call: its index and gauss_next, and the generation's
// words when the generation changed (otherwise py's words already are the generation's); the
// ring holds the new generation and its two successors, off updated to match.  Returns the new
// generation's number (0: unchanged).  Every lane of the (one-wave) workgroup must reach it.
template <bool RESET>
__device__ __forceinline__ uint32_t py_call(const Soa& S, const Level& L, const LdsLevel& lv,
                                            uint32_t* W, uint32_t& off, int action,
                                            tg_pystate* py, uint32_t q0, int has_gauss,
                                            double gauss_next, TgOne* out, uint32_t tstep,
                                            unsigned long long* __restrict__ stats,
                                            uint32_t* __restrict__ err_or, int* ticks = nullptr,
                                            const uint32_t* mk = nullptr,
                                            unsigned long long* stamps = nullptr) {
  __shared__ uint32_t out_g, out_lo, out_idx;
  const int lane = threadIdx.x;
  StepResult r{0, 0, 0, 0};
  uint32_t draws = 0;
  if (lane == 0) {
    const Map m{reinterpret_cast<const uint8_t*>(lv.grid), L.W, L.H, mk};
    PyRng rng{W, q0, 0u, 0u, off};
    Env e;
    unpack(S.st4[0], S.ang[0], e);
    int2 ep = S.ep[0];
    double o[9];
    if (stamps) stamps[0] = __builtin_amdgcn_s_memrealtime();
    if (RESET) {
      GaussNext g{has_gauss != 0, gauss_next};
      reset_env_gauss(L, e, rng, g);
      py->has_gauss = g.has ? 1u : 0u;
      py->gauss_next = g.has ? g.v : 0.0;
      ep = make_int2(0, (int32_t)tstep);  // the episode starts with the next step
    } else {
      r = env_step(L, lv.trig, m, e, action, rng);
      ep.x += r.reward;  // (ep.y: the episode's start step)
    }
    if (stamps) stamps[1] = __builtin_amdgcn_s_memrealtime();
    observe(level_div(L), e, o);  // by f64 division, as k_run (the table's loads: 0.48 us)
    if (stamps) stamps[2] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 9; ++k) out->obs[k] = o[k];
    out->reward = r.reward;
    out->valid = (uint8_t)r.ran;
    out->done = (uint8_t)r.done;
    S.st4[0] = pack(e);
    S.ang[0] = make_double2(e.ang0, e.ang1);
    S.ep[0] = ep;
    if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
    // CPython's state after the last word read: its generation and the index past it
    const uint32_t g = rng.q == q0 ? 0u : (rng.q - 1u) / MT_N;
    out_g = g;
    out_lo = rng.lo;
    out_idx = rng.q == q0 ? q0 : rng.q - g * MT_N;
    draws = rng.draws;
  }
  __syncthreads();
  if (stamps && lane == 0) stamps[3] = __builtin_amdgcn_s_memrealtime();
  const uint32_t g = out_g;
  if (g != 0u) {  // the caller's generation changed
    const uint32_t* src = W + ((g + off) % PY_GENS) * MT_N;
    for (int i = lane; i < MT_N; i += 64) py->mt[i] = src[i];
    // the ring: generations g, g + 1, g + 2 (it holds out_lo .. out_lo + 2, g among them; the
    // missing successors are twisted over generations older than g)
    for (uint32_t hi = out_lo + PY_GENS - 1; hi < g + PY_GENS - 1; ++hi)
      lds_twist64(W + ((hi + off) % PY_GENS) * MT_N, W + ((hi + 1 + off) % PY_GENS) * MT_N);
    off = (off + g) % PY_GENS;
  }
  if (lane == 0) py->index = out_idx;
  lane0_stats(stats, !RESET ? 1 : 0, r.ran, r.ticks, (int)draws, 0);
  if (ticks) *ticks = r.ticks;
  if (stamps && lane == 0) stamps[4] = __builtin_amdgcn_s_memrealtime();
  return g;
}
// the ring from the caller's state (py, pinned host memory): its generation and two successors
__device__ __forceinline__ void py_ring_cold(uint32_t* W, const tg_pystate* py) {
  for (int i = threadIdx.x; i < MT_N; i += 64) W[i] = py->mt[i];
  __syncthreads();
  lds_twist64(W, W + MT_N);
  lds_twist64(W + MT_N, W + 2 * MT_N);
}
__device__ __forceinline__ void py_level(LdsLevel& lv, const Level& L, const uint32_t* __restrict__ grid) {
  const int nwords = ((L.W + 2 * PAD) * (L.H + 2 * PAD) + 3) / 4;
  for (int i = threadIdx.x; i < nwords; i += 64) lv.grid[i] = grid[i];
  if (threadIdx.x < 12) lv.trig[threadIdx.x] = L.trig[threadIdx.x >> 1][threadIdx.x & 1];
}
// The Python stream's generation and its two successors, kept on the device between calls
// (tg_batch::pyc, generation j in slot j): cache_in is it when the caller's state is the one the
// last call returned (the host compares them), else null and the ring is built from the
// caller's state.  q0 / gauss: the caller's index and gauss_next, as kernel arguments (no
// host-memory reads in the common case).  On return py holds the state after the call and
// cache_out the new generation and its two successors.
template <bool RESET>
__global__ __launch_bounds__(64) void k_py1(Soa S, Level L, const uint32_t* __restrict__ grid,
                                            int action, tg_pystate* py, const uint32_t* cache_in,
                                            uint32_t* cache_out, uint32_t q0, int has_gauss,
                                            double gauss_next, TgOne* out, uint32_t tstep,
                                            unsigned long long* __restrict__ stats,
                                            uint32_t* __restrict__ err_or) {
  __shared__ uint32_t W[PY_GENS * MT_N];
  __shared__ LdsLevel lv;
  const int lane = threadIdx.x;
  py_level(lv, L, grid);
  if (cache_in) {
    for (int i = lane; i < PY_GENS * MT_N; i += 64) W[i] = cache_in[i];
    __syncthreads();
  } else {
    py_ring_cold(W, py);
  }
  uint32_t off = 0;
  const uint32_t g = py_call<RESET>(S, L, lv, W, off, action, py, q0, has_gauss, gauss_next, out,
                                    tstep, stats, err_or);
  if (g != 0u || !cache_in)
    for (int j = 0; j < PY_GENS; ++j)
      for (int i = lane; i < MT_N; i += 64) cache_out[j * MT_N + i] = W[((j + off) % PY_GENS) * MT_N + i];
}

// ---- the N = 1 server (tg_batch::serve) ------------------------------------------------------
// One wave, resident for a 1-env handle's tg_step1 / tg_step1_py / tg_step1_pywords /
// tg_reset1_py / tg_available_mask1: it polls the
// mailbox's seq (a system-scope load of pinned host memory), serves a new command with the same
// device code as k_step<POL_IMMEDIATE> / k_py1 (step_env, py_call), writes the result row and
// the stream state into pinned host memory, releases them at system scope and then stores
// done = seq, which the host spins on.  The level, the env's state and the Python stream's ring
// (rotated by off) stay in LDS between commands (the private stream's code window is primed
// afresh by each step, as in k_step).  Every lane leaves together, on SRV_QUIT or
// after `idle` ticks of s_memrealtime (100 MHz) without a command; a leaving server writes the
// ring to pyc (generation j in slot j), where the next server or k_py1 finds it.
__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
// Resident for many commands, the server keeps in LDS what a step would otherwise fetch from
// HBM each time: the env's state (st4 / ang / ep: written back to HBM when it leaves), the level
// bitmasks and, when it fits (`stage`: dynamic LDS, sized at launch), the GoTable.  (get_state
// divides, as k_run: no quotient table.)
constexpr uint32_t SRV_STAGE_GOTAB = 1u;
__global__ __launch_bounds__(64) void k_serve1(Soa Sg, Level Lg, const uint32_t* __restrict__ grid,
                                               SrvBox* box, tg_pystate* py, uint32_t* pyc,
                                               TgOne* out, EpQueue q, int64_t g0, uint32_t idle,
                                               int trace, uint32_t stage,
                                               unsigned long long* __restrict__ stats,
                                               uint32_t* __restrict__ err_or) {
  __shared__ __attribute__((aligned(16))) uint8_t win[WIN_WAVE_BYTES];
  __shared__ uint32_t W[PY_GENS * MT_N];
  __shared__ LdsLevel lv;
  __shared__ uint4 st4_l;
  __shared__ double2 ang_l;
  __shared__ int2 ep_l;
  __shared__ uint32_t mk_l[MK_MAX_WORDS];  // the level bitmasks (Map::mk), as k_run's
  extern __shared__ __attribute__((aligned(16))) uint8_t srv_dyn[];
  const int lane = threadIdx.x;
  py_level(lv, Lg, grid);
  if (Lg.masks)
    for (int i = lane; i < mk_words(Lg.W, Lg.H); i += 64) mk_l[i] = Lg.masks[i];
  const uint32_t* const mk = Lg.masks ? mk_l : nullptr;
  Level L = Lg;
  if (stage & SRV_STAGE_GOTAB) {
    uint32_t* const gd = reinterpret_cast<uint32_t*>(srv_dyn);
    const int ng = Lg.W * Lg.H * 32;
    for (int i = lane; i < ng; i += 64) gd[i] = Lg.gotab[i];
    L.gotab = gd;
  }
  if (lane == 0) {
    st4_l = Sg.st4[0];
    ang_l = Sg.ang[0];
    ep_l = Sg.ep[0];
  }
  __syncthreads();
  const Soa S{&st4_l, &ang_l, &ep_l, Sg.mt, Sg.mc};
  const Map m{reinterpret_cast<const uint8_t*>(lv.grid), L.W, L.H, mk};
  bool ring = false;  // W holds the Python stream's ring
  uint32_t off = 0;
  uint32_t served = sys_load(&box->done);
  unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
  __shared__ TgOne row_l;  // the command's result row, written to host memory in one burst
  __shared__ unsigned long long phase_l[5];  // TG_SERVE_TRACE: py_call's phase stamps
  TgOne* const row = &row_l;
  while (true) {
    // the command group in one load (volatile: system scope, no cache)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 cg = *reinterpret_cast<const volatile u32x4*>(box);
    const uint32_t s = __builtin_amdgcn_readfirstlane(cg.w);
    if (s == served) {
      if (__builtin_amdgcn_s_memrealtime() - t_last > idle) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // what the host wrote before seq
    const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
    int ticks = 0;
    const uint32_t word = __builtin_amdgcn_readfirstlane(cg.x);
    const uint32_t kind = word & 15u;
    if (kind == SRV_QUIT) {
      served = s;
      break;
    }
    const int action = (int)((word >> 4) & 31u) - 16;
    const uint32_t tstep = __builtin_amdgcn_readfirstlane(cg.y);
    if (kind == SRV_MASK) {  // available_mask (TG/:83-89), as k_mask
      if (lane == 0) {
        Env e;
        unpack(S.st4[0], S.ang[0], e);
        box->mask = available_mask(L, m, e);
      }
    } else if (kind == SRV_RESET) {  // reset() on the env's own stream, as k_reset
      Env e;
      e.mti = 0u;
      if (lane == 0) {
        unpack(S.st4[0], S.ang[0], e);
        Rng rng(S.mt, e.mti, S.mc);
        reset_env(L, e, rng);
        e.mti = rng.finish();
        double o[9];
        observe(level_div(L), e, o);
#pragma unroll
        for (int k = 0; k < 9; ++k) row->obs[k] = o[k];
        row->reward = 0;
        row->valid = 0;
        row->done = 0;
      }
      wave_refill(__ballot(lane == 0 && (e.mti & MT_STALE)), S.mt, S.mc, e.mti, (lds_u32*)win);
      if (lane == 0) {
        e.mti &= ~(MT_STALE | MT_LISTED);
        S.st4[0] = pack(e);
        S.ang[0] = make_double2(e.ang0, e.ang1);
        S.ep[0] = make_int2(0, (int32_t)tstep);  // the episode starts with the next step
      }
    } else if (kind == SRV_STEP) {
      const StepIO io{nullptr, row->obs, &row->reward, &row->valid, &row->done, nullptr,
                      POL_IMMEDIATE, (uint64_t)(int64_t)action, 0, tstep};
      ticks = step_env<false, false, POL_IMMEDIATE, true>(S, 1, L, lv.trig, m, (lds_u8*)win, lane, io,
                                                          q, g0, stats, err_or).ticks;
    } else {
      const bool warm = (word >> 9) & 1u;
      const int has_gauss = (int)((word >> 10) & 1u);
      const uint32_t q0 = word >> 11;
      double gauss_next = 0.0;
      if (kind == SRV_RESET_PY) {
        const uint32_t* gp = reinterpret_cast<const uint32_t*>(&box->gauss_bits);
        gauss_next = __builtin_bit_cast(double, (uint64_t)sys_load(gp) | (uint64_t)sys_load(gp + 1) << 32);
      }
      if (!ring || !warm) {  // a new server, or draws on the stream since the last call
        if (warm) {
          for (int i = lane; i < PY_GENS * MT_N; i += 64) W[i] = pyc[i];
          __syncthreads();
        } else {
          py_ring_cold(W, py);
        }
        off = 0;
        ring = true;
      }
      if (kind == SRV_RESET_PY)
        py_call<true>(S, L, lv, W, off, 0, py, q0, has_gauss, gauss_next, row, tstep, stats, err_or,
                      &ticks, mk);
      else
        py_call<false>(S, L, lv, W, off, action, py, q0, has_gauss, gauss_next, row, tstep, stats,
                       err_or, &ticks, mk, trace ? phase_l : nullptr);
    }
    __syncthreads();
    if (kind != SRV_MASK && lane < (int)(sizeof(TgOne) / 8))
      reinterpret_cast<uint64_t*>(out)[lane] = reinterpret_cast<const uint64_t*>(row)[lane];
    // the row and the state (host memory; the env's state and MT ring in HBM for the next
    // command) before the answer
    if (trace && lane == 0) {
      box->t_seen = t_seen;
      box->t_end = __builtin_amdgcn_s_memrealtime();
      box->ticks = (uint32_t)ticks;
      for (int j = 0; j < 5; ++j) box->phase[j] = kind == SRV_STEP_PY ? phase_l[j] : 0ull;
    }
    __syncthreads();  // (the release below covers the row the lanes wrote: one wave)
    if (lane == 0) __hip_atomic_store(&box->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    served = s;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (ring)
    for (int j = 0; j < PY_GENS; ++j)
      for (int i = lane; i < MT_N; i += 64) pyc[j * MT_N + i] = W[((j + off) % PY_GENS) * MT_N + i];
  __syncthreads();
  if (lane == 0) {
    Sg.st4[0] = st4_l;
    Sg.ang[0] = ang_l;
    Sg.ep[0] = ep_l;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (lane == 0) __hip_atomic_store(&box->done, served, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// tg_probe_dispatch: nothing (a dependent kernel boundary's cost alone)
__global__ __launch_bounds__(BLOCK) void k_null() {}

__global__ __launch_bounds__(BLOCK) void k_errors(const uint4* __restrict__ st4, int64_t n,
                                                   uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t f = i < n ? (st4[i].y & E_MASK) : 0u;
  if (f) atomicOr(out, f);
}
#endif  // TG_FLOW_TU

}  // namespace

// k_flow<AR, POL> is instantiated in its own translation unit, tg_flow.hip, which is built
// without MachineLICM (the pass hoisted values out of the flow's work loop and
// held them live across it, 123-182 VGPRs; without it 121-129, 4 waves per SIMD)
namespace tg {
const void* flow_kernel(bool ar, int pol);
}

#ifndef TG_FLOW_TU

namespace {
int grid_for(int64_t n) { return (int)((n + BLOCK - 1) / BLOCK); }
// k_run needs one wave per 64-lane chunk of the worklists, each option padded to whole chunks:
// at most n/64 + NLIST chunks (idle blocks interleaved among the option blocks, so that MT
// regenerations start at once, measured no faster for the masked policy and slower for the
// uniform one: DESIGN.md §3.3)
int run_grid_for(int64_t n) { return grid_for(n) + (NLIST * 64 + BLOCK - 1) / BLOCK; }
// one launch-counter slot per workgroup of the widest step launch (k_run)
int stat_slots(int64_t n) { return run_grid_for(n); }

// Timing (tg_set_timing): the kernels of a sampled step launch (and every k_regen launch while
// timing is on) fold their in-kernel span stamps into the launch's record (kst_end): no event or
// other packet goes on the stream.  Records: KST_MAX step samples (two kernels each) and KST_MAX
// k_regen launches, KST_SLOTS slots per kernel.
constexpr int KST_MAX = 512;
constexpr int64_t KST_KSLOTS = (int64_t)KST_MAX * 3 * KST_SLOTS;  // slots of all records
unsigned long long* kst_step(tg_batch* h, int k, int kernel) {
  return h->kst + ((size_t)k * 2 + kernel) * KST_STRIDE * KST_SLOTS;
}
unsigned long long* kst_regen(tg_batch* h, int k) {
  return h->kst + ((size_t)KST_MAX * 2 + k) * KST_STRIDE * KST_SLOTS;
}
int kst_reset(tg_batch* h) {  // every record to (no start, no end)
  if (!h->kst && hipMalloc((void**)&h->kst, sizeof(unsigned long long) * KST_STRIDE * KST_KSLOTS) !=
                     hipSuccess)
    return fail(TG_E_NOMEM, "timing records");
  hipLaunchKernelGGL(k_kst_init, dim3((unsigned)((KST_KSLOTS + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0,
                     h->kst, KST_KSLOTS);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  h->kst_steps = 0;
  h->kst_regens = 0;
  h->kst_k.clear();
  return TG_OK;
}
// a kernel record's span in ms (first wave start to last wave end; 0 if it never ran)
double kst_span_ms(const unsigned long long* rec) {
  unsigned long long t0 = ~0ull, t1 = 0ull;
  for (int j = 0; j < KST_SLOTS; ++j) {
    if (rec[KST_STRIDE * j] < t0) t0 = rec[KST_STRIDE * j];
    if (rec[KST_STRIDE * j + 1] > t1) t1 = rec[KST_STRIDE * j + 1];
  }
  return t1 > t0 ? (double)(t1 - t0) * 1e-5 : 0.0;  // 100 MHz ticks
}
int flush_timing(tg_batch* h) {
  if (!h->kst_steps && !h->kst_regens) return TG_OK;
  HIP_TRY(hipDeviceSynchronize());
  std::vector<unsigned long long> rec((size_t)KST_STRIDE * KST_KSLOTS);
  HIP_TRY(hipMemcpy(rec.data(), h->kst, sizeof(unsigned long long) * rec.size(), hipMemcpyDeviceToHost));
  const size_t kr = (size_t)KST_STRIDE * KST_SLOTS;  // u64 per kernel record
  for (int k = 0; k < h->kst_steps; ++k) {
    const double c = kst_span_ms(rec.data() + (k * 2 + 0) * kr), r = kst_span_ms(rec.data() + (k * 2 + 1) * kr);
    h->classify_ms_done += c;
    h->run_ms_done += r;
    h->kernel_ms_done += c + r;
    h->timed_launches += k < (int)h->kst_k.size() ? h->kst_k[(size_t)k] : 1;  // k_flow: K steps
  }
  for (int k = 0; k < h->kst_regens; ++k) {
    h->regen_ms_done += kst_span_ms(rec.data() + ((size_t)KST_MAX * 2 + k) * kr);
    ++h->regen_timed;
  }
  return kst_reset(h);
}
// whether this step launch is sampled; if so ks0 / ks1 are its kernels' records
bool timing_begin(tg_batch* h, int& rc, unsigned long long*& ks0, unsigned long long*& ks1) {
  rc = TG_OK;
  ks0 = ks1 = nullptr;
  if (!h->timing_every || (h->timing_calls++ % (uint64_t)h->timing_every) != 0) return false;
  if (h->kst_steps >= KST_MAX && (rc = flush_timing(h))) return false;
  ks0 = kst_step(h, h->kst_steps, 0);
  ks1 = kst_step(h, h->kst_steps, 1);
  ++h->kst_steps;
  h->kst_k.push_back(1);
  return true;
}


// a stepper's buffers for envs [off, off + n) (StepCtx)
int alloc_ctx(StepCtx& c, int64_t off, int64_t n) {
  c.off = off;
  c.n = n;
#define ALLOC_C(ptr, bytes)                                             \
  if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess)                \
    return fail(TG_E_NOMEM, "hipMalloc %zu B for " #ptr, (size_t)(bytes));
  ALLOC_C(c.stats, sizeof(unsigned long long) * ST_COUNT * (size_t)stat_slots(n));
  // a worklist shard holds the envs of every WSHARDS-th workgroup; a refill list those of every
  // SHARDS-th, REGEN_STEPS steps of them
  c.shard_cap = (int64_t)((grid_for(n) + WSHARDS - 1) / WSHARDS) * BLOCK;
  ALLOC_C(c.wl, sizeof(int32_t) * NSEG * (size_t)c.shard_cap);
  ALLOC_C(c.wst4, sizeof(uint4) * NSEG * (size_t)c.shard_cap);
  ALLOC_C(c.wang, sizeof(double2) * NSEG * (size_t)c.shard_cap);
  ALLOC_C(c.wep, sizeof(int2) * NSEG * (size_t)c.shard_cap);
  ALLOC_C(c.wctr, sizeof(int32_t) * 2 * NCTR * CTR_STRIDE);
  // a shard's list holds at most its workgroups' envs per pending step
  c.rcap = (int64_t)((grid_for(n) + SHARDS - 1) / SHARDS) * BLOCK * REGEN_STEPS;
  ALLOC_C(c.refill, sizeof(uint32_t) * SHARDS * (size_t)c.rcap);
  ALLOC_C(c.regen_ctr, sizeof(int32_t) * 2 * RCTR_N * CTR_STRIDE);
#undef ALLOC_C
  HIP_TRY(hipMemset(c.stats, 0, sizeof(unsigned long long) * ST_COUNT * (size_t)stat_slots(n)));
  HIP_TRY(hipMemset(c.wctr, 0, sizeof(int32_t) * 2 * NCTR * CTR_STRIDE));
  HIP_TRY(hipMemset(c.regen_ctr, 0, sizeof(int32_t) * 2 * RCTR_N * CTR_STRIDE));
  return TG_OK;
}
void free_ctx(StepCtx& c) {
  void* bufs[] = {c.stats, c.wl, c.wst4, c.wang, c.wep, c.wctr, c.refill, c.regen_ctr};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c.ev) (void)hipEventDestroy(c.ev);
  if (c.st) (void)hipStreamDestroy(c.st);
  c = StepCtx{};
}
}  // namespace

namespace {
void flow_free(tg_batch* h);  // TG_MODE_FLOW's buffers (below)
}

extern "C" {

const char* tg_last_error(void) { return tg::g_err.c_str(); }
const char* tg_version(void) { return "tg_amd 0.1 gfx950"; }
int64_t tg_num_envs(const tg_batch* h) { return h ? h->n : 0; }

int tg_create(tg_batch** out, int64_t n, uint64_t seed_base, int64_t global_offset, int device,
              const char* dom, const char* objs, const char* inter) {
  if (!out || n <= 0 || global_offset < 0) return fail(TG_E_INVAL, "tg_create: bad arguments");
  // every env's seed seed_base + global_offset + i must be a 64-bit init_by_array key
  if ((uint64_t)global_offset > ~seed_base || (uint64_t)(n - 1) > ~(seed_base + (uint64_t)global_offset))
    return fail(TG_E_INVAL, "tg_create: seed_base + global_offset + num_envs - 1 exceeds 2^64 - 1");
  *out = nullptr;
  if (!dom && !objs && !inter) {
    dom = kDefaultDomain;
    objs = kDefaultObjects;
    inter = kDefaultInteractions;
  } else if (!dom || !objs || !inter) {
    return fail(TG_E_INVAL, "tg_create: give all three level texts or none");
  }
  Level L;
  std::vector<uint8_t> grid;
  std::string perr;
  if (parse_level(dom, objs, inter, L, grid, perr)) return fail(TG_E_INVAL, "%s", perr.c_str());
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(TG_E_NODEV, "tg_create: no HIP device %d (found %d)", device, ndev);
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(TG_E_NODEV, "tg_create: device %d is %s, this build targets gfx950", device,
                prop.gcnArchName);

  tg_batch* h = new tg_batch();
  h->device = device;
  h->cus = prop.multiProcessorCount;
  h->n = n;
  h->g0 = global_offset;
  h->seed0 = seed_base;
  h->domain = dom;
  h->flow_debug = getenv("TG_FLOW_DEBUG") != nullptr;
  if (const char* sp = getenv("TG_FLOW_SKIP_PART")) h->flow_skip = atoi(sp);
  if (const char* sv = getenv("TG_SERVE")) h->serve = atoi(sv) != 0;
  h->srv_trace = getenv("TG_SERVE_TRACE") != nullptr;
  // the server's idle limit: 500 us by default (a stream it shares a hardware queue with waits
  // at most this long behind it)
  const char* si = getenv("TG_SERVE_IDLE_US");
  h->srv_idle = 100u * (uint32_t)std::min(std::max(si ? atoi(si) : 500, 1), 1000000);
  // completed-episode queue: drained by tg_episodes; records beyond it are counted as dropped
  const int64_t cap = 4 * n > (1 << 16) ? 4 * n : (1 << 16);
  h->eps_cap = (int32_t)(cap < (1 << 28) ? cap : (1 << 28));
  auto cleanup = [&](int code) {
    tg_destroy(h);
    return code;
  };
  uint32_t gen[MT_N];
  gen[0] = 19650218u;  // init_genrand(19650218) — the common prefix of init_by_array
  for (int i = 1; i < MT_N; ++i) gen[i] = 1812433253u * (gen[i - 1] ^ (gen[i - 1] >> 30)) + (uint32_t)i;
#define ALLOC(ptr, bytes)                                                                   \
  if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess)                                    \
    return cleanup(fail(TG_E_NOMEM, "hipMalloc %zu B for " #ptr, (size_t)(bytes)));
  grid.resize((grid.size() + 3) & ~(size_t)3, 0);
  ALLOC(h->grid, grid.size());
  ALLOC(h->genrand, sizeof gen);
  const std::vector<uint32_t> gotab = build_gotab(L, grid);
  ALLOC(h->gotab, sizeof(uint32_t) * gotab.size());
  L.gotab = h->gotab;
  const std::vector<uint32_t> masks = build_masks(L, grid);
  if (!masks.empty()) ALLOC(h->masks, sizeof(uint32_t) * masks.size());
  L.masks = h->masks;
  const std::vector<double> obs_q = build_obs_q(L);
  ALLOC(h->obs_q, sizeof(double) * obs_q.size());
  L.obs_q = h->obs_q;
  h->L = L;
  ALLOC(h->S.st4, sizeof(uint4) * n);
  ALLOC(h->S.ang, sizeof(double2) * n);
  ALLOC(h->S.ep, sizeof(int2) * n);
  ALLOC(h->S.mt, sizeof(uint32_t) * MT_STORE * (size_t)n);
  ALLOC(h->S.mc, sizeof(uint8_t) * MT_CODES * (size_t)n);
  ALLOC(h->eps, sizeof(tg_episode) * (size_t)h->eps_cap);
  ALLOC(h->eps_count, sizeof(int32_t));
  ALLOC(h->err, sizeof(uint32_t));
#undef ALLOC
  if (const int rc = alloc_ctx(h->main, 0, n)) return cleanup(rc);
  if (hipMemcpy(h->grid, grid.data(), grid.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->genrand, gen, sizeof gen, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->gotab, gotab.data(), sizeof(uint32_t) * gotab.size(), hipMemcpyHostToDevice) != hipSuccess ||
      (h->masks && hipMemcpy(h->masks, masks.data(), sizeof(uint32_t) * masks.size(),
                             hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(h->obs_q, obs_q.data(), sizeof(double) * obs_q.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(h->eps_count, 0, sizeof(int32_t)) != hipSuccess ||
      hipMemset(h->err, 0, sizeof(uint32_t)) != hipSuccess)
    return cleanup(fail(TG_E_HIP, "tg_create: upload failed"));
  // seed -> generation 1 (first half) -> generation 2 (second half) -> the constructor's draws
  hipLaunchKernelGGL(k_create, dim3(grid_for(n)), dim3(BLOCK), 0, 0, h->S, n,
                     seed_base + (uint64_t)global_offset, h->genrand);
  hipLaunchKernelGGL(k_gen_twist, dim3(grid_for(n)), dim3(BLOCK), 0, 0, h->S, n,
                     MT_SEED_OFF, 0, 2 * MT_HALF_GENS);
  hipLaunchKernelGGL(k_reset, dim3(grid_for(n)), dim3(BLOCK), 0, 0, h->S, n, h->L,
                     (const uint8_t*)nullptr, (double*)nullptr, 0u);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) return cleanup(fail(TG_E_HIP, "k_create: %s", hipGetErrorString(e)));
  *out = h;
  return TG_OK;
}

void tg_destroy(tg_batch* h) {
  if (!h) return;
  int cur = -1;
  if (hipGetDevice(&cur) == hipSuccess && cur != h->device) (void)hipSetDevice(h->device);
  if (h->srv_live) (void)srv_stop(h);
  srv_register(h, false);
  if (h->srv_trace && h->srv_calls)
    fprintf(stderr, "[serve] calls %lld launches %lld: mean per call %.2f us to post, %.2f us post -> "
            "answer, of which %.2f us between the server's pickup and its answer\n",
            (long long)h->srv_calls, (long long)h->srv_launches, h->srv_post_ns / h->srv_calls / 1e3,
            h->srv_rt_ns / h->srv_calls / 1e3, h->srv_gpu_ns / h->srv_calls / 1e3);
  if (h->srv_trace && h->srv_calls > 2) {  // server time = a + b * ticks (least squares)
    const double n = (double)h->srv_calls, sk = h->srv_fit[0], skk = h->srv_fit[1];
    const double sg = h->srv_gpu_ns, sgk = h->srv_fit[2];
    const double b = (n * sgk - sk * sg) / (n * skk - sk * sk), a = (sg - b * sk) / n;
    fprintf(stderr, "[serve] ticks per command %.2f; server time = %.2f us + %.3f us x ticks "
            "(GoTable in LDS: %d, %zu B)\n", sk / n, a / 1e3, b / 1e3, h->srv_stage, h->srv_dyn);
    if (h->srv_phase_n)
      fprintf(stderr, "[serve] py steps %lld, mean us: pickup -> option %.3f, option %.3f, observe "
              "%.3f, -> barrier %.3f, -> py_call return %.3f, -> answer %.3f\n",
              (long long)h->srv_phase_n, h->srv_phase[0] / h->srv_phase_n / 1e3,
              h->srv_phase[1] / h->srv_phase_n / 1e3, h->srv_phase[2] / h->srv_phase_n / 1e3,
              h->srv_phase[3] / h->srv_phase_n / 1e3, h->srv_phase[4] / h->srv_phase_n / 1e3,
              h->srv_phase[5] / h->srv_phase_n / 1e3);
  }
  if (h->srv_ev) (void)hipEventDestroy(h->srv_ev);
  if (h->srv_dep) (void)hipEventDestroy(h->srv_dep);
  if (h->srv_st) (void)hipStreamDestroy(h->srv_st);
  if (h->box) (void)hipHostFree(h->box);
  render_free(h->rs);
  flow_free(h);
  void* bufs[] = {h->grid, h->genrand, h->gotab, h->masks, h->obs_q, h->S.st4, h->S.ang, h->S.ep,
                  h->S.mt, h->S.mc, h->eps, h->eps_count, h->err, h->obs_scratch, h->kst};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  free_ctx(h->main);
  for (auto& c : h->grp) free_ctx(c);
  if (h->fork) (void)hipEventDestroy(h->fork);
  if (h->one) (void)hipHostFree(h->one);
  if (h->py) (void)hipHostFree(h->py);
  if (h->mask1) (void)hipHostFree(h->mask1);
  if (h->pyc) (void)hipFree(h->pyc);
  delete h;
}

int tg_reset(tg_batch* h, const uint8_t* mask, double* obs, void* stream) {
  BIND(h);
  hipLaunchKernelGGL(k_reset, dim3(grid_for(h->n)), dim3(BLOCK), 0, (hipStream_t)stream, h->S,
                     h->n, h->L, mask, obs, h->tstep);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

}  // extern "C"

namespace {
// k_regen over the pending refill-list slots (timed with its own event pair when timing is on)
// a stepper's envs as a Soa view (StepCtx: envs [off, off + n) of the handle)
Soa soa_of(const tg_batch* h, const StepCtx& c) {
  return Soa{h->S.st4 + c.off, h->S.ang + c.off, h->S.ep + c.off, h->S.mt + c.off * (int64_t)MT_STORE,
             h->S.mc + c.off * (int64_t)MT_CODES};
}
int launch_regen(tg_batch* h, StepCtx& c, hipStream_t st) {
  if (!c.rpend) return TG_OK;
  unsigned long long* ks = nullptr;
  if (h->timing_every && &c == &h->main) {
    if (h->kst_regens >= KST_MAX) {
      const int rc = flush_timing(h);
      if (rc) return rc;
    }
    ks = kst_regen(h, h->kst_regens++);
  }
  // Workgroups take list regions from the counter of their XCD (blockIdx.x % 8) until it runs
  // out, so the grid needs at least 8 of them (one per counter; fewer would leave the regions
  // of the missing counters undone) and no more than are resident at once (a second round
  // would find the counters exhausted and only pay its launch).  Block b adds its halves to
  // stats slot b % stat_slots.  The counters alternate between two sets by launch parity: each
  // launch zeroes the other set for the next one (no memset launch).
  if (!h->regen_per_cu) {
    int nb = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k_regen),
                                                         BLOCK, 0));
    h->regen_per_cu = nb > 0 ? nb : 1;
  }
  // (the lists' lengths are on the device: the grid is sized for ~0.25 entries per env and step,
  // 64 per wave)
  const int64_t bound = ((c.n + 63) >> 6) * c.rpend;
  int64_t grid = (int64_t)h->cus * h->regen_per_cu;
  if (grid > (bound + 3) / 4) grid = (bound + 3) / 4;  // 4 waves per workgroup
  if (grid < 8) grid = 8;
  int32_t* const cur = c.regen_ctr + c.regen_parity * RCTR_N * CTR_STRIDE;
  int32_t* const nxt = c.regen_ctr + (c.regen_parity ^ 1) * RCTR_N * CTR_STRIDE;
  c.regen_parity ^= 1;
  hipLaunchKernelGGL(k_regen, dim3((unsigned)grid), dim3(BLOCK), 0, st, soa_of(h, c), c.refill,
                     c.rcap, cur, nxt, c.stats, stat_slots(c.n), ks);
  HIP_TRY(hipGetLastError());
  c.rpend = 0;
  ++h->regen_launches;
  return TG_OK;
}
// one step's kernels for a stepper's envs on `st` (io: the whole handle's arrays; the stepper's
// rows start at c.off), their spans sampled when timing is on (the handle's own stepper only)
int launch_step(tg_batch* h, StepCtx& c, const StepIO& io_in, bool ar, hipStream_t st,
                uint32_t tstep, hipEvent_t mid = nullptr) {
  StepIO io = io_in;
  io.tstep = tstep;
  if (c.off) {
    if (io.actions) io.actions += c.off;
    io.obs += c.off * 9;
    io.reward += c.off;
    io.valid += c.off;
    io.done += c.off;
    if (io.final_obs) io.final_obs += c.off * 9;
  }
  const bool fo = io.final_obs != nullptr;
  int rc = TG_OK;
  unsigned long long *ks0 = nullptr, *ks1 = nullptr;
  if (&c == &h->main || &c == h->grp.data()) timing_begin(h, rc, ks0, ks1);
  if (rc) return rc;
  const EpQueue q{h->eps, h->eps_count, h->eps_cap};
  const dim3 grid(grid_for(c.n)), block(BLOCK);
  const Soa S = soa_of(h, c);
  const int64_t g0 = h->g0 + c.off;
  if (h->mode == TG_MODE_DIRECT) {
    decltype(&k_step<true, true>) kern;
    if (io.policy == TG_POLICY_UNIFORM)
      kern = ar ? (fo ? k_step<true, true, 0> : k_step<true, false, 0>)
                : (fo ? k_step<false, true, 0> : k_step<false, false, 0>);
    else if (io.policy == TG_POLICY_MASKED)
      kern = ar ? (fo ? k_step<true, true, 1> : k_step<true, false, 1>)
                : (fo ? k_step<false, true, 1> : k_step<false, false, 1>);
    else
      kern = ar ? (fo ? k_step<true, true> : k_step<true, false>)
                : (fo ? k_step<false, true> : k_step<false, false>);
    hipLaunchKernelGGL(kern, grid, block, 0, st, S, c.n, h->L, h->grid, io, q, g0, c.stats, h->err,
                       ks1);
  } else {
    // counters double-buffered by step parity: k_classify zeroes the next step's set (the
    // previous k_run, which read it, has finished), so no memset launch per step
    int32_t* const cur = c.wctr + (c.parity ? NCTR * CTR_STRIDE : 0);
    int32_t* const nxt = c.wctr + (c.parity ? 0 : NCTR * CTR_STRIDE);
    c.parity ^= 1;
    // the refill lists append until k_regen drains them (every REGEN_STEPS steps), counted in
    // the set the next k_regen reads
    const Work w{c.wl,     c.wst4, c.wang, c.wep, cur, nxt, c.refill,
                 c.regen_ctr + (c.regen_parity * RCTR_N + RCTR_LIST) * CTR_STRIDE, c.rcap,
                 c.shard_cap};
    decltype(&k_classify<true, true>) kc;
    if (io.policy == TG_POLICY_UNIFORM)
      kc = ar ? (fo ? k_classify<true, true, 0> : k_classify<true, false, 0>)
              : (fo ? k_classify<false, true, 0> : k_classify<false, false, 0>);
    else if (io.policy == TG_POLICY_MASKED)
      kc = ar ? (fo ? k_classify<true, true, 1> : k_classify<true, false, 1>)
              : (fo ? k_classify<false, true, 1> : k_classify<false, false, 1>);
    else
      kc = ar ? (fo ? k_classify<true, true> : k_classify<true, false>)
              : (fo ? k_classify<false, true> : k_classify<false, false>);
    auto kr = ar ? (fo ? k_run<true, true> : k_run<true, false>)
                 : (fo ? k_run<false, true> : k_run<false, false>);
    hipLaunchKernelGGL(kc, grid, block, 0, st, S, c.n, h->L, h->grid, io, q, w, g0, c.stats, h->err,
                       ks0);
    HIP_TRY(hipGetLastError());
    if (mid) HIP_TRY(hipEventRecord(mid, st));  // (tg_rollout's stagger between groups)
    hipLaunchKernelGGL(kr, dim3(run_grid_for(c.n) * (BLOCK / RUN_BLOCK)), dim3(RUN_BLOCK), 0, st, S,
                       c.n, h->L, h->grid, io, q, w,
                       g0, c.stats, h->err, ks1);
  }
  HIP_TRY(hipGetLastError());
  if (h->mode != TG_MODE_DIRECT && ++c.rpend == REGEN_STEPS) return launch_regen(h, c, st);
  return TG_OK;
}
// every stepper's pending refill lists drained on `st` (the groups' lists name halves the
// handle's own k_classify will not list again, and the reverse)
int regen_all(tg_batch* h, hipStream_t st) {
  int rc = launch_regen(h, h->main, st);
  for (auto& c : h->grp)
    if (!rc) rc = launch_regen(h, c, st);
  return rc;
}

// ---- TG_MODE_FLOW (tg_flow.h) ----------------------------------------------------------------
void flow_free(tg_batch* h) {
  auto& F = h->fl;
  void* bufs[] = {F.ctl[0], F.ctl[1], F.q[0], F.q[1], F.fill[0], F.fill[1], F.list, F.outst};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  F = {};
}
// the XCD census (sub-problems) and the work structures, at the first flow rollout
int flow_init(tg_batch* h) {
  auto& F = h->fl;
  if (F.ready) return TG_OK;
  uint32_t* dmask = nullptr;
  if (hipMalloc((void**)&dmask, sizeof(uint32_t)) != hipSuccess) return fail(TG_E_NOMEM, "flow census");
  uint32_t mask = 0;
  hipError_t e = hipMemset(dmask, 0, sizeof(uint32_t));
  if (e == hipSuccess) {
    // several workgroups per CU: every XCD of the device gets some (dispatch is round-robin)
    hipLaunchKernelGGL(k_census, dim3((unsigned)(h->cus * 8)), dim3(64), 0, 0, dmask);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(&mask, dmask, sizeof mask, hipMemcpyDeviceToHost);
  (void)hipFree(dmask);
  if (e != hipSuccess) return fail(TG_E_HIP, "flow census: %s", hipGetErrorString(e));
  mask &= 0xFFu;
  F.P = 0;
  F.xmap = 0xFFFFFFFFu;
  for (int id = 0; id < 8; ++id)
    if ((mask >> id) & 1u) F.xmap = (F.xmap & ~(0xFu << (4 * id))) | ((uint32_t)F.P++ << (4 * id));
  if (F.P == 0) return fail(TG_E_HIP, "flow census: no XCC id in 0..7");
  if (h->flow_debug) fprintf(stderr, "[flow] census mask %08x P %d\n", mask, F.P);
  const int64_t C = (h->n + 63) / 64, cxm = (C + F.P - 1) / F.P;
  if (C > 0xFFFFFF) return fail(TG_E_INVAL, "flow mode: at most 2^24 chunks of 64 envs");
  F.C = (int32_t)C;
  F.lcap = cxm * 64;
  F.jcap = cxm + 1;
  F.qcap = (int64_t)FLOW_MAX_K * (2 * cxm + NLIST);  // run items + chunks to classify, per step
  const size_t nctl = (size_t)F.P * CTL_WORDS, nq = (size_t)F.P * F.qcap,
               nfill = (size_t)F.P * FLOW_MAX_K * NLIST * F.jcap,
               nlist = (size_t)F.P * FLOW_MAX_K * NLIST * F.lcap;
  bool ok = true;
  for (int k = 0; k < 2; ++k)
    ok = ok && hipMalloc((void**)&F.ctl[k], sizeof(int32_t) * nctl) == hipSuccess &&
         hipMalloc((void**)&F.q[k], sizeof(uint32_t) * nq) == hipSuccess &&
         hipMalloc((void**)&F.fill[k], sizeof(int32_t) * nfill) == hipSuccess &&
         hipMemset(F.ctl[k], 0, sizeof(int32_t) * nctl) == hipSuccess &&
         hipMemset(F.q[k], 0xFF, sizeof(uint32_t) * nq) == hipSuccess &&
         hipMemset(F.fill[k], 0, sizeof(int32_t) * nfill) == hipSuccess;
  ok = ok && hipMalloc((void**)&F.list, sizeof(int32_t) * nlist) == hipSuccess &&
       hipMalloc((void**)&F.outst, sizeof(int32_t) * (size_t)C) == hipSuccess;
  if (!ok) {
    flow_free(h);
    return fail(TG_E_NOMEM, "flow work structures (%zu MB of lists)", nlist * 4 >> 20);
  }
  HIP_TRY(hipDeviceSynchronize());
  F.ready = true;
  return TG_OK;
}
// k steps (<= FLOW_MAX_K) of the handle's own stepper in one k_flow launch; outputs at step s0
// of the rollout's [K][N] arrays
int launch_flow(tg_batch* h, int k, const FlowIO& io, bool ar, int pol, hipStream_t st) {
  auto& F = h->fl;
  StepCtx& c = h->main;
  // the MT slack (k_regen every REGEN_STEPS steps): drain first if these steps would overrun it
  if (c.rpend + k > REGEN_STEPS) {
    const int rc = launch_regen(h, c, st);
    if (rc) return rc;
  }
  const void* const kern = tg::flow_kernel(ar, pol);
  int& bpc = F.bpc[ar ? 1 : 0][pol ? 1 : 0];
  if (!bpc) {
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kern, BLOCK, 0));
    if (bpc < 1) bpc = 1;
  }
  unsigned long long* ks = nullptr;
  if (h->timing_every && (h->timing_calls++ % (uint64_t)h->timing_every) == 0) {
    if (h->kst_steps >= KST_MAX) {
      const int rc = flush_timing(h);
      if (rc) return rc;
    }
    ks = kst_step(h, h->kst_steps, 1);
    ++h->kst_steps;
    h->kst_k.push_back(k);
  }
  const int p = F.parity;
  F.parity ^= 1;
  Flow f{F.ctl[p], F.q[p], F.fill[p], F.list, F.outst, F.ctl[p ^ 1], F.q[p ^ 1], F.fill[p ^ 1],
         c.refill, c.regen_ctr + (c.regen_parity * RCTR_N + RCTR_LIST) * CTR_STRIDE, c.rcap,
         F.qcap, F.jcap, F.lcap, F.C, F.P, k, F.xmap, h->flow_skip, nullptr, nullptr, nullptr};
#ifdef TG_FLOW_DBG
  if (const int rc = flow_diag_setup(h, f)) return rc;
#endif
  const EpQueue q{h->eps, h->eps_count, h->eps_cap};
  if (h->flow_debug)
    fprintf(stderr, "[flow] launching k %d grid %d x %d lcap %lld qcap %lld jcap %lld C %d\n", k, h->cus, bpc,
            (long long)F.lcap, (long long)F.qcap, (long long)F.jcap, F.C);
  {  // k_flow's arguments, in its parameter order and types
    Soa a_s = h->S;
    int64_t a_n = h->n;
    Level a_l = h->L;
    const uint32_t* a_grid = h->grid;
    FlowIO a_io = io;
    EpQueue a_q = q;
    int64_t a_g0 = h->g0;
    unsigned long long* a_stats = c.stats;
    int a_nstat = stat_slots(h->n);
    uint32_t* a_err = h->err;
    unsigned long long* a_ks = ks;
    void* args[] = {&a_s, &a_n, &a_l, &a_grid, &a_io, &a_q, &f,
                    &a_g0, &a_stats, &a_nstat, &a_err, &a_ks};
    HIP_TRY(hipLaunchKernel(kern, dim3((unsigned)(h->cus * bpc)), dim3(BLOCK), args, 0, st));
  }
  HIP_TRY(hipGetLastError());
  ++F.launches;
  // every sub-problem's chunks finished (no XCD the census saw went without waves)
  hipLaunchKernelGGL(k_flow_check, dim3(1), dim3(64), 0, st, F.ctl[p], F.P, F.C, h->err);
  HIP_TRY(hipGetLastError());
#ifdef TG_FLOW_DBG
  if (const int rc = flow_diag_after(h, f, k, bpc, st)) return rc;
#endif
  if (h->flow_debug) {  // diagnostics: the census and every sub-problem's counters
    HIP_TRY(hipDeviceSynchronize());
    std::vector<int32_t> cw((size_t)F.P * CTL_WORDS);
    HIP_TRY(hipMemcpy(cw.data(), F.ctl[p], sizeof(int32_t) * cw.size(), hipMemcpyDeviceToHost));
    uint32_t err = 0;
    HIP_TRY(hipMemcpy(&err, h->err, sizeof err, hipMemcpyDeviceToHost));
    fprintf(stderr, "[flow] launch %lld k %d P %d xmap %08x grid %d err %08x\n", (long long)F.launches,
            k, F.P, F.xmap, h->cus * bpc, err);
    for (int x = 0; x < F.P; ++x) {
      const int32_t* c0 = cw.data() + (size_t)x * CTL_WORDS;
      fprintf(stderr, "[flow]  x %d init %d qhead %d qtail %d fin %d done %d cls", x, c0[FC_INIT * FC_STRIDE],
              c0[FC_QHEAD * FC_STRIDE], c0[FC_QTAIL * FC_STRIDE], c0[FC_FIN * FC_STRIDE], c0[FC_DONE * FC_STRIDE]);
      for (int t = 0; t < k; ++t) fprintf(stderr, " %d", c0[(FC_CLS + t) * FC_STRIDE]);
      fprintf(stderr, "\n");
    }
  }
  c.rpend += k;
  if (c.rpend >= REGEN_STEPS) return launch_regen(h, c, st);
  return TG_OK;
}
}  // namespace

extern "C" {

int tg_step(tg_batch* h, const int32_t* actions, double* obs, int32_t* reward, uint8_t* valid,
            uint8_t* done, double* final_obs, uint32_t flags, void* stream) {
  BIND(h);
  if (!actions || !obs || !reward || !valid || !done)
    return fail(TG_E_INVAL, "tg_step: actions/obs/reward/valid/done are required");
  const StepIO io{const_cast<int32_t*>(actions), obs, reward, valid, done, final_obs, -1, 0, 0};
  return launch_step(h, h->main, io, (flags & TG_STEP_AUTORESET) != 0, (hipStream_t)stream,
                     h->tstep++);
}

}  // extern "C"

namespace {
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
// the N = 1 calls' result row: pinned, coherent host memory the kernel (or server) writes
int one_row(tg_batch* h) {
  if (h->one) return TG_OK;
  if (hipHostMalloc((void**)&h->one, sizeof(TgOne), hipHostMallocMapped | hipHostMallocCoherent) !=
      hipSuccess)
    return fail(TG_E_NOMEM, "tg_step1: pinned result buffer");
  HIP_TRY(hipHostGetDevicePointer((void**)&h->one_dev, h->one, 0));
  return TG_OK;
}

// launch k_serve1 on the server's stream, after the work queued on the caller's stream
int srv_start(tg_batch* h, hipStream_t caller) {
  // every buffer the server may write, whichever call launches it (a server first launched by
  // tg_available_mask1 serves the steps after it too)
  if (const int rc = one_row(h)) return rc;
  if (!h->box) {
    if (hipHostMalloc((void**)&h->box, sizeof(SrvBox), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
      return fail(TG_E_NOMEM, "tg_step1: pinned server mailbox");
    memset(h->box, 0, sizeof(SrvBox));
    HIP_TRY(hipHostGetDevicePointer((void**)&h->box_dev, h->box, 0));
    HIP_TRY(hipStreamCreateWithFlags(&h->srv_st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&h->srv_ev, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&h->srv_dep, hipEventDisableTiming));
    h->srv_seq = 0;
  }
  if (!h->py) {  // (the server's kernel argument; only SRV_*_PY commands touch it)
    if (hipHostMalloc((void**)&h->py, sizeof(tg_pystate), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
      return fail(TG_E_NOMEM, "tg_step1: pinned stream state");
    HIP_TRY(hipHostGetDevicePointer((void**)&h->py_dev, h->py, 0));
  }
  if (!h->pyc) {
    if (hipMalloc((void**)&h->pyc, sizeof(uint32_t) * PY_GENS * MT_N) != hipSuccess)
      return fail(TG_E_NOMEM, "tg_step1: stream cache");
    h->py_warm = false;
  }
  HIP_TRY(hipEventRecord(h->srv_dep, caller));
  HIP_TRY(hipStreamWaitEvent(h->srv_st, h->srv_dep, 0));
  const EpQueue q{h->eps, h->eps_count, h->eps_cap};
  if (h->srv_stage < 0) {  // the level's tables into the server's LDS, those that fit
    hipFuncAttributes fa{};
    int dev_max = 0;
    HIP_TRY(hipFuncGetAttributes(&fa, (const void*)k_serve1));
    HIP_TRY(hipDeviceGetAttribute(&dev_max, hipDeviceAttributeMaxSharedMemoryPerBlock, h->device));
    const size_t room = dev_max > (int)fa.sharedSizeBytes ? (size_t)dev_max - fa.sharedSizeBytes : 0;
    const size_t gb = h->L.gotab ? sizeof(uint32_t) * (size_t)h->L.W * h->L.H * 32 : 0;
    uint32_t stage = 0;
    size_t dyn = 0;
    if (gb && gb <= room) {
      stage = SRV_STAGE_GOTAB;
      dyn = gb;
    }
    if (dyn > 65536 &&
        hipFuncSetAttribute((const void*)k_serve1, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)dyn) != hipSuccess) {
      (void)hipGetLastError();
      stage = 0u;
      dyn = 0;
    }
    h->srv_stage = (int)stage;
    h->srv_dyn = dyn;
  }
  if (!h->box_dev || !h->py_dev || !h->pyc || !h->one_dev || !h->S.st4 || !h->S.ang || !h->S.ep ||
      !h->S.mt || !h->S.mc || !h->grid || !h->main.stats || !h->err)
    return fail(TG_E_HIP, "k_serve1: a buffer it writes is not allocated");
  hipLaunchKernelGGL(k_serve1, dim3(1), dim3(64), h->srv_dyn, h->srv_st, h->S, h->L, h->grid,
                     h->box_dev, h->py_dev, h->pyc, h->one_dev, q, h->g0, h->srv_idle,
                     (int)h->srv_trace, (uint32_t)h->srv_stage, h->main.stats, h->err);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(h->srv_ev, h->srv_st));
  h->srv_live = true;
  srv_register(h, true);
  h->srv_t_last = now_ns();
  ++h->srv_launches;
  return TG_OK;
}

// post a command and spin on its answer; a server that left (idle) before it saw the command is
// relaunched, and the new one serves it (it starts from the mailbox's done)
int srv_call(tg_batch* h, const SrvBox& c, hipStream_t caller) {
  // a server idle for more than half its limit (host clock, which starts after the server's)
  // may have left: ask its event before posting
  const int64_t t0 = now_ns();
  if (!h->srv_live ||
      (t0 - h->srv_t_last > (int64_t)h->srv_idle * 5 && hipEventQuery(h->srv_ev) == hipSuccess)) {
    if (const int rc = srv_start(h, caller)) return rc;
  }
  SrvBox* const b = h->box;
  const uint32_t seq = ++h->srv_seq;
  b->word = c.word;
  b->tstep = c.tstep;
  b->gauss_bits = c.gauss_bits;
  const int64_t tp = h->srv_trace ? now_ns() : 0;
  __atomic_store_n(&b->seq, seq, __ATOMIC_RELEASE);
  ++h->srv_calls;
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) {
      h->srv_t_last = now_ns();
      if (h->srv_trace) {
        const double g = 10.0 * (double)(b->t_end - b->t_seen), k = (double)b->ticks;
        h->srv_post_ns += (double)(tp - t0);
        h->srv_rt_ns += (double)(h->srv_t_last - tp);
        h->srv_gpu_ns += g;
        h->srv_fit[0] += k;
        h->srv_fit[1] += k * k;
        h->srv_fit[2] += g * k;
        if (b->phase[0]) {  // py_call's phases: pickup -> option start -> end -> observe ->
          const uint64_t t[7] = {b->t_seen, b->phase[0], b->phase[1], b->phase[2], b->phase[3],
                                 b->phase[4], b->t_end};  // barrier -> its return -> answer
          for (int j = 0; j < 6; ++j) h->srv_phase[j] += 10.0 * (double)(t[j + 1] - t[j]);
          ++h->srv_phase_n;
        }
      }
      return TG_OK;
    }
    __builtin_ia32_pause();
    if ((it & 4095) == 0) {
      const hipError_t e = hipEventQuery(h->srv_ev);
      if (e == hipSuccess) {  // the server left: a new one serves the command
        if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) continue;
        if (const int rc = srv_start(h, caller)) return rc;
      } else if (e != hipErrorNotReady) {
        h->srv_live = false;
        return fail(TG_E_HIP, "tg_step1 server: %s", hipGetErrorString(e));
      } else if (now_ns() - t0 > 20000000000ll) {
        return fail(TG_E_HIP, "tg_step1 server: no answer to command %u in 20 s", seq);
      }
    }
  }
}
}  // namespace

namespace {
// Handles whose server may be running.  At exit (the library's static destructors run before
// those of libamdhip64, which it depends on) every one still running is told to quit and waited
// for, at most a second each: no server outlives the process's pinned mailbox.
std::mutex g_srv_mu;
std::vector<tg_batch*> g_srv_handles;
void srv_register(tg_batch* h, bool live) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  auto it = std::find(g_srv_handles.begin(), g_srv_handles.end(), h);
  if (live && it == g_srv_handles.end()) g_srv_handles.push_back(h);
  if (!live && it != g_srv_handles.end()) g_srv_handles.erase(it);
}
void srv_post_quit(tg_batch* h) {
  SrvBox* const b = h->box;
  b->word = srv_word(SRV_QUIT, 0, false, false, 0);
  __atomic_store_n(&b->seq, ++h->srv_seq, __ATOMIC_RELEASE);
}
struct SrvReaper {
  ~SrvReaper() {
    std::lock_guard<std::mutex> lk(g_srv_mu);
    for (tg_batch* h : g_srv_handles) {
      if (!h->srv_live || hipSetDevice(h->device) != hipSuccess) continue;
      if (hipEventQuery(h->srv_ev) == hipErrorNotReady) srv_post_quit(h);
      const int64_t t0 = now_ns();
      while (hipEventQuery(h->srv_ev) == hipErrorNotReady && now_ns() - t0 < 1000000000ll) {
      }
      h->srv_live = false;
    }
    g_srv_handles.clear();
  }
} g_srv_reaper;
}  // namespace

namespace tg {
int srv_stop(tg_batch* h) {
  if (!h->srv_live) return TG_OK;
  h->srv_live = false;
  srv_register(h, false);
  if (hipEventQuery(h->srv_ev) != hipSuccess) srv_post_quit(h);
  HIP_TRY(hipEventSynchronize(h->srv_ev));
  // gone: a QUIT it left (idle) without reading is void, not a command for the next server
  h->box->done = h->box->seq;
  return TG_OK;
}
}  // namespace tg

extern "C" {

int tg_step1(tg_batch* h, int32_t action, double* obs, int32_t* reward, uint8_t* valid,
             uint8_t* done, void* stream) {
  BIND_SERVE(h);
  if (h->n != 1 || !obs || !reward || !valid || !done)
    return fail(TG_E_INVAL, "tg_step1: a 1-env handle and host obs/reward/valid/done");
  if (const int rc = one_row(h)) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (h->serve) {
    SrvBox c{};
    c.word = srv_word(SRV_STEP, action, false, false, 0);
    c.tstep = h->tstep++;
    if (const int rc = srv_call(h, c, st)) return rc;
  } else {
    TgOne* const d = h->one_dev;
    const StepIO io{nullptr, d->obs, &d->reward, &d->valid, &d->done, nullptr, POL_IMMEDIATE,
                    (uint64_t)(int64_t)action, 0, h->tstep++};
    const EpQueue q{h->eps, h->eps_count, h->eps_cap};
    hipLaunchKernelGGL((k_step<false, false, POL_IMMEDIATE>), dim3(1), dim3(BLOCK), 0, st, h->S,
                       h->n, h->L, h->grid, io, q, h->g0, h->main.stats, h->err, nullptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
  }
  memcpy(obs, h->one->obs, sizeof h->one->obs);
  *reward = h->one->reward;
  *valid = h->one->valid;
  *done = h->one->done;
  return TG_OK;
}

int tg_available_mask1(tg_batch* h, uint16_t* mask, void* stream) {
  BIND_SERVE(h);
  if (h->n != 1 || !mask) return fail(TG_E_INVAL, "tg_available_mask1: a 1-env handle and a host output");
  if (h->serve) {
    SrvBox c{};
    c.word = srv_word(SRV_MASK, 0, false, false, 0);
    if (const int rc = srv_call(h, c, (hipStream_t)stream)) return rc;
    *mask = (uint16_t)h->box->mask;
    return TG_OK;
  }
  if (!h->mask1) {
    if (hipHostMalloc((void**)&h->mask1, sizeof(uint16_t), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
      return fail(TG_E_NOMEM, "tg_available_mask1: pinned result");
    HIP_TRY(hipHostGetDevicePointer((void**)&h->mask1_dev, h->mask1, 0));
  }
  hipLaunchKernelGGL(k_mask, dim3(1), dim3(BLOCK), 0, (hipStream_t)stream, h->S, h->n, h->L, h->grid,
                     h->mask1_dev);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  *mask = *h->mask1;
  return TG_OK;
}

int tg_reset1(tg_batch* h, double* obs, void* stream) {
  BIND_SERVE(h);
  if (h->n != 1) return fail(TG_E_INVAL, "tg_reset1: a 1-env handle");
  if (h->serve) {
    SrvBox c{};
    c.word = srv_word(SRV_RESET, 0, false, false, 0);
    c.tstep = h->tstep;  // the next step's index: the new episode's start (as tg_reset)
    if (const int rc = srv_call(h, c, (hipStream_t)stream)) return rc;
  } else {
    if (const int rc = one_row(h)) return rc;
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(BLOCK), 0, (hipStream_t)stream, h->S, h->n, h->L,
                       (const uint8_t*)nullptr, h->one_dev->obs, h->tstep);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  }
  if (obs) memcpy(obs, h->one->obs, sizeof h->one->obs);
  return TG_OK;
}

int tg_set_serve(tg_batch* h, int on) {
  BIND(h);  // (stops a running server)
  h->serve = on != 0;
  return TG_OK;
}

}  // extern "C"

namespace {
// one k_py1 launch (or server command): the caller's stream state in, the result row and the
// advanced state out.  The state is the 624 words, the index and (may be null: a step draws no
// gauss) has_gauss / gauss_next, wherever the caller keeps them: a tg_pystate, or the words and
// index of a CPython random.Random object (tg_step1_pywords).
template <bool RESET>
int launch_py1(tg_batch* h, int32_t action, uint32_t* words, uint32_t* index, uint32_t* has_gauss,
               double* gauss_next, hipStream_t stream) {
  if (h->n != 1 || !words || !index) return fail(TG_E_INVAL, "tg_*1_py: a 1-env handle and a stream state");
  if (*index > (uint32_t)MT_N)
    return fail(TG_E_INVAL, "tg_*1_py: index %u outside [0, 624]", *index);
  if (const int rc = one_row(h)) return rc;
  if (!h->py) {
    if (hipHostMalloc((void**)&h->py, sizeof(tg_pystate), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
      return fail(TG_E_NOMEM, "tg_*1_py: pinned stream state");
    HIP_TRY(hipHostGetDevicePointer((void**)&h->py_dev, h->py, 0));
  }
  if (!h->pyc) {
    if (hipMalloc((void**)&h->pyc, sizeof(uint32_t) * PY_GENS * MT_N) != hipSuccess)
      return fail(TG_E_NOMEM, "tg_*1_py: stream cache");
    h->py_warm = false;
  }
  // the device's cached generations serve the call iff the caller's state is the one the last
  // call returned (no other draws on the stream since: the user's own, another env's)
  const bool warm = h->py_warm && *index == h->py_last.index &&
                    (!has_gauss || (*has_gauss == h->py_last.has_gauss &&
                                    memcmp(gauss_next, &h->py_last.gauss_next, sizeof(double)) == 0)) &&
                    memcmp(words, h->py_last.mt, sizeof h->py_last.mt) == 0;
  if (!warm) {
    memcpy(h->py->mt, words, sizeof h->py->mt);
    h->py->index = *index;
  }
  if (has_gauss) {
    h->py->has_gauss = *has_gauss;
    h->py->gauss_next = *gauss_next;
  }
  const uint32_t q0 = *index;
  const int hg = has_gauss ? (int)*has_gauss : 0;
  const double gn = has_gauss ? *gauss_next : 0.0;
  // a step's tstep is its index; a reset's, the next step's (the new episode's start)
  const uint32_t tstep = RESET ? h->tstep : h->tstep++;
  h->py_warm = false;  // until the call has returned
  if (h->serve) {
    SrvBox c{};
    c.word = srv_word(RESET ? SRV_RESET_PY : SRV_STEP_PY, action, warm, hg != 0, q0);
    c.tstep = tstep;
    memcpy(&c.gauss_bits, &gn, sizeof c.gauss_bits);
    if (const int rc = srv_call(h, c, stream)) return rc;
  } else {
    hipLaunchKernelGGL(k_py1<RESET>, dim3(1), dim3(64), 0, stream, h->S, h->L, h->grid, (int)action,
                       h->py_dev, warm ? h->pyc : nullptr, h->pyc, q0, hg, gn, h->one_dev, tstep,
                       h->main.stats, h->err);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(stream));
  }
  memcpy(words, h->py->mt, sizeof h->py->mt);
  *index = h->py->index;
  memcpy(h->py_last.mt, words, sizeof h->py_last.mt);
  h->py_last.index = *index;
  if (has_gauss) {
    *has_gauss = h->py->has_gauss;
    *gauss_next = h->py->gauss_next;
    h->py_last.has_gauss = *has_gauss;
    h->py_last.gauss_next = *gauss_next;
  }
  h->py_warm = true;
  return TG_OK;
}
int row_out(const tg_batch* h, double* obs, int32_t* reward, uint8_t* valid, uint8_t* done) {
  memcpy(obs, h->one->obs, sizeof h->one->obs);
  *reward = h->one->reward;
  *valid = h->one->valid;
  *done = h->one->done;
  return TG_OK;
}
}  // namespace

extern "C" {

int tg_step1_py(tg_batch* h, int32_t action, tg_pystate* st, double* obs, int32_t* reward,
                uint8_t* valid, uint8_t* done, void* stream) {
  BIND_SERVE(h);
  if (!obs || !reward || !valid || !done || !st) return fail(TG_E_INVAL, "tg_step1_py: null output");
  const int rc = launch_py1<false>(h, action, st->mt, &st->index, &st->has_gauss, &st->gauss_next,
                                   (hipStream_t)stream);
  return rc ? rc : row_out(h, obs, reward, valid, done);
}

int tg_step1_pywords(tg_batch* h, int32_t action, uint32_t* words, int32_t* index, double* obs,
                     int32_t* reward, uint8_t* valid, uint8_t* done, void* stream) {
  BIND_SERVE(h);
  if (!obs || !reward || !valid || !done || !words || !index)
    return fail(TG_E_INVAL, "tg_step1_pywords: null argument");
  if (*index < 0) return fail(TG_E_INVAL, "tg_step1_pywords: index %d < 0", *index);
  const int rc = launch_py1<false>(h, action, words, reinterpret_cast<uint32_t*>(index), nullptr,
                                   nullptr, (hipStream_t)stream);
  return rc ? rc : row_out(h, obs, reward, valid, done);
}

int tg_reset1_py(tg_batch* h, tg_pystate* st, double* obs, void* stream) {
  BIND_SERVE(h);
  if (!st) return fail(TG_E_INVAL, "tg_reset1_py: null stream state");
  const int rc = launch_py1<true>(h, 0, st->mt, &st->index, &st->has_gauss, &st->gauss_next,
                                  (hipStream_t)stream);
  if (rc) return rc;
  if (obs) memcpy(obs, h->one->obs, sizeof h->one->obs);
  return TG_OK;
}

int tg_rollout(tg_batch* h, int32_t steps, uint64_t action_seed, int64_t t0, int policy,
               uint32_t flags, int32_t* actions, double* obs, int32_t* reward, uint8_t* valid,
               uint8_t* done, void* stream) {
  BIND(h);
  if (steps == 0) return TG_OK;
  if (steps < 0 || !reward || !valid || !done ||
      (policy != TG_POLICY_UNIFORM && policy != TG_POLICY_MASKED))
    return fail(TG_E_INVAL, "tg_rollout: bad arguments");
  const int64_t n = h->n;
  if (!obs && !h->obs_scratch)  // the step kernels always write an obs row
    if (hipMalloc((void**)&h->obs_scratch, sizeof(double) * 9 * (size_t)n) != hipSuccess)
      return fail(TG_E_NOMEM, "tg_rollout: obs scratch");
  const bool ar = (flags & TG_STEP_AUTORESET) != 0;
  hipStream_t cs = (hipStream_t)stream;
  const uint32_t tb = h->tstep;
  h->tstep += (uint32_t)steps;
  auto io_of = [&](int32_t s) {
    return StepIO{actions ? actions + (size_t)s * n : nullptr,
                  obs ? obs + (size_t)s * n * 9 : h->obs_scratch,
                  reward + (size_t)s * n, valid + (size_t)s * n, done + (size_t)s * n,
                  nullptr, policy, action_seed, t0 + s};
  };
  if (h->mode == TG_MODE_FLOW) {  // k_flow, up to FLOW_MAX_K steps per launch (no groups: tg_set_mode)
    int rc = flow_init(h);
    for (int32_t s = 0; s < steps && !rc; s += FLOW_MAX_K) {
      const int k = steps - s < FLOW_MAX_K ? steps - s : FLOW_MAX_K;
      const FlowIO io{actions ? actions + (size_t)s * n : nullptr,
                      obs ? obs + (size_t)s * n * 9 : h->obs_scratch, obs ? n * 9 : 0,
                      reward + (size_t)s * n, valid + (size_t)s * n, done + (size_t)s * n,
                      action_seed, t0 + s, tb + (uint32_t)s};
      rc = launch_flow(h, k, io, ar, policy == TG_POLICY_MASKED ? 1 : 0, cs);
    }
    return rc;
  }
  if (h->grp.empty() || h->mode != TG_MODE_COMPACT) {
    for (int32_t s = 0; s < steps; ++s) {
      const int rc = launch_step(h, h->main, io_of(s), ar, cs, tb + (uint32_t)s);
      if (rc) return rc;
    }
    return TG_OK;
  }
  // Groups (tg_set_groups): each steps its envs on a stream of its own, so one group's
  // latency-bound k_run tail overlaps the others' bandwidth-bound k_classify / k_regen.  The
  // handle's own pending refill lists go first (the groups' k_classify would not list those
  // halves again), each group drains its own at the end, then the caller's stream joins.
  int rc = launch_regen(h, h->main, cs);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(h->fork, cs));
  for (auto& c : h->grp) HIP_TRY(hipStreamWaitEvent(c.st, h->fork, 0));
  for (int32_t s = 0; s < steps; ++s)
    for (size_t g = 0; g < h->grp.size(); ++g) {
      StepCtx& c = h->grp[g];
      // stagger: group g + 1 starts after group g's first k_classify (half a step apart)
      hipEvent_t mid = (s == 0 && h->stagger && g + 1 < h->grp.size()) ? h->grp[g + 1].ev : nullptr;
      if ((rc = launch_step(h, c, io_of(s), ar, c.st, tb + (uint32_t)s, mid))) return rc;
      if (mid) HIP_TRY(hipStreamWaitEvent(h->grp[g + 1].st, mid, 0));
    }
  for (auto& c : h->grp) {
    if ((rc = launch_regen(h, c, c.st))) return rc;
    HIP_TRY(hipEventRecord(c.ev, c.st));
    HIP_TRY(hipStreamWaitEvent(cs, c.ev, 0));
  }
  return TG_OK;
}

int tg_set_groups(tg_batch* h, int32_t groups, int32_t stagger) {
  BIND(h);
  if (groups > 1 && h->mode == TG_MODE_FLOW)
    return fail(TG_E_INVAL, "tg_set_groups: groups are a TG_MODE_COMPACT rollout form (TG_MODE_FLOW "
                            "steps the whole batch in one k_flow launch)");
  if (groups < 1 || groups > 16 || (int64_t)groups * 4096 > h->n)
    return fail(TG_E_INVAL, "tg_set_groups: %d groups of %lld envs (1..16, >= 4096 envs each)",
                groups, (long long)h->n);
  HIP_TRY(hipDeviceSynchronize());
  int rc = regen_all(h, 0);  // the old groups' pending lists
  if (rc) return rc;
  HIP_TRY(hipDeviceSynchronize());
  if (!h->grp.empty()) {  // the old groups' launch counters go on with the handle's own
    std::vector<unsigned long long> slot0(ST_COUNT);
    HIP_TRY(hipMemcpy(slot0.data(), h->main.stats, sizeof(unsigned long long) * ST_COUNT,
                      hipMemcpyDeviceToHost));
    for (auto& c : h->grp) {
      std::vector<unsigned long long> part((size_t)stat_slots(c.n) * ST_COUNT);
      HIP_TRY(hipMemcpy(part.data(), c.stats, sizeof(unsigned long long) * part.size(),
                        hipMemcpyDeviceToHost));
      for (size_t i = 0; i < part.size(); ++i) slot0[i % ST_COUNT] += part[i];
    }
    HIP_TRY(hipMemcpy(h->main.stats, slot0.data(), sizeof(unsigned long long) * ST_COUNT,
                      hipMemcpyHostToDevice));
  }
  for (auto& c : h->grp) free_ctx(c);
  h->grp.clear();
  h->stagger = stagger != 0;
  if (groups == 1) return TG_OK;
  if (!h->fork) HIP_TRY(hipEventCreateWithFlags(&h->fork, hipEventDisableTiming));
  // contiguous groups of whole 256-env workgroups
  const int64_t per = ((h->n + groups - 1) / groups + BLOCK - 1) / BLOCK * BLOCK;
  h->grp.resize((size_t)groups);
  for (int g = 0; g < groups; ++g) {
    const int64_t off = per * g, cnt = std::min(per, h->n - off);
    StepCtx& c = h->grp[(size_t)g];
    if (cnt <= 0 || (rc = alloc_ctx(c, off, cnt))) {
      for (auto& x : h->grp) free_ctx(x);
      h->grp.clear();
      return rc ? rc : fail(TG_E_INVAL, "tg_set_groups: empty group");
    }
    HIP_TRY(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
  }
  return TG_OK;
}

int tg_available_mask(tg_batch* h, uint16_t* mask, void* stream) {
  BIND(h);
  if (!mask) return fail(TG_E_INVAL, "tg_available_mask: null output");
  hipLaunchKernelGGL(k_mask, dim3(grid_for(h->n)), dim3(BLOCK), 0, (hipStream_t)stream, h->S,
                     h->n, h->L, h->grid, mask);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_observe(tg_batch* h, double* obs, void* stream) {
  BIND(h);
  if (!obs) return fail(TG_E_INVAL, "tg_observe: null output");
  hipLaunchKernelGGL(k_observe, dim3(grid_for(h->n)), dim3(BLOCK), 0, (hipStream_t)stream, h->S,
                     h->n, h->L, obs);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_policy_actions(tg_batch* h, uint64_t a0, int64_t t, int policy, int32_t* actions,
                      void* stream) {
  BIND(h);
  if (!actions || (policy != TG_POLICY_UNIFORM && policy != TG_POLICY_MASKED))
    return fail(TG_E_INVAL, "tg_policy_actions: bad arguments");
  hipLaunchKernelGGL(k_actions, dim3(grid_for(h->n)), dim3(BLOCK), 0, (hipStream_t)stream, h->S,
                     h->n, h->L, h->grid, a0, h->g0, t, policy, actions);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_episodes(tg_batch* h, tg_episode* out, int32_t* count, int32_t cap, void* stream) {
  BIND(h);
  if (!out || !count || cap < 0) return fail(TG_E_INVAL, "tg_episodes: bad arguments");
  hipLaunchKernelGGL(k_drain_episodes, dim3(1), dim3(BLOCK), 0, (hipStream_t)stream, h->eps,
                     h->eps_count, h->eps_cap, out, count, cap);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_errors(tg_batch* h, uint32_t* out, void* stream) {
  BIND(h);
  if (!out) return fail(TG_E_INVAL, "tg_errors: null output");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_errors, dim3(grid_for(h->n)), dim3(BLOCK), 0, st, h->S.st4, h->n, h->err);
  HIP_TRY(hipGetLastError());
  uint32_t v = 0;
  HIP_TRY(hipMemcpyAsync(&v, h->err, sizeof v, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *out = v;
  return TG_OK;
}

int tg_set_mode(tg_batch* h, int mode, int run_blocks) {
  BIND(h);
  if (mode != TG_MODE_DIRECT && mode != TG_MODE_COMPACT && mode != TG_MODE_FLOW)
    return fail(TG_E_INVAL, "tg_set_mode: unknown mode %d", mode);
  if (mode == TG_MODE_FLOW && !h->grp.empty())
    return fail(TG_E_INVAL, "tg_set_mode: TG_MODE_FLOW steps the whole batch in one k_flow launch; "
                            "call tg_set_groups(h, 1, 0) first");
  h->mode = mode;
  (void)run_blocks;  // reserved
  return TG_OK;
}

int tg_regenerate(tg_batch* h, void* stream) {
  BIND(h);
  return regen_all(h, (hipStream_t)stream);
}

int tg_set_timing(tg_batch* h, int every) {
  BIND(h);
  if (every < 0) return fail(TG_E_INVAL, "tg_set_timing: every %d < 0", every);
  HIP_TRY(hipDeviceSynchronize());
  int rc = flush_timing(h);  // records of the previous setting are kept in the sums
  if (rc) return rc;
  if (every && !h->kst && (rc = kst_reset(h))) return rc;
  h->timing_every = every;
  h->timing_calls = 0;
  return TG_OK;
}

int tg_set_episode_capacity(tg_batch* h, int32_t cap) {
  BIND(h);
  if (cap < 1 || cap > (1 << 28)) return fail(TG_E_INVAL, "tg_set_episode_capacity: cap %d", cap);
  HIP_TRY(hipDeviceSynchronize());
  tg_episode* eps = nullptr;
  if (hipMalloc((void**)&eps, sizeof(tg_episode) * (size_t)cap) != hipSuccess)
    return fail(TG_E_NOMEM, "tg_set_episode_capacity: %d records", cap);
  (void)hipFree(h->eps);
  h->eps = eps;
  h->eps_cap = cap;
  HIP_TRY(hipMemset(h->eps_count, 0, sizeof(int32_t)));
  return TG_OK;
}

int tg_predicate_table(tg_batch* h, int32_t x0, int32_t x1, int32_t y0, int32_t y1,
                       uint32_t door_bits, uint8_t* out, void* stream) {
  BIND(h);
  if (!out || x1 <= x0 || y1 <= y0 || x0 < -4096 || x1 > 32000 || y0 < -4096 || y1 > 32000)
    return fail(TG_E_INVAL, "tg_predicate_table: bad box or null output");
  const int64_t cells = (int64_t)(x1 - x0) * (y1 - y0);
  hipLaunchKernelGGL(k_predicates, dim3((unsigned)((cells + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     (hipStream_t)stream, h->L, h->grid, x0, x1, y0, y1, door_bits, out);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_get_stats(tg_batch* h, tg_stats* out) {
  BIND(h);
  if (!out) return fail(TG_E_INVAL, "tg_get_stats: null output");
  HIP_TRY(hipDeviceSynchronize());
  int rc = flush_timing(h);
  if (rc) return rc;
  unsigned long long s[ST_COUNT] = {};
  std::vector<StepCtx*> ctxs{&h->main};
  for (auto& c : h->grp) ctxs.push_back(&c);
  for (StepCtx* c : ctxs) {
    const size_t nb = (size_t)stat_slots(c->n);
    std::vector<unsigned long long> part(nb * ST_COUNT);
    HIP_TRY(hipMemcpy(part.data(), c->stats, sizeof(unsigned long long) * part.size(),
                      hipMemcpyDeviceToHost));
    for (size_t b = 0; b < nb; ++b)
      for (int k = 0; k < ST_COUNT; ++k) s[k] += part[b * ST_COUNT + k];
  }
  out->steps = (int64_t)s[ST_STEPS];
  out->valid_steps = (int64_t)s[ST_VALID];
  out->ticks = (int64_t)s[ST_TICKS];
  out->draws = (int64_t)s[ST_DRAWS];
  out->episodes = (int64_t)s[ST_EPISODES];
  out->episodes_dropped = (int64_t)s[ST_EP_OVERFLOW];
  out->launches = out->steps / (h->n ? h->n : 1);
  out->kernel_ms = h->kernel_ms_done;
  out->regens = (int64_t)s[ST_REGENS] * MT_HALF_GENS;  // halves -> generations
  out->wave_ticks = (int64_t)s[ST_WTICKS];
  out->timed_launches = h->timed_launches;
  out->run_ms = h->run_ms_done;
  out->regen_ms = h->regen_ms_done;
  out->regen_timed = h->regen_timed;
  out->regen_launches = h->regen_launches;
  out->classify_ms = h->classify_ms_done;
  return TG_OK;
}

int tg_stats_reset(tg_batch* h) {
  BIND(h);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemset(h->main.stats, 0, sizeof(unsigned long long) * ST_COUNT * (size_t)stat_slots(h->n)));
  for (auto& c : h->grp)
    HIP_TRY(hipMemset(c.stats, 0, sizeof(unsigned long long) * ST_COUNT * (size_t)stat_slots(c.n)));
  if (h->kst) {
    const int rc = kst_reset(h);  // drops the unflushed records
    if (rc) return rc;
  }
  h->kernel_ms_done = 0.0;
  h->run_ms_done = 0.0;
  h->classify_ms_done = 0.0;
  h->timed_launches = 0;
  h->regen_ms_done = 0.0;
  h->regen_timed = 0;
  h->regen_launches = 0;
  return TG_OK;
}

int tg_probe_dispatch(int32_t kernels, int32_t blocks, void* stream) {
  if (kernels < 0 || blocks < 1) return fail(TG_E_INVAL, "tg_probe_dispatch: bad arguments");
  for (int32_t k = 0; k < kernels; ++k)
    hipLaunchKernelGGL(k_null, dim3((unsigned)blocks), dim3(BLOCK), 0, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

int tg_mt_layout(int32_t* ring_words, int32_t* stored_words, int32_t* code_bytes) {
  if (ring_words) *ring_words = MT_WORDS;
  if (stored_words) *stored_words = MT_STORE;
  if (code_bytes) *code_bytes = MT_CODES;
  return TG_OK;
}

int tg_kernel_info(tg_batch* h, int kernel, int32_t* blocks_per_cu, int32_t* vgprs, int32_t* sgprs,
                   int32_t* lds_bytes) {
  BIND(h);
  const void* k = kernel == TG_KERNEL_CLASSIFY ? reinterpret_cast<const void*>(k_classify<true, false>)
                  : kernel == TG_KERNEL_RUN    ? reinterpret_cast<const void*>(k_run<true, false>)
                  : kernel == TG_KERNEL_REGEN  ? reinterpret_cast<const void*>(k_regen)
                                               : nullptr;
  if (!k) return fail(TG_E_INVAL, "tg_kernel_info: unknown kernel %d", kernel);
  hipFuncAttributes fa;
  HIP_TRY(hipFuncGetAttributes(&fa, k));
  int nb = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kernel == TG_KERNEL_RUN ? RUN_BLOCK : BLOCK,
                                                       0));
  if (blocks_per_cu) *blocks_per_cu = nb;
  if (vgprs) *vgprs = fa.numRegs;
  if (sgprs) *sgprs = -1;  // not reported by hipFuncGetAttributes
  if (lds_bytes) *lds_bytes = (int32_t)fa.sharedSizeBytes;
  return TG_OK;
}

int tg_read_state(tg_batch* h, int32_t* pos, uint32_t* flags, int32_t* objs, double* ang,
                  uint32_t* mt, uint32_t* mt_pos, int32_t* ep) {
  BIND(h);
  HIP_TRY(hipDeviceSynchronize());
  const int64_t n = h->n;
  std::vector<uint4> st;
  if (pos || flags || objs || mt || mt_pos) {
    st.resize((size_t)n);
    HIP_TRY(hipMemcpy(st.data(), h->S.st4, sizeof(uint4) * n, hipMemcpyDeviceToHost));
  }
  if (pos || flags || objs) {
    for (int64_t i = 0; i < n; ++i) {
      const uint4 s = st[(size_t)i];
      if (pos) {
        pos[2 * i] = (int16_t)(s.x & 0xFFFFu);
        pos[2 * i + 1] = (int16_t)(s.x >> 16);
      }
      if (flags) flags[i] = s.y;
      if (objs) {
        objs[4 * i] = (int8_t)(s.z & 0xFF);
        objs[4 * i + 1] = (int8_t)((s.z >> 8) & 0xFF);
        objs[4 * i + 2] = (int8_t)((s.z >> 16) & 0xFF);
        objs[4 * i + 3] = (int8_t)(s.z >> 24);
      }
    }
  }
  if (ang) HIP_TRY(hipMemcpy(ang, h->S.ang, sizeof(double2) * n, hipMemcpyDeviceToHost));
  if (ep) {  // (return, start step) -> (return, length): the steps since the start
    HIP_TRY(hipMemcpy(ep, h->S.ep, sizeof(int2) * n, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) ep[2 * i + 1] = (int32_t)(h->tstep - (uint32_t)ep[2 * i + 1]);
  }
  if (mt_pos) {
    // CPython's index into the generation holding the position
    for (int64_t i = 0; i < n; ++i) mt_pos[i] = (st[(size_t)i].w & MT_POS_MASK) % MT_N;
  }
  if (mt) {
    // the generations, gathered on the device into a bounded staging buffer (<= 64 Ki envs,
    // 160 MB) and copied out in one transfer per chunk
    const int64_t chunk = n < (1 << 16) ? n : (1 << 16);
    uint32_t* stage = nullptr;
    if (hipMalloc((void**)&stage, sizeof(uint32_t) * MT_N * (size_t)chunk) != hipSuccess)
      return fail(TG_E_NOMEM, "tg_read_state: staging buffer");
    int rc = TG_OK;
    for (int64_t first = 0; first < n && rc == TG_OK; first += chunk) {
      const int64_t cnt = n - first < chunk ? n - first : chunk;
      const int64_t threads = cnt * (MT_N / 4);
      hipLaunchKernelGGL(k_gather_mt, dim3((unsigned)((threads + BLOCK - 1) / BLOCK)), dim3(BLOCK),
                         0, 0, h->S, first, cnt, stage);
      hipError_t e = hipGetLastError();
      if (e == hipSuccess)
        e = hipMemcpy(mt + first * MT_N, stage, sizeof(uint32_t) * MT_N * (size_t)cnt,
                      hipMemcpyDeviceToHost);
      if (e != hipSuccess) rc = fail(TG_E_HIP, "tg_read_state: %s", hipGetErrorString(e));
    }
    (void)hipFree(stage);
    if (rc) return rc;
  }
  return TG_OK;
}

int tg_write_state(tg_batch* h, const int32_t* pos, const uint32_t* flags, const int32_t* objs,
                   const double* ang, const uint32_t* mt, const uint32_t* mt_pos,
                   const int32_t* ep) {
  BIND(h);
  if (!pos || !flags || !objs || !ang || !mt || !mt_pos)
    return fail(TG_E_INVAL, "tg_write_state: pos, flags, objs, ang, mt and mt_pos are required");
  const int64_t n = h->n;
  std::vector<uint4> st((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t p = mt_pos[i];
    if (p > (uint32_t)MT_N || (p & 1u))
      return fail(TG_E_INVAL, "tg_write_state: env %lld: mt_pos %u (must be even, <= 624: "
                  "random() consumes words in pairs)", (long long)i, p);
    for (int k = 0; k < 2; ++k)
      if (pos[2 * i + k] < -32768 || pos[2 * i + k] > 32767)
        return fail(TG_E_INVAL, "tg_write_state: env %lld: position out of range", (long long)i);
    for (int k = 0; k < 4; ++k)
      if (objs[4 * i + k] < -128 || objs[4 * i + k] > 127)
        return fail(TG_E_INVAL, "tg_write_state: env %lld: object cell out of range", (long long)i);
    Env e{};
    e.px = pos[2 * i], e.py = pos[2 * i + 1];
    e.f = flags[i];
    e.kx = objs[4 * i], e.ky = objs[4 * i + 1], e.gx = objs[4 * i + 2], e.gy = objs[4 * i + 3];
    // the given generation goes to the ring's first slot, its successors to the others
    // (fresh); index 624 is the start of the successor (CPython twists before its next draw)
    e.mti = p;
    uint4 w;
    w.x = ((uint32_t)e.px & 0xFFFFu) | ((uint32_t)e.py << 16);
    w.y = e.f;
    w.z = ((uint32_t)e.kx & 0xFF) | (((uint32_t)e.ky & 0xFF) << 8) | (((uint32_t)e.gx & 0xFF) << 16) |
          ((uint32_t)e.gy << 24);
    w.w = e.mti;
    st[(size_t)i] = w;
  }
  HIP_TRY(hipDeviceSynchronize());
  // validated: the pending refill lists name the old states' halves, and every ring is rebuilt
  h->main.rpend = 0;
  for (auto& c : h->grp) c.rpend = 0;
  HIP_TRY(hipMemset(h->main.regen_ctr, 0, sizeof(int32_t) * 2 * RCTR_N * CTR_STRIDE));
  for (auto& c : h->grp) HIP_TRY(hipMemset(c.regen_ctr, 0, sizeof(int32_t) * 2 * RCTR_N * CTR_STRIDE));
  HIP_TRY(hipMemcpy(h->S.st4, st.data(), sizeof(uint4) * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->S.ang, ang, sizeof(double2) * n, hipMemcpyHostToDevice));
  {  // (return, length) -> (return, start step)
    std::vector<int2> e2((size_t)n);
    for (int64_t i = 0; i < n; ++i)
      e2[(size_t)i] = ep ? make_int2(ep[2 * i], (int32_t)(h->tstep - (uint32_t)ep[2 * i + 1]))
                         : make_int2(0, (int32_t)h->tstep);
    HIP_TRY(hipMemcpy(h->S.ep, e2.data(), sizeof(int2) * n, hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy2D(h->S.mt, sizeof(uint32_t) * MT_STORE, mt, sizeof(uint32_t) * MT_N,
                      sizeof(uint32_t) * MT_N, (size_t)n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_gen_codes, dim3(grid_for(n)), dim3(BLOCK), 0, 0, h->S, n);
  hipLaunchKernelGGL(k_gen_twist, dim3(grid_for(n)), dim3(BLOCK), 0, 0, h->S, n, 0u, 1,
                     2 * MT_HALF_GENS - 1);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  return TG_OK;
}

#ifdef TG_DIAG_STAMPS
int tg_diag_stamps(unsigned long long* out, int n_waves) {
  if (n_waves > NSTAMP_WAVES) n_waves = NSTAMP_WAVES;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * NSTAMP * n_waves));
  return TG_OK;
}
#endif

}  // extern "C"
#endif  // TG_FLOW_TU
