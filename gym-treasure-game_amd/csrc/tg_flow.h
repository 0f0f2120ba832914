// tg_flow.h — k_flow: tg_rollout's K steps in ONE launch, each env advancing to its next step
// as soon as its own option is done (TG_MODE_FLOW, §8f row 3).  Included by tg_amd.hip inside
// its anonymous namespace, after the per-step kernels whose pieces it reuses (RngCodesT,
// finish_step, record_episodes, wave_stats).
//
// Why: the reference's step is per env (TG/:91-96 -> OP/:20-36): env i's step
// t + 1 depends on env i's step t only.  The per-step kernels put a batch-wide barrier after
// every step, so a step costs one maximal option chain (k_run ends with its slowest option
// waves, ~50 us at the uniform policy, while only ~3.4 waves per SIMD carry work).  Round 5's
// form handed steps on per 64-env chunk: a chunk was classified for t + 1 when all its envs
// were done with t, so each chunk still waited, every step, for the slowest option among its
// envs (chunks of 128 and 256 envs measured slower still, profiles/r06/r06c_*).  Here the hand-
// off is per env: the lane that finishes env i's option at step t keeps the env in registers
// and classifies it itself for t + 1, t + 2, ... ("run-ahead"), finishing in place every step
// whose option cannot run (~79 % at the uniform policy: reward None, state and MT stream
// untouched, OP/:22-23), until an option can run; only then is the env listed.
//
// Work, per sub-problem (one per XCD, below; the envs of 64-env chunks x, x + P, ...):
//   deal: chunk x + P j, dealt out by a counter: one lane per env (coalesced loads), each lane
//     runs its env ahead from step 0.
//   run (t, k, j): 64-entry chunk j of list (t, k), one lane per entry, as k_run: the option
//     loop, the rows of step t; then each lane runs its env ahead from t + 1.
//   run-ahead ends with the env listed at (t', k') — its entry appended to the list, its state
//     stored for its run item — or with the env done with step K - 1.
//   A list chunk is pushed on the sub-problem's run queue by the writer whose entry completes it
//   (64 entries, counted per chunk in `fill`); the partial last chunk of every list of step t
//   by the wave that completes step t's count of classified envs (FC_CLS + t: every env listed
//   at t or finished t in place).  Waves take run items by ticket (one atomic on the queue head)
//   and wait on their ticket's slot; the deal goes first.  A sub-problem is done when all its
//   envs have finished step K - 1; waves holding tickets past the last item then leave.
//
// Coherence (MI355X_MICROARCH.md, inter-workgroup visibility): each XCD has its own L2, not
// coherent with the others, and a CU's L1 is not refreshed by other CUs' stores.  So the batch
// is split into sub-problems by XCD: chunk c belongs to sub-problem c % P, and a wave serves the
// sub-problem of the XCD it runs on (HW_REG_XCC_ID, mapped by a census at first use), so every
// hand-off stays inside one L2.  Producers store plainly (the L1 writes through) and wait for
// their stores (`s_waitcnt vmcnt(0)`) before the atomic that publishes them; every load of
// handed-off bytes (env state, list entries, queue slots, the MT codes and words, which an
// env's per-lane regeneration may have rewritten on another CU) bypasses L1 (sc1 loads, sc1
// LDS-DMA; regen_half_flow invalidates L1 first).  Nothing assumes blockIdx -> XCD, but the
// chunks of sub-problem x are stepped only by waves running on XCD x: a launch that places no
// workgroup on an XCD the census saw (a CU-masked stream, another partition layout) leaves that
// sub-problem unstepped, and no wave of it waits to time out.  k_flow_check, launched after every
// k_flow on its stream, compares each sub-problem's finished chunks with its chunk count and
// sets TG_ERR_FLOW on a mismatch.
//
// Every spin is bounded (FLOW_DEADLINE of the 100 MHz clock): a wave that waits longer sets
// TG_ERR_FLOW and its sub-problem's done word, so a bug ends the launch instead of hanging it.
#pragma once

constexpr int FLOW_MAX_K = REGEN_STEPS;  // steps per launch (the MT slack: k_regen every 16)
constexpr int FLOW_MAX_PARTS = 8;        // sub-problems: one per XCD
constexpr uint32_t Q_EMPTY = 0xFFFFFFFFu;
constexpr unsigned long long FLOW_DEADLINE = 400000000ull;  // 4 s of s_memrealtime
constexpr uint32_t E_FLOW = 1u << 30;    // TG_ERR_FLOW: a k_flow wait ran past FLOW_DEADLINE (a bug)
// a sub-problem's control words, each on a 128-B line of its own
enum : int {
  FC_INIT = 0,  // step-0 classification: next chunk to deal out
  FC_QHEAD,     // run queue: tickets taken
  FC_QTAIL,     //   slots pushed
  FC_FIN,       // chunks done with the launch (every env past step K - 1)
  FC_DONE,      // set when FC_FIN reaches the sub-problem's chunks (or on a deadline)
  FC_CLS,       // + t: envs classified for step t (listed at t, or finished t in place)
  FC_LTAIL = FC_CLS + FLOW_MAX_K,  // + t * NLIST + k: entries reserved in list (t, k)
  FC_N = FC_LTAIL + FLOW_MAX_K * NLIST
};
constexpr int FC_STRIDE = 32;  // int32 per control word: 128 B
constexpr int CTL_WORDS = FC_N * FC_STRIDE;
// per-wave LDS: the option loop's code window, or the classification's obs-row staging
constexpr int FLOW_WAVE_BYTES = (WIN_WAVE_BYTES > 64 * 9 * 8 ? WIN_WAVE_BYTES : 64 * 9 * 8);
static_assert(FLOW_WAVE_BYTES % 16 == 0, "16-B aligned windows for the LDS-DMA");
// queue item: step (4 bits), list (4 bits), entries - 1 (6 bits), list chunk (18 bits); or
// (0, Q_CLASSIFY, 0, chunk): a chunk made ready for its next round
constexpr int Q_CLASSIFY = 15;
static_assert(FLOW_MAX_K <= 16 && NLIST < Q_CLASSIFY, "item fields");
constexpr int FLOW_MAX_JCAP = 1 << 18;
// the first-in-line wave seals a partial list chunk after waiting this long with nothing to run
// (s_memrealtime ticks: 10 ns)
#ifndef TG_FLOW_SEAL_AFTER
#define TG_FLOW_SEAL_AFTER 200
#endif
constexpr unsigned long long FLOW_SEAL_AFTER = TG_FLOW_SEAL_AFTER;

struct Flow {
  int32_t* ctl;      // [P][CTL_WORDS] this launch's control words (zero at launch)
  uint32_t* q;       // [P][qcap] run items (Q_EMPTY until pushed)
  int32_t* fill;     // [P][FLOW_MAX_K][NLIST][jcap] entries written per list chunk (zero)
  int32_t* list;     // [P][FLOW_MAX_K][NLIST][lcap] env indices
  int32_t* outst;    // [C] envs of chunk c listed in its current round whose option has not run
  int32_t* cstep;    // [N] the env's next step (written by its run item, or K by its round)
  // the other parity's control words, run queue and fill counters: the previous launch's,
  // zeroed here for the next one (grid-stride, at the start)
  int32_t* ctl_next;
  uint32_t* q_next;
  int32_t* fill_next;
  uint32_t* refill;  // k_regen's lists (list c % SHARDS, as k_classify's shards)
  int32_t* rcnt;
  int64_t rcap, qcap, jcap, lcap;
  int32_t seal_below;  // idle seals only below this list chunk (cxm: later entries still fit)
  int32_t C, P, K;   // chunks, sub-problems, steps
  uint32_t xmap;     // nibble x: the sub-problem of XCC id x (0xF: none)
  int32_t skip;      // test hook (TG_FLOW_SKIP_PART): this sub-problem's waves leave at once, as
                     // if its XCD had no workgroup (k_flow_check must flag it); -1: none
  uint32_t* dbg;     // TG_FLOW_DBG builds: per-wave progress in mapped host memory (else null)
  uint32_t* dbgc;    // TG_FLOW_DBG builds: [C][16] classifications, [P][16][NLIST][jcap] runs
  uint32_t* dbgl;    // TG_FLOW_DBG builds: event log (count at [0], 32-B records from [16])
};
// the rollout's outputs, step-major [K][N] (obs_stride 0: one scratch row set for all steps)
struct FlowIO {
  int32_t* actions;  // may be null
  double* obs;
  int64_t obs_stride;
  int32_t* reward;
  uint8_t* valid;
  uint8_t* done;
  uint64_t a0;       // the policy's action seed
  int64_t t0;        // the policy's step index of step 0
  uint32_t tb;       // the handle's step count at step 0 (episode start / length bookkeeping)
};

__device__ __forceinline__ int32_t* fcw(int32_t* ctl, int w) { return ctl + w * FC_STRIDE; }
// the envs of sub-problem x: those of its 64-env chunks x, x + P, ... below C (the last chunk of
// the batch may be partial)
__host__ __device__ __forceinline__ int32_t flow_envs(int32_t C, int P, int64_t n, int x) {
  const int32_t Cx = (C - x + P - 1) / P;
  return Cx <= 0 ? 0 : Cx * 64 - ((C - 1) % P == x ? (int32_t)((int64_t)C * 64 - n) : 0);
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int32_t ld_sc1(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 B at byte offset off of base, past this CU's L1 (buffer_load_dwordx4 ... sc1)
__device__ __forceinline__ uint4 ld16_sc1(const void* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /* sc1 */);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
// write-through (sc1) stores of handed-off bytes: they leave the CU for the XCD's L2 before the
// storing wave's `s_waitcnt vmcnt(0)` lets it publish them (plain stores were seen stale by the
// consumer: the bring-up runs read unwritten list entries)
__device__ __forceinline__ void st_sc1(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st16_sc1(void* base, uint32_t off, uint4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, -1, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void st_ep_sc1(int2* p, int64_t i, int2 v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p + i),
                     (uint64_t)(uint32_t)v.x | ((uint64_t)(uint32_t)v.y << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 d2u4(double2 d) {
  const uint64_t a = (uint64_t)__double_as_longlong(d.x), b = (uint64_t)__double_as_longlong(d.y);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}
__device__ __forceinline__ double2 ld_ang_sc1(const double2* a, int64_t i) {
  const uint4 v = ld16_sc1(a, (uint32_t)i * 16u);
  return make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
}
__device__ __forceinline__ int2 ld_ep_sc1(const int2* p, int64_t i) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p + i), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
}
// the 100 MHz constant clock, read where it stands (volatile: never hoisted out of a spin)
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x;
}

#ifdef TG_FLOW_DBG
#include "tg_flow_diag.h"  // (diagnostic builds only: the bring-up instrumentation)
#else
// the product: every diagnostic hook is a no-op
#define FLOW_DBG(code, a, b, c) (void)0
#define FLOW_EV(ty, a, b, c, d) (void)0
#define FLOW_EV_WAVE(ty, a, b) (void)0
#define FLOW_EV_LANE(ty, a, b, c, d) (void)0
#define FLOW_DIAG_WAVE_STATE (void)0
#define FLOW_DIAG_PUSH(t, k, j) (void)0
#define FLOW_DIAG_RUN(item, i, live, mcnt, tail, lidx, j) (void)0
#define FLOW_DIAG_TAKE(item, h) (void)0
#define FLOW_DIAG_PATH(p) (void)0
#define FLOW_DIAG_CLASSIFY(c, t) (void)0
#define FLOW_DIAG_TAIL(v) (void)0
#endif

#ifndef TG_FLOW_TU  // (launched by tg_amd.hip's host code: the main unit only)
// the XCC ids the device's workgroups run on (one bit each): the flow's sub-problems
__global__ void k_census(uint32_t* mask) {
  if (threadIdx.x == 0) atomicOr(mask, 1u << (xcc_id() & 31u));
}
// after every k_flow launch, on its stream (one wave): a sub-problem whose chunks did not all
// finish the launch sets TG_ERR_FLOW (no wave ran on its XCD; see "Coherence" above)
__global__ void k_flow_check(const int32_t* __restrict__ ctl, int P, int32_t C,
                             uint32_t* __restrict__ err_or) {
  const int x = (int)threadIdx.x;
  if (x < P) {
    const int Cx = (C - x + P - 1) / P;
    if (Cx > 0 && ctl[(int64_t)x * CTL_WORDS + FC_FIN * FC_STRIDE] != Cx) atomicOr(err_or, E_FLOW);
  }
}
#endif

// 4 waves per SIMD (<= 128 VGPRs; built without MachineLICM, tg_flow.hip) — r05j A/B (round 5's
// chunk form): uniform 0.1111 vs 0.1163 ms per step at 3 waves, masked 0.3309 vs 0.3491
template <bool AR, int POL>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(4))) void k_flow(Soa S, int64_t n, Level L,
                                                const uint32_t* __restrict__ grid, FlowIO io,
                                                EpQueue eq, Flow f, int64_t g0,
                                                unsigned long long* __restrict__ stats, int nstat,
                                                uint32_t* __restrict__ err_or,
                                                unsigned long long* __restrict__ ks) {
  const unsigned long long kt0 = kst_begin(ks);
  const unsigned long long t_start = realtime();
  // the previous launch's control words, queue and fill counters, zeroed for the next launch
  {
    const int64_t gt = (int64_t)blockIdx.x * BLOCK + threadIdx.x, gs = (int64_t)gridDim.x * BLOCK;
    for (int64_t w = gt; w < (int64_t)f.P * FC_N; w += gs) f.ctl_next[w * FC_STRIDE] = 0;
    for (int64_t w = gt; w < (int64_t)f.P * f.qcap; w += gs) f.q_next[w] = Q_EMPTY;
    const int64_t nf = (int64_t)f.P * FLOW_MAX_K * NLIST * f.jcap;
    for (int64_t w = gt; w < nf; w += gs) f.fill_next[w] = 0;
  }
  __shared__ uint4 flds[((BLOCK / 64) * FLOW_WAVE_BYTES + MAX_CELLS + 4 * MK_MAX_WORDS) / 16];
  __shared__ uint32_t ltrig[12];
  uint8_t* const wall = reinterpret_cast<uint8_t*>(flds);
  uint32_t* const lgrid = reinterpret_cast<uint32_t*>(wall + (BLOCK / 64) * FLOW_WAVE_BYTES);
  uint32_t* const lmk = lgrid + grid_words(L.W, L.H);
  stage_cells<BLOCK>(lgrid, ltrig, grid, L, lmk);  // the only barrier
  const uint32_t* const trig = ltrig;
  const Map m{reinterpret_cast<const uint8_t*>(lgrid), L.W, L.H, L.masks ? lmk : nullptr};

  const int lane = threadIdx.x & 63;
  uint8_t* const warea = wall + (threadIdx.x >> 6) * FLOW_WAVE_BYTES;
  const int x = (int)((f.xmap >> (4u * (xcc_id() & 7u))) & 0xFu);
  FLOW_DBG(1, x, 0, 0);
  if (x >= f.P || x == f.skip) {  // an XCD the census did not see: no sub-problem (the workgroup)
    kst_end(ks, kt0);
    return;
  }
  const int P = f.P, K = f.K;
  const int Cx = (f.C - x + P - 1) / P;  // chunks x, x + P, ... below C
  if (Cx <= 0) {  // a batch of fewer chunks than sub-problems
    kst_end(ks, kt0);
    return;
  }
  const int32_t nx = flow_envs(f.C, P, n, x);  // the sub-problem's envs
  int32_t* const ctl = f.ctl + (int64_t)x * CTL_WORDS;
  uint32_t* const q = f.q + (int64_t)x * f.qcap;
  int32_t* const fill = f.fill + (int64_t)x * FLOW_MAX_K * NLIST * f.jcap;
  int32_t* const list = f.list + (int64_t)x * FLOW_MAX_K * NLIST * f.lcap;
  const int64_t slot = (int64_t)blockIdx.x % nstat;
  FLOW_DIAG_WAVE_STATE;
  if (lane == 0) FLOW_EV(10, x, 0, 0, 0);

  // a run item on the queue (by the lane that calls it): chunk j of list (t, k), cnt entries
  auto push = [&](int t, int k, int j, int cnt) {
    FLOW_DIAG_PUSH(t, k, j);
    const int at = atomicAdd(fcw(ctl, FC_QTAIL), 1);
    const uint32_t item = ((uint32_t)t << 28) | ((uint32_t)k << 24) | ((uint32_t)(cnt - 1) << 18) | (uint32_t)j;
    FLOW_EV(4, item, at, 0, x);
    if ((int64_t)at < f.qcap) st_sc1(q + at, item);
    else atomicOr(err_or, E_FLOW);  // (capacity is the bound of the pushes: unreachable)
  };
  // add to list chunk j's fill word; the adder that completes it pushes it.  The low byte counts
  // entries written (a sealed chunk's missing places are added by its sealer), bits 8+ hold a
  // sealed chunk's entry count (0: a full chunk of 64)
  auto fill_add = [&](int t, int k, int j, int add) {
    const int nv = atomicAdd(&fill[(int64_t)(t * NLIST + k) * f.jcap + j], add) + add;
    if ((nv & 0xFF) == 64) push(t, k, j, (nv >> 8) ? (nv >> 8) : 64);
  };
  // seal the partial chunk at list (t, k)'s tail: its tail moves to the next chunk (one CAS,
  // so no reservation lands in the sealed places), and the chunk is pushed with the entries it
  // holds once they are written.  `reserve`: only below the first cxm chunks (every later entry
  // then still fits lcap); the flush of a finished step seals unconditionally
  auto seal = [&](int t, int k, bool reserve) -> bool {
    int32_t* const lt = fcw(ctl, FC_LTAIL + t * NLIST + k);
    const int v = ld_sc1(lt);
    if (!(v & 63) || (reserve && (v >> 6) >= f.seal_below)) return false;
    if (atomicCAS(lt, v, (v | 63) + 1) != v) return false;
    const int r = v & 63;
    fill_add(t, k, v >> 6, (64 - r) + (r << 8));
    return true;
  };
  auto step_io = [&](int t) {
    return StepIO{nullptr, io.obs + (int64_t)t * io.obs_stride, io.reward + (int64_t)t * n,
                  io.valid + (int64_t)t * n, io.done + (int64_t)t * n, nullptr, POL, io.a0,
                  io.t0 + t, io.tb + (uint32_t)t};
  };

  // one run item: chunk j of list (t, k), cnt entries, one lane per entry, as k_run: the option
  // loops of step t, the rows and the state; each lane then records its env's next step
  // (cstep) and decrements its env's chunk's `outst`; returns the lanes whose env's chunk became
  // ready (its chunk in cl)
  auto run = [&](uint32_t item, int& cl) -> unsigned long long {
    const int t = (int)(item >> 28), k = (int)((item >> 24) & 15u), j = (int)(item & 0x3FFFFu);
    // a cheap guard: an item or entry out of range is a protocol bug; it sets
    // TG_ERR_FLOW and runs nothing instead of addressing memory with it
    const bool item_ok = t < K && k < NLIST && (int64_t)j < f.jcap;
    const int lidx = item_ok ? t * NLIST + k : 0;
    FLOW_DIAG_TAIL(tail);
    const int mcnt = item_ok ? (int)((item >> 18) & 63u) + 1 : 0;
    bool live = lane < mcnt;
    int64_t i = 0;
    if (live) i = ld_sc1(list + (int64_t)lidx * f.lcap + 64 * j + lane);
    const bool bad = live && (i < 0 || i >= n || (int)((i >> 6) % P) != x);
    if (lane == 0 && (!item_ok || __ballot(bad))) atomicOr(err_or, E_FLOW);
    live = live && !bad;
    FLOW_DIAG_RUN(item, i, live, mcnt, tail, lidx, j);
    const StepIO st = step_io(t);
    StepResult r{0, 0, 0, 0};
    Env e;
    e.mti = 0u;
    int2 ep = make_int2(0, 0);
    uint32_t draws = 0;
    int lregen = 0;
    if (live) {
      unpack(ld16_sc1(S.st4, (uint32_t)i * 16u), ld_ang_sc1(S.ang, i), e);
      ep = ld_ep_sc1(S.ep, i);
      RngCodesT<true> rng(S.mt + i * MT_STORE, S.mc + i * MT_CODES, e.mti, (lds_u8*)warea);
      rng.prime();
      if (k != O_GO_LEFT && k != O_GO_RIGHT && k != O_INTERACT) __builtin_amdgcn_s_setprio(PRIO_SLOW);
      if (k != L_RESET) run_option(L, trig, m, e, k, rng, r);  // k is wave-uniform
      r.done = is_done(e);
      finish_step<AR, false, false>(level_div(L), e, rng, i, r, ep, st);  // valid: at listing
      e.mti = rng.finish();
      draws = rng.draws;
      lregen = (int)rng.regens;
      if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
    }
    if (AR) record_episodes(live && r.done, g0 + i, ep, st.tstep, eq, stats, slot);
    if (live) {
      st16_sc1(S.st4, (uint32_t)i * 16u, pack(e));
      st16_sc1(S.ang, (uint32_t)i * 16u, d2u4(make_double2(e.ang0, e.ang1)));
      st_ep_sc1(S.ep, i, ep);
      st_sc1(f.cstep + i, t + 1);
    }
    __builtin_amdgcn_s_setprio(0);
    wave_stats(stats, 0, 0, r.ticks, (int)draws, AR ? (live && r.done) : 0,
               __ballot(lregen != 0) ? wave_sum(lregen) : 0, true, slot);
    // this wave's stores first, then the chunks' counters: the lane that takes its env's chunk
    // to 0 hands the chunk to the wave (its next round below, in lane order)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (live) old = atomicSub(&f.outst[i >> 6], 1);
    const unsigned long long ready = __ballot(live && old == 1);
    if (lane == 0) FLOW_EV(7, item, (uint32_t)__popcll(ready), (uint32_t)mcnt, x);
    cl = (int)(i >> 6);
    return ready;
  };

  // One round of chunk c: every env of the chunk not yet done with step K - 1, one lane per env
  // (coalesced loads), at its own next step (0 in the first round, the deal; later the step
  // after the one its last option ran at, cstep).  Run-ahead (TG/:91-96 -> OP/:20-36: env i's
  // step t + 1 depends on env i's step t alone): each lane classifies its env for its step t,
  // t + 1, ... as k_classify would — the policy's action, can_run — and finishes every step
  // whose option cannot run in place (reward None, state and MT stream untouched, OP/:22-23),
  // until an option can run (the env is listed at (t', k)) or the launch's last step is past.
  // The lanes advance in lockstep, so the rows of one step's lanes are adjacent.  The state is
  // the same at every step of a run-ahead, so what depends on it alone is evaluated once: the 9
  // options' can_run (available_mask, TG/:83-89), the obs row (get_state, TG/:94), done, and
  // the policy's hash keyed by the env alone (policy_action's inner two rounds).  An env
  // entering done with auto-reset on and no option to run goes on L_RESET (first round only: a
  // run with auto-reset resets the env it finishes).  Returns the envs listed (0: the chunk is
  // done with the launch).
  auto round = [&](int c, bool first) -> int {
    const int64_t i = (int64_t)c * 64 + lane;
    bool live = i < n;
    int t = 0;
    if (live && !first) t = ld_sc1(f.cstep + i);
    live = live && t < K;
    Env e;
    e.mti = 0u;
    e.ang0 = e.ang1 = 0.0;
    int2 ep = make_int2(0, 0);
    if (live) {
      unpack(ld16_sc1(S.st4, (uint32_t)i * 16u), ld_ang_sc1(S.ang, i), e);
      ep = ld_ep_sc1(S.ep, i);
    }
    const uint32_t f0 = e.f, mt0 = e.mti;
    // a stale MT half not listed yet goes on k_regen's list c % SHARDS (MT_LISTED), as k_classify
    const bool stale = live && (e.mti & (MT_STALE | MT_LISTED)) == MT_STALE;
    const unsigned long long sb = __ballot(stale);
    int sbase = 0;
    if (sb && lane == 0) sbase = atomicAdd(&f.rcnt[(c % SHARDS) * CTR_STRIDE], __popcll(sb));
    if (stale) e.mti |= MT_LISTED;
    const int tf = t;  // the lane's first classified step
    int kl = -1, nvalid = 0;
    if (live) {
      const uint32_t avail = available_mask(L, m, e);
      const bool done0 = is_done(e);
      double orow[9];
      observe(L, e, orow);
      const uint64_t hb = sm64(io.a0 ^ sm64((uint64_t)(g0 + i)));
      const int nav = __popc(avail);
      while (t < K) {
        const uint64_t hh = sm64(hb ^ (uint64_t)(io.t0 + t));
        int act = (int)(hh % 9ull);  // policy_action, from the hoisted mask and hash
        if (POL == TG_POLICY_MASKED && nav) {
          uint32_t kk = (uint32_t)(hh % (uint64_t)nav), mm = avail;
          while (kk--) mm &= mm - 1u;
          act = __ffs(mm) - 1;
        }
        if (io.actions) io.actions[(int64_t)t * n + i] = act;
        const int k = option_index(act);
        const bool runs = k >= 0 && ((avail >> k) & 1u);
        if (k < 0) e.f |= E_ACTION;
        const StepIO st = step_io(t);
        st.valid[i] = (uint8_t)runs;
        if (runs) {
          kl = k;
          nvalid = 1;
          break;
        }
        if (AR && done0) {
          kl = L_RESET;
          break;
        }
        st.reward[i] = 0;  // reward None (finish_step of a step whose option did not run)
        st.done[i] = (uint8_t)done0;
        store_obs(st.obs, i, orow);
        ++t;
      }
      if (e.f & E_MASK) atomicOr(err_or, e.f & E_MASK);
    }
    FLOW_EV_WAVE(14, c, 0);  // (timing log: the run-ahead done)
    const int tl = t;  // the listing step, or K
    const bool listed = live && tl < K;
    // the entries: lanes grouped by list (tl, k), one reservation per group (one atomic
    // instruction of the groups' leads)
    const int key = listed ? tl * NLIST + kl : -1;
    int rank = 0, lead = 0, nb = 0, base = 0;
    {
      unsigned long long pend = __ballot(listed);
      while (pend) {
        const int first_l = __ffsll((long long)pend) - 1;
        const int k0 = __builtin_amdgcn_readlane(key, first_l);
        const unsigned long long b = __ballot(key == k0);
        if (key == k0) {
          rank = __popcll(b & ((1ull << lane) - 1ull));
          lead = first_l;
          nb = __popcll(b);
        }
        pend &= ~b;
      }
    }
    if (listed && lane == lead) base = atomicAdd(fcw(ctl, FC_LTAIL + key), nb);
    const int cnt = __popcll(__ballot(listed));
    // the handed-off bytes: refill entries, the state (when classification changed its flags:
    // the env's run item loads it), the finished envs' next step (K), the list entries, the
    // chunk's count; then publish: this wave's stores first; then the fill counts (the writer
    // whose entries complete a list chunk pushes it), the steps classified (the wave that
    // completes a step's count flushes its partial list chunks), a finished chunk
    sbase = __builtin_amdgcn_readlane(sbase, 0);
    if (stale)
      f.refill[(c % SHARDS) * f.rcap + sbase + __popcll(sb & ((1ull << lane) - 1ull))] =
          (uint32_t)i | (mt_half(e.mti & MT_POS_MASK) ? 0x80000000u : 0u);
    if (live && (e.f != f0 || e.mti != mt0)) st16_sc1(S.st4, (uint32_t)i * 16u, pack(e));
    if (live && !listed) st_sc1(f.cstep + i, K);
    const int gbase = __shfl(base, lead, 64);
    if (listed) st_sc1(list + (int64_t)key * f.lcap + gbase + rank, (int32_t)i);
    if (cnt && lane == 0) st_sc1(f.outst + c, cnt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (listed && lane == lead) {
      const int j0 = base >> 6, in0 = min(nb, 64 - (base & 63));
      fill_add(tl, kl, j0, in0);
      if (nb > in0) fill_add(tl, kl, j0 + 1, nb - in0);
    }
    // steps classified: tf .. min(tl, K - 1) (the listing step's entry is written)
    const int thi = live ? min(tl, K - 1) : -1;
    const int s0 = __builtin_amdgcn_readfirstlane(wave_min_i(live && tf <= thi ? tf : K));
    const int s1 = __builtin_amdgcn_readfirstlane(wave_max(thi));
    for (int sp = s0; sp <= s1; ++sp) {
      const int cs = __popcll(__ballot(live && tf <= sp && sp <= thi));
      int last = 0;
      if (cs && lane == 0) last = atomicAdd(fcw(ctl, FC_CLS + sp), cs) + cs == nx;
      if (__builtin_amdgcn_readlane(last, 0) && lane < NLIST) seal(sp, lane, false);  // step sp's partial chunks
    }
    wave_stats(stats, live ? thi - tf + 1 : 0, nvalid, 0, 0, 0, 0, false, slot);
    FLOW_EV_WAVE(15, c, cnt);  // (timing log: published)
    return cnt;
  };

  // The wave's work loop: one unit per iteration, chosen by wave-uniform values only (each read
  // back with readfirstlane, so the loop's branches stay scalar: with the work in nested loops
  // whose exits the compiler did not prove uniform, round 5's bring-up saw a divergent loop
  // nest).  In order: the first rounds of the chunks, dealt out by a counter; then the queue:
  // run items, and the chunks other waves' run items made ready (a run item's envs come from up
  // to 64 chunks; the first it readies runs its next round in this wave, the others go on the
  // queue for any wave).  A chunk whose round lists no env is done with the launch.
  bool deal = true;
  int cl = 0;  // (per lane) the chunk of the lane's env in the last run item
  while (true) {
    int c;
    bool first = false;
    if (deal) {
      int j = 0;
      if (lane == 0) j = atomicAdd(fcw(ctl, FC_INIT), 1);
      j = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(j, 0));
      if (j >= Cx) {
        deal = false;
        continue;
      }
      FLOW_DIAG_PATH(3);
      FLOW_EV_WAVE(16, j, 0);  // (timing log: a deal chunk)
      c = x + P * j;
      first = true;
    } else {
      // an item by ticket: wait for its slot (lane 0 polls, the wave reads its answer)
      int h = 0;
      if (lane == 0) h = atomicAdd(fcw(ctl, FC_QHEAD), 1);
      h = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(h, 0));
      FLOW_DBG(2, h, x, 0);
      if (lane == 0) FLOW_EV(8, h, x, 0, 0);
      uint32_t item = Q_EMPTY;
      int stop = 0;
      unsigned long long t_wait = realtime();
      while (!stop) {
        uint32_t it = Q_EMPTY;
        int dn = 0, head = 0;
        if (lane == 0) {
          if ((int64_t)h < f.qcap) it = ld_sc1(q + h);
          if (it == Q_EMPTY) {
            dn = ld_sc1(fcw(ctl, FC_DONE));
            head = h == ld_sc1(fcw(ctl, FC_QTAIL));
          }
        }
        item = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(it, 0));
        dn = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(dn, 0));
        head = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(head, 0));
        if (item != Q_EMPTY || dn) {
          stop = 1;
        } else if (head && realtime() - t_wait > FLOW_SEAL_AFTER) {
          // first in line and nothing to run: seal the partial list chunk of the lowest step
          // (the fullest of that step's lists).  Besides latency this is what keeps a launch
          // live: an env listed at a far step waits for that step's flush, which waits for a
          // chunk-mate's next round, which waits for the far env's run (tests/native/flow_sim)
          int best = -1, bt = K, bk = 0;
          for (int t0 = 0; t0 < K && best < 0; t0 += 64 / NLIST) {
            const int tc = t0 + lane / NLIST, kc = lane % NLIST;
            int r = -1;
            if (lane < (64 / NLIST) * NLIST && tc < K) {
              const int v = ld_sc1(fcw(ctl, FC_LTAIL + tc * NLIST + kc));
              if ((v & 63) && (v >> 6) < f.seal_below) r = ((K - tc) << 6) | (v & 63);
            }
            best = wave_max(r);
            if (best >= 0) {
              const unsigned long long bl = __ballot(r == best);
              const int bl0 = __ffsll((long long)bl) - 1;
              bt = __builtin_amdgcn_readlane(tc, bl0);
              bk = __builtin_amdgcn_readlane(kc, bl0);
            }
          }
          if (best >= 0 && lane == 0) seal(bt, bk, true);
          t_wait = realtime();
        } else if (realtime() - t_start > FLOW_DEADLINE) {
          if (lane == 0) {
            atomicOr(err_or, E_FLOW);
            __hip_atomic_store(fcw(ctl, FC_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          stop = 1;
        } else {
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (item == Q_EMPTY) break;
      FLOW_DBG(3, h, item, x);
      if (lane == 0) FLOW_EV(5, h, item, x, 0);
      FLOW_DIAG_TAKE(item, h);
      FLOW_DIAG_PATH(2);
      if (((item >> 24) & 15u) == Q_CLASSIFY) {  // a chunk another wave's run item made ready
        c = (int)(item & 0x3FFFFu);
        if (c >= f.C || c % P != x) {  // (the run item's guard, for these items)
          if (lane == 0) atomicOr(err_or, E_FLOW);
          continue;
        }
      } else {
        const unsigned long long rd = run(item, cl);
        // (readfirstlane returns int: each half is cast back to 32 bits before it widens, or
        // lane 31's bit sign-extends over lanes 32-63)
        const unsigned long long ready =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(rd >> 32)) << 32) |
            (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rd);
        if (!ready) continue;
        // the first readied chunk's next round runs here, the others by whichever waves take them
        const int l0 = __ffsll((long long)ready) - 1;
        c = __builtin_amdgcn_readlane(cl, l0);
        if (((ready >> lane) & 1ull) && lane != l0) push(0, Q_CLASSIFY, cl, 1);
      }
    }
    FLOW_DIAG_CLASSIFY(c, 0);
    if (__builtin_amdgcn_readfirstlane(round(c, first)) == 0 && lane == 0 &&
        atomicAdd(fcw(ctl, FC_FIN), 1) + 1 == Cx)  // the chunk is done with the launch
      __hip_atomic_store(fcw(ctl, FC_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  FLOW_DBG(9, 0, 0, 0);
  if (lane == 0) FLOW_EV(9, x, 0, 0, 0);
  kst_end(ks, kt0);
}
