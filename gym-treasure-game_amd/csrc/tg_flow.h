// tg_flow.h — k_flow: tg_rollout's K steps in ONE launch, each 64-env chunk advancing to its
// next step as soon as its own envs have finished the current one (TG_MODE_FLOW, §8f row 3).
// Included by tg_amd.hip inside its anonymous namespace, after the per-step kernels whose
// pieces it reuses (RngCodesT, finish_step, store_obs_wave, record_episodes, wave_stats).
//
// Why: the reference's step is per env (TG/:91-96 -> OP/:20-36): env i's step
// t + 1 depends on env i's step t only.  The per-step kernels put a batch-wide barrier after
// every step, so a step costs one maximal option chain (k_run ends with its slowest option
// waves, ~50 us at the uniform policy, while only ~3.4 waves per SIMD carry work).  Here a chunk
// whose envs are all done with step t is classified for step t + 1 at once, by the wave that
// finished its last env, so chains of different steps overlap and the SIMDs stay busy.
//
// Work, per sub-problem (one per XCD, below):
//   classify (c, t): chunk c (envs 64c .. 64c + 63) at step t, one lane per env, as k_classify:
//     the policy's action, can_run, the rows of the envs whose option cannot run (coalesced,
//     through LDS), the stale-MT-half listing for k_regen; the rest are appended to the list
//     (t, k) of their option k (L_RESET: entering done with auto-reset on), and the chunk's
//     `outst` counter is set to their number.
//   run (t, k, j): 64-entry chunk j of list (t, k), one lane per entry, as k_run: the option
//     loop, the rows, the state; each lane then decrements its env's chunk's `outst`, and the
//     lane that takes it to 0 hands the chunk to its wave, which classifies it for t + 1.
//   A list chunk is pushed on the sub-problem's run queue by the writer whose entries complete
//   it (64 entries, counted per chunk in `fill`); the partial last chunk of every list of step t
//   by the wave that classifies step t's last chunk.  Waves take run items by ticket (one
//   atomic on the queue head) and wait on their ticket's slot; the chunks' step-0 classification
//   is dealt out first by a counter.  A sub-problem is done when all its chunks have finished
//   step K - 1; waves holding tickets past the last item then leave.
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
constexpr int Q_CLASSIFY = 15;  // the list field of a queue item that is a chunk to classify
constexpr unsigned long long FLOW_DEADLINE = 400000000ull;  // 4 s of s_memrealtime
constexpr uint32_t E_FLOW = 1u << 30;    // TG_ERR_FLOW: a k_flow wait ran past FLOW_DEADLINE (a bug)
// a sub-problem's control words, each on a 128-B line of its own
enum : int {
  FC_INIT = 0,  // step-0 classification: next chunk to deal out
  FC_QHEAD,     // run queue: tickets taken
  FC_QTAIL,     //   slots pushed
  FC_FIN,       // chunks done with step K - 1
  FC_DONE,      // set when FC_FIN reaches the sub-problem's chunks (or on a deadline)
  FC_CLS,       // + t: chunks classified for step t
  FC_LTAIL = FC_CLS + FLOW_MAX_K,  // + t * NLIST + k: entries reserved in list (t, k)
  FC_N = FC_LTAIL + FLOW_MAX_K * NLIST
};
constexpr int FC_STRIDE = 32;  // int32 per control word: 128 B
constexpr int CTL_WORDS = FC_N * FC_STRIDE;
// per-wave LDS: the option loop's code window, or the classification's obs-row staging
constexpr int FLOW_WAVE_BYTES = (WIN_WAVE_BYTES > 64 * 9 * 8 ? WIN_WAVE_BYTES : 64 * 9 * 8);
static_assert(FLOW_WAVE_BYTES % 16 == 0, "16-B aligned windows for the LDS-DMA");
// queue item: step (4 bits), list (4 bits), list chunk (24 bits); or step, Q_CLASSIFY, chunk
static_assert(FLOW_MAX_K <= 16 && NLIST < Q_CLASSIFY, "item fields");

struct Flow {
  int32_t* ctl;      // [P][CTL_WORDS] this launch's control words (zero at launch)
  uint32_t* q;       // [P][qcap] run items (Q_EMPTY until pushed)
  int32_t* fill;     // [P][FLOW_MAX_K][NLIST][jcap] entries written per list chunk (zero)
  int32_t* list;     // [P][FLOW_MAX_K][NLIST][lcap] env indices
  int32_t* outst;    // [C] envs of chunk c whose option is still running this step
  // the other parity's control words, run queue and fill counters: the previous launch's,
  // zeroed here for the next one (grid-stride, at the start)
  int32_t* ctl_next;
  uint32_t* q_next;
  int32_t* fill_next;
  uint32_t* refill;  // k_regen's lists (list c % SHARDS, as k_classify's shards)
  int32_t* rcnt;
  int64_t rcap, qcap, jcap, lcap;
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
#endif

#ifndef TG_FLOW_TU  // (launched by tg_amd.hip's host code: the main unit only)
// the XCC ids the device's workgroups run on (one bit each): the flow's sub-problems
__global__ void k_census(uint32_t* mask) {
  if (threadIdx.x == 0) atomicOr(mask, 1u << (xcc_id() & 31u));
}
// after every k_flow launch, on its stream (one wave): a sub-problem whose chunks did not all
// finish step K - 1 sets TG_ERR_FLOW (no wave ran on its XCD; see "Coherence" above)
__global__ void k_flow_check(const int32_t* __restrict__ ctl, int P, int32_t C,
                             uint32_t* __restrict__ err_or) {
  const int x = (int)threadIdx.x;
  if (x < P) {
    const int Cx = (C - x + P - 1) / P;
    if (Cx > 0 && ctl[(int64_t)x * CTL_WORDS + FC_FIN * FC_STRIDE] != Cx) atomicOr(err_or, E_FLOW);
  }
}
#endif

// 4 waves per SIMD (<= 128 VGPRs; built without MachineLICM, tg_flow.hip: 123-131 VGPRs
// unconstrained) — r05j A/B: uniform 0.1111 vs 0.1163 ms per step at 3 waves, masked 0.3309 vs
// 0.3491
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
  int32_t* const ctl = f.ctl + (int64_t)x * CTL_WORDS;
  uint32_t* const q = f.q + (int64_t)x * f.qcap;
  int32_t* const fill = f.fill + (int64_t)x * FLOW_MAX_K * NLIST * f.jcap;
  int32_t* const list = f.list + (int64_t)x * FLOW_MAX_K * NLIST * f.lcap;
  const int64_t slot = (int64_t)blockIdx.x % nstat;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  FLOW_DIAG_WAVE_STATE;
  if (lane == 0) FLOW_EV(10, x, 0, 0, 0);

  // a run item on the queue (by the lane that calls it)
  auto push = [&](int t, int k, int j, int src) {
    FLOW_DIAG_PUSH(t, k, j);
    const int at = atomicAdd(fcw(ctl, FC_QTAIL), 1);
    FLOW_EV(4, ((uint32_t)t << 28) | ((uint32_t)k << 24) | (uint32_t)j, at, src, x);
    if ((int64_t)at < f.qcap) st_sc1(q + at, ((uint32_t)t << 28) | ((uint32_t)k << 24) | (uint32_t)j);
    else atomicOr(err_or, E_FLOW);  // (capacity is the bound of the pushes: unreachable)
  };
  auto step_io = [&](int t) {
    return StepIO{nullptr, io.obs + (int64_t)t * io.obs_stride, io.reward + (int64_t)t * n,
                  io.valid + (int64_t)t * n, io.done + (int64_t)t * n, nullptr, POL, io.a0,
                  io.t0 + t, io.tb + (uint32_t)t};
  };

  // classify chunk c for step t (k_classify's per-env work); returns the envs it listed
  auto classify = [&](int c, int t) -> int {
    const int64_t i = (int64_t)c * 64 + lane;
    const bool live = i < n;
    const StepIO st = step_io(t);
    uint4 s4 = make_uint4(0, 0, 0, 0);
    double2 a2 = make_double2(0.0, 0.0);
    int2 ep = make_int2(0, 0);
    if (live) {
      s4 = ld16_sc1(S.st4, (uint32_t)i * 16u);
      a2 = ld_ang_sc1(S.ang, i);
      ep = ld_ep_sc1(S.ep, i);
    }
    Env e;
    e.mti = 0u;
    int k = -1;
    bool runs = false;
    if (live) {
      unpack_st4(s4, e);
      FLOW_EV_WAVE(11, c, t);  // (timing log: the state loads returned)
      const int act = policy_action(L, m, e, POL, io.a0, g0 + i, io.t0 + t);
      if (io.actions) io.actions[(int64_t)t * n + i] = act;
      k = option_index(act);
      runs = k >= 0 && can_run(L, m, e, k);
      if (k < 0) e.f |= E_ACTION;
    }
    const bool rst = AR && live && !runs && is_done(e);  // entering done: reset (L_RESET)
    const int bk = runs ? k : rst ? L_RESET : -1;
    // The atomics that reserve this chunk's places go out first, their round trips overlapping
    // the rows below (each one on the chain cost a classification ~1 us, the r05h event log):
    // stale MT halves not listed yet go on k_regen's list c % SHARDS ...
    const bool stale = live && (e.mti & (MT_STALE | MT_LISTED)) == MT_STALE;
    const unsigned long long sb = __ballot(stale);
    int sbase = 0;
    if (sb && lane == 0) sbase = atomicAdd(&f.rcnt[(c % SHARDS) * CTR_STRIDE], __popcll(sb));
    if (stale) e.mti |= MT_LISTED;
    // ... and the listed lanes, grouped by list (rank in the group, its first lane and size),
    // reserve their entries
    const unsigned long long lb = __ballot(bk >= 0);
    const int cnt = __popcll(lb);
    int rank = 0, lead = 0, nb = 0;
    unsigned long long pend = lb;
    while (pend) {
      const int first = __ffsll((long long)pend) - 1;
      const int b0 = __builtin_amdgcn_readlane(bk, first);
      const unsigned long long b = __ballot(bk == b0);
      if (bk == b0) {
        rank = __popcll(b & lt_mask);
        lead = first;
        nb = __popcll(b);
      }
      pend &= ~b;
    }
    const int lidx = t * NLIST + (bk >= 0 ? bk : 0);
    int base = 0;
    if (bk >= 0 && lane == lead) base = atomicAdd(fcw(ctl, FC_LTAIL + lidx), nb);
    // every env's valid row, coalesced (as k_classify); the rows of the envs whose option cannot
    // run: reward None, state unchanged (TG/:91-96, OP/:22-23)
    if (live) st.valid[i] = (uint8_t)runs;
    const bool fin = live && !runs && !rst;
    double orow[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (fin) {
      e.ang0 = a2.x;
      e.ang1 = a2.y;
      Rng rng(S.mt + i * MT_STORE, e.mti, S.mc + i * MT_CODES);  // no draws without a reset
      StepResult r{0, 0, (int)is_done(e), 0};
      finish_step<false, false, false>(L, e, rng, i, r, ep, st, orow);
    }
    if (fin && (e.f & E_MASK)) atomicOr(err_or, e.f & E_MASK);
    store_obs_wave(st.obs, (int64_t)c * 64, __ballot(fin), orow, reinterpret_cast<double*>(warea));
    FLOW_EV_WAVE(12, c, t);  // (timing log: the rows issued)
    // the handed-off bytes: refill entries, list entries, the state, the chunk's count
    sbase = __builtin_amdgcn_readlane(sbase, 0);
    if (stale)
      f.refill[(c % SHARDS) * f.rcap + sbase + __popcll(sb & lt_mask)] =
          (uint32_t)i | (mt_half(e.mti & MT_POS_MASK) ? 0x80000000u : 0u);
    base = __shfl(base, lead, 64);
    if (bk >= 0) st_sc1(list + (int64_t)lidx * f.lcap + base + rank, (int32_t)i);
    if (live) {
      const uint4 s4n = pack(e);
      if (s4n.x != s4.x || s4n.y != s4.y || s4n.z != s4.z || s4n.w != s4.w)
        st16_sc1(S.st4, (uint32_t)i * 16u, s4n);
    }
    if (cnt && lane == 0) st_sc1(f.outst + c, cnt);
    // publish: this wave's stores first (with no listed env, the chain goes on with the chunk's
    // next step in this wave: its stores land first too); then the fill counts and the step's
    // classified-chunk count together (the flush reads only the list tails, reserved above)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FLOW_EV_WAVE(13, c, t);  // (timing log: the stores complete)
    int32_t* const fl = fill + (int64_t)lidx * f.jcap;
    const int j0 = base >> 6, in0 = min(nb, 64 - (base & 63));
    int f0 = 0, f1 = 0, last = 0;
    if (bk >= 0 && lane == lead) {
      f0 = atomicAdd(&fl[j0], in0) + in0;
      if (nb > in0) f1 = atomicAdd(&fl[j0 + 1], nb - in0) + (nb - in0);
    }
    if (lane == 0) last = atomicAdd(fcw(ctl, FC_CLS + t), 1) + 1 == Cx;
    if (bk >= 0 && lane == lead) {
      if (f0 == 64) push(t, bk, j0, 0);
      if (f1 == 64) push(t, bk, j0 + 1, 1);
    }
    wave_stats(stats, live ? 1 : 0, runs ? 1 : 0, 0, 0, 0, 0, false, slot);
    // the last chunk classified for step t flushes step t's partial list chunks
    if (lane == 0) FLOW_EV(2, c, t, cnt, x);
    if (__builtin_amdgcn_readlane(last, 0) && lane < NLIST) {
      const int tail = ld_sc1(fcw(ctl, FC_LTAIL + t * NLIST + lane));
      if (tail & 63) push(t, lane, tail >> 6, 2 | (tail << 8));
    }
    return cnt;
  };
  // one run item: the option loops of a 64-entry list chunk (k_run's per-env work); returns the
  // lanes whose env's chunk became ready (its chunk in cl)
  auto run = [&](uint32_t item, int& cl) -> unsigned long long {
      const int t = (int)(item >> 28), k = (int)((item >> 24) & 15u), j = (int)(item & 0xFFFFFFu);
      // a cheap guard: an item or entry out of range is a protocol bug; it sets
      // TG_ERR_FLOW and runs nothing instead of addressing memory with it
      const bool item_ok = t < K && k < NLIST && (int64_t)j < f.jcap;
      const int lidx = item_ok ? t * NLIST + k : 0;
      int tail = 0;
      if (lane == 0 && item_ok) tail = ld_sc1(fcw(ctl, FC_LTAIL + lidx));
      tail = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(tail, 0));
      const int mcnt = item_ok ? min(64, tail - 64 * j) : 0;
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
        finish_step<AR, false, false>(level_div(L), e, rng, i, r, ep, st);
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
      }
      __builtin_amdgcn_s_setprio(0);
      wave_stats(stats, 0, 0, r.ticks, (int)draws, AR ? (live && r.done) : 0,
                 __ballot(lregen != 0) ? wave_sum(lregen) : 0, true, slot);
      // this wave's stores first, then the chunks' counters: the lane that takes its env's chunk
      // to 0 hands the chunk to the wave (classified for t + 1 below, in lane order)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int old = 0;
      if (live) old = atomicSub(&f.outst[i >> 6], 1);
      if (live) FLOW_EV_LANE(3, item, (uint32_t)i, (uint32_t)old, (uint32_t)lane | ((uint32_t)mcnt << 8) | ((uint32_t)x << 16));
      unsigned long long ready = __ballot(live && old == 1);
      if (lane == 0) FLOW_EV(7, item, (uint32_t)__popcll(ready), (uint32_t)mcnt, x);
      cl = (int)(i >> 6);
      return ready;
  };

  // The wave's work loop: one unit of work per iteration, chosen by wave-uniform values only
  // (each read back with readfirstlane, so the loop's branches stay scalar: with the work in
  // nested loops whose exits the compiler did not prove uniform, it built a divergent loop
  // nest whose lanes could sit in different iterations, and a wave re-classified chunk 0
  // forever).  In order: a chunk carried to its next step (none of its envs ran an option, or
  // the first chunk the wave's last run item completed), the step-0 chunks dealt out by a
  // counter, then the queue: run items and the chunks other waves' run items completed (a run
  // item's envs come from up to 64 chunks, and late in a step many of them complete together:
  // classified by their one wave in turn they left the others waiting on the queue, 58 % of
  // the waves' time in the r05g event log)
  bool phase0 = true;
  int cl = 0;                    // (per lane) the chunk of the lane's env in the last run item
  int cc = -1, ct = 0;           // the carried chunk and its step
  while (true) {
    int c, t;
    FLOW_DIAG_PATH(cc >= 0 ? 1 : phase0 ? 3 : 2);
    if (cc >= 0) {
      c = cc;
      t = ct;
      cc = -1;
    } else if (phase0) {
      int j = 0;
      if (lane == 0) j = atomicAdd(fcw(ctl, FC_INIT), 1);
      j = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(j, 0));
      if (j >= Cx) {
        phase0 = false;
        continue;
      }
      c = x + P * j;
      t = 0;
    } else {
      // an item by ticket: wait for its slot (lane 0 polls, the wave reads its answer)
      int h = 0;
      if (lane == 0) h = atomicAdd(fcw(ctl, FC_QHEAD), 1);
      h = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(h, 0));
      FLOW_DBG(2, h, x, 0);
      if (lane == 0) FLOW_EV(8, h, x, 0, 0);
      uint32_t item = Q_EMPTY;
      int stop = 0;
      while (!stop) {
        uint32_t it = Q_EMPTY;
        int dn = 0;
        if (lane == 0) {
          if ((int64_t)h < f.qcap) it = ld_sc1(q + h);
          if (it == Q_EMPTY) dn = ld_sc1(fcw(ctl, FC_DONE));
        }
        item = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(it, 0));
        dn = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(dn, 0));
        if (item != Q_EMPTY || dn) {
          stop = 1;
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
      t = (int)(item >> 28);
      if (((item >> 24) & 15u) == Q_CLASSIFY) {  // a chunk another wave's run item completed
        c = (int)(item & 0xFFFFFFu);
        if (t >= K || c >= f.C || c % P != x) {  // (the guard above, for classification items)
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
        FLOW_DBG(4, h, item, (uint32_t)__popcll(ready));
        if (!ready) continue;
        ++t;
        if (t >= K) {  // chunks done with the last step
          if (lane == 0) {
            const int nr = __popcll(ready);
            if (atomicAdd(fcw(ctl, FC_FIN), nr) + nr == Cx)
              __hip_atomic_store(fcw(ctl, FC_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          continue;
        }
        // the first completed chunk is classified here, the others by whichever waves take them
        const int l0 = __ffsll((long long)ready) - 1;
        c = __builtin_amdgcn_readlane(cl, l0);
        if (((ready >> lane) & 1ull) && lane != l0) push(t, Q_CLASSIFY, cl, 3);
      }
    }
    // chunk c at step t: classified, or, past the last step, finished
    if (t >= K) {
      if (lane == 0 && atomicAdd(fcw(ctl, FC_FIN), 1) + 1 == Cx)
        __hip_atomic_store(fcw(ctl, FC_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    FLOW_DBG(10 + t, c, x, 0);
    FLOW_DIAG_CLASSIFY(c, t);
    const int cnt = __builtin_amdgcn_readfirstlane(classify(c, t));
    FLOW_DBG(30 + t, c, x, cnt);
    if (cnt == 0) {  // no env of the chunk runs an option: its next step at once
      cc = c;
      ct = t + 1;
    }
  }
  FLOW_DBG(9, 0, 0, 0);
  if (lane == 0) FLOW_EV(9, x, 0, 0, 0);
  kst_end(ks, kt0);
}
