// tg_flow_diag.h — DIAGNOSTIC BUILDS ONLY (-DTG_FLOW_DBG, optionally -DTG_FLOW_WAVELOG /
// -DTG_FLOW_LANES; scripts/build_variant.py): k_flow's bring-up instrumentation, kept out of the
// product.  tg_flow.h includes this header only when TG_FLOW_DBG is defined; otherwise every
// hook below is a no-op defined there.  What it records:
//   FLOW_DBG      per-wave progress words in host-mapped memory (the host watches a launch)
//   FLOW_EV       a 32-B event record (type, a, b, c, d, wave, clock) per call: the event log
//                 that scripts/flow_log.py reads (TG_FLOW_WAVELOG: wave-local slots, no atomics)
//   FLOW_DIAG_*   duplicate-push / duplicate-run / duplicate-classification / bad-entry checks,
//                 whose first hit goes to the reserved progress slots 4091-4095
// Host side: flow_diag_setup() before a launch (buffers, the Flow's diagnostic pointers) and
// flow_diag_after() after it (watches the progress words for up to 8 s, writes the event log).
#pragma once

#define FLOW_DBG(code, a, b, c)                                                                  \
  do {                                                                                           \
    const int64_t gw_ = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;                        \
    if (f.dbg && lane == 0 && gw_ < 4096) {                                                      \
      __hip_atomic_store(f.dbg + gw_ * 4 + 0, (uint32_t)(code), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
      __hip_atomic_store(f.dbg + gw_ * 4 + 1, (uint32_t)(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);    \
      __hip_atomic_store(f.dbg + gw_ * 4 + 2, (uint32_t)(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);    \
      __hip_atomic_store(f.dbg + gw_ * 4 + 3, (uint32_t)(c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);    \
    }                                                                                            \
  } while (0)
constexpr uint32_t FLOW_EVCAP = 1u << 22;
#ifdef TG_FLOW_WAVELOG
constexpr uint32_t FLOW_EVW = 1024;
#define FLOW_EV(ty, a, b, c, d)                                                                   \
  do {                                                                                           \
    if (f.dbgl && (ty) != 3 && (ty) != 4 && evn_ < FLOW_EVW) {                                   \
      const int64_t gw_ = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;                      \
      const unsigned long long tm_ = realtime();                                                 \
      uint4* r_ = reinterpret_cast<uint4*>(f.dbgl + 16) + 2 * (gw_ * FLOW_EVW + evn_++);           \
      r_[0] = make_uint4((uint32_t)(ty), (uint32_t)(a), (uint32_t)(b), (uint32_t)(c));            \
      r_[1] = make_uint4((uint32_t)(d), (uint32_t)gw_, (uint32_t)tm_, (uint32_t)(tm_ >> 32));     \
    }                                                                                            \
  } while (0)
#define FLOW_EV_WAVE(ty, a, b) \
  do {                         \
    if (lane == 0) FLOW_EV(ty, a, b, 0, 0); \
  } while (0)  // (timing-log-only events)
#else
#define FLOW_EV(ty, a, b, c, d)                                                                   \
  do {                                                                                           \
    if (f.dbgl) {                                                                                \
      const uint32_t k_ = atomicAdd(f.dbgl, 1u);                                                 \
      if (k_ < FLOW_EVCAP) {                                                                     \
        const unsigned long long tm_ = realtime();                                               \
        uint4* r_ = reinterpret_cast<uint4*>(f.dbgl + 16) + 2 * (int64_t)k_;                      \
        r_[0] = make_uint4((uint32_t)(ty), (uint32_t)(a), (uint32_t)(b), (uint32_t)(c));          \
        r_[1] = make_uint4((uint32_t)(d), (uint32_t)(((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6), \
                           (uint32_t)tm_, (uint32_t)(tm_ >> 32));                                \
      }                                                                                          \
    }                                                                                            \
  } while (0)
#define FLOW_EV_WAVE(ty, a, b) (void)0
#endif
#ifdef TG_FLOW_LANES
#define FLOW_EV_LANE(ty, a, b, c, d) FLOW_EV(ty, a, b, c, d)
#else
#define FLOW_EV_LANE(ty, a, b, c, d) (void)0
#endif

// per-wave diagnostic state, declared at the top of the kernel
#define FLOW_DIAG_WAVE_STATE \
  uint32_t evn_ = 0;         \
  int path_ = 0;             \
  uint32_t item_ = 0;        \
  (void)evn_; (void)path_; (void)item_

// a second push of one list chunk (slot 4093)
#define FLOW_DIAG_PUSH(t, k, j)                                                                   \
  do {                                                                                           \
    if (f.dbgc && (k) != Q_CLASSIFY) {                                                           \
      const int64_t base2_ = (int64_t)f.C * 16 + (int64_t)f.P * FLOW_MAX_K * NLIST * f.jcap;      \
      const uint32_t o_ = atomicAdd(&f.dbgc[base2_ + ((int64_t)x * FLOW_MAX_K * NLIST + (t) * NLIST + (k)) * f.jcap + (j)], 1u); \
      if (o_ && atomicCAS(f.dbg + 4093 * 4, 0u, 97u) == 0u) {                                    \
        f.dbg[4093 * 4 + 1] = ((uint32_t)(t) << 28) | ((uint32_t)(k) << 24) | (uint32_t)(j);      \
        f.dbg[4093 * 4 + 2] = (uint32_t)ld_sc1(fcw(ctl, FC_LTAIL + (t) * NLIST + (k))) | ((uint32_t)x << 24); \
        f.dbg[4093 * 4 + 3] = (uint32_t)ld_sc1(fill + (int64_t)((t) * NLIST + (k)) * f.jcap + (j)) | \
                              ((uint32_t)ld_sc1(fcw(ctl, FC_CLS + (t))) << 16);                  \
      }                                                                                          \
    }                                                                                            \
  } while (0)

// every entry of a run item an env of this sub-problem (slot 4092); the chunk's fill count = the
// entries run (slot 4091)
#define FLOW_DIAG_RUN(item, i, live, mcnt, tail, lidx, j)                                         \
  do {                                                                                           \
    if (f.dbgc) {                                                                                \
      const bool bad_ = (live) && ((i) < 0 || (i) >= n || (int)(((i) >> 6) % P) != x);          \
      if (__ballot(bad_) && lane == __ffsll((long long)__ballot(bad_)) - 1 &&                    \
          atomicCAS(f.dbg + 4092 * 4, 0u, 96u) == 0u) {                                          \
        f.dbg[4092 * 4 + 1] = (item);                                                            \
        f.dbg[4092 * 4 + 2] = (uint32_t)(i);                                                     \
        f.dbg[4092 * 4 + 3] = (uint32_t)lane | ((uint32_t)(mcnt) << 8) | ((uint32_t)x << 16);    \
      }                                                                                          \
      if (lane == 0) {                                                                           \
        const int fl_ = ld_sc1(fill + (int64_t)(lidx) * f.jcap + (j));                           \
        if (fl_ != (mcnt) && atomicCAS(f.dbg + 4091 * 4, 0u, 95u) == 0u) {                       \
          f.dbg[4091 * 4 + 1] = (item);                                                          \
          f.dbg[4091 * 4 + 2] = (uint32_t)fl_ | ((uint32_t)x << 24);                              \
          f.dbg[4091 * 4 + 3] = (uint32_t)(tail);                                                \
        }                                                                                        \
      }                                                                                          \
    }                                                                                            \
  } while (0)

// an item taken twice (slot 4094)
#define FLOW_DIAG_TAKE(item, h)                                                                   \
  do {                                                                                           \
    item_ = (item);                                                                              \
    if (lane == 0 && f.dbgc && (((item) >> 24) & 15u) != Q_CLASSIFY) {                           \
      const int it_l_ = (int)(((item) >> 28) * NLIST + (((item) >> 24) & 15u));                  \
      const uint32_t o_ = atomicAdd(&f.dbgc[(int64_t)f.C * 16 + ((int64_t)x * FLOW_MAX_K * NLIST + it_l_) * f.jcap + ((item) & 0xFFFFFFu)], 1u); \
      if (o_ && atomicCAS(f.dbg + 4094 * 4, 0u, 98u) == 0u) {                                    \
        f.dbg[4094 * 4 + 1] = (item);                                                            \
        f.dbg[4094 * 4 + 2] = (uint32_t)(h);                                                     \
        f.dbg[4094 * 4 + 3] = (uint32_t)x;                                                       \
      }                                                                                          \
    }                                                                                            \
  } while (0)

#define FLOW_DIAG_PATH(p) (path_ = (p))

// a chunk classified twice for one step (slot 4095)
#define FLOW_DIAG_CLASSIFY(c, t)                                                                  \
  do {                                                                                           \
    if (lane == 0) FLOW_EV(1, c, t, path_, x);                                                   \
    if (lane == 0 && f.dbgc) {                                                                   \
      const uint32_t o_ = atomicAdd(&f.dbgc[(int64_t)(c) * 16 + (t)], 1u);                       \
      if (o_ && atomicCAS(f.dbg + 4095 * 4, 0u, 99u) == 0u) {                                    \
        f.dbg[4095 * 4 + 1] = (uint32_t)(c);                                                     \
        f.dbg[4095 * 4 + 2] = (uint32_t)(t) | ((uint32_t)path_ << 8) | ((uint32_t)x << 16);      \
        f.dbg[4095 * 4 + 3] = item_;                                                             \
      }                                                                                          \
    }                                                                                            \
  } while (0)

#ifndef TG_FLOW_TU
// ---- host side (tg_amd.hip launch_flow) ---------------------------------------------------------
// the diagnostic buffers behind the Flow's dbg / dbgc / dbgl pointers
static uint32_t* g_flow_dbg_host = nullptr;  // the progress words (host-mapped)
inline int flow_diag_setup(tg_batch* h, Flow& f) {
  auto& F = h->fl;
  uint32_t*& dbg_host = g_flow_dbg_host;
  static uint32_t* dbg_dev = nullptr;
  if (!dbg_host) {
    HIP_TRY(hipHostMalloc((void**)&dbg_host, 4096 * 4 * sizeof(uint32_t), hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void**)&dbg_dev, dbg_host, 0));
  }
  memset(dbg_host, 0, 4096 * 4 * sizeof(uint32_t));
  f.dbg = dbg_dev;
  static uint32_t* dbgc = nullptr;
  const size_t ndc = (size_t)F.C * 16 + 2 * (size_t)F.P * FLOW_MAX_K * NLIST * F.jcap;
  if (!dbgc) HIP_TRY(hipMalloc((void**)&dbgc, sizeof(uint32_t) * ndc));
  HIP_TRY(hipMemset(dbgc, 0, sizeof(uint32_t) * ndc));
  f.dbgc = dbgc;
#ifdef TG_FLOW_WAVELOG
  f.dbg = nullptr;  // a timing log: no host-mapped progress words, no duplicate counters
  f.dbgc = nullptr;
#endif
  static uint32_t* dbgl = nullptr;
  if (getenv("TG_FLOW_LOG")) {
#ifdef TG_FLOW_WAVELOG
    const size_t evb = 64 + 32 * (size_t)FLOW_EVW * (size_t)h->cus * 8 * (BLOCK / 64);
    if (!dbgl) HIP_TRY(hipMalloc((void**)&dbgl, evb));
    HIP_TRY(hipMemset(dbgl, 0, evb));
#else
    if (!dbgl) HIP_TRY(hipMalloc((void**)&dbgl, 64 + 32 * (size_t)FLOW_EVCAP));
    HIP_TRY(hipMemset(dbgl, 0, 64));
#endif
    f.dbgl = dbgl;
  }
  return TG_OK;
}
// watch the waves' progress for up to 8 s; print the progress histogram and the first hits of
// the duplicate / bad-entry checks; write the event log (TG_FLOW_LOG) for scripts/flow_log.py
inline int flow_diag_after(tg_batch* h, const Flow& f, int k, int bpc, hipStream_t st) {
  auto& F = h->fl;
  for (int ms = 0; ms < 8000 && hipStreamQuery(st) == hipErrorNotReady; ms += 10) usleep(10000);
  const bool hung = hipStreamQuery(st) == hipErrorNotReady;
  const uint32_t* const host_words = g_flow_dbg_host;
  int hist[64] = {0};
  for (int w = 0; w < 4096 && f.dbg; ++w) hist[host_words[w * 4] & 63]++;
  fprintf(stderr, "[flowdbg] launch %lld %s; waves by code:", (long long)F.launches, hung ? "HUNG" : "done");
  for (int c = 0; c < 64; ++c)
    if (hist[c]) fprintf(stderr, " %d:%d", c, hist[c]);
  fprintf(stderr, "\n");
  for (int w = 4091; w < 4096 && f.dbg; ++w)
    if (host_words[w * 4])
      fprintf(stderr, "[flowdbg]  DUP slot %d: code %u %u %08x %08x\n", w, host_words[w * 4],
              host_words[w * 4 + 1], host_words[w * 4 + 2], host_words[w * 4 + 3]);
  const char* logp = getenv("TG_FLOW_LOG");
  if (logp && f.dbgl && !hung) {
    uint32_t cnt = 0;
#ifdef TG_FLOW_WAVELOG
    std::vector<uint32_t> ev((size_t)FLOW_EVW * h->cus * bpc * (BLOCK / 64) * 8);
    HIP_TRY(hipMemcpy(ev.data(), f.dbgl + 16, ev.size() * 4, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < ev.size() / 8; ++r)  // the non-empty records, in place
      if (ev[r * 8]) {
        std::copy(ev.begin() + r * 8, ev.begin() + r * 8 + 8, ev.begin() + (size_t)cnt * 8);
        ++cnt;
      }
    ev.resize((size_t)cnt * 8);
#else
    HIP_TRY(hipMemcpy(&cnt, f.dbgl, 4, hipMemcpyDeviceToHost));
    if (cnt > FLOW_EVCAP) cnt = FLOW_EVCAP;
    std::vector<uint32_t> ev((size_t)cnt * 8);
    HIP_TRY(hipMemcpy(ev.data(), f.dbgl + 16, ev.size() * 4, hipMemcpyDeviceToHost));
#endif
    char path[512];
    snprintf(path, sizeof path, "%s.%lld.bin", logp, (long long)F.launches);
    if (FILE* fp = fopen(path, "wb")) {
      const uint32_t hdr[8] = {cnt, (uint32_t)F.C, (uint32_t)F.P, (uint32_t)k, F.xmap, (uint32_t)F.jcap, 0, 0};
      fwrite(hdr, 4, 8, fp);
      fwrite(ev.data(), 4, ev.size(), fp);
      fclose(fp);
    }
    fprintf(stderr, "[flowdbg] %u events -> %s\n", cnt, path);
  }
  if (hung) {
    fflush(stderr);
    _exit(3);
  }
  return TG_OK;
}
#endif  // TG_FLOW_TU
