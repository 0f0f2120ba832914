// tg_batch.h — the handle behind include/tg_amd.h, shared by the step (tg_amd.hip) and render
// (tg_render.hip) translation units of libtg_amd.so.  Internal: not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/tg_amd.h"
#include "tg_core.h"

namespace tg {

extern thread_local std::string g_err;  // tg_last_error() text (tg_amd.hip)
inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(TG_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct Soa {
  uint4* st4;
  double2* ang;
  int2* ep;
  uint32_t* mt;   // [N][MT_STORE]: the ring's even generations (tg_core.h)
  uint8_t* mc;    // [N][MT_CODES]: the draw codes of the ring's generations (tg_core.h draw_code)
};

// tg_step1's result row (one env)
struct TgOne {
  double obs[9];
  int32_t reward;
  uint8_t valid, done;
};
static_assert(sizeof(TgOne) == 80, "TgOne: ten 8-B words (k_serve1 copies it out by word)");

// The N = 1 server's mailbox (k_serve1, tg_amd.hip): pinned, coherent host memory (line 2:
// TG_SERVE_TRACE's stamps).  Line 0 is
// the host's: a command is one 16-B group (seq last: the server reads the group with one load,
// and a group whose seq is new carries the command's fields) and, for a reset, gauss_next
// (read after the group).  Line 1 is the server's: done, the last command it served (a server
// that starts reads it, so a command posted while none ran is served by the next one).
enum : uint32_t { SRV_STEP = 1, SRV_STEP_PY = 2, SRV_RESET_PY = 3, SRV_QUIT = 4, SRV_MASK = 5,
                  SRV_RESET = 6 };
// the command word: kind | (action + 16) << 4 | warm << 9 | has_gauss << 10 | q0 << 11
inline uint32_t srv_word(uint32_t kind, int32_t action, bool warm, bool has_gauss, uint32_t q0) {
  return kind | (uint32_t)((action + 16) & 31) << 4 | (warm ? 1u : 0u) << 9 |
         (has_gauss ? 1u : 0u) << 10 | (q0 & 1023u) << 11;
}
struct SrvBox {
  uint32_t word;        // srv_word
  uint32_t tstep;       // the step's index (h->tstep)
  uint32_t pad0;
  uint32_t seq;         // the last command posted (written last)
  uint64_t gauss_bits;  // SRV_RESET_PY: the caller's gauss_next
  uint8_t pad1[64 - 24];
  uint32_t done;
  uint32_t mask;           // SRV_MASK's answer: available_mask's bits
  uint32_t pad2[2];
  uint64_t t_seen, t_end;  // TG_SERVE_TRACE: the server's clock at the command's pickup / answer
  uint32_t ticks;          //   and the command's ticks
  uint32_t pad3[7];
  uint64_t phase[5];       // TG_SERVE_TRACE: py_call's phase stamps (SRV_STEP_PY)
  uint64_t pad4[3];
};
static_assert(sizeof(SrvBox) == 192, "SrvBox: three 64-B lines");

struct RenderState;  // tg_render.hip
void render_free(RenderState* rs);

// One stepper over envs [off, off + n) of the handle: its worklists, counters, refill lists and
// launch counters.  The handle's own covers every env (tg_step, tg_rollout); with tg_set_groups
// each group has one, and tg_rollout steps the groups on streams of their own (tg_amd.hip).
struct StepCtx {
  int64_t off = 0, n = 0;
  unsigned long long* stats = nullptr;  // [stat_slots(n)][ST_COUNT] launch counters
  int32_t* wl = nullptr;   // per-(option, shard) worklists (compact mode)
  uint4* wst4 = nullptr;   // the listed envs' state in worklist order (k_classify -> k_run)
  double2* wang = nullptr;
  int2* wep = nullptr;
  int32_t* wctr = nullptr; // sharded counters, two sets (step parity)
  uint32_t* refill = nullptr;  // stale MT halves listed by k_classify: SHARDS lists (k_regen)
  int64_t rcap = 0;            // entries per list: a shard's envs x REGEN_STEPS
  int64_t shard_cap = 0;
  int parity = 0;  // which half of wctr this compact step counts in
  int rpend = 0;   // compact steps whose refill lists k_regen has not drained
  int32_t* regen_ctr = nullptr;  // per XCD: k_regen's grab counters and the lists' lengths, two
                                 // sets (k_regen zeroes the other set for the next launch)
  int regen_parity = 0;          // which set the next k_regen counts in
  hipStream_t st = nullptr;      // a group's stream (groups only)
  hipEvent_t ev = nullptr;       //   and its join event
};

}  // namespace tg

// the handle (tg_amd.h tg_batch)
struct tg_batch {
  int device = 0;
  int64_t n = 0;
  int64_t g0 = 0;
  uint64_t seed0 = 0;
  tg::Level L{};
  uint32_t* grid = nullptr;  // bordered cell grid, padded to whole words
  uint32_t* genrand = nullptr;
  // GoTable (tg_core.h go_lookup): W * H * 32 entries
  uint32_t* gotab = nullptr;
  uint32_t* masks = nullptr;  // the level bitmasks (tg_core.h Map::mk), or null
  double* obs_q = nullptr;    // get_state's quotient table (tg_core.h Level::obs_q)
  int cus = 0;  // compute units
  tg::Soa S{};
  tg_episode* eps = nullptr;
  int32_t* eps_count = nullptr;
  int32_t eps_cap = 0;
  uint32_t* err = nullptr;
  int mode = TG_MODE_COMPACT;
  tg::StepCtx main;                // the stepper over every env
  std::vector<tg::StepCtx> grp;    // tg_set_groups: the groups' steppers (tg_rollout)
  hipEvent_t fork = nullptr;       //   the groups' fork event
  bool stagger = false;            //   group g + 1 starts after group g's first k_classify
  uint32_t tstep = 0;  // steps taken by the handle (mod 2^32): S.ep holds each episode's start step
  int timing_every = 0;        // HIP-event timing of every k-th step launch (0: off)
  uint64_t timing_calls = 0;   // step launches since timing was enabled
  unsigned long long* kst = nullptr;  // in-kernel span records of the timed launches (tg_amd.hip)
  int kst_steps = 0, kst_regens = 0;  // records in use
  double kernel_ms_done = 0.0;  // the timed step launches' kernel spans (in-kernel stamps)
  double classify_ms_done = 0.0;  //   of which k_classify
  double run_ms_done = 0.0;     //   and k_run (or k_step)
  int64_t timed_launches = 0;
  int regen_per_cu = 0;             // k_regen workgroups resident per CU (occupancy API, first use)
  double regen_ms_done = 0.0;       // the timed k_regen launches' spans (in-kernel stamps)
  int64_t regen_launches = 0;       // k_regen launches (timed or not)
  int64_t regen_timed = 0;
  std::string domain;              // domain.txt text (the renderer's cell sprites)
  double* obs_scratch = nullptr;   // tg_rollout without an obs output
  tg::TgOne* one = nullptr;            // tg_step1's row: pinned host memory the kernel writes
  tg::TgOne* one_dev = nullptr;        //   (its device-side address)
  uint16_t* mask1 = nullptr;           // tg_available_mask1's answer without the server (pinned)
  uint16_t* mask1_dev = nullptr;
  tg_pystate* py = nullptr;            // tg_step1_py / tg_reset1_py's stream state (pinned)
  tg_pystate* py_dev = nullptr;
  uint32_t* pyc = nullptr;  // the Python stream's generation + 2 successors, on the device
  tg_pystate py_last{};     // the state the last tg_*1_py call returned
  bool py_warm = false;     // pyc matches py_last
  // the N = 1 calls' resident server (k_serve1): tg_step1 / tg_step1_py / tg_reset1_py post a
  // command to its mailbox and spin on the answer instead of a launch and a synchronisation
  // each; every other entry point stops it first (BIND)
  bool serve = true;               // tg_set_serve / TG_SERVE (read at tg_create)
  uint32_t srv_idle = 0;           // the server leaves after this many 10-ns ticks without a command
  tg::SrvBox* box = nullptr;       // the mailbox (pinned, coherent) and its device address
  tg::SrvBox* box_dev = nullptr;
  hipStream_t srv_st = nullptr;    // the server's stream: after the caller's stream (srv_dep)
  hipEvent_t srv_ev = nullptr;     //   recorded after each server launch: complete = it left
  hipEvent_t srv_dep = nullptr;
  bool srv_live = false;           // a server was launched and not stopped
  uint32_t srv_seq = 0;
  int64_t srv_t_last = 0;          // host clock (ns) at the last answer
  int64_t srv_launches = 0, srv_calls = 0;
  int srv_stage = -1;              // the level tables the server keeps in LDS (k_serve1 stage; -1:
  size_t srv_dyn = 0;              //   not chosen yet) and their dynamic LDS bytes
  bool srv_trace = false;          // TG_SERVE_TRACE: sums printed at tg_destroy (diagnostic)
  double srv_rt_ns = 0.0, srv_gpu_ns = 0.0, srv_post_ns = 0.0, srv_fit[3] = {0.0, 0.0, 0.0};
  double srv_phase[6] = {0, 0, 0, 0, 0, 0};
  int64_t srv_phase_n = 0;
  tg::RenderState* rs = nullptr;   // tg_render_init
  std::vector<int> kst_k;          // steps each in-use step record covers (a k_flow launch: K)
  // TG_MODE_FLOW's work structures (tg_flow.h Flow; allocated at the first flow rollout)
  struct {
    bool ready = false;
    int P = 0;                // sub-problems: the XCDs the census saw
    uint32_t xmap = 0;        // XCC id -> sub-problem (nibbles)
    int32_t C = 0;            // 64-env chunks
    int64_t qcap = 0, jcap = 0, lcap = 0;
    int32_t* ctl[2] = {nullptr, nullptr};  // two parities: a launch zeroes the other's
    uint32_t* q[2] = {nullptr, nullptr};
    int32_t* fill[2] = {nullptr, nullptr};
    int32_t* list = nullptr;
    int32_t* outst = nullptr;
    int parity = 0;
    int bpc[2][2] = {{0, 0}, {0, 0}};  // k_flow<AR, POL> workgroups per CU (occupancy API)
    int64_t launches = 0;
  } fl;
  // read once at tg_create: TG_FLOW_DEBUG (print the census and every k_flow launch's
  // sub-problem counters; synchronises after each launch) and the test hook TG_FLOW_SKIP_PART
  // (sub-problem x's waves leave at once: tests/test_gpu_flow.py checks TG_ERR_FLOW is raised)
  bool flow_debug = false;
  int flow_skip = -1;
};

namespace tg {
inline int bind(const tg_batch* h) {
  int cur = -1;
  HIP_TRY(hipGetDevice(&cur));
  if (cur != h->device) HIP_TRY(hipSetDevice(h->device));
  return TG_OK;
}
int srv_stop(tg_batch* h);  // tg_amd.hip: stop the N = 1 server (if one runs) and wait for it
// every entry point: the handle's device current, and the N = 1 server stopped (it steps the
// env on a stream of its own: nothing else may touch the handle's state while it runs)
#define BIND(h)                       \
  do {                                \
    if (!(h)) return fail(TG_E_INVAL, "null handle"); \
    int rc_ = bind(h);                \
    if (!rc_ && (h)->srv_live) rc_ = srv_stop(h); \
    if (rc_) return rc_;              \
  } while (0)
// the N = 1 calls the server serves
#define BIND_SERVE(h)                 \
  do {                                \
    if (!(h)) return fail(TG_E_INVAL, "null handle"); \
    int rc_ = bind(h);                \
    if (rc_) return rc_;              \
  } while (0)

}  // namespace tg
