// tg_core.h — per-env Treasure Game step physics for the MI355X kernel (gfx950).
//
// Everything here is `__host__ __device__` integer code operating on one env held in
// registers.  tg_amd.hip wraps it in the batched kernels (one wavefront lane per env, level
// grid in LDS, struct-of-arrays state in HBM).  The host instantiation exists only so the
// test harness (tests/native/) can run the exact same code on the build machine, which has
// no GPU; the product API never executes it on the CPU.
//
// Differences in FORM from the reference (not in results — parity is pinned by the oracle):
//   * collision predicates (IM/:232-288) are evaluated on the 48x48-cell grid with a handful
//     of branch-free cell lookups instead of up to 104 pixel probes: the reference pixel map
//     is constant per cell (build_map IM/:204-216, door.update_map OB/:246-253) and OOB is
//     WALL (IM/:218-225) — here a 2-cell WALL border around the grid plus clamping;
//   * near_enough (OB/:46-53) is the exact integer test d^2 < r^2 (inputs are integers);
//   * the trigger cascade (OB/:76-94) is an explicit 8-bit-frame stack in one u64 register;
//   * MT19937 keeps two pre-twisted generations per env; consumption only reads (Rng); the
//     option loops read one code byte per draw (its noisy / jump / flip outcomes, draw_code)
//     instead of the double;
//   * each option's policy/tick loop is specialised at compile time to the primitive actions
//     that option can issue (a wave runs one option in the compacted kernel).
// Prefixes: TG/ treasure_game.py, IM/ _treasure_game_impl.py, OB/ _objects.py,
// MO/ _move_options.py, OP/ _option.py under gym_treasure_game/envs/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TG_HD __host__ __device__ __forceinline__

namespace tg {

constexpr int S = 48;          // xscale == yscale (_scale.py:8-9)
constexpr int INCR = S / 10;   // x_incr / y_incr (IM/:46-47)
constexpr int HALFW = S / 4;   // player_width // 2 (IM/:49)
constexpr int MT_N = 624, MT_M = 397;
constexpr int TICK_CAP = 1 << 14;  // the reference has no cap (OP/:28-31); observed max 105
// random() draws a tick without INTERACT can take (a move or a jump: 1), with margin.  An
// INTERACT tick can take more: each handle flip is 1 draw plus one wiggle per handle change of
// its cascade, and since process_trigger clears previously_triggered on return (OB/:76-94) a
// cascade can change one handle several times.  Its bound depends on the level's trigger
// table: Level::interact_draws (tg_level.h interact_draw_bound), at most MAX_TICK_DRAWS.
constexpr uint32_t TICK_DRAWS = 8;
constexpr uint32_t MAX_TICK_DRAWS = 48;  // what a refilled code window always holds (tg_amd.hip)
constexpr int PAD = 2;         // WALL cells around the grid in LDS (probes reach <= 60 px out)

// Cell bits in the LDS grid.  A door object's cell carries only its one-hot door bit: its type
// is 'D' or ' ' by the door's state (update_map overwrites whatever the file had there).
enum : uint32_t { B_OPEN = 1, B_LADDER = 2, B_WALL = 4, B_DOOR = 8, B_DOOROBJ = 16 /* << i */ };
// primitive actions (_actions.py:7-13)
enum : int { P_NOP = 0, P_UP, P_DOWN, P_LEFT, P_RIGHT, P_JUMP, P_INTERACT };
// options in create_options order (IM/:495)
enum : int { O_GO_LEFT = 0, O_GO_RIGHT, O_UP_LADDER, O_DOWN_LADDER, O_INTERACT, O_DOWN_LEFT,
             O_DOWN_RIGHT, O_JUMP_LEFT, O_JUMP_RIGHT, O_COUNT };

// ---- per-env flag word -------------------------------------------------------------------
// interactive object i (0..2 doors, 3..4 handles, 5 bolt) keeps its boolean at bit 6+i:
// door.closed, handle.up, bolt.locked.
constexpr uint32_t F_JT = 0x1Fu;          // jump_ticker (0..23)
constexpr uint32_t F_FACING = 1u << 5;    // facing_right (render only)
constexpr int F_OBJ = 6;                  // first interactive-object bit
constexpr int F_BAGLEN = 12;              // 3 bits: len(player_bag)
constexpr int F_BAGITEM = 15;             // 7 bits: item i is gold (1) or key (0)
constexpr uint32_t E_TICKCAP = 1u << 24;  // option exceeded TICK_CAP
constexpr uint32_t E_BAG = 1u << 25;      // bag overflow (unreachable in the default level)
constexpr uint32_t E_ACTION = 1u << 26;   // action outside [-9, 8] (reference: IndexError)
constexpr uint32_t E_NEARINT = 1u << 27;  // a reset's gauss landed within 1e-9 of an int()
                                          // boundary (device libm vs glibc watch)
constexpr uint32_t E_WINDOW = 1u << 29;   // a lane drew past its staged code window (a bug)
constexpr uint32_t E_MASK = 0xFF000000u;

// ---- level (kernel argument; the grid and the trigger table are staged in LDS) -------------
struct Level {
  int32_t W, H;              // cells (IM/:196-197)
  int32_t start_x, start_y;  // first non-WALL description cell (IM/:173-176)
  int8_t door_cx[3], door_cy[3];
  int8_t handle_cx[2], handle_cy[2];
  int8_t key_cx, key_cy, bolt_cx, bolt_cy, gold_cx, gold_cy;
  uint32_t init_flags;       // door/handle/bolt initial booleans at their F_OBJ bits
  uint32_t trig[6][2];       // trigger lists [object][polarity]: count(4b) + 7 x (target 3b, val 1b)
  uint32_t interact_draws;   // most random() draws one INTERACT tick can take (>= TICK_DRAWS)
  // go_left / go_right can_run and target per (cell, door state, key home?, gold home?)
  // (GoTable; device global memory, built at tg_create; null: computed directly)
  const uint32_t* gotab;
  // the level bitmasks (Map::mk; mk_words(W, H) words, device global memory, staged into LDS
  // by the kernels that use them; null: the level is too large, cell probes)
  const uint32_t* masks;
  // get_state's quotients (observe): obs_q[i] = (double)(Q_MIN + i) / (W * 48) for
  // i < qx_n, then obs_q[qx_n + i] = (double)(Q_MIN + i) / (H * 48) for i < qy_n, each the IEEE
  // quotient the division would give (built on the host, tg_level.h build_obs_q); null: divide
  const double* obs_q;
  int32_t qx_n, qy_n;
};
constexpr int Q_MIN = -2 * S;  // the smallest pixel coordinate the quotient table covers

// ---- per-env state (registers) -------------------------------------------------------------
struct Env {
  int px, py;            // playerx / playery (IM/:42)
  uint32_t f;            // flags above
  int kx, ky, gx, gy;    // key / goldcoin cell (OB/:34-38)
  double ang0, ang1;     // handle angles (OB/:111-114)
  uint32_t mti;          // MT state word: position ([0, MT_WORDS), even) | MT_STALE (see Rng)
};

TG_HD int floordiv(int a, int b) {  // Python // for b > 0
  int q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}
TG_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Pixel -> cell in the tick loops.  A 32-bit division by the constant 48 compiles to 32-bit
// magic-number multiplies (v_mul_hi_u32 / v_mul_lo_u32, slower VALU); 24-bit operands take
// the full-rate v_mul_u32_u24 instead.  v * 21846 >> 20 equals v / 48 for 0 <= v < 32,700
// (21846 / 2^20 - 1/48 = 6.4e-7; 6.4e-7 * 32,700 < 1/48) — levels are at most 124 cells
// (5,952 px) per side with the border.
static_assert(S == 48, "div48 constants");
TG_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TG_NO_MUL24)
  return __umul24(a, b);
#else
  return a * b;
#endif
}
TG_HD int div48(int v) { return (int)(mul24((uint32_t)v, 21846u) >> 20); }  // 0 <= v < 32,700
TG_HD int floordiv48(int a) { return div48(a + 16 * S) - 16; }              // -768 <= a < 31,900

// ==========================================================================================
// CPython random over a ring of pre-twisted generations.
//   CPython (_randommodule.c genrand_uint32) regenerates all 624 words at once ("twist")
//   whenever its index reaches 624, then tempers one word per call; random() takes two.
//   Here each env keeps a ring of 2 x MT_HALF_GENS consecutive generations, two halves of
//   MT_HALF_GENS generations each (words [0, MT_HALF) and [MT_HALF, MT_WORDS)), and a position
//   pos in [0, MT_WORDS) (always even: random() is the only consumer).  Consumption only
//   reads: the generation holding pos is CPython's mt[] with index pos % 624, and the ring
//   always holds the NEXT generations after it, so crossing a generation or half boundary
//   continues the stream without a twist.
//   The half a lane has left is stale (2 x MT_HALF_GENS generations behind) until it is
//   regenerated: MT_HALF_GENS twists in sequence from the last generation of the half the
//   lane is in (twist_half); the env's state word carries MT_STALE meanwhile.  The kernels
//   regenerate it later, a whole wavefront per env, coalesced, the chained twists in LDS
//   (tg_amd.hip twist_chain: k_regen every 16 steps, k_reset, k_step).  A launch that
//   would enter a stale half (> MT_HALF draws since the refill) regenerates it first, per
//   lane.  Seeding (init_by_array) fills the ring's last generation; 2 x MT_HALF_GENS twists
//   then give generations 1 .. 2 x MT_HALF_GENS, pos 0 (init_mt).
//   Why a ring of 8 + 8: a half's regeneration reads one generation (its
//   source) and writes MT_HALF_GENS of them, 3,120 B per generation instead of the 5,304 of
//   a two-generation ring whose every twist re-reads its source from HBM, and the refill
//   list is an eighth as long (A/B, 1M envs: 2 + 2 / 4 + 4 / 8 + 8 per half: uniform 0.172 /
//   0.168 / 0.164 ms, masked 0.399 / 0.391 / 0.368 ms per step; 1 + 1: 0.176 / 0.483).
//   Stored words (round 4): only the EVEN generations of the ring (gens 0, 2, ..., 14 of the
//   16; MT_STORE words per env, mt_store_off), the codes of all.  The option loops read codes;
//   the words serve the rare draws that need their double (handle angles, an auto-reset's
//   gauss) and the twists.  An odd generation's word is the twist of the stored generation
//   before it (twist_at: <= 4 twist_word evaluations on that generation's words, mt_pair), and
//   a half's regeneration starts from the other half's generation 7 = the twist of its stored
//   generation 6.  A regenerated generation costs 312 B of codes + 1,248 B of words instead of
//   312 + 2,496.  20 KB of words + 5 KB of codes per env.
// ==========================================================================================
constexpr int MT_HALF_GENS = 8;                // generations per half
constexpr int MT_HALF = MT_HALF_GENS * MT_N;   // ring positions per half (words of 8 generations)
constexpr int MT_WORDS = 2 * MT_HALF;          // ring positions per env
constexpr int MT_STORE = MT_WORDS / 2;         // words stored per env: the even generations
static_assert(MT_HALF_GENS % 2 == 0, "a half starts on a stored generation");
// word offset in the stored words of ring generation g (even; g = ring position / MT_N)
TG_HD uint32_t mt_store_off(uint32_t g) { return (g >> 1) * (uint32_t)MT_N; }
constexpr uint32_t MT_STALE = 1u << 31;   // state word: the half not holding pos is stale
constexpr uint32_t MT_LISTED = 1u << 30;  // state word: that stale half is on a refill list (k_regen)
constexpr uint32_t MT_POS_MASK = 0xFFFFu;
static_assert(MT_WORDS <= (int)MT_POS_MASK, "positions fit the state word");
constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu;

TG_HD uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & MT_UPPER) | (b & MT_LOWER);
  return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
TG_HD uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
// random_random (53-bit) from two consecutive words, exact in double (FMA-safe)
TG_HD double mt_double(uint32_t w0, uint32_t w1) {
  const uint32_t a = mt_temper(w0) >> 5, b = mt_temper(w1) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}
// dst = the generation after src (genrand_uint32's twist, out of place)
TG_HD void twist_gen(const uint32_t* src, uint32_t* dst) {
  for (int p = 0; p < MT_N - MT_M; ++p) dst[p] = mt_twist(src[p], src[p + 1], src[p + MT_M]);
  for (int p = MT_N - MT_M; p < MT_N - 1; ++p)
    dst[p] = mt_twist(src[p], src[p + 1], dst[p - (MT_N - MT_M)]);
  dst[MT_N - 1] = mt_twist(src[MT_N - 1], dst[0], dst[MT_M - 1]);
}
// the same in place: twist_gen reads src only at or after the word it writes and dst only
// before it, so src == dst is CPython's own in-place loop
TG_HD void twist_gen_inplace(uint32_t* w) { twist_gen(w, w); }
// Word i (< 623) of the generation after g, from g's words alone: new word i reads new word
// i - 227 for i >= 227 (twist_gen), so it is a chain of d = i / 227 (0-2) twist words on top of
// new word j0 = i - 227 d (< 227, which reads old words only).  The chain's old words are at
// fixed offsets from j0 and all load unconditionally (indices clamped into the generation):
// one memory round trip, and no divergence between lanes of different chain lengths.
// (Ld: how a stored word is read — plain, or k_flow's L1-bypassing load, tg_amd.hip)
struct PlainLd {
  TG_HD uint32_t operator()(const uint32_t* p) const { return *p; }
};
template <class Ld = PlainLd>
TG_HD uint32_t twist_at_lo(const uint32_t* g, int i, const Ld& ld = Ld()) {
  constexpr int K = MT_N - MT_M;  // 227
  const int d = i >= 2 * K ? 2 : i >= K ? 1 : 0;
  const int j0 = i - K * d;
  const int c2 = j0 + 2 * K < MT_N - 1 ? j0 + 2 * K : MT_N - 2;
  const uint32_t a0 = ld(g + j0), b0 = ld(g + j0 + 1), c0 = ld(g + j0 + MT_M);
  const uint32_t a1 = ld(g + j0 + K), b1 = ld(g + j0 + K + 1);
  const uint32_t a2 = ld(g + c2), b2 = ld(g + c2 + 1);
  uint32_t w = mt_twist(a0, b0, c0);
  const uint32_t w1 = mt_twist(a1, b1, w);
  w = d >= 1 ? w1 : w;
  const uint32_t w2 = mt_twist(a2, b2, w);
  return d >= 2 ? w2 : w;
}
// word i of the generation after g (word 623 reads new words 0 and 396)
TG_HD uint32_t twist_at(const uint32_t* g, int i) {
  return i < MT_N - 1 ? twist_at_lo(g, i)
                      : mt_twist(g[MT_N - 1], twist_at_lo(g, 0), twist_at_lo(g, MT_M - 1));
}
// The two words at ring position p (even) from the stored generations: an even generation's
// are stored, an odd one's are twisted from the generation before it (the rare draws that need
// their double).  Branch-free: every lane issues the loads of both cases (~20 words) at once,
// so a wave whose lanes sit in even and odd generations pays one memory round trip, not two.
template <class Ld = PlainLd>
TG_HD void mt_pair(const uint32_t* mt, uint32_t p, uint32_t& w0, uint32_t& w1, const Ld& ld = Ld()) {
  const uint32_t g = p / (uint32_t)MT_N, i = p - g * (uint32_t)MT_N;  // i even, <= 622
  const uint32_t* const cur = mt + mt_store_off(g & ~1u);  // g's own words if g is even
  const uint32_t* const prev = mt + mt_store_off(g == 0u ? 0u : (g - 1u) & ~1u);
  const uint32_t e0 = ld(cur + i), e1 = ld(cur + i + 1);
  const uint32_t o0 = twist_at_lo(prev, (int)i, ld);
  // word i + 1: a chain of its own, or, for i + 1 = 623, the twist of old word 623 with new
  // words 0 and 396
  const bool last = i + 1u == (uint32_t)MT_N - 1u;
  const uint32_t x = twist_at_lo(prev, last ? MT_M - 1 : (int)i + 1, ld);
  const uint32_t y0 = twist_at_lo(prev, 0, ld);
  const uint32_t o1 = last ? mt_twist(ld(prev + MT_N - 1), y0, x) : x;
  w0 = (g & 1u) ? o0 : e0;
  w1 = (g & 1u) ? o1 : e1;
}
// the same with a branch (few registers, inline: tg::Rng, whose draws of doubles in the step
// kernels are resets of envs whose option did not run, rarer still)
TG_HD void mt_pair_branchy(const uint32_t* mt, uint32_t p, uint32_t& w0, uint32_t& w1) {
  const uint32_t g = p / (uint32_t)MT_N, i = p - g * (uint32_t)MT_N;
  if (g & 1u) {
    const uint32_t* const prev = mt + mt_store_off(g - 1u);
    w0 = twist_at(prev, (int)i);
    w1 = twist_at(prev, (int)i + 1);
  } else {
    w0 = mt[mt_store_off(g) + i];
    w1 = mt[mt_store_off(g) + i + 1];
  }
}
// mt_pair out of line (RngCodes, the option loops' draws: its loads and chains would
// otherwise add ~30 VGPRs to k_run's allocation)
struct WordPair {
  uint32_t w0, w1;
};
__host__ __device__ inline __attribute__((noinline)) WordPair mt_pair_ool(const uint32_t* mt, uint32_t p) {
  WordPair r;
  mt_pair(mt, p, r.w0, r.w1);
  return r;
}
// word offset of the half holding word position pos
TG_HD uint32_t mt_half(uint32_t pos) { return pos >= (uint32_t)MT_HALF ? (uint32_t)MT_HALF : 0u; }

// ---- draw codes ------------------------------------------------------------------------------
// Every random() value the option loops consume decides one of four things, each a comparison
// of the double r against constants, computed with the reference's own IEEE expressions:
//   noisy(+4) (IM/:361-366): int(round(uniform(2.0, 4)))   = rint(2.0 + 2.0 * r) in {2, 3, 4}
//   noisy(-4):                int(round(uniform(-4, -2.0))) = rint(-4.0 + 2.0 * r) in {-4, -3, -2}
//   the jump ticker (IM/:317-319): random() > 0.25
//   handle.flip (OB/:117-122):     uniform(0, 1) <= 0.8  (== r exactly)
// so each generation is stored twice: its 624 words (for the next twist and for the rare
// draws that need the double itself: handle angles, the reset's gauss) and one code byte per
// draw (MT_CODES per env, the generation at word offset g at g / 2) holding those four
// outcomes.  Whoever regenerates a half writes both.  Tick loops read bytes (16 draws per 16-B
// load) and do no f64 work.
constexpr int MT_CODES = MT_WORDS / 2;  // one per random() draw of the ring
constexpr uint32_t CODE_POS = 3u;        // rint(2 + 2r) - 2
constexpr uint32_t CODE_NEG_SHIFT = 2;   // rint(-4 + 2r) + 4, bits 2-3
constexpr uint32_t CODE_JUMP = 1u << 4;  // r > 0.25
constexpr uint32_t CODE_FLIP = 1u << 5;  // r <= 0.8
TG_HD uint32_t draw_code(double r) {
  const uint32_t pos = (uint32_t)((int)rint(2.0 + 2.0 * r) - 2);
  const uint32_t neg = (uint32_t)((int)rint(-4.0 + 2.0 * r) + 4);
  return pos | (neg << CODE_NEG_SHIFT) | (r > 0.25 ? CODE_JUMP : 0u) | (r <= 0.8 ? CODE_FLIP : 0u);
}
// draw_code from the draw's first word: r lies in [a / 2^27, (a + 1) / 2^27) for a = the top
// 27 bits (mt_double), and every outcome in draw_code is monotone in r, so the code is constant
// on that interval unless one of the thresholds 0.25, 0.75, 0.8 lies in it or next to it
// (CODE_SLOW: then the exact f64 path, ~3 draws in 2^25).  Checked for every a against
// draw_code at both ends of its interval (tests/test_core_host.py).  k_regen's code pass takes
// it: one word tempered instead of two, integer compares instead of f64 work.
constexpr uint32_t CODE_SLOW = 0xFFu;
TG_HD uint32_t code_of_top27(uint32_t a) {
  constexpr uint32_t Q1 = 1u << 25, Q3 = 3u << 25, F8 = 107374182u;  // floor(x * 2^27)
  if (a - (Q1 - 1u) < 3u || a - (Q3 - 1u) < 3u || a - (F8 - 1u) < 3u) return CODE_SLOW;
  constexpr uint32_t LOW = CODE_FLIP;                                            // r < 0.25
  constexpr uint32_t MID = 1u | (1u << CODE_NEG_SHIFT) | CODE_JUMP | CODE_FLIP;  // < 0.75
  constexpr uint32_t HIGH = 2u | (2u << CODE_NEG_SHIFT) | CODE_JUMP;             // > 0.75
  return a < Q1 ? LOW : a < Q3 ? MID : a < F8 ? (HIGH | CODE_FLIP) : HIGH;
}
TG_HD uint32_t draw_code_words(uint32_t w0, uint32_t w1) {
  const uint32_t c = code_of_top27(mt_temper(w0) >> 5);
  return c != CODE_SLOW ? c : draw_code(mt_double(w0, w1));
}
// code_of_top27 in fewer instructions (the wave twist's code pass, tg_twist.h, is VALU-bound):
// for an `a` that is not next to a threshold the outcome classes r < 0.25 | < 0.75 | <= 0.8 |
// > 0.8 are a's top two bits (0 | 1, 2 | 3) plus one compare against F8 (F8 >= 3 * 2^25: only
// class 3 splits); byte k of TOP27_LUT is class k's code.  top27_slow is a superset of
// code_of_top27's CODE_SLOW set (a within one of any multiple of 2^25 — 0.25 and 0.75 are 2^25
// and 3 * 2^25, the others harmless extra slow cases — or of F8): there the exact f64 path
// runs.  Checked against code_of_top27 for every a (tests/test_core_host.py).
constexpr uint32_t TOP27_F8 = 107374182u;  // floor(0.8 * 2^27), as code_of_top27
constexpr uint32_t TOP27_LUT = CODE_FLIP |
                               ((1u | (1u << CODE_NEG_SHIFT) | CODE_JUMP | CODE_FLIP) << 8) |
                               ((1u | (1u << CODE_NEG_SHIFT) | CODE_JUMP | CODE_FLIP) << 16) |
                               ((2u | (2u << CODE_NEG_SHIFT) | CODE_JUMP | CODE_FLIP) << 24);
static_assert(TOP27_F8 >= (3u << 25), "only the top class splits at 0.8");
TG_HD bool top27_slow(uint32_t a) {
  return (((a + 1u) & 0x1FFFFFFu) < 3u) | (a - (TOP27_F8 - 1u) < 3u);
}
TG_HD uint32_t top27_code(uint32_t a) {
  const uint32_t c = (TOP27_LUT >> ((a >> 22) & 0x18u)) & 0xFFu;
  return a >= TOP27_F8 ? c ^ CODE_FLIP : c;
}
// the noisy step of a code: +2..+4 (DIR > 0: RIGHT / DOWN) or -4..-2 (LEFT / UP)
TG_HD int code_step(uint32_t c, bool neg) {
  return neg ? (int)((c >> CODE_NEG_SHIFT) & 3u) - 4 : (int)(c & CODE_POS) + 2;
}
TG_HD void gen_codes(const uint32_t* words, uint8_t* c) {
  for (int k = 0; k < MT_N / 2; ++k) c[k] = (uint8_t)draw_code(mt_double(words[2 * k], words[2 * k + 1]));
}
// Regenerate half h (ring position 0 / MT_HALF): its generations in sequence from the one
// before it — the other half's generation 7, the twist of its stored generation 6, or, with
// seeded, the 624 words already in the half's last stored slot (init_mt) — its even
// generations' words and, with mc, all its codes (per-lane form of tg_twist.h twist_chain).
// The half's 4 stored slots are the work space: slot 3 holds the source until generation 5,
// each odd generation goes to the next slot and becomes the even one after it in place;
// generation 7 (codes only) is twisted in place over generation 6, which is then made again
// from generation 4 (two extra twists on this rare per-lane path, no other scratch).
// (Ops: the whole-generation loops, inline here; tg_amd.hip's regen_half calls them out of line
// so that k_run's register allocation does not grow around its rare call)
struct GenOps {
  TG_HD void twist(const uint32_t* src, uint32_t* dst) const { twist_gen(src, dst); }
  TG_HD void codes(const uint32_t* w, uint8_t* c) const { gen_codes(w, c); }
};
template <class Ops = GenOps>
TG_HD void twist_half(uint32_t* mt, uint32_t h, uint8_t* mc = nullptr, bool seeded = false,
                      const Ops& op = Ops()) {
  const uint32_t g0 = h / (uint32_t)MT_N;  // ring generation of the half's first (0 / 8)
  uint32_t* const s = mt + mt_store_off(g0);
  uint32_t* const s3 = s + 3 * MT_N;
  if (!seeded) op.twist(mt + mt_store_off((g0 + (uint32_t)MT_HALF_GENS + 6u) % (2u * MT_HALF_GENS)), s3);
  uint8_t* const c = mc ? mc + h / 2 : nullptr;
  // generation g: 0 from slot 3 into slot 0; odd 2k + 1 from slot k into slot k + 1; even
  // 2k + 2 in place in slot k + 1; 7 (codes only) in place in slot 3
  const int last = c ? MT_HALF_GENS : MT_HALF_GENS - 1;
  for (int g = 0; g < last; ++g) {
    const int to = (g + 1) >> 1 < 3 ? (g + 1) >> 1 : 3;
    const uint32_t* const from = g == 0 ? s3 : (g & 1) ? s + (g >> 1) * MT_N : s + to * MT_N;
    op.twist(from, s + to * MT_N);
    if (c) op.codes(s + to * MT_N, c + g * (MT_N / 2));
  }
  if (c) {  // generation 6 again, from 4 through 5
    op.twist(s + 2 * MT_N, s3);
    op.twist(s3, s3);
  }
}

// Plain ticks of a walk along one axis (the go / ladder loops' plain phases, run_option_k):
// while the coordinate x is inside its span (x <= lim moving in +, x >= lim moving in -), at
// least TICK_DRAWS draws are staged (rng.has) and fewer than `cap` ticks were taken, one draw
// moves x by its noisy step (IM/:361-366: +2..+4 or -4..-2).  Returns the ticks taken.  The
// device's RngCodes takes them four draws per LDS read (RngCodes::walk), with the same result.
template <int DIR, class R>
TG_HD int walk_ticks(R& rng, int& x, int lim, int cap) {
  int t = 0;
  while ((DIR > 0 ? x <= lim : x >= lim) && rng.has(TICK_DRAWS) && t < cap) {
    x += code_step(rng.code(), DIR < 0);
    ++t;
  }
  return t;
}

// Direct-load consumer (few draws per launch: create/reset/classify, and the host checks).
struct Rng {
  uint32_t* mt;    // this env's MT_STORE stored words (the ring's even generations)
  uint32_t pos;    // [0, MT_WORDS), even
  uint32_t draws;  // random() calls (instrumentation for the roofline)
  bool crossed;    // the half not holding pos is stale (MT_STALE on entry, or entered one)
  bool entered;    // entered a half in this launch (the one left is stale)
  uint8_t* mc;     // the env's MT_CODES (device), kept in step when a half is regenerated

  TG_HD Rng(uint32_t* m, uint32_t state, uint8_t* c = nullptr)
      : mt(m), pos(state & MT_POS_MASK), draws(0u), crossed((state & MT_STALE) != 0u),
        entered(false), mc(c) {}

  TG_HD double random() {
    uint32_t w0, w1;
    mt_pair_branchy(mt, pos, w0, w1);
    pos += 2;
    if (pos == (uint32_t)MT_WORDS) pos = 0u;
    if (pos == 0u || pos == (uint32_t)MT_HALF) {
      // entering the other half; a second crossing in one launch finds it stale (a whole ring
      // behind): regenerate it from the half just left before reading it
      if (crossed) twist_half(mt, pos, mc);
      crossed = entered = true;
    }
    ++draws;
    return mt_double(w0, w1);
  }
  // Random.uniform = a + (b-a)*random(); built with -ffp-contract=off (no FMA)
  TG_HD double uniform(double a, double b) { return a + (b - a) * random(); }
  // a draw consumed for its outcome only (see draw_code)
  TG_HD uint32_t code() { return draw_code(random()); }
  // draws come straight from the words: nothing to stage (the device's RngCodes stages codes)
  TG_HD void reserve(uint32_t) {}
  TG_HD bool has(uint32_t) const { return true; }
  TG_HD bool overrun() const { return false; }
  TG_HD void phase(int) {}  // per-phase timing hook of the diagnostic build (tg_amd.hip RngCodes)
  template <int DIR>
  TG_HD int walk(int& x, int lim, int cap) { return walk_ticks<DIR>(*this, x, lim, cap); }
  // the state word to store: position, and whether the other half is stale
  TG_HD uint32_t finish() const { return pos | (crossed ? MT_STALE : 0u); }
  // the same when a refill of the half that was stale on entry is already queued
  TG_HD uint32_t finish_queued() const { return pos | (entered ? MT_STALE : 0u); }
};
// regenerate the stale half (per-lane form of wave_refill); returns the clean state word
TG_HD uint32_t refill_after(uint32_t* mt, uint32_t state, uint8_t* mc = nullptr) {
  const uint32_t pos = state & MT_POS_MASK;
  if (state & MT_STALE) twist_half(mt, (uint32_t)MT_HALF - mt_half(pos), mc);
  return pos;
}

// init_by_array([seed lo, seed hi?]) into 624 words (CPython's state before its first twist)
TG_HD void seed_mt(uint32_t* mt, const uint32_t* genrand19650218, uint64_t seed) {
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  const uint32_t klen = key1 ? 2u : 1u;
  // pass 1: k = max(N, klen) = N iterations starting at i = 1 (wraps once onto mt[1])
  uint32_t prev = genrand19650218[0];
  uint32_t m0 = prev;
  uint32_t j = 0;
  uint32_t i = 1;
  for (int k = 0; k < MT_N; ++k) {
    const uint32_t cur = (i == 1 && k == MT_N - 1) ? mt[1] : genrand19650218[i];
    const uint32_t key = (j == 0) ? key0 : key1;
    const uint32_t v = (cur ^ ((prev ^ (prev >> 30)) * 1664525u)) + key + j;
    mt[i] = v;
    prev = v;
    ++i;
    ++j;
    if (i >= (uint32_t)MT_N) { m0 = mt[MT_N - 1]; prev = m0; i = 1; }
    if (j >= klen) j = 0;
  }
  mt[0] = m0;
  // pass 2: N-1 iterations
  for (int k = 0; k < MT_N - 1; ++k) {
    const uint32_t cur = mt[i];
    const uint32_t v = (cur ^ ((prev ^ (prev >> 30)) * 1566083941u)) - i;
    mt[i] = v;
    prev = v;
    ++i;
    if (i >= (uint32_t)MT_N) { mt[0] = mt[MT_N - 1]; prev = mt[0]; i = 1; }
  }
  mt[0] = 0x80000000u;
}
// random.seed(seed) into an env's ring (per-lane form of tg_create: k_create + k_gen_twist):
// the seeded words (the state before the first twist) in half 0's last stored slot, then the
// ring's generations from them, pos 0
constexpr uint32_t MT_SEED_OFF = 3 * MT_N;  // mt_store_off(6)
TG_HD void init_mt(uint32_t* mt, const uint32_t* genrand19650218, uint64_t seed,
                   uint8_t* mc = nullptr) {
  seed_mt(mt + MT_SEED_OFF, genrand19650218, seed);
  twist_half(mt, 0u, mc, true);
  twist_half(mt, (uint32_t)MT_HALF, mc);
}

// ==========================================================================================
// Map probes.  Every probe is a clamped index into the bordered grid plus one LDS byte read;
// predicates combine probes with bitwise &/| so their LDS reads issue back to back.
// ==========================================================================================
// The cells one air tick at (px, py) can probe, as two 6-bit masks (bit 2*ri + ci: row r0 + ri,
// column c0 + ci): every probe x of the tick lies in [px - 16, px + 16] (33 px: columns c0 =
// colx(px - 16) and c0 + 1), every probe y in [py - 4, py + 53] (58 px: rows r0 = rowy(py - 4)
// .. r0 + 2), the moved player's can_fall4 included (|x step| <= 4).  A probe's cell is then two
// compares against the column / row starts instead of a clamped pixel -> cell division and an
// LDS read; past the border the compares select the clamped cell, as colx / rowy do.
struct AirCells {
  // per window column (A: c0, B: c0 + 1) the rows r0 .. r0 + 2 (bits 0..2) that are OPEN /
  // hold a WALL or a closed door (can_go_side's blockers)
  uint32_t oA, oB, bA, bB;
  int bx, by1;   // first pixel of column c0 + 1 and of row r0 + 1
  uint32_t dc;   // the door state the masks were built for
  // still the window of (dc, px, py): colx(px - 16) == c0 and rowy(py - 4) == r0 (at a clamped
  // border this is false even right after a rebuild: the caller then takes the full tick)
  TG_HD bool holds(uint32_t d, int px, int py) const {
    return (d == dc) & (px - (HALFW + INCR) < bx) & (px - (HALFW + INCR) >= bx - S) &
           (py - INCR < by1) & (py - INCR >= by1 - S);
  }
};

// The air tick's predicates inside its window.  With s = bx - px and t = by1 - py the window
// holds iff s in (-16, 32] and t in [-3, 44], so a probe at px + o lies in column B iff o >= s,
// and one at py + o in row (o >= t) + (o >= t + 48): row 0 for o = -4, row 1 for o = 44, row 1 +
// (t <= 2) for o = 50; each predicate is a few compares and selects of 3-bit row masks
// (AirCells: every probe of the tick, the moved player's fall included, lies in the window).
struct AirProbe {
  const AirCells& ac;
  int s, t;
  TG_HD AirProbe(const AirCells& a, int px, int py) : ac(a), s(a.bx - px), t(a.by1 - py) {}
  static TG_HD uint32_t bit(uint32_t m, uint32_t r) { return (m >> r) & 1u; }
  TG_HD uint32_t open_col(int o) const { return o >= s ? ac.oB : ac.oA; }
  TG_HD uint32_t block_col(int o) const { return o >= s ? ac.bB : ac.bA; }
  TG_HD bool can_fall() const {  // can_fall_at: px -+ 10 at py and py + 50
    const uint32_t c = open_col(-(HALFW - 2)) & open_col(HALFW - 2);
    return (bit(c, (uint32_t)(t <= 0)) & bit(c, 1u + (uint32_t)(t <= 2))) != 0;
  }
  TG_HD bool side(int dir) const {  // can_go_side: px + 16 dir at py + 4 and py + 44
    const uint32_t c = block_col(dir * (HALFW + INCR));
    return (bit(c, (uint32_t)(t <= INCR)) | bit(c, 1u)) == 0;
  }
  TG_HD bool up_clear() const {  // px -+ 4 at py - 4 and py - 1
    const uint32_t c = open_col(-INCR) & open_col(INCR);
    return (bit(c, 0u) & bit(c, (uint32_t)(t <= -1))) != 0;
  }
  // the distance of a downward move of yd <= 4 px (IM/:341-348, Map::fall) after the player's
  // x moved to px2 (by <= 4: still in the window): the probes at py + k and py + 50 + k (k < 4)
  // enter their next row at k = t (if t > 0) / t - 2 (if t > 2); the others at >= 43
  TG_HD int fall(int px2, int yd) const {
    const int s2 = ac.bx - px2;
    const uint32_t c = (-(HALFW - 2) >= s2 ? ac.oB : ac.oA) & ((HALFW - 2) >= s2 ? ac.oB : ac.oA);
    if (!(bit(c, (uint32_t)(t <= 0)) & bit(c, 1u + (uint32_t)(t <= 2)))) return yd;
    int d = yd;
    if (!bit(c, (uint32_t)(t <= 3))) d = min(d, t > 0 ? t : t + S);
    if (!bit(c, 1u + (uint32_t)(t <= 5))) d = min(d, t > 2 ? t - 2 : t + S - 2);
    return d;
  }
};

// ---- level bitmasks (Map::mk) -------------------------------------------------------------------
// For levels of at most MK_DIM - 2 PAD cells a side (the default 14 x 13 is 18 x 17 bordered):
// per bordered column (index c + PAD) the rows holding a LADDER (bit r + PAD); per door state and
// column the OPEN rows; per door state and bordered row the OPEN columns and the WALL-or-closed-
// door columns (bit c + PAD).  Built on the host from the grid (tg_level.h build_masks) and
// staged with it; a predicate that would read several cells of one column or row reads one word
// and tests bits (the ladder and go loops' span limits).  Null: the cell probes.
constexpr int MK_DIM = 32;
constexpr int MK_MAX_WORDS = 25 * MK_DIM;  // 9 column tables + 16 row tables
TG_HD int mk_words(int W, int H) { return 9 * (W + 2 * PAD) + 16 * (H + 2 * PAD); }

struct Map {
  const uint8_t* g;  // LDS on device: (H + 2*PAD) rows of (W + 2*PAD) cells
  int W, H;
  const uint32_t* mk = nullptr;  // the level bitmasks (LDS on device), or null

  TG_HD int pw() const { return W + 2 * PAD; }
  TG_HD int ph() const { return H + 2 * PAD; }
  // mask words: c / r are clamped column / row indices (colx / rowy)
  TG_HD uint32_t mk_lad(int c) const { return mk[c + PAD]; }
  TG_HD uint32_t mk_colopen(uint32_t dc, int c) const { return mk[pw() * (1 + (int)dc) + c + PAD]; }
  TG_HD uint32_t mk_rowopen(uint32_t dc, int r) const { return mk[9 * pw() + ph() * (int)dc + r + PAD]; }
  TG_HD uint32_t mk_rowblk(uint32_t dc, int r) const {
    return mk[9 * pw() + ph() * (8 + (int)dc) + r + PAD];
  }
  TG_HD uint32_t rbit(int y) const { return (uint32_t)(rowy(y) + PAD); }  // row bit of pixel y
  // object_type_at_cell (IM/:227-230) as cell bits; anything outside the grid is WALL
  TG_HD uint32_t cellb(int cx, int cy) const {
    cx = clampi(cx, -PAD, W + PAD - 1);
    cy = clampi(cy, -PAD, H + PAD - 1);
    return g[mul24((uint32_t)(cy + PAD), (uint32_t)pw()) + cx + PAD];
  }
  // the cell column / row atb() probes for pixel x / y (clamped into the WALL border)
  TG_HD int colx(int x) const { return div48(clampi(x, -PAD * S, (W + PAD) * S - 1) + PAD * S) - PAD; }
  TG_HD int rowy(int y) const { return div48(clampi(y, -PAD * S, (H + PAD) * S - 1) + PAD * S) - PAD; }
  // object_type_at (IM/:218-225) as cell bits
  TG_HD uint32_t atb(int x, int y) const {
    x = clampi(x, -PAD * S, (W + PAD) * S - 1) + PAD * S;
    y = clampi(y, -PAD * S, (H + PAD) * S - 1) + PAD * S;
    return g[mul24((uint32_t)div48(y), (uint32_t)pw()) + div48(x)];
  }
  // door state -> type: `dc` = closed-door bits (f >> F_OBJ) & 7
  static TG_HD bool is_open(uint32_t c, uint32_t dc) {
    return ((c & B_OPEN) | ((c >> 4) & ~dc & 7u)) != 0;
  }
  static TG_HD bool is_ladder(uint32_t c) { return (c & B_LADDER) != 0; }
  static TG_HD bool is_wall(uint32_t c) { return (c & B_WALL) != 0; }
  static TG_HD bool is_door(uint32_t c, uint32_t dc) {
    return ((c & B_DOOR) | ((c >> 4) & dc)) != 0;
  }
  static TG_HD uint32_t dc_of(uint32_t f) { return (f >> F_OBJ) & 7u; }

  TG_HD bool open_at(uint32_t dc, int x, int y) const { return is_open(atb(x, y), dc); }
  TG_HD bool open_cell(uint32_t dc, int cx, int cy) const { return is_open(cellb(cx, cy), dc); }

  // up_clear (IM/:232-238): xs {px-4, px, px+4} x ys [py-4, py-1] all OPEN; the three xs
  // span at most two columns and the four ys at most two rows
  TG_HD bool up_clear(const Env& e) const {
    const uint32_t dc = dc_of(e.f);
    const int x0 = e.px - INCR, x1 = e.px + INCR, y0 = e.py - INCR, y1 = e.py - 1;
    return open_at(dc, x0, y0) & open_at(dc, x1, y0) & open_at(dc, x0, y1) & open_at(dc, x1, y1);
  }
  // can_go_up (IM/:240-250): ys {py-4, py, py+44} x xs {px-12, px+12}, any LADDER
  TG_HD bool can_go_up(const Env& e) const {
    const int xa = e.px - HALFW, xb = e.px + HALFW;
    const int y0 = e.py - INCR, y1 = e.py, y2 = e.py + S - INCR;
    const uint32_t any = atb(xa, y0) | atb(xb, y0) | atb(xa, y1) | atb(xb, y1) | atb(xa, y2) |
                         atb(xb, y2);
    return (e.py > 1) & is_ladder(any);
  }
  // can_go_down (IM/:252-257): ys [py, py+51] x xs {px-12, px+12}, any LADDER.  The 52 ys span
  // at most three rows; rows outside the grid are WALL, so probing the clamped rows
  // y, y+24, y+51 (every row of the span contains one of them) is exact.
  TG_HD bool can_go_down(const Env& e) const {
    const int xa = e.px - HALFW, xb = e.px + HALFW;
    const int y0 = e.py, y1 = e.py + S / 2, y2 = e.py + S + INCR - 1;
    const uint32_t any = atb(xa, y0) | atb(xb, y0) | atb(xa, y1) | atb(xb, y1) | atb(xa, y2) |
                         atb(xb, y2);
    return is_ladder(any);
  }
  // can_go_left / can_go_right (IM/:259-281): x = px -/+ 16 at ys {py+4, py+44}
  TG_HD bool can_go_side(const Env& e, int dir) const {
    const uint32_t dc = dc_of(e.f);
    const int x = e.px + dir * (HALFW + INCR);
    const uint32_t ta = atb(x, e.py + INCR), tb = atb(x, e.py + S - INCR);
    return !(is_wall(ta | tb) | is_door(ta, dc) | is_door(tb, dc));
  }
  // can_fall (IM/:283-288): xs {px-10, px+10} x ys {py, py+50} all OPEN
  TG_HD bool can_fall_at(uint32_t dc, int px, int py) const {
    const int xa = px - HALFW + 2, xb = px + HALFW - 2, ya = py, yb = py + S + 2;
    return open_at(dc, xa, ya) & open_at(dc, xa, yb) & open_at(dc, xb, ya) & open_at(dc, xb, yb);
  }
  TG_HD bool can_fall(const Env& e) const { return can_fall_at(dc_of(e.f), e.px, e.py); }
  // AirCells at (px, py): six LDS reads in one batch (rows and the second column clamped)
  TG_HD AirCells air_cells(uint32_t dc, int px, int py) const {
    const int c0 = colx(px - (HALFW + INCR)), r0 = rowy(py - INCR);
    const uint32_t x0 = (uint32_t)(c0 + PAD), x1 = (uint32_t)(c0 + 1 < W + PAD ? c0 + 1 + PAD : c0 + PAD);
    uint32_t oa = 0, ob = 0, ba = 0, bb = 0;
#pragma unroll
    for (int ri = 0; ri < 3; ++ri) {
      const int r = r0 + ri < H + PAD ? r0 + ri : H + PAD - 1;
      const uint8_t* const row = g + mul24((uint32_t)(r + PAD), (uint32_t)pw());
      const uint32_t ca = row[x0], cb = row[x1];
      oa |= (uint32_t)is_open(ca, dc) << ri;
      ob |= (uint32_t)is_open(cb, dc) << ri;
      ba |= (uint32_t)(is_wall(ca) | is_door(ca, dc)) << ri;
      bb |= (uint32_t)(is_wall(cb) | is_door(cb, dc)) << ri;
    }
    return AirCells{oa, ob, ba, bb, (c0 + 1) * S, (r0 + 1) * S, dc};
  }
  // integrate y on a downward move of yd <= 4 px (IM/:341-348): with can_fall at py the player
  // falls pixel by pixel while can_fall holds, so the distance is the first k in 1..yd-1 with
  // !can_fall(py + k), else yd.  The probes (px -+ 10 at py + k and py + 50 + k, k < 4) span at
  // most two rows each, entering the second at k = ka / kb: 8 lookups instead of 16, and the
  // first failing k in closed form (rows past the border clamp to the same WALL row, where
  // both lookups agree anyway)
  TG_HD int fall(uint32_t dc, int px, int py, int yd) const {
    const int ca = colx(px - HALFW + 2), cb = colx(px + HALFW - 2);
    const int ya = py, yb = py + S + 2;
    const int ra0 = rowy(ya), ra1 = rowy(ya + 3), rb0 = rowy(yb), rb1 = rowy(yb + 3);
    const bool a0 = is_open(cellb(ca, ra0), dc) & is_open(cellb(cb, ra0), dc);
    const bool a1 = is_open(cellb(ca, ra1), dc) & is_open(cellb(cb, ra1), dc);
    const bool b0 = is_open(cellb(ca, rb0), dc) & is_open(cellb(cb, rb0), dc);
    const bool b1 = is_open(cellb(ca, rb1), dc) & is_open(cellb(cb, rb1), dc);
    if (!(a0 & b0)) return yd;
    const int ka = S - (ya - floordiv48(ya) * S), kb = S - (yb - floordiv48(yb) * S);
    int d = yd;
    if (!a1) d = min(d, ka);
    if (!b1) d = min(d, kb);
    return d;
  }
};

// The ladder options' probes from the level bitmasks: px is fixed while a ladder option runs
// (its primitives UP / DOWN / NOP and the gravity move only py), and so are the door states, so
// the columns of every probe are: LADDER rows at px -+ 12 (can_go_up / can_go_down), OPEN rows at
// both px -+ 10 (can_fall) and at both px -+ 4 (up_clear, for a leftover jump ticker).
struct LadMasks {
  uint32_t lad, fall, up;
  TG_HD LadMasks(const Map& m, uint32_t dc, int px)
      : lad(m.mk_lad(m.colx(px - HALFW)) | m.mk_lad(m.colx(px + HALFW))),
        fall(m.mk_colopen(dc, m.colx(px - HALFW + 2)) & m.mk_colopen(dc, m.colx(px + HALFW - 2))),
        up(m.mk_colopen(dc, m.colx(px - INCR)) & m.mk_colopen(dc, m.colx(px + INCR))) {}
  // Map::can_go_up / can_go_down / can_fall_at / up_clear / fall at (px, py)
  TG_HD bool can_go_up(const Map& m, int py) const {
    return (py > 1) & ((((lad >> m.rbit(py - INCR)) | (lad >> m.rbit(py)) | (lad >> m.rbit(py + S - INCR))) & 1u) != 0);
  }
  TG_HD bool can_go_down(const Map& m, int py) const {
    return (((lad >> m.rbit(py)) | (lad >> m.rbit(py + S / 2)) | (lad >> m.rbit(py + S + INCR - 1))) & 1u) != 0;
  }
  TG_HD bool can_fall(const Map& m, int py) const {
    return ((fall >> m.rbit(py)) & (fall >> m.rbit(py + S + 2)) & 1u) != 0;
  }
  TG_HD bool up_clear(const Map& m, int py) const {
    return ((up >> m.rbit(py - INCR)) & (up >> m.rbit(py - 1)) & 1u) != 0;
  }
  TG_HD int fall_dist(const Map& m, int py, int yd) const {
    const int ya = py, yb = py + S + 2;
    if (!((fall >> m.rbit(ya)) & (fall >> m.rbit(yb)) & 1u)) return yd;
    const int ka = S - (ya - floordiv48(ya) * S), kb = S - (yb - floordiv48(yb) * S);
    int d = yd;
    if (!((fall >> m.rbit(ya + 3)) & 1u)) d = min(d, ka);
    if (!((fall >> m.rbit(yb + 3)) & 1u)) d = min(d, kb);
    return d;
  }
};

// ==========================================================================================
// Objects, bag, triggers (OB/, IM/:402-445)
// ==========================================================================================
// near_enough (OB/:46-53) for the player probe (px, py + 24): centre (cx*48+24, cy*48+24)
TG_HD bool near_cell(const Env& e, int cx, int cy, int r2) {
  const int dx = e.px - (cx * S + S / 2);
  const int dy = e.py - cy * S;
  return dx * dx + dy * dy < r2;
}
constexpr int R2_OBJ = (S / 2) * (S / 2);            // radius xscale/2 (OB/:23)
constexpr int R2_HANDLE = (S * 3 / 4) * (S * 3 / 4);  // radius xscale*0.75 (OB/:115)

TG_HD int bag_len(uint32_t f) { return (f >> F_BAGLEN) & 7; }
TG_HD uint32_t bag_items(uint32_t f) { return (f >> F_BAGITEM) & 0x7F; }
TG_HD bool got_key(uint32_t f) {   // player_got_key (IM/:418-422)
  const uint32_t live = (1u << bag_len(f)) - 1u;
  return (~bag_items(f) & live) != 0;
}
TG_HD bool got_gold(uint32_t f) {  // player_got_goldcoin (IM/:424-428)
  const uint32_t live = (1u << bag_len(f)) - 1u;
  return (bag_items(f) & live) != 0;
}
TG_HD void bag_push(uint32_t& f, bool gold) {
  const int n = bag_len(f);
  if (n >= 7) { f |= E_BAG; return; }
  f = (f & ~(7u << F_BAGLEN)) | ((uint32_t)(n + 1) << F_BAGLEN);
  if (gold) f |= 1u << (F_BAGITEM + n);
}
// drop_key (IM/:434-439): remove the first key, move it to (-1,-1)
TG_HD void drop_key(Env& e) {
  const int n = bag_len(e.f);
  const uint32_t items = bag_items(e.f);
  const uint32_t keys = ~items & ((1u << n) - 1u);
  if (!keys) return;
  const int i = __builtin_ctz(keys);
  const uint32_t lo = items & ((1u << i) - 1u), hi = (items >> (i + 1)) << i;
  e.f = (e.f & ~((7u << F_BAGLEN) | (0x7Fu << F_BAGITEM))) | ((uint32_t)(n - 1) << F_BAGLEN) |
        ((lo | hi) << F_BAGITEM);
  e.kx = -1;
  e.ky = -1;
}

// is_object_at (IM/:402-409): handles, closed doors, bolt, gold, key at the cell
TG_HD bool is_object_at(const Level& L, const Env& e, int xc, int yc) {
  bool r = ((xc == L.handle_cx[0]) & (yc == L.handle_cy[0])) |
           ((xc == L.handle_cx[1]) & (yc == L.handle_cy[1])) |
           ((xc == L.bolt_cx) & (yc == L.bolt_cy)) | ((xc == e.gx) & (yc == e.gy)) |
           ((xc == e.kx) & (yc == e.ky));
#pragma unroll
  for (int i = 0; i < 3; ++i)
    r |= (xc == L.door_cx[i]) & (yc == L.door_cy[i]) & (((e.f >> (F_OBJ + i)) & 1u) != 0);
  return r;
}
// is_closed_door_at (IM/:411-416)
TG_HD bool is_closed_door_at(const Level& L, const Env& e, int xc, int yc) {
  bool r = false;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    r |= (xc == L.door_cx[i]) & (yc == L.door_cy[i]) & (((e.f >> (F_OBJ + i)) & 1u) != 0);
  return r;
}

// handle.set_angle_wiggle (OB/:127-131)
template <class R>
TG_HD void wiggle(Env& e, int h, R& rng) {
  const bool up = (e.f >> (F_OBJ + 3 + h)) & 1u;
  const double a = up ? rng.uniform(0.85, 1.0) : rng.uniform(0, 0.15);
  if (h == 0) e.ang0 = a; else e.ang1 = a;
}
// set_val of door (OB/:231-235) / handle (OB/:145-149) / bolt (OB/:175-178): apply only
template <class R>
TG_HD bool set_val(Env& e, int o, int v, R& rng) {
  const uint32_t bit = 1u << (F_OBJ + o);
  if ((((e.f & bit) != 0) ? 1 : 0) == v) return false;
  e.f ^= bit;
  if (o == 3 || o == 4) wiggle(e, o - 3, rng);
  return true;
}
// set_val(o0, v0) followed by the process_trigger cascade (OB/:76-94), depth-first in file
// order with the previously_triggered guard; frames are 8 bits of one u64.  `trig` is the
// level's [6][2] trigger table (LDS on device).
template <class R>
TG_HD void cascade(const uint32_t* trig, Env& e, int o0, int v0, R& rng) {
  if (!set_val(e, o0, v0, rng)) return;
  uint64_t stack = (uint64_t)(o0 | (v0 << 3));
  uint32_t prev = 1u << o0;
  int depth = 1;
  while (depth > 0) {
    const uint32_t fr = (uint32_t)(stack & 0xFFu);
    const int o = fr & 7, v = (fr >> 3) & 1, ei = fr >> 4;
    const uint32_t list = trig[o * 2 + v];
    if (ei < (int)(list & 0xFu)) {
      stack += 0x10u;
      const uint32_t edge = (list >> (4 + 4 * ei)) & 0xFu;
      const int t = edge & 7, tv = (edge >> 3) & 1;
      if (!(prev & (1u << t)) && set_val(e, t, tv, rng)) {
        stack = (stack << 8) | (uint64_t)(t | (tv << 3));
        prev |= 1u << t;
        ++depth;
      }
    } else {
      stack >>= 8;
      prev &= ~(1u << o);
      --depth;
    }
  }
}
// handle.flip (OB/:117-122): uniform(0, 1) <= 0.8 (== random() exactly: CODE_FLIP)
template <class R>
TG_HD void flip(const uint32_t* trig, Env& e, int h, R& rng) {
  if (rng.code() & CODE_FLIP) {
    const int up = (e.f >> (F_OBJ + 3 + h)) & 1u;
    cascade(trig, e, 3 + h, !up, rng);
  } else {
    wiggle(e, h, rng);
  }
}

// pickups in object order: key then goldcoin (IM/:350-354).  near_cell needs |dx| < 24 for
// r = 24, so a tick whose player is 24 px or more from both objects' centres in x (nearly every
// tick) skips the rest with one combined test.
TG_HD void pickups(const Level& L, Env& e) {
  const int dkx = e.px - (e.kx * S + S / 2), dgx = e.px - (e.gx * S + S / 2);
  if (((uint32_t)(dkx + (S / 2 - 1)) >= (uint32_t)(S - 1)) & ((uint32_t)(dgx + (S / 2 - 1)) >= (uint32_t)(S - 1)))
    return;
  if (near_cell(e, e.kx, e.ky, R2_OBJ)) {
    e.kx = L.W - 1 - bag_len(e.f);
    e.ky = L.H - 1;
    bag_push(e.f, false);
  }
  if (near_cell(e, e.gx, e.gy, R2_OBJ)) {
    e.gx = L.W - 1 - bag_len(e.f);
    e.gy = L.H - 1;
    bag_push(e.f, true);
  }
}

// ==========================================================================================
// Primitive tick: _TreasureGameImpl.step (IM/:290-359).  PM is the set of primitive actions
// the caller can issue (a compile-time mask); the others compile away.
// ==========================================================================================
constexpr uint32_t PM_ALL = 0x7Fu;
template <uint32_t PM>
TG_HD bool may(int prim, int p) { return ((PM >> p) & 1u) && prim == p; }

template <uint32_t PM, class R>
TG_HD int tick(const Level& L, const uint32_t* trig, const Map& m, Env& e, int prim, R& rng) {
  int xd = 0, yd = 0;
  // the action's precondition (IM/:297-319); moves and the jump share one draw site
  bool ok = false;
  if (may<PM>(prim, P_UP)) ok = m.can_go_up(e);
  else if (may<PM>(prim, P_DOWN)) ok = m.can_go_down(e);
  else if (may<PM>(prim, P_LEFT)) ok = m.can_go_side(e, -1);
  else if (may<PM>(prim, P_RIGHT)) ok = m.can_go_side(e, +1);
  else if (may<PM>(prim, P_JUMP)) ok = !m.can_go_down(e) && m.up_clear(e);
  if (ok) {
    const uint32_t c = rng.code();
    if (may<PM>(prim, P_JUMP)) {  // jump_ticker = 22, or 23 if random() > 0.25 (IM/:317-319)
      e.f = (e.f & ~F_JT) | ((c & CODE_JUMP) ? 23u : 22u);
    } else {
      // noisy(+-4) (IM/:361-366): int(round(uniform(-4, -2.0))) or int(round(uniform(2.0, 4))),
      // uniform = a + (b-a)*r with b-a = 2.0 exactly; round() half-to-even == rint (draw_code)
      const bool neg = may<PM>(prim, P_UP) | may<PM>(prim, P_LEFT);
      const int d = code_step(c, neg);
      if (may<PM>(prim, P_LEFT) | may<PM>(prim, P_RIGHT)) {
        xd = d;
        e.f = may<PM>(prim, P_RIGHT) ? (e.f | F_FACING) : (e.f & ~F_FACING);
      } else {
        yd = d;
      }
    }
  }
  if (may<PM>(prim, P_INTERACT)) {  // object list order: handles (3,4) before the bolt (6)
    if (near_cell(e, L.handle_cx[0], L.handle_cy[0], R2_HANDLE)) flip(trig, e, 0, rng);
    if (near_cell(e, L.handle_cx[1], L.handle_cy[1], R2_HANDLE)) flip(trig, e, 1, rng);
    if (near_cell(e, L.bolt_cx, L.bolt_cy, R2_OBJ) && got_key(e.f)) {
      cascade(trig, e, 5, 0, rng);  // try_unlock -> bolt.unlock (IM/:430-432)
      drop_key(e);
    }
  }
  // jump ticker / gravity (IM/:331-337), both at the pre-move x
  const uint32_t jt = e.f & F_JT;
  if (jt > 0) {
    if (m.up_clear(e)) yd = -INCR;
    e.f = (e.f & ~F_JT) | (jt - 1);
  } else if (m.can_fall(e)) {
    yd = INCR;  // jump_ticker already 0
  }
  e.px += xd;
  // integrate y (IM/:341-348): with yd > 0 and can_fall, fall pixel by pixel while can_fall
  // holds: the distance is the first k in 1..yd-1 with !can_fall(py + k), else yd (yd <= 4)
  if (yd > 0) yd = m.fall(Map::dc_of(e.f), e.px, e.py, yd);
  e.py += yd;
  pickups(L, e);
  return may<PM>(prim, P_JUMP) ? -5 : -1;  // JUMP_REWARD / STEP_REWARD (IM/:15-16)
}

// ==========================================================================================
// Options (MO/)
// ==========================================================================================
TG_HD void player_cell(const Env& e, int& xc, int& yc) {  // IM/:441-445
  xc = floordiv48(e.px);  // floordiv(px, S); players stay inside the level
  yc = floordiv48(e.py + S / 2);
}
// close_enough_to / close_enough_x: |tx*48 + 24 - px| < 4 (MO/:69-72 and its copies)
TG_HD bool close_x(const Env& e, int txc) {
  const int d = txc * S + S / 2 - e.px;
  return (d < 0 ? -d : d) < INCR;
}
// go_left / go_right is_target_cell (MO/:54-67, 126-139)
TG_HD bool go_is_target(const Level& L, const Map& m, const Env& e, int dir, int xc, int yc) {
  const uint32_t dc = Map::dc_of(e.f);
  const uint32_t up = m.cellb(xc, yc - 1), dn = m.cellb(xc, yc + 1), sd = m.cellb(xc + dir, yc),
                 sdn = m.cellb(xc + dir, yc + 1);
  return Map::is_ladder(up | dn) | Map::is_wall(sd) | is_object_at(L, e, xc, yc) |
         is_closed_door_at(L, e, xc + dir, yc) | Map::is_open(sdn, dc);
}
// get_target_cell (MO/:43-52; MO/:115-124 whose xc<0 test can never fire going right, and
// terminates because OOB is WALL)
TG_HD bool go_target(const Level& L, const Map& m, const Env& e, int dir, int xc, int yc, int& tx) {
  int x = xc + dir;
  while (!go_is_target(L, m, e, dir, x, yc)) {
    x += dir;
    if (x < 0) return false;
  }
  tx = x;
  return true;
}
// jump landing (MO/:281-287)
TG_HD bool landing(const Map& m, const Env& e, int xc, int yc) {
  return m.open_cell(Map::dc_of(e.f), xc, yc) & Map::is_wall(m.cellb(xc, yc + 1));
}

// ---- GoTable: the go options' can_run and target, precomputed --------------------------------
// go_left / go_right's can_run (MO/:23-41, 95-113) and target (MO/:43-67, 115-139) read only
// the player's cell (xc, yc), cell types of rows yc - 1 .. yc + 1, the door states and, through
// is_object_at (IM/:402-409), the key's and the gold's cells on row yc.  The key is at home, in
// the bag (row H - 1) or at (-1, -1); the gold at home or in the bag.  So for a player cell
// inside the grid whose row holds neither a moved key nor a bagged gold (row H - 1 is a wall
// in every playable level), the answer depends on (cell, door state, key at home, gold at
// home) only: entry ((yc * W + xc) * 8 + doors) * 4 + key_home * 2 + gold_home holds
// bit 0 / 1 = can_run left / right, bits 8-15 / 16-23 = target column + 1.
TG_HD bool go_lookup(const Level& L, const Env& e, int xc, int yc, uint32_t& out) {
  if (!L.gotab || xc < 0 || xc >= L.W || yc < 0 || yc >= L.H) return false;
  const bool kh = e.kx == L.key_cx && e.ky == L.key_cy, gh = e.gx == L.gold_cx && e.gy == L.gold_cy;
  if ((!kh && e.ky == yc) || (!gh && e.gy == yc)) return false;
  out = L.gotab[((yc * L.W + xc) * 8 + (int)Map::dc_of(e.f)) * 4 + (kh ? 2 : 0) + (gh ? 1 : 0)];
  return true;
}
TG_HD bool can_run(const Level& L, const Map& m, const Env& e, int k) {
  int xc, yc;
  player_cell(e, xc, yc);
  const uint32_t dc = Map::dc_of(e.f);
  switch (k) {
    case O_GO_LEFT:
    case O_GO_RIGHT: {  // MO/:23-41, 95-113
      const int dir = k == O_GO_LEFT ? -1 : 1;
      uint32_t gt;
      if (go_lookup(L, e, xc, yc, gt)) return (gt >> (k == O_GO_LEFT ? 0 : 1)) & 1u;
      int tc;
      if (!go_target(L, m, e, dir, xc, yc, tc)) return false;
      for (int x = xc; dir < 0 ? x >= tc : x <= tc; x += dir) {
        if (!m.open_cell(dc, x, yc)) return false;
        if (m.open_cell(dc, x, yc + 1)) return false;
      }
      return true;
    }
    case O_UP_LADDER: return m.can_go_up(e);      // MO/:165-166
    case O_DOWN_LADDER: return m.can_go_down(e);  // MO/:181-182
    case O_INTERACT:                              // MO/:446-455
      return near_cell(e, L.handle_cx[0], L.handle_cy[0], R2_HANDLE) ||
             near_cell(e, L.handle_cx[1], L.handle_cy[1], R2_HANDLE) ||
             (near_cell(e, L.bolt_cx, L.bolt_cy, R2_OBJ) && got_key(e.f));
    case O_DOWN_LEFT:
    case O_DOWN_RIGHT: {  // MO/:199-209, 394-404
      const int dir = k == O_DOWN_LEFT ? -1 : 1;
      return m.open_cell(dc, xc + dir, yc) & m.open_cell(dc, xc + dir, yc + 1);
    }
    case O_JUMP_LEFT:
    case O_JUMP_RIGHT: {  // MO/:254-267, 324-337
      const int dir = k == O_JUMP_LEFT ? -1 : 1;
      return m.open_cell(dc, xc, yc - 1) & m.open_cell(dc, xc + dir, yc - 1) &
             (landing(m, e, xc + dir, yc - 1) | landing(m, e, xc + 2 * dir, yc - 1));
    }
  }
  return false;
}

TG_HD uint32_t available_mask(const Level& L, const Map& m, const Env& e) {  // TG/:83-89
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < O_COUNT; ++k) r |= (uint32_t)can_run(L, m, e, k) << k;
  return r;
}

// option-local state (start_cell / target_cell are None between steps, MO/:80-83 etc.)
struct Opt {
  int tx;      // target cell x
  bool init;   // target computed
  bool done;
};

// primitive actions each option's policy can return
constexpr uint32_t prims_of(int k) {
  return k == O_GO_LEFT ? (1u << P_LEFT)
       : k == O_GO_RIGHT ? (1u << P_RIGHT)
       : k == O_UP_LADDER ? (1u << P_UP) | (1u << P_NOP)
       : k == O_DOWN_LADDER ? (1u << P_DOWN) | (1u << P_NOP)
       : k == O_INTERACT ? (1u << P_INTERACT)
       : k == O_DOWN_LEFT ? (1u << P_LEFT) | (1u << P_NOP)
       : k == O_DOWN_RIGHT ? (1u << P_RIGHT) | (1u << P_NOP)
       : (1u << P_JUMP) | (1u << P_LEFT) | (1u << P_RIGHT) | (1u << P_NOP);
}

// policy_step of option K (MO/)
template <int K>
TG_HD int policy(const Level& L, const Map& m, const Env& e, Opt& o) {
  int xc, yc;
  if (K == O_GO_LEFT || K == O_GO_RIGHT) {  // MO/:74-85, 146-157
    constexpr int dir = K == O_GO_LEFT ? -1 : 1;
    if (!o.init) {
      player_cell(e, xc, yc);
      uint32_t gt;
      if (go_lookup(L, e, xc, yc, gt)) o.tx = (int)((gt >> (dir < 0 ? 8 : 16)) & 0xFFu) - 1;
      else go_target(L, m, e, dir, xc, yc, o.tx);  // exists: can_run checked it
      o.init = true;
    }
    if (close_x(e, o.tx)) o.done = true;
    return dir < 0 ? P_LEFT : P_RIGHT;
  } else if (K == O_UP_LADDER) {  // MO/:168-173
    if (!m.can_go_up(e)) { o.done = true; return P_NOP; }
    return P_UP;
  } else if (K == O_DOWN_LADDER) {  // MO/:184-189
    if (!m.can_go_down(e)) { o.done = true; return P_NOP; }
    return P_DOWN;
  } else if (K == O_INTERACT) {  // MO/:457-460
    o.done = true;
    return P_INTERACT;
  } else if (K == O_DOWN_LEFT || K == O_DOWN_RIGHT) {  // MO/:231-244, 426-439
    constexpr int dir = K == O_DOWN_LEFT ? -1 : 1;
    if (!o.init) {
      // get_target_cell (MO/:211-221, 406-416) scans down column xc+dir for the first
      // non-open cell; only its x is ever used (close_enough_x).  It returns None only if
      // the scan leaves the grid, after which the reference raises TypeError; the bottom
      // row of a walled level never lets that happen.
      player_cell(e, xc, yc);
      o.tx = xc + dir;
      o.init = true;
    }
    if (close_x(e, o.tx)) {
      if (!m.can_fall(e)) o.done = true;
      return P_NOP;
    }
    return dir < 0 ? P_LEFT : P_RIGHT;
  } else {  // O_JUMP_LEFT / O_JUMP_RIGHT (MO/:297-314, 367-384)
    constexpr int dir = K == O_JUMP_LEFT ? -1 : 1;
    if (!o.init) {
      player_cell(e, xc, yc);
      o.tx = landing(m, e, xc + dir, yc - 1) ? xc + dir : xc + 2 * dir;  // MO/:269-279
      o.init = true;
      return P_JUMP;
    }
    if (close_x(e, o.tx)) {
      if (!m.can_fall(e)) o.done = true;
      return P_NOP;
    }
    const bool back = !m.can_fall(e) && !m.can_go_side(e, dir);
    return (back ? -dir : dir) < 0 ? P_LEFT : P_RIGHT;
  }
}

// ==========================================================================================
// Observation (IM/:368-378 + OB/:157-158,186-190,202-203,215-216) and done (TG/:95)
// ==========================================================================================
// v / d, from the level's quotient table when v is inside it (the table holds the same IEEE
// quotients: an f64 division is ~11 VALU instructions on the device, the reciprocal among them)
TG_HD double obs_div(const Level& L, int v, int base, int n, double d) {
  const uint32_t i = (uint32_t)(v - Q_MIN);
  return (L.obs_q && i < (uint32_t)n) ? L.obs_q[base + (int)i] : (double)v / d;
}
TG_HD void observe(const Level& L, const Env& e, double o[9]) {
  const double w = (double)(L.W * S), h = (double)(L.H * S);
  o[0] = obs_div(L, e.px, 0, L.qx_n, w);
  o[1] = obs_div(L, e.py, L.qx_n, L.qy_n, h);
  o[2] = e.ang0;
  o[3] = e.ang1;
  o[4] = obs_div(L, e.kx * S, 0, L.qx_n, w);
  o[5] = obs_div(L, e.ky * S, L.qx_n, L.qy_n, h);
  o[6] = ((e.f >> (F_OBJ + 5)) & 1u) ? 1.0 : 0.0;
  o[7] = obs_div(L, e.gx * S, 0, L.qx_n, w);
  o[8] = obs_div(L, e.gy * S, L.qx_n, L.qy_n, h);
}
TG_HD bool is_done(const Env& e) {
  int xc, yc;
  player_cell(e, xc, yc);
  return got_gold(e.f) && yc == 0;
}

// ==========================================================================================
// reset_game (IM/:55-73): objects re-read (handle angles, 2 draws), start position (gauss
// pair, 2 draws), empty bag.  Keeps the error bits.
// ==========================================================================================
template <class R>
TG_HD void reset_env(const Level& L, Env& e, R& rng) {
  rng.reserve(4);
  e.f = (e.f & E_MASK) | L.init_flags | F_FACING;
  e.ang0 = ((L.init_flags >> (F_OBJ + 3)) & 1u) ? rng.uniform(0.85, 1.0) : rng.uniform(0, 0.15);
  e.ang1 = ((L.init_flags >> (F_OBJ + 4)) & 1u) ? rng.uniform(0.85, 1.0) : rng.uniform(0, 0.15);
  e.kx = L.key_cx;
  e.ky = L.key_cy;
  e.gx = L.gold_cx;
  e.gy = L.gold_cy;
  // player_initial_position (IM/:168-178) with Random.gauss's pair (gauss_next consumed)
  const double x2pi = rng.random() * (2.0 * 3.141592653589793);
  const double g2rad = sqrt(-2.0 * log(1.0 - rng.random()));
  const double zx = 0.0 + (cos(x2pi) * g2rad) * (S / 24.0);
  const double zy = fabs(0.0 + (sin(x2pi) * g2rad) * (S / 36.0));
  const double fx = fabs(zx) - floor(fabs(zx)), fy = zy - floor(zy);
  if ((fabs(zx) >= 0.5 && (fx < 1e-9 || fx > 1.0 - 1e-9)) || (zy >= 0.5 && (fy < 1e-9 || fy > 1.0 - 1e-9)))
    e.f |= E_NEARINT;
  e.px = L.start_x * S + S / 2 + (int)zx;
  e.py = L.start_y * S + (int)zy;
}

// Random.gauss's cached second value (CPython random.py gauss: gauss_next), for an env that
// draws from a shared Python-level stream (the N=1 drop-in's default, tg_reset1_py)
struct GaussNext {
  bool has;
  double v;
};
// z of Random.gauss (the caller applies mu + z * sigma): the cached value if there is one,
// else a fresh pair (2 draws) whose second value is cached
template <class R>
TG_HD double gauss_z(R& rng, GaussNext& g) {
  if (g.has) {
    g.has = false;
    return g.v;
  }
  const double x2pi = rng.random() * (2.0 * 3.141592653589793);
  const double g2rad = sqrt(-2.0 * log(1.0 - rng.random()));
  g.v = sin(x2pi) * g2rad;
  g.has = true;
  return cos(x2pi) * g2rad;
}
// reset_env with the stream's gauss_next carried in and out (reset_env assumes it unset, as
// after random.seed, and leaves it unset: the two gauss calls consume one pair)
template <class R>
TG_HD void reset_env_gauss(const Level& L, Env& e, R& rng, GaussNext& g) {
  e.f = (e.f & E_MASK) | L.init_flags | F_FACING;
  e.ang0 = ((L.init_flags >> (F_OBJ + 3)) & 1u) ? rng.uniform(0.85, 1.0) : rng.uniform(0, 0.15);
  e.ang1 = ((L.init_flags >> (F_OBJ + 4)) & 1u) ? rng.uniform(0.85, 1.0) : rng.uniform(0, 0.15);
  e.kx = L.key_cx;
  e.ky = L.key_cy;
  e.gx = L.gold_cx;
  e.gy = L.gold_cy;
  const double zx = 0.0 + gauss_z(rng, g) * (S / 24.0);
  const double zy = fabs(0.0 + gauss_z(rng, g) * (S / 36.0));
  const double fx = fabs(zx) - floor(fabs(zx)), fy = zy - floor(zy);
  if ((fabs(zx) >= 0.5 && (fx < 1e-9 || fx > 1.0 - 1e-9)) || (zy >= 0.5 && (fy < 1e-9 || fy > 1.0 - 1e-9)))
    e.f |= E_NEARINT;
  e.px = L.start_x * S + S / 2 + (int)zx;
  e.py = L.start_y * S + (int)zy;
}

// ==========================================================================================
// One env-step: TreasureGame.step (TG/:91-96) -> _Option.run (OP/:20-36)
// ==========================================================================================
struct StepResult {
  int reward;  // sum of tick rewards (0 when the option could not run)
  int ran;     // 0 == the reference returns reward None
  int done;    // got gold and back in row 0
  int ticks;
};
// ==========================================================================================
// Plain go ticks.  While a go option walks on flat ground, its tick (policy MO/:74-85 +
// IM/:290-359) probes the same cells and finds: not close to the target, side clear, no
// jump ticker, no fall, no object in reach.  Such a tick is exactly: one draw, px += the
// noisy step, facing set, reward -1.  go_plain_limit() returns how far px may go in the
// direction of motion with all of those facts unchanged (INT_MIN / INT_MAX: not at all):
//   * the probed columns px + 16*dir (can_go_side) and px -/+ 10 (can_fall) stay in their
//     48-px cells (rows fixed: py does not change);
//   * close_x: |T - px| >= 4 until 4 px short of the target centre T;
//   * near_cell(key | gold): dx^2 + dy^2 < 24^2 needs |dx| < 24, so an object whose row is
//     within reach bounds the span 24 px short of its centre.
// Motion is monotonic (steps of 2-4 px in dir), so one bound per fact suffices.  A plain
// tick whose step leaves the span checks the pickups at its new px as the full tick does;
// the next tick is a full one, which computes the next span.
// ==========================================================================================
template <int DIR>
TG_HD int go_plain_limit(const Map& m, const Env& e, int tx) {
  constexpr int NONE = DIR > 0 ? -0x40000000 : 0x40000000;
  if ((e.f & F_JT) || !m.can_go_side(e, DIR) || m.can_fall(e) || close_x(e, tx)) return NONE;
  const int P = e.px;
  // target and objects (px never reaches them inside the span)
  const int T = tx * S + S / 2;
  int lim = DIR > 0 ? T - INCR : T + INCR;
  const int ocx[2] = {e.kx, e.gx}, ocy[2] = {e.ky, e.gy};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int dy = e.py - ocy[j] * S;
    if (dy * dy >= R2_OBJ) continue;
    const int X = ocx[j] * S + S / 2;
    if ((P - X < 0 ? X - P : P - X) < S / 2) return NONE;
    if (DIR > 0 && X > P) lim = min(lim, X - S / 2);
    if (DIR < 0 && X < P) lim = max(lim, X + S / 2);
  }
  if (DIR > 0 ? lim < P : lim > P) return NONE;
  // the probed rows are fixed (py does not change in the span)
  const uint32_t dc = Map::dc_of(e.f);
  const int rs1 = m.rowy(e.py + INCR), rs2 = m.rowy(e.py + S - INCR);  // can_go_side
  const int rf1 = m.rowy(e.py), rf2 = m.rowy(e.py + S + 2);            // can_fall
  if (m.mk) {  // the same two scans as bit scans over the rows' column masks (below)
    const int off = DIR * (HALFW + INCR);
    const int c0 = m.colx(P + off) + PAD, c1 = m.colx(lim + off) + PAD;  // bit indices
    const uint32_t blk = m.mk_rowblk(dc, rs1) | m.mk_rowblk(dc, rs2);
    // columns strictly ahead of c0 up to c1
    const uint32_t ahead = DIR > 0 ? ~((2u << c0) - 1u) & ((2u << c1) - 1u)
                                   : ((1u << c0) - 1u) & ~((1u << c1) - 1u);
    const uint32_t hit = blk & ahead;
    if (hit) {
      const int c = (DIR > 0 ? __builtin_ctz(hit) : 31 - __builtin_clz(hit)) - PAD;
      lim = DIR > 0 ? min(lim, c * S - off - 1) : max(lim, c * S + S - 1 - off + 1);
    }
    // can_fall: F(c) = both probed cells of column c OPEN; F(lead0) bounds the span at once
    // (the trailing probe reaches lead0); else the first F column ahead, up to lead1, does
    // when the trailing probe reaches it (the loop below: an F column right after an F lead0
    // would bound it later than lead0 already has)
    const int d = HALFW - 2;  // 10
    const int l0 = m.colx(P + DIR * d) + PAD, l1 = m.colx(lim + DIR * d) + PAD;
    const uint32_t F = m.mk_rowopen(dc, rf1) & m.mk_rowopen(dc, rf2);
    int cf = -1000;
    if ((F >> l0) & 1u) {
      cf = l0;
    } else {
      const uint32_t fa = F & (DIR > 0 ? ~((2u << l0) - 1u) & ((2u << l1) - 1u)
                                       : ((1u << l0) - 1u) & ~((1u << l1) - 1u));
      if (fa) cf = DIR > 0 ? __builtin_ctz(fa) : 31 - __builtin_clz(fa);
    }
    if (cf != -1000) {
      const int c = cf - PAD;
      const int p_both = DIR > 0 ? c * S + d : c * S + S - 1 - d;
      lim = DIR > 0 ? min(lim, p_both - 1) : max(lim, p_both + 1);
    }
    return lim;
  }
  // can_go_side(p) reads column colx(p + 16*dir): the span ends before the first column ahead
  // whose two cells hold a WALL or a closed door
  {
    const int off = DIR * (HALFW + INCR);
    const int c0 = m.colx(P + off), c1 = m.colx(lim + off);
    for (int c = c0 + DIR; DIR > 0 ? c <= c1 : c >= c1; c += DIR) {
      const uint32_t ta = m.cellb(c, rs1), tb = m.cellb(c, rs2);
      if (Map::is_wall(ta | tb) | Map::is_door(ta, dc) | Map::is_door(tb, dc)) {
        // first p with colx(p + off) == c
        lim = DIR > 0 ? min(lim, c * S - off - 1) : max(lim, c * S + S - 1 - off + 1);
        break;
      }
    }
  }
  // can_fall(p) = F(colx(p - 10)) & F(colx(p + 10)), F(c) = both probed cells OPEN: the span
  // ends before the first p ahead where the leading column and the trailing one are both F
  {
    const int d = HALFW - 2;  // 10
    const int lead0 = m.colx(P + DIR * d), lead1 = m.colx(lim + DIR * d);
    bool fprev = Map::is_open(m.cellb(lead0, rf1), dc) & Map::is_open(m.cellb(lead0, rf2), dc);
    if (fprev) {  // the trailing probe (not F now: can_fall is false) reaches lead0
      const int p_both = DIR > 0 ? lead0 * S + d : lead0 * S + S - 1 - d;
      lim = DIR > 0 ? min(lim, p_both - 1) : max(lim, p_both + 1);
    }
    for (int c = lead0 + DIR; DIR > 0 ? c <= lead1 : c >= lead1; c += DIR) {
      const bool fc = Map::is_open(m.cellb(c, rf1), dc) & Map::is_open(m.cellb(c, rf2), dc);
      if (fc) {
        // the leading probe enters c at p_in; the trailing one reaches c at p_both
        const int p_in = DIR > 0 ? c * S - d : c * S + S - 1 + d;
        const int p_both = DIR > 0 ? c * S + d : c * S + S - 1 - d;
        const int p = fprev ? p_in : p_both;
        lim = DIR > 0 ? min(lim, p - 1) : max(lim, p + 1);
        break;
      }
      fprev = fc;
    }
  }
  return lim;
}

// ==========================================================================================
// Plain ladder ticks.  While up_ladder / down_ladder (MO/:160-189) climbs with its ladder
// predicate true, can_fall false, no jump ticker and no key / gold in reach, its tick (policy
// + IM/:290-359) is exactly: one draw, py += noisy(-4) or noisy(+4), reward -1 (x, facing and
// everything else unchanged; a DOWN tick's can_fall4 finds can_fall false).  The predicates
// depend on py only through the rows their probes fall in (px is fixed), so they are constant
// between row breakpoints: ladder_plain_limit() walks those intervals in the direction of
// motion (at most LADDER_SPAN_INTERVALS of them) and returns the farthest py such that every
// start position between it and the current py makes a plain tick (INT_MIN / INT_MAX: none).
// near_cell (OB/:46-53) with px fixed bounds the span before any object's reach.
// ==========================================================================================
constexpr int LADDER_SPAN_INTERVALS = 8;
TG_HD int isqrt_below(int v) {  // largest t >= 0 with t * t < v (v >= 1)
  int t = (int)sqrtf((float)v);
  while (t * t >= v) --t;
  while ((t + 1) * (t + 1) < v) ++t;
  return t;
}
// (the predicates at px for a start position py: the cell probes, or the level bitmasks)
struct LadProbe {
  const Map& m;
  const Env& e;
  TG_HD bool lad(int dir, int y) const {
    Env p = e;
    p.py = y;
    return dir < 0 ? m.can_go_up(p) : m.can_go_down(p);
  }
  TG_HD bool fall(uint32_t dc, int y) const { return m.can_fall_at(dc, e.px, y); }
};
struct LadProbeMk {
  const Map& m;
  const LadMasks& lm;
  TG_HD bool lad(int dir, int y) const { return dir < 0 ? lm.can_go_up(m, y) : lm.can_go_down(m, y); }
  TG_HD bool fall(uint32_t, int y) const { return lm.can_fall(m, y); }
};
template <int DIR, class P = LadProbe>  // -1: up_ladder (py decreases), +1: down_ladder
TG_HD int ladder_plain_limit(const Map& m, const Env& e, const P& pr) {
  constexpr int NONE = DIR > 0 ? -0x40000000 : 0x40000000;
  if (e.f & F_JT) return NONE;
  const uint32_t dc = Map::dc_of(e.f);
  // objects: near(y) <=> (y - oy*48)^2 < R2_OBJ - dx^2; the span stops short of that range
  int bound = DIR > 0 ? 0x3FFFFFFF : -0x3FFFFFFF;
  const int ocx[2] = {e.kx, e.gx}, ocy[2] = {e.ky, e.gy};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int dx = e.px - (ocx[j] * S + S / 2);
    if (dx * dx >= R2_OBJ) continue;
    const int t = isqrt_below(R2_OBJ - dx * dx), Y = ocy[j] * S;  // near <=> |y - Y| <= t
    if ((e.py - Y < 0 ? Y - e.py : e.py - Y) <= t) return NONE;
    if (DIR < 0 && Y < e.py) bound = max(bound, Y + t + 1);
    if (DIR > 0 && Y > e.py) bound = min(bound, Y - t - 1);
  }
  if (DIR < 0) bound = max(bound, 2);  // can_go_up needs py > 1
  int y = e.py, lim = NONE;
  for (int it = 0; it < LADDER_SPAN_INTERVALS; ++it) {
    if (DIR < 0 ? y < bound : y > bound) break;
    if (!pr.lad(DIR, y) || pr.fall(dc, y)) break;
    // the interval of start positions whose probes (rows of y + o) all stay in their rows
    int end;
    if (DIR < 0) {  // can_go_up: y - 4, y, y + 44; can_fall: y, y + 50
      end = max(max(floordiv(y - INCR, S) * S + INCR, floordiv(y, S) * S),
                max(floordiv(y + S - INCR, S) * S - (S - INCR), floordiv(y + S + 2, S) * S - (S + 2)));
      end = max(end, bound);
    } else {        // can_go_down: y, y + 24, y + 51; can_fall: y, y + 50
      end = min(min(floordiv(y, S) * S + S - 1, floordiv(y + S / 2, S) * S + S - 1 - S / 2),
                min(floordiv(y + S + INCR - 1, S) * S + S - 1 - (S + INCR - 1),
                    floordiv(y + S + 2, S) * S + S - 1 - (S + 2)));
      end = min(end, bound);
    }
    lim = end;
    y = end + DIR;
  }
  return lim;
}

// ==========================================================================================
// Fused air tick: policy<K> (jump_left / jump_right MO/:297-314, 367-384; down_left /
// down_right MO/:231-244, 426-439) after its first tick, followed by the primitive tick
// (IM/:290-359), with every predicate the pair may need at the start position evaluated once
// and up front (their lookups issue as one batch): can_fall (the policy's, and the tick's
// gravity test at the same position), can_go_side both ways (the policy's back test, the
// tick's precondition), up_clear (the jump ticker's rise).  Same outcomes and draws as
// policy<K> + tick<prims_of(K)>.
// ==========================================================================================
// ac: the option loop's AirCells, rebuilt only when the player leaves its window (a jump
// changes cell column or row every ~12 ticks)
template <int K, class R>
TG_HD int air_tick(const Level& L, const uint32_t* trig, const Map& m, Env& e, Opt& o, R& rng,
                   AirCells& ac) {
  constexpr int DIR = (K == O_JUMP_LEFT || K == O_DOWN_LEFT) ? -1 : 1;
  constexpr bool JUMP = K == O_JUMP_LEFT || K == O_JUMP_RIGHT;
  const uint32_t dc = Map::dc_of(e.f);
  if (!ac.holds(dc, e.px, e.py)) {
    ac = m.air_cells(dc, e.px, e.py);
    if (!ac.holds(dc, e.px, e.py)) {  // a clamped window (a player past the border): full tick
      const int prim = policy<K>(L, m, e, o);
      return tick<prims_of(K), R>(L, trig, m, e, prim, rng);
    }
  }
  const AirProbe ap(ac, e.px, e.py);
  const bool cf0 = ap.can_fall();
  const bool fwd = ap.side(DIR);
  int mv = 0;  // the primitive: -1 LEFT, +1 RIGHT, 0 NOP
  if (close_x(e, o.tx)) {
    if (!cf0) o.done = true;
  } else {
    mv = (JUMP && !cf0 && !fwd) ? -DIR : DIR;  // MO/:311-314: back off when blocked on the floor
  }
  int xd = 0, yd = 0;
  // can_go_left / can_go_right (IM/:303-311): forward is fwd; backward only after !fwd, when
  // it is the other side's blockers
  if (mv != 0 && (mv == DIR ? fwd : ap.side(-DIR))) {
    xd = code_step(rng.code(), mv < 0);
    e.f = mv > 0 ? (e.f | F_FACING) : (e.f & ~F_FACING);
  }
  const uint32_t jt = e.f & F_JT;  // IM/:331-337, at the pre-move x
  if (jt > 0) {
    if (ap.up_clear()) yd = -INCR;
    e.f = (e.f & ~F_JT) | (jt - 1);
  } else if (cf0) {
    yd = INCR;
  }
  e.px += xd;
  if (yd > 0) yd = ap.fall(e.px, yd);  // IM/:341-348
  e.py += yd;
  pickups(L, e);
  return -1;  // STEP_REWARD (no JUMP after the first tick)
}

// A ladder option's full tick from the level bitmasks: policy<K> (MO/:168-173, 184-189) and
// tick<prims_of(K)> (IM/:290-359) fused — UP / DOWN when the ladder predicate holds (the tick
// re-tests it at the same state: the same answer), else NOP and done; then the jump ticker /
// gravity, the fall integration and the pickups, as tick<>.  Same outcomes and draws.
template <int DIR, class R>
TG_HD int ladder_tick(const Level& L, const Map& m, const LadMasks& lm, Env& e, Opt& o, R& rng) {
  int yd = 0;
  if (DIR < 0 ? lm.can_go_up(m, e.py) : lm.can_go_down(m, e.py)) yd = code_step(rng.code(), DIR < 0);
  else o.done = true;
  const uint32_t jt = e.f & F_JT;  // IM/:331-337
  if (jt > 0) {
    if (lm.up_clear(m, e.py)) yd = -INCR;
    e.f = (e.f & ~F_JT) | (jt - 1);
  } else if (lm.can_fall(m, e.py)) {
    yd = INCR;
  }
  if (yd > 0) yd = lm.fall_dist(m, e.py, yd);
  e.py += yd;
  pickups(L, e);
  return -1;  // STEP_REWARD
}

// The ladder options' while-not-done loop (OP/:28-31): a plain phase (ladder_plain_limit's
// span; one draw and py += noisy per tick, as the full tick there), then one full tick, which
// may open the next span.  One loop for both probe forms (two copies of the
// plain-tick / full-tick / TICK_CAP control flow): `pr` gives the span's predicates (cell probes
// or the level bitmasks), `full()` the full tick (policy<K> + tick<>, or ladder_tick).  (A
// batched walk here, RngCodes::walk, took k_run from 82 to 98 VGPRs: 4 instead of 5 waves per
// SIMD.)
template <int DIR, class R, class P, class Full>
TG_HD void ladder_loop(const Level& L, const Map& m, Env& e, Opt& o, R& rng, StepResult& r,
                       const P& pr, Full full) {
  int lim = DIR > 0 ? -0x40000000 : 0x40000000;  // no plain tick before the first full one
  do {
    rng.phase(0);
    bool capped = false;
    while ((DIR > 0 ? e.py <= lim : e.py >= lim) && rng.has(TICK_DRAWS)) {
      e.py += code_step(rng.code(), DIR < 0);
      r.reward += -1;
      if (DIR > 0 ? e.py > lim : e.py < lim) pickups(L, e);  // left the span: as the full tick
      if (++r.ticks >= TICK_CAP) {
        e.f |= E_TICKCAP;
        capped = true;
        lim = DIR > 0 ? -0x40000000 : 0x40000000;
      }
    }
    if (capped) break;
    rng.phase(1);
    rng.reserve(TICK_DRAWS);
    rng.phase(2);
    r.reward += full();
    if (!o.done) lim = ladder_plain_limit<DIR>(m, e, pr);
    rng.phase(3);
    if (++r.ticks >= TICK_CAP) {
      e.f |= E_TICKCAP;
      break;
    }
  } while (!o.done);
}

// the while-not-done loop of _Option.run (OP/:28-31) for option K, whose can_run held
template <int K, class R>
TG_HD void run_option_k(const Level& L, const uint32_t* trig, const Map& m, Env& e, R& rng,
                        StepResult& r) {
  r.ran = 1;
  Opt o{0, false, false};
  if constexpr (K == O_GO_LEFT || K == O_GO_RIGHT) {
    constexpr int DIR = K == O_GO_LEFT ? -1 : 1;
    int lim = DIR > 0 ? -0x40000000 : 0x40000000;  // no plain tick before the first full one
    // Two phases per round.  Plain phase: every lane inside its span takes plain ticks until
    // it leaves it (the loop body is just the plain tick).  Full phase: then no lane of the wave is in a span, and each takes one full
    // tick, which may open a new span.  Each lane's own tick sequence is the reference's; only
    // the interleaving across lanes differs, and the full tick's code runs once per round.
    do {
      // a lane leaves when its span ends; the wave when all have (a per-lane loop: a
      // ballot-driven one, with the idle lanes kept inside, made the compiler copy ~26
      // loop-carried registers per iteration and was slower)
      // (the plain phase also ends when the staged draws run low: the full tick restocks them
      // in rng.reserve, so the plain loop's body holds no refill code)
      rng.phase(0);
      if (const int t = rng.template walk<DIR>(e.px, lim, TICK_CAP - r.ticks)) {  // plain ticks
        e.f = DIR > 0 ? (e.f | F_FACING) : (e.f & ~F_FACING);
        r.reward -= t;
        r.ticks += t;
        if (DIR > 0 ? e.px > lim : e.px < lim) pickups(L, e);  // left the span: as the full tick
        if (r.ticks >= TICK_CAP) {
          e.f |= E_TICKCAP;
          break;
        }
      }
      rng.phase(1);
      rng.reserve(TICK_DRAWS);
      rng.phase(2);
      const int prim = policy<K>(L, m, e, o);
      r.reward += tick<prims_of(K), R>(L, trig, m, e, prim, rng);
      if (!o.done) lim = go_plain_limit<DIR>(m, e, o.tx);
      rng.phase(3);
      if (++r.ticks >= TICK_CAP) {
        e.f |= E_TICKCAP;
        break;
      }
    } while (!o.done);
    return;
  }
  if constexpr (K == O_UP_LADDER || K == O_DOWN_LADDER) {
    constexpr int DIR = K == O_UP_LADDER ? -1 : 1;
    if (m.mk) {  // the level bitmasks: full ticks and span limits test bits, no cell probes
      const LadMasks lm(m, Map::dc_of(e.f), e.px);
      ladder_loop<DIR>(L, m, e, o, rng, r, LadProbeMk{m, lm},
                       [&]() { return ladder_tick<DIR>(L, m, lm, e, o, rng); });
      return;
    }
    ladder_loop<DIR>(L, m, e, o, rng, r, LadProbe{m, e}, [&]() {
      const int prim = policy<K>(L, m, e, o);
      return tick<prims_of(K), R>(L, trig, m, e, prim, rng);
    });
    return;
  }
  if constexpr (K == O_JUMP_LEFT || K == O_JUMP_RIGHT || K == O_DOWN_LEFT || K == O_DOWN_RIGHT) {
    AirCells ac{0u, 0u, 0u, 0u, -0x40000000, 0, 0u};  // holds nothing: built on the first air tick
    do {
      rng.phase(0);
      rng.phase(1);
      rng.reserve(TICK_DRAWS);
      rng.phase(2);
      if (o.init) {
        r.reward += air_tick<K>(L, trig, m, e, o, rng, ac);
      } else {  // the first tick (the jump itself; the drop's target)
        const int prim = policy<K>(L, m, e, o);
        r.reward += tick<prims_of(K), R>(L, trig, m, e, prim, rng);
      }
      rng.phase(3);
      if (++r.ticks >= TICK_CAP) {
        e.f |= E_TICKCAP;
        break;
      }
    } while (!o.done);
    return;
  }
  do {
    rng.reserve(K == O_INTERACT ? L.interact_draws : TICK_DRAWS);
    const int prim = policy<K>(L, m, e, o);
    r.reward += tick<prims_of(K), R>(L, trig, m, e, prim, rng);
    if (++r.ticks >= TICK_CAP) {
      e.f |= E_TICKCAP;
      break;
    }
  } while (!o.done);
}
template <class R>
TG_HD void run_option(const Level& L, const uint32_t* trig, const Map& m, Env& e, int k,
                      R& rng, StepResult& r) {
  switch (k) {
    case O_GO_LEFT: run_option_k<O_GO_LEFT>(L, trig, m, e, rng, r); break;
    case O_GO_RIGHT: run_option_k<O_GO_RIGHT>(L, trig, m, e, rng, r); break;
    case O_UP_LADDER: run_option_k<O_UP_LADDER>(L, trig, m, e, rng, r); break;
    case O_DOWN_LADDER: run_option_k<O_DOWN_LADDER>(L, trig, m, e, rng, r); break;
    case O_INTERACT: run_option_k<O_INTERACT>(L, trig, m, e, rng, r); break;
    case O_DOWN_LEFT: run_option_k<O_DOWN_LEFT>(L, trig, m, e, rng, r); break;
    case O_DOWN_RIGHT: run_option_k<O_DOWN_RIGHT>(L, trig, m, e, rng, r); break;
    case O_JUMP_LEFT: run_option_k<O_JUMP_LEFT>(L, trig, m, e, rng, r); break;
    default: run_option_k<O_JUMP_RIGHT>(L, trig, m, e, rng, r); break;
  }
}
// option_list[a] (TG/:92): -1 for an out-of-range action (the reference raises IndexError)
TG_HD int option_index(int a) {
  if (a < -O_COUNT || a >= O_COUNT) return -1;
  return a < 0 ? a + O_COUNT : a;  // Python negative indexing
}
template <class R>
TG_HD StepResult env_step(const Level& L, const uint32_t* trig, const Map& m, Env& e, int a,
                          R& rng) {
  StepResult r{0, 0, 0, 0};
  const int k = option_index(a);
  if (k < 0) e.f |= E_ACTION;
  else if (can_run(L, m, e, k)) run_option(L, trig, m, e, k, rng, r);  // OP/:22-23 gate
  r.done = is_done(e);
  return r;
}

}  // namespace tg
