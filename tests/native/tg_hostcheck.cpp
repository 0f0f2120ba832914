// tg_hostcheck.cpp — TEST INFRASTRUCTURE ONLY.
//
// Host-only build of the product's per-env core (gym-treasure-game_amd/csrc/tg_core.h), so
// the exact code the gfx950 kernel runs per lane can be checked against the oracle on the
// build machine, which has no GPU.  It replays k_step's per-lane sequence (env_step, observe,
// optional auto-reset) one env at a time.  The product library never contains or calls this.
// Built by tests/native/Makefile with hipcc --offload-host-only.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../gym-treasure-game_amd/csrc/tg_core.h"
#include "../../gym-treasure-game_amd/csrc/tg_level.h"
#include "../../gym-treasure-game_amd/csrc/tg_render.h"

using namespace tg;

namespace {
uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
uint64_t rec_hash(uint64_t h, const double o[9], int32_t r, int v, int d) {
  for (int i = 0; i < 9; ++i) {
    uint64_t b;
    memcpy(&b, &o[i], 8);
    h = sm64(h ^ b);
  }
  return sm64(h ^ ((uint64_t)(uint32_t)r | ((uint64_t)v << 32) | ((uint64_t)d << 40)));
}
}  // namespace

extern "C" {

// go_left / go_right answered from the GoTable as on the device (1, default) or directly (0)
static int g_gotab = 1;
void hc_set_gotab(int on) { g_gotab = on; }
// the level bitmasks (tg_core.h Map::mk) as on the device's option loops (1, default) or not (0)
static int g_masks = 1;
void hc_set_masks(int on) { g_masks = on; }
static std::vector<uint32_t> g_mk;  // the last loaded level's masks
static std::vector<double> g_q;     // and quotient table

static bool load_level(const char* dom, const char* objs, const char* inter, Level& L,
                       std::vector<uint8_t>& grid, std::vector<uint32_t>& tab) {
  std::string err;
  if (!dom) {
    dom = kDefaultDomain;
    objs = kDefaultObjects;
    inter = kDefaultInteractions;
  }
  if (parse_level(dom, objs, inter, L, grid, err) != 0) return false;
  if (g_gotab) {
    tab = build_gotab(L, grid);
    L.gotab = tab.data();
  }
  g_mk = g_masks ? build_masks(L, grid) : std::vector<uint32_t>();
  L.masks = g_mk.empty() ? nullptr : g_mk.data();
  g_q = build_obs_q(L);  // observe's quotient table, as on the device
  L.obs_q = g_q.data();
  return true;
}

// Level texts as tg_create takes them (NULL = built-in default).
// obs/final_obs [n][steps+1][9], reward/valid/done [n][steps+1], hash/draws/ticks [n]
int hc_run(const char* dom, const char* objs, const char* inter, uint64_t seed_base, int64_t g0,
           int64_t n, int steps, uint64_t a0, int policy, int autoreset, double* obs,
           int32_t* reward, uint8_t* valid, uint8_t* done, double* final_obs, uint64_t* hash,
           int64_t* draws, int64_t* ticks) {
  Level Lv;
  std::vector<uint8_t> grid;
  std::vector<uint32_t> tab;
  if (!load_level(dom, objs, inter, Lv, grid, tab)) return -1;
  const Level* L = &Lv;
  uint32_t gen[MT_N];
  gen[0] = 19650218u;
  for (int i = 1; i < MT_N; ++i) gen[i] = 1812433253u * (gen[i - 1] ^ (gen[i - 1] >> 30)) + (uint32_t)i;
  const Map m{grid.data(), L->W, L->H, L->masks};
  const uint32_t* trig = &L->trig[0][0];
  const int64_t T1 = (int64_t)steps + 1;
  std::vector<uint32_t> mt(MT_WORDS);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t g = (uint64_t)(g0 + i);
    init_mt(mt.data(), gen, seed_base + g);  // k_create + k_gen_twist
    Env e{};
    int64_t ndraws = 0;
    {  // construct + reset, each a separate launch on the device (k_reset)
      Rng rng(mt.data(), 0u);
      reset_env(*L, e, rng);
      e.mti = refill_after(mt.data(), rng.finish());  // k_reset refills at once
      Rng rng2(mt.data(), e.mti);
      reset_env(*L, e, rng2);
      e.mti = refill_after(mt.data(), rng2.finish());
      ndraws += rng.draws + rng2.draws;
    }
    double o[9], fo[9];
    observe(*L, e, o);
    uint64_t h = rec_hash(g, o, 0, 0, 0);
    int64_t nt = 0;
    if (obs) memcpy(&obs[i * T1 * 9], o, sizeof o);
    if (final_obs) memcpy(&final_obs[i * T1 * 9], o, sizeof o);
    if (reward) reward[i * T1] = 0;
    if (valid) valid[i * T1] = 0;
    if (done) done[i * T1] = 0;
    for (int t = 0; t < steps; ++t) {
      const uint64_t hh = sm64(sm64(a0 ^ sm64(g)) ^ (uint64_t)t);
      int a = (int)(hh % 9ull);
      if (policy == 1) {
        const uint32_t mk = available_mask(*L, m, e);
        const int c = __builtin_popcount(mk);
        if (c) {
          uint32_t k = (uint32_t)(hh % (uint64_t)c), mm = mk;
          while (k--) mm &= mm - 1u;
          a = __builtin_ctz(mm);
        }
      }
      e.mti = refill_after(mt.data(), e.mti);  // the classify pass: last step's stale half
      Rng rng(mt.data(), e.mti);  // per step, as each launch
      const StepResult r = env_step(*L, trig, m, e, a, rng);
      nt += r.ticks;
      observe(*L, e, fo);
      memcpy(o, fo, sizeof o);
      if (autoreset && r.done) {
        reset_env(*L, e, rng);
        observe(*L, e, o);
      }
      e.mti = rng.finish();  // may carry MT_STALE into the next step
      ndraws += rng.draws;
      h = rec_hash(h, fo, r.reward, r.ran, r.done);
      const int64_t j = i * T1 + t + 1;
      if (obs) memcpy(&obs[j * 9], o, sizeof o);
      if (final_obs) memcpy(&final_obs[j * 9], fo, sizeof fo);
      if (reward) reward[j] = r.reward;
      if (valid) valid[j] = (uint8_t)r.ran;
      if (done) done[j] = (uint8_t)r.done;
    }
    if (hash) hash[i] = h;
    if (draws) draws[i] = ndraws;  // includes the 8 construct + reset draws
    if (ticks) ticks[i] = nt;
  }
  return 0;
}

// random.seed(seed); then launches[j] calls of random() per "launch", the generation buffer
// handled as the kernels do: a stale half is refilled before launch j when j % defer == 0
// (the classify pass), otherwise the launch starts with it stale and must regenerate it
// itself if it gets there.  out = every value, in order.
int hc_rng_stream(uint64_t seed, const int32_t* launches, int nl, int defer, double* out) {
  uint32_t gen[MT_N];
  gen[0] = 19650218u;
  for (int i = 1; i < MT_N; ++i) gen[i] = 1812433253u * (gen[i - 1] ^ (gen[i - 1] >> 30)) + (uint32_t)i;
  std::vector<uint32_t> mt(MT_WORDS);
  init_mt(mt.data(), gen, seed);
  uint32_t state = 0;
  int64_t k = 0;
  for (int j = 0; j < nl; ++j) {
    if (defer > 0 && j % defer == 0) state = refill_after(mt.data(), state);
    Rng rng(mt.data(), state);
    for (int d = 0; d < launches[j]; ++d) out[k++] = rng.random();
    state = rng.finish();
  }
  return 0;
}

// code_of_top27 against draw_code at both ends of every top-27-bit interval it decides (the
// outcomes are monotone in r, so the ends decide the interval); returns the mismatches and the
// number of intervals left to the exact path
int64_t hc_check_code_top27(int64_t* slow) {
  int64_t bad = 0, ns = 0;
  for (uint32_t a = 0; a < (1u << 27); ++a) {
    const uint32_t c = tg::code_of_top27(a);
    if (c == tg::CODE_SLOW) {
      ++ns;
      continue;
    }
    const double lo = (a * 67108864.0) * (1.0 / 9007199254740992.0);
    const double hi = (a * 67108864.0 + 67108863.0) * (1.0 / 9007199254740992.0);
    bad += (tg::draw_code(lo) != c) + (tg::draw_code(hi) != c);
  }
  *slow = ns;
  return bad;
}

// mt_pair (branch-free, RngCodes on the device), mt_pair_branchy (tg::Rng) and the plain
// twist against each other and against full generations: a seeded ring, every even position
// of all 16 generations.  Returns the mismatches.
int64_t hc_check_mt_pair(uint64_t seed) {
  uint32_t gen[MT_N];
  gen[0] = 19650218u;
  for (int i = 1; i < MT_N; ++i) gen[i] = 1812433253u * (gen[i - 1] ^ (gen[i - 1] >> 30)) + (uint32_t)i;
  std::vector<uint32_t> mt(MT_STORE), full((size_t)(2 * MT_HALF_GENS + 1) * MT_N);
  init_mt(mt.data(), gen, seed);
  seed_mt(full.data(), gen, seed);  // generation -1, then 16 twists: the ring's generations
  for (int g = 0; g < 2 * MT_HALF_GENS; ++g) twist_gen(&full[(size_t)g * MT_N], &full[(size_t)(g + 1) * MT_N]);
  int64_t bad = 0;
  for (uint32_t p = 0; p < (uint32_t)MT_WORDS; p += 2) {
    uint32_t a0, a1, b0, b1;
    mt_pair(mt.data(), p, a0, a1);
    mt_pair_branchy(mt.data(), p, b0, b1);
    const WordPair c = mt_pair_ool(mt.data(), p);
    const uint32_t f0 = full[MT_N + p], f1 = full[MT_N + p + 1];
    bad += (a0 != f0) + (a1 != f1) + (b0 != f0) + (b1 != f1) + (c.w0 != f0) + (c.w1 != f1);
  }
  return bad;
}

// top27_code / top27_slow (the wave twist's code pass, tg_twist.h) against code_of_top27 for
// every a: equal wherever top27_slow is false, and top27_slow covers every CODE_SLOW interval;
// returns the mismatches and the number of slow intervals
int64_t hc_check_code_lean(int64_t* slow) {
  int64_t bad = 0, ns = 0;
  for (uint32_t a = 0; a < (1u << 27); ++a) {
    const uint32_t c = tg::code_of_top27(a);
    if (tg::top27_slow(a)) {
      ++ns;
      continue;
    }
    bad += (c == tg::CODE_SLOW) + (tg::top27_code(a) != c);
  }
  *slow = ns;
  return bad;
}

// the six collision predicates at a pixel position / door state (same bit order as the
// oracle's tgo_predicates)
unsigned hc_predicates(int px, int py, unsigned door_bits) {
  static Level L;
  static std::vector<uint8_t> grid;
  static std::vector<uint32_t> tab;
  if (grid.empty() && !load_level(nullptr, nullptr, nullptr, L, grid, tab)) return ~0u;
  const Map m{grid.data(), L.W, L.H};
  Env e{};
  e.px = px;
  e.py = py;
  e.f = (door_bits & 7u) << F_OBJ;
  return (unsigned)m.up_clear(e) | (unsigned)m.can_go_up(e) << 1 | (unsigned)m.can_go_down(e) << 2 |
         (unsigned)m.can_go_side(e, -1) << 3 | (unsigned)m.can_go_side(e, +1) << 4 |
         (unsigned)m.can_fall(e) << 5;
}

void hc_predicate_table(int x0, int x1, int y0, int y1, unsigned door_bits, uint8_t* out) {
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x)
      out[(size_t)(y - y0) * (size_t)(x1 - x0) + (size_t)(x - x0)] =
          (uint8_t)hc_predicates(x, y, door_bits);
}

// render('rgb_array') of env g = seed_base + envs[i] after `steps` steps of the hc_run
// action stream, composed by tg_render.h exactly as k_render's lanes do (band by band, row by
// row, 16-B chunk by chunk), with the static layer built by tg_render_init's host code.
// frames [n][H*48][W*48][3].  Returns the OR of the TG_ERR_RENDER bits, or -1.
int hc_render_run(const char* dom, const char* objs, const char* inter, uint64_t seed_base,
                  const int64_t* envs, int64_t n, int steps, uint64_t a0, int policy,
                  int autoreset, const uint8_t* sprites, int sw, int sh, uint8_t* frames) {
  Level Lv;
  std::vector<uint8_t> grid;
  std::vector<uint32_t> tab;
  if (!load_level(dom, objs, inter, Lv, grid, tab)) return -1;
  const Level* L = &Lv;
  std::vector<std::string> desc;
  for (auto& l : lines_of(dom ? dom : kDefaultDomain)) desc.push_back(strip(l));
  while (!desc.empty() && desc.back().empty()) desc.pop_back();
  const std::vector<uint32_t> sc = scale_sprites(sprites, sw, sh);
  const std::vector<uint32_t> bg32 = static_layer(desc, L->W, L->H, sc);
  const std::vector<uint8_t> bg = rgb_bytes(bg32);
  const std::vector<uint32_t> dyn = dynamic_sprites(sc);
  const std::vector<uint8_t> tiles = rgb_bytes(cell_tiles(bg32, L->W, L->H, dyn));
  uint32_t err = 0;
  RenderArgs A;
  A.bg = reinterpret_cast<const uint4*>(bg.data());
  A.tiles = reinterpret_cast<const uint4*>(tiles.data());
  A.W = L->W;
  A.spr = dyn.data();
  A.err = &err;
  A.Wpx = L->W * RS, A.Hpx = L->H * RS, A.CH = A.Wpx * 3 / 16, A.H = L->H;
  A.knob = knob_table(KNOB_R);
  for (int k = 0; k < 3; ++k) A.door_cx[k] = L->door_cx[k], A.door_cy[k] = L->door_cy[k];
  for (int k = 0; k < 2; ++k) A.handle_cx[k] = L->handle_cx[k], A.handle_cy[k] = L->handle_cy[k];
  A.bolt_cx = L->bolt_cx, A.bolt_cy = L->bolt_cy;
  uint32_t gen[MT_N];
  gen[0] = 19650218u;
  for (int i = 1; i < MT_N; ++i) gen[i] = 1812433253u * (gen[i - 1] ^ (gen[i - 1] >> 30)) + (uint32_t)i;
  const Map m{grid.data(), L->W, L->H};
  const uint32_t* trig = &L->trig[0][0];
  std::vector<uint32_t> mt(MT_WORDS);
  const size_t fb = (size_t)A.Hpx * A.Wpx * 3;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t g = (uint64_t)envs[i];
    init_mt(mt.data(), gen, seed_base + g);
    Env e{};
    for (int r = 0; r < 2; ++r) {  // construct + reset
      Rng rng(mt.data(), e.mti);
      reset_env(*L, e, rng);
      e.mti = refill_after(mt.data(), rng.finish());
    }
    for (int t = 0; t < steps; ++t) {
      const uint64_t hh = sm64(sm64(a0 ^ sm64(g)) ^ (uint64_t)t);
      int a = (int)(hh % 9ull);
      if (policy == 1) {
        const uint32_t mk = available_mask(*L, m, e);
        const int c = __builtin_popcount(mk);
        if (c) {
          uint32_t k = (uint32_t)(hh % (uint64_t)c), mm = mk;
          while (k--) mm &= mm - 1u;
          a = __builtin_ctz(mm);
        }
      }
      e.mti = refill_after(mt.data(), e.mti);
      Rng rng(mt.data(), e.mti);
      const StepResult r = env_step(*L, trig, m, e, a, rng);
      if (autoreset && r.done) reset_env(*L, e, rng);
      e.mti = rng.finish();
    }
    uint4 st;  // k_render reads the SoA state words
    st.x = ((uint32_t)e.px & 0xFFFFu) | ((uint32_t)e.py << 16);
    st.y = e.f;
    st.z = ((uint32_t)e.kx & 0xFF) | (((uint32_t)e.ky & 0xFF) << 8) | (((uint32_t)e.gx & 0xFF) << 16) |
           ((uint32_t)e.gy << 24);
    st.w = e.mti;
    double2 an;
    an.x = e.ang0, an.y = e.ang1;
    uint4* out = reinterpret_cast<uint4*>(frames + (size_t)i * fb);
    for (int band = 0; band < A.H; ++band) {
      const int ylo = band * RS;
      Layer lay[NLAYER];
      uint32_t live_mask = 0;
      for (int k = 0; k < NLAYER; ++k) {
        bool live = false;
        err |= make_layer(A, k, st, an, lay[k], live);
        live = live && lay[k].y1 > ylo && lay[k].y0 < ylo + RS && lay[k].x1 > 0 && lay[k].x0 < A.Wpx;
        live_mask |= (uint32_t)live << k;
      }
      std::vector<uint16_t> sel((size_t)A.W);
      cell_sources(lay, live_mask, band, A.W, sel.data());
      for (int r = 0; r < RS; ++r) {
        const int y = ylo + r;
        const uint32_t rm = row_items(lay, live_mask, y);
        for (int q = 0; q < A.CH; ++q) {
          const uint4 v = A.bg[(size_t)y * A.CH + q];
          out[(size_t)y * A.CH + q] = rm ? render_chunk(A, lay, rm, sel.data(), band, r, q, v) : v;
        }
      }
    }
  }
  return (int)err;
}

}  // extern "C"
