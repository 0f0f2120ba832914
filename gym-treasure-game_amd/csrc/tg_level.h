// tg_level.h — level text (the reference's three file formats) -> tg::Level + LDS grid codes.
// Host-only C++.  Follows get_file_description / build_map / read_objects /
// extract_interactives / player_initial_position (IM/:75-202) and door.update_map (OB/:246-253).
#pragma once
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tg_core.h"

namespace tg {

constexpr int MAX_CELLS = 48 * 48;  // LDS grid capacity incl. the border (default level: 18 x 17)

inline int level_err(std::string& err, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int level_err(std::string& err, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  err = buf;
  return -1;
}

inline const char* const kDefaultDomain =
    "////L/////////\n/          ///\n//////////L///\n/    /////L///\n/            / \n"
    "/////   //////\n/     /      /\n///L//////////\n/  L         / \n/  L      ////\n"
    "/  L     /////\n/       //////\n//////////////\n";
inline const char* const kDefaultObjects =
    "door 9 1 True\ndoor 9 4 False\ndoor 10 8 True\nhandle 1 1 True\nhandle 12 4 False\n"
    "key 1 4\nbolt 1 11 True\ngold 12 8\n";
inline const char* const kDefaultInteractions =
    "handle 0 True door 0 True\nhandle 0 False door 0 False\nhandle 0 True door 1 False\n"
    "handle 0 False door 1 True\nhandle 0 True handle 1 False\nhandle 0 False handle 1 True\n"
    "handle 1 False door 0 True\nhandle 1 True door 0 False\nhandle 1 False door 1 False\n"
    "handle 1 True door 1 True\nhandle 1 False handle 0 True\nhandle 1 True handle 0 False\n"
    "bolt 0 True door 2 True\nbolt 0 False door 2 False\n";

inline std::vector<std::string> lines_of(const char* s) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = s; *p; ++p) {
    if (*p == '\n') {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}
inline std::string strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) ++a;
  while (b > a && isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}
inline std::vector<std::string> words(const std::string& s) {
  std::vector<std::string> w;
  std::string cur;
  for (char c : s) {
    if (isspace((unsigned char)c)) {
      if (!cur.empty()) w.push_back(cur), cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) w.push_back(cur);
  return w;
}

// random() draws of a cascade, counted (the values do not matter: a cascade's path depends on
// the objects' booleans only)
struct CountingRng {
  uint32_t draws = 0;
  double uniform(double, double) { ++draws; return 0.5; }
};
// The most draws one INTERACT tick (IM/:321-329) can take on this level: handle 0's flip, then
// handle 1's, then the bolt's unlock (object order), each flip 1 draw plus its cascade's
// wiggles (or 1 wiggle when it fails, OB/:117-122), over every boolean state of the six
// interactive objects and every flip outcome.  An upper bound: it does not ask whether the
// player can be near both handles and the bolt at once.
inline uint32_t interact_draw_bound(const Level& L) {
  const uint32_t* trig = &L.trig[0][0];
  uint32_t most = 0;
  for (uint32_t s = 0; s < 64; ++s)
    for (int outcome = 0; outcome < 4; ++outcome)
      for (int bolt = 0; bolt < 2; ++bolt) {
        Env e{};
        e.f = s << F_OBJ;
        CountingRng r;
        for (int h = 0; h < 2; ++h) {
          ++r.draws;  // the flip's uniform(0, 1) <= 0.8
          if ((outcome >> h) & 1) cascade(trig, e, 3 + h, !((e.f >> (F_OBJ + 3 + h)) & 1u), r);
          else wiggle(e, h, r);
        }
        if (bolt) cascade(trig, e, 5, 0, r);
        if (r.draws > most) most = r.draws;
      }
  return most;
}

// Returns 0, or -1 with a message in `err`.
inline int parse_level(const char* dom, const char* objs, const char* inter, Level& L,
                       std::vector<uint8_t>& grid, std::string& err) {
  memset(&L, 0, sizeof L);
  std::vector<std::string> desc;
  for (auto& l : lines_of(dom)) desc.push_back(strip(l));  // get_file_description
  while (!desc.empty() && desc.back().empty()) desc.pop_back();
  if (desc.empty()) return level_err(err, "level: empty domain");
  L.W = (int)desc[0].size();
  L.H = (int)desc.size();
  const int PW = L.W + 2 * PAD, PH = L.H + 2 * PAD;
  if (PW * PH > MAX_CELLS || L.W > 120 || L.H > 120)
    return level_err(err, "level: %dx%d (+%d-cell border) exceeds the %d-cell LDS grid", L.W,
                     L.H, PAD, MAX_CELLS);
  // bordered grid of cell bits (tg_core.h B_*): the border is WALL, like the reference's
  // out-of-bounds probes (IM/:218-225)
  grid.assign((size_t)PW * PH, (uint8_t)B_WALL);
  bool found = false;
  for (int y = 0; y < L.H; ++y) {
    if ((int)desc[y].size() != L.W) return level_err(err, "level: ragged row %d", y);
    for (int x = 0; x < L.W; ++x) {
      const char c = desc[y][x];
      grid[(y + PAD) * PW + x + PAD] = c == ' ' ? B_OPEN : c == '/' ? B_WALL : c == 'L' ? B_LADDER
                                       : c == 'D' ? B_DOOR : 0;
      if (!found && c != '/') {  // player_initial_position (IM/:173-176)
        L.start_x = x;
        L.start_y = y;
        found = true;
      }
    }
  }
  if (!found) return level_err(err, "level: no non-wall cell for the start position");
  // read_objects (IM/:119-166): this kernel is specialised to the reference roster, in file
  // order door, door, door, handle, handle, key, bolt, gold
  static const char* kRoster[8] = {"door", "door", "door", "handle", "handle", "key", "bolt", "gold"};
  int k = 0;
  for (auto& l : lines_of(objs)) {
    const char* p = l.c_str();
    const char* t = !strncmp(p, "door", 4) ? "door" : !strncmp(p, "key", 3) ? "key"
                    : !strncmp(p, "bolt", 4) ? "bolt" : !strncmp(p, "gold", 4) ? "gold"
                    : !strncmp(p, "handle", 6) ? "handle" : nullptr;
    if (!t) continue;
    auto w = words(l);
    if (k >= 8 || strcmp(t, kRoster[k]) || w.size() < 3)
      return level_err(err, "level: object roster must be door x3, handle x2, key, bolt, gold");
    const int cx = atoi(w[1].c_str()), cy = atoi(w[2].c_str());
    const bool flag = w.size() > 3 && w[3] == "True";
    if (cx < 0 || cy < 0 || cx >= L.W || cy >= L.H)
      return level_err(err, "level: object %d outside the grid", k);
    if (k < 3) {
      L.door_cx[k] = (int8_t)cx;
      L.door_cy[k] = (int8_t)cy;
      grid[(cy + PAD) * PW + cx + PAD] = (uint8_t)(B_DOOROBJ << k);  // type from the door state
      if (flag) L.init_flags |= 1u << (F_OBJ + k);
    } else if (k < 5) {
      L.handle_cx[k - 3] = (int8_t)cx;
      L.handle_cy[k - 3] = (int8_t)cy;
      if (flag) L.init_flags |= 1u << (F_OBJ + k);
    } else if (k == 5) {
      L.key_cx = (int8_t)cx;
      L.key_cy = (int8_t)cy;
    } else if (k == 6) {
      L.bolt_cx = (int8_t)cx;
      L.bolt_cy = (int8_t)cy;
      if (flag) L.init_flags |= 1u << (F_OBJ + 5);
    } else {
      L.gold_cx = (int8_t)cx;
      L.gold_cy = (int8_t)cy;
    }
    ++k;
  }
  if (k != 8) return level_err(err, "level: object roster incomplete (%d of 8)", k);
  for (int a = 0; a < 3; ++a)
    for (int b = a + 1; b < 3; ++b)
      if (L.door_cx[a] == L.door_cx[b] && L.door_cy[a] == L.door_cy[b])
        return level_err(err, "level: two doors share a cell");
  // extract_interactives (IM/:75-117): per-object trigger lists in file order
  for (auto& l : lines_of(inter)) {
    auto w = words(l);
    if (w.empty()) continue;
    if (w.size() != 6) return level_err(err, "level: bad interaction line '%s'", l.c_str());
    auto id = [](const std::string& t, int idx) -> int {
      if (t == "door" && idx >= 0 && idx < 3) return idx;
      if (t == "handle" && idx >= 0 && idx < 2) return 3 + idx;
      if (t == "bolt" && idx == 0) return 5;
      return -1;
    };
    const int src = id(w[0], atoi(w[1].c_str())), dst = id(w[3], atoi(w[4].c_str()));
    if (src < 0 || dst < 0) return level_err(err, "level: bad interaction '%s'", l.c_str());
    const int pol = w[2] == "True", val = w[5] == "True";
    uint32_t& list = L.trig[src][pol];
    const uint32_t cnt = list & 0xFu;
    if (cnt >= 7) return level_err(err, "level: more than 7 triggers on one object");
    list = (list & ~0xFu) | (cnt + 1) | ((uint32_t)(dst | (val << 3)) << (4 + 4 * cnt));
  }
  // the option loops stage draws in a per-lane window and reserve a tick's worth before it
  const uint32_t d = interact_draw_bound(L);
  if (d > MAX_TICK_DRAWS)
    return level_err(err, "level: one INTERACT tick can draw %u times (trigger cascades), more "
                     "than the %u this build stages per tick", d, MAX_TICK_DRAWS);
  L.interact_draws = d > TICK_DRAWS ? d : TICK_DRAWS;
  return 0;
}

// The GoTable (tg_core.h go_lookup) of a parsed level, W * H * 32 entries, evaluated with the
// direct go_target / can_run code at a player standing in the middle of each cell: the key and
// the gold at home, or off the row (a position go_lookup never answers from the table).
inline std::vector<uint32_t> build_gotab(const Level& Lin, const std::vector<uint8_t>& grid) {
  Level L = Lin;
  L.gotab = nullptr;  // evaluate directly
  const Map m{grid.data(), L.W, L.H};
  std::vector<uint32_t> tab((size_t)L.W * L.H * 32);
  for (int yc = 0; yc < L.H; ++yc)
    for (int xc = 0; xc < L.W; ++xc)
      for (int dc = 0; dc < 8; ++dc)
        for (int kg = 0; kg < 4; ++kg) {
          Env e{};
          e.px = xc * S + S / 2;
          e.py = yc * S;
          e.f = (uint32_t)dc << F_OBJ;
          e.kx = (kg & 2) ? L.key_cx : -1;
          e.ky = (kg & 2) ? L.key_cy : -1;
          e.gx = (kg & 1) ? L.gold_cx : -1;
          e.gy = (kg & 1) ? L.gold_cy : -1;
          uint32_t v = 0;
          for (int d = 0; d < 2; ++d) {
            const int dir = d ? 1 : -1;
            int tc = -1;
            go_target(L, m, e, dir, xc, yc, tc);
            v |= (uint32_t)can_run(L, m, e, d ? O_GO_RIGHT : O_GO_LEFT) << d;
            v |= (uint32_t)((tc + 1) & 0xFF) << (8 + 8 * d);
          }
          tab[(((size_t)yc * L.W + xc) * 8 + dc) * 4 + kg] = v;
        }
  return tab;
}

// get_state's quotient table (tg_core.h Level::obs_q): pixel coordinates Q_MIN .. (W + 2) * 48
// over W * 48 and Q_MIN .. (H + 2) * 48 over H * 48 (every player and object coordinate the
// level can produce, with margin; outside it observe divides), each the IEEE double quotient
// (the host's division: correctly rounded, as the device's).  Sets L.qx_n / L.qy_n.
inline std::vector<double> build_obs_q(Level& L) {
  L.qx_n = (L.W + 2) * S - Q_MIN + 1;
  L.qy_n = (L.H + 2) * S - Q_MIN + 1;
  std::vector<double> q((size_t)(L.qx_n + L.qy_n));
  const double w = (double)(L.W * S), h = (double)(L.H * S);
  for (int i = 0; i < L.qx_n; ++i) q[(size_t)i] = (double)(Q_MIN + i) / w;
  for (int i = 0; i < L.qy_n; ++i) q[(size_t)(L.qx_n + i)] = (double)(Q_MIN + i) / h;
  return q;
}

// The level bitmasks (tg_core.h Map::mk) of a parsed level's bordered grid, or empty when a
// bordered side exceeds MK_DIM cells.
inline std::vector<uint32_t> build_masks(const Level& L, const std::vector<uint8_t>& grid) {
  const int PW = L.W + 2 * PAD, PH = L.H + 2 * PAD;
  if (PW > MK_DIM || PH > MK_DIM) return {};
  std::vector<uint32_t> mk((size_t)mk_words(L.W, L.H), 0u);
  for (int ri = 0; ri < PH; ++ri)
    for (int ci = 0; ci < PW; ++ci) {
      const uint32_t c = grid[(size_t)ri * PW + ci];
      if (Map::is_ladder(c)) mk[ci] |= 1u << ri;
      for (uint32_t dc = 0; dc < 8; ++dc) {
        if (Map::is_open(c, dc)) {
          mk[PW * (1 + dc) + ci] |= 1u << ri;
          mk[9 * PW + PH * dc + ri] |= 1u << ci;
        }
        if (Map::is_wall(c) | Map::is_door(c, dc)) mk[9 * PW + PH * (8 + dc) + ri] |= 1u << ci;
      }
    }
  return mk;
}

}  // namespace tg
