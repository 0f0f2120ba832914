// tg_render.h — per-chunk frame composition for render('rgb_array'), shared by the gfx950
// kernel (tg_render.hip k_render) and the host-only check build (tests/native), plus the
// host-side construction of the static layer at tg_render_init.
//
// Reference: TG/:98-105 render() -> _TreasureGameDrawer.draw_domain (DR/:136-163) and
// draw_object (DR/:238-269); DR/ = _treasure_game_impl/_treasure_game_drawer.py.
// Pixel rules (pygame 1.9.6 / SDL 1.2, restated independently in oracle/tg_oracle.c):
//   * transform.scale to 48x48: nearest neighbour, source index floor(d * s / 48);
//   * blit of a per-pixel-alpha sprite onto the XRGB screen: per channel
//     d + ((s - d) * a >> 8), a == 255 copies, a == 0 leaves d;
//   * the 5-px handle shaft: 5 Bresenham lines (both ends, error term from 0) offset by
//     0, +1, -1, +2, -2 along y when |dx| > |dy|, else along x;
//   * the knob: the scanlines of draw_fillellipse(x, y, 4, 4).
// PARITY UNPINNED against the reference itself: pygame is absent from this image.
#pragma once
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tg_amd.h"
#include "tg_core.h"

namespace tg {

constexpr int RS = 48;        // on-screen sprite size (xscale, yscale)
constexpr int RS2 = RS * RS;
// dynamic sprites (device table order)
enum : int { D_DOOR_CLOSED = 0, D_DOOR_OPEN, D_KEY, D_GOLD, D_BOLT_OPEN, D_BOLT_LOCKED, D_HERO,
             D_HERO_FLIP, D_HANDLE_BASE, D_COUNT };
constexpr uint32_t SHAFT_RGB = 0x2F4F4Fu;  // (47, 79, 79), DR/:263
constexpr uint32_t KNOB_RGB = 0xFF0000u;   // (255, 0, 0), DR/:264
constexpr int KNOB_R = RS / 10;            // int(xscale / 10)
constexpr int NLAYER = 9;                  // 8 objects in file order + the hero

// Everything the composition reads besides the env's state words.
struct RenderArgs {
  const uint4* bg;       // static layer, RGB bytes [Hpx][Wpx*3] as 16-B chunks
  const uint4* tiles;    // static layer + one cell-aligned sprite, per (cell, D_* sprite):
                         // [H*W][D_COUNT][48 rows][9 chunks]
  const uint32_t* spr;   // dynamic sprites [D_COUNT][48*48] ARGB
  uint32_t* err;         // device error word (TG_ERR_RENDER)
  int Wpx, Hpx, CH, H;   // pixels, 16-B chunks per row, cell rows (= bands)
  int W;                 // cell columns
  uint64_t knob;         // knob half width + 1 per scanline dy = -4..4, 4 bits each
  int8_t door_cx[3], door_cy[3], handle_cx[2], handle_cy[2], bolt_cx, bolt_cy;
};

// One dynamic item with its bounding box [x0, x1) x [y0, y1).
struct Layer {
  int x0, x1, y0, y1;
  int ox, oy, spr;  // sprite origin and table index
  // handle shaft: the base line visits (lx, ly) + t*(mx, my) + floor(t*dm/dM)*(nx, ny) for
  // t = 0..dM-1 (major / minor axis steps); the 5 lines are it shifted by k*(ux, uy),
  // k in {0, 1, -1, 2, -2}; knob centre (ex, ey).  handle == 0: a plain sprite.
  int handle, lx, ly, mx, my, nx, ny, dM, dm, magic, ux, uy, ex, ey;
  int sx0, sx1, sy0, sy1;  // the shaft + knob's own bounding box (handles)
};
constexpr int CELL_CHUNKS = RS * 3 / 16;  // 9: a cell row is 144 B, whole 16-B chunks
constexpr uint32_t HERO_ITEM = 1u << 8, HANDLE_ITEMS = (1u << 3) | (1u << 4);
constexpr uint16_t SRC_STATIC = 0xFFFFu, SRC_COMPOSE = 0xFFFEu;  // per-cell source selectors

TG_HD uint32_t blend_px(uint32_t d, uint32_t s) {
  const uint32_t a = s >> 24;
  if (a == 0u) return d;
  if (a == 255u) return s & 0xFFFFFFu;
  const int ia = (int)a;
  const int r = (int)((d >> 16) & 255), g = (int)((d >> 8) & 255), b = (int)(d & 255);
  const int sr = (int)((s >> 16) & 255), sg = (int)((s >> 8) & 255), sb = (int)(s & 255);
  return ((uint32_t)(r + (((sr - r) * ia) >> 8)) << 16) |
         ((uint32_t)(g + (((sg - g) * ia) >> 8)) << 8) | (uint32_t)(b + (((sb - b) * ia) >> 8));
}

TG_HD int imin(int a, int b) { return a < b ? a : b; }
TG_HD int imax(int a, int b) { return a > b ? a : b; }
TG_HD int iabs(int a) { return a < 0 ? -a : a; }

// Item i of the draw order for one env: 0-2 doors, 3-4 handles, 5 key, 6 bolt, 7 gold
// (domain-objects.txt order, DR/:160-161 loop), 8 the hero.  Returns TG_ERR_RENDER when a
// handle end point lands within 1e-9 of an integer (the int() truncation, libm watch) or
// the shaft leaves the screen; *live = false for a key / gold moved off-screen (obj.x < 0).
TG_HD uint32_t make_layer(const RenderArgs& A, int i, const uint4 st, const double2 ang,
                          Layer& l, bool& live) {
  uint32_t err = 0;
  l.handle = 0;
  const uint32_t f = st.y;
  int cx = 0, cy = 0;
  live = true;
  if (i < 3) {  // doors (DR/:244-248)
    cx = A.door_cx[i], cy = A.door_cy[i];
    l.spr = ((f >> (F_OBJ + i)) & 1u) ? D_DOOR_CLOSED : D_DOOR_OPEN;
  } else if (i < 5) {  // handles (DR/:257-266)
    cx = A.handle_cx[i - 3], cy = A.handle_cy[i - 3];
    l.spr = D_HANDLE_BASE;
  } else if (i == 5 || i == 7) {  // key, gold (DR/:249-252)
    const uint32_t z = st.z >> (i == 5 ? 0 : 16);
    cx = (int)(int8_t)(z & 0xFF), cy = (int)(int8_t)((z >> 8) & 0xFF);
    l.spr = i == 5 ? D_KEY : D_GOLD;
    live = cx >= 0;
  } else if (i == 6) {  // bolt (DR/:253-256)
    cx = A.bolt_cx, cy = A.bolt_cy;
    l.spr = ((f >> (F_OBJ + 5)) & 1u) ? D_BOLT_LOCKED : D_BOLT_OPEN;
  }
  if (i < 8) {
    l.ox = cx * RS, l.oy = cy * RS;
  } else {  // the hero at (playerx - xscale / 2, playery), mirrored facing left (DR/:157-161)
    l.ox = (int)(int16_t)(st.x & 0xFFFFu) - RS / 2;
    l.oy = (int)(int16_t)(st.x >> 16);
    l.spr = (f & F_FACING) ? D_HERO : D_HERO_FLIP;
  }
  l.x0 = l.ox, l.x1 = l.ox + RS, l.y0 = l.oy, l.y1 = l.oy + RS;
  if (i == 3 || i == 4) {
    const double a = i == 3 ? ang.x : ang.y;
    const double pi = 3.141592653589793;  // math.pi
    const double th = ((pi / 2.0) * a) + pi / 4.0;
    const double r = RS * 0.75;
    const double sx = l.ox + RS / 2.0, sy = (double)(l.oy + RS);
    const double ex = sx + (r * cos(th)), ey = sy - (r * sin(th));
    if (fabs(ex - rint(ex)) < 1e-9 || fabs(ey - rint(ey)) < 1e-9) err |= TG_ERR_RENDER;
    const int x1 = (int)sx, y1 = (int)sy, x2 = (int)ex, y2 = (int)ey;  // int() truncates
    const int dx = x2 - x1, dy = y2 - y1;
    const int sgx = dx < 0 ? -1 : 1, sgy = dy < 0 ? -1 : 1;
    const int adx = sgx * dx + 1, ady = sgy * dy + 1;
    const bool major_x = !(adx < ady);  // drawline swaps axes only when deltax < deltay
    l.handle = 1;
    l.lx = x1, l.ly = y1;
    l.mx = major_x ? sgx : 0, l.my = major_x ? 0 : sgy;
    l.nx = major_x ? 0 : sgx, l.ny = major_x ? sgy : 0;
    l.dM = major_x ? adx : ady;
    l.dm = major_x ? ady : adx;
    // floor(n / dM) == (n * magic) >> 20 for n * dM < 2^20 (n = t * dm <= 37 * 37 here)
    l.magic = (int)(((1u << 20) + (uint32_t)l.dM - 1u) / (uint32_t)l.dM);
    const bool off_y = iabs(dx) > iabs(dy);  // clip_and_draw_line_width's xinc / yinc
    l.ux = off_y ? 0 : 1, l.uy = off_y ? 1 : 0;
    l.ex = x2, l.ey = y2;
    l.sx0 = imin(imin(x1, x2) - 2 * l.ux, x2 - KNOB_R);
    l.sx1 = imax(imax(x1, x2) + 2 * l.ux + 1, x2 + KNOB_R + 1);
    l.sy0 = imin(imin(y1, y2) - 2 * l.uy, y2 - KNOB_R);
    l.sy1 = imax(imax(y1, y2) + 2 * l.uy + 1, y2 + KNOB_R + 1);
    l.x0 = imin(l.x0, l.sx0), l.x1 = imax(l.x1, l.sx1);
    l.y0 = imin(l.y0, l.sy0), l.y1 = imax(l.y1, l.sy1);
    if (l.x0 < 0 || l.y0 < 0 || l.x1 > A.Wpx || l.y1 > A.Hpx) err |= TG_ERR_RENDER;
  }
  return err;
}

TG_HD bool on_shaft(const Layer& l, int X, int Y) {
  bool hit = false;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int off = k == 0 ? 0 : ((k & 1) ? (k + 1) >> 1 : -((k + 1) >> 1));  // 0, 1, -1, 2, -2
    const int a = X - l.lx - off * l.ux, b = Y - l.ly - off * l.uy;
    const int t = a * l.mx + b * l.my, n = a * l.nx + b * l.ny;
    hit |= t >= 0 && t < l.dM &&
           n == (int)(((uint32_t)(t * l.dm) * (uint32_t)l.magic) >> 20);
  }
  return hit;
}

// item l drawn over pixel (X, Y) of colour c (the row test is the caller's)
TG_HD uint32_t apply_layer(const Layer& l, const RenderArgs& A, uint32_t c, int X, int Y) {
  if (X < l.x0 || X >= l.x1) return c;
  if (l.handle) {
    if (on_shaft(l, X, Y)) c = SHAFT_RGB;
    const int dx = X - l.ex, dy = Y - l.ey;
    if (dy >= -KNOB_R && dy <= KNOB_R) {
      const int hw = (int)((A.knob >> (4 * (dy + KNOB_R))) & 15u) - 1;
      if (dx >= -hw && dx <= hw) c = KNOB_RGB;
    }
  }
  const int u = X - l.ox, v = Y - l.oy;
  if ((unsigned)u < (unsigned)RS && (unsigned)v < (unsigned)RS)
    c = blend_px(c, A.spr[l.spr * RS2 + v * RS + u]);
  return c;
}

// the 24-bit RGB byte stream of one XRGB pixel, R first
TG_HD uint32_t px3(uint32_t c) { return ((c >> 16) & 0xFFu) | (c & 0xFF00u) | ((c & 0xFFu) << 16); }

TG_HD uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t o) {  // ({hi,lo} >> 8o)[31:0]
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, o);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * o));
#endif
}

// The 16 frame bytes [16q, 16q+16) of pixel row y, given the items `hit` (bit i = lay[i])
// touching them and the static layer's bytes `v` there.  The chunk starts in pixel
// p0 = 16q/3 at byte o = q % 3 and spans 6 pixels; blending is per channel, so the pixels are
// rebuilt from v's bytes alone (the 2 bytes of the end pixels outside the chunk are never
// written back).
TG_HD uint4 compose_chunk(const RenderArgs& A, const Layer* lay, uint32_t hit, int y, int q,
                          const uint4 v) {
  const int p0 = (16 * q) / 3;
  const uint32_t o = (uint32_t)(q % 3);
  // the 18-byte stream of pixels p0..p0+5 as 5 words (stream byte o + i = chunk byte i)
  uint32_t s0, s1, s2, s3, s4;
  if (o == 0u) {
    s0 = v.x, s1 = v.y, s2 = v.z, s3 = v.w, s4 = 0u;
  } else {
    const uint32_t sh = 4u - o;
    s0 = align_bytes(v.x, 0u, sh), s1 = align_bytes(v.y, v.x, sh), s2 = align_bytes(v.z, v.y, sh);
    s3 = align_bytes(v.w, v.z, sh), s4 = align_bytes(0u, v.w, sh);
  }
  auto rgb = [](uint32_t r, uint32_t g, uint32_t b) { return ((r & 255u) << 16) | ((g & 255u) << 8) | (b & 255u); };
  uint32_t c[6];
  c[0] = rgb(s0, s0 >> 8, s0 >> 16);
  c[1] = rgb(s0 >> 24, s1, s1 >> 8);
  c[2] = rgb(s1 >> 16, s1 >> 24, s2);
  c[3] = rgb(s2 >> 8, s2 >> 16, s2 >> 24);
  c[4] = rgb(s3, s3 >> 8, s3 >> 16);
  c[5] = rgb(s3 >> 24, s4, s4 >> 8);
  for (uint32_t m = hit; m; m &= m - 1) {
    const Layer& l = lay[__builtin_ctz(m)];
#pragma unroll
    for (int j = 0; j < 6; ++j) c[j] = apply_layer(l, A, c[j], p0 + j, y);
  }
  const uint32_t a0 = px3(c[0]), a1 = px3(c[1]), a2 = px3(c[2]), a3 = px3(c[3]), a4 = px3(c[4]),
                 a5 = px3(c[5]);
  const uint32_t w0 = a0 | (a1 << 24), w1 = (a1 >> 8) | (a2 << 16), w2 = (a2 >> 16) | (a3 << 8),
                 w3 = a4 | (a5 << 24), w4 = a5 >> 8;
  uint4 out;
  out.x = align_bytes(w1, w0, o);
  out.y = align_bytes(w2, w1, o);
  out.z = align_bytes(w3, w2, o);
  out.w = align_bytes(w4, w3, o);
  return out;
}

// bit i set: lay[i] (live) covers row y and overlaps the chunk's pixels p0 .. p0+5
TG_HD uint32_t row_items(const Layer* lay, uint32_t live, int y) {
  uint32_t rm = 0;
  for (uint32_t m = live; m; m &= m - 1) {
    const int i = __builtin_ctz(m);
    if (y >= lay[i].y0 && y < lay[i].y1) rm |= 1u << i;
  }
  return rm;
}
TG_HD uint32_t chunk_items(const Layer* lay, uint32_t row, int q) {
  const int p0 = (16 * q) / 3;
  uint32_t hit = 0;
  for (uint32_t m = row; m; m &= m - 1) {
    const int i = __builtin_ctz(m);
    if (p0 < lay[i].x1 && p0 + 5 >= lay[i].x0) hit |= 1u << i;
  }
  return hit;
}

// Source of each cell of band `band` for one env: SRC_STATIC, the tile of the one
// cell-aligned item there (doors, handle bases, key, bolt, gold all sit on whole cells), or
// SRC_COMPOSE where two share a cell.  sel has W entries.
TG_HD void cell_sources(const Layer* lay, uint32_t live, int band, int W, uint16_t* sel) {
  for (int c = 0; c < W; ++c) sel[c] = SRC_STATIC;
  for (uint32_t m = live & 0xFFu; m; m &= m - 1) {
    const Layer& l = lay[__builtin_ctz(m)];
    if (l.oy != band * RS) continue;
    const int c = l.ox / RS;
    sel[c] = sel[c] == SRC_STATIC ? (uint16_t)l.spr : SRC_COMPOSE;
  }
}

// The 16 frame bytes [16q, 16q+16) of row y (row r of band `band`) for one env: `rm` = its
// items on the row, `sel` its cell sources, `v` the static chunk.  Chunks a handle's shaft or
// knob touches (or a two-item cell) are composed from the static layer with every item in
// draw order; elsewhere the cell's tile (static + its item) is the base and only the hero,
// drawn last, is composited over it.
TG_HD uint4 render_chunk(const RenderArgs& A, const Layer* lay, uint32_t rm, const uint16_t* sel,
                         int band, int r, int q, const uint4 v) {
  const uint32_t hit = rm ? chunk_items(lay, rm, q) : 0u;
  if (!hit) return v;
  const int y = band * RS + r, cc = q / CELL_CHUNKS;
  const uint16_t s = sel[cc];
  bool full = s == SRC_COMPOSE;
  const int p0 = (16 * q) / 3;
  for (uint32_t m = hit & HANDLE_ITEMS; m; m &= m - 1) {
    const Layer& l = lay[__builtin_ctz(m)];
    full |= y >= l.sy0 && y < l.sy1 && p0 < l.sx1 && p0 + 5 >= l.sx0;
  }
  if (full) return compose_chunk(A, lay, hit, y, q, v);
  const uint4 src = s == SRC_STATIC
                        ? v
                        : A.tiles[((size_t)(band * A.W + cc) * D_COUNT + s) * (RS * CELL_CHUNKS) +
                                  (size_t)r * CELL_CHUNKS + (q - cc * CELL_CHUNKS)];
  return (hit & HERO_ITEM) ? compose_chunk(A, lay, HERO_ITEM, y, q, src) : src;
}

// ---- host: the static layer (tg_render_init) ---------------------------------------------
// CPython Random(seed).choice (DR/:83-86): seq[_randbelow(n)], getrandbits(n.bit_length())
// until < n, over MT19937 seeded by init_by_array([seed]).
struct PyChoice {
  uint32_t mt[MT_N];
  int idx = MT_N;
  explicit PyChoice(uint32_t seed) {
    mt[0] = 19650218u;
    for (int i = 1; i < MT_N; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int i = 1;
    for (int k = MT_N; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + seed;
      if (++i >= MT_N) mt[0] = mt[MT_N - 1], i = 1;
    }
    for (int k = MT_N - 1; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      if (++i >= MT_N) mt[0] = mt[MT_N - 1], i = 1;
    }
    mt[0] = 0x80000000u;
  }
  uint32_t next() {
    if (idx >= MT_N) {  // the in-place twist: words k + 397 >= 624 and mt[0] are already new
      for (int k = 0; k < MT_N; ++k)
        mt[k] = mt_twist(mt[k], mt[(k + 1) % MT_N], mt[(k + MT_M) % MT_N]);
      idx = 0;
    }
    return mt_temper(mt[idx++]);
  }
  int choice(int n) {
    int k = 0;
    while ((1 << k) <= n) ++k;
    int v;
    do v = (int)(next() >> (32 - k));
    while (v >= n);
    return v;
  }
};

// draw_fillellipse(x, y, r, r) scanlines (pygame draw.c, rx <= ry branch): half width per
// dy in [-r, r], -1 where nothing is drawn, packed as RenderArgs::knob
inline uint64_t knob_table(int r) {
  int hw[2 * KNOB_R + 1];
  for (int d = 0; d <= 2 * r; ++d) hw[d] = -1;
  auto row = [&](int dy, int half) {
    if (half > hw[dy + r]) hw[dy + r] = half;
  };
  int ix = 0, iy = r * 64, h, i, oh = 0xFFFF, oi = 0xFFFF;
  do {
    h = (ix + 32) >> 6;
    i = (iy + 32) >> 6;
    if (oi != i && oh != i) {  // j = h * rx / ry = h
      row(i, h);
      row(-i, h);
      oi = i;
    }
    if (oh != h && oi != h && i != h) {  // k = i
      row(h, i);
      row(-h, i);
      oh = h;
    }
    ix = ix + iy / r;
    iy = iy - ix / r;
  } while (i > h);
  uint64_t t = 0;
  for (int d = 0; d <= 2 * r; ++d) t |= (uint64_t)(hw[d] + 1) << (4 * d);
  return t;
}

// Sprites (TG_SPR_COUNT RGBA8 images of sw x sh) -> 48x48 ARGB (convert_alpha + scale).
inline std::vector<uint32_t> scale_sprites(const uint8_t* sprites, int sw, int sh) {
  std::vector<uint32_t> sc((size_t)TG_SPR_COUNT * RS2);
  for (int k = 0; k < TG_SPR_COUNT; ++k)
    for (int v = 0; v < RS; ++v)
      for (int u = 0; u < RS; ++u) {
        const uint8_t* p =
            sprites + (((size_t)k * sh + (size_t)(v * sh / RS)) * sw + (size_t)(u * sw / RS)) * 4;
        sc[(size_t)k * RS2 + v * RS + u] =
            ((uint32_t)p[3] << 24) | ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2];
      }
  return sc;
}

// draw_domain's cell loop (DR/:140-153) on a black XRGB screen of W x H cells.
inline std::vector<uint32_t> static_layer(const std::vector<std::string>& desc, int W, int H,
                                          const std::vector<uint32_t>& sc) {
  const int Wpx = W * RS;
  std::vector<uint32_t> bg((size_t)Wpx * H * RS, 0u);
  PyChoice rg(12);  // random_generator.seed(self.seed), self.seed = 12 (DR/:50, 137)
  auto cell = [&](int k, int i, int j) {
    const uint32_t* s = &sc[(size_t)k * RS2];
    for (int v = 0; v < RS; ++v)
      for (int u = 0; u < RS; ++u) {
        uint32_t& d = bg[(size_t)(i * RS + v) * Wpx + j * RS + u];
        d = blend_px(d, s[v * RS + u]);
      }
  };
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      const char c = desc[i][j];
      if (c == '/')
        cell((i > 0 && desc[i - 1][j] != '/' ? TG_SPR_FLOOR : TG_SPR_WALL) + rg.choice(5), i, j);
      else if (c == 'L')
        cell(TG_SPR_LADDER, i, j);
      else if (c == ' ')
        cell(TG_SPR_BACKGROUND + rg.choice(5), i, j);
    }
  return bg;
}

// The dynamic sprite table: [D_COUNT][48*48], the hero also mirrored (transform.flip).
inline std::vector<uint32_t> dynamic_sprites(const std::vector<uint32_t>& sc) {
  std::vector<uint32_t> dyn((size_t)D_COUNT * RS2);
  const int src_of[D_COUNT] = {TG_SPR_DOOR_CLOSED, TG_SPR_DOOR_OPEN, TG_SPR_KEY,  TG_SPR_GOLD,
                               TG_SPR_BOLT_OPEN,   TG_SPR_BOLT_LOCKED, TG_SPR_HERO, TG_SPR_HERO,
                               TG_SPR_HANDLE_BASE};
  for (int d = 0; d < D_COUNT; ++d)
    for (int v = 0; v < RS; ++v)
      for (int u = 0; u < RS; ++u)
        dyn[(size_t)d * RS2 + v * RS + u] =
            sc[(size_t)src_of[d] * RS2 + v * RS + (d == D_HERO_FLIP ? RS - 1 - u : u)];
  return dyn;
}

// Tiles: every cell of the static layer with each cell-aligned sprite blended over it
// ([W*H][D_COUNT][48][48] XRGB; the hero slots are unused), as RGB bytes by rgb_bytes().
inline std::vector<uint32_t> cell_tiles(const std::vector<uint32_t>& bg, int W, int H,
                                        const std::vector<uint32_t>& dyn) {
  const int Wpx = W * RS;
  std::vector<uint32_t> t((size_t)W * H * D_COUNT * RS2);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j)
      for (int d = 0; d < D_COUNT; ++d) {
        uint32_t* o = &t[((size_t)(i * W + j) * D_COUNT + d) * RS2];
        const bool hero = d == D_HERO || d == D_HERO_FLIP;
        for (int v = 0; v < RS; ++v)
          for (int u = 0; u < RS; ++u) {
            const uint32_t b = bg[(size_t)(i * RS + v) * Wpx + j * RS + u];
            o[v * RS + u] = hero ? b : blend_px(b, dyn[(size_t)d * RS2 + v * RS + u]);
          }
      }
  return t;
}

inline std::vector<uint8_t> rgb_bytes(const std::vector<uint32_t>& px) {
  std::vector<uint8_t> rgb(px.size() * 3);
  for (size_t p = 0; p < px.size(); ++p) {
    rgb[3 * p] = (uint8_t)(px[p] >> 16);
    rgb[3 * p + 1] = (uint8_t)(px[p] >> 8);
    rgb[3 * p + 2] = (uint8_t)px[p];
  }
  return rgb;
}

}  // namespace tg
