// tg_render.hip — TreasureGame.render('rgb_array') for a whole batch (tg_render_init /
// tg_render / tg_frame_shape of include/tg_amd.h).
//
// Reference: TG/:98-105 render() -> _TreasureGameDrawer.draw_domain (DR/:136-163) and
// draw_object (DR/:238-269); ObservationWrapper (TG/:38-51) renders after every reset/step.
// DR/ = _treasure_game_impl/_treasure_game_drawer.py.
//
// A frame is the env's screen as RGB bytes, [H*48][W*48][3] (surfarray.array3d().swapaxes(0,1)).
// It splits into
//   * a STATIC layer, identical for every env and every step: black, then one 48x48 sprite per
//     description cell — wall or floor (a wall under a non-wall) or background, each a
//     Random(12).choice over 5 variants in row-major cell order (draw_domain reseeds the
//     generator every frame, DR/:137), ladders fixed.  Built once on the host at
//     tg_render_init and kept in HBM (a few MB, L2-resident while the kernel streams);
//   * a DYNAMIC layer of <= 9 items drawn over it in the reference's order: the 8 objects in
//     file order (3 doors open/closed, 2 handles = 5-px shaft + r=4 knob + base sprite, key
//     and gold unless moved off-screen, bolt open/locked), then the hero (mirrored when facing
//     left).  They cover ~6 % of the pixels.
// k_render: one workgroup per (group of 4 envs, band of 48 pixel rows), one wave per row,
// one lane per 16-B chunk of the row's RGB bytes (coalesced, every byte of every frame written
// exactly once).  The lane loads its static chunk once and stores it into the 4 frames,
// except where a dynamic item touches the chunk: there it composites the chunk's 6 pixels in
// draw order and repacks.  The kernel is HBM-write bound: 1,257,984 B per frame of the
// default level; the static layer is read once per 4 frames (from L2 / Infinity Cache).
//
// The per-chunk composition and the static-layer construction live in tg_render.h (shared
// with the host-only check build); the pixel rules are listed there.  PARITY UNPINNED against
// the reference (pygame is absent here); pinned against the oracle's restatement.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "tg_batch.h"
#include "tg_level.h"
#include "tg_render.h"

namespace tg {

constexpr int RBLOCK = 256;  // 4 waves (1,024 threads lost 1.5-9 ms)

struct RenderState {
  int Wpx = 0, Hpx = 0, CH = 0;  // pixels, 16-B chunks per row
  uint4* bg = nullptr;           // static layer, RGB bytes [Hpx][Wpx*3]
  uint4* tiles = nullptr;        // static layer + each cell-aligned sprite, per cell
  uint32_t* spr = nullptr;       // [D_COUNT][48*48] ARGB
  uint64_t knob = 0;             // knob half widths + 1, 4 bits per row dy = -4..4
};

void render_free(RenderState* rs) {
  if (!rs) return;
  void* bufs[] = {rs->bg, rs->tiles, rs->spr};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete rs;
}

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// frame stores are non-temporal: streamed once, never re-read here (plain, sc1, sc0 sc1 and
// nt sc1 stores measured equal or up to 0.8 ms slower)
__device__ __forceinline__ void store16(uint4* p, const uint4 x) {
  u32x4 v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

constexpr int RG = 4;  // envs per workgroup: each static-layer chunk is loaded once per RG frames
constexpr int MAX_W = 128;  // cell columns (levels are at most 120 wide, tg_level.h)

// block = (group of RG envs, band of 48 rows): lane l of wave w renders chunks 64w + l,
// 64(w + 4) + l, ... of the band, for each env of the group in turn: the static chunk is
// loaded once and stored RG times (composited where an item covers it).
__global__ __launch_bounds__(RBLOCK) void k_render(RenderArgs A, const uint4* __restrict__ st4,
                                                   const double2* __restrict__ angs,
                                                   int64_t first, int64_t count,
                                                   uint4* __restrict__ out) {
  __shared__ Layer lay[RG][NLAYER];
  __shared__ uint32_t live[RG];
  __shared__ uint16_t rows[RG][RS];  // items covering each row of the band, per env
  __shared__ uint16_t sel[RG][MAX_W];  // each cell's source, per env
  const int64_t grp = blockIdx.x / A.H;
  const int band = (int)(blockIdx.x - grp * A.H);
  const int ylo = band * RS;
  const int64_t e0 = grp * RG;
  const int ne = (int)(count - e0 < RG ? count - e0 : RG);
  if (threadIdx.x < RG) live[threadIdx.x] = 0u;
  __syncthreads();
  for (int t = threadIdx.x; t < RG * NLAYER; t += RBLOCK) {
    const int k = t / NLAYER, i = t - k * NLAYER;
    if (k < ne) {
      Layer l;
      bool on = false;
      const int64_t g = first + e0 + k;
      const uint32_t err = make_layer(A, i, st4[g], angs[g], l, on);
      if (err) atomicOr(A.err, err);
      if (on && l.y1 > ylo && l.y0 < ylo + RS && l.x1 > 0 && l.x0 < A.Wpx) {
        lay[k][i] = l;
        atomicOr(&live[k], 1u << i);
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < RG * RS; t += RBLOCK) {
    const int k = t / RS, r = t - k * RS;
    rows[k][r] = (uint16_t)(k < ne ? row_items(lay[k], live[k], ylo + r) : 0u);
  }
  if (threadIdx.x < RG && (int)threadIdx.x < ne)
    cell_sources(lay[threadIdx.x], live[threadIdx.x], band, A.W, sel[threadIdx.x]);
  __syncthreads();
  // The band is one contiguous, 128-B aligned run of 48 * CH chunks in every frame (a frame
  // row, 2,016 B, is not a whole number of 128-B lines): waves take 1-KB segments of it, so
  // every store instruction writes 8 whole lines; a segment may straddle two pixel rows.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t frame_chunks = (int64_t)A.Hpx * A.CH;
  const int band_chunks = RS * A.CH;
  uint4* const base = out + e0 * frame_chunks + (int64_t)ylo * A.CH;
  const uint4* const bgb = A.bg + (int64_t)ylo * A.CH;
  for (int c0 = wave * 64; c0 < band_chunks; c0 += RBLOCK) {
    const int c = c0 + lane;
    if (c >= band_chunks) break;
    const int rs = c0 / A.CH;                            // wave-uniform first row of the segment
    const int r = c - rs * A.CH >= A.CH ? rs + 1 : rs;  // this lane's row
    const int q = c - r * A.CH;
    const uint4 v = bgb[c];
    uint4* dst = base + c;
    for (int k = 0; k < ne; ++k, dst += frame_chunks) {
      const uint32_t rm = rows[k][r];
      store16(dst, rm ? render_chunk(A, lay[k], rm, sel[k], band, r, q, v) : v);
    }
  }
}

}  // namespace
}  // namespace tg

using namespace tg;

extern "C" {

int tg_render_init(tg_batch* h, const uint8_t* sprites, int32_t sw, int32_t sh) {
  BIND(h);
  if (!sprites || sw <= 0 || sh <= 0 || sw > 4096 || sh > 4096)
    return fail(TG_E_INVAL, "tg_render_init: bad sprite sheet");
  // description cells (get_file_description, IM/:180-202)
  std::vector<std::string> desc;
  for (auto& l : lines_of(h->domain.c_str())) desc.push_back(strip(l));
  while (!desc.empty() && desc.back().empty()) desc.pop_back();
  const int W = h->L.W, H = h->L.H, Wpx = W * RS, Hpx = H * RS;
  if ((int)desc.size() != H) return fail(TG_E_INVAL, "tg_render_init: level text mismatch");
  // handle shafts + knobs must stay on the surface: x - 5 .. x + 53, y + 8 .. y + 50 (angles
  // in [0, 1]: end point within 26 px across and 12..36 px above the pivot (x + 24, y + 48))
  for (int k = 0; k < 2; ++k) {
    const int x = h->L.handle_cx[k] * RS, y = h->L.handle_cy[k] * RS;
    if (x - 6 < 0 || x + 55 > Wpx || y + 52 > Hpx)
      return fail(TG_E_INVAL, "tg_render_init: handle %d's shaft would leave the screen", k);
  }
  const std::vector<uint32_t> sc = scale_sprites(sprites, sw, sh);
  const std::vector<uint32_t> bg32 = static_layer(desc, W, H, sc);
  const std::vector<uint8_t> rgb = rgb_bytes(bg32);
  const std::vector<uint32_t> dyn = dynamic_sprites(sc);
  const std::vector<uint8_t> tiles = rgb_bytes(cell_tiles(bg32, W, H, dyn));
  RenderState* rs = new RenderState();
  rs->Wpx = Wpx, rs->Hpx = Hpx, rs->CH = Wpx * 3 / 16;  // W * 144 bytes per row: whole chunks
  rs->knob = knob_table(KNOB_R);
  auto undo = [&](int code) {
    render_free(rs);
    return code;
  };
  if (hipMalloc((void**)&rs->bg, rgb.size()) != hipSuccess ||
      hipMalloc((void**)&rs->tiles, tiles.size()) != hipSuccess ||
      hipMalloc((void**)&rs->spr, dyn.size() * 4) != hipSuccess)
    return undo(fail(TG_E_NOMEM, "tg_render_init: device allocation failed"));
  if (hipMemcpy(rs->bg, rgb.data(), rgb.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(rs->tiles, tiles.data(), tiles.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(rs->spr, dyn.data(), dyn.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return undo(fail(TG_E_HIP, "tg_render_init: upload failed"));
  render_free(h->rs);
  h->rs = rs;
  return TG_OK;
}

int tg_frame_shape(const tg_batch* h, int32_t* height, int32_t* width) {
  if (!h) return fail(TG_E_INVAL, "null handle");
  if (height) *height = h->L.H * RS;
  if (width) *width = h->L.W * RS;
  return TG_OK;
}

int tg_render(tg_batch* h, int64_t first, int64_t count, uint8_t* rgb, void* stream) {
  BIND(h);
  if (!h->rs) return fail(TG_E_STATE, "tg_render: call tg_render_init first");
  if (first < 0 || count < 0 || first + count > h->n || (count && !rgb))
    return fail(TG_E_INVAL, "tg_render: envs [%lld, %lld) outside [0, %lld)", (long long)first,
                (long long)(first + count), (long long)h->n);
  if (((uintptr_t)rgb & 15u) != 0) return fail(TG_E_INVAL, "tg_render: rgb must be 16-B aligned");
  if (!count) return TG_OK;
  const RenderState* rs = h->rs;
  RenderArgs A;
  A.bg = rs->bg, A.tiles = rs->tiles, A.spr = rs->spr, A.err = h->err;
  A.Wpx = rs->Wpx, A.Hpx = rs->Hpx, A.CH = rs->CH, A.H = h->L.H, A.W = h->L.W;
  A.knob = rs->knob;
  for (int k = 0; k < 3; ++k) A.door_cx[k] = h->L.door_cx[k], A.door_cy[k] = h->L.door_cy[k];
  for (int k = 0; k < 2; ++k) A.handle_cx[k] = h->L.handle_cx[k], A.handle_cy[k] = h->L.handle_cy[k];
  A.bolt_cx = h->L.bolt_cx, A.bolt_cy = h->L.bolt_cy;
  const int64_t blocks = (count + RG - 1) / RG * h->L.H;
  if (blocks > 0x7FFFFFFF) return fail(TG_E_INVAL, "tg_render: too many envs in one call");
  hipLaunchKernelGGL(k_render, dim3((unsigned)blocks), dim3(RBLOCK), 0, (hipStream_t)stream, A,
                     h->S.st4, h->S.ang, first, count, reinterpret_cast<uint4*>(rgb));
  HIP_TRY(hipGetLastError());
  return TG_OK;
}

}  // extern "C"
