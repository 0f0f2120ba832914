// tg_flow.hip — k_flow's own translation unit (tg_flow.h: TG_MODE_FLOW's one-launch rollout).
//
// Built with `-mllvm -disable-machine-licm` (gym_treasure_game_amd/build.py, FLOW_FLAGS): in
// tg_amd.hip's unit MachineLICM hoisted loop-invariant values out of k_flow's work loop and kept
// them live across it (123-182 VGPRs, 2-3 waves per SIMD); without the pass 121-129, 4 waves
// (DESIGN.md §9.2).  The pass stays on for every other kernel.  This unit includes tg_amd.hip
// for the device helpers k_flow shares with the per-step kernels (TG_FLOW_TU leaves out the
// host code and every other kernel, so the library holds one copy of each) and exports the
// k_flow instantiations' handles, which tg_amd.hip's launch_flow launches with hipLaunchKernel.
#define TG_FLOW_TU 1
#include "tg_amd.hip"

namespace tg {
const void* flow_kernel(bool ar, int pol) {
  if (ar) return pol ? reinterpret_cast<const void*>(k_flow<true, 1>)
                     : reinterpret_cast<const void*>(k_flow<true, 0>);
  return pol ? reinterpret_cast<const void*>(k_flow<false, 1>)
             : reinterpret_cast<const void*>(k_flow<false, 0>);
}
}  // namespace tg
