// k_wave_g: several envs per wavefront (sfl_wave.h run_groups), G lanes per env, SFL_GROUP_BLOCK / G envs per
// block.  Shared by the translation units that instantiate it: sfl.hip (every shape but variant 7) and
// sfl_kwave_v7.hip (variant 7, the bench's c3 shape, compiled with the register-minimising scheduler).
//
// Waves per SIMD the grouped kernel is register-budgeted for (sfl::kVariants[v].OCC): shapes with one train
// slot per lane (TW <= G) 4 -- c2 (variant 6): 918 M vs 805 M at 3 (VGPR-bound, spills a little; 5: 589 M) --,
// two slots per lane 4 with the prefetch ring (SFL_PF_RING: the LDS then allows 4 blocks per CU), 3 without it.
#pragma once
#include <hip/hip_runtime.h>

#include "sfl_engine.h"
#include "sfl_wave.h"

namespace sflk {

template <int PPL, int SPL, int TW, bool TRACE, int G, int OCC, bool TIMED = false, bool LM = false>
__global__ void __launch_bounds__(SFL_GROUP_BLOCK) __attribute__((amdgpu_waves_per_eu(OCC)))
k_wave_g(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s, const sfl::SflCtl* __restrict__ c) {
  sfl::wave::run_groups<PPL, SPL, TW, TRACE, G, TIMED, LM>(*m, *s, *c);
}

// variant 7's three launches (traced, phase-timed, plain): explicit instantiation definitions in
// sfl_kwave_v7.hip, declarations (extern template) in sfl.hip
#define SFL_KWAVE_V7_ONE(PFX, TRACE, TIMED)                                                                        \
  PFX __global__ void k_wave_g<sfl::kVariants[7].PPL, sfl::kVariants[7].SPL, sfl::kVariants[7].TW, TRACE,           \
                               sfl::kVariants[7].G, sfl::kVariants[7].OCC, TIMED>(                                 \
      const sfl::SflMap* __restrict__, const sfl::SflState* __restrict__, const sfl::SflCtl* __restrict__);
#define SFL_KWAVE_V7(PFX)              \
  namespace sflk {                     \
  SFL_KWAVE_V7_ONE(PFX, true, false)   \
  SFL_KWAVE_V7_ONE(PFX, false, true)   \
  SFL_KWAVE_V7_ONE(PFX, false, false)  \
  }

#ifdef SFL_PROFILE
// (tuning builds) variant 7's phase cycles, read and cleared -- they count into sfl_kwave_v7.hip's own g_prof
void kwave_v7_prof_take(unsigned long long* pr);
#endif

}  // namespace sflk
