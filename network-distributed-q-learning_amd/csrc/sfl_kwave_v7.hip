// Variant 7 of k_wave_g (sfl::kVariants[7]: 4 envs per wavefront, two train slots per lane -- the bench's c3
// shape, 64 switches / 32 trains) in a translation unit of its own, so that build.py can compile it with LLVM's
// register-minimising machine scheduler (-mllvm -amdgpu-sched-strategy=iterative-minreg, build.TU_FLAGS): at the
// 128-VGPR budget of 4 waves per SIMD it spills less, c3 +6.5 % (profiles/r05p_sched_strategy_ab.txt), while
// every other shape loses with it (c2 -5.6 %, c5 -1.5 %, the partitioned step -5.7 %) and stays in sfl.hip.
#include "sfl_kwave_g.h"

namespace sflk {
static_assert(sfl::kVariants[7].G == 16 && sfl::kVariants[7].TW == 32, "variant 7 is the c3 shape");
}
SFL_KWAVE_V7(template)

#ifdef SFL_PROFILE
namespace sflk {
void kwave_v7_prof_take(unsigned long long* pr) {
  hipMemcpyFromSymbol(pr, HIP_SYMBOL(sfl::wave::g_prof), 32 * sizeof(unsigned long long));
  unsigned long long z[32] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(sfl::wave::g_prof), z, sizeof z);
}
}  // namespace sflk
#endif
