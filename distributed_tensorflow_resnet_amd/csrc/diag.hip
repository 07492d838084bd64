// Diagnostics kernels.
//
// plan_delay: one wave that spins on the 100 MHz wall clock for `ticks` (10 ns
// each) and then exits.  The plan's schedule-perturbation race check
// (Plan::set_perturb, utils/racecheck.py) puts these in front of randomly chosen
// launches on every stream, so that work a missing fork or join leaves unordered
// really does overlap in a different order from run to run.  The clock read is
// the only memory-side effect: no loads, no stores.
#include "common.h"
#include "kernels.h"

namespace dtr {

__global__ void __launch_bounds__(64) plan_delay_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void plan_delay(long long ticks, hipStream_t s) {
  if (ticks <= 0) return;
  hipLaunchKernelGGL(plan_delay_kernel, dim3(1), dim3(64), 0, s, ticks);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
