// Diagnostics kernels.
//
// plan_delay: one wave that spins on the 100 MHz wall clock for `ticks` (10 ns
// each) and then exits.  The plan's schedule-perturbation race check
// (Plan::set_perturb, utils/racecheck.py) puts these in front of randomly chosen
// launches on every stream, so that work a missing fork or join leaves unordered
// really does overlap in a different order from run to run.  The clock read is
// the only memory-side effect: no loads, no stores.
#include <algorithm>
#include <stdexcept>

#include "comm.h"
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

// cu_where: which compute unit each workgroup ran on (CU-mask checks,
// scripts/cu_mask_probe.py).  One wave per workgroup; lane 0 stores (vector store)
// the HW_ID register (cu_id bits 11:8, sh_id 12, se_id 15:13) and XCC_ID, then the
// wave spins `ticks` so the grid's workgroups are resident together and spread out.
__global__ void __launch_bounds__(64) cu_where_kernel(unsigned* out, long long ticks) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void cu_where(unsigned* out, int blocks, long long ticks, hipStream_t s) {
  if (blocks <= 0 || out == nullptr) throw std::invalid_argument("cu_where: blocks > 0, out");
  hipLaunchKernelGGL(cu_where_kernel, dim3(blocks), dim3(64), 0, s, out, ticks);
  DTR_CHECK_LAUNCH();
}

// Loopback communicator (comm.h): the diagnostics stand-in for an all-reduce,
// buf *= factor in place.  A grid-stride loop; the factor of the tests (2) is
// exact in fp32 and bf16, so any element the scale missed or saw twice differs.
template <typename T>
__global__ void __launch_bounds__(256) scale_inplace_kernel(T* p, size_t n, float f) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = (T)((float)p[i] * f);
}

void comm_scale_inplace(void* buf, size_t count, int dtype, float factor, hipStream_t s) {
  if (count == 0) return;
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, 2048);
  if (dtype == 9)
    hipLaunchKernelGGL(scale_inplace_kernel<bf16>, dim3(grid), dim3(256), 0, s,
                       static_cast<bf16*>(buf), count, factor);
  else
    hipLaunchKernelGGL(scale_inplace_kernel<float>, dim3(grid), dim3(256), 0, s,
                       static_cast<float*>(buf), count, factor);
}

}  // namespace dtr
