// mpcx_prime.hip -- launchers of the safe-prime kernels (Fermat base 2,
// Miller-Rabin; thread per candidate) and the device self-test.
#include "mpcx_device.hpp"

namespace mpcx {

// Device self-test of the cross-lane primitives the kernels rely on.
__global__ void k_selftest(uint32_t* out) {
  const int lane = threadIdx.x;
  out[lane] = from_next_lane(1000u + lane);
  out[64 + lane] = from_prev_lane(1000u + lane);
  out[128 + lane] = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane / 7) * 7) * 4, (int)(2000 + lane));
  const uint64_t acc = (uint64_t)(0xFFFFFFF0u + lane) * (0xFFFFFFF7u - lane) + 0xFFFFFFFFFFFFull;
  out[192 + lane] = (uint32_t)(acc >> 32);
}

}  // namespace mpcx

extern "C" {

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_fermat2(const mpcx::FermatArgs* a, uint32_t blocks,
                                                                    hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_fermat2<MPCX_C0_K, MPCX_WAVES_PER_EU_FERMAT>), dim3(blocks), dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_mr(const mpcx::MrArgs* a, uint32_t blocks,
                                                               hipStream_t st) {
  hipLaunchKernelGGL((mpcx::k_mr<MPCX_C0_K, MPCX_WAVES_PER_EU_MR>), dim3(blocks), dim3(64), 0, st, *a);
  return hipGetLastError();
}

__attribute__((visibility("hidden"))) hipError_t mpcx_launch_selftest(uint32_t* d_out, hipStream_t st) {
  hipLaunchKernelGGL(mpcx::k_selftest, dim3(1), dim3(64), 0, st, d_out);
  return hipGetLastError();
}

}  // extern "C"
