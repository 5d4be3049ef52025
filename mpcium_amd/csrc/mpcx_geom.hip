// mpcx_geom.hip -- one k_modexp geometry per translation unit (compiled once
// per geometry id with -DMPCX_GEOM_ID=g, in parallel, by mpcium_amd/build.py).
#include "mpcx_device.hpp"

#ifndef MPCX_GEOM_ID
#error "compile with -DMPCX_GEOM_ID=<geometry id>"
#endif

// waves per SIMD each geometry's kernel is compiled for (register budget)
#ifndef MPCX_WPE
#if MPCX_GEOM_ID == 0
#define MPCX_WPE 2
#elif MPCX_GEOM_ID == 1
#define MPCX_WPE 3
#elif MPCX_GEOM_ID == 2
#define MPCX_WPE 2
#elif MPCX_GEOM_ID == 3 || MPCX_GEOM_ID == 4
#define MPCX_WPE 8
#elif MPCX_GEOM_ID == 5
#define MPCX_WPE 2  // K = 37 per lane, as geometry 2
#else
#define MPCX_WPE 3
#endif
#endif

// the multi-batch kernel's own budget (A/B: -DMPCX_WPE_MULTI_G<id>=n): the
// 2048-bit main geometry's multi kernel fits 128 VGPRs without scratch and
// runs 4 waves per SIMD (profiles/r03/wpe4: keygen 385 vs 368 sessions/s,
// signing +2-4%, two interleaved rounds)
#if MPCX_GEOM_ID == 1
#ifndef MPCX_WPE_MULTI_G1
#define MPCX_WPE_MULTI_G1 4
#endif
#define MPCX_WPE_MULTI MPCX_WPE_MULTI_G1
#endif
#ifndef MPCX_WPE_MULTI
#define MPCX_WPE_MULTI MPCX_WPE
#endif
// the single-batch k_modexp's budget (A/B: -DMPCX_WPE_SINGLE_G1=n)
#if MPCX_GEOM_ID == 1 && defined(MPCX_WPE_SINGLE_G1)
#define MPCX_WPE_SINGLE MPCX_WPE_SINGLE_G1
#endif
#ifndef MPCX_WPE_SINGLE
#define MPCX_WPE_SINGLE MPCX_WPE
#endif

#define MPCX_CAT2(a, b) a##b
#define MPCX_CAT(a, b) MPCX_CAT2(a, b)
#define MPCX_THIS_KERNEL \
  mpcx::k_modexp<MPCX_GEOM_P(MPCX_GEOM_ID), MPCX_GEOM_K(MPCX_GEOM_ID), MPCX_GEOM_G(MPCX_GEOM_ID), MPCX_WPE_SINGLE>

extern "C" {

__attribute__((visibility("hidden"))) hipError_t MPCX_CAT(mpcx_launch_modexp_g, MPCX_GEOM_ID)(
    const mpcx::ModexpArgs* a, uint32_t waves, hipStream_t st) {
#if MPCX_GEOM_ID == 2 || MPCX_GEOM_ID == 5
  if (a->mx_img) {  // the reduction on the matrix cores (mpcx_mx.hpp), MX_WG wavefronts per workgroup
    hipLaunchKernelGGL((mpcx::k_modexp_mx<MPCX_GEOM_P(MPCX_GEOM_ID), MPCX_GEOM_K(MPCX_GEOM_ID),
                                          MPCX_GEOM_G(MPCX_GEOM_ID), MPCX_WPE_SINGLE>),
                       dim3((waves + MX_WG - 1) / MX_WG), dim3(64 * MX_WG), 0, st, *a);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL((MPCX_THIS_KERNEL), dim3(waves), dim3(64), 0, st, *a);
  return hipGetLastError();
}

// several batches in one launch: segs / first are device arrays of nsegs entries
__attribute__((visibility("hidden"))) hipError_t MPCX_CAT(mpcx_launch_modexp_multi_g, MPCX_GEOM_ID)(
    const mpcx::ModexpArgs* segs, const uint32_t* first, uint32_t nsegs, uint32_t waves, int mx, hipStream_t st) {
#if MPCX_GEOM_ID == 2
  if (mx) {  // `waves` counts MX_WG-wavefront workgroups here
    hipLaunchKernelGGL((mpcx::k_modexp_multi_mx<MPCX_GEOM_P(MPCX_GEOM_ID), MPCX_GEOM_K(MPCX_GEOM_ID),
                                                MPCX_GEOM_G(MPCX_GEOM_ID), MPCX_WPE_SINGLE>),
                       dim3(waves), dim3(64 * MX_WG), 0, st, segs, first, nsegs);
    return hipGetLastError();
  }
#else
  if (mx) return hipErrorInvalidValue;
#endif
  hipLaunchKernelGGL((mpcx::k_modexp_multi<MPCX_GEOM_P(MPCX_GEOM_ID), MPCX_GEOM_K(MPCX_GEOM_ID),
                                           MPCX_GEOM_G(MPCX_GEOM_ID), MPCX_WPE_MULTI>),
                     dim3(waves), dim3(64), 0, st, segs, first, nsegs);
  return hipGetLastError();
}

#if MPCX_GEOM_ID == MPCX_FULL_GEOM(0) || MPCX_GEOM_ID == MPCX_FULL_GEOM(1)
// fixed-base comb kernel: the comb-table layouts (full-width geometries of the <= 2080-bit classes);
// `split` wavefronts per workgroup share its G operands' windows
#define MPCX_FB_ARGS MPCX_GEOM_P(MPCX_GEOM_ID), MPCX_GEOM_K(MPCX_GEOM_ID), MPCX_GEOM_G(MPCX_GEOM_ID)
__attribute__((visibility("hidden"))) hipError_t MPCX_CAT(mpcx_launch_fixedbase_g, MPCX_GEOM_ID)(
    const mpcx::FixedBaseArgs* a, uint32_t blocks, uint32_t split, hipStream_t st) {
  const size_t lds = (size_t)mpcx::fb_lds_slice_words<MPCX_FB_ARGS>() * 4u * split;
  hipLaunchKernelGGL((mpcx::k_fixedbase<MPCX_FB_ARGS, MPCX_WPE>), dim3(blocks), dim3(64 * split), lds, st, *a);
  return hipGetLastError();
}

// several comb batches in one launch: segs / first are device arrays of nsegs entries
__attribute__((visibility("hidden"))) hipError_t MPCX_CAT(mpcx_launch_fixedbase_multi_g, MPCX_GEOM_ID)(
    const mpcx::FixedBaseArgs* segs, const uint32_t* first, uint32_t nsegs, uint32_t blocks, uint32_t split,
    hipStream_t st) {
  const size_t lds = (size_t)mpcx::fb_lds_slice_words<MPCX_FB_ARGS>() * 4u * split;
  hipLaunchKernelGGL((mpcx::k_fixedbase_multi<MPCX_FB_ARGS, MPCX_WPE>), dim3(blocks), dim3(64 * split), lds, st,
                     segs, first, nsegs);
  return hipGetLastError();
}
#undef MPCX_FB_ARGS
#endif

// resident 64-thread blocks (= wavefronts) per CU
__attribute__((visibility("hidden"))) hipError_t MPCX_CAT(mpcx_modexp_occupancy_g, MPCX_GEOM_ID)(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, MPCX_THIS_KERNEL, 64, 0);
}

}  // extern "C"
