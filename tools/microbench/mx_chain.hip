// Squaring chains on one 4096-bit modulus: montmul_mx (reduction on the i8
// matrix cores, mpcx_mx.hpp) against montmul<4, 37> (the CIOS row loop of
// geometry 2), plus a 16x16x64 i8 MFMA lane-map check. Driven by mx_chain.py:
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o mx_chain.so mx_chain.hip
#include <hip/hip_runtime.h>

#include "../../mpcium_amd/csrc/mpcx_device.hpp"

using namespace mpcx;
constexpr int MX_P = MxG2::P, MX_K = MxG2::K, MX_L = MxG2::L, MX_G = MxG2::G, MX_ROW = MxG2::ROW;

// one MFMA: C = A B with per-lane fragments a[lane], b[lane] (16 bytes each)
__global__ __launch_bounds__(64) void k_mfma_map(const mx_v4i* a, const mx_v4i* b, mx_v4i* c) {
  const int l = threadIdx.x;
  c[l] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], mx_v4i{0, 0, 0, 0}, 0, 0, 0);
}

// x: count x 148 radix-2^28 digits (< 2m); out: the same after S squarings.
// MX_WG wavefronts per workgroup share the LDS tables (img: mpcx_mx_tables).
#ifndef MXB_WPE
#define MXB_WPE 2
#endif
__global__ __launch_bounds__(64 * MX_WG) __attribute__((amdgpu_waves_per_eu(MXB_WPE))) void k_chain_mx(
    const uint32_t* x, uint32_t* out, const uint32_t* img, const uint32_t* md_g, uint32_t S, uint32_t count,
    uint32_t* dbg) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[MxG2::LDS_WORDS_WG];
  for (int i = (int)threadIdx.x; i < MxG2::IMG_BYTES / 4; i += 64 * MX_WG) lds[i] = img[i];
  for (int i = (int)threadIdx.x; i < MxG2::L; i += 64 * MX_WG) lds[MxG2::IMG_BYTES / 4 + i] = md_g[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* rows = lds + MxG2::IMG_BYTES / 4 + MxG2::L + 4 + wave * MxG2::WAVE_WORDS;
  const uint32_t* md = lds + MxG2::IMG_BYTES / 4;
  const int g = lane >> 2, p = lane & 3;
  const uint32_t blk = blockIdx.x * MX_WG + wave;
  const uint32_t op = blk * MX_G + g;
  uint32_t A[MX_K];
#pragma unroll
  for (int k = 0; k < MX_K; ++k) A[k] = op < count ? x[(size_t)op * MX_L + p * MX_K + k] : 0u;
  const MxConsts c = mx_consts<MxG2>(reinterpret_cast<const uint8_t*>(lds), lane);
#ifdef MXB_STAGGER
  // the workgroup's second half (sharing SIMDs with the first) starts later, so
  // one wave's matrix-core phase meets the other's VALU product loop
  if (wave >= MX_WG / 2)
    for (int i = 0; i < MXB_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif
#ifdef MXB_PRIO_HALF
  if (wave >= MX_WG / 2) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef MX_PROF
  MxProf prof{};
#define PROF_ARG , &prof
#else
#define PROF_ARG
#endif
  for (uint32_t s = 0; s < S; ++s) {
    lds_store_sqr<MX_K>(rows + g * MxG2::ROW, p, A);
    wave_lds_fence();
    montmul_mx<MxG2, true, (bool)MPCX_SQR_B2>(A, rows, md, c, lane PROF_ARG);
    wave_lds_fence();
  }
#ifdef MX_PROF
  // per-wave phase cycles (s_memtime ticks) after the rows' debug copy
  if (dbg && lane == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) dbg[MX_G * MX_ROW + blk * 8 + i] = (uint32_t)(prof.t[i] >> 8);
  }
#endif
  if (op < count) {
#pragma unroll
    for (int k = 0; k < MX_K; ++k) out[(size_t)op * MX_L + p * MX_K + k] = A[k];
  }
  if (dbg && blk == 0) {  // wavefront 0's rows after the last product (U + m digits)
    for (int i = lane; i < MX_G * MX_ROW; i += 64) dbg[i] = rows[i];
  }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_chain_cios(
    const uint32_t* x, uint32_t* out, const uint32_t* nd, uint32_t n0inv, uint32_t S, uint32_t count) {
  __shared__ uint32_t lds[(MX_G + 1) * MX_L + 2];
  const int lane = threadIdx.x;
  const int g = lane >> 2, p = lane & 3;
  const uint32_t op = blockIdx.x * MX_G + g;
  uint32_t A[MX_K], Nd[MX_K];
#pragma unroll
  for (int k = 0; k < MX_K; ++k) {
    A[k] = op < count ? x[(size_t)op * MX_L + p * MX_K + k] : 0u;
    Nd[k] = nd[p * MX_K + k];
  }
  uint32_t* bl = lds + g * MX_L;
  for (uint32_t s = 0; s < S; ++s) {
    lds_store_sqr<MX_K>(bl, p, A);
    wave_lds_fence();
    montmul<MX_P, MX_K, true, (bool)MPCX_SQR_B2>(A, bl, Nd, n0inv, 0, p);
    wave_lds_fence();
  }
  if (op < count) {
#pragma unroll
    for (int k = 0; k < MX_K; ++k) out[(size_t)op * MX_L + p * MX_K + k] = A[k];
  }
}

static float timed(hipStream_t s, void (*launch)(hipStream_t, void*), void* arg) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  launch(s, arg);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = -1.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

struct MxArgs {
  const uint32_t* x;
  uint32_t* out;
  const uint32_t* img;
  const uint32_t* md;
  uint32_t S, count;
  uint32_t* dbg;
};
struct CiosArgs {
  const uint32_t* x;
  uint32_t* out;
  const uint32_t* nd;
  uint32_t n0inv, S, count;
};

extern "C" {

int mxb_mfma_map(const void* a, const void* b, void* c) {
  hipLaunchKernelGGL(k_mfma_map, dim3(1), dim3(64), 0, nullptr, (const mx_v4i*)a, (const mx_v4i*)b, (mx_v4i*)c);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

// returns milliseconds (< 0 on a launch error)
float mxb_chain_mx(const void* x, void* out, const void* img, const void* md, uint32_t S, uint32_t count,
                   void* dbg) {
  MxArgs a{(const uint32_t*)x, (uint32_t*)out, (const uint32_t*)img, (const uint32_t*)md, S, count, (uint32_t*)dbg};
  const float ms = timed(
      nullptr,
      [](hipStream_t s, void* v) {
        const MxArgs& a = *(const MxArgs*)v;
        const uint32_t waves = (a.count + MX_G - 1) / MX_G;
        hipLaunchKernelGGL(k_chain_mx, dim3((waves + MX_WG - 1) / MX_WG), dim3(64 * MX_WG), 0, s, a.x, a.out, a.img,
                           a.md, a.S, a.count, a.dbg);
      },
      &a);
  return hipGetLastError() == hipSuccess ? ms : -1.f;
}

float mxb_chain_cios(const void* x, void* out, const void* nd, uint32_t n0inv, uint32_t S, uint32_t count) {
  CiosArgs a{(const uint32_t*)x, (uint32_t*)out, (const uint32_t*)nd, n0inv, S, count};
  const float ms = timed(
      nullptr,
      [](hipStream_t s, void* v) {
        const CiosArgs& a = *(const CiosArgs*)v;
        hipLaunchKernelGGL(k_chain_cios, dim3((a.count + MX_G - 1) / MX_G), dim3(64), 0, s, a.x, a.out, a.nd, a.n0inv,
                           a.S, a.count);
      },
      &a);
  return hipGetLastError() == hipSuccess ? ms : -1.f;
}

}  // extern "C"
