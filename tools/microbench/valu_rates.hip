// Microbenchmark: sustained issue rate of the integer/fp multiply instructions
// the Montgomery kernels can be built from, on gfx950 (MI355X).
// Each lane runs NCH independent dependency chains of one instruction kind.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define NCH 8
#define ITERS 4096

__global__ void k_mad64(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  uint64_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      uint64_t cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cy) : "v"(a), "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad64_carry(uint64_t* out, uint32_t a0, uint32_t b0) {
  // mad with carry-out into VCC-like sgpr pair + addc consuming it
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  uint64_t acc[NCH]; uint32_t top[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) { acc[c] = c + threadIdx.x; top[c] = 0; }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                   : "+v"(acc[c]), "+v"(top[c]) : "v"(a), "v"(b) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c] + top[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t b = b0 ^ threadIdx.x;
  uint32_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = a0 + c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t b = b0 ^ threadIdx.x;
  uint32_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = a0 + c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad24(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  uint32_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t b = b0 ^ threadIdx.x;
  uint32_t acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = a0 + c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t a0, uint32_t b0) {
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.9999999;
  double acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = c + a0 * 1e-9;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma32(uint64_t* out, uint32_t a0, uint32_t b0) {
  float a = 1.0000001f + threadIdx.x * 1e-9f, b = 0.9999999f;
  float acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = c + a0 * 1e-9f;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_pkfma32(uint64_t* out, uint32_t a0, uint32_t b0) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a = {1.0000001f, 1.0000002f}, b = {0.9999999f, 0.9999998f};
  f2 acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) { acc[c].x = c; acc[c].y = a0 * 1e-9f; }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) s += acc[c].x + acc[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t);

int main() {
  struct K { const char* name; kfn f; double ops_per_inst; const char* unit; } ks[] = {
    {"v_mad_u64_u32", k_mad64, 1, "32x32+64 MAC"},
    {"v_mad_u64_u32+v_addc (carry-out)", k_mad64_carry, 1, "MAC (pair)"},
    {"v_mul_lo_u32", k_mullo, 1, "mul"},
    {"v_mul_hi_u32", k_mulhi, 1, "mul"},
    {"v_mad_u32_u24", k_mad24, 1, "mad24"},
    {"v_add_co+v_addc (pair)", k_addc, 1, "pair"},
    {"v_fma_f64", k_fma64, 1, "fma"},
    {"v_fma_f32", k_fma32, 1, "fma"},
    {"v_pk_fma_f32", k_pkfma32, 2, "fma"},
  };
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  const int threads = 256;
  for (int wpsimd : {1, 2, 4, 8}) {
    int blocks = prop.multiProcessorCount * wpsimd;  // 4 waves per block => wpsimd waves per SIMD
    uint64_t* d; hipMalloc(&d, (size_t)blocks * threads * 8);
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u, 2u);
      hipDeviceSynchronize();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u, 2u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double insts = (double)reps * blocks * threads * ITERS * NCH;  // lane-instructions
      double rate = insts / (ms * 1e-3);
      // cycles per wave-instruction per SIMD at 2.4 GHz nominal:
      double simds = prop.multiProcessorCount * 4.0;
      double cyc = simds * 2.4e9 / (rate / 64.0);
      printf("waves/SIMD %d  %-36s %8.2f T lane-inst/s  (%.2f T %s/s)  ~%.2f cyc/wave-inst/SIMD @2.4GHz\n",
             wpsimd, k.name, rate / 1e12, rate * k.ops_per_inst / 1e12, k.unit, cyc);
      hipEventDestroy(e0); hipEventDestroy(e1);
    }
    hipFree(d);
  }
  return 0;
}
