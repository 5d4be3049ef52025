// FETCH_SIZE / WRITE_SIZE calibration for the access width libmpcx's
// window tables use (one 4-byte dword per lane per buffer access, a wave
// touching 256 contiguous bytes), as MI355X_MICROARCH.md's HBM section
// prescribes for uncalibrated widths: read and write a known byte count far
// larger than the 256 MiB Infinity Cache, then compare with the counters.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib    (then --pmc WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

// each wave reads `iters` consecutive 256-B rows (one dword per lane per row)
__global__ void k_read(const unsigned* __restrict__ src, unsigned* __restrict__ out, unsigned iters) {
  const unsigned lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned* p = src + (size_t)wave * iters * 64u + lane;
  unsigned acc = 0;
  for (unsigned i = 0; i < iters; ++i) acc += p[(size_t)i * 64u] ^ i;
  out[(size_t)wave * 64u + lane] = acc;  // 256 B per wave: counted in WRITE_SIZE, negligible here
}

// each wave writes `iters` consecutive 256-B rows (one dword per lane per row)
__global__ void k_write(unsigned* __restrict__ dst, unsigned iters) {
  const unsigned lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  unsigned* p = dst + (size_t)wave * iters * 64u + lane;
  for (unsigned i = 0; i < iters; ++i) p[(size_t)i * 64u] = i * 2654435761u + lane;
}

int main() {
  const unsigned waves = 1u << 16, iters = 64;  // 65,536 waves x 64 rows x 256 B = 1 GiB
  const size_t words = (size_t)waves * iters * 64u;
  unsigned *buf = nullptr, *out = nullptr;
  if (hipMalloc((void**)&buf, words * 4) != hipSuccess || hipMalloc((void**)&out, (size_t)waves * 64u * 4) != hipSuccess) {
    std::fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  const dim3 block(256), grid(waves * 64u / 256u);
  k_write<<<grid, block>>>(buf, iters);   // dispatch 1: writes 1 GiB
  k_read<<<grid, block>>>(buf, out, iters);  // dispatch 2: reads 1 GiB (+ 16 MiB of results)
  if (hipDeviceSynchronize() != hipSuccess) {
    std::fprintf(stderr, "kernel failed\n");
    return 1;
  }
  std::printf("{\"bytes_written_k_write\": %zu, \"bytes_read_k_read\": %zu, \"bytes_written_k_read\": %zu}\n",
              words * 4, words * 4, (size_t)waves * 64u * 4);
  hipFree(buf);
  hipFree(out);
  return 0;
}
