// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE for the access shapes of the k-NN
// kernels (the guide's x2 gfx950 correction is measured for 16-B streaming reads
// only). Three kernels read known byte counts from buffers far larger than the Infinity Cache,
// each launched once per run; run under `rocprofv3 --pmc FETCH_SIZE` and compare FETCH_SIZE x
// 1024 with the bytes below (tools/fetch_calib.py):
//   stream   every lane reads 16 B, the wave 1 KiB contiguous (the guide's calibrated shape)
//   gather16 every lane reads 16 B from its own random 128-B line (a float4 photon / query record
//            gathered through a permutation): 16 B used per line touched
//   gather64 every lane reads 64 B (4 x 16 B) from its own random 128-B-aligned line
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

__global__ void stream_kernel(const float4 *p, int64_t n, float *out) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1.2345f) out[0] = acc;  // keeps the loads
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// reads `per` consecutive float4 from line mix(i) % lines of a buffer of `lines` 128-B lines
template <int PER>
__global__ void gather_kernel(const float4 *p, int64_t lines, int64_t n, float *out) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = (int64_t)(mix((uint64_t)i) % (uint64_t)lines);
#pragma unroll
    for (int k = 0; k < PER; k++) {
      float4 v = p[l * 8 + k];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 1.2345f) out[0] = acc;
}

int main() {
  const size_t bytes = (size_t)4 << 30;  // 4 GiB >> 256 MiB Infinity Cache
  float4 *p;
  float *out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  CK(hipMemset(p, 0, bytes));
  const int64_t n16 = (int64_t)(bytes / 16), lines = (int64_t)(bytes / 128);
  const int64_t ng = (int64_t)1 << 22;  // 4 M gathers over 33.5 M lines: ~6 % touch a line twice
  CK(hipDeviceSynchronize());
  stream_kernel<<<65536, 256>>>(p, n16 / 4, out);  // 1 GiB
  CK(hipDeviceSynchronize());
  gather_kernel<1><<<65536, 256>>>(p, lines, ng, out);
  CK(hipDeviceSynchronize());
  gather_kernel<4><<<65536, 256>>>(p, lines, ng, out);
  CK(hipDeviceSynchronize());
  printf("{\"stream_bytes\": %lld, \"gather16_lines\": %lld, \"gather64_lines\": %lld, \"lines_total\": %lld}\n",
         (long long)(n16 / 4 * 16), (long long)ng, (long long)ng, (long long)lines);
  CK(hipFree(p));
  CK(hipFree(out));
  return 0;
}
