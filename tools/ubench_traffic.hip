// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on the stream engine's own access
// patterns (diagnostic; MI355X_MICROARCH.md: "calibrate on a known byte count in your own
// access pattern before trusting an absolute"). One dispatch per pattern, known bytes:
//   k_log_store4   one lane stores consecutive 4-B words (placement-log columns)
//   k_log_store8   one lane stores consecutive 8-B words
//   k_wave_store4  a wave stores 64 consecutive 4-B words per instruction (reference)
//   k_rand_load4   64 lanes gather 4-B words at random rows of a 1 GiB table (holder_of,
//                  res_nbytes reads)
//   k_rand_load8   the same, 8-B words
//   k_rand_store8  64 lanes store 8-B words at random rows (state / marks)
//   k_seq_load16   a wave streams 16 B per lane (the guide's calibrated case)
//   hipcc --offload-arch=gfx950 -O3 -o tools/_ubench_traffic tools/ubench_traffic.hip
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- tools/_ubench_traffic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_log_store4(uint32_t* out, long long n) {
  if (threadIdx.x != 0) return;
  for (long long i = 0; i < n; i++) out[i] = (uint32_t)(i * 2654435761u);
}
__global__ void k_log_store8(uint64_t* out, long long n) {
  if (threadIdx.x != 0) return;
  for (long long i = 0; i < n; i++) out[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
}
__global__ void k_wave_store4(uint32_t* out, long long n) {
  for (long long i = threadIdx.x; i < n; i += 64) out[i] = (uint32_t)i;
}
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}
__global__ void k_rand_load4(const uint32_t* tab, long long rows, long long n, uint32_t* sink) {
  uint32_t acc = 0;
  for (long long i = threadIdx.x; i < n; i += 64) acc += tab[mix((uint64_t)i) % (uint64_t)rows];
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}
__global__ void k_rand_load8(const uint64_t* tab, long long rows, long long n, uint64_t* sink) {
  uint64_t acc = 0;
  for (long long i = threadIdx.x; i < n; i += 64) acc += tab[mix((uint64_t)i + 7) % (uint64_t)rows];
  if (acc == 0x12345678ull) sink[threadIdx.x] = acc;
}
__global__ void k_rand_store8(uint64_t* tab, long long rows, long long n) {
  for (long long i = threadIdx.x; i < n; i += 64) tab[mix((uint64_t)i + 11) % (uint64_t)rows] = (uint64_t)i;
}
__global__ void k_seq_load16(const uint4* in, long long n16, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const long long nlog = 1 << 22;           // 4M log entries
  const long long rows = (1ll << 30) / 8;   // 1 GiB table of 8-B rows (past the 256 MiB Infinity Cache)
  const long long nrand = 1 << 21;          // 2M random accesses
  const long long n16 = (1ll << 28) / 16;   // 256 MiB streamed
  uint32_t* log4;
  uint64_t *log8, *tab, *sink;
  uint4* strm;
  CK(hipMalloc(&log4, nlog * 4));
  CK(hipMalloc(&log8, nlog * 8));
  CK(hipMalloc(&tab, rows * 8));
  CK(hipMalloc(&sink, 64 * 16));
  CK(hipMalloc(&strm, n16 * 16));
  CK(hipMemset(tab, 1, rows * 8));
  CK(hipMemset(strm, 1, n16 * 16));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_log_store4, dim3(1), dim3(64), 0, 0, log4, nlog);
  hipLaunchKernelGGL(k_log_store8, dim3(1), dim3(64), 0, 0, log8, nlog);
  hipLaunchKernelGGL(k_wave_store4, dim3(1), dim3(64), 0, 0, log4, nlog);
  hipLaunchKernelGGL(k_rand_load4, dim3(1), dim3(64), 0, 0, (const uint32_t*)tab, rows * 2, nrand, (uint32_t*)sink);
  hipLaunchKernelGGL(k_rand_load8, dim3(1), dim3(64), 0, 0, (const uint64_t*)tab, rows, nrand, sink);
  hipLaunchKernelGGL(k_rand_store8, dim3(1), dim3(64), 0, 0, tab, rows, nrand);
  hipLaunchKernelGGL(k_seq_load16, dim3(1024), dim3(256), 0, 0, (const uint4*)strm, n16, (uint4*)sink);
  CK(hipDeviceSynchronize());
  printf("{\"log_entries\": %lld, \"random_accesses\": %lld, \"table_bytes\": %lld, \"stream_bytes\": %lld}\n",
         nlog, nrand, rows * 8, n16 * 16);
  return 0;
}
