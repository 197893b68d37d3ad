// Micro-benchmark of basic per-wave latencies on gfx950 (diagnostic; one wave):
// dependent LDS load, ds_bpermute, v_readlane -> SGPR -> VALU chains, fp64 divide,
// s_memtime itself. Prints cycles per operation (s_memtime ticks).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench_lat.hip && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned long long* out, int iters, double seed) {
  __shared__ int lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = (i + 1) & 1023;
  __syncthreads();
  // 0: s_memtime back-to-back
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  // 1: dependent LDS loads (pointer chase)
  int p = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) p = lds[p];
  t1 = __builtin_amdgcn_s_memtime();
  out[1] = (t1 - t0) / iters;
  // 2: dependent ds_bpermute chain
  int v = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) v = __shfl(v + p, (v + 1) & 63);
  t1 = __builtin_amdgcn_s_memtime();
  out[2] = (t1 - t0) / iters;
  // 3: readlane chain (lane index depends on previous result)
  int r = lane + v;
  int idx = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) idx = __builtin_amdgcn_readlane(r + idx, (i & 63)) & 63;
  t1 = __builtin_amdgcn_s_memtime();
  out[3] = (t1 - t0) / iters;
  // 4: dependent fp64 divide
  double d = seed + lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) d = d / (1.0000001 + (double)idx);
  t1 = __builtin_amdgcn_s_memtime();
  out[4] = (t1 - t0) / iters;
  // 5: dependent fp64 add chain
  double a = d;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) a = a * 1.0000001 + 0.5;
  t1 = __builtin_amdgcn_s_memtime();
  out[5] = (t1 - t0) / iters;
  // 6: ballot + ctz + readlane loop step
  unsigned long long acc = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    unsigned long long m = __ballot((lane + i + (int)acc) % 3 == 0);
    acc += __builtin_amdgcn_readlane(lane * 3 + (int)acc, __builtin_ctzll(m | 1));
  }
  t1 = __builtin_amdgcn_s_memtime();
  out[6] = (t1 - t0) / iters;
  // 7: LDS atomic add with return, dependent
  int q = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) q = atomicAdd(&lds[(q + lane) & 1023], 1) & 1023;
  t1 = __builtin_amdgcn_s_memtime();
  out[7] = (t1 - t0) / iters;
  // 8: global load chain (L2 hit)
  const unsigned long long* g = out + 64;
  unsigned long long gi = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) gi = __hip_atomic_load(&g[(gi + lane) & 63], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 63;
  t1 = __builtin_amdgcn_s_memtime();
  out[8] = (t1 - t0) / iters;
  // 9: s_memrealtime vs s_memtime over a fixed spin (clock ratio)
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 20000; i++) __builtin_amdgcn_s_sleep(1);
  unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  t1 = __builtin_amdgcn_s_memtime();
  out[9] = t1 - t0;
  out[10] = rt1 - rt0;
  if (lane == 0) out[11] = p + v + idx + (unsigned long long)a + acc + q + gi + (unsigned long long)d;
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 128 * 8);
  hipMemset(d, 0, 128 * 8);
  k<<<1, 64>>>(d, 1000, 1.5);
  hipDeviceSynchronize();
  k<<<1, 64>>>(d, 1000, 1.5);
  unsigned long long h[16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"s_memtime pair", "LDS load chain", "bpermute chain", "readlane chain", "f64 div chain",
                         "f64 mul+add chain", "ballot/ctz/readlane step", "LDS atomic rtn chain", "global load chain (L2)"};
  for (int i = 0; i < 9; i++) printf("%-28s %llu cycles\n", names[i], h[i]);
  printf("memtime ticks %llu vs realtime(100MHz) %llu -> memtime clock %.0f MHz\n", h[9], h[10], 100.0 * h[9] / h[10]);
  return 0;
}
