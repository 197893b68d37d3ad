// Micro-benchmark of the executor's cross-lane patterns on gfx950 (diagnostic; one wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/_ubench_pat tools/ubench_pat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

__global__ void k(unsigned long long* out, int iters, double seed, unsigned long long msk) {
  const int lane = threadIdx.x;
  double key = seed + (lane * 37 % 64);
  long long nb = lane * 11;
  int w = lane;
  int acc = 0;
  unsigned long long t0, t1;
  // A: per candidate, 5 readlanes (f64 key, i64 nb, i32 w) + lexicographic VALU compare
  t0 = clk();
  for (int it = 0; it < iters; it++) {
    const int l = it & 63;
    const double qk = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(key) >> 32), l) << 32) |
                                           (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(key), l));
    const long long qn = ((long long)__builtin_amdgcn_readlane((int)(nb >> 32), l) << 32) | (unsigned)__builtin_amdgcn_readlane((int)nb, l);
    const int qw = __builtin_amdgcn_readlane(w, l);
    const bool less = qk != key ? qk < key : (qn != nb ? qn < nb : qw < w);
    acc += less;
  }
  t1 = clk();
  out[0] = (t1 - t0) / iters;
  // B: same, iterating a lane mask with ctz (the loop control on SALU only)
  t0 = clk();
  for (int it = 0; it < iters / 4; it++) {
    for (unsigned long long rm = msk; rm; rm &= rm - 1) {
      const int l = __builtin_ctzll(rm);
      const double qk = __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(key) >> 32), l) << 32) |
                                             (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(key), l));
      const int qw = __builtin_amdgcn_readlane(w, l);
      acc += (qk < key || (qk == key && qw < w));
    }
  }
  t1 = clk();
  out[1] = (t1 - t0) / (iters / 4 * __builtin_popcountll(msk));
  // C: divergent if with two statements (exec-mask branch)
  long long s2 = 0;
  t0 = clk();
  for (int it = 0; it < iters; it++) {
    if (((lane + it + acc) & 7) == 0) {
      s2 += nb * it;
      acc ^= it;
    }
  }
  t1 = clk();
  out[2] = (t1 - t0) / iters;
  // D: ballot -> ctz -> readlane -> SALU use (dependent)
  int x = lane;
  t0 = clk();
  for (int it = 0; it < iters; it++) {
    const unsigned long long m = __ballot(((x + it) & 3) == 0) | 1ull;
    x += __builtin_amdgcn_readlane(x, __builtin_ctzll(m)) & 7;
  }
  t1 = clk();
  out[3] = (t1 - t0) / iters;
  // E: a plain dependent VALU int chain (issue + dependency)
  int y = lane;
  t0 = clk();
  for (int it = 0; it < iters; it++) y = (y * 3 + it) ^ (y >> 2);
  t1 = clk();
  out[4] = (t1 - t0) / iters;
  // F: 8 independent VALU int chains (throughput)
  int z0 = lane, z1 = lane + 1, z2 = lane + 2, z3 = lane + 3, z4 = lane + 4, z5 = lane + 5, z6 = lane + 6, z7 = lane + 7;
  t0 = clk();
  for (int it = 0; it < iters; it++) {
    z0 = z0 * 3 + it; z1 = z1 * 3 + it; z2 = z2 * 3 + it; z3 = z3 * 3 + it;
    z4 = z4 * 3 + it; z5 = z5 * 3 + it; z6 = z6 * 3 + it; z7 = z7 * 3 + it;
  }
  t1 = clk();
  out[5] = (t1 - t0) / iters;
  // G: uniform SALU-only chain (s_mul/s_add on readfirstlane'd value)
  int u = __builtin_amdgcn_readfirstlane(lane + 5);
  t0 = clk();
  for (int it = 0; it < iters; it++) u = (u * 3 + it) ^ (u >> 2);
  t1 = clk();
  out[6] = (t1 - t0) / iters;
  // H: v_cmp -> ballot -> popcount -> VALU (VALU->SALU->VALU round trip)
  int h = lane;
  t0 = clk();
  for (int it = 0; it < iters; it++) h += __builtin_popcountll(__ballot(((h + it) & 1) == 0));
  t1 = clk();
  out[7] = (t1 - t0) / iters;
  if (lane == 0) out[8] = acc + s2 + x + y + z0 + z1 + z2 + z3 + z4 + z5 + z6 + z7 + u + h;
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 64 * 8);
  k<<<1, 64>>>(d, 1024, 1.5, 0x0000100100011001ull);
  hipDeviceSynchronize();
  k<<<1, 64>>>(d, 1024, 1.5, 0x0000100100011001ull);
  unsigned long long h[9];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"A readlane x5 + key compare", "B mask-iter + readlane + cmp", "C divergent if (2 stmts)",
                         "D ballot->ctz->readlane dep", "E dependent VALU int op x3", "F 8 indep VALU chains (x8)",
                         "G SALU dependent chain x3", "H v_cmp->ballot->popc->VALU"};
  for (int i = 0; i < 8; i++) printf("%-32s %llu cycles/iter\n", names[i], h[i]);
  return 0;
}
