// Microbenchmark (not product): dependent-chain latency of FP64 ops on one wave (unrolled x64)
#include <hip/hip_runtime.h>
#include <cstdio>
#define R64(x) x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x
__global__ void k(int mode, double* out, long long* cyc) {
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0000001, c = 0.5;
  unsigned u = threadIdx.x;
  long long t0 = clock64();
  if (mode == 0) { R64(a = __dadd_rn(a, b);) }
  else if (mode == 1) { R64(a = __dmul_rn(a, b);) }
  else if (mode == 2) { R64(a = __builtin_fmin(a, c + a);) }
  else if (mode == 3) { R64(a = __ddiv_rn(a, b);) }
  else if (mode == 4) { R64(u = u * 3u + 1u;) a += u; }
  else if (mode == 5) { R64(a = (double)(unsigned)a + b;) }
  long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* o; long long* c; (void)hipMalloc(&o, 64 * 8); (void)hipMalloc(&c, 8);
  const char* names[] = {"dadd", "dmul", "fmin(a, c+a)", "ddiv", "u32 mad", "cvt u32<->f64 + add"};
  for (int m = 0; m < 6; m++) {
    long long best = 1ll << 60;
    for (int r = 0; r < 3; r++) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, m, o, c);
      long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }
    printf("%-22s %.1f cycles per dependent op\n", names[m], best / 64.0);
  }
  return 0;
}
