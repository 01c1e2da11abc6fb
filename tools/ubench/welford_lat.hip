// Microbenchmark (not product): cycles per dependent step of the t-digest Welford update
// (W += w; mean += (v - mean) * w / W) in FP64 on one wave, and of its parts.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int mode, int n, double* out, long long* cyc) {
  double mean = 1.0 + threadIdx.x * 1e-3, W = 100.0, v = 3.0 + threadIdx.x, w = 1.0;
  long long t0 = clock64();
  if (mode == 0) {  // full step
    for (int s = 0; s < n; s++) {
      W = __dadd_rn(W, w);
      mean = __dadd_rn(mean, __ddiv_rn(__dmul_rn(__dsub_rn(v, mean), w), W));
    }
  } else if (mode == 1) {  // division only (dependent)
    for (int s = 0; s < n; s++) mean = __ddiv_rn(mean, W);
  } else if (mode == 2) {  // add only
    for (int s = 0; s < n; s++) mean = __dadd_rn(mean, W);
  } else if (mode == 3) {  // full step, two independent chains
    double m2 = mean + 1, W2 = W + 3;
    for (int s = 0; s < n; s++) {
      W = __dadd_rn(W, w);
      mean = __dadd_rn(mean, __ddiv_rn(__dmul_rn(__dsub_rn(v, mean), w), W));
      W2 = __dadd_rn(W2, w);
      m2 = __dadd_rn(m2, __ddiv_rn(__dmul_rn(__dsub_rn(v, m2), w), W2));
    }
    mean += m2;
  } else if (mode == 4) {  // reciprocal multiply (not exact; latency reference)
    for (int s = 0; s < n; s++) {
      W = __dadd_rn(W, w);
      mean = __dadd_rn(mean, __dmul_rn(__dmul_rn(__dsub_rn(v, mean), w), __drcp_rn(W)));
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = mean + W;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* o; long long* c; hipMalloc(&o, 64 * 8); hipMalloc(&c, 8);
  const char* names[] = {"welford step", "ddiv only", "dadd only", "welford x2 chains", "rcp-mul step"};
  for (int m = 0; m < 5; m++) {
    long long best = 1ll << 60;
    for (int r = 0; r < 3; r++) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, m, 1000, o, c);
      long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }
    printf("%-20s %.1f cycles per step\n", names[m], best / 1000.0);
  }
  return 0;
}
