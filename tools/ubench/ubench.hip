// Single-wave latency calibration for the exact t-digest replay (gfx950).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../veneur_amd/csrc ubench.hip -o ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "gomath.h"

using namespace vn;

__global__ void k_bench(unsigned long long* out, const double* g, int iters) {
  __shared__ unsigned int lds[4096];
  __shared__ double ldsd[4096];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4096; i += 64) {
    lds[i] = (i * 97 + 13) & 4095;
    ldsd[i] = 0.001 * i;
  }
  __syncthreads();
  long long t0, t1;
  // 0: clock64 overhead
  t0 = clock64();
  t1 = clock64();
  if (lane == 0) out[0] = t1 - t0;
  // 1: dependent LDS u32 loads (per-lane distinct addresses)
  unsigned p = lane;
  t0 = clock64();
  for (int i = 0; i < iters; i++) p = lds[p];
  t1 = clock64();
  if (lane == 0) out[1] = (t1 - t0) / iters;
  // 2: dependent LDS f64 loads + add
  double x = 0.5;
  unsigned q = lane;
  t0 = clock64();
  for (int i = 0; i < iters; i++) {
    x = dadd(x, ldsd[q]);
    q = (q + (unsigned)x) & 4095;
  }
  t1 = clock64();
  if (lane == 0) out[2] = (t1 - t0) / iters;
  // 3: dependent f64 add
  double a = g[lane], b = g[lane + 64];
  t0 = clock64();
  for (int i = 0; i < iters; i++) a = dadd(a, b);
  t1 = clock64();
  if (lane == 0) out[3] = (t1 - t0) / iters;
  // 4: dependent ddiv
  double d = 1.0 + g[lane];
  t0 = clock64();
  for (int i = 0; i < iters; i++) d = ddiv(d, 1.0000001);
  t1 = clock64();
  if (lane == 0) out[4] = (t1 - t0) / iters;
  // 5: dependent index_estimate
  double k = 0.3 + 0.001 * lane;
  t0 = clock64();
  for (int i = 0; i < iters; i++) k = index_estimate(100.0, k * 0.01);
  t1 = clock64();
  if (lane == 0) out[5] = (t1 - t0) / iters;
  // 6: ballot + ctz + readlane step (chain-walk inner step)
  double base = 0.0, kv = 0.001 * lane;
  unsigned from = 0, cnt = 0;
  t0 = clock64();
  for (int i = 0; i < iters; i++) {
    bool c = lane >= (int)from && dsub(kv, base) > -1.0;
    unsigned long long bal = __ballot(c);
    unsigned f = bal ? (unsigned)__builtin_ctzll(bal) : 0u;
    int lo = __builtin_amdgcn_readlane(__double2loint(kv), f);
    int hi = __builtin_amdgcn_readlane(__double2hiint(kv), f);
    base = __hiloint2double(hi, lo) - 1e-9;
    from = (f + 1) & 63;
    cnt += f;
  }
  t1 = clock64();
  if (lane == 0) out[6] = (t1 - t0) / iters;
  // 7: dependent global loads (L2-resident, 8 KB)
  unsigned gp = lane;
  const unsigned* gu = reinterpret_cast<const unsigned*>(g);
  t0 = clock64();
  for (int i = 0; i < iters; i++) gp = gu[gp & 2047] & 2047;
  t1 = clock64();
  if (lane == 0) out[7] = (t1 - t0) / iters;
  // 8: __syncthreads in a one-wave block
  t0 = clock64();
  for (int i = 0; i < iters; i++) __syncthreads();
  t1 = clock64();
  if (lane == 0) out[8] = (t1 - t0) / iters;
  // 9: dependent LDS load with s_waitcnt + shfl (ds_bpermute)
  double s = 0.001 * lane;
  t0 = clock64();
  for (int i = 0; i < iters; i++) s = __shfl_up(s, 1, 64) + 1e-9;
  t1 = clock64();
  if (lane == 0) out[9] = (t1 - t0) / iters;
  if (lane == 0) out[15] = p + (unsigned)x + (unsigned)a + (unsigned)d + (unsigned)k + cnt + gp + (unsigned)s;
}

int main() {
  double* g;
  unsigned long long* o;
  hipMalloc(&g, 8192 * 8);
  hipMalloc(&o, 16 * 8);
  double h[8192];
  for (int i = 0; i < 8192; i++) h[i] = (double)((i * 131 + 7) % 2048) * 1e-300 + 1e-3 * (i % 7);
  unsigned* hu = reinterpret_cast<unsigned*>(h);
  for (int i = 0; i < 2048; i++) hu[i] = (unsigned)((i * 613 + 5) & 2047);
  hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, o, g, 1000);
    hipDeviceSynchronize();
  }
  unsigned long long r[16];
  hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  const char* names[] = {"clock64 pair", "LDS u32 dep load", "LDS f64 load+add dep", "f64 add dep", "ddiv dep",
                         "index_estimate dep", "ballot+ctz+readlane step", "global L2 dep load", "syncthreads 1-wave",
                         "shfl_up f64 dep"};
  for (int i = 0; i < 10; i++) printf("%-28s %llu cycles\n", names[i], r[i]);
  return 0;
}
