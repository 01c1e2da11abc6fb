// Host cost of hipLaunchKernel on MI355X while other streams hold long-running kernels.
// Build: hipcc -O2 --offload-arch=gfx950 launch_probe.hip -o launch_probe
// Cases: idle device; a long kernel on a second stream; the same on a CU-masked stream;
// small (16 B) vs large (512 B) kernel arguments; launches into a captured hipGraph.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { unsigned long long v[64]; };

__global__ void k_small(unsigned* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[1] += 1; }
__global__ void k_big(Big b, unsigned* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[1] += (unsigned)b.v[3]; }
__global__ void k_spin(unsigned long long cycles, unsigned* p) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) p[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  unsigned* p;
  CK(hipMalloc(&p, 64));
  hipStream_t s1, s2, s3;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
  for (int i = 6; i < 8; i++) mask[i] = 0;  // CUs [192, 256) left out
  CK(hipExtStreamCreateWithCUMask(&s3, (uint32_t)mask.size(), mask.data()));
  Big b{};
  b.v[3] = 1;
  const int N = 400;
  auto run = [&](const char* name, hipStream_t busy, bool big) -> int {
    CK(hipDeviceSynchronize());
    if (busy) hipLaunchKernelGGL(k_spin, dim3(2048), dim3(64), 0, busy, 200000000ull, p);  // ~0.1 s
    if (busy == s1) {  // the launching stream itself is behind: a deep queue on s1, plus s2 and s3
      hipLaunchKernelGGL(k_spin, dim3(1024), dim3(64), 0, s2, 200000000ull, p);
      hipLaunchKernelGGL(k_spin, dim3(1024), dim3(64), 0, s3, 200000000ull, p);
    }
    double t0 = now_us();
    for (int i = 0; i < N; i++) {
      if (big) hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, s1, b, p);
      else hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, s1, p);
    }
    double t1 = now_us();
    CK(hipStreamSynchronize(s1));
    double t2 = now_us();
    CK(hipDeviceSynchronize());
    printf("%-40s launch %7.2f us/launch, drain %7.2f us/kernel\n", name, (t1 - t0) / N, (t2 - t0) / N);
    return 0;
  };
  for (int rep = 0; rep < 2; rep++) {
    if (run("idle, 16 B args", nullptr, false)) return 1;
    if (run("idle, 512 B args", nullptr, true)) return 1;
    if (run("busy stream, 16 B args", s2, false)) return 1;
    if (run("busy stream, 512 B args", s2, true)) return 1;
    if (run("busy CU-masked stream, 16 B args", s3, false)) return 1;
    if (run("busy CU-masked stream, 512 B args", s3, true)) return 1;
    if (run("launching stream busy (deep queue), 16 B", s1, false)) return 1;
    if (run("launching stream busy (deep queue), 512 B", s1, true)) return 1;
  }
  // graph of N launches
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_big, dim3(1024), dim3(256), 0, s1, b, p);
  CK(hipStreamEndCapture(s1, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int rep = 0; rep < 3; rep++) {
    CK(hipDeviceSynchronize());
    double t0 = now_us();
    CK(hipGraphLaunch(ge, s1));
    double t1 = now_us();
    CK(hipStreamSynchronize(s1));
    double t2 = now_us();
    printf("graph of %d: launch %8.1f us, drain %7.2f us/kernel\n", N, t1 - t0, (t2 - t0) / N);
  }
  return 0;
}
