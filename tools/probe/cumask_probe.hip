// Which CUs does a CU-masked stream's kernel run on?  Each workgroup records its XCC, SE, SH
// and CU (s_getreg HW_ID / XCC_ID).  For a few candidate masks the host prints how many CUs
// of each (XCC, SE) the masked kernel used -- the layout the engine's side/replay masks need.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <set>
#include <vector>

__global__ void k_where(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    // gfx9 HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
    out[blockIdx.x] = ((xcc & 0xf) << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
    uint64_t t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < 20000) {}
  }
}

static void run(hipStream_t st, const char* what) {
  const int nb = 16384;
  uint32_t* d;
  (void)hipMalloc(&d, nb * 4);
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, st, d);
  (void)hipStreamSynchronize(st);
  std::vector<uint32_t> h(nb);
  (void)hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
  std::set<uint32_t> cus(h.begin(), h.end());
  std::map<uint32_t, int> per;  // (xcc, se) -> CUs
  for (auto c : cus) per[c >> 8]++;
  printf("%-10s %3zu CUs |", what, cus.size());
  for (auto& kv : per) printf(" x%u.se%u:%d", kv.first >> 8, kv.first & 7, kv.second);
  printf("\n");
  (void)hipFree(d);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const uint32_t ncu = p.multiProcessorCount;
  hipStream_t a;
  (void)hipStreamCreate(&a);
  run(a, "unmasked");
  struct M {
    const char* name;
    int kind;
  };
  for (M m : {M{"i/8%4!=3", 0}, M{"i%4!=3", 1}, M{"i%8!=7", 2}, M{"i<32", 3}, M{"i<8", 4}, M{"i%32<4", 5}}) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (uint32_t i = 0; i < ncu; i++) {
      bool on = m.kind == 0   ? (i / 8) % 4 != 3
                : m.kind == 1 ? i % 4 != 3
                : m.kind == 2 ? i % 8 != 7
                : m.kind == 3 ? i < 32
                : m.kind == 4 ? i < 8
                              : (i % 32) < 4;
      if (on) mask[i / 32] |= 1u << (i % 32);
    }
    hipStream_t b;
    if (hipExtStreamCreateWithCUMask(&b, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
      printf("%s: create failed\n", m.name);
      continue;
    }
    run(b, m.name);
    (void)hipStreamDestroy(b);
  }
  return 0;
}
