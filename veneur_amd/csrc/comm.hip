// comm.hip -- RCCL and in-process transports of the cross-GPU exchange (comm.h).
#include <dlfcn.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "comm.h"

namespace vn {

// ---------------------------------------------------------------- RCCL, bound at run time
namespace {

struct NcclId {
  char internal[128];
};
using nccl_res = int;
struct Rccl {
  void* so = nullptr;
  nccl_res (*get_unique_id)(NcclId*) = nullptr;
  nccl_res (*comm_init_rank)(void**, int, NcclId, int) = nullptr;
  nccl_res (*comm_destroy)(void*) = nullptr;
  nccl_res (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  nccl_res (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  nccl_res (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
  nccl_res (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
  nccl_res (*group_start)() = nullptr;
  nccl_res (*group_end)() = nullptr;
  const char* (*error_string)(nccl_res) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

// The RCCL of the process: a copy already loaded (e.g. by PyTorch), else the one that sits
// beside the HIP runtime the engine runs on (PyTorch's bundle or /opt/rocm), else the soname.
const Rccl& rccl() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.so) return g_rccl;
  void* so = nullptr;
  for (const char* n : {"librccl.so.1", "librccl.so"})
    if (!so) so = dlopen(n, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
  if (!so) {
    Dl_info info{};
    hipError_t (*probe)(void**, size_t) = &hipMalloc;  // a symbol of the HIP runtime in use
    if (dladdr(reinterpret_cast<void*>(probe), &info) && info.dli_fname) {
      std::string dir(info.dli_fname);
      dir = dir.substr(0, dir.find_last_of('/') + 1);
      for (const char* n : {"librccl.so.1", "librccl.so"})
        if (!so) so = dlopen((dir + n).c_str(), RTLD_NOW | RTLD_GLOBAL);
    }
  }
  if (!so) so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!so) throw std::runtime_error(std::string("cannot load librccl: ") + dlerror());
  Rccl r;
  r.so = so;
  auto sym = [&](auto& fp, const char* name) {
    fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(so, name));
    if (!fp) throw std::runtime_error(std::string("librccl lacks ") + name);
  };
  sym(r.get_unique_id, "ncclGetUniqueId");
  sym(r.comm_init_rank, "ncclCommInitRank");
  sym(r.comm_destroy, "ncclCommDestroy");
  sym(r.all_reduce, "ncclAllReduce");
  sym(r.all_gather, "ncclAllGather");
  sym(r.send, "ncclSend");
  sym(r.recv, "ncclRecv");
  sym(r.group_start, "ncclGroupStart");
  sym(r.group_end, "ncclGroupEnd");
  sym(r.error_string, "ncclGetErrorString");
  g_rccl = r;
  return g_rccl;
}

void nccl_check(nccl_res r, const char* what) {
  if (r != 0) throw std::runtime_error(std::string(what) + ": " + rccl().error_string(r));
}

// ncclDataType_t / ncclRedOp_t (rccl.h)
int nccl_dtype(DType t) {
  switch (t) {
    case kU8: return 1;    // ncclUint8
    case kU32: return 3;   // ncclUint32
    case kU64: return 5;   // ncclUint64
    case kI64: return 4;   // ncclInt64
    case kF64: return 8;   // ncclFloat64
  }
  return 1;
}
int nccl_op(ROp o) { return o == kSum ? 0 : (o == kMax ? 2 : 3); }

}  // namespace

// ---------------------------------------------------------------- in-process group
struct LocalGroup {
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> send;
  std::vector<const uint64_t*> soff;
  explicit LocalGroup(int n_) : n(n_), send(n_), soff(n_) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

size_t dtype_size(DType t) { return t == kU8 ? 1 : (t == kU32 ? 4 : 8); }

template <class T>
__device__ __forceinline__ T rop(T a, T b, int op) {
  return op == kSum ? a + b : (op == kMax ? (a > b ? a : b) : (a < b ? a : b));
}
// recv[i] = op over r of src[r * count + i]
template <class T>
__global__ void k_local_reduce(const T* __restrict__ src, T* __restrict__ recv, size_t count, int n, int op) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    T v = src[i];
    for (int r = 1; r < n; r++) v = rop(v, src[(size_t)r * count + i], op);
    recv[i] = v;
  }
}

void comm_allreduce(vn_comm* c, const void* send, void* recv, size_t count, DType t, ROp op, hipStream_t st) {
  if (!count) return;
  const size_t bytes = count * dtype_size(t);
  if (c->nccl) {
    nccl_check(rccl().all_reduce(send, recv, count, nccl_dtype(t), nccl_op(op), c->nccl, st), "ncclAllReduce");
    return;
  }
  LocalGroup& g = *c->group;
  if (g.n == 1) {
    if (send != recv) VN_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, st));
    return;
  }
  if (c->scratch_cap < bytes * g.n) {
    if (c->scratch) (void)hipFree(c->scratch);
    c->scratch = nullptr;
    c->scratch_cap = 0;
    VN_HIP_CHECK(hipMalloc(&c->scratch, bytes * g.n));
    c->scratch_cap = bytes * g.n;
  }
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.send[c->rank] = send;
  g.barrier();
  // copies on the caller's stream, complete before the barrier (a device-to-device hipMemcpy
  // may return before its copy is done)
  for (int r = 0; r < g.n; r++)
    VN_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(c->scratch) + (size_t)r * bytes, g.send[r], bytes,
                                hipMemcpyDeviceToDevice, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.barrier();  // every rank holds every operand: recv (which may be send) can be written
  const int grid = (int)std::min<size_t>((count + 255) / 256, 4096);
  switch (t) {
    case kU8: hipLaunchKernelGGL(k_local_reduce<uint8_t>, dim3(grid), dim3(256), 0, st,
                                 static_cast<const uint8_t*>(c->scratch), static_cast<uint8_t*>(recv), count, g.n, (int)op); break;
    case kU32: hipLaunchKernelGGL(k_local_reduce<uint32_t>, dim3(grid), dim3(256), 0, st,
                                  static_cast<const uint32_t*>(c->scratch), static_cast<uint32_t*>(recv), count, g.n, (int)op); break;
    case kU64: hipLaunchKernelGGL(k_local_reduce<uint64_t>, dim3(grid), dim3(256), 0, st,
                                  static_cast<const uint64_t*>(c->scratch), static_cast<uint64_t*>(recv), count, g.n, (int)op); break;
    case kI64: hipLaunchKernelGGL(k_local_reduce<int64_t>, dim3(grid), dim3(256), 0, st,
                                  static_cast<const int64_t*>(c->scratch), static_cast<int64_t*>(recv), count, g.n, (int)op); break;
    case kF64: hipLaunchKernelGGL(k_local_reduce<double>, dim3(grid), dim3(256), 0, st,
                                  static_cast<const double*>(c->scratch), static_cast<double*>(recv), count, g.n, (int)op); break;
  }
  VN_HIP_CHECK(hipStreamSynchronize(st));
}

void comm_allgather(vn_comm* c, const void* send, void* recv, size_t bytes, hipStream_t st) {
  if (!bytes) return;
  if (c->nccl) {
    nccl_check(rccl().all_gather(send, recv, bytes, 1, c->nccl, st), "ncclAllGather");
    return;
  }
  LocalGroup& g = *c->group;
  if (g.n == 1) {
    if (send != recv) VN_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, st));
    return;
  }
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.send[c->rank] = send;
  g.barrier();
  for (int r = 0; r < g.n; r++)
    VN_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)r * bytes, g.send[r], bytes,
                                hipMemcpyDeviceToDevice, st));
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.barrier();
}

void comm_alltoallv(vn_comm* c, const void* send, const uint64_t* soff, void* recv, const uint64_t* roff,
                    hipStream_t st) {
  const int n = c->nranks, me = c->rank;
  if (c->nccl) {
    const Rccl& R = rccl();
    nccl_check(R.group_start(), "ncclGroupStart");
    for (int p = 0; p < n; p++) {
      const uint64_t sb = soff[p + 1] - soff[p], rb = roff[p + 1] - roff[p];
      if (p == me) {
        if (sb) VN_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + roff[p], static_cast<const char*>(send) + soff[p],
                                            sb, hipMemcpyDeviceToDevice, st));
        continue;
      }
      if (sb) nccl_check(R.send(static_cast<const char*>(send) + soff[p], sb, 1, p, c->nccl, st), "ncclSend");
      if (rb) nccl_check(R.recv(static_cast<char*>(recv) + roff[p], rb, 1, p, c->nccl, st), "ncclRecv");
    }
    nccl_check(R.group_end(), "ncclGroupEnd");
    return;
  }
  LocalGroup& g = *c->group;
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.send[me] = send;
  g.soff[me] = soff;
  g.barrier();
  for (int p = 0; p < n; p++) {
    const uint64_t a = g.soff[p][me], b = g.soff[p][me + 1];
    if (b - a != roff[p + 1] - roff[p]) throw std::runtime_error("alltoallv: send and receive sizes disagree");
    if (b > a)
      VN_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + roff[p], static_cast<const char*>(g.send[p]) + a, b - a,
                                  hipMemcpyDeviceToDevice, st));
  }
  VN_HIP_CHECK(hipStreamSynchronize(st));
  g.barrier();
}

}  // namespace vn

using namespace vn;

extern "C" {

int vn_comm_unique_id(uint8_t* id) {
  if (!id) return VN_EINVAL;
  try {
    NcclId u;
    nccl_check(rccl().get_unique_id(&u), "ncclGetUniqueId");
    std::memcpy(id, u.internal, sizeof(u.internal));
    return VN_OK;
  } catch (const std::exception&) {
    return VN_EHIP;
  }
}

int vn_comm_init(const uint8_t* id, int nranks, int rank, int device, vn_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return VN_EINVAL;
  *out = nullptr;
  vn_comm* c = new vn_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  try {
    VN_HIP_CHECK(hipSetDevice(device));
    VN_HIP_CHECK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    NcclId u;
    std::memcpy(u.internal, id, sizeof(u.internal));
    nccl_check(rccl().comm_init_rank(&c->nccl, nranks, u, rank), "ncclCommInitRank");
  } catch (const HipError& h) {
    c->err = std::string("HIP: ") + hipGetErrorString(h.err);
    *out = c;
    return VN_EHIP;
  } catch (const std::exception& x) {
    c->err = x.what();
    *out = c;
    return VN_EHIP;
  }
  *out = c;
  return VN_OK;
}

int vn_comm_init_local(int nranks, int device, vn_comm** out) {
  if (!out || nranks < 1) return VN_EINVAL;
  auto g = std::make_shared<LocalGroup>(nranks);
  try {
    VN_HIP_CHECK(hipSetDevice(device));
    for (int r = 0; r < nranks; r++) {
      vn_comm* c = new vn_comm();
      c->nranks = nranks;
      c->rank = r;
      c->device = device;
      c->group = g;
      VN_HIP_CHECK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
      out[r] = c;
    }
  } catch (const HipError&) {
    return VN_EHIP;
  }
  return VN_OK;
}

void vn_comm_destroy(vn_comm* c) {
  if (!c) return;
  if (c->st) (void)hipStreamSynchronize(c->st);
  if (c->nccl) (void)rccl().comm_destroy(c->nccl);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

const char* vn_comm_last_error(const vn_comm* c) { return c ? c->err.c_str() : "null comm"; }

int vn_comm_rank(const vn_comm* c) { return c ? c->rank : -1; }
int vn_comm_nranks(const vn_comm* c) { return c ? c->nranks : -1; }

int vn_comm_allreduce(vn_comm* c, const void* send, void* recv, uint64_t count, int dtype, int op) {
  if (!c || dtype < kU8 || dtype > kF64 || op < kSum || op > kMin) return VN_EINVAL;
  try {
    VN_HIP_CHECK(hipSetDevice(c->device));
    comm_allreduce(c, send, recv, count, (DType)dtype, (ROp)op, c->st);
    VN_HIP_CHECK(hipStreamSynchronize(c->st));
    return VN_OK;
  } catch (const HipError& h) {
    c->err = std::string("HIP: ") + hipGetErrorString(h.err);
    return VN_EHIP;
  } catch (const std::exception& x) {
    c->err = x.what();
    return VN_EHIP;
  }
}

}  // extern "C"
