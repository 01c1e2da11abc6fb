// comm.h -- the engine's cross-GPU exchange: one engine per GPU, keys sharded by veneur's worker
// routing (Digest % N, server.go:655), and split (hot) keys combined at flush.
//
// Two transports behind one interface:
//   RCCL   ncclAllReduce / ncclAllGather / grouped ncclSend+ncclRecv on the engine's stream
//          (xGMI).  librccl is opened at vn_comm_init (dlopen, the copy already in the process
//          or the one next to the HIP runtime in use), so the engine library has no link-time
//          dependency on it and a process that never forms a group never loads it.
//   local  an in-process group of engines on one device (tests on a one-GPU box, and the
//          one-rank group of a single engine): each rank's collective runs in its own host
//          thread, meets the others at a barrier and copies device to device.
#pragma once
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/veneur_amd.h"
#include "primitives.h"

namespace vn {

enum DType { kU8 = 0, kU32 = 1, kU64 = 2, kI64 = 3, kF64 = 4 };
enum ROp { kSum = 0, kMax = 1, kMin = 2 };

struct LocalGroup;

}  // namespace vn

struct vn_comm {
  int nranks = 1, rank = 0, device = 0;
  void* nccl = nullptr;                       // ncclComm_t (RCCL transport)
  std::shared_ptr<vn::LocalGroup> group;      // local transport
  hipStream_t st = nullptr;                   // stream of vn_comm_allreduce (control plane)
  void* scratch = nullptr;                    // local transport: gathered operands of a reduction
  size_t scratch_cap = 0;
  std::string err;
};

namespace vn {

size_t dtype_size(DType t);
// recv = op over ranks of send (count elements); send may equal recv
void comm_allreduce(vn_comm* c, const void* send, void* recv, size_t count, DType t, ROp op, hipStream_t st);
// recv = concatenation over ranks of each rank's `bytes` bytes of send
void comm_allgather(vn_comm* c, const void* send, void* recv, size_t bytes, hipStream_t st);
// personalised exchange: this rank sends send[soff[p], soff[p+1]) to rank p and receives rank p's
// part for it into recv[roff[p], roff[p+1]) (byte offsets, host arrays of nranks + 1)
void comm_alltoallv(vn_comm* c, const void* send, const uint64_t* soff, void* recv, const uint64_t* roff,
                    hipStream_t st);

}  // namespace vn
