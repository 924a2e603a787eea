// tcmp_dist_internal.h -- the device-side collectives the shared-tree rounds use
// (tcmp_plan_run_shared, tcmp_engine.hip), implemented over the communicator's RCCL handle in
// tcmp_dist.cpp.  Every call is enqueued on the caller's stream (the engine's), in place on
// device memory, so the rounds stay stream-ordered; world 1 makes each a no-op.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

struct tcmp_comm;

namespace tcmp_dist {

struct Bcast {
  void* ptr;     // the same device address range on every rank (in-place broadcast)
  size_t bytes;
  int root;
};

int rank(const tcmp_comm* c);
int world(const tcmp_comm* c);
int device(const tcmp_comm* c);
// in place: d[0..n) = min over ranks
int allreduce_min_i64(tcmp_comm* c, int64_t* d, int n, hipStream_t s);
// recv[q * n + i] = rank q's send[i]
int allgather_i64(tcmp_comm* c, const int64_t* send, int64_t* recv, int n, hipStream_t s);
// one RCCL group of in-place broadcasts
int bcast_group(tcmp_comm* c, const Bcast* ops, int n_ops, hipStream_t s);

}  // namespace tcmp_dist
