// tcmp_dist_internal.h -- the exchanges of a shared-tree round (tcmp_engine.hip
// shared_rounds) behind one interface, so that every transport runs the same round loop:
//
//  * RcclExchange (tcmp_dist.cpp): one process per GPU, RCCL collectives over the
//    communicator of tcmp_dist_init (tcmp_plan_run_shared);
//  * GroupExchange (tcmp_engine.hip): several engines of one process, one host thread each,
//    meeting at a host barrier and copying device memory peer to peer (tcmp_plan_run_group,
//    which the single-GPU tests drive).
//
// Every call is enqueued on / ordered with the caller's stream (the engine's), in place on
// device memory; world 1 makes each a no-op.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

struct tcmp_comm;

namespace tcmp_dist {

struct Bcast {
  void* ptr;     // the same address range of every rank's own buffers (in-place broadcast)
  size_t bytes;
  int root;
};

class RoundExchange {
 public:
  virtual ~RoundExchange() {}
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // in place: d[0..n) = min over ranks
  virtual int min_i64(int64_t* d, int n, hipStream_t s) = 0;
  // recv[q * n + i] = rank q's send[i]
  virtual int allgather_i64(const int64_t* send, int64_t* recv, int n, hipStream_t s) = 0;
  // every op's range of rank `root` to the same range of every other rank
  virtual int bcast(const Bcast* ops, int n_ops, hipStream_t s) = 0;
};

int rank(const tcmp_comm* c);
int world(const tcmp_comm* c);
int device(const tcmp_comm* c);

// the RCCL transport of a communicator (valid while the communicator lives)
class RcclExchange : public RoundExchange {
 public:
  explicit RcclExchange(tcmp_comm* c) : c_(c) {}
  int rank() const override { return tcmp_dist::rank(c_); }
  int world() const override { return tcmp_dist::world(c_); }
  int min_i64(int64_t* d, int n, hipStream_t s) override;
  int allgather_i64(const int64_t* send, int64_t* recv, int n, hipStream_t s) override;
  int bcast(const Bcast* ops, int n_ops, hipStream_t s) override;

 private:
  tcmp_comm* c_;
};

// Receive layout of tcmp_gather_paths on rank 0 (tcmp_gather_layout in the C-ABI): from the
// all-gathered (queries, rows) per rank, each rank's first header row and first body row in
// the rank-ordered staging buffer, and the totals.
void gather_layout(int world, const int64_t* sizes, int64_t* q_off, int64_t* r_off,
                   int64_t* total_q, int64_t* total_r);

}  // namespace tcmp_dist
