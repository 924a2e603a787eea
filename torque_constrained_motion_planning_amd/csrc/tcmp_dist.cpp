// tcmp_dist.cpp -- the multi-GPU side of libtcmp.so, C-ABI in include/tcmp.h.
//
// Independent planning queries shard over one process per GPU with no data-path collective
// (the reference plans them in a host loop, collect_data.py:74-85).  The only exchange is
// the gather of the solved trajectories to rank 0 at the end of a step: a size all-gather,
// then ncclGroupStart; ncclSend / ncclRecv; ncclGroupEnd over RCCL (xGMI point-to-point
// links, each rank's buffer on its own link into rank 0).  No PyTorch anywhere: rank 0's
// ncclUniqueId reaches the other ranks through a small TCP rendezvous (tcmp_rendezvous, the
// launcher's MASTER_ADDR and a port).  A one-rank job needs no communicator at all: the
// gather is then a local copy, with the same packing, and touches no GPU.
//
// Wire format of one rank's contribution: header int64 [n_local][2] = (query id, rows) and
// body float64 [rows_total][22] = trajectory rows [q(7) qd(7) qdd(7) dt(1)] (shard.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tcmp.h"
#include "tcmp_dist_internal.h"

// tcmp_engine.hip's thread-local error string
extern "C" const char* tcmp_last_error(void);
namespace tcmp_err {
int set(int code, const std::string& msg);
}

namespace {

constexpr int kCols = TCMP_TRAJ_COLS;
constexpr uint64_t kMagic = 0x74636d7064697374ull;  // "tcmpdist"

int fail(int code, const std::string& m) { return tcmp_err::set(code, m); }

#define HIPD(x)                                                                        \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(-2, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCLD(x)                                                                       \
  do {                                                                                 \
    ncclResult_t r_ = (x);                                                             \
    if (r_ != ncclSuccess) return fail(-5, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* p, size_t n, int timeout_ms) {
  char* c = static_cast<char*>(p);
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, timeout_ms) <= 0) return false;
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

struct Hello {
  uint64_t magic;
  uint64_t job;  // job identity: a stale or concurrent job on the same port is turned away
  int32_t rank, world, nbytes, pad;
};

// FNV-1a of the launcher's run id (TCMP_JOB_ID, else TORCHELASTIC_RUN_ID) and the world size
uint64_t job_nonce(int world, int port) {
  const char* id = std::getenv("TCMP_JOB_ID");
  if (!id || !*id) id = std::getenv("TORCHELASTIC_RUN_ID");
  uint64_t x = 1469598103934665603ull;
  auto mix = [&](unsigned char b) { x = (x ^ b) * 1099511628211ull; };
  for (const char* p = id ? id : ""; *p; ++p) mix((unsigned char)*p);
  for (int k = 0; k < 4; ++k) mix((unsigned char)(world >> (8 * k)));
  for (int k = 0; k < 4; ++k) mix((unsigned char)(port >> (8 * k)));
  return x;
}

}  // namespace

struct tcmp_comm {
  int rank = 0, world = 1, device = -1;
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  void* dbuf = nullptr;   // device staging (headers + bodies)
  size_t dcap = 0;
  int stage(size_t bytes) {
    if (bytes <= dcap) return 0;
    if (dbuf) (void)hipFree(dbuf);
    dbuf = nullptr;
    dcap = 0;
    HIPD(hipMalloc(&dbuf, bytes));
    dcap = bytes;
    return 0;
  }
};

namespace tcmp_dist {

int rank(const tcmp_comm* c) { return c->rank; }
int world(const tcmp_comm* c) { return c->world; }
int device(const tcmp_comm* c) { return c->device; }

int RcclExchange::min_i64(int64_t* d, int n, hipStream_t s) {
  if (c_->world == 1 || n <= 0) return 0;
  NCCLD(ncclAllReduce(d, d, (size_t)n, ncclInt64, ncclMin, c_->nccl, s));
  return 0;
}

int RcclExchange::allgather_i64(const int64_t* send, int64_t* recv, int n, hipStream_t s) {
  if (n <= 0) return 0;
  if (c_->world == 1) {
    HIPD(hipMemcpyAsync(recv, send, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    return 0;
  }
  NCCLD(ncclAllGather(send, recv, (size_t)n, ncclInt64, c_->nccl, s));
  return 0;
}

int RcclExchange::bcast(const Bcast* ops, int n_ops, hipStream_t s) {
  if (c_->world == 1 || n_ops <= 0) return 0;
  NCCLD(ncclGroupStart());
  for (int i = 0; i < n_ops; ++i) {
    if (ops[i].bytes == 0) continue;
    const ncclResult_t r = ncclBroadcast(ops[i].ptr, ops[i].ptr, ops[i].bytes, ncclUint8,
                                         ops[i].root, c_->nccl, s);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return fail(-5, std::string("ncclBroadcast: ") + ncclGetErrorString(r));
    }
  }
  NCCLD(ncclGroupEnd());
  return 0;
}

void gather_layout(int world, const int64_t* sizes, int64_t* q_off, int64_t* r_off,
                   int64_t* total_q, int64_t* total_r) {
  int64_t q = 0, r = 0;
  for (int k = 0; k < world; ++k) {
    if (q_off) q_off[k] = q;
    if (r_off) r_off[k] = r;
    q += sizes[2 * k];
    r += sizes[2 * k + 1];
  }
  if (total_q) *total_q = q;
  if (total_r) *total_r = r;
}

}  // namespace tcmp_dist

extern "C" {

int tcmp_rendezvous(int32_t rank, int32_t world, const char* addr, int32_t port, void* blob,
                    int32_t nbytes, int32_t timeout_ms) {
  if (world < 1 || rank < 0 || rank >= world || nbytes < 0 || (nbytes > 0 && !blob) || !addr ||
      port <= 0 || port > 65535)
    return fail(-1, "tcmp_rendezvous: bad arguments");
  if (world == 1) return 0;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  if (::getaddrinfo(addr, ps.c_str(), &hints, &res) != 0 || !res)
    return fail(-1, std::string("tcmp_rendezvous: cannot resolve ") + addr);
  sockaddr_in sa;
  std::memcpy(&sa, res->ai_addr, sizeof(sa));
  ::freeaddrinfo(res);
  const uint64_t job = job_nonce(world, port);
  if (rank == 0) {
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return fail(-1, "tcmp_rendezvous: socket");
    int one = 1;
    ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(ls, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(ls, world) != 0) {
      ::close(ls);
      return fail(-1, "tcmp_rendezvous: cannot listen on " + std::string(addr) + ":" + ps);
    }
    // phase 1: every other rank introduces itself; the connections stay open
    std::vector<int> fds(world, -1);
    int got = 0, rc = 0;
    while (got < world - 1) {
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                           deadline - std::chrono::steady_clock::now()).count();
      pollfd pf{ls, POLLIN, 0};
      if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
        rc = fail(-1, "tcmp_rendezvous: timed out waiting for " + std::to_string(world - 1 - got) +
                          " rank(s)");
        break;
      }
      const int fd = ::accept(ls, nullptr, nullptr);
      if (fd < 0) continue;
      Hello h{};
      if (recv_all(fd, &h, sizeof(h), 5000) && h.magic == kMagic && h.job == job &&
          h.world == world && h.nbytes == nbytes && h.rank > 0 && h.rank < world &&
          fds[h.rank] < 0) {
        fds[h.rank] = fd;
        ++got;
      } else {
        ::close(fd);  // a stranger, a stale job, or a duplicate rank
      }
    }
    ::close(ls);
    // phase 2: the blob goes out only once the whole world has arrived; on a timeout every
    // connection closes unanswered, so every waiting rank fails instead of one part of the
    // job entering the communicator set-up without the others
    for (int r = 1; r < world && !rc; ++r) {
      Hello ack{kMagic, job, 0, world, nbytes, 0};
      if (!send_all(fds[r], &ack, sizeof(ack)) || !send_all(fds[r], blob, (size_t)nbytes))
        rc = fail(-1, "tcmp_rendezvous: lost rank " + std::to_string(r));
    }
    for (int fd : fds)
      if (fd >= 0) ::close(fd);
    return rc;
  }
  // other ranks: connect (rank 0 may not be listening yet), introduce, receive the blob
  while (true) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return fail(-1, "tcmp_rendezvous: socket");
    if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
      Hello h{kMagic, job, rank, world, nbytes, 0}, ack{};
      const bool ok = send_all(fd, &h, sizeof(h)) && recv_all(fd, &ack, sizeof(ack), timeout_ms) &&
                      ack.magic == kMagic && ack.job == job && ack.world == world &&
                      ack.nbytes == nbytes && recv_all(fd, blob, (size_t)nbytes, timeout_ms);
      ::close(fd);
      if (ok) return 0;
      return fail(-1, "tcmp_rendezvous: handshake with rank 0 failed");
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline)
      return fail(-1, "tcmp_rendezvous: cannot reach rank 0 at " + std::string(addr) + ":" + ps);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

int tcmp_dist_init(int32_t rank, int32_t world, int32_t device, const char* addr, int32_t port,
                   tcmp_comm** out) {
  if (!out) return fail(-1, "null out");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return fail(-1, "bad rank / world size");
  tcmp_comm* c = new tcmp_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  if (world > 1) {
    ncclUniqueId id;
    std::memset(&id, 0, sizeof(id));
    int rc = 0;
    if (rank == 0) {
      const ncclResult_t r = ncclGetUniqueId(&id);
      if (r != ncclSuccess) rc = fail(-5, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    }
    rc = rc ? rc : tcmp_rendezvous(rank, world, addr, port, &id, (int)sizeof(id), 300000);
    if (!rc) {
      hipError_t e = hipSetDevice(device);
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
      if (e != hipSuccess) rc = fail(-2, std::string("tcmp_dist_init: ") + hipGetErrorString(e));
    }
    if (!rc) {
      const ncclResult_t r = ncclCommInitRank(&c->nccl, world, id, rank);
      if (r != ncclSuccess) rc = fail(-5, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    if (rc) {
      if (c->stream) (void)hipStreamDestroy(c->stream);
      delete c;
      return rc;
    }
  }
  *out = c;
  return 0;
}

int tcmp_dist_destroy(tcmp_comm* c) {
  if (!c) return 0;
  if (c->nccl) {
    (void)hipSetDevice(c->device);
    (void)ncclCommDestroy(c->nccl);
  }
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int tcmp_dist_allreduce(tcmp_comm* c, double* v, int32_t n, int32_t op) {
  if (!c || n < 0 || (n > 0 && !v) || (op != TCMP_REDUCE_SUM && op != TCMP_REDUCE_MAX))
    return fail(-1, "bad arguments");
  if (c->world == 1 || n == 0) return 0;
  HIPD(hipSetDevice(c->device));
  if (int rc = c->stage((size_t)n * sizeof(double))) return rc;
  double* d = static_cast<double*>(c->dbuf);
  HIPD(hipMemcpyAsync(d, v, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  NCCLD(ncclAllReduce(d, d, (size_t)n, ncclFloat64, op == TCMP_REDUCE_MAX ? ncclMax : ncclSum,
                      c->nccl, c->stream));
  HIPD(hipMemcpyAsync(v, d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPD(hipStreamSynchronize(c->stream));
  return 0;
}

int tcmp_dist_barrier(tcmp_comm* c) {
  if (!c) return fail(-1, "null comm");
  if (c->world == 1) return 0;
  HIPD(hipSetDevice(c->device));
  HIPD(hipDeviceSynchronize());  // every engine stream of this rank has drained
  double one = 1.0;
  return tcmp_dist_allreduce(c, &one, 1, TCMP_REDUCE_SUM);
}

int tcmp_dist_allgather_i64(tcmp_comm* c, const int64_t* in, int32_t n, int64_t* out) {
  if (!c || n < 0 || (n > 0 && (!in || !out))) return fail(-1, "bad arguments");
  if (n == 0) return 0;
  if (c->world == 1) {
    std::memcpy(out, in, (size_t)n * sizeof(int64_t));
    return 0;
  }
  HIPD(hipSetDevice(c->device));
  const size_t w = (size_t)c->world;
  if (int rc = c->stage((w + 1) * n * sizeof(int64_t))) return rc;
  int64_t* d = static_cast<int64_t*>(c->dbuf);
  HIPD(hipMemcpyAsync(d, in, n * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  NCCLD(ncclAllGather(d, d + n, (size_t)n, ncclInt64, c->nccl, c->stream));
  HIPD(hipMemcpyAsync(out, d + n, w * n * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPD(hipStreamSynchronize(c->stream));
  return 0;
}

int tcmp_gather_layout(int32_t world, const int64_t* sizes, int64_t* q_off, int64_t* r_off,
                       int64_t* total_q, int64_t* total_r) {
  if (world < 1 || !sizes) return fail(-1, "bad arguments");
  for (int k = 0; k < 2 * world; ++k)
    if (sizes[k] < 0) return fail(-1, "negative size");
  tcmp_dist::gather_layout(world, sizes, q_off, r_off, total_q, total_r);
  return 0;
}

int tcmp_gather_pack(int32_t n_local, const int64_t* ids, const int64_t* rows, const double* data,
                     int64_t* hdr, double* body) {
  if (n_local < 0 || (n_local > 0 && (!ids || !rows || !hdr))) return fail(-1, "bad arguments");
  int64_t my_rows = 0;
  for (int i = 0; i < n_local; ++i) {
    if (rows[i] < 0) return fail(-1, "negative row count");
    my_rows += rows[i];
  }
  if (my_rows > 0 && (!data || !body)) return fail(-1, "null trajectory rows");
  for (int i = 0; i < n_local; ++i) {
    hdr[2 * i] = ids[i];
    hdr[2 * i + 1] = rows[i];
  }
  if (my_rows && body != data) std::memmove(body, data, (size_t)my_rows * kCols * sizeof(double));
  return 0;
}

int tcmp_gather_unpack(int32_t world, const int64_t* sizes, const int64_t* hdr_all,
                       const double* body_all, int64_t cap_queries, int64_t cap_rows,
                       int64_t* out_ids, int64_t* out_rows, double* out_data, int64_t* n_queries,
                       int64_t* n_rows) {
  if (world < 1 || !sizes || !n_queries || !n_rows) return fail(-1, "bad arguments");
  std::vector<int64_t> q_off((size_t)world), r_off((size_t)world);
  int64_t tq = 0, tr = 0;
  if (int rc = tcmp_gather_layout(world, sizes, q_off.data(), r_off.data(), &tq, &tr)) return rc;
  *n_queries = tq;
  *n_rows = tr;
  if ((tq && !hdr_all) || (tr && !body_all)) return fail(-1, "null staged wire form");
  // every rank's header rows must add up to the rows it announced: a transport that dropped,
  // duplicated or misplaced part of a rank's message fails here, not in the caller's unpacking
  for (int k = 0; k < world; ++k) {
    int64_t s = 0;
    for (int64_t i = 0; i < sizes[2 * k]; ++i) {
      const int64_t r = hdr_all[2 * (q_off[k] + i) + 1];
      if (r < 0) return fail(-6, "rank " + std::to_string(k) + ": negative row count received");
      s += r;
    }
    if (s != sizes[2 * k + 1])
      return fail(-6, "rank " + std::to_string(k) + ": header rows " + std::to_string(s) +
                          " against " + std::to_string(sizes[2 * k + 1]) + " announced");
  }
  if (tq > cap_queries || tr > cap_rows)
    return fail(-4, "gather output capacity too small (need " + std::to_string(tq) + " queries, " +
                        std::to_string(tr) + " rows)");
  if ((tq && (!out_ids || !out_rows)) || (tr && !out_data)) return fail(-1, "null output arrays");
  for (int64_t i = 0; i < tq; ++i) {
    out_ids[i] = hdr_all[2 * i];
    out_rows[i] = hdr_all[2 * i + 1];
  }
  if (tr) std::memcpy(out_data, body_all, (size_t)tr * kCols * sizeof(double));
  return 0;
}

int tcmp_gather_paths(tcmp_comm* c, int32_t n_local, const int64_t* ids, const int64_t* rows,
                      const double* data, const int64_t* sizes_in, int64_t cap_queries,
                      int64_t cap_rows, int64_t* out_ids, int64_t* out_rows, double* out_data,
                      int64_t* n_queries, int64_t* n_rows) {
  if (!c || n_local < 0 || (n_local > 0 && (!ids || !rows)) || !n_queries || !n_rows)
    return fail(-1, "bad arguments");
  int64_t my_rows = 0;
  for (int i = 0; i < n_local; ++i) {
    if (rows[i] < 0) return fail(-1, "negative row count");
    my_rows += rows[i];
  }
  if (my_rows > 0 && !data) return fail(-1, "null trajectory rows");
  // 1. sizes of every rank's contribution (unless the caller already all-gathered them)
  const int W = c->world;
  std::vector<int64_t> sizes(2 * (size_t)W);
  if (sizes_in) {
    std::memcpy(sizes.data(), sizes_in, sizes.size() * sizeof(int64_t));
    if (sizes[2 * c->rank] != n_local || sizes[2 * c->rank + 1] != my_rows)
      return fail(-1, "sizes[rank] does not match this rank's paths");
  } else {
    const int64_t mine[2] = {n_local, my_rows};
    if (int rc = tcmp_dist_allgather_i64(c, mine, 2, sizes.data())) return rc;
  }
  // 2. rank 0's receive layout: each rank's header / body rows in rank order
  std::vector<int64_t> q_off((size_t)W), r_off((size_t)W);
  int64_t tq = 0, tr = 0;
  tcmp_dist::gather_layout(W, sizes.data(), q_off.data(), r_off.data(), &tq, &tr);
  *n_queries = c->rank == 0 ? tq : 0;
  *n_rows = c->rank == 0 ? tr : 0;
  // this rank's wire form (tcmp_gather_pack: the body is the caller's rows as they lie)
  std::vector<int64_t> hdr(2 * (size_t)n_local);
  if (int rc = tcmp_gather_pack(n_local, ids, rows, data, hdr.data(), const_cast<double*>(data)))
    return rc;
  std::vector<int64_t> all_hdr;
  std::vector<double> all_body;
  if (W > 1) {
    HIPD(hipSetDevice(c->device));
    // device staging on rank 0: headers of all ranks, then bodies of all ranks; elsewhere
    // the rank's own header and body
    const size_t hb = (size_t)(c->rank == 0 ? tq : n_local) * 2 * sizeof(int64_t);
    const size_t bb = (size_t)(c->rank == 0 ? tr : my_rows) * kCols * sizeof(double);
    const size_t hpad = (hb + 255) & ~size_t(255);
    if (int rc = c->stage(hpad + bb + 256)) return rc;
    char* base = static_cast<char*>(c->dbuf);
    int64_t* dh = reinterpret_cast<int64_t*>(base);
    double* db = reinterpret_cast<double*>(base + hpad);
    if (n_local)
      HIPD(hipMemcpyAsync(dh, hdr.data(), hdr.size() * sizeof(int64_t), hipMemcpyHostToDevice,
                          c->stream));
    if (my_rows)
      HIPD(hipMemcpyAsync(db, data, (size_t)my_rows * kCols * sizeof(double),
                          hipMemcpyHostToDevice, c->stream));
    NCCLD(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    if (c->rank == 0) {
      for (int k = 1; k < W && r == ncclSuccess; ++k) {
        const int64_t nq = sizes[2 * k], nr = sizes[2 * k + 1];
        if (nq) r = ncclRecv(dh + 2 * q_off[k], (size_t)(2 * nq), ncclInt64, k, c->nccl, c->stream);
        if (nr && r == ncclSuccess)
          r = ncclRecv(db + kCols * r_off[k], (size_t)(kCols * nr), ncclFloat64, k, c->nccl,
                       c->stream);
      }
    } else {
      if (n_local) r = ncclSend(dh, (size_t)(2 * n_local), ncclInt64, 0, c->nccl, c->stream);
      if (my_rows && r == ncclSuccess)
        r = ncclSend(db, (size_t)(kCols * my_rows), ncclFloat64, 0, c->nccl, c->stream);
    }
    // the group is closed on every path, so later RCCL calls on this thread still work
    const ncclResult_t re = ncclGroupEnd();
    if (r != ncclSuccess) return fail(-5, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    if (re != ncclSuccess) return fail(-5, std::string("ncclGroupEnd: ") + ncclGetErrorString(re));
    if (c->rank == 0) {
      all_hdr.resize(2 * (size_t)tq);
      all_body.resize((size_t)tr * kCols);
      if (tq) HIPD(hipMemcpyAsync(all_hdr.data(), dh, all_hdr.size() * sizeof(int64_t),
                                  hipMemcpyDeviceToHost, c->stream));
      if (tr) HIPD(hipMemcpyAsync(all_body.data(), db, all_body.size() * sizeof(double),
                                  hipMemcpyDeviceToHost, c->stream));
    }
    HIPD(hipStreamSynchronize(c->stream));
  } else {
    all_hdr = hdr;
    all_body.assign(data, data + (size_t)my_rows * kCols);
  }
  if (c->rank != 0) return 0;
  // rank 0: every rank's wire form at tcmp_gather_layout's offsets -> the outputs
  return tcmp_gather_unpack(W, sizes.data(), all_hdr.data(), all_body.data(), cap_queries,
                            cap_rows, out_ids, out_rows, out_data, n_queries, n_rows);
}

int tcmp_dist_rccl_ranks(const tcmp_comm* c, int32_t* n) {
  if (!c || !n) return fail(-1, "bad arguments");
  *n = 0;
  if (!c->nccl) return 0;  // a one-rank job has no communicator
  int k = 0;
  NCCLD(ncclCommCount(c->nccl, &k));
  *n = k;
  return 0;
}

int tcmp_dist_rank(const tcmp_comm* c, int32_t* rank, int32_t* world) {
  if (!c || !rank || !world) return fail(-1, "bad arguments");
  *rank = c->rank;
  *world = c->world;
  return 0;
}

}  // extern "C"
