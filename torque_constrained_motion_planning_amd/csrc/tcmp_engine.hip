// tcmp_engine.hip -- MI355X (gfx950) engine for the torque-constrained RRT* hot path and its
// C-ABI (include/tcmp.h).
//
// Reference path replaced: rrt_star.py:151-211 (rrt_star_force_aware) with its callbacks
// utils.py:2985-3218 (sample/distance/extend/collision), panda_primitives.py:13-193,295-318
// (torque tests, dynam_fn), rne.py:198-254, min_jerk_v2.py:80-222.
//
// Round structure (batched frontier, B candidates per round, one HIP stream):
//   k_sample        Philox4x32-10 candidate draws (or host-provided draws)
//   nearest         per-round radix-tree cell index of the snapshot (tcmp_nn.h) and the
//                   pruned exact scan k_nearest_wave32 (tcmp_nn32.h); tcmp_nearest runs
//                   the same index and scan over a caller's tree
//   k_edges         persistent lane-refill edge walker: extend steps, collision, torque
//   k_ins_*         lane-ordered insertion (device-wide scan), goal test (tcmp_insert.h)
//   k_rewire_scan   neighbours within radius of each new node (snapshot)
//   k_rewire_apply  sequential rewire per new node (rrt_star.py:187-192)
// then k_retrace / k_traj (min-jerk + final dynamic torque validation).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tcmp_device.h"
#include "../../include/tcmp.h"
#include "tcmp_dist_internal.h"

using namespace tcmp;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Process-wide dispatch lock.  Every C-ABI entry point that touches a device holds it shared
// (reentrant per thread: nested entries take it once); a round-graph capture (tcmp_plan_run)
// holds it exclusively from hipStreamBeginCapture through the graph's instantiation and first
// launch, so no other engine's thread enqueues, allocates, frees or synchronizes while a graph
// is captured or instantiated.  Writer-preferring: a waiting capture blocks new entries, so
// engines kept busy back to back from several threads (bench.py --pipeline, C4) cannot starve
// it.  Entry points never wait on one another while holding it (only on their own streams).
class DispatchLock {
 public:
  void lock_shared() {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return !writer_ && waiting_ == 0; });
    ++readers_;
  }
  void unlock_shared() {
    std::lock_guard<std::mutex> lk(m_);
    if (--readers_ == 0) cv_.notify_all();
  }
  void lock() {
    std::unique_lock<std::mutex> lk(m_);
    ++waiting_;
    cv_.wait(lk, [&] { return !writer_ && readers_ == 0; });
    --waiting_;
    writer_ = true;
  }
  void unlock() {
    std::lock_guard<std::mutex> lk(m_);
    writer_ = false;
    cv_.notify_all();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int readers_ = 0, waiting_ = 0;
  bool writer_ = false;
};
DispatchLock g_dispatch;
thread_local int t_entry_depth = 0;
thread_local bool t_capturing = false;  // DBuf::ensure refuses to allocate while set

struct Entry {
  Entry() {
    if (t_entry_depth++ == 0) g_dispatch.lock_shared();
  }
  ~Entry() {
    if (--t_entry_depth == 0) g_dispatch.unlock_shared();
  }
  Entry(const Entry&) = delete;
  Entry& operator=(const Entry&) = delete;
};

// exclusive for a capture: the thread's shared hold (an Entry is live) is traded for the
// exclusive one and given back at the end of the scope
struct CaptureScope {
  CaptureScope() {
    g_dispatch.unlock_shared();
    g_dispatch.lock();
    t_capturing = true;
  }
  ~CaptureScope() {
    t_capturing = false;
    g_dispatch.unlock();
    g_dispatch.lock_shared();
  }
  CaptureScope(const CaptureScope&) = delete;
  CaptureScope& operator=(const CaptureScope&) = delete;
};

}  // namespace

#define TCMP_ENTER(h)          \
  Entry tcmp_entry_;           \
  if (int rc_ = set_dev(h)) return rc_

// error channel shared with tcmp_dist.cpp (same thread-local message)
namespace tcmp_err {
int set(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace tcmp_err

namespace {

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail(-2, std::string(#x) + ": " + hipGetErrorString(e_));                 \
  } while (0)

constexpr int kNbrCap = 8;     // stored rewire neighbours per flagged new node
constexpr int kNnTile = 256;   // snapshot nodes per LDS tile of k_rewire_scan

struct DevState {
  long long n_nodes;
  long long snap;
  long long new_count;
  long long goal_node;
  long long samples;
  long long W, ni, K, first_fail;
  unsigned long long edge_steps, pairs_tested, pairs_sat, pairs_exact, nn_pairs, rewires;
  unsigned long long nn_box_tests;
  unsigned long long rewire_steps;   // the rewire edges' share of edge_steps (k_rewire_apply)
  unsigned long long snap_sum;       // sum over rounds of the snapshot size T_r
  unsigned long long nn_full_pairs;  // sum over rounds of T_r * B_r (brute-force-equivalent)
  long long ins_total;   // accepted edges of the current round (k_ins_scan), this engine's lanes
  long long ins_off;     // where this engine's new nodes start after the snapshot (0 alone;
                         // the lower ranks' accepted edges in a shared-tree round)
  long long ins_all;     // accepted edges of the round over all ranks (ins_total alone)
  long long ins_goal;    // lowest goal-reaching new node of the round (k_ins_write)
  double goal_cost;      // the goal node's cost and depth (k_retrace)
  long long goal_depth;
  int work_counter;
  int nn_counter;
  int round_goal;
  int rw_count;
  int status;
  int overflow;
  int nn_queue[8];       // per-XCD work queues of k_nearest_wave32
  int nn_cells;          // cells of the current nearest-neighbour index (k_nn_starts)
  int nn_supers;         // super-cells of the index
  unsigned long long prof[16];  // TCMP_PROF builds: k_edges clock breakdown + exact-test stats
  unsigned long long prof_nn[8]; // TCMP_PROF builds: nearest-scan clocks [0..4] and visit counts [5..7]
};

struct PlanParams {
  double start[7], goal[7], w[7], res[7];
  double radius, goal_prob, goal_tol, mass, exec_time;
  double nn_cmax;  // bound on |q| of nodes and candidates (fp32 error terms of tcmp_nn32.h)
  unsigned long long seed;
  int torque_mode;
  int uniform_w;
  long long max_nodes;
};

struct Tree {
  double* cfg;     // [N][8]: q0..q6, cost
  int* parent;     // [N]
  double* tgt;     // [N][8]: extend target q0..q6
  int2* meta;      // [N]: (n_steps, n_safe)
};

__device__ __forceinline__ void load7(const double* p, double q[7]) {
  const double4 a = *reinterpret_cast<const double4*>(p);
  const double2 b = *reinterpret_cast<const double2*>(p + 4);
  q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w; q[4] = b.x; q[5] = b.y; q[6] = p[6];
}
__device__ __forceinline__ void store7(double* p, const double q[7]) {
#pragma unroll
  for (int k = 0; k < 7; ++k) p[k] = q[k];
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// ------------------------------------------------------------------------------------------
// k_sample: uniform configurations (utils.py:2941-2990 convex_combination of the limits)
// ------------------------------------------------------------------------------------------
// (lane j of the round; the fused multi-plan rounds of tcmp_fleet.h call the same body)
__device__ __forceinline__ void sample_lane(const PlanParams* __restrict__ Pd, DevState* st,
                                            long long base, int nb, double* cand,
                                            unsigned char* cgoal, int j) {
  const PlanParams P = *Pd;
  if (j >= nb) return;
  const long long it = base + j;
  double u[8];
  philox_uniforms(P.seed, (uint64_t)it, u);
  {
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < 7; ++k) cand[8 * (size_t)j + k] = (1 - u[k]) * kLo[k] + u[k] * kHi[k];
  }
  cgoal[j] = 0;
  if (st->goal_node >= 0) return;  // goal reached: no goal-biased lane (round_goal stays INT_MAX)
  // The round's lowest selecting lane.  Every wave first evaluates the selection of lanes
  // 0..63 (their Philox draws, one per lane): one of them selects with probability
  // 1 - (1 - goal_prob)^64, and then that is the answer -- one plain store, instead of 4,096
  // waves' atomics on one address (~40 us per round).  Otherwise each wave adds its lowest
  // selecting lane with one atomic.
  const int lane = lane_id();
  double v[8];
  philox_uniforms(P.seed, (uint64_t)(base + lane), v);
  const uint64_t m0 = __ballot(lane < nb && (base + lane == 0 || v[7] < P.goal_prob));
  if (m0) {
    if (j == 0) st->round_goal = __builtin_ctzll(m0);
    return;
  }
  const bool raw = it == 0 || u[7] < P.goal_prob;
  const uint64_t m = __ballot(raw);
  if (m && lane == __builtin_ctzll(m)) atomicMin(&st->round_goal, j);
}
__global__ void k_sample(const PlanParams* __restrict__ Pd, DevState* st, long long base, int nb,
                         double* cand, unsigned char* cgoal) {
  sample_lane(Pd, st, base, nb, cand, cgoal, blockIdx.x * blockDim.x + threadIdx.x);
}

// ------------------------------------------------------------------------------------------
// k_goal_fix: the round's goal-biased lane takes the goal configuration (rrt_star.py:160-161)
// ------------------------------------------------------------------------------------------
// Done by the first kernel of the round's nearest search (k_node_keys or k_nn_root), which
// runs after k_sample has chosen the lane and before anything reads the candidates.
struct GoalFix {
  double* cand;          // null: no fix (host-supplied samples, tcmp_nearest)
  unsigned char* cgoal;
};
__device__ __forceinline__ void goal_fix(const PlanParams* __restrict__ Pd, DevState* st,
                                         GoalFix gf, int nb) {
  const int j = st->round_goal;
  if (gf.cand && j < nb) {
#pragma unroll
    for (int k = 0; k < 7; ++k) gf.cand[8 * (size_t)j + k] = Pd->goal[k];
    gf.cgoal[j] = 1;
  }
}

// ------------------------------------------------------------------------------------------
// Morton keys of snapshot nodes and candidates for the nearest-neighbour index (tcmp_nn.h):
// 9 bits per joint over the joint limits, interleaved, and only the top kKeyBits kept --
// 2^36 cells leave at most a handful of nodes per cell, and the radix sorts run 5 digit
// passes instead of 8.
// ------------------------------------------------------------------------------------------
#ifndef TCMP_KEY_BITS
#define TCMP_KEY_BITS 36
#endif
constexpr int kKeyBits = TCMP_KEY_BITS;
// rocprim picks a block-sort + merge-sort chain (~15 launches) below 1M items by default;
// the Onesweep radix sort (one histogram pass + one launch per 8-bit digit) is faster here
using OnesweepCfg = rocprim::default_config;
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           OnesweepCfg, 16384>;

__device__ __forceinline__ unsigned long long morton7(const double q[7]) {
  unsigned u[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    double t = (q[k] - kLo[k]) / (kHi[k] - kLo[k]);
    t = fmin(fmax(t, 0.0), 1.0);
    u[k] = (unsigned)(t * 511.0);
  }
  unsigned long long key = 0;
#pragma unroll
  for (int b = 8; b >= 0; --b)
#pragma unroll
    for (int k = 0; k < 7; ++k) key = (key << 1) | ((u[k] >> b) & 1u);
  return key;
}

__global__ void k_node_keys(DevState* st, const double* cfg, long long T_bound,
                            unsigned long long* keys, int* vals, const PlanParams* __restrict__ Pd,
                            GoalFix gf, int nb) {
  if (blockIdx.x == 0 && threadIdx.x == 0) goal_fix(Pd, st, gf, nb);
  const long long T = st->n_nodes;
  for (long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x; n < T_bound;
       n += (long long)gridDim.x * blockDim.x) {
    // the largest key: the stable sort puts these nodes (indices >= T) after every real one,
    // and nothing reads the sorted keys past T
    unsigned long long key = (1ull << kKeyBits) - 1;
    if (n < T) {
      double q[7];
      load7(cfg + 8 * n, q);
      key = morton7(q) >> (63 - kKeyBits);
    }
    keys[n] = key;
    vals[n] = (int)n;
  }
}

// vals: the candidate's index for the radix sort, or (cbits > 0) its top-cbits key bin for the
// counting sort
__global__ void k_cand_keys(const double* cand, int nb, unsigned long long* keys, int* vals,
                            int cbits, int* hist) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nb) return;
  double q[7];
  load7(cand + 8 * (size_t)j, q);
  const unsigned long long k = morton7(q) >> (63 - kKeyBits);
  keys[j] = k;
  if (cbits > 0) {
    const int b = (int)(k >> (kKeyBits - cbits));
    vals[j] = b;
    atomicAdd(&hist[b], 1);  // the counting sort's histogram
  } else {
    vals[j] = j;
  }
}


// ---- counting sort of n items by a small integer bin: perm lists the items bin by bin.  Used
// for the longest-first edge order, which only serves load balance -- every result is
// independent of the order -- so items within a bin keep whatever order the atomics give them.  Three launches and no memset: the scan
// leaves the histogram zeroed for the next sort (it is zeroed once when allocated).
constexpr int kCsLdsBins = 1024;  // up to this many bins, per-block LDS histograms
__global__ __launch_bounds__(256) void k_cs_hist(const int* bin, int n, int nbins, int* hist) {
  __shared__ int lh[kCsLdsBins];
  const bool lds = nbins <= kCsLdsBins;
  if (lds) {
    for (int b = threadIdx.x; b < nbins; b += 256) lh[b] = 0;
    __syncthreads();
  }
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    if (lds) atomicAdd(&lh[bin[i]], 1);
    else atomicAdd(&hist[bin[i]], 1);
  }
  if (lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += 256)
      if (lh[b]) atomicAdd(&hist[b], lh[b]);
  }
}
// one block: hoff = exclusive scan of hist, hist zeroed
__device__ __forceinline__ void cs_scan_block(int* hist, int nbins, int* hoff) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (nbins + 1023) / 1024, b0 = t * per, b1 = min(nbins, b0 + per);
  int sum = 0;
  for (int b = b0; b < b1; ++b) sum += hist[b];
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int x = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int b = b0; b < b1; ++b) {
    const int c = hist[b];
    hoff[b] = run;
    run += c;
    hist[b] = 0;
  }
}
__global__ __launch_bounds__(1024) void k_cs_scan(int* hist, int nbins, int* hoff) {
  cs_scan_block(hist, nbins, hoff);
}
// perm[hoff[bin] + rank] = item; with few bins each block reserves its range per bin once
__device__ __forceinline__ void cs_scatter_block(const int* bin, int n, int nbins, int* hoff,
                                                 int* perm, int blk) {
  __shared__ int lc[kCsLdsBins];
  const bool lds = nbins <= kCsLdsBins;
  const int i = blk * 256 + threadIdx.x;
  const int b = i < n ? bin[i] : 0;
  if (!lds) {
    if (i < n) perm[atomicAdd(&hoff[b], 1)] = i;
    return;
  }
  for (int k = threadIdx.x; k < nbins; k += 256) lc[k] = 0;
  __syncthreads();
  const int r = i < n ? atomicAdd(&lc[b], 1) : 0;
  __syncthreads();
  for (int k = threadIdx.x; k < nbins; k += 256)
    if (lc[k]) lc[k] = atomicAdd(&hoff[k], lc[k]);
  __syncthreads();
  if (i < n) perm[lc[b] + r] = i;
}
__global__ __launch_bounds__(256) void k_cs_scatter(const int* bin, int n, int nbins, int* hoff,
                                                    int* perm) {
  cs_scatter_block(bin, n, nbins, hoff, perm, blockIdx.x);
}

#include "tcmp_nn.h"
#include "tcmp_nn32.h"
#include "tcmp_insert.h"
#include "tcmp_ik.h"
#include "tcmp_base.h"

// ------------------------------------------------------------------------------------------
// k_edges: safe_path_force_aware(extend(from, to)) for n edges (rrt_star.py:90-98).
// Persistent: each lane walks one edge step by step; a lane whose edge ends (first failing
// step or last step) takes the next edge from a global queue (one atomic per wave), so
// lanes never idle behind the longest edge of their wave.
// ------------------------------------------------------------------------------------------
struct EdgeJob {
  const double* from_base;  // stride 8
  const int* from_idx;      // nullable: from = from_base[from_idx[e]]
  const double* to;         // stride 8
  int n;
  int* nsafe;
  int* nsteps;
  double* last;             // stride 8
  const int* order;         // nullable: the k-th edge taken is order[k] (longest first)
  int* accepted;            // nullable: accepted edges (nsafe > 0) per 256 edges, cleared before
  double* rec;              // the k-th edge taken, as k_edges fetches it (k_edge_records): its
                            // from-configuration q0..q6 and (edge index, planned steps) packed
                            // in the 8th double -- one 64-B load per fetch
};

// The work records k_edges' lanes fetch (launch_edges runs this first): record k = the edge
// taken k-th (order[k], or k), its from-configuration (from_base[from_idx[e]] or from_base[e])
// and its planned step count num_steps(from, to[e]) (utils.py:3072).  A fetch is then one
// dependent load after the work counter, where it was three (order, from_idx, the rows) and a
// num_steps on the wave-step that fetched.
__device__ __forceinline__ void edge_record(const EdgeJob& J, const PlanParams* __restrict__ Pd,
                                            int k) {
  if (k >= J.n) return;
  const int e = J.order ? J.order[k] : k;
  const long long src = J.from_idx ? (long long)J.from_idx[e] : (long long)e;
  double a[7], b[7], res[7];
  load7(J.from_base + 8 * src, a);
  load7(J.to + 8 * (size_t)e, b);
#pragma unroll
  for (int j = 0; j < 7; ++j) res[j] = Pd->res[j];
  const int n = num_steps(a, b, res);
  double* r = J.rec + 8 * (size_t)k;
  *reinterpret_cast<double4*>(r) = make_double4(a[0], a[1], a[2], a[3]);
  *reinterpret_cast<double4*>(r + 4) = make_double4(a[4], a[5], a[6], __hiloint2double(n, e));
}
__global__ __launch_bounds__(256) void k_edge_records(EdgeJob J, const PlanParams* __restrict__ Pd) {
  edge_record(J, Pd, blockIdx.x * 256 + threadIdx.x);
}

#ifndef TCMP_EDGE_SPLIT
#define TCMP_EDGE_SPLIT 4  // small rounds: up to this many lanes per edge (k_edges SPLIT)
#endif
#ifndef TCMP_EDGE_MINW
#define TCMP_EDGE_MINW 2  // min waves per SIMD the register allocation must allow
#endif
// SPLIT = 2 or 4 (rounds with at most a half / a quarter of the resident lanes' edges, e.g.
// C2's 65,536 and 34,464): SPLIT adjacent lanes share an edge and check SPLIT consecutive
// steps at a time -- lane k of the group step i + k, its configuration reached by the same
// k + 1 refine steps (so the same bits) -- and the edge advances past the passing prefix and
// ends at the first failing step, exactly the sequential walk's result; the checks past a
// failure are wasted only in an edge's last iteration.  The counted extend steps are the
// sequential walk's (nsafe + 1 on a failure, else n).

template <bool MESH, int SPLIT>
__global__ __launch_bounds__(256, TCMP_EDGE_MINW) void k_edges(EdgeJob J, const PlanParams* __restrict__ Pd, Scene sc_g, Geo g_g,
                                               DevState* st) {
  const PlanParams P = *Pd;
  extern __shared__ double tcmp_lds[];
  Scene sc;
  Geo g;
  stage_lds<!MESH>(sc_g, g_g, tcmp_lds, sc, g);
  const int lane = lane_id();
  const int sub = lane & (SPLIT - 1);  // position in the lane group of an edge
  int e = -1, i = 0, n = 0;
  bool done = false;
  double q[7];  // last safe configuration of the lane's edge (the target is re-read per step)
#pragma unroll
  for (int k = 0; k < 7; ++k) q[k] = 0.5 * (kLo[k] + kHi[k]);
  StepStats ss = {};
  unsigned steps = 0;  // extend steps: the wave's (SPLIT == 1, uniform) or this lane's
#ifdef TCMP_PROF
  unsigned long long c_total = 0, c_fetch = 0, c_coll = 0, c_torque = 0, c_tail = 0, c_sincos = 0;
  const unsigned long long c_start = clock64();
#endif
  while (true) {
#ifdef TCMP_PROF
    unsigned long long c0 = clock64();
#endif
    const bool need = !done && e < 0;
    const uint64_t m = __ballot(need && sub == 0);
    if (m) {
      const int leader = __builtin_ctzll(m);
      int base = 0;
      if (lane == leader) base = atomicAdd(&st->work_counter, (int)__popcll(m));
      base = __shfl(base, leader);
      if (need) {
        // (the other lanes of a group take its first lane's slot: all hold the same edge)
        const int my = base + (int)__popcll(m & ((1ull << (lane - sub)) - 1ull));
        if (my < J.n) {
          // the edge's record (k_edge_records): from-configuration, edge index, planned steps
          const double4 ra = *reinterpret_cast<const double4*>(J.rec + 8 * (size_t)my);
          const double4 rb = *reinterpret_cast<const double4*>(J.rec + 8 * (size_t)my + 4);
          q[0] = ra.x; q[1] = ra.y; q[2] = ra.z; q[3] = ra.w;
          q[4] = rb.x; q[5] = rb.y; q[6] = rb.z;
          e = __double2loint(rb.w);
          n = __double2hiint(rb.w);
          i = 0;
        } else {
          done = true;
        }
      }
    }
    if (__ballot(!done) == 0) break;
#ifdef TCMP_PROF
    { const unsigned long long c1 = clock64(); c_fetch += c1 - c0; c0 = c1; }
#endif
    // lane k of a group checks step i + k (none past the edge's last step)
    const bool active = e >= 0 && (SPLIT == 1 || i + sub < n);
    // The step's configuration qn, its sin/cos and the torque test come first; during the
    // collision check only q (the last safe configuration) and cq/sq stay live -- the target
    // q2 is re-read from memory and qn regenerated (the same arithmetic, so the same bits)
    // afterwards, which keeps the check's register peak below the spill point.
    bool tok = true, lim = false;
    double cq[7], sq[7];
    {
      double qn[7], q2[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) qn[k] = q[k];
      if (active) {
        load7(J.to + 8 * (size_t)e, q2);
        refine_step(qn, q2, n, i);
        for (int k = 1; k <= sub; ++k) refine_step(qn, q2, n, i + k);
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) sincos(qn[k], &sq[k], &cq[k]);
      lim = active && limits_violated(qn);
    }
#ifdef TCMP_PROF
    { const unsigned long long c1 = clock64(); c_sincos += c1 - c0; c0 = c1; }
#endif
    // torque test (panda_primitives.py:155-193) -- independent of the collision result, so
    // its order against the collision check does not matter (rrt_star.py:93-96)
    if (active && !lim && P.torque_mode != TCMP_TORQUE_BASE) {
      const double z[7] = {0, 0, 0, 0, 0, 0, 0};
      tok = P.torque_mode == TCMP_TORQUE_DYN ? torque_ok_dyn<false>(cq, sq, z, z, P.mass)
                                             : torque_ok<false>(cq, sq, z, z, P.mass);
    }
#ifdef TCMP_PROF
    { const unsigned long long c1 = clock64(); c_torque += c1 - c0; c0 = c1; }
#endif
    // lanes already failing (limits or torque) need no obstacle pairs
    // every lane calls it (wave-cooperative); lanes already failing only ride along
    const bool coll = collides_wave<MESH>(cq, sq, active && !lim && tok, sc, g, ss) || lim;
#ifdef TCMP_PROF
    { const unsigned long long c1 = clock64(); c_coll += c1 - c0; c0 = c1; }
#endif
    const bool ok = active && !coll && tok;
    if (SPLIT == 1) {
      steps += (unsigned)__popcll(__ballot(active));  // wave total
      if (active) {
        if (ok) {
          double q2[7];
          load7(J.to + 8 * (size_t)e, q2);
          refine_step(q, q2, n, i);
          ++i;
        }
        if (!ok || i == n) {
          if (J.accepted && i > 0) atomicAdd(&J.accepted[e >> 8], 1);
          J.nsafe[e] = i;
          J.nsteps[e] = n;
          store7(J.last + 8 * (size_t)e, q);
          e = -1;
        }
      }
    } else {
      // the group's verdicts: it advances past its passing prefix (all lanes reach the ballot)
      const uint64_t okm = __ballot(ok);
      const unsigned gb = (unsigned)(okm >> (lane - sub)) & ((1u << SPLIT) - 1u);
      if (e >= 0) {
        const int na = min(SPLIT, n - i);               // steps the group checked
        const int adv = min(__builtin_ctz(~gb), na);    // passing prefix
        if (adv) {
          double q2[7];
          load7(J.to + 8 * (size_t)e, q2);
          for (int k = 0; k < adv; ++k) refine_step(q, q2, n, i + k);
          i += adv;
        }
        const bool failed = adv < na;
        if (failed || i == n) {
          if (sub == 0) {
            steps += (unsigned)(failed ? i + 1 : n);
            if (J.accepted && i > 0) atomicAdd(&J.accepted[e >> 8], 1);
            J.nsafe[e] = i;
            J.nsteps[e] = n;
            store7(J.last + 8 * (size_t)e, q);
          }
          e = -1;
        }
      }
    }
#ifdef TCMP_PROF
    c_tail += clock64() - c0;
#endif
  }
  // steps: a wave total for SPLIT == 1, per group leader otherwise; ss: wave totals
  const unsigned long long a = SPLIT == 1 ? (unsigned long long)steps
                                          : wave_sum_u64((unsigned long long)steps),
                           b = 10ull * (unsigned long long)sc_g.n_obs * ss.live_steps,
                           c = ss.pairs_sat, d = ss.pairs_exact;
  if (lane == 0) {
    atomicAdd(&st->edge_steps, a);
    atomicAdd(&st->pairs_tested, b);
    atomicAdd(&st->pairs_sat, c);
    atomicAdd(&st->pairs_exact, d);
#ifdef TCMP_PROF
    c_total = clock64() - c_start;
    atomicAdd(&st->prof[0], c_total);
    atomicAdd(&st->prof[1], c_fetch);
    atomicAdd(&st->prof[2], c_coll);
    atomicAdd(&st->prof[3], c_torque);
    atomicAdd(&st->prof[4], c_tail);
    atomicAdd(&st->prof[5], ss.cyc_exact);
    atomicAdd(&st->prof[6], c_sincos);
    atomicAdd(&st->prof[7], ss.cyc_t123);
#endif
  }
}

// ------------------------------------------------------------------------------------------
// rewire (rrt_star.py:183-192): neighbours of each new node within `radius` among the
// round's snapshot, visited in index order; reparent when cheaper and the edge is safe.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void rewire_scan_block(const PlanParams* __restrict__ Pd, DevState* st,
                                                  const Tree& tr, const int* rwlist, int* nbr,
                                                  int* ncount, int blk) {
  const PlanParams P = *Pd;
  // neighbours within `radius` of each flagged new node among the snapshot, in index order
  // (the order rrt_star.py:187 visits them); the snapshot streams through LDS tiles
  __shared__ double4 tile[2 * kNnTile];
  const int tid = threadIdx.x;
  const long long R = st->rw_count, T = st->snap;
  if ((long long)blk * 256 >= R) return;  // block-uniform
  const long long t = (long long)blk * 256 + tid;
  const bool act = t < R;
  double qn[7];
  if (act) load7(tr.cfg + 8 * (long long)rwlist[t], qn);
  else for (int k = 0; k < 7; ++k) qn[k] = 1e30;
  const double r2 = P.radius * P.radius;
  int c = 0;
  const double4* t4 = reinterpret_cast<const double4*>(tr.cfg);
  for (long long base = 0; base < T; base += kNnTile) {
    const long long n = base + tid;
    if (n < T) {
      tile[2 * tid] = t4[2 * n];
      tile[2 * tid + 1] = t4[2 * n + 1];
    }
    __syncthreads();
    const int cnt = (int)min((long long)kNnTile, T - base);
    for (int jj = 0; jj < cnt; ++jj) {
      const double4 a = tile[2 * jj], b = tile[2 * jj + 1];
      const double d0 = qn[0] - a.x, d1 = qn[1] - a.y, d2 = qn[2] - a.z, d3 = qn[3] - a.w,
                   d4 = qn[4] - b.x, d5 = qn[5] - b.y, d6 = qn[6] - b.z;
      double dd = P.w[0] * (d0 * d0);
      dd = fma(P.w[1] * d1, d1, dd); dd = fma(P.w[2] * d2, d2, dd); dd = fma(P.w[3] * d3, d3, dd);
      dd = fma(P.w[4] * d4, d4, dd); dd = fma(P.w[5] * d5, d5, dd); dd = fma(P.w[6] * d6, d6, dd);
      if (dd < r2 * 1.000001) {
        const double nq[7] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z};
        if (distance(nq, qn, P.w) < P.radius) {
          if (c < kNbrCap) nbr[t * kNbrCap + c] = (int)(base + jj);
          ++c;
        }
      }
    }
    __syncthreads();
  }
  if (act) ncount[t] = c;
}
__global__ __launch_bounds__(256) void k_rewire_scan(const PlanParams* __restrict__ Pd, DevState* st, Tree tr,
                                                     const int* rwlist, int* nbr, int* ncount) {
  rewire_scan_block(Pd, st, tr, rwlist, nbr, ncount, blockIdx.x);
}

template <bool MESH>
__device__ __forceinline__ void rewire_apply_block(const PlanParams* __restrict__ Pd, DevState* st,
                                                   const Tree& tr, const int* rwlist,
                                                   const int* nbr, const int* ncount,
                                                   const Scene& sc_g, const Geo& g_g, int blk) {
  const PlanParams P = *Pd;
  extern __shared__ double tcmp_lds[];
  Scene sc;
  Geo g;
  stage_lds<!MESH>(sc_g, g_g, tcmp_lds, sc, g);
  const long long R = st->rw_count, T = st->snap;
  const long long t = (long long)blk * blockDim.x + threadIdx.x;
  const bool act = t < R && ncount[t] > 0;
  if (__ballot(act) == 0) return;  // wave-uniform
  const long long me = act ? rwlist[t] : 0;
  double qn[7];
  double cost_new = 0;
  int cnt = 0;
  if (act) {
    load7(tr.cfg + 8 * me, qn);
    cost_new = tr.cfg[8 * me + 7];
    cnt = ncount[t];
  } else {
    for (int k = 0; k < 7; ++k) qn[k] = 0.5 * (kLo[k] + kHi[k]);
  }
  StepStats ss = {0, 0, 0};
  int c = 0;
  int prev = -1;
  unsigned long long rew = 0;
  unsigned steps = 0;  // extend steps of the rewire edges (counted like k_edges')
  while (true) {
    // next neighbour in index order (stored list, then a serial rescan past the list)
    int nidx = -1;
    if (act && c < cnt) {
      if (c < kNbrCap) {
        nidx = nbr[t * kNbrCap + c];
      } else {
        for (long long n = prev + 1; n < T; ++n) {
          double a[7];
          load7(tr.cfg + 8 * n, a);
          if (distance(a, qn, P.w) < P.radius) { nidx = (int)n; break; }
        }
      }
    }
    if (__ballot(nidx >= 0) == 0) break;
    ++c;
    if (nidx >= 0) prev = nidx;
    double qs[7];
    double d = 0, cn = 0;
    bool alive = false;
    int ns = 0, i = 0;
    if (nidx >= 0) {
      load7(tr.cfg + 8 * (size_t)nidx, qs);
      cn = tr.cfg[8 * (size_t)nidx + 7];
      d = distance(qs, qn, P.w);
      alive = cn + d < cost_new;
      ns = num_steps(qs, qn, P.res);
    } else {
      for (int k = 0; k < 7; ++k) qs[k] = qn[k];
    }
    const bool cond = alive;
    double q[7];
    for (int k = 0; k < 7; ++k) q[k] = qs[k];
    while (__ballot(alive)) {
      double qq[7];
      for (int k = 0; k < 7; ++k) qq[k] = q[k];
      if (alive) refine_step(qq, qn, ns, i);
      double cq[7], sq[7];
      for (int k = 0; k < 7; ++k) sincos(qq[k], &sq[k], &cq[k]);
      const bool lim = alive && limits_violated(qq);
      const bool coll = collides_wave<MESH>(cq, sq, alive && !lim, sc, g, ss) || lim;
      bool ok = alive && !coll;
      if (ok && P.torque_mode != TCMP_TORQUE_BASE) {
        const double z[7] = {0, 0, 0, 0, 0, 0, 0};
        ok = P.torque_mode == TCMP_TORQUE_DYN ? torque_ok_dyn<false>(cq, sq, z, z, P.mass)
                                              : torque_ok<false>(cq, sq, z, z, P.mass);
      }
      if (alive) {
        ++steps;
        if (ok) {
          for (int k = 0; k < 7; ++k) q[k] = qq[k];
          ++i;
          if (i == ns) alive = false;
        } else {
          alive = false;
        }
      }
    }
    if (cond && i > 0 && distance(qn, q, P.w) < 1e-6) {
      // new.rewire(n, d, path[:-1]) (rrt_star.py:192, 47-58)
      cost_new = cn + d;
      tr.cfg[8 * me + 7] = cost_new;
      tr.parent[me] = nidx;
      store7(tr.tgt + 8 * me, qn);
      tr.meta[me] = make_int2(ns, i);
      ++rew;
    }
  }
  const unsigned long long r = wave_sum_u64(rew), sn = wave_sum_u64((unsigned long long)steps);
  if (lane_id() == 0 && r) atomicAdd(&st->rewires, r);
  if (lane_id() == 0 && sn) {
    atomicAdd(&st->edge_steps, sn);
    atomicAdd(&st->rewire_steps, sn);
  }
}
template <bool MESH>
__global__ __launch_bounds__(256) void k_rewire_apply(const PlanParams* __restrict__ Pd, DevState* st, Tree tr,
                                                      const int* rwlist, const int* nbr,
                                                      const int* ncount, Scene sc_g, Geo g_g) {
  rewire_apply_block<MESH>(Pd, st, tr, rwlist, nbr, ncount, sc_g, g_g, blockIdx.x);
}

// ------------------------------------------------------------------------------------------
// peak microbenchmarks (tcmp_microbench): kMbAcc independent FMA chains per thread (fp64, and
// packed fp32 = v_pk_fma_f32, the form the spec's 157.3 TF counts), and a float4 HBM copy
// ------------------------------------------------------------------------------------------
constexpr int kMbAcc = 16;
__global__ __launch_bounds__(256) void k_mb_fp64(double* out, int iters) {
  double acc[kMbAcc];
  const double x = 1.0 + 1e-9 * threadIdx.x, y = 1e-7;
#pragma unroll
  for (int k = 0; k < kMbAcc; ++k) acc[k] = 1.0 + k * 1e-3;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < kMbAcc; ++k) acc[k] = fma(acc[k], x, -y);
  double s = 0;
#pragma unroll
  for (int k = 0; k < kMbAcc; ++k) s += acc[k];
  if (s == 12345.678) out[0] = s;  // keeps the chains alive, never true
}
__global__ __launch_bounds__(256) void k_mb_fp32(double* out, int iters) {
  f32x2 acc[kMbAcc];
  const f32x2 x = {1.0f + 1e-7f * threadIdx.x, 1.0f - 1e-7f * threadIdx.x}, y = {1e-6f, 2e-6f};
#pragma unroll
  for (int k = 0; k < kMbAcc; ++k) acc[k] = f32x2{1.0f + k * 1e-3f, 1.0f - k * 1e-3f};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int k = 0; k < kMbAcc; ++k) acc[k] = __builtin_elementwise_fma(acc[k], x, -y);
  float s = 0;
#pragma unroll
  for (int k = 0; k < kMbAcc; ++k) s += acc[k].x + acc[k].y;
  if (s == 12345.678f) out[0] = s;
}
// one pass, no grid stride: each thread moves V float4 (all loads in flight before the stores,
// consecutive lanes on consecutive 16 B: 1 KiB per wave-instruction), the stores nontemporal
// (streamed past the caches); n a multiple of 256 * V.  tcmp_microbench reports the best of
// V = 2, 4, 8 and of the persistent form below.
template <int kMbCopyV>
__global__ __launch_bounds__(256) void k_mb_copy(const float4* __restrict__ src, float4* __restrict__ dst,
                                                 long long n) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4* s = reinterpret_cast<const f32x4*>(src);
  f32x4* d = reinterpret_cast<f32x4*>(dst);
  const long long base = (long long)blockIdx.x * (256 * kMbCopyV) + threadIdx.x;
  f32x4 v[kMbCopyV];
#pragma unroll
  for (int k = 0; k < kMbCopyV; ++k) v[k] = s[base + 256 * k];
#pragma unroll
  for (int k = 0; k < kMbCopyV; ++k) __builtin_nontemporal_store(v[k], &d[base + 256 * k]);
}
// persistent form: a grid of a few blocks per CU strides over the buffer, V float4 per thread
// per pass, nontemporal stores (and loads, NTL)
template <int kMbCopyV, bool NTL>
__global__ __launch_bounds__(256) void k_mb_copy_gs(const float4* __restrict__ src,
                                                    float4* __restrict__ dst, long long n) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4* s = reinterpret_cast<const f32x4*>(src);
  f32x4* d = reinterpret_cast<f32x4*>(dst);
  const long long step = (long long)gridDim.x * (256 * kMbCopyV);
  for (long long base = (long long)blockIdx.x * (256 * kMbCopyV) + threadIdx.x; base < n;
       base += step) {
    f32x4 v[kMbCopyV];
#pragma unroll
    for (int k = 0; k < kMbCopyV; ++k)
      v[k] = NTL ? __builtin_nontemporal_load(&s[base + 256 * k]) : s[base + 256 * k];
#pragma unroll
    for (int k = 0; k < kMbCopyV; ++k) __builtin_nontemporal_store(v[k], &d[base + 256 * k]);
  }
}

// ------------------------------------------------------------------------------------------
// tree digest (tcmp_plan_digest): sum over nodes i of mix(i, cfg bits, cost bits, parent) mod
// 2^64 -- order-independent, so one reduction; two trees have the same digest iff (up to a
// 2^-64 collision) every node's record is the same.  mix = splitmix64 chained over the words.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__global__ __launch_bounds__(256) void k_tree_digest(const DevState* st, const double* cfg,
                                                     const int* parent, unsigned long long* out) {
  const long long T = st->n_nodes;
  unsigned long long acc = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < T; i += (long long)gridDim.x * 256) {
    unsigned long long x = splitmix64((unsigned long long)i);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      x = splitmix64(x ^ (unsigned long long)__double_as_longlong(cfg[8 * i + k]));
    x = splitmix64(x ^ (unsigned long long)(unsigned)parent[i]);
    acc += x;
  }
  acc = wave_sum_u64(acc);
  if (lane_id() == 0 && acc) atomicAdd(out, acc);
}

// ------------------------------------------------------------------------------------------
// retrace (rrt_star.py:42-45, 202): [start] + for each edge root->goal the first n_safe-1
// regenerated extend points + the node's configuration.  One block.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_retrace(const PlanParams* __restrict__ Pd, DevState* st, Tree tr,
                                                 long long* chain, double* wp, long long wp_cap) {
  const PlanParams P = *Pd;
  __shared__ long long sL;
  __shared__ long long part[256];
  const int tid = threadIdx.x;
  const long long goal = st->goal_node;
  if (goal < 0) return;
  if (tid == 0) {
    long long L = 0;
    const long long cap = st->n_nodes;
    for (long long n = goal; n > 0 && L < cap; n = tr.parent[n]) chain[L++] = n;
    sL = L;
    st->goal_cost = tr.cfg[8 * goal + 7];
    st->goal_depth = L;
  }
  __syncthreads();
  const long long L = sL;
  long long run = 1;  // waypoint 0 = start
  for (long long b0 = 0; b0 < L; b0 += 256) {
    const long long k = b0 + tid;  // root->goal order
    long long node = -1;
    long long cnt = 0;
    if (k < L) {
      node = chain[L - 1 - k];
      cnt = tr.meta[node].y;
    }
    part[tid] = cnt;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const long long v = tid >= o ? part[tid - o] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    const long long off = run + part[tid] - cnt;
    if (node >= 0 && off + cnt <= wp_cap) {
      double q[7], tq[7];
      load7(tr.cfg + 8 * (size_t)tr.parent[node], q);
      load7(tr.tgt + 8 * node, tq);
      const int2 mt = tr.meta[node];
      for (int i = 0; i < mt.y - 1; ++i) {
        refine_step(q, tq, mt.x, i);
        store7(wp + 7 * (off + i), q);
      }
      double qn[7];
      load7(tr.cfg + 8 * node, qn);
      store7(wp + 7 * (off + mt.y - 1), qn);
    }
    run += part[255];
    __syncthreads();
  }
  if (tid == 0) {
    double q0[7];
    load7(tr.cfg, q0);
    store7(wp, q0);
    st->W = run;
    if (run > wp_cap) { st->status = -3; return; }
    // dynam_fn: num_intervals = move_time * 1000 / len(path) (panda_primitives.py:308)
    const long long ni = (long long)(P.exec_time * 1000.0 / (double)run);
    st->ni = ni;
    st->K = ni > 0 ? (run - 1) * ni : 0;
    st->first_fail = -1;
    if (ni <= 0) st->status = TCMP_PLAN_MINJERK_ASSERT;
  }
}

// ------------------------------------------------------------------------------------------
// min-jerk sample i of a waypoint path (min_jerk_v2.py:80-222 with unit durations)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double gv_at(const double* wp, long long nseg, long long s, int k) {
  // goal velocity of segment s (waypoint s+1), min_jerk_v2.py:109-118
#pragma clang fp contract(off)
  if (s >= nseg - 1) return 0.0;
  const double v0 = (wp[7 * (s + 1) + k] - wp[7 * s + k]) / 1.0;
  const double v1 = (wp[7 * (s + 2) + k] - wp[7 * (s + 1) + k]) / 1.0;
  return (v0 * v1 >= 1e-10) ? 0.5 * (v0 + v1) : 0.0;
}

__device__ __forceinline__ void minjerk_sample(const double* wp, long long nwp, long long ni,
                                               long long i, double x[7], double v[7],
                                               double a[7]) {
#pragma clang fp contract(off)
  const long long nseg = nwp - 1;
  const long long s = i / ni, j = i % ni;
  const double interval = 1.0 / (double)ni;
  double t;
  if (ni > 1) {
    const double step = (1.0 - interval) / (double)(ni - 1);
    t = (j == ni - 1) ? 1.0 : ((double)j * step + interval);
  } else {
    t = 0.0 * (1.0 - interval) + interval;
  }
  const double t2 = pow(t, 2.0), t3 = pow(t, 3.0), t4 = pow(t, 4.0), t5 = pow(t, 5.0);
  const double T = 1.0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double x0 = wp[7 * s + k];
    const double v0 = s > 0 ? gv_at(wp, nseg, s - 1, k) : 0.0;
    const double a0 = 0.0;
    const double gx = wp[7 * (s + 1) + k];
    const double gv = gv_at(wp, nseg, s, k);
    const double ga = 0.0;
    const double A = (gx - (x0 + v0 * T + (a0 / 2.0) * T * T)) / (T * T * T);
    const double B = (gv - (v0 + a0 * T)) / (T * T);
    const double C = (ga - a0) / T;
    const double c0 = x0, c1 = v0, c2 = a0 / 2.0;
    const double c3 = 10 * A - 4 * B + 0.5 * C;
    const double c4 = (-15 * A + 7 * B - C) / T;
    const double c5 = (6 * A - 3 * B + 0.5 * C) / (T * T);
    x[k] = c0 + c1 * t + c2 * t2 + c3 * t3 + c4 * t4 + c5 * t5;
    v[k] = c1 + 2 * c2 * t + 3 * c3 * t2 + 4 * c4 * t3 + 5 * c5 * t4;
    a[k] = 2 * c2 + 6 * c3 * t + 12 * c4 * t2 + 20 * c5 * t3;
  }
}

// the planner's torque test on one sample (mode fixed per kernel instantiation), from cos /
// sin of q computed once by the caller
template <int MODE>
__device__ __forceinline__ bool torque_test_m(double mass, const double cq[7], const double sq[7],
                                              const double qd[7], const double qdd[7]) {
  if constexpr (MODE == TCMP_TORQUE_BASE) return true;
  if constexpr (MODE == TCMP_TORQUE_NOV) {
    const double z[7] = {0, 0, 0, 0, 0, 0, 0};
    return torque_ok<false>(cq, sq, z, z, mass);
  }
  if constexpr (MODE == TCMP_TORQUE_DYN) return torque_ok_dyn<true>(cq, sq, qd, qdd, mass);
  return torque_ok<true>(cq, sq, qd, qdd, mass);
}
__device__ __forceinline__ void sincos7(const double q[7], double cq[7], double sq[7]) {
#pragma unroll
  for (int k = 0; k < 7; ++k) sincos(q[k], &sq[k], &cq[k]);
}
// a kernel template instantiated per torque mode, picked on the host
#define TCMP_BY_MODE(K, mode) \
  ((mode) == TCMP_TORQUE_BASE ? K<TCMP_TORQUE_BASE> : (mode) == TCMP_TORQUE_NOV ? K<TCMP_TORQUE_NOV> \
   : (mode) == TCMP_TORQUE_DYN ? K<TCMP_TORQUE_DYN> : K<TCMP_TORQUE_RNE>)

// dynam_fn + final validation for the planner's path, one row per thread; Conf.torques follow
// in k_traj_tau (one RNE per kernel keeps both at two waves per SIMD)
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == 3 ? 1 : 2))) void k_traj(const PlanParams* __restrict__ Pd, DevState* st, const double* wp,
                       double* oq, double* oqd, double* oqdd, double* opsg, long long kcap) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (st->goal_node < 0) return;
  if (st->status != 0 && st->status != TCMP_PLAN_VALIDATION_FAILED) return;
  const long long K = st->K, ni = st->ni, W = st->W;
  if (K > kcap || i >= K) return;  // K > kcap: the host grows the rows and launches again
  const double exec_time = Pd->exec_time, mass = Pd->mass;
  double x[7], v[7], a[7];
  minjerk_sample(wp, W, ni, i, x, v, a);
  store7(oq + 7 * i, x);
  store7(oqd + 7 * i, v);
  store7(oqdd + 7 * i, a);
  {
#pragma clang fp contract(off)
    opsg[i] = (exec_time * (double)i) / (double)K;  // panda_primitives.py:315
  }
  double cq[7], sq[7];
  sincos7(x, cq, sq);
  if (!torque_test_m<MODE>(mass, cq, sq, v, a)) atomicMin(&st->first_fail, i);
}

// Conf.torques of the path's rows: rne without payload (utils.py:3376)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void k_traj_tau(const DevState* st, const double* q, const double* qd,
                           const double* qdd, double* otau, long long kcap) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (st->goal_node < 0) return;
  if (st->status != 0 && st->status != TCMP_PLAN_VALIDATION_FAILED) return;
  const long long K = st->K;
  if (K > kcap || i >= K) return;
  double x[7], v[7], a[7], cq[7], sq[7], tau[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) x[k] = q[7 * i + k];
  sincos7(x, cq, sq);
  // the rates are loaded after the sin / cos (shorter live ranges: no spill)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    v[k] = qd[7 * i + k];
    a[k] = qdd[7 * i + k];
  }
  rne<true>(cq, sq, v, a, 0.0, tau);
  store7(otau + 7 * i, tau);
}

// first_fail uses LLONG_MAX as "none" during the kernel
__global__ void k_traj_prep(DevState* st) {
  if (st->goal_node >= 0 && st->status == 0) st->first_fail = LLONG_MAX;
}
__global__ void k_traj_post(DevState* st) {
  if (st->goal_node < 0) return;
  if (st->first_fail == LLONG_MAX) st->first_fail = -1;
  else if (st->status == 0 && st->first_fail >= 0) st->status = TCMP_PLAN_VALIDATION_FAILED;
}

// ------------------------------------------------------------------------------------------
// utility kernels behind the batched C-ABI entry points
// ------------------------------------------------------------------------------------------
// collision_fn (limits, then every moving link); no_limits: the links only (body-level check)
template <bool MESH>
__global__ __launch_bounds__(256) void k_check_configs(const double* q, long long n, Scene sc_g,
                                                       Geo g_g, int* collides, int no_limits) {
  extern __shared__ double tcmp_lds[];
  Scene sc;
  Geo g;
  stage_lds<!MESH>(sc_g, g_g, tcmp_lds, sc, g);
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  double x[7];
  if (act) load7(q + 8 * i, x);
  else for (int k = 0; k < 7; ++k) x[k] = 0.5 * (kLo[k] + kHi[k]);
  double cq[7], sq[7];
  for (int k = 0; k < 7; ++k) sincos(x[k], &sq[k], &cq[k]);
  StepStats ss = {0, 0, 0};
  const bool lim = act && !no_limits && limits_violated(x);
  const bool c = collides_wave<MESH>(cq, sq, act && !lim, sc, g, ss) || lim;
  if (act) collides[i] = c ? 1 : 0;
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == 3 ? 1 : 2))) void k_torque(const double* q, const double* qd, const double* qdd, long long n,
                         double mass, int* ok) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x[7], v[7], a[7], cq[7], sq[7];
  load7(q + 8 * i, x);
  if (qd) load7(qd + 8 * i, v); else for (int k = 0; k < 7; ++k) v[k] = 0;
  if (qdd) load7(qdd + 8 * i, a); else for (int k = 0; k < 7; ++k) a[k] = 0;
  sincos7(x, cq, sq);
  ok[i] = torque_test_m<MODE>(mass, cq, sq, v, a) ? 1 : 0;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_rne(const double* q, const double* qd, const double* qdd, long long n,
                      double mp, double* tau) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x[7], v[7], a[7], cq[7], sq[7], t[7];
  load7(q + 8 * i, x);
  load7(qd + 8 * i, v);
  load7(qdd + 8 * i, a);
  for (int k = 0; k < 7; ++k) sincos(x[k], &sq[k], &cq[k]);
  rne<true>(cq, sq, v, a, mp > 0 ? mp : 0.0, t);
  store7(tau + 7 * i, t);
}

__global__ void k_minjerk(const double* wp, long long nwp, long long ni, double* oq, double* oqd,
                          double* oqdd) {
  const long long K = (nwp - 1) * ni;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < K;
       i += (long long)gridDim.x * blockDim.x) {
    double x[7], v[7], a[7];
    minjerk_sample(wp, nwp, ni, i, x, v, a);
    store7(oq + 7 * i, x);
    store7(oqd + 7 * i, v);
    store7(oqdd + 7 * i, a);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == 3 ? 1 : 2))) void k_validate(const double* q, const double* qd, const double* qdd, long long n,
                           double mass, unsigned long long* first_fail) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x[7], v[7], a[7], cq[7], sq[7];
  load7(q + 8 * i, x);
  load7(qd + 8 * i, v);
  load7(qdd + 8 * i, a);
  sincos7(x, cq, sq);
  if (!torque_test_m<MODE>(mass, cq, sq, v, a)) atomicMin(first_fail, (unsigned long long)i);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  int ensure(size_t want) {
    if (want <= n) return 0;
    // a captured graph must not bake in a buffer freed under it, and hipFree / hipMalloc
    // synchronize the device: the capture is abandoned and the rounds run directly
    if (t_capturing) return fail(-2, "buffer growth during a round-graph capture");
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T));
    if (e != hipSuccess) return fail(-2, std::string("hipMalloc: ") + hipGetErrorString(e));
    n = want;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// F_NNSCAN times the k_nearest_wave launch alone (inside F_NEAREST, not added to totals)
// F_EDGE_PREP: the edge order's counting sort and k_edge_records, so that F_EDGES times
// k_edges alone (its roofline divides by that time)
enum Fam { F_NEAREST = 0, F_EDGES, F_INSERT, F_REWIRE, F_FINISH, F_NNSCAN, F_EDGE_PREP, F_COUNT };

// one family's span between two recorded events; adjacent families share the boundary event
// (one record per boundary: each record is an event node of ~5 us in a round graph)
struct EventPair {
  hipEvent_t a, b;
  int fam;
};

// A captured sequence of device-sampled rounds (tcmp_plan_run) -- replayed with one
// hipGraphLaunch instead of ~45 launches per round.  Kernels read the plan parameters and
// state from device memory, so a graph serves every query of the same shape; `key` covers
// the shape (first sample index, samples, batch) and every buffer, scene and kernel choice
// baked into the nodes.
struct RoundGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  std::vector<EventPair> events;
  std::vector<hipEvent_t> owned;  // the events its nodes record (destroyed with the graph)
  unsigned long long key = 0;
  int rounds = 0;
  int scans = 0;
};

}  // namespace

struct tcmp_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  int cu_count = 0;
  DBuf<double> verts, planes, edges;
  DBuf<double> obs;
  DBuf<float> obs32;
  DBuf<float> verts32, planes32;
  DBuf<unsigned short> eidx;
  int n_obs = 0;
  // scene on the host: boxes (tcmp_set_scene) and convex meshes (tcmp_set_meshes); the device
  // obstacle list is the boxes followed by the meshes' outer boxes
  std::vector<double> box15;
  int n_box = 0, n_mesh = 0;
  int self_coll = 0;  // tcmp_set_self_collision: link hulls appended as meshes n_mesh + j
  bool mesh_kernels() const { return n_mesh > 0 || self_coll; }
  std::vector<double> mesh_v, mesh_p, mesh_box;
  std::vector<int> mesh_e, mesh_voff, mesh_poff, mesh_eoff;
  DBuf<int> mrange;
  std::vector<int> mrange_h;
  DBuf<double> mib, mv64, mp64, me64;
  DBuf<double> base_geo;  // panda_link0 hull (tcmp_base.h), uploaded on first use
  DBuf<double> base_pd;
  DBuf<float> mv32, mp32, me32;
  DBuf<float> lv32[2], lp32[2], le32[2];      // mesh LOD hulls (inner, outer), world frame
  DBuf<float> mcl, lcl[2];                    // Gauss-map clusters of me32 / le32 (gauss_clusters)
  // host copies of the user meshes' LOD hulls (tcmp_set_mesh_lods; cleared by tcmp_set_meshes)
  bool user_lods = false;
  std::vector<double> lod_v[2], lod_p[2];
  std::vector<int> lod_e[2], lod_vo[2], lod_po[2], lod_eo[2];
  DBuf<float> lodv3[2], lodpl[2];             // link LOD hulls (panda_lod.inc), link frames
  DBuf<unsigned short> lodei[2];
  DBuf<float> lodev[2], geo_ev;               // link hull edge vectors (fp64 -> fp32)
  // inscribed spheres (certificates): rows [0, 10 * TCMP_NSPH) the links' (panda_spheres.inc,
  // link frames), then TCMP_NSPH per mesh (tcmp_set_mesh_spheres; link meshes: the links' own)
  bool user_sph = false;
  bool use_sph = true;  // TCMP_SPHERES=0 turns the certificate off (A/B)
  std::vector<double> sph_h;
  DBuf<float> sph;
  DevState* st = nullptr;
  // plan: parameters on the host and their device copies (kernels read dP, so a captured
  // round graph replays for any query of the same shape); dPx for the standalone entry points
  PlanParams P{};
  PlanParams* dP = nullptr;
  PlanParams* dPx = nullptr;
  bool plan_open = false;
  int max_batch = 0;
  DBuf<double> cfg, tgt;
  DBuf<int> parent;
  DBuf<int2> meta;
  DBuf<double> cand, last;
  DBuf<double> erec;  // k_edges' work records (k_edge_records), one per edge of a round
  DBuf<unsigned char> cgoal;
  DBuf<int> nn, nsafe, nsteps, nbr, ncount, rwlist;
  DBuf<double> nnscore;  // the last round's best exact score per candidate (tcmp_plan_debug_round)
  int last_nb = 0;
  // Morton-chunked snapshot
  DBuf<unsigned long long> nkeys_in, skeys, ckeys_in, ckeys;
  DBuf<int> nvals_in, svals, cvals_in, cperm;
  DBuf<double> stree, cbox;
  DBuf<float> srow;  // the scan's first-pass node rows (32 B per node; tcmp_nn.h k_nn_rows)
  DBuf<float> cboxf, sboxf, bboxf;
  DBuf<int> chome, bcount, boff;
  DBuf<int> cflag, cid, cstart, sflag, sid, sstart;
  DBuf<unsigned long long> ckey;
  DBuf<unsigned char> sort_tmp;
  DevState* st_nn = nullptr;  // state of tcmp_nearest's standalone index (keeps a plan's intact)
  int nn_waves_per_cu = (kNnBlock / 64) * TCMP_NN_MINB;  // the scan's resident waves per CU
  hipEvent_t ins_ev = nullptr;     // open F_INSERT mark between round_search and round_finish
  DBuf<long long> xch;             // shared-tree round exchange slots (k_sr_*)
  DBuf<int> cs_hist, cs_hoff;      // counting-sort histogram (kept zeroed) and bin offsets
  // pinned host staging of a plan's begin / finish (async copies, one host wait per call)
  struct Pin {
    double sg[16];     // start, goal rows of 8
    double root[8];
    int m1;
    int2 z;
    int coll[2];
    DevState st;
    PlanParams P;
  };
  Pin* pin = nullptr;
  DBuf<unsigned char> dpin;     // the Pin block's device copy (plan_begin: one upload)
  size_t fin_W = 0, fin_K = 0;  // the finished plan's waypoint / trajectory rows (plan_fetch)
  long long kcap = 0;           // trajectory rows allocated at plan_begin (exec_time * 1000 + 2)
  int nn_cand_bits = 16;           // top key bits the candidates are sorted by
  int nn_cand_count_bits = 12;     // > 0: a counting sort by that many top bits instead (0: the radix sort)
  DBuf<double> second;
  DBuf<long long> chain;
  DBuf<double> wp, tq, tqd, tqdd, tpsg, ttau;
  long long samples_issued = 0;
  // generic scratch
  DBuf<double> s0, s1, s2, s3;
  DBuf<int> i0, i1, i2;
  DBuf<unsigned long long> u0;
  // timing
  std::vector<EventPair> ev_used;   // spans to read at the next collect_events
  std::vector<hipEvent_t> ev_rec;   // pool events recorded since (returned to the pool there)
  std::vector<hipEvent_t> ev_pool;
  RoundGraph rg;
  bool use_graphs = true;          // TCMP_GRAPHS=0 disables; a failed capture disables
  bool capturing = false;
  int graph_failures = 0;          // captures abandoned (two: launch directly from then on)
  long long graph_launches = 0;    // round-graph launches of the open plan
  // per-family event timing (tcmp_plan_result.ms_*); tcmp_set_timing(h, 0) records no events,
  // so a captured round graph then holds kernel nodes only
  bool timing = true;
  double ms[F_COUNT] = {};
  long long launches_nearest = 0;
  long long launches_scan = 0;      // k_nearest_wave32 launches of the open plan
  int edge_blocks = 0;
  // fused multi-plan rounds (tcmp_plan_run_fused, tcmp_fleet.h) led by this engine: the plan
  // descriptors (FleetPlan[K], FleetNN[K]), each plan's first row in the fleet's node index,
  // and the event the other engines' streams wait on.  The fleet's index lives in this
  // engine's index buffers and st_nn.
  DBuf<unsigned char> f_desc;
  DBuf<long long> f_off;
  std::vector<unsigned char> f_host;
  hipEvent_t dep_ev = nullptr;
  int fused_plans = 0;  // plans of the fused rounds the open plan grew in (0: none)
  // pinned host staging of the scene's records (upload_scene: no host wait; the buffer is
  // reused once the event of its last copy has passed)
  void* scene_pin = nullptr;
  size_t scene_pin_n = 0;
  hipEvent_t scene_ev = nullptr;
  // pinned staging of a finished plan's trajectory rows (tcmp_plan_fetch: DMA copies instead of
  // blit kernels through pageable memory), sized at plan_begin for kcap rows
  void* fetch_pin = nullptr;
  size_t fetch_pin_n = 0;
  int edge_split = 4;  // most lanes per edge in small rounds (environment TCMP_EDGE_SPLIT=1/2/4)
  int edge_wps = 2;    // k_edges' persistent grid, blocks per CU (environment TCMP_EDGE_WPS=1/2)

  Geo geo() const {
    return Geo{verts.p, planes.p, edges.p, verts32.p,
               reinterpret_cast<const float4*>(planes32.p),
               reinterpret_cast<const ushort4*>(eidx.p)};
  }
  Scene scene() const {
    Scene s{};
    s.obs = obs.p;
    s.n_obs = n_obs;
    s.obs32 = obs32.p;
    s.mrange = mrange.p;
    s.mib = mib.p;
    s.mv64 = reinterpret_cast<const double4*>(mv64.p);
    s.mv32 = reinterpret_cast<const float4*>(mv32.p);
    s.mp64 = reinterpret_cast<const double4*>(mp64.p);
    s.mp32 = reinterpret_cast<const float4*>(mp32.p);
    s.me64 = me64.p;
    s.me32 = me32.p;
    s.mcl = reinterpret_cast<const float4*>(mcl.p);
    for (int i = 0; i < 2; ++i) {
      s.lv32[i] = reinterpret_cast<const float4*>(lv32[i].p);
      s.lp32[i] = reinterpret_cast<const float4*>(lp32[i].p);
      s.le32[i] = le32[i].p;
      s.lcl[i] = reinterpret_cast<const float4*>(lcl[i].p);
      s.lodv3[i] = lodv3[i].p;
      s.lodpl[i] = reinterpret_cast<const float4*>(lodpl[i].p);
      s.lodei[i] = reinterpret_cast<const ushort4*>(lodei[i].p);
      s.lodev[i] = reinterpret_cast<const float4*>(lodev[i].p);
    }
    s.geo_ev = reinterpret_cast<const float4*>(geo_ev.p);
    s.sph = reinterpret_cast<const float4*>(sph.p);
    s.n_mesh = n_mesh;
    s.self_coll = self_coll;
    return s;
  }

  hipEvent_t get_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  // during a capture the records become external event nodes of the graph (timestamps on
  // every replay) and the events belong to the graph
  void record(hipEvent_t e) {
    if (capturing) (void)hipEventRecordWithFlags(e, stream, hipEventRecordExternal);
    else (void)hipEventRecord(e, stream);
  }
  hipEvent_t mark() {
    if (!timing) return nullptr;
    hipEvent_t e = capturing ? new_event() : get_event();
    record(e);
    (capturing ? rg.owned : ev_rec).push_back(e);
    return e;
  }
  void span(int fam, hipEvent_t a, hipEvent_t b) {
    if (!a || !b) return;  // timing off (tcmp_set_timing)
    (capturing ? rg.events : ev_used).push_back(EventPair{a, b, fam});
  }
  void mark_begin(int fam, hipEvent_t* out) {
    *out = mark();
    (void)fam;
  }
  // ends family fam at a new event and returns it (the next family's begin, if adjacent)
  hipEvent_t mark_end(int fam, hipEvent_t a) {
    const hipEvent_t b = mark();
    span(fam, a, b);
    return b;
  }
  hipEvent_t new_event() {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void collect_events() {
    for (auto& p : ev_used) {
      float t = 0;
      if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) ms[p.fam] += t;
    }
    ev_used.clear();
    for (auto e : ev_rec) ev_pool.push_back(e);
    ev_rec.clear();
  }
  void drop_graph() {
    if (rg.exec) (void)hipGraphExecDestroy(rg.exec);
    if (rg.graph) (void)hipGraphDestroy(rg.graph);
    for (auto e : rg.owned) (void)hipEventDestroy(e);
    rg = RoundGraph{};
  }
};

namespace {

int set_dev(tcmp_handle* h) {
  if (!h) return fail(-1, "null handle");
  HIPCHK(hipSetDevice(h->device));
  return 0;
}

// A host wait on the handle's stream.  It lets go of the dispatch lock while it waits (the
// thread holds it once, shared, whatever its entry depth), so a round-graph capture on another
// engine waits only for the other threads' enqueues, never for their queries to finish: with
// several queries in flight, a capture would otherwise drain the GPU (bench.py --pipeline).
int sync_stream(tcmp_handle* h) {
  const bool held = t_entry_depth > 0 && !t_capturing;
  if (held) g_dispatch.unlock_shared();
  const hipError_t e = hipStreamSynchronize(h->stream);
  if (held) g_dispatch.lock_shared();
  if (e != hipSuccess) return fail(-2, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  return 0;
}

// host rows of 7 -> device rows of 8
int upload7(tcmp_handle* h, DBuf<double>& buf, const double* src, long long n) {
  int rc = buf.ensure((size_t)n * 8);
  if (rc) return rc;
  std::vector<double> tmp((size_t)n * 8, 0.0);
  for (long long i = 0; i < n; ++i)
    for (int k = 0; k < 7; ++k) tmp[8 * i + k] = src[7 * i + k];
  HIPCHK(hipMemcpyAsync(buf.p, tmp.data(), tmp.size() * sizeof(double), hipMemcpyHostToDevice,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

unsigned lds_bytes(const tcmp_handle* h) {
  return h->mesh_kernels() ? stage_lds_bytes_lean(h->n_obs) : stage_lds_bytes(h->n_obs);
}

unsigned grid_for(long long n, int block) { return (unsigned)std::max<long long>(1, (n + block - 1) / block); }

// Index buffers for trees of up to N nodes and up to B candidates per scan, plus the sort
// and scan temporaries they need (shared by the plan's rounds and tcmp_nearest: nothing in
// them outlives one index build + scan).
// hist_done: the bins' producer already added them to h->cs_hist (ensure_index sized it)
int count_sort(tcmp_handle* h, const int* bin, int n, int nbins, int* perm, bool hist_done = false) {
  if (n <= 0) return 0;
  if ((size_t)nbins > h->cs_hist.n) {
    if (hist_done) return fail(-1, "counting sort histogram too small");
    if (int rc = h->cs_hist.ensure((size_t)nbins)) return rc;
    if (int rc = h->cs_hoff.ensure((size_t)nbins)) return rc;
    HIPCHK(hipMemsetAsync(h->cs_hist.p, 0, h->cs_hist.n * sizeof(int), h->stream));
  }
  if (!hist_done)
    hipLaunchKernelGGL(k_cs_hist, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, bin, n, nbins,
                       h->cs_hist.p);
  hipLaunchKernelGGL(k_cs_scan, dim3(1), dim3(1024), 0, h->stream, h->cs_hist.p, nbins,
                     h->cs_hoff.p);
  hipLaunchKernelGGL(k_cs_scatter, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, bin, n, nbins,
                     h->cs_hoff.p, perm);
  HIPCHK(hipGetLastError());
  return 0;
}

int ensure_index(tcmp_handle* h, size_t N, size_t B) {
  int rc = h->nkeys_in.ensure(N);
  rc = rc ? rc : h->skeys.ensure(N);
  rc = rc ? rc : h->nvals_in.ensure(N);
  rc = rc ? rc : h->svals.ensure(N);
  rc = rc ? rc : h->stree.ensure(N * 8);
  rc = rc ? rc : h->srow.ensure(N * 8);
  rc = rc ? rc : h->cboxf.ensure((N + 1) * 16);  // worst case: one cell per node
  rc = rc ? rc : h->sboxf.ensure((N + 1) * 16);
  rc = rc ? rc : h->bboxf.ensure((N / 64 + 2) * 16);
  rc = rc ? rc : h->cflag.ensure(N);
  rc = rc ? rc : h->cid.ensure(N);
  rc = rc ? rc : h->cstart.ensure(N + 1);
  rc = rc ? rc : h->sflag.ensure(N);
  rc = rc ? rc : h->sid.ensure(N);
  rc = rc ? rc : h->sstart.ensure(N + 1);
  rc = rc ? rc : h->ckey.ensure(N);
  rc = rc ? rc : h->chome.ensure(2 * B);
  rc = rc ? rc : h->ckeys_in.ensure(B);
  rc = rc ? rc : h->cvals_in.ensure(B);
  rc = rc ? rc : h->cperm.ensure(B);
  if (rc) return rc;
  if (h->cs_hist.n < 65536) {  // the counting sorts' histogram, zeroed once (self-cleaning)
    rc = h->cs_hist.ensure(65536);
    rc = rc ? rc : h->cs_hoff.ensure(65536);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(h->cs_hist.p, 0, h->cs_hist.n * sizeof(int), h->stream));
  }
  rc = h->ckeys.ensure(B);
  if (rc) return rc;
  size_t t1 = 0, t2 = 0, t3 = 0;
  HIPCHK(rocprim::radix_sort_pairs<SortCfg>(nullptr, t1, h->nkeys_in.p, h->skeys.p, h->nvals_in.p,
                                             h->svals.p, N, 0, 64, h->stream));
  HIPCHK(rocprim::radix_sort_pairs<SortCfg>(nullptr, t2, h->ckeys_in.p, h->ckeys.p, h->cvals_in.p,
                                             h->cperm.p, B, 0, 64, h->stream));
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, t3, h->cflag.p, h->cid.p, (int)N, h->stream));
  return h->sort_tmp.ensure(std::max(std::max(t1, t2), t3));
}

// the first round: nearest = the root, score = its exact score (the scan's arithmetic), second
// bound +inf; also the resets k_nn_home does for the scan and the edge kernel
__device__ __forceinline__ void nn_root_lane(const PlanParams* __restrict__ Pd, DevState* st,
                                             const double* cfg, const double* cand, int nb, int* nn,
                                             double* second, double* score, GoalFix gf,
                                             int* bcount, int j) {
  if (j < 8) st->nn_queue[j] = 0;
  if (j == 0) {
    st->nn_counter = 0;
    st->work_counter = 0;
  }
  if (bcount && j < (nb + 255) / 256) bcount[j] = 0;  // k_edges' accepted-edge counts per 256 lanes
  if (j >= nb) return;
  const PlanParams P = *Pd;
  double a[7], s[7];
  load7(cfg, a);
  // the goal lane's candidate is the goal (its thread substitutes it: nothing else reads it here)
  if (gf.cand && j == st->round_goal) {
    goal_fix(Pd, st, gf, nb);
#pragma unroll
    for (int k = 0; k < 7; ++k) s[k] = P.goal[k];
  } else {
    load7(cand + 8 * (size_t)j, s);
  }
  const double d0 = s[0] - a[0], d1 = s[1] - a[1], d2 = s[2] - a[2], d3 = s[3] - a[3],
               d4 = s[4] - a[4], d5 = s[5] - a[5], d6 = s[6] - a[6];
  double dd;
  if (P.uniform_w) {
    dd = d0 * d0;
    dd = fma(d1, d1, dd); dd = fma(d2, d2, dd); dd = fma(d3, d3, dd);
    dd = fma(d4, d4, dd); dd = fma(d5, d5, dd); dd = fma(d6, d6, dd);
  } else {
    dd = P.w[0] * (d0 * d0);
    dd = fma(P.w[1] * d1, d1, dd); dd = fma(P.w[2] * d2, d2, dd); dd = fma(P.w[3] * d3, d3, dd);
    dd = fma(P.w[4] * d4, d4, dd); dd = fma(P.w[5] * d5, d5, dd); dd = fma(P.w[6] * d6, d6, dd);
  }
  nn[j] = 0;
  if (second) second[j] = INFINITY;
  if (score) score[j] = dd;
}
__global__ void k_nn_root(const PlanParams* __restrict__ Pd, DevState* st, const double* cfg,
                          const double* cand, int nb, int* nn, double* second, double* score,
                          GoalFix gf, int* bcount) {
  nn_root_lane(Pd, st, cfg, cand, nb, nn, second, score, gf, bcount,
               blockIdx.x * blockDim.x + threadIdx.x);
}

// Exact nearest node of nb candidates (rows of 8) among the st->n_nodes <= T_bound tree rows
// cfg (rows of 8): the radix-tree cell index (tcmp_nn.h), then k_nearest_wave32.  Outputs:
// nn (index), second (a lower bound of the second-smallest score, the rewire test's input),
// score (nullable: the winner's exact fp64 score).  The plan's rounds and tcmp_nearest both
// come here; st is the plan's state or st_nn.
int launch_nearest(tcmp_handle* h, const PlanParams& P, const PlanParams* dP, DevState* st,
                   const double* cfg,
                   long long T_bound, const double* cand, int nb, int* nn, double* second,
                   double* score, hipEvent_t* scan_end = nullptr, GoalFix gf = GoalFix{},
                   int* bcount = nullptr) {
  if (T_bound == 1) {
    // a one-node snapshot (the first round): the root is every candidate's nearest node and
    // there is no second one -- no index to build
    hipLaunchKernelGGL(k_nn_root, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, dP, st, cfg,
                       cand, nb, nn, second, score, gf, bcount);
    HIPCHK(hipGetLastError());
    return 0;
  }
  hipLaunchKernelGGL(k_node_keys, dim3(std::min<unsigned>(grid_for(T_bound, 256), 4096)), dim3(256),
                     0, h->stream, st, cfg, T_bound, h->nkeys_in.p, h->nvals_in.p, dP, gf, nb);
  HIPCHK(hipGetLastError());
  size_t tb = h->sort_tmp.n;
  // double-buffer form: the sorted keys / values stay in whichever buffer the last digit pass
  // wrote (the pass count depends only on the size, so a captured round graph stays valid) --
  // no copy back into fixed output buffers
  rocprim::double_buffer<unsigned long long> kdb(h->nkeys_in.p, h->skeys.p);
  rocprim::double_buffer<int> vdb(h->nvals_in.p, h->svals.p);
  HIPCHK(rocprim::radix_sort_pairs<SortCfg>(h->sort_tmp.p, tb, kdb, vdb, (size_t)T_bound, 0,
                                             kKeyBits, h->stream));
  unsigned long long* const skeys = kdb.current();
  const int* const svals = vdb.current();
  // rows in key order, radix-tree cells of <= 64 nodes, their bounds, super-cells
  hipLaunchKernelGGL(k_nn_rows, dim3(grid_for(T_bound, 256)), dim3(256), 0, h->stream, st,
                     dP, cfg, svals, h->stree.p, h->srow.p, T_bound, h->cflag.p, h->sflag.p);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_nn_cut<kNnC>, dim3(grid_for(T_bound, 256)), dim3(256), 0, h->stream,
                     &st->n_nodes, (const int*)nullptr, skeys, h->cflag.p);
  HIPCHK(hipGetLastError());
  tb = h->sort_tmp.n;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(h->sort_tmp.p, tb, h->cflag.p, h->cid.p, (int)T_bound,
                                          h->stream));
  hipLaunchKernelGGL(k_nn_starts, dim3(grid_for(T_bound, 256)), dim3(256), 0, h->stream,
                     &st->n_nodes, (const int*)nullptr, h->cflag.p, h->cid.p, h->cstart.p,
                     &st->nn_cells);
  HIPCHK(hipGetLastError());
  // one wave per cell, grid-stride: the cell count is device-side
  const unsigned idx_grid = (unsigned)std::min<long long>(grid_for(T_bound * 64, 256),
                                                          (long long)h->cu_count * 8);
  hipLaunchKernelGGL(k_nn_cell_boxes, dim3(idx_grid), dim3(256), 0, h->stream,
                     st, h->stree.p, h->cstart.p, skeys, h->cboxf.p, h->ckey.p);
  HIPCHK(hipGetLastError());
  // super-cells: the same radix-tree cut over the cells' first keys
  hipLaunchKernelGGL(k_nn_cut<kNnS>, dim3(grid_for(T_bound, 256)), dim3(256), 0, h->stream,
                     (const long long*)nullptr, &st->nn_cells, h->ckey.p, h->sflag.p);
  HIPCHK(hipGetLastError());
  tb = h->sort_tmp.n;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(h->sort_tmp.p, tb, h->sflag.p, h->sid.p, (int)T_bound,
                                          h->stream));
  hipLaunchKernelGGL(k_nn_starts, dim3(grid_for(T_bound, 256)), dim3(256), 0, h->stream,
                     (const long long*)nullptr, &st->nn_cells, h->sflag.p, h->sid.p,
                     h->sstart.p, &st->nn_supers);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_nn_build_supers, dim3(idx_grid), dim3(256), 0,
                     h->stream, st, h->sstart.p, h->cboxf.p, h->sboxf.p);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_nn_build_blocks, dim3(std::min<unsigned>(grid_for(T_bound + 128, 256), 1024)), dim3(256), 0,
                     h->stream, st, h->sboxf.p, h->bboxf.p);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_cand_keys, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, cand, nb,
                     h->ckeys_in.p, h->cvals_in.p, h->nn_cand_count_bits, h->cs_hist.p);
  HIPCHK(hipGetLastError());
  // candidates only need locality (the scan order never changes a result): their top key
  // bits (rocPRIM's Onesweep; a 65,536-bin counting sort measured 0.3 ms per query slower)
  if (h->nn_cand_count_bits > 0) {
    if (int rc = count_sort(h, h->cvals_in.p, nb, 1 << h->nn_cand_count_bits, h->cperm.p, true))
      return rc;
  } else {
    tb = h->sort_tmp.n;
    HIPCHK(rocprim::radix_sort_pairs<SortCfg>(h->sort_tmp.p, tb, h->ckeys_in.p, h->ckeys.p,
                                               h->cvals_in.p, h->cperm.p, (size_t)nb,
                                               kKeyBits - h->nn_cand_bits, kKeyBits, h->stream));
  }
  hipLaunchKernelGGL(k_nn_home, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, st,
                     skeys, h->ckeys_in.p, h->cperm.p, h->cid.p, h->sid.p, nb, h->chome.p,
                     bcount);
  HIPCHK(hipGetLastError());
  // one wave per candidate at a time; contiguous Morton-sorted runs per wave (k_nn_home
  // cleared the queues)
  const long long waves = std::min<long long>(nb, (long long)h->cu_count * h->nn_waves_per_cu);
  const int per_wave = (int)((nb + waves - 1) / waves);
  const unsigned blocks = grid_for((nb + per_wave - 1) / per_wave * 64, kNnBlock);
  hipEvent_t e0;
  h->launches_scan++;
  h->mark_begin(F_NNSCAN, &e0);
#define TCMP_NNW(UWV, SWV)                                                                   \
  hipLaunchKernelGGL((k_nearest_wave32<UWV, SWV>), dim3(blocks), dim3(kNnBlock), 0, h->stream, dP, st, \
                     h->stree.p, h->srow.p, h->cboxf.p, h->sboxf.p, h->bboxf.p, cand,             \
                     h->cperm.p, h->chome.p, nb, nn, second, score)
  // two cells per scan round: same-box A/B of 1 / 2 / 3 / 4 / 5 gave 4.44 / 4.03 / 4.21 /
  // 4.23 / 4.27 ms of scan per C3 query (eight: 137 VGPRs cost a wave per SIMD)
#ifndef TCMP_NN_SW
#define TCMP_NN_SW 2
#endif
  if (P.uniform_w) TCMP_NNW(true, TCMP_NN_SW); else TCMP_NNW(false, TCMP_NN_SW);
#undef TCMP_NNW
  HIPCHK(hipGetLastError());
  const hipEvent_t e1 = h->mark_end(F_NNSCAN, e0);
  if (scan_end) *scan_end = e1;
  return 0;
}

// planned step count of each round edge (nearest node -> candidate) as an ascending sort key
// for longest-first scheduling of k_edges
constexpr int kEdgeOrderMin = 4096;
// (the counting sort's histogram is built here too: one launch fewer)
__device__ __forceinline__ void edge_order_block(const PlanParams* __restrict__ Pd, const double* cfg,
                                                 const int* nn, const double* cand, int nb,
                                                 int* bins, int* hist, int blk) {
  __shared__ int lh[256];
  lh[threadIdx.x] = 0;
  __syncthreads();
  const int e = blk * blockDim.x + threadIdx.x;
  if (e < nb) {
    double a[7], b[7];
    load7(cfg + 8 * (size_t)nn[e], a);
    load7(cand + 8 * (size_t)e, b);
    const int n = num_steps(a, b, Pd->res);
    const int bin = 255 - min(n, 255);
    bins[e] = bin;
    atomicAdd(&lh[bin], 1);
  }
  __syncthreads();
  if (lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
}
__global__ __launch_bounds__(256) void k_edge_order_keys(const PlanParams* __restrict__ Pd, const double* cfg,
                                                         const int* nn, const double* cand, int nb,
                                                         int* bins, int* hist) {
  edge_order_block(Pd, cfg, nn, cand, nb, bins, hist, blockIdx.x);
}

// reset_counter = false: the plan's k_nn_home already cleared the work counter
// kernel_begin (nullable): an event recorded between k_edge_records and k_edges (timing on)
int launch_edges(tcmp_handle* h, const EdgeJob& J, const PlanParams* dP, bool reset_counter = true,
                 hipEvent_t* kernel_begin = nullptr) {
  if (J.n <= 0) return 0;
  if (reset_counter) HIPCHK(hipMemsetAsync(&h->st->work_counter, 0, sizeof(int), h->stream));
  // persistent grid bounded by residency (256-thread blocks hold one wave per SIMD each).
  // Above it, lanes refill from the longest-first queue; below it, one edge per lane --
  // halving the lanes of a small round (65,536 edges) would leave half the chip idle.
  const long long cap = (long long)h->cu_count * std::max(1, std::min(h->edge_wps, TCMP_EDGE_MINW));
  long long lanes = std::max<long long>(64, J.n);
  long long blocks = (lanes + 255) / 256;
  blocks = std::min(blocks, cap);
  blocks = std::max<long long>(blocks, 1);
  h->edge_blocks = (int)blocks;
  // a round with at most a half / a quarter of the resident lanes' edges: two / four lanes
  // per edge (k_edges SPLIT)
  int split = 1;
  while (split < std::min(TCMP_EDGE_SPLIT, h->edge_split) && 2LL * split * J.n <= cap * 256)
    split *= 2;
  if (split > 1) blocks = std::min(cap, ((long long)split * J.n + 255) / 256);
  h->edge_blocks = (int)blocks;
  hipLaunchKernelGGL(k_edge_records, dim3(grid_for(J.n, 256)), dim3(256), 0, h->stream, J, dP);
  if (kernel_begin) *kernel_begin = h->mark();
  const bool mk = h->mesh_kernels();
  auto kern = split == 4 ? (mk ? k_edges<true, 4> : k_edges<false, 4>)
              : split == 2 ? (mk ? k_edges<true, 2> : k_edges<false, 2>)
                           : (mk ? k_edges<true, 1> : k_edges<false, 1>);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds_bytes(h), h->stream, J, dP,
                     h->scene(), h->geo(), h->st);
  HIPCHK(hipGetLastError());
  return 0;
}

PlanParams default_params() {
  PlanParams P{};
  for (int k = 0; k < 7; ++k) {
    P.w[k] = 10.0;
    P.res[k] = 0.1;
  }
  P.radius = 0.01;
  P.goal_prob = 0.2;
  P.goal_tol = 1e-2;
  P.uniform_w = 1;
  P.max_nodes = LLONG_MAX;
  P.nn_cmax = 8.0;  // planner configurations lie in the joint-limit box (|q| <= 3.7525)
  return P;
}

int upload_spheres(tcmp_handle* h);  // (below) the links' and meshes' inscribed spheres
int fleet_lds_limits();  // (tcmp_fleet.h) the fused kernels' dynamic-LDS limits, set once
}  // namespace

// ==========================================================================================
// C-ABI
// ==========================================================================================
extern "C" {

const char* tcmp_last_error(void) { return g_err.c_str(); }
int tcmp_version(void) { return 1; }

int tcmp_debug_counters(tcmp_handle* h, uint64_t* out, int32_t n) {
  TCMP_ENTER(h);
  if (!out || n < 0 || n > 128) return fail(-1, "bad arguments");
  DevState s;
  HIPCHK(hipMemcpyAsync(&s, h->st, sizeof(s), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  // prof[] has 16 entries; 12..35 are the exact-test stats of TCMP_PROF_EXACT builds
  // 36..43 are the nearest scan's clocks and visit counts (prof_nn)
  // 44..51 the exact-test stats 24..31
  for (int i = 0; i < n; ++i)
    out[i] = i < 16 ? s.prof[i] : (i >= 36 && i < 44) ? s.prof_nn[i - 36] : 0;
#ifdef TCMP_PROF_EXACT
  unsigned long long ex[32];
  HIPCHK(hipMemcpyFromSymbol(ex, HIP_SYMBOL(g_exact_stats), sizeof(ex)));
  for (int i = 0; i < 24 && 12 + i < n && 12 + i < 36; ++i) out[12 + i] = ex[i];
  for (int i = 24; i < 32 && 20 + i < n; ++i) out[20 + i] = ex[i];
  // 52..83: the mesh chain's head-overlap histogram (g_fa_hist)
  unsigned long long fh[32];
  HIPCHK(hipMemcpyFromSymbol(fh, HIP_SYMBOL(g_fa_hist), sizeof(fh)));
  for (int i = 0; i < 32 && 52 + i < n; ++i) out[52 + i] = fh[i];
  // 84..115: the same pairs by the sphere certificate's best overlap (g_sb_hist)
  HIPCHK(hipMemcpyFromSymbol(fh, HIP_SYMBOL(g_sb_hist), sizeof(fh)));
  for (int i = 0; i < 32 && 84 + i < n; ++i) out[84 + i] = fh[i];
  // 116..119: the full fp32 stage's clocks (g_full_clk)
  HIPCHK(hipMemcpyFromSymbol(fh, HIP_SYMBOL(g_full_clk), 4 * sizeof(unsigned long long)));
  for (int i = 0; i < 4 && 116 + i < n; ++i) out[116 + i] = fh[i];
  // 120..127: phase B's pass structure (g_pass_stats)
  HIPCHK(hipMemcpyFromSymbol(fh, HIP_SYMBOL(g_pass_stats), 8 * sizeof(unsigned long long)));
  for (int i = 0; i < 8 && 120 + i < n; ++i) out[120 + i] = fh[i];
#endif
  return 0;
}

int tcmp_synchronize(tcmp_handle* h) {
  TCMP_ENTER(h);
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_device_count(int* n) {
  if (!n) return fail(-1, "null");
  HIPCHK(hipGetDeviceCount(n));
  return 0;
}

int tcmp_create(int device, tcmp_handle** out) {
  Entry entry;
  if (!out) return fail(-1, "null out");
  *out = nullptr;
  int nd = 0;
  HIPCHK(hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd) return fail(-1, "device index out of range");
  HIPCHK(hipSetDevice(device));
  tcmp_handle* h = new tcmp_handle();
  h->device = device;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  h->cu_count = prop.multiProcessorCount;
  HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  int rc = h->verts.ensure(TCMP_TOTAL_VERTS * 4);
  rc = rc ? rc : h->planes.ensure(TCMP_TOTAL_PLANES * 8);
  rc = rc ? rc : h->edges.ensure(TCMP_TOTAL_EDGES * 16);
  if (rc) { delete h; return rc; }
  HIPCHK(hipMemcpy(h->verts.p, tcmp_geo_verts, sizeof(tcmp_geo_verts), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->planes.p, tcmp_geo_planes, sizeof(tcmp_geo_planes), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->edges.p, tcmp_geo_edges, sizeof(tcmp_geo_edges), hipMemcpyHostToDevice));
  {
    // fp32 geometry for the exact test's first pass (staged in LDS by the kernels)
    std::vector<float> v32(3 * TCMP_TOTAL_VERTS), p32(4 * TCMP_TOTAL_PLANES);
    for (int v = 0; v < TCMP_TOTAL_VERTS; ++v)
      for (int k = 0; k < 3; ++k) v32[3 * v + k] = (float)tcmp_geo_verts[4 * v + k];
    for (int f = 0; f < TCMP_TOTAL_PLANES; ++f)
      for (int k = 0; k < 4; ++k) p32[4 * f + k] = (float)tcmp_geo_planes[8 * f + k];
    rc = h->verts32.ensure(v32.size());
    rc = rc ? rc : h->planes32.ensure(p32.size());
    rc = rc ? rc : h->eidx.ensure(4 * TCMP_TOTAL_EDGES);
    if (rc) { delete h; return rc; }
    HIPCHK(hipMemcpy(h->verts32.p, v32.data(), v32.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->planes32.p, p32.data(), p32.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->eidx.p, tcmp_geo_edge_idx, sizeof(tcmp_geo_edge_idx), hipMemcpyHostToDevice));
    {
      std::vector<float> ev(4 * TCMP_TOTAL_EDGES, 0.f);
      for (int e = 0; e < TCMP_TOTAL_EDGES; ++e) {
        const unsigned short* q = tcmp_geo_edge_idx + 4 * e;
        for (int k = 0; k < 3; ++k)
          ev[4 * e + k] = (float)(tcmp_geo_verts[4 * q[1] + k] - tcmp_geo_verts[4 * q[0] + k]);
      }
      rc = h->geo_ev.ensure(ev.size());
      if (rc) { delete h; return rc; }
      HIPCHK(hipMemcpy(h->geo_ev.p, ev.data(), ev.size() * 4, hipMemcpyHostToDevice));
    }
    // link LOD hulls (fp32 vertices [V][3], planes float4, edge rows)
    const double* lv[2] = {tcmp_lod_in_verts, tcmp_lod_out_verts};
    const double* lp[2] = {tcmp_lod_in_planes, tcmp_lod_out_planes};
    const unsigned short* le[2] = {tcmp_lod_in_edges, tcmp_lod_out_edges};
    const size_t nv[2] = {TCMP_LOD_IN_V, TCMP_LOD_OUT_V}, nf[2] = {TCMP_LOD_IN_F, TCMP_LOD_OUT_F},
                 ne[2] = {TCMP_LOD_IN_E, TCMP_LOD_OUT_E};
    for (int i = 0; i < 2; ++i) {
      std::vector<float> a(lv[i], lv[i] + 3 * nv[i]), b(lp[i], lp[i] + 4 * nf[i]);
      rc = h->lodv3[i].ensure(a.size());
      rc = rc ? rc : h->lodpl[i].ensure(b.size());
      rc = rc ? rc : h->lodei[i].ensure(4 * ne[i]);
      if (rc) { delete h; return rc; }
      HIPCHK(hipMemcpy(h->lodv3[i].p, a.data(), a.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(h->lodpl[i].p, b.data(), b.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(h->lodei[i].p, le[i], 4 * ne[i] * sizeof(unsigned short), hipMemcpyHostToDevice));
      std::vector<float> ev(4 * ne[i], 0.f);
      for (size_t e = 0; e < ne[i]; ++e)
        for (int k = 0; k < 3; ++k)
          ev[4 * e + k] = (float)(lv[i][3 * le[i][4 * e + 1] + k] - lv[i][3 * le[i][4 * e] + k]);
      rc = h->lodev[i].ensure(ev.size());
      if (rc) { delete h; return rc; }
      HIPCHK(hipMemcpy(h->lodev[i].p, ev.data(), ev.size() * 4, hipMemcpyHostToDevice));
    }
    // the links' inscribed spheres (box and mesh certificates in phase B)
    rc = upload_spheres(h);
    if (rc) { delete h; return rc; }
    // dynamic LDS above 64 KiB per workgroup must be allowed explicitly
    const int lim = (int)stage_lds_bytes(kMaxObstacles);
    for (const void* k : {(const void*)k_edges<false, 1>, (const void*)k_edges<true, 1>,
                          (const void*)k_edges<false, 2>, (const void*)k_edges<true, 2>,
                          (const void*)k_edges<false, 4>, (const void*)k_edges<true, 4>,
                          (const void*)k_check_configs<false>, (const void*)k_check_configs<true>,
                          (const void*)k_rewire_apply<false>, (const void*)k_rewire_apply<true>})
      HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    if (int rc2 = fleet_lds_limits()) { delete h; return rc2; }
  }
  HIPCHK(hipMalloc(&h->st, sizeof(DevState)));
  HIPCHK(hipMemset(h->st, 0, sizeof(DevState)));
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h->pin), sizeof(tcmp_handle::Pin)));
  HIPCHK(hipMalloc(&h->st_nn, sizeof(DevState)));
  HIPCHK(hipMalloc(&h->dP, sizeof(PlanParams)));
  HIPCHK(hipMalloc(&h->dPx, sizeof(PlanParams)));
  HIPCHK(hipMemset(h->st_nn, 0, sizeof(DevState)));
  if (const char* e = getenv("TCMP_NN_WAVES_PER_CU")) h->nn_waves_per_cu = std::max(1, atoi(e));
  if (const char* e = getenv("TCMP_GRAPHS")) h->use_graphs = atoi(e) != 0;
  if (const char* e = getenv("TCMP_SPHERES")) h->use_sph = atoi(e) != 0;
  if (const char* e = getenv("TCMP_NN_CBITS")) h->nn_cand_bits = std::min(16, std::max(8, atoi(e)));
  if (const char* e = getenv("TCMP_EDGE_SPLIT")) {
    // lanes per edge: a power of two (k_edges<., 1|2|4>), rounded down
    const int v = std::max(1, std::min(4, atoi(e)));
    h->edge_split = v >= 4 ? 4 : v >= 2 ? 2 : 1;
  }
  if (const char* e = getenv("TCMP_EDGE_WPS")) h->edge_wps = std::max(1, std::min(2, atoi(e)));
  if (const char* e = getenv("TCMP_NN_CSORT")) h->nn_cand_count_bits = std::min(16, std::max(0, atoi(e)));
  *out = h;
  return 0;
}

int tcmp_destroy(tcmp_handle* h) {
  if (!h) return 0;
  Entry entry;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->stream);
  h->verts32.release();
  h->planes32.release();
  h->eidx.release();
  h->geo_ev.release();
  h->sph.release();
  h->obs32.release();
  h->mrange.release();
  for (auto* b : {&h->mib, &h->mv64, &h->mp64, &h->me64, &h->base_geo, &h->base_pd}) b->release();
  for (auto* b : {&h->mv32, &h->mp32, &h->me32, &h->mcl, &h->lcl[0], &h->lcl[1]}) b->release();
  for (int i = 0; i < 2; ++i) {
    for (auto* b : {&h->lv32[i], &h->lp32[i], &h->le32[i], &h->lodv3[i], &h->lodpl[i], &h->lodev[i]})
      b->release();
    h->lodei[i].release();
  }
  for (auto* b : {&h->verts, &h->planes, &h->edges, &h->obs, &h->cfg, &h->tgt, &h->cand,
                  &h->last, &h->erec, &h->wp, &h->tq, &h->tqd, &h->tqdd, &h->tpsg, &h->ttau, &h->s0,
                  &h->s1, &h->s2, &h->s3})
    b->release();
  for (auto* b : {&h->parent, &h->nn, &h->nsafe, &h->nsteps, &h->nbr, &h->ncount, &h->i0,
                  &h->i1, &h->i2, &h->rwlist})
    b->release();
  h->nnscore.release();
  h->f_desc.release();
  h->f_off.release();
  h->dpin.release();
  if (h->dep_ev) (void)hipEventDestroy(h->dep_ev);
  if (h->scene_ev) (void)hipEventDestroy(h->scene_ev);
  if (h->scene_pin) (void)hipHostFree(h->scene_pin);
  if (h->fetch_pin) (void)hipHostFree(h->fetch_pin);
  for (auto* b : {&h->nkeys_in, &h->skeys, &h->ckeys_in, &h->ckeys}) b->release();
  h->cs_hist.release();
  h->cs_hoff.release();
  for (auto* b : {&h->nvals_in, &h->svals, &h->cvals_in, &h->cperm}) b->release();
  h->stree.release();
  h->srow.release();
  h->cbox.release();
  h->cboxf.release();
  h->sboxf.release();
  h->bboxf.release();
  h->chome.release();
  h->cflag.release();
  h->cid.release();
  h->cstart.release();
  h->sflag.release();
  h->sid.release();
  h->sstart.release();
  h->ckey.release();
  h->bcount.release();
  h->boff.release();
  h->sort_tmp.release();
  h->meta.release();
  h->cgoal.release();
  h->second.release();
  h->chain.release();
  h->u0.release();
  for (auto e : h->ev_rec) (void)hipEventDestroy(e);
  h->drop_graph();
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->st) (void)hipFree(h->st);
  if (h->pin) (void)hipHostFree(h->pin);
  if (h->st_nn) (void)hipFree(h->st_nn);
  if (h->dP) (void)hipFree(h->dP);
  if (h->dPx) (void)hipFree(h->dPx);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

}  // extern "C"

namespace {

// Device obstacle list = boxes then the meshes' outer boxes (records of 16 doubles, kind in
// [15]) plus the fp32 tier-0 records (world AABB centre, half extent - kPen + margin).
// Gauss-map edge records of world-frame hulls (rows of 16): c = -n1, d = -n2 (the obstacle
// enters the Minkowski difference negated), unit(d x c), edge vector vb - va, endpoint va.
void edge_records(const double* verts, const int32_t* vert_off, const double* planes,
                  const int32_t* plane_off, const int32_t* edges, const int32_t* edge_off,
                  int n, double* out) {
  for (int m = 0; m < n; ++m)
    for (int e = edge_off[m]; e < edge_off[m + 1]; ++e) {
      const int* q = edges + 4 * e;
      const double* va = verts + 3 * (vert_off[m] + q[0]);
      const double* vb = verts + 3 * (vert_off[m] + q[1]);
      const double* n1 = planes + 4 * (plane_off[m] + q[2]);
      const double* n2 = planes + 4 * (plane_off[m] + q[3]);
      double* o = out + 16 * e;
      for (int k = 0; k < 3; ++k) { o[k] = -n1[k]; o[3 + k] = -n2[k]; }
      double w[3] = {o[4] * o[2] - o[5] * o[1], o[5] * o[0] - o[3] * o[2], o[3] * o[1] - o[4] * o[0]};
      const double wl = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
      for (int k = 0; k < 3; ++k) o[6 + k] = wl > 0 ? w[k] / wl : 0.0;
      for (int k = 0; k < 3; ++k) { o[9 + k] = vb[k] - va[k]; o[12 + k] = va[k]; }
      o[15] = 0.0;
    }
}

// Sorts the Gauss-map records [e0, e1) of one hull (rows of 16 doubles, edge_records) by the
// direction of their arcs -- the arc c -> d lies in the cone (unit(c + d), half the c-d angle)
// -- and cuts them into at most kMaxGaussClusters clusters of consecutive records, appending
// each cluster's cone to cl (8 floats: axis, cos, sin of the half-angle, first and end record
// as int bits, 0): the axis is the normalized sum of its arcs' axes, the half-angle the largest
// (angle to an arc's axis + that arc's half-angle), plus 1e-3 rad.  Returns the clusters'
// index range in cl through c0 / c1.  Record order does not matter anywhere else (every
// consumer takes a minimum over all records).
// (at most 128 clusters of at least 2 records: C5 11.15M -> 12.05M samples/s against 32 of at
// least 8, k_fl_edges_mesh 61.1 -> 55.9 ms per launch, same-box A/B, profiles/r9zj_ab_c5_clusters/:
// the pass-2 walks shrink faster than the pass-1 cone tests grow; >= 2 records another 0.5 %,
// 192 / 256 clusters slower, profiles/r9zk_ab_c5_clusters/)
#ifndef TCMP_GAUSS_MINREC
#define TCMP_GAUSS_MINREC 2  // records per cluster at least
#endif
void gauss_clusters(double* rec, int e0, int e1, std::vector<float>& cl, int* c0, int* c1) {
  const int n = e1 - e0;
  *c0 = (int)(cl.size() / 8);
  if (n <= 0) {
    *c1 = *c0;
    return;
  }
  struct Arc {
    double ax[3], half;
    unsigned key;
    int row;
  };
  std::vector<Arc> arcs((size_t)n);
  for (int i = 0; i < n; ++i) {
    const double* r = rec + 16 * (size_t)(e0 + i);
    Arc& a = arcs[(size_t)i];
    double s[3] = {r[0] + r[3], r[1] + r[4], r[2] + r[5]};
    const double sl = sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    const double cd = std::max(-1.0, std::min(1.0, r[0] * r[3] + r[1] * r[4] + r[2] * r[5]));
    if (sl > 1e-9) {
      for (int k = 0; k < 3; ++k) a.ax[k] = s[k] / sl;
      a.half = 0.5 * acos(cd);
    } else {  // antipodal normals: no cone smaller than the sphere
      a.ax[0] = 1; a.ax[1] = 0; a.ax[2] = 0;
      a.half = 3.14159265358979323846;
    }
    // cube-map face of the axis, then a 4-bit-per-coordinate Morton code on that face
    int f = 0;
    for (int k = 1; k < 3; ++k)
      if (fabs(a.ax[k]) > fabs(a.ax[f])) f = k;
    const int u = (f + 1) % 3, v = (f + 2) % 3;
    const double m = fabs(a.ax[f]) > 0 ? fabs(a.ax[f]) : 1.0;
    const unsigned qu = (unsigned)std::min(15.0, std::max(0.0, (a.ax[u] / m + 1.0) * 8.0));
    const unsigned qv = (unsigned)std::min(15.0, std::max(0.0, (a.ax[v] / m + 1.0) * 8.0));
    unsigned mort = 0;
    for (int b = 3; b >= 0; --b) mort = (mort << 2) | (((qu >> b) & 1u) << 1) | ((qv >> b) & 1u);
    a.key = ((unsigned)(2 * f + (a.ax[f] < 0 ? 1 : 0)) << 8) | mort;
    a.row = e0 + i;
  }
  std::stable_sort(arcs.begin(), arcs.end(), [](const Arc& x, const Arc& y) { return x.key < y.key; });
  std::vector<double> tmp((size_t)n * 16);
  for (int i = 0; i < n; ++i)
    memcpy(tmp.data() + 16 * (size_t)i, rec + 16 * (size_t)arcs[(size_t)i].row, 16 * sizeof(double));
  memcpy(rec + 16 * (size_t)e0, tmp.data(), tmp.size() * sizeof(double));
  const int K = std::max(TCMP_GAUSS_MINREC, (n + kMaxGaussClusters - 1) / kMaxGaussClusters);
  for (int s0 = 0; s0 < n; s0 += K) {
    const int s1 = std::min(n, s0 + K);
    double b[3] = {0, 0, 0};
    for (int i = s0; i < s1; ++i)
      for (int k = 0; k < 3; ++k) b[k] += arcs[(size_t)i].ax[k];
    const double bl = sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
    double half = 0.0;
    if (bl > 1e-9) {
      for (int k = 0; k < 3; ++k) b[k] /= bl;
      for (int i = s0; i < s1; ++i) {
        const Arc& a = arcs[(size_t)i];
        const double c = std::max(-1.0, std::min(1.0, b[0] * a.ax[0] + b[1] * a.ax[1] + b[2] * a.ax[2]));
        half = std::max(half, acos(c) + a.half);
      }
      half += 1e-3;
    } else {
      b[0] = 1; b[1] = 0; b[2] = 0;
      half = 3.14159265358979323846;
    }
    half = std::min(half, 3.14159265358979323846);
    int r0 = e0 + s0, r1 = e0 + s1;
    float f[8] = {(float)b[0], (float)b[1], (float)b[2], (float)cos(half), (float)sin(half), 0.f, 0.f,
                  0.f};
    memcpy(&f[5], &r0, 4);
    memcpy(&f[6], &r1, 4);
    cl.insert(cl.end(), f, f + 8);
  }
  *c1 = (int)(cl.size() / 8);
}

int check_hulls(const tcmp_hulls* H, int n, const char* what) {
  if (!H || !H->verts || !H->vert_off || !H->planes || !H->plane_off || !H->edges || !H->edge_off)
    return fail(-1, std::string("null ") + what + " hull array");
  if (H->vert_off[0] != 0 || H->plane_off[0] != 0 || H->edge_off[0] != 0)
    return fail(-1, std::string(what) + " hull offsets must start at 0");
  for (int m = 0; m < n; ++m) {
    const int nv = H->vert_off[m + 1] - H->vert_off[m], nf = H->plane_off[m + 1] - H->plane_off[m];
    if (nv < 4 || nf < 4 || H->edge_off[m + 1] - H->edge_off[m] < 6)
      return fail(-1, std::string(what) + " hull " + std::to_string(m) + " is not a 3-D hull");
    for (int e = H->edge_off[m]; e < H->edge_off[m + 1]; ++e) {
      const int* q = H->edges + 4 * e;
      if (q[0] < 0 || q[0] >= nv || q[1] < 0 || q[1] >= nv || q[2] < 0 || q[2] >= nf || q[3] < 0 ||
          q[3] >= nf)
        return fail(-1, std::string(what) + " hull " + std::to_string(m) + ": edge index out of range");
    }
  }
  return 0;
}

int upload_lods(tcmp_handle* h);
int upload_spheres(tcmp_handle* h);

// Device mesh arrays from the host copies: the user meshes, then (self-collision on) the 10
// link hulls in their own link frames as meshes n_mesh + j; then their LOD rows.
int upload_meshes(tcmp_handle* h) {
  const int n_user = h->n_mesh, n_self = h->self_coll ? TCMP_NLINKS : 0;
  const int n_mesh = n_user + n_self;
  std::vector<double> verts(h->mesh_v), planes(h->mesh_p), boxes(h->mesh_box);
  std::vector<int> edges(h->mesh_e), vert_off(h->mesh_voff), plane_off(h->mesh_poff),
      edge_off(h->mesh_eoff);
  if (vert_off.empty()) vert_off.assign(1, 0);
  if (plane_off.empty()) plane_off.assign(1, 0);
  if (edge_off.empty()) edge_off.assign(1, 0);
  for (int j = 0; j < n_self; ++j) {
    const int v0 = tcmp_geo_vert_off[j], f0 = tcmp_geo_plane_off[j];
    for (int v = v0; v < tcmp_geo_vert_off[j + 1]; ++v)
      for (int k = 0; k < 3; ++k) verts.push_back(tcmp_geo_verts[4 * v + k]);
    for (int f = f0; f < tcmp_geo_plane_off[j + 1]; ++f)
      for (int k = 0; k < 4; ++k) planes.push_back(tcmp_geo_planes[8 * f + k]);
    for (int e = tcmp_geo_edge_off[j]; e < tcmp_geo_edge_off[j + 1]; ++e) {
      const unsigned short* q = tcmp_geo_edge_idx + 4 * e;
      edges.push_back(q[0] - v0); edges.push_back(q[1] - v0);
      edges.push_back(q[2] - f0); edges.push_back(q[3] - f0);
    }
    for (int k = 0; k < 18; ++k) boxes.push_back(tcmp_geo_boxes[18 * j + k]);
    vert_off.push_back(vert_off.back() + tcmp_geo_vert_off[j + 1] - v0);
    plane_off.push_back(plane_off.back() + tcmp_geo_plane_off[j + 1] - f0);
    edge_off.push_back(edge_off.back() + tcmp_geo_edge_off[j + 1] - tcmp_geo_edge_off[j]);
  }
  const int V = vert_off[n_mesh], F = plane_off[n_mesh], E = edge_off[n_mesh];
  // device records: vertex/plane rows, Gauss-map edge records (global rows), inner boxes
  std::vector<int> rg((size_t)std::max(n_mesh, 1) * kMrange, 0);
  std::vector<double> ib((size_t)std::max(n_mesh, 1) * 16, 0.0);
  std::vector<double> v64((size_t)std::max(V, 1) * 4, 0.0), p64((size_t)std::max(F, 1) * 4, 0.0),
      e64((size_t)std::max(E, 1) * 16, 0.0);
  for (int m = 0; m < n_mesh; ++m) {
    int* r = rg.data() + kMrange * m;
    r[0] = vert_off[m]; r[1] = vert_off[m + 1];
    r[2] = plane_off[m]; r[3] = plane_off[m + 1];
    r[4] = edge_off[m]; r[5] = edge_off[m + 1];
    const double* b = boxes.data() + 18 * m;
    double* d = ib.data() + 16 * m;
    for (int k = 0; k < 12; ++k) d[k] = b[k];
    for (int k = 0; k < 3; ++k) d[12 + k] = b[15 + k];
  }
  edge_records(verts.data(), vert_off.data(), planes.data(), plane_off.data(), edges.data(),
               edge_off.data(), n_mesh, e64.data());
  std::vector<float> mcl;
  for (int m = 0; m < n_mesh; ++m)
    gauss_clusters(e64.data(), edge_off[m], edge_off[m + 1], mcl, &rg[kMrange * m + 20],
                   &rg[kMrange * m + 21]);
  if (mcl.empty()) mcl.assign(8, 0.f);
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < 3; ++k) v64[4 * v + k] = verts[3 * v + k];
  for (int f = 0; f < F; ++f)
    for (int k = 0; k < 4; ++k) p64[4 * f + k] = planes[4 * f + k];
  std::vector<float> v32(v64.begin(), v64.end()), p32(p64.begin(), p64.end()), e32(e64.begin(), e64.end());
  int rc = h->mrange.ensure(rg.size());
  rc = rc ? rc : h->mib.ensure(ib.size());
  rc = rc ? rc : h->mv64.ensure(v64.size());
  rc = rc ? rc : h->mp64.ensure(p64.size());
  rc = rc ? rc : h->me64.ensure(e64.size());
  rc = rc ? rc : h->mv32.ensure(v32.size());
  rc = rc ? rc : h->mp32.ensure(p32.size());
  rc = rc ? rc : h->me32.ensure(e32.size());
  rc = rc ? rc : h->mcl.ensure(mcl.size());
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h->mcl.p, mcl.data(), mcl.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mrange.p, rg.data(), rg.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mib.p, ib.data(), ib.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mv64.p, v64.data(), v64.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mp64.p, p64.data(), p64.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->me64.p, e64.data(), e64.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mv32.p, v32.data(), v32.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->mp32.p, p32.data(), p32.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->me32.p, e32.data(), e32.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  h->mrange_h = rg;
  if (int rc = upload_lods(h)) return rc;
  return upload_spheres(h);
}

// Inscribed spheres (mrange flag 19): the links' rows first, then the user meshes'
// (tcmp_set_mesh_spheres, world frame) and, self-collision on, the links' own for the link
// meshes n_mesh + j (link frames).
int upload_spheres(tcmp_handle* h) {
  const int n_user = h->n_mesh, n_self = h->self_coll ? TCMP_NLINKS : 0, nm = n_user + n_self;
  constexpr int K = TCMP_NSPH;
  std::vector<float> a((size_t)(TCMP_NLINKS + nm) * K * 4, 0.f);
  for (int i = 0; i < TCMP_NLINKS * K * 4; ++i) a[i] = (float)tcmp_link_spheres[i];
  std::vector<int> rg = h->mrange_h;
  for (int m = 0; m < nm; ++m) {
    const double* src = nullptr;
    if (m < n_user) {
      if (h->user_sph) src = h->sph_h.data() + (size_t)m * K * 4;
    } else {
      src = tcmp_link_spheres + (size_t)(m - n_user) * K * 4;
    }
    rg[kMrange * m + 19] = (src && h->use_sph) ? 1 : 0;
    if (src)
      for (int i = 0; i < K * 4; ++i) a[(size_t)(TCMP_NLINKS + m) * K * 4 + i] = (float)src[i];
  }
  int rc = h->sph.ensure(a.size());
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h->sph.p, a.data(), a.size() * 4, hipMemcpyHostToDevice, h->stream));
  if (nm)
    HIPCHK(hipMemcpyAsync(h->mrange.p, rg.data(), rg.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  h->mrange_h = rg;
  return 0;
}

// Level-of-detail hulls of the meshes (rows 6..17 of mrange, flag 18): the user meshes'
// (tcmp_set_mesh_lods, world frame) followed, self-collision on, by the links' own LODs
// (panda_lod.inc, link frames) for the link meshes n_mesh + j.
int upload_lods(tcmp_handle* h) {
  const int n_user = h->user_lods ? h->n_mesh : 0, n_self = h->self_coll ? TCMP_NLINKS : 0;
  if (n_user + n_self == 0) return 0;
  std::vector<int> rg = h->mrange_h;
  const double* lv[2] = {tcmp_lod_in_verts, tcmp_lod_out_verts};
  const double* lp[2] = {tcmp_lod_in_planes, tcmp_lod_out_planes};
  const unsigned short* le[2] = {tcmp_lod_in_edges, tcmp_lod_out_edges};
  const int* lvo[2] = {tcmp_lod_in_vert_off, tcmp_lod_out_vert_off};
  const int* lpo[2] = {tcmp_lod_in_plane_off, tcmp_lod_out_plane_off};
  const int* leo[2] = {tcmp_lod_in_edge_off, tcmp_lod_out_edge_off};
  for (int i = 0; i < 2; ++i) {
    std::vector<double> v, pl;
    std::vector<int> e, vo{0}, po{0}, eo{0};
    if (n_user) {
      v = h->lod_v[i]; pl = h->lod_p[i]; e = h->lod_e[i];
      vo = h->lod_vo[i]; po = h->lod_po[i]; eo = h->lod_eo[i];
    }
    for (int j = 0; j < n_self; ++j) {
      for (int r = lvo[i][j]; r < lvo[i][j + 1]; ++r)
        for (int k = 0; k < 3; ++k) v.push_back(lv[i][3 * r + k]);
      for (int r = lpo[i][j]; r < lpo[i][j + 1]; ++r)
        for (int k = 0; k < 4; ++k) pl.push_back(lp[i][4 * r + k]);
      for (int r = leo[i][j]; r < leo[i][j + 1]; ++r) {
        const unsigned short* q = le[i] + 4 * r;
        e.push_back(q[0] - lvo[i][j]); e.push_back(q[1] - lvo[i][j]);
        e.push_back(q[2] - lpo[i][j]); e.push_back(q[3] - lpo[i][j]);
      }
      vo.push_back(vo.back() + lvo[i][j + 1] - lvo[i][j]);
      po.push_back(po.back() + lpo[i][j + 1] - lpo[i][j]);
      eo.push_back(eo.back() + leo[i][j + 1] - leo[i][j]);
    }
    const int nm = n_user + n_self, V = vo[nm], F = po[nm], E = eo[nm];
    std::vector<double> e64((size_t)E * 16);
    edge_records(v.data(), vo.data(), pl.data(), po.data(), e.data(), eo.data(), nm, e64.data());
    std::vector<float> lcl;
    std::vector<int> cr(2 * (size_t)nm);
    for (int m = 0; m < nm; ++m) gauss_clusters(e64.data(), eo[m], eo[m + 1], lcl, &cr[2 * m], &cr[2 * m + 1]);
    if (lcl.empty()) lcl.assign(8, 0.f);
    std::vector<float> v32((size_t)V * 4, 0.f), p32(pl.begin(), pl.end()), e32(e64.begin(), e64.end());
    for (int r = 0; r < V; ++r)
      for (int k = 0; k < 3; ++k) v32[4 * r + k] = (float)v[3 * r + k];
    int rc = h->lv32[i].ensure(v32.size());
    rc = rc ? rc : h->lp32[i].ensure(p32.size());
    rc = rc ? rc : h->le32[i].ensure(e32.size());
    rc = rc ? rc : h->lcl[i].ensure(lcl.size());
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(h->lcl[i].p, lcl.data(), lcl.size() * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->lv32[i].p, v32.data(), v32.size() * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->lp32[i].p, p32.data(), p32.size() * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->le32[i].p, e32.data(), e32.size() * 4, hipMemcpyHostToDevice, h->stream));
    if (int rc_s = sync_stream(h)) return rc_s;  // host staging buffers go out of scope
    for (int m = 0; m < nm; ++m) {
      // LOD hull m belongs to mesh m (user) or to link mesh h->n_mesh + (m - n_user)
      const int mesh = m < n_user ? m : h->n_mesh + (m - n_user);
      int* r = rg.data() + kMrange * mesh + 6 + 6 * i;
      r[0] = vo[m]; r[1] = vo[m + 1];
      r[2] = po[m]; r[3] = po[m + 1];
      r[4] = eo[m]; r[5] = eo[m + 1];
      rg[kMrange * mesh + 22 + 2 * i] = cr[2 * m];
      rg[kMrange * mesh + 23 + 2 * i] = cr[2 * m + 1];
      rg[kMrange * mesh + 18] = 1;
    }
  }
  HIPCHK(hipMemcpyAsync(h->mrange.p, rg.data(), rg.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  h->mrange_h = rg;
  return 0;
}


// Tier-0 record of an obstacle (fp32, 8 floats): axis i's world-AABB bounds shrunk by kPen
// (less a rounding margin), as tier 0 compares them -- [hi_x, hi_y, hi_z, 0, -lo_x, -lo_y,
// -lo_z, 0] with hi = c + H', lo = c - H', H' = half extent - kPen + margin, each rounded once
// from fp64 (the margin, 1e-5 + 1e-6 (|c| + H), covers that rounding and the link side's).
static void tier0_bounds(float* f, int i, double c, double Hs) {
  f[i] = (float)(c + Hs);
  f[4 + i] = (float)(Hs - c);
  f[3] = 0.f;
  f[7] = 0.f;
}

int upload_scene(tcmp_handle* h) {
  const int n = h->n_box + h->n_mesh;
  const int n_self = h->self_coll ? TCMP_NLINKS : 0;
  std::vector<double> tmp((size_t)std::max(n + n_self, 1) * 16, 0.0);
  std::vector<float> t32((size_t)std::max(n, 1) * 8, 0.f);
  for (int o = 0; o < h->n_box; ++o) {
    const double* s = h->box15.data() + 15 * o;
    double* d = tmp.data() + 16 * o;
    for (int k = 0; k < 15; ++k) d[k] = s[k];
    const double* R = s + 3;
    const bool aligned = R[0] == 1.0 && R[4] == 1.0 && R[8] == 1.0 && R[1] == 0.0 &&
                         R[2] == 0.0 && R[3] == 0.0 && R[5] == 0.0 && R[6] == 0.0 &&
                         R[7] == 0.0;
    d[15] = aligned ? 1.0 : 0.0;
    float* f = t32.data() + 8 * o;
    for (int i = 0; i < 3; ++i) {
      const double H = fabs(d[3 + 3 * i]) * d[12] + fabs(d[4 + 3 * i]) * d[13] +
                       fabs(d[5 + 3 * i]) * d[14];
      tier0_bounds(f, i, d[i], H - kPen + 1e-5 + 1e-6 * (fabs(d[i]) + H));
    }
  }
  for (int m = 0; m < h->n_mesh; ++m) {
    const double* b = h->mesh_box.data() + 18 * m;
    double* d = tmp.data() + 16 * (h->n_box + m);
    for (int k = 0; k < 15; ++k) d[k] = b[k];
    d[15] = -(double)(m + 1);
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int v = h->mesh_voff[m]; v < h->mesh_voff[m + 1]; ++v)
      for (int i = 0; i < 3; ++i) {
        lo[i] = std::min(lo[i], h->mesh_v[3 * v + i]);
        hi[i] = std::max(hi[i], h->mesh_v[3 * v + i]);
      }
    float* f = t32.data() + 8 * (h->n_box + m);
    for (int i = 0; i < 3; ++i) {
      const double c = 0.5 * (lo[i] + hi[i]), H = 0.5 * (hi[i] - lo[i]);
      tier0_bounds(f, i, c, H - kPen + 1e-5 + 1e-6 * (fabs(c) + H));
    }
  }
  // self-collision: link j's outer box in its own frame, as the record of mesh n_mesh + j
  for (int j = 0; j < n_self; ++j) {
    const double* b = tcmp_geo_boxes + 18 * j;
    double* d = tmp.data() + 16 * (n + j);
    for (int k = 0; k < 15; ++k) d[k] = b[k];
    d[15] = -(double)(h->n_mesh + j + 1);
  }
  if (int rc = h->obs.ensure(tmp.size())) return rc;
  if (int rc = h->obs32.ensure(t32.size())) return rc;
  // through the handle's pinned staging: the copies are queued and the call returns (a query's
  // set_scene no longer waits for the engine's stream); the staging is reused only after the
  // previous scene's copies have been done
  const size_t b64 = tmp.size() * sizeof(double), b32 = t32.size() * sizeof(float);
  if (h->scene_ev) HIPCHK(hipEventSynchronize(h->scene_ev));
  else HIPCHK(hipEventCreateWithFlags(&h->scene_ev, hipEventDisableTiming));
  if (h->scene_pin_n < b64 + b32) {
    if (h->scene_pin) HIPCHK(hipHostFree(h->scene_pin));
    h->scene_pin = nullptr;
    h->scene_pin_n = 0;
    HIPCHK(hipHostMalloc(&h->scene_pin, b64 + b32));
    h->scene_pin_n = b64 + b32;
  }
  unsigned char* pin = static_cast<unsigned char*>(h->scene_pin);
  memcpy(pin, tmp.data(), b64);
  memcpy(pin + b64, t32.data(), b32);
  HIPCHK(hipMemcpyAsync(h->obs.p, pin, b64, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->obs32.p, pin + b64, b32, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipEventRecord(h->scene_ev, h->stream));
  h->n_obs = n;
  return 0;
}

}  // namespace

extern "C" {

int tcmp_set_scene(tcmp_handle* h, const double* obb, int32_t n_obs) {
  TCMP_ENTER(h);
  if (n_obs < 0 || (n_obs > 0 && !obb)) return fail(-1, "bad obstacle array");
  if (n_obs + h->n_mesh > kMaxObstacles)
    return fail(-1, "too many obstacles (" + std::to_string(n_obs + h->n_mesh) + " > " +
                        std::to_string(kMaxObstacles) + ", the LDS-staged scene limit)");
  for (int o = 0; o < n_obs; ++o) {
    const double* s = obb + 15 * o;
    if (!(s[12] >= 0 && s[13] >= 0 && s[14] >= 0)) return fail(-1, "negative half extent");
  }
  h->box15.assign(obb, obb + 15 * (size_t)n_obs);
  h->n_box = n_obs;
  return upload_scene(h);
}

int tcmp_set_meshes(tcmp_handle* h, const double* verts, const int32_t* vert_off,
                    const double* planes, const int32_t* plane_off, const int32_t* edges,
                    const int32_t* edge_off, const double* boxes, int32_t n_mesh) {
  TCMP_ENTER(h);
  if (n_mesh < 0) return fail(-1, "bad mesh count");
  if (n_mesh > 0 && (!verts || !vert_off || !planes || !plane_off || !edges || !edge_off || !boxes))
    return fail(-1, "null mesh array");
  if (h->n_box + n_mesh > kMaxObstacles)
    return fail(-1, "too many obstacles (" + std::to_string(h->n_box + n_mesh) + " > " +
                        std::to_string(kMaxObstacles) + ", the LDS-staged scene limit)");
  const int V = n_mesh ? vert_off[n_mesh] : 0, F = n_mesh ? plane_off[n_mesh] : 0,
            E = n_mesh ? edge_off[n_mesh] : 0;
  if (n_mesh && (vert_off[0] != 0 || plane_off[0] != 0 || edge_off[0] != 0))
    return fail(-1, "mesh offsets must start at 0");
  for (int m = 0; m < n_mesh; ++m) {
    const int nv = vert_off[m + 1] - vert_off[m], nf = plane_off[m + 1] - plane_off[m],
              ne = edge_off[m + 1] - edge_off[m];
    if (nv < 4 || nf < 4 || ne < 6) return fail(-1, "mesh " + std::to_string(m) + " is not a 3-D hull");
    for (int e = edge_off[m]; e < edge_off[m + 1]; ++e) {
      const int* q = edges + 4 * e;
      if (q[0] < 0 || q[0] >= nv || q[1] < 0 || q[1] >= nv || q[2] < 0 || q[2] >= nf || q[3] < 0 ||
          q[3] >= nf)
        return fail(-1, "mesh " + std::to_string(m) + ": edge index out of range");
    }
    const double* b = boxes + 18 * m;
    for (int k = 12; k < 18; ++k)
      if (!(b[k] >= 0)) return fail(-1, "mesh " + std::to_string(m) + ": negative box half extent");
  }
  h->mesh_v.assign(verts, verts + 3 * (size_t)V);
  h->mesh_p.assign(planes, planes + 4 * (size_t)F);
  h->mesh_e.assign(edges, edges + 4 * (size_t)E);
  h->mesh_box.assign(boxes, boxes + 18 * (size_t)n_mesh);
  if (n_mesh > 0) {
    h->mesh_voff.assign(vert_off, vert_off + n_mesh + 1);
    h->mesh_poff.assign(plane_off, plane_off + n_mesh + 1);
    h->mesh_eoff.assign(edge_off, edge_off + n_mesh + 1);
  } else {
    h->mesh_voff.assign(1, 0);
    h->mesh_poff.assign(1, 0);
    h->mesh_eoff.assign(1, 0);
  }
  h->n_mesh = n_mesh;
  h->user_lods = false;  // new meshes: their LODs come with the next tcmp_set_mesh_lods
  h->user_sph = false;   // and their spheres with the next tcmp_set_mesh_spheres
  if (int rc = upload_meshes(h)) return rc;
  return upload_scene(h);
}

int tcmp_set_mesh_lods(tcmp_handle* h, const tcmp_hulls* inner, const tcmp_hulls* outer,
                       int32_t n_mesh) {
  TCMP_ENTER(h);
  if (n_mesh != h->n_mesh) return fail(-1, "LOD count differs from the mesh count");
  if (n_mesh == 0) return 0;
  if (int rc = check_hulls(inner, n_mesh, "inner")) return rc;
  if (int rc = check_hulls(outer, n_mesh, "outer")) return rc;
  const tcmp_hulls* H[2] = {inner, outer};
  for (int i = 0; i < 2; ++i) {
    const int V = H[i]->vert_off[n_mesh], F = H[i]->plane_off[n_mesh], E = H[i]->edge_off[n_mesh];
    h->lod_v[i].assign(H[i]->verts, H[i]->verts + 3 * (size_t)V);
    h->lod_p[i].assign(H[i]->planes, H[i]->planes + 4 * (size_t)F);
    h->lod_e[i].assign(H[i]->edges, H[i]->edges + 4 * (size_t)E);
    h->lod_vo[i].assign(H[i]->vert_off, H[i]->vert_off + n_mesh + 1);
    h->lod_po[i].assign(H[i]->plane_off, H[i]->plane_off + n_mesh + 1);
    h->lod_eo[i].assign(H[i]->edge_off, H[i]->edge_off + n_mesh + 1);
  }
  h->user_lods = true;
  return upload_lods(h);
}

int tcmp_set_mesh_spheres(tcmp_handle* h, const double* spheres, int32_t n_mesh, int32_t k) {
  TCMP_ENTER(h);
  if (n_mesh != h->n_mesh) return fail(-1, "sphere count differs from the mesh count");
  if (k != TCMP_NSPH) return fail(-1, "spheres per mesh must be " + std::to_string(TCMP_NSPH));
  if (n_mesh == 0) return 0;
  if (!spheres) return fail(-1, "null sphere array");
  for (int i = 0; i < n_mesh * k; ++i) {
    const double* s = spheres + 4 * (size_t)i;
    if (!(s[3] >= 0.0) || !std::isfinite(s[0]) || !std::isfinite(s[1]) || !std::isfinite(s[2]) ||
        !std::isfinite(s[3]))
      return fail(-1, "bad sphere row " + std::to_string(i));
    // the certificates are sound only for balls inside the hull: n.c + r <= d on every facet
    const int m = i / k;
    double out = -INFINITY;
    for (int f = h->mesh_poff[m]; f < h->mesh_poff[m + 1]; ++f) {
      const double* p = h->mesh_p.data() + 4 * (size_t)f;
      out = std::max(out, p[0] * s[0] + p[1] * s[1] + p[2] * s[2] - p[3]);
    }
    if (out + s[3] > 1e-9)
      return fail(-1, "sphere row " + std::to_string(i) + " is not inside mesh " +
                          std::to_string(m) + "'s hull");
  }
  h->sph_h.assign(spheres, spheres + (size_t)n_mesh * k * 4);
  h->user_sph = true;
  return upload_spheres(h);
}

int tcmp_set_self_collision(tcmp_handle* h, int32_t enable) {
  TCMP_ENTER(h);
  const int on = enable ? 1 : 0;
  if (on == h->self_coll) return 0;
  h->self_coll = on;
  if (int rc = upload_meshes(h)) return rc;
  return upload_scene(h);
}

int tcmp_set_timing(tcmp_handle* h, int32_t enable) {
  TCMP_ENTER(h);
  h->timing = enable != 0;  // part of the round-graph key: a changed setting captures anew
  return 0;
}

int tcmp_rne_batch(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                   int64_t n, double payload_mass, double* tau) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!q || !qd || !qdd || !tau))) return fail(-1, "bad arguments");
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, q, n);
  rc = rc ? rc : upload7(h, h->s1, qd, n);
  rc = rc ? rc : upload7(h, h->s2, qdd, n);
  rc = rc ? rc : h->s3.ensure((size_t)n * 7);
  if (rc) return rc;
  hipLaunchKernelGGL(k_rne, dim3(grid_for(n, 128)), dim3(128), 0, h->stream, h->s0.p, h->s1.p,
                     h->s2.p, (long long)n, payload_mass, h->s3.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(tau, h->s3.p, (size_t)n * 7 * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_ik(tcmp_handle* h, const double* poses, const double* free_q7, int64_t n, double* sols,
            int32_t* count) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!poses || !free_q7 || !sols || !count)))
    return fail(-1, "bad arguments");
  if (n == 0) return 0;
  int rc = h->s0.ensure((size_t)n * 12);
  rc = rc ? rc : h->s1.ensure((size_t)n);
  rc = rc ? rc : h->s2.ensure((size_t)n * 56);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h->s0.p, poses, (size_t)n * 12 * sizeof(double), hipMemcpyHostToDevice,
                        h->stream));
  HIPCHK(hipMemcpyAsync(h->s1.p, free_q7, (size_t)n * sizeof(double), hipMemcpyHostToDevice,
                        h->stream));
  hipLaunchKernelGGL(k_ik, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, h->s0.p, h->s1.p,
                     (long long)n, h->s2.p, h->i0.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(sols, h->s2.p, (size_t)n * 56 * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  HIPCHK(hipMemcpyAsync(count, h->i0.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_fk(tcmp_handle* h, const double* q, int64_t n, double* poses) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!q || !poses))) return fail(-1, "bad arguments");
  if (n == 0) return 0;
  int rc = h->s0.ensure((size_t)n * 7);
  rc = rc ? rc : h->s1.ensure((size_t)n * 12);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h->s0.p, q, (size_t)n * 7 * sizeof(double), hipMemcpyHostToDevice,
                        h->stream));
  hipLaunchKernelGGL(k_fk8, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, h->s0.p,
                     (long long)n, h->s1.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(poses, h->s1.p, (size_t)n * 12 * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_torque_ok(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                   int64_t n, int32_t torque_mode, double payload_mass, int32_t* ok) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!q || !ok))) return fail(-1, "bad arguments");
  if (torque_mode < 0 || torque_mode > 3) return fail(-1, "unknown torque mode");
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, q, n);
  if (!rc && qd) rc = upload7(h, h->s1, qd, n);
  if (!rc && qdd) rc = upload7(h, h->s2, qdd, n);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  if (rc) return rc;
  hipLaunchKernelGGL(TCMP_BY_MODE(k_torque, torque_mode), dim3(grid_for(n, 256)), dim3(256), 0,
                     h->stream, h->s0.p, qd ? h->s1.p : nullptr, qdd ? h->s2.p : nullptr,
                     (long long)n, payload_mass, h->i0.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ok, h->i0.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_check_configs(tcmp_handle* h, const double* q, int64_t n, int32_t* collides) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!q || !collides))) return fail(-1, "bad arguments");
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, q, n);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  if (rc) return rc;
  hipLaunchKernelGGL(h->mesh_kernels() ? k_check_configs<true> : k_check_configs<false>, dim3(grid_for(n, 256)), dim3(256), lds_bytes(h), h->stream, h->s0.p,
                     (long long)n, h->scene(), h->geo(), h->i0.p, 0);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(collides, h->i0.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

// panda_link0 against every obstacle of the scene (boxes, then user meshes) into h->base_pd
static int launch_base_pd(tcmp_handle* h) {
  const int nb = h->n_box + h->n_mesh;
  if (nb == 0) return 0;
  if (!h->base_geo.p) {
    std::vector<double> g((size_t)4 * (TCMP_BASE_NV + TCMP_BASE_NF + TCMP_BASE_NE), 0.0);
    double* gv = g.data();
    double* gn = gv + 4 * TCMP_BASE_NV;
    double* ge = gn + 4 * TCMP_BASE_NF;
    for (int i = 0; i < 4 * TCMP_BASE_NV; ++i) gv[i] = tcmp_base_verts[i];
    for (int i = 0; i < 4 * TCMP_BASE_NF; ++i) gn[i] = tcmp_base_planes[i];
    for (int i = 0; i < TCMP_BASE_NE; ++i) {
      const double* a = tcmp_base_verts + 4 * tcmp_base_edges[4 * i];
      const double* b = tcmp_base_verts + 4 * tcmp_base_edges[4 * i + 1];
      double e[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
      const double l = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
      for (int k = 0; k < 3; ++k) ge[4 * i + k] = e[k] / l;
    }
    if (int rc = h->base_geo.ensure(g.size())) return rc;
    HIPCHK(hipMemcpy(h->base_geo.p, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  if (int rc = h->base_pd.ensure((size_t)nb)) return rc;
  const double4* b4 = reinterpret_cast<const double4*>(h->base_geo.p);
  BaseGeo bg{b4, b4 + TCMP_BASE_NV, b4 + TCMP_BASE_NV + TCMP_BASE_NF};
  hipLaunchKernelGGL(k_base_pd, dim3(nb), dim3(kBaseThreads), 0, h->stream, h->scene(), bg,
                     h->n_box, h->base_pd.p);
  HIPCHK(hipGetLastError());
  return 0;
}

int tcmp_base_pd(tcmp_handle* h, double* pd, int32_t n) {
  TCMP_ENTER(h);
  if (n != h->n_box + h->n_mesh) return fail(-1, "n must be the scene's boxes + meshes");
  if (n == 0) return 0;
  if (!pd) return fail(-1, "bad arguments");
  if (int rc = launch_base_pd(h)) return rc;
  HIPCHK(hipMemcpyAsync(pd, h->base_pd.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_check_body(tcmp_handle* h, const double* q, int64_t n, int32_t* collides) {
  TCMP_ENTER(h);
  if (n < 0 || (n > 0 && (!q || !collides))) return fail(-1, "bad arguments");
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, q, n);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  rc = rc ? rc : launch_base_pd(h);
  if (rc) return rc;
  // robot vs obstacles only (pairwise_collision(robot, b) for b in obstacles): the arm's
  // self pairs of tcmp_set_self_collision are not part of the body-level check
  Scene sc = h->scene();
  sc.self_coll = 0;
  const bool mk = h->n_mesh > 0;
  hipLaunchKernelGGL(mk ? k_check_configs<true> : k_check_configs<false>,
                     dim3(grid_for(n, 256)), dim3(256),
                     mk ? stage_lds_bytes_lean(h->n_obs) : stage_lds_bytes(h->n_obs), h->stream,
                     h->s0.p, (long long)n, sc, h->geo(), h->i0.p, 1);
  HIPCHK(hipGetLastError());
  const int nb = h->n_box + h->n_mesh;
  if (nb) {
    hipLaunchKernelGGL(k_body_merge, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, h->i0.p,
                       (long long)n, h->base_pd.p, nb);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpyAsync(collides, h->i0.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_check_edges(tcmp_handle* h, const double* from, const double* to, int64_t n,
                     const double* resolutions, int32_t torque_mode, double payload_mass,
                     int32_t* n_safe, int32_t* n_steps, double* last) {
  TCMP_ENTER(h);
  if (n < 0 || n > INT_MAX || (n > 0 && (!from || !to || !n_safe || !n_steps || !last)))
    return fail(-1, "bad arguments");
  if (torque_mode < 0 || torque_mode > 3) return fail(-1, "unknown torque mode");
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, from, n);
  rc = rc ? rc : upload7(h, h->s1, to, n);
  rc = rc ? rc : h->s2.ensure((size_t)n * 8);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  rc = rc ? rc : h->i1.ensure((size_t)n);
  if (rc) return rc;
  PlanParams P = default_params();
  if (resolutions)
    for (int k = 0; k < 7; ++k) P.res[k] = resolutions[k];
  P.torque_mode = torque_mode;
  P.mass = payload_mass;
  if ((rc = h->erec.ensure((size_t)n * 8))) return rc;
  EdgeJob J{h->s0.p, nullptr, h->s1.p, (int)n, h->i0.p, h->i1.p, h->s2.p, nullptr, nullptr,
            h->erec.p};
  HIPCHK(hipMemcpyAsync(h->dPx, &P, sizeof(P), hipMemcpyHostToDevice, h->stream));
  if ((rc = launch_edges(h, J, h->dPx))) return rc;
  std::vector<double> tmp((size_t)n * 8);
  HIPCHK(hipMemcpyAsync(n_safe, h->i0.p, n * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(n_steps, h->i1.p, n * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(tmp.data(), h->s2.p, tmp.size() * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  for (long long i = 0; i < n; ++i)
    for (int k = 0; k < 7; ++k) last[7 * i + k] = tmp[8 * i + k];
  return 0;
}

int tcmp_nearest(tcmp_handle* h, const double* tree, int64_t T, const double* samples,
                 int64_t n, const double* weights, int32_t* idx) {
  TCMP_ENTER(h);
  if (T <= 0 || T > INT_MAX || n < 0 || n > INT_MAX || !tree || (n > 0 && (!samples || !idx)))
    return fail(-1, "bad arguments");
  if (n == 0) return 0;
  PlanParams P = default_params();
  bool uw = true;
  if (weights) {
    for (int k = 0; k < 7; ++k) {
      if (!(weights[k] > 0) || !std::isfinite(weights[k])) return fail(-1, "weights must be positive");
      P.w[k] = weights[k];
      uw &= weights[k] == weights[0];
    }
  }
  P.uniform_w = uw ? 1 : 0;
  // the scan's fp32 error terms need a bound on |q| (8 covers the joint-limit box)
  double cmax = 8.0;
  for (long long i = 0; i < 7 * T; ++i) {
    if (!std::isfinite(tree[i])) return fail(-1, "non-finite tree coordinate");
    cmax = std::max(cmax, fabs(tree[i]));
  }
  for (long long i = 0; i < 7 * n; ++i) {
    if (!std::isfinite(samples[i])) return fail(-1, "non-finite sample coordinate");
    cmax = std::max(cmax, fabs(samples[i]));
  }
  P.nn_cmax = cmax * (1.0 + 1e-6);
  int rc = upload7(h, h->s0, tree, T);
  rc = rc ? rc : upload7(h, h->s1, samples, n);
  rc = rc ? rc : h->i0.ensure((size_t)n);
  rc = rc ? rc : h->s2.ensure((size_t)n);
  rc = rc ? rc : ensure_index(h, (size_t)T, (size_t)n);
  if (rc) return rc;
  DevState s;
  memset(&s, 0, sizeof(s));
  s.n_nodes = T;
  HIPCHK(hipMemcpyAsync(h->st_nn, &s, sizeof(s), hipMemcpyHostToDevice, h->stream));
  const size_t ev_before = h->ev_used.size(), rec_before = h->ev_rec.size();
  HIPCHK(hipMemcpyAsync(h->dPx, &P, sizeof(P), hipMemcpyHostToDevice, h->stream));
  rc = launch_nearest(h, P, h->dPx, h->st_nn, h->s0.p, T, h->s1.p, (int)n, h->i0.p, h->s2.p,
                      nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(idx, h->i0.p, n * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  // the scan's timing events belong to no plan
  h->ev_used.resize(ev_before);
  while (h->ev_rec.size() > rec_before) {
    h->ev_pool.push_back(h->ev_rec.back());
    h->ev_rec.pop_back();
  }
  return 0;
}

int tcmp_minjerk(tcmp_handle* h, const double* waypoints, int64_t n_wp, int64_t ni, double* q,
                 double* qd, double* qdd) {
  TCMP_ENTER(h);
  if (ni <= 0) return fail(-1, "Invalid number of intervals chosen (must be greater than 0)");
  if (n_wp < 1 || !waypoints) return fail(-1, "bad arguments");
  const long long K = (n_wp - 1) * ni;
  if (K == 0) return 0;
  if (!q || !qd || !qdd) return fail(-1, "bad arguments");
  int rc = h->s0.ensure((size_t)n_wp * 7);
  rc = rc ? rc : h->s1.ensure((size_t)K * 7);
  rc = rc ? rc : h->s2.ensure((size_t)K * 7);
  rc = rc ? rc : h->s3.ensure((size_t)K * 7);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h->s0.p, waypoints, n_wp * 7 * sizeof(double), hipMemcpyHostToDevice,
                        h->stream));
  hipLaunchKernelGGL(k_minjerk, dim3(std::min<unsigned>(grid_for(K, 256), 4096)), dim3(256), 0,
                     h->stream, h->s0.p, (long long)n_wp, (long long)ni, h->s1.p, h->s2.p, h->s3.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(q, h->s1.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(qd, h->s2.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(qdd, h->s3.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_validate_traj(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                       int64_t n, int32_t torque_mode, double payload_mass, int64_t* first_fail,
                       double* tau) {
  TCMP_ENTER(h);
  if (n < 0 || !first_fail || (n > 0 && (!q || !qd || !qdd))) return fail(-1, "bad arguments");
  if (torque_mode < 0 || torque_mode > 3) return fail(-1, "unknown torque mode");
  *first_fail = -1;
  if (n == 0) return 0;
  int rc = upload7(h, h->s0, q, n);
  rc = rc ? rc : upload7(h, h->s1, qd, n);
  rc = rc ? rc : upload7(h, h->s2, qdd, n);
  rc = rc ? rc : h->s3.ensure((size_t)n * 7);
  rc = rc ? rc : h->u0.ensure(1);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(h->u0.p, 0xff, sizeof(unsigned long long), h->stream));
  hipLaunchKernelGGL(TCMP_BY_MODE(k_validate, torque_mode), dim3(grid_for(n, 256)), dim3(256), 0,
                     h->stream, h->s0.p, h->s1.p, h->s2.p, (long long)n, payload_mass, h->u0.p);
  HIPCHK(hipGetLastError());
  if (tau) {
    // Conf.torques: rne without payload (utils.py:3376)
    hipLaunchKernelGGL(k_rne, dim3(grid_for(n, 256)), dim3(256), 0, h->stream, h->s0.p, h->s1.p,
                       h->s2.p, (long long)n, 0.0, h->s3.p);
    HIPCHK(hipGetLastError());
  }
  unsigned long long ff = 0;
  HIPCHK(hipMemcpyAsync(&ff, h->u0.p, sizeof(ff), hipMemcpyDeviceToHost, h->stream));
  if (tau)
    HIPCHK(hipMemcpyAsync(tau, h->s3.p, n * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  *first_fail = ff == ~0ull ? -1 : (int64_t)ff;
  return 0;
}

// ---- planner ----------------------------------------------------------------------------
}  // extern "C"

namespace {

// tcmp_plan_begin in two halves: everything up to the queued start / goal check and uploads,
// then the one host wait and the status -- so that tcmp_plan_begin_many waits once for many
// a plan's initial device state from the begin block (one upload of the handle's pinned Pin):
// the root node (OptimalNode(start), rrt_star.py:155), the plan state and parameters
__global__ void k_plan_init(const tcmp_handle::Pin* b, double* cfg, double* tgt, int* parent,
                            int2* meta, DevState* st, PlanParams* dP) {
  const int t = threadIdx.x;
  if (t < 8) {
    cfg[t] = b->root[t];
    tgt[t] = b->root[t];
  }
  if (t == 0) {
    parent[0] = b->m1;
    meta[0] = b->z;
  }
  const unsigned* s = reinterpret_cast<const unsigned*>(&b->st);
  unsigned* d = reinterpret_cast<unsigned*>(st);
  for (int i = t; i < (int)(sizeof(DevState) / 4); i += blockDim.x) d[i] = s[i];
  const unsigned* sp = reinterpret_cast<const unsigned*>(&b->P);
  unsigned* dp = reinterpret_cast<unsigned*>(dP);
  for (int i = t; i < (int)(sizeof(PlanParams) / 4); i += blockDim.x) dp[i] = sp[i];
}

int plan_begin_launch(tcmp_handle* h, const tcmp_plan_cfg* cfg, tcmp_plan_result* result) {
  if (!cfg || !result) return fail(-1, "null cfg/result");
  if (cfg->torque_mode < 0 || cfg->torque_mode > 3) return fail(-1, "unknown torque mode");
  if (cfg->max_nodes < 2 || cfg->max_batch < 1) return fail(-1, "bad capacities");
  memset(result, 0, sizeof(*result));
  result->goal_node = -1;
  result->first_fail = -1;
  PlanParams P = default_params();
  for (int k = 0; k < 7; ++k) {
    P.start[k] = cfg->start[k];
    P.goal[k] = cfg->goal[k];
    P.w[k] = cfg->weights[k];
    P.res[k] = cfg->resolutions[k];
  }
  P.uniform_w = 1;
  for (int k = 1; k < 7; ++k) P.uniform_w &= P.w[k] == P.w[0];
  P.radius = cfg->radius;
  P.goal_prob = cfg->goal_probability;
  P.goal_tol = cfg->goal_tolerance;
  P.mass = cfg->payload_mass;
  P.exec_time = cfg->execution_time;
  P.seed = cfg->seed;
  P.torque_mode = cfg->torque_mode;
  P.max_nodes = cfg->max_nodes;
  h->P = P;
  const size_t N = (size_t)cfg->max_nodes, B = (size_t)cfg->max_batch;
  int rc = h->cfg.ensure(N * 8);
  rc = rc ? rc : h->tgt.ensure(N * 8);
  rc = rc ? rc : h->parent.ensure(N);
  rc = rc ? rc : h->meta.ensure(N);
  rc = rc ? rc : h->chain.ensure(N);
  rc = rc ? rc : h->cand.ensure(B * 8);
  rc = rc ? rc : h->last.ensure(B * 8);
  rc = rc ? rc : h->erec.ensure(B * 8);
  rc = rc ? rc : h->cgoal.ensure(B);
  rc = rc ? rc : h->nn.ensure(B);
  rc = rc ? rc : h->nsafe.ensure(B);
  rc = rc ? rc : h->nsteps.ensure(B);
  rc = rc ? rc : h->nbr.ensure(B * kNbrCap);
  rc = rc ? rc : h->ncount.ensure(B);
  rc = rc ? rc : h->second.ensure(B);
  rc = rc ? rc : h->rwlist.ensure(B);
  rc = rc ? rc : h->nnscore.ensure(B);
  rc = rc ? rc : h->bcount.ensure(B / 256 + 1);
  rc = rc ? rc : h->boff.ensure(B / 256 + 1);
  rc = rc ? rc : ensure_index(h, N, B);
  rc = rc ? rc : h->i0.ensure(2);
  if (rc) return rc;
  h->max_batch = cfg->max_batch;
  h->samples_issued = 0;
  h->collect_events();
  for (double& m : h->ms) m = 0;
  h->launches_nearest = 0;
  h->fused_plans = 0;
  h->launches_scan = 0;
  h->graph_launches = 0;
  // the finish's buffers, sized here so that tcmp_plan_finish needs one host wait: waypoints
  // (bounded by the chain's total n_safe; generous, checked on the device) and trajectory
  // rows K = (W - 1) * floor(exec_time * 1000 / W) < exec_time * 1000 (k_retrace)
  {
    const size_t wcap = std::max<size_t>(1024, N * 64);
    rc = h->wp.ensure(std::min<size_t>(wcap, (size_t)1 << 26) * 7);
    const double kc = std::max(0.0, cfg->execution_time) * 1000.0 + 2.0;
    h->kcap = (long long)std::min(kc, (double)(1 << 22));
    rc = rc ? rc : h->tq.ensure((size_t)h->kcap * 7);
    rc = rc ? rc : h->tqd.ensure((size_t)h->kcap * 7);
    rc = rc ? rc : h->tqdd.ensure((size_t)h->kcap * 7);
    rc = rc ? rc : h->tpsg.ensure((size_t)h->kcap);
    rc = rc ? rc : h->ttau.ensure((size_t)h->kcap * 7);
    // (grown only when a larger execution time raises kcap: the first plan of an engine)
    const size_t fb = (size_t)h->kcap * 29 * sizeof(double);
    if (!rc && h->fetch_pin_n < fb) {
      if (h->fetch_pin) HIPCHK(hipHostFree(h->fetch_pin));
      h->fetch_pin = nullptr;
      h->fetch_pin_n = 0;
      HIPCHK(hipHostMalloc(&h->fetch_pin, fb));
      h->fetch_pin_n = fb;
    }
    rc = rc ? rc : h->s0.ensure(16);
    rc = rc ? rc : h->i0.ensure(2);
    if (rc) return rc;
  }
  h->fin_W = 0;
  h->fin_K = 0;
  // one upload and one host wait: the handle's pinned block holds the start / goal rows, the
  // root, the plan state and parameters; k_plan_init scatters them on the device
  if (int rc2 = h->dpin.ensure(sizeof(tcmp_handle::Pin))) return rc2;
  tcmp_handle::Pin& pn = *h->pin;
  memset(pn.sg, 0, sizeof(pn.sg));
  memcpy(pn.sg, cfg->start, sizeof(double) * 7);
  memcpy(pn.sg + 8, cfg->goal, sizeof(double) * 7);
  memset(pn.root, 0, sizeof(pn.root));
  for (int k = 0; k < 7; ++k) pn.root[k] = cfg->start[k];
  pn.m1 = -1;
  pn.z = make_int2(0, 0);
  memset(&pn.st, 0, sizeof(pn.st));
  pn.st.n_nodes = 1;
  pn.st.goal_node = -1;
  pn.st.first_fail = -1;
  pn.st.round_goal = INT_MAX;
  pn.P = h->P;
  const tcmp_handle::Pin* dpn = reinterpret_cast<const tcmp_handle::Pin*>(h->dpin.p);
  HIPCHK(hipMemcpyAsync(h->dpin.p, &pn, sizeof(pn), hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_plan_init, dim3(1), dim3(128), 0, h->stream, dpn, h->cfg.p, h->tgt.p,
                     h->parent.p, h->meta.p, h->st, h->dP);
  // collision(start) or collision(goal) (rrt_star.py:152)
  hipLaunchKernelGGL(h->mesh_kernels() ? k_check_configs<true> : k_check_configs<false>,
                     dim3(1), dim3(256), lds_bytes(h), h->stream,
                     reinterpret_cast<const double*>(h->dpin.p + offsetof(tcmp_handle::Pin, sg)), 2LL, h->scene(),
                     h->geo(), h->i0.p, 0);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(pn.coll, h->i0.p, 2 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  return 0;
}

int plan_begin_complete(tcmp_handle* h, tcmp_plan_result* result) {
  tcmp_handle::Pin& pn = *h->pin;
  if (int rc_s = sync_stream(h)) return rc_s;
  h->plan_open = true;
  result->n_nodes = 1;
  result->status = (pn.coll[0] || pn.coll[1]) ? TCMP_PLAN_START_GOAL_COLLISION : TCMP_PLAN_OK;
  if (result->status) h->plan_open = false;
  return 0;
}

}  // namespace

extern "C" {

int tcmp_plan_begin(tcmp_handle* h, const tcmp_plan_cfg* cfg, tcmp_plan_result* result) {
  TCMP_ENTER(h);
  if (int rc = plan_begin_launch(h, cfg, result)) return rc;
  return plan_begin_complete(h, result);
}

int tcmp_plan_begin_many(tcmp_handle* const* hs, int32_t n, const tcmp_plan_cfg* cfgs,
                         tcmp_plan_result* results) {
  Entry entry;
  if (!hs || n < 1 || !cfgs || !results) return fail(-1, "bad arguments");
  for (int q = 0; q < n; ++q) {
    int rc = set_dev(hs[q]);
    rc = rc ? rc : plan_begin_launch(hs[q], cfgs + q, results + q);
    if (rc) {
      // the engines already launched have begin work queued (the device-to-host copy into
      // their pinned block among it): wait for it, so that no later begin rewrites that block
      // while the copy is pending; their plans stay closed
      const std::string why = "plan " + std::to_string(q) + ": " + tcmp_last_error();
      for (int p = 0; p < q; ++p) {
        if (set_dev(hs[p]) == 0) (void)sync_stream(hs[p]);
        hs[p]->plan_open = false;
      }
      return fail(rc, why);
    }
  }
  for (int q = 0; q < n; ++q) {
    if (int rc = set_dev(hs[q])) return rc;
    if (int rc = plan_begin_complete(hs[q], results + q))
      return fail(rc, "plan " + std::to_string(q) + ": " + tcmp_last_error());
  }
  return 0;
}

// identity of a captured round sequence: its shape and everything its nodes bake in
static unsigned long long round_graph_key(const tcmp_handle* h, long long n_samples, int batch) {
  unsigned long long x = 1469598103934665603ull;
  auto mix = [&](unsigned long long v) {
    for (int i = 0; i < 8; ++i) {
      x ^= (v >> (8 * i)) & 0xffull;
      x *= 1099511628211ull;
    }
  };
  auto mixp = [&](const void* p) { mix((unsigned long long)(uintptr_t)p); };
  mix((unsigned long long)h->samples_issued);
  mix((unsigned long long)n_samples);
  mix((unsigned long long)batch);
  mix((unsigned long long)h->P.uniform_w);
  mix((unsigned long long)h->mesh_kernels());
  mix((unsigned long long)lds_bytes(h));
  mix((unsigned long long)h->nn_waves_per_cu);
  mix((unsigned long long)h->nn_cand_bits);
  mix((unsigned long long)h->edge_split);
  mix((unsigned long long)h->nn_cand_count_bits);
  mix((unsigned long long)h->sort_tmp.n);
  mix((unsigned long long)h->timing);
  mix((unsigned long long)h->edge_wps);
  mix((unsigned long long)h->cu_count);
  for (const void* p : {(const void*)h->cfg.p, (const void*)h->tgt.p, (const void*)h->parent.p,
                        (const void*)h->meta.p, (const void*)h->cand.p, (const void*)h->last.p,
                        (const void*)h->cgoal.p, (const void*)h->nn.p, (const void*)h->nsafe.p,
                        (const void*)h->nsteps.p, (const void*)h->nbr.p, (const void*)h->ncount.p,
                        (const void*)h->second.p, (const void*)h->rwlist.p, (const void*)h->nnscore.p,
                        (const void*)h->nkeys_in.p, (const void*)h->skeys.p, (const void*)h->nvals_in.p,
                        (const void*)h->svals.p, (const void*)h->stree.p, (const void*)h->srow.p,
                        (const void*)h->cboxf.p, (const void*)h->sboxf.p, (const void*)h->bboxf.p,
                        (const void*)h->cflag.p, (const void*)h->cid.p, (const void*)h->cstart.p,
                        (const void*)h->sflag.p, (const void*)h->sid.p, (const void*)h->sstart.p,
                        (const void*)h->ckey.p, (const void*)h->chome.p, (const void*)h->ckeys_in.p,
                        (const void*)h->cs_hist.p, (const void*)h->cvals_in.p, (const void*)h->cperm.p,
                        (const void*)h->cs_hoff.p, (const void*)h->ckeys.p,
                        (const void*)h->sort_tmp.p, (const void*)h->bcount.p, (const void*)h->boff.p,
                        (const void*)h->erec.p,
                        (const void*)h->st, (const void*)h->dP})
    mixp(p);
  const Scene sc = h->scene();
  const Geo g = h->geo();
  const unsigned char* b = reinterpret_cast<const unsigned char*>(&sc);
  for (size_t i = 0; i < sizeof(sc); ++i) mix(b[i]);
  b = reinterpret_cast<const unsigned char*>(&g);
  for (size_t i = 0; i < sizeof(g); ++i) mix(b[i]);
  return x;
}

// ---- one round, in phases.  A lone engine runs them back to back (plan_round_impl); the
// engines of a shared-tree round (tcmp_plan_run_shared / tcmp_plan_run_group) each own a
// consecutive range of the round's lanes and exchange four small things between the phases:
// the round's goal lane, their accepted-edge counts, the lowest goal-reaching new node, and
// finally their new node records -- so every engine ends the round with the tree a lone
// engine would have built from the whole round.
//
// sample: the host's draws (samples != NULL), or Philox lanes [lo, lo + nb) of a round of B
static int round_sample(tcmp_handle* h, const double* samples, const uint8_t* is_goal, int32_t nb,
                        long long lo, long long B) {
  if (samples) {
    std::vector<double> tmp((size_t)nb * 8, 0.0);
    double cmax = 0.0;
    for (int j = 0; j < nb; ++j)
      for (int k = 0; k < 7; ++k) {
        const double x = samples[7 * j + k];
        if (!std::isfinite(x)) return fail(-1, "non-finite sample coordinate");
        cmax = std::max(cmax, fabs(x));
        tmp[8 * j + k] = x;
      }
    if (cmax > h->P.nn_cmax) {
      // a caller's sampler reached outside the joint-limit box: widen the nearest scan's
      // fp32 error terms (tcmp_nn32.h) so it stays exact
      h->P.nn_cmax = cmax * (1.0 + 1e-6);
      HIPCHK(hipMemcpyAsync(h->dP, &h->P, sizeof(PlanParams), hipMemcpyHostToDevice, h->stream));
    }
    HIPCHK(hipMemcpyAsync(h->cand.p, tmp.data(), tmp.size() * sizeof(double),
                          hipMemcpyHostToDevice, h->stream));
    std::vector<unsigned char> g((size_t)nb, 0);
    if (is_goal)
      for (int j = 0; j < nb; ++j) g[j] = is_goal[j] ? 1 : 0;
    HIPCHK(hipMemcpyAsync(h->cgoal.p, g.data(), nb, hipMemcpyHostToDevice, h->stream));
    if (int rc_s = sync_stream(h)) return rc_s;  // host staging buffers go out of scope
  } else {
    hipLaunchKernelGGL(k_sample, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, h->dP, h->st,
                       (long long)h->samples_issued + lo, nb, h->cand.p, h->cgoal.p);
    HIPCHK(hipGetLastError());
  }
  h->samples_issued += B;
  return 0;
}

// goal lane fix, nearest, extend (edge kernel), and the count/scan half of the insertion
static int round_search(tcmp_handle* h, bool device_samples, int32_t nb, long long B) {
  const PlanParams& P = h->P;
  hipEvent_t e0;
  h->mark_begin(F_NEAREST, &e0);
  const GoalFix gf{device_samples ? h->cand.p : nullptr, h->cgoal.p};
  const int nblk = (int)grid_for(nb, 256);
  if (int rc = h->bcount.ensure(nblk)) return rc;
  if (int rc = h->boff.ensure(nblk)) return rc;
  // the snapshot holds at most 1 + (samples issued before this round) nodes
  hipEvent_t e1 = nullptr;  // the scan's end event also ends the family and begins the edges
  {
    const long long T_bound = 1 + h->samples_issued - B;
    if (int rc = launch_nearest(h, P, h->dP, h->st, h->cfg.p, T_bound, h->cand.p, nb, h->nn.p,
                                h->second.p, h->nnscore.p, &e1, gf, h->bcount.p))
      return rc;
  }
  h->last_nb = nb;
  if (!e1) e1 = h->mark();
  h->span(F_NEAREST, e0, e1);
  h->launches_nearest++;
  EdgeJob J{h->cfg.p, h->nn.p, h->cand.p, nb, h->nsafe.p, h->nsteps.p, h->last.p, nullptr,
            nullptr, h->erec.p};
  if (nb >= kEdgeOrderMin) {
    // longest planned edges first (the persistent lanes then finish together): a counting
    // sort by 255 - min(n, 255) in the candidate-sort buffers, which the nearest scan is done with
    hipLaunchKernelGGL(k_edge_order_keys, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, h->dP,
                       h->cfg.p, h->nn.p, h->cand.p, nb, h->cvals_in.p, h->cs_hist.p);
    HIPCHK(hipGetLastError());
    if (int rc = count_sort(h, h->cvals_in.p, nb, 256, h->cperm.p, true)) return rc;
    J.order = h->cperm.p;
  }
  // k_edges counts the accepted edges per 256 lanes (bcount, cleared by the nearest search's
  // first kernel); the scan turns them into the insertion offsets
  J.accepted = h->bcount.p;
  hipEvent_t ek = nullptr;
  if (int rc = launch_edges(h, J, h->dP, false, &ek)) return rc;
  h->span(F_EDGE_PREP, e1, ek);
  h->ins_ev = h->mark_end(F_EDGES, ek);
  hipLaunchKernelGGL(k_ins_scan, dim3(1), dim3(1024), 0, h->stream, h->st, h->bcount.p, nblk,
                     h->boff.p);
  HIPCHK(hipGetLastError());
  return 0;
}

// the new nodes, in lane order after the snapshot (and after the lower ranks' new nodes)
static int round_write(tcmp_handle* h, int32_t nb) {
  Tree tr{h->cfg.p, h->parent.p, h->tgt.p, h->meta.p};
  const int nblk = (int)grid_for(nb, 256);
  hipLaunchKernelGGL(k_ins_write, dim3(nblk), dim3(256), 0, h->stream, h->dP, h->st, tr, h->nn.p,
                     h->cand.p, h->cgoal.p, h->nsafe.p, h->nsteps.p, h->last.p, nb, h->boff.p,
                     h->second.p, h->rwlist.p);
  HIPCHK(hipGetLastError());
  return 0;
}

// node count / goal bookkeeping, then the rewire of this engine's new nodes
static int round_finish(tcmp_handle* h, int32_t nb) {
  Tree tr{h->cfg.p, h->parent.p, h->tgt.p, h->meta.p};
  hipLaunchKernelGGL(k_ins_final, dim3(1), dim3(1), 0, h->stream, h->dP, h->st, nb);
  HIPCHK(hipGetLastError());
  const hipEvent_t e0 = h->mark_end(F_INSERT, h->ins_ev);
  hipLaunchKernelGGL(k_rewire_scan, dim3(grid_for(nb, 256)), dim3(256), 0, h->stream, h->dP, h->st,
                     tr, h->rwlist.p, h->nbr.p, h->ncount.p);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(h->mesh_kernels() ? k_rewire_apply<true> : k_rewire_apply<false>, dim3(grid_for(nb, 256)), dim3(256), lds_bytes(h), h->stream, h->dP, h->st,
                     tr, h->rwlist.p, h->nbr.p, h->ncount.p, h->scene(), h->geo());
  HIPCHK(hipGetLastError());
  h->mark_end(F_REWIRE, e0);
  return 0;
}

static int plan_round_impl(tcmp_handle* h, const double* samples, const uint8_t* is_goal,
                           int32_t nb) {
  if (int rc = round_sample(h, samples, is_goal, nb, 0, nb)) return rc;
  if (int rc = round_search(h, samples == nullptr, nb, nb)) return rc;
  if (int rc = round_write(h, nb)) return rc;
  return round_finish(h, nb);
}

// ---- shared-tree rounds: the exchanges ------------------------------------------------------
// xch (int64, per engine): [0] the round's goal lane (global lane index, LLONG_MAX for none),
// [1] this engine's accepted edges, [2] the lowest goal-reaching new node, [3 + q] engine q's
// accepted edges (gathered).
__global__ void k_sr_put_lane(DevState* st, long long lo, long long* xch) {
  xch[0] = st->round_goal == INT_MAX ? LLONG_MAX : lo + (long long)st->round_goal;
}
__global__ void k_sr_take_lane(DevState* st, long long lo, int nb, const long long* xch) {
  const long long g = xch[0];
  st->round_goal = (g >= lo && g < lo + nb) ? (int)(g - lo) : INT_MAX;
}
__global__ void k_sr_put_count(const DevState* st, long long* xch) { xch[1] = st->ins_total; }
__global__ void k_sr_take_counts(DevState* st, int rank, int world, const long long* xch) {
  long long off = 0, all = 0;
  for (int q = 0; q < world; ++q) {
    if (q < rank) off += xch[3 + q];
    all += xch[3 + q];
  }
  st->ins_off = off;
  st->ins_all = all;
}
__global__ void k_sr_put_goal(const DevState* st, long long* xch) { xch[2] = st->ins_goal; }
__global__ void k_sr_take_goal(DevState* st, const long long* xch) { st->ins_goal = xch[2]; }

// lanes of engine q in a round of B lanes over W engines
static inline long long sr_lo(long long B, int q, int W) { return B * q / W; }

// a host-side copy of the tree size, advanced like k_ins_final does
static int sr_tree_size(tcmp_handle* h, long long* T) {
  HIPCHK(hipMemcpyAsync(T, &h->st->n_nodes, sizeof(*T), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

static int sr_check(tcmp_handle* h, long long n_samples, int batch, int world) {
  if (!h->plan_open) return fail(-1, "no open plan (tcmp_plan_begin first)");
  if (batch < world) return fail(-1, "a shared-tree round needs at least one lane per engine");
  if ((batch + world - 1) / world > h->max_batch)
    return fail(-1, "batch / engines exceeds the plan's max_batch");
  if (h->samples_issued + n_samples + 1 > h->P.max_nodes) return fail(-3, "tree capacity exceeded");
  return h->xch.ensure(3 + (size_t)world);
}
int tcmp_plan_round(tcmp_handle* h, const double* samples, const uint8_t* is_goal, int32_t nb,
                    int32_t* goal_found) {
  TCMP_ENTER(h);
  if (!h->plan_open) return fail(-1, "no open plan (tcmp_plan_begin first)");
  if (nb < 1 || nb > h->max_batch) return fail(-1, "batch size out of range");
  if (h->samples_issued + nb + 1 > h->P.max_nodes) return fail(-3, "tree capacity exceeded");
  if (int rc = plan_round_impl(h, samples, is_goal, nb)) return rc;
  if (goal_found) {
    long long g = -1;
    HIPCHK(hipMemcpyAsync(&g, &h->st->goal_node, sizeof(g), hipMemcpyDeviceToHost, h->stream));
    if (int rc_s = sync_stream(h)) return rc_s;
    *goal_found = g >= 0;
  }
  return 0;
}

// The rounds of one engine in a shared tree, over any transport (tcmp_dist_internal.h): the
// RCCL communicator of tcmp_plan_run_shared and the host-thread group of tcmp_plan_run_group
// run this same loop, so the group tests on one GPU cover the multi-GPU round logic.
static int shared_rounds(tcmp_handle* h, tcmp_dist::RoundExchange& X, long long n_samples,
                         int batch) {
  const int W = X.world(), r = X.rank();
  long long T = 0;
  if (int rc = sr_tree_size(h, &T)) return rc;
  std::vector<long long> cnt((size_t)W, 0);
  long long* x = h->xch.p;
  int64_t* x64 = reinterpret_cast<int64_t*>(x);
  for (long long left = n_samples; left > 0;) {
    const long long B = std::min<long long>(left, batch);
    const long long lo = sr_lo(B, r, W);
    const int nb = (int)(sr_lo(B, r + 1, W) - lo);
    if (int rc = round_sample(h, nullptr, nullptr, nb, lo, B)) return rc;
    // the round's goal lane: the lowest selecting lane of the whole round (k_sample's rule)
    hipLaunchKernelGGL(k_sr_put_lane, dim3(1), dim3(1), 0, h->stream, h->st, lo, x);
    if (int rc = X.min_i64(x64, 1, h->stream)) return rc;
    hipLaunchKernelGGL(k_sr_take_lane, dim3(1), dim3(1), 0, h->stream, h->st, lo, nb, x);
    if (int rc = round_search(h, true, nb, B)) return rc;
    // accepted edges of every rank: this rank's insertion offset and the round's total
    hipLaunchKernelGGL(k_sr_put_count, dim3(1), dim3(1), 0, h->stream, h->st, x);
    if (int rc = X.allgather_i64(x64 + 1, x64 + 3, 1, h->stream)) return rc;
    hipLaunchKernelGGL(k_sr_take_counts, dim3(1), dim3(1), 0, h->stream, h->st, r, W, x);
    HIPCHK(hipMemcpyAsync(cnt.data(), x + 3, W * sizeof(long long), hipMemcpyDeviceToHost,
                          h->stream));
    if (int rc = round_write(h, nb)) return rc;
    // the lowest goal-reaching new node of the round
    hipLaunchKernelGGL(k_sr_put_goal, dim3(1), dim3(1), 0, h->stream, h->st, x);
    if (int rc = X.min_i64(x64 + 2, 1, h->stream)) return rc;
    hipLaunchKernelGGL(k_sr_take_goal, dim3(1), dim3(1), 0, h->stream, h->st, x);
    if (int rc = round_finish(h, nb)) return rc;
    if (int rc_s = sync_stream(h)) return rc_s;  // cnt
    long long all = 0;
    for (long long v : cnt) all += v;
    if (T + all <= h->P.max_nodes) {
      // every rank's new nodes (rewired) to every other rank, in place
      std::vector<tcmp_dist::Bcast> ops;
      long long off = T;
      for (int q = 0; q < W; ++q) {
        const size_t k = (size_t)cnt[q];
        if (k) {
          ops.push_back({h->cfg.p + 8 * (size_t)off, k * 8 * sizeof(double), q});
          ops.push_back({h->tgt.p + 8 * (size_t)off, k * 8 * sizeof(double), q});
          ops.push_back({h->parent.p + off, k * sizeof(int), q});
          ops.push_back({h->meta.p + off, k * sizeof(int2), q});
        }
        off += cnt[q];
      }
      if (int rc = X.bcast(ops.data(), (int)ops.size(), h->stream)) return rc;
      T += all;
    }
    left -= B;
  }
  return 0;
}

namespace {

// Engines of one process on host threads: each exchange is a host barrier around device
// copies (values through pinned host slots, node records peer to peer).  A failing engine
// aborts the group so no thread waits on a barrier that can never fill.
struct GroupState {
  explicit GroupState(int n) : n(n), vals((size_t)n * 8), ops((size_t)n) {}
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long long gen = 0;
  bool aborted = false;
  std::vector<int64_t> vals;                       // n x (up to 8) posted values
  std::vector<const tcmp_dist::Bcast*> ops;        // each engine's broadcast list
  int barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return -1;
    const long long g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return 0;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return aborted ? -1 : 0;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

class GroupExchange : public tcmp_dist::RoundExchange {
 public:
  GroupExchange(GroupState* g, int rank) : g_(g), r_(rank) {}
  int rank() const override { return r_; }
  int world() const override { return g_->n; }
  int min_i64(int64_t* d, int n, hipStream_t s) override {
    if (n > 8) return fail(-1, "group exchange: too many values");
    if (int rc = post(d, n, s)) return rc;
    std::vector<int64_t> m((size_t)n, LLONG_MAX);
    for (int q = 0; q < g_->n; ++q)
      for (int i = 0; i < n; ++i) m[i] = std::min(m[i], g_->vals[8 * q + i]);
    if (g_->barrier()) return fail(-1, "group exchange aborted");  // all have read vals
    HIPCHK(hipMemcpyAsync(d, m.data(), (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
  }
  int allgather_i64(const int64_t* send, int64_t* recv, int n, hipStream_t s) override {
    if (n > 8) return fail(-1, "group exchange: too many values");
    if (int rc = post(send, n, s)) return rc;
    std::vector<int64_t> all((size_t)g_->n * n);
    for (int q = 0; q < g_->n; ++q)
      for (int i = 0; i < n; ++i) all[(size_t)q * n + i] = g_->vals[8 * q + i];
    if (g_->barrier()) return fail(-1, "group exchange aborted");
    HIPCHK(hipMemcpyAsync(recv, all.data(), all.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
  }
  int bcast(const tcmp_dist::Bcast* ops, int n_ops, hipStream_t s) override {
    // the roots' ranges are final once every engine's stream has drained
    HIPCHK(hipStreamSynchronize(s));
    g_->ops[r_] = ops;
    if (g_->barrier()) return fail(-1, "group exchange aborted");
    for (int i = 0; i < n_ops; ++i) {
      const int root = ops[i].root;
      if (root == r_ || ops[i].bytes == 0) continue;
      HIPCHK(hipMemcpyAsync(ops[i].ptr, g_->ops[root][i].ptr, ops[i].bytes, hipMemcpyDefault, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    // nobody reuses its list (or writes the ranges) before every copy has landed
    if (g_->barrier()) return fail(-1, "group exchange aborted");
    return 0;
  }

 private:
  // this engine's n device values into its host slot, then wait for every engine's
  int post(const int64_t* d, int n, hipStream_t s) {
    int64_t v[8];
    HIPCHK(hipMemcpyAsync(v, d, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i) g_->vals[8 * r_ + i] = v[i];
    if (g_->barrier()) return fail(-1, "group exchange aborted");
    return 0;
  }
  GroupState* g_;
  int r_;
};

}  // namespace

int tcmp_plan_run_shared(tcmp_handle* h, tcmp_comm* c, int64_t n_samples, int32_t batch) {
  TCMP_ENTER(h);
  if (!c) return fail(-1, "null comm");
  const int W = tcmp_dist::world(c);
  if (W == 1) return tcmp_plan_run(h, n_samples, batch);
  if (int rc = sr_check(h, n_samples, batch, W)) return rc;
  tcmp_dist::RcclExchange X(c);
  return shared_rounds(h, X, n_samples, batch);
}

int tcmp_plan_run_group(tcmp_handle* const* hs, int32_t n, int64_t n_samples, int32_t batch) {
  Entry entry;  // the engines' threads below run inside this entry (they take no lock)
  if (!hs || n < 1) return fail(-1, "bad arguments");
  if (n == 1) return tcmp_plan_run(hs[0], n_samples, batch);
  for (int q = 0; q < n; ++q) {
    if (!hs[q]) return fail(-1, "null handle");
    for (int p = 0; p < q; ++p)
      if (hs[p] == hs[q]) return fail(-1, "the same engine twice in a group");
    if (int rc = set_dev(hs[q])) return rc;
    if (int rc = sr_check(hs[q], n_samples, batch, n)) return rc;
    if (hs[q]->samples_issued != hs[0]->samples_issued)
      return fail(-1, "the engines' plans are not at the same round");
  }
  GroupState g(n);
  std::vector<int> rc((size_t)n, 0);
  std::vector<std::string> err((size_t)n);
  std::vector<std::thread> th;
  th.reserve(n);
  for (int q = 0; q < n; ++q)
    th.emplace_back([&, q] {
      GroupExchange X(&g, q);
      int r = set_dev(hs[q]);
      if (!r) r = shared_rounds(hs[q], X, n_samples, batch);
      if (r) {
        rc[q] = r;
        err[q] = tcmp_last_error();  // the error string is thread-local
        g.abort();
      }
    });
  for (auto& t : th) t.join();
  // report the first engine that failed on its own (not one that only saw the abort)
  int first = -1;
  for (int q = 0; q < n; ++q)
    if (rc[q] && err[q].find("aborted") == std::string::npos) { first = q; break; }
  if (first < 0)
    for (int q = 0; q < n; ++q)
      if (rc[q]) { first = q; break; }
  if (first >= 0) return fail(rc[first], "engine " + std::to_string(first) + ": " + err[first]);
  return 0;
}

int tcmp_plan_goal(tcmp_handle* h, int64_t* node, double* cost) {
  TCMP_ENTER(h);
  if (!node) return fail(-1, "null node");
  if (!h->plan_open) return fail(-1, "no open plan (tcmp_plan_begin first)");
  long long g = -1;
  HIPCHK(hipMemcpyAsync(&g, &h->st->goal_node, sizeof(g), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  *node = g;
  if (cost) {
    double c = INFINITY;
    if (g >= 0) {
      HIPCHK(hipMemcpyAsync(&c, h->cfg.p + 8 * (size_t)g + 7, sizeof(c), hipMemcpyDeviceToHost,
                            h->stream));
      if (int rc_s = sync_stream(h)) return rc_s;
    }
    *cost = c;
  }
  return 0;
}

int tcmp_plan_run(tcmp_handle* h, int64_t n_samples, int32_t batch) {
  TCMP_ENTER(h);
  if (!h->plan_open) return fail(-1, "no open plan (tcmp_plan_begin first)");
  if (batch < 1 || batch > h->max_batch) return fail(-1, "batch size out of range");
  if (h->samples_issued + n_samples + 1 > h->P.max_nodes) return fail(-3, "tree capacity exceeded");
  auto run_rounds = [&]() -> int {
    long long left = n_samples;
    while (left > 0) {
      const int nb = (int)std::min<long long>(left, batch);
      if (int rc = plan_round_impl(h, nullptr, nullptr, nb)) return rc;
      left -= nb;
    }
    return 0;
  };
  if (!h->use_graphs || n_samples <= 0) return run_rounds();
  const unsigned long long key = round_graph_key(h, n_samples, batch);
  auto account = [&]() {
    h->samples_issued += n_samples;
    h->launches_nearest += h->rg.rounds;
    h->launches_scan += h->rg.scans;
    h->last_nb = (int)(n_samples % batch ? n_samples % batch : batch);
  };
  if (!(h->rg.exec && h->rg.key == key)) {
    // Capture, instantiate and first launch with every other engine's thread held off (the
    // dispatch lock, exclusive): the round-4 C5 trace aborted with a malformed AQL packet after
    // two engines had captured their round graphs while the other engine's thread was
    // dispatching.  Nothing may allocate or free meanwhile (DBuf::ensure
    // refuses): the graph would bake in a pointer freed under it.
    int rc = 0;
    // The graph of another shape may still be running, and its event nodes' spans wait in
    // ev_used for the next collect_events: the stream drains and the spans are read before
    // the graph and its events are destroyed (plan_run(n1, B) then plan_run(n2, B) on one
    // engine aborted in the HIP runtime, reading the destroyed events at plan_finish).
    if (h->rg.exec) {
      if (int rc_s = sync_stream(h)) return rc_s;
      h->collect_events();
    }
    {
      CaptureScope excl;
      h->drop_graph();
      const long long issued = h->samples_issued, launches = h->launches_nearest,
                      scans = h->launches_scan;
      const int last_nb = h->last_nb;
      if (hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed) != hipSuccess) {
        rc = -2;
      } else {
        h->capturing = true;
        rc = run_rounds();
        h->capturing = false;
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(h->stream, &g);
        if (rc == 0 && e == hipSuccess && g &&
            hipGraphInstantiate(&h->rg.exec, g, nullptr, nullptr, 0) == hipSuccess) {
          h->rg.graph = g;
          h->rg.key = key;
          h->rg.rounds = (int)(h->launches_nearest - launches);
          h->rg.scans = (int)(h->launches_scan - scans);
        } else {
          if (g) (void)hipGraphDestroy(g);
          h->drop_graph();
          rc = rc ? rc : -2;
        }
      }
      (void)hipGetLastError();
      h->samples_issued = issued;  // nothing ran yet
      h->launches_nearest = launches;
      h->launches_scan = scans;
      h->last_nb = last_nb;
      if (!rc) {
        HIPCHK(hipGraphLaunch(h->rg.exec, h->stream));
        account();
        ++h->graph_launches;
        for (const auto& p : h->rg.events) h->ev_used.push_back(p);
        return 0;
      }
    }
    // abandoned (a buffer had to grow, or capture is unsupported here): these rounds run
    // directly, under the shared lock again; the shape is captured anew when it comes back,
    // and after two abandoned captures the engine launches directly from then on
    if (++h->graph_failures >= 2) h->use_graphs = false;
    return run_rounds();
  }
  HIPCHK(hipGraphLaunch(h->rg.exec, h->stream));
  account();
  ++h->graph_launches;
  for (const auto& p : h->rg.events) h->ev_used.push_back(p);
  return 0;
}

// traj = false: retrace only (tcmp_plan_retrace, a foreign dynam_fn takes the waypoints).
// In two halves like the begin: the finish's kernels and the state's copy, then the host wait
// and the result (tcmp_plan_finish_many waits once for many plans).
static void finish_launch_traj(tcmp_handle* h) {
  hipLaunchKernelGGL(k_traj_prep, dim3(1), dim3(1), 0, h->stream, h->st);
  const dim3 gt(grid_for(h->kcap, 256));
  hipLaunchKernelGGL(TCMP_BY_MODE(k_traj, h->P.torque_mode), gt, dim3(256), 0, h->stream, h->dP,
                     h->st, h->wp.p, h->tq.p, h->tqd.p, h->tqdd.p, h->tpsg.p, h->kcap);
  hipLaunchKernelGGL(k_traj_tau, gt, dim3(256), 0, h->stream, h->st, h->tq.p, h->tqd.p,
                     h->tqdd.p, h->ttau.p, h->kcap);
  hipLaunchKernelGGL(k_traj_post, dim3(1), dim3(1), 0, h->stream, h->st);
}
static int plan_finish_launch(tcmp_handle* h, tcmp_plan_result* r, bool traj) {
  if (!r) return fail(-1, "null result");
  if (!h->plan_open) return fail(-1, "no open plan");
  memset(r, 0, sizeof(*r));
  r->first_fail = -1;
  // retrace + min-jerk + validation are launched unconditionally (they do nothing without a
  // goal node) into the buffers tcmp_plan_begin sized, so the host waits once
  hipEvent_t e0;
  h->mark_begin(F_FINISH, &e0);
  hipLaunchKernelGGL(k_retrace, dim3(1), dim3(256), 0, h->stream, h->dP, h->st,
                     Tree{h->cfg.p, h->parent.p, h->tgt.p, h->meta.p}, h->chain.p, h->wp.p,
                     (long long)(h->wp.n / 7));
  if (traj) finish_launch_traj(h);
  HIPCHK(hipGetLastError());
  h->mark_end(F_FINISH, e0);
  HIPCHK(hipMemcpyAsync(&h->pin->st, h->st, sizeof(DevState), hipMemcpyDeviceToHost, h->stream));
  return 0;
}
static int plan_finish_complete(tcmp_handle* h, tcmp_plan_result* r, bool traj) {
  DevState& s = h->pin->st;
  if (int rc_s = sync_stream(h)) return rc_s;
  r->goal_node = s.goal_node;
  if (s.overflow == 1) return fail(-3, "tree capacity exceeded");
  h->fin_W = 0;
  h->fin_K = 0;
  if (s.goal_node >= 0) {
    if (s.status == -3) return fail(-3, "waypoint capacity exceeded");
    if (!traj) {
      // no min-jerk ran: the retrace's own K / status (MINJERK_ASSERT) describe nothing
      s.K = 0;
      s.status = 0;
      s.first_fail = -1;
    } else if (s.K > h->kcap) {
      // an execution time past the preallocated rows: grow and run the trajectory again
      const long long K = s.K;
      int rc = h->tq.ensure(K * 7);
      rc = rc ? rc : h->tqd.ensure(K * 7);
      rc = rc ? rc : h->tqdd.ensure(K * 7);
      rc = rc ? rc : h->tpsg.ensure(K);
      rc = rc ? rc : h->ttau.ensure(K * 7);
      if (rc) return rc;
      h->kcap = K;
      finish_launch_traj(h);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(&s, h->st, sizeof(s), hipMemcpyDeviceToHost, h->stream));
      if (int rc_s = sync_stream(h)) return rc_s;
    }
    r->n_waypoints = s.W;
    r->n_traj = s.status == TCMP_PLAN_MINJERK_ASSERT ? 0 : s.K;
    r->first_fail = s.first_fail;
    r->status = s.status;
    r->goal_found = 1;
    h->fin_W = (size_t)s.W;
    h->fin_K = (size_t)r->n_traj;
  } else {
    r->status = TCMP_PLAN_NO_GOAL;
  }
  h->collect_events();
  r->n_nodes = s.n_nodes;
  r->n_samples = s.samples;
  r->edge_steps = s.edge_steps;
  r->pairs_tested = s.pairs_tested;
  r->pairs_sat = s.pairs_sat;
  r->pairs_exact = s.pairs_exact;
  r->nn_pairs = s.nn_pairs;
  r->ms_nearest = h->ms[F_NEAREST];
  r->ms_edges = h->ms[F_EDGES];
  r->ms_insert = h->ms[F_INSERT];
  r->ms_rewire = h->ms[F_REWIRE];
  r->ms_finish = h->ms[F_FINISH];
  r->launches_nearest = h->launches_nearest;
  r->launches_nn_scan = h->launches_scan;
  r->nn_box_tests = s.nn_box_tests;
  r->ms_nn_scan = h->ms[F_NNSCAN];
  r->ms_edge_prep = h->ms[F_EDGE_PREP];
  r->fused_plans = h->fused_plans;
  r->goal_cost = s.goal_node >= 0 ? s.goal_cost : 0.0;
  r->goal_depth = s.goal_node >= 0 ? s.goal_depth : 0;
  r->snap_sum = s.snap_sum;
  r->nn_full_pairs = s.nn_full_pairs;
  r->n_rewires = s.rewires;
  r->rewire_steps = s.rewire_steps;
  r->graph_launches = h->graph_launches;
  return 0;
}

static int plan_finish_impl(tcmp_handle* h, tcmp_plan_result* r, bool traj) {
  TCMP_ENTER(h);
  if (int rc = plan_finish_launch(h, r, traj)) return rc;
  return plan_finish_complete(h, r, traj);
}

int tcmp_plan_finish(tcmp_handle* h, tcmp_plan_result* r) { return plan_finish_impl(h, r, true); }

int tcmp_plan_retrace(tcmp_handle* h, tcmp_plan_result* r) { return plan_finish_impl(h, r, false); }

int tcmp_plan_finish_many(tcmp_handle* const* hs, int32_t n, tcmp_plan_result* results) {
  Entry entry;
  if (!hs || n < 1 || !results) return fail(-1, "bad arguments");
  for (int q = 0; q < n; ++q) {
    if (int rc = set_dev(hs[q])) return rc;
    if (int rc = plan_finish_launch(hs[q], results + q, true))
      return fail(rc, "plan " + std::to_string(q) + ": " + tcmp_last_error());
  }
  for (int q = 0; q < n; ++q) {
    if (int rc = set_dev(hs[q])) return rc;
    if (int rc = plan_finish_complete(hs[q], results + q, true))
      return fail(rc, "plan " + std::to_string(q) + ": " + tcmp_last_error());
  }
  return 0;
}

int tcmp_plan_fetch(tcmp_handle* h, double* waypoints, double* q, double* qd, double* qdd,
                    double* psg, double* tau) {
  TCMP_ENTER(h);
  // the sizes tcmp_plan_finish read (it waited for the plan); no other state read here
  if (h->fin_W == 0) return fail(-1, "no plan to fetch");
  const long long W = (long long)h->fin_W, K = (long long)h->fin_K;
  if (waypoints && W)
    HIPCHK(hipMemcpyAsync(waypoints, h->wp.p, W * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (K && (size_t)K * 29 * sizeof(double) <= h->fetch_pin_n) {
    // the trajectory rows through the pinned staging: one DMA per array, one host wait, then
    // host copies into the caller's arrays
    struct Part { double* dst; const double* src; size_t n; };
    const Part parts[5] = {{q, h->tq.p, (size_t)K * 7}, {qd, h->tqd.p, (size_t)K * 7},
                           {qdd, h->tqdd.p, (size_t)K * 7}, {psg, h->tpsg.p, (size_t)K},
                           {tau, h->ttau.p, (size_t)K * 7}};
    double* pin = static_cast<double*>(h->fetch_pin);
    size_t off = 0;
    for (const Part& p : parts) {
      if (p.dst) HIPCHK(hipMemcpyAsync(pin + off, p.src, p.n * sizeof(double),
                                       hipMemcpyDeviceToHost, h->stream));
      off += p.n;
    }
    if (int rc_s = sync_stream(h)) return rc_s;
    off = 0;
    for (const Part& p : parts) {
      if (p.dst) memcpy(p.dst, pin + off, p.n * sizeof(double));
      off += p.n;
    }
    return 0;
  }
  if (K) {
    if (q) HIPCHK(hipMemcpyAsync(q, h->tq.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (qd) HIPCHK(hipMemcpyAsync(qd, h->tqd.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (qdd) HIPCHK(hipMemcpyAsync(qdd, h->tqdd.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (psg) HIPCHK(hipMemcpyAsync(psg, h->tpsg.p, K * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (tau) HIPCHK(hipMemcpyAsync(tau, h->ttau.p, K * 7 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  }
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

int tcmp_microbench(tcmp_handle* h, double* out) {
  TCMP_ENTER(h);
  if (!out) return fail(-1, "null out");
  // best of 5 launches each, HIP events on the handle's stream
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  auto best_ms = [&](auto launch) -> double {
    double best = 1e30;
    for (int r = 0; r < 6; ++r) {
      (void)hipEventRecord(a, h->stream);
      launch();
      (void)hipEventRecord(b, h->stream);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      if (r > 0) best = std::min(best, (double)ms);  // the first launch warms up
    }
    return best;
  };
  int rc = h->s0.ensure(4 * 65536);
  if (rc) return rc;
  const int blocks = std::max(1, h->cu_count) * 8, iters = 4096;
  const double threads = (double)blocks * 256;
  double ms = best_ms([&] {
    hipLaunchKernelGGL(k_mb_fp64, dim3(blocks), dim3(256), 0, h->stream, h->s0.p, iters);
  });
  out[0] = 2.0 * kMbAcc * iters * threads / (ms * 1e-3) / 1e12;
  ms = best_ms([&] {
    hipLaunchKernelGGL(k_mb_fp32, dim3(blocks), dim3(256), 0, h->stream, h->s0.p, iters);
  });
  out[1] = 4.0 * kMbAcc * iters * threads / (ms * 1e-3) / 1e12;
  // HBM: 1 GiB float4 copy (2 GiB moved per launch), far past the caches
  const size_t n4 = ((size_t)1 << 30) / 16;
  float4 *src = nullptr, *dst = nullptr;
  HIPCHK(hipMalloc(&src, n4 * 16));
  if (hipMalloc(&dst, n4 * 16) != hipSuccess) {
    (void)hipFree(src);
    return fail(-2, "microbench: hipMalloc");
  }
  (void)hipMemsetAsync(src, 0, n4 * 16, h->stream);
  ms = best_ms([&] {
    hipLaunchKernelGGL(k_mb_copy<4>, dim3((unsigned)(n4 / (256 * 4))), dim3(256), 0, h->stream,
                       src, dst, (long long)n4);
  });
  ms = std::min(ms, best_ms([&] {
    hipLaunchKernelGGL(k_mb_copy<2>, dim3((unsigned)(n4 / (256 * 2))), dim3(256), 0, h->stream,
                       src, dst, (long long)n4);
  }));
  ms = std::min(ms, best_ms([&] {
    hipLaunchKernelGGL(k_mb_copy<8>, dim3((unsigned)(n4 / (256 * 8))), dim3(256), 0, h->stream,
                       src, dst, (long long)n4);
  }));
  // (out[3]: the best variant -- 0 one-pass, 1..6 persistent 4 / 8 / 16 blocks per CU with
  // V = 4 or 8 and nontemporal loads, 7..12 the same with plain loads)
  double best1 = ms;
  int var = 0, vi = 0;
  for (int ntl = 1; ntl >= 0; --ntl)
    for (int per_cu : {4, 8, 16})
      for (int v : {4, 8}) {
        ++vi;
        const unsigned gs = (unsigned)(std::max(1, h->cu_count) * per_cu);
        auto k = v == 4 ? (ntl ? k_mb_copy_gs<4, true> : k_mb_copy_gs<4, false>)
                        : (ntl ? k_mb_copy_gs<8, true> : k_mb_copy_gs<8, false>);
        const double t = best_ms([&] {
          hipLaunchKernelGGL(k, dim3(gs), dim3(256), 0, h->stream, src, dst, (long long)n4);
        });
        if (t < best1) { best1 = t; var = vi; }
      }
  ms = best1;
  out[2] = 2.0 * (double)n4 * 16 / (ms * 1e-3) / 1e9;
  out[3] = (double)var;
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  HIPCHK(hipGetLastError());
  return 0;
}

int tcmp_plan_digest(tcmp_handle* h, uint64_t* digest, int64_t* n_nodes) {
  TCMP_ENTER(h);
  if (!digest || !n_nodes) return fail(-1, "null argument");
  if (!h->plan_open) return fail(-1, "no open plan");
  if (int rc = h->u0.ensure(1)) return rc;
  HIPCHK(hipMemsetAsync(h->u0.p, 0, sizeof(unsigned long long), h->stream));
  long long cap = h->P.max_nodes;
  hipLaunchKernelGGL(k_tree_digest, dim3(grid_for(std::min<long long>(cap, 1 << 20), 256)),
                     dim3(256), 0, h->stream, h->st, h->cfg.p, h->parent.p, h->u0.p);
  HIPCHK(hipGetLastError());
  long long nn = 0;
  unsigned long long d = 0;
  HIPCHK(hipMemcpyAsync(&d, h->u0.p, sizeof(d), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&nn, &h->st->n_nodes, sizeof(nn), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  *digest = d;
  *n_nodes = nn;
  return 0;
}

int tcmp_plan_tree(tcmp_handle* h, int64_t cap, double* cfg, double* cost, int32_t* parent,
                   int64_t* n) {
  TCMP_ENTER(h);
  if (!n) return fail(-1, "null n");
  long long nn = 0;
  HIPCHK(hipMemcpyAsync(&nn, &h->st->n_nodes, sizeof(nn), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  *n = nn;
  const long long m = std::min<long long>(nn, cap);
  if (m <= 0) return 0;
  std::vector<double> tmp((size_t)m * 8);
  HIPCHK(hipMemcpyAsync(tmp.data(), h->cfg.p, tmp.size() * sizeof(double), hipMemcpyDeviceToHost,
                        h->stream));
  if (parent)
    HIPCHK(hipMemcpyAsync(parent, h->parent.p, m * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  for (long long i = 0; i < m; ++i) {
    if (cfg)
      for (int k = 0; k < 7; ++k) cfg[7 * i + k] = tmp[8 * i + k];
    if (cost) cost[i] = tmp[8 * i + 7];
  }
  return 0;
}

int tcmp_plan_debug_round(tcmp_handle* h, int64_t cap, double* cand, int32_t* nn,
                          double* score, int64_t* snap, int32_t* nb) {
  TCMP_ENTER(h);
  if (!snap || !nb || cap < 0) return fail(-1, "bad arguments");
  if (!h->plan_open) return fail(-1, "no open plan");
  long long T = 0;
  HIPCHK(hipMemcpyAsync(&T, &h->st->snap, sizeof(T), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  *snap = T;
  *nb = h->last_nb;
  const long long m = std::min<long long>(cap, h->last_nb);
  if (m <= 0) return 0;
  if (cand) {
    std::vector<double> tmp((size_t)m * 8);
    HIPCHK(hipMemcpyAsync(tmp.data(), h->cand.p, tmp.size() * sizeof(double),
                          hipMemcpyDeviceToHost, h->stream));
    if (int rc_s = sync_stream(h)) return rc_s;
    for (long long i = 0; i < m; ++i)
      for (int k = 0; k < 7; ++k) cand[7 * i + k] = tmp[8 * i + k];
  }
  if (nn) HIPCHK(hipMemcpyAsync(nn, h->nn.p, m * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  if (score)
    HIPCHK(hipMemcpyAsync(score, h->nnscore.p, m * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (int rc_s = sync_stream(h)) return rc_s;
  return 0;
}

}  // extern "C"

#include "tcmp_fleet.h"
