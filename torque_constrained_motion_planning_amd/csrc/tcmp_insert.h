// tcmp_insert.h -- lane-ordered insertion of a round's accepted edges (rrt_star.py:173-180),
// as a device-wide scan: k_edges counts the accepted edges per 256 lanes as they finish, one
// block scans the counts, then every block writes its nodes at (snapshot size + block offset +
// in-block rank).  Node order is therefore lane order, exactly as the single-pass reference
// loop appends them.  In a shared-tree round (tcmp_plan_run_shared) the engines own
// consecutive lane ranges and add ins_off = the lower ranks' accepted edges, so the global
// order is still lane order.
// Included by tcmp_engine.hip after the state types.
#pragma once

__device__ __forceinline__ void ins_scan_block(DevState* st, const int* bcount, int nblocks,
                                               int* boff) {
  __shared__ int sc[1024];
  const int tid = threadIdx.x;
  int run = 0;
  for (int b0 = 0; b0 < nblocks; b0 += 1024) {
    const int b = b0 + tid;
    const int v = b < nblocks ? bcount[b] : 0;
    sc[tid] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int x = tid >= o ? sc[tid - o] : 0;
      __syncthreads();
      sc[tid] += x;
      __syncthreads();
    }
    if (b < nblocks) boff[b] = run + sc[tid] - v;
    run += sc[1023];
    __syncthreads();
  }
  if (tid == 0) {
    st->ins_total = run;
    st->ins_off = 0;
    st->ins_all = run;
    st->ins_goal = LLONG_MAX;
    st->rw_count = 0;
  }
}
__global__ __launch_bounds__(1024) void k_ins_scan(DevState* st, const int* bcount, int nblocks,
                                                   int* boff) {
  ins_scan_block(st, bcount, nblocks, boff);
}

__device__ __forceinline__ void ins_write_block(const PlanParams* __restrict__ Pd, DevState* st,
                                                const Tree& tr, const int* nn, const double* cand,
                                                const unsigned char* cgoal, const int* nsafe,
                                                const int* nsteps, const double* last, int nb,
                                                const int* boff, const double* second,
                                                int* rwlist, int blk) {
  const PlanParams P = *Pd;
  __shared__ int wc[4];
  const long long T = st->n_nodes + st->ins_off;
  if (st->n_nodes + st->ins_all > P.max_nodes) return;  // k_ins_final flags the overflow
  const bool goal_open = st->goal_node < 0;
  const int j = blk * 256 + threadIdx.x;
  const bool v = j < nb && nsafe[j] > 0;
  const uint64_t m = __ballot(v);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  if (lane == 0) wc[w] = (int)__popcll(m);
  __syncthreads();
  int before = 0;
  for (int i = 0; i < w; ++i) before += wc[i];
  if (!v) return;
  const long long idx = T + boff[blk] + before + (int)__popcll(m & ((1ull << lane) - 1ull));
  const int par = nn[j];
  double pc[7], lq[7], tq[7];
  load7(tr.cfg + 8 * (size_t)par, pc);
  load7(last + 8 * (size_t)j, lq);
  load7(cand + 8 * (size_t)j, tq);
  const double d = distance(pc, lq, P.w);
  double* dst = tr.cfg + 8 * idx;
  store7(dst, lq);
  dst[7] = tr.cfg[8 * (size_t)par + 7] + d;
  tr.parent[idx] = par;
  store7(tr.tgt + 8 * idx, tq);
  tr.meta[idx] = make_int2(nsteps[j], nsafe[j]);
  if (goal_open && cgoal[j] && distance(lq, P.goal, P.w) < P.goal_tol)
    atomicMin(&st->ins_goal, idx);
  // rewire bound (tcmp_nn32.h): neighbour scan only if the second-nearest bound passes it
  double e2 = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double dd = lq[k] - tq[k];
    e2 = fma(P.uniform_w ? dd : P.w[k] * dd, dd, e2);
  }
  const double r = P.uniform_w ? P.radius / sqrt(P.w[0]) : P.radius;
  const double t = sqrt(e2) + r;
  if (second[j] < t * t * (1.0 + 1e-9) + 1e-300) rwlist[atomicAdd(&st->rw_count, 1)] = (int)idx;
}
__global__ __launch_bounds__(256) void k_ins_write(const PlanParams* __restrict__ Pd, DevState* st, Tree tr,
                                                   const int* nn, const double* cand,
                                                   const unsigned char* cgoal, const int* nsafe,
                                                   const int* nsteps, const double* last, int nb,
                                                   const int* boff, const double* second,
                                                   int* rwlist) {
  ins_write_block(Pd, st, tr, nn, cand, cgoal, nsafe, nsteps, last, nb, boff, second, rwlist,
                  blockIdx.x);
}

__device__ __forceinline__ void ins_final(const PlanParams* __restrict__ Pd, DevState* st, int nb) {
  const PlanParams P = *Pd;
  const long long T = st->n_nodes, total = st->ins_all;
  st->snap = T;
  if (T + total > P.max_nodes) {
    st->overflow = 1;
    st->new_count = 0;
    st->rw_count = 0;
  } else {
    st->new_count = total;
    st->n_nodes = T + total;
    if (st->goal_node < 0 && st->ins_goal != LLONG_MAX) st->goal_node = st->ins_goal;
  }
  st->samples += nb;
  st->snap_sum += (unsigned long long)T;
  st->nn_full_pairs += (unsigned long long)T * (unsigned long long)nb;
  st->round_goal = INT_MAX;
}
__global__ void k_ins_final(const PlanParams* __restrict__ Pd, DevState* st, int nb) {
  ins_final(Pd, st, nb);
}
