// tcmp_fleet.h -- fused multi-plan rounds (tcmp_plan_run_fused): one set of launches per round
// serves the lanes of several independent open plans (C4's queries, collect_data.py:74-85 plans
// the approach / grasp / place queries one after another), instead of one set per plan.
//
// Each plan keeps its own engine, buffers, scene and tree; the fused kernels index a device
// array of plan descriptors (FleetPlan, FleetNN).  Lanes are laid out plan-major with a stride
// bp = the batch rounded up to 256, so every 256-thread block belongs to one plan and the
// per-plan kernels (sampling, edge order, records, insertion, rewire) run their single-plan
// bodies on that plan's buffers.  Two stages are fused for real:
//   - the nearest-neighbour index: one Morton sort over every plan's nodes with the plan id in
//     the top key bits (pb bits; the all-ones plan value marks the unused node slots), cells
//     and super-cells forced to start at each plan's first node, so a plan's nodes, cells and
//     super-cells are contiguous ranges; one k_nearest_wave32<FLEET> launch walks each
//     candidate's own plan's super-cells (tcmp_nn32.h);
//   - the edge walk (k_fl_edges): a persistent 512-thread grid with every plan's obstacles in
//     LDS; a wave takes one plan's edges at a time and moves on to the next plan when that
//     queue runs dry.
// Everything a plan computes -- its samples (its own Philox seed), nearest nodes (exact, ties
// by its own node index), edges, node order and rewires -- is what tcmp_plan_run computes for
// it alone: a fleet's trees are bit-identical to the lone engines' (tests/test_gpu_fleet.py).
// Scope: identical distance weights and scan bound (nn_cmax) across the plans; box scenes may
// differ per plan, convex-mesh scenes (or self-collision pairs) must be one scene for the whole
// fleet (k_fl_edges_mesh stages the lead's); everything else may differ per plan.
#pragma once

namespace {

constexpr int kFleetMax = 31;  // plans per fused round (plan ids need at most 5 key bits)
constexpr unsigned kFleetLdsCap = 160u * 1024u;  // k_fl_edges' LDS (a CU's whole 160 KB)

// One open plan of a fused multi-plan round: everything its share of a fused launch reads or
// writes -- the plan's own buffers, so that each plan's tree is exactly the
// one a lone engine would have grown from the same seed.
struct FleetPlan {
  const PlanParams* P;
  DevState* st;
  Tree tr;
  EdgeJob J;          // the round's edges: from cfg[nn[e]] to cand[e], longest first
  double* cand;
  unsigned char* cgoal;
  int* nn;
  double* second;
  double* score;
  int* bins;          // the edge order's counting sort (bins, histogram, offsets)
  int* hist;
  int* hoff;
  int* bcount;
  int* boff;
  int* rwlist;
  int* nbr;
  int* ncount;
  Scene sc;           // box obstacles (obs, obs32, n_obs)
  int lds_obs;        // first row of this plan's obstacles in the fused k_edges' LDS
};

// k_fl_edges' LDS: every plan's obstacle records (f64 [n][16], then f32 [n][8]), the hull
// geometry, one pair queue per wave of a 512-thread block, and behind the queues each lane's
// last safe configuration, [7][512] doubles (in LDS, not in 14 VGPRs: 80 -> 16 B of scratch
// per lane, C3 fleet edges 3.25 -> 3.16 ms)
__host__ __device__ constexpr unsigned fleet_lds_bytes(int n_obs_total) {
  return scene_lds_bytes(n_obs_total) + geo_lds_bytes() + 8 * kQwaveBytes +
         7 * 512 * sizeof(double);
}
__device__ __forceinline__ void fleet_stage_lds(const FleetPlan* __restrict__ fp, int n_plans,
                                                const Geo& g_g, double* lds, double** o64p,
                                                float** o32p, Scene& so, Geo& go) {
  const int tot = max(1, fp[n_plans - 1].lds_obs + fp[n_plans - 1].sc.n_obs);
  double* o64 = lds;
  float* o32 = reinterpret_cast<float*>(lds + 16 * tot);
  float4* pl = reinterpret_cast<float4*>(o32 + 8 * tot);
  float* vt = reinterpret_cast<float*>(pl + TCMP_TOTAL_PLANES);
  uint2* ei = reinterpret_cast<uint2*>(vt + 3 * TCMP_TOTAL_VERTS);
  unsigned* wq = reinterpret_cast<unsigned*>(ei + TCMP_TOTAL_EDGES) +
                 (threadIdx.x >> 6) * (kQwaveBytes / 4);
  for (int q = 0; q < n_plans; ++q) {
    const int n = fp[q].sc.n_obs, off = fp[q].lds_obs;
    const double* s64 = fp[q].sc.obs;
    const float* s32 = fp[q].sc.obs32;
    for (int i = threadIdx.x; i < n * 16; i += blockDim.x) o64[16 * off + i] = s64[i];
    for (int i = threadIdx.x; i < n * 8; i += blockDim.x) o32[8 * off + i] = s32[i];
  }
  for (int i = threadIdx.x; i < TCMP_TOTAL_PLANES; i += blockDim.x) pl[i] = g_g.planes32[i];
  for (int i = threadIdx.x; i < 3 * TCMP_TOTAL_VERTS; i += blockDim.x) vt[i] = g_g.verts32[i];
  const uint2* gei = reinterpret_cast<const uint2*>(g_g.eidx);
  for (int i = threadIdx.x; i < TCMP_TOTAL_EDGES; i += blockDim.x) ei[i] = gei[i];
  __syncthreads();
  *o64p = o64;
  *o32p = o32;
  so.wq = wq;
  so.cv32 = vt;
  go = g_g;
  go.planes32 = pl;
  go.verts32 = vt;
  go.eidx = reinterpret_cast<const ushort4*>(ei);
}
// ---- per-plan block kernels: block b of a launch is block b % bpb of plan b / bpb ----------
__global__ __launch_bounds__(256) void k_fl_sample(const FleetPlan* __restrict__ fp, long long base,
                                                   int nb, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  sample_lane(fp[q].P, fp[q].st, base, nb, fp[q].cand, fp[q].cgoal, b * 256 + threadIdx.x);
}

// the first round (one-node trees): the root is every candidate's nearest node
__global__ __launch_bounds__(256) void k_fl_root(const FleetPlan* __restrict__ fp, int nb, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  const FleetPlan& f = fp[q];
  nn_root_lane(f.P, f.st, f.tr.cfg, f.cand, nb, f.nn, f.second, f.score,
               GoalFix{f.cand, f.cgoal}, f.bcount, b * 256 + threadIdx.x);
}

// round start of an indexed round: each plan's first node row in the fleet index (off[q], the
// prefix of the plans' node counts), the fleet's node count and scan queues, the plans' goal
// lanes (k_sample chose them) and their work counters and accepted-edge counts
__global__ __launch_bounds__(256) void k_fl_prep(const FleetPlan* __restrict__ fp, int K,
                                                 DevState* fst, long long* off, int nb) {
  const int t = threadIdx.x;
  if (t == 0) {
    long long o = 0;
    for (int q = 0; q < K; ++q) {
      off[q] = o;
      o += fp[q].st->n_nodes;
    }
    off[K] = o;
    fst->n_nodes = o;
    fst->nn_counter = 0;
    fst->work_counter = 0;
  }
  if (t < 8) fst->nn_queue[t] = 0;
  if (t < K) {
    const FleetPlan& f = fp[t];
    goal_fix(f.P, f.st, GoalFix{f.cand, f.cgoal}, nb);
    f.st->work_counter = 0;
    f.st->nn_counter = 0;
  }
  const int nblk = (nb + 255) / 256;
  for (int i = t; i < K * nblk; i += 256) fp[i / nblk].bcount[i % nblk] = 0;
}

// node slot s = q * Tb + n (Tb = the round's node bound, every plan's): key = plan id over the
// node's Morton key, or the all-ones key past the plan's node count (sorted to the very end)
__global__ __launch_bounds__(256) void k_fl_node_keys(const FleetPlan* __restrict__ fp, long long Tb,
                                                      long long slots, int pb,
                                                      unsigned long long* keys, int* vals) {
  for (long long s = (long long)blockIdx.x * 256 + threadIdx.x; s < slots;
       s += (long long)gridDim.x * 256) {
    const int q = (int)(s / Tb);
    const long long n = s - (long long)q * Tb;
    unsigned long long key = (1ull << (kKeyBits + pb)) - 1;
    if (n < fp[q].st->n_nodes) {
      double c[7];
      load7(fp[q].tr.cfg + 8 * n, c);
      key = ((unsigned long long)q << kKeyBits) | (morton7(c) >> (63 - kKeyBits));
    }
    keys[s] = key;
    vals[s] = (int)s;
  }
}

// rows in key order (k_nn_rows over the plans' trees: the 8th column is the plan's own node
// index); the cell flags start out set at each plan's first row, the super-cell flags clear
__global__ __launch_bounds__(256) void k_fl_rows(const FleetPlan* __restrict__ fp, const DevState* fst,
                                                 const long long* off, const int* svals,
                                                 long long Tb, long long slots, double* stree,
                                                 float* srow, int* cflag, int* sflag) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= slots) return;
  sflag[p] = 0;
  if (p >= fst->n_nodes) {
    cflag[p] = 0;
    return;
  }
  const int s = svals[p];
  const int q = (int)(s / Tb);
  const long long n = s - (long long)q * Tb;
  cflag[p] = p == off[q] ? 1 : 0;
  double c[7];
  load7(fp[q].tr.cfg + 8 * n, c);
  store7(stree + 8 * p, c);
  stree[8 * p + 7] = (double)n;
  float4* d32 = reinterpret_cast<float4*>(srow + 8 * p);
  d32[0] = make_float4((float)c[0], (float)c[1], (float)c[2], (float)c[3]);
  d32[1] = make_float4((float)c[4], (float)c[5], (float)c[6], 0.f);
}

// super-cells start at each plan's first cell too
__global__ void k_fl_super_flags(const long long* off, const int* cid, int* sflag, int K) {
  const int q = threadIdx.x;
  if (q < K) sflag[cid[off[q]] - 1] = 1;
}

// each plan's super-cells [s0, s1) for the scan
__global__ void k_fl_ranges(const long long* off, const int* cid, const int* sid,
                            const DevState* fst, FleetNN* fnn, int K) {
  const int q = threadIdx.x;
  if (q >= K) return;
  fnn[q].s0 = sid[cid[off[q]] - 1] - 1;
  fnn[q].s1 = q + 1 < K ? sid[cid[off[q + 1]] - 1] - 1 : fst->nn_supers;
}

// candidate slot g = q * bp + j: plan id over the Morton key, all ones for the padding lanes
__global__ __launch_bounds__(256) void k_fl_cand_keys(const FleetPlan* __restrict__ fp, int nb, int bp,
                                                      int pb, unsigned long long* keys, int* vals) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  const int q = g / bp, j = g - q * bp;
  unsigned long long key = (1ull << (kKeyBits + pb)) - 1;
  if (j < nb) {
    double c[7];
    load7(fp[q].cand + 8 * (size_t)j, c);
    key = ((unsigned long long)q << kKeyBits) | (morton7(c) >> (63 - kKeyBits));
  }
  keys[g] = key;
  vals[g] = g;
}

// home cell of each sorted candidate: its key's lower bound among its own plan's rows
__global__ __launch_bounds__(256) void k_fl_home(const long long* off, const unsigned long long* skeys,
                                                 const unsigned long long* ckeys, const int* cperm,
                                                 const int* cid, const int* sid, int nbt, int bp,
                                                 int* home) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= nbt) return;
  const int g = cperm[j];
  const int q = g / bp;
  const unsigned long long k = ckeys[g];
  const long long first = off[q], last = off[q + 1] - 1;
  long long lo = first, hi = last + 1;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (skeys[mid] < k) lo = mid + 1; else hi = mid;
  }
  const int c = cid[min(lo, last)] - 1;
  home[j] = c;
  home[nbt + j] = sid[c] - 1;
}

// ---- edges ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fl_edge_order(const FleetPlan* __restrict__ fp, int nb, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  const FleetPlan& f = fp[q];
  edge_order_block(f.P, f.tr.cfg, f.nn, f.cand, nb, f.bins, f.hist, b);
}
__global__ __launch_bounds__(1024) void k_fl_cs_scan(const FleetPlan* __restrict__ fp) {
  cs_scan_block(fp[blockIdx.x].hist, 256, fp[blockIdx.x].hoff);
}
__global__ __launch_bounds__(256) void k_fl_cs_scatter(const FleetPlan* __restrict__ fp, int nb, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  cs_scatter_block(fp[q].bins, nb, 256, fp[q].hoff, const_cast<int*>(fp[q].J.order), b);
}
__global__ __launch_bounds__(256) void k_fl_edge_records(const FleetPlan* __restrict__ fp, int nb,
                                                         int ordered, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  EdgeJob J = fp[q].J;
  J.n = nb;
  if (!ordered) J.order = nullptr;
  edge_record(J, fp[q].P, b * 256 + threadIdx.x);
}
// k_edges over every plan's edges (box scenes, one lane per edge): the same persistent walk and
// the same per-step tests (rrt_star.py:90-98), with each wave bound to one plan at a time.  A
// wave starts at plan (its index * K / waves); when that plan's queue is empty and its lanes
// have finished, it posts its counts to the plan and takes the next plan, until it has been
// through all K.  nb: the round's edge count (every plan's).
// behind the lanes' last safe configurations, their edges' targets ([7][512] doubles, written
// at fetch) when the fleet's LDS has room for them (C3 fleets of four; not C4's sixteen): the
// two target reads per step are LDS reads instead of L2 round trips, k_fl_edges 3.152 -> 3.118 ms
// per C3 launch (same-box A/B, profiles/r9w_ab_fetch/; reserving 16 work slots per counter
// atomic instead of a step's need measured no change and is not kept)
__host__ __device__ constexpr unsigned fleet_q2_bytes() { return 7u * 512u * sizeof(double); }
__global__ __launch_bounds__(512, 1) void k_fl_edges(const FleetPlan* __restrict__ fp, int K, int nb,
                                                     Geo g_g, int q2lds) {
  extern __shared__ double tcmp_lds[];
  Scene s0{};
  Geo g;
  double* o64;
  float* o32;
  fleet_stage_lds(fp, K, g_g, tcmp_lds, &o64, &o32, s0, g);
  const int lane = lane_id();
  const int waves = gridDim.x * (blockDim.x >> 6);
  int plan = (int)((long long)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * K / waves);
  // behind the eight pair queues: [7][512] doubles, this lane's column (its last safe
  // configuration, read and written once per step)
  double* const qcol = reinterpret_cast<double*>(
      reinterpret_cast<unsigned char*>(s0.wq - (threadIdx.x >> 6) * (kQwaveBytes / 4)) +
      8 * kQwaveBytes) + threadIdx.x;
  // the plan's fields are read through F where they are used: scalar loads from the constant
  // address space, which the compiler may repeat instead of keeping the values live in
  // registers across the collision check
  typedef const __attribute__((address_space(4))) FleetPlan CFleetPlan;
  CFleetPlan* const fc = (CFleetPlan*)(uintptr_t)fp;
  CFleetPlan* F = fc + plan;
  // a plan's queue never refills once empty, so each wave visits each plan once
  int visited = 1;
  int e = -1, i = 0, n = 0;
  bool done = false;
  auto get_q = [&](double o[7]) {
#pragma unroll
    for (int k = 0; k < 7; ++k) o[k] = qcol[512 * k];
  };
  auto put_q = [&](const double o[7]) {
#pragma unroll
    for (int k = 0; k < 7; ++k) qcol[512 * k] = o[k];
  };
  // the edge's target: its LDS column behind qcol's (written at fetch) or global memory
  double* const tcol = qcol + 7 * 512;
  auto get_t = [&](double o[7]) {
    if (q2lds) {
#pragma unroll
      for (int k = 0; k < 7; ++k) o[k] = tcol[512 * k];
    } else {
      load7(F->J.to + 8 * (size_t)e, o);
    }
  };
  {
    const double mid[7] = {0.5 * (kLo[0] + kHi[0]), 0.5 * (kLo[1] + kHi[1]), 0.5 * (kLo[2] + kHi[2]),
                           0.5 * (kLo[3] + kHi[3]), 0.5 * (kLo[4] + kHi[4]), 0.5 * (kLo[5] + kHi[5]),
                           0.5 * (kLo[6] + kHi[6])};
    put_q(mid);  // (lanes without an edge ride along on a valid configuration)
  }
  StepStats ss = {};
  unsigned steps = 0;
  while (true) {
    const bool need = !done && e < 0;
    const uint64_t m = __ballot(need);
    if (m) {
      const int leader = __builtin_ctzll(m);
      int base = 0;
      if (lane == leader) base = atomicAdd(&F->st->work_counter, (int)__popcll(m));
      base = __shfl(base, leader);
      if (need) {
        const int my = base + (int)__popcll(m & ((1ull << lane) - 1ull));
        if (my < nb) {
          const double* rec = F->J.rec + 8 * (size_t)my;
          const double4 ra = *reinterpret_cast<const double4*>(rec);
          const double4 rb4 = *reinterpret_cast<const double4*>(rec + 4);
          const double qf[7] = {ra.x, ra.y, ra.z, ra.w, rb4.x, rb4.y, rb4.z};
          put_q(qf);
          e = __double2loint(rb4.w);
          n = __double2hiint(rb4.w);
          i = 0;
          if (q2lds) {
            double q2[7];
            load7(F->J.to + 8 * (size_t)e, q2);
#pragma unroll
            for (int k = 0; k < 7; ++k) tcol[512 * k] = q2[k];
          }
        } else {
          done = true;
        }
      }
    }
    if (__ballot(!done) == 0) {
      // this plan's queue is empty and its lanes are done: its counts, then the next plan
      if (lane == 0 && steps) {
        DevState* st = F->st;
        atomicAdd(&st->edge_steps, (unsigned long long)steps);
        atomicAdd(&st->pairs_tested, 10ull * (unsigned long long)F->sc.n_obs * ss.live_steps);
        atomicAdd(&st->pairs_sat, (unsigned long long)ss.pairs_sat);
        atomicAdd(&st->pairs_exact, (unsigned long long)ss.pairs_exact);
      }
      steps = 0;
      ss = StepStats{};
      if (visited++ == K) break;
      plan = plan + 1 == K ? 0 : plan + 1;
      F = fc + plan;
      done = false;
      continue;
    }
    const bool active = e >= 0;
    bool tok = true, lim = false;
    double cq[7], sq[7];
    {
      double qn[7], q2[7];
      get_q(qn);
      if (active) {
        get_t(q2);
        refine_step(qn, q2, n, i);
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) sincos(qn[k], &sq[k], &cq[k]);
      lim = active && limits_violated(qn);
    }
    const int tm = F->P->torque_mode;
    if (active && !lim && tm != TCMP_TORQUE_BASE) {
      const double z[7] = {0, 0, 0, 0, 0, 0, 0};
      const double mass = F->P->mass;
      tok = tm == TCMP_TORQUE_DYN ? torque_ok_dyn<false>(cq, sq, z, z, mass)
                                  : torque_ok<false>(cq, sq, z, z, mass);
    }
    Scene sc = s0;
    sc.obs = o64 + 16 * F->lds_obs;
    sc.obs32 = o32 + 8 * F->lds_obs;
    sc.n_obs = F->sc.n_obs;
    const bool coll = collides_wave<false>(cq, sq, active && !lim && tok, sc, g, ss) || lim;
    const bool ok = active && !coll && tok;
    steps += (unsigned)__popcll(__ballot(active));
    if (active) {
      double qc[7];
      get_q(qc);
      if (ok) {
        double q2[7];
        get_t(q2);
        refine_step(qc, q2, n, i);
        put_q(qc);
        ++i;
      }
      if (!ok || i == n) {
        if (i > 0) atomicAdd(&F->J.accepted[e >> 8], 1);
        F->J.nsafe[e] = i;
        F->J.nsteps[e] = n;
        store7(F->J.last + 8 * (size_t)e, qc);
        e = -1;
      }
    }
  }
}

// The same walk over convex-mesh scenes, for fleets whose plans share one scene (replica trees
// of one query, C5): the lead's scene is staged as k_edges<true, 1> stages it (256-thread blocks,
// the lean LDS layout with the waves' stashes), and each lane's configuration stays in
// registers (the mesh kernel's LDS has no room for it).  sc_g: the lead engine's scene.
__global__ __launch_bounds__(256, TCMP_EDGE_MINW) void k_fl_edges_mesh(const FleetPlan* __restrict__ fp,
                                                                      int K, int nb, Scene sc_g,
                                                                      Geo g_g) {
  extern __shared__ double tcmp_lds[];
  Scene sc;
  Geo g;
  stage_lds<false>(sc_g, g_g, tcmp_lds, sc, g);
  const int lane = lane_id();
  const int waves = gridDim.x * (blockDim.x >> 6);
  int plan = (int)((long long)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * K / waves);
  typedef const __attribute__((address_space(4))) FleetPlan CFleetPlan;
  CFleetPlan* const fc = (CFleetPlan*)(uintptr_t)fp;
  CFleetPlan* F = fc + plan;
  int visited = 1;
  int e = -1, i = 0, n = 0;
  bool done = false;
  double q[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) q[k] = 0.5 * (kLo[k] + kHi[k]);
  StepStats ss = {};
  unsigned steps = 0;
  while (true) {
    const bool need = !done && e < 0;
    const uint64_t m = __ballot(need);
    if (m) {
      const int leader = __builtin_ctzll(m);
      int base = 0;
      if (lane == leader) base = atomicAdd(&F->st->work_counter, (int)__popcll(m));
      base = __shfl(base, leader);
      if (need) {
        const int my = base + (int)__popcll(m & ((1ull << lane) - 1ull));
        if (my < nb) {
          const double* rec = F->J.rec + 8 * (size_t)my;
          const double4 ra = *reinterpret_cast<const double4*>(rec);
          const double4 rb = *reinterpret_cast<const double4*>(rec + 4);
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
    if (__ballot(!done) == 0) {
      if (lane == 0 && steps) {
        DevState* st = F->st;
        atomicAdd(&st->edge_steps, (unsigned long long)steps);
        atomicAdd(&st->pairs_tested, 10ull * (unsigned long long)sc_g.n_obs * ss.live_steps);
        atomicAdd(&st->pairs_sat, (unsigned long long)ss.pairs_sat);
        atomicAdd(&st->pairs_exact, (unsigned long long)ss.pairs_exact);
      }
      steps = 0;
      ss = StepStats{};
      if (visited++ == K) break;
      plan = plan + 1 == K ? 0 : plan + 1;
      F = fc + plan;
      done = false;
      continue;
    }
    const bool active = e >= 0;
    bool tok = true, lim = false;
    double cq[7], sq[7];
    {
      double qn[7], q2[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) qn[k] = q[k];
      if (active) {
        load7(F->J.to + 8 * (size_t)e, q2);
        refine_step(qn, q2, n, i);
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) sincos(qn[k], &sq[k], &cq[k]);
      lim = active && limits_violated(qn);
    }
    const int tm = F->P->torque_mode;
    if (active && !lim && tm != TCMP_TORQUE_BASE) {
      const double z[7] = {0, 0, 0, 0, 0, 0, 0};
      const double mass = F->P->mass;
      tok = tm == TCMP_TORQUE_DYN ? torque_ok_dyn<false>(cq, sq, z, z, mass)
                                  : torque_ok<false>(cq, sq, z, z, mass);
    }
    const bool coll = collides_wave<true>(cq, sq, active && !lim && tok, sc, g, ss) || lim;
    const bool ok = active && !coll && tok;
    steps += (unsigned)__popcll(__ballot(active));
    if (active) {
      if (ok) {
        double q2[7];
        load7(F->J.to + 8 * (size_t)e, q2);
        refine_step(q, q2, n, i);
        ++i;
      }
      if (!ok || i == n) {
        if (i > 0) atomicAdd(&F->J.accepted[e >> 8], 1);
        F->J.nsafe[e] = i;
        F->J.nsteps[e] = n;
        store7(F->J.last + 8 * (size_t)e, q);
        e = -1;
      }
    }
  }
}

// ---- insertion and rewire ------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_fl_ins_scan(const FleetPlan* __restrict__ fp, int nblk) {
  const FleetPlan& f = fp[blockIdx.x];
  ins_scan_block(f.st, f.bcount, nblk, f.boff);
}
__global__ __launch_bounds__(256) void k_fl_ins_write(const FleetPlan* __restrict__ fp, int nb, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  const FleetPlan& f = fp[q];
  ins_write_block(f.P, f.st, f.tr, f.nn, f.cand, f.cgoal, f.J.nsafe, f.J.nsteps, f.J.last, nb,
                  f.boff, f.second, f.rwlist, b);
}
__global__ void k_fl_ins_final(const FleetPlan* __restrict__ fp, int K, int nb) {
  const int q = threadIdx.x;
  if (q < K) ins_final(fp[q].P, fp[q].st, nb);
}
__global__ __launch_bounds__(256) void k_fl_rewire_scan(const FleetPlan* __restrict__ fp, int bpb) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  const FleetPlan& f = fp[q];
  rewire_scan_block(f.P, f.st, f.tr, f.rwlist, f.nbr, f.ncount, b);
}
template <bool MESH>
__global__ __launch_bounds__(256) void k_fl_rewire_apply(const FleetPlan* __restrict__ fp, int bpb, Geo g) {
  const int q = blockIdx.x / bpb, b = blockIdx.x - q * bpb;
  const FleetPlan& f = fp[q];
  rewire_apply_block<MESH>(f.P, f.st, f.tr, f.rwlist, f.nbr, f.ncount, f.sc, g, b);
}

// ---- host ----------------------------------------------------------------------------------
struct Fleet {
  tcmp_handle* h;          // the lead engine: stream, index buffers, descriptors
  int K;
  int bp, pb;              // lane stride per plan, plan-id key bits
  int lds_obs;             // obstacles over all plans (the fused k_edges' LDS)
  int max_obs;             // the largest plan scene (k_fl_rewire_apply's LDS)
  bool mesh;               // mesh scenes: every plan's scene is the lead's
  FleetPlan* fp;           // device descriptors
  FleetNN* fnn;
};

int fleet_round(const Fleet& F, int nb, long long base) {
  tcmp_handle* h = F.h;
  const int K = F.K, bpb = F.bp / 256, nblk = (nb + 255) / 256;
  const dim3 pg((unsigned)(K * bpb)), b256(256);
  // (event timing on the lead engine, when on: the fleet's kernel times are its)
  hipEvent_t e0, e1 = nullptr;
  h->mark_begin(F_NEAREST, &e0);
  hipLaunchKernelGGL(k_fl_sample, pg, b256, 0, h->stream, F.fp, base, nb, bpb);
  HIPCHK(hipGetLastError());
  const long long Tb = 1 + base;  // the snapshot bound: 1 + samples issued before the round
  if (Tb == 1) {
    hipLaunchKernelGGL(k_fl_root, pg, b256, 0, h->stream, F.fp, nb, bpb);
    HIPCHK(hipGetLastError());
  } else {
    DevState* fst = h->st_nn;
    long long* off = h->f_off.p;
    const long long slots = (long long)K * Tb;
    hipLaunchKernelGGL(k_fl_prep, dim3(1), b256, 0, h->stream, F.fp, K, fst, off, nb);
    hipLaunchKernelGGL(k_fl_node_keys, dim3(std::min<unsigned>(grid_for(slots, 256), 8192)), b256,
                       0, h->stream, F.fp, Tb, slots, F.pb, h->nkeys_in.p, h->nvals_in.p);
    HIPCHK(hipGetLastError());
    size_t tb = h->sort_tmp.n;
    rocprim::double_buffer<unsigned long long> kdb(h->nkeys_in.p, h->skeys.p);
    rocprim::double_buffer<int> vdb(h->nvals_in.p, h->svals.p);
    HIPCHK(rocprim::radix_sort_pairs<SortCfg>(h->sort_tmp.p, tb, kdb, vdb, (size_t)slots, 0,
                                               kKeyBits + F.pb, h->stream));
    unsigned long long* const skeys = kdb.current();
    const int* const svals = vdb.current();
    hipLaunchKernelGGL(k_fl_rows, dim3(grid_for(slots, 256)), b256, 0, h->stream, F.fp, fst, off,
                       svals, Tb, slots, h->stree.p, h->srow.p, h->cflag.p, h->sflag.p);
    hipLaunchKernelGGL(k_nn_cut<kNnC>, dim3(grid_for(slots, 256)), b256, 0, h->stream,
                       &fst->n_nodes, (const int*)nullptr, skeys, h->cflag.p);
    HIPCHK(hipGetLastError());
    tb = h->sort_tmp.n;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(h->sort_tmp.p, tb, h->cflag.p, h->cid.p, (int)slots,
                                            h->stream));
    hipLaunchKernelGGL(k_nn_starts, dim3(grid_for(slots, 256)), b256, 0, h->stream, &fst->n_nodes,
                       (const int*)nullptr, h->cflag.p, h->cid.p, h->cstart.p, &fst->nn_cells);
    const unsigned idx_grid = (unsigned)std::min<long long>(grid_for(slots * 64, 256),
                                                            (long long)h->cu_count * 8);
    hipLaunchKernelGGL(k_nn_cell_boxes, dim3(idx_grid), b256, 0, h->stream, fst, h->stree.p,
                       h->cstart.p, skeys, h->cboxf.p, h->ckey.p);
    hipLaunchKernelGGL(k_nn_cut<kNnS>, dim3(grid_for(slots, 256)), b256, 0, h->stream,
                       (const long long*)nullptr, &fst->nn_cells, h->ckey.p, h->sflag.p);
    hipLaunchKernelGGL(k_fl_super_flags, dim3(1), dim3(64), 0, h->stream, off, h->cid.p,
                       h->sflag.p, K);
    HIPCHK(hipGetLastError());
    tb = h->sort_tmp.n;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(h->sort_tmp.p, tb, h->sflag.p, h->sid.p, (int)slots,
                                            h->stream));
    hipLaunchKernelGGL(k_nn_starts, dim3(grid_for(slots, 256)), b256, 0, h->stream,
                       (const long long*)nullptr, &fst->nn_cells, h->sflag.p, h->sid.p,
                       h->sstart.p, &fst->nn_supers);
    hipLaunchKernelGGL(k_nn_build_supers, dim3(idx_grid), b256, 0, h->stream, fst, h->sstart.p,
                       h->cboxf.p, h->sboxf.p);
    hipLaunchKernelGGL(k_nn_build_blocks, dim3(std::min<unsigned>(grid_for(slots + 128, 256), 1024)),
                       b256, 0, h->stream, fst, h->sboxf.p, h->bboxf.p);
    hipLaunchKernelGGL(k_fl_ranges, dim3(1), dim3(64), 0, h->stream, off, h->cid.p, h->sid.p, fst,
                       F.fnn, K);
    HIPCHK(hipGetLastError());
    // candidates: plan-major, Morton order within a plan (locality only): plan id and Morton
    // bits together at most 16, i.e. two Onesweep passes (19 bits, three passes, measured the
    // same scan and ~0.2 ms more index build per C3 fleet)
    const int nbt = K * nb, cslots = K * F.bp;
    const int cbits = std::min(h->nn_cand_bits, 16 - F.pb);
    hipLaunchKernelGGL(k_fl_cand_keys, pg, b256, 0, h->stream, F.fp, nb, F.bp, F.pb,
                       h->ckeys_in.p, h->cvals_in.p);
    HIPCHK(hipGetLastError());
    const int top = kKeyBits + F.pb;
    tb = h->sort_tmp.n;
    HIPCHK(rocprim::radix_sort_pairs<SortCfg>(h->sort_tmp.p, tb, h->ckeys_in.p, h->ckeys.p,
                                               h->cvals_in.p, h->cperm.p, (size_t)cslots,
                                               std::max(0, top - cbits - F.pb), top,
                                               h->stream));
    hipLaunchKernelGGL(k_fl_home, dim3(grid_for(nbt, 256)), b256, 0, h->stream, off, skeys,
                       h->ckeys_in.p, h->cperm.p, h->cid.p, h->sid.p, nbt, F.bp, h->chome.p);
    HIPCHK(hipGetLastError());
    const long long waves = std::min<long long>(nbt, (long long)h->cu_count * h->nn_waves_per_cu);
    const int per_wave = (int)((nbt + waves - 1) / waves);
    const unsigned blocks = grid_for((nbt + per_wave - 1) / per_wave * 64, kNnBlock);
#define TCMP_FNNW(UWV)                                                                          \
  hipLaunchKernelGGL((k_nearest_wave32<UWV, TCMP_NN_SW, true>), dim3(blocks), dim3(kNnBlock), 0,  \
                     h->stream, h->dP, fst, h->stree.p, h->srow.p, h->cboxf.p, h->sboxf.p,         \
                     h->bboxf.p, (const double*)nullptr, h->cperm.p, h->chome.p, nbt,             \
                     (int*)nullptr, (double*)nullptr, (double*)nullptr, F.fnn, F.bp)
    const hipEvent_t s0 = h->mark();
    if (h->P.uniform_w) TCMP_FNNW(true); else TCMP_FNNW(false);
#undef TCMP_FNNW
    HIPCHK(hipGetLastError());
    e1 = h->mark_end(F_NNSCAN, s0);
  }
  if (!e1) e1 = h->mark();
  h->span(F_NEAREST, e0, e1);
  // edges: each plan's longest-first order (counting sort), work records, one fused k_edges
  const bool ordered = nb >= kEdgeOrderMin;
  if (ordered) {
    hipLaunchKernelGGL(k_fl_edge_order, pg, b256, 0, h->stream, F.fp, nb, bpb);
    hipLaunchKernelGGL(k_fl_cs_scan, dim3(K), dim3(1024), 0, h->stream, F.fp);
    hipLaunchKernelGGL(k_fl_cs_scatter, pg, b256, 0, h->stream, F.fp, nb, bpb);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_fl_edge_records, pg, b256, 0, h->stream, F.fp, nb, ordered ? 1 : 0, bpb);
  HIPCHK(hipGetLastError());
  const hipEvent_t ek = h->mark();
  h->span(F_EDGE_PREP, e1, ek);
  if (F.mesh) {
    // (launch_edges' residency cap, the engine's edge_wps included)
    const long long cap = (long long)h->cu_count * std::max(1, std::min(h->edge_wps, TCMP_EDGE_MINW));
    const long long blocks = std::min<long long>(cap, ((long long)K * nb + 255) / 256);
    hipLaunchKernelGGL(k_fl_edges_mesh, dim3((unsigned)std::max<long long>(1, blocks)), dim3(256),
                       lds_bytes(h), h->stream, F.fp, K, nb, h->scene(), h->geo());
  } else {
    const long long blocks = std::min<long long>(h->cu_count, ((long long)K * nb + 511) / 512);
    const unsigned lds = fleet_lds_bytes(F.lds_obs);
    const int q2lds = lds + fleet_q2_bytes() <= kFleetLdsCap;
    hipLaunchKernelGGL(k_fl_edges, dim3((unsigned)std::max<long long>(1, blocks)), dim3(512),
                       lds + (q2lds ? fleet_q2_bytes() : 0u), h->stream, F.fp, K, nb, h->geo(),
                       q2lds);
  }
  HIPCHK(hipGetLastError());
  const hipEvent_t ee = h->mark_end(F_EDGES, ek);
  // insertion in lane order per plan, bookkeeping, rewire
  hipLaunchKernelGGL(k_fl_ins_scan, dim3(K), dim3(1024), 0, h->stream, F.fp, nblk);
  hipLaunchKernelGGL(k_fl_ins_write, pg, b256, 0, h->stream, F.fp, nb, bpb);
  hipLaunchKernelGGL(k_fl_ins_final, dim3(1), dim3(64), 0, h->stream, F.fp, K, nb);
  const hipEvent_t ei = h->mark_end(F_INSERT, ee);
  hipLaunchKernelGGL(k_fl_rewire_scan, pg, b256, 0, h->stream, F.fp, bpb);
  if (F.mesh)
    hipLaunchKernelGGL(k_fl_rewire_apply<true>, pg, b256, lds_bytes(h), h->stream, F.fp, bpb,
                       h->geo());
  else
    hipLaunchKernelGGL(k_fl_rewire_apply<false>, pg, b256, stage_lds_bytes(F.max_obs), h->stream,
                       F.fp, bpb, h->geo());
  HIPCHK(hipGetLastError());
  h->mark_end(F_REWIRE, ei);
  return 0;
}

// the scene every kernel of a plan sees: boxes, meshes (and their LODs and spheres) and the
// self-collision switch, as the host uploaded them
bool same_scene(const tcmp_handle* a, const tcmp_handle* b) {
  bool same = a->n_box == b->n_box && a->n_mesh == b->n_mesh && a->self_coll == b->self_coll &&
              a->box15 == b->box15 && a->mesh_v == b->mesh_v && a->mesh_p == b->mesh_p &&
              a->mesh_e == b->mesh_e && a->mesh_voff == b->mesh_voff &&
              a->mesh_poff == b->mesh_poff && a->mesh_eoff == b->mesh_eoff &&
              a->mesh_box == b->mesh_box && a->user_lods == b->user_lods &&
              a->user_sph == b->user_sph && a->use_sph == b->use_sph && a->sph_h == b->sph_h;
  for (int i = 0; same && a->user_lods && i < 2; ++i)
    same = a->lod_v[i] == b->lod_v[i] && a->lod_p[i] == b->lod_p[i] && a->lod_e[i] == b->lod_e[i] &&
           a->lod_vo[i] == b->lod_vo[i] && a->lod_po[i] == b->lod_po[i] &&
           a->lod_eo[i] == b->lod_eo[i];
  return same;
}

// The fused kernels' dynamic-LDS limits, at the largest any fleet may launch them with (the
// fleet LDS cap of k_fl_edges, the largest box / lean mesh stage): called by every
// tcmp_create, never per fleet -- a limit is global to its function, and a per-call value
// set by one thread could be lowered by another's smaller fleet before the first one launches.
int fleet_lds_limits() {
  const struct { const void* k; unsigned b; } lim[] = {
      {(const void*)k_fl_edges, kFleetLdsCap},
      {(const void*)k_fl_rewire_apply<false>, stage_lds_bytes(kMaxObstacles)},
      {(const void*)k_fl_edges_mesh, stage_lds_bytes_lean(kMaxObstacles)},
      {(const void*)k_fl_rewire_apply<true>, stage_lds_bytes_lean(kMaxObstacles)}};
  for (const auto& x : lim)
    HIPCHK(hipFuncSetAttribute(x.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)x.b));
  return 0;
}

}  // namespace

extern "C" {

int tcmp_plan_run_fused(tcmp_handle* const* hs, int32_t n, int64_t n_samples, int32_t batch) {
  if (!hs || n < 1 || n > kFleetMax) return fail(-1, "fused rounds take 1..31 engines");
  tcmp_handle* h = hs[0];
  TCMP_ENTER(h);
  if (batch < 1) return fail(-1, "batch size out of range");
  for (int q = 0; q < n; ++q) {
    tcmp_handle* e = hs[q];
    if (!e) return fail(-1, "null handle");
    for (int p = 0; p < q; ++p)
      if (hs[p] == e) return fail(-1, "the same engine twice in a fleet");
    if (e->device != h->device) return fail(-1, "a fleet's engines share one device");
    if (!e->plan_open) return fail(-1, "no open plan (tcmp_plan_begin first)");
    if (batch > e->max_batch) return fail(-1, "batch size out of range");
    if (e->samples_issued != h->samples_issued)
      return fail(-1, "the fleet's plans are not at the same round");
    if (e->samples_issued + n_samples + 1 > e->P.max_nodes) return fail(-3, "tree capacity exceeded");
    // mesh scenes (and self-collision pairs): one scene for the whole fleet, the lead's --
    // replica trees of one query (C5)
    if ((e->mesh_kernels() || h->mesh_kernels()) && !same_scene(e, h))
      return fail(-1, "a fleet over convex-mesh scenes shares one scene");
    if (e->P.uniform_w != h->P.uniform_w || e->P.nn_cmax != h->P.nn_cmax ||
        memcmp(e->P.w, h->P.w, sizeof(h->P.w)) != 0)
      return fail(-1, "a fleet's plans share the distance weights");
  }
  if (n_samples <= 0) return 0;
  Fleet F{};
  F.h = h;
  F.K = n;
  F.bp = (batch + 255) / 256 * 256;
  F.pb = 1;
  while ((1 << F.pb) <= n) ++F.pb;  // the all-ones plan id stays free for unused slots
  int tot = 0, mx = 0;
  for (int q = 0; q < n; ++q) {
    tot += hs[q]->n_obs;
    mx = std::max(mx, hs[q]->n_obs);
  }
  F.lds_obs = tot;
  F.max_obs = mx;
  F.mesh = h->mesh_kernels();
  if (!F.mesh && fleet_lds_bytes(tot) > kFleetLdsCap)
    return fail(-1, "too many obstacles over the fleet's scenes for the fused edge kernel");
  // the fleet index lives in the lead engine's index buffers (its own plan uses none of them
  // during a fused round), sized for every plan's nodes and lanes
  const long long Tmax = 1 + h->samples_issued + n_samples;
  if ((long long)n * Tmax >= INT_MAX || (long long)n * F.bp >= INT_MAX)
    return fail(-1, "a fleet's node or lane slots exceed 2^31 (fewer plans per fleet)");
  if (int rc = ensure_index(h, (size_t)n * (size_t)Tmax, (size_t)n * (size_t)F.bp)) return rc;
  if (int rc = h->chome.ensure(2 * (size_t)n * (size_t)F.bp)) return rc;
  if (int rc = h->f_off.ensure((size_t)n + 1)) return rc;
  const size_t dbytes = sizeof(FleetPlan) * n + sizeof(FleetNN) * n;
  if (int rc = h->f_desc.ensure(dbytes)) return rc;
  F.fp = reinterpret_cast<FleetPlan*>(h->f_desc.p);
  F.fnn = reinterpret_cast<FleetNN*>(h->f_desc.p + sizeof(FleetPlan) * n);
  h->f_host.assign(dbytes, 0);
  FleetPlan* hp = reinterpret_cast<FleetPlan*>(h->f_host.data());
  FleetNN* hn = reinterpret_cast<FleetNN*>(h->f_host.data() + sizeof(FleetPlan) * n);
  int lds_off = 0;
  for (int q = 0; q < n; ++q) {
    tcmp_handle* e = hs[q];
    FleetPlan f{};
    f.P = e->dP;
    f.st = e->st;
    f.tr = Tree{e->cfg.p, e->parent.p, e->tgt.p, e->meta.p};
    f.J = EdgeJob{e->cfg.p, e->nn.p, e->cand.p, 0, e->nsafe.p, e->nsteps.p, e->last.p,
                  e->cperm.p, e->bcount.p, e->erec.p};
    f.cand = e->cand.p;
    f.cgoal = e->cgoal.p;
    f.nn = e->nn.p;
    f.second = e->second.p;
    f.score = e->nnscore.p;
    f.bins = e->cvals_in.p;
    f.hist = e->cs_hist.p;
    f.hoff = e->cs_hoff.p;
    f.bcount = e->bcount.p;
    f.boff = e->boff.p;
    f.rwlist = e->rwlist.p;
    f.nbr = e->nbr.p;
    f.ncount = e->ncount.p;
    f.sc = e->scene();
    f.lds_obs = lds_off;
    lds_off += e->n_obs;
    hp[q] = f;
    hn[q] = FleetNN{e->cand.p, e->nn.p, e->second.p, e->nnscore.p, e->st, 0, 0};
  }
  HIPCHK(hipMemcpyAsync(h->f_desc.p, h->f_host.data(), dbytes, hipMemcpyHostToDevice, h->stream));
  // (the kernels' dynamic-LDS limits are set once, at their largest, by tcmp_create:
  // fleet_lds_limits)
  // the other engines' queued work (their plan_begin) comes first; they wait for the rounds
  for (int q = 1; q < n; ++q) {
    if (!hs[q]->dep_ev) HIPCHK(hipEventCreateWithFlags(&hs[q]->dep_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(hs[q]->dep_ev, hs[q]->stream));
    HIPCHK(hipStreamWaitEvent(h->stream, hs[q]->dep_ev, 0));
  }
  int rounds = 0, scans = 0;
  long long base = h->samples_issued;
  for (long long left = n_samples; left > 0;) {
    const int nb = (int)std::min<long long>(left, batch);
    if (base > 0) ++scans;
    if (int rc = fleet_round(F, nb, base)) return rc;
    ++rounds;
    base += nb;
    left -= nb;
  }
  if (!h->dep_ev) HIPCHK(hipEventCreateWithFlags(&h->dep_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(h->dep_ev, h->stream));
  const int last_nb = (int)(n_samples % batch ? n_samples % batch : batch);
  for (int q = 0; q < n; ++q) {
    tcmp_handle* e = hs[q];
    if (q) HIPCHK(hipStreamWaitEvent(e->stream, h->dep_ev, 0));
    e->samples_issued += n_samples;
    e->launches_nearest += rounds;
    e->launches_scan += scans;
    e->last_nb = last_nb;
    e->fused_plans = n;
  }
  return 0;
}

}  // extern "C"
