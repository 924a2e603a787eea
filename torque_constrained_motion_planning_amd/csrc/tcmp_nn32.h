// tcmp_nn32.h -- k_nearest_wave32: the exact nearest-neighbour scan of tcmp_nn.h with an fp32
// first pass.  Included by
// tcmp_engine.hip after tcmp_nn.h.
//
// Every (candidate, node) pair is first evaluated in fp32 on the f32 rows srow (half the bytes
// of the fp64 rows, twice the VALU rate).  A node is re-evaluated exactly in fp64 (the same
// arithmetic as the reference's distance fn, so the winner and its distance are bit-identical)
// only when its fp32 value r32 could belong to a node at least as close as the wave's current
// best m:
//
//   |q| <= cmax (P.nn_cmax: 8 > the joint-limit magnitude 3.7525 on the planner's path; the
//   data's own bound for tcmp_nearest), so each fp32 coordinate difference is within
//   e = 4 u cmax of the exact one (u = 2^-24), and with
//   D = exact weighted distance, E = e sqrt(sum w):   r32 <= (1 + g) (D + E)^2,  g = 16 u.
//   Refine iff r32 <= R(m) = (1 + g)(sqrt(m) + E)^2 (rounded up, with slack).
//
// (16-bit first-pass rows were measured in round 3 and dropped: DESIGN.md section 4.)
//
// Nodes that are not refined feed the second-smallest distance through the matching lower
// bound LB(r32) = (sqrt(r32 / (1 + g)) - E)^2, so `second` is a lower bound of the exact value:
// k_ins_write's rewire flag (a "may need the neighbour scan" test) stays conservative, and the
// neighbour scan itself is exact.  Pruning uses the exact fp64 best, as before.
//
// The pruning threshold is the nearest search's own, thr >= m (rounded up): every node the scan
// never looked at is farther than the final thr, so second = min(second over the nodes looked
// at, thr) is still a lower bound of the true second-smallest distance.  k_ins_write flags a
// new node for the neighbour scan when second < (|q_new - s| + r)^2; that ball lies inside the
// searched one unless the edge advanced less than r, and then second <= thr < (.. + r)^2 flags
// it anyway.  (Round 1 padded the threshold to (sqrt(m) + r)^2 instead, so that `second` was
// exact out to the rewire ball: a 7-D search ball a few percent wider.)
//
// Work distribution: eight queues, one per XCD, each over a contiguous eighth of the
// Morton-sorted candidates; a wave pulls batches of four from its own XCD's queue
// (HW_REG_XCC_ID) so the nodes one XCD touches stay in its L2, and moves on to the next queue
// when it runs dry.
#pragma once

constexpr double kNnU32 = 5.9604644775390625e-08;  // 2^-24
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr double kNnG = 16.0 * kNnU32;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

// Lower bound of the weighted squared distance from s to a float box, in fp32, never above
// the exact value.  sh = s32 + G and sl = s32 - G (rounded to nearest) with G = 8 u cmax:
// |s32 - s| <= u cmax and the roundings of sh, sl and of the two subtractions add at most
// 3 u cmax more, so each computed gap max(lo - sh, sl - hi, 0) stays below the exact gap
// max(lo - s, s - hi, 0); the weighted sum of squares is scaled down by 1e-6 relative to cover
// its own rounding.
template <bool UW>
__device__ __forceinline__ float box_lb32(const float* b, const float sh[7], const float sl[7],
                                          const float w[7], int* start = nullptr,
                                          int* count = nullptr) {
  const float4 l0 = *reinterpret_cast<const float4*>(b);
  const float4 l1 = *reinterpret_cast<const float4*>(b + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(b + 8);
  const float4 h1 = *reinterpret_cast<const float4*>(b + 12);
  if (start) *start = __float_as_int(l1.w);
  if (count) *count = __float_as_int(h1.w);
  // the two gaps of a coordinate pair per packed subtraction (v_pk_add_f32), the squares
  // accumulated per pair (v_pk_fma_f32); any association of the seven terms is covered by
  // the 1e-6 relative scale-down
  const f32x2 a01 = f32x2{l0.x, l0.y} - f32x2{sh[0], sh[1]};
  const f32x2 a23 = f32x2{l0.z, l0.w} - f32x2{sh[2], sh[3]};
  const f32x2 a45 = f32x2{l1.x, l1.y} - f32x2{sh[4], sh[5]};
  const f32x2 b01 = f32x2{sl[0], sl[1]} - f32x2{h0.x, h0.y};
  const f32x2 b23 = f32x2{sl[2], sl[3]} - f32x2{h0.z, h0.w};
  const f32x2 b45 = f32x2{sl[4], sl[5]} - f32x2{h1.x, h1.y};
  const float a6 = l1.z - sh[6], b6 = sl[6] - h1.z;
  const f32x2 g01 = {fmaxf(fmaxf(a01.x, b01.x), 0.f), fmaxf(fmaxf(a01.y, b01.y), 0.f)};
  const f32x2 g23 = {fmaxf(fmaxf(a23.x, b23.x), 0.f), fmaxf(fmaxf(a23.y, b23.y), 0.f)};
  const f32x2 g45 = {fmaxf(fmaxf(a45.x, b45.x), 0.f), fmaxf(fmaxf(a45.y, b45.y), 0.f)};
  const float g6 = fmaxf(fmaxf(a6, b6), 0.f);
  f32x2 acc;
  float lb;
  if (UW) {
    acc = g01 * g01;
    acc = __builtin_elementwise_fma(g23, g23, acc);
    acc = __builtin_elementwise_fma(g45, g45, acc);
    lb = fmaf(g6, g6, acc.x + acc.y);
  } else {
    acc = (f32x2{w[0], w[1]} * g01) * g01;
    acc = __builtin_elementwise_fma(f32x2{w[2], w[3]} * g23, g23, acc);
    acc = __builtin_elementwise_fma(f32x2{w[4], w[5]} * g45, g45, acc);
    lb = fmaf(w[6] * g6, g6, acc.x + acc.y);
  }
  return lb * 0.999999f;
}

#ifndef TCMP_NN_MINB
#define TCMP_NN_MINB 1  // min blocks per CU the register allocation must allow
#endif
// The scan's workgroups are 1024 threads (16 waves, one workgroup per CU at 4 waves per SIMD)
// and hold the super-cell boxes in LDS when there are at most kNnLdsSup of them (128 KB, which
// costs no occupancy: the VGPRs already allow one workgroup per CU; a fused round's index over
// four 1e6-sample plans has ~1,600 super-cells -- 4.65 -> 4.31 ms per C3 fleet scan): the
// super-cell tests then cost an LDS round trip instead of an L2 one, and the block level (whose
// only job is to save super-cell box loads) is skipped.  Larger indexes walk the blocks from
// global memory as before.  (One walk over a flat pointer serving both was 5 % slower.)
#ifndef TCMP_NN_BLOCK
#define TCMP_NN_BLOCK 1024
#endif
constexpr int kNnBlock = TCMP_NN_BLOCK;
#ifndef TCMP_NN_LDS_SUP
#define TCMP_NN_LDS_SUP 2048
#endif
constexpr int kNnLdsSup = TCMP_NN_LDS_SUP;
// SW: cells per scan round (2 in the engine).  Passing cells queue up across super-cells (the queue
// holds at most SW) and a round loads all their rows at once: fewer dependent round trips
// per candidate than one round per super-cell.
// FLEET (tcmp_fleet.h): one index over several plans' trees (each plan's nodes a contiguous
// key range, its cells and super-cells [s0, s1) its own); candidate slot g belongs to plan
// g / bp, row g % bp of that plan's buffers, and walks only its plan's super-cells.
struct FleetNN {
  const double* cand;
  int* nn;
  double* second;
  double* score;
  DevState* st;   // the plan's counters (nn_pairs, nn_box_tests)
  int s0, s1;     // the plan's super-cells in this round's index (k_fl_ranges)
};

template <bool UW, int SW, bool FLEET = false>
__global__ __launch_bounds__(kNnBlock, TCMP_NN_MINB) void k_nearest_wave32(const PlanParams* __restrict__ Pd, DevState* st,
                                                        const double* stree,
                                                        const float* srow, const float* cbox,
                                                        const float* sbox, const float* bbox,
                                                        const double* cand,
                                                        const int* cperm, const int* home, int nb,
                                                        int* nn, double* second, double* score,
                                                        const FleetNN* __restrict__ fnn = nullptr,
                                                        int bp = 0) {
  const PlanParams P = *Pd;
  const int lane = lane_id();
  const long long T = st->n_nodes;
  const int nsup = st->nn_supers;
  __shared__ float4 lsup[4 * kNnLdsSup];
  const bool sup_lds = nsup <= kNnLdsSup;
  if (sup_lds) {
    const float4* g4 = reinterpret_cast<const float4*>(sbox);
    for (int i = threadIdx.x; i < 4 * nsup; i += blockDim.x) lsup[i] = g4[i];
    __syncthreads();
  }
  const float* lsupf = reinterpret_cast<const float*>(lsup);
  double w[7], wsum = 0;
  float w32[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    w[k] = P.w[k];
    w32[k] = (float)w[k];
    wsum += w[k];
  }
  const double E = 4.0 * kNnU32 * P.nn_cmax * sqrt(UW ? 7.0 : wsum) * (1.0 + 1e-6);
  const float G = (float)(8.0 * kNnU32 * P.nn_cmax);  // box_lb32's coordinate shift
  const float E32 = __double2float_ru(E * (1.0 + 1e-9));
  const float kRfac = __double2float_ru((1.0 + kNnG) * (1.0 + 3e-6));
  unsigned long long pairs = 0, tests = 0;
  int cur = -1;  // FLEET: the plan whose counters pairs / tests hold
#ifdef TCMP_PROF
  // clocks: [0] setup + home chunk, [1] super-chunk bounds, [2] chunk bounds, [3] chunk scans,
  // [4] final reduction
  unsigned long long pc[5] = {0, 0, 0, 0, 0};
  // visits: [0] super-cell box wave tests (passing blocks), [1] cell box wave tests (passing
  // super-cells), [2] cells pushed to the scan queue
  unsigned long long pv[3] = {0, 0, 0};
  unsigned long long t0 = clock64();
#define NN_TICK(k) { const unsigned long long t1 = clock64(); pc[k] += t1 - t0; t0 = t1; }
#else
#define NN_TICK(k)
#endif
  // Candidates are taken kNnBatch at a time: one atomic per batch, the batch's cperm / home /
  // candidate rows loaded once by lanes 0..3, and the next batch's atomic issued before this
  // batch's work so its latency overlaps the first chunk loads.
#ifndef TCMP_NN_BATCH
#define TCMP_NN_BATCH 4
#endif
  constexpr int kNnBatch = TCMP_NN_BATCH;
  int qi = (int)xcc_id(), tried = 0;
  int jb = -1, jn = 0;
  auto grab_slow = [&]() {
    jb = -1;
    jn = 0;
    while (tried < 8) {
      const int lo = (int)((long long)nb * qi / 8), hi = (int)((long long)nb * (qi + 1) / 8);
      int t = 0;
      if (lane == 0) t = atomicAdd(&st->nn_queue[qi], kNnBatch);
      t = __shfl(t, 0);
      if (lo + t < hi) {
        jb = lo + t;
        jn = min(kNnBatch, hi - jb);
        return;
      }
      qi = (qi + 1) & 7;
      ++tried;
    }
  };
  grab_slow();
  while (jb >= 0) {
    const bool bl = lane < jn;
    const int ljl = bl ? cperm[jb + lane] : 0;
    const int hml = bl ? home[jb + lane] : 0;
    const int hsu = bl ? home[nb + jb + lane] : 0;
    const int hsl = bl ? __float_as_int(cbox[16 * (size_t)hml + 7]) : 0;
    const int hnl = bl ? __float_as_int(cbox[16 * (size_t)hml + 15]) : 0;
    double sl[7];
    if (bl) {
      if (FLEET) {
        const int pl = ljl / bp;
        load7(fnn[pl].cand + 8 * (size_t)(ljl - pl * bp), sl);
      } else {
        load7(cand + 8 * (size_t)ljl, sl);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 7; ++k) sl[k] = 0.0;
    }
    const int qlo = (int)((long long)nb * qi / 8), qhi = (int)((long long)nb * (qi + 1) / 8);
    int tn = 0;
    if (lane == 0) tn = atomicAdd(&st->nn_queue[qi], kNnBatch);
  for (int ib = 0; ib < jn; ++ib) {
    const int lj = __builtin_amdgcn_readlane(ljl, ib);
    const int fpl = FLEET ? lj / bp : 0;  // plan of the candidate, its super-cells [fs0, fs1)
    const int fs0 = FLEET ? fnn[fpl].s0 : 0, fs1 = FLEET ? fnn[fpl].s1 : nsup;
    if (FLEET && fpl != cur) {
      if (cur >= 0 && lane == 0) {
        atomicAdd(&fnn[cur].st->nn_pairs, pairs);
        atomicAdd(&fnn[cur].st->nn_box_tests, tests);
      }
      pairs = tests = 0;
      cur = fpl;
    }
    double s[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) s[k] = readlane_d(sl[k], ib);
    float s32[7], sh[7], sl32[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      // wave-uniform: readfirstlane puts them back in SGPRs (the VALU arithmetic leaves them
      // in VGPRs otherwise, 21 registers the scan loop needs)
      s32[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int((float)s[k])));
      sh[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s32[k] + G)));
      sl32[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s32[k] - G)));
    }
    const int hc = __builtin_amdgcn_readlane(hml, ib);
    const int hcs = __builtin_amdgcn_readlane(hsl, ib), hcn = __builtin_amdgcn_readlane(hnl, ib);
    const int hs = __builtin_amdgcn_readlane(hsu, ib);
    double b1 = INFINITY, b2 = INFINITY;
    int bi = INT_MAX;
    float r2 = INFINITY;   // smallest fp32 value among this lane's unrefined nodes
    float Rf = INFINITY;   // refine threshold R(m) (wave-uniform)
    bool imp = false;      // this lane's exact best improved since the last refresh
    auto refine = [&](long long n) {
      const double* nd = stree + 8 * n;
      const double4 a = *reinterpret_cast<const double4*>(nd);
      const double4 b = *reinterpret_cast<const double4*>(nd + 4);
      const double d0 = s[0] - a.x, d1 = s[1] - a.y, d2 = s[2] - a.z, d3 = s[3] - a.w,
                   d4 = s[4] - b.x, d5 = s[5] - b.y, d6 = s[6] - b.z;
      double dd;
      if (UW) {
        dd = d0 * d0;
        dd = fma(d1, d1, dd); dd = fma(d2, d2, dd); dd = fma(d3, d3, dd);
        dd = fma(d4, d4, dd); dd = fma(d5, d5, dd); dd = fma(d6, d6, dd);
      } else {
        dd = w[0] * (d0 * d0);
        dd = fma(w[1] * d1, d1, dd); dd = fma(w[2] * d2, d2, dd); dd = fma(w[3] * d3, d3, dd);
        dd = fma(w[4] * d4, d4, dd); dd = fma(w[5] * d5, d5, dd); dd = fma(w[6] * d6, d6, dd);
      }
      const int idx = (int)b.w;
      if (dd < b1 || (dd == b1 && idx < bi)) {
        b2 = b1;
        b1 = dd;
        bi = idx;
        imp = true;
      } else {
        b2 = fmin(b2, dd);
      }
    };
    // packed fp32 (v_pk_add / v_pk_fma: two joints per instruction); any association of the
    // seven terms stays inside the error model's g = 16 u
    const f32x2 w01 = {w32[0], w32[1]}, w23 = {w32[2], w32[3]}, w45 = {w32[4], w32[5]},
                w6 = {w32[6], 0.f};
    const f32x2 s01 = {s32[0], s32[1]}, s23 = {s32[2], s32[3]}, s45 = {s32[4], s32[5]},
                s6 = {s32[6], 0.f};
    auto dist32 = [&](const float4 a, const float4 b) {
      const f32x2 d01 = s01 - f32x2{a.x, a.y}, d23 = s23 - f32x2{a.z, a.w},
                  d45 = s45 - f32x2{b.x, b.y}, d6 = s6 - f32x2{b.z, 0.f};
      f32x2 acc;
      if (UW) {
        acc = d01 * d01;
        acc = __builtin_elementwise_fma(d23, d23, acc);
        acc = __builtin_elementwise_fma(d45, d45, acc);
        acc = __builtin_elementwise_fma(d6, d6, acc);
      } else {
        acc = (w01 * d01) * d01;
        acc = __builtin_elementwise_fma(w23 * d23, d23, acc);
        acc = __builtin_elementwise_fma(w45 * d45, d45, acc);
        acc = __builtin_elementwise_fma(w6 * d6, d6, acc);
      }
      return acc.x + acc.y;
    };
    // refresh the pruning threshold and the refine threshold from the exact best m, in fp32
    // rounded upward (m32 >= m, so both thresholds only grow: pruning and refinement stay
    // conservative)
    auto refresh = [&]() {
      // (each round-to-nearest step is covered by a 1e-6 relative margin, >> 2^-24)
      const float m32 = wave_minf_bc(__double2float_ru(b1));
      const float sm = sqrtf(m32) * 1.000001f;
      const float t = sm * 1.000001f;
      const float tr = (sm + E32) * 1.000001f;
      Rf = tr * tr * kRfac;
      return t * t * 1.000003f;
    };
    // up to SW cells (count 0 = none), all row loads in flight before any use
    auto scanw = [&](const int cs[SW], const int cn[SW]) -> void {
      float4 A[SW], Bq[SW];
      bool val[SW];
#pragma unroll
      for (int u = 0; u < SW; ++u) {
        // wave-uniform row base + lane offset
        const int c0 = __builtin_amdgcn_readfirstlane(cs[u]);
        const int cnt = __builtin_amdgcn_readfirstlane(cn[u]);
        val[u] = lane < cnt;
        const float4* rp = reinterpret_cast<const float4*>(srow) + 2 * (unsigned)c0;
        if (val[u]) {
          A[u] = rp[2 * lane];
          Bq[u] = rp[2 * lane + 1];
        }
        pairs += (unsigned long long)cnt;
      }
      // the SW distances first, then one branch: refinement (r <= Rf) is the rare case
      float r[SW];
      float rm = INFINITY;
#pragma unroll
      for (int u = 0; u < SW; ++u) {
        r[u] = val[u] ? dist32(A[u], Bq[u]) : INFINITY;
        rm = fminf(rm, r[u]);
      }
      if (rm <= Rf) {
#pragma unroll
        for (int u = 0; u < SW; ++u) {
          if (r[u] <= Rf) refine((long long)cs[u] + lane);
          else r2 = fminf(r2, r[u]);
        }
      } else {
        r2 = fminf(r2, rm);
      }
    };
    // queue of passing cells (wave-uniform), scanned SW at a time
    int pcs[SW], pcn[SW], np = 0;
#pragma unroll
    for (int u = 0; u < SW; ++u) { pcs[u] = 0; pcn[u] = 0; }
    float thr;
    auto flush = [&]() {
      if (np) {
        scanw(pcs, pcn);
        // the thresholds only move when some lane's exact best improved
        if (__ballot(imp)) {
          thr = refresh();
          imp = false;
        }
        np = 0;
#pragma unroll
        for (int u = 0; u < SW; ++u) pcn[u] = 0;
      }
    };
    auto push = [&](int cs, int cn) {
#pragma unroll
      for (int u = 0; u < SW; ++u)
        if (u == np) { pcs[u] = cs; pcn[u] = cn; }
      if (++np == SW) flush();
    };
    {
      // home cell: R = inf, every node exact
      if (lane < hcn) refine((long long)hcs + lane);
      pairs += (unsigned long long)hcn;
      thr = refresh();
      imp = false;
    }
    NN_TICK(0);
    // the cells of a passing super-cell: one box test per lane, passing cells to the queue
    auto super_cells = [&](int S0, int Sn) {
      const int c = S0 + lane;
      const bool cv = lane < Sn && c != hc;
      int cst = 0, ccn = 0;
      const float lbc = cv ? box_lb32<UW>(cbox + 16 * (size_t)c, sh, sl32, w32, &cst, &ccn) : INFINITY;
      tests += (unsigned long long)Sn;
#ifdef TCMP_PROF
      ++pv[1];
#endif
      uint64_t cmask = __ballot(lbc <= thr);
      NN_TICK(2);
      while (cmask) {
        const int k = __builtin_ctzll(cmask);
        cmask &= cmask - 1;
        if (readlane_f(lbc, k) <= thr) {
#ifdef TCMP_PROF
          ++pv[2];
#endif
          push(__builtin_amdgcn_readlane(cst, k), __builtin_amdgcn_readlane(ccn, k));
        }
      }
      NN_TICK(3);
    };
    if (sup_lds) {
      // super-cells from LDS, 64 per test round, zig-zagging out from the home super-cell
      const int nsp = fs1 - fs0;
      for (int gs = 0; gs < nsp; gs += 64) {
        const int zi = zigzag(hs - fs0, gs + lane, nsp);
        const int sidx = zi >= 0 ? fs0 + zi : -1;
        int sc0 = 0, scn = 0;
        const float lbs =
            sidx >= 0 ? box_lb32<UW>(lsupf + 16 * sidx, sh, sl32, w32, &sc0, &scn) : INFINITY;
        tests += (unsigned long long)min(64, nsp - gs);
#ifdef TCMP_PROF
        ++pv[0];
#endif
        uint64_t smask = __ballot(lbs <= thr);
        NN_TICK(1);
        while (smask) {
          const int i = __builtin_ctzll(smask);
          smask &= smask - 1;
          if (readlane_f(lbs, i) > thr) continue;
          super_cells(__builtin_amdgcn_readlane(sc0, i), __builtin_amdgcn_readlane(scn, i));
        }
      }
    } else {
      // blocks of 64 super-cells, zig-zagging out from the home block (one box test each);
      // a passing block's super-cells are tested one per lane, starting at the home super
      // (a plan's blocks: those overlapping [fs0, fs1); the blocks at its ends may hold
      // other plans' super-cells, which the super-cell loop skips)
      const int b0 = fs0 >> 6, nblk = ((fs1 - 1) >> 6) - b0 + 1, hb = (hs >> 6) - b0;
      for (int gb = 0; gb < nblk; gb += 64) {
        const int zb = zigzag(hb, gb + lane, nblk);
        const int bidx = zb >= 0 ? b0 + zb : -1;
        const float lbb = bidx >= 0 ? box_lb32<UW>(bbox + 16 * (size_t)bidx, sh, sl32, w32) : INFINITY;
        tests += (unsigned long long)min(64, nblk - gb);
        uint64_t bmask = __ballot(lbb <= thr);
        while (bmask) {
          const int ib = __builtin_ctzll(bmask);
          bmask &= bmask - 1;
          if (readlane_f(lbb, ib) > thr) continue;
          const int blk = __builtin_amdgcn_readlane(bidx, ib);
          const int rot = blk == (hs >> 6) ? (hs & 63) : 0;
          const int sidx = 64 * blk + ((lane + rot) & 63);
          int sc0 = 0, scn = 0;
          const float lbs = (sidx < fs1 && sidx >= fs0)
                                ? box_lb32<UW>(sbox + 16 * (size_t)sidx, sh, sl32, w32, &sc0, &scn)
                                : INFINITY;
          tests += (unsigned long long)min(64, fs1 - 64 * blk);
#ifdef TCMP_PROF
          ++pv[0];
#endif
          uint64_t smask = __ballot(lbs <= thr);
          NN_TICK(1);
          while (smask) {
            const int i = __builtin_ctzll(smask);
            smask &= smask - 1;
            if (readlane_f(lbs, i) > thr) continue;
            super_cells(__builtin_amdgcn_readlane(sc0, i), __builtin_amdgcn_readlane(scn, i));
          }
        }
      }
    }
    flush();
    const double m = wave_min(b1);
    const int wi = wave_min_int(b1 == m ? bi : INT_MAX);
    const bool winner = (b1 == m) && (bi == wi);
    double lb2 = INFINITY;
    if (r2 < INFINITY) {
      const double t = sqrt((double)r2 / (1.0 + kNnG)) - E;
      lb2 = t > 0.0 ? t * t * (1.0 - 1e-7) : 0.0;
    }
    const double mine = winner ? fmin(b2, lb2) : fmin(fmin(b1, b2), lb2);
    const double sec = wave_min(mine);
    if (lane == 0) {
      int* no = nn;
      double *so = second, *sco = score;
      int oi = lj;
      if (FLEET) {
        no = fnn[fpl].nn;
        so = fnn[fpl].second;
        sco = fnn[fpl].score;
        oi = lj - fpl * bp;
      }
      no[oi] = wi == INT_MAX ? 0 : wi;
      if (so) so[oi] = fmin(sec, (double)thr);
      if (sco) sco[oi] = m;
    }
    NN_TICK(4);
  }
    tn = __shfl(tn, 0);
    if (qlo + tn < qhi) {
      jb = qlo + tn;
      jn = min(kNnBatch, qhi - jb);
    } else {
      qi = (qi + 1) & 7;
      ++tried;
      grab_slow();
    }
  }
  if (lane == 0 && (!FLEET || cur >= 0)) {
    DevState* const sp = FLEET ? fnn[cur].st : st;
    atomicAdd(&sp->nn_pairs, pairs);
    atomicAdd(&sp->nn_box_tests, tests);
#ifdef TCMP_PROF
    for (int k = 0; k < 5; ++k) atomicAdd(&st->prof_nn[k], pc[k]);
    for (int k = 0; k < 3; ++k) atomicAdd(&st->prof_nn[5 + k], pv[k]);
#endif
  }
#undef NN_TICK
}

