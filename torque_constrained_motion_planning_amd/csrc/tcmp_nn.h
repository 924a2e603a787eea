// tcmp_nn.h -- exact nearest neighbour (rrt_star.py:9-14,171) over the Morton-sorted tree
// snapshot, one candidate per wavefront.  Included by tcmp_engine.hip after its state types.
//
// Layout, rebuilt once per round from the snapshot (k_node_keys + radix sort + the two
// build kernels below):
//   stree [T][8] f64   nodes in Morton order: q0..q6, original node index
//   stree32 [T][8] f32 the same coordinates rounded to fp32 (k_nearest_wave32's first pass)
//   cbox  [T/64][16]   f32 bounds of each 64-node chunk (lo rounded down, hi rounded up)
//   sbox  [T/4096][16] f32 bounds of each super-chunk (64 chunks)
// A wave takes Morton-sorted candidates one at a time: it scans the candidate's home chunk
// (lane = node), then tests super-chunk bounds 64 at a time (lane = super-chunk, zig-zag
// order out from the home super-chunk), and inside every super-chunk whose lower bound is
// within the current threshold tests its 64 chunk bounds (lane = chunk) and scans the
// chunks that pass.  Threshold = (sqrt(best) + rewire radius)^2: nodes that can matter for
// the nearest OR for k_insert's rewire bound are never pruned, so nearest index and the
// second-smallest distance are exactly those of the full scan.  Ties: (distance, original
// index) lexicographic, i.e. the first index wins as in rrt_star.py:14.
#pragma once

constexpr int kNnC = 64;              // nodes per chunk
constexpr int kNnS = 64;              // chunks per super-chunk

__global__ __launch_bounds__(256) void k_nn_build_chunks(DevState* st, const double* cfg,
                                                         const int* svals, double* stree,
                                                         float* stree32, float* cbox) {
  const long long T = st->n_nodes;
  if ((long long)blockIdx.x * 256 >= T) return;  // block-uniform
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  double lo[7], hi[7];
  if (p < T) {
    double q[7];
    const int n = svals[p];
    load7(cfg + 8 * (size_t)n, q);
    store7(stree + 8 * p, q);
    stree[8 * p + 7] = (double)n;
    float4* d32 = reinterpret_cast<float4*>(stree32 + 8 * p);
    d32[0] = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
    d32[1] = make_float4((float)q[4], (float)q[5], (float)q[6], 0.f);
#pragma unroll
    for (int k = 0; k < 7; ++k) { lo[k] = q[k]; hi[k] = q[k]; }
  } else {
#pragma unroll
    for (int k = 0; k < 7; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = wave_min(lo[k]);
    hi[k] = wave_max(hi[k]);
  }
  const long long c = p >> 6;  // one wave = one chunk
  if (lane_id() == 0 && c * kNnC < T) {
    float* b = cbox + 16 * c;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      b[k] = __double2float_rd(lo[k]);
      b[8 + k] = __double2float_ru(hi[k]);
    }
    b[7] = 0.f;
    b[15] = 0.f;
  }
}

__global__ __launch_bounds__(256) void k_nn_build_supers(DevState* st, const float* cbox,
                                                         float* sbox) {
  const long long T = st->n_nodes;
  const long long nch = (T + kNnC - 1) / kNnC, nsup = (nch + kNnS - 1) / kNnS;
  const long long sw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (sw >= nsup) return;  // wave-uniform
  const long long c = sw * kNnS + lane_id();
  float lo[7], hi[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = c < nch ? cbox[16 * c + k] : INFINITY;
    hi[k] = c < nch ? cbox[16 * c + 8 + k] : -INFINITY;
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
      hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
    }
  }
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      sbox[16 * sw + k] = lo[k];
      sbox[16 * sw + 8 + k] = hi[k];
    }
    sbox[16 * sw + 7] = 0.f;
    sbox[16 * sw + 15] = 0.f;
  }
}

// home position of each Morton-sorted candidate in the sorted snapshot (lower bound)
__global__ void k_nn_home(DevState* st, const unsigned long long* skeys,
                          const unsigned long long* ckeys, int nb, int* home) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nb) return;
  const long long T = st->n_nodes;
  const unsigned long long k = ckeys[j];
  long long lo = 0, hi = T;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (skeys[mid] < k) lo = mid + 1; else hi = mid;
  }
  home[j] = (int)min(lo, T - 1);
}

template <bool UW>
__device__ __forceinline__ double box_lb(const float* b, const double s[7], const double w[7]) {
  const float4 l0 = *reinterpret_cast<const float4*>(b);
  const float4 l1 = *reinterpret_cast<const float4*>(b + 4);
  const float4 h0 = *reinterpret_cast<const float4*>(b + 8);
  const float4 h1 = *reinterpret_cast<const float4*>(b + 12);
  const double lo[7] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z};
  const double hi[7] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z};
  double lb = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double g = fmax(0.0, fmax(lo[k] - s[k], s[k] - hi[k]));
    lb = fma(UW ? g : w[k] * g, g, lb);
  }
  return lb;
}


// position p of the zig-zag walk out from h over [0, n): h, h+1, h-1, h+2, h-2, ...;
// once one side is exhausted the walk continues on the other.  -1 if p >= n.
__device__ __forceinline__ int zigzag(int h, int p, int n) {
  if (p >= n) return -1;
  if (p == 0) return h;
  const int up = n - 1 - h, dn = h, m = min(up, dn);
  const int k = p - 1;
  if (k < 2 * m) return (k & 1) ? h - (k / 2 + 1) : h + (k / 2 + 1);
  const int r = k - 2 * m;
  return up > dn ? h + m + 1 + r : h - (m + 1 + r);
}

template <bool UW>
__global__ __launch_bounds__(256) void k_nearest_wave(PlanParams P, DevState* st,
                                                      const double* stree, const float* cbox,
                                                      const float* sbox, const double* cand,
                                                      const int* cperm, const int* home, int nb,
                                                      int per_wave, int* nn, double* second) {
  const int lane = lane_id();
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  (void)gw;
  (void)per_wave;
  const long long T = st->n_nodes;
  const int nch = (int)((T + kNnC - 1) / kNnC), nsup = (nch + kNnS - 1) / kNnS;
  double w[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) w[k] = P.w[k];
  const double ru = UW ? P.radius / sqrt(P.w[0]) : P.radius;
  unsigned long long pairs = 0, tests = 0;
  while (true) {
    // dynamic queue over the Morton-sorted candidates: one atomic per candidate per wave
    int jq = 0;
    if (lane == 0) jq = atomicAdd(&st->nn_counter, 1);
    jq = __shfl(jq, 0);
    if (jq >= nb) break;
    const long long j = jq;
    const int lj = cperm[j];
    double s[7];
    load7(cand + 8 * (size_t)lj, s);
    const int hc = min(nch - 1, home[j] / kNnC);
    const int hs = hc / kNnS;
    double b1 = INFINITY, b2 = INFINITY;
    int bi = INT_MAX;
    auto scan = [&](int c) {
      const long long n = (long long)c * kNnC + lane;
      if (n < T) {
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
        } else {
          b2 = fmin(b2, dd);
        }
      }
      pairs += (unsigned long long)min((long long)kNnC, T - (long long)c * kNnC);
      const double t = sqrt(wave_min(b1)) + ru;
      return t * t * (1.0 + 1e-9) + 1e-300;
    };
    auto upd = [&](const double4 a, const double4 b) {
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
      } else {
        b2 = fmin(b2, dd);
      }
    };
    // scan up to four chunks (-1 = none) with all their loads in flight before any use
    auto scan4 = [&](int c0, int c1, int c2, int c3) {
      const int cs[4] = {c0, c1, c2, c3};
      double4 A[4], Bq[4];
      bool val[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long n = (long long)cs[u] * kNnC + lane;
        val[u] = cs[u] >= 0 && n < T;
        if (val[u]) {
          A[u] = *reinterpret_cast<const double4*>(stree + 8 * n);
          Bq[u] = *reinterpret_cast<const double4*>(stree + 8 * n + 4);
        }
        if (cs[u] >= 0) pairs += (unsigned long long)min((long long)kNnC, T - (long long)cs[u] * kNnC);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (val[u]) upd(A[u], Bq[u]);
      const double t = sqrt(wave_min(b1)) + ru;
      return t * t * (1.0 + 1e-9) + 1e-300;
    };
    double thr = scan(hc);
    for (int g = 0; g < nsup; g += 64) {
      const int sidx = zigzag(hs, g + lane, nsup);
      const double lbs = sidx >= 0 ? box_lb<UW>(sbox + 16 * (size_t)sidx, s, w) : INFINITY;
      tests += (unsigned long long)min(64, nsup - g);
      uint64_t smask = __ballot(lbs <= thr);
      while (smask) {
        const int i = __builtin_ctzll(smask);
        smask &= smask - 1;
        if (__shfl(lbs, i) > thr) continue;
        const int S = __shfl(sidx, i);
        const int c = S * kNnS + lane;
        const bool cv = c < nch && c != hc;
        const double lbc = cv ? box_lb<UW>(cbox + 16 * (size_t)c, s, w) : INFINITY;
        tests += (unsigned long long)min(kNnS, nch - S * kNnS);
        uint64_t cmask = __ballot(lbc <= thr);
        while (cmask) {
          // up to 4 chunks per pass: their node loads are independent, so all are in flight
          // together; the threshold is refreshed once per pass
          auto take = [&]() -> int {
            while (cmask) {
              const int k = __builtin_ctzll(cmask);
              cmask &= cmask - 1;
              if (__shfl(lbc, k) <= thr) return S * kNnS + k;
            }
            return -1;
          };
          const int ca = take(), cb = take(), cc = take(), cd = take();
          if (ca >= 0) thr = scan4(ca, cb, cc, cd);
        }
      }
    }
    // lexicographic (distance, index) winner and the second-smallest distance
    const double m = wave_min(b1);
    const int wi = wave_min_int(b1 == m ? bi : INT_MAX);
    const bool winner = (b1 == m) && (bi == wi);
    const double sec = wave_min(winner ? b2 : b1);
    if (lane == 0) {
      nn[lj] = wi == INT_MAX ? 0 : wi;
      if (second) second[lj] = sec;
    }
  }
  if (lane == 0) {
    atomicAdd(&st->nn_pairs, pairs);
    atomicAdd(&st->nn_box_tests, tests);
  }
}
