// tcmp_nng.h -- k_nearest_bfs: the exact nearest-neighbour scan over the snapshot index of
// tcmp_nn.h, level by level.  Included by tcmp_engine.hip after tcmp_nn32.h (whose fp32
// error model, box bound and helpers it shares).
//
// The depth-first scan of k_nearest_wave32 walks block -> super-cells -> cells -> rows one
// passing box at a time, so a candidate costs a few dozen DEPENDENT L2 round trips (the
// counters show its waves waiting ~60 % of their cycles).  Here each level is one batch of
// independent loads:
//   1. home cell (exact) -> first threshold;
//   2. every block box, one per lane -> passing blocks;
//   3. the 64 super-cell boxes of up to 4 passing blocks per round (4 loads in flight per
//      lane) -> passing super-cells appended to a per-wave LDS list;
//   4. the cell boxes of up to 4 listed super-cells per round -> passing cells appended,
//      with their lower bound, to a second LDS list;
//   5. the listed cells, in list order (Morton proximity: near cells first), re-filtered
//      against the current threshold (it only shrinks) and scanned four at a time.
// Boxes are tested against the threshold current at the time (never smaller than the final
// one), so no node that can matter is skipped: results are exact, as in k_nearest_wave32.
#pragma once

constexpr int kBfsSupCap = 320;   // listed super-cells per wave (flushed above cap - 256)
constexpr int kBfsCellCap = 512;  // listed cells per wave (flushed above cap - 256)

template <bool UW>
__global__ __launch_bounds__(256, TCMP_NN_MINB) void k_nearest_bfs(
    PlanParams P, DevState* st, const double* stree, const float* stree32, const float* cbox,
    const float* sbox, const float* bbox, const double* cand, const int* cperm, const int* home,
    int nb, int* nn, double* second, double* score) {
  __shared__ int2 s_sup[4][kBfsSupCap];     // (first cell, cell count) of passing super-cells
  __shared__ int2 s_cell[4][kBfsCellCap];   // (first row, row count) of passing cells
  __shared__ float s_clb[4][kBfsCellCap];   // their lower bounds
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  int2* sup = s_sup[wv];
  int2* cel = s_cell[wv];
  float* clb = s_clb[wv];
  const int nsup = st->nn_supers;
  double w[7], wsum = 0;
  float w32[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    w[k] = P.w[k];
    w32[k] = (float)w[k];
    wsum += w[k];
  }
  const double E = 4.0 * kNnU32 * P.nn_cmax * sqrt(UW ? 7.0 : wsum) * (1.0 + 1e-6);
  const float gap = (float)(1.25e-7 * P.nn_cmax);
  const double ru = UW ? P.radius / sqrt(P.w[0]) : P.radius;
  const float E32 = __double2float_ru(E * (1.0 + 1e-9)), ru32 = __double2float_ru(ru);
  const float kRfac = __double2float_ru((1.0 + kNnG) * (1.0 + 3e-6));
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  unsigned long long pairs = 0, tests = 0;
  constexpr int kNnBatch = 4;
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
      load7(cand + 8 * (size_t)ljl, sl);
    } else {
#pragma unroll
      for (int k = 0; k < 7; ++k) sl[k] = 0.0;
    }
    const int qlo = (int)((long long)nb * qi / 8), qhi = (int)((long long)nb * (qi + 1) / 8);
    int tn = 0;
    if (lane == 0) tn = atomicAdd(&st->nn_queue[qi], kNnBatch);
    for (int ib = 0; ib < jn; ++ib) {
      const int lj = __builtin_amdgcn_readlane(ljl, ib);
      double s[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) s[k] = readlane_d(sl[k], ib);
      float s32[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) s32[k] = (float)s[k];
      const int hc = __builtin_amdgcn_readlane(hml, ib);
      const int hcs = __builtin_amdgcn_readlane(hsl, ib), hcn = __builtin_amdgcn_readlane(hnl, ib);
      const int hs = __builtin_amdgcn_readlane(hsu, ib);
      double b1 = INFINITY, b2 = INFINITY;
      int bi = INT_MAX;
      float r2 = INFINITY;  // smallest fp32 value among this lane's unrefined nodes
      float Rf = INFINITY;  // refine threshold R(m) (wave-uniform)
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
        } else {
          b2 = fmin(b2, dd);
        }
      };
      auto upd = [&](const float4 a, const float4 b, long long n) {
        const float d0 = s32[0] - a.x, d1 = s32[1] - a.y, d2 = s32[2] - a.z, d3 = s32[3] - a.w,
                    d4 = s32[4] - b.x, d5 = s32[5] - b.y, d6 = s32[6] - b.z;
        float r;
        if (UW) {
          r = d0 * d0;
          r = fmaf(d1, d1, r); r = fmaf(d2, d2, r); r = fmaf(d3, d3, r);
          r = fmaf(d4, d4, r); r = fmaf(d5, d5, r); r = fmaf(d6, d6, r);
        } else {
          r = w32[0] * (d0 * d0);
          r = fmaf(w32[1] * d1, d1, r); r = fmaf(w32[2] * d2, d2, r); r = fmaf(w32[3] * d3, d3, r);
          r = fmaf(w32[4] * d4, d4, r); r = fmaf(w32[5] * d5, d5, r); r = fmaf(w32[6] * d6, d6, r);
        }
        if (r <= Rf) refine(n);
        else r2 = fminf(r2, r);
      };
      auto refresh = [&]() {
        const float m32 = wave_minf(__double2float_ru(b1));
        const float sm = sqrtf(m32) * 1.000001f;
        const float t = (sm + ru32) * 1.000001f;
        const float tr = (sm + E32) * 1.000001f;
        Rf = tr * tr * kRfac;
        return t * t * 1.000003f;
      };
      auto scan4 = [&](const int cs[4], const int cn[4]) {
        float4 A[4], Bq[4];
        bool val[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long long n = (long long)cs[u] + lane;
          val[u] = lane < cn[u];
          if (val[u]) {
            A[u] = *reinterpret_cast<const float4*>(stree32 + 8 * n);
            Bq[u] = *reinterpret_cast<const float4*>(stree32 + 8 * n + 4);
          }
          pairs += (unsigned long long)cn[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (val[u]) upd(A[u], Bq[u], (long long)cs[u] + lane);
        return refresh();
      };
      float thr;
      {
        if (lane < hcn) refine((long long)hcs + lane);
        pairs += (unsigned long long)hcn;
        thr = refresh();
      }
      int nsl = 0, ncl = 0;
      // 5. scan the listed cells in list order, re-filtered against the shrinking threshold
      auto flush_cells = [&]() {
        for (int base = 0; base < ncl; base += 64) {
          const int i = base + lane;
          int2 ce = make_int2(0, 0);
          float lb = INFINITY;
          if (i < ncl) {
            ce = cel[i];
            lb = clb[i];
          }
          uint64_t m = __ballot(lb <= thr);
          while (m) {
            int cs4[4], cn4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              cs4[u] = 0;
              cn4[u] = 0;
              while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                if (readlane_f(lb, k) <= thr) {
                  cs4[u] = __builtin_amdgcn_readlane(ce.x, k);
                  cn4[u] = __builtin_amdgcn_readlane(ce.y, k);
                  break;
                }
              }
            }
            if (cn4[0] > 0) thr = scan4(cs4, cn4);
          }
        }
        ncl = 0;
      };
      // 4. cell boxes of the listed super-cells, four super-cells per round
      auto flush_supers = [&]() {
        for (int i = 0; i < nsl; i += 4) {
          int cst[4], ccn[4];
          float lbc[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            cst[u] = 0;
            ccn[u] = 0;
            lbc[u] = INFINITY;
            if (i + u < nsl) {
              const int2 sp = sup[i + u];
              const int c = sp.x + lane;
              if (lane < sp.y && c != hc) {
                lbc[u] = box_lb32<UW>(cbox + 16 * (size_t)c, s32, w32, gap, &cst[u], &ccn[u]);
              }
              tests += (unsigned long long)sp.y;
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool p = lbc[u] <= thr;
            const uint64_t m = __ballot(p);
            if (p) {
              const int pos = ncl + (int)__popcll(m & lt_mask);
              cel[pos] = make_int2(cst[u], ccn[u]);
              clb[pos] = lbc[u];
            }
            ncl += (int)__popcll(m);
          }
          if (ncl > kBfsCellCap - 256) flush_cells();
        }
        nsl = 0;
      };
      // 2-3. blocks (zig-zag from the home block), then the super-cells of passing blocks
      const int nblk = (nsup + 63) >> 6, hb = hs >> 6;
      for (int gb = 0; gb < nblk; gb += 64) {
        const int bidx = zigzag(hb, gb + lane, nblk);
        const float lbb = bidx >= 0 ? box_lb32<UW>(bbox + 16 * (size_t)bidx, s32, w32, gap) : INFINITY;
        tests += (unsigned long long)min(64, nblk - gb);
        uint64_t bmask = __ballot(lbb <= thr);
        while (bmask) {
          int blk[4];
          float lbs[4];
          int sc0[4], scn[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            blk[u] = -1;
            lbs[u] = INFINITY;
            sc0[u] = 0;
            scn[u] = 0;
            if (bmask) {
              const int ib = __builtin_ctzll(bmask);
              bmask &= bmask - 1;
              blk[u] = __builtin_amdgcn_readlane(bidx, ib);
              const int rot = blk[u] == hb ? (hs & 63) : 0;
              const int sidx = 64 * blk[u] + ((lane + rot) & 63);
              if (sidx < nsup)
                lbs[u] = box_lb32<UW>(sbox + 16 * (size_t)sidx, s32, w32, gap, &sc0[u], &scn[u]);
              tests += (unsigned long long)min(64, nsup - 64 * blk[u]);
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool p = lbs[u] <= thr;
            const uint64_t m = __ballot(p);
            if (p) sup[nsl + (int)__popcll(m & lt_mask)] = make_int2(sc0[u], scn[u]);
            nsl += (int)__popcll(m);
          }
          if (nsl > kBfsSupCap - 256) flush_supers();
        }
      }
      flush_supers();
      flush_cells();
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
        nn[lj] = wi == INT_MAX ? 0 : wi;
        if (second) second[lj] = sec;
        if (score) score[lj] = m;
      }
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
  if (lane == 0) {
    atomicAdd(&st->nn_pairs, pairs);
    atomicAdd(&st->nn_box_tests, tests);
  }
}
