// tcmp_nn.h -- the per-round spatial index of the tree snapshot for the exact nearest-neighbour
// scan (rrt_star.py:9-14,171).  Included by tcmp_engine.hip after its state types; the scan
// itself is k_nearest_wave32 (tcmp_nn32.h).
//
// Build, once per round:
//   1. k_node_keys + radix sort: Morton keys of the snapshot nodes (9 bits per joint
//      interleaved, the top kKeyBits = 36 kept; rocPRIM Onesweep radix sort).
//   2. k_nn_rows: in key order, stree [T][8] f64 (q0..q6, original index) and the rows the
//      scan's first pass reads, srow: [T][8] f32 (q0..q6, 0).
//   3. k_nn_cut<kNnC>: the implicit binary radix tree of the sorted keys (Karras 2012: every
//      internal node's key range from its neighbours' common-prefix lengths) cut into
//      "cells": the largest radix-tree subtrees holding at most kNnC nodes.  A cell is a
//      contiguous key range that is also an axis-aligned Morton cell, so its bounding box is
//      compact -- unlike fixed 64-node runs, which straddle cell boundaries and stretch over
//      half the joint range.  Each cell start is flagged; an inclusive scan numbers the cells.
//   4. k_nn_starts / k_nn_cell_boxes: per cell its start, node count and f32 bounding box
//      (lo rounded down, hi rounded up): cbox [C][16] = lo0..6, start, hi0..6, count.
//   5. k_nn_cut<kNnS> over the cells' first keys: super-cells = radix-tree subtrees of <= 64
//      cells (compact too); k_nn_build_supers: their f32 bounds, first cell and cell count.
//   6. candidates: Morton keys, sorted; k_nn_home finds each candidate's home cell.
#pragma once

constexpr int kNnC = 64;              // max nodes per cell (one per lane)
constexpr int kNnS = 64;              // cells per super-cell

// (16-bit first-pass rows, round 3: 3.4x less HBM fetch but a slower scan -- DESIGN.md
// section 4; dropped.)

__global__ __launch_bounds__(256) void k_nn_rows(DevState* st, const PlanParams* __restrict__ Pd,
                                                 const double* cfg, const int* svals,
                                                 double* stree, float* srow, long long T_bound,
                                                 int* cflag, int* sflag) {
  const long long T = st->n_nodes;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= T_bound) return;
  // the cut kernels only set flags: clear both flag arrays here (no memset launches)
  cflag[p] = 0;
  sflag[p] = 0;
  if (p >= T) return;
  double q[7];
  const int n = svals[p];
  load7(cfg + 8 * (size_t)n, q);
  store7(stree + 8 * p, q);
  stree[8 * p + 7] = (double)n;
  float4* d32 = reinterpret_cast<float4*>(srow + 8 * p);
  d32[0] = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
  d32[1] = make_float4((float)q[4], (float)q[5], (float)q[6], 0.f);
}

// common-prefix length of keys i and j (ties broken by the index), -1 outside [0, T)
__device__ __forceinline__ int nn_delta(const unsigned long long* k, long long T, long long i,
                                        long long j) {
  if (j < 0 || j >= T) return -1;
  const unsigned long long a = k[i], b = k[j];
  if (a == b) return 64 + __clzll((unsigned long long)(i ^ j));
  return __clzll(a ^ b);
}

// internal node i of the radix tree over keys[0, T): its range and split (Karras 2012, §4);
// flags the start of every child range of <= cap keys whose parent holds more.  Used twice:
// over the node keys (cells of <= kNnC nodes) and over the cells' first keys (super-cells of
// <= kNnS cells).  *count is the device-side number of keys.
template <int cap>
__global__ __launch_bounds__(256) void k_nn_cut(const long long* count_ll, const int* count_i,
                                                const unsigned long long* keys, int* flag) {
  const long long T = count_ll ? *count_ll : (long long)*count_i;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i == 0) flag[0] = 1;
  if (i >= T - 1) return;
  const int d = nn_delta(keys, T, i, i + 1) - nn_delta(keys, T, i, i - 1) > 0 ? 1 : -1;
  const int dmin = nn_delta(keys, T, i, i - d);
  long long lmax = 2;
  while (nn_delta(keys, T, i, i + lmax * d) > dmin) lmax <<= 1;
  long long l = 0;
  for (long long t = lmax >> 1; t >= 1; t >>= 1)
    if (nn_delta(keys, T, i, i + (l + t) * d) > dmin) l += t;
  const long long j = i + l * d;
  const int dnode = nn_delta(keys, T, i, j);
  long long s = 0;
  for (long long t = (l + 1) >> 1;; t = (t + 1) >> 1) {
    if (nn_delta(keys, T, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const long long g = i + s * d + min(d, 0);
  const long long a = min(i, j), b = max(i, j);
  if (b - a + 1 <= cap) return;           // not a parent of a cut subtree
  if (g - a + 1 <= cap) flag[a] = 1;      // left child is cut
  if (b - g <= cap) flag[g + 1] = 1;      // right child is cut
}

// cid = inclusive scan of flag: group of position p is cid[p] - 1; writes the group starts
// and the group count
__global__ __launch_bounds__(256) void k_nn_starts(const long long* count_ll, const int* count_i,
                                                   const int* flag, const int* cid, int* cstart,
                                                   int* groups) {
  const long long T = count_ll ? *count_ll : (long long)*count_i;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= T) return;
  if (flag[p]) cstart[cid[p] - 1] = (int)p;
  if (p == T - 1) {
    cstart[cid[p]] = (int)T;
    *groups = cid[p];
  }
}

// one wave per cell: bounds of its rows; also the cell's first key (for the super-cell cut)
__global__ __launch_bounds__(256) void k_nn_cell_boxes(DevState* st, const double* stree,
                                                       const int* cstart,
                                                       const unsigned long long* skeys,
                                                       float* cbox, unsigned long long* ckey) {
  const int C = st->nn_cells;
  // grid-stride over cells, one wave per cell (the count is device-side)
  for (long long c = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6; c < C;
       c += ((long long)gridDim.x * 256) >> 6) {
  const int a = cstart[c], b = cstart[c + 1];
  const long long p = a + lane_id();
  double lo[7], hi[7];
  if (p < b) {
    double q[7];
    load7(stree + 8 * p, q);
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
  if (lane_id() == 0) {
    float* bx = cbox + 16 * c;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      bx[k] = __double2float_rd(lo[k]);
      bx[8 + k] = __double2float_ru(hi[k]);
    }
    bx[7] = __int_as_float(a);
    bx[15] = __int_as_float(b - a);
    ckey[c] = skeys[a];
  }
  }
}

// one wave per super-cell (a radix-tree subtree of <= kNnS cells): union of its cells' bounds;
// sbox [S][16] = lo0..6, first cell, hi0..6, cell count
__global__ __launch_bounds__(256) void k_nn_build_supers(DevState* st, const int* sstart,
                                                         const float* cbox, float* sbox) {
  const int nsup = st->nn_supers;
  for (long long sw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; sw < nsup;
       sw += ((long long)gridDim.x * blockDim.x) >> 6) {
  const int c0 = sstart[sw], c1 = sstart[sw + 1];
  const long long c = c0 + lane_id();
  float lo[7], hi[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = c < c1 ? cbox[16 * c + k] : INFINITY;
    hi[k] = c < c1 ? cbox[16 * c + 8 + k] : -INFINITY;
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = wave_minf(lo[k]);
    hi[k] = wave_maxf(hi[k]);
  }
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      sbox[16 * sw + k] = lo[k];
      sbox[16 * sw + 8 + k] = hi[k];
    }
    sbox[16 * sw + 7] = __int_as_float(c0);
    sbox[16 * sw + 15] = __int_as_float(c1 - c0);
  }
  }
}

// blocks of 64 consecutive super-cells (Morton order): their f32 bounds, one wave per block,
// so the scan skips a whole block of super-cell boxes with one box test
__global__ __launch_bounds__(256) void k_nn_build_blocks(DevState* st, const float* sbox,
                                                         float* bbox) {
  const int nsup = st->nn_supers;
  for (long long b = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; b * 64 < nsup;
       b += ((long long)gridDim.x * blockDim.x) >> 6) {
  const long long sp = b * 64 + lane_id();
  float lo[7], hi[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = sp < nsup ? sbox[16 * sp + k] : INFINITY;
    hi[k] = sp < nsup ? sbox[16 * sp + 8 + k] : -INFINITY;
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    lo[k] = wave_minf(lo[k]);
    hi[k] = wave_maxf(hi[k]);
  }
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      bbox[16 * b + k] = lo[k];
      bbox[16 * b + 8 + k] = hi[k];
    }
    bbox[16 * b + 7] = 0.f;
    bbox[16 * b + 15] = 0.f;
  }
  }
}

// home cell of each Morton-ordered candidate (j-th in cperm order, its key ckeys[cperm[j]]):
// the cell holding its key's lower bound, and its super-cell: home[j] = cell, home[nb + j] =
// super-cell
__global__ void k_nn_home(DevState* st, const unsigned long long* skeys,
                          const unsigned long long* ckeys, const int* cperm, const int* cid,
                          const int* sid, int nb, int* home, int* bcount) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < 8) st->nn_queue[j] = 0;  // the scan's per-XCD queues (next launch)
  if (bcount && j < (nb + 255) / 256) bcount[j] = 0;  // k_edges' accepted-edge counts
  if (j == 0) {
    st->nn_counter = 0;
    st->work_counter = 0;          // k_edges' lane-refill counter (launched after the scan)
  }
  if (j >= nb) return;
  const long long T = st->n_nodes;
  const unsigned long long k = ckeys[cperm[j]];
  long long lo = 0, hi = T;
  while (lo < hi) {
    const long long mid = (lo + hi) >> 1;
    if (skeys[mid] < k) lo = mid + 1; else hi = mid;
  }
  const int c = cid[min(lo, T - 1)] - 1;
  home[j] = c;
  home[nb + j] = sid[c] - 1;
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
