// tcmp_mesh.h -- exact link-hull vs convex-mesh penetration depth (gfx950, wave-cooperative).
//
// Reference semantics: utils.py:2833-2880 -- Bullet closest points between the link's convex
// hull and an obstacle's convex hull with distance = -MAX_DISTANCE; a pair collides iff the
// penetration depth is >= 0.04 m (kPen).  Bullet is absent (parity unpinned against it); the
// CPU oracle (oracle/tcmp_oracle.c orc_hull_mesh_pd_*) restates the same depth.
//
// Penetration depth of two convex polytopes = min over the facets of their Minkowski
// difference A - B of the support h_{A-B}(n).  Those facets come from (1) facets of B,
// (2) facets of A and (3) edge pairs (eA, eB) whose Gauss-map arcs intersect
// (Gregorius' Minkowski-face test).  For an edge pair the support is exact from the edge
// points themselves: n.(a0 - b0) with n = eA x eB oriented into A's normal cone.
// Everything is evaluated in the world frame: the obstacle's hull data is stored there
// (tcmp_set_meshes), the link's is rotated per lane.
//
// fp32 first pass (LDS link geometry, scalar-loaded mesh data) -> result, or NaN when an
// axis is too close to degenerate for fp32 (nearly parallel edges, ambiguous orientation);
// the caller re-evaluates in fp64 whenever the fp32 value is within kExactGuard of kPen or
// NaN, so the collision decision is always the fp64 one.  A borderline Gauss-map sign in
// fp32 can only add or drop an axis whose edge-formula value is within (angle error) x
// (hull diameter) ~ 1e-6 m of a neighbouring exact facet axis, far inside kExactGuard.
#pragma once

namespace tcmp {

#ifdef TCMP_PROF_EXACT
#define TCMP_MSTAT(i) if (lane_id() == 0) atomicAdd(&g_exact_stats[i], 1ull)
// the full fp32 hull-vs-hull stage's clocks: [0] pairs it proves free, [1] / [2] the facet / edge
// parts of the pairs that run to the end
__device__ unsigned long long g_full_clk[4];
#define TCMP_FCLK(i, t) if (STAT && lane_id() == 0) atomicAdd(&g_full_clk[i], clock64() - (t))
#else
#define TCMP_MSTAT(i)
#define TCMP_FCLK(i, t)
#endif

// A hull in a link frame (rotated per lane into the world): vertices [V][3], planes (n, d),
// edges (va, vb, f1, f2) as rows of those arrays; [x0, x1) ranges of this hull.
struct HullA32 {
  const float* v3;
  const float4* pl;
  const ushort4* ei;
  const float4* ev;  // [E]: vb - va (rounded from fp64)
  int v0, v1, f0, f1, e0, e1;
};
// A world-frame obstacle hull: vertices, planes, Gauss-map edge records [E][16]
// (c = -n1, d = -n2, unit(d x c), edge vector, endpoint), sorted by the direction of their
// arcs and cut into at most 32 clusters [c0, c1) of consecutive records, each with a cone on
// the Gauss sphere holding all its arcs (gauss_clusters, tcmp_engine.hip): two float4 per
// cluster, (axis, cos half-angle), (sin half-angle, first record, end record, 0) with the
// record indices as int bits.
struct HullB32 {
  const float4* v;
  const float4* pl;
  const float* er;
  int v0, v1, f0, f1, e0, e1;
  const float4* cl;
  int c0, c1;
};
#ifndef TCMP_GAUSS_CL
#define TCMP_GAUSS_CL 128  // Gauss-map clusters per hull at most (<= 128: two mask words)
#endif
constexpr int kMaxGaussClusters = TCMP_GAUSS_CL;
constexpr int kClWords = (kMaxGaussClusters + 63) / 64;  // 64-bit candidate mask words per lane
static_assert(kClWords <= 4, "cluster masks: at most four 64-bit words");
#ifndef TCMP_REC_UNROLL
#define TCMP_REC_UNROLL 2  // Gauss records loaded together in the hull-vs-hull edge walk
#endif
// slack on the cone test's cosine: far above the fp32 error of the rotated axes (~1e-6), so a
// pair of arcs that intersect is never pruned
constexpr float kConeSlack = 2e-3f;

// Wave-uniform streams of read-only hull data go through the constant address space, so they
// become scalar loads (s_load_dwordx4 / _dwordx16 into SGPRs, the scalar cache) instead of
// vector loads of one address by every lane.
typedef const __attribute__((address_space(4))) float cfloat;

// Facet passes: lanes own 64*J facets, the other hull's vertices stream wave-uniformly;
// returns this lane's minimum of (facet offset - support), INFINITY for empty slots.
// BF: B's facets (moved into A's frame) against A's vertices; else A's facets (moved into
// the world frame) against B's vertices.
template <int J, bool BF>
__device__ __forceinline__ float facet_pass32(const HullA32& A, const HullB32& B, const float R[9],
                                              const float p[3], int base) {
  const int lane = lane_id();
  const int f1 = BF ? B.f1 : A.f1;
  float nx[J], ny[J], nz[J], dd[J], mn[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int f = base + lane + 64 * j;
    float4 w = make_float4(0.f, 0.f, 0.f, INFINITY);
    if (f < f1) w = BF ? B.pl[f] : A.pl[f];
    if (BF) {
      nx[j] = R[0] * w.x + R[3] * w.y + R[6] * w.z;
      ny[j] = R[1] * w.x + R[4] * w.y + R[7] * w.z;
      nz[j] = R[2] * w.x + R[5] * w.y + R[8] * w.z;
      dd[j] = w.w - (w.x * p[0] + w.y * p[1] + w.z * p[2]);
    } else {
      nx[j] = R[0] * w.x + R[1] * w.y + R[2] * w.z;
      ny[j] = R[3] * w.x + R[4] * w.y + R[5] * w.z;
      nz[j] = R[6] * w.x + R[7] * w.y + R[8] * w.z;
      dd[j] = w.w + (nx[j] * p[0] + ny[j] * p[1] + nz[j] * p[2]);
    }
    mn[j] = INFINITY;
  }
  // the vertex streams are wave-uniform loads: unrolled so that four are in flight per wait
  if (BF) {
    cfloat* v3 = (cfloat*)A.v3;
#pragma unroll 4
    for (int v = A.v0; v < A.v1; ++v) {
      const float x = v3[3 * v], y = v3[3 * v + 1], z = v3[3 * v + 2];
#pragma unroll
      for (int j = 0; j < J; ++j) mn[j] = fminf(mn[j], nx[j] * x + ny[j] * y + nz[j] * z);
    }
  } else {
    cfloat* bv = (cfloat*)B.v;
#pragma unroll 4
    for (int v = B.v0; v < B.v1; ++v) {
      const float4 P4 = make_float4(bv[4 * v], bv[4 * v + 1], bv[4 * v + 2], 0.f);
#pragma unroll
      for (int j = 0; j < J; ++j) mn[j] = fminf(mn[j], nx[j] * P4.x + ny[j] * P4.y + nz[j] * P4.z);
    }
  }
  float loc = INFINITY;
#pragma unroll
  for (int j = 0; j < J; ++j) loc = fminf(loc, dd[j] - mn[j]);
  return loc;
}

// All facets of one hull in passes of 256 / 128 / 64 (so a hull of <= 64 facets costs one
// vertex stream with one facet per lane).
template <bool BF>
__device__ __forceinline__ float facets32(const HullA32& A, const HullB32& B, const float R[9],
                                          const float p[3]) {
  const int f0 = BF ? B.f0 : A.f0, f1 = BF ? B.f1 : A.f1;
  float loc = INFINITY;
  for (int base = f0; base < f1;) {
    const int rem = f1 - base;
    if (rem > 128) {
      loc = fminf(loc, facet_pass32<4, BF>(A, B, R, p, base));
      base += 256;
    } else if (rem > 64) {
      loc = fminf(loc, facet_pass32<2, BF>(A, B, R, p, base));
      base += 128;
    } else {
      loc = fminf(loc, facet_pass32<1, BF>(A, B, R, p, base));
      base += 64;
    }
  }
  return loc;
}

// fp32 penetration depth of hull A (pose R, p) against hull B, wave-cooperative.  Returns as
// soon as a stage's minimum falls below `stop` (then the value is only an upper bound below
// `stop`), NaN when an edge axis is too degenerate for fp32 (see the header comment).
template <bool STAT>
__device__ __forceinline__ float hull_hull_wave32(const HullA32 A, const HullB32 B,
                                                  const float R[9], const float p[3], float stop) {
  const int lane = lane_id();
#ifdef TCMP_PROF_EXACT
  const unsigned long long tf0 = clock64();
#endif
  // (1) B's facets (moved into A's frame) against A's vertices (uniform stream)
  float pd = wave_minf(facets32<true>(A, B, R, p));
  if (pd < stop) { if (STAT) TCMP_MSTAT(8); TCMP_FCLK(0, tf0); return pd; }
  // (2) A's facets (moved into the world frame) against B's vertices
  pd = fminf(pd, wave_minf(facets32<false>(A, B, R, p)));
  if (pd < stop) { if (STAT) TCMP_MSTAT(9); TCMP_FCLK(0, tf0); return pd; }
#ifdef TCMP_PROF_EXACT
  const unsigned long long te0 = clock64();
#endif
  float loc = INFINITY;
  // (3) edge pairs whose Gauss-map arcs intersect (Gregorius' Minkowski-face test).  Lanes own
  // A's edges, 64 at a time.  Pass 1: each lane's arc a -> b (A's facet normals in the world) is
  // held by the cone (unit(a + b), half the a-b angle); a cluster of B's arcs can hold an arc that
  // intersects it only if the two cones overlap, angle(axes) <= sum of half-angles -- one bit per
  // cluster.  Pass 2: the (edge, cluster) candidates in rank order, one per lane (a wave prefix
  // sum of the per-lane counts and a six-step binary search over the lanes, as exact_pd_wave32's
  // edge pass): the lane rebuilds the edge and walks the cluster's records.  The axes evaluated
  // are the unpruned loop's (the cones are conservative by kConeSlack), so the minimum is too.
  bool deg = false;
  const int nC = B.c1 - B.c0;
  for (int base = A.e0; base < A.e1; base += 64) {
    // this lane's edge of A in the world: adjacent facet normals a, b, unit(b x a), edge
    // vector, endpoint
    auto a_edge = [&](int e, float& ax, float& ay, float& az, float& bx, float& by, float& bz,
                      float& ux, float& uy, float& uz, float& ex, float& ey, float& ez,
                      float& px, float& py, float& pz) {
      const ushort4 ix = A.ei[e];
      const float4 na = A.pl[ix.z], nb = A.pl[ix.w];
      ax = R[0] * na.x + R[1] * na.y + R[2] * na.z;
      ay = R[3] * na.x + R[4] * na.y + R[5] * na.z;
      az = R[6] * na.x + R[7] * na.y + R[8] * na.z;
      bx = R[0] * nb.x + R[1] * nb.y + R[2] * nb.z;
      by = R[3] * nb.x + R[4] * nb.y + R[5] * nb.z;
      bz = R[6] * nb.x + R[7] * nb.y + R[8] * nb.z;
      ux = by * az - bz * ay;
      uy = bz * ax - bx * az;
      uz = bx * ay - by * ax;
      const float il = rsqrtf(ux * ux + uy * uy + uz * uz);
      ux *= il; uy *= il; uz *= il;
      const float x0 = A.v3[3 * ix.x], y0 = A.v3[3 * ix.x + 1], z0 = A.v3[3 * ix.x + 2];
      const float4 ed = A.ev[e];
      ex = R[0] * ed.x + R[1] * ed.y + R[2] * ed.z;
      ey = R[3] * ed.x + R[4] * ed.y + R[5] * ed.z;
      ez = R[6] * ed.x + R[7] * ed.y + R[8] * ed.z;
      px = R[0] * x0 + R[1] * y0 + R[2] * z0 + p[0];
      py = R[3] * x0 + R[4] * y0 + R[5] * z0 + p[1];
      pz = R[6] * x0 + R[7] * y0 + R[8] * z0 + p[2];
    };
    // pass 1: bit k of cm[k / 64] = cluster c0 + k may hold an arc crossing this lane's
    unsigned long long cm[kClWords];
#pragma unroll
    for (int w = 0; w < kClWords; ++w) cm[w] = 0;
    {
      const int e = base + lane;
      if (e < A.e1) {
        const ushort4 ix = A.ei[e];
        const float4 na = A.pl[ix.z], nb = A.pl[ix.w];
        // the arc's cone in A's frame, its axis rotated into the world
        const float sx = na.x + nb.x, sy = na.y + nb.y, sz = na.z + nb.z;
        const float s2 = sx * sx + sy * sy + sz * sz;
        if (!(s2 > 1e-6f)) {
          // a knife edge: no cone, every cluster
#pragma unroll
          for (int w = 0; w < kClWords; ++w) {
            const int r = nC - 64 * w;
            cm[w] = r >= 64 ? ~0ull : r > 0 ? ((1ull << r) - 1) : 0ull;
          }
        } else {
          const float is = rsqrtf(s2);
          const float qx = (R[0] * sx + R[1] * sy + R[2] * sz) * is;
          const float qy = (R[3] * sx + R[4] * sy + R[5] * sz) * is;
          const float qz = (R[6] * sx + R[7] * sy + R[8] * sz) * is;
          const float cab = na.x * nb.x + na.y * nb.y + na.z * nb.z;
          const float ca = sqrtf(fmaxf(0.f, 0.5f * (1.f + cab))),
                      sa = sqrtf(fmaxf(0.f, 0.5f * (1.f - cab)));
          // the cluster cones are wave-uniform: scalar loads through the constant address space
          // (vector loads of one address by every lane were 3 % slower on C5, profiles/r9q_*)
          cfloat* cl = (cfloat*)(B.cl + 2 * B.c0);
#pragma unroll
          for (int w = 0; w < kClWords; ++w) {
            unsigned long long bits = 0;
            for (int k = 64 * w; k < min(nC, 64 * w + 64); ++k) {
              const float4 c = make_float4(cl[8 * k], cl[8 * k + 1], cl[8 * k + 2], cl[8 * k + 3]);
              const float4 s = make_float4(cl[8 * k + 4], 0.f, 0.f, 0.f);
              // the cones overlap iff angle(axes) <= half_a + half_b: always when that sum
              // reaches pi (half_b >= pi - half_a, i.e. cos half_b <= -cos half_a; half_a <=
              // pi / 2), else cos(angle) >= cos(half_a + half_b), less the slack
              if (c.w <= -ca + kConeSlack ||
                  qx * c.x + qy * c.y + qz * c.z >= ca * c.w - sa * s.x - kConeSlack)
                bits |= 1ull << (k - 64 * w);
            }
            cm[w] = bits;
          }
        }
      }
    }
    int cnt = 0;
#pragma unroll
    for (int w = 0; w < kClWords; ++w) cnt += __popcll(cm[w]);
    int pre = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(pre, o);
      if (lane >= o) pre += t;
    }
    const int total = __shfl(pre, 63);
    pre -= cnt;  // lane l's candidates are ranks [pre, pre + cnt)
    for (int w0 = 0; w0 < total; w0 += 64) {
      const int w = w0 + lane;
      int src = 0;  // the last lane whose prefix is <= w
#pragma unroll
      for (int step = 32; step; step >>= 1)
        if (__shfl(pre, src + step) <= w) src += step;
      unsigned long long mw[kClWords];
#pragma unroll
      for (int x = 0; x < kClWords; ++x) mw[x] = (unsigned long long)__shfl((long long)cm[x], src);
      int kk = w - __shfl(pre, src);
      if (w < total) {
        // the kk-th candidate of lane src: its word, then its bit
        unsigned long long m = mw[0];
        int cbase = 0;
        bool found = false;
#pragma unroll
        for (int x = 0; x < kClWords; ++x) {
          const int n = __popcll(mw[x]);
          if (!found) {
            if (kk < n) { m = mw[x]; cbase = 64 * x; found = true; }
            else kk -= n;
          }
        }
        for (int j = 0; j < kk; ++j) m &= m - 1;
        const float4 cs = B.cl[2 * (B.c0 + cbase + __builtin_ctzll(m)) + 1];
        const int r0 = __float_as_int(cs.y), r1 = __float_as_int(cs.z);
        float ax, ay, az, bx, by, bz, ux, uy, uz, ex, ey, ez, px, py, pz;
        a_edge(base + src, ax, ay, az, bx, by, bz, ux, uy, uz, ex, ey, ez, px, py, pz);
        const float el2 = ex * ex + ey * ey + ez * ez;
        // one record: its arc (c -> d) against the lane's edge (Gregorius' test), the axis if
        // they intersect; r0v / r1v: the record's first 32 bytes, loaded by the caller
        auto rec = [&](int k, const float4 r0v, const float4 r1v) {
          const float4* E4 = reinterpret_cast<const float4*>(B.er + 16 * k);
          const float cba = r0v.x * ux + r0v.y * uy + r0v.z * uz;
          const float dba = r0v.w * ux + r1v.x * uy + r1v.y * uz;
          if (cba * dba < 0.f) {
            const float4 r2v = E4[2], r3v = E4[3];  // w z | edge vector | endpoint x, endpoint y z
            const float wx = r1v.z, wy = r1v.w, wz = r2v.x;
            const float adc = ax * wx + ay * wy + az * wz;
            const float bdc = bx * wx + by * wy + bz * wz;
            if (adc * bdc < 0.f && cba * bdc > 0.f) {
              const float fx = r2v.y, fy = r2v.z, fz = r2v.w;
              float n0 = ey * fz - ez * fy, n1 = ez * fx - ex * fz, n2 = ex * fy - ey * fx;
              const float len2 = n0 * n0 + n1 * n1 + n2 * n2;
              const float fl2 = fx * fx + fy * fy + fz * fz;
              if (!(len2 > 1e-4f * el2 * fl2)) {
                deg = true;  // nearly parallel (or degenerate) edges: the axis needs fp64
              } else {
                const float il = rsqrtf(len2);
                const float ori = n0 * (ax + bx) + n1 * (ay + by) + n2 * (az + bz);
                deg |= fabsf(ori) * il < 1e-4f;
                if (ori < 0.f) { n0 = -n0; n1 = -n1; n2 = -n2; }
                const float ov = n0 * (px - r3v.x) + n1 * (py - r3v.y) + n2 * (pz - r3v.z);
                loc = fminf(loc, ov * il);
              }
            }
          }
        };
        // the cluster's records TCMP_REC_UNROLL at a time, their first halves all in flight
        // before the first test (a record's walk is otherwise one dependent gather at a time)
        int k = r0;
#pragma unroll 1
        for (; k + TCMP_REC_UNROLL <= r1; k += TCMP_REC_UNROLL) {
          float4 h0[TCMP_REC_UNROLL], h1[TCMP_REC_UNROLL];
#pragma unroll
          for (int u = 0; u < TCMP_REC_UNROLL; ++u) {
            const float4* E4 = reinterpret_cast<const float4*>(B.er + 16 * (k + u));
            h0[u] = E4[0];
            h1[u] = E4[1];
          }
#pragma unroll
          for (int u = 0; u < TCMP_REC_UNROLL; ++u) rec(k + u, h0[u], h1[u]);
        }
#pragma unroll 1
        for (; k < r1; ++k) {
          const float4* E4 = reinterpret_cast<const float4*>(B.er + 16 * k);
          rec(k, E4[0], E4[1]);
        }
      }
      if ((w0 + 64 < total || base + 64 < A.e1) && !__ballot(deg)) {
        const float lf = fminf(pd, wave_minf(loc));
        if (lf < stop) { if (STAT) TCMP_MSTAT(10); TCMP_FCLK(0, tf0); return lf; }
      }
    }
  }
  TCMP_FCLK(1, tf0 + (clock64() - te0));  // the facet part: te0 - tf0
  TCMP_FCLK(2, te0);
  if (__ballot(deg)) { if (STAT) TCMP_MSTAT(13); return __builtin_nanf(""); }
  const float res = fminf(pd, wave_minf(loc));
  if (STAT) {
    if (res >= (float)kPen) { TCMP_MSTAT(11); } else { TCMP_MSTAT(12); }
  }
  return res;
}

// fp64 restatement of hull_hull_wave32 on the full hulls (same axes, strict Gauss-map test, no degeneracy
// shortcuts): the decision-maker near kPen.  Every lane of the wave calls it.
// pose: R[9], p[3] in the wave's LDS pose slot; pointers one by one (no argument in scratch)
// The edge pairs are pruned by the mesh's Gauss-map clusters exactly as in hull_hull_wave32
// (a cluster whose cone cannot meet the lane's arc holds no intersecting arc; the cones are
// conservative by kConeSlack), so the minimum is the unpruned one.
__device__ __noinline__ double exact_mesh_wave(int link, const double* pose, int m,
                                               const int* __restrict__ mrange,
                                               const double4* __restrict__ mp64,
                                               const double4* __restrict__ mv64,
                                               const double* __restrict__ me64,
                                               const float4* __restrict__ mcl,
                                               const double* __restrict__ gverts,
                                               const double* __restrict__ gplanes,
                                               const double* __restrict__ gedges) {
  const int lane = lane_id();
  const struct { const double* verts; const double* planes; const double* edges; } g = {
      gverts, gplanes, gedges};
  const struct { const double4* mp64; const double4* mv64; const double* me64; } sc = {mp64, mv64,
                                                                                         me64};
  const int* rg = mrange + kMrange * m;
  const int v0 = rg[0], v1 = rg[1], f0 = rg[2], f1 = rg[3], e0 = rg[4], e1 = rg[5];
  const int lv0 = tcmp_geo_vert_off[link], lv1 = tcmp_geo_vert_off[link + 1];
  const int lf0 = tcmp_geo_plane_off[link], lf1 = tcmp_geo_plane_off[link + 1];
  const int le0 = tcmp_geo_edge_off[link], le1 = tcmp_geo_edge_off[link + 1];
  const double* R = pose;
  const double* p = pose + 9;
  double loc = INFINITY;
  for (int f = f0 + lane; f < f1; f += 64) {
    const double4 w = sc.mp64[f];
    const double nx = R[0] * w.x + R[3] * w.y + R[6] * w.z;
    const double ny = R[1] * w.x + R[4] * w.y + R[7] * w.z;
    const double nz = R[2] * w.x + R[5] * w.y + R[8] * w.z;
    const double dd = w.w - (w.x * p[0] + w.y * p[1] + w.z * p[2]);
    double mn = INFINITY;
    typedef const __attribute__((address_space(4))) double cdouble;
    cdouble* gv = (cdouble*)g.verts;  // wave-uniform stream: scalar loads
    for (int v = lv0; v < lv1; ++v)
      mn = fmin(mn, nx * gv[4 * v] + ny * gv[4 * v + 1] + nz * gv[4 * v + 2]);
    loc = fmin(loc, dd - mn);
  }
  double pd = wave_min(loc);
  if (pd < kPen) return pd;
  for (int f = lf0 + lane; f < lf1; f += 64) {
    const double* W = g.planes + 8 * f;
    const double nx = R[0] * W[0] + R[1] * W[1] + R[2] * W[2];
    const double ny = R[3] * W[0] + R[4] * W[1] + R[5] * W[2];
    const double nz = R[6] * W[0] + R[7] * W[1] + R[8] * W[2];
    const double dd = W[3] + (nx * p[0] + ny * p[1] + nz * p[2]);
    double mn = INFINITY;
    typedef const __attribute__((address_space(4))) double cdouble;
    cdouble* mv = (cdouble*)sc.mv64;  // wave-uniform stream: scalar loads
    for (int v = v0; v < v1; ++v)
      mn = fmin(mn, nx * mv[4 * v] + ny * mv[4 * v + 1] + nz * mv[4 * v + 2]);
    loc = fmin(loc, dd - mn);
  }
  pd = fmin(pd, wave_min(loc));
  if (pd < kPen) return pd;
  for (int e = le0 + lane; e < le1; e += 64) {
    const double* L = g.edges + 16 * e;  // e | va | n1 | n2 (link frame)
    const double ax = R[0] * L[8] + R[1] * L[9] + R[2] * L[10];
    const double ay = R[3] * L[8] + R[4] * L[9] + R[5] * L[10];
    const double az = R[6] * L[8] + R[7] * L[9] + R[8] * L[10];
    const double bx = R[0] * L[12] + R[1] * L[13] + R[2] * L[14];
    const double by = R[3] * L[12] + R[4] * L[13] + R[5] * L[14];
    const double bz = R[6] * L[12] + R[7] * L[13] + R[8] * L[14];
    const double ux = by * az - bz * ay, uy = bz * ax - bx * az, uz = bx * ay - by * ax;
    const double ex = R[0] * L[0] + R[1] * L[1] + R[2] * L[2];
    const double ey = R[3] * L[0] + R[4] * L[1] + R[5] * L[2];
    const double ez = R[6] * L[0] + R[7] * L[1] + R[8] * L[2];
    const double px = R[0] * L[4] + R[1] * L[5] + R[2] * L[6] + p[0];
    const double py = R[3] * L[4] + R[4] * L[5] + R[5] * L[6] + p[1];
    const double pz = R[6] * L[4] + R[7] * L[5] + R[8] * L[6] + p[2];
    // the lane's arc a -> b in its cone (unit(a + b), half the a-b angle), fp32
    const double sx = ax + bx, sy = ay + by, sz = az + bz;
    const double s2 = sx * sx + sy * sy + sz * sz;
    const bool knife = !(s2 > 1e-6);  // antipodal normals: no cone, every cluster
    const float is = knife ? 0.f : (float)(1.0 / sqrt(s2));
    const float qx = (float)sx * is, qy = (float)sy * is, qz = (float)sz * is;
    const double cab = ax * bx + ay * by + az * bz;
    const float ca = (float)sqrt(fmax(0.0, 0.5 * (1.0 + cab))), sa = (float)sqrt(fmax(0.0, 0.5 * (1.0 - cab)));
    for (int c = rg[20]; c < rg[21]; ++c) {
      const float4 cw = mcl[2 * c], cs = mcl[2 * c + 1];
      if (!knife && !(cw.w <= -ca + kConeSlack ||
                      qx * cw.x + qy * cw.y + qz * cw.z >= ca * cw.w - sa * cs.x - kConeSlack))
        continue;
      const int k1 = __float_as_int(cs.z);
      for (int k = __float_as_int(cs.y); k < k1; ++k) {
        const double* E = sc.me64 + 16 * k;
        const double cba = E[0] * ux + E[1] * uy + E[2] * uz;
        const double dba = E[3] * ux + E[4] * uy + E[5] * uz;
        if (!(cba * dba < 0)) continue;
        const double adc = ax * E[6] + ay * E[7] + az * E[8];
        const double bdc = bx * E[6] + by * E[7] + bz * E[8];
        if (!(adc * bdc < 0 && cba * bdc > 0)) continue;
        double n0 = ey * E[11] - ez * E[10], n1 = ez * E[9] - ex * E[11], n2 = ex * E[10] - ey * E[9];
        const double len2 = n0 * n0 + n1 * n1 + n2 * n2;
        if (len2 < 1e-24) continue;
        if (n0 * (ax + bx) + n1 * (ay + by) + n2 * (az + bz) < 0) { n0 = -n0; n1 = -n1; n2 = -n2; }
        loc = fmin(loc, (n0 * (px - E[12]) + n1 * (py - E[13]) + n2 * (pz - E[14])) / sqrt(len2));
      }
    }
  }
  return fmin(pd, wave_min(loc));
}

}  // namespace tcmp
