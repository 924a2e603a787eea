// Static base link (panda_link0) against the scene: the part of the body-level check
// pairwise_collision(robot, b) (utils.py:2872-2880 -> body_collision :2866 ->
// get_closest_points(max_distance=-MAX_DISTANCE) :2833) that the moving-link collision_fn
// does not cover.  The reference runs it on the grasp configuration
// (franka_ik_fast.py:78, panda_primitives.py:260).  link0 sits at the base = world frame,
// so its depth against each obstacle does not depend on q: one workgroup per obstacle
// computes it once per call.
//
// Depth = minimum overlap over every candidate axis of the two hulls (facets of both, every
// edge-pair cross product), fp64, the brute-force definition of the oracle's
// hull_pd_brute.  A box enters as its 3 face axes, 3 edge directions and an analytic
// support (|n.a| h per axis); a mesh as its world-frame hull rows (Scene::mv64 / mp64 /
// me64).  At most 200 + 300 + 300 x E_mesh axes per obstacle: a fraction of a millisecond
// for 256 meshes -- this is a once-per-grasp check, not a hot kernel.
#pragma once

#include "panda_base.inc"

struct BaseGeo {
  const double4* v;  // [TCMP_BASE_NV] x y z 0
  const double4* n;  // [TCMP_BASE_NF] unit facet normal, dmax
  const double4* e;  // [TCMP_BASE_NE] unit edge direction, 0
};

constexpr int kBaseThreads = 256;

__global__ __launch_bounds__(kBaseThreads) void k_base_pd(Scene sc, BaseGeo bg, int n_box,
                                                          double* pd) {
  __shared__ double4 av[TCMP_BASE_NV];
  __shared__ double red[kBaseThreads];
  for (int i = threadIdx.x; i < TCMP_BASE_NV; i += kBaseThreads) av[i] = bg.v[i];
  __syncthreads();
  const int o = blockIdx.x;
  const bool box = o < n_box;
  double c[3] = {0, 0, 0}, R[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, h[3] = {0, 0, 0};
  int v0 = 0, v1 = 0, f0 = 0, f1 = 0, e0 = 0, e1 = 0;
  if (box) {
    const double* rec = sc.obs + 16 * o;
    for (int k = 0; k < 3; ++k) c[k] = rec[k];
    for (int k = 0; k < 9; ++k) R[k] = rec[3 + k];
    for (int k = 0; k < 3; ++k) h[k] = rec[12 + k];
  } else {
    const int* r = sc.mrange + kMrange * (o - n_box);
    v0 = r[0]; v1 = r[1]; f0 = r[2]; f1 = r[3]; e0 = r[4]; e1 = r[5];
  }
  const int nfb = box ? 3 : f1 - f0, neb = box ? 3 : e1 - e0;
  const int total = TCMP_BASE_NF + nfb + TCMP_BASE_NE * neb;
  double best = INFINITY;
  for (int t = threadIdx.x; t < total; t += kBaseThreads) {
    double n[3];
    if (t < TCMP_BASE_NF) {
      const double4 a = bg.n[t];
      n[0] = a.x; n[1] = a.y; n[2] = a.z;
    } else if (t < TCMP_BASE_NF + nfb) {
      const int j = t - TCMP_BASE_NF;
      if (box) {
        for (int k = 0; k < 3; ++k) n[k] = R[3 * k + j];
      } else {
        const double4 a = sc.mp64[f0 + j];
        n[0] = a.x; n[1] = a.y; n[2] = a.z;
      }
    } else {
      const int k = t - TCMP_BASE_NF - nfb;
      const int i = k / neb, j = k - (k / neb) * neb;
      const double4 ea = bg.e[i];
      double eb[3];
      if (box) {
        for (int q = 0; q < 3; ++q) eb[q] = R[3 * q + j];
      } else {
        const double* rec = sc.me64 + 16 * (e0 + j);
        for (int q = 0; q < 3; ++q) eb[q] = rec[9 + q];
      }
      const double lb = sqrt(eb[0] * eb[0] + eb[1] * eb[1] + eb[2] * eb[2]);
      for (int q = 0; q < 3; ++q) eb[q] /= lb;
      n[0] = ea.y * eb[2] - ea.z * eb[1];
      n[1] = ea.z * eb[0] - ea.x * eb[2];
      n[2] = ea.x * eb[1] - ea.y * eb[0];
      const double l2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
      if (l2 < 1e-12) continue;  // parallel edges: no axis (hull_pd_brute's rule)
      const double il = 1.0 / sqrt(l2);
      for (int q = 0; q < 3; ++q) n[q] *= il;
    }
    double amn = INFINITY, amx = -INFINITY;
    for (int i = 0; i < TCMP_BASE_NV; ++i) {
      const double d = n[0] * av[i].x + n[1] * av[i].y + n[2] * av[i].z;
      amn = fmin(amn, d);
      amx = fmax(amx, d);
    }
    double bmn, bmx;
    if (box) {
      const double cc = n[0] * c[0] + n[1] * c[1] + n[2] * c[2];
      double ext = 0;
      for (int a = 0; a < 3; ++a)
        ext += fabs(n[0] * R[a] + n[1] * R[3 + a] + n[2] * R[6 + a]) * h[a];
      bmn = cc - ext;
      bmx = cc + ext;
    } else {
      bmn = INFINITY;
      bmx = -INFINITY;
      for (int i = v0; i < v1; ++i) {
        const double4 b = sc.mv64[i];
        const double d = n[0] * b.x + n[1] * b.y + n[2] * b.z;
        bmn = fmin(bmn, d);
        bmx = fmax(bmx, d);
      }
    }
    best = fmin(best, fmin(amx - bmn, bmx - amn));
  }
  red[threadIdx.x] = best;
  __syncthreads();
  for (int s = kBaseThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) pd[o] = red[0];
}

// body-level flags: the moving links' flags (limits not tested) or any base depth >= kPen
__global__ void k_body_merge(int* collides, long long n, const double* base_pd, int n_base) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool hit = false;
  for (int j = 0; j < n_base; ++j) hit |= base_pd[j] >= kPen;
  if (hit) collides[i] = 1;
}
