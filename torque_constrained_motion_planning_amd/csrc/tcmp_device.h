// tcmp_device.h -- per-lane device math of the torque-constrained RRT* hot path (gfx950).
//
// Everything here is fp64 (the reference is numpy float64).  One wavefront lane owns one
// configuration / edge; the only cross-lane code is the wave-cooperative exact
// hull-vs-box test (exact_pd_wave), which every lane of the wave must reach together.
//
// Reference semantics restated (file:line in /root/reference/src):
//   extend/refine      utils.py:3031-3041, 3068-3077
//   distance           utils.py:3010-3017
//   limits             utils.py:3154-3163, 1150-1154
//   collision          utils.py:3165-3218, 2833-2880 (pybullet hull closest points, -0.04)
//   rne                rne.py:198-254 (spatial RNE, modified DH rne.py:46-63)
//   torque tests       panda_primitives.py:13-16, 118-153, 155-193
//   min-jerk           min_jerk_v2.py:80-222, panda_primitives.py:295-318
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TCMP_GEO_QUAL static constexpr
#include "panda_geometry.inc"
#include "panda_lod.inc"
#include "panda_spheres.inc"

namespace tcmp {

constexpr double kPen = 0.04;  // utils.py:2781 MAX_DISTANCE, used as distance=-0.04

// panda_mod.urdf joint limits / efforts
constexpr double kLo[7] = {-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973};
constexpr double kHi[7] = {2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973};
constexpr double kEffort[7] = {87.0, 87.0, 87.0, 87.0, 12.0, 12.0, 12.0};

// modified DH (rne.py:47-54): a, d, cos(alpha), sin(alpha) with libm values of +-pi/2
constexpr double kC90 = 6.123233995736766e-17;
constexpr double kDhA[8] = {0.0, 0.0, 0.0, 0.0825, -0.0825, 0.0, 0.088, 0.0};
constexpr double kDhD[8] = {0.333, 0.0, 0.316, 0.0, 0.384, 0.0, 0.0, 0.107};
constexpr double kDhCa[8] = {1.0, kC90, kC90, kC90, kC90, kC90, kC90, 1.0};
constexpr double kDhSa[8] = {0.0, -1.0, 1.0, 1.0, -1.0, 1.0, 1.0, 0.0};

// inertials rne.py:65-136 (link1..7); composite flange+hand(+payload) handled in rne()
constexpr double kMass[7] = {4.970684, 0.646926, 3.228604, 3.587895, 1.225946, 1.666555,
                             7.35522e-01};
constexpr double kCom[7][3] = {{3.875e-03, 2.081e-03, -0.1750},
                               {-3.141e-03, -2.872e-02, 3.495e-03},
                               {2.7518e-02, 3.9252e-02, -6.6502e-02},
                               {-5.317e-02, 1.04419e-01, 2.7454e-02},
                               {-1.1953e-02, 4.1065e-02, -3.8437e-02},
                               {6.0149e-02, -1.4117e-02, -1.0517e-02},
                               {1.0517e-02, -4.252e-03, 6.1597e-02}};
// ixx ixy ixz iyy iyz izz
constexpr double kInertia[7][6] = {
    {7.0337e-01, -1.3900e-04, 6.7720e-03, 7.0661e-01, 1.9169e-02, 9.1170e-03},
    {7.9620e-03, -3.9250e-03, 1.0254e-02, 2.8110e-02, 7.0400e-04, 2.5995e-02},
    {3.7242e-02, -4.7610e-03, -1.1396e-02, 3.6155e-02, -1.2805e-02, 1.0830e-02},
    {2.5853e-02, 7.7960e-03, -1.3320e-03, 1.9552e-02, 8.6410e-03, 2.8323e-02},
    {3.5549e-02, -2.1170e-03, -4.0370e-03, 2.9474e-02, 2.2900e-04, 8.6270e-03},
    {1.9640e-03, 1.0900e-04, -1.1580e-03, 4.3540e-03, 3.4100e-04, 5.4330e-03},
    {1.2516e-02, -4.2800e-04, -1.1960e-03, 1.0027e-02, -7.4100e-04, 4.8150e-03}};
constexpr double kHandMass = 0.68;         // rne.py:134
constexpr double kFlangeHandI = 0.101;     // link8 I=0.001 (rne.py:73) + hand I=0.1 (:74)
constexpr double kPayloadR = 0.165;        // new_inertia([0,0,0.14+0.025], m) (rne.py:187)
constexpr double kPayloadMin = 0.01;       // panda_primitives.py:142,178

// URDF joint origins (panda_mod.urdf joint1..7) -- pybullet link frames for collision
constexpr double kJx[7] = {0, 0, 0, 0.0825, -0.0825, 0, 0.088};
constexpr double kJy[7] = {0, 0, -0.316, 0, 0.384, 0, 0};
constexpr double kJz[7] = {0.333, 0, 0, 0, 0, 0, 0};
constexpr double kCr = 4.8965888601467475e-12;  // cos(1.57079632679)
constexpr double kJcr[7] = {1.0, kCr, kCr, kCr, kCr, kCr, kCr};
constexpr double kJsr[7] = {0.0, -1.0, 1.0, 1.0, -1.0, 1.0, 1.0};
constexpr double kFlangeZ = 0.107;
constexpr double kHandCy = 0.7071067811868645, kHandSy = -0.7071067811862305;  // rz(-0.785398163397)
constexpr double kFingerZ = 0.0584, kFingerOpen = 0.04;

// ------------------------------------------------------------------------------------------
// scene / geometry views
// ------------------------------------------------------------------------------------------
struct Geo {
  const double* __restrict__ verts;   // [V][4]
  const double* __restrict__ planes;  // [F][8] n(3) dmax wmin
  const double* __restrict__ edges;   // [E][16] e | va | n1 | n2
  // fp32 copy for the first pass of the exact test (kernels stage it in LDS)
  const float* __restrict__ verts32;    // [V][3]
  const float4* __restrict__ planes32;  // [F]: n, dmax
  const ushort4* __restrict__ eidx;     // [E]: va vb (vertex rows) f1 f2 (plane rows)
};
__host__ __device__ constexpr unsigned geo_lds_bytes() {
  return TCMP_TOTAL_PLANES * 16u + TCMP_TOTAL_VERTS * 12u + TCMP_TOTAL_EDGES * 8u;
}

// obstacle record on device: c(3) B(9 row-major, columns = axes) h(3) kind(1) -> 16.
// kind: 1 axis-aligned box, 0 oriented box, -(1 + m) convex mesh m (c, B, h = its outer box).
struct Scene {
  const double* __restrict__ obs;    // [n][16]
  int n_obs;
  const float* __restrict__ obs32;   // [n][8]: world-AABB centre(3), H - kPen + margin (3)
  unsigned* wq;                      // this wave's LDS pair queue (collides_wave), kQcap + 2
  // convex-mesh obstacles (tcmp_set_meshes), world frame, global memory
  const int* __restrict__ mrange;    // [m][32]: v0 v1 f0 f1 e0 e1 (rows of the arrays below),
                                     // the same for the inner / outer LODs [6..17], has-LOD
                                     // flag [18], spheres flag [19], Gauss-map clusters of the
                                     // full hull [20, 21) and of the LODs [22..25]
  const double* __restrict__ mib;    // [m][16]: inner box record (c, B, inner half, 0)
  const double4* __restrict__ mv64;  // [V]: x y z 0
  const float4* __restrict__ mv32;
  const double4* __restrict__ mp64;  // [F]: n (unit, outward), d = max n.v
  const float4* __restrict__ mp32;
  const double* __restrict__ me64;   // [E][16]: c = -n1, d = -n2, dxc = unit(d x c), e, v0
  const float* __restrict__ me32;    // [E][16]
  const float4* __restrict__ mcl;    // Gauss-map clusters of me32's records (HullB32::cl)
  // level-of-detail hulls of the meshes ([0] inner, [1] outer; mrange [6..17], flag [18])
  const float4* lv32[2];
  const float4* lp32[2];
  const float* le32[2];
  const float4* lcl[2];              // Gauss-map clusters of le32's records
  // the links' level-of-detail hulls (panda_lod.inc), fp32 link frames: [0] inner, [1] outer
  const float* lodv3[2];
  const float4* lodpl[2];
  const ushort4* lodei[2];
  // edge vectors vb - va of the link hulls (fp64 differences rounded to fp32: an fp32
  // difference of nearby vertices would lose the direction of short edges)
  const float4* lodev[2];
  const float4* geo_ev;
  // inscribed spheres [(10 + meshes) * TCMP_NSPH]: the links' (link frames), then each mesh's
  // (mrange flag 19), the lane-parallel certificates of phase B (sphere_cert)
  const float4* sph;
  // the certificates' link data: the link balls (sph rows [0, 10 * TCMP_NSPH)) and the fp32
  // link vertices [V][3] -- LDS copies in the mesh kernels (stage_lds), else global
  const float4* csph;
  const float* cv32;
  // self-collision pairs (tcmp_set_self_collision): the 10 link hulls are appended to the
  // mesh arrays as meshes n_mesh + j in their own link frames, and their outer-box records
  // follow the obstacles (obs rows n_obs + j, not in tier 0's obstacle loop)
  int n_mesh;
  int self_coll;
};
constexpr int kMrange = 32;  // ints per mesh in Scene::mrange
__device__ __forceinline__ int obs_mesh(const double* ob) {
  return ob[15] < 0.0 ? (int)(-ob[15]) - 1 : -1;
}
constexpr int kQcap = 128;           // queued (lane, link, obstacle) pairs per wave
// per wave: the pair queue, the wave's collision mask (u64) and a 12-double pose slot that hands
// a pair's link pose to the out-of-line fp64 exact tests (so no argument goes through scratch)
constexpr unsigned kQwaveBytes = (kQcap + 2) * 4 + 12 * 8;
__device__ __forceinline__ double* wave_pose_slot(unsigned* wq) {
  return reinterpret_cast<double*>(wq + kQcap + 2);
}

// Obstacle records and the fp32 hull geometry are staged in LDS by every kernel that runs
// collision checks (dynamic shared memory, stage_lds_bytes(n) per block): the per-(link,
// obstacle) loop then reads LDS broadcasts instead of waiting on a global load per obstacle,
// and the exact test's gathers hit LDS.  Layout: o64 [n][16] f64 | o32 [n][8] f32 |
// planes32 [F] float4 | verts32 [V][3] | eidx [E] ushort4.
constexpr int kMaxObstacles = 384;
__host__ __device__ constexpr unsigned scene_lds_bytes(int n_obs) {
  return (unsigned)(n_obs > 0 ? n_obs : 1) * (16 * sizeof(double) + 8 * sizeof(float));
}
__host__ __device__ constexpr unsigned stage_lds_bytes(int n_obs) {
  return scene_lds_bytes(n_obs) + geo_lds_bytes() + 4 * kQwaveBytes;  // 256-thread blocks
}
// Mesh scenes (up to kMaxObstacles records, hull-vs-hull exact tests) stage only the fp32
// tier-0 records and the pair queues, so that LDS does not cap residency at one 256-thread
// block per CU; the fp64 records and the hull geometry are then read through the caches.
// Behind the four pair queues, each wave of a mesh kernel parks its lanes' sin/cos (14 x 64
// doubles) and the link poses of its pending exact pairs (12 x 64 doubles) in LDS, so that
// neither stays in registers across the hull-vs-hull tests.
constexpr unsigned kStashDoubles = 26 * 64;
constexpr unsigned kCertLdsBytes = 10 * TCMP_NSPH * 16 + TCMP_TOTAL_VERTS * 12;
__host__ __device__ constexpr unsigned stage_lds_bytes_lean(int n_obs) {
  return (unsigned)(n_obs > 0 ? n_obs : 1) * (8 * sizeof(float)) + 4 * kQwaveBytes +
         4 * kStashDoubles * sizeof(double) + kCertLdsBytes;
}
__device__ __forceinline__ double* wave_stash(unsigned* wq) {
  const unsigned w = threadIdx.x >> 6;
  return reinterpret_cast<double*>(wq + (4 - w) * (kQwaveBytes / 4)) + w * kStashDoubles;
}
template <bool FULL>
__device__ __forceinline__ void stage_lds(const Scene sc, const Geo g, double* lds, Scene& so,
                                          Geo& go) {
  const int n = sc.n_obs > 0 ? sc.n_obs : 1;
  if (!FULL) {
    float* o32 = reinterpret_cast<float*>(lds);
    unsigned* wq = reinterpret_cast<unsigned*>(o32 + 8 * n) + (threadIdx.x >> 6) * (kQwaveBytes / 4);
    for (int i = threadIdx.x; i < sc.n_obs * 8; i += blockDim.x) o32[i] = sc.obs32[i];
    // behind the four queues and the four stashes: the link balls and vertices (sphere_cert)
    float4* cs = reinterpret_cast<float4*>(reinterpret_cast<unsigned char*>(o32 + 8 * n) +
                                           4 * kQwaveBytes + 4 * kStashDoubles * sizeof(double));
    float* cv = reinterpret_cast<float*>(cs + 10 * TCMP_NSPH);
    for (int i = threadIdx.x; i < 10 * TCMP_NSPH; i += blockDim.x) cs[i] = sc.sph[i];
    for (int i = threadIdx.x; i < 3 * TCMP_TOTAL_VERTS; i += blockDim.x) cv[i] = g.verts32[i];
    __syncthreads();
    so = sc;
    so.obs32 = o32;
    so.wq = wq;
    so.csph = cs;
    so.cv32 = cv;
    go = g;
    return;
  }
  double* o64 = lds;
  float* o32 = reinterpret_cast<float*>(lds + 16 * n);
  float4* pl = reinterpret_cast<float4*>(o32 + 8 * n);
  float* vt = reinterpret_cast<float*>(pl + TCMP_TOTAL_PLANES);
  uint2* ei = reinterpret_cast<uint2*>(vt + 3 * TCMP_TOTAL_VERTS);
  unsigned* wq = reinterpret_cast<unsigned*>(ei + TCMP_TOTAL_EDGES) +
                 (threadIdx.x >> 6) * (kQwaveBytes / 4);
  for (int i = threadIdx.x; i < sc.n_obs * 16; i += blockDim.x) o64[i] = sc.obs[i];
  for (int i = threadIdx.x; i < sc.n_obs * 8; i += blockDim.x) o32[i] = sc.obs32[i];
  for (int i = threadIdx.x; i < TCMP_TOTAL_PLANES; i += blockDim.x) pl[i] = g.planes32[i];
  for (int i = threadIdx.x; i < 3 * TCMP_TOTAL_VERTS; i += blockDim.x) vt[i] = g.verts32[i];
  const uint2* gei = reinterpret_cast<const uint2*>(g.eidx);
  for (int i = threadIdx.x; i < TCMP_TOTAL_EDGES; i += blockDim.x) ei[i] = gei[i];
  __syncthreads();
  so = sc;
  so.obs = o64;
  so.obs32 = o32;
  so.wq = wq;
  so.csph = sc.sph;
  so.cv32 = vt;
  go = g;
  go.planes32 = pl;
  go.verts32 = vt;
  go.eidx = reinterpret_cast<const ushort4*>(ei);
}

struct TorqueCfg {
  int mode;      // 0 base, 1 nov, 2 rne
  double mass;   // problem.payload_mass
};

// ------------------------------------------------------------------------------------------
// utils.py closures
// ------------------------------------------------------------------------------------------
// get_refine_fn step (utils.py:3037): q <- (1/(n-i)) * (q2 - q) + q.  No FMA contraction so
// the intermediate edge points match numpy bit for bit.
__device__ __forceinline__ void refine_step(double q[7], const double q2[7], int n, int i) {
#pragma clang fp contract(off)
  const double r = 1.0 / (double)(n - i);
#pragma unroll
  for (int k = 0; k < 7; ++k) q[k] = r * (q2[k] - q[k]) + q[k];
}

// int(norm(diff / resolution, 2)) + 1 (utils.py:3072 + refine num_steps+1)
__device__ __forceinline__ int num_steps(const double q1[7], const double q2[7],
                                         const double res[7]) {
#pragma clang fp contract(off)
  double s = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double x = (q2[k] - q1[k]) / res[k];
    s += x * x;
  }
  const double r = sqrt(s);
  // bounded so a corrupt input can never spin a lane forever
  return (r < 1048576.0) ? (int)r + 1 : 1048577;
}

// sqrt(dot(w, diff*diff)) (utils.py:3010-3017)
__device__ __forceinline__ double distance(const double a[7], const double b[7],
                                           const double w[7]) {
#pragma clang fp contract(off)
  double s = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const double d = b[k] - a[k];
    s += w[k] * (d * d);
  }
  return sqrt(s);
}

__device__ __forceinline__ bool limits_violated(const double q[7]) {
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 7; ++k) bad |= !(kLo[k] <= q[k]) || !(q[k] <= kHi[k]);
  return bad;
}

// ------------------------------------------------------------------------------------------
// rne.py: recursive Newton-Euler, 7 links + composite (flange, hand, payload) body.
// The reference builds 6x6 spatial matrices per body (rne.py:9-27, 216-251); this is the
// same recursion written on 3-vectors with the Panda's bodies 8..10 merged (identity
// transforms, zero joint rates between them), identical up to rounding.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// R^T x for the DH rotation of row j (rows of tf_mat, rne.py:39-42)
__device__ __forceinline__ void dh_rt(int j, double c, double s, const double x[3], double o[3]) {
  const double ca = kDhCa[j], sa = kDhSa[j];
  // R = [[c, -s, 0], [s ca, c ca, -sa], [s sa, c sa, ca]]
  o[0] = c * x[0] + (s * ca) * x[1] + (s * sa) * x[2];
  o[1] = -s * x[0] + (c * ca) * x[1] + (c * sa) * x[2];
  o[2] = -sa * x[1] + ca * x[2];
}
__device__ __forceinline__ void dh_r(int j, double c, double s, const double x[3], double o[3]) {
  const double ca = kDhCa[j], sa = kDhSa[j];
  o[0] = c * x[0] - s * x[1];
  o[1] = (s * ca) * x[0] + (c * ca) * x[1] - sa * x[2];
  o[2] = (s * sa) * x[0] + (c * sa) * x[1] + ca * x[2];
}

// tau[7] = rne(q, qd, qdd) with payload mass mp (0 = no payload).  cq/sq = cos/sin(q).
template <bool DYN>
__device__ __forceinline__ void rne(const double cq[7], const double sq[7], const double qd[7],
                                    const double qdd[7], double mp, double tau[7]) {
  double w[3] = {0, 0, 0}, v[3] = {0, 0, 0}, al[3] = {0, 0, 0}, ac[3] = {0, 0, 9.81};
  double fl[8][3], fa[8][3];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double c = i < 7 ? cq[i] : 1.0, s = i < 7 ? sq[i] : 0.0;
    const double p[3] = {kDhA[i], -kDhSa[i] * kDhD[i], kDhCa[i] * kDhD[i]};
    double wn[3], vn[3], aln[3], acn[3];
    if (DYN) {
      double t[3], u[3];
      cross3(w, p, t);
      u[0] = v[0] + t[0]; u[1] = v[1] + t[1]; u[2] = v[2] + t[2];
      dh_rt(i, c, s, u, vn);
      double Ew[3];
      dh_rt(i, c, s, w, Ew);
      const double qdi = i < 7 ? qd[i] : 0.0, qddi = i < 7 ? qdd[i] : 0.0;
      wn[0] = Ew[0]; wn[1] = Ew[1]; wn[2] = Ew[2] + qdi;
      cross3(al, p, t);
      u[0] = ac[0] + t[0]; u[1] = ac[1] + t[1]; u[2] = ac[2] + t[2];
      dh_rt(i, c, s, u, acn);
      // + v_i x (qd e_z)
      acn[0] += vn[1] * qdi; acn[1] -= vn[0] * qdi;
      dh_rt(i, c, s, al, aln);
      // + (E w) x (qd e_z)
      aln[0] += Ew[1] * qdi; aln[1] -= Ew[0] * qdi; aln[2] += qddi;
    } else {
      dh_rt(i, c, s, ac, acn);
    }
    // body forces f = I a + crf(v) I v
    if (i < 7) {
      const double m = kMass[i];
      const double* cc = kCom[i];
      const double* In = kInertia[i];
      if (DYN) {
        double t[3], vc[3], acc[3], hl[3], ha[3], Iw[3], Ial[3];
        cross3(wn, cc, t);
        vc[0] = vn[0] + t[0]; vc[1] = vn[1] + t[1]; vc[2] = vn[2] + t[2];
        cross3(aln, cc, t);
        acc[0] = acn[0] + t[0]; acc[1] = acn[1] + t[1]; acc[2] = acn[2] + t[2];
        hl[0] = m * vc[0]; hl[1] = m * vc[1]; hl[2] = m * vc[2];
        Iw[0] = In[0] * wn[0] + In[1] * wn[1] + In[2] * wn[2];
        Iw[1] = In[1] * wn[0] + In[3] * wn[1] + In[4] * wn[2];
        Iw[2] = In[2] * wn[0] + In[4] * wn[1] + In[5] * wn[2];
        Ial[0] = In[0] * aln[0] + In[1] * aln[1] + In[2] * aln[2];
        Ial[1] = In[1] * aln[0] + In[3] * aln[1] + In[4] * aln[2];
        Ial[2] = In[2] * aln[0] + In[4] * aln[1] + In[5] * aln[2];
        double cv[3], ca2[3];
        cross3(cc, vc, cv);
        cross3(cc, acc, ca2);
        ha[0] = Iw[0] + m * cv[0]; ha[1] = Iw[1] + m * cv[1]; ha[2] = Iw[2] + m * cv[2];
        double wxh[3], vxh[3], wxha[3];
        cross3(wn, hl, wxh);
        cross3(vn, hl, vxh);
        cross3(wn, ha, wxha);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          fl[i][k] = m * acc[k] + wxh[k];
          fa[i][k] = Ial[k] + m * ca2[k] + vxh[k] + wxha[k];
        }
      } else {
        double ca2[3];
        cross3(cc, acn, ca2);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          fl[i][k] = m * acn[k];
          fa[i][k] = m * ca2[k];
        }
      }
    } else {
      // composite flange (m 0, I .001) + hand (m .68, I .1) + payload (m mp, I diag(mr^2,mr^2,0))
      const double m = kHandMass + mp;
      if (DYN) {
        const double Ixy = kFlangeHandI + mp * (kPayloadR * kPayloadR), Iz = kFlangeHandI;
        double hl[3] = {m * vn[0], m * vn[1], m * vn[2]};
        double ha[3] = {Ixy * wn[0], Ixy * wn[1], Iz * wn[2]};
        double wxh[3], vxh[3], wxha[3];
        cross3(wn, hl, wxh);
        cross3(vn, hl, vxh);
        cross3(wn, ha, wxha);
        fl[i][0] = m * acn[0] + wxh[0];
        fl[i][1] = m * acn[1] + wxh[1];
        fl[i][2] = m * acn[2] + wxh[2];
        fa[i][0] = Ixy * aln[0] + vxh[0] + wxha[0];
        fa[i][1] = Ixy * aln[1] + vxh[1] + wxha[1];
        fa[i][2] = Iz * aln[2] + vxh[2] + wxha[2];
      } else {
        fl[i][0] = m * acn[0]; fl[i][1] = m * acn[1]; fl[i][2] = m * acn[2];
        fa[i][0] = 0; fa[i][1] = 0; fa[i][2] = 0;
      }
    }
    if (DYN) {
#pragma unroll
      for (int k = 0; k < 3; ++k) { w[k] = wn[k]; v[k] = vn[k]; al[k] = aln[k]; }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) ac[k] = acn[k];
  }
  // backward pass (rne.py:247-251): f_{i-1} += Ad(Xup_i)^T f_i
#pragma unroll
  for (int i = 7; i >= 1; --i) {
    const double c = i < 7 ? cq[i] : 1.0, s = i < 7 ? sq[i] : 0.0;
    const double p[3] = {kDhA[i], -kDhSa[i] * kDhD[i], kDhCa[i] * kDhD[i]};
    double Rf[3], Rn[3], pxRf[3];
    dh_r(i, c, s, fl[i], Rf);
    dh_r(i, c, s, fa[i], Rn);
    cross3(p, Rf, pxRf);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      fl[i - 1][k] += Rf[k];
      fa[i - 1][k] += pxRf[k] + Rn[k];
    }
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) tau[i] = fa[i][2];
}

// torque test: true = within limits (joint 7 unchecked, `>=` fails)
template <bool DYN>
__device__ __forceinline__ bool torque_ok(const double cq[7], const double sq[7],
                                          const double qd[7], const double qdd[7],
                                          double mass) {
  double tau[7];
  rne<DYN>(cq, sq, qd, qdd, mass > kPayloadMin ? mass : 0.0, tau);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 6; ++i) ok &= !(fabs(tau[i]) >= kEffort[i]);
  return ok;
}

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave reductions, all in DPP (no LDS round trips, one readlane): two quad_perm and two row_ror
// steps reduce each 16-lane row, row_bcast:15 folds rows 0 -> 1 and 2 -> 3, row_bcast:31 folds
// row 1 -> rows 2 and 3 (lanes outside a broadcast's row mask keep their value through `old`),
// so lane 63 holds the result.  Wave-uniform.  Call with every lane of the wave active.
template <int C>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, true);
}
template <int C>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<C>(__float_as_int(v)));
}
template <int C>
__device__ __forceinline__ double dpp_d(double v) {
  return __hiloint2double(dpp_i<C>(__double2hiint(v)), dpp_i<C>(__double2loint(v)));
}
__device__ __forceinline__ int bc15_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false);
}
__device__ __forceinline__ int bc31_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false);
}
__device__ __forceinline__ float bc15_f(float v) { return __int_as_float(bc15_i(__float_as_int(v))); }
__device__ __forceinline__ float bc31_f(float v) { return __int_as_float(bc31_i(__float_as_int(v))); }
__device__ __forceinline__ double bc15_d(double v) {
  return __hiloint2double(bc15_i(__double2hiint(v)), bc15_i(__double2loint(v)));
}
__device__ __forceinline__ double bc31_d(double v) {
  return __hiloint2double(bc31_i(__double2hiint(v)), bc31_i(__double2loint(v)));
}
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ double wave_min(double x) {
  x = fmin(x, dpp_d<0xB1>(x));
  x = fmin(x, dpp_d<0x4E>(x));
  x = fmin(x, dpp_d<0x124>(x));
  x = fmin(x, dpp_d<0x128>(x));
  x = fmin(x, bc15_d(x));
  x = fmin(x, bc31_d(x));
  return readlane_d(x, 63);
}
__device__ __forceinline__ double wave_max(double x) {
  x = fmax(x, dpp_d<0xB1>(x));
  x = fmax(x, dpp_d<0x4E>(x));
  x = fmax(x, dpp_d<0x124>(x));
  x = fmax(x, dpp_d<0x128>(x));
  x = fmax(x, bc15_d(x));
  x = fmax(x, bc31_d(x));
  return readlane_d(x, 63);
}
// OR over the wave (every lane active), wave-uniform
__device__ __forceinline__ unsigned wave_or_u32(unsigned x) {
  int v = (int)x;
  v |= dpp_i<0xB1>(v);
  v |= dpp_i<0x4E>(v);
  v |= dpp_i<0x124>(v);
  v |= dpp_i<0x128>(v);
  v |= bc15_i(v);
  v |= bc31_i(v);
  return (unsigned)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(v, 63));
}
__device__ __forceinline__ int wave_min_int(int x) {
  x = min(x, dpp_i<0xB1>(x));
  x = min(x, dpp_i<0x4E>(x));
  x = min(x, dpp_i<0x124>(x));
  x = min(x, dpp_i<0x128>(x));
  x = min(x, bc15_i(x));
  x = min(x, bc31_i(x));
  return __builtin_amdgcn_readlane(x, 63);
}

// ------------------------------------------------------------------------------------------
// exact hull-vs-box penetration depth, wave-cooperative (every lane of the wave calls it
// with identical arguments).  Penetration = min over the facets of the Minkowski
// difference: box faces, hull facets, silhouette hull edges x box axes (Gauss-map pruning).
// R,p: link pose (world); ob: obstacle record.  Early-outs once < kPen (result only
// compared against kPen).
// ------------------------------------------------------------------------------------------
struct Pose {
  double R[9];
  double p[3];
};

// pose: R[9], p[3] in the wave's LDS pose slot (wave_pose_slot); the geometry pointers are
// passed one by one, so every argument travels in registers
__device__ __noinline__ double exact_pd_wave(int link, const double* pose,
                                             const double* __restrict__ ob,
                                             const double* __restrict__ gverts,
                                             const double* __restrict__ gplanes,
                                             const double* __restrict__ gedges) {
  const int lane = lane_id();
  const double* R = pose;
  const double* p = pose + 9;
  const struct { const double* verts; const double* planes; const double* edges; } g = {
      gverts, gplanes, gedges};
  // box in the link frame
  const double d[3] = {ob[0] - p[0], ob[1] - p[1], ob[2] - p[2]};
  double cl[3], A[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cl[i] = R[0 + i] * d[0] + R[3 + i] * d[1] + R[6 + i] * d[2];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A[3 * i + j] = R[0 + i] * ob[3 + j] + R[3 + i] * ob[6 + j] + R[6 + i] * ob[9 + j];
  }
  const double h[3] = {ob[12], ob[13], ob[14]};
  const int v0 = tcmp_geo_vert_off[link], v1 = tcmp_geo_vert_off[link + 1];
  const int f0 = tcmp_geo_plane_off[link], f1 = tcmp_geo_plane_off[link + 1];
  const int e0 = tcmp_geo_edge_off[link], e1 = tcmp_geo_edge_off[link + 1];
  // box face facets: hull support along +-a_i
  double mn0 = INFINITY, mn1 = INFINITY, mn2 = INFINITY;
  double mx0 = -INFINITY, mx1 = -INFINITY, mx2 = -INFINITY;
  for (int v = v0 + lane; v < v1; v += 64) {
    const double4 P = *reinterpret_cast<const double4*>(g.verts + 4 * v);
    const double d0 = A[0] * P.x + A[3] * P.y + A[6] * P.z;
    const double d1 = A[1] * P.x + A[4] * P.y + A[7] * P.z;
    const double d2 = A[2] * P.x + A[5] * P.y + A[8] * P.z;
    mn0 = fmin(mn0, d0); mx0 = fmax(mx0, d0);
    mn1 = fmin(mn1, d1); mx1 = fmax(mx1, d1);
    mn2 = fmin(mn2, d2); mx2 = fmax(mx2, d2);
  }
  mn0 = wave_min(mn0); mn1 = wave_min(mn1); mn2 = wave_min(mn2);
  mx0 = wave_max(mx0); mx1 = wave_max(mx1); mx2 = wave_max(mx2);
  double pd = INFINITY;
  {
    const double pc0 = A[0] * cl[0] + A[3] * cl[1] + A[6] * cl[2];
    const double pc1 = A[1] * cl[0] + A[4] * cl[1] + A[7] * cl[2];
    const double pc2 = A[2] * cl[0] + A[5] * cl[1] + A[8] * cl[2];
    pd = fmin(pd, fmin(mx0 - pc0 + h[0], pc0 + h[0] - mn0));
    pd = fmin(pd, fmin(mx1 - pc1 + h[1], pc1 + h[1] - mn1));
    pd = fmin(pd, fmin(mx2 - pc2 + h[2], pc2 + h[2] - mn2));
  }
  if (pd < kPen) return pd;
  double loc = INFINITY;
  // hull facets
  for (int f = f0 + lane; f < f1; f += 64) {
    const double* P = g.planes + 8 * f;
    const double4 n = *reinterpret_cast<const double4*>(P);
    const double wmin = P[4];
    (void)wmin;
    const double pc = n.x * cl[0] + n.y * cl[1] + n.z * cl[2];
    const double rad = h[0] * fabs(n.x * A[0] + n.y * A[3] + n.z * A[6]) +
                       h[1] * fabs(n.x * A[1] + n.y * A[4] + n.z * A[7]) +
                       h[2] * fabs(n.x * A[2] + n.y * A[5] + n.z * A[8]);
    loc = fmin(loc, n.w - pc + rad);
  }
  // silhouette edges x box axes
  for (int e = e0 + lane; e < e1; e += 64) {
    const double* E = g.edges + 16 * e;
    const double4 ev = *reinterpret_cast<const double4*>(E);
    const double4 va = *reinterpret_cast<const double4*>(E + 4);
    const double4 n1 = *reinterpret_cast<const double4*>(E + 8);
    const double4 n2 = *reinterpret_cast<const double4*>(E + 12);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double ax0 = A[0 + i], ax1 = A[3 + i], ax2 = A[6 + i];
      const double s1 = n1.x * ax0 + n1.y * ax1 + n1.z * ax2;
      const double s2 = n2.x * ax0 + n2.y * ax1 + n2.z * ax2;
      if (s1 * s2 < 0) {
        double m0 = ev.y * ax2 - ev.z * ax1, m1 = ev.z * ax0 - ev.x * ax2,
               m2 = ev.x * ax1 - ev.y * ax0;
        const double len2 = m0 * m0 + m1 * m1 + m2 * m2;
        if (len2 >= 1e-24) {
          if (m0 * (n1.x + n2.x) + m1 * (n1.y + n2.y) + m2 * (n1.z + n2.z) < 0) {
            m0 = -m0; m1 = -m1; m2 = -m2;
          }
          const double hv = m0 * va.x + m1 * va.y + m2 * va.z;
          const double pc = m0 * cl[0] + m1 * cl[1] + m2 * cl[2];
          const double rad = h[0] * fabs(m0 * A[0] + m1 * A[3] + m2 * A[6]) +
                             h[1] * fabs(m0 * A[1] + m1 * A[4] + m2 * A[7]) +
                             h[2] * fabs(m0 * A[2] + m1 * A[5] + m2 * A[8]);
          loc = fmin(loc, (hv - pc + rad) / sqrt(len2));
        }
      }
    }
  }
  return fmin(pd, wave_min(loc));
}

__device__ __forceinline__ float wave_minf(float x) {
  x = fminf(x, dpp_f<0xB1>(x));
  x = fminf(x, dpp_f<0x4E>(x));
  x = fminf(x, dpp_f<0x124>(x));
  x = fminf(x, dpp_f<0x128>(x));
  x = fminf(x, bc15_f(x));
  x = fminf(x, bc31_f(x));
  return readlane_f(x, 63);
}
__device__ __forceinline__ float wave_minf_bc(float x) {
  x = fminf(x, dpp_f<0xB1>(x));
  x = fminf(x, dpp_f<0x4E>(x));
  x = fminf(x, dpp_f<0x124>(x));
  x = fminf(x, dpp_f<0x128>(x));
  x = fminf(x, bc15_f(x));
  x = fminf(x, bc31_f(x));
  return readlane_f(x, 63);
}
__device__ __forceinline__ float wave_maxf(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x128>(x));
  x = fmaxf(x, bc15_f(x));
  x = fmaxf(x, bc31_f(x));
  return readlane_f(x, 63);
}

// fp32 first pass of exact_pd_wave on the LDS geometry.  Same candidate axes and the same
// early-out; returns NaN when an axis is too close to degenerate for fp32 to classify it the
// way fp64 does (silhouette sign, tiny cross product, orientation), so the caller falls back
// to the fp64 test.  Otherwise |result - fp64 result| is far below kExactGuard (errors of a
// few 1e-6 m for coordinates of a few metres), and only results within kExactGuard of kPen
// are re-evaluated in fp64: the collision decision is always the fp64 one.
constexpr float kExactGuard = 1e-4f;
constexpr int max_link_edges() {
  int m = 0;
  for (int l = 0; l < TCMP_NLINKS; ++l) {
    const int n = tcmp_geo_edge_off[l + 1] - tcmp_geo_edge_off[l];
    m = n > m ? n : m;
  }
  return m;
}
#ifdef TCMP_PROF_EXACT
// mesh chain pairs past the head stage by the head's overlap excess (fa - kPen: buckets of
// 2.5 mm doubling to 32 cm, [9] no head, [10] head without an axis) and verdict ([16 + b]
// collision)
__device__ unsigned long long g_fa_hist[32];
// the same pairs by the sphere certificate's best ball-pair overlap (phase B): buckets
// < -8 cm, -4, -2, -1, 0, 1, 2, 3, 4 cm, [9] no spheres; [16 + b] collision
__device__ unsigned long long g_sb_hist[32];
// exact32 outcomes: [0] box-face exit, [1] facet exit, [2] full or edge-pass exit,
// [3] degenerate (fp64 fallback)
// phase-B pass structure: [0] passes, [1] entries, [2] distinct source lanes, [3] distinct
// (lane, link), [4] entries of links 7..9, [5] clocks from a pass's start to its exact loop
__device__ unsigned long long g_pass_stats[8];
__device__ unsigned long long g_exact_stats[32];  // [4..7]: mesh pairs (exact_pair),
                                                  // [8..13]: hull_hull_wave32 exits,
                                                  // [16..20]: exact_pair mesh-stage clocks
#endif
__device__ __forceinline__ float exact_pd_wave32(int link, const Pose pose,
                                              const double* __restrict__ ob, const Geo g,
                                              bool box_pair = false) {
  const int lane = lane_id();
#ifdef TCMP_PROF_EXACT
  // box pairs: stage clocks in g_exact_stats[16..19] (box faces, -, facets, edges) -- slots
  // the mesh stages use in mesh scenes
  unsigned long long tb = clock64();
#define TCMP_BOX_CLK(i) if (box_pair) { const unsigned long long t1 = clock64(); \
    if (lane == 0) atomicAdd(&g_exact_stats[16 + (i)], t1 - tb); tb = t1; }
#else
#define TCMP_BOX_CLK(i)
#endif
  const double* R = pose.R;
  const double* p = pose.p;
  const double d[3] = {ob[0] - p[0], ob[1] - p[1], ob[2] - p[2]};
  float cl[3], A[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cl[i] = (float)(R[0 + i] * d[0] + R[3 + i] * d[1] + R[6 + i] * d[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A[3 * i + j] = (float)(R[0 + i] * ob[3 + j] + R[3 + i] * ob[6 + j] + R[6 + i] * ob[9 + j]);
  }
  const float h[3] = {(float)ob[12], (float)ob[13], (float)ob[14]};
  constexpr float P = (float)kPen;
  const int v0 = tcmp_geo_vert_off[link], v1 = tcmp_geo_vert_off[link + 1];
  const int f0 = tcmp_geo_plane_off[link], f1 = tcmp_geo_plane_off[link + 1];
  const int e0 = tcmp_geo_edge_off[link], e1 = tcmp_geo_edge_off[link + 1];
  float mn0 = INFINITY, mn1 = INFINITY, mn2 = INFINITY;
  float mx0 = -INFINITY, mx1 = -INFINITY, mx2 = -INFINITY;
  for (int v = v0 + lane; v < v1; v += 64) {
    const float x = g.verts32[3 * v], y = g.verts32[3 * v + 1], z = g.verts32[3 * v + 2];
    const float d0 = A[0] * x + A[3] * y + A[6] * z;
    const float d1 = A[1] * x + A[4] * y + A[7] * z;
    const float d2 = A[2] * x + A[5] * y + A[8] * z;
    mn0 = fminf(mn0, d0); mx0 = fmaxf(mx0, d0);
    mn1 = fminf(mn1, d1); mx1 = fmaxf(mx1, d1);
    mn2 = fminf(mn2, d2); mx2 = fmaxf(mx2, d2);
  }
  mn0 = wave_minf(mn0); mn1 = wave_minf(mn1); mn2 = wave_minf(mn2);
  mx0 = wave_maxf(mx0); mx1 = wave_maxf(mx1); mx2 = wave_maxf(mx2);
  float pd;
  {
    const float pc0 = A[0] * cl[0] + A[3] * cl[1] + A[6] * cl[2];
    const float pc1 = A[1] * cl[0] + A[4] * cl[1] + A[7] * cl[2];
    const float pc2 = A[2] * cl[0] + A[5] * cl[1] + A[8] * cl[2];
    pd = fminf(fminf(mx0 - pc0 + h[0], pc0 + h[0] - mn0),
               fminf(fminf(mx1 - pc1 + h[1], pc1 + h[1] - mn1),
                     fminf(mx2 - pc2 + h[2], pc2 + h[2] - mn2)));
  }
  TCMP_BOX_CLK(0);
  if (pd < P - kExactGuard) {
#ifdef TCMP_PROF_EXACT
    if (lane == 0) atomicAdd(&g_exact_stats[0], 1ull);
#endif
    return pd;
  }
  TCMP_BOX_CLK(1);
  float loc = INFINITY;
  for (int f = f0 + lane; f < f1; f += 64) {
    const float4 n = g.planes32[f];
    const float pc = n.x * cl[0] + n.y * cl[1] + n.z * cl[2];
    const float rad = h[0] * fabsf(n.x * A[0] + n.y * A[3] + n.z * A[6]) +
                      h[1] * fabsf(n.x * A[1] + n.y * A[4] + n.z * A[7]) +
                      h[2] * fabsf(n.x * A[2] + n.y * A[5] + n.z * A[8]);
    loc = fminf(loc, n.w - pc + rad);
  }
  // facet axes are exact overlaps: one below kPen - guard already proves "free"
  {
    const float lf = fminf(pd, wave_minf(loc));
    TCMP_BOX_CLK(2);
    if (lf < P - kExactGuard) {
#ifdef TCMP_PROF_EXACT
      if (lane == 0) atomicAdd(&g_exact_stats[1], 1ull);
#endif
      return lf;
    }
  }
  // Edge axes in two passes.  Pass 1 (one edge per lane) marks the (edge, box axis) pairs
  // whose adjacent facet normals straddle the plane normal to the axis -- a few per cent of
  // them; pass 2 evaluates only the marked pairs, one per lane, each lane finding its pair by
  // its rank among the marks (a wave prefix sum of the per-lane counts, then a binary search
  // over the lanes).  The axis set is the one-pass test's, so the minimum is too.
  static_assert(max_link_edges() <= 640, "pass-1 marks: 3 bits per 64-edge slice in 32");
  bool deg = false;
  unsigned sil = 0;  // bit 3 it + i: edge e0 + 64 it + lane against box axis i
  for (int it = 0, base = e0; base < e1; ++it, base += 64) {
    const int e = base + lane;
    if (e < e1) {
      const ushort4 ix = g.eidx[e];
      const float4 n1 = g.planes32[ix.z];
      const float4 n2 = g.planes32[ix.w];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float a0 = A[0 + i], a1 = A[3 + i], a2 = A[6 + i];
        const float s1 = n1.x * a0 + n1.y * a1 + n1.z * a2;
        const float s2 = n2.x * a0 + n2.y * a1 + n2.z * a2;
        deg |= ((int)(fabsf(s1) < 1e-5f) | (int)(fabsf(s2) < 1e-5f)) != 0;
        if (s1 * s2 < 0.f) sil |= 1u << (3 * it + i);
      }
    }
  }
  const int cnt = __builtin_popcount(sil);
  int pre = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(pre, o);
    if (lane >= o) pre += t;
  }
  const int total = __shfl(pre, 63);
  pre -= cnt;  // exclusive prefix: lane l's marks are pairs [pre, pre + cnt)
  for (int w0 = 0; w0 < total; w0 += 64) {
    const int w = w0 + lane;
    int src = 0;  // the last lane whose prefix is <= w
#pragma unroll
    for (int step = 32; step; step >>= 1)
      if (__shfl(pre, src + step) <= w) src += step;
    unsigned m = (unsigned)__shfl((int)sil, src);
    const int k = w - __shfl(pre, src);
    if (w < total) {
      for (int j = 0; j < k; ++j) m &= m - 1;
      const int bit = __builtin_ctz(m);
      const int it = bit / 3, i = bit - 3 * it;
      const ushort4 ix = g.eidx[e0 + 64 * it + src];
      const float ax0 = g.verts32[3 * ix.x], ay0 = g.verts32[3 * ix.x + 1], az0 = g.verts32[3 * ix.x + 2];
      const float ex = g.verts32[3 * ix.y] - ax0, ey = g.verts32[3 * ix.y + 1] - ay0,
                  ez = g.verts32[3 * ix.y + 2] - az0;
      const float4 n1 = g.planes32[ix.z];
      const float4 n2 = g.planes32[ix.w];
      const float el2 = ex * ex + ey * ey + ez * ez;
      const float a0 = i == 0 ? A[0] : i == 1 ? A[1] : A[2];
      const float a1 = i == 0 ? A[3] : i == 1 ? A[4] : A[5];
      const float a2 = i == 0 ? A[6] : i == 1 ? A[7] : A[8];
      float m0 = ey * a2 - ez * a1, m1 = ez * a0 - ex * a2, m2 = ex * a1 - ey * a0;
      const float len2 = m0 * m0 + m1 * m1 + m2 * m2;
      if (len2 < 1e-8f * el2) {
        deg = true;
      } else {
        const float ori = m0 * (n1.x + n2.x) + m1 * (n1.y + n2.y) + m2 * (n1.z + n2.z);
        const float il = rsqrtf(len2);
        deg |= fabsf(ori) * il < 1e-4f;
        if (ori < 0.f) { m0 = -m0; m1 = -m1; m2 = -m2; }
        const float hv = m0 * ax0 + m1 * ay0 + m2 * az0;
        const float pc = m0 * cl[0] + m1 * cl[1] + m2 * cl[2];
        const float rad = h[0] * fabsf(m0 * A[0] + m1 * A[3] + m2 * A[6]) +
                          h[1] * fabsf(m0 * A[1] + m1 * A[4] + m2 * A[7]) +
                          h[2] * fabsf(m0 * A[2] + m1 * A[5] + m2 * A[8]);
        loc = fminf(loc, (hv - pc + rad) * il);
      }
    }
    // early "free" once a trustworthy axis is below kPen - guard (no degenerate axis so far)
    if (w0 + 64 < total && !__ballot(deg)) {
      const float lf = fminf(pd, wave_minf(loc));
      if (lf < P - kExactGuard) {
#ifdef TCMP_PROF_EXACT
        if (lane == 0) atomicAdd(&g_exact_stats[2], 1ull);
        if (lane == 0 && box_pair) atomicAdd(&g_exact_stats[27], 1ull);  // box: early edge exit
#endif
        return lf;
      }
    }
  }
#ifdef TCMP_PROF_EXACT
  if (lane == 0) atomicAdd(&g_exact_stats[__ballot(deg) ? 3 : 2], 1ull);
#endif
  if (__ballot(deg)) return __builtin_nanf("");
  const float full = fminf(pd, wave_minf(loc));
#ifdef TCMP_PROF_EXACT
  // box pairs through the whole edge pass: collision / free
  if (lane == 0 && box_pair) atomicAdd(&g_exact_stats[full >= P ? 28 : 29], 1ull);
#endif
  TCMP_BOX_CLK(3);
  return full;
#undef TCMP_BOX_CLK
}

}  // namespace tcmp
#include "tcmp_mesh.h"
namespace tcmp {

// Wave-cooperative facet trial axes, the first stage of the mesh chain (exact_pair): the pairs
// that reach it are those the lane-parallel certificates (sphere_cert) left open, and on those
// the exact test's minimising axis is mostly a facet normal of one hull (tools/cert_study.py).
// The most-overlapping ball pair (256 pairs, four per lane, wave argmax) gives the direction
// b (link frame) / a = R b (world); the mesh facet whose outward normal is closest to -a and
// the link facet whose normal is closest to b (wave argmax each) are tested with the full
// hulls' supports (link vertices from LDS, mesh vertices from global).  Returns the smaller
// of the two overlaps -- an upper bound of the depth ("free" below kPen - guard).
__device__ __forceinline__ float facet_axes_wave(int link, const float R[9], const float p[3], int mi,
                                                 const int* rg, const Scene sc, const Geo g) {
  const int lane = lane_id();
  const float4* LS = sc.csph + TCMP_NSPH * link;
  const float4* MS = sc.sph + TCMP_NSPH * (TCMP_NLINKS + mi);
  float best = -INFINITY, bx = 1.f, by = 0.f, bz = 0.f;
#pragma unroll
  for (int k = lane; k < TCMP_NSPH * TCMP_NSPH; k += 64) {
    const float4 t = MS[k % TCMP_NSPH];
    const float4 s = LS[k / TCMP_NSPH];
    const float dx = t.x - p[0], dy = t.y - p[1], dz = t.z - p[2];
    const float ex = R[0] * dx + R[3] * dy + R[6] * dz - s.x;
    const float ey = R[1] * dx + R[4] * dy + R[7] * dz - s.y;
    const float ez = R[2] * dx + R[5] * dy + R[8] * dz - s.z;
    const float ov = s.w + t.w - __builtin_sqrtf(ex * ex + ey * ey + ez * ez);
    if (ov > best) { best = ov; bx = ex; by = ey; bz = ez; }
  }
  {
    const float m = wave_maxf(best);
    const int L = __builtin_ctzll(__ballot(best == m));
    bx = __shfl(bx, L); by = __shfl(by, L); bz = __shfl(bz, L);
    const float l2 = bx * bx + by * by + bz * bz;
    if (!(l2 > 1e-12f)) return INFINITY;
    const float il = rsqrtf(l2);
    bx *= il; by *= il; bz *= il;
  }
  const float ax = R[0] * bx + R[1] * by + R[2] * bz;
  const float ay = R[3] * bx + R[4] * by + R[5] * bz;
  const float az = R[6] * bx + R[7] * by + R[8] * bz;
  int fm = rg[2], fl = tcmp_geo_plane_off[link];
  {
    float sm = -INFINITY, sl = -INFINITY;
    const int m1 = rg[3];
    for (int f = rg[2] + lane; f < m1; f += 64) {
      const float4 n = sc.mp32[f];
      const float v = -(n.x * ax + n.y * ay + n.z * az);
      if (v > sm) { sm = v; fm = f; }
    }
    const int l1 = tcmp_geo_plane_off[link + 1];
    for (int f = fl + lane; f < l1; f += 64) {
      const float4 n = g.planes32[f];
      const float v = n.x * bx + n.y * by + n.z * bz;
      if (v > sl) { sl = v; fl = f; }
    }
    const float mm = wave_maxf(sm), ml = wave_maxf(sl);
    fm = __builtin_amdgcn_readfirstlane(__shfl(fm, __builtin_ctzll(__ballot(sm == mm))));
    fl = __builtin_amdgcn_readfirstlane(__shfl(fl, __builtin_ctzll(__ballot(sl == ml))));
  }
  const float4 N = sc.mp32[fm];
  const float4 F = g.planes32[fl];
  const float qx = -(R[0] * N.x + R[3] * N.y + R[6] * N.z);  // -n in the link frame
  const float qy = -(R[1] * N.x + R[4] * N.y + R[7] * N.z);
  const float qz = -(R[2] * N.x + R[5] * N.y + R[8] * N.z);
  const float wx = R[0] * F.x + R[1] * F.y + R[2] * F.z;     // the link facet's world normal
  const float wy = R[3] * F.x + R[4] * F.y + R[5] * F.z;
  const float wz = R[6] * F.x + R[7] * F.y + R[8] * F.z;
  float h = -INFINITY, gm = INFINITY;
  const int v1 = tcmp_geo_vert_off[link + 1];
  for (int v = tcmp_geo_vert_off[link] + lane; v < v1; v += 64)
    h = fmaxf(h, sc.cv32[3 * v] * qx + sc.cv32[3 * v + 1] * qy + sc.cv32[3 * v + 2] * qz);
  const int w1 = rg[1];
  for (int w = rg[0] + lane; w < w1; w += 64) {
    const float4 x = sc.mv32[w];
    gm = fminf(gm, x.x * wx + x.y * wy + x.z * wz);
  }
  h = wave_maxf(h);
  gm = wave_minf(gm);
  const float o1 = h - (p[0] * N.x + p[1] * N.y + p[2] * N.z) + N.w;
  const float o2 = F.w + (p[0] * wx + p[1] * wy + p[2] * wz) - gm;
  return fminf(o1, o2);
}

// Exact penetration depth of one (link, obstacle) pair, wave-cooperative (all lanes, same
// arguments); only its comparison with kPen is used.  Boxes: the hull-vs-box test.  Meshes:
// the link hull against the mesh's outer box ("free" below kPen - guard, the mesh lies inside
// it) and against its inner box ("collision" at kPen + guard and above, it lies inside the
// mesh) -- both hull-vs-box -- then the hull-vs-hull test.  fp32 first, fp64 near kPen.
template <bool MESH>
__device__ __forceinline__ double exact_pair(int link, const Pose PL0, const double* ps,
                                             const double* ob, const Scene sc, const Geo g,
                                             float sbest = -INFINITY) {
  const int mi = MESH ? obs_mesh(ob) : -1;
  // mesh kernels: the pose is re-read from the wave's LDS stash (ps: its column, stride 64) at
  // each use instead of living in 24 VGPRs across the hull-vs-hull tests; the clobber keeps
  // the re-reads from being merged
  auto pose = [&]() -> Pose {
    if (!MESH) return PL0;
    __asm__ volatile("" ::: "memory");
    Pose x;
#pragma unroll
    for (int k = 0; k < 9; ++k) x.R[k] = ps[k * 64];
#pragma unroll
    for (int k = 0; k < 3; ++k) x.p[k] = ps[(9 + k) * 64];
    return x;
  };
  // the fp64 restatements are out of line; the pose reaches them through the wave's LDS slot
  auto pose_to_lds = [&]() {
    double* slot = wave_pose_slot(sc.wq);
    const Pose PL = pose();
    if (lane_id() == 0) {
#pragma unroll
      for (int k = 0; k < 9; ++k) slot[k] = PL.R[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) slot[9 + k] = PL.p[k];
    }
    __builtin_amdgcn_wave_barrier();
    return (const double*)slot;
  };
  if (!MESH || mi < 0) {
    const float pd32 = exact_pd_wave32(link, pose(), ob, g, true);
    if (pd32 == pd32 && fabsf(pd32 - (float)kPen) > kExactGuard) return (double)pd32;
    return exact_pd_wave(link, pose_to_lds(), ob, g.verts, g.planes, g.edges);
  }
#ifdef TCMP_PROF_EXACT
#define TCMP_MESH_STAT(i) if (lane_id() == 0) atomicAdd(&g_exact_stats[i], 1ull)
  unsigned long long tclk = clock64();
#define TCMP_MESH_CLK(i) { const unsigned long long t1 = clock64(); \
    if (lane_id() == 0) atomicAdd(&g_exact_stats[16 + (i)], t1 - tclk); tclk = t1; }
#else
#define TCMP_MESH_STAT(i)
#define TCMP_MESH_CLK(i)
#endif
  constexpr float P = (float)kPen;
  const int* rg = sc.mrange + kMrange * mi;
#ifdef TCMP_PROF_EXACT
  int fab = 9;
  const int sbb = !(sbest > -1e30f) ? 9 : sbest < -0.08f ? 0 : sbest < -0.04f ? 1 : sbest < -0.02f ? 2
                : sbest < -0.01f ? 3 : sbest < 0.f ? 4 : sbest < 0.01f ? 5 : sbest < 0.02f ? 6
                : sbest < 0.03f ? 7 : 8;
#define TCMP_FA_REC(v) if (lane_id() == 0) { \
    atomicAdd(&g_fa_hist[((v) >= kPen ? 16 : 0) + fab], 1ull); \
    atomicAdd(&g_sb_hist[((v) >= kPen ? 16 : 0) + sbb], 1ull); }
#else
#define TCMP_FA_REC(v)
#endif
  if (rg[19]) {
    float Rf[9], pf[3];
    {
      const Pose PL = pose();
#pragma unroll
      for (int k = 0; k < 9; ++k) Rf[k] = (float)PL.R[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) pf[k] = (float)PL.p[k];
    }
    const float fa = facet_axes_wave(link, Rf, pf, mi, rg, sc, g);
    TCMP_MESH_CLK(10);  // slot 26
    if (fa < P - kExactGuard) { TCMP_MESH_STAT(23); return (double)fa; }
#ifdef TCMP_PROF_EXACT
    {
      const float e = fa - P;
      fab = !(e < 1e30f) ? 10 : e < 0.0025f ? 0 : e < 0.005f ? 1 : e < 0.01f ? 2 : e < 0.02f ? 3
          : e < 0.04f ? 4 : e < 0.08f ? 5 : e < 0.16f ? 6 : e < 0.32f ? 7 : 8;
    }
#endif
  }
  float R[9], p[3];
  {
    const Pose PL = pose();
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = (float)PL.R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) p[k] = (float)PL.p[k];
  }
  // level-of-detail certificates: outer LODs contain the hulls ("free" below kPen - guard),
  // inner LODs lie inside them ("collision" above kPen + guard).  The pairs the lane-parallel
  // certificates leave open collide far more often than the rest, and a failing "free" test
  // runs to completion (every axis) while a failing "collision" test exits at its first axis
  // below the threshold: so, with the certificates on, the inner LODs go first.
  const bool inner_first = rg[18] && rg[19];
  auto inner_lod = [&]() -> float {
    const HullA32 Ai{sc.lodv3[0], sc.lodpl[0], sc.lodei[0], sc.lodev[0], tcmp_lod_in_vert_off[link],
                     tcmp_lod_in_vert_off[link + 1], tcmp_lod_in_plane_off[link],
                     tcmp_lod_in_plane_off[link + 1], tcmp_lod_in_edge_off[link],
                     tcmp_lod_in_edge_off[link + 1]};
    const HullB32 Bi{sc.lv32[0], sc.lp32[0], sc.le32[0], rg[6], rg[7], rg[8], rg[9], rg[10], rg[11],
                     sc.lcl[0], rg[22], rg[23]};
    return hull_hull_wave32<false>(Ai, Bi, R, p, P + kExactGuard);
  };
  if (inner_first) {
    const float pi = inner_lod();
    TCMP_MESH_CLK(2);
    if (pi == pi && pi > P + kExactGuard) { TCMP_MESH_STAT(6); TCMP_FA_REC(pi); return (double)pi; }
  }
  // The box and outer-LOD stages run only without the sphere certificates: with them, the pairs
  // that reach the chain are mostly ones those stages cannot decide (the outer LOD proved ~15 %
  // free, the outer box ~17 %), and the full hulls' facet passes decide them anyway -- without
  // the outer LOD C5 edges took 10 % less time, without the outer and inner boxes 1 % less
  // (same-box A/Bs, profiles/r9g_ab_c5_chain, r9j_ab_c5_boxes).
  if (!inner_first) {
    const float po = exact_pd_wave32(link, pose(), ob, g);
    TCMP_MESH_CLK(0);
    if (po == po && po < P - kExactGuard) { TCMP_MESH_STAT(4); TCMP_FA_REC(po); return (double)po; }
  }
  if (rg[18] && !inner_first) {
    const HullA32 Ao{sc.lodv3[1], sc.lodpl[1], sc.lodei[1], sc.lodev[1], tcmp_lod_out_vert_off[link],
                     tcmp_lod_out_vert_off[link + 1], tcmp_lod_out_plane_off[link],
                     tcmp_lod_out_plane_off[link + 1], tcmp_lod_out_edge_off[link],
                     tcmp_lod_out_edge_off[link + 1]};
    const HullB32 Bo{sc.lv32[1], sc.lp32[1], sc.le32[1], rg[12], rg[13], rg[14], rg[15], rg[16], rg[17],
                     sc.lcl[1], rg[24], rg[25]};
    const float pl = hull_hull_wave32<false>(Ao, Bo, R, p, P - kExactGuard);
    TCMP_MESH_CLK(1);
    if (pl == pl && pl < P - kExactGuard) { TCMP_MESH_STAT(5); TCMP_FA_REC(pl); return (double)pl; }
    if (!inner_first) {
      const float pi = inner_lod();
      TCMP_MESH_CLK(2);
      if (pi == pi && pi > P + kExactGuard) { TCMP_MESH_STAT(6); TCMP_FA_REC(pi); return (double)pi; }
    }
  } else if (!inner_first) {
    // the mesh's inner box ("collision" above kPen + guard): meshes without LODs
    const double* ib = sc.mib + 16 * mi;
    if (ib[12] > 0.0) {
      const float pi = exact_pd_wave32(link, pose(), ib, g);
      if (pi == pi && pi > P + kExactGuard) { TCMP_MESH_STAT(6); TCMP_FA_REC(pi); return (double)pi; }
    }
  }
  const HullA32 A{g.verts32, g.planes32, g.eidx, sc.geo_ev, tcmp_geo_vert_off[link],
                  tcmp_geo_vert_off[link + 1], tcmp_geo_plane_off[link],
                  tcmp_geo_plane_off[link + 1], tcmp_geo_edge_off[link], tcmp_geo_edge_off[link + 1]};
  const HullB32 B{sc.mv32, sc.mp32, sc.me32, rg[0], rg[1], rg[2], rg[3], rg[4], rg[5], sc.mcl,
                  rg[20], rg[21]};
  const float pm = hull_hull_wave32<true>(A, B, R, p, P - kExactGuard);
  TCMP_MESH_CLK(3);
  if (pm == pm && fabsf(pm - P) > kExactGuard) { TCMP_FA_REC(pm); return (double)pm; }
  TCMP_MESH_STAT(7);
  const double r64 = exact_mesh_wave(link, pose_to_lds(), mi, sc.mrange, sc.mp64, sc.mv64, sc.me64,
                                     sc.mcl, g.verts, g.planes, g.edges);
  TCMP_MESH_CLK(4);
  TCMP_FA_REC(r64);
  return r64;
#undef TCMP_MESH_STAT
#undef TCMP_MESH_CLK
#undef TCMP_FA_REC
}

// ------------------------------------------------------------------------------------------
// configuration check: collision (limits + 10 links x obstacles) and torque test.
// MUST be called by every lane of the wave (uniform control flow); `active` masks lanes.
// Collision tiers per (link, obstacle): (1) link-OBB extent on the obstacle's axes < pen ->
// free; (2) outer-OBB SAT < pen -> free; (3) inner-box SAT >= pen -> collision;
// (4) otherwise the exact wave-cooperative hull test.  (1)-(3) are conservative bounds of
// (4) (inner box subset hull subset outer OBB), so the answer is exactly (4)'s.
// ------------------------------------------------------------------------------------------
// wave totals (wave-uniform: popcounts of ballots, so they stay in SGPRs)
// Wave totals (wave-uniform, SGPRs).  Tier-0 tests are counted as live lane-steps: the wave
// total of 10 x n_obs tests per live lane overflowed 32 bits after ~26k steps of one
// persistent wave at 256 meshes; pairs_tested() scales them in 64 bits.
struct StepStats {
  unsigned live_steps;    // lane-steps that tested their obstacle pairs (tier 0)
  unsigned pairs_sat;     // tier-2/3 evaluations (at most 64 per flush pass)
  unsigned pairs_exact;   // tier-4 evaluations (one per wave-serial exact test)
#ifdef TCMP_PROF
  unsigned long long cyc_exact = 0;  // shader clocks spent in tier 4 (profiling builds)
  unsigned long long cyc_t123 = 0;   // ... in tiers 1-3 (maybe branch, excluding tier 4)
#endif
};

// Products with a compile-time zero factor are skipped (the joint rotations' and offsets' zero
// entries, the identity rotations of the flange and finger frames): x * 0 adds a signed zero, so
// for finite operands the sums are the full expressions' up to the sign of a zero result.
// (Multiplication by a constant 1 the compiler folds itself.)
__device__ __forceinline__ bool zconst(double k) { return __builtin_constant_p(k) && k == 0.0; }
__device__ __forceinline__ double zmul(double a, double b) {
  return (zconst(a) || zconst(b)) ? 0.0 : a * b;
}
__device__ __forceinline__ double zdot3(double a0, double b0, double a1, double b1, double a2,
                                        double b2) {
  const bool z0 = zconst(a0) || zconst(b0), z1 = zconst(a1) || zconst(b1),
             z2 = zconst(a2) || zconst(b2);
  if (z0 && z1 && z2) return 0.0;
  if (z0 && z1) return a2 * b2;
  if (z0 && z2) return a1 * b1;
  if (z1 && z2) return a0 * b0;
  if (z0) return a1 * b1 + a2 * b2;
  if (z1) return a0 * b0 + a2 * b2;
  if (z2) return a0 * b0 + a1 * b1;
  return a0 * b0 + a1 * b1 + a2 * b2;
}
__device__ __forceinline__ void frame_step_full(double R[9], double p[3], const double Rl[9],
                                                const double t[3]) {
  double nR[9], np[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      nR[3 * i + j] = R[3 * i + 0] * Rl[0 + j] + R[3 * i + 1] * Rl[3 + j] + R[3 * i + 2] * Rl[6 + j];
    np[i] = R[3 * i + 0] * t[0] + R[3 * i + 1] * t[1] + R[3 * i + 2] * t[2] + p[i];
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = nR[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = np[k];
}
__device__ __forceinline__ void frame_step(double R[9], double p[3], const double Rl[9],
                                           const double t[3]) {
  double nR[9], np[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      nR[3 * i + j] = zdot3(R[3 * i + 0], Rl[0 + j], R[3 * i + 1], Rl[3 + j], R[3 * i + 2], Rl[6 + j]);
    np[i] = zdot3(R[3 * i + 0], t[0], R[3 * i + 1], t[1], R[3 * i + 2], t[2]) + p[i];
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = nR[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = np[k];
}

// dyn mode (panda_primitives.py:60-116, get_torque_limits_not_exceded_test_v2):
// tau = M qdd + C qd + g + J^T [0, 0, m g, 0, 0, 0].  The reference takes M, C, g from
// panda_dynamics_model, which it does not ship: here they are rne.py's model without payload
// (parity unpinned against pdm).  J is pybullet's Jacobian at panda_grasptarget; its linear z
// row is (z_i x (p_target - o_i))_z for joint axis z_i through the URDF joint frame origin
// o_i; the grasp target sits 0.107 + 0.105 along link7's z axis (the hand only turns about z).
// The payload mass enters only through the force term, with no 0.01 kg threshold.
template <bool DYN>
__device__ __forceinline__ bool torque_ok_dyn(const double cq[7], const double sq[7],
                                              const double qd[7], const double qdd[7],
                                              double mass) {
  double tau[7];
  rne<DYN>(cq, sq, qd, qdd, 0.0, tau);
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
  double zx[7], zy[7], ox[7], oy[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const double cr = kJcr[j], sr = kJsr[j], c = cq[j], s = sq[j];
    const double Rl[9] = {c, -s, 0.0, zmul(cr, s), zmul(cr, c), -sr, zmul(sr, s), zmul(sr, c), cr};
    const double t[3] = {kJx[j], kJy[j], kJz[j]};
    frame_step(R, p, Rl, t);
    zx[j] = R[2];
    zy[j] = R[5];
    ox[j] = p[0];
    oy[j] = p[1];
  }
  constexpr double kTarget = kFlangeZ + 0.105;
  const double px = p[0] + R[2] * kTarget, py = p[1] + R[5] * kTarget;
  const double f = mass * 9.81;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double t = tau[i] + f * (zx[i] * (py - oy[i]) - zy[i] * (px - ox[i]));
    ok &= !(fabs(t) >= kEffort[i]);
  }
  return ok;
}

// classify one (link, obstacle) pair with the link pose (R, p):
// 0 free, 1 collision, 2 undecided (needs the exact test).  hin: the obstacle's inner half
// extents (a box: its own half extents; a mesh: the box inside its hull, same centre/axes).
__device__ __forceinline__ int classify_pair(int link, const double R[9], const double p[3],
                                             const double wc[3], const double U[9],
                                             const double aabb[3],
                                             const double* __restrict__ ob,
                                             const double* __restrict__ hin, bool& sat) {
  const double* bx = tcmp_geo_boxes + 18 * link;
  const double h0 = ob[12], h1 = ob[13], h2 = ob[14];
  const bool aligned = ob[15] > 0.0;
  // tier 1: link OBB extent along the obstacle axes
  double dc[3] = {wc[0] - ob[0], wc[1] - ob[1], wc[2] - ob[2]};
  if (aligned) {
    if ((h0 + aabb[0]) - fabs(dc[0]) < kPen) return 0;
    if ((h1 + aabb[1]) - fabs(dc[1]) < kPen) return 0;
    if ((h2 + aabb[2]) - fabs(dc[2]) < kPen) return 0;
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double bk0 = ob[3 + k], bk1 = ob[6 + k], bk2 = ob[9 + k];
      const double dk = bk0 * dc[0] + bk1 * dc[1] + bk2 * dc[2];
      double r = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        r += bx[12 + i] * fabs(bk0 * U[0 + i] + bk1 * U[3 + i] + bk2 * U[6 + i]);
      if ((ob[12 + k] + r) - fabs(dk) < kPen) return 0;
    }
  }
  sat = true;
  // tiers 2/3: 15-axis SAT in the link-box frame (M = U^T B, t = U^T (c - w))
  double M[9], aM[9], t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    t[i] = -(U[0 + i] * dc[0] + U[3 + i] * dc[1] + U[6 + i] * dc[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      M[3 * i + j] = U[0 + i] * ob[3 + j] + U[3 + i] * ob[6 + j] + U[6 + i] * ob[9 + j];
      aM[3 * i + j] = fabs(M[3 * i + j]);
    }
  }
  const double oh[3] = {bx[12], bx[13], bx[14]};
  const double ih[3] = {bx[15], bx[16], bx[17]};
  const double hb[3] = {h0, h1, h2};
  const double hi[3] = {hin[0], hin[1], hin[2]};
  bool inner_all = ih[0] > 0.0 && hi[0] > 0.0;
  constexpr double P2 = kPen * kPen;
  // link box axes
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double rb = hb[0] * aM[3 * i + 0] + hb[1] * aM[3 * i + 1] + hb[2] * aM[3 * i + 2];
    const double rbi = hi[0] * aM[3 * i + 0] + hi[1] * aM[3 * i + 1] + hi[2] * aM[3 * i + 2];
    const double dist = fabs(t[i]);
    if (oh[i] + rb - dist < kPen) return 0;
    inner_all &= (ih[i] + rbi - dist >= kPen);
  }
  // obstacle axes
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ra = oh[0] * aM[j] + oh[1] * aM[3 + j] + oh[2] * aM[6 + j];
    const double ri = ih[0] * aM[j] + ih[1] * aM[3 + j] + ih[2] * aM[6 + j];
    const double dist = fabs(t[0] * M[j] + t[1] * M[3 + j] + t[2] * M[6 + j]);
    if (ra + hb[j] - dist < kPen) return 0;
    inner_all &= (ri + hi[j] - dist >= kPen);
  }
  // cross axes U_i x B_j, |n|^2 = 1 - M_ij^2
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const double n2 = 1.0 - M[3 * i + j] * M[3 * i + j];
      if (n2 < 1e-12) continue;
      const double ra = oh[i1] * aM[3 * i2 + j] + oh[i2] * aM[3 * i1 + j];
      const double ri = ih[i1] * aM[3 * i2 + j] + ih[i2] * aM[3 * i1 + j];
      const double rb = hb[j1] * aM[3 * i + j2] + hb[j2] * aM[3 * i + j1];
      const double rbi = hi[j1] * aM[3 * i + j2] + hi[j2] * aM[3 * i + j1];
      const double dist = fabs(t[i2] * M[3 * i1 + j] - t[i1] * M[3 * i2 + j]);
      const double ov = ra + rb - dist;
      if (ov < 0 || ov * ov < P2 * n2) return 0;
      const double oi = ri + rbi - dist;
      inner_all &= (oi >= 0 && oi * oi >= P2 * n2);
    }
  }
  return inner_all ? 1 : 2;
}

// Self-collision pairs of get_self_link_pairs(panda, arm joints) (utils.py:3125-3149):
// links whose sets of moving ancestor joints differ (get_moving_pairs), minus parent/child
// pairs (are_links_adjacent, utils.py:1766); link7, link8, the hand and the fingers share the
// ancestor set {joint1..joint7}, link0 is the base (not in get_links), link8 has no geometry.
// Pair p checks link kSelfA[p] against link kSelfB[p] (link indices of the collision links).
constexpr int kNumSelfPairs = 33;
__device__ constexpr int kSelfA[kNumSelfPairs] = {
    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 3, 3, 4,
    0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5};
__device__ constexpr int kSelfB[kNumSelfPairs] = {
    2, 3, 4, 5, 6, 3, 4, 5, 6, 4, 5, 6, 5, 6, 6,
    7, 8, 9, 7, 8, 9, 7, 8, 9, 7, 8, 9, 7, 8, 9, 7, 8, 9};

// phase A's frame steps: zero-skipping in the box kernels, plain in the mesh kernels (the same
// values; the mesh kernels' register allocation spills 48 B per lane with the plain steps
// against 80 B, at the same speed, profiles/r9zr_ab_c5_frames/)
#define TCMP_FSA(...) (MESH ? frame_step_full(__VA_ARGS__) : frame_step(__VA_ARGS__))
// tier 0's boxes of the hand and the two fingers (collision links 7..9) in their own frames:
// centre, half extents of their hull vertices (panda_geometry.npz verts; the fp64 min / max,
// so the box holds the hull up to ~1e-17 m, inside tier 0's 1e-5 margin)
constexpr double kT0Box[3][6] = {
    {-1.0067597031593323e-05, -0.0017819218337535858, 0.020018674433231354,
     0.03162585012614727, 0.10220779851078987, 0.045943476259708405},
    {7.68294557929039e-06, 0.013135369845258538, 0.02699036512785824,
     0.010487135965377092, 0.013268012575281318, 0.026858668883505743},
    {-7.682945576062937e-06, -0.013135369845260508, 0.02699036512785824,
     0.010487135965377196, 0.013268012575281492, 0.026858668883505743}};

// Returns collision flag; all lanes must call.  `active` lanes only contribute.
//
// Phase A (every step): the 10 link frames are generated incrementally and each link's world
// AABB is kept in fp32 registers; then every obstacle's world AABB (one LDS broadcast) is
// tested against all ten (tier 0, branch-free; "maybe" iff the overlap could reach kPen on
// all three axes -- AABBs contain the shapes, so a penetration >= kPen always gives a
// "maybe").  Maybe pairs are queued in this wave's LDS queue as (lane, link, obstacle).
// Phase B (flush, when the queue could overflow and at the end): the queued pairs are
// processed lane-parallel -- each lane rebuilds its pair's link pose in fp64 from the owning
// lane's cos/sin and runs tiers 1-3 (classify_pair) -- and the undecided ones go through the
// wave-cooperative exact test (fp32 first pass, fp64 when near kPen or degenerate).
// Tiers 0-3 are conservative bounds of the exact test, so the answer is the exact test's.
// world frame of `link` (0..9) as collides_wave's phase A builds it, for per-lane links
// FULL: the frame steps without the zero-skipping (the box kernels' phase B: the same values,
// and their register allocation spills 16 B per lane instead of 64; the mesh kernels' the
// other way round, 80 B instead of 144)
template <bool FULL = false>
__device__ __forceinline__ void link_pose(int link, const double cq[7], const double sq[7],
                                          double Ro[9], double po[3]) {
  auto fstep = [](double R[9], double p[3], const double Rl[9], const double t[3]) {
    if (FULL) frame_step_full(R, p, Rl, t); else frame_step(R, p, Rl, t);
  };
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const double cr = kJcr[j], sr = kJsr[j], c = cq[j], s = sq[j];
    const double Rl[9] = {c, -s, 0.0, zmul(cr, s), zmul(cr, c), -sr, zmul(sr, s), zmul(sr, c), cr};
    const double t[3] = {kJx[j], kJy[j], kJz[j]};
    fstep(R, p, Rl, t);
    if (j == link) {
#pragma unroll
      for (int k = 0; k < 9; ++k) Ro[k] = R[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) po[k] = p[k];
    }
  }
  const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const double tz[3] = {0, 0, kFlangeZ};
  fstep(R, p, I, tz);
  const double Rz[9] = {kHandCy, -kHandSy, 0, kHandSy, kHandCy, 0, 0, 0, 1};
  const double z0[3] = {0, 0, 0};
  fstep(R, p, Rz, z0);
  if (link >= 7) {
    const double tf[3] = {0, link == 8 ? kFingerOpen : -kFingerOpen, kFingerZ};
    if (link > 7) fstep(R, p, I, tf);
#pragma unroll
    for (int k = 0; k < 9; ++k) Ro[k] = R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) po[k] = p[k];
  }
}

__device__ __forceinline__ void link_obb(int link, const double R[9], const double p[3],
                                         double wc[3], double U[9], double aabb[3]) {
  const double* bx = tcmp_geo_boxes + 18 * link;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    wc[i] = R[3 * i + 0] * bx[0] + R[3 * i + 1] * bx[1] + R[3 * i + 2] * bx[2] + p[i];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      U[3 * i + j] = R[3 * i + 0] * bx[3 + j] + R[3 * i + 1] * bx[6 + j] + R[3 * i + 2] * bx[9 + j];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    aabb[i] = bx[12] * fabs(U[3 * i + 0]) + bx[13] * fabs(U[3 * i + 1]) + bx[14] * fabs(U[3 * i + 2]);
}

#ifndef TCMP_SC_JUNROLL
#define TCMP_SC_JUNROLL 4   // sphere_cert's ball-pair loops: mesh balls (outer) ...
#endif
#ifndef TCMP_SC_IUNROLL
#define TCMP_SC_IUNROLL 16  // ... and link balls (inner)
#endif
#ifndef TCMP_SC_UNROLL
#define TCMP_SC_UNROLL 8  // stream unroll of sphere_cert's LOD / vertex loops
#endif
// Lane-parallel certificates for one pending (link, mesh) pair of phase B, ahead of the
// wave-cooperative exact chain (exact_pair), which handles one pair at a time with the whole
// wave.  Inscribed spheres of both hulls (Scene::sph, spheres.py / panda_spheres.inc): a sphere
// pair overlapping by >= kPen + guard proves "collision" (penetration depth is monotone under
// inclusion, utils.py:2833's -0.04 threshold).  The direction between the most-overlapping
// pair's centres is then a trial axis: the full hulls' projections on it overlapping by less
// than kPen - guard prove "free" (the depth is the minimum projection overlap over all
// directions).  fp32 throughout; its error (a few 1e-7 m for coordinates of a few metres) is
// far inside the 1e-4 guard, so the decision is the exact test's.  Returns 0 free,
// 1 collision, 2 undecided.  Mesh m: rows TCMP_NSPH * (10 + m) of sph, world frame (link
// meshes of self pairs: their own link frame, as the pose is then).
__device__ __forceinline__ int sphere_cert(int link, const float R[9], const float p[3], int mi,
                                            const Scene sc, const Geo g, float* bo = nullptr) {
  const float4* LS = sc.csph + TCMP_NSPH * link;               // LDS (mesh kernels)
  const float4* MS = sc.sph + TCMP_NSPH * (TCMP_NLINKS + mi);  // global
  // every mesh ball into the link frame once (u = R^T (t - p)), against the link's balls;
  // best: the largest overlap r_i + r_j - |u_j - s_i|, its link-frame direction s_i -> u_j
  float best = -INFINITY, ax = 1.f, ay = 0.f, az = 0.f;
  int bi = 0, bj = 0;
#pragma unroll TCMP_SC_JUNROLL
  for (int j = 0; j < TCMP_NSPH; ++j) {
    const float4 t = MS[j];
    const float dx = t.x - p[0], dy = t.y - p[1], dz = t.z - p[2];
    const float ux = R[0] * dx + R[3] * dy + R[6] * dz;
    const float uy = R[1] * dx + R[4] * dy + R[7] * dz;
    const float uz = R[2] * dx + R[5] * dy + R[8] * dz;
#pragma unroll TCMP_SC_IUNROLL
    for (int i = 0; i < TCMP_NSPH; ++i) {
      const float4 s = LS[i];
      const float ex = ux - s.x, ey = uy - s.y, ez = uz - s.z;
      const float ov = s.w + t.w - __builtin_sqrtf(ex * ex + ey * ey + ez * ez);
      if (ov > best) { best = ov; ax = ex; ay = ey; az = ez; bi = i; bj = j; }
    }
  }
#ifdef TCMP_PROF_EXACT
  if (bo) *bo = best;
#endif
  if (best >= (float)kPen + kExactGuard) return 1;
  const int* rg = sc.mrange + kMrange * mi;
  if (rg[18]) {
    // the best pair's balls against the other body's inner LOD hull (inside the full hull):
    // a ball whose centre c lies inside a convex polytope penetrates it by exactly
    // r + min over its facets of (d - n.c), so that value (>= 0 slack) is a lower bound of
    // the pair's depth
    float sl = INFINITY, sm = INFINITY;
    {
      const float4 t = MS[bj];  // the mesh ball in the link frame
      const float dx = t.x - p[0], dy = t.y - p[1], dz = t.z - p[2];
      const float lx = R[0] * dx + R[3] * dy + R[6] * dz;
      const float ly = R[1] * dx + R[4] * dy + R[7] * dz;
      const float lz = R[2] * dx + R[5] * dy + R[8] * dz;
      const int f1 = tcmp_lod_in_plane_off[link + 1];
#pragma unroll TCMP_SC_UNROLL
      for (int f = tcmp_lod_in_plane_off[link]; f < f1; ++f) {
        const float4 n = sc.lodpl[0][f];
        sl = fminf(sl, n.w - (n.x * lx + n.y * ly + n.z * lz));
      }
      sl = (sl >= 0.f && sl < 1e30f) ? sl + t.w : -INFINITY;
    }
    {
      const float4 s = LS[bi];  // the link ball in the world frame
      const float cx = R[0] * s.x + R[1] * s.y + R[2] * s.z + p[0];
      const float cy = R[3] * s.x + R[4] * s.y + R[5] * s.z + p[1];
      const float cz = R[6] * s.x + R[7] * s.y + R[8] * s.z + p[2];
      const int f1 = rg[9];
#pragma unroll TCMP_SC_UNROLL
      for (int f = rg[8]; f < f1; ++f) {
        const float4 n = sc.lp32[0][f];
        sm = fminf(sm, n.w - (n.x * cx + n.y * cy + n.z * cz));
      }
      sm = (sm >= 0.f && sm < 1e30f) ? sm + s.w : -INFINITY;
    }
    if (fmaxf(sl, sm) >= (float)kPen + kExactGuard) return 1;
  }
  const float l2 = ax * ax + ay * ay + az * az;
  if (!(l2 > 1e-12f)) return 2;
  const float il = rsqrtf(l2);
  // trial axis: b in the link frame, a = R b in the world
  const float bx = ax * il, by = ay * il, bz = az * il;
  ax = R[0] * bx + R[1] * by + R[2] * bz;
  ay = R[3] * bx + R[4] * by + R[5] * bz;
  az = R[6] * bx + R[7] * by + R[8] * bz;
  {
    // overlap along a: the link's support (its vertices, LDS) minus the mesh's minimum
    float hl = -INFINITY;
    const int v1 = tcmp_geo_vert_off[link + 1];
#pragma unroll TCMP_SC_UNROLL
    for (int v = tcmp_geo_vert_off[link]; v < v1; ++v)
      hl = fmaxf(hl, sc.cv32[3 * v] * bx + sc.cv32[3 * v + 1] * by + sc.cv32[3 * v + 2] * bz);
    float hm = INFINITY;
    const int w1 = rg[1];
#pragma unroll TCMP_SC_UNROLL
    for (int w = rg[0]; w < w1; ++w) {
      const float4 x = sc.mv32[w];
      hm = fminf(hm, x.x * ax + x.y * ay + x.z * az);
    }
    if (hl + (p[0] * ax + p[1] * ay + p[2] * az) - hm < (float)kPen - kExactGuard) return 0;
  }
  return 2;
}

// MESH = false: a scene without convex meshes (tcmp_set_meshes count 0) -- the mesh tiers
// are compiled out, which keeps the box-only kernels' register allocation unchanged.
// The joint-limit test (inclusive, utils.py:3181-3182) is the caller's: `active` lanes are
// those within the limits that still need their obstacle (and self) pairs.
template <bool MESH>
__device__ __forceinline__ bool collides_wave(const double cq[7], const double sq[7],
                                              bool active, const Scene sc, const Geo g,
                                              StepStats& st) {
  bool coll = false;
  if (sc.n_obs == 0 && !(MESH && sc.self_coll)) return coll;
  const int lane = lane_id();
  unsigned* queue = sc.wq;
  unsigned long long* cmask = reinterpret_cast<unsigned long long*>(sc.wq + kQcap);
  if (lane == 0) *cmask = 0ull;
  __builtin_amdgcn_wave_barrier();
  int count = 0;  // wave-uniform
  const bool live = active && !coll;
  // mesh kernels: cq / sq are read back from the wave's LDS stash (stored once here), so they
  // are not live in registers across phase B; the clobber keeps the reads real loads
  double* stash = MESH ? wave_stash(sc.wq) : nullptr;
  if (MESH) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      stash[k * 64 + lane] = cq[k];
      stash[(7 + k) * 64 + lane] = sq[k];
    }
    __asm__ volatile("" ::: "memory");
  }
  auto cq_of = [&](int k, int l) { return MESH ? stash[k * 64 + l] : __shfl(cq[k], l); };
  auto sq_of = [&](int k, int l) { return MESH ? stash[(7 + k) * 64 + l] : __shfl(sq[k], l); };
  // ---- phase B ------------------------------------------------------------------------
  auto flush = [&]() {
    __builtin_amdgcn_wave_barrier();
#ifdef TCMP_PROF
    const unsigned long long tf0 = clock64();
#endif
    for (int b = 0; b < count; b += 64) {
      const bool has = b + lane < count;
      const unsigned ent = has ? queue[b + lane] : 0u;
      const int src = (int)(ent & 63u), lk = (int)((ent >> 6) & 15u), o = (int)(ent >> 10);
      double c[7], s[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        c[k] = cq_of(k, src);
        s[k] = sq_of(k, src);
      }
      double R[9], p[3];
      link_pose<!MESH>(lk, c, s, R, p);
      // obstacle record row: the obstacle, or for a self pair the other link's outer box in
      // its own frame (row n_obs + j) -- the pose then becomes lk's pose in link j's frame
      int orow = o;
      if (MESH && o >= sc.n_obs) {
        const int j = kSelfB[o - sc.n_obs];
        orow = sc.n_obs + j;
        double Rj[9], pj[3];
        link_pose(j, c, s, Rj, pj);
        double Rr[9], pr[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
          for (int b = 0; b < 3; ++b)
            Rr[3 * a + b] = Rj[a] * R[b] + Rj[3 + a] * R[3 + b] + Rj[6 + a] * R[6 + b];
          pr[a] = Rj[a] * (p[0] - pj[0]) + Rj[3 + a] * (p[1] - pj[1]) + Rj[6 + a] * (p[2] - pj[2]);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = Rr[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) p[k] = pr[k];
      }
#ifdef TCMP_PROF_EXACT
      const unsigned long long tp0 = clock64();
      {
        unsigned dl = 0, dl2 = 0, dlk = 0;
        const unsigned sb = has ? 1u << (src & 31) : 0u;
        dl = __popc(wave_or_u32(src < 32 ? sb : 0u)) + __popc(wave_or_u32(src >= 32 ? sb : 0u));
        for (int l = 0; l < 10; ++l) {
          const bool on = has && lk == l;
          dlk += __popc(wave_or_u32(on && src < 32 ? sb : 0u)) +
                 __popc(wave_or_u32(on && src >= 32 ? sb : 0u));
        }
        dl2 = (unsigned)__popcll(__ballot(has && lk >= 7));
        const unsigned long long ne = __popcll(__ballot(has));
        if (lane == 0) {
          atomicAdd(&g_pass_stats[0], 1ull);
          atomicAdd(&g_pass_stats[1], ne);
          atomicAdd(&g_pass_stats[2], (unsigned long long)dl);
          atomicAdd(&g_pass_stats[3], (unsigned long long)dlk);
          atomicAdd(&g_pass_stats[4], (unsigned long long)dl2);
        }
      }
#endif
      int cls = 0, mi = -1;
#ifdef TCMP_PROF_EXACT
      float sbest = -INFINITY;  // the sphere certificate's best ball-pair overlap (prof stats)
#endif
      bool sat = false;
      if (has) {
        double wc[3], U[9], aabb[3];
        link_obb(lk, R, p, wc, U, aabb);
        const double* ob = sc.obs + 16 * orow;
        mi = MESH ? obs_mesh(ob) : -1;
        cls = classify_pair(lk, R, p, wc, U, aabb, ob, mi < 0 ? ob + 12 : sc.mib + 16 * mi + 12, sat);
      }
      if (MESH && __ballot(cls == 2)) {
        // the undecided pairs' poses go to the stash: R / p (fp64) die here instead of living
        // across the sphere certificates and every hull-vs-hull test of the wave
        double* ps = stash + 14 * 64;
#pragma unroll
        for (int k = 0; k < 9; ++k) ps[k * 64 + lane] = R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) ps[(9 + k) * 64 + lane] = p[k];
        __asm__ volatile("" ::: "memory");
        // lane-parallel sphere certificates before the wave-serial exact chain (fp32 pose)
        const bool sp = cls == 2 && mi >= 0 && sc.mrange[kMrange * mi + 19] != 0;
        if (__ballot(sp) && sp) {
          float Rf[9], pf[3];
#pragma unroll
          for (int k = 0; k < 9; ++k) Rf[k] = (float)ps[k * 64 + lane];
#pragma unroll
          for (int k = 0; k < 3; ++k) pf[k] = (float)ps[(9 + k) * 64 + lane];
#ifdef TCMP_PROF_EXACT
          cls = sphere_cert(lk, Rf, pf, mi, sc, g, &sbest);
#else
          cls = sphere_cert(lk, Rf, pf, mi, sc, g);
#endif
#ifdef TCMP_PROF_EXACT
          if (cls != 2) atomicAdd(&g_exact_stats[cls ? 14 : 15], 1ull);
#endif
        }
      }
      st.pairs_sat += (unsigned)__popcll(__ballot(sat));
      if (cls == 1) atomicOr(cmask, 1ull << src);
      uint64_t pend = __ballot(cls == 2);
#ifdef TCMP_PROF_EXACT
      if (lane == 0) atomicAdd(&g_pass_stats[5], clock64() - tp0);
#endif
      while (pend) {
        const int L = __builtin_ctzll(pend);
        pend &= pend - 1;
        // wave-uniform by construction; readfirstlane tells the compiler, so the hull data
        // indexed by them is scalar-loaded
        const int sL = __builtin_amdgcn_readfirstlane(__shfl(src, L));
        __builtin_amdgcn_wave_barrier();
        if ((*cmask >> sL) & 1ull) continue;  // that lane already collides
        const int lL = __builtin_amdgcn_readfirstlane(__shfl(lk, L)),
                  oL = __builtin_amdgcn_readfirstlane(__shfl(orow, L));
        Pose PL;
        if (!MESH) {
#pragma unroll
          for (int k = 0; k < 9; ++k) PL.R[k] = __shfl(R[k], L);
#pragma unroll
          for (int k = 0; k < 3; ++k) PL.p[k] = __shfl(p[k], L);
        }
        const double* ob = sc.obs + 16 * oL;
#ifdef TCMP_PROF
        const unsigned long long te0 = clock64();
#endif
#ifdef TCMP_PROF_EXACT
        const double pd = exact_pair<MESH>(lL, PL, MESH ? stash + 14 * 64 + L : nullptr, ob, sc, g,
                                           __shfl(sbest, L));
#else
        const double pd = exact_pair<MESH>(lL, PL, MESH ? stash + 14 * 64 + L : nullptr, ob, sc, g);
#endif
#ifdef TCMP_PROF
        st.cyc_exact += clock64() - te0;
#endif
        st.pairs_exact++;
        if (lane == 0 && pd >= kPen) atomicOr(cmask, 1ull << sL);
      }
    }
    __builtin_amdgcn_wave_barrier();
    count = 0;
#ifdef TCMP_PROF
    st.cyc_t123 += clock64() - tf0;
#endif
  };
  // ---- phase A ------------------------------------------------------------------------
  st.live_steps += (unsigned)__popcll(__ballot(live));
  // A queue that fills up is flushed after the loop and phase A resumes at (o_res, l_res);
  // the link AABBs are rebuilt on resume, so nothing of phase A is live across a flush.
  int o_res = 0, l_res = 0;
  while (true) {
    // world AABBs of the 10 links in fp32 (centre, half extent + rounding margin)
    float bc[10][3], bh[10][3];
    {
      auto put = [&](int link, const double Rr[9], const double pr[3]) {
        double wc[3], aabb[3];
        if (link >= 7) {
          // the hand and fingers: their hulls' boxes in their own frames (U = R: no axis
          // products; as tight as their OBBs, which are within 4 degrees of the frame axes)
          const double* b = kT0Box[link - 7];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            wc[i] = Rr[3 * i + 0] * b[0] + Rr[3 * i + 1] * b[1] + Rr[3 * i + 2] * b[2] + pr[i];
            aabb[i] = b[3] * fabs(Rr[3 * i + 0]) + b[4] * fabs(Rr[3 * i + 1]) + b[5] * fabs(Rr[3 * i + 2]);
          }
        } else {
          double U[9];
          link_obb(link, Rr, pr, wc, U, aabb);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          bc[link][i] = (float)wc[i];
          bh[link][i] = (float)aabb[i] + 1e-5f;
        }
      };
      double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        // (the joints' cos(alpha) = kCr = 4.9e-12 as an exact 0 here, which drops a third of
        // each frame step's products: the frames move by < 1e-10 m, far inside the boxes'
        // 1e-5 margin; phase B and the exact tests keep kCr.  With the hand boxes below and
        // the zero-skipping frame steps: k_fl_edges 3.13 -> 3.10 ms per C3 launch, same-box
        // A/B, profiles/r9z_ab_tier0/)
        const double cr = j > 0 ? 0.0 : kJcr[j], sr = kJsr[j],
                     c = MESH ? stash[j * 64 + lane] : cq[j],
                     s = MESH ? stash[(7 + j) * 64 + lane] : sq[j];
        const double Rl[9] = {c, -s, 0.0, zmul(cr, s), zmul(cr, c), -sr, zmul(sr, s), zmul(sr, c), cr};
        const double t[3] = {kJx[j], kJy[j], kJz[j]};
        TCMP_FSA(R, p, Rl, t);
        put(j, R, p);
      }
      const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      const double tz[3] = {0, 0, kFlangeZ};
      TCMP_FSA(R, p, I, tz);
      const double Rz[9] = {kHandCy, -kHandSy, 0, kHandSy, kHandCy, 0, 0, 0, 1};
      const double z0[3] = {0, 0, 0};
      TCMP_FSA(R, p, Rz, z0);
      put(7, R, p);
      double Rf[9], pf[3];
#pragma unroll
      for (int k = 0; k < 9; ++k) Rf[k] = R[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) pf[k] = p[k];
      const double tl[3] = {0, kFingerOpen, kFingerZ};
      TCMP_FSA(Rf, pf, I, tl);
      put(8, Rf, pf);
      const double tr[3] = {0, -kFingerOpen, kFingerZ};
      TCMP_FSA(R, p, I, tr);
      put(9, R, p);
    }
    // self pairs whose link AABBs overlap by kPen on all three axes (tier 0 of a self pair;
    // bh carries the rounding margin of both boxes)
    uint64_t smask = 0;
    if (MESH && sc.self_coll) {
      constexpr float P = (float)kPen;
#pragma unroll
      for (int q = 0; q < kNumSelfPairs; ++q) {
        const int a = kSelfA[q], b = kSelfB[q];
        smask |= (uint64_t)((int)(fabsf(bc[a][0] - bc[b][0]) <= bh[a][0] + bh[b][0] - P) &
                            (int)(fabsf(bc[a][1] - bc[b][1]) <= bh[a][1] + bh[b][1] - P) &
                            (int)(fabsf(bc[a][2] - bc[b][2]) <= bh[a][2] + bh[b][2] - P)) << q;
      }
    }
    const int n_tier0 = sc.n_obs + ((MESH && sc.self_coll) ? kNumSelfPairs : 0);
    // the link AABBs as bounds, three packed pairs per link: (lo x, lo y), (lo z, -hi x),
    // (-hi y, -hi z); against an obstacle's (hi x, hi y), (hi z, -lo x), (-lo y, -lo z) the six
    // differences are all negative iff the boxes overlap (three v_pk_add_f32 and a max per link)
    typedef float t0f2 __attribute__((ext_vector_type(2)));
    t0f2 t0a[10], t0b[10], t0c[10];
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      t0a[l] = t0f2{bc[l][0] - bh[l][0], bc[l][1] - bh[l][1]};
      t0b[l] = t0f2{bc[l][2] - bh[l][2], -(bc[l][0] + bh[l][0])};
      t0c[l] = t0f2{-(bc[l][1] + bh[l][1]), -(bc[l][2] + bh[l][2])};
    }
    // tier 0, obstacle-major: one LDS broadcast per obstacle serves all ten links
    bool full = false;
    for (int o = o_res; o < n_tier0 && !full; ++o) {
      unsigned lm = 0;
      if (o < sc.n_obs) {
        // the obstacle's (hi x, hi y), (hi z, -lo x), (-lo y, -lo z), kPen-shrunk (tier0_bounds)
        const float4 oa = *reinterpret_cast<const float4*>(sc.obs32 + 8 * o);
        const float4 ob4 = *reinterpret_cast<const float4*>(sc.obs32 + 8 * o + 4);
        const t0f2 oA = {oa.x, oa.y};
        const t0f2 oB = {oa.z, ob4.x};
        const t0f2 oC = {ob4.y, ob4.z};
#pragma unroll
        for (int l = 0; l < 10; ++l) {
          const t0f2 d1 = t0a[l] - oA, d2 = t0b[l] - oB, d3 = t0c[l] - oC;
          // all six negative (overlap on every axis): the sign bits of two v_max3 results
          const float mx = fmaxf(fmaxf(d1.x, d1.y), d2.x), my = fmaxf(fmaxf(d2.y, d3.x), d3.y);
          lm |= ((__float_as_uint(mx) & __float_as_uint(my)) >> 31) << l;
        }
      } else if (MESH) {
        const int q = o - sc.n_obs;
        lm = (unsigned)((smask >> q) & 1ull) << kSelfA[q];
      }
      if (!live) lm = 0;
      if (o == o_res) lm &= ~((1u << l_res) - 1u);  // links already queued before a flush
      if (__ballot(lm != 0u) == 0) continue;
      // only the links some lane queues (usually one or two of the ten): a wave-uniform walk
      // over the set bits of the wave's OR, instead of a ballot and branch for every link
      unsigned um = wave_or_u32(lm);
#pragma unroll 1
      while (um) {
        const int l = __builtin_ctz(um);
        um &= um - 1u;
        const bool m = (lm >> l) & 1u;
        const uint64_t bm = __ballot(m);
        if (count + (int)__popcll(bm) > kQcap) {
          o_res = o;
          l_res = l;
          full = true;
          break;
        }
        if (m) queue[count + (int)__popcll(bm & ((1ull << lane) - 1ull))] =
            (unsigned)lane | ((unsigned)l << 6) | ((unsigned)o << 10);
        count += (int)__popcll(bm);
      }
    }
    // one flush call site (a full queue always holds pairs): phase B is inlined once
    if (count) flush();
    if (!full) break;
  }
  __builtin_amdgcn_wave_barrier();
  coll |= active && ((*cmask >> lane) & 1ull);
  return coll;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 sample stream (same definition as oracle/tcmp_oracle.c)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox_uniforms(uint64_t seed, uint64_t k, double u[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t c0 = (uint32_t)k, c1 = (uint32_t)(k >> 32), c2 = (uint32_t)j, c3 = 0x7463u;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
      const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
      const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
      c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    const uint64_t a = ((uint64_t)c0 << 32) | c1, b = ((uint64_t)c2 << 32) | c3;
    u[2 * j] = (double)(a >> 11) * 0x1.0p-53;
    u[2 * j + 1] = (double)(b >> 11) * 0x1.0p-53;
  }
}

}  // namespace tcmp
