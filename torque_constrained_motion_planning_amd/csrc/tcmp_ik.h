// tcmp_ik.h -- goal IK on device: closed-form Panda IK of panda_link0 ->
// panda_link8 with joint 7 free, the solver the reference runs through its ikfast module
// (ikfast_panda_arm.cpp ComputeIk :12770, get_ik :12839; FK ComputeFk :307) for every
// free-joint draw of ikfast_inverse_kinematics (ikfast.py:136-169).
//
// Geometry (modified DH, rne.py:47-54):  with q7 fixed the wrist point O6 (= O5) is known;
// |O2 - O6| fixes q4 (two branches), the z5 component of O2 - O5 seen from frame 6 fixes q6
// (two branches), its in-plane direction fixes q5, and the remaining shoulder rotation
// R_0^3 = Rz(q1) Ry(q2) Rz(q3) gives q1..q3 (two signs of q2).  Branch b = 4*i4 + 2*i6 + i2.
// All angles come back in (-pi, pi] like ikfast's (e.g. :470-483); the limit filter is the
// caller's (ikfast.py:166).  One lane per (pose, free value).
#pragma once
// Included by tcmp_engine.hip inside its kernel namespace.

__device__ __forceinline__ double wrap_pi(double a) {
  constexpr double kPi = 3.141592653589793, k2Pi = 6.283185307179586;
  if (a > kPi) a -= k2Pi;
  if (a <= -kPi) a += k2Pi;
  return a;
}

// T_0^8 by the DH chain (rne.py get_tf_mat rows 0..7): R row-major, p.
__device__ __forceinline__ void fk8(const double q[7], double R[9], double p[3]) {
  double A[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    double c = 1.0, s = 0.0;
    if (j < 7) sincos(q[j], &s, &c);
    const double ca = kDhCa[j], sa = kDhSa[j], a = kDhA[j], d = kDhD[j];
    const double Rl[9] = {c, -s, 0.0, s * ca, c * ca, -sa, s * sa, c * sa, ca};
    const double tl[3] = {a, -sa * d, ca * d};
    frame_step(A, t, Rl, tl);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = A[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = t[k];
}

// Valid solutions written packed to out[c][7] in branch order (the loops below visit the
// branches b = 4*i4 + 2*i6 + i2 in increasing order, so no per-branch staging array -- which
// the compiler kept in scratch -- is needed); returns their count.
__device__ __forceinline__ int ik8(const double R[9], const double p[3], double q7,
                                   double* __restrict__ out) {
  constexpr double a = 0.0825, b = 0.384, d = 0.316, d1 = 0.333, a7 = 0.088, d8 = 0.107;
  constexpr double kPi = 3.141592653589793;
  double s7, c7;
  sincos(q7, &s7, &c7);
  // frame 6 axes: x6 = R (c7, -s7, 0), y6 = -z8, z6 = R (s7, c7, 0)
  double x6[3], y6[3], z6[3], u[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    x6[i] = R[3 * i] * c7 - R[3 * i + 1] * s7;
    y6[i] = -R[3 * i + 2];
    z6[i] = R[3 * i] * s7 + R[3 * i + 1] * c7;
    // O6 = p - d8 z8 - a7 x6 ; u = O2 - O6
    const double o6 = p[i] - d8 * R[3 * i + 2] - a7 * x6[i];
    u[i] = (i == 2 ? d1 : 0.0) - o6;
  }
  const double L2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  constexpr double K0 = 2 * a * a + b * b + d * d, K1 = 2 * (b * d - a * a), K2 = 2 * a * (b + d);
  const double r4 = hypot(K1, K2), phi = atan2(K2, K1);
  const double C4 = (L2 - K0) / r4;
  int c = 0;
  if (!(fabs(C4) <= 1.0)) return 0;
  const double acos4 = atan2(sqrt(1.0 - C4 * C4), C4);
  const double u6x = x6[0] * u[0] + x6[1] * u[1] + x6[2] * u[2];
  const double u6y = y6[0] * u[0] + y6[1] * u[1] + y6[2] * u[2];
  const double u6z = z6[0] * u[0] + z6[1] * u[1] + z6[2] * u[2];
  const double r6 = hypot(u6x, u6y), beta = atan2(u6y, u6x);
  for (int i4 = 0; i4 < 2; ++i4) {
    const double q4 = wrap_pi(-phi + (i4 ? -acos4 : acos4));
    double s4, c4;
    sincos(q4, &s4, &c4);
    const double K = -b + a * s4 - d * c4;  // z5 . (O2 - O5)
    const double W = a - a * c4 - d * s4;   // in-plane length, sign fixes q5
    if (!(r6 > 0.0) || !(fabs(K / r6) <= 1.0)) continue;
    const double S6 = K / r6, as6 = atan2(S6, sqrt(1.0 - S6 * S6));
    for (int i6 = 0; i6 < 2; ++i6) {
      const double q6 = wrap_pi(i6 ? (kPi - as6 - beta) : (as6 - beta));
      double s6, c6;
      sincos(q6, &s6, &c6);
      // u in frame 5: R_5^6 u6, R_5^6 = [[c6,-s6,0],[0,0,-1],[s6,c6,0]]
      const double u5x = c6 * u6x - s6 * u6y, u5y = -u6z;
      const double sg = W >= 0.0 ? 1.0 : -1.0;
      const double q5 = atan2(-u5y * sg, u5x * sg);
      double s5, c5;
      sincos(q5, &s5, &c5);
      // R3 = R6 (R_5^6)^T (R_4^5)^T (R_3^4)^T; only the entries Rz Ry Rz needs.
      // columns of R5 = R6 (R_5^6)^T: x5 = c6 x6 - s6 y6 ... from rows of R_5^6
      double x5[3], y5[3], z5[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        x5[i] = c6 * x6[i] - s6 * y6[i];
        y5[i] = -z6[i];
        z5[i] = s6 * x6[i] + c6 * y6[i];
      }
      // R4 = R5 (R_4^5)^T, R_4^5 = [[c5,-s5,0],[0,0,1],[-s5,-c5,0]]
      double x4[3], y4[3], z4[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        x4[i] = c5 * x5[i] - s5 * y5[i];
        y4[i] = z5[i];
        z4[i] = -s5 * x5[i] - c5 * y5[i];
      }
      // R3 = R4 (R_3^4)^T, R_3^4 = [[c4,-s4,0],[0,0,-1],[s4,c4,0]]
      double x3[3], y3[3], z3[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        x3[i] = c4 * x4[i] - s4 * y4[i];
        y3[i] = -z4[i];
        z3[i] = s4 * x4[i] + c4 * y4[i];
      }
      // R3 = Rz(q1) Ry(q2) Rz(q3): z3 = (c1 s2, s1 s2, c2), row 2 = (-s2 c3, s2 s3, c2)
      const double sb = sqrt(z3[0] * z3[0] + z3[1] * z3[1]);
      for (int i2 = 0; i2 < 2; ++i2) {
        const double sgn = i2 ? -1.0 : 1.0;
        const double q2 = atan2(sgn * sb, z3[2]);
        double q1, q3;
        if (sb > 1e-12) {
          q1 = atan2(sgn * z3[1], sgn * z3[0]);
          q3 = atan2(sgn * y3[2], -sgn * x3[2]);
        } else {  // q2 = 0 / pi: only q1 +- q3 is fixed; take q1 = 0
          q1 = 0.0;
          q3 = atan2(x3[1], x3[0]) * (z3[2] > 0.0 ? 1.0 : -1.0);
        }
        double* o = out + 7 * c++;
        o[0] = q1; o[1] = q2; o[2] = q3; o[3] = q4;
        o[4] = q5; o[5] = q6; o[6] = q7;
      }
    }
  }
  return c;
}

// one lane per (pose, free value): poses n x 12 (R row-major, p), free n; out n x 8 x 7,
// count n (valid solutions packed first, branch order kept)
__global__ __launch_bounds__(256) void k_ik(const double* __restrict__ poses,
                                            const double* __restrict__ free_q7, long long n,
                                            double* __restrict__ out, int* __restrict__ count) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double R[9], p[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = poses[12 * i + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = poses[12 * i + 9 + k];
  count[i] = ik8(R, p, free_q7[i], out + 56 * i);
}

__global__ __launch_bounds__(256) void k_fk8(const double* __restrict__ q, long long n,
                                             double* __restrict__ poses) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double qq[7], R[9], p[3];
#pragma unroll
  for (int k = 0; k < 7; ++k) qq[k] = q[7 * i + k];
  fk8(qq, R, p);
#pragma unroll
  for (int k = 0; k < 9; ++k) poses[12 * i + k] = R[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) poses[12 * i + 9 + k] = p[k];
}

