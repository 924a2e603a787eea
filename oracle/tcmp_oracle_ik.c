/*
 * tcmp_oracle_ik.c -- CPU restatement of the goal-IK pieces.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as tcmp_oracle.c: only tests/, smoke() and bench.py's
 * cpu_baseline leg load it; libtcmp.so never does).
 *
 * The reference solves panda_link0 -> panda_link8 IK with an OpenRAVE ikfast module
 * (src/ikfast_panda_arm.cpp, ComputeIk :12770 / get_ik :12839, one free joint = joint7,
 * :397-398) and FK with ComputeFk (:307).  That module cannot be built here (ikfast.h:41
 * includes "python2.7/Python.h", absent from the image; stand-in headers are not allowed), so
 * its 12.9k generated lines are restated by their published result: the closed-form
 * solution of the Panda's kinematics for a fixed joint 7, up to 8 branches
 * (q4: 2 x q6: 2 x q2 sign: 2).  Pinning: the FK below is the reference's own DH chain
 * (rne.py:32-63, golden tests/golden/fk_golden.npz) and every IK solution must map back
 * through it to the requested pose; the ikfast solution ORDER is not reproduced (the
 * reference shuffles it anyway, ikfast.py:163 randomize).  Written with explicit DH matrices
 * and 3x3 products; the HIP version (csrc/tcmp_ik.h) is expanded by hand.
 */
#include <math.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* rne.py:47-54 rows (a, d, alpha); theta = q_i, row 7 (flange) theta = 0 */
static const double IK_DH[8][3] = {
    {0.0, 0.333, 0.0},         {0.0, 0.0, -M_PI / 2},   {0.0, 0.316, M_PI / 2},
    {0.0825, 0.0, M_PI / 2},   {-0.0825, 0.384, -M_PI / 2}, {0.0, 0.0, M_PI / 2},
    {0.088, 0.0, M_PI / 2},    {0.0, 0.107, 0.0}};

/* get_tf_mat (rne.py:32-44) rotation and translation */
static void dh_tf(int row, double q, double R[3][3], double t[3]) {
  const double a = IK_DH[row][0], d = IK_DH[row][1], al = IK_DH[row][2];
  R[0][0] = cos(q); R[0][1] = -sin(q); R[0][2] = 0;
  R[1][0] = sin(q) * cos(al); R[1][1] = cos(q) * cos(al); R[1][2] = -sin(al);
  R[2][0] = sin(q) * sin(al); R[2][1] = cos(q) * sin(al); R[2][2] = cos(al);
  t[0] = a; t[1] = -sin(al) * d; t[2] = cos(al) * d;
}

static void mm3(const double A[3][3], const double B[3][3], double C[3][3]) {
  double T[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
  memcpy(C, T, sizeof(T));
}
static void mtm3(const double A[3][3], const double B[3][3], double C[3][3]) { /* A B^T */
  double T[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = A[i][0] * B[j][0] + A[i][1] * B[j][1] + A[i][2] * B[j][2];
  memcpy(C, T, sizeof(T));
}

/* T_0^8 = prod_i get_tf_mat(i) (the inverse of rne.get_parent_to_child_transform(q,0,8)) */
ORC_API void orc_fk8(const double* q, double* R9, double* p3) {
  double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, p[3] = {0, 0, 0};
  for (int row = 0; row < 8; ++row) {
    double Ri[3][3], ti[3];
    dh_tf(row, row < 7 ? q[row] : 0.0, Ri, ti);
    for (int k = 0; k < 3; ++k) p[k] += R[k][0] * ti[0] + R[k][1] * ti[1] + R[k][2] * ti[2];
    mm3(R, Ri, R);
  }
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) R9[3 * i + j] = R[i][j];
    p3[i] = p[i];
  }
}

static double wrap_pi(double a) {
  while (a > M_PI) a -= 2 * M_PI;
  while (a <= -M_PI) a += 2 * M_PI;
  return a;
}

/* IK for link8 pose (R9 row-major, p3) with joint 7 = q7.  sols: 8 x 7, branch b =
 * 4*(q4 branch) + 2*(q6 branch) + (q2 sign); valid[b] = 1 when the branch exists.
 * Returns the number of valid branches. */
ORC_API int orc_ik8(const double* R9, const double* p3, double q7, double* sols, int* valid) {
  const double a = 0.0825, b = 0.384, d = 0.316, d1 = 0.333, d8 = 0.107;
  double R8[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R8[i][j] = R9[3 * i + j];
  /* frame 7 = frame 8 rotated by I; origin O7 = p - d8 z8 */
  double O7[3], R67[3][3], t67[3], R6[3][3], O6[3];
  for (int k = 0; k < 3; ++k) O7[k] = p3[k] - d8 * R8[k][2];
  dh_tf(6, q7, R67, t67);           /* T_6^7 */
  mtm3(R8, R67, R6);                /* R6 = R7 (R_6^7)^T */
  for (int k = 0; k < 3; ++k)
    O6[k] = O7[k] - (R6[k][0] * t67[0] + R6[k][1] * t67[1] + R6[k][2] * t67[2]);
  /* u = O2 - O6, O2 = (0, 0, d1) */
  const double u[3] = {-O6[0], -O6[1], d1 - O6[2]};
  const double L2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  /* |O2 - O5|^2 = K0 + K1 cos q4 - K2 sin q4 (frame-3 chain, rows 3/4) */
  const double K0 = 2 * a * a + b * b + d * d, K1 = 2 * (b * d - a * a), K2 = 2 * a * (b + d);
  const double r4 = hypot(K1, K2), phi = atan2(K2, K1);
  const double C4 = (L2 - K0) / r4;
  int n = 0;
  for (int k = 0; k < 8; ++k) valid[k] = 0;
  if (!(fabs(C4) <= 1.0)) return 0;
  const double acos4 = atan2(sqrt(1.0 - C4 * C4), C4);
  /* u in frame 6 */
  double u6[3];
  for (int k = 0; k < 3; ++k) u6[k] = R6[0][k] * u[0] + R6[1][k] * u[1] + R6[2][k] * u[2];
  const double r6 = hypot(u6[0], u6[1]), beta = atan2(u6[1], u6[0]);
  for (int i4 = 0; i4 < 2; ++i4) {
    const double q4 = wrap_pi(-phi + (i4 ? -acos4 : acos4));
    const double s4 = sin(q4), c4 = cos(q4);
    /* z5 . (O2 - O5) and the in-plane length (frame-5 chain) */
    const double K = -b + a * s4 - d * c4;
    const double W = a - a * c4 - d * s4;
    if (!(r6 > 0) || !(fabs(K / r6) <= 1.0)) continue;
    const double S6 = K / r6, as6 = atan2(S6, sqrt(1.0 - S6 * S6));
    for (int i6 = 0; i6 < 2; ++i6) {
      const double q6 = wrap_pi(i6 ? (M_PI - as6 - beta) : (as6 - beta));
      double R56[3][3], t56[3], R5[3][3], u5[3];
      dh_tf(5, q6, R56, t56);
      mtm3(R6, R56, R5);
      for (int k = 0; k < 3; ++k) u5[k] = R5[0][k] * u[0] + R5[1][k] * u[1] + R5[2][k] * u[2];
      const double sg = W >= 0 ? 1.0 : -1.0;
      const double q5 = atan2(-u5[1] * sg, u5[0] * sg);
      double R45[3][3], R34[3][3], t[3], R4[3][3], R3[3][3];
      dh_tf(4, q5, R45, t);
      mtm3(R5, R45, R4);
      dh_tf(3, q4, R34, t);
      mtm3(R4, R34, R3);
      /* R3 = Rz(q1) Ry(q2) Rz(q3) (rows 0-2 with alpha 0, -pi/2, pi/2) */
      const double sb = sqrt(R3[0][2] * R3[0][2] + R3[1][2] * R3[1][2]);
      for (int i2 = 0; i2 < 2; ++i2) {
        const double sgn = i2 ? -1.0 : 1.0;
        const double q2 = atan2(sgn * sb, R3[2][2]);
        double q1, q3;
        if (sb > 1e-12) {
          q1 = atan2(sgn * R3[1][2], sgn * R3[0][2]);
          q3 = atan2(sgn * R3[2][1], -sgn * R3[2][0]);
        } else { /* wrist-1 singular: q1 + q3 (or q1 - q3) fixed; take q1 = 0 */
          q1 = 0.0;
          q3 = atan2(R3[1][0], R3[0][0]) * (R3[2][2] > 0 ? 1.0 : -1.0);
        }
        const int slot = 4 * i4 + 2 * i6 + i2;
        double* o = sols + 7 * slot;
        o[0] = q1; o[1] = q2; o[2] = q3; o[3] = q4; o[4] = q5; o[5] = q6; o[6] = q7;
        valid[slot] = 1;
        ++n;
      }
    }
  }
  return n;
}
