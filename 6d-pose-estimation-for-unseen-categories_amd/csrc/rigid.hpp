// Rigid fits shared by RANSAC (H13) and ICP (f4): the rotation that maximises
// sum d·(R s) over SO(3) — what Eigen::umeyama(with_scaling=false) returns, SVD with the
// det sign fix — via Horn's quaternion: the top eigenvector of the symmetric traceless
// 4x4 N(S) of the centred cross-covariance S[r][c] = sum (s_r - ms_r)(d_c - md_c).
#pragma once
#include "common.hpp"

namespace pk_rigid {

// Jacobi eigen-decomposition of a symmetric 4x4 (a, in place) -> eigenvector of the
// largest eigenvalue in q.
__host__ __device__ inline void top_eigvec4(double a[4][4], double q[4]) {
  double v[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 12; ++sweep) {
    double off = 0.0;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int r = p + 1; r < 4; ++r) off += a[p][r] * a[p][r];
    if (off < 1e-30 * (a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2] + a[3][3] * a[3][3]) + 1e-300)
      break;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int r = p + 1; r < 4; ++r) {
        const double apr = a[p][r];
        if (apr == 0.0) continue;
        const double theta = (a[r][r] - a[p][p]) / (2.0 * apr);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // A <- J^T A J
          const double akp = a[k][p], akr = a[k][r];
          a[k][p] = c * akp - s * akr;
          a[k][r] = s * akp + c * akr;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double apk = a[p][k], ark = a[r][k];
          a[p][k] = c * apk - s * ark;
          a[r][k] = s * apk + c * ark;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double vkp = v[k][p], vkr = v[k][r];
          v[k][p] = c * vkp - s * vkr;
          v[k][r] = s * vkp + c * vkr;
        }
      }
    }
  }
  double best = a[0][0];
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = v[k][0];
#pragma unroll
  for (int m = 1; m < 4; ++m) {
    const bool take = a[m][m] > best;  // static indices only (no scratch)
    best = take ? a[m][m] : best;
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = take ? v[k][m] : q[k];
  }
}

// 3 x 3 determinant of rows (a, b, c)
__host__ __device__ __forceinline__ double det3(double a0, double a1, double a2, double b0, double b1, double b2, double c0,
                                       double c1, double c2) {
  return a0 * (b1 * c2 - b2 * c1) - a1 * (b0 * c2 - b2 * c0) + a2 * (b0 * c1 - b1 * c0);
}

// Top eigenvector of Horn's traceless symmetric N(S) the QCP way (Theobald 2005): the largest
// root of det(N - l I) = l^4 + c2 l^2 + c1 l + c0 (c2 = -2 |S|_F^2, c1 = -8 det S, c0 = det N)
// by Newton from the upper bound |S|_F sqrt(3) >= the nuclear norm of S >= l_max (monotone
// from above), then the eigenvector as the largest column of adj(N - l I). Returns false when
// that column is tiny relative to the scale (a near-multiple top eigenvalue: 4 draws with a
// repeated or collinear correspondence), where the caller falls back to Jacobi.
__host__ __device__ inline bool top_eigvec4_qcp(const double N[4][4], const double S[3][3], double q[4]) {
  double f2 = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) f2 += S[r][c] * S[r][c];
  if (!(f2 > 0.0)) return false;
  const double c2 = -2.0 * f2;
  const double c1 = -8.0 * det3(S[0][0], S[0][1], S[0][2], S[1][0], S[1][1], S[1][2], S[2][0], S[2][1], S[2][2]);
  // det N by Laplace on 2 x 2 minors of rows (0, 1) and (2, 3)
  const double s01 = N[0][0] * N[1][1] - N[0][1] * N[1][0], s02 = N[0][0] * N[1][2] - N[0][2] * N[1][0];
  const double s03 = N[0][0] * N[1][3] - N[0][3] * N[1][0], s12 = N[0][1] * N[1][2] - N[0][2] * N[1][1];
  const double s13 = N[0][1] * N[1][3] - N[0][3] * N[1][1], s23 = N[0][2] * N[1][3] - N[0][3] * N[1][2];
  const double t01 = N[2][0] * N[3][1] - N[2][1] * N[3][0], t02 = N[2][0] * N[3][2] - N[2][2] * N[3][0];
  const double t03 = N[2][0] * N[3][3] - N[2][3] * N[3][0], t12 = N[2][1] * N[3][2] - N[2][2] * N[3][1];
  const double t13 = N[2][1] * N[3][3] - N[2][3] * N[3][1], t23 = N[2][2] * N[3][3] - N[2][3] * N[3][2];
  const double c0 = s01 * t23 - s02 * t13 + s03 * t12 + s12 * t03 - s13 * t02 + s23 * t01;
  double l = sqrt(3.0 * f2);
  for (int it = 0; it < 60; ++it) {
    const double l2 = l * l;
    const double p = (l2 + c2) * l2 + c1 * l + c0;
    const double dp = (4.0 * l2 + 2.0 * c2) * l + c1;
    if (!(dp > 0.0)) break;
    const double nl = l - p / dp;
    if (!(fabs(nl - l) > 1e-15 * l)) {
      l = nl;
      break;
    }
    l = nl;
  }
  // adjugate of M = N - l I: column j = cofactors C_ij (M symmetric)
  double m[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) m[r][c] = N[r][c] - (r == c ? l : 0.0);
  double best = -1.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // minor without row i, column j
      double a[3][3];
      int rr = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r == i) continue;
        int cc = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c == j) continue;
          a[rr][cc] = m[r][c];
          ++cc;
        }
        ++rr;
      }
      const double d = det3(a[0][0], a[0][1], a[0][2], a[1][0], a[1][1], a[1][2], a[2][0], a[2][1], a[2][2]);
      v[i] = ((i + j) & 1) ? -d : d;
    }
    const double nv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    const bool take = nv > best;
    best = take ? nv : best;
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = take ? v[i] : q[i];
  }
  // |adj| ~ product of the three eigen-gaps (<= (2 l)^3): tiny means a near-multiple root
  const double scale = 8.0 * l * l * l;
  return best > 1e-16 * scale * scale;
}

// R (row-major) and t with d ≈ R s + t from the centred cross-covariance S (any positive
// scale) and the two centroids.
__host__ __device__ inline void rigid_from_cov(const double S[3][3], const double ms[3], const double md[3], double R[9],
                                      double t[3]) {
  const double Sxx = S[0][0], Sxy = S[0][1], Sxz = S[0][2];
  const double Syx = S[1][0], Syy = S[1][1], Syz = S[1][2];
  const double Szx = S[2][0], Szy = S[2][1], Szz = S[2][2];
  double N[4][4] = {
      {Sxx + Syy + Szz, Syz - Szy, Szx - Sxz, Sxy - Syx},
      {Syz - Szy, Sxx - Syy - Szz, Sxy + Syx, Szx + Sxz},
      {Szx - Sxz, Sxy + Syx, -Sxx + Syy - Szz, Syz + Szy},
      {Sxy - Syx, Szx + Sxz, Syz + Szy, -Sxx - Syy + Szz}};
  double q[4];
  if (!top_eigvec4_qcp(N, S, q)) top_eigvec4(N, q);  // (near-)degenerate top eigenvalue: Jacobi
  const double nq = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double w = q[0] / nq, x = q[1] / nq, y = q[2] / nq, z = q[3] / nq;
  R[0] = w * w + x * x - y * y - z * z;
  R[1] = 2.0 * (x * y - w * z);
  R[2] = 2.0 * (x * z + w * y);
  R[3] = 2.0 * (x * y + w * z);
  R[4] = w * w - x * x + y * y - z * z;
  R[5] = 2.0 * (y * z - w * x);
  R[6] = 2.0 * (x * z - w * y);
  R[7] = 2.0 * (y * z + w * x);
  R[8] = w * w - x * x - y * y + z * z;
#pragma unroll
  for (int r = 0; r < 3; ++r) t[r] = md[r] - ((R[3 * r] * ms[0] + R[3 * r + 1] * ms[1]) + R[3 * r + 2] * ms[2]);
}

// Rigid fit of n = 4 pairs: R (row-major) and t with d ≈ R s + t.
__device__ inline void rigid_fit4(const double s[4][3], const double d[4][3], double R[9], double t[3]) {
  double ms[3] = {0, 0, 0}, md[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      ms[c] += s[k][c];
      md[c] += d[k][c];
    }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    ms[c] *= 0.25;
    md[c] *= 0.25;
  }
  double S[3][3] = {};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) S[r][c] += (s[k][r] - ms[r]) * (d[k][c] - md[c]);
  rigid_from_cov(S, ms, md, R, t);
}

}  // namespace pk_rigid
