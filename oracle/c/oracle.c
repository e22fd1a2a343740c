/* Plain-C restatements of the sequential / quadratic hot-path pieces.
 * TEST INFRASTRUCTURE ONLY: used by tests/ (parity at sizes the Python oracle is
 * too slow for) and by bench.py's cpu_baseline leg (kind "port"). Compiled with
 * -O2 -ffp-contract=off so every product/sum is rounded like numpy / torch-CPU.
 *
 *  oc_fps          upstream DPFM farthest_point_sample,
 *                  called at dataset/object.py:145-148
 *  oc_ball_query   dataset/object.py:281-288 find_positives (+ :311-317 get_overlap)
 *  oc_ransac       scripts/test_RANSAC.py:288-310 -> Open3D 0.17
 *                  RegistrationRANSACBasedOnCorrespondence with
 *                  Eigen::umeyama(with_scaling=false); OpenMP over hypotheses
 *  oc_hyp_index    the documented hypothesis hash of include/posekern.h
 *  oc_icp          scripts/test_RANSAC.py:436-446 -> Open3D 0.17 RegistrationICP,
 *                  point-to-point (semantics of csrc/icp.hip, brute-force nearest target)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- FPS */
int oc_fps(const float* xyz /* [n,3] */, int n, int start, int npoint, int64_t* out) {
  if (n <= 0 || npoint <= 0) return 0;
  float* dist = (float*)malloc(sizeof(float) * (size_t)n);
  if (!dist) return -1;
  for (int i = 0; i < n; ++i) dist[i] = 1e10f;
  int far = start;
  for (int it = 0; it < npoint; ++it) {
    out[it] = far;
    const float cx = xyz[3 * far], cy = xyz[3 * far + 1], cz = xyz[3 * far + 2];
    float best = -1.f;
    int besti = 0;
    for (int i = 0; i < n; ++i) {
      const float dx = xyz[3 * i] - cx, dy = xyz[3 * i + 1] - cy, dz = xyz[3 * i + 2] - cz;
      const float d = (dx * dx + dy * dy) + dz * dz;
      if (d < dist[i]) dist[i] = d;
      if (dist[i] > best) { best = dist[i]; besti = i; } /* first maximal index */
    }
    far = besti;
  }
  free(dist);
  return 0;
}

/* ---------------------------------------------------------------- ball query */
/* Returns the number of pairs; writes up to cap (i, j) pairs in row-major order. */
int64_t oc_ball_query(const double* pc1, int n1, const double* pc2, int n2, double r,
                      int64_t* pairs, int64_t cap, int8_t* ov12, int8_t* ov21) {
  int64_t cnt = 0;
  if (ov12) memset(ov12, 0, (size_t)n1);
  if (ov21) memset(ov21, 0, (size_t)n2);
  for (int i = 0; i < n1; ++i) {
    for (int j = 0; j < n2; ++j) {
      const double dx = pc1[3 * i] - pc2[3 * j];
      const double dy = pc1[3 * i + 1] - pc2[3 * j + 1];
      const double dz = pc1[3 * i + 2] - pc2[3 * j + 2];
      const double s = (dx * dx + dy * dy) + dz * dz;
      if (sqrt(s) <= r) {
        if (cnt < cap) { pairs[2 * cnt] = i; pairs[2 * cnt + 1] = j; }
        if (ov12) ov12[i] = 1;
        if (ov21) ov21[j] = 1;
        ++cnt;
      }
    }
  }
  return cnt;
}

/* ---------------------------------------------------------------- hypothesis hash */
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
/* Hypothesis h, draw j (0..3) -> correspondence row in [0, n). */
int32_t oc_hyp_index(uint64_t seed, int64_t h, int j, int32_t n) {
  const uint64_t x = splitmix64(seed ^ splitmix64((uint64_t)h * 4u + (uint64_t)j));
  return (int32_t)(x % (uint64_t)n);
}

/* ---------------------------------------------------------------- Umeyama */
/* One-sided Jacobi SVD of a 3x3 (columns orthogonalised), Eigen-umeyama semantics:
 * R = U diag(1,1,det(U)det(V)<0 ? -1 : 1) V^T, t = mu_d - R mu_s. */
static void svd3(const double A[9], double U[9], double S[3], double V[9]) {
  double a[9];
  memcpy(a, A, sizeof(a));
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int k = 0; k < 3; ++k) {
          alpha += a[3 * k + p] * a[3 * k + p];
          beta += a[3 * k + q] * a[3 * k + q];
          gamma += a[3 * k + p] * a[3 * k + q];
        }
        off = fmax(off, fabs(gamma) / (sqrt(alpha * beta) + 1e-300));
        if (fabs(gamma) < 1e-300) continue;
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int k = 0; k < 3; ++k) {
          const double x = a[3 * k + p], y = a[3 * k + q];
          a[3 * k + p] = c * x - s * y;
          a[3 * k + q] = s * x + c * y;
          const double vx = V[3 * k + p], vy = V[3 * k + q];
          V[3 * k + p] = c * vx - s * vy;
          V[3 * k + q] = s * vx + c * vy;
        }
      }
    if (off < 1e-15) break;
  }
  for (int j = 0; j < 3; ++j) {
    S[j] = sqrt(a[j] * a[j] + a[3 + j] * a[3 + j] + a[6 + j] * a[6 + j]);
  }
  /* U columns = a columns / S; complete degenerate columns with cross products. */
  int order[3] = {0, 1, 2};
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (S[order[j]] > S[order[i]]) { int t = order[i]; order[i] = order[j]; order[j] = t; }
  double Uc[3][3];
  for (int c = 0; c < 3; ++c) {
    const int j = order[c];
    if (S[j] > 1e-12 * (S[order[0]] + 1e-300)) {
      for (int k = 0; k < 3; ++k) Uc[c][k] = a[3 * k + j] / S[j];
    } else if (c == 0) { /* rank 0 (all-zero sigma): U = I */
      Uc[0][0] = 1.0; Uc[0][1] = 0.0; Uc[0][2] = 0.0;
    } else if (c == 2) {
      Uc[2][0] = Uc[0][1] * Uc[1][2] - Uc[0][2] * Uc[1][1];
      Uc[2][1] = Uc[0][2] * Uc[1][0] - Uc[0][0] * Uc[1][2];
      Uc[2][2] = Uc[0][0] * Uc[1][1] - Uc[0][1] * Uc[1][0];
    } else { /* rank <= 1: any orthonormal completion */
      double e[3] = {0, 0, 0};
      int m = fabs(Uc[0][0]) < 0.5 ? 0 : (fabs(Uc[0][1]) < 0.5 ? 1 : 2);
      e[m] = 1.0;
      double d = e[0] * Uc[0][0] + e[1] * Uc[0][1] + e[2] * Uc[0][2];
      double n2 = 0;
      for (int k = 0; k < 3; ++k) { Uc[1][k] = e[k] - d * Uc[0][k]; n2 += Uc[1][k] * Uc[1][k]; }
      for (int k = 0; k < 3; ++k) Uc[1][k] /= sqrt(n2);
    }
  }
  double Vs[9];
  memcpy(Vs, V, sizeof(Vs));
  double Ss[3];
  for (int c = 0; c < 3; ++c) {
    Ss[c] = S[order[c]];
    for (int k = 0; k < 3; ++k) {
      U[3 * k + c] = Uc[c][k];
      V[3 * k + c] = Vs[3 * k + order[c]];
    }
  }
  memcpy(S, Ss, sizeof(Ss));
}

static double det3(const double M[9]) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
         M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* src/dst: the n matched points, [n,3]. Writes R (row-major 3x3) and t. */
void oc_umeyama(const double* src, const double* dst, int n, double R[9], double t[3]) {
  double ms[3] = {0, 0, 0}, md[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) { ms[k] += src[3 * i + k]; md[k] += dst[3 * i + k]; }
  const double inv = 1.0 / n;
  for (int k = 0; k < 3; ++k) { ms[k] *= inv; md[k] *= inv; }
  double sig[9] = {0};
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) sig[3 * r + c] += (dst[3 * i + r] - md[r]) * (src[3 * i + c] - ms[c]);
  for (int k = 0; k < 9; ++k) sig[k] *= inv;
  double U[9], S[3], V[9];
  svd3(sig, U, S, V);
  const double dsgn = (det3(U) * det3(V) < 0) ? -1.0 : 1.0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      R[3 * r + c] = U[3 * r + 0] * V[3 * c + 0] + U[3 * r + 1] * V[3 * c + 1] + dsgn * U[3 * r + 2] * V[3 * c + 2];
  for (int r = 0; r < 3; ++r) t[r] = md[r] - (R[3 * r] * ms[0] + R[3 * r + 1] * ms[1] + R[3 * r + 2] * ms[2]);
}

/* ---------------------------------------------------------------- RANSAC */
/* Evaluates H hypotheses (ransac_n = 4, drawn by oc_hyp_index or taken from hyps[H*4])
 * and returns the best by (fitness desc, rmse asc, hypothesis index asc).
 * out: T (4x4 row-major), out_stats: fitness, rmse, best index. */
int oc_ransac(const double* src, const double* dst, const int32_t* corres /* [n,2] */, int n,
              const int32_t* hyps /* [H,4] or NULL */, uint64_t seed, int64_t H, double max_dist,
              double* T, double* out_stats) {
  for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  out_stats[0] = 0.0; out_stats[1] = 0.0; out_stats[2] = -1.0;
  if (n < 4 || max_dist <= 0.0 || H <= 0) return 0;
  const double max_d2 = max_dist * max_dist;
  double best_f = -1.0, best_r = 0.0;
  int64_t best_h = -1;
  double best_R[9], best_t[3];
#pragma omp parallel
  {
    double lf = -1.0, lr = 0.0;
    int64_t lh = -1;
    double lR[9], lt[3];
#pragma omp for schedule(static)
    for (int64_t h = 0; h < H; ++h) {
      double s4[12], d4[12];
      for (int j = 0; j < 4; ++j) {
        const int32_t c = hyps ? hyps[4 * h + j] : oc_hyp_index(seed, h, j, n);
        memcpy(s4 + 3 * j, src + 3 * (int64_t)corres[2 * c], 3 * sizeof(double));
        memcpy(d4 + 3 * j, dst + 3 * (int64_t)corres[2 * c + 1], 3 * sizeof(double));
      }
      double R[9], t[3];
      oc_umeyama(s4, d4, 4, R, t);
      int good = 0;
      double err = 0.0;
      for (int i = 0; i < n; ++i) {
        const double* s = src + 3 * (int64_t)corres[2 * i];
        const double* d = dst + 3 * (int64_t)corres[2 * i + 1];
        const double ex = ((R[0] * s[0] + R[1] * s[1]) + R[2] * s[2]) + t[0] - d[0];
        const double ey = ((R[3] * s[0] + R[4] * s[1]) + R[5] * s[2]) + t[1] - d[1];
        const double ez = ((R[6] * s[0] + R[7] * s[1]) + R[8] * s[2]) + t[2] - d[2];
        const double d2 = (ex * ex + ey * ey) + ez * ez;
        if (d2 < max_d2) { ++good; err += d2; }
      }
      const double f = good ? (double)good / n : 0.0;
      const double r = good ? sqrt(err / good) : 0.0;
      if (f > lf || (f == lf && r < lr)) { lf = f; lr = r; lh = h; memcpy(lR, R, sizeof(lR)); memcpy(lt, t, sizeof(lt)); }
    }
#pragma omp critical
    {
      if (lh >= 0 && (lf > best_f || (lf == best_f && (lr < best_r || (lr == best_r && lh < best_h))))) {
        best_f = lf; best_r = lr; best_h = lh; memcpy(best_R, lR, sizeof(lR)); memcpy(best_t, lt, sizeof(lt));
      }
    }
  }
  if (best_h >= 0) {
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) T[4 * r + c] = best_R[3 * r + c];
      T[4 * r + 3] = best_t[r];
    }
    out_stats[0] = best_f; out_stats[1] = best_r; out_stats[2] = (double)best_h;
  }
  return 0;
}

/* Open3D 0.17 RegistrationRANSACBasedOnCorrespondence's per-iteration cost shape, for the
 * CPU baseline (bench.py cpu_ransac_baseline): like oc_ransac, but each hypothesis copies
 * and transforms the WHOLE source cloud (V1 points; Open3D: `pcd = source;
 * pcd.Transform(T)`) before scoring the correspondences on the transformed copy. Same
 * selection rule and draws as oc_ransac. */
int oc_ransac_o3d(const double* src, int V1, const double* dst, const int32_t* corres, int n,
                  const int32_t* hyps, uint64_t seed, int64_t H, double max_dist, double* T, double* out_stats) {
  for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  out_stats[0] = 0.0; out_stats[1] = 0.0; out_stats[2] = -1.0;
  if (n < 4 || max_dist <= 0.0 || H <= 0) return 0;
  const double max_d2 = max_dist * max_dist;
  double best_f = -1.0, best_r = 0.0;
  int64_t best_h = -1;
  double best_R[9], best_t[3];
#pragma omp parallel
  {
    double lf = -1.0, lr = 0.0;
    int64_t lh = -1;
    double lR[9], lt[3];
    double* pcd = (double*)malloc(sizeof(double) * 3 * (size_t)V1);
#pragma omp for schedule(static)
    for (int64_t h = 0; h < H; ++h) {
      double s4[12], d4[12];
      for (int j = 0; j < 4; ++j) {
        const int32_t c = hyps ? hyps[4 * h + j] : oc_hyp_index(seed, h, j, n);
        memcpy(s4 + 3 * j, src + 3 * (int64_t)corres[2 * c], 3 * sizeof(double));
        memcpy(d4 + 3 * j, dst + 3 * (int64_t)corres[2 * c + 1], 3 * sizeof(double));
      }
      double R[9], t[3];
      oc_umeyama(s4, d4, 4, R, t);
      for (int i = 0; i < V1; ++i) {
        const double* s = src + 3 * (int64_t)i;
        for (int r = 0; r < 3; ++r) pcd[3 * i + r] = ((R[3 * r] * s[0] + R[3 * r + 1] * s[1]) + R[3 * r + 2] * s[2]) + t[r];
      }
      int good = 0;
      double err = 0.0;
      for (int i = 0; i < n; ++i) {
        const double* p = pcd + 3 * (int64_t)corres[2 * i];
        const double* d = dst + 3 * (int64_t)corres[2 * i + 1];
        const double ex = p[0] - d[0], ey = p[1] - d[1], ez = p[2] - d[2];
        const double d2 = (ex * ex + ey * ey) + ez * ez;
        if (d2 < max_d2) { ++good; err += d2; }
      }
      const double f = good ? (double)good / n : 0.0;
      const double r = good ? sqrt(err / good) : 0.0;
      if (f > lf || (f == lf && r < lr)) { lf = f; lr = r; lh = h; memcpy(lR, R, sizeof(lR)); memcpy(lt, t, sizeof(lt)); }
    }
    free(pcd);
#pragma omp critical
    {
      if (lh >= 0 && (lf > best_f || (lf == best_f && (lr < best_r || (lr == best_r && lh < best_h))))) {
        best_f = lf; best_r = lr; best_h = lh; memcpy(best_R, lR, sizeof(lR)); memcpy(best_t, lt, sizeof(lt));
      }
    }
  }
  if (best_h >= 0) {
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) T[4 * r + c] = best_R[3 * r + c];
      T[4 * r + 3] = best_t[r];
    }
    out_stats[0] = best_f; out_stats[1] = best_r; out_stats[2] = (double)best_h;
  }
  return 0;
}

/* ---------------------------------------------------------------- ICP */
/* One evaluation of Open3D's GetRegistrationResultAndCorrespondences: every source point
 * p = T s takes its nearest target point (exact fp64 distance, first index on ties); a pair iff
 * d^2 < r^2. Fills the matched points (p, q) and returns the pair count; *err = sum d^2. */
static int icp_eval(const double* src, int ns, const double* tgt, int nt, const double T[16], double r2,
                    double* mp, double* mq, double* err) {
  int cnt = 0;
  double e = 0.0;
  for (int i = 0; i < ns; ++i) {
    const double* s = src + 3 * (int64_t)i;
    double p[3];
    for (int k = 0; k < 3; ++k) p[k] = ((T[4 * k] * s[0] + T[4 * k + 1] * s[1]) + T[4 * k + 2] * s[2]) + T[4 * k + 3];
    double best = INFINITY;
    int bj = -1;
    for (int j = 0; j < nt; ++j) {
      const double dx = p[0] - tgt[3 * j], dy = p[1] - tgt[3 * j + 1], dz = p[2] - tgt[3 * j + 2];
      const double d2 = (dx * dx + dy * dy) + dz * dz;
      if (d2 < best) { best = d2; bj = j; }
    }
    if (bj >= 0 && best < r2) {
      memcpy(mp + 3 * cnt, p, sizeof(p));
      memcpy(mq + 3 * cnt, tgt + 3 * bj, 3 * sizeof(double));
      e += best;
      ++cnt;
    }
  }
  *err = e;
  return cnt;
}

/* Open3D RegistrationICP loop: result_0 = eval(T0); then up to max_iter times: U = umeyama of the
 * pairs (identity without pairs), T <- U T, result = eval(T), stop when both relative criteria
 * hold. T: 4x4 row-major in/out (init in T_init); stats: fitness, rmse, updates, converged. */
int oc_icp(const double* src, int ns, const double* tgt, int nt, const double* T_init, double max_dist,
           int max_iter, double rel_fit, double rel_rmse, double* T, double* stats) {
  double* mp = (double*)malloc(sizeof(double) * 3 * (size_t)(ns > 0 ? ns : 1));
  double* mq = (double*)malloc(sizeof(double) * 3 * (size_t)(ns > 0 ? ns : 1));
  if (!mp || !mq) { free(mp); free(mq); return -1; }
  memcpy(T, T_init, 16 * sizeof(double));
  const double r2 = max_dist * max_dist;
  double err;
  int cnt = icp_eval(src, ns, tgt, nt, T, r2, mp, mq, &err);
  double fit = (cnt > 0 && ns > 0) ? (double)cnt / ns : 0.0;
  double rmse = cnt > 0 ? sqrt(err / cnt) : 0.0;
  int it = 0, conv = 0;
  for (; it < max_iter; ++it) {
    double U[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    if (cnt > 0) {
      double R[9], t[3];
      oc_umeyama(mp, mq, cnt, R, t);
      for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) U[4 * r + c] = R[3 * r + c];
        U[4 * r + 3] = t[r];
      }
    }
    double Tn[16];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c)
        Tn[4 * r + c] = ((U[4 * r] * T[c] + U[4 * r + 1] * T[4 + c]) + U[4 * r + 2] * T[8 + c]) + U[4 * r + 3] * T[12 + c];
    memcpy(T, Tn, sizeof(Tn));
    const double pf = fit, pr = rmse;
    cnt = icp_eval(src, ns, tgt, nt, T, r2, mp, mq, &err);
    fit = (cnt > 0 && ns > 0) ? (double)cnt / ns : 0.0;
    rmse = cnt > 0 ? sqrt(err / cnt) : 0.0;
    if (fabs(pf - fit) < rel_fit && fabs(pr - rmse) < rel_rmse) { ++it; conv = 1; break; }
  }
  stats[0] = fit; stats[1] = rmse; stats[2] = (double)it; stats[3] = (double)conv;
  free(mp); free(mq);
  return 0;
}
