// H14 — pose metrics of scripts/test_RANSAC.py:77-81, 154-238, batched over crops, fp64.
//
//  per point x of the CAD model (pose_2_R_t / transform, :144-160):
//    add_i      = ||(R_e x + t_e) - (R_g x + t_g)||              -> ADD = mean_i   (add, :162-173)
//    xyz_i[r]   = |(R_e[r]·x + t_e[r]) - (R_g[r]·x + t_g[r])|     (compute_add_score, :186-201:
//                 one 1-D projection per row r, the reference's "xyz direction" quirk)
//    adds_i[r]  = min_j |e_i[r] - g_j[r]| with e/g the per-row projections of the
//                 estimated / GT pose (compute_adds_score, :203-222: sklearn KDTree 1-NN on
//                 1-D data, reported as sqrt(d*d))
//  Outputs per crop: out[b] = {ADD, mean xyz[0..2], mean adds[0..2]} (means in fp64; the
//  reference's np.mean uses pairwise summation, so results agree to rounding).
//  A crop with more points than the capacity nmax is not evaluated: its outputs are NaN.
#include "common.hpp"

namespace {

__device__ __forceinline__ double proj(const double* T, int r, double x, double y, double z) {
  // R[i].reshape((1,3)).dot(pts.T) + t[i]
  return ((T[4 * r] * x + T[4 * r + 1] * y) + T[4 * r + 2] * z) + T[4 * r + 3];
}

// grid (ceil(nmax/256), B), block 256: per-point ADD and per-row distances; also caches the
// GT projections g[b, r, i] used by the ADD-S pass.
__global__ __launch_bounds__(256) void pm_point_kernel(const double* __restrict__ cad,
                                                       const int64_t* __restrict__ off,
                                                       const double* __restrict__ Te,
                                                       const double* __restrict__ Tg, int nmax,
                                                       double* __restrict__ per /*[B,7,nmax]*/,
                                                       double* __restrict__ g /*[B,3,nmax]*/,
                                                       double* __restrict__ e /*[B,3,nmax]*/) {
  const int b = blockIdx.y;
  const int64_t o = off[b];
  const int n = (int)(off[b + 1] - o);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || n > nmax) return;
  const double* p = cad + 3 * (o + i);
  const double x = p[0], y = p[1], z = p[2];
  const double* te = Te + 16 * b;
  const double* tg = Tg + 16 * b;
  double d2 = 0.0;
  for (int r = 0; r < 3; ++r) {
    const double pe = proj(te, r, x, y, z), pg = proj(tg, r, x, y, z);
    const double d = pe - pg;
    d2 = r == 0 ? d * d : d2 + d * d;
    per[((int64_t)b * 7 + 1 + r) * nmax + i] = sqrt(d * d);
    g[((int64_t)b * 3 + r) * nmax + i] = pg;
    e[((int64_t)b * 3 + r) * nmax + i] = pe;
  }
  per[((int64_t)b * 7 + 0) * nmax + i] = sqrt(d2);
}

// grid (ceil(nmax/256), 3, B): 1-D nearest GT projection for every estimated projection.
__global__ __launch_bounds__(256) void pm_adds_kernel(const int64_t* __restrict__ off, int nmax,
                                                      const double* __restrict__ g, const double* __restrict__ e,
                                                      double* __restrict__ per) {
  __shared__ double tile[1024];
  const int b = blockIdx.z, r = blockIdx.y;
  const int n = (int)(off[b + 1] - off[b]);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x * 256 >= n || n > nmax) return;
  const double ei = i < n ? e[((int64_t)b * 3 + r) * nmax + i] : 0.0;
  double best = __builtin_huge_val();
  for (int t0 = 0; t0 < n; t0 += 1024) {
    const int tn = min(1024, n - t0);
    __syncthreads();
    for (int k = threadIdx.x; k < tn; k += 256) tile[k] = g[((int64_t)b * 3 + r) * nmax + t0 + k];
    __syncthreads();
    for (int k = 0; k < tn; ++k) {
      const double d = ei - tile[k];
      best = fmin(best, d * d);
    }
  }
  if (i < n) per[((int64_t)b * 7 + 4 + r) * nmax + i] = sqrt(best);
}

// grid (7, B), block 256: means.
__global__ __launch_bounds__(256) void pm_mean_kernel(const int64_t* __restrict__ off, int nmax,
                                                      const double* __restrict__ per, double* __restrict__ out) {
  __shared__ double ws[4];
  const int b = blockIdx.y, q = blockIdx.x;
  const int n = (int)(off[b + 1] - off[b]);
  if (n > nmax) {  // over capacity: not evaluated
    if (threadIdx.x == 0) out[b * 7 + q] = __builtin_nan("");
    return;
  }
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += per[((int64_t)b * 7 + q) * nmax + i];
  s = pk::wave_sum_f64(s);
  if (pk::lane_id() == 0) ws[pk::wave_id()] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[b * 7 + q] = n > 0 ? ((ws[0] + ws[1]) + (ws[2] + ws[3])) / (double)n : 0.0;
}

}  // namespace

extern "C" int pk_pose_metrics(const double* cad, const int64_t* off, int B, int nmax, const double* T_est,
                               const double* T_gt, double* work, double* out, void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(cad && off && T_est && T_gt && work && out);
  hipStream_t s = pk::as_stream(stream);
  double* per = work;                            // [B, 7, nmax]
  double* g = work + (int64_t)B * 7 * nmax;      // [B, 3, nmax]
  double* e = g + (int64_t)B * 3 * nmax;         // [B, 3, nmax]
  if (nmax > 0) {
    hipLaunchKernelGGL(pm_point_kernel, dim3((nmax + 255) / 256, B), dim3(256), 0, s, cad, off, T_est, T_gt, nmax,
                       per, g, e);
    PK_CHECK_LAUNCH();
    hipLaunchKernelGGL(pm_adds_kernel, dim3((nmax + 255) / 256, 3, B), dim3(256), 0, s, off, nmax, g, e, per);
    PK_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(pm_mean_kernel, dim3(7, B), dim3(256), 0, s, off, nmax, per, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
