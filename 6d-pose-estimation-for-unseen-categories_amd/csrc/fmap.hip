// H9 — regularized functional-map solve (modeling/dpfm.py:154-195, RegularizedFMNet):
//   for every crop b and row i:  M_i = AAt_b + lambda * diag(D_b[i, :])
//                                C_b[i, :] = (M_i^{-1} (BAt_b)[i, :]^T)^T
// The reference runs 30 sequential batched torch.inverse calls (LU, partial pivoting)
// plus a bmm; here every (b, i) system is one wave: Gauss-Jordan elimination with
// partial pivoting in fp64 (first maximal |pivot|, like LAPACK idamax), lanes = rows,
// up to two right-hand sides. Backward (x = M^{-1} v, M symmetric):
//   w = M^{-1} g;  dL/dv = w;  dL/dAAt += -w x^T  (per (b, i) slab, summed by the caller).
#include "common.hpp"

namespace {

constexpr int kN = 30;  // n_fmap (config/dpfm_orig.yaml:2) — checked on the host

template <int NRHS>
__device__ __forceinline__ void gj_solve(double (&row)[kN + NRHS], int lane, int& var) {
  bool used = lane >= kN;  // rows beyond 30 never pivot
  var = -1;
#pragma unroll
  for (int k = 0; k < kN; ++k) {
    // pivot: max |row[k]| over unused rows, lowest row index on ties
    const double a = used ? -1.0 : fabs(row[k]);
    uint32_t key_hi = (uint32_t)(__double_as_longlong(a) >> 32);
    if (used) key_hi = 0u;
    const uint32_t mhi = pk::wave_max_u32_s(key_hi);
    const uint32_t lo = (uint32_t)(__double_as_longlong(a) & 0xffffffffull);
    const uint32_t mlo = pk::wave_max_u32_s((!used && key_hi == mhi) ? lo : 0u);
    const bool cand = !used && key_hi == mhi && lo == mlo;
    const uint64_t bal = __ballot(cand);
    const int p = bal ? (__ffsll((unsigned long long)bal) - 1) : k;
    // broadcast the pivot row
    double prow[kN + NRHS];
#pragma unroll
    for (int j = 0; j < kN + NRHS; ++j) {
      const long long bits = __double_as_longlong(row[j]);
      const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)(bits >> 32), p);
      const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)(bits & 0xffffffff), p);
      prow[j] = __longlong_as_double(((long long)h << 32) | l);
    }
    const double inv = 1.0 / prow[k];
    if (lane == p) {
#pragma unroll
      for (int j = 0; j < kN + NRHS; ++j) row[j] = prow[j] * inv;
      used = true;
      var = k;
    } else {
      const double f = row[k] * inv;
#pragma unroll
      for (int j = 0; j < kN + NRHS; ++j) row[j] = fma(-f, prow[j], row[j]);
    }
  }
}

__device__ __forceinline__ double bcast_from_var(double v, int var_owner_lane) {
  const long long bits = __double_as_longlong(v);
  const uint32_t h = (uint32_t)__builtin_amdgcn_readlane((int)(bits >> 32), var_owner_lane);
  const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)(bits & 0xffffffff), var_owner_lane);
  return __longlong_as_double(((long long)h << 32) | l);
}

// grid (ceil(B*30/4)), block 256: one wave per (b, i).
template <bool BWD>
__global__ __launch_bounds__(256) void fmap_solve_kernel(const float* __restrict__ AAt,
                                                         const float* __restrict__ BAt,
                                                         const float* __restrict__ D, float lambda, int B,
                                                         const float* __restrict__ G,
                                                         float* __restrict__ C,
                                                         float* __restrict__ dBAt,
                                                         float* __restrict__ dAAt_part) {
  constexpr int NRHS = BWD ? 2 : 1;
  const int w = blockIdx.x * 4 + pk::wave_id();
  if (w >= B * kN) return;
  const int b = w / kN, i = w % kN;
  const int lane = pk::lane_id();
  const float* __restrict__ Ab = AAt + (int64_t)b * kN * kN;
  double row[kN + NRHS];
  const double reg = lane < kN ? (double)lambda * (double)D[((int64_t)b * kN + i) * kN + lane] : 0.0;
#pragma unroll
  for (int j = 0; j < kN; ++j) {
    const double a = lane < kN ? (double)Ab[lane * kN + j] : 0.0;
    row[j] = j == lane ? a + reg : a;  // static index: no scratch
  }
  row[kN] = lane < kN ? (double)BAt[((int64_t)b * kN + i) * kN + lane] : 0.0;
  if (BWD) row[kN + 1] = lane < kN ? (double)G[((int64_t)b * kN + i) * kN + lane] : 0.0;
  int var;
  gj_solve<NRHS>(row, lane, var);
  // lane with var == k holds x_k (row[kN]) and w_k (row[kN+1])
  const int64_t o = ((int64_t)b * kN + i) * kN;
  if (!BWD) {
    if (var >= 0) C[o + var] = (float)row[kN];
  } else {
    if (var >= 0) dBAt[o + var] = (float)row[kN + 1];
    // owner lane of each variable c
    float* __restrict__ slab = dAAt_part + ((int64_t)b * kN + i) * kN * kN;
    const double wr = row[kN + 1];
#pragma unroll
    for (int c = 0; c < kN; ++c) {
      const uint64_t own = __ballot(var == c);
      const int ol = own ? (__ffsll((unsigned long long)own) - 1) : 0;
      const double xc = bcast_from_var(row[kN], ol);
      if (var >= 0) slab[var * kN + c] = (float)(-wr * xc);
    }
  }
}

}  // namespace

extern "C" int pk_fmap_solve(const float* AAt, const float* BAt, const float* D, float lambda, int B, int K,
                             float* C, void* stream) {
  PK_REQUIRE(B >= 0 && K == kN);
  if (B == 0) return PK_OK;
  PK_REQUIRE(AAt && BAt && D && C);
  hipLaunchKernelGGL(fmap_solve_kernel<false>, dim3((B * kN + 3) / 4), dim3(256), 0, pk::as_stream(stream),
                     AAt, BAt, D, lambda, B, nullptr, C, nullptr, nullptr);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_fmap_solve_backward(const float* AAt, const float* BAt, const float* D, float lambda,
                                      int B, int K, const float* G, float* dBAt, float* dAAt_part,
                                      void* stream) {
  PK_REQUIRE(B >= 0 && K == kN);
  if (B == 0) return PK_OK;
  PK_REQUIRE(AAt && BAt && D && G && dBAt && dAAt_part);
  hipLaunchKernelGGL(fmap_solve_kernel<true>, dim3((B * kN + 3) / 4), dim3(256), 0, pk::as_stream(stream),
                     AAt, BAt, D, lambda, B, G, nullptr, dBAt, dAAt_part);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// ---------------------------------------------------------------------------------
// H9 resolvent mask (upstream dpfm/utils.py::get_mask, called per crop at
// modeling/dpfm.py:171-176 and models/dpfm.py:76) for every crop in one launch:
//   s = max(max evals1, max evals2); g1 = (evals1 / s)^gamma; g2 = (evals2 / s)^gamma
//   D[j][i] = (g2_j / (g2_j^2 + 1) - g1_i / (g1_i^2 + 1))^2 + (1 / (g2_j^2 + 1) - 1 / (g1_i^2 + 1))^2
// One workgroup per crop, one thread per (j, i). gamma = 0.5 takes sqrt (as aten's pow).
namespace {

__global__ __launch_bounds__(1024) void resolvent_mask_kernel(const float* __restrict__ ev1, int ld1,
                                                              const float* __restrict__ ev2, int ld2, int K,
                                                              float gamma, float* __restrict__ D) {
  __shared__ float red[16];
  __shared__ float g1s[64], g2s[64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* e1 = ev1 + (int64_t)b * ld1;
  const float* e2 = ev2 + (int64_t)b * ld2;
  float mx = -__builtin_huge_valf();
  if (tid < K) mx = fmaxf(e1[tid], e2[tid]);
  for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  float s = red[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) s = fmaxf(s, red[w]);
  if (tid < K) {
    const float a = e1[tid] / s, c = e2[tid] / s;
    g1s[tid] = gamma == 0.5f ? sqrtf(a) : powf(a, gamma);
    g2s[tid] = gamma == 0.5f ? sqrtf(c) : powf(c, gamma);
  }
  __syncthreads();
  if (tid < K * K) {
    const int j = tid / K, i = tid - j * K;
    const float g1 = g1s[i], g2 = g2s[j];
    const float q1 = g1 * g1 + 1.f, q2 = g2 * g2 + 1.f;
    const float re = g2 / q2 - g1 / q1;
    const float im = 1.f / q2 - 1.f / q1;
    D[(int64_t)b * K * K + tid] = re * re + im * im;
  }
}

}  // namespace

extern "C" int pk_resolvent_mask(const float* evals1, int ld1, const float* evals2, int ld2, int B, int K, float gamma,
                                 float* D, void* stream) {
  PK_REQUIRE(B >= 0 && K > 0 && K <= 32 && ld1 >= K && ld2 >= K);
  if (B == 0) return PK_OK;
  PK_REQUIRE(evals1 && evals2 && D);
  hipLaunchKernelGGL(resolvent_mask_kernel, dim3(B), dim3(1024), 0, pk::as_stream(stream), evals1, ld1, evals2, ld2, K,
                     gamma, D);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
