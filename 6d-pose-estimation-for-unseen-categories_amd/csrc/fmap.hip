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
