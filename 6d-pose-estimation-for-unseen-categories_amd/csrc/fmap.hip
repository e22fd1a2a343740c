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
  // every operand load issued before the first use, unconditionally at a clamped lane (round 2's
  // per-element conditional loads were each waited for: 30+ serial memory round trips)
  const bool lv = lane < kN;
  const int lc = lv ? lane : 0;
  float af[kN];
#pragma unroll
  for (int j = 0; j < kN; ++j) af[j] = Ab[lc * kN + j];
  const float dv = D[((int64_t)b * kN + i) * kN + lc];
  const float bv = BAt[((int64_t)b * kN + i) * kN + lc];
  const float gv = BWD ? G[((int64_t)b * kN + i) * kN + lc] : 0.f;
  const double reg = lv ? (double)lambda * (double)dv : 0.0;
#pragma unroll
  for (int j = 0; j < kN; ++j) {
    const double a = lv ? (double)af[j] : 0.0;
    row[j] = j == lane ? a + reg : a;  // static index: no scratch
  }
  row[kN] = lv ? (double)bv : 0.0;
  if (BWD) row[kN + 1] = lv ? (double)gv : 0.0;
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

// ---------------------------------------------------------------------------------
// H9 fmap head around the solve (modeling/dpfm.py:154-176, the batched branch that always
// runs; models/dpfm.py:66-72 for evecs_trans):
//   W = evecs[:, :K] * mass (f32 products, the reference's evecs_trans before its transpose)
//   A = W_x^T F_x, Bm = W_y^T F_y            [K, C] per crop (F = refined features [N, C])
//   AAt = A A^T, BAt = Bm A^T, D = get_mask(evals_x, evals_y)   -> pk_fmap_solve
// Forward in two launches: 128-point chunks of both sides spread over the chip (W and F staged
// through LDS, the chunk's 30 x 32 partial product into a work buffer), then one workgroup per
// crop sums the partials in chunk order and forms the K x K products and the mask;
// backward in two: the K x C gradients of A and Bm (dAAt = the solve backward's per-row slabs
// summed in row order), then dF = (W dA) / (W dBm) per point, written straight into the
// caller's feature-gradient layout. Replaces the evecs * mass products, four batched GEMMs,
// the mask launch and, backward, six GEMMs, the slab sum and the gradient additions.
namespace {

constexpr int kHK = 30, kHC = 32;

struct FeatRef {  // element (b, n, c) at base + b * sb + n * sn + c * sc
  const float* base;
  int64_t sb, sn, sc;
};

constexpr int kPChunk = 128;  // points per partial-projection workgroup
constexpr int kLdF = kHC + 4;  // 16-B aligned feature rows in LDS

// grid (ceil(N1 / 128) + ceil(N2 / 128), B), block 256: the 30 x 32 partial product W^T F of
// one 128-point chunk of one side -> part[b, p] (p < P_x: x side chunk p, else y side).
// Threads 0..239: output (k = tid / 8, channels 4 (tid % 8) .. + 3).
__global__ __launch_bounds__(256) void fmap_head_part_kernel(const float* __restrict__ ex, int ldex,
                                                             const float* __restrict__ mx, const FeatRef fx, int N1,
                                                             const float* __restrict__ ey, int ldey,
                                                             const float* __restrict__ my, const FeatRef fy, int N2,
                                                             int Px, float* __restrict__ part) {
  __shared__ float Ws[kPChunk][kHK + 1];
  __shared__ __attribute__((aligned(16))) float Fs[kPChunk][kLdF];
  const int b = blockIdx.y, p = blockIdx.x, tid = threadIdx.x;
  const bool xs = p < Px;
  const int N = xs ? N1 : N2, lde = xs ? ldex : ldey;
  const float* __restrict__ ev = xs ? ex : ey;
  const float* __restrict__ ms = xs ? mx : my;
  const FeatRef f = xs ? fx : fy;
  const int n0 = (xs ? p : p - Px) * kPChunk;
  const int m = min(kPChunk, N - n0);
  for (int e = tid; e < kPChunk * kHK; e += 256) {
    const int r = e / kHK, kk = e - r * kHK;
    float v = 0.f;
    if (r < m) {
      const int64_t n = (int64_t)b * N + n0 + r;
      v = ev[n * lde + kk] * ms[n];  // f32 product, as evecs[:, :, :k] * mass[:, :, None]
    }
    Ws[r][kk] = v;
  }
  // consecutive threads walk the unit-stride axis of the features (points for channels-first
  // storage, channels for rows), so the staging loads coalesce either way
  const bool pts_fast = f.sn == 1;
  for (int e = tid; e < kPChunk * kHC; e += 256) {
    const int r = pts_fast ? e % kPChunk : e / kHC, cc = pts_fast ? e / kPChunk : e % kHC;
    Fs[r][cc] = r < m ? f.base[(int64_t)b * f.sb + (int64_t)(n0 + r) * f.sn + (int64_t)cc * f.sc] : 0.f;
  }
  __syncthreads();
  if (tid >= kHK * 8) return;
  const int k = tid >> 3, c = (tid & 7) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < m; ++r) {
    const float w = Ws[r][k];
    const float4 x = *reinterpret_cast<const float4*>(&Fs[r][c]);
    acc.x = fmaf(w, x.x, acc.x);
    acc.y = fmaf(w, x.y, acc.y);
    acc.z = fmaf(w, x.z, acc.z);
    acc.w = fmaf(w, x.w, acc.w);
  }
  *reinterpret_cast<float4*>(&part[(((int64_t)b * gridDim.x + p) * kHK + k) * kHC + c]) = acc;
}

// grid (B), block 512: A / Bm = the chunk partials summed in chunk order; AAt, BAt; the mask
__global__ __launch_bounds__(512) void fmap_head_fin_kernel(const float* __restrict__ part, int Px, int P,
                                                            const float* __restrict__ evx, int ldvx,
                                                            const float* __restrict__ evy, int ldvy, float gamma,
                                                            float* __restrict__ A, float* __restrict__ Bm,
                                                            float* __restrict__ AAt, float* __restrict__ BAt,
                                                            float* __restrict__ D) {
  __shared__ float As[kHK][kHC + 1], Bs[kHK][kHC + 1];
  __shared__ float red[8], g1s[kHK], g2s[kHK];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* pb = part + (int64_t)b * P * kHK * kHC;
  for (int e = tid; e < kHK * kHC; e += blockDim.x) {
    const int k = e / kHC, c = e - k * kHC;
    float sa = 0.f, sb = 0.f;
    for (int q = 0; q < Px; ++q) sa += pb[(int64_t)q * kHK * kHC + e];
    for (int q = Px; q < P; ++q) sb += pb[(int64_t)q * kHK * kHC + e];
    As[k][c] = sa;
    Bs[k][c] = sb;
    A[(int64_t)b * kHK * kHC + e] = sa;
    Bm[(int64_t)b * kHK * kHC + e] = sb;
  }
  __syncthreads();
  for (int e = tid; e < kHK * kHK; e += blockDim.x) {
    const int i = e / kHK, j = e - i * kHK;
    float s = 0.f, t = 0.f;
#pragma unroll 8
    for (int c = 0; c < kHC; ++c) {
      s = fmaf(As[i][c], As[j][c], s);
      t = fmaf(Bs[i][c], As[j][c], t);
    }
    AAt[(int64_t)b * kHK * kHK + e] = s;
    BAt[(int64_t)b * kHK * kHK + e] = t;
  }
  // the resolvent mask (resolvent_mask_kernel's arithmetic)
  float mxv = -__builtin_huge_valf();
  if (tid < kHK) mxv = fmaxf(evx[(int64_t)b * ldvx + tid], evy[(int64_t)b * ldvy + tid]);
  for (int off = 32; off >= 1; off >>= 1) mxv = fmaxf(mxv, __shfl_xor(mxv, off));
  if ((tid & 63) == 0) red[tid >> 6] = mxv;
  __syncthreads();
  float s = red[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) s = fmaxf(s, red[w]);
  if (tid < kHK) {
    const float a = evx[(int64_t)b * ldvx + tid] / s, c = evy[(int64_t)b * ldvy + tid] / s;
    g1s[tid] = gamma == 0.5f ? sqrtf(a) : powf(a, gamma);
    g2s[tid] = gamma == 0.5f ? sqrtf(c) : powf(c, gamma);
  }
  __syncthreads();
  for (int e = tid; e < kHK * kHK; e += blockDim.x) {
    const int j = e / kHK, i = e - j * kHK;
    const float g1 = g1s[i], g2 = g2s[j];
    const float q1 = g1 * g1 + 1.f, q2 = g2 * g2 + 1.f;
    const float re = g2 / q2 - g1 / q1;
    const float im = 1.f / q2 - 1.f / q1;
    D[(int64_t)b * kHK * kHK + e] = re * re + im * im;
  }
}

// grid (B), block 512: dAAt = sum_j part[b, j] (row order); dA = (dAAt + dAAt^T) A + dBAt^T Bm;
// dBm = dBAt A.
__global__ __launch_bounds__(512) void fmap_head_grad_kernel(const float* __restrict__ part,
                                                             const float* __restrict__ dBAt,
                                                             const float* __restrict__ A,
                                                             const float* __restrict__ Bm,
                                                             float* __restrict__ dA, float* __restrict__ dBm) {
  __shared__ float G[kHK][kHK + 1], H[kHK][kHK + 1];
  __shared__ float As[kHK][kHC + 1], Bs[kHK][kHC + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < kHK * kHK; e += blockDim.x) {
    const float* p = part + (int64_t)b * kHK * kHK * kHK + e;
    float s = 0.f;
    for (int j = 0; j < kHK; ++j) s += p[(int64_t)j * kHK * kHK];
    G[e / kHK][e % kHK] = s;
    H[e / kHK][e % kHK] = dBAt[(int64_t)b * kHK * kHK + e];
  }
  for (int e = tid; e < kHK * kHC; e += blockDim.x) {
    As[e / kHC][e % kHC] = A[(int64_t)b * kHK * kHC + e];
    Bs[e / kHC][e % kHC] = Bm[(int64_t)b * kHK * kHC + e];
  }
  __syncthreads();
  for (int e = tid; e < kHK * kHC; e += blockDim.x) {
    const int k = e / kHC, c = e - k * kHC;
    float da = 0.f, db = 0.f;
    for (int j = 0; j < kHK; ++j) {
      da = fmaf(G[k][j] + G[j][k], As[j][c], da);
      da = fmaf(H[j][k], Bs[j][c], da);
      db = fmaf(H[k][j], As[j][c], db);
    }
    dA[(int64_t)b * kHK * kHC + e] = da;
    dBm[(int64_t)b * kHK * kHC + e] = db;
  }
}

// grid (ceil(Nmax / 64), B, 2), block 256: dF[n, c] = sum_k W[n, k] dA[k, c] for the x side
// (z = 0) / y side (z = 1), W = evecs * mass; written to dF (element (b, n, c) at b sb + n sn
// + c sc: the caller's layout). Threads: 64 points x 4 channel groups of 8.
struct FeatOut {
  float* base;
  int64_t sb, sn, sc;
};

__global__ __launch_bounds__(256) void fmap_head_expand_kernel(const float* __restrict__ ex, int ldex,
                                                               const float* __restrict__ mx, int N1,
                                                               const float* __restrict__ ey, int ldey,
                                                               const float* __restrict__ my, int N2,
                                                               const float* __restrict__ dA,
                                                               const float* __restrict__ dBm, FeatOut ox,
                                                               FeatOut oy) {
  __shared__ float Gs[kHK][kHC];
  const int b = blockIdx.y, tid = threadIdx.x;
  const bool xs = blockIdx.z == 0;
  const int N = xs ? N1 : N2;
  const int n0 = blockIdx.x * 64;
  if (n0 >= N) return;
  const float* g = (xs ? dA : dBm) + (int64_t)b * kHK * kHC;
  for (int e = tid; e < kHK * kHC; e += 256) Gs[e / kHC][e % kHC] = g[e];
  __syncthreads();
  const int n = n0 + (tid & 63), cg = (tid >> 6) * 8;
  if (n >= N) return;
  const float* ev = xs ? ex : ey;
  const int lde = xs ? ldex : ldey;
  const int64_t row = (int64_t)b * N + n;
  const float m = (xs ? mx : my)[row];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < kHK; ++k) {
    const float w = ev[row * lde + k] * m;
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = fmaf(w, Gs[k][cg + q], acc[q]);
  }
  const FeatOut o = xs ? ox : oy;
#pragma unroll
  for (int q = 0; q < 8; ++q) o.base[(int64_t)b * o.sb + (int64_t)n * o.sn + (int64_t)(cg + q) * o.sc] = acc[q];
}

}  // namespace

extern "C" int64_t pk_fmap_head_work_len(int B, int N1, int N2) {
  if (B <= 0 || N1 <= 0 || N2 <= 0) return 0;
  return (int64_t)B * ((N1 + kPChunk - 1) / kPChunk + (N2 + kPChunk - 1) / kPChunk) * kHK * kHC;
}

extern "C" int pk_fmap_head_fwd(const float* evecs_x, int ldex, const float* mass_x, const float* fx,
                                const int64_t* fx_strides, int N1, const float* evecs_y, int ldey,
                                const float* mass_y, const float* fy, const int64_t* fy_strides, int N2,
                                const float* evals_x, int ldvx, const float* evals_y, int ldvy, int B, int K, int C,
                                float gamma, float* A, float* Bm, float* AAt, float* BAt, float* D, float* work,
                                int64_t work_len, void* stream) {
  PK_REQUIRE(B >= 0 && K == kHK && C == kHC && N1 > 0 && N2 > 0 && ldex >= K && ldey >= K && ldvx >= K && ldvy >= K);
  if (B == 0) return PK_OK;
  PK_REQUIRE(evecs_x && mass_x && fx && fx_strides && evecs_y && mass_y && fy && fy_strides && evals_x && evals_y);
  PK_REQUIRE(A && Bm && AAt && BAt && D && work);
  const int Px = (N1 + kPChunk - 1) / kPChunk, P = Px + (N2 + kPChunk - 1) / kPChunk;
  PK_REQUIRE(work_len >= pk_fmap_head_work_len(B, N1, N2));
  const FeatRef rx{fx, fx_strides[0], fx_strides[1], fx_strides[2]};
  const FeatRef ry{fy, fy_strides[0], fy_strides[1], fy_strides[2]};
  hipStream_t s = pk::as_stream(stream);
  hipLaunchKernelGGL(fmap_head_part_kernel, dim3(P, B), dim3(256), 0, s, evecs_x, ldex, mass_x, rx, N1, evecs_y, ldey,
                     mass_y, ry, N2, Px, work);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(fmap_head_fin_kernel, dim3(B), dim3(512), 0, s, work, Px, P, evals_x, ldvx, evals_y, ldvy, gamma,
                     A, Bm, AAt, BAt, D);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_fmap_head_bwd(const float* part, const float* dBAt, const float* A, const float* Bm,
                                const float* evecs_x, int ldex, const float* mass_x, int N1, const float* evecs_y,
                                int ldey, const float* mass_y, int N2, int B, int K, int C, float* dA, float* dBm,
                                float* dfx, const int64_t* dfx_strides, float* dfy, const int64_t* dfy_strides,
                                void* stream) {
  PK_REQUIRE(B >= 0 && K == kHK && C == kHC && N1 > 0 && N2 > 0 && ldex >= K && ldey >= K);
  if (B == 0) return PK_OK;
  PK_REQUIRE(part && dBAt && A && Bm && evecs_x && mass_x && evecs_y && mass_y && dA && dBm);
  PK_REQUIRE(dfx && dfx_strides && dfy && dfy_strides);
  hipStream_t s = pk::as_stream(stream);
  hipLaunchKernelGGL(fmap_head_grad_kernel, dim3(B), dim3(512), 0, s, part, dBAt, A, Bm, dA, dBm);
  PK_CHECK_LAUNCH();
  const FeatOut ox{dfx, dfx_strides[0], dfx_strides[1], dfx_strides[2]};
  const FeatOut oy{dfy, dfy_strides[0], dfy_strides[1], dfy_strides[2]};
  const int Nmax = N1 > N2 ? N1 : N2;
  hipLaunchKernelGGL(fmap_head_expand_kernel, dim3((Nmax + 63) / 64, B, 2), dim3(256), 0, s, evecs_x, ldex, mass_x, N1,
                     evecs_y, ldey, mass_y, N2, dA, dBm, ox, oy);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
