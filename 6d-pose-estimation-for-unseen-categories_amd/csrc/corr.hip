// Correspondence post-processing and per-crop labels:
//
//  pk_rigidity_filter  H11 second half — fmap2pointmap_solvers/spacial_filtering.py:42-75:
//      three rounds; in each, for the surviving candidates (c_i, p_i)
//        score_j = mean_i | ||CAD[c_i] - CAD[c_j]|| - ||PC[p_i] - PC[p_j]|| |
//      keep score < tau * diam with tau = 0.3, 0.15, then 0.055 (0.065 if 0.055 keeps
//      nothing). Computed pairwise on the fly (the reference materialises [n,n,3] twice
//      per round); order of survivors preserved.
//  pk_inlier_ratio     H12 — utils/utils.py:81-105: mean(||CAD[c]-PC_al[p]|| < thr), 0 if
//      no correspondences (f32, correctly rounded sqrt).
//  pk_cgt_lstsq        H15 — utils/utils.py:67-79 C_from_sparse_P: least squares
//      evecs2[P1] X = evecs1[P0] via fp64 normal equations + Gauss-Jordan (partial pivoting).
#include "common.hpp"

namespace {

constexpr int kTile = 1024;

// grid (ceil(nmax/256), B), block 256: score for every listed candidate of crop b.
__global__ __launch_bounds__(256) void rigid_score_kernel(const int64_t* __restrict__ list, int ldl,
                                                          const int32_t* __restrict__ nlist,
                                                          const int64_t* __restrict__ cand, int ldc,
                                                          const float* __restrict__ cad, int ldcad,
                                                          const float* __restrict__ pc, int ldpc,
                                                          float* __restrict__ score) {
  __shared__ float s[kTile * 6];
  const int b = blockIdx.y;
  const int n = nlist[b];
  const int jj = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x * 256 >= n) return;
  const int64_t* L = list + (int64_t)b * ldl;
  const int64_t* Cd = cand + (int64_t)b * ldc * 2;
  const float* CA = cad + (int64_t)b * ldcad * 3;
  const float* PCb = pc + (int64_t)b * ldpc * 3;
  float ax = 0, ay = 0, az = 0, px = 0, py = 0, pz = 0;
  if (jj < n) {
    const int64_t k = L[jj];
    const int64_t c = Cd[2 * k], p = Cd[2 * k + 1];
    ax = CA[3 * c]; ay = CA[3 * c + 1]; az = CA[3 * c + 2];
    px = PCb[3 * p]; py = PCb[3 * p + 1]; pz = PCb[3 * p + 2];
  }
  float acc = 0.f;
  for (int t0 = 0; t0 < n; t0 += kTile) {
    const int tn = min(kTile, n - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn; e += 256) {
      const int64_t k = L[t0 + e];
      const int64_t c = Cd[2 * k], p = Cd[2 * k + 1];
      s[6 * e + 0] = CA[3 * c]; s[6 * e + 1] = CA[3 * c + 1]; s[6 * e + 2] = CA[3 * c + 2];
      s[6 * e + 3] = PCb[3 * p]; s[6 * e + 4] = PCb[3 * p + 1]; s[6 * e + 5] = PCb[3 * p + 2];
    }
    __syncthreads();
    if (jj < n) {
      for (int e = 0; e < tn; ++e) {
        const float dx = s[6 * e] - ax, dy = s[6 * e + 1] - ay, dz = s[6 * e + 2] - az;
        const float ex = s[6 * e + 3] - px, ey = s[6 * e + 4] - py, ez = s[6 * e + 5] - pz;
        const float a = __builtin_amdgcn_sqrtf((dx * dx + dy * dy) + dz * dz);
        const float bb = __builtin_amdgcn_sqrtf((ex * ex + ey * ey) + ez * ez);
        acc += fabsf(a - bb);
      }
    }
  }
  if (jj < n) score[(int64_t)b * ldl + jj] = acc / (float)n;
}

// One block per crop: ordered compaction of list entries whose score < tau * diam.
// round 3 (fallback > 0): if nothing passes tau, use the fallback threshold.
// thr f32 [B, 4]: tau * diam_cad for tau = 0.3, 0.15, 0.055, 0.065, evaluated in double and
// rounded once (the reference compares an f32 tensor with the Python float tau * diam).
__global__ __launch_bounds__(1024) void rigid_compact_kernel(const int64_t* __restrict__ list_in, int ldl,
                                                             const int32_t* __restrict__ nin,
                                                             const float* __restrict__ score,
                                                             const float* __restrict__ thr4, int round,
                                                             int64_t* __restrict__ list_out,
                                                             int32_t* __restrict__ nout) {
  __shared__ int ws[16];
  __shared__ int carry;
  __shared__ float thr_s;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = nin[b];
  const float* S = score + (int64_t)b * ldl;
  if (tid == 0) {
    carry = 0;
    thr_s = thr4[b * 4 + round];
  }
  __syncthreads();
  if (round == 2) {
    int c = 0;
    for (int i = tid; i < n; i += 1024) c += S[i] < thr_s ? 1 : 0;
    c = pk::wave_sum_i32_s(c);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += ws[w];
      if (tot == 0) thr_s = thr4[b * 4 + 3];
    }
    __syncthreads();
  }
  const float thr = thr_s;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const bool keep = i < n && S[i] < thr;
    const uint64_t bal = __ballot(keep);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = __popcll(bal);
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < pk::wave_id(); ++w) pre += ws[w];
    if (keep) list_out[(int64_t)b * ldl + pre + __popcll(bal & ((1ull << pk::lane_id()) - 1ull))] =
        list_in[(int64_t)b * ldl + i];
    __syncthreads();
    if (tid == 1023) carry = pre + __popcll(bal);
    __syncthreads();
  }
  if (tid == 0) nout[b] = carry;
}

__global__ void iota_kernel(int64_t* __restrict__ list, int ldl, const int32_t* __restrict__ n) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n[b]) list[(int64_t)b * ldl + i] = i;
}

// grid (B), block 256: IR per crop.
__global__ __launch_bounds__(256) void ir_kernel(const int64_t* __restrict__ pairs, int ldp, int pair_stride,
                                                 int col_cad, int col_pc, const int32_t* __restrict__ npairs,
                                                 const float* __restrict__ cad, int ldcad,
                                                 const float* __restrict__ pcal, int ldpc,
                                                 const float* __restrict__ thr, float* __restrict__ ir) {
  __shared__ int ws[4];
  const int b = blockIdx.x;
  const int n = npairs[b];
  const float t = thr[b];
  int c = 0;
  for (int k = threadIdx.x; k < n; k += 256) {
    const int64_t* pr = pairs + (int64_t)b * ldp * 2;
    const int64_t ci = pr[col_cad * (pair_stride == 1 ? ldp : 1) + k * (pair_stride == 1 ? 1 : 2)];
    const int64_t pi = pr[col_pc * (pair_stride == 1 ? ldp : 1) + k * (pair_stride == 1 ? 1 : 2)];
    const float* a = cad + ((int64_t)b * ldcad + ci) * 3;
    const float* p = pcal + ((int64_t)b * ldpc + pi) * 3;
    const float dx = a[0] - p[0], dy = a[1] - p[1], dz = a[2] - p[2];
    const float d = __fsqrt_rn((dx * dx + dy * dy) + dz * dz);
    c += d < t ? 1 : 0;
  }
  c = pk::wave_sum_i32_s(c);
  if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = ws[0] + ws[1] + ws[2] + ws[3];
    ir[b] = n > 0 ? (float)tot / (float)n : 0.f;
  }
}

// ---------------------------------------------------------------- C_gt (normal equations)
constexpr int kF = 30;

constexpr int kCgtPairs = 256;  // pairs per partial-sum block
constexpr int kGH = kF * 2 * kF;   // 30 x 60 entries of [G | H]

// grid (ceil(ldp / 256), B), block 256: partial [G | H] = A^T [A | Bm] over 256 pairs of
// crop b (A = e2[p1], Bm = e1[p0], fp32 inputs, exact products, fp64 accumulation).
__global__ __launch_bounds__(256) void cgt_partial_kernel(const int64_t* __restrict__ pairs, int ldp,
                                                          const int64_t* __restrict__ npairs,
                                                          const float* __restrict__ e1, int ld1, int V1max,
                                                          const float* __restrict__ e2, int ld2, int V2max,
                                                          double* __restrict__ part) {
  __shared__ float r1[64][kF], r2[64][kF];
  const int b = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
  const int64_t n = npairs[b] < ldp ? npairs[b] : ldp;
  const int64_t p_begin = (int64_t)s * kCgtPairs;
  if (p_begin >= n) return;
  const int64_t p_end = min(n, p_begin + kCgtPairs);
  double acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.0;
  const int64_t* P = pairs + (int64_t)b * ldp * 2;
  for (int64_t p0 = p_begin; p0 < p_end; p0 += 64) {
    const int pn = (int)min((int64_t)64, p_end - p0);
    __syncthreads();
    for (int e = tid; e < 64 * kF; e += 256) {
      const int r = e / kF, k = e % kF;
      float a = 0.f, c = 0.f;
      if (r < pn) {
        const int64_t i0 = P[2 * (p0 + r)], i1 = P[2 * (p0 + r) + 1];
        c = e1[((int64_t)b * V1max + i0) * ld1 + k];
        a = e2[((int64_t)b * V2max + i1) * ld2 + k];
      }
      r2[r][k] = a;
      r1[r][k] = c;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + 256 * q;
      if (e >= kGH) break;
      const int row = e / (2 * kF), col = e % (2 * kF);
      double sacc = acc[q];
      for (int r = 0; r < pn; ++r) {
        const double u = (double)r2[r][row];
        const double v = col < kF ? (double)r2[r][col] : (double)r1[r][col - kF];
        sacc = fma(u, v, sacc);
      }
      acc[q] = sacc;
    }
  }
  const int S = gridDim.x;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = tid + 256 * q;
    if (e < kGH) part[((int64_t)b * S + s) * kGH + e] = acc[q];
  }
}

// grid (B), block 256: sum the active partials (in slice order), then one wave solves
// G X = H by Gauss-Jordan with partial pivoting; C_gt = X.
__global__ __launch_bounds__(256) void cgt_solve_kernel(const double* __restrict__ part, int S,
                                                        const int64_t* __restrict__ npairs, int ldp,
                                                        float* __restrict__ Cgt) {
  __shared__ double GH[kF][2 * kF + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t n = npairs[b] < ldp ? npairs[b] : ldp;
  const int active = (int)((n + kCgtPairs - 1) / kCgtPairs);
  for (int e = tid; e < kGH; e += 256) {
    double v = 0.0;
    for (int s = 0; s < active && s < S; ++s) v += part[((int64_t)b * S + s) * kGH + e];
    GH[e / (2 * kF)][e % (2 * kF)] = v;
  }
  __syncthreads();
  if (tid >= 64) return;
  const int lane = tid;
  bool used = lane >= kF;
  int var = -1;
  for (int k = 0; k < kF; ++k) {
    const double a = used ? -1.0 : fabs(GH[lane][k]);
    uint32_t hi = used ? 0u : (uint32_t)(__double_as_longlong(a) >> 32);
    const uint32_t mhi = pk::wave_max_u32_s(hi);
    const uint32_t lo = (uint32_t)(__double_as_longlong(a) & 0xffffffffull);
    const uint32_t mlo = pk::wave_max_u32_s((!used && hi == mhi) ? lo : 0u);
    const uint64_t bal = __ballot(!used && hi == mhi && lo == mlo);
    const int p = bal ? (__ffsll((unsigned long long)bal) - 1) : 0;
    const double piv = GH[p][k];
    const double f = (lane != p && lane < kF) ? GH[lane][k] / piv : 0.0;
    __builtin_amdgcn_s_barrier();  // single wave: keeps the reads above ahead of the writes
    for (int c = 0; c < 2 * kF; ++c) {
      if (lane < kF) {
        const double pc = GH[p][c];
        if (lane != p) GH[lane][c] = fma(-f, pc, GH[lane][c]);
      }
    }
    __builtin_amdgcn_s_barrier();
    if (lane == p) {
      for (int c = 0; c < 2 * kF; ++c) GH[lane][c] = GH[lane][c] / piv;
      used = true;
      var = k;
    }
    __builtin_amdgcn_s_barrier();
  }
  if (var >= 0)
    for (int c = 0; c < kF; ++c) Cgt[((int64_t)b * kF + var) * kF + c] = (float)GH[lane][kF + c];
}

}  // namespace

extern "C" int pk_rigidity_filter(const int64_t* cand, int ldc, const int32_t* ncand, const float* cad,
                                  int ldcad, const float* pc, int ldpc, const float* thr4, int B, int nmax,
                                  int64_t* list_a, int64_t* list_b, int32_t* n_a, int32_t* n_b, float* score,
                                  void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && ldc >= nmax);
  if (B == 0) return PK_OK;
  PK_REQUIRE(cand && ncand && cad && pc && thr4 && list_a && list_b && n_a && n_b && score);
  hipStream_t s = pk::as_stream(stream);
  const dim3 g((nmax + 255) / 256, B);
  hipLaunchKernelGGL(iota_kernel, g, dim3(256), 0, s, list_a, ldc, ncand);
  PK_CHECK_LAUNCH();
  const int32_t* nin = ncand;
  int64_t* lin = list_a;
  int64_t* lout = list_b;
  int32_t* nout = n_b;
  int32_t* nspare = n_a;
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(rigid_score_kernel, g, dim3(256), 0, s, lin, ldc, nin, cand, ldc, cad, ldcad, pc, ldpc,
                       score);
    PK_CHECK_LAUNCH();
    hipLaunchKernelGGL(rigid_compact_kernel, dim3(B), dim3(1024), 0, s, lin, ldc, nin, score, thr4, r, lout,
                       nout);
    PK_CHECK_LAUNCH();
    nin = nout;
    int64_t* t = lin;
    lin = lout;
    lout = t;
    int32_t* tn = nspare;
    nspare = nout;
    nout = tn;
  }
  // after 3 rounds the survivors are in list_b / n_b (a -> b -> a -> b)
  return PK_OK;
}

extern "C" int pk_inlier_ratio(const int64_t* pairs, int ldp, int layout, const int32_t* npairs, const float* cad,
                               int ldcad, const float* pc_aligned, int ldpc, const float* thr, int B, float* ir,
                               void* stream) {
  PK_REQUIRE(B >= 0 && (layout == 0 || layout == 1));
  if (B == 0) return PK_OK;
  PK_REQUIRE(pairs && npairs && cad && pc_aligned && thr && ir);
  // layout 0: pairs [B, ldp, 2] (cad, pc); layout 1: [B, 2, ldp] (row 0 cad, row 1 pc)
  hipLaunchKernelGGL(ir_kernel, dim3(B), dim3(256), 0, pk::as_stream(stream), pairs, ldp, layout == 1 ? 1 : 2, 0, 1,
                     npairs, cad, ldcad, pc_aligned, ldpc, thr, ir);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_cgt_lstsq(const int64_t* pairs, int ldp, const int64_t* npairs, const float* evecs1, int ld1,
                            int V1max, const float* evecs2, int ld2, int V2max, int B, int K, double* work,
                            float* Cgt, void* stream) {
  PK_REQUIRE(B >= 0 && K == kF && ld1 >= kF && ld2 >= kF && ldp >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(pairs && npairs && evecs1 && evecs2 && work && Cgt);
  hipStream_t s = pk::as_stream(stream);
  const int S = ldp > 0 ? (ldp + kCgtPairs - 1) / kCgtPairs : 1;
  if (ldp > 0) {
    hipLaunchKernelGGL(cgt_partial_kernel, dim3(S, B), dim3(256), 0, s, pairs, ldp, npairs, evecs1, ld1, V1max, evecs2,
                       ld2, V2max, work);
    PK_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(cgt_solve_kernel, dim3(B), dim3(256), 0, s, work, S, npairs, ldp, Cgt);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
