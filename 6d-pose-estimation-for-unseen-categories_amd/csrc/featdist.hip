// H10 / H11 (first half) — pairwise spectral feature distance + argmin / top-5.
//
// Reference: fmap2pointmap_solvers/naive.py:6-34 and spacial_filtering.py:5-38:
//     emb  = evecs_x[:, :30] @ C12.T                       [V1, 30]
//     dist = torch.cdist(emb, evecs_y[:, :30])             [V1, V2]
//     naive: p2p[j] = dist.argmin(dim=-2)                  (first minimal i)
//     spatial: idx = dist.sort(dim=-2)[1].T[:, :5]         (5 nearest i per j)
// torch.cdist (V > 25) evaluates the mm expansion with K = 32:
//     [-2 x, |x|^2, 1] · [y, 1, |y|^2]^T, clamp_min(1e-30), sqrt
// The kernel computes exactly that augmented K = 32 contraction on the f32 MFMA
// (v_mfma_f32_16x16x4_f32: f32 products, f32 accumulation), clamps, and keeps per
// column a running argmin (or sorted top-5) in the epilogue; sqrt is monotone and is
// applied to the emitted distances only. Ties resolve to the lowest row index.
//
// Layout: per crop, rows i < n1[b] of evecs_x [B, V1max, ldx], C [B, 30, 30], rows
// j < n2[b] of evecs_y [B, V2max, ldy]. Pass 1 (prep) builds the augmented operands
// A [B, V1max, 32], Bq [B, V2max, 32]; pass 2 tiles 64 columns per workgroup (16 per
// wave) and streams all rows through LDS in 64-row chunks.
#include "common.hpp"

namespace {

constexpr int kF = 30;   // n_fmap
constexpr int kK = 32;   // augmented contraction length
using f32x4 = __attribute__((ext_vector_type(4))) float;

// grid (ceil(max(V1,V2)/256), B, 2): z = 0 -> A rows (x side), z = 1 -> B rows (y side).
__global__ __launch_bounds__(256) void fd_prep_kernel(const float* __restrict__ ex, int ldx,
                                                      const float* __restrict__ C,
                                                      const float* __restrict__ ey, int ldy,
                                                      const int32_t* __restrict__ n1,
                                                      const int32_t* __restrict__ n2, int V1max,
                                                      int V2max, float* __restrict__ A,
                                                      float* __restrict__ Bq) {
  const int b = blockIdx.y;
  const int r = blockIdx.x * 256 + threadIdx.x;
  __shared__ float sC[kF * kF];
  if (blockIdx.z == 0) {
    for (int e = threadIdx.x; e < kF * kF; e += 256) sC[e] = C[(int64_t)b * kF * kF + e];
    __syncthreads();
    if (r >= V1max) return;
    float* o = A + ((int64_t)b * V1max + r) * kK;
    if (r >= n1[b]) {
      for (int c = 0; c < kK; ++c) o[c] = 0.f;
      return;
    }
    const float* e = ex + ((int64_t)b * V1max + r) * ldx;
    float x[kF];
#pragma unroll
    for (int k = 0; k < kF; ++k) x[k] = e[k];
    float nrm = 0.f;
#pragma unroll
    for (int c = 0; c < kF; ++c) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kF; ++k) s = fmaf(x[k], sC[c * kF + k], s);  // emb = x C^T
      o[c] = -2.f * s;
      nrm = fmaf(s, s, nrm);
    }
    o[kF] = nrm;
    o[kF + 1] = 1.f;
  } else {
    if (r >= V2max) return;
    float* o = Bq + ((int64_t)b * V2max + r) * kK;
    if (r >= n2[b]) {
      for (int c = 0; c < kK; ++c) o[c] = 0.f;
      return;
    }
    const float* e = ey + ((int64_t)b * V2max + r) * ldy;
    float nrm = 0.f;
#pragma unroll
    for (int k = 0; k < kF; ++k) {
      const float y = e[k];
      o[k] = y;
      nrm = fmaf(y, y, nrm);
    }
    o[kF] = 1.f;
    o[kF + 1] = nrm;
  }
}

template <int TOPK>
struct TopK {
  float v[TOPK];
  int i[TOPK];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      v[k] = __builtin_huge_valf();
      i[k] = 0x7fffffff;
    }
  }
  // rows arrive in increasing index order: strict < keeps the lowest index on ties
  __device__ __forceinline__ void push(float x, int idx) {
    if (!(x < v[TOPK - 1])) return;
    float cv = x;
    int ci = idx;
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      const bool sw = cv < v[k];
      const float tv = sw ? v[k] : cv;
      const int ti = sw ? i[k] : ci;
      v[k] = sw ? cv : v[k];
      i[k] = sw ? ci : i[k];
      cv = tv;
      ci = ti;
    }
  }
  // merge an incoming sorted list (ties: lower index first)
  __device__ __forceinline__ void merge(const float (&ov)[TOPK], const int (&oi)[TOPK]) {
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      float cv = ov[k];
      int ci = oi[k];
#pragma unroll
      for (int m = 0; m < TOPK; ++m) {
        const bool sw = cv < v[m] || (cv == v[m] && ci < i[m]);
        const float tv = sw ? v[m] : cv;
        const int ti = sw ? i[m] : ci;
        v[m] = sw ? cv : v[m];
        i[m] = sw ? ci : i[m];
        cv = tv;
        ci = ti;
      }
    }
  }
};

constexpr int kRowsChunk = 64;
constexpr int kLdsRow = kK + 4;  // padded row (floats)

// grid (ceil(V2max/64), B), block 256 (4 waves x 16 columns).
template <int TOPK>
__global__ __launch_bounds__(256) void fd_main_kernel(const float* __restrict__ A, const float* __restrict__ Bq,
                                                      const int32_t* __restrict__ n1,
                                                      const int32_t* __restrict__ n2, int V1max, int V2max,
                                                      int64_t* __restrict__ out_idx,
                                                      float* __restrict__ out_dist) {
  __shared__ __attribute__((aligned(16))) float sA[kRowsChunk * kLdsRow];
  const int b = blockIdx.y;
  const int lane = pk::lane_id(), wave = pk::wave_id();
  const int g = lane >> 4, c16 = lane & 15;
  const int j = blockIdx.x * 64 + wave * 16 + c16;
  const int N1 = n1[b], N2 = n2[b];
  // B operand: lane supplies Bq[j][4s + g] for step s
  float bop[8];
  {
    const float* br = Bq + ((int64_t)b * V2max + min(j, V2max - 1)) * kK;
#pragma unroll
    for (int s = 0; s < 8; ++s) bop[s] = br[4 * s + g];
  }
  TopK<TOPK> best;
  best.init();
  for (int i0 = 0; i0 < N1; i0 += kRowsChunk) {
    __syncthreads();
    // stage rows [i0, i0+64) of A as [row][g][s] (k = 4s + g) so a lane's 8 operands are contiguous
    for (int e = threadIdx.x; e < kRowsChunk * kK; e += 256) {
      const int rr = e / kK, k = e % kK;
      const int i = i0 + rr;
      const float v = i < N1 ? A[((int64_t)b * V1max + i) * kK + k] : 0.f;
      sA[rr * kLdsRow + (k & 3) * 8 + (k >> 2)] = v;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kRowsChunk / 16; ++t) {
      const float4* ap = reinterpret_cast<const float4*>(&sA[(t * 16 + c16) * kLdsRow + g * 8]);
      const float4 a0 = ap[0], a1 = ap[1];
      const float aop[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aop[s], bop[s], acc, 0, 0, 0);
      // lane holds D[i0 + 16t + 4g + r][j]
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + t * 16 + 4 * g + r;
        float v = fmaxf(acc[r], 1e-30f);  // clamp_min(1e-30) (cdist mm path)
        if (i >= N1) v = __builtin_huge_valf();
        best.push(v, i);
      }
    }
  }
  // merge the 4 lane groups of each column (lanes c16, c16+16, c16+32, c16+48)
#pragma unroll
  for (int off = 16; off <= 32; off <<= 1) {
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      ov[k] = __shfl_xor(best.v[k], off);
      oi[k] = __shfl_xor(best.i[k], off);
    }
    best.merge(ov, oi);
  }
  if (g == 0 && j < N2) {
    const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      out_idx[o + k] = best.i[k] == 0x7fffffff ? -1 : best.i[k];
      if (out_dist) out_dist[o + k] = sqrtf(best.v[k]);
    }
  }
}

}  // namespace

extern "C" int pk_feat_dist_topk(const float* evecs_x, int ldx, const float* C, const float* evecs_y, int ldy,
                                 const int32_t* n1, const int32_t* n2, int B, int V1max, int V2max, int topk,
                                 float* A, float* Bq, int64_t* out_idx, float* out_dist, void* stream) {
  PK_REQUIRE(B >= 0 && V1max >= 0 && V2max >= 0 && ldx >= kF && ldy >= kF && (topk == 1 || topk == 5));
  if (B == 0 || V2max == 0) return PK_OK;
  PK_REQUIRE(evecs_x && C && evecs_y && n1 && n2 && A && Bq && out_idx);
  hipStream_t s = pk::as_stream(stream);
  const int vm = V1max > V2max ? V1max : V2max;
  hipLaunchKernelGGL(fd_prep_kernel, dim3((vm + 255) / 256, B, 2), dim3(256), 0, s, evecs_x, ldx, C, evecs_y, ldy,
                     n1, n2, V1max, V2max, A, Bq);
  PK_CHECK_LAUNCH();
  if (topk == 1)
    hipLaunchKernelGGL(fd_main_kernel<1>, dim3((V2max + 63) / 64, B), dim3(256), 0, s, A, Bq, n1, n2, V1max,
                       V2max, out_idx, out_dist);
  else
    hipLaunchKernelGGL(fd_main_kernel<5>, dim3((V2max + 63) / 64, B), dim3(256), 0, s, A, Bq, n1, n2, V1max,
                       V2max, out_idx, out_dist);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
