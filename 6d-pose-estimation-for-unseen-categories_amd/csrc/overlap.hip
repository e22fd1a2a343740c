// H8 overlap head, fused: modeling/dpfm.py:125-145 (OverlapPredictorNet)
//   n = F.normalize(x, dim=-1); h = ReLU(W0 n + b0) (Linear 32 -> 32); s = sigmoid(w1 . h + b1)
// for the CAD and crop features of a batch in one launch per direction. Round 2 ran it as
// pk_l2_normalize_fwd + a 32 -> 32 MFMA layer + a thin 32 -> 1 layer per shape (and, backward,
// the thin 1 -> 32 input gradient with the sigmoid backward folded in, the 32 -> 32 input
// gradient and pk_l2_normalize_bwd): 12 launches per training step, ~150 us, each a few MB
// (latency-bound). Here one thread owns one point for the whole chain and the arithmetic is
// the same operations in the same order as those kernels, so every output is bit-identical:
//   * the normalization: the sum of squares in channel order (separately rounded), sqrtf, the
//     IEEE division by max(||x||, 1e-12);
//   * the 32 -> 32 layers: the per-point layer kernels run on v_mfma_f32_16x16x4f32, an exact
//     fmaf chain whose step (q, i) takes k = 16 q + 4 g + i for lane groups g = 0..3 in slot
//     order — replayed here as an fmaf chain over that k order (mfma_k), bias after the sum;
//   * the 32 -> 1 layer: fmaf chain in k order starting from the bias (the thin kernel);
//   * backward: dz = ds (s (1 - s)), dh = [h > 0] fmaf(dz, w1, 0), the l2 backward on
//     dn (+ the NCE term's rows gradient) as pk_l2_normalize_bwd.
// Rows outputs / inputs ([B N, 32]: the normalized rows for the NCE term and the weight
// gradients, h, dh) move through a per-wave LDS tile so each global access instruction covers
// 256 contiguous bytes; x / n / dx keep the features' own storage (channels-first in the step:
// coalesced per channel).
#include "common.hpp"
#include "../../include/posekern.h"

namespace {

constexpr int kC = 32;
constexpr int kTS = kC + 1;  // LDS row stride of a wave's [64][33] rows tile (conflict-free)

struct OvhShape {
  const float* x;
  int64_t sb, sn, sc;
  int N, pad;
  float* n;
  float* nrm;
  float* nrows;
  float* h;
  float* s;
  const float* ds;
  const float* dnr;
  float* g;
  float* dh;
  float* dx;
  const float* dadd;
};
struct OvhArgs {
  OvhShape sh[2];
  int B, pad;
};

// contraction position j (0..31) -> channel k of the MFMA layer kernels' accumulation order
__device__ __forceinline__ constexpr int mfma_k(int j) { return (j & 16) | ((j & 3) << 2) | ((j >> 2) & 3); }

// this wave's 64 points x 32 values, lane = point, written to rows [p][32] starting at dst
// (points >= nvalid skipped) as 256-B contiguous stores
__device__ __forceinline__ void rows_store(float* __restrict__ dst, int64_t nvalid, const float (&v)[kC],
                                           float* __restrict__ T) {
  const int lane = pk::lane_id();
#pragma unroll
  for (int c = 0; c < kC; ++c) T[lane * kTS + c] = v[c];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (nvalid >= 64) {  // wave-uniform: a full wave stores without per-element guards
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const int f = j * 64 + lane;
      dst[f] = T[(f >> 5) * kTS + (f & 31)];
    }
  } else {
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const int f = j * 64 + lane, p = f >> 5, c = f & 31;
      if (p < nvalid) dst[f] = T[p * kTS + c];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void rows_load(const float* __restrict__ src, int64_t nvalid, float (&v)[kC],
                                          float* __restrict__ T) {
  const int lane = pk::lane_id();
  // unconditional loads at clamped indices (nvalid >= 1), then selects: no branch and no
  // memory wait per element
  float v2[kC];
#pragma unroll
  for (int j = 0; j < kC; ++j) {
    const int f = j * 64 + lane;
    v2[j] = src[(f >> 5) < nvalid ? f : 0];
  }
#pragma unroll
  for (int j = 0; j < kC; ++j) {
    const int f = j * 64 + lane, p = f >> 5, c = f & 31;
    T[p * kTS + c] = p < nvalid ? v2[j] : 0.f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int c = 0; c < kC; ++c) v[c] = T[lane * kTS + c];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// grid (ceil(max R / 256), 2 shapes), block 256 (4 waves x 64 points)
__global__ __launch_bounds__(256) void ovh_fwd_kernel(const OvhArgs a, const float* __restrict__ w0,
                                                      const float* __restrict__ b0, const float* __restrict__ w1,
                                                      const float* __restrict__ b1) {
  __shared__ float W0T[kC][kC];  // [k][o]
  __shared__ float sb0[kC], sw1[kC], sb1;
  __shared__ float T[4][64 * kTS];
  const OvhShape& S = a.sh[blockIdx.y];
  const int64_t R = (int64_t)a.B * S.N;
  const int lane = pk::lane_id(), wave = pk::wave_id();
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  const int64_t r = r0 + lane;
  const bool ok = r < R;
  // the point's features first (in flight while the weights are staged)
  const int64_t b = ok ? r / S.N : 0, nn = ok ? r - b * S.N : 0;
  const int64_t off = b * S.sb + nn * S.sn;  // point 0 for lanes past R (loaded, not used)
  float x[kC];
  if (r0 < R) {  // wave-uniform; unconditional loads (no per-load branch / wait)
#pragma unroll
    for (int c = 0; c < kC; ++c) x[c] = S.x[off + c * S.sc];
  }
  for (int e = threadIdx.x; e < kC * kC; e += 256) W0T[e & 31][e >> 5] = w0[e];
  if (threadIdx.x < kC) {
    sb0[threadIdx.x] = b0[threadIdx.x];
    sw1[threadIdx.x] = w1[threadIdx.x];
  }
  if (threadIdx.x == 0) sb1 = b1[0];
  __syncthreads();
  if (r0 >= R) return;  // wave-uniform
  float* Tw = T[wave];
  // F.normalize (pk_l2_normalize_fwd's arithmetic)
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < kC; ++c) ss += x[c] * x[c];
  const float nr = sqrtf(ss);
  const float d = fmaxf(nr, 1e-12f);
#pragma unroll
  for (int c = 0; c < kC; ++c) x[c] = x[c] / d;
  if (ok) {
#pragma unroll
    for (int c = 0; c < kC; ++c) S.n[off + c * S.sc] = x[c];
    S.nrm[r] = nr;
  }
  if (S.nrows != nullptr) rows_store(S.nrows + r0 * kC, R - r0, x, Tw);
  // Linear(32, 32) + ReLU: the MFMA kernels' fmaf chain order, bias after the sum
  float h[kC];
#pragma unroll
  for (int o = 0; o < kC; ++o) h[o] = 0.f;
#pragma unroll
  for (int j = 0; j < kC; ++j) {
    const int k = mfma_k(j);
    const float v = x[k];
#pragma unroll
    for (int o = 0; o < kC; ++o) h[o] = fmaf(v, W0T[k][o], h[o]);
  }
#pragma unroll
  for (int o = 0; o < kC; ++o) h[o] = fmaxf(h[o] + sb0[o], 0.f);
  if (S.h != nullptr) rows_store(S.h + r0 * kC, R - r0, h, Tw);
  // Linear(32, 1) + Sigmoid: fmaf chain in k order from the bias (the thin kernel)
  float z = sb1;
#pragma unroll
  for (int k = 0; k < kC; ++k) z = fmaf(h[k], sw1[k], z);
  if (ok) S.s[r] = 1.f / (1.f + expf(-z));
}

__global__ __launch_bounds__(256) void ovh_bwd_kernel(const OvhArgs a, const float* __restrict__ w0,
                                                      const float* __restrict__ w1) {
  __shared__ float W0[kC][kC];  // [o][k]
  __shared__ float sw1[kC];
  __shared__ float T[4][64 * kTS];
  const OvhShape& S = a.sh[blockIdx.y];
  const int64_t R = (int64_t)a.B * S.N;
  const int lane = pk::lane_id(), wave = pk::wave_id();
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  const int64_t r = r0 + lane;
  const bool ok = r < R;
  const int64_t b = ok ? r / S.N : 0, nn = ok ? r - b * S.N : 0;
  const int64_t off = b * S.sb + nn * S.sn;
  float dsv = 0.f, sv = 0.f, nr = 1.f;
  float nv[kC];
  if (r0 < R) {  // wave-uniform; unconditional loads at point 0 for lanes past R
    const int64_t rc = ok ? r : 0;
    dsv = S.ds[rc];
    sv = S.s[rc];
    nr = S.nrm[rc];
#pragma unroll
    for (int c = 0; c < kC; ++c) nv[c] = S.n[off + c * S.sc];
  }
  for (int e = threadIdx.x; e < kC * kC; e += 256) W0[e >> 5][e & 31] = w0[e];
  if (threadIdx.x < kC) sw1[threadIdx.x] = w1[threadIdx.x];
  __syncthreads();
  if (r0 >= R) return;  // wave-uniform
  float* Tw = T[wave];
  // sigmoid backward folded into the 1 -> 32 input gradient (thin kernel: pre / pre_out)
  const float gz = dsv * (sv * (1.f - sv));
  if (ok) S.g[r] = gz;
  float hd[kC];
  rows_load(S.h + r0 * kC, R - r0, hd, Tw);
#pragma unroll
  for (int o = 0; o < kC; ++o) hd[o] = hd[o] <= 0.f ? 0.f : fmaf(gz, sw1[o], 0.f);  // ReLU backward on h
  rows_store(S.dh + r0 * kC, R - r0, hd, Tw);
  // the 32 -> 32 input gradient dn = dh W0 (transposed weight; the MFMA kernels' order over o)
  float dn[kC];
#pragma unroll
  for (int k = 0; k < kC; ++k) dn[k] = 0.f;
#pragma unroll
  for (int j = 0; j < kC; ++j) {
    const int o = mfma_k(j);
    const float v = hd[o];
#pragma unroll
    for (int k = 0; k < kC; ++k) dn[k] = fmaf(v, W0[o][k], dn[k]);
  }
  if (S.dnr != nullptr) {  // the NCE term's gradient on the rows copy, added after (as dy + dy_rows)
    float e[kC];
    rows_load(S.dnr + r0 * kC, R - r0, e, Tw);
#pragma unroll
    for (int c = 0; c < kC; ++c) dn[c] += e[c];
  }
  // F.normalize backward (pk_l2_normalize_bwd's arithmetic)
  float yd = 0.f;
#pragma unroll
  for (int c = 0; c < kC; ++c) yd += nv[c] * dn[c];
  const bool clamped = !(nr > 1e-12f);
  if (ok) {
    // dadd: another consumer's gradient of x (x's storage), added to this one (the sum autograd
    // would form where the two consumers meet)
    float ad[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) ad[c] = S.dadd != nullptr ? S.dadd[off + c * S.sc] : 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const float v = clamped ? dn[c] / 1e-12f : (dn[c] - nv[c] * yd) / nr;
      S.dx[off + c * S.sc] = S.dadd != nullptr ? v + ad[c] : v;
    }
  }
}

OvhArgs ovh_args(const pk_overlap_head_args* a) {
  OvhArgs k{};
  for (int s = 0; s < 2; ++s) {
    OvhShape& S = k.sh[s];
    S.x = a->x[s];
    S.sb = a->strides[s][0];
    S.sn = a->strides[s][1];
    S.sc = a->strides[s][2];
    S.N = a->N[s];
    S.n = a->n[s];
    S.nrm = a->nrm[s];
    S.nrows = a->nrows[s];
    S.h = a->h[s];
    S.s = a->s[s];
    S.ds = a->ds[s];
    S.dnr = a->dnr[s];
    S.g = a->g[s];
    S.dh = a->dh[s];
    S.dx = a->dx[s];
    S.dadd = a->dadd[s];
  }
  k.B = a->B;
  return k;
}

}  // namespace

extern "C" int pk_overlap_head_fwd(const pk_overlap_head_args* a, void* stream) {
  PK_REQUIRE(a != nullptr && a->B >= 0 && a->N[0] >= 0 && a->N[1] >= 0);
  const int64_t R = (int64_t)a->B * (a->N[0] > a->N[1] ? a->N[0] : a->N[1]);
  if (R == 0) return PK_OK;
  PK_REQUIRE(a->w0 && a->b0 && a->w1 && a->b1);
  for (int s = 0; s < 2; ++s) {
    if ((int64_t)a->B * a->N[s] == 0) continue;
    PK_REQUIRE(a->x[s] && a->n[s] && a->nrm[s] && a->s[s]);
  }
  const OvhArgs k = ovh_args(a);
  hipLaunchKernelGGL(ovh_fwd_kernel, dim3((unsigned)((R + 255) / 256), 2), dim3(256), 0, pk::as_stream(stream), k,
                     a->w0, a->b0, a->w1, a->b1);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_overlap_head_bwd(const pk_overlap_head_args* a, void* stream) {
  PK_REQUIRE(a != nullptr && a->B >= 0 && a->N[0] >= 0 && a->N[1] >= 0);
  const int64_t R = (int64_t)a->B * (a->N[0] > a->N[1] ? a->N[0] : a->N[1]);
  if (R == 0) return PK_OK;
  PK_REQUIRE(a->w0 && a->w1);
  for (int s = 0; s < 2; ++s) {
    if ((int64_t)a->B * a->N[s] == 0) continue;
    PK_REQUIRE(a->n[s] && a->nrm[s] && a->h[s] && a->s[s] && a->ds[s] && a->g[s] && a->dh[s] && a->dx[s]);
  }
  const OvhArgs k = ovh_args(a);
  hipLaunchKernelGGL(ovh_bwd_kernel, dim3((unsigned)((R + 255) / 256), 2), dim3(256), 0, pk::as_stream(stream), k,
                     a->w0, a->w1);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
