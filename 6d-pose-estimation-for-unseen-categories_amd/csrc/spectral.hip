// H7 — spectral diffusion of DiffusionNet's LearnedTimeDiffusion (upstream diffusion-net
// layers.py, used by models/dpfm.py:22-30), forward and backward, fp32.
//
//   forward : spec = Phi^T (m ⊙ x)           [K, C]   (to_basis)
//             y    = Phi (E ⊙ spec),  E[k,c] = exp(-lambda_k t_c)   (from_basis)
//   backward: gs   = Phi^T g                  [K, C]
//             gx   = Phi (E ⊙ gs) ⊙ m  (per row)
//             gt_c = -sum_k lambda_k E[k,c] spec[k,c] gs[k,c]   (per crop; caller sums b)
// One code path serves both (`mode`): reduce (Phi^T · rows) -> combine (+E, +gt) ->
// expand (Phi · coefficients [· m]). Layout: x / y [B, N, C], Phi [B, N, K] row-major,
// m [B, N], lambda [B, K], t [C]; N is the padded per-crop point count.
#include "common.hpp"

namespace {

constexpr int kRows = 64;     // rows of Phi reduced per block in pass 1
constexpr int kSub = 32;      // rows staged in LDS per step
constexpr int kKC = 64;       // K == C == 64 (C_width, k_eig) — checked on the host

// pass 1: part[b, s] = sum_{rows in chunk s} Phi[r, :]^T (w_r * x[r, :]), w = mass or 1.
// grid (S, B), block 256 = 16 x 16 threads, each owning a 4 x 4 output micro-tile.
__global__ __launch_bounds__(256) void spec_reduce_kernel(const float* __restrict__ x, int ldx,
                                                          const float* __restrict__ mass,
                                                          const float* __restrict__ evecs, int N, int S,
                                                          float* __restrict__ part) {
  __shared__ float4 sphi[kSub][kKC / 4 + 1];
  __shared__ float4 sx[kSub][kKC / 4 + 1];
  const int s = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int ty = tid >> 4, tx = tid & 15;
  const float* __restrict__ phi = evecs + (int64_t)b * N * kKC;
  const float* __restrict__ xb = x + (int64_t)b * N * ldx;
  const float* __restrict__ mb = mass ? mass + (int64_t)b * N : nullptr;
  float acc[4][4] = {};
  const int r_begin = s * kRows;
  const int r_end = min(N, r_begin + kRows);
  for (int r0 = r_begin; r0 < r_end; r0 += kSub) {
    __syncthreads();
    for (int e = tid; e < kSub * (kKC / 4); e += 256) {
      const int rr = e / (kKC / 4), q = e % (kKC / 4);
      const int r = r0 + rr;
      float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), xv = pv;
      if (r < r_end) {
        pv = reinterpret_cast<const float4*>(phi + (int64_t)r * kKC)[q];
        xv = reinterpret_cast<const float4*>(xb + (int64_t)r * ldx)[q];
        if (mb) {
          const float w = mb[r];
          xv.x *= w; xv.y *= w; xv.z *= w; xv.w *= w;
        }
      }
      sphi[rr][q] = pv;
      sx[rr][q] = xv;
    }
    __syncthreads();
#pragma unroll 4
    for (int rr = 0; rr < kSub; ++rr) {
      const float4 p = sphi[rr][ty];
      const float4 v = sx[rr][tx];
      const float pk[4] = {p.x, p.y, p.z, p.w};
      const float vc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(pk[i], vc[j], acc[i][j]);
    }
  }
  float* __restrict__ o = part + ((int64_t)b * S + s) * kKC * kKC;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    reinterpret_cast<float4*>(o + (ty * 4 + i) * kKC)[tx] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
}

// pass 2: coef = sum_s part; save raw (optional), scaled = E ⊙ coef; optional gt partial
// gt[b, c] = -sum_k lambda_k E[k,c] saved[k,c] coef[k,c]. grid (B), block 1024: thread
// (k-quad, c) sums its 4 rows over the S partials as 4 independent chains.
// clamp_t: use max(t, 1e-8) (LearnedTimeDiffusion's in-place clamp_(min=1e-8) of the
// parameter, upstream layers.py) and, in the forward, write it back (block 0; every block
// computes the same value, so the concurrent reads see either value and use the clamped one).
// gt (backward): this crop's dL/dt partial, written over the first row of its own partial
// slab region (already consumed by this block) for the expand pass to sum in crop order.
__global__ __launch_bounds__(1024) void spec_combine_kernel(float* __restrict__ part, int S,
                                                            const float* __restrict__ evals,
                                                            float* __restrict__ t, int clamp_t, int write_t,
                                                            float* __restrict__ raw,
                                                            float* __restrict__ scaled,
                                                            const float* __restrict__ saved, int want_gt) {
  __shared__ double gsum[16][kKC];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int c = tid & 63, k0 = (tid >> 6) * 4;
  const float* pb = part + (int64_t)b * S * kKC * kKC + k0 * kKC + c;
  const float tc = clamp_t ? fmaxf(t[c], 1e-8f) : t[c];
  // the S slab partials (64 rows each) are summed in fp64: at N ~ 5000 CAD vertices a serial
  // fp32 sum over ~80 slabs dominated the error of the diffusion-time gradient, a
  // cancellation-prone contraction of two such sums
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  int s = 0;
  for (; s + 4 <= S; s += 4) {  // 4 slabs' loads issued together, added in slab order
    float ld[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) ld[u][i] = pb[(int64_t)(s + u) * kKC * kKC + i * kKC];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += (double)ld[u][i];
  }
  for (; s < S; ++s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += (double)pb[(int64_t)s * kKC * kKC + i * kKC];
  }
  double g = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + i;
    const float lam = evals[b * kKC + k];
    const float E = expf(-lam * tc);
    const int64_t o = (int64_t)b * kKC * kKC + k * kKC + c;
    const float vf = (float)v[i];
    if (raw) raw[o] = vf;
    scaled[o] = E * vf;
    if (want_gt) g = fma(-(double)lam * (double)E, (double)saved[o] * v[i], g);
  }
  if (write_t && b == 0 && tid < kKC) t[c] = tc;
  if (want_gt) {
    gsum[tid >> 6][c] = g;
    __syncthreads();  // also orders this block's partial reads before the overwrite below
    if (tid < kKC) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) a += gsum[q][c];
      part[(int64_t)b * S * kKC * kKC + c] = (float)a;
    }
  }
}

// pass 3: y[r, :] = Phi[r, :] · coef (· mass[r] if given). grid (ceil(N/64), B), block 256:
// 16 x 16 threads, 4 rows x 4 cols each.
// gtb (backward): block (0, 0) also sums the per-crop dL/dt partials in crop order into gt.
__global__ __launch_bounds__(256) void spec_expand_kernel(const float* __restrict__ evecs,
                                                          const float* __restrict__ coef,
                                                          const float* __restrict__ mass, int N,
                                                          float* __restrict__ y, int ldy, int accumulate,
                                                          const float* __restrict__ gtb, int64_t gt_stride,
                                                          float* __restrict__ gt) {
  __shared__ float4 scoef[kKC][kKC / 4];
  __shared__ float sphi[64][kKC + 1];
  const int tile = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int ty = tid >> 4, tx = tid & 15;
  if (gt && tile == 0 && b == 0 && tid < kKC) {
    float a = 0.f;
    for (int q = 0; q < (int)gridDim.y; ++q) a += gtb[(int64_t)q * gt_stride + tid];
    gt[tid] = a;
  }
  const float* __restrict__ cb = coef + (int64_t)b * kKC * kKC;
  {
    float4 cvv[kKC * kKC / 4 / 256];
#pragma unroll
    for (int j = 0; j < kKC * kKC / 4 / 256; ++j) cvv[j] = reinterpret_cast<const float4*>(cb)[tid + 256 * j];
#pragma unroll
    for (int j = 0; j < kKC * kKC / 4 / 256; ++j) scoef[(tid + 256 * j) / 16][(tid + 256 * j) % 16] = cvv[j];
  }
  const int r0 = tile * 64;
  const float* __restrict__ phi = evecs + (int64_t)b * N * kKC;
  {
    float4 pvv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // unconditional at clamped rows, then selected
      const int e = tid + 256 * j, rr = e / 16, q = e % 16;
      const int r = r0 + rr < N ? r0 + rr : r0;
      pvv[j] = reinterpret_cast<const float4*>(phi + (int64_t)r * kKC)[q];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + 256 * j, rr = e / 16, q = e % 16;
      const float4 v = r0 + rr < N ? pvv[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      sphi[rr][4 * q + 0] = v.x;
      sphi[rr][4 * q + 1] = v.y;
      sphi[rr][4 * q + 2] = v.z;
      sphi[rr][4 * q + 3] = v.w;
    }
  }
  // the epilogue's operands (mass, the accumulated output) in flight during the products
  float wr[4];
  float4 old[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty * 4 + i < N ? r0 + ty * 4 + i : r0;
    wr[i] = mass ? mass[(int64_t)b * N + r] : 1.f;
    old[i] = accumulate ? reinterpret_cast<const float4*>(y + ((int64_t)b * N + r) * ldy)[tx]
                        : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  float acc[4][4] = {};
#pragma unroll 8
  for (int k = 0; k < kKC; ++k) {
    const float4 cv = scoef[k][tx];
    const float cc[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = sphi[ty * 4 + i][k];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(p, cc[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty * 4 + i;
    if (r >= N) continue;
    const float w = wr[i];
    float4* yp = reinterpret_cast<float4*>(y + ((int64_t)b * N + r) * ldy) + tx;
    float4 v = make_float4(acc[i][0] * w, acc[i][1] * w, acc[i][2] * w, acc[i][3] * w);
    if (accumulate) {
      const float4 o = old[i];
      v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
    }
    *yp = v;
  }
}

// ---- Round 4: passes 1 and 3 on the f32 MFMA (v_mfma_f32_16x16x4_f32). The scalar-FMA forms
// above ran at 0.8-1.2 TB/s (0.10-0.15 of HBM) on these 8-17 MB passes; the products are 2 N K C
// flops per crop, small next to the bytes, so the MFMA forms are bound by the row streams.
// Lane map as in attention.hip: A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15],
// D[4 (l >> 4) + rr][l & 15]. Every lane loads whole float4s of a row, and the matrix indices are
// permuted to match (documented per kernel), so no operand goes through LDS shuffles.
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// pass 1: part[b, s] (64 x 64) over the kCPB x 64 rows of slab s; grid (S, B), block 256 = 4 waves.
// Per 64-row chunk, wave w contracts the 16 rows r0 + 16 w + 4 q + g (K-steps q < 4, g = l >> 4);
// lane (u = l & 15, g) loads the float4s Phi[r][4u .. 4u+3] and w_r x[r][4u .. 4u+3] once, the
// next chunk's loads in flight during this chunk's MFMAs. Tile (kt, ct) holds the output rows
// k = 4 i + kt (A = component kt of the Phi float4 of lane (i, g)) and columns c = 4 j + ct (B =
// component ct of the x float4 of lane (j, g)): register rr of tile (kt, ct) in lane (j, g) is the
// wave's part[4 (4 g + rr) + kt][4 j + ct], accumulated over the block's chunks in order. The four
// waves' 64 x 64 partials meet in LDS and are added in wave order. Round 5: kCPB = 4 chunks per
// block (was 1): the partial slabs written and re-read by the combine drop 4x (they were 0.5 B per
// input byte, the round-4 PMC excess of 1.8x the algorithmic bytes).
constexpr int kCPB = 4;
__global__ __launch_bounds__(256) void spec_reduce_mfma_kernel(const float* __restrict__ x, int ldx,
                                                               const float* __restrict__ mass,
                                                               const float* __restrict__ evecs, int N, int S,
                                                               float* __restrict__ part) {
  __shared__ float4 red[4][kKC * kKC / 4];  // [wave][k][c / 4]
  const int s = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, u = l & 15, g = l >> 4;
  const float* __restrict__ phi = evecs + (int64_t)b * N * kKC;
  const float* __restrict__ xb = x + (int64_t)b * N * ldx;
  const float* __restrict__ mb = mass ? mass + (int64_t)b * N : nullptr;
  const int r0 = s * kCPB * kRows;
  const int nch = min(kCPB, (N - r0 + kRows - 1) / kRows);  // chunks of this block (>= 1)
  float4 pv[4], xv[4];
  float wv[4];
  auto load = [&](int ch) {
    const int rw = r0 + ch * kRows + 16 * w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rw + 4 * q + g;
      const int rc = r < N ? r : N - 1;  // clamped, then zeroed
      pv[q] = reinterpret_cast<const float4*>(phi + (int64_t)rc * kKC)[u];
      xv[q] = reinterpret_cast<const float4*>(xb + (int64_t)rc * ldx)[u];
      wv[q] = mb ? mb[rc] : 1.f;
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[kt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int ch = 0; ch < nch; ++ch) {
    const int rw = r0 + ch * kRows + 16 * w;
    float a[4][4], xs[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = rw + 4 * q + g < N;
      const float wr = ok ? wv[q] : 0.f;
      a[q][0] = pv[q].x, a[q][1] = pv[q].y, a[q][2] = pv[q].z, a[q][3] = pv[q].w;
      xs[q][0] = mb ? xv[q].x * wr : (ok ? xv[q].x : 0.f);
      xs[q][1] = mb ? xv[q].y * wr : (ok ? xv[q].y : 0.f);
      xs[q][2] = mb ? xv[q].z * wr : (ok ? xv[q].z : 0.f);
      xs[q][3] = mb ? xv[q].w * wr : (ok ? xv[q].w : 0.f);
    }
    if (ch + 1 < nch) load(ch + 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[kt][ct] = mfma4(a[q][kt], xs[q][ct], acc[kt][ct]);
  }
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      red[w][(4 * (4 * g + rr) + kt) * (kKC / 4) + u] =
          make_float4(acc[kt][0][rr], acc[kt][1][rr], acc[kt][2][rr], acc[kt][3][rr]);
  __syncthreads();
  float4* __restrict__ o = reinterpret_cast<float4*>(part + ((int64_t)b * S + s) * kKC * kKC);
#pragma unroll
  for (int j = 0; j < kKC * kKC / 4 / 256; ++j) {
    const int e = tid + 256 * j;
    const float4 v0 = red[0][e], v1 = red[1][e], v2 = red[2][e], v3 = red[3][e];
    o[e] = make_float4(((v0.x + v1.x) + v2.x) + v3.x, ((v0.y + v1.y) + v2.y) + v3.y, ((v0.z + v1.z) + v2.z) + v3.z,
                       ((v0.w + v1.w) + v2.w) + v3.w);
  }
}

// pass 2 for the MFMA passes: spec_combine_kernel's sums over 4 x as many blocks (grid (B, 4),
// block 1024: thread (k = 16 y + (tid >> 6), c = tid & 63) sums its one coefficient over the S
// slabs in slab order, fp64, 8 slabs' loads in flight). gt (backward): block y's partial over its
// 16 rows k goes to row 16 y of its crop's slab 0 (read by this block only, consumed before the
// barrier); spec_expand_mfma_kernel adds the 4 per crop, then the crops, in order.
__global__ __launch_bounds__(1024) void spec_combine4_kernel(float* __restrict__ part, int S,
                                                             const float* __restrict__ evals,
                                                             float* __restrict__ t, int clamp_t, int write_t,
                                                             float* __restrict__ raw, float* __restrict__ scaled,
                                                             const float* __restrict__ saved, int want_gt) {
  __shared__ double gsum[16][kKC];
  const int b = blockIdx.x, y = blockIdx.y, tid = threadIdx.x;
  const int c = tid & 63, k = 16 * y + (tid >> 6);
  const float* pb = part + (int64_t)b * S * kKC * kKC + k * kKC + c;
  const float tc = clamp_t ? fmaxf(t[c], 1e-8f) : t[c];
  double v = 0.0;
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    float ld[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) ld[q] = pb[(int64_t)(s + q) * kKC * kKC];
#pragma unroll
    for (int q = 0; q < 8; ++q) v += (double)ld[q];
  }
  for (; s < S; ++s) v += (double)pb[(int64_t)s * kKC * kKC];
  const float lam = evals[b * kKC + k];
  const float E = expf(-lam * tc);
  const int64_t o = (int64_t)b * kKC * kKC + k * kKC + c;
  const float vf = (float)v;
  if (raw) raw[o] = vf;
  scaled[o] = E * vf;
  if (write_t && b == 0 && y == 0 && tid < kKC) t[c] = tc;
  if (want_gt) {
    gsum[tid >> 6][c] = -(double)lam * (double)E * ((double)saved[o] * v);
    __syncthreads();
    if (tid < kKC) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) a += gsum[q][c];
      part[(int64_t)b * S * kKC * kKC + (16 * y) * kKC + c] = (float)a;
    }
  }
}

// pass 3: y[r, :] = Phi[r, :] · coef (· mass[r]) (+ y). grid (ceil(N / 64), B), block 256: wave w
// owns the 16 rows r0 + 16 w + (0..15), all 64 columns (4 tiles). Lane (i = l & 15, g = l >> 4)
// loads Phi[r][16 t + 4 g .. +3] (t < 4), so K-step (t, e) pairs A[i][g] = Phi[r][16 t + 4 g + e]
// with B[g][j] = coef[16 t + 4 g + e][4 j + ct] (one ds_read_b128 of the LDS copy of coef gives
// all 4 tiles); D register rr of tile ct in lane (j, g) is y[r0 + 16 w + 4 g + rr][4 j + ct].
// FUSED (the forward): no combine launch — every block sums its crop's S partial slabs itself
// (fp64, slab order: spec_combine4_kernel's arithmetic, so raw / scaled are bit-identical),
// scales by exp(-lambda t) into its LDS copy of the coefficients, and the crop's block 0 writes
// raw (saved for the backward) and, for crop 0, the clamped diffusion time. The slabs are read
// from L2 (a crop's row blocks share an XCD), so the partials cross HBM once, when written.
struct SpecFuse {
  const float* part;
  int S, clamp_t, write_t, pad;
  const float* evals;
  float* t;
  float* raw;
};

template <bool FUSED>
__global__ __launch_bounds__(256) void spec_expand_mfma_kernel(const float* __restrict__ evecs,
                                                               const float* __restrict__ coef,
                                                               const float* __restrict__ mass, int N,
                                                               float* __restrict__ y, int ldy, int accumulate,
                                                               const float* __restrict__ gtb, int64_t gt_stride,
                                                               float* __restrict__ gt, SpecFuse fz) {
  __shared__ float4 scoef[kKC * kKC / 4];  // [k][c / 4]
  // a crop's row blocks on one XCD: its 16 KB of coefficients come from HBM once per crop, not
  // once per XCD (the round-5 PMC pass counted the re-fetches at ~15 MB per launch)
  const int3 lb = pk::xcd_block3();
  const int tile = lb.x, b = lb.y, tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, u = l & 15, g = l >> 4;
  if constexpr (FUSED) {
    // thread: coefficients (k, 4 c4 .. 4 c4 + 3) for e = tid + 256 j, k = e >> 4, c4 = e & 15
    constexpr int PER = kKC * kKC / 4 / 256;
    const float* pb = fz.part + (int64_t)b * fz.S * kKC * kKC;
    double v[PER][4];
#pragma unroll
    for (int j = 0; j < PER; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[j][q] = 0.0;
    for (int s0 = 0; s0 < fz.S; ++s0) {
      float4 ld[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) ld[j] = reinterpret_cast<const float4*>(pb + (int64_t)s0 * kKC * kKC)[tid + 256 * j];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        v[j][0] += (double)ld[j].x;
        v[j][1] += (double)ld[j].y;
        v[j][2] += (double)ld[j].z;
        v[j][3] += (double)ld[j].w;
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + 256 * j, k = e >> 4, c4 = e & 15;
      const float lam = fz.evals[b * kKC + k];
      float o[4], r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * c4 + q;
        const float tc = fz.clamp_t ? fmaxf(fz.t[c], 1e-8f) : fz.t[c];
        const float E = expf(-lam * tc);
        r[q] = (float)v[j][q];
        o[q] = E * r[q];
      }
      scoef[e] = make_float4(o[0], o[1], o[2], o[3]);
      if (tile == 0 && fz.raw != nullptr)
        reinterpret_cast<float4*>(fz.raw + (int64_t)b * kKC * kKC)[e] = make_float4(r[0], r[1], r[2], r[3]);
    }
    if (fz.write_t && tile == 0 && b == 0 && tid < kKC) fz.t[tid] = fmaxf(fz.t[tid], 1e-8f);
  } else {
    const float* __restrict__ cb = coef + (int64_t)b * kKC * kKC;
    float4 cv[kKC * kKC / 4 / 256];
#pragma unroll
    for (int j = 0; j < kKC * kKC / 4 / 256; ++j) cv[j] = reinterpret_cast<const float4*>(cb)[tid + 256 * j];
#pragma unroll
    for (int j = 0; j < kKC * kKC / 4 / 256; ++j) scoef[tid + 256 * j] = cv[j];
  }
  const int rw = tile * 64 + 16 * w;  // this wave's first row
  const float* __restrict__ phi = evecs + (int64_t)b * N * kKC;
  float4 pv[4];
  {
    const int r = rw + u < N ? rw + u : N - 1;
#pragma unroll
    for (int t = 0; t < 4; ++t) pv[t] = reinterpret_cast<const float4*>(phi + (int64_t)r * kKC)[4 * t + g];
  }
  // the epilogue's operands in flight during the products
  float wr[4];
  float4 old[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = rw + 4 * g + rr < N ? rw + 4 * g + rr : N - 1;
    wr[rr] = mass ? mass[(int64_t)b * N + r] : 1.f;
    old[rr] = accumulate ? reinterpret_cast<const float4*>(y + ((int64_t)b * N + r) * ldy)[u]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float pa[4] = {pv[t].x, pv[t].y, pv[t].z, pv[t].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float4 bv = scoef[(16 * t + 4 * g + e) * (kKC / 4) + u];
      acc[0] = mfma4(pa[e], bv.x, acc[0]);
      acc[1] = mfma4(pa[e], bv.y, acc[1]);
      acc[2] = mfma4(pa[e], bv.z, acc[2]);
      acc[3] = mfma4(pa[e], bv.w, acc[3]);
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = rw + 4 * g + rr;
    if (r >= N) continue;
    const float m = wr[rr];
    float4 v = make_float4(acc[0][rr] * m, acc[1][rr] * m, acc[2][rr] * m, acc[3][rr] * m);
    if (accumulate) {
      const float4 o = old[rr];
      v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
    }
    reinterpret_cast<float4*>(y + ((int64_t)b * N + r) * ldy)[u] = v;
  }
  // after this block's rows: one block sums dL/dt, off the other blocks' critical path
  if (gt && tile == 0 && b == 0 && tid < kKC) {  // spec_combine4_kernel's 4 partials per crop
    float a = 0.f;
    const int nq = (int)gridDim.y;
    for (int q0 = 0; q0 < nq; q0 += 8) {  // 8 crops' 32 loads in flight, added in crop order
      float v[8][4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float* gq = gtb + (int64_t)(q0 + q < nq ? q0 + q : q0) * gt_stride + tid;
#pragma unroll
        for (int y = 0; y < 4; ++y) v[q][y] = gq[16 * kKC * y];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q0 + q < nq) a += ((v[q][0] + v[q][1]) + v[q][2]) + v[q][3];
    }
    gt[tid] = a;
  }
}

#ifdef PK_DEVBUILD
static bool spec_scalar() {  // PK_SPEC_SCALAR=1: round 1's scalar-FMA passes 1 and 3 (A/B)
  static const bool v = getenv("PK_SPEC_SCALAR") != nullptr && atoi(getenv("PK_SPEC_SCALAR")) != 0;
  return v;
}
#else
constexpr bool spec_scalar() { return false; }
#endif

}  // namespace

// mode 0 (forward): in = x, out = y, raw = spec (saved for backward), reduce weights = mass.
// mode 1 (backward): in = g, out = gx, saved = spec from forward, gt = dL/dt [C] summed over
//                    crops; expand weights = mass.
extern "C" int pk_spectral_diffusion(const float* in, int ld_in, const float* mass, const float* evecs,
                                     const float* evals, float* t, int clamp_t, int B, int N, int K, int C,
                                     int mode, float* work, float* raw, float* scaled, const float* saved,
                                     float* gt, float* out, int ld_out, int accumulate, void* stream) {
  PK_REQUIRE(B >= 0 && N >= 0 && K == kKC && C == kKC && (mode == 0 || mode == 1));
  PK_REQUIRE(ld_in >= C && ld_out >= C && ld_in % 4 == 0 && ld_out % 4 == 0);
  if (B == 0 || N == 0) return PK_OK;
  PK_REQUIRE(in && evecs && evals && t && work && scaled && out);
  PK_REQUIRE(mode == 0 || (saved && gt));
  hipStream_t s = pk::as_stream(stream);
  // slabs per crop: 64 rows each for the scalar passes, kCPB x 64 for the MFMA reduce
  const int S = spec_scalar() ? (N + kRows - 1) / kRows : (N + kCPB * kRows - 1) / (kCPB * kRows);
  if (spec_scalar())
    hipLaunchKernelGGL(spec_reduce_kernel, dim3(S, B), dim3(256), 0, s, in, ld_in, mode == 0 ? mass : nullptr,
                       evecs, N, S, work);
  else
    hipLaunchKernelGGL(spec_reduce_mfma_kernel, dim3(S, B), dim3(256), 0, s, in, ld_in,
                       mode == 0 ? mass : nullptr, evecs, N, S, work);
  PK_CHECK_LAUNCH();
  if (!spec_scalar() && mode == 0) {  // forward: the combine inside the expand (no third launch)
    SpecFuse fz{work, S, clamp_t, (int)(clamp_t != 0), 0, evals, t, raw};
    hipLaunchKernelGGL(spec_expand_mfma_kernel<true>, dim3((N + 63) / 64, B), dim3(256), 0, s, evecs, scaled,
                       nullptr, N, out, ld_out, accumulate, work, (int64_t)S * kKC * kKC, nullptr, fz);
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  if (spec_scalar())
    hipLaunchKernelGGL(spec_combine_kernel, dim3(B), dim3(1024), 0, s, work, S, evals, t, clamp_t,
                       (int)(clamp_t && mode == 0), raw, scaled, mode == 1 ? saved : nullptr, (int)(mode == 1));
  else
    hipLaunchKernelGGL(spec_combine4_kernel, dim3(B, 4), dim3(1024), 0, s, work, S, evals, t, clamp_t,
                       (int)(clamp_t && mode == 0), raw, scaled, mode == 1 ? saved : nullptr, (int)(mode == 1));
  PK_CHECK_LAUNCH();
  if (spec_scalar())
    hipLaunchKernelGGL(spec_expand_kernel, dim3((N + 63) / 64, B), dim3(256), 0, s, evecs, scaled,
                       mode == 1 ? mass : nullptr, N, out, ld_out, accumulate, work, (int64_t)S * kKC * kKC,
                       mode == 1 ? gt : nullptr);
  else
    hipLaunchKernelGGL(spec_expand_mfma_kernel<false>, dim3((N + 63) / 64, B), dim3(256), 0, s, evecs, scaled,
                       mode == 1 ? mass : nullptr, N, out, ld_out, accumulate, work, (int64_t)S * kKC * kKC,
                       mode == 1 ? gt : nullptr, SpecFuse{});
  PK_CHECK_LAUNCH();
  return PK_OK;
}
