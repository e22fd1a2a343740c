// Weight / bias gradients of the per-point layers of H7 / H8 (DiffusionNet MiniMLP and
// first/last_lin, models/dpfm.py:22-30; refinement Conv1d(k=1) projections and MLPs,
// modeling/dpfm.py:16-26, 45-54, 63, 82-95, 120-130):
//     dW[o, i] = sum_r dY[r, o] X[r, i],   db[o] = sum_r dY[r, o]
// over every point of every crop (r = B * N rows, 32768-65536 per call) into a tiny
// [O <= 128, I <= 128] result. A library GEMM tiles the output (a handful of tiles) and
// walks all rows serially; here the rows are split into 128-row slices, one workgroup per
// slice, each contracting its slice on the f32 MFMA (v_mfma_f32_16x16x4f32: exact f32
// products, f32 accumulation) into a partial [O, I]; a second pass sums the partials in
// slice order (deterministic).
//
// Layouts: 0 = rows x channels ([R, C] row-major, nn.Linear), 1 = channels-first
// ([Bn, C, N], Conv1d with kernel 1; row r = (r / N, r % N)).
#include "common.hpp"
#include "../../include/posekern.h"

#include <cstdlib>
#include <vector>

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kChunk = 32;          // rows staged per step (8 MFMA k-steps)
constexpr int kSlice = 128;         // rows per workgroup
constexpr int kMaxC = 128;          // I, O <= 128
constexpr int kStride = kMaxC + 16; // LDS row stride (mod 64 = 16: conflict-free A/B reads)
constexpr int kMaxTilesPerWave = 8;  // O * I <= 128 * 64

__device__ __forceinline__ float load_rc(const float* __restrict__ p, int layout, int C, int N, int64_t r,
                                         int c) {
  if (layout == 0) return p[r * C + c];
  const int64_t b = r / N, n = r - b * N;
  return p[(b * C + c) * N + n];
}

// Stage rows [r0, r0 + kChunk) of a [R, C] operand into s[row][c] (zero padded). All
// global loads of the chunk are issued before the first LDS store (one wait per chunk).
__device__ __forceinline__ void stage_rows(const float* __restrict__ p, int layout, int C, int N, int64_t R,
                                           int64_t r0, float* __restrict__ s) {
  const int cp = (C + 15) & ~15;
  const int total = kChunk * cp;
  constexpr int kPer = kChunk * kMaxC / 256;
  float v[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = threadIdx.x + q * 256;
    const int row = layout == 0 ? e / cp : e % kChunk;  // channels-first: threads walk rows
    const int c = layout == 0 ? e % cp : e / kChunk;    // (contiguous in memory)
    const int64_t r = r0 + row;
    v[q] = (e < total && c < C && r < R) ? load_rc(p, layout, C, N, r, c) : 0.f;
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = threadIdx.x + q * 256;
    const int row = layout == 0 ? e / cp : e % kChunk;
    const int c = layout == 0 ? e % cp : e / kChunk;
    if (e < total) s[row * kStride + c] = v[q];
  }
}

__global__ __launch_bounds__(256) void wgrad_partial_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ dy, int layout,
                                                            int64_t R, int I, int O, int N,
                                                            float* __restrict__ part,
                                                            float* __restrict__ partb) {
  __shared__ float Xs[kChunk * kStride];
  __shared__ float Ys[kChunk * kStride];
  const int s = blockIdx.x;
  const int lane = pk::lane_id(), g = lane >> 4, c = lane & 15, w = pk::wave_id();
  const int It = (I + 15) >> 4, Ot = (O + 15) >> 4, T = It * Ot;
  f32x4 acc[kMaxTilesPerWave];
#pragma unroll
  for (int j = 0; j < kMaxTilesPerWave; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const int64_t r_begin = (int64_t)s * kSlice;
  const int64_t r_end = r_begin + kSlice < R ? r_begin + kSlice : R;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kChunk) {
    __syncthreads();
    stage_rows(x, layout, I, N, r_end, r0, Xs);
    stage_rows(dy, layout, O, N, r_end, r0, Ys);
    __syncthreads();
    if (threadIdx.x < O) {
#pragma unroll 8
      for (int r = 0; r < kChunk; ++r) bacc += Ys[r * kStride + threadIdx.x];
    }
#pragma unroll
    for (int j = 0; j < kMaxTilesPerWave; ++j) {
      const int t = w + 4 * j;
      if (t < T) {
        const int to = t / It, ti = t - to * It;
#pragma unroll
        for (int k = 0; k < kChunk / 4; ++k) {
          const float a = Ys[(4 * k + g) * kStride + to * 16 + c];  // dY^T [o][r]
          const float b = Xs[(4 * k + g) * kStride + ti * 16 + c];  // X [r][i]
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        }
      }
    }
  }
  float* __restrict__ ps = part + (int64_t)s * O * I;
#pragma unroll
  for (int j = 0; j < kMaxTilesPerWave; ++j) {
    const int t = w + 4 * j;
    if (t < T) {
      const int to = t / It, ti = t - to * It;
      const int i = ti * 16 + c;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int o = to * 16 + 4 * g + rr;
        if (o < O && i < I) ps[o * I + i] = acc[j][rr];
      }
    }
  }
  if (threadIdx.x < O) partb[(int64_t)s * O + threadIdx.x] = bacc;
}

// dw[e] = sum_s part[s, e] (e < O*I), db[o] = sum_s partb[s, o]. Block = 64 outputs x
// 16 slice groups (two interleaved chains each), combined by a fixed pairwise tree:
// deterministic, and 16 loads in flight per output instead of a serial walk over S.
constexpr int kRedGroups = 16;
__global__ __launch_bounds__(64 * kRedGroups) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                                       const float* __restrict__ partb, int S,
                                                                       int OI, int O, float* __restrict__ dw,
                                                                       float* __restrict__ db, int accumulate) {
  __shared__ float red[kRedGroups][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const bool is_w = e < OI;
  const bool is_b = !is_w && e < OI + O && db != nullptr;
  float v = 0.f;
  if (is_w || is_b) {
    const float* p = is_w ? part + e : partb + (e - OI);
    const int64_t st = is_w ? OI : O;
    const int s0 = (S * grp) / kRedGroups, s1 = (S * (grp + 1)) / kRedGroups;
    float a0 = 0.f, a1 = 0.f;
    int s = s0;
    for (; s + 2 <= s1; s += 2) {
      a0 += p[(int64_t)s * st];
      a1 += p[(int64_t)(s + 1) * st];
    }
    if (s < s1) a0 += p[(int64_t)s * st];
    v = a0 + a1;
  }
  red[grp][threadIdx.x & 63] = v;
  __syncthreads();
#pragma unroll
  for (int half = kRedGroups / 2; half >= 1; half >>= 1) {
    if (grp < half) red[grp][threadIdx.x & 63] += red[grp + half][threadIdx.x & 63];
    __syncthreads();
  }
  if (grp == 0 && (is_w || is_b)) {
    const float r = red[0][threadIdx.x & 63];
    float* dst = is_w ? dw + e : db + (e - OI);
    *dst = accumulate ? *dst + r : r;  // += : a weight used by several layers' calls
  }
}

// ---------------------------------------------------------------------------------
// Direct-load variant (the default): v_mfma_f32_32x32x2_f32 takes its operands straight
// from global memory, no LDS staging and no barriers in the row loop.
//   A[m][k] = dY[row k][o0 + m], B[k][n] = X[row k][i0 + n]  ->  D = dW tile [32 x 32]
// Lane l supplies A[l & 31][l >> 5] and B[l >> 5][l & 31], i.e. one value of row
// r(step, h = l >> 5) at channel (l & 31). Rows are taken in batches of 16 (8 k-steps):
//   layout 0 ([R, C]): r = rb + 2 s + h       (32 lanes read 128 contiguous bytes)
//   layout 1 ([Bn, C, N]): r = rb + 8 h + s  (a lane's 8 rows are 8 consecutive n of one
//            channel: two 16-byte loads when N % 16 == 0, else 8 scalar loads with the tail
//            rows past the slice end read as 0)
// Both operands use the same r(s, h), so the contraction is the same sum over rows.
// Workgroup = one row slice; its 4 waves split the 32x32 output tiles (T = To * Ti <= 16)
// and, when there are fewer than 4 tiles, the slice's batches; wave row groups are
// combined through LDS in a fixed order (deterministic). Bias = row sums of the A values
// of the tiles with ti == 0.
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int LAYOUT>
__device__ __forceinline__ void load8(const float* __restrict__ p, int C, int c, int N, int64_t rb, int64_t r1,
                                      int h, float (&v)[8], int64_t sb) {
  if (LAYOUT == 0) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t r = rb + 2 * s + h;
      v[s] = (c < C && r < r1) ? p[r * C + c] : 0.f;
    }
  } else if (N & 15) {  // ragged items (N % 16 != 0): a 16-row batch may straddle two items
    const int64_t cs = sb ? sb : (int64_t)C * N;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int64_t r = rb + 8 * h + s;
      const int64_t b = r / N;
      v[s] = (c < C && r < r1) ? p[b * cs + (int64_t)c * N + (r - b * N)] : 0.f;
    }
  } else {
    if (c < C) {  // batch stride sb (0: dense C N)
      const int64_t b = rb / N;
      const int64_t n = rb - b * N + 8 * h;
      const float4* q = reinterpret_cast<const float4*>(p + b * (sb ? sb : (int64_t)C * N) + (int64_t)c * N + n);
      const float4 u = q[0], w = q[1];
      v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
      v[4] = w.x; v[5] = w.y; v[6] = w.z; v[7] = w.w;
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = 0.f;
    }
  }
}

// Operands of one 16-row batch for a wave's J tiles.
template <int J>
struct WgradBatch {
  float a[J][8], b[J][8];
};

template <int LAYOUT, int J>
__device__ __forceinline__ void wgrad_load(WgradBatch<J>& B, const float* __restrict__ x, const float* __restrict__ dy,
                                           int I, int O, int N, int Ti, int T, int tw, int WT, int m, int h,
                                           int64_t rb, int64_t r1, int64_t sbx, int64_t sbdy) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = tw + WT * j;
    if (t < T) {
      const int to = t / Ti, ti = t - to * Ti;
      load8<LAYOUT>(dy, O, to * 32 + m, N, rb, r1, h, B.a[j], sbdy);
      load8<LAYOUT>(x, I, ti * 32 + m, N, rb, r1, h, B.b[j], sbx);
    }
  }
}

template <int J>
__device__ __forceinline__ void wgrad_mma(const WgradBatch<J>& B, f32x16 (&acc)[J], float (&bs)[J], int Ti, int T,
                                          int tw, int WT) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = tw + WT * j;
    if (t < T) {
#pragma unroll
      for (int st = 0; st < 8; ++st) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(B.a[j][st], B.b[j][st], acc[j], 0, 0, 0);
      if (t % Ti == 0) {
#pragma unroll
        for (int st = 0; st < 8; ++st) bs[j] += B.a[j][st];
      }
    }
  }
}

// 8 waves per workgroup: WT = min(T, 8) tile lanes x WR = 8 / WT row groups; J tiles per
// wave (J = 2 only for T = 16). The next batch's loads are issued before the current
// batch's MFMAs (two register buffers, statically indexed).
constexpr int kV2Waves = 8;

// Slice s of one problem; comb / combb: the workgroup's [kV2Waves][16 * 64] / [kV2Waves][64]
// LDS (declared by the calling kernel, so a kernel instantiating both layouts allocates it once).
template <int LAYOUT, int J>
__device__ __forceinline__ void wgrad_v2_body(const float* __restrict__ x, const float* __restrict__ dy, int64_t R,
                                              int I, int O, int N, int SL, float* __restrict__ part,
                                              float* __restrict__ partb, int s, float (*comb)[16 * 64],
                                              float (*combb)[64], int64_t sbx, int64_t sbdy) {
  const int lane = pk::lane_id(), w = pk::wave_id();
  const int m = lane & 31, h = lane >> 5;
  const int To = (O + 31) >> 5, Ti = (I + 31) >> 5, T = To * Ti;
  const int WT = T < kV2Waves ? T : kV2Waves;
  const int WR = kV2Waves / WT;
  const int tw = w % WT, g = w / WT;
  const bool active = g < WR;
  f32x16 acc[J];
  float bs[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    bs[j] = 0.f;
  }
  const int64_t r0 = (int64_t)s * SL;
  const int64_t r1 = r0 + SL < R ? r0 + SL : R;
  const int nb = (int)((r1 - r0 + 15) / 16);
  if (active) {
    WgradBatch<J> b0, b1;
    int q = g;
    if (q < nb) wgrad_load<LAYOUT, J>(b0, x, dy, I, O, N, Ti, T, tw, WT, m, h, r0 + 16ll * q, r1, sbx, sbdy);
    for (; q < nb; q += 2 * WR) {
      const bool has1 = q + WR < nb;
      if (has1) wgrad_load<LAYOUT, J>(b1, x, dy, I, O, N, Ti, T, tw, WT, m, h, r0 + 16ll * (q + WR), r1, sbx, sbdy);
      wgrad_mma<J>(b0, acc, bs, Ti, T, tw, WT);
      if (has1) {
        if (q + 2 * WR < nb)
          wgrad_load<LAYOUT, J>(b0, x, dy, I, O, N, Ti, T, tw, WT, m, h, r0 + 16ll * (q + 2 * WR), r1, sbx, sbdy);
        wgrad_mma<J>(b1, acc, bs, Ti, T, tw, WT);
      }
    }
  }
  // combine row groups (only when WT < 8, i.e. one tile per wave) in group order
  if (WR > 1) {
    if (active) {
#pragma unroll
      for (int e = 0; e < 16; ++e) comb[w][e * 64 + lane] = acc[0][e];
      combb[w][lane] = bs[0];
    }
    __syncthreads();
    if (!active || g != 0) return;
    for (int gg = 1; gg < WR; ++gg) {
      const int src = tw + WT * gg;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[0][e] += comb[src][e * 64 + lane];
      bs[0] += combb[src][lane];
    }
  }
  if (!active) return;
  float* __restrict__ ps = part + (int64_t)s * O * I;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = tw + WT * j;
    if (t < T) {
      const int to = t / Ti, ti = t - to * Ti;
      const int i = ti * 32 + m;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = to * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (o < O && i < I) ps[(int64_t)o * I + i] = acc[j][e];
      }
      if (ti == 0) {
        const float tot = bs[j] + __shfl_xor(bs[j], 32);  // the two row halves
        const int o = to * 32 + m;
        if (h == 0 && o < O) partb[(int64_t)s * O + o] = tot;
      }
    }
  }
}

template <int LAYOUT, int J>
__global__ __launch_bounds__(64 * kV2Waves) void wgrad_v2_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ dy, int64_t R, int I,
                                                                 int O, int N, int SL, float* __restrict__ part,
                                                                 float* __restrict__ partb) {
  __shared__ float comb[kV2Waves][16 * 64];
  __shared__ float combb[kV2Waves][64];
  wgrad_v2_body<LAYOUT, J>(x, dy, R, I, O, N, SL, part, partb, blockIdx.x, comb, combb, 0, 0);
}

// ---------------------------------------------------------------------------------
// Grouped weight gradients: every per-point layer of a backward pass in two launches
// (partials, then reduction) instead of two launches per layer. The problem tables travel
// as kernel arguments (captured into a HIP graph node by value). Block b belongs to the
// problem whose [blk0, blk0 + S) holds b; each problem runs the same slice body as
// pk_linear_wgrad. An output fed by two calls of one forward (a shared layer) reduces both
// partial sets, first call first: r = reduce(seg 0) + reduce(seg 1), the same rounding as
// autograd's grad = grad_0 + grad_1.
constexpr int kGroupMax = 32;

struct WgradProblem {
  const float* x;
  const float* dy;
  float* part;   // S * O * I weight partials, then S * O bias partials
  int64_t R;
  int I, O, N, layout, SL, S, blk0, pad;  // pad: the pipeline kernel's development variant (0)
  int64_t sbx, sbdy;  // channels-first batch strides (0: dense)
};
struct WgradProblems {
  int G;
  WgradProblem p[kGroupMax];
};

__global__ __launch_bounds__(64 * kV2Waves) void wgrad_grouped_kernel(const WgradProblems tab) {
  __shared__ float comb[kV2Waves][16 * 64];
  __shared__ float combb[kV2Waves][64];
  const int b = blockIdx.x;
  int g = 0;
  while (g + 1 < tab.G && b >= tab.p[g + 1].blk0) ++g;  // block-uniform scan (G <= 32)
  const WgradProblem& P = tab.p[g];
  const int s = b - P.blk0;
  float* partb = P.part + (int64_t)P.S * P.O * P.I;
  if (P.layout == 0) wgrad_v2_body<0, 1>(P.x, P.dy, P.R, P.I, P.O, P.N, P.SL, P.part, partb, s, comb, combb, 0, 0);
  else wgrad_v2_body<1, 1>(P.x, P.dy, P.R, P.I, P.O, P.N, P.SL, P.part, partb, s, comb, combb, P.sbx, P.sbdy);
}

struct WgradOut {
  const float* part[2];  // partial sets of the (up to two) calls feeding this output
  float* dw;
  float* db;
  int S[2];
  int nseg, OI, O, blk0;
};
struct WgradOuts {
  int G;
  WgradOut p[kGroupMax];
};

// The tree of wgrad_reduce_kernel for output element e of one partial set (all threads of
// the block call it; red = the block's [kRedGroups][64] LDS).
__device__ __forceinline__ float wgrad_tree(const float* __restrict__ part, int S, int OI, int O, int e,
                                            float (*red)[64]) {
  const int grp = threadIdx.x >> 6;
  const bool is_w = e < OI, is_b = !is_w && e < OI + O;
  float v = 0.f;
  if (is_w || is_b) {
    const float* p = is_w ? part + e : part + (int64_t)S * OI + (e - OI);
    const int64_t st = is_w ? OI : O;
    const int s0 = (S * grp) / kRedGroups, s1 = (S * (grp + 1)) / kRedGroups;
    float a0 = 0.f, a1 = 0.f;
    int s = s0;
    for (; s + 2 <= s1; s += 2) {
      a0 += p[(int64_t)s * st];
      a1 += p[(int64_t)(s + 1) * st];
    }
    if (s < s1) a0 += p[(int64_t)s * st];
    v = a0 + a1;
  }
  __syncthreads();  // red reused across calls
  red[grp][threadIdx.x & 63] = v;
  __syncthreads();
#pragma unroll
  for (int half = kRedGroups / 2; half >= 1; half >>= 1) {
    if (grp < half) red[grp][threadIdx.x & 63] += red[grp + half][threadIdx.x & 63];
    __syncthreads();
  }
  return red[0][threadIdx.x & 63];
}

__global__ __launch_bounds__(64 * kRedGroups) void wgrad_grouped_reduce_kernel(const WgradOuts tab) {
  __shared__ float red[kRedGroups][64];
  const int b = blockIdx.x;
  int g = 0;
  while (g + 1 < tab.G && b >= tab.p[g + 1].blk0) ++g;
  const WgradOut& P = tab.p[g];
  const int e = (b - P.blk0) * 64 + (threadIdx.x & 63);
  float r = wgrad_tree(P.part[0], P.S[0], P.OI, P.O, e, red);
  if (P.nseg > 1) r = r + wgrad_tree(P.part[1], P.S[1], P.OI, P.O, e, red);
  if ((threadIdx.x >> 6) == 0 && e < P.OI + P.O) {
    if (e < P.OI) P.dw[e] = r;
    else if (P.db) P.db[e - P.OI] = r;
  }
}

// Rows per slice of a grouped problem: ~kGroupSlices slices (whole 16-row batches, >= 128
// rows); the group supplies the parallelism the single-layer launch gets from ~320 slices.
constexpr int kGroupSlices = 64;
inline int64_t grouped_slice_rows(int64_t R) {
  int64_t SL = (R + kGroupSlices - 1) / kGroupSlices;
  SL = (SL + 15) / 16 * 16;
  return SL < kSlice ? kSlice : SL;
}

}  // namespace

#ifdef PK_DEVBUILD
// Development hook (not in include/posekern.h): the LDS-staged slice kernel, for A/B timing.
extern "C" int pkdev_linear_wgrad_v1(const float* x, const float* dy, int layout, int64_t R, int I, int O, int N,
                                     float* work, float* dw, float* db, void* stream) {
  hipStream_t s = pk::as_stream(stream);
  const int S = (int)((R + kSlice - 1) / kSlice);
  if (S == 0) return PK_ERR_ARG;
  float* part = work;
  float* partb = work + (int64_t)S * O * I;
  hipLaunchKernelGGL(wgrad_partial_kernel, dim3(S), dim3(256), 0, s, x, dy, layout, R, I, O, N, part, partb);
  PK_CHECK_LAUNCH();
  const int total = O * I + O;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(64 * kRedGroups), 0, s, part, partb, S, O * I, O,
                     dw, db, 0);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
#endif  // PK_DEVBUILD

extern "C" int pk_linear_wgrad(const float* x, const float* dy, int layout, int64_t R, int I, int O, int N,
                               float* work, float* dw, float* db, int accumulate, void* stream) {
  PK_REQUIRE((layout == 0 || layout == 1) && R >= 0 && I > 0 && O > 0 && I <= kMaxC && O <= kMaxC);
  PK_REQUIRE(layout == 0 || N > 0);
  PK_REQUIRE(((I + 15) / 16) * ((O + 15) / 16) <= 4 * kMaxTilesPerWave);
  PK_REQUIRE(dw != nullptr);
  hipStream_t s = pk::as_stream(stream);
  const int S = (int)((R + kSlice - 1) / kSlice);
  if (S == 0) {
    if (accumulate) return PK_OK;  // no rows: nothing to add
    hipError_t e = pk::zero_async(dw, sizeof(float) * O * I, s);
    if (e == hipSuccess && db) e = pk::zero_async(db, sizeof(float) * O, s);
    return e == hipSuccess ? PK_OK : (int)e;
  }
  PK_REQUIRE(x && dy && work);
  float* part = work;
  // direct-load kernel: slices of >= 128 rows (so S never exceeds the documented work
  // size), ~320 slices for the large calls
  int S2;
  {
    int64_t SL = (R + 319) / 320;
    SL = (SL + 15) / 16 * 16;
    if (SL < kSlice) SL = kSlice;
    S2 = (int)((R + SL - 1) / SL);
    float* partb = work + (int64_t)S2 * O * I;
    const int T = ((O + 31) / 32) * ((I + 31) / 32);
    const int J = T <= kV2Waves ? 1 : 2;
#define PK_WGRAD_V2(L, JJ)                                                                                   \
  hipLaunchKernelGGL((wgrad_v2_kernel<L, JJ>), dim3(S2), dim3(64 * kV2Waves), 0, s, x, dy, R, I, O, N, (int)SL, \
                     part, partb)
    if (layout == 0) {
      if (J == 1) PK_WGRAD_V2(0, 1);
      else PK_WGRAD_V2(0, 2);
    } else {
      if (J == 1) PK_WGRAD_V2(1, 1);
      else PK_WGRAD_V2(1, 2);
    }
#undef PK_WGRAD_V2
  }
  PK_CHECK_LAUNCH();
  const int total = O * I + O;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(64 * kRedGroups), 0, s, part,
                     work + (int64_t)S2 * O * I, S2, O * I, O, dw, db, accumulate);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

namespace {

// ---------------------------------------------------------------------------------
// Per-point layer products (forward and input gradient) of the same layers:
//   forward   y = x W^T (+ b) (then ReLU if asked)       W [O, I]
//   dgrad     dx = dy W            (= the forward with the weight transposed, no bias)
// in both layouts (0: [R, C] rows, nn.Linear; 1: [Bn, C, N], Conv1d(k=1)). I, O <= 128.
// One wave computes 32 points x all outputs on v_mfma_f32_32x32x2_f32 (up to four 32x32
// accumulators); the weight sits in LDS, the points' operands are loaded straight from
// global memory once. Contraction index k is split in halves across the lane halves
// (k = h * KH + s at step s), so a lane reads one contiguous half-row (layout 0) or the
// same column of KH consecutive channel rows (layout 1, 128-B coalesced across lanes).
// Replaces the library GEMM + separate bias / transpose kernels of these tall-skinny
// shapes (32k-65k points x <= 128 channels).
constexpr int kLfMaxC = 128;
// rows kernel grid cap (development knob PK_ROWS_BLOCKS at build time; 4 waves per block)
#ifndef PK_ROWS_BLOCKS
#define PK_ROWS_BLOCKS 4096
#endif
constexpr int kRowsMaxBlocks = PK_ROWS_BLOCKS;
constexpr int kRowsPersistCUs = 256;  // persistent rows grid: 2 blocks per CU of MI355X

// ReLU backward folded into an input-gradient epilogue: mask = the forward output of the layer
// whose gradient this is (aten threshold_backward(grad, mask, 0): mask <= 0 -> 0)
__device__ __forceinline__ float relu_mask(float v, const float* __restrict__ mask, int64_t i) {
  return (mask != nullptr && mask[i] <= 0.f) ? 0.f : v;
}

// Output side of a per-point layer launch (pk_linear_ex): where y goes and what the epilogue
// folds in. Strides are element strides: rows layout — row stride; channels-first — batch
// stride (the channel stride is N). v = acc + bias; ReLU; mask (contiguous, the ReLU backward
// of the producing layer); + add (columns < add_cols); then stored to y (columns < split) or
// y2 (columns >= split, at column - split), or channels-first when store_cf (rows kernels).
struct LinEpi {
  float* y;
  int64_t sy;
  float* y2;
  int64_t sy2;
  int split;
  const float* add;
  int64_t sa;
  int add_cols;
  const float* mask;
  int relu;  // 0 none, 1 ReLU, 2 sigmoid (1 / (1 + exp(-v)))
  int store_cf;
  int N;
  const float* pre;  // thin kernels: input x scaled by pre (1 - pre) first (sigmoid backward)
  float* pre_out;    // ... and that scaled input written here (same indexing as x)
  const float* add2;  // channels-first kernels: a second added operand (every output), batch stride sa2
  int64_t sa2;
  const float* w2;    // stacked weight rows >= wsplit (lr_stage), and bias entries >= wsplit from bias2
  const float* bias2;
  int wsplit;
};

__device__ __forceinline__ float lin_act(int act, float v) {
  return act == 1 ? fmaxf(v, 0.f) : act == 2 ? 1.f / (1.f + expf(-v)) : v;
}

__device__ __forceinline__ float lin_epi(const LinEpi& e, float v, int64_t mask_i) {
  return relu_mask(lin_act(e.relu, v), e.mask, mask_i);
}

// rows-layout store of output column o of point r (Cout outputs per point)
__device__ __forceinline__ void lin_store_row(const LinEpi& e, int64_t r, int o, int Cout, float v) {
  v = lin_epi(e, v, r * Cout + o);
  if (e.add != nullptr && o < e.add_cols) v += e.add[r * e.sa + o];
  if (e.store_cf) {
    const int64_t b = r / e.N, n = r - b * e.N;
    e.y[b * e.sy + (int64_t)o * e.N + n] = v;
  } else if (o >= e.split) {
    e.y2[r * e.sy2 + (o - e.split)] = v;
  } else {
    e.y[r * e.sy + o] = v;
  }
}

template <int LAYOUT>
__global__ __launch_bounds__(256) void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ bias, int64_t R, int N, int Cin,
                                                         int Cout, int transw, int relu, const float* __restrict__ mask,
    float* __restrict__ y) {
  // weight as Ws[out][k], out < Cout, k < KP (zero padded); row stride KP + 1 (odd);
  // dynamic LDS of Cout * (KP + 1) floats (<= 64.5 KiB)
  extern __shared__ float Ws[];
  const int KP = (Cin + 3) & ~3, KH = KP >> 1, ST = KP + 1;
  for (int e = threadIdx.x; e < Cout * KP; e += 256) {
    const int o = e / KP, k = e - o * KP;
    float v = 0.f;
    if (k < Cin) v = transw ? w[(int64_t)k * Cout + o] : w[(int64_t)o * Cin + k];
    Ws[o * ST + k] = v;
  }
  __syncthreads();
  const int lane = pk::lane_id(), wave = pk::wave_id();
  const int m = lane & 31, h = lane >> 5;
  const int TO = (Cout + 31) >> 5;
  // 32 points per wave: rows r0 .. r0 + 31 of the flattened point index
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 32;
  if (r0 >= R) return;
  const int64_t r = r0 + m;  // this lane's point (its A / B operand column)
  const bool ok = r < R;
  int64_t bb = 0, nn = 0;
  if (LAYOUT == 1) {
    bb = r / N;
    nn = r - bb * N;
  }
  float xa[kLfMaxC / 2];
#pragma unroll
  for (int s = 0; s < kLfMaxC / 2; ++s) {
    if (s < KH) {
      const int k = h * KH + s;
      float v = 0.f;
      if (ok && k < Cin) v = LAYOUT == 0 ? x[r * Cin + k] : x[(bb * Cin + k) * N + nn];
      xa[s] = v;
    }
  }
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  // layout 0: D[point m][out n] = sum_k x[m][k] W[n][k]  (A = points, B = weight)
  // layout 1: D[out m][point n] = sum_k W[m][k] x[k][n]  (A = weight, B = points)
#pragma unroll
  for (int s = 0; s < kLfMaxC / 2; ++s) {
    if (s < KH) {
      const int k = h * KH + s;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < TO) {
          const int o = t * 32 + m;
          const float wv = o < Cout ? Ws[o * ST + k] : 0.f;
          acc[t] = LAYOUT == 0 ? __builtin_amdgcn_mfma_f32_32x32x2f32(xa[s], wv, acc[t], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_32x32x2f32(wv, xa[s], acc[t], 0, 0, 0);
        }
      }
    }
  }
  // D element (row 8 (e / 4) + 4 h + e % 4, column m)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < TO) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = 8 * (e >> 2) + 4 * h + (e & 3);
        if (LAYOUT == 0) {
          const int64_t pr = r0 + rr;
          const int o = t * 32 + m;
          if (pr < R && o < Cout) {
            float v = acc[t][e] + (bias != nullptr ? bias[o] : 0.f);
            if (relu) v = fmaxf(v, 0.f);
            y[pr * Cout + o] = relu_mask(v, mask, pr * Cout + o);
          }
        } else {
          const int o = t * 32 + rr;
          if (ok && o < Cout) {
            float v = acc[t][e] + (bias != nullptr ? bias[o] : 0.f);
            if (relu) v = fmaxf(v, 0.f);
            y[(bb * Cout + o) * N + nn] = relu_mask(v, mask, (bb * Cout + o) * N + nn);
          }
        }
      }
    }
  }
}

// Row layout (0) with Cin % 16 == 0: one wave computes 16 points x all outputs per tile on
// v_mfma_f32_16x16x4_f32 and walks tiles grid-stride, loading the next tile's operands
// while the current tile's MFMAs run. Contraction index at step (q, i) for lane group g:
// k = 16 q + 4 g + i, so each lane's operands are float4s of its own point row (one load
// instruction covers 16 rows x 64 contiguous bytes) and the weight row chunk is one
// ds_read_b128 from Ws[o][k] (row stride KP + 4: conflict-free over 8-lane phases).

template <int Q>
__device__ __forceinline__ void lr_load(const float* __restrict__ x, int64_t sx, int64_t row, int64_t R, int g,
                                        f32x4 (&xa)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q)
    xa[q] = row < R ? *reinterpret_cast<const f32x4*>(x + row * sx + 16 * q + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
}

// Weight staging shared by the MFMA per-point kernels: Ws[o][k] (o < 16 TO, zero rows past
// Cout; row stride 16 Q + 4), from W [Cout, 16 Q] or, with transw, from W^T's [16 Q, Cout].
// w2 / wsplit: stored weight rows >= wsplit come from w2 (row - wsplit) — two layers' weights
// stacked without a concatenation kernel (transw = 0: rows = outputs; transw = 1: rows = the
// stored [Cin, Cout] tensor's rows); w2 == nullptr: every row from w.
template <int Q, int TO>
__device__ __forceinline__ void lr_stage(const float* w, int Cout, int transw, float* Ws, const float* w2,
                                         int wsplit) {  // callers without a second weight pass w2 = w
                                                        // (arithmetic on a null w2 crashed clang-22's inliner)
  constexpr int CI = 16 * Q, ST = CI + 4;
  if (!transw) {  // W [Cout, CI] rows: float4 reads, all issued before the LDS writes
    constexpr int NV = TO * 16 * CI / 4, PER = (NV + 255) / 256;
    f32x4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + 256 * i, o = e / (CI / 4);
      const float* src = o < wsplit ? w + 4 * (int64_t)e : w2 + 4 * (int64_t)(e - wsplit * (CI / 4));
      v[i] = (e < NV && o < Cout) ? *reinterpret_cast<const f32x4*>(src) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + 256 * i, o = e / (CI / 4), k4 = e - o * (CI / 4);
      if (e < NV) *reinterpret_cast<f32x4*>(&Ws[o * ST + 4 * k4]) = v[i];
    }
  } else {  // W^T from a [CI, Cout] tensor: read along Cout
    constexpr int NE = TO * 16 * CI, PER = (NE + 255) / 256;
    float v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + 256 * i, k = e / (TO * 16), o = e - k * (TO * 16);
      const float* src = k < wsplit ? w + (int64_t)k * Cout + o : w2 + (int64_t)(k - wsplit) * Cout + o;
      v[i] = (e < NE && o < Cout) ? *src : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + 256 * i, k = e / (TO * 16), o = e - k * (TO * 16);
      if (e < NE) Ws[o * ST + k] = v[i];
    }
  }
}

template <int Q, int TO, bool GEN>  // Cin = 16 Q, Cout <= 16 TO; GEN: mask / add / split / cf epilogue
__global__ __launch_bounds__(256) void linear_fwd_rows_kernel(const float* __restrict__ x, int64_t sx,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, int64_t R, int Cin,
                                                              int Cout, int transw, LinEpi e) {
  extern __shared__ float Ws[];  // [16 TO][Cin + 4]
  constexpr int CI = 16 * Q, ST = CI + 4;
  const int lane = pk::lane_id(), m = lane & 15, g = lane >> 4;
  const int64_t T = (R + 15) >> 4, stride = (int64_t)gridDim.x * 4;
  int64_t tile = (int64_t)blockIdx.x * 4 + pk::wave_id();
  // the first tile's operands are in flight while the weight is staged
  f32x4 cur[Q], nxt[Q];
  lr_load<Q>(x, sx, tile < T ? tile * 16 + m : R, R, g, cur);
  lr_stage<Q, TO>(w, Cout, transw, Ws, w, 1 << 30);
  __syncthreads();
  if (tile >= T) return;
  constexpr int TH = TO < 4 ? TO : 4, NH = TO / TH;
  float bv[TO];
#pragma unroll
  for (int t = 0; t < TO; ++t) {
    const int o = t * 16 + m;
    bv[t] = (bias != nullptr && o < Cout) ? bias[o] : 0.f;
  }
  for (;;) {
    const int64_t tn = tile + stride;
    if (tn < T) lr_load<Q>(x, sx, tn * 16 + m, R, g, nxt);
    // outputs in groups of TH = 4 column tiles (Cout = 128 runs two passes over the same
    // operands): acc / wv / epilogue operands stay at TH tiles, so TO = 8 keeps 4 waves per SIMD
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
    __builtin_amdgcn_sched_barrier(0);  // one output group's registers live at a time
    // D[point 4 g + r][out t * 16 + m]; the epilogue's operand loads (mask, add) for all
    // TH x 4 outputs are issued before this group's MFMAs (their latency hides behind them),
    // not one dependent load per store
    // (workgroup-uniform branches around unconditional loads at clamped indices: no per-load
    // exec-mask branch, so no wait per load)
    float mk[TH][4], ad[TH][4];
    if (GEN && e.mask != nullptr) {
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t pr = tile * 16 + 4 * g + r;
          const int o = (hh * TH + t) * 16 + m;
          const float v = e.mask[(pr < R && o < Cout) ? pr * Cout + o : 0];
          mk[t][r] = v;
        }
    } else {
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mk[t][r] = 1.f;
    }
    if (GEN && e.add != nullptr && hh * TH * 16 < e.add_cols) {
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t pr = tile * 16 + 4 * g + r;
          const int o = (hh * TH + t) * 16 + m;
          const bool ok = pr < R && o < e.add_cols;
          const float v = e.add[ok ? pr * e.sa + o : 0];
          ad[t][r] = ok ? v : 0.f;
        }
    } else {
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) ad[t][r] = 0.f;
    }
    f32x4 acc[TH];
#pragma unroll
    for (int t = 0; t < TH; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      {
        f32x4 wv[TH];
#pragma unroll
        for (int t = 0; t < TH; ++t)
          wv[t] = *reinterpret_cast<const f32x4*>(&Ws[((hh * TH + t) * 16 + m) * ST + 16 * q + 4 * g]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int t = 0; t < TH; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur[q][i], wv[t][i], acc[t], 0, 0, 0);
          }
        __builtin_amdgcn_sched_barrier(0);  // keep the weight reads per chunk (no hoisting of all Q x TH)
      }
    }
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      const int o = (hh * TH + t) * 16 + m;
      const int64_t p0 = tile * 16 + 4 * g;
      if (GEN && e.store_cf && ((e.N | e.sy) & 3) == 0 && (reinterpret_cast<uintptr_t>(e.y) & 15) == 0 && p0 + 3 < R) {
        // channels-first store: the lane's 4 consecutive points of channel o (one item, as
        // N % 4 == 0) as one 16-B store
        if (o < Cout) {
          f32x4 v4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = lin_act(e.relu, acc[t][r] + bv[hh * TH + t]);
            v = mk[t][r] <= 0.f ? 0.f : v;
            v4[r] = v + ad[t][r];
          }
          const int64_t b = p0 / e.N, n = p0 - b * e.N;
          *reinterpret_cast<f32x4*>(e.y + b * e.sy + (int64_t)o * e.N + n) = v4;
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t pr = tile * 16 + 4 * g + r;
        if (pr < R && o < Cout) {
          float v = lin_act(e.relu, acc[t][r] + bv[hh * TH + t]);
          v = mk[t][r] <= 0.f ? 0.f : v;  // relu_mask
          v += ad[t][r];  // 0 without add / past add_cols
          if (GEN && e.store_cf) {
            const int64_t b = pr / e.N, n = pr - b * e.N;
            e.y[b * e.sy + (int64_t)o * e.N + n] = v;
          } else if (GEN && o >= e.split) {
            e.y2[pr * e.sy2 + (o - e.split)] = v;
          } else {
            e.y[pr * e.sy + o] = v;
          }
        }
      }
    }
    }
    if (tn >= T) break;
    tile = tn;
#pragma unroll
    for (int q = 0; q < Q; ++q) cur[q] = nxt[q];
  }
}

// Rows layout, LDS-DMA pipeline (the production rows path since round 4 for Cin in {32, 64, 128}):
// round 3 found the per-point layers bound by serialisation, not bytes — every wave resident from
// the start, all loads in one burst, then all MFMAs, then the stores (DESIGN.md §5 'Per-point
// layers'). Here a block is 4 waves, one per SIMD, walking 16-point tiles grid-stride through a
// ring of D LDS slots per wave filled by global_load_lds_dwordx4 (no VGPR cost, so D - 1 tiles
// are in flight while the MFMAs of the current tile run):
//   * slot = the tile's x rows (16 x Cin), then, with GEN, its mask rows and residual rows
//     (16 x 16 TO each), every 16-B chunk XOR-swizzled on the SOURCE address (the LDS image of a
//     glds is lane-linear) so the fragment reads are conflict-free;
//   * the weight sits in VGPRs (A operand: lane (g, m) of output tile t at step (q, i) holds
//     W[16 t + m][16 q + 4 g + i]), so D[out][point]: a lane ends with 4 CONSECUTIVE outputs of one
//     point — bias, mask, residual and the store move as 16-B vectors;
//   * the contraction order (k = 16 q + 4 g + i at step (q, i)) and the epilogue are those of
//     linear_fwd_rows_kernel: results are bit-identical to it;
//   * counted waits: every tile issues the same G glds (tiles past the end are loaded again at a
//     clamped index), so "tile k landed" is s_waitcnt vmcnt((D - 1) G): vector-memory ops retire
//     in issue order and at least the next D - 1 tiles' glds are younger (the stores in between
//     are left out of the count, which only makes the wait more conservative).
// MASK / ADD (GEN epilogues): the ReLU-backward mask rows (shaped like the output) and the
// residual rows (row stride sa, columns < add_cols) ride in the slot; SPLIT: outputs >= split
// (a multiple of 16) go to y2. Cout % 16 == 0, act 0 / 1, no channels-first store (host checks).
__device__ __forceinline__ void vm_wait(int n) {  // s_waitcnt vmcnt(n), expcnt / lgkmcnt untouched
  switch (n) {
#define PK_VMW(N) case N: __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8)); break;
    PK_VMW(0) PK_VMW(1) PK_VMW(2) PK_VMW(3) PK_VMW(4) PK_VMW(5) PK_VMW(6) PK_VMW(7) PK_VMW(8) PK_VMW(9)
    PK_VMW(10) PK_VMW(11) PK_VMW(12) PK_VMW(13) PK_VMW(14) PK_VMW(15) PK_VMW(16) PK_VMW(17) PK_VMW(18)
    PK_VMW(19) PK_VMW(20) PK_VMW(21) PK_VMW(22) PK_VMW(23) PK_VMW(24) PK_VMW(25) PK_VMW(26) PK_VMW(27)
    PK_VMW(28) PK_VMW(29) PK_VMW(30) PK_VMW(31) PK_VMW(32) PK_VMW(33) PK_VMW(34) PK_VMW(35) PK_VMW(36)
    PK_VMW(37) PK_VMW(38) PK_VMW(39) PK_VMW(40) PK_VMW(41) PK_VMW(42) PK_VMW(43) PK_VMW(44) PK_VMW(45)
    PK_VMW(46) PK_VMW(47) PK_VMW(48) PK_VMW(49) PK_VMW(50) PK_VMW(51) PK_VMW(52) PK_VMW(53) PK_VMW(54)
    PK_VMW(55) PK_VMW(56) PK_VMW(57) PK_VMW(58) PK_VMW(59) PK_VMW(60) PK_VMW(61) PK_VMW(62)
#undef PK_VMW
    default: __builtin_amdgcn_s_waitcnt((63 & 15) | ((63 >> 4) << 14) | (7 << 4) | (15 << 8)); break;
  }
}

// 16 rows x CW floats (row stride ld, columns >= cols_ok read at column 0 of the row: valid
// memory, masked at use) into an LDS region of 16 x CW floats, chunk (row, c) at position
// row * CW / 4 + (c ^ (row & (CW / 4 - 1) & 15)): CW / 16 glds per wave
template <int CW>
__device__ __forceinline__ void glds_rows(const float* __restrict__ src, int64_t ld, int64_t row0, int64_t R,
                                          int cols_ok, float* lds_dst, int lane) {
  constexpr int CPR = CW / 4, NI = CW / 16;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int p = j * 64 + lane;
    const int row = p / CPR, cl = p % CPR;
    const int c = cl ^ (row & (CPR - 1) & 15);
    const int64_t gr = min(row0 + row, R - 1);
    const int col = 4 * c < cols_ok ? 4 * c : 0;
    __builtin_amdgcn_global_load_lds(src + gr * ld + col, (__attribute__((address_space(3))) void*)(lds_dst + j * 256),
                                     16, 0, 0);
  }
}

template <int CW>
__device__ __forceinline__ f32x4 lds_chunk(const float* region, int row, int c) {
  constexpr int CPR = CW / 4;
  return *reinterpret_cast<const f32x4*>(region + 4 * (row * CPR + (c ^ (row & (CPR - 1) & 15))));
}

// Per-lane float offsets of the 16-B chunks of a glds_rows<CW> image within one 16-row block (row
// stride ld, columns >= cols_ok at column 0), computed once: a tile whose 16 rows are all in range
// is then issued from a scalar base (glds_issue16) without per-lane 64-bit address arithmetic,
// which on gfx950 would be VALU work serialised with the f32 MFMAs.
template <int CW>
__device__ __forceinline__ void glds_rows_off(int64_t ld, int cols_ok, int lane, int (&off)[CW / 16]) {
  constexpr int CPR = CW / 4;
#pragma unroll
  for (int j = 0; j < CW / 16; ++j) {
    const int p = j * 64 + lane;
    const int row = p / CPR, cl = p % CPR;
    const int c = cl ^ (row & (CPR - 1) & 15);
    off[j] = (int)(row * ld) + (4 * c < cols_ok ? 4 * c : 0);
  }
}

// the same for a glds_cf<C> image: chunk (c, pos) holds floats 4 (pos ^ ((c >> 2) & 3)) .. + 3
// of channel c (channel stride N)
template <int C>
__device__ __forceinline__ void glds_cf_off(int N, int lane, int (&off)[C / 16]) {
#pragma unroll
  for (int j = 0; j < C / 16; ++j) {
    const int p = j * 64 + lane;
    const int c = p >> 2, pos = p & 3;
    off[j] = c * N + 4 * (pos ^ ((c >> 2) & 3));
  }
}

template <int NI, int BYTES>
__device__ __forceinline__ void glds_issue(const float* base, const int* off, float* lds_dst) {  // off[NI]
  static_assert(BYTES == 16 || BYTES == 4, "glds piece");
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    auto* d = (__attribute__((address_space(3))) void*)(lds_dst + j * BYTES * 16);
    if constexpr (BYTES == 16) __builtin_amdgcn_global_load_lds(base + off[j], d, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(base + off[j], d, 4, 0, 0);
  }
}

template <int Q, int TO, bool MASK, bool ADD, bool SPLIT>
__global__ __launch_bounds__(256, 1) void linear_glds_rows_kernel(const float* __restrict__ x, int64_t sx,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias, int64_t R, int Cin,
                                                                  int Cout, int transw, LinEpi e) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int CI = 16 * Q, CO = 16 * TO;
  constexpr int SLOT = 16 * CI + (MASK ? 16 * CO : 0) + (ADD ? 16 * CO : 0);  // floats
  constexpr int G = Q + (MASK ? TO : 0) + (ADD ? TO : 0);  // glds per tile
  constexpr int D = 3 * 4 * SLOT * 4 <= 159 * 1024 ? 3 : 2;  // ring depth within the CU's LDS
  const int lane = pk::lane_id(), wv = pk::wave_id(), m = lane & 15, g = lane >> 4;
  // weight -> VGPRs through the (not yet used) ring: Ws[o][k], row stride CI + 4
  lr_stage<Q, TO>(w, Cout, transw, lds, w, 1 << 30);
  __syncthreads();
  f32x4 wf[TO][Q];
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int q = 0; q < Q; ++q)
      wf[t][q] = *reinterpret_cast<const f32x4*>(&lds[(t * 16 + m) * (CI + 4) + 16 * q + 4 * g]);
  f32x4 bv[TO];  // bias of outputs 16 t + 4 g + r
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 16 * t + 4 * g + r;
      bv[t][r] = (bias != nullptr && o < Cout) ? bias[o] : 0.f;
    }
  __syncthreads();  // every wave holds its weight: the ring may now overwrite the stage
  float* ring = lds + (int64_t)wv * D * SLOT;
  const int64_t T = (R + 15) >> 4, stride = (int64_t)gridDim.x * 4;
  const int64_t t0 = (int64_t)blockIdx.x * 4 + wv;
  if (t0 >= T) return;
  const int64_t nt = (T - 1 - t0) / stride + 1;  // tiles of this wave
  // lane offsets of the glds chunks, computed once (a full tile is then issued from a scalar base)
  int offx[Q], offm[MASK ? TO : 1], offa[ADD ? TO : 1];
  glds_rows_off<CI>(sx, CI, lane, offx);
  if constexpr (MASK) glds_rows_off<CO>(Cout, Cout, lane, offm);
  if constexpr (ADD) glds_rows_off<CO>(e.sa, e.add_cols, lane, offa);
  auto issue = [&](int64_t k) {  // glds of this wave's k-th tile (clamped: constant op count)
    const int64_t tile = t0 + min(k, nt - 1) * stride;
    float* s = ring + (k % D) * SLOT;
    const int64_t r0 = tile * 16;
    if (r0 + 16 <= R) {  // (wave-uniform) every row in range
      glds_issue<Q, 16>(x + r0 * sx, offx, s);
      if constexpr (MASK) glds_issue<TO, 16>(e.mask + r0 * Cout, offm, s + 16 * CI);
      if constexpr (ADD) glds_issue<TO, 16>(e.add + r0 * e.sa, offa, s + 16 * CI + (MASK ? 16 * CO : 0));
    } else {
      glds_rows<CI>(x, sx, r0, R, CI, s, lane);
      if constexpr (MASK) glds_rows<CO>(e.mask, Cout, r0, R, Cout, s + 16 * CI, lane);
      if constexpr (ADD) glds_rows<CO>(e.add, e.sa, r0, R, e.add_cols, s + 16 * CI + (MASK ? 16 * CO : 0), lane);
    }
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k) issue(k);
  for (int64_t k = 0; k < nt; ++k) {
    issue(k + D - 1);
    // tile k landed: at least the (D - 1) G glds of tiles k+1 .. k+D-1 are younger than its own
    // (vector-memory ops retire in issue order); the stores issued in between are not counted,
    // so the wait also drains the oldest of them — conservative whatever the stores' exec masks
    vm_wait((D - 1) * G);
    const float* s = ring + (k % D) * SLOT;
    const int64_t tile = t0 + k * stride;
    f32x4 acc[TO];
#pragma unroll
    for (int t = 0; t < TO; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const f32x4 xv = lds_chunk<CI>(s, m, 4 * q + g);  // point m, features 16 q + 4 g .. + 3
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < TO; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[t][q][i], xv[i], acc[t], 0, 0, 0);
    }
    // D[out 16 t + 4 g + r][point m]
    const int64_t pr = tile * 16 + m;
#pragma unroll
    for (int t = 0; t < TO; ++t) {
      f32x4 mk = {1.f, 1.f, 1.f, 1.f}, ad = {0.f, 0.f, 0.f, 0.f};
      if constexpr (MASK) mk = lds_chunk<CO>(s + 16 * CI, m, 4 * t + g);
      if constexpr (ADD) {
        if (16 * t + 4 * g < e.add_cols) ad = lds_chunk<CO>(s + 16 * CI + (MASK ? 16 * CO : 0), m, 4 * t + g);
      }
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 16 * t + 4 * g + r;
        float u = acc[t][r] + bv[t][r];
        u = e.relu ? fmaxf(u, 0.f) : u;  // (act 0 / 1 only here: the host routes sigmoid elsewhere)
        u = mk[r] <= 0.f ? 0.f : u;      // relu_mask
        v[r] = ADD ? u + (o < e.add_cols ? ad[r] : 0.f) : u;
      }
      const int o0 = 16 * t + 4 * g;
      if (pr < R) {
        if (SPLIT && 16 * t >= e.split)  // (split % 16 == 0: wave-uniform per output tile)
          *reinterpret_cast<f32x4*>(&e.y2[pr * e.sy2 + (o0 - e.split)]) = v;
        else
          *reinterpret_cast<f32x4*>(&e.y[pr * e.sy + o0]) = v;
      }
    }
  }
  vm_wait(0);
}

// ---- Weight gradients on the LDS-DMA pipeline (round 4, the grouped path's default) ----
// Round 3's wgrad_v2_body gave each of 8 waves one 32 x 32 output tile and had every wave load
// its own columns of x and dy straight into VGPRs: each row was fetched by To + Ti waves and
// only two 16-row batches were in flight per wave (0.20 ms/step at 0.2 of the f32 MFMA rate and
// 0.3 of HBM). Here a block is 4 waves, one per SIMD, over one slice of one problem's rows; wave
// w walks the slice's 16-row tiles w, w + 4, ... through a ring of D LDS slots filled by
// global_load_lds_dwordx4 (x rows, then dy rows: each byte fetched once, D - 1 tiles in flight
// at no VGPR cost), and holds the WHOLE [O, I] gradient as TO x TI 16 x 16 accumulators
// (v_mfma_f32_16x16x4f32: A[o][k] = dY[row k][o], B[k][i] = X[row k][i]). The 4 waves' sums are
// added through LDS in wave order and written as the block's partial; the grouped reduction sums
// the partials in block order (deterministic, as before).
//   layout 0 ([R, C]): the slot holds glds_rows images (row-major, 16-B chunks XOR-swizzled per
//     row); k-step q, lane (g, m) takes row 4 q + g and the TO (TI) CONSECUTIVE channels
//     TO m .. TO m + TO - 1 of dy (x) in one vector read: accumulator tile t holds o = TO m' + t.
//     The last tile of a problem may be ragged: its clamped rows get dy = 0.
//   layout 1 ([Bn, C, N], N % 16 == 0, batch stride 4-aligned): the slot holds per channel the
//     tile's 16 rows, 16-B chunk j of channel c at position j ^ ((c >> 2) & 3) (XOR on the
//     SOURCE address: conflict-free reads); lane (g, m) reads rows 4 g .. 4 g + 3 of channel
//     m + 16 t as one vector, i.e. k-step q takes row 4 g + q (any bijection works: A and B use
//     the same one). Tile t holds o = m' + 16 t.
// Bias: db[o] = the sum of the dy values the lanes feed the MFMAs (fixed order).
constexpr int kWgBlocks = 1024;  // blocks per grouped launch: 4 x the CU count (MI355X: 256; wg_budget)
constexpr int kWgLdsBytes = 4 * 3 * 16 * (128 + 64) * 4;  // 3 slots per wave of the largest (I + O = 192)
// ring depth: as many slots as the LDS holds, <= 8 (bytes in flight per CU = 4 (D - 1) slots:
// the thin problems are HBM-bound and need the depth, the wide ones have the MFMA work)
constexpr int wg_depth(int slot_floats) {
  return kWgLdsBytes / (4 * slot_floats * 4) < 8 ? kWgLdsBytes / (4 * slot_floats * 4) : 8;
}

// NV consecutive floats NV m .. NV m + NV - 1 of row `row` of a glds_rows<CW> image (chunks
// XOR-swizzled per row; NV = 1, 2, 4 or 8)
template <int CW, int NV>
__device__ __forceinline__ void lds_rowvec(const float* region, int row, int m, float (&v)[NV]) {
  constexpr int CPR = CW / 4;
  const int sw = row & (CPR - 1) & 15;
  if constexpr (NV >= 4) {
#pragma unroll
    for (int h = 0; h < NV / 4; ++h) {
      const int c = (NV / 4) * m + h;
      const f32x4 u = *reinterpret_cast<const f32x4*>(region + 4 * (row * CPR + (c ^ sw)));
      v[4 * h] = u[0]; v[4 * h + 1] = u[1]; v[4 * h + 2] = u[2]; v[4 * h + 3] = u[3];
    }
  } else {
    const int c = (NV * m) >> 2, off = (NV * m) & 3;
    const float* p = region + 4 * (row * CPR + (c ^ sw)) + off;
    if constexpr (NV == 2) {
      const float2 u = *reinterpret_cast<const float2*>(p);
      v[0] = u.x; v[1] = u.y;
    } else {
      v[0] = p[0];
    }
  }
}

// 16 rows [row0, row0 + 16) of a channels-first operand (item b = row0 / N) into a [C][16] LDS image
template <int C>
__device__ __forceinline__ void glds_cf(const float* __restrict__ src, int64_t sb, int N, int64_t row0, float* lds_dst,
                                        int lane) {
  const int64_t b = row0 / N, n0 = row0 - b * N;
#pragma unroll
  for (int j = 0; j < C / 16; ++j) {
    const int p = j * 64 + lane;
    const int c = p >> 2, pos = p & 3;
    const int ch = pos ^ ((c >> 2) & 3);
    __builtin_amdgcn_global_load_lds(src + b * sb + (int64_t)c * N + n0 + 4 * ch,
                                     (__attribute__((address_space(3))) void*)(lds_dst + j * 256), 16, 0, 0);
  }
}

// Rows [row0, row0 + 16) of a thin rows-layout operand (C < 16 channels: 16 C contiguous
// floats) by 4-byte glds, lane p taking float p (indices clamped to the tensor: a ragged last
// tile reads valid memory, its rows past R are masked at use): ceil(16 C / 64) instructions.
template <int C>
__device__ __forceinline__ void glds_thin(const float* __restrict__ src, int64_t row0, int64_t R, float* lds_dst,
                                          int lane) {
#pragma unroll
  for (int j = 0; j < (16 * C + 63) / 64; ++j) {
    const int64_t idx = min(row0 * C + j * 64 + lane, R * C - 1);
    __builtin_amdgcn_global_load_lds(src + idx, (__attribute__((address_space(3))) void*)(lds_dst + j * 64), 4, 0,
                                     0);
  }
}

// XT / DT > 0: x (dy) is a thin rows-layout operand of XT (DT) < 16 channels (TI = 1 / TO = 1):
// the input layer 3 -> 64 and the 32 -> 1 heads; lanes m >= XT (DT) feed zeros.
template <int LAYOUT, int TI, int TO, int XT = 0, int DT = 0>
__device__ __forceinline__ void wgrad_glds_body(const WgradProblem& P, int s, float* lds) {
  static_assert((XT == 0 || (TI == 1 && LAYOUT == 0)) && (DT == 0 || (TO == 1 && LAYOUT == 0)), "thin operands");
  constexpr int I = 16 * TI, O = 16 * TO;
  constexpr int XS = XT ? 64 * ((16 * XT + 63) / 64) : 16 * I;  // slot floats of the x rows
  constexpr int DS = DT ? 64 * ((16 * DT + 63) / 64) : 16 * O;  // and of the dy rows
  constexpr int SLOT = XS + DS;
  constexpr int G = (XT ? (16 * XT + 63) / 64 : I / 16) + (DT ? (16 * DT + 63) / 64 : O / 16);  // glds per tile
  constexpr int kWgD = wg_depth(SLOT);
  const int lane = pk::lane_id(), wv = pk::wave_id(), m = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)s * P.SL;
  const int64_t r1 = r0 + P.SL < P.R ? r0 + P.SL : P.R;
  const int64_t ntile = (r1 - r0 + 15) >> 4;
  const int64_t nt = ntile > wv ? (ntile - 1 - wv) / 4 + 1 : 0;  // tiles of this wave
  const int64_t sbx = P.sbx ? P.sbx : (int64_t)I * P.N, sbdy = P.sbdy ? P.sbdy : (int64_t)O * P.N;
  float* ring = lds + wv * kWgD * SLOT;
  constexpr int NX = XT ? (16 * XT + 63) / 64 : I / 16, ND = DT ? (16 * DT + 63) / 64 : O / 16;
  int offx[NX], offd[ND];  // lane offsets of the glds chunks (4-B pieces for a thin operand)
  if constexpr (LAYOUT == 0) {
    if constexpr (XT > 0) {
#pragma unroll
      for (int j = 0; j < NX; ++j) offx[j] = j * 64 + lane;
    } else {
      glds_rows_off<I>(I, I, lane, offx);
    }
    if constexpr (DT > 0) {
#pragma unroll
      for (int j = 0; j < ND; ++j) offd[j] = j * 64 + lane;
    } else {
      glds_rows_off<O>(O, O, lane, offd);
    }
  } else {
    glds_cf_off<I>(P.N, lane, offx);
    glds_cf_off<O>(P.N, lane, offd);
  }
  // channels-first issue cursor: item cb, first point cn of the next tile to issue (tiles of a
  // wave step by 64 rows; N % 16 == 0, so a 16-row tile never straddles two items)
  int64_t cb = 0, cn = 0, lb = 0, ln = 0, lrow = 0;
  if constexpr (LAYOUT == 1) {
    const int64_t rs = r0 + 16 * wv;
    cb = rs / P.N;
    cn = rs - cb * P.N;
  }
  auto issue = [&](int64_t k) {  // glds of the wave's k-th tile (clamped: constant op count)
    float* sl = ring + (k % kWgD) * SLOT;
    if (k < nt) {
      lrow = r0 + 16 * (wv + 4 * k);
      if constexpr (LAYOUT == 1) {
        lb = cb;
        ln = cn;
        cn += 64;
        while (cn >= P.N) {
          cn -= P.N;
          ++cb;
        }
      }
    }
    const int64_t row0 = lrow;
    if constexpr (LAYOUT == 0) {
      // thin operands: every lane of the 4-B glds loads one float, 64 per instruction, past the
      // tile's 16 C: always clamped to the tensor (glds_thin), whatever the tile
      const bool full = row0 + 16 <= P.R;  // (wave-uniform) all rows in range
      if constexpr (XT > 0) glds_thin<XT>(P.x, row0, P.R, sl, lane);
      else if (full) glds_issue<NX, 16>(P.x + row0 * I, offx, sl);
      else glds_rows<I>(P.x, I, row0, P.R, I, sl, lane);
      if constexpr (DT > 0) glds_thin<DT>(P.dy, row0, P.R, sl + XS, lane);
      else if (full) glds_issue<ND, 16>(P.dy + row0 * O, offd, sl + XS);
      else glds_rows<O>(P.dy, O, row0, P.R, O, sl + XS, lane);
    } else {
      glds_issue<NX, 16>(P.x + lb * sbx + ln, offx, sl);
      glds_issue<ND, 16>(P.dy + lb * sbdy + ln, offd, sl + XS);
    }
  };
  f32x4 acc[TO][TI];
  float bs[TO];
#pragma unroll
  for (int t = 0; t < TO; ++t) {
    bs[t] = 0.f;
#pragma unroll
    for (int u = 0; u < TI; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (nt > 0) {
#pragma unroll
    for (int k = 0; k < kWgD - 1; ++k) issue(k);
    for (int64_t k = 0; k < nt; ++k) {
      issue(k + kWgD - 1);
      vm_wait((kWgD - 1) * G);  // tile k landed (glds retire in issue order)
      if (P.pad == 2) continue;  // (development variant: the glds stream alone)
      const float* sx = ring + (k % kWgD) * SLOT;
      const float* sd = sx + XS;
      if constexpr (LAYOUT == 0) {
        const int64_t row0 = r0 + 16 * (wv + 4 * k);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 4 * q + g;
          float a[TO], b[TI];
          if constexpr (DT > 0) a[0] = m < DT ? sd[row * DT + m] : 0.f;
          else lds_rowvec<O, TO>(sd, row, m, a);
          if constexpr (XT > 0) b[0] = m < XT ? sx[row * XT + m] : 0.f;
          else lds_rowvec<I, TI>(sx, row, m, b);
          if (row0 + 16 > P.R) {  // (wave-uniform) clamped rows of a ragged last tile: dy = 0
            const bool ok = row0 + row < P.R;
#pragma unroll
            for (int t = 0; t < TO; ++t) a[t] = ok ? a[t] : 0.f;
          }
#pragma unroll
          for (int t = 0; t < TO; ++t) bs[t] += a[t];
          if (P.pad == 1) {  // (development variant: the operand stream without the MFMAs)
            acc[0][0][0] += b[0];
            continue;
          }
#pragma unroll
          for (int t = 0; t < TO; ++t)
#pragma unroll
            for (int u = 0; u < TI; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[u], acc[t][u], 0, 0, 0);
        }
      } else {
        f32x4 a[TO], b[TI];
#pragma unroll
        for (int t = 0; t < TO; ++t) {
          const int c = m + 16 * t;
          a[t] = *reinterpret_cast<const f32x4*>(sd + 16 * c + 4 * (g ^ ((c >> 2) & 3)));
          bs[t] += (a[t][0] + a[t][1]) + (a[t][2] + a[t][3]);
        }
#pragma unroll
        for (int u = 0; u < TI; ++u) {
          const int c = m + 16 * u;
          b[u] = *reinterpret_cast<const f32x4*>(sx + 16 * c + 4 * (g ^ ((c >> 2) & 3)));
        }
        if (P.pad == 1) {  // (development variant: the operand stream without the MFMAs)
          acc[0][0] += b[0];
          continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < TO; ++t)
#pragma unroll
            for (int u = 0; u < TI; ++u)
              acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][q], b[u][q], acc[t][u], 0, 0, 0);
      }
    }
  }
  vm_wait(0);
  // bias: the four row groups g of a channel, fixed order
#pragma unroll
  for (int t = 0; t < TO; ++t) {
    bs[t] += __shfl_xor(bs[t], 16);
    bs[t] += __shfl_xor(bs[t], 32);
  }
  __syncthreads();  // every wave is done with its ring: the LDS now holds waves 1..3's sums
  constexpr int NA = TO * TI * 4;
  if (wv > 0) {
    float* dst = lds + (wv - 1) * (NA + TO) * 64;
#pragma unroll
    for (int t = 0; t < TO; ++t)
#pragma unroll
      for (int u = 0; u < TI; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[((t * TI + u) * 4 + r) * 64 + lane] = acc[t][u][r];
#pragma unroll
    for (int t = 0; t < TO; ++t) dst[(NA + t) * 64 + lane] = bs[t];
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float* src = lds + w * (NA + TO) * 64;
#pragma unroll
    for (int t = 0; t < TO; ++t) {
#pragma unroll
      for (int u = 0; u < TI; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][u][r] += src[((t * TI + u) * 4 + r) * 64 + lane];
      bs[t] += src[(NA + t) * 64 + lane];
    }
  }
  float* ps = P.part + (int64_t)s * P.O * P.I;
  float* pb = P.part + (int64_t)P.S * P.O * P.I + (int64_t)s * P.O;
#pragma unroll
  for (int t = 0; t < TO; ++t) {
#pragma unroll
    for (int u = 0; u < TI; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ol = 4 * g + r;
        const int o = LAYOUT == 0 ? TO * ol + t : ol + 16 * t;
        const int i = LAYOUT == 0 ? TI * m + u : m + 16 * u;
        if ((XT == 0 || i < XT) && (DT == 0 || o < DT)) ps[o * P.I + i] = acc[t][u][r];
      }
    const int ob = LAYOUT == 0 ? TO * m + t : m + 16 * t;
    if (g == 0 && (DT == 0 || ob < DT)) pb[ob] = bs[t];
  }
}

// Shapes on the pipeline: I, O in {16, 32, 64, 128}, O I <= 8192 (the acc of one wave), and the
// thin rows-layout shapes below.
// Thin rows-layout shapes (the step's 3 -> 64 input layer and 32 -> 1 heads): ids 16, 17.
__host__ __device__ constexpr int wg_shape_id(int I, int O, int layout = 0) {
  return (I == 16 || I == 32 || I == 64 || I == 128) && (O == 16 || O == 32 || O == 64 || O == 128) && I * O <= 8192
             ? (I == 16 ? 0 : I == 32 ? 1 : I == 64 ? 2 : 3) * 4 + (O == 16 ? 0 : O == 32 ? 1 : O == 64 ? 2 : 3)
         : layout == 0 && I == 3 && O == 64 ? 16
         : layout == 0 && I == 32 && O == 1 ? 17
                                            : -1;
}

template <int LAYOUT>
__device__ __forceinline__ void wgrad_glds_dispatch(const WgradProblem& P, int s, float* lds) {
  switch (wg_shape_id(P.I, P.O, LAYOUT)) {
#define PK_WG(I_, O_) case wg_shape_id(I_, O_): wgrad_glds_body<LAYOUT, I_ / 16, O_ / 16>(P, s, lds); break;
    PK_WG(16, 16) PK_WG(16, 32) PK_WG(16, 64) PK_WG(16, 128)
    PK_WG(32, 16) PK_WG(32, 32) PK_WG(32, 64) PK_WG(32, 128)
    PK_WG(64, 16) PK_WG(64, 32) PK_WG(64, 64) PK_WG(64, 128)
    PK_WG(128, 16) PK_WG(128, 32) PK_WG(128, 64)
#undef PK_WG
    case 16:
      if constexpr (LAYOUT == 0) wgrad_glds_body<0, 1, 4, 3, 0>(P, s, lds);
      break;
    case 17:
      if constexpr (LAYOUT == 0) wgrad_glds_body<0, 2, 1, 0, 1>(P, s, lds);
      break;
    default: break;
  }
}

__global__ __launch_bounds__(256, 1) void wgrad_glds_grouped_kernel(const WgradProblems tab) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x;
  int g = 0;
  while (g + 1 < tab.G && b >= tab.p[g + 1].blk0) ++g;  // block-uniform scan
  const WgradProblem& P = tab.p[g];
  if (P.layout == 0) wgrad_glds_dispatch<0>(P, b - P.blk0, lds);
  else wgrad_glds_dispatch<1>(P, b - P.blk0, lds);
}

// Channels-first layout (1) [Bn, C, N] with Cin in {16, 32, 64, 128}: one wave computes 16 SUB
// consecutive points of one item x all outputs; tpc tiles per item (SUB > 1 needs N % (16 SUB)
// == 0; with SUB = 1 an item's last tile may be ragged: its columns past N compute on a clamped
// point and are not stored — the MFMA columns are independent points). A = weight
// (Ws[o][k] chunks, ds_read_b128), B = points: lane (j, g) loads its SUB consecutive points
// as one vector per channel row k = 16 q + 4 g + i, and element u of that
// vector is column j of point sub-tile u (sub-tile u holds points SUB j + u), so loads and
// the D stores (float SUB vectors of consecutive points) are both contiguous per lane.
template <int SUB> struct LcVec;
template <> struct LcVec<1> { using T = float; };
template <> struct LcVec<2> { using T = __attribute__((ext_vector_type(2))) float; };
template <> struct LcVec<4> { using T = f32x4; };

template <int Q, int TO, int SUB>
__device__ __forceinline__ void linear_cf_body(const float* __restrict__ x, int64_t sx, const float* __restrict__ w,
                                               const float* __restrict__ bias, int64_t R, int N, int Cout, int transw,
                                               const LinEpi& e, int64_t tpc, int64_t blk, float* Ws) {
  using V = typename LcVec<SUB>::T;
  constexpr int CI = 16 * Q, ST = CI + 4, P = 16 * SUB;
  const int lane = pk::lane_id(), m = lane & 15, g = lane >> 4;
  const int64_t T = (R / N) * tpc;
  const int64_t tile = blk * 4 + pk::wave_id();
  // the tile's operands are in flight while the weight is staged
  V xv[Q][4];
  int64_t bb = 0, n0 = 0;
  bool live = true;  // this lane's point column exists (only a SUB = 1 ragged tail has dead ones)
  if (tile < T) {
    bb = tile / tpc;
    n0 = (tile - bb * tpc) * P;
    if (SUB == 1) live = n0 + m < N;
    const float* xb = x + bb * sx + n0 + (live ? SUB * m : 0);
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[q][i] = *reinterpret_cast<const V*>(xb + (int64_t)(16 * q + 4 * g + i) * N);
  }
  lr_stage<Q, TO>(w, Cout, transw, Ws, e.w2 ? e.w2 : w, e.w2 ? e.wsplit : (1 << 30));
  __syncthreads();
  if (tile >= T) return;
  f32x4 acc[TO][SUB];
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int u = 0; u < SUB; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    f32x4 wv[TO];
#pragma unroll
    for (int t = 0; t < TO; ++t) wv[t] = *reinterpret_cast<const f32x4*>(&Ws[(t * 16 + m) * ST + 16 * q + 4 * g]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < SUB; ++u)
#pragma unroll
        for (int t = 0; t < TO; ++t) {
          float b;
          if constexpr (SUB == 1) b = xv[q][i]; else b = xv[q][i][u];
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[t][i], b, acc[t][u], 0, 0, 0);
        }
    __builtin_amdgcn_sched_barrier(0);
  }
  // D[out t * 16 + 4 g + r][column m of sub-tile u] = point n0 + SUB m + u
  const int64_t pn = n0 + (live ? SUB * m : 0);
  float* yb = e.y + bb * e.sy + pn;
  const int64_t mb = bb * Cout * (int64_t)N + pn;  // contiguous index (mask)
  // epilogue operands (mask, add) of all TO x 4 output rows loaded before the first use:
  // workgroup-uniform branches around unconditional loads at clamped rows
  V mv[TO][4], av[TO][4];
  float bo4[TO][4];
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = t * 16 + 4 * g + r;
      bo4[t][r] = 0.f;
      if (bias != nullptr) {
        const int oc = o < Cout ? o : 0;
        const float b = (e.bias2 != nullptr && oc >= e.wsplit) ? e.bias2[oc - e.wsplit] : bias[oc];
        bo4[t][r] = o < Cout ? b : 0.f;
      }
    }
  if (e.mask != nullptr) {
#pragma unroll
    for (int t = 0; t < TO; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = t * 16 + 4 * g + r;
        mv[t][r] = *reinterpret_cast<const V*>(e.mask + mb + (int64_t)(o < Cout ? o : 0) * N);
      }
  }
  if (e.add != nullptr) {
#pragma unroll
    for (int t = 0; t < TO; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = t * 16 + 4 * g + r;
        av[t][r] = *reinterpret_cast<const V*>(e.add + bb * e.sa + (int64_t)(o < e.add_cols ? o : 0) * N + pn);
      }
  }
  V a2v[TO][4];
  if (e.add2 != nullptr) {
#pragma unroll
    for (int t = 0; t < TO; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = t * 16 + 4 * g + r;
        a2v[t][r] = *reinterpret_cast<const V*>(e.add2 + bb * e.sa2 + (int64_t)(o < Cout ? o : 0) * N + pn);
      }
  }
#pragma unroll
  for (int t = 0; t < TO; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = t * 16 + 4 * g + r;
      if (o < Cout && live) {
        const float bo = bo4[t][r];
        const bool has_add = e.add != nullptr && o < e.add_cols;
        V v;
#pragma unroll
        for (int u = 0; u < SUB; ++u) {
          float z = lin_act(e.relu, acc[t][u][r] + bo);
          if (e.mask != nullptr) {
            float mz;
            if constexpr (SUB == 1) mz = mv[t][r]; else mz = mv[t][r][u];
            z = mz <= 0.f ? 0.f : z;
          }
          if (has_add) {
            if constexpr (SUB == 1) z += av[t][r]; else z += av[t][r][u];
          }
          if (e.add2 != nullptr) {  // (z + add) + add2: the order of autograd's two accumulations
            if constexpr (SUB == 1) z += a2v[t][r]; else z += a2v[t][r][u];
          }
          if constexpr (SUB == 1) v = z; else v[u] = z;
        }
        *reinterpret_cast<V*>(yb + (int64_t)o * N) = v;
      }
    }
}

template <int Q, int TO, int SUB>
__global__ __launch_bounds__(256) void linear_fwd_cf_kernel(const float* __restrict__ x, int64_t sx,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias, int64_t R, int N, int Cout,
                                                            int transw, LinEpi e, int64_t tpc) {
  extern __shared__ float Ws[];
  linear_cf_body<Q, TO, SUB>(x, sx, w, bias, R, N, Cout, transw, e, tpc, blockIdx.x, Ws);
}

// Two independent channels-first layers in one launch (pk_linear_ex2): blocks [0, nb0) run
// problem 0, the rest problem 1 — the pair shares one launch's ramp and tail (the refinement's
// q / stacked k-v projections, Pq^T / [Pk; Pv]^T, the two shapes' last_lin).
struct CfProb {
  const float* x;
  int64_t sx;
  const float* w;
  const float* bias;
  int64_t R;
  int N, Cout, transw, pad;
  int64_t tpc;
  LinEpi e;
};

template <int Q0, int TO0, int Q1, int TO1, int SUB>
__global__ __launch_bounds__(256) void linear_cf_pair_kernel(const CfProb p0, const CfProb p1, int nb0) {
  extern __shared__ float Ws[];
  if ((int)blockIdx.x < nb0)
    linear_cf_body<Q0, TO0, SUB>(p0.x, p0.sx, p0.w, p0.bias, p0.R, p0.N, p0.Cout, p0.transw, p0.e, p0.tpc,
                                 blockIdx.x, Ws);
  else
    linear_cf_body<Q1, TO1, SUB>(p1.x, p1.sx, p1.w, p1.bias, p1.R, p1.N, p1.Cout, p1.transw, p1.e, p1.tpc,
                                 (int64_t)blockIdx.x - nb0, Ws);
}

// Thin layers (Cin <= 4 or Cout <= 4: DiffusionNet's first_lin 3 -> 64, the overlap head's
// 32 -> 1 and its input gradient 1 -> 32): too little contraction for MFMA tiles, so plain
// FMAs with the weight in LDS, organised for coalesced memory traffic.
//   rows layout: thread = (point, 4 consecutive outputs), one float4 store per thread
//   channels-first: thread = point n of an item, Cout coalesced row stores
constexpr int kThinMaxW = 4096;  // Cout * Cin floats in LDS

template <int LAYOUT, int CINT>  // CINT: compile-time Cin (1..4), or 0 (runtime Cin, Cout <= 4)
__global__ __launch_bounds__(256) void linear_thin_kernel(const float* __restrict__ x, int64_t sx,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias, int64_t R, int N, int Cin_,
                                                          int Cout, int transw, LinEpi e) {
  const int relu = e.relu;
  const float* __restrict__ mask = e.mask;
  float* __restrict__ y = e.y;
  __shared__ float Ws[kThinMaxW];  // Ws[o * Cin + k]
  __shared__ float bs[kLfMaxC];
  const int Cin = CINT > 0 ? CINT : Cin_;
  // rows layout, compile-time Cin, no prologue (first_lin 3 -> 64): the point's inputs are in
  // flight while the weight is staged (one memory latency instead of two before the stores)
  float xe[CINT > 0 ? CINT : 1];
  if (LAYOUT == 0 && CINT > 0) {
    const int G = (Cout + 3) >> 2;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = t < R * G ? t / G : 0;
#pragma unroll
    for (int k = 0; k < (CINT > 0 ? CINT : 1); ++k) xe[k] = (t < R * G && e.pre == nullptr) ? x[r * sx + k] : 0.f;
  }
  for (int e = threadIdx.x; e < Cout * Cin; e += 256) {
    const int o = e / Cin, k = e - o * Cin;
    Ws[e] = transw ? w[(int64_t)k * Cout + o] : w[e];
  }
  for (int o = threadIdx.x; o < Cout; o += 256) bs[o] = bias ? bias[o] : 0.f;
  __syncthreads();
  if (LAYOUT == 0) {
    const int G = (Cout + 3) >> 2;  // output quads per point
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= R * G) return;
    const int64_t r = t / G;
    const int o0 = (int)(t - r * G) * 4;
    float acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = o0 + u < Cout ? bs[o0 + u] : 0.f;
    int k0 = 0;
    if (CINT == 0 && e.pre == nullptr && ((sx | Cin) & 3) == 0 && (((uintptr_t)x) & 15) == 0) {
      // wide input rows (e.g. the overlap head's 32 -> 1): 16-B loads, all issued up front
      const float4* xr = reinterpret_cast<const float4*>(x + r * sx);
      for (; k0 + 16 <= Cin; k0 += 16) {
        float4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = xr[(k0 >> 2) + j];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xs[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int k = k0 + 4 * j + i;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (o0 + u < Cout) acc[u] = fmaf(xs[i], Ws[(o0 + u) * Cin + k], acc[u]);
          }
        }
      }
    }
#pragma unroll 4
    for (int k = k0; k < Cin; ++k) {
      float xv = (CINT > 0 && e.pre == nullptr) ? xe[CINT > 0 ? k : 0] : x[r * sx + k];
      if (e.pre) {
        const float s = e.pre[r * sx + k];
        xv = xv * (s * (1.f - s));
        if (e.pre_out && o0 == 0) e.pre_out[r * sx + k] = xv;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (o0 + u < Cout) acc[u] = fmaf(xv, Ws[(o0 + u) * Cin + k], acc[u]);
    }
    float mk[4] = {1.f, 1.f, 1.f, 1.f};
    if (mask != nullptr) {  // workgroup-uniform; the loads at clamped indices, then one wait
#pragma unroll
      for (int u = 0; u < 4; ++u) mk[u] = mask[r * Cout + (o0 + u < Cout ? o0 + u : 0)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mk[u] <= 0.f ? 0.f : lin_act(relu, acc[u]);
    if ((Cout & 3) == 0 && (e.sy & 3) == 0) {
      *reinterpret_cast<float4*>(y + r * e.sy + o0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (o0 + u < Cout) y[r * e.sy + o0 + u] = acc[u];
    }
  } else {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= R) return;
    const int64_t b = t / N, n = t - b * N;
    const float* __restrict__ xb = x + b * sx + n;
    float* __restrict__ yb = y + b * e.sy + n;
    const int64_t mo = b * Cout * (int64_t)N + n - (yb - y);  // mask index = (yb - y) + mo + o N
    if (CINT > 0) {  // few inputs in registers, one coalesced row store per output
      float xv[CINT > 0 ? CINT : 1];
#pragma unroll
      for (int k = 0; k < CINT; ++k) {
        xv[k] = xb[(int64_t)k * N];
        if (e.pre) {
          const int64_t xi = (xb - x) + (int64_t)k * N;
          const float s = e.pre[xi];
          xv[k] = xv[k] * (s * (1.f - s));
          if (e.pre_out) e.pre_out[xi] = xv[k];
        }
      }
      for (int o = 0; o < Cout; ++o) {
        float a = bs[o];
#pragma unroll
        for (int k = 0; k < CINT; ++k) a = fmaf(xv[k], Ws[o * CINT + k], a);
        yb[(int64_t)o * N] = relu_mask(lin_act(relu, a), mask, (yb - y) + mo + (int64_t)o * N);
      }
    } else {  // Cout <= 4: one coalesced row load per input channel
      float acc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = u < Cout ? bs[u] : 0.f;
#pragma unroll 8
      for (int k = 0; k < Cin; ++k) {
        float xv = xb[(int64_t)k * N];
        if (e.pre) {
          const int64_t xi = (xb - x) + (int64_t)k * N;
          const float s = e.pre[xi];
          xv = xv * (s * (1.f - s));
          if (e.pre_out) e.pre_out[xi] = xv;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < Cout) acc[u] = fmaf(xv, Ws[u * Cin + k], acc[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < Cout) yb[(int64_t)u * N] = relu_mask(lin_act(relu, acc[u]), mask, (yb - y) + mo + (int64_t)u * N);
    }
  }
}

}  // namespace

// argument checks and the epilogue record of one pk_linear_ex call (PK_OK or an error status)
static int lin_setup(const pk_linear_args* a, LinEpi& e, int64_t& sx_out) {
  PK_REQUIRE(a != nullptr);
  const int layout = a->layout, Cin = a->Cin, Cout = a->Cout, N = a->N;
  const int64_t R = a->R;
  PK_REQUIRE((layout == 0 || layout == 1) && R >= 0 && Cin > 0 && Cout > 0 && Cin <= kLfMaxC && Cout <= kLfMaxC);
  PK_REQUIRE(layout == 0 || (N > 0 && R % N == 0));
  PK_REQUIRE(a->act >= 0 && a->act <= 2);
  if (R == 0) return PK_OK;
  PK_REQUIRE(a->x && a->w && a->y);
  const int split = a->y2 ? a->split : Cout;
  PK_REQUIRE(split >= 1 && split <= Cout && (a->y2 == nullptr || (layout == 0 && !a->store_cf && split < Cout)));
  PK_REQUIRE(a->store_cf == 0 || (layout == 0 && N > 0 && R % N == 0));
  PK_REQUIRE(a->add == nullptr || (a->add_cols >= 1 && a->add_cols <= Cout));
  sx_out = a->ldx ? a->ldx : (layout == 0 ? Cin : (int64_t)Cin * N);
  e = LinEpi{};
  e.y = a->y;
  e.sy = a->ldy ? a->ldy : (layout == 0 && !a->store_cf ? split : (int64_t)Cout * N);
  e.y2 = a->y2;
  e.sy2 = a->ldy2 ? a->ldy2 : Cout - split;
  e.split = split;
  e.add = a->add;
  e.sa = a->lda ? a->lda : (layout == 0 ? (int64_t)(a->add_cols > 0 ? a->add_cols : Cout) : (int64_t)Cout * N);
  e.add_cols = a->add ? a->add_cols : 0;
  e.mask = a->mask;
  e.relu = a->act;
  e.store_cf = a->store_cf;
  e.N = N;
  e.pre = a->pre;
  e.pre_out = a->pre_out;
  e.add2 = a->add2;
  e.sa2 = a->lda2 ? a->lda2 : (int64_t)Cout * N;
  e.w2 = a->w2;
  e.bias2 = a->bias2;
  e.wsplit = a->w2 ? a->wsplit : (1 << 30);
  PK_REQUIRE((a->w2 == nullptr && a->add2 == nullptr && a->bias2 == nullptr) ||
             (layout == 1 && (Cin == 16 || Cin == 32 || Cin == 64 || Cin == 128) &&
              Cin > 4 && Cout > 4 && !a->store_cf && a->y2 == nullptr));
  PK_REQUIRE(a->w2 == nullptr || (a->wsplit > 0 && a->wsplit < (a->transw ? Cin : Cout)));
  PK_REQUIRE(a->bias2 == nullptr || (a->w2 != nullptr && !a->transw));
  PK_REQUIRE((e.pre == nullptr && e.relu != 2) || ((Cin <= 4 || Cout <= 4) && Cin * Cout <= kThinMaxW));
  return PK_OK;
}

// points per wave of the channels-first kernel: 16 SUB, as many as keep >= 1024 waves and <= 64
// operand VGPRs; SUB-aligned items and strides for the vector loads / stores
// development knob PK_CF_SUBMAX (1, 2, 4): cap on the channels-first points-per-lane choice
static int cf_submax() {
#ifdef PK_DEVBUILD
  static const int v = [] { const char* e = std::getenv("PK_CF_SUBMAX"); return e ? std::atoi(e) : 4; }();
  return v;
#else
  return 4;
#endif
}

static int cf_sub(int64_t R, int N, int Cin, int64_t sx, const LinEpi& e) {
  // 16 points per wave below 131,072 rows (round 6: the configs[1] step's 65,536-row layers ran
  // 11 % faster than with 32 — more waves in flight per CU; tools/cf_sub_ab.sh)
  int sub = R >= 131072 ? 4 : 1;
  sub = std::min(sub, cf_submax());
  sub = std::min(sub, 256 / Cin);
  while (sub > 1 && N % (16 * sub)) sub >>= 1;  // N % 16 != 0: SUB = 1 with ragged item tails
  while (sub > 1 && ((sx % sub) || (e.sy % sub) || (e.add && (e.sa % sub)) || (e.add2 && (e.sa2 % sub)))) sub >>= 1;
  return sub;
}

extern "C" int pk_linear_ex2(const pk_linear_args* a0, const pk_linear_args* a1, void* stream) {
  PK_REQUIRE(a0 != nullptr && a1 != nullptr);
  LinEpi e0, e1;
  int64_t sx0 = 0, sx1 = 0;
  int rc = lin_setup(a0, e0, sx0);
  if (rc != PK_OK) return rc;
  rc = lin_setup(a1, e1, sx1);
  if (rc != PK_OK) return rc;
  auto cf_ok = [](const pk_linear_args* a) {
    return a->layout == 1 && a->R > 0 && (a->Cin == 32 || a->Cin == 64) && (a->Cout == 32 || a->Cout == 64) &&
           a->y2 == nullptr && !a->store_cf && a->pre == nullptr && a->act <= 1;
  };
  const int sub0 = cf_ok(a0) ? cf_sub(a0->R, a0->N, a0->Cin, sx0, e0) : 0;
  const int sub1 = cf_ok(a1) ? cf_sub(a1->R, a1->N, a1->Cin, sx1, e1) : 0;
  if (sub0 == 0 || sub0 != sub1 || sub0 == 4) {  // not a pair this kernel takes: two launches
    rc = pk_linear_ex(a0, stream);
    return rc != PK_OK ? rc : pk_linear_ex(a1, stream);
  }
  auto prob = [](const pk_linear_args* a, const LinEpi& e, int64_t sx, int sub) {
    CfProb p{};
    p.x = a->x;
    p.sx = sx;
    p.w = a->w;
    p.bias = a->bias;
    p.R = a->R;
    p.N = a->N;
    p.Cout = a->Cout;
    p.transw = a->transw;
    p.tpc = (a->N + 16 * sub - 1) / (16 * sub);
    p.e = e;
    return p;
  };
  const CfProb p0 = prob(a0, e0, sx0, sub0), p1 = prob(a1, e1, sx1, sub1);
  const int64_t nb0 = ((a0->R / a0->N) * p0.tpc + 3) / 4, nb1 = ((a1->R / a1->N) * p1.tpc + 3) / 4;
  PK_REQUIRE(nb0 + nb1 <= (int64_t)INT32_MAX);
  const int TO0 = a0->Cout / 16, TO1 = a1->Cout / 16;
  const size_t lds = sizeof(float) * std::max((size_t)(16 * TO0) * (a0->Cin + 4), (size_t)(16 * TO1) * (a1->Cin + 4));
  hipStream_t st = pk::as_stream(stream);
  const dim3 grid((unsigned)(nb0 + nb1));
#define PK_CFP(Q0, T0, Q1, T1, S) \
  hipLaunchKernelGGL((linear_cf_pair_kernel<Q0, T0, Q1, T1, S>), grid, dim3(256), lds, st, p0, p1, (int)nb0)
#define PK_CFP_S(Q0, T0, Q1, T1) \
  do { if (sub0 == 2) PK_CFP(Q0, T0, Q1, T1, 2); else PK_CFP(Q0, T0, Q1, T1, 1); } while (0)
#define PK_CFP_1(Q0, T0)                                                    \
  do {                                                                      \
    const int q1 = a1->Cin / 16;                                            \
    if (q1 == 2 && TO1 == 2) PK_CFP_S(Q0, T0, 2, 2);                        \
    else if (q1 == 2) PK_CFP_S(Q0, T0, 2, 4);                               \
    else if (TO1 == 2) PK_CFP_S(Q0, T0, 4, 2);                              \
    else PK_CFP_S(Q0, T0, 4, 4);                                            \
  } while (0)
  const int q0 = a0->Cin / 16;
  if (q0 == 2 && TO0 == 2) PK_CFP_1(2, 2);
  else if (q0 == 2) PK_CFP_1(2, 4);
  else if (TO0 == 2) PK_CFP_1(4, 2);
  else PK_CFP_1(4, 4);
#undef PK_CFP_1
#undef PK_CFP_S
#undef PK_CFP
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_linear_ex(const pk_linear_args* a, void* stream) {
  PK_REQUIRE(a != nullptr);
  const int layout = a->layout, Cin = a->Cin, Cout = a->Cout, N = a->N;
  const int64_t R = a->R;
  PK_REQUIRE((layout == 0 || layout == 1) && R >= 0 && Cin > 0 && Cout > 0 && Cin <= kLfMaxC && Cout <= kLfMaxC);
  PK_REQUIRE(layout == 0 || (N > 0 && R % N == 0));
  PK_REQUIRE(a->act >= 0 && a->act <= 2);
  if (R == 0) return PK_OK;
  PK_REQUIRE(a->x && a->w && a->y);
  const int split = a->y2 ? a->split : Cout;
  PK_REQUIRE(split >= 1 && split <= Cout && (a->y2 == nullptr || (layout == 0 && !a->store_cf && split < Cout)));
  PK_REQUIRE(a->store_cf == 0 || (layout == 0 && N > 0 && R % N == 0));
  PK_REQUIRE(a->add == nullptr || (a->add_cols >= 1 && a->add_cols <= Cout));
  // default strides: contiguous
  const int64_t sx = a->ldx ? a->ldx : (layout == 0 ? Cin : (int64_t)Cin * N);
  const int64_t sy = a->ldy ? a->ldy : (layout == 0 && !a->store_cf ? split : (int64_t)Cout * N);
  LinEpi e{};
  e.y = a->y;
  e.sy = sy;
  e.y2 = a->y2;
  e.sy2 = a->ldy2 ? a->ldy2 : Cout - split;
  e.split = split;
  e.add = a->add;
  e.sa = a->lda ? a->lda : (layout == 0 ? (int64_t)(a->add_cols > 0 ? a->add_cols : Cout) : (int64_t)Cout * N);
  e.add_cols = a->add ? a->add_cols : 0;
  e.mask = a->mask;
  e.relu = a->act;
  e.store_cf = a->store_cf;
  e.N = N;
  e.pre = a->pre;
  e.pre_out = a->pre_out;
  e.add2 = a->add2;
  e.sa2 = a->lda2 ? a->lda2 : (int64_t)Cout * N;
  e.w2 = a->w2;
  e.bias2 = a->bias2;
  e.wsplit = a->w2 ? a->wsplit : (1 << 30);
  // stacked weights and the second add operand: channels-first MFMA kernel only
  PK_REQUIRE((a->w2 == nullptr && a->add2 == nullptr && a->bias2 == nullptr) ||
             (layout == 1 && (Cin == 16 || Cin == 32 || Cin == 64 || Cin == 128) &&
              Cin > 4 && Cout > 4 && !a->store_cf && a->y2 == nullptr));
  PK_REQUIRE(a->w2 == nullptr || (a->wsplit > 0 && a->wsplit < (a->transw ? Cin : Cout)));
  PK_REQUIRE(a->bias2 == nullptr || (a->w2 != nullptr && !a->transw));
  const float* x = a->x;
  const float* w = a->w;
  const float* bias = a->bias;
  const int transw = a->transw;
  hipStream_t st = pk::as_stream(stream);
  const bool plain_out = e.y2 == nullptr && e.add == nullptr && !e.store_cf;
  PK_REQUIRE((e.pre == nullptr && e.relu != 2) || ((Cin <= 4 || Cout <= 4) && Cin * Cout <= kThinMaxW));
  if ((Cin <= 4 || Cout <= 4) && Cin * Cout <= kThinMaxW) {
    PK_REQUIRE(plain_out);  // the thin kernels take strides only
    const int64_t threads = layout == 0 ? R * ((Cout + 3) / 4) : R;
    const dim3 grid((unsigned)((threads + 255) / 256));
#define PK_THIN(L, C)                                                                                           \
  hipLaunchKernelGGL((linear_thin_kernel<L, C>), grid, dim3(256), 0, st, x, sx, w, bias, R, N, Cin, Cout, transw, e)
    const int ct = Cin <= 4 ? Cin : 0;  // Cin > 4 here means Cout <= 4
    if (layout == 0) {
      if (ct == 1) PK_THIN(0, 1); else if (ct == 2) PK_THIN(0, 2); else if (ct == 3) PK_THIN(0, 3);
      else if (ct == 4) PK_THIN(0, 4); else PK_THIN(0, 0);
    } else {
      if (ct == 1) PK_THIN(1, 1); else if (ct == 2) PK_THIN(1, 2); else if (ct == 3) PK_THIN(1, 3);
      else if (ct == 4) PK_THIN(1, 4); else PK_THIN(1, 0);
    }
#undef PK_THIN
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  if (layout == 0 && (Cin == 16 || Cin == 32 || Cin == 64 || Cin == 128) && sx % 4 == 0) {
    // 16-point tiles, 4 per block, at most two blocks per CU's worth of waves in flight
    const int64_t tiles = (R + 15) / 16;
    const unsigned blocks = (unsigned)std::min<int64_t>((tiles + 3) / 4, (int64_t)kRowsMaxBlocks);
    const int TO = Cout <= 16 ? 1 : Cout <= 32 ? 2 : Cout <= 64 ? 4 : 8;
    auto pick = [&](auto q, auto gen) {
      constexpr int Q = decltype(q)::value;
      constexpr bool G = decltype(gen)::value;
      return TO == 1 ? linear_fwd_rows_kernel<Q, 1, G>
             : TO == 2 ? linear_fwd_rows_kernel<Q, 2, G>
             : TO == 4 ? linear_fwd_rows_kernel<Q, 4, G> : linear_fwd_rows_kernel<Q, 8, G>;
    };
    auto pickq = [&](auto gen) {
      return Cin == 16 ? pick(std::integral_constant<int, 1>{}, gen)
             : Cin == 32 ? pick(std::integral_constant<int, 2>{}, gen)
             : Cin == 64 ? pick(std::integral_constant<int, 4>{}, gen) : pick(std::integral_constant<int, 8>{}, gen);
    };
    // plain: no mask, no residual add, one contiguous output (split == Cout)
    const bool plain = e.mask == nullptr && e.add == nullptr && e.y2 == nullptr && !e.store_cf && e.split >= Cout;
#ifdef PK_DEVBUILD
    static const bool glds_on = getenv("PK_ROWS_GLDS") == nullptr || atoi(getenv("PK_ROWS_GLDS")) != 0;
#else
    constexpr bool glds_on = true;
#endif
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool glds_ok = glds_on && Cin >= 32 && Cout >= 32 && Cout % 16 == 0 && TO * (Cin / 16) <= 32 &&
                         e.relu <= 1 && !e.store_cf && al16(x) && al16(e.y) && e.sy % 4 == 0 &&
                         (e.y2 == nullptr || (al16(e.y2) && e.sy2 % 4 == 0 && split % 16 == 0)) &&
                         (e.mask == nullptr || al16(e.mask)) && (e.add == nullptr || (al16(e.add) && e.sa % 4 == 0));
    if (glds_ok) {
      const bool MK = e.mask != nullptr, AD = e.add != nullptr, SP = e.y2 != nullptr;
      const int slot = 16 * Cin + (MK ? 16 * Cout : 0) + (AD ? 16 * Cout : 0);
      const int D = 3 * 4 * slot * 4 <= 159 * 1024 ? 3 : 2;  // (the kernel's own constexpr D)
      const size_t ldsg = std::max((size_t)D * 4 * slot, (size_t)(16 * TO) * (Cin + 4)) * sizeof(float);
      const unsigned bg = (unsigned)std::min<int64_t>((tiles + 3) / 4, (int64_t)kRowsPersistCUs);
      auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(bg), dim3(256), ldsg, st, x, sx, w, bias, R, Cin, Cout, transw, e);
      };
      auto pe = [&](auto q, auto to) {
        constexpr int Qv = decltype(q)::value, TOv = decltype(to)::value;
        if (SP) {
          if (MK && AD) launch(linear_glds_rows_kernel<Qv, TOv, true, true, true>);
          else if (MK) launch(linear_glds_rows_kernel<Qv, TOv, true, false, true>);
          else if (AD) launch(linear_glds_rows_kernel<Qv, TOv, false, true, true>);
          else launch(linear_glds_rows_kernel<Qv, TOv, false, false, true>);
        } else {
          if (MK && AD) launch(linear_glds_rows_kernel<Qv, TOv, true, true, false>);
          else if (MK) launch(linear_glds_rows_kernel<Qv, TOv, true, false, false>);
          else if (AD) launch(linear_glds_rows_kernel<Qv, TOv, false, true, false>);
          else launch(linear_glds_rows_kernel<Qv, TOv, false, false, false>);
        }
      };
      using I2 = std::integral_constant<int, 2>;
      using I4 = std::integral_constant<int, 4>;
      using I8 = std::integral_constant<int, 8>;
      auto pt = [&](auto q) {  // TO x Q <= 32 (the weight's VGPRs)
        if (TO == 2) pe(q, I2{});
        else if (TO == 4) pe(q, I4{});
        else if constexpr (decltype(q)::value <= 4) pe(q, I8{});
      };
      if (Cin == 32) pt(I2{}); else if (Cin == 64) pt(I4{}); else pt(I8{});
      PK_CHECK_LAUNCH();
      return PK_OK;
    }
    auto kern = plain ? pickq(std::integral_constant<bool, false>{}) : pickq(std::integral_constant<bool, true>{});
    const size_t lds = sizeof(float) * (size_t)(16 * TO) * (Cin + 4);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, st, x, sx, w, bias, R, Cin, Cout, transw, e);
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  if (layout == 1 && (Cin == 16 || Cin == 32 || Cin == 64 || Cin == 128) && N > 0) {
    PK_REQUIRE(e.y2 == nullptr && !e.store_cf);
    // points per wave: 16 SUB (SUB = 4 from 131,072 rows, else 1: cf_sub), <= 64 operand VGPRs
    int sub = R >= 131072 ? 4 : 1;  // (as cf_sub)
    sub = std::min(sub, cf_submax());
    sub = std::min(sub, 256 / Cin);
    while (sub > 1 && N % (16 * sub)) sub >>= 1;  // N % 16 != 0: SUB = 1 with ragged item tails
    // vector loads / stores of SUB points need SUB-aligned batch strides
    while (sub > 1 && ((sx % sub) || (e.sy % sub) || (e.add && (e.sa % sub)) || (e.add2 && (e.sa2 % sub)))) sub >>= 1;
    const int TO = Cout <= 16 ? 1 : Cout <= 32 ? 2 : Cout <= 64 ? 4 : 8;
    auto pick = [&](auto q, auto u) {
      constexpr int Q = decltype(q)::value, U = decltype(u)::value;
      return TO == 1 ? linear_fwd_cf_kernel<Q, 1, U>
             : TO == 2 ? linear_fwd_cf_kernel<Q, 2, U>
             : TO == 4 ? linear_fwd_cf_kernel<Q, 4, U> : linear_fwd_cf_kernel<Q, 8, U>;
    };
    auto pickq = [&](auto u) {
      return Cin == 16 ? pick(std::integral_constant<int, 1>{}, u)
             : Cin == 32 ? pick(std::integral_constant<int, 2>{}, u)
             : Cin == 64 ? pick(std::integral_constant<int, 4>{}, u) : pick(std::integral_constant<int, 8>{}, u);
    };
    auto kern = sub == 4 ? pickq(std::integral_constant<int, 4>{})
                : sub == 2 ? pickq(std::integral_constant<int, 2>{}) : pickq(std::integral_constant<int, 1>{});
    const int64_t tpc = (N + 16 * sub - 1) / (16 * sub);
    const int64_t tiles = (R / N) * tpc;
    const size_t lds = sizeof(float) * (size_t)(16 * TO) * (Cin + 4);
    hipLaunchKernelGGL(kern, dim3((unsigned)((tiles + 3) / 4)), dim3(256), lds, st, x, sx, w, bias, R, N, Cout,
                       transw, e, tpc);
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  // generic fallback kernel: contiguous operands only
  PK_REQUIRE(plain_out && sx == (layout == 0 ? Cin : (int64_t)Cin * N) &&
             e.sy == (layout == 0 ? Cout : (int64_t)Cout * N));
  const unsigned blocks = (unsigned)((R + 127) / 128);
  const size_t lds = sizeof(float) * (size_t)Cout * (((Cin + 3) & ~3) + 1);
  if (layout == 0)
    hipLaunchKernelGGL(linear_fwd_kernel<0>, dim3(blocks), dim3(256), lds, st, x, w, bias, R, N, Cin, Cout, transw,
                       e.relu, e.mask, e.y);
  else
    hipLaunchKernelGGL(linear_fwd_kernel<1>, dim3(blocks), dim3(256), lds, st, x, w, bias, R, N, Cin, Cout, transw,
                       e.relu, e.mask, e.y);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_linear_fwd(const float* x, const float* w, const float* bias, int layout, int64_t R, int N,
                             int Cin, int Cout, int transw, int relu, const float* mask, float* y, void* stream) {
  pk_linear_args a{};
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.layout = layout;
  a.R = R;
  a.N = N;
  a.Cin = Cin;
  a.Cout = Cout;
  a.transw = transw;
  a.act = relu ? 1 : 0;
  a.mask = mask;
  a.y = y;
  a.pre = nullptr;
  a.pre_out = nullptr;
  return pk_linear_ex(&a, stream);
}

// Slicing of a grouped call list. Pipeline problems (wgrad_glds_grouped_kernel: shape on
// wg_shape_id, channels-first only with N % 16 == 0, 16-B aligned operands) get blocks in
// proportion to their cost (wg_cost), about kWgBlocks in all (slices of whole 16-row tiles, >= 64
// rows); the others keep round 3's wgrad_v2 slicing. S[c] partials of call c, SL[c] rows each.
// development variants of the pipeline kernel (limiter study): 1 no MFMAs, 2 no LDS reads either
static int wg_variant() {
#ifdef PK_DEVBUILD
  static const int v = getenv("PK_WG_VAR") ? atoi(getenv("PK_WG_VAR")) : 0;
  return v;
#else
  return 0;
#endif
}

static bool wg_on_pipeline(const pk_wgrad_call& k) {
#ifdef PK_DEVBUILD
  static const bool on = getenv("PK_WG_GLDS") == nullptr || atoi(getenv("PK_WG_GLDS")) != 0;
  if (!on) return false;
#endif
  return k.R > 0 && wg_shape_id(k.I, k.O, k.layout) >= 0 && (k.layout == 0 || k.N % 16 == 0) &&
         ((reinterpret_cast<uintptr_t>(k.x) | reinterpret_cast<uintptr_t>(k.dy)) & 15) == 0;
}

// a problem's time at the chip's rates, in HBM bytes: max(its bytes, its flops / (157.3 TF /
// 8 TB/s)) — the thin layers are byte-bound, the 128 x 64 ones flop-bound
static double wg_cost(const pk_wgrad_call& k) {
  const double bytes = 4.0 * (double)k.R * (k.I + k.O), flops = 2.0 * (double)k.R * k.I * k.O;
  return bytes > flops / 19.66 ? bytes : flops / 19.66;
}

// Blocks: one resident per CU (each holds 144 KB of LDS), so the launch runs in rounds; 4 x the
// CU count lets the dispatcher balance what the cost model misses (measured, tools/wg_bench.py
// under rocprofv3, whole step's call list: 240 / 248 / 252 / 256 blocks 243-248 us — one round,
// bound by its slowest slice — 496 135 us, 1024 136 us, 2048 155 us). Shares of the budget by
// cost, floored (>= 1 block, >= 64 rows each), leftovers to the largest remainders.
static int wg_budget() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = kWgBlocks / 4;
    n *= 4;
#ifdef PK_DEVBUILD
    if (const char* e = getenv("PK_WG_BUDGET")) n = atoi(e) > 0 ? atoi(e) : n;  // (development knob)
#endif
    return n;
  }();
  return cus;
}

static void wg_plan(const pk_wgrad_call* calls, int n, std::vector<int64_t>& S, std::vector<int64_t>& SL,
                    std::vector<char>& glds) {
  S.assign(n, 0);
  SL.assign(n, 0);
  glds.assign(n, 0);
  double wtot = 0.0;
  int ne = 0;
  for (int c = 0; c < n; ++c)
    if (wg_on_pipeline(calls[c])) {
      wtot += wg_cost(calls[c]);
      ++ne;
    }
  std::vector<int64_t> nb(n, 0);
  std::vector<double> want(n, 0.0);
  if (ne > 0) {
    const int budget = wg_budget() > ne ? wg_budget() : ne;
    int64_t tot = 0;
    for (int c = 0; c < n; ++c) {
      if (!wg_on_pipeline(calls[c])) continue;
      const int64_t cap = (calls[c].R + 63) / 64;
      want[c] = wg_cost(calls[c]) / wtot * budget;
      int64_t v = (int64_t)want[c];
      nb[c] = v < 1 ? 1 : v > cap ? cap : v;
      tot += nb[c];
    }
    while (tot > budget) {  // (only from the >= 1 floors) take from the largest
      int best = -1;
      for (int c = 0; c < n; ++c)
        if (nb[c] > 1 && (best < 0 || nb[c] > nb[best])) best = c;
      if (best < 0) break;
      --nb[best];
      --tot;
    }
    while (tot < budget) {  // leftover CUs to the largest remainders (below their row cap)
      int best = -1;
      double rem = -1e300;
      for (int c = 0; c < n; ++c) {
        if (!wg_on_pipeline(calls[c]) || nb[c] >= (calls[c].R + 63) / 64) continue;
        const double r = want[c] - (double)nb[c];
        if (r > rem) {
          rem = r;
          best = c;
        }
      }
      if (best < 0) break;
      ++nb[best];
      ++tot;
    }
  }
  for (int c = 0; c < n; ++c) {
    const pk_wgrad_call& k = calls[c];
    if (k.R <= 0) continue;
    if (wg_on_pipeline(k)) {
      glds[c] = 1;
      SL[c] = ((k.R + nb[c] - 1) / nb[c] + 15) / 16 * 16;
    } else {
      SL[c] = grouped_slice_rows(k.R);
    }
    S[c] = (k.R + SL[c] - 1) / SL[c];
  }
}

extern "C" int64_t pk_linear_wgrad_grouped_work(const pk_wgrad_call* calls, int n) {
  if (n < 0 || (n > 0 && calls == nullptr)) return -1;
  std::vector<int64_t> S, SL;
  std::vector<char> glds;
  wg_plan(calls, n, S, SL, glds);
  int64_t tot = 0;
  for (int c = 0; c < n; ++c) tot += S[c] * ((int64_t)calls[c].O * calls[c].I + calls[c].O);
  return tot;
}

extern "C" int pk_linear_wgrad_grouped(const pk_wgrad_call* calls, int n, float* work, int64_t work_elems,
                                       void* stream) {
  PK_REQUIRE(n >= 0 && (n == 0 || calls != nullptr));
  hipStream_t st = pk::as_stream(stream);
  // validate; a call with accumulate = 1 must name the dw (and db) of an earlier call
  std::vector<int> first(n, -1), second(n, -1);
  for (int c = 0; c < n; ++c) {
    const pk_wgrad_call& k = calls[c];
    PK_REQUIRE(k.dw && k.R >= 0 && k.I > 0 && k.O > 0 && k.I <= kMaxC && k.O <= kMaxC);
    PK_REQUIRE(((k.O + 31) / 32) * ((k.I + 31) / 32) <= kV2Waves);  // one 32x32 tile per wave
    PK_REQUIRE(k.layout == 0 || (k.layout == 1 && k.N > 0));
    PK_REQUIRE((k.sx == 0 && k.sdy == 0) || (k.layout == 1 && k.sx >= 0 && k.sdy >= 0 && k.sx % 4 == 0 &&
                                               k.sdy % 4 == 0));
    PK_REQUIRE(k.R == 0 || (k.x && k.dy));
    if (k.accumulate) {
      int f = -1;
      for (int q = 0; q < c; ++q)
        if (calls[q].dw == k.dw && !calls[q].accumulate) f = q;
      PK_REQUIRE(f >= 0 && second[f] < 0 && calls[f].I == k.I && calls[f].O == k.O && calls[f].db == k.db);
      second[f] = c;
    }
  }
  const int64_t need = pk_linear_wgrad_grouped_work(calls, n);
  PK_REQUIRE(need <= work_elems && (need == 0 || work != nullptr));
  std::vector<int64_t> S, SLv, off(n, 0);
  std::vector<char> glds;
  wg_plan(calls, n, S, SLv, glds);
  int64_t o = 0;
  for (int c = 0; c < n; ++c) {
    off[c] = o;
    o += S[c] * ((int64_t)calls[c].O * calls[c].I + calls[c].O);
  }
  // pipeline partials: chunks of <= kGroupMax problems
  {
    WgradProblems tp{};
    int blocks = 0;
    auto flush = [&]() -> int {
      if (tp.G == 0) return PK_OK;
      hipLaunchKernelGGL(wgrad_glds_grouped_kernel, dim3(blocks), dim3(256), kWgLdsBytes, st, tp);
      PK_CHECK_LAUNCH();
      tp.G = 0;
      blocks = 0;
      return PK_OK;
    };
    for (int c = 0; c < n; ++c) {
      const pk_wgrad_call& k = calls[c];
      if (S[c] == 0 || !glds[c]) continue;
      WgradProblem& P = tp.p[tp.G++];
      P = WgradProblem{k.x, k.dy, work + off[c], k.R, k.I, k.O, k.N, k.layout, (int)SLv[c], (int)S[c], blocks,
                       wg_variant(), k.sx, k.sdy};
      blocks += (int)S[c];
      if (tp.G == kGroupMax) {
        const int rc = flush();
        if (rc != PK_OK) return rc;
      }
    }
    const int rc = flush();
    if (rc != PK_OK) return rc;
  }
  // partials: chunks of <= kGroupMax problems
  WgradProblems tp{};
  int blocks = 0;
  auto flush_p = [&]() -> int {
    if (tp.G == 0) return PK_OK;
    hipLaunchKernelGGL(wgrad_grouped_kernel, dim3(blocks), dim3(64 * kV2Waves), 0, st, tp);
    PK_CHECK_LAUNCH();
    tp.G = 0;
    blocks = 0;
    return PK_OK;
  };
  for (int c = 0; c < n; ++c) {
    const pk_wgrad_call& k = calls[c];
    if (S[c] == 0 || glds[c]) continue;
    WgradProblem& P = tp.p[tp.G++];
    P = WgradProblem{k.x, k.dy, work + off[c], k.R, k.I, k.O, k.N, k.layout, (int)SLv[c], (int)S[c], blocks, 0,
                     k.sx, k.sdy};
    blocks += (int)S[c];
    if (tp.G == kGroupMax) {
      const int rc = flush_p();
      if (rc != PK_OK) return rc;
    }
  }
  int rc = flush_p();
  if (rc != PK_OK) return rc;
  // reductions: one output per non-accumulating call (plus its accumulating partner)
  WgradOuts to{};
  blocks = 0;
  auto flush_r = [&]() -> int {
    if (to.G == 0) return PK_OK;
    hipLaunchKernelGGL(wgrad_grouped_reduce_kernel, dim3(blocks), dim3(64 * kRedGroups), 0, st, to);
    PK_CHECK_LAUNCH();
    to.G = 0;
    blocks = 0;
    return PK_OK;
  };
  for (int c = 0; c < n; ++c) {
    const pk_wgrad_call& k = calls[c];
    if (k.accumulate) continue;
    int segs[2] = {c, second[c]};
    WgradOut W{};
    W.dw = k.dw;
    W.db = k.db;
    W.OI = k.O * k.I;
    W.O = k.O;
    W.nseg = 0;
    for (int q = 0; q < 2; ++q) {
      const int cc = segs[q];
      if (cc < 0 || S[cc] == 0) continue;  // no rows: contributes zero
      W.part[W.nseg] = work + off[cc];
      W.S[W.nseg] = (int)S[cc];
      ++W.nseg;
    }
    if (W.nseg == 0) {  // no rows in any feeding call: the gradient is zero
      hipError_t e = pk::zero_async(k.dw, sizeof(float) * k.O * k.I, st);
      if (e == hipSuccess && k.db) e = pk::zero_async(k.db, sizeof(float) * k.O, st);
      if (e != hipSuccess) return (int)e;
      continue;
    }
    W.blk0 = blocks;
    to.p[to.G++] = W;
    blocks += (W.OI + W.O + 63) / 64;
    if (to.G == kGroupMax) {
      rc = flush_r();
      if (rc != PK_OK) return rc;
    }
  }
  return flush_r();
}
