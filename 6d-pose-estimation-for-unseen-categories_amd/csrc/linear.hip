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
// 4 slice quarters (4 interleaved chains each), combined in a fixed order: deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                           const float* __restrict__ partb, int S,
                                                           int OI, int O, float* __restrict__ dw,
                                                           float* __restrict__ db) {
  __shared__ float red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int qtr = threadIdx.x >> 6;
  const bool is_w = e < OI;
  const bool is_b = !is_w && e < OI + O && db != nullptr;
  float v = 0.f;
  if (is_w || is_b) {
    const float* p = is_w ? part + e : partb + (e - OI);
    const int64_t st = is_w ? OI : O;
    const int s0 = (S * qtr) / 4, s1 = (S * (qtr + 1)) / 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
      a0 += p[(int64_t)s * st];
      a1 += p[(int64_t)(s + 1) * st];
      a2 += p[(int64_t)(s + 2) * st];
      a3 += p[(int64_t)(s + 3) * st];
    }
    for (; s < s1; ++s) a0 += p[(int64_t)s * st];
    v = (a0 + a1) + (a2 + a3);
  }
  red[qtr][threadIdx.x & 63] = v;
  __syncthreads();
  if (qtr == 0 && (is_w || is_b)) {
    const int t = threadIdx.x;
    const float r = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    if (is_w) dw[e] = r;
    else db[e - OI] = r;
  }
}

}  // namespace

extern "C" int pk_linear_wgrad(const float* x, const float* dy, int layout, int64_t R, int I, int O, int N,
                               float* work, float* dw, float* db, void* stream) {
  PK_REQUIRE((layout == 0 || layout == 1) && R >= 0 && I > 0 && O > 0 && I <= kMaxC && O <= kMaxC);
  PK_REQUIRE(layout == 0 || N > 0);
  PK_REQUIRE(((I + 15) / 16) * ((O + 15) / 16) <= 4 * kMaxTilesPerWave);
  PK_REQUIRE(dw != nullptr);
  hipStream_t s = pk::as_stream(stream);
  const int S = (int)((R + kSlice - 1) / kSlice);
  if (S == 0) {
    hipError_t e = pk::zero_async(dw, sizeof(float) * O * I, s);
    if (e == hipSuccess && db) e = pk::zero_async(db, sizeof(float) * O, s);
    return e == hipSuccess ? PK_OK : (int)e;
  }
  PK_REQUIRE(x && dy && work);
  float* part = work;
  float* partb = work + (int64_t)S * O * I;
  hipLaunchKernelGGL(wgrad_partial_kernel, dim3(S), dim3(256), 0, s, x, dy, layout, R, I, O, N, part, partb);
  PK_CHECK_LAUNCH();
  const int total = O * I + O;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(256), 0, s, part, partb, S, O * I, O,
                     dw, db);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
