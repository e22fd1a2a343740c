// H7 DiffusionNet block MLP, forward fused (upstream diffusion_net/layers.py
// DiffusionNetBlock.forward as configured at models/dpfm.py:22-30, C_width = 64):
//   cat = [x_in, x_diffuse]                                   [R, 128]
//   h1  = relu(cat W1^T + b1)        W1 [64, 128]              [R, 64]
//   h2  = relu(h1 W2^T + b2)         W2 [64, 64]
//   y   = h2 W3^T + b3 + x_in        W3 [64, 64]  (the block's residual)
// One launch instead of cat + three layer launches + the residual add; h1 / h2 stay in the
// wave between layers (LDS transpose of the 16 x 64 tile from MFMA D layout to A layout).
// cat, h1 and h2 are written because the backward needs them (the weight gradients' x and
// the ReLU masks). f32 MFMA v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation):
//   A[m][k] = activation of point m at channel k, B[k][n] = W[o = 16 t + n][k]
//   -> lane (m, g) holds D[point 4 g + r][output 16 t + m], r = 0..3.
// Block = 8 waves, weights staged once in LDS (68 KB) plus a 16 x 68 float tile per wave
// (35 KB); waves walk 16-point tiles grid-stride with the next tile's
// inputs in flight.
#include "common.hpp"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kC = 64;            // C_width
constexpr int kWaves = 8;
constexpr int kS1 = 2 * kC + 4;   // W1 row stride (16-B aligned, conflict-spread)
constexpr int kS2 = kC + 4;       // W2 / W3 / activation tile row stride

template <int Q, int S>
__device__ __forceinline__ void mma_layer(const f32x4* a, const float* __restrict__ Ws, int m, int g,
                                          f32x4 (&acc)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    f32x4 wv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wv[t] = *reinterpret_cast<const f32x4*>(&Ws[(t * 16 + m) * S + 16 * q + 4 * g]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][i], wv[t][i], acc[t], 0, 0, 0);
  }
}

__global__ __launch_bounds__(64 * kWaves) void mlp3_fwd_kernel(
    const float* __restrict__ xa, const float* __restrict__ xb, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ w3, const float* __restrict__ b3, int64_t R, float* __restrict__ cat_out,
    float* __restrict__ h1_out, float* __restrict__ h2_out, float* __restrict__ y_out) {
  __shared__ __attribute__((aligned(16))) float W1s[kC * kS1];
  __shared__ __attribute__((aligned(16))) float W2s[kC * kS2];
  __shared__ __attribute__((aligned(16))) float W3s[kC * kS2];
  __shared__ __attribute__((aligned(16))) float act[kWaves * 16 * kS2];
  const int tid = threadIdx.x, lane = pk::lane_id(), w = pk::wave_id();
  const int m = lane & 15, g = lane >> 4;
  for (int e = tid; e < kC * 2 * kC / 4; e += 64 * kWaves) {
    const int o = e / (2 * kC / 4), k4 = e - o * (2 * kC / 4);
    *reinterpret_cast<f32x4*>(&W1s[o * kS1 + 4 * k4]) = *reinterpret_cast<const f32x4*>(w1 + 4 * (int64_t)e);
  }
  for (int e = tid; e < kC * kC / 4; e += 64 * kWaves) {
    const int o = e / (kC / 4), k4 = e - o * (kC / 4);
    *reinterpret_cast<f32x4*>(&W2s[o * kS2 + 4 * k4]) = *reinterpret_cast<const f32x4*>(w2 + 4 * (int64_t)e);
    *reinterpret_cast<f32x4*>(&W3s[o * kS2 + 4 * k4]) = *reinterpret_cast<const f32x4*>(w3 + 4 * (int64_t)e);
  }
  float bv1[4], bv2[4], bv3[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bv1[t] = b1[t * 16 + m];
    bv2[t] = b2[t * 16 + m];
    bv3[t] = b3[t * 16 + m];
  }
  __syncthreads();
  float* at = act + w * 16 * kS2;
  const int64_t T = (R + 15) >> 4, stride = (int64_t)gridDim.x * kWaves;
  int64_t tile = (int64_t)blockIdx.x * kWaves + w;
  f32x4 cur[8], nxt[8];
  auto load = [&](int64_t tl, f32x4 (&v)[8]) {
    const int64_t row = tl * 16 + m;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float* src = q < 4 ? xa + row * kC + 16 * q + 4 * g : xb + row * kC + 16 * (q - 4) + 4 * g;
      v[q] = row < R ? *reinterpret_cast<const f32x4*>(src) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (tile < T) load(tile, cur);
  for (; tile < T; tile += stride) {
    const int64_t tn = tile + stride;
    if (tn < T) load(tn, nxt);
    const int64_t row = tile * 16 + m;
    if (row < R) {
#pragma unroll
      for (int q = 0; q < 8; ++q) *reinterpret_cast<f32x4*>(cat_out + row * 2 * kC + 16 * q + 4 * g) = cur[q];
    }
    f32x4 acc[4];
    // layer 1: [x_in, x_diffuse] (from registers) -> h1
    mma_layer<8, kS1>(cur, W1s, m, g, acc);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = fmaxf(acc[t][r] + bv1[t], 0.f);
        at[(4 * g + r) * kS2 + t * 16 + m] = h;
        const int64_t pr = tile * 16 + 4 * g + r;
        if (pr < R) h1_out[pr * kC + t * 16 + m] = h;
      }
    __builtin_amdgcn_wave_barrier();  // the tile is complete (a wave's LDS ops run in order)
    f32x4 a2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a2[q] = *reinterpret_cast<const f32x4*>(&at[m * kS2 + 16 * q + 4 * g]);
    __builtin_amdgcn_wave_barrier();
    // layer 2: h1 -> h2
    mma_layer<4, kS2>(a2, W2s, m, g, acc);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = fmaxf(acc[t][r] + bv2[t], 0.f);
        at[(4 * g + r) * kS2 + t * 16 + m] = h;
        const int64_t pr = tile * 16 + 4 * g + r;
        if (pr < R) h2_out[pr * kC + t * 16 + m] = h;
      }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) a2[q] = *reinterpret_cast<const f32x4*>(&at[m * kS2 + 16 * q + 4 * g]);
    __builtin_amdgcn_wave_barrier();
    // layer 3: h2 -> y = h2 W3^T + b3 + x_in
    mma_layer<4, kS2>(a2, W3s, m, g, acc);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t pr = tile * 16 + 4 * g + r;
        if (pr < R) {
          const int o = t * 16 + m;
          y_out[pr * kC + o] = (acc[t][r] + bv3[t]) + xa[pr * kC + o];
        }
      }
#pragma unroll
    for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
  }
}

}  // namespace

extern "C" int pk_mlp3_fwd(const float* x_in, const float* x_diff, const float* w1, const float* b1, const float* w2,
                           const float* b2, const float* w3, const float* b3, int64_t R, int C, float* cat, float* h1,
                           float* h2, float* y, void* stream) {
  PK_REQUIRE(R >= 0 && C == kC);
  if (R == 0) return PK_OK;
  PK_REQUIRE(x_in && x_diff && w1 && b1 && w2 && b2 && w3 && b3 && cat && h1 && h2 && y);
  const int64_t tiles = (R + 15) / 16;
  const unsigned blocks = (unsigned)(((tiles + kWaves - 1) / kWaves) < 256 ? (tiles + kWaves - 1) / kWaves : 256);
  hipLaunchKernelGGL(mlp3_fwd_kernel, dim3(blocks), dim3(64 * kWaves), 0, pk::as_stream(stream), x_in, x_diff, w1, b1,
                     w2, b2, w3, b3, R, cat, h1, h2, y);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
