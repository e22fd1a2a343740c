// Development probes (not in include/posekern.h): memory-stream shapes of the per-point layer
// kernels without their arithmetic, to separate what bounds linear_fwd_rows_kernel (20 us for a
// 128 -> 64 layer over 65,536 rows = 50 MB, 2.5 TB/s, while a torch copy of that size reaches
// 6 TB/s). y[r][o] = x[r][o] + x[r][64 + o] for o < 64 (x [R, 128], y [R, 64]):
//   mode 0  lane-linear 16-B loads and stores, one thread per (row, 4 outputs), many blocks
//   mode 1  the rows kernel's access shapes: one wave per 16-row tile, fragment loads (lane
//           (m, g) reads float4 16 q + 4 g of row m: 16 rows x 64 B per instruction), 4-B stores
//           in MFMA D layout (row 4 g + r, column 16 t + m), one tile per wave
//   mode 2  mode 1 plus the layer kernels' weight staging (64 x 132 floats into LDS from an L2-
//           resident weight, one barrier) before the tile is consumed
//   mode 3  mode 1 with 16-B stores (a lane owns 4 consecutive outputs of one row)
#include "common.hpp"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

__global__ __launch_bounds__(256) void probe_linear_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           int64_t R) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (row, quad)
  if (t >= R * 16) return;
  const int64_t r = t >> 4;
  const int q = (int)(t & 15);
  const float4 a = *reinterpret_cast<const float4*>(x + r * 128 + 4 * q);
  const float4 b = *reinterpret_cast<const float4*>(x + r * 128 + 64 + 4 * q);
  *reinterpret_cast<float4*>(y + r * 64 + 4 * q) = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int MODE>
__global__ __launch_bounds__(256) void probe_tile_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         float* __restrict__ y, int64_t R) {
  extern __shared__ float Ws[];
  const int lane = pk::lane_id(), m = lane & 15, g = lane >> 4;
  const int64_t tile = (int64_t)blockIdx.x * 4 + pk::wave_id();
  const int64_t T = (R + 15) >> 4;
  f32x4 v[8];
  const int64_t row = tile * 16 + m;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    v[q] = (tile < T && row < R) ? *reinterpret_cast<const f32x4*>(x + row * 128 + 16 * q + 4 * g)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
  if (MODE == 2) {  // 64 x 128 weight, float4 reads, row stride 132 in LDS
    f32x4 s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = threadIdx.x + 256 * i;
      s[i] = *reinterpret_cast<const f32x4*>(w + 4 * (int64_t)e);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = threadIdx.x + 256 * i, o = e >> 5, k4 = e & 31;
      *reinterpret_cast<f32x4*>(&Ws[o * 132 + 4 * k4]) = s[i];
    }
    __syncthreads();
  }
  if (tile >= T) return;
  // lane (m, g) holds x[row m][16 q + 4 g + i]; the probe's output: column c = 16 t + m (t < 4) of row
  // 4 g + r gets a value built from the lane's registers (no cross-lane exchange: same traffic)
  float wsum = MODE == 2 ? Ws[m * 132 + g] : 0.f;
  if (MODE == 3) {
    const int64_t pr = tile * 16 + m;
    if (pr < R) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f32x4 a = v[2 * t], b = v[2 * t + 1];
        *reinterpret_cast<f32x4*>(y + pr * 64 + 16 * t + 4 * g) = f32x4{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]};
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t pr = tile * 16 + 4 * g + r;
      if (pr < R) y[pr * 64 + 16 * t + m] = v[2 * t][r] + v[2 * t + 1][r] + wsum;
    }
}

// Clock probe for MFMA-bound kernels: every wave runs `iters` x CH independent accumulation
// chains of 8 v_mfma_f32_16x16x4f32 on operands derived from its lane (non-trivial bits), as
// the feature-distance pass does per tile; one store per lane at the end. Also stamps
// s_memtime / s_memrealtime around the loop (wave 0 of block 0) into stamp[0..3].
template <int CH>
__global__ __launch_bounds__(512, 2) void probe_mfma_kernel(const float* __restrict__ seed, int iters,
                                                            float* __restrict__ out, long long* __restrict__ stamp) {
  const int lane = threadIdx.x & 63;
  float a[8], b[CH][8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    a[s] = seed[(lane * 8 + s) & 1023];
#pragma unroll
    for (int c = 0; c < CH; ++c) b[c][s] = seed[(lane * 8 + s + 77 * c + 512) & 1023];
  }
  f32x4 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool stamper = blockIdx.x == 0 && threadIdx.x == 0;
  long long t0 = 0, r0 = 0;
  if (stamper) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int s = 0; s < 8; ++s) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[c][s], acc[c], 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 8; ++s) a[s] = acc[s & (CH - 1)][s & 3];  // next operands depend on this step
  }
  if (stamper) {
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    stamp[0] = t0; stamp[1] = t1; stamp[2] = r0; stamp[3] = r1;
  }
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) sum += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

// MFMA / VALU co-issue probe: like probe_mfma_kernel<2> (two accumulation chains of 8
// v_mfma_f32_16x16x4f32 per step, the feature-distance tile shape), plus NV independent integer
// VALU ops per 8 MFMAs (v_min_i32 on a state that does not feed the MFMAs, as the selection does).
// Two waves per SIMD (512-thread blocks, one per CU). Time vs NV tells whether VALU issue hides
// under the f32 MFMAs of the other wave / the same wave.
template <int NV>
__global__ __launch_bounds__(512, 1) void probe_mfma_valu_kernel(const float* __restrict__ seed, int iters,
                                                                 float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  float a[8], b[2][8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    a[s] = seed[(lane * 8 + s) & 1023];
#pragma unroll
    for (int c = 0; c < 2; ++c) b[c][s] = seed[(lane * 8 + s + 77 * c + 512) & 1023];
  }
  int z[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) z[k] = __float_as_int(seed[(lane + 9 * k) & 1023]);
  f32x4 acc[2];
  for (int it = 0; it < iters; ++it) {
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1] = acc[0];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[0][s], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[1][s], acc[1], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < NV / 4; ++v)  // NV per 8 MFMAs: NV / 8 per MFMA, in pairs
        asm volatile("v_min_i32_e32 %0, %1, %0" : "+v"(z[(s + v) & 7]) : "v"(z[(s + v + 3) & 7]));
    }
    // the selection-like consumer of the finished tile (keeps the MFMAs alive)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z[r] = min(z[r], __float_as_int(acc[0][r]));
      z[r + 4] = min(z[r + 4], __float_as_int(acc[1][r]));
    }
  }
  int sum = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) sum ^= z[k];
  out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = (float)sum;
}

// f32 MFMA accumulation-order probe: one wave per 16 x 16 tile, K = 32 in 8 chained
// v_mfma_f32_16x16x4f32 (slot (step s, lane group g) = k 4 s + g, the feature-distance layout),
// D[i][j] = sum_k A[i][k] B[k][j]; beside it each lane forms its 4 outputs (rows 4 g + r, column
// c) three ways: H1 one fmaf chain over k = 0..31 in order; H2 per instruction the 4 products
// exact (fp64) summed with the accumulator, one rounding to f32; H3 per instruction an fmaf
// chain of its 4 products from 0, then added to the accumulator. out [tiles][4][256]: MFMA, H1-H3.
__global__ __launch_bounds__(64) void probe_mfma_order_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                            float* __restrict__ out) {
  const int t = blockIdx.x, lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const float* At = A + (int64_t)t * 16 * 32;  // [16][32]
  const float* Bt = B + (int64_t)t * 32 * 16;  // [32][16]
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 8; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(At[c * 32 + 4 * s + g], Bt[(4 * s + g) * 16 + c], acc, 0, 0, 0);
  float* o = out + (int64_t)t * 4 * 256;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * g + r;
    float h1 = 0.f, h3 = 0.f;
    double h2d = 0.0;
    float h2 = 0.f;
    for (int s = 0; s < 8; ++s) {
      double p = 0.0;
      float h3i = 0.f;
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * s + q;
        const float a = At[i * 32 + k], b = Bt[k * 16 + c];
        h1 = fmaf(a, b, h1);
        p += (double)a * (double)b;
        h3i = fmaf(a, b, h3i);
      }
      h2 = (float)((double)h2 + p);
      h3 = h3 + h3i;
      (void)h2d;
    }
    o[0 * 256 + i * 16 + c] = acc[r];
    o[1 * 256 + i * 16 + c] = h1;
    o[2 * 256 + i * 16 + c] = h2;
    o[3 * 256 + i * 16 + c] = h3;
  }
}

}  // namespace

extern "C" int pkdev_probe_mfma_order(const float* A, const float* B, int tiles, float* out, void* stream) {
  if (tiles <= 0) return PK_ERR_ARG;
  hipLaunchKernelGGL(probe_mfma_order_kernel, dim3(tiles), dim3(64), 0, pk::as_stream(stream), A, B, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pkdev_probe_mfma_valu(const float* seed, int blocks, int iters, int nv, float* out, void* stream) {
  if (blocks <= 0 || iters <= 0) return PK_ERR_ARG;
  hipStream_t s = pk::as_stream(stream);
#define PK_PMV(N) hipLaunchKernelGGL(probe_mfma_valu_kernel<N>, dim3(blocks), dim3(512), 0, s, seed, iters, out)
  switch (nv) {
    case 0: PK_PMV(0); break;
    case 8: PK_PMV(8); break;
    case 16: PK_PMV(16); break;
    case 24: PK_PMV(24); break;
    case 32: PK_PMV(32); break;
    case 48: PK_PMV(48); break;
    case 64: PK_PMV(64); break;
    default: return PK_ERR_ARG;
  }
#undef PK_PMV
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pkdev_probe_mfma(const float* seed, int blocks, int iters, float* out, long long* stamp,
                                void* stream) {
  if (blocks <= 0 || iters <= 0) return PK_ERR_ARG;
  hipLaunchKernelGGL(probe_mfma_kernel<4>, dim3(blocks), dim3(512), 0, pk::as_stream(stream), seed, iters, out,
                     stamp);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pkdev_probe_linear(const float* x, const float* w, float* y, int64_t R, int mode, void* stream) {
  if (R <= 0 || mode < 0 || mode > 3) return PK_ERR_ARG;
  hipStream_t s = pk::as_stream(stream);
  if (mode == 0) {
    hipLaunchKernelGGL(probe_linear_kernel, dim3((unsigned)((R * 16 + 255) / 256)), dim3(256), 0, s, x, y, R);
  } else {
    const unsigned nb = (unsigned)(((R + 15) / 16 + 3) / 4);
    const size_t lds = mode == 2 ? sizeof(float) * 64 * 132 : 0;
    if (mode == 1) hipLaunchKernelGGL(probe_tile_kernel<1>, dim3(nb), dim3(256), lds, s, x, w, y, R);
    else if (mode == 2) hipLaunchKernelGGL(probe_tile_kernel<2>, dim3(nb), dim3(256), lds, s, x, w, y, R);
    else hipLaunchKernelGGL(probe_tile_kernel<3>, dim3(nb), dim3(256), lds, s, x, w, y, R);
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}
