// H8 refinement MLP's InstanceNorm1d(C) + ReLU (modeling/dpfm.py:16-26: Conv1d -> InstanceNorm1d
// (affine=False, eps 1e-5, statistics over all N points of a crop, padding included) -> ReLU),
// forward and backward fused: one wave per (crop, channel) row of the channels-first
// [B, C, N] activation. torch runs batch_norm_collect_statistics + transform + threshold
// forward and threshold_backward + batch_norm_backward (+ its reductions) backward.
//   forward   mean = sum x / N, var = sum (x - mean)^2 / N (biased, two passes over the row
//             held in registers), invstd = 1 / sqrt(var + eps), y = max((x - mean) invstd, 0)
//   backward  g = dy [xhat > 0], dx = invstd (g - mean(g) - xhat mean(g xhat))
#include "common.hpp"

namespace {

constexpr int kMaxPerLane = 32;  // N <= 2048 held in registers (64 lanes x 32)

template <int PER>
__global__ __launch_bounds__(256) void instnorm_relu_fwd_kernel(const float* __restrict__ x, int64_t rows, int N,
                                                                float eps, float* __restrict__ y,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ invstd_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + pk::wave_id();
  if (r >= rows) return;
  const int lane = pk::lane_id();
  const float* __restrict__ xr = x + r * N;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int n = lane + 64 * k;
    v[k] = n < N ? xr[n] : 0.f;
    s += v[k];
  }
  const float mean = pk::wave_sum_f32(s) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int n = lane + 64 * k;
    const float d = v[k] - mean;
    q += n < N ? d * d : 0.f;
  }
  const float var = pk::wave_sum_f32(q) / (float)N;
  const float invstd = 1.f / sqrtf(var + eps);
  float* __restrict__ yr = y + r * N;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int n = lane + 64 * k;
    if (n < N) yr[n] = fmaxf((v[k] - mean) * invstd, 0.f);
  }
  if (lane == 0) {
    mean_out[r] = mean;
    invstd_out[r] = invstd;
  }
}

template <int PER>
__global__ __launch_bounds__(256) void instnorm_relu_bwd_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ dy,
                                                                const float* __restrict__ mean_in,
                                                                const float* __restrict__ invstd_in, int64_t rows,
                                                                int N, float* __restrict__ dx) {
  const int64_t r = (int64_t)blockIdx.x * 4 + pk::wave_id();
  if (r >= rows) return;
  const int lane = pk::lane_id();
  const float mean = mean_in[r], invstd = invstd_in[r];
  const float* __restrict__ xr = x + r * N;
  const float* __restrict__ gr = dy + r * N;
  float xh[PER], g[PER];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int n = lane + 64 * k;
    const float xv = n < N ? xr[n] : 0.f;
    const float gv = n < N ? gr[n] : 0.f;
    xh[k] = (xv - mean) * invstd;
    g[k] = xh[k] > 0.f ? gv : 0.f;  // ReLU backward on the normalized value (= the output)
    sg += g[k];
    sgx += g[k] * xh[k];
  }
  const float mg = pk::wave_sum_f32(sg) / (float)N;
  const float mgx = pk::wave_sum_f32(sgx) / (float)N;
  float* __restrict__ dr = dx + r * N;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int n = lane + 64 * k;
    if (n < N) dr[n] = invstd * ((g[k] - mg) - xh[k] * mgx);
  }
}

// rows longer than the register tile (N > 2048, e.g. 4096-point crops): the same arithmetic
// re-reading the row from memory (L2-resident) for each pass
__global__ __launch_bounds__(256) void instnorm_relu_fwd_long_kernel(const float* __restrict__ x, int64_t rows, int N,
                                                                     float eps, float* __restrict__ y,
                                                                     float* __restrict__ mean_out,
                                                                     float* __restrict__ invstd_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + pk::wave_id();
  if (r >= rows) return;
  const int lane = pk::lane_id();
  const float* __restrict__ xr = x + r * N;
  float s = 0.f;
  for (int n = lane; n < N; n += 64) s += xr[n];
  const float mean = pk::wave_sum_f32(s) / (float)N;
  float q = 0.f;
  for (int n = lane; n < N; n += 64) {
    const float d = xr[n] - mean;
    q += d * d;
  }
  const float invstd = 1.f / sqrtf(pk::wave_sum_f32(q) / (float)N + eps);
  for (int n = lane; n < N; n += 64) y[r * N + n] = fmaxf((xr[n] - mean) * invstd, 0.f);
  if (lane == 0) {
    mean_out[r] = mean;
    invstd_out[r] = invstd;
  }
}

__global__ __launch_bounds__(256) void instnorm_relu_bwd_long_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ dy,
                                                                     const float* __restrict__ mean_in,
                                                                     const float* __restrict__ invstd_in,
                                                                     int64_t rows, int N, float* __restrict__ dx) {
  const int64_t r = (int64_t)blockIdx.x * 4 + pk::wave_id();
  if (r >= rows) return;
  const int lane = pk::lane_id();
  const float mean = mean_in[r], invstd = invstd_in[r];
  const float* __restrict__ xr = x + r * N;
  const float* __restrict__ gr = dy + r * N;
  float sg = 0.f, sgx = 0.f;
  for (int n = lane; n < N; n += 64) {
    const float xh = (xr[n] - mean) * invstd;
    const float g = xh > 0.f ? gr[n] : 0.f;
    sg += g;
    sgx += g * xh;
  }
  const float mg = pk::wave_sum_f32(sg) / (float)N, mgx = pk::wave_sum_f32(sgx) / (float)N;
  for (int n = lane; n < N; n += 64) {
    const float xh = (xr[n] - mean) * invstd;
    const float g = xh > 0.f ? gr[n] : 0.f;
    dx[r * N + n] = invstd * ((g - mg) - xh * mgx);
  }
}

}  // namespace

extern "C" int pk_instnorm_relu_fwd(const float* x, int64_t rows, int N, float eps, float* y, float* mean,
                                    float* invstd, void* stream) {
  PK_REQUIRE(rows >= 0 && N > 0);
  if (rows == 0) return PK_OK;
  PK_REQUIRE(x && y && mean && invstd);
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = pk::as_stream(stream);
  if (N <= 512) hipLaunchKernelGGL(instnorm_relu_fwd_kernel<8>, grid, dim3(256), 0, s, x, rows, N, eps, y, mean, invstd);
  else if (N <= 1024) hipLaunchKernelGGL(instnorm_relu_fwd_kernel<16>, grid, dim3(256), 0, s, x, rows, N, eps, y, mean, invstd);
  else if (N <= 2048) hipLaunchKernelGGL(instnorm_relu_fwd_kernel<32>, grid, dim3(256), 0, s, x, rows, N, eps, y, mean, invstd);
  else hipLaunchKernelGGL(instnorm_relu_fwd_long_kernel, grid, dim3(256), 0, s, x, rows, N, eps, y, mean, invstd);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_instnorm_relu_bwd(const float* x, const float* dy, const float* mean, const float* invstd,
                                    int64_t rows, int N, float* dx, void* stream) {
  PK_REQUIRE(rows >= 0 && N > 0);
  if (rows == 0) return PK_OK;
  PK_REQUIRE(x && dy && mean && invstd && dx);
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = pk::as_stream(stream);
  if (N <= 512) hipLaunchKernelGGL(instnorm_relu_bwd_kernel<8>, grid, dim3(256), 0, s, x, dy, mean, invstd, rows, N, dx);
  else if (N <= 1024) hipLaunchKernelGGL(instnorm_relu_bwd_kernel<16>, grid, dim3(256), 0, s, x, dy, mean, invstd, rows, N, dx);
  else if (N <= 2048) hipLaunchKernelGGL(instnorm_relu_bwd_kernel<32>, grid, dim3(256), 0, s, x, dy, mean, invstd, rows, N, dx);
  else hipLaunchKernelGGL(instnorm_relu_bwd_long_kernel, grid, dim3(256), 0, s, x, dy, mean, invstd, rows, N, dx);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// ---------------------------------------------------------------------------------
// H15 overlap term: upstream DPFM WeightedBCELoss per crop (restated in oracle/
// dpfm_model_oracle.py::weighted_bce; called from utils/loss.py:79-83), loss and gradient
// in one pass, one workgroup per (crop, tensor):
//   wn = sum_n t_n / N;  w_n = t_n >= 0.5 ? 1 - wn : wn
//   bce_n = (t_n - 1) max(log1p(-p_n), -100) - t_n max(log p_n, -100)   (ATen's formula)
//   loss = sum_n w_n bce_n / N;  dloss/dp_n = w_n (p_n - t_n) / max(p_n (1 - p_n), 1e-12) / N
// Sums in a fixed order (deterministic).
namespace {

constexpr int kBceThreads = 256;

__device__ __forceinline__ float block_sum_f32(float v, float* red) {
  v = pk::wave_sum_f32(v);
  __syncthreads();
  if (pk::lane_id() == 0) red[pk::wave_id()] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kBceThreads / 64; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(kBceThreads) void wbce_kernel(const float* __restrict__ p0, const int8_t* __restrict__ t0,
                                                           int N0, const float* __restrict__ p1,
                                                           const int8_t* __restrict__ t1, int N1, int B,
                                                           float* __restrict__ loss, float* __restrict__ g0,
                                                           float* __restrict__ g1) {
  __shared__ float red[kBceThreads / 64];
  const int b = blockIdx.x % B, which = blockIdx.x / B;
  const int N = which ? N1 : N0;
  const float* __restrict__ p = (which ? p1 : p0) + (int64_t)b * N;
  const int8_t* __restrict__ t = (which ? t1 : t0) + (int64_t)b * N;
  float* __restrict__ g = g0 ? (which ? g1 : g0) + (int64_t)b * N : nullptr;
  float st = 0.f;
  for (int n = threadIdx.x; n < N; n += kBceThreads) st += (float)t[n];
  const float wn = block_sum_f32(st, red) / (float)N;
  float sl = 0.f;
  const float invN = 1.f / (float)N;
  for (int n = threadIdx.x; n < N; n += kBceThreads) {
    const float pv = p[n], tv = (float)t[n];
    const float w = tv >= 0.5f ? 1.f - wn : wn;
    const float l = (tv - 1.f) * fmaxf(log1pf(-pv), -100.f) - tv * fmaxf(logf(pv), -100.f);
    sl += w * l;
    if (g) g[n] = w * invN * ((pv - tv) / fmaxf((1.f - pv) * pv, 1e-12f));
  }
  const float s = block_sum_f32(sl, red);
  if (threadIdx.x == 0) loss[which * B + b] = s * invN;
}

}  // namespace

extern "C" int pk_wbce(const float* p12, const int8_t* t12, int N1, const float* p21, const int8_t* t21, int N2,
                       int B, float* loss, float* g12, float* g21, void* stream) {
  PK_REQUIRE(B >= 0 && N1 > 0 && N2 > 0 && (g12 == nullptr) == (g21 == nullptr));
  if (B == 0) return PK_OK;
  PK_REQUIRE(p12 && t12 && p21 && t21 && loss);
  hipLaunchKernelGGL(wbce_kernel, dim3(2 * B), dim3(kBceThreads), 0, pk::as_stream(stream), p12, t12, N1, p21, t21,
                     N2, B, loss, g12, g21);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// ---------------------------------------------------------------------------------
// F.normalize(x, p=2, dim=-1, eps=1e-12) over the channel dim of [B, N, C] features stored
// rows or channels-first (the overlap head's input, modeling/dpfm.py:140-145), forward and
// backward: one thread per point, element (b, n, c) at b * sb + n * sn + c * sc (the output
// and gradients use the same strides as the input).
//   y = x / max(||x||, eps);  dx = (dy - y (y . dy)) / ||x||  (dy / eps where clamped)
namespace {

struct L2View {
  int64_t sb, sn, sc;
};

template <int CC>  // CC > 0: compile-time channel count (all loads in flight); 0: runtime C
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* __restrict__ x, L2View v, int B, int N, int C,
                                                         float* __restrict__ y, float* __restrict__ nrm,
                                                         float* __restrict__ y_rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * N) return;
  const int Cn = CC > 0 ? CC : C;
  const int64_t b = i / N, n = i - b * N;
  const int64_t o = b * v.sb + n * v.sn;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < Cn; ++c) {
    const float a = x[o + c * v.sc];
    s += a * a;
  }
  const float nr = sqrtf(s);
  const float d = fmaxf(nr, 1e-12f);
#pragma unroll
  for (int c = 0; c < Cn; ++c) {
    const float q = x[o + c * v.sc] / d;
    y[o + c * v.sc] = q;
    if (y_rows) y_rows[i * Cn + c] = q;  // the same values, rows layout [B, N, C]
  }
  nrm[i] = nr;
}

template <int CC>
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                                         const float* __restrict__ dy_rows,
                                                         const float* __restrict__ nrm, L2View v, int B, int N, int C,
                                                         float* __restrict__ dx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * N) return;
  const int Cn = CC > 0 ? CC : C;
  const int64_t b = i / N, n = i - b * N;
  const int64_t o = b * v.sb + n * v.sn;
  const float nr = nrm[i];
  // the incoming gradient: dy (x's layout) + dy_rows (rows layout), either may be absent
  auto grad = [&](int c) {
    float g = dy ? dy[o + c * v.sc] : 0.f;
    if (dy_rows) g += dy_rows[i * Cn + c];
    return g;
  };
  float yd = 0.f;
#pragma unroll
  for (int c = 0; c < Cn; ++c) yd += y[o + c * v.sc] * grad(c);
  const bool clamped = !(nr > 1e-12f);
#pragma unroll
  for (int c = 0; c < Cn; ++c) {
    const float g = grad(c);
    dx[o + c * v.sc] = clamped ? g / 1e-12f : (g - y[o + c * v.sc] * yd) / nr;
  }
}

}  // namespace

extern "C" int pk_l2_normalize_fwd(const float* x, const int64_t* strides, int B, int N, int C, float* y, float* nrm,
                                   float* y_rows, void* stream) {
  PK_REQUIRE(B >= 0 && N >= 0 && C > 0 && strides);
  if ((int64_t)B * N == 0) return PK_OK;
  PK_REQUIRE(x && y && nrm);
  const L2View v{strides[0], strides[1], strides[2]};
  const dim3 grid((unsigned)(((int64_t)B * N + 255) / 256));
  if (C == 32)
    hipLaunchKernelGGL(l2norm_fwd_kernel<32>, grid, dim3(256), 0, pk::as_stream(stream), x, v, B, N, C, y, nrm, y_rows);
  else
    hipLaunchKernelGGL(l2norm_fwd_kernel<0>, grid, dim3(256), 0, pk::as_stream(stream), x, v, B, N, C, y, nrm, y_rows);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_l2_normalize_bwd(const float* y, const float* dy, const float* nrm, const int64_t* strides, int B,
                                   int N, int C, float* dx, const float* dy_rows, void* stream) {
  PK_REQUIRE(B >= 0 && N >= 0 && C > 0 && strides);
  if ((int64_t)B * N == 0) return PK_OK;
  PK_REQUIRE(y && (dy || dy_rows) && nrm && dx);
  const L2View v{strides[0], strides[1], strides[2]};
  const dim3 grid((unsigned)(((int64_t)B * N + 255) / 256));
  if (C == 32)
    hipLaunchKernelGGL(l2norm_bwd_kernel<32>, grid, dim3(256), 0, pk::as_stream(stream), y, dy, dy_rows, nrm, v, B, N,
                       C, dx);
  else
    hipLaunchKernelGGL(l2norm_bwd_kernel<0>, grid, dim3(256), 0, pk::as_stream(stream), y, dy, dy_rows, nrm, v, B, N,
                       C, dx);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// models/dpfm.py:53 + :61-66 (the shared encoder pass): features = cat((v1 - 110) / 50,
// (v2 - 110) / 50) in one launch. `mul` is the host-rounded reciprocal: torch evaluates a
// division by a Python scalar on the GPU as a product with the f32 reciprocal, so this is
// the same rounding as the reference's two elementwise kernels and the concatenation copy.
namespace {
__global__ __launch_bounds__(256) void affine_cat_kernel(const float* __restrict__ a, int64_t na,
                                                         const float* __restrict__ b, int64_t nb, float sub,
                                                         float mul, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < na) out[i] = (a[i] - sub) * mul;
  else if (i < na + nb) out[i] = (b[i - na] - sub) * mul;
}
}  // namespace

extern "C" int pk_affine_cat(const float* a, int64_t na, const float* b, int64_t nb, float sub, float mul, float* out,
                             void* stream) {
  PK_REQUIRE(na >= 0 && nb >= 0);
  if (na + nb == 0) return PK_OK;
  PK_REQUIRE(out && (na == 0 || a) && (nb == 0 || b));
  hipLaunchKernelGGL(affine_cat_kernel, dim3((unsigned)((na + nb + 255) / 256)), dim3(256), 0, pk::as_stream(stream),
                     a, na, b, nb, sub, mul, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
