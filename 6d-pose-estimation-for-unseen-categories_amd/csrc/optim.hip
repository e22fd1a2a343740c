// H15 optimizer tail of the training step (scripts/train.py:121-124):
//   torch.nn.utils.clip_grad_norm_(params, max_norm=5.0)      (L2 over every gradient)
//   RMSprop(lr=5e-4).step()   (config/dpfm_orig.gin:62-63; alpha 0.99, eps 1e-8, no momentum,
//                              not centered, no weight decay)
// in two launches. torch runs ~20 kernels here (per-tensor norms, their norm, the clip
// multiply, then the foreach RMSprop chain over ~60 small tensors); here the tensors are one
// flattened index space (pointer table with prefix offsets, passed by value), 64 chunks:
// pass 1 writes each chunk's sum of g^2, pass 2 (every block) adds the 64 partials in a
// fixed order and updates its chunk:
//   total = sqrt(sum over tensors of sum g^2)     (fixed order: deterministic)
//   coef  = min(max_norm / (total + 1e-6), 1)      (clip_grad_norm_'s clamped coefficient)
//   g    *= coef                                   (clip_grad_norm_ writes the grads back)
//   sq    = sq * alpha + ((1 - alpha) * g) * g     (addcmul_, value = 1 - alpha)
//   p     = p + (-lr) * (g / (sqrt(sq) + eps))     (addcdiv_)
//   step += 1                                      (the optimizer's per-parameter counter)
// Products and sums rounded separately as ATen's kernels do (TU built -ffp-contract=off).
#include "common.hpp"

namespace {

constexpr int kMaxTensors = 96;
constexpr int kThreads = 256;
constexpr int kBlocks = 64;  // chunks of the flattened parameter space (one partial norm each)

struct OptTable {
  int n;
  int64_t total;
  float* p[kMaxTensors];
  float* g[kMaxTensors];
  float* sq[kMaxTensors];
  float* step[kMaxTensors];
  int64_t off[kMaxTensors + 1];  // prefix offsets of the flattened parameter space
};

__device__ __forceinline__ int tensor_of(const OptTable& t, int64_t e) {
  int lo = 0, hi = t.n - 1;  // last k with off[k] <= e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = pk::wave_sum_f32(v);
  if (pk::lane_id() == 0) red[pk::wave_id()] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  return s;
}

// pass 1: partial sums of g^2 over chunk b of the flattened gradients
__global__ __launch_bounds__(kThreads) void grad_sumsq_kernel(const OptTable t, float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  const int64_t chunk = (t.total + kBlocks - 1) / kBlocks;
  const int64_t e0 = blockIdx.x * chunk, e1 = e0 + chunk < t.total ? e0 + chunk : t.total;
  float acc = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
    const int k = tensor_of(t, e);
    const float g = t.g[k][e - t.off[k]];
    acc += g * g;
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// pass 2: every block forms the same total from the partials (fixed order), then clips and
// applies RMSprop to its chunk
__global__ __launch_bounds__(kThreads) void clip_rmsprop_kernel(const OptTable t, const float* __restrict__ part,
                                                                float max_norm, float lr, float alpha,
                                                                float one_minus_alpha, float eps,
                                                                float* __restrict__ norm_out) {
  float s = 0.f;
  for (int q = 0; q < kBlocks; ++q) s += part[q];  // uniform: identical in every thread and block
  const float total = sqrtf(s);
  const float c = max_norm / (total + 1e-6f);
  const float coef = c < 1.f ? c : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) *norm_out = total;
  const int64_t chunk = (t.total + kBlocks - 1) / kBlocks;
  const int64_t e0 = blockIdx.x * chunk, e1 = e0 + chunk < t.total ? e0 + chunk : t.total;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
    const int k = tensor_of(t, e);
    const int64_t i = e - t.off[k];
    const float gc = t.g[k][i] * coef;
    t.g[k][i] = gc;
    const float sq = t.sq[k][i] * alpha + (one_minus_alpha * gc) * gc;
    t.sq[k][i] = sq;
    const float avg = sqrtf(sq) + eps;
    t.p[k][i] = t.p[k][i] + (-lr) * (gc / avg);
  }
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < t.n; k += kThreads)
      if (t.step[k]) t.step[k][0] = t.step[k][0] + 1.f;
  }
}

}  // namespace

extern "C" int pk_clip_rmsprop(float* const* params, float* const* grads, float* const* square_avg,
                               float* const* steps, const int64_t* numel, int n, float max_norm, float lr,
                               float alpha, float one_minus_alpha, float eps, float* work, float* norm_out,
                               void* stream) {
  PK_REQUIRE(n >= 0 && n <= kMaxTensors);
  if (n == 0) return PK_OK;
  PK_REQUIRE(params && grads && square_avg && numel);
  OptTable t{};
  t.n = n;
  int64_t o = 0;
  for (int k = 0; k < n; ++k) {
    PK_REQUIRE(params[k] && grads[k] && square_avg[k] && numel[k] >= 0);
    t.p[k] = params[k];
    t.g[k] = grads[k];
    t.sq[k] = square_avg[k];
    t.step[k] = steps ? steps[k] : nullptr;
    t.off[k] = o;
    o += numel[k];
  }
  t.off[n] = o;
  t.total = o;
  PK_REQUIRE(work != nullptr);
  hipStream_t s = pk::as_stream(stream);
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(kBlocks), dim3(kThreads), 0, s, t, work);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(clip_rmsprop_kernel, dim3(kBlocks), dim3(kThreads), 0, s, t, work, max_norm, lr, alpha,
                     one_minus_alpha, eps, norm_out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
