// Strided block copy: rows blocks of n floats from src (block stride ld_src) to dst (ld_dst).
// The fused AttentionalPropagation node (dpfm_amd/attnprop.py) forms the concatenation
// torch.cat([x, message], dim=1) of reference modeling/dpfm.py:67 in one [B, 2C, N] buffer: the
// merge layer writes the message half in its epilogue, this kernel the x half (B blocks of C N
// floats, block stride 2 C N). Lane-linear 16-B loads and stores, 4 float4 per thread in
// flight; a scalar path when a pointer, n or a stride is not a multiple of 4 floats.
#include <algorithm>

#include "common.hpp"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kPer = 4;  // float4s per thread

__global__ __launch_bounds__(256) void copy_rows_v4_kernel(float* __restrict__ dst, int64_t ld_dst,
                                                           const float* __restrict__ src, int64_t ld_src,
                                                           int64_t n4) {
  const int64_t row = blockIdx.y;
  const int64_t base = (int64_t)blockIdx.x * 256 * kPer + threadIdx.x;
  const f32x4* s = reinterpret_cast<const f32x4*>(src + row * ld_src);
  f32x4* d = reinterpret_cast<f32x4*>(dst + row * ld_dst);
  f32x4 v[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int64_t e = base + 256 * i;
    v[i] = s[e < n4 ? e : n4 - 1];  // clamped: every load issued before the first store
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int64_t e = base + 256 * i;
    if (e < n4) d[e] = v[i];
  }
}

__global__ __launch_bounds__(256) void copy_rows_kernel(float* __restrict__ dst, int64_t ld_dst,
                                                        const float* __restrict__ src, int64_t ld_src, int64_t n) {
  const int64_t row = blockIdx.y;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    dst[row * ld_dst + e] = src[row * ld_src + e];
}

}  // namespace

extern "C" int pk_copy_rows(float* dst, int64_t ld_dst, const float* src, int64_t ld_src, int64_t rows, int64_t n,
                            void* stream) {
  PK_REQUIRE(rows >= 0 && n >= 0 && ld_dst >= n && ld_src >= n && rows <= 65535);
  if (rows == 0 || n == 0) return PK_OK;
  PK_REQUIRE(dst != nullptr && src != nullptr);
  hipStream_t s = pk::as_stream(stream);
  const bool v4 = (n % 4 == 0) && (ld_dst % 4 == 0) && (ld_src % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(dst) % 16 == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0);
  if (v4) {
    const int64_t n4 = n / 4;
    const dim3 grid((unsigned)((n4 + 256 * kPer - 1) / (256 * kPer)), (unsigned)rows);
    hipLaunchKernelGGL(copy_rows_v4_kernel, grid, dim3(256), 0, s, dst, ld_dst, src, ld_src, n4);
  } else {
    const dim3 grid((unsigned)std::min<int64_t>((n + 255) / 256, 1024), (unsigned)rows);
    hipLaunchKernelGGL(copy_rows_kernel, grid, dim3(256), 0, s, dst, ld_dst, src, ld_src, n);
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}
