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


// Channels-first [C, N] items (item b from src0 + b sb for b < B0, else src1 + (b - B0) sb) into
// one rows-layout [B, N, C] buffer: the refinement's first_lin backward turns the two shapes'
// channels-first d desc (modeling/dpfm.py:98 `.transpose(1, 2)`) into the rows-layout gradient
// of the encoder features. Block = 64 points x C channels of one item through LDS (row stride
// C + 1: conflict-free both ways); loads coalesced along n, stores along c.
template <int C>
__global__ __launch_bounds__(256) void transpose_cf_rows_kernel(const float* __restrict__ src0,
                                                                const float* __restrict__ src1, int B0, int N,
                                                                int64_t sb, float* __restrict__ dst) {
  __shared__ float t[64 * (C + 1)];
  const int b = blockIdx.y, n0 = blockIdx.x * 64;
  const float* src = (b < B0 ? src0 + (int64_t)b * sb : src1 + (int64_t)(b - B0) * sb);
  const int np = min(64, N - n0);
  for (int e = threadIdx.x; e < 64 * C; e += 256) {
    const int c = e >> 6, n = e & 63;
    if (n < np) t[n * (C + 1) + c] = src[(int64_t)c * N + n0 + n];
  }
  __syncthreads();
  float* d = dst + ((int64_t)b * N + n0) * C;
  for (int e = threadIdx.x; e < np * C; e += 256) {
    const int n = e / C, c = e - n * C;
    d[e] = t[n * (C + 1) + c];
  }
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

extern "C" int pk_transpose_cf_rows(const float* src0, const float* src1, int B0, int B, int C, int N, int64_t sb,
                                    float* dst, void* stream) {
  PK_REQUIRE(B >= 0 && B0 >= 0 && B0 <= B && N >= 0 && (C == 16 || C == 32 || C == 64 || C == 128) && sb >= (int64_t)C * N);
  if (B == 0 || N == 0) return PK_OK;
  PK_REQUIRE(dst != nullptr && (B0 == 0 || src0 != nullptr) && (B0 == B || src1 != nullptr) && B <= 65535);
  hipStream_t s = pk::as_stream(stream);
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)B);
  switch (C) {
    case 16: hipLaunchKernelGGL(transpose_cf_rows_kernel<16>, grid, dim3(256), 0, s, src0, src1, B0, N, sb, dst); break;
    case 32: hipLaunchKernelGGL(transpose_cf_rows_kernel<32>, grid, dim3(256), 0, s, src0, src1, B0, N, sb, dst); break;
    case 64: hipLaunchKernelGGL(transpose_cf_rows_kernel<64>, grid, dim3(256), 0, s, src0, src1, B0, N, sb, dst); break;
    default: hipLaunchKernelGGL(transpose_cf_rows_kernel<128>, grid, dim3(256), 0, s, src0, src1, B0, N, sb, dst); break;
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}
