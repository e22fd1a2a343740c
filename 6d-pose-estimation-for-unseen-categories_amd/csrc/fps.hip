// H3 — farthest-point sampling, one workgroup per crop.
//
// Reference: dataset/object.py:145-148 calls upstream DPFM
// `dpfm/utils.py::farthest_point_sample(xyz[3,N], ratio)` (restated in
// oracle/dpfm_oracle.py::farthest_point_sample). Per iteration i:
//   centroids[i] = farthest
//   dist = sum((xyz - xyz[farthest])**2, -1)          (fp32, ((dx²+dy²)+dz²))
//   distance[dist < distance] = dist                   (strict <)
//   farthest = max(distance, -1)[1]                    (first maximal index)
// The kernel is bit-exact against that recipe: every product and sum is rounded
// separately (TU compiled with -ffp-contract=off) and the argmax is a max over the
// 64-bit key (float_bits(distance) << 32 | ~index), so ties go to the lowest index.
//
// Layout: crops are packed back to back, xyz fp32 AoS [total, 3], crop b spans
// rows [offsets[b], offsets[b+1]). Each thread keeps PPT points (strided by the
// block size) and their running distances in registers; a structure-of-arrays copy
// of the crop sits in LDS so the current centroid is a broadcast read. One barrier
// per iteration (the per-wave maxima are double-buffered in LDS).
#include "common.hpp"

namespace {

constexpr int kFpsThreads = 1024;
constexpr int kFpsWaves = kFpsThreads / pk::kWave;
constexpr int kFpsMaxLds = 13312;  // points whose SoA copy fits in LDS (156 KiB)

template <int PPT, bool LDS>
__global__ __launch_bounds__(kFpsThreads) void fps_kernel(
    const float* __restrict__ xyz, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ start, const int32_t* __restrict__ npoint,
    int64_t* __restrict__ out, int out_stride) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t base = offsets[b];
  const int n = (int)(offsets[b + 1] - base);
  const int np = npoint[b];
  const float* __restrict__ p = xyz + base * 3;

  // slots[2][kFpsWaves] u64 first (16-B aligned), then SoA x/y/z.
  uint64_t* slots = reinterpret_cast<uint64_t*>(smem);
  float* sx = reinterpret_cast<float*>(smem + 2 * kFpsWaves * sizeof(uint64_t));
  const int n_pad = (n + 3) & ~3;
  float* sy = sx + n_pad;
  float* sz = sy + n_pad;

  float px[PPT], py[PPT], pz[PPT], pd[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int idx = tid + k * kFpsThreads;
    if (idx < n) {
      px[k] = p[3 * idx + 0];
      py[k] = p[3 * idx + 1];
      pz[k] = p[3 * idx + 2];
      pd[k] = 1e10f;
      if (LDS) {
        sx[idx] = px[k];
        sy[idx] = py[k];
        sz[idx] = pz[k];
      }
    } else {
      px[k] = py[k] = pz[k] = 0.f;
      pd[k] = -1.f;  // marks an empty slot
    }
  }
  if (n <= 0 || np <= 0) return;
  __syncthreads();

  int far = start[b];
  int64_t* __restrict__ o = out + (int64_t)b * out_stride;
  for (int i = 0; i < np; ++i) {
    if (tid == 0) o[i] = far;
    float cx, cy, cz;
    if (LDS) {
      cx = sx[far];
      cy = sy[far];
      cz = sz[far];
    } else {
      cx = p[3 * far + 0];
      cy = p[3 * far + 1];
      cz = p[3 * far + 2];
    }
    uint64_t best = 0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const float dx = px[k] - cx;
      const float dy = py[k] - cy;
      const float dz = pz[k] - cz;
      const float d = (dx * dx + dy * dy) + dz * dz;  // no contraction (TU flag)
      if (pd[k] >= 0.f) {
        pd[k] = d < pd[k] ? d : pd[k];
        const uint32_t idx = (uint32_t)(tid + k * kFpsThreads);
        const uint64_t key = ((uint64_t)pk::f32_bits(pd[k]) << 32) | (uint64_t)(~idx);
        best = key > best ? key : best;
      }
    }
    best = pk::wave_max_u64(best);
    uint64_t* s = slots + (i & 1) * kFpsWaves;
    if (pk::lane_id() == 0) s[pk::wave_id()] = best;
    __syncthreads();
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint64_t m = 0;
#pragma unroll
    for (int w = 0; w < kFpsWaves / 2; ++w) {
      const uint4 q = s4[w];
      const uint64_t a = ((uint64_t)q.y << 32) | q.x;
      const uint64_t c = ((uint64_t)q.w << 32) | q.z;
      m = a > m ? a : m;
      m = c > m ? c : m;
    }
    far = (int)(~(uint32_t)(m & 0xffffffffu));
  }
}

template <int PPT>
int launch_fps(const float* xyz, const int64_t* offsets, const int32_t* start,
               const int32_t* npoint, int64_t* out, int out_stride, int B, int nmax,
               hipStream_t s) {
  if (nmax <= kFpsMaxLds) {
    const int n_pad = (nmax + 3) & ~3;
    const size_t lds = 2 * kFpsWaves * sizeof(uint64_t) + 3 * (size_t)n_pad * sizeof(float);
    hipLaunchKernelGGL((fps_kernel<PPT, true>), dim3(B), dim3(kFpsThreads), lds, s, xyz,
                       offsets, start, npoint, out, out_stride);
  } else {
    const size_t lds = 2 * kFpsWaves * sizeof(uint64_t);
    hipLaunchKernelGGL((fps_kernel<PPT, false>), dim3(B), dim3(kFpsThreads), lds, s, xyz,
                       offsets, start, npoint, out, out_stride);
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}

}  // namespace

extern "C" int pk_fps(const float* xyz, const int64_t* offsets, int B, int nmax,
                      const int32_t* start, const int32_t* npoint, int64_t* out,
                      int out_stride, void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && out_stride >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(xyz && offsets && start && npoint && out);
  hipStream_t s = pk::as_stream(stream);
  const int ppt = (nmax + kFpsThreads - 1) / kFpsThreads;
  if (ppt <= 1) return launch_fps<1>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (ppt <= 2) return launch_fps<2>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (ppt <= 4) return launch_fps<4>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (ppt <= 8) return launch_fps<8>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (ppt <= 13) return launch_fps<13>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (ppt <= 32) return launch_fps<32>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  return PK_ERR_ARG;  // > 32768 points per crop
}
