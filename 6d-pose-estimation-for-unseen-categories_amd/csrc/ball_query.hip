// H5 — ball query ("find_positives") and overlap masks.
//
// Reference: dataset/object.py:281-288
//     distances = np.linalg.norm(pc1[:, np.newaxis] - pc2, axis=2)   # fp64
//     mask = distances <= r
//     return np.argwhere(mask)                                       # row-major (i, j)
// and dataset/object.py:311-317 `get_overlap` (int8 "has a partner" masks).
//
// Exactness: numpy evaluates s = ((dx*dx + dy*dy) + dz*dz) in fp64 with every
// operation rounded, then sqrt_rn(s) <= r. sqrt_rn is monotone, so that test equals
// s <= T(r) with T(r) = the largest double whose correctly rounded sqrt is <= r.
// The host computes T(r) once per crop (dpfm_amd/ops.py::ball_threshold); the kernel
// never calls sqrt. With -ffp-contract=off the fp64 sums are rounded exactly as
// numpy rounds them, so the mask and the pair list are bit-exact.
//
// Three launches, all stream-ordered, no host sync:
//   1. pk_ball_query_mask : dense uint8 mask [B, n1max, ld] (the reference's `mask`)
//                           + per-row partner counts (HBM-write bound).
//   2. scan               : exclusive prefix sum of the row counts per crop.
//   3. compaction         : ordered pair list (i, j) int64 [B, cap, 2] + overlaps.
// pk_ball_query_pairs chains 2 and 3 after 1 (or recomputes distances if no mask).
#include "common.hpp"

namespace {

constexpr int kColsPerLane = 16;                    // 16 mask bytes = one 16-B store
constexpr int kColsPerWave = kColsPerLane * pk::kWave;  // 1024 columns per wave
constexpr int kRowsPerWave = 16;
constexpr int kBqThreads = 256;
constexpr int kRowsPerBlock = kRowsPerWave * (kBqThreads / pk::kWave);  // 64

__device__ __forceinline__ bool within(double ax, double ay, double az, double bx, double by,
                                       double bz, double thr2) {
  const double dx = ax - bx;
  const double dy = ay - by;
  const double dz = az - bz;
  const double s = (dx * dx + dy * dy) + dz * dz;  // rounded like numpy (no FMA)
  return s <= thr2;
}

// grid: (ceil(n2max / 1024), ceil(n1max / 64), B); block 256 = 4 waves.
// A lane owns 16 consecutive columns (their pc coords stay in registers) and walks
// 16 rows; each row produces one 16-byte store.
__global__ __launch_bounds__(kBqThreads) void bq_mask_kernel(
    const double* __restrict__ cad, const int64_t* __restrict__ cad_off,
    const double* __restrict__ pc, const int64_t* __restrict__ pc_off,
    const double* __restrict__ thr2v, int n1max, int ld, uint8_t* __restrict__ mask,
    int32_t* __restrict__ rowcount) {
  const int b = blockIdx.z;
  const int64_t c0 = cad_off[b], p0 = pc_off[b];
  const int n1 = (int)(cad_off[b + 1] - c0);
  const int n2 = (int)(pc_off[b + 1] - p0);
  const double thr2 = thr2v[b];
  const int lane = pk::lane_id();
  const int j0 = blockIdx.x * kColsPerWave + lane * kColsPerLane;
  const int row0 = blockIdx.y * kRowsPerBlock + pk::wave_id() * kRowsPerWave;
  if (row0 >= n1max) return;

  double qx[kColsPerLane], qy[kColsPerLane], qz[kColsPerLane];
#pragma unroll
  for (int c = 0; c < kColsPerLane; ++c) {
    const int j = j0 + c;
    if (j < n2) {
      const double* q = pc + (p0 + j) * 3;
      qx[c] = q[0];
      qy[c] = q[1];
      qz[c] = q[2];
    } else {
      qx[c] = qy[c] = qz[c] = __builtin_huge_val();  // never within (inf - x = inf)
    }
  }

  for (int r = 0; r < kRowsPerWave; ++r) {
    const int i = row0 + r;
    if (i >= n1max) break;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    int cnt = 0;
    if (i < n1) {
      const double* a = cad + (c0 + i) * 3;
      const double ax = a[0], ay = a[1], az = a[2];
#pragma unroll
      for (int c = 0; c < kColsPerLane; ++c) {
        const bool in = within(ax, ay, az, qx[c], qy[c], qz[c], thr2);
        w[c >> 2] |= (in ? 1u : 0u) << ((c & 3) * 8);
        cnt += in ? 1 : 0;
      }
    }
    if (mask != nullptr && j0 < ld) {
      uint4* dst = reinterpret_cast<uint4*>(mask + ((int64_t)b * n1max + i) * ld + j0);
      *dst = make_uint4(w[0], w[1], w[2], w[3]);
    }
    cnt = pk::wave_sum_i32(cnt);
    if (lane == 0 && cnt != 0) atomicAdd(rowcount + (int64_t)b * n1max + i, cnt);
  }
}

// fp32-screened variant (the default). Coordinates are centred on the crop's first CAD
// point in fp64 and rounded to fp32 once per point. Each pair's squared distance is
// evaluated in fp32 by the expansion s32 = (|a|² + |b|²) - 2 a·b (one add + three FMAs
// with -2b and |b|² precomputed per column) and classified against
// [thr2 - margin, thr2 + margin]; only pairs inside that band are recomputed with the
// exact fp64 recipe, so the mask stays bit-exact. `margin` bounds |s32 - s64| for any
// pair that can land on either side of thr2 (DESIGN.md §Ball query has the derivation).
//
// grid (ceil(n1max / 64), B), block 256 = 4 waves; a wave owns 16 CAD rows and walks
// every 1024-column chunk of the crop (lane = 16 consecutive columns, one 16-B store
// per row and chunk), so row counts are complete per wave: plain stores, no atomics.
__global__ __launch_bounds__(kBqThreads) void bq_mask_f32_kernel(
    const double* __restrict__ cad, const int64_t* __restrict__ cad_off,
    const double* __restrict__ pc, const int64_t* __restrict__ pc_off,
    const double* __restrict__ thr2v, int n1max, int ld, uint8_t* __restrict__ mask,
    int32_t* __restrict__ rowcount) {
  const int b = blockIdx.y;
  const int64_t c0 = cad_off[b], p0 = pc_off[b];
  const int n1 = (int)(cad_off[b + 1] - c0);
  const int n2 = (int)(pc_off[b + 1] - p0);
  const double thr2 = thr2v[b];
  const int lane = pk::lane_id();
  const int row0 = __builtin_amdgcn_readfirstlane(blockIdx.x * kRowsPerBlock + pk::wave_id() * kRowsPerWave);
  if (row0 >= n1max) return;
  const double ox = n1 > 0 ? cad[c0 * 3 + 0] : 0.0;
  const double oy = n1 > 0 ? cad[c0 * 3 + 1] : 0.0;
  const double oz = n1 > 0 ? cad[c0 * 3 + 2] : 0.0;
  const float u = 5.9604645e-8f;  // 2^-24
  const float thr2f = (float)thr2;
  const float R = sqrtf(thr2f) * 1.001f;
  const int ncols = mask != nullptr ? ld : n2;

  __shared__ int cnt_s[kBqThreads / pk::kWave][kRowsPerWave];  // per-wave row totals
  int* cnt = cnt_s[pk::wave_id()];
  if (lane < kRowsPerWave) cnt[lane] = 0;

  for (int jc = 0; jc < ncols; jc += kColsPerWave) {
    const int j0 = jc + lane * kColsPerLane;
    float mx[kColsPerLane], my[kColsPerLane], mz[kColsPerLane], b2[kColsPerLane];
    float bm = 0.f;
#pragma unroll
    for (int c = 0; c < kColsPerLane; ++c) {
      const int j = j0 + c;
      if (j < n2) {
        const double* q = pc + (p0 + j) * 3;
        const float bx = (float)(q[0] - ox), by = (float)(q[1] - oy), bz = (float)(q[2] - oz);
        mx[c] = -2.f * bx;
        my[c] = -2.f * by;
        mz[c] = -2.f * bz;
        b2[c] = fmaf(bz, bz, fmaf(by, by, bx * bx));
        bm = fmaxf(bm, fmaxf(fabsf(bx), fmaxf(fabsf(by), fabsf(bz))));
      } else {
        mx[c] = my[c] = mz[c] = 0.f;
        b2[c] = __builtin_huge_valf();  // never within
      }
    }
#pragma unroll 1
    for (int r = 0; r < kRowsPerWave; ++r) {
      const int i = row0 + r;
      if (i >= n1max) break;
      uint32_t inm = 0;
      if (i < n1) {
        const double* a = cad + (c0 + i) * 3;
        const double ax64 = a[0], ay64 = a[1], az64 = a[2];
        const float ax = (float)(ax64 - ox), ay = (float)(ay64 - oy), az = (float)(az64 - oz);
        const float a2 = fmaf(az, az, fmaf(ay, ay, ax * ax));
        const float S = fmaxf(fabsf(ax), fmaxf(fabsf(ay), fabsf(az))) + bm;
        const float E0 = 1.01f * u * S;
        const float margin = 2.f * (3.f * E0 * (2.f * R + E0) + 21.f * u * S * S + 2.f * u * thr2f) + 1e-30f;
        const float lo = thr2f - margin, hi = thr2f + margin;
        uint32_t him = 0;
#pragma unroll
        for (int c = 0; c < kColsPerLane; ++c) {
          const float sq = fmaf(ax, mx[c], fmaf(ay, my[c], fmaf(az, mz[c], a2 + b2[c])));
          inm |= (sq <= lo ? 1u : 0u) << c;
          him |= (sq <= hi ? 1u : 0u) << c;
        }
        uint32_t amb = him & ~inm;
        if (__builtin_expect(amb != 0, 0)) {  // rare: exact fp64 recheck of the band
          while (amb) {
            const int c = __ffs(amb) - 1;
            amb &= amb - 1;
            const double* q = pc + (p0 + j0 + c) * 3;
            if (within(ax64, ay64, az64, q[0], q[1], q[2], thr2)) inm |= 1u << c;
          }
        }
        const int tot = pk::wave_sum_i32_s(__popc(inm));
        if (lane == 0) cnt[r] += tot;  // same wave only: program order, no barrier
      }
      if (mask != nullptr && j0 < ld) {
        // spread 4 mask bits into 4 bytes: (nibble * 0x204081) & 0x01010101
        const uint32_t w0 = ((inm & 0xfu) * 0x204081u) & 0x01010101u;
        const uint32_t w1 = (((inm >> 4) & 0xfu) * 0x204081u) & 0x01010101u;
        const uint32_t w2 = (((inm >> 8) & 0xfu) * 0x204081u) & 0x01010101u;
        const uint32_t w3 = (((inm >> 12) & 0xfu) * 0x204081u) & 0x01010101u;
        uint4* dst = reinterpret_cast<uint4*>(mask + ((int64_t)b * n1max + i) * ld + j0);
        *dst = make_uint4(w0, w1, w2, w3);
      }
    }
  }
  if (lane < kRowsPerWave && row0 + lane < n1max) rowcount[(int64_t)b * n1max + row0 + lane] = cnt[lane];
}

// Count-only variant (no mask); same arithmetic.
__global__ __launch_bounds__(kBqThreads) void bq_count_kernel(
    const double* __restrict__ cad, const int64_t* __restrict__ cad_off,
    const double* __restrict__ pc, const int64_t* __restrict__ pc_off,
    const double* __restrict__ thr2v, int n1max, int32_t* __restrict__ rowcount) {
  const int b = blockIdx.z;
  const int64_t c0 = cad_off[b], p0 = pc_off[b];
  const int n1 = (int)(cad_off[b + 1] - c0);
  const int n2 = (int)(pc_off[b + 1] - p0);
  const double thr2 = thr2v[b];
  const int lane = pk::lane_id();
  const int j0 = blockIdx.x * kColsPerWave + lane * kColsPerLane;
  const int row0 = blockIdx.y * kRowsPerBlock + pk::wave_id() * kRowsPerWave;
  if (row0 >= n1) return;
  double qx[kColsPerLane], qy[kColsPerLane], qz[kColsPerLane];
#pragma unroll
  for (int c = 0; c < kColsPerLane; ++c) {
    const int j = j0 + c;
    if (j < n2) {
      const double* q = pc + (p0 + j) * 3;
      qx[c] = q[0];
      qy[c] = q[1];
      qz[c] = q[2];
    } else {
      qx[c] = qy[c] = qz[c] = __builtin_huge_val();
    }
  }
  for (int r = 0; r < kRowsPerWave; ++r) {
    const int i = row0 + r;
    if (i >= n1) break;
    const double* a = cad + (c0 + i) * 3;
    const double ax = a[0], ay = a[1], az = a[2];
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < kColsPerLane; ++c) cnt += within(ax, ay, az, qx[c], qy[c], qz[c], thr2) ? 1 : 0;
    cnt = pk::wave_sum_i32(cnt);
    if (lane == 0 && cnt != 0) atomicAdd(rowcount + (int64_t)b * n1max + i, cnt);
  }
}

// Exclusive scan of row counts per crop. grid (B), block 1024.
__global__ __launch_bounds__(1024) void bq_scan_kernel(const int32_t* __restrict__ rowcount,
                                                       int n1max, int64_t* __restrict__ rowoff,
                                                       int64_t* __restrict__ total) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry_s;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < n1max; base += 1024) {
    const int i = base + tid;
    const int64_t v = i < n1max ? (int64_t)rowcount[(int64_t)b * n1max + i] : 0;
    const int64_t inc = pk::wave_inclusive_scan_i64(v);
    if (pk::lane_id() == 63) wsum[pk::wave_id()] = inc;
    __syncthreads();
    int64_t pre = carry_s;
    for (int w = 0; w < pk::wave_id(); ++w) pre += wsum[w];
    if (i < n1max) rowoff[(int64_t)b * n1max + i] = pre + inc - v;
    __syncthreads();
    if (tid == 1023) carry_s = pre + inc;
    __syncthreads();
  }
  if (tid == 0) total[b] = carry_s;
}

// Ordered compaction: one wave per row. grid (ceil(n1max/4), B), block 256.
// Reads the mask row (16 bytes per lane per 1024-column chunk) or recomputes it.
__global__ __launch_bounds__(256) void bq_pairs_kernel(
    const double* __restrict__ cad, const int64_t* __restrict__ cad_off,
    const double* __restrict__ pc, const int64_t* __restrict__ pc_off,
    const double* __restrict__ thr2v, int n1max, int n2max, int ld,
    const uint8_t* __restrict__ mask, const int32_t* __restrict__ rowcount,
    const int64_t* __restrict__ rowoff, int64_t* __restrict__ pairs, int64_t cap,
    int8_t* __restrict__ ov12, int8_t* __restrict__ ov21) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 4 + pk::wave_id();
  const int64_t c0 = cad_off[b], p0 = pc_off[b];
  const int n1 = (int)(cad_off[b + 1] - c0);
  const int n2 = (int)(pc_off[b + 1] - p0);
  if (i >= n1max) return;
  const int lane = pk::lane_id();
  const int cnt_row = i < n1 ? rowcount[(int64_t)b * n1max + i] : 0;
  if (ov12 != nullptr && lane == 0) ov12[(int64_t)b * n1max + i] = cnt_row > 0 ? 1 : 0;
  if (cnt_row == 0) return;
  const double thr2 = thr2v[b];
  const double* a = cad + (c0 + i) * 3;
  const double ax = a[0], ay = a[1], az = a[2];
  int64_t off = rowoff[(int64_t)b * n1max + i];
  int64_t* __restrict__ pb = pairs + (int64_t)b * cap * 2;
  for (int jc = 0; jc < n2; jc += kColsPerWave) {
    const int j0 = jc + lane * kColsPerLane;
    uint32_t bits = 0;
    if (mask != nullptr) {
      if (j0 < ld) {
        const uint4 m = *reinterpret_cast<const uint4*>(mask + ((int64_t)b * n1max + i) * ld + j0);
        const uint32_t wv[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
        for (int c = 0; c < kColsPerLane; ++c) bits |= ((wv[c >> 2] >> ((c & 3) * 8)) & 1u) << c;
      }
    } else {
#pragma unroll
      for (int c = 0; c < kColsPerLane; ++c) {
        const int j = j0 + c;
        if (j < n2) {
          const double* q = pc + (p0 + j) * 3;
          bits |= (within(ax, ay, az, q[0], q[1], q[2], thr2) ? 1u : 0u) << c;
        }
      }
    }
    const int mine = __popc(bits);
    const int inc = pk::wave_inclusive_scan_i32(mine);
    int64_t w = off + inc - mine;
    while (bits) {
      const int c = __ffs(bits) - 1;
      bits &= bits - 1;
      const int j = j0 + c;
      if (w < cap) {
        pb[2 * w + 0] = i;
        pb[2 * w + 1] = j;
      }
      if (ov21 != nullptr) ov21[(int64_t)b * n2max + j] = 1;
      ++w;
    }
    off += __shfl(inc, 63);
  }
}

}  // namespace

extern "C" int pk_ball_query_mask(const double* cad, const int64_t* cad_off, const double* pc,
                                  const int64_t* pc_off, const double* thr2, int B, int n1max,
                                  int n2max, uint8_t* mask, int ld, int32_t* rowcount,
                                  void* stream) {
  PK_REQUIRE(B >= 0 && n1max >= 0 && n2max >= 0);
  if (B == 0 || n1max == 0) return PK_OK;
  PK_REQUIRE(cad && cad_off && pc && pc_off && thr2 && rowcount);
  PK_REQUIRE(mask == nullptr || (ld >= n2max && ld % kColsPerLane == 0));
  hipStream_t s = pk::as_stream(stream);
  dim3 grid((n1max + kRowsPerBlock - 1) / kRowsPerBlock, B);
  hipLaunchKernelGGL(bq_mask_f32_kernel, grid, dim3(kBqThreads), 0, s, cad, cad_off, pc, pc_off,
                     thr2, n1max, ld, mask, rowcount);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// Development hook (not in include/posekern.h): the all-fp64 mask kernel, for A/B timing.
extern "C" int pkdev_ball_query_mask64(const double* cad, const int64_t* cad_off, const double* pc,
                                       const int64_t* pc_off, const double* thr2, int B, int n1max,
                                       int n2max, uint8_t* mask, int ld, int32_t* rowcount,
                                       void* stream) {
  hipStream_t s = pk::as_stream(stream);
  hipError_t e = hipMemsetAsync(rowcount, 0, sizeof(int32_t) * (size_t)B * n1max, s);
  if (e != hipSuccess) return (int)e;
  dim3 grid((ld + kColsPerWave - 1) / kColsPerWave, (n1max + kRowsPerBlock - 1) / kRowsPerBlock, B);
  hipLaunchKernelGGL(bq_mask_kernel, grid, dim3(kBqThreads), 0, s, cad, cad_off, pc, pc_off, thr2,
                     n1max, ld, mask, rowcount);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_ball_query_pairs(const double* cad, const int64_t* cad_off, const double* pc,
                                   const int64_t* pc_off, const double* thr2, int B, int n1max,
                                   int n2max, const uint8_t* mask, int ld,
                                   const int32_t* rowcount, int64_t* rowoff, int64_t* pairs,
                                   int64_t cap, int64_t* count, int8_t* ov12, int8_t* ov21,
                                   void* stream) {
  PK_REQUIRE(B >= 0 && n1max >= 0 && n2max >= 0 && cap >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(cad && cad_off && pc && pc_off && thr2 && rowcount && rowoff && count);
  PK_REQUIRE(pairs != nullptr || cap == 0);
  PK_REQUIRE(mask == nullptr || (ld >= n2max && ld % kColsPerLane == 0));
  hipStream_t s = pk::as_stream(stream);
  if (ov21 != nullptr) {
    hipError_t e = hipMemsetAsync(ov21, 0, (size_t)B * n2max, s);
    if (e != hipSuccess) return (int)e;
  }
  if (n1max == 0) {
    hipError_t e = hipMemsetAsync(count, 0, sizeof(int64_t) * B, s);
    return e == hipSuccess ? PK_OK : (int)e;
  }
  hipLaunchKernelGGL(bq_scan_kernel, dim3(B), dim3(1024), 0, s, rowcount, n1max, rowoff, count);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(bq_pairs_kernel, dim3((n1max + 3) / 4, B), dim3(256), 0, s, cad, cad_off, pc,
                     pc_off, thr2, n1max, n2max, ld, mask, rowcount, rowoff, pairs, cap, ov12,
                     ov21);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
