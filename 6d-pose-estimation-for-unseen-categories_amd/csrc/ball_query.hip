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

// ---------------------------------------------------------------------------------
// Streaming mask kernel (the default for n2max < 65536).
//
// Same fp32 screen + exact fp64 band recheck as bq_mask_f32_kernel, re-arranged so
// that the per-pair VALU work is ~6 instructions and the kernel runs at the mask-write
// (HBM) rate:
//   * per workgroup, the crop's columns are converted ONCE into LDS as float4
//     {-2bx, -2by, -2bz, |b|^2} (lane-major slots: conflict-free ds_read_b128), and
//     the 64 rows' per-row constants {ax, ay, az, lo'', W} once by wave 0;
//   * per pair: q = fma-chain(|b|^2; a.(-2b)) (3 FMA), d = q - lo'' (1 sub) where
//     lo'' = nextafter(fl(lo - |a|^2), +inf); "in" <=> q <= fl(lo - |a|^2) <=> sign(d);
//     the in-bits of 4 columns are gathered into one 4-byte word by two v_perm_b32
//     sign-replicating selects;
//   * ambiguity: a lane tracks min_u32(bits(d)); non-negative floats order as their
//     bits and negative ones sort above them, so one unsigned compare against
//     bits(W), W = fl(hi'' - lo''), flags any pair in (lo, hi] (rare -> fp64 recheck);
//   * the q / d arithmetic runs on packed f32 pairs (v_pk_fma_f32, v_pk_add_f32: two
//     columns per instruction at the scalar issue rate, each half rounded as the
//     scalar op) -- the kernel is VALU-issue bound, not store bound, without them;
//   * a lane keeps one running in-count per row (v_sad_u8 over the byte-summed mask
//     words, no popcounts); the wave reduces them once, at the end;
//   * blocks are renumbered so that a crop's row blocks land on one XCD (shared L2
//     for its column data).
// The classification is the one bq_mask_f32_kernel proves exact: the
// margin is unchanged, and moving |a|^2 to the threshold side replaces one rounding
// of (|a|^2 + |b|^2) by one rounding of (lo - |a|^2), covered by the 2u*thr2 term.
constexpr int kStageCols = 2048;  // columns converted into LDS per stage (32 KiB)
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
using f32x2 = __attribute__((ext_vector_type(2))) float;

__device__ __forceinline__ float next_up(float x) {  // nextafter(x, +inf) for finite x
  const uint32_t b = __float_as_uint(x);
  if (x == 0.f) return __uint_as_float(1u);  // +-0 -> smallest positive subnormal
  return __uint_as_float(x > 0.f ? b + 1u : b - 1u);
}

template <bool NT>  // NT: nontemporal mask stores (the product choice)
__global__ __launch_bounds__(kBqThreads) void bq_mask_stream_kernel(
    const double* __restrict__ cad, const int64_t* __restrict__ cad_off,
    const double* __restrict__ pc, const int64_t* __restrict__ pc_off,
    const double* __restrict__ thr2v, int n1max, int ld, int nrb, uint8_t* __restrict__ mask,
    int32_t* __restrict__ rowcount) {
  __shared__ __attribute__((aligned(16))) float4 scol[kStageCols];
  __shared__ __attribute__((aligned(16))) float4 srow[kRowsPerBlock];
  __shared__ uint32_t srowW[kRowsPerBlock];
  __shared__ uint32_t sbm[kBqThreads / pk::kWave];

  // XCD-aware renumbering: hardware block L runs on XCD L % 8; give each XCD a
  // contiguous range of logical blocks (bijective for any grid size).
  const int G = gridDim.x, L = blockIdx.x;
  const int q8 = G >> 3, r8 = G & 7, x8 = L & 7;
  const int logical = x8 * q8 + min(x8, r8) + (L >> 3);
  const int b = logical / nrb;
  const int rb = logical - b * nrb;

  const int64_t c0 = cad_off[b], p0 = pc_off[b];
  const int n1 = (int)(cad_off[b + 1] - c0);
  const int n2 = (int)(pc_off[b + 1] - p0);
  const double thr2 = thr2v[b];
  const int tid = threadIdx.x, lane = pk::lane_id(), wave = pk::wave_id();
  const int rowblk0 = rb * kRowsPerBlock;
  const int row0 = rowblk0 + wave * kRowsPerWave;
  const double ox = n1 > 0 ? cad[c0 * 3 + 0] : 0.0;
  const double oy = n1 > 0 ? cad[c0 * 3 + 1] : 0.0;
  const double oz = n1 > 0 ? cad[c0 * 3 + 2] : 0.0;
  const float u = 5.9604645e-8f;  // 2^-24
  const float thr2f = (float)thr2;
  const float R = sqrtf(thr2f) * 1.001f;
  const int ncols = mask != nullptr ? ld : n2;

  uint32_t cnt[kRowsPerWave] = {};  // this lane's in-pairs of row row0 + r (<= 16 per chunk)

  for (int s0 = 0; s0 < ncols; s0 += kStageCols) {
    const int scols = min(kStageCols, ncols - s0);
    const int spad = (scols + kColsPerWave - 1) & ~(kColsPerWave - 1);
    __syncthreads();  // previous stage's readers are done with scol / srow
    // ---- columns -> LDS. Column jj (stage-relative) of chunk k = jj / 1024 sits in
    // slot k*1024 + (jj % 16) * 64 + (jj % 1024) / 16: lane l's c-th column is
    // contiguous across lanes for every c. Slots past the crop get never-within padding.
    float bm = 0.f;
    for (int jj = tid; jj < spad; jj += kBqThreads) {
      const int j = s0 + jj;
      float4 v;
      if (j < n2) {
        const double* qd = pc + (p0 + j) * 3;
        const float bx = (float)(qd[0] - ox), by = (float)(qd[1] - oy), bz = (float)(qd[2] - oz);
        v = make_float4(-2.f * bx, -2.f * by, -2.f * bz, fmaf(bz, bz, fmaf(by, by, bx * bx)));
        bm = fmaxf(bm, fmaxf(fabsf(bx), fmaxf(fabsf(by), fabsf(bz))));
      } else {
        v = make_float4(0.f, 0.f, 0.f, __builtin_huge_valf());
      }
      const int k = jj >> 10, w = jj & 1023;
      scol[(k << 10) + ((w & 15) << 6) + (w >> 4)] = v;
    }
    uint32_t bmb = pk::wave_max_u32_s(__float_as_uint(bm));  // bm >= 0: bits order = value order
    if (lane == 0) sbm[wave] = bmb;
    __syncthreads();
    bmb = max(max(sbm[0], sbm[1]), max(sbm[2], sbm[3]));
    // ---- per-row constants (wave 0), with this stage's column bound
    if (wave == 0) {
      const int i = rowblk0 + lane;
      float4 rv = make_float4(0.f, 0.f, 0.f, -__builtin_huge_valf());  // padding row: d = +inf
      uint32_t wb = 0u;
      if (i < n1) {
        const double* a = cad + (c0 + i) * 3;
        const float ax = (float)(a[0] - ox), ay = (float)(a[1] - oy), az = (float)(a[2] - oz);
        const float a2 = fmaf(az, az, fmaf(ay, ay, ax * ax));
        const float S = fmaxf(fabsf(ax), fmaxf(fabsf(ay), fabsf(az))) + __uint_as_float(bmb);
        const float E0 = 1.01f * u * S;
        const float margin = 2.f * (3.f * E0 * (2.f * R + E0) + 21.f * u * S * S + 2.f * u * thr2f) + 1e-30f;
        const float lo_r = (thr2f - margin) - a2;
        const float hi_r = (thr2f + margin) - a2;
        const float lo2 = next_up(lo_r);
        const float W = hi_r - lo2;
        rv = make_float4(ax, ay, az, lo2);
        wb = W > 0.f ? __float_as_uint(W) : 0u;
      }
      srow[lane] = rv;
      srowW[lane] = wb;
    }
    __syncthreads();
    if (row0 >= n1max) continue;  // every barrier above stays uniform

    for (int ch = 0; ch < scols; ch += kColsPerWave) {
      const int j0 = s0 + ch + lane * kColsPerLane;  // first column of this lane
      // column pairs in packed registers: one v_pk_fma_f32 / v_pk_add_f32 does two
      // columns at the scalar rate, each lane-half rounded exactly as v_fma_f32 / v_sub_f32
      f32x2 mx[kColsPerLane / 2], my[kColsPerLane / 2], mz[kColsPerLane / 2], b2[kColsPerLane / 2];
#pragma unroll
      for (int c = 0; c < kColsPerLane; ++c) {
        const float4 v = scol[ch + (c << 6) + lane];
        mx[c >> 1][c & 1] = v.x;
        my[c >> 1][c & 1] = v.y;
        mz[c >> 1][c & 1] = v.z;
        b2[c >> 1][c & 1] = v.w;
      }
      const bool store = mask != nullptr && (ch + lane * kColsPerLane) < scols;
      uint8_t* rowp = store ? mask + ((int64_t)b * n1max + row0) * ld + j0 : nullptr;
#pragma unroll
      for (int r = 0; r < kRowsPerWave; ++r) {
        const int i = row0 + r;
        if (i >= n1max) break;  // wave-uniform
        const float4 rv = srow[wave * kRowsPerWave + r];
        const uint32_t Wb = srowW[wave * kRowsPerWave + r];
        const f32x2 ax2 = {rv.x, rv.x}, ay2 = {rv.y, rv.y}, az2 = {rv.z, rv.z}, lo2 = {rv.w, rv.w};
        float d[kColsPerLane];
        uint32_t mn = 0xffffffffu;
#pragma unroll
        for (int c2 = 0; c2 < kColsPerLane / 2; ++c2) {
          const f32x2 qv = __builtin_elementwise_fma(
              ax2, mx[c2], __builtin_elementwise_fma(ay2, my[c2], __builtin_elementwise_fma(az2, mz[c2], b2[c2])));
          const f32x2 dv = qv - lo2;
          d[2 * c2] = dv.x;
          d[2 * c2 + 1] = dv.y;
          mn = min(min(mn, __float_as_uint(dv.x)), __float_as_uint(dv.y));  // v_min3_u32
        }
        // 0x01 where sign(d) = 1 (in). v_perm_b32 selectors 9 / 11 replicate the sign
        // bit of src1 / src0 into a byte; 12 gives 0x00.
        uint32_t w[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(d[4 * m + 1]), __float_as_uint(d[4 * m]),
                                                    0x0c0c0b09u);
          const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(d[4 * m + 3]), __float_as_uint(d[4 * m + 2]),
                                                    0x0b090c0cu);
          w[m] = (lo | hi) & 0x01010101u;
        }
        if (__builtin_expect(mn <= Wb, 0)) {  // rare: exact fp64 recheck of the band
          uint32_t amb = 0;
#pragma unroll
          for (int c = 0; c < kColsPerLane; ++c) amb |= (__float_as_uint(d[c]) <= Wb ? 1u : 0u) << c;
          const double* a = cad + (c0 + i) * 3;
          const double ax64 = a[0], ay64 = a[1], az64 = a[2];
          uint32_t fix = 0, todo = amb;
          while (todo) {
            const int c = __ffs(todo) - 1;
            todo &= todo - 1;
            const double* qd = pc + (p0 + j0 + c) * 3;
            fix |= (within(ax64, ay64, az64, qd[0], qd[1], qd[2], thr2) ? 1u : 0u) << c;
          }
#pragma unroll
          for (int m = 0; m < 4; ++m) {  // spread 4 bits to 4 bytes: (nibble * 0x204081) & 0x01010101
            const uint32_t clr = ((((amb >> (4 * m)) & 0xfu) * 0x204081u) & 0x01010101u) * 0xffu;
            const uint32_t set = (((fix >> (4 * m)) & 0xfu) * 0x204081u) & 0x01010101u;
            w[m] = (w[m] & ~clr) | set;
          }
        }
        // bytes are 0/1, so the byte-wise sum of the four words has no carries (<= 4 per
        // byte) and v_sad_u8 against 0 adds its four bytes to the row's running count
        cnt[r] = __builtin_amdgcn_sad_u8(w[0] + w[1] + w[2] + w[3], 0u, cnt[r]);
        if (store) {
          const u32x4 val = {w[0], w[1], w[2], w[3]};
          if constexpr (NT) {
            __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(rowp + (int64_t)r * ld));
          } else {
            *reinterpret_cast<u32x4*>(rowp + (int64_t)r * ld) = val;
          }
        }
      }
    }
  }
  if (row0 >= n1max) return;
  // row totals, two rows per reduction (16-bit fields: a row holds < 65536 pairs); lane r
  // keeps row r's count
  uint32_t mine = 0;
#pragma unroll
  for (int rp = 0; rp < kRowsPerWave; rp += 2) {
    const uint32_t t = (uint32_t)pk::wave_sum_i32_s((int)(cnt[rp] | (cnt[rp + 1] << 16)));
    if ((lane >> 1) == (rp >> 1)) mine = (lane & 1) ? (t >> 16) : (t & 0xffffu);
  }
  if (lane < kRowsPerWave && row0 + lane < n1max) rowcount[(int64_t)b * n1max + row0 + lane] = (int32_t)mine;
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
                                                       int64_t* __restrict__ total, int8_t* __restrict__ ov21,
                                                       int32_t* __restrict__ colcount, int n2max) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry_s;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  // crop b's ov21 flags cleared here (the pairs kernel after this launch sets them): no
  // separate zero-fill launch
  if (ov21 != nullptr)
    for (int j = tid; j < n2max; j += 1024) ov21[(int64_t)b * n2max + j] = 0;
  if (colcount != nullptr)  // (likewise the per-column pair counts the pairs kernel accumulates)
    for (int j = tid; j < n2max; j += 1024) colcount[(int64_t)b * n2max + j] = 0;
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
    int8_t* __restrict__ ov12, int8_t* __restrict__ ov21, const int64_t* __restrict__ count, int B,
    int32_t* __restrict__ over, int32_t* __restrict__ colcount) {
  const int b = blockIdx.y;
  if (over != nullptr && blockIdx.x == 0 && b == 0) {  // the pass-1 totals are final: any above cap?
    int o = 0;
    for (int k = threadIdx.x; k < B; k += 256) o |= count[k] > cap;
    o = __syncthreads_or(o);
    if (threadIdx.x == 0) over[0] = o;
  }
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
        // pairs per crop point among the kept list (C_gt's G row weights; integer atomics: exact)
        if (colcount != nullptr) atomicAdd(&colcount[(int64_t)b * n2max + j], 1);
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
  const int nrb = (n1max + kRowsPerBlock - 1) / kRowsPerBlock;
  if (n2max < 65536 && (int64_t)nrb * B < (1ll << 31)) {
#define PK_BQS(NT)                                                                              \
  hipLaunchKernelGGL((bq_mask_stream_kernel<NT>), dim3(nrb * B), dim3(kBqThreads), 0, s, cad, cad_off, \
                     pc, pc_off, thr2, n1max, ld, nrb, mask, rowcount)
#ifdef PK_DEVBUILD
    // PK_BQ_VAR=1: plain mask stores (A/B only: 0.40 vs 0.56 of HBM peak for nt, profiles/r06_bq_ramp.txt)
    static const int var = [] { const char* e = std::getenv("PK_BQ_VAR"); return e ? std::atoi(e) : 0; }();
    if (var == 1) {
      PK_BQS(false);
    } else {
      PK_BQS(true);
    }
#else
    PK_BQS(true);
#endif
#undef PK_BQS
  } else {
    dim3 grid(nrb, B);
    hipLaunchKernelGGL(bq_mask_f32_kernel, grid, dim3(kBqThreads), 0, s, cad, cad_off, pc, pc_off,
                       thr2, n1max, ld, mask, rowcount);
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}

#ifdef PK_DEVBUILD
// Development hook (not in include/posekern.h): the previous fp32-screen kernel, for A/B timing.
extern "C" int pkdev_ball_query_mask_v1(const double* cad, const int64_t* cad_off, const double* pc,
                                        const int64_t* pc_off, const double* thr2, int B, int n1max,
                                        int n2max, uint8_t* mask, int ld, int32_t* rowcount,
                                        void* stream) {
  hipStream_t s = pk::as_stream(stream);
  dim3 grid((n1max + kRowsPerBlock - 1) / kRowsPerBlock, B);
  hipLaunchKernelGGL(bq_mask_f32_kernel, grid, dim3(kBqThreads), 0, s, cad, cad_off, pc, pc_off,
                     thr2, n1max, ld, mask, rowcount);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
#endif  // PK_DEVBUILD

#ifdef PK_DEVBUILD
// Development hook (not in include/posekern.h): the all-fp64 mask kernel, for A/B timing.
extern "C" int pkdev_ball_query_mask64(const double* cad, const int64_t* cad_off, const double* pc,
                                       const int64_t* pc_off, const double* thr2, int B, int n1max,
                                       int n2max, uint8_t* mask, int ld, int32_t* rowcount,
                                       void* stream) {
  hipStream_t s = pk::as_stream(stream);
  hipError_t e = pk::zero_async(rowcount, sizeof(int32_t) * (size_t)B * n1max, s);
  if (e != hipSuccess) return (int)e;
  dim3 grid((ld + kColsPerWave - 1) / kColsPerWave, (n1max + kRowsPerBlock - 1) / kRowsPerBlock, B);
  hipLaunchKernelGGL(bq_mask_kernel, grid, dim3(kBqThreads), 0, s, cad, cad_off, pc, pc_off, thr2,
                     n1max, ld, mask, rowcount);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
#endif  // PK_DEVBUILD

extern "C" int pk_ball_query_pairs(const double* cad, const int64_t* cad_off, const double* pc,
                                   const int64_t* pc_off, const double* thr2, int B, int n1max,
                                   int n2max, const uint8_t* mask, int ld,
                                   const int32_t* rowcount, int64_t* rowoff, int64_t* pairs,
                                   int64_t cap, int64_t* count, int8_t* ov12, int8_t* ov21,
                                   int32_t* over, int32_t* colcount, void* stream) {
  PK_REQUIRE(B >= 0 && n1max >= 0 && n2max >= 0 && cap >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(cad && cad_off && pc && pc_off && thr2 && rowcount && rowoff && count);
  PK_REQUIRE(pairs != nullptr || cap == 0);
  PK_REQUIRE(mask == nullptr || (ld >= n2max && ld % kColsPerLane == 0));
  hipStream_t s = pk::as_stream(stream);
  if (n1max == 0) {
    hipError_t e = ov21 != nullptr ? pk::zero_async(ov21, (size_t)B * n2max, s) : hipSuccess;
    if (e == hipSuccess) e = pk::zero_async(count, sizeof(int64_t) * B, s);
    if (e == hipSuccess && over != nullptr) e = pk::zero_async(over, sizeof(int32_t), s);
    if (e == hipSuccess && colcount != nullptr) e = pk::zero_async(colcount, sizeof(int32_t) * (size_t)B * n2max, s);
    return e == hipSuccess ? PK_OK : (int)e;
  }
  hipLaunchKernelGGL(bq_scan_kernel, dim3(B), dim3(1024), 0, s, rowcount, n1max, rowoff, count, ov21, colcount, n2max);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(bq_pairs_kernel, dim3((n1max + 3) / 4, B), dim3(256), 0, s, cad, cad_off, pc,
                     pc_off, thr2, n1max, n2max, ld, mask, rowcount, rowoff, pairs, cap, ov12,
                     ov21, count, B, over, colcount);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
