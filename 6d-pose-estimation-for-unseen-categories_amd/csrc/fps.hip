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
// separately (TU compiled with -ffp-contract=off); the argmax is done in two 32-bit
// steps (max of the distance bits, then min of the indices holding that max), so ties
// go to the lowest index exactly like torch.max.
//
// Layout: crops are packed back to back, xyz fp32 AoS [total, 3], crop b spans
// rows [offsets[b], offsets[b+1]). Each thread keeps PPT points (strided by the
// block size, so a thread's points are in increasing index order) and their running
// distances in registers; a structure-of-arrays copy of the crop sits in LDS so the
// current centroid is a broadcast read. Per iteration: branch-free update of the
// running distances and of the thread's (best, index) pair, DPP row reductions +
// readlane for the wave result, one LDS slot per wave, ONE barrier (slots are
// double-buffered), then a 16-lane DPP reduction of the slots that every wave
// repeats, leaving the next centroid in a scalar register.
#include "common.hpp"

#include <cstdlib>

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// row b's entries past npoint[b] (the whole row for an empty crop) are written as 0 by the
// kernel itself, so the caller's output needs no fill launch
__device__ __forceinline__ void fps_zero_tail(int64_t* __restrict__ out, int out_stride, int b, int np) {
  int64_t* __restrict__ o = out + (int64_t)b * out_stride;
  for (int i = (np > 0 ? np : 0) + (int)threadIdx.x; i < out_stride; i += (int)blockDim.x) o[i] = 0;
}

__device__ __forceinline__ float vmin_f32(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

constexpr int kFpsMaxLds = 13312;  // points whose SoA copy fits in LDS (156 KiB)

template <int NT, int PPT, bool LDS>
__global__ __launch_bounds__(NT) void fps_kernel(
    const float* __restrict__ xyz, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ start, const int32_t* __restrict__ npoint,
    int64_t* __restrict__ out, int out_stride) {
  constexpr int NW = NT / pk::kWave;
  static_assert(NW <= 16, "slot reduction assumes <= 16 waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = pk::lane_id();
  const int64_t base = offsets[b];
  const int n = (int)(offsets[b + 1] - base);
  const int np = npoint[b];
  const float* __restrict__ p = xyz + base * 3;

  uint2* slots = reinterpret_cast<uint2*>(smem);  // [2][16] (bits, index)
  float* sx = reinterpret_cast<float*>(smem + 2 * 16 * sizeof(uint2));
  const int n_pad = (n + 3) & ~3;
  float* sy = sx + n_pad;
  float* sz = sy + n_pad;

  float px[PPT], py[PPT], pz[PPT], pd[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int idx = tid + k * NT;
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
      pd[k] = -1.f;  // empty slot: min(-1, d >= 0) keeps it at -1, never selected
    }
  }
  fps_zero_tail(out, out_stride, b, np);
  if (n <= 0 || np <= 0) return;
  __syncthreads();

  int far = start[b];
  const int kmax = (n + NT - 1) / NT;
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
    float bd = -1.f;
    int bk = 0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      if (k < kmax) {  // block-uniform: crops smaller than the template bound skip work
        const float dx = px[k] - cx;
        const float dy = py[k] - cy;
        const float dz = pz[k] - cz;
        const float d = (dx * dx + dy * dy) + dz * dz;  // no contraction (TU flag)
        pd[k] = fminf(pd[k], d);                        // == (d < pd ? d : pd): no NaNs
        const bool gt = pd[k] > bd;                     // strict: lowest k wins ties
        bd = gt ? pd[k] : bd;
        bk = gt ? k : bk;
      }
    }
    const bool valid = bd >= 0.f;
    const uint32_t bits = valid ? pk::f32_bits(bd) : 0u;
    const uint32_t gidx = valid ? (uint32_t)(tid + bk * NT) : 0xffffffffu;
    const uint32_t wmax = pk::wave_max_u32_s(bits);
    const uint32_t widx = pk::wave_min_u32_s(bits == wmax ? gidx : 0xffffffffu);
    uint2* s = slots + (i & 1) * 16;
    if (lane == 0) s[pk::wave_id()] = make_uint2(wmax, widx);
    __syncthreads();
    uint2 v = make_uint2(0u, 0xffffffffu);
    if (lane < NW) v = s[lane];
    const uint32_t m = pk::readlane(pk::row_max_u32(v.x), 0);
    far = (int)pk::readlane(pk::row_min_u32(v.x == m ? v.y : 0xffffffffu), 0);
  }
}

// Pruned variant (the production path). A wave's k-th slot column — indices
// w*64 + lane + k*NT, 64 consecutive points, a short run of image row in the crop's
// pixel order — is a bucket with a bounding box and its current max running distance
// (lane k of the wave holds bucket k's box, max and argmax). Per iteration all buckets of
// a wave are tested at once (one lane each): if the box lies at computed squared
// distance lb from the new centroid with lb (1 - 2^-19) >= the bucket max, every point
// of the bucket has fl(d) >= its running distance (fl(d) >= (1 - 5u) d_true, d_true >=
// box distance, lb <= (1 + 5u) box distance; 2^-19 > 11u), so fminf leaves it unchanged
// and the bucket is skipped bit-exactly. Only buckets near the centroid are updated; the
// wave's best is a reduction over its bucket maxima.
template <int NT, int PPT>
__global__ __launch_bounds__(NT) void fps_pruned_kernel(
    const float* __restrict__ xyz, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ start, const int32_t* __restrict__ npoint,
    int64_t* __restrict__ out, int out_stride) {
  constexpr int NW = NT / pk::kWave;
  static_assert(NW <= 16 && PPT <= pk::kWave, "bucket/slot layout limits");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = pk::lane_id();
  const int64_t base = offsets[b];
  const int n = (int)(offsets[b + 1] - base);
  const int np = npoint[b];
  const float* __restrict__ p = xyz + base * 3;

  uint2* slots = reinterpret_cast<uint2*>(smem);  // [2][16] (bits, index)
  float* sx = reinterpret_cast<float*>(smem + 2 * 16 * sizeof(uint2));
  const int n_pad = (n + 3) & ~3;
  float* sy = sx + n_pad;
  float* sz = sy + n_pad;

  float px[PPT], py[PPT], pz[PPT], pd[PPT];
  // lane k: box of bucket k, its max running distance (as bits) and argmax
  float bx0 = 0.f, bx1 = 0.f, by0 = 0.f, by1 = 0.f, bz0 = 0.f, bz1 = 0.f;
  uint32_t bmb = 0u, bmi = 0xffffffffu;
  bool bval = false;
  // every point's coordinates first, unconditionally at a clamped index (a conditional load is a
  // branch + a wait: PPT serial memory round trips before the first iteration)
  if (n > 0) {  // block-uniform (an empty crop's base may be the end of the buffer)
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int idx = tid + k * NT;
      const int ic = idx < n ? idx : 0;
      px[k] = p[3 * ic + 0];
      py[k] = p[3 * ic + 1];
      pz[k] = p[3 * ic + 2];
    }
  }
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int idx = tid + k * NT;
    const bool ok = idx < n;
    if (ok) {
      pd[k] = 1e10f;
      sx[idx] = px[k];
      sy[idx] = py[k];
      sz[idx] = pz[k];
    } else {
      px[k] = py[k] = pz[k] = 0.f;
      pd[k] = -1.f;  // empty slot: min(-1, d >= 0) keeps it at -1, never selected
    }
    const uint64_t any = __ballot(ok);
    if (any) {  // wave-uniform: bucket k has points
      const float inf = __builtin_huge_valf();
      const uint32_t x0 = pk::wave_min_u32_s(pk::f32_ordered(ok ? px[k] : inf));
      const uint32_t x1 = pk::wave_max_u32_s(pk::f32_ordered(ok ? px[k] : -inf));
      const uint32_t y0 = pk::wave_min_u32_s(pk::f32_ordered(ok ? py[k] : inf));
      const uint32_t y1 = pk::wave_max_u32_s(pk::f32_ordered(ok ? py[k] : -inf));
      const uint32_t z0 = pk::wave_min_u32_s(pk::f32_ordered(ok ? pz[k] : inf));
      const uint32_t z1 = pk::wave_max_u32_s(pk::f32_ordered(ok ? pz[k] : -inf));
      if (lane == k) {
        bx0 = pk::f32_unordered(x0);
        bx1 = pk::f32_unordered(x1);
        by0 = pk::f32_unordered(y0);
        by1 = pk::f32_unordered(y1);
        bz0 = pk::f32_unordered(z0);
        bz1 = pk::f32_unordered(z1);
        bmb = pk::f32_bits(1e10f);
        bmi = (uint32_t)(pk::wave_id() * pk::kWave + k * NT + (__ffsll((unsigned long long)any) - 1));
        bval = true;
      }
    }
  }
  fps_zero_tail(out, out_stride, b, np);
  if (n <= 0 || np <= 0) return;
  __syncthreads();

  int far = start[b];
  int64_t* __restrict__ o = out + (int64_t)b * out_stride;
  for (int i = 0; i < np; ++i) {
    if (tid == 0) o[i] = far;
    const float cx = sx[far], cy = sy[far], cz = sz[far];
    // one lane per bucket: can the centroid lower any running distance in it?
    const float ddx = fmaxf(fmaxf(bx0 - cx, cx - bx1), 0.f);
    const float ddy = fmaxf(fmaxf(by0 - cy, cy - by1), 0.f);
    const float ddz = fmaxf(fmaxf(bz0 - cz, cz - bz1), 0.f);
    const float lb = (ddx * ddx + ddy * ddy) + ddz * ddz;
    const bool need = bval && !(lb * 0.99999809f >= __uint_as_float(bmb));
    const uint64_t mask = __ballot(need);
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      if ((mask >> k) & 1ull) {  // wave-uniform (bit k is clear for empty buckets)
        const float dx = px[k] - cx;
        const float dy = py[k] - cy;
        const float dz = pz[k] - cz;
        const float d = (dx * dx + dy * dy) + dz * dz;  // no contraction (TU flag)
        pd[k] = fminf(pd[k], d);
        const bool valid = pd[k] >= 0.f;
        const uint32_t bits = valid ? pk::f32_bits(pd[k]) : 0u;
        const uint32_t wmax = pk::wave_max_u32_s(bits);
        // lanes hold the bucket's indices in increasing order: the first lane at the max
        // is the lowest index (torch.max's tie rule), no second reduction needed
        const uint64_t at = __ballot(valid && bits == wmax);
        const uint32_t widx = (uint32_t)(pk::wave_id() * pk::kWave + k * NT + (__ffsll((unsigned long long)at) - 1));
        if (lane == k) {
          bmb = wmax;
          bmi = widx;
        }
      }
    }
    // best bucket of the wave: lane k = bucket k and buckets are in increasing index order,
    // so the first lane at the max holds the lowest index
    const uint32_t bb = bval ? bmb : 0u;
    const uint32_t wmax = PPT <= 16 ? pk::readlane(pk::row_max_u32(bb), 0) : pk::wave_max_u32_s(bb);
    const uint64_t top = __ballot(bval && bb == wmax);
    const uint32_t widx = top ? pk::readlane(bmi, __ffsll((unsigned long long)top) - 1) : 0xffffffffu;
    uint2* s = slots + (i & 1) * 16;
    if (lane == 0) s[pk::wave_id()] = make_uint2(wmax, widx);
    __syncthreads();
    uint2 v = make_uint2(0u, 0xffffffffu);
    if (lane < NW) v = s[lane];
    const uint32_t m = pk::readlane(pk::row_max_u32(v.x), 0);
    far = (int)pk::readlane(pk::row_min_u32(v.x == m ? v.y : 0xffffffffu), 0);
  }
}

// Per-lane buckets (crops above the LDS bound of fps_pruned_kernel). Thread t holds PPT CONSECUTIVE points
// (indices t PPT .. t PPT + PPT - 1: a short run of image row in the crop's pixel order, so a
// compact box), and the lane's running maximum bd is exactly its bucket maximum — tracked
// anyway for the argmax, so the skip test costs no reduction. A lane updates its points only
// when the centroid can lower one of them (box distance lb with lb (1 - 2^-19) < bd; the
// exactness argument of fps_pruned_kernel), and a wave none of whose lanes needs the centroid
// skips the whole iteration body, reusing its cached (max, index, coordinates). The block
// result carries the winner's coordinates (no LDS / global read for the next centroid); one
// barrier per iteration (double-buffered slots). Ties: first maximal index, as torch.max
// (strict > over a lane's increasing indices; min index among equal maxima across lanes).
template <int NT, int PPT>
__global__ __launch_bounds__(NT) void fps_lane_kernel(
    const float* __restrict__ xyz, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ start, const int32_t* __restrict__ npoint,
    int64_t* __restrict__ out, int out_stride) {
  constexpr int NW = NT / pk::kWave;
  static_assert(NW <= 16, "slot layout limit");
  __shared__ uint32_t slot_b[2][16], slot_i[2][16];
  __shared__ float slot_x[2][16], slot_y[2][16], slot_z[2][16];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = pk::lane_id(), w = pk::wave_id();
  const int64_t base = offsets[b];
  const int n = (int)(offsets[b + 1] - base);
  const int np = npoint[b];
  const float* __restrict__ p = xyz + base * 3;

  float px[PPT], py[PPT], pz[PPT], pd[PPT];
  const float inf = __builtin_huge_valf();
  float bx0 = inf, bx1 = -inf, by0 = inf, by1 = -inf, bz0 = inf, bz1 = -inf;
  const int i0 = tid * PPT;
  if (n > 0) {  // unconditional loads at a clamped index (block-uniform guard: empty crop)
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int ic = i0 + k < n ? i0 + k : 0;
      px[k] = p[3 * ic + 0];
      py[k] = p[3 * ic + 1];
      pz[k] = p[3 * ic + 2];
    }
  }
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const bool ok = i0 + k < n;
    px[k] = ok ? px[k] : 0.f;
    py[k] = ok ? py[k] : 0.f;
    pz[k] = ok ? pz[k] : 0.f;
    pd[k] = ok ? 1e10f : -1.f;  // empty slot: min(-1, d >= 0) keeps it at -1, never selected
    if (ok) {
      bx0 = fminf(bx0, px[k]); bx1 = fmaxf(bx1, px[k]);
      by0 = fminf(by0, py[k]); by1 = fmaxf(by1, py[k]);
      bz0 = fminf(bz0, pz[k]); bz1 = fmaxf(bz1, pz[k]);
    }
  }
  const bool lval = i0 < n;
  fps_zero_tail(out, out_stride, b, np);
  if (n <= 0 || np <= 0) return;

  // the lane's current maximum running distance, its point and that point's coordinates
  float bd = lval ? 1e10f : -1.f;
  int bk = 0;
  float qx = px[0], qy = py[0], qz = pz[0];
  int far = start[b];
  float cx = p[3 * far + 0], cy = p[3 * far + 1], cz = p[3 * far + 2];
  uint32_t wbits = 0u, widx = 0xffffffffu;
  float wx = 0.f, wy = 0.f, wz = 0.f;
  int64_t* __restrict__ o = out + (int64_t)b * out_stride;
  for (int i = 0; i < np; ++i) {
    if (tid == 0) o[i] = far;
    const float ddx = fmaxf(fmaxf(bx0 - cx, cx - bx1), 0.f);
    const float ddy = fmaxf(fmaxf(by0 - cy, cy - by1), 0.f);
    const float ddz = fmaxf(fmaxf(bz0 - cz, cz - bz1), 0.f);
    const float lb = (ddx * ddx + ddy * ddy) + ddz * ddz;
    const bool need = lval && !(lb * 0.99999809f >= bd);
    if (__ballot(need)) {  // wave-uniform
      if (need) {
        bd = -1.f;
#pragma unroll
        for (int k = 0; k < PPT; ++k) {
          const float dx = px[k] - cx;
          const float dy = py[k] - cy;
          const float dz = pz[k] - cz;
          const float d = (dx * dx + dy * dy) + dz * dz;  // no contraction (TU flag)
          pd[k] = fminf(pd[k], d);
          const bool gt = pd[k] > bd;  // strict: lowest index on ties
          bd = gt ? pd[k] : bd;
          bk = gt ? k : bk;
          qx = gt ? px[k] : qx;
          qy = gt ? py[k] : qy;
          qz = gt ? pz[k] : qz;
        }
      }
      const bool valid = bd >= 0.f;
      const uint32_t bits = valid ? pk::f32_bits(bd) : 0u;
      const uint32_t gidx = valid ? (uint32_t)(i0 + bk) : 0xffffffffu;
      wbits = pk::wave_max_u32_s(bits);
      const uint64_t at = __ballot(valid && bits == wbits);
      int wl;
      if ((at & (at - 1)) == 0) {  // one lane at the max: lanes hold increasing index runs
        wl = __ffsll((unsigned long long)at) - 1;
      } else {  // several lanes: the first one holds the lowest index
        wl = __ffsll((unsigned long long)at) - 1;
      }
      widx = pk::readlane(gidx, wl);
      wx = __uint_as_float(pk::readlane(__float_as_uint(qx), wl));
      wy = __uint_as_float(pk::readlane(__float_as_uint(qy), wl));
      wz = __uint_as_float(pk::readlane(__float_as_uint(qz), wl));
    }
    const int par = i & 1;
    if (lane == 0) {
      slot_b[par][w] = wbits;
      slot_i[par][w] = widx;
      slot_x[par][w] = wx;
      slot_y[par][w] = wy;
      slot_z[par][w] = wz;
    }
    __syncthreads();
    uint32_t vb = 0u, vi = 0xffffffffu;
    float vx = 0.f, vy = 0.f, vz = 0.f;
    if (lane < NW) {
      vb = slot_b[par][lane];
      vi = slot_i[par][lane];
      vx = slot_x[par][lane];
      vy = slot_y[par][lane];
      vz = slot_z[par][lane];
    }
    // waves hold increasing index ranges too: the first wave at the max has the lowest index
    const uint32_t m = pk::readlane(pk::row_max_u32(vb), 0);
    const int l = __ffsll((unsigned long long)__ballot(lane < NW && vb == m)) - 1;
    far = (int)pk::readlane(vi, l);
    cx = __uint_as_float(pk::readlane(__float_as_uint(vx), l));
    cy = __uint_as_float(pk::readlane(__float_as_uint(vy), l));
    cz = __uint_as_float(pk::readlane(__float_as_uint(vz), l));
  }
}

// Flat variant (the production path up to 8192 points). Thread t owns the PPT CONSECUTIVE
// points t PPT .. t PPT + PPT - 1 (so lane order = index order), their running distances and
// their box; the lane's running maximum bd and its first argmax bk are kept exactly. Per
// iteration a lane updates its points only when the centroid can lower one of them (box
// distance lb with lb (1 - 2^-19) < bd, the exactness argument of fps_pruned_kernel), a wave
// whose lanes all skip reuses its cached best, and the block argmax is ONE LDS atomic per wave:
// ds_max_u64 of key = (distance bits << 32) | ~index (max distance, then lowest index, torch.max's
// tie rule) into a triple-buffered word, one barrier, one broadcast read. Round 2's kernels spent
// ~0.7 us per iteration in per-bucket / per-wave reductions and a 16-slot second stage.
// Round 6 (phase stamps, profiles/r06_fps_variants.txt): an iteration is paced by the updating
// wave's dependent chain (distances, max, argmax, wave reduction, key), so that chain was cut:
// the argmax runs with the whole wave active beside the wave reduction (the compiler places its
// compare -> select wait states under the DPP chain), the reduction is a signed max of the
// distance bits (no validity select), the skip ballot is the bare compare, and the TU is built
// without the atomic optimizer: 0.49 -> 0.41 us per iteration on the kbench crops, indices
// unchanged. (An inline-asm select reading per-compare SGPR masks measured 0.40 but is not kept:
// hipcc does not pad the VALU-mask-write -> v_cndmask hazard into an asm statement, and it pads
// two wait states there for its own code.)
#ifdef PK_DEVBUILD
// (development: per-wave phase cycle sums of the stamped flat kernel, tools/fps_stamps.py)
__device__ unsigned long long g_fps_stamps[64 * 16 * 8];
#endif

template <int NT, int PPT, bool STAMP = false, bool TRIM = true>
__global__ __launch_bounds__(NT) void fps_flat_kernel(
    const float* __restrict__ xyz, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ start, const int32_t* __restrict__ npoint,
    int64_t* __restrict__ out, int out_stride, int prio) {
  pk::set_wave_prio(prio);
  // STAMP (dev only): per wave, cycles in read + box test / update + wave reduction / atomic +
  // barrier, and the number of updating iterations
  [[maybe_unused]] unsigned long long st_box = 0, st_upd = 0, st_bar = 0, st_nupd = 0, t0 = 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);  // [3] (4 words reserved)
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = pk::lane_id();
  const int64_t base = offsets[b];
  const int n = (int)(offsets[b + 1] - base);
  const int np = npoint[b];
  const float* __restrict__ p = xyz + base * 3;
  float* sx = reinterpret_cast<float*>(smem + 4 * sizeof(unsigned long long));
  const int n_pad = (n + 3) & ~3;
  float* sy = sx + n_pad;
  float* sz = sy + n_pad;

  const float inf = __builtin_huge_valf();
  // the lane's points in pairs (packed f32 arithmetic: v_pk_add / v_pk_mul round each element
  // like the scalar ops); an odd PPT's last pair carries an empty slot (distance -1)
  constexpr int PH = (PPT + 1) / 2;
  f32x2 X[PH], Y[PH], Z[PH], D[PH];
  float bx0 = inf, bx1 = -inf, by0 = inf, by1 = -inf, bz0 = inf, bz1 = -inf;
  const int i0 = tid * PPT;
  if (n > 0) {  // unconditional loads at a clamped index (block-uniform guard: empty crop)
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int ic = i0 + k < n ? i0 + k : 0;
      X[k >> 1][k & 1] = p[3 * ic + 0];
      Y[k >> 1][k & 1] = p[3 * ic + 1];
      Z[k >> 1][k & 1] = p[3 * ic + 2];
    }
  }
#pragma unroll
  for (int k = 0; k < 2 * PH; ++k) {
    const bool ok = k < PPT && i0 + k < n;
    const float x = ok ? X[k >> 1][k & 1] : 0.f, y = ok ? Y[k >> 1][k & 1] : 0.f, z = ok ? Z[k >> 1][k & 1] : 0.f;
    X[k >> 1][k & 1] = x;
    Y[k >> 1][k & 1] = y;
    Z[k >> 1][k & 1] = z;
    D[k >> 1][k & 1] = ok ? 1e10f : -1.f;  // empty slot: min(-1, d >= 0) keeps it at -1, never selected
    if (ok) {
      sx[i0 + k] = x;
      sy[i0 + k] = y;
      sz[i0 + k] = z;
      bx0 = fminf(bx0, x); bx1 = fmaxf(bx1, x);
      by0 = fminf(by0, y); by1 = fmaxf(by1, y);
      bz0 = fminf(bz0, z); bz1 = fmaxf(bz1, z);
    }
  }
  if (tid < 3) keys[tid] = 0ull;
  fps_zero_tail(out, out_stride, b, np);
  if (n <= 0 || np <= 0) return;  // block-uniform
  const bool lval = i0 < n;
  float bd = lval ? 1e10f : -1.f;  // the lane's max running distance, first reached at k = bk
  int bk = 0;
  __syncthreads();
  int far = start[b];
  float cx = sx[far], cy = sy[far], cz = sz[far];
  unsigned long long wkey = 0ull;  // the wave's best (cached while its lanes skip)
  int64_t* __restrict__ o = out + (int64_t)b * out_stride;
  if (STAMP) t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < np; ++i) {
    if (tid == 0) o[i] = far;
    const float ddx = fmaxf(fmaxf(bx0 - cx, cx - bx1), 0.f);
    const float ddy = fmaxf(fmaxf(by0 - cy, cy - by1), 0.f);
    const float ddz = fmaxf(fmaxf(bz0 - cz, cz - bz1), 0.f);
    const float lb = (ddx * ddx + ddy * ddy) + ddz * ddz;
    // an empty lane's bd = -1 fails the test by itself (its box bound is +inf), so the ballot is the
    // bare compare's mask
    const bool need = TRIM ? !(lb * 0.99999809f >= bd) : lval && !(lb * 0.99999809f >= bd);
    const uint64_t needm = __ballot(need);
    unsigned long long t1 = 0;
    if (STAMP) {
      t1 = __builtin_amdgcn_s_memtime();
      st_box += t1 - t0;
    }
    if (needm) {  // wave-uniform
      if (STAMP) ++st_nupd;
      if (need) {
        const f32x2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
        for (int j = 0; j < PH; ++j) {
          const f32x2 dx = X[j] - c2x;
          const f32x2 dy = Y[j] - c2y;
          const f32x2 dz = Z[j] - c2z;
          const f32x2 d = (dx * dx + dy * dy) + dz * dz;  // no contraction (TU flag)
          // plain v_min_f32: fminf would canonicalise the loop-carried D first (one v_max per point;
          // both operands are finite here, so the result is fminf's)
          D[j][0] = vmin_f32(D[j][0], d[0]);
          D[j][1] = vmin_f32(D[j][1], d[1]);
        }
        float m = D[0][0];
#pragma unroll
        for (int k = 1; k < PPT; ++k) m = fmaxf(m, D[k >> 1][k & 1]);
        bd = m;
        if (!TRIM) {  // (development A/B: the round-5 chain, PK_FPS_TRIM=0)
          int kk = PPT - 1;
#pragma unroll
          for (int k = PPT - 2; k >= 0; --k) kk = D[k >> 1][k & 1] == m ? k : kk;
          bk = kk;
        }
      }
      uint32_t wbits, widx;
      if (!TRIM) {
        const bool valid = bd >= 0.f;
        const uint32_t bits = valid ? pk::f32_bits(bd) : 0u;
        wbits = pk::wave_max_u32_s(bits);
        const uint64_t at = __ballot(valid && bits == wbits);
        widx = pk::readlane((uint32_t)(i0 + bk), __ffsll((unsigned long long)at) - 1);
      } else {
        // the argmax with the whole wave active (a lane that skipped finds its unchanged bk again),
        // so the compiler can place its compare -> select wait states under the wave reduction's DPP
        // chain (plain code: the compiler pads every hazard; an inline-asm select would not be)
        {
          int kk = PPT - 1;
#pragma unroll
          for (int k = PPT - 2; k >= 0; --k) kk = D[k >> 1][k & 1] == bd ? k : kk;  // first k at the max
          bk = kk;
        }
        // signed max of the distance bits: an empty lane's -1.0f is negative and never the max; the
        // valid lanes are a prefix of the wave, so the first lane at the max is a valid one
        const int bits = __float_as_int(bd);
        wbits = (uint32_t)pk::wave_max_i32_s(bits);
        const uint64_t at = __builtin_amdgcn_uicmp((uint32_t)bits, wbits, 32 /* EQ */);
        widx = pk::readlane((uint32_t)(i0 + bk), __ffsll((unsigned long long)at) - 1);
      }
      wkey = ((unsigned long long)wbits << 32) | (unsigned long long)(0xffffffffu - widx);
    }
    unsigned long long t2 = 0;
    if (STAMP) {
      t2 = __builtin_amdgcn_s_memtime();
      st_upd += t2 - t1;
    }
    if (lane == 0 && wkey != 0ull) atomicMax(&keys[i % 3], wkey);
    if (tid == 0) keys[(i + 1) % 3] = 0ull;  // last read after barrier i - 2: every wave is past it
    __syncthreads();
    if (STAMP) {
      t0 = __builtin_amdgcn_s_memtime();
      st_bar += t0 - t2;
    }
    const unsigned long long key = keys[i % 3];
    far = (int)(0xffffffffu - (uint32_t)(key & 0xffffffffull));
    cx = sx[far];
    cy = sy[far];
    cz = sz[far];
  }
#ifdef PK_DEVBUILD
  if (STAMP && lane == 0 && b < 64) {
    unsigned long long* g = g_fps_stamps + ((size_t)b * 16 + pk::wave_id()) * 8;
    g[0] = st_box;
    g[1] = st_upd;
    g[2] = st_bar;
    g[3] = st_nupd;
    g[4] = (unsigned long long)np;
  }
#endif
}

template <int NT, int PPT, bool STAMP = false>
int launch_fps_flat(const float* xyz, const int64_t* offsets, const int32_t* start, const int32_t* npoint,
                    int64_t* out, int out_stride, int B, int nmax, hipStream_t s) {
  const int n_pad = (nmax + 3) & ~3;
  const size_t lds = 4 * sizeof(unsigned long long) + 3 * (size_t)n_pad * sizeof(float);
#ifdef PK_DEVBUILD
  static const bool untrimmed = getenv("PK_FPS_TRIM") && atoi(getenv("PK_FPS_TRIM")) == 0;
  if (untrimmed) {
    hipLaunchKernelGGL((fps_flat_kernel<NT, PPT, STAMP, false>), dim3(B), dim3(NT), lds, s, xyz, offsets, start,
                       npoint, out, out_stride, pk::side_prio());
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
#endif
  hipLaunchKernelGGL((fps_flat_kernel<NT, PPT, STAMP>), dim3(B), dim3(NT), lds, s, xyz, offsets, start, npoint, out,
                     out_stride, pk::side_prio());
  PK_CHECK_LAUNCH();
  return PK_OK;
}

template <int NT, int PPT>
int launch_fps_lane(const float* xyz, const int64_t* offsets, const int32_t* start, const int32_t* npoint,
                    int64_t* out, int out_stride, int B, hipStream_t s) {
  hipLaunchKernelGGL((fps_lane_kernel<NT, PPT>), dim3(B), dim3(NT), 0, s, xyz, offsets, start, npoint, out,
                     out_stride);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

template <int NT, int PPT>
int launch_fps(const float* xyz, const int64_t* offsets, const int32_t* start,
               const int32_t* npoint, int64_t* out, int out_stride, int B, int nmax,
               hipStream_t s) {
  const size_t slots = 2 * 16 * sizeof(uint2);
  if (nmax <= kFpsMaxLds) {
    const int n_pad = (nmax + 3) & ~3;
    const size_t lds = slots + 3 * (size_t)n_pad * sizeof(float);
    hipLaunchKernelGGL((fps_pruned_kernel<NT, PPT>), dim3(B), dim3(NT), lds, s, xyz, offsets,
                       start, npoint, out, out_stride);
  } else {
    hipLaunchKernelGGL((fps_kernel<NT, PPT, false>), dim3(B), dim3(NT), slots, s, xyz, offsets,
                       start, npoint, out, out_stride);
  }
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// The unpruned kernel at a forced configuration (dev comparisons).
template <int NT, int PPT>
int launch_fps_plain(const float* xyz, const int64_t* offsets, const int32_t* start,
                     const int32_t* npoint, int64_t* out, int out_stride, int B, int nmax,
                     hipStream_t s) {
  const size_t slots = 2 * 16 * sizeof(uint2);
  const int n_pad = (nmax + 3) & ~3;
  const size_t lds = slots + 3 * (size_t)n_pad * sizeof(float);
  if (nmax > kFpsMaxLds) return PK_ERR_ARG;
  hipLaunchKernelGGL((fps_kernel<NT, PPT, true>), dim3(B), dim3(NT), lds, s, xyz, offsets, start,
                     npoint, out, out_stride);
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
  if (pk::diag_skip("fps")) return PK_OK;  // (development diagnostics only: see common.hpp)
  if (pk::diag_twice("fps")) {
    static thread_local bool inner = false;
    if (!inner) {
      inner = true;
      const int rc = pk_fps(xyz, offsets, B, nmax, start, npoint, out, out_stride, stream);
      inner = false;
      if (rc != PK_OK) return rc;
    }
  }
#ifndef PK_FPS_ROUND2  // flat kernel (one LDS atomic per wave per iteration) up to 8192 points
  if (nmax <= 1024) return launch_fps_flat<1024, 1>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (nmax <= 2048) return launch_fps_flat<1024, 2>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (nmax <= 4096) return launch_fps_flat<1024, 4>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (nmax <= 8192) return launch_fps_flat<1024, 8>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  // up to the LDS bound (3 x 13312 floats + the key words = 156 KiB): the bench's 640x480 crops
  // (8-9k points) ran the pruned kernel at 0.78 us per iteration; the flat one measured 0.53 at 1024 threads
  // 10 points per lane up to 10,240 (the bench's synthetic frames: up to 9,289 mask pixels): an
  // updating wave's distance / argmax work scales with the points per lane
  if (nmax <= 10240) return launch_fps_flat<1024, 10>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  if (nmax <= kFpsMaxLds) return launch_fps_flat<1024, 13>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
#endif
#define PK_FPS(NT, PPT) return launch_fps<NT, PPT>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s)
#ifdef PK_DEVBUILD
  // development knob (read once): PK_FPS_NT=256 / 512 runs the pruned kernel with fewer waves per
  // crop above 4096 points (less of each CU held while crop formation overlaps the step)
  static const int fps_nt = getenv("PK_FPS_NT") ? atoi(getenv("PK_FPS_NT")) : 1024;
  if (nmax > 4096 && nmax <= 8192 && fps_nt == 512) PK_FPS(512, 16);
  if (nmax > 4096 && nmax <= 13312 && fps_nt == 512) PK_FPS(512, 26);
  if (nmax > 4096 && nmax <= 8192 && fps_nt == 256) PK_FPS(256, 32);
  if (nmax > 4096 && nmax <= 13312 && fps_nt == 256) PK_FPS(256, 52);
#endif
  // 1024-thread workgroups above 4096 points: measured 0.712 us per FPS step against 0.78
  // (512 threads) and 1.09 (256) on the bench's crops (n <= 6588, profiles/r02_kbench_fps.txt)
  if (nmax <= 1024) PK_FPS(256, 4);
  if (nmax <= 2048) PK_FPS(256, 8);
  if (nmax <= 4096) PK_FPS(256, 16);
#ifdef PK_FPS_LANE_ABOVE_4096  // development variant: per-lane buckets (no LDS point copy) above 4096
  if (nmax <= 8192) return launch_fps_lane<1024, 8>(xyz, offsets, start, npoint, out, out_stride, B, s);
  if (nmax <= 13312) return launch_fps_lane<1024, 13>(xyz, offsets, start, npoint, out, out_stride, B, s);
#endif
  if (nmax <= 8192) PK_FPS(1024, 8);
  if (nmax <= 13312) PK_FPS(1024, 13);
#undef PK_FPS
  // beyond the LDS copy of the pruned kernel: per-lane buckets, points in registers only
  if (nmax <= 16384) return launch_fps_lane<1024, 16>(xyz, offsets, start, npoint, out, out_stride, B, s);
  if (nmax <= 24576) return launch_fps_lane<1024, 24>(xyz, offsets, start, npoint, out, out_stride, B, s);
  if (nmax <= 32768) return launch_fps<1024, 32>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  return PK_ERR_ARG;  // > 32768 points per crop
}

#ifdef PK_DEVBUILD
// Development hook (not part of include/posekern.h): force the block size / points
// per thread, flat with phase stamps (pruned = 6), flat (4), per-lane buckets (3), pruned (1) or plain (0), for tools/kbench.py's sweeps.
extern "C" int pkdev_fps_cfg(const float* xyz, const int64_t* offsets, int B, int nmax,
                             const int32_t* start, const int32_t* npoint, int64_t* out,
                             int out_stride, int nt, int pruned, void* stream) {
  hipStream_t s = pk::as_stream(stream);
  const int ppt = (nmax + nt - 1) / nt;
#define PK_FPS(NT, PPT)                                                                          \
  if (nt == NT && ppt <= PPT)                                                                    \
    return pruned == 6 ? launch_fps_flat<NT, PPT, true>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s) \
           : pruned == 4 ? launch_fps_flat<NT, PPT>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s) \
           : pruned == 3 ? launch_fps_lane<NT, PPT>(xyz, offsets, start, npoint, out, out_stride, B, s) \
           : pruned ? launch_fps<NT, PPT>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s) \
                  : launch_fps_plain<NT, PPT>(xyz, offsets, start, npoint, out, out_stride, B, nmax, s);
  PK_FPS(256, 4) PK_FPS(256, 8) PK_FPS(256, 16) PK_FPS(256, 32)
  PK_FPS(512, 2) PK_FPS(512, 4) PK_FPS(512, 8) PK_FPS(512, 16) PK_FPS(512, 26)
  PK_FPS(1024, 2) PK_FPS(1024, 4) PK_FPS(1024, 8) PK_FPS(1024, 10) PK_FPS(1024, 13)
#undef PK_FPS
  return PK_ERR_ARG;
}
#endif  // PK_DEVBUILD

#ifdef PK_DEVBUILD
extern "C" int pkdev_fps_stamps(unsigned long long* host, int n) {
  if (n > 64 * 16 * 8) n = 64 * 16 * 8;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fps_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif  // PK_DEVBUILD
