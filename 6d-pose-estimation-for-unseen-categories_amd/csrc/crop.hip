// H1 / H2 / H4 — crop formation on the device, stream-ordered, no host round trips.
//
//  pk_backproject   dataset/object.py:73-88 dpt_2_pcld (+ :52-71 erode_seg_mask, :137
//                   `seg == 255`): plus-shaped 3x3 erosion (pixels outside the image do
//                   not erode, cv2's default border), row-major ordered compaction of the
//                   surviving pixels, back-projection in fp64 exactly as numpy evaluates
//                     z32 = f32(depth) / f32(cam_scale)
//                     X = (((u - cx) * f64(z32)) / fx) * 100,  Y likewise,  Z = f64(z32) * 100
//  pk_sor           dataset/object.py:33-50 -> Open3D RemoveStatisticalOutliers(20, 0.3):
//                   brute-force kNN-20 (self included) in fp64, per-point mean of the
//                   sqrt distances summed in ascending order, cloud mean / Bessel std
//                   accumulated in point order, keep 0 < avg < mean + 0.3 std (ordered).
//  pk_gather_transform  pcd[idx0] (object.py:148) + transform(pcd, R, t, inv=True)
//                   (object.py:174, 304-309) -> align_pc f64, plus the f32 copy the model
//                   consumes (object.py:263 `astype(np.float32)`).
//  pk_fps_npoint    object.py:145-147 policy: npoint = int(2000/n * n) when n > 2000
//                   (else n, no FPS), or a fixed npoint (benchmark configs), per crop.
//  pk_segment_scan / pk_offsets_from_counts  offsets of packed outputs.
#include <algorithm>
#include <climits>

#include "common.hpp"

namespace {

// sqrt rounded to nearest, independent of how the compiler lowers sqrt(double):
// Tuckerman's test with exact FMA residual signs — s = RN(sqrt(x)) iff
// s * pred(s) < x <= s * succ(s).
__device__ __forceinline__ double sqrt_rn(double x) {
  if (!(x > 0.0) || x == __builtin_huge_val()) return sqrt(x);
  double s = sqrt(x);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const long long bits = __double_as_longlong(s);  // s > 0 and finite
    const double dn = __longlong_as_double(bits - 1);
    const double up = __longlong_as_double(bits + 1);
    if (fma(s, dn, -x) >= 0.0) {
      s = dn;
    } else if (fma(s, up, -x) < 0.0) {
      s = up;
    }
  }
  return s;
}

__device__ __forceinline__ bool eroded(const uint8_t* __restrict__ m, int H, int W, int v, int u) {
  if (m[(int64_t)v * W + u] != 255) return false;
  if (v > 0 && m[(int64_t)(v - 1) * W + u] != 255) return false;
  if (v + 1 < H && m[(int64_t)(v + 1) * W + u] != 255) return false;
  if (u > 0 && m[(int64_t)v * W + u - 1] != 255) return false;
  if (u + 1 < W && m[(int64_t)v * W + u + 1] != 255) return false;
  return true;
}

// grid (H, F), block 256: count eroded pixels per image row.
__global__ __launch_bounds__(256) void bp_count_kernel(const uint8_t* __restrict__ mask, int H, int W,
                                                       int32_t* __restrict__ rowcnt) {
  const int v = blockIdx.x, f = blockIdx.y;
  const uint8_t* m = mask + (int64_t)f * H * W;
  int c = 0;
  for (int u = threadIdx.x; u < W; u += blockDim.x) c += eroded(m, H, W, v, u) ? 1 : 0;
  c = pk::wave_sum_i32_s(c);
  __shared__ int ws[4];
  if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) rowcnt[(int64_t)f * H + v] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Generic per-segment exclusive scan of int32 counts -> int64 offsets (+ totals).
// grid (S), block 1024; segment s covers cnt[s*n .. s*n+n).
__global__ __launch_bounds__(1024) void seg_scan_kernel(const int32_t* __restrict__ cnt, int n,
                                                        int64_t* __restrict__ off,
                                                        int64_t* __restrict__ total) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry_s;
  const int s = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const int64_t v = i < n ? (int64_t)cnt[(int64_t)s * n + i] : 0;
    const int64_t inc = pk::wave_inclusive_scan_i64(v);
    if (pk::lane_id() == 63) wsum[pk::wave_id()] = inc;
    __syncthreads();
    int64_t pre = carry_s;
    for (int w = 0; w < pk::wave_id(); ++w) pre += wsum[w];
    if (i < n) off[(int64_t)s * n + i] = pre + inc - v;
    __syncthreads();
    if (tid == 1023) carry_s = pre + inc;
    __syncthreads();
  }
  if (tid == 0 && total) total[s] = carry_s;
}

// off[0] = 0, off[b+1] = off[b] + counts[b] (one thread; B is a batch size).
__global__ void offsets_kernel(const int64_t* __restrict__ counts, int B, int64_t* __restrict__ off) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t acc = 0;
  off[0] = 0;
  for (int b = 0; b < B; ++b) {
    acc += counts[b];
    off[b + 1] = acc;
  }
}

// grid (H, F), block 64 (one wave walks the row in 64-pixel chunks, ordered by ballot).
__global__ __launch_bounds__(64) void bp_write_kernel(
    const uint16_t* __restrict__ depth, const uint8_t* __restrict__ mask, int H, int W,
    const double* __restrict__ K, const float* __restrict__ cam_scale,
    const int64_t* __restrict__ rowoff, const int64_t* __restrict__ frame_off, double* __restrict__ out,
    int64_t cap, int32_t* __restrict__ pix, int32_t* __restrict__ idxmap) {
  const int v = blockIdx.x, f = blockIdx.y;
  const uint8_t* m = mask + (int64_t)f * H * W;
  const uint16_t* d = depth + (int64_t)f * H * W;
  const double fx = K[f * 9 + 0], cx = K[f * 9 + 2], fy = K[f * 9 + 4], cy = K[f * 9 + 5];
  const float cs = cam_scale[f];
  int64_t o = frame_off[f] + rowoff[(int64_t)f * H + v];
  const int lane = threadIdx.x;
  for (int u0 = 0; u0 < W; u0 += 64) {
    const int u = u0 + lane;
    const bool keep = u < W && eroded(m, H, W, v, u);
    const uint64_t bal = __ballot(keep);
    if (idxmap != nullptr && u < W)
      idxmap[(int64_t)f * H * W + (int64_t)v * W + u] =
          keep ? (int32_t)(o - frame_off[f] + __popcll(bal & ((1ull << lane) - 1ull))) : -1;
    if (keep) {
      const int64_t w = o + __popcll(bal & ((1ull << lane) - 1ull));
      if (pix != nullptr && w < cap) pix[w] = v * W + u;
      if (w < cap) {
        const float z32 = (float)d[(int64_t)v * W + u] / cs;  // f32 / f32, correctly rounded
        const double z = (double)z32;
        const double X = (((double)u - cx) * z) / fx;
        const double Y = (((double)v - cy) * z) / fy;
        out[3 * w + 0] = X * 100.0;
        out[3 * w + 1] = Y * 100.0;
        out[3 * w + 2] = z * 100.0;
      }
    }
    o += __popcll(bal);
  }
}

// ---- Round 5: one wave per image row, 16 consecutive pixels per lane (64 x 16 = 1024-pixel
// segments), the erosion of the lane's pixels as bit operations on three rows' is-255 masks.
// Every mask / depth load of a segment is issued at once (16-B vectors when the rows are
// 16-B aligned): round 4's kernels walked a row in 64-pixel chunks, five dependent byte loads
// each, one block per row (15,360 blocks of one wave at 640 x 480 x 32).
constexpr int kBpPx = 16;
struct BpRow {  // bit c: pixel u0 + c of the segment
  uint32_t keep;  // eroded (255 with every in-image 4-neighbour 255)
  uint32_t valid; // u0 + c < W
};

__device__ __forceinline__ uint32_t bp_is255_16(const uint8_t* __restrict__ row, int u0, int W, bool vec) {
  uint32_t m = 0;
  if (vec && u0 + kBpPx <= W) {
    const uint4 q = *reinterpret_cast<const uint4*>(row + u0);
    const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int c = 0; c < kBpPx; ++c) m |= (((w4[c >> 2] >> (8 * (c & 3))) & 0xFFu) == 0xFFu ? 1u : 0u) << c;
  } else {
    uint8_t b[kBpPx];
#pragma unroll
    for (int c = 0; c < kBpPx; ++c) b[c] = row[u0 + c < W ? u0 + c : 0];  // unconditional, masked below
#pragma unroll
    for (int c = 0; c < kBpPx; ++c) m |= (u0 + c < W && b[c] == 255 ? 1u : 0u) << c;
  }
  return m;
}

__device__ __forceinline__ BpRow bp_erode16(const uint8_t* __restrict__ m, int H, int W, int v, int u0, bool vec) {
  BpRow r;
  r.valid = u0 >= W ? 0u : (W - u0 >= kBpPx ? 0xFFFFu : ((1u << (W - u0)) - 1u));
  if (u0 >= W) {
    r.keep = 0;
    return r;
  }
  const uint8_t* row = m + (int64_t)v * W;
  const uint32_t c = bp_is255_16(row, u0, W, vec);
  const uint32_t up = v > 0 ? bp_is255_16(row - W, u0, W, vec) : 0xFFFFu;
  const uint32_t dn = v + 1 < H ? bp_is255_16(row + W, u0, W, vec) : 0xFFFFu;
  const uint32_t lb = u0 > 0 ? (row[u0 - 1] == 255 ? 1u : 0u) : 1u;  // left neighbour of pixel 0
  const int ur = u0 + kBpPx;                                          // right neighbour of pixel 15
  const uint32_t rb = ur < W ? (row[ur] == 255 ? 1u : 0u) : 1u;
  // pixel W - 1 (inside the segment) has no right neighbour: its bit of c >> 1 is forced
  const uint32_t edge = (W - 1 - u0 >= 0 && W - 1 - u0 < kBpPx) ? (1u << (W - 1 - u0)) : 0u;
  const uint32_t left = (c << 1) | lb, right = (c >> 1) | (rb << (kBpPx - 1)) | edge;
  r.keep = c & up & dn & left & right & r.valid;
  return r;
}

// grid (ceil(H / 4), F), block 256: wave w counts row 4 blockIdx.x + w.
__global__ __launch_bounds__(256) void bp_count16_kernel(const uint8_t* __restrict__ mask, int H, int W,
                                                         int32_t* __restrict__ rowcnt) {
  const int v = blockIdx.x * 4 + pk::wave_id(), f = blockIdx.y, lane = pk::lane_id();
  if (v >= H) return;
  const uint8_t* m = mask + (int64_t)f * H * W;
  const bool vec = (W % 16) == 0 && (((uintptr_t)mask) & 15) == 0;
  int c = 0;
  for (int s0 = 0; s0 < W; s0 += 64 * kBpPx) c += __popc(bp_erode16(m, H, W, v, s0 + kBpPx * lane, vec).keep);
  c = pk::wave_sum_i32_s(c);
  if (lane == 0) rowcnt[(int64_t)f * H + v] = c;
}

// grid (ceil(H / 4), F), block 256: wave w writes row 4 blockIdx.x + w in pixel order.
__global__ __launch_bounds__(256) void bp_write16_kernel(
    const uint16_t* __restrict__ depth, const uint8_t* __restrict__ mask, int H, int W,
    const double* __restrict__ K, const float* __restrict__ cam_scale,
    const int64_t* __restrict__ rowoff, const int64_t* __restrict__ count, int64_t* __restrict__ frame_off,
    double* __restrict__ out, int64_t cap, int32_t* __restrict__ pix, int32_t* __restrict__ idxmap) {
  const int v = blockIdx.x * 4 + pk::wave_id(), f = blockIdx.y, lane = pk::lane_id();
  if (v >= H) return;
  const uint8_t* m = mask + (int64_t)f * H * W;
  const uint16_t* d = depth + (int64_t)f * H * W + (int64_t)v * W;
  const bool vec = (W % 16) == 0 && (((uintptr_t)mask) & 15) == 0;
  const double fx = K[f * 9 + 0], cx = K[f * 9 + 2], fy = K[f * 9 + 4], cy = K[f * 9 + 5];
  const float cs = cam_scale[f];
  // the frame's base = sum of the earlier frames' counts (round 5: no crop-offset launch);
  // block (0, 0)'s first wave also writes the offsets array for the later stages
  int64_t fo = 0;
  for (int q0 = 0; q0 < f; q0 += 64) fo += q0 + lane < f ? count[q0 + lane] : 0;
  fo = pk::wave_sum_i64(fo);
  if (blockIdx.x == 0 && f == 0 && pk::wave_id() == 0) {
    const int F = gridDim.y;
    int64_t carry = 0;
    for (int q0 = 0; q0 <= F; q0 += 64) {
      const int q = q0 + lane;
      const int64_t cv = q < F ? count[q] : 0;
      const int64_t inc = pk::wave_inclusive_scan_i64(cv);
      if (q <= F) frame_off[q] = carry + inc - cv;
      carry += __shfl(inc, 63);
    }
  }
  int64_t o = fo + rowoff[(int64_t)f * H + v];
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int s0 = 0; s0 < W; s0 += 64 * kBpPx) {
    const BpRow r = bp_erode16(m, H, W, v, s0 + kBpPx * lane, vec);
    // the stores go pixel-major (pass j: pixels s0 + 64 j + lane, consecutive lanes writing
    // consecutive points and index-map entries); each pass takes its keep bits from the lane
    // that eroded them (lane 4 j + lane / 16, bit lane % 16)
    uint16_t dz[kBpPx];
    uint32_t kp = 0;  // bit j: pass j's pixel kept (all shuffles issued before the passes)
#pragma unroll
    for (int j = 0; j < kBpPx; ++j) {
      const int u = s0 + 64 * j + lane;
      dz[j] = d[u < W ? u : 0];
      kp |= (u < W ? (((uint32_t)__shfl((int)r.keep, 4 * j + (lane >> 4)) >> (lane & 15)) & 1u) : 0u) << j;
    }
#pragma unroll
    for (int j = 0; j < kBpPx; ++j) {
      const int u = s0 + 64 * j + lane;
      const bool keep = (kp >> j) & 1u;
      const uint64_t bal = __ballot(keep);
      const int64_t w = o + __popcll(bal & lt);
      if (idxmap != nullptr && u < W) idxmap[(int64_t)f * H * W + (int64_t)v * W + u] = keep ? (int32_t)(w - fo) : -1;
      if (keep) {
        if (pix != nullptr && w < cap) pix[w] = v * W + u;
        if (w < cap) {
          const float z32 = (float)dz[j] / cs;  // f32 / f32, correctly rounded
          const double z = (double)z32;
          const double X = (((double)u - cx) * z) / fx;
          const double Y = (((double)v - cy) * z) / fy;
          out[3 * w + 0] = X * 100.0;
          out[3 * w + 1] = Y * 100.0;
          out[3 * w + 2] = z * 100.0;
        }
      }
      o += __popcll(bal);
      if (s0 + 64 * (j + 1) >= W) break;  // (wave-uniform) past the row
    }
  }
}

// ---------------------------------------------------------------- SOR (H2)
constexpr int kKnn = 20;
constexpr int kSorThreads = 256;
constexpr int kSorTile = 1024;

__device__ __forceinline__ void topk_insert(double (&best)[kKnn], double v) {
#pragma unroll
  for (int k = 0; k < kKnn; ++k) {  // bubble v into the sorted list
    const double lo = fmin(best[k], v), hi = fmax(best[k], v);
    best[k] = lo;
    v = hi;
  }
}

__device__ __forceinline__ double sqdist(double ax, double ay, double az, const double* b) {
  const double dx = ax - b[0], dy = ay - b[1], dz = az - b[2];
  return (dx * dx + dy * dy) + dz * dz;  // nanoflann L2: ((dx²+dy²)+dz²)
}

// grid (ceil(nmax/256), B), block 256: one query point per thread.
//  pass 1 (pixel window, when pix/idxmap are given): exact distances to the points of the
//         5x5 pixel neighbourhood (9x9, 17x17 where that holds fewer than knn points, near
//         the mask border); if >= knn of them exist, T = their knn-th smallest
//         squared distance bounds the true knn-th neighbour distance (>= knn points lie
//         within T). Otherwise T = +inf.
//  pass 2a (K given, T finite, Z_q > r = sqrt(T)): every crop point within r of the query
//         lies in the pixel box |du| <= fx r (1 + tx) / Z_q, |dv| <= fy r (1 + ty) / Z_q
//         (tx = max|u - cx| / fx over the image), +1 px slack for the
//         rounding of X/Z vs (u - cx)/fx. That box is scanned exactly in fp64.
//  pass 2b (otherwise, or when the box exceeds kSorMaxBox pixels): every point of the
//         crop (LDS tiles of fp32 coordinates centred on the crop's first point) is
//         screened with an fp32 distance against T + margin, where margin = 2^-19 (T +
//         (|a| + |b|)^2) bounds the fp32 error; survivors are
//         re-evaluated exactly in fp64 and inserted if <= T.
// The kept set is a superset of the true knn nearest (ties included), so the sorted
// top-knn values are exactly those of a full brute-force search.
constexpr int kSorMaxBox = 1024;
#ifndef PK_SOR_BATCH
#define PK_SOR_BATCH 4
#endif
#ifndef PK_SOR_MINW
#define PK_SOR_MINW 4
#endif
constexpr int kSorBatch = PK_SOR_BATCH;  // pixels of a window row gathered together (loads in flight at once)

// distances from the query to the points of pixels uu .. min(uu + 7, u1) of an index-map row;
// bit t of the result: pixel uu + t holds a point (s[t] valid). All index loads, then all
// coordinate loads, are issued before the first use (memory-level parallelism).
__device__ __forceinline__ int sor_gather(const int32_t* __restrict__ row, int uu, int u1,
                                          const double* __restrict__ p, double q0, double q1, double q2,
                                          double (&s)[kSorBatch]) {
  int j[kSorBatch];
#pragma unroll
  for (int t = 0; t < kSorBatch; ++t) {  // unconditional at a clamped pixel (no branch + wait per load)
    const int32_t v = row[uu + t <= u1 ? uu + t : uu];
    j[t] = uu + t <= u1 ? v : -1;
  }
  double c[kSorBatch][3];
#pragma unroll
  for (int t = 0; t < kSorBatch; ++t) {
    const double* pj = p + 3 * (j[t] >= 0 ? j[t] : 0);
    c[t][0] = pj[0];
    c[t][1] = pj[1];
    c[t][2] = pj[2];
  }
  int m = 0;
#pragma unroll
  for (int t = 0; t < kSorBatch; ++t) {
    s[t] = sqdist(q0, q1, q2, c[t]);
    m |= (j[t] >= 0 ? 1 : 0) << t;
  }
  return m;
}


// grid (tiles x B): workgroup = (crop, 256-query tile), crops interleaved; a persistent grid
// (fewer workgroups looping over the items) measured slower with no gain in overlap.

__global__ __launch_bounds__(kSorThreads, PK_SOR_MINW) void sor_knn_kernel(const double* __restrict__ xyz,
                                                                 const int64_t* __restrict__ off, int knn,
                                                                 const int32_t* __restrict__ pix,
                                                                 const int32_t* __restrict__ idxmap, int H, int W,
                                                                 const double* __restrict__ Kmat, int tiles, int B,
                                                                 double* __restrict__ avg, int prio) {
  pk::set_wave_prio(prio);
  __shared__ float4 tile[kSorTile];
  {
  const int item = blockIdx.x;
  const int b = item % B, bx = item / B;
  const int64_t base = off[b];
  const int n = (int)(off[b + 1] - base);
  const int i = bx * kSorThreads + threadIdx.x;
  if (bx * kSorThreads >= n) return;  // workgroup-uniform
  const bool act = i < n;
  const double* p = xyz + base * 3;
  const double ox = p[0], oy = p[1], oz = p[2];
  double q0 = 0.0, q1 = 0.0, q2 = 0.0;
  if (act) {
    q0 = p[3 * i];
    q1 = p[3 * i + 1];
    q2 = p[3 * i + 2];
  }
  const int kk = knn < n ? knn : n;
  double best[kKnn];
#pragma unroll
  for (int k = 0; k < kKnn; ++k) best[k] = __builtin_huge_val();
  double T = __builtin_huge_val();
  bool done = false;
  if (act && pix != nullptr && idxmap != nullptr) {
    const int pp = pix[base + i];
    const int v = pp / W, u = pp % W;
    const int32_t* im = idxmap + (int64_t)b * H * W;
    int found = 0, Rw = -1;
    for (int R = 2; R <= 8; R *= 2) {  // 5x5, then 9x9, 17x17 near the mask border
      found = 0;
#pragma unroll
      for (int k = 0; k < kKnn; ++k) best[k] = __builtin_huge_val();
      for (int vv = max(v - R, 0); vv <= min(v + R, H - 1); ++vv) {
        const int32_t* row = im + vv * W;
        const int u1 = min(u + R, W - 1);
        for (int uu = max(u - R, 0); uu <= u1; uu += kSorBatch) {
          double s[kSorBatch];
          const int m = sor_gather(row, uu, u1, p, q0, q1, q2, s);
#pragma unroll
          for (int t = 0; t < kSorBatch; ++t)
            if ((m >> t) & 1) topk_insert(best, s[t]);
          found += __builtin_popcount(m);
        }
      }
      if (found >= kk) {
        Rw = R;
        break;
      }
    }
    if (Rw >= 0) {
#pragma unroll
      for (int k = 0; k < kKnn; ++k)
        if (k == kk - 1) T = best[k];  // static register index (no scratch)
    }
    // pass 2a: best keeps the window's kk smallest (all <= T, real points), and the box scan
    // adds the box pixels outside that window: the kk smallest of window + box are exact
    bool box = false;
    int u0 = 0, u1 = -1, v0 = 0, v1 = -1;
    if (Kmat != nullptr && T < __builtin_huge_val()) {
      const double* Kb = Kmat + 9 * b;
      const double fx = Kb[0], cx = Kb[2], fy = Kb[4], cy = Kb[5];
      const double r = sqrt(T) * (1.0 + 1e-9) + 1e-300;
      if (fx > 0.0 && fy > 0.0 && q2 > r) {
        // a candidate c within r of q: |X_q/Z_q - X_c/Z_c| <= (r/Z_q) sqrt(1 + t_c^2) (Cauchy-
        // Schwarz on (X_q - X_c) + t_c (Z_c - Z_q)), with |t_c| <= the image bound tx and
        // |t_c| <= (|t_q| + rho) / (1 - rho), rho = r / Z_q (SOR camera box)
        const double rho = r / q2;
        const double tx = fmin(fmax(fabs(cx), fabs((double)(W - 1) - cx)) / fx, (fabs(q0 / q2) + rho) / (1.0 - rho));
        const double ty = fmin(fmax(fabs(cy), fabs((double)(H - 1) - cy)) / fy, (fabs(q1 / q2) + rho) / (1.0 - rho));
        const double bu = fx * rho * sqrt(1.0 + tx * tx), bv = fy * rho * sqrt(1.0 + ty * ty);
        if (bu < 64.0 && bv < 64.0) {
          const int ru = (int)ceil(bu * (1.0 + 1e-9)) + 1, rv = (int)ceil(bv * (1.0 + 1e-9)) + 1;
          if ((2 * ru + 1) * (2 * rv + 1) <= kSorMaxBox) {
            box = true;
            v0 = max(v - rv, 0);
            v1 = min(v + rv, H - 1);
            u0 = max(u - ru, 0);
            u1 = min(u + ru, W - 1);
          }
        }
      }
    }
    if (box) {
      for (int vv = v0; vv <= v1; ++vv) {
        const int32_t* row = im + vv * W;
        const bool in_w = vv >= v - Rw && vv <= v + Rw;  // this row's window pixels are in best
        for (int seg = 0; seg < 2; ++seg) {
          const int a = in_w ? (seg == 0 ? u0 : max(u0, u + Rw + 1)) : (seg == 0 ? u0 : 1);
          const int c = in_w ? (seg == 0 ? min(u1, u - Rw - 1) : u1) : (seg == 0 ? u1 : 0);
          for (int uu = a; uu <= c; uu += kSorBatch) {
            double s[kSorBatch];
            const int m = sor_gather(row, uu, c, p, q0, q1, q2, s);
#pragma unroll
            for (int t = 0; t < kSorBatch; ++t)
              if (((m >> t) & 1) && s[t] <= T && s[t] < best[kKnn - 1]) topk_insert(best, s[t]);
          }
        }
      }
      done = true;
    } else {
#pragma unroll
      for (int k = 0; k < kKnn; ++k) best[k] = __builtin_huge_val();
    }
  }
  if (__syncthreads_or(act && !done)) {
    const float qx = (float)(q0 - ox), qy = (float)(q1 - oy), qz = (float)(q2 - oz);
    const float qa = fmaxf(fabsf(qx), fmaxf(fabsf(qy), fabsf(qz)));
    const float Tf = T == __builtin_huge_val() ? __builtin_huge_valf() : (float)T;
    for (int t0 = 0; t0 < n; t0 += kSorTile) {
      const int tn = min(kSorTile, n - t0);
      __syncthreads();
      for (int e = threadIdx.x; e < tn; e += kSorThreads) {
        const double* c = p + 3 * (t0 + e);
        const float cx = (float)(c[0] - ox), cy = (float)(c[1] - oy), cz = (float)(c[2] - oz);
        tile[e] = make_float4(cx, cy, cz, fmaxf(fabsf(cx), fmaxf(fabsf(cy), fabsf(cz))));
      }
      __syncthreads();
      if (act && !done) {
        for (int e = 0; e < tn; ++e) {
          const float4 c = tile[e];
          const float dx = qx - c.x, dy = qy - c.y, dz = qz - c.z;
          const float d32 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
          const float sa = qa + c.w;
          const float lim = fmaf(1.9073486e-6f, fmaf(sa, sa, Tf), Tf);  // T + 2^-19 (T + S^2)
          if (d32 <= lim) {
            const double s = sqdist(q0, q1, q2, p + 3 * (t0 + e));
            if (s <= T && s < best[kKnn - 1]) topk_insert(best, s);
          }
        }
      }
    }
  }
  if (act) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < kKnn; ++k)
      if (k < kk) acc = acc + sqrt_rn(best[k]);
    avg[base + i] = kk > 0 ? acc / (double)kk : -1.0;
  }
  }
}

// One block per crop: cloud mean over avg > 0, then the Bessel std, accumulated in point
// order exactly like std::accumulate / std::inner_product: s = s + t_k, k = 0 .. n-1, IEEE
// double round-to-nearest-even at every step. The terms are >= 0 (masked values, squared
// deviations), so the running sum only grows, and while it stays in one binade
// [2^(e-1), 2^e) (ulp U = 2^(e-53), s = S U with the integer S in [2^52, 2^53)) one step is
//   s + t = (S + r) U rounded to an integer multiple of U,  r = t / U = q + f (q integer):
//   = (S + q + [f > 1/2]) U   unless f == 1/2 exactly (a tie: the even neighbour, which
//   depends on S's parity) or the result leaves the binade (rounded at 2U).
// So a block takes 8192 terms at a time: per term m = q + [f > 1/2] (int64), an exclusive
// scan gives every term's S before it, and the first term that ties, is >= s, or would reach
// 2^53 is a break: s = (S + P) U exactly up to it, then that one term is added by the FPU
// (the true sequential step) and the next round restarts after it. Breaks happen at binade
// crossings (~log2 n of them: the first 1024 terms are added sequentially from LDS, where most
// crossings are) and at exact ties, so a crop takes a handful of rounds instead of n
// dependent fp64 additions.
constexpr int kStatThreads = 1024;
constexpr int kSeqPer = 8;     // terms per thread per round
constexpr int kSeqWarm = 1024;  // first terms added one by one (one per thread loaded into LDS)

struct SeqShared {
  double s;
  int k;
  int brk;
  int64_t part[kStatThreads / 64];
  double s_next;
  double warm[kSeqWarm];  // the first terms, loaded by all threads at once
};

template <class F>
__device__ double seq_sum_exact(F term, int n, SeqShared& sh) {
  const int tid = threadIdx.x, lane = pk::lane_id(), w = pk::wave_id();
  // the first terms one by one (same order) from LDS: every thread loads one, so the warm-up
  // costs one memory round trip (round 4's thread 0 waited for 16 batches of 16 loads)
  const int m = min(n, kSeqWarm);
  if (tid < m) sh.warm[tid] = term(tid);
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int k = 0; k < m; ++k) s = s + sh.warm[k];
    sh.s = s;
    sh.k = m;
  }
  __syncthreads();
  while (true) {
    const double s = sh.s;
    const int k = sh.k;
    if (k >= n) break;  // block-uniform
    __syncthreads();    // everyone has read sh before it changes
    int e = 0;
    (void)frexp(s, &e);  // s in [2^(e-1), 2^e) (s == 0: every term breaks, the FPU adds it)
    const int64_t S = s > 0.0 ? (int64_t)ldexp(s, 53 - e) : 0;
    const int64_t kTop = (int64_t)1 << 53;
    const int j0 = k + tid * kSeqPer;
    int64_t mv[kSeqPer];
    bool bad[kSeqPer];
    int64_t tot = 0;
    double tv[kSeqPer];  // the chunk's terms, unconditionally at clamped indices (k < n is valid)
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) tv[i] = term(j0 + i < n ? j0 + i : k);
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
      const int j = j0 + i;
      mv[i] = 0;
      bad[i] = false;
      if (j < n) {
        const double t = tv[i];
        const double r = ldexp(t, 53 - e);
        if (s == 0.0) {  // 0 + t: exact, but the binade is unknown; zeros leave s at 0
          bad[i] = t != 0.0;
        } else if (!(r < 9007199254740992.0)) {  // t >= s (or inf / nan): the FPU step
          bad[i] = true;
        } else {
          const double q = floor(r), f = r - q;
          bad[i] = f == 0.5;
          mv[i] = (int64_t)q + (f > 0.5 ? 1 : 0);
        }
      }
      tot += mv[i];
    }
    // exclusive scan of the per-thread totals (clamped: a total >= 2^52 already forces a break)
    const int64_t tc = tot < ((int64_t)1 << 52) ? tot : ((int64_t)1 << 52);
    const int64_t inc = pk::wave_inclusive_scan_i64(tc);
    if (lane == 63) sh.part[w] = inc;
    if (tid == 0) sh.brk = INT_MAX;
    __syncthreads();
    int64_t base = inc - tc;
    for (int q = 0; q < w; ++q) base += sh.part[q];
    int64_t P = base;
    int mybrk = INT_MAX;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
      if (j0 + i < n && mybrk == INT_MAX && (bad[i] || S + P + mv[i] >= kTop)) mybrk = j0 + i;
      P += mv[i];
    }
    if (mybrk != INT_MAX) atomicMin(&sh.brk, mybrk);
    __syncthreads();
    const int jb = sh.brk;
    const int kend = min(k + kStatThreads * kSeqPer, n);
    // the thread owning the break (or the chunk's last term) publishes the new state
    if (jb != INT_MAX) {
      if (jb >= j0 && jb < j0 + kSeqPer) {
        int64_t Pb = base;
#pragma unroll
        for (int i = 0; i < kSeqPer; ++i)
          if (j0 + i < jb) Pb += mv[i];
        const double before = s > 0.0 ? ldexp((double)(S + Pb), e - 53) : 0.0;  // exact (S + Pb < 2^53)
        sh.s = before + term(jb);  // the sequential FPU step
        sh.k = jb + 1;
      }
    } else if (kend - 1 >= j0 && kend - 1 < j0 + kSeqPer) {
      sh.s = ldexp((double)(S + P), e - 53);
      sh.k = kend;
    }
    __syncthreads();
  }
  return sh.s;
}

__global__ __launch_bounds__(kStatThreads) void sor_stats_kernel(const double* __restrict__ avg,
                                                                 const int64_t* __restrict__ off,
                                                                 double std_ratio, double* __restrict__ thr,
                                                                 int prio) {
  pk::set_wave_prio(prio);
  __shared__ SeqShared sh;
  const int b = blockIdx.x;
  const int64_t base = off[b];
  const int n = (int)(off[b + 1] - base);
  if (n <= 0) {
    if (threadIdx.x == 0) thr[b] = -1.0;
    return;
  }
  const double* __restrict__ a = avg + base;
  const double sum = seq_sum_exact([&](int j) { const double v = a[j]; return v > 0 ? v : 0.0; }, n, sh);
  const double mean = sum / (double)n;
  __syncthreads();
  const double ss = seq_sum_exact(
      [&](int j) {
        const double v = a[j];
        return v > 0 ? (v - mean) * (v - mean) : 0.0;
      },
      n, sh);
  if (threadIdx.x == 0) {
    const double sd = n > 1 ? sqrt_rn(ss / (double)(n - 1)) : __builtin_nan("");
    thr[b] = mean + std_ratio * sd;
  }
}

// development entry (tests): out[0] = the ordered sum of v[0..n) (terms >= 0) by seq_sum_exact
__global__ __launch_bounds__(kStatThreads) void seq_sum_dev_kernel(const double* __restrict__ v, int n,
                                                                   double* __restrict__ out) {
  __shared__ SeqShared sh;
  const double r = seq_sum_exact([&](int j) { return v[j]; }, n, sh);
  if (threadIdx.x == 0) out[0] = r;
}

// grid (ceil(nmax/1024), B) block 1024: per-chunk keep counts.
__global__ __launch_bounds__(1024) void sor_count_kernel(const double* __restrict__ avg,
                                                         const int64_t* __restrict__ off,
                                                         const double* __restrict__ thr, int nchunk,
                                                         int32_t* __restrict__ ccount) {
  const int b = blockIdx.y;
  const int64_t base = off[b];
  const int n = (int)(off[b + 1] - base);
  const int i = blockIdx.x * 1024 + threadIdx.x;
  const double t = thr[b];
  bool keep = false;
  if (i < n) {
    const double a = avg[base + i];
    keep = a > 0 && a < t;
  }
  int c = __popcll(__ballot(keep));
  __shared__ int ws[16];
  if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < 16; ++w) s += ws[w];
    ccount[(int64_t)b * nchunk + blockIdx.x] = s;
  }
}

// Ordered write of kept points: f64 copy (packed by out_off) + f32 copy. The offsets come from
// the chunk counts in the kernel itself (round 5: no per-crop scan and crop-offset launches):
// block (c, b) sums the chunk counts of the crops before b (the crop's base) and of its crop's
// chunks before c, in the same barrier as its wave counts; block (0, b) writes kept[b],
// out_off[b] (and out_off[B] for the last crop), block (c, b) coff[b, c].
__global__ __launch_bounds__(1024) void sor_write_kernel(
    const double* __restrict__ xyz, const double* __restrict__ avg, const int64_t* __restrict__ off,
    const double* __restrict__ thr, int nchunk, const int32_t* __restrict__ ccount, int B,
    int64_t* __restrict__ coff, int64_t* __restrict__ kept, int64_t* __restrict__ out_off,
    double* __restrict__ out64, float* __restrict__ out32, int64_t* __restrict__ kept_idx) {
  const int b = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
  const int64_t base = off[b];
  const int n = (int)(off[b + 1] - base);
  const int i = c * 1024 + tid;
  const double t = thr[b];
  bool keep = false;
  if (i < n) {
    const double a = avg[base + i];
    keep = a > 0 && a < t;
  }
  // chunk counts: [0, b nchunk) -> the crop base; [b nchunk, b nchunk + c) -> the chunk base
  int64_t cb = 0, cc = 0;
  for (int e = tid; e < b * nchunk + c; e += 1024) {
    const int64_t v = ccount[e];
    if (e < b * nchunk) cb += v;
    else cc += v;
  }
  cb = pk::wave_sum_i64(cb);
  cc = pk::wave_sum_i64(cc);
  const uint64_t bal = __ballot(keep);
  __shared__ int ws[16];
  __shared__ int64_t wb[16], wc[16];
  if (pk::lane_id() == 0) {
    ws[pk::wave_id()] = __popcll(bal);
    wb[pk::wave_id()] = cb;
    wc[pk::wave_id()] = cc;
  }
  __syncthreads();
  int pre = 0;
  for (int w = 0; w < pk::wave_id(); ++w) pre += ws[w];
  int64_t crop0 = 0, chunk0 = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    crop0 += wb[w];
    chunk0 += wc[w];
  }
  if (tid == 0) {
    if (coff) coff[(int64_t)b * nchunk + c] = chunk0;
    if (c == 0) {
      int64_t k = 0;
      for (int q = 0; q < nchunk; ++q) k += ccount[(int64_t)b * nchunk + q];
      kept[b] = k;
      out_off[b] = crop0;
      if (b == B - 1) out_off[B] = crop0 + k;
    }
  }
  if (keep) {
    const int64_t w = crop0 + chunk0 + pre + __popcll(bal & ((1ull << pk::lane_id()) - 1ull));
    const double* q = xyz + (base + i) * 3;
    if (out64) {
      out64[3 * w] = q[0];
      out64[3 * w + 1] = q[1];
      out64[3 * w + 2] = q[2];
    }
    if (out32) {
      out32[3 * w] = (float)q[0];
      out32[3 * w + 1] = (float)q[1];
      out32[3 * w + 2] = (float)q[2];
    }
    if (kept_idx) kept_idx[w] = i;  // index local to the input crop
  }
}

// npoint policy, start index (hash of seed, crop) and the packed offsets of the result.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// One wave: lane b of each 64-crop chunk computes its crop's policy and start draw (the 64-bit
// modulo is a long software sequence: round 4's single thread ran the B of them in series, ~13 us),
// then a wave scan of |npoint| carried across chunks gives the packed offsets.
__global__ __launch_bounds__(64) void npoint_kernel(const int64_t* __restrict__ off, int B, int fixed, int limit,
                                                     uint64_t seed, int64_t base, int32_t* __restrict__ npoint,
                                                     int32_t* __restrict__ start, int64_t* __restrict__ out_off) {
  const int lane = threadIdx.x;
  int64_t carry = 0;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + lane;
    int64_t cnt = 0;
    if (b < B) {
      const int n = (int)(off[b + 1] - off[b]);
      int np;
      if (fixed > 0) {
        // a fixed target acts as the reference's limit without its int(ratio * n) rounding:
        // FPS to exactly `fixed` when the crop is larger, every point (in order) otherwise
        np = n > fixed ? fixed : -n;
      } else if (n > limit) {
        const double ratio = (double)limit / (double)n;  // object.py:146
        np = (int)(ratio * (double)n);                   // int(ratio * N) in upstream FPS
      } else {
        np = -n;  // no FPS: keep all n points in order (encoded negative)
      }
      npoint[b] = np;
      if (start) start[b] = n > 0 ? (int32_t)(splitmix64(seed ^ splitmix64((uint64_t)(base + b))) % (uint64_t)n) : 0;
      cnt = np < 0 ? -np : np;
    }
    const int64_t inc = pk::wave_inclusive_scan_i64(cnt);
    if (b < B) out_off[b] = carry + inc - cnt;
    carry += __shfl(inc, 63);
  }
  if (lane == 0) out_off[B] = carry;
}

// pcd[idx] (f64) -> align = pcd @ R + (-t @ R) with left-to-right 3-term dots, plus f32
// copy of pcd[idx]. One thread per output point; crop b writes rows out_off[b]..
__global__ __launch_bounds__(256) void gather_transform_kernel(
    const double* __restrict__ pcd, const int64_t* __restrict__ off, const int64_t* __restrict__ idx,
    int idx_stride, const int32_t* __restrict__ npoint, const int64_t* __restrict__ out_off,
    const double* __restrict__ R, const double* __restrict__ t, double* __restrict__ sel64,
    double* __restrict__ align64, float* __restrict__ sel32, int32_t* __restrict__ status, int ld,
    float* __restrict__ pad_sel, float* __restrict__ pad_align, int32_t* __restrict__ pad_counts) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int np = npoint[b];
  const int cnt = np < 0 ? -np : np;
  const int64_t nb = off[b + 1] - off[b];
  // collate's padded f32 copies (pk_gather_transform_pad): rows >= the crop's count are zero
  if (pad_counts != nullptr && blockIdx.x == 0 && threadIdx.x == 0) pad_counts[b] = cnt < ld ? cnt : ld;
  if (j >= cnt && j < ld) {
    if (pad_sel) {
      pad_sel[((int64_t)b * ld + j) * 3] = 0.f;
      pad_sel[((int64_t)b * ld + j) * 3 + 1] = 0.f;
      pad_sel[((int64_t)b * ld + j) * 3 + 2] = 0.f;
    }
    if (pad_align) {
      pad_align[((int64_t)b * ld + j) * 3] = 0.f;
      pad_align[((int64_t)b * ld + j) * 3 + 1] = 0.f;
      pad_align[((int64_t)b * ld + j) * 3 + 2] = 0.f;
    }
  }
  if (status && blockIdx.x == 0) {  // the crop's index check (written for every crop: no init needed)
    int bad = 0;
    if (np >= 0)
      for (int k = threadIdx.x; k < cnt; k += 256) {
        const int64_t i = idx[(int64_t)b * idx_stride + k];
        bad |= (i < 0 || i >= nb) ? 1 : 0;
      }
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) status[b] = bad;
  }
  if (j >= cnt) return;
  const int64_t i = np < 0 ? j : idx[(int64_t)b * idx_stride + j];
  const bool inr = i >= 0 && i < nb;  // an out-of-range index is not read: its outputs are NaN
  const int64_t src = off[b] + (inr ? i : 0);
  const double nan = __builtin_nan("");
  const double x = inr ? pcd[3 * src] : nan, y = inr ? pcd[3 * src + 1] : nan, z = inr ? pcd[3 * src + 2] : nan;
  const double* Rb = R + 9 * b;  // row-major R_m2c
  const double* tb = t + 3 * b;
  const int64_t w = out_off[b] + j;
  if (sel64) {
    sel64[3 * w] = x;
    sel64[3 * w + 1] = y;
    sel64[3 * w + 2] = z;
  }
  if (sel32) {
    sel32[3 * w] = (float)x;
    sel32[3 * w + 1] = (float)y;
    sel32[3 * w + 2] = (float)z;
  }
  const bool padr = j < ld;
  if (pad_sel && padr) {
    pad_sel[((int64_t)b * ld + j) * 3] = (float)x;
    pad_sel[((int64_t)b * ld + j) * 3 + 1] = (float)y;
    pad_sel[((int64_t)b * ld + j) * 3 + 2] = (float)z;
  }
  if (align64 || (pad_align && padr)) {
    const double nt0 = -1.0 * tb[0], nt1 = -1.0 * tb[1], nt2 = -1.0 * tb[2];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double tt = (nt0 * Rb[c] + nt1 * Rb[3 + c]) + nt2 * Rb[6 + c];
      const double a = ((x * Rb[c] + y * Rb[3 + c]) + z * Rb[6 + c]) + tt;
      if (align64) align64[3 * w + c] = a;
      if (pad_align && padr) pad_align[((int64_t)b * ld + j) * 3 + c] = (float)a;
    }
  }
}

// collate (dataset/helpers.py:22-50) for one packed field: torch.Tensor(x) (-> f32) then
// pad_sequence(batch_first=True) with zeros. grid (ceil(ld*C/256), B); crop b's rows
// [0, min(n_b, ld)) are copied (cast to f32), rows up to ld are zero.
template <typename T>
__global__ __launch_bounds__(256) void collate_pad_kernel(const T* __restrict__ src, int C,
                                                          const int64_t* __restrict__ off, int ld,
                                                          float* __restrict__ dst, int32_t* __restrict__ counts) {
  const int b = blockIdx.y;
  const int64_t o = off[b];
  const int64_t n = off[b + 1] - o;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (counts != nullptr && blockIdx.x == 0 && threadIdx.x == 0) counts[b] = (int32_t)(n < ld ? n : ld);
  if (e >= (int64_t)ld * C) return;
  const int64_t row = e / C;
  dst[(int64_t)b * ld * C + e] = row < n ? (float)src[o * C + e] : 0.f;
}

}  // namespace

extern "C" int pk_collate_pad(const void* src, int src_f64, int C, const int64_t* off, int B, int ld, float* dst,
                              int32_t* counts, void* stream) {
  PK_REQUIRE(B >= 0 && C > 0 && ld >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(off && (dst || ld == 0) && (src || ld == 0));
  if (ld == 0 && counts == nullptr) return PK_OK;
  dim3 grid((unsigned)(((int64_t)ld * C + 255) / 256 > 0 ? ((int64_t)ld * C + 255) / 256 : 1), B);
  hipStream_t s = pk::as_stream(stream);
  if (src_f64)
    hipLaunchKernelGGL(collate_pad_kernel<double>, grid, dim3(256), 0, s, static_cast<const double*>(src), C, off, ld,
                       dst, counts);
  else
    hipLaunchKernelGGL(collate_pad_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(src), C, off, ld,
                       dst, counts);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_backproject(const uint16_t* depth, const uint8_t* mask, int F, int H, int W,
                              const double* K, const float* cam_scale, int32_t* rowcnt,
                              int64_t* rowoff, int64_t* count, int64_t* off, double* xyz, int64_t cap,
                              int32_t* pix, int32_t* idxmap, void* stream) {
  PK_REQUIRE(F >= 0 && H > 0 && W > 0 && cap >= 0);
  if (F == 0) return PK_OK;
  PK_REQUIRE(depth && mask && K && cam_scale && rowcnt && rowoff && count && off && (xyz || cap == 0));
  hipStream_t s = pk::as_stream(stream);
  hipLaunchKernelGGL(bp_count16_kernel, dim3((H + 3) / 4, F), dim3(256), 0, s, mask, H, W, rowcnt);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(seg_scan_kernel, dim3(F), dim3(1024), 0, s, rowcnt, H, rowoff, count);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(bp_write16_kernel, dim3((H + 3) / 4, F), dim3(256), 0, s, depth, mask, H, W, K, cam_scale,
                     rowoff, count, off, xyz, cap, pix, idxmap);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_sor(const double* xyz, const int64_t* off, int B, int nmax, int knn,
                      double std_ratio, const int32_t* pix, const int32_t* idxmap, int H, int W,
                      const double* K, double* avg, double* thr, int32_t* ccount, int64_t* coff,
                      int64_t* kept, int64_t* out_off, double* out64, float* out32,
                      int64_t* kept_idx, void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && knn > 0 && knn <= kKnn);
  if (B == 0) return PK_OK;
  PK_REQUIRE(xyz && off && avg && thr && ccount && coff && kept && out_off);
  PK_REQUIRE((pix == nullptr) == (idxmap == nullptr) && (pix == nullptr || (H > 0 && W > 0)));
  hipStream_t s = pk::as_stream(stream);
  const int nchunk = (nmax + 1023) / 1024;
  if (nmax > 0 && !pk::diag_skip("sorknn")) {
    const int tiles = (nmax + kSorThreads - 1) / kSorThreads;
    for (int rep = 0; rep < (pk::diag_twice("sorknn") ? 2 : 1); ++rep) {
      hipLaunchKernelGGL(sor_knn_kernel, dim3((unsigned)((int64_t)tiles * B)),
                         dim3(kSorThreads), 0, s, xyz, off, knn, pix, idxmap, H, W,
                         pix != nullptr ? K : nullptr, tiles, B, avg, pk::side_prio());
      PK_CHECK_LAUNCH();
    }
  }
  for (int rep = 0; rep < (pk::diag_twice("sorstats") ? 2 : 1); ++rep) {
    hipLaunchKernelGGL(sor_stats_kernel, dim3(B), dim3(kStatThreads), 0, s, avg, off, std_ratio, thr, pk::side_prio());
    PK_CHECK_LAUNCH();
  }
  if (nchunk > 0) {
    hipLaunchKernelGGL(sor_count_kernel, dim3(nchunk, B), dim3(1024), 0, s, avg, off, thr, nchunk, ccount);
    PK_CHECK_LAUNCH();
  }
  if (nchunk > 0 && (out64 || out32 || kept_idx)) {  // the write forms coff / kept / out_off itself
    hipLaunchKernelGGL(sor_write_kernel, dim3(nchunk, B), dim3(1024), 0, s, xyz, avg, off, thr, nchunk, ccount,
                       B, coff, kept, out_off, out64, out32, kept_idx);
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  if (nchunk > 0) {
    hipLaunchKernelGGL(seg_scan_kernel, dim3(B), dim3(1024), 0, s, ccount, nchunk, coff, kept);
    PK_CHECK_LAUNCH();
  } else {
    hipError_t e = pk::zero_async(kept, sizeof(int64_t) * B, s);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(64), 0, s, kept, B, out_off);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_offsets_from_counts(const int64_t* counts, int B, int64_t* off, void* stream) {
  PK_REQUIRE(B >= 0 && counts && off);
  hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(64), 0, pk::as_stream(stream), counts, B, off);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_segment_scan(const int32_t* cnt, int S, int n, int64_t* off, int64_t* total,
                               void* stream) {
  PK_REQUIRE(S >= 0 && n >= 0);
  if (S == 0) return PK_OK;
  PK_REQUIRE(cnt && off);
  hipLaunchKernelGGL(seg_scan_kernel, dim3(S), dim3(1024), 0, pk::as_stream(stream), cnt, n, off, total);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_fps_npoint(const int64_t* off, int B, int fixed, int limit, uint64_t seed, int64_t base,
                             int32_t* npoint, int32_t* start, int64_t* out_off, void* stream) {
  PK_REQUIRE(B >= 0 && limit > 0 && base >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(off && npoint && out_off);
  hipLaunchKernelGGL(npoint_kernel, dim3(1), dim3(64), 0, pk::as_stream(stream), off, B, fixed, limit,
                     seed, base, npoint, start, out_off);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_gather_transform(const double* pcd, const int64_t* off, int B, const int64_t* idx,
                                   int idx_stride, const int32_t* npoint, int npmax,
                                   const int64_t* out_off, const double* R, const double* t,
                                   double* sel64, double* align64, float* sel32, int32_t* status,
                                   void* stream) {
  PK_REQUIRE(B >= 0 && npmax >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(pcd && off && npoint && out_off && R && t);
  hipLaunchKernelGGL(gather_transform_kernel, dim3(std::max(1, (npmax + 255) / 256), B), dim3(256), 0,
                     pk::as_stream(stream), pcd, off, idx, idx_stride, npoint, out_off, R, t, sel64,
                     align64, sel32, status, 0, nullptr, nullptr, nullptr);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_gather_transform_pad(const double* pcd, const int64_t* off, int B, const int64_t* idx,
                                       int idx_stride, const int32_t* npoint, int npmax,
                                       const int64_t* out_off, const double* R, const double* t,
                                       double* sel64, double* align64, float* sel32, int32_t* status, int ld,
                                       float* pad_sel32, float* pad_align32, int32_t* counts, void* stream) {
  PK_REQUIRE(B >= 0 && npmax >= 0 && ld >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(pcd && off && npoint && out_off && R && t);
  const int rows = std::max(npmax, ld);
  hipLaunchKernelGGL(gather_transform_kernel, dim3(std::max(1, (rows + 255) / 256), B), dim3(256), 0,
                     pk::as_stream(stream), pcd, off, idx, idx_stride, npoint, out_off, R, t, sel64,
                     align64, sel32, status, ld, pad_sel32, pad_align32, counts);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// ---------------------------------------------------------------- erosion alone (object.py:52-71)
namespace {
__global__ __launch_bounds__(256) void erode_kernel(const uint8_t* __restrict__ mask, int H, int W,
                                                    uint8_t* __restrict__ out) {
  const int f = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int v = (int)(p / W), u = (int)(p % W);
  out[(int64_t)f * H * W + p] = eroded(mask + (int64_t)f * H * W, H, W, v, u) ? 1 : 0;
}

// H16 — bilinear sampling of an RGB / feature image at projected 3D points (build-defined;
// the reference loads RGB only when color=True, dataset/scene.py:95-97, 153-156).
// u = fx X / Z + cx, v = fy Y / Z + cy (pixels); bilinear with zero padding outside the
// image, i.e. torch grid_sample(align_corners=True, padding_mode="zeros") on pixel
// centres. img uint8 [F, H, W, C] channels-last; pts f64 [T,3] packed per frame (cm, camera
// frame); out f32 [T, C] in [0, 1].
__global__ __launch_bounds__(256) void sample_rgb_kernel(const uint8_t* __restrict__ img, int H, int W, int C,
                                                         const double* __restrict__ K,
                                                         const double* __restrict__ pts,
                                                         const int64_t* __restrict__ off, float* __restrict__ out) {
  const int f = blockIdx.y;
  const int64_t o = off[f];
  const int n = (int)(off[f + 1] - o);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double* p = pts + 3 * (o + i);
  const double* Kf = K + 9 * f;
  const float u = (float)(Kf[0] * p[0] / p[2] + Kf[2]);
  const float v = (float)(Kf[4] * p[1] / p[2] + Kf[5]);
  const float u0f = floorf(u), v0f = floorf(v);
  const int u0 = (int)u0f, v0 = (int)v0f;
  const float au = u - u0f, av = v - v0f;
  const uint8_t* im = img + (int64_t)f * H * W * C;
  for (int c = 0; c < C; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int dv = 0; dv < 2; ++dv)
#pragma unroll
      for (int du = 0; du < 2; ++du) {
        const int uu = u0 + du, vv = v0 + dv;
        const float w = (du ? au : 1.f - au) * (dv ? av : 1.f - av);
        if (uu >= 0 && uu < W && vv >= 0 && vv < H) acc = fmaf(w, (float)im[((int64_t)vv * W + uu) * C + c], acc);
      }
    out[(o + i) * C + c] = acc * (1.f / 255.f);
  }
}

// H16, f32 backbone features: the same projection and bilinear weights on an f32 feature
// map [F, C, H, W] (channels-first, as a CNN backbone emits it). Thread = (point, channel),
// channel fastest, so the [T, C] output rows are written contiguously.
__global__ __launch_bounds__(256) void sample_feat_kernel(const float* __restrict__ fmap, int C, int H, int W,
                                                          const double* __restrict__ K,
                                                          const double* __restrict__ pts,
                                                          const int64_t* __restrict__ off, int nmax,
                                                          float* __restrict__ out) {
  const int f = blockIdx.y;
  const int64_t o = off[f];
  const int n = (int)(off[f + 1] - o);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int i = (int)(e / C), c = (int)(e - (int64_t)i * C);
  if (i >= n || i >= nmax) return;
  const double* p = pts + 3 * (o + i);
  const double* Kf = K + 9 * f;
  const float u = (float)(Kf[0] * p[0] / p[2] + Kf[2]);
  const float v = (float)(Kf[4] * p[1] / p[2] + Kf[5]);
  const float u0f = floorf(u), v0f = floorf(v);
  const int u0 = (int)u0f, v0 = (int)v0f;
  const float au = u - u0f, av = v - v0f;
  const float* pl = fmap + ((int64_t)f * C + c) * H * W;
  float acc = 0.f;
#pragma unroll
  for (int dv = 0; dv < 2; ++dv)
#pragma unroll
    for (int du = 0; du < 2; ++du) {
      const int uu = u0 + du, vv = v0 + dv;
      const float w = (du ? au : 1.f - au) * (dv ? av : 1.f - av);
      if (uu >= 0 && uu < W && vv >= 0 && vv < H) acc = fmaf(w, pl[(int64_t)vv * W + uu], acc);
    }
  out[(o + i) * C + c] = acc;
}
}  // namespace

extern "C" int pk_sample_features(const float* fmap, int F, int C, int H, int W, const double* K, const double* pts,
                                  const int64_t* off, int nmax, float* out, void* stream) {
  PK_REQUIRE(F >= 0 && H > 0 && W > 0 && C > 0 && nmax >= 0);
  if (F == 0 || nmax == 0) return PK_OK;
  PK_REQUIRE(fmap && K && pts && off && out);
  const int64_t blocks = ((int64_t)nmax * C + 255) / 256;
  PK_REQUIRE(blocks < (1LL << 31));
  hipLaunchKernelGGL(sample_feat_kernel, dim3((unsigned)blocks, F), dim3(256), 0, pk::as_stream(stream), fmap, C, H,
                     W, K, pts, off, nmax, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_erode_mask(const uint8_t* mask, int F, int H, int W, uint8_t* out, void* stream) {
  PK_REQUIRE(F >= 0 && H > 0 && W > 0);
  if (F == 0) return PK_OK;
  PK_REQUIRE(mask && out);
  hipLaunchKernelGGL(erode_kernel, dim3((H * W + 255) / 256, F), dim3(256), 0, pk::as_stream(stream), mask, H, W,
                     out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_sample_rgb(const uint8_t* img, int F, int H, int W, int C, const double* K, const double* pts,
                             const int64_t* off, int nmax, float* out, void* stream) {
  PK_REQUIRE(F >= 0 && H > 0 && W > 0 && C > 0 && nmax >= 0);
  if (F == 0 || nmax == 0) return PK_OK;
  PK_REQUIRE(img && K && pts && off && out);
  hipLaunchKernelGGL(sample_rgb_kernel, dim3((nmax + 255) / 256, F), dim3(256), 0, pk::as_stream(stream), img, H, W,
                     C, K, pts, off, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

#ifdef PK_DEVBUILD
extern "C" int pkdev_seq_sum(const double* v, int n, double* out, void* stream) {
  PK_REQUIRE(n >= 0 && out && (n == 0 || v));
  hipLaunchKernelGGL(seq_sum_dev_kernel, dim3(1), dim3(kStatThreads), 0, pk::as_stream(stream), v, n, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
#endif  // PK_DEVBUILD
