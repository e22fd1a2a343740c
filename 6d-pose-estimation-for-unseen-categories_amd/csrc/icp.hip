// (f4) Point-to-point ICP refinement after RANSAC, batched over crops.
//
// Reference: scripts/test_RANSAC.py:436-446 -> Open3D 0.17 registration_icp(source, target,
// threshold = 0.2, trans_init = T_RANSAC, TransformationEstimationPointToPoint(),
// ICPConvergenceCriteria(max_iteration = 2000)) (relative_fitness = relative_rmse = 1e-6, the
// defaults). Open3D's loop:
//   result_0 = evaluate(T_0)
//   for i < max_iteration: U = umeyama(matched source, matched target); T <- U T;
//                          result_{i+1} = evaluate(T);
//                          stop if |dfitness| < rel_fitness and |drmse| < rel_rmse
// evaluate(T): every source point p = T s takes its nearest target point (KD-tree hybrid search,
// radius = threshold, max_nn = 1: a pair iff d^2 < threshold^2, nanoflann's strict radius test);
// fitness = pairs / |source|, inlier_rmse = sqrt(sum d^2 / pairs) (0 without pairs); no pairs
// gives U = I. Deviations (documented, parity unpinned against Open3D): the source is
// transformed by the accumulated T each iteration (Open3D re-transforms its working copy by
// every U, compounding roundings), and an exact distance tie goes to the lowest target index
// (a KD-tree returns either).
//
// The reference aligns the CAD to the GT-posed CAD (its target); the host mirror also offers
// the observed crop as the target (pose refinement without ground truth).
//
// Design: the source queries are visited in x order under T_init (so the 64 slabs of a wave
// overlap and their candidate loads share cache lines) and the target of each crop is sorted once by x (rank by counting, fp64 keys, index
// tie-break; SoA x / y / z / index) with a 1024-bucket x table; a query scans only the x-slab
// [px - r, px + r], starting one bucket before its lower edge and loading candidates 8 at a
// time (independent loads, so the scan is not a chain of memory latencies), so a 0.2 cm radius
// on a 10-20 cm object touches ~100 candidates instead of the whole target. Per iteration two launches: match (grid = source blocks x crops: nearest target,
// pair test, block partial sums of count, sum d^2, the matched source and target points and
// their products, shifted by the crop's first target point against cancellation) and update
// (one wave per crop: partials in block order, the convergence test, Horn's quaternion fit of
// the centred cross-covariance — pk_rigid, shared with RANSAC — and T <- U T). Converged crops
// return at the top of both kernels, so a host loop can enqueue iterations in batches and
// poll a device count of active crops.
#include "common.hpp"
#include "rigid.hpp"

namespace {

constexpr int kIThreads = 256;
constexpr int kWin = 1536;  // LDS candidate window of a match block (28 B per target point)
constexpr int kNPart = 17;  // count, sum d^2, sum p (3), sum q (3), sum p q^T (9)

struct IcpState {  // per crop, in the work buffer
  double T[16];
  double fit, rmse, prev_fit, prev_rmse;
  double xmin, inv_w;  // x-bucket table of the sorted target: bucket k starts at xmin + k / inv_w
  int iter, active, converged, pad;
};

constexpr int kNBuckets = 1024;

struct IcpWork {
  IcpState* st;
  double* sx;     // [B][ntgt_max] target x, y, z in x order (SoA)
  double* sy;
  double* sz;
  int32_t* sidx;  // [B][ntgt_max] original index
  int32_t* tbl;   // [B][kNBuckets + 1] first sorted index of each x bucket
  int32_t* perm;  // [B][nsrc_max] source points in x order under T_init (query order)
  double* part;   // [B][nblk][kNPart]
};

__host__ __device__ inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

__host__ __device__ inline IcpWork carve(void* w, int B, int nsrc_max, int ntgt_max) {
  char* p = static_cast<char*>(w);
  IcpWork o;
  o.st = reinterpret_cast<IcpState*>(p);
  p += al256((int64_t)B * sizeof(IcpState));
  o.sx = reinterpret_cast<double*>(p);
  p += al256((int64_t)B * ntgt_max * 8);
  o.sy = reinterpret_cast<double*>(p);
  p += al256((int64_t)B * ntgt_max * 8);
  o.sz = reinterpret_cast<double*>(p);
  p += al256((int64_t)B * ntgt_max * 8);
  o.sidx = reinterpret_cast<int32_t*>(p);
  p += al256((int64_t)B * ntgt_max * 4);
  o.tbl = reinterpret_cast<int32_t*>(p);
  p += al256((int64_t)B * (kNBuckets + 1) * 4);
  o.perm = reinterpret_cast<int32_t*>(p);
  p += al256((int64_t)B * nsrc_max * 4);
  o.part = reinterpret_cast<double*>(p);
  return o;
}

inline int64_t work_bytes_for(int B, int nsrc_max, int ntgt_max) {
  const int64_t nblk = (nsrc_max + kIThreads - 1) / kIThreads;
  return al256((int64_t)B * sizeof(IcpState)) + 3 * al256((int64_t)B * ntgt_max * 8) +
         al256((int64_t)B * ntgt_max * 4) + al256((int64_t)B * (kNBuckets + 1) * 4) +
         al256((int64_t)B * nsrc_max * 4) + al256((int64_t)B * (nblk > 0 ? nblk : 1) * kNPart * 8);
}

// grid (B): T <- T_init, counters reset. A crop whose source or target exceeds the capacity
// (nsrc_max / ntgt_max, the work buffer's per-crop rows) never runs: inactive, converged = -1
// (the result's overflow flag), T = T_init.
__global__ void icp_init_kernel(const double* __restrict__ T_init, const int64_t* __restrict__ src_off,
                                const int64_t* __restrict__ tgt_off, int nsrc_max, int ntgt_max,
                                IcpState* __restrict__ st) {
  const int b = blockIdx.x;
  if (threadIdx.x < 16) st[b].T[threadIdx.x] = T_init[16 * b + threadIdx.x];
  if (threadIdx.x == 0) {
    const bool over = src_off[b + 1] - src_off[b] > nsrc_max || tgt_off[b + 1] - tgt_off[b] > ntgt_max;
    st[b].fit = st[b].rmse = st[b].prev_fit = st[b].prev_rmse = 0.0;
    st[b].xmin = st[b].inv_w = 0.0;
    st[b].iter = 0;
    st[b].active = over ? 0 : 1;
    st[b].converged = over ? -1 : 0;
  }
}

__device__ __forceinline__ uint64_t ordered_bits(double x) {  // monotone map double -> uint64
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// grid (ceil(nmax / 256), B): each point's rank in (x, index) order by counting over the crop's
// keys staged through LDS (x as order-preserving uint64 bits: integer compares; index tie-break);
// scatter. With M (4x4 row-major per crop, the initial poses) the key is the x of M p — the
// source query order; sx / sy / sz may then be NULL and only the permutation is written.
__global__ __launch_bounds__(kIThreads) void icp_sort_kernel(const double* __restrict__ pts,
                                                             const int64_t* __restrict__ off, int nmax,
                                                             const double* __restrict__ M,
                                                             double* __restrict__ sx, double* __restrict__ sy,
                                                             double* __restrict__ sz, int32_t* __restrict__ sidx) {
  constexpr int kTile = 4096;
  __shared__ uint64_t ks[kTile];
  const int b = blockIdx.y;
  const int64_t p0 = off[b];
  const int n = (int)(off[b + 1] - p0);
  if ((int)blockIdx.x * kIThreads >= n || n > nmax) return;  // block-uniform (over capacity: skipped, see init)
  const double* P = pts + 3 * p0;
  const double* Mb = M ? M + 16 * b : nullptr;
  auto key_x = [&](int j) {
    const double* q = P + 3 * j;
    return Mb ? ((Mb[0] * q[0] + Mb[1] * q[1]) + Mb[2] * q[2]) + Mb[3] : q[0];
  };
  const int i = blockIdx.x * kIThreads + threadIdx.x;
  const bool own = i < n;
  const uint64_t ki = own ? ordered_bits(key_x(i)) : 0ull;
  int rank = 0;
  for (int j0 = 0; j0 < n; j0 += kTile) {
    const int jn = min(kTile, n - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < jn; j += kIThreads) ks[j] = ordered_bits(key_x(j0 + j));
    __syncthreads();
    if (own) {
      const int lim = min(jn, i - j0);  // keys before i: ties count (index tie-break)
      int j = 0;
#pragma unroll 8
      for (; j < jn; ++j) rank += (ks[j] < ki) || (ks[j] == ki && j < lim);
    }
  }
  if (!own) return;
  const int64_t o = (int64_t)b * nmax + rank;
  if (sx) {
    sx[o] = P[3 * i];
    sy[o] = P[3 * i + 1];
    sz[o] = P[3 * i + 2];
  }
  sidx[o] = i;
}

// grid (B), block 1024, dynamic LDS P x 12 B + 16 KiB (P = the power of two >= nmax, <= 8192): the
// same (x key, index) order as icp_sort_kernel by a bucket sort: keys binned into 2048 x-buckets
// (monotone in x: floor((x - xmin) * NB / (xmax - xmin))), histogram + scan + scatter in LDS, then
// every bucket insertion-sorted by (key, index) by one thread — a few keys per bucket, so ~10
// LDS passes instead of bitonic's log2(P)(log2(P)+1)/2 = 91 block-wide passes. The scatter order
// inside a bucket does not matter (the insertion sort fixes it), so the result is deterministic.
// A bucket above 64 keys (heavily repeated x) sends the whole crop through a block bitonic sort.
constexpr int kSortBuckets = 2048;
__global__ __launch_bounds__(1024) void icp_bucket_sort_kernel(const double* __restrict__ pts,
                                                               const int64_t* __restrict__ off, int nmax, int P,
                                                               const double* __restrict__ M, double* __restrict__ sx,
                                                               double* __restrict__ sy, double* __restrict__ sz,
                                                               int32_t* __restrict__ sidx) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  uint64_t* key = lds;                                       // [P] keys in bucket order
  int32_t* val = reinterpret_cast<int32_t*>(lds + P);        // [P]
  int32_t* cnt = val + P;                                    // [kSortBuckets]
  int32_t* fill = cnt + kSortBuckets;                        // [kSortBuckets]
  __shared__ double rmin[16], rmax[16];
  __shared__ int maxcnt;
  const int b = blockIdx.x;
  const int64_t p0 = off[b];
  const int n = (int)(off[b + 1] - p0);
  if (n > nmax) return;  // over capacity: skipped (see icp_init_kernel)
  const double* Pt = pts + 3 * p0;
  const double* Mb = M ? M + 16 * b : nullptr;
  auto key_x = [&](int t) {  // recomputed per pass (keeps LDS at 12 B per key: P <= 8192 fits)
    const double* q = Pt + 3 * t;
    return Mb ? ((Mb[0] * q[0] + Mb[1] * q[1]) + Mb[2] * q[2]) + Mb[3] : q[0];
  };
  double lo = INFINITY, hi = -INFINITY;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const double x = key_x(t);
    lo = fmin(lo, x);
    hi = fmax(hi, x);
  }
  for (int t = threadIdx.x; t < kSortBuckets; t += blockDim.x) cnt[t] = fill[t] = 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o));
    hi = fmax(hi, __shfl_xor(hi, o));
  }
  if (pk::lane_id() == 0) {
    rmin[pk::wave_id()] = lo;
    rmax[pk::wave_id()] = hi;
  }
  if (threadIdx.x == 0) maxcnt = 0;
  __syncthreads();
  lo = rmin[0];
  hi = rmax[0];
  for (int w = 1; w < 16; ++w) {
    lo = fmin(lo, rmin[w]);
    hi = fmax(hi, rmax[w]);
  }
  const double scale = hi > lo ? (double)kSortBuckets / (hi - lo) : 0.0;
  auto bucket_of = [&](double x) {
    const int k = (int)((x - lo) * scale);
    return k < 0 ? 0 : (k >= kSortBuckets ? kSortBuckets - 1 : k);
  };
  for (int t = threadIdx.x; t < n; t += blockDim.x) atomicAdd(&cnt[bucket_of(key_x(t))], 1);
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the bucket counts by one wave (32 per lane)
    constexpr int per = kSortBuckets / 64;
    int local = 0, mx = 0;
    for (int q = 0; q < per; ++q) {
      const int c = cnt[threadIdx.x * per + q];
      local += c;
      mx = max(mx, c);
    }
    const int incl = pk::wave_inclusive_scan_i32(local);
    int run = incl - local;
    for (int q = 0; q < per; ++q) {
      const int c = cnt[threadIdx.x * per + q];
      fill[threadIdx.x * per + q] = run;  // bucket start
      run += c;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    if (threadIdx.x == 0) maxcnt = mx;
  }
  __syncthreads();
  if (maxcnt > 64) {  // skewed: bitonic over (key, index) in place of the bucket pass
    for (int t = threadIdx.x; t < P; t += blockDim.x) {
      key[t] = t < n ? ordered_bits(key_x(t)) : ~0ull;
      val[t] = t;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = threadIdx.x; t < P; t += blockDim.x) {
          const int u = t ^ j;
          if (u > t) {
            const uint64_t ka = key[t], kb = key[u];
            const int va = val[t], vb = val[u];
            const bool b_less = kb < ka || (kb == ka && vb < va);
            if (b_less == ((t & k) == 0)) {
              key[t] = kb;
              key[u] = ka;
              val[t] = vb;
              val[u] = va;
            }
          }
        }
        __syncthreads();
      }
    }
  } else {
    for (int t = threadIdx.x; t < n; t += blockDim.x) {  // scatter (in-bucket order arbitrary)
      const double x = key_x(t);
      const int pos = atomicAdd(&fill[bucket_of(x)], 1);
      key[pos] = ordered_bits(x);
      val[pos] = t;
    }
    __syncthreads();
    for (int bk = threadIdx.x; bk < kSortBuckets; bk += blockDim.x) {  // insertion sort per bucket
      const int e = fill[bk], s0 = e - cnt[bk];
      for (int i = s0 + 1; i < e; ++i) {
        const uint64_t kk = key[i];
        const int vv = val[i];
        int j = i - 1;
        while (j >= s0 && (key[j] > kk || (key[j] == kk && val[j] > vv))) {
          key[j + 1] = key[j];
          val[j + 1] = val[j];
          --j;
        }
        key[j + 1] = kk;
        val[j + 1] = vv;
      }
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const int i = val[t];
    const int64_t o = (int64_t)b * nmax + t;
    if (sx) {
      sx[o] = Pt[3 * i];
      sy[o] = Pt[3 * i + 1];
      sz[o] = Pt[3 * i + 2];
    }
    sidx[o] = i;
  }
}

// grid (B), block 1024: the x-bucket table of the sorted target: tbl[k] = first sorted index
// with x >= xmin + k w (w = (xmax - xmin) / kNBuckets), by binary search per bucket. A query's
// slab scan starts at the bucket BEFORE its lower edge's bucket, so a rounding of the bucket
// index can only start the scan early (points left of the slab are never pairs: d^2 >= dx^2 > r^2).
__global__ __launch_bounds__(1024) void icp_bucket_kernel(const int64_t* __restrict__ tgt_off, int ntgt_max,
                                                          const double* __restrict__ sx, IcpState* __restrict__ st,
                                                          int32_t* __restrict__ tbl) {
  const int b = blockIdx.x;
  const int nt = (int)(tgt_off[b + 1] - tgt_off[b]);
  if (nt > ntgt_max) return;  // over capacity: the crop stays inactive (icp_init_kernel)
  const double* X = sx + (int64_t)b * ntgt_max;
  int32_t* Tb = tbl + (int64_t)b * (kNBuckets + 1);
  const double xmin = nt > 0 ? X[0] : 0.0, xmax = nt > 0 ? X[nt - 1] : 0.0;
  const double w = (xmax - xmin) / kNBuckets;
  const double inv_w = w > 0.0 ? 1.0 / w : 0.0;
  if (threadIdx.x == 0) {
    st[b].xmin = xmin;
    st[b].inv_w = inv_w;
  }
  for (int k = threadIdx.x; k <= kNBuckets; k += blockDim.x) {
    const double edge = xmin + (double)k * w;
    int lo = 0, hi = nt;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (X[mid] < edge) lo = mid + 1;
      else hi = mid;
    }
    Tb[k] = (k == 0) ? 0 : lo;
  }
}

__device__ __forceinline__ void block_sum(double v[kNPart], double* __restrict__ out) {
  __shared__ double red[kIThreads / 64][kNPart];
#pragma unroll
  for (int k = 0; k < kNPart; ++k) {
    double x = v[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
    v[k] = x;
  }
  if (pk::lane_id() == 0)
#pragma unroll
    for (int k = 0; k < kNPart; ++k) red[pk::wave_id()][k] = v[k];
  __syncthreads();
  if (threadIdx.x < kNPart) {
    double s = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kIThreads / 64; ++w) s += red[w][threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// grid (nblk, B): nearest target point of each transformed source point inside the x-slab;
// the block's partial sums of the matched pairs (shifted by the crop's first target point).
__global__ __launch_bounds__(kIThreads) void icp_match_kernel(
    const double* __restrict__ src, const int64_t* __restrict__ src_off, const double* __restrict__ tgt,
    const int64_t* __restrict__ tgt_off, double r, int ntgt_max, int nblk, const IcpState* __restrict__ st,
    const double* __restrict__ sx, const double* __restrict__ sy, const double* __restrict__ sz,
    const int32_t* __restrict__ sidx, const int32_t* __restrict__ tbl, const int32_t* __restrict__ perm,
    int nsrc_max, double* __restrict__ part) {
  const int b = blockIdx.y;
  if (!st[b].active) return;  // block-uniform
  const int64_t s0 = src_off[b];
  const int ns = (int)(src_off[b + 1] - s0);
  const int64_t t0 = tgt_off[b];
  const int nt = (int)(tgt_off[b + 1] - t0);
  const int i = blockIdx.x * kIThreads + threadIdx.x;
  double acc[kNPart];
#pragma unroll
  for (int k = 0; k < kNPart; ++k) acc[k] = 0.0;
  const bool own = i < ns && nt > 0;
  int k0 = 0, k1 = 0;
  double qpx = 0.0, qpy = 0.0, qpz = 0.0, qlo = 0.0, qhi = 0.0;
  if (own) {
    const double* M = st[b].T;
    const double* s = src + 3 * (s0 + perm[(int64_t)b * nsrc_max + i]);  // x-ordered queries: a wave's slabs overlap
    const double x = s[0], y = s[1], z = s[2];
    const double px = ((M[0] * x + M[1] * y) + M[2] * z) + M[3];
    const double py = ((M[4] * x + M[5] * y) + M[6] * z) + M[7];
    const double pz = ((M[8] * x + M[9] * y) + M[10] * z) + M[11];
    const double lo_x = px - r, hi_x = px + r;
    // scan start: the bucket before the slab's lower edge (see icp_bucket_kernel)
    const double kb = (lo_x - st[b].xmin) * st[b].inv_w;
    k0 = 0;
    if (kb >= 1.0) k0 = tbl[(int64_t)b * (kNBuckets + 1) + (kb >= (double)kNBuckets ? kNBuckets : (int)kb) - 1];
    // scan end bound: the start of the bucket two past the slab's upper edge (every later
    // point has x > hi_x even after rounding of the bucket index)
    const double kh = (hi_x - st[b].xmin) * st[b].inv_w;
    k1 = nt;
    if (kh < (double)(kNBuckets - 2) && kh >= -1.0) k1 = tbl[(int64_t)b * (kNBuckets + 1) + (int)kh + 2];
    if (kh < -1.0) k1 = k0;
    qpx = px;
    qpy = py;
    qpz = pz;
    qlo = lo_x;
    qhi = hi_x;
  }
  // the block's candidate window [min k0, max k1): staged in LDS when it fits (x-ordered queries
  // make the 256 slabs of a block overlap: a few hundred target points instead of 256 x ~100
  // scattered L2 gathers), scanned from global memory otherwise (block-uniform choice)
  __shared__ int wlo[kIThreads / 64], whi[kIThreads / 64];
  __shared__ double wxs[kWin], wys[kWin], wzs[kWin];
  __shared__ int wid[kWin];
  int lo = own ? k0 : INT32_MAX, hi = own ? k1 : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o));
    hi = max(hi, __shfl_xor(hi, o));
  }
  if (pk::lane_id() == 0) {
    wlo[pk::wave_id()] = lo;
    whi[pk::wave_id()] = hi;
  }
  __syncthreads();
  lo = wlo[0];
  hi = whi[0];
#pragma unroll
  for (int w = 1; w < kIThreads / 64; ++w) {
    lo = min(lo, wlo[w]);
    hi = max(hi, whi[w]);
  }
  const int64_t tb = (int64_t)b * ntgt_max;
  const double* X = sx + tb;
  const double* Y = sy + tb;
  const double* Z = sz + tb;
  const int32_t* I = sidx + tb;
  double best = INFINITY;
  int bi = INT32_MAX, bk = -1;
  if (hi > lo && hi - lo <= kWin) {
    for (int j = threadIdx.x; j < hi - lo; j += kIThreads) {
      wxs[j] = X[lo + j];
      wys[j] = Y[lo + j];
      wzs[j] = Z[lo + j];
      wid[j] = I[lo + j];
    }
    __syncthreads();
    if (own) {
      for (int k = k0; k < k1; ++k) {
        const double qx = wxs[k - lo];
        if (qx > qhi) break;
        const double dx = qpx - qx, dy = qpy - wys[k - lo], dz = qpz - wzs[k - lo];
        const double d2 = (dx * dx + dy * dy) + dz * dz;
        const int id = wid[k - lo];
        if (d2 < best || (d2 == best && id < bi)) {
          best = d2;
          bi = id;
          bk = k;
        }
      }
    }
  } else if (own) {
    // candidates in batches of 8 independent loads (no load waits on the previous candidate)
    for (int k = k0; k < nt; k += 8) {
      double qx[8], qy[8], qz[8];
      int id[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool in = k + j < nt;
        const int kk = in ? k + j : k;
        qx[j] = in ? X[kk] : INFINITY;
        qy[j] = Y[kk];
        qz[j] = Z[kk];
        id[j] = I[kk];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double dx = qpx - qx[j], dy = qpy - qy[j], dz = qpz - qz[j];
        const double d2 = (dx * dx + dy * dy) + dz * dz;
        const bool take = d2 < best || (d2 == best && id[j] < bi);
        best = take ? d2 : best;
        bi = take ? id[j] : bi;
        bk = take ? k + j : bk;
      }
      if (qx[7] > qhi) break;
    }
  }
  if (own) {
    const double px = qpx, py = qpy, pz = qpz;
    if (bk >= 0 && best < r * r) {
      const double* c = tgt + 3 * t0;  // shift: the crop's first target point
      const double ax = px - c[0], ay = py - c[1], az = pz - c[2];
      const double bx = X[bk] - c[0], by = Y[bk] - c[1], bz = Z[bk] - c[2];
      acc[0] = 1.0;
      acc[1] = best;
      acc[2] = ax; acc[3] = ay; acc[4] = az;
      acc[5] = bx; acc[6] = by; acc[7] = bz;
      acc[8] = ax * bx; acc[9] = ax * by; acc[10] = ax * bz;
      acc[11] = ay * bx; acc[12] = ay * by; acc[13] = ay * bz;
      acc[14] = az * bx; acc[15] = az * by; acc[16] = az * bz;
    }
  }
  block_sum(acc, part + ((int64_t)b * nblk + blockIdx.x) * kNPart);
}

// grid (B), one wave: partials in block order -> (fitness, rmse); convergence test against the
// previous evaluation; otherwise U = rigid fit of the pairs and T <- U T.
__global__ __launch_bounds__(64) void icp_update_kernel(const int64_t* __restrict__ src_off,
                                                        const double* __restrict__ tgt,
                                                        const int64_t* __restrict__ tgt_off, int nblk, int max_iter,
                                                        double rel_fit, double rel_rmse, IcpState* __restrict__ st,
                                                        const double* __restrict__ part) {
  const int b = blockIdx.x;
  IcpState& S = st[b];
  if (!S.active) return;
  const int lane = threadIdx.x;
  double v = 0.0;
  if (lane < kNPart)
    for (int k = 0; k < nblk; ++k) v += part[((int64_t)b * nblk + k) * kNPart + lane];
  double a[kNPart];
#pragma unroll
  for (int k = 0; k < kNPart; ++k) a[k] = __shfl(v, k);
  if (lane != 0) return;
  const int ns = (int)(src_off[b + 1] - src_off[b]);
  const double cnt = a[0];
  const double fit = (cnt > 0.0 && ns > 0) ? cnt / (double)ns : 0.0;
  const double rmse = cnt > 0.0 ? sqrt(a[1] / cnt) : 0.0;
  const int e = S.iter;
  bool done = false;
  if (e > 0 && fabs(S.fit - fit) < rel_fit && fabs(S.rmse - rmse) < rel_rmse) {
    done = true;
    S.converged = 1;
  } else if (e >= max_iter) {
    done = true;
  }
  S.prev_fit = S.fit;
  S.prev_rmse = S.rmse;
  S.fit = fit;
  S.rmse = rmse;
  if (done) {
    S.active = 0;
    return;
  }
  double U[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  if (cnt > 0.0) {
    const double inv = 1.0 / cnt;
    const double* c = tgt + 3 * tgt_off[b];
    double ms[3], md[3], Sg[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ms[k] = a[2 + k] * inv;
      md[k] = a[5 + k] * inv;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) Sg[r][q] = a[8 + 3 * r + q] * inv - ms[r] * md[q];
    double R[9], t[3];
    pk_rigid::rigid_from_cov(Sg, ms, md, R, t);
    // t was fitted in shifted coordinates: p - c -> R (p - c) + t = R p + (t + c - R c)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      U[4 * r + 0] = R[3 * r + 0];
      U[4 * r + 1] = R[3 * r + 1];
      U[4 * r + 2] = R[3 * r + 2];
      U[4 * r + 3] = (t[r] + c[r]) - ((R[3 * r] * c[0] + R[3 * r + 1] * c[1]) + R[3 * r + 2] * c[2]);
    }
  }
  double Tn[16];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      Tn[4 * r + q] = ((U[4 * r] * S.T[q] + U[4 * r + 1] * S.T[4 + q]) + U[4 * r + 2] * S.T[8 + q]) +
                      U[4 * r + 3] * S.T[12 + q];
#pragma unroll
  for (int k = 0; k < 16; ++k) S.T[k] = Tn[k];
  S.iter = e + 1;
}

// grid (1): number of crops still iterating.
__global__ void icp_count_kernel(const IcpState* __restrict__ st, int B, int32_t* __restrict__ out) {
  int c = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) c += st[b].active;
  c = pk::wave_sum_i32(c);
  if (threadIdx.x == 0) *out = c;
}

// grid (B): T and (fitness, inlier_rmse, iterations, converged).
__global__ void icp_result_kernel(const IcpState* __restrict__ st, double* __restrict__ T,
                                  double* __restrict__ stats) {
  const int b = blockIdx.x;
  if (threadIdx.x < 16) T[16 * b + threadIdx.x] = st[b].T[threadIdx.x];
  if (threadIdx.x == 0) {
    stats[4 * b + 0] = st[b].fit;
    stats[4 * b + 1] = st[b].rmse;
    stats[4 * b + 2] = (double)st[b].iter;
    stats[4 * b + 3] = (double)st[b].converged;
  }
}

}  // namespace

extern "C" int64_t pk_icp_work_size(int B, int nsrc_max, int ntgt_max) {
  if (B <= 0 || nsrc_max < 0 || ntgt_max < 0) return 0;
  return work_bytes_for(B, nsrc_max, ntgt_max);
}

extern "C" int pk_icp_init(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off,
                           const double* T_init, int B, int nsrc_max, int ntgt_max, void* work, int64_t work_bytes,
                           void* stream) {
  PK_REQUIRE(B >= 0 && nsrc_max >= 0 && ntgt_max >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(src && src_off && tgt && tgt_off && T_init && work);
  PK_REQUIRE(work_bytes >= work_bytes_for(B, nsrc_max, ntgt_max));
  hipStream_t s = pk::as_stream(stream);
  const IcpWork w = carve(work, B, nsrc_max, ntgt_max);
  hipLaunchKernelGGL(icp_init_kernel, dim3(B), dim3(64), 0, s, T_init, src_off, tgt_off, nsrc_max, ntgt_max, w.st);
  PK_CHECK_LAUNCH();
  // x order of the targets (and of the source queries under T_init): bucket sort in LDS up to
  // 8192 points per crop, rank counting beyond
  auto sort = [&](const double* p, const int64_t* o, int nm, const double* M, double* x, double* y, double* z,
                  int32_t* idx) -> int {
    if (nm <= 0) return PK_OK;
    int P = 1;
    while (P < nm) P <<= 1;
    if (P <= 8192) {
      hipLaunchKernelGGL(icp_bucket_sort_kernel, dim3(B), dim3(1024), (size_t)P * 12 + kSortBuckets * 8, s, p, o, nm, P,
                         M, x, y, z, idx);
    } else {
      hipLaunchKernelGGL(icp_sort_kernel, dim3((nm + kIThreads - 1) / kIThreads, B), dim3(kIThreads), 0, s, p, o, nm, M,
                         x, y, z, idx);
    }
    PK_CHECK_LAUNCH();
    return PK_OK;
  };
  int rc = sort(tgt, tgt_off, ntgt_max, nullptr, w.sx, w.sy, w.sz, w.sidx);
  if (rc) return rc;
  rc = sort(src, src_off, nsrc_max, T_init, nullptr, nullptr, nullptr, w.perm);
  if (rc) return rc;
  hipLaunchKernelGGL(icp_bucket_kernel, dim3(B), dim3(1024), 0, s, tgt_off, ntgt_max, w.sx, w.st, w.tbl);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_icp_iterate(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off,
                              double max_dist, int max_iter, double rel_fitness, double rel_rmse, int B, int nsrc_max,
                              int ntgt_max, int steps, void* work, int64_t work_bytes, int32_t* active_count,
                              void* stream) {
  PK_REQUIRE(B >= 0 && nsrc_max >= 0 && ntgt_max >= 0 && steps >= 0 && max_iter >= 0 && max_dist > 0.0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(src && src_off && tgt && tgt_off && work);
  PK_REQUIRE(work_bytes >= work_bytes_for(B, nsrc_max, ntgt_max));
  hipStream_t s = pk::as_stream(stream);
  const IcpWork w = carve(work, B, nsrc_max, ntgt_max);
  const int nblk = nsrc_max > 0 ? (nsrc_max + kIThreads - 1) / kIThreads : 1;
  for (int k = 0; k < steps; ++k) {
    hipLaunchKernelGGL(icp_match_kernel, dim3(nblk, B), dim3(kIThreads), 0, s, src, src_off, tgt, tgt_off, max_dist,
                       ntgt_max, nblk, w.st, w.sx, w.sy, w.sz, w.sidx, w.tbl, w.perm, nsrc_max, w.part);
    PK_CHECK_LAUNCH();
    hipLaunchKernelGGL(icp_update_kernel, dim3(B), dim3(64), 0, s, src_off, tgt, tgt_off, nblk, max_iter,
                       rel_fitness, rel_rmse, w.st, w.part);
    PK_CHECK_LAUNCH();
  }
  if (active_count) {
    hipLaunchKernelGGL(icp_count_kernel, dim3(1), dim3(64), 0, s, w.st, B, active_count);
    PK_CHECK_LAUNCH();
  }
  return PK_OK;
}

extern "C" int pk_icp_result(const void* work, int B, double* T, double* stats, void* stream) {
  PK_REQUIRE(B >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(work && T && stats);
  const IcpWork w = carve(const_cast<void*>(work), B, 0, 0);
  hipLaunchKernelGGL(icp_result_kernel, dim3(B), dim3(64), 0, pk::as_stream(stream), w.st, T, stats);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// Blocking driver: init, then batches of `poll` iterations until no crop is active (one
// 4-byte device-to-host read per batch), then the result. Every crop runs at most
// max_iter + 1 evaluations.
extern "C" int pk_icp(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off,
                      const double* T_init, double max_dist, int max_iter, double rel_fitness, double rel_rmse, int B,
                      int nsrc_max, int ntgt_max, int poll, void* work, int64_t work_bytes, int32_t* dev_count,
                      double* T, double* stats, void* stream) {
  PK_REQUIRE(poll > 0 && dev_count);
  int rc = pk_icp_init(src, src_off, tgt, tgt_off, T_init, B, nsrc_max, ntgt_max, work, work_bytes, stream);
  if (rc) return rc;
  if (B == 0) return PK_OK;
  hipStream_t s = pk::as_stream(stream);
  for (int done = 0; done <= max_iter;) {
    const int steps = min(poll, max_iter + 1 - done);
    rc = pk_icp_iterate(src, src_off, tgt, tgt_off, max_dist, max_iter, rel_fitness, rel_rmse, B, nsrc_max, ntgt_max,
                        steps, work, work_bytes, dev_count, stream);
    if (rc) return rc;
    done += steps;
    int32_t active = 0;
    hipError_t e = hipMemcpyAsync(&active, dev_count, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return (int)e;
    if (active == 0) break;
  }
  return pk_icp_result(work, B, T, stats, stream);
}
