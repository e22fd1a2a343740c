// H13 — RANSAC + Umeyama pose fit from correspondences.
//
// Reference: scripts/test_RANSAC.py:288-310 -> Open3D 0.17
// registration_ransac_based_on_correspondence(source = CAD, target = crop, corres,
// max_correspondence_distance = 0.05, PointToPoint(with_scaling=False) = Eigen::umeyama,
// ransac_n = 4, RANSACConvergenceCriteria(4000000, confidence 80000 -> clamped to 1), so
// every hypothesis runs). Per hypothesis: 4 correspondences drawn with replacement, a
// rigid fit, and over ALL correspondences: inlier if ||T s - d||^2 < d_max^2,
// fitness = inliers / n, rmse = sqrt(sum inlier d^2 / inliers); best = max fitness, then
// min rmse (then lowest hypothesis index, making the result deterministic where
// Open3D's OpenMP merge is not).
//
// Hypothesis sampling is deterministic and shared with the oracle (include/posekern.h):
//   corres row of draw j of hypothesis h = splitmix64(seed ^ splitmix64(4h + j)) % n.
// Rigid fit: the maximiser of sum d·(R s) over SO(3) (what Umeyama's SVD with the det
// sign fix returns) via Horn's quaternion: top eigenvector of the symmetric 4x4 N(S),
// cyclic Jacobi in fp64 registers. Scoring: one hypothesis per lane, correspondences
// staged in LDS (fp64) and broadcast; ((R0 s)·... ) + t - d evaluated in fp64 without
// contraction like the C oracle.
#include "common.hpp"
#include "rigid.hpp"

namespace {

using pk_rigid::rigid_fit4;

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ int hyp_index(uint64_t seed, int64_t h, int j, int n) {
  return (int)(splitmix64(seed ^ splitmix64((uint64_t)h * 4u + (uint64_t)j)) % (uint64_t)n);
}


constexpr int kRThreads = 256;
constexpr int kRTile = 2048;  // correspondences per LDS tile (96 KiB fp64)
constexpr int kRChunkMin = 64;  // fewest correspondences a scoring block takes
constexpr int kRTargetBlocks = 2048;  // scoring grid to aim for (8 blocks per CU)

__device__ __forceinline__ bool better(int g1, double r1, int64_t h1, int g2, double r2, int64_t h2) {
  if (g1 != g2) return g1 > g2;
  if (r1 != r2) return r1 < r2;
  return h1 < h2;
}

__device__ __forceinline__ void load_hyp(const double* __restrict__ src, const double* __restrict__ dst,
                                         int64_t ns, int64_t nd, const int32_t* __restrict__ cr, int n, uint64_t seed,
                                         int64_t h,
                                         const int32_t* __restrict__ hyps, double s4[4][3], double d4[4][3]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = hyps ? hyps[4 * h + j] : hyp_index(seed, h, j, n);
    // out-of-range rows are read at 0 (no fault) and reported by ransac_final_kernel
    const int cc = (c >= 0 && c < n) ? c : 0;
    const int64_t si0 = cr[2 * cc], di0 = cr[2 * cc + 1];
    const int64_t si = (si0 >= 0 && si0 < ns) ? si0 : 0, di = (di0 >= 0 && di0 < nd) ? di0 : 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s4[j][k] = src[3 * si + k];
      d4[j][k] = dst[3 * di + k];
    }
  }
}

// Scratch of one pk_ransac call (see pk_ransac_work_size): per crop b the fitted poses
// RT [12][H] (R row-major, then t; hypothesis-contiguous), the per-chunk partial scores
// pg int32 / pe f64 [C][H], and the per-block bests of the reduction [nhb].
struct RansacWork {
  double* RT;
  int32_t* pg;
  double* pe;
  int* bgood;
  double* brmse;
  int64_t* bh;
};

__host__ __device__ inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

__host__ __device__ inline RansacWork carve(void* work, int B, int64_t H, int C, int nhb) {
  char* p = static_cast<char*>(work);
  RansacWork w;
  w.RT = reinterpret_cast<double*>(p);
  p += align256((int64_t)B * 12 * H * 8);
  w.pe = reinterpret_cast<double*>(p);
  p += align256((int64_t)B * C * H * 8);
  w.pg = reinterpret_cast<int32_t*>(p);
  p += align256((int64_t)B * C * H * 4);
  w.brmse = reinterpret_cast<double*>(p);
  p += align256((int64_t)B * nhb * 8);
  w.bh = reinterpret_cast<int64_t*>(p);
  p += align256((int64_t)B * nhb * 8);
  w.bgood = reinterpret_cast<int*>(p);
  return w;
}

inline int chunks_for(int B, int64_t H, int nmax) {
  const int64_t nhb = (H + kRThreads - 1) / kRThreads;
  const int64_t by_n = (nmax + kRChunkMin - 1) / kRChunkMin;
  const int64_t want = (kRTargetBlocks + nhb * B - 1) / (nhb * B > 0 ? nhb * B : 1);
  int64_t C = want < by_n ? want : by_n;
  return (int)(C < 1 ? 1 : C);
}

// pass 1 — grid (ceil(H / 256), B): one hypothesis per thread: draw its 4 correspondences,
// fit [R | t], store it hypothesis-contiguous (coalesced for the scoring pass).
__global__ __launch_bounds__(kRThreads) void ransac_fit_kernel(
    const double* __restrict__ src, const int64_t* __restrict__ src_off, const double* __restrict__ dst,
    const int64_t* __restrict__ dst_off, const int32_t* __restrict__ corres, const int64_t* __restrict__ cor_off,
    const int32_t* __restrict__ hyps, const int64_t* __restrict__ hyp_off, uint64_t seed, int64_t H,
    double* __restrict__ RT) {
  const int b = blockIdx.y;
  const int64_t h = (int64_t)blockIdx.x * kRThreads + threadIdx.x;
  const int64_t c0 = cor_off[b];
  const int n = (int)(cor_off[b + 1] - c0);
  if (h >= H || n < 4) return;
  double s4[4][3], d4[4][3], R[9], t[3];
  load_hyp(src + 3 * src_off[b], dst + 3 * dst_off[b], src_off[b + 1] - src_off[b], dst_off[b + 1] - dst_off[b],
           corres + 2 * c0, n, seed, h, hyps ? hyps + 4 * hyp_off[b] : nullptr, s4, d4);
  rigid_fit4(s4, d4, R, t);
  double* o = RT + (int64_t)b * 12 * H + h;
#pragma unroll
  for (int k = 0; k < 9; ++k) o[k * H] = R[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) o[(9 + k) * H] = t[k];
}

// pass 2 — grid (ceil(H / 256) * C, B): block (hypothesis tile, correspondence chunk c):
// the chunk's pairs are staged in LDS (fp64) and broadcast; each thread scores its
// hypothesis over the chunk in order ((R s + t) - d, no contraction, as the C oracle) and
// writes the chunk's inlier count and error sum. C is sized so one crop's few hypotheses
// (configs[4]: H = 1024) still fill the chip: 4 tiles x 64 chunks = 256 blocks.
__global__ __launch_bounds__(kRThreads) void ransac_score_kernel(
    const double* __restrict__ src, const int64_t* __restrict__ src_off, const double* __restrict__ dst,
    const int64_t* __restrict__ dst_off, const int32_t* __restrict__ corres, const int64_t* __restrict__ cor_off,
    int64_t H, double max_d2, int nhb, int C, int tile_len, const double* __restrict__ RT,
    int32_t* __restrict__ pg, double* __restrict__ pe) {
  extern __shared__ __attribute__((aligned(16))) double sp[];  // [tile][6] (s xyz, d xyz)
  const int b = blockIdx.y;
  const int tile = blockIdx.x % nhb, chunk = blockIdx.x / nhb;
  const int64_t c0 = cor_off[b];
  const int n = (int)(cor_off[b + 1] - c0);
  const int clen = (n + C - 1) / C;
  const int e0 = chunk * clen, e1 = min(n, e0 + clen);
  const int64_t h = (int64_t)tile * kRThreads + threadIdx.x;
  const bool act = h < H && n >= 4;
  const int32_t* cr = corres + 2 * c0;
  const double* S = src + 3 * src_off[b];
  const double* Dp = dst + 3 * dst_off[b];
  const int64_t ns = src_off[b + 1] - src_off[b], nd = dst_off[b + 1] - dst_off[b];
  double R[9], t[3];
  if (act) {
    const double* r = RT + (int64_t)b * 12 * H + h;
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = r[k * H];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = r[(9 + k) * H];
  }
  int good = 0;
  double err = 0.0;
  for (int t0 = e0; t0 < e1; t0 += tile_len) {  // tile_len = the LDS rows allocated
    const int tn = min(tile_len, e1 - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn; e += kRThreads) {
      const int64_t si0 = cr[2 * (t0 + e)], di0 = cr[2 * (t0 + e) + 1];
      const int64_t si = (si0 >= 0 && si0 < ns) ? si0 : 0, di = (di0 >= 0 && di0 < nd) ? di0 : 0;
      sp[6 * e + 0] = S[3 * si];
      sp[6 * e + 1] = S[3 * si + 1];
      sp[6 * e + 2] = S[3 * si + 2];
      sp[6 * e + 3] = Dp[3 * di];
      sp[6 * e + 4] = Dp[3 * di + 1];
      sp[6 * e + 5] = Dp[3 * di + 2];
    }
    __syncthreads();
    if (act) {
      for (int e = 0; e < tn; ++e) {
        const double sx = sp[6 * e], sy = sp[6 * e + 1], sz = sp[6 * e + 2];
        const double ex = (((R[0] * sx + R[1] * sy) + R[2] * sz) + t[0]) - sp[6 * e + 3];
        const double ey = (((R[3] * sx + R[4] * sy) + R[5] * sz) + t[1]) - sp[6 * e + 4];
        const double ez = (((R[6] * sx + R[7] * sy) + R[8] * sz) + t[2]) - sp[6 * e + 5];
        const double d2 = (ex * ex + ey * ey) + ez * ez;
        if (d2 < max_d2) {
          ++good;
          err += d2;
        }
      }
    }
  }
  if (h < H) {
    const int64_t o = ((int64_t)b * C + chunk) * H + h;
    pg[o] = good;
    pe[o] = err;
  }
}

// pass 3 — grid (ceil(H / 256), B): per hypothesis the chunks' counts and error sums in chunk
// order -> (inliers, rmse); the block's best (fitness desc, rmse asc, index asc).
__global__ __launch_bounds__(kRThreads) void ransac_reduce_kernel(const int64_t* __restrict__ cor_off, int64_t H,
                                                                  int nhb, int C, const int32_t* __restrict__ pg,
                                                                  const double* __restrict__ pe, int* __restrict__ bgood,
                                                                  double* __restrict__ brmse, int64_t* __restrict__ bh) {
  __shared__ int sg[4];
  __shared__ double sr[4];
  __shared__ int64_t shh[4];
  const int b = blockIdx.y;
  const int n = (int)(cor_off[b + 1] - cor_off[b]);
  const int64_t h = (int64_t)blockIdx.x * kRThreads + threadIdx.x;
  const bool act = h < H && n >= 4;
  int good = -1;
  double rmse = 0.0;
  int64_t hh = INT64_MAX;
  if (act) {
    int g = 0;
    double err = 0.0;
    for (int c = 0; c < C; ++c) {
      const int64_t o = ((int64_t)b * C + c) * H + h;
      g += pg[o];
      err += pe[o];
    }
    good = g;
    rmse = g ? sqrt(err / g) : 0.0;
    hh = h;
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const int og = __shfl_xor(good, off);
    const double orm = __shfl_xor(rmse, off);
    const int64_t oh = __shfl_xor(hh, off);
    if (better(og, orm, oh, good, rmse, hh)) {
      good = og;
      rmse = orm;
      hh = oh;
    }
  }
  if (pk::lane_id() == 0) {
    sg[pk::wave_id()] = good;
    sr[pk::wave_id()] = rmse;
    shh[pk::wave_id()] = hh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (better(sg[w], sr[w], shh[w], good, rmse, hh)) {
        good = sg[w];
        rmse = sr[w];
        hh = shh[w];
      }
    const int64_t o = (int64_t)b * nhb + blockIdx.x;
    bgood[o] = good;
    brmse[o] = rmse;
    bh[o] = hh;
  }
}

// grid (B), block 256: best over blocks; the winner's stored pose -> T (4x4 row-major), stats.
// The index check of every crop (status[b] = 1 when a correspondence row lies outside its crop's
// source / target points, or a caller-given hypothesis row outside [0, n): those reads went to
// row 0 instead of faulting) — written for every crop, so status needs no initialisation.
__global__ __launch_bounds__(256) void ransac_final_kernel(const int64_t* __restrict__ cor_off, int64_t H, int nblk,
                                                           const double* __restrict__ RT,
                                                           const int* __restrict__ bgood,
                                                           const double* __restrict__ brmse,
                                                           const int64_t* __restrict__ bh, double* __restrict__ T,
                                                           double* __restrict__ stats, const int32_t* __restrict__ corres,
                                                           const int64_t* __restrict__ src_off,
                                                           const int64_t* __restrict__ dst_off,
                                                           const int32_t* __restrict__ hyps,
                                                           const int64_t* __restrict__ hyp_off,
                                                           int32_t* __restrict__ status) {
  __shared__ int sg[4];
  __shared__ double sr[4];
  __shared__ int64_t shh[4];
  const int b = blockIdx.x;
  if (status) {
    const int64_t c0 = cor_off[b], nc = cor_off[b + 1] - c0;
    const int64_t ns = src_off[b + 1] - src_off[b], nd = dst_off[b + 1] - dst_off[b];
    int bad = 0;
    for (int64_t e = threadIdx.x; e < nc; e += 256) {
      const int64_t si = corres[2 * (c0 + e)], di = corres[2 * (c0 + e) + 1];
      bad |= (si < 0 || si >= ns || di < 0 || di >= nd) ? 1 : 0;
    }
    if (hyps && nc >= 4)
      for (int64_t e = threadIdx.x; e < 4 * H; e += 256) {
        const int c = hyps[4 * hyp_off[b] + e];
        bad |= (c < 0 || c >= nc) ? 1 : 0;
      }
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) status[b] = bad;
  }
  int good = -1;
  double rmse = 0.0;
  int64_t hh = INT64_MAX;
  for (int k = threadIdx.x; k < nblk; k += 256) {
    const int64_t o = (int64_t)b * nblk + k;
    if (better(bgood[o], brmse[o], bh[o], good, rmse, hh)) {
      good = bgood[o];
      rmse = brmse[o];
      hh = bh[o];
    }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    const int og = __shfl_xor(good, off);
    const double orm = __shfl_xor(rmse, off);
    const int64_t oh = __shfl_xor(hh, off);
    if (better(og, orm, oh, good, rmse, hh)) {
      good = og;
      rmse = orm;
      hh = oh;
    }
  }
  if (pk::lane_id() == 0) {
    sg[pk::wave_id()] = good;
    sr[pk::wave_id()] = rmse;
    shh[pk::wave_id()] = hh;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int w = 1; w < 4; ++w)
    if (better(sg[w], sr[w], shh[w], good, rmse, hh)) {
      good = sg[w];
      rmse = sr[w];
      hh = shh[w];
    }
  const int n = (int)(cor_off[b + 1] - cor_off[b]);
  double* Tb = T + 16 * b;
  for (int k = 0; k < 16; ++k) Tb[k] = (k % 5 == 0) ? 1.0 : 0.0;
  stats[3 * b + 0] = 0.0;
  stats[3 * b + 1] = 0.0;
  stats[3 * b + 2] = -1.0;
  if (good < 0 || hh == INT64_MAX || n < 4) return;
  const double* r = RT + (int64_t)b * 12 * H + hh;
  for (int i = 0; i < 3; ++i) {
    for (int c = 0; c < 3; ++c) Tb[4 * i + c] = r[(3 * i + c) * H];
    Tb[4 * i + 3] = r[(9 + i) * H];
  }
  stats[3 * b + 0] = good > 0 ? (double)good / (double)n : 0.0;
  stats[3 * b + 1] = rmse;
  stats[3 * b + 2] = (double)hh;
}

}  // namespace

extern "C" int64_t pk_ransac_work_size(int B, int64_t H, int nmax) {
  if (B <= 0 || H < 0 || nmax < 0) return 0;
  const int C = chunks_for(B, H, nmax);
  const int64_t nhb = (H + kRThreads - 1) / kRThreads;
  return align256((int64_t)B * 12 * H * 8) + align256((int64_t)B * C * H * 8) + align256((int64_t)B * C * H * 4) +
         2 * align256((int64_t)B * nhb * 8) + align256((int64_t)B * nhb * 4);
}

extern "C" int pk_ransac(const double* src, const int64_t* src_off, const double* dst, const int64_t* dst_off,
                         const int32_t* corres, const int64_t* cor_off, const int32_t* hyps, const int64_t* hyp_off,
                         uint64_t seed, int64_t H, double max_dist, int B, int nmax, void* work, int64_t work_bytes,
                         double* T, double* stats, int32_t* status, void* stream) {
  PK_REQUIRE(B >= 0 && H >= 0 && max_dist > 0.0 && nmax >= 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(src && src_off && dst && dst_off && corres && cor_off && work && T && stats);
  PK_REQUIRE(hyps == nullptr || hyp_off != nullptr);
  PK_REQUIRE(work_bytes >= pk_ransac_work_size(B, H, nmax));
  hipStream_t s = pk::as_stream(stream);
  const int nhb = (int)((H + kRThreads - 1) / kRThreads);
  const int C = chunks_for(B, H, nmax);
  const RansacWork w = carve(work, B, H, C, nhb);
  if (nhb > 0) {
    hipLaunchKernelGGL(ransac_fit_kernel, dim3(nhb, B), dim3(kRThreads), 0, s, src, src_off, dst, dst_off, corres,
                       cor_off, hyps, hyp_off, seed, H, w.RT);
    PK_CHECK_LAUNCH();
    const int tile = min(kRTile, (nmax + C - 1) / C > 0 ? (nmax + C - 1) / C : 1);
    hipLaunchKernelGGL(ransac_score_kernel, dim3(nhb * C, B), dim3(kRThreads), tile * 6 * sizeof(double), s, src,
                       src_off, dst, dst_off, corres, cor_off, H, max_dist * max_dist, nhb, C, tile, w.RT, w.pg, w.pe);
    PK_CHECK_LAUNCH();
    hipLaunchKernelGGL(ransac_reduce_kernel, dim3(nhb, B), dim3(kRThreads), 0, s, cor_off, H, nhb, C, w.pg, w.pe,
                       w.bgood, w.brmse, w.bh);
    PK_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(ransac_final_kernel, dim3(B), dim3(256), 0, s, cor_off, H, nhb, w.RT, w.bgood, w.brmse, w.bh,
                     T, stats, corres, src_off, dst_off, hyps, hyp_off, status);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
