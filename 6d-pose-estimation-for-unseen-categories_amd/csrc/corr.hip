// Correspondence post-processing and per-crop labels:
//
//  pk_rigidity_filter  H11 second half — fmap2pointmap_solvers/spacial_filtering.py:42-75:
//      three rounds; in each, for the surviving candidates (c_i, p_i)
//        score_j = mean_i | ||CAD[c_i] - CAD[c_j]|| - ||PC[p_i] - PC[p_j]|| |
//      keep score < tau * diam with tau = 0.3, 0.15, then 0.055 (0.065 if 0.055 keeps
//      nothing). Computed pairwise on the fly (the reference materialises [n,n,3] twice
//      per round); order of survivors preserved.
//  pk_inlier_ratio     H12 — utils/utils.py:81-105: mean(||CAD[c]-PC_al[p]|| < thr), 0 if
//      no correspondences (f32, correctly rounded sqrt).
//  pk_cgt_lstsq        H15 — utils/utils.py:67-79 C_from_sparse_P: least squares
//      evecs2[P1] X = evecs1[P0] via fp64 normal equations + Gauss-Jordan (partial pivoting).
#include "common.hpp"

namespace {

constexpr int kTile = 1024;

// grid (ceil(nmax/256), B), block 256: score for every listed candidate of crop b.
__global__ __launch_bounds__(256) void rigid_score_kernel(const int64_t* __restrict__ list, int ldl,
                                                          const int32_t* __restrict__ nlist,
                                                          const int64_t* __restrict__ cand, int ldc,
                                                          const float* __restrict__ cad, int ldcad,
                                                          const float* __restrict__ pc, int ldpc,
                                                          float* __restrict__ score) {
  __shared__ float s[kTile * 6];
  const int b = blockIdx.y;
  const int n = nlist[b];
  const int jj = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x * 256 >= n) return;
  const int64_t* L = list + (int64_t)b * ldl;
  const int64_t* Cd = cand + (int64_t)b * ldc * 2;
  const float* CA = cad + (int64_t)b * ldcad * 3;
  const float* PCb = pc + (int64_t)b * ldpc * 3;
  float ax = 0, ay = 0, az = 0, px = 0, py = 0, pz = 0;
  if (jj < n) {
    const int64_t k = L[jj];
    const int64_t c = Cd[2 * k], p = Cd[2 * k + 1];
    ax = CA[3 * c]; ay = CA[3 * c + 1]; az = CA[3 * c + 2];
    px = PCb[3 * p]; py = PCb[3 * p + 1]; pz = PCb[3 * p + 2];
  }
  float acc = 0.f;
  for (int t0 = 0; t0 < n; t0 += kTile) {
    const int tn = min(kTile, n - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn; e += 256) {
      const int64_t k = L[t0 + e];
      const int64_t c = Cd[2 * k], p = Cd[2 * k + 1];
      s[6 * e + 0] = CA[3 * c]; s[6 * e + 1] = CA[3 * c + 1]; s[6 * e + 2] = CA[3 * c + 2];
      s[6 * e + 3] = PCb[3 * p]; s[6 * e + 4] = PCb[3 * p + 1]; s[6 * e + 5] = PCb[3 * p + 2];
    }
    __syncthreads();
    if (jj < n) {
      for (int e = 0; e < tn; ++e) {
        const float dx = s[6 * e] - ax, dy = s[6 * e + 1] - ay, dz = s[6 * e + 2] - az;
        const float ex = s[6 * e + 3] - px, ey = s[6 * e + 4] - py, ez = s[6 * e + 5] - pz;
        const float a = __builtin_amdgcn_sqrtf((dx * dx + dy * dy) + dz * dz);
        const float bb = __builtin_amdgcn_sqrtf((ex * ex + ey * ey) + ez * ez);
        acc += fabsf(a - bb);
      }
    }
  }
  if (jj < n) score[(int64_t)b * ldl + jj] = acc / (float)n;
}

// Symmetric scoring: the pair term |‖CAD_i − CAD_j‖ − ‖PC_i − PC_j‖| is the same for (i, j) and
// (j, i), so each unordered pair is evaluated once (two sqrt per pair instead of four). Grid
// (T (T + 1) / 2, B) over 64 x 64 tile pairs I <= J of the current list (T = ceil(nmax / 64));
// block 256 = 16 x 16 threads, 4 x 4 pairs each. A block writes, for every list entry x of tile
// I, the sum over tile J (part[b][J][x]) and, when I != J, for every entry of tile J the sum over
// tile I (part[b][I][x]): each (tile, entry) slot is written exactly once, and rigid_reduce_kernel
// adds the slots in tile order (deterministic).
constexpr int kRT = 64;
__global__ __launch_bounds__(256) void rigid_pair_kernel(const int64_t* __restrict__ list, int ldl,
                                                         const int32_t* __restrict__ nlist,
                                                         const int64_t* __restrict__ cand, int ldc,
                                                         const float* __restrict__ cad, int ldcad,
                                                         const float* __restrict__ pc, int ldpc, int T,
                                                         float* __restrict__ part) {
  __shared__ float si[kRT][7], sj[kRT][7];
  __shared__ float red[16][kRT + 1];
  const int b = blockIdx.y;
  const int n = nlist[b];
  const int t = blockIdx.x;
  int J = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((J + 1) * (J + 2) / 2 <= t) ++J;
  while (J * (J + 1) / 2 > t) --J;
  const int I = t - J * (J + 1) / 2;
  if (J * kRT >= n) return;  // block-uniform: tile outside this round's list
  const int64_t* L = list + (int64_t)b * ldl;
  const int64_t* Cd = cand + (int64_t)b * ldc * 2;
  const float* CA = cad + (int64_t)b * ldcad * 3;
  const float* PCb = pc + (int64_t)b * ldpc * 3;
  const int tid = threadIdx.x;
  if (tid < 2 * kRT) {
    const int e = tid & (kRT - 1);
    const int x = (tid < kRT ? I : J) * kRT + e;
    float (*dst)[7] = tid < kRT ? si : sj;
    if (x < n) {
      const int64_t k = L[x];
      const int64_t c = Cd[2 * k], q = Cd[2 * k + 1];
      dst[e][0] = CA[3 * c]; dst[e][1] = CA[3 * c + 1]; dst[e][2] = CA[3 * c + 2];
      dst[e][3] = PCb[3 * q]; dst[e][4] = PCb[3 * q + 1]; dst[e][5] = PCb[3 * q + 2];
      dst[e][6] = 1.f;
    } else {
      dst[e][0] = dst[e][1] = dst[e][2] = dst[e][3] = dst[e][4] = dst[e][5] = 0.f;
      dst[e][6] = 0.f;
    }
  }
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  float ra[4] = {0.f, 0.f, 0.f, 0.f}, ca[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ty * 4 + r;
    const float ax = si[i][0], ay = si[i][1], az = si[i][2], px = si[i][3], py = si[i][4], pz = si[i][5];
    const float vi = si[i][6];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = tx * 4 + c;
      const float dx = sj[j][0] - ax, dy = sj[j][1] - ay, dz = sj[j][2] - az;
      const float ex = sj[j][3] - px, ey = sj[j][4] - py, ez = sj[j][5] - pz;
      const float a = __builtin_amdgcn_sqrtf((dx * dx + dy * dy) + dz * dz);
      const float bb = __builtin_amdgcn_sqrtf((ex * ex + ey * ey) + ez * ez);
      const float v = fabsf(a - bb) * (vi * sj[j][6]);  // invalid entries contribute 0
      ra[r] += v;
      ca[c] += v;
    }
  }
  float* P = part + (int64_t)b * T * ldl;
  // row sums of tile I over tile J: reduce over tx in order
#pragma unroll
  for (int r = 0; r < 4; ++r) red[tx][ty * 4 + r] = ra[r];
  __syncthreads();
  if (tid < kRT) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += red[q][tid];
    const int x = I * kRT + tid;
    if (x < n) P[(int64_t)J * ldl + x] = acc;
  }
  if (I == J) return;  // block-uniform; the diagonal tile's row sums already cover both orders
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 4; ++c) red[ty][tx * 4 + c] = ca[c];
  __syncthreads();
  if (tid < kRT) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += red[q][tid];
    const int x = J * kRT + tid;
    if (x < n) P[(int64_t)I * ldl + x] = acc;
  }
}

// ---- Packed coordinates, 128 x 128 pair tiles (rounds 2 and 3 of the filter).
// Round 2's rigid_pair_kernel spent most of a block on its prologue: every entry of both tiles
// was a dependent gather list -> cand -> cad / pc (three global loads in a chain) for only 16
// pairs per thread. Here the coordinates of the current list live in a packed array (one
// 32-B record per entry: {cad_x, pc_x, cad_y, pc_y, cad_z, pc_z, valid, 0}); the first round's is
// gathered once (rigid_gather_kernel) and each compaction carries the survivors' records
// along (rigid_compact_pts_kernel), so a pair block loads its two tiles with plain 16-B loads.
// The pair term is two rigid_dist (FMA sums of squares, v_sqrt_f32) and |a - b| folded into the
// row and column sums as a source modifier; kPS x kPS (16 x 16) pairs per thread.
constexpr int kRT2 = 256;            // entries per tile (rounds 2, 3)
constexpr int kPS = kRT2 / 16;       // entries per thread per side
typedef float rf2 __attribute__((ext_vector_type(2)));

struct __attribute__((aligned(16))) RigidRec {
  rf2 x, y;  // {cad_x, pc_x}, {cad_y, pc_y}
  rf2 z, v;  // {cad_z, pc_z}, {valid, 0}
};

// grid (ceil(nmax/256), B): list[i] = i and the packed record of candidate i (round 1).
__global__ __launch_bounds__(256) void rigid_gather_kernel(const int64_t* __restrict__ cand, int ldc,
                                                           const int32_t* __restrict__ ncand,
                                                           const float* __restrict__ cad, int ldcad,
                                                           const float* __restrict__ pc, int ldpc,
                                                           int64_t* __restrict__ list, RigidRec* __restrict__ pts) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ncand[b]) return;
  const int64_t c = cand[((int64_t)b * ldc + i) * 2], p = cand[((int64_t)b * ldc + i) * 2 + 1];
  const float* CA = cad + ((int64_t)b * ldcad + c) * 3;
  const float* PC = pc + ((int64_t)b * ldpc + p) * 3;
  RigidRec r;
  r.x = rf2{CA[0], PC[0]};
  r.y = rf2{CA[1], PC[1]};
  r.z = rf2{CA[2], PC[2]};
  r.v = rf2{1.f, 0.f};
  pts[(int64_t)b * ldc + i] = r;
  list[(int64_t)b * ldc + i] = i;
}

// One side of the pair term: the distance ||p - q|| with the squares summed as
// (dx^2 + dy^2) + dz^2 in two fused multiply-adds (dx dx, then + dy dy, then + dz dz: each
// partial sum rounded once; the reference's unfused form rounds the squares too, a <= 1-ulp
// difference per term, below the f32 error of the n-term mean it feeds).
__device__ __forceinline__ float rigid_dist(float px, float py, float pz, float qx, float qy, float qz) {
  const float dx = qx - px, dy = qy - py, dz = qz - pz;
  return __builtin_amdgcn_sqrtf(__builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)));
}

// kPS x kPS pairs of one thread: rows i = ty + 16 r, columns j = tx + 16 c. ra[r]: this thread's
// row sums (over its kPS columns), ca[c]: its column sums. Scalar VALU: on MI355X a v_pk_*_f32
// costs the issue of two scalar ops (measured: round 3's packed form ran at the scalar rate).
template <bool EDGE>
__device__ __forceinline__ void rigid_tile_pairs(const RigidRec* __restrict__ si, const RigidRec* __restrict__ sj,
                                                 int tx, int ty, float (&ra)[kPS], float (&ca)[kPS]) {
  float ax[kPS], ay[kPS], az[kPS], px[kPS], py[kPS], pz[kPS], cv[kPS];  // column entries
#pragma unroll
  for (int c = 0; c < kPS; ++c) {
    const RigidRec q = sj[tx + 16 * c];
    ax[c] = q.x.x; ay[c] = q.y.x; az[c] = q.z.x;
    px[c] = q.x.y; py[c] = q.y.y; pz[c] = q.z.y;
    cv[c] = q.v.x;
  }
#pragma unroll 2
  for (int r = 0; r < kPS; ++r) {
    const RigidRec ci = si[ty + 16 * r];
    float rs = 0.f;
#pragma unroll
    for (int c = 0; c < kPS; ++c) {
      const float a = rigid_dist(ci.x.x, ci.y.x, ci.z.x, ax[c], ay[c], az[c]);
      const float bb = rigid_dist(ci.x.y, ci.y.y, ci.z.y, px[c], py[c], pz[c]);
      float v = fabsf(a - bb);
      if (EDGE) v = v * (cv[c] * ci.v.x);  // invalid entries contribute 0
      rs += v;
      ca[c] += v;
    }
    ra[r] = rs;
  }
}

// The same kPS x kPS pairs with the crop half from a table: the survivors of a round keep
// nn_query's order, so a tile's entries come in runs that share one crop point (what is left of
// each group of 5). tab[u * RJ + w] = rigid_dist(run u of tile I, run w of tile J) is computed
// once per run pair from the runs' own (bitwise-equal) coordinates, so the looked-up value is
// bit-identical to rigid_tile_pairs' second rigid_dist; si[].v.y carries u * RJ, sj[].v.y w.
template <bool EDGE>
__device__ __forceinline__ void rigid_tile_pairs_tab(const RigidRec* __restrict__ si, const RigidRec* __restrict__ sj,
                                                     const float* __restrict__ tab, int tx, int ty, float (&ra)[kPS],
                                                     float (&ca)[kPS]) {
  float ax[kPS], ay[kPS], az[kPS], cv[kPS];
  int cj[kPS];
#pragma unroll
  for (int c = 0; c < kPS; ++c) {
    const RigidRec q = sj[tx + 16 * c];
    ax[c] = q.x.x; ay[c] = q.y.x; az[c] = q.z.x;
    cv[c] = q.v.x;
    cj[c] = __float_as_int(q.v.y);
  }
#pragma unroll 2
  for (int r = 0; r < kPS; ++r) {
    const RigidRec ci = si[ty + 16 * r];
    const float* __restrict__ trow = tab + __float_as_int(ci.v.y);
    float rs = 0.f;
#pragma unroll
    for (int c = 0; c < kPS; ++c) {
      const float a = rigid_dist(ci.x.x, ci.y.x, ci.z.x, ax[c], ay[c], az[c]);
      float v = fabsf(a - trow[cj[c]]);
      if (EDGE) v = v * (cv[c] * ci.v.x);
      rs += v;
      ca[c] += v;
    }
    ra[r] = rs;
  }
}

constexpr int kTab = 8192;  // run-pair table entries (32 KB of LDS)

// Grid (T (T + 1) / 2, B) over kRT2 x kRT2 tile pairs I <= J (T = ceil(nmax / kRT2)), XCD-aware
// (a crop's tile pairs share one XCD's L2); block 256 = 16 x 16 threads. As rigid_pair_kernel:
// part[b][J][x] = sum over tile J of entry x of tile I, and for I != J part[b][I][y] for the
// entries y of tile J; every slot written once, summed in tile order by rigid_reduce_kernel.
// Fixed-order reductions (16-lane butterflies, then the 4 waves' column partials in wave order).
// When the two tiles' crop-point runs give at most kTab run pairs (and use_tab), the crop
// distances come from the run-pair table (rigid_tile_pairs_tab): one crop sqrt per run pair
// instead of per entry pair; otherwise (a general candidate order, sparse survivors) both
// distances per pair. Either way the pair values, and so the partial sums, are the same bits.
__global__ __launch_bounds__(256) void rigid_pair2_kernel(const int32_t* __restrict__ nlist, int ldl,
                                                          const RigidRec* __restrict__ pts, int T,
                                                          float* __restrict__ part, int use_tab) {
  __shared__ RigidRec si[kRT2], sj[kRT2];
  __shared__ float red[4][kRT2];
  __shared__ float tab[kTab];
  __shared__ float rq[2][3][kRT2];  // the runs' crop points (tile I, tile J)
  __shared__ int rcnt[2][4];        // runs starting in each wave's 64 entries
  const int3 lb = pk::xcd_block3();
  const int b = lb.y;
  const int n = nlist[b];
  const int t = lb.x;
  int J = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((J + 1) * (J + 2) / 2 <= t) ++J;
  while (J * (J + 1) / 2 > t) --J;
  const int I = t - J * (J + 1) / 2;
  if (J * kRT2 >= n) return;  // block-uniform: tile outside this round's list
  const RigidRec* P0 = pts + (int64_t)b * ldl;
  const int tid = threadIdx.x;
  for (int e2 = tid; e2 < 2 * kRT2; e2 += 256) {
    const int e = e2 & (kRT2 - 1);
    const int x = (e2 < kRT2 ? I : J) * kRT2 + e;
    RigidRec r;
    if (x < n) r = P0[x];
    else r.x = r.y = r.z = r.v = rf2{0.f, 0.f};
    (e2 < kRT2 ? si : sj)[e] = r;
  }
  __syncthreads();
  bool tbl = false;
  if (use_tab) {  // block-uniform
    // runs of bitwise-equal crop points; entry tid of each tile (kRT2 == blockDim)
    const int w = pk::wave_id(), lane = pk::lane_id();
    bool head[2];
    int loc[2];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const RigidRec* s = sd ? sj : si;
      const RigidRec c = s[tid];
      bool h = tid == 0;
      if (tid > 0) {
        const RigidRec p = s[tid - 1];
        h = __float_as_uint(c.x.y) != __float_as_uint(p.x.y) || __float_as_uint(c.y.y) != __float_as_uint(p.y.y) ||
            __float_as_uint(c.z.y) != __float_as_uint(p.z.y);
      }
      const uint64_t bal = __ballot(h);
      loc[sd] = __popcll(bal & ((1ull << lane) - 1ull));  // heads before this entry in its wave
      if (lane == 0) rcnt[sd][w] = __popcll(bal);
      head[sd] = h;
    }
    __syncthreads();
    int rid[2], R[2];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      int off = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        off += q < w ? rcnt[sd][q] : 0;
        tot += rcnt[sd][q];
      }
      rid[sd] = off + loc[sd] + (head[sd] ? 0 : -1);  // run of this entry
      R[sd] = tot;
      if (head[sd]) {
        const RigidRec c = (sd ? sj : si)[tid];
        rq[sd][0][rid[sd]] = c.x.y;
        rq[sd][1][rid[sd]] = c.y.y;
        rq[sd][2][rid[sd]] = c.z.y;
      }
    }
    tbl = R[0] * R[1] <= kTab;
    if (tbl) {
      si[tid].v.y = __int_as_float(rid[0] * R[1]);
      sj[tid].v.y = __int_as_float(rid[1]);
    }
    __syncthreads();
    if (tbl) {
      const int RJ = R[1], per = kRT2 / RJ;
      const int cj = tid % RJ, r0 = tid / RJ;
      if (r0 < per) {
        const float qx = rq[1][0][cj], qy = rq[1][1][cj], qz = rq[1][2][cj];
        for (int u = r0; u < R[0]; u += per)
          tab[u * RJ + cj] = rigid_dist(rq[0][0][u], rq[0][1][u], rq[0][2][u], qx, qy, qz);
      }
      __syncthreads();
    }
  }
  const int tx = tid & 15, ty = tid >> 4;
  float ra[kPS], ca[kPS];
#pragma unroll
  for (int r = 0; r < kPS; ++r) ra[r] = ca[r] = 0.f;
  const bool edge = (J + 1) * kRT2 > n;
  if (tbl) {
    if (edge) rigid_tile_pairs_tab<true>(si, sj, tab, tx, ty, ra, ca);
    else rigid_tile_pairs_tab<false>(si, sj, tab, tx, ty, ra, ca);
  } else {
    if (edge) rigid_tile_pairs<true>(si, sj, tx, ty, ra, ca);
    else rigid_tile_pairs<false>(si, sj, tx, ty, ra, ca);
  }
  float* P = part + (int64_t)b * T * ldl;
  // row sums of tile I over tile J: the 16 tx lanes are one DPP row (quad_perm / half-mirror /
  // mirror adds: VALU only, no LDS round trips); lane tx = 0's association order is fixed
#pragma unroll
  for (int r = 0; r < kPS; ++r) {
    float v = ra[r];
    v += __int_as_float((int)PK_DPP(__float_as_int(v), 0xB1));
    v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x4E));
    v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x141));
    v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x140));
    const int x = I * kRT2 + ty + 16 * r;
    if (tx == 0 && x < n) P[(int64_t)J * ldl + x] = v;
  }
  if (I == J) return;  // block-uniform; the diagonal tile's row sums already cover both orders
  // column sums of tile J over tile I: the wave's 4 ty rows by butterfly, then the 4 waves in order
  const int w = pk::wave_id();
#pragma unroll
  for (int c = 0; c < kPS; ++c) {
    float v = ca[c];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if ((tid & 63) < 16) red[w][tx + 16 * c] = v;
  }
  __syncthreads();
  for (int e = tid; e < kRT2; e += 256) {
    const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    const int x = J * kRT2 + e;
    if (x < n) P[(int64_t)I * ldl + x] = v;
  }
}

// ---- Round 1 (round-4 path): the candidates of nn_query come in groups of K = 5 that share one
// crop point (spacial_filtering.py:36-38: p2p = stack([idx, idx_p]).reshape(2, -1), crop point
// p repeated for its 5 nearest CAD points), so the crop half of the pair term,
// ||PC[p_i] - PC[p_j]||, is the same for all 25 pairs of two groups. Tiles of 64 groups
// (320 entries); thread (tx, ty) of 16 x 16 owns row groups ty + 16 r and column groups tx + 16 h
// (r, h < 4): per group pair one crop distance, then 25 CAD distances. The pair value |a - b| is
// bit-identical to rigid_pair2_kernel's (same rigid_dist); only the association of the sums
// differs (fixed).
// A tile pair whose groups do not share their crop coordinates (a caller passing another
// candidate order) takes the general form of the same loop (both sqrt per pair), so any
// candidate list is scored correctly. Partials as rigid_pair2_kernel, tiles of kRG entries.
constexpr int kGK = 5;              // candidates per crop point (nn_query's K)
constexpr int kGT = 64;             // groups per tile
constexpr int kGS = kGT / 16;       // groups per thread per side (thread (tx, ty) of 16 x 16)
constexpr int kRG = kGK * kGT;      // entries per tile

// Thread (tx, ty): row groups ty + 16 r and column groups tx + 16 h (r, h < kGS): kGS^2 group
// pairs = 25 kGS^2 pairs (400), so the per-thread prologue and the row / column reductions stay
// a few % of the pair work (12.7 VALU per pair with 100 pairs per thread).
template <bool SHARED, bool EDGE>
__device__ __forceinline__ void rigid_group_pairs(const RigidRec* __restrict__ si, const RigidRec* __restrict__ sj,
                                                  int tx, int ty, float (&ra)[kGS][kGK], float (&ca)[kGS][kGK]) {
  float cx[kGS][kGK], cy[kGS][kGK], cz[kGS][kGK], cv[kGS][kGK];  // column entries' CAD point, validity
  float qx[kGS], qy[kGS], qz[kGS];                                 // column groups' crop point
#pragma unroll
  for (int h = 0; h < kGS; ++h) {
#pragma unroll
    for (int l = 0; l < kGK; ++l) {
      const RigidRec q = sj[kGK * (tx + 16 * h) + l];
      cx[h][l] = q.x.x;
      cy[h][l] = q.y.x;
      cz[h][l] = q.z.x;
      cv[h][l] = q.v.x;
      if (l == 0) {
        qx[h] = q.x.y;
        qy[h] = q.y.y;
        qz[h] = q.z.y;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kGS; ++r) {
    const int P = ty + 16 * r;
    float bq[kGS];
    if (SHARED) {  // one crop distance per (P, Q_h)
      const RigidRec p = si[kGK * P];
#pragma unroll
      for (int h = 0; h < kGS; ++h) bq[h] = rigid_dist(p.x.y, p.y.y, p.z.y, qx[h], qy[h], qz[h]);
    }
#pragma unroll
    for (int k = 0; k < kGK; ++k) {
      const RigidRec ci = si[kGK * P + k];
#pragma unroll
      for (int h = 0; h < kGS; ++h)
#pragma unroll
        for (int l = 0; l < kGK; ++l) {
          const float a = rigid_dist(ci.x.x, ci.y.x, ci.z.x, cx[h][l], cy[h][l], cz[h][l]);
          float b;
          if (SHARED) {
            b = bq[h];
          } else {  // (general candidate order: the column entry's own crop point, from LDS)
            const RigidRec q = sj[kGK * (tx + 16 * h) + l];
            b = rigid_dist(ci.x.y, ci.y.y, ci.z.y, q.x.y, q.y.y, q.z.y);
          }
          float v = fabsf(a - b);
          if (EDGE) v = v * (cv[h][l] * ci.v.x);  // invalid entries contribute 0
          ra[r][k] += v;
          ca[h][l] += v;
        }
    }
  }
}

// Grid (T (T + 1) / 2, B) over kRG x kRG tile pairs I <= J (T = ceil(nmax / kRG)), XCD-aware;
// block 256. Writes part[b][J][x] (x in tile I) and, for I != J, part[b][I][y] (y in tile J).
__global__ __launch_bounds__(256) void rigid_group_kernel(const int32_t* __restrict__ nlist, int ldl,
                                                          const RigidRec* __restrict__ pts, int T,
                                                          float* __restrict__ part) {
  __shared__ RigidRec si[kRG], sj[kRG];
  __shared__ float red[4][kRG];
  const int3 lb = pk::xcd_block3();
  const int b = lb.y;
  const int n = nlist[b];
  const int t = lb.x;
  int J = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((J + 1) * (J + 2) / 2 <= t) ++J;
  while (J * (J + 1) / 2 > t) --J;
  const int I = t - J * (J + 1) / 2;
  if (J * kRG >= n) return;  // block-uniform: tile outside the list
  const RigidRec* P0 = pts + (int64_t)b * ldl;
  const int tid = threadIdx.x;
  for (int e = tid; e < 2 * kRG; e += 256) {
    const int loc = e < kRG ? e : e - kRG;
    const int x = (e < kRG ? I : J) * kRG + loc;
    RigidRec r;
    if (x < n) r = P0[x];
    else r.x = r.y = r.z = r.v = rf2{0.f, 0.f};
    (e < kRG ? si : sj)[loc] = r;
  }
  __syncthreads();
  // do the valid members of every group carry their group's crop coordinates (bitwise)?
  int split = 0;
  if (tid < 2 * kGT) {
    const RigidRec* g = (tid < kGT ? si : sj) + kGK * (tid & (kGT - 1));
    for (int k = 1; k < kGK; ++k)
      if (g[k].v.x != 0.f && (__float_as_uint(g[k].x.y) != __float_as_uint(g[0].x.y) ||
                              __float_as_uint(g[k].y.y) != __float_as_uint(g[0].y.y) ||
                              __float_as_uint(g[k].z.y) != __float_as_uint(g[0].z.y)))
        split = 1;
  }
  const bool shared = !__syncthreads_or(split);
  const bool edge = (J + 1) * kRG > n;
  const int tx = tid & 15, ty = tid >> 4;
  float ra[kGS][kGK], ca[kGS][kGK];
#pragma unroll
  for (int r = 0; r < kGS; ++r)
#pragma unroll
    for (int l = 0; l < kGK; ++l) ra[r][l] = ca[r][l] = 0.f;
  if (shared) {
    if (edge) rigid_group_pairs<true, true>(si, sj, tx, ty, ra, ca);
    else rigid_group_pairs<true, false>(si, sj, tx, ty, ra, ca);
  } else {
    if (edge) rigid_group_pairs<false, true>(si, sj, tx, ty, ra, ca);
    else rigid_group_pairs<false, false>(si, sj, tx, ty, ra, ca);
  }
  float* Pp = part + (int64_t)b * T * ldl;
  // row sums of tile I over tile J: the 16 tx lanes of a DPP row, fixed association
#pragma unroll
  for (int r = 0; r < kGS; ++r) {
#pragma unroll
    for (int k = 0; k < kGK; ++k) {
      float v = ra[r][k];
      v += __int_as_float((int)PK_DPP(__float_as_int(v), 0xB1));
      v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x4E));
      v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x141));
      v += __int_as_float((int)PK_DPP(__float_as_int(v), 0x140));
      const int x = I * kRG + kGK * (ty + 16 * r) + k;
      if (tx == 0 && x < n) Pp[(int64_t)J * ldl + x] = v;
    }
  }
  if (I == J) return;  // block-uniform; the diagonal tile's row sums cover both orders
  // column sums of tile J over tile I: the wave's 4 ty rows by butterfly, then the 4 waves in order
  const int w = pk::wave_id();
#pragma unroll
  for (int l = 0; l < kGK; ++l) {
#pragma unroll
    for (int h = 0; h < kGS; ++h) {
      float v = ca[h][l];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if ((tid & 63) < 16) red[w][kGK * (tx + 16 * h) + l] = v;
    }
  }
  __syncthreads();
  for (int e = tid; e < kRG; e += 256) {
    const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    const int x = J * kRG + e;
    if (x < n) Pp[(int64_t)I * ldl + x] = v;
  }
}

// One block per crop: rigid_compact_kernel's ordered compaction, carrying the survivors' packed
// records into the next round's array.
__global__ __launch_bounds__(1024) void rigid_compact_pts_kernel(const int64_t* __restrict__ list_in, int ldl,
                                                                 const int32_t* __restrict__ nin,
                                                                 const float* __restrict__ score,
                                                                 const float* __restrict__ thr4, int round,
                                                                 const RigidRec* __restrict__ pts_in,
                                                                 int64_t* __restrict__ list_out,
                                                                 RigidRec* __restrict__ pts_out,
                                                                 int32_t* __restrict__ nout) {
  __shared__ int ws[16];
  __shared__ int carry;
  __shared__ float thr_s;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = nin[b];
  const float* S = score + (int64_t)b * ldl;
  if (tid == 0) {
    carry = 0;
    thr_s = thr4[b * 4 + round];
  }
  __syncthreads();
  if (round == 2) {
    int c = 0;
    for (int i = tid; i < n; i += 1024) c += S[i] < thr_s ? 1 : 0;
    c = pk::wave_sum_i32_s(c);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += ws[w];
      if (tot == 0) thr_s = thr4[b * 4 + 3];
    }
    __syncthreads();
  }
  const float thr = thr_s;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const bool keep = i < n && S[i] < thr;
    const uint64_t bal = __ballot(keep);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = __popcll(bal);
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < pk::wave_id(); ++w) pre += ws[w];
    if (keep) {
      const int64_t o = (int64_t)b * ldl + pre + __popcll(bal & ((1ull << pk::lane_id()) - 1ull));
      list_out[o] = list_in[(int64_t)b * ldl + i];
      if (pts_out != nullptr) pts_out[o] = pts_in[(int64_t)b * ldl + i];
    }
    __syncthreads();
    if (tid == 1023) carry = pre + __popcll(bal);
    __syncthreads();
  }
  if (tid == 0) nout[b] = carry;
}

// grid (ceil(nmax / 256), B): score[x] = (sum over tiles in order of part[b][tile][x]) / n,
// tiles of `rt` entries.
__global__ __launch_bounds__(256) void rigid_reduce_kernel(const int32_t* __restrict__ nlist, int ldl,
                                                           const float* __restrict__ part, int T, int rt,
                                                           float* __restrict__ score) {
  const int b = blockIdx.y;
  const int n = nlist[b];
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  const int nt = (n + rt - 1) / rt;
  const float* P = part + (int64_t)b * T * ldl + x;
  float acc = 0.f;
  for (int q = 0; q < nt; ++q) acc += P[(int64_t)q * ldl];
  score[(int64_t)b * ldl + x] = acc / (float)n;
}

// One block per crop: ordered compaction of list entries whose score < tau * diam.
// round 3 (fallback > 0): if nothing passes tau, use the fallback threshold.
// thr f32 [B, 4]: tau * diam_cad for tau = 0.3, 0.15, 0.055, 0.065, evaluated in double and
// rounded once (the reference compares an f32 tensor with the Python float tau * diam).
__global__ __launch_bounds__(1024) void rigid_compact_kernel(const int64_t* __restrict__ list_in, int ldl,
                                                             const int32_t* __restrict__ nin,
                                                             const float* __restrict__ score,
                                                             const float* __restrict__ thr4, int round,
                                                             int64_t* __restrict__ list_out,
                                                             int32_t* __restrict__ nout) {
  __shared__ int ws[16];
  __shared__ int carry;
  __shared__ float thr_s;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = nin[b];
  const float* S = score + (int64_t)b * ldl;
  if (tid == 0) {
    carry = 0;
    thr_s = thr4[b * 4 + round];
  }
  __syncthreads();
  if (round == 2) {
    int c = 0;
    for (int i = tid; i < n; i += 1024) c += S[i] < thr_s ? 1 : 0;
    c = pk::wave_sum_i32_s(c);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += ws[w];
      if (tot == 0) thr_s = thr4[b * 4 + 3];
    }
    __syncthreads();
  }
  const float thr = thr_s;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const bool keep = i < n && S[i] < thr;
    const uint64_t bal = __ballot(keep);
    if (pk::lane_id() == 0) ws[pk::wave_id()] = __popcll(bal);
    __syncthreads();
    int pre = carry;
    for (int w = 0; w < pk::wave_id(); ++w) pre += ws[w];
    if (keep) list_out[(int64_t)b * ldl + pre + __popcll(bal & ((1ull << pk::lane_id()) - 1ull))] =
        list_in[(int64_t)b * ldl + i];
    __syncthreads();
    if (tid == 1023) carry = pre + __popcll(bal);
    __syncthreads();
  }
  if (tid == 0) nout[b] = carry;
}

__global__ void iota_kernel(int64_t* __restrict__ list, int ldl, const int32_t* __restrict__ n) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n[b]) list[(int64_t)b * ldl + i] = i;
}

// grid (B), block 256: IR per crop.
__global__ __launch_bounds__(256) void ir_kernel(const int64_t* __restrict__ pairs, int ldp, int pair_stride,
                                                 int col_cad, int col_pc, const int32_t* __restrict__ npairs,
                                                 const float* __restrict__ cad, int ldcad,
                                                 const float* __restrict__ pcal, int ldpc,
                                                 const float* __restrict__ thr, float* __restrict__ ir,
                                                 int32_t* __restrict__ status) {
  __shared__ int ws[4];
  const int b = blockIdx.x;
  const int n = npairs[b];
  const float t = thr[b];
  int c = 0, bad = 0;
  for (int k = threadIdx.x; k < n; k += 256) {
    const int64_t* pr = pairs + (int64_t)b * ldp * 2;
    int64_t ci, pi;
    if (pair_stride == 0) {  // point map: CAD index per crop point k, crop index k
      ci = pairs[(int64_t)b * ldp + k];
      pi = k;
    } else {
      ci = pr[col_cad * (pair_stride == 1 ? ldp : 1) + k * (pair_stride == 1 ? 1 : 2)];
      pi = pr[col_pc * (pair_stride == 1 ? ldp : 1) + k * (pair_stride == 1 ? 1 : 2)];
    }
    // an index outside its array is not read: the pair counts as an outlier and status[b] = 1
    if (ci < 0 || ci >= ldcad || pi < 0 || pi >= ldpc) {
      bad = 1;
      continue;
    }
    const float* a = cad + ((int64_t)b * ldcad + ci) * 3;
    const float* p = pcal + ((int64_t)b * ldpc + pi) * 3;
    const float dx = a[0] - p[0], dy = a[1] - p[1], dz = a[2] - p[2];
    const float d = __fsqrt_rn((dx * dx + dy * dy) + dz * dz);
    c += d < t ? 1 : 0;
  }
  bad = __syncthreads_or(bad);
  if (status && threadIdx.x == 0) status[b] = bad;
  c = pk::wave_sum_i32_s(c);
  if (pk::lane_id() == 0) ws[pk::wave_id()] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = ws[0] + ws[1] + ws[2] + ws[3];
    ir[b] = n > 0 ? (float)tot / (float)n : 0.f;
  }
}

// ---------------------------------------------------------------- C_gt (normal equations)
// Least squares A X = Bm with A = e2[P[:,1], :30], Bm = e1[P[:,0], :30] (utils.py:67-79)
// via the normal equations G X = H in fp64, G = A^T A, H = A^T Bm:
//   G = sum_j cnt_j e2[j]^T e2[j]   (cnt_j = pairs with crop index j: V2 rows, not P)
//   H = sum_p e2[j_p]^T e1[i_p]     (256-pair slices staged as four 64-pair chunks, one partial per slice)
// fp32 inputs, fp64 products and sums; partials reduced in slice order (deterministic),
// then one wave per crop runs Gauss-Jordan with partial pivoting, rows in registers.
constexpr int kF = 30;
constexpr int kCgtRows = 64;   // pairs (H) or crop rows (G) per staged chunk
constexpr int kCgtChunks = 4;  // chunks per partial slice (round 5: 4 x fewer fp64 partials to write and reduce)
constexpr int kCgtSlice = kCgtRows * kCgtChunks;
constexpr int kFF = kF * kF;

// grid (ceil(ldp/256), B): cnt[b, j] += 1 for every pair of crop b (integer atomics).
__global__ __launch_bounds__(256) void cgt_count_kernel(const int64_t* __restrict__ pairs, int ldp,
                                                        const int64_t* __restrict__ npairs, int V2max,
                                                        int32_t* __restrict__ cnt) {
  const int b = blockIdx.y;
  const int64_t n = npairs[b] < ldp ? npairs[b] : ldp;
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const int64_t j = pairs[((int64_t)b * ldp + p) * 2 + 1];
  atomicAdd(&cnt[(int64_t)b * V2max + j], 1);
}

// grid (SH + SG, B), block 256. Slice s < SH: H partial over pairs [64 s, 64 s + 64);
// s >= SH: G partial over crop rows [64 (s - SH), ...). Rows staged in LDS as fp64
// (u = e2 row, v = e1 row or cnt * e2 row); wave w takes rows w, w+4, ...; lane
// (kb, lb) owns the 4 x 4 block rows 4kb.., cols 4lb..; waves combined in fixed order.
__global__ __launch_bounds__(256) void cgt_partial_kernel(const int64_t* __restrict__ pairs, int ldp,
                                                          const int64_t* __restrict__ npairs,
                                                          const float* __restrict__ e1, int ld1, int V1max,
                                                          const float* __restrict__ e2, int ld2, int V2max,
                                                          const int32_t* __restrict__ cnt, int ldc, int SH,
                                                          double* __restrict__ partH,
                                                          double* __restrict__ partG) {
  __shared__ double UV[2 * kCgtRows * 32];  // U rows, then V rows; reused for the wave combine
  double(*U)[32] = reinterpret_cast<double(*)[32]>(UV);
  double(*V)[32] = reinterpret_cast<double(*)[32]>(UV + kCgtRows * 32);
  double(*red)[kFF] = reinterpret_cast<double(*)[kFF]>(UV);
  static_assert(4 * kFF <= 2 * kCgtRows * 32, "combine buffer fits in the staging buffer");
  const int b = blockIdx.y, tid = threadIdx.x;
  const bool isH = (int)blockIdx.x < SH;
  const int s = isH ? blockIdx.x : blockIdx.x - SH;
  const int64_t n = isH ? (npairs[b] < ldp ? npairs[b] : ldp) : V2max;
  const int64_t rs0 = (int64_t)s * kCgtSlice;
  if (rs0 >= n) return;  // inactive slice: the reduction skips it
  const int w = pk::wave_id(), lane = pk::lane_id();
  const int kb = lane >> 3, lb = lane & 7;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int ch = 0; ch < kCgtChunks; ++ch) {  // (block-uniform bounds)
  const int64_t r0 = rs0 + (int64_t)ch * kCgtRows;
  if (r0 >= n) break;
  const int rn = (int)min((int64_t)kCgtRows, n - r0);
  if (ch > 0) __syncthreads();  // the previous chunk's rows are consumed
  {  // staging: thread (row group rb, column k) takes rows rb + 8 i; every index load, then every
     // row load, issued before the first use, unconditionally at clamped rows / columns (round 4
     // waited for each row's pair -> row chain in turn: 8 serial round trips per thread)
    constexpr int kPer = kCgtRows * 32 / 256;
    const int k = tid & 31, rb = tid >> 5, kc = k < kF ? k : 0;
    int64_t ja[kPer], ia[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int r = rb + 8 * i, rc = r < rn ? r : rn - 1;
      if (isH) {
        const int64_t* P = pairs + ((int64_t)b * ldp + r0 + rc) * 2;
        ia[i] = P[0];
        ja[i] = P[1];
      } else {
        ja[i] = r0 + rc;
        ia[i] = 0;
      }
    }
    float fu[kPer], fv[kPer];
    int cv[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      fu[i] = e2[((int64_t)b * V2max + ja[i]) * ld2 + kc];
      if (isH) fv[i] = e1[((int64_t)b * V1max + ia[i]) * ld1 + kc];
      else cv[i] = cnt[(int64_t)b * ldc + (ja[i] < ldc ? ja[i] : ldc - 1)];
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int r = rb + 8 * i;
      const bool ok = r < rn && k < kF;
      const double u = ok ? (double)fu[i] : 0.0;
      U[r][k] = u;
      V[r][k] = ok ? (isH ? (double)fv[i] : (ja[i] < ldc ? u * (double)cv[i] : 0.0)) : 0.0;
    }
  }
  __syncthreads();
  for (int r = w; r < rn; r += 4) {
    double u[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u[i] = U[r][4 * kb + i];
      v[i] = V[r][4 * lb + i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fma(u[i], v[j], acc[i][j]);
  }
  }  // chunks
  __syncthreads();  // staging buffer becomes the combine buffer
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * kb + i, l = 4 * lb + j;
      if (k < kF && l < kF) red[w][k * kF + l] = acc[i][j];
    }
  __syncthreads();
  double* out = (isH ? partH + ((int64_t)b * SH + s) * kFF
                     : partG + ((int64_t)b * gridDim.x - (int64_t)b * SH + s) * kFF);
  for (int e = tid; e < kFF; e += 256) out[e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
}

// grid (ceil(1800 / 64), B), block 256: GH[b] = [G | H] (30 x 60), partials summed over the
// active slices in 4 quarters + a fixed-order combine.
__global__ __launch_bounds__(256) void cgt_reduce_kernel(const double* __restrict__ partH,
                                                         const double* __restrict__ partG, int SH, int SG,
                                                         const int64_t* __restrict__ npairs, int ldp,
                                                         int V2max, double* __restrict__ GH) {
  __shared__ double q4[4][64];
  const int b = blockIdx.y;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), qtr = threadIdx.x >> 6;
  double v = 0.0;
  const bool valid = e < 2 * kFF;
  if (valid) {
    const bool isG = e < kFF;  // row-major [G | H]: entry (k, c) -> G if c < 30
    const int ee = isG ? e : e - kFF;
    const int64_t n = isG ? V2max : (npairs[b] < ldp ? npairs[b] : ldp);
    const int S = isG ? SG : SH;
    const int active = (int)min((int64_t)S, (n + kCgtSlice - 1) / kCgtSlice);
    const double* p = (isG ? partG + (int64_t)b * SG * kFF : partH + (int64_t)b * SH * kFF) + ee;
    const int s0 = (active * qtr) / 4, s1 = (active * (qtr + 1)) / 4;
    double a0 = 0.0, a1 = 0.0;
    int s = s0;
    for (; s + 2 <= s1; s += 2) {
      a0 += p[(int64_t)s * kFF];
      a1 += p[(int64_t)(s + 1) * kFF];
    }
    if (s < s1) a0 += p[(int64_t)s * kFF];
    v = a0 + a1;
  }
  q4[qtr][threadIdx.x & 63] = v;
  __syncthreads();
  if (qtr == 0 && valid) {
    const int t = threadIdx.x;
    const double r = (q4[0][t] + q4[1][t]) + (q4[2][t] + q4[3][t]);
    const bool isG = e < kFF;
    const int ee = isG ? e : e - kFF;
    const int k = ee / kF, c = ee - k * kF;
    GH[(int64_t)b * 2 * kFF + k * 2 * kF + (isG ? c : kF + c)] = r;
  }
}

// Minimum-norm least squares for a rank-deficient (or empty) pair list. This is a deliberate
// deviation: the reference calls C_from_sparse_P on evecs already on the GPU (train.py:92,101),
// where torch.linalg.lstsq uses the 'gels' driver (QR, no rank handling: garbage or NaN for a
// rank-deficient system), so parity with the reference is unpinned for such crops. We return
// what torch's CPU driver (LAPACK gelsy: complete orthogonal factorization) returns:
// X = V diag(w) V^T H with G = V diag(lambda) V^T (cyclic Jacobi, fp64) and w_i = 1/lambda_i
// for lambda_i > rcond^2 lambda_max (sigma_i > rcond sigma_max of A), else 0; rcond =
// eps_f32 * max(P, 30), torch's default for f32 inputs. One wave; lane k < 30 owns index k.
__device__ void cgt_min_norm(const double* __restrict__ gh, int64_t npairs, float* __restrict__ out) {
  __shared__ double G[kF][kF + 1], V[kF][kF + 1], Hs[kF][kF + 1], Ts[kF][kF + 1];
  const int k = threadIdx.x;
  const bool ok = k < kF;
  if (ok) {
    for (int c = 0; c < kF; ++c) {
      G[k][c] = gh[k * 2 * kF + c];
      Hs[k][c] = gh[k * 2 * kF + kF + c];
      V[k][c] = k == c ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0, dia = 0.0;
    if (ok)
      for (int c = 0; c < kF; ++c) {
        const double g = G[k][c];
        if (c == k) dia += g * g; else off += g * g;
      }
    off = pk::wave_sum_f64(off);
    dia = pk::wave_sum_f64(dia);
    if (!(off > 1e-32 * dia)) break;  // converged (also: all-zero G)
    for (int p = 0; p < kF - 1; ++p)
      for (int q = p + 1; q < kF; ++q) {
        const double apq = G[p][q];
        if (fabs(apq) <= 1e-300) continue;  // uniform: every lane read the same LDS word
        const double theta = (G[q][q] - G[p][p]) / (2.0 * apq);
        const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        __syncthreads();
        if (ok) {  // A J (columns p, q), V J
          const double gp = G[k][p], gq = G[k][q];
          G[k][p] = c * gp - s * gq;
          G[k][q] = s * gp + c * gq;
          const double vp = V[k][p], vq = V[k][q];
          V[k][p] = c * vp - s * vq;
          V[k][q] = s * vp + c * vq;
        }
        __syncthreads();
        if (ok) {  // J^T (A J) (rows p, q)
          const double gp = G[p][k], gq = G[q][k];
          G[p][k] = c * gp - s * gq;
          G[q][k] = s * gp + c * gq;
        }
        __syncthreads();
      }
  }
  double lam = ok ? G[k][k] : 0.0;
  double lmax = lam;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) lmax = fmax(lmax, __shfl_xor(lmax, o));
  const double rcond = 1.1920928955078125e-07 * (double)(npairs > kF ? npairs : kF);
  const double w = (ok && lam > rcond * rcond * lmax && lam > 0.0) ? 1.0 / lam : 0.0;
  if (ok)  // T = diag(w) V^T H: row k
    for (int c = 0; c < kF; ++c) {
      double acc = 0.0;
      for (int j = 0; j < kF; ++j) acc = fma(V[j][k], Hs[j][c], acc);
      Ts[k][c] = w * acc;
    }
  __syncthreads();
  if (ok)  // X = V T: row k
    for (int c = 0; c < kF; ++c) {
      double acc = 0.0;
      for (int j = 0; j < kF; ++j) acc = fma(V[k][j], Ts[j][c], acc);
      out[k * kF + c] = (float)acc;
    }
}

// grid (B), block 64 (one wave): Gauss-Jordan with partial pivoting on [G | H]. Lane l holds
// row r = l & 31 (r < 30), columns 30 h .. 30 h + 29 with h = l >> 5, in registers. A crop
// whose pivots span more than 1e6 (rank-deficient or nearly so: fewer than 30 distinct
// matched crop rows, or no pairs) takes the minimum-norm path above instead.
__global__ __launch_bounds__(64) void cgt_solve_kernel(const double* __restrict__ GH, const int64_t* __restrict__ npairs,
                                                       int ldp, float* __restrict__ Cgt) {
  __shared__ double piv_s[2 * kF];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const bool row_ok = r < kF;
  double a[kF];
#pragma unroll
  for (int c = 0; c < kF; ++c) {  // unconditional at a clamped row (no branch + wait per load)
    const double v = GH[(int64_t)b * 2 * kFF + (row_ok ? r : 0) * 2 * kF + h * kF + c];
    a[c] = row_ok ? v : 0.0;
  }
  bool used = !row_ok;
  int var = -1;
  double pmin = __builtin_inf(), pmax = 0.0;
  // fully unrolled: G[r][k] is a static register (round 4 selected it with 30 fp64 cndmasks per
  // step), and the pivot search is two DPP max reductions of the |G[r][k]| bit pattern instead of
  // five ds_bpermute butterflies of (value, row) pairs
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    // pivot: max |G[r][k]| over unused rows (half-0 lanes), lowest row on ties. |x| >= 0 orders
    // as its bit pattern; candidates carry hi + 1 so no candidate ties an excluded lane's 0 (a
    // NaN, which the elimination's pmin / pmax check sends to the fallback path, orders last)
    const double ak = a[k];
    const double fa = fabs(ak);
    const bool cand = h == 0 && !used;
    const uint64_t bits = (uint64_t)__double_as_longlong(fa == fa ? fa : 0.0);
    const uint32_t khi = cand ? (uint32_t)(bits >> 32) + 1u : 0u;
    const uint32_t mhi = pk::wave_max_u32_s(khi);
    const uint32_t klo = (cand && khi == mhi) ? (uint32_t)bits : 0u;
    const uint32_t mlo = pk::wave_max_u32_s(klo);
    const uint64_t win = __ballot(cand && khi == mhi && klo == mlo);
    const int p = win ? __ffsll((unsigned long long)win) - 1 : 0;  // lane = row (half 0)
    const double pivot = __shfl(ak, p);  // G[p][k] from half 0
    pmin = fmin(pmin, fabs(pivot));
    pmax = fmax(pmax, fabs(pivot));
    const double f0 = (row_ok && r != p) ? ak / pivot : 0.0;
    const double f = __shfl(f0, r);        // half-1 lanes take their row's factor
    if (r == p) {
#pragma unroll
      for (int c = 0; c < kF; ++c) piv_s[h * kF + c] = a[c];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (row_ok && r != p) {
#pragma unroll
      for (int c = 0; c < kF; ++c) a[c] = fma(-f, piv_s[h * kF + c], a[c]);
    }
    if (r == p) {
      // one fp64 division per step (a v_div_scale / fixup sequence each), then products:
      // 30 divisions per step made this 30-step elimination ~70 us on the training path
      const double inv = 1.0 / pivot;
#pragma unroll
      for (int c = 0; c < kF; ++c) a[c] = a[c] * inv;
      used = true;
      var = k;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!(pmin > 1e-6 * pmax)) {  // wave-uniform: rank-deficient, empty or non-finite
    const int64_t n = npairs[b] < ldp ? npairs[b] : ldp;
    cgt_min_norm(GH + (int64_t)b * 2 * kFF, n, Cgt + (int64_t)b * kFF);
    return;
  }
  if (h == 1 && var >= 0) {
#pragma unroll
    for (int c = 0; c < kF; ++c) Cgt[((int64_t)b * kF + var) * kF + c] = (float)a[c];
  }
}

}  // namespace

// scratch: the tile partials [B][T][ldc] f32 (T = ceil(nmax / 128)), then two packed-record
// arrays [B][ldc] (the current and the next round's list), 16-B aligned
static int64_t rigid_part_bytes(int B, int nmax, int ldc) {
  const int64_t b = (int64_t)B * ((nmax + kRT2 - 1) / kRT2) * ldc * (int64_t)sizeof(float);
  return (b + 255) & ~(int64_t)255;
}

#ifdef PK_DEVBUILD
static int g_rigid_variant = 0;  // pkdev_rigidity_variant (A/B timing): 1 round 2's 64-tile gather path,
                                 // 2 round 3's ungrouped first round, 3 no run-pair crop tables
#else
constexpr int g_rigid_variant = 0;
#endif

extern "C" int64_t pk_rigidity_filter_work_size(int B, int nmax, int ldc) {
  if (B <= 0 || nmax <= 0) return 0;
  const int64_t v2 = rigid_part_bytes(B, nmax, ldc) + 2 * (int64_t)B * ldc * (int64_t)sizeof(RigidRec);
  const int64_t v1 = (int64_t)B * ((nmax + kRT - 1) / kRT) * ldc * (int64_t)sizeof(float);
  return v2 > v1 ? v2 : v1;
}

#ifdef PK_DEVBUILD
extern "C" int pkdev_rigidity_variant(int v) {
  const int old = g_rigid_variant;
  if (v >= 0) g_rigid_variant = v;
  return old;
}
#endif  // PK_DEVBUILD

extern "C" int pk_rigidity_filter(const int64_t* cand, int ldc, const int32_t* ncand, const float* cad,
                                  int ldcad, const float* pc, int ldpc, const float* thr4, int B, int nmax,
                                  int64_t* list_a, int64_t* list_b, int32_t* n_a, int32_t* n_b, float* score,
                                  float* partial, void* stream) {
  PK_REQUIRE(B >= 0 && nmax >= 0 && ldc >= nmax);
  if (B == 0) return PK_OK;
  PK_REQUIRE(cand && ncand && cad && pc && thr4 && list_a && list_b && n_a && n_b && score);
  hipStream_t s = pk::as_stream(stream);
  const dim3 g((nmax + 255) / 256, B);
  const int T2 = (nmax + kRT2 - 1) / kRT2;
  const int T1 = (nmax + kRG - 1) / kRG;  // <= T2: the grouped round's partial rows fit
  const bool packed = partial != nullptr && T2 > 0 && g_rigid_variant != 1;
  RigidRec* pa = nullptr;
  RigidRec* pb = nullptr;
  if (packed) {
    pa = reinterpret_cast<RigidRec*>(reinterpret_cast<char*>(partial) + rigid_part_bytes(B, nmax, ldc));
    pb = pa + (int64_t)B * ldc;
    hipLaunchKernelGGL(rigid_gather_kernel, g, dim3(256), 0, s, cand, ldc, ncand, cad, ldcad, pc, ldpc, list_a, pa);
  } else {
    hipLaunchKernelGGL(iota_kernel, g, dim3(256), 0, s, list_a, ldc, ncand);
  }
  PK_CHECK_LAUNCH();
  const int32_t* nin = ncand;
  int64_t* lin = list_a;
  int64_t* lout = list_b;
  int32_t* nout = n_b;
  int32_t* nspare = n_a;
  const int T = (nmax + kRT - 1) / kRT;
  for (int r = 0; r < 3; ++r) {
    if (packed && r == 0 && g_rigid_variant != 2) {  // grouped first round (T1 <= T2 partial rows)
      hipLaunchKernelGGL(rigid_group_kernel, dim3(T1 * (T1 + 1) / 2, B), dim3(256), 0, s, nin, ldc, pa, T1, partial);
      PK_CHECK_LAUNCH();
      hipLaunchKernelGGL(rigid_reduce_kernel, g, dim3(256), 0, s, nin, ldc, partial, T1, kRG, score);
    } else if (packed) {
      hipLaunchKernelGGL(rigid_pair2_kernel, dim3(T2 * (T2 + 1) / 2, B), dim3(256), 0, s, nin, ldc, pa, T2, partial,
                         (int)(g_rigid_variant != 3));
      PK_CHECK_LAUNCH();
      hipLaunchKernelGGL(rigid_reduce_kernel, g, dim3(256), 0, s, nin, ldc, partial, T2, kRT2, score);
    }
    if (packed) {
      PK_CHECK_LAUNCH();
      hipLaunchKernelGGL(rigid_compact_pts_kernel, dim3(B), dim3(1024), 0, s, lin, ldc, nin, score, thr4, r, pa, lout,
                         r < 2 ? pb : nullptr, nout);
      PK_CHECK_LAUNCH();
      RigidRec* tp = pa;
      pa = pb;
      pb = tp;
    } else if (partial && T > 0) {  // round 2: symmetric 64-tiles with gathers, ordered reduction
      hipLaunchKernelGGL(rigid_pair_kernel, dim3(T * (T + 1) / 2, B), dim3(256), 0, s, lin, ldc, nin, cand, ldc, cad,
                         ldcad, pc, ldpc, T, partial);
      PK_CHECK_LAUNCH();
      hipLaunchKernelGGL(rigid_reduce_kernel, g, dim3(256), 0, s, nin, ldc, partial, T, kRT, score);
    } else {
      hipLaunchKernelGGL(rigid_score_kernel, g, dim3(256), 0, s, lin, ldc, nin, cand, ldc, cad, ldcad, pc, ldpc,
                         score);
    }
    PK_CHECK_LAUNCH();
    if (!packed) {
      hipLaunchKernelGGL(rigid_compact_kernel, dim3(B), dim3(1024), 0, s, lin, ldc, nin, score, thr4, r, lout,
                         nout);
      PK_CHECK_LAUNCH();
    }
    nin = nout;
    int64_t* t = lin;
    lin = lout;
    lout = t;
    int32_t* tn = nspare;
    nspare = nout;
    nout = tn;
  }
  // after 3 rounds the survivors are in list_b / n_b (a -> b -> a -> b)
  return PK_OK;
}

extern "C" int pk_inlier_ratio(const int64_t* pairs, int ldp, int layout, const int32_t* npairs, const float* cad,
                               int ldcad, const float* pc_aligned, int ldpc, const float* thr, int B, float* ir,
                               int32_t* status, void* stream) {
  PK_REQUIRE(B >= 0 && layout >= 0 && layout <= 2);
  if (B == 0) return PK_OK;
  PK_REQUIRE(pairs && npairs && cad && pc_aligned && thr && ir);
  // layout 0: pairs [B, ldp, 2] (cad, pc); layout 1: [B, 2, ldp] (row 0 cad, row 1 pc);
  // layout 2: [B, ldp] CAD index of crop point k (a point map; pc index = k)
  hipLaunchKernelGGL(ir_kernel, dim3(B), dim3(256), 0, pk::as_stream(stream), pairs, ldp,
                     layout == 2 ? 0 : layout == 1 ? 1 : 2, 0, 1,
                     npairs, cad, ldcad, pc_aligned, ldpc, thr, ir, status);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// mean of n floats: 256 lane sums over a stride, then one wave adds them in a fixed tree order
__global__ __launch_bounds__(256) void mean_f32_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float part[256];
  float a = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) a += x[i];
  part[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0] / (float)n;
}

extern "C" int pk_mean_f32(const float* x, int64_t n, float* out, void* stream) {
  PK_REQUIRE(n >= 1 && x && out);
  hipLaunchKernelGGL(mean_f32_kernel, dim3(1), dim3(256), 0, pk::as_stream(stream), x, n, out);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int64_t pk_cgt_lstsq_work_size(int ldp, int V2max, int B) {
  const int64_t SH = ldp > 0 ? (ldp + kCgtSlice - 1) / kCgtSlice : 0;
  const int64_t SG = (V2max + kCgtSlice - 1) / kCgtSlice;
  return (int64_t)B * ((SH + SG) * kFF + 2 * kFF) + ((int64_t)B * V2max + 1) / 2;
}

extern "C" int pk_cgt_lstsq(const int64_t* pairs, int ldp, const int64_t* npairs, const float* evecs1, int ld1,
                            int V1max, const float* evecs2, int ld2, int V2max, int B, int K, const int32_t* cnt,
                            int ldc, double* work, float* Cgt, void* stream) {
  PK_REQUIRE(B >= 0 && K == kF && ld1 >= kF && ld2 >= kF && ldp >= 0 && V2max > 0);
  PK_REQUIRE(cnt == nullptr || ldc > 0);
  if (B == 0) return PK_OK;
  PK_REQUIRE(pairs && npairs && evecs1 && evecs2 && work && Cgt);
  hipStream_t s = pk::as_stream(stream);
  const int SH = ldp > 0 ? (ldp + kCgtSlice - 1) / kCgtSlice : 0;
  const int SG = (V2max + kCgtSlice - 1) / kCgtSlice;
  double* partH = work;
  double* partG = partH + (int64_t)B * SH * kFF;
  double* GH = partG + (int64_t)B * SG * kFF;
  if (cnt == nullptr) {  // the per-row pair counts: counted here (a fill + an atomic-count launch)
    int32_t* own = reinterpret_cast<int32_t*>(GH + (int64_t)B * 2 * kFF);
    hipError_t e = pk::zero_async(own, sizeof(int32_t) * (size_t)B * V2max, s);
    if (e != hipSuccess) return (int)e;
    if (ldp > 0) {
      hipLaunchKernelGGL(cgt_count_kernel, dim3((ldp + 255) / 256, B), dim3(256), 0, s, pairs, ldp, npairs, V2max,
                         own);
      PK_CHECK_LAUNCH();
    }
    cnt = own;
    ldc = V2max;
  }
  hipLaunchKernelGGL(cgt_partial_kernel, dim3(SH + SG, B), dim3(256), 0, s, pairs, ldp, npairs, evecs1, ld1,
                     V1max, evecs2, ld2, V2max, cnt, ldc, SH, partH, partG);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(cgt_reduce_kernel, dim3((2 * kFF + 63) / 64, B), dim3(256), 0, s, partH, partG, SH, SG,
                     npairs, ldp, V2max, GH);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(cgt_solve_kernel, dim3(B), dim3(64), 0, s, GH, npairs, ldp, Cgt);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// ---------------------------------------------------------------- NCE pair selection
// utils/loss.py:27-30: per crop, `num` distinct rows of its pair list drawn uniformly
// without replacement (np.random.choice(P, num, replace=False)), all rows when the crop
// has fewer. Drawn on the device with a keyed pseudo-random bijection of [0, m)
// (m = min(count, cap)): position i < min(num, m) takes row perm(i), so rows are
// distinct by construction; perm = cycle-walked composition of invertible maps on
// [0, 2^p) (odd multiply + add mod 2^p, xor-shift right). No sort, no memset, no host
// RNG: capture-safe. The key mixes (seed, *ctr, crop); *ctr advances by one per call.
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t perm_step(uint32_t x, uint32_t mask, int sh, const uint32_t (&k)[3]) {
  x = (x * 0x9E3779B1u + k[0]) & mask;
  x ^= x >> sh;
  x = (x * 0x85EBCA77u + k[1]) & mask;
  x ^= x >> sh;
  x = (x * 0xC2B2AE3Du + k[2]) & mask;
  x ^= x >> sh;
  return x;
}

// grid (ceil(k / 256), B), block 256
__global__ __launch_bounds__(256) void nce_select_kernel(const int64_t* __restrict__ count, int64_t cap, int k,
                                                         uint64_t seed, const int64_t* __restrict__ ctr,
                                                         int64_t* __restrict__ rows, uint8_t* __restrict__ valid) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= k) return;
  const int64_t m64 = count[b] < cap ? count[b] : cap;
  const uint32_t m = (uint32_t)(m64 > 0 ? m64 : 0);
  const int64_t o = (int64_t)b * k + i;
  if ((uint32_t)i >= m) {  // fewer pairs than draws: the tail is padding
    rows[o] = 0;
    valid[o] = 0;
    return;
  }
  int p = 1;
  while ((1u << p) < m) ++p;
  const uint32_t mask = (p >= 32) ? 0xffffffffu : ((1u << p) - 1u);
  const int sh = (p + 1) / 2;
  const uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)ctr[0] * 0x100000001B3ull + (uint64_t)b));
  const uint32_t kk[3] = {(uint32_t)h, (uint32_t)(h >> 32), (uint32_t)splitmix64(h)};
  uint32_t y = (uint32_t)i;
  do {
    y = perm_step(y, mask, sh, kk);
  } while (y >= m);  // cycle walking: terminates on i's own cycle
  rows[o] = (int64_t)y;
  valid[o] = 1;
}

__global__ void ctr_advance_kernel(int64_t* ctr) { ctr[0] += 1; }

}  // namespace

extern "C" int pk_nce_select(const int64_t* count, int B, int64_t cap, int num, uint64_t seed, int64_t* ctr,
                             int64_t* rows, uint8_t* valid, void* stream) {
  PK_REQUIRE(B >= 0 && cap >= 0 && num >= 0 && cap < (1ll << 31));
  const int k = (int)(num < cap ? num : cap);
  if (B == 0 || k == 0) return PK_OK;
  PK_REQUIRE(count && ctr && rows && valid);
  hipStream_t s = pk::as_stream(stream);
  hipLaunchKernelGGL(nce_select_kernel, dim3((k + 255) / 256, B), dim3(256), 0, s, count, cap, k, seed, ctr, rows,
                     valid);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(ctr_advance_kernel, dim3(1), dim3(1), 0, s, ctr);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
