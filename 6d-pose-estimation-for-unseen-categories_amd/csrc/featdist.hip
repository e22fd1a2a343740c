// H10 / H11 (first half) — pairwise spectral feature distance + argmin / top-5.
//
// Reference: fmap2pointmap_solvers/naive.py:6-34 and spacial_filtering.py:5-38:
//     emb  = evecs_x[:, :30] @ C12.T                       [V1, 30]
//     dist = torch.cdist(emb, evecs_y[:, :30])             [V1, V2]
//     naive: p2p[j] = dist.argmin(dim=-2)                  (first minimal i)
//     spatial: idx = dist.sort(dim=-2)[1].T[:, :5]         (5 nearest i per j)
// torch.cdist (V > 25) evaluates the mm expansion with K = 32:
//     [-2 x, |x|^2, 1] · [y, 1, |y|^2]^T, clamp_min(1e-30), sqrt
// The kernel computes exactly that augmented K = 32 contraction on the f32 MFMA
// (v_mfma_f32_16x16x4_f32: f32 products, f32 accumulation), clamps, and keeps per
// column a running argmin (or sorted top-5) in the epilogue; sqrt is monotone and is
// applied to the emitted distances only. Ties resolve to the lowest row index.
//
// Pass 1 (prep) writes both augmented operands straight into MFMA operand order:
// for a 16-row tile T, lane l = 16 g + c (g = k mod 4 group, c = row in tile) owns the
// 8 floats k = 4 s + g, s = 0..7, of row 16 T + c — so pass 2 loads one operand set
// with two 16-byte loads per lane and no LDS, no transposes, no barriers.
//   A  [B, T1, 64 lanes, 8]  T1 = ceil16(V1max) / 16   (x side, rows reduced over)
//   Bq [B, T2, 64 lanes, 8]  T2 = ceil16(V2max) / 16   (y side, one column set per wave)
// Pass 2: a wave owns 32 columns (two B operands in 16 VGPRs) and a quarter of the row
// tiles of A, streamed through registers two tiles per step (four independent
// accumulators, 32 MFMAs per A tile pair) with the next two tiles' loads in flight, so
// the matrix pipe issues back to back while the other waves on the SIMD run their
// epilogues; the four row parts of a column pair merge through LDS.
#include "common.hpp"

namespace {

constexpr int kF = 30;   // n_fmap
constexpr int kK = 32;   // augmented contraction length
using f32x4 = __attribute__((ext_vector_type(4))) float;

// grid (ceil(max(T1, T2) * 16 / 64), B, 2), block 256: thread = (row r = tid / 4, group
// g = tid % 4) computes the 8 augmented entries k = 4 s + g of its row.
//   z = 0 (x side): emb = x C^T; entries -2 emb[k] (k < 30), |emb|^2 (k = 30), 1 (k = 31)
//   z = 1 (y side): y[k] (k < 30), 1 (k = 30), |y|^2 (k = 31)
// |.|^2 is the fmaf chain over k = 0..29 in order (the 4 lanes of a row exchange their
// values). Rows r >= n[b] (and the tile padding up to 16) are written as zeros.
__global__ __launch_bounds__(256) void fd_prep_kernel(const float* __restrict__ ex, int ldx,
                                                      const float* __restrict__ C,
                                                      const float* __restrict__ ey, int ldy,
                                                      const int32_t* __restrict__ n1,
                                                      const int32_t* __restrict__ n2, int V1max, int V2max,
                                                      int T1, int T2, float* __restrict__ A,
                                                      float* __restrict__ Bq) {
  const int b = blockIdx.y;
  const int g = threadIdx.x & 3;
  const int r = blockIdx.x * 64 + (threadIdx.x >> 2);
  const bool xside = blockIdx.z == 0;
  const int T = xside ? T1 : T2;
  // C transposed per thread group: sCt[k][g][s] = C[4 s + g][k] (0 for rows 30, 31), so a
  // thread's 8 coefficients of one k are two 16-byte LDS reads
  __shared__ __attribute__((aligned(16))) float sCt[kF * 4 * 8];
  if (xside) {
    for (int e = threadIdx.x; e < kF * 32; e += 256) {
      const int k = e >> 5, gg = (e >> 3) & 3, ss = e & 7;
      const int c = 4 * ss + gg;
      sCt[e] = c < kF ? C[((int64_t)b * kF + c) * kF + k] : 0.f;
    }
    __syncthreads();
  }
  if (r >= T * 16) return;  // whole rows (4 adjacent lanes) leave together
  const int nvalid = xside ? n1[b] : n2[b];
  const bool valid = r < nvalid;
  float e[8];  // emb (x side) or y (y side) at k = 4 s + g
  if (xside) {
    const float* er = ex + ((int64_t)b * V1max + (valid ? r : 0)) * ldx;
#pragma unroll
    for (int s = 0; s < 8; ++s) e[s] = 0.f;
#pragma unroll 6
    for (int k = 0; k < kF; ++k) {  // emb[c] = sum_k x[k] C[c][k], fmaf chain in k order
      const float xk = valid ? er[k] : 0.f;
      const float4* cp = reinterpret_cast<const float4*>(&sCt[(k * 4 + g) * 8]);
      const float4 c0 = cp[0], c1 = cp[1];
      e[0] = fmaf(xk, c0.x, e[0]);
      e[1] = fmaf(xk, c0.y, e[1]);
      e[2] = fmaf(xk, c0.z, e[2]);
      e[3] = fmaf(xk, c0.w, e[3]);
      e[4] = fmaf(xk, c1.x, e[4]);
      e[5] = fmaf(xk, c1.y, e[5]);
      e[6] = fmaf(xk, c1.z, e[6]);
      e[7] = fmaf(xk, c1.w, e[7]);
    }
  } else {
    const float* er = ey + ((int64_t)b * V2max + (valid ? r : 0)) * ldy;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int c = 4 * s + g;
      e[s] = (valid && c < kF) ? er[c] : 0.f;
    }
  }
  float nrm = 0.f;
  const int base = threadIdx.x & ~3;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const float q = __shfl(e[s], base | gg);
      if (4 * s + gg < kF) nrm = fmaf(q, q, nrm);
    }
  }
  float v[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = xside ? -2.f * e[s] : e[s];
  if (!valid) {
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = 0.f;
  } else if (g >= 2) {  // k = 30, 31
    v[7] = (xside == (g == 2)) ? nrm : 1.f;
  }
  const int tile = r >> 4, c16 = r & 15;
  float* dst = (xside ? A + (int64_t)b * T1 * 512 : Bq + (int64_t)b * T2 * 512) +
               ((int64_t)tile * 64 + g * 16 + c16) * 8;
  reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

template <int TOPK>
struct TopK {
  float v[TOPK];
  int i[TOPK];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      v[k] = __builtin_huge_valf();
      i[k] = 0x7fffffff;
    }
  }
  // rows arrive in increasing index order: strict < keeps the lowest index on ties
  __device__ __forceinline__ void push(float x, int idx) {
    if (TOPK == 1) {
      const bool lt = x < v[0];
      v[0] = lt ? x : v[0];
      i[0] = lt ? idx : i[0];
      return;
    }
    if (!(x < v[TOPK - 1])) return;
    float cv = x;
    int ci = idx;
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      const bool sw = cv < v[k];
      const float tv = sw ? v[k] : cv;
      const int ti = sw ? i[k] : ci;
      v[k] = sw ? cv : v[k];
      i[k] = sw ? ci : i[k];
      cv = tv;
      ci = ti;
    }
  }
  // merge an incoming sorted list (ties: lower index first)
  __device__ __forceinline__ void merge(const float (&ov)[TOPK], const int (&oi)[TOPK]) {
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      float cv = ov[k];
      int ci = oi[k];
#pragma unroll
      for (int m = 0; m < TOPK; ++m) {
        const bool sw = cv < v[m] || (cv == v[m] && ci < i[m]);
        const float tv = sw ? v[m] : cv;
        const int ti = sw ? i[m] : ci;
        v[m] = sw ? cv : v[m];
        i[m] = sw ? ci : i[m];
        cv = tv;
        ci = ti;
      }
    }
  }
};

__device__ __forceinline__ void load_tile(const float* __restrict__ At, int t, int lane, float (&a)[8]) {
  const float4* p = reinterpret_cast<const float4*>(At + ((int64_t)t * 64 + lane) * 8);
  const float4 u = p[0], w = p[1];
  a[0] = u.x; a[1] = u.y; a[2] = u.z; a[3] = u.w;
  a[4] = w.x; a[5] = w.y; a[6] = w.z; a[7] = w.w;
}

template <int TOPK>
__device__ __forceinline__ void epilogue(const f32x4& acc, int ibase, int N1, bool partial, TopK<TOPK>& best) {
  if (TOPK == 1) {
    // the 4 rows of this lane in one go: min of the clamped values (2 min + 1 max), and
    // only when it beats the running best (rare once warmed up) find its first row
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (partial && ibase + r >= N1) ? __builtin_huge_valf() : acc[r];
    const float mc = fmaxf(fminf(fminf(v[0], v[1]), fminf(v[2], v[3])), 1e-30f);  // clamp_min(1e-30)
    if (mc < best.v[0]) {
      int r = 3;
      if (fmaxf(v[2], 1e-30f) == mc) r = 2;
      if (fmaxf(v[1], 1e-30f) == mc) r = 1;
      if (fmaxf(v[0], 1e-30f) == mc) r = 0;
      best.v[0] = mc;
      best.i[0] = ibase + r;
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ibase + r;
    float v = fmaxf(acc[r], 1e-30f);  // clamp_min(1e-30) (cdist mm path)
    if (partial && i >= N1) v = __builtin_huge_valf();
    best.push(v, i);
  }
}

template <int TOPK>
__device__ __forceinline__ void lanegroup_merge(TopK<TOPK>& best) {
#pragma unroll
  for (int off = 16; off <= 32; off <<= 1) {
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      ov[k] = __shfl_xor(best.v[k], off);
      oi[k] = __shfl_xor(best.i[k], off);
    }
    best.merge(ov, oi);
  }
}

// grid (B * ceil(T2 / CW)), block 64 RP: the block owns CW column tiles (their B operands
// stay in registers, so every A tile load feeds 8 CW MFMAs) and wave q takes the q-th of
// RP parts of the row tiles; the parts merge through LDS (ties: lower row first). One
// step = two row tiles x CW column tiles on 2 CW independent accumulators, the next
// step's A tiles in flight (two register sets, written out twice so nothing is copied).
template <int TOPK, int CW, int RP, bool NOEPI = false, bool NOLOAD = false>
__global__ __launch_bounds__(64 * RP) void fd_main_kernel(const float* __restrict__ A, const float* __restrict__ Bq,
                                                          const int32_t* __restrict__ n1,
                                                          const int32_t* __restrict__ n2, int T1, int T2, int V2max,
                                                          int64_t* __restrict__ out_idx,
                                                          float* __restrict__ out_dist) {
  __shared__ float xv[RP][CW][16][TOPK];
  __shared__ int xi[RP][CW][16][TOPK];
  // 1-D grid of B x NC blocks (NC = column groups per crop), renumbered so that all blocks
  // of crop b run on XCD b % 8 (hardware block L lands on XCD L % 8): a crop's A operand
  // (128 KiB at V1 = 1024) is then read from one XCD's L2 instead of all eight.
  const int NC = (T2 + CW - 1) / CW;
  const int B = (int)(gridDim.x / NC);
  int b, cg;
  {
    const int L = blockIdx.x, x8 = L & 7, k = L >> 3;
    if ((B & 7) == 0) {
      b = x8 + 8 * (k / NC);
      cg = k - (k / NC) * NC;
    } else {
      b = L / NC;
      cg = L - b * NC;
    }
  }
  const int lane = pk::lane_id(), q = pk::wave_id();
  const int g = lane >> 4, c16 = lane & 15;
  const int ct0 = cg * CW;
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;  // row tiles holding valid rows
  const int t_begin = (nt * q) / RP, t_end = (nt * (q + 1)) / RP;
  TopK<TOPK> best[CW];
  float bop[CW][8];
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    best[c].init();
    if (ct0 + c < T2) load_tile(Bq + (int64_t)b * T2 * 512, ct0 + c, lane, bop[c]);
    else {
#pragma unroll
      for (int s = 0; s < 8; ++s) bop[c][s] = 0.f;
    }
  }
  const float* At = A + (int64_t)b * T1 * 512;
  float p0[8], p1[8], q0[8], q1[8];
  const bool ragged = (N1 & 15) != 0;  // only then does the last tile need row masking
  auto step = [&](int t, const float (&a0)[8], const float (&a1)[8]) {
    f32x4 c0[CW], c1[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) c0[c] = c1[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int c = 0; c < CW; ++c) {
        c0[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], bop[c][s], c0[c], 0, 0, 0);
        c1[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], bop[c][s], c1[c], 0, 0, 0);
      }
    }
    // lane holds D[16 t + 4 g + r][col] (c0) and D[16 (t+1) + 4 g + r][col] (c1)
    const bool two = t + 1 < t_end;
    if (NOEPI) {  // development variant: MFMA + operand streaming only
#pragma unroll
      for (int c = 0; c < CW; ++c) best[c].v[0] += c0[c][0] + c1[c][3];
      return;
    }
    if (ragged && t + 2 >= nt) {  // wave-uniform: the crop's last, partial tile
#pragma unroll
      for (int c = 0; c < CW; ++c) {
        epilogue<TOPK>(c0[c], t * 16 + 4 * g, N1, true, best[c]);
        if (two) epilogue<TOPK>(c1[c], (t + 1) * 16 + 4 * g, N1, true, best[c]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < CW; ++c) {
        epilogue<TOPK>(c0[c], t * 16 + 4 * g, N1, false, best[c]);
        if (two) epilogue<TOPK>(c1[c], (t + 1) * 16 + 4 * g, N1, false, best[c]);
      }
    }
  };
  if (t_begin < t_end) load_tile(At, t_begin, lane, p0);
  if (t_begin + 1 < t_end) load_tile(At, t_begin + 1, lane, p1);
  if (NOLOAD) {  // development variant: operands loaded once, reused every step
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      q0[s] = p0[s];
      q1[s] = p1[s];
    }
  }
  for (int t = t_begin; t < t_end; t += 4) {
    if (!NOLOAD && t + 2 < t_end) load_tile(At, t + 2, lane, q0);
    if (!NOLOAD && t + 3 < t_end) load_tile(At, t + 3, lane, q1);
    step(t, p0, p1);
    if (t + 2 >= t_end) break;
    if (!NOLOAD && t + 4 < t_end) load_tile(At, t + 4, lane, p0);
    if (!NOLOAD && t + 5 < t_end) load_tile(At, t + 5, lane, p1);
    step(t + 2, q0, q1);
  }
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    lanegroup_merge<TOPK>(best[c]);
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < TOPK; ++k) {
        xv[q][c][c16][k] = best[c].v[k];
        xi[q][c][c16][k] = best[c].i[k];
      }
    }
  }
  __syncthreads();
  // lanes 16 cw + c16 of wave 0 (cw < CW) finish column tile ct0 + cw
  const int cw = lane >> 4;
  if (q != 0 || cw >= CW || ct0 + cw >= T2) return;
  TopK<TOPK> fin;
#pragma unroll
  for (int k = 0; k < TOPK; ++k) {
    fin.v[k] = xv[0][cw][c16][k];
    fin.i[k] = xi[0][cw][c16][k];
  }
#pragma unroll
  for (int qq = 1; qq < RP; ++qq) {
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      ov[k] = xv[qq][cw][c16][k];
      oi[k] = xi[qq][cw][c16][k];
    }
    fin.merge(ov, oi);
  }
  const int j = (ct0 + cw) * 16 + c16;
  if (j < N2) {
    const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
    for (int k = 0; k < TOPK; ++k) {
      out_idx[o + k] = fin.i[k] == 0x7fffffff ? -1 : fin.i[k];
      if (out_dist) out_dist[o + k] = sqrtf(fin.v[k]);
    }
  }
}

constexpr int kFdCW = 2;  // column tiles per wave (4 measured slower: 136 VGPRs)
constexpr int kFdRP = 4;  // row parts (waves) per block

}  // namespace

extern "C" int pk_feat_dist_topk(const float* evecs_x, int ldx, const float* C, const float* evecs_y, int ldy,
                                 const int32_t* n1, const int32_t* n2, int B, int V1max, int V2max, int topk,
                                 float* A, float* Bq, int64_t* out_idx, float* out_dist, void* stream) {
  PK_REQUIRE(B >= 0 && V1max >= 0 && V2max >= 0 && ldx >= kF && ldy >= kF && (topk == 1 || topk == 5));
  if (B == 0 || V2max == 0) return PK_OK;
  PK_REQUIRE(evecs_x && C && evecs_y && n1 && n2 && A && Bq && out_idx);
  hipStream_t s = pk::as_stream(stream);
  const int T1 = (V1max + 15) / 16, T2 = (V2max + 15) / 16;
  const int rows = (T1 > T2 ? T1 : T2) * 16;
  hipLaunchKernelGGL(fd_prep_kernel, dim3((rows + 63) / 64, B, 2), dim3(256), 0, s, evecs_x, ldx, C, evecs_y, ldy,
                     n1, n2, V1max, V2max, T1, T2, A, Bq);
  PK_CHECK_LAUNCH();
  const dim3 grid(((T2 + kFdCW - 1) / kFdCW) * B), block(64 * kFdRP);
  if (topk == 1)
    hipLaunchKernelGGL((fd_main_kernel<1, kFdCW, kFdRP>), grid, block, 0, s, A, Bq, n1, n2, T1, T2, V2max, out_idx,
                       out_dist);
  else
    hipLaunchKernelGGL((fd_main_kernel<5, kFdCW, kFdRP>), grid, block, 0, s, A, Bq, n1, n2, T1, T2, V2max, out_idx,
                       out_dist);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

// Development hook (not in include/posekern.h): the main pass without its top-k epilogue,
// on operands already prepared by pk_feat_dist_topk (A, Bq), to time the MFMA pipeline.
extern "C" int pkdev_fd_main_noepi(const float* A, const float* Bq, const int32_t* n1, const int32_t* n2, int B,
                                   int V1max, int V2max, int64_t* out_idx, int noload, void* stream) {
  const int T1 = (V1max + 15) / 16, T2 = (V2max + 15) / 16;
  const dim3 grid(((T2 + kFdCW - 1) / kFdCW) * B), block(64 * kFdRP);
  if (noload)
    hipLaunchKernelGGL((fd_main_kernel<1, kFdCW, kFdRP, true, true>), grid, block, 0, pk::as_stream(stream), A, Bq, n1,
                       n2, T1, T2, V2max, out_idx, nullptr);
  else
    hipLaunchKernelGGL((fd_main_kernel<1, kFdCW, kFdRP, true>), grid, block, 0, pk::as_stream(stream), A, Bq, n1, n2,
                       T1, T2, V2max, out_idx, nullptr);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
