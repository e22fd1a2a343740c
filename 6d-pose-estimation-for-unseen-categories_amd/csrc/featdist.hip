// H10 / H11 (first half) — pairwise spectral feature distance + argmin / top-5.
//
// Reference: fmap2pointmap_solvers/naive.py:6-34 and spacial_filtering.py:5-38:
//     emb  = evecs_x[:, :30] @ C12.T                       [V1, 30]
//     dist = torch.cdist(emb, evecs_y[:, :30])             [V1, V2]
//     naive: p2p[j] = dist.argmin(dim=-2)                  (first minimal i)
//     spatial: idx = dist.sort(dim=-2)[1].T[:, :5]         (5 nearest i per j)
// torch.cdist (V > 25) evaluates the mm expansion with K = 32:
//     [-2 x, |x|^2, 1] · [y, 1, |y|^2]^T, clamp_min(1e-30), sqrt
//
// Precision modes (the contraction only; the selection epilogue is shared):
//   0 (default, the parity path): exactly that augmented K = 32 contraction on the f32 MFMA
//     (v_mfma_f32_16x16x4_f32: f32 products, f32 accumulation).
//   1 bf16: the cross term -2 x·y on v_mfma_f32_16x16x32_bf16 (K = 30 padded to 32, one
//     instruction per 16 x 16 tile), |x|^2 + |y|^2 added in f32 in the epilogue.
//   2 bf16x3: the cross term as hi·hi + hi·lo + lo·hi of a two-term bf16 split of both
//     operands (three bf16 MFMAs, ~16 significant bits), norms in f32 as in mode 1.
// Modes 1 / 2 are opt-in (configs[4]'s "4096 x 4096 bf16"); tests report their argmin
// agreement with mode 0.
//
// Pass 1 (prep): one thread per row computes the row's operand (x side: emb = x C^T, an fmaf
// chain over k in order; y side: y) and its squared norm, and writes the operand straight
// into MFMA operand-tile order (16-row tiles, lane l = 16 g + c holding row c's k values of
// its group g), so pass 2 moves whole tiles with 16-byte loads and no transposes.
// Pass 2 (main, fd_main_direct_kernel): a block = 4 waves over 4 column tiles and the block's
// row tiles; each wave takes 2 column tiles (B operands in registers) and half the rows, and
// streams its rows' fragments from L2 into registers one chunk ahead of the MFMAs (every A
// fragment feeds two accumulation chains). Epilogue per 16 x 16 tile: running argmin / sorted
// top-5 per column (ties: lowest row); the two row halves merge through LDS at the end. With
// RS > 1 the blocks' row parts write partial lists that pass 3 merges (same tie rule), so one
// 4096-point crop (configs[4]) still spreads over the chip. fd_main_kernel (development knob
// PK_FD_DIRECT=0) is the earlier pass: one column tile per wave, rows staged through an LDS
// ring shared by the block's 4 waves (measured slower: DESIGN.md §5).
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

namespace {

constexpr int kF = 30;   // n_fmap
constexpr int kK = 32;   // contraction length (K padded)
constexpr int kCW = 1;   // column tiles per wave
constexpr int kWaves = 4;
constexpr int kCols = kWaves * kCW * 16;  // columns per block
constexpr int kCH = 8;   // row tiles per LDS stage
using f32x4 = __attribute__((ext_vector_type(4))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

// bytes of one 16-row operand tile per mode (f32: 64 lanes x 8 floats; bf16: 64 x 8 bf16;
// bf16x3: hi then lo)
__host__ __device__ constexpr int tile_bytes(int mode) { return mode == 0 ? 2048 : mode == 1 ? 1024 : 2048; }

__device__ __forceinline__ __bf16 to_bf16(float v) { return (__bf16)v; }

// grid (ceil(max(T1, T2) / 8), B, 2), block 512: wave = one 16-row tile of one side (z = 0:
// x side, 1: y side). Lane (g, c) = (lane >> 4, lane & 15).
//   x side: emb = x C^T on the f32 MFMA ([16 x 32] x [32 x 32], two 16 x 16 output tiles,
//           K = 30 zero-padded; an f32 MFMA accumulates as the fmaf chain over k in order),
//           then through LDS into the operand layout;
//   y side: y itself.
// The squared norm of a row is its lane group's 8 values summed per lane, then across the 4
// lanes of the row (fixed order). Rows >= n (and the tile padding) are written as zeros.
constexpr int kPrepWaves = 8;  // one 16-row tile per wave, 8 waves per block

template <int MODE>
__global__ __launch_bounds__(64 * kPrepWaves) void fd_prep_kernel(const float* __restrict__ ex, int ldx,
                                                      const float* __restrict__ C, const float* __restrict__ ey,
                                                      int ldy, const int32_t* __restrict__ n1,
                                                      const int32_t* __restrict__ n2, int V1max, int V2max, int T1,
                                                      int T2, char* __restrict__ A, char* __restrict__ Bq,
                                                      float* __restrict__ nA, float* __restrict__ nB) {
  __shared__ float E[kPrepWaves][16][kK + 1];  // per wave: the tile's rows (emb or y), k padded to 32
  const int b = blockIdx.y;
  const bool xside = blockIdx.z == 0;
  const int w = pk::wave_id(), lane = pk::lane_id(), g = lane >> 4, c16 = lane & 15;
  const int T = xside ? T1 : T2;
  const int tile = blockIdx.x * kPrepWaves + w;
  if (tile >= T) return;
  const int r = tile * 16 + c16;
  // every operand load is issued before the first wait: the row at a clamped index (its
  // validity against n applied by select afterwards), the C entries (both sides: C is tiny),
  // and n itself — a load addressed through n, or behind the x-side branch, would add a round
  // trip each
  const float* rowp = xside ? ex + ((int64_t)b * V1max + min(r, V1max - 1)) * ldx
                            : ey + ((int64_t)b * V2max + min(r, V2max - 1)) * ldy;
  // this lane's 8 row values at k = 4 s + g (the f32 MFMA operand layout), 0 past k = 29
  float xv[8];
  float cvs[2][8];
#pragma unroll
  for (int s = 0; s < 8; ++s) xv[s] = rowp[min(4 * s + g, kF - 1)];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      cvs[n][s] = C[((int64_t)b * kF + min(16 * n + c16, kF - 1)) * kF + min(4 * s + g, kF - 1)];
  const int nval = xside ? n1[b] : n2[b];
  const bool valid = r < nval;
  // the empty asm pins the loads above this point (else the compiler sinks them under the
  // select / the x-side branch, behind a wait of their own)
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" : "+v"(cvs[n][s]));
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    asm volatile("" : "+v"(xv[s]));
    xv[s] = (valid && 4 * s + g < kF) ? xv[s] : 0.f;
  }
  float (*Ew)[kK + 1] = E[w];
  if (xside) {
    // D[row 4 g' + q][col c] of output tile n: emb[row][16 n + c] = sum_k x[row][k] C[16 n + c][k]
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int cc = 16 * n + c16;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[s], (cc < kF && 4 * s + g < kF) ? cvs[n][s] : 0.f, acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) Ew[4 * g + q][cc] = acc[q];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) Ew[c16][4 * s + g] = xv[s];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // the lane's operand values (mode 0: k = 4 s + g; bf16 modes: k = 8 g + j) and the row norm
  float v[8];
  float part = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = MODE == 0 ? 4 * s + g : 8 * g + s;
    v[s] = (valid && k < kF) ? Ew[c16][k] : 0.f;
    part = fmaf(v[s], v[s], part);
  }
  const float p1 = __shfl_xor(part, 16), p2 = __shfl_xor(part, 32), p3 = __shfl_xor(part, 48);
  const float mine[4] = {part, p1, p2, p3};  // lane group g, g^1, g^2, g^3
  float nrm = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];  // groups 0, 1, 2, 3 in that order
  // padding rows: y side zeros; x side a row whose distance to every column is +inf (mode 0:
  // the |x|^2 slot; bf16 modes: the norm), so the main pass needs no row mask
  if (!valid) nrm = xside ? __builtin_huge_valf() : 0.f;
  char* base = (xside ? A + (int64_t)b * T1 * tile_bytes(MODE) : Bq + (int64_t)b * T2 * tile_bytes(MODE)) +
               (int64_t)tile * tile_bytes(MODE);
  if (MODE == 0) {
    // augmented operand: x side [-2 emb, |emb|^2, 1], y side [y, 1, |y|^2]
    float o[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) o[s] = xside ? -2.f * v[s] : v[s];
    if (g >= 2 && valid) o[7] = (xside == (g == 2)) ? nrm : 1.f;  // k = 30 (g = 2), 31 (g = 3)
    if (g == 2 && xside && !valid) o[7] = nrm;                      // +inf |x|^2 slot
    float4* d = reinterpret_cast<float4*>(base + (size_t)lane * 32);
    d[0] = make_float4(o[0], o[1], o[2], o[3]);
    d[1] = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    // bf16 cross-term operand: x side -2 emb, y side y (k < 30, zero pad); k = 8 g + j
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = xside ? -2.f * v[j] : v[j];
      const __bf16 h = to_bf16(f);
      hi[j] = h;
      lo[j] = to_bf16(f - (float)h);
    }
    *reinterpret_cast<bf16x8*>(base + (size_t)lane * 16) = hi;
    if (MODE == 2) *reinterpret_cast<bf16x8*>(base + 1024 + (size_t)lane * 16) = lo;
    if (g == 0) (xside ? nA + (int64_t)b * T1 * 16 : nB + (int64_t)b * T2 * 16)[r] = nrm;
  }
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

// 4 distances of this lane (rows ibase .. ibase + 3 of its column) into the running top-k
template <int TOPK>
__device__ __forceinline__ void epilogue(const float (&d)[4], int ibase, TopK<TOPK>& best) {
#pragma unroll
  for (int r = 0; r < 4; ++r) best.push(fmaxf(d[r], 1e-30f), ibase + r);  // clamp_min(1e-30) (cdist mm path)
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

// One 16 x 16 tile (rows of A tile `a`, this wave's column tile) -> 4 values per lane
// (rows 4 g + r, column c16).
template <int MODE>
struct Frag;
template <> struct Frag<0> { float a[8]; };
template <> struct Frag<1> { bf16x8 hi; float n[4]; };
template <> struct Frag<2> { bf16x8 hi, lo; float n[4]; };

template <int MODE>
__device__ __forceinline__ void read_frag(const char* __restrict__ tile, const float* __restrict__ ntile, int lane,
                                          Frag<MODE>& f) {
  if constexpr (MODE == 0) {
    const float4* p = reinterpret_cast<const float4*>(tile + lane * 32);
    const float4 u = p[0], w = p[1];
    f.a[0] = u.x; f.a[1] = u.y; f.a[2] = u.z; f.a[3] = u.w;
    f.a[4] = w.x; f.a[5] = w.y; f.a[6] = w.z; f.a[7] = w.w;
  } else {
    f.hi = *reinterpret_cast<const bf16x8*>(tile + lane * 16);
    if constexpr (MODE == 2) f.lo = *reinterpret_cast<const bf16x8*>(tile + 1024 + lane * 16);
    const float4 n = *reinterpret_cast<const float4*>(ntile + 4 * (lane >> 4));
    f.n[0] = n.x; f.n[1] = n.y; f.n[2] = n.z; f.n[3] = n.w;
  }
}

template <int MODE>
struct BOp;
template <> struct BOp<0> { float b[8]; };
template <> struct BOp<1> { bf16x8 hi; float n; };
template <> struct BOp<2> { bf16x8 hi, lo; float n; };

template <int MODE>
__device__ __forceinline__ void tile_dist(const Frag<MODE>& a, const BOp<MODE>& b, float (&d)[4]) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 0) {
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.a[s], b.b[s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = acc[r];
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
    if constexpr (MODE == 2) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = (acc[r] + a.n[r]) + b.n;  // |x|^2 - 2 x.y + |y|^2
  }
}

// Top-1 running state of a lane: per row offset r (rows 16 t + 4 g + r of its column) the
// smallest clamped distance so far, as its f32 bit pattern (clamped values are positive, so
// their bit patterns order as the values do), and the tile t holding it. Per distance: integer
// max (the clamp), difference, sign mask, bit-select, integer min — no compare-to-VCC, so the
// four chains interleave with each other and the MFMAs without hazard stalls. Ties stay with
// the earliest tile because tiles arrive in increasing order and only a strictly smaller key
// moves the tile.
struct Top1x4 {
  int k[4];
  int t[4];
};

// kCH row tiles of one LDS chunk against this wave's column tile
// (all kCH fragments are read from LDS before the first MFMA: one LDS latency per chunk instead
// of one per tile, and kCH independent accumulation chains for the MFMA pipe)
template <int MODE>
__device__ __forceinline__ void chunk_dist(const char* rb, const float* nb, const BOp<MODE>& bo, int lane,
                                           float (&d)[kCH][4]) {
  Frag<MODE> f[kCH];
#pragma unroll
  for (int t = 0; t < kCH; ++t) read_frag<MODE>(rb + tile_bytes(MODE) * t, nb + t * 16, lane, f[t]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < kCH; ++t) tile_dist<MODE>(f[t], bo, d[t]);
}

// the selection over one chunk's distances (tiles c0 .. c0 + kCH - 1)
template <int TOPK>
__device__ __forceinline__ void chunk_select(const float (&d)[kCH][4], int c0, int g, TopK<TOPK>& best, Top1x4& b4) {
  if constexpr (TOPK == 1) {
    constexpr int kClamp = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)
#pragma unroll
    for (int t = 0; t < kCH; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = max(__float_as_int(d[t][r]), kClamp);
        const int m = (key - b4.k[r]) >> 31;  // -1 iff key < best (both in [kClamp, 0x7fffffff])
        b4.t[r] = (m & (c0 + t)) | (~m & b4.t[r]);
        b4.k[r] = min(key, b4.k[r]);
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < kCH; ++t) epilogue<TOPK>(d[t], (c0 + t) * 16 + 4 * g, best);
  }
}

// grid (B * NCG * RS) (1-D, XCD-aware), block 256. Block = (crop b, column group cg: wave w
// takes column tile 4 cg + w, row split rs: row tiles [tb, te) of the crop's valid ones).
template <int TOPK, int MODE>
__global__ __launch_bounds__(64 * kWaves) void fd_main_kernel(
    const char* __restrict__ A, const char* __restrict__ Bq, const float* __restrict__ nA,
    const float* __restrict__ nB, const int32_t* __restrict__ n1, const int32_t* __restrict__ n2, int T1, int T2,
    int V2max, int NCG, int RS, int64_t* __restrict__ out_idx, float* __restrict__ out_dist,
    float* __restrict__ part_v, int32_t* __restrict__ part_i) {
  constexpr int TB = tile_bytes(MODE);
  __shared__ __attribute__((aligned(16))) char ring[2][kCH][TB];
  __shared__ __attribute__((aligned(16))) float nring[2][kCH][16];
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 (hardware block L lands on XCD L % 8) when B % 8 == 0
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / per);
      k = q - (q / per) * per;
    } else {
      b = L / per;
      k = L - b * per;
    }
  }
  const int cg = k % NCG, rs = k / NCG;
  const int lane = pk::lane_id(), w = pk::wave_id();
  const int g = lane >> 4, c16 = lane & 15;
  const int ct = cg * kWaves + w;  // this wave's column tile
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;
  const int tb = (nt * rs) / RS, te = (nt * (rs + 1)) / RS;
  const bool col_ok = ct < T2 && ct * 16 < N2;
  BOp<MODE> bo;
  if (col_ok) {
    const char* bt = Bq + ((int64_t)b * T2 + ct) * TB;
    if constexpr (MODE == 0) {
      const float4* p = reinterpret_cast<const float4*>(bt + lane * 32);
      const float4 u = p[0], v = p[1];
      bo.b[0] = u.x; bo.b[1] = u.y; bo.b[2] = u.z; bo.b[3] = u.w;
      bo.b[4] = v.x; bo.b[5] = v.y; bo.b[6] = v.z; bo.b[7] = v.w;
    } else {
      bo.hi = *reinterpret_cast<const bf16x8*>(bt + lane * 16);
      if constexpr (MODE == 2) bo.lo = *reinterpret_cast<const bf16x8*>(bt + 1024 + lane * 16);
      bo.n = nB[((int64_t)b * T2 + ct) * 16 + c16];
    }
  } else {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 8; ++s) bo.b[s] = 0.f;
    } else {
      bo.hi = bf16x8{};
      if constexpr (MODE == 2) bo.lo = bf16x8{};
      bo.n = 0.f;
    }
  }
  TopK<TOPK> best;
  best.init();
  Top1x4 b4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    b4.k[r] = 0x7f800000;  // +inf: never replaced by an equal key
    b4.t[r] = 0x7fffffff;
  }
  const char* At = A + (int64_t)b * T1 * TB;
  const float* nAt = MODE != 0 ? nA + (int64_t)b * T1 * 16 : nullptr;
  // staging: a chunk of kCH tiles = kCH * TB bytes, 16 B per thread per step
  constexpr int VPT = kCH * TB / 16 / (64 * kWaves);  // float4s per thread per chunk
  float4 stage[VPT];
  float nst = 0.f;  // one norm per thread (threads < kCH * 16)
  // (unconditional loads at a clamped element: a guarded load would put an
  // exec-mask branch and a wait for it inside the MFMA loop)
  // exec-mask branch and a wait for it inside the MFMA loop); the padding select happens at the
  // LDS store, after the chunk's MFMAs, so nothing reads the loaded registers early
  int lim = 0;
  auto gload = [&](int c0, int cn) {
    const float4* src = reinterpret_cast<const float4*>(At + (int64_t)c0 * TB);
    lim = cn * TB / 16;
#pragma unroll
    for (int v = 0; v < VPT; ++v) stage[v] = src[min((int)threadIdx.x + 64 * kWaves * v, lim - 1)];
    if (MODE != 0 && threadIdx.x < kCH * 16) nst = nAt[(int64_t)c0 * 16 + min((int)threadIdx.x, cn * 16 - 1)];
  };
  auto lstore = [&](int buf) {
    float4* dst = reinterpret_cast<float4*>(&ring[buf][0][0]);
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const int e = threadIdx.x + 64 * kWaves * v;
      // past the row part: padding rows (+inf |x|^2 slot in mode 0: lane group 2, k = 30)
      const int q = e % (TB / 16);
      const bool inf_slot = MODE == 0 && (q & 1) && (q >> 5) == 2;
      const bool in = e < lim;
      const float4 x = stage[v];
      dst[e] = make_float4(in ? x.x : 0.f, in ? x.y : 0.f, in ? x.z : 0.f,
                           in ? x.w : (inf_slot ? __builtin_huge_valf() : 0.f));
    }
    if (MODE != 0 && threadIdx.x < kCH * 16)
      (&nring[buf][0][0])[threadIdx.x] = (int)threadIdx.x < lim / (TB / 16) * 16 ? nst : __builtin_huge_valf();
  };
  const int nch = (te - tb + kCH - 1) / kCH;
  if (nch > 0) {
    gload(tb, min(kCH, te - tb));
    lstore(0);
  }
  __syncthreads();
  // vmcnt(0) on every path into the loop (the column operand's loads included): otherwise the
  // wait counter pass keeps them pending at the loop header and waits for the next chunk's
  // loads inside the MFMA loop
  __builtin_amdgcn_s_waitcnt(0x0F70);
  // software pipeline: the selection over chunk ci - 1 (registers) runs beside the MFMAs of
  // chunk ci; dp starts as +inf (never selected)
  float dp[kCH][4];
#pragma unroll
  for (int t = 0; t < kCH; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dp[t][r] = __builtin_huge_valf();
  int cp = 0;
  for (int ci = 0; ci < nch; ++ci) {
    const int c0 = tb + ci * kCH;
    if (ci + 1 < nch) gload(c0 + kCH, min(kCH, te - c0 - kCH));
    if (col_ok) {
      float d[kCH][4];
      chunk_dist<MODE>(&ring[ci & 1][0][0], &nring[ci & 1][0][0], bo, lane, d);
      chunk_select<TOPK>(dp, cp, g, best, b4);
#pragma unroll
      for (int t = 0; t < kCH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) dp[t][r] = d[t][r];
      cp = c0;
    }
    if (ci + 1 < nch) lstore((ci + 1) & 1);
    __syncthreads();
  }
  if (!col_ok) return;
  chunk_select<TOPK>(dp, cp, g, best, b4);
  if constexpr (TOPK == 1) {  // the 4 row offsets: smallest value, ties lowest row
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = b4.t[r] == 0x7fffffff ? 0x7fffffff : b4.t[r] * 16 + 4 * g + r;
      const float v = __int_as_float(b4.k[r]);
      const bool take = v < best.v[0] || (v == best.v[0] && row < best.i[0]);
      best.v[0] = take ? v : best.v[0];
      best.i[0] = take ? row : best.i[0];
    }
  }
  lanegroup_merge<TOPK>(best);
  const int j = ct * 16 + c16;
  if (g != 0 || j >= N2) return;
  if (RS == 1) {
    const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      out_idx[o + q] = best.i[q] == 0x7fffffff ? -1 : best.i[q];
      if (out_dist) out_dist[o + q] = sqrtf(best.v[q]);
    }
  } else {
    const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * TOPK;
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      part_v[o + q] = best.v[q];
      part_i[o + q] = best.i[q];
    }
  }
}

// The main pass without LDS staging (the default; PK_FD_DIRECT=0 selects the LDS-ring pass
// above). Block = 4 waves = 2 column pairs x 2 row halves: wave (wc, wr) takes column tiles
// 4 cg + 2 wc and 4 cg + 2 wc + 1 and half wr of the block's row tiles, reading the rows' MFMA
// fragments straight from L2 into registers one chunk of CHD tiles ahead of the MFMAs (two
// register buffers: the next chunk's loads are in flight during this chunk's 16 * CHD MFMAs).
// Every A fragment feeds both column tiles (two independent accumulation chains per row tile,
// half the L2 traffic per MFMA of a one-column wave); no barrier until the end, where the
// second row half hands its lists through LDS to the first, which merges them (ties: lower
// row) and writes the block's columns.
template <int TOPK, int MODE>
__global__ __launch_bounds__(64 * kWaves) void fd_main_direct_kernel(
    const char* __restrict__ A, const char* __restrict__ Bq, const float* __restrict__ nA,
    const float* __restrict__ nB, const int32_t* __restrict__ n1, const int32_t* __restrict__ n2, int T1, int T2,
    int V2max, int NCG, int RS, int64_t* __restrict__ out_idx, float* __restrict__ out_dist,
    float* __restrict__ part_v, int32_t* __restrict__ part_i) {
  constexpr int TB = tile_bytes(MODE);
  constexpr int CHD = MODE == 2 ? 2 : 4;
  __shared__ float hv[2][2][16][TOPK];  // second row half's lists: [wc][column tile][column][k]
  __shared__ int hi_[2][2][16][TOPK];
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 (hardware block L lands on XCD L % 8) when B % 8 == 0
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / per);
      k = q - (q / per) * per;
    } else {
      b = L / per;
      k = L - b * per;
    }
  }
  const int cg = k % NCG, rs = k / NCG;
  const int lane = pk::lane_id(), w = pk::wave_id();
  const int g = lane >> 4, c16 = lane & 15;
  // (readfirstlane: the wave-uniform values in scalar registers, so the chunk loop is a scalar
  // loop and not an exec-masked one whose wait counts the compiler cannot track)
  const int wc = __builtin_amdgcn_readfirstlane(w & 1), wr = __builtin_amdgcn_readfirstlane(w >> 1);
  const int ct0 = cg * kWaves + 2 * wc;  // this wave's column tiles ct0, ct0 + 1
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;
  const int tb0 = (nt * rs) / RS, te0 = (nt * (rs + 1)) / RS;      // the block's row part
  const int tb = tb0 + ((te0 - tb0) * wr) / 2, te = tb0 + ((te0 - tb0) * (wr + 1)) / 2;  // this wave's half
  BOp<MODE> bo[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {  // (a column tile past T2 reads tile T2 - 1; its lists are not written)
    const char* bt = Bq + ((int64_t)b * T2 + min(ct0 + c, T2 - 1)) * TB;
    if constexpr (MODE == 0) {
      const float4* p = reinterpret_cast<const float4*>(bt + lane * 32);
      const float4 u = p[0], v = p[1];
      bo[c].b[0] = u.x; bo[c].b[1] = u.y; bo[c].b[2] = u.z; bo[c].b[3] = u.w;
      bo[c].b[4] = v.x; bo[c].b[5] = v.y; bo[c].b[6] = v.z; bo[c].b[7] = v.w;
    } else {
      bo[c].hi = *reinterpret_cast<const bf16x8*>(bt + lane * 16);
      if constexpr (MODE == 2) bo[c].lo = *reinterpret_cast<const bf16x8*>(bt + 1024 + lane * 16);
      bo[c].n = nB[((int64_t)b * T2 + min(ct0 + c, T2 - 1)) * 16 + c16];
    }
  }
  const char* At = A + (int64_t)b * T1 * TB;
  const float* nAt = MODE != 0 ? nA + (int64_t)b * T1 * 16 : nullptr;
  TopK<TOPK> best[2];
  Top1x4 b4[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    best[c].init();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b4[c].k[r] = 0x7f800000;  // +inf: never replaced by an equal key
      b4[c].t[r] = 0x7fffffff;
    }
  }
  // tiles past te are loaded at te - 1 (unconditional loads: no branch, no early wait) and
  // their distances masked to +inf before the selection
  auto load = [&](Frag<MODE> (&f)[CHD], int c0) {
#pragma unroll
    for (int t = 0; t < CHD; ++t) {
      const int tt = min(c0 + t, te - 1);
      read_frag<MODE>(At + (int64_t)tt * TB, nAt ? nAt + (int64_t)tt * 16 : nullptr, lane, f[t]);
    }
  };
  auto compute = [&](const Frag<MODE> (&f)[CHD], int c0) {
#pragma unroll
    for (int t = 0; t < CHD; ++t) {
      float d[2][4];
      tile_dist<MODE>(f[t], bo[0], d[0]);
      tile_dist<MODE>(f[t], bo[1], d[1]);
      const bool in = c0 + t < te;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if constexpr (TOPK == 1) {
          constexpr int kClamp = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = in ? max(__float_as_int(d[c][r]), kClamp) : 0x7f800000;
            const int m = (key - b4[c].k[r]) >> 31;  // -1 iff key < best
            b4[c].t[r] = (m & (c0 + t)) | (~m & b4[c].t[r]);
            b4[c].k[r] = min(key, b4[c].k[r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) d[c][r] = in ? d[c][r] : __builtin_huge_valf();
          epilogue<TOPK>(d[c], (c0 + t) * 16 + 4 * g, best[c]);
        }
      }
    }
  };
  const int nch = __builtin_amdgcn_readfirstlane(te > tb ? (te - tb + CHD - 1) / CHD : 0);
  if (nch > 0) {
    // (sched_barrier: the scheduler would otherwise sink each load next to its first use)
    Frag<MODE> fa[CHD], fb[CHD];
    load(fa, tb);
    // (no early exit: every iteration issues both loads, so a chunk's loads are always in
    // flight across the previous chunk's MFMAs, the back edge included)
    for (int ci = 0; ci < nch; ci += 2) {
      const int c0 = tb + ci * CHD;
      load(fb, c0 + CHD);
      __builtin_amdgcn_sched_barrier(0);
      compute(fa, c0);
      load(fa, c0 + 2 * CHD);
      __builtin_amdgcn_sched_barrier(0);
      if (ci + 1 < nch) compute(fb, c0 + CHD);
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if constexpr (TOPK == 1) {  // the 4 row offsets: smallest value, ties lowest row
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b4[c].t[r] == 0x7fffffff ? 0x7fffffff : b4[c].t[r] * 16 + 4 * g + r;
        const float v = __int_as_float(b4[c].k[r]);
        const bool take = v < best[c].v[0] || (v == best[c].v[0] && row < best[c].i[0]);
        best[c].v[0] = take ? v : best[c].v[0];
        best[c].i[0] = take ? row : best[c].i[0];
      }
    }
    lanegroup_merge<TOPK>(best[c]);
  }
  // the second row half's lists to the first (ties: lower row — the merge's index rule)
  if (wr == 1 && g == 0) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < TOPK; ++q) {
        hv[wc][c][c16][q] = best[c].v[q];
        hi_[wc][c][c16][q] = best[c].i[q];
      }
  }
  __syncthreads();
  if (wr == 1 || g != 0) return;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      ov[q] = hv[wc][c][c16][q];
      oi[q] = hi_[wc][c][c16][q];
    }
    best[c].merge(ov, oi);
    const int ct = ct0 + c;
    const int j = ct * 16 + c16;
    if (ct >= T2 || j >= N2) continue;
    if (RS == 1) {
      const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
      for (int q = 0; q < TOPK; ++q) {
        out_idx[o + q] = best[c].i[q] == 0x7fffffff ? -1 : best[c].i[q];
        if (out_dist) out_dist[o + q] = sqrtf(best[c].v[q]);
      }
    } else {
      const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * TOPK;
#pragma unroll
      for (int q = 0; q < TOPK; ++q) {
        part_v[o + q] = best[c].v[q];
        part_i[o + q] = best[c].i[q];
      }
    }
  }
}

// The fused fp32 pass (mode 0, the default since round 4): prep and main in ONE launch, no
// operand round trip through HBM. Block = NW waves = (crop b, column group cg, row part rs);
// wave w owns column tiles CT * (NW cg + w) + c, c < CT (their B operands, the y side, stay in
// registers for the whole launch) and every wave streams the block's row part.
//
// Contraction-slot order. The MFMA sums over its 32 k-slots in a fixed order; which feature
// sits in which slot is free as long as the A (row) and B (column) operands agree. Here slot
// (step s = 4 n + q, lane group g) holds feature k = 16 n + 4 g + q, so:
//   * a lane's 8 y values are two contiguous float4 of its row (two 16-B loads per column tile);
//   * the row embedding emb = x C^T computed on the MFMA as D' = C x^T (M = emb feature, N = x
//     row) comes out of the accumulators already in A-operand order: lane (g, c) of output tile
//     n holds emb[row c][16 n + 4 g + q], q = 0..3 (no transposition, no LDS round trip for it);
//   * the emb contraction over x's features uses the same order (two float4 x loads per row).
// Slots k = 30, 31 (lane group 3, steps 6 and 7; features >= 30 are zero) carry the augmented
// terms of torch.cdist's mm path: A [-2 emb, |emb|^2, 1] . B [y, 1, |y|^2] (padding rows: an
// +inf |x|^2 slot, never selected). The squared norms are fmaf chains over a lane's 8 slots,
// then the 4 lane groups summed in the order 0, 1, 2, 3.
//
// Row loop: chunks of NW row tiles; wave w computes the emb tile of chunk row tile w (16 f32
// MFMAs, C read from LDS in operand order) and stores it into a double-buffered LDS chunk in
// operand order; one barrier per chunk; then every wave runs its CT column tiles against the
// chunk's NW row tiles (CT independent accumulation chains per A fragment), the selection of
// each tile software-pipelined behind the next tile's MFMAs. The x rows of the next chunk are
// loaded at the top of the chunk (registers) and consumed after its MFMAs. With RS > 1 every
// block writes its columns' partial lists and fd_merge_kernel combines them in row-part order.
template <int TOPK, int CT, int NW, int VAR = 0>
__global__ __launch_bounds__(64 * NW, 2) void fd_fused_kernel(
    const float* __restrict__ ex, int ldx, const float* __restrict__ C, const float* __restrict__ ey, int ldy,
    const int32_t* __restrict__ n1, const int32_t* __restrict__ n2, int V1max, int V2max, int NCG, int RS,
    int64_t* __restrict__ out_idx, float* __restrict__ out_dist, float* __restrict__ part_v,
    int32_t* __restrict__ part_i, int32_t* __restrict__ arrivals) {
  __shared__ __attribute__((aligned(16))) f32x4 chunk[2][NW][2][64];  // A tiles in operand order
  __shared__ int last_arrival;
  __shared__ __attribute__((aligned(16))) f32x4 cop[2][2][64];        // C in emb-MFMA A order [n][h][lane]
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 (hardware block L lands on XCD L % 8) when B % 8 == 0
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / per);
      k = q - (q / per) * per;
    } else {
      b = L / per;
      k = L - b * per;
    }
  }
  const int cg = k % NCG, rs = k / NCG;
  const int lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  const int g = lane >> 4, c16 = lane & 15;
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;
  const int tb = (nt * rs) / RS, te = (nt * (rs + 1)) / RS;  // the block's row tiles
  const float* Cb = C + (int64_t)b * kF * kF;
  // C in the emb MFMA's A order: lane (g, m) of output tile n, step s = 4 h + q holds
  // C[16 n + m][16 h + 4 g + q] (zero past row / feature 29); 4 KB, staged once per block
  if (threadIdx.x < 256) {
    const int n = threadIdx.x >> 7, h = (threadIdx.x >> 6) & 1, l = threadIdx.x & 63;
    const int m = l & 15, gg = l >> 4, row = 16 * n + m;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 16 * h + 4 * gg + q;
      v[q] = (row < kF && f < kF) ? Cb[row * kF + f] : 0.f;
    }
    cop[n][h][l] = f32x4{v[0], v[1], v[2], v[3]};
  }
  // column operands (y side): lane (g, c) of column tile ct holds y[16 ct + c][16 n + 4 g + q]
  // at step 4 n + q; slot k = 30 -> 1, k = 31 -> |y|^2
  float bo[CT][8];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int ct = CT * (NW * cg + w) + c;
    const int j = ct * 16 + c16;
    const float* yr = ey + ((int64_t)b * V2max + min(j, V2max - 1)) * ldy;
    const float4 y0 = *reinterpret_cast<const float4*>(yr + 4 * g);
    const float4 y1 = *reinterpret_cast<const float4*>(yr + 16 + 4 * g);
    const bool ok = j < N2;
    float v[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bool in = ok && (s < 6 || g < 3);  // feature 16 (s >> 2) + 4 g + (s & 3) < 30
      v[s] = in ? v[s] : 0.f;
      part = fmaf(v[s], v[s], part);
    }
    const float p1 = __shfl_xor(part, 16), p2 = __shfl_xor(part, 32), p3 = __shfl_xor(part, 48);
    const float mine[4] = {part, p1, p2, p3};
    float nrm = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];
    if (g == 3) {
      v[6] = 1.f;
      v[7] = nrm;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) bo[c][s] = v[s];
  }
  // x rows of row tile `tt` (features 16 h + 4 g .. + 3 of row 16 tt + c16), unmasked loads at
  // a clamped row; the feature / row masks apply at use
  const float* xb = ex + (int64_t)b * V1max * ldx;
  auto xload = [&](int tt, float4 (&xv)[2]) {
    const int row = min(tt * 16 + c16, V1max - 1);
    const float* xr = xb + (int64_t)row * ldx;
    xv[0] = *reinterpret_cast<const float4*>(xr + 4 * g);
    xv[1] = *reinterpret_cast<const float4*>(xr + 16 + 4 * g);
  };
  // emb tile of row tile tt -> A operand [-2 emb, |emb|^2, 1] into LDS chunk slot (buf, w)
  auto emb_tile = [&](int tt, const float4 (&xv)[2], int buf) {
    const int row = tt * 16 + c16;
    const bool rok = row < N1;
    float xs[8] = {xv[0].x, xv[0].y, xv[0].z, xv[0].w, xv[1].x, xv[1].y, xv[1].z, xv[1].w};
#pragma unroll
    for (int s = 0; s < 8; ++s) xs[s] = (rok && (s < 6 || g < 3)) ? xs[s] : 0.f;
    float e[8];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x4 c0 = cop[n][0][lane], c1 = cop[n][1][lane];
      const float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(cv[s], xs[s], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) e[4 * n + q] = acc[q];  // emb[row c16][16 n + 4 g + q]
    }
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) part = fmaf(e[s], e[s], part);
    const float p1 = __shfl_xor(part, 16), p2 = __shfl_xor(part, 32), p3 = __shfl_xor(part, 48);
    const float mine[4] = {part, p1, p2, p3};
    float nrm = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];
    float o[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) o[s] = -2.f * e[s];
    if (g == 3) {
      o[6] = rok ? nrm : __builtin_huge_valf();  // padding row: +inf |x|^2 slot
      o[7] = 1.f;
    }
    chunk[buf][w][0][lane] = f32x4{o[0], o[1], o[2], o[3]};
    chunk[buf][w][1][lane] = f32x4{o[4], o[5], o[6], o[7]};
  };
  TopK<TOPK> best[CT];
  Top1x4 b4[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    best[c].init();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b4[c].k[r] = 0x7f800000;  // +inf: never replaced by an equal key
      b4[c].t[r] = 0x7fffffff;
    }
  }
  // selection of one tile's distances (tile index tt, masked to +inf past the part)
  auto select = [&](const float (&d)[CT][4], int tt, bool in) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      if constexpr (TOPK == 1) {
        constexpr int kClamp = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = in ? max(__float_as_int(d[c][r]), kClamp) : 0x7f800000;
          const int m = (key - b4[c].k[r]) >> 31;  // -1 iff key < best
          b4[c].t[r] = (m & tt) | (~m & b4[c].t[r]);
          b4[c].k[r] = min(key, b4[c].k[r]);
        }
      } else {
        float dd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) dd[r] = in ? d[c][r] : __builtin_huge_valf();
        epilogue<TOPK>(dd, tt * 16 + 4 * g, best[c]);
      }
    }
  };
  const int nchunk = te > tb ? (te - tb + NW - 1) / NW : 0;
  float4 xv[2];
  if (nchunk > 0) {
    xload(min(tb + w, te - 1), xv);
    __syncthreads();  // cop staged
    emb_tile(tb + w, xv, 0);
  }
  __syncthreads();
  float dprev[CT][4];
  int tprev = -1;
  for (int ch = 0; ch < nchunk; ++ch) {
    const int c0 = tb + ch * NW;
    const int buf = ch & 1;
    const bool more = ch + 1 < nchunk;
    if (more) xload(min(c0 + NW + w, te - 1), xv);
    const int ntile = min(NW, te - c0);
    for (int t = 0; t < ntile; ++t) {
      const f32x4 a0 = chunk[buf][t][0][lane], a1 = chunk[buf][t][1][lane];
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      float d[CT][4];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (VAR == 2 || VAR == 3) {  // (development variants: no main-loop MFMAs)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = av[r] + av[4 + r] * bo[c][r];
        } else {
#pragma unroll
          for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bo[c][s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) d[c][r] = acc[r];
      }
      if constexpr (VAR == 1 || VAR == 3) {  // (development variants: no selection, one VALU op)
        if (tprev >= 0) b4[0].k[0] ^= __float_as_int(dprev[0][0] + dprev[CT - 1][3]);
      } else {
        if (tprev >= 0) select(dprev, tprev, true);  // the previous tile, beside these MFMAs
      }
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) dprev[c][r] = d[c][r];
      tprev = c0 + t;
    }
    if (more) emb_tile(c0 + NW + w, xv, buf ^ 1);
    __syncthreads();
  }
  if (tprev >= 0) select(dprev, tprev, true);
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if constexpr (TOPK == 1) {  // the 4 row offsets: smallest value, ties lowest row
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b4[c].t[r] == 0x7fffffff ? 0x7fffffff : b4[c].t[r] * 16 + 4 * g + r;
        const float v = __int_as_float(b4[c].k[r]);
        const bool take = v < best[c].v[0] || (v == best[c].v[0] && row < best[c].i[0]);
        best[c].v[0] = take ? v : best[c].v[0];
        best[c].i[0] = take ? row : best[c].i[0];
      }
    }
    lanegroup_merge<TOPK>(best[c]);
  }
  if (g == 0) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int j = (CT * (NW * cg + w) + c) * 16 + c16;
      if (j >= N2) continue;
      if (RS == 1) {
        const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
        for (int q = 0; q < TOPK; ++q) {
          out_idx[o + q] = best[c].i[q] == 0x7fffffff ? -1 : best[c].i[q];
          if (out_dist) out_dist[o + q] = sqrtf(best[c].v[q]);
        }
      } else {
        const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * TOPK;
#pragma unroll
        for (int q = 0; q < TOPK; ++q) {
          part_v[o + q] = best[c].v[q];
          part_i[o + q] = best[c].i[q];
        }
      }
    }
  }
  if (RS == 1) return;
  // in-launch combine of the RS row parts (cdna_hip_programming.md §6 Guideline 16, counter
  // form): every wave drains its partial stores, one agent-scope release, one relaxed ticket per
  // block on arrivals[b][cg]; the block that draws RS - 1 acquires, merges the RS lists of each of
  // its columns in row-part order (ties: lower row) and resets the ticket to 0 (the word is zero
  // before the first launch on this buffer and after every launch)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(arrivals + (int64_t)b * NCG + cg, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    last_arrival = old == RS - 1;
    if (old == RS - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(arrivals + (int64_t)b * NCG + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last_arrival) return;
  for (int jj = threadIdx.x; jj < NW * CT * 16; jj += 64 * NW) {
    const int j = CT * NW * 16 * cg + jj;
    if (j >= N2) continue;
    TopK<TOPK> m;
    m.init();
    for (int r = 0; r < RS; ++r) {
      const int64_t o = (((int64_t)b * RS + r) * V2max + j) * TOPK;
      float ov[TOPK];
      int oi[TOPK];
#pragma unroll
      for (int q = 0; q < TOPK; ++q) {
        ov[q] = part_v[o + q];
        oi[q] = part_i[o + q];
      }
      m.merge(ov, oi);
    }
    const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      out_idx[o + q] = m.i[q] == 0x7fffffff ? -1 : m.i[q];
      if (out_dist) out_dist[o + q] = sqrtf(m.v[q]);
    }
  }
}

// The fp32 parity path since round 4: fd_rows_kernel + fd_cols_kernel.
//
// Contraction-slot order. The MFMA sums over its 32 k-slots in a fixed order; which feature
// sits in which slot is free as long as the A (row) and B (column) operands agree. Here slot
// (step s = 4 n + q, lane group g) holds feature k = 16 n + 4 g + q, so:
//   * a lane's 8 y values are two contiguous float4 of its row (two 16-B loads per column tile);
//   * the row embedding emb = x C^T computed on the MFMA as D' = C x^T (M = emb feature, N = x
//     row) comes out of the accumulators already in A-operand order: lane (g, c) of output tile
//     n holds emb[row c][16 n + 4 g + q], q = 0..3 (no transposition through LDS);
//   * the emb contraction over x's features uses the same order (two float4 x loads per row).
// Slots k = 30, 31 (lane group 3, steps 6 and 7; features >= 30 are zero) carry the augmented
// terms of torch.cdist's mm path: A [-2 emb, |emb|^2, 1] . B [y, 1, |y|^2] (padding rows: an
// +inf |x|^2 slot, never selected). The squared norms are fmaf chains over a lane's 8 slots,
// then the 4 lane groups summed in the order 0, 1, 2, 3.
//
// fd_rows_kernel: grid (ceil(T1 / 4), B), 4 waves, one 16-row tile per wave: x rows (two 16-B
// loads per lane), C from L2 in the emb MFMA's A order, 16 f32 MFMAs, norms, and the tile's A
// operand stored as two lane-contiguous 1 KB halves (slots 0-3, 4-7).
__global__ __launch_bounds__(256) void fd_rows_kernel(const float* __restrict__ ex, int ldx,
                                                     const float* __restrict__ C, const int32_t* __restrict__ n1,
                                                     int V1max, int T1, f32x4* __restrict__ A) {
  const int b = blockIdx.y;
  const int lane = pk::lane_id(), g = lane >> 4, c16 = lane & 15;
  const int tt = blockIdx.x * 4 + pk::wave_id();
  if (tt >= T1) return;
  const int row = tt * 16 + c16;
  const float* xr = ex + ((int64_t)b * V1max + min(row, V1max - 1)) * ldx;
  const float4 x0 = *reinterpret_cast<const float4*>(xr + 4 * g);
  const float4 x1 = *reinterpret_cast<const float4*>(xr + 16 + 4 * g);
  // C operand: lane (g, m) of output tile n at step s = 4 h + q holds C[16 n + m][16 h + 4 g + q]
  const float* Cb = C + (int64_t)b * kF * kF;
  float cv[2][8];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int r = 16 * n + c16, f = 16 * (s >> 2) + 4 * g + (s & 3);
      cv[n][s] = Cb[min(r, kF - 1) * kF + min(f, kF - 1)];
    }
  const bool rok = row < n1[b];
  float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int s = 0; s < 8; ++s) xs[s] = (rok && (s < 6 || g < 3)) ? xs[s] : 0.f;  // feature < 30
  float e[8];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int r = 16 * n + c16;
      const bool cok = r < kF && (s < 6 || g < 3);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(cok ? cv[n][s] : 0.f, xs[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) e[4 * n + q] = acc[q];  // emb[row c16][16 n + 4 g + q]
  }
  float part = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) part = fmaf(e[s], e[s], part);
  const float p1 = __shfl_xor(part, 16), p2 = __shfl_xor(part, 32), p3 = __shfl_xor(part, 48);
  const float mine[4] = {part, p1, p2, p3};
  float nrm = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];  // lane groups 0, 1, 2, 3 in that order
  float o[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) o[s] = -2.f * e[s];
  if (g == 3) {
    o[6] = rok ? nrm : __builtin_huge_valf();  // padding row: +inf |x|^2 slot
    o[7] = 1.f;
  }
  f32x4* At = A + ((int64_t)b * T1 + tt) * 128;
  At[lane] = f32x4{o[0], o[1], o[2], o[3]};
  At[64 + lane] = f32x4{o[4], o[5], o[6], o[7]};
}

// fd_cols_kernel: grid B * NCG * RS (1-D, XCD-aware), NW waves. Block = (crop b, column group
// cg of CT column tiles, row part rs); every wave holds the group's CT column operands (the y
// side, two 16-B loads per lane and tile, norms in-wave) in registers and takes 1/NW of the row
// part's tiles, streaming their A operands from L2 two tiles ahead (two 16-B loads per lane and
// tile); per tile CT independent accumulation chains of 8 MFMAs, the selection of each tile
// software-pipelined behind the next tile's MFMAs. The NW waves' lists merge through LDS in wave
// (= row) order; with RS > 1 the block writes partial lists that fd_merge_kernel combines.
template <int TOPK, int CT, int NW>
__global__ __launch_bounds__(64 * NW, 2) void fd_cols_kernel(
    const f32x4* __restrict__ A, const float* __restrict__ ey, int ldy, const int32_t* __restrict__ n1,
    const int32_t* __restrict__ n2, int V2max, int T1, int NCG, int RS, int64_t* __restrict__ out_idx,
    float* __restrict__ out_dist, float* __restrict__ part_v, int32_t* __restrict__ part_i) {
  __shared__ float mv[NW][CT][16][TOPK];
  __shared__ int mi[NW][CT][16][TOPK];
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 (hardware block L lands on XCD L % 8) when B % 8 == 0
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / per);
      k = q - (q / per) * per;
    } else {
      b = L / per;
      k = L - b * per;
    }
  }
  const int cg = k % NCG, rs = k / NCG;
  const int lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  const int g = lane >> 4, c16 = lane & 15;
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;
  const int tb0 = (nt * rs) / RS, te0 = (nt * (rs + 1)) / RS;  // the block's row part
  const int nb = te0 - tb0;
  const int tb = __builtin_amdgcn_readfirstlane(tb0 + (nb * w) / NW);
  const int te = __builtin_amdgcn_readfirstlane(tb0 + (nb * (w + 1)) / NW);  // this wave's tiles
  // column operands: lane (g, c) of column tile ct holds y[16 ct + c][16 n + 4 g + q] at step
  // 4 n + q; slot k = 30 -> 1, k = 31 -> |y|^2
  float bo[CT][8];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int j = (cg * CT + c) * 16 + c16;
    const float* yr = ey + ((int64_t)b * V2max + min(j, V2max - 1)) * ldy;
    const float4 y0 = *reinterpret_cast<const float4*>(yr + 4 * g);
    const float4 y1 = *reinterpret_cast<const float4*>(yr + 16 + 4 * g);
    const bool ok = j < N2;
    float v[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      v[s] = (ok && (s < 6 || g < 3)) ? v[s] : 0.f;
      part = fmaf(v[s], v[s], part);
    }
    const float p1 = __shfl_xor(part, 16), p2 = __shfl_xor(part, 32), p3 = __shfl_xor(part, 48);
    const float mine[4] = {part, p1, p2, p3};
    float nrm = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];
    if (g == 3) {
      v[6] = 1.f;
      v[7] = nrm;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) bo[c][s] = v[s];
  }
  TopK<TOPK> best[CT];
  Top1x4 b4[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    best[c].init();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b4[c].k[r] = 0x7f800000;  // +inf: never replaced by an equal key
      b4[c].t[r] = 0x7fffffff;
    }
  }
  auto select = [&](const float (&d)[CT][4], int tt) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      if constexpr (TOPK == 1) {
        constexpr int kClamp = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = max(__float_as_int(d[c][r]), kClamp);
          const int m = (key - b4[c].k[r]) >> 31;  // -1 iff key < best
          b4[c].t[r] = (m & tt) | (~m & b4[c].t[r]);
          b4[c].k[r] = min(key, b4[c].k[r]);
        }
      } else {
        epilogue<TOPK>(d[c], tt * 16 + 4 * g, best[c]);
      }
    }
  };
  const f32x4* Ab = A + (int64_t)b * T1 * 128;
  if (te > tb) {
    // A fragments two tiles ahead (unconditional loads at a clamped tile: no branch in the loop)
    f32x4 a0[3], a1[3];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const f32x4* at = Ab + (int64_t)min(tb + p, te - 1) * 128;
      a0[p] = at[lane];
      a1[p] = at[64 + lane];
    }
    float dprev[CT][4];
    for (int t = tb; t < te; ++t) {
      {
        const f32x4* at = Ab + (int64_t)min(t + 2, te - 1) * 128;
        a0[2] = at[lane];
        a1[2] = at[64 + lane];
      }
      const float av[8] = {a0[0][0], a0[0][1], a0[0][2], a0[0][3], a1[0][0], a1[0][1], a1[0][2], a1[0][3]};
      float d[CT][4];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bo[c][s], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) d[c][r] = acc[r];
      }
      if (t > tb) select(dprev, t - 1);  // the previous tile, beside these MFMAs
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) dprev[c][r] = d[c][r];
      a0[0] = a0[1]; a1[0] = a1[1];
      a0[1] = a0[2]; a1[1] = a1[2];
    }
    select(dprev, te - 1);
  }
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    if constexpr (TOPK == 1) {  // the 4 row offsets: smallest value, ties lowest row
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b4[c].t[r] == 0x7fffffff ? 0x7fffffff : b4[c].t[r] * 16 + 4 * g + r;
        const float v = __int_as_float(b4[c].k[r]);
        const bool take = v < best[c].v[0] || (v == best[c].v[0] && row < best[c].i[0]);
        best[c].v[0] = take ? v : best[c].v[0];
        best[c].i[0] = take ? row : best[c].i[0];
      }
    }
    lanegroup_merge<TOPK>(best[c]);
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < TOPK; ++q) {
        mv[w][c][c16][q] = best[c].v[q];
        mi[w][c][c16][q] = best[c].i[q];
      }
    }
  }
  __syncthreads();
  // wave c < CT merges column tile c's NW lists in wave order (row order; ties: lower row)
  if (w >= CT || g != 0) return;
  const int c = w;
  TopK<TOPK> m;
#pragma unroll
  for (int q = 0; q < TOPK; ++q) {
    m.v[q] = mv[0][c][c16][q];
    m.i[q] = mi[0][c][c16][q];
  }
#pragma unroll
  for (int ww = 1; ww < NW; ++ww) {
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      ov[q] = mv[ww][c][c16][q];
      oi[q] = mi[ww][c][c16][q];
    }
    m.merge(ov, oi);
  }
  const int j = (cg * CT + c) * 16 + c16;
  if (j >= N2) return;
  if (RS == 1) {
    const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      out_idx[o + q] = m.i[q] == 0x7fffffff ? -1 : m.i[q];
      if (out_dist) out_dist[o + q] = sqrtf(m.v[q]);
    }
  } else {
    const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * TOPK;
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      part_v[o + q] = m.v[q];
      part_i[o + q] = m.i[q];
    }
  }
}

// fd_wide_kernel (mode 0, top-1: the naive solver's argmin, the training step's and the IR's
// feature-distance pass): ONE launch, one wave per SIMD. Block = 4 waves = one CU = (crop b,
// column group cg of 4 x CT column tiles, row part rs); wave w holds column tiles
// CT (4 cg + w) + c, c < CT, in registers (their y operands, CT x 8 VGPRs) and every wave
// streams the block's row part from a double-buffered LDS chunk of 8 row tiles, which the four
// waves fill with the rows' emb operands (two tiles each, computed on the MFMA from x in the
// permuted slot order above: no transposition), one barrier per chunk. Per row tile a wave runs
// 4 groups of 4 column tiles x 8 MFMAs (4 independent accumulation chains); the selection of
// each group's 16 distances is interleaved into the next group's MFMAs at compile time (one
// wave per SIMD issues in order: the VALU selection fills the MFMA issue gaps). Row parts
// (RS > 1) combine in the launch: each block stores its columns' (distance bits, row) keys as
// 8-byte write-through stores, drains, and takes a ticket on arrivals[b][cg]; the block that
// draws RS - 1 reads the RS keys of each column with write-through loads (no fence: every
// handed-off byte is stored and loaded sc1, cdna_hip_programming.md §6 Guideline 16), keeps the
// smallest (value, then row) and resets the ticket (zero before the first launch on the buffer,
// zero after every launch).
__device__ __forceinline__ int med3i(int a, int b, int c) {  // v_med3_i32: the median of three
  int d;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
constexpr int kWideCT = 8;
constexpr int kWideChunk = 8;

template <int CT, int VAR = 0>
__global__ __launch_bounds__(256, 2) void fd_wide_kernel(
    const float* __restrict__ ex, int ldx, const float* __restrict__ C, const float* __restrict__ ey, int ldy,
    const int32_t* __restrict__ n1, const int32_t* __restrict__ n2, int V1max, int V2max, int NCG, int RS,
    int64_t* __restrict__ out_idx, float* __restrict__ out_dist, unsigned long long* part,
    int32_t* arrivals) {
  __shared__ __attribute__((aligned(16))) f32x4 lds[2 * kWideChunk * 128 + 4 * 64 + 4];
  f32x4* chunk = lds;                            // [2][kWideChunk][2][64]: A tiles in operand order
  f32x4* cop = lds + 2 * kWideChunk * 128;       // [2][2][64]: C in the emb MFMA's A order
  int* flag = reinterpret_cast<int*>(lds + 2 * kWideChunk * 128 + 4 * 64);
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 (hardware block L lands on XCD L % 8) when B % 8 == 0
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / per);
      k = q - (q / per) * per;
    } else {
      b = L / per;
      k = L - b * per;
    }
  }
  const int cg = k % NCG, rs = k / NCG;
  if constexpr (VAR == 7) {  // (development variant: an AGPR operand in the kernel, so the
    float z = 0.f;           // MFMAs are selected in their AGPR-accumulator form)
    asm volatile("; agpr %0" ::"a"(z));
  }
  const int lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  const int g = lane >> 4, c16 = lane & 15;
  const int N1 = n1[b], N2 = n2[b];
  const int nt = (N1 + 15) >> 4;
  const int tb = (nt * rs) / RS, te = (nt * (rs + 1)) / RS;  // the block's row tiles
  {  // C operand, staged once: thread (n, h, l) holds C[16 n + m][16 h + 4 gg + q], q = 0..3
    const float* Cb = C + (int64_t)b * kF * kF;
    const int n = threadIdx.x >> 7, h = (threadIdx.x >> 6) & 1, l = threadIdx.x & 63;
    const int m = l & 15, gg = l >> 4, row = 16 * n + m;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 16 * h + 4 * gg + q;
      v[q] = (row < kF && f < kF) ? Cb[min(row, kF - 1) * kF + min(f, kF - 1)] : 0.f;
    }
    cop[threadIdx.x] = f32x4{v[0], v[1], v[2], v[3]};
  }
  // column operands
  float bo[CT][8];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int j = (CT * (4 * cg + w) + c) * 16 + c16;
    const float* yr = ey + ((int64_t)b * V2max + min(j, V2max - 1)) * ldy;
    const float4 y0 = *reinterpret_cast<const float4*>(yr + 4 * g);
    const float4 y1 = *reinterpret_cast<const float4*>(yr + 16 + 4 * g);
    const bool ok = j < N2;
    float v[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    float part_ = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      v[s] = (ok && (s < 6 || g < 3)) ? v[s] : 0.f;
      part_ = fmaf(v[s], v[s], part_);
    }
    const float p1 = __shfl_xor(part_, 16), p2 = __shfl_xor(part_, 32), p3 = __shfl_xor(part_, 48);
    const float mine[4] = {part_, p1, p2, p3};
    float nrm = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];
    if (g == 3) {
      v[6] = 1.f;
      v[7] = nrm;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) bo[c][s] = v[s];
  }
  // x rows of two row tiles (this wave's emb share of a chunk), unmasked at a clamped row
  const float* xb = ex + (int64_t)b * V1max * ldx;
  auto xload = [&](int t0, float4 (&xv)[2][2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = min((t0 + u) * 16 + c16, V1max - 1);
      const float* xr = xb + (int64_t)row * ldx;
      xv[u][0] = *reinterpret_cast<const float4*>(xr + 4 * g);
      xv[u][1] = *reinterpret_cast<const float4*>(xr + 16 + 4 * g);
    }
  };
  auto emb_tile = [&](int tt, const float4 (&xv)[2], f32x4* dst) {
    const int row = tt * 16 + c16;
    const bool rok = row < N1;
    float xs[8] = {xv[0].x, xv[0].y, xv[0].z, xv[0].w, xv[1].x, xv[1].y, xv[1].z, xv[1].w};
#pragma unroll
    for (int s = 0; s < 8; ++s) xs[s] = (rok && (s < 6 || g < 3)) ? xs[s] : 0.f;
    float e[8];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x4 c0 = cop[(2 * n) * 64 + lane], c1 = cop[(2 * n + 1) * 64 + lane];
      const float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(cv[s], xs[s], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) e[4 * n + q] = acc[q];
    }
    float part_ = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) part_ = fmaf(e[s], e[s], part_);
    const float p1 = __shfl_xor(part_, 16), p2 = __shfl_xor(part_, 32), p3 = __shfl_xor(part_, 48);
    const float mine[4] = {part_, p1, p2, p3};
    float nrm = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) nrm += mine[q ^ g];
    float o[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) o[s] = -2.f * e[s];
    if (g == 3) {
      o[6] = rok ? nrm : __builtin_huge_valf();
      o[7] = 1.f;
    }
    dst[lane] = f32x4{o[0], o[1], o[2], o[3]};
    dst[64 + lane] = f32x4{o[4], o[5], o[6], o[7]};
  };
  // running (key, tile) per column tile and row offset r (Top1x4's scheme)
  int bk[CT][4], bt[CT][4];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bk[c][r] = 0x7f800000;
      bt[c][r] = 0x7fffffff;
    }
  constexpr int kClamp = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)
  auto sel = [&](const f32x4 (&acc)[4], int grp, int tt) {
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * grp + cc;
        if constexpr (VAR == 9) {  // (development variant: value only, one v_med3_i32)
          bk[c][r] = med3i(__float_as_int(acc[cc][r]), kClamp, bk[c][r]);
          continue;
        }
        if constexpr (VAR == 8) {  // (development variant: clamp + min in one v_med3_i32)
          const int nb = med3i(__float_as_int(acc[cc][r]), kClamp, bk[c][r]);  // bk >= kClamp
          bt[c][r] = nb < bk[c][r] ? tt : bt[c][r];
          bk[c][r] = nb;
          continue;
        }
        const int key = max(__float_as_int(acc[cc][r]), kClamp);
        if constexpr (VAR == 5) {  // (development variant: the value only, no row index)
          bk[c][r] = min(key, bk[c][r]);
          continue;
        }
        if constexpr (VAR == 6) {  // (development variant: round 4's integer select; the asm
          int dif = key - bk[c][r];  // hides the difference's range, else LLVM rewrites it as
          asm volatile("" : "+v"(dif));  // the compare + select below)
          int m = dif >> 31;  // -1 iff key < best (both keys in [kClamp, 0x7f800000])
          asm volatile("" : "+v"(m));
          bt[c][r] = (m & tt) | (~m & bt[c][r]);
          bk[c][r] = min(key, bk[c][r]);
          continue;
        }
        // compare + select (v_cmp into an SGPR pair, v_cndmask): 5 % faster than the integer
        // select (VAR 6) — on gfx950 the f32 MFMAs never co-execute with VALU work
        // (SQ_VALU_MFMA_COEXEC_CYCLES = 0 on this kernel), so every selection instruction adds
        // to the MFMA time; see DESIGN.md §5 'Feature distance'
        bt[c][r] = key < bk[c][r] ? tt : bt[c][r];
        bk[c][r] = min(key, bk[c][r]);
      }
  };
  const int nchunk = te > tb ? (te - tb + kWideChunk - 1) / kWideChunk : 0;
  float4 xv[2][2];
  if (nchunk > 0) xload(tb + 2 * w, xv);
  __syncthreads();  // cop staged
  if (nchunk > 0) {
    emb_tile(tb + 2 * w, xv[0], chunk + (2 * w) * 128);
    emb_tile(tb + 2 * w + 1, xv[1], chunk + (2 * w + 1) * 128);
  }
  __syncthreads();
  f32x4 acc[2][4];  // [group parity: group g accumulates into acc[g & 1]][column tile of the group]
  int prev_grp = -1, prev_t = 0;
  for (int ch = 0; ch < nchunk; ++ch) {
    const int c0 = tb + ch * kWideChunk;
    const f32x4* cb = chunk + (ch & 1) * kWideChunk * 128;
    const bool more = ch + 1 < nchunk;
    if (more) xload(c0 + kWideChunk + 2 * w, xv);
    const int ntile = min(kWideChunk, te - c0);
    f32x4 n0 = cb[lane], n1 = cb[64 + lane];  // the next tile's A fragment, one tile ahead
    for (int t = 0; t < ntile; ++t) {
      const f32x4 a0 = n0, a1 = n1;
      {
        const int tn = min(t + 1, ntile - 1);
        n0 = cb[tn * 128 + lane];
        n1 = cb[tn * 128 + 64 + lane];
      }
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
      for (int grp = 0; grp < CT / 4; ++grp) {
        f32x4 (&cur)[4] = acc[grp & 1];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) cur[cc] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (VAR == 2 || VAR == 3) {  // (development variants: no MFMAs)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
#pragma unroll
            for (int r = 0; r < 4; ++r) cur[cc][r] = av[r] + bo[4 * grp + cc][r];
        } else {
#pragma unroll
          for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              cur[cc] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bo[4 * grp + cc][s], cur[cc], 0, 0, 0);
        }
        // the previous group's selection, interleaved into this group's MFMAs
        if constexpr (VAR == 1 || VAR == 3) {  // (development variants: no selection)
          bk[grp][0] ^= __float_as_int(acc[(grp + 1) & 1][0][0]);
        } else if (grp > 0) {
          sel(acc[(grp - 1) & 1], grp - 1, c0 + t);
        } else if (prev_grp >= 0) {
          sel(acc[(CT / 4 - 1) & 1], CT / 4 - 1, prev_t);
        }
        if constexpr (VAR != 4) {  // (VAR 4, development variant: the compiler's own schedule)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // 5 VALU
          }
        }
      }
      prev_grp = CT / 4 - 1;
      prev_t = c0 + t;
    }
    if (more) {
      f32x4* nb = chunk + ((ch + 1) & 1) * kWideChunk * 128;
      emb_tile(c0 + kWideChunk + 2 * w, xv[0], nb + (2 * w) * 128);
      emb_tile(c0 + kWideChunk + 2 * w + 1, xv[1], nb + (2 * w + 1) * 128);
    }
    __syncthreads();
  }
  if (prev_grp >= 0) sel(acc[(CT / 4 - 1) & 1], CT / 4 - 1, prev_t);
  // per column tile: the 4 row offsets (smallest value, ties lowest row), then the lane groups
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    unsigned long long best = ~0ull;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned row = bt[c][r] == 0x7fffffff ? 0x7fffffffu : (unsigned)(bt[c][r] * 16 + 4 * g + r);
      const unsigned long long key = ((unsigned long long)(unsigned)bk[c][r] << 32) | row;
      best = key < best ? key : best;
    }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const unsigned long long o = ((unsigned long long)(unsigned)__shfl_xor((int)(best >> 32), off) << 32) |
                                   (unsigned)__shfl_xor((int)(best & 0xffffffffu), off);
      best = o < best ? o : best;
    }
    const int j = (CT * (4 * cg + w) + c) * 16 + c16;
    if (g != 0 || j >= N2) continue;
    if (RS == 1) {
      const unsigned row = (unsigned)(best & 0xffffffffu);
      out_idx[(int64_t)b * V2max + j] = row >= 0x7fffffffu ? -1 : (int64_t)row;
      if (out_dist) out_dist[(int64_t)b * V2max + j] = sqrtf(__int_as_float((int)(best >> 32)));
    } else {
      __hip_atomic_store(part + ((int64_t)b * RS + rs) * V2max + j, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (RS == 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through keys
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(arrivals + (int64_t)b * NCG + cg, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == RS - 1;
    if (last) __hip_atomic_store(arrivals + (int64_t)b * NCG + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (orders the loads after the ticket)
  for (int jj = threadIdx.x; jj < 4 * CT * 16; jj += 256) {
    const int j = CT * 4 * 16 * cg + jj;
    if (j >= N2) continue;
    unsigned long long best = ~0ull;
    for (int r = 0; r < RS; ++r) {
      const unsigned long long key =
          __hip_atomic_load(part + ((int64_t)b * RS + r) * V2max + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      best = key < best ? key : best;
    }
    const unsigned row = (unsigned)(best & 0xffffffffu);
    out_idx[(int64_t)b * V2max + j] = row >= 0x7fffffffu ? -1 : (int64_t)row;
    if (out_dist) out_dist[(int64_t)b * V2max + j] = sqrtf(__int_as_float((int)(best >> 32)));
  }
}

// pass 3 (RS > 1): grid (ceil(V2max / 256), B): merge the RS partial lists of each column in
// row-split order (ties: lower row).
template <int TOPK>
__global__ __launch_bounds__(256) void fd_merge_kernel(const float* __restrict__ part_v,
                                                       const int32_t* __restrict__ part_i,
                                                       const int32_t* __restrict__ n2, int V2max, int RS,
                                                       int64_t* __restrict__ out_idx, float* __restrict__ out_dist) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n2[b]) return;
  TopK<TOPK> best;
  best.init();
  for (int rs = 0; rs < RS; ++rs) {
    const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * TOPK;
    float ov[TOPK];
    int oi[TOPK];
#pragma unroll
    for (int q = 0; q < TOPK; ++q) {
      ov[q] = part_v[o + q];
      oi[q] = part_i[o + q];
    }
    best.merge(ov, oi);
  }
  const int64_t o = ((int64_t)b * V2max + j) * TOPK;
#pragma unroll
  for (int q = 0; q < TOPK; ++q) {
    out_idx[o + q] = best.i[q] == 0x7fffffff ? -1 : best.i[q];
    if (out_dist) out_dist[o + q] = sqrtf(best.v[q]);
  }
}

struct FdPlan {
  int T1, T2, NCG, RS;
  int64_t a_bytes, b_bytes, na_bytes, nb_bytes, pv_bytes, pi_bytes;
};

inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

inline FdPlan fd_plan(int B, int V1max, int V2max, int topk, int mode) {
  FdPlan p{};
  p.T1 = (V1max + 15) / 16;
  p.T2 = (V2max + 15) / 16;
  p.NCG = (p.T2 + kWaves * kCW - 1) / (kWaves * kCW);
  const int64_t blocks = (int64_t)B * p.NCG;
  int rs = blocks >= 512 ? 1 : (int)((512 + blocks - 1) / blocks);
  const int max_rs = std::max(1, p.T1 / (2 * kCH));  // at least two chunks per row part
  p.RS = std::min(rs, max_rs);
  const int TB = tile_bytes(mode);
  p.a_bytes = al256((int64_t)B * p.T1 * TB);
  p.b_bytes = al256((int64_t)B * p.T2 * TB);
  p.na_bytes = mode ? al256((int64_t)B * p.T1 * 16 * 4) : 0;
  p.nb_bytes = mode ? al256((int64_t)B * p.T2 * 16 * 4) : 0;
  p.pv_bytes = p.RS > 1 ? al256((int64_t)B * p.RS * V2max * topk * 4) : 0;
  p.pi_bytes = p.pv_bytes;
  return p;
}

// the fused fp32 pass: NW = 8 waves per block, CT column tiles per wave (4 for the argmin, 2 for
// the top-5 lists), row parts RS so that the grid holds >= 512 blocks (two per CU)
constexpr int kFusedNW = 8;
inline int fused_ct(int topk) { return topk == 1 ? 4 : 2; }

struct FusedPlan {
  int NCG, RS;
  int64_t ctr_bytes, pv_bytes;
};

inline FusedPlan fused_plan(int B, int V1max, int V2max, int topk) {
  FusedPlan p{};
  const int T1 = (V1max + 15) / 16, T2 = (V2max + 15) / 16;
  p.NCG = std::max(1, (T2 + kFusedNW * fused_ct(topk) - 1) / (kFusedNW * fused_ct(topk)));
  const int64_t blocks = (int64_t)B * p.NCG;
  const int rs = blocks >= 512 ? 1 : (int)((512 + blocks - 1) / blocks);
  p.RS = std::max(1, std::min(rs, T1));
  p.pv_bytes = p.RS > 1 ? al256((int64_t)B * p.RS * V2max * topk * 4) : 0;
  p.ctr_bytes = al256((int64_t)B * std::max(T2, 1) * 4);  // (>= B x NCG of every one-launch plan)
  return p;
}

struct WidePlan {
  int NCG, RS;
  int64_t part_bytes;
};

inline WidePlan wide_plan(int B, int V1max, int V2max) {
  WidePlan p{};
  const int T1 = (V1max + 15) / 16, T2 = (V2max + 15) / 16;
  p.NCG = std::max(1, (T2 + 4 * kWideCT - 1) / (4 * kWideCT));
  const int64_t blocks = (int64_t)B * p.NCG;
#ifdef PK_DEVBUILD
  static const int target = [] {  // development knob PK_FD_BLOCKS: grid target (256 = 1 per CU)
    const char* e = std::getenv("PK_FD_BLOCKS");
    return e ? std::atoi(e) : 256;
  }();
#else
  constexpr int target = 256;
#endif
  const int rs = blocks >= target ? 1 : (int)((target + blocks - 1) / blocks);
  p.RS = std::max(1, std::min(rs, T1));
  p.part_bytes = p.RS > 1 ? al256((int64_t)B * p.RS * V2max * 8) : 0;
  return p;
}

// the split fp32 path: CT column tiles per block (one column group), NW waves splitting the rows
constexpr int kColsNW = 8;
inline int cols_ct(int topk) { return topk == 1 ? 4 : 2; }

struct ColsPlan {
  int T1, NCG, RS;
  int64_t a_bytes, pv_bytes;
};

inline ColsPlan cols_plan(int B, int V1max, int V2max, int topk) {
  ColsPlan p{};
  p.T1 = (V1max + 15) / 16;
  const int T2 = (V2max + 15) / 16;
  p.NCG = std::max(1, (T2 + cols_ct(topk) - 1) / cols_ct(topk));
  const int64_t blocks = (int64_t)B * p.NCG;
  const int rs = blocks >= 512 ? 1 : (int)((512 + blocks - 1) / blocks);
  p.RS = std::max(1, std::min(rs, p.T1 / kColsNW));
  p.a_bytes = al256((int64_t)B * p.T1 * 2048);
  p.pv_bytes = p.RS > 1 ? al256((int64_t)B * p.RS * V2max * topk * 4) : 0;
  return p;
}

}  // namespace

extern "C" int64_t pk_feat_dist_work_size(int B, int V1max, int V2max, int topk, int mode) {
  if (B < 0 || V1max < 0 || V2max < 0 || !(topk == 1 || topk == 5) || mode < 0 || mode > 2) return -1;
  const FdPlan p = fd_plan(B, V1max, V2max, topk, mode);
  const int64_t two_pass = p.a_bytes + p.b_bytes + p.na_bytes + p.nb_bytes + p.pv_bytes + p.pi_bytes;
  if (mode != 0) return two_pass;
  // mode 0: the fused pass's arrival words lead the buffer (pk_feat_dist_counter_bytes), then the
  // larger of its partial lists and the fallback paths' scratch (unaligned operand rows)
  const FusedPlan f = fused_plan(B, V1max, V2max, topk);
  const ColsPlan c = cols_plan(B, V1max, V2max, topk);
  const WidePlan wp = wide_plan(B, V1max, V2max);
  return f.ctr_bytes + std::max(std::max(std::max(two_pass, 2 * f.pv_bytes), c.a_bytes + 2 * c.pv_bytes), wp.part_bytes);
}

extern "C" int64_t pk_feat_dist_counter_bytes(int B, int V1max, int V2max, int topk, int mode) {
  if (B < 0 || V1max < 0 || V2max < 0 || !(topk == 1 || topk == 5) || mode < 0 || mode > 2) return -1;
  return mode == 0 ? fused_plan(B, V1max, V2max, topk).ctr_bytes : 0;
}

extern "C" int pk_feat_dist_topk(const float* evecs_x, int ldx, const float* C, const float* evecs_y, int ldy,
                                 const int32_t* n1, const int32_t* n2, int B, int V1max, int V2max, int topk,
                                 int mode, void* work, int64_t work_bytes, int64_t* out_idx, float* out_dist,
                                 void* stream) {
  PK_REQUIRE(B >= 0 && V1max >= 0 && V2max >= 0 && ldx >= kF && ldy >= kF && (topk == 1 || topk == 5));
  PK_REQUIRE(mode >= 0 && mode <= 2);
  if (B == 0 || V2max == 0) return PK_OK;
  PK_REQUIRE(evecs_x && C && evecs_y && n1 && n2 && work && out_idx);
  PK_REQUIRE(work_bytes >= pk_feat_dist_work_size(B, V1max, V2max, topk, mode));
  hipStream_t s = pk::as_stream(stream);
  const bool aligned = (ldx % 4) == 0 && (ldy % 4) == 0 && (reinterpret_cast<uintptr_t>(evecs_x) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(evecs_y) & 15) == 0;
#ifdef PK_DEVBUILD
  static const int path = [] {  // development knob PK_FD_PATH: 0 default (top-1: one launch, top-5: two
                                //   passes), 1 rows + cols, 2 two-pass, 3 fused 8-wave pass
    const char* e = std::getenv("PK_FD_PATH");
    return e ? std::atoi(e) : 0;
  }();
#else
  constexpr int path = 0;
#endif
  // mode 0 work layout: [arrival words][scratch of the path taken]
  const int64_t ctr_bytes = mode == 0 ? fused_plan(B, V1max, V2max, topk).ctr_bytes : 0;
  int32_t* arrivals = static_cast<int32_t*>(work);
  work = static_cast<char*>(work) + ctr_bytes;
  if (mode == 0 && aligned && V1max > 0 && topk == 1 && path == 0) {  // one wave per SIMD, one launch
    const WidePlan wp = wide_plan(B, V1max, V2max);
    auto* part = static_cast<unsigned long long*>(work);
    const dim3 wgrid((unsigned)((int64_t)B * wp.NCG * wp.RS));
#ifdef PK_DEVBUILD
    static const int wvar = [] {  // development knob PK_FD_VAR: 1 no selection, 2 no MFMAs, 3 neither,
      // 4 no sched_group_barrier, 5 value-only selection, 6 integer select, 7 AGPR accumulators,
      // 8 med3 + compare + select, 9 value-only med3
      const char* e = std::getenv("PK_FD_VAR");
      return e ? std::atoi(e) : 0;
    }();
#define PK_FDW(V) hipLaunchKernelGGL((fd_wide_kernel<kWideCT, V>), wgrid, dim3(256), 0, s, evecs_x, ldx, C, evecs_y, \
                                     ldy, n1, n2, V1max, V2max, wp.NCG, wp.RS, out_idx, out_dist, part, arrivals)
    if (wvar == 1) PK_FDW(1); else if (wvar == 2) PK_FDW(2); else if (wvar == 3) PK_FDW(3);
    else if (wvar == 4) PK_FDW(4); else if (wvar == 5) PK_FDW(5); else if (wvar == 6) PK_FDW(6); else if (wvar == 7) PK_FDW(7); else if (wvar == 8) PK_FDW(8); else if (wvar == 9) PK_FDW(9); else PK_FDW(0);
#undef PK_FDW
#else
    hipLaunchKernelGGL(fd_wide_kernel<kWideCT>, wgrid, dim3(256), 0, s, evecs_x, ldx, C, evecs_y, ldy, n1, n2, V1max,
                       V2max, wp.NCG, wp.RS, out_idx, out_dist, part, arrivals);
#endif
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  if (mode == 0 && aligned && V1max > 0 && path == 1) {  // rows + cols
    const ColsPlan c = cols_plan(B, V1max, V2max, topk);
    f32x4* A = static_cast<f32x4*>(work);
    float* pv = c.RS > 1 ? reinterpret_cast<float*>(static_cast<char*>(work) + c.a_bytes) : nullptr;
    int32_t* pi = c.RS > 1 ? reinterpret_cast<int32_t*>(static_cast<char*>(work) + c.a_bytes + c.pv_bytes) : nullptr;
    hipLaunchKernelGGL(fd_rows_kernel, dim3((c.T1 + 3) / 4, B), dim3(256), 0, s, evecs_x, ldx, C, n1, V1max, c.T1, A);
    PK_CHECK_LAUNCH();
    const dim3 grid((unsigned)((int64_t)B * c.NCG * c.RS)), block(64 * kColsNW);
    if (topk == 1)
      hipLaunchKernelGGL((fd_cols_kernel<1, 4, kColsNW>), grid, block, 0, s, A, evecs_y, ldy, n1, n2, V2max, c.T1, c.NCG,
                         c.RS, out_idx, out_dist, pv, pi);
    else
      hipLaunchKernelGGL((fd_cols_kernel<5, 2, kColsNW>), grid, block, 0, s, A, evecs_y, ldy, n1, n2, V2max, c.T1, c.NCG,
                         c.RS, out_idx, out_dist, pv, pi);
    PK_CHECK_LAUNCH();
    if (c.RS > 1) {
      const dim3 mg((V2max + 255) / 256, B);
      if (topk == 1)
        hipLaunchKernelGGL(fd_merge_kernel<1>, mg, dim3(256), 0, s, pv, pi, n2, V2max, c.RS, out_idx, out_dist);
      else
        hipLaunchKernelGGL(fd_merge_kernel<5>, mg, dim3(256), 0, s, pv, pi, n2, V2max, c.RS, out_idx, out_dist);
      PK_CHECK_LAUNCH();
    }
    return PK_OK;
  }
  if (mode == 0 && aligned && V1max > 0 && path == 3) {  // the fused pass
    const FusedPlan f = fused_plan(B, V1max, V2max, topk);
    float* pv = f.RS > 1 ? static_cast<float*>(work) : nullptr;
    int32_t* pi = f.RS > 1 ? reinterpret_cast<int32_t*>(static_cast<char*>(work) + f.pv_bytes) : nullptr;
    const dim3 grid((unsigned)((int64_t)B * f.NCG * f.RS)), block(64 * kFusedNW);
#ifdef PK_DEVBUILD
    static const int var = [] {  // development knob PK_FD_VAR (limiter study): 1 no selection, 2 no
      const char* e = std::getenv("PK_FD_VAR");  // main-loop MFMAs, 3 neither
      return e ? std::atoi(e) : 0;
    }();
    if (topk == 1 && var >= 1 && var <= 3) {
#define PK_FDV(V) hipLaunchKernelGGL((fd_fused_kernel<1, 4, kFusedNW, V>), grid, block, 0, s, evecs_x, ldx, C, evecs_y, \
                                     ldy, n1, n2, V1max, V2max, f.NCG, f.RS, out_idx, out_dist, pv, pi, arrivals)
      if (var == 1) PK_FDV(1); else if (var == 2) PK_FDV(2); else PK_FDV(3);
#undef PK_FDV
    } else
#endif
    if (topk == 1)
      hipLaunchKernelGGL((fd_fused_kernel<1, 4, kFusedNW>), grid, block, 0, s, evecs_x, ldx, C, evecs_y, ldy, n1, n2,
                         V1max, V2max, f.NCG, f.RS, out_idx, out_dist, pv, pi, arrivals);
    else
      hipLaunchKernelGGL((fd_fused_kernel<5, 2, kFusedNW>), grid, block, 0, s, evecs_x, ldx, C, evecs_y, ldy, n1, n2,
                         V1max, V2max, f.NCG, f.RS, out_idx, out_dist, pv, pi, arrivals);
    PK_CHECK_LAUNCH();
    return PK_OK;
  }
  const FdPlan p = fd_plan(B, V1max, V2max, topk, mode);
  char* wp = static_cast<char*>(work);
  char* A = wp;
  char* Bq = A + p.a_bytes;
  float* nA = mode ? reinterpret_cast<float*>(Bq + p.b_bytes) : nullptr;
  float* nB = mode ? reinterpret_cast<float*>(Bq + p.b_bytes + p.na_bytes) : nullptr;
  float* pv = p.RS > 1 ? reinterpret_cast<float*>(Bq + p.b_bytes + p.na_bytes + p.nb_bytes) : nullptr;
  int32_t* pi = p.RS > 1 ? reinterpret_cast<int32_t*>(reinterpret_cast<char*>(pv) + p.pv_bytes) : nullptr;
  const dim3 pg((std::max(p.T1, p.T2) + kPrepWaves - 1) / kPrepWaves, B, 2);
#define PK_FD_PREP(M)                                                                                              \
  hipLaunchKernelGGL((fd_prep_kernel<M>), pg, dim3(64 * kPrepWaves), 0, s, evecs_x, ldx, C, evecs_y, ldy, n1, n2, V1max, V2max, \
                     p.T1, p.T2, A, Bq, nA, nB)
  if (mode == 0) PK_FD_PREP(0); else if (mode == 1) PK_FD_PREP(1); else PK_FD_PREP(2);
#undef PK_FD_PREP
  PK_CHECK_LAUNCH();
  const dim3 grid((unsigned)((int64_t)B * p.NCG * p.RS)), block(64 * kWaves);
#ifdef PK_DEVBUILD
  static const int direct = [] {  // development knob PK_FD_DIRECT: 0 = LDS-ring main pass
    const char* e = std::getenv("PK_FD_DIRECT");
    return e ? std::atoi(e) : 1;
  }();
#define PK_FD_MAIN(K, M)                                                                                          \
  do {                                                                                                            \
    if (direct)                                                                                                   \
      hipLaunchKernelGGL((fd_main_direct_kernel<K, M>), grid, block, 0, s, A, Bq, nA, nB, n1, n2, p.T1, p.T2,     \
                         V2max, p.NCG, p.RS, out_idx, out_dist, pv, pi);                                          \
    else                                                                                                          \
      hipLaunchKernelGGL((fd_main_kernel<K, M>), grid, block, 0, s, A, Bq, nA, nB, n1, n2, p.T1, p.T2, V2max,     \
                         p.NCG, p.RS, out_idx, out_dist, pv, pi);                                                 \
  } while (0)
#else
#define PK_FD_MAIN(K, M)                                                                                          \
  hipLaunchKernelGGL((fd_main_direct_kernel<K, M>), grid, block, 0, s, A, Bq, nA, nB, n1, n2, p.T1, p.T2, V2max,  \
                     p.NCG, p.RS, out_idx, out_dist, pv, pi)
#endif
  if (topk == 1) {
    if (mode == 0) PK_FD_MAIN(1, 0); else if (mode == 1) PK_FD_MAIN(1, 1); else PK_FD_MAIN(1, 2);
  } else {
    if (mode == 0) PK_FD_MAIN(5, 0); else if (mode == 1) PK_FD_MAIN(5, 1); else PK_FD_MAIN(5, 2);
  }
#undef PK_FD_MAIN
  PK_CHECK_LAUNCH();
  if (p.RS > 1) {
    const dim3 mg((V2max + 255) / 256, B);
    if (topk == 1)
      hipLaunchKernelGGL(fd_merge_kernel<1>, mg, dim3(256), 0, s, pv, pi, n2, V2max, p.RS, out_idx, out_dist);
    else
      hipLaunchKernelGGL(fd_merge_kernel<5>, mg, dim3(256), 0, s, pv, pi, n2, V2max, p.RS, out_idx, out_dist);
    PK_CHECK_LAUNCH();
  }
  return PK_OK;
}
