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
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

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

// Top-1 fp32 (round 5, the default argmin of the training step's naive point map and the IR):
// nothing kept across calls (no arrival words, no zeroing contract on `work`).
//
// Pass 1, fd_top1_prep_kernel (one wave per 16-row tile of x): the row operand
// A = [-2 emb, |emb|^2, 1] with emb = x C^T, computed once per tile on the f32 MFMA and stored in
// the main contraction's A-operand order (2 KB per tile) — rather than by every column group that
// reads the tile (each tile feeds 8 blocks at configs[1]: 16 of every 80 MFMAs were emb MFMAs).
// Contraction-slot order: slot (step s = 4 n + q, lane group g) holds feature 16 n + 4 g + q, so
// the emb MFMA's D layout (C x^T: lane (point c, group g) holds features 16 n + 4 g + q) IS the
// A-operand layout, and a lane's y values are two contiguous float4 of its row. Slots 30, 31
// carry torch.cdist's augmented terms [-2 emb, |emb|^2, 1] . [y, 1, |y|^2]; padding rows get an
// +inf |emb|^2 slot (never selected).
// Pass 2, fd_top1_kernel: block = (crop b, column group of kTop1CT = 8 column tiles = 128
// columns, row part rs); its 8 waves (two per SIMD) share the group's B operands (staged once per
// block through LDS, then in registers) and split the row part's tiles, streaming their A tiles
// from L2 two tiles ahead; so every column's argmin over the row part is finished inside the
// block (the waves' results meet in LDS). Per tile: 8 column tiles in pairs of accumulation
// chains, the selection of a pair behind the next pair's MFMAs. Selection per distance: compare
// into a lane mask, select the tile, min (the running (key, tile) of each (column tile, row offset
// r) per lane; key = the distance's bits as a signed int; ties keep the earlier tile, then the
// lower r / lane group / wave = the lower row). torch.cdist's clamp_min(1e-30) is not applied per
// distance: a column whose best key is <= bits(1e-30) (a zero, tiny or negative expansion) is
// rescanned for its first row at or below the clamp (wave-uniform, rare: coincident features).
// With RS > 1 (small batches) the row parts' keys go to scratch and fd_top1_merge_kernel takes
// the minimum. The development variant PK_FD_VAR=20 forms the emb operands inside the main pass
// instead (one launch; the round-5 first form, A/B).
constexpr int kTop1CT = 8;
constexpr int kTop1Waves = 8;  // two per SIMD: one wave's dependency stalls are the other's MFMA time
#ifdef PK_DEVBUILD
__device__ unsigned long long g_fd_stamps[4096 * 16];  // (development: VAR 13 phase stamps per block)
#define FD_STAMP(i, v)                                                  \
  do {                                                                  \
    if constexpr (VAR == 13) {                                          \
      if (threadIdx.x == 0) g_fd_stamps[blockIdx.x * 16 + (i)] = (v);   \
    }                                                                   \
  } while (0)
#else
#define FD_STAMP(i, v) \
  do {                 \
  } while (0)
#endif
constexpr int kClampBits = 0x0da24260;  // bits of 1e-30f: clamp_min(1e-30) (cdist mm path)

// -2 C in the emb MFMA's A order: lane (m, gg) holds -2 C[16 n + m][16 h + 4 gg + q] at s = 4 h + q
__device__ __forceinline__ void top1_cv(const float* __restrict__ Cb, int c16, int g, float (&cv)[2][8]) {
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int row = 16 * n + c16, f = 16 * (s8 >> 2) + 4 * g + (s8 & 3);
      const float cval = Cb[min(row, kF - 1) * kF + min(f, kF - 1)];  // (unconditional load)
      cv[n][s8] = (row < kF && f < kF) ? -2.f * cval : 0.f;
    }
}

// x row t*16 + c16 of a crop (a padding row reads row 0: finite, its distance is +inf anyway)
__device__ __forceinline__ void top1_xload(const float* __restrict__ xb, int ldx, int N1, int t, int c16, int g,
                                           float4 (&xv)[2]) {
  const int r0 = t * 16 + c16;
  const float* xr = xb + (int64_t)(r0 < N1 ? r0 : 0) * ldx;
  xv[0] = *reinterpret_cast<const float4*>(xr + 4 * g);
  xv[1] = *reinterpret_cast<const float4*>(xr + 16 + 4 * g);
}

// -2 emb of a tile on the MFMA with -2 C (exact power-of-two scaling of emb)
__device__ __forceinline__ void top1_emb_mfma(const float (&cv)[2][8], const float4 (&xv)[2], f32x4 (&e)[2]) {
  const float xs[8] = {xv[0].x, xv[0].y, xv[0].z, xv[0].w, xv[1].x, xv[1].y, xv[1].z, xv[1].w};
#pragma unroll
  for (int n = 0; n < 2; ++n) e[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int n = 0; n < 2; ++n) e[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(cv[n][s], xs[s], e[n], 0, 0, 0);
}

// the A operand [-2 emb, |emb|^2, 1]: |emb|^2 = (the sum of squares of -2 emb) / 4 (exact), the
// lane groups' partials added in the order 0, 1, 2, 3; every lane gets them by row swaps (VALU,
// no LDS round trip): the 16-swap pairs rows (0,1) / (2,3), the 32-swaps then rows 0-1 with 2-3
__device__ __forceinline__ void top1_emb_norm(int t, int N1, int c16, int g, const f32x4 (&e)[2], float (&a)[8]) {
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int q = 0; q < 4; ++q) a[4 * n + q] = e[n][q];
  float part_ = 0.f;
#pragma unroll
  for (int s = 0; s < 8; ++s) part_ = fmaf(a[s], a[s], part_);
  const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(part_), __float_as_uint(part_), false, false);
  const auto e32 = __builtin_amdgcn_permlane32_swap(s16[0], s16[0], false, false);  // {p0, p2}
  const auto o32 = __builtin_amdgcn_permlane32_swap(s16[1], s16[1], false, false);  // {p1, p3}
  const float nrm = 0.25f * (((__uint_as_float(e32[0]) + __uint_as_float(o32[0])) + __uint_as_float(e32[1])) +
                             __uint_as_float(o32[1]));
  const bool g3 = g == 3;
  a[6] = g3 ? (t * 16 + c16 < N1 ? nrm : __builtin_huge_valf()) : a[6];
  a[7] = g3 ? 1.f : a[7];
}

// pass 1: grid NTG * B (NTG = ceil(T1 / 8) tile groups per crop), 8 waves: wave = one 16-row tile
// of crop b's x side, its A tile [-2 emb, |emb|^2, 1]; -2 C staged once per block in LDS with a
// 32-float row pitch so each lane reads its 16 C values as four 16-B loads. Tiles at or past a
// crop's valid rows are skipped (pass 2 never reads them). Blocks are numbered as pass 2's (crop
// b's blocks on XCD b % 8 when B % 8 == 0), and each also touches its share of crop b's y rows —
// pass 2's column operands — with loads issued beside its own and consumed at the end, so pass 2's
// staging finds them warm on the XCD that reads them.
__global__ __launch_bounds__(512) void fd_top1_prep_kernel(const float* __restrict__ ex, int ldx,
                                                          const float* __restrict__ C,
                                                          const int32_t* __restrict__ n1, int V1max, int T1,
                                                          f32x4* __restrict__ Atile, const float* __restrict__ ey,
                                                          int ldy, const int32_t* __restrict__ n2, int V2max,
                                                          int NTG) {
  __shared__ __attribute__((aligned(16))) float sc[kK * 32];
  const int lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  const int g = lane >> 4, c16 = lane & 15;
  const int B = (int)(gridDim.x / NTG);
  int b, tg;
  {
    const int L = blockIdx.x;
    if ((B & 7) == 0) {
      const int x8 = L & 7, q = L >> 3;
      b = x8 + 8 * (q / NTG);
      tg = q - (q / NTG) * NTG;
    } else {
      b = L / NTG;
      tg = L - b * NTG;
    }
  }
  const int t = tg * 8 + w;
  const int N1 = n1[b];
  const bool act = t < T1 && t * 16 < N1;
  float4 xv[2];
  if (act) top1_xload(ex + (int64_t)b * V1max * ldx, ldx, N1, t, c16, g, xv);
  f32x4 yt[4];  // the y touch: rows [r0, r1) of crop b, 8 x 16 B each (up to 256 rows per block)
  {
    const int N2 = n2[b];
    const int r0 = (int)((int64_t)N2 * tg / NTG), r1 = (int)((int64_t)N2 * (tg + 1) / NTG);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = threadIdx.x + 512 * u;
      yt[u] = e < (r1 - r0) * 8
                  ? *reinterpret_cast<const f32x4*>(ey + ((int64_t)b * V2max + r0 + (e >> 3)) * ldy + 4 * (e & 7))
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const float* Cb = C + (int64_t)b * kF * kF;
  for (int e = threadIdx.x; e < kK * 32; e += 512) {  // -2 C, zero-padded to 32 x 32
    const int row = e >> 5, f = e & 31;
    const float cval = Cb[min(row, kF - 1) * kF + min(f, kF - 1)];
    sc[e] = (row < kF && f < kF) ? -2.f * cval : 0.f;
  }
  __syncthreads();
  if (act) {
    float cv[2][8];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 v4 = *reinterpret_cast<const f32x4*>(sc + (16 * n + c16) * 32 + 16 * h + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) cv[n][4 * h + q] = v4[q];
      }
    f32x4 e[2];
    top1_emb_mfma(cv, xv, e);
    float a[8];
    top1_emb_norm(t, N1, c16, g, e, a);
    f32x4* dst = Atile + ((int64_t)b * T1 + t) * 128;
    dst[lane] = f32x4{a[0], a[1], a[2], a[3]};
    dst[64 + lane] = f32x4{a[4], a[5], a[6], a[7]};
  }
  asm volatile("" ::"v"(yt[0]), "v"(yt[1]), "v"(yt[2]), "v"(yt[3]));  // (keeps the touch loads)
}

// pass 2 (EMB: form the emb operands in this pass instead of reading pass 1's tiles)
template <int VAR = 0, bool EMB = false>
__global__ __launch_bounds__(64 * kTop1Waves, 1) void fd_top1_kernel(
    const float* __restrict__ ex, int ldx, const float* __restrict__ C, const f32x4* __restrict__ Atile, int T1,
    const float* __restrict__ ey, int ldy, const int32_t* __restrict__ n1, const int32_t* __restrict__ n2, int V1max,
    int V2max, int NCG, int RS, int64_t* __restrict__ out_idx, float* __restrict__ out_dist,
    unsigned long long* __restrict__ part) {
  __shared__ f32x4 sB[kTop1CT][2][64];      // the column operands in B order (16 KB)
  __shared__ float sPart[4][kTop1CT * 16];  // per lane group partial |y|^2
  __shared__ unsigned long long wkeys[kTop1Waves][kTop1CT * 16];
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
  FD_STAMP(0, __builtin_amdgcn_s_memtime());
  FD_STAMP(5, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  FD_STAMP(6, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20));
  const int j0 = cg * kTop1CT * 16;
  const int tid = threadIdx.x, lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  // the column operands' loads go out beside the crop sizes' (their addresses do not need them)
  const int sjj = tid & (kTop1CT * 16 - 1), sgy = tid >> 7;  // staging: column sjj, lane group sgy
  const float* syr = ey + ((int64_t)b * V2max + min(j0 + sjj, V2max - 1)) * ldy;
  const float4 sy0 = *reinterpret_cast<const float4*>(syr + 4 * sgy);
  const float4 sy1 = *reinterpret_cast<const float4*>(syr + 16 + 4 * sgy);
  const int N1 = n1[b], N2 = n2[b];
  const int g = lane >> 4, c16 = lane & 15;
  const int nt = (N1 + 15) >> 4;
  const int Q = RS * kTop1Waves, qw = rs * kTop1Waves + w;
  const int tb = (int)((int64_t)nt * qw / Q), te = (int)((int64_t)nt * (qw + 1) / Q);  // this wave's row tiles
  const float* xb = ex + (int64_t)b * V1max * ldx;
  const f32x4* Ab = Atile + (int64_t)b * T1 * 128;
  // the operand of tile t: pass 1's A tile (two 16-B loads per lane), or x rows to embed here
  auto opload = [&](int t, float4 (&xv)[2]) {
    if constexpr (EMB) {
      top1_xload(xb, ldx, N1, t, c16, g, xv);
    } else {
      const f32x4 u0 = Ab[(int64_t)t * 128 + lane], u1 = Ab[(int64_t)t * 128 + 64 + lane];
      xv[0] = make_float4(u0[0], u0[1], u0[2], u0[3]);
      xv[1] = make_float4(u1[0], u1[1], u1[2], u1[3]);
    }
  };
  float cv[2][8];
  if constexpr (EMB) top1_cv(C + (int64_t)b * kF * kF, c16, g, cv);
  auto emb = [&](int t, const float4 (&xv)[2], float (&a)[8]) {
    if constexpr (EMB) {
      f32x4 e[2];
      top1_emb_mfma(cv, xv, e);
      top1_emb_norm(t, N1, c16, g, e, a);
    } else {
      a[0] = xv[0].x, a[1] = xv[0].y, a[2] = xv[0].z, a[3] = xv[0].w;
      a[4] = xv[1].x, a[5] = xv[1].y, a[6] = xv[1].z, a[7] = xv[1].w;
    }
  };
  float4 xc[2], xn[2];
  float a[8];
  if (tb < te) {
    opload(tb, xc);
    opload(min(tb + 1, te - 1), xn);
  }
  float bo[kTop1CT][8];
  {  // staging: the block's 128 columns' [y, 1, |y|^2] in B order, through LDS
    const int jj = sjj, gy = sgy;  // column jj of the block, lane group gy
    const int j = j0 + jj;
    const bool ok = j < N2;
    float v[8] = {sy0.x, sy0.y, sy0.z, sy0.w, sy1.x, sy1.y, sy1.z, sy1.w};
    float part_ = 0.f;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      v[s8] = (ok && (s8 < 6 || gy < 3)) ? v[s8] : 0.f;
      part_ = fmaf(v[s8], v[s8], part_);
    }
    sPart[gy][jj] = part_;
    if (j0 >= N2) return;  // (block-uniform; after the loads' consumers, so they are not sunk past it)
    if (tb < te) emb(tb, xc, a);  // (the first tile's operand while the partials meet)
    __syncthreads();
    if (gy == 3) {  // |y|^2: the lane groups' partials in the order 0, 1, 2, 3
      float nrm = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) nrm += sPart[q][jj];
      v[6] = 1.f;
      v[7] = nrm;
    }
    const int c = jj >> 4, l = gy * 16 + (jj & 15);
    sB[c][0][l] = f32x4{v[0], v[1], v[2], v[3]};
    sB[c][1][l] = f32x4{v[4], v[5], v[6], v[7]};
    __syncthreads();
#pragma unroll
    for (int c2 = 0; c2 < kTop1CT; ++c2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 t4 = sB[c2][h][lane];
#pragma unroll
        for (int q = 0; q < 4; ++q) bo[c2][4 * h + q] = t4[q];
      }
  }
  FD_STAMP(1, __builtin_amdgcn_s_memtime());
  int bk[kTop1CT][4], bt[kTop1CT][4];
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bk[c][r] = 0x7f800000;
      bt[c][r] = 0x07ffffff;  // no row yet: its row index (16 bt + 4 g + r) >= 0x7ffffff0
    }
  // per distance: compare into a lane mask, select the tile, min. Four compares into four SGPR
  // pairs before their selects (no VCC write -> read hazard wait states between them)
  auto sel = [&](const f32x4& acc, int c, int t) {
    unsigned long long m0, m1, m2, m3;
    asm("v_cmp_lt_i32_e64 %[m0], %[k0], %[b0]\n\t"
        "v_cmp_lt_i32_e64 %[m1], %[k1], %[b1]\n\t"
        "v_cmp_lt_i32_e64 %[m2], %[k2], %[b2]\n\t"
        "v_cmp_lt_i32_e64 %[m3], %[k3], %[b3]\n\t"
        "v_min_i32_e32 %[b0], %[k0], %[b0]\n\t"
        "v_min_i32_e32 %[b1], %[k1], %[b1]\n\t"
        "v_min_i32_e32 %[b2], %[k2], %[b2]\n\t"
        "v_min_i32_e32 %[b3], %[k3], %[b3]\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[tv], %[m0]\n\t"
        "v_cndmask_b32_e64 %[t1], %[t1], %[tv], %[m1]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t2], %[tv], %[m2]\n\t"
        "v_cndmask_b32_e64 %[t3], %[t3], %[tv], %[m3]"
        : [b0] "+v"(bk[c][0]), [b1] "+v"(bk[c][1]), [b2] "+v"(bk[c][2]), [b3] "+v"(bk[c][3]),
          [t0] "+v"(bt[c][0]), [t1] "+v"(bt[c][1]), [t2] "+v"(bt[c][2]), [t3] "+v"(bt[c][3]),
          [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3)
        : [k0] "v"(__float_as_int(acc[0])), [k1] "v"(__float_as_int(acc[1])), [k2] "v"(__float_as_int(acc[2])),
          [k3] "v"(__float_as_int(acc[3])), [tv] "v"(t));
  };
  // software pipeline: tile t's 8 column tiles in pairs (two accumulation chains each), the
  // selection of pair p - 1 behind pair p's MFMAs, tile t + 1's operand (loaded two tiles ahead;
  // with EMB its emb MFMAs) behind the last pair; no branch in the body (loads past the wave's
  // last tile re-read its last tile, never used)
  for (int t = tb; t < te; ++t) {
    f32x4 acc[kTop1CT];
#pragma unroll
    for (int p = 0; p < kTop1CT / 2; ++p) {
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bo[2 * p][s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bo[2 * p + 1][s], a1, 0, 0, 0);
      }
      acc[2 * p] = a0;
      acc[2 * p + 1] = a1;
      if (p > 0) {
        sel(acc[2 * p - 2], 2 * p - 2, t);
        sel(acc[2 * p - 1], 2 * p - 1, t);
      }
    }
    if constexpr (EMB) {
      f32x4 e[2];
      top1_emb_mfma(cv, xn, e);
      opload(min(t + 2, te - 1), xn);
      sel(acc[kTop1CT - 2], kTop1CT - 2, t);
      sel(acc[kTop1CT - 1], kTop1CT - 1, t);
      top1_emb_norm(t + 1, N1, c16, g, e, a);
    } else {
      emb(t + 1, xn, a);
      opload(min(t + 2, te - 1), xn);
      sel(acc[kTop1CT - 2], kTop1CT - 2, t);
      sel(acc[kTop1CT - 1], kTop1CT - 1, t);
    }
  }
  FD_STAMP(2, __builtin_amdgcn_s_memtime());
  // per column tile: the lane's best (value, row) over its 4 row offsets: the smallest key, then
  // the lowest row holding it
  int bv[kTop1CT];
  unsigned br[kTop1CT];
  int vmin = 0x7fffffff;
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c) {
    bv[c] = min(min(bk[c][0], bk[c][1]), min(bk[c][2], bk[c][3]));
    br[c] = 0xffffffffu;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned row = (unsigned)(bt[c][r] * 16 + 4 * g + r);
      br[c] = bk[c][r] == bv[c] ? min(br[c], row) : br[c];
    }
    vmin = min(vmin, bv[c]);
  }
  // a column with a distance at or below torch.cdist's clamp: its first such row (rare)
  if (__builtin_amdgcn_ballot_w64(vmin <= kClampBits)) {
    for (int c = 0; c < kTop1CT; ++c) {
      if (!__builtin_amdgcn_ballot_w64(bv[c] <= kClampBits)) continue;  // (wave-uniform)
      unsigned frow = 0x7fffffffu;
      for (int t = tb; t < te; ++t) {
        float4 xv[2];
        opload(t, xv);
        float at[8];
        emb(t, xv, at);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s], bo[c][s], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (frow == 0x7fffffffu && __float_as_int(acc[r]) <= kClampBits) frow = (unsigned)(t * 16 + 4 * g + r);
      }
      if (frow != 0x7fffffffu) {
        bv[c] = kClampBits;
        br[c] = frow;
      }
    }
  }
  // the 4 lane groups of each column (rows 4 g + r of every tile) by row swaps, then the waves
  // through LDS. Keys (value bits, row) compare as one unsigned 64-bit number: the values are
  // positive here (a clamped column holds the clamp's bits)
  auto xg = [&](int c, bool by32) {
    const auto sv = by32 ? __builtin_amdgcn_permlane32_swap((unsigned)bv[c], (unsigned)bv[c], false, false)
                         : __builtin_amdgcn_permlane16_swap((unsigned)bv[c], (unsigned)bv[c], false, false);
    const auto sr = by32 ? __builtin_amdgcn_permlane32_swap(br[c], br[c], false, false)
                         : __builtin_amdgcn_permlane16_swap(br[c], br[c], false, false);
    const unsigned long long k0 = ((unsigned long long)sv[0] << 32) | sr[0];
    const unsigned long long k1 = ((unsigned long long)sv[1] << 32) | sr[1];
    const unsigned long long kk = k0 < k1 ? k0 : k1;
    bv[c] = (int)(kk >> 32);
    br[c] = (unsigned)kk;
  };
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c) xg(c, false);
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c) xg(c, true);
  if (g == 0) {
#pragma unroll
    for (int c = 0; c < kTop1CT; ++c)
      wkeys[w][c * 16 + c16] = ((unsigned long long)(unsigned)bv[c] << 32) | br[c];
  }
  FD_STAMP(3, __builtin_amdgcn_s_memtime());
  __syncthreads();
  if (tid < kTop1CT * 16) {
    const int jj = tid, j = j0 + jj;
    if (j < N2) {
      unsigned long long bb = wkeys[0][jj];
#pragma unroll
      for (int v = 1; v < kTop1Waves; ++v) bb = wkeys[v][jj] < bb ? wkeys[v][jj] : bb;  // ties: lower wave = lower row
      if (RS == 1) {
        const unsigned row = (unsigned)(bb & 0xffffffffu);
        out_idx[(int64_t)b * V2max + j] = row >= 0x7ffffff0u ? -1 : (int64_t)row;
        if (out_dist) out_dist[(int64_t)b * V2max + j] = sqrtf(__int_as_float((int)(bb >> 32)));
      } else {
        part[((int64_t)b * RS + rs) * V2max + j] = bb;
      }
    }
  }
  FD_STAMP(4, __builtin_amdgcn_s_memtime());
}

// RS > 1: grid (ceil(V2max / 256), B): the smallest of each column's RS row-part keys (value,
// then row: the first index), written as the index and the clamped distance
__global__ __launch_bounds__(256) void fd_top1_merge_kernel(const unsigned long long* __restrict__ part,
                                                            const int32_t* __restrict__ n2, int V2max, int RS,
                                                            int64_t* __restrict__ out_idx, float* __restrict__ out_dist) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n2[b]) return;
  unsigned long long best = ~0ull;
  for (int r = 0; r < RS; ++r) {
    const unsigned long long key = part[((int64_t)b * RS + r) * V2max + j];
    best = key < best ? key : best;
  }
  const unsigned row = (unsigned)(best & 0xffffffffu);
  out_idx[(int64_t)b * V2max + j] = row >= 0x7ffffff0u ? -1 : (int64_t)row;
  if (out_dist) out_dist[(int64_t)b * V2max + j] = sqrtf(__int_as_float((int)(best >> 32)));
}

// ---------------------------------------------------------------------------------------------
// Top-5 fp32 (round 6): the configured solver's candidates, nn_query's dist.sort(dim=-2)[1].T[:, :5]
// (spacial_filtering.py:32-38; config/dpfm_orig.gin:71). Pass 1 is fd_top1_prep_kernel. Pass 2,
// fd_top5_kernel, keeps fd_top1_kernel's layout (block = crop b x 128 columns x row part rs, 8 waves
// splitting the row tiles, the columns' B operands in registers) and its selection cost: on gfx950
// the f32 MFMAs and the VALU issue one after the other (tools/mfma_valu_probe.py: every VALU op
// adds its issue cycles to the MFMA time), so the per-distance work is 4 instructions. Per STREAM =
// (column tile c, row offset r) of a lane — rows 16 t + 4 g + r of its column over the wave's
// tiles — the smallest key with its tile (compare, min, select: the top-1 pass's three) and the
// second smallest key's value (v_med3). The column's five are found among the streams after the
// loop:
//   E0/E1  T = the 5th smallest of the column's 32 lane minima (min over r): 32 distinct rows'
//          distances, so an upper bound of the 5th smallest distance;
//   E2     every stream whose minimum is <= T writes a 16-byte record (row, key, second value,
//          stream) into the column's candidate list in LDS (16 slots, one slot-range reservation
//          per lane and column);
//   E3     four threads per column rank each candidate by (value, row) against the whole list;
//          ranks 0..4 are the five. A kept stream other than the fifth whose second value is <= the
//          fifth value may hold more members: its rows (counted in closed form from the waves'
//          tile ranges) are recomputed exactly (the f32 MFMA accumulates as one fmaf chain over the
//          contraction slots in order, bit for bit: tools/mfma_order_probe.py), one row per thread
//          of the block (a task list in LDS, E3b); the few below the column's fifth key go to a
//          short per-column list that one thread merges (E3c);
//   slow   a column with more than 16 candidates, or a distance at or below torch.cdist's
//          clamp_min(1e-30), is recomputed whole by one wave (clamped; ties to the lower row).
// RS > 1: each row part writes its five to part_v / part_i and fd_merge_kernel<5> merges them.
constexpr int kT5Slots = 16;
constexpr int kT5Tasks = 1536;  // rows recomputed per block (E3b)
constexpr int kT5X = 8;         // recomputed rows below a column's fifth key kept for its merge (E3c)

// the exact distance of row `row` (tile t, in-tile i) and block column jj, as the MFMA chain forms it
__device__ __forceinline__ float t5_exact(const f32x4* __restrict__ Ab, int t, int i, const f32x4 (*sB)[2][64],
                                          int jj) {
  float acc = 0.f;
  const f32x4* At = Ab + (int64_t)t * 128;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q)  // step s = 4 h + q, then the lane groups in order
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        acc = fmaf(At[h * 64 + gg * 16 + i][q], sB[jj >> 4][h][gg * 16 + (jj & 15)][q], acc);
  return acc;
}

// insert key (value bits << 32 | row, unsigned order) into an ascending 5-list
__device__ __forceinline__ void t5_insert(unsigned long long (&best)[5], unsigned long long key) {
  if (!(key < best[4])) return;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const bool sw = key < best[q];
    const unsigned long long tv = sw ? best[q] : key;
    best[q] = sw ? key : best[q];
    key = tv;
  }
}

// any of the four lanes 4c..4c+3 (a column's E3 threads)
__device__ __forceinline__ bool t5_any4(bool v) {
  int x = v ? 1 : 0;
  x |= __shfl_xor(x, 1);
  x |= __shfl_xor(x, 2);
  return x != 0;
}

// the lowest five of this lane's and lane ^ off's ascending 5-lists (unique keys but the ~0
// padding), ascending, with their slots: the elementwise minimum against the partner's reversed
// list is a bitonic sequence holding the lowest five, then a 5-input sorting network
__device__ __forceinline__ void t5_merge_xor(unsigned long long (&bst)[5], int (&bsl)[5], int off) {
  unsigned long long o[5];
  int os[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const unsigned lo = __shfl_xor((unsigned)(bst[q] & 0xffffffffu), off);
    const unsigned hi = __shfl_xor((unsigned)(bst[q] >> 32), off);
    o[q] = ((unsigned long long)hi << 32) | lo;
    os[q] = __shfl_xor(bsl[q], off);
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const bool tk = o[4 - q] < bst[q];
    bst[q] = tk ? o[4 - q] : bst[q];
    bsl[q] = tk ? os[4 - q] : bsl[q];
  }
  auto ce = [&](int x, int y) {
    const bool sw = bst[y] < bst[x];
    const unsigned long long kx = bst[x], ky = bst[y];
    const int sx = bsl[x], sy = bsl[y];
    bst[x] = sw ? ky : kx;
    bst[y] = sw ? kx : ky;
    bsl[x] = sw ? sy : sx;
    bsl[y] = sw ? sx : sy;
  };
  ce(0, 1); ce(3, 4); ce(2, 4); ce(2, 3); ce(0, 3); ce(0, 2); ce(1, 4); ce(1, 3); ce(1, 2);
}

// a candidate record's (value, row) key
__device__ __forceinline__ unsigned long long t5_reckey(const u32x4& r) {
  return ((unsigned long long)r[1] << 32) | r[0];
}

// value-only compare-exchange and the sorted merges of E1
__device__ __forceinline__ void ce_i(int& a, int& b) {
  const int lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}

template <int VAR = 0>
__global__ __launch_bounds__(64 * kTop1Waves, 1) void fd_top5_kernel(
    const f32x4* __restrict__ Atile, int T1, const float* __restrict__ ey, int ldy, const int32_t* __restrict__ n1,
    const int32_t* __restrict__ n2, int V2max, int NCG, int RS, int64_t* __restrict__ out_idx,
    float* __restrict__ out_dist, float* __restrict__ part_v, int32_t* __restrict__ part_i) {
  constexpr int NC = kTop1CT * 16;  // columns per block
  __shared__ f32x4 sB[kTop1CT][2][64];
  __shared__ float sPart[4][NC];
  __shared__ int sLm[NC][4 * kTop1Waves + 1];
  __shared__ int sT[NC];
  __shared__ int sCnt[NC];
  // candidate lists, rows padded by one entry: a wave's 16 columns at one slot spread over the banks
  __shared__ u32x4 sRec[NC][kT5Slots + 1];  // {row, key bits, second key bits, stream}: the key is the
                                            // first 8 bytes read as one unsigned 64-bit (value, row)
  __shared__ int sSlow[NC];
  __shared__ int sNslow, sNtask;
  __shared__ unsigned long long sBest[NC][5];  // E3: each column's five (rank order) and their slots
  __shared__ int sBsl[NC][5];
  __shared__ int sTR[kTop1Waves][2];
  __shared__ int sTask[kT5Tasks];
  __shared__ unsigned long long sFifth[NC];  // each column's fifth key after E3 (~0: fewer than five)
  __shared__ int sXcnt[NC], sXflag[NC];       // recomputed rows below it; the column takes the slow path
  __shared__ unsigned long long sX[NC][kT5X];
  const int per = NCG * RS;
  const int B = (int)(gridDim.x / per);
  int b, k;
  {  // all blocks of crop b on XCD b % 8 when B % 8 == 0 (as fd_top1_kernel)
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
  FD_STAMP(0, __builtin_amdgcn_s_memtime());
  const int j0 = cg * NC;
  const int tid = threadIdx.x, lane = pk::lane_id(), w = __builtin_amdgcn_readfirstlane(pk::wave_id());
  // the column operands' loads go out beside the crop sizes' (as fd_top1_kernel)
  const int sjj = tid & (NC - 1), sgy = tid >> 7;
  const float* syr = ey + ((int64_t)b * V2max + min(j0 + sjj, V2max - 1)) * ldy;
  const float4 sy0 = *reinterpret_cast<const float4*>(syr + 4 * sgy);
  const float4 sy1 = *reinterpret_cast<const float4*>(syr + 16 + 4 * sgy);
  const int N1 = n1[b], N2 = n2[b];
  const int g = lane >> 4, c16 = lane & 15;
  const int nt = (N1 + 15) >> 4;
  const int Q = RS * kTop1Waves;
  const int qw = rs * kTop1Waves + w;
  const int tb = (int)((int64_t)nt * qw / Q), te = (int)((int64_t)nt * (qw + 1) / Q);  // this wave's row tiles
  const f32x4* Ab = Atile + (int64_t)b * T1 * 128;
  auto opload = [&](int t, float4 (&xv)[2]) {
    const f32x4 u0 = Ab[(int64_t)t * 128 + lane], u1 = Ab[(int64_t)t * 128 + 64 + lane];
    xv[0] = make_float4(u0[0], u0[1], u0[2], u0[3]);
    xv[1] = make_float4(u1[0], u1[1], u1[2], u1[3]);
  };
  float4 xc[2], xn[2];
  float a[8];
  if (tb < te) {
    opload(tb, xc);
    opload(min(tb + 1, te - 1), xn);
  }
  float bo[kTop1CT][8];
  {  // staging: the block's 128 columns' [y, 1, |y|^2] in B order, through LDS (as fd_top1_kernel)
    const int jj = sjj, gy = sgy;
    const int j = j0 + jj;
    const bool ok = j < N2;
    float v[8] = {sy0.x, sy0.y, sy0.z, sy0.w, sy1.x, sy1.y, sy1.z, sy1.w};
    float part_ = 0.f;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      v[s8] = (ok && (s8 < 6 || gy < 3)) ? v[s8] : 0.f;
      part_ = fmaf(v[s8], v[s8], part_);
    }
    sPart[gy][jj] = part_;
    if (j0 >= N2) return;  // (block-uniform; after the loads' consumers)
    if (tb < te) {
      a[0] = xc[0].x, a[1] = xc[0].y, a[2] = xc[0].z, a[3] = xc[0].w;
      a[4] = xc[1].x, a[5] = xc[1].y, a[6] = xc[1].z, a[7] = xc[1].w;
    }
    if (tid < NC) sCnt[tid] = 0;
    if (lane == 0) {  // the waves' row-tile ranges (E3's task listing reads them)
      sTR[w][0] = tb;
      sTR[w][1] = te;
    }
    if (tid == 0) {
      sNslow = 0;
      sNtask = 0;
    }
    __syncthreads();
    if (gy == 3) {
      float nrm = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) nrm += sPart[q][jj];
      v[6] = 1.f;
      v[7] = nrm;
    }
    const int c = jj >> 4, l = gy * 16 + (jj & 15);
    sB[c][0][l] = f32x4{v[0], v[1], v[2], v[3]};
    sB[c][1][l] = f32x4{v[4], v[5], v[6], v[7]};
    __syncthreads();
#pragma unroll
    for (int c2 = 0; c2 < kTop1CT; ++c2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 t4 = sB[c2][h][lane];
#pragma unroll
        for (int q = 0; q < 4; ++q) bo[c2][4 * h + q] = t4[q];
      }
  }
  FD_STAMP(1, __builtin_amdgcn_s_memtime());
  int k1[kTop1CT][4], t1[kTop1CT][4], k2[kTop1CT][4];
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      k1[c][r] = 0x7f800000;  // +inf: never replaced by an equal key (padding rows are +inf)
      k2[c][r] = 0x7f800000;
      t1[c][r] = 0x07ffffff;
    }
  // per distance: compare (lane mask), second value = med3(key, min, second), min, select the tile
  auto sel = [&](const f32x4& acc, int c, int t) {
    unsigned long long m0, m1, m2, m3;
    asm("v_cmp_lt_i32_e64 %[m0], %[k0], %[b0]\n\t"
        "v_cmp_lt_i32_e64 %[m1], %[k1], %[b1]\n\t"
        "v_cmp_lt_i32_e64 %[m2], %[k2], %[b2]\n\t"
        "v_cmp_lt_i32_e64 %[m3], %[k3], %[b3]\n\t"
        "v_med3_i32 %[s0], %[k0], %[b0], %[s0]\n\t"
        "v_med3_i32 %[s1], %[k1], %[b1], %[s1]\n\t"
        "v_med3_i32 %[s2], %[k2], %[b2], %[s2]\n\t"
        "v_med3_i32 %[s3], %[k3], %[b3], %[s3]\n\t"
        "v_min_i32_e32 %[b0], %[k0], %[b0]\n\t"
        "v_min_i32_e32 %[b1], %[k1], %[b1]\n\t"
        "v_min_i32_e32 %[b2], %[k2], %[b2]\n\t"
        "v_min_i32_e32 %[b3], %[k3], %[b3]\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[tv], %[m0]\n\t"
        "v_cndmask_b32_e64 %[t1], %[t1], %[tv], %[m1]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t2], %[tv], %[m2]\n\t"
        "v_cndmask_b32_e64 %[t3], %[t3], %[tv], %[m3]"
        : [b0] "+v"(k1[c][0]), [b1] "+v"(k1[c][1]), [b2] "+v"(k1[c][2]), [b3] "+v"(k1[c][3]),
          [s0] "+v"(k2[c][0]), [s1] "+v"(k2[c][1]), [s2] "+v"(k2[c][2]), [s3] "+v"(k2[c][3]),
          [t0] "+v"(t1[c][0]), [t1] "+v"(t1[c][1]), [t2] "+v"(t1[c][2]), [t3] "+v"(t1[c][3]),
          [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3)
        : [k0] "v"(__float_as_int(acc[0])), [k1] "v"(__float_as_int(acc[1])), [k2] "v"(__float_as_int(acc[2])),
          [k3] "v"(__float_as_int(acc[3])), [tv] "v"(t));
  };
  for (int t = tb; t < te; ++t) {  // (the top-1 pass's software pipeline)
    f32x4 acc[kTop1CT];
#pragma unroll
    for (int p = 0; p < kTop1CT / 2; ++p) {
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bo[2 * p][s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bo[2 * p + 1][s], a1, 0, 0, 0);
      }
      acc[2 * p] = a0;
      acc[2 * p + 1] = a1;
      if (p > 0) {
        sel(acc[2 * p - 2], 2 * p - 2, t);
        sel(acc[2 * p - 1], 2 * p - 1, t);
      }
    }
    a[0] = xn[0].x, a[1] = xn[0].y, a[2] = xn[0].z, a[3] = xn[0].w;
    a[4] = xn[1].x, a[5] = xn[1].y, a[6] = xn[1].z, a[7] = xn[1].w;
    opload(min(t + 2, te - 1), xn);
    sel(acc[kTop1CT - 2], kTop1CT - 2, t);
    sel(acc[kTop1CT - 1], kTop1CT - 1, t);
  }
  FD_STAMP(2, __builtin_amdgcn_s_memtime());
  // E0: the lane minima (over r) of every column, per (wave, lane group)
#pragma unroll
  for (int c = 0; c < kTop1CT; ++c)
    sLm[c * 16 + c16][w * 4 + g] = min(min(k1[c][0], k1[c][1]), min(k1[c][2], k1[c][3]));
  __syncthreads();
  {  // E1: T = the 5th smallest of a column's 32 lane minima (4 threads per column, 8 values each)
    const int col = tid >> 2, qq = tid & 3;
    int v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = sLm[col][8 * qq + i];
    // 8-input sorting network (19 compare-exchanges)
    ce_i(v[0], v[1]); ce_i(v[2], v[3]); ce_i(v[4], v[5]); ce_i(v[6], v[7]);
    ce_i(v[0], v[2]); ce_i(v[1], v[3]); ce_i(v[4], v[6]); ce_i(v[5], v[7]);
    ce_i(v[1], v[2]); ce_i(v[5], v[6]); ce_i(v[0], v[4]); ce_i(v[3], v[7]);
    ce_i(v[1], v[5]); ce_i(v[2], v[6]);
    ce_i(v[1], v[4]); ce_i(v[3], v[6]);
    ce_i(v[2], v[4]); ce_i(v[3], v[5]);
    ce_i(v[3], v[4]);
#pragma unroll
    for (int off = 1; off <= 2; off <<= 1) {  // merge with the partner's sorted five: lowest five
      int o[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) o[i] = __shfl_xor(v[i], off);
#pragma unroll
      for (int i = 0; i < 5; ++i) v[i] = min(v[i], o[4 - i]);  // a bitonic sequence holding the lowest five
      // 5-input sorting network (9 compare-exchanges)
      ce_i(v[0], v[1]); ce_i(v[3], v[4]); ce_i(v[2], v[4]); ce_i(v[2], v[3]); ce_i(v[0], v[3]);
      ce_i(v[0], v[2]); ce_i(v[1], v[4]); ce_i(v[1], v[3]); ce_i(v[1], v[2]);
    }
    if (qq == 0) sT[col] = v[4];
  }
  __syncthreads();
  FD_STAMP(3, __builtin_amdgcn_s_memtime());
  // E2: the candidate streams of each column (minimum <= T). One slot-range reservation per
  // (lane, column) for all of its candidate streams, the 8 reservations in flight together
  {
    int base[kTop1CT];
    unsigned cm[kTop1CT];
#pragma unroll
    for (int c = 0; c < kTop1CT; ++c) {
      const int T = sT[c * 16 + c16];
      cm[c] = (k1[c][0] <= T ? 1u : 0u) | (k1[c][1] <= T ? 2u : 0u) | (k1[c][2] <= T ? 4u : 0u) |
              (k1[c][3] <= T ? 8u : 0u);
      base[c] = atomicAdd(&sCnt[c * 16 + c16], __popc(cm[c]));  // (unconditional: no branch per column)
    }
#pragma unroll
    for (int c = 0; c < kTop1CT; ++c) {
      const int col = c * 16 + c16;
      int slot = base[c];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // branch-free: a stream that is not a candidate writes the pad entry
        const bool on = ((cm[c] >> r) & 1u) && slot < kT5Slots;
        const int dst = on ? slot : kT5Slots;
        const unsigned row = (unsigned)(t1[c][r] * 16 + 4 * g + r);
        sRec[col][dst] = u32x4{row, (unsigned)k1[c][r], (unsigned)k2[c][r], (unsigned)((w << 4) | (g << 2) | r)};
        slot += (cm[c] >> r) & 1u;
      }
    }
  }
  __syncthreads();
  FD_STAMP(4, __builtin_amdgcn_s_memtime());
  // E3: four threads per column (tid = 4 col + qd, lanes of one wave) rank the column's candidates
  // qd, qd + 4, ... against all of them; thread qd then lists the recompute rows of kept stream qd
  // (E3b computes them with every thread of the block, one row each, and keeps those below the
  // column's fifth key; E3c: thread 0 of the column merges them — all rows distinct: a stream's
  // rows belong to it alone, and its kept row is not listed).
  unsigned long long best[5];
  int bsl[5];  // candidate slot of each kept entry
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    best[q] = ~0ull;
    bsl[q] = -1;
  }
  const int col = tid >> 2, qd = tid & 3;
  const bool colok = j0 + col < N2;
  int tbase = 0, tcnt = 0;
  const int n = colok ? sCnt[col] : 0;
  bool slow = n > kT5Slots;
  // each candidate's rank among the column's n by (value, row) (keys are unique: distinct rows);
  // ranks 0..4 are the five, written in place (the four threads are lanes of one wave: LDS
  // program order, no barrier)
  if (qd == 0) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      sBest[col][q] = ~0ull;
      sBsl[col][q] = -1;
    }
  }
  if (!slow) {
    unsigned long long kl[kT5Slots];  // the column's list in registers (entries past n: never smaller)
#pragma unroll
    for (int j = 0; j < kT5Slots; ++j) kl[j] = j < n ? t5_reckey(sRec[col][j]) : ~0ull;
    for (int i = qd; i < n; i += 4) {
      const unsigned long long key = t5_reckey(sRec[col][i]);
      const int hi = (int)(key >> 32);
      if (hi <= kClampBits) slow = true;        // a clamped distance: the slow path orders them
      if (hi >= 0x7f800000) continue;           // no row (padding)
      int rank = 0;
#pragma unroll
      for (int j = 0; j < kT5Slots; ++j) rank += kl[j] < key ? 1 : 0;
      if (rank < 5) {
        sBest[col][rank] = key;
        sBsl[col][rank] = i;
      }
    }
  }
  FD_STAMP(13, __builtin_amdgcn_s_memtime());
  slow = t5_any4(slow);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    best[q] = sBest[col][q];
    bsl[q] = sBsl[col][q];
  }
  FD_STAMP(14, __builtin_amdgcn_s_memtime());
  if (qd == 0) {  // (before the listing below: a full task list flags the column after it)
    sFifth[col] = best[4];
    sXcnt[col] = 0;
    sXflag[col] = slow ? 1 : 0;
  }
  if (!slow && colok) {
    // kept stream qd (ranks 0..3) whose second value is <= the fifth value may hold more members:
    // its rows (but the kept one) become recompute tasks. (The fifth value only falls as rows are
    // merged, so the streams listed against the first selection cover every stream that can still
    // hold a member.)
    const int S = best[4] == ~0ull ? 0x7f800000 : (int)(best[4] >> 32);
    const u32x4 rec = bsl[qd] >= 0 ? sRec[col][bsl[qd]] : u32x4{0u, 0u, 0x7fffffffu, 0u};
    if (bsl[qd] >= 0 && (int)rec[2] <= S) {
      const int st = (int)rec[3];
      const int stb = sTR[st >> 4][0];
      const int i = ((st >> 2) & 3) * 4 + (st & 3);
      const int stm = min(sTR[st >> 4][1], (N1 - i + 15) >> 4);  // tiles whose row t 16 + i exists
      const int known = (int)(best[qd] & 0xffffffffu);        // one of them: the kept row
      tcnt = max(0, stm - stb - 1);
      if (tcnt > 0) {
        tbase = atomicAdd(&sNtask, tcnt);
        if (tbase + tcnt > kT5Tasks) {
          sXflag[col] = 1;  // (task list full: the slow path takes the column)
          tcnt = 0;
        } else {
          int k = tbase;
          for (int t = stb; t < stm; ++t)
            if (t * 16 + i != known) sTask[k++] = (t << 11) | (col << 4) | i;
        }
      }
    }
  }
  __syncthreads();
  FD_STAMP(5, __builtin_amdgcn_s_memtime());
  {  // E3b: every listed row's exact distance, one per thread; the few below the column's fifth
     // key go to its short list (any other can never enter the five)
    const int ntask = min(sNtask, kT5Tasks);
    for (int k = tid; k < ntask; k += 64 * kTop1Waves) {
      const int d = sTask[k], t = d >> 11, cc = (d >> 4) & (NC - 1), i = d & 15;
      const float v = t5_exact(Ab, t, i, sB, cc);
      const unsigned long long key = ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)(t * 16 + i);
      if (__float_as_int(v) <= kClampBits) {
        sXflag[cc] = 1;  // a clamped distance: the slow path
      } else if (key < sFifth[cc]) {
        const int slot = atomicAdd(&sXcnt[cc], 1);
        if (slot < kT5X) sX[cc][slot] = key; else sXflag[cc] = 1;
      }
    }
  }
  __syncthreads();
  FD_STAMP(6, __builtin_amdgcn_s_memtime());
  if (qd == 0 && colok) {  // E3c: merge the column's short list
    slow = sXflag[col] != 0;
    if (!slow) {
      const int nx = min(sXcnt[col], kT5X);
      for (int x = 0; x < nx; ++x) t5_insert(best, sX[col][x]);
    }
  }
  FD_STAMP(8, __builtin_amdgcn_s_memtime());
  FD_STAMP(9, __builtin_amdgcn_s_memtime());
  auto emit = [&](int col, const unsigned long long (&bst)[5]) {
    const int j = j0 + col;
    if (RS == 1) {
      const int64_t o = ((int64_t)b * V2max + j) * 5;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const bool none = bst[q] == ~0ull;
        out_idx[o + q] = none ? -1 : (int64_t)(bst[q] & 0xffffffffu);
        if (out_dist) out_dist[o + q] = none ? __builtin_huge_valf() : sqrtf(__uint_as_float((unsigned)(bst[q] >> 32)));
      }
    } else {
      const int64_t o = (((int64_t)b * RS + rs) * V2max + j) * 5;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const bool none = bst[q] == ~0ull;
        part_v[o + q] = none ? __builtin_huge_valf() : __uint_as_float((unsigned)(bst[q] >> 32));
        part_i[o + q] = none ? 0x7fffffff : (int32_t)(bst[q] & 0xffffffffu);
      }
    }
  };
  if (qd == 0 && colok) {
    if (slow) {
      sSlow[atomicAdd(&sNslow, 1)] = col;
    } else {
      emit(col, best);
    }
  }
  __syncthreads();
  // slow path: one wave per column, every row of this row part, clamped distances, lower row first
  const int nslow = sNslow;
  FD_STAMP(10, __builtin_amdgcn_s_memtime());
  FD_STAMP(11, (unsigned long long)nslow);
  FD_STAMP(12, (unsigned long long)sNtask);
  const int pt0 = (int)((int64_t)nt * (rs * kTop1Waves) / Q), pt1 = (int)((int64_t)nt * (rs * kTop1Waves + kTop1Waves) / Q);
  for (int si = w; si < nslow; si += kTop1Waves) {
    const int col = sSlow[si];
    unsigned long long bl[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) bl[q] = ~0ull;
    for (int row = pt0 * 16 + lane; row < min(pt1 * 16, N1); row += 64) {  // rows ascending per lane
      const float d = t5_exact(Ab, row >> 4, row & 15, sB, col);
      const unsigned v = __float_as_int(d) <= kClampBits ? (unsigned)kClampBits : __float_as_uint(d);
      t5_insert(bl, ((unsigned long long)v << 32) | (unsigned)row);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // the wave's lists, merged pairwise (keys are unique)
      unsigned long long o[5];
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const unsigned lo = __shfl_xor((unsigned)(bl[q] & 0xffffffffu), off);
        const unsigned hi = __shfl_xor((unsigned)(bl[q] >> 32), off);
        o[q] = ((unsigned long long)hi << 32) | lo;
      }
#pragma unroll
      for (int q = 0; q < 5; ++q) t5_insert(bl, o[q]);
    }
    if (lane == 0) emit(col, bl);
  }
  FD_STAMP(7, __builtin_amdgcn_s_memtime());
}

struct Top1Plan {
  int T1, T2, NCG, RS;
  int64_t a_bytes, b_bytes, part_bytes;
};

inline int64_t al256_(int64_t x) { return (x + 255) & ~(int64_t)255; }

inline Top1Plan top1_plan(int B, int V1max, int V2max) {
  Top1Plan p{};
  const int T1 = (V1max + 15) / 16, T2 = (V2max + 15) / 16;
  p.NCG = std::max(1, (T2 + kTop1CT - 1) / kTop1CT);
  const int64_t blocks = (int64_t)B * p.NCG;
  // row parts only when the batch leaves the chip short of blocks (each wave keeps >= 2 row tiles)
  const int rs = blocks >= 192 ? 1 : (int)((256 + blocks - 1) / blocks);
  p.RS = std::max(1, std::min(rs, T1 / (2 * kTop1Waves)));
  p.T1 = T1;
  p.T2 = T2;
  p.a_bytes = al256_((int64_t)B * T1 * 2048);
  p.b_bytes = al256_((int64_t)B * T2 * 2048);
  p.part_bytes = p.RS > 1 ? al256_((int64_t)B * p.RS * V2max * 8) : 0;
  return p;
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

}  // namespace

extern "C" int64_t pk_feat_dist_work_size(int B, int V1max, int V2max, int topk, int mode) {
  if (B < 0 || V1max < 0 || V2max < 0 || !(topk == 1 || topk == 5) || mode < 0 || mode > 2) return -1;
  const FdPlan p = fd_plan(B, V1max, V2max, topk, mode);
  const int64_t two_pass = p.a_bytes + p.b_bytes + p.na_bytes + p.nb_bytes + p.pv_bytes + p.pi_bytes;
  if (mode != 0) return two_pass;
  // mode 0: the prep + main pass's operand tiles and row-part keys (top-1) / lists (top-5), or the
  // two-pass fallback's scratch (unaligned operand rows); none keeps anything across calls
  const Top1Plan tp = top1_plan(B, V1max, V2max);
  const int64_t t5parts = tp.RS > 1 ? 2 * al256_((int64_t)B * tp.RS * V2max * 5 * 4) : 0;
  return std::max(two_pass, tp.a_bytes + (topk == 1 ? tp.part_bytes : t5parts));
}

extern "C" int pk_feat_dist_topk(const float* evecs_x, int ldx, const float* C, const float* evecs_y, int ldy,
                                 const int32_t* n1, const int32_t* n2, int B, int V1max, int V2max, int topk,
                                 int mode, void* work, int64_t work_bytes, int64_t* out_idx, float* out_dist,
                                 void* stream) {
  PK_REQUIRE(B >= 0 && V1max >= 0 && V2max >= 0 && ldx >= kF && ldy >= kF && (topk == 1 || topk == 5));
  PK_REQUIRE(mode >= 0 && mode <= 2);
  if (B == 0 || V2max == 0) return PK_OK;
  PK_REQUIRE(evecs_x && C && evecs_y && n1 && n2 && out_idx);
  const int64_t need = pk_feat_dist_work_size(B, V1max, V2max, topk, mode);
  PK_REQUIRE(work_bytes >= need && (work || need == 0));
  hipStream_t s = pk::as_stream(stream);
  const bool aligned = (ldx % 4) == 0 && (ldy % 4) == 0 && (reinterpret_cast<uintptr_t>(evecs_x) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(evecs_y) & 15) == 0;
#ifdef PK_DEVBUILD
  static const bool old_top5 = [] {  // development knob PK_FD_TOP5_OLD=1: the round-3 two-pass top-5
    const char* e = std::getenv("PK_FD_TOP5_OLD");
    return e && std::atoi(e) == 1;
  }();
#else
  constexpr bool old_top5 = false;
#endif
  if (mode == 0 && aligned && V1max > 0 && topk == 5 && !old_top5) {  // prep + main (+ merge when RS > 1)
    const Top1Plan tp = top1_plan(B, V1max, V2max);
    auto* At = static_cast<f32x4*>(work);
    float* pv = tp.RS > 1 ? reinterpret_cast<float*>(static_cast<char*>(work) + tp.a_bytes) : nullptr;
    int32_t* pi = tp.RS > 1 ? reinterpret_cast<int32_t*>(reinterpret_cast<char*>(pv) +
                                                         al256_((int64_t)B * tp.RS * V2max * 5 * 4))
                            : nullptr;
    hipLaunchKernelGGL(fd_top1_prep_kernel, dim3((unsigned)(((tp.T1 + 7) / 8) * B)), dim3(512), 0, s, evecs_x, ldx, C,
                       n1, V1max, tp.T1, At, evecs_y, ldy, n2, V2max, (tp.T1 + 7) / 8);
    PK_CHECK_LAUNCH();
#define PK_FD5(V)                                                                                                \
  hipLaunchKernelGGL((fd_top5_kernel<V>), dim3((unsigned)((int64_t)B * tp.NCG * tp.RS)), dim3(64 * kTop1Waves), 0, s, \
                     At, tp.T1, evecs_y, ldy, n1, n2, V2max, tp.NCG, tp.RS, out_idx, out_dist, pv, pi)
#ifdef PK_DEVBUILD
    static const int t5var = [] {  // development knob PK_FD_VAR=13: phase stamps (tools/fd_stamps.py)
      const char* e = std::getenv("PK_FD_VAR");
      return e ? std::atoi(e) : 0;
    }();
    if (t5var == 13) PK_FD5(13); else PK_FD5(0);
#else
    PK_FD5(0);
#endif
#undef PK_FD5
    PK_CHECK_LAUNCH();
    if (tp.RS > 1) {
      hipLaunchKernelGGL(fd_merge_kernel<5>, dim3((V2max + 255) / 256, B), dim3(256), 0, s, pv, pi, n2, V2max, tp.RS,
                         out_idx, out_dist);
      PK_CHECK_LAUNCH();
    }
    return PK_OK;
  }
  if (mode == 0 && aligned && V1max > 0 && topk == 1) {  // two launches (+ a merge launch when RS > 1)
    const Top1Plan tp = top1_plan(B, V1max, V2max);
    auto* At = static_cast<f32x4*>(work);
    auto* part = reinterpret_cast<unsigned long long*>(static_cast<char*>(work) + tp.a_bytes);
    const dim3 grid((unsigned)((int64_t)B * tp.NCG * tp.RS));
#ifdef PK_DEVBUILD
    static const int tvar = [] {  // development knob PK_FD_VAR: 13 phase stamps, 20 emb in the main pass
      const char* e = std::getenv("PK_FD_VAR");
      return e ? std::atoi(e) : 0;
    }();
#else
    constexpr int tvar = 0;
#endif
    if (tvar != 20) {
      hipLaunchKernelGGL(fd_top1_prep_kernel, dim3((unsigned)(((tp.T1 + 7) / 8) * B)), dim3(512), 0, s, evecs_x, ldx,
                         C, n1, V1max, tp.T1, At, evecs_y, ldy, n2, V2max, (tp.T1 + 7) / 8);
      PK_CHECK_LAUNCH();
    }
#define PK_FDT(V, E)                                                                                              \
  hipLaunchKernelGGL((fd_top1_kernel<V, E>), grid, dim3(64 * kTop1Waves), 0, s, evecs_x, ldx, C, At, tp.T1, evecs_y, \
                     ldy, n1, n2, V1max, V2max, tp.NCG, tp.RS, out_idx, out_dist, part)
#ifdef PK_DEVBUILD
    if (tvar == 13) PK_FDT(13, false); else if (tvar == 20) PK_FDT(0, true); else PK_FDT(0, false);
#else
    PK_FDT(0, false);
#endif
#undef PK_FDT
    PK_CHECK_LAUNCH();
    if (tp.RS > 1) {
      hipLaunchKernelGGL(fd_top1_merge_kernel, dim3((V2max + 255) / 256, B), dim3(256), 0, s, part, n2, V2max, tp.RS,
                         out_idx, out_dist);
      PK_CHECK_LAUNCH();
    }
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
#define PK_FD_MAIN(K, M)                                                                                          \
  hipLaunchKernelGGL((fd_main_direct_kernel<K, M>), grid, block, 0, s, A, Bq, nA, nB, n1, n2, p.T1, p.T2, V2max,  \
                     p.NCG, p.RS, out_idx, out_dist, pv, pi)
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

#ifdef PK_DEVBUILD
// development: the VAR 13 phase stamps of the last fd_top1_kernel launch (8 per block)
extern "C" int pkdev_fd_stamps(unsigned long long* host, int n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fd_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif
