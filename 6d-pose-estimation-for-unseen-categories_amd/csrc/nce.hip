// H15 NCE term of the DPFM loss, fused forward + gradients.
//
// Reference: utils/loss.py:17-40 NCESoftmaxLoss.forward, per crop:
//   q = normalize(f1)[map21[sel, 0]], k = normalize(f2)[map21[sel, 1]]      (S <= 512 pairs)
//   logits = -cdist(q, k) / nce_t;  loss = cross_entropy(logits, arange(S))
// torch.cdist at these sizes takes its matmul path (torch _euclidean_dist):
//   d = sqrt(max(|q|^2 + |k|^2 - 2 q.k, 0)),  d(d)/dq = (q - k) / d (0 where d == 0).
// The batched torch version (dpfm_amd/utils/loss.py, before this kernel) ran ~25 kernels
// forward and ~35 backward per step (normalize, gathers, cdist, masked log-softmax,
// diagonal, their backwards, scatter-adds); here it is three launches:
//   zero(g1, g2) -> row pass -> column pass.
// Each pass is two f32 MFMA contractions (v_mfma_f32_16x16x4f32: exact f32, an fmaf chain
// over the 32 channels in order, so both passes see bit-identical distances), two waves per
// 16 own rows, each over one half of the partners (8 waves per block = 4 row groups x 2 halves,
// two waves per SIMD so one's MFMAs run under the other's exp / sqrt; grid S/64 x B), the other
// side's S <= 512 normalized vectors staged once per block in LDS:
//   G^T[256 x 16] = O[half x 32] . V^T[32 x 16]: lane (row r = lane % 16, group g = lane / 16)
//     holds its row's distances to partners 16 t + 4 g + v (t in the half's 16 tiles, v < 4) in
//     64 VGPRs;
//   row pass: max / sum over a row = in-lane over 64, then xor 16, 32, then the two halves
//     through LDS (min exactly; sums half 0 + half 1) -> lse[a],
//     term[a] = lse[a] - logit[a][a];  column pass: the softmax rows' lse from the row pass;
//   r[a][o] = dL/dd = -(softmax - [o == a]) / (n_valid t d)  (0 where d == 0 or invalid),
//     written over the distances (the A operand of the next product, same register layout);
//   dQ[16 x 32] = R[16 x 512] . O[512 x 32]  (k-slot g of step (t, v) = partner 16 t + 4 g + v;
//     per half, half 1's partial added to half 0's through LDS);
//   dq_a = q_a sum_o r - (R O)_a  (torch's _euclidean_dist_backward), then F.normalize's
//   backward, written as slot a's gradient row dx[a] (scratch [B, S, 32]).
// A CAD / crop point can sit in several pairs (torch's gather backward scatter_adds them); a
// third launch (nce_scatter_kernel, one block per crop and side) zero-fills g and adds each
// point's slot rows in ascending slot order: the gradients are deterministic (the float
// atomics of round 2 made the graphed and eager steps differ in the last bits).
// Column pass: the same per key column o -> g2;  block (0, b) also writes
//   loss[b] = sum_a term[a] / max(n_valid, 1) in a fixed order (deterministic).
// prenorm: f1 / f2 are already F.normalize'd (the overlap head's l2-normalize writes a rows
// copy for this term): no normalization here, and g1 / g2 are the gradients with respect to
// those normalized features (the l2-normalize backward then takes both heads' gradients);
// such rows are staged with 16-B loads, 8 lanes per row.
// Rows past a crop's pair count (valid == 0) contribute nothing; a crop without pairs has
// loss 0 (the batched host code's clamp(min=1) convention; the reference would give NaN).
#include <cstdint>

#include "common.hpp"

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));

constexpr int kC = 32;           // feature width (n_feat, config/dpfm_orig.yaml)
constexpr int kMaxS = 512;       // nce_num_pairs (config/dpfm_orig.gin:58)
constexpr int kPT = kMaxS / 16;  // partner tiles of 16
constexpr int kRowsPerWave = 16;
constexpr int kGroups = 4;  // row groups of 16 per block
constexpr int kHalves = 2;  // partner halves: wave (group, half) takes partners [256 half, 256 half + 256)
constexpr int kWaves = kGroups * kHalves;  // one block per CU (LDS), two waves per SIMD
constexpr int kTile = kRowsPerWave * kGroups;  // rows per block
constexpr int kHT = kPT / kHalves;  // partner tiles per wave
constexpr int kLd = kC + 2;  // LDS row stride: the G operand reads (row r, channel 4 s + g) hit distinct banks

struct FeatView {  // f[b, n, c] = base[b * sb + n * sn + c * sc] (rows or channels-first storage)
  const float* base;
  int64_t sb, sn, sc;
};

__device__ __forceinline__ const float* nce_row_ptr(const FeatView& f, const int64_t* __restrict__ pairs, int cap,
                                                    const int64_t* __restrict__ rows, int S, int b, int slot,
                                                    int side, int64_t* idx_out) {
  const int64_t r = rows[(int64_t)b * S + slot];
  const int64_t idx = pairs[((int64_t)b * cap + r) * 2 + side];
  *idx_out = idx;
  return f.base + (int64_t)b * f.sb + idx * f.sn;
}

// one feature row into dst[0..31]: x / max(||x||, 1e-12) (F.normalize, sequential fmaf norm),
// or as is under prenorm; returns the pre-normalization norm (1 under prenorm)
__device__ __forceinline__ float stage_row(const float* p, int64_t sc, bool ok, int prenorm, float* dst,
                                           const float* safe) {
  float x[kC];
  float ss = 0.f;
  const float* q = ok ? p : safe;  // unconditional loads at a valid address (no branch + wait per load)
#pragma unroll
  for (int c = 0; c < kC; ++c) {
    const float v = q[c * sc];
    x[c] = ok ? v : 0.f;
  }
#pragma unroll
  for (int c = 0; c < kC; ++c) ss = fmaf(x[c], x[c], ss);
  const float nrm = prenorm ? 1.f : sqrtf(ss);
  const float nc = fmaxf(nrm, 1e-12f);
#pragma unroll
  for (int c = 0; c < kC; ++c) dst[c] = ok ? (prenorm ? x[c] : x[c] / nc) : 0.f;
  return nrm;
}

template <bool COLS>
__global__ __launch_bounds__(64 * kWaves) void nce_pass_kernel(
    const FeatView f1, const FeatView f2, int64_t N1, int64_t N2,
    const int64_t* __restrict__ pairs, int cap, const int64_t* __restrict__ rows,
    const uint8_t* __restrict__ valid, int S, float inv_t, int prenorm, float* __restrict__ lse,
    float* __restrict__ term, float* __restrict__ loss, float* __restrict__ dx_own) {
  __shared__ __attribute__((aligned(16))) float Os[kMaxS * kLd];  // the other side's normalized vectors
  __shared__ __attribute__((aligned(16))) float on_s[kMaxS];      // their |u|^2 (+inf: invalid slot)
  __shared__ __attribute__((aligned(16))) float lse_s[kMaxS];     // COLS: the softmax rows' lse
  __shared__ float Ws[kTile * kLd];  // this block's own rows, normalized
  __shared__ float wn_s[kTile];      // their norms (-1: invalid row)
  __shared__ float vn_s[kTile];      // their |v|^2
  __shared__ int64_t widx_s[kTile];  // their feature indices
  __shared__ int64_t ooff_s[kMaxS];  // the other side's row offsets (-1: invalid slot)
  __shared__ int nv_s[kWaves];
  __shared__ float xst_s[2][kGroups][kHalves][16];       // the row statistics of each half (min d, sum)
  __shared__ float xacc_s[kGroups][9][64];               // half 1's (R O) partial and row sums
  const int b = blockIdx.y;
  const int lane = pk::lane_id(), w = pk::wave_id();
  const uint8_t* __restrict__ vb = valid + (int64_t)b * S;
  // own side: rows pass = queries (f1, pairs[..,0]); column pass = keys (f2, pairs[..,1])
  const FeatView f_own = COLS ? f2 : f1;
  const FeatView f_oth = COLS ? f1 : f2;
  const int64_t N_own = COLS ? N2 : N1;
  const int side_own = COLS ? 1 : 0;

  // Staging in three round trips instead of one dependent chain per row: (1) every slot's
  // valid flag / row / pair index, all loads unconditional at clamped addresses (an invalid slot's
  // row may hold anything) and the own rows' features alongside; (2) every other-side feature
  // row, all of a thread's loads in flight together (the round-4 loop waited for each row's
  // three dependent loads in turn: 16 serial chains per thread, most of the pass).
  constexpr int kOPer = kMaxS / (64 * kWaves);  // other-side slots per thread
  int nv = 0;
  {
    int64_t rr[kOPer];
    bool okv[kOPer];
#pragma unroll
    for (int i = 0; i < kOPer; ++i) {
      const int o = threadIdx.x + i * 64 * kWaves;
      const int oc = o < S ? o : S - 1;
      okv[i] = o < S && vb[oc] != 0;
      rr[i] = rows[(int64_t)b * S + oc];
    }
#pragma unroll
    for (int i = 0; i < kOPer; ++i) {
      const int64_t r = rr[i] < 0 ? 0 : rr[i] >= cap ? cap - 1 : rr[i];
      rr[i] = pairs[((int64_t)b * cap + r) * 2 + (1 - side_own)];
    }
#pragma unroll
    for (int i = 0; i < kOPer; ++i) {
      const int o = threadIdx.x + i * 64 * kWaves;
      ooff_s[o] = okv[i] ? (int64_t)b * f_oth.sb + rr[i] * f_oth.sn : -1;
      nv += okv[i] ? 1 : 0;
    }
  }
  nv = pk::wave_sum_i32(nv);
  if (lane == 0) nv_s[w] = nv;
  // this block's own rows (their dependent index / feature loads overlap the loads above)
  if (threadIdx.x < kTile) {
    const int a = blockIdx.x * kTile + threadIdx.x;
    const int ac = a < S ? a : S - 1;
    const bool ok = a < S && vb[ac] != 0;
    int64_t r = rows[(int64_t)b * S + ac];
    r = r < 0 ? 0 : r >= cap ? cap - 1 : r;
    const int64_t idx = ok ? pairs[((int64_t)b * cap + r) * 2 + side_own] : 0;
    const float* p = f_own.base + (int64_t)b * f_own.sb + idx * f_own.sn;
    float* dst = &Ws[threadIdx.x * kLd];
    const float nrm = stage_row(ok ? p : nullptr, f_own.sc, ok, prenorm, dst, f_own.base);
    float vn = 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) vn = fmaf(dst[c], dst[c], vn);
    wn_s[threadIdx.x] = ok ? nrm : -1.f;
    vn_s[threadIdx.x] = vn;
    widx_s[threadIdx.x] = idx;
  }
  __syncthreads();
  // the other side (slots >= S and invalid slots: zeros)
  const bool vec = prenorm && f_oth.sc == 1 && (((uintptr_t)f_oth.base) & 15) == 0 && (f_oth.sn & 3) == 0 &&
                   (f_oth.sb & 3) == 0;
  if (vec) {  // normalized rows storage: 8 lanes per row, 16 B each, kMaxS * 8 / 256 = 16 loads per thread
    constexpr int kVPer = kMaxS * 8 / (64 * kWaves);
    float4 x[kVPer];
#pragma unroll
    for (int i = 0; i < kVPer; ++i) {
      const int e = threadIdx.x + i * 64 * kWaves;
      const int64_t off = ooff_s[e >> 3];
      x[i] = *reinterpret_cast<const float4*>(f_oth.base + (off < 0 ? 0 : off) + 4 * (e & 7));
      if (off < 0) x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < kVPer; ++i) {
      const int e = threadIdx.x + i * 64 * kWaves;
      float2* d2 = reinterpret_cast<float2*>(&Os[(e >> 3) * kLd + 4 * (e & 7)]);  // 8-B aligned (kLd even)
      d2[0] = make_float2(x[i].x, x[i].y);
      d2[1] = make_float2(x[i].z, x[i].w);
    }
  } else {
    for (int o = threadIdx.x; o < kMaxS; o += 64 * kWaves) {
      const int64_t off = ooff_s[o];
      stage_row(off >= 0 ? f_oth.base + off : nullptr, f_oth.sc, off >= 0, prenorm, &Os[o * kLd], f_oth.base);
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < kMaxS; o += 64 * kWaves) {  // |u|^2: the same fmaf chain in both passes
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) s = fmaf(Os[o * kLd + c], Os[o * kLd + c], s);
    on_s[o] = (o < S && vb[o] != 0) ? s : __builtin_huge_valf();
    if (COLS) lse_s[o] = o < S ? lse[(int64_t)b * S + o] : 0.f;
  }
  __syncthreads();
  nv = 0;
#pragma unroll
  for (int q = 0; q < kWaves; ++q) nv += nv_s[q];
  const float sc = 1.f / (float)(nv > 0 ? nv : 1);

  if (COLS && blockIdx.x == 0 && w == 0) {  // loss[b], fixed summation order
    float t = 0.f;
    for (int a = lane; a < S; a += pk::kWave) t += term[(int64_t)b * S + a];
    t = pk::wave_sum_f32(t);
    if (lane == 0) loss[b] = t * sc;
  }
  if (COLS && dx_own == nullptr) return;  // block-uniform
  // wave (row group rg, partner half hf); every wave runs to the end (the halves meet at
  // barriers): a row group past S computes on its zero rows (ok = false) and stores nothing
  const int rg = w % kGroups, hf = w / kGroups;
  const int a0 = blockIdx.x * kTile + rg * kRowsPerWave;
  const int r = lane & 15, g = lane >> 4;
  const int tr = rg * kRowsPerWave + r;  // the lane's row within the staged tile
  const int a = a0 + r;
  const bool ok = a < S && wn_s[tr] >= 0.f;
  const float vn = vn_s[tr];
  const int t0 = hf * kHT;

  // d[t][v]: distance to partner 16 (t0 + t) + 4 g + v (-1: no logit there)
  float bv[kC / 4];
#pragma unroll
  for (int s = 0; s < kC / 4; ++s) bv[s] = Ws[tr * kLd + 4 * s + g];
  float d[kHT][4];
#pragma unroll
  for (int t = 0; t < kHT; ++t) {
    fx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kC / 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Os[(16 * (t0 + t) + r) * kLd + 4 * s + g], bv[s], acc, 0, 0, 0);
    const float4 on = *reinterpret_cast<const float4*>(&on_s[16 * (t0 + t) + 4 * g]);
    const float onv[4] = {on.x, on.y, on.z, on.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float d2 = fmaxf((vn + onv[v]) - 2.f * acc[v], 0.f);
      d[t][v] = ok && onv[v] < __builtin_huge_valf() ? __builtin_amdgcn_sqrtf(d2) : -1.f;  // v_sqrt_f32 (1 ulp)
    }
  }
  // row pass: the row's softmax statistics over both halves (exchanged through LDS: the min
  // exactly, the sums as half 0 + half 1); max logit = -(min d) / t exactly (monotone rounding)
  float mx = 0.f, is = 0.f, lse_a = 0.f;
  if (!COLS) {
    float dm = __builtin_huge_valf();
#pragma unroll
    for (int t = 0; t < kHT; ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (d[t][v] >= 0.f) dm = fminf(dm, d[t][v]);
    dm = fminf(dm, __shfl_xor(dm, 16));
    dm = fminf(dm, __shfl_xor(dm, 32));
    if (g == 0) xst_s[0][rg][hf][r] = dm;
    __syncthreads();
    dm = fminf(xst_s[0][rg][0][r], xst_s[0][rg][1][r]);
    mx = ok ? -dm * inv_t : 0.f;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < kHT; ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v) s += d[t][v] >= 0.f ? __expf(-d[t][v] * inv_t - mx) : 0.f;
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0) xst_s[1][rg][hf][r] = s;
    __syncthreads();
    s = xst_s[1][rg][0][r] + xst_s[1][rg][1][r];
    is = __builtin_amdgcn_rcpf(s);
    lse_a = mx + __logf(s);
  }
  // r = dL/dd over the distances; the row pass also picks the diagonal logit (in half a / 256)
  const float k_r = -sc * inv_t;
  float rs = 0.f, ldg = 0.f;
#pragma unroll
  for (int t = 0; t < kHT; ++t) {
    float lo[4] = {0.f, 0.f, 0.f, 0.f};
    if (COLS) {
      const float4 l4 = *reinterpret_cast<const float4*>(&lse_s[16 * (t0 + t) + 4 * g]);
      lo[0] = l4.x; lo[1] = l4.y; lo[2] = l4.z; lo[3] = l4.w;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float dd = d[t][v];
      const float lg = -dd * inv_t;
      const bool diag = 16 * (t0 + t) + 4 * g + v == a;
      const float p = dd >= 0.f ? (COLS ? __expf(lg - lo[v]) : __expf(lg - mx) * is) : 0.f;
      if (!COLS && diag) ldg = lg;
      const float gg = p - (diag ? 1.f : 0.f);
      const float rr = dd > 0.f ? gg * k_r * __builtin_amdgcn_rcpf(dd) : 0.f;  // implies ok, partner valid
      rs += rr;
      d[t][v] = rr;
    }
  }
  rs += __shfl_xor(rs, 16);
  rs += __shfl_xor(rs, 32);
  if (!COLS) {
    ldg += __shfl_xor(ldg, 16);  // one group holds it, the others add zeros
    ldg += __shfl_xor(ldg, 32);
    if (hf == ((a0 / (16 * kHT)) & 1) && g == 0 && a < S) {  // the half holding the row's diagonal
      lse[(int64_t)b * S + a] = ok ? lse_a : 0.f;
      term[(int64_t)b * S + a] = ok ? lse_a - ldg : 0.f;
    }
    if (dx_own == nullptr) return;  // block-uniform
  }
  // (R O)[row 4 g + v][channel 16 h + r] over this half's partners
  fx4 acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int t = 0; t < kHT; ++t)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float* orow = &Os[(16 * (t0 + t) + 4 * g + v) * kLd + r];
#pragma unroll
      for (int h = 0; h < 2; ++h) acc2[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(d[t][v], orow[16 * h], acc2[h], 0, 0, 0);
    }
  // half 1 hands its partial product and row sums to half 0 (added as half 0 + half 1)
  if (hf == 1) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int v = 0; v < 4; ++v) xacc_s[rg][4 * h + v][lane] = acc2[h][v];
    xacc_s[rg][8][lane] = rs;
  }
  __syncthreads();
  if (hf == 1) return;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc2[h][v] += xacc_s[rg][4 * h + v][lane];
  rs += xacc_s[rg][8][lane];
  // dq, then F.normalize backward: (dv - v (v . dv)) / n  (dv / 1e-12 when clamped)
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int rw = 4 * g + v;               // row of this accumulator slot
    const float rs_w = __shfl(rs, rw);      // lane rw holds row rw's sum (group 0)
    const int trw = rg * kRowsPerWave + rw;
    const bool okw = a0 + rw < S && wn_s[trw] >= 0.f;
    const float nw = wn_s[trw];
    float vc[2], dv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      vc[h] = Ws[trw * kLd + 16 * h + r];
      dv[h] = vc[h] * rs_w - acc2[h][v];
    }
    float vdv = vc[0] * dv[0] + vc[1] * dv[1];
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) vdv += __shfl_xor(vdv, off);  // the row's 16 lanes
    if (!okw) continue;
    const int64_t base = ((int64_t)b * S + a0 + rw) * kC + r;  // slot row (the scatter sums them)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float dx = prenorm ? dv[h] : nw > 1e-12f ? (dv[h] - vc[h] * vdv) / nw : dv[h] / 1e-12f;
      dx_own[base + 16 * h] = dx;
    }
  }
}

// g[b, idx] = sum of the slot rows dx[b, a] with idx(a) = idx, in ascending slot order (0 for
// points in no valid slot). Blocks (crop, side, part): each 512-thread block sorts the (idx, slot)
// keys of the crop's slots in LDS (bitonic, 512 keys; every part repeats it), so every point's
// slots form one ascending run, and owns the points [part N / kScP, (part + 1) N / kScP): it zero-fills
// their rows and, for the sorted positions whose point it owns (one contiguous range), work item
// (sorted position, channel) at a run's head sums the run (128-B coalesced rows). Round 4 ran one
// block per (crop, side): 64 blocks on 256 CUs, every block's loads and stores in series.
constexpr int kScT = 512;
constexpr int kScP = 4;
__global__ __launch_bounds__(kScT) void nce_scatter_kernel(const int64_t* __restrict__ pairs, int cap,
                                                           const int64_t* __restrict__ rows,
                                                           const uint8_t* __restrict__ valid, int S, int64_t N1,
                                                           int64_t N2, const float* __restrict__ dxr,
                                                           float* __restrict__ g1, float* __restrict__ g2) {
  __shared__ int64_t key[kMaxS];
  const int b = blockIdx.x, side = blockIdx.y, B = gridDim.x;
  const int t = threadIdx.x;
  const int64_t N = side ? N2 : N1;
  const int64_t per = (N + kScP - 1) / kScP;
  const int64_t lo = blockIdx.z * per, hi = lo + per < N ? lo + per : N;
  float* __restrict__ g = (side ? g2 : g1) + (int64_t)b * N * kC;
  const float* __restrict__ dx = dxr + ((int64_t)side * B + b) * S * kC;
  constexpr int64_t kNone = 0x7fffffffffffffffLL;
  static_assert(kScT == kMaxS, "one key per thread");
  int64_t kk = kNone;
  if (t < S && valid[(int64_t)b * S + t] != 0) {
    const int64_t r = rows[(int64_t)b * S + t];
    kk = (pairs[((int64_t)b * cap + r) * 2 + side] << 9) | t;
  }
  float4* gz = reinterpret_cast<float4*>(g);  // N * 32 floats, 16-B aligned (torch allocation, N * 128 B rows)
  for (int64_t e = lo * (kC / 4) + t; e < hi * (kC / 4); e += kScT) gz[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  // bitonic sort, one key per thread: partners within a wave (j < 64) by lane shuffles, only the
  // 6 wider stages through LDS (12 barriers instead of 45)
  for (int k = 2; k <= kMaxS; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      int64_t other;
      if (j >= 64) {
        key[t] = kk;
        __syncthreads();
        other = key[t ^ j];
        __syncthreads();
      } else {
        const uint32_t klo = (uint32_t)(uint64_t)kk, khi = (uint32_t)((uint64_t)kk >> 32);
        const uint32_t olo = (uint32_t)__shfl_xor((int)klo, j), ohi = (uint32_t)__shfl_xor((int)khi, j);
        other = (int64_t)(((uint64_t)ohi << 32) | olo);
      }
      const bool up = (t & k) == 0, lower = (t & j) == 0;
      kk = (lower == up) ? (kk < other ? kk : other) : (kk > other ? kk : other);
    }
  key[t] = kk;
  // the sorted positions of this part's points: [p0, p1) (sentinels sort last, above every point)
  const int p0 = __syncthreads_count((kk >> 9) < lo);
  const int p1 = __syncthreads_count((kk >> 9) < hi);
  // every owned position's first row value is loaded up front (all in flight together; a run's
  // further rows — points in several slots, rare — are added after)
  const int c = t & (kC - 1);
  constexpr int kStep = kScT / kC;  // positions per pass of the block
  constexpr int kPer = kMaxS / kStep;
  float v[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int p = p0 + t / kC + kStep * i;
    const int64_t k = key[p < p1 ? p : p0];
    v[i] = dx[(p < p1 ? (k & 511) : 0) * kC + c];  // slot 0's row stands in past the range
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int p = p0 + t / kC + kStep * i;
    if (p >= p1) break;
    const int64_t k = key[p];
    const int64_t idx = k >> 9;
    if (p > 0 && (key[p - 1] >> 9) == idx) continue;  // not the head of its run
    float s = v[i];
    for (int q = p + 1; q < kMaxS; ++q) {  // the run's further slots, ascending
      const int64_t kq = key[q];
      if (kq == kNone || (kq >> 9) != idx) break;
      s += dx[(kq & 511) * kC + c];
    }
    g[idx * kC + c] = s;
  }
}

}  // namespace

extern "C" int pk_nce_loss(const float* f1, const int64_t* st1, const float* f2, const int64_t* st2, int B,
                           int64_t N1, int64_t N2, int C,
                           const int64_t* pairs, int cap, const int64_t* rows, const uint8_t* valid, int S,
                           float nce_t, int prenorm, float* lse, float* term, float* loss, float* g1, float* g2,
                           float* dx_rows, void* stream) {
  PK_REQUIRE(B >= 0 && C == kC && S >= 0 && S <= kMaxS && cap >= 0 && nce_t > 0.f);
  PK_REQUIRE((g1 == nullptr) == (g2 == nullptr));
  PK_REQUIRE(g1 == nullptr || dx_rows != nullptr);
  if (B == 0) return PK_OK;
  PK_REQUIRE(loss != nullptr);
  hipStream_t s = pk::as_stream(stream);
  if (S == 0) {
    hipError_t e = pk::zero_async(loss, sizeof(float) * B, s);
    if (g1 && e == hipSuccess) e = pk::zero_async(g1, sizeof(float) * (size_t)B * N1 * kC, s);
    if (g1 && e == hipSuccess) e = pk::zero_async(g2, sizeof(float) * (size_t)B * N2 * kC, s);
    return e == hipSuccess ? PK_OK : (int)e;
  }
  PK_REQUIRE(f1 && f2 && pairs && rows && valid && lse && term && cap > 0);
  const float inv_t = 1.f / nce_t;
  const dim3 grid((S + kTile - 1) / kTile, B);
  const FeatView v1{f1, st1 ? st1[0] : N1 * kC, st1 ? st1[1] : kC, st1 ? st1[2] : 1};
  const FeatView v2{f2, st2 ? st2[0] : N2 * kC, st2 ? st2[1] : kC, st2 ? st2[2] : 1};
  hipLaunchKernelGGL(nce_pass_kernel<false>, grid, dim3(64 * kWaves), 0, s, v1, v2, N1, N2, pairs, cap, rows, valid,
                     S, inv_t, prenorm, lse, term, loss, g1 ? dx_rows : nullptr);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(nce_pass_kernel<true>, grid, dim3(64 * kWaves), 0, s, v1, v2, N1, N2, pairs, cap, rows, valid,
                     S, inv_t, prenorm, lse, term, loss, g2 ? dx_rows + (size_t)B * S * kC : nullptr);
  PK_CHECK_LAUNCH();
  if (g1) {
    hipLaunchKernelGGL(nce_scatter_kernel, dim3(B, 2, kScP), dim3(kScT), 0, s, pairs, cap, rows, valid, S, N1, N2, dx_rows,
                       g1, g2);
    PK_CHECK_LAUNCH();
  }
  return PK_OK;
}
