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
// Row pass, one wave per 16 query rows a, taken 4 at a time (4 waves per block; grid S/64 x B):
//   logits of row a against all S keys (8 columns per lane, keys normalized once per block
//   into LDS), wave max / sum -> lse[a], term[a] = lse[a] - logit[a][a];
//   dlogit[a][o] = (softmax - [o == a]) / n_valid;  r = -dlogit / (t d);
//   dq_a = q_a sum_o r - sum_o r k_o  (torch's _euclidean_dist_backward), then through
//   F.normalize's backward, added into g1[b, idx1(a)] (global f32 atomics: a CAD point can
//   sit in several pairs, as torch's gather-backward scatter_add).
// Column pass: the same per key column o, with the softmax rows' lse from the row pass:
//   dk_o = k_o sum_a r - sum_a r q_a  -> g2[b, idx2(o)];  block (0, b) also writes
//   loss[b] = sum_a term[a] / max(n_valid, 1) in a fixed order (deterministic).
// prenorm: f1 / f2 are already F.normalize'd (the overlap head's l2-normalize writes a rows
// copy for this term): no normalization here, and g1 / g2 are the gradients with respect to
// those normalized features (the l2-normalize backward then takes both heads' gradients).
// Rows past a crop's pair count (valid == 0) contribute nothing; a crop without pairs has
// loss 0 (the batched host code's clamp(min=1) convention; the reference would give NaN).
#include "common.hpp"

namespace {

typedef float fx2 __attribute__((ext_vector_type(2)));  // v_pk_fma_f32 operands

constexpr int kC = 32;         // feature width (n_feat, config/dpfm_orig.yaml)
constexpr int kMaxS = 512;     // nce_num_pairs (config/dpfm_orig.gin:58)
constexpr int kPerLane = kMaxS / pk::kWave;
constexpr int kRowsPerWave = 16;
constexpr int kGroup = 4;     // rows evaluated together (partner reads amortized over them)
constexpr int kWaves = 4;     // one wave per SIMD (LDS holds one block per CU): 256 VGPRs + AGPRs each
constexpr int kTile = kRowsPerWave * kWaves;  // rows per block
constexpr int kLdO = kC + 1;                  // odd LDS row stride: lanes read rows o = lane + 64 j
constexpr int kLdW = kC + 4;                  // own rows: 16-B aligned (broadcast ds_read_b128)

// normalized feature row of pair slot `slot` (side 0: f1 via pairs[.., 0]; side 1: f2 via
// pairs[.., 1]) and its pre-normalization norm
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

template <bool COLS>
__global__ __launch_bounds__(64 * kWaves) void nce_pass_kernel(
    const FeatView f1, const FeatView f2, int64_t N1, int64_t N2,
    const int64_t* __restrict__ pairs, int cap, const int64_t* __restrict__ rows,
    const uint8_t* __restrict__ valid, int S, float inv_t, int prenorm, float* __restrict__ lse,
    float* __restrict__ term, float* __restrict__ loss, float* __restrict__ g_own) {
  __shared__ float Os[kMaxS * kLdO];  // the other side's normalized vectors
  __shared__ float lse_s[kMaxS];      // COLS: softmax rows' lse
  __shared__ float4 rbuf[kWaves][kMaxS];  // per wave: r of its kGroup rows, [partner][row]
  __shared__ int nv_s[kWaves];
  __shared__ __attribute__((aligned(16))) float Ws[kTile * kLdW];  // this block's own rows, normalized
  __shared__ float wn_s[kTile];                                     // their norms (0: invalid row)
  __shared__ int64_t widx_s[kTile];                                 // their feature indices
  const int b = blockIdx.y;
  const int lane = pk::lane_id(), w = pk::wave_id();
  const uint8_t* __restrict__ vb = valid + (int64_t)b * S;
  // own side: rows pass = queries (f1, pairs[..,0]); column pass = keys (f2, pairs[..,1])
  const FeatView f_own = COLS ? f2 : f1;
  const FeatView f_oth = COLS ? f1 : f2;
  const int64_t N_own = COLS ? N2 : N1, N_oth = COLS ? N1 : N2;
  const int side_own = COLS ? 1 : 0;

  // number of valid slots (identical in every block of the crop)
  int nv = 0;
  for (int o = threadIdx.x; o < S; o += 64 * kWaves) nv += vb[o] ? 1 : 0;
  nv = pk::wave_sum_i32(nv);
  if (lane == 0) nv_s[w] = nv;
  // stage the other side, normalized as F.normalize: x / max(||x||, 1e-12), with the same
  // sequential fmaf norm as the own side below (both passes then see identical vectors)
  for (int o = threadIdx.x; o < kMaxS; o += 64 * kWaves) {  // rows >= S: zeros
    float x[kC];
    float ss = 0.f;
    const bool ok = o < S && vb[o] != 0;
    int64_t idx = 0;
    const float* p = ok ? nce_row_ptr(f_oth, pairs, cap, rows, S, b, o, 1 - side_own, &idx) : nullptr;
#pragma unroll
    for (int c = 0; c < kC; ++c) x[c] = ok ? p[c * f_oth.sc] : 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) ss = fmaf(x[c], x[c], ss);
    const float nc = prenorm ? 1.f : fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
    for (int c = 0; c < kC; ++c) Os[o * kLdO + c] = ok ? (prenorm ? x[c] : x[c] / nc) : 0.f;
    if (COLS) lse_s[o] = o < S ? lse[(int64_t)b * S + o] : 0.f;
  }
  // stage this block's own rows (all their dependent index / feature loads in parallel)
  if (threadIdx.x < kTile) {
    const int a = blockIdx.x * kTile + threadIdx.x;
    const bool ok = a < S && vb[a] != 0;
    int64_t idx = 0;
    float x[kC];
    const float* p = ok ? nce_row_ptr(f_own, pairs, cap, rows, S, b, a, side_own, &idx) : nullptr;
#pragma unroll
    for (int c = 0; c < kC; ++c) x[c] = ok ? p[c * f_own.sc] : 0.f;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) ss = fmaf(x[c], x[c], ss);
    const float nrm = prenorm ? 1.f : sqrtf(ss);
    const float nc = fmaxf(nrm, 1e-12f);
#pragma unroll
    for (int c = 0; c < kC; ++c) Ws[threadIdx.x * kLdW + c] = ok ? (prenorm ? x[c] : x[c] / nc) : 0.f;
    wn_s[threadIdx.x] = ok ? nrm : -1.f;  // -1: invalid slot
    widx_s[threadIdx.x] = idx;
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
  if (COLS && g_own == nullptr) return;

  // |u|^2 of the lane's other-side columns (same expression in both passes)
  float on[kPerLane];
#pragma unroll
  for (int j = 0; j < kPerLane; ++j) {
    const int o = lane + pk::kWave * j;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kC; ++c) s = fmaf(Os[o * kLdO + c], Os[o * kLdO + c], s);
    on[j] = s;
  }

  // kGroup rows at a time: every partner vector read from LDS serves kGroup dot products
  for (int rg = 0; rg < kRowsPerWave; rg += kGroup) {
    const int a0 = blockIdx.x * kTile + w * kRowsPerWave + rg;  // wave-uniform
    if (a0 >= S) break;
    bool ok[kGroup];
    int64_t idx[kGroup];
    float v[kGroup][kC], nrm[kGroup], vn[kGroup];
    bool any = false;
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
      const int a = a0 + g;
      const int t = a - blockIdx.x * kTile;  // row within the block's staged tile
      nrm[g] = wn_s[t];
      ok[g] = a < S && nrm[g] >= 0.f;
      any = any || ok[g];
      idx[g] = widx_s[t];
      if (!ok[g] && !COLS && a < S && lane == 0) {
        lse[(int64_t)b * S + a] = 0.f;
        term[(int64_t)b * S + a] = 0.f;
      }
      vn[g] = 0.f;
#pragma unroll
      for (int c = 0; c < kC; c += 4) {  // broadcast reads of the staged (normalized) row
        const float4 q = *reinterpret_cast<const float4*>(&Ws[t * kLdW + c]);
        v[g][c] = q.x; v[g][c + 1] = q.y; v[g][c + 2] = q.z; v[g][c + 3] = q.w;
      }
#pragma unroll
      for (int c = 0; c < kC; ++c) vn[g] = fmaf(v[g][c], v[g][c], vn[g]);
    }
    if (!any) continue;
    // distances and logits against all S partners (8 per lane); rows paired for packed FMAs
    float d[kGroup][kPerLane], lg[kGroup][kPerLane];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const int o = lane + pk::kWave * j;
      const bool vo = o < S && vb[o] != 0;
      fx2 dot01 = {0.f, 0.f}, dot23 = {0.f, 0.f};
#pragma unroll
      for (int c = 0; c < kC; ++c) {
        const float u = Os[o * kLdO + c];
        const fx2 uu = {u, u};
        dot01 = __builtin_elementwise_fma((fx2){v[0][c], v[1][c]}, uu, dot01);
        dot23 = __builtin_elementwise_fma((fx2){v[2][c], v[3][c]}, uu, dot23);
      }
      const float dot[kGroup] = {dot01.x, dot01.y, dot23.x, dot23.y};
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        const float d2 = fmaxf((vn[g] + on[j]) - 2.f * dot[g], 0.f);
        const bool on_ = vo && ok[g];
        d[g][j] = on_ ? __builtin_amdgcn_sqrtf(d2) : 0.f;  // v_sqrt_f32 (1 ulp)
        lg[g][j] = on_ ? -d[g][j] * inv_t : -__builtin_huge_valf();
      }
    }
    // softmax weights p[g][j] (row pass: this row's softmax; column pass: row o's, from lse)
    float p[kGroup][kPerLane];
    if (!COLS) {
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        float m = lg[g][0];
#pragma unroll
        for (int j = 1; j < kPerLane; ++j) m = fmaxf(m, lg[g][j]);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        if (!ok[g]) m = 0.f;  // all -inf: keep exp finite-free (0)
        const int a = a0 + g;
        float ld = 0.f;  // logit of the diagonal (a, a): lane a % 64, slot a / 64
#pragma unroll
        for (int j = 0; j < kPerLane; ++j)
          if (j == a / pk::kWave) ld = lg[g][j];
        ld = __shfl(ld, a % pk::kWave);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
          p[g][j] = __expf(lg[g][j] - m);
          s += p[g][j];
        }
        s = pk::wave_sum_f32(s);
        const float sm = m + __logf(s);
        const float is = __builtin_amdgcn_rcpf(s);
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) p[g][j] *= is;
        if (!ok[g]) continue;  // wave-uniform
        if (lane == 0) {
          lse[(int64_t)b * S + a] = sm;
          term[(int64_t)b * S + a] = sm - ld;
        }
      }
      if (g_own == nullptr) continue;
    } else {
#pragma unroll
      for (int j = 0; j < kPerLane; ++j) {
        const float l_oth = lse_s[lane + pk::kWave * j];
#pragma unroll
        for (int g = 0; g < kGroup; ++g) p[g][j] = __expf(lg[g][j] - l_oth);
      }
    }
    // r[g][o] = dL/dd = -(p - [o == a]) * sc / (t d)   (0 where d == 0 or invalid)
    float rs[kGroup];
#pragma unroll
    for (int g = 0; g < kGroup; ++g) rs[g] = 0.f;
    const float k_r = -sc * inv_t;
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const int o = lane + pk::kWave * j;
      float r4[kGroup];
#pragma unroll
      for (int g = 0; g < kGroup; ++g) {
        const float gg = p[g][j] - (o == a0 + g ? 1.f : 0.f);
        const float r = d[g][j] > 0.f ? gg * k_r * __builtin_amdgcn_rcpf(d[g][j]) : 0.f;  // implies ok[g], o valid
        r4[g] = r;
        rs[g] += r;
      }
      rbuf[w][o] = make_float4(r4[0], r4[1], r4[2], r4[3]);
    }
    __builtin_amdgcn_wave_barrier();  // rbuf rows complete (one wave's LDS ops run in order)
#pragma unroll
    for (int g = 0; g < kGroup; ++g) rs[g] = pk::wave_sum_f32(rs[g]);
    // sum_o r[g][o] u_o[c]: lane (c, half h) over half of the partners, then the two halves
    const int c = lane & 31, h = lane >> 5;
    fx2 acc01 = {0.f, 0.f}, acc23 = {0.f, 0.f};
    const float4* __restrict__ rb = &rbuf[w][h * (kMaxS / 2)];
    const float* __restrict__ os = &Os[(h * (kMaxS / 2)) * kLdO + c];
#pragma unroll 8
    for (int o = 0; o < kMaxS / 2; ++o) {
      const float4 r = rb[o];
      const float u = os[o * kLdO];
      const fx2 uu = {u, u};
      acc01 = __builtin_elementwise_fma((fx2){r.x, r.y}, uu, acc01);
      acc23 = __builtin_elementwise_fma((fx2){r.z, r.w}, uu, acc23);
    }
    float acc[kGroup] = {acc01.x, acc01.y, acc23.x, acc23.y};
#pragma unroll
    for (int g = 0; g < kGroup; ++g) {
      acc[g] += __shfl_xor(acc[g], 32);
      if (!ok[g]) continue;  // wave-uniform
      // d/dv, then F.normalize backward: (dv - v (v . dv)) / n  (dv / 1e-12 when clamped)
      const float vc = lane < kC ? Ws[(a0 + g - blockIdx.x * kTile) * kLdW + c] : 0.f;  // staged row
      const float dv = vc * rs[g] - acc[g];
      const float vdv = pk::wave_sum_f32(lane < kC ? vc * dv : 0.f);
      const float dx = prenorm ? dv : nrm[g] > 1e-12f ? (dv - vc * vdv) / nrm[g] : dv / 1e-12f;
      if (lane < kC) atomicAdd(g_own + ((int64_t)b * N_own + idx[g]) * kC + c, dx);
    }
    __builtin_amdgcn_wave_barrier();  // all lanes done reading rbuf before the next group
  }
}

}  // namespace

extern "C" int pk_nce_loss(const float* f1, const int64_t* st1, const float* f2, const int64_t* st2, int B,
                           int64_t N1, int64_t N2, int C,
                           const int64_t* pairs, int cap, const int64_t* rows, const uint8_t* valid, int S,
                           float nce_t, int prenorm, float* lse, float* term, float* loss, float* g1, float* g2,
                           void* stream) {
  PK_REQUIRE(B >= 0 && C == kC && S >= 0 && S <= kMaxS && cap >= 0 && nce_t > 0.f);
  PK_REQUIRE((g1 == nullptr) == (g2 == nullptr));
  if (B == 0) return PK_OK;
  PK_REQUIRE(loss != nullptr);
  hipStream_t s = pk::as_stream(stream);
  if (g1) {
    hipError_t e = pk::zero_async(g1, sizeof(float) * (size_t)B * N1 * kC, s);
    if (e == hipSuccess) e = pk::zero_async(g2, sizeof(float) * (size_t)B * N2 * kC, s);
    if (e != hipSuccess) return (int)e;
  }
  if (S == 0) return pk::zero_async(loss, sizeof(float) * B, s) == hipSuccess ? PK_OK : PK_ERR_ARG;
  PK_REQUIRE(f1 && f2 && pairs && rows && valid && lse && term && cap > 0);
  const float inv_t = 1.f / nce_t;
  const dim3 grid((S + kTile - 1) / kTile, B);
  const FeatView v1{f1, st1 ? st1[0] : N1 * kC, st1 ? st1[1] : kC, st1 ? st1[2] : 1};
  const FeatView v2{f2, st2 ? st2[0] : N2 * kC, st2 ? st2[1] : kC, st2 ? st2[2] : 1};
  hipLaunchKernelGGL(nce_pass_kernel<false>, grid, dim3(64 * kWaves), 0, s, v1, v2, N1, N2, pairs, cap, rows, valid,
                     S, inv_t, prenorm, lse, term, loss, g1);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(nce_pass_kernel<true>, grid, dim3(64 * kWaves), 0, s, v1, v2, N1, N2, pairs, cap, rows, valid,
                     S, inv_t, prenorm, lse, term, loss, g2);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
