// H8 — fused multi-head attention of the cross-attention refinement (fwd + bwd).
//
// Reference: modeling/dpfm.py:29-37 `attention(query, key, value)` on [B, dim, heads, N]
// views of the Conv1d projections (:50-54, heads interleaved: channel = d * heads + h):
//     scores = einsum('bdhn,bdhm->bhnm', q, k) / dim**.5 ;  prob = softmax(scores, -1)
//     out    = einsum('bhnm,bdhm->bdhn', prob, v)
// The reference materialises scores and prob ([B, heads, N, M] fp32, twice per layer);
// here they live only in registers (online softmax, FlashAttention-2 style), in fp32:
// products on the f32 MFMA (v_mfma_f32_16x16x4_f32). dim = 16 (gnn_dim 32 / 2 heads,
// config/dpfm_orig.yaml), so 1/sqrt(dim) = 0.25 (an exact pre-scale of one operand).
// Softmax terms are exp2((s - m) * log2 e) on v_exp_f32: the scaling multiplies the
// small difference s - m, not s, so no extra rounding proportional to |s| enters. The
// forward saves per query the row max m and 1 / sum (ms [B, heads, N, 2]); the backward
// rebuilds P = exp2((s - m) log2 e) / sum exactly as the reference's softmax does.
// K/V (resp. Q/dO) tiles are double-buffered: the next tile's global loads are in
// flight while the current tile is contracted.
//
// MFMA lane maps (16x16x4): A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15],
// D[row = 4 (l >> 4) + r][col = l & 15]. A 16x16 D tile of S^T = K Q^T leaves lane l
// with keys 4g + r (g = l >> 4) of query l & 15, which is directly the B operand of the
// next contraction over keys when step r pairs key 4g + r with A's lane group g.
//
// Kernels (one workgroup = 4 waves x 16 rows = 64 rows of one (crop, head)):
//   attn_fwd_kernel     queries; streams 64-key tiles of K, V through LDS; writes out
//                       and (m, 1 / sum) per query (saved for the backward)
//   attn_bwd_dq_kernel  queries; delta = rowsum(dO * O) then dQ = 0.25 dS K
//   attn_bwd_dkv_kernel keys; streams 64-query tiles of Q, dO; dV = P^T dO,
//                       dK = 0.25 dS^T Q with dS = P (dP - delta), dP = dO V^T
#include "common.hpp"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int kD = 16;       // head dim
constexpr int kT = 64;       // rows per tile / per workgroup
constexpr int kSR = 80;      // LDS stride of [d][row] arrays (bank-conflict-free MFMA reads)
constexpr int kSC = 20;      // LDS stride of [row][d] arrays
constexpr float kScale = 0.25f;  // 1 / sqrt(dim) for the gradients

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float grp_max(float v) {  // over the 4 lane groups (same l & 15)
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

__device__ __forceinline__ float grp_sum(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }

// A 64-row tile of a [D, H, L] slab (row index contiguous), 4 elements per thread:
// element e = tid + 256 j -> (d = e >> 6, row = e & 63); rows >= L read as 0.
struct Tile {
  float x[4];
};

__device__ __forceinline__ Tile load_tile(const float* __restrict__ src, int HL, int L, int r0) {
  Tile t;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = threadIdx.x + 256 * j;
    const int d = e >> 6, r = e & 63;
    t.x[j] = r0 + r < L ? src[(int64_t)d * HL + r0 + r] : 0.f;
  }
  return t;
}

// into LDS as [d][row] (stride kSR) and/or [row][d] (stride kSC)
__device__ __forceinline__ void store_tile(const Tile& t, float* __restrict__ dr, float* __restrict__ rd) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = threadIdx.x + 256 * j;
    const int d = e >> 6, r = e & 63;
    if (dr) dr[d * kSR + r] = t.x[j];
    if (rd) rd[r * kSC + d] = t.x[j];
  }
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ q,
                                                       const float* __restrict__ k,
                                                       const float* __restrict__ v, int H, int N,
                                                       int M, int64_t sbk, int64_t sbv, float* __restrict__ out,
                                                       float* __restrict__ lse) {
  __shared__ float Ks[kD * kSR];
  __shared__ float Vs[kT * kSC];
  const int3 lb = pk::xcd_block3();  // a (crop, head)'s query blocks share one XCD's L2 (K / V)
  const int h = lb.y, b = lb.z;
  const int lane = pk::lane_id(), g = lane >> 4, c = lane & 15;
  const int qi = lb.x * kT + pk::wave_id() * 16 + c;
  const float* qb = q + ((int64_t)b * kD * H + h) * N;
  const float* kb = k + (int64_t)b * sbk + (int64_t)h * M;
  const float* vb = v + (int64_t)b * sbv + (int64_t)h * M;
  float qr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qr[s] = qi < N ? qb[(int64_t)(4 * s + g) * H * N + qi] * kScale : 0.f;
  // one accumulator per 16-key sub-tile: four independent MFMA chains (a serial chain over
  // M ~ 5000 keys of a real CAD measured 4-5x torch's gradient error; split, it is within 1.5x)
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -__builtin_huge_valf(), l = 0.f;
  Tile kt = load_tile(kb, H * M, M, 0), vt = load_tile(vb, H * M, M, 0);
  for (int k0 = 0; k0 < M; k0 += kT) {
    __syncthreads();
    store_tile(kt, Ks, nullptr);
    store_tile(vt, nullptr, Vs);
    __syncthreads();
    if (k0 + kT < M) {  // next tile in flight during this one
      kt = load_tile(kb, H * M, M, k0 + kT);
      vt = load_tile(vb, H * M, M, k0 + kT);
    }
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) st[t] = mfma(Ks[(4 * s + g) * kSR + 16 * t + c], qr[s], st[t]);
    }
    if (k0 + kT > M) {  // workgroup-uniform: only a ragged last tile has keys past M
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (k0 + 16 * t + 4 * g + r >= M) st[t][r] = -__builtin_huge_valf();
    }
    float mt = -__builtin_huge_valf();
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mt = fmaxf(mt, st[t][r]);
    mt = grp_max(mt);
    const float mn = fmaxf(m, mt);
    const float alpha = m == -__builtin_huge_valf() ? 0.f : exp2_((m - mn) * kLog2e);
    m = mn;
    // (s - m) log2 e on packed f32 pairs (v_pk_add_f32 / v_pk_mul_f32: the same per-element
    // rounding), row sums in two pair lanes
    const f32x2 mn2 = {mn, mn}, l2e = {kLog2e, kLog2e};
    f32x2 ps2 = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        f32x2 d = {st[t][r], st[t][r + 1]};
        d = (d - mn2) * l2e;
        const f32x2 p = {exp2_(d.x), exp2_(d.y)};
        st[t][r] = p.x;
        st[t][r + 1] = p.y;
        ps2 += p;
      }
    l = l * alpha + (ps2.x + ps2.y);
    const f32x2 al2 = {alpha, alpha};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x2 a0 = {acc[t][0], acc[t][1]}, a1 = {acc[t][2], acc[t][3]};
      a0 *= al2;
      a1 *= al2;
      acc[t] = f32x4{a0.x, a0.y, a1.x, a1.y};
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mfma(Vs[(16 * t + 4 * g + r) * kSC + c], st[t][r], acc[t]);
  }
  l = grp_sum(l);
  const f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (qi < N) {
    const float inv = 1.f / l;
    float* ob = out + ((int64_t)b * kD * H + h) * N;
#pragma unroll
    for (int r = 0; r < 4; ++r) ob[(int64_t)(4 * g + r) * H * N + qi] = accs[r] * inv;
    if (g == 0) {
      float2* ms = reinterpret_cast<float2*>(lse) + ((int64_t)b * H + h) * N + qi;
      *ms = make_float2(m, inv);
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ o, const float* __restrict__ dout, const float* __restrict__ lse,
    int H, int N, int M, int64_t sbk, int64_t sbv, float* __restrict__ delta, float* __restrict__ dq) {
  __shared__ float Ks[kD * kSR];
  __shared__ float Vs[kD * kSR];
  __shared__ float KT[kT * kSC];
  const int3 lb = pk::xcd_block3();  // a (crop, head)'s query blocks share one XCD's L2 (K / V)
  const int h = lb.y, b = lb.z;
  const int lane = pk::lane_id(), g = lane >> 4, c = lane & 15;
  const int qi = lb.x * kT + pk::wave_id() * 16 + c;
  const int64_t qoff = ((int64_t)b * kD * H + h) * N;
  const float* kb = k + (int64_t)b * sbk + (int64_t)h * M;
  const float* vb = v + (int64_t)b * sbv + (int64_t)h * M;
  float qr[4], dor[4];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t a = qoff + (int64_t)(4 * s + g) * H * N + qi;
    qr[s] = qi < N ? q[a] * kScale : 0.f;
    dor[s] = qi < N ? dout[a] : 0.f;
    dl = fmaf(dor[s], qi < N ? o[a] : 0.f, dl);
  }
  dl = grp_sum(dl);  // delta = sum_d dO * O for query qi
  const float2 ms = qi < N ? reinterpret_cast<const float2*>(lse)[((int64_t)b * H + h) * N + qi]
                           : make_float2(__builtin_huge_valf(), 0.f);
  if (qi < N && g == 0) delta[((int64_t)b * H + h) * N + qi] = dl;
  f32x4 acc[4];  // independent chains per 16-key sub-tile (accuracy, see the forward)
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  Tile kt = load_tile(kb, H * M, M, 0), vt = load_tile(vb, H * M, M, 0);
  for (int k0 = 0; k0 < M; k0 += kT) {
    __syncthreads();
    store_tile(kt, Ks, KT);
    store_tile(vt, Vs, nullptr);
    __syncthreads();
    if (k0 + kT < M) {
      kt = load_tile(kb, H * M, M, k0 + kT);
      vt = load_tile(vb, H * M, M, k0 + kT);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma(Ks[(4 * s + g) * kSR + 16 * t + c], qr[s], st);
        dp = mfma(Vs[(4 * s + g) * kSR + 16 * t + c], dor[s], dp);
      }
      // packed pairs (v_pk_*: the same per-element rounding as the scalar ops)
      float pr[4], dsr[4];
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        f32x2 d = {st[r], st[r + 1]};
        d = (d - f32x2{ms.x, ms.x}) * f32x2{kLog2e, kLog2e};
        f32x2 pp = f32x2{exp2_(d.x), exp2_(d.y)} * f32x2{ms.y, ms.y};
        const f32x2 ds = pp * (f32x2{dp[r], dp[r + 1]} - f32x2{dl, dl});
        pr[r] = pp.x;
        pr[r + 1] = pp.y;
        dsr[r] = ds.x;
        dsr[r + 1] = ds.y;
      }
      if (k0 + kT > M) {  // workgroup-uniform: keys past M (ragged last tile) carry no weight
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (k0 + 16 * t + 4 * g + r >= M) dsr[r] = 0.f;
      }
      (void)pr;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mfma(KT[(16 * t + 4 * g + r) * kSC + c], dsr[r], acc[t]);
    }
  }
  const f32x4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (qi < N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) dq[qoff + (int64_t)(4 * g + r) * H * N + qi] = accs[r] * kScale;
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    int H, int N, int M, int64_t sbk, int64_t sbv, int64_t sbdk, int64_t sbdv, float* __restrict__ dk,
    float* __restrict__ dv) {
  __shared__ float Qs[kD * kSR];
  __shared__ float Os[kD * kSR];  // dO as [d][q]
  __shared__ float QT[kT * kSC];
  __shared__ float OT[kT * kSC];  // dO as [q][d]
  __shared__ __attribute__((aligned(16))) float Ls[kT];
  __shared__ __attribute__((aligned(16))) float Is[kT];
  __shared__ __attribute__((aligned(16))) float Ds[kT];
  const int3 xb = pk::xcd_block3();  // a (crop, head)'s key blocks share one XCD's L2 (Q / dO)
  const int h = xb.y, b = xb.z;
  const int lane = pk::lane_id(), g = lane >> 4, c = lane & 15;
  const int kj = xb.x * kT + pk::wave_id() * 16 + c;
  const float* qb = q + ((int64_t)b * kD * H + h) * N;
  const float* gb = dout + ((int64_t)b * kD * H + h) * N;
  const float2* lb = reinterpret_cast<const float2*>(lse) + ((int64_t)b * H + h) * N;
  const float* db = delta + ((int64_t)b * H + h) * N;
  float kr[4], vr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t a = (int64_t)h * M + (int64_t)(4 * s + g) * H * M + (kj < M ? kj : 0);
    const float kv = k[(int64_t)b * sbk + a], vv = v[(int64_t)b * sbv + a];  // unconditional
    kr[s] = kj < M ? kv * kScale : 0.f;
    vr[s] = kj < M ? vv : 0.f;
  }
  // the per-query (m, 1 / sum) and delta of a 64-query tile, one query per thread < kT, loaded a
  // tile ahead like Q / dO (a load issued between the loop's barriers exposed a full memory
  // latency per tile)
  auto load_md = [&](int q0, float2& msv, float& dv) {
    const int qq = q0 + (int)threadIdx.x;
    const int qc = qq < N ? qq : 0;
    const float2 m2 = lb[qc];
    const float d1 = db[qc];
    msv = qq < N ? m2 : make_float2(__builtin_huge_valf(), 0.f);  // exp2(-inf) = 0
    dv = qq < N ? d1 : 0.f;
  };
  float2 msn = make_float2(0.f, 0.f);
  float dn = 0.f;
  if (threadIdx.x < kT) load_md(0, msn, dn);
  // two independent chains (even / odd 16-query sub-tiles; accuracy, see the forward): four
  // would cost this kernel its third wave per SIMD
  f32x4 dka[2], dva[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) dka[t] = dva[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  Tile qt = load_tile(qb, H * N, N, 0), gt = load_tile(gb, H * N, N, 0);
  for (int q0 = 0; q0 < N; q0 += kT) {
    __syncthreads();
    store_tile(qt, Qs, QT);
    store_tile(gt, Os, OT);
    if (threadIdx.x < kT) {
      Ls[threadIdx.x] = msn.x;
      Is[threadIdx.x] = msn.y;
      Ds[threadIdx.x] = dn;
    }
    __syncthreads();
    if (q0 + kT < N) {
      qt = load_tile(qb, H * N, N, q0 + kT);
      gt = load_tile(gb, H * N, N, q0 + kT);
      if (threadIdx.x < kT) load_md(q0 + kT, msn, dn);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma(Qs[(4 * s + g) * kSR + 16 * t + c], kr[s], st);  // S[q][key]
        dp = mfma(Os[(4 * s + g) * kSR + 16 * t + c], vr[s], dp);  // dP[q][key]
      }
      // per-query (m, 1 / sum, delta) of queries 16 t + 4 g .. + 3 as 16-B LDS reads; packed pairs
      const float4 L4 = *reinterpret_cast<const float4*>(&Ls[16 * t + 4 * g]);
      const float4 I4 = *reinterpret_cast<const float4*>(&Is[16 * t + 4 * g]);
      const float4 D4 = *reinterpret_cast<const float4*>(&Ds[16 * t + 4 * g]);
      float pr[4], dsr[4];
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f32x2 Lp = r == 0 ? f32x2{L4.x, L4.y} : f32x2{L4.z, L4.w};
        const f32x2 Ip = r == 0 ? f32x2{I4.x, I4.y} : f32x2{I4.z, I4.w};
        const f32x2 Dp = r == 0 ? f32x2{D4.x, D4.y} : f32x2{D4.z, D4.w};
        f32x2 d = (f32x2{st[r], st[r + 1]} - Lp) * f32x2{kLog2e, kLog2e};
        const f32x2 pp = f32x2{exp2_(d.x), exp2_(d.y)} * Ip;
        const f32x2 ds = pp * (f32x2{dp[r], dp[r + 1]} - Dp);
        pr[r] = pp.x;
        pr[r + 1] = pp.y;
        dsr[r] = ds.x;
        dsr[r + 1] = ds.y;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = 16 * t + 4 * g + r;
        dva[t & 1] = mfma(OT[qq * kSC + c], pr[r], dva[t & 1]);   // dV^T[d][key] += dO^T[d][q] P[q][key]
        dka[t & 1] = mfma(QT[qq * kSC + c], dsr[r], dka[t & 1]);  // dK^T[d][key] += Q^T[d][q] dS[q][key]
      }
    }
  }
  const f32x4 dks = dka[0] + dka[1], dvs = dva[0] + dva[1];
  if (kj < M) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t a = (int64_t)h * M + (int64_t)(4 * g + r) * H * M + kj;
      dk[(int64_t)b * sbdk + a] = dks[r] * kScale;
      dv[(int64_t)b * sbdv + a] = dvs[r];
    }
  }
}

}  // namespace

extern "C" int pk_attention_fwd(const float* q, const float* k, const float* v, int B, int D, int H,
                                int N, int M, int64_t sbk, int64_t sbv, float* out, float* lse, void* stream) {
  PK_REQUIRE(B >= 0 && H > 0 && N >= 0 && M >= 0 && D == kD && sbk >= 0 && sbv >= 0);
  if (B == 0 || N == 0) return PK_OK;
  PK_REQUIRE(M > 0 && q && k && v && out && lse);
  const int64_t dense = (int64_t)kD * H * M;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((N + kT - 1) / kT, H, B), dim3(256), 0, pk::as_stream(stream),
                     q, k, v, H, N, M, sbk ? sbk : dense, sbv ? sbv : dense, out, lse);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_attention_bwd(const float* q, const float* k, const float* v, const float* out,
                                const float* dout, const float* lse, int B, int D, int H, int N,
                                int M, int64_t sbk, int64_t sbv, float* delta, float* dq, float* dk, float* dv,
                                int64_t sbdk, int64_t sbdv, void* stream) {
  PK_REQUIRE(B >= 0 && H > 0 && N >= 0 && M >= 0 && D == kD && sbk >= 0 && sbv >= 0 && sbdk >= 0 && sbdv >= 0);
  if (B == 0 || N == 0 || M == 0) return PK_OK;
  PK_REQUIRE(q && k && v && out && dout && lse && delta && dq && dk && dv);
  hipStream_t s = pk::as_stream(stream);
  const int64_t dense = (int64_t)kD * H * M;
  sbk = sbk ? sbk : dense;
  sbv = sbv ? sbv : dense;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((N + kT - 1) / kT, H, B), dim3(256), 0, s, q, k, v, out, dout,
                     lse, H, N, M, sbk, sbv, delta, dq);
  PK_CHECK_LAUNCH();
  hipLaunchKernelGGL(attn_bwd_dkv_kernel, dim3((M + kT - 1) / kT, H, B), dim3(256), 0, s, q, k, v, dout, lse,
                     delta, H, N, M, sbk, sbv, sbdk ? sbdk : dense, sbdv ? sbdv : dense, dk, dv);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
