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
// Kernels:
//   attn_fwd_kernel            one workgroup = 4 waves x 16 queries = 64 queries of one (crop,
//                              head); streams 64-key tiles of K, V through LDS; writes out and
//                              (m, 1 / sum) per query (saved for the backward)
//   attn_bwd_kernel            one workgroup = 8 waves x 32 keys = 256 keys of one (crop, head);
//                              streams 64-query tiles of Q, dO, O; delta = rowsum(dO * O),
//                              dV = P^T dO, dK = 0.25 dS^T Q, and a dQ = 0.25 dS K partial per key
//                              block (dS = P (dP - delta), dP = dO V^T): each contraction once
//   attn_bwd_dq_reduce_kernel  the dQ partials added in key-block order
#include <type_traits>

#include "common.hpp"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
constexpr int kD = 16;       // head dim
constexpr int kT = 64;       // rows per tile / per workgroup
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

constexpr int kKB = 256;   // keys per block (backward)
constexpr int kSA = 20;    // [row][p(d)] stride
constexpr int kSQ = 68;    // [d][row] stride
constexpr int kSTs = 36;   // dS transpose tile [q][32 keys] stride
constexpr int kSRq = 20;   // dQ partial [q][d] stride
constexpr int kOA = 0, kOG = kT * kSA, kOQT = 2 * kT * kSA, kOGT = kOQT + kD * kSQ, kOMI = kOGT + kD * kSQ;
constexpr int kTileF = kOMI + 3 * kT;  // floats per query-tile buffer
// LDS banking (MI355X_MICROARCH.md §LDS): a ds_read_b128 is served in four 16-lane groups, each
// holding every c = l & 15 once and lane groups g, g ^ 1 split as c in [4, 12) vs the rest. Rows
// c of a stride with an odd count of 16-B chunks fall on 16 distinct chunk slots, so a read of
// (row c, chunk g) is conflict-free once the chunk index is XORed with swz(c) = [4 <= c < 12]:
// the group then reads one chunk column. Every [row][.] / [d][.] tile below stores chunk j of row
// r at j ^ swz(r & 15).
__device__ __forceinline__ int swz(int c) { return ((c + 4) >> 3) & 1; }

// Forward: one workgroup = 8 waves x 16 queries = 128 queries of one (crop, head); 64-key tiles of
// K and V staged once per block in LDS, double-buffered with one barrier per tile (the next tile's
// global loads in flight during this one), K as [key][p(d)] and V as [d][key] so each MFMA operand
// quad is one conflict-free ds_read_b128 (8 per lane per tile).
constexpr int kFQ = 128;                            // queries per forward block
constexpr int kFKV = kT * kSA + kD * kSQ;           // floats per K / V tile buffer
__global__ __launch_bounds__(512) void attn_fwd_kernel(const float* __restrict__ q,
                                                       const float* __restrict__ k,
                                                       const float* __restrict__ v, int H, int N,
                                                       int M, int64_t sbk, int64_t sbv, float* __restrict__ out,
                                                       float* __restrict__ lse) {
  __shared__ __attribute__((aligned(16))) float KV[2 * kFKV];
  const int3 lb = pk::xcd_block3();  // a (crop, head)'s query blocks share one XCD's L2 (K / V)
  const int h = lb.y, b = lb.z;
  const int lane = pk::lane_id(), g = lane >> 4, c = lane & 15;
  const int qi = lb.x * kFQ + pk::wave_id() * 16 + c;
  const float* qb = q + ((int64_t)b * kD * H + h) * N;
  const float* kb = k + (int64_t)b * sbk + (int64_t)h * M;
  const float* vb = v + (int64_t)b * sbv + (int64_t)h * M;
  const int HM = H * M;
  float qr[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qr[s] = qi < N ? qb[(int64_t)(4 * s + g) * H * N + qi] * kScale : 0.f;
  // staging: threads 0-255 carry K, 256-511 V; thread -> (key sk = (tid & 255) >> 2, d 4 sp .. + 3)
  const int sk = (threadIdx.x & 255) >> 2, sp = threadIdx.x & 3;
  const bool stage_k = threadIdx.x < 256;
  const float* src = stage_k ? kb : vb;
  float pf[4];
  auto issue = [&](int k0) {
    const int kk = k0 + sk, kc = kk < M ? kk : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pf[i] = src[(int64_t)(4 * sp + i) * HM + kc];
  };
  auto stage = [&](int k0, float* buf) {
    const bool ok = k0 + sk < M;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = ok ? pf[i] : 0.f;
      const int d = 4 * sp + i;
      if (stage_k) buf[sk * kSA + 4 * (i ^ swz(sk & 15)) + sp] = x;  // K [key][p(d)], p(d) = 4 i + sp
      else buf[kT * kSA + d * kSQ + 4 * ((sk >> 2) ^ swz(d)) + (sk & 3)] = x;  // V [d][key]
    }
  };
  // one accumulator per 16-key sub-tile: four independent MFMA chains (a serial chain over
  // M ~ 5000 keys of a real CAD measured 4-5x torch's gradient error; split, it is within 1.5x)
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -__builtin_huge_valf(), l = 0.f;
  issue(0);
  stage(0, KV);
  if (kT < M) issue(kT);
  const int gs = 4 * (g ^ swz(c));
  // one 64-key tile; RAG: the ragged last tile (keys past M masked to -inf) — a separate
  // instantiation, so the full tiles carry no masking code (a uniform branch the compiler would
  // otherwise if-convert into every tile)
  auto tile = [&](const float* buf, int k0, auto rag) {
    constexpr bool RAG = decltype(rag)::value;
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 ka = *reinterpret_cast<const f32x4*>(&buf[(16 * t + c) * kSA + gs]);  // K[16t + c][4s + g]
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) st[t] = mfma(ka[s], qr[s], st[t]);  // S^T[key 16t + 4g + r][q c]
    }
    if constexpr (RAG) {
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
    l *= alpha;
    const f32x2 al2 = {alpha, alpha};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x2 a0 = {acc[t][0], acc[t][1]}, a1 = {acc[t][2], acc[t][3]};
      a0 *= al2;
      a1 *= al2;
      acc[t] = f32x4{a0.x, a0.y, a1.x, a1.y};
    }
    // (s - m) log2 e on packed f32 pairs (v_pk_add_f32 / v_pk_mul_f32: the same per-element
    // rounding), row sums in two pair lanes
    const f32x2 mn2 = {m, m}, l2e = {kLog2e, kLog2e};
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
    l += ps2.x + ps2.y;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 va = *reinterpret_cast<const f32x4*>(&buf[kT * kSA + c * kSQ + 16 * t + gs]);  // V[16t + 4g + r][c]
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mfma(va[r], st[t][r], acc[t]);
    }
  };
  auto sync_stage = [&](int j) {
    const int k0 = j * kT;
    __syncthreads();  // tile j staged; the buffer of tile j - 1 free
    if (k0 + kT < M) {
      stage(k0 + kT, KV + ((j + 1) & 1) * kFKV);
      if (k0 + 2 * kT < M) issue(k0 + 2 * kT);
    }
  };
  const int nfull = M / kT;
  int j = 0;
  for (; j < nfull; ++j) {
    sync_stage(j);
    tile(KV + (j & 1) * kFKV, j * kT, std::false_type{});
  }
  if (j * kT < M) {  // the ragged last tile
    sync_stage(j);
    tile(KV + (j & 1) * kFKV, j * kT, std::true_type{});
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

// One-pass backward (round 5): one workgroup of 8 waves per (crop, head, 256-key block); wave w
// owns keys kb0 + 32 w .. + 31 (two 16-key sub-tiles) with K, V (and K^T for dQ) in registers and
// walks every 64-query tile of the crop, staged once per block in LDS. Per 16 x 16 (query, key)
// sub-tile it forms S and dP (8 MFMAs), P and dS in registers, dV^T += dO^T P and dK^T += Q^T dS
// (8 MFMAs; P and dS in the S D-layout are directly the B operands), and dQ^T += K^T dS^T
// (4 MFMAs) after moving dS through a wave-private LDS tile (the one transposition the two
// contractions need: 4 ds_write_b32 + 1 ds_read_b128 per sub-tile). That is the 5 algorithmic
// contractions once each — the two-kernel form recomputed S and dP in both (7).
// dQ: the 8 waves' 32-key partials of a 64-query tile are added in wave order through LDS; the
// block's 256-key sum is written to partial slot p = key block (slot 0 is dq itself, the others
// the caller's work buffer) and attn_bwd_dq_reduce_kernel adds the slots in slot order and scales
// (deterministic; a single key block writes dq scaled, no reduce launch).
// delta = rowsum(dO * O) is formed per query as the tile is staged (fmaf over d in order, the
// four lanes' partial sums of a query added as (p0 + p1) + (p2 + p3)).

__global__ __launch_bounds__(512, 1) void attn_bwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ o, const float* __restrict__ dout, const float* __restrict__ lse, int H, int N,
    int M, int64_t sbk, int64_t sbv, int64_t sbdk, int64_t sbdv, float* __restrict__ dq,
    float* __restrict__ part, float* __restrict__ dk, float* __restrict__ dv) {
  // two query-tile buffers, each: Q [q][p(d)] (p(4 s + g) = 4 g + s), dO [q][p(d)], Q [d][q],
  // dO [d][q], then (m, 1 / sum, delta) per query; two dQ-partial buffers [wave][q][d]; the per-wave
  // dS transpose tiles. One barrier per query tile: tile j + 1 is staged and tile j - 1's partials
  // are added while tile j is contracted.
  __shared__ __attribute__((aligned(16))) float TB[2 * kTileF];
  __shared__ __attribute__((aligned(16))) float RQ[2 * 8 * kT * kSRq];
  __shared__ __attribute__((aligned(16))) float TS[8 * 16 * kSTs];
  const int3 xb = pk::xcd_block3();  // a (crop, head)'s key blocks share one XCD's L2 (Q / dO / O)
  const int kblk = xb.x, h = xb.y, b = xb.z;
  const int wave = pk::wave_id(), lane = pk::lane_id(), g = lane >> 4, c = lane & 15;
  const int HN = H * N;
  const int64_t qoff = ((int64_t)b * kD * H + h) * N;
  const float2* lb = reinterpret_cast<const float2*>(lse) + ((int64_t)b * H + h) * N;
  // this wave's keys: kk(t) = kb0 + 16 t + c (S / dP operands), kk(t, r) = kb0 + 16 t + 4 g + r (K^T)
  const int kb0 = kblk * kKB + 32 * wave;
  const float* kbp = k + (int64_t)b * sbk + (int64_t)h * M;
  const float* vbp = v + (int64_t)b * sbv + (int64_t)h * M;
  float kr[2][4], vr[2][4], kt[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kj = kb0 + 16 * t + c;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t a = (int64_t)(4 * s + g) * H * M + (kj < M ? kj : 0);
      const float kv = kbp[a], vv = vbp[a];  // unconditional at a clamped key
      kr[t][s] = kj < M ? kv * kScale : 0.f;
      vr[t][s] = kj < M ? vv : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kj2 = kb0 + 16 * t + 4 * g + r;
      const float kv = kbp[(int64_t)c * H * M + (kj2 < M ? kj2 : 0)];
      kt[t][r] = kj2 < M ? kv : 0.f;
    }
  }
  // keys past M: S starts at -inf (the MFMA chain's initial accumulator), so P = exp2(-inf) = 0 and
  // dS = 0 — no per-element mask (K, V, K^T are 0 there, dP = 0)
  f32x4 s0[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float z = kb0 + 16 * t + c < M ? 0.f : -__builtin_huge_valf();
    s0[t] = f32x4{z, z, z, z};
  }
  // staging: waves 0-3 carry dO and O (and form delta), waves 4-7 Q and (m, 1 / sum); thread ->
  // (query sq = (tid & 255) >> 2, channels 4 sp .. 4 sp + 3)
  const int sq = (threadIdx.x & 255) >> 2, sp = threadIdx.x & 3;
  const bool stage_g = threadIdx.x < 256;
  float pf[8];
  float2 pm = make_float2(0.f, 0.f);
  auto issue = [&](int q0) {
    const int qq = q0 + sq, qc = qq < N ? qq : 0;
    const float* src0 = stage_g ? dout : q;
#pragma unroll
    for (int i = 0; i < 4; ++i) pf[i] = src0[qoff + (int64_t)(4 * sp + i) * HN + qc];
    if (stage_g) {
#pragma unroll
      for (int i = 0; i < 4; ++i) pf[4 + i] = o[qoff + (int64_t)(4 * sp + i) * HN + qc];
    } else if (sp == 0) {
      pm = lb[qc];
    }
  };
  auto stage = [&](int q0, float* tb) {
    const bool ok = q0 + sq < N;
    float* A = tb + (stage_g ? kOG : kOA);
    float* T = tb + (stage_g ? kOGT : kOQT);
    float* MI = tb + kOMI;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = ok ? pf[i] : 0.f;
      const int d = 4 * sp + i;
      A[sq * kSA + 4 * (i ^ swz(sq & 15)) + sp] = x;  // p(d) = 4 i + sp: chunk i
      T[d * kSQ + 4 * ((sq >> 2) ^ swz(d)) + (sq & 3)] = x;
    }
    if (stage_g) {
      float dl = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) dl = fmaf(ok ? pf[i] : 0.f, ok ? pf[4 + i] : 0.f, dl);
      const float d1 = dl + __shfl_xor(dl, 1);
      const float d2 = d1 + __shfl_xor(d1, 2);
      if (sp == 0) MI[2 * kT + sq] = d2;
    } else if (sp == 0) {
      MI[sq] = ok ? pm.x : __builtin_huge_valf();  // exp2(-inf) * 0 = 0: padding queries carry no weight
      MI[kT + sq] = ok ? pm.y : 0.f;
    }
  };
  f32x4 dka[2][2], dva[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e) dka[t][e] = dva[t][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* ts = TS + wave * 16 * kSTs;
  const int P = gridDim.x;
  float* dst = kblk == 0 ? dq : part + (int64_t)(kblk - 1) * ((int64_t)gridDim.z * kD * HN);
  const float osc = P == 1 ? kScale : 1.f;  // one key block: dq final here
  // the 8 waves' partials of tile q0 (buffer rb) added in wave order: waves 0-3, thread = (query qq,
  // channels 4 j .. 4 j + 3), conflict-free ds_read_b128 rows
  auto reduce = [&](int q0, const float* rb) {
    if (threadIdx.x < 256) {
      const int qq = threadIdx.x & 63, j = threadIdx.x >> 6;
      f32x4 sum = *reinterpret_cast<const f32x4*>(&rb[qq * kSRq + 4 * j]);
#pragma unroll
      for (int w = 1; w < 8; ++w) sum += *reinterpret_cast<const f32x4*>(&rb[w * kT * kSRq + qq * kSRq + 4 * j]);
      if (q0 + qq < N) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[qoff + (int64_t)(4 * j + i) * HN + q0 + qq] = sum[i] * osc;
      }
    }
  };
  issue(0);
  stage(0, TB);
  if (kT < N) issue(kT);
  int j = 0;
  for (;; ++j) {
    const int q0 = j * kT;
    const float* tb = TB + (j & 1) * kTileF;
    __syncthreads();  // tile j staged; tile j - 1's partials complete; buffers of tile j - 1 free
    if (j > 0) reduce(q0 - kT, RQ + ((j - 1) & 1) * 8 * kT * kSRq);
    if (q0 + kT < N) {
      stage(q0 + kT, TB + ((j + 1) & 1) * kTileF);
      if (q0 + 2 * kT < N) issue(q0 + 2 * kT);
    }
    const float* QA = tb + kOA;
    const float* GA = tb + kOG;
    const float* QT = tb + kOQT;
    const float* GT = tb + kOGT;
    const float* MI = tb + kOMI;
    float* rq = RQ + (j & 1) * 8 * kT * kSRq + wave * kT * kSRq;
    f32x4 dqa[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gs = 4 * (g ^ swz(c));
      const f32x4 qa = *reinterpret_cast<const f32x4*>(&QA[(16 * u + c) * kSA + gs]);
      const f32x4 ga = *reinterpret_cast<const f32x4*>(&GA[(16 * u + c) * kSA + gs]);
      const f32x4 qtv = *reinterpret_cast<const f32x4*>(&QT[c * kSQ + 16 * u + gs]);
      const f32x4 gtv = *reinterpret_cast<const f32x4*>(&GT[c * kSQ + 16 * u + gs]);
      const f32x4 L4 = *reinterpret_cast<const f32x4*>(&MI[16 * u + 4 * g]);
      const f32x4 I4 = *reinterpret_cast<const f32x4*>(&MI[kT + 16 * u + 4 * g]);
      const f32x4 D4 = *reinterpret_cast<const f32x4*>(&MI[2 * kT + 16 * u + 4 * g]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 st = s0[t], dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma(qa[s], kr[t][s], st);  // S[q 16u + 4g + r][key 16t + c]
          dp = mfma(ga[s], vr[t][s], dp);  // dP
        }
        float pr[4], dsr[4];
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 Lp = {L4[r], L4[r + 1]}, Ip = {I4[r], I4[r + 1]}, Dp = {D4[r], D4[r + 1]};
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
          dva[t][u & 1] = mfma(gtv[r], pr[r], dva[t][u & 1]);   // dV^T[d][key] += dO^T[d][q] P[q][key]
          dka[t][u & 1] = mfma(qtv[r], dsr[r], dka[t][u & 1]);  // dK^T[d][key] += Q^T[d][q] dS[q][key]
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(4 * g + r) * kSTs + 4 * ((4 * t + (c >> 2)) ^ swz(4 * g + r)) + (c & 3)] = dsr[r];
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x4 dsT = *reinterpret_cast<const f32x4*>(&ts[c * kSTs + 16 * t + 4 * (g ^ swz(c))]);  // dS[q c][key 16t + 4g + r]
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma(kt[t][r], dsT[r], acc);  // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
      }
      dqa[u] = acc;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<f32x4*>(&rq[(16 * u + c) * kSRq + 4 * g]) = dqa[u];
    if (q0 + kT >= N) break;
  }
  __syncthreads();
  reduce(j * kT, RQ + (j & 1) * 8 * kT * kSRq);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kj = kb0 + 16 * t + c;
    if (kj < M) {
      const f32x4 dks = dka[t][0] + dka[t][1], dvs = dva[t][0] + dva[t][1];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t a = (int64_t)h * M + (int64_t)(4 * g + r) * H * M + kj;
        dk[(int64_t)b * sbdk + a] = dks[r] * kScale;
        dv[(int64_t)b * sbdv + a] = dvs[r];
      }
    }
  }
}

// dq = 0.25 (slot 0 + slot 1 + ... + slot P - 1), slots added in order; slot 0 is dq itself
template <typename V>
__global__ __launch_bounds__(256) void attn_bwd_dq_reduce_kernel(float* __restrict__ dq,
                                                                 const float* __restrict__ part, int64_t n, int P) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    V s = reinterpret_cast<const V*>(dq)[i];
    for (int p = 1; p < P; ++p) s += reinterpret_cast<const V*>(part)[(int64_t)(p - 1) * n + i];
    reinterpret_cast<V*>(dq)[i] = s * kScale;
  }
}

}  // namespace

extern "C" int pk_attention_fwd(const float* q, const float* k, const float* v, int B, int D, int H,
                                int N, int M, int64_t sbk, int64_t sbv, float* out, float* lse, void* stream) {
  PK_REQUIRE(B >= 0 && H > 0 && N >= 0 && M >= 0 && D == kD && sbk >= 0 && sbv >= 0);
  if (B == 0 || N == 0) return PK_OK;
  PK_REQUIRE(M > 0 && q && k && v && out && lse);
  const int64_t dense = (int64_t)kD * H * M;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((N + kFQ - 1) / kFQ, H, B), dim3(512), 0, pk::as_stream(stream),
                     q, k, v, H, N, M, sbk ? sbk : dense, sbv ? sbv : dense, out, lse);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int64_t pk_attention_bwd_work_size(int B, int D, int H, int N, int M) {
  if (B <= 0 || H <= 0 || N <= 0 || M <= 0 || D != kD) return 0;
  const int64_t P = (M + kKB - 1) / kKB;
  return (P - 1) * (int64_t)B * kD * H * N * (int64_t)sizeof(float);
}

extern "C" int pk_attention_bwd(const float* q, const float* k, const float* v, const float* out,
                                const float* dout, const float* lse, int B, int D, int H, int N,
                                int M, int64_t sbk, int64_t sbv, float* work, float* dq, float* dk, float* dv,
                                int64_t sbdk, int64_t sbdv, void* stream) {
  PK_REQUIRE(B >= 0 && H > 0 && N >= 0 && M >= 0 && D == kD && sbk >= 0 && sbv >= 0 && sbdk >= 0 && sbdv >= 0);
  if (B == 0 || N == 0 || M == 0) return PK_OK;
  const int P = (M + kKB - 1) / kKB;
  PK_REQUIRE(q && k && v && out && dout && lse && dq && dk && dv && (work || P == 1));
  PK_REQUIRE((int64_t)P * B * H <= (int64_t)INT32_MAX && (int64_t)H * N <= (int64_t)INT32_MAX);
  hipStream_t s = pk::as_stream(stream);
  const int64_t dense = (int64_t)kD * H * M;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(P, H, B), dim3(512), 0, s, q, k, v, out, dout, lse, H, N, M,
                     sbk ? sbk : dense, sbv ? sbv : dense, sbdk ? sbdk : dense, sbdv ? sbdv : dense, dq, work, dk, dv);
  PK_CHECK_LAUNCH();
  if (P > 1) {
    const int64_t n = (int64_t)B * kD * H * N;
    if (n % 4 == 0 && (reinterpret_cast<uintptr_t>(dq) & 15) == 0 && (reinterpret_cast<uintptr_t>(work) & 15) == 0) {
      const unsigned g = (unsigned)std::min<int64_t>((n / 4 + 255) / 256, 2048);
      hipLaunchKernelGGL(attn_bwd_dq_reduce_kernel<f32x4>, dim3(g), dim3(256), 0, s, dq, work, n / 4, P);
    } else {
      const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
      hipLaunchKernelGGL(attn_bwd_dq_reduce_kernel<float>, dim3(g), dim3(256), 0, s, dq, work, n, P);
    }
    PK_CHECK_LAUNCH();
  }
  return PK_OK;
}
