// H15 — the scalar head of DPFMLoss and the scaling of its input gradients.
//
// Reference: utils/loss.py:44-99 (DPFMLoss.forward) with FrobeniusLoss (:8-15):
//   fmap_loss = w_fmap * mean_b clamp(sum_ij (C12 - C_gt)^2, -1, 1000)
//   nce_loss  = sum_b nce_b * w_nce / m          (nce_b from pk_nce_loss)
//   acc_loss  = sum_b (wbce12_b + wbce21_b) * w_acc / m   (from pk_wbce)
//   loss      = fmap_loss + acc_loss + nce_loss
// The NCE and WBCE kernels already produce their per-crop losses and input gradients; this
// launch forms the four scalars and dloss/dC12, and pk_loss_scale multiplies the saved input
// gradients by the incoming gradient in one grouped launch. Together they replace the ~22
// forward and ~20 backward torch kernels of the composed loss (subtraction, pow, sums, clamp
// and its where-mask backward, means, products, the fill of the seed gradient ...).
#include <algorithm>

#include "common.hpp"

namespace {

constexpr int kLossThreads = 1024;
constexpr int kMaxScale = 8;

struct ScaleTable {
  const float* src[kMaxScale];
  float* dst[kMaxScale];
  float s[kMaxScale];
  int64_t start[kMaxScale + 1];  // element offsets of the tensors in the flattened range
  int count;
};

// one block: wave w handles crops w, w + 16, ...: f_b = sum (a - b)^2 (lane-strided partials,
// fixed-order wave sum), then dC for that crop; thread 0 forms the scalars in crop order.
__global__ __launch_bounds__(kLossThreads) void loss_head_kernel(const float* __restrict__ C12,
                                                                 const float* __restrict__ Cgt, int B, int KK,
                                                                 const float* __restrict__ nce,
                                                                 const float* __restrict__ wb, float w_fmap,
                                                                 float w_acc, float w_nce, float* __restrict__ loss,
                                                                 float* __restrict__ logs, float* __restrict__ dC) {
  __shared__ float fb[1024], snce[1024], swb[1024];
  const int lane = pk::lane_id(), w = pk::wave_id();
  constexpr int NW = kLossThreads / pk::kWave;
  constexpr int kPer = 16;  // K * K <= 1024 elements per crop: 16 per lane, loaded together
  const float scale = 2.f * (w_fmap / (float)B);  // d mean_b / d f_b * d f_b / d (a - b), per unit gradient
  // the per-crop scalars of the other terms into LDS by many threads (thread 0 then reads LDS,
  // not 3 B dependent global loads)
  for (int b = threadIdx.x; b < B; b += kLossThreads) {
    snce[b] = nce[b];
    swb[b] = wb[b] + wb[B + b];
  }
  for (int b = w; b < B; b += NW) {
    const float* a = C12 + (int64_t)b * KK;
    const float* g = Cgt + (int64_t)b * KK;
    // all of the lane's elements in flight at once (round 2's loop waited for each pair of loads)
    float d[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = lane + pk::kWave * i;
      const int ec = e < KK ? e : 0;
      const float av = a[ec], gv = g[ec];
      d[i] = e < KK ? av - gv : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      if (lane + pk::kWave * i < KK) s = fmaf(d[i], d[i], s);  // the same per-lane order as before
    s = pk::wave_sum_f32(s);  // butterfly: every lane holds the same sum
    if (lane == 0) fb[b] = s;
    const bool pass = s >= -1.f && s <= 1000.f;  // clamp's gradient mask (inclusive bounds)
    float* o = dC + (int64_t)b * KK;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = lane + pk::kWave * i;
      if (e < KK) o[e] = pass ? scale * d[i] : 0.f;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float fm = 0.f, nl = 0.f, al = 0.f;
    const float m = (float)B;
    for (int b = 0; b < B; ++b) {
      fm += fminf(fmaxf(fb[b], -1.f), 1000.f);
      nl += snce[b] * w_nce / m;
      al += swb[b] * w_acc / m;
    }
    const float fmap_loss = fm / m * w_fmap;
    loss[0] = (fmap_loss + al) + nl;
    logs[0] = nl;         // nce_loss
    logs[1] = al;         // acc_loss
    logs[2] = fmap_loss;  // fmap_loss
  }
}

// grid-stride over the concatenated element range of the table: dst = src * (s * g[0])
__global__ __launch_bounds__(256) void loss_scale_kernel(ScaleTable t, const float* __restrict__ g) {
  const float gv = g[0];
  const int64_t total = t.start[t.count];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    int i = 0;
    while (i + 1 < t.count && e >= t.start[i + 1]) ++i;
    const int64_t k = e - t.start[i];
    t.dst[i][k] = t.src[i][k] * (t.s[i] * gv);
  }
}

}  // namespace

extern "C" int pk_loss_head(const float* C12, const float* Cgt, int B, int K, const float* nce, const float* wb,
                            float w_fmap, float w_acc, float w_nce, float* loss, float* logs, float* dC,
                            void* stream) {
  PK_REQUIRE(B >= 1 && B <= 1024 && K >= 1 && K * K <= 1024);
  PK_REQUIRE(C12 && Cgt && nce && wb && loss && logs && dC);
  hipLaunchKernelGGL(loss_head_kernel, dim3(1), dim3(kLossThreads), 0, pk::as_stream(stream), C12, Cgt, B, K * K,
                     nce, wb, w_fmap, w_acc, w_nce, loss, logs, dC);
  PK_CHECK_LAUNCH();
  return PK_OK;
}

extern "C" int pk_loss_scale(const float* const* src, float* const* dst, const int64_t* numel, const float* scale,
                             int n, const float* g, void* stream) {
  PK_REQUIRE(n >= 0 && n <= kMaxScale);
  if (n == 0) return PK_OK;
  PK_REQUIRE(src && dst && numel && scale && g);
  ScaleTable t{};
  t.count = n;
  t.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    PK_REQUIRE(numel[i] >= 0 && (numel[i] == 0 || (src[i] && dst[i])));
    t.src[i] = src[i];
    t.dst[i] = dst[i];
    t.s[i] = scale[i];
    t.start[i + 1] = t.start[i] + numel[i];
  }
  const int64_t total = t.start[n];
  if (total == 0) return PK_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(loss_scale_kernel, dim3(blocks), dim3(256), 0, pk::as_stream(stream), t, g);
  PK_CHECK_LAUNCH();
  return PK_OK;
}
