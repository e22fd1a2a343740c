/* posekern.h — C-ABI of libposekern.so, the MI355X (gfx950) drop-in for the RGB-D
 * pose-inference hot path of m13ammed/6D-Pose-Estimation-for-Unseen-Categories.
 *
 * The reference has no FFI of its own: its "operator API" is a set of Python call
 * signatures. Each entry point below names the reference function
 * it replaces (file:line under the reference tree); dpfm_amd/ keeps those Python
 * signatures and calls these functions through ctypes.
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless stated; the caller allocates every
 *     buffer. `stream` is a hipStream_t (void* here so the header needs no HIP
 *     include); work is stream-ordered, nothing blocks the host.
 *   - Return: 0 ok; 1000 invalid argument; 1001 capacity exceeded; any other value
 *     is the hipError_t of the failing launch.
 *   - Ragged batches are PACKED: rows of crop b are rows [off[b], off[b+1]) of a
 *     row-major array; `off` is int64 [B+1] on the device. `*max` arguments bound the
 *     largest crop (host knowledge, no device read-back).
 *   - Variable-size outputs take a per-crop capacity and report the true count;
 *     entries beyond the capacity are dropped (the caller re-runs with more room).
 */
#ifndef POSEKERN_H
#define POSEKERN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* H3 farthest-point sampling. Replaces upstream DPFM dpfm/utils.py::
 * farthest_point_sample(xyz[3,N], ratio) as called at dataset/object.py:145-148
 * (the random start becomes the explicit start[b]).
 *   xyz    f32 [T,3] packed crops, off int64 [B+1], nmax = max crop size
 *   start  int32 [B] first centroid, npoint int32 [B] samples per crop
 *   out    int64 [B, out_stride]; row b holds npoint[b] indices local to crop b, then zeros
 *          (written by the call: out needs no initialisation)
 * Bit-exact: fp32 ((dx²+dy²)+dz²), strict-< update, first-index argmax. */
int pk_fps(const float* xyz, const int64_t* off, int B, int nmax, const int32_t* start,
           const int32_t* npoint, int64_t* out, int out_stride, void* stream);

/* H5 ball query, pass 1. Replaces the dense part of dataset/object.py:281-286
 * find_positives: mask[b,i,j] = ||cad_i - pc_j|| <= r_b, fp64, bit-exact.
 *   cad f64 [T1,3] / cad_off, pc f64 [T2,3] / pc_off (packed crops)
 *   thr2 f64 [B]: largest double s with sqrt(s) <= r_b (computed on the host)
 *   mask uint8 [B, n1max, ld] (ld % 16 == 0, ld >= n2max) or NULL (counts only)
 *   rowcount int32 [B, n1max] partners per CAD point */
int pk_ball_query_mask(const double* cad, const int64_t* cad_off, const double* pc,
                       const int64_t* pc_off, const double* thr2, int B, int n1max, int n2max,
                       uint8_t* mask, int ld, int32_t* rowcount, void* stream);

/* H5 ball query, pass 2. Replaces np.argwhere(mask) (dataset/object.py:288) and
 * get_overlap (dataset/object.py:311-317).
 *   mask from pass 1 or NULL (distances recomputed), rowcount from pass 1
 *   rowoff int64 [B, n1max] scratch (exclusive scan of rowcount)
 *   pairs int64 [B, cap, 2] (i, j) in row-major order, count int64 [B] true totals
 *   ov12 int8 [B, n1max], ov21 int8 [B, n2max] (either may be NULL)
 *   over int32 [1] or NULL: 1 when some crop's count exceeds cap (its pair list was truncated)
 *   colcount int32 [B, n2max] or NULL: per crop point j, the pairs (i, j) among the first cap of
 *            the list (the row weights of C_gt's normal equations: pk_cgt_lstsq's cnt) */
int pk_ball_query_pairs(const double* cad, const int64_t* cad_off, const double* pc,
                        const int64_t* pc_off, const double* thr2, int B, int n1max, int n2max,
                        const uint8_t* mask, int ld, const int32_t* rowcount, int64_t* rowoff,
                        int64_t* pairs, int64_t cap, int64_t* count, int8_t* ov12, int8_t* ov21,
                        int32_t* over, int32_t* colcount, void* stream);

/* H1 crop formation. Replaces dataset/object.py:73-88 dpt_2_pcld (with the plus-shaped
 * erode_seg_mask of :52-71 and `seg == 255` of :137) for F frames at once.
 *   depth uint16 [F,H,W], mask uint8 [F,H,W] (mask_visib png values; 255 = object)
 *   K f64 [F,9] row-major intrinsics, cam_scale f32 [F] = 1000 / depth_scale
 *   rowcnt int32 [F,H], rowoff int64 [F,H] scratch
 *   count int64 [F] points per frame, off int64 [F+1] packed offsets
 *   xyz f64 [cap,3] packed back-projected points in cm, row-major pixel order.
 *   pix int32 [cap] (may be NULL): v*W+u of each point; idxmap int32 [F,H,W] (may be
 *   NULL): point index within its frame, -1 for pixels that are not points.
 * Bit-exact vs numpy: z32 = f32(depth)/f32(cam_scale); X = (((u-cx)*z)/fx)*100. */
int pk_backproject(const uint16_t* depth, const uint8_t* mask, int F, int H, int W,
                   const double* K, const float* cam_scale, int32_t* rowcnt, int64_t* rowoff,
                   int64_t* count, int64_t* off, double* xyz, int64_t cap, int32_t* pix,
                   int32_t* idxmap, void* stream);

/* H2 statistical outlier removal. Replaces dataset/object.py:33-50 remove_outliers
 * (Open3D RemoveStatisticalOutliers(nb_neighbors=20, std_ratio=0.3)).
 *   xyz f64 [T,3] packed / off, knn <= 20
 *   pix / idxmap (optional, from pk_backproject, crop b = frame b): an exact kNN bound
 *   from the 5x5 pixel window prunes the brute-force scan (results unchanged)
 *   K f64 [B,9] (optional, with pix): camera intrinsics of frame b; bounds the pixel box
 *   that can hold a point within the kNN radius so only that box is scanned
 *   avg f64 [T] mean kNN distance, thr f64 [B] keep threshold
 *   ccount int32 [B, ceil(nmax/1024)], coff int64 (same shape) scratch
 *   kept int64 [B] survivors, out_off int64 [B+1] their packed offsets
 *   out64 f64 [T,3], out32 f32 [T,3] (either may be NULL) survivors in input order
 *   kept_idx int64 [T] (may be NULL) survivor index within its input crop */
int pk_sor(const double* xyz, const int64_t* off, int B, int nmax, int knn, double std_ratio,
           const int32_t* pix, const int32_t* idxmap, int H, int W, const double* K, double* avg,
           double* thr,
           int32_t* ccount, int64_t* coff, int64_t* kept, int64_t* out_off, double* out64,
           float* out32, int64_t* kept_idx, void* stream);

/* FPS sample-count policy of dataset/object.py:145-147 on device counts (no host sync):
 * fixed > 0: npoint = fixed if n > fixed, else -n; fixed <= 0: npoint = int(limit/n * n)
 * if n > limit, else -n (negative = keep all n points in order, no FPS: the reference's
 * `if pcd.shape[0] > 2000` branch). start[b] = splitmix64(seed ^ splitmix64(base + b)) % n
 * (replaces upstream torch.randint; may be NULL; base = the global index of crop 0, so a
 * rank's shard draws the starts the whole batch would). out_off int64 [B+1]. */
int pk_fps_npoint(const int64_t* off, int B, int fixed, int limit, uint64_t seed, int64_t base,
                  int32_t* npoint, int32_t* start, int64_t* out_off, void* stream);

/* H4 pcd[idx0] (dataset/object.py:148) + transform(pcd, R, t, inv=True) (:174, :304-309).
 *   pcd f64 [T,3] packed / off; idx int64 [B, idx_stride] FPS output (unused when
 *   npoint[b] < 0); R f64 [B,9] row-major R_m2c, t f64 [B,3] (cm)
 *   sel64 f64 / align64 f64 / sel32 f32 [sum npoint, 3] packed by out_off (any NULL)
 *   status int32 [B] or NULL: 1 when an index of crop b lies outside [0, off[b+1] - off[b])
 *   (that point is not read: its outputs are NaN), else 0; written for every crop. */
int pk_gather_transform(const double* pcd, const int64_t* off, int B, const int64_t* idx,
                        int idx_stride, const int32_t* npoint, int npmax, const int64_t* out_off,
                        const double* R, const double* t, double* sel64, double* align64,
                        float* sel32, int32_t* status, void* stream);

/* pk_gather_transform plus H6's collate of its two fields in the same launch (the crop-formation
 * path's pk_collate_pad calls on sel64 and align64, dataset/helpers.py:22-50): pad_sel32 /
 * pad_align32 f32 [B, ld, 3] (any NULL) = f32(sel64) / f32(align64) of crop b's first
 * min(count_b, ld) points, zero rows after; counts int32 [B] (or NULL) = min(count_b, ld). */
int pk_gather_transform_pad(const double* pcd, const int64_t* off, int B, const int64_t* idx,
                            int idx_stride, const int32_t* npoint, int npmax, const int64_t* out_off,
                            const double* R, const double* t, double* sel64, double* align64,
                            float* sel32, int32_t* status, int ld, float* pad_sel32, float* pad_align32,
                            int32_t* counts, void* stream);

/* H6 collate (dataset/helpers.py:22-50: torch.Tensor(x) then pad_sequence(batch_first=True))
 * of one packed per-crop field: src [T, C] f64 (src_f64 = 1) or f32, packed by off [B+1];
 * dst f32 [B, ld, C] with crop b's first min(n_b, ld) rows cast to f32 and every later row
 * zero (ld = the batch maximum reproduces collate exactly). counts int32 [B] (may be NULL)
 * receives min(n_b, ld). */
int pk_collate_pad(const void* src, int src_f64, int C, const int64_t* off, int B, int ld, float* dst,
                   int32_t* counts, void* stream);

/* Packed-layout helpers: per-segment exclusive scan of int32 counts (S segments of n),
 * and off[b+1] = off[b] + counts[b]. */
int pk_segment_scan(const int32_t* cnt, int S, int n, int64_t* off, int64_t* total, void* stream);
int pk_offsets_from_counts(const int64_t* counts, int B, int64_t* off, void* stream);

/* H7 spectral diffusion of DiffusionNet's LearnedTimeDiffusion (upstream layers.py,
 * models/dpfm.py:22-30), fp32, K = C = 64:
 *   mode 0: out = Phi (E ⊙ raw), raw = Phi^T (mass ⊙ in), E[k,c] = exp(-evals_k t_c)
 *   mode 1: out = mass ⊙ Phi (E ⊙ Phi^T in) (= dL/dx), gt[c] = -sum_b sum_k evals E saved (Phi^T in)
 *   in [B,N] rows of row stride ld_in, out rows of row stride ld_out (>= C, multiples of 4: a
 *   slice of a wider concatenation buffer), mass [B,N], evecs [B,N,K], evals [B,K], t [C];
 *   clamp_t: use max(t, 1e-8), and in mode 0 write it back into t (the reference's in-place
 *   diffusion_time.clamp_(min=1e-8) before every diffusion);
 *   work f32 [B, ceil(N/64), K, C]; raw (mode 0, may be NULL) / scaled [B,K,C] (scratch: mode 0
 *   forms the coefficients inside the expand pass and leaves it unwritten);
 *   saved = raw of the forward (mode 1); gt [C] (mode 1, summed over crops in crop order);
 *   accumulate: out += result (a gradient summed into an existing one) instead of out = result */
int pk_spectral_diffusion(const float* in, int ld_in, const float* mass, const float* evecs, const float* evals,
                          float* t, int clamp_t, int B, int N, int K, int C, int mode, float* work, float* raw,
                          float* scaled, const float* saved, float* gt, float* out, int ld_out, int accumulate,
                          void* stream);

/* H9 regularized fmap solve. Replaces the 30 sequential torch.inverse + bmm of
 * modeling/dpfm.py:185-193: C[b,i,:] = ((AAt_b + lambda diag(D_b[i,:]))^-1 BAt_b[i,:]^T)^T.
 * fp64 Gauss-Jordan with partial pivoting, one wave per (b, i). K must be 30.
 *   AAt, BAt, D, C: f32 [B,K,K]. Backward: G = dL/dC; dBAt f32 [B,K,K];
 *   dAAt_part f32 [B,K,K,K] per-row slabs -w_i x_i^T (dL/dAAt = sum over axis 1). */
int pk_fmap_solve(const float* AAt, const float* BAt, const float* D, float lambda, int B, int K,
                  float* C, void* stream);
int pk_fmap_solve_backward(const float* AAt, const float* BAt, const float* D, float lambda, int B,
                           int K, const float* G, float* dBAt, float* dAAt_part, void* stream);

/* H8 fused multi-head attention. Replaces modeling/dpfm.py:29-37 `attention` (einsum
 * scores / sqrt(dim), softmax over keys, einsum with values) without materialising the
 * [B, heads, N, M] score/probability tensors. fp32, dim D = 16 only.
 *   q f32 [B, D, H, N], k / v f32 [B, D, H, M] (heads interleaved as the reference's
 *   view(B, dim, heads, N) of a [B, D*H, N] projection), out f32 [B, D, H, N],
 *   lse f32 [B, H, N, 2]: per query the row max m and 1 / sum of exp(s - m) (for the backward).
 * Backward: dout like out; dq like q, dk / dv like k; work: pk_attention_bwd_work_size bytes of
 * scratch (any contents, nothing kept across calls; NULL when that size is 0, i.e. M <= 256). One
 * pass over (query tile, 256-key block) forms S, dP, dV, dK and a dQ partial per key block; the
 * partials (slot 0 in dq, the others in work) are added in key-block order by a second launch.
 * sbk / sbv (sbdk / sbdv): batch strides in elements of k / v (dk / dv); 0 = dense D H M. A
 * batch stride of 2 D H M reads (writes) the key and value halves of one [B, 2 D H, M] buffer:
 * the stacked key / value projection (one launch for modeling/dpfm.py:63-67's proj[1], proj[2]). */
int pk_attention_fwd(const float* q, const float* k, const float* v, int B, int D, int H, int N,
                     int M, int64_t sbk, int64_t sbv, float* out, float* lse, void* stream);
int64_t pk_attention_bwd_work_size(int B, int D, int H, int N, int M);
int pk_attention_bwd(const float* q, const float* k, const float* v, const float* out,
                     const float* dout, const float* lse, int B, int D, int H, int N, int M,
                     int64_t sbk, int64_t sbv, float* work, float* dq, float* dk, float* dv, int64_t sbdk,
                     int64_t sbdv, void* stream);

/* Weight/bias gradients of the per-point layers of H7/H8 (DiffusionNet Linear layers,
 * models/dpfm.py:22-30; refinement Conv1d(k=1), modeling/dpfm.py:16-26,45-54,82-95):
 * dw[o,i] = sum_r dy[r,o] x[r,i], db[o] = sum_r dy[r,o] over all R = B*N points.
 *   layout 0: x [R, I], dy [R, O] row-major; layout 1: x [R/N, I, N], dy [R/N, O, N]
 *   I, O <= 128, O * I <= 8192; work f32 [ceil(R/128) * (O*I + O)]; db may be NULL.
 *   accumulate = 1 adds to dw / db instead of overwriting them (a weight shared by several
 *   calls of one forward, e.g. the refinement layer applied twice at modeling/dpfm.py:100-104,
 *   accumulates its gradient the way autograd's AccumulateGrad does). */
int pk_linear_wgrad(const float* x, const float* dy, int layout, int64_t R, int I, int O, int N,
                    float* work, float* dw, float* db, int accumulate, void* stream);

/* Grouped weight gradients: every pk_linear_wgrad of one backward pass in two launches
 * (all layers' slice partials, then all reductions) instead of two per layer. `calls` is a
 * HOST array read during the call (its contents are baked into the launches' kernel
 * arguments, so a HIP-graph capture replays them). Per call as pk_linear_wgrad, with
 * (O/32 rounded up) * (I/32 rounded up) <= 8 and N % 16 == 0 for layout 1. A call with
 * accumulate = 1 adds to the dw / db of the one earlier call (accumulate = 0) naming the
 * same dw: r = partials(earlier) + partials(later), autograd's accumulation order for a
 * layer applied twice (modeling/dpfm.py:100-104). work: f32, pk_linear_wgrad_grouped_work()
 * elements (host-computed from the calls). */
typedef struct pk_wgrad_call {
  const float* x;
  const float* dy;
  float* dw;
  float* db;
  int64_t R;
  int32_t I, O, N, layout, accumulate, pad;
  int64_t sx, sdy; /* layout 1: batch strides of x / dy in elements (0: dense I N / O N), so a
                    * channel slice of a wider buffer (the stacked key / value gradients) is read
                    * in place */
} pk_wgrad_call;
int64_t pk_linear_wgrad_grouped_work(const pk_wgrad_call* calls, int n);
int pk_linear_wgrad_grouped(const pk_wgrad_call* calls, int n, float* work, int64_t work_elems, void* stream);

/* Optimizer tail of one training step (scripts/train.py:121-124): clip_grad_norm_(max_norm)
 * over every gradient, then RMSprop (config/dpfm_orig.gin:62-63: no momentum, not centered,
 * no weight decay) — two launches. work: f32 [64] scratch (partial norms). HOST arrays of n <= 96 device pointers: params, grads
 * (clipped in place), square_avg state, steps (f32 [1] counters, +1 each; may be NULL) and
 * numel (host int64). one_minus_alpha = float(1 - alpha) computed in double by the caller
 * (torch passes value = 1 - alpha as a Python float). norm_out (f32 [1], may be NULL)
 * receives the total gradient norm before clipping. */
int pk_clip_rmsprop(float* const* params, float* const* grads, float* const* square_avg, float* const* steps,
                    const int64_t* numel, int n, float max_norm, float lr, float alpha, float one_minus_alpha,
                    float eps, float* work, float* norm_out, void* stream);

/* H8 refinement MLP's InstanceNorm1d(C, affine=False, eps) + ReLU (modeling/dpfm.py:16-26),
 * fused, on a channels-first activation viewed as rows = B*C rows of N points:
 *   fwd: y = max((x - mean) * invstd, 0) per row (biased variance), mean / invstd f32 [rows]
 *   bwd: dx from dy (the gradient of y), x and the saved mean / invstd. */
int pk_instnorm_relu_fwd(const float* x, int64_t rows, int N, float eps, float* y, float* mean, float* invstd,
                         void* stream);
int pk_instnorm_relu_bwd(const float* x, const float* dy, const float* mean, const float* invstd, int64_t rows,
                         int N, float* dx, void* stream);

/* H15 overlap term: upstream WeightedBCELoss (utils/loss.py:79-83) for both directions of
 * B crops in one launch. p12 f32 [B, N1] / p21 [B, N2] sigmoid outputs, t12 / t21 int8 0/1
 * masks; loss f32 [2, B] (row 0: 12, row 1: 21); g12 / g21 (both or neither) receive
 * d loss[., b] / d p. */
int pk_wbce(const float* p12, const int8_t* t12, int N1, const float* p21, const int8_t* t21, int N2, int B,
            float* loss, float* g12, float* g21, void* stream);

/* models/dpfm.py:53,61-66: out = cat((a - sub) * mul, (b - sub) * mul) over na + nb f32
 * elements (the shared encoder's input features; mul = float32(1) / 50, the reciprocal torch
 * multiplies by when dividing by a Python scalar on the GPU). */
int pk_affine_cat(const float* a, int64_t na, const float* b, int64_t nb, float sub, float mul, float* out,
                  void* stream);

/* F.normalize(x, p=2, dim=-1) over the C channels of [B, N, C] features (overlap head,
 * modeling/dpfm.py:140-145), forward and backward. strides = HOST int64[3] element strides
 * {batch, point, channel} shared by x / y / dy / dx (rows or channels-first storage);
 * nrm f32 [B * N] = ||x|| per point (saved by the forward for the backward).
 * y_rows (may be NULL): the same normalized values also in rows layout [B, N, C] (the NCE
 * term's gathers read whole rows, utils/loss.py:17-40); dy_rows (may be NULL; dy may be NULL
 * when it is given): a second incoming gradient in rows layout, summed with dy. */
int pk_l2_normalize_fwd(const float* x, const int64_t* strides, int B, int N, int C, float* y, float* nrm,
                        float* y_rows, void* stream);
int pk_l2_normalize_bwd(const float* y, const float* dy, const float* nrm, const int64_t* strides, int B, int N,
                        int C, float* dx, const float* dy_rows, void* stream);

/* H8 overlap head, fused (modeling/dpfm.py:125-145 OverlapPredictorNet: F.normalize(x, dim=-1)
 * -> Linear(32, 32) -> ReLU -> Linear(32, 1) -> Sigmoid), both shapes in one launch per
 * direction. Replaces pk_l2_normalize_fwd + two pk_linear_ex launches per shape (forward) and
 * the sigmoid-backward thin layer + the 32 -> 32 input gradient + pk_l2_normalize_bwd
 * (backward) with the same arithmetic in the same order (bit-identical outputs).
 * Per shape s (0: CAD, 1: crop): x[s] f32 [B, N[s], 32] at element strides[s] {batch, point,
 * channel} (rows or channels-first storage); w0 [32, 32], b0 [32], w1 [1, 32], b1 [1].
 * Forward writes n[s] (the normalized features, x's storage), nrm[s] [B N] (||x||),
 * s[s] [B N] (the scores); nrows[s] / h[s] (may be NULL): the normalized features and the
 * hidden ReLU output as rows [B N, 32] (the NCE term's input and the weight gradients' input).
 * Backward reads n, nrm, h, s and ds[s] [B N] (d loss / d score), dnr[s] (may be NULL: a
 * second gradient on the rows copy of n, the NCE term's), writes g[s] [B N] (d loss / d the
 * last layer's pre-activation), dh[s] [B N, 32] (d loss / d the first layer's
 * pre-activation, ReLU applied) and dx[s] (x's storage); dadd[s] (may be NULL; x's storage): a
 * gradient of x from another consumer, added to dx[s] (the features' second consumer, the fmap
 * head, models/dpfm.py:80-90). */
typedef struct pk_overlap_head_args {
  const float* x[2];
  int64_t strides[2][3];
  int32_t N[2];
  int32_t B, pad;
  const float* w0;
  const float* b0;
  const float* w1;
  const float* b1;
  float* n[2];
  float* nrm[2];
  float* nrows[2];
  float* h[2];
  float* s[2];
  const float* ds[2];
  const float* dnr[2];
  float* g[2];
  float* dh[2];
  float* dx[2];
  const float* dadd[2];
} pk_overlap_head_args;
int pk_overlap_head_fwd(const pk_overlap_head_args* a, void* stream);
int pk_overlap_head_bwd(const pk_overlap_head_args* a, void* stream);

/* H7 DiffusionNet block MLP forward, fused (upstream DiffusionNetBlock.forward at
 * models/dpfm.py:22-30: mlp(cat[x_in, x_diffuse]) + x_in, MiniMLP 128 -> 64 -> ReLU -> 64 ->
 * ReLU -> 64). x_in / x_diff f32 [R, C], C = 64; W1 [64, 128], W2 / W3 [64, 64], biases
 * [64]; writes cat [R, 128], h1 / h2 [R, 64] (post-ReLU, kept for the backward) and
 * y [R, 64] = h2 W3^T + b3 + x_in. */
int pk_mlp3_fwd(const float* x_in, const float* x_diff, const float* w1, const float* b1, const float* w2,
                const float* b2, const float* w3, const float* b3, int64_t R, int C, float* cat, float* h1, float* h2,
                float* y, void* stream);

/* H9 fmap head around the solve (modeling/dpfm.py:154-176, models/dpfm.py:66-72), K = 30,
 * C = 32: W = evecs[:, :K] * mass (f32 products); A = W_x^T F_x, Bm = W_y^T F_y [B,K,C];
 * AAt = A A^T, BAt = Bm A^T [B,K,K]; D = get_mask(evals_x[:K], evals_y[:K], gamma) [B,K,K].
 *   evecs f32 [B,N,lde], mass f32 [B,N], F (refined features [B,N,C]) at HOST int64[3]
 *   element strides {batch, point, channel}; evals f32 [B, ldv].
 * Backward: part = pk_fmap_solve_backward's dAAt slabs [B,K,K,K], dBAt [B,K,K] ->
 *   dA, dBm [B,K,C] (scratch outputs) and dF_x = W_x dA, dF_y = W_y dBm written at the
 *   HOST strides dfx_strides / dfy_strides.
 * work: f32 scratch of pk_fmap_head_work_len(B, N1, N2) floats (the 128-point chunk partials
 *   of the projections); PK_ERR_ARG when work_len is smaller. */
int64_t pk_fmap_head_work_len(int B, int N1, int N2);
int pk_fmap_head_fwd(const float* evecs_x, int ldex, const float* mass_x, const float* fx, const int64_t* fx_strides,
                     int N1, const float* evecs_y, int ldey, const float* mass_y, const float* fy,
                     const int64_t* fy_strides, int N2, const float* evals_x, int ldvx, const float* evals_y, int ldvy,
                     int B, int K, int C, float gamma, float* A, float* Bm, float* AAt, float* BAt, float* D,
                     float* work, int64_t work_len, void* stream);
int pk_fmap_head_bwd(const float* part, const float* dBAt, const float* A, const float* Bm, const float* evecs_x,
                     int ldex, const float* mass_x, int N1, const float* evecs_y, int ldey, const float* mass_y, int N2,
                     int B, int K, int C, float* dA, float* dBm, float* dfx, const int64_t* dfx_strides, float* dfy,
                     const int64_t* dfy_strides, void* stream);

/* H9 resolvent mask: upstream dpfm/utils.py::get_mask(evals1[:K], evals2[:K], gamma) for every
 * crop (the per-crop branch that always runs, modeling/dpfm.py:164-182). evals1 / evals2 f32
 * [B, ld] (first K used, K <= 32); D f32 [B, K, K], D[b][j][i] from evals2[j], evals1[i]. */
int pk_resolvent_mask(const float* evals1, int ld1, const float* evals2, int ld2, int B, int K, float gamma, float* D,
                      void* stream);

/* Forward / input gradient of the same per-point layers (nn.Linear at models/dpfm.py:22-30
 * and modeling/dpfm.py:16-26,90-91,113-116; Conv1d(k=1) at modeling/dpfm.py:16-26,49-50):
 *   y = x W^T (+ bias) (ReLU if relu), W f32 [Cout, Cin]; with transw = 1 the weight is
 *   read as W^T (W stored [Cin, Cout]): the input gradient dx = dy W of a layer is
 *   pk_linear_fwd(dy, W, NULL, ..., Cin = O, Cout = I, transw = 1).
 *   layout 0: x [R, Cin] -> y [R, Cout]; layout 1: x [R/N, Cin, N] -> y [R/N, Cout, N].
 *   Cin, Cout <= 128; bias may be NULL. mask (may be NULL; same layout as y): outputs where
 *   mask <= 0 are written as 0 — the ReLU backward (aten threshold_backward) of the layer
 *   feeding this one, folded into its input gradient (mask = that layer's output). */
int pk_linear_fwd(const float* x, const float* w, const float* bias, int layout, int64_t R, int N, int Cin,
                  int Cout, int transw, int relu, const float* mask, float* y, void* stream);

/* pk_linear_fwd with explicit output placement and epilogue (one launch where torch would
 * add concatenations, residual adds, slices and transposed copies around the layer):
 *   ldx: rows layout — x row stride; channels-first — x batch stride (0: contiguous);
 *   y / ldy: output (same stride meaning; 0: contiguous);
 *   store_cf (rows layout): y written channels-first [R/N, Cout, N] (ldy = its batch stride);
 *   y2 / split / ldy2 (rows layout): output columns >= split go to y2 at column - split;
 *   add / lda / add_cols: y[.., o] += add[.., o] for o < add_cols, after bias / ReLU / mask
 *   (residual connections, gradient accumulation of a split input);
 *   act: 0 none, 1 ReLU, 2 sigmoid (thin kernels); mask: contiguous [R, Cout] / [R/N, Cout, N]
 *   (see pk_linear_fwd);
 *   pre / pre_out (thin kernels): the input is first scaled elementwise by pre (1 - pre) —
 *   a following sigmoid's backward (pre = its output) folded into the input gradient — and
 *   the scaled input written to pre_out (for the weight gradient), same indexing as x.
 * The thin kernels (Cin or Cout <= 4) take strides only. */
typedef struct pk_linear_args {
  const float* x;
  const float* w;
  const float* bias;
  int32_t layout;
  int32_t N;
  int64_t R;
  int32_t Cin, Cout, transw, act;
  const float* mask;
  int64_t ldx;
  float* y;
  int64_t ldy;
  float* y2;
  int64_t ldy2;
  int32_t split, store_cf;
  const float* add;
  int64_t lda;
  int32_t add_cols, pad;
  const float* pre;
  float* pre_out;
  /* channels-first MFMA kernel only (layout 1, Cin in {16, 32, 64, 128}, N % 16 == 0):
   *   w2 / wsplit: stored weight rows >= wsplit are read from w2 (row - wsplit): two layers'
   *     weights stacked with no concatenation (transw = 0: rows = outputs, e.g. the key and value
   *     projections of modeling/dpfm.py:63-67 as one 32 -> 64 launch; transw = 1: rows of the stored
   *     [Cin, Cout] weight, e.g. their input gradients summed in one 64 -> 32 launch); bias2: bias
   *     entries >= wsplit (transw = 0);
   *   add2 / lda2: a second added operand over every output, after add (gradient accumulation of
   *     an input used three times). NULL / 0: unused. */
  const float* w2;
  const float* bias2;
  int32_t wsplit, pad2;
  const float* add2;
  int64_t lda2;
} pk_linear_args;
int pk_linear_ex(const pk_linear_args* a, void* stream);
/* Two independent pk_linear_ex calls; when both are channels-first layers with Cin, Cout in
 * {32, 64} and the same points-per-wave choice they share one launch (the refinement's q and
 * stacked k / v projections, Pq^T and [Pk; Pv]^T, both shapes' last_lin: modeling/dpfm.py:50-54,
 * 111-112), otherwise they run as two. Same arguments and results as two pk_linear_ex calls. */
int pk_linear_ex2(const pk_linear_args* a0, const pk_linear_args* a1, void* stream);

/* H10 / H11 correspondence head. Replaces fmap2pointmap_solvers/naive.py:20-34
 * (topk = 1: dist.argmin(dim=-2)) and spacial_filtering.py:19-38 (topk = 5: the first 5
 * rows of dist.sort(dim=-2)) with dist = cdist(evecs_x[:, :30] @ C^T, evecs_y[:, :30]).
 *   evecs_x f32 [B,V1max,ldx] (first 30 columns used), C f32 [B,30,30],
 *   evecs_y f32 [B,V2max,ldy]; n1/n2 int32 [B] valid rows
 *   mode 0: fp32 MFMA on torch.cdist's augmented K = 32 operands (the parity path);
 *   mode 1: bf16 MFMA cross term + f32 norms; mode 2: bf16x3 (hi/lo split, three bf16 MFMAs)
 *   work: scratch of pk_feat_dist_work_size(B, V1max, V2max, topk, mode) bytes (may be 0 and
 *     NULL), any contents: nothing in it is read before this call writes it, and nothing is kept
 *     across calls (round 5: the mode-0 top-1 pass finishes every column inside one workgroup,
 *     or writes row-part keys that a second launch merges — no arrival words, no zeroing contract;
 *     round 6: the mode-0 top-5 pass likewise — exact five per column, recomputing only the rows
 *     of kept streams that may hold more members; row parts merged by a second launch).
 *   out_idx int64 [B,V2max,topk] ascending distance (ties: lower index); out_dist f32
 *   [B,V2max,topk] Euclidean distances (may be NULL). Fused selection epilogue. */
int64_t pk_feat_dist_work_size(int B, int V1max, int V2max, int topk, int mode);
int pk_feat_dist_topk(const float* evecs_x, int ldx, const float* C, const float* evecs_y, int ldy,
                      const int32_t* n1, const int32_t* n2, int B, int V1max, int V2max, int topk, int mode,
                      void* work, int64_t work_bytes, int64_t* out_idx, float* out_dist, void* stream);

/* H11 rigidity filter (fmap2pointmap_solvers/spacial_filtering.py:42-75), three rounds
 * on device with the 0.055 -> 0.065 fallback.
 *   cand int64 [B,ldc,2] (cad idx, pc idx), ncand int32 [B]; cad f32 [B,ldcad,3],
 *   pc f32 [B,ldpc,3]; thr4 f32 [B,4] = diam * (0.3, 0.15, 0.055, 0.065)
 *   list_a/list_b int64 [B,ldc], n_a/n_b int32 [B], score f32 [B,ldc] scratch;
 *   partial f32 scratch of pk_rigidity_filter_work_size(B, nmax, ldc) bytes, or NULL: with it each
 *   unordered candidate pair is evaluated once (64 x 64 tile pairs, per-tile partial sums added in
 *   tile order); without it every candidate sums over all others itself.
 * Result: survivors' candidate rows in list_b[b, :n_b[b]] (input order). */
int64_t pk_rigidity_filter_work_size(int B, int nmax, int ldc);
int pk_rigidity_filter(const int64_t* cand, int ldc, const int32_t* ncand, const float* cad, int ldcad,
                       const float* pc, int ldpc, const float* thr4, int B, int nmax, int64_t* list_a,
                       int64_t* list_b, int32_t* n_a, int32_t* n_b, float* score, float* partial, void* stream);

/* H12 inlier ratio (utils/utils.py:81-105) per crop: mean(||cad[c] - pc_aligned[p]|| < thr),
 * 0 when there are no correspondences.
 *   pairs int64: layout 0 [B,ldp,2] (cad, pc), layout 1 [B,2,ldp], or layout 2 [B,ldp] the CAD
 *   index of crop point k (a point map: pc index = k); npairs int32 [B]
 *   cad f32 [B,ldcad,3], pc_aligned f32 [B,ldpc,3], thr f32 [B] -> ir f32 [B]
 *   status int32 [B] or NULL: 1 when a CAD index of crop b lies outside [0, ldcad) or a crop index
 *   outside [0, ldpc) (such a pair is not read and counts as an outlier), else 0; every crop written */
int pk_inlier_ratio(const int64_t* pairs, int ldp, int layout, const int32_t* npairs, const float* cad,
                    int ldcad, const float* pc_aligned, int ldpc, const float* thr, int B, float* ir,
                    int32_t* status, void* stream);
/* The batch's mean inlier ratio (train.py:116 `IR.mean()` over the crops' ratios): out f32 [1] =
 * (sum of x[0..n)) / n, the sum in a fixed order (deterministic). */
int pk_mean_f32(const float* x, int64_t n, float* out, void* stream);

/* H15 C_gt (utils/utils.py:67-79 C_from_sparse_P): least squares
 * evecs2[P[:,1], :30] X = evecs1[P[:,0], :30] per crop (fp64 normal equations: G from the
 * per-row pair counts, H over 64-pair slices; Gauss-Jordan with partial pivoting).
 * pairs int64 [B,ldp,2] (any order), npairs int64 [B]; evecs f32 [B,Vmax,ld]; K must be
 * 30; work f64 [pk_cgt_lstsq_work_size(ldp, V2max, B)]; Cgt f32 [B,30,30].
 * cnt int32 [B, ldc] or NULL: per crop row j the pairs with crop index j among the first
 * min(npairs, ldp) (pk_ball_query_pairs' colcount, formed with the crops; rows j >= ldc count 0);
 * NULL: counted here (one fill + one integer-atomic count launch). */
int64_t pk_cgt_lstsq_work_size(int ldp, int V2max, int B);

/* NCE pair selection (utils/loss.py:27-30: np.random.choice(P, num, replace=False) per
 * crop, every row when P <= num). count int64 [B] pair-list lengths (capped at cap);
 * k = min(num, cap); rows int64 [B, k] distinct rows of [0, min(count, cap)) drawn by a
 * keyed pseudo-random bijection, valid uint8 [B, k] (0 on the padding tail, whose rows
 * are 0). ctr int64 [1] device step counter mixed into the key, incremented per call. */
int pk_nce_select(const int64_t* count, int B, int64_t cap, int num, uint64_t seed, int64_t* ctr,
                  int64_t* rows, uint8_t* valid, void* stream);
/* H15 NCE term (utils/loss.py:17-40 NCESoftmaxLoss.forward) for a batch of crops, with
 * its input gradients. Per crop b: S pair slots, slot a selects pair rows[b,a] of
 * pairs[b] (int64 [B, cap, 2]: CAD index, crop index) when valid[b,a] (uint8);
 *   q_a = normalize(f1[b, pairs[..,0]]), k_a = normalize(f2[b, pairs[..,1]]),
 *   logits = -cdist(q, k) / nce_t, loss[b] = mean over valid a of CE(logits[a], a)
 * (0 for a crop without valid slots). f1 f32 [B, N1, C], f2 f32 [B, N2, C], C = 32, element
 * strides st1 / st2 = HOST int64[3] {batch, point, channel} (NULL: contiguous rows), so a
 * channels-first [B, C, N] storage is read in place;
 * S <= 512. lse / term f32 [B, S] scratch. g1 / g2 (both or neither) f32 [B, N1|N2, C]
 * receive d loss[b] / d f1[b], f2[b]: the passes write each slot's gradient row into
 * dx_rows (f32 [2, B, S, C] scratch, required with g1 / g2), and a third launch sums a
 * point's slot rows in ascending slot order (torch's gather backward, deterministic).  * prenorm = 1: f1 / f2 are already F.normalize'd; g1 / g2 are then the gradients with
 * respect to the normalized features (no normalize backward).
 */
int pk_nce_loss(const float* f1, const int64_t* st1, const float* f2, const int64_t* st2, int B, int64_t N1,
                int64_t N2, int C, const int64_t* pairs,
                int cap, const int64_t* rows, const uint8_t* valid, int S, float nce_t, int prenorm, float* lse,
                float* term, float* loss, float* g1, float* g2, float* dx_rows, void* stream);

/* H15 DPFMLoss scalar head (utils/loss.py:44-99, FrobeniusLoss :8-15), one launch:
 *   fmap = w_fmap * mean_b clamp(sum (C12_b - Cgt_b)^2, -1, 1000); nce = sum_b nce[b] w_nce / B;
 *   acc = sum_b (wb[b] + wb[B + b]) w_acc / B; loss[0] = (fmap + acc) + nce;
 *   logs = {nce, acc, fmap}; dC = dloss/dC12 for a unit incoming gradient.
 * C12 / Cgt / dC f32 [B,K,K]; nce f32 [B] (pk_nce_loss); wb f32 [2,B] (pk_wbce). B <= 1024. */
int pk_loss_head(const float* C12, const float* Cgt, int B, int K, const float* nce, const float* wb,
                 float w_fmap, float w_acc, float w_nce, float* loss, float* logs, float* dC, void* stream);
/* dst[i] = src[i] * (scale[i] * g[0]) for n <= 8 tensors (HOST pointer tables; numel HOST
 * int64[n]) in one launch: the loss head's saved input gradients times the incoming one. */
int pk_loss_scale(const float* const* src, float* const* dst, const int64_t* numel, const float* scale, int n,
                  const float* g, void* stream);
int pk_cgt_lstsq(const int64_t* pairs, int ldp, const int64_t* npairs, const float* evecs1, int ld1,
                 int V1max, const float* evecs2, int ld2, int V2max, int B, int K, const int32_t* cnt,
                 int ldc, double* work, float* Cgt, void* stream);

/* H13 RANSAC + Umeyama (scripts/test_RANSAC.py:288-310, Open3D 0.17 semantics, ransac_n 4).
 *   src f64 (CAD) / dst f64 (crop, camera frame) packed [T,3] with src_off/dst_off [B+1];
 *   corres int32 [sum n_b, 2] (src row, dst row) packed by cor_off int64 [B+1]; nmax >= every
 *   n_b (host bound: sizes the correspondence chunks that spread one crop over the chip)
 *   hyps int32 [sum H_b, 4] correspondence rows (packed by hyp_off) or NULL: then draw j
 *   of hypothesis h is splitmix64(seed ^ splitmix64(4h + j)) % n_b
 *   H hypotheses per crop; inlier iff ||T s - d||^2 < max_dist^2
 *   work: scratch of pk_ransac_work_size(B, H, nmax) bytes (fitted poses, per-chunk scores)
 *   T f64 [B,4,4] row-major best pose, stats f64 [B,3] (fitness, inlier rmse, best h).
 * Best = (fitness desc, rmse asc, index asc). A crop's error sum is taken per chunk in
 * correspondence order, then over chunks in order.
 *   status int32 [B] or NULL: 1 when a correspondence row of crop b lies outside its source /
 *   target points or a given hypothesis row outside [0, n_b) (read as row 0 instead of faulting),
 *   else 0; written for every crop. */
int64_t pk_ransac_work_size(int B, int64_t H, int nmax);
int pk_ransac(const double* src, const int64_t* src_off, const double* dst, const int64_t* dst_off,
              const int32_t* corres, const int64_t* cor_off, const int32_t* hyps, const int64_t* hyp_off,
              uint64_t seed, int64_t H, double max_dist, int B, int nmax, void* work, int64_t work_bytes,
              double* T, double* stats, int32_t* status, void* stream);

/* H14 pose metrics of scripts/test_RANSAC.py:77-81, 154-238 for B crops:
 *   cad f64 [T,3] packed / off (model points in the object frame), T_est / T_gt f64
 *   [B,4,4] row-major; work f64 [13 * B * nmax] scratch
 *   out f64 [B,7] = {ADD (add), mean per-row |.| x3 (compute_add_score's xyz-direction
 *   distances), mean per-row 1-D nearest-GT distance x3 (compute_adds_score)}; a crop with more
 *   than nmax points (the scratch capacity) is not evaluated: its row is NaN */
int pk_pose_metrics(const double* cad, const int64_t* off, int B, int nmax, const double* T_est,
                    const double* T_gt, double* work, double* out, void* stream);

/* erode_seg_mask alone (dataset/object.py:52-71): plus-shaped 3x3 erosion of
 * `mask == 255`, border pixels not eroded by the image edge. out uint8 [F,H,W] 0/1. */
int pk_erode_mask(const uint8_t* mask, int F, int H, int W, uint8_t* out, void* stream);

/* H16 RGB(-feature) sampling at projected 3D points (north-star row; the reference loads
 * RGB only with color=True, dataset/scene.py:95-97, and never feeds it to the model).
 * img uint8 [F,H,W,C]; pts f64 [T,3] camera-frame cm, packed per frame by off [F+1];
 * bilinear at u = fx X/Z + cx, v = fy Y/Z + cy, zero outside the image
 * (= grid_sample(align_corners=True, padding_mode="zeros")); out f32 [T,C] / 255. */
int pk_sample_rgb(const uint8_t* img, int F, int H, int W, int C, const double* K, const double* pts,
                  const int64_t* off, int nmax, float* out, void* stream);

/* H16 (north-star "RGB-backbone feature sampling at projected 3D points"): the same
 * projection and bilinear weights as pk_sample_rgb on an f32 feature map fmap [F, C, H, W]
 * (channels-first), zero outside the image (= grid_sample(align_corners=True,
 * padding_mode="zeros")); out f32 [T, C], no scaling. pts / off / nmax as pk_sample_rgb. */
int pk_sample_features(const float* fmap, int F, int C, int H, int W, const double* K, const double* pts,
                       const int64_t* off, int nmax, float* out, void* stream);

/* (f4) Point-to-point ICP after RANSAC (scripts/test_RANSAC.py:436-446: Open3D 0.17
 * registration_icp(source, target, threshold 0.2, trans_init = T_RANSAC, PointToPoint,
 * ICPConvergenceCriteria(max_iteration 2000), relative fitness / rmse 1e-6)), batched.
 *   src f64 [Ts,3] packed by src_off [B+1] (the CAD), tgt f64 [Tt,3] packed by tgt_off [B+1]
 *   (the reference's GT-posed CAD, or the observed crop); T_init f64 [B,4,4] row-major;
 *   nsrc_max / ntgt_max: per-crop capacities (grid and scratch sizing); a crop whose source or
 *   target is larger is not refined (T = T_init, stats converged = -1: capacity exceeded).
 * Per evaluation every source point T s takes its nearest target point (ties: lowest index);
 * a pair iff d^2 < max_dist^2; fitness = pairs / |src|, rmse = sqrt(sum d^2 / pairs) (0 without
 * pairs). Update: Umeyama (no scaling) of the pairs (identity without pairs), T <- U T. Stop
 * when |dfitness| < rel_fitness and |drmse| < rel_rmse, or after max_iter updates.
 *   pk_icp_init       sorts each crop's target by x (slab search), orders the source queries by x
 *                     under T_init, and loads T_init;
 *   pk_icp_iterate    enqueues `steps` evaluations (converged crops return at once) and, if
 *                     active_count != NULL, writes the number of crops still iterating (int32,
 *                     device) — a host loop polls it; capture-safe (no host synchronisation);
 *   pk_icp_result     T f64 [B,4,4], stats f64 [B,4] = (fitness, inlier rmse, updates, converged);
 *   pk_icp            blocking driver of the three: polls dev_count (int32, device) every `poll`
 *                     evaluations (one 4-byte read and a stream synchronisation each).
 * work: pk_icp_work_size(B, nsrc_max, ntgt_max) bytes, kept between the calls of one run. */
int64_t pk_icp_work_size(int B, int nsrc_max, int ntgt_max);
int pk_icp_init(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off,
                const double* T_init, int B, int nsrc_max, int ntgt_max, void* work, int64_t work_bytes, void* stream);
int pk_icp_iterate(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off,
                   double max_dist, int max_iter, double rel_fitness, double rel_rmse, int B, int nsrc_max,
                   int ntgt_max, int steps, void* work, int64_t work_bytes, int32_t* active_count, void* stream);
int pk_icp_result(const void* work, int B, double* T, double* stats, void* stream);
int pk_icp(const double* src, const int64_t* src_off, const double* tgt, const int64_t* tgt_off, const double* T_init,
           double max_dist, int max_iter, double rel_fitness, double rel_rmse, int B, int nsrc_max, int ntgt_max,
           int poll, void* work, int64_t work_bytes, int32_t* dev_count, double* T, double* stats, void* stream);

/* (f2) TEASER++ robust registration, the alternative pose solver (scripts/test_teaser.py:
 * 327-331, 362-435: RobustRegistrationSolver, cbar2 1, noise_bound 0.05, no scaling, GNC-TLS
 * rotation with gnc factor 1.4 / 100 iterations / cost threshold 1e-12; PMC_EXACT max clique with
 * the 0.5 k-core heuristic; CHAIN rotation TIMs). Restated from the public TEASER++ algorithm
 * (parity unpinned: teaserpp_python is absent).
 *   pk_teaser_graph (device): src / dst f64 [T,3] — the matched points (CAD side, crop side), packed
 *     by off [B+1] (device); adj uint64 [B][nmax][ceil(nmax/64)] (bit j of row i: pair (i, j)
 *     consistent: ||src_j - src_i| - |dst_j - dst_i|| <= beta, beta = 2 noise sqrt(cbar2));
 *     deg int32 [B][nmax] row degrees. Rows >= n_b are zero.
 *   pk_teaser_solve (HOST pointers only, blocking, `threads` host threads over crops): max clique
 *     (or the max k-core when its core number exceeds kcore_heuristic_threshold * n), GNC-TLS
 *     rotation over the chain TIMs of the sorted clique, adaptive-voting translation over the
 *     clique. T f64 [B,4,4] (identity when invalid), clique int32 [B][nmax] (sorted, clique_size
 *     [B] entries valid), info int32 [B][4] = (valid, clique mode: 1 exact / 0 node budget hit /
 *     2 k-core heuristic, rotation inliers, translation inliers). */
typedef struct pk_teaser_params {
  double noise_bound;                /* 0.05 */
  double cbar2;                      /* 1 */
  double rotation_gnc_factor;        /* 1.4 */
  double rotation_cost_threshold;    /* 1e-12 */
  double kcore_heuristic_threshold;  /* 0.5 */
  int32_t rotation_max_iterations;   /* 100 */
  int32_t pad;
  int64_t max_clique_nodes;          /* branch-and-bound node budget */
} pk_teaser_params;
int pk_teaser_graph(const double* src, const double* dst, const int64_t* off, int B, int nmax, double beta,
                    uint64_t* adj, int32_t* deg, void* stream);
int pk_teaser_solve(const double* src, const double* dst, const int64_t* off, int B, int nmax, const uint64_t* adj,
                    const int32_t* deg, const pk_teaser_params* params, int threads, double* T, int32_t* clique,
                    int32_t* clique_size, int32_t* info);

/* (f1) Spectral operators on the device (dataset/object.py:214, 246 -> upstream diffusion-net
 * geometry.compute_operators: robust_laplacian.point_cloud_laplacian for crops, potpourri3d
 * cotan_laplacian + vertex areas for the CAD mesh, scipy eigsh(L + eps I, 64, M, sigma = eps)).
 * Parity unpinned (those packages are absent); see csrc/operators.hip for the deviations.
 *   pk_knn           pts f64 [T,3] packed by off; idx int32 [T,k] (crop-local, ties to the lower
 *                    index; -1 when the crop has fewer points), d2 f64 [T,k] (may be NULL); k <= 32.
 *   pk_pc_local_tri  per point the Delaunay triangles of its tangent-plane neighbourhood incident to
 *                    it: tri int32 [T,k,2] (the other two corners, crop-local), ntri int32 [T],
 *                    normals f64 [T,3] (PCA; may be NULL).
 *   pk_cotan_dense   dense cotan Laplacian L f64 [B,nmax,nmax] (off-diagonal -sum cot/2, diagonal
 *                    = minus the row sum) and lumped mass f64 [B,nmax] (area / 3 per corner) of the
 *                    soup (tri / ntri / k) or of mesh faces (int32 [F,3] crop-local, packed by foff
 *                    [B+1], fmax >= every crop's face count); everything times `scale`.
 *   pk_sym_scale     A = D^-1/2 (L + eps I) D^-1/2 in place (D = diag(mass)); rows / columns past n_b
 *                    become pad_diag * I.
 *   pk_dgemm_cheb    out = alpha A Y + beta Y + gamma X (X may be NULL), A [B,n,n], X / Y / out [B,n,m].
 *   pk_dgemm_tn      G [B,m,m] = X^T Y. */
int pk_knn(const double* pts, const int64_t* off, int B, int nmax, int k, int omit_self, int32_t* idx, double* d2,
           void* stream);
int pk_pc_local_tri(const double* pts, const int64_t* off, int B, int nmax, const int32_t* knn, int k, int32_t* tri,
                    int32_t* ntri, double* normals, void* stream);
int pk_cotan_dense(const double* pts, const int64_t* off, int B, int nmax, const int32_t* tri, const int32_t* ntri,
                   int k, const int32_t* faces, const int64_t* foff, int fmax, double scale, double denom_eps,
                   double* L, double* mass, void* stream);
int pk_sym_scale(const int64_t* off, int B, int nmax, double eps, const double* mass, double pad_diag, double* A,
                 void* stream);
int pk_dgemm_cheb(const double* A, const double* Y, const double* X, int B, int n, int m, double alpha, double beta,
                  double gamma, double* out, void* stream);
int pk_dgemm_tn(const double* X, const double* Y, int B, int n, int m, double* G, void* stream);
/* Shift-invert support: pk_dpotrf factors A[b] + tau I = L L^T in place (lower triangle, blocked by
 * 64; fail int32 [B] = 1 where a pivot was not positive); pk_dpotrs solves X <- (L L^T)^-1 X in
 * place for X [B,n,m]. */
int pk_dpotrf(double* A, int B, int n, double tau, int32_t* fail, void* stream);
int pk_dpotrs(const double* L, double* X, int B, int n, int m, void* stream);
/* (f1) robust_laplacian.point_cloud_laplacian's intrinsic stage (replaces the third-party call at
 * the end of diffusion-net compute_operators, reached from dataset/object.py:246), HOST code, one
 * cloud per call: the soup tri int32 [ntri,3] (cloud-local; pk_pc_local_tri's fans as (center,
 * u, v) triples) over pts f64 [n,3] is mollified (mollify_factor x mean edge length), lifted to
 * its tufted cover, flipped to intrinsic Delaunay, and its cotan Laplacian / lumped mass scaled
 * by 1/6 (cover x soup multiplicity) returned as the distinct off-diagonal pairs i < j with the
 * weight w_ij (L = sum_ij w_ij (e_i - e_j)(e_i - e_j)^T; ii/jj int32 [cap], ww f64 [cap], sorted
 * by (i, j); nnz = their count — when nnz > cap nothing is written, call again with cap >= nnz;
 * 3 ntri always suffices) and mass f64 [n]; nflips (may be NULL) = the flips performed. */
int pk_tufted_laplacian(const double* pts, int64_t n, const int32_t* tri, int64_t ntri, double mollify_factor,
                        int64_t cap, int32_t* ii, int32_t* jj, double* ww, int64_t* nnz, double* mass,
                        int64_t* nflips);

/* pk_copy_rows: rows blocks of n floats from src (block stride ld_src floats) to dst (ld_dst):
 * the x half of torch.cat([x, message], dim=1) (modeling/dpfm.py:67) in the fused
 * AttentionalPropagation node's [B, 2C, N] buffer (rows = B, n = C N, ld_dst = 2 C N). */
int pk_copy_rows(float* dst, int64_t ld_dst, const float* src, int64_t ld_src, int64_t rows, int64_t n,
                 void* stream);

/* pk_transpose_cf_rows: channels-first items [C, N] (item b at src0 + b sb for b < B0, else at
 * src1 + (b - B0) sb) into one rows-layout buffer dst [B, N, C]; C in {16, 32, 64, 128}. The
 * refinement's first_lin backward (modeling/dpfm.py:98, desc = first_lin(x).transpose(1, 2)): the
 * two shapes' channels-first gradients of desc as the rows-layout dy of the layer. */
int pk_transpose_cf_rows(const float* src0, const float* src1, int B0, int B, int C, int N, int64_t sb,
                         float* dst, void* stream);

/* Runtime helpers of the pipelined executors (host only; no reference counterpart: the reference
 * overlaps crop formation with training through DataLoader worker PROCESSES, train.py /
 * dataset/object.py:117-274; here the overlap is two HIP streams on one device).
 *   pk_device_cu_count        the current device's CU count
 *   pk_stream_create_cu_mask  a stream restricted to the CUs of mask (bit i of word i/32 = CU i;
 *                             hipExtStreamCreateWithCUMask), released by pk_stream_destroy
 *   pk_stream_get_cu_mask     the mask a stream runs with */
int pk_device_cu_count(int* out);
int pk_stream_create_cu_mask(const uint32_t* mask, int words, void** stream);
int pk_stream_get_cu_mask(void* stream, int words, uint32_t* mask);
int pk_stream_destroy(void* stream);

/* pk_build_id: the library's build identity (no reference counterpart): writes the 64 hex digits
 * + NUL of the sha256 over the sources it was built from (the csrc .hip / .hpp / .cpp files, this header and the
 * Makefile, concatenated in sorted path order) into the HOST buffer out (cap >= 65). A test
 * recomputes the hash from the tree to prove the loaded binary is built from those sources. */
int pk_build_id(char* out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* POSEKERN_H */
