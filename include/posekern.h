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
 *   out    int64 [B, out_stride]; row b holds npoint[b] indices local to crop b
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
 *   ov12 int8 [B, n1max], ov21 int8 [B, n2max] (either may be NULL) */
int pk_ball_query_pairs(const double* cad, const int64_t* cad_off, const double* pc,
                        const int64_t* pc_off, const double* thr2, int B, int n1max, int n2max,
                        const uint8_t* mask, int ld, const int32_t* rowcount, int64_t* rowoff,
                        int64_t* pairs, int64_t cap, int64_t* count, int8_t* ov12, int8_t* ov21,
                        void* stream);

/* H1 crop formation. Replaces dataset/object.py:73-88 dpt_2_pcld (with the plus-shaped
 * erode_seg_mask of :52-71 and `seg == 255` of :137) for F frames at once.
 *   depth uint16 [F,H,W], mask uint8 [F,H,W] (mask_visib png values; 255 = object)
 *   K f64 [F,9] row-major intrinsics, cam_scale f32 [F] = 1000 / depth_scale
 *   rowcnt int32 [F,H], rowoff int64 [F,H] scratch
 *   count int64 [F] points per frame, off int64 [F+1] packed offsets
 *   xyz f64 [cap,3] packed back-projected points in cm, row-major pixel order.
 * Bit-exact vs numpy: z32 = f32(depth)/f32(cam_scale); X = (((u-cx)*z)/fx)*100. */
int pk_backproject(const uint16_t* depth, const uint8_t* mask, int F, int H, int W,
                   const double* K, const float* cam_scale, int32_t* rowcnt, int64_t* rowoff,
                   int64_t* count, int64_t* off, double* xyz, int64_t cap, void* stream);

/* H2 statistical outlier removal. Replaces dataset/object.py:33-50 remove_outliers
 * (Open3D RemoveStatisticalOutliers(nb_neighbors=20, std_ratio=0.3)).
 *   xyz f64 [T,3] packed / off, knn <= 20
 *   avg f64 [T] mean kNN distance, thr f64 [B] keep threshold
 *   ccount int32 [B, ceil(nmax/1024)], coff int64 (same shape) scratch
 *   kept int64 [B] survivors, out_off int64 [B+1] their packed offsets
 *   out64 f64 [T,3], out32 f32 [T,3] (either may be NULL) survivors in input order
 *   kept_idx int64 [T] (may be NULL) survivor index within its input crop */
int pk_sor(const double* xyz, const int64_t* off, int B, int nmax, int knn, double std_ratio,
           double* avg, double* thr, int32_t* ccount, int64_t* coff, int64_t* kept,
           int64_t* out_off, double* out64, float* out32, int64_t* kept_idx, void* stream);

/* FPS sample-count policy of dataset/object.py:145-147 on device counts (no host sync):
 * fixed > 0: npoint = fixed; else npoint = int(limit/n * n) if n > limit, else -n
 * (negative = keep all n points, no FPS). start[b] = splitmix64(seed ^ splitmix64(b))
 * % n (replaces upstream torch.randint; may be NULL). out_off int64 [B+1]. */
int pk_fps_npoint(const int64_t* off, int B, int fixed, int limit, uint64_t seed,
                  int32_t* npoint, int32_t* start, int64_t* out_off, void* stream);

/* H4 pcd[idx0] (dataset/object.py:148) + transform(pcd, R, t, inv=True) (:174, :304-309).
 *   pcd f64 [T,3] packed / off; idx int64 [B, idx_stride] FPS output (unused when
 *   npoint[b] < 0); R f64 [B,9] row-major R_m2c, t f64 [B,3] (cm)
 *   sel64 f64 / align64 f64 / sel32 f32 [sum npoint, 3] packed by out_off (any NULL) */
int pk_gather_transform(const double* pcd, const int64_t* off, int B, const int64_t* idx,
                        int idx_stride, const int32_t* npoint, int npmax, const int64_t* out_off,
                        const double* R, const double* t, double* sel64, double* align64,
                        float* sel32, void* stream);

/* Packed-layout helpers: per-segment exclusive scan of int32 counts (S segments of n),
 * and off[b+1] = off[b] + counts[b]. */
int pk_segment_scan(const int32_t* cnt, int S, int n, int64_t* off, int64_t* total, void* stream);
int pk_offsets_from_counts(const int64_t* counts, int B, int64_t* off, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POSEKERN_H */
