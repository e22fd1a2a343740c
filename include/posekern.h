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

#ifdef __cplusplus
}
#endif
#endif /* POSEKERN_H */
