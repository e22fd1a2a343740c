"""ctypes binding of libposekern.so (the C-ABI declared in include/posekern.h).

The library is built in-tree by `make -C 6d-pose-estimation-for-unseen-categories_amd`
(or __graft_entry__.build()). There is no CPU fallback: if the library is missing or
a tensor is not on a HIP device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (loads torch's HIP runtime first so the library binds to it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libposekern.so")
# the same sources built with -DPK_DEVBUILD (development pkdev_* entry points, PK_* environment
# switches): loaded only by tests / tools that exercise a development hook, never by dpfm_amd
DEV_LIB_PATH = os.path.join(_HERE, "lib", "libposekern_dev.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_D = ctypes.c_double
_F = ctypes.c_float



class LinearArgs(ctypes.Structure):
    """pk_linear_args (include/posekern.h)."""
    _fields_ = [("x", _P), ("w", _P), ("bias", _P), ("layout", ctypes.c_int32), ("N", ctypes.c_int32),
                ("R", _I64), ("Cin", ctypes.c_int32), ("Cout", ctypes.c_int32), ("transw", ctypes.c_int32),
                ("act", ctypes.c_int32), ("mask", _P), ("ldx", _I64), ("y", _P), ("ldy", _I64), ("y2", _P),
                ("ldy2", _I64), ("split", ctypes.c_int32), ("store_cf", ctypes.c_int32), ("add", _P), ("lda", _I64),
                ("add_cols", ctypes.c_int32), ("pad", ctypes.c_int32), ("pre", _P), ("pre_out", _P),
                ("w2", _P), ("bias2", _P), ("wsplit", ctypes.c_int32), ("pad2", ctypes.c_int32), ("add2", _P),
                ("lda2", _I64)]


class OverlapHeadArgs(ctypes.Structure):
    """pk_overlap_head_args (include/posekern.h)."""
    _fields_ = [("x", _P * 2), ("strides", (_I64 * 3) * 2), ("N", ctypes.c_int32 * 2), ("B", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("w0", _P), ("b0", _P), ("w1", _P), ("b1", _P), ("n", _P * 2),
                ("nrm", _P * 2), ("nrows", _P * 2), ("h", _P * 2), ("s", _P * 2), ("ds", _P * 2), ("dnr", _P * 2),
                ("g", _P * 2), ("dh", _P * 2), ("dx", _P * 2), ("dadd", _P * 2)]


# name -> argtypes, mirroring include/posekern.h one for one.
SIGNATURES = {
    "pk_fps": [_P, _P, _I, _I, _P, _P, _P, _I, _P],
    "pk_ball_query_mask": [_P, _P, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P],
    "pk_ball_query_pairs": [_P, _P, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    "pk_backproject": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P],
    "pk_sor": [_P, _P, _I, _I, _I, _D, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "pk_fps_npoint": [_P, _I, _I, _I, _U64, _I64, _P, _P, _P, _P],
    "pk_gather_transform": [_P, _P, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    "pk_gather_transform_pad": [_P, _P, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P],
    "pk_collate_pad": [_P, _I, _I, _P, _I, _I, _P, _P, _P],
    "pk_segment_scan": [_P, _I, _I, _P, _P, _P],
    "pk_offsets_from_counts": [_P, _I, _P, _P],
    "pk_spectral_diffusion": [_P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _P],
    "pk_linear_ex": [_P, _P],
    "pk_linear_ex2": [_P, _P, _P],
    "pk_fmap_head_work_len": [_I, _I, _I],
    "pk_fmap_head_fwd": [_P, _I, _P, _P, _P, _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _I, _I, _I, _F, _P, _P, _P, _P,
                         _P, _P, _I64, _P],
    "pk_fmap_head_bwd": [_P, _P, _P, _P, _P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "pk_fmap_solve": [_P, _P, _P, _F, _I, _I, _P, _P],
    "pk_fmap_solve_backward": [_P, _P, _P, _F, _I, _I, _P, _P, _P, _P],
    "pk_attention_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I64, _I64, _P, _P, _P],
    "pk_attention_bwd": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I64, _I64, _P, _P, _P, _P, _I64, _I64, _P],
    "pk_linear_wgrad": [_P, _P, _I, _I64, _I, _I, _I, _P, _P, _P, _I, _P],
    "pk_linear_wgrad_grouped_work": [_P, _I],
    "pk_linear_wgrad_grouped": [_P, _I, _P, _I64, _P],
    "pk_nce_loss": [_P, _P, _P, _P, _I, _I64, _I64, _I, _P, _I, _P, _P, _I, _F, _I, _P, _P, _P, _P, _P, _P, _P],
    "pk_affine_cat": [_P, _I64, _P, _I64, _F, _F, _P, _P],
    "pk_loss_head": [_P, _P, _I, _I, _P, _P, _F, _F, _F, _P, _P, _P, _P],
    "pk_loss_scale": [_P, _P, _P, _P, _I, _P, _P],
    "pk_clip_rmsprop": [_P, _P, _P, _P, _P, _I, _F, _F, _F, _F, _F, _P, _P, _P],
    "pk_instnorm_relu_fwd": [_P, _I64, _I, _F, _P, _P, _P, _P],
    "pk_instnorm_relu_bwd": [_P, _P, _P, _P, _I64, _I, _P, _P],
    "pk_wbce": [_P, _P, _I, _P, _P, _I, _I, _P, _P, _P, _P],
    "pk_l2_normalize_fwd": [_P, _P, _I, _I, _I, _P, _P, _P, _P],
    "pk_l2_normalize_bwd": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P],
    "pk_overlap_head_fwd": [_P, _P],
    "pk_overlap_head_bwd": [_P, _P],
    "pk_mlp3_fwd": [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I, _P, _P, _P, _P, _P],
    "pk_resolvent_mask": [_P, _I, _P, _I, _I, _I, _F, _P, _P],
    "pk_linear_fwd": [_P, _P, _P, _I, _I64, _I, _I, _I, _I, _I, _P, _P, _P],
    "pk_feat_dist_work_size": [_I, _I, _I, _I, _I],
    "pk_attention_bwd_work_size": [_I, _I, _I, _I, _I],
    "pk_feat_dist_topk": [_P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _I64, _P, _P, _P],
    "pk_rigidity_filter_work_size": [_I, _I, _I],
    "pk_rigidity_filter": [_P, _I, _P, _P, _I, _P, _I, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "pk_inlier_ratio": [_P, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P, _P, _P],
    "pk_cgt_lstsq_work_size": [_I, _I, _I],
    "pk_nce_select": [_P, _I, _I64, _I, ctypes.c_uint64, _P, _P, _P, _P],
    "pk_cgt_lstsq": [_P, _I, _P, _P, _I, _I, _P, _I, _I, _I, _I, _P, _I, _P, _P, _P],
    "pk_ransac_work_size": [_I, _I64, _I],
    "pk_ransac": [_P, _P, _P, _P, _P, _P, _P, _P, _U64, _I64, _D, _I, _I, _P, _I64, _P, _P, _P, _P],
    "pk_pose_metrics": [_P, _P, _I, _I, _P, _P, _P, _P, _P],
    "pk_erode_mask": [_P, _I, _I, _I, _P, _P],
    "pk_sample_rgb": [_P, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P],
    "pk_sample_features": [_P, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P],
    "pk_icp_work_size": [_I, _I, _I],
    "pk_icp_init": [_P, _P, _P, _P, _P, _I, _I, _I, _P, _I64, _P],
    "pk_icp_iterate": [_P, _P, _P, _P, _D, _I, _D, _D, _I, _I, _I, _I, _P, _I64, _P, _P],
    "pk_icp_result": [_P, _I, _P, _P, _P],
    "pk_icp": [_P, _P, _P, _P, _P, _D, _I, _D, _D, _I, _I, _I, _I, _P, _I64, _P, _P, _P, _P],
    "pk_teaser_graph": [_P, _P, _P, _I, _I, _D, _P, _P, _P],
    "pk_knn": [_P, _P, _I, _I, _I, _I, _P, _P, _P],
    "pk_pc_local_tri": [_P, _P, _I, _I, _P, _I, _P, _P, _P, _P],
    "pk_cotan_dense": [_P, _P, _I, _I, _P, _P, _I, _P, _P, _I, _D, _D, _P, _P, _P],
    "pk_sym_scale": [_P, _I, _I, _D, _P, _D, _P, _P],
    "pk_dgemm_cheb": [_P, _P, _P, _I, _I, _I, _D, _D, _D, _P, _P],
    "pk_dgemm_tn": [_P, _P, _I, _I, _I, _P, _P],
    "pk_dpotrf": [_P, _I, _I, _D, _P, _P],
    "pk_dpotrs": [_P, _P, _I, _I, _I, _P],
    "pk_tufted_laplacian": [_P, _I64, _P, _I64, _D, _I64, _P, _P, _P, _P, _P, _P],
    "pk_teaser_solve": [_P, _P, _P, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P],  # host pointers
    "pk_transpose_cf_rows": [_P, _P, _I, _I, _I, _I, _I64, _P, _P],
    "pk_mean_f32": [_P, _I64, _P, _P],
    "pk_copy_rows": [_P, _I64, _P, _I64, _I64, _I64, _P],
    "pk_device_cu_count": [_P],
    "pk_stream_create_cu_mask": [_P, _I, _P],
    "pk_stream_get_cu_mask": [_P, _I, _P],
    "pk_stream_destroy": [_P],
    "pk_build_id": [_P, _I],  # host buffer
}

RESTYPES = {"pk_cgt_lstsq_work_size": _I64, "pk_linear_wgrad_grouped_work": _I64, "pk_ransac_work_size": _I64,
            "pk_feat_dist_work_size": _I64, "pk_fmap_head_work_len": _I64, "pk_icp_work_size": _I64,
            "pk_rigidity_filter_work_size": _I64, "pk_attention_bwd_work_size": _I64}  # everything else returns an int status

_lib: Optional[ctypes.CDLL] = None
_dev_lib: Optional[ctypes.CDLL] = None


class WgradCall(ctypes.Structure):
    """pk_wgrad_call (include/posekern.h)."""
    _fields_ = [("x", _P), ("dy", _P), ("dw", _P), ("db", _P), ("R", _I64), ("I", ctypes.c_int32),
                ("O", ctypes.c_int32), ("N", ctypes.c_int32), ("layout", ctypes.c_int32),
                ("accumulate", ctypes.c_int32), ("pad", ctypes.c_int32), ("sx", _I64), ("sdy", _I64)]


class TeaserParams(ctypes.Structure):
    """pk_teaser_params (include/posekern.h); defaults = scripts/test_teaser.py:357-364."""
    _fields_ = [("noise_bound", _D), ("cbar2", _D), ("rotation_gnc_factor", _D), ("rotation_cost_threshold", _D),
                ("kcore_heuristic_threshold", _D), ("rotation_max_iterations", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("max_clique_nodes", _I64)]


class PoseKernError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PoseKernError(
                f"libposekern.so not found at {LIB_PATH}: build it with "
                "`make -C 6d-pose-estimation-for-unseen-categories_amd` (no CPU fallback exists)")
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(l, name)
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _lib = l
    return _lib


def dev_lib() -> ctypes.CDLL:
    """libposekern_dev.so (pkdev_* hooks; the pk_* entry points bound as in lib()). Its kernels
    are its own copies: device buffers are shared, library state is not."""
    global _dev_lib
    if _dev_lib is None:
        if not os.path.exists(DEV_LIB_PATH):
            raise PoseKernError(f"libposekern_dev.so not found at {DEV_LIB_PATH}: `make -C "
                                "6d-pose-estimation-for-unseen-categories_amd`")
        l = ctypes.CDLL(DEV_LIB_PATH, mode=ctypes.RTLD_LOCAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(l, name)
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _dev_lib = l
    return _dev_lib


def use_dev_lib() -> None:
    """Route every dpfm_amd call of this process through libposekern_dev.so (tools/ only: the
    A/B and probe scripts toggle pkdev_* variants of the kernels ops.* launches)."""
    global _lib
    if _lib is not None and _lib is not dev_lib():
        raise PoseKernError("use_dev_lib() must run before the first library call")
    _lib = dev_lib()


_ERRORS = {1000: "invalid argument", 1001: "output capacity exceeded"}
_probe = None


def build_id(l: Optional[ctypes.CDLL] = None) -> str:
    """The sha256 the library was built from (pk_build_id)."""
    buf = ctypes.create_string_buffer(65)
    st = (l or lib()).pk_build_id(buf, 65)
    if st != 0:
        raise PoseKernError(f"pk_build_id failed: {st}")
    return buf.value.decode()


def tree_build_id() -> str:
    """The same hash recomputed from the source tree next to this package (the Makefile's recipe:
    its sorted ID_SRCS list, contents concatenated)."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    names = sorted([os.path.relpath(f, pkg) for pat in ("*.hip", "*.hpp", "*.cpp")
                    for f in glob.glob(os.path.join(pkg, "csrc", pat))] + ["../include/posekern.h", "Makefile"])
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(pkg, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def set_probe(hook) -> None:
    """Install hook(name, thunk, work) around every call (bench.py's per-kernel HIP events).
    `work` is the launch's algorithmic work ("hbm", bytes) / ("mfma", flops) or None."""
    global _probe
    _probe = hook


def call(name: str, *args, work=None) -> None:
    fn = getattr(lib(), name)
    status = _probe(name, lambda: fn(*args), work) if _probe is not None else fn(*args)
    if status != 0:
        msg = _ERRORS.get(status, f"hipError_t {status}")
        raise PoseKernError(f"{name} failed: {msg}")


def ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise PoseKernError("posekern ops take HIP device tensors only (no CPU fallback)")
    if not t.is_contiguous():
        raise PoseKernError("posekern ops need contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
