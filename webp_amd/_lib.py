"""ctypes binding of webp_amd/libwebpgpu.so (the C ABI in include/webpgpu.h).

The library is built in-tree for gfx950 (``make -C webp_amd``).  There is no
fallback: if the shared object is missing or a call fails, an exception is
raised.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WEBPGPU_LIB", os.path.join(_HERE, "libwebpgpu.so"))


class WebpGpuError(RuntimeError):
    pass


def _load():
    # torch first: libwebpgpu.so and torch must share one HIP runtime.  Loaded
    # before torch, the library pulls in /opt/rocm's libamdhip64 and torch then
    # binds to that copy instead of its own, after which the library saw no HIP
    # device (hipGetDevice failed in a pytest run that imported a test module
    # using webp_amd before any module imported torch).
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise WebpGpuError(
            f"{LIB_PATH} not found: build it with `make -C webp_amd` (hipcc --offload-arch=gfx950); "
            "webp_amd has no CPU fallback")
    return ctypes.CDLL(LIB_PATH)


lib = _load()

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64

# name -> argtypes (all return int status unless listed in _RES)
SIGNATURES = {
    "wg_last_error": [],
    "wg_version": [],
    "wg_device_check": [],
    "wg_pred_luma4": [_vp, _vp, _i64, _vp, _i32, _i32, _vp],
    "wg_pred_luma16": [_vp, _vp, _i64, _vp, _i32, _i32, _vp],
    "wg_pred_chroma8": [_vp, _vp, _i64, _vp, _i32, _i32, _vp],
    "wg_transform": [_i32, _vp, _i64, _vp, _i64, _i32, _vp],
    "wg_transform_wht": [_vp, _vp, _i32, _vp],
    "wg_ftransform_wht": [_vp, _vp, _i32, _vp],
    "wg_itransform": [_vp, _vp, _vp, _i64, _i32, _i32, _vp],
    "wg_ftransform": [_vp, _vp, _i64, _vp, _i32, _i32, _vp],
    "wg_metric": [_i32, _vp, _vp, _i64, _vp, _i32, _vp],
    "wg_ssim_get": [_vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp],
    "wg_filter": [_i32, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _i32, _vp],
    "wg_upsample_line_pairs": [_i32, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _i32,
                               _i32, _vp],
    "wg_debug_inject_timeout": [_i32, _vp],
    "wg_point_sample_rows": [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _i32, _i32, _vp],
    "wg_convert_argb_to_y": [_vp, _i64, _vp, _i64, _i32, _i32, _vp],
    "wg_convert_argb_to_uv": [_vp, _i64, _vp, _vp, _i64, _i32, _i32, _i32, _vp],
    "wg_accumulate_rgba": [_vp, _vp, _vp, _vp, _i32, _i64, _vp, _i64, _i32, _i32, _vp],
    "wg_convert_rgba32_to_uv": [_vp, _i64, _vp, _vp, _i64, _i32, _i32, _vp],
    "wg_random_init_host": [_vp, ctypes.c_float],
    "wg_convert_rgba32_to_uv_dithered": [_vp, _i64, _vp, _vp, _i64, _i32, _vp, _i32, _vp],
    "wg_sse_planes": [_vp, _vp, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i32, _vp],
    "wg_psnr_from_sse": [_vp, _vp, _vp, _i32, _vp],
    "wg_disto_stats_blocks": [_vp, _vp, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i32, _vp],
    "wg_ssim_from_stats": [_vp, _i32, _vp, _i32, _vp],
    "wg_decode_work_bytes": [_i32, _i32, _i32],
    "wg_decode_frames": [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp],
    "wg_vp8_parse": [_vp, ctypes.c_size_t, _vp, _vp, _vp, _i64],
    "wg_decode_status": [_vp, _i32, _i32, _vp],
    "wg_decode_kernel": [_i32, _i32],
    "wg_import_rgba": [_vp, _i32, _i32, _i32, _i64, _i32, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "wg_dither_amp": [ctypes.c_float, _i32],
    "wg_dither_plan_bytes": [_i32, _i32],
    "wg_dither_plan": [_i32, _i32, _vp, _vp],
    "wg_dither_plan_host": [_i32, _i32, _vp],
    "wg_import_rgba_dithered": [_vp, _i32, _i32, _i32, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "wg_analysis_alphas": [_vp, _vp, _vp, _i32, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp],
    "wg_upsample_nrgba": [_vp, _i32, _i64, _vp, _vp, _i32, _i64, _vp, _i64, _i32, _i32, _vp, _i64, _i32, _vp],
    "wg_plane_ssim_work_bytes": [_i32, _i32, _i32],
    "wg_plane_ssim_row_partials": [_i32],
    "wg_plane_ssim_rows": [_vp, _i32, _i64, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp],
    "wg_plane_ssim_reduce": [_vp, _i64, _i32, _vp, _vp],
    "wg_plane_ssim": [_vp, _i32, _i64, _vp, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp],
    "wg_vp8l_residual_image_rows": [_vp, _i32, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp],
    "wg_vp8l_residual_image": [_vp, _i32, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp],
    "wg_vp8l_inverse_work_bytes": [_i32, _i32, _i32],
    "wg_vp8l_inverse_predictor": [_vp, _i32, _i32, _i32, _i64, _i32, _vp, _vp, _vp, _vp],
    "wg_vp8l_inverse_status": [_vp, _vp],
    "wg_vp8l_green": [_vp, _i64, _i32, _vp],
    "wg_vp8l_slog2_lut_host": [_vp, _i32],
    "wg_vp8l_color_space_transform": [_vp, _i32, _i32, _i64, _i32, _i32, _vp, _vp],
    "wg_vp8l_color_space_inverse": [_vp, _i32, _i32, _i32, _i64, _i32, _vp, _vp, _vp],
    "wg_vp8l_color_index_inverse": [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp],
    "wg_alpha_filter": [_i32, _vp, _vp, _i32, _i32, _i64, _i32, _vp],
    "wg_alpha_unfilter_work_bytes": [_i32, _i32, _i32],
    "wg_alpha_unfilter": [_i32, _vp, _i32, _i32, _i64, _i32, _vp, _vp],
    "wg_alpha_unfilter_status": [_vp, _vp],
    "wg_alpha_estimate_work_bytes": [_i32],
    "wg_alpha_estimate_filter": [_vp, _i32, _i32, _i64, _i32, _vp, _vp, _vp, _vp],
    "wg_apply_alpha_multiply": [_vp, _i32, _i32, _i32, _i32, _i64, _i32, _i32, _vp],
    "wg_mult_argb": [_vp, _i64, _i32, _vp],
    "wg_apply_alpha_multiply_4444": [_vp, _i32, _i32, _i32, _i64, _i32, _vp],
    "wg_dispatch_alpha": [_vp, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _vp],
    "wg_extract_alpha": [_vp, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _vp],
    "wg_has_alpha": [_vp, _i64, _i32, _vp, _vp],
    "wg_alpha_replace": [_vp, _i64, ctypes.c_uint32, _vp],
    "wg_dispatch_alpha_to_green": [_vp, _i32, _i32, _i32, _vp, _i32, _vp],
    "wg_extract_green": [_vp, _vp, _i64, _vp],
    "wg_pack_rgb": [_vp, _vp, _vp, _i64, _i32, _vp, _vp],
    "wg_rescaler_plan_bytes": [_i32, _i32],
    "wg_rescaler_plan_host": [_i32, _i32, _i32, _i32, _vp, _vp],
    "wg_rescaler_plan": [_i32, _i32, _i32, _i32, _vp, _vp, _vp],
    "wg_rescale": [_vp, _i32, _i32, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _vp],
    "wg_sharpyuv_work_bytes": [_i32, _i32, _i32],
    "wg_sharpyuv_convert": [_vp, _i32, _i32, _i32, _i64, _vp, _i32, _vp, _i32, _i64, _vp, _vp, _i32, _i64, _vp, _vp],
    "wg_sharpyuv_tables_host": [_vp, _vp],
    "wg_sharpyuv_convert_ex": [_vp, _i32, _i32, _i32, _i64, _vp, _i32, _i32, _i32, _vp, _i32, _i64, _vp, _vp, _i32,
                               _i64, _vp, _vp],
    "wg_sharpyuv_transfer_tables_host": [_i32, _vp, _vp, _vp],
    "wg_sharpyuv_iterations": [_vp, _i32, _i32, _i32, _vp, _vp],
    "wg_setup_segment": [_i32, _vp, _i32, _i32, _vp],
    "wg_encode_work_bytes": [_i32, _i32, _i32],
    "wg_encode_mbs": [_vp, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _i32, _i32, _vp, _vp, _vp, _vp,
                      _vp, _vp],
    "wg_fixed_costs_i4_host": [_vp],
    "wg_encoder_config": [_i32] * 8 + [_vp],
    "wg_segment_analysis": [_vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i64, _vp, _vp],
    "wg_encode_status": [_vp, _i32, _i32, _vp],
    "wg_encode_row_order": [_vp, _i32, _i32, _i32, _vp, _vp],
    "wg_encode_frames_devices": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "wg_vp8l_residual_image_devices": [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp],
    "wg_plane_ssim_devices": [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _i32, _vp],
}
_RES = {"wg_last_error": ctypes.c_char_p, "wg_decode_work_bytes": ctypes.c_size_t,
        "wg_plane_ssim_work_bytes": ctypes.c_size_t, "wg_vp8l_inverse_work_bytes": ctypes.c_size_t,
        "wg_sharpyuv_work_bytes": ctypes.c_size_t, "wg_encode_work_bytes": ctypes.c_size_t,
        "wg_alpha_unfilter_work_bytes": ctypes.c_size_t, "wg_alpha_estimate_work_bytes": ctypes.c_size_t,
        "wg_rescaler_plan_bytes": ctypes.c_size_t, "wg_dither_plan_bytes": ctypes.c_size_t,
        "wg_dither_amp": ctypes.c_int32, "wg_random_init_host": None}

for _name, _args in SIGNATURES.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = _RES.get(_name, ctypes.c_int)

ABI_VERSION = 2  # WG_ABI_VERSION of include/webpgpu.h this binding is written against
if lib.wg_version() != ABI_VERSION:
    raise WebpGpuError(f"{LIB_PATH}: ABI version {lib.wg_version()}, this binding needs {ABI_VERSION} (rebuild it)")


def check(rc, what=""):
    if rc != 0:
        msg = lib.wg_last_error().decode(errors="replace")
        raise WebpGpuError(f"{what or 'webpgpu call'} failed (status {rc}): {msg}")
    return rc


def call(name, *args):
    """Invoke a status-returning entry point and raise on failure."""
    return check(getattr(lib, name)(*args), name)
