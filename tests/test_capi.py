"""CPU: the C-ABI library loads and exports every symbol include/webpgpu.h
declares (no compute calls without a GPU), the Python mirror binds them, and
argument validation rejects bad shapes without touching the device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "webpgpu.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(wg_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert len(syms) >= 20, syms


def test_library_exports_every_declared_symbol():
    from webp_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from webp_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_invalid_arguments_are_rejected_without_gpu():
    from webp_amd import _lib
    lib = _lib.lib
    assert lib.wg_decode_frames(None, None, 2, 1, 1, 1, None, None, None, None, None) == -1
    assert b"invalid argument" in lib.wg_last_error()
    assert lib.wg_import_rgba(None, 0, 0, 0, 0, 0, None, None, None, 0, 0, 1, None) == -1
    assert lib.wg_transform(9, None, 0, None, 0, 1, None) == -1
    assert lib.wg_filter(12, None, 0, 0, 0, 0, None, None, None, 1, None) == -1
    assert lib.wg_encode_row_order(None, 120, 68, 1, None, None) == -1
    assert lib.wg_encode_frames_devices(None, 1, None, 64, 64, 1, 0, None, None, None, None, None, None, None) == -1
    assert lib.wg_plane_ssim_devices(None, 1, None, 8, None, 8, 8, 8, None) == -1
    assert lib.wg_decode_kernel(0, 1) == -1 and lib.wg_decode_kernel(68, 0) == -1


def test_work_size_helpers():
    from webp_amd import _lib
    # top records | ctl[4] | reconstruction progress | filter progress (k_decode_split), 16-B aligned
    # | one 128-B bottom-rows record per MB column (a band's hand-off to the next band)
    head = 2 * 120 * 32 + 4 * (2 * 2 * 68 + 4)
    assert _lib.lib.wg_decode_work_bytes(120, 68, 2) == ((head + 15) & ~15) + 2 * 120 * 128
    assert _lib.lib.wg_decode_work_bytes(0, 68, 2) == 0
    # ctl (16 B) | one {pixel, tag} granule per column of each band's last row
    assert _lib.lib.wg_vp8l_inverse_work_bytes(100, 130, 2) == 16 + 8 * 2 * 5 * 100  # 32-row bands
    assert _lib.lib.wg_vp8l_inverse_work_bytes(100, 0, 2) == 0
    assert _lib.lib.wg_plane_ssim_work_bytes(33, 17, 1) == 8 * 1 * 2  # one 58-column strip, two tile rows
    assert _lib.lib.wg_plane_ssim_row_partials(59) == 2 and _lib.lib.wg_plane_ssim_row_partials(58) == 1
    # hand-off records (128 B a column: 11 {word, tag} granules) | ctl[4] | row-schedule tag[4] | row order |
    # slack | band order (17 bands of 4 rows per frame) (wg_encode_row_order)
    assert _lib.lib.wg_encode_work_bytes(120, 68, 2) == 2 * 120 * 128 + 4 * 4 + 4 * (4 + 2 * 68 + 2 + 2 * 17)
    assert _lib.lib.wg_encode_work_bytes(120, 0, 2) == 0


def test_library_is_gfx950_only():
    """The shipped code object targets gfx950 and nothing else."""
    from webp_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert other not in blob


@pytest.mark.parametrize("mod", ["webp_amd.dsp", "webp_amd.frames"])
def test_modules_import(mod):
    __import__(mod)


def test_encode_refuses_small_frames_and_bad_alignment():
    """wg_encode_mbs returns WG_EINVAL before any device work for mbh < 4
    (encode.go:1356 encodes those serially) and for misaligned buffers."""
    from webp_amd import _lib
    lib = _lib.lib
    p = 1 << 20  # never dereferenced: validation fails first
    args = lambda w, h, out: (p, p, p, 256 * 8 * 8, 64 * 8 * 8, w, h, 1, None, p, 0, p, 4, 75, out, p, p, p, p, None)
    assert lib.wg_encode_mbs(*args(64, 48, p)) == -1
    assert b"mbh >= 4" in lib.wg_last_error()
    assert lib.wg_encode_mbs(*args(64, 64, p + 8)) == -1  # out not 16-byte aligned
    assert lib.wg_encode_mbs(*(args(64, 64, p)[:3] + (100,) + args(64, 64, p)[4:])) == -1  # y pitch too small


def test_segment_analysis_validates_without_gpu():
    from webp_amd import _lib, frames
    lib = _lib.lib
    cfg = frames.encoder_config()
    p = 1 << 20
    assert lib.wg_segment_analysis(cfg.ctypes.data, p, p, 0, 4, 1, p, p, 896, None, None) == -1
    assert lib.wg_segment_analysis(cfg.ctypes.data, p, p, 4, 4, 1, p, p, 100, None, None) == -1  # pitch < 4 segments
    assert lib.wg_encoder_config(101, 4, 50, 60, 0, 1, 4, 0, cfg.ctypes.data) == -1
