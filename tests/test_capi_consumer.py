"""A compiled C consumer of the ABI (VERDICT r03 missing 3): tests/capi_consumer.c
is built with gcc against include/webpgpu.h and linked to
webp_amd/libwebpgpu.so, as cgo would build INTEGRATION.md's preambles.

CPU: the host-only entry points and argument validation, compared with the
Python binding of the same library (and the parse with the one the GPU tests
use).  GPU: INTEGRATION.md's ITransform override and decodeFrameHIP call
sequences through hipMalloc'd buffers, checked against the oracle."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "capi_consumer.c")
LIBDIR = os.path.join(ROOT, "webp_amd")
FIXTURE = os.path.join(ROOT, "tests", "golden", "libwebp_decode.npz")


def build(tmp_path, gpu):
    exe = str(tmp_path / ("capi_gpu" if gpu else "capi_cpu"))
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"), SRC,
           "-L" + LIBDIR, "-lwebpgpu", "-Wl,-rpath," + LIBDIR, "-o", exe]
    if gpu:  # hip_runtime_api.h is C (not pedantic C99); the GPU mode allocates device memory as the Go side does
        cmd[1:1] = ["-DWG_WITH_HIP", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        cmd += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    else:  # the header and the consumer alone: strict C99
        cmd.insert(2, "-pedantic")
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-3000:]
    return exe


def fnv(b):
    h = 1469598103934665603
    for x in bytes(b):
        h = ((h ^ x) * 1099511628211) & (2**64 - 1)
    return h


def stream_file(tmp_path, name="parts"):
    data = np.load(FIXTURE)["v_%s_webp" % name].tobytes()
    p = tmp_path / (name + ".webp")
    p.write_bytes(data)
    return str(p), data


def test_c_consumer_cpu_paths(tmp_path):
    from webp_amd import _lib, frames
    exe = build(tmp_path, gpu=False)
    path, data = stream_file(tmp_path)
    p = subprocess.run([exe, "cpu", path], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, (p.stdout, p.stderr)
    kv = dict(ln.split("=", 1) for ln in p.stdout.splitlines() if "=" in ln)
    assert kv["fails"] == "0"
    assert int(kv["decode_work_bytes"]) == _lib.lib.wg_decode_work_bytes(120, 68, 2)
    assert int(kv["encode_work_bytes"]) == _lib.lib.wg_encode_work_bytes(120, 68, 64)
    seg = frames.setup_segment(30)
    assert int(kv["segment_fnv"]) == fnv(seg.tobytes())
    assert int(kv["fixed_i4_fnv"]) == fnv(frames.fixed_costs_i4().astype("<u2").tobytes())
    dims, mb, co = frames.vp8_parse(data)
    assert kv["dims"] == ",".join(str(dims[k]) for k in ("width", "height", "filter_type", "mbw", "mbh"))
    assert int(kv["mb_fnv"]) == fnv(mb.tobytes()) and int(kv["coeffs_fnv"]) == fnv(co.tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["parts", "q10"])
def test_c_consumer_gpu_sequences(cuda, tmp_path, name):
    from webp_amd import frames
    exe = build(tmp_path, gpu=True)
    path, data = stream_file(tmp_path, name)
    out = tmp_path / "out.bin"
    p = subprocess.run([exe, "gpu", path, str(out)], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, (p.stdout, p.stderr)
    raw = np.frombuffer(out.read_bytes(), np.uint8)
    ysz = 17 * 32 + 9 * 32  # WG_YUV_SIZE
    ref, coef, got = raw[:ysz], raw[ysz:ysz + 64].view(np.int16), raw[ysz + 64:2 * ysz + 64]
    exp = ref.copy()
    # ITransform(ref, in, dst, doTwo=true) with ref == dst at offset 0 (dsp_hip.go)
    O.lib.or_itransform(O.u8(exp), O.i16(np.ascontiguousarray(coef)), O.u8(exp), 1)
    assert (got == exp).all()
    dims, mb, co = frames.vp8_parse(data)
    mbw, mbh = dims["mbw"], dims["mbh"]
    planes = raw[2 * ysz + 64:]
    Y = planes[:256 * mbw * mbh].reshape(16 * mbh, 16 * mbw)
    U = planes[256 * mbw * mbh:320 * mbw * mbh].reshape(8 * mbh, 8 * mbw)
    V = planes[320 * mbw * mbh:].reshape(8 * mbh, 8 * mbw)
    eY, eU, eV = O.decode_frame(mb, co, dims["filter_type"], mbw, mbh)
    assert (Y == eY).all() and (U == eU).all() and (V == eV).all()
    assert hashlib.sha256(Y.tobytes()).hexdigest() == hashlib.sha256(eY.tobytes()).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,kind,q,method", [(96, 80, "noise", 75, 4), (200, 72, "blobs", 40, 6),
                                               (64, 64, "grad", 90, 3)])
def test_c_consumer_encode_sequence(cuda, tmp_path, w, h, kind, q, method):
    """INTEGRATION.md's encodeFramePhaseAHIP over the whole device encode path
    (wg_encoder_config -> wg_import_rgba -> wg_analysis_alphas ->
    wg_segment_analysis -> wg_encode_row_order -> wg_encode_mbs ->
    wg_encode_status), driven from C through hipMalloc'd buffers as cgo would:
    every wg_mb_enc field, the reconstruction, the segment ids and the frame
    record equal the oracle's EncodeFrame up to Phase A."""
    from tools import synth
    from webp_amd import frames
    exe = build(tmp_path, gpu=True)
    gen = {"noise": lambda: synth.noise_rgba(w, h, seed=w), "blobs": lambda: synth.blobs_rgba(w, h, seed=h),
           "grad": lambda: synth.gradient_rgba(w, h)}[kind]
    rgba = np.ascontiguousarray(gen()[..., :4]).copy()
    rgba[..., 3] = 255
    proba = O.default_proba()
    frame = tmp_path / "frame.bin"
    frame.write_bytes(np.array([w, h, q, method], "<i4").tobytes() + rgba.tobytes() + proba.tobytes())
    out = tmp_path / "enc.bin"
    p = subprocess.run([exe, "encode", str(frame), str(out)], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, (p.stdout, p.stderr)
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    nmb = mbw * mbh
    raw = np.frombuffer(out.read_bytes(), np.uint8)
    k = nmb * frames.MB_ENC_DTYPE.itemsize
    got = raw[:k].view(frames.MB_ENC_DTYPE)
    ysz, uvsz = 256 * nmb, 64 * nmb
    ry = raw[k:k + ysz].reshape(16 * mbh, 16 * mbw)
    ru = raw[k + ysz:k + ysz + uvsz].reshape(8 * mbh, 8 * mbw)
    rv = raw[k + ysz + uvsz:k + ysz + 2 * uvsz].reshape(8 * mbh, 8 * mbw)
    ids = raw[k + ysz + 2 * uvsz:k + ysz + 2 * uvsz + nmb]
    info = raw[k + ysz + 2 * uvsz + nmb:].view(frames.FRAME_SEGS_DTYPE)[0]
    Y, U, V = O.import_rgba(rgba, has_alpha=False)
    enc, (ey, eu, ev), e_ids, e_info = O.encode_frame(Y, U, V, w, h, O.encoder_config(quality=q, method=method))
    assert (ids == e_ids).all()
    for f in ("num_segments", "base_quant", "filter_level", "quant", "fstrength", "update_map"):
        assert (info[f] == e_info[f]).all(), f
    for f in frames.MB_ENC_DTYPE.names:
        if f != "pad":
            assert (got[f] == enc[f]).all(), f
    # (the luma reconstruction is exported inside the image only, as the
    # Python-path tests compare it: exportParallel's rows / columns)
    assert (ry[:h, :w] == ey[:h, :w]).all() and (ru == eu).all() and (rv == ev).all()
