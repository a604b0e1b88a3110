"""Run in a fresh process by tests/test_gpu_concurrency.py (never imported by
pytest itself).

mode "race": the ABI used the way the reference is used concurrently
(race_test.go:33 TestConcurrentEncodeDeterminism, :137-193 the concurrent
encode / decode races; SURVEY 8(b): <= 6 row workers call the functions at
once).  Six host threads, each with its own HIP stream, make the process's
FIRST library calls at the same moment -- so the encoder's one-time constant
table upload (encode_rd.hip g_tables_mu), the decoder's launch configuration,
the gamma tables (wg_yuv.h call_once) and the device's timeout record
(runtime.hip diag_words) are all initialised under the race -- and repeat
them: wg_encode_mbs (through encode_frames: import -> analysis -> segments ->
row order -> Phase A, status checked), wg_decode_frames (+ status) and
wg_upsample_nrgba.  Afterwards the same jobs run serially on the default
stream; every output must be byte-identical to its serial run.

mode "diag": the *_status report of a timed-out wait: an
injected timeout is reported by the next status call of its kernel family
only, and later clean launches report WG_OK again.

Prints one JSON line; exit status 0 iff every check passed."""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

THREADS = 6
REPEATS = 3


def enc_input(k):
    """two 160x96 frames per job: a gradient and seeded noise (mbh 6 >= 4)"""
    h, w = 96, 160
    y, x = np.mgrid[0:h, 0:w]
    a = np.empty((h, w, 4), np.uint8)
    a[..., 0], a[..., 1], a[..., 2], a[..., 3] = (x + 7 * k) % 256, (y * 3) % 256, (x + y) % 256, 255
    b = np.random.default_rng(k).integers(0, 256, (h, w, 4), dtype=np.uint8)
    b[..., 3] = 255
    return np.stack([a, b])


def job_encode(k):
    from webp_amd import frames
    rgba = torch.from_numpy(enc_input(k)).cuda()

    def run():
        out, rec, seg_ids, _, _ = frames.encode_frames(rgba)  # check=True: status after Phase A
        return [out, rec[0], rec[1], rec[2], seg_ids]
    return run


def job_decode(k):
    from webp_amd import frames
    fx = np.load(os.path.join(ROOT, "tests", "golden", "libwebp_decode.npz"))
    names = sorted(n[2:-5] for n in fx.files if n.endswith("_webp"))
    dims, mb, co = frames.vp8_parse(fx["v_%s_webp" % names[k % len(names)]].tobytes())
    mbi = frames.mb_info_tensor(mb)
    cof = torch.from_numpy(co).cuda()

    def run():
        Y, U, V = frames.decode_frames(mbi, cof, dims["filter_type"], dims["mbw"], dims["mbh"], check=True)
        return [Y, U, V]
    return run


def job_upsample(k):
    from webp_amd import frames
    r = np.random.default_rng(100 + k)
    w, h = 333 + k, 201 + 2 * k
    Y = torch.from_numpy(r.integers(0, 256, (1, h, w), dtype=np.uint8)).cuda()
    U = torch.from_numpy(r.integers(0, 256, (1, (h + 1) // 2, (w + 1) // 2), dtype=np.uint8)).cuda()
    V = torch.from_numpy(r.integers(0, 256, (1, (h + 1) // 2, (w + 1) // 2), dtype=np.uint8)).cuda()

    def run():
        return [frames.build_nrgba(Y, U, V, w, h)]
    return run


JOBS = [job_encode, job_decode, job_upsample]


def race():
    # inputs are made (and moved to the device) before any library call; the
    # threads' first calls into libwebpgpu.so happen together at the barrier
    runs = [JOBS[k % 3](k) for k in range(THREADS)]
    torch.cuda.synchronize()
    start = threading.Barrier(THREADS)
    results, errors = [None] * THREADS, []

    def worker(k):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                torch.zeros(64, device="cuda")  # the stream's first kernel (webpgpu.h: queues before persistent kernels)
                s.synchronize()
                start.wait()
                outs = []
                for _ in range(REPEATS):
                    outs.append([t.clone() for t in runs[k]()])
                s.synchronize()
            results[k] = [[t.cpu().numpy() for t in o] for o in outs]
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            errors.append(f"thread {k}: {type(e).__name__}: {e}")

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(THREADS)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    mismatches = []
    if not errors:
        for k in range(THREADS):
            serial = [t.cpu().numpy() for t in runs[k]()]
            for rep, got in enumerate(results[k]):
                for j, (a, b) in enumerate(zip(got, serial)):
                    if a.shape != b.shape or not np.array_equal(a, b):
                        mismatches.append((k, rep, j))
    ok = not errors and not mismatches
    print(json.dumps({"mode": "race", "ok": ok, "threads": THREADS, "repeats": REPEATS, "errors": errors,
                      "mismatches": mismatches}), flush=True)
    return ok


def diag():
    from webp_amd import frames
    from webp_amd._lib import WebpGpuError, call
    stream = torch.cuda.current_stream().cuda_stream
    rgba = torch.from_numpy(enc_input(1)).cuda()
    frames.encode_frames(rgba)  # clean: status OK
    checks = {}
    call("wg_debug_inject_timeout", 0, stream)  # one timed-out encoder wait
    mbw, mbh, n = 10, 6, 2
    w = torch.zeros(frames.lib.wg_encode_work_bytes(mbw, mbh, n), dtype=torch.uint8, device="cuda")
    # a decode status is not affected by an encoder timeout
    fx = np.load(os.path.join(ROOT, "tests", "golden", "libwebp_decode.npz"))
    dims, mb, co = frames.vp8_parse(fx["v_q10_webp"].tobytes())
    frames.decode_frames(frames.mb_info_tensor(mb), torch.from_numpy(co).cuda(), dims["filter_type"], dims["mbw"],
                         dims["mbh"], check=True)
    checks["decode_unaffected"] = True
    try:
        frames.encode_status(w, mbw, n)
        checks["reported"] = False
    except WebpGpuError as e:
        checks["reported"] = "earlier launch" in str(e) and "1 new" in str(e)
    try:
        frames.encode_frames(rgba)  # the next clean launch reports WG_OK again
        frames.encode_status(w, mbw, n)
        checks["recovered"] = True
    except WebpGpuError:
        checks["recovered"] = False
    ok = all(checks.values())
    print(json.dumps({"mode": "diag", "ok": ok, "checks": checks}), flush=True)
    return ok


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "race"
    sys.exit(0 if (race() if mode == "race" else diag()) else 1)
