"""HBM counter calibration and the measured copy ceiling (tools/libprobe.so).

  python tools/fetch_calib.py                 # launch every probe once (run under rocprofv3 --pmc ...)
  python tools/fetch_calib.py --copy          # print the measured copy-kernel GB/s
  python tools/fetch_calib.py --summarize OUT.json fetch.csv write.csv

MI355X_MICROARCH.md (HBM): FETCH_SIZE reads half the bytes of a wide
16-B-per-lane coalesced stream on gfx950; other access widths are
uncalibrated.  k_encode_rows reads its source rows as per-lane 32-B (Y: two
16-B loads) and 32-B (U / V: four 8-B loads) pieces of 16 different rows per
wave instruction, a row's pieces ~70 us apart, so each variant here moves a
known byte count in one of those patterns, and the summary divides the
counters by it.  tools/pmc_summary.py applies the measured factor.
"""
import ctypes
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "libprobe.so")

PITCH = 1920               # a 1080p luma row
ROWS = 16 * 16384          # 503 MB: past the 256 MiB infinity cache
STREAM_BYTES = 1 << 30

# kernel name (template args kept) -> (bytes moved, what it stands for)
VARIANTS = {
    "k_probe_read_stream": (STREAM_BYTES, "16 B/lane lane-contiguous stream (the guide's x2 case)"),
    "k_probe_read_rows<32, false>": (ROWS * PITCH, "32-B row pieces (two 16-B loads), 16 rows per wave instruction"),
    "k_probe_read_rows<32, true>": (ROWS * PITCH, "same, ~14 us between a row's pieces (k_encode_rows' Y import)"),
    "k_probe_read_rows<8, false>": (ROWS * PITCH, "8-B row pieces, 16 rows per wave instruction"),
    "k_probe_read_rows<8, true>": (ROWS * PITCH, "same, ~14 us between pieces (k_encode_rows' U / V import)"),
    "k_probe_write_rows<32, false>": (ROWS * PITCH, "32-B row-piece stores (two 16-B stores)"),
    "k_probe_write_rows<32, true>": (ROWS * PITCH, "same, ~14 us apart (k_encode_rows' reconstruction export)"),
    "k_probe_write_rows<8, true>": (ROWS * PITCH, "8-B row-piece stores, ~14 us apart"),
}


def _lib():
    if not os.path.exists(PROBE):
        raise RuntimeError(f"{PROBE} missing: make -C tools")
    lib = ctypes.CDLL(PROBE)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    lib.probe_copy.argtypes = [vp, vp, i64, i32, vp]
    lib.probe_read_stream.argtypes = [vp, i64, i32, vp, vp]
    lib.probe_read_rows.argtypes = [vp, i64, i64, i32, i32, i32, vp, vp]
    lib.probe_write_rows.argtypes = [vp, i64, i64, i32, i32, i32, vp]
    return lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


def copy_peak(device=None, nbytes=2 << 30, reps=5):
    """Measured device-to-device copy rate (read + write bytes / time, GB/s) of
    the nontemporal probe_copy and of torch's copy_, best of `reps` each, timed
    with HIP events on the current stream."""
    import torch
    lib = _lib()
    dev = device or torch.device("cuda", torch.cuda.current_device())
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    s = torch.cuda.current_stream(dev).cuda_stream
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    res = {}
    for name, fn in (("probe_copy", lambda: _check(lib.probe_copy(dst.data_ptr(), src.data_ptr(), nbytes, cus * 8, s),
                                                  "probe_copy")),
                     ("torch_copy", lambda: dst.copy_(src))):
        fn()
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        res[name] = round(2 * nbytes / (best / 1e3) / 1e9, 1)
    del src, dst
    return {"GB/s": max(res.values()), "by_kernel": res, "bytes_per_copy": 2 * nbytes,
            "method": "read+write bytes / best of %d event-timed launches" % reps}


def launch_all():
    import torch
    lib = _lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    buf = torch.randint(0, 255, (max(STREAM_BYTES, ROWS * PITCH),), dtype=torch.uint8, device=dev)
    out = torch.empty(ROWS // 16 * 64 + 4 * 256 * 256 * 8, dtype=torch.int32, device=dev)
    grid = torch.cuda.get_device_properties(dev).multi_processor_count * 8
    _check(lib.probe_read_stream(buf.data_ptr(), STREAM_BYTES, grid, out.data_ptr(), s), "read_stream")
    for piece in (32, 8):
        for slow in (0, 1):
            _check(lib.probe_read_rows(buf.data_ptr(), PITCH, ROWS, PITCH, piece, slow, out.data_ptr(), s), "read_rows")
    dst = torch.empty(ROWS * PITCH, dtype=torch.uint8, device=dev)
    for piece, slow in ((32, 0), (32, 1), (8, 1)):
        _check(lib.probe_write_rows(dst.data_ptr(), PITCH, ROWS, PITCH, piece, slow, s), "write_rows")
    torch.cuda.synchronize()
    print("probes launched:", ", ".join(VARIANTS))


def _kname(raw):
    n = raw.replace("(anonymous namespace)::", "").removeprefix("void ").strip()
    head, _, rest = n.partition("(")
    return head.strip()


def summarize(out, paths):
    """Counter / known bytes per probe variant (FETCH_SIZE and WRITE_SIZE are in KB)."""
    vals = {}
    for path in paths:
        for row in csv.DictReader(open(path)):
            k = _kname(row["Kernel_Name"])
            if k in VARIANTS:
                vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]) * 1024)
    rec = {}
    for k, (nbytes, what) in VARIANTS.items():
        c = vals.get(k, {})
        r = {"bytes": nbytes, "pattern": what}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            if ctr in c:
                v = sum(c[ctr]) / len(c[ctr])
                r[ctr.lower() + "_bytes"] = int(v)
                r[ctr.lower() + "_per_byte"] = round(v / nbytes, 4)
        rec[k] = r
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--summarize"]:
        summarize(sys.argv[2], sys.argv[3:])
    elif sys.argv[1:2] == ["--copy"]:
        print(json.dumps(copy_peak()))
    else:
        launch_all()
