"""WRITE_SIZE per store site of k_decode_bands.

The bench batch's decode (64 x 1080p, the three parsed libwebp q75
bitstreams in turn, normal filter: bench.make_inputs) launched 3 times alone.
Run under `rocprofv3 --pmc WRITE_SIZE` once per build of
webp_amd/libwebpgpu_skipw<mask>.so (make -C webp_amd variant NAME=skipw<mask>
DEFS=-DWG_DEC_SKIPW=<mask>: the masked store sites are dropped);
tools/gpu_dec_write_sites.sh differences the per-launch WRITE_SIZE into
bytes per site.  `--summarize out.json dir...` does the differencing.
Algorithmic bytes per site (per launch, 64 x 8160 MBs): frame Y 256 B/MB,
U+V 128 B/MB, top record 32 B and bottom record 128 B per MB of a band's
last row (rows 3, 7, ... except the image's last)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B, MBW, MBH = 64, 120, 68


def algorithmic():
    hand_rows = len([y for y in range(MBH) if y % 4 == 3 and y < MBH - 1])
    mbs = B * MBW * MBH
    return {"Y rows (frame)": 256 * mbs, "U/V rows (frame)": 128 * mbs,
            "top records": 32 * B * MBW * hand_rows, "bottom records": 128 * B * MBW * hand_rows}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--summarize":
        res = json.load(open(sys.argv[2]))
        base = res["0"]
        sites = {"top records (1)": "1", "bottom records (2)": "2", "Y rows 0..12 (4)": "4", "U/V rows 0..4 (8)": "8",
                 "Y rows 13..15 above (16)": "16", "U/V rows 5..7 above (32)": "32"}
        per = {k: base - res[m] for k, m in sites.items() if m in res}
        rest = base - res["63"] if "63" in res else None
        summary = {"write_bytes_per_launch": base, "by_site": per, "all_sites_dropped": res.get("63"),
                   "left_with_every_site_dropped": rest, "algorithmic": algorithmic()}
        json.dump(summary, open(sys.argv[3], "w"), indent=1)
        print(json.dumps(summary, indent=1))
        return
    import torch
    import bench
    from webp_amd import frames
    rgba, mb, co, _ = bench.make_inputs(B, 0, "cuda")
    del rgba
    dY = torch.empty((B, 16 * MBH, 16 * MBW), dtype=torch.uint8, device="cuda")
    dU = torch.empty((B, 8 * MBH, 8 * MBW), dtype=torch.uint8, device="cuda")
    dV = torch.empty_like(dU)
    from webp_amd import _lib
    work = torch.empty(_lib.lib.wg_decode_work_bytes(MBW, MBH, B), dtype=torch.uint8, device="cuda")
    ts = []
    for _ in range(int(os.environ.get("LAUNCHES", "3"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        frames.decode_frames(mb, co, 2, MBW, MBH, B, out=(dY, dU, dV), work=work)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print("ok", os.environ.get("WEBPGPU_LIB", "default"), int(dY.sum()) & 0xffff,
          "median %.3f ms of %d launches" % (sorted(ts)[len(ts) // 2], len(ts)))


if __name__ == "__main__":
    main()
