"""Summarise rocprofv3 PMC csv files per kernel.

  python tools/pmc_summary.py run_counter_collection.csv ...           # table
  python tools/pmc_summary.py --json out.json fetch.csv write.csv      # HBM bytes per launch

FETCH_SIZE / WRITE_SIZE are in KB.  MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane) streaming reads,
so the HBM byte figure doubles it; WRITE_SIZE is exact for 16-B stores.  Both
raw and corrected values are written so the correction stays visible.

The undercount is of 128-B requests (tallied at 64 B).  k_encode_rows never
makes one: each lane reads its own row's 32-B (Y) / 8-B (U, V) pieces, a
wave instruction touching 16 different rows, plus 4- to 16-B hand-off and
table words.  Its raw FETCH_SIZE equals the bytes it has to read (source
1.5 B/px = 200.5 MB per 64 x 1080p, hand-off records and top-right words
27 MB, segment ids 0.5 MB, cost tables: ~229 MB against 236 MB counted), so it is taken as
is; doubling it would claim twice what the kernel can read.
"""
import collections
import csv
import json
import sys

NARROW_READS = {"k_encode_rows"}  # no 128-B read requests: FETCH_SIZE is not halved (see above)


def load(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        for row in csv.DictReader(open(path)):
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].strip()
            name = name.removeprefix("void ").split("<")[0]  # "void k_encode_rows<true>" -> "k_encode_rows"
            agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return agg


SQ_COUNTERS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES",
               "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE")


def valu_json(out, paths):
    """Per-kernel averages of the SQ / GRBM pass (one launch each)."""
    agg = load(paths)
    rec = {}
    for name, ctrs in agg.items():
        if not name.startswith("k_") or "SQ_INSTS_VALU" not in ctrs:
            continue
        rec[name] = {c: sum(ctrs[c]) / len(ctrs[c]) for c in SQ_COUNTERS if c in ctrs}
        rec[name]["launches"] = len(ctrs["SQ_INSTS_VALU"])
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


def main(argv):
    out = None
    if argv and argv[0] == "--valu-json":
        return valu_json(argv[1], argv[2:])
    if argv and argv[0] == "--json":
        out, argv = argv[1], argv[2:]
    agg = load(argv)
    if out is None:
        for name, ctrs in agg.items():
            print(name, "|", "; ".join(f"{c}: n={len(v)} avg={sum(v) / len(v):.4g}" for c, v in ctrs.items()))
        return
    rec = {}
    for name, ctrs in agg.items():
        if "FETCH_SIZE" not in ctrs or "WRITE_SIZE" not in ctrs or not name.startswith("k_"):
            continue
        f = sum(ctrs["FETCH_SIZE"]) / len(ctrs["FETCH_SIZE"]) * 1024
        w = sum(ctrs["WRITE_SIZE"]) / len(ctrs["WRITE_SIZE"]) * 1024
        narrow = name in NARROW_READS
        rec[name] = {"fetch_size_bytes_raw": int(f), "write_size_bytes": int(w),
                     "hbm_bytes_per_launch": int((1 if narrow else 2) * f + w), "launches": len(ctrs["FETCH_SIZE"]),
                     "correction": ("FETCH_SIZE x1 (no 128-B read requests, tools/pmc_summary.py) + WRITE_SIZE"
                                    if narrow else "FETCH_SIZE x2 (gfx950 wide-read undercount) + WRITE_SIZE")}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
