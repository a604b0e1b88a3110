"""Summarise rocprofv3 PMC csv files per kernel.

  python tools/pmc_summary.py run_counter_collection.csv ...           # table
  python tools/pmc_summary.py --json out.json fetch.csv write.csv      # HBM bytes per launch

FETCH_SIZE / WRITE_SIZE are in KB.  MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane) streaming reads.
tools/fetch_calib.py measured the same factor for every read width the
kernels here use (profiles/r03_fetch_calibration.json): 32-B and 8-B per-lane
row pieces, 16 rows per wave instruction, count 0.50 of their bytes when a
line's pieces are read close together, i.e. every L2 miss fills a 128-B line
and is tallied at 64 B; read far apart (k_encode_rows' pattern) they count
0.83 and 2.09, which is 0.5 x the real re-fetch (lines evicted between
pieces).  So FETCH_SIZE is doubled for every kernel (round 2 took k_encode_rows'
raw count, which the calibration does not support).  WRITE_SIZE is exact for
32-B stores close together (1.01) and counts the real partial-line write
traffic when they are far apart (1.86 for 32-B, 6.8 for 8-B pieces).  Raw and
corrected values are both written.
"""
import collections
import csv
import json
import sys



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


def any_json(out, paths):
    """Per-kernel per-launch averages of every counter in the files."""
    agg = load(paths)
    rec = {}
    for name, ctrs in agg.items():
        if not name.startswith("k_"):
            continue
        rec[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        rec[name]["launches"] = max(len(v) for v in ctrs.values())
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


def main(argv):
    out = None
    if argv and argv[0] == "--any-json":
        return any_json(argv[1], argv[2:])
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
        rec[name] = {"fetch_size_bytes_raw": int(f), "write_size_bytes": int(w),
                     "hbm_bytes_per_launch": int(2 * f + w), "launches": len(ctrs["FETCH_SIZE"]),
                     "correction": "FETCH_SIZE x2 (128-B line fills tallied at 64 B; measured for these access widths "
                                   "in profiles/r03_fetch_calibration.json) + WRITE_SIZE"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
