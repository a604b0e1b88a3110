"""Summarise rocprofv3 PMC csv (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel."""
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, ctrs in agg.items():
    parts = [f"{c}: n={len(v)} avg={sum(v)/len(v):.1f} KB" for c, v in ctrs.items()]
    print(name, "|", "; ".join(parts))
