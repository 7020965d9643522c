"""Summarise rocprofv3 --pmc csv passes per kernel (average per dispatch).
Applies the gfx950 corrections of MI355X_MICROARCH.md: FETCH_SIZE reads half
(doubled here); SQ_*CYCLES counters are in quad-cycles."""
import collections
import csv
import glob
import sys


def load(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"].replace("(anonymous namespace)", "anon")
            name = kn.split("(")[0].split("<")[0].split("::")[-1] or kn[:40]
            acc[name][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    out = {}
    for k, d in acc.items():
        per = collections.defaultdict(list)
        for (cn, _), vals in d.items():
            per[cn].append(sum(vals))
        out[k] = {cn: sum(v) / len(v) for cn, v in per.items()}
    return out


if __name__ == "__main__":
    res = load(sys.argv[1])
    for k, d in sorted(res.items()):
        if "FETCH_SIZE" in d:
            d["FETCH_SIZE_corrected_KB"] = 2 * d["FETCH_SIZE"]
        print(k)
        for cn in sorted(d):
            print(f"   {cn:28s} {d[cn]:.4g}")
