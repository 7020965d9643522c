"""Summarise rocprofv3 --pmc csv passes per kernel (average per dispatch).
Applies the gfx950 corrections of MI355X_MICROARCH.md: FETCH_SIZE reads half
(doubled here); SQ_*CYCLES counters are in quad-cycles."""
import collections
import csv
import glob
import gzip
import sys


def load(root, by_grid=False):
    """{kernel: {counter: average per dispatch}}; by_grid: keys "name@grid" (the
    same kernel launched at several sizes, e.g. the batch and a single frame)."""
    # rows of one pass (one rocprofv3 run, its own file) are summed per dispatch;
    # a counter collected in several passes (SQ_WAVES is in every SQ group) is
    # averaged over them -- summing it across passes doubled SQ_WAVES and halved
    # every per-wave figure through r05
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    files = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True) + \
        glob.glob(f"{root}/**/*counter_collection.csv.gz", recursive=True)
    for f in files:
        for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            kn = r["Kernel_Name"].replace("(anonymous namespace)", "anon")
            name = kn.split("(")[0].split("<")[0].split("::")[-1] or kn[:40]
            if by_grid:
                name = f"{name}@{r['Grid_Size']}"
            acc[name][(r["Counter_Name"], r["Dispatch_Id"])][f] += float(r["Counter_Value"])
    out = {}
    for k, d in acc.items():
        per = collections.defaultdict(list)
        for (cn, _), by_pass in d.items():
            per[cn].append(sum(by_pass.values()) / len(by_pass))
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
