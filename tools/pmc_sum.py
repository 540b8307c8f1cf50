"""Sum rocprofv3 counter_collection.csv values per kernel (last dispatch of each kernel name)."""
import csv
import sys
from collections import defaultdict


def summarize(path, kernels=("mtb_replay",)):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not any(x in k for x in kernels):
            continue
        per[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    last = {}
    for (k, d), v in per.items():
        if k not in last or d > last[k][0]:
            last[k] = (d, dict(v))
    return {k: v for k, (d, v) in last.items()}


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for k, v in summarize(p).items():
            print(p, k.split("(")[0], {c: round(x) for c, x in sorted(v.items())})
