"""Summarize rocprofv3 --pmc counter CSVs (SQ block) for the replay kernel (plain or ticket-scheduled): totals and per op.
usage: python tools/sq_summary.py OPS_PER_DISPATCH out.json csv [csv ...]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    ops = float(sys.argv[1])
    out = sys.argv[2]
    tot = defaultdict(float)
    disp = set()
    for path in sys.argv[3:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Kernel_Name"] not in ("mtb_replay_kernel", "mtb_replay_tick_kernel", "mtb_replay_pass_kernel", "mtb_replay_few_kernel"):
                    continue
                disp.add((path, r["Dispatch_Id"]))
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    nd = len({d for _, d in disp}) or 1
    per_op = {k: v / (ops * nd) for k, v in tot.items()}
    res = {"what": f"rocprofv3 --pmc SQ counters of the replay kernel, {nd} dispatch(es) per pass x {ops:.0f} ops; "
                   "totals and per op (SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are per-wave quad-cycle counts)",
           "totals": dict(tot), "per_op": per_op}
    if tot.get("SQ_WAVE_CYCLES"):
        res["wait_any_frac"] = tot.get("SQ_WAIT_ANY", 0) / tot["SQ_WAVE_CYCLES"]
        res["issue_frac"] = tot.get("SQ_ACTIVE_INST_ANY", 0) / tot["SQ_WAVE_CYCLES"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: round(v, 1) for k, v in per_op.items()}))


if __name__ == "__main__":
    main()
