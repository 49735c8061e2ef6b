"""Shrinks rocprofv3 output in gpurun_out/ in place (run on the GPU box, before the
files travel back): per-kernel duration quantiles from the kernel trace, per-kernel
PMC counter averages from a --pmc pass; the large per-dispatch CSVs are removed.
usage: python tools/reduce_profile.py trace|pmc <dir> <prefix>"""
import collections
import csv
import json
import os
import sys


def short(name):
    for k in ["kNNForward", "kConvL", "kGpoolBias", "kHeadsL", "kSelect", "kBackup", "kCommit", "kRows", "kCacheWrite",
              "kCompact", "kFakeNet", "kInit", "fillBuffer", "copyBuffer"]:
        if k in name:
            return k
    return name[:40]


def main():
    kind, d, prefix = sys.argv[1], sys.argv[2], sys.argv[3]
    if kind == "trace":
        path = os.path.join(d, prefix + "_kernel_trace.csv")
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out = {}
        for k, v in dur.items():
            v.sort()
            out[k] = {"calls": len(v), "avg_ns": sum(v) / len(v), "p10_ns": v[len(v) // 10], "p50_ns": v[len(v) // 2],
                      "p90_ns": v[(9 * len(v)) // 10], "max_ns": v[-1]}
        json.dump(out, open(os.path.join(d, prefix + "_durations.json"), "w"), indent=1)
        os.remove(path)
    else:
        path = os.path.join(d, prefix + "_counter_collection.csv")
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        out = collections.defaultdict(dict)
        for (k, c), v in agg.items():
            out[k][c] = {"dispatches": len(v), "avg": sum(v) / len(v)}
        json.dump(out, open(os.path.join(d, prefix + "_pmc_avg.json"), "w"), indent=1)
        os.remove(path)


if __name__ == "__main__":
    main()
