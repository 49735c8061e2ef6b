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
    for k in ["kNNForwardCap", "kNNForward", "kConv1L", "kConvLB", "kConvL", "kGpoolBias", "kHeadsL", "kBackupSelect", "kResolve", "kSelect", "kBackup", "kCommit", "kRows", "kCacheWrite",
              "kCompact", "kFakeNet", "kInit", "fillBuffer", "copyBuffer"]:
        if k in name:
            return k
    return name[:40]


def main():
    kind, d, prefix = sys.argv[1], sys.argv[2], sys.argv[3]
    if kind == "trace":
        path = os.path.join(d, prefix + "_kernel_trace.csv")
        dur = collections.defaultdict(list)
        seq = []
        for r in csv.DictReader(open(path)):
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur[short(r["Kernel_Name"])].append(b - a)
            seq.append((a, b, short(r["Kernel_Name"])))
        # idle time between consecutive dispatches, per (previous -> next) kernel pair
        seq.sort()
        gaps = collections.defaultdict(list)
        for (a0, b0, k0), (a1, b1, k1) in zip(seq, seq[1:]):
            if 0 <= a1 - b0 < 1000000:
                gaps[k0 + "->" + k1].append(a1 - b0)
        out = {}
        for k, v in dur.items():
            v.sort()
            out[k] = {"calls": len(v), "avg_ns": sum(v) / len(v), "p10_ns": v[len(v) // 10], "p50_ns": v[len(v) // 2],
                      "p90_ns": v[(9 * len(v)) // 10], "max_ns": v[-1]}
        for k, v in gaps.items():
            v.sort()
            out["gap " + k] = {"calls": len(v), "avg_ns": sum(v) / len(v), "p50_ns": v[len(v) // 2]}
        # the longest dispatches (> 1 ms) with what else ran while they were in flight
        t0 = seq[0][0] if seq else 0
        starts = [a for a, _, _ in seq]
        longest = sorted(seq, key=lambda x: x[0] - x[1])[:8]
        outl = []
        for a, b, k in longest:
            if b - a < 1000000:
                break
            import bisect
            lo = bisect.bisect_left(starts, a - 50000000)
            hi = bisect.bisect_right(starts, b)
            over = collections.Counter(k2 for a2, b2, k2 in seq[lo:hi] if b2 > a and a2 < b and (a2, b2) != (a, b))
            outl.append({"kernel": k, "start_ms": (a - t0) / 1e6, "dur_ms": (b - a) / 1e6,
                         "overlapping": dict(over.most_common(8))})
        out["outliers_over_1ms"] = outl
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
