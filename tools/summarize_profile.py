"""Turns a profile_session.sh run (gpurun_out/) into committed summaries under profiles/.

  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<round>_pmc.json           per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch,
                                      with the gfx950 correction (FETCH_SIZE x2 for 16-B/lane
                                      streaming reads, MI355X_MICROARCH.md "HBM"), in bytes
  profiles/<round>_bench.json         the bench.py JSON line of the same session
  profiles/traffic_latest.json        network-kernel HBM bytes per launch, read by bench.py
usage: python tools/summarize_profile.py r01
"""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def short(name):
    for k in ["kNNForward", "kSelect", "kBackup", "kCommit", "kRows", "kCacheWrite", "kCompact", "kFakeNet", "kInit",
              "fillBuffer", "copyBuffer"]:
        if k in name:
            return k
    return name[:40]


def pmc(path, counter):
    """Per-kernel average of `counter` from a reduced PMC pass (tools/reduce_profile.py)."""
    red = json.load(open(path))
    return {k: v[counter]["avg"] for k, v in red.items() if counter in v}


def main():
    rnd = sys.argv[1]
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof_trace", "trace_kernel_stats.csv"), os.path.join(PROF, rnd + "_kernel_stats.csv"))
    fetch = pmc(os.path.join(OUT, "prof_fetch", "fetch_pmc_avg.json"), "FETCH_SIZE")
    write = pmc(os.path.join(OUT, "prof_write", "write_pmc_avg.json"), "WRITE_SIZE")
    dur = os.path.join(OUT, "prof_trace", "trace_durations.json")
    if os.path.exists(dur):
        shutil.copy(dur, os.path.join(PROF, rnd + "_kernel_durations.json"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f_kb, w_kb = fetch.get(k, 0.0), write.get(k, 0.0)
        kernels[k] = {"FETCH_SIZE_KB_raw": f_kb, "WRITE_SIZE_KB_raw": w_kb,
                      "hbm_read_bytes": 2.0 * f_kb * 1024.0, "hbm_write_bytes": w_kb * 1024.0,
                      "hbm_bytes": 2.0 * f_kb * 1024.0 + w_kb * 1024.0}
    stats = {}
    for r in csv.DictReader(open(os.path.join(PROF, rnd + "_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                   "pct": float(r["Percentage"])}
    summary = {"round": rnd, "note": "per-dispatch averages; FETCH_SIZE doubled per the gfx950 correction",
               "kernels": kernels, "kernel_stats": stats}
    json.dump(summary, open(os.path.join(PROF, rnd + "_pmc.json"), "w"), indent=1)
    bench = os.path.join(OUT, "bench.json")
    if os.path.exists(bench):
        line = [l for l in open(bench).read().splitlines() if l.startswith("{")][-1]
        open(os.path.join(PROF, rnd + "_bench.json"), "w").write(line + "\n")
    nn = kernels.get("kNNForward")
    if nn:
        json.dump({"round": rnd, "network_bytes_per_launch": nn["hbm_bytes"],
                   "select_bytes_per_launch": kernels.get("kSelect", {}).get("hbm_bytes"),
                   "backup_bytes_per_launch": kernels.get("kBackup", {}).get("hbm_bytes")},
                  open(os.path.join(PROF, "traffic_latest.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
