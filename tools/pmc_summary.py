"""Committed summaries of a tools/profile_r0N.sh session (gpurun_out/ -> profiles/):
  profiles/<round>_c2_kernel_stats.csv / _kernel_durations.json   rocprofv3 --kernel-trace --stats of the C2 bench
  profiles/<round>_c3|c5_kernel_stats.csv / _kernel_durations.json   the same for C3 / C5 (layered network)
  profiles/<round>_pmc.json, profiles/traffic_latest.json         per-dispatch FETCH_SIZE / WRITE_SIZE bytes
FETCH_SIZE is doubled (gfx950: it reports half the bytes of 16-B/lane streaming reads,
MI355X_MICROARCH.md HBM section); WRITE_SIZE is in KB.
usage: python tools/pmc_summary.py r02"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def main():
    rnd = sys.argv[1]
    for tag, d, prefix in [("c2", "prof_trace", "trace"), ("c3", "prof_c3", "c3"), ("c5", "prof_c5", "c5")]:
        src = os.path.join(OUT, d)
        if os.path.exists(os.path.join(src, prefix + "_kernel_stats.csv")):
            shutil.copy(os.path.join(src, prefix + "_kernel_stats.csv"),
                        os.path.join(PROF, "%s_%s_kernel_stats.csv" % (rnd, tag)))
        if os.path.exists(os.path.join(src, prefix + "_durations.json")):
            shutil.copy(os.path.join(src, prefix + "_durations.json"),
                        os.path.join(PROF, "%s_%s_kernel_durations.json" % (rnd, tag)))
    fetch = json.load(open(os.path.join(OUT, "prof_fetch", "fetch_pmc_avg.json")))
    write = json.load(open(os.path.join(OUT, "prof_write", "write_pmc_avg.json")))
    per = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, {}).get("FETCH_SIZE", {"avg": 0.0, "dispatches": 0})
        w = write.get(k, {}).get("WRITE_SIZE", {"avg": 0.0, "dispatches": 0})
        fb, wb = 2.0 * f["avg"] * 1024.0, w["avg"] * 1024.0
        per[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb, "dispatches": max(f["dispatches"], w["dispatches"])}
    method = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over `bench.py --no-cpu-baseline --warmup 16 "
              "--steps 8 --rounds-per-step 250`; per-dispatch averages; FETCH_SIZE KB x 1024 x 2 (gfx950: FETCH_SIZE "
              "reports half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM section), WRITE_SIZE KB x "
              "1024; counters include Infinity-Cache hits")
    summary = {"round": rnd, "method": method, "per_kernel": per}
    json.dump(summary, open(os.path.join(PROF, rnd + "_pmc.json"), "w"), indent=1)
    traffic = dict(summary)
    traffic["network_bytes_per_launch"] = per.get("kNNForward", {}).get("bytes")
    traffic["select_bytes_per_launch"] = per.get("kSelect", {}).get("bytes")
    traffic["backup_bytes_per_launch"] = per.get("kBackup", {}).get("bytes")
    json.dump(traffic, open(os.path.join(PROF, "traffic_latest.json"), "w"), indent=1)
    print(json.dumps({k: v["bytes"] for k, v in per.items()}, indent=1))


if __name__ == "__main__":
    main()
