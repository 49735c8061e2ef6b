"""profiles/traffic_latest.json from the round-5 PMC passes (tools/profile_r05.sh c2pmc corrpmc) and
the round-6 steady-state C4 search passes (tools/profile_r06.sh c4pmc: counters for dispatches
3000-3399 of kSelect / kBackup / kCompact only):
per-dispatch FETCH_SIZE (x 1024 x 2: gfx950 reports half the bytes of 16-B/lane streaming
reads, MI355X_MICROARCH.md HBM section) and WRITE_SIZE (x 1024) averages per kernel, and the
per-launch keys bench.py reads.  usage: python tools/traffic_r05.py"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")


def main():
    per = {}
    for tag in ("c2", "c2corr"):
        f = json.load(open(os.path.join(PROF, "r05", "r05_%s_fetch_pmc_avg.json" % tag)))
        w = json.load(open(os.path.join(PROF, "r05", "r05_%s_write_pmc_avg.json" % tag)))
        for k in sorted(set(f) | set(w)):
            fc = f.get(k, {}).get("FETCH_SIZE", {"avg": 0.0, "dispatches": 0})
            wc = w.get(k, {}).get("WRITE_SIZE", {"avg": 0.0, "dispatches": 0})
            fb, wb = 2.0 * fc["avg"] * 1024.0, wc["avg"] * 1024.0
            per["%s/%s" % (tag, k)] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb,
                                       "dispatches": max(fc["dispatches"], wc["dispatches"])}
    f = json.load(open(os.path.join(PROF, "r06", "prof", "r06_c4steady_fetch_pmc_avg.json")))
    w = json.load(open(os.path.join(PROF, "r06", "prof", "r06_c4steady_write_pmc_avg.json")))
    for k in sorted(set(f) | set(w)):
        fc = f.get(k, {}).get("FETCH_SIZE", {"avg": 0.0, "dispatches": 0})
        wc = w.get(k, {}).get("WRITE_SIZE", {"avg": 0.0, "dispatches": 0})
        fb, wb = 2.0 * fc["avg"] * 1024.0, wc["avg"] * 1024.0
        per["c4steady/%s" % k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb,
                                  "dispatches": max(fc["dispatches"], wc["dispatches"])}
    b = lambda k: per.get(k, {}).get("bytes")
    out = {"round": "r05 (C2), r06 (C4 steady state)",
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over `bench.py --no-cpu-baseline "
                     "--no-compliant-line --window short --warmup 8 --steps 6 --rounds-per-step 200` at --precision "
                     "fast (c2) and corrected (c2corr) (tools/profile_r05.sh c2pmc corrpmc; profiles/r05/r05_c2*_pmc_avg"
                     ".json; built by tools/traffic_r05.py); per-dispatch averages; FETCH_SIZE KB x 1024 x 2 (gfx950: "
                     "FETCH_SIZE reports half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM section), "
                     "WRITE_SIZE KB x 1024; counters include Infinity-Cache hits; c4steady/*: round 6, `bench.py "
                     "--config C4 --window short --warmup 9 --steps 1 --rounds-per-step 200` with --kernel-include-regex "
                     "kSelect|kBackup|kCompact --kernel-iteration-range [3000-3399] (steady per-move trees)",
           "per_kernel": per,
           "network_bytes_per_launch": b("c2/kNNForward"),
           # the corrected instance plus its (nearly always empty) re-evaluation launch
           "network_bytes_per_launch_corrected": b("c2corr/kNNForwardCap") + (b("c2corr/kNNForward") or 0.0),
           "select_bytes_per_launch": b("c2/kSelect"),
           "backup_bytes_per_launch": b("c2/kBackup"),
           "backup_select_bytes_per_launch": b("c2/kBackupSelect")}
    json.dump(out, open(os.path.join(PROF, "traffic_latest.json"), "w"), indent=1)
    print({k: v for k, v in out.items() if k.endswith("per_launch") or k.endswith("corrected")})


if __name__ == "__main__":
    main()
