"""profiles/traffic_latest.json from the round-6 PMC passes (tools/profile_r06.sh c2pmc corrpmc
accpmc c4pmc): per-dispatch FETCH_SIZE (x 1024 x 2: gfx950 reports half the bytes of 16-B/lane
streaming reads, MI355X_MICROARCH.md HBM section) and WRITE_SIZE (x 1024) averages per kernel,
and the per-launch keys bench.py reads.  The C2 passes ran the bench's default layout (four game
groups: 1024 games per search launch, ~450 boards per network launch).
usage: python tools/traffic_r06.py"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles", "r06", "prof")


def main():
    per = {}
    for tag in ("c2", "c2corr", "c2acc", "c4steady"):
        f = json.load(open(os.path.join(PROF, "r06_%s_fetch_pmc_avg.json" % tag)))
        w = json.load(open(os.path.join(PROF, "r06_%s_write_pmc_avg.json" % tag)))
        for k in sorted(set(f) | set(w)):
            if not k.startswith("k"):
                continue
            fc = f.get(k, {}).get("FETCH_SIZE", {"avg": 0.0, "dispatches": 0})
            wc = w.get(k, {}).get("WRITE_SIZE", {"avg": 0.0, "dispatches": 0})
            fb, wb = 2.0 * fc["avg"] * 1024.0, wc["avg"] * 1024.0
            per["%s/%s" % (tag, k)] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb,
                                       "dispatches": max(fc["dispatches"], wc["dispatches"])}
    b = lambda k: per.get(k, {}).get("bytes")
    out = {"round": "r06",
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over `bench.py --no-cpu-baseline "
                     "--no-compliant-line --trained-steps 0 --window short --warmup 8 --steps 6 --rounds-per-step "
                     "200` (4 game groups, 8 HW queues) at --precision fast (c2), corrected (c2corr) and accurate "
                     "(c2acc); c4steady: `--config C4 --window short --warmup 9 --steps 1 --rounds-per-step 200` "
                     "with --kernel-include-regex kSelect|kBackup|kCompact --kernel-iteration-range [3000-3399] "
                     "(tools/profile_r06.sh; built by tools/traffic_r06.py); per-dispatch averages; FETCH_SIZE KB x "
                     "1024 x 2 (gfx950), WRITE_SIZE KB x 1024; counters include Infinity-Cache hits",
           "per_kernel": per,
           "network_bytes_per_launch": b("c2/kNNForward"),
           # a corrected launch is the corrected kernel plus its (nearly always empty)
           # re-evaluation on the capped accurate kernel: two kNNForwardCap dispatches per round
           "network_bytes_per_launch_corrected": 2.0 * b("c2corr/kNNForwardCap"),
           "network_bytes_per_launch_accurate": b("c2acc/kNNForwardCap"),
           "select_bytes_per_launch": b("c2/kSelect"),
           "backup_bytes_per_launch": b("c2/kBackup"),
           "backup_select_bytes_per_launch": b("c2/kBackupSelect")}
    json.dump(out, open(os.path.join(REPO, "profiles", "traffic_latest.json"), "w"), indent=1)
    print({k: v for k, v in out.items() if "per_launch" in k})


if __name__ == "__main__":
    main()
