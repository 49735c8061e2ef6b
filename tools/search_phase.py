"""Cycle accounting of the search kernels on the bench workload (C2).
Needs the profiling build:  make -C katacoffee_amd/csrc prof
usage: python tools/search_phase.py [--games 4096] [--rounds 300] [--warmup 600]"""
import argparse
import ctypes
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KATACOFFEE_LIB", os.path.join(REPO, "tools", "_build", "libkatacoffee_prof.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--visits", type=int, default=600)
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--probe", action="store_true", help="count evaluated leaves whose state repeats (NN-cache bound)")
    ap.add_argument("--nn-cache-log2", type=int, default=21)
    a = ap.parse_args()
    import katacoffee_amd as kc
    L = kc.lib()
    prof = (ctypes.c_ulonglong * 32)()
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model("b6c96", 0xC0FFEE, path)
    sp = kc.Selfplay(5, 5, 4, num_games=a.games, max_visits=a.visits, seed=1, model_path=path, commit_interval=8,
                     nn_cache_log2=a.nn_cache_log2)
    sp.step(a.warmup)
    sp.sync()
    if a.probe:
        import torch
        keys = torch.zeros(1 << 24, dtype=torch.int64, device="cuda")
        L.coffee_debug_probe_table(ctypes.c_void_p(keys.data_ptr()), ctypes.c_ulonglong(1 << 24))
    L.coffee_debug_search_profile(prof, 1)
    sp.step(a.rounds)
    sp.sync()
    L.coffee_debug_search_profile(prof, 1)
    p = list(prof)
    nb, nk = max(p[0], 1), max(p[10], 1)
    print("select: %d blocks over %d rounds" % (p[0], a.rounds))
    for name, i in [("total", 1), ("loadGame", 2), ("descend", 3), ("  selectBest", 5), ("  expansion", 6),
                    ("encode+slot", 7)]:
        print("  %-14s %8.0f cycles/block" % (name, p[i] / nb))
    print("  path levels    %8.2f per block" % (p[4] / nb))
    print("  slowest select block %d cycles (mean of per-slot maxima %.0f), deepest path %d" %
          (p[24], p[27] / max(1, a.games), p[25]))
    print("  slowest backup block %d cycles (mean of per-slot maxima %.0f)" % (p[26], p[28] / max(1, a.games)))
    if a.probe:
        print("NN-cache bound: %d of %d evaluated leaves repeat an earlier state (%.1f%%)" %
              (p[9], p[10], 100.0 * p[9] / max(1, p[10])))
    print("backup: %d blocks" % p[10])
    for name, i in [("total", 11), ("post+order", 12), ("leaf value", 14), ("path backup", 13)]:
        print("  %-14s %8.0f cycles/block" % (name, p[i] / nk))
    nc = max(p[16], 1)
    print("commit: %d blocks, %d finished games, %.0f live nodes kept per move" % (p[16], p[23], p[22] / nc))
    for name, i in [("total", 17), ("choice+targets", 18), ("tree reuse", 19)]:
        print("  %-14s %8.0f cycles/block" % (name, p[i] / nc))
    nf = max(p[23], 1)
    for name, i in [("finishGame", 20), ("startGame", 21)]:
        print("  %-14s %8.0f cycles/finished game" % (name, p[i] / nf))


if __name__ == "__main__":
    main()
