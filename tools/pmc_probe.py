"""Minimal self-play run for bisecting profiler problems:
python tools/pmc_probe.py [fake|net] [rounds] [games] [cache_log2] [timing_every]"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "fake"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    games = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    cache = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    timing = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    import katacoffee_amd as kc
    path = None
    if mode == "net":
        path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
        kc.write_random_model("b6c96", 0xC0FFEE, path)
    sp = kc.Selfplay(5, 5, 4, num_games=games, max_visits=600, seed=1, model_path=path, commit_interval=8,
                     nn_cache_log2=cache)
    if timing:
        sp.enable_timing(timing)
    for _ in range(rounds // 50):
        sp.step(50)
        sp.sync()
    print("probe ok", mode, sp.stats()["playouts"], flush=True)
    sp.close()


if __name__ == "__main__":
    main()
