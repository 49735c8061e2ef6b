"""Self-play trajectory on the bench workload: per chunk of rounds, the rate of
moves (rows), playouts and network evaluations, and games finished, to see where the
synchronized opening ends and the steady state begins (bench.py burn-in)."""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--visits", type=int, default=600)
    ap.add_argument("--chunk", type=int, default=1000)
    ap.add_argument("--chunks", type=int, default=30)
    ap.add_argument("--nn-cache-log2", type=int, default=21)
    ap.add_argument("--nn-batch-cap", type=int, default=0)
    a = ap.parse_args()
    import katacoffee_amd as kc
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model("b6c96", 0xC0FFEE, path)
    sp = kc.Selfplay(5, 5, 4, num_games=a.games, max_visits=a.visits, seed=20250217, model_path=path,
                     commit_interval=8, nn_cache_log2=a.nn_cache_log2, nn_batch_cap=a.nn_batch_cap)
    prev = sp.stats()
    for c in range(a.chunks):
        t0 = time.perf_counter()
        sp.step(a.chunk)
        sp.sync()
        dt = time.perf_counter() - t0
        sp.drain_rows()
        st = sp.stats()
        d = {k: st[k] - prev[k] for k in ("moves", "playouts", "nn_evals", "games_finished")}
        prev = st
        print("rounds %6d  rows/s %8.0f  playouts/s %9.0f  evals/playout %.3f  games %5d  ms/round %.3f" % (
            (c + 1) * a.chunk, d["moves"] / dt, d["playouts"] / dt, d["nn_evals"] / max(1, d["playouts"]),
            d["games_finished"], 1000 * dt / a.chunk), flush=True)


if __name__ == "__main__":
    main()
