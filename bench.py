"""Self-play benchmark: BASELINE.json config C2 (5x5 connect-4 Coffee, 4096 games per
GPU, 600 visits, random-init b6c96; the network runs fp16 MFMA with f32 accumulation
-- same rate as bf16 on gfx950, more mantissa) on N GPUs of one node.

A "step" is `--rounds-per-step` (1000) rounds of the hot path over the whole batch of
games (one round = select/expand for every game -> one batched network
evaluation -> backup, plus the periodic move-commit launch).  Games shard across
ranks (slot_base = rank * games); finished rows are drained each step and, for
N > 1, gathered to rank 0 over RCCL (the only collective).

value = training rows/s over the timed steps for the whole job.  In benchmark mode
(one row per move at full visits) a row is fixed the moment its move is
committed; rows are emitted to the buffer when the game ends.  We count committed
moves (= rows) in the window; rows actually drained in the window are reported too.

Self-play clears the search tree before every move, as the reference does for
self-play (play.cpp:1941-1946), so every row costs a full 600-visit search.

All games start together and stay roughly in phase (a 5x5 game at 600 visits lasts
about 11000 rounds), so rates swing by up to 2x from one 1000-round chunk to the next
(tools/steady_state.py prints the trajectory).  The defaults (20 warm-up steps =
20k rounds, then 60 timed steps = 60k rounds, about 5 game cycles) average the swings
out: over 100k+ rounds the long-run rate is within a few percent of this window's.
Short --steps/--warmup values time a partial cycle and can be off by 30%.

The network batch is capped at one full wave of network workgroups (compute units x
8 boards = 2048 rows; coffee_selfplay_config.nn_batch_cap): a launch's cost steps with
its number of workgroup waves, so rows past the cap wait one round (round-robin, so no
row waits long) instead of paying for a mostly idle second wave.

The NN evaluation cache is on at the reference's own selfplay1.cfg size
(nnCacheSizePowerOfTwo = 21, nneval.cpp:611-623): a search leaf whose state was
evaluated earlier, by any game, takes that evaluation instead of the network, as in
the reference; nn_evals_per_sec counts only real network evaluations.  The CPU
baseline runs the same cache.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_F16_TFLOPS = 2500.0    # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--visits", type=int, default=600)
    ap.add_argument("--arch", default="b6c96")
    ap.add_argument("--rounds-per-step", type=int, default=1000)
    ap.add_argument("--commit-interval", type=int, default=8)
    ap.add_argument("--nn-cache-log2", type=int, default=21,
                    help="NN evaluation cache entries = 2^k (selfplay1.cfg nnCacheSizePowerOfTwo = 21); 0 = off")
    ap.add_argument("--nn-batch-cap", type=int, default=0,
                    help="rows per network launch (0 = one full wave of network workgroups)")
    ap.add_argument("--play", choices=["benchmark", "production"], default="benchmark",
                    help="benchmark: SURVEY 8d (one row per move at full visits, the metric's mode); "
                         "production: selfplay1.cfg play settings (configs/selfplay1_coffee5.cfg)")
    ap.add_argument("--seed", type=int, default=20250217)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP event timing")
    ap.add_argument("--timing-every", type=int, default=16,
                    help="time every N-th launch of each kernel group (an event pair costs a few us of stream gap)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of the network kernel from a PMC pass (see profiles/)")
    return ap.parse_args()


# selfplay1.cfg play settings (cpp/configs/training/selfplay1.cfg lines 24-76)
PRODUCTION = dict(init_games_with_policy=1, policy_init_area_prop=0.04, side_position_prob=0.02,
                  cheap_search_prob=0.75, cheap_search_visits=100, cheap_search_target_weight=0.0, reduce_visits=1,
                  reduce_visits_threshold=0.9, reduce_visits_threshold_lookback=3, reduced_visits_min=100,
                  reduced_visits_weight=0.1, policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1,
                  early_fork_game_prob=0.04, early_fork_game_expected_move_prop=0.025, fork_game_prob=0.01,
                  fork_game_min_choices=3, early_fork_game_max_choices=12, fork_game_max_choices=36)


def cpu_baseline(model_path, visits, seconds, cache_log2):
    """The oracle (C++ CPU restatement: same rules/search/rows, fp32 Eigen-semantics
    network) on this host's cores: a bounded sample of the same workload."""
    import numpy as np  # noqa: F401
    from oracle import oracle

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(cores, 16))
    games = 2 * cores
    model = oracle.Model(model_path)
    sp = oracle.Selfplay(5, 5, 4, games=games, max_visits=visits, node_cap=max(2048, 3 * visits), seed=1,
                         nn_mode=1, model=model, nn_threads=cores, nn_cache_log2=cache_log2)
    sp.rounds(8)  # warm-up: root evaluations
    i0 = [sp.info(g) for g in range(games)]
    t0 = time.perf_counter()
    rounds = 0
    while time.perf_counter() - t0 < seconds:
        sp.rounds(16)
        rounds += 16
    dt = time.perf_counter() - t0
    i1 = [sp.info(g) for g in range(games)]
    moves = sum(b["movesMade"] - a["movesMade"] for a, b in zip(i0, i1))
    playouts = sum(b["playouts"] - a["playouts"] for a, b in zip(i0, i1))
    return {
        "value": moves / dt,
        "unit": "rows/s",
        "playouts_per_sec": playouts / dt,
        "cores": cores,
        "kind": "port",
        "sample": "oracle C++ self-play, %d games x %d visits, b6c96 fp32, %d rounds in %.1f s (%d moves, %d playouts)"
                  % (games, visits, rounds, dt, moves, playouts),
    }


def main():
    args = parse()
    import torch

    import katacoffee_amd as kc
    from katacoffee_amd import rows as kcrows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    tmpdir = tempfile.mkdtemp(prefix="kcbench%d_" % rank)
    model_path = os.path.join(tmpdir, "%s.cfnn" % args.arch)
    kc.write_random_model(args.arch, 0xC0FFEE, model_path)
    flops_per_eval = kc.model_flops(model_path, 25)

    sp = kc.Selfplay(5, 5, 4, num_games=args.games, max_visits=args.visits, seed=args.seed,
                     slot_base=rank * args.games, model_path=model_path, commit_interval=args.commit_interval,
                     nn_cache_log2=args.nn_cache_log2, nn_batch_cap=args.nn_batch_cap)
    for _ in range(args.warmup):
        sp.step(args.rounds_per_step)
        sp.sync()  # bounded launch queue (a profiler's per-dispatch state stays small)
    s0 = sp.stats()
    sp.drain_rows()
    if not args.no_timing:
        sp.enable_timing(args.timing_every)
    base_ms = [sp.kernel_time(i) for i in range(4)]
    base_timed_evals = sp.timed_nn_evals()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    rows_gathered = 0
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sp.step(args.rounds_per_step)
        rows = sp.drain_rows()
        n = len(rows["meta"])
        if dist is not None:
            # RCCL gather of this step's finished rows to rank 0 (the writer rank)
            got = kcrows.gather_to_rank0(rows, 5, 5, dist, torch.device("cuda", local))
            if rank == 0:
                rows_gathered += len(got["meta"])
        else:
            rows_gathered += n
    sp.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = sp.stats()
    moves = s1["moves"] - s0["moves"]
    playouts = s1["playouts"] - s0["playouts"]
    evals = s1["nn_evals"] - s0["nn_evals"]
    kt = [sp.kernel_time(i) for i in range(4)]
    timed_evals = sp.timed_nn_evals() - base_timed_evals
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([moves, playouts, evals], dtype=torch.float64, device="cuda")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        moves, playouts, evals = [float(v) for v in c.tolist()]
    rows_per_sec = moves / elapsed
    out = None
    if rank == 0:
        names = ["select", "network", "backup", "commit"]
        kernels = {}
        for i, nm in enumerate(names):
            ms = kt[i][0] - base_ms[i][0]
            n = kt[i][1] - base_ms[i][1]
            kernels[nm] = {"ms_timed": ms, "launches_timed": n, "avg_us": 1000.0 * ms / n if n else None}
        net = kernels["network"]
        roof = None
        if net["launches_timed"]:
            # the timed launches' own batch sizes (kCompact sums them on the device)
            per_launch = timed_evals / net["launches_timed"]
            avg_s = net["avg_us"] * 1e-6
            achieved = per_launch * flops_per_eval / avg_s / 1e12
            traffic = None
            if os.path.exists(args.traffic_json):
                try:
                    traffic = json.load(open(args.traffic_json)).get("network_bytes_per_launch")
                except Exception:
                    traffic = None
            roof = {"kernel": "kNNForward (fused b6c96 forward)", "bound": "mfma", "achieved": achieved,
                    "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s", "frac": achieved / PEAK_F16_TFLOPS,
                    "traffic": traffic, "evals_per_launch": per_launch, "flops_per_eval": flops_per_eval,
                    "avg_launch_us": net["avg_us"], "timed_launches": net["launches_timed"],
                    "timing": "HIP events on the engine stream around every %d-th launch" % args.timing_every}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(model_path, args.visits, args.cpu_seconds, args.nn_cache_log2)
        out = {
            "metric": "self-play training rows/sec + MCTS playouts/sec, 5x5 Coffee b6c96 @600 visits",
            "value": rows_per_sec,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16",
            "data": "synthetic: self-play from empty 5x5 boards, random-init b6c96 (seed 0xC0FFEE)",
            "config": {"workload": "C2: 5x5 connect-4, %d games/GPU, %d visits, b6c96 (fp16 MFMA)" % (args.games, args.visits),
                       "games_per_gpu": args.games, "visits": args.visits, "rounds_per_step": args.rounds_per_step,
                       "commit_interval": args.commit_interval, "nn_cache_log2": args.nn_cache_log2,
                       "nn_batch_cap": args.nn_batch_cap or "one workgroup wave",
                       "play_settings": args.play,
                       "parallelism": "game-sharded x%d" % world},
            "playouts_per_sec": playouts / elapsed,
            "moves_per_sec": moves / elapsed,
            "nn_evals_per_sec": evals / elapsed,
            "rows_drained": rows_gathered,
            "kernels": kernels,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu"] = rows_per_sec / cpu["value"] if cpu["value"] > 0 else None
        print(json.dumps(out))
    sp.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
