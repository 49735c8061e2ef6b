"""Self-play benchmark (BASELINE.json): training rows/s + MCTS playouts/s of the
MI355X Coffee self-play engine, one process per GPU.

Workloads (BASELINE.json configs; --config, default C2, the config the metric is
quoted on):
  C2  5x5 connect-4, 4096 games/GPU, 600 visits, b6c96       (fused network kernel)
  C3  5x5 connect-4, 16384 games/GPU, 600 visits, b10c128    (layered network kernels)
  C4  7x7 connect-5, 8192 games/GPU, 800 visits, b10c128     (layered)
  C5  9x9 connect-5, 4096 games/GPU, 1600 visits, b18c384nbt (layered, nested bottlenecks)
Networks are random-init (seed 0xC0FFEE); positions start from empty boards.  The
network computes with fp16 MFMA operands, f32 accumulation and f32 residual trunk
(--precision fast, the configs' bf16/fp16), or fp16 hi/lo pairs (--precision accurate).

A "step" is --rounds-per-step rounds of the hot path over every game of the GPU
(one round = select/expand -> one batched network evaluation -> backup, plus the
periodic move-commit launch).  Games shard across ranks (slot_base = rank * games);
each step's finished rows are drained from the device and, for N > 1, gathered to
rank 0 over RCCL (the only collective); a writer thread on rank 0 writes them to
.npz files (the reference's trainingwrite row format) inside the timed region.

value = training rows written per second in the timed window, whole job (the rows a
step drains from the device -- those of games that ended -- gathered to rank 0 and
written to .npz by the writer thread before the clock stops).  In the benchmark play
settings (one row per move at full visits) every committed move becomes
exactly one row when its game ends, so in steady state rows/s = moves/s.  Steady state
(--window steady, the default for C2-C4): game starts are staggered over one game length
(a seeded per-slot idle delay) and the warm-up covers 1.5 game lengths (rounds per step
are raised to fit the --warmup steps), so game ends arrive at their steady rate through
the whole window.  --window short (C5 default, whose games last ~65k rounds): value is
committed moves/s and says so in value_kind.

--gpus N without a torch.distributed launcher starts N ranks itself (one process per
GPU, RCCL world size N); under torchrun the environment's WORLD_SIZE is used.
"""
import argparse
import faulthandler
import json
import math
import os
import queue
import shutil
import socket
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_F16_TFLOPS = 2500.0    # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0       # HBM3E
# SURVEY 8d canonical record sizes for the tree roofline: node stats 32 B, per child
# a 16 B edge + the child's 32 B stats
NODE_B, CHILD_B = 32, 48

CONFIGS = {
    "C2": dict(X=5, Y=5, W=4, games=4096, visits=600, arch="b6c96", rounds=1000,
               label="C2: 5x5 connect-4, 4096 games/GPU, 600 visits, b6c96"),
    "C3": dict(X=5, Y=5, W=4, games=16384, visits=600, arch="b10c128", rounds=200,
               label="C3: 5x5 connect-4, 16384 games/GPU, 600 visits, b10c128"),
    "C4": dict(X=7, Y=7, W=5, games=8192, visits=800, arch="b10c128", rounds=200,
               label="C4: 7x7 connect-5, 8192 games/GPU, 800 visits, b10c128"),
    "C5": dict(X=9, Y=9, W=5, games=4096, visits=1600, arch="b18c384nbt", rounds=40,
               label="C5: 9x9 connect-5, 4096 games/GPU, 1600 visits, b18c384nbt"),
}

# selfplay1.cfg play settings (cpp/configs/training/selfplay1.cfg lines 24-76)
PRODUCTION = dict(init_games_with_policy=1, policy_init_area_prop=0.04, side_position_prob=0.02,
                  cheap_search_prob=0.75, cheap_search_visits=100, cheap_search_target_weight=0.0, reduce_visits=1,
                  reduce_visits_threshold=0.9, reduce_visits_threshold_lookback=3, reduced_visits_min=100,
                  reduced_visits_weight=0.1, policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1,
                  early_fork_game_prob=0.04, early_fork_game_expected_move_prop=0.025, fork_game_prob=0.01,
                  fork_game_min_choices=3, early_fork_game_max_choices=12, fork_game_max_choices=36)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C2")
    ap.add_argument("--games", type=int, default=0, help="games per GPU (0 = the config's)")
    ap.add_argument("--visits", type=int, default=0, help="visits per move (0 = the config's)")
    ap.add_argument("--rounds-per-step", type=int, default=0,
                    help="0 = the config's, raised so the warm-up covers 1.5 game lengths (--window steady)")
    ap.add_argument("--window", choices=["steady", "short"], default=None,
                    help="steady: warm-up past the first game ends, value = rows written/s; short: value = moves/s "
                         "(default: steady except C5)")
    ap.add_argument("--precision", choices=["fast", "default", "accurate", "fast-layered", "corrected"], default=None,
                    help="network precision of the headline window (default: fast for C2 -- fp16 operands, the "
                         "configs' fp16/bf16 dtype class, within 1e-3 of fp32 on this random-init benchmark net "
                         "(tests/test_gpu_nn.py) but not on trained nets; 'default' for C3-C5, the layered nets' "
                         "1e-3 path.  A fast headline also measures a window at 'default', the product's "
                         "1e-3 path (the C ABI's, the CLI's and the configs' precision), which the CPU speed-up "
                         "is quoted on)")
    ap.add_argument("--trained-steps", type=int, default=-1,
                    help="also measure the default precision on a trained net: one generation of the reference's "
                         "loop on this GPU (the engine's own self-play rows from the random-init net, then N Adam "
                         "steps of katacoffee_amd.train); -1: 200 for C2, 0 otherwise; 0: skip")
    # 16: a game whose search is done waits at most 15 rounds for its move, and every
    # group's round chain carries half the commit / row launches of 8 (C2: +2.4 %)
    ap.add_argument("--commit-interval", type=int, default=16)
    ap.add_argument("--nn-cache-log2", type=int, default=21,
                    help="NN evaluation cache entries = 2^k (selfplay1.cfg nnCacheSizePowerOfTwo = 21); 0 = off")
    ap.add_argument("--nn-batch-cap", type=int, default=0,
                    help="rows per network launch (0 = engine default: one workgroup wave for the fused kernel)")
    ap.add_argument("--play", choices=["benchmark", "production"], default="benchmark",
                    help="benchmark: SURVEY 8d (one row per move at full visits, the metric's mode); "
                         "production: selfplay1.cfg play settings")
    ap.add_argument("--opening-prop", type=float, default=0.0,
                    help="short-game variant (benchmark play): each game opens with floor(-ln(u) A P) moves "
                         "sampled from the raw policy without search or rows (initGamesWithPolicy, "
                         "playutils.cpp:147-176), the rest is searched at full visits, one row per searched move: "
                         "rows/s of a long-game config (C5) measured on disk within a short window")
    ap.add_argument("--stagger", type=int, default=-1,
                    help="per-slot start delay range in rounds (-1 = min(one game, 90%% of the warm-up))")
    ap.add_argument("--groups", type=int, default=0,
                    help="independent game groups per GPU, each on its own stream (overlaps one group's network "
                         "with another's search kernels; the reference's numNNServerThreadsPerModel); "
                         "0 = 4 at C2-C4, 1 for b18c384nbt (C5), whose forward is throughput-bound")
    ap.add_argument("--reload-every", type=int, default=0,
                    help="hot reload every K timed steps: rank 0 writes a new random model and broadcasts its "
                         "bytes over RCCL; every engine switches (the reference's model hot reload)")
    ap.add_argument("--seed", type=int, default=20250217)
    ap.add_argument("--no-npz", action="store_true", help="do not write .npz files in the timed region")
    ap.add_argument("--row-sink", choices=["local", "gather"], default="local",
                    help="N > 1: local = every rank writes its own games' rows (sharded games, no collective in "
                         "the loop); gather = rows gathered to rank 0 over RCCL each step (one writer)")
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="timed CPU-baseline window (saturated run)")
    ap.add_argument("--cpu-curve-seconds", type=float, default=10.0,
                    help="timed window of the single-thread run and of each point of the CPU thread-scaling curve "
                         "(2, 4, 8 threads below the share: the linearity the whole-host extrapolation rests on; "
                         "0: no curve, the single-thread run then takes --cpu-seconds)")
    ap.add_argument("--cpu-c1-seconds", type=float, default=10.0, help="timed CPU-baseline window (C1)")
    ap.add_argument("--cpu-warmup-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-whole-host", action="store_true",
                    help="also time the CPU baseline on every CPU of the affinity mask (default: extrapolated, "
                         "since the GPU box asks to stay within its CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-compliant-line", dest="compliant_line", action="store_false",
                    help="skip the second window at the 1e-3-compliant (default) precision")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP event timing")
    ap.add_argument("--timing-every", type=int, default=16,
                    help="time every N-th launch of each kernel group (an event pair costs a few us of stream gap)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes per kernel from a PMC pass (see profiles/)")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = "fast" if args.config == "C2" else "default"
    if args.trained_steps < 0:
        args.trained_steps = 200 if args.config == "C2" else 0
    if args.commit_interval < 1:
        ap.error("--commit-interval must be >= 1")
    if args.groups < 0 or args.steps < 1 or args.warmup < 0:
        ap.error("--groups >= 0, --steps >= 1, --warmup >= 0")
    return args


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, script=None, argv=None):
    """One process per GPU (torch.distributed.run's environment contract: RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT), started as children before anything
    here touches the GPU; rank 0 prints the JSON line.  Returns the worst exit code."""
    port = free_port()
    script = script or os.path.abspath(__file__)
    argv = sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def trained_model(kc, torch, cfg, steps, src_model, path, seed):
    """One generation of the reference's training loop on this GPU, from seeds only (no
    weights are committed): the engine self-plays 512 games at 64 visits with the random-init
    net (benchmark play, fast precision: this is data generation), katacoffee_amd.train
    (python/train.py's policy / value losses) runs `steps` Adam steps on minibatches of 512
    of those rows, and the net is written as CFNN (desc.cpp's format) to `path`."""
    import numpy as np
    from katacoffee_amd import train
    X, Y, W = cfg["X"], cfg["Y"], cfg["W"]
    t0 = time.perf_counter()
    sp = kc.Selfplay(X, Y, W, num_games=512, max_visits=64, seed=seed, model_path=src_model, node_cap=128,
                     nn_cache_log2=16, nn_precision="fast")
    parts, n = [], 0
    for _ in range(8):
        sp.step(1024)
        r = sp.drain_rows()
        parts.append(r)
        n += len(r["meta"])
        if n >= 4096:
            break
    sp.close()
    rows = {k: np.concatenate([q[k] for q in parts]) for k in parts[0]}
    batch = train.rows_to_batch(rows, X, Y, device="cuda")
    torch.manual_seed(seed)
    net = train.CoffeeNet(cfg["arch"]).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(seed)
    losses = None
    for _ in range(steps):
        idx = torch.randint(0, n, (min(512, n),), generator=g).cuda()
        losses = train.train_step(net, opt, {k: v[idx] for k, v in batch.items()})
    with torch.no_grad():
        pol, val, misc = net(batch["binp"][:2048], batch["glob"][:2048])
        mx = max(float(t.abs().max()) for t in (pol, val, misc))
    train.save_cfnn(net.cpu(), path)
    h = kc.Network(path, X, Y, W, precision="default")
    resolved, calib = h.precision  # the load-time calibration
    h.close()
    return {"default_resolves_to": resolved, "calibration_max_abs_diff": calib, "adam_steps": steps, "minibatch": min(512, n), "rows": n, "selfplay": "512 games x 64 visits, random-init net",
            "final_losses": {"policy": losses[0], "value": losses[1]} if losses else None,
            "max_abs_logit_on_rows": mx, "seconds": time.perf_counter() - t0}


def physical_cores(cpus):
    """Physical cores behind a set of logical CPUs (SMT siblings counted once)."""
    cores = set()
    for c in cpus:
        try:
            sib = open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c).read().strip()
        except OSError:
            sib = str(c)
        cores.add(sib)
    return len(cores)


def cpu_info():
    """Threads the CPU baseline uses: OMP_NUM_THREADS (the GPU box sets 16, its CPU share
    per GPU, and asks that worker pools stay within it), else the affinity mask; the
    machine's totals (logical CPUs, physical cores) are reported beside it."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if cores <= 0:
        cores = len(aff)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    n = os.cpu_count()
    return cores, model, {"nproc": n, "affinity": len(aff), "physical_cores": physical_cores(range(n)),
                          "affinity_physical_cores": physical_cores(aff),
                          "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_run(oracle, model, X, Y, W, games, visits, threads, warm_s, timed_s, cache_log2):
    """The oracle's self-play on `threads` host threads: `threads` independent game groups
    of games / threads games, one per thread, each with its own search, network batch
    (single-threaded forward) and NN cache (1/threads of the entries) -- the reference's
    shape on a CPU, numGameThreads game threads feeding NN server threads that each run
    whole batches (selfplay.cpp:271-357, nneval.cpp:341-364), rather than one round-
    synchronous batch split across threads (0.37 efficiency at 16 threads in round 4).
    ctypes drops the GIL inside each group's rounds call, so the groups run concurrently.
    Rows (= committed moves in benchmark play) and playouts per second over the window."""
    gpt = max(1, games // threads)
    sps = [oracle.Selfplay(X, Y, W, games=gpt, max_visits=visits, node_cap=max(2048, 3 * visits), seed=1,
                           slot_base=i * gpt, nn_mode=1, model=model, nn_threads=1,
                           nn_cache_log2=max(0, cache_log2 - (threads - 1).bit_length()) if cache_log2 else 0)
           for i in range(threads)]
    phase = [0]  # 1: window open, 2: window closed
    marks = [[None, None] for _ in range(threads)]  # per group: (time, rounds, counters) at open / close
    errs = []

    def counters(sp):
        return [sum(sp.info(g)[key] for g in range(gpt)) for key in ("movesMade", "playouts", "nnEvals")]

    def worker(k):
        # each group's counters are read by its own thread between its rounds calls
        try:
            done = 0
            while phase[0] < 2 or marks[k][1] is None:
                sps[k].rounds(8)
                done += 8
                for p in (1, 2):
                    if phase[0] >= p and marks[k][p - 1] is None:
                        marks[k][p - 1] = (time.perf_counter(), done, counters(sps[k]))
        except Exception as e:  # surfaced after the window
            errs.append(e)
            for p in (0, 1):
                marks[k][p] = marks[k][p] or (time.perf_counter(), 0, [0, 0, 0])

    ths = [threading.Thread(target=worker, args=(k,), daemon=True) for k in range(threads)]
    for t in ths:
        t.start()
    time.sleep(warm_s)
    phase[0] = 1
    time.sleep(timed_s)
    phase[0] = 2
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    rate = [0.0, 0.0, 0.0]
    tot = [0, 0, 0]
    for (t0, r0, c0), (t1, r1, c1) in marks:
        for j in range(3):
            rate[j] += (c1[j] - c0[j]) / (t1 - t0)
            tot[j] += c1[j] - c0[j]
    dt = sum(m[1][0] - m[0][0] for m in marks) / threads
    return dict(rows_per_sec=rate[0], playouts_per_sec=rate[1], nn_evals_per_sec=rate[2],
                rounds=sum(m[1][1] - m[0][1] for m in marks) // threads, seconds=dt, moves=tot[0], playouts=tot[1],
                games_per_thread=gpt)


def cpu_baseline(args, cfg, model_path):
    """The oracle (C++ restatement: same rules / search / rows, fp32 forward with
    eigenbackend.cpp semantics, convolutions as im2col + a register-blocked AVX2
    SGEMM) on this host: C1 (1 game, 200 visits) and the GPU's workload on the host's CPU
    share (cpu_run: one independent game group of 8 games per thread), plus the same on one
    thread for the scaling efficiency and a 1/2/4/8/... thread curve."""
    from oracle import oracle
    cores, model_name, machine = cpu_info()
    model = oracle.Model(model_path)
    visits = args.visits or cfg["visits"]
    gpt = 8
    run = lambda games, v, threads, secs, warm=args.cpu_warmup_seconds: cpu_run(
        oracle, model, cfg["X"], cfg["Y"], cfg["W"], games, v, threads, warm, secs, args.nn_cache_log2)
    c1 = None
    if cfg["arch"] == "b6c96" and (cfg["X"], cfg["Y"]) == (5, 5):
        c1 = run(1, 200, 1, args.cpu_c1_seconds, 5.0)
    sat = run(gpt * cores, visits, cores, args.cpu_seconds)
    # the single-thread run and the curve's points share one regime (the saturated run's
    # warm-up, then cpu_curve_seconds) and run back to back, so the per-thread rates they
    # compare saw the same game phase (a group's rate still rises after its first rounds:
    # +5 % from 5 s to 30 s of warm-up, +28 % to 60 s in the build container) and the same
    # load from the host's other tenants
    curve_s = args.cpu_curve_seconds if args.cpu_curve_seconds > 0 else args.cpu_seconds
    one = run(gpt, visits, 1, curve_s) if cores > 1 else sat
    eff = sat["playouts_per_sec"] / (cores * one["playouts_per_sec"]) if one["playouts_per_sec"] > 0 else None
    curve = {}
    t = 2
    while t < cores and args.cpu_curve_seconds > 0:
        curve[t] = run(gpt * t, visits, t, curve_s)["playouts_per_sec"]
        t *= 2
    curve[1], curve[cores] = one["playouts_per_sec"], sat["playouts_per_sec"]
    desc = lambda r, g, t, w=args.cpu_warmup_seconds: ("%d games x %d visits on %d threads (%d independent groups of %d), %.0f s warm-up "
                                   "then %.1f s (%d rounds per group, %d moves, %d playouts)"
                                   % (g, visits, t, t, r["games_per_thread"], w, r["seconds"], r["rounds"], r["moves"],
                                      r["playouts"]))
    out = {
        "value": sat["rows_per_sec"], "unit": "rows/s", "cores": cores, "kind": "port",
        "playouts_per_sec": sat["playouts_per_sec"], "nn_evals_per_sec": sat["nn_evals_per_sec"],
        "cpu_model": model_name, "host_cpus": machine,
        "sample": "oracle C++ self-play (fp32 im2col+SGEMM forward), %s workload, %s"
                  % (cfg["label"].split(":")[0], desc(sat, gpt * cores, cores, args.cpu_warmup_seconds)),
        "single_thread": {"rows_per_sec": one["rows_per_sec"], "playouts_per_sec": one["playouts_per_sec"],
                          "sample": desc(one, gpt, 1), "scaling_efficiency_at_%d" % cores: eff},
        # the points below the share: the single-thread run's regime; the share's own point
        # is the saturated run (its longer window)
        "thread_curve_playouts_per_sec": {str(k): curve[k] for k in sorted(curve)},
        # playouts/s at t threads / (t x the 1-thread rate): the whole-host extrapolation's premise
        "thread_curve_efficiency": {str(k): curve[k] / (k * curve[1]) if curve.get(1) else None for k in sorted(curve)},
    }
    # Whole host (all physical cores).  The GPU box asks that worker pools stay
    # within its CPU share (16 threads per GPU), so the whole host is not run by default: the
    # share's measured per-thread rate (groups are independent: the thread curve above is the
    # check that it scales linearly) is extrapolated to the machine's physical cores, and,
    # as an upper bound, to every logical CPU (SMT siblings counted as full cores).  The
    # speed-up is quoted against the upper bound.  --cpu-whole-host measures it instead.
    nproc = machine["nproc"] or cores
    phys = machine["physical_cores"] or nproc
    if cores >= nproc:  # the share is the whole machine: the saturated run measured it
        out["whole_host"] = {"value": sat["rows_per_sec"], "unit": "rows/s", "threads": cores, "kind": "measured",
                             "physical_cores": phys, "sample": out["sample"]}
    elif args.cpu_whole_host:
        t = machine["affinity"]
        wh = run(gpt * t, visits, t, args.cpu_seconds)
        out["whole_host"] = {"value": wh["rows_per_sec"], "unit": "rows/s", "threads": t, "kind": "measured",
                             "physical_cores": machine["physical_cores"],
                             "sample": desc(wh, gpt * t, t, args.cpu_warmup_seconds)}
    else:
        # value: the physical cores (SMT siblings are not cores; SURVEY 8d asks for all physical
        # cores); logical_cpus_value counts every SMT sibling as a full core (an upper bound)
        out["whole_host"] = {"value": sat["rows_per_sec"] * phys / cores, "unit": "rows/s", "threads": phys,
                             "physical_cores": phys, "kind": "extrapolated",
                             "logical_cpus": nproc, "logical_cpus_value": sat["rows_per_sec"] * nproc / cores,
                             "method": "measured %d-thread rate (1->%d thread efficiency %s: independent game groups) "
                                       "x %d physical cores / %d, linear; logical_cpus_value: x %d logical CPUs / %d"
                                       % (cores, cores, "%.2f" % eff if eff else "n/a", phys, cores, nproc, cores),
                             "why_not_measured": "the GPU box's CPU share is %d threads per GPU (OMP_NUM_THREADS); "
                                                 "worker pools stay within it" % cores}
    if c1:
        out["C1"] = {"rows_per_sec": c1["rows_per_sec"], "playouts_per_sec": c1["playouts_per_sec"], "threads": 1,
                     "sample": "1 game x 200 visits, b6c96 fp32, 5 s warm-up then %.1f s (%d moves, %d playouts)"
                               % (c1["seconds"], c1["moves"], c1["playouts"])}
    return out


class NpzWriter:
    """Writes row blocks to .npz files on a background thread (trainingwrite.cpp
    writeToZipFile :566-587 then rename :765-769, via the native coffee_write_npz)."""

    def __init__(self, kc, X, Y, outdir, prefix="rows"):
        self.kc, self.X, self.Y, self.dir, self.prefix = kc, X, Y, outdir, prefix
        self.q = queue.Queue()
        self.rows = 0
        self.files = 0
        self.err = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            rows = self.q.get()
            if rows is None:
                return
            try:
                n = len(rows["meta"])
                if n:
                    path = os.path.join(self.dir, "%s%06d.npz" % (self.prefix, self.files))
                    self.kc.write_npz(path + ".tmp", rows, self.X, self.Y)
                    os.replace(path + ".tmp", path)
                    self.files += 1
                    self.rows += n
            except Exception as e:  # surfaced by close()
                self.err = e

    def put(self, rows):
        self.q.put(rows)

    def close(self):
        self.q.put(None)
        self.t.join()
        if self.err:
            raise self.err


class Groups:
    """K independent engines over disjoint game slots, each on its own HIP stream
    (the engine's), stepped in interleaved chunks so one group's network launch
    overlaps another group's select / backup kernels (the reference's
    numNNServerThreadsPerModel: several batching servers per GPU).  Each group keeps
    its own NN cache (the reference's servers share one), so every group is as
    deterministic as a single engine.  Each group's round is still its own serial
    chain select -> compact -> network -> backup; two groups overlap those chains."""

    def __init__(self, kc, k, games, slot_base, chunk=8, **kw):
        self.chunk = chunk
        # floor / ceil shares over contiguous slot ranges (any k <= games)
        sizes = [games // k + (1 if i < games % k else 0) for i in range(k)]
        starts = [slot_base + sum(sizes[:i]) for i in range(k)]
        self.g = [kc.Selfplay(num_games=n, slot_base=s0, **kw) for n, s0 in zip(sizes, starts)]

    def step(self, rounds):
        # chunks of the commit interval: an engine's step() also commits on its last
        # round, so shorter chunks would commit more often than the interval asks
        done = 0
        while done < rounds:
            n = min(self.chunk, rounds - done)
            for e in self.g:
                e.step(n)
            done += n

    def sync(self):
        for e in self.g:
            e.sync()

    def stats(self):
        out = {}
        for e in self.g:
            for k, v in e.stats().items():
                out[k] = (max(out.get(k, 0), v) if k in ("edge_pool_peak", "edge_pool_cap", "nn_precision",
                                                          "nn_audit_max_diff")
                          else out.get(k, 0) + v)
        return out

    def drain_rows(self):
        parts = [e.drain_rows() for e in self.g]
        return {k: __import__("numpy").concatenate([p[k] for p in parts]) for k in parts[0]}

    def drain_games(self):
        for e in self.g:
            e.drain_games()

    # device-resident row hand-off: each engine packs its rows into a device block on
    # its own stream (coffee_selfplay_stage_rows) at the end of a step; the block of step
    # s is gathered / copied while step s + 1 runs (two slots)
    def setup_staging(self, torch, kc, X, Y):
        rb = kc.row_bytes(X, Y)
        self.stage_buf = [[torch.empty((e.row_capacity(), rb), dtype=torch.uint8, device="cuda") for e in self.g]
                          for _ in range(2)]
        self.stage_cnt = torch.zeros((2, len(self.g)), dtype=torch.int64).pin_memory()
        self.streams = [torch.cuda.ExternalStream(e.stream_ptr()) for e in self.g]
        self.events = [[torch.cuda.Event() for _ in self.g] for _ in range(2)]
        self.torch = torch

    def stage(self, i):
        for k, e in enumerate(self.g):
            e.stage_rows(self.stage_buf[i][k], self.stage_cnt[i, k])
            self.events[i][k].record(self.streams[k])

    def collect(self, i):
        """This rank's rows staged into slot i, as one device block [n][row_bytes]
        (waits for the staging only, not for the steps enqueued after it)."""
        parts = []
        for k in range(len(self.g)):
            self.events[i][k].synchronize()
            parts.append(self.stage_buf[i][k][:int(self.stage_cnt[i, k])])
        return self.torch.cat(parts) if len(parts) > 1 else parts[0]

    def enable_timing(self, every):
        for e in self.g:
            e.enable_timing(every)

    def kernel_time(self, i):
        t = [e.kernel_time(i) for e in self.g]
        return sum(a for a, _ in t), sum(b for _, b in t)

    def timed_nn_evals(self):
        return sum(e.timed_nn_evals() for e in self.g)

    def set_model_bytes(self, data):
        for e in self.g:
            e.set_model_bytes(data)

    def close(self):
        for e in self.g:
            e.close()


def load_traffic(path):
    try:
        return json.load(open(path))
    except Exception:
        return {}


# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default): with
# more streams than queues, streams share a queue and their kernels serialise.  The bench
# runs one stream per game group plus torch's, so 4 groups need more than 4 queues (C2,
# same box: 4 groups on 4 queues 10.4 k rows/s at the default precision, on 8 queues 17.1 k;
# profiles/r06/groups_hwqueues_ab.txt).  Raised to at least 8 (the GPU box exports 4) before
# anything initialises the HIP runtime; ranks started by launch_ranks inherit it.
HW_QUEUES = 8


def main():
    faulthandler.enable()  # a native fault prints the Python stack too
    try:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        queues = 0
    if queues < HW_QUEUES:
        os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    cfg = CONFIGS[args.config]
    X, Y, W = cfg["X"], cfg["Y"], cfg["W"]
    games = args.games or cfg["games"]
    visits = args.visits or cfg["visits"]
    rps = args.rounds_per_step or cfg["rounds"]
    window = args.window or ("short" if args.config == "C5" else "steady")
    # rounds per game: (visits + root evaluations) per move x ~A/2 moves
    # (with --opening-prop P the first min(O, L) of a game's L ~ A/2 moves are unsearched
    # openings, O exponential with mean A P: E = A P (1 - exp(-L / (A P))))
    L = X * Y / 2.0
    mo = args.opening_prop * X * Y
    game_rounds = int((visits + 4) * max(4.0, L - (mo * (1.0 - __import__("math").exp(-L / mo)) if mo > 0 else 0.0)))
    if window == "steady" and not args.rounds_per_step:
        rps = max(rps, -(-3 * game_rounds // (2 * max(1, args.warmup))))
    import numpy as np  # noqa: F401
    import torch

    import katacoffee_amd as kc
    from katacoffee_amd import rows as kcrows
    from katacoffee_amd import weights as kcweights

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    kc.check(kc.lib().coffee_set_device(local))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    tmpdir = tempfile.mkdtemp(prefix="kcbench%d_" % rank)
    model_path = os.path.join(tmpdir, "%s.cfnn" % cfg["arch"])
    kc.write_random_model(cfg["arch"], 0xC0FFEE, model_path)
    flops_per_eval = kc.model_flops(model_path, X * Y)

    warm_rounds = args.warmup * rps
    if args.stagger >= 0:
        stagger = args.stagger
    else:
        stagger = game_rounds if window == "steady" else min(game_rounds, int(0.9 * warm_rounds))
    play = PRODUCTION if args.play == "production" else {}
    if args.opening_prop > 0:
        if args.play != "benchmark":
            raise SystemExit("--opening-prop is a benchmark-play variant")
        play = dict(init_games_with_policy=1, policy_init_area_prop=args.opening_prop)
    # benchmark mode clears the tree before every move: a search holds at
    # most visits + 1 nodes; production's cheap searches reuse the tree
    node_cap = (visits + 64 + 63) // 64 * 64 if args.play == "benchmark" else 0
    if args.groups == 0:
        # latency-bound rounds gain from overlapped chains (measured: two groups C2 +8 %, C3
        # +12 %, C4 +10 % rows/s over one; four groups on 8 hardware queues over two: C2 +5 %
        # fast, +2.5 % default precision, C3 +4.8 %, C4 +3.4 %; five or more -30 %:
        # profiles/r06/groups_hwqueues_ab*.txt, line_c3_4groups.json, line_c4_4groups.json);
        # b18c384nbt's forward is throughput-bound (C5: -12 % playouts/s with two)
        args.groups = 4 if cfg["arch"] != "b18c384nbt" else 1
    def measure(precision, with_cpu, model_path=model_path):
        """One timed window at `precision` with the network `model_path`; rank 0 returns the
        JSON dict."""
        # nn_batch_cap 0: the engines split the fused network's one wave of workgroups
        # (engines_per_device); the layered network has no batch cap (its cost grows with the batch)
        sp = Groups(kc, args.groups, games, rank * games, chunk=args.commit_interval, X=X, Y=Y, W=W, max_visits=visits, seed=args.seed,
                    model_path=model_path, commit_interval=args.commit_interval, nn_cache_log2=args.nn_cache_log2,
                    nn_batch_cap=args.nn_batch_cap // args.groups, nn_precision=precision, start_stagger=stagger,
                    node_cap=node_cap, engines_per_device=args.groups, **play)
        tw = time.perf_counter()

        def progress(what, i, n, t):  # stderr, rank 0: a long window keeps printing
            if rank == 0:
                print("bench: %s step %d/%d  %.1f s" % (what, i + 1, n, time.perf_counter() - t), file=sys.stderr,
                      flush=True)

        for i in range(args.warmup):
            sp.step(rps)
            sp.sync()  # bounded launch queue (a profiler's per-dispatch state stays small)
            progress("warm-up", i, args.warmup, tw)
            if i == 0 and os.environ.get("KATACOFFEE_DUMP_MAPS"):
                # diagnosis of host faults under profilers: the process map (libraries and
                # device-memory mappings) once every engine buffer exists, to resolve a
                # native stack trace's addresses afterwards
                shutil.copyfile("/proc/self/maps", os.environ["KATACOFFEE_DUMP_MAPS"])
        sp.drain_rows()
        sp.drain_games()
        if not args.no_timing:
            sp.enable_timing(args.timing_every)
        s0 = sp.stats()
        # the precision the engines run (the default one resolved by its calibration check)
        precision = kc.PRECISION_NAMES.get(s0["nn_precision"], precision) if s0["nn_precision"] else precision
        base_ms = [sp.kernel_time(i) for i in range(5)]
        base_timed_evals = sp.timed_nn_evals()
        writer = None
        local_sink = dist is None or args.row_sink == "local"
        if (rank == 0 or local_sink) and not args.no_npz:
            os.makedirs(os.path.join(tmpdir, "tdata"), exist_ok=True)
            # one writer per rank (local sink: each rank's own files), or rank 0's for all
            writer = NpzWriter(kc, X, Y, os.path.join(tmpdir, "tdata"), prefix="rank%d_rows" % rank)
        sink = kcrows.RowSink(X, Y, dist, "local" if local_sink else "gather", writer)

        def barrier():
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()

        def reload(k):
            # rank 0 "trains" a new network; its bytes reach every rank over RCCL
            path = os.path.join(tmpdir, "reload%d.cfnn" % k)
            if rank == 0:
                kc.write_random_model(cfg["arch"], 0xC0FFEE + k, path)
            data = open(path, "rb").read() if dist is None else \
                kcweights.broadcast_model(path, dist, torch.device("cuda", local))
            sp.set_model_bytes(data)

        reloads = 0
        sp.setup_staging(torch, kc, X, Y)

        def process(i):
            # step i's rows: device block -> this rank's host -> its writer thread (local
            # sink), or -> RCCL gather to rank 0 first (gather sink), while the next step's
            # kernels run on the engine streams
            sink.put(sp.collect(i))
            torch.cuda.current_stream().synchronize()  # slot i's blocks are free for step + 2

        barrier()
        t0 = time.perf_counter()
        prev = None
        for step in range(args.steps):
            if args.reload_every and step and step % args.reload_every == 0:
                reloads += 1
                reload(reloads)
            sp.step(rps)
            sp.stage(step % 2)
            if prev is not None:
                process(prev)
            prev = step % 2
            progress("timed", step, args.steps, t0)
        process(prev)
        sp.sync()
        if writer:
            writer.close()  # every drained row is on disk before the clock stops
        barrier()
        elapsed = time.perf_counter() - t0
        s1 = sp.stats()
        d = {k: s1[k] - s0[k] for k in ("moves", "playouts", "nn_evals", "tree_levels", "tree_children")}
        kt = [sp.kernel_time(i) for i in range(5)]
        timed_evals = sp.timed_nn_evals() - base_timed_evals
        rows_gathered, npz_rows, npz_files, rank_rows = sink.totals(
            torch.device("cuda", local), writer.rows if writer else 0, writer.files if writer else 0)
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            keys = ["moves", "playouts", "nn_evals"]
            c = torch.tensor([d[k] for k in keys], dtype=torch.float64, device="cuda")
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            for k, v in zip(keys, c.tolist()):
                d[k] = v
        if rank == 0:
            # backup_select: a round's backup and the next round's selection in one kernel
            # (every round not followed by a commit); select / backup: the other rounds
            names = ["select", "network", "backup", "commit", "backup_select"]
            kernels = {}
            for i, nm in enumerate(names):
                ms = kt[i][0] - base_ms[i][0]
                n = kt[i][1] - base_ms[i][1]
                kernels[nm] = {"ms_timed": ms, "launches_timed": n, "avg_us": 1000.0 * ms / n if n else None}
            rounds_run = args.steps * rps
            traffic = load_traffic(args.traffic_json)
            roof_all = {}
            net = kernels["network"]
            if net["launches_timed"]:
                per_launch = timed_evals / net["launches_timed"]
                achieved = per_launch * flops_per_eval / (net["avg_us"] * 1e-6) / 1e12
                fused = precision in ("fast", "accurate", "corrected") and cfg["arch"] == "b6c96"
                # MFMA work per model product, in fp16-MFMA equivalents: split pairs 3, corrected
                # 1 fp16 + 2 cross terms on e4m3 MFMAs at twice the rate
                mfma_factor = {"accurate": 3, "corrected": 2}.get(precision, 1)
                roof_all["network"] = {
                    "kernel": "kNNForward (fused %s forward)" % cfg["arch"] if fused else
                              "kConvL/kGpoolBias/kHeadsL (layered %s forward, one launch group)" % cfg["arch"],
                    "bound": "mfma", "achieved": achieved, "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_F16_TFLOPS,
                    # PMC bytes of this precision's instance (profiles/traffic_latest.json), else null
                    "traffic": traffic.get("network_bytes_per_launch" + ("" if precision == "fast" else "_" + precision))
                               if fused and args.config == "C2" else None,
                    "evals_per_launch": per_launch, "flops_per_eval": flops_per_eval,
                    "mfma_per_product": mfma_factor, "avg_launch_us": net["avg_us"],
                    "timed_launches": net["launches_timed"],
                    # the game groups' launches overlap, so a launch's own rate understates the
                    # chip's: all network evaluations of the window x FLOP / the window
                    "chip_level": {"achieved": d["nn_evals"] / world / elapsed * flops_per_eval / 1e12,
                                   "frac": d["nn_evals"] / world / elapsed * flops_per_eval / 1e12 / PEAK_F16_TFLOPS,
                                   "concurrent_groups": args.groups}}
                if fused:
                    # a fused launch runs one workgroup per CU (5 boards each when the batch bound
                    # fits 5 per CU, else 8; nn.hip NNEngine::forward): its peak is that share of
                    # the chip's, which the kernel's own efficiency is measured against
                    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
                    cap = (args.nn_batch_cap // args.groups if args.nn_batch_cap else
                           (cus * 8 // args.groups if precision == "fast" else min(cus * 5, cus * 8 // args.groups)))
                    bound = min(-(-games // args.groups), cap)  # the launch's grid bound (selfplay.cpp step)
                    nb = 8 if precision == "fast" and bound > 5 * cus else 5
                    wgs = int(math.ceil(per_launch / nb))
                    share = min(1.0, wgs / cus)
                    roof_all["network"]["occupied_cu_share"] = {
                        "workgroups_per_launch": wgs, "boards_per_workgroup": nb, "cus": cus,
                        "peak": PEAK_F16_TFLOPS * share, "frac": achieved / (PEAK_F16_TFLOPS * share)}
            # tree roofline: per descent, sum over path nodes of 32 B + k * 48 B,
            # counted on the device (tree_levels, tree_children)
            tree_bytes = NODE_B * d["tree_levels"] + CHILD_B * d["tree_children"]
            for nm in ("select", "backup", "backup_select"):
                k = kernels[nm]
                if k["launches_timed"] and rounds_run:
                    # the fused kernel walks two paths per game: one backup, one descent
                    per_launch_b = tree_bytes / rounds_run * (2 if nm == "backup_select" else 1)
                    ach = per_launch_b / (k["avg_us"] * 1e-6) / 1e9
                    roof_all[nm] = {"kernel": {"select": "kSelect", "backup": "kBackup"}.get(nm, "kBackupSelect"),
                                    "bound": "hbm",
                                    "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                                    "traffic": traffic.get("%s_bytes_per_launch" % nm) if args.config == "C2" else None,
                                    "algorithmic_bytes_per_launch": per_launch_b,
                                    "path_nodes_per_playout": d["tree_levels"] / max(1, d["playouts"]),
                                    "children_per_path_node": d["tree_children"] / max(1, d["tree_levels"]),
                                    "avg_launch_us": k["avg_us"]}
            # every kind is timed on the same every-N-th-launch schedule: summed timed ms ranks them
            total_ms = {nm: kernels[nm]["ms_timed"] for nm in names}
            dominant = max(("network", "select", "backup", "backup_select"),
                           key=lambda nm: total_ms[nm] if nm in roof_all else -1)
            roof = dict(roof_all.get(dominant, {}))
            if roof:
                roof["timing"] = "HIP events on the engine stream around every %d-th launch" % args.timing_every
            cpu = None
            if with_cpu and world == 1 and not args.no_cpu_baseline:
                cpu = cpu_baseline(args, cfg, model_path)
            # whole-job rows written (every rank's, on disk before the clock stopped)
            rows_per_sec = rows_gathered / elapsed if window == "steady" else d["moves"] / elapsed
            out = {
                "metric": "self-play training rows/sec + MCTS playouts/sec, 5x5 Coffee b6c96 @600 visits",
                "value": rows_per_sec,
                "unit": "rows/s",
                "value_kind": "rows written per second (steady state)" if window == "steady" else
                              "committed moves per second (window shorter than one game: rows/s in steady state)",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": 1000.0 * elapsed / args.steps,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": {"accurate": "fp16x2 (split hi/lo)",
                          "corrected": "fp16 + e4m3 cross terms"}.get(precision, "fp16"),
                "data": "synthetic: self-play from empty %dx%d boards, random-init %s (seed 0xC0FFEE)" % (X, Y, cfg["arch"]),
                "config": {"workload": cfg["label"] + (" (%d games, %d visits)" % (games, visits)
                                                       if (games, visits) != (cfg["games"], cfg["visits"]) else ""),
                           "config": args.config, "games_per_gpu": games, "visits": visits, "arch": cfg["arch"],
                           "board": "%dx%d win %d" % (X, Y, W), "precision": precision,
                           "network_path": "fused" if precision in ("fast", "accurate", "corrected") and cfg["arch"] == "b6c96"
                           else "layered",
                           "rounds_per_step": rps, "window": window, "game_rounds_estimate": game_rounds,
                           "warmup_rounds": warm_rounds, "commit_interval": args.commit_interval,
                           "nn_cache_log2": args.nn_cache_log2, "nn_batch_cap": args.nn_batch_cap or "engine default",
                           "play_settings": args.play + (" + policy openings (area prop %g)" % args.opening_prop
                                                         if args.opening_prop > 0 else ""),
                           "start_stagger_rounds": stagger, "groups": args.groups,
                           "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "node_cap": node_cap or "default",
                           "parallelism": ("game-sharded x%d (%s)" % (world, "rows written per rank, no collective in "
                                                                         "the loop" if local_sink else "RCCL row gather "
                                                                         "to rank 0")) if world > 1 else "1 GPU"},
                "rccl_world_size": world,
                "rows_per_rank": rank_rows,
                "playouts_per_sec": d["playouts"] / elapsed,
                "moves_per_sec": d["moves"] / elapsed,
                "nn_evals_per_sec": d["nn_evals"] / elapsed,
                "rows_drained": rows_gathered,
                "rows_written_npz": npz_rows if writer else None,
                "model_reloads": reloads,
                "rows_written_npz_per_sec": (npz_rows / elapsed) if writer else None,
                "npz_files": npz_files if writer else None,
                # node-pool / edge-pool headroom of the run (the edge pool is sized
                # by a heuristic; its peak use is reported beside its capacity)
                "edge_pool": {"peak_entries": s1["edge_pool_peak"], "cap_entries": s1["edge_pool_cap"]},
                # the default precision's audit on self-play's own batches (corrected instance only)
                "nn_audit": {"audited_launches": s1["nn_audits"], "max_abs_diff_vs_accurate": s1["nn_audit_max_diff"],
                             "switches_to_accurate": s1["nn_audit_switches"]},
                "kernels": kernels,
                "roofline": roof or None,
                "roofline_all": roof_all,
                "cpu_baseline": cpu,
            }
            sp.close()
            return out
        sp.close()
        return None

    out = measure(args.precision, True)

    def side_window(comp, tolerance):
        return {"precision": "default -> %s" % comp["config"]["precision"], "dtype": comp["dtype"],
                "value": comp["value"], "unit": comp["unit"],
                "value_kind": comp["value_kind"], "ms_per_step": comp["ms_per_step"],
                "playouts_per_sec": comp["playouts_per_sec"], "rows_written_npz": comp["rows_written_npz"],
                "tolerance": tolerance, "nn_audit": comp["nn_audit"], "roofline": comp["roofline"],
                "kernels": comp["kernels"]}

    compliant = out if args.precision == "default" else None
    if args.compliant_line and args.precision == "fast":
        # the north-star tolerance (logits within 1e-3 of fp32 on any net, trained ones
        # included) holds for the default precision (corrected or accurate: the engine's
        # load-time calibration decides), not for fp16 operands on a trained net (DESIGN.md
        # 3a): its window is measured here too and reported beside the headline
        comp = measure("default", False)
        if rank == 0:
            compliant = comp
            out["compliant"] = side_window(comp, "logits within 1e-3 absolute of fp32 (tests/test_gpu_train.py, "
                                            "tests/test_gpu_nn.py)")
            h = kc.Network(model_path, X, Y, W, precision="default")
            out["compliant"]["calibration_max_abs_diff"] = h.precision[1]
            h.close()
    if args.trained_steps > 0:
        # the same precision on a trained net: the calibration then decides on the nets
        # production loads (cpp/program/setup.cpp:240-248 useFP16 auto)
        tpath = os.path.join(tmpdir, "trained_%s.cfnn" % cfg["arch"])
        info = None
        if rank == 0:
            info = trained_model(kc, torch, cfg, args.trained_steps, model_path, tpath, 0xC0FFEE)
        if dist is not None:  # every rank evaluates rank 0's net
            data = kcweights.broadcast_model(tpath, dist, torch.device("cuda", local))
            if rank != 0:
                open(tpath, "wb").write(data)
        comp = measure("default", False, tpath)
        if rank == 0:
            out["compliant_trained"] = side_window(comp, "logits within 1e-3 absolute of fp32 "
                                                    "(tests/test_gpu_train.py, trained b6c96)")
            out["compliant_trained"]["trained_net"] = info
    if rank == 0:
        if args.precision == "fast":
            out["precision_note"] = ("headline at fp16 operands (the configs' fp16/bf16 class): within 1e-3 of fp32 on "
                                     "this random-init benchmark net (tests/test_gpu_nn.py), not on trained nets; "
                                     "'compliant' is the product's default (1e-3) precision, the speed-up basis")
        cpu = out.get("cpu_baseline")
        if cpu and cpu["value"] > 0:
            # the product's 1e-3 path against the whole host's physical cores;
            # the headline's and the CPU share's ratios beside it
            basis = compliant if compliant is not None else out
            out["speedup_vs_cpu"] = basis["value"] / cpu["whole_host"]["value"]
            out["speedup_vs_cpu_basis"] = "%s window vs the whole host's physical cores (%s)" % (
                "compliant (default precision)" if compliant is not None and compliant is not out else
                "headline (%s)" % args.precision, cpu["whole_host"]["kind"])
            out["speedup_vs_cpu_headline"] = out["value"] / cpu["whole_host"]["value"]
            out["speedup_vs_cpu_share"] = basis["value"] / cpu["value"]
        print(json.dumps(out), flush=True)
    shutil.rmtree(tmpdir, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
