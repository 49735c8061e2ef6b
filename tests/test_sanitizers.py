"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer
(sanitizers on the CPU build; the survey found the reference's own encoder
overflow this way, cpp/game/board.cpp:400).  tests/san/Makefile builds

  * host_check: the product's host code -- CFNN model I/O (model.cpp), the .npz row
    writer (npzwrite.cpp), geometry / Zobrist tables (tables.cpp, refrand.cpp) and the
    CLI config layer (cli_config.h) -- host side only (hipcc -Xarch_host -fsanitize=...);
  * liboracle_san.so: the oracle (test infrastructure) with gcc's sanitizers, driven
    from python with the ASan runtime preloaded;
  * katago_tsan / bench_writer_tsan: the host programs' threads under ThreadSanitizer
    (the reference's threads: command/selfplay.cpp:271-394 game/server threads and the
    model poll; selfplaymanager.cpp:330) -- the CLI with several engine threads per
    device, the shared models-directory watch (a hot reload mid-run: real CFNN files
    through the product's loader), the game counter, the log and SIGTERM; bench.py's
    engine loop with its .npz writer thread, rows drained or staged -- over the
    PRODUCT's host code, instrumented: capi.cpp (C ABI, thread-local errors, the
    process-wide device-table cache), selfplay.cpp (engine, round loop, timing events,
    drain / stage / game records, model switch), model.cpp, tables.cpp, refrand.cpp and
    npzwrite.cpp, on san/fake_device.cpp (host memory for the GPU, stand-in kernels).

Any sanitizer report aborts the run (-fno-sanitize-recover=all), so every check here is
"exit status 0 and the expected output".  No GPU is touched."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SAN = os.path.join(HERE, "san")
HOST = os.path.join(SAN, "_build", "host_check")
ORA = os.path.join(SAN, "_build", "liboracle_san.so")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j4", "-C", SAN], check=True)


def _run(args, **kw):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.update(kw.pop("env", {}))
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=600, **kw)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_model_io_under_sanitizers(built, tmp_path):
    """Write / load / re-write every architecture byte-exact; every truncation is
    rejected; corrupted header sizes are rejected before any tensor is sized."""
    out = _run([HOST, "models", str(tmp_path)])
    assert out.count("8/8 prefixes rejected") == 5, out


def test_npz_writer_under_sanitizers(built, tmp_path):
    out = _run([HOST, "npz", str(tmp_path)])
    assert "npz ok" in out
    shapes = {"binaryInputNCHWPacked": (np.uint8, lambda X, Y: (15, (X * Y + 7) // 8)),
              "globalInputNC": (np.float32, lambda X, Y: (1,)),
              "policyTargetsNCMove": (np.int16, lambda X, Y: (2, 4 * X * Y)),
              "globalTargetsNC": (np.float32, lambda X, Y: (64,)),
              "valueTargetsNCHW": (np.int8, lambda X, Y: (5, Y, X))}
    for X, Y in [(5, 5), (7, 7), (9, 9), (6, 4)]:
        for n in (0, 1, 37):
            base = os.path.join(str(tmp_path), "r_%d_%d_%d" % (X, Y, n))
            with np.load(base + ".npz") as z:
                assert sorted(z.files) == sorted(shapes)
                for k, (dt, shp) in shapes.items():
                    raw = np.fromfile(base + ".%s.bin" % k, dtype=dt).reshape((n,) + shp(X, Y))
                    assert z[k].dtype == dt and z[k].shape == raw.shape
                    np.testing.assert_array_equal(z[k], raw)


def test_tables_under_sanitizers(built):
    assert "tables ok" in _run([HOST, "tables"])


def test_cli_config_parser_under_sanitizers(built, tmp_path):
    good = tmp_path / "good.cfg"
    good.write_text("# selfplay1.cfg-like\nbSizes = 7,9,9 # first entry\nwinLen=5\n numGameThreads = 1024\n"
                    "maxVisits = 800\ncpuctExploration = 1.25\nrootNoiseEnabled = false\nnnPrecision = accurate\n"
                    "recordTreePositions = true\nnot a key value line\n= no key\nnumGpus=2\n"
                    "numNNServerThreadsPerModel = 3\nnnCacheSizePowerOfTwo = -4\n")
    bad_int = tmp_path / "bad_int.cfg"
    bad_int.write_text("maxVisits = 80x0\n")
    bad_float = tmp_path / "bad_float.cfg"
    bad_float.write_text("cpuctExploration = fast\n")
    bad_size = tmp_path / "bad_size.cfg"
    bad_size.write_text("bSizes = ,5\n")
    bad_prec = tmp_path / "bad_prec.cfg"
    bad_prec.write_text("nnPrecision = bf16\n")
    huge = tmp_path / "huge.cfg"
    huge.write_text("numGameThreads = 99999999999999999999\n" + "x = " + "y" * 100000 + "\n")
    files = [good, bad_int, bad_float, bad_size, bad_prec, huge, tmp_path / "missing.cfg"]
    lines = _run([HOST, "config"] + [str(f) for f in files]).strip().splitlines()
    got = dict(line.split(": ", 1) for line in lines)
    assert got[str(good)] == ("x=7 y=7 win=5 games=1024 gpus=2 servers=3 rows=10000 cache=0 prec=1 visits=800 "
                              "cpuct=1.2500 noise=0 tree=1")
    assert "maxVisits" in got[str(bad_int)] and got[str(bad_int)].startswith("error")
    assert "cpuctExploration" in got[str(bad_float)]
    assert "bSizes" in got[str(bad_size)]
    assert "nnPrecision" in got[str(bad_prec)]
    assert "numGameThreads" in got[str(huge)]
    assert got[str(tmp_path / "missing.cfg")] == "unreadable"


ORACLE_SCRIPT = r"""
import numpy as np
import katacoffee_amd as kc
from oracle import oracle
rng = np.random.default_rng(5)
for (X, Y, W) in [(5, 5, 4), (6, 4, 3), (7, 7, 5), (9, 9, 5), (10, 10, 5)]:
    n, A = 64, X * Y
    colors = rng.integers(0, 3, (n, A)).astype(np.uint8)
    lc = rng.integers(-1, A, n).astype(np.int8)
    ld = np.where(lc < 0, 4, rng.integers(0, 4, n)).astype(np.int8)
    pla = rng.integers(1, 3, n).astype(np.uint8)
    legal, has = oracle.rules_batch(X, Y, W, colors, lc, ld, pla)
    mv = np.array([np.flatnonzero(l)[0] if l.any() else 0 for l in legal], np.int32)
    oracle.play_batch(X, Y, W, colors[has == 1], lc[has == 1], ld[has == 1], pla[has == 1], mv[has == 1])
    hc = np.where(rng.random((n, 5)) < 0.7, rng.integers(0, A, (n, 5)), -1).astype(np.int8)
    hd = np.where(hc >= 0, rng.integers(0, 4, (n, 5)), 4).astype(np.int8)
    binp, glob = oracle.encode_batch(X, Y, W, colors, hc, hd, pla, rng.integers(0, 8, n).astype(np.int32))
    oracle.fake_net(X, Y, W, binp)
kc.write_random_model("b2c32nbt", 3, "MODEL")
m = oracle.Model("MODEL")
for X, Y, W in [(5, 5, 4), (7, 7, 5)]:
    binp, glob = oracle.encode_batch(X, Y, W, np.zeros((3, X * Y), np.uint8), np.full((3, 5), -1, np.int8),
                                     np.full((3, 5), 4, np.int8), np.ones(3, np.uint8), np.arange(3, dtype=np.int32))
    for mode in (0, 1, 2):
        m.forward(X, Y, binp, glob.reshape(3, 1), mode=mode, threads=2)
for (X, Y, W), model in [((5, 5, 4), None), ((9, 9, 5), None), ((5, 5, 4), m)]:
    sp = oracle.Selfplay(X, Y, W, games=4, max_visits=16, node_cap=64, seed=3, nn_cache_log2=6, nn_batch_cap=3,
                         nn_mode=1 if model else 0, model=model,
                         cheap_search_prob=0.5, cheap_search_visits=4, reduce_visits=1, reduced_visits_min=4,
                         policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1, init_games_with_policy=1,
                         early_fork_game_prob=0.5, fork_game_prob=0.5, side_position_prob=0.3,
                         record_tree_positions=1, record_tree_threshold=2, record_tree_target_weight=0.5)
    sp.rounds(500)
    for g in range(4):
        sp.game_tree(g)
        sp.nodes(g, cap=64)
        sp.root_noised(g)
    print("selfplay", X, Y, len(sp.rows()["meta"]))
print("oracle ok")
"""


def test_oracle_under_sanitizers(built, tmp_path):
    """The checker itself: rules, play, encoder, stand-in net, NN forward (both modes,
    nested bottlenecks) and self-play with every variety feature at 5x5 and 9x9."""
    asan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    script = ORACLE_SCRIPT.replace("MODEL", str(tmp_path / "m.cfnn"))
    out = _run([sys.executable, "-c", script], cwd=REPO,
               env={"LD_PRELOAD": asan, "ORACLE_LIB": ORA, "PYTHONPATH": REPO})
    assert "oracle ok" in out and out.count("selfplay") == 3, out


def _tsan(args, **kw):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    env.update(kw.pop("env", {}))
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=600, **kw)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    return r


@pytest.mark.parametrize("mode", ["drain", "stage"])
def test_bench_writer_threads_under_tsan(built, tmp_path, mode):
    r = _tsan([os.path.join(SAN, "_build", "bench_writer_tsan"), str(tmp_path), "2", "30", mode])
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "written in 30 files" in r.stdout, r.stdout
    files = sorted(f for f in os.listdir(tmp_path) if f.endswith(".npz"))
    assert len(files) == 30
    with np.load(os.path.join(str(tmp_path), files[-1])) as z:
        assert z["binaryInputNCHWPacked"].shape[1:] == (15, 4) and z["globalInputNC"].shape[0] > 0


def _models(d, names):
    import katacoffee_amd as kc
    d.mkdir()
    for i, n in enumerate(names):
        kc.write_random_model("b2c32nbt", 7 + i, str(d / (n + ".cfnn")))


def test_cli_threads_under_tsan(built, tmp_path):
    """2 devices x 2 engines, a newer model appearing mid-run (every engine switches and
    writes under the new name), then -max-games-total stops all engines."""
    import threading
    import time
    models = tmp_path / "models"
    _models(models, ["netA"])
    staged = tmp_path / "staged"
    _models(staged, ["netB"])
    out = tmp_path / "out"

    def drop_new_model():
        time.sleep(1.5)
        os.replace(staged / "netB.cfnn", models / "netB.cfnn")
        os.utime(models / "netB.cfnn", (time.time() + 5, time.time() + 5))

    t = threading.Thread(target=drop_new_model)
    t.start()
    cmd = [os.path.join(SAN, "_build", "katago_tsan"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "60000", "-override-config",
           "numGameThreads=64,numGpus=2,numNNServerThreadsPerModel=4,maxRowsPerTrainFile=500,modelPollSeconds=0.05"]
    r = _tsan(cmd)
    t.join()
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    log = r.stdout
    for g in ("0.0", "0.1", "1.0", "1.1"):
        assert "gpu %s done" % g in log, log[-3000:]
        assert "gpu %s: switched to model" % g in log, log[-3000:]
    for name in ("netA", "netB"):
        assert os.listdir(out / name / "tdata"), name
        assert os.listdir(out / name / "sgfs"), name


def test_cli_sigterm_under_tsan(built, tmp_path):
    """SIGTERM (selfplay.cpp:22-29): every engine thread flushes its rows and exits 0."""
    import signal
    import time
    models = tmp_path / "models"
    _models(models, ["netA"])
    out = tmp_path / "out"
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.Popen([os.path.join(SAN, "_build", "katago_tsan"), "selfplay", "-config",
                          os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models),
                          "-output-dir", str(out), "-override-config",
                          "numGameThreads=64,numGpus=2,numNNServerThreadsPerModel=2,maxRowsPerTrainFile=100000"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    time.sleep(2.0)
    p.send_signal(signal.SIGTERM)
    so, se = p.communicate(timeout=120)
    assert "ThreadSanitizer" not in se, se[-6000:]
    assert p.returncode == 0, so[-2000:] + se[-2000:]
    assert "gpu 0.0 done" in so and "gpu 1.0 done" in so
    assert os.listdir(out / "netA" / "tdata")  # the pending rows were flushed


def test_tsan_harness_sees_the_product_cache(built, tmp_path):
    """Negative control: the same CLI run over a copy of capi.cpp whose device-table cache
    lock (kc::tablesFor, the cache every engine thread shares) is removed must be reported
    by ThreadSanitizer -- the harness instruments the product's host code itself."""
    cs = os.path.join(REPO, "katacoffee_amd", "csrc")
    src = open(os.path.join(cs, "capi.cpp")).read()
    lock = "  std::lock_guard<std::mutex> lk(gTablesMu);\n"
    assert src.count(lock) == 1
    racy = tmp_path / "capi_racy.cpp"
    racy.write_text(src.replace(lock, ""))
    obj = tmp_path / "capi_racy.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-std=c++17", "-O1", "-g", "-fPIC",
                    "-ffp-contract=off", "-Xarch_host", "-fsanitize=thread", "-Xarch_host", "-fno-omit-frame-pointer",
                    "-I", cs, "-c", str(racy), "-o", str(obj)], check=True)
    tobj = os.path.join(SAN, "_build", "t")
    others = [os.path.join(tobj, f) for f in sorted(os.listdir(tobj)) if f.endswith(".o") and f != "capi.o"]
    exe = tmp_path / "katago_racy"
    subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "-std=c++17", "-O1", "-g", "-fPIC", "-fsanitize=thread", "-o",
                    str(exe), os.path.join(cs, "cli_selfplay.cpp"), str(obj)] + others + ["-lpthread"], check=True)
    models = tmp_path / "models"
    _models(models, ["netA"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), "selfplay", "-config", os.path.join(REPO, "configs", "selfplay_coffee5.cfg"),
                        "-models-dir", str(models), "-output-dir", str(tmp_path / "out"), "-max-games-total", "2000",
                        "-override-config", "numGameThreads=64,numGpus=2,numNNServerThreadsPerModel=4"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert "ThreadSanitizer: data race" in r.stderr and "tablesFor" in r.stderr, r.stderr[-3000:]
