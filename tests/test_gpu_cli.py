"""`katago selfplay` (the process boundary, command/selfplay.cpp:44-72): runs the CLI
for a few games and reads its .npz output back with numpy, like python/train.py."""
import glob
import os
import subprocess

import numpy as np
import pytest

import katacoffee_amd as kc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cli_selfplay_writes_training_npz(tmp_path):
    models = tmp_path / "models"
    models.mkdir()
    kc.write_random_model("b6c96", 5, str(models / "b6c96-s0.cfnn"))
    out = tmp_path / "out"
    cmd = [os.path.join(REPO, "katacoffee_amd", "katago"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "40", "-override-config", "numGameThreads=64,maxVisits=16,maxRowsPerTrainFile=100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    files = glob.glob(str(out / "b6c96-s0" / "tdata" / "*.npz"))
    assert files, r.stdout
    assert glob.glob(str(out / "log*.log"))
    total = 0
    for f in files:
        with np.load(f) as z:
            n = z["globalTargetsNC"].shape[0]
            assert 0 < n <= 100
            assert z["binaryInputNCHWPacked"].shape == (n, 15, 4) and z["binaryInputNCHWPacked"].dtype == np.uint8
            assert z["globalInputNC"].shape == (n, 1)
            assert z["policyTargetsNCMove"].shape == (n, 2, 100) and z["policyTargetsNCMove"].dtype == np.int16
            assert z["valueTargetsNCHW"].shape == (n, 5, 5, 5) and z["valueTargetsNCHW"].dtype == np.int8
            np.testing.assert_array_equal(z["globalTargetsNC"][:, 63], 1.0)
            assert z["policyTargetsNCMove"][:, 0].sum(axis=1).min() > 0
            total += n
    assert total >= 40 * 5  # every finished game has at least five moves


def test_cli_two_engines_per_gpu(tmp_path):
    """numNNServerThreadsPerModel = 2 on one GPU: two engines (own streams, batches and
    caches) split the GPU's games and both write rows and records."""
    models = tmp_path / "models"
    models.mkdir()
    kc.write_random_model("b6c96", 5, str(models / "b6c96-s0.cfnn"))
    out = tmp_path / "out"
    cmd = [os.path.join(REPO, "katacoffee_amd", "katago"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "40", "-override-config",
           "numGameThreads=64,maxVisits=16,maxRowsPerTrainFile=100,numNNServerThreadsPerModel=2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    log = r.stdout + r.stderr
    assert "gpu 0.0 done" in log and "gpu 0.1 done" in log, log
    files = glob.glob(str(out / "b6c96-s0" / "tdata" / "*.npz"))
    assert files, log
    total = 0
    for f in files:
        with np.load(f) as z:
            total += z["globalTargetsNC"].shape[0]
    assert total >= 40 * 5
    games = _sgf_games(glob.glob(str(out / "b6c96-s0" / "sgfs" / "*.sgfs")))
    ids = {g.split("gameId=")[1].split(":")[0] for g in games}
    assert any(int(i) < 32 for i in ids) and any(int(i) >= 32 for i in ids), ids


def _sgf_games(paths):
    games = []
    for p in paths:
        with open(p) as f:
            games += [line.strip() for line in f if line.strip()]
    return games


def _replay_sgf(g, X, Y, W):
    """Plays an SGF line's moves with the oracle's rules; returns (moves, final winner, RE)."""
    import re
    from oracle import oracle
    assert g.startswith("(;FF[4]GM[Coffee]SZ[%d]WLL[%d]" % (X, W)) and g.endswith(")")
    re_res = re.search(r"RE\[([^\]]*)\]", g).group(1)
    moves = re.findall(r";([BW])\[([a-z])([a-z])([a-d])\]", g)
    colors = np.zeros((1, X * Y), np.uint8)
    last_cell, last_dir, pla, winner = np.array([-1], np.int8), np.array([4], np.int8), np.array([1], np.uint8), 0
    for i, (c, xs, ys, ds) in enumerate(moves):
        assert c == ("B" if i % 2 == 0 else "W")
        cell, d = (ord(ys) - 97) * X + (ord(xs) - 97), ord(ds) - 97
        mv = np.array([d * X * Y + cell], np.int32)
        legal, _ = oracle.rules_batch(X, Y, W, colors, last_cell, last_dir, pla)
        assert legal[0, mv[0]], (g, i)
        res = oracle.play_batch(X, Y, W, colors, last_cell, last_dir, pla, mv)
        colors = res["colors"]
        last_cell, last_dir, pla = np.array([cell], np.int8), np.array([d], np.int8), 3 - pla
        finished, winner = int(res["finished"][0]), int(res["winner"][0])
        assert finished == (i + 1 == len(moves)), (g, i)
    return len(moves), winner, re_res


def test_cli_writes_sgfs_and_hot_reloads(tmp_path):
    import time
    models = tmp_path / "models"
    models.mkdir()
    kc.write_random_model("b6c96", 5, str(models / "net-a.cfnn"))
    out = tmp_path / "out"
    cmd = [os.path.join(REPO, "katacoffee_amd", "katago"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "2500", "-override-config",
           "numGameThreads=64,maxVisits=64,maxRowsPerTrainFile=100,modelPollSeconds=0.5"]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        deadline = time.time() + 240
        while time.time() < deadline and not glob.glob(str(out / "net-a" / "sgfs" / "*.sgfs")):
            time.sleep(0.5)
        time.sleep(1.5)  # a newer file: the watcher picks it up on its next poll
        kc.write_random_model("b6c96", 6, str(models / "net-b.cfnn.tmp"))
        os.replace(str(models / "net-b.cfnn.tmp"), str(models / "net-b.cfnn"))
        stdout, _ = p.communicate(timeout=240)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, stdout
    assert "switched to model" in stdout, stdout
    assert glob.glob(str(out / "net-b" / "tdata" / "*.npz")) or glob.glob(str(out / "net-b" / "sgfs" / "*.sgfs"))
    games = _sgf_games(glob.glob(str(out / "*" / "sgfs" / "*.sgfs")))
    assert len(games) >= 2500
    for g in games[:60]:
        n, winner, res = _replay_sgf(g, 5, 5, 4)
        assert res == {1: "B+", 2: "W+", 0: "0"}[winner]
        if winner:
            assert n >= 7  # a connect-4 win needs at least 7 stones on the board


def test_cli_production_play_settings(tmp_path):
    """The selfplay1.cfg play settings through the CLI: rows are weighted (cheap
    searches mostly write none), fork games and side-position rows appear, and every
    SGF still replays legally from the empty board."""
    models = tmp_path / "models"
    models.mkdir()
    kc.write_random_model("b6c96", 7, str(models / "net.cfnn"))
    out = tmp_path / "out"
    cmd = [os.path.join(REPO, "katacoffee_amd", "katago"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay1_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "300", "-override-config",
           "numGameThreads=64,maxVisits=24,cheapSearchVisits=8,reducedVisitsMin=8,maxRowsPerTrainFile=200,"
           "sidePositionProb=0.2,earlyForkGameProb=0.3,forkGameProb=0.2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    gts = []
    for f in glob.glob(str(out / "net" / "tdata" / "*.npz")):
        with np.load(f) as z:
            gts.append(z["globalTargetsNC"])
    gt = np.concatenate(gts)
    assert len(gt) > 0
    assert (gt[:, 55] == 2.0).any()          # fork games
    assert (gt[:, 27] == 0.0).any()          # side-position rows
    assert gt[:, 60].min() >= 8 and gt[:, 60].max() <= 24
    games = _sgf_games(glob.glob(str(out / "net" / "sgfs" / "*.sgfs")))
    assert len(games) >= 300
    for g in games[:80]:
        _replay_sgf(g, 5, 5, 4)
