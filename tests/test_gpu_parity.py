"""GPU parity: the HIP path (through the C ABI) against the reference fixtures and
the CPU oracle.

  rules / play / hashes : bit-exact vs tests/golden/rules_*.npz (reference cpp/game output)
  encoder               : bit-exact vs the oracle restatement, 8 symmetries
  stand-in network      : bit-exact vs the oracle
  residual network      : |logit diff| <= 1e-3 vs the oracle fp16-emulation mode
                          (same roundings, different f32 accumulation order);
                          vs the fp32 oracle (Eigen-backend semantics) <= 1e-3 (north star)
  self-play (stand-in net): bit-exact game state, canonical search trees, root
                          priors and training rows vs the oracle, round for round
"""
import glob
import os

import numpy as np
import pytest

import katacoffee_amd as kc
from oracle import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = sorted(glob.glob(os.path.join(HERE, "golden", "rules_*.npz")))


def _last_cell(d):
    X = int(d["dims"][0])
    return np.where(d["last_x"] >= 0, d["last_y"] * X + d["last_x"], -1)


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_rules_bit_exact_vs_reference(path):
    d = np.load(path)
    X, Y, W, _ = map(int, d["dims"])
    legal, has = kc.rules_batch(X, Y, W, d["colors"], _last_cell(d), d["last_dir"], d["pla"])
    np.testing.assert_array_equal(legal, d["legal"])
    np.testing.assert_array_equal(has, d["has_legal"])


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_play_win_hash_bit_exact_vs_reference(path):
    d = np.load(path)
    X, Y, W, _ = map(int, d["dims"])
    z = np.load(os.path.join(HERE, "golden", "zobrist.npz"))
    sel = d["move_pos"] >= 0
    mp = d["move_pos"][sel]
    cells, fin, win, mr, ph, sh = kc.play_batch(X, Y, W, d["colors"][sel], _last_cell(d)[sel], d["last_dir"][sel],
                                                d["pla"][sel], mp)
    after, ha = d["after"][sel], d["hash_after"][sel]
    np.testing.assert_array_equal(mr, after[:, 2])
    np.testing.assert_array_equal(ph, ha[:, 0:2])
    won = after[:, 0] == 1
    assert np.all(fin[won] == 1)
    np.testing.assert_array_equal(win[won], after[won, 1])
    assert np.all(win[~won] == 0)
    # placed stone
    A = X * Y
    np.testing.assert_array_equal(cells[np.arange(len(mp)), mp % A], d["pla"][sel])
    # transposition key = reference sitHash ^ ZOBRIST_BOARD_HASH2[last move] ^ (game over)
    cell, dr = mp % A, mp // A
    spot = (cell % X + 1) + (cell // X + 1) * (X + 1)
    st = sh ^ z["board2"][spot, dr]
    st = np.where(fin[:, None] == 1, st ^ z["game_over"][None, :], st)
    np.testing.assert_array_equal(st, ha[:, 2:4])
    # and equals the oracle's key
    o = oracle.play_batch(X, Y, W, d["colors"][sel], _last_cell(d)[sel], d["last_dir"][sel], d["pla"][sel], mp)
    np.testing.assert_array_equal(sh, o["state_hash"])
    np.testing.assert_array_equal(fin, o["finished"])


def _positions_with_history(path, limit=600):
    d = np.load(path)
    X, Y, W, _ = map(int, d["dims"])
    n = min(limit, len(d["game"]))
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    for i in range(n):
        k = 0
        j = i - 1
        while k < 5 and j >= 0 and d["game"][j] == d["game"][i]:
            mv = d["move_pos"][j]
            hc[i, k] = mv % (X * Y)
            hd[i, k] = mv // (X * Y)
            k += 1
            j -= 1
    return d, X, Y, W, n, hc, hd


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_encoder_bit_exact_vs_oracle(path):
    d, X, Y, W, n, hc, hd = _positions_with_history(path)
    rng = np.random.default_rng(0)
    sym = rng.integers(0, 8, n).astype(np.int32)
    packed, planes = kc.encode_batch(X, Y, W, d["colors"][:n], hc, hd, d["pla"][:n], sym)
    ob, og = oracle.encode_batch(X, Y, W, d["colors"][:n], hc, hd, d["pla"][:n], sym)
    np.testing.assert_array_equal(planes, ob)
    np.testing.assert_array_equal(og, W)
    # packed bits agree with the planes (bit i = plane*A + cell)
    A = X * Y
    bits = np.unpackbits(packed.view(np.uint8), axis=1, bitorder="little")[:, :15 * A]
    np.testing.assert_array_equal(bits.reshape(n, 15, A), planes.astype(np.uint8))


def test_fake_net_bit_exact_vs_oracle():
    d, X, Y, W, n, hc, hd = _positions_with_history(GOLD[[i for i, p in enumerate(GOLD) if "5x5" in p][0]], 300)
    sym = np.zeros(n, np.int32)
    packed, planes = kc.encode_batch(X, Y, W, d["colors"][:n], hc, hd, d["pla"][:n], sym)
    np.testing.assert_array_equal(kc.fake_net(X, Y, W, packed), oracle.fake_net(X, Y, W, planes))


@pytest.fixture(scope="module")
def model_path(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("m") / "b6c96.cfnn")
    kc.write_random_model("b6c96", 0xC0FFEE, p)
    return p


def test_network_logits_vs_oracle(model_path):
    path = [p for p in GOLD if "5x5" in p][0]
    d, X, Y, W, n, hc, hd = _positions_with_history(path, 203)  # ragged: not a multiple of 8 boards
    sym = np.random.default_rng(1).integers(0, 8, n).astype(np.int32)
    packed, planes = kc.encode_batch(X, Y, W, d["colors"][:n], hc, hd, d["pla"][:n], sym)
    net = kc.Network(model_path, X, Y, W)
    out = net.forward(packed)
    m = oracle.Model(model_path)
    glob_in = np.full((n, 1), float(W), np.float32)
    A = X * Y
    for mode, tol in [(1, 1e-3), (0, 1e-3)]:
        pol, val, misc = m.forward(X, Y, planes, glob_in, mode=mode, threads=8)
        ref = np.concatenate([pol.reshape(n, 4 * A), val, misc], axis=1)
        err = np.abs(out - ref).max()
        print("mode", mode, "max |diff|", err, "max |ref|", np.abs(ref).max())
        assert err <= tol, (mode, err)
    # batch-size independence: evaluating a subset gives identical rows
    np.testing.assert_array_equal(net.forward(packed[:17]), out[:17])
    net.close()


INFO_KEYS = [("phase", "phase"), ("rootK", "rootK"), ("liveCount", "nodeCount"), ("gameNum", "gameNum"),
             ("turn", "turn"), ("pla", "pla"), ("playouts", "playouts"), ("nnEvals", "nnEvals"),
             ("moves", "movesMade"), ("gamesFinished", "gamesFinished"), ("rngCtr", "rngCtr"),
             ("lastCell", "lastCell"), ("lastDir", "lastDir")]


def _sorted_rows(r):
    order = np.lexsort((r["meta"][:, 2], r["meta"][:, 1], r["meta"][:, 0]))
    return {k: v[order] for k, v in r.items()}


# selfplay1.cfg's play settings (cheap searches, reduced visits, surprise-weighted
# rows) with the visit counts scaled to the test's max_visits
PRODUCTION = dict(cheap_search_prob=0.75, cheap_search_visits=10, cheap_search_target_weight=0.0, reduce_visits=1,
                  reduce_visits_threshold=0.9, reduce_visits_threshold_lookback=3, reduced_visits_min=10,
                  reduced_visits_weight=0.1, policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1)
# forks at high rates (selfplay1.cfg: 0.04 / 0.01) so these short runs fork often
FORKS = dict(early_fork_game_prob=0.5, early_fork_game_expected_move_prop=0.2, fork_game_prob=0.5,
             fork_game_min_choices=2, early_fork_game_max_choices=5, fork_game_max_choices=7)
# reduceVisits alone, with a low threshold so the reduction triggers in these short games
REDUCED = dict(reduce_visits=1, reduce_visits_threshold=0.2, reduced_visits_min=8, reduced_visits_weight=0.3)


# The round schedules the tests pin (commit interval, forced fused rounds, staggered
# starts): interval 1 (a move is committed in the round its search ends); the product's
# interval 16 (bench.py, the CLI) with staggered starts on separate kernels, and the same
# with fused rounds (kBackupSelect + kResolve: the bench's fast headline).  Games whose
# root reached its visit limit idle until the commit round; the oracle restates that
# schedule (ora_sp_rounds), so with a shared NN cache -- where a hit depends on the
# other games' timing -- the device is compared with the oracle on the same schedule.
SCHEDULES = [(1, False, 0), (16, False, 37), (16, True, 37)]
SCHEDULE_IDS = ["ci1", "ci16-stagger", "ci16-stagger-fused"]


def _scheduled_engine(sched, X=5, Y=5, W=4, **kw):
    ci, fused, stagger = sched
    return _engine(fused, X, Y, W, commit_interval=ci, start_stagger=stagger, **kw)


# cache_log2: 0 = no NN cache; 5 = a 32-entry cache, so slots are contended and
# overwritten every round (the round-synchronous write order decides the contents);
# 14 = hits across games (SPEC a7).  play: benchmark mode ({}) or selfplay1.cfg-like.
@pytest.mark.parametrize("sched", SCHEDULES, ids=SCHEDULE_IDS)
@pytest.mark.parametrize("games,visits,rounds,seed,cache_log2,play",
                         [(6, 40, 1200, 3, 0, {}), (4, 24, 900, 99, 0, {}), (8, 40, 1400, 3, 5, {}),
                          (12, 32, 1000, 7, 14, {}), (8, 40, 1200, 11, 0, PRODUCTION), (8, 32, 1200, 5, 12, REDUCED),
                          (10, 32, 1400, 13, 12, dict(nn_batch_cap=3)),
                          (8, 32, 1400, 17, 5, dict(PRODUCTION, nn_batch_cap=2)),
                          (8, 32, 1200, 19, 12, dict(PRODUCTION, init_games_with_policy=1)),
                          (8, 24, 1200, 23, 0, dict(init_games_with_policy=1, policy_init_area_prop=0.3,
                                                    policy_init_area_temperature=2.0)),
                          (8, 24, 1600, 29, 12, FORKS),
                          (8, 24, 1800, 43, 0, dict(side_position_prob=0.3)),
                          (8, 24, 1800, 37, 10, dict(PRODUCTION, init_games_with_policy=1, cheap_search_visits=8,
                                                     reduced_visits_min=8, nn_batch_cap=5, side_position_prob=0.2,
                                                     **FORKS)),
                          # the smallest searches: one game at one visit (the root's evaluation
                          # alone picks the move), two games at two visits with a contended cache
                          (1, 1, 300, 31, 0, {}), (2, 2, 400, 41, 5, {})],
                         ids=["bench-a", "bench-b", "cache32", "cache16k", "production", "reduced", "batch-cap",
                              "production-cap", "production-init", "policy-init", "forks", "side-positions",
                              "everything", "one-game-one-visit", "two-visits"])
def test_selfplay_fake_net_bit_exact_vs_oracle(games, visits, rounds, seed, cache_log2, play, sched):
    cap = 128
    if sched[0] > 1:
        rounds *= 2  # idle rounds (commit waits, staggered starts): finish games all the same
    gpu = _scheduled_engine(sched, num_games=games, max_visits=visits, seed=seed, node_cap=cap,
                            nn_cache_log2=cache_log2, row_capacity=1 << 15, **play)
    gpu.enable_timing(1)
    ora = oracle.Selfplay(5, 5, 4, games=games, max_visits=visits, node_cap=cap, seed=seed,
                          nn_cache_log2=cache_log2, commit_interval=sched[0], start_stagger=sched[2], **play)
    done = 0
    for chunk in [1, 4, 20, 61, rounds]:  # step ends fall inside commit intervals too
        step = chunk - done
        if step <= 0:
            continue
        gpu.step(step)
        ora.rounds(step)
        done = chunk
        for g in range(games):
            gi, oi = gpu.game_info(g), ora.info(g)
            for a, b in INFO_KEYS:
                assert gi[a] == oi[b], (done, g, a, gi[a], oi[b])
            gn, ge = gpu.game_tree(g)
            on, oe = ora.game_tree(g)
            np.testing.assert_array_equal(gn, on, err_msg="round %d game %d nodes" % (done, g))
            np.testing.assert_array_equal(ge, oe, err_msg="round %d game %d edges" % (done, g))
            if gi["phase"] == 1:
                np.testing.assert_array_equal(gpu.root_policy(g), ora.root_noised(g))
    st = gpu.stats()
    assert st["games_finished"] > 0 and st["rows_dropped"] == 0
    gr = _sorted_rows(gpu.drain_rows())
    orr = _sorted_rows(ora.rows())
    assert len(gr["meta"]) == len(orr["meta"]) > 0
    for k in orr:
        np.testing.assert_array_equal(gr[k], orr[k], err_msg=k)
    # the schedule ran as named: fused launches (kernel 4) only in the fused schedule
    fused_launches = gpu.kernel_time(4)[1]
    assert (fused_launches > rounds // 2) if sched[1] else (fused_launches == 0), fused_launches
    gpu.close()


def test_selfplay_network_smoke(model_path):
    sp = kc.Selfplay(5, 5, 4, num_games=64, max_visits=16, seed=5, model_path=model_path, commit_interval=4)
    sp.step(800)
    st = sp.stats()
    assert st["playouts"] > 0 and st["nn_evals"] > 0 and st["moves"] > 0
    assert st["games_finished"] > 0
    assert st["errors"] == 0
    r = sp.drain_rows()
    n = len(r["meta"])
    assert n == st["rows_pending"] and n > 0
    assert r["policyTargetsNCMove"][:, 0].sum(axis=1).min() > 0
    np.testing.assert_array_equal(r["globalTargetsNC"][:, 63], 1.0)
    sp.close()


def _engine(fused, X=5, Y=5, W=4, separate_resolve=False, **kw):
    # the engine reads COFFEE_FUSED_ROUNDS / COFFEE_SEPARATE_RESOLVE when it is created
    env = {"COFFEE_FUSED_ROUNDS": "1" if fused else "0", "COFFEE_SEPARATE_RESOLVE": "1" if separate_resolve else "0"}
    old = {k: os.environ.pop(k, None) for k in env}
    os.environ.update(env)
    try:
        return kc.Selfplay(X, Y, W, **kw)
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


# Fused rounds (kBackupSelect + kResolve) against separate kSelect / kBackup launches:
# with commit intervals > 1 most rounds run fused, and a 32-entry cache has nearly every
# lookup hit a slot that the same round's backups write (the kResolve path).  Every game's
# state, search tree and row must be identical.  (Both are also pinned against the oracle
# on the same schedule: test_selfplay_fake_net_bit_exact_vs_oracle's ci16 cases.)
@pytest.mark.parametrize("games,visits,rounds,seed,cache_log2,ci,play,net,geo",
                         [(64, 32, 700, 61, 5, 4, {}, False, (5, 5, 4)),
                          (48, 24, 900, 67, 12, 16, PRODUCTION, False, (5, 5, 4)),
                          (32, 24, 600, 71, 5, 3, dict(FORKS, side_position_prob=0.3), False, (5, 5, 4)),
                          (64, 16, 500, 73, 5, 8, {}, True, (5, 5, 4)),
                          (48, 24, 2400, 79, 6, 4, {}, False, (7, 7, 5)),
                          (32, 24, 3000, 83, 6, 5, PRODUCTION, False, (9, 9, 5))],
                         ids=["cache32-ci4", "production-ci16", "forks-side-ci3", "network-ci8", "7x7-ci4",
                              "9x9-production-ci5"])
def test_fused_rounds_match_separate_kernels(games, visits, rounds, seed, cache_log2, ci, play, net, geo,
                                             model_path):
    X, Y, W = geo
    kw = dict(X=X, Y=Y, W=W, num_games=games, max_visits=visits, seed=seed, node_cap=visits + 96,
              commit_interval=ci, nn_cache_log2=cache_log2, **play)
    if net:
        kw["model_path"] = model_path
    a, b = _engine(True, **kw), _engine(False, **kw)
    a.enable_timing(1)
    b.enable_timing(1)
    done = 0
    for chunk in [5, 37, 200, rounds]:  # step ends fall inside commit intervals too
        a.step(chunk - done)
        b.step(chunk - done)
        done = chunk
        for g in range(games):
            ga, gb = a.game_info(g), b.game_info(g)
            assert ga == gb, (done, g, ga, gb)
            na, ea = a.game_tree(g)
            nb, eb = b.game_tree(g)
            np.testing.assert_array_equal(na, nb, err_msg="round %d game %d nodes" % (done, g))
            np.testing.assert_array_equal(ea, eb, err_msg="round %d game %d edges" % (done, g))
    sa, sb = a.stats(), b.stats()
    assert sa["games_finished"] > 0 and sa["moves"] > 0
    for k in ("playouts", "nn_evals", "moves", "games_finished", "rows_pending"):
        assert sa[k] == sb[k], k
    ra, rb = _sorted_rows(a.drain_rows()), _sorted_rows(b.drain_rows())
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
    assert a.kernel_time(4)[1] > rounds // 2 and b.kernel_time(4)[1] == 0  # fused launches ran in a only
    a.close()
    b.close()


# The pending selections and tag clears of a fused round run inside kCompact's dispatch
# (the default) or in a separate kResolve launch (COFFEE_SEPARATE_RESOLVE=1): the same
# games, trees and rows.  The 32-entry cache sends most lookups down the pending path.
@pytest.mark.parametrize("games,visits,rounds,seed,cache_log2,ci,net",
                         [(64, 32, 700, 61, 5, 4, False), (96, 16, 500, 73, 5, 16, True)],
                         ids=["cache32-ci4", "network-ci16"])
def test_resolve_in_compact_matches_separate_resolve(games, visits, rounds, seed, cache_log2, ci, net, model_path):
    kw = dict(num_games=games, max_visits=visits, seed=seed, node_cap=visits + 96, commit_interval=ci,
              nn_cache_log2=cache_log2)
    if net:
        kw["model_path"] = model_path
    a, b = _engine(True, **kw), _engine(True, separate_resolve=True, **kw)
    done = 0
    for chunk in [37, rounds]:  # the first step ends inside a commit interval
        a.step(chunk - done)
        b.step(chunk - done)
        done = chunk
        for g in range(games):
            assert a.game_info(g) == b.game_info(g), (chunk, g)
            na, ea = a.game_tree(g)
            nb, eb = b.game_tree(g)
            np.testing.assert_array_equal(na, nb, err_msg="round %d game %d nodes" % (chunk, g))
            np.testing.assert_array_equal(ea, eb, err_msg="round %d game %d edges" % (chunk, g))
    sa, sb = a.stats(), b.stats()
    for k in ("playouts", "nn_evals", "moves", "games_finished", "rows_pending"):
        assert sa[k] == sb[k], k
    assert sa["games_finished"] > 0
    ra, rb = _sorted_rows(a.drain_rows()), _sorted_rows(b.drain_rows())
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
    a.close()
    b.close()


def test_game_records_match_rows_and_rules(model_path):
    """Finished-game records (SGF source) agree with the rows of the same games and
    replay legally under the reference-pinned rules to the recorded result."""
    sp = kc.Selfplay(5, 5, 4, num_games=32, max_visits=16, seed=9, model_path=model_path, commit_interval=1)
    parts, hs, ms = [], [], []
    for _ in range(10):  # drain every 250 rounds (record buffer: 2 x num_games)
        sp.step(250)
        parts.append(sp.drain_rows())
        h, m = sp.drain_games()
        hs.append(h)
        ms.append(m)
    rows = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    header, moves = np.concatenate(hs), np.concatenate(ms)
    assert len(header) > 0 and sp.stats()["games_dropped"] == 0
    nmoves = {(int(m[0]), int(m[1])): int(m[3]) for m in rows["meta"]}
    fin = {}
    for m, v in zip(rows["meta"], rows["valueTargetsNCHW"]):
        if int(m[2]) == 0:
            fin[(int(m[0]), int(m[1]))] = v[0]  # final board from Black's (turn 0 mover) view
    for h, mv in zip(header, moves):
        key = (int(h[0]), int(h[1]))
        assert nmoves.get(key) == int(h[2])
        colors = np.zeros((1, 25), np.uint8)
        lc, ld, pla = np.array([-1], np.int8), np.array([4], np.int8), np.array([1], np.uint8)
        for t in range(int(h[2])):
            cell, d = int(mv[t, 0]), int(mv[t, 1])
            legal, _ = oracle.rules_batch(5, 5, 4, colors, lc, ld, pla)
            assert legal[0, d * 25 + cell]
            res = oracle.play_batch(5, 5, 4, colors, lc, ld, pla, np.array([d * 25 + cell], np.int32))
            colors, lc, ld, pla = res["colors"], np.array([cell], np.int8), np.array([d], np.int8), 3 - pla
        assert int(res["finished"][0]) == 1 and int(res["winner"][0]) == int(h[3])
        assert np.all(mv[int(h[2]):] == 0xFF)
        board = np.where(colors[0] == 1, 1, np.where(colors[0] == 2, -1, 0)).reshape(5, 5)
        np.testing.assert_array_equal(board, fin[key])
    # hot reload: a different network takes over for every game; the engine keeps running
    other = model_path.replace(".cfnn", "-other.cfnn")
    kc.write_random_model("b6c96", 77, other)
    sp.set_model(other)
    sp.step(300)
    sp.sync()
    assert sp.stats()["rounds"] == 2800
    with pytest.raises(kc.CoffeeError):
        sp.set_model(model_path + ".missing")
    sp.step(10)
    sp.sync()


def _compare_game(gpu, ora, g, og, done):
    gi, oi = gpu.game_info(g), ora.info(og)
    for a, b in INFO_KEYS:
        assert gi[a] == oi[b], (done, g, a, gi[a], oi[b])
    gn, ge = gpu.game_tree(g)
    on, oe = ora.game_tree(og)
    np.testing.assert_array_equal(gn, on, err_msg="round %d game %d nodes" % (done, g))
    np.testing.assert_array_equal(ge, oe, err_msg="round %d game %d edges" % (done, g))
    if gi["phase"] == 1:
        np.testing.assert_array_equal(gpu.root_policy(g), ora.root_noised(og))


# The NI = 4 (7x7, P = 196) and NI = 6 (9x9, P = 324) instantiations of the search
# kernels: game state, trees, root priors and rows bit-exact vs the oracle.
@pytest.mark.parametrize("X,Y,W,games,visits,rounds,seed,cache_log2,play",
                         [(7, 7, 5, 6, 32, 1500, 3, 0, {}), (7, 7, 5, 8, 24, 1500, 5, 12, PRODUCTION),
                          (9, 9, 5, 4, 24, 1500, 7, 0, {}), (9, 9, 5, 6, 20, 1500, 11, 12,
                                                             dict(PRODUCTION, side_position_prob=0.2, **FORKS)),
                          # the largest board the ABI takes (10x10: P = 400, NI = 7) and a
                          # rectangular one (4 symmetries instead of 8)
                          (10, 10, 5, 3, 16, 1500, 13, 0, {}), (6, 4, 4, 6, 24, 1200, 17, 12, PRODUCTION)],
                         ids=["7x7-bench", "7x7-production", "9x9-bench", "9x9-everything", "10x10-max", "6x4-rect"])
@pytest.mark.parametrize("sched", [SCHEDULES[0], SCHEDULES[2]], ids=[SCHEDULE_IDS[0], SCHEDULE_IDS[2]])
def test_selfplay_geometries_bit_exact_vs_oracle(X, Y, W, games, visits, rounds, seed, cache_log2, play, sched):
    cap = 128
    if sched[0] > 1:
        rounds *= 2
    gpu = _scheduled_engine(sched, X, Y, W, num_games=games, max_visits=visits, seed=seed, node_cap=cap,
                            nn_cache_log2=cache_log2, row_capacity=1 << 15, **play)
    ora = oracle.Selfplay(X, Y, W, games=games, max_visits=visits, node_cap=cap, seed=seed,
                          nn_cache_log2=cache_log2, commit_interval=sched[0], start_stagger=sched[2], **play)
    done = 0
    for chunk in [1, 7, 200, rounds]:
        gpu.step(chunk - done)
        ora.rounds(chunk - done)
        done = chunk
        for g in range(games):
            _compare_game(gpu, ora, g, g, done)
    st = gpu.stats()
    assert st["errors"] == 0 and st["rows_dropped"] == 0 and st["moves"] > 0
    gr = _sorted_rows(gpu.drain_rows())
    orr = _sorted_rows(ora.rows())
    assert len(gr["meta"]) == len(orr["meta"])
    for k in orr:
        np.testing.assert_array_equal(gr[k], orr[k], err_msg=k)
    gpu.close()


# Tree positions (recordTreePositions play.cpp:710-860): side rows from the finished
# searches' trees, bit-exact vs the oracle, alone and with every other variety feature.
TREE = dict(record_tree_positions=1, record_tree_threshold=2, record_tree_target_weight=0.6)


@pytest.mark.parametrize("X,Y,W,games,visits,rounds,seed,cache_log2,play",
                         [(5, 5, 4, 8, 32, 1500, 61, 0, TREE),
                          (5, 5, 4, 8, 24, 1800, 67, 12, dict(PRODUCTION, side_position_prob=0.3, **FORKS,
                                                              record_tree_positions=1, record_tree_threshold=3,
                                                              record_tree_target_weight=1.0)),
                          (9, 9, 5, 4, 24, 1200, 71, 0, TREE)],
                         ids=["5x5-tree", "5x5-tree-everything", "9x9-tree"])
def test_selfplay_tree_positions_bit_exact_vs_oracle(X, Y, W, games, visits, rounds, seed, cache_log2, play):
    cap = 128
    gpu = kc.Selfplay(X, Y, W, num_games=games, max_visits=visits, seed=seed, node_cap=cap, commit_interval=1,
                      nn_cache_log2=cache_log2, row_capacity=1 << 16, **play)
    ora = oracle.Selfplay(X, Y, W, games=games, max_visits=visits, node_cap=cap, seed=seed,
                          nn_cache_log2=cache_log2, **play)
    done = 0
    for chunk in [1, 7, 200, rounds]:
        gpu.step(chunk - done)
        ora.rounds(chunk - done)
        done = chunk
        for g in range(games):
            _compare_game(gpu, ora, g, g, done)
    st = gpu.stats()
    assert st["errors"] == 0 and st["rows_dropped"] == 0 and st["moves"] > 0
    gr = _sorted_rows(gpu.drain_rows())
    orr = _sorted_rows(ora.rows())
    assert len(gr["meta"]) == len(orr["meta"])
    tree = orr["globalTargetsNC"][:, 27] == 0.0
    assert tree.sum() > 0
    for k in orr:
        np.testing.assert_array_equal(gr[k], orr[k], err_msg=k)
    gpu.close()


def test_tree_position_weight_above_one_rejected():
    """play.cpp:1349-1350: recordTreeTargetWeight > 1 is an error."""
    with pytest.raises(kc.CoffeeError):
        kc.Selfplay(5, 5, 4, num_games=2, max_visits=8, node_cap=64, record_tree_positions=1,
                    record_tree_target_weight=1.5)


@pytest.mark.parametrize("sched", [(1, False, 0), (16, True, 600)], ids=["ci1", "ci16-stagger-fused"])
def test_selfplay_full_scale_sampled_slots_bit_exact(sched):
    """C2 scale on the device (4096 games, 600 visits, node_cap 2048, deep trees) with
    the stand-in network; 12 sampled slots replayed one by one in the oracle from the
    same per-slot streams (slot_base).  Games are independent once the NN cache is off
    and the batch cap never binds (cap = games), so each slot must match exactly -- also
    on the bench's schedule (commit interval 16, fused rounds, staggered starts), which
    the oracle restates per slot."""
    G, visits, rounds, cap = 4096, 600, 2600, 2048
    ci, fused, stagger = sched
    gpu = _engine(fused, 5, 5, 4, num_games=G, max_visits=visits, seed=2025, node_cap=cap, commit_interval=ci,
                  nn_cache_log2=0, nn_batch_cap=G, start_stagger=stagger)
    for chunk in (rounds // 2, rounds - rounds // 2):  # the bench steps in chunks
        gpu.step(chunk)
    st = gpu.stats()
    assert st["errors"] == 0 and st["moves"] >= G  # every game committed moves
    slots = [0, 1, 17, 511, 777, 1024, 2047, 2048, 3000, 3333, 4000, 4095]
    for s in slots:
        ora = oracle.Selfplay(5, 5, 4, games=1, max_visits=visits, node_cap=cap, seed=2025, slot_base=s,
                              commit_interval=ci, start_stagger=stagger)
        ora.rounds(rounds // 2)
        ora.rounds(rounds - rounds // 2)
        _compare_game(gpu, ora, s, 0, rounds)
    gpu.close()


# Deep trees at the full C4 and C5 scales (stand-in network, benchmark play, the bench's
# benchmark-mode node cap visits + 64): every game of the device engine runs, a sample of
# slots is replayed one by one in the oracle from the same per-slot streams.  NN cache off
# and a batch cap of G keep the games independent.  >= 3 committed moves per sampled slot.
@pytest.mark.parametrize("X,Y,W,G,visits,rounds,slots",
                         [(7, 7, 5, 8192, 800, 2600, [0, 1, 999, 4095, 4096, 6000, 8191]),
                          (9, 9, 5, 4096, 1600, 5000, [0, 7, 2048, 3001, 4095])],
                         ids=["C4-7x7-8192x800", "C5-9x9-4096x1600"])
def test_selfplay_deep_trees_full_scale_sampled_slots(X, Y, W, G, visits, rounds, slots):
    cap = visits + 64
    gpu = kc.Selfplay(X, Y, W, num_games=G, max_visits=visits, seed=4242, node_cap=cap, commit_interval=1,
                      nn_cache_log2=0, nn_batch_cap=G)
    gpu.step(rounds)
    st = gpu.stats()
    assert st["errors"] == 0 and st["moves"] >= 3 * G
    for s in slots:
        ora = oracle.Selfplay(X, Y, W, games=1, max_visits=visits, node_cap=cap, seed=4242, slot_base=s)
        ora.rounds(rounds)
        assert ora.info(0)["movesMade"] >= 3
        _compare_game(gpu, ora, s, 0, rounds)
    gpu.close()


# Edge pool (search.h): child slots past 16 live in per-node blocks of the game's pool,
# grown 48 -> P-16 and compacted into the other buffer when a cheap search keeps the
# subtree (reuseTree).  Wide 9x9 roots (P = 324) at 600 visits grow blocks past 64 slots;
# selfplay1.cfg's cheap searches reuse trees.  Bit-exact vs the oracle (which has no pool).
# (cpuct 8 spreads the visits so the root passes 64 children)
@pytest.mark.parametrize("play", [dict(cpuct_exploration=8.0),
                                  dict(PRODUCTION, cheap_search_visits=60, reduced_visits_min=60,
                                       cpuct_exploration=8.0)],
                         ids=["9x9-wide-bench", "9x9-wide-reuse"])
def test_selfplay_edge_pool_growth_and_compaction(play):
    X, Y, W, G, visits, cap, rounds = 9, 9, 5, 4, 600, 700, 2600
    gpu = kc.Selfplay(X, Y, W, num_games=G, max_visits=visits, seed=515, node_cap=cap, commit_interval=1,
                      nn_cache_log2=0, **play)
    ora = oracle.Selfplay(X, Y, W, games=G, max_visits=visits, node_cap=cap, seed=515, **play)
    done = 0
    wide = 0
    # round 590: still the first (empty-board, 324 legal moves) search, the widest roots
    for chunk in [400, 590, 1000, rounds]:
        gpu.step(chunk - done)
        ora.rounds(chunk - done)
        done = chunk
        for g in range(G):
            _compare_game(gpu, ora, g, g, done)
            gn, _ = gpu.game_tree(g)
            wide = max(wide, int((gn[:, 10] & 0xFFFF).max()))
    st = gpu.stats()
    assert st["errors"] == 0 and st["moves"] > 0
    assert wide > 64  # some node used a grown (P - 16) pool block
    gr = _sorted_rows(gpu.drain_rows())
    orr = _sorted_rows(ora.rows())
    assert len(gr["meta"]) == len(orr["meta"])
    for k in orr:
        np.testing.assert_array_equal(gr[k], orr[k], err_msg=k)
    gpu.close()


def test_rows_record_network_switch(model_path):
    """Hot reload mid-game (switchNetsMidGame, play.cpp:1210-1226): rows of games that
    span the switch carry globalTargets[49] = 1 and [50] = reloads after the row's turn
    (trainingwrite.cpp:459-461, :844-850); games entirely on one network carry 0, 0."""
    sp = kc.Selfplay(5, 5, 4, num_games=32, max_visits=16, seed=41, model_path=model_path, commit_interval=1)
    sp.step(150)
    other = model_path.replace(".cfnn", "-switch.cfnn")
    kc.write_random_model("b6c96", 78, other)
    sp.set_model(other)
    sp.step(1500)
    rows = sp.drain_rows()
    assert sp.stats()["errors"] == 0
    gt, meta = rows["globalTargetsNC"], rows["meta"]
    spanning = 0
    for key in sorted({(int(m[0]), int(m[1])) for m in meta}):
        sel = [i for i, m in enumerate(meta) if (int(m[0]), int(m[1])) == key]
        sel.sort(key=lambda i: int(meta[i][2]))
        f49 = gt[sel, 49]
        f50 = gt[sel, 50]
        assert np.all(f49 == f49[0]) and f49[0] in (0.0, 1.0)
        if f49[0] == 0.0:
            assert np.all(f50 == 0.0)
        else:
            assert set(np.unique(f50)) <= {0.0, 1.0} and np.all(np.diff(f50) <= 0)
            spanning += int(f50[0] == 1.0 and f50[-1] == 0.0)
    assert spanning > 0
    sp.close()


def test_set_model_bytes_matches_file_reload(model_path):
    """coffee_selfplay_set_model_bytes (weights broadcast from rank 0) switches the
    network exactly like coffee_selfplay_set_model on the same file."""
    other = model_path.replace(".cfnn", "-bytes.cfnn")
    kc.write_random_model("b6c96", 91, other)
    a = kc.Selfplay(5, 5, 4, num_games=16, max_visits=12, seed=8, model_path=model_path, commit_interval=1)
    b = kc.Selfplay(5, 5, 4, num_games=16, max_visits=12, seed=8, model_path=model_path, commit_interval=1)
    for e in (a, b):
        e.step(120)
    a.set_model(other)
    b.set_model_bytes(open(other, "rb").read())
    with pytest.raises(kc.CoffeeError):
        b.set_model_bytes(open(other, "rb").read()[:-4])  # truncated image: rejected, network kept
    for e in (a, b):
        e.step(900)
    ra, rb = _sorted_rows(a.drain_rows()), _sorted_rows(b.drain_rows())
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])
    a.close()
    b.close()
