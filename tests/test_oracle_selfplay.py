"""CPU checks of the oracle's self-play restatement (the checker the GPU parity
tests trust): determinism, game/row invariants, row format."""
import numpy as np

from oracle import oracle


def _run(seed, rounds=700):
    sp = oracle.Selfplay(5, 5, 4, games=3, max_visits=24, node_cap=128, seed=seed)
    sp.rounds(rounds)
    return sp


def test_deterministic_and_seed_sensitive():
    a, b, c = _run(11), _run(11), _run(12)
    ra, rb, rc = a.rows(), b.rows(), c.rows()
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])
    assert len(ra["meta"]) != len(rc["meta"]) or any(not np.array_equal(ra[k], rc[k]) for k in ra)


def test_row_invariants():
    sp = _run(5, rounds=900)
    r = sp.rows()
    n = len(r["meta"])
    assert n > 0
    meta = r["meta"]
    # every finished game contributes numMoves consecutive rows, turns 0..numMoves-1
    for slot, gnum in {(int(m[0]), int(m[1])) for m in meta}:
        sel = (meta[:, 0] == slot) & (meta[:, 1] == gnum)
        turns = np.sort(meta[sel, 2])
        np.testing.assert_array_equal(turns, np.arange(meta[sel, 3][0]))
    pol = r["policyTargetsNCMove"]
    assert pol.min() >= 0 and pol[:, 0].sum(axis=1).min() > 0
    gt = r["globalTargetsNC"]
    np.testing.assert_array_equal(gt[:, 63], 1.0)
    np.testing.assert_array_equal(gt[:, 25], 1.0)
    # TD value targets are (win, loss) pairs summing to <= 1
    for f in range(5):
        s = gt[:, 2 * f] + gt[:, 2 * f + 1]
        assert np.all(s <= 1.0 + 1e-5) and np.all(s >= -1e-6)
    v = r["valueTargetsNCHW"]
    assert set(np.unique(v[:, 0])) <= {-1, 0, 1}
    assert np.all(v[:, 1] == 0)
    assert v[:, 4].max() >= 4  # every game ends in a win (run >= winLen) or a draw
    # global input = win length
    np.testing.assert_array_equal(r["globalInputNC"][:, 0], 4.0)


def test_tree_export_is_canonical():
    sp = _run(3, rounds=150)
    nodes, edges = sp.game_tree(0)
    assert len(nodes) > 1
    # root visits = 1 + sum of edge visits into its children after reuse-free start
    root_children = nodes[0, 10] & 0xFFFF
    assert root_children > 0
    child_idx = edges[0, :root_children, 0]
    assert np.all(child_idx < len(nodes))


def test_nn_cache_cuts_evaluations():
    """SPEC a7: with the evaluation cache on, repeated states across games and moves
    skip the network; the search stays deterministic and rows keep their invariants."""
    G = 64

    def run(cache):
        sp = oracle.Selfplay(5, 5, 4, games=G, max_visits=32, node_cap=128, seed=4, nn_cache_log2=cache)
        sp.rounds(400)
        info = [sp.info(g) for g in range(G)]
        # search-leaf evaluations per playout (root evaluations: 4 symmetries per move)
        leaf = sum(i["nnEvals"] - 4 * i["movesMade"] for i in info)
        return leaf / sum(i["playouts"] for i in info), sp
    r0, _ = run(0)
    r1, a = run(14)
    _, b = run(14)
    assert r0 > 0.95 and r1 < 0.95 * r0
    ra, rb = a.rows(), b.rows()
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])


def test_benchmark_mode_searches_every_move_from_a_cleared_tree():
    # self-play clears the search before every move (play.cpp:1941-1946, :1009-1010),
    # so each row's root has exactly max_visits visits (tree reuse would overshoot)
    r = _run(7, rounds=900).rows()
    assert len(r["meta"]) > 0
    np.testing.assert_array_equal(r["globalTargetsNC"][:, 60], 24.0)


PRODUCTION = dict(cheap_search_prob=0.75, cheap_search_visits=8, cheap_search_target_weight=0.0, reduce_visits=1,
                  reduce_visits_threshold=0.9, reduce_visits_threshold_lookback=3, reduced_visits_min=8,
                  reduced_visits_weight=0.1, policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1)


def test_production_play_settings():
    """selfplay1.cfg play settings (visit counts scaled to max_visits 24): cheap searches
    (rows only when surprising), reduced visits, surprise-weighted and resolved weights."""
    sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=24, node_cap=128, seed=21, **PRODUCTION)
    sp.rounds(1500)
    moves = sum(sp.info(g)["movesMade"] for g in range(6))
    r = sp.rows()
    meta, gt = r["meta"], r["globalTargetsNC"]
    assert len(meta) > 0
    visits = gt[:, 60]
    assert visits.min() >= 8 and visits.max() <= 24
    # most moves are cheap searches without rows: fewer rows than finished-game moves
    finished_moves = sum(int(m[3]) for m in {(int(a[0]), int(a[1]), int(a[3])): a for a in meta}.values())
    assert len(meta) < finished_moves <= moves
    # a turn may be written several times (weight > 1); all copies carry the same targets
    keys = [tuple(m[:3]) for m in meta]
    for k in set(keys):
        idx = [i for i, kk in enumerate(keys) if kk == k]
        for i in idx[1:]:
            np.testing.assert_array_equal(r["policyTargetsNCMove"][i], r["policyTargetsNCMove"][idx[0]])
    assert np.all(meta[:, 2] < meta[:, 3])
    # determinism
    sp2 = oracle.Selfplay(5, 5, 4, games=6, max_visits=24, node_cap=128, seed=21, **PRODUCTION)
    sp2.rounds(1500)
    r2 = sp2.rows()
    for k in r:
        np.testing.assert_array_equal(r[k], r2[k])


def test_batch_cap_defers_leaves_without_losing_them():
    """A network batch cap (the device's one-wave kCompact cap) defers leaves to the
    next round; every game still completes its searches and the rows stay well formed."""
    sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=24, node_cap=128, seed=9, nn_batch_cap=2)
    sp.rounds(2500)
    info = [sp.info(g) for g in range(6)]
    assert all(i["gamesFinished"] > 0 for i in info)
    r = sp.rows()
    np.testing.assert_array_equal(r["globalTargetsNC"][:, 60], 24.0)
    # with the cap, each round evaluates at most 2 leaves
    assert sum(i["nnEvals"] for i in info) <= 2 * 2500 + 6


def test_policy_init_openings():
    """initGamesWithPolicy: games open with floor(Exp(1) * A * prop) unsearched policy
    moves; their turns carry no rows and the rows record the start turn (gt[53])."""
    sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=16, node_cap=128, seed=31, init_games_with_policy=1,
                         policy_init_area_prop=0.3)
    sp.rounds(1500)
    r = sp.rows()
    meta, gt = r["meta"], r["globalTargetsNC"]
    assert len(meta) > 0
    start = gt[:, 53]
    assert start.max() > 0                       # some games opened with policy moves
    np.testing.assert_array_equal(gt[:, 51], meta[:, 2])  # turn index is absolute
    assert np.all(meta[:, 2] >= start)           # no row for an opening move
    np.testing.assert_array_equal(gt[:, 60], 16.0)
    # every game contributes one row per searched turn (benchmark weights)
    for slot, gnum in {(int(m[0]), int(m[1])) for m in meta}:
        sel = (meta[:, 0] == slot) & (meta[:, 1] == gnum)
        t0 = int(start[sel][0])
        np.testing.assert_array_equal(np.sort(meta[sel, 2]), np.arange(t0, meta[sel, 3][0]))


FORKS = dict(early_fork_game_prob=0.5, early_fork_game_expected_move_prop=0.2, fork_game_prob=0.5,
             fork_game_min_choices=2, early_fork_game_max_choices=5, fork_game_max_choices=7)


def test_fork_games():
    """Forks (Play::maybeForkGame): some of a slot's games start from a position of its
    previous game plus the best of a few random moves; their rows carry mode 2 (gt[55])
    and start after the replayed prefix."""
    sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=16, node_cap=128, seed=41, **FORKS)
    sp.rounds(2500)
    r = sp.rows()
    meta, gt = r["meta"], r["globalTargetsNC"]
    fork = gt[:, 55] == 2.0
    assert fork.any() and (~fork).any()
    assert set(np.unique(gt[:, 55])) <= {0.0, 2.0}
    assert np.all(gt[fork, 53] >= 1) and np.all(gt[~fork, 53] == 0)
    assert np.all(meta[:, 2] >= gt[:, 53])
    np.testing.assert_array_equal(gt[:, 60], 16.0)


def test_side_positions():
    """Side positions (play.cpp:1328-1345, :1576-1662): searched after the game, one row
    each with the search's value as every TD target, no next-move policy (gt[28] = 0),
    no ownership / future boards (gt[27] = gt[33] = 0, value planes zero)."""
    sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=16, node_cap=128, seed=47, side_position_prob=0.3)
    sp.rounds(2500)
    r = sp.rows()
    gt, val = r["globalTargetsNC"], r["valueTargetsNCHW"]
    side = gt[:, 27] == 0.0
    assert side.any() and (~side).any()
    np.testing.assert_array_equal(gt[side, 28], 0.0)
    np.testing.assert_array_equal(gt[side, 33], 0.0)
    assert np.all(val[side] == 0)
    for f in range(1, 5):  # a single value target: every TD horizon equals it
        np.testing.assert_array_equal(gt[side, 2 * f], gt[side, 0])
    np.testing.assert_array_equal(gt[:, 60], 16.0)
    np.testing.assert_array_equal(r["policyTargetsNCMove"][side, 1], 1)


def test_tree_positions():
    """Tree positions (recordTreePositions play.cpp:710-860): with no side positions and
    no forks every row without ownership targets comes from the search trees: policy
    targets of searched children, the root's visit count in gt[60], one value target."""
    base = dict(games=6, max_visits=24, node_cap=128, seed=53)
    plain = oracle.Selfplay(5, 5, 4, **base)
    plain.rounds(1500)
    assert np.all(plain.rows()["globalTargetsNC"][:, 27] != 0.0)
    sp = oracle.Selfplay(5, 5, 4, record_tree_positions=1, record_tree_threshold=2, record_tree_target_weight=1.0,
                         **base)
    sp.rounds(1500)
    r = sp.rows()
    gt, val, pol = r["globalTargetsNC"], r["valueTargetsNCHW"], r["policyTargetsNCMove"]
    tree = gt[:, 27] == 0.0
    assert tree.sum() > (~tree).sum() > 0
    np.testing.assert_array_equal(gt[:, 60], 24.0)
    assert np.all(val[tree] == 0)
    for f in range(1, 5):
        np.testing.assert_array_equal(gt[tree, 2 * f], gt[tree, 0])
    np.testing.assert_array_equal(pol[tree, 1], 1)
    # a recorded node has children (>= threshold visits along the path): scaled to >= 10
    assert np.all(pol[tree, 0].max(axis=1) >= 10)
    # positions lie 1..5 moves past a searched turn
    assert np.all(gt[tree, 51] >= 1)
    # weight 0.5 resolves to 0 or 1 copies
    half = oracle.Selfplay(5, 5, 4, record_tree_positions=1, record_tree_threshold=2, record_tree_target_weight=0.5,
                           **base)
    half.rounds(1500)
    n_half = int((half.rows()["globalTargetsNC"][:, 27] == 0.0).sum())
    assert 0 < n_half < tree.sum()


def test_external_network_hook_matches_builtin():
    """The composition tests' hook (nnMode 3): an external network fed the batch's
    packed V1 rows.  Plugging in the stand-in network through it (unpack -> oracle
    fake_net) must reproduce the built-in stand-in run exactly, with NN cache and a
    binding batch cap, so the hook itself adds nothing to the search."""
    A = 25
    calls = []

    def net(packed):
        n = packed.shape[0]
        calls.append(n)
        bits = np.unpackbits(packed.view(np.uint8), axis=1, bitorder="little")[:, :15 * A]
        return oracle.fake_net(5, 5, 4, bits.reshape(n, 15, A).astype(np.float32))

    kw = dict(games=6, max_visits=24, node_cap=128, seed=21, nn_cache_log2=6, nn_batch_cap=4)
    a = oracle.Selfplay(5, 5, 4, **kw)
    b = oracle.Selfplay(5, 5, 4, **kw)
    b.set_net(net)
    a.rounds(2000)
    b.rounds(2000)
    assert calls and max(calls) <= 4
    for g in range(6):
        na, ea = a.game_tree(g)
        nb, eb = b.game_tree(g)
        np.testing.assert_array_equal(na, nb)
        np.testing.assert_array_equal(ea, eb)
    ra, rb = a.rows(), b.rows()
    assert len(ra["meta"]) > 0
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])


def _games_rows(r):
    """rows keyed by (slot, game number), each game's rows in turn order"""
    out = {}
    meta = r["meta"]
    for key in {(int(m[0]), int(m[1])) for m in meta}:
        sel = np.flatnonzero((meta[:, 0] == key[0]) & (meta[:, 1] == key[1]))
        sel = sel[np.argsort(meta[sel, 2], kind="stable")]
        out[key] = {k: v[sel] for k, v in r.items()}
    return out


def test_commit_interval_and_stagger_delay_but_do_not_change_independent_games():
    """The device's round schedule (commit_interval, start_stagger) restated: a game whose
    root reached its visit limit idles until the commit round, and a staggered slot idles
    before its first game.  With nothing shared between games (NN cache off, batch cap not
    binding) this only shifts each game in time: every game both runs finish has the same
    rows.  (With a shared NN cache it does not hold -- hits depend on the other games'
    timing; the GPU tests pin that case against the oracle run on the same schedule.)"""
    kw = dict(games=6, max_visits=24, node_cap=128, seed=31)
    a = oracle.Selfplay(5, 5, 4, **kw)
    b = oracle.Selfplay(5, 5, 4, commit_interval=16, start_stagger=200, **kw)
    for n in (5, 100, 1500):  # commits also fall on the last round of every rounds() call
        a.rounds(n)
        b.rounds(n)
    ga, gb = _games_rows(a.rows()), _games_rows(b.rows())
    both = set(ga) & set(gb)
    assert len(both) >= 6 and len(gb) < len(ga)  # b lost rounds to idling
    for key in both:
        for k in ga[key]:
            np.testing.assert_array_equal(ga[key][k], gb[key][k], err_msg="%s %s" % (key, k))
    # at the end of a rounds() call every game has been committed: none waits in PH_COMMIT
    assert all(b.info(g)["phase"] != 2 for g in range(6))
    # the idle rounds: fewer playouts than rounds for b, one per round (after the root
    # evaluations) for a
    assert sum(b.info(g)["playouts"] for g in range(6)) < sum(a.info(g)["playouts"] for g in range(6))


def test_schedule_rejected_after_first_round():
    sp = oracle.Selfplay(5, 5, 4, games=2, max_visits=8, node_cap=64, seed=1)
    sp.rounds(1)
    assert sp.L.ora_sp_set_schedule(sp.h, 16, 0) != 0
