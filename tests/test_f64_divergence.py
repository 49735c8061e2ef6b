"""The oracle's search with f64 statistics (the reference's precision, searchnode.h:18-44)
against the f32 restatement the device follows (SPEC): same seeds,
same stand-in network.  The f64 build is a measurement instrument, so the test checks
that it runs the same search (most positions get the same most-visited move and the
same targets) and that the comparison tool works; the measured divergence at C2 visits
is in profiles/f64_divergence_r02_*.json."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from oracle import oracle  # noqa: E402


def test_f64_search_matches_f32_search_closely():
    import f64_divergence
    runs = []
    for f64 in (False, True):
        sp = oracle.Selfplay(5, 5, 4, games=6, max_visits=96, node_cap=256, seed=31, f64=f64)
        sp.rounds(4000)
        assert sp.f64 == f64
        runs.append(sp.rows())
    r = f64_divergence.compare(runs[0], runs[1])
    assert r["games_compared"] >= 6 and r["positions_compared"] > 20
    assert r["most_visited_move_agrees"] >= 0.9 * r["positions_compared"]
    assert r["policy_targets_identical"] >= 0.8 * r["positions_compared"]
    assert r["value_target_max_abs_diff_identical_games"] < 1e-3


def test_f64_node_dump_refused():
    sp = oracle.Selfplay(5, 5, 4, games=1, max_visits=8, node_cap=64, seed=1, f64=True)
    sp.rounds(5)
    try:
        sp.nodes(0)
    except ValueError:
        return
    raise AssertionError("f64 node records must not be read with the f32 layout")
