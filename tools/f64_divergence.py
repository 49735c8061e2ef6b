"""How far the f32 search restatement (the device's arithmetic, SPEC) drifts from the
reference's f64 search statistics (searchnode.h:18-44): the same self-play run in the
oracle with float and with double statistics (liboracle_f64.so, ORA_REAL=double), same
seeds, same stand-in network, compared game by game.

Per (slot, game) present in both runs, rows are compared turn by turn while the
positions agree (identical V1 input planes); the first turn whose position differs (or
that only one run recorded) marks where the games parted.  Reported: games with identical move sequences, the
first-divergence turns, and over the positions both runs searched: identical policy
targets (the int16 visit distributions), their L1 distance, agreement of the
most-visited move, and the value-target difference.

usage: python tools/f64_divergence.py [--games 32] [--visits 600] [--rounds 12000] [--out profiles/f64_divergence_r02.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def by_game(rows):
    games = {}
    for i, m in enumerate(rows["meta"]):
        games.setdefault((int(m[0]), int(m[1])), []).append(i)
    for k in games:
        games[k].sort(key=lambda i: int(rows["meta"][i][2]))
    return games


def compare(a, b):
    import numpy as np
    ga, gb = by_game(a), by_game(b)
    keys = sorted(set(ga) & set(gb))
    same_games, first_div, n_pos, same_pol, l1s, argmax_ok, vdiff = 0, [], 0, 0, [], 0, 0.0
    for k in keys:
        # rows by turn (production play records only some turns)
        ta = {int(a["meta"][i][2]): i for i in ga[k]}
        tb = {int(b["meta"][i][2]): i for i in gb[k]}
        turns = sorted(set(ta) | set(tb))
        div = None
        for t in turns:
            if t not in ta or t not in tb:
                div = t  # recorded in one run only: the searches' limits or weights differed
                break
            ra, rb = ta[t], tb[t]
            if not np.array_equal(a["binaryInputNCHWPacked"][ra], b["binaryInputNCHWPacked"][rb]):
                div = t
                break
            n_pos += 1
            pa = a["policyTargetsNCMove"][ra, 0].astype(np.float64)
            pb = b["policyTargetsNCMove"][rb, 0].astype(np.float64)
            same_pol += int(np.array_equal(pa, pb))
            l1s.append(float(np.abs(pa / max(pa.sum(), 1) - pb / max(pb.sum(), 1)).sum()))
            argmax_ok += int(int(np.argmax(pa)) == int(np.argmax(pb)))
        if div is not None:
            first_div.append(div)
        else:
            same_games += 1
            # TD value targets blend every later search value and the result, so
            # they are comparable only within games that stayed identical
            for t in turns:
                ra, rb = ta[t], tb[t]
                vdiff = max(vdiff, float(np.abs(a["globalTargetsNC"][ra, :10] - b["globalTargetsNC"][rb, :10]).max()))
    return dict(games_compared=len(keys), games_identical=same_games,
                first_divergence_turns=sorted(first_div),
                positions_compared=n_pos, policy_targets_identical=same_pol,
                policy_target_l1_mean=float(np.mean(l1s)) if l1s else 0.0,
                policy_target_l1_max=float(np.max(l1s)) if l1s else 0.0,
                most_visited_move_agrees=argmax_ok, value_target_max_abs_diff_identical_games=vdiff)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=32)
    ap.add_argument("--visits", type=int, default=600)
    ap.add_argument("--rounds", type=int, default=12000)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--play", choices=["benchmark", "production"], default="benchmark")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from oracle import oracle
    play = {}
    if a.play == "production":
        play = dict(cheap_search_prob=0.75, cheap_search_visits=100, reduce_visits=1, reduced_visits_min=100,
                    policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1)
    runs = []
    for f64 in (False, True):
        sp = oracle.Selfplay(5, 5, 4, games=a.games, max_visits=a.visits, node_cap=max(2048, a.visits + 64),
                             seed=a.seed, f64=f64, **play)
        sp.rounds(a.rounds)
        runs.append(sp.rows())
    res = dict(config=dict(board="5x5 win 4", games=a.games, visits=a.visits, rounds=a.rounds, seed=a.seed,
                           play=a.play, network="oracle stand-in (deterministic hash net)"),
               **compare(runs[0], runs[1]))
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
