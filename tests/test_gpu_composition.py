"""Self-play with the REAL network, composed: the oracle's search (oracle/ora_search.cpp)
is fed the device network's outputs for its own batches (oracle.Selfplay.set_net ->
kc.Network.forward on the GPU), and the device engine runs the same games with the same
network end to end.  Game state, canonical trees, root priors and training rows must be
bit-identical.  This pins the hand-off the stand-in-network parity tests cannot see:
the batch's row indirection into the network (kCompact -> forward with rowIdx), real
logits through post-processing (nneval.cpp:702-844: legal mask, softmax, the inverse
symmetry of the row's random orientation), NN-cache payloads of real outputs, and
batch-cap deferral, on the fused b6c96 kernel (5- and 8-board instances, one and two
game groups) and on the layered kernels (b10c128 @ 5x5, b18c384nbt @ 9x9, the split
"accurate" precision).  Reference: cpp/neuralnet/nneval.cpp:588-844 feeding
cpp/search/searchnnhelpers.cpp:39-129.

It relies on the network being a pure function of each row's input: the same row gives
the same logits at any batch position, batch size and workgroup variant -- asserted
first (test_network_row_independence)."""
import os

import numpy as np
import pytest

import katacoffee_amd as kc
from oracle import oracle

pytestmark = pytest.mark.gpu

INFO_KEYS = [("phase", "phase"), ("rootK", "rootK"), ("liveCount", "nodeCount"), ("gameNum", "gameNum"),
             ("turn", "turn"), ("pla", "pla"), ("playouts", "playouts"), ("nnEvals", "nnEvals"),
             ("moves", "movesMade"), ("gamesFinished", "gamesFinished"), ("rngCtr", "rngCtr"),
             ("lastCell", "lastCell"), ("lastDir", "lastDir")]


def _sorted_rows(r):
    order = np.lexsort((r["meta"][:, 2], r["meta"][:, 1], r["meta"][:, 0]))
    return {k: v[order] for k, v in r.items()}


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


@pytest.fixture(scope="module")
def nets(tmp_path_factory):
    d = tmp_path_factory.mktemp("nets")
    out = {}
    for arch in ["b6c96", "b10c128", "b18c384nbt"]:
        p = str(d / ("%s.cfnn" % arch))
        kc.write_random_model(arch, 0xC0FFEE, p)
        out[arch] = p
    return out


def _rows_of_game_positions(X, Y, W, n, seed):
    """n encoded positions from oracle self-play-like random boards (device encoder)."""
    rng = np.random.default_rng(seed)
    A = X * Y
    cells = np.zeros((n, A), np.uint8)
    for i in range(n):
        k = int(rng.integers(0, A // 2))
        idx = rng.choice(A, size=k, replace=False)
        cells[i, idx] = rng.integers(1, 3, size=k)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    hc[:, 0] = rng.integers(0, A, n)
    hd[:, 0] = rng.integers(0, 4, n)
    pla = rng.integers(1, 3, n).astype(np.uint8)
    sym = rng.integers(0, 8, n).astype(np.int32)
    packed, _ = kc.encode_batch(X, Y, W, cells, hc, hd, pla, sym, want_planes=False)
    return packed


@pytest.mark.parametrize("arch,X,Y,W,precision", [("b6c96", 5, 5, 4, "fast"), ("b6c96", 5, 5, 4, "accurate"),
                                                  ("b6c96", 5, 5, 4, "corrected"),
                                                  ("b10c128", 5, 5, 4, "fast"),
                                                  ("b18c384nbt", 9, 9, 5, "fast")],
                         ids=["b6c96-fused", "b6c96-accurate", "b6c96-corrected", "b10c128-layered",
                              "b18c384nbt-layered"])
def test_network_row_independence(nets, arch, X, Y, W, precision):
    """A row's logits do not depend on its batch position, the batch size or (fused)
    the 5- / 8-board workgroup variant: a permuted batch gives the permuted outputs."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    # fused: n > 5 x CUs selects the 8-board instance, the prefix the small (5-board) one
    n = 5 * cus + 37 if arch == "b6c96" else 203  # fused: two waves of 5-board workgroups
    packed = _rows_of_game_positions(X, Y, W, n, seed=n)
    net = kc.Network(nets[arch], X, Y, W, precision=precision)
    full = net.forward(packed)
    perm = np.random.default_rng(1).permutation(n)
    np.testing.assert_array_equal(net.forward(packed[perm]), full[perm])
    np.testing.assert_array_equal(net.forward(packed[perm[:203]]), full[perm[:203]])
    np.testing.assert_array_equal(net.forward(packed[5:6]), full[5:6])
    net.close()


# name: arch, geometry, precision, games per group, groups, visits, cache, batch cap, rounds, extra play settings
PRODUCTION = dict(cheap_search_prob=0.75, cheap_search_visits=8, cheap_search_target_weight=0.0, reduce_visits=1,
                  reduce_visits_threshold=0.9, reduce_visits_threshold_lookback=3, reduced_visits_min=8,
                  reduced_visits_weight=0.1, policy_surprise_data_weight=0.5, value_surprise_data_weight=0.1)
CASES = {
    # C2 settings: fused fast b6c96, NN cache, binding batch cap above 5 x CUs (8-board kernel)
    "c2-fused-nb8": ("b6c96", (5, 5, 4), "fast", 1536, 1, 24, 14, 1300, 420, {}),
    # two game groups on their own streams, each capped (5-board kernel), selfplay1.cfg play
    "c2-fused-two-groups": ("b6c96", (5, 5, 4), "fast", 384, 2, 24, 14, 300, 700, PRODUCTION),
    # split-precision network in self-play
    "c2-accurate": ("b6c96", (5, 5, 4), "accurate", 128, 1, 24, 12, 0, 900, {}),
    # corrected network (the benchmarked 1e-3 path): two groups, binding cap, selfplay1.cfg play
    "c2-corrected-two-groups": ("b6c96", (5, 5, 4), "corrected", 384, 2, 24, 14, 300, 700, PRODUCTION),
    # the bench's C2 layout: four game groups on their own streams (fast fused, and the
    # default precision -> corrected on this net, audited), binding caps, selfplay1.cfg play
    "c2-fused-four-groups": ("b6c96", (5, 5, 4), "fast", 256, 4, 24, 14, 200, 600, PRODUCTION),
    "c2-default-four-groups": ("b6c96", (5, 5, 4), "default", 256, 4, 24, 14, 200, 600, PRODUCTION),
    # C3 network on the layered kernels
    "c3-layered": ("b10c128", (5, 5, 4), "fast", 256, 1, 24, 12, 200, 900, {}),
    # C3 and C4 as the bench runs them: the default precision (the split "accurate" layered
    # path), game groups on their own streams; C4's 7x7 / 5 with selfplay1.cfg play
    "c3-layered-default": ("b10c128", (5, 5, 4), "default", 192, 2, 24, 12, 150, 900, {}),
    "c4-layered-default": ("b10c128", (7, 7, 5), "default", 96, 2, 16, 12, 0, 1500, PRODUCTION),
    # C5 network (nested bottlenecks) at 9x9 / 5 on the layered kernels
    "c5-layered": ("b18c384nbt", (9, 9, 5), "fast", 24, 1, 12, 12, 0, 1500, {}),
    # and at the default (split) precision C5's bench line runs
    "c5-layered-default": ("b18c384nbt", (9, 9, 5), "default", 16, 1, 12, 12, 0, 1200, {}),
}


def _engine(fused, X, Y, W, **kw):
    # the engine reads COFFEE_FUSED_ROUNDS when it is created (None: its own choice)
    old = os.environ.pop("COFFEE_FUSED_ROUNDS", None)
    if fused is not None:
        os.environ["COFFEE_FUSED_ROUNDS"] = "1" if fused else "0"
    try:
        return kc.Selfplay(X, Y, W, **kw)
    finally:
        os.environ.pop("COFFEE_FUSED_ROUNDS", None)
        if old is not None:
            os.environ["COFFEE_FUSED_ROUNDS"] = old


@pytest.mark.parametrize("name", [n for n in CASES if "four-groups" not in n])
def test_selfplay_real_network_bit_exact_vs_oracle(nets, name):
    _run_case(nets, name, (1, None, 0))


# The product's round schedule with the real networks: commit interval 16 (bench.py, the
# CLI), staggered starts, each group's NN cache shared by its games -- so a lookup's hit
# depends on the other games' timing -- with separate and with fused round kernels
# (the fast headline fuses; the corrected network runs them separately by default).
# The oracle runs the same schedule (oracle.Selfplay commit_interval / start_stagger).
@pytest.mark.parametrize("sched", [(16, False, 29), (16, True, 29)], ids=["ci16-stagger", "ci16-stagger-fused"])
@pytest.mark.parametrize("name", ["c2-fused-nb8", "c2-corrected-two-groups", "c4-layered-default"])
def test_selfplay_real_network_scheduled_bit_exact_vs_oracle(nets, name, sched):
    _run_case(nets, name, sched)


# bench.py's default C2 layout (4 groups, commit interval 16, staggered starts; the fast
# network fuses the rounds, the default precision runs them separately)
@pytest.mark.parametrize("name,sched", [("c2-fused-four-groups", (16, True, 29)),
                                        ("c2-default-four-groups", (16, False, 29))],
                         ids=["fast-fused", "default-separate"])
def test_selfplay_bench_layout_bit_exact_vs_oracle(nets, name, sched):
    _run_case(nets, name, sched)


def _run_case(nets, name, sched):
    ci, fused, stagger = sched
    arch, (X, Y, W), precision, G, groups, visits, cache, cap, rounds, play = CASES[name]
    path = nets[arch]
    net = kc.Network(path, X, Y, W, precision=precision)
    calls = []

    def device_net(packed):
        calls.append(packed.shape[0])
        return net.forward(packed)

    cap_node = 4 * visits + 32
    gpus, oras = [], []
    for k in range(groups):
        gpus.append(_engine(fused, X, Y, W, num_games=G, max_visits=visits, seed=777, slot_base=k * G,
                            model_path=path, node_cap=cap_node, commit_interval=ci, start_stagger=stagger,
                            nn_cache_log2=cache, nn_batch_cap=cap, nn_precision=precision, row_capacity=1 << 16,
                            **play))
        gpus[-1].enable_timing(1)
        ora = oracle.Selfplay(X, Y, W, games=G, max_visits=visits, node_cap=cap_node, seed=777, slot_base=k * G,
                              nn_cache_log2=cache, nn_batch_cap=cap, commit_interval=ci, start_stagger=stagger, **play)
        ora.set_net(device_net)
        oras.append(ora)
    sample = sorted(set(list(range(min(G, 8))) + list(np.random.default_rng(3).integers(0, G, 24))))
    done = 0
    for chunk in [1, 30, 97, rounds]:
        for gpu in gpus:  # the groups' rounds overlap on their streams
            gpu.step(chunk - done)
        for ora in oras:
            ora.rounds(chunk - done)
        done = chunk
        for gpu, ora in zip(gpus, oras):
            gpu.sync()
            for g in sample:
                _compare_game(gpu, ora, g, g, done)
    if cap:
        assert max(calls) == cap  # the cap binds
    for gpu, ora in zip(gpus, oras):
        st = gpu.stats()
        assert st["errors"] == 0 and st["rows_dropped"] == 0 and st["games_finished"] > 0
        gr = _sorted_rows(gpu.drain_rows())
        orr = _sorted_rows(ora.rows())
        assert len(gr["meta"]) == len(orr["meta"]) > 0
        for k in orr:
            bad = np.argwhere(gr[k].reshape(len(gr[k]), -1) != orr[k].reshape(len(orr[k]), -1))
            if len(bad):  # which rows (slot, game, turn) and which columns differ
                print(k, "mismatches (meta, column):", [(gr["meta"][r].tolist(), int(c)) for r, c in bad[:20]])
            np.testing.assert_array_equal(gr[k], orr[k], err_msg=k)
        if fused is not None:  # the schedule ran as named
            n4 = gpu.kernel_time(4)[1]
            assert (n4 > rounds // 2) if fused else (n4 == 0), n4
        gpu.close()
    net.close()
