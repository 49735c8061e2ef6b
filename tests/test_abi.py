"""The C-ABI library (CPU-only checks): it builds for gfx950, loads, exports every
symbol include/katacoffee.h declares, reports errors through coffee_last_error,
and its host-built tables match the reference fixtures.  No kernel is launched."""
import ctypes
import os
import re

import numpy as np
import pytest

import katacoffee_amd as kc
from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "katacoffee.h")


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(kc.LIB_PATH):
        kc.build()
    return kc.lib()


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(coffee_[a-z0-9_]+)\s*\(", src))


def test_header_and_exports_agree(L):
    decl = declared_functions()
    assert decl == set(kc.EXPORTS), decl ^ set(kc.EXPORTS)
    for name in sorted(decl):
        assert hasattr(L, name), name


def test_abi_version_and_defaults(L):
    assert L.coffee_abi_version() == 108
    p = kc.default_search_params()
    # cpp/configs/training/selfplay1.cfg values
    assert p.max_visits == 600
    assert abs(p.cpuct_exploration - 1.1) < 1e-6
    assert abs(p.fpu_reduction_max - 0.2) < 1e-6
    assert p.root_fpu_reduction_max == 0.0
    assert abs(p.root_dirichlet_noise_total_concentration - 10.83) < 1e-5
    assert abs(p.subtree_value_bias_factor - 0.3) < 1e-6
    assert p.root_num_symmetries_to_sample == 4 and p.use_graph_search == 1
    # play settings default to the benchmark mode (one row per move at full visits)
    assert p.cheap_search_prob == 0.0 and p.reduce_visits == 0
    assert p.policy_surprise_data_weight == 0.0 and p.value_surprise_data_weight == 0.0
    assert p.cheap_search_visits == 100 and p.reduced_visits_min == 100
    # PlaySettings defaults the reference's selfplay loader leaves in place (playsettings.cpp:14)
    assert p.side_position_prob == 0.0
    assert p.record_tree_positions == 0 and p.record_tree_threshold == 0 and p.record_tree_target_weight == 0.0


def test_invalid_arguments_fail_loudly(L):
    rc = L.coffee_rules_batch(11, 5, 4, 1, None, None, None, None, None, None, None)
    assert rc == -1
    assert b"board size" in L.coffee_last_error()
    rc = L.coffee_rules_batch(5, 5, 9, 1, None, None, None, None, None, None, None)
    assert rc == -1 and b"win_len" in L.coffee_last_error()
    with pytest.raises(kc.CoffeeError):
        kc.check(L.coffee_model_flops(b"/nonexistent/model.cfnn", 25, ctypes.byref(ctypes.c_double())))


def test_cdf_table_matches_reference_fixture(L):
    # DistributionTable(tdistpdf/cdf nu=3, -50..50, 2000) as the reference computes it
    # (search.cpp:111-116), emitted by oracle/ref/refgen -> tests/golden/tdist3.npz.
    ref = np.load(os.path.join(REPO, "tests", "golden", "tdist3.npz"))["cdf"].astype(np.float32)
    ours = kc.cdf_table(5, 5, 4)
    np.testing.assert_array_equal(ours, ref)


def test_random_model_roundtrip(L, tmp_path):
    path = str(tmp_path / "b6c96.cfnn")
    kc.write_random_model("b6c96", 7, path)
    flops = kc.model_flops(path, 25)
    assert 47e6 < flops < 50e6  # 48.6 M for the KataGo trunk; Coffee head/input differ < 2 %
    m = oracle.Model(path)  # the oracle reads the same CFNN v1 file
    X = np.zeros((1, 15, 25), np.float32)
    X[0, 0] = 1.0
    pol, val, misc = m.forward(5, 5, X, np.array([[4.0]], np.float32))
    assert np.all(np.isfinite(pol)) and np.all(np.isfinite(val))


@pytest.mark.parametrize("X,Y,W", [(5, 5, 4), (7, 7, 5), (9, 9, 5), (10, 10, 5), (6, 4, 3)])
def test_zobrist_tables_match_reference(L, X, Y, W):
    # Board::initHash board.cpp:134-178 as the reference computes it (tests/golden/zobrist.npz
    # was written by oracle/ref/refgen from the reference sources), indexed by our cell order.
    z = np.load(os.path.join(REPO, "tests", "golden", "zobrist.npz"))
    t = kc.zobrist_tables(X, Y, W)
    cells = np.arange(X * Y)
    spot = (cells % X + 1) + (cells // X + 1) * (X + 1)
    np.testing.assert_array_equal(t["board"], z["board"][spot, :3])
    np.testing.assert_array_equal(t["board2"], z["board2"][spot])
    np.testing.assert_array_equal(t["player"], z["player"][:3])
    np.testing.assert_array_equal(t["init"], z["size_x"][X] ^ z["size_y"][Y])
    np.testing.assert_array_equal(t["game_over"], z["game_over"])


def test_npz_writer_roundtrip(L, tmp_path):
    # rows from the oracle engine, written by the native writer, read back with numpy
    sp = oracle.Selfplay(5, 5, 4, games=2, max_visits=12, node_cap=64, seed=3)
    sp.rounds(400)
    rows = sp.rows()
    assert len(rows["meta"]) > 0
    path = str(tmp_path / "rows.npz")
    kc.write_npz(path, rows, 5, 5)
    assert not os.path.exists(path + ".tmp")
    with np.load(path) as z:
        assert sorted(z.files) == sorted(["binaryInputNCHWPacked", "globalInputNC", "policyTargetsNCMove",
                                          "globalTargetsNC", "valueTargetsNCHW"])
        for k in z.files:
            assert z[k].dtype == rows[k].dtype, k
            np.testing.assert_array_equal(z[k], rows[k])
    import zipfile
    with zipfile.ZipFile(path) as zf:
        assert zf.testzip() is None
        raw = zf.read("globalTargetsNC")
        assert raw[:6] == b"\x93NUMPY" and len(raw) == 256 + rows["globalTargetsNC"].nbytes  # 256-byte header
