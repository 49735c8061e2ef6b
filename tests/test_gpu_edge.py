"""GPU edge cases of the C ABI's batch entry points.  The reference's own tests feed single
positions and whole games; the empty and one-row batches, a batch that is not a multiple of
a workgroup's boards, and the argument checks belong to the boundary (include/katacoffee.h):
every batch call accepts n = 0 and returns nothing, one row alone equals the same row inside
a larger batch, and malformed arguments fail with an error instead of launching."""
import ctypes
import glob
import os

import numpy as np
import pytest

import katacoffee_amd as kc

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD5 = [p for p in sorted(glob.glob(os.path.join(HERE, "golden", "rules_*.npz"))) if "5x5" in p][0]


@pytest.fixture(scope="module")
def model_path(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("m") / "b6c96.cfnn")
    kc.write_random_model("b6c96", 0xC0FFEE, p)
    return p


def _positions(n):
    d = np.load(GOLD5)
    last = np.where(d["last_x"] >= 0, d["last_y"] * 5 + d["last_x"], -1)
    return d["colors"][:n], last[:n], d["last_dir"][:n], d["pla"][:n]


def test_empty_batches(model_path):
    A, words = 25, (15 * 25 + 63) // 64
    cells, last, ldir, pla = (np.zeros((0, A), np.uint8), np.zeros(0, np.int8), np.zeros(0, np.int8),
                              np.zeros(0, np.uint8))
    legal, has = kc.rules_batch(5, 5, 4, cells, last, ldir, pla)
    assert legal.shape == (0, 4 * A) and has.shape == (0,)
    out = kc.play_batch(5, 5, 4, cells, last, ldir, pla, np.zeros(0, np.int32))
    assert all(len(o) == 0 for o in out)
    packed, planes = kc.encode_batch(5, 5, 4, cells, np.zeros((0, 5), np.int8), np.zeros((0, 5), np.int8), pla,
                                     np.zeros(0, np.int32))
    assert packed.shape == (0, words) and planes.shape == (0, 15, A)
    assert kc.fake_net(5, 5, 4, packed).shape == (0, 4 * A + 4)
    for prec in ("fast", "default", "accurate"):
        net = kc.Network(model_path, 5, 5, 4, precision=prec)
        assert net.forward(packed).shape == (0, 4 * A + 4)
        assert net.forward_canonical(packed, np.zeros(0, np.int32)).shape == (0, 4 * A + 4)
        net.close()


@pytest.mark.parametrize("prec", ["fast", "default", "accurate"])
def test_one_row_equals_row_in_ragged_batch(model_path, prec):
    """A batch of 203 rows (not a multiple of the 5- or 8-board workgroups) and each of a few
    of its rows alone: the same logits, bit for bit (no result depends on the batch)."""
    n = 203
    cells, last, ldir, pla = _positions(n)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    hc[:, 0] = last
    hd[:, 0] = np.where(last >= 0, ldir, 4)
    sym = (np.arange(n) % 8).astype(np.int32)
    packed, _ = kc.encode_batch(5, 5, 4, cells, hc, hd, pla, sym, want_planes=False)
    net = kc.Network(model_path, 5, 5, 4, precision=prec)
    full = net.forward(packed)
    for i in (0, 4, 5, 7, 8, 131, n - 1):
        np.testing.assert_array_equal(net.forward(packed[i:i + 1]), full[i:i + 1], err_msg="row %d" % i)
    net.close()


def test_malformed_arguments_fail():
    L = kc.lib()
    null = ctypes.c_void_p()
    # negative counts, impossible geometries, missing buffers: an error code, nothing launched
    assert L.coffee_rules_batch(5, 5, 4, -1, null, null, null, null, null, null, None) != 0
    assert L.coffee_rules_batch(11, 5, 4, 0, null, null, null, null, null, null, None) != 0
    assert L.coffee_rules_batch(5, 5, 6, 0, null, null, null, null, null, null, None) != 0
    assert L.coffee_rules_batch(5, 5, 4, 3, null, null, null, null, null, null, None) != 0
    assert L.coffee_fake_net(5, 5, 4, -2, null, null, None) != 0
    assert L.coffee_nn_forward(null, 0, null, null, None) != 0
    assert kc.lib().coffee_last_error()  # the message of the last failure
    with pytest.raises(kc.CoffeeError):
        kc.Network("/nonexistent/model.cfnn", 5, 5, 4)
    # and the library still works afterwards
    cells, last, ldir, pla = _positions(4)
    legal, has = kc.rules_batch(5, 5, 4, cells, last, ldir, pla)
    assert legal.shape == (4, 100) and has.shape == (4,)


def test_selfplay_rejects_bad_configuration():
    """coffee_selfplay_create checks its arguments before allocating anything: a node pool
    (rounded up to a multiple of 64) that cannot hold one full search (max_visits + 4
    nodes), one past the 16-bit node index, a negative batch cap."""
    for kw in (dict(max_visits=100, node_cap=64), dict(max_visits=32, node_cap=70000),
               dict(max_visits=32, nn_batch_cap=-1)):
        with pytest.raises(kc.CoffeeError):
            kc.Selfplay(5, 5, 4, num_games=4, seed=1, **kw)
    sp = kc.Selfplay(5, 5, 4, num_games=4, max_visits=60, node_cap=64, seed=1)  # the smallest pool
    sp.step(400)
    st = sp.stats()
    assert st["errors"] == 0 and st["moves"] > 0
    sp.close()
