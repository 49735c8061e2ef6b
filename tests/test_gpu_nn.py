"""GPU parity of the network paths (NeuralNet::getOutput replacement, nninterface.h:31-171)
against the CPU oracle (eigenbackend.cpp semantics, oracle/ora_nn.cpp) for every
BASELINE architecture and board geometry:

  C2  b6c96 @ 5x5        fused kernel (fast and split "accurate" instances) and layered kernels
  C3  b10c128 @ 5x5      layered kernels
  C4  b10c128 @ 7x7      layered kernels
  C5  b18c384nbt @ 9x9   layered kernels (nested bottleneck blocks)

Tolerances (on policy/value/misc logits):
  accurate precision vs the fp32 oracle: 1e-3 absolute (north star) for every net
  corrected precision (fp16 products + e4m3 cross terms; the fused kernel for b6c96 @ 5x5,
                     the layered accurate kernels otherwise) vs the fp32 oracle: 1e-3
                     absolute; vs the oracle's corrected emulation (same roundings):
                     1e-4 x max(1, max|logit|)
  fast precision     vs the oracle's fp16-emulation mode (same operand roundings,
                     different f32 accumulation order, so an fp16 operand can round
                     the other way and the flip propagates through the trunk):
                     2e-3 x max(1, max|logit|);
                     vs the fp32 oracle: 1e-3 absolute for the C2 benchmark net
                     (b6c96 random init); deeper nets are printed (fp16 operand noise
                     grows with depth, ~1e-3 of the largest logit for b18c384nbt)
"""
import os

import numpy as np
import pytest

import katacoffee_amd as kc
from oracle import oracle

pytestmark = pytest.mark.gpu


def _pack_u64(planes):
    """[n][15][A] {0,1} -> [n][ceil(15A/64)] u64, bit i of the flat index in word i>>6."""
    n = planes.shape[0]
    flat = planes.reshape(n, -1).astype(np.uint8)
    words = (flat.shape[1] + 63) // 64
    bits = np.zeros((n, words * 64), np.uint8)
    bits[:, :flat.shape[1]] = flat
    return np.packbits(bits, axis=1, bitorder="little").view("<u8").reshape(n, words)


def _boards(n, X, Y, W, seed):
    """Random legal-looking positions (random stones, up to 5 history moves, random
    symmetry) encoded by the oracle's V1 encoder."""
    rng = np.random.default_rng(seed)
    A = X * Y
    colors = np.zeros((n, A), np.uint8)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    for i in range(n):
        k = int(rng.integers(0, A // 2))
        idx = rng.choice(A, size=k, replace=False)
        colors[i, idx] = rng.integers(1, 3, size=k)
        h = min(k, int(rng.integers(0, 6)))
        hc[i, :h] = idx[:h]
        hd[i, :h] = rng.integers(0, 4, size=h)
    pla = rng.integers(1, 3, size=n).astype(np.uint8)
    sym = rng.integers(0, 8, size=n).astype(np.int32)
    binp, glob = oracle.encode_batch(X, Y, W, colors, hc, hd, pla, sym)
    return binp, glob.reshape(n, 1).astype(np.float32)


def _ref(path, X, Y, binp, glob, mode):
    n = binp.shape[0]
    pol, val, misc = oracle.Model(path).forward(X, Y, binp, glob, mode=mode, threads=8)
    return np.concatenate([pol.reshape(n, -1), val, misc], axis=1)


CASES = [
    # arch, X, Y, W, boards (ragged: not a multiple of the boards per workgroup)
    ("b6c96", 5, 5, 4, 203),
    ("b10c128", 5, 5, 4, 131),
    ("b10c128", 7, 7, 5, 67),
    ("b2c32nbt", 5, 5, 4, 45),
    ("b18c384nbt", 9, 9, 5, 13),
]


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    d = tmp_path_factory.mktemp("nets")
    out = {}
    for arch in sorted({c[0] for c in CASES}):
        p = str(d / ("%s.cfnn" % arch))
        kc.write_random_model(arch, 0xC0FFEE, p)
        out[arch] = p
    return out


@pytest.mark.parametrize("arch,X,Y,W,n", CASES, ids=["%s-%dx%d" % (c[0], c[1], c[2]) for c in CASES])
@pytest.mark.parametrize("precision", ["fast", "fast-layered", "accurate", "corrected"])
def test_network_vs_oracle(models, arch, X, Y, W, n, precision):
    path = models[arch]
    binp, glob = _boards(n, X, Y, W, seed=n)
    net = kc.Network(path, X, Y, W, precision=precision)
    assert net.fused == (precision in ("fast", "accurate", "corrected") and arch == "b6c96")
    out = net.forward(_pack_u64(binp))
    net.close()
    ref32 = _ref(path, X, Y, binp, glob, 0)
    err32 = float(np.abs(out - ref32).max())
    if precision == "corrected" and arch == "b6c96":
        errc = float(np.abs(out - _ref(path, X, Y, binp, glob, 2)).max())
        print(arch, precision, "max |diff| vs fp32", err32, "vs corrected emulation", errc, "max |ref|",
              np.abs(ref32).max())
        assert err32 <= 1e-3
        assert errc <= 1e-4 * max(1.0, float(np.abs(ref32).max()))
    elif precision in ("accurate", "corrected"):
        print(arch, precision, "max |diff| vs fp32", err32, "max |ref|", np.abs(ref32).max())
        assert err32 <= 1e-3
    else:
        ref16 = _ref(path, X, Y, binp, glob, 1)
        err16 = float(np.abs(out - ref16).max())
        print(arch, precision, "max |diff| vs fp16-emulation", err16, "vs fp32", err32, "max |ref|",
              np.abs(ref32).max())
        assert err16 <= 2e-3 * max(1.0, float(np.abs(ref32).max()))
        if arch == "b6c96":
            assert err32 <= 1e-3
        else:
            # fp16 operand noise grows with depth: the C3-C5 lines' fast-layered networks
            # against fp32 (random init), relative to the largest logit
            assert err32 <= 2e-3 * max(1.0, float(np.abs(ref32).max()))


def test_borderless_accurate_matches_bordered(models):
    """The 5-board borderless split instance (zero row instead of per-board borders,
    2-slot weight ring) computes the same MFMA sequence per output as the 2-board
    bordered one: identical logits, bit for bit (ragged batch)."""
    path = models["b6c96"]
    binp, _ = _boards(203, 5, 5, 4, seed=11)
    packed = _pack_u64(binp)
    a = kc.Network(path, 5, 5, 4, precision="accurate")
    b = kc.Network(path, 5, 5, 4, precision="accurate-nb2")
    oa, ob = a.forward(packed), b.forward(packed)
    a.close()
    b.close()
    np.testing.assert_array_equal(oa, ob)


def test_layered_batch_indirection(models):
    """count from the device and row indirection (the self-play batch protocol):
    rows beyond the count are untouched, row r reads input rowIdx[r] and writes
    output rowIdx[r] -- exercised by self-play below; here the plain batch equals
    the per-board results of a bigger batch (no cross-board leakage)."""
    path = models["b10c128"]
    binp, glob = _boards(40, 7, 7, 5, seed=5)
    packed = _pack_u64(binp)
    net = kc.Network(path, 7, 7, 5, precision="fast-layered")
    full = net.forward(packed)
    part = net.forward(packed[7:19])
    net.close()
    np.testing.assert_array_equal(full[7:19], part)


@pytest.mark.parametrize("arch,X,Y,W", [("b10c128", 7, 7, 5), ("b18c384nbt", 9, 9, 5)])
def test_selfplay_runs_on_layered_network(models, arch, X, Y, W):
    """Self-play on the C4 / C5 networks: games advance, rows appear, no device errors."""
    sp = kc.Selfplay(X, Y, W, num_games=64, max_visits=8, seed=3, model_path=models[arch], node_cap=64,
                     nn_cache_log2=12)
    sp.step(400)
    st = sp.stats()
    sp.close()
    assert st["errors"] == 0
    assert st["moves"] > 0 and st["nn_evals"] > 0


def _symmetry_maps(X, Y, W):
    """symCell[s][c], symDir[s][d] derived from the oracle's (reference-pinned) V1
    encoder, independently of the device tables: a lone own stone at c lights plane 1
    at symCell[s][c]; a last move in direction d lights plane 3 + symDir[s][d]."""
    A = X * Y
    cells = np.zeros((8 * A, A), np.uint8)
    cells[np.arange(8 * A), np.tile(np.arange(A), 8)] = 1
    hc = np.full((8 * A, 5), -1, np.int8)
    hd = np.full((8 * A, 5), 4, np.int8)
    sym = np.repeat(np.arange(8), A).astype(np.int32)
    binp, _ = oracle.encode_batch(X, Y, W, cells, hc, hd, np.ones(8 * A, np.uint8), sym)
    sym_cell = binp[:, 1, :].argmax(axis=1).reshape(8, A)
    cells = np.zeros((32, A), np.uint8)
    cells[:, A // 2] = 2
    hc = np.full((32, 5), -1, np.int8)
    hd = np.full((32, 5), 4, np.int8)
    hc[:, 0] = A // 2
    hd[:, 0] = np.tile(np.arange(4), 8)
    sym = np.repeat(np.arange(8), 4).astype(np.int32)
    binp, _ = oracle.encode_batch(X, Y, W, cells, hc, hd, np.ones(32, np.uint8), sym)
    sym_dir = binp[:, 3:7, :].sum(axis=2).argmax(axis=1).reshape(8, 4)
    return sym_cell, sym_dir


@pytest.mark.parametrize("arch,X,Y,W,precision", [("b6c96", 5, 5, 4, "accurate"), ("b6c96", 5, 5, 4, "fast"),
                                                  ("b10c128", 7, 7, 5, "accurate")])
def test_forward_canonical_frame_vs_oracle(models, arch, X, Y, W, precision):
    """coffee_nn_forward2 = NeuralNet::getOutput (eigenbackend.cpp:1776-1796): rows
    encoded under symmetry s come back with policy logits in the canonical frame.
    Reference: the oracle's fp32 forward of the same (symmetric-frame) planes, mapped
    back with maps taken from the oracle encoder; value/misc unchanged."""
    A, P = X * Y, 4 * X * Y
    n = 96
    rng = np.random.default_rng(11)
    sym = rng.integers(0, 8, n).astype(np.int32)
    sym[:8] = np.arange(8)
    # re-encode the same positions under the chosen symmetries through the oracle encoder
    colors = np.zeros((n, A), np.uint8)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    for i in range(n):
        k = int(rng.integers(1, A // 2))
        idx = rng.choice(A, size=k, replace=False)
        colors[i, idx] = rng.integers(1, 3, size=k)
        hc[i, 0] = idx[0]
        hd[i, 0] = int(rng.integers(0, 4))
    pla = rng.integers(1, 3, n).astype(np.uint8)
    binp, glob = oracle.encode_batch(X, Y, W, colors, hc, hd, pla, sym)
    glob = glob.reshape(n, 1).astype(np.float32)
    packed = _pack_u64(binp)
    net = kc.Network(models[arch], X, Y, W, precision=precision)
    canon = net.forward_canonical(packed, sym)
    raw = net.forward(packed)
    np.testing.assert_array_equal(net.forward_canonical(packed, np.zeros(n, np.int32)), raw)
    net.close()
    sym_cell, sym_dir = _symmetry_maps(X, Y, W)
    src = np.zeros((8, P), np.int64)
    for s in range(8):
        for d in range(4):
            src[s, d * A:(d + 1) * A] = sym_dir[s, d] * A + sym_cell[s]
    # the device's own symmetric-frame output, mapped back: exact
    expect = raw.copy()
    expect[:, :P] = np.take_along_axis(raw[:, :P], src[sym], axis=1)
    np.testing.assert_array_equal(canon, expect)
    # and against the oracle's fp32 forward mapped back the same way
    ref = _ref(models[arch], X, Y, binp, glob, 0)
    ref[:, :P] = np.take_along_axis(ref[:, :P], src[sym], axis=1)
    err = float(np.abs(canon - ref).max())
    print(arch, precision, "canonical-frame max |diff| vs fp32 oracle", err)
    assert err <= (1e-3 if precision == "accurate" else 2e-3 * max(1.0, float(np.abs(ref).max())))
    assert not np.array_equal(src[sym[1]], np.arange(P))  # a non-identity symmetry is exercised
