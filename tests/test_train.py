"""CPU checks of the training side: the torch CoffeeNet computes what
the engine's network computes (pinned to the fp32 oracle forward, eigenbackend.cpp
semantics), CFNN v1 files round-trip between the engine's writer and the trainer,
and a few optimizer steps on engine-format rows reduce the loss."""
import os
import tempfile

import numpy as np
import pytest
import torch

import katacoffee_amd as kc
from katacoffee_amd import train
from oracle import oracle


def _boards(n, X, Y, W, seed):
    rng = np.random.default_rng(seed)
    A = X * Y
    colors = rng.integers(0, 3, size=(n, A)).astype(np.uint8)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    for i in range(n):
        k = int(rng.integers(0, 6))
        hc[i, :k] = rng.choice(A, size=k, replace=False)
        hd[i, :k] = rng.integers(0, 4, size=k)
    pla = rng.integers(1, 3, size=n).astype(np.uint8)
    sym = np.zeros(n, np.int32)
    return oracle.encode_batch(X, Y, W, colors, hc, hd, pla, sym)


@pytest.mark.parametrize("arch,X,Y,W", [("b2c32", 5, 5, 4), ("b6c96", 5, 5, 4), ("b2c32", 7, 7, 5),
                                        ("b2c32nbt", 5, 5, 4), ("b10c128", 7, 7, 5), ("b18c384nbt", 9, 9, 5)])
def test_torch_net_matches_oracle_forward(arch, X, Y, W):
    d = tempfile.mkdtemp()
    path = os.path.join(d, "m.cfnn")
    kc.write_random_model(arch, 7, path)
    net = train.load_cfnn(path)
    binp, glob = _boards(24, X, Y, W, seed=3)
    pol_o, val_o, misc_o = oracle.Model(path).forward(X, Y, binp, glob, mode=0, threads=4)
    with torch.no_grad():
        pol, val, misc = net(torch.from_numpy(binp.reshape(24, 15, Y, X)), torch.from_numpy(glob.reshape(24, 1)))
    np.testing.assert_allclose(pol.numpy(), pol_o.reshape(24, -1), atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(val.numpy(), val_o, atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(misc.numpy(), misc_o, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("arch", ["b6c96", "b2c32nbt", "b18c384nbt"])
def test_cfnn_roundtrip_is_byte_exact(arch):
    d = tempfile.mkdtemp()
    a, b = os.path.join(d, "a.cfnn"), os.path.join(d, "b.cfnn")
    kc.write_random_model(arch, 11, a)
    train.save_cfnn(train.load_cfnn(a), b)
    assert open(a, "rb").read() == open(b, "rb").read()
    assert open(a, "rb").read()[4] == (2 if "nbt" in arch else 1)
    # a torch-initialised net is readable by the engine's loader (flops query parses it)
    c = os.path.join(d, "c.cfnn")
    train.save_cfnn(train.CoffeeNet("b10c128"), c)
    assert kc.model_flops(c, 49) > 0
    with pytest.raises(ValueError):
        open(os.path.join(d, "bad.cfnn"), "wb").write(b"CFNN\x02\x00\x00\x00" + b"\x00" * 40)
        train.load_cfnn(os.path.join(d, "bad.cfnn"))


def test_rows_roundtrip_and_training_reduces_loss():
    sp = oracle.Selfplay(5, 5, 4, games=4, max_visits=24, node_cap=128, seed=21)
    sp.rounds(1500)
    rows = sp.rows()
    n = len(rows["meta"])
    assert n >= 20
    d = tempfile.mkdtemp()
    path = os.path.join(d, "rows.npz")
    kc.write_npz(path, rows, 5, 5)
    back = train.load_rows(path)
    for k in train.ROW_KEYS:
        np.testing.assert_array_equal(back[k], rows[k])
    batch = train.rows_to_batch(back, 5, 5)
    # the unpacked planes are the encoder's planes (plane 0 = on-board everywhere)
    assert torch.all(batch["binp"][:, 0] == 1.0)
    assert torch.allclose(batch["policy"].sum(dim=1), torch.ones(n))
    assert torch.allclose(batch["value"].sum(dim=1), torch.ones(n))
    torch.manual_seed(0)
    net = train.CoffeeNet("b2c32")
    opt = torch.optim.Adam(net.parameters(), lr=2e-3)
    with torch.no_grad():
        p0, v0 = (float(x) for x in train.losses(net, batch))
    for _ in range(60):
        train.train_step(net, opt, batch)
    with torch.no_grad():
        p1, v1 = (float(x) for x in train.losses(net, batch))
    assert p1 < 0.8 * p0 and v1 < v0
    # the trained net goes back into an engine-loadable file
    out = os.path.join(d, "trained.cfnn")
    train.save_cfnn(net, out)
    for a, b in zip(train.load_cfnn(out).tensors(), net.tensors()):
        assert torch.equal(a, b.detach())
