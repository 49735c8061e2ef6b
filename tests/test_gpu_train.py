"""GPU check of the training loop's hand-off: a net trained by the
torch side on engine-format rows, written as CFNN, evaluates on the MI355X network
kernel to the logits of the torch model.  Tolerances are relative to the largest
logit: the kernel keeps the residual trunk in fp16, so one-ulp rounding flips of a
trunk value of magnitude m move logits by about m·2^-11; the 1e-3 absolute north-star
bound holds for the benchmark net's activation range (tests/test_gpu_parity.py), a
trained net with larger activations sees ~1e-3 relative."""
import os
import tempfile

import numpy as np
import pytest
import torch

import katacoffee_amd as kc
from katacoffee_amd import train
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


def test_trained_net_runs_on_device_kernel():
    sp = oracle.Selfplay(5, 5, 4, games=4, max_visits=24, node_cap=128, seed=33)
    sp.rounds(1500)
    rows = sp.rows()
    batch = train.rows_to_batch(rows, 5, 5)
    torch.manual_seed(1)
    net = train.CoffeeNet("b6c96")
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    for _ in range(10):
        train.train_step(net, opt, batch)
    path = os.path.join(tempfile.mkdtemp(), "trained.cfnn")
    train.save_cfnn(net, path)
    with torch.no_grad():
        pol, val, misc = net(batch["binp"], batch["glob"])
    ref = np.concatenate([pol.numpy(), val.numpy(), misc.numpy()], axis=1)
    planes = batch["binp"].numpy().reshape(len(ref), 15, 25)
    dev = kc.Network(path, 5, 5, 4)
    out = dev.forward(_pack_u64(planes))
    dev.close()
    pol16, val16, misc16 = oracle.Model(path).forward(5, 5, planes, batch["glob"].numpy(), mode=1, threads=8)
    ref16 = np.concatenate([pol16.reshape(len(ref), -1), val16, misc16], axis=1)
    err16 = np.abs(out - ref16).max()
    err = np.abs(out - ref).max()
    print("max |diff| vs fp16 oracle", err16, "vs torch fp32", err, "max |ref|", np.abs(ref).max())
    scale = max(1.0, float(np.abs(ref).max()))
    assert err16 <= 2e-3 * scale
    assert err <= 2e-3 * scale
