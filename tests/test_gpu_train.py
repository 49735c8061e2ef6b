"""GPU check of the training loop's hand-off: a net trained by the
torch side on engine-format rows, written as CFNN, evaluates on the MI355X network
kernels to the logits of the torch model.

  accurate precision (fp16 hi/lo operand pairs): within 1e-3 absolute of the torch
      fp32 model -- the north-star bound, for a trained net;
  corrected precision (fp16 products + e4m3 cross terms, the benchmarked path): within
      1e-3 absolute of the torch fp32 model, and within 2e-4 x max(1, max|logit|) of the
      oracle's corrected emulation;
  fast precision (fp16 operands, f32 accumulation and trunk): within 2e-3 of the
      largest logit of the oracle's fp16-emulation mode (same roundings, different
      accumulation order, so single operands may round the other way).  Against fp32
      its error is set by fp16 operand rounding (~1e-3 of the largest logit for this
      net) and is printed, not asserted."""
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
    packed = _pack_u64(planes)
    acc = kc.Network(path, 5, 5, 4, precision="accurate")
    assert acc.fused  # the split-precision instance of the fused kernel
    out_acc = acc.forward(packed)
    acc.close()
    cor = kc.Network(path, 5, 5, 4, precision="corrected")
    assert cor.fused
    out_cor = cor.forward(packed)
    cor.close()
    polc, valc, miscc = oracle.Model(path).forward(5, 5, planes, batch["glob"].numpy(), mode=2, threads=8)
    refc = np.concatenate([polc.reshape(len(ref), -1), valc, miscc], axis=1)
    fast = kc.Network(path, 5, 5, 4)
    assert fast.fused
    out = fast.forward(packed)
    fast.close()
    pol16, val16, misc16 = oracle.Model(path).forward(5, 5, planes, batch["glob"].numpy(), mode=1, threads=8)
    ref16 = np.concatenate([pol16.reshape(len(ref), -1), val16, misc16], axis=1)
    err_acc = float(np.abs(out_acc - ref).max())
    err16 = float(np.abs(out - ref16).max())
    err = float(np.abs(out - ref).max())
    err_cor = float(np.abs(out_cor - ref).max())
    err_cor_emu = float(np.abs(out_cor - refc).max())
    print("accurate vs torch fp32", err_acc, "| corrected vs torch fp32", err_cor, "vs corrected emulation",
          err_cor_emu, "| fast vs fp16 oracle", err16, "fast vs torch fp32", err, "| max |ref|", np.abs(ref).max())
    assert err_acc <= 1e-3
    assert err_cor <= 1e-3
    assert err_cor_emu <= 2e-4 * max(1.0, float(np.abs(ref).max()))
    assert err16 <= 2e-3 * max(1.0, float(np.abs(ref).max()))
    # the fast (fp16-operand) path against fp32 on a trained net: fp16 rounding of the
    # weights and activations moves the logits by ~1e-3 of the largest logit (DESIGN.md
    # section 5: 7e-3 measured on logits up to 6.4); bound asserted at 3e-3 of it.  The
    # absolute 1e-3 of north_star is met by the accurate path above.
    assert err <= 3e-3 * max(1.0, float(np.abs(ref).max()))
