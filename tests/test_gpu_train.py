"""GPU check of the training loop's hand-off: a net trained by the
torch side on engine-format rows, written as CFNN, evaluates on the MI355X network
kernels to the logits of the torch model.

  accurate precision (fp16 hi/lo operand pairs): within 1e-3 absolute of the torch
      fp32 model -- the north-star bound, for a trained net;
  corrected precision (fp16 products + block-scaled e4m3 cross terms, the benchmarked
      path): within 1e-3 absolute of the torch fp32 model, and within 2e-4 x max(1,
      max|logit|) of the oracle's corrected emulation -- on the 10-step net, on a net
      trained 200 Adam steps (logits ~20), and on a net whose activations reach 20000
      entering a convolution (past e4m3's 448: those boards are flagged and re-evaluated on
      the accurate instance; a fixed clamp at 448 lost their cross terms);
  default precision (the C ABI's, the CLI's and the configs'): the corrected instance or,
      when its calibration check against the accurate instance exceeds 2.5e-4, the
      accurate one -- within 1e-3 absolute of fp32 on every net here;
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


def _trained(steps):
    """tools/precision_study.py trained_net: oracle self-play rows, `steps` Adam steps."""
    sp = oracle.Selfplay(5, 5, 4, games=4, max_visits=24, node_cap=128, seed=33)
    sp.rounds(1500)
    rows = sp.rows()
    batch = train.rows_to_batch(rows, 5, 5)
    torch.manual_seed(1)
    net = train.CoffeeNet("b6c96")
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    for _ in range(steps):
        train.train_step(net, opt, batch)
    return net, batch


def _eval(net, batch, precision):
    path = os.path.join(tempfile.mkdtemp(), "net.cfnn")
    train.save_cfnn(net, path)
    with torch.no_grad():
        pol, val, misc = net(batch["binp"], batch["glob"])
    ref = np.concatenate([pol.numpy(), val.numpy(), misc.numpy()], axis=1)
    planes = batch["binp"].numpy().reshape(len(ref), 15, 25)
    h = kc.Network(path, 5, 5, 4, precision=precision)
    assert h.fused
    out = h.forward(_pack_u64(planes))
    prec = h.precision
    h.close()
    return out, ref, planes, path, prec


@pytest.mark.parametrize("steps", [200])
def test_deeper_trained_net_within_north_star(steps):
    """Longer training grows the logits (~20 at 200 steps) and with them the corrected
    path's error (~2^-14 of the products: 8.2e-4 in tools/precision_study.py); the default
    precision checks itself at load time and falls back to the split path if needed."""
    net, batch = _trained(steps)
    out_c, ref, planes, path, _ = _eval(net, batch, "corrected")
    out_a, _, _, _, _ = _eval(net, batch, "accurate")
    out_d, _, _, _, (pd, calib) = _eval(net, batch, "default")
    polc, valc, miscc = oracle.Model(path).forward(5, 5, planes, batch["glob"].numpy(), mode=2, threads=8)
    refc = np.concatenate([polc.reshape(len(ref), -1), valc, miscc], axis=1)
    e_c, e_a, e_d = (float(np.abs(o - ref).max()) for o in (out_c, out_a, out_d))
    e_emu = float(np.abs(out_c - refc).max())
    print("steps", steps, "max |logit|", np.abs(ref).max(), "| corrected", e_c, "vs emulation", e_emu, "| accurate", e_a,
          "| default ->", pd, "calibration", calib, "error", e_d)
    assert np.abs(ref).max() > 10.0  # the regime the test is for
    assert e_c <= 1e-3
    assert e_emu <= 2e-4 * max(1.0, float(np.abs(ref).max()))
    assert e_a <= 1e-4
    assert pd in ("corrected", "accurate") and e_d <= 1e-3
    assert (pd == "corrected") == (calib <= 2.5e-4)


@torch.no_grad()
def _hot_net(net, batch, M):
    """tools/precision_study.py hot_net: block 0's BN2 scaled so its conv2 reads activations
    up to M, the later blocks' BN1 and the tip BN by the inverse (weights untouched)."""
    import torch.nn.functional as F
    b0 = net.blocks[0]
    x = F.conv2d(batch["binp"], net.convInit, padding=1) + (batch["glob"] @ net.globInit.t())[:, :, None, None]
    a = F.relu(x * b0.bn1s[:, None, None] + b0.bn1b[:, None, None])
    a2 = F.relu(F.conv2d(a, b0.conv1, padding=1) * b0.bn2s[:, None, None] + b0.bn2b[:, None, None])
    f = M / float(a2.max())
    b0.bn2s.mul_(f)
    b0.bn2b.mul_(f)
    for b in net.blocks[1:]:
        b.bn1s.div_(f)
    net.tips.div_(f)
    return f


def test_corrected_activations_past_e4m3_range():
    """Activations up to 20000 entering a convolution: with round 4's fixed clamp at e4m3's
    448 the cross terms of those products were lost (1.3e-3 in tools/precision_study.py
    --hot); now the corrected kernel flags those boards and the accurate instance
    re-evaluates them (the default precision's calibration then picks accurate outright)."""
    net, batch = _trained(200)
    f = _hot_net(net, batch, 20000.0)  # block 0's conv2 now reads activations up to 20000
    out_c, ref, planes, path, _ = _eval(net, batch, "corrected")
    polc, valc, miscc = oracle.Model(path).forward(5, 5, planes, batch["glob"].numpy(), mode=2, threads=8)
    refc = np.concatenate([polc.reshape(len(ref), -1), valc, miscc], axis=1)
    e_c = float(np.abs(out_c - ref).max())
    e_emu = float(np.abs(out_c - refc).max())
    print("hot net: BN2 x %.1f, max |logit| %.3f, corrected vs fp32 %.3e, vs emulation %.3e" %
          (f, np.abs(ref).max(), e_c, e_emu))
    assert np.isfinite(out_c).all()
    assert e_c <= 1e-3
    assert e_emu <= 2e-4 * max(1.0, float(np.abs(ref).max()))
    out_d, _, _, _, (pd, calib) = _eval(net, batch, "default")
    print("hot net default ->", pd, "calibration", calib, "error", float(np.abs(out_d - ref).max()))
    assert pd == "accurate" and float(np.abs(out_d - ref).max()) <= 1e-3


def test_trained_net_runs_on_device_kernel():
    net, batch = _trained(10)
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
    fast = kc.Network(path, 5, 5, 4, precision="fast")
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


@pytest.mark.parametrize("arch,X,Y,W,steps", [("b10c128", 5, 5, 4, 200), ("b10c128", 7, 7, 5, 60),
                                              ("b18c384nbt", 9, 9, 5, 30)],
                         ids=["b10c128-5x5", "b10c128-7x7", "b18c384nbt-9x9"])
def test_layered_trained_net_within_north_star(arch, X, Y, W, steps):
    """The C3-C5 nets on the layered kernels after training (the configs' compliant path:
    the default precision, which runs the split kernels for these nets): within 1e-3
    absolute of the torch fp32 model (eigenbackend.cpp semantics; model_pytorch.py
    :678-958 for the nested bottleneck blocks).  Trained on the GPU, reference on the CPU."""
    sp = oracle.Selfplay(X, Y, W, games=4, max_visits=16, node_cap=96, seed=5)
    sp.rounds(1200 if X == 5 else 2500)
    rows = sp.rows()
    assert len(rows["globalTargetsNC"]) > 16
    batch = train.rows_to_batch(rows, X, Y, device="cuda")
    torch.manual_seed(2)
    net = train.CoffeeNet(arch).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    for _ in range(steps):
        train.train_step(net, opt, batch)
    net = net.cpu()
    cpu = {k: v.cpu() for k, v in batch.items()}
    with torch.no_grad():
        pol, val, misc = net(cpu["binp"], cpu["glob"])
    ref = np.concatenate([pol.numpy(), val.numpy(), misc.numpy()], axis=1)
    path = os.path.join(tempfile.mkdtemp(), "net.cfnn")
    train.save_cfnn(net, path)
    planes = cpu["binp"].numpy().reshape(len(ref), 15, X * Y)
    h = kc.Network(path, X, Y, W, precision="default")
    assert not h.fused and h.precision[0] == "accurate"
    out = h.forward(_pack_u64(planes))
    h.close()
    f = kc.Network(path, X, Y, W, precision="fast")
    out_f = f.forward(_pack_u64(planes))
    f.close()
    err, err_f = float(np.abs(out - ref).max()), float(np.abs(out_f - ref).max())
    print("%s %dx%d after %d steps: max |logit| %.2f, default (split) vs fp32 %.3e, fast-layered %.3e" %
          (arch, X, Y, steps, np.abs(ref).max(), err, err_f))
    assert err <= 1e-3
