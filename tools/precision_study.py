"""Where does the fp16 network's error against fp32 come from, on a trained net?

Builds the trained b6c96 of tests/test_gpu_train.py (oracle self-play rows, 10 Adam
steps), then evaluates it in float64 with every convolution's operands rounded the way
a candidate kernel would round them, and reports the max |logit error| against the
exact forward.  Schemes per convolution (ordinal: 0 stem, 1..2*nblocks block convs,
last = head 1x1):
  f32      exact operands
  f16      fp16 weights and activations (the "fast" kernel)
  wsplit   exact weights (hi+lo), fp16 activations       (2 MFMAs)
  asplit   fp16 weights, exact activations (hi+lo)       (2 MFMAs)
  split3   hi*hi + lo(w)*hi(x) + hi(w)*lo(x)             (3 MFMAs: "accurate")
  f8c      hi*hi (fp16) + e4m3(lo(w)*S)/S * e4m3(x) + e4m3(w) * e4m3(lo(x)*S)/S
           (one fp16 MFMA + two fp8 MFMAs at twice the rate: 2 fp16-MFMA equivalents)
  f8cw     hi*hi + e4m3(lo(w)*S)/S * e4m3(x) (weights corrected only)
  f8cs     the shipped corrected kernel (round 5): f8c with the weights' e4m3 at the
           convolution's block exponent (largest weight in (224, 448], oracle/ora_nn.cpp
           f8Exp), e4m3(w) and e4m3(x) converted from the fp16 values (the device converts
           the fp16 fragments in registers), and boards whose activations pass e4m3's 448
           re-evaluated exactly (the device: on the split instance)
Usage: python tools/precision_study.py [--per-layer] [--steps N] [--big-act F]
  --steps N     Adam steps of the trained net (10: the test_gpu_train.py net)
  --big-act F   scale the first block's BN2 by F and its conv2 by 1/F (same function,
                activations F times larger entering that convolution; the weights get
                F times smaller, so fp16 subnormals hurt every fp16 scheme)
  --hot M       scale the first block's BN2 so its conv2 reads activations up to M, and
                the later blocks' BN1 and the tip BN by the same 1/F (weights untouched;
                tests/test_gpu_train.py's large-activation net)
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from katacoffee_amd import train  # noqa: E402
from oracle import oracle  # noqa: E402

S = 2.0 ** 11


def r16(t):
    return t.to(torch.float32).to(torch.float16).to(torch.float64)


def r8(t):
    return t.clamp(-448, 448).to(torch.float32).to(torch.float8_e4m3fn).to(torch.float64)


def r8n(t):
    """e4m3 without the clamp (the scaled operands never exceed 448)."""
    return t.to(torch.float32).to(torch.float8_e4m3fn).to(torch.float64)


def f8exp(m):
    """oracle/ora_nn.cpp f8Exp: s with m 2^-s in (224, 448]; 0 for m == 0."""
    f, e = torch.frexp(m)
    s = e - 9 + (f > 0.875).to(e.dtype)
    return torch.where(m > 0, s, torch.zeros_like(s)).clamp(-100, 100).to(torch.float64)


def e4m3s(v, s):
    return r8n(v * torch.pow(2.0, -s)) * torch.pow(2.0, s)


def quant_conv(x, w, scheme, conv):
    if scheme == "f32":
        return conv(x, w)
    xh, wh = r16(x), r16(w)
    xl, wl = x - xh, w - wh
    if scheme == "f16":
        return conv(xh, wh)
    if scheme == "wsplit":
        return conv(xh, w)
    if scheme == "asplit":
        return conv(x, wh)
    if scheme == "split3":
        return conv(xh, wh) + conv(xh, r16(wl)) + conv(r16(xl), wh)
    if scheme == "f8c":
        return conv(xh, wh) + conv(r8(x), r8(wl * S) / S) + conv(r8(xl * S) / S, r8(w))
    if scheme == "f8cs":
        sw = f8exp(w.abs().max())
        HOT[0] = HOT[0] | (x.abs().flatten(1).max(1).values > 448)
        return conv(xh, wh) + conv(r8(xh), e4m3s(wl * S, sw) / S) + conv(r8(xl * S) / S, e4m3s(wh, sw))
    if scheme in ("f8cs_xex", "f8cs_wex", "f8mx", "f8bx"):
        sw = f8exp(w.abs().max())
        HOT[0] = HOT[0] | (x.abs().flatten(1).max(1).values > 448)
        if scheme == "f8cs_xex":  # only the weights' e4m3 rounding in the cross terms
            return conv(xh, wh) + conv(xh, e4m3s(wl * S, sw) / S) + conv(xl, e4m3s(wh, sw))
        if scheme == "f8cs_wex":  # only the activations' e4m3 rounding in the cross terms
            return conv(xh, wh) + conv(r8(xh), wl) + conv(r8(xl * S) / S, wh)
        if scheme == "f8bx":  # one exponent per board for hi(x) and one for lo(x)
            def sc(v):
                return e4m3s(v, f8exp(v.abs().flatten(1).max(1).values)[:, None, None, None])
        else:  # per (board, position, 32-channel group) exponents: MX blocks along channels
            def sc(v):
                n, c, h, ww = v.shape
                g = v.reshape(n, c // 32, 32, h, ww) if c % 32 == 0 else v.reshape(n, 1, c, h, ww)
                m = g.abs().amax(2, keepdim=True)
                return e4m3s(g, f8exp(m)).reshape(n, c, h, ww)
        return conv(xh, wh) + conv(sc(xh), e4m3s(wl * S, sw) / S) + conv(sc(xl * S) / S, e4m3s(wh, sw))
    if scheme == "f8cw":
        return conv(xh, wh) + conv(r8(x), r8(wl * S) / S)
    raise ValueError(scheme)


HOT = [False]  # f8cs: boards with an activation past e4m3's range (re-evaluated exactly)


def forward(net, binp, glob, schemes):
    """train.CoffeeNet.forward in float64 with per-convolution operand rounding (f8cs:
    hot boards take the exact forward's outputs)."""
    if any(s.startswith("f8cs") or s in ("f8mx", "f8bx") for s in schemes):
        HOT[0] = torch.zeros(len(binp), dtype=torch.bool)
        out = forward_(net, binp, glob, schemes)
        if HOT[0].any():
            out[HOT[0]] = forward_(net, binp[HOT[0]], glob[HOT[0]], ["split3"] * len(schemes))
        return out
    return forward_(net, binp, glob, schemes)


def forward_(net, binp, glob, schemes):
    it = iter(schemes)
    c3 = lambda x, w: F.conv2d(x, w, padding=1)
    c1 = lambda x, w: torch.einsum("nchw,oc->nohw", x, w)
    P = {k: v.detach().to(torch.float64) for k, v in net.named_parameters()}
    x = quant_conv(binp, P["convInit"], next(it), c3) + (glob @ P["globInit"].t())[:, :, None, None]
    for i, b in enumerate(net.blocks):
        p = lambda n: P["blocks.%d.%s" % (i, n)]
        a = F.relu(x * p("bn1s")[:, None, None] + p("bn1b")[:, None, None])
        s1 = next(it)
        if b.kind == 1:
            w1 = torch.cat([p("conv1"), p("conv1g")], 0)
            hh = quant_conv(a, w1, s1, c3)
            Cr = p("conv1").shape[0]
            h, g = hh[:, :Cr], hh[:, Cr:]
            g = F.relu(g * p("bngs")[:, None, None] + p("bngb")[:, None, None])
            h = h + (train._gpool(g) @ p("linG").t())[:, :, None, None]
        else:
            h = quant_conv(a, p("conv1"), s1, c3)
        a2 = F.relu(h * p("bn2s")[:, None, None] + p("bn2b")[:, None, None])
        x = x + quant_conv(a2, p("conv2"), next(it), c3)
    a = F.relu(x * P["tips"][:, None, None] + P["tipb"][:, None, None])
    wh = torch.cat([P["pConv1"], P["pConvG"], P["vConv1"]], 0)
    hh = quant_conv(a, wh, next(it), c1)
    p1, g1 = P["pConv1"].shape[0], P["pConvG"].shape[0]
    p, pg, v = hh[:, :p1], hh[:, p1:p1 + g1], hh[:, p1 + g1:]
    pg = F.relu(pg + P["pBiasG"][:, None, None])
    pb = train._gpool(pg) @ P["pLinG"].t()
    p = F.relu(p + pb[:, :, None, None] + P["pBias2"][:, None, None])
    policy = torch.einsum("nchw,oc->nohw", p, P["pConv2"]).flatten(1)
    v = F.relu(v + P["vBias1"][:, None, None])
    vh = F.relu(train._gpool(v, value_head=True) @ P["vLin2"].t() + P["vB2"])
    return torch.cat([policy, vh @ P["vLin3"].t() + P["vB3"], vh @ P["vLinM"].t() + P["vBM"]], 1)


@torch.no_grad()
def hot_net(net, batch, M):
    """Scale block 0's BN2 by F so its conv2 reads activations up to M (trunk F times
    larger from there), and the later blocks' BN1 and the tip BN by 1/F (weights untouched,
    logits stay moderate).  Returns F.  (tests/test_gpu_train.py _hot_net: the same.)"""
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


def trained_net(steps=10):
    """The net of tests/test_gpu_train.py (same seeds; 10 steps there)."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-layer", action="store_true", help="f16 everywhere except one layer exact, and vice versa")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--big-act", type=float, default=0.0)
    ap.add_argument("--hot", type=float, default=0.0)
    ap.add_argument("--schemes", default="f16,wsplit,asplit,f8cw,f8c,f8cs,f8cs_xex,f8cs_wex,f8bx,f8mx,split3")
    args = ap.parse_args()
    net, batch = trained_net(args.steps)
    if args.big_act:
        with torch.no_grad():
            b = net.blocks[0]
            b.bn2s.mul_(args.big_act)
            b.bn2b.mul_(args.big_act)
            b.conv2.div_(args.big_act)
    if args.hot:
        F_ = hot_net(net, batch, args.hot)
        print("hot: block 0 BN2 x %.1f" % F_)
    binp = batch["binp"].to(torch.float64)
    glob = batch["glob"].to(torch.float64)
    nconv = 2 + 2 * len(net.blocks)
    with torch.no_grad():
        ref = forward(net, binp, glob, ["f32"] * nconv)
        print("n=%d max|logit| %.3f" % (len(ref), ref.abs().max().item()))
        for sch in args.schemes.split(","):
            out = forward(net, binp, glob, [sch] * nconv)
            e = (out - ref).abs()
            print("%-7s max err %.3e  (policy %.3e, value %.3e, misc %.3e)" % (
                sch, e.max().item(), e[:, :100].max().item(), e[:, 100:102].max().item(), e[:, 102:].max().item()))
        if args.per_layer:
            for k in range(nconv):
                s = ["f16"] * nconv
                s[k] = "f32"
                e1 = (forward(net, binp, glob, s) - ref).abs().max().item()
                s = ["f32"] * nconv
                s[k] = "f16"
                e2 = (forward(net, binp, glob, s) - ref).abs().max().item()
                print("conv %2d: f16 elsewhere, exact here %.3e | exact elsewhere, f16 here %.3e" % (k, e1, e2))


if __name__ == "__main__":
    main()
