"""Training side of the self-play loop.

The reference's python trainer reads KataGo V7 rows and builds Go heads
(data_processing_pytorch.py:22-45, :87-96; model_pytorch.py:1066-1152, :1373-1374), so
it cannot train on Coffee rows.  This module is the Coffee-aware
replacement:

* ``load_rows`` / ``rows_to_batch`` read the ``.npz`` files the engine writes
  (trainingwrite.cpp:185-205 layout: 15 bit-packed planes, policy [2][4A] without a
  pass move, 64 global targets, 5 value planes);
* ``CoffeeNet`` is the engine's network as a torch module — the same layer list and
  tensor layouts as the CFNN v1 file (csrc/model.h), the same arithmetic as the
  oracle's fp32 forward (oracle/ora_nn.cpp, eigenbackend.cpp semantics): fixup-style
  per-channel affine norms (the merged BatchNorm of the file), KataGPool, gpool bias,
  a 4-direction policy head and a 2-logit value head;
* ``save_cfnn`` / ``load_cfnn`` write and read CFNN v1/v2, so a trained net goes straight
  back into ``katago selfplay -models-dir`` (hot reload) or ``coffee_nn_create``;
* ``losses`` / ``train_step``: policy cross-entropy against the normalised visit
  target, value cross-entropy against the final outcome (draws split evenly between
  the two logits, matching the engine's two-way softmax of the value head).

Nothing here runs on the self-play hot path; it is plain PyTorch (any device).
"""
import struct

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# csrc/model.cpp modelCfgByName (modelconfigs.py:129-180 for the two named nets)
ARCHS = {
    "b6c96": dict(C=96, Cg=32, p1=32, g1=32, v1=32, v2=64, kinds=[0, 0, 1, 0, 1, 0]),
    "b18c384nbt": dict(C=384, mid=192, Cg=64, p1=48, g1=48, v1=96, v2=128,
                       kinds=[2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 3, 2, 2, 2]),
    "b2c32nbt": dict(C=64, mid=32, Cg=16, p1=16, g1=16, v1=16, v2=32, kinds=[3, 2]),
    "b10c128": dict(C=128, Cg=32, p1=32, g1=32, v1=32, v2=80, kinds=[0, 0, 0, 0, 1, 0, 0, 1, 0, 0]),
    "b2c32": dict(C=32, Cg=16, p1=16, g1=16, v1=16, v2=32, kinds=[0, 1]),
}
NUM_SPATIAL = 15


def _affine(n, scale=1.0):
    return nn.Parameter(torch.full((n,), float(scale))), nn.Parameter(torch.zeros(n))


def _gpool(x, value_head=False):
    """KataGPool over [N, C, Y, X] (eigenbackend.cpp:141-186, mask == 1): mean,
    mean·(√A − 14)/10, then max (trunk / policy) or mean·((√A − 14)²/100 − 0.1) (value)."""
    A = x.shape[2] * x.shape[3]
    sq = float(np.float32(np.sqrt(np.float32(A))) - np.float32(14.0))
    flat = x.flatten(2)
    mean = flat.sum(dim=2) / A
    third = mean * ((sq * sq) / 100.0 - 0.1) if value_head else flat.amax(dim=2)
    return torch.cat([mean, mean * (sq / 10.0), third], dim=1)


class _Block(nn.Module):
    """kind 0 regular / 1 gpool (ResBlock, model_pytorch.py:678-746) at trunk width C;
    kind 2 / 3 nested bottleneck (NestedBottleneckResBlock :860-958): 1x1 C->mid,
    two inner blocks at width mid (the first a gpool block for kind 3), 1x1 mid->C."""

    def __init__(self, kind, C, Cg, mid=0):
        super().__init__()
        self.kind = kind
        if kind >= 2:
            self.bnPs, self.bnPb = _affine(C)
            self.convP = nn.Parameter(torch.empty(mid, C))
            self.inner = nn.ModuleList([_Block(1 if kind == 3 else 0, mid, Cg), _Block(0, mid, Cg)])
            self.bnQs, self.bnQb = _affine(mid)
            self.convQ = nn.Parameter(torch.empty(C, mid))
            return
        Cr = C - Cg if kind == 1 else C
        self.bn1s, self.bn1b = _affine(C)
        self.conv1 = nn.Parameter(torch.empty(Cr, C, 3, 3))
        if kind == 1:
            self.conv1g = nn.Parameter(torch.empty(Cg, C, 3, 3))
            self.bngs, self.bngb = _affine(Cg)
            self.linG = nn.Parameter(torch.empty(Cr, 3 * Cg))
        self.bn2s, self.bn2b = _affine(Cr)
        self.conv2 = nn.Parameter(torch.empty(C, Cr, 3, 3))

    def forward(self, x):
        if self.kind >= 2:
            a = F.relu(x * self.bnPs[:, None, None] + self.bnPb[:, None, None])
            y = torch.einsum("nchw,oc->nohw", a, self.convP)
            for b in self.inner:
                y = b(y)
            aq = F.relu(y * self.bnQs[:, None, None] + self.bnQb[:, None, None])
            return x + torch.einsum("nchw,oc->nohw", aq, self.convQ)
        a = F.relu(x * self.bn1s[:, None, None] + self.bn1b[:, None, None])
        h = F.conv2d(a, self.conv1, padding=1)
        if self.kind == 1:
            g = F.relu(F.conv2d(a, self.conv1g, padding=1) * self.bngs[:, None, None] + self.bngb[:, None, None])
            h = h + (_gpool(g) @ self.linG.t())[:, :, None, None]
        a2 = F.relu(h * self.bn2s[:, None, None] + self.bn2b[:, None, None])
        return x + F.conv2d(a2, self.conv2, padding=1)

    def tensors(self):
        """CFNN tensor order (csrc/model.h)."""
        if self.kind >= 2:
            return ([self.bnPs, self.bnPb, self.convP] + self.inner[0].tensors() + self.inner[1].tensors() +
                    [self.bnQs, self.bnQb, self.convQ])
        if self.kind == 0:
            return [self.bn1s, self.bn1b, self.conv1, self.bn2s, self.bn2b, self.conv2]
        return [self.bn1s, self.bn1b, self.conv1, self.conv1g, self.bngs, self.bngb, self.linG, self.bn2s, self.bn2b,
                self.conv2]


class CoffeeNet(nn.Module):
    """The engine's residual network (CFNN v1 tensors, model_pytorch.py trunk shape)."""

    def __init__(self, arch="b6c96", cin=NUM_SPATIAL, gin=1):
        super().__init__()
        cfg = dict(ARCHS[arch]) if isinstance(arch, str) else dict(arch)
        self.cfg = dict(cfg, cin=cin, gin=gin)
        C, Cg, p1, g1, v1, v2 = (cfg[k] for k in ("C", "Cg", "p1", "g1", "v1", "v2"))
        self.convInit = nn.Parameter(torch.empty(C, cin, 3, 3))
        self.globInit = nn.Parameter(torch.empty(C, gin))
        self.blocks = nn.ModuleList(_Block(k, C, Cg, cfg.get("mid", 0)) for k in cfg["kinds"])
        self.tips, self.tipb = _affine(C)
        self.pConv1 = nn.Parameter(torch.empty(p1, C))
        self.pConvG = nn.Parameter(torch.empty(g1, C))
        self.pBiasG = nn.Parameter(torch.zeros(g1))
        self.pLinG = nn.Parameter(torch.empty(p1, 3 * g1))
        self.pBias2 = nn.Parameter(torch.zeros(p1))
        self.pConv2 = nn.Parameter(torch.empty(4, p1))
        self.vConv1 = nn.Parameter(torch.empty(v1, C))
        self.vBias1 = nn.Parameter(torch.zeros(v1))
        self.vLin2 = nn.Parameter(torch.empty(v2, 3 * v1))
        self.vB2 = nn.Parameter(torch.zeros(v2))
        self.vLin3 = nn.Parameter(torch.empty(2, v2))
        self.vB3 = nn.Parameter(torch.zeros(2))
        self.vLinM = nn.Parameter(torch.empty(2, v2))
        self.vBM = nn.Parameter(torch.zeros(2))
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, seed=0):
        """He-normal convolutions and linears, unit norms (csrc/model.cpp randomModel shape)."""
        g = torch.Generator().manual_seed(seed)
        for name, p in self.named_parameters():
            if p.dim() >= 2:
                fan_in = p[0].numel()
                scale = 0.5 if name.endswith("conv2") or name.endswith("convQ") else 1.0
                p.copy_(torch.randn(p.shape, generator=g) * (scale * np.sqrt(2.0 / fan_in)))

    def forward(self, binp, glob):
        """binp [N, 15, Y, X] f32, glob [N, gin] -> policy [N, 4A] (direction-major),
        value [N, 2] (win, loss logits of the player to move), misc [N, 2]."""
        x = F.conv2d(binp, self.convInit, padding=1) + (glob @ self.globInit.t())[:, :, None, None]
        for b in self.blocks:
            x = b(x)
        a = F.relu(x * self.tips[:, None, None] + self.tipb[:, None, None])
        p = torch.einsum("nchw,oc->nohw", a, self.pConv1)
        pg = F.relu(torch.einsum("nchw,oc->nohw", a, self.pConvG) + self.pBiasG[:, None, None])
        pb = _gpool(pg) @ self.pLinG.t()
        p = F.relu(p + pb[:, :, None, None] + self.pBias2[:, None, None])
        policy = torch.einsum("nchw,oc->nohw", p, self.pConv2).flatten(1)
        v = F.relu(torch.einsum("nchw,oc->nohw", a, self.vConv1) + self.vBias1[:, None, None])
        vh = F.relu(_gpool(v, value_head=True) @ self.vLin2.t() + self.vB2)
        return policy, vh @ self.vLin3.t() + self.vB3, vh @ self.vLinM.t() + self.vBM

    # -- CFNN v1 (csrc/model.h) -------------------------------------------------
    def tensors(self):
        """The file's tensor sequence."""
        out = [self.convInit, self.globInit]
        for b in self.blocks:
            out += b.tensors()
        out += [self.tips, self.tipb, self.pConv1, self.pConvG, self.pBiasG, self.pLinG, self.pBias2, self.pConv2,
                self.vConv1, self.vBias1, self.vLin2, self.vB2, self.vLin3, self.vB3, self.vLinM, self.vBM]
        return out


def save_cfnn(net, path):
    """Writes CFNN v1 (v2 when a block is a nested bottleneck), to path + '.tmp' then
    renamed, like the row files."""
    import os
    c = net.cfg
    fields = [c["cin"], c["gin"], c["C"], c["Cg"], c["p1"], c["g1"], c["v1"], c["v2"], len(c["kinds"])]
    if any(k >= 2 for k in c["kinds"]):
        hdr = struct.pack("<4si10i", b"CFNN", 2, *fields, c["mid"])
    else:
        hdr = struct.pack("<4si9i", b"CFNN", 1, *fields)
    body = [np.asarray(c["kinds"], "<i4").tobytes()]
    body += [t.detach().cpu().to(torch.float32).contiguous().numpy().astype("<f4").tobytes() for t in net.tensors()]
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(hdr)
        for b in body:
            f.write(b)
    os.replace(tmp, path)


def load_cfnn(path):
    """Reads CFNN v1/v2 into a CoffeeNet (raises ValueError on a malformed file)."""
    with open(path, "rb") as f:
        data = f.read()
    ver = struct.unpack_from("<i", data, 4)[0] if len(data) >= 8 else 0
    if len(data) < 44 or data[:4] != b"CFNN" or ver not in (1, 2):
        raise ValueError("not a CFNN v1/v2 model: %s" % path)
    cin, gin, C, Cg, p1, g1, v1, v2, nb = struct.unpack_from("<9i", data, 8)
    mid = struct.unpack_from("<i", data, 44)[0] if ver == 2 else 0
    hdr = 48 if ver == 2 else 44
    if not 1 <= nb <= 64:
        raise ValueError("bad block count in %s" % path)
    kinds = list(struct.unpack_from("<%di" % nb, data, hdr))
    if any(k < 0 or k > 3 or (k >= 2 and mid <= 0) for k in kinds):
        raise ValueError("bad block kinds in %s" % path)
    net = CoffeeNet(dict(C=C, Cg=Cg, p1=p1, g1=g1, v1=v1, v2=v2, kinds=kinds, mid=mid), cin=cin, gin=gin)
    off = hdr + 4 * nb
    with torch.no_grad():
        for t in net.tensors():
            n = t.numel()
            if off + 4 * n > len(data):
                raise ValueError("truncated model file %s" % path)
            t.copy_(torch.from_numpy(np.frombuffer(data, "<f4", n, off).copy()).view(t.shape))
            off += 4 * n
    if off != len(data):
        raise ValueError("trailing bytes in model file %s" % path)
    return net


# -- rows ---------------------------------------------------------------------
ROW_KEYS = ("binaryInputNCHWPacked", "globalInputNC", "policyTargetsNCMove", "globalTargetsNC", "valueTargetsNCHW")


def load_rows(paths):
    """Concatenates the arrays of one or more engine .npz files (np.load, no pickle)."""
    if isinstance(paths, str):
        paths = [paths]
    parts = {k: [] for k in ROW_KEYS}
    for p in paths:
        with np.load(p) as z:
            for k in ROW_KEYS:
                parts[k].append(z[k])
    return {k: np.concatenate(v) for k, v in parts.items()}


def unpack_planes(packed, X, Y):
    """[N, 15, ceil(A/8)] big-endian bit-packed planes (trainingwrite.cpp packBits
    :218-232) -> [N, 15, Y, X] f32."""
    A = X * Y
    bits = np.unpackbits(packed, axis=-1, bitorder="big")[..., :A]
    return bits.reshape(packed.shape[0], packed.shape[1], Y, X).astype(np.float32)


def rows_to_batch(rows, X, Y, device="cpu"):
    """Tensors for one training batch: inputs, the normalised policy target of the move
    played (row policy [0]), its weight, and the (win, loss) value target with draws
    split (final outcome = globalTargets[0:2], trainingwrite.cpp fillValueTDTargets
    with now-factor 0)."""
    binp = torch.from_numpy(unpack_planes(rows["binaryInputNCHWPacked"], X, Y)).to(device)
    glob = torch.from_numpy(rows["globalInputNC"].astype(np.float32)).to(device)
    pol = rows["policyTargetsNCMove"][:, 0, :].astype(np.float32)
    psum = pol.sum(axis=1, keepdims=True)
    pw = (psum[:, 0] > 0).astype(np.float32)
    pol = pol / np.maximum(psum, 1.0)
    gt = rows["globalTargetsNC"]
    win, loss = gt[:, 0], gt[:, 1]
    draw = np.clip(1.0 - win - loss, 0.0, 1.0)
    vt = np.stack([win + 0.5 * draw, loss + 0.5 * draw], axis=1).astype(np.float32)
    return dict(binp=binp, glob=glob, policy=torch.from_numpy(pol).to(device),
                policy_weight=torch.from_numpy(pw).to(device), value=torch.from_numpy(vt).to(device))


def losses(net, batch):
    policy, value, _ = net(batch["binp"], batch["glob"])
    pl = -(batch["policy"] * F.log_softmax(policy, dim=1)).sum(dim=1)
    pl = (pl * batch["policy_weight"]).sum() / batch["policy_weight"].sum().clamp(min=1.0)
    vl = -(batch["value"] * F.log_softmax(value, dim=1)).sum(dim=1).mean()
    return pl, vl


def train_step(net, opt, batch, value_weight=1.0):
    opt.zero_grad()
    pl, vl = losses(net, batch)
    total = pl + value_weight * vl
    total.backward()
    opt.step()
    return pl.item(), vl.item()
