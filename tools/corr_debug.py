"""Corrected-precision network vs the oracle's fp32 / fp16 / corrected emulations for
the library in KATACOFFEE_LIB (A/B builds with -DKC_F8C_DEBUG, nn.hip)."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import katacoffee_amd as kc  # noqa: E402
from oracle import oracle  # noqa: E402
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_gpu_nn import _boards, _pack_u64  # noqa: E402

path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
kc.write_random_model("b6c96", 0xC0FFEE, path)
binp, glob = _boards(203, 5, 5, 4, seed=203)
m = oracle.Model(path)
ref = {}
for mode in (0, 1, 2):
    p, v, mi = m.forward(5, 5, binp, glob, mode=mode, threads=8)
    ref[mode] = np.concatenate([p.reshape(203, -1), v, mi], axis=1)
for prec in ("fast", "accurate", "corrected"):
    net = kc.Network(path, 5, 5, 4, precision=prec)
    out = net.forward(_pack_u64(binp))
    net.close()
    print(os.environ.get("KATACOFFEE_LIB", "main"), prec, " ".join(
        "vs%s %.3e" % (n, np.abs(out - ref[k]).max()) for k, n in ((0, "fp32"), (1, "fp16"), (2, "corr"))), flush=True)

# error structure of the corrected path: per board, per output block
net = kc.Network(path, 5, 5, 4, precision="corrected")
out = net.forward(_pack_u64(binp))
fastn = kc.Network(path, 5, 5, 4, precision="fast")
outf = fastn.forward(_pack_u64(binp))
e = np.abs(out - ref[0])
print("per-board max err (first 12):", np.round(e.max(axis=1)[:12], 4).tolist())
print("boards with err > 1e-3:", int((e.max(axis=1) > 1e-3).sum()), "of", len(e))
print("policy / value / misc max err:", e[:, :100].max(), e[:, 100:102].max(), e[:, 102:].max())
print("corrected - fast max:", np.abs(out - outf).max(), " oracle corr - fp16:", np.abs(ref[2] - ref[1]).max())
for n in (1, 2, 5, 6):
    o = net.forward(_pack_u64(binp[:n]))
    print("n=%d max err %.3e" % (n, np.abs(o - ref[0][:n]).max()))
