"""Network-only timing: the fused forward over a batch of random V1 positions.
usage: python tools/nn_bench.py [--n 4096] [--iters 50] [--arch b6c96]"""
import argparse
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--arch", default="b6c96")
    a = ap.parse_args()
    import numpy as np
    import torch

    import katacoffee_amd as kc
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model(a.arch, 1, path)
    rng = np.random.default_rng(0)
    n = a.n
    cells = rng.integers(0, 3, size=(n, 25)).astype(np.uint8)
    hc = np.full((n, 5), -1, np.int8)
    hd = np.full((n, 5), 4, np.int8)
    pla = rng.integers(1, 3, size=n).astype(np.uint8)
    sym = rng.integers(0, 8, size=n).astype(np.int32)
    packed, _ = kc.encode_batch(5, 5, 4, cells, hc, hd, pla, sym, want_planes=False)
    net = kc.Network(path, 5, 5, 4)
    din = torch.from_numpy(packed.view(np.int64)).cuda()
    out = torch.zeros((n, 104), dtype=torch.float32, device="cuda")
    for _ in range(3):
        net.forward_device(n, din, out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        net.forward_device(n, din, out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    flops = kc.model_flops(path, 25) * n
    print("n=%d  %.1f us/launch  %.1f TFLOP/s" % (n, ms * 1000, flops / (ms * 1e-3) / 1e12))


if __name__ == "__main__":
    main()
