"""Network-only timing over batches of random V1 positions (fused or layered path).
usage: python tools/nn_bench.py [--arch b6c96] [--board 5] [--precision fast] [--n 512,2048] [--iters 20]"""
import argparse
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="4096")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--arch", default="b6c96")
    ap.add_argument("--board", type=int, default=5)
    ap.add_argument("--precision", default="fast")
    a = ap.parse_args()
    import numpy as np
    import torch

    import katacoffee_amd as kc
    X = Y = a.board
    W = 4 if X == 5 else 5
    A = X * Y
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model(a.arch, 1, path)
    net = kc.Network(path, X, Y, W, precision=a.precision)
    flops1 = kc.model_flops(path, A)
    for n in [int(v) for v in a.n.replace("/", ",").split(",")]:
        rng = np.random.default_rng(0)
        cells = rng.integers(0, 3, size=(n, A)).astype(np.uint8)
        hc = np.full((n, 5), -1, np.int8)
        hd = np.full((n, 5), 4, np.int8)
        pla = rng.integers(1, 3, size=n).astype(np.uint8)
        sym = rng.integers(0, 8, size=n).astype(np.int32)
        packed, _ = kc.encode_batch(X, Y, W, cells, hc, hd, pla, sym, want_planes=False)
        din = torch.from_numpy(packed.view(np.int64)).cuda()
        out = torch.zeros((n, 4 * A + 4), dtype=torch.float32, device="cuda")
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
        print("%s %dx%d %s fused=%d n=%d  %.1f us/forward  %.1f TFLOP/s (%.3f of 2.5 PF)" %
              (a.arch, X, Y, a.precision, net.fused, n, ms * 1000, flops1 * n / (ms * 1e-3) / 1e12,
               flops1 * n / (ms * 1e-3) / 2.5e15), flush=True)
    net.close()


if __name__ == "__main__":
    main()
