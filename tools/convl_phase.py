"""Cycle accounting of the layered 3x3 conv kernel (kConvLB, or kConvL with --precision accurate) over network forwards of
random positions: per workgroup, the cycles of its prologue, weight waits (vmcnt +
barrier per tap group), slice stage stores (with the wait for the slice's loads) and
epilogue, against the MFMA issue floor of its K loop.
Needs the profiling build:  make -C katacoffee_amd/csrc prof
usage: python tools/convl_phase.py [--arch b10c128] [--board 5] [--n 4450] [--iters 10]"""
import argparse
import ctypes
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KATACOFFEE_LIB", os.path.join(REPO, "tools", "_build", "libkatacoffee_prof.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="b10c128")
    ap.add_argument("--board", type=int, default=5)
    ap.add_argument("--n", default="4450")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--precision", default="fast", help="fast: kConvLB (fast-layered); accurate: kConvL split")
    a = ap.parse_args()
    import numpy as np
    import torch

    import katacoffee_amd as kc
    L = kc.lib()
    L.coffee_debug_convl_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    X = Y = a.board
    W = 4 if X == 5 else 5
    A = X * Y
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model(a.arch, 1, path)
    net = kc.Network(path, X, Y, W, precision=a.precision)
    prof = (ctypes.c_ulonglong * 8)()
    for n in [int(v) for v in a.n.split(",")]:
        rng = np.random.default_rng(0)
        cells = rng.integers(0, 3, size=(n, A)).astype(np.uint8)
        hc = np.full((n, 5), -1, np.int8)
        hd = np.full((n, 5), 4, np.int8)
        pla = rng.integers(1, 3, size=n).astype(np.uint8)
        sym = rng.integers(0, 8, size=n).astype(np.int32)
        packed, _ = kc.encode_batch(X, Y, W, cells, hc, hd, pla, sym, want_planes=False)
        din = torch.from_numpy(packed.view(np.int64)).cuda()
        out = torch.zeros((n, 4 * A + 4), dtype=torch.float32, device="cuda")
        net.forward_device(n, din, out)
        torch.cuda.synchronize()
        L.coffee_debug_convl_profile(prof, 1)
        for _ in range(a.iters):
            net.forward_device(n, din, out)
        torch.cuda.synchronize()
        L.coffee_debug_convl_profile(prof, 1)
        wgs = max(1, prof[0])
        names = ["total", "prologue", "weight waits", "stage stores", "epilogue"]
        row = {nm: prof[i + 1] / wgs for i, nm in enumerate(names)}
        row["k loop rest"] = row["total"] - sum(row[k] for k in names[1:])
        print("%s %dx%d n=%d %s: %d %s workgroups/forward; cycles per workgroup: %s" %
              (a.arch, X, Y, n, a.precision, prof[0] // a.iters, "kConvLB" if a.precision.startswith("fast") else "kConvL", ", ".join("%s %.0f" % (k, v) for k, v in row.items())),
              flush=True)
    net.close()


if __name__ == "__main__":
    main()
