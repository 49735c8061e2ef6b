import os, sys, tempfile
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import katacoffee_amd as kc
from katacoffee_amd import train
import test_gpu_train as T
net, batch = T._trained(10)
f = T._hot_net(net, batch, 20000.0)
path = os.path.join(tempfile.mkdtemp(), "h.cfnn"); train.save_cfnn(net, path)
planes = batch["binp"].numpy().reshape(-1, 15, 25); packed = T._pack_u64(planes)
with torch.no_grad():
    pol, val, misc = net(batch["binp"], batch["glob"])
ref = np.concatenate([pol.numpy(), val.numpy(), misc.numpy()], axis=1)
out = {}
for p in ("corrected", "accurate", "fast"):
    h = kc.Network(path, 5, 5, 4, precision=p); out[p] = h.forward(packed); h.close()
c, a = out["corrected"], out["accurate"]
same = (np.abs(c - a).max(axis=1) == 0)
print("boards", len(c), "identical to accurate:", int(same.sum()), "corrected err", np.abs(c - ref).max(), "accurate err", np.abs(a - ref).max(), "fast err", np.abs(out["fast"] - ref).max())
e = np.abs(c - ref).max(axis=1)
print("per-board corrected err (first 20):", np.round(e[:20], 4).tolist())
print("nan in corrected:", np.isnan(c).sum())
