"""Network weights across ranks: rank 0 broadcasts a new CFNN image over the process
group (RCCL on GPU ranks, gloo on CPU), every rank hands it to its engine
(coffee_selfplay_set_model_bytes).  The reference's hot reload has every self-play
process re-read the models directory (cpp/command/selfplay.cpp:366-384); with one
process per GPU the file is read once and the bytes travel over xGMI.  SURVEY §5: the
second of the two collectives (besides the row gather, rows.py)."""
import numpy as np


def broadcast_model(path, dist, device, src=0):
    """Returns the CFNN image (bytes) of `path` on rank `src` on every rank.  `path` is
    ignored on the other ranks.  Two broadcasts: the size, then the bytes."""
    import torch
    rank = dist.get_rank()
    if rank == src:
        with open(path, "rb") as f:
            data = np.frombuffer(f.read(), dtype=np.uint8)
        size = torch.tensor([data.size], dtype=torch.int64, device=device)
    else:
        data = None
        size = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(size, src)
    n = int(size.item())
    buf = torch.from_numpy(data.copy()).to(device) if rank == src else torch.empty(n, dtype=torch.uint8, device=device)
    dist.broadcast(buf, src)
    return buf.cpu().numpy().tobytes()
