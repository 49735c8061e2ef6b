"""Training-row blocks: packing for the cross-rank gather and the .npz row format.

Row arrays (trainingwrite.cpp:185-205, numpywrite.cpp:100-175), per row at area A,
policy size P = 4A, pb = ceil(A/8):
  binaryInputNCHWPacked  u8  [15][pb]
  globalInputNC          f32 [1]
  policyTargetsNCMove    i16 [2][P]
  globalTargetsNC        f32 [64]
  valueTargetsNCHW       i8  [5][Y][X]
  meta                   i32 [4]   (slot, game number, turn, moves) — engine bookkeeping
"""
import numpy as np

FIELDS = [("binaryInputNCHWPacked", np.uint8), ("globalInputNC", np.float32), ("policyTargetsNCMove", np.int16),
          ("globalTargetsNC", np.float32), ("valueTargetsNCHW", np.int8), ("meta", np.int32)]
NPZ_FIELDS = [f for f, _ in FIELDS if f != "meta"]


def shapes(X, Y):
    A = X * Y
    return {"binaryInputNCHWPacked": (15, (A + 7) // 8), "globalInputNC": (1,), "policyTargetsNCMove": (2, 4 * A),
            "globalTargetsNC": (64,), "valueTargetsNCHW": (5, Y, X), "meta": (4,)}


def row_bytes(X, Y):
    sh = shapes(X, Y)
    return sum(int(np.prod(sh[f])) * np.dtype(t).itemsize for f, t in FIELDS)


def pack(rows, X, Y):
    """dict of row arrays -> contiguous uint8 [n][row_bytes]."""
    n = len(rows["meta"])
    parts = [np.ascontiguousarray(rows[f], dtype=t).reshape(n, -1).view(np.uint8) for f, t in FIELDS]
    return np.concatenate(parts, axis=1) if n else np.zeros((0, row_bytes(X, Y)), np.uint8)


def unpack(buf, X, Y):
    sh = shapes(X, Y)
    n = buf.shape[0]
    out, off = {}, 0
    for f, t in FIELDS:
        nb = int(np.prod(sh[f])) * np.dtype(t).itemsize
        out[f] = np.ascontiguousarray(buf[:, off:off + nb]).view(t).reshape((n,) + sh[f])
        off += nb
    return out


def gather_to_rank0(rows, X, Y, dist, device):
    """Gathers every rank's row block to rank 0 (the writer rank), the engine's only
    collective.  Counts are all-gathered, blocks padded to the largest.
    Returns the concatenated rows on rank 0 and None elsewhere."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    buf = pack(rows, X, Y)
    n = buf.shape[0]
    cnt = torch.tensor([n], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    counts = [int(c.item()) for c in cnts]
    mx = max(counts)
    rb = row_bytes(X, Y)
    pad = torch.zeros((max(mx, 1), rb), dtype=torch.uint8, device=device)
    if n:
        pad[:n] = torch.from_numpy(buf).to(device)
    outs = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, outs, dst=0)
    if rank != 0:
        return None
    blocks = [o[:c].cpu().numpy() for o, c in zip(outs, counts)]
    return unpack(np.concatenate(blocks, axis=0), X, Y)
