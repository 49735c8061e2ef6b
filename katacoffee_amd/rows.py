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
    if n == 0:
        return np.zeros((0, row_bytes(X, Y)), np.uint8)
    parts = [np.ascontiguousarray(rows[f], dtype=t).reshape(n, -1).view(np.uint8) for f, t in FIELDS]
    return np.concatenate(parts, axis=1)


def unpack(buf, X, Y):
    sh = shapes(X, Y)
    n = buf.shape[0]
    out, off = {}, 0
    for f, t in FIELDS:
        nb = int(np.prod(sh[f])) * np.dtype(t).itemsize
        out[f] = np.ascontiguousarray(buf[:, off:off + nb]).view(t).reshape((n,) + sh[f])
        off += nb
    return out


def gather_packed_to_rank0(packed, dist):
    """Gathers every rank's packed row block (uint8 tensor [n][row_bytes] on the process
    group's device: the engines' staged rows, coffee_selfplay_stage_rows) to rank 0, the
    writer rank -- the engine's only collective.  The counts are all-gathered
    (one small host read on the collective's stream), blocks padded to the largest and
    gathered (RCCL over xGMI for "nccl"; the rows never visit this rank's host).  Returns
    the concatenated block on rank 0 (same device) and None elsewhere."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    n, rb = packed.shape
    cnt = torch.tensor([n], dtype=torch.int64, device=packed.device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    counts = [int(c.item()) for c in cnts]
    pad = torch.zeros((max(max(counts), 1), rb), dtype=torch.uint8, device=packed.device)
    if n:
        pad[:n] = packed
    outs = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, outs, dst=0)
    if rank != 0:
        return None
    return torch.cat([o[:c] for o, c in zip(outs, counts)])


def gather_to_rank0(rows, X, Y, dist, device):
    """gather_packed_to_rank0 for host row dicts: packed, gathered on `device`, unpacked
    on rank 0 (None elsewhere)."""
    import torch
    buf = torch.from_numpy(pack(rows, X, Y)).to(device)
    out = gather_packed_to_rank0(buf, dist)
    return None if out is None else unpack(out.cpu().numpy(), X, Y)


class RowSink:
    """Where a rank's staged row block goes after every bench step.

    mode "local" (the default): every rank unpacks its own block and hands it to its own
    writer (its own .npz files) -- games are sharded, so no collective runs in the data
    path and no rank waits for another inside the loop; "gather": the blocks are gathered
    to rank 0 over RCCL first (gather_packed_to_rank0: one writer for the job, a global
    synchronisation point per step).  `writer` (None: count only) takes row dicts.
    totals() all-reduces the counts once the timed window is over."""

    def __init__(self, X, Y, dist=None, mode="local", writer=None):
        if mode not in ("local", "gather"):
            raise ValueError("row sink mode must be local or gather")
        self.X, self.Y, self.dist, self.mode, self.writer = X, Y, dist, mode, writer
        self.handed = 0    # rows this rank staged
        self.received = 0  # rows this rank unpacked for writing (every rank's in gather mode on rank 0)

    def put(self, packed):
        """packed: uint8 tensor [n][row_bytes] on this rank's device."""
        self.handed += int(packed.shape[0])
        if self.mode == "gather" and self.dist is not None:
            packed = gather_packed_to_rank0(packed, self.dist)
            if packed is None:
                return
        rows = unpack(packed.cpu().numpy(), self.X, self.Y)
        self.received += len(rows["meta"])
        if self.writer is not None:
            self.writer.put(rows)

    def totals(self, device, written=0, files=0):
        """(rows received for writing, rows written, files written) summed over the job,
        and the rows each rank staged (list by rank)."""
        if self.dist is None:
            return self.received, written, files, [self.handed]
        import torch
        t = torch.tensor([self.received, written, files], dtype=torch.int64, device=device)
        self.dist.all_reduce(t)
        h = torch.tensor([self.handed], dtype=torch.int64, device=device)
        per = [torch.zeros_like(h) for _ in range(self.dist.get_world_size())]
        self.dist.all_gather(per, h)
        r, w, f = (int(x) for x in t.tolist())
        return r, w, f, [int(x.item()) for x in per]
