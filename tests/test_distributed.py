"""World-size-2 gloo test (CPU) of the multi-GPU data path: ranks own disjoint game
slots (slot_base = rank * games) and rank 0 gathers every rank's finished rows.
Rows come from the oracle engine here (same row format as the device engine)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from katacoffee_amd import rows as R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    games = 2
    sp = oracle.Selfplay(5, 5, 4, games=games, max_visits=12, node_cap=64, seed=7, slot_base=rank * games)
    sp.rounds(400)
    rows = sp.rows()
    got = R.gather_to_rank0(rows, 5, 5, dist, "cpu")
    if rank == 0:
        q.put({k: v for k, v in got.items()})
    else:
        q.put(len(rows["meta"]))
    dist.barrier()
    dist.destroy_process_group()


def test_row_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gathered = [r for r in res if isinstance(r, dict)][0]
    other = [r for r in res if not isinstance(r, dict)][0]
    slots = set(gathered["meta"][:, 0].tolist())
    # rank 0 owns slots {0,1}, rank 1 owns {2,3}: both ranks' rows arrive, disjoint slots
    assert slots & {0, 1} and slots & {2, 3}
    assert (gathered["meta"][:, 0] >= 2).sum() == other
    # rows of rank 1 equal what a standalone engine with the same slot_base produces
    from oracle import oracle
    sp = oracle.Selfplay(5, 5, 4, games=2, max_visits=12, node_cap=64, seed=7, slot_base=2)
    sp.rounds(400)
    ref = sp.rows()
    sel = gathered["meta"][:, 0] >= 2
    for k in R.NPZ_FIELDS + ["meta"]:
        np.testing.assert_array_equal(gathered[k][sel], ref[k])


def _packed_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    rb = R.row_bytes(5, 5)
    n = [3, 0, 7][rank]  # ragged blocks, one rank with no rows
    blk = torch.full((n, rb), rank + 1, dtype=torch.uint8)
    if n:
        blk[:, 0] = torch.arange(n, dtype=torch.uint8)
    got = R.gather_packed_to_rank0(blk, dist)
    q.put((rank, None if got is None else got.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_packed_gather_world3_ragged():
    """The device-block gather (bench.py's path, here on CPU tensors): ragged counts and
    an empty rank arrive on rank 0 in rank order, nothing elsewhere."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_packed_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None and res[2] is None
    got = res[0]
    assert got.shape == (10, R.row_bytes(5, 5))
    np.testing.assert_array_equal(got[:3, 1], 1)
    np.testing.assert_array_equal(got[3:, 1], 3)
    np.testing.assert_array_equal(got[:3, 0], np.arange(3))
    np.testing.assert_array_equal(got[3:, 0], np.arange(7))


def test_pack_roundtrip():
    rng = np.random.default_rng(0)
    n = 5
    sh = R.shapes(5, 5)
    rows = {f: (rng.integers(-100, 100, size=(n,) + sh[f]).astype(t)) for f, t in R.FIELDS}
    back = R.unpack(R.pack(rows, 5, 5), 5, 5)
    for f, _ in R.FIELDS:
        np.testing.assert_array_equal(back[f], rows[f])
    assert R.row_bytes(5, 5) == 15 * 4 + 4 + 400 + 256 + 125 + 16


def _bcast_worker(rank, world, port, path, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from katacoffee_amd import weights
    data = weights.broadcast_model(path if rank == 0 else None, dist, "cpu")
    q.put((rank, data))
    dist.barrier()
    dist.destroy_process_group()


def test_model_broadcast_world2(tmp_path):
    """Hot reload across ranks: rank 0 broadcasts the new CFNN image and
    every rank receives the file's exact bytes, which load as the same network."""
    import katacoffee_amd as kc
    path = str(tmp_path / "new.cfnn")
    kc.write_random_model("b6c96", 99, path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = open(path, "rb").read()
    assert got[0] == ref and got[1] == ref
    back = str(tmp_path / "received.cfnn")
    open(back, "wb").write(got[1])
    assert kc.model_flops(back, 25) == kc.model_flops(path, 25)


class _ListWriter:
    def __init__(self):
        self.blocks = []

    def put(self, rows):
        self.blocks.append(rows)


def _sink_worker(rank, world, port, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    rng = np.random.default_rng(rank)
    sh = R.shapes(5, 5)
    w = _ListWriter() if (mode == "local" or rank == 0) else None
    sink = R.RowSink(5, 5, dist, mode, w)
    sent = []
    for step in range(3):  # bench.py's steps: ragged blocks, one empty
        n = [(2, 5), (0, 4), (3, 1)][step][rank]
        rows = {f: rng.integers(0, 100, size=(n,) + sh[f]).astype(t) for f, t in R.FIELDS}
        rows["meta"][:, 0] = rank
        sent.append(rows)
        sink.put(torch.from_numpy(R.pack(rows, 5, 5)))
    tot = sink.totals("cpu", written=sum(len(b["meta"]) for b in w.blocks) if w else 0, files=len(w.blocks) if w else 0)
    q.put((rank, tot, None if w is None else [b["meta"] for b in w.blocks], [r["meta"] for r in sent]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["local", "gather"])
def test_row_sink_world2(mode):
    """bench.py's per-step row hand-off at world size 2: local -- each rank writes exactly
    its own rows and no collective runs until totals(); gather -- rank 0 writes every
    rank's rows in rank order.  Both report the same job totals."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sink_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = 2 + 5 + 0 + 4 + 3 + 1
    for rank in (0, 1):
        received, written, files, per_rank = res[rank][0]
        assert (received, written) == (total, total) and per_rank == [5, 10]
    if mode == "local":
        for rank in (0, 1):
            got, sent = res[rank][1], res[rank][2]
            assert np.concatenate(got).tolist() == np.concatenate(sent).tolist()
        assert res[0][0][2] == 6  # every rank's writer got its 3 blocks
    else:
        got = np.concatenate(res[0][1])
        exp = np.concatenate([np.concatenate([res[0][2][s], res[1][2][s]]) for s in range(3)])
        assert got.tolist() == exp.tolist()
        assert res[1][1] is None and res[0][0][2] == 3  # rank 0's writer got one block per step
