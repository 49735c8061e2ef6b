"""Device-resident row hand-off (coffee_selfplay_stage_rows, the bench's multi-GPU row
path): the packed device block of an engine equals, row for row and byte for
byte, what coffee_selfplay_drain_rows copies out of an identical engine; staging is
stream-ordered (later steps may be enqueued before the rows are consumed) and empties
the row buffer (and, on request, the finished-game records)."""
import numpy as np
import pytest
import torch

import katacoffee_amd as kc
from katacoffee_amd import rows as R

pytestmark = pytest.mark.gpu


def _engine():
    return kc.Selfplay(5, 5, 4, num_games=64, max_visits=12, seed=21, node_cap=64, commit_interval=4,
                       nn_cache_log2=8, use_fake_net=True)


def test_stage_rows_matches_drain():
    a, b = _engine(), _engine()
    a.step(600)
    b.step(600)
    ref = a.drain_rows()
    n_ref = len(ref["meta"])
    assert n_ref > 0
    rb = kc.row_bytes(5, 5)
    assert rb == R.row_bytes(5, 5)
    buf = torch.empty((b.row_capacity(), rb), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64).pin_memory()
    stream = torch.cuda.ExternalStream(b.stream_ptr())
    ev = torch.cuda.Event()
    b.stage_rows(buf, cnt[0], discard_games=True)
    ev.record(stream)
    b.step(200)  # enqueued behind the staging: must not touch the staged block
    ev.synchronize()
    n = int(cnt[0])
    assert n == n_ref
    # rows take their buffer slots by atomic counter, so the two engines' row orders may
    # differ: compare the sets of packed records (each row byte for byte)
    got = buf[:n].cpu().numpy()
    want = R.pack(ref, 5, 5).reshape(n, rb)
    assert got.shape == want.shape
    order = lambda a: a[np.lexsort(a.T[::-1])]
    np.testing.assert_array_equal(order(got), order(want))
    R.unpack(got, 5, 5)  # the staged block parses as rows.py records
    b.sync()
    st = b.stats()
    # the buffer restarted from empty: rows written count both the staged and the new ones
    assert st["rows_written"] == n + st["rows_pending"]
    header, _ = b.drain_games()
    hdr_a, _ = a.drain_games()
    assert len(hdr_a) > 0 and len(header) < len(hdr_a)  # the staged step dropped its records
    a.close()
    b.close()


def test_stage_rows_rejects_small_destination():
    e = _engine()
    rb = kc.row_bytes(5, 5)
    small = torch.empty((e.row_capacity() - 1, rb), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64).pin_memory()
    with pytest.raises(kc.CoffeeError):
        e.stage_rows(small, cnt[0])
    # a flat byte buffer with as many "rows" as the capacity holds far fewer rows
    flat = torch.empty((e.row_capacity(),), dtype=torch.uint8, device="cuda")
    with pytest.raises(AssertionError):
        e.stage_rows(flat, cnt[0])
    wide = torch.empty((e.row_capacity(), rb - 1), dtype=torch.uint8, device="cuda")
    with pytest.raises(AssertionError):
        e.stage_rows(wide, cnt[0])
    e.close()
