"""Child script for tests/test_bench_launcher.py: joins the process group the
bench launcher's environment describes (gloo on CPU) and checks its rank/world."""
import json
import os
import sys

import torch
import torch.distributed as dist

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
assert rank == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"])
assert world == int(os.environ["WORLD_SIZE"]) == int(sys.argv[1])
t = torch.tensor([rank + 1])
dist.all_reduce(t)
out = sys.argv[2]
with open("%s.%d" % (out, rank), "w") as f:
    json.dump({"rank": rank, "world": world, "sum": int(t.item())}, f)
dist.destroy_process_group()
