"""bench.py --gpus N starts N ranks itself (the driver's N-GPU command): the launcher's
children see torch.distributed.run's environment (RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1) and form one process group of world size N (gloo on CPU here;
RCCL on the GPU box)."""
import json
import os
import sys

import bench

HERE = os.path.dirname(os.path.abspath(__file__))


def test_launcher_forms_world_of_two(tmp_path):
    out = str(tmp_path / "probe")
    rc = bench.launch_ranks(2, script=os.path.join(HERE, "helpers", "rank_probe.py"), argv=["2", out])
    assert rc == 0
    got = [json.load(open("%s.%d" % (out, r))) for r in range(2)]
    assert [g["rank"] for g in got] == [0, 1]
    assert all(g["world"] == 2 and g["sum"] == 3 for g in got)


def test_configs_cover_baseline():
    """Every BASELINE.json GPU config has a bench workload (C2 default)."""
    cfg = json.load(open(os.path.join(os.path.dirname(HERE), "BASELINE.json")))["configs"]
    assert len(cfg) == 5 and set(bench.CONFIGS) == {"C2", "C3", "C4", "C5"}
    assert bench.CONFIGS["C2"]["games"] == 4096 and bench.CONFIGS["C2"]["visits"] == 600
    assert (bench.CONFIGS["C5"]["X"], bench.CONFIGS["C5"]["arch"]) == (9, "b18c384nbt")
