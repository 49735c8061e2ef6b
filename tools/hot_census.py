"""How often does the corrected network fall back (activations past e4m3's 448)?  Prints,
for random-init and bench nets, the default precision's choice, its calibration difference
and the corrected-vs-accurate difference on game positions.
usage: python tools/hot_census.py"""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import katacoffee_amd as kc  # noqa: E402
from test_gpu_composition import _rows_of_game_positions  # noqa: E402

for seed in (0xC0FFEE, 1, 2, 3):
    path = os.path.join(tempfile.mkdtemp(), "m.cfnn")
    kc.write_random_model("b6c96", seed, path)
    packed = _rows_of_game_positions(5, 5, 4, 2048, seed=7)
    d = kc.Network(path, 5, 5, 4, precision="default")
    c = kc.Network(path, 5, 5, 4, precision="corrected")
    a = kc.Network(path, 5, 5, 4, precision="accurate")
    oc, oa = c.forward(packed), a.forward(packed)
    print("b6c96 seed %#x: default -> %s (calibration %.3g); corrected vs accurate on 2048 positions: max %.3g, "
          "rows identical to accurate (fell back): %d" % ((seed,) + d.precision + (float(np.abs(oc - oa).max()),
          int((np.abs(oc - oa).max(axis=1) == 0).sum()))), flush=True)
    for h in (d, c, a):
        h.close()
