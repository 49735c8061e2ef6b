"""`katago selfplay` (the process boundary, command/selfplay.cpp:44-72): runs the CLI
for a few games and reads its .npz output back with numpy, like python/train.py."""
import glob
import os
import subprocess

import numpy as np
import pytest

import katacoffee_amd as kc

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cli_selfplay_writes_training_npz(tmp_path):
    models = tmp_path / "models"
    models.mkdir()
    kc.write_random_model("b6c96", 5, str(models / "b6c96-s0.cfnn"))
    out = tmp_path / "out"
    cmd = [os.path.join(REPO, "katacoffee_amd", "katago"), "selfplay", "-config",
           os.path.join(REPO, "configs", "selfplay_coffee5.cfg"), "-models-dir", str(models), "-output-dir", str(out),
           "-max-games-total", "40", "-override-config", "numGameThreads=64,maxVisits=16,maxRowsPerTrainFile=100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    files = glob.glob(str(out / "b6c96-s0" / "tdata" / "*.npz"))
    assert files, r.stdout
    assert glob.glob(str(out / "log*.log"))
    total = 0
    for f in files:
        with np.load(f) as z:
            n = z["globalTargetsNC"].shape[0]
            assert 0 < n <= 100
            assert z["binaryInputNCHWPacked"].shape == (n, 15, 4) and z["binaryInputNCHWPacked"].dtype == np.uint8
            assert z["globalInputNC"].shape == (n, 1)
            assert z["policyTargetsNCMove"].shape == (n, 2, 100) and z["policyTargetsNCMove"].dtype == np.int16
            assert z["valueTargetsNCHW"].shape == (n, 5, 5, 5) and z["valueTargetsNCHW"].dtype == np.int8
            np.testing.assert_array_equal(z["globalTargetsNC"][:, 63], 1.0)
            assert z["policyTargetsNCMove"][:, 0].sum(axis=1).min() > 0
            total += n
    assert total >= 40 * 5  # every finished game has at least five moves
