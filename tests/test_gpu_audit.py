"""GPU check of the default precision's audit on self-play's own positions (the
load-time calibration sees only seeded random-play positions).  An engine whose default
precision resolved to the corrected instance re-evaluates the first rows of every N-th
network batch on the accurate instance; the largest difference is read at each stats /
drain call, and past the tolerance (NNEngine::NN_AUTO_TOL = 2.5e-4) the engine switches
to the accurate instance for the rest of the run (selfplay.cpp auditCheck)."""
import os

import numpy as np
import pytest

import katacoffee_amd as kc

pytestmark = pytest.mark.gpu


def _engine(tmp_path, env):
    path = str(tmp_path / "b6c96.cfnn")
    kc.write_random_model("b6c96", 0xC0FFEE, path)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:  # the engine reads the overrides when it is created
        return kc.Selfplay(5, 5, 4, num_games=256, max_visits=32, seed=9, model_path=path, node_cap=128,
                           nn_cache_log2=14, commit_interval=4, nn_precision="default")
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_audit_keeps_corrected_within_tolerance(tmp_path):
    """The random-init benchmark net: audited every launch, the corrected instance stays
    far inside the tolerance and the engine keeps it."""
    sp = _engine(tmp_path, {"COFFEE_NN_AUDIT_EVERY": "1"})
    sp.step(300)
    st = sp.stats()
    sp.close()
    print("audits", st["nn_audits"], "max |diff|", st["nn_audit_max_diff"], "precision", st["nn_precision"])
    assert kc.PRECISION_NAMES[st["nn_precision"]] == "corrected"
    assert st["nn_audits"] == 300 and st["nn_audit_switches"] == 0
    assert 0.0 < st["nn_audit_max_diff"] <= 2.5e-4
    assert st["errors"] == 0


def test_audit_switches_to_accurate_past_tolerance(tmp_path):
    """A tolerance no corrected evaluation meets: the first stats call after an audit
    switches the engine to the accurate instance (same model), self-play continues on it
    and no more audits run."""
    sp = _engine(tmp_path, {"COFFEE_NN_AUDIT_EVERY": "8", "COFFEE_NN_AUDIT_TOL": "1e-12"})
    sp.step(40)
    st = sp.stats()
    assert st["nn_audit_switches"] == 1 and st["nn_audits"] == 5
    assert kc.PRECISION_NAMES[st["nn_precision"]] == "accurate"
    moves = st["moves"]
    sp.step(400)
    st2 = sp.stats()
    rows = sp.drain_rows()
    sp.close()
    assert st2["nn_audits"] == 5 and st2["nn_audit_switches"] == 1
    assert st2["errors"] == 0 and st2["moves"] > moves and len(rows["meta"]) > 0


def test_audit_switch_is_reproducible(tmp_path):
    """The switch happens at the stats / drain calls, so two runs with the same call
    sequence switch at the same round and play the same games afterwards."""
    env = {"COFFEE_NN_AUDIT_EVERY": "8", "COFFEE_NN_AUDIT_TOL": "1e-12"}
    runs = []
    for _ in range(2):
        sp = _engine(tmp_path, env)
        sp.step(40)
        st = sp.stats()
        assert st["nn_audit_switches"] == 1
        sp.step(300)
        trees = [sp.game_tree(g) for g in (0, 7, 101, 255)]
        info = [sp.game_info(g) for g in (0, 7, 101, 255)]
        rows = sp.drain_rows()
        sp.close()
        runs.append((trees, info, rows))
    (t0, i0, r0), (t1, i1, r1) = runs
    for a, b in zip(t0, t1):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    assert i0 == i1
    for k in r0:
        np.testing.assert_array_equal(r0[k], r1[k])
