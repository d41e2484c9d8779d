"""Data parallelism at world 3 / 4 / 8 on CPU (gloo), through our launcher: the flagship
trainer in lockstep with a rank-consistent NaN skip under both DP plans, ZeRO-1 shard padding at
non-power-of-two worlds, ZeRO vs all-reduce agreement, and uneven validation shards whose global metrics
equal the single-process ones."""
import os
import sys

import pytest

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch

HERE = os.path.dirname(os.path.abspath(__file__))
ENV = {"OMP_NUM_THREADS": "1", "PYTHONWARNINGS": "ignore"}


@pytest.mark.parametrize("world", [3, 4, 8])
def test_world_n_plans_and_uneven_val_shards(tmp_path, world):
    out = str(tmp_path / "wn")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "world_n.py"), out], nproc=world, extra_env=ENV)
    assert rc == 0
    rows = [open(f"{out}.{r}").read().split() for r in range(world)]
    for row in rows:
        assert row[0] == "1", row
    assert len({" ".join(r[2:]) for r in rows}) == 1   # every rank reports the same global metrics


@pytest.mark.parametrize("world,plan", [(3, "zero"), (3, "allreduce"), (4, "zero"), (8, "zero"), (8, "allreduce")])
def test_flagship_lockstep_and_nan_skip_world_n(tmp_path, world, plan):
    out = str(tmp_path / "fl")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "flagship_dp.py"), out], nproc=world,
                extra_env=dict(ENV, QDML_DP_PLAN=plan))
    assert rc == 0
    for r in range(world):
        same, skipped, flag = open(f"{out}.{r}").read().split()
        assert same == "1" and skipped == "1" and float(flag) >= 1.0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_flagship_strong_scaling_is_dataparallel_semantics(tmp_path, world):
    """FlagshipConfig.scaling="strong" (bench.py --scaling strong): each rank holds its contiguous part of ONE
    global batch, the NMSE denominators are the global batch's, the QSC matches a 1-process run on the whole
    batch, and the ranks stay bit-identical (tests/dist_scripts/flagship_strong.py)."""
    out = str(tmp_path / "st")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "flagship_strong.py"), out], nproc=world,
                extra_env=ENV)
    assert rc == 0
    for r in range(world):
        row = open(f"{out}.{r}").read()
        assert row.split()[0] == "1", row
