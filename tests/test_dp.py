"""Multi-process data parallelism on CPU (gloo, world 2) through our launcher."""
import os
import sys

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch

HERE = os.path.dirname(os.path.abspath(__file__))


def test_dp_equivalence_and_collectives(tmp_path):
    out = str(tmp_path / "res")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "dp_equivalence.py"), out], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2"})
    assert rc == 0
    rows = [open(f"{out}.{r}").read().split(" ", 3) for r in range(2)]
    for err, a, b, _ in rows:
        assert float(err) < 1e-5, err           # DP step == 1-process step on the union batch
        assert float(a) == 3.0 and float(b) == 50.0  # all-reduce of raw sums
    assert rows[0][3] != rows[1][3]             # ranks sample different indices


def test_launcher_propagates_failure():
    rc = launch([sys.executable, "-c", "import os,sys; sys.exit(3 if os.environ['RANK']=='1' else 0)"], nproc=2)
    assert rc == 3


def test_flagship_dp_lockstep_and_rank_consistent_nan_skip(tmp_path):
    out = str(tmp_path / "fl")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "flagship_dp.py"), out], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2"})
    assert rc == 0
    for r in range(2):
        same, skipped, flag = open(f"{out}.{r}").read().split()
        assert same == "1"           # parameters bit-identical across ranks after every step
        assert skipped == "1"        # the NaN on rank 1 made BOTH ranks skip
        assert float(flag) >= 1.0    # the summed skip flag
