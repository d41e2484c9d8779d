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


import pytest  # noqa: E402


@pytest.mark.parametrize("plan", ["zero", "allreduce"])
def test_flagship_dp_lockstep_and_rank_consistent_nan_skip(tmp_path, plan):
    out = str(tmp_path / "fl")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "flagship_dp.py"), out], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2", "QDML_DP_PLAN": plan})
    assert rc == 0
    for r in range(2):
        same, skipped, flag = open(f"{out}.{r}").read().split()
        assert same == "1"           # parameters bit-identical across ranks after every step
        assert skipped == "1"        # the NaN on rank 1 made BOTH ranks skip
        assert float(flag) >= 1.0    # the summed skip flag


def test_zero_plan_bit_identical_to_allreduce_plan(tmp_path):
    """ZeRO-1 FC optimizer (reduce-scatter, Adam on a 1/world shard, all-gather) == all-reduce plan."""
    out = str(tmp_path / "z")
    rc = launch([sys.executable, os.path.join(HERE, "dist_scripts", "zero_vs_allreduce.py"), out], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2"})
    assert rc == 0
    for r in range(2):
        rec = open(f"{out}.{r}").read().split()
        assert rec[0] == "1", rec


def _bench(args, env_extra=None, timeout=600):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"OMP_NUM_THREADS": "2", "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    env.update(env_extra or {})
    root = os.path.dirname(HERE)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=root)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


SMALL = ["--steps", "2", "--warmup", "1", "--batch", "4", "--data-len", "200", "--qubits", "4", "--dtype", "fp32"]


def test_bench_self_launches_n_ranks():
    """`python bench.py --gpus 2` without torchrun starts 2 ranks itself and reports dp2 (one JSON line)."""
    rc, recs, err = _bench(["--gpus", "2"] + SMALL + ["--phase-steps", "0"])
    assert rc == 0, err[-2000:]
    assert len(recs) == 1, recs
    r = recs[0]
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["global_batch"] == 2 * r["config"]["per_gpu_batch"]
    # the plan is chosen at the real world size by timing both candidates
    sel = r["config"]["plan_select_ms"]
    assert set(sel) == {"zero", "allreduce"} and r["config"]["dp_plan"] == min(sel, key=sel.get)
    assert r["dp_fallback"] is None


def test_bench_strong_scaling_line():
    """`bench.py --gpus 2 --scaling strong`: one global batch of 9 x batch rows per step, split over the ranks
    (the reference's DataParallel semantics) -- the line says "strong" and the per-rank batch."""
    rc, recs, err = _bench(["--gpus", "2", "--scaling", "strong", "--dp-plan", "allreduce"] + SMALL +
                           ["--phase-steps", "0"])
    assert rc == 0, err[-2000:]
    assert len(recs) == 1, recs
    r = recs[0]
    assert r["scaling"] == "strong" and r["config"]["per_rank_stream_batch"] == 2
    assert r["config"]["global_batch"] == 9 * 4 and r["config"]["per_gpu_batch"] == 9 * 2


def test_bench_supervisor_falls_back_when_a_rank_fails():
    """A rank that fails in the first attempt makes EVERY rank restart with the 5-graph plan; exactly one
    JSON line (the successful attempt's) is printed, and it names the fallback."""
    rc, recs, err = _bench(["--gpus", "2"] + SMALL + ["--phase-steps", "0", "--dp-plan", "allreduce"],
                           env_extra={"QDML_BENCH_FAIL_RANK": "1"})
    assert rc == 0, err[-2000:]
    assert len(recs) == 1, recs
    assert recs[0]["dp_fallback"] and "rank 1" in recs[0]["dp_fallback"], recs[0]
    assert recs[0]["config"]["dp_graph"] == "five"


def test_bench_world_mismatch_is_an_error():
    rc, recs, err = _bench(["--gpus", "2"] + SMALL, env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not recs
    assert "WORLD_SIZE" in err


def test_capture_preflight_ranks_agree_and_fall_back(tmp_path):
    """bench.py's RCCL capture pre-flight (parallel/capture_probe.py): each rank's child probe fails here
    (no GPU) and both ranks agree on False -- the 5-graph DP plan -- without touching a GPU themselves."""
    import os
    import sys
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "pf")
    rc = launch([sys.executable, os.path.join(here, "dist_scripts", "preflight_agree.py"), out], nproc=2,
                extra_env={"OMP_NUM_THREADS": "1"})
    assert rc == 0
    assert [open(f"{out}.{r}").read().strip() for r in range(2)] == ["0", "0"]


def test_rccl_gpu_check_is_per_node():
    """One GPU per rank OF THIS NODE: a 2 x 8 job (WORLD_SIZE 16) on 8-GPU nodes is fine; 9 local ranks,
    or a LOCAL_RANK past the node's GPUs, are not."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import check_local_gpus
    check_local_gpus(local_rank=7, local_world=8, n_gpus=8)   # (WORLD_SIZE is not an argument at all)
    for lr, lw in ((8, 8), (0, 9)):
        with pytest.raises(RuntimeError):
            check_local_gpus(local_rank=lr, local_world=lw, n_gpus=8)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_reference_dp_semantics_matches_one_process(tmp_path, world):
    """dp_semantics="reference" (DataParallel's split of one global batch, R:144-148) == one process on the
    whole batch, for the BN-free classical SC; the HDCE trainer runs in lockstep (rank-identical weights)."""
    import torch
    one = str(tmp_path / "one")
    assert launch([sys.executable, os.path.join(HERE, "dist_scripts", "ref_semantics.py"), one], nproc=1,
                  extra_env={"OMP_NUM_THREADS": "2", "PYTHONWARNINGS": "ignore"}) == 0
    many = str(tmp_path / "many")
    assert launch([sys.executable, os.path.join(HERE, "dist_scripts", "ref_semantics.py"), many], nproc=world,
                  extra_env={"OMP_NUM_THREADS": "1", "PYTHONWARNINGS": "ignore"}) == 0
    a = torch.load(f"{one}.0.pt", weights_only=True)
    for r in range(world):
        b = torch.load(f"{many}.{r}.pt", weights_only=True)
        assert torch.allclose(a["sc"], b["sc"], rtol=1e-4, atol=1e-6), float((a["sc"] - b["sc"]).abs().max())
        assert torch.allclose(a["sc_loss"], b["sc_loss"], rtol=1e-5)
        same, hl, _ = open(f"{many}.{r}").read().split()
        assert same == "1" and float(hl) == float(hl)


def test_dp_qsc_placement_needs_the_one_graph_plan():
    """cfg.dp_qsc "fwd" forks the QSC branch in g1a and joins it in g2: only the one-graph DP plan holds both in
    one capture, so any other plan refuses it (instead of silently running the "g2" placement)."""
    import torch
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)
    ctx = DistContext(device=torch.device("cpu"))
    for bad in (dict(dp_qsc="fwd", split_graphs=True), dict(dp_qsc="later")):
        with pytest.raises(ValueError, match="dp_qsc"):
            FlagshipTrainer(FlagshipConfig(n_qubits=4, batch=4, data_len=100, dtype="fp32", **bad), ctx)
