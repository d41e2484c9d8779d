#!/usr/bin/env python3
"""Flagship training benchmark (driver contract).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric: training samples/sec of the P128 RIS system named in BASELINE.json
("P128 RIS, 8-qubit QuantumNAT QNN + CNN estimator, bf16"): one step = the QSC scenario
classifier (8 qubits, 3 layers, QuantumNAT noise) + the HDCE estimator (3 scenario
experts + shared 4096->2048 FC, per-stream NMSE) forward + backward + optimizer on
9 streams x 256 samples PER GPU (weak scaling; reference step R:181-204 / R:335-370),
synthetic DeepMIMO-shaped data resident in HBM, random-init weights.

W untimed warm-up steps, then K timed steps bracketed by barrier + device sync; the
slowest rank's time is used; rank 0 prints ONE JSON line with the whole-job value.
The reference publishes no throughput, so vs_baseline is null.

``python bench.py --gpus N`` (N > 1) without a torchrun environment starts the N ranks itself
(one child process per GPU through parallel/launch.py, BEFORE this process imports torch or
touches a GPU), relays rank 0's JSON line on stdout and exits non-zero if any rank fails.  Under
torchrun, WORLD_SIZE must equal --gpus (a mismatch is an error, never a silent 1-rank run).
At N > 1:
  * every rank is a SUPERVISOR that runs the benchmark in a child process (it never touches the GPU
    itself).  If any rank's child fails (exit, crash, timeout) all supervisors stop their children
    and start a second attempt with the 5-graph DP plan (``--dp-graph five``: no captured collectives);
    the JSON line then carries ``dp_fallback`` with the reason.  Only a fully successful attempt's
    JSON line is printed (rank 0's supervisor relays it), so stdout never holds two.
  * the DP plan is CHOSEN AT THE REAL WORLD SIZE: with ``--dp-plan auto`` both plans (ZeRO-1 and
    all-reduce) are built on the graph mode the capture pre-flight allows -- on the one-graph plan
    each with its QSC placements (``--dp-qsc auto``: beside the conv backward, forked after the gather, or --
    all-reduce plan -- the independent QSC chain with its own bucket) -- each timed over ``--select-steps`` steps
    after its warm-up (max over ranks), and the fastest is benchmarked; ``plan_select_ms`` records every candidate.
  * ``phases_ms``: per-phase times (max over ranks) on extra steps AFTER the timed region: HIP events
    between the 5-graph plan's replays, device clock stamps captured inside the one-graph plan's graph
    (FlagshipTrainer.phase_times); ``phases_src`` says which.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-stream batch (batch_size_DML)")
    ap.add_argument("--qubits", type=int, default=8)
    ap.add_argument("--pilot", type=int, default=128, choices=[128, 256], help="Pilot_num (P128 / P256 configs)")
    ap.add_argument("--layers", type=int, default=3, help="QNN layers")
    ap.add_argument("--data-len", type=int, default=20000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="estimator compute dtype (fp8: e4m3 FC forward GEMM, bf16 convs/backward)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-quantumnat", action="store_true")
    ap.add_argument("--gradient-pruning", action="store_true",
                    help="the QSC's on-chip gradient pruning (|g| > 0.1 mask fused into its AdamW, reference "
                         "apply_gradient_pruning E:205-228; FlagshipConfig.use_gradient_pruning): BASELINE config 5's "
                         "\"on-chip QNN\"")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = batch_size_DML per stream on EVERY rank (each rank its own data); strong = "
                         "the reference's DataParallel semantics (R:144-148): ONE global batch of batch_size_DML per "
                         "stream per step, cut into N contiguous parts (FlagshipConfig.scaling)")
    ap.add_argument("--split-graphs", action="store_true", help="the DP plan (5 graphs around the collectives) even at 1 GPU")
    ap.add_argument("--steps-per-graph", type=int, default=10,
                    help="training steps captured per graph replay at world 1 (each gathers its own batch)")
    ap.add_argument("--dp-plan", default="auto", choices=["auto", "zero", "allreduce"],
                    help="world > 1: ZeRO-1 FC optimizer (reduce-scatter / shard Adam / all-gather) or all-reduce; "
                         "auto = allreduce with the one-graph step, zero with the 5-graph step")
    ap.add_argument("--dp-graph", default="auto", choices=["auto", "one", "five"],
                    help="world > 1: the DP step as one HIP graph with the RCCL collectives captured, or 5 graphs "
                         "with the collectives launched between them; auto = one if every rank's capture "
                         "pre-flight (parallel/capture_probe.py) succeeds, else five")
    ap.add_argument("--dp-one-graph", action="store_true",
                    help="DP plan: capture the whole step, RCCL collectives included, in one HIP graph")
    ap.add_argument("--phase-steps", type=int, default=20,
                    help="N > 1: extra steps (after the timed region) timed per phase with HIP events; 0 = off")
    ap.add_argument("--dp-qsc", default="auto", choices=["auto", "g2", "fwd", "indep"],
                    help="N > 1, one-graph DP plan: the QSC branch beside the conv backward (g2), forked after the "
                         "gather (fwd), or an independent chain with its own bucket (indep, all-reduce plan); auto = "
                         "timed at the real world size with the plans (FlagshipConfig.dp_qsc)")
    ap.add_argument("--select-steps", type=int, default=30,
                    help="N > 1, --dp-plan auto: steps timed per candidate plan to choose the fastest (three "
                         "10-step replays; 0 = no timing: allreduce with the one-graph step, zero with the 5-graph step)")
    ap.add_argument("--lead-in", type=int, default=1,
                    help="steps replayed one per graph at the start of every run (FlagshipConfig.lead_in)")
    ap.add_argument("--ramp", type=int, default=4,
                    help="steps of the one replay between the lead-in and the k-step replays (FlagshipConfig.ramp: "
                         "keeps each graph's host submission behind the previous replay's GPU work; 0 = off)")
    ap.add_argument("--settle-steps", type=int, default=25,
                    help="untimed steps replayed right before the timed region, after the warm-up and the graph "
                         "capture (rounded up to whole graph replays): the first replays of a fresh graph run "
                         "slower (profiles/r3_01_window.txt); reported in the JSON line")
    ap.add_argument("--gemm-cfg", default=None,
                    help="FC GEMM tile configurations 'fwd,wgrad,dgrad' (knobs.KNOBS.gemm_cfg; default: the shipped ones)")
    ap.add_argument("--spread-windows", type=int, default=8,
                    help="extra event-timed windows after the timed region (step_spread in the JSON line); 0 = off")
    ap.add_argument("--stream-mode", default="indep", choices=["serial", "dagq", "indep"],
                    help="how the step's independent branches run (FlagshipTrainer): one chain, or the QSC branch "
                         "forked off the HDCE chain")
    ap.add_argument("--qsc-start", default="step", choices=["step", "conv"],
                    help="(stream mode indep) when each step's QSC chain starts: with the step, or after the HDCE conv "
                         "forward (FlagshipConfig.qsc_start)")
    ap.add_argument("--qsc-grid-bwd", type=int, default=0,
                    help="QSC backward workgroups (FlagshipConfig.qsc_grid_bwd; 0 = at most 256, balanced: 192 at 2304 samples)")
    ap.add_argument("--hdce-priority", action="store_true",
                    help="(stream mode indep) capture on a high-priority stream (FlagshipConfig.hdce_priority)")
    ap.add_argument("--fc-adam-next", type=int, default=0, metavar="WORKGROUPS",
                    help="(stream mode indep) > 0: the FC weight's Adam on a side stream overlapping the next step's "
                         "gather + conv forward, on at most this many workgroups (FlagshipConfig.fc_adam_next; 0 = off)")
    ap.add_argument("--fc-adam-side", type=int, default=0,
                    help="world 1: the FC weight's Adam on a side stream beside the conv backward, capped at this many "
                         "workgroups (FlagshipConfig.fc_adam_side; 0 = off)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="set a knobs.KNOBS switch for this run (repeatable; bools as 0/1), e.g. qsim_mfma_bwd=0")
    ap.add_argument("--qsim-mfma12", type=int, default=None, choices=[0, 1],
                    help="12 qubits: the MFMA simulator (knobs.KNOBS.qsim_mfma12) or qsim_big.hip's VALU kernels")
    ap.add_argument("--f8-producers", type=int, default=None, choices=[0, 1],
                    help="fp8 estimator: the e4m3 GEMMs with producer waves (knobs.KNOBS.f8_producers; default: shipped)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return self_launch(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", 1))
    if world_env != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    if world_env > 1 and os.environ.get("QDML_BENCH_WORKER") != "1":
        return supervise(sys.argv[1:], args)

    inj = os.environ.get("QDML_BENCH_FAIL_RANK")   # (fault injection for the supervisor tests)
    if inj is not None and os.environ.get("RANK") == inj and not os.environ.get("QDML_DP_FALLBACK"):
        print(f"[bench] rank {inj}: injected failure", file=sys.stderr, flush=True)
        return 7
    capture_ok = None
    one_graph = args.dp_one_graph or args.dp_graph == "one"
    forced = world_env == 1 and os.environ.get("QDML_FORCE_DIST") == "1"   # (a one-rank RCCL group: rehearsal)
    if args.dp_graph == "auto" and not args.dp_one_graph and (world_env > 1 or forced) and not args.no_graphs \
            and os.environ.get("QDML_DIST_BACKEND", "rccl") in ("rccl", "nccl"):
        # (before this process touches the GPU: the probe runs in a child of every rank)
        import torch
        n_dev = torch.cuda.device_count()   # (no GPU initialisation on this image)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.capture_probe import preflight
        capture_ok = preflight()
        one_graph = capture_ok
        if n_dev > 0 and torch._C._cuda_getDeviceCount() == 0:
            print(f"error: {n_dev} GPU(s) visible before the capture pre-flight, none after", file=sys.stderr)
            return 3
    import torch

    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import init_distributed, shutdown
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)

    if args.gemm_cfg or args.f8_producers is not None or args.qsim_mfma12 is not None or args.knob:
        from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
        for kv in args.knob:
            name, val = kv.split("=", 1)
            cur = getattr(KNOBS, name)   # (AttributeError for an unknown knob)
            setattr(KNOBS, name, bool(int(val)) if isinstance(cur, bool) else type(cur)(val))
        if args.gemm_cfg:
            KNOBS.gemm_cfg = args.gemm_cfg
        if args.f8_producers is not None:
            KNOBS.f8_producers = bool(args.f8_producers)
        if args.qsim_mfma12 is not None:
            KNOBS.qsim_mfma12 = bool(args.qsim_mfma12)
    ctx = init_distributed("auto")   # (rendezvous + failure-detector timeout: QDML_PG_TIMEOUT, default 600 s)
    if ctx.world != args.gpus:
        print(f"error: --gpus {args.gpus} but the process group has {ctx.world} rank(s)", file=sys.stderr)
        return 2
    sync = torch.cuda.synchronize if ctx.device.type == "cuda" else (lambda: None)

    def make(cand, og: bool, store=None) -> FlagshipTrainer:
        plan, qsc = cand
        cfg = FlagshipConfig(pilot_num=args.pilot, n_qubits=args.qubits, n_layers=args.layers, batch=args.batch,
                             data_len=args.data_len, dtype=args.dtype, hip_graphs=not args.no_graphs,
                             use_quantumnat=not args.no_quantumnat, use_gradient_pruning=args.gradient_pruning,
                             scaling=args.scaling, split_graphs=args.split_graphs or ctx.forced,
                             stream_mode=args.stream_mode, qsc_start=args.qsc_start,
                             steps_per_graph=args.steps_per_graph,
                             dp_plan=plan, dp_one_graph=og, dp_qsc=qsc, lead_in=args.lead_in,
                             ramp=args.ramp, fc_adam_side=args.fc_adam_side, fc_adam_next=args.fc_adam_next,
                             hdce_priority=args.hdce_priority, qsc_grid_bwd=args.qsc_grid_bwd)
        return FlagshipTrainer(cfg, ctx, store=store)

    def warm(tr: FlagshipTrainer, n: int) -> None:
        """Capture every graph set run(n) will replay and replay each once (a fresh graph's first replays run
        slower, profiles/r3_01_window.txt): untimed steps."""
        tr.prepare(n)
        for kk in sorted(set(tr._reps(n))):
            tr._replay(kk)

    def timed(tr: FlagshipTrainer, n: int, settle: int = 0):
        """(seconds of n timed steps, max over ranks; host enqueue seconds).  ``settle``: untimed steps
        replayed first, after any capture (every rank runs the same count: they hold collectives)."""
        tr.prepare(n)   # (graph capture, if the timed run needs a set the warm-up did not)
        if settle > 0:
            k = tr._k()
            ns = (settle + k - 1) // k * k
            warm(tr, ns)   # (the settle run's own graph sets captured and warm: its wall time is the GPU's rate)
            sync()
            t0 = time.perf_counter()
            tr.run(ns)
            sync()
            # the replay plan from this box's measured rates: GPU seconds per step (this settle run, 5 % margin) and
            # the host's submission cost (fitted over the replays so far) -- FlagshipTrainer._reps_calibrated
            tr.calibrate(0.95 * (time.perf_counter() - t0) / ns)
            warm(tr, n)
        sync()
        ctx.barrier()
        sync()
        t0 = time.perf_counter()
        tr.run(n)
        host = time.perf_counter() - t0   # host enqueue time (a launch-bound run shows it ~= wall)
        sync()
        ctx.barrier()
        sync()
        return ctx.max_scalar(time.perf_counter() - t0), host

    # the DP plan: chosen at THIS world size by timing every candidate (ZeRO-1 vs all-reduce) on the graph
    # mode the pre-flight allows; a user-fixed plan is a single candidate
    dp_run = ctx.world > 1 or ctx.forced or args.split_graphs
    if not dp_run:
        plans = ["allreduce"]   # (world 1: the plan field is unused)
    elif args.dp_plan != "auto":
        plans = [args.dp_plan]
    elif args.select_steps <= 0 or args.dtype == "fp8":   # (fp8: no ZeRO plan, see FlagshipTrainer)
        plans = ["allreduce" if one_graph or args.dtype == "fp8" else "zero"]
    else:
        plans = ["allreduce", "zero"]
    # the QSC branch's place in the DP step (one-graph plan only): timed with the plans unless fixed
    if not (dp_run and one_graph and not args.no_graphs):
        qscs = ["g2"]
    elif args.dp_qsc != "auto":
        qscs = [args.dp_qsc]
    else:
        qscs = ["g2", "fwd", "indep"] if args.select_steps > 0 else ["g2"]
    cands = [(p, q) for p in plans for q in qscs if not (q == "indep" and p != "allreduce")]
    if not cands:
        print("error: --dp-qsc indep runs on the all-reduce plan (--dp-plan allreduce)", file=sys.stderr)
        return 2
    select = {}
    tr, store = None, None
    for cand in cands:
        t = make(cand, one_graph, store)
        store = t.store
        if len(cands) > 1:
            t.run(args.warmup)
            el, _ = timed(t, args.select_steps)
            key = cand[0] if len(qscs) == 1 else f"{cand[0]}/{cand[1]}"
            select[key] = round(el / args.select_steps * 1e3, 4)
            if tr is None or el < best:
                if tr is not None:
                    tr.close()   # (its graphs released now, after a device sync: not by a later GC)
                tr, tr_cand, best = t, cand, el
            else:
                t.close()
        else:
            tr, tr_cand = t, cand
    cfg = tr.cfg
    t = None
    if len(cands) > 1 and ctx.device.type == "cuda":
        torch.cuda.empty_cache()

    tr.run(args.warmup)
    k = tr._k()
    settle = (max(0, args.settle_steps) + k - 1) // k * k
    elapsed, host = timed(tr, args.steps, settle)

    # spread: after the timed window, 8 more windows of `steps_per_graph` steps each timed with HIP events (no
    # host sync inside a window; the max over ranks per window) -- the run-to-run spread the single timed window
    # cannot show
    spread = None
    if ctx.device.type == "cuda" and args.spread_windows > 0:
        k = tr._k()
        warm(tr, k)   # (the windows' graph sets captured and warmed outside them)
        evs = []
        for _ in range(args.spread_windows):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            tr.run(k)
            b.record()
            evs.append((a, b))
        sync()
        per = [x.elapsed_time(y) / k for x, y in evs]
        per = ctx.max_vector(per)
        srt = sorted(per)
        spread = {"windows": len(per), "steps_per_window": k, "min_ms": round(srt[0], 4),
                  "median_ms": round(srt[len(srt) // 2], 4), "max_ms": round(srt[-1], 4)}
    hbm_peak = torch.cuda.max_memory_allocated(ctx.device) / 2 ** 30 if ctx.device.type == "cuda" else None

    hl = tr.hloss.tolist()
    ql = float(tr.qloss.item())
    n = ctx.world
    samples = tr.samples_per_step * n * args.steps
    value = samples / elapsed
    dp = len(tr.graphs) == 5 or (one_graph and (ctx.world > 1 or cfg.split_graphs))
    phases = None
    if args.phase_steps > 0 and dp:
        phases = tr.phase_times(args.phase_steps)
    if phases is not None:
        keys = sorted(phases)
        phases = dict(zip(keys, (round(v, 4) for v in ctx.max_vector([phases[k] for k in keys]))))
    if ctx.is_main:
        rec = {
            "metric": "NMSE(dB) vs SNR + samples/sec, P128 RIS estimator at 1/2/4/8 MI355X"
                      if args.pilot == 128 else f"samples/sec, P{args.pilot} RIS estimator",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": settle,
            "lead_in": args.lead_in,
            "ramp": args.ramp,
            "replays": tr._reps(args.steps),
            # (the calibrated plan's inputs: host submit ms = a + c * steps, GPU ms per step)
            "replay_rates_ms": {"submit_a": round(1e3 * tr._sub_est[0], 4), "submit_c": round(1e3 * tr._sub_est[1], 4),
                                "gpu": round(1e3 * tr._g_est, 4)} if getattr(tr, "_g_est", None) else None,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "host_ms_per_step": round(host / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": cfg.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (DeepMIMO-shaped geometric channels, HBM-resident), random-init weights",
            "config": {
                "model": f"P{args.pilot} RIS, {args.qubits}-qubit {'QuantumNAT ' if cfg.use_quantumnat else ''}QNN + CNN "
                     f"estimator (HDCE: 3x Conv_P{args.pilot} + FC_P{args.pilot})",
                "global_batch": tr.samples_per_step * n,
                "per_gpu_batch": tr.samples_per_step,
                "per_rank_stream_batch": tr.B,
                "streams": tr.S,
                "batch_size_DML": args.batch,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "hip_graphs": bool(tr.graphed.enabled),
                "graphs_per_step": len(tr.graphs),
                "stream_mode": tr.mode,
                "dp_plan": ("zero" if tr.zero else "allreduce") if dp else None,
                "dp_graph": ("one" if one_graph else "five") if dp else None,
                "dp_qsc": tr.cfg.dp_qsc if dp else None,
                "capture_preflight": capture_ok,
                "plan_select_ms": select or None,
                "dist_backend": ctx.backend,
                "steps_per_graph": tr._k(),
                "quantumnat": cfg.use_quantumnat,
                "gradient_pruning": cfg.use_gradient_pruning,
                # which kernels the timed step ran: the FC forward (hand_plain / hand / hand_f8 / library), the
                # FC gradients, the 8-qubit circuit forward on the matrix cores
                "fc_forward": getattr(tr.hstep, "fc_path", None),
                "fc_grad_gemms": sorted(tr.hstep.hand_gemm & {"wgrad", "dgrad"}) if tr.hstep.hip else None,
                "fc_gemm_cfg": list(tr.hstep.gemm_cfg) if tr.hstep.hip else None,
                "qsim_mfma_forward": bool(getattr(getattr(tr.cstep, "hip", None), "mfma", False)),
                "qsim_mfma12": bool(getattr(getattr(tr.cstep, "hip", None), "mfma12", False)),
                "qsim_mfma_bwd": bool(getattr(getattr(tr.cstep, "hip", None), "mfma_bwd", False)),
                "fc_adam_side": cfg.fc_adam_side if getattr(tr, "fc_adam_side", False) else 0,
                "fc_adam_next": cfg.fc_adam_next if getattr(tr, "fc_adam_next", False) else 0,
                "hdce_priority": bool(cfg.hdce_priority),
            },
            "final_losses": {"hdce_nmse": hl[0], "hdce_nmse_perf": hl[1], "qsc_nll": ql},
            "steps_trained": getattr(tr, "steps_done", None),   # (the losses' step count: the warm-ups vary with the plan)
            "step_spread": spread,
            # (torch's caching allocator: everything the run allocated on this GPU -- dataset, weights, optimizer
            # state, activations, graph pools -- out of 288 GB of HBM3E)
            "hbm_peak_gib": round(hbm_peak, 3) if hbm_peak is not None else None,
        }
        if dp:
            rec["phases_ms"] = phases
            rec["phases_src"] = None if phases is None else ("events" if len(tr.graphs) == 5 else "stamps")
        fb = os.environ.get("QDML_DP_FALLBACK")
        if ctx.world > 1:
            rec["dp_fallback"] = fb or None
        line = json.dumps(rec)
        dest = os.environ.get("QDML_BENCH_JSON")
        if dest:   # (supervised rank: the supervisor prints it once every rank has succeeded)
            with open(dest, "w") as f:
                f.write(line + "\n")
        else:
            print(line, flush=True)
    tr.close()
    shutdown()
    return 0


def supervise(argv, args) -> int:
    """Run this rank's benchmark in a child process (this process never touches the GPU) and agree with
    the other ranks' supervisors, through a TCPStore, on whether the attempt succeeded.  On any rank's
    failure every supervisor stops its child and all start the fallback attempt (the 5-graph DP plan,
    no captured collectives) on a fresh rendezvous port.  Children are started as new processes (never an
    exec).  Rank 0 prints the successful attempt's JSON line; returns the exit code."""
    import datetime
    import signal
    import subprocess
    import tempfile

    from torch.distributed import TCPStore   # (no GPU initialisation)

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    base = int(os.environ.get("MASTER_PORT", "29500"))
    store = TCPStore(host, base + 11, world, rank == 0, timeout=datetime.timedelta(seconds=3600))
    attempts = [(list(argv), None)]
    if args.dp_graph != "five" or args.dp_one_graph:
        fb = [a for a in argv if a != "--dp-one-graph"]
        attempts.append((fb + ["--dp-graph", "five"], "first attempt failed on rank {r} (exit {rc}); 5-graph DP plan"))
    limit = float(os.environ.get("QDML_BENCH_ATTEMPT_TIMEOUT", "900"))
    json_path = os.path.join(tempfile.gettempdir(), f"qdml_bench_{os.getpid()}.json")
    rc = 1
    for i, (av, why) in enumerate(attempts):
        env = dict(os.environ, QDML_BENCH_WORKER="1", MASTER_PORT=str(base + 20 + 10 * i), QDML_BENCH_JSON=json_path)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # (the worker's process group hosts its own store)
        if why:
            env["QDML_DP_FALLBACK"] = why.format(r=fail_rank, rc=fail_rc)
        if os.path.exists(json_path):
            os.remove(json_path)
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + av, env=env, start_new_session=True)
        key, t0, killed = f"qdml_bench_fail_{i}", time.time(), None
        while True:
            rc = p.poll()
            if rc is not None:
                break
            if killed is None and (store.check([key]) or time.time() - t0 > limit):
                if not store.check([key]):   # (this rank timed out: tell the others)
                    store.set(key, f"{rank} 124")
                os.killpg(p.pid, signal.SIGTERM)
                killed = time.time()
            elif killed is not None and time.time() - killed > 20:
                os.killpg(p.pid, signal.SIGKILL)
            time.sleep(0.2)
        if rc != 0 and killed is None:
            store.set(key, f"{rank} {rc}")
        store.set(f"qdml_bench_rc_{i}_{rank}", str(rc))
        rcs = [int(store.get(f"qdml_bench_rc_{i}_{r}")) for r in range(world)]   # (blocks until every rank is done)
        if all(c == 0 for c in rcs):
            if rank == 0:
                with open(json_path) as f:
                    sys.stdout.write(f.read())
                sys.stdout.flush()
            rc = 0
            break
        fail_rank, fail_rc = (store.get(key).decode().split() + ["?", "?"])[:2] if store.check([key]) else ("?", "?")
        print(f"[bench supervisor] rank {rank}: attempt {i} failed (exit codes {rcs})", file=sys.stderr, flush=True)
        rc = next(c for c in rcs if c != 0)
    if os.path.exists(json_path):
        os.remove(json_path)
    # (rank 0 hosts the store: the others must be done with it first)
    store.set(f"qdml_bench_exit_{rank}", "1")
    if rank == 0:
        store.wait([f"qdml_bench_exit_{r}" for r in range(world)])
    return rc


def self_launch(n: int) -> int:
    """Start ``n`` ranks of this same command (torchrun environment contract) and wait for them.
    Only the standard library is imported here: no torch, no GPU, before the children exist."""
    import importlib.util

    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "quantum_distributed_machine_learning_ris_channel_estimation_amd", "parallel", "launch.py")
    spec = importlib.util.spec_from_file_location("_qdml_launch", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rc = mod.launch([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], nproc=n,
                    extra_env={"QDML_SELF_LAUNCHED": "1"})
    if rc != 0:
        print(f"error: a rank of the {n}-rank bench failed (exit {rc})", file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
