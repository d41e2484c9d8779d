"""Command-line interface.

    python -m quantum_distributed_machine_learning_ris_channel_estimation_amd <command> [options]

Commands
  train-qsc | train-hdce | train-sc | train-all    Y2HRunner trainers (reference R:134, R:307)
  eval                                              model_val NMSE/accuracy sweep (Test.py)
  gen-data                                          write synthetic streams as reference .npy files
  bench                                             the flagship throughput benchmark (bench.py)
  launch --nproc N -- <command ...>                 one process per GPU (torchrun-compatible)

Config: ``--config file.{yaml,json}`` and repeated ``--set key=value`` (reference knob names,
see config.py); e.g. ``train-qsc --set n_qubits=8 --set n_epochs=20``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def _cfg(args, cls):
    from .config import load_config_file, parse_overrides
    cfg = cls()
    if args.config:
        cfg.update_from_dict(load_config_file(args.config))
    cfg.update_from_dict(parse_overrides(args.set))
    return cfg


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="qdml", description="MI355X-native RIS channel estimation framework")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("train-qsc", "train-hdce", "train-sc", "train-all", "eval", "gen-data"):
        p = sub.add_parser(name)
        p.add_argument("--config", default=None)
        p.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    b = sub.add_parser("bench")
    b.add_argument("rest", nargs=argparse.REMAINDER)
    la = sub.add_parser("launch")
    la.add_argument("--nproc", type=int, required=True)
    la.add_argument("rest", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)

    if args.cmd == "launch":
        from .parallel.launch import launch
        rest = args.rest[1:] if args.rest and args.rest[0] == "--" else args.rest
        return launch([sys.executable, "-m", __package__] + rest, args.nproc)
    if args.cmd == "bench":
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.argv = [os.path.join(root, "bench.py")] + args.rest
        sys.path.insert(0, root)
        import bench
        return bench.main()
    if args.cmd == "eval":
        from .config import EvalConfig
        from .train.evaluate import model_val
        mv = model_val(_cfg(args, EvalConfig))
        rc = mv.test_for_CE_P128_for_all_scenarios()
        print(json.dumps(mv.results))
        return rc
    from .config import RunnerConfig
    cfg = _cfg(args, RunnerConfig)
    if args.cmd == "gen-data":
        from .data.datasets import generate_stream, save_stream_npy
        for s in range(cfg.n_scenarios):
            for u in range(cfg.n_users):
                st = generate_stream(cfg.data_len, s, u, cfg.SNRdb, cfg.Pilot_num, "train", cfg.seed)
                save_stream_npy(cfg.data_dir, st, s, u, cfg.Pilot_num, cfg.SNRdb, cfg.data_len)
                print(f"wrote scenario {s} user {u} -> {cfg.data_dir}")
        return 0
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and cfg.dp_graphs == "auto" and cfg.hip_graphs \
            and cfg.device != "cpu" and os.environ.get("QDML_DIST_BACKEND", "rccl") in ("rccl", "nccl"):
        # (before anything touches the GPU: every rank's child captures the collective pattern, rank 0 decides)
        from .parallel.capture_probe import preflight
        os.environ["QDML_DP_GRAPHS"] = "1" if preflight() else "0"
    from .train.runner import Y2HRunner
    r = Y2HRunner(cfg)
    {"train-qsc": r.train_QSC_P128, "train-hdce": r.train_Conv_Linear_of_HDCE, "train-sc": r.train_SC_P128,
     "train-all": r.train_all}[args.cmd]()
    from .parallel.dp import shutdown
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
