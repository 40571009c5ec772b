"""Reference-compatible command line (ref main.py).

    python main.py n_procs n_rows n_cols input_dir is_real dataset is_coded n_stragglers \\
                   partitions coded_ver num_collect add_delay update_rule  [--extension flags]

Single GPU / CPU: run directly.  Several MI355X of one node: one process per GPU,
    python main.py <13 args> --gpus N      (relaunches itself under torch.distributed.run, like
                                            the reference's single mpirun command, ref
                                            run_approx_coding.sh:47-49)
    torchrun --nproc-per-node N --master-addr 127.0.0.1 main.py <13 args> [flags]
The n_procs argument keeps the reference meaning (1 master + n_procs-1 logical workers);
the logical workers are spread over however many processes were launched.
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional

from .config import RunConfig

USAGE = ("Usage: python main.py n_procs n_rows n_cols input_dir is_real dataset is_coded n_stragglers "
         "partial_straggler_partitions coded_ver num_itrs")  # verbatim (stale) reference usage line, ref main.py:21


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="main.py", add_help=True)
    p.add_argument("positional", nargs="*")
    g = p.add_argument_group("extensions (defaults reproduce the reference)")
    g.add_argument("--precision", default="fp64", choices=["fp64", "fp32", "bf16"])
    g.add_argument("--loss", default="auto", choices=["auto", "logistic", "least_squares"])
    g.add_argument("--num-itrs", type=int, default=100)
    g.add_argument("--lr", type=float, default=10.0)
    g.add_argument("--lr-schedule", default="const", choices=["const", "invscaling", "exponential"],
                   help="the reference's commented alternatives (ref main.py:40-46)")
    g.add_argument("--lr-t0", type=float, default=90.0)
    g.add_argument("--lr-decay", type=float, default=0.98)
    g.add_argument("--alpha", type=float, default=None)
    g.add_argument("--seed", type=int, default=None)
    g.add_argument("--data", default="files", choices=["files", "synthetic"])
    g.add_argument("--data-seed", type=int, default=0)
    g.add_argument("--allow-uneven-groups", action="store_true")
    g.add_argument("--drain", default=None, choices=["all", "carry", "lazy"],
                   help="straggler tail after the stop rule: all = the master waits for every message before the "
                        "next beta (ref Waitall, FRC/AGC default); carry = no wait, late workers deliver every round "
                        "in order (the reference's other schemes); lazy = no wait, and a worker still busy when the "
                        "next beta is out skips the stale round (default: the scheme's reference behaviour)")
    g.add_argument("--delay-mode", default="exp", choices=["exp", "fixed", "none", "worker"],
                   help="injected delay distribution; worker = exp slept on the worker rank (--delay-on worker)")
    g.add_argument("--delay-on", default="collector", choices=["collector", "worker"],
                   help="virtual arrival time on the master (collector) or a physically late worker rank")
    g.add_argument("--slow-ranks", nargs="*", default=[], metavar="RANK:FACTOR",
                   help="physically slow GPU ranks: each runs its gradient FACTOR times per round")
    g.add_argument("--fixed-stragglers", type=int, nargs="*", default=[])
    g.add_argument("--fixed-sleep", type=float, default=0.5)
    g.add_argument("--kill-workers", type=int, nargs="*", default=[])
    g.add_argument("--force-delay", action="store_true")
    g.add_argument("--round-timeout", type=float, default=600.0)
    g.add_argument("--fix-quirks", action="store_true")
    g.add_argument("--save-linear", action="store_true")
    g.add_argument("--full-precision-outputs", action="store_true")
    g.add_argument("--no-eval", action="store_true")
    g.add_argument("--quiet", action="store_true")
    g.add_argument("--checkpoint-every", type=int, default=0)
    g.add_argument("--checkpoint-path", default=None)
    g.add_argument("--resume", default=None, help="continue from a checkpoint written by --checkpoint-every")
    g.add_argument("--trace", action="store_true")
    g.add_argument("--verify-beta", action="store_true", help="race detector: checksum beta on every worker")
    g.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    g.add_argument("--gpus", type=int, default=0,
                   help="N > 1: start N ranks (one per GPU) under torch.distributed.run from this command")
    g.add_argument("--transport", default="auto", choices=["auto", "ipc", "rccl", "loopback", "gloo"])
    g.add_argument("--device-loop", default="auto", choices=["auto", "graph", "stream", "off"],
                   help="single-process runs without injected delay: rounds captured in hipGraphs (auto/graph), "
                        "enqueued back to back (stream) or host-driven (off)")
    g.add_argument("--share-partitions", action="store_true",
                   help="stream each distinct partition once per GPU and encode the local messages on the device")
    g.add_argument("--tie-break", default="permute", choices=["permute", "worker"],
                   help="order of simultaneous arrivals: seeded per-round worker permutation (default) or worker id")
    g.add_argument("--tie-seed", type=int, default=0)
    g.add_argument("--shard", default="auto", choices=["auto", "message", "partition"],
                   help="placement unit on several ranks: whole messages, the reference topology (auto) or "
                        "partition shards (bandwidth, no physical straggler tolerance)")
    g.add_argument("--no-integrity", action="store_true",
                   help="IPC messages without (round, rank, checksum) tags (A/B runs only)")
    g.add_argument("--dedicated-master", action="store_true",
                   help="rank 0 runs the master only, the workers go on ranks 1..N-1 (the reference topology)")
    g.add_argument("--device-records", action="store_true",
                   help="keep per-round device stamps of every rank (put landed, spins, gates, beta puts)")
    return p


def parse_slow_ranks(items) -> dict:
    """['3:4', '5:2'] -> {3: 4, 5: 2}."""
    out = {}
    for it in items or []:
        r, _, f = str(it).partition(":")
        out[int(r)] = int(f or 2)
    return out


def parse(argv: List[str]):
    a = build_parser().parse_args(argv)
    if len(a.positional) != 13:
        return None, a
    (n_procs, n_rows, n_cols, input_dir, is_real, dataset, is_coded, n_stragglers, partitions, coded_ver,
     num_collect, add_delay, update_rule) = a.positional
    cfg = RunConfig(int(n_procs), int(n_rows), int(n_cols), input_dir, int(is_real), dataset, int(is_coded),
                    int(n_stragglers), int(partitions), int(coded_ver), int(num_collect), int(add_delay),
                    update_rule, num_itrs=a.num_itrs, alpha=a.alpha, lr=a.lr,
                    lr_kind=a.lr_schedule, lr_t0=a.lr_t0, lr_decay=a.lr_decay, precision=a.precision, loss=a.loss,
                    seed=a.seed, data=a.data, data_seed=a.data_seed, allow_uneven_groups=a.allow_uneven_groups,
                    drain=a.drain, delay_mode=a.delay_mode, fixed_stragglers=a.fixed_stragglers,
                    fixed_sleep=a.fixed_sleep, kill_workers=a.kill_workers, force_delay=a.force_delay,
                    round_timeout=a.round_timeout, fix_quirks=a.fix_quirks, save_linear=a.save_linear,
                    full_precision_outputs=a.full_precision_outputs, evaluate=not a.no_eval, verbose=not a.quiet,
                    checkpoint_every=a.checkpoint_every, checkpoint_path=a.checkpoint_path, resume=a.resume, trace=a.trace, verify_beta=a.verify_beta,
                    transport=a.transport, share_partitions=a.share_partitions, device_loop=a.device_loop,
                    tie_break=a.tie_break, tie_seed=a.tie_seed, shard=a.shard,
                    integrity=not a.no_integrity, delay_on=a.delay_on, slow_ranks=parse_slow_ranks(a.slow_ranks),
                    dedicated_master=a.dedicated_master, device_records=a.device_records)
    return cfg, a


def relaunch(n: int, argv: List[str]) -> int:
    """Start n ranks of main.py as a child torch.distributed.run (before anything touches the GPU)."""
    import os
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    main_py = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "main.py")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if int(env.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:  # erasurehead_amd/__init__.py: per-peer p2p streams
        env["GPU_MAX_HW_QUEUES"] = "16"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", main_py, *argv]
    return subprocess.call(cmd, env=env)


def main(argv: Optional[List[str]] = None) -> int:
    import os

    argv = sys.argv[1:] if argv is None else argv
    cfg, a = parse(argv)
    if cfg is None:
        print(USAGE)
        return 0
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(a.gpus, argv)
    from .codes.schemes import SchemeError
    from .engine import Trainer, evaluate
    from .parallel.dist import init_distributed
    from .utils import tracing

    tracing.enable(cfg.trace)
    env = init_distributed(a.device)
    try:
        try:
            trainer = Trainer(cfg, env)
        except SchemeError as e:  # the reference prints and exits 0 (ref src/replication.py:24-26)
            if env.is_master:
                print(str(e))
            return 0
        res = trainer.run()
        if env.is_master and cfg.evaluate:
            evaluate(trainer, res)
        env.barrier()
        trainer.close()
    finally:
        env.shutdown()
    return 0
