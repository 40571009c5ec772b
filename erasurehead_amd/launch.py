"""Multi-node launcher: a hosts file -> one ``torchrun`` per MI355X node (ref tools/*).

The reference brings up an EC2 cluster (tools/pytorch_ec2.py), writes ``hosts`` files
(``<ip>\\t<alias>`` per line, ref tools/hosts:1-30), copies the repo with scp/pdsh
(ref tools/remote_script.sh, local_script.sh) and starts one MPI rank per host with
``mpirun -n N_PROCS --hostfile hosts`` (ref run_approx_coding.sh:47-49).

Here a node is an 8-GPU MI355X box and a rank is a GPU.  This launcher reads the same hosts
file format (first line = the master node), and starts, over ssh, one
``python -m torch.distributed.run --nnodes H --node-rank j --nproc-per-node G`` per node with
a static rendezvous on the first host.  Logical workers (``n_procs - 1``) are placed on the
H * G ranks by the engine; inside a node messages move over the IPC mailbox / xGMI, across
nodes over RCCL (``--transport auto`` picks RCCL as soon as the job spans nodes).  The
repository must already be present at the same path on every node (shared filesystem or a
copy), as in the reference.

    python -m erasurehead_amd.launch --hosts hosts --gpus-per-node 8 [--dry-run] \\
           [--script main.py] -- <13 positional args and flags>
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
from typing import List, Sequence, Tuple


def read_hosts(path: str) -> List[Tuple[str, str]]:
    """[(address, alias)] from a reference-style hosts file: ``addr<ws>alias`` or ``addr`` per line."""
    out = []
    with open(path) as f:
        for ln in f:
            ln = ln.split("#", 1)[0].strip()
            if not ln:
                continue
            parts = ln.split()
            out.append((parts[0], parts[1] if len(parts) > 1 else parts[0]))
    if not out:
        raise ValueError(f"{path}: no hosts")
    return out


def node_commands(hosts: Sequence[Tuple[str, str]], gpus_per_node: int, script: str, args: Sequence[str],
                  port: int = 29500, workdir: str = ".", python: str = "python") -> List[Tuple[str, str]]:
    """(ssh target, shell command) for every node; node 0 hosts the rendezvous and rank 0 (the master)."""
    if gpus_per_node < 1:
        raise ValueError("gpus_per_node must be >= 1")
    master = hosts[0][0]
    n = len(hosts)
    cmds = []
    for j, (addr, _alias) in enumerate(hosts):
        run = [python, "-m", "torch.distributed.run", f"--nnodes={n}", f"--node-rank={j}",
               f"--nproc-per-node={gpus_per_node}", f"--master-addr={master}", f"--master-port={port}",
               script, *args]
        env = "HSA_ENABLE_IPC_MODE_LEGACY=0"
        cmds.append((addr, f"cd {shlex.quote(workdir)} && {env} " + " ".join(shlex.quote(a) for a in run)))
    return cmds


def main(argv: Sequence[str] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    rest: List[str] = []
    if "--" in argv:
        k = argv.index("--")
        argv, rest = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--hosts", required=True, help="hosts file (first line = master node)")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--script", default="main.py")
    ap.add_argument("--port", type=int, default=29500)
    ap.add_argument("--workdir", default=os.getcwd())
    ap.add_argument("--python", default="python")
    ap.add_argument("--ssh", default="ssh -o BatchMode=yes")
    ap.add_argument("--dry-run", action="store_true", help="print the per-node commands only")
    a = ap.parse_args(argv)
    hosts = read_hosts(a.hosts)
    cmds = node_commands(hosts, a.gpus_per_node, a.script, rest, a.port, a.workdir, a.python)
    if a.dry_run:
        for addr, c in cmds:
            print(f"{addr}: {c}")
        return 0
    procs = [subprocess.Popen(shlex.split(a.ssh) + [addr, c]) for addr, c in cmds]
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
