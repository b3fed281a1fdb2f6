"""torchrun-compatible single-node launcher.

    python -m pytorch_distributed_tutorials_amd.launch --nproc_per_node=8 [trainer flags]
    python -m pytorch_distributed_tutorials_amd.launch --nproc_per_node=2 script.py [args]
    python -m pytorch_distributed_tutorials_amd.launch --nproc_per_node=2 -m pkg.module [args]

The reference expects ``python -m torch.distributed.launch --nproc_per_node=N
main.py`` (``resnet/main.py:52``).  This launcher exports the same env contract
as torch's elastic agent (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
GROUP_RANK, MASTER_ADDR, MASTER_PORT; torch/distributed/elastic/agent/server/
local_elastic_agent.py:306-319) and, like the legacy launcher, can also pass
``--local-rank=N`` (``--use-local-rank-arg``).  One process per GPU; if any
rank fails the others are terminated and the launcher exits non-zero (fail
fast instead of hanging in a collective).  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is
kept in the child environment (dmabuf IPC, required by RCCL on this driver).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def parse(argv):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=1)
    p.add_argument("--master_addr", "--master-addr", default="127.0.0.1")
    p.add_argument("--master_port", "--master-port", type=int, default=29500)
    p.add_argument("-m", "--module", action="store_true",
                   help="treat the first positional argument as a module name (python -m)")
    p.add_argument("--no-python", action="store_true", help="run the first positional as an executable")
    p.add_argument("--use-local-rank-arg", action="store_true",
                   help="also pass --local-rank=N (torch.distributed.launch style)")
    argv = list(sys.argv[1:] if argv is None else argv)
    # launcher options come first; everything from the first unknown token on belongs to
    # the per-rank program (like torchrun: options, then script/module, then its args)
    valued = {"--nproc_per_node", "--nproc-per-node", "--master_addr", "--master-addr",
              "--master_port", "--master-port"}
    flags = {"-m", "--module", "--no-python", "--use-local-rank-arg", "-h", "--help"}
    i = 0
    while i < len(argv):
        tok = argv[i]
        name = tok.split("=", 1)[0]
        if name in valued:
            i += 1 if "=" in tok else 2
        elif tok in flags:
            i += 1
        else:
            break
    a = p.parse_args(argv[:i])
    a.rest = argv[i:]
    return a


DEFAULT_MODULE = "pytorch_distributed_tutorials_amd.train"


def _command(a):
    rest = list(a.rest)
    if rest and rest[0] == "--":
        rest = rest[1:]
    if a.no_python:
        return rest
    if a.module:
        return [sys.executable, "-m", rest[0]] + rest[1:]
    if rest and rest[0].endswith(".py"):
        return [sys.executable, "-u", rest[0]] + rest[1:]
    return [sys.executable, "-m", DEFAULT_MODULE] + rest   # trainer flags only


def main(argv=None) -> int:
    a = parse(argv)
    n = a.nproc_per_node
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0",
                    "MASTER_ADDR": a.master_addr, "MASTER_PORT": str(a.master_port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env.setdefault("OMP_NUM_THREADS", "1")
        cmd = _command(a)
        if a.use_local_rank_arg:
            cmd.append(f"--local-rank={r}")
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        alive = set(range(n))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in alive:
                        procs[q].send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for pr in procs:
            pr.send_signal(signal.SIGTERM)
        rc = 130
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
