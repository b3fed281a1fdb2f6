"""Worker for tests/test_comm_setup_cpu.py: the native-communicator bring-up protocol on gloo/CPU.

Runs ``parallel.comm.native_comm`` -- agreement through the real TCPStore, then the communicator
constructor -- with the RCCL class replaced by a recorder (there is no GPU here), so the exact
decision logic the GPU runs take is exercised across real processes.  Fault injection through
``PDT_FAULT_NATIVE`` (a rank that cannot build / never arrives).  Prints one RESULT line.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_tutorials_amd.parallel import comm as pcomm  # noqa: E402


class FakeRcclComm:
    inits = []

    def __init__(self, uid, rank, world, device, **kw):
        FakeRcclComm.inits.append(dict(rank=rank, world=world, uid=hashlib.sha1(uid).hexdigest(), **kw))

    @staticmethod
    def unique_id():
        return os.urandom(128)


class FakeC:
    RcclComm = FakeRcclComm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timeout", type=float, default=5.0)
    a = ap.parse_args()
    env = pcomm.init_distributed("gloo")
    import pytorch_distributed_tutorials_amd.ops._ext as ext
    ext.native = lambda: FakeC  # the communicator class only; agreement + decisions are real
    pcomm._can_build = lambda device: (True, "")
    opts = pcomm.CommOptions(init_timeout=a.timeout, op_timeout=a.timeout)
    t0 = time.monotonic()
    res = {"rank": env.rank}
    try:
        pcomm.native_comm(torch.device("cpu"), options=opts)
        res["outcome"] = "built"
        res["init"] = FakeRcclComm.inits[-1]
    except pcomm.CommSetupError as e:
        res["outcome"] = "refused"
        res["error"] = str(e)
    except pcomm.CommSetupTimeout as e:
        res["outcome"] = "timeout"
        res["error"] = str(e)
    res["seconds"] = time.monotonic() - t0
    print("RESULT " + json.dumps(res), flush=True)
    if res["outcome"] == "timeout":
        sys.stderr.write(res["error"] + "\n")
        return 3
    if res["outcome"] == "built":
        # the uid must be the same on every rank
        h = torch.tensor(list(bytes.fromhex(res["init"]["uid"])), dtype=torch.int64)
        hs = [torch.zeros_like(h) for _ in range(env.world_size)]
        dist.all_gather(hs, h)
        assert all(torch.equal(x, hs[0]) for x in hs), "ranks initialised with different unique ids"
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
