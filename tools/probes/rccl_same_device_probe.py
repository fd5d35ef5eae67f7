"""Can two ranks share the one GPU of a gpurun box over RCCL ("nccl")?  If so,
the RCCL branches of shard.py / bench.py (device-tensor all_gather,
all_reduce) can be rehearsed before the driver's 8-GPU job.

  python tools/probes/rccl_same_device_probe.py   -> one JSON line
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        x = torch.full((4,), float(rank + 1), device=dev)
        out = torch.empty(4 * world, device=dev)
        dist.all_gather_into_tensor(out, x)
        r = torch.tensor([float(rank)], device=dev)
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize(dev)
        q.put({"rank": rank, "ok": True, "gather": out.cpu().tolist(), "max": r.item()})
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- the probe reports whatever RCCL says
        q.put({"rank": rank, "ok": False, "error": f"{type(e).__name__}: {e}"[:400]})


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    for _ in procs:
        try:
            res.append(q.get(timeout=90))
        except Exception:  # noqa: BLE001
            res.append({"ok": False, "error": "no answer in 90 s"})
    for p in procs:
        p.join(10)
        if p.is_alive():
            p.kill()
    print(json.dumps({"probe": "rccl_two_ranks_one_gpu", "results": res}))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
