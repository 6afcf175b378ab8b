"""Can two RCCL ranks share the one GPU of a gpurun box?  (If so, the multi-GPU step's RCCL
transport -- summary all-gather and the point-to-point flow gather -- can run on real hardware at
world size 2.)  Two spawned ranks on cuda:0, nccl backend, one all_gather and one isend/irecv.
Prints one JSON line from rank 0."""
import json
import os
import sys

import torch.multiprocessing as mp


def rank(r, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      LOCAL_RANK="0")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=r, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((4,), r, dtype=torch.int64, device="cuda")
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
        y = torch.arange(8, dtype=torch.int64, device="cuda") + 100 * r
        if r == 1:
            dist.send(y, 0)
        elif r == 0:
            z = torch.empty_like(y)
            dist.recv(z, 1)
            assert z.tolist() == list(range(100, 108))
        torch.cuda.synchronize()
        q.put((r, "ok", [int(t[0]) for t in out]))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang
        q.put((r, "error", f"{type(e).__name__}: {e}"[:400]))


def main():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    print(json.dumps({"rccl_two_ranks_one_gpu": sorted(res)}), flush=True)
    return 0 if all(x[1] == "ok" for x in res) else 1


if __name__ == "__main__":
    sys.exit(main())
