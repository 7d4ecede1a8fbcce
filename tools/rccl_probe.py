"""RCCL on this pool's one-GPU boxes.  Default: two processes, backend "nccl", both on cuda:0, one dist.gather
of device tensors into rank 0 and one all_reduce — RCCL refuses that ("Duplicate GPU detected",
profiles/r06/rccl_two_ranks_one_gpu_r6h.log).  --single: one rank (world size 1) through the same calls and
through dist.gather_records' code path with RCCL initialised on the MI355X.  Prints one JSON line per rank.
usage: python tools/rccl_probe.py [--single]   (spawns its ranks itself; 127.0.0.1 rendezvous)"""
import json
import os
import socket
import sys
import time


def rank_main(rank: int, world: int, port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"rank": rank}
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.full((4, 1024), rank + 1, dtype=torch.uint8, device=dev)
        parts = [torch.empty_like(x) for _ in range(world)] if rank == 0 else None
        t0 = time.perf_counter()
        dist.gather(x, gather_list=parts, dst=0)
        y = torch.tensor([float(rank + 1)], device=dev)
        dist.all_reduce(y)
        torch.cuda.synchronize(dev)
        out["ms"] = round(1e3 * (time.perf_counter() - t0), 3)
        out["all_reduce"] = float(y.item())
        if rank == 0:
            out["gather_ok"] = all(bool((p == r + 1).all()) for r, p in enumerate(parts))
        out["backend"] = dist.get_backend()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report whatever RCCL says
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] != "--single":
        rank_main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
    else:
        world = 1 if "--single" in sys.argv else 2
        import subprocess
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        ps = [subprocess.Popen([sys.executable, __file__, str(r), str(world), str(port)]) for r in range(world)]
        rc = [p.wait(timeout=150) for p in ps]
        sys.exit(max(rc))
