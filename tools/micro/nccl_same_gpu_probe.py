"""Can two RCCL ranks share the one GPU of a test box?  (The nccl branches of parallel/shuffle.py
need distinct devices per rank; this probe records what RCCL does with two ranks on device 0.)

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/micro/nccl_same_gpu_probe.py
"""
import datetime
import os

import torch
import torch.distributed as dist


def main():
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=r, world_size=w, timeout=datetime.timedelta(seconds=60),
                            device_id=torch.device("cuda", 0))
    x = torch.full((4,), r, dtype=torch.int32, device="cuda")
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    print(f"rank {r}: all_to_all_single ok {y.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
