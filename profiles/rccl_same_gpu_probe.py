import os, sys, torch, torch.distributed as dist, torch.multiprocessing as mp
def worker(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    t = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(rank, "all_reduce ok", float(t[0]), flush=True)
    dist.destroy_process_group()
if __name__ == "__main__":
    mp.spawn(worker, args=(2,), nprocs=2)
