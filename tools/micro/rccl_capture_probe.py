"""RCCL collectives captured into HIP graphs (world-1 group): capture, replay, destroy, capture
again -- which sequences does the runtime accept?

  python tools/micro/rccl_capture_probe.py <case>   (case: keep | drop | fork | gather | mix | mixs)
  mix / mixs: an eager all-reduce (on the default stream / on a side stream) before each capture"""
import gc
import os
import socket
import sys

import torch
import torch.distributed as dist

dev = torch.device("cuda", 0)
s_ = socket.socket()
s_.bind(("127.0.0.1", 0))
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s_.getsockname()[1]))
s_.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
x = torch.ones(1 << 20, device=dev)
dist.all_reduce(x)
torch.cuda.synchronize()
case = sys.argv[1]
alive = []


def capture(fork):
    s, comm = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        x.add_(1.0)
        if fork:
            e = torch.cuda.Event()
            e.record(s)
            comm.wait_event(e)
            with torch.cuda.stream(comm):
                w = dist.all_reduce(x, async_op=True)
            w.wait()
        else:
            dist.all_reduce(x)
        if case == "gather":
            y = torch.empty(1 << 20, device=dev)
            dist.all_gather_into_tensor(y, x)
        x.add_(1.0)
    torch.cuda.synchronize()
    return g


side = torch.cuda.Stream(dev)
for i in range(3):
    if case in ("mix", "mixs"):
        with torch.cuda.stream(side if case == "mixs" else torch.cuda.current_stream(dev)):
            dist.all_reduce(torch.zeros(1, device=dev))
        torch.cuda.synchronize()
    g = capture(case in ("fork", "gather", "mix", "mixs"))
    x.fill_(1.0)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    print(f"{case} capture {i}: x = {float(x[0])} (expect 5)", flush=True)
    if case == "keep":
        alive.append(g)
    else:
        del g
        gc.collect()
dist.destroy_process_group()
print(f"{case}: done", flush=True)
