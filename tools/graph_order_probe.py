"""How does a replayed hipGraph start two independent branches captured one after the other?
Branch R (captured first, on its own stream) and branch M (on the capture stream) share no
data.  Prints, from rocprofv3-free host timing, the step time of: R alone, M alone, R then M
captured whole, M then R, and the two interleaved node by node."""
import time

import torch

dev = torch.device("cuda", 0)
n = 1536
a = [torch.randn(n, n, device=dev, dtype=torch.bfloat16) for _ in range(4)]
b = [torch.randn(n, n, device=dev, dtype=torch.bfloat16) for _ in range(4)]
oa = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
ob = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
NR, NM = 60, 60
rs = torch.cuda.Stream()


def r_node(i):
    torch.mm(a[i % 4], a[(i + 1) % 4], out=oa)


def m_node(i):
    torch.mm(b[i % 4], b[(i + 1) % 4], out=ob)


def capture(order):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            r_node(i), m_node(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        main = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(main)
        rs.wait_event(fork)
        if order == "R":
            with torch.cuda.stream(rs):
                for i in range(NR):
                    r_node(i)
        elif order == "M":
            for i in range(NM):
                m_node(i)
        elif order == "RM":
            with torch.cuda.stream(rs):
                for i in range(NR):
                    r_node(i)
            for i in range(NM):
                m_node(i)
        elif order == "MR":
            for i in range(NM):
                m_node(i)
            with torch.cuda.stream(rs):
                for i in range(NR):
                    r_node(i)
        elif order == "interleave":
            for i in range(max(NR, NM)):
                if i < NR:
                    with torch.cuda.stream(rs):
                        r_node(i)
                if i < NM:
                    m_node(i)
        join = torch.cuda.Event()
        join.record(rs)
        main.wait_event(join)
    return g


for order in ("R", "M", "RM", "MR", "interleave", "RM", "interleave"):
    g = capture(order)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    print(f"{order:10s} {(time.perf_counter() - t0) / 20 * 1e3:8.3f} ms", flush=True)
