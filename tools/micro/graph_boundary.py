"""What a hipGraph boundary costs on the GPU: the same sleep kernels replayed as many small graphs
back to back vs as one graph, for single-stream graphs and for fork/join graphs (a second stream
beside the first, joined at the end -- the DP stage graphs' shape).  Per boundary = (time of N
replays - time of one graph holding the same N bodies) / N.

  python tools/micro/graph_boundary.py"""
import torch

dev = torch.device("cuda", 0)
CYC = 20 * 2100                   # ~20 us per sleep kernel


def body(fork, s, side):
    if fork:
        e = torch.cuda.Event()
        e.record(s)
        side.wait_event(e)
        with torch.cuda.stream(side):
            for _ in range(5):
                torch.cuda._sleep(CYC)
    for _ in range(10):
        torch.cuda._sleep(CYC)
    if fork:
        e2 = torch.cuda.Event()
        e2.record(side)
        s.wait_event(e2)


def capture(fork, reps):
    s, side = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            body(fork, s, side)
    torch.cuda.synchronize()
    return g


def timed(fn, n=3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(n):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        t = a.elapsed_time(b) * 1e3
        best = t if best is None else min(best, t)
    return best


N = 20
for fork in (False, True):
    small, big = capture(fork, 1), capture(fork, N)

    def many():
        for _ in range(N):
            small.replay()
    t_many, t_big = timed(many), timed(big.replay)
    print(f"{'fork/join' if fork else 'single-stream'} graphs: {N} replays {t_many:8.1f} us, one graph of {N} bodies "
          f"{t_big:8.1f} us -> {(t_many - t_big) / N:6.1f} us per graph boundary", flush=True)
