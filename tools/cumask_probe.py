"""Can the next batch's frozen ResNet run beside the step on a SUBSET of the CUs?

The pipelined step's trace (tools/gpu/r02c_diag.sh) shows the ResNet's large grids
taking the whole chip at the start of every replay: the chain starts ~1.4 ms late.
Here the ResNet runs on a HIP stream created with a CU mask
(hipExtStreamCreateWithCUMask), the step's chain on an ordinary stream:

  single      the engine's one captured pipelined graph (the bench path)
  res@K       the ResNet alone on K CUs (graph replay / eager launches)
  two@K       chain graph + ResNet on K CUs concurrently, GPU time per step

  python tools/cumask_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
L = pkg.lib
B = 64
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000, pipeline=True)
pool = [pkg.synthetic.make_batch(B, 32, 224, seed=s) for s in range(2)]
pool = [{k: (torch.as_tensor(v).cuda() if v is not None else None) for k, v in b.items()} for b in pool]
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
eng.prime(pool[0]["image_tensors"])
eng.load_batch(pool[0], next_images=pool[1]["image_tensors"])
eng.capture()
single = eng.graph
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
MAIN, RES = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with pkg.engine.no_gc_capture():
    with torch.cuda.graph(MAIN, stream=s):
        eng._run_step_streams()
    with torch.cuda.graph(RES, stream=s):
        eng._run(eng.res_calls)
torch.cuda.synchronize()

hip = ctypes.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", ncu, flush=True)


def masked_stream(bits):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


def timed(fn, steps=20, warm=3):
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(steps + warm):
        if i == warm:
            torch.cuda.synchronize()
            e0.record(cur)
        fn(i)
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def join(cur, streams):
    for st in streams:
        j = torch.cuda.Event()
        j.record(st)
        cur.wait_event(j)


def res_only(rs, eager):
    def f(i):
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        rs.wait_event(ev)
        if eager:
            h = L.stream_handle(rs)
            for c in eng.res_calls:
                c(h)
        else:
            with torch.cuda.stream(rs):
                RES.replay()
        join(cur, [rs])
    return f


def two(rs, ms, eager):
    def f(i):
        cur = torch.cuda.current_stream()
        eng.F4.copy_(eng.F4N)
        ev = torch.cuda.Event()
        ev.record(cur)
        ms.wait_event(ev)
        rs.wait_event(ev)
        with torch.cuda.stream(ms):
            MAIN.replay()
        if eager:
            h = L.stream_handle(rs)
            for c in eng.res_calls:
                c(h)
        else:
            with torch.cuda.stream(rs):
                RES.replay()
        join(cur, [ms, rs])
        eng.load_batch(pool[i % 2], next_images=pool[(i + 1) % 2]["image_tensors"])
    return f


def single_step(i):
    for g in single:
        g() if callable(g) else g.replay()
    eng.load_batch(pool[i % 2], next_images=pool[(i + 1) % 2]["image_tensors"])


ms = torch.cuda.Stream()
plain = torch.cuda.Stream()
print(f"single (bench graph)       {timed(single_step):7.3f} ms/step", flush=True)
print(f"main graph alone           {timed(lambda i: MAIN.replay()):7.3f} ms", flush=True)
print(f"res graph alone, all CUs   {timed(res_only(plain, False)):7.3f} ms", flush=True)
print(f"two, all CUs               {timed(two(plain, ms, False)):7.3f} ms/step", flush=True)
for k in (32, 64, 96, 128):
    for pat in ("strided", "low"):
        bits = [int(j * ncu / k) for j in range(k)] if pat == "strided" else list(range(k))
        rs = masked_stream(bits)
        r_g = timed(res_only(rs, False))
        r_e = timed(res_only(rs, True))
        t_g = timed(two(rs, ms, False))
        t_e = timed(two(rs, ms, True))
        print(f"K={k:3d} {pat:7s}: res alone graph {r_g:6.3f} eager {r_e:6.3f} | two graph {t_g:6.3f} "
              f"eager {t_e:6.3f} ms/step", flush=True)
print(f"single (bench graph)       {timed(single_step):7.3f} ms/step", flush=True)
