"""How do two independent branches of the forward (frozen ResNet + ConvT on one
stream, T5 encoder on another) actually overlap on MI355X?  Times, with HIP
events on the launching stream:
  serial        both branches on one stream
  eager2        eager launches, branches on two streams (interleaved issue)
  graph1        one graph captured with the two-stream fork/join
  graph2        two single-chain graphs replayed on two streams
"""
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
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=224, warmup=10, total=1000)
eng.load_batch(pkg.synthetic.make_batch(B, 32, 224, seed=1))
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
f = eng.fwd_calls
p0, p1, p2 = eng._fsplit
vis, txt = f[p0:p1], f[p1:p2]
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
hm, hs = L.stream_handle(main), L.stream_handle(side)


def serial():
    for c in vis + txt:
        c(hm)


def eager2():
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    j = 0
    for i, c in enumerate(vis):
        c(hm)
        upto = (i + 1) * len(txt) // len(vis)
        while j < upto:
            txt[j](hs)
            j += 1
    for c in txt[j:]:
        c(hs)
    ev2 = torch.cuda.Event()
    ev2.record(side)
    main.wait_event(ev2)


def vis_only():
    for c in vis:
        c(hm)


def txt_only():
    for c in txt:
        c(hm)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record(main)
    for _ in range(reps):
        fn()
    en.record(main)
    en.synchronize()
    return st.elapsed_time(en) / reps * 1e3


res = {}
res["vis_only"] = timeit(vis_only)
res["txt_only"] = timeit(txt_only)
res["serial"] = timeit(serial)
res["eager2"] = timeit(eager2)
# graph1: one graph, two-stream fork/join captured
cs = torch.cuda.Stream()
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1, stream=cs):
    cur = torch.cuda.current_stream()
    hm2 = L.stream_handle(cur)
    ev = torch.cuda.Event()
    ev.record(cur)
    side.wait_event(ev)
    j = 0
    for i, c in enumerate(vis):
        c(hm2)
        upto = (i + 1) * len(txt) // len(vis)
        while j < upto:
            txt[j](hs)
            j += 1
    for c in txt[j:]:
        c(hs)
    ev2 = torch.cuda.Event()
    ev2.record(side)
    cur.wait_event(ev2)
res["graph1"] = timeit(g1.replay)
# graph2: two linear graphs on two streams
gv, gt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.graph(gv, stream=cs):
    h = L.stream_handle(torch.cuda.current_stream())
    for c in vis:
        c(h)
with torch.cuda.graph(gt, stream=cs):
    h = L.stream_handle(torch.cuda.current_stream())
    for c in txt:
        c(h)
res["graph_vis"] = timeit(gv.replay)
res["graph_txt"] = timeit(gt.replay)


def graph2():
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        gt.replay()
    gv.replay()
    ev2 = torch.cuda.Event()
    ev2.record(side)
    main.wait_event(ev2)


res["graph2"] = timeit(graph2)
for k, v in res.items():
    print(f"{k:10s} {v:9.1f} us", flush=True)

# ---- ResNet (next batch) beside the backward + optimizer of this step
eng.forward()
torch.cuda.synchronize()
bo = eng.bwd_calls + eng.opt_calls
gb, gvis = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
saved = eng.opt_state.clone()
with torch.cuda.graph(gb, stream=cs):
    h = L.stream_handle(torch.cuda.current_stream())
    for c in bo:
        c(h)
vis_nct = vis[:-1]                                   # ResNet without the ConvT (it needs the updated scaler)
with torch.cuda.graph(gvis, stream=cs):
    h = L.stream_handle(torch.cuda.current_stream())
    for c in vis_nct:
        c(h)


def bwd_only():
    gb.replay()


def res_only():
    gvis.replay()


def bwd_res_serial():
    gb.replay()
    gvis.replay()


def bwd_res_overlap():
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        gvis.replay()
    gb.replay()
    ev2 = torch.cuda.Event()
    ev2.record(side)
    main.wait_event(ev2)


for nm, fn in (("bwd+opt", bwd_only), ("resnet", res_only), ("serial", bwd_res_serial), ("overlap", bwd_res_overlap)):
    print(f"{nm:10s} {timeit(fn):9.1f} us", flush=True)
eng.opt_state.copy_(saved)
