"""Reference point for the frozen ResNet-50 feature extractor: the same network (eval BN,
up to layer4) through torch / MIOpen, bf16 channels-last, B=64 at 224x224, timed with HIP
events -- against the engine's own ResNet chain (engine.res_calls) on the same box.

  python tools/resnet_miopen_ref.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import tv_stub  # noqa: E402
from __graft_entry__ import load_package  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, H = 64, 224


def timed(fn):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps


net = tv_stub.resnet50()
body = torch.nn.Sequential(net.conv1, net.bn1, net.relu, net.maxpool, net.layer1, net.layer2, net.layer3,
                           net.layer4).eval().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
x = torch.randn(B, 3, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
torch.backends.cudnn.benchmark = True
with torch.no_grad():
    t_eager = timed(lambda: body(x))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(x)
        with torch.cuda.graph(g):
            y = body(x)
    torch.cuda.current_stream().wait_stream(s)
    t_graph = timed(g.replay)
print(f"torch/MIOpen ResNet-50 to layer4, bf16 NHWC, B={B}: eager {t_eager:.3f} ms, graph {t_graph:.3f} ms "
      f"(out {tuple(y.shape)})")

pkg = load_package()
sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=32, image_size=H, warmup=10, total=1000, pipeline=True)
eng.load_batch(pkg.synthetic.make_batch(B, 32, H, seed=1), next_images=pkg.synthetic.make_batch(B, 32, H, seed=2)["image_tensors"])
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
st = pkg.lib.stream_handle()
t_eng = timed(lambda: eng._run(eng.res_calls))
print(f"engine ResNet chain (res_calls, {len(eng.res_calls)} launches, eager ctypes replay): {t_eng:.3f} ms")
