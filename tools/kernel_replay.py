"""Replay selected launches of the benched step alone, for rocprofv3 PMC passes.

  python tools/kernel_replay.py MANIFEST.json [REPS]

Builds the engine exactly as bench.py does (B=64, 224x224, L=32, tuned tiles; mode c5: as
bench.py --config5 builds it, 384x384, T5-large, 6 blocks, fp8),
runs one forward/backward so every buffer holds real data, then replays, REPS
times each and in this order: the whole-arena AdamW pass, the ConvTranspose2d
weight-gradient GEMM, the largest e4m3 launch (config 5), and every SGA launch bench.py's
sga_mfma counts.  The
manifest lists (tag, kernel call name, FLOP, algorithmic bytes) per dispatch in
issue order, so tools/pmc_step.py can map the LAST dispatches of a profile to
them."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402
from bench import call_bytes  # noqa: E402  (the algorithmic byte model bench.py reports)

out_path = sys.argv[1]
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
MODE = sys.argv[3] if len(sys.argv) > 3 else "default"     # "res": every frozen-ResNet launch instead;
pkg = load_package()                                         # "c5": the config-5 engine (bench.py --config5)
L = pkg.lib
dev = torch.device("cuda", 0)
C5 = MODE == "c5"
B, Lq, H = 64, 32, (384 if C5 else 224)
lm, NB = ("t5-large", 6) if C5 else ("t5-base", 3)
sd = pkg.synthetic.make_state_dict("resnet50", seed=0, num_attention_blocks=NB, language_model=lm)
eng = pkg.engine.VQAEngine(sd, vision="resnet50", batch=B, seq_len=Lq, image_size=H, device=dev, warmup=10,
                           total=100000, dropout=0.1, seed=0, num_blocks=NB, language_model=lm, fp8=C5)
del sd
eng.load_batch(pkg.synthetic.make_batch(B, Lq, H, seed=1))
eng.forward()
eng.backward()
eng.autotune(table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"))
eng.forward()
eng.backward()
eng.optimizer_step()          # leaves the update pending, so the AdamW replays below do the full pass
torch.cuda.synchronize()
s = L.stream_handle()


def gemm_flop(c):
    if c.name == "vqa_gemm":
        return 2.0 * c.desc.m * c.desc.n * c.desc.k * max(1, c.desc.batch)
    if c.name == "vqa_gemm_pair":
        return sum(2.0 * d.m * d.n * d.k for d in c.desc)
    d = c.desc
    return (4.0 if c.name == "vqa_attn_fwd" else 8.0) * d.batch * d.heads * d.lq * d.lk * d.dh


plan = [("adamw", eng.adam_full, 0.0, 38.0 * eng.lay.total)]
if MODE == "res":
    plan = [(f"res{i:02d}", c, gemm_flop(c) if c.name == "vqa_gemm" else 0.0, call_bytes(c))
            for i, c in enumerate(eng.res_calls)]
    # the T5 layer-0 forward GEMMs for comparison
    t5 = [c for c in eng.fwd_calls[eng._t5_layer_start[0]:eng._t5_layer_start[1]] if c.name == "vqa_gemm"]
    plan += [(f"t5_{i}", c, gemm_flop(c), call_bytes(c)) for i, c in enumerate(t5)]
if MODE != "res":
    wg = eng.scaler_dw_call                                  # the tap-batched scaler dW GEMM
    plan.append(("convT_dW", wg, gemm_flop(wg), call_bytes(wg)))
    f8 = [c for c in eng.res_calls + eng.fwd_calls + eng.bwd_calls if c.name == "vqa_gemm" and c.desc.fp8]
    if f8:                                                   # bench roofline_fp8: the largest e4m3 launch
        c8 = max(f8, key=gemm_flop)
        plan.append(("fp8_gemm", c8, gemm_flop(c8), call_bytes(c8)))
    sga = [c for c in eng.sga_vision_calls + eng.fwd_calls[eng._fsplit[2]:] + eng.bwd_calls[:eng._bsplit[0]]
           if c.name in ("vqa_gemm", "vqa_gemm_pair", "vqa_attn_fwd", "vqa_attn_bwd")]
    for c in sga:
        plan.append(("sga_gemm" if c.name.startswith("vqa_gemm") else "sga_attn", c, gemm_flop(c), call_bytes(c)))
man = []
for tag, c, fl, by in plan:
    for _ in range(REPS):
        c(s)
        # a paired launch is one dispatch; every call here is one kernel dispatch
        d = c.desc if c.name == "vqa_gemm" else None
        man.append({"tag": tag, "call": c.name, "flop": fl, "bytes": by,
                    "shape": [d.m, d.n, d.k, d.config, d.splitk] if d is not None else None})
torch.cuda.synchronize()
json.dump({"reps": REPS, "dispatches": man}, open(out_path, "w"))
print(f"replayed {len(man)} dispatches", flush=True)
