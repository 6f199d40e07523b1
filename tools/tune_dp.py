"""Time the GEMM shapes that only a data-parallel engine has (the T5 weight gradients
batched in dp.DP_T5_DW_GROUPS) on one GPU and write the merged tuning table, so every
rank of a multi-GPU bench picks its tiles from the committed table instead of timing
them at start-up.

  python tools/tune_dp.py OUT.json"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
B, L, H = 64, 32, 224
eng = pkg.engine.VQAEngine(pkg.synthetic.make_state_dict("resnet50", seed=0), vision="resnet50", batch=B, seq_len=L,
                           image_size=H, device="cuda", warmup=10, total=100000, dropout=0.1, seed=0, pipeline=True,
                           t5_dw_group=pkg.dp.DP_T5_DW_GROUPS)
nb = {k: torch.as_tensor(v).cuda() for k, v in pkg.synthetic.make_batch(B, L, H, seed=1).items() if v is not None}
eng.prime(nb["image_tensors"])
eng.F4.copy_(eng.F4N)
eng.load_batch(nb, next_images=nb["image_tensors"])
eng.forward()
eng.backward()
eng.autotune(reps=20, table=os.path.join(ROOT, "t5-resnet-vqa_amd", "tuning", "gemm_gfx950.json"), save=sys.argv[1])
torch.cuda.synchronize()
print("saved", sys.argv[1], flush=True)
