"""The DP leg at the benched shape: WORLD DataParallelStep ranks (tests/dp_worker.py mode c5full:
B = 64 per rank, 384^2, T5-large, 6 SGA blocks at 1024, e4m3 forward weight GEMMs -- BASELINE
config 5; or c2full: B = 64 per rank, 224^2, t5-base, 3 SGA blocks -- config 2, and config 3 at
WORLD 8), pipelined and graphed, gloo on the one GPU, for 3 steps against ONE engine on the
WORLD x 64-row global batch (eager), as tests/test_a_dp2_gpu.py's two-rank tests do at B = 4, 64^2.
Writes OUT.json with the measured errors and the bounds those tests use (config 5's).
  python tools/dp_full_parity.py OUT.json [c5full|c2full] [WORLD]"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else "c5full"
    world, steps = (int(sys.argv[3]) if len(sys.argv) > 3 else 2), 3
    c5 = mode == "c5full"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    tmp = tempfile.mkdtemp()
    outs = [os.path.join(tmp, f"r{r}.npz") for r in range(world)]
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_worker.py"), str(r), str(world), port,
                               outs[r], str(steps), "1", "1", mode]) for r in range(world)]
    rcs = [p.wait(timeout=1500) for p in procs]
    assert rcs == [0] * world, rcs
    res = [np.load(o) for o in outs]
    lock = all(np.array_equal(r["p32"], res[0]["p32"]) and np.array_equal(r["norms"], res[0]["norms"])
               for r in res[1:])
    print("ranks done, lockstep", lock, flush=True)
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    B, L, H = 64, 32, (384 if c5 else 224)
    kw = dict(language_model="t5-large", num_blocks=6, fp8=True) if c5 else {}
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0, **({"num_attention_blocks": 6, "language_model": "t5-large"}
                                                              if c5 else {}))
    ref = pkg.engine.VQAEngine(sd, batch=world * B, seq_len=L, image_size=H, warmup=1, total=20, dropout=0.0,
                               device="cuda:0", **kw)
    gloss, gnorm = [], []
    for i in range(steps):
        ref.load_batch(pkg.synthetic.make_batch(world * B, L, H, seed=40 + i))
        ref.train_step()
        torch.cuda.synchronize()
        gloss.append(float(ref.LOSS.item()))
        gnorm.append(ref.last_grad_norm())
        print("reference step", i, flush=True)
    ref.flush_optimizer()
    p_ref = ref.P32.cpu().numpy()
    dloss = np.abs(np.mean([r["losses"] for r in res], axis=0) - gloss) / np.abs(gloss)
    dnorm = np.abs(res[0]["norms"] - gnorm) / np.array(gnorm)
    p0 = ref.lay.pack(sd)
    upd = float(np.linalg.norm(res[0]["p32"].astype(np.float64) - p_ref) /
                np.linalg.norm(p_ref.astype(np.float64) - p0))
    ok = bool(lock and dloss[0] <= 1e-5 and dnorm[0] <= 1e-4 and (dloss <= 2e-3).all() and (dnorm <= 2e-2).all()
              and upd <= 5e-2)
    rep = {"what": f"{'config 5' if c5 else 'config 2/3'} DP leg at the benched shape: {world} ranks x B=64 "
                   f"(gloo, one GPU, pipelined, graphed) vs one eager engine on the {world * B}-row global batch, "
                   "3 steps, dropout 0", "mode": mode, "world": world,
           "ranks_lockstep": bool(lock), "loss_rel": dloss.tolist(), "grad_norm_rel": dnorm.tolist(),
           "update_rel_l2": upd, "losses_dp": np.mean([r["losses"] for r in res], axis=0).tolist(),
           "losses_ref": gloss,
           "bounds (tests/test_a_dp2_gpu.py::test_dp_config5_two_ranks_match_global_batch)":
               "loss step 0 <= 1e-5, norm step 0 <= 1e-4; every step loss <= 2e-3, norm <= 2e-2; update <= 5e-2",
           "pass": ok}
    json.dump(rep, open(out, "w"), indent=1)
    print(json.dumps(rep))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
