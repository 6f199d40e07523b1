"""The data-parallel step (bucketed async RCCL all-reduce overlapped with the
segmented backward graphs + (id, row) all-gather for the embedding) at
world_size 1 on one MI355X: every exchange is then an identity, so it must
reproduce the single-GPU graph step bit for bit.  Multi-rank arithmetic is
covered by tests/test_dp_cpu.py (gloo)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("graph", [False, True])
def test_dp_world1_matches_single_gpu(pg, pkg, graph):
    B, L, H = 4, 32, 96
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    nb = pkg.synthetic.make_batch(B, L, H, seed=1)
    e1 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20)
    # the DP engine batches the T5 weight gradients in groups of 4 layers (bench.py), the
    # single-GPU one over all 12: same bits, different bucket boundaries
    e2 = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=20, t5_dw_group=4)
    e1.load_batch(nb)
    e2.load_batch(nb)
    step = pkg.dp.DataParallelStep(e2, bucket_mb=8, use_graph=graph)
    assert len(step.buckets) >= 5
    for _ in range(3):
        e1.train_step()
        step.step()
    torch.cuda.synchronize()
    assert float(e1.LOSS) == float(e2.LOSS)
    assert torch.equal(e1.G32, e2.G32)
    assert torch.equal(e1.P32, e2.P32)
