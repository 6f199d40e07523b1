"""Parity of the N > 1 training step at the benched size, on one GPU.

test_dp_step_b64_matches_oracle: dp.DataParallelStep -- the step bench.py runs at N > 1
(the backward as stage graphs with the single-GPU stream placement, the bucketed collectives
issued between them, gathered embedding rows, then the finish graph: embedding scatter,
grad-norm partials, clip, AdamW) -- over a world-1 RCCL
group on the DP engine (R50, B=64, 224x224, L=32, pipelined frozen ResNet, tuned tiles,
deferred AdamW, dropout 0.1, T5 weight-gradient groups (4, 4, 3, 1)), stepped 3 times
against the CPU fp32 oracle on the same batches and dropout masks
(trainer/faster_rcnn_vqa_trainer.py:391-406).  Same tolerances as the single-GPU benched
step (tests/bench_step_worker.py)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DELTA_RTOL = 0.1


def test_dp_step_b64_matches_oracle(parity_report):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    sys.path.insert(0, HERE)
    import bench_step_worker
    rep, fails = bench_step_worker.run("dp")
    parity_report["dp_world1_b64"] = rep
    assert rep["buckets"] >= 4, rep["buckets"]
    assert not fails, (fails, rep)
    assert max(rep["update_rel_l2"].values()) <= DELTA_RTOL, rep["update_rel_l2"]
