"""The collate's image path on the GPU (vqa_resize_linear_u8 through data.ImageBatcher /
data.DaquarCollate) against the CPU restatement (oracle/image_oracle.py): bit-exact
fp32 output for variable-size images, up- and down-scaling, borders, files decoded
from disk; and a training step fed straight from it
(dataset_utils/resnet_vqa_daquar_dataset.py:145-231)."""
import numpy as np
import pytest
import torch

from oracle import image_oracle as io

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("oh,ow", [(256, 256), (224, 224), (37, 300), (1, 1)])
def test_resize_matches_oracle_bit_exact(cuda, pkg, oh, ow):
    imgs = pkg.data.synthetic_images(6, seed=oh + ow, min_side=1, max_side=700)
    imgs += [np.full((1, 1, 3), 9, np.uint8), np.random.default_rng(5).integers(0, 256, (2 * oh, 2 * ow, 3),
                                                                                 dtype=np.uint8)]
    got = pkg.data.ImageBatcher(oh, ow)(imgs).cpu().numpy()
    ref = io.collate_images(imgs, oh, ow)
    assert got.shape == ref.shape
    bad = np.argwhere(got != ref)
    assert bad.size == 0, (len(bad), bad[:5])


def test_collate_from_files_and_train_step(cuda, pkg, tmp_path):
    """Images written to disk (PNG, lossless), decoded on the host, resized on the GPU
    directly into a pipelined engine's image buffer, then one training step."""
    from PIL import Image
    B, L, H = 4, 16, 64
    imgs = pkg.data.synthetic_images(B, seed=11, min_side=40, max_side=120)
    pts = []
    for i, a in enumerate(imgs):
        p = tmp_path / f"im{i}.png"
        Image.fromarray(a).save(p)
        pts.append({"image_path": str(p), "question_ids": [32100] + list(range(5, 5 + 3 * i)) + [1],
                    "annotation_id": 7 * i})
    col = pkg.data.DaquarCollate(resizing_dimensions=(H, H), max_question_length=L)
    sd = pkg.synthetic.make_state_dict("resnet50", seed=0)
    eng = pkg.engine.VQAEngine(sd, batch=B, seq_len=L, image_size=H, warmup=1, total=10)
    batch = col(pts, out=eng.IMG)                      # resized straight into the engine's buffer
    assert batch["image_tensors"].data_ptr() == eng.IMG.data_ptr()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(eng.IMG.cpu().numpy(), io.collate_images(imgs, H, H))
    assert batch["question_input_ids"].shape == (B, L) and int(batch["question_attention_masks"][3].sum()) == 11
    lp, loss = eng.forward_backward({k: v for k, v in batch.items() if k != "image_tensors"} | {
        "image_tensors": eng.IMG})
    assert np.isfinite(loss) and lp.shape == (B, 170)
