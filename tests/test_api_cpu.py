"""Argument validation of the reference-interface mirror (no GPU needed: it fails before any allocation)."""
import pytest


def test_model_rejects_unsupported_configs(pkg):
    with pytest.raises(ValueError):
        pkg.model.ResnetVQAModel("faster-rcnn", "t5-base", 170)
    with pytest.raises(ValueError):
        pkg.model.ResnetVQAModel("resnet50", "t5-3b", 170)
    with pytest.raises(ValueError):
        pkg.model.ResnetVQAModel("resnet50", "t5-base", 170, num_attention_blocks=0)


def test_trainer_signature_mirrors_reference(pkg):
    import inspect
    sig = inspect.signature(pkg.trainer.VQATrainer.train_one_step)
    assert list(sig.parameters)[:2] == ["self", "data_items"]
    fwd = inspect.signature(pkg.model.ResnetVQAModel.forward)
    # resnet_vqa_model.py:101-112 keyword set
    assert list(fwd.parameters)[1:] == ["question_input_ids", "decoder_question_input_ids",
                                        "question_attention_masks", "decoder_question_attention_masks",
                                        "annotation_ids", "image_tensors", "answer_input_ids", "pixel_values",
                                        "answer_attention_masks", "question_type_ids"]


def test_collate_refuses_interpolations_without_a_kernel(pkg):
    """resnet_vqa_daquar_dataset.py:156-164 accepts LINEAR / LANCZOS4 / CUBIC; the GPU collate
    has the INTER_LINEAR kernel only and says so instead of training on other pixels."""
    for strategy in ("LANCZOS4", "CUBIC", 4):
        with pytest.raises(NotImplementedError):
            pkg.data.DaquarCollate(interpolation_strategy=strategy, device="cpu")


def test_short_batch_rows_are_padded_with_real_rows_and_ignored_targets(pkg):
    """A loader's short last batch (no drop_last in the reference, faster_rcnn_vqa_trainer.py:172-197)
    on a planned-B engine: rows past B' are copies of rows 0..B'-1 (every activation stays a real
    sample's) and their targets NLLLoss's ignore_index, so the head's mean runs over B' rows."""
    import torch
    E = pkg.engine
    dst = torch.full((7, 3), -1.0)
    src = torch.arange(9.0).reshape(3, 3)
    E.load_rows(dst, src, 3)
    assert torch.equal(dst, src[torch.tensor([0, 1, 2, 0, 1, 2, 0])])
    tgt = torch.zeros(7, dtype=torch.int64)
    E.load_rows(tgt, torch.tensor([5, 6, 7]), 3, fill=E.IGNORE_INDEX)
    assert tgt.tolist() == [5, 6, 7, -100, -100, -100, -100]
    full = torch.zeros(7, dtype=torch.int64)
    E.load_rows(full, torch.arange(7), 7, fill=E.IGNORE_INDEX)
    assert full.tolist() == list(range(7))
    assert E.batch_rows({"q": torch.zeros(5, 2)}, "q", 7) == 5
    for bad in (0, 8):
        with pytest.raises(ValueError):
            E.batch_rows({"q": torch.zeros(bad, 2)}, "q", 7)


def test_empty_data_parallel_rank_rows(pkg):
    """A data-parallel rank whose share of the global batch is empty (engine.use_global_rows):
    batch_rows accepts 0 rows only with allow_empty, and load_rows fills every row -- targets with
    ignore_index (the rank's gradient is exactly zero), inputs with a finite constant (masks 1)."""
    import torch
    E = pkg.engine
    assert E.batch_rows({"q": torch.zeros(0, 2)}, "q", 7, allow_empty=True) == 0
    with pytest.raises(ValueError):
        E.batch_rows({"q": torch.zeros(8, 2)}, "q", 7, allow_empty=True)
    img = torch.full((4, 3), float("nan"))
    E.load_rows(img, torch.zeros(0, 3), 0)
    assert torch.equal(img, torch.zeros(4, 3))
    mask = torch.zeros(4, 5, dtype=torch.int64)
    E.load_rows(mask, torch.zeros(0, 5, dtype=torch.int64), 0, empty_fill=1)
    assert bool((mask == 1).all())
    tgt = torch.zeros(4, dtype=torch.int64)
    E.load_rows(tgt, torch.zeros(0, dtype=torch.int64), 0, fill=E.IGNORE_INDEX)
    assert tgt.tolist() == [-100] * 4
