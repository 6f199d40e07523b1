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
