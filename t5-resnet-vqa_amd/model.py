"""`ResnetVQAModel` — the reference's model API (model/resnet_vqa_model.py:28-165)
over the MI355X engine.

Same constructor arguments, same `forward(**batch)` keyword set and return
value `(log_probs [B, answer_spaces], loss or None)`, the same state-dict keys
 and the attribute names the reference trainer reads
(`vision_model_name`, `device`).  What differs, by design:

* shapes are planned once: `batch_size`, `seq_len` and `image_size` are fixed
  at construction (the hipGraph step has static buffers).  A batch of FEWER rows
  -- the short last batch of the reference's loaders, which have no drop_last
  (faster_rcnn_vqa_trainer.py:172-197) -- is padded to the planned batch with
  copies of its own rows whose targets are ignore_index: the loss is the mean
  over the real rows and the padding gets no gradient, so the step equals the
  reference's step on the short batch; log-probs come back for the real rows.
  More rows, or another question length / image size, raise ValueError;
* weights come from a reference `state_dict` (e.g. `torch.load(best-model.pt,
  weights_only=True)`) or, offline, from the deterministic synthetic init —
  `from_pretrained` downloads are not available here;
* backward / the optimizer live in `trainer.VQATrainer.train_one_step`, which
  runs zero_grad → forward → backward → clip → AdamW → scheduler as one graph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import synthetic as S
from .engine import VQAEngine

SUPPORTED_VISION = ("resnet50", "resnet34", "resnet18")


class ParameterGroup:
    """The reference sub-module attribute a trainer reads (`model.lang_model`,
    `model.sga_modules`, ...; faster_rcnn_vqa_trainer.py:231-263): its `parameters()` /
    `named_parameters()` are live device views into the engine's flat fp32 arena (each with
    `.grad` = the matching gradient view), `state_dict()` gives the reference entries.
    The frozen ResNet (`vision_model`) and the unused scaler are plain fp32 tensors: the
    reference never gives them a gradient.  Writes through the views reach
    the fp32 masters; call `model.engine.refresh_shadow()` before the next step so the bf16
    GEMM operands follow."""

    def __init__(self, model, prefix, trainable=True):
        self._model, self.prefix, self.trainable = model, prefix, trainable

    def _keys(self):
        m = self._model
        return [k for k in S.model_specs(m.vision_model_name, m.answer_spaces, m.num_attention_blocks,
                                         m.language_model_name) if k.startswith(self.prefix + ".")]

    def named_parameters(self):
        e = self._model.engine
        for k in self._keys():
            if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
                continue
            v = e.param_view(k) if self.trainable else None
            if v is None:
                t = torch.as_tensor(np.asarray(e._frozen[k]))
                yield k[len(self.prefix) + 1:], t
            else:
                p, g = v
                p.grad = g
                yield k[len(self.prefix) + 1:], p

    def parameters(self):
        for _, p in self.named_parameters():
            yield p

    def state_dict(self):
        sd = self._model.engine.state_dict()
        return {k[len(self.prefix) + 1:]: torch.from_numpy(np.ascontiguousarray(np.asarray(sd[k])))
                for k in self._keys() if k in sd}

    def __getitem__(self, i):                          # sga_modules[n]
        return ParameterGroup(self._model, f"{self.prefix}.{int(i)}", self.trainable)

    def __len__(self):
        return self._model.num_attention_blocks if self.prefix == "sga_modules" else len(self._keys())

    def eval(self):
        return self

    def train(self, mode=True):
        return self


class ResnetVQAModel:
    def __init__(self, vision_model_name, language_model_name, answer_spaces, fine_tune_lm_encoder=True,
                 fine_tune_lm_decoder=True, fine_tune_vision=True, num_attention_blocks=3, device="cuda",
                 *, batch_size=64, seq_len=32, image_size=224, state_dict=None, seed=0, dropout=0.1,
                 dropout_seed=0):
        # resnet_vqa_model.py:51-58 builds only resnet18/34/50 and fails later for other names;
        # fail here, with the reason.
        if vision_model_name not in SUPPORTED_VISION:
            raise ValueError(f"vision_model_name {vision_model_name!r}: this path supports {SUPPORTED_VISION}")
        # t5-base is the reference's model (resnet_vqa_model.py:60-62); t5-large is BASELINE
        # configs[4]: the encoder of the published t5-large sizes with the SGA blocks, scaler,
        # pooler and classifier built at its width 1024 (the reference hard-codes 768 only in
        # those constructors, multi_head_vision_text_attn.py:9,19, resnet_vqa_model.py:64-89)
        if language_model_name not in S.LM_DIMS:
            raise ValueError(f"language_model_name must be one of {tuple(S.LM_DIMS)}")
        if num_attention_blocks < 1:
            raise ValueError("num_attention_blocks must be >= 1")
        self.vision_model_name = vision_model_name
        self.language_model_name = language_model_name
        self.answer_spaces = int(answer_spaces)
        self.num_attention_blocks = int(num_attention_blocks)
        self.device = torch.device(device)
        self.batch_size, self.seq_len, self.image_size = int(batch_size), int(seq_len), int(image_size)
        self._cfg = dict(dropout=float(dropout), seed=int(dropout_seed))
        if state_dict is None:
            state_dict = S.make_state_dict(vision_model_name, seed=seed, answer_spaces=self.answer_spaces,
                                           num_attention_blocks=self.num_attention_blocks,
                                           language_model=language_model_name)
        self._build(state_dict)
        self.training = True
        # the sub-module attributes the reference trainer reads (faster_rcnn_vqa_trainer.py:231-263)
        scaler = "downscale_layer" if vision_model_name == "resnet50" else "upscale_layer"
        self.vision_model = ParameterGroup(self, "vision_model", trainable=False)
        self.lang_model = ParameterGroup(self, "lang_model")
        self.downscale_layer = ParameterGroup(self, "downscale_layer", trainable=scaler == "downscale_layer")
        self.upscale_layer = ParameterGroup(self, "upscale_layer", trainable=scaler == "upscale_layer")
        self.sga_modules = ParameterGroup(self, "sga_modules")
        self.attention_pooler = ParameterGroup(self, "attention_pooler")
        self.classification_layer = ParameterGroup(self, "classification_layer")

    # ------------------------------------------------------------------ engine
    def _build(self, state_dict, **kw):
        sd = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
              for k, v in state_dict.items()}
        missing = [k for k in S.model_specs(self.vision_model_name, self.answer_spaces, self.num_attention_blocks,
                                            self.language_model_name) if k not in sd]
        if missing:
            raise KeyError(f"state_dict lacks {len(missing)} reference keys, e.g. {missing[:3]}")
        opt = dict(getattr(self, "_opt", {}))
        opt.update(kw)
        self.engine = VQAEngine(sd, vision=self.vision_model_name, batch=self.batch_size, seq_len=self.seq_len,
                                image_size=self.image_size, device=self.device, answer_spaces=self.answer_spaces,
                                num_blocks=self.num_attention_blocks, language_model=self.language_model_name,
                                **self._cfg, **opt)
        self._opt = opt

    def train(self, mode=True):
        """nn.Module.train: dropout on (the reference trains with p = 0.1 at every site)."""
        self.training = bool(mode)
        self.engine.set_training(self.training)
        return self

    def eval(self):
        return self.train(False)

    # ------------------------------------------------------------------ forward
    def _check_batch(self, question_input_ids, image_tensors):
        n = int(question_input_ids.shape[0])
        lo = 0 if self.engine.allow_empty_rows else 1         # 0: an empty data-parallel rank
        if not lo <= n <= self.batch_size:
            raise ValueError(f"batch of {n} rows: the model is planned for {lo}..{self.batch_size} rows")
        want_q = (n, self.seq_len)
        want_i = (n, 3, self.image_size, self.image_size)
        if tuple(question_input_ids.shape) != want_q:
            raise ValueError(f"question_input_ids shape {tuple(question_input_ids.shape)} != planned {want_q}")
        if tuple(image_tensors.shape) != want_i:
            raise ValueError(f"image_tensors shape {tuple(image_tensors.shape)} != planned {want_i}")

    def load_items(self, items):
        """The reference collate's batch dict (the keys train_one_step passes on)."""
        self.load_batch(items["question_input_ids"], items["question_attention_masks"], items["image_tensors"],
                        items.get("annotation_ids"))

    def load_batch(self, question_input_ids, question_attention_masks, image_tensors, annotation_ids=None):
        self._check_batch(question_input_ids, image_tensors)
        self.engine.load_batch({"question_input_ids": question_input_ids,
                                "question_attention_masks": question_attention_masks,
                                "image_tensors": image_tensors, "annotation_ids": annotation_ids})

    def forward(self, question_input_ids, decoder_question_input_ids=None, question_attention_masks=None,
                decoder_question_attention_masks=None, annotation_ids=None, image_tensors=None,
                answer_input_ids=None, pixel_values=None, answer_attention_masks=None, question_type_ids=None):
        """resnet_vqa_model.py:101-165: returns (log_probs, loss); loss is None without
        annotation_ids.  decoder_*, answer_*, pixel_values and question_type_ids are
        accepted and ignored, as in the reference."""
        if question_attention_masks is None or image_tensors is None:
            raise TypeError("forward() needs question_attention_masks and image_tensors")
        self.load_batch(question_input_ids, question_attention_masks, image_tensors, annotation_ids)
        self.engine.forward()
        log_probs = self.engine.LOGP[:self.engine.rows].clone()
        loss = self.engine.LOSS[0].clone() if annotation_ids is not None else None
        return log_probs, loss

    __call__ = forward

    def generate_answers(self, question_input_ids, decoder_question_input_ids=None, question_attention_masks=None,
                         decoder_question_attention_masks=None, image_tensors=None, annotation_ids=None,
                         answer_input_ids=None, pixel_values=None, answer_attention_masks=None,
                         question_type_ids=None):
        """resnet_vqa_model.py:167-231: the forward plus the frozen ResNet's layer4 map,
        returned as (log_probs, loss or None, {"features": [B, C, h, w] fp32}) (the kernels
        hold the map in bf16, so the features carry bf16 rounding)."""
        log_probs, loss = self.forward(question_input_ids, decoder_question_input_ids, question_attention_masks,
                                       decoder_question_attention_masks, annotation_ids, image_tensors)
        return log_probs, loss, {"features": self.engine.layer4_features()}

    @staticmethod
    def convert_logits_to_predictions(lm_logits):
        """faster_rcnn_vqa_trainer.py:484-488: argmax of exp(log-probs) over the answers."""
        return torch.argmax(torch.exp(lm_logits), dim=1)

    # ------------------------------------------------------------------ weights
    def state_dict(self):
        """Reference keys -> fp32 CPU tensors (loadable by the reference ResnetVQAModel)."""
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in self.engine.state_dict().items()}

    def load_state_dict(self, state_dict, strict=True):
        """Load reference weights (optimizer state restarts, as in the reference's init_model,
        train_faster_rcnn_vqa.py:40-45)."""
        sd = dict(state_dict)
        if not strict:
            cur = self.state_dict()
            cur.update({k: v for k, v in sd.items() if k in cur})
            sd = cur
        training = self.training
        self._build(sd)
        if getattr(self, "_optim_cfg", None):             # the trainer's AdamW / schedule settings survive
            self.engine.configure_optimizer(**self._optim_cfg)
        self.train(training)

    def configure_optimizer(self, **kw):
        """Optimizer / schedule settings (trainer._init_optimizer); kept on the model so a
        later load_state_dict rebuilds the engine with them."""
        self._optim_cfg = dict(getattr(self, "_optim_cfg", None) or {}, **kw)
        self.engine.configure_optimizer(**kw)

    def parameters_count(self):
        return self.engine.lay.num_params


VIT_NAMES = ("google/vit-base-patch16-224-in21k",)


class _VitGroup(ParameterGroup):
    """ParameterGroup over the config-4 engine (the ViT trainer's groups, vit_vqa_trainer.py:300-316)."""

    def _keys(self):
        from . import vit_model as VM
        return [k for k in VM.model_specs(self._model.answer_spaces, self._model.image_size)
                if k.startswith(self.prefix + ".")]

    def __len__(self):
        return len(self._keys())


class VitVQAModel:
    """`VitVQAModel` (model/vit_vqa_model.py:127-351) -- BASELINE config 4 -- over
    `vit_engine.VitVQAEngine`: the same constructor names, `forward(**batch)` ->
    (log_probs, loss), `generate_answers`, the reference state-dict keys and the
    sub-modules the ViT trainer reads (`vision_model`, `lang_model`, `fusing_layer`,
    `classification_layer`).  Shapes are fixed at construction (batch, question and
    decoder lengths, image size), as for ResnetVQAModel."""

    def __init__(self, vision_model_name="google/vit-base-patch16-224-in21k", language_model_name="t5-base",
                 answer_spaces=170, fine_tune_lm_encoder=True, fine_tune_lm_decoder=True, fine_tune_vision=True,
                 device="cuda", *, batch_size=64, seq_len=32, dec_len=20, image_size=224, state_dict=None, seed=0,
                 dropout=0.1, dropout_seed=0):
        from . import vit_model as VM
        if vision_model_name not in VIT_NAMES:
            raise ValueError(f"vision_model_name {vision_model_name!r}: this path supports {VIT_NAMES}")
        if language_model_name != "t5-base":
            raise ValueError("language_model_name must be 't5-base' (vit_vqa_model.py:146-147)")
        self.vision_model_name, self.language_model_name = vision_model_name, language_model_name
        self.answer_spaces, self.device = int(answer_spaces), torch.device(device)
        self.batch_size, self.seq_len, self.dec_len, self.image_size = int(batch_size), int(seq_len), int(dec_len), \
            int(image_size)
        self.num_beams, self.max_answer_length = 2, 5                   # :163-164 (beam search is not wired)
        self._cfg = dict(dropout=float(dropout), seed=int(dropout_seed))
        if state_dict is None:
            state_dict = VM.make_state_dict(seed=seed, answer_spaces=self.answer_spaces, image=self.image_size)
        self._build(state_dict)
        self.training = True
        self.vision_model = _VitGroup(self, "vision_model", trainable=False)
        self.lang_model = _VitGroup(self, "lang_model")
        self.fusing_layer = _VitGroup(self, "fusing_layer")
        self.classification_layer = _VitGroup(self, "classification_layer")

    def _build(self, state_dict):
        from . import vit_model as VM
        from .vit_engine import VitVQAEngine
        sd = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
              for k, v in state_dict.items()}
        if "lang_model.shared.weight" in sd:
            for k in VM.TIED:
                sd.setdefault(k, sd["lang_model.shared.weight"])
        missing = [k for k in VM.model_specs(self.answer_spaces, self.image_size) if k not in sd]
        if missing:
            raise KeyError(f"state_dict lacks {len(missing)} reference keys, e.g. {missing[:3]}")
        self.engine = VitVQAEngine(sd, batch=self.batch_size, seq_len=self.seq_len, dec_len=self.dec_len,
                                   image_size=self.image_size, device=self.device, answer_spaces=self.answer_spaces,
                                   **self._cfg)

    def train(self, mode=True):
        self.training = bool(mode)
        self.engine.set_training(self.training)
        return self

    def eval(self):
        return self.train(False)

    def load_items(self, items):
        """The ViT collate's batch dict (dataset_utils/vit_vqa_daquar_dataset.py:168-195)."""
        q = items.get("question_input_ids")
        n = int(q.shape[0]) if q is not None else 0
        if not 1 <= n <= self.batch_size:                 # a short last batch is padded (ResnetVQAModel)
            raise ValueError(f"batch of {n} rows: the model is planned for 1..{self.batch_size} rows")
        want = {"pixel_values": (n, 3, self.image_size, self.image_size),
                "question_input_ids": (n, self.seq_len),
                "decoder_question_input_ids": (n, self.dec_len)}
        for k, shape in want.items():
            if items.get(k) is None or tuple(items[k].shape) != shape:
                raise ValueError(f"{k}: expected shape {shape}")
        self.engine.load_batch(items)

    def forward(self, question_input_ids, decoder_question_input_ids=None, question_attention_masks=None,
                decoder_question_attention_masks=None, annotation_ids=None, pixel_values=None, image_tensors=None,
                answer_input_ids=None, answer_attention_masks=None, question_type_ids=None):
        """vit_vqa_model.py:166-225 -> (log_probs, loss); loss is None without annotation_ids."""
        self.load_items({"question_input_ids": question_input_ids, "question_attention_masks": question_attention_masks,
                         "decoder_question_input_ids": decoder_question_input_ids,
                         "decoder_question_attention_masks": decoder_question_attention_masks,
                         "pixel_values": pixel_values, "annotation_ids": annotation_ids})
        self.engine.forward()
        e = self.engine
        return e.LOGP[:e.rows].clone(), (e.LOSS[0].clone() if annotation_ids is not None else None)

    __call__ = forward

    def generate_answers(self, question_input_ids, decoder_question_input_ids=None, question_attention_masks=None,
                         decoder_question_attention_masks=None, pixel_values=None, image_tensors=None,
                         answer_input_ids=None, answer_attention_masks=None, annotation_ids=None,
                         question_type_ids=None):
        """:229-290 -> (log_probs, loss or None, attention_tensors): the forward, with the frozen
        ViT's attention probabilities (output_attentions=True: a tuple of 12 [B, 12, 197, 197]
        fp32 tensors, written by vqa_attn_probs beside the online-softmax attention)."""
        e = self.engine
        self.load_items({"question_input_ids": question_input_ids, "question_attention_masks": question_attention_masks,
                         "decoder_question_input_ids": decoder_question_input_ids,
                         "decoder_question_attention_masks": decoder_question_attention_masks,
                         "pixel_values": pixel_values, "annotation_ids": annotation_ids})
        atts = e.forward_with_attentions()
        loss = e.LOSS[0].clone() if annotation_ids is not None else None
        return e.LOGP[:e.rows].clone(), loss, tuple(a[:e.rows].clone() for a in atts)

    @staticmethod
    def convert_logits_to_predictions(lm_logits):
        return torch.argmax(torch.exp(lm_logits), dim=1)

    @staticmethod
    def trainer_group_lr(optimizer_kwargs):
        """vit_vqa_trainer.py:300-316: lang_model at lm_encoder_lr, fusing and classifier layers
        at classifier_lr (the vision group gets no gradient)."""
        c = float(optimizer_kwargs.get("classifier_lr", 1e-5))
        return {"lang_model": float(optimizer_kwargs.get("lm_encoder_lr", 5e-3)), "fusing_layer": c,
                "classification_layer": c}

    def state_dict(self):
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in self.engine.state_dict().items()}

    def load_state_dict(self, state_dict, strict=True):
        sd = dict(state_dict)
        if not strict:
            cur = self.state_dict()
            cur.update({k: v for k, v in sd.items() if k in cur})
            sd = cur
        training = self.training
        self._build(sd)
        if getattr(self, "_optim_cfg", None):
            self.engine.configure_optimizer(**self._optim_cfg)
        self.train(training)

    def configure_optimizer(self, **kw):
        self._optim_cfg = dict(getattr(self, "_optim_cfg", None) or {}, **kw)
        self.engine.configure_optimizer(**kw)

    def parameters_count(self):
        return self.engine.lay.num_params
