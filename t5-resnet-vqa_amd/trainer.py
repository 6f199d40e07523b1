"""`VQATrainer` — the hot loop of the reference trainer
(trainer/faster_rcnn_vqa_trainer.py:231-406, ≡ cross_attention_vqa_trainer.py)
over the MI355X engine.

Mirrors:
  _init_optimizer   AdamW(amsgrad) param groups: lang_model `lm_encoder_lr`,
                    scaler / SGA / pooler 5e-4 (hard-coded :244-261),
                    classifier `classifier_lr`; `kwargs` (weight_decay,
                    amsgrad=True, betas, eps)                     :231-267
  _init_lr_scheduler linear warm-up/decay, warmup = min(T//10 if -1,
                    max_warmup_steps)                            :279-287
  train_one_step    zero_grad -> forward -> backward -> clip_grad_norm_
                    (gradient_clipping) -> step -> sched; returns
                    (loss.item(), log-probs)                      :391-406
  train_one_epoch   the batch loop with the "secs/batch" timing log, averaged
                    every 10% of the epoch                        :314-360
  valid_one_step    eval-mode forward (dropout off), no update    :408-430
  valid_one_epoch   the validation loop: average loss and exp/argmax
                    predictions vs targets (WUPS needs nltk's WordNet, not
                    on this path: accuracy is reported instead)   :408-480
  convert_logits_to_predictions  argmax(exp(log-probs))            :484-488
The whole train step is one replayed hipGraph; the only host sync per step is
the `loss.item()` the reference API returns (pass sync=False to skip it).

Data parallel (the reference trains on one device,
faster_rcnn_vqa_trainer.py:61-62): with torch.distributed initialised and more
than one rank in `process_group` (or data_parallel=True), each rank trains on its
own batch and `train_one_step` runs `dp.DataParallelStep` -- the gradient buckets
all-reduced over RCCL while the backward runs, the embedding rows all-gathered --
so every rank applies the same update.  The returned loss / log-probs are the
rank's own (its batch), the clip norm is the global one.
"""
from __future__ import annotations

import inspect
import time

import numpy as np
import torch

from . import dp
from . import synthetic as S
from .model import ResnetVQAModel

HARD_CODED_LR = 5e-4          # faster_rcnn_vqa_trainer.py:244-261


class VQATrainer:
    def __init__(self, model: ResnetVQAModel, optimizer_kwargs: dict, lr_scheduler_kwargs: dict,
                 num_training_steps: int, gradient_clipping=1.0, use_graph=True, logger=print,
                 data_parallel=None, process_group=None, bucket_mb=24, shard_optimizer=False):
        if optimizer_kwargs.get("type", "AdamW") != "AdamW":
            raise ValueError("only AdamW is on this path (vit_daquar_config.json:41)")
        kw = dict(optimizer_kwargs.get("kwargs", {}))
        if not kw.get("amsgrad", True):
            raise ValueError("the reference trains with amsgrad=True; plain AdamW is not planned here")
        self.model = model
        self.logger = logger
        if data_parallel is None:
            data_parallel = (torch.distributed.is_available() and torch.distributed.is_initialized()
                             and torch.distributed.get_world_size(process_group) > 1)
        self.data_parallel = bool(data_parallel)
        if self.data_parallel and not hasattr(model.engine, "ready_marks"):
            raise ValueError("data parallel training is planned for ResnetVQAModel (BASELINE configs[2]); "
                             "the ViT configuration (configs[3]) is a single-GPU one")
        self.process_group, self.bucket_mb = process_group, int(bucket_mb)
        self.shard_optimizer = bool(shard_optimizer)      # DP: reduce-scatter + sharded AdamW + all-gather
        self._dp = None
        groups = dp.dp_t5_dw_groups(model.engine.nl) if self.data_parallel else None
        if self.data_parallel and model.engine.t5_dw_groups != list(groups):
            # DP layout: T5 weight gradients in groups that let the buckets become final (and be
            # all-reduced) while the backward runs; rebuilt before the optimizer is configured
            model._build(model.state_dict(), t5_dw_group=groups)
        if self.data_parallel:
            # the NLL mean over the GLOBAL batch: unequal rows per rank, or none on a rank
            # (engine.use_global_rows; the DP step all-reduces the valid-row count each step)
            model.engine.use_global_rows(torch.distributed.get_world_size(process_group))
        self.num_training_steps = int(num_training_steps)
        warm = lr_scheduler_kwargs.get("num_warmup_steps", -1)
        warm = self.num_training_steps // 10 if warm == -1 else int(warm)
        warm = min(warm, int(lr_scheduler_kwargs.get("max_warmup_steps", warm)))
        self.num_warmup_steps = warm
        if hasattr(model, "trainer_group_lr"):             # VitVQAModel: the ViT trainer's groups
            group_lr = model.trainer_group_lr(optimizer_kwargs)
        else:
            group_lr = {"lang_model": float(optimizer_kwargs.get("lm_encoder_lr", 5e-3)),
                        "scaler": HARD_CODED_LR, "sga_modules": HARD_CODED_LR, "attention_pooler": HARD_CODED_LR,
                        "classification_layer": float(optimizer_kwargs.get("classifier_lr", 1e-5))}
        self.group_lr = dict(group_lr)
        self.vision_lr = float(optimizer_kwargs.get("vision_lr", 8e-3))
        self.adam_kwargs = {"betas": tuple(kw.get("betas", (0.9, 0.999))), "eps": float(kw.get("eps", 1e-8)),
                            "weight_decay": float(kw.get("weight_decay", 1e-2)), "amsgrad": True}
        model.configure_optimizer(group_lr=group_lr, warmup=warm, total=self.num_training_steps,
                                         max_norm=float(gradient_clipping or 0.0),
                                         weight_decay=float(kw.get("weight_decay", 1e-2)),
                                         betas=tuple(kw.get("betas", (0.9, 0.999))), eps=float(kw.get("eps", 1e-8)))
        self.use_graph = use_graph
        self.total_training_time = 0.0

    # ------------------------------------------------------------------ steps
    def train_one_step(self, data_items, sync=True):
        """Returns (loss.item(), log_probs) like the reference (:391-406)."""
        m = self.model
        if not m.training:
            m.train()
        m.load_items(data_items)
        e = m.engine
        if self.data_parallel:
            if self._dp is None:
                self._dp = dp.DataParallelStep(e, group=self.process_group, bucket_mb=self.bucket_mb,
                                               use_graph=self.use_graph, shard_optimizer=self.shard_optimizer)
            self._dp.step()
        else:
            if self.use_graph and e.graph is None:
                e.capture()
            e.train_step()
        loss = float(e.LOSS.item()) if sync else e.LOSS[0]
        return loss, e.LOGP[:e.rows]

    @torch.no_grad()
    def valid_one_step(self, data_items):
        """Eval-mode forward (dropout off); returns (loss.item() or None, log_probs)."""
        m = self.model
        was = m.training
        m.eval()
        names = inspect.signature(m.forward).parameters
        lp, loss = m(**{k: v for k, v in data_items.items() if k in names})
        m.train(was)
        return (float(loss) if loss is not None else None), lp

    def train_one_epoch(self, batches, epoch=0):
        """The reference's epoch loop without the WUPS/wandb tail: returns {avg_loss,
        secs_per_batch, steps, predictions, targets}; predictions are the exp/argmax
        answers of every step (:336-343), kept on the device until the epoch ends (one
        host copy per epoch instead of a .tolist() sync per step)."""
        total, n, t_epoch = 0.0, 0, 0.0
        window = max(1, len(batches) // 10) if hasattr(batches, "__len__") else 10
        win_loss, win_time = 0.0, 0.0
        preds, targets = [], []
        for i, data_items in enumerate(batches):
            t0 = time.time()
            loss, lp = self.train_one_step(data_items)
            dt = time.time() - t0
            preds.append(self.convert_logits_to_predictions(lp))
            targets.append(torch.as_tensor(data_items["annotation_ids"]).reshape(-1))
            total += loss
            n += 1
            t_epoch += dt
            win_loss += loss
            win_time += dt
            if (i + 1) % window == 0 and self.logger:
                self.logger(f"Epoch {epoch} - iter {i}/{n} - total loss {win_loss / window:.4f}"
                            f" - secs/batch {win_time / window:.4f}")
                win_loss, win_time = 0.0, 0.0
        self.total_training_time += t_epoch
        return {"avg_loss": total / max(1, n), "secs_per_batch": t_epoch / max(1, n), "steps": n,
                "predictions": torch.cat(preds).tolist() if preds else [],
                "targets": torch.cat([t.cpu() for t in targets]).tolist() if targets else []}

    def valid_one_epoch(self, batches):
        """faster_rcnn_vqa_trainer.py:408-480 without WUPS / checkpoint callbacks: eval mode,
        no update; returns {avg_loss, predictions, targets, accuracy}."""
        total, n = 0.0, 0
        preds, targets = [], []
        for data_items in batches:
            loss, lp = self.valid_one_step(data_items)
            total += loss if loss is not None else 0.0
            n += 1
            preds.append(self.convert_logits_to_predictions(lp))
            targets.append(torch.as_tensor(data_items["annotation_ids"]).reshape(-1))
        p = torch.cat(preds).cpu() if preds else torch.zeros(0, dtype=torch.long)
        t = torch.cat([x.cpu() for x in targets]) if targets else torch.zeros(0, dtype=torch.long)
        acc = float((p == t).float().mean()) if len(t) else 0.0
        return {"avg_loss": total / max(1, n), "predictions": p.tolist(), "targets": t.tolist(), "accuracy": acc}

    # ------------------------------------------------------------------ optimizer checkpoints
    # The reference saves {'epoch', 'scheduler', 'optimizer'} with torch.save (callbacks.py:118-125)
    # and reloads the optimizer from state_dict_checkpoint.pt (faster_rcnn_vqa_trainer.py:269-277).
    # Here the same dict, with the optimizer and scheduler state in torch's own AdamW / LambdaLR
    # state_dict formats over the reference's parameter order (its six groups, :231-263), so a
    # checkpoint written here loads into the reference's optimizer and back.
    def _param_groups(self):
        m = self.model
        if hasattr(m, "trainer_group_lr"):
            # VitVQAModel: the ViT trainer's four groups (vit_vqa_trainer.py:298-316), parameters in
            # module order with the tied embedding once (lang_model.parameters() de-duplicates it)
            from . import vit_model as VM
            specs = [k for k in VM.model_specs(m.answer_spaces, m.image_size) if k not in VM.TIED]
            names = [("vision_model", "Vision Model", self.vision_lr),
                     ("lang_model", "Language Model", self.group_lr["lang_model"]),
                     ("fusing_layer", "Fusion Layer", self.group_lr["fusing_layer"]),
                     ("classification_layer", "Classifier Layer", self.group_lr["classification_layer"])]
            return [(label, lr, [k for k in specs if k.split(".", 1)[0] == top]) for top, label, lr in names]
        scaler = "downscale_layer" if m.vision_model_name == "resnet50" else "upscale_layer"
        names = [("vision_model", "Vision Model"), ("lang_model", "Language Model"),
                 (scaler, "DownScaler Layer" if scaler == "downscale_layer" else "UpScaler Layer"),
                 ("sga_modules", "Self-Guided Attention Module"), ("attention_pooler", "Attention Pooler"),
                 ("classification_layer", "Classifier Layer")]
        specs = S.model_specs(m.vision_model_name, m.answer_spaces, m.num_attention_blocks, m.language_model_name)
        params = [k for k in specs if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
        groups = []
        for top, label in names:
            keys = [k for k in params if k.split(".", 1)[0] == top]
            lr = self.vision_lr if top == "vision_model" else \
                self.group_lr.get("scaler" if top == scaler else top, HARD_CODED_LR)
            groups.append((label, lr, keys))
        return groups

    def optimizer_state_dict(self):
        """torch.optim.AdamW(amsgrad=True).state_dict() of the reference's parameter groups.
        With the sharded DP optimizer this is a COLLECTIVE (every rank's chunk moments are
        all-gathered first): call it on every rank, as save_state_dict_checkpoint does."""
        self._param_groups()                               # fails early for models without this state
        e = self.model.engine
        if self._dp is not None:
            self._dp.sync_optimizer_state()                # sharded: every chunk's moments on this rank
        m, v, vm, step, _ = e.optimizer_state()
        state, pgroups, idx = {}, [], 0
        for label, lr, keys in self._param_groups():
            ids = []
            for k in keys:
                if k in m and step > 0:                     # the frozen ResNet / unused scaler: no state
                    state[idx] = {"step": torch.tensor(step), "exp_avg": torch.from_numpy(m[k]),
                                  "exp_avg_sq": torch.from_numpy(v[k]), "max_exp_avg_sq": torch.from_numpy(vm[k])}
                ids.append(idx)
                idx += 1
            pgroups.append({"lr": lr * self._lr_factor(step), "initial_lr": lr, "model_name": label,
                            "betas": self.adam_kwargs["betas"], "eps": self.adam_kwargs["eps"],
                            "weight_decay": self.adam_kwargs["weight_decay"], "amsgrad": True, "maximize": False,
                            "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                            "decoupled_weight_decay": True, "params": ids})
        return {"state": state, "param_groups": pgroups}

    def _lr_factor(self, step):
        """get_linear_schedule_with_warmup's multiplier at `step` (TF/optimization.py:101-107)."""
        w, t = self.num_warmup_steps, self.num_training_steps
        return step / max(1, w) if step < w else max(0.0, (t - step) / max(1, t - w))

    def scheduler_state_dict(self):
        """LambdaLR.state_dict() of the reference's schedule (last_epoch = optimizer steps taken)."""
        step = int(self.model.engine.opt_state[0].item())
        base = [lr for _, lr, _ in self._param_groups()]
        return {"base_lrs": base, "last_epoch": step, "_step_count": step + 1, "_is_initial": False,
                "_get_lr_called_within_step": False, "_last_lr": [b * self._lr_factor(step) for b in base],
                "lr_lambdas": [None] * len(base)}

    def save_state_dict_checkpoint(self, path, epoch, write=None):
        """callbacks.py:118-125: torch.save({'epoch', 'scheduler', 'optimizer'}) (+ this engine's
        dropout RNG counter, so a resumed run draws the same masks).

        Data parallel: call it on EVERY rank (the sharded optimizer gathers the moments with
        collectives; a save guarded by `if rank == 0` would leave rank 0 waiting for the others).
        Only the ranks with `write` true write the file -- by default rank 0 of the process group
        when training data-parallel, every caller otherwise."""
        e = self.model.engine
        opt = self.optimizer_state_dict()                  # collective under the sharded optimizer
        if write is None:
            write = not self.data_parallel or torch.distributed.get_rank(self.process_group) == 0
        if not write:
            return
        rng = e.optimizer_state()[4]
        torch.save({"epoch": int(epoch), "scheduler": self.scheduler_state_dict(),
                    "optimizer": opt, "vqa_rng": torch.from_numpy(rng.astype(np.int64))}, path)

    def load_state_dict_checkpoint(self, path):
        """faster_rcnn_vqa_trainer.py:269-277: resume the optimizer (and the schedule position) from
        a checkpoint in the format above; loaded with weights_only=True.  Returns the epoch."""
        ck = torch.load(path, weights_only=True)
        opt = ck["optimizer"]
        groups = self._param_groups()
        if len(opt["param_groups"]) != len(groups):
            raise ValueError("optimizer checkpoint has another parameter-group structure")
        m, v, vm, step = {}, {}, {}, 0.0
        for (label, _, keys), pg in zip(groups, opt["param_groups"]):
            if len(pg["params"]) != len(keys):
                raise ValueError(f"optimizer checkpoint group {label!r}: {len(pg['params'])} parameters, expected "
                                 f"{len(keys)}")
            for k, i in zip(keys, pg["params"]):
                st = opt["state"].get(i)
                if st is None:
                    continue
                m[k], v[k], vm[k] = (st[n].numpy() for n in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"))
                step = float(st["step"])
        sched = ck.get("scheduler", {})
        if "last_epoch" in sched and not m:
            step = float(sched["last_epoch"])
        rng = ck["vqa_rng"].numpy() if "vqa_rng" in ck else None
        self.model.engine.load_optimizer_state(m, v, vm, step, rng)
        return int(ck.get("epoch", 0))

    @staticmethod
    def convert_logits_to_predictions(lm_logits):
        """:484-488 -- argmax over exp(log-probs)."""
        return torch.argmax(torch.exp(lm_logits), dim=1)

    def grad_norm(self):
        """clip_grad_norm_'s returned total norm of the last step."""
        return self.model.engine.last_grad_norm()
