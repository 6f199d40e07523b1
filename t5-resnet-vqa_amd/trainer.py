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

import torch

from . import dp
from .model import ResnetVQAModel

HARD_CODED_LR = 5e-4          # faster_rcnn_vqa_trainer.py:244-261


class VQATrainer:
    def __init__(self, model: ResnetVQAModel, optimizer_kwargs: dict, lr_scheduler_kwargs: dict,
                 num_training_steps: int, gradient_clipping=1.0, use_graph=True, logger=print,
                 data_parallel=None, process_group=None, bucket_mb=24):
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
        self._dp = None
        groups = dp.dp_t5_dw_groups(model.engine.nl) if self.data_parallel else None
        if self.data_parallel and model.engine.t5_dw_groups != list(groups):
            # DP layout: T5 weight gradients in groups that let the buckets become final (and be
            # all-reduced) while the backward runs; rebuilt before the optimizer is configured
            model._build(model.state_dict(), t5_dw_group=groups)
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
                                               use_graph=self.use_graph)
            self._dp.step()
        else:
            if self.use_graph and e.graph is None:
                e.capture()
            e.train_step()
        loss = float(e.LOSS.item()) if sync else e.LOSS[0]
        return loss, e.LOGP

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

    @staticmethod
    def convert_logits_to_predictions(lm_logits):
        """:484-488 -- argmax over exp(log-probs)."""
        return torch.argmax(torch.exp(lm_logits), dim=1)

    def grad_norm(self):
        """clip_grad_norm_'s returned total norm of the last step."""
        return self.model.engine.last_grad_norm()
