"""``training_structures/dino_train.py`` of the reference on the MI355X engine.

  pretrain_dino                 dino_train.py:104-186   the training_structures DINO loop
                                (BASELINE config 1's path): AdamW(lr) with torch's default
                                weight_decay 0.01, per batch zero_grad -> forward -> dino_loss
                                -> backward -> step -> update_teacher (EMA AFTER the step),
                                per-epoch CSV log and best-loss checkpoint
  dino_loss / unimodal_dino_loss the loss callables pretrain_dino takes (the Lightning modules'
                                dino_loss, dino.py:822-854 / 1596-1635, as free functions)
  train_downstream, train_knn_classifier, feature_extraction_loop,
  compute_classification_metrics, compute_accuracies    -> avdino.downstream (re-exported)

Deviation, documented: the reference's pretrain_dino unpacks ``student_out, teacher_out =
model(batch)``, while its current models return three values (dino.py:727, 1398) and would
raise there; this loop takes the first two.  ``align=True`` needs a model exposing
``student.loss_align`` (the reference's archived alignment encoders), none of which is on the
hot path.
"""
import csv
import json
import os
from datetime import datetime

import torch

from .downstream import (compute_accuracies, compute_classification_metrics,  # noqa: F401
                         feature_extraction_loop, train_downstream, train_knn_classifier)
from .models import FlatAdam, _DinoLossFn


def dino_loss(student_outputs, teacher_outputs, alignment_loss=None, tau_s=0.1, tau_t=0.04):
    """MultiModalDINOLightning.dino_loss (dino.py:822-854) as a free function: fused HIP
    kernel, differentiable w.r.t. student_outputs."""
    loss = _DinoLossFn.apply(student_outputs, teacher_outputs, tau_s, tau_t, False)
    return loss if alignment_loss is None else loss + alignment_loss


def unimodal_dino_loss(student_outputs, teacher_outputs, tau_s=0.1, tau_t=0.04):
    """UniModalDINOLightning.dino_loss (dino.py:1596-1635): the teacher additionally centred
    by its per-view batch mean."""
    return _DinoLossFn.apply(student_outputs, teacher_outputs, tau_s, tau_t, True)


def _stamp(path, stamp):
    return path.replace(".pt", f"_{stamp}.pt") if path.endswith(".pt") else \
        path.replace(".csv", f"_{stamp}.csv")


def pretrain_dino(model, trainloader, dino_loss, align=False, num_epochs=100, learning_rate=0.0001,
                  save_path="pretrained_dino.pt", log_path="pretrain_log.csv", write_logs=True):
    """dino_train.py:104-186 -> the trained model (``model.epoch_losses`` holds the per-epoch
    means, ``model.step_losses`` the per-step losses as one device tensor per epoch)."""
    if align:
        raise NotImplementedError("align=True needs an alignment encoder (not on the hot path)")
    opt = FlatAdam(model.trainable_arenas(), lr=learning_rate, weight_decay=0.01, decoupled=True)
    stamp = datetime.now().strftime("%Y-%m-%d %H-%M-%S")
    if write_logs:
        for path in (save_path, log_path):
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
        save_path, log_path = _stamp(save_path, stamp), _stamp(log_path, stamp)
        info = {"start_time": stamp, "learning_rate": learning_rate,
                "batch_size": getattr(trainloader, "batch_size", None), "epochs": num_epochs,
                "model_name": "MultiModalDINO"}
        with open(log_path, "w", newline="") as f:
            csv.writer(f).writerow(["epoch", "train_loss", f"# {json.dumps(info)}"])
    best = float("inf")
    model.epoch_losses, model.step_losses = [], []
    for epoch in range(num_epochs):
        model.train()
        losses = []
        for batch in trainloader:
            opt.zero_grad()
            student_out, teacher_out = model(tuple(batch[:4]))[:2]
            loss = dino_loss(student_out, teacher_out, tau_s=0.1, tau_t=0.04)
            loss.backward()
            opt.step()
            model.update_teacher()       # EMA of the post-step student
            losses.append(loss.detach().reshape(1))
        step = torch.cat(losses)
        avg = step.mean().item()
        model.step_losses.append(step)
        model.epoch_losses.append(avg)
        if write_logs:
            with open(log_path, "a", newline="") as f:
                csv.writer(f).writerow([epoch + 1, avg])
        if avg < best:
            best = avg
            if write_logs:
                torch.save({"epoch": epoch, "model_state_dict": {k: v.detach().cpu() for k, v in
                                                                 model.state_dict().items()},
                            "optimizer_state_dict": opt.state_dict(), "loss": best}, save_path)
    return model
