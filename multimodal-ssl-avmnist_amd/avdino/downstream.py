"""Downstream evaluation of a trained DINO student: the reference's
``training_structures/dino_train.py`` functions and ``models/dino.py``'s downstream modules,
on libavdino kernels with every tensor on the device.

  FeatureExtractor              models/dino.py:1816-1850  frozen deep copy, eval mode
  DownstreamClassifier          models/dino.py:1764-1814  copy + Linear(D,128)-ReLU-Linear(128,10)
  feature_extraction_loop       dino_train.py:331-347
  KNeighborsClassifier          sklearn's (n_neighbors=5; brute force, euclidean, uniform
                                weights): distance GEMM (avd_gemm, exact-f32 MFMA) + per-row
                                top-k and vote (avd_knn_select)
  train_knn_classifier          dino_train.py:349-369
  train_downstream              dino_train.py:188-329  10 epochs AdamW(lr 1e-3, wd 0.01) +
                                CosineAnnealingLR(T_max=epochs), best-val-accuracy checkpoint,
                                test evaluation
  compute_classification_metrics dino_train.py:47-102
  compute_accuracies            run_dino.py:481-501

Semantics kept from the reference: the encoder is a deep copy of ``pretrained.student`` (the
trained model is never touched); the classifier's training epochs run the copy in TRAIN mode
(``model.train()`` reaches the copy: batch-stat BatchNorm whose running statistics update the
copy, fusion dropout active) and evaluation in EVAL mode; the best epoch is the first with the
highest validation accuracy (strict ``>``), and its classifier AND the copy's running
statistics (``model.state_dict()``) are what the test set sees.  The reference runs under fp16
autocast + GradScaler on CUDA; here the classifier is fp32 and the encoder copy runs in the
pretrained model's activation dtype.
"""
import csv
import json
import os
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .probe import LinearProbe
from .trainer import cosine_lr


def _source(pretrained_model, is_dino_based=True):
    """(ParamStore, kind, D, E, act dtype, fusion dropout) of a DINO model's student."""
    if not is_dino_based:
        raise NotImplementedError("downstream evaluation of non-DINO encoders (SimCLR / InfoNCE "
                                  "notebooks) is outside the MI355X hot path")
    m = pretrained_model.model if hasattr(pretrained_model, "configure_optimizers") else pretrained_model
    enc = m.student_spec
    kind = getattr(enc, "kind", None) or enc.arch
    act = torch.bfloat16 if str(getattr(m, "precision", "bf16")) in ("bf16", "16-mixed", "bf16-mixed") \
        else torch.float32
    return (m.store, kind, m.output_dim, getattr(m, "encoder_output_dim", None), act,
            getattr(m.hp, "fusion_dropout", 0.3))


def _as_batch(batch, device):
    images, audios, labels = batch[0], batch[1], batch[2]
    return (images.to(device, non_blocking=True).float(), audios.to(device, non_blocking=True).float(),
            labels.to(device, non_blocking=True).long())


class FeatureExtractor(nn.Module):
    """Frozen deep copy of ``pretrained_model.student``; ``forward(images, spectrograms)`` ->
    eval-mode features [B, output_dim] (f32, on the device)."""

    def __init__(self, pretrained_model, is_dino_based=True):
        super().__init__()
        store, kind, D, E, act, fd = _source(pretrained_model, is_dino_based)
        self.probe = LinearProbe(store, kind, D, E, act_dtype=act, fusion_dropout=fd)
        self.output_dim = D
        self.modality = getattr(self.probe, "modality", None)
        self.is_unimodal = self.modality is not None

    def forward(self, images, spectrograms=None):
        with torch.no_grad():
            N = (images if images is not None else spectrograms).shape[0]
            feat = self.probe._features(images, spectrograms, False)
            return feat.view(N, -1).clone()


class DownstreamClassifier(nn.Module):
    """Frozen student copy + classifier Linear(D, 128) - ReLU - Linear(128, num_classes).
    ``train()`` / ``eval()`` switch the copy's BatchNorm / dropout mode as in the reference;
    ``forward`` returns logits [B, num_classes]; ``train_step`` is one AdamW step."""

    def __init__(self, pretrained_model, num_classes=10, trainable_encoder=False, is_dino_based=True,
                 lr=1e-3, weight_decay=0.01, seed=0, classifier_state=None):
        super().__init__()
        if trainable_encoder:
            raise NotImplementedError("fine-tuning the encoder is not on the reference's path")
        if num_classes != 10:
            raise NotImplementedError("AVMNIST has 10 classes")
        store, kind, D, E, act, fd = _source(pretrained_model, is_dino_based)
        self.probe = LinearProbe(store, kind, D, E, lr=lr, weight_decay=weight_decay, act_dtype=act,
                                 fusion_dropout=fd, seed=seed, classifier_state=classifier_state)
        self.output_dim = D
        self.modality = getattr(self.probe, "modality", None)
        self.is_unimodal = self.modality is not None

    @property
    def lr(self):
        return self.probe.lr

    @lr.setter
    def lr(self, v):
        self.probe.lr = v

    def forward(self, images, spectrograms=None):
        with torch.no_grad():
            N = (images if images is not None else spectrograms).shape[0]
            feat = self.probe._features(images, spectrograms, self.training)
            _, _, logits = self.probe._logits(feat, N)
            return logits.view(N, -1).clone()

    def train_step(self, images, spectrograms, labels, loss_out):
        """One optimizer step on the classifier (the copy in train mode)."""
        self.probe.train_batch(images, spectrograms, labels, loss_out)

    # the reference's ``model.state_dict()`` (classifier + the copy's BN running statistics)
    def snapshot(self):
        p = self.probe
        p.store.flush_nbt()
        return {"classifier": p.cls.student.clone(), "buffers": p.store.buf_arena.clone(),
                "counters": p.store.nbt_arena.clone(), "adam": (p.cls.adam_m.clone(), p.cls.adam_v.clone(), p.t)}

    def restore(self, snap):
        p = self.probe
        p.cls.student.copy_(snap["classifier"])
        p.store.buf_arena.copy_(snap["buffers"])
        p.store.nbt_arena.copy_(snap["counters"])

    def classifier_state_dict(self):
        return {k: v.detach().clone() for k, v in self.probe.cls.state_dict().items()}


# ---------------------------------------------------------------------------- kNN
class KNeighborsClassifier:
    """sklearn.neighbors.KNeighborsClassifier(n_neighbors) with algorithm='brute',
    metric='euclidean', weights='uniform' (what 'auto' picks for 256-dim features), on the
    device: candidates by |x_j|^2 - 2 q.x_j from one exact-f32 MFMA GEMM per query chunk, the
    best 16 re-ranked by their direct distance, top-k (ties to the smaller train index) and
    majority vote (ties to the smallest class)."""

    def __init__(self, n_neighbors=5, query_chunk=4096):
        self.n_neighbors = n_neighbors
        self.query_chunk = query_chunk

    def fit(self, X, y):
        X = torch.as_tensor(X)
        dev = X.device if X.is_cuda else torch.device("cuda")
        self._X = X.to(dev, torch.float32).contiguous()
        y = torch.as_tensor(y).to(dev).long()
        self.classes_ = torch.unique(y)              # sorted, like sklearn's classes_
        self._y = torch.searchsorted(self.classes_, y).contiguous()
        N, D = self._X.shape
        if len(self.classes_) > 64 or not (1 <= self.n_neighbors <= min(16, N)):
            raise ValueError("device kNN: n_neighbors <= 16 (and <= n_samples), <= 64 classes")
        self._xnorm = torch.empty(N, device=dev)
        ops.row_sqnorm(self._X, N, D, self._xnorm)
        return self

    def _run(self, Q, want_nbr):
        Q = torch.as_tensor(Q).to(self._X.device, torch.float32).contiguous()
        M, D = Q.shape
        N = self._X.shape[0]
        K = self.n_neighbors
        pred = torch.empty(M, dtype=torch.int64, device=Q.device)
        nbr = torch.empty(M, K, dtype=torch.int64, device=Q.device) if want_nbr else None
        for a in range(0, M, self.query_chunk):
            m = min(self.query_chunk, M - a)
            S = torch.empty(m, N, device=Q.device)
            # S = -2 Q X^T  (A = Q rows [a, a+m), B = X^T: b[k, n] = X[n, k])
            ops.gemm(m, N, D, Q, D, 1, self._X, 1, D, S, N, alpha=-2.0, a_off=a * D,
                     mode=ops.GEMM_F32_MFMA)
            ops.knn_select(S, N, self._xnorm, m, N, K, self._y, len(self.classes_),
                           None if nbr is None else nbr[a:a + m], pred[a:a + m],
                           Q=Q[a:a + m], X=self._X, D=D)
        return pred, nbr

    def predict(self, Q):
        pred, _ = self._run(Q, False)
        return self.classes_[pred]

    def kneighbors(self, Q, n_neighbors=None, return_distance=False):
        if n_neighbors not in (None, self.n_neighbors):
            raise NotImplementedError("n_neighbors is fixed at construction")
        _, nbr = self._run(Q, True)
        if return_distance:
            Qd = torch.as_tensor(Q).to(self._X.device, torch.float32)
            d = (Qd[:, None, :] - self._X[nbr]).norm(dim=2)
            return d, nbr
        return nbr

    def score(self, Q, y):
        y = torch.as_tensor(y).to(self._X.device).long()
        return (self.predict(Q) == y).float().mean().item()


def feature_extraction_loop(device, model, dataloader):
    """(features [N, D], labels [N]) on the device (dino_train.py:331-347 returns numpy)."""
    feats, labels = [], []
    for batch in dataloader:
        images, audios, lab = _as_batch(batch, device)
        feats.append(model(images, audios))
        labels.append(lab)
    return torch.cat(feats), torch.cat(labels)


def train_knn_classifier(pretrained_dino, train_dataloader, test_dataloader, n_neighbors=5,
                         device="cuda", is_dino_based=True):
    """dino_train.py:349-369 -> (knn, accuracy %)."""
    fe = FeatureExtractor(pretrained_dino, is_dino_based=is_dino_based)
    trf, trl = feature_extraction_loop(device, fe, train_dataloader)
    tef, tel = feature_extraction_loop(device, fe, test_dataloader)
    knn = KNeighborsClassifier(n_neighbors=n_neighbors).fit(trf, trl)
    accuracy = 100 * knn.score(tef, tel)
    print(f"KNN Accuracy (k={n_neighbors}): {accuracy:.4f}%")
    return knn, accuracy


# ---------------------------------------------------------------------------- MLP probe
def _evaluate(model, dataloader, device):
    """evaluate() of train_downstream (dino_train.py:231-263): eval mode; mean of per-batch
    CE, accuracy %, labels, predictions, softmax probabilities (device tensors)."""
    model.eval()
    losses, labels, preds, probs = [], [], [], []
    for batch in dataloader:
        images, audios, lab = _as_batch(batch, device)
        N = lab.shape[0]
        logits = model(images, audios)
        p = model.probe
        parts = p.ws.get("d.parts", N)
        ops.softmax_xent(logits.reshape(-1), 10, N, 10, lab, 0, False, False, 1.0 / N, parts, None,
                         10, False)
        l1 = torch.empty(1, device=logits.device)
        ops.sum_to(parts, N, 1.0 / N, l1)
        idx = torch.empty(N, dtype=torch.int64, device=logits.device)
        ops.argmax_rows(logits.reshape(-1), 10, N, 10, idx)
        losses.append(l1)
        labels.append(lab)
        preds.append(idx)
        probs.append(torch.softmax(logits, 1))
    labels, preds = torch.cat(labels), torch.cat(preds)
    acc = 100.0 * (preds == labels).sum().item() / labels.numel()
    return torch.cat(losses).mean().item(), acc, labels, preds, torch.cat(probs)


def _stamp(path, stamp):
    root, ext = os.path.splitext(path)
    return f"{root}_{stamp}{ext}"


def train_downstream(pretrained_model, trainloader, validloader, testloader, num_epochs=10,
                     device="cuda", learning_rate=0.001, save_path="downstream_model.pt",
                     train_log_path="downstream_train_log.csv",
                     test_log_path="downstream_test_log.csv", is_dino_based=True, seed=0,
                     classifier_state=None, write_logs=True):
    """dino_train.py:188-329.  Returns the DownstreamClassifier holding the best epoch's state
    (its ``history`` has the per-epoch train/val losses and accuracies, ``test_accuracy`` the
    test result)."""
    model = DownstreamClassifier(pretrained_model, is_dino_based=is_dino_based, lr=learning_rate,
                                 weight_decay=0.01, seed=seed, classifier_state=classifier_state)
    stamp = datetime.now().strftime("%Y-%m-%d %H-%M-%S")
    if write_logs:
        for path in (save_path, train_log_path, test_log_path):
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
        save_path, train_log_path, test_log_path = (_stamp(p, stamp) for p in
                                                    (save_path, train_log_path, test_log_path))
        info = {"start_time": stamp, "learning_rate": learning_rate, "epochs": num_epochs,
                "criterion": "CrossEntropyLoss", "optimizer": "AdamW",
                "scheduler": "CosineAnnealingLR", "model_name": "DinoClassifier"}
        with open(train_log_path, "w", newline="") as f:
            csv.writer(f).writerow(["epoch", "train_loss", "val_loss", "val_accuracy", f"# {json.dumps(info)}"])
    best_acc, best = 0.0, None
    history = []
    for epoch in range(num_epochs):
        model.train()
        # CosineAnnealingLR(T_max=num_epochs) stepped once per epoch, in closed form
        model.lr = cosine_lr(learning_rate, epoch, num_epochs)
        # the loader is streamed (one batch alive at a time); the per-batch losses stay in one
        # device buffer, sized from len(loader) when it has one (no host sync inside the epoch)
        n = len(trainloader) if hasattr(trainloader, "__len__") else 0
        losses = torch.empty(max(n, 1), device=device)
        i = 0
        for batch in trainloader:
            if i >= losses.numel():
                losses = torch.cat([losses, torch.empty(losses.numel(), device=device)])
            images, audios, lab = _as_batch(batch, device)
            model.train_step(images, audios, lab, losses[i:i + 1])
            i += 1
        train_loss = losses[:i].mean().item()
        val_loss, val_acc, *_ = _evaluate(model, validloader, device)
        history.append({"epoch": epoch + 1, "train_loss": train_loss, "val_loss": val_loss,
                        "val_accuracy": val_acc, "train_losses": losses[:i].cpu().numpy()})
        if write_logs:
            with open(train_log_path, "a", newline="") as f:
                csv.writer(f).writerow([epoch + 1, train_loss, val_loss, val_acc])
        print(f"Epoch {epoch + 1}: Train Loss: {train_loss:.4f}, Val Loss: {val_loss:.4f}, "
              f"Val Acc: {val_acc:.2f}%")
        if val_acc > best_acc:
            best_acc, best = val_acc, model.snapshot()
            best["epoch"] = epoch
            if write_logs:
                torch.save({"epoch": epoch, "model_state_dict": model.classifier_state_dict(),
                            "accuracy": best_acc}, save_path)
    if best is not None:
        model.restore(best)
    model.best_epoch = None if best is None else best["epoch"]
    test_loss, test_acc, labels, preds, probs = _evaluate(model, testloader, device)
    if write_logs:
        with open(test_log_path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["true_label", "predicted_label", "probabilities"])
            for lab, pr, pb in zip(labels.cpu().numpy(), preds.cpu().numpy(), probs.cpu().numpy()):
                w.writerow([lab, pr, ",".join(map(str, pb))])
    print(f"\nTest Accuracy: {test_acc:.2f}%")
    model.history, model.test_accuracy, model.test_loss = history, test_acc, test_loss
    return model


def compute_classification_metrics(model, dataloader, device="cuda"):
    """dino_train.py:47-102: confusion matrix (+ row-normalised), accuracy %, per-class
    accuracy, predictions, labels, probabilities (numpy, as the reference returns)."""
    _, acc, labels, preds, probs = _evaluate(model, dataloader, device)
    y, p = labels.cpu().numpy(), preds.cpu().numpy()
    C = int(max(y.max(initial=0), p.max(initial=0))) + 1
    cm = np.zeros((C, C), np.int64)
    np.add.at(cm, (y, p), 1)
    present = np.unique(np.concatenate([y, p]))
    cm = cm[np.ix_(present, present)]            # sklearn's confusion_matrix over seen labels
    with np.errstate(invalid="ignore", divide="ignore"):
        cmn = cm.astype(float) / cm.sum(axis=1)[:, None]
        per_class = np.diag(cm) / cm.sum(axis=1)
    return {"confusion_matrix": cm, "normalized_confusion_matrix": cmn, "accuracy": acc,
            "per_class_accuracy": per_class, "predictions": p, "true_labels": y,
            "probabilities": probs.cpu().numpy()}


def compute_accuracies(pretrained_dino, traindata, validdata, testdata, model_dir_scratch,
                       model_name, num_epochs=10):
    """run_dino.py:481-501 -> (knn accuracy, MLP accuracy, classifier)."""
    device = torch.device("cuda", torch.cuda.current_device())
    _, knn_accuracy = train_knn_classifier(pretrained_dino, traindata, testdata, n_neighbors=5,
                                           device=device)
    mlp = train_downstream(pretrained_dino, traindata, validdata, testdata, num_epochs=num_epochs,
                           device=device,
                           save_path=f"{model_dir_scratch}/downstream/{model_name}.pt",
                           train_log_path=f"{model_dir_scratch}/downstream/{model_name}_train_log.csv",
                           test_log_path=f"{model_dir_scratch}/downstream/{model_name}_test_log.csv")
    mlp_accuracy = compute_classification_metrics(mlp, testdata, device)["accuracy"]
    return knn_accuracy, mlp_accuracy, mlp
