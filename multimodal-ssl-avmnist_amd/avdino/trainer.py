"""The part of Lightning's ``Trainer`` the reference's training path uses, for images without
``lightning`` (run_dino.py:337-386: ``pl.Trainer(max_epochs, devices, strategy="ddp" if
num_gpus > 1, precision='16-mixed', callbacks=[ModelCheckpoint(monitor=metric)])``,
``trainer.fit(model, data)``, ``trainer.save_checkpoint``, ``ModelClass.load_from_checkpoint``).

Automatic optimisation exactly as Lightning 2.x runs it for a module with one optimizer and
an epoch-interval scheduler:

  per batch   optimizer.step(closure), closure = training_step -> zero_grad -> backward
  per epoch   callbacks' on_train_epoch_end (non-monitoring) -> module.on_train_epoch_end ->
              monitoring callbacks (ModelCheckpoint) -> lr_scheduler.step()

``train_loss`` logged with ``on_epoch=True`` is reduced to the epoch mean (per-step losses are
kept in a device buffer: no host sync inside the epoch).  ``strategy="ddp"`` is the
reference's DDP on the engine's flat arenas (avdino.dist): rank 0's parameters broadcast once
at setup, rank 0's buffers before every forward (``broadcast_buffers``), one all-reduce of
the flat gradient arena per step; each rank reads its own shard of the batches.

Where ``lightning`` IS installed the model classes are real LightningModules and
``lightning.pytorch.Trainer`` drives them unchanged (the optimizer is a torch Optimizer, the
loss is a differentiable tensor); this class exists so the same loop runs here and on the
GPU box, which have no lightning.
"""
import math
import os
import time

import numpy as np
import torch

from . import dist as avdist


class Callback:
    """lightning.pytorch.Callback's hooks that the reference's training path uses."""

    def on_train_start(self, trainer, module):
        pass

    def on_train_epoch_start(self, trainer, module):
        pass

    def on_train_batch_start(self, trainer, module, batch, batch_idx):
        pass

    def on_train_batch_end(self, trainer, module, outputs, batch, batch_idx):
        pass

    def on_train_epoch_end(self, trainer, module):
        pass

    def on_train_end(self, trainer, module):
        pass


class _Clock:
    """Stream-ordered timestamps: HIP events on the device (no host sync per batch; read back at
    the epoch end), host perf_counter on CPU."""

    def __init__(self, device):
        self.dev = torch.device(device) if device is not None else torch.device("cpu")
        self.gpu = self.dev.type == "cuda"

    def mark(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.dev))
            return e
        return time.perf_counter()

    def seconds(self, a, b):
        if self.gpu:
            b.synchronize()
            return a.elapsed_time(b) / 1e3
        return b - a


class ModelStatsCallback(Callback):
    """run_dino.py:191-225: per-epoch ``epoch_time`` and ``avg_batch_time`` (logged, so they
    reach the CSV log and ``callback_metrics``), ``total_training_time`` at the end.  A batch's
    time is the device time from its first launch to its last (HIP events recorded in stream
    order), so the asynchronous engine is timed without a host synchronisation per batch --
    what time.time() around a synchronous step measures in the reference."""

    def __init__(self):
        super().__init__()
        self.batch_times = []
        self._marks = []
        self.epoch_start_time = None
        self.training_start_time = None
        self.total_training_time = None
        self._clock = None

    def on_train_start(self, trainer, module):
        self._clock = _Clock(getattr(getattr(module, "model", None), "device", None))
        self.training_start_time = time.time()

    def on_train_epoch_start(self, trainer, module):
        self.epoch_start_time = self._clock.mark()
        self._marks = []
        self.batch_times = []

    def on_train_batch_start(self, trainer, module, batch, batch_idx):
        self._marks.append([self._clock.mark(), None])

    def on_train_batch_end(self, trainer, module, outputs, batch, batch_idx):
        self._marks[-1][1] = self._clock.mark()

    def on_train_epoch_end(self, trainer, module):
        end = self._clock.mark()
        epoch_time = self._clock.seconds(self.epoch_start_time, end)
        self.batch_times = [self._clock.seconds(a, b) for a, b in self._marks if b is not None]
        avg_batch_time = float(np.mean(self.batch_times)) if self.batch_times else 0.0
        module.log("epoch_time", epoch_time)
        module.log("avg_batch_time", avg_batch_time)

    def on_train_end(self, trainer, module):
        self.total_training_time = time.time() - self.training_start_time
        if trainer.logger is not None:
            trainer.logger.log_metrics({"total_training_time": self.total_training_time},
                                       step=max(trainer.global_step - 1, 0))
            trainer.logger.save()
        else:
            print(f"Total training time: {self.total_training_time:.2f} seconds")


class CSVLogger:
    """lightning CSVLogger(save_dir, name): ``{save_dir}/{name}/version_{n}/metrics.csv`` (one
    row per ``log_metrics`` call with its ``step``; the header is the sorted union of every key
    seen, the file rewritten when a new key appears, as Lightning's _ExperimentWriter does) and
    ``hparams.yaml``.  run_dino.py:355 builds one per seed (``logs_seed{seed}``)."""

    def __init__(self, save_dir, name="lightning_logs", version=None):
        self.save_dir, self.name = str(save_dir), name
        root = os.path.join(self.save_dir, name)
        if version is None:
            os.makedirs(root, exist_ok=True)
            have = [int(d.split("_", 1)[1]) for d in os.listdir(root)
                    if d.startswith("version_") and d.split("_", 1)[1].isdigit()]
            version = max(have) + 1 if have else 0
        self.version = version
        self.log_dir = os.path.join(root, f"version_{version}")
        self.metrics_file_path = os.path.join(self.log_dir, "metrics.csv")
        self.metrics, self.metrics_keys = [], []
        self.hparams = {}

    def log_hyperparams(self, params):
        self.hparams.update({k: v for k, v in dict(params).items()
                             if isinstance(v, (int, float, str, bool, type(None)))})

    def log_metrics(self, metrics, step=None):
        row = {k: (v.item() if torch.is_tensor(v) else v) for k, v in metrics.items()}
        row["step"] = len(self.metrics) if step is None else int(step)
        self.metrics.append(row)

    def save(self):
        import csv
        import yaml
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, "hparams.yaml"), "w") as f:
            yaml.safe_dump(self.hparams, f)
        if not self.metrics:
            return
        new = sorted(set().union(*self.metrics) - set(self.metrics_keys))
        exists = os.path.isfile(self.metrics_file_path)
        if new:
            self.metrics_keys = sorted(self.metrics_keys + new)
            if exists:       # rewrite the rows already on disk under the wider header
                with open(self.metrics_file_path, newline="") as f:
                    old = list(csv.DictReader(f))
                self.metrics = old + self.metrics
                exists = False
        with open(self.metrics_file_path, "a" if exists else "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self.metrics_keys)
            if not exists:
                w.writeheader()
            w.writerows(self.metrics)
        self.metrics = []

    def finalize(self, status="success"):
        self.save()


class ModelCheckpoint(Callback):
    """lightning ModelCheckpoint(dirpath, monitor, save_top_k=1, mode): keeps the best epoch's
    checkpoint at ``best_model_path`` (run_dino.py:329, 386)."""

    monitoring = True

    def __init__(self, dirpath=".", monitor=None, save_top_k=1, mode="min", filename=None):
        self.dirpath, self.monitor, self.mode = dirpath, monitor, mode
        self.save_top_k, self.filename = save_top_k, filename
        self.best_model_score = None
        self.best_model_path = ""

    def on_train_epoch_end(self, trainer, module):
        if self.save_top_k == 0:
            return
        score = trainer.callback_metrics.get(self.monitor) if self.monitor else None
        if self.monitor and score is None:
            return
        score = None if score is None else float(score)
        better = (self.best_model_score is None or score is None or
                  (score < self.best_model_score if self.mode == "min" else score > self.best_model_score))
        if not better:
            return
        name = self.filename or f"epoch={trainer.current_epoch}-step={trainer.global_step}"
        path = os.path.join(self.dirpath, name + ".ckpt")
        if trainer.is_global_zero:
            os.makedirs(self.dirpath, exist_ok=True)
            trainer.save_checkpoint(path)
            if self.best_model_path and self.best_model_path != path and os.path.exists(self.best_model_path):
                os.remove(self.best_model_path)
        self.best_model_score, self.best_model_path = score, path


class Trainer:
    def __init__(self, max_epochs=1000, devices="auto", strategy="auto", precision="16-mixed",
                 log_every_n_steps=50, logger=None, callbacks=None, deterministic=False,
                 limit_train_batches=None, accelerator="auto", enable_progress_bar=True,
                 process_group=None):
        self.max_epochs = max_epochs
        self.strategy, self.precision, self.devices = strategy, precision, devices
        self.callbacks = list(callbacks or [])
        self.limit_train_batches = limit_train_batches
        self.log_every_n_steps = log_every_n_steps
        self.logger = logger
        self.group = process_group
        self.current_epoch = 0
        self.global_step = 0
        self.callback_metrics = {}
        self.logged_metrics = {}
        self.model = None
        self.optimizers, self.lr_schedulers = [], []

    # ------------------------------------------------------------------ distributed
    @property
    def world_size(self):
        return avdist.world(self.group)

    @property
    def global_rank(self):
        return avdist.rank(self.group)

    @property
    def is_global_zero(self):
        return self.global_rank == 0

    def _setup_ddp(self, module):
        if self.strategy != "ddp" or self.world_size == 1:
            return
        store = module.model.store
        eng = module.model._need_engine()
        avdist.broadcast_parameters(store, group=self.group)
        eng.grad_hook = avdist.grad_allreduce_hook(self.group)
        eng.buffer_hook = lambda st: avdist.broadcast_buffers(st, group=self.group)
        if hasattr(eng, "group"):
            eng.group = self.group

    # ------------------------------------------------------------------ fit
    def _configure(self, module):
        conf = module.configure_optimizers()
        if isinstance(conf, dict):
            opt = conf["optimizer"]
            sch = conf.get("lr_scheduler")
            sch = sch.get("scheduler") if isinstance(sch, dict) else sch
        elif isinstance(conf, (list, tuple)):
            opt, sch = conf[0], (conf[1] if len(conf) > 1 else None)
        else:
            opt, sch = conf, None
        self.optimizers = [opt]
        self.lr_schedulers = [sch] if sch is not None else []
        return opt, sch

    def _loader(self, train_dataloaders, datamodule):
        if train_dataloaders is not None:
            return train_dataloaders
        if datamodule is not None:
            if hasattr(datamodule, "setup"):
                datamodule.setup("fit")
            return datamodule.train_dataloader()
        return self.model.train_dataloader()

    def fit(self, model, train_dataloaders=None, datamodule=None):
        self.model = model
        model.trainer = self
        self._setup_ddp(model)
        opt, sch = self._configure(model)
        loader = self._loader(train_dataloaders, datamodule)
        dev = model.model.device
        if self.logger is not None and hasattr(self.logger, "log_hyperparams"):
            self.logger.log_hyperparams(dict(getattr(model, "hparams", {}) or {}))
        self._hook("on_train_start", model)
        for epoch in range(self.current_epoch, self.max_epochs):
            self.current_epoch = epoch
            model.train()
            model.logged_history = {}
            if hasattr(loader, "set_epoch"):
                loader.set_epoch(epoch)
            self._hook("on_train_epoch_start", model)
            n = self.limit_train_batches
            losses, first_step = [], self.global_step
            # one batch of look-ahead: after a step is issued the module may queue the next
            # batch's input work under it (model.prefetch: the device augmentation)
            prefetch = getattr(model, "prefetch", None)
            it = iter(loader)
            batch, i = next(it, None), 0
            while batch is not None and (n is None or i < n):
                nxt = next(it, None) if (n is None or i + 1 < n) else None
                out = {}
                self._hook("on_train_batch_start", model, batch, i)

                def closure(batch=batch, i=i):
                    loss = model.training_step(batch, i)
                    opt.zero_grad()
                    loss.backward()
                    out["loss"] = loss
                    return loss

                opt.step(closure)
                if nxt is not None and prefetch is not None:
                    prefetch(nxt)
                losses.append(out["loss"].detach().reshape(1))
                self._hook("on_train_batch_end", model, out, batch, i)
                self.global_step += 1
                batch, i = nxt, i + 1
            self._epoch_metrics(model, losses, dev)
            for cb in self.callbacks:
                if not getattr(cb, "monitoring", False):
                    cb.on_train_epoch_end(self, model)
            model.on_train_epoch_end()
            self._collect(model)
            for cb in self.callbacks:
                if getattr(cb, "monitoring", False):
                    cb.on_train_epoch_end(self, model)
            for s in self.lr_schedulers:
                s.step()
            self._log_epoch(epoch, losses, first_step)
        self.current_epoch = self.max_epochs
        self._hook("on_train_end", model)
        if self.logger is not None and hasattr(self.logger, "save"):
            self.logger.save()
        return self

    def _hook(self, name, model, *args):
        for cb in self.callbacks:
            fn = getattr(cb, name, None)
            if fn is not None:
                fn(self, model, *args)

    def _log_epoch(self, epoch, losses, first_step):
        """Lightning's logger rows for ``self.log('train_loss', on_step=True, on_epoch=True)``:
        ``train_loss_step`` every ``log_every_n_steps`` steps (step index s with (s+1) % n == 0),
        then one epoch-end row with the epoch-level metrics.  The step losses stay on the device
        during the epoch; they are read back here, once."""
        if self.logger is None or not hasattr(self.logger, "log_metrics"):
            return
        if losses:
            vals = torch.cat(losses).float().cpu().tolist()
            for j, v in enumerate(vals):
                s = first_step + j
                if (s + 1) % max(self.log_every_n_steps, 1) == 0:
                    self.logger.log_metrics({"train_loss_step": v, "epoch": epoch}, step=s)
        self.logger.log_metrics(dict(self.logged_metrics, epoch=epoch), step=max(self.global_step - 1, 0))

    def _epoch_metrics(self, model, losses, dev):
        """on_epoch=True reduction of train_loss: the mean of this epoch's step losses (in DDP,
        the mean over ranks too, as Lightning's sync_dist would)."""
        if not losses:
            return
        m = torch.cat(losses).float().mean()
        if self.strategy == "ddp" and self.world_size > 1:
            m = m.clone()
            torch.distributed.all_reduce(m, group=self.group)
            m /= self.world_size
        self.callback_metrics["train_loss"] = m.item()
        self.logged_metrics["train_loss_epoch"] = self.callback_metrics["train_loss"]

    def _collect(self, model):
        for k, v in getattr(model, "logged", {}).items():
            if k == "train_loss":
                continue
            self.callback_metrics[k] = v.item() if torch.is_tensor(v) else v
            self.logged_metrics[k] = self.callback_metrics[k]

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, path):
        """Lightning's checkpoint dict: epoch, global_step, state_dict (the reference's keys,
        ``model.student.…``), hyper_parameters, optimizer and scheduler states."""
        save_checkpoint(self.model, path, epoch=self.current_epoch, global_step=self.global_step,
                        optimizers=self.optimizers, lr_schedulers=self.lr_schedulers)


def save_checkpoint(module, path, epoch=0, global_step=0, optimizers=(), lr_schedulers=()):
    ckpt = {
        "epoch": epoch,
        "global_step": global_step,
        "pytorch-lightning_version": "2.5.0.post0",
        "state_dict": {k: v.detach().cpu().clone() for k, v in module.state_dict().items()},
        "hyper_parameters": dict(getattr(module, "hparams", {}) or {}),
        "optimizer_states": [o.state_dict() for o in optimizers],
        "lr_schedulers": [s.state_dict() for s in lr_schedulers],
    }
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save(ckpt, path)
    return ckpt


def load_checkpoint(path):
    """A checkpoint's dict, loaded with ``weights_only=True`` (nothing executed from the
    file).  A reference Lightning checkpoint pickles class objects in ``hyper_parameters``;
    the safe loader refuses those -- pass its ``state_dict`` instead."""
    return torch.load(path, map_location="cpu", weights_only=True)


def cosine_lr(base_lr, epoch, T_max, eta_min=0.0):
    """CosineAnnealingLR's closed form (the value after ``epoch`` scheduler steps)."""
    return eta_min + (base_lr - eta_min) * (1 + math.cos(math.pi * epoch / T_max)) / 2
