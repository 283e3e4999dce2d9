"""Training driver with the reference's run_dino.py command line and YAML config schema
(AVMNIST_Experiments/run_dino.py:528-600 main(), 603-664 model construction, 300-386
experiment(); configs/config_multimodal_dino.yaml).

    python -m avdino.run_dino --model multi_central --training_mode mse \\
        --config configs/config_multimodal_dino.yaml [--steps-per-epoch 50] [--epochs 2]
    # hardware.num_gpus > 1: one process per GPU, strategy="ddp" (run_dino.py:359)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m avdino.run_dino --model multi_central --training_mode infonce --config ...

Model selection, training modes and the hyperparameters read from the config are the
reference's; the loop is Lightning's automatic optimisation (avdino.trainer.Trainer:
training_step -> zero_grad -> backward -> Adam per batch, on_train_epoch_end's linear probe,
ModelCheckpoint on ``--metric``, CosineAnnealingLR per epoch), then ``load_from_checkpoint``
of the best epoch and the downstream kNN (k=5) + 10-epoch MLP evaluation
(``compute_accuracies``, run_dino.py:481-501) when labelled data is available.

Data: with the AVMNIST files under ``data.data_dir`` (get_data.py's layout) the batches come
from the HBM-resident loader and the device augmentation (avdino.data / avdino.augment, the
config's ``best_augments`` mapped as process_augment_config does); without them (``--synthetic``
or no files) batches are synthetic AVMNIST-shaped device tensors (pixel values randint/255).
--hyperparameter_tune / --hyperparameter_tune_augments (Optuna) are out of scope.
"""
import argparse
import json
import os

import yaml

MULTI_MODES = ["default", "semi_supervised", "mse", "infonce"]


def parse_args(argv=None):
    from .models import MODEL_MAP, UNIMODAL_MODEL_MAP
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    g = p.add_mutually_exclusive_group(required=True)
    g.add_argument("--model", choices=list(MODEL_MAP))
    g.add_argument("--unimodal_model", choices=list(UNIMODAL_MODEL_MAP))
    p.add_argument("--training_mode", default="default", choices=MULTI_MODES)
    p.add_argument("--config", required=True)
    p.add_argument("--metric", default="mlp_acc", choices=["mlp_acc", "train_loss"])
    p.add_argument("--hyperparameter_tune", action="store_true")
    p.add_argument("--hyperparameter_tune_augments", action="store_true")
    p.add_argument("--epochs", type=int, default=None, help="override num_epochs")
    p.add_argument("--steps-per-epoch", type=int, default=20,
                   help="batches per epoch (synthetic data; caps the real loader too)")
    p.add_argument("--batch-size", type=int, default=None, help="override batch_size")
    p.add_argument("--probe-batches", type=int, default=4,
                   help="labelled batches for the epoch-end probe (synthetic data)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "32"])
    p.add_argument("--synthetic", action="store_true", help="synthetic batches even if data exists")
    p.add_argument("--out", default=None, help="checkpoint directory (default: a temp dir)")
    p.add_argument("--downstream", action="store_true",
                   help="after fit: load the best checkpoint, kNN + MLP downstream accuracies")
    a = p.parse_args(argv)
    if a.unimodal_model and a.training_mode != "default":
        raise SystemExit(f"--training_mode '{a.training_mode}' is only compatible with --model "
                         f"(multimodal models).")   # run_dino.py:584-585
    if a.hyperparameter_tune or a.hyperparameter_tune_augments:
        raise SystemExit("Optuna hyperparameter search is outside the MI355X hot path")
    return a


def load_config(path):
    with open(path) as f:
        return yaml.safe_load(f)


def build_model(args, config, device="cuda", group=None):
    """run_dino.py:629-664: the Lightning-shaped module from the config's hyperparameters."""
    from .models import MODEL_MAP, MULTIMODAL_WRAPPERS, UNIMODAL_MODEL_MAP, UniModalDINOLightning
    h = config["hyperparameters"]
    common = dict(data_dir=config["data"]["data_dir"], projection_dim=h["projection_dim"],
                  output_dim=h["output_dim"], momentum=h["momentum"],
                  center_momentum=h["center_momentum"], teacher_temperature=h["teacher_temperature"],
                  learning_rate=h["learning_rate"], num_epochs=h["num_epochs"],
                  weight_decay=h["weight_decay"], dropout=h["dropout"],
                  data_augmentation=h.get("data_augmentation", "burst_noise"),
                  device=device, precision=args.precision, seed=config["experiment"]["seed"])
    if args.model:
        cls = MULTIMODAL_WRAPPERS[args.training_mode]
        return cls(encoder_class=MODEL_MAP[args.model], encoder_output_dim=h["encoder_output_dim"],
                   student_temperature=h["student_temperature"], use_mixed_precision=True,
                   group=group, **common)
    return UniModalDINOLightning(encoder_class=UNIMODAL_MODEL_MAP[args.unimodal_model],
                                 cosine_loss_alpha=h["cosine_loss_alpha"], **common)


def synthetic_batch(B, G, L, device, gen, multimodal_mode):
    import torch

    def px(*shape):
        return torch.randint(0, 256, shape, generator=gen, device=device, dtype=torch.int32).float() / 255.0

    views = (px(B, G, 1, 28, 28), px(B, G, 1, 112, 112), px(B, L, 1, 28, 28), px(B, L, 1, 112, 112))
    if multimodal_mode in (None, "default"):
        return views
    return (px(B, 1, 28, 28), px(B, 1, 112, 112),
            torch.randint(0, 10, (B,), generator=gen, device=device), views)


class SyntheticDinoLoader:
    """AVMNIST-shaped synthetic batches in the DINO data modules' tuple layout (get_data.py:
    480-509), generated on the device; ``steps`` batches per epoch."""

    def __init__(self, B, G, L, steps, device, seed, multimodal_mode):
        import torch
        self.B, self.G, self.L, self.steps, self.mode = B, G, L, steps, multimodal_mode
        self.device = device
        self.gen = torch.Generator(device=device).manual_seed(seed)

    def __len__(self):
        return self.steps

    def __iter__(self):
        for _ in range(self.steps):
            yield synthetic_batch(self.B, self.G, self.L, self.device, self.gen, self.mode)


def synthetic_labelled(B, n, device, seed):
    """(images, audios, labels) batches like AVMNISTDataModule's loaders (get_data.py:412-472)."""
    import torch
    gen = torch.Generator(device=device).manual_seed(seed)
    out = []
    for _ in range(n):
        b = synthetic_batch(B, 1, 0, device, gen, "mse")
        out.append((b[0], b[1], torch.randint(0, 10, (B,), generator=gen, device=device)))
    return out


def _have_data(config, h):
    from .data import avmnist_paths
    paths = avmnist_paths(config["data"]["data_dir"], h.get("data_augmentation", "burst_noise"))
    return all(os.path.exists(p) for split in paths.values() for p in split)


def _init_distributed():
    """torchrun env -> one process per GPU over RCCL (backend "nccl")."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    if not dist.is_initialized():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    return dist.get_rank(), dist.get_world_size()


class _EpochPrinter:
    """One JSON line per epoch on rank 0: train_loss (epoch mean), lr used, probe results."""

    monitoring = True

    def on_train_epoch_end(self, trainer, module):
        if not trainer.is_global_zero:
            return
        rec = {"epoch": trainer.current_epoch, "train_loss": trainer.callback_metrics.get("train_loss"),
               "lr": trainer.optimizers[0].param_groups[0]["lr"]}
        for k in ("val_loss", "mlp_acc"):
            if k in trainer.callback_metrics:
                rec[k] = trainer.callback_metrics[k]
        print(json.dumps(rec), flush=True)


def main(argv=None):
    import tempfile

    import torch

    from .trainer import ModelCheckpoint, Trainer
    args = parse_args(argv)
    config = load_config(args.config)
    h = config["hyperparameters"]
    if not torch.cuda.is_available():
        raise SystemExit("run_dino needs a ROCm device: the MI355X engine has no CPU fallback")
    rank, world = _init_distributed()
    ddp = config["hardware"].get("num_gpus", 1) > 1 and world > 1
    dev = torch.device("cuda", torch.cuda.current_device())
    model = build_model(args, config, device=dev)
    epochs = args.epochs or h["num_epochs"]
    B = args.batch_size or h["batch_size"]
    G, L = h.get("n_global_views", 2), h.get("n_local_views", 4)
    seed = config["experiment"]["seed"] + 7919 * rank
    mode = args.training_mode if args.model else None
    real = not args.synthetic and _have_data(config, h)
    if real:
        from .augment import MultiModalAugmentation, process_augment_config
        from .data import AVMNISTDinoLoader, AVMNISTLabelledLoader
        aug = MultiModalAugmentation(G, L, augment_values=process_augment_config(config))
        loader = AVMNISTDinoLoader(config["data"]["data_dir"], B, G, L,
                                   h.get("data_augmentation", "burst_noise"), aug, dev,
                                   seed=config["experiment"]["seed"], multimodal_mode=mode,
                                   rank=rank, world=world)
        lab = dict(data_dir=config["data"]["data_dir"], batch_size=128, device=dev,
                   type=h.get("data_augmentation", "burst_noise"), seed=config["experiment"]["seed"])
        traindata = AVMNISTLabelledLoader(split="train", **lab)
        validdata = AVMNISTLabelledLoader(split="val", **lab)
        testdata = AVMNISTLabelledLoader(split="test", **lab)
    else:
        loader = SyntheticDinoLoader(B, G, L, args.steps_per_epoch, dev, seed, mode)
        traindata = synthetic_labelled(B, args.probe_batches, dev, seed + 1)
        validdata = testdata = traindata[:1]
    if args.probe_batches or real:
        model.traindata, model.validdata = traindata, validdata
    out = args.out or tempfile.mkdtemp(prefix="avdino_run_")
    ckpt = ModelCheckpoint(dirpath=out, monitor=args.metric, save_top_k=1,
                           mode="max" if args.metric == "mlp_acc" else "min")
    trainer = Trainer(max_epochs=epochs, strategy="ddp" if ddp else "auto", precision="16-mixed",
                      callbacks=[ckpt, _EpochPrinter()],
                      limit_train_batches=args.steps_per_epoch if real else None)
    trainer.fit(model, loader)
    if args.downstream and trainer.is_global_zero and ckpt.best_model_path:
        from .downstream import compute_accuracies
        best = type(model).load_from_checkpoint(ckpt.best_model_path, device=dev,
                                                precision=args.precision)
        knn, mlp, _ = compute_accuracies(best.model, traindata, validdata, testdata, out, "model",
                                         num_epochs=2 if not real else 10)
        print(json.dumps({"knn_acc": knn, "mlp_acc": mlp}), flush=True)
    model.trainer_ = trainer
    return model


if __name__ == "__main__":
    main()
