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
(``compute_accuracies``, run_dino.py:481-501) with ``--downstream``.  As experiment()
(run_dino.py:346-402) this runs once per seed (1, 2, 3 by default, ``--seeds``), every seed
from the same initial weights, and reports the mean and standard deviation of the seeds' kNN /
MLP accuracies in ``final_results_*.csv`` / ``performance_summary.txt``.

Data: with the AVMNIST files under ``data.data_dir`` (get_data.py's layout) the batches come
from the HBM-resident loader and the device augmentation (avdino.data / avdino.augment, the
config's ``best_augments`` mapped as process_augment_config does); without them (``--synthetic``
or no files) batches are synthetic AVMNIST-shaped device tensors (pixel values randint/255).
--hyperparameter_tune / --hyperparameter_tune_augments (Optuna) are out of scope.
"""
import argparse
import math
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
    p.add_argument("--steps-per-epoch", type=int, default=None,
                   help="batches per epoch: synthetic data default 20; with real data the "
                        "loader's full epoch (the reference's Trainer has no batch limit) unless "
                        "given, then it caps the epoch like limit_train_batches")
    p.add_argument("--batch-size", type=int, default=None, help="override batch_size")
    p.add_argument("--probe-batches", type=int, default=4,
                   help="labelled batches for the epoch-end probe (synthetic data)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "32"])
    p.add_argument("--synthetic", action="store_true", help="synthetic batches even if data exists")
    p.add_argument("--out", default=None, help="checkpoint directory (default: a temp dir)")
    p.add_argument("--downstream", action="store_true",
                   help="after fit: load the best checkpoint, kNN + MLP downstream accuracies")
    p.add_argument("--seeds", default="1,2,3",
                   help="comma-separated seeds; one full fit (+ downstream) per seed from the same "
                        "initial weights (run_dino.py:346: seeds = [1, 2, 3])")
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


def build_model(args, config, device="cuda", group=None, seed=None):
    """run_dino.py:629-664: the Lightning-shaped module from the config's hyperparameters
    (``seed``: the module's initialisation / dropout seed, default the config's)."""
    from .models import MODEL_MAP, MULTIMODAL_WRAPPERS, UNIMODAL_MODEL_MAP, UniModalDINOLightning
    h = config["hyperparameters"]
    common = dict(data_dir=config["data"]["data_dir"], projection_dim=h["projection_dim"],
                  output_dim=h["output_dim"], momentum=h["momentum"],
                  center_momentum=h["center_momentum"], teacher_temperature=h["teacher_temperature"],
                  learning_rate=h["learning_rate"], num_epochs=h["num_epochs"],
                  weight_decay=h["weight_decay"], dropout=h["dropout"],
                  data_augmentation=h.get("data_augmentation", "burst_noise"),
                  device=device, precision=args.precision,
                  seed=config["experiment"]["seed"] if seed is None else seed)
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


def _stack_macs(stack):
    """Multiply-adds of one sample through a conv stack (Conv2d: Ho*Wo*Cout*Cin*K*K)."""
    macs = 0
    for (ci, co, k, _p), (_h, ho, _hp) in zip(stack.convs, stack.layer_dims()):
        macs += ho * ho * co * ci * k * k
    return macs


def model_stats(model, G, L):
    """(GFLOPs per sample, parameter count) for run_dino's performance summary
    (calculate_gflops, run_dino.py:243-283: torchinfo's total_mult_adds of the eval-mode forward
    over one batch / batch size, and total_params).  Analytic here (no torchinfo): Conv2d and
    Linear multiply-adds of the student over the G+L views, the teacher over the G global views,
    their projection heads and, for the modes with heads, the originals through the student
    branches and both heads; parameters = every parameter tensor of the state dict (student,
    teacher, heads, incl. the CentralNet fc1/fc2 the reference builds but never runs)."""
    from .spec import MULTI_ENCODERS, UNI_ENCODERS
    m = model.model
    spec = m.store.spec
    params = sum(int(math.prod(shp)) for k, (shp, kind) in spec.items()
                 if kind in ("w", "b", "bn_w", "bn_b"))

    def lin(key):
        shp = spec[key + ".weight"][0]
        return shp[0] * shp[1]

    def head(prefix):
        return lin(prefix + ".mlp.0") + lin(prefix + ".mlp.4")

    arch = getattr(m.student_spec, "arch", None)
    if arch in MULTI_ENCODERS:
        ist, il, ast_, al, _ = MULTI_ENCODERS[arch]
        branch_i = _stack_macs(ist("student")) + lin("student." + il)
        branch_a = _stack_macs(ast_("student")) + lin("student." + al)
        enc = branch_i + branch_a + lin("student.fusion.0") + lin("student.fusion.3")
        macs = (G + L) * (enc + head("student_projection")) + G * (enc + head("teacher_projection"))
        heads = [k[:-len(".mlp.0.weight")] for k in spec if k.endswith(".mlp.0.weight")
                 and not k.startswith(("student_projection", "teacher_projection"))]
        if heads:
            macs += branch_i + branch_a + sum(head(h) for h in heads)
    else:
        kind = m.student_spec.kind
        _mod, stack, lins, _sd = UNI_ENCODERS[kind]
        enc = _stack_macs(stack("student")) + sum(lin(f"student.{k}") for k in lins)
        macs = (G + L) * (enc + head("student_projection")) + G * (enc + head("teacher_projection"))
    return macs / 1e9, params


def write_run_summary(model, args, config, out, G, L, stats_cb, trainer, training_time,
                      knn=None, mlp=None):
    """run_dino.py:409-464: ``final_results_{model}.csv`` (one row, the reference's columns) and
    ``performance_summary.txt`` (key: value lines + the augmentation summary).  ``knn`` / ``mlp``:
    the per-seed accuracies (lists; their mean and population std, np.mean / np.std as
    run_dino.py:395-398), or None without the downstream evaluation; the rest describes the last
    seed's run, as the reference's summary does."""
    import csv
    from datetime import datetime

    import numpy as np
    knn_m = knn_s = mlp_m = mlp_s = None
    if knn:
        knn_m, knn_s = float(np.mean(knn)), float(np.std(knn))
    if mlp:
        mlp_m, mlp_s = float(np.mean(mlp)), float(np.std(mlp))
    h = config["hyperparameters"]
    gflops, params = model_stats(model, G, L)
    name = config.get("model", {}).get("name") or (args.model or args.unimodal_model)
    cm = trainer.callback_metrics
    epoch_time, avg_batch = cm.get("epoch_time"), cm.get("avg_batch_time")
    results = {
        "model": name, "best_train_loss": cm.get("train_loss"), "best_mlp_acc": cm.get("mlp_acc"),
        "learning_rate": h["learning_rate"], "batch_size": args.batch_size or h["batch_size"],
        "momentum": h["momentum"], "center_momentum": h["center_momentum"],
        "projection_dim": h["projection_dim"], "output_dim": h["output_dim"],
        "data_augmentation": h.get("data_augmentation", "burst_noise"),
        "n_global_views": G, "n_local_views": L, "gflops": gflops, "params": params,
        "params_millions": params / 1e6, "total_training_time": training_time,
        "avg_epoch_time": epoch_time, "avg_batch_time": avg_batch,
        "timestamp": datetime.now().strftime("%Y-%m-%d %H:%M:%S")}
    with open(os.path.join(out, f"final_results_{name}.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(results))
        w.writeheader()
        w.writerow(results)
    metric = args.metric
    perf = {
        "model_name": name, "parameters": f"{params / 1e6:.2f}M", "gflops": f"{gflops:.2f}",
        "n_global_views": G, "n_local_views": L,
        "training_time_hours": f"{training_time / 3600:.2f}",
        "avg_epoch_time_minutes": f"{epoch_time / 60:.2f}" if epoch_time else "N/A",
        "best_train_loss": f"{float(cm.get('train_loss', 0) or 0):.4f}",
        f"best_{metric}": f"{float(cm.get(metric, 0) or 0):.4f}",
        "downstream_mlp_acc": f"{mlp_m:.4f}" if mlp_m is not None else "N/A",
        "downstream_knn_accuracy": f"{knn_m:.4f}" if knn_m is not None else "N/A",
        "downstream_mlp_acc_std": f"{mlp_s:.4f}" if mlp_s is not None else "N/A",
        "downstream_knn_accuracy_std": f"{knn_s:.4f}" if knn_s is not None else "N/A",
        # gate_image / gate_audio exist only on the gated encoders (not on the MI355X path)
        "final_audio_gate": "N/A", "final_image_gate": "N/A",
    }
    with open(os.path.join(out, "performance_summary.txt"), "w") as f:
        for k, v in perf.items():
            f.write(f"{k}: {v}\n")
        aug = getattr(model, "augment_summary", None)
        if aug:
            f.write("\n# Augmentation Summary\n" + str(aug) + "\n")
    return results, perf


def _set_seed(seed):
    """set_seed (run_dino.py's helper): Python, numpy and torch RNGs."""
    import random

    import numpy as np
    import torch
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def main(argv=None):
    import copy
    import tempfile
    import time

    import torch

    from .trainer import CSVLogger, ModelCheckpoint, ModelStatsCallback, Trainer
    args = parse_args(argv)
    config = load_config(args.config)
    h = config["hyperparameters"]
    if not torch.cuda.is_available():
        raise SystemExit("run_dino needs a ROCm device: the MI355X engine has no CPU fallback")
    rank, world = _init_distributed()
    ddp = config["hardware"].get("num_gpus", 1) > 1 and world > 1
    dev = torch.device("cuda", torch.cuda.current_device())
    seeds = [int(v) for v in str(args.seeds).split(",") if v.strip()]
    if not seeds:
        raise SystemExit("--seeds: at least one seed")
    # run_dino.py:300: the initial weights every seed starts from
    initial = copy.deepcopy(build_model(args, config, device=dev).state_dict())
    epochs = args.epochs or h["num_epochs"]
    B = args.batch_size or h["batch_size"]
    G, L = h.get("n_global_views", 2), h.get("n_local_views", 4)
    mode = args.training_mode if args.model else None
    real = not args.synthetic and _have_data(config, h)
    out = args.out or tempfile.mkdtemp(prefix="avdino_run_")
    # run_dino.py:333: ONE ModelCheckpoint for all seeds -- its best score carries over, so a
    # later seed's best_model_path is that seed's best epoch only if it beats the earlier seeds'
    ckpt = ModelCheckpoint(dirpath=out, monitor=args.metric, save_top_k=1,
                           mode="max" if args.metric == "mlp_acc" else "min")
    stats_cb = ModelStatsCallback()
    name = config.get("model", {}).get("name") or (args.model or args.unimodal_model)
    knns, mlps = [], []
    for s in seeds:
        _set_seed(s)
        seed = s + 7919 * rank
        model = build_model(args, config, device=dev, seed=seed)
        model.load_state_dict(initial)
        if real:
            from .augment import MultiModalAugmentation, process_augment_config
            from .data import AVMNISTDinoLoader, AVMNISTLabelledLoader
            aug = MultiModalAugmentation(G, L, augment_values=process_augment_config(config))
            loader = AVMNISTDinoLoader(config["data"]["data_dir"], B, G, L,
                                       h.get("data_augmentation", "burst_noise"), aug, dev,
                                       seed=s, multimodal_mode=mode, rank=rank, world=world,
                                       staged=hasattr(model, "prefetch") and mode is not None)
            lab = dict(data_dir=config["data"]["data_dir"], batch_size=128, device=dev,
                       type=h.get("data_augmentation", "burst_noise"), seed=config["experiment"]["seed"])
            traindata = AVMNISTLabelledLoader(split="train", **lab)
            validdata = AVMNISTLabelledLoader(split="val", **lab)
            testdata = AVMNISTLabelledLoader(split="test", **lab)
        else:
            loader = SyntheticDinoLoader(B, G, L, args.steps_per_epoch or 20, dev, seed, mode)
            traindata = synthetic_labelled(B, args.probe_batches, dev, seed + 1)
            validdata = testdata = traindata[:1]
        if args.probe_batches or real:
            model.traindata, model.validdata = traindata, validdata
        # run_dino.py:355-365: CSVLogger per seed, log_every_n_steps=10, [checkpoint, stats]
        logger = CSVLogger(out, name=f"logs_seed{s}") if rank == 0 else None
        trainer = Trainer(max_epochs=epochs, strategy="ddp" if ddp else "auto", precision="16-mixed",
                          callbacks=[ckpt, stats_cb, _EpochPrinter()], log_every_n_steps=10,
                          logger=logger, deterministic=True,
                          limit_train_batches=args.steps_per_epoch if real else None)
        t0 = time.time()
        trainer.fit(model, loader)
        training_time = time.time() - t0
        if trainer.is_global_zero:
            trainer.save_checkpoint(os.path.join(out, f"{name}.ckpt"))       # run_dino.py:379
        if args.downstream and trainer.is_global_zero and ckpt.best_model_path:
            from .downstream import compute_accuracies
            best = type(model).load_from_checkpoint(ckpt.best_model_path, device=dev,
                                                    precision=args.precision)
            knn, mlp, _ = compute_accuracies(best.model, traindata, validdata, testdata, out, "model",
                                             num_epochs=2 if not real else 10)
            knns.append(knn)
            mlps.append(mlp)
            print(json.dumps({"seed": s, "knn_acc": knn, "mlp_acc": mlp}), flush=True)
    if trainer.is_global_zero:
        write_run_summary(model, args, config, out, G, L, stats_cb, trainer, training_time,
                          knns or None, mlps or None)
        if knns:
            print(json.dumps({"knn_acc_mean": sum(knns) / len(knns), "mlp_acc_mean": sum(mlps) / len(mlps),
                              "seeds": seeds}), flush=True)
    model.trainer_ = trainer
    model.out_dir_ = out
    model.seed_accuracies_ = {"knn": knns, "mlp": mlps}
    return model


if __name__ == "__main__":
    main()
