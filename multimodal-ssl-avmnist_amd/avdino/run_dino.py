"""Training driver with the reference's run_dino.py command line and YAML config schema
(AVMNIST_Experiments/run_dino.py:528-600 main(), 603-664 model construction, 300-372
experiment(); configs/config_multimodal_dino.yaml).

    python -m avdino.run_dino --model multi_central --training_mode mse \\
        --config configs/config_multimodal_dino.yaml [--steps-per-epoch 50] [--epochs 2]

Model selection, training modes and the hyperparameters read from the config are the
reference's.  What differs, and why:
  * data: the AVMNIST on-disk loader and the CPU augmentation pipeline are SURVEY 8(f) "next"
    work, so batches are synthetic AVMNIST-shaped device tensors (pixel values randint/255,
    2 global + 4 local views per sample, as get_data.py produces) -- the training step itself
    is the real one;
  * Lightning's Trainer is replaced by its automatic-optimisation loop: training_step ->
    backward_and_step per batch, CosineAnnealingLR.step() per epoch, the linear probe at the
    end of each epoch (on synthetic labelled batches);
  * --hyperparameter_tune / --hyperparameter_tune_augments (Optuna) are out of scope.
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
    p.add_argument("--steps-per-epoch", type=int, default=20)
    p.add_argument("--batch-size", type=int, default=None, help="override batch_size")
    p.add_argument("--probe-batches", type=int, default=4)
    p.add_argument("--precision", default="bf16", choices=["bf16", "32"])
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


def build_model(args, config, device="cuda"):
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
                   student_temperature=h["student_temperature"], use_mixed_precision=True, **common)
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


def main(argv=None):
    import torch
    args = parse_args(argv)
    config = load_config(args.config)
    h = config["hyperparameters"]
    if not torch.cuda.is_available():
        raise SystemExit("run_dino needs a ROCm device: the MI355X engine has no CPU fallback")
    model = build_model(args, config)
    epochs = args.epochs or h["num_epochs"]
    B = args.batch_size or h["batch_size"]
    G, L = h.get("n_global_views", 2), h.get("n_local_views", 4)
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(config["experiment"]["seed"])
    sched = model.configure_optimizers()["lr_scheduler"]["scheduler"]
    mode = args.training_mode if args.model else None
    for epoch in range(epochs):
        losses = []
        for step in range(args.steps_per_epoch):
            loss = model.training_step(synthetic_batch(B, G, L, dev, gen, mode), step)
            model.backward_and_step()
            losses.append(loss)
        sched.step()
        probe = [(synthetic_batch(B, 1, 0, dev, gen, "mse")[0], synthetic_batch(B, 1, 0, dev, gen, "mse")[1],
                  torch.randint(0, 10, (B,), generator=gen, device=dev)) for _ in range(args.probe_batches)]
        out = model.on_train_epoch_end(probe, probe[:1]) if args.probe_batches else None
        rec = {"epoch": epoch, "train_loss": float(torch.stack([x.reshape(()) for x in losses]).mean()),
               "lr": sched.get_last_lr()[0]}
        if out:
            rec.update(val_loss=out["val_loss"], mlp_acc=out["mlp_acc"])
        print(json.dumps(rec), flush=True)
    return model


if __name__ == "__main__":
    main()
