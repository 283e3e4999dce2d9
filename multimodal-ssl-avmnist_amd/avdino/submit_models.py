"""The reference's job submitter (AVMNIST_Experiments/batch_files/submit_models.py:8-93) for one
MI355X node: same command line, one run_dino job per model, each launched as one process per
GPU (``python -m torch.distributed.run --nproc-per-node N``, N = the config's
hardware.num_gpus) instead of a SLURM ``sbatch run_gpu.sbatch`` line.

    python -m avdino.submit_models --models multi_central image_simple --training_mode mse \\
        --config configs/config_multimodal_dino.yaml [--dry-run] [--log-dir DIR] [-- extra run_dino args]

Models of the reference's list that are not on the MI355X hot path (ViT / LSTM / ResNet /
gated / cross-attention encoders) are rejected with the list of supported ones.  Jobs run one
after another (the node's GPUs are shared by the ranks of one job); stdout / stderr go to
``{log_dir}/{model}{_mode}_{metric}_{timestamp}.out/.err`` as the reference names them.
"""
import argparse
import os
import subprocess
import sys
import time

import yaml

ALL_MODELS = ["multi_simple", "multi_simple_gated", "multi_lstm", "multi_vit", "multi_dual_vit",
              "multi_mobile_vit", "multi_resnet", "multi_cross_attention", "multi_central",
              "image_simple", "spectrogram_simple", "spectrogram_central", "spectrogram_lstm",
              "spectrogram_resnet", "spectrogram_vit", "spectrogram_mobile_vit"]
MULTIMODAL = {"multi_central", "multi_simple"}
UNIMODAL = {"image_simple", "spectrogram_simple", "spectrogram_central"}


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--models", nargs="+", choices=ALL_MODELS)
    p.add_argument("--training_mode", default="default",
                   choices=["default", "semi_supervised", "mse", "infonce"])
    p.add_argument("--config", default="config_multimodal_dino.yaml")
    p.add_argument("--metric", default="mlp_acc", choices=["mlp_acc", "train_loss"])
    p.add_argument("--hyperparameter_tune", action="store_true")
    p.add_argument("--hyperparameter_tune_augments", action="store_true")
    p.add_argument("--dry-run", action="store_true", help="print the commands only")
    p.add_argument("--log-dir", default="runs/debugging")
    p.add_argument("extra", nargs=argparse.REMAINDER, help="-- then extra run_dino arguments")
    return p.parse_args(argv)


def job_command(model, args, num_gpus):
    """The run_dino command of one job (run_gpu.sbatch's python line, per GPU)."""
    flag = "--model" if model in MULTIMODAL else "--unimodal_model"
    cmd = ["-m", "avdino.run_dino", flag, model, "--config", args.config, "--metric", args.metric]
    if model in MULTIMODAL:
        cmd += ["--training_mode", args.training_mode]
    if args.hyperparameter_tune:
        cmd.append("--hyperparameter_tune")
    if args.hyperparameter_tune_augments:
        cmd.append("--hyperparameter_tune_augments")
    extra = [a for a in (args.extra or []) if a != "--"]
    if num_gpus > 1:
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                f"--nproc-per-node={num_gpus}", "--master-addr=127.0.0.1", "--master-port=29511"] + cmd + extra
    return [sys.executable] + cmd + extra


def main(argv=None):
    args = parse_args(argv)
    models = args.models or ALL_MODELS
    bad = [m for m in models if m not in MULTIMODAL | UNIMODAL]
    if bad:
        raise SystemExit(f"not on the MI355X hot path: {bad}; supported: "
                         f"{sorted(MULTIMODAL | UNIMODAL)}")
    with open(args.config) as f:
        num_gpus = int(yaml.safe_load(f).get("hardware", {}).get("num_gpus", 1) or 1)
    stamp = time.strftime("%d%m%Y_%H%M%S")
    mode = "" if args.training_mode == "default" else f"_{args.training_mode}"
    cmds = []
    for model in models:
        cmd = job_command(model, args, num_gpus)
        base = os.path.join(args.log_dir, f"{model}{mode}_{args.metric}_{stamp}")
        print("Submitting:", " ".join(cmd), flush=True)
        cmds.append(cmd)
        if args.dry_run:
            continue
        os.makedirs(args.log_dir, exist_ok=True)
        env = dict(os.environ)
        pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = pkg + os.pathsep + env.get("PYTHONPATH", "")
        with open(base + ".out", "w") as out, open(base + ".err", "w") as err:
            rc = subprocess.run(cmd, stdout=out, stderr=err, env=env).returncode
        print(f"  {model}: exit {rc}", flush=True)
    return cmds


if __name__ == "__main__":
    main()
