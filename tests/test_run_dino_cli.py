"""run_dino command line and YAML config surface (reference run_dino.py:528-664): argument
rules and the hyperparameter mapping, on CPU (no training: the engine needs a GPU)."""
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(REPO, "configs", "config_multimodal_dino.yaml")


def test_cli_rules_and_config_mapping():
    from avdino import run_dino as R
    a = R.parse_args(["--model", "multi_central", "--training_mode", "mse", "--config", CFG,
                      "--precision", "32"])
    cfg = R.load_config(CFG)
    m = R.build_model(a, cfg, device="cpu")
    h = cfg["hyperparameters"]
    assert type(m).__name__ == "MultiModalDINOWithMSELightning"
    assert m.learning_rate == h["learning_rate"] and m.num_epochs == h["num_epochs"]
    assert m.model.hp.tau_t == h["teacher_temperature"] and m.model.hp.wd == h["weight_decay"]
    assert m.model.store["center"].shape == (1, h["projection_dim"])
    assert m.model.engine is None                      # CPU: no engine, no fallback
    u = R.build_model(R.parse_args(["--unimodal_model", "image_simple", "--config", CFG]), cfg, "cpu")
    assert type(u).__name__ == "UniModalDINOLightning" and u.cosine_loss_alpha == 0
    with pytest.raises(SystemExit):   # training modes are multimodal-only (run_dino.py:584)
        R.parse_args(["--unimodal_model", "image_simple", "--training_mode", "mse", "--config", CFG])
    with pytest.raises(SystemExit):
        R.parse_args(["--model", "multi_central", "--unimodal_model", "image_simple", "--config", CFG])
    with pytest.raises(RuntimeError):
        m.training_step(None, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("argv", [["--model", "multi_central", "--training_mode", "mse"],
                                  ["--model", "multi_central", "--training_mode", "semi_supervised"],
                                  ["--unimodal_model", "spectrogram_simple"]])
def test_run_dino_two_epochs_on_device(argv, capsys):
    """The driver end to end on the GPU: 2 epochs x 3 steps, cosine LR per epoch, probe."""
    import json
    from avdino import run_dino as R
    m = R.main(argv + ["--config", CFG, "--epochs", "2", "--steps-per-epoch", "3",
                       "--batch-size", "8", "--probe-batches", "2", "--synthetic", "--seeds", "1"])
    recs = [json.loads(line) for line in capsys.readouterr().out.splitlines() if line.startswith("{")]
    assert len(recs) == 2 and all(r["train_loss"] == r["train_loss"] for r in recs)
    assert 0 <= recs[-1]["mlp_acc"] <= 100
    # lr used in each epoch: CosineAnnealingLR(T_max=num_epochs) stepped per epoch
    assert recs[1]["lr"] < recs[0]["lr"] == pytest.approx(1e-4)
    assert m.model.engine.step_idx == 6
    assert m.trainer_.global_step == 6


@pytest.mark.gpu
def test_run_dino_three_seeds_downstream(tmp_path, capsys):
    """experiment() (run_dino.py:346-402): seeds 1-3 from the same initial weights, each a full
    fit + best-checkpoint reload + kNN / MLP downstream; the summary holds the seeds' mean and
    population std (np.mean / np.std), one CSVLogger directory per seed."""
    import json

    import numpy as np
    from avdino import run_dino as R
    m = R.main(["--model", "multi_central", "--training_mode", "mse", "--config", CFG, "--epochs", "1",
                "--steps-per-epoch", "2", "--batch-size", "8", "--probe-batches", "2", "--synthetic",
                "--downstream", "--out", str(tmp_path)])
    recs = [json.loads(line) for line in capsys.readouterr().out.splitlines() if line.startswith("{")]
    per = [r for r in recs if "seed" in r]
    assert [r["seed"] for r in per] == [1, 2, 3]
    knn = [r["knn_acc"] for r in per]
    mlp = [r["mlp_acc"] for r in per]
    assert m.seed_accuracies_ == {"knn": knn, "mlp": mlp}
    summ = dict(line.split(": ", 1) for line in open(tmp_path / "performance_summary.txt").read().splitlines()
                if ": " in line)
    assert float(summ["downstream_knn_accuracy"]) == pytest.approx(np.mean(knn), abs=1e-4)
    assert float(summ["downstream_mlp_acc_std"]) == pytest.approx(np.std(mlp), abs=1e-4)
    for s in (1, 2, 3):
        assert (tmp_path / f"logs_seed{s}").is_dir()
    assert (tmp_path / "multi_central.ckpt").exists() or any(tmp_path.glob("*.ckpt"))


def test_seeds_argument():
    from avdino import run_dino as R
    a = R.parse_args(["--model", "multi_central", "--config", CFG])
    assert a.seeds == "1,2,3"                     # run_dino.py:346


def test_submit_models_surface(tmp_path):
    """batch_files/submit_models.py's command line: one run_dino job per model, unsupported
    encoders rejected, torchrun with nproc = hardware.num_gpus when > 1."""
    import yaml
    from avdino import submit_models as SM
    cmds = SM.main(["--models", "multi_central", "image_simple", "--training_mode", "mse",
                    "--config", CFG, "--dry-run"])
    assert cmds[0][1:] == ["-m", "avdino.run_dino", "--model", "multi_central", "--config", CFG,
                           "--metric", "mlp_acc", "--training_mode", "mse"]
    assert "--unimodal_model" in cmds[1] and "--training_mode" not in cmds[1]
    with pytest.raises(SystemExit):
        SM.main(["--models", "multi_vit", "--config", CFG, "--dry-run"])
    cfg = yaml.safe_load(open(CFG))
    cfg["hardware"]["num_gpus"] = 8
    p8 = tmp_path / "c8.yaml"
    p8.write_text(yaml.safe_dump(cfg))
    c8 = SM.main(["--models", "multi_central", "--config", str(p8), "--dry-run"])[0]
    assert "torch.distributed.run" in c8 and "--nproc-per-node=8" in c8
