"""The Lightning-shaped boundary on CPU (no engine: no compute, no CPU fallback): module
structure, reference state-dict keys, .ckpt save/load (run_dino.py:379, 386) and the
best_augments mapping (objective_augment.py:68-96)."""
import os

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(REPO, "configs", "config_multimodal_dino.yaml")


def test_modules_are_nn_modules_with_reference_keys():
    from avdino.models import CentralMultiModalEncoder, MultiModalDINOWithMSELightning
    from oracle import spec as OS
    m = MultiModalDINOWithMSELightning(encoder_class=CentralMultiModalEncoder, encoder_output_dim=32,
                                       output_dim=32, projection_dim=16, device="cpu")
    assert isinstance(m, torch.nn.Module) and isinstance(m.model, torch.nn.Module)
    keys = list(m.state_dict().keys())
    assert keys == ["model." + k for k in OS.multimodal_dino_spec("mse", 32, 32, 16)]
    names = dict(m.named_parameters())
    assert names["model.arena"].requires_grad
    assert not names["model.teacher_arena"].requires_grad
    assert not names["model.arena_frozen"].requires_grad        # dead fc1/fc2: grad None
    with pytest.raises(RuntimeError, match="arenas"):
        m.to(torch.float64)
    with pytest.raises(RuntimeError):
        m.training_step(None, 0)                                  # no engine on CPU


def test_checkpoint_round_trip(tmp_path):
    from avdino.models import CentralMultiModalEncoder, MultiModalDINOWithINFONCELightning
    from avdino.trainer import load_checkpoint, save_checkpoint
    from oracle import spec as OS
    from oracle.params import make_state
    m = MultiModalDINOWithINFONCELightning(encoder_class=CentralMultiModalEncoder, encoder_output_dim=32,
                                           output_dim=32, projection_dim=16, device="cpu",
                                           learning_rate=3e-4, num_epochs=7)
    state = make_state(OS.multimodal_dino_spec("infonce", 32, 32, 16), 5)
    m.load_state_dict({"model." + k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    path = str(tmp_path / "x.ckpt")
    save_checkpoint(m, path, epoch=3, global_step=12)
    ck = load_checkpoint(path)
    assert ck["epoch"] == 3 and ck["global_step"] == 12
    assert ck["hyper_parameters"]["learning_rate"] == 3e-4
    assert ck["hyper_parameters"]["encoder_class"] == "CentralMultiModalEncoder"
    m2 = MultiModalDINOWithINFONCELightning.load_from_checkpoint(path, device="cpu")
    assert m2.learning_rate == 3e-4 and m2.num_epochs == 7
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    bad = dict(m.state_dict())
    bad.pop(next(iter(bad)))
    with pytest.raises(RuntimeError, match="Missing"):
        m2.load_state_dict(bad)


def test_process_augment_config():
    from avdino.augment import process_augment_config
    from avdino.run_dino import load_config
    cfg = load_config(CFG)
    out = process_augment_config(cfg)
    g = out["augmentations"]["global_views"]
    assert g["frequency_mask"] == {"freq_mask_param": 5}
    assert "p" not in g["random_resized_crop"]
    assert out["augmentation_probabilities"]["local_views"]["grouped_masking"] == pytest.approx(0.9763835472062644)
    with pytest.raises(ValueError):
        process_augment_config({})
