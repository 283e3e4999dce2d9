"""Generate golden vectors by running the REFERENCE hot path in this container.

Usage (only where /root/reference exists; the GPU box never runs this):
    python tests/golden/gen_golden.py [--out tests/golden]

How the reference is run: the reference is pure Python; its
hot-path modules import only fine after placeholder modules for the absent
third-party packages (lightning, torchvision, torchaudio, torchmetrics) are put
first on sys.path.  Those placeholders are written to /tmp at run time and are
never part of this repo.  The *Lightning wrappers are not instantiated (their
__init__ loads AVMNIST data from disk, models/dino.py:795-802); the loss methods
are called unbound with a SimpleNamespace as ``self`` and Lightning's automatic
optimisation order is replayed by hand: forward -> loss -> update_teacher
(dino.py:1233) -> zero_grad -> backward -> Adam.step (dino.py:953-962).

All dropout modules are set to p=0 so the vectors are deterministic.
Parameters and inputs come from oracle/params.py (a pure function of seed and
state-dict key), so fixtures only hold outputs.

Each fixture stores, per tensor: the full array when it has <= FULL_MAX
elements, otherwise its float64 sum, L2 norm and SAMPLE entries at seeded
indices (the check is then on those size-independent properties).
"""
import argparse
import os
import sys
import textwrap
import types
import zlib

import numpy as np

REF = "/root/reference/AVMNIST_Experiments"
STUB_DIR = "/tmp/avdino_ref_stubs"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import spec as ospec  # noqa: E402
from oracle.params import make_state, make_multimodal_batch, make_simclr_batch  # noqa: E402

FULL_MAX = 8192
SAMPLE = 256

STUBS = {
    "lightning/__init__.py": "from . import pytorch\n",
    "lightning/pytorch/__init__.py": textwrap.dedent("""
        import torch.nn as nn
        class LightningModule(nn.Module):
            def save_hyperparameters(self, *a, **k): pass
            def log(self, *a, **k): pass
        class LightningDataModule: pass
        class Callback: pass
        def seed_everything(*a, **k): pass
        """),
    "lightning/pytorch/callbacks.py": "class ModelCheckpoint: pass\n",
    "lightning/pytorch/loggers.py": "class CSVLogger: pass\n",
    "torchvision/__init__.py": "from . import transforms, models\n",
    "torchvision/transforms.py": "".join(
        f"class {n}:\n    def __init__(self, *a, **k): pass\n"
        for n in ["Compose", "RandomResizedCrop", "RandomRotation", "RandomAffine",
                  "RandomErasing", "RandomApply", "ElasticTransform", "GaussianBlur",
                  "Resize", "ToTensor", "Normalize", "RandomCrop", "Lambda"]),
    "torchvision/models/__init__.py": "",
    "torchvision/models/mobilenetv3.py": "def mobilenet_v3_small(*a, **k): raise RuntimeError('stub')\n",
    "torchvision/models/resnet.py": "def resnet18(*a, **k): raise RuntimeError('stub')\n",
    "torchaudio/__init__.py": "from . import transforms\n",
    "torchaudio/transforms.py": "".join(
        f"class {n}:\n    def __init__(self, *a, **k): pass\n"
        for n in ["TimeStretch", "FrequencyMasking", "TimeMasking", "Spectrogram"]),
    "torchmetrics/__init__.py": "",
    "torchinfo/__init__.py": "def summary(*a, **k): raise RuntimeError('stub')\n",
    "torchmetrics/classification.py": "class Accuracy:\n    def __init__(self, *a, **k): pass\n",
}


def write_stubs():
    for rel, src in STUBS.items():
        path = os.path.join(STUB_DIR, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(src)
    sys.path.insert(0, REF)
    sys.path.insert(0, STUB_DIR)


STORE = {"dtype": np.float32}


def summarize(prefix, arr, out):
    """Store a tensor fully or as (sum, norm, sampled entries)."""
    a = np.asarray(arr, dtype=np.float64)
    if a.size <= FULL_MAX:
        out[prefix] = a.astype(STORE["dtype"])
        return
    flat = a.reshape(-1)
    g = np.random.Generator(np.random.PCG64([zlib.crc32(prefix.encode()), 3]))
    idx = np.sort(g.choice(flat.size, size=SAMPLE, replace=False))
    out[prefix + "@sum"] = np.float64(flat.sum())
    out[prefix + "@norm"] = np.float64(np.sqrt((flat * flat).sum()))
    out[prefix + "@idx"] = idx.astype(np.int64)
    out[prefix + "@val"] = flat[idx].astype(STORE["dtype"])


def load_into(model, spec, state):
    import torch
    sd = model.state_dict()
    keys = list(sd.keys())
    assert keys == list(spec.keys()), (
        "state-dict key mismatch:\n" +
        "\n".join(f"{a} | {b}" for a, b in zip(keys, spec.keys()) if a != b)[:2000])
    for k, (shp, _kind) in spec.items():
        assert tuple(sd[k].shape) == tuple(shp), (k, sd[k].shape, shp)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})


def zero_dropout(model):
    import torch.nn as nn
    for m in model.modules():
        if isinstance(m, nn.Dropout):
            m.p = 0.0


HP = dict(lr=1e-4, wd=1e-6, momentum=0.996, center_momentum=0.9, tau_s=0.1, tau_t=0.04)


def multimodal_case(name, mode, E, D, P, B, G, L, pseed, bseed, steps, out_dir, dt="float32",
                    encoder="multi_central"):
    import torch
    dt = getattr(torch, dt)
    import torch.nn as nn
    import models.dino as rd

    cls = {"default": rd.MultiModalDINO, "mse": rd.MultiModalDINOWithMSE,
           "infonce": rd.MultiModalDINOWithINFONCE,
           "semi_supervised": rd.MultiModalDINOSemiSupervised}[mode]
    lcls = {"default": rd.MultiModalDINOLightning, "mse": rd.MultiModalDINOWithMSELightning,
            "infonce": rd.MultiModalDINOWithINFONCELightning,
            "semi_supervised": rd.MultiModalDINOSemiSupervisedLightning}[mode]
    torch.manual_seed(0)
    enc = {"multi_central": rd.CentralMultiModalEncoder,
           "multi_simple": rd.SimpleMultiModalEncoder}[encoder]   # run_dino.py:530-540
    model = cls(encoder_class=enc, output_dim=D, encoder_output_dim=E,
                projection_dim=P, momentum=HP["momentum"], center_momentum=HP["center_momentum"],
                dropout=0.0)
    spec = ospec.multimodal_dino_spec(mode, E, D, P, encoder=encoder)
    state = make_state(spec, pseed)
    load_into(model, spec, state)
    zero_dropout(model)
    model = model.to(dt)
    model.train()
    selfns = types.SimpleNamespace(student_temperature=HP["tau_s"], teacher_temperature=HP["tau_t"],
                                   alpha=1, ce_loss=nn.CrossEntropyLoss())
    opt = torch.optim.Adam(model.parameters(), lr=HP["lr"], weight_decay=HP["wd"])
    out = {"meta_mode": np.array(mode), "meta_dims": np.array([E, D, P, B, G, L, pseed, bseed]),
           "meta_encoder": np.array(encoder)}
    curve = []
    for step in range(steps):
        b = make_multimodal_batch(B, G, L, bseed + step)
        t = {k: torch.from_numpy(v) for k, v in b.items()}
        t = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in t.items()}
        views = (t["g_img"], t["g_aud"], t["l_img"], t["l_aud"])
        if mode == "default":
            s_out, t_out, _ = model(views)
            dino = lcls.dino_loss(selfns, s_out, t_out)
            aux = torch.zeros(())
            loss = dino
        else:
            f_i, f_a, s_out, t_out = model((t["image"], t["audio"], views))
            dino = lcls.dino_loss(selfns, s_out, t_out)
            if mode == "mse":
                aux = lcls.mse_loss(selfns, f_i, f_a)
            elif mode == "infonce":
                aux = lcls.infoNCE_loss(selfns, f_i, f_a)
            else:
                aux = lcls.supervised_loss(selfns, f_i, f_a, t["label"])
            loss = dino + 1 * aux
        model.update_teacher()
        opt.zero_grad()
        loss.backward()
        if step == 0:
            out["loss"] = np.float64(loss.item())
            out["dino_loss"] = np.float64(dino.item())
            out["aux_loss"] = np.float64(aux.item())
            summarize("s_out", s_out.detach().numpy(), out)
            summarize("t_out", t_out.detach().numpy(), out)
            if mode != "default":
                summarize("f_img", f_i.detach().numpy(), out)
                summarize("f_aud", f_a.detach().numpy(), out)
            for k, p in model.named_parameters():
                if p.grad is not None:
                    summarize("grad/" + k, p.grad.numpy(), out)
            out["live_keys"] = np.array([k for k, p in model.named_parameters() if p.grad is not None])
        opt.step()
        if step == 0:
            sd = model.state_dict()
            for k, v in sd.items():
                if k.endswith("running_mean") or k.endswith("running_var"):
                    summarize("rs/" + k, v.numpy(), out)
                elif k.startswith("teacher") and not k.endswith("num_batches_tracked"):
                    summarize("ema/" + k, v.numpy(), out)
                elif k == "center":
                    out["center_after"] = v.numpy().astype(STORE["dtype"])
                elif not k.endswith("num_batches_tracked"):
                    summarize("post/" + k, v.numpy(), out)
        curve.append(loss.item())
    out["curve"] = np.array(curve, np.float64)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)
    print(f"{name}: loss={out['loss']:.8f} curve={np.array(curve)}")


def unimodal_case(name, D, P, B, pseed, bseed, steps, out_dir, dt="float32", modality="image",
                  L=0, cos_alpha=0.0):
    import torch
    dt = getattr(torch, dt)
    import models.dino as rd
    torch.manual_seed(0)
    enc = {"image": rd.ImageEncoder, "audio": rd.SpectrogramEncoder,
           "spectrogram_central": rd.SpectrogramEncoderCentral}[modality]
    model = rd.UniModalDINO(encoder_class=enc, output_dim=D, projection_dim=P,
                            momentum=HP["momentum"], center_momentum=HP["center_momentum"],
                            dropout=0.0)
    spec = ospec.unimodal_dino_spec(modality, D, P)
    state = make_state(spec, pseed)
    load_into(model, spec, state)
    zero_dropout(model)
    model = model.to(dt)
    model.train()
    selfns = types.SimpleNamespace(student_temperature=HP["tau_s"], teacher_temperature=HP["tau_t"])
    opt = torch.optim.Adam(model.parameters(), lr=HP["lr"], weight_decay=HP["wd"])
    out = {"meta_dims": np.array([D, P, B, 2, L, pseed, bseed]), "meta_modality": np.array(modality),
           "meta_cos_alpha": np.float64(cos_alpha)}
    curve = []
    for step in range(steps):
        b = make_multimodal_batch(B, 2, L, bseed + step, with_originals=False)
        t = {k: torch.from_numpy(v).to(dt) for k, v in b.items()}
        s_out, t_out, emb = model((t["g_img"], t["g_aud"], t["l_img"], t["l_aud"]))
        # UniModalDINOLightning.training_step (dino.py:1637-1668), replayed unbound
        loss = rd.UniModalDINOLightning.dino_loss(selfns, s_out, t_out)
        if cos_alpha > 0:
            cos = rd.UniModalDINOLightning._cosine_consistency_loss(selfns, emb)
            loss = loss + cos_alpha * cos
        model.update_teacher()
        opt.zero_grad()
        loss.backward()
        if step == 0:
            out["loss"] = np.float64(loss.item())
            summarize("s_out", s_out.detach().numpy(), out)
            summarize("t_out", t_out.detach().numpy(), out)
            for k, p in model.named_parameters():
                if p.grad is not None:
                    summarize("grad/" + k, p.grad.numpy(), out)
            out["live_keys"] = np.array([k for k, p in model.named_parameters() if p.grad is not None])
        opt.step()
        if step == 0:
            for k, v in model.state_dict().items():
                if k.endswith("running_mean") or k.endswith("running_var"):
                    summarize("rs/" + k, v.numpy(), out)
                elif k == "center":
                    out["center_after"] = v.numpy().astype(STORE["dtype"])
                elif k.startswith("teacher") and not k.endswith("num_batches_tracked"):
                    summarize("ema/" + k, v.numpy(), out)
                elif not k.endswith("num_batches_tracked"):
                    summarize("post/" + k, v.numpy(), out)
        curve.append(loss.item())
    out["curve"] = np.array(curve, np.float64)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)
    print(f"{name}: loss={out['loss']:.8f} curve={np.array(curve)}")


def simclr_case(name, D, P, B, pseed, bseed, out_dir, dt="float32"):
    import torch
    dt = getattr(torch, dt)
    sys.path.insert(0, os.path.join(REF, "other_ssl", "multimodal_simclr"))
    import multimodal_simclr as rs
    out = {"meta_dims": np.array([D, P, B, pseed, bseed])}
    for mode in range(4):
        torch.manual_seed(0)
        model = rs.MultiModalSimCLRModel(output_dim=D, projection_dim=P)
        spec = ospec.simclr_spec(D, P)
        state = make_state(spec, pseed)
        load_into(model, spec, state)
        zero_dropout(model)
        model = model.to(dt)
        model.train()
        b = make_simclr_batch(B, bseed)
        t = [torch.from_numpy(b[k]).to(dt) for k in ("img1", "spec1", "img2", "spec2")]
        real_randint = torch.randint
        torch.randint = lambda *a, **k: torch.tensor([mode])
        real_float = torch.Tensor.float
        torch.Tensor.float = lambda self: self  # forward() calls .float(); keep dt
        try:
            z1, z2 = model(tuple(t))
        finally:
            torch.randint = real_randint
            torch.Tensor.float = real_float
        loss = rs.MultiModalSimCLRLightning.nt_xent_loss(None, torch.cat([z1, z2], 0))
        loss.backward()
        out[f"m{mode}/loss"] = np.float64(loss.item())
        summarize(f"m{mode}/z1", z1.detach().numpy(), out)
        summarize(f"m{mode}/z2", z2.detach().numpy(), out)
        for k, p in model.named_parameters():
            if p.grad is not None:
                summarize(f"m{mode}/grad/" + k, p.grad.numpy(), out)
        print(f"{name} mode {mode}: loss={loss.item():.8f}")
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)


def probe_case(name, kind, E, D, P, B, nb_train, nb_valid, pseed, bseed, out_dir, dt="float32",
               lr=1e-3):
    """on_train_epoch_end's linear probe (dino.py:878-951 / 1670-1735): DownstreamClassifier
    over a frozen copy of the student, the copy in train mode for the probe epoch, AdamW on the
    classifier, then evaluate() in eval mode.  Replayed on CPU without the CUDA-only fp16
    autocast / GradScaler; the copy's dropout set to 0."""
    import torch
    import torch.nn as nn
    dt = getattr(torch, dt)
    import models.dino as rd
    torch.manual_seed(0)
    if kind == "multi_central":
        model = rd.MultiModalDINO(encoder_class=rd.CentralMultiModalEncoder, output_dim=D,
                                  encoder_output_dim=E, projection_dim=P, dropout=0.0)
        spec = ospec.multimodal_dino_spec("default", E, D, P)
    else:
        enc = {"image_simple": rd.ImageEncoder, "spectrogram_simple": rd.SpectrogramEncoder}[kind]
        model = rd.UniModalDINO(encoder_class=enc, output_dim=D, projection_dim=P, dropout=0.0)
        spec = ospec.unimodal_dino_spec(kind, D, P)
    state = make_state(spec, pseed)
    load_into(model, spec, state)
    model = model.to(dt)
    clf = rd.DownstreamClassifier(model, trainable_encoder=False).to(dt)
    zero_dropout(clf)
    cspec = ospec.classifier_spec(D)
    cstate = make_state(cspec, pseed + 1)
    with torch.no_grad():
        for k, v in cstate.items():
            dict(clf.named_parameters())[k].copy_(torch.from_numpy(v).to(dt))
    crit = nn.CrossEntropyLoss()
    opt = torch.optim.AdamW(clf.classifier.parameters(), lr=lr)
    clf.train()
    out = {"meta_dims": np.array([E, D, P, B, nb_train, nb_valid, pseed, bseed]),
           "meta_kind": np.array(kind), "meta_lr": np.float64(lr)}
    losses = []
    for i in range(nb_train):
        b = make_multimodal_batch(B, 1, 0, bseed + i)
        im, au = torch.from_numpy(b["image"]).to(dt), torch.from_numpy(b["audio"]).to(dt)
        opt.zero_grad()
        loss = crit(clf(im, au), torch.from_numpy(b["label"]))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    out["train_losses"] = np.array(losses, np.float64)
    clf.eval()
    tot, correct, n, logits = 0.0, 0, 0, []
    with torch.no_grad():
        for i in range(nb_valid):
            b = make_multimodal_batch(B, 1, 0, bseed + 1000 + i)
            im, au = torch.from_numpy(b["image"]).to(dt), torch.from_numpy(b["audio"]).to(dt)
            o = clf(im, au)
            lab = torch.from_numpy(b["label"])
            tot += crit(o, lab).item()
            correct += int((o.argmax(1) == lab).sum())
            n += len(lab)
            logits.append(o.numpy())
    out["eval_loss"] = np.float64(tot / nb_valid)
    out["mlp_acc"] = np.float64(100.0 * correct / n)
    summarize("logits", np.concatenate(logits), out)
    for k, v in clf.named_parameters():
        if k.startswith("classifier"):
            summarize("cls/" + k, v.detach().numpy(), out)
    for k, v in clf.encoder.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            summarize("rs/student." + k, v.numpy(), out)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)
    print(f"{name}: train losses {np.array(losses)} eval {out['eval_loss']:.6f} acc {out['mlp_acc']}")


def downstream_case(name, kind, E, D, P, B, nb_train, nb_valid, nb_test, epochs, pseed, bseed,
                    out_dir, dt="float32", lr=1e-3):
    """compute_accuracies' two evaluations (run_dino.py:481-501), by calling the reference's
    own training_structures/dino_train.py functions on CPU:
      train_knn_classifier (349-369): FeatureExtractor + sklearn KNeighborsClassifier(5);
      train_downstream (188-329): DownstreamClassifier, AdamW + CosineAnnealingLR, best-val
        checkpoint, test evaluation (the CUDA-only autocast / GradScaler disable themselves).
    Harness-only changes: DownstreamClassifier / FeatureExtractor are subclassed inside
    dino_train's namespace to (a) load the classifier weights from oracle/params.py instead of
    torch's RNG and (b) cast the inputs to the run dtype (the functions cast them to float32);
    the model's dropout is set to 0."""
    import csv as _csv
    import tempfile
    import torch
    from torch.utils.data import DataLoader, TensorDataset
    dtt = getattr(torch, dt)
    import models.dino as rd
    import training_structures.dino_train as tdt
    torch.manual_seed(0)
    if kind == "multi_central":
        model = rd.MultiModalDINO(encoder_class=rd.CentralMultiModalEncoder, output_dim=D,
                                  encoder_output_dim=E, projection_dim=P, dropout=0.0)
        spec = ospec.multimodal_dino_spec("default", E, D, P)
    else:
        enc = {"image_simple": rd.ImageEncoder, "spectrogram_simple": rd.SpectrogramEncoder}[kind]
        model = rd.UniModalDINO(encoder_class=enc, output_dim=D, projection_dim=P, dropout=0.0)
        spec = ospec.unimodal_dino_spec(kind, D, P)
    state = make_state(spec, pseed)
    load_into(model, spec, state)
    zero_dropout(model)
    model = model.to(dtt)
    cstate = make_state(ospec.classifier_spec(D), pseed + 1)

    class DC(rd.DownstreamClassifier):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.to(dtt)
            with torch.no_grad():
                for kk, v in cstate.items():
                    dict(self.named_parameters())[kk].copy_(torch.from_numpy(v).to(dtt))

        def forward(self, images, spectrograms=None):
            return super().forward(images.to(dtt), None if spectrograms is None else spectrograms.to(dtt))

    class FE(rd.FeatureExtractor):
        def forward(self, images, spectrograms=None):
            return super().forward(images.to(dtt), None if spectrograms is None else spectrograms.to(dtt))

    tdt.DownstreamClassifier, tdt.FeatureExtractor = DC, FE

    def loader(n, seed):
        bs = [make_multimodal_batch(B, 1, 0, seed + i) for i in range(n)]
        cat = lambda k: torch.from_numpy(np.concatenate([b[k] for b in bs]))  # noqa: E731
        return DataLoader(TensorDataset(cat("image"), cat("audio"), cat("label")), batch_size=B,
                          shuffle=False)

    tr, va, te = loader(nb_train, bseed), loader(nb_valid, bseed + 1000), loader(nb_test, bseed + 2000)
    out = {"meta_dims": np.array([E, D, P, B, nb_train, nb_valid, nb_test, epochs, pseed, bseed]),
           "meta_kind": np.array(kind), "meta_lr": np.float64(lr)}
    knn, acc = tdt.train_knn_classifier(model, tr, te, n_neighbors=5, device="cpu")
    fe = FE(model)
    trf, _ = tdt.feature_extraction_loop("cpu", fe, tr)
    tef, tel = tdt.feature_extraction_loop("cpu", fe, te)
    out["knn_acc"] = np.float64(acc)
    out["knn_pred"] = knn.predict(tef).astype(np.int64)
    out["knn_nbr"] = knn.kneighbors(tef, return_distance=False).astype(np.int64)
    summarize("feat_train", trf, out)
    summarize("feat_test", tef, out)
    with tempfile.TemporaryDirectory() as tmp:
        clf = tdt.train_downstream(model, tr, va, te, num_epochs=epochs, device="cpu",
                                   learning_rate=lr, save_path=f"{tmp}/d/m.pt",
                                   train_log_path=f"{tmp}/d/train.csv",
                                   test_log_path=f"{tmp}/d/test.csv")
        logs = sorted(os.listdir(f"{tmp}/d"))
        tr_log = [f for f in logs if f.startswith("train")][0]
        te_log = [f for f in logs if f.startswith("test")][0]
        with open(f"{tmp}/d/{tr_log}") as f:
            rows = list(_csv.reader(f))[1:]
        out["history"] = np.array([[float(r[1]), float(r[2]), float(r[3])] for r in rows], np.float64)
        with open(f"{tmp}/d/{te_log}") as f:
            rows = list(_csv.reader(f))[1:]
        out["test_preds"] = np.array([int(r[1]) for r in rows], np.int64)
        out["test_labels"] = np.array([int(r[0]) for r in rows], np.int64)
    met = tdt.compute_classification_metrics(clf, te, device="cpu")
    out["test_acc"] = np.float64(met["accuracy"])
    out["confusion_matrix"] = met["confusion_matrix"].astype(np.int64)
    for k, v in clf.named_parameters():
        if k.startswith("classifier"):
            summarize("cls/" + k, v.detach().numpy(), out)
    for k, v in clf.encoder.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            summarize("rs/student." + k, v.numpy(), out)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)
    print(f"{name}: knn {acc:.2f}% history {out['history'].tolist()} test {out['test_acc']:.2f}%")


def pretrain_case(name, D, P, B, pseed, bseed, epochs, nb, out_dir, dt="float32", lr=1e-4):
    """training_structures/dino_train.py:104-186 pretrain_dino (BASELINE config 1's CPU path),
    by calling the reference's own function on CPU: AdamW(model.parameters(), lr) (torch's
    default weight_decay 0.01), per batch zero_grad -> forward -> dino_loss(tau_s=0.1,
    tau_t=0.04) -> backward -> step -> update_teacher (EMA AFTER the step, unlike the Lightning
    path), epochs x nb batches of UniModalDINO(ImageEncoder) over 2 global views.
    Harness-only adapters: the reference's current UniModalDINO.forward returns (student,
    teacher, embeddings) while pretrain_dino unpacks two values, so a wrapper returns the first
    two; dino_loss is UniModalDINOLightning.dino_loss called unbound with the given
    temperatures (recording each step's loss); dropout 0."""
    import csv as _csv
    import tempfile
    import torch
    from torch.utils.data import DataLoader, TensorDataset
    dtt = getattr(torch, dt)
    import models.dino as rd
    import training_structures.dino_train as tdt
    torch.manual_seed(0)
    model = rd.UniModalDINO(encoder_class=rd.ImageEncoder, output_dim=D, projection_dim=P,
                            momentum=HP["momentum"], center_momentum=HP["center_momentum"], dropout=0.0)
    spec = ospec.unimodal_dino_spec("image", D, P)
    state = make_state(spec, pseed)
    load_into(model, spec, state)
    zero_dropout(model)
    model = model.to(dtt)

    class Two(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, batch):
            s_out, t_out, _ = self.m(batch)
            return s_out, t_out

        def update_teacher(self):
            self.m.update_teacher()

    losses = []

    def dino_loss(s_out, t_out, tau_s=0.1, tau_t=0.04):
        ns = types.SimpleNamespace(student_temperature=tau_s, teacher_temperature=tau_t)
        loss = rd.UniModalDINOLightning.dino_loss(ns, s_out, t_out)
        losses.append(loss.item())
        return loss

    bs = [make_multimodal_batch(B, 2, 0, bseed + i, with_originals=False) for i in range(nb)]
    cat = lambda k: torch.from_numpy(np.concatenate([b[k] for b in bs])).to(dtt)  # noqa: E731
    loader = DataLoader(TensorDataset(cat("g_img"), cat("g_aud"), cat("l_img"), cat("l_aud")),
                        batch_size=B, shuffle=False)
    with tempfile.TemporaryDirectory() as tmp:
        tdt.pretrain_dino(Two(model), loader, dino_loss, num_epochs=epochs, learning_rate=lr,
                          save_path=f"{tmp}/p/m.pt", log_path=f"{tmp}/p/log.csv")
        log = [f for f in os.listdir(f"{tmp}/p") if f.startswith("log")][0]
        with open(f"{tmp}/p/{log}") as f:
            rows = list(_csv.reader(f))[1:]
    out = {"meta_dims": np.array([D, P, B, epochs, nb, pseed, bseed]), "meta_lr": np.float64(lr),
           "step_losses": np.array(losses, np.float64),
           "epoch_losses": np.array([float(r[1]) for r in rows], np.float64)}
    for k, v in model.state_dict().items():
        if k == "center":
            out["center"] = v.numpy().astype(STORE["dtype"])
        elif not k.endswith("num_batches_tracked"):
            summarize("state/" + k, v.numpy(), out)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **out)
    print(f"{name}: step losses {np.array(losses)} epochs {out['epoch_losses']}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default="", help="comma-separated case names (default: all)")
    args = ap.parse_args()
    write_stubs()
    import torch
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    o = args.out
    only = set(args.only.split(",")) if args.only else None
    # Each case twice: the reference executed in fp32 (its CPU numerics) and in float64
    # (the same algorithm without rounding noise: the tight pin for the oracle).
    cases = [
        ("mm_mse_small", multimodal_case, ("mse", 32, 32, 16, 4, 2, 4, 101, 1001, 5), {}),
        ("mm_default_small", multimodal_case, ("default", 32, 32, 16, 4, 2, 4, 102, 1002, 3), {}),
        ("mm_infonce_small", multimodal_case, ("infonce", 32, 32, 16, 4, 2, 4, 103, 1003, 3), {}),
        ("mm_semi_small", multimodal_case, ("semi_supervised", 32, 32, 16, 4, 2, 4, 104, 1004, 3), {}),
        # full E=D=256, P=128 dims, a 5-step free-running curve (north_star's 1e-4 loss-curve bar)
        ("mm_mse_full", multimodal_case, ("mse", 256, 256, 128, 2, 2, 4, 105, 1005, 5), {}),
        # --model multi_simple (SimpleMultiModalEncoder over the 3x3 image/audio encoders)
        ("mm_simple_mse_small", multimodal_case, ("mse", 32, 32, 16, 3, 2, 2, 116, 1016, 3),
         dict(encoder="multi_simple")),
        ("mm_simple_default_small", multimodal_case, ("default", 32, 32, 16, 3, 2, 2, 117, 1017, 2),
         dict(encoder="multi_simple")),
        ("uni_image_g2l0", unimodal_case, (256, 128, 8, 106, 1006, 3), {}),
        ("uni_image_g2l4_cos", unimodal_case, (64, 32, 6, 108, 1008, 3),
         dict(modality="image", L=4, cos_alpha=0.3)),
        ("uni_audio_g2l2_cos", unimodal_case, (64, 32, 3, 109, 1009, 2),
         dict(modality="audio", L=2, cos_alpha=0.3)),
        ("uni_speccentral_g2l2", unimodal_case, (32, 16, 3, 110, 1010, 2),
         dict(modality="spectrogram_central", L=2, cos_alpha=0.0)),
        ("probe_multi_central", probe_case, ("multi_central", 32, 32, 16, 6, 3, 2, 111, 1011), {}),
        ("probe_image_simple", probe_case, ("image_simple", 0, 64, 32, 6, 3, 2, 112, 1012), {}),
        ("simclr_small", simclr_case, (256, 256, 4, 107, 1007), {}),
        ("pretrain_image_simple", pretrain_case, (64, 32, 8, 115, 1015, 2, 2), {}),
        ("downstream_multi_central", downstream_case,
         ("multi_central", 32, 32, 16, 8, 4, 2, 2, 3, 113, 1013), {}),
        ("downstream_image_simple", downstream_case,
         ("image_simple", 0, 64, 32, 8, 4, 2, 2, 3, 114, 1014), {}),
    ]
    # Each case twice: the reference executed in fp32 (its CPU numerics) and in float64
    # (the same algorithm without rounding noise: the tight pin for the oracle).
    for dt, sfx, store in (("float32", "", np.float32), ("float64", "_f64", np.float64)):
        STORE["dtype"] = store
        for name, fn, a, kw in cases:
            if only is None or name in only:
                fn(name + sfx, *a, out_dir=o, dt=dt, **kw)


if __name__ == "__main__":
    main()
