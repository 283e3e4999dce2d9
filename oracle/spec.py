"""Architecture tables and state-dict specs for the oracle.

TEST INFRASTRUCTURE ONLY: nothing under ``oracle/`` is imported by the product
path (``multimodal-ssl-avmnist_amd/``).  Only ``tests/``, ``__graft_entry__.smoke``
and ``bench.py``'s ``cpu_baseline`` leg use it, as the checker.

The tables restate the module trees of the reference so that parameter names,
shapes and order match its ``state_dict`` exactly:

* CentralNet LeNets  -- reference models/unimodal.py:105-221
  (conv5x5 -> BN2d -> ReLU -> maxpool2, headless; fc1/fc2 built but unused)
* 3x3 CNNs           -- reference models/dino.py:18-73 (image_encoder / audio_encoder)
* CentralMultiModalEncoder -- models/dino.py:454-468 (+ fusion from 214-234)
* SimpleMultiModalEncoder  -- models/dino.py:214-234 (image_encoder / audio_encoder + fusion)
* ProjectionHead     -- models/dino.py:1240-1254
* MultiModalDINO(+MSE/INFONCE/SemiSupervised) -- models/dino.py:588-632, 964-970,
  1053-1058, 1156-1161
* UniModalDINO + ImageEncoder -- models/dino.py:1257-1297, 483-499
* MultiModalSimCLRModel -- other_ssl/multimodal_simclr/multimodal_simclr.py:12-20
"""
from collections import OrderedDict

# (cin, cout, k, pad) per conv block; every block is conv -> BN -> ReLU -> maxpool2
CENTRAL_IMAGE = dict(convs=[(1, 32, 5, 2), (32, 64, 5, 0)], hw=28, flat=64 * 5 * 5,
                     fc1=(1024, 64 * 5 * 5), fc2=(10, 1024), gap=False)
CENTRAL_AUDIO = dict(convs=[(1, 8, 5, 2), (8, 16, 5, 2), (16, 32, 5, 2), (32, 64, 5, 2)],
                     hw=112, flat=64 * 7 * 7, fc1=(1024, 64 * 7 * 7), fc2=(10, 1024), gap=False)
# 3x3 CNNs end in AdaptiveAvgPool2d(1) + Flatten + Linear(cout_last, out)
CNN3_IMAGE = dict(convs=[(1, 32, 3, 1), (32, 64, 3, 1), (64, 128, 3, 1)], hw=28, flat=128, gap=True)
CNN3_AUDIO = dict(convs=[(1, 32, 3, 1), (32, 64, 3, 1), (64, 128, 3, 1), (128, 256, 3, 1)],
                  hw=112, flat=256, gap=True)

PROJ_HIDDEN = 512


def _dense(sd, key, out_f, in_f, conv_k=None):
    shape = (out_f, in_f, conv_k, conv_k) if conv_k else (out_f, in_f)
    sd[key + ".weight"] = (shape, "dense_w")
    sd[key + ".bias"] = ((out_f,), "dense_b")


def _bn(sd, key, c):
    sd[key + ".weight"] = ((c,), "bn_w")
    sd[key + ".bias"] = ((c,), "bn_b")
    sd[key + ".running_mean"] = ((c,), "rm")
    sd[key + ".running_var"] = ((c,), "rv")
    sd[key + ".num_batches_tracked"] = ((), "nbt")


def central_lenet_spec(sd, prefix, arch):
    """CentralUnimodalImage/Audio: conv{i}, bn{i}, (dropout), fc1, fc2."""
    for i, (ci, co, k, _p) in enumerate(arch["convs"], 1):
        _dense(sd, f"{prefix}.conv{i}", co, ci, k)
        _bn(sd, f"{prefix}.bn{i}", co)
    _dense(sd, f"{prefix}.fc1", *arch["fc1"])
    _dense(sd, f"{prefix}.fc2", *arch["fc2"])


def cnn3_spec(sd, prefix, arch, out_dim):
    """nn.Sequential(conv,bn,relu,pool, ... , gap, flatten, linear): conv at 4i, bn at 4i+1."""
    n = len(arch["convs"])
    for i, (ci, co, k, _p) in enumerate(arch["convs"]):
        _dense(sd, f"{prefix}.{4 * i}", co, ci, k)
        _bn(sd, f"{prefix}.{4 * i + 1}", co)
    _dense(sd, f"{prefix}.{4 * n + 2}", out_dim, arch["flat"])


def central_multimodal_spec(sd, prefix, E, D):
    central_lenet_spec(sd, f"{prefix}.image_encoder.0", CENTRAL_IMAGE)
    _dense(sd, f"{prefix}.image_encoder.1", E, CENTRAL_IMAGE["flat"])
    central_lenet_spec(sd, f"{prefix}.audio_encoder.0", CENTRAL_AUDIO)
    _dense(sd, f"{prefix}.audio_encoder.1", E, CENTRAL_AUDIO["flat"])
    _dense(sd, f"{prefix}.fusion.0", E, 2 * E)
    _dense(sd, f"{prefix}.fusion.3", D, E)


def simple_multimodal_spec(sd, prefix, E, D):
    """SimpleMultiModalEncoder (models/dino.py:214-234, ``--model multi_simple``):
    image_encoder(E), audio_encoder(E), fusion -- registration order = state-dict order."""
    cnn3_spec(sd, f"{prefix}.image_encoder", CNN3_IMAGE, E)
    cnn3_spec(sd, f"{prefix}.audio_encoder", CNN3_AUDIO, E)
    _dense(sd, f"{prefix}.fusion.0", E, 2 * E)
    _dense(sd, f"{prefix}.fusion.3", D, E)


MULTIMODAL_ENCODERS = {"multi_central": central_multimodal_spec, "multi_simple": simple_multimodal_spec}


def projection_head_spec(sd, prefix, in_dim, out_dim, hidden=PROJ_HIDDEN):
    _dense(sd, f"{prefix}.mlp.0", hidden, in_dim)
    _bn(sd, f"{prefix}.mlp.1", hidden)
    _dense(sd, f"{prefix}.mlp.4", out_dim, hidden)


def multimodal_dino_spec(mode="mse", E=256, D=256, P=128, num_classes=10, encoder="multi_central"):
    """State-dict spec of MultiModalDINO* with CentralMultiModalEncoder (``multi_central``) or
    SimpleMultiModalEncoder (``multi_simple``)."""
    build = MULTIMODAL_ENCODERS[encoder]
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")
    build(sd, "student", E, D)
    build(sd, "teacher", E, D)
    projection_head_spec(sd, "student_projection", D, P)
    projection_head_spec(sd, "teacher_projection", D, P)
    if mode in ("mse", "infonce"):
        projection_head_spec(sd, "image_projection_head", E, P)
        projection_head_spec(sd, "audio_projection_head", E, P)
    elif mode == "semi_supervised":
        projection_head_spec(sd, "image_classifier", E, num_classes)
        projection_head_spec(sd, "audio_classifier", E, num_classes)
    elif mode != "default":
        raise ValueError(mode)
    return sd


def image_encoder_spec(sd, prefix, out_dim):
    """ImageEncoder (models/dino.py:483-499): encoder=image_encoder(512), projection=Linear(512,out)."""
    cnn3_spec(sd, f"{prefix}.encoder", CNN3_IMAGE, 512)
    _dense(sd, f"{prefix}.projection.0", out_dim, 512)


def spectrogram_encoder_spec(sd, prefix, out_dim):
    """SpectrogramEncoder (models/dino.py:502-513): encoder=audio_encoder(out)."""
    cnn3_spec(sd, f"{prefix}.encoder", CNN3_AUDIO, out_dim)


def unimodal_image_dino_spec(D=256, P=128):
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")  # module-own buffers precede children in state_dict
    image_encoder_spec(sd, "student", D)
    image_encoder_spec(sd, "teacher", D)
    projection_head_spec(sd, "student_projection", D, P)
    projection_head_spec(sd, "teacher_projection", D, P)
    return sd


def spectrogram_central_spec(sd, prefix, out_dim):
    """SpectrogramEncoderCentral (models/dino.py:515-523): CentralUnimodalAudio + Linear(3136,out)."""
    central_lenet_spec(sd, f"{prefix}.encoder.0", CENTRAL_AUDIO)
    _dense(sd, f"{prefix}.encoder.1", out_dim, 64 * 7 * 7)


def unimodal_dino_spec(modality="image", D=256, P=128):
    """UniModalDINO (models/dino.py:1257-1297) over an UNIMODAL_MODEL_MAP encoder
    (run_dino.py:542-550): "image"/"image_simple", "audio"/"spectrogram_simple",
    "spectrogram_central"."""
    kind = {"image": "image_simple", "audio": "spectrogram_simple"}.get(modality, modality)
    if kind == "image_simple":
        return unimodal_image_dino_spec(D, P)
    build = {"spectrogram_simple": spectrogram_encoder_spec,
             "spectrogram_central": spectrogram_central_spec}[kind]
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")
    build(sd, "student", D)
    build(sd, "teacher", D)
    projection_head_spec(sd, "student_projection", D, P)
    projection_head_spec(sd, "teacher_projection", D, P)
    return sd


def simclr_spec(D=256, P=256):
    sd = OrderedDict()
    image_encoder_spec(sd, "image_encoder", D)
    spectrogram_encoder_spec(sd, "audio_encoder", D)
    projection_head_spec(sd, "image_projection_head", D, P)
    projection_head_spec(sd, "audio_projection_head", D, P)
    return sd


def is_live_student(key, mode):
    """Parameters that receive gradients (fc1/fc2 of the LeNets never run)."""
    if ".fc1." in key or ".fc2." in key:
        return False
    if key.startswith("teacher") or key == "center":
        return False
    return True


def classifier_spec(D, hidden=128, num_classes=10):
    """DownstreamClassifier.classifier (models/dino.py:1782-1786): Linear(D,128)-ReLU-Linear(128,10)."""
    sd = OrderedDict()
    _dense(sd, "classifier.0", hidden, D)
    _dense(sd, "classifier.2", num_classes, hidden)
    return sd
