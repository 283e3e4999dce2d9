"""Architecture tables of the reference's hot-path models and their state-dict layout.

Names, shapes and order reproduce the reference's ``state_dict`` keys exactly so that
checkpoints interoperate:
  CentralUnimodalImage/Audio      reference models/unimodal.py:105-221
  image_encoder / audio_encoder   models/dino.py:18-73
  CentralMultiModalEncoder        models/dino.py:454-468 (fusion: 214-234)
  SimpleMultiModalEncoder         models/dino.py:214-234 (image_encoder / audio_encoder, 18-73)
  ProjectionHead                  models/dino.py:1240-1254
  MultiModalDINO*                 models/dino.py:588-632, 964-970, 1053-1058, 1156-1161
  UniModalDINO / ImageEncoder     models/dino.py:1257-1297, 483-499
  SpectrogramEncoder              models/dino.py:502-513
  MultiModalSimCLRModel           other_ssl/multimodal_simclr/multimodal_simclr.py:12-20
"""
from collections import OrderedDict


class ConvStackSpec:
    """[conv(K, pad) -> BN2d -> ReLU -> maxpool2] x L (+ AdaptiveAvgPool2d(1) if gap)."""

    def __init__(self, convs, hw, gap, conv_keys, bn_keys):
        self.convs = convs            # [(cin, cout, k, pad)]
        self.hw = hw
        self.gap = gap
        self.conv_keys = conv_keys
        self.bn_keys = bn_keys

    def layer_dims(self):
        """[(H_in, Ho, Hpool)] per layer (square maps)."""
        out, h = [], self.hw
        for (_ci, _co, k, pad) in self.convs:
            ho = h + 2 * pad - k + 1
            out.append((h, ho, ho // 2))
            h = ho // 2
        return out

    @property
    def flat(self):
        co = self.convs[-1][1]
        hp = self.layer_dims()[-1][2]
        return co if self.gap else co * hp * hp


CENTRAL_IMAGE_CONVS = [(1, 32, 5, 2), (32, 64, 5, 0)]
CENTRAL_AUDIO_CONVS = [(1, 8, 5, 2), (8, 16, 5, 2), (16, 32, 5, 2), (32, 64, 5, 2)]
CNN3_IMAGE_CONVS = [(1, 32, 3, 1), (32, 64, 3, 1), (64, 128, 3, 1)]
CNN3_AUDIO_CONVS = [(1, 32, 3, 1), (32, 64, 3, 1), (64, 128, 3, 1), (128, 256, 3, 1)]
PROJ_HIDDEN = 512


def central_stack(prefix, convs, hw):
    n = len(convs)
    return ConvStackSpec(convs, hw, False, [f"{prefix}.conv{i + 1}" for i in range(n)],
                         [f"{prefix}.bn{i + 1}" for i in range(n)])


def cnn3_stack(prefix, convs, hw):
    n = len(convs)
    return ConvStackSpec(convs, hw, True, [f"{prefix}.{4 * i}" for i in range(n)],
                         [f"{prefix}.{4 * i + 1}" for i in range(n)])


# ------------------------------------------------------------------ state-dict builders
def _dense(sd, key, out_f, in_f, k=None):
    sd[key + ".weight"] = ((out_f, in_f, k, k) if k else (out_f, in_f), "w")
    sd[key + ".bias"] = ((out_f,), "b")


def _bn(sd, key, c):
    sd[key + ".weight"] = ((c,), "bn_w")
    sd[key + ".bias"] = ((c,), "bn_b")
    sd[key + ".running_mean"] = ((c,), "rm")
    sd[key + ".running_var"] = ((c,), "rv")
    sd[key + ".num_batches_tracked"] = ((), "nbt")


def _central_lenet(sd, prefix, convs, fc1_in):
    for i, (ci, co, k, _p) in enumerate(convs, 1):
        _dense(sd, f"{prefix}.conv{i}", co, ci, k)
        _bn(sd, f"{prefix}.bn{i}", co)
    _dense(sd, f"{prefix}.fc1", 1024, fc1_in)   # built but never executed (with_head=False)
    _dense(sd, f"{prefix}.fc2", 10, 1024)


def _cnn3(sd, prefix, convs, out_dim):
    n = len(convs)
    for i, (ci, co, k, _p) in enumerate(convs):
        _dense(sd, f"{prefix}.{4 * i}", co, ci, k)
        _bn(sd, f"{prefix}.{4 * i + 1}", co)
    _dense(sd, f"{prefix}.{4 * n + 2}", out_dim, convs[-1][1])


def central_multimodal_sd(sd, prefix, E, D):
    _central_lenet(sd, f"{prefix}.image_encoder.0", CENTRAL_IMAGE_CONVS, 64 * 5 * 5)
    _dense(sd, f"{prefix}.image_encoder.1", E, 64 * 5 * 5)
    _central_lenet(sd, f"{prefix}.audio_encoder.0", CENTRAL_AUDIO_CONVS, 64 * 7 * 7)
    _dense(sd, f"{prefix}.audio_encoder.1", E, 64 * 7 * 7)
    _dense(sd, f"{prefix}.fusion.0", E, 2 * E)
    _dense(sd, f"{prefix}.fusion.3", D, E)


def simple_multimodal_sd(sd, prefix, E, D):
    """SimpleMultiModalEncoder (``--model multi_simple``): image_encoder(E), audio_encoder(E)
    (nn.Sequential 3x3 CNNs, Linear at index 14 / 18), fusion."""
    _cnn3(sd, f"{prefix}.image_encoder", CNN3_IMAGE_CONVS, E)
    _cnn3(sd, f"{prefix}.audio_encoder", CNN3_AUDIO_CONVS, E)
    _dense(sd, f"{prefix}.fusion.0", E, 2 * E)
    _dense(sd, f"{prefix}.fusion.3", D, E)


# MODEL_MAP encoders that run on the engine (run_dino.py:530-540):
#   arch -> (image stack(prefix), image Linear key, audio stack(prefix), audio Linear key, sd builder)
MULTI_ENCODERS = {
    "multi_central": (lambda p: central_stack(f"{p}.image_encoder.0", CENTRAL_IMAGE_CONVS, 28), "image_encoder.1",
                      lambda p: central_stack(f"{p}.audio_encoder.0", CENTRAL_AUDIO_CONVS, 112), "audio_encoder.1",
                      central_multimodal_sd),
    "multi_simple": (lambda p: cnn3_stack(f"{p}.image_encoder", CNN3_IMAGE_CONVS, 28), "image_encoder.14",
                     lambda p: cnn3_stack(f"{p}.audio_encoder", CNN3_AUDIO_CONVS, 112), "audio_encoder.18",
                     simple_multimodal_sd),
}


def projection_head_sd(sd, prefix, in_dim, out_dim, hidden=PROJ_HIDDEN):
    _dense(sd, f"{prefix}.mlp.0", hidden, in_dim)
    _bn(sd, f"{prefix}.mlp.1", hidden)
    _dense(sd, f"{prefix}.mlp.4", out_dim, hidden)


HEAD_NAMES = {"mse": ("image_projection_head", "audio_projection_head"),
              "infonce": ("image_projection_head", "audio_projection_head"),
              "semi_supervised": ("image_classifier", "audio_classifier")}


def multimodal_dino_sd(mode, E, D, P, num_classes=10, encoder="multi_central"):
    build = MULTI_ENCODERS[encoder][4]
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")
    build(sd, "student", E, D)
    build(sd, "teacher", E, D)
    projection_head_sd(sd, "student_projection", D, P)
    projection_head_sd(sd, "teacher_projection", D, P)
    if mode in HEAD_NAMES:
        hi, ha = HEAD_NAMES[mode]
        out = num_classes if mode == "semi_supervised" else P
        projection_head_sd(sd, hi, E, out)
        projection_head_sd(sd, ha, E, out)
    elif mode != "default":
        raise ValueError(f"unknown training mode {mode!r}")
    return sd


def image_encoder_sd(sd, prefix, out_dim):
    _cnn3(sd, f"{prefix}.encoder", CNN3_IMAGE_CONVS, 512)
    _dense(sd, f"{prefix}.projection.0", out_dim, 512)


def spectrogram_encoder_sd(sd, prefix, out_dim):
    _cnn3(sd, f"{prefix}.encoder", CNN3_AUDIO_CONVS, out_dim)


def unimodal_image_dino_sd(D, P):
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")
    image_encoder_sd(sd, "student", D)
    image_encoder_sd(sd, "teacher", D)
    projection_head_sd(sd, "student_projection", D, P)
    projection_head_sd(sd, "teacher_projection", D, P)
    return sd


def spectrogram_central_sd(sd, prefix, out_dim):
    _central_lenet(sd, f"{prefix}.encoder.0", CENTRAL_AUDIO_CONVS, 64 * 7 * 7)
    _dense(sd, f"{prefix}.encoder.1", out_dim, 64 * 7 * 7)


# UNIMODAL_MODEL_MAP encoders that run on the engine (run_dino.py:542-550):
#   kind -> (modality, stack builder(prefix), [Linear keys after the stack, relative to prefix],
#            state-dict builder)
UNI_ENCODERS = {
    "image_simple": ("image", lambda p: cnn3_stack(f"{p}.encoder", CNN3_IMAGE_CONVS, 28),
                     ["encoder.14", "projection.0"], image_encoder_sd),
    "spectrogram_simple": ("audio", lambda p: cnn3_stack(f"{p}.encoder", CNN3_AUDIO_CONVS, 112),
                           ["encoder.18"], spectrogram_encoder_sd),
    "spectrogram_central": ("audio", lambda p: central_stack(f"{p}.encoder.0", CENTRAL_AUDIO_CONVS, 112),
                            ["encoder.1"], spectrogram_central_sd),
}
UNI_ALIASES = {"image": "image_simple", "audio": "spectrogram_simple"}


def unimodal_dino_sd(kind, D, P):
    """UniModalDINO (models/dino.py:1257-1297) state dict over an UNI_ENCODERS kind."""
    kind = UNI_ALIASES.get(kind, kind)
    build = UNI_ENCODERS[kind][3]
    sd = OrderedDict()
    sd["center"] = ((1, P), "center")
    build(sd, "student", D)
    build(sd, "teacher", D)
    projection_head_sd(sd, "student_projection", D, P)
    projection_head_sd(sd, "teacher_projection", D, P)
    return sd


def simclr_sd(D, P):
    sd = OrderedDict()
    image_encoder_sd(sd, "image_encoder", D)
    spectrogram_encoder_sd(sd, "audio_encoder", D)
    projection_head_sd(sd, "image_projection_head", D, P)
    projection_head_sd(sd, "audio_projection_head", D, P)
    return sd
