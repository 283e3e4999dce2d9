"""PyTorch-CPU restatement of the reference's multimodal-DINO step -- the CPU BASELINE.

TEST INFRASTRUCTURE ONLY (see oracle/spec.py): used by bench.py's cpu_baseline leg
("kind": "port") to time the reference algorithm on the GPU box's host cores, where the
reference itself does not exist.  It runs the same ATen ops in the same order as the
reference (per-view encoder calls, Python EMA loop, torch.optim.Adam), fp32:

  CentralUnimodalImage/Audio   models/unimodal.py:105-221
  CentralMultiModalEncoder     models/dino.py:454-468 (+ SimpleMultiModalEncoder 214-234)
  ProjectionHead               models/dino.py:1240-1254
  MultiModalDINO(+WithMSE)     models/dino.py:588-727, 1156-1171
  MultiModalDINOSemiSupervised models/dino.py:964-980 (mode="semi_supervised")
  dino_loss / mse_loss         models/dino.py:822-854, 1193-1211
  supervised_loss              models/dino.py:1001-1025
  step order                   dino.py:1214-1238 (1027-1051) + Lightning automatic optimisation
Checked against the numpy oracle in tests/test_torch_port.py.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class LeNetBlock(nn.Module):
    def __init__(self, convs, fc1_in):
        super().__init__()
        for i, (ci, co, k, p) in enumerate(convs, 1):
            setattr(self, f"conv{i}", nn.Conv2d(ci, co, k, padding=p))
            setattr(self, f"bn{i}", nn.BatchNorm2d(co))
        self.n = len(convs)
        self.dropout = nn.Dropout(0.5)
        self.fc1 = nn.Linear(fc1_in, 1024)
        self.fc2 = nn.Linear(1024, 10)

    def forward(self, x):
        for i in range(1, self.n + 1):
            x = F.max_pool2d(F.relu(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x))), 2)
        return x.view(x.size(0), -1)


class CentralMM(nn.Module):
    def __init__(self, E, D, fusion_dropout=0.3):
        super().__init__()
        self.image_encoder = nn.Sequential(LeNetBlock([(1, 32, 5, 2), (32, 64, 5, 0)], 1600),
                                           nn.Linear(1600, E))
        self.audio_encoder = nn.Sequential(
            LeNetBlock([(1, 8, 5, 2), (8, 16, 5, 2), (16, 32, 5, 2), (32, 64, 5, 2)], 3136),
            nn.Linear(3136, E))
        self.fusion = nn.Sequential(nn.Linear(2 * E, E), nn.ReLU(), nn.Dropout(fusion_dropout),
                                    nn.Linear(E, D))

    def forward(self, img, aud):
        return self.fusion(torch.cat([self.image_encoder(img), self.audio_encoder(aud)], 1))


def head(i, o, p=0.0):
    m = nn.Module()
    m.mlp = nn.Sequential(nn.Linear(i, 512), nn.BatchNorm1d(512), nn.GELU(), nn.Dropout(p),
                          nn.Linear(512, o))
    return m


class DinoMSE(nn.Module):
    """MultiModalDINOWithMSE(CentralMultiModalEncoder); state-dict keys as the reference.
    mode="semi_supervised": MultiModalDINOSemiSupervised (dino.py:964-980) -- the two heads are
    ``image_classifier`` / ``audio_classifier`` = ProjectionHead(E, num_classes) and forward
    returns their logits in place of the MSE features."""

    def __init__(self, E=256, D=256, P=128, dropout=0.3, fusion_dropout=0.3, mode="mse",
                 num_classes=10):
        super().__init__()
        self.student = CentralMM(E, D, fusion_dropout)
        self.teacher = CentralMM(E, D, fusion_dropout)
        self.teacher.load_state_dict(self.student.state_dict())
        for p in self.teacher.parameters():
            p.requires_grad = False
        self.student_projection = head(D, P, dropout)
        self.teacher_projection = head(D, P)
        self.teacher_projection.load_state_dict(self.student_projection.state_dict())
        for p in self.teacher_projection.parameters():
            p.requires_grad = False
        self.register_buffer("center", torch.zeros(1, P))
        self.mode = mode
        if mode == "semi_supervised":
            self.image_classifier = head(E, num_classes)
            self.audio_classifier = head(E, num_classes)
        else:
            self.image_projection_head = head(E, P)
            self.audio_projection_head = head(E, P)

    @torch.no_grad()
    def update_teacher(self, m=0.996):
        for s, t in zip(self.student.parameters(), self.teacher.parameters()):
            t.data = m * t.data + (1 - m) * s.data
        for s, t in zip(self.student_projection.parameters(), self.teacher_projection.parameters()):
            t.data = m * t.data + (1 - m) * s.data

    def forward(self, image, audio, g_img, g_aud, l_img, l_aud, cm=0.9):
        G, L = g_img.shape[1], l_img.shape[1]
        sf = [self.student(g_img[:, v], g_aud[:, v]) for v in range(G)]
        sf += [self.student(l_img[:, v], l_aud[:, v]) for v in range(L)]
        sf = torch.cat(sf)
        with torch.no_grad():
            tf = torch.cat([self.teacher(g_img[:, v], g_aud[:, v]) for v in range(G)])
        sp = self.student_projection.mlp(sf)
        with torch.no_grad():
            tp = self.teacher_projection.mlp(tf)
            tc = tp - self.center
            self.center = self.center * cm + tp.mean(0, keepdim=True) * (1 - cm)
        B = g_img.shape[0]
        hi, ha = ((self.image_classifier, self.audio_classifier) if self.mode == "semi_supervised"
                  else (self.image_projection_head, self.audio_projection_head))
        fi = hi.mlp(self.student.image_encoder(image))
        fa = ha.mlp(self.student.audio_encoder(audio))
        return fi, fa, sp.view(G + L, B, -1), tc.view(G, B, -1)


def dino_loss(s, t, tau_s=0.1, tau_t=0.04):
    s = F.normalize(s, p=2, dim=-1)
    t = F.normalize(t, p=2, dim=-1)
    pt = F.softmax(t / tau_t, dim=-1)
    ls = F.log_softmax(s / tau_s, dim=-1)
    total = 0
    for i in range(s.shape[0]):
        for j in range(t.shape[0]):
            total = total + (-(pt[j] * ls[i]).sum(-1).mean())
    return total / (s.shape[0] * t.shape[0])


def mse_loss(a, b):
    return F.mse_loss(F.normalize(a, p=2, dim=1), F.normalize(b, p=2, dim=1))


def supervised_loss(il, al, labels):
    """CE(image logits) + CE(audio logits), mean over the batch (dino.py:1001-1025)."""
    return F.cross_entropy(il, labels) + F.cross_entropy(al, labels)


def make_optimizer(model, lr=1e-4, wd=1e-6):
    return torch.optim.Adam(model.parameters(), lr=lr, weight_decay=wd)


def train_step(model, opt, batch):
    """fwd -> loss -> update_teacher -> zero_grad -> backward -> Adam (dino.py:1214-1238)."""
    fi, fa, s, t = model(batch["image"], batch["audio"], batch["g_img"], batch["g_aud"],
                         batch["l_img"], batch["l_aud"])
    if model.mode == "semi_supervised":
        loss = dino_loss(s, t) + supervised_loss(fi, fa, batch["label"])
    else:
        loss = dino_loss(s, t) + mse_loss(fi, fa)
    model.update_teacher()
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss.detach()


# ---------------------------------------------------------------------------- config 1
def _cnn3(chans):
    layers = []
    for ci, co in zip(chans[:-1], chans[1:]):
        layers += [nn.Conv2d(ci, co, 3, padding=1), nn.BatchNorm2d(co), nn.ReLU(), nn.MaxPool2d(2)]
    return layers


class ImageEnc(nn.Module):
    """ImageEncoder (dino.py:18-42, 483-499): 3x[conv3x3 -> BN -> ReLU -> pool] 1->32->64->128,
    GAP, Linear(128, 512), projection Linear(512, D)."""

    def __init__(self, D):
        super().__init__()
        self.encoder = nn.Sequential(*_cnn3([1, 32, 64, 128]), nn.AdaptiveAvgPool2d(1), nn.Flatten(),
                                     nn.Linear(128, 512))
        self.projection = nn.Sequential(nn.Linear(512, D))

    def forward(self, x):
        return self.projection(self.encoder(x))


class UniImageDINO(nn.Module):
    """UniModalDINO(ImageEncoder) (dino.py:1257-1398); state-dict keys as the reference."""

    def __init__(self, D=256, P=128, dropout=0.3):
        super().__init__()
        self.student, self.teacher = ImageEnc(D), ImageEnc(D)
        self.teacher.load_state_dict(self.student.state_dict())
        self.student_projection, self.teacher_projection = head(D, P, dropout), head(D, P)
        self.teacher_projection.load_state_dict(self.student_projection.state_dict())
        for p in list(self.teacher.parameters()) + list(self.teacher_projection.parameters()):
            p.requires_grad = False
        self.register_buffer("center", torch.zeros(1, P))

    update_teacher = DinoMSE.update_teacher

    def forward(self, g_img, cm=0.9):
        G = g_img.shape[1]
        sp = self.student_projection.mlp(torch.cat([self.student(g_img[:, v]) for v in range(G)]))
        with torch.no_grad():
            tp = self.teacher_projection.mlp(torch.cat([self.teacher(g_img[:, v]) for v in range(G)]))
            tc = tp - self.center
            self.center = self.center * cm + tp.mean(0, keepdim=True) * (1 - cm)
        B = g_img.shape[0]
        return sp.view(G, B, -1), tc.view(G, B, -1)


def unimodal_dino_loss(s, t, tau_s=0.1, tau_t=0.04):
    """UniModalDINOLightning.dino_loss (dino.py:1596-1635): after L2-normalising, the teacher
    is also centred by its per-view batch mean."""
    s = F.normalize(s, p=2, dim=-1)
    t = F.normalize(t, p=2, dim=-1)
    pt = F.softmax((t - t.mean(dim=1, keepdim=True)) / tau_t, dim=-1)
    ls = F.log_softmax(s / tau_s, dim=-1)
    total = 0
    for i in range(s.shape[0]):
        for j in range(t.shape[0]):
            total = total + (-(pt[j] * ls[i]).sum(-1).mean())
    return total / (s.shape[0] * t.shape[0])


def pretrain_step(model, opt, g_img):
    """training_structures.pretrain_dino's inner loop (dino_train.py:143-161): zero_grad ->
    forward -> dino_loss -> backward -> AdamW.step -> update_teacher."""
    opt.zero_grad()
    s, t = model(g_img)
    loss = unimodal_dino_loss(s, t)
    loss.backward()
    opt.step()
    model.update_teacher()
    return loss.detach()
