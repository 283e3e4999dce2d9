"""Debug: is the multi-stream training step's graph replay timing-dependent?  Serial steps (no
prefetch, one staging set, one graph), REPS runs each, with a NOISE stream running unrelated
matmuls during every replay, compared with a run without noise.  Variants inline chosen
side-stream pieces onto the main stream:
  N       noise, the step as shipped
  T / H / I   noise, with the teacher forward / the originals' heads forward / the image-branch
              backward run inline instead of on the side stream
  IL      noise, the heads backward not interleaved (queued after the main chain, on the side)
  ALL     noise, every _on_side piece inline and no interleave (main stream only)
    python tools/dbg_race.py REPS N T H I IL ALL"""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
import torch  # noqa: E402

from tests.test_gpu_augment import _fake_avmnist  # noqa: E402
from avdino import engine as EN  # noqa: E402
from avdino.data import AVMNISTDinoLoader  # noqa: E402
from avdino.params import ParamStore  # noqa: E402
from avdino.spec import multimodal_dino_sd  # noqa: E402

_orig_on_side = EN.MultiCentralEngine._on_side


def piece(fn):
    n = getattr(fn, "__name__", "")
    names = fn.__code__.co_names if hasattr(fn, "__code__") else ()
    if "_teacher_fwd" in names:
        return "T"
    if n == "heads":
        return "H"
    if n in ("image_convs", "image_branch"):
        return "I"
    if "drain" in names:
        return "IL"
    return "?"


def make_on_side(inline):
    def on_side(self, fn, after=None):
        if piece(fn) in inline:
            return fn(), None
        return _orig_on_side(self, fn, after)
    return on_side


def run(root, variant, noise):
    import gc
    gc.collect()                 # retire the previous run's graphs before any new capture
    torch.cuda.synchronize()
    inline = {"T": {"T"}, "H": {"H"}, "I": {"I"}, "ALL": {"T", "H", "I", "IL"}}.get(variant, set())
    EN.MultiCentralEngine._on_side = make_on_side(inline)
    EN.MultiCentralEngine.INTERLEAVE = variant not in ("IL", "ALL")
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", 32, 32, 16,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16)
    eng.use_graph = True
    eng.graph.warmup = 1
    ns = torch.cuda.Stream()
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    losses = []
    for i, b in enumerate(batches):
        if noise:
            ns.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(ns):
                for _ in range(1 + (i * 7 + noise) % 5):
                    a = (a @ a) * 0.01
        losses.append(eng.step(b).item())
    torch.cuda.synchronize()
    out = losses, store.student.clone()
    del eng
    return out


def main():
    reps = int(sys.argv[1])
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    for variant in sys.argv[2:]:
        l0, s0 = run(root, variant, 0)
        bad = []
        for r in range(reps):
            l1, s1 = run(root, variant, r + 1)
            if l1 != l0 or not torch.equal(s0, s1):
                bad.append([k for k in range(len(l0)) if l0[k] != l1[k]])
        print(f"{variant}: {len(bad)} of {reps} runs differ; first differing steps {bad[:5]}", flush=True)
    EN.MultiCentralEngine._on_side = _orig_on_side
    EN.MultiCentralEngine.INTERLEAVE = True


if __name__ == "__main__":
    main()
