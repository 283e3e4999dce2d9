"""Debug: canary guards after every workspace buffer (Workspace.GUARD bytes of 0xA5); after each
step the device is synchronised and every guard checked -- a clobbered guard names the buffer
whose writer ran past its end.  Runs the prefetch test's setting (serial and prefetched,
graph-replayed) and a synthetic multi_central step per mode at a larger batch.
    python tools/dbg_guard.py [GUARD_BYTES] [B]"""
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


def wss(eng):
    out = {}
    for nm in ("ws", "tws", "iws"):
        w = getattr(eng, nm, None)
        if w is not None and id(w) not in {id(v) for v in out.values()}:
            out[nm] = w
    return out


def check(eng, tag):
    torch.cuda.synchronize()
    bad = []
    for nm, w in wss(eng).items():
        bad += [(nm,) + b for b in w.check_guards()]
    if bad:
        print(f"   {tag}: CLOBBERED {bad}", flush=True)
    return bad


def real_data(root, pre, mode):
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode=mode, device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd(mode, 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, mode, 32, 32, 16, EN.Hyper(dropout=0.0, fusion_dropout=0.0),
                                act_dtype=torch.bfloat16)
    eng.use_graph = True
    eng.graph.warmup = 1
    nbad = 0
    for i, b in enumerate(batches):
        n = batches[i + 1] if (pre and i + 1 < len(batches)) else None
        eng.step(b, next_batch=n)
        nbad += len(check(eng, f"{mode} pre={pre} step {i}"))
    return nbad


def synthetic(mode, B, fp8=False, steps=4):
    sys.path.insert(0, REPO)
    from bench import synthetic_pool
    E, D, P, G, L = 256, 256, 128, 2, 4
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda:0", seed=0)
    eng = EN.MultiCentralEngine(store, mode, E, D, P, EN.Hyper(), act_dtype=torch.bfloat16,
                                negatives="global", conv_fp8=fp8)
    eng.use_graph = True
    pool = synthetic_pool(2, B, G, L, "cuda:0", 1234)
    nbad = 0
    for i in range(steps):
        eng.step(pool[i % 2])
        nbad += len(check(eng, f"{mode} B={B} fp8={fp8} step {i}"))
    print(f"   {mode} B={B} fp8={fp8}: {nbad} clobbered", flush=True)
    return nbad


def main():
    EN.Workspace.GUARD = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    tot = 0
    for mode in ("semi_supervised", "mse"):
        for pre in (False, True):
            tot += real_data(root, pre, mode)
    print(f"guard check (real data): {tot} clobbered guards", flush=True)
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    for mode in ("mse", "infonce", "semi_supervised"):
        tot += synthetic(mode, B)
    tot += synthetic("semi_supervised", B, fp8=True)
    print(f"guard check: {tot} clobbered guards", flush=True)


if __name__ == "__main__":
    main()
