"""Debug: which ingredient does the prefetch mismatch need?  REPS runs per variant, graph-replayed,
no synchronisation between steps (the test's setting), compared with the serial run:
  A  the round-5 prefetch: the data stream overlaps the current step (two staging sets)
  F  as shipped: the data stream waits for the whole queued step (no overlap)
  G  overlap, but the data stream writes a private scratch set that the main stream copies into
     the staging set after the step (no graph-referenced memory written concurrently)
  I  overlap, one stream per step (concurrent=False: no side streams inside the graphs)
  X_eager   variant X without graph capture (every step launched eagerly)
  X_keepev  variant X with every torch.cuda.Event kept alive for the whole run (no event is
            destroyed while a stream may still wait on it)
  C  variant A, and after each prefetch the device is synchronised and the prefetched views are
     compared with the same augmentation redone on the main stream (are the INPUTS wrong, or
     the step computed from right inputs?)
    python tools/dbg_prefetch5.py REPS A F G I C"""
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

_orig_pf = EN.MultiCentralEngine.prefetch
_orig_bufs = EN.MultiCentralEngine._aug_bufs
_orig_stage = EN.MultiCentralEngine.stage


def pf_wait_all(self, batch):          # F: as shipped since round 6
    return _orig_pf(self, batch)


def stage_mark(self, batch, with_orig, training=True):
    out = _orig_stage(self, batch, with_orig, training)
    if training:        # everything queued before this step: the last readers of the other set
        self._ev_free = torch.cuda.Event()
        self._ev_free.record(torch.cuda.current_stream())
    return out


def pf_overlap(self, batch):
    """The round-5 prefetch: the data stream waits only for the event stage() recorded in front
    of the step just queued, so the augmentation overlaps that step."""
    ds = self.dstream
    if ds is None:
        return _orig_pf(self, batch)
    ev = getattr(self, "_ev_free", None)
    orig_wait = ds.wait_stream
    ds.wait_stream = (lambda s: ds.wait_event(ev)) if ev is not None else orig_wait
    try:
        return _orig_pf(self, batch)
    finally:
        del ds.wait_stream


def bufs_scratch(self, batch, with_orig, par):
    # prefetch() asks for set `par`: hand it a scratch set; stage() copies it over on main
    if getattr(self, "_in_pf", False):
        x_img, x_aud, B, G, L = _orig_bufs(self, batch, with_orig, par)
        si = self.ws.get("scr.img", x_img.numel(), x_img.dtype)
        sa = self.ws.get("scr.aud", x_aud.numel(), x_aud.dtype)
        self._scr = (si, sa, x_img, x_aud)
        return si, sa, B, G, L
    return _orig_bufs(self, batch, with_orig, par)


def pf_scratch(self, batch):
    self._in_pf = True
    try:
        return pf_overlap(self, batch)
    finally:
        self._in_pf = False


def stage_scratch(self, batch, with_orig, training=True):
    pf = self._pf
    out = stage_mark(self, batch, with_orig, training)
    if pf is not None and pf[0] is batch:
        si, sa, x_img, x_aud = self._scr
        x_img.copy_(si)
        x_aud.copy_(sa)
        out = (x_img, x_aud) + tuple(out[2:])
    return out


CHK = []


def pf_check(self, batch):
    aug = batch["aug"]
    c0 = (aug.image.calls, aug.audio.calls)
    ok = pf_overlap(self, batch)
    torch.cuda.synchronize()
    c1 = (aug.image.calls, aug.audio.calls)
    x_img, x_aud = self._pf[3][0], self._pf[3][1]
    si, sa = torch.empty_like(x_img), torch.empty_like(x_aud)
    aug.image.calls, aug.audio.calls = c0
    aug.stage(batch["idx"], si, sa, self.heads is not None)
    torch.cuda.synchronize()
    aug.image.calls, aug.audio.calls = c1
    CHK.append(torch.equal(si, x_img) and torch.equal(sa, x_aud))
    return ok


_KEEP = []
_OrigEvent = torch.cuda.Event


class _KeptEvent(_OrigEvent):
    def __new__(cls, *a, **k):
        e = _OrigEvent.__new__(cls, *a, **k)
        _KEEP.append(e)
        return e


def run(pre, root, variant):
    keep = variant.endswith("keepev")
    torch.cuda.Event = torch.cuda.streams.Event = _KeptEvent if keep else _OrigEvent
    import gc
    gc.collect()
    torch.cuda.synchronize()
    EN.MultiCentralEngine.prefetch = {"F": pf_wait_all, "G": pf_scratch, "C": pf_check}.get(variant[:1], pf_overlap)
    EN.MultiCentralEngine._aug_bufs = bufs_scratch if variant[:1] == "G" else _orig_bufs
    EN.MultiCentralEngine.stage = {"G": stage_scratch, "F": _orig_stage}.get(variant[:1], stage_mark)
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", 32, 32, 16,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16,
                                concurrent=variant[:1] != "I")
    eng.use_graph = not variant.endswith("eager")
    eng.graph.warmup = 1
    losses = []
    for i, b in enumerate(batches):
        n = batches[i + 1] if (pre and i + 1 < len(batches)) else None
        losses.append(eng.step(b, next_batch=n).item())
    torch.cuda.synchronize()
    out = losses, store.student.clone()
    torch.cuda.Event = torch.cuda.streams.Event = _OrigEvent
    return out


def main():
    reps = int(sys.argv[1])
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    for variant in sys.argv[2:]:
        l0, s0 = run(False, root, variant)
        bad = []
        for r in range(reps):
            CHK.clear()
            l1, s1 = run(True, root, variant)
            if CHK:
                print(f"   {variant} rep {r}: prefetched inputs equal to redone: {CHK}", flush=True)
            if l1 != l0 or not torch.equal(s0, s1):
                ks = [k for k in range(len(l0)) if l0[k] != l1[k]]
                bad.append(ks)
                if ks:
                    k = ks[0]
                    print(f"   {variant} rep {r}: step {k} loss {l1[k]!r} vs serial {l0[k]!r} "
                          f"(d {l1[k] - l0[k]:.3e}); finite params {bool(torch.isfinite(s1).all())}", flush=True)
        print(f"{variant}: {len(bad)} of {reps} runs differ; first differing steps {bad[:5]}", flush=True)


if __name__ == "__main__":
    main()
