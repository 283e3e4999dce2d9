"""Debug: isolate the prefetch mismatch (tools/dbg_prefetch3.py showed it with graphs even with a
device synchronisation after every step, never eagerly or on one stream).  Variants, all
graph-replayed with a synchronisation after every step, REPS runs each, compared with the serial
run (one staging set, no data stream):
  A       prefetch as shipped (data stream overlaps the step, two staging sets -> two graphs)
  B       as A, every graph key captured into its OWN memory pool
  E       no data stream; the staging set alternates 0/1 per step (two graphs, serial staging)
  F       prefetch, the data stream waits for the whole queued step (no overlap; two graphs)
    python tools/dbg_prefetch4.py REPS A B E F"""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
import torch  # noqa: E402

from tests.test_gpu_augment import _fake_avmnist  # noqa: E402
from avdino import capture as CAP  # noqa: E402
from avdino import engine as EN  # noqa: E402
from avdino.data import AVMNISTDinoLoader  # noqa: E402
from avdino.params import ParamStore  # noqa: E402
from avdino.spec import multimodal_dino_sd  # noqa: E402

_orig_run = CAP.GraphedStep.run
_orig_pf = EN.MultiCentralEngine.prefetch


def run_own_pool(self, key, body):
    if key not in self.graphs and self.seen.get(key, 0) >= self.warmup:
        self.pool = None                     # -> a fresh pool for this capture
    return _orig_run(self, key, body)


def pf_wait_all(self, batch):
    self._ev_free = None
    return _orig_pf(self, batch)


def run(pre, root, variant):
    CAP.GraphedStep.run = run_own_pool if variant == "B" else _orig_run
    EN.MultiCentralEngine.prefetch = pf_wait_all if variant == "F" else _orig_pf
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", 32, 32, 16,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16)
    eng.use_graph = True
    eng.graph.warmup = 1
    losses = []
    for i, b in enumerate(batches):
        use_pf = pre and variant != "E"
        n = batches[i + 1] if (use_pf and i + 1 < len(batches)) else None
        if pre and variant == "E":
            eng._par = i % 2
        losses.append(eng.step(b, next_batch=n).item())
        torch.cuda.synchronize()
    return losses, store.student.clone()


def main():
    reps = int(sys.argv[1])
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    l0, s0 = run(False, root, "A")
    for variant in sys.argv[2:]:
        bad = []
        for r in range(reps):
            l1, s1 = run(True, root, variant)
            if l1 != l0 or not torch.equal(s0, s1):
                bad.append([k for k in range(len(l0)) if l0[k] != l1[k]])
        print(f"{variant}: {len(bad)} of {reps} runs differ; first differing steps {bad[:5]}", flush=True)


if __name__ == "__main__":
    main()
