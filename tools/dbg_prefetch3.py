"""Debug: bisect the prefetch race.  Runs the bitwise prefetched-vs-serial comparison of
tests/test_gpu_augment.py (graph-replayed, no synchronisation between steps) REPS times per
variant and counts loss / parameter mismatches:
  graph        the engine as shipped (side + weight-gradient streams inside the captured step)
  graph_noside concurrent=False: one stream, a single-branch graph
  eager        no graphs
  graph_sync   torch.cuda.synchronize() after every step
    python tools/dbg_prefetch3.py REPS variant ..."""
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


def run(pre, root, variant):
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", 32, 32, 16,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16,
                                concurrent=variant != "graph_noside")
    eng.use_graph = variant != "eager"
    eng.graph.warmup = 1
    losses = []
    for i, b in enumerate(batches):
        n = batches[i + 1] if (pre and i + 1 < len(batches)) else None
        losses.append(eng.step(b, next_batch=n).item())
        if variant == "graph_sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return losses, store.student.clone()


def main():
    reps = int(sys.argv[1])
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    for variant in sys.argv[2:]:
        l0, s0 = run(False, root, variant)
        bad = []
        for r in range(reps):
            l1, s1 = run(True, root, variant)
            if l1 != l0 or not torch.equal(s0, s1):
                bad.append([k for k in range(len(l0)) if l0[k] != l1[k]])
        print(f"{variant}: {len(bad)} of {reps} runs differ; first differing steps {bad[:6]}", flush=True)


if __name__ == "__main__":
    main()
