"""Debug helper: does any kernel of a training step write outside its buffers into the second
staging set (which a prefetch fills concurrently)?  Serial eager steps of the
test_prefetched_augmentation_steps_equal_serial_steps setup; the second staging set is allocated
where a prefetch would allocate it (after step 0), filled with a sentinel, and checked after every
libavdino call.
    python tools/dbg_oob.py
"""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "multimodal-ssl-avmnist_amd"))
import torch  # noqa: E402

from tests.test_gpu_augment import _fake_avmnist  # noqa: E402
from avdino import engine as EN  # noqa: E402
from avdino import ops  # noqa: E402
from avdino.data import AVMNISTDinoLoader  # noqa: E402
from avdino.params import ParamStore  # noqa: E402
from avdino.spec import multimodal_dino_sd  # noqa: E402


def main():
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    E, D, P = 32, 32, 16
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", E, D, P), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", E, D, P,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16)
    eng.use_graph = False
    eng.step(batches[0]).item()
    torch.cuda.synchronize()
    sets = eng._aug_bufs(batches[1], True, 1)[:2]      # where prefetch() would allocate them
    guard = [torch.empty(4096, device="cuda") for _ in range(8)]   # a few neighbours more
    bufs = list(sets) + guard
    for b in bufs:
        b.view(torch.int16).fill_(0x5A5A) if b.dtype == torch.bfloat16 else b.fill_(12345.0)
    ref = [b.clone() for b in bufs]
    orig = ops.call
    count = [0]

    def hooked(name, *args):
        rc = orig(name, *args)
        torch.cuda.synchronize()
        count[0] += 1
        for i, (b, r) in enumerate(zip(bufs, ref)):
            if not torch.equal(b, r):
                n = (b != r).sum().item()
                print(f"call {count[0]} {name}: buffer {i} changed ({n} elements)", flush=True)
                b.copy_(r)
        return rc

    ops.call = hooked
    for i, b in enumerate(batches[1:], 1):
        eng.step(b).item()
    print("checked", count[0], "calls", flush=True)


if __name__ == "__main__":
    main()
