"""Uninitialised-LDS detector: a training step run with avd_lds_poison (every CU's LDS filled with
NaN bit patterns) launched right before EVERY libavdino call must give bit-identical results to
the same step without it -- a kernel that reads LDS it never wrote would pick up NaN.  When the
results differ, each call is then poisoned alone to name the kernels that do.
    python tools/lds_poison.py [small|config2] ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from avdino import engine as EN  # noqa: E402
from avdino import ops  # noqa: E402
from avdino.params import ParamStore  # noqa: E402
from avdino.spec import multimodal_dino_sd  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402

CASES = {"small": ("semi_supervised", 32, 32, 16, 8, 2, 4), "config2": ("mse", 256, 256, 128, 64, 2, 4),
         "infonce": ("infonce", 256, 256, 128, 64, 2, 4)}
_orig_call = ops.call


def step(case, poison):
    mode, E, D, P, B, G, L = CASES[case]
    state = {k: torch.from_numpy(np.array(v)) for k, v in
             make_state(OS.multimodal_dino_spec(mode, E, D, P), 41).items()}
    batch = {k: torch.from_numpy(v).cuda() for k, v in make_multimodal_batch(B, G, L, 42).items()}
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda")
    store.load_state_dict(state)
    eng = EN.MultiCentralEngine(store, mode, E, D, P, EN.Hyper(dropout=0.0, fusion_dropout=0.0),
                                act_dtype=torch.bfloat16)
    names = []

    def hooked(name, *args):
        k = len(names)
        names.append(name)
        if poison is not None and name != "avd_lds_poison" and (poison == "all" or k in poison):
            _orig_call("avd_lds_poison", ops.stream())
        return _orig_call(name, *args)

    ops.call = hooked
    try:
        loss = eng.step(batch).item()
        torch.cuda.synchronize()
    finally:
        ops.call = _orig_call
    return loss, store.student.clone(), names


def main():
    for case in sys.argv[1:] or ["small"]:
        l0, s0, names = step(case, None)
        l1, s1, _ = step(case, "all")
        same = l0 == l1 and torch.equal(s0, s1)
        print(f"{case}: {len(names)} calls; poisoned before every call: "
              f"{'identical' if same else f'DIFFERENT (loss {l1!r} vs {l0!r})'}", flush=True)
        if same:
            continue
        bad = []
        for k in range(len(names)):
            lk, sk, _ = step(case, {k})
            if lk != l0 or not torch.equal(sk, s0):
                bad.append((k, names[k], lk))
        for k, n, lk in bad:
            print(f"   call {k} {n}: loss {lk!r}", flush=True)


if __name__ == "__main__":
    main()
