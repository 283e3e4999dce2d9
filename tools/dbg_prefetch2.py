"""Debug: WHEN does a prefetched (data-stream) staging set go wrong under graph replay?

Serial run: every step's staged set is snapshotted after the step.  Prefetch run (repeated):
after step t the device is synchronised and the set the NEXT step will read -- written by the
data stream under step t -- is snapshotted ("pre"), and after step t + 1 the same set again
("post").  Each is compared with the serial snapshot of that batch; for a differing view the
wrong elements are matched against the set's previous content (the batch two steps back) and
against the other views of the same batch."""
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

NV = 2 + 4 + 1


def snap(eng, par):
    sfx = "" if par == 0 else ".1"
    return (eng.ws.bufs["in.img" + sfx].float().clone(), eng.ws.bufs["in.aud" + sfx].float().clone())


def run(pre, root, steps=8):
    ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                           multimodal_mode="semi_supervised", device="cuda", staged=True)
    batches = list(ld)[:4] * 2
    store = ParamStore(multimodal_dino_sd("semi_supervised", 32, 32, 16), "cuda:0", seed=1)
    eng = EN.MultiCentralEngine(store, "semi_supervised", 32, 32, 16,
                                EN.Hyper(dropout=0.0, fusion_dropout=0.0), act_dtype=torch.bfloat16)
    eng.use_graph = True
    eng.graph.warmup = 1
    used, nxt, losses, kinds = {}, {}, [], []
    for i, b in enumerate(batches[:steps]):
        caps = eng.graph.captures
        n = batches[i + 1] if (pre and i + 1 < steps) else None
        losses.append(eng.step(b, next_batch=n).item())
        torch.cuda.synchronize()
        kinds.append("capture" if eng.graph.captures > caps else ("replay" if eng.graph.graphs.get(
            next(iter(eng.graph.graphs), None)) is not None and i >= 4 else "eager"))
        used[i] = snap(eng, eng._par)
        if n is not None:
            nxt[i + 1] = snap(eng, 1 - eng._par)
    return losses, used, nxt, kinds


def views(t):
    return t.view(NV, -1)


def main():
    root = _fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    l0, ser, _, kinds = run(False, root)
    print("serial losses", l0, kinds, flush=True)
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
        l1, post, pre, _ = run(True, root)
        bad = []
        for t in range(1, len(l1)):
            for m, j in (("img", 0), ("aud", 1)):
                for what, src in (("pre", pre.get(t)), ("post", post[t])):
                    if src is None:
                        continue
                    a, b = views(src[j]), views(ser[t][j])
                    for v in range(NV):
                        if not torch.equal(a[v], b[v]):
                            d = (a[v] != b[v]).nonzero().flatten()
                            info = f"step {t} {m} view {v} {what}: {d.numel()} elems [{d[0].item()}..{d[-1].item()}]"
                            if t >= 2:
                                old = views(ser[t - 2][j])[v]
                                info += f"; == batch t-2 there: {torch.equal(a[v][d], old[d])}"
                            info += f"; other views equal there: " + ",".join(
                                str(u) for u in range(NV) if u != v and torch.equal(a[v][d], b[u][d]))
                            info += f"; zeros: {bool((a[v][d] == 0).all())}"
                            bad.append(info)
        print(f"rep {rep}: losses {'equal' if l1 == l0 else 'DIFF'}", flush=True)
        for x in bad:
            print("   ", x, flush=True)


if __name__ == "__main__":
    main()
