"""Debug: which input of the prefetched augmentation goes wrong?  Variant A of dbg_prefetch5
(data stream overlapping the replayed step), with every ViewAugmenter call made during a
prefetch recorded (sample ids, device records, bitmasks, output view); after the prefetch the
device is synchronised and, per call: the ids on the device are compared with the host ids, the
records / bitmasks are drawn again on the main stream with the same counter, and the views are
rebuilt on the main stream from the recorded (device) records.  Prints the first bad piece.
    python tools/dbg_prefetch6.py REPS"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dbg_prefetch5 as D5  # noqa: E402
from avdino import augment as AU  # noqa: E402
from avdino import engine as EN  # noqa: E402

REC = []
ON = [False]
_orig_call = AU.ViewAugmenter.__call__
_orig_apply = AU.ViewAugmenter.apply


def call(self, idx, chain, n_views, out=None, order=0):
    if ON[0]:
        self._dbg = (self.calls, chain)
    return _orig_call(self, idx, chain, n_views, out, order)


def apply(self, idx, rec, gm, n_views, out=None, order=0, kinds=None):
    prev = out.clone() if (ON[0] and out is not None) else None    # data stream, before the kernel
    o = _orig_apply(self, idx, rec, gm, n_views, out, order, kinds)
    if ON[0]:
        info = getattr(self, "_dbg", None)
        self._dbg = None
        REC.append(dict(aug=self, idx=np.asarray(idx, np.int64).copy(), rec=rec, gm=gm, n_views=n_views,
                        out=o, order=order, kinds=kinds, calls_after=self.calls, info=info,
                        snap=o.clone(), prev=prev))     # on the data stream, right after the kernel
    return o


CUR = [None]


from avdino import ops as OPS  # noqa: E402
_orig_views = OPS.augment_views
LDS = []
NOLDS = [False]


def views_chk(src_u8, idx, lut, rec, gm, group, seed, V, H, W, out, order=0, kinds=None):
    if not ON[0] or kinds is not None or out.dtype != torch.bfloat16:
        return _orig_views(src_u8, idx, lut, rec, gm, group, seed, V, H, W, out, order, kinds)
    if NOLDS[0]:
        OPS.call("avd_augment_views_nolds", OPS.p(src_u8), OPS.p(idx), idx.numel(), V, H, W, OPS.p(lut),
                 OPS.p(rec), OPS.p(gm), gm.shape[1] if gm is not None else 0, group, seed & (2**64 - 1),
                 order, OPS.p(out), OPS.stream())
        return
    chk = torch.zeros(3, dtype=torch.int32, device=out.device)
    seen = torch.full_like(rec, -7.0)
    OPS.call("avd_augment_views_lds_check", OPS.p(src_u8), OPS.p(idx), idx.numel(), V, H, W, OPS.p(lut),
             OPS.p(rec), OPS.p(gm), gm.shape[1] if gm is not None else 0, group, seed & (2**64 - 1),
             order, OPS.p(out), OPS.p(chk), OPS.p(seen), OPS.stream())
    LDS.append((H, V, chk, seen, rec))


def pf_diag(self, batch):
    LDS.clear()
    CUR[0] = self
    REC.clear()
    ON[0] = True
    try:
        ok = D5.pf_overlap(self, batch)
    finally:
        ON[0] = False
    torch.cuda.synchronize()
    bad = []
    for k, r in enumerate(REC):
        aug = r["aug"]
        tag = f"call {k} ({'img' if aug.H == 28 else 'aud'} V={r['n_views']} {'ident' if r['info'] is None else 'chain'})"
        rec, gm = r["rec"], r["gm"]
        saved = aug.calls
        if r["info"] is not None and isinstance(rec, torch.Tensor):
            c0, chain = r["info"]
            aug.calls = c0
            rec2, gm2 = aug.records_dev(chain, r["idx"].shape[0], r["n_views"])
            torch.cuda.synchronize()
            if not torch.equal(rec2, rec):
                bad.append(f"{tag}: records differ ({int((rec2 != rec).any(1).sum())} rows)")
            if gm is not None and not torch.equal(gm2, gm):
                bad.append(f"{tag}: bitmasks differ")
        # rebuild the views from the recorded records on the main stream, same seed counter
        aug.calls = r["calls_after"] - 1
        out2 = torch.empty_like(r["out"])
        _orig_apply(aug, r["idx"], rec, gm, r["n_views"], out2, r["order"], r["kinds"])
        torch.cuda.synchronize()
        aug.calls = saved
        if not torch.equal(out2, r["out"]):
            d = (out2.float() - r["out"].float()).abs().reshape(r["n_views"] if r["order"] else -1, -1)
            bad.append(f"{tag}: views differ given the same records (rows {d.amax(1).nonzero().flatten().tolist()[:8]}, max {d.max().item():.3g})")
            fo, fs, fr = r["out"].reshape(-1).float(), r["snap"].reshape(-1).float(), out2.reshape(-1).float()
            pos = (fo != fr).nonzero().flatten()
            bad.append(f"   snapshot after kernel == rebuilt: {torch.equal(fs, fr)}; final == snapshot: "
                       f"{torch.equal(fo, fs)}; {pos.numel()} of {fo.numel()} elements differ, "
                       f"index range [{int(pos[0])}, {int(pos[-1])}] (view = {fo.numel() // r['n_views']} elems); "
                       f"final {fo[pos[:6]].tolist()} rebuilt {fr[pos[:6]].tolist()}")
            HW = aug.H * aug.W
            B = r["idx"].shape[0]
            where = [(int(i) // (B * HW), (int(i) % (B * HW)) // HW, (int(i) % HW) // aug.W, int(i) % aug.W)
                     for i in pos[:40]]
            bad.append(f"   (view, sample, y, x) of the differing elements: {where}")
            if r["prev"] is not None:
                fp = r["prev"].reshape(-1).float()
                bad.append(f"   final == content before the kernel at those elements: "
                           f"{int((fo[pos] == fp[pos]).sum())} of {pos.numel()}")
            # do the bad values appear anywhere in the other views / other set?
            eng = CUR[0]
            for nm, buf in eng.ws.bufs.items():
                if nm.startswith("in.img") and buf.numel() >= fo.numel():
                    bad.append(f"   {nm} data_ptr {buf.data_ptr():#x} out {r['out'].data_ptr():#x}")
    lds = [(h, v, c.tolist()) for h, v, c, _, _ in LDS if int(c[0])]
    for h, v, _, seen, rec in LDS:
        keep = torch.ones(rec.shape[1], dtype=torch.bool, device=rec.device)
        # fields the kernel truncates to int: compare as the kernel saw them
        ints = [0, 1, 2, 3, 17, 18, 19, 20, 22, 23, 24, 25, 26, 27]
        ref = rec.clone()
        ref[:, ints] = ref[:, ints].trunc()
        dif = (seen != ref) & keep
        if dif.any():
            rows = dif.any(1).nonzero().flatten().tolist()
            r0 = rows[0]
            cols = dif[r0].nonzero().flatten().tolist()
            bad.append(f"RECORD SEEN BY THE KERNEL != RECORD IN MEMORY (H={h}): rows {rows[:8]}, "
                       f"row {r0} fields {cols}: seen {seen[r0, cols].tolist()} memory {rec[r0, cols].tolist()}")
    if lds:
        bad.append(f"LDS words changed during the kernel (H, V, [count, first word, block]): {lds}")
    if bad:
        print("      " + "\n      ".join(bad), flush=True)
    D5.CHK.append(not bad)
    return ok


def main():
    AU.ViewAugmenter.__call__ = call
    AU.ViewAugmenter.apply = apply
    OPS.augment_views = views_chk
    AU.ops.augment_views = views_chk
    D5.pf_check = pf_diag
    import tempfile
    reps = int(sys.argv[1])
    NOLDS[0] = len(sys.argv) > 2 and sys.argv[2] == "nolds"
    print("gather kernel:", "no LDS (source bytes from global memory)" if NOLDS[0] else "LDS-staged", flush=True)
    root = D5._fake_avmnist(__import__("pathlib").Path(tempfile.mkdtemp()), n=40)
    l0, s0 = D5.run(False, root, "A")
    nbad = 0
    for r in range(reps):
        D5.CHK.clear()
        EN.MultiCentralEngine.prefetch = pf_diag
        l1, s1 = run_c(root)
        diff = l1 != l0 or not torch.equal(s0, s1)
        nbad += diff
        print(f"   rep {r}: inputs ok {D5.CHK} run differs {diff}", flush=True)
    print(f"D: {nbad} of {reps} runs differ", flush=True)


def run_c(root):
    # dbg_prefetch5.run with the prefetch replaced by pf_diag ("C" picks D5.pf_check)
    return D5.run(True, root, "C")


if __name__ == "__main__":
    main()
