"""Device data path on the GPU: avd_augment_views against the numpy
restatement (oracle/augment.py) -- bit-exact for records without noise, |diff| <= 1e-5 with
noise (device logf/cosf vs numpy) -- and the HBM-resident AVMNIST loader feeding a training
step through the C ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from avdino import augment as A  # noqa: E402
from avdino import ops  # noqa: E402
from oracle import augment as OA  # noqa: E402

from .test_augment_data import _fake_avmnist  # noqa: E402


def _records(chain, B, V, H, W, seed):
    aug = A.ViewAugmenter.__new__(A.ViewAugmenter)
    aug.rng, aug.H, aug.W = np.random.default_rng(seed), H, W
    return A.ViewAugmenter.records(aug, chain, B, V)


@pytest.mark.parametrize("view,mod", [("global", "image"), ("local", "image"),
                                      ("global", "audio"), ("local", "audio")])
@pytest.mark.parametrize("order", [0, 1])
def test_augment_kernel_matches_oracle(view, mod, order):
    H = W = 28 if mod == "image" else 112
    N, B, V = 11, 5, 3
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, (N, H * W), dtype=np.uint8)
    idx = rng.integers(0, N, B)
    lut = OA.normalise_lut(mod)
    rec, gm = _records(A.default_chains()[view][mod], B, V, H, W, 9)
    seed = 0xDEADBEEF12345
    out = torch.empty((B, V, H, W) if order == 0 else (V, B, H, W), device="cuda")
    ops.augment_views(torch.from_numpy(src).cuda(), torch.from_numpy(idx).cuda(),
                      torch.from_numpy(lut).cuda(), torch.from_numpy(rec).cuda(),
                      None if gm is None else torch.from_numpy(gm.view(np.int32)).cuda(),
                      4, seed, V, H, W, out, order)
    got = out.cpu().numpy()
    ref = OA.augment_views(src, idx, lut, rec, gm, V, H, W, seed, order)
    noisy = (rec[:, 21] != 0).reshape(B, V)
    if order == 1:
        noisy = noisy.T
    np.testing.assert_array_equal(got[~noisy], ref[~noisy])
    np.testing.assert_allclose(got[noisy], ref[noisy], rtol=0, atol=1e-5)
    assert np.isfinite(got).all()


def test_augment_identity_is_the_normalised_row():
    rng = np.random.default_rng(5)
    src = torch.from_numpy(rng.integers(0, 256, (7, 12544), dtype=np.uint8)).cuda()
    lut = torch.from_numpy(OA.normalise_lut("audio")).cuda()
    aug = A.ViewAugmenter(src, lut, 112, 112, seed=1)
    out = aug.identity([6, 0, 3])
    ref = lut.cpu().numpy()[src.cpu().numpy()[[6, 0, 3]]].reshape(3, 1, 112, 112)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    with pytest.raises(IndexError):
        aug.identity([7])


def test_loader_batches_feed_a_training_step(tmp_path):
    from avdino.data import AVMNISTDinoLoader
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    root = _fake_avmnist(tmp_path, n=40)
    loader = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                               multimodal_mode="mse")
    assert len(loader.train_idx) == 36 and len(loader) == 5
    batches = list(loader)
    assert len(batches) == 5
    img, aud, lab, (gi, ga, li, la) = batches[0]
    assert img.shape == (8, 1, 28, 28) and aud.shape == (8, 1, 112, 112) and lab.shape == (8,)
    assert gi.shape == (8, 2, 1, 28, 28) and ga.shape == (8, 2, 1, 112, 112)
    assert li.shape == (8, 4, 1, 28, 28) and la.shape == (8, 4, 1, 112, 112)
    assert img.min() >= 0 and img.max() <= 1
    E, D, P = 32, 32, 16
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda:0")
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0))
    batch = dict(image=img, audio=aud, label=lab, g_img=gi, g_aud=ga, l_img=li, l_aud=la)
    loss = eng.step(batch).item()
    assert np.isfinite(loss)


# ---------------------------------------------------------------------- device parameter draws
def _dev_records(chain, n, H, W, seed):
    src = torch.zeros(1, H * W, dtype=torch.uint8, device="cuda")
    aug = A.ViewAugmenter(src, torch.zeros(256, device="cuda"), H, W, seed=seed)
    rec, gm = aug.records_dev(chain, n, 1)
    return rec.cpu().numpy(), None if gm is None else gm.cpu().numpy().view(np.uint32)


def _stats(rec, gm, H, W):
    fl = rec[:, 23].astype(np.int64)
    crop, aff, rot, tw = (fl & 1) > 0, (fl & 2) > 0, (fl & 4) > 0, (fl & 8) > 0
    er = rec[:, 26] > 0
    out = {"p_crop": crop.mean(), "p_aff": aff.mean(), "p_rot": rot.mean(), "p_tw": tw.mean(),
           "p_erase": er.mean(), "p_noise": (rec[:, 21] != 0).mean(), "p_gm": (rec[:, 22] >= 0).mean(),
           "p_fmask": (rec[:, 18] > rec[:, 17]).mean(), "p_tmask": (rec[:, 20] > rec[:, 19]).mean()}
    if crop.any():
        out["crop_area"] = (rec[crop, 2] * rec[crop, 3]).mean() / (H * W)
        out["crop_top"] = rec[crop, 0].mean() / H
    if aff.any():
        out["aff_scale"] = np.hypot(rec[aff, 4], rec[aff, 5]).mean()
        out["aff_tx"] = np.abs(rec[aff, 6]).mean() / W
    if rot.any():
        out["rot_sin"] = np.abs(rec[rot, 11]).mean()
    if tw.any():
        out["rate"] = rec[tw, 16].mean()
    if er.any():
        out["erase_area"] = (rec[er, 26] * rec[er, 27]).mean() / (H * W)
    fm = rec[:, 18] > rec[:, 17]
    if fm.any():
        out["fmask_w"] = (rec[fm, 18] - rec[fm, 17]).mean()
    return out


@pytest.mark.parametrize("view,mod", [("global", "image"), ("local", "image"),
                                      ("global", "audio"), ("local", "audio")])
def test_device_param_draws_match_the_host_distributions(view, mod):
    """avd_augment_records vs the numpy sampler (the get_params rules): 20000 draws each;
    probabilities within 0.015, mean box areas / scales / rates within 3 % (the streams differ,
    the distributions must not)."""
    H = W = 28 if mod == "image" else 112
    chain = A.default_chains()[view][mod]
    n = 20000
    drec, dgm = _dev_records(chain, n, H, W, 77)
    hrec, hgm = _records(chain, n, 1, H, W, 78)
    ds, hs = _stats(drec, dgm, H, W), _stats(hrec, hgm, H, W)
    assert ds.keys() == hs.keys()
    for k in ds:
        if k.startswith("p_"):
            assert abs(ds[k] - hs[k]) < 0.015, (k, ds[k], hs[k])
        else:
            assert abs(ds[k] - hs[k]) <= 0.03 * max(abs(hs[k]), 1e-3) + 0.002, (k, ds[k], hs[k])


def test_device_param_draws_bounds_and_exact_masks():
    chain = A.default_chains()["local"]["audio"]
    H = W = 112
    rec, gm = _dev_records(chain, 4096, H, W, 5)
    crop = (rec[:, 23].astype(np.int64) & 1) > 0
    t, l_, h, w = rec[crop, 0], rec[crop, 1], rec[crop, 2], rec[crop, 3]
    assert (h > 0).all() and (w > 0).all() and (t >= 0).all() and (l_ >= 0).all()
    assert (t + h <= H).all() and (l_ + w <= W).all()
    ng = (H // 4) * (W // 4)
    k = int(0.6 * ng)
    on = rec[:, 22] >= 0
    pop = np.array([bin(int(x)).count("1") for x in gm.reshape(-1)]).reshape(gm.shape).sum(1)
    assert (pop[on] == k).all() and (pop[~on] == 0).all()
    assert (rec[on, 22] == np.nonzero(on)[0]).all()
    # deterministic in the seed
    rec2, gm2 = _dev_records(chain, 4096, H, W, 5)
    assert np.array_equal(rec, rec2) and np.array_equal(gm, gm2)


def test_staged_bf16_views_equal_the_f32_views_rounded():
    """The views written straight into the staged bf16 input equal the f32 views (same
    records, same noise seed) rounded to bf16."""
    rng = np.random.default_rng(6)
    src = torch.from_numpy(rng.integers(0, 256, (9, 12544), dtype=np.uint8)).cuda()
    lut = torch.from_numpy(OA.normalise_lut("audio")).cuda()
    chain = A.default_chains()["local"]["audio"]
    idx = np.array([3, 1, 8, 0])
    a32 = A.ViewAugmenter(src, lut, 112, 112, seed=2)
    a16 = A.ViewAugmenter(src, lut, 112, 112, seed=2)
    v32 = a32(idx, chain, 3, order=1)
    out = torch.empty(3 * 4 * 12544, dtype=torch.bfloat16, device="cuda")
    a16(idx, chain, 3, out=out, order=1)
    assert torch.equal(out.view_as(v32), v32.to(torch.bfloat16))


def test_engine_step_from_staged_augmentation_equals_collated_views(tmp_path):
    """MultiCentralEngine.stage({"aug", "idx"}) builds the views in place; the same seeds
    through the collated f32 views + avd_stage_views give the same staged bits and loss."""
    from avdino.data import AVMNISTDinoLoader
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    root = _fake_avmnist(tmp_path, n=40)
    mk = lambda: AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,  # noqa: E731
                                   multimodal_mode="mse", device="cuda", shuffle=False)
    la, lb = mk(), mk()
    idx = la._order()[:8]
    E, D, P = 32, 32, 16
    res = []
    for batch in (la.staged_batch(idx), None):
        store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda:0", seed=1)
        eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                                 act_dtype=torch.bfloat16)
        if batch is None:
            img, aud, lab, (gi, ga, li, la_) = lb.batch(idx)
            batch = dict(image=img, audio=aud, label=lab, g_img=gi, g_aud=ga, l_img=li, l_aud=la_)
        staged = eng.stage(batch, True)
        loss = eng._forward_staged(staged, training=True).item()
        res.append((staged[0].clone(), staged[1].clone(), loss))
    (xi0, xa0, l0), (xi1, xa1, l1) = res
    assert torch.equal(xi0, xi1) and torch.equal(xa0, xa1)
    assert l0 == l1


def _config_chains():
    """The audio chains of the reference's own config (configs/config_multimodal_dino.yaml
    best_augments through process_augment_config, get_data.py:195-231): YAML key order, i.e.
    masks and noise BEFORE the time stretch and the crop -- not the gather kernel's order."""
    import os
    import yaml
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "configs", "config_multimodal_dino.yaml")) as f:
        cfg = yaml.safe_load(f)
    aug = A.MultiModalAugmentation(2, 4, augment_values=A.process_augment_config(cfg))
    return {"global": aug.global_transforms["audio"], "local": aug.local_transforms["audio"]}


@pytest.mark.parametrize("view", ["global", "local"])
@pytest.mark.parametrize("order", [0, 1])
def test_sequential_kernel_matches_oracle_on_the_config_chains(view, order):
    """avd_augment_views_seq vs the stage-by-stage restatement (OA.augment_one_seq) on the
    reference config's chains (every stage forced on in half the records): bit-exact without
    noise, |diff| <= 2e-5 with it (device logf/cosf, then interpolated by later stages)."""
    chain = _config_chains()[view]
    assert not A.fixed_order(chain)
    H = W = 112
    N, B, V = 9, 4, 3
    rng = np.random.default_rng(21)
    src = rng.integers(0, 256, (N, H * W), dtype=np.uint8)
    idx = rng.integers(0, N, B)
    lut = OA.normalise_lut("audio")
    rec_on, gm = _records([(k, kw, 1.0) for k, kw, _p in chain], B, V, H, W, 3)
    rec_p, _ = _records(chain, B, V, H, W, 4)
    rec = np.where((np.arange(B * V) % 2 == 0)[:, None], rec_on, rec_p)
    if gm is None:
        rec[:, 22] = -1
    kinds = A.chain_kinds(chain)
    seed = 0x1234567
    out = torch.empty((B, V, H, W) if order == 0 else (V, B, H, W), device="cuda")
    ops.augment_views(torch.from_numpy(src).cuda(), torch.from_numpy(idx).cuda(),
                      torch.from_numpy(lut).cuda(), torch.from_numpy(np.ascontiguousarray(rec)).cuda(),
                      None if gm is None else torch.from_numpy(gm.view(np.int32)).cuda(),
                      4, seed, V, H, W, out, order, kinds)
    got = out.cpu().numpy()
    ref = OA.augment_views(src, idx, lut, rec, gm, V, H, W, seed, order, kinds=kinds)
    noisy = (rec[:, 21] != 0).reshape(B, V)
    if order == 1:
        noisy = noisy.T
    np.testing.assert_array_equal(got[~noisy], ref[~noisy])
    np.testing.assert_allclose(got[noisy], ref[noisy], rtol=0, atol=2e-5)


@pytest.mark.parametrize("view,mod", [("global", "image"), ("local", "image"),
                                      ("global", "audio"), ("local", "audio")])
def test_sequential_kernel_equals_gather_kernel_in_fixed_order(view, mod):
    """The default chains through both kernels: identical views, noise included."""
    H = W = 28 if mod == "image" else 112
    rng = np.random.default_rng(8)
    src = torch.from_numpy(rng.integers(0, 256, (12, H * W), dtype=np.uint8)).cuda()
    lut = torch.from_numpy(OA.normalise_lut(mod)).cuda()
    chain = A.default_chains()[view][mod]
    idx = np.array([3, 1, 8, 0, 11])
    outs = []
    for seq in (False, True):
        aug = A.ViewAugmenter(src, lut, H, W, seed=7, sequential=seq)
        outs.append(aug(idx, chain, 4, order=1))
    assert torch.equal(outs[0], outs[1])


def test_config_chains_stage_bf16_views():
    """MultiModalAugmentation(augment_values=the config's best_augments).stage: the staged bf16
    views equal the f32 views of the same seeds rounded, originals included."""
    rng = np.random.default_rng(9)
    srcs = {"image": torch.from_numpy(rng.integers(0, 256, (10, 784), dtype=np.uint8)).cuda(),
            "audio": torch.from_numpy(rng.integers(0, 256, (10, 12544), dtype=np.uint8)).cuda()}
    luts = {k: torch.from_numpy(OA.normalise_lut(k)).cuda() for k in srcs}
    ch = _config_chains()
    idx = np.array([4, 9, 2])

    def mk():
        aug = A.MultiModalAugmentation(2, 4)
        aug.global_transforms["audio"], aug.local_transforms["audio"] = ch["global"], ch["local"]
        return aug.bind(A.ViewAugmenter(srcs["image"], luts["image"], 28, 28, seed=1),
                        A.ViewAugmenter(srcs["audio"], luts["audio"], 112, 112, seed=2))

    x_img = torch.empty(7 * 3 * 784, dtype=torch.bfloat16, device="cuda")
    x_aud = torch.empty(7 * 3 * 12544, dtype=torch.bfloat16, device="cuda")
    mk().stage(idx, x_img, x_aud, True)
    a32 = mk()
    gi, ga, li, la = a32(idx)
    ref = torch.cat([ga.transpose(0, 1).reshape(-1), la.transpose(0, 1).reshape(-1),
                     a32.audio.identity(idx).reshape(-1)])
    assert torch.equal(x_aud, ref.to(torch.bfloat16))
    assert torch.isfinite(ref).all() and (ref != 0).any()


def test_grouped_masking_kernel_equals_the_references_output():
    """avd_augment_views_seq with the reference's own randperm groups (tests/golden/
    augment_ref.npz, GroupedMasking.forward run here, get_data.py:60-108): bit-identical."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "augment_ref.npz"))
    src = z["src_u8"].reshape(6, 12544)
    gms, refs = [], []
    for r in range(3):
        gm = np.zeros(25, np.uint32)
        for g in z[f"gm{r}_idx"]:
            gm[g >> 5] |= np.uint32(1) << np.uint32(g & 31)
        gms.append(gm)
        refs.append(z[f"gm{r}_out"])
    rec = np.zeros((3, A.REC), np.float32)
    rec[:, 22] = np.arange(3)
    out = torch.empty((3, 1, 112, 112), device="cuda")
    ops.augment_views(torch.from_numpy(src).cuda(), torch.arange(3, device="cuda"),
                      torch.from_numpy(z["lut"]).cuda(), torch.from_numpy(rec).cuda(),
                      torch.from_numpy(np.stack(gms).view(np.int32)).cuda(), 4, 0, 1, 112, 112, out, 0,
                      [OA.K_GMASK])
    np.testing.assert_array_equal(out.cpu().numpy()[:, 0], np.stack(refs))


def test_workspace_allocation_leaves_no_queued_work():
    """The round-5 prefetch race: a workspace buffer allocated on the main stream
    while that stream still had queued kernels could be a block those kernels were using, and the
    data stream then wrote into it.  Workspace.get now synchronises after every (re)allocation,
    so a new buffer is safe for any stream: nothing is pending on the allocating stream after
    it, and a regrowth drops its old buffer only then."""
    from avdino.engine import Workspace
    ws = Workspace(torch.device("cuda"))
    a = torch.randn(2048, 2048, device="cuda")
    for _ in range(20):                      # a few ms of queued work on the current stream
        a = a @ a
        a /= a.norm()
    b = ws.get("x", 1 << 20)
    assert torch.cuda.current_stream().query(), "allocation returned with work still queued"
    for _ in range(20):
        a = a @ a
    ws.get("x", 1 << 21)                    # regrowth
    assert torch.cuda.current_stream().query()
    assert ws.get("x", 1 << 20).data_ptr() == ws.bufs["x"].data_ptr() != b.data_ptr()


@pytest.mark.parametrize("graph", [False, True])
def test_prefetched_augmentation_steps_equal_serial_steps(tmp_path, graph):
    """Real-data steps whose next batch is prefetched on the data stream (engine.prefetch,
    double-buffered staged inputs; the data stream starts after the step just queued, DESIGN
    3.6) give the same losses and parameters, bit for bit, as steps that augment each batch in
    front of it -- eager and graph-replayed."""
    from avdino.data import AVMNISTDinoLoader
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    root = _fake_avmnist(tmp_path, n=40)
    E, D, P = 32, 32, 16
    res = []
    for pre in (False, True):
        ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                               multimodal_mode="semi_supervised", device="cuda", staged=True)
        batches = list(ld)[:4] * 2
        store = ParamStore(multimodal_dino_sd("semi_supervised", E, D, P), "cuda:0", seed=1)
        eng = MultiCentralEngine(store, "semi_supervised", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                                 act_dtype=torch.bfloat16)
        eng.use_graph = graph
        eng.graph.warmup = 1
        losses = []
        for i, b in enumerate(batches):
            nxt = batches[i + 1] if (pre and i + 1 < len(batches)) else None
            losses.append(eng.step(b, next_batch=nxt).item())
        assert eng._pf is None
        res.append((losses, store.student.clone(), store.teacher.clone()))
    (l0, s0, t0), (l1, s1, t1) = res
    assert l0 == l1
    assert torch.equal(s0, s1) and torch.equal(t0, t1)


def test_trainer_prefetches_staged_batches(tmp_path):
    """Trainer.fit over a staged loader (one batch of look-ahead, model.prefetch after each
    optimizer step) equals the same fit over the collated views."""
    from avdino.data import AVMNISTDinoLoader
    from avdino.models import CentralMultiModalEncoder, MultiModalDINOWithMSELightning
    from avdino.trainer import Trainer
    root = _fake_avmnist(tmp_path, n=40)
    out = []
    for staged in (False, True):
        ld = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                               multimodal_mode="mse", device="cuda", staged=staged)
        torch.manual_seed(0)
        m = MultiModalDINOWithMSELightning(encoder_class=CentralMultiModalEncoder, projection_dim=16,
                                           output_dim=32, encoder_output_dim=32, dropout=0.0,
                                           device="cuda", precision="bf16", seed=0)
        tr = Trainer(max_epochs=1, limit_train_batches=3, logger=None)
        tr.fit(m, ld)
        out.append(m.model.store.student.clone())
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("view,mod", [("local", "image"), ("global", "audio")])
def test_augment_diagnostic_kernels_equal_the_gather_kernel(view, mod):
    """DESIGN 3.6's diagnostic builds of the gather kernel (tools/dbg_prefetch6.py): the LDS
    self-check build and the LDS-free build give the shipped kernel's bf16 views bit for bit on
    device-drawn records; the self-check finds its staged row intact and reports the record
    fields it used."""
    H = W = 28 if mod == "image" else 112
    rng = np.random.default_rng(6)
    src = torch.from_numpy(rng.integers(0, 256, (9, H * W), dtype=np.uint8)).cuda()
    lut = torch.from_numpy(OA.normalise_lut(mod)).cuda()
    aug = A.ViewAugmenter(src, lut, H, W, seed=3)
    B, V = 6, 4
    rec, gm = aug.records_dev(A.default_chains()[view][mod], B, V)
    idx = torch.from_numpy(rng.integers(0, 9, B)).cuda()
    seed, words = 0x5EED, gm.shape[1] if gm is not None else 0
    ref = torch.empty(V * B * H * W, dtype=torch.bfloat16, device="cuda")
    ops.augment_views(src, idx, lut, rec, gm, 4, seed, V, H, W, ref, 1)
    a = torch.empty_like(ref)
    b = torch.empty_like(ref)
    chk = torch.zeros(3, dtype=torch.int32, device="cuda")
    seen = torch.full_like(rec, -7.0)
    ops.call("avd_augment_views_lds_check", ops.p(src), ops.p(idx), B, V, H, W, ops.p(lut), ops.p(rec),
             ops.p(gm), words, 4, seed, 1, ops.p(a), ops.p(chk), ops.p(seen), ops.stream())
    ops.call("avd_augment_views_nolds", ops.p(src), ops.p(idx), B, V, H, W, ops.p(lut), ops.p(rec),
             ops.p(gm), words, 4, seed, 1, ops.p(b), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, ref) and torch.equal(b, ref)
    assert chk.tolist()[0] == 0
    ints = [0, 1, 2, 3, 17, 18, 19, 20, 22, 23, 24, 25, 26, 27]
    want = rec.clone()
    want[:, ints] = want[:, ints].trunc()
    assert torch.equal(seen, want)
