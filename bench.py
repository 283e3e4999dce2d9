#!/usr/bin/env python3
"""Benchmark: AVMNIST audio-image pairs/sec of the multimodal-DINO training step
(BASELINE.json metric), BASELINE config 2: multi_central, training_mode mse, B=1024 per GPU,
2 global + 4 local views, E=D=256, P=128, bf16 activations (fp32 params/accumulation).

A step = everything the reference's training step does: staging of the views,
student (6 views + originals) and teacher (2 views) encoders, projections, DINO + MSE losses,
centre update, teacher EMA, full backward, gradient all-reduce (N>1), Adam.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank/GPU)

Rank 0 prints ONE JSON line.  Inputs are synthetic AVMNIST-shaped tensors (pixel values
randint(0,256)/255) generated on the device before the timed region; weights random-init.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

METRIC = "AVMNIST audio-image pairs/sec (multimodal DINO step) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# dense, no sparsity; fp8 = the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (2x bf16) the fp8
# mode's conv kernels run on
MFMA_PEAK_TFS = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0}   # fp8: the dense block-scaled peak
# SURVEY 8(d) "BN-barrier" algorithmic HBM bytes per pair of a whole training step (inputs read
# once, each train-mode-BN'd conv output written once and read once forward, saved output read
# + its gradient written / read backward; weights amortised), bf16 storage; f32 doubles them
STEP_BYTES_PER_PAIR_BF16 = {"mse": 17.37e6, "infonce": 17.37e6, "semi_supervised": 17.37e6,
                            "default": 15.15e6, "simclr": 8.0e6, "uni": 1.24e6}
STEP_FLOPS_PER_PAIR = {"mse": 1794.6e6, "infonce": 1794.6e6, "semi_supervised": 1793.9e6,
                       "default": 1561.1e6, "simclr": 1104.3e6, "uni": 124.6e6}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="pairs per GPU per step (default: the workload's BASELINE config)")
    ap.add_argument("--mode", default="mse", choices=["default", "mse", "infonce", "semi_supervised"])
    ap.add_argument("--workload", default="dino", choices=["dino", "uni", "simclr"],
                    help="dino = MultiModalDINO* (--mode; config 2 mse / config 3 infonce with "
                         "all-gathered negatives / config 5 semi_supervised); uni = UniModalDINO "
                         "ImageEncoder 2 global views B=64 (config 1); simclr = multimodal SimCLR "
                         "with all-gathered NT-Xent negatives, B=2048/GPU (config 4)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32", "fp8"],
                    help="fp8: the mid-layer convs' forward, input gradient and weight gradient "
                         "on the block-scaled e4m3 MFMA (config 5); maps stored bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every kernel from Python each step instead of replaying the "
                         "captured hipGraph of the step")
    ap.add_argument("--pipeline", action="store_true",
                    help="multimodal DINO: run each step's teacher forward under the previous "
                         "step's backward (engine.pipeline; same losses, measured no faster)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo only to rehearse N>1 with several "
                         "ranks sharing one GPU")
    ap.add_argument("--cpu-batch", type=int, default=1024,
                    help="pairs per CPU step (config 2's B; the sample is >= 2 timed steps)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--probe-dominant", type=int, default=0, metavar="K",
                    help="after warm-up, replay only the dominant launch K times and exit "
                         "(run under rocprofv3 --pmc; tools/pmc_traffic.py turns the last K "
                         "dispatches into the roofline's per-launch HBM traffic)")
    ap.add_argument("--dominant", default=None, metavar="KEY",
                    help="use this launch key as the roofline kernel instead of the warm-up's "
                         "most expensive one (tools/gpu_pmc.sh passes the bench line's key)")
    ap.add_argument("--probe", action="store_true",
                    help="--mode semi_supervised (config 5): after the timed region, time one "
                         "epoch-end linear-probe epoch (on_train_epoch_end, dino.py:878-951: 55000 "
                         "train + 5000 validation samples in batches of 128, dino.py:795-802) and "
                         "report it separately under \"probe\" (SURVEY 8(d)); not part of value")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"),
                    help="PMC traffic table written by tools/pmc_traffic.py")
    return ap.parse_args()


def load_traffic(path, key):
    """Per-launch HBM bytes of ``key`` measured by a separate rocprofv3 --pmc pass (FETCH_SIZE
    doubled per the gfx950 correction + WRITE_SIZE), or None if that launch was not probed."""
    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    # (the bytes of a launch do not depend on the stream it was issued on)
    base = key.replace(" @side", "")
    e = tab.get(key) or tab.get(base) or tab.get(base + " @side")
    return None if e is None else e.get("traffic_bytes")


def synthetic_pool(n, B, G, L, device, seed):
    """Device-resident AVMNIST-shaped batches (get_data.py:456-467 value range)."""
    gen = torch.Generator(device=device).manual_seed(seed)
    pool = []

    def px(*shape):
        return torch.randint(0, 256, shape, generator=gen, device=device, dtype=torch.int32).float() / 255.0

    for _ in range(n):
        pool.append({"g_img": px(B, G, 1, 28, 28), "g_aud": px(B, G, 1, 112, 112),
                     "l_img": px(B, L, 1, 28, 28), "l_aud": px(B, L, 1, 112, 112),
                     "image": px(B, 1, 28, 28), "audio": px(B, 1, 112, 112),
                     "label": torch.randint(0, 10, (B,), generator=gen, device=device)})
    return pool


def build_workload(args, device, act, world, rank, avdist):
    """(engine, device batch pool, pairs per GPU per step, config text, model name)."""
    from avdino.engine import Hyper, MultiCentralEngine, SimCLREngine, UniModalEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd, simclr_sd, unimodal_dino_sd
    hook = avdist.grad_allreduce_hook() if world > 1 else None
    if args.workload == "uni":
        B, D, P = args.batch or 64, 256, 128
        store = ParamStore(unimodal_dino_sd("image_simple", D, P), device, seed=0)
        if world > 1:
            avdist.broadcast_parameters(store)
        eng = UniModalEngine(store, "image_simple", D, P, Hyper(), act_dtype=act, cos_alpha=0.0,
                             grad_hook=hook, buffer_hook=avdist.broadcast_buffers if world > 1 else None,
                             seed=rank, step_order="pretrain")
        pool = synthetic_pool(2, B, 2, 0, device, 1234 + rank)
        return (eng, pool, B, f"UniModalDINO ImageEncoder, 2 global views, B={B}/GPU, D={D}, P={P}, "
                              f"training_structures.pretrain_dino step (AdamW, EMA after the step; "
                              f"BASELINE config 1)", "image_simple")
    if args.workload == "simclr":
        B, D, P = args.batch or 2048, 256, 256
        store = ParamStore(simclr_sd(D, P), device, seed=0, has_teacher=False,
                           groups=SimCLREngine.GROUPS)
        if world > 1:
            avdist.broadcast_parameters(store)
        eng = SimCLREngine(store, D, P, Hyper(weight_decay=0.0), act_dtype=act, negatives="global",
                           grad_hook=hook)
        gen = torch.Generator(device=device).manual_seed(1234 + rank)

        def px(*shape):
            return torch.randint(0, 256, shape, generator=gen, device=device, dtype=torch.int32).float() / 255.0

        pool = [{"img1": px(B, 1, 28, 28), "spec1": px(B, 1, 112, 112), "img2": px(B, 1, 28, 28),
                 "spec2": px(B, 1, 112, 112)} for _ in range(2)]
        return (eng, pool, B, f"multimodal SimCLR, random modality pair per step, NT-Xent over "
                              f"all-gathered negatives, B={B}/GPU, D=P={D} (BASELINE config 4)",
                "multimodal_simclr")
    E, D, P, G, L = 256, 256, 128, 2, 4
    B = args.batch or (4096 if args.mode == "semi_supervised" else 1024)
    store = ParamStore(multimodal_dino_sd(args.mode, E, D, P), device, seed=0)
    if world > 1:
        avdist.broadcast_parameters(store)
    # DDP semantics of the reference's multi-GPU run: rank-0 buffers broadcast before each
    # forward, one averaged all-reduce of the flat live-gradient arena after backward
    eng = MultiCentralEngine(store, args.mode, E, D, P, Hyper(), act_dtype=act, grad_hook=hook,
                             buffer_hook=avdist.broadcast_buffers if world > 1 else None, seed=rank,
                             negatives="global", conv_fp8=args.dtype == "fp8")
    eng.pipeline = args.pipeline
    pool = synthetic_pool(2, B, G, L, device, 1234 + rank)
    prec = ("block-scaled e4m3 MFMA mid-layer conv forward, input gradient and weight gradient, "
            "bf16 maps" if args.dtype == "fp8" else args.dtype)
    cfg = {"mse": "BASELINE config 2", "infonce": "BASELINE config 3 shape, all-gathered negatives",
           "semi_supervised": f"BASELINE config 5 shape, {prec}",
           "default": "default mode"}[args.mode]
    return (eng, pool, B, f"multi_central {args.mode} training step, B={B}/GPU, {G} global + {L} "
                          f"local views, E=D={E}, P={P} ({cfg})", "multi_central")


def time_probe(eng, args, device, act, rank):
    """One epoch-end linear-probe epoch over the trained student (avdino.probe.LinearProbe =
    DownstreamClassifier + AdamW over the reference's AVMNISTDataModule loaders, batch 128):
    synthetic labelled samples resident in HBM, one warm-up pass over a few batches (workspace
    sizing), then the full epoch timed with a device sync on both sides."""
    from avdino.probe import LinearProbe
    n_train, n_val, pb = 55000, 5000, 128
    gen = torch.Generator(device=device).manual_seed(4321 + rank)

    def split(n):
        img = torch.randint(0, 256, (n, 1, 28, 28), generator=gen, device=device, dtype=torch.int32).float() / 255.0
        aud = torch.randint(0, 256, (n, 1, 112, 112), generator=gen, device=device, dtype=torch.int32).float() / 255.0
        lab = torch.randint(0, 10, (n,), generator=gen, device=device)
        return [(img[i:i + pb], aud[i:i + pb], lab[i:i + pb]) for i in range(0, n, pb)]

    train, valid = split(n_train), split(n_val)
    probe = LinearProbe(eng.store, "multi_central", eng.D, eng.E, lr=eng.hp.lr, act_dtype=act,
                        fusion_dropout=eng.hp.fusion_dropout)
    probe.run_epoch(train[:3], valid[:2])             # warm-up: workspaces, first launches
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = probe.run_epoch(train, valid)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"epoch_ms": round(el * 1e3, 2), "samples_per_s": round((n_train + n_val) / el, 1),
            "train_batches": len(train), "valid_batches": len(valid), "batch": pb,
            "train_samples": n_train, "valid_samples": n_val, "dtype": args.dtype if args.dtype != "fp8" else "bf16",
            "mlp_acc": round(out["mlp_acc"], 3), "val_loss": round(out["val_loss"], 5),
            "what": "on_train_epoch_end linear probe (dino.py:878-951): frozen train-mode student copy, "
                    "Linear(D,128)-ReLU-Linear(128,10) with AdamW per batch over the train split, then "
                    "eval-mode evaluate() over the validation split; synthetic AVMNIST-shaped data in HBM"}


def host_cpu():
    """The host CPU the baseline ran on (lscpu's model name and core counts, read from
    /proc/cpuinfo: lscpu may be absent on the GPU box): model, physical cores, logical CPUs, the
    CPUs this process may run on (affinity), the physical cores among them, and the cgroup CPU
    quota (cpu.max) when one is set."""
    model, phys, cpu2core = None, set(), {}
    cur = {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in list(f) + [""]:
                if not line.strip():
                    if "physical id" in cur and "core id" in cur:
                        core = (cur["physical id"], cur["core id"])
                        phys.add(core)
                        if "processor" in cur:
                            cpu2core[int(cur["processor"])] = core
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                cur[k] = v
                if k == "model name" and model is None:
                    model = v
    except OSError:
        pass
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = list(range(os.cpu_count() or 1))
    aff_cores = len({cpu2core[c] for c in aff if c in cpu2core}) or None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = -(-int(q) // int(per))
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "physical_cores": len(phys) or None, "logical_cpus": os.cpu_count(),
            "affinity_cpus": len(aff), "affinity_physical_cores": aff_cores, "cgroup_cpu_quota": quota}


def cpu_threads(host):
    """Threads for the CPU baseline: one per physical core this process may use (BASELINE.md
    section 2: torch.set_num_threads(cpu count)) -- the physical cores of its affinity set,
    capped by a cgroup CPU quota when the box enforces one.  ``cores`` in the line is this
    number: one thread per physical core."""
    n = host.get("affinity_physical_cores") or host.get("affinity_cpus") or os.cpu_count() or 1
    if host.get("cgroup_cpu_quota"):
        n = min(n, host["cgroup_cpu_quota"])
    return max(1, int(n))


class _Threads:
    """torch.set_num_threads(n) for a block, restored afterwards."""

    def __init__(self, n):
        self.n = n

    def __enter__(self):
        self.old = torch.get_num_threads()
        torch.set_num_threads(self.n)

    def __exit__(self, *exc):
        torch.set_num_threads(self.old)


def cpu_baseline_uni(batch, seconds):
    """Config 1's reference path on the host cores: training_structures.pretrain_dino's step
    (oracle/torch_port.py UniImageDINO + pretrain_step: AdamW, EMA after the step), fp32."""
    host = host_cpu()
    with _Threads(cpu_threads(host)):
        return _cpu_baseline_uni(batch, seconds, host)


def _cpu_baseline_uni(batch, seconds, host):
    from oracle import torch_port as TP
    torch.manual_seed(0)
    model = TP.UniImageDINO()
    model.train()
    opt = torch.optim.AdamW(list(model.parameters()), lr=1e-4)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (batch, 2, 1, 28, 28), generator=g).float() / 255.0
    TP.pretrain_step(model, opt, x)
    n, t0 = 0, time.perf_counter()
    while True:
        TP.pretrain_step(model, opt, x)
        n += 1
        el = time.perf_counter() - t0
        if (n >= 2 and el >= seconds) or n >= 2000:
            break
    return {"value": round(batch * n / el, 2), "unit": "pairs/s", "cores": torch.get_num_threads(),
            "kind": "port", "host": host,
            "sample": f"oracle/torch_port.py UniImageDINO training_structures.pretrain_dino step "
                      f"(dino_train.py:143-161), fp32, B={batch}, 2 global views, {n} timed steps "
                      f"({el:.1f} s) after 1 warm-up, torch CPU {torch.get_num_threads()} threads, one per "
                      f"physical core"}


def cpu_baseline(batch, seconds):
    """The reference algorithm on the host cores (oracle/torch_port.py, fp32, per-view loops,
    Python EMA, torch.optim.Adam) on a bounded sample: B pairs/step, >= 2 timed steps."""
    host = host_cpu()
    with _Threads(cpu_threads(host)):
        return _cpu_baseline(batch, seconds, host)


def _cpu_baseline(batch, seconds, host):
    from oracle import torch_port as TP
    torch.manual_seed(0)
    model = TP.DinoMSE()
    model.train()
    opt = TP.make_optimizer(model)
    g = torch.Generator().manual_seed(1)

    def px(*shape):
        return torch.randint(0, 256, shape, generator=g).float() / 255.0

    def mk(n):
        return {"g_img": px(n, 2, 1, 28, 28), "g_aud": px(n, 2, 1, 112, 112),
                "l_img": px(n, 4, 1, 28, 28), "l_aud": px(n, 4, 1, 112, 112),
                "image": px(n, 1, 28, 28), "audio": px(n, 1, 112, 112)}

    TP.train_step(model, opt, mk(32))  # warm-up (code paths, allocator) on a small batch
    b = mk(batch)
    n, t0 = 0, time.perf_counter()
    while True:
        TP.train_step(model, opt, b)
        n += 1
        el = time.perf_counter() - t0
        if (n >= 2 and el >= seconds) or n >= 400:
            break
    return {"value": round(batch * n / el, 2), "unit": "pairs/s", "cores": torch.get_num_threads(),
            "kind": "port", "host": host,
            "sample": f"oracle/torch_port.py multi_central mse step (the reference's Lightning "
                      f"training_step ops, dino.py:1214-1238), fp32, B={batch}, 2 global + 4 local "
                      f"views, {n} timed steps ({el:.1f} s) after a B=32 warm-up step, torch CPU "
                      f"{torch.get_num_threads()} threads, one per physical core"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    local = local % max(torch.cuda.device_count(), 1)   # (rehearsal: ranks may share a GPU)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    from avdino import ops
    from avdino import dist as avdist
    act = torch.float32 if args.dtype == "f32" else torch.bfloat16
    if args.dtype == "fp8" and args.workload != "dino":
        raise SystemExit("--dtype fp8 is the multimodal DINO conv path (config 5); use --workload dino")
    eng, pool, B, workload, model = build_workload(args, device, act, world, rank, avdist)

    last = [-1]

    def step(i):
        """Step i of the run over the batch pool (multimodal DINO: the next batch rides along
        for the pipelined teacher forward)."""
        last[0] = i
        if getattr(eng, "pipeline", False):
            return eng.step(pool[i % len(pool)], next_batch=pool[(i + 1) % len(pool)])
        return eng.step(pool[i % len(pool)])

    # warm-up: eager steps (the second one times every instrumented kernel to find the dominant
    # one; the first one's launches are cold), then -- graph mode -- the step's capture
    # graph replay needs one eager warm-up step (it sizes every workspace) and the capture
    # inside the warm-up: with fewer than 2 warm-up steps the bench runs eagerly
    use_graph = not args.no_graph and not args.probe_dominant and args.warmup >= 2
    eng.use_graph = use_graph
    eng.graph.warmup = min(2, max(args.warmup - 1, 0))
    ops.TIMER = None
    wtimer = None
    # the timed warm-up step must run eagerly: with graphs, calls >= graph.warmup capture (and
    # events recorded inside a capture have no timestamps)
    t_idx = min(1, args.warmup - 1)
    if use_graph and t_idx >= eng.graph.warmup:
        t_idx = -1
    dominant = hbm_dom = watch = None

    def hbm_bound(d):
        return d["bytes"] / (HBM_PEAK_GBS * 1e9) >= d["flops"] / (MFMA_PEAK_TFS[args.dtype] * 1e12)

    def pick_watch():
        """The dominant launch (largest summed time in the timed eager warm-up step) and the
        largest HBM-bound one (roofline_hbm: when the dominant launch trades HBM bytes for
        recompute it is not a streaming kernel).  In graph mode these are only the eager
        estimate: the candidates (the top launches of both kinds) are then timed inside the
        replayed step (select_in_graph) and the bench reports the in-graph maxima."""
        summ = wtimer.summary() if wtimer is not None else {}
        dom = max(summ, key=lambda k: summ[k]["ms"]) if summ else None
        if args.dominant:
            if args.dominant not in summ:
                raise SystemExit(f"--dominant {args.dominant!r}: no such launch key")
            dom = args.dominant
        hk = [k for k in summ if k != dom and hbm_bound(summ[k])]
        hd = max(hk, key=lambda k: summ[k]["ms"]) if hk else None
        return summ, dom, hd, [k for k in (dom, hd) if k is not None] or None

    def candidates(summ, n_top=6, n_hbm=3):
        order = sorted(summ, key=lambda k: -summ[k]["ms"])
        c = order[:n_top] + [k for k in order if hbm_bound(summ[k])][:n_hbm]
        return list(dict.fromkeys(c))

    def select_in_graph(summ, watch):
        """Replay the captured step (spans on every candidate), pick the dominant and the
        HBM-bound launch by their summed in-graph time, then capture again with spans on those
        two only (what the timed region carries)."""
        spans = ops.SPANS
        spans.reset()
        for _ in range(3):
            step(last[0] + 1)
        torch.cuda.synchronize()
        ing = spans.read()
        ms = {k: ing[k.replace(" @side", "")][1] / 1e3 for k in watch if ing.get(k.replace(" @side", ""))}
        if not ms:
            return None
        dom = args.dominant or max(ms, key=ms.get)
        hk = [k for k in ms if k != dom and hbm_bound(summ[k])]
        hd = max(hk, key=ms.get) if hk else None
        if rank == 0:
            print("in-graph candidates (ms over 3 steps): " +
                  ", ".join(f"{k} {v:.3f}" for k, v in sorted(ms.items(), key=lambda kv: -kv[1])),
                  file=sys.stderr, flush=True)
        return dom, hd

    summ = {}
    for i in range(args.warmup):
        ops.TIMER = ops.KernelTimer() if i == t_idx else None
        wtimer = ops.TIMER or wtimer
        step(i)
        if i == t_idx:
            ops.TIMER = None
            summ, dominant, hbm_dom, watch = pick_watch()
            if use_graph and watch and not args.probe_dominant:
                # in-graph spans of the candidate launch sites, captured with the step: their
                # duration inside the replayed step (no host hook exists there)
                watch = candidates(summ)
                ops.SPANS = ops.SpanTimer(device, watch)
    ops.TIMER = None
    if use_graph and ops.SPANS is not None and not args.probe_dominant and args.workload != "simclr":
        sel = select_in_graph(summ, watch)
        if sel is not None:
            dominant, hbm_dom = sel
            watch = [k for k in (dominant, hbm_dom) if k is not None]
            ops.SPANS = ops.SpanTimer(device, watch)
            eng.graph.recapture()
            step(last[0] + 1)                # the capture with the two watched launches
            step(last[0] + 1)
    if use_graph and args.workload == "simclr":
        # SimCLR draws a modality pair per step (one captured graph per pair): capture all four
        # before the timed region (explicit modes do not consume the engine's mode draws)
        for m in range(4):
            while eng.graph.segments((m, B)) is None:
                eng.step(pool[0], mode=m)
    if dominant is None and watch is None and wtimer is not None:
        summ, dominant, hbm_dom, watch = pick_watch()
    ops.TIMER = None if use_graph else ops.KernelTimer(only=watch)

    if args.probe_dominant:
        ops.TIMER = ops.KernelTimer(only=dominant)
        eng.step(pool[0])                 # captures the dominant launch (inputs stay live)
        torch.cuda.synchronize()
        fn = ops.TIMER.replay
        for _ in range(args.probe_dominant):
            fn()
        torch.cuda.synchronize()
        if rank == 0:
            print(json.dumps({"probe": dominant, "replays": args.probe_dominant,
                              "algorithmic_bytes": int(summ[dominant]["bytes"] / summ[dominant]["calls"])}),
                  flush=True)
        return

    spans = ops.SPANS
    if spans is not None:
        spans.reset()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i0 = last[0] + 1
    for i in range(i0, i0 + args.steps):
        loss = step(i)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    lv = loss.item()
    if not math.isfinite(lv):
        raise SystemExit(f"non-finite loss {lv}")
    in_graph = spans.read() if spans is not None else {}
    ops.SPANS = None
    if use_graph:
        # HIP events around the watched launches in eager steps after the timed region as well
        # (eager_avg_launch_us); the in-graph spans of the timed region are the primary figure
        eng.use_graph = False
        ops.TIMER = ops.KernelTimer(only=watch)
        for _ in range(3):
            step(last[0] + 1)
        torch.cuda.synchronize()

    timed = ops.TIMER.summary()
    eager = dict(timed)
    for k in list(timed):
        sp = in_graph.get(k.replace(" @side", ""))
        if sp:
            n, us, nb, fl = sp
            timed[k] = {"calls": n, "ms": us / 1e3, "bytes": nb * n, "flops": fl * n, "in_graph": True}
    if dominant is None and timed:
        dominant = max(timed, key=lambda k: timed[k]["ms"])

    def roofline_of(k):
        if k not in timed:
            return None
        d = timed[k]
        avg_s = d["ms"] / d["calls"] / 1e3
        nb = d["bytes"] / d["calls"]
        fl = d["flops"] / d["calls"]
        peak_tf = MFMA_PEAK_TFS[args.dtype]
        hbm_bound = nb / (HBM_PEAK_GBS * 1e9) >= fl / (peak_tf * 1e12)
        if hbm_bound:
            ach, peak, unit = nb / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
        else:
            ach, peak, unit = fl / avg_s / 1e12, peak_tf, "TFLOP/s"
        r = {"bound": "hbm" if hbm_bound else "mfma", "kernel": k,
             "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
             "traffic": load_traffic(args.traffic, k),
             "avg_launch_us": round(avg_s * 1e6, 2),
             "timing": ("in-graph span marks over the timed region" if d.get("in_graph") else
                        "HIP events, eager steps" + (" after the timed region" if use_graph else "")),
             "algorithmic_bytes": int(nb), "algorithmic_flops": int(fl),
             "kernel_share_of_step": round(d["ms"] / (args.steps if d.get("in_graph") or not use_graph else 3) /
                                           (elapsed * 1e3 / args.steps), 4)}
        if d.get("in_graph") and k in eager:
            e = eager[k]
            r["eager_avg_launch_us"] = round(e["ms"] / e["calls"] * 1e3, 2)
        return r

    def isolated(k, reps=10):
        """The launch replayed alone (same inputs, its own stream idle otherwise), HIP events
        around ``reps`` back-to-back replays: the kernel's own speed, free of the time-sharing
        with the other streams' kernels that the in-step duration includes."""
        ops.TIMER = ops.KernelTimer(only=[k])
        step(last[0] + 1)          # consecutive: a pipelined step expects the previous next_batch
        torch.cuda.synchronize()
        fn, ops.TIMER = ops.TIMER.replay, None
        if fn is None:
            return None
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / reps

    roof = roofline_of(dominant)
    roof_hbm = roofline_of(hbm_dom) if hbm_dom is not None else None
    for r in (roof, roof_hbm):
        if r is None:
            continue
        iso = isolated(r["kernel"])
        if iso:
            d = timed[r["kernel"]]
            amount = (d["bytes"] if r["unit"] == "GB/s" else d["flops"]) / d["calls"]
            ach = amount / (iso * 1e-6) / (1e9 if r["unit"] == "GB/s" else 1e12)
            r["isolated_avg_launch_us"] = round(iso, 2)
            r["isolated_achieved"] = round(ach, 2)
            r["isolated_frac"] = round(ach / r["peak"], 4)

    total_pairs = world * B * args.steps
    value = total_pairs / elapsed
    # whole-step roofline: pairs/s per GPU against min(HBM ceiling, MFMA ceiling)
    key = args.mode if args.workload == "dino" else args.workload
    bpp = STEP_BYTES_PER_PAIR_BF16[key] * (2 if args.dtype == "f32" else 1)
    fpp = STEP_FLOPS_PER_PAIR[key]
    ceil_hbm = HBM_PEAK_GBS * 1e9 / bpp
    ceil_mfma = MFMA_PEAK_TFS[args.dtype] * 1e12 / fpp
    per_gpu = value / world
    step_roof = {"bound": "hbm" if ceil_hbm <= ceil_mfma else "mfma",
                 "bytes_per_pair": bpp, "flops_per_pair": fpp,
                 "ceiling_pairs_per_s_per_gpu": round(min(ceil_hbm, ceil_mfma), 1),
                 "achieved_GBps": round(per_gpu * bpp / 1e9, 1),
                 "achieved_TFLOPs": round(per_gpu * fpp / 1e12, 2),
                 "frac": round(per_gpu / min(ceil_hbm, ceil_mfma), 4),
                 "traffic_bytes_per_pair": load_traffic(args.traffic, "step:" + key)}
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic: randint(0,256)/255 AVMNIST-shaped views resident in HBM; random-init weights",
        "config": {"workload": workload,
                   "model": model, "global_batch": world * B, "seq_len": None,
                   "parallelism": f"dp{world}"},
        "roofline": roof,
        "roofline_hbm": roof_hbm,
        "step_roofline": step_roof,
        "timed_region_s": round(elapsed, 4),
        "host_issue_ms_per_step": round(t_issue * 1e3 / args.steps, 3),
        "graph": use_graph,
        "teacher_pipelined": bool(getattr(eng, "pipeline", False)),
        "final_loss": round(lv, 6),
    }
    if args.probe:
        if args.workload != "dino" or args.mode != "semi_supervised":
            raise SystemExit("--probe: the epoch-end probe is timed for --mode semi_supervised (config 5)")
        out["probe"] = time_probe(eng, args, device, act, rank)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "dino" \
            and args.mode == "mse":
        out["cpu_baseline"] = cpu_baseline(args.cpu_batch, args.cpu_seconds)
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "uni":
        out["cpu_baseline"] = cpu_baseline_uni(B, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
