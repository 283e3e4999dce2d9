"""Run-level telemetry of run_dino.experiment() (run_dino.py:191-225, 355, 409-464) on CPU:
the CSVLogger metrics.csv schema, ModelStatsCallback's logged keys, the performance summary's
model statistics; plus the --model multi_simple module surface and the graph-staleness rule
(no compute: these run without a GPU)."""
import csv
import os

import pytest
import torch


class _Mod:
    """What the callbacks touch on a LightningModule: log() and .model.device."""

    def __init__(self):
        self.logged = {}
        self.model = type("M", (), {"device": torch.device("cpu")})()

    def log(self, k, v, **kw):
        self.logged[k] = v


def test_csv_logger_schema(tmp_path):
    from avdino.trainer import CSVLogger
    lg = CSVLogger(str(tmp_path), name="logs_seed1")
    assert lg.log_dir.endswith(os.path.join("logs_seed1", "version_0"))
    lg.log_hyperparams({"learning_rate": 1e-4, "encoder_class": object})
    for s in (9, 19):
        lg.log_metrics({"train_loss_step": 1.0 / s, "epoch": 0}, step=s)
    lg.save()
    lg.log_metrics({"train_loss_epoch": 0.5, "mlp_acc": 10.0, "epoch_time": 2.0, "avg_batch_time": 0.1,
                    "epoch": 0}, step=19)
    lg.save()                                   # new keys: header widened, rows rewritten
    with open(lg.metrics_file_path) as f:
        rows = list(csv.reader(f))
    assert rows[0] == sorted(["avg_batch_time", "epoch", "epoch_time", "mlp_acc", "step",
                              "train_loss_epoch", "train_loss_step"])
    assert len(rows) == 4
    d = [dict(zip(rows[0], r)) for r in rows[1:]]
    assert [r["step"] for r in d] == ["9", "19", "19"]
    assert d[0]["train_loss_epoch"] == "" and d[2]["train_loss_step"] == ""
    assert os.path.exists(os.path.join(lg.log_dir, "hparams.yaml"))
    assert CSVLogger(str(tmp_path), name="logs_seed1").version == 1


def test_model_stats_callback_logs_reference_keys():
    from avdino.trainer import ModelStatsCallback
    cb, mod = ModelStatsCallback(), _Mod()
    tr = type("T", (), {"logger": None, "global_step": 3})()
    cb.on_train_start(tr, mod)
    cb.on_train_epoch_start(tr, mod)
    for i in range(3):
        cb.on_train_batch_start(tr, mod, None, i)
        cb.on_train_batch_end(tr, mod, None, None, i)
    cb.on_train_epoch_end(tr, mod)
    assert set(mod.logged) == {"epoch_time", "avg_batch_time"}
    assert len(cb.batch_times) == 3 and mod.logged["epoch_time"] >= 0
    cb.on_train_end(tr, mod)
    assert cb.total_training_time >= 0


@pytest.mark.parametrize("model", ["multi_central", "multi_simple"])
def test_model_stats_and_summary(tmp_path, model):
    import yaml
    from avdino import run_dino as R
    cfg = yaml.safe_load(open(os.path.join(os.path.dirname(__file__), "..", "configs",
                                           "config_multimodal_dino.yaml")))
    args = R.parse_args(["--model", model, "--training_mode", "mse", "--config",
                         os.path.join(os.path.dirname(__file__), "..", "configs", "config_multimodal_dino.yaml")])
    m = R.build_model(args, cfg, device="cpu")
    gflops, params = R.model_stats(m, 2, 4)
    n_state = sum(v.numel() for k, v in m.model.store.state_dict().items()
                  if not k.endswith(("running_mean", "running_var", "num_batches_tracked")) and k != "center")
    assert params == n_state
    assert gflops > 0
    tr = type("T", (), {"callback_metrics": {"train_loss": 5.0, "epoch_time": 60.0, "avg_batch_time": 0.5}})()
    res, perf = R.write_run_summary(m, args, cfg, str(tmp_path), 2, 4, None, tr, 120.0)
    name = res["model"]
    assert os.path.exists(tmp_path / f"final_results_{name}.csv")
    txt = (tmp_path / "performance_summary.txt").read_text()
    for k in ("model_name", "parameters", "gflops", "training_time_hours", "avg_epoch_time_minutes",
              "best_train_loss", "downstream_mlp_acc", "final_audio_gate"):
        assert k + ":" in txt


def test_multi_simple_module_reference_keys():
    from avdino.models import MODEL_MAP, MultiModalDINOWithMSELightning, SimpleMultiModalEncoder
    from oracle import spec as OS
    assert MODEL_MAP["multi_simple"] is SimpleMultiModalEncoder
    m = MultiModalDINOWithMSELightning(encoder_class=SimpleMultiModalEncoder, encoder_output_dim=32,
                                       output_dim=32, projection_dim=16, device="cpu")
    keys = list(m.state_dict().keys())
    assert keys == ["model." + k for k in OS.multimodal_dino_spec("mse", 32, 32, 16, encoder="multi_simple")]
    assert "model.student.image_encoder.14.weight" in keys and "model.student.audio_encoder.18.weight" in keys
    assert "arena_frozen" not in dict(m.model.named_parameters())      # no dead fc1/fc2 here


def test_graph_staleness_rule():
    """GraphedStep replays a graph only while none of the buffers it depends on moved since its
    capture: each Workspace keeps its own epoch, so another workspace growing (a probe's, a
    loss helper's) does not retire the graph."""
    from avdino import ops
    from avdino.engine import GraphedStep, Workspace
    ws = Workspace(torch.device("cpu"))
    other = Workspace(torch.device("cpu"))
    e0, g0 = ws.epoch, ops.alloc_epoch()
    ws.get("a", 10)
    assert ws.epoch == e0 + 1
    ws.get("a", 5)                      # fits: no reallocation
    assert ws.epoch == e0 + 1
    ws.get("a", 20)
    assert ws.epoch == e0 + 2
    assert ops.alloc_epoch() == g0      # the shared scratch epoch is not a workspace's

    class FakeGraph:
        replays = 0

        def replay(self):
            FakeGraph.replays += 1

    g = GraphedStep(warmup=1, deps=lambda: (ops.alloc_epoch(), ws.epoch))
    g.graphs["k"] = ([FakeGraph()], g.deps())
    g.seen["k"] = 1
    calls = []
    g.run("k", lambda: calls.append(1))
    assert FakeGraph.replays == 1 and not calls
    other.get("z", 1 << 10)             # someone else's workspace: still replayed
    g.run("k", lambda: calls.append(1))
    assert FakeGraph.replays == 2 and not calls
    ws.get("b", 4)                      # one of ITS buffers moved: the graph is stale
    g.warmup = 2                        # (keep the re-run eager: no capture on CPU)
    g.run("k", lambda: calls.append(1))
    assert "k" not in g.graphs and calls == [1] and FakeGraph.replays == 2
    assert g.pool is None               # the last graph went with its pool


def test_segmented_replay_order():
    """A captured step with host points replays as graph, collective, graph, ... in order;
    outside a capture a host point just runs its collective."""
    from avdino import ops
    from avdino.capture import GraphedStep, capturing, host_point
    order = []

    class Seg:
        def __init__(self, i):
            self.i = i

        def replay(self):
            order.append(("g", self.i))

    g = GraphedStep(warmup=1)
    g.graphs["k"] = ([Seg(0), lambda: order.append(("c", 0)), Seg(1),
                      lambda: order.append(("c", 1)), Seg(2)], ops.alloc_epoch())
    g.run("k", lambda: order.append("eager"))
    assert order == [("g", 0), ("c", 0), ("g", 1), ("c", 1), ("g", 2)]
    assert g.segments("k") == 3 and g.segments("x") is None
    assert not capturing()
    hit = []
    host_point(lambda: hit.append(1))
    assert hit == [1]


def test_workspace_canary_guards(monkeypatch):
    """Workspace.GUARD (tools/dbg_guard.py): a canary after every buffer; check_guards() names a
    buffer whose writer ran past its end, and production (GUARD = 0) allocates no guard."""
    from avdino.engine import Workspace
    ws = Workspace(torch.device("cpu"))
    ws.get("a", 10)
    assert ws.guards == {} and ws.check_guards() == []
    monkeypatch.setattr(Workspace, "GUARD", 16)
    ws = Workspace(torch.device("cpu"))
    a = ws.get("a", 10)
    b = ws.get("b", 3, torch.int64)
    a.fill_(1.0)
    b.fill_(-1)
    assert ws.check_guards() == []
    ws.guards["b"][0].view(torch.uint8)[3 * 8 + 5] = 0      # one byte past b's end
    assert ws.check_guards() == [("b", 5, 1)]
    assert ws.get("a", 10).numel() == 10


def test_event_ring_is_installed():
    """avdino.capture holds events past the work that waits on them: importing it
    makes Stream.wait_stream's temporaries the holding subclass, bounded to the last 4096."""
    from avdino import capture
    assert torch.cuda.streams.Event is capture._HeldEvent
    assert issubclass(capture._HeldEvent, torch.cuda.Event) and torch.cuda.Event is not capture._HeldEvent
    assert capture._RING.maxlen == 4096
