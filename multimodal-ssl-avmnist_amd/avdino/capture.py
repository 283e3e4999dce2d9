"""hipGraph capture of a training step, in segments around host points.

A step's device work is captured once per input shape and replayed (one host call per segment
instead of ~200 launches).  Data-parallel steps have host points inside the step: a
collective issued by the host (``torch.distributed`` over RCCL, or gloo in the rehearsal) that
reads and writes FIXED device buffers -- the global-negative all-gather / reduce-scatter of
InfoNCE (config 3) and NT-Xent (config 4), the early gradient bucket's all-reduce.  The step
body calls :func:`host_point` there.  Eagerly that just runs the collective; while capturing it
closes the current graph segment, executes it, runs the collective and opens the next segment,
so a replay is ``graph_0, collective_0, graph_1, ..., graph_n`` on the caller's stream, every
collective in the same order on every rank.  Work forked to side streams must be joined
before a host point (a segment, like any captured graph, ends with every forked stream
rejoined); callers join exactly there and nowhere else.
"""
import collections

import torch

from . import ops

_ACTIVE = None     # the _Capture in progress (host_point's target), else None



# Event lifetimes.  On this stack a HIP event destroyed while the device may still reach it
# (a fork / join event of a step queued ahead of the GPU, or one recorded into a capture) can
# corrupt the runtime: replays then segfaulted on the host in hipGraphLaunch
# (tests/test_gpu_step.py followed by tests/test_gpu_graph.py in one process, 4 of 4 runs; 0 of
# 2 with events kept alive, tools/pytest_keep_events.py).  So every event the engine creates
# (new_event) and every temporary of Stream.wait_stream / record_event (torch.cuda.streams.Event
# is this class from import on) stays referenced for the next 4096 event creations, and events
# created during a capture for as long as the graph exists.
_RING = collections.deque(maxlen=4096)
_HOLD = None


class _HeldEvent(torch.cuda.Event):
    def __new__(cls, *args, **kwargs):
        ev = super().__new__(cls, *args, **kwargs)
        _RING.append(ev)
        if _HOLD is not None:
            _HOLD.append(ev)
        return ev


torch.cuda.streams.Event = _HeldEvent


def new_event(**kwargs):
    """A torch.cuda.Event held alive past the work that waits on it (see above)."""
    return _HeldEvent(**kwargs)


class _Capture:
    def __init__(self, pool):
        self.pool, self.seq, self.g = pool, [], None

    def begin(self):
        self.g = torch.cuda.CUDAGraph()
        self.g.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def end(self):
        self.g.capture_end()
        self.seq.append(self.g)
        self.g.replay()            # capturing executed nothing: run the segment now
        self.g = None

    def cut(self, fn):
        self.end()
        fn()
        self.seq.append(fn)
        self.begin()


def host_point(fn):
    """Run the host-issued collective ``fn()`` at this point of the step (see module doc).
    ``fn`` must only touch buffers whose addresses are fixed across steps."""
    if _ACTIVE is None:
        fn()
    else:
        _ACTIVE.cut(fn)


def capturing():
    return _ACTIVE is not None


class GraphedStep:
    """A training step's device work captured once per input shape as a sequence of hipGraphs
    (torch.cuda.CUDAGraph over HIP stream capture, side streams joined by events) separated by
    host points, and replayed.  The first ``warmup`` calls per shape run eagerly (they size
    every workspace), the next one captures.

    A graph holds the device pointers of the scratch buffers it was captured over; when any of
    them is reallocated later (a larger key's eager warm-up grows a shared buffer, e.g. SimCLR's
    image/image mode captured before its audio/audio mode was first seen) the graph is stale:
    each capture records ``deps()`` after it -- the allocation epochs of exactly the buffers
    the step uses (its engine's workspaces and the shared GEMM / row-sum scratch; default: the
    shared scratch epoch alone) -- and is dropped and re-captured instead of replayed once
    they have moved."""

    def __init__(self, warmup=2, deps=None):
        self.warmup = warmup
        self.deps = deps if deps is not None else ops.alloc_epoch
        self.graphs = {}     # key -> (segments, allocation epoch after the capture, held events)
        self.seen = {}
        self.captures = 0
        self.pool = None
        self.stream = None

    def recapture(self):
        """Drop every captured graph; each key captures again at its next call (no eager
        warm-up: its workspaces are sized already) -- e.g. after changing what is captured
        with the step (bench.py's span marks)."""
        for key in self.graphs:
            self.seen[key] = self.warmup
        self.graphs = {}
        self.pool = None

    def segments(self, key):
        """Number of graph segments of the capture for ``key`` (None: not captured)."""
        ent = self.graphs.get(key)
        return None if ent is None else sum(1 for s in ent[0] if hasattr(s, "replay"))

    def run(self, key, body):
        global _ACTIVE
        ent = self.graphs.get(key)
        if ent is not None:
            if ent[1] == self.deps():
                for s in ent[0]:
                    if hasattr(s, "replay"):
                        s.replay()
                    else:
                        s()          # a host point's collective
                return
            del self.graphs[key]            # captured over buffers that have since moved
            self.seen[key] = self.warmup - 1
            if not self.graphs:
                # the last graph on the shared memory pool is gone, and with it the pool: the
                # next capture needs a new one (the allocator refuses a pool nobody holds)
                self.pool = None
        n = self.seen.get(key, 0)
        if n < self.warmup:
            self.seen[key] = n + 1
            body()
            return
        if _ACTIVE is not None:
            raise RuntimeError("nested step capture")
        torch.cuda.synchronize()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
            self.stream = torch.cuda.Stream()
        main = torch.cuda.current_stream()
        self.stream.wait_stream(main)
        cap = _Capture(self.pool)
        global _HOLD
        held = []
        with torch.cuda.stream(self.stream):
            _ACTIVE = cap
            _HOLD = held
            try:
                cap.begin()
                body()
                cap.end()
            except BaseException:
                if cap.g is not None:       # leave no stream in capture mode behind
                    try:
                        cap.g.capture_end()
                    except Exception:
                        pass
                raise
            finally:
                _ACTIVE = None
                _HOLD = None
        main.wait_stream(self.stream)
        self.graphs[key] = (cap.seq, self.deps(), held)
        self.captures += 1
