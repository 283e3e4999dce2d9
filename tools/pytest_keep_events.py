"""Debug: run pytest with every torch.cuda.Event kept alive for the whole session (no event is
destroyed while a captured graph or a queued wait may still refer to it); KEEP_EVENTS_RING=n
keeps only the last n.
    python tools/pytest_keep_events.py <pytest args>"""
import os
import sys

import pytest
import torch

import collections

_n = int(os.environ.get("KEEP_EVENTS_RING", "0"))
_KEEP = collections.deque(maxlen=_n) if _n else []
_Orig = torch.cuda.Event


class _KeptEvent(_Orig):
    def __new__(cls, *a, **k):
        e = _Orig.__new__(cls, *a, **k)
        _KEEP.append(e)
        return e


torch.cuda.Event = torch.cuda.streams.Event = _KeptEvent
sys.exit(pytest.main(sys.argv[1:]))
