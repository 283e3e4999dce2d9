"""bench.py with engine class attributes overridden, for same-box A/Bs of route switches:
    python tools/ab_attr.py "ConvBranch.WGRAD_MAIN=frozenset({3})" -- --no-cpu-baseline --steps 30
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "multimodal-ssl-avmnist_amd"))

from avdino import engine  # noqa: E402

sep = sys.argv.index("--")
for spec in sys.argv[1:sep]:
    lhs, rhs = spec.split("=", 1)
    cls, attr = lhs.split(".")
    setattr(getattr(engine, cls), attr, eval(rhs))
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[sep + 1:]
import bench  # noqa: E402
bench.main()
