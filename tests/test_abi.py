"""The C-ABI library loads and exports every symbol include/avdino.h declares, the ctypes
prototypes cover them, and host-side validation rejects bad arguments before any launch
(no GPU needed: nothing here launches a kernel)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "avdino.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    fns = header_functions()
    assert "avd_cl_conv_fwd" in fns and "avd_adam" in fns and len(fns) >= 25


def test_library_exports_every_declared_symbol():
    from avdino import _lib
    missing = [f for f in header_functions() if not hasattr(_lib.lib, f)]
    assert not missing, missing


def test_ctypes_prototypes_cover_header():
    from avdino import _lib
    declared = set(header_functions()) - {"avd_last_error"}
    assert declared == set(_lib.PROTOS), (declared ^ set(_lib.PROTOS))


def test_host_helpers():
    from avdino._lib import lib
    assert lib.avd_version() >= 1
    assert lib.avd_cl_stat_rows(112, 112, 512, 5, 8, 16, 1) == 57344
    assert lib.avd_cl_stat_rows(14, 14, 512, 3, 32, 64, 1) == 1024
    assert lib.avd_cl_wgrad_chunks(7168, 16, 8, 5) == 512
    assert lib.avd_cl_wgrad_chunks(7168, 64, 32, 5) == 256
    assert lib.avd_cl_wgrad_chunks(12, 16, 8, 5) == 12
    assert lib.avd_colstats_parts(6144) == 384       # 16-row partials


def test_argument_validation_without_launch():
    from avdino._lib import lib
    # null pointers -> AVD_ERR_ARG; bad shapes -> AVD_ERR_SHAPE; bad dtype -> AVD_ERR_DTYPE
    assert lib.avd_cl_conv_fwd(None, None, None, None, None, 1, 1, 1, 8, 28, 28, 16, 5, 2, None) == -4
    dummy = ctypes.c_void_p(16)
    assert lib.avd_cl_conv_fwd(dummy, dummy, None, dummy, None, 1, 1, 1, 8, 28, 28, 16, 7, 2, None) == -1
    assert lib.avd_cl_conv_fwd(dummy, dummy, None, dummy, None, 7, 1, 1, 8, 28, 28, 16, 5, 2, None) == -4
    assert lib.avd_bn_finalize(dummy, 0, 1, 1, 2, dummy, dummy, 1e-5, 0.1, dummy, dummy, dummy,
                               dummy, None, None, None, 0, None) == -1
    assert lib.avd_stage_views(dummy, 2, None, 1, None, 4, 784, dummy, 0, None) == -4
    assert lib.avd_stage_views(dummy, 2, None, 0, None, 4, 783, dummy, 0, None) == -1
    assert lib.avd_act_fwd(dummy, dummy, 0, None, None, 4, 1, 8, 1.0, 0, None) == -1


def test_product_fails_loudly_without_library(tmp_path, monkeypatch):
    """No silent fallback: pointing the loader at a missing library raises on import."""
    import importlib
    import sys
    monkeypatch.setenv("AVDINO_LIB", str(tmp_path / "nope.so"))
    sys.modules.pop("avdino._lib", None)
    with pytest.raises(ImportError):
        importlib.import_module("avdino._lib")
    monkeypatch.delenv("AVDINO_LIB")
    sys.modules.pop("avdino._lib", None)
    importlib.import_module("avdino._lib")
