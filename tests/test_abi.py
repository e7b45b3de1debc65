"""CPU-side checks of the C ABI: the built library loads and exports every function
include/daclip_hip.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared():
    src = open(os.path.join(ROOT, "include", "daclip_hip.h")).read()
    return sorted(set(re.findall(r"\b(dac_[a-z_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared()
    for n in ("dac_create", "dac_set_weight", "dac_finalize_weights", "dac_encode_image",
              "dac_unet_forward", "dac_sde_reverse", "dac_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from daclip_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdaclip_hip.so not built")
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing
    assert sorted(_lib.EXPORTS) == declared()


def test_create_without_gpu_fails_cleanly():
    import torch
    from daclip_amd import _lib
    if torch.cuda.is_available() or not os.path.exists(_lib.LIB_PATH):
        pytest.skip("CPU-only check")
    with pytest.raises(RuntimeError, match="GPU"):
        _lib.Handle(torch.device("cuda", 0), "fp32", _lib.DacConfig())


def test_config_struct_matches_header():
    """daclip_amd._lib.DacConfig must list dac_config's fields in header order (the library
    reads the whole struct)."""
    from daclip_amd import _lib
    src = open(os.path.join(ROOT, "include", "daclip_hip.h")).read()
    body = re.search(r"typedef struct dac_config \{(.*?)\} dac_config;", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        assert decl.startswith("int "), decl
        names += [re.sub(r"\[.*\]", "", n).strip() for n in decl[4:].split(",")]
    assert [f[0] for f in _lib.DacConfig._fields_] == names


def test_build_id_matches_sources():
    """The library carries the hash of the sources it was built from (Makefile); a stale
    build (sources edited after `make`) is caught here, before any GPU run."""
    from daclip_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdaclip_hip.so not built")
    info = _lib.build_info()
    assert info["matches"], info
