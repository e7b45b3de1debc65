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


def test_host_asan_argument_validation():
    """the C ABI's argument-validation paths under a host AddressSanitizer build
    (tools/abi_asan.cpp, `make -C da-clip_amd asan`: capi.cpp / engine.cpp with -fsanitize=address
    on the host side). Null handles and pointers, bad dtypes / configs and (on a GPU box) a
    handle driven through set_weight / forward-before-finalize / strict-load errors must return
    their DAC_E* codes with no heap error or leak."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "abi_asan")
    if not os.path.exists(exe):
        r = subprocess.run(["make", "-C", os.path.join(ROOT, "da-clip_amd"), "-j8", "asan"],
                           capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip("host ASan build unavailable: " + r.stderr[-300:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-2000:]
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "all checks passed" in r.stdout
